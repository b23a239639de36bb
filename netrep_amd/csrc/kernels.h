// Launch parameter blocks shared by kernels.hip and engine.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nr {

enum { NR_IDX_PRP = 0, NR_IDX_TABLE = 1, NR_IDX_DIRECT = 2 };

constexpr int kProfileWaves = 4;  // waves of the 256-thread profile workgroup (NR_WAVES)
constexpr int kPackedLayoutK = 320;  // modules of the packed kernel's compile-time LDS layout

// phase-stamp slots of the summary-profile kernel (nr_set_stamps)
constexpr int NR_N_STAMPS = 16;

// The small class of summary-profile items: Lanczos dimension min(k, S) at
// most kSmallDim, solved by workgroups of kSmallWaves waves (several items per
// CU in flight instead of three 4-wave items); per-node arrays of modules
// longer than kSmallDim in the slot's scratch.
constexpr int kSmallDim = 112;
constexpr int kSmallWaves = 2;  // (one wave per item measured slower: profiles/r03/small_class/)
// The wave class (round 5, variant 7): Lanczos dimension at most kWaveDim, one
// wave per item with the item's whole Gram in its registers (kernels.hip).
constexpr int kWaveBlocks = 7;                // 16-row blocks of the Gram's side (<= 112)
constexpr int kWaveVec = 16 * kWaveBlocks;     // LDS vector length and Lanczos basis columns
constexpr int kWaveDim = kWaveVec - 1;         // the side is the dimension plus the ones column

// Where the test column of module node c comes from.
struct IndexSource {
  int mode;                    // NR_IDX_*
  uint64_t seed;               // PRP key
  int64_t perm_base;           // global index of local permutation 0
  uint32_t n_null;             // null-pool size
  const int32_t* null_idx;     // [n_null] test columns of the null pool
  const int32_t* null_pos;     // [nodes] null-pool position of each module node
  const uint32_t* pi;          // [n_perm x n_null] explicit shuffles (TABLE)
  const int32_t* direct_idx;   // [nodes] test column of each node (DIRECT)
};

struct NetParams {
  const double2* pairs;        // interleaved {corr, net}, column-major n x n (es = 1), or the
                               // Gram table: {corr, net}, {gram, net^T} per (i, j) (es = 2)
  int32_t es;                  // element stride of pairs in double2 units (1 or 2)
  const double* colsum;        // [n_nodes] column sums of the data (Gram table only)
  int64_t n_nodes;
  int symmetric;               // both matrices exactly symmetric
  IndexSource src;
  const int64_t* node_off;     // [n_mod + 1]
  const int64_t* cv_off;       // [n_mod + 1] CorrVector offsets (k(k-1)/2)
  const double* disc_cv;       // discovery CorrVector (NULL: no statistics)
  const double* disc_wd;       // discovery weighted degree
  const double* cv_shift;      // [n_mod] one-pass shift for the discovery corr values
  const int32_t* mod_order;    // [n_present] module processing order (large first)
  int32_t n_perm;              // permutations in this launch
  int32_t k_max;
  const int32_t* row_of;       // [n_mod] output row
  int32_t n_rows, n_stat;
  int32_t slot_avg_weight, slot_cor_cor, slot_cor_degree, slot_avg_cor;
  double* out;                 // cube slice (NULL in vector mode)
  double* cv_out;              // vector outputs (NULL unless vector mode)
  double* wd_out;
  double* avgw_out;            // [n_mod] average edge weight (vector mode)
  int64_t n_items;             // items of this launch (set by launch_net)
  // Modules too large for the per-node arrays in LDS: a persistent grid of
  // big_slots workgroups, each with big_stride doubles of global scratch
  double* big_scratch;
  int64_t big_stride;
  int32_t big_slots;
};

struct ProfileParams {
  const double* data;          // n_samples x (n_nodes + 2), column-major, scaled; column n_nodes
                               // all ones, n_nodes + 1 zeros (the Gram's virtual columns)
  int64_t n_samples;
  int64_t ones_off;            // n_nodes * n_samples: offset of the ones column
  IndexSource src;
  const int64_t* node_off;
  const double* disc_nc;       // discovery contribution (NULL: vector mode)
  const int32_t* mod_order;
  int32_t n_perm;
  int32_t n_items;
  int32_t k_max, m_max;
  int32_t ld;                  // leading dimension of the per-slot Gram (full storage)
  int64_t gram_doubles;        // doubles reserved for the Gram per slot
  const int32_t* row_of;
  int32_t n_rows, n_stat;
  int32_t slot_coherence, slot_cor_contrib, slot_avg_contrib;
  double* out;
  double* sp_out;              // [n_mod x n_samples] summary profiles (vector mode)
  double* nc_out;              // [nodes] node contributions (vector mode)
  double* coh_out;             // [n_mod] coherence (vector mode)
  double* scratch;             // per-slot Gram (ld x ld) + Lanczos basis (k_max x m_max)
  int64_t scratch_stride;
  int* queue;                  // work-queue head, zeroed before launch
  int* diag;                   // [0] Lanczos step-cap hits, [1] items, [2] Lanczos steps, [3] reorthogonalisations
  unsigned long long* stamps;  // [8] per-phase shader cycles (diagnostics; NULL = off)
  int part_global;             // 1: matvec partials (4 x k_max) at the end of the slot's scratch
  int32_t kvec;                // LDS vector length (0: k_max); larger (dual) modules keep their
                               // per-node arrays in the slot's scratch
  int64_t basis_doubles;       // Lanczos basis doubles per slot (behind the Gram)
  int64_t g32_off;             // doubles from the slot start to the fp32 copy of the packed Gram
                               // (relaxed Lanczos steps; 0: no copy, fp64 matvecs throughout)
  int32_t vec_global;          // 1: the Lanczos vectors, per-node arrays and index set in the slot's
                               // scratch too (Lanczos dimensions beyond the LDS vectors: variant 6)
  int32_t order_tail;          // queue order: 0 = module-major (large modules first); T > 0 =
                               // permutation-major over all modules (a size mix in flight) for the
                               // first n_perm - T permutations, the last T module-major
  // Gram table (packed kernel only): the network statistics of each item are
  // computed in the profile workgroup from one gather per pair of the table,
  // which also fills the item's packed Gram (no matrix-core Gram for k <= S)
  int32_t fused;                // 1: Gram-table items (network statistics + Gram from the table)
  NetParams net;
};

// The column sweep (sweep.hip): network statistics of a batch organised by
// test column (each column chunk streamed into LDS once, every occurrence of
// the column reads its rows there) instead of one random gather per pair.
constexpr int kSweepWaves = 16;                   // waves per (column, chunk) workgroup: one per CU
// Lanes per occurrence: 8 (16: 2-5% slower at C4 / C2, r05/l8b), except where a
// module exceeds kSweepWideK nodes (C5): 16 lanes halve each
// occurrence's serial run over its entries, and at C5's 64-permutation
// launches (~64 occurrences per column) eight-lane batches fill only half of
// a workgroup's 16 waves (C5 sweep 12.8 ms per 64 permutations at 16 lanes,
// 16.3 at 8: profiles/r05/final3/C5.json, profiles/r05/sweep16/)
constexpr int kSweepWideK = 1024;
constexpr int kSweepMaxChunks = 16;               // chunks per column (n <= 65,535)
constexpr int kSweepMaxK = 4096;                  // module nodes (LDS of the per-item kernels)
constexpr int64_t kSweepChunkBytes = 160000;      // LDS per (column, chunk) workgroup
constexpr int kSweepRec = 12;                     // doubles per (occurrence, chunk) record
struct SweepParams {
  const double2* pairs;        // {corr, net} (es = 1) or the Gram table (es = 2), column-major n x n
  int64_t n_nodes;
  int32_t es;
  IndexSource src;
  int64_t n_node_total;        // module nodes of the present modules (CSR)
  int32_t n_present;
  const int64_t* node_off;     // [n_present + 1]
  const int32_t* mod_order;    // [n_present] modules by size, descending
  const int64_t* cv_off;       // [n_present + 1] CorrVector offsets
  const double* disc_cv;       // discovery CorrVector (NULL: no CorrVector statistics)
  int64_t n_cv;                // its length
  int32_t finite;              // 1: the test correlations and disc_cv are all finite (no complete-case tests)
  const double* disc_wd;       // discovery weighted degree
  const double* cv_shift;      // [n_present] one-pass shift of the discovery values
  int32_t n_perm;              // permutations of this batch
  int32_t k_max;
  int64_t n_occ;               // n_perm x n_node_total occurrences
  int64_t chunk_rows;          // rows per column chunk
  int32_t n_chunks;
  // per batch work buffers
  int32_t* col;                // [n_occ] test column of each (permutation, node)
  uint32_t* sorted;            // [n_occ] per item: (column << 16 | position), sorted by column
  int32_t* rank;               // [n_occ] sorted rank of each position
  int32_t* count;              // [n_nodes] occurrences per column
  int32_t* col_off;            // [n_nodes + 1]
  const double* zero;          // >= 32 zero bytes: the address of a lane with nothing to load
  double* sink;                // [256] the address of a lane with nothing to store
  double* dabs;                // [n_nodes] |diagonal| of each column with occurrences (written by the sweep)
  int32_t* lrank;              // [n_occ] slot of each occurrence within its column
  uint4* meta;                 // [n_occ x 2] by column slot: item base, jj | rank << 16, CorrVector base,
                               //   b1 | k << 16; CorrVector shifts {module, item}
  uint32_t* bndh;              // [n_chunks x n_occ] by slot (more than two chunks): e0 | e1 << 16 of the chunk
  double* rec;                 // [n_occ x n_chunks x kSweepRec] one record per (occurrence, chunk)
  const int32_t* row_of;
  int32_t n_rows, n_stat;
  int32_t slot_avg_weight, slot_cor_cor, slot_cor_degree, slot_avg_cor;
  double* out;
};
// rows per chunk for LDS elements of elem_bytes (16: {corr, net}; 8: net only)
int64_t sweep_chunk_rows(int64_t n_nodes, int elem_bytes);
bool sweep_supported(int64_t n_nodes, int k_max);
hipError_t launch_sweep(const SweepParams& P, hipStream_t st);

size_t net_kernel_lds(int k_max);
bool net_kernel_big(int k_max);        // per-node arrays in global scratch
size_t net_big_slot_bytes(int k_max);  // global scratch per workgroup in that mode
size_t profile_kernel_lds(int k_max, int m_max, int n_samples, int variant);
// Doubles of the packed (chunked column-group) Gram of side kc, rounded to 32.
int64_t packed_gram_doubles(int kc);
int profile_kvec_max(int m_max);  // longest LDS vectors of the large-module layout (variant 4)
hipError_t launch_net(const NetParams& P, int64_t n_items, hipStream_t st);
// Whether the packed kernel's LDS (vectors of kvec, basis mmax) holds the
// network item's per-node arrays (the fused Gram-table path).
bool fused_net_fits(int kvec, int mmax, int nw);
// waves per workgroup of the Gram-table kernel (2 waves x 5 per CU measured
// 13% slower, profiles/r03/table_waves/), its LDS bytes and workgroups per CU
constexpr int kTableWaves = 4;
size_t profile_table_lds();
int profile_table_per_cu();
// The Gram table of a dataset with data: gram[i + j n] = x_i . x_j over the
// n_samples rows of X (n_samples x (n + 2), the virtual columns behind), and
// colsum[j] = sum of column j.
hipError_t launch_gram_full(const double* X, int64_t S, int64_t n, double* gram, double* colsum, hipStream_t st);
// {corr, net} pairs (es = 1) + gram -> the table layout (es = 2):
// out[2e] = in[e], out[2e + 1] = {gram[e], net(j, i)} for e = i + j n.
hipError_t launch_widen_pairs(const double2* in, const double* gram, double2* out, int64_t n, int symmetric,
                              hipStream_t st);
// the small class (variant 5): its LDS bytes per workgroup and workgroups per CU
size_t profile_small_lds();
int profile_small_per_cu();
// the wave class (variant 7): its LDS bytes per workgroup and workgroups per CU
size_t profile_wave_lds();
int profile_wave_per_cu();
// variant 0 full Gram, 2 packed Gram, 4 full Gram with the partials in scratch,
// 5 the small class, 6 full Gram with the partials and every vector in scratch,
// 7 the wave class (register-resident Gram)
hipError_t launch_profile(const ProfileParams& P, int n_slots, int variant, int wg_per_cu,
                          hipStream_t st);
hipError_t launch_interleave(const double* corr, const double* net, double2* out, int64_t n_elem,
                             hipStream_t st);
hipError_t launch_symmetry(const double2* a, int64_t n, int* asym, hipStream_t st);
hipError_t launch_scale(const double* in, double* out, int64_t S, int64_t N, hipStream_t st);
// XDR (big-endian) doubles -> native: into pairs[i].x (half 0) / .y (half 1), or `plain`
hipError_t launch_xdr(const void* raw, double2* pairs, int half, double* plain, int64_t n, hipStream_t st);
hipError_t launch_finite(const double* a, int64_t n, int* nonfinite, hipStream_t st);
hipError_t launch_export(const IndexSource& src, int64_t n_nodes_total, int32_t* out,
                         int64_t n_perm, hipStream_t st);

}  // namespace nr
