// The column sweep: module network statistics (avg.weight, cor.cor,
// cor.degree, avg.cor; CorrVector + WeightedDegree, src/netStats.cpp:124-204,
// src/permutations.cpp:75-97, src/permutationsNoData.cpp:66-85) for a batch of
// permutations, organised by TEST COLUMN instead of by item.
//
// Every pair a module-permutation item reads, corr/net(I_r, I_c), lies in the
// column of one of its nodes, I_c. Gathered per item, each pair is a random
// 16-byte read of an N x N matrix, i.e. one random HBM/Infinity-Cache line:
// the item-major kernel (module_net_kernel) runs at the chip's random-line
// rate. Here each column chunk of the {corr, net} array is streamed into LDS
// once per batch (coalesced), and every occurrence of that column in the
// batch -- a (permutation, module node) whose permuted test column it is --
// reads its rows from LDS. For node c of an item the column holds everything
// the node contributes: its weighted degree is the column sum |net(I_r, I_c)|
// over the item's rows (WeightedDegree's colsum, src/netStats.cpp:136-151),
// and its CorrVector pairs are the rows of later module positions
// (corr(idx[ii], idx[jj]) for ii > jj, src/netStats.cpp:196-201).
//
// Steps per batch (launch_sweep):
//  1. sweep_cols_kernel   per item: the permuted test columns (the index
//     source of the other kernels, GetRandomIdx src/utils.cpp:193-199), the
//     column histogram of the batch and each occurrence's slot within its
//     column (the atomics' return values; items in module-size order);
//  2. sweep_scan_kernel   column offsets (exclusive scan of the histogram);
//  3. sweep_prep_kernel   per item: the columns' sorted order (SortNodes,
//     src/netStats.cpp:23-32) as packed (column, position) entries, each
//     position's sorted rank, the entries' split over the column chunks, the
//     CorrVector shift of the item, and each occurrence's slot record (what
//     the sweep needs of it) written to its column's slot;
//  4. sweep_column_kernel one workgroup per (column, chunk): the chunk in LDS,
//     eight lanes per occurrence over the item's sorted entries in the
//     chunk, the next occurrences' metadata and entries in flight while the
//     current ones are summed; one partial record (weighted-degree parts,
//     CorrVector sums) per (occurrence, chunk);
//  5. sweep_finish_kernel one wave per item: the records in chunk order, the
//     reference's weighted degree per node (the fixed-point cancellation model
//     of kernels.hip), the item's four statistics into the cube.
// Every sum runs in a fixed order (records by chunk, lanes by DPP butterflies,
// nodes by position): the results do not depend on the schedule.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <type_traits>
#include <stdint.h>
#include <math.h>

#include "prp.h"
#include "kernels.h"
#include "device_common.h"

namespace nr {

// Record of one (occurrence, chunk), kSweepRec fields: weighted-degree parts of
// the column node (0 plain sum, 1 first same-parity term after the diagonal),
// the CorrVector sums of its pairs with later module positions (complete
// cases, shifted: 2 n, 3 sx, 4 sy, 5 sxx, 6 syy, 7 sxy, 8 sum(sign(x) y)) and
// the fixed-point weighted-degree parts (uint64: 9 before the diagonal, 10
// other parity, 11 same-parity tail).

// Packed sorted entry: test column (high 16 bits), module position (low 16).
__device__ __forceinline__ uint32_t sw_pack(uint32_t col, uint32_t pos) { return (col << 16) | pos; }

// Items run in module-size order, largest first: block b is module
// mod_order[b / n_perm] of permutation b % n_perm, so the column slots handed
// out by the atomics below fill roughly by module size, and the lane groups of
// a sweep wave carry items of similar size. The slot order within a column is
// whatever the atomics give; every record is per occurrence, so the results
// do not depend on it.
struct SwItem {
  int64_t p, item, off, base;
  int m, k;
};
__device__ __forceinline__ SwItem sw_item(const SweepParams& P, int64_t b) {
  SwItem it;
  const int64_t mi = b / P.n_perm;
  it.p = b - mi * P.n_perm;
  it.m = P.mod_order[mi];
  it.item = it.p * P.n_present + it.m;
  it.off = P.node_off[it.m];
  it.k = (int)(P.node_off[it.m + 1] - it.off);
  it.base = it.p * P.n_node_total + it.off;
  return it;
}

// ---- 1. per item: test columns, column histogram, slots within columns ------
__global__ void __launch_bounds__(256) sweep_cols_kernel(SweepParams P) {
  const SwItem it = sw_item(P, blockIdx.x);
  nr_prp_key key;
  if (P.src.mode == NR_IDX_PRP) key = nr_prp_make_key(P.src.seed, (uint64_t)(P.src.perm_base + it.p), P.src.n_null);
  for (int c = threadIdx.x; c < it.k; c += 256) {
    const int32_t ic = node_index(P.src, key, it.p, it.off + c);
    P.col[it.base + c] = ic;
    P.lrank[it.base + c] = atomicAdd(&P.count[ic], 1);
  }
}

// ---- 2. column offsets ------------------------------------------------------
// One 1024-thread workgroup: off[c] = sum of count[< c].
__global__ void __launch_bounds__(1024) sweep_scan_kernel(const int32_t* count, int32_t* off, int64_t n) {
  __shared__ int32_t s[1024];
  const int t = threadIdx.x;
  const int64_t per = (n + 1023) / 1024;
  const int64_t a = t * per, b = a + per < n ? a + per : n;
  int32_t sum = 0;
  for (int64_t i = a; i < b; ++i) sum += count[i];
  s[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int32_t v = t >= o ? s[t - o] : 0;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  int32_t run = s[t] - sum;  // exclusive prefix of this thread's range
  for (int64_t i = a; i < b; ++i) {
    off[i] = run;
    run += count[i];
  }
  if (t == 1023) off[n] = s[t];
}

// ---- 3. per item: sorted entries, chunk split, occurrences into their slots --
// One 256-thread workgroup per item. LDS: the item's k columns and sorted
// ranks, the per-chunk counts. Each occurrence's 32-byte slot record (what
// the sweep needs of it) goes to its column's slot: item entry base, jj |
// rank << 16, CorrVector base of jj's pairs, b1 | k << 16 (the first entry of
// chunk 1 and the item size: the range of a one- or two-chunk sweep; more
// chunks write bndh), then the CorrVector shifts {discovery (module), test
// (item)}.
__global__ void __launch_bounds__(256) sweep_prep_kernel(SweepParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const SwItem it = sw_item(P, blockIdx.x);
  const int k = it.k;
  uint32_t* cols = reinterpret_cast<uint32_t*>(smem);  // [k]
  int32_t* rnk = reinterpret_cast<int32_t*>(smem) + k;  // [k]
  __shared__ int s_cnt[kSweepMaxChunks + 1];
  __shared__ double s_ys;
  for (int i = threadIdx.x; i <= kSweepMaxChunks; i += 256) s_cnt[i] = 0;
  for (int c = threadIdx.x; c < k; c += 256) cols[c] = (uint32_t)P.col[it.base + c];
  __syncthreads();
  for (int c = threadIdx.x; c < k; c += 256) {
    const uint32_t ic = cols[c];
    int r = 0;
    for (int q = 0; q < k; ++q) r += cols[q] < ic;  // distinct columns: one shuffle per permutation
    P.sorted[it.base + r] = sw_pack(ic, (uint32_t)c);
    P.rank[it.base + c] = r;
    rnk[c] = r;
    atomicAdd(&s_cnt[ic / P.chunk_rows + 1], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int h = 0; h < P.n_chunks; ++h) s_cnt[h + 1] += s_cnt[h];  // s_cnt[h] = first entry of chunk h
    // CorrVector shift of the test side: the item's first pair (net_item)
    double ys = 0.0;
    if (k > 1) {
      const double y0 = P.pairs[((int64_t)cols[1] + (int64_t)cols[0] * P.n_nodes) * P.es].x;
      ys = isfinite(y0) ? y0 : 0.0;
    }
    s_ys = ys;
  }
  __syncthreads();
  const uint32_t b1 = P.n_chunks > 1 ? (uint32_t)s_cnt[1] : (uint32_t)k;
  const double xs = P.cv_shift ? P.cv_shift[it.m] : 0.0;
  const int64_t cvo = P.disc_cv ? P.cv_off[it.m] : 0;
  for (int c = threadIdx.x; c < k; c += 256) {
    const int32_t s = P.col_off[cols[c]] + P.lrank[it.base + c];
    // CorrVector base of c's pairs: v(ii, c) = cv_off + c (2k - c - 1) / 2 + ii - c - 1
    const uint32_t cvb = P.disc_cv ? (uint32_t)(cvo + (int64_t)c * (2 * (int64_t)k - c - 1) / 2 - c - 1) : 0u;
    uint4* mt = P.meta + 2 * (int64_t)s;
    mt[0] = make_uint4((uint32_t)it.base, (uint32_t)c | ((uint32_t)rnk[c] << 16), cvb, b1 | ((uint32_t)k << 16));
    if (P.disc_cv) mt[1] = __builtin_bit_cast(uint4, make_double2(xs, s_ys));
    if (P.n_chunks > 2)
      for (int h = 0; h < P.n_chunks; ++h)
        P.bndh[(int64_t)h * P.n_occ + s] = (uint32_t)s_cnt[h] | ((uint32_t)s_cnt[h + 1] << 16);
  }
}

// ---- 4. the sweep ------------------------------------------------------------
template <uint32_t CTRL>
__device__ __forceinline__ unsigned long long sw_dpp_u64(unsigned long long v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, false);
  return ((unsigned long long)hi << 32) | lo;
}

// Sixteen-lane groups (modules beyond kSweepWideK nodes): sums of v[0..16)
// over the 16 lanes of each row, transposed: afterwards lane gl of the row
// holds the total of v[gl]. Four DPP exchange levels on lane bits 3..0,
// halving the values at each (15 exchanges, not 64); fixed order.
__device__ __forceinline__ double sw_transpose16(const double (&v)[16], int lane) {
  const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2, b0 = lane & 1;
  double a8[8], a4[4], a2[2];
#pragma unroll
  for (int i = 0; i < 8; ++i) a8[i] = (b3 ? v[i + 8] : v[i]) + nr_dpp<NR_DPP_ROR8>(b3 ? v[i] : v[i + 8]);
#pragma unroll
  for (int i = 0; i < 4; ++i)  // lane ^ 7: the partner's bits 1, 0 differ too; later levels cover them
    a4[i] = (b2 ? a8[i + 4] : a8[i]) + nr_dpp<NR_DPP_HALF_MIRROR>(b2 ? a8[i] : a8[i + 4]);
#pragma unroll
  for (int i = 0; i < 2; ++i) a2[i] = (b1 ? a4[i + 2] : a4[i]) + nr_dpp<NR_DPP_XOR2>(b1 ? a4[i] : a4[i + 2]);
  return (b0 ? a2[1] : a2[0]) + nr_dpp<NR_DPP_XOR1>(b0 ? a2[0] : a2[1]);
}
// ... and four exact integer sums: lanes with bits (3, 2) = (i, j) hold the
// total of v[2i + j].
__device__ __forceinline__ unsigned long long sw_transpose4_u64(const unsigned long long (&v)[4], int lane) {
  const bool b3 = lane & 8, b2 = lane & 4;
  unsigned long long a2[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) a2[i] = (b3 ? v[i + 2] : v[i]) + sw_dpp_u64<NR_DPP_ROR8>(b3 ? v[i] : v[i + 2]);
  unsigned long long x = (b2 ? a2[1] : a2[0]) + sw_dpp_u64<NR_DPP_HALF_MIRROR>(b2 ? a2[0] : a2[1]);
  x += sw_dpp_u64<NR_DPP_XOR2>(x);
  return x + sw_dpp_u64<NR_DPP_XOR1>(x);
}

// Eight-lane groups: the same exchanges over lane bits 2..0 (mirror within
// 8, XOR 2, XOR 1), 16 values -> 2 per lane: lane bits (b2 b1 b0) hold the
// totals of v[8 b2 + 4 b1 + 2 b0] and the next one.
__device__ __forceinline__ double2 sw_transpose16_8(const double (&v)[16], int lane) {
  const bool b2 = lane & 4, b1 = lane & 2, b0 = lane & 1;
  double a8[8], a4[4];
#pragma unroll
  for (int i = 0; i < 8; ++i)  // lane ^ 7
    a8[i] = (b2 ? v[i + 8] : v[i]) + nr_dpp<NR_DPP_HALF_MIRROR>(b2 ? v[i] : v[i + 8]);
#pragma unroll
  for (int i = 0; i < 4; ++i) a4[i] = (b1 ? a8[i + 4] : a8[i]) + nr_dpp<NR_DPP_XOR2>(b1 ? a8[i] : a8[i + 4]);
  double2 r;
  r.x = (b0 ? a4[2] : a4[0]) + nr_dpp<NR_DPP_XOR1>(b0 ? a4[0] : a4[2]);
  r.y = (b0 ? a4[3] : a4[1]) + nr_dpp<NR_DPP_XOR1>(b0 ? a4[1] : a4[3]);
  return r;
}
// ... and four integer sums over 8 lanes: lane bits (b2 b1) hold v[2 b2 + b1].
__device__ __forceinline__ unsigned long long sw_transpose4_u64_8(const unsigned long long (&v)[4], int lane) {
  const bool b2 = lane & 4, b1 = lane & 2;
  unsigned long long a2[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) a2[i] = (b2 ? v[i + 2] : v[i]) + sw_dpp_u64<NR_DPP_HALF_MIRROR>(b2 ? v[i] : v[i + 2]);
  unsigned long long x = (b1 ? a2[1] : a2[0]) + sw_dpp_u64<NR_DPP_XOR2>(b1 ? a2[0] : a2[1]);
  return x + sw_dpp_u64<NR_DPP_XOR1>(x);
}

// Eight sums (the finite-data record: no pair count) over the 8 lanes: three
// exchange levels leave each lane one total, of v[4 b2 + 2 b1 + b0].
__device__ __forceinline__ double sw_transpose8_8(const double (&v)[8], int lane) {
  const bool b2 = lane & 4, b1 = lane & 2, b0 = lane & 1;
  double a4[4], a2[2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    a4[i] = (b2 ? v[i + 4] : v[i]) + nr_dpp<NR_DPP_HALF_MIRROR>(b2 ? v[i] : v[i + 4]);
#pragma unroll
  for (int i = 0; i < 2; ++i) a2[i] = (b1 ? a4[i + 2] : a4[i]) + nr_dpp<NR_DPP_XOR2>(b1 ? a4[i] : a4[i + 2]);
  return (b0 ? a2[1] : a2[0]) + nr_dpp<NR_DPP_XOR1>(b0 ? a2[0] : a2[1]);
}

constexpr int kSweepPre = 6;  // entries per lane in flight per occurrence (4 / 8: r05/sweep A/B)

// One occurrence's metadata (column slot s; zero past the column's end).
struct SwOcc {
  uint4 mt;     // item entry base, jj | rank << 16, CorrVector base of jj's pairs, chunk split (below)
  uint32_t bd;  // the item's entries in this chunk, e0 | e1 << 16
  double2 sh;   // CorrVector shifts {discovery (module), test (item)}
};

// The sweep loop's loads go through buffer descriptors (one per array, built
// from kernel arguments, so wave-uniform): a lane with nothing to load gives
// an offset past the descriptor's range and reads 0 without a branch. A load
// under a branch would leave the compiler no static count of the memory
// operations issued after an earlier load, and its wait for that load would
// become a wait for everything in flight (the prefetches included).
typedef unsigned int sw_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int sw_u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kSwOff = 0xFFFFFFF0u;  // past every descriptor's range: reads 0

struct SwRsrc {
  __amdgpu_buffer_rsrc_t meta, bndh, sorted, dcv;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t sw_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)(uint32_t)bytes, 0x00020000);
}

// mt.w = b1 | k << 16 (the item's first entry of chunk 1, its size): the
// chunk range of a one- or two-chunk sweep; more chunks read bndh.
template <bool X>
__device__ __forceinline__ void sw_fetch(const SweepParams& P, const SwRsrc& R, int h, int32_t s, int32_t o1,
                                         SwOcc& q) {
  const bool in = s < o1;
  q.mt = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(R.meta, in ? (uint32_t)s * 32u : kSwOff, 0, 0));
  q.bd = P.n_chunks > 2
             ? __builtin_amdgcn_raw_buffer_load_b32(R.bndh, in ? ((uint32_t)h * (uint32_t)P.n_occ + (uint32_t)s) * 4u : kSwOff, 0, 0)
             : 0u;
  if (X)
    q.sh = __builtin_bit_cast(double2,
                              __builtin_amdgcn_raw_buffer_load_b128(R.meta, in ? (uint32_t)s * 32u + 16u : kSwOff, 0, 0));
}

// The chunk range e0 | e1 << 16 (from mt.w unless read from bndh).
__device__ __forceinline__ uint32_t sw_range(const SweepParams& P, const SwOcc& q, int h) {
  if (P.n_chunks > 2) return q.bd;
  return h == 0 ? (q.mt.w & 0xFFFFu) << 16 : q.mt.w;
}

// Lane gl's entries gl + 16 (t0 + t) of the occurrence's chunk range: one
// offset, the steps as immediates. Entries past the range (the next item's,
// or past the array: 0) are loaded but never used (sw_block skips them).
template <int L>
__device__ __forceinline__ void sw_entries(const SwRsrc& R, const SwOcc& q, uint32_t bd, int gl, int t0,
                                           uint32_t (&u)[kSweepPre]) {
  const uint32_t off = (q.mt.x + (bd & 0xFFFFu) + (uint32_t)gl + (uint32_t)(L * t0)) * 4u;
#pragma unroll
  for (int t = 0; t < kSweepPre; ++t)
    u[t] = __builtin_amdgcn_raw_buffer_load_b32(R.sorted, off + (uint32_t)(t * L * 4), 0, 0);
}

// The discovery CorrVector values of the lane's pairs (ii = r > jj, jj),
// v(ii, jj) = base + ii: issued together, before the next occurrences'
// prefetches (vector-memory counters retire in order).
// (Entries past the range give some in-range or out-of-range offset: read,
// never used.) A pair with ii <= jj reads 0.
__device__ __forceinline__ void sw_xv(const SwRsrc& R, const SwOcc& q, const uint32_t (&u)[kSweepPre],
                                      double (&xv)[kSweepPre]) {
  const int jj = (int)(q.mt.y & 0xFFFFu);
#pragma unroll
  for (int t = 0; t < kSweepPre; ++t) {
    const int r = (int)(u[t] & 0xFFFFu);
    // base + ii >= 0 for ii > jj: inside the module's vector
    const uint32_t off = r > jj ? (uint32_t)((int32_t)q.mt.z + r) * 8u : kSwOff;
    xv[t] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(R.dcv, off, 0, 0));
  }
}

// Running sums of one lane for its occurrence. The lane's entries e = e0 + gl
// + 16t all have the parity of e0 + gl, so a lane either shares the diagonal's
// accumulator (same parity as its rank pj: terms before it, the first term
// after it, the tail) or holds only other-parity terms: `fine` is the
// fixed-point sum before the diagonal on the first kind and the other-parity
// sum on the second, split when the record is written.
struct SwAcc {
  double plain = 0.0, ff = 0.0;
  unsigned long long fine = 0, tn = 0;
  double a[7] = {0, 0, 0, 0, 0, 0, 0};
};

// llrint(min(v, 2^61)) for v >= 0 (wd_fx's rounding): below 2^52 the sum v +
// 2^52 rounds to the nearest even integer and its bit pattern is 2^52's plus
// that integer. Infinite / NaN terms make the node's plain sum non-finite, so
// their fixed-point value is never used.
__device__ __forceinline__ unsigned long long sw_fx(double v) {
  unsigned long long q = __builtin_bit_cast(unsigned long long, v + 4503599627370496.0) - 0x4330000000000000ull;
  const bool big = !(v < 4503599627370496.0);  // 2^52 (or NaN)
  if (__builtin_amdgcn_ballot_w64(big)) {      // wave-uniform: weights this large are rare
    asm volatile("");                          // a real branch (not both paths and a select)
    const double c = v < 2.305843009213694e18 ? v : 2.305843009213694e18;  // 2^61: caught by the range check
    if (big) q = (unsigned long long)llrint(c);
  }
  return q;
}

// The lane's entries t0 .. t0 + kSweepPre of its occurrence. The column's own
// row (every occurrence's diagonal entry, r == jj) is zero in LDS, so it adds
// nothing and needs no test; entries past the range are skipped (a wave past
// it skips the body), the rest is branch-free. FIN: the test correlations and
// the discovery CorrVector are all finite (no complete-case tests; xv is
// already 0 off the pairs).
template <bool X, bool FIN, int L>
__device__ __forceinline__ void sw_block(const void* colv_, int64_t row0, const SwOcc& q, uint32_t bd, int gl,
                                         int t0, const uint32_t (&u)[kSweepPre], const double (&xv)[kSweepPre],
                                         int gj, SwAcc& A) {
  using E = typename std::conditional<X, double2, double>::type;
  const E* colv = reinterpret_cast<const E*>(colv_);
  const int e0 = (int)(bd & 0xFFFFu), e1 = (int)(bd >> 16);
  const int jj = (int)(q.mt.y & 0xFFFFu), pj = (int)(q.mt.y >> 16);
  const bool same = ((pj ^ (e0 + gl)) & 1) == 0;
#pragma unroll
  for (int t = 0; t < kSweepPre; ++t) {
    const int e = e0 + gl + L * (t0 + t);
    if (e >= e1) continue;
    const int r = (int)(u[t] & 0xFFFFu);
    const E v = colv[(int64_t)(u[t] >> 16) - row0];
    double y;
    if constexpr (X) y = v.y; else y = v;
    const double av = fabs(y);
    A.plain += av;
    if (gj != WD_NO_GRID) {  // workgroup-uniform
      // every fixed-point term into `fine`, the tail's into `tn` too; the
      // record subtracts tn and the first term after the diagonal (entry
      // pj + 2, which sw_ff takes out of the sum: the same integers, exact)
      const bool is_tail = same && e > pj + 2;
      const unsigned long long fx = sw_fx(ldexp(av, (is_tail ? 0 : WD_FX_BITS) - gj));
      A.tn += is_tail ? fx : 0ull;
      A.fine += fx;
    }
    if constexpr (X) {
      // CorrVector pair (ii = r, jj), complete cases (src/netStats.cpp:43-61)
      const double x = xv[t], yc = v.x;
      const bool ok = FIN ? r > jj : (r > jj && isfinite(x) && isfinite(yc));
      const double w = ok ? 1.0 : 0.0;
      const double xo = FIN ? x : (ok ? x : 0.0);
      const double yo = FIN ? w * yc : (ok ? yc : 0.0);
      const double dx = fma(-w, q.sh.x, xo), dy = fma(-w, q.sh.y, yo);  // x - xs, y - ys (exact products)
      if (!FIN) A.a[0] += w;  // finite data: every pair complete, n = k (k - 1) / 2 (sweep_finish_kernel)
      A.a[1] += dx;
      A.a[2] += dy;
      A.a[3] += dx * dx;
      A.a[4] += dy * dy;
      A.a[5] += dx * dy;
      A.a[6] = fma(xo > 0.0 ? 1.0 : (xo < 0.0 ? -1.0 : 0.0), yo, A.a[6]);  // sign(x) y (exact product)
    }
  }
  if constexpr (X) {
    // a use of every CorrVector value outside the entries' branches, so the
    // compiler keeps their loads where sw_xv issued them (one sunk into its
    // entry's branch would be waited for with everything issued before it)
#pragma unroll
    for (int t = 0; t < kSweepPre; ++t) asm volatile("" ::"v"(xv[t]));
  }
}

// The first same-parity term after the diagonal (entry pj + 2 of the item's
// sorted order, if it lies in this chunk) on the lane whose entries hold it:
// its plain value is the record's ff part, and its fixed-point value comes out
// of `fine` (sw_block added it there). Then `fine` drops the tail's terms,
// which sw_block added to both. (Round 6: per pair this was a compare and two
// selects in sw_block; C4's column sweep is issue-bound.)
template <bool X, int L>
__device__ __forceinline__ void sw_ff(const SwRsrc& R, const void* colv_, int64_t row0, const SwOcc& q, uint32_t bd,
                                      int gl, int gj, SwAcc& A) {
  using E = typename std::conditional<X, double2, double>::type;
  const E* colv = reinterpret_cast<const E*>(colv_);
  if (gj == WD_NO_GRID) return;  // workgroup-uniform
  A.fine -= A.tn;
  const int e0 = (int)(bd & 0xFFFFu), e1 = (int)(bd >> 16);
  const int ef = (int)(q.mt.y >> 16) + 2;
  if (ef >= e0 && ef < e1 && (ef - e0 - gl) % L == 0) {
    const uint32_t u = __builtin_amdgcn_raw_buffer_load_b32(R.sorted, (q.mt.x + (uint32_t)ef) * 4u, 0, 0);
    const E v = colv[(int64_t)(u >> 16) - row0];
    double y;
    if constexpr (X) y = v.y; else y = v;
    const double av = fabs(y);
    A.ff = av;
    A.fine -= sw_fx(ldexp(av, WD_FX_BITS - gj));
  }
}

// One workgroup of kSweepWaves waves per (column c, chunk h): the chunk's rows
// of column c in LDS ({corr, net} with CorrVector statistics, net alone
// without); each wave takes eight occurrences at a time, eight lanes per
// occurrence over the item's sorted entries in the chunk; one partial record
// per (occurrence, chunk), summed in chunk order by sweep_finish_kernel. The
// next batch's entries and the one after's metadata load while a batch is
// summed.
template <bool X, bool FIN, int L>
__global__ void __launch_bounds__(kSweepWaves * 64) sweep_column_kernel(SweepParams P) {
  using E = typename std::conditional<X, double2, double>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  E* colv = reinterpret_cast<E*>(smem);
  const int64_t c = blockIdx.x;
  const int h = blockIdx.y;
  const int32_t o0 = P.col_off[c], o1 = P.col_off[c + 1];
  const int64_t row0 = (int64_t)h * P.chunk_rows;
  const int64_t rows = P.n_nodes - row0 < P.chunk_rows ? P.n_nodes - row0 : P.chunk_rows;
  if (o1 <= o0 || rows <= 0) return;  // uniform: the whole workgroup leaves
  {
    const double2* src = P.pairs + (row0 + c * P.n_nodes) * P.es;
    constexpr int U = 8;
    for (int64_t i0 = threadIdx.x; i0 < rows; i0 += U * (int64_t)blockDim.x) {
      E t[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // clamped, unconditional loads: all U in flight together
        const int64_t i = i0 + u * (int64_t)blockDim.x < rows ? i0 + u * (int64_t)blockDim.x : rows - 1;
        if constexpr (X) t[u] = src[i * P.es]; else t[u] = src[i * P.es].y;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + u * (int64_t)blockDim.x;
        if (i < rows) {
          if (i == c - row0) {  // the column's own row: the diagonal entry of every occurrence
            if constexpr (X) t[u] = make_double2(0.0, 0.0); else t[u] = 0.0;
          }
          colv[i] = t[u];
        }
      }
    }
  }
  // |diag| of the column node (WeightedDegree subtracts it; the grid of the
  // fixed-point model)
  const double dg = fabs(P.pairs[(c + c * P.n_nodes) * P.es].y);
  const int gj = wd_grid_exp(dg);
  if (h == 0 && threadIdx.x == 0) P.dabs[c] = dg;  // for the finish kernel's weighted degrees
  __syncthreads();
  constexpr int G = 64 / L;  // occurrences per wave batch
  constexpr int32_t stride = G * kSweepWaves;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane / L, gl = lane % L;
  SwRsrc R;
  R.meta = sw_rsrc(P.meta, P.n_occ * 32);
  R.bndh = sw_rsrc(P.bndh, P.n_chunks > 2 ? P.n_occ * 4 * P.n_chunks : 0);
  R.sorted = sw_rsrc(P.sorted, P.n_occ * 4);
  R.dcv = sw_rsrc(P.disc_cv, X ? P.n_cv * 8 : 0);
  SwOcc cur, nxt;
  uint32_t uc[kSweepPre];
  int32_t sb = o0 + G * wave;
  sw_fetch<X>(P, R, h, sb + grp, o1, cur);
  sw_entries<L>(R, cur, sw_range(P, cur, h), gl, 0, uc);
  sw_fetch<X>(P, R, h, sb + stride + grp, o1, nxt);
  // the previous batch's record stores, issued at the top of the next
  // iteration ahead of its loads (vector-memory counters retire in order: a
  // store issued last would hold up the next wait for a prefetched load)
  double* st_d = P.sink + lane;
  unsigned long long* st_i = reinterpret_cast<unsigned long long*>(P.sink) + 64 + lane;
  double2* st_d2 = reinterpret_cast<double2*>(P.sink + 128) + lane;
  double ds = 0.0;
  double2 ds2 = make_double2(0.0, 0.0);
  unsigned long long is = 0;
  for (; sb < o1; sb += stride) {  // wave-uniform
    *st_d = ds;
    *st_i = is;
    if constexpr (!FIN && L == 8) *st_d2 = ds2;
    const uint32_t bdc = sw_range(P, cur, h);
    double xv[kSweepPre];
    if (X) sw_xv(R, cur, uc, xv);
    uint32_t un[kSweepPre];
    sw_entries<L>(R, nxt, sw_range(P, nxt, h), gl, 0, un);
    SwOcc nn;
    sw_fetch<X>(P, R, h, sb + 2 * stride + grp, o1, nn);
    SwAcc A;
    sw_block<X, FIN, L>(colv, row0, cur, bdc, gl, 0, uc, xv, gj, A);
    {
      const int e0 = (int)(bdc & 0xFFFFu), e1 = (int)(bdc >> 16);
      for (int t0 = kSweepPre; e0 + L * t0 < e1; t0 += kSweepPre) {  // long chunk ranges
        uint32_t ux[kSweepPre];
        sw_entries<L>(R, cur, bdc, gl, t0, ux);
        if (X) sw_xv(R, cur, ux, xv);
        sw_block<X, FIN, L>(colv, row0, cur, bdc, gl, t0, ux, xv, gj, A);
      }
    }
    sw_ff<X, L>(R, colv, row0, cur, bdc, gl, gj, A);
    // record fields: 0 plain, 1 ff, 2..7 the CorrVector sums sx, sy, sxx, syy,
    // sxy, sum sign(x) y, 8 their pair count (not written for finite data),
    // 9..11 the fixed-point parts
    const double dv[16] = {A.plain, A.ff, A.a[1], A.a[2], A.a[3], A.a[4], A.a[5], A.a[6], A.a[0], 0, 0, 0, 0, 0, 0, 0};
    const double dv8[8] = {A.plain, A.ff, A.a[1], A.a[2], A.a[3], A.a[4], A.a[5], A.a[6]};
    const bool same = (((cur.mt.y >> 16) ^ ((bdc & 0xFFFFu) + (uint32_t)gl)) & 1u) == 0;
    const unsigned long long iv[4] = {same ? A.fine : 0ull, same ? 0ull : A.fine, A.tn, 0};
    // the record by occurrence (item entry base + jj), so the finish kernel
    // reads an item's records contiguously; lanes with nothing to store
    // write P.sink
    const bool live = sb + grp < o1;
    double* rec = P.rec + ((int64_t)(cur.mt.x + (cur.mt.y & 0xFFFFu)) * P.n_chunks + h) * kSweepRec;
    if constexpr (L == 16) {
      // lane gl: double field gl (8 fields for finite data, 9 otherwise);
      // lanes 0, 4, 8: integer fields 9..11
      ds = sw_transpose16(dv, lane);
      is = sw_transpose4_u64(iv, lane);
      st_d = live && gl < (FIN ? 8 : 9) ? rec + gl : P.sink + lane;
      st_i = live && (gl & 3) == 0 && gl < 12 ? reinterpret_cast<unsigned long long*>(rec) + 9 + (gl >> 2)
                                               : reinterpret_cast<unsigned long long*>(P.sink) + 64 + lane;
    } else if constexpr (FIN) {
      // lane (b2 b1 b0): double field 4 b2 + 2 b1 + b0; lanes with b0 = 0: integer field 9 + 2 b2 + b1
      ds = sw_transpose8_8(dv8, lane);
      is = sw_transpose4_u64_8(iv, lane);
      const int fi = 2 * ((gl >> 2) & 1) + ((gl >> 1) & 1);
      st_d = live ? rec + gl : P.sink + lane;
      st_i = live && (gl & 1) == 0 && fi < 3 ? reinterpret_cast<unsigned long long*>(rec) + 9 + fi
                                              : reinterpret_cast<unsigned long long*>(P.sink) + 64 + lane;
    } else {
      // lane (b2 b1 b0): double fields 8 b2 + 4 b1 + 2 b0 and the next (field 8
      // alone: 9 is an integer field); lanes with b0 = 0: integer field 9 + 2 b2 + b1
      ds2 = sw_transpose16_8(dv, lane);
      ds = ds2.x;
      is = sw_transpose4_u64_8(iv, lane);
      const int f0 = 8 * ((gl >> 2) & 1) + 4 * ((gl >> 1) & 1) + 2 * (gl & 1);
      const int fi = 2 * ((gl >> 2) & 1) + ((gl >> 1) & 1);
      st_d2 = live && f0 < 8 ? reinterpret_cast<double2*>(rec + f0) : reinterpret_cast<double2*>(P.sink + 128) + lane;
      st_d = live && f0 == 8 ? rec + 8 : P.sink + lane;
      st_i = live && (gl & 1) == 0 && fi < 3 ? reinterpret_cast<unsigned long long*>(rec) + 9 + fi
                                              : reinterpret_cast<unsigned long long*>(P.sink) + 64 + lane;
    }
    cur = nxt;
    nxt = nn;
#pragma unroll
    for (int t = 0; t < kSweepPre; ++t) uc[t] = un[t];
  }
  *st_d = ds;
  *st_i = is;
  if constexpr (!FIN && L == 8) *st_d2 = ds2;
}

// ---- 5. per item ---------------------------------------------------------------
// The reference's weighted degree from a node's summed parts (kernels.hip
// wd_final, the same model).
__device__ __forceinline__ double sw_wd_final(double plain, double ff, unsigned long long pb, unsigned long long on,
                                              unsigned long long tn, double d, int rk, int k) {
  if (!isfinite(d)) return nr_nan();
  if (!isfinite(plain)) return plain;
  const int ge = wd_grid_exp(d);
  if (ge == WD_NO_GRID) return plain;
  if (ldexp(plain, WD_FX_BITS - ge) >= 1.1529215046068470e18) return plain;  // 2^60
  const double s = ldexp(1.0, ge - WD_FX_BITS);
  const double g = ldexp(1.0, ge);
  double x = (double)pb * s + d;
  if (rk + 2 < k) x = x + ff;
  if (!(x > 0.0) || ilogb(x) - 52 != ge) return plain;
  const double chain = x + (double)tn * g;
  if (ilogb(chain) - 52 != ge) return plain;
  return (chain + (double)on * s) - d;
}

// One wave per item; the node's weighted degrees in LDS for the two-pass
// cor.degree.
__global__ void __launch_bounds__(256) sweep_finish_kernel(SweepParams P, int64_t n_items) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* wdv = reinterpret_cast<double*>(smem) + (int64_t)wave * P.k_max;
  const int64_t item = blockIdx.x * 4 + wave;
  if (item >= n_items) return;
  const int64_t p = item / P.n_present;
  const int m = (int)(item - p * P.n_present);
  const int64_t off = P.node_off[m];
  const int k = (int)(P.node_off[m + 1] - off);
  const int64_t base = p * P.n_node_total + off;
  double acc[7] = {0, 0, 0, 0, 0, 0, 0};
  double a1[4] = {0, 0, 0, 0};  // sum(all wd), n, sx, sy
  for (int c = lane; c < k; c += 64) {
    double plain = 0.0, ff = 0.0;
    unsigned long long pb = 0, on = 0, tn = 0;
    for (int h = 0; h < P.n_chunks; ++h) {  // chunk order: deterministic
      const double* rec = P.rec + ((base + c) * P.n_chunks + h) * kSweepRec;
      const unsigned long long* irec = reinterpret_cast<const unsigned long long*>(rec);
      plain += rec[0];
      ff += rec[1];
#pragma unroll
      for (int i = 1; i < 7; ++i) acc[i] += rec[1 + i];
      if (!P.finite) acc[0] += rec[8];
      pb += irec[9];
      on += irec[10];
      tn += irec[11];
    }
    const double d = P.dabs[P.col[base + c]];
    const double y = sw_wd_final(plain, ff, pb, on, tn, d, P.rank[base + c], k);
    wdv[c] = y;
    const double xv = P.disc_wd ? P.disc_wd[off + c] : nr_nan();
    a1[0] += y;
    if (isfinite(xv) && isfinite(y)) {
      a1[1] += 1.0;
      a1[2] += xv;
      a1[3] += y;
    }
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) acc[i] = nr_wave_sum(acc[i]);
  if (P.finite) acc[0] = 0.5 * (double)k * (double)(k - 1);  // finite data: every pair complete
#pragma unroll
  for (int i = 0; i < 4; ++i) a1[i] = nr_wave_sum(a1[i]);
  const double mx = a1[2] / a1[1], my = a1[3] / a1[1];
  double a2[3] = {0, 0, 0};
  for (int c = lane; c < k; c += 64) {
    const double y = wdv[c];
    const double xv = P.disc_wd ? P.disc_wd[off + c] : nr_nan();
    if (isfinite(xv) && isfinite(y)) {
      const double dx = xv - mx, dy = y - my;
      a2[0] += dx * dx;
      a2[1] += dy * dy;
      a2[2] += dx * dy;
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) a2[i] = nr_wave_sum(a2[i]);
  if (lane == 0 && P.out) {
    // AverageEdgeWeight src/netStats.cpp:154-162: unsigned int pair count
    const uint32_t ku = (uint32_t)k;
    const double avg_weight = a1[0] / (double)(uint32_t)(ku * ku - ku);
    const double cor_degree = a1[1] >= 1.0 ? a2[2] / (sqrt(a2[0]) * sqrt(a2[1])) : nr_nan();
    const double cor_cor = pearson_sums(acc[0], acc[1], acc[2], acc[3], acc[4], acc[5]);
    const double avg_cor = acc[0] >= 1.0 ? acc[6] / acc[0] : nr_nan();
    double* o = P.out + (int64_t)P.row_of[m] + (int64_t)P.n_rows * (int64_t)P.n_stat * p;
    o[(int64_t)P.n_rows * P.slot_avg_weight] = na_fill(avg_weight);
    o[(int64_t)P.n_rows * P.slot_cor_cor] = na_fill(cor_cor);
    o[(int64_t)P.n_rows * P.slot_cor_degree] = na_fill(cor_degree);
    o[(int64_t)P.n_rows * P.slot_avg_cor] = na_fill(avg_cor);
  }
}

// ---- launcher ---------------------------------------------------------------------
bool sweep_supported(int64_t n_nodes, int k_max) {
  // packed entries hold a column in 16 bits, chunk bounds an entry index in 16
  return n_nodes > 0 && n_nodes < 65536 && k_max >= 1 && k_max <= kSweepMaxK &&
         (n_nodes + sweep_chunk_rows(n_nodes, 16) - 1) / sweep_chunk_rows(n_nodes, 16) <= kSweepMaxChunks;
}

int64_t sweep_chunk_rows(int64_t n_nodes, int elem_bytes) {
  // chunks of at most kSweepChunkBytes of LDS, balanced, whole 64-row groups
  // (within the budget: the cap is a multiple of 64 rows)
  const int64_t cap = kSweepChunkBytes / elem_bytes / 64 * 64;
  const int64_t n_chunks = (n_nodes + cap - 1) / cap;
  const int64_t rows = (n_nodes + n_chunks - 1) / n_chunks;
  return std::min(cap, (rows + 63) / 64 * 64);
}

hipError_t launch_sweep(const SweepParams& P0, hipStream_t st) {
  SweepParams P = P0;
  const int64_t n_items = (int64_t)P.n_perm * P.n_present;
  if (n_items <= 0) return hipSuccess;
  if (P.n_occ != (int64_t)P.n_perm * P.n_node_total || P.n_chunks < 1 || P.n_chunks > kSweepMaxChunks ||
      P.chunk_rows * P.n_chunks < P.n_nodes || P.chunk_rows * (P.disc_cv ? 16 : 8) > kSweepChunkBytes ||
      P.n_occ * 32 >= ((int64_t)1 << 32) || P.n_occ * 4 * P.n_chunks >= ((int64_t)1 << 32) ||
      P.n_cv * 8 >= ((int64_t)1 << 32))
    return hipErrorInvalidValue;  // the buffer descriptors' 32-bit byte offsets
  hipError_t e = hipMemsetAsync(P.count, 0, sizeof(int32_t) * (size_t)P.n_nodes, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(sweep_cols_kernel, dim3((unsigned)n_items), dim3(256), 0, st, P);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(sweep_scan_kernel, dim3(1), dim3(1024), 0, st, P.count, P.col_off, P.n_nodes);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(sweep_prep_kernel, dim3((unsigned)n_items), dim3(256), 2 * sizeof(uint32_t) * (size_t)P.k_max, st,
                     P);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const dim3 grid((unsigned)P.n_nodes, (unsigned)P.n_chunks);
  // lanes per occurrence by module size only (one numerical path per shape)
#define NR_SWEEP_LAUNCH(L_)                                                                                    \
  do {                                                                                                         \
    if (P.disc_cv && P.finite)                                                                                 \
      hipLaunchKernelGGL((sweep_column_kernel<true, true, L_>), grid, dim3(kSweepWaves * 64),                  \
                         16 * (size_t)P.chunk_rows, st, P);                                                    \
    else if (P.disc_cv)                                                                                        \
      hipLaunchKernelGGL((sweep_column_kernel<true, false, L_>), grid, dim3(kSweepWaves * 64),                 \
                         16 * (size_t)P.chunk_rows, st, P);                                                    \
    else                                                                                                       \
      hipLaunchKernelGGL((sweep_column_kernel<false, false, L_>), grid, dim3(kSweepWaves * 64),                \
                         8 * (size_t)P.chunk_rows, st, P);                                                     \
  } while (0)
  if (P.k_max > kSweepWideK)
    NR_SWEEP_LAUNCH(16);
  else
    NR_SWEEP_LAUNCH(8);
#undef NR_SWEEP_LAUNCH
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(sweep_finish_kernel, dim3((unsigned)((n_items + 3) / 4)), dim3(256),
                     4 * sizeof(double) * (size_t)P.k_max, st, P, n_items);
  return hipGetLastError();
}

}  // namespace nr
