// Engine layer of the C ABI (include/netrep_gpu.h): per-GPU context, dataset
// residency in HBM, batched permutation launches, progress and cancellation.
//
// Replaces PermutationProcedure's thread pool (src/permutations.cpp:334-380):
// instead of nThreads contiguous chunks of permutations walked one module at a
// time, a launch evaluates every (permutation, module) item of a batch of
// permutations; batches run back to back on one stream, and the host thread
// only polls progress / cancellation between batches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <string>
#include <set>
#include <vector>

#include "../../include/netrep_gpu.h"
#include "kernels.h"
#include "prp.h"
#include "rds_reader.h"

namespace {

thread_local std::string g_create_error;

// Host -> device bytes moved by the library since it was loaded (nr_h2d_bytes):
// every upload path adds what it copies, so a caller can check that a
// resident dataset is not uploaded again.
std::atomic<int64_t> g_h2d_bytes{0};

// Default host threads of the staging copies for new contexts (nr_set_host_threads).
std::atomic<int> g_host_threads{8};

struct DeviceTimer {
  double ms = 0.0;
  int64_t launches = 0;
  int64_t items = 0;
};

}  // namespace

struct nr_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::mutex mu;
  int host_threads = 8;  // host threads of this context's staging copies (nr_ctx_set_host_threads)

  // resident dataset
  double2* d_pairs = nullptr;
  int32_t pairs_es = 1;          // d_pairs element stride in double2: 2 = the Gram table layout,
                                 // 0 = the packed lower triangle (symmetric matrices; pack rule below)
  double* d_colsum = nullptr;    // [n_nodes] column sums of the data (Gram table)
  int64_t table_checked = -1;    // modules_serial the Gram-table decision was made for
  double table_ms = 0.0;         // wall time of the last Gram-table build
  double* d_data = nullptr;
  int64_t n_nodes = 0, n_samples = 0;
  std::vector<std::string> node_names;  // column names of a dataset loaded from files
  int64_t data_gen = 0;                 // bumped by every dataset change (reset_dataset)
  int64_t modules_gen = -1;             // data_gen the modules were validated against
  int64_t modules_serial = 0;           // bumped by every nr_set_modules
  int64_t null_gen = -1;                // data_gen the null pool was validated against
  int symmetric = 0;
  int corr_finite = 0, net_finite = 0;  // CheckFinite of the resident matrices
  int disc_cv_finite = 0;               // the present modules' discovery CorrVector is all finite

  // modules
  int32_t n_rows = 0, n_present = 0, k_max = 0;
  int64_t n_node_total = 0, n_cv_total = 0;
  int64_t null_pos_max = -1;  // largest null-pool position of any module node (-1: none)
  std::vector<int64_t> node_off_h, cv_off_h;
  int32_t* d_row_of = nullptr;
  int64_t* d_node_off = nullptr;
  int64_t* d_cv_off = nullptr;
  int32_t* d_test_idx = nullptr;
  int32_t* d_null_pos = nullptr;
  double* d_disc_cv = nullptr;
  double* d_disc_wd = nullptr;
  double* d_disc_nc = nullptr;
  double* d_cv_shift = nullptr;
  int32_t* d_mod_order = nullptr;
  std::vector<int32_t> order_k_h;  // module sizes in d_mod_order's order (descending)

  // null pool
  int32_t* d_null_idx = nullptr;
  int64_t n_null = 0;

  // run buffers
  double* d_out = nullptr;
  size_t out_cap = 0;
  double* h_stage = nullptr;
  size_t stage_cap = 0;
  uint32_t* d_pi = nullptr;
  size_t pi_cap = 0;
  double* d_scratch = nullptr;
  size_t scratch_cap = 0;
  double* d_net_scratch = nullptr;  // per-workgroup node arrays of modules too large for LDS
  size_t net_scratch_cap = 0;
  int* d_counters = nullptr;  // [0] queue head, [1..4] lanczos diagnostics, [5] flag
  int64_t batch = 0;          // 0 = automatic
  // the second output / staging buffer of run_impl's two batches in flight
  double* d_out2 = nullptr;
  size_t out2_cap = 0;
  double* h_stage2 = nullptr;
  size_t stage2_cap = 0;
  double* h_scale = nullptr;  // nr_scale's pinned staging (4 column chunks)
  size_t scale_cap = 0;
  double* d_scale = nullptr;  // and its device chunks (kept between calls, released as scratch)
  size_t d_scale_cap = 0;
  hipEvent_t ev_copy[2] = {nullptr, nullptr};

  // The observed statistics' own lane (nr_observed_async): stream, scratch and
  // work queue, so that they run beside the first permutation batch instead
  // of ahead of it (at C5 the one-item-per-module launch held the GPU ~85 ms
  // per PermutationProcedure call with 40 workgroups busy).
  hipStream_t obs_stream = nullptr;
  double* obs_scratch = nullptr;
  size_t obs_scratch_cap = 0;
  double* obs_net_scratch = nullptr;
  size_t obs_net_cap = 0;
  int* obs_counters = nullptr;
  double* d_obs = nullptr;
  size_t obs_cap = 0;
  bool obs_pending = false;  // cleared by every change of dataset, modules or null pool

  // the column sweep's per-batch work buffers (sweep.hip), one set per lane
  struct SweepBuf {
    int32_t *col = nullptr, *rank = nullptr, *lrank = nullptr, *count = nullptr, *col_off = nullptr;
    uint32_t *sorted = nullptr, *bndh = nullptr;
    uint4* meta = nullptr;
    double *rec = nullptr, *dabs = nullptr;
    double* zs = nullptr;  // [4] zeros + [256] sink (sweep.hip: lanes with nothing to load / store)
    size_t occ_cap = 0, col_cap = 0;
    int32_t chunk_cap = 0;
  } sweep[2];

  std::atomic<int64_t> done{0}, total{0};
  std::atomic<bool> cancel{false};

  bool timing = false;
  unsigned long long* d_stamps = nullptr;  // phase stamps (nr_set_stamps)
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  bool ev_pending[2] = {false, false};
  DeviceTimer timers[2];
};

namespace {

int fail(nr_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

int hip_fail(nr_ctx* ctx, hipError_t e, const char* what) {
  return fail(ctx, e == hipErrorOutOfMemory ? NR_ERR_OOM : NR_ERR_HIP,
              std::string(what) + ": " + hipGetErrorString(e));
}

#define NR_HIP(ctx, call)                              \
  do {                                                 \
    hipError_t e_ = (call);                            \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, #call); \
  } while (0)

template <typename T>
void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

// Every host -> device copy of the library goes through here (counted).
hipError_t h2d_async(void* dst, const void* src, size_t bytes, hipStream_t st) {
  g_h2d_bytes.fetch_add((int64_t)bytes);
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
}

template <typename T>
int upload(nr_ctx* ctx, T*& dst, const T* src, size_t n) {
  dfree(dst);
  if (n == 0 || src == nullptr) return NR_OK;
  NR_HIP(ctx, hipMalloc((void**)&dst, n * sizeof(T)));
  NR_HIP(ctx, h2d_async(dst, src, n * sizeof(T), ctx->stream));
  return NR_OK;
}

template <typename T>
int ensure(nr_ctx* ctx, T*& buf, size_t& cap, size_t n) {
  if (n <= cap && buf) return NR_OK;
  dfree(buf);
  NR_HIP(ctx, hipMalloc((void**)&buf, n * sizeof(T)));
  cap = n;
  return NR_OK;
}

int ensure_stage(nr_ctx* ctx, double*& h, size_t& cap, size_t n) {
  if (n <= cap && h) return NR_OK;
  if (h) (void)hipHostFree(h);
  h = nullptr;
  NR_HIP(ctx, hipHostMalloc((void**)&h, n * sizeof(double), hipHostMallocDefault));
  cap = n;
  return NR_OK;
}

__global__ void na_fill_kernel(double* p, int64_t n) {
  const double na = __longlong_as_double(0x7FF00000000007A2ll);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = na;
}

__global__ void fill_kernel(double* p, int64_t n, double v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// The Gram's virtual columns behind the resident data block: column N all
// ones, column N + 1 zeros (ProfileParams::ones_off).
int fill_virtual_columns(nr_ctx* ctx, int64_t n_nodes, int64_t n_samples) {
  double* ones = ctx->d_data + n_nodes * n_samples;
  hipLaunchKernelGGL(fill_kernel, dim3(64), dim3(256), 0, ctx->stream, ones, n_samples, 1.0);
  NR_HIP(ctx, hipGetLastError());
  NR_HIP(ctx, hipMemsetAsync(ones + n_samples, 0, (size_t)n_samples * sizeof(double), ctx->stream));
  return NR_OK;
}

int fill_na(nr_ctx* ctx, double* d, int64_t n, hipStream_t st = nullptr) {
  if (n <= 0) return NR_OK;
  const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(na_fill_kernel, dim3(g), dim3(256), 0, st ? st : ctx->stream, d, n);
  NR_HIP(ctx, hipGetLastError());
  return NR_OK;
}

int n_stat_of(const nr_ctx* ctx) { return ctx->d_data ? NR_NSTAT_DATA : NR_NSTAT_NODATA; }

// Bytes of the resident {corr, net} array in its layout (pairs_es).
size_t pair_bytes_of(const nr_ctx* ctx) {
  const size_t n = (size_t)ctx->n_nodes;
  return n * n * sizeof(double2) * (size_t)ctx->pairs_es;
}

// No dataset: buffers freed, shape zero. Modules validated against an earlier
// dataset (their node indices) stop being usable: check_ready demands a new
// nr_set_modules after any dataset change.
// Wait for an observed launch still running on the second lane (before its
// inputs are replaced or freed) and drop its result: nr_observed_wait then
// refuses until nr_observed_async is called again.
void sync_obs(nr_ctx* ctx) {
  if (ctx->obs_stream) (void)hipStreamSynchronize(ctx->obs_stream);
  ctx->obs_pending = false;
}

void reset_dataset(nr_ctx* ctx) {
  sync_obs(ctx);
  dfree(ctx->d_pairs);
  dfree(ctx->d_data);
  dfree(ctx->d_colsum);
  ctx->pairs_es = 1;
  ctx->table_checked = -1;
  ctx->node_names.clear();
  ctx->n_nodes = 0;
  ctx->n_samples = 0;
  ctx->symmetric = 0;
  ctx->corr_finite = ctx->net_finite = 0;
  ++ctx->data_gen;
}

// Lanczos basis columns per item: 160 covers every C2/C3 module (<= 46 steps
// measured); large modules (C5: up to 2,000 nodes, spectra with small gaps)
// get 320.
int profile_m_max(int k_max) { return k_max <= 320 ? std::min(k_max, 160) : 320; }
// Leading dimension of the per-slot Gram: k module columns + the ones column,
// padded to a 32-column super-tile.
int gram_ld(int k_max) { return (k_max + 1 + 31) / 32 * 32; }

// Launch plan of one summary-profile launch (one size class of modules):
//   variant 2: the packed symmetric Gram in global scratch, 4-wave
//              workgroups, 3 per CU (module_profile_packed4_kernel; the
//              compile-time LDS layout of 320-node modules, or a runtime one);
//   variant 0: the full Gram, where the packed layout's LDS does not fit;
//   variant 4: the full Gram with the matvec partials in scratch, where even
//              that does not fit; `big`: the per-node arrays in scratch too
//              (modules beyond the LDS vectors; dual Gram only);
//   variant 6: variant 4 with every Lanczos vector and the index set in
//              scratch (Lanczos dimension min(k, S) beyond the LDS vectors).
// Modules with k > S use the S x S dual Gram. One numerical path per layout:
// no run-time switch selects another (round-2 A/B variants are compile-time
// history, profiles/r02/profile_variants.txt and profiles/r03/).
struct ProfilePlan {
  int variant = 0;
  int slots = 0;
  int per_cu = 1;
  int64_t gram_doubles = 0, stride = 0;
  int k_gram = 0;     // side of the largest Gram (minus the ones column)
  int m = 0;          // Lanczos basis columns
  int kvec = 0;       // LDS vector length
  bool big = false;   // modules beyond kvec (per-node arrays in scratch)
  int64_t basis_doubles = 0;
  int64_t g32_off = 0;  // fp32 Gram copy (relaxed Lanczos steps), 0: none
};

// Queue order of the summary-profile items. Module-major (every permutation
// of the largest module, then the next: largest-first scheduling) balances
// the slots best, but keeps the largest Grams in flight together: at C3 the
// 768 slots' first items (modules of 289-300 nodes, a ~350 KB packed Gram
// plus its Lanczos basis each, ~365 MB) overflow the 256 MiB Infinity Cache,
// so their matvecs stream from HBM. Permutation-major order keeps the size
// mix of the whole launch in flight; its last T permutations (about one
// slot's worth of items) run module-major, largest first, so the slots still
// drain together. It is chosen only where it helps: when the largest items'
// working set would overflow the cache budget and the mix fits it (C3:
// 18.75 -> 18.17 ms); with Grams that overflow it either way (C5, S = 1000:
// 445 vs 387 ms module-major) or fit it either way (C2), module-major.
int profile_order_tail(int slots, const std::vector<int32_t>& k_sorted, int first, int n_mod, int64_t n_perm,
                       int n_samples) {
  if (n_mod <= 1) return 0;
  const int64_t t = (slots + n_mod - 1) / n_mod;
  if (t >= n_perm) return 0;
  // per-slot working set of a module: packed Gram (+ its fp32 copy) and a
  // ~40-column Lanczos basis of the Gram's side
  auto live = [&](int k) {
    const int side = std::min(k, n_samples);
    return (double)nr::packed_gram_doubles(side + 1) * 12.0 + 40.0 * 8.0 * side;
  };
  double mix = 0.0;
  for (int i = 0; i < n_mod; ++i) mix += live(k_sorted[first + i]);
  mix = mix / n_mod * slots;
  double top = 0.0;  // the first `slots` items of module-major order
  int64_t left = slots;
  for (int i = 0; i < n_mod && left > 0; ++i) {
    const int64_t c = std::min<int64_t>(left, n_perm);
    top += live(k_sorted[first + i]) * (double)c;
    left -= c;
  }
  const double budget = 256.0 * (1 << 20);  // the Infinity Cache
  return (top > budget && mix <= budget) ? (int)t : 0;
}

int plan_profile(nr_ctx* ctx, int64_t n_items, int k_max, int n_samples, ProfilePlan* plan, int64_t data_doubles) {
  int dev_cu = 256;
  (void)hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, ctx->device);
  int variant = 2;
  // the dual (S x S) Gram of modules with k > S: the Gram side is min(k, S),
  // and so is every Lanczos dimension (basis columns of that length)
  plan->k_gram = std::min(k_max, n_samples);
  // (its buffer loads take 32-bit byte offsets into the data block)
  if (plan->k_gram <= nr::kWaveDim && data_doubles * 8 < ((int64_t)1 << 31)) {
    // the wave class (kernels.h): one wave per item, the Gram in its
    // registers; the slot's scratch holds the Lanczos basis, and the per-node
    // arrays of modules longer than the LDS vectors
    plan->variant = 7;
    plan->m = nr::kWaveVec;
    plan->kvec = nr::kWaveVec;
    plan->big = k_max > nr::kWaveVec;
    plan->per_cu = nr::profile_wave_per_cu();
    plan->slots = (int)std::max<int64_t>(1, std::min<int64_t>(n_items, (int64_t)dev_cu * plan->per_cu));
    plan->gram_doubles = 0;
    plan->basis_doubles = (int64_t)plan->k_gram * nr::kWaveVec;
    plan->stride = plan->basis_doubles + (plan->big ? 5 * (int64_t)k_max : 0);
    plan->stride = (plan->stride + 31) / 32 * 32;
    plan->g32_off = 0;
    return NR_OK;
  }
  if (plan->k_gram <= nr::kSmallDim) {
    // the small class (kernels.h): several small-workgroup items per CU;
    // modules longer than its LDS vectors keep their per-node arrays in the
    // slot's scratch
    plan->variant = 5;
    plan->m = nr::kSmallDim;
    plan->kvec = nr::kSmallDim;
    plan->big = k_max > nr::kSmallDim;
    plan->per_cu = nr::profile_small_per_cu();
    plan->slots = (int)std::max<int64_t>(1, std::min<int64_t>(n_items, (int64_t)dev_cu * plan->per_cu));
    plan->gram_doubles = nr::packed_gram_doubles(plan->k_gram + 1);
    plan->basis_doubles = (int64_t)plan->k_gram * nr::kSmallDim;
    plan->stride = plan->gram_doubles + plan->basis_doubles + (plan->big ? 5 * (int64_t)k_max : 0);
    plan->stride = (plan->stride + 31) / 32 * 32;
    plan->g32_off = plan->stride;
    plan->stride += (plan->gram_doubles / 2 + 31) / 32 * 32;
    return NR_OK;
  }
  const int mg = profile_m_max(plan->k_gram);
  plan->m = mg;
  int kvec = k_max;
  plan->big = false;
  if (nr::profile_kernel_lds(kvec, mg, n_samples, 2) > 160 * 1024) {
    // Large modules on the packed Gram too (half the Lanczos bytes of the
    // full ld x ld Gram): LDS vectors as long as fit, and the per-node arrays
    // of modules longer than them in the slot's scratch, as long as every
    // Lanczos dimension min(k, S) fits the vectors.
    int kp = (k_max + 15) / 16 * 16;
    while (kp > 16 && nr::profile_kernel_lds(kp, mg, n_samples, 2) > 160 * 1024) kp -= 16;
    if (plan->k_gram <= kp) {
      kvec = kp;
      plan->big = k_max > kp;
    } else {
      variant = 0;
    }
  }
  // Large modules: the per-wave matvec partials (4 x k doubles) move from LDS
  // to the slot's scratch, which leaves LDS for the six Lanczos vectors only.
  if (variant == 0 && nr::profile_kernel_lds(kvec, mg, n_samples, 0) > 160 * 1024) variant = 4;
  // Modules beyond even those vectors (any k up to N, as src/netStats.cpp:
  // 217-280): Lanczos runs on the dual Gram (dimension S <= kvec) and their
  // per-node arrays live in the slot's scratch; where the Lanczos dimension
  // min(k, S) itself can exceed the LDS vectors (S > kvec), every vector and
  // the index set move to the slot's scratch too (variant 6: no size limit
  // but device memory).
  if (variant == 4 && nr::profile_kernel_lds(kvec, mg, n_samples, 4) > 160 * 1024) {
    kvec = nr::profile_kvec_max(mg);
    if (n_samples > kvec) {
      variant = 6;
      kvec = k_max;
    } else {
      plan->big = true;
    }
  }
  plan->kvec = kvec;
  const size_t lds = nr::profile_kernel_lds(kvec, mg, n_samples, variant);
  if (lds > 160 * 1024)
    return fail(ctx, NR_ERR_UNSUPPORTED, "module too large for the summary-profile kernel's LDS budget");
  const int want = variant == 4 || variant == 6 ? 1 : 3;
  const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(want, (160 * 1024) / lds));
  plan->variant = variant;
  plan->per_cu = per_cu;
  plan->slots = (int)std::max<int64_t>(1, std::min<int64_t>(n_items, (int64_t)dev_cu * per_cu));
  if (variant == 2) {
    const int64_t kc = plan->k_gram + 1;
    plan->gram_doubles = nr::packed_gram_doubles((int)kc);  // packed triangle in chunked column groups
  } else {
    const int64_t ld = gram_ld(plan->k_gram);
    plan->gram_doubles = ld * ld;
  }
  plan->basis_doubles = (int64_t)plan->k_gram * mg;
  plan->stride = plan->gram_doubles + plan->basis_doubles +
                 (variant == 4 || variant == 6 ? (int64_t)nr::kProfileWaves * kvec : 0) +
                 (plan->big ? 5 * (int64_t)k_max : 0) +  // x.u, means, squares, contributions, index set
                 (variant == 6 ? 6 * (int64_t)kvec + (kvec + 1) / 2 : 0);  // six vectors + index set
  plan->g32_off = 0;
  if (variant == 2) {  // fp32 copy of the packed Gram at the slot's end (relaxed Lanczos steps)
    plan->stride = (plan->stride + 31) / 32 * 32;
    plan->g32_off = plan->stride;
    plan->stride += (plan->gram_doubles / 2 + 31) / 32 * 32;
  }
  return NR_OK;
}

// The device resources one stream of launches uses: the permutation batches
// run on the context's own (main_lane), the observed statistics of a
// PermutationProcedure call on a second set (obs_lane) beside them.
struct Lane {
  hipStream_t st;
  double** scratch;
  size_t* scratch_cap;
  double** net_scratch;
  size_t* net_cap;
  int* counters;  // [0] queue head, [1..4] Lanczos diagnostics
  bool timed;     // kernel timers (nr_set_timing) follow the main lane only
  int id;         // 0 = main, 1 = observed (the lane's side stream)
};

Lane main_lane(nr_ctx* ctx) {
  return {ctx->stream, &ctx->d_scratch, &ctx->scratch_cap, &ctx->d_net_scratch, &ctx->net_scratch_cap,
          ctx->d_counters, true, 0};
}

Lane obs_lane(nr_ctx* ctx) {
  return {ctx->obs_stream, &ctx->obs_scratch, &ctx->obs_scratch_cap, &ctx->obs_net_scratch, &ctx->obs_net_cap,
          ctx->obs_counters, false, 1};
}

// Summary-profile launches over the module order sorted by size (descending,
// k_sorted[i] = size of d_order[i]), one per size class, each with its own
// work queue, k_max and layout: the modules beyond the packed kernel's
// compile-time 320-node layout first (full or runtime-layout Gram), then the
// rest on the packed kernel at 3 workgroups per CU. (Round 2 launched every
// module on the layout of the largest one: at C5 the small modules ran on the
// one-workgroup-per-CU full-Gram kernel too.)
int launch_profiles(nr_ctx* ctx, nr::ProfileParams pp, const int32_t* d_order,
                    const std::vector<int32_t>& k_sorted, int64_t n_perm, const Lane& ln,
                    const nr::NetParams* table_np = nullptr, int* fused_from = nullptr) {
  const hipStream_t st = ln.st;
  const int n_mod = (int)k_sorted.size();
  int n_big = 0;
  while (n_big < n_mod && k_sorted[n_big] > nr::kPackedLayoutK) ++n_big;
  struct Seg {
    int first, count;
    ProfilePlan plan;
  } seg[2];
  int ns = 0;
  if (n_big > 0) seg[ns++] = {0, n_big, {}};
  if (n_big < n_mod) seg[ns++] = {n_big, n_mod - n_big, {}};
  // every segment's scratch (slots x stride) is one allocation, carved in turn
  int64_t total = 0;
  bool fuse[2] = {false, false};
  int fuse_kind[2] = {0, 0};  // ProfileParams::fused
  for (int i = 0; i < ns; ++i) {
    const int rc = plan_profile(ctx, (int64_t)seg[i].count * n_perm, k_sorted[seg[i].first], (int)pp.n_samples,
                                &seg[i].plan, pp.ones_off + 2 * pp.n_samples);
    if (rc) return rc;
    // Gram table: the packed class (compile-time layout, no dual items) takes
    // its network statistics and Gram from the table's gathers, on the table
    // kernel's own workgroup shape
    const int k_max = k_sorted[seg[i].first];
    const bool fuse_table = table_np && table_np->es == 2 && seg[i].plan.variant == 2 &&
                            k_max <= nr::kPackedLayoutK && k_max <= pp.n_samples &&
                            nr::fused_net_fits(nr::kPackedLayoutK, std::min(nr::kPackedLayoutK, 160), nr::kTableWaves);
    fuse_kind[i] = fuse_table ? 1 : 0;
    fuse[i] = fuse_kind[i] != 0;
    total = std::max<int64_t>(total, seg[i].plan.stride * seg[i].plan.slots);
  }
  // segments run one after the other on one stream: they share the scratch
  if (int rc = ensure(ctx, *ln.scratch, *ln.scratch_cap, (size_t)total)) return rc;
  for (int i = 0; i < ns; ++i) {
    const ProfilePlan& plan = seg[i].plan;
    const int k_max = k_sorted[seg[i].first];
    pp.mod_order = d_order + seg[i].first;
    pp.n_items = (int32_t)((int64_t)seg[i].count * n_perm);
    pp.k_max = k_max;
    pp.ld = gram_ld(plan.k_gram);
    pp.m_max = plan.m;
    pp.kvec = plan.kvec;
    pp.basis_doubles = plan.basis_doubles;
    pp.gram_doubles = plan.gram_doubles;
    pp.scratch = *ln.scratch;
    pp.scratch_stride = plan.stride;
    pp.part_global = plan.variant == 4 || plan.variant == 6 ? 1 : 0;
    pp.vec_global = plan.variant == 6 ? 1 : 0;
    pp.order_tail =
        profile_order_tail(plan.slots, k_sorted, seg[i].first, seg[i].count, n_perm, (int)pp.n_samples);
    pp.g32_off = plan.g32_off;
    pp.fused = fuse_kind[i];
    if (pp.fused) {
      pp.net = *table_np;
      pp.net.mod_order = pp.mod_order;
      if (fused_from) *fused_from = seg[i].first;
    }
    NR_HIP(ctx, hipMemsetAsync(pp.queue, 0, sizeof(int), st));
    NR_HIP(ctx, nr::launch_profile(pp, plan.slots, plan.variant, plan.per_cu, st));
  }
  return NR_OK;
}

// Kernel timers: events on the kernel's own stream; collected (synchronised)
// only after both kernels of a batch are enqueued, so timing does not
// serialise the two streams.
void timer_begin(nr_ctx* ctx, int which, hipStream_t st) {
  if (ctx->timing) (void)hipEventRecord(ctx->ev[2 * which], st);
}

void timer_end(nr_ctx* ctx, int which, int64_t items, hipStream_t st) {
  if (!ctx->timing) return;
  (void)hipEventRecord(ctx->ev[2 * which + 1], st);
  ctx->ev_pending[which] = true;
  ctx->timers[which].launches += 1;
  ctx->timers[which].items += items;
}

void timer_collect(nr_ctx* ctx) {
  for (int which = 0; which < 2; ++which) {
    if (!ctx->ev_pending[which]) continue;
    ctx->ev_pending[which] = false;
    (void)hipEventSynchronize(ctx->ev[2 * which + 1]);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, ctx->ev[2 * which], ctx->ev[2 * which + 1]);
    ctx->timers[which].ms += ms;
  }
}

nr::IndexSource make_source(const nr_ctx* ctx, int mode, uint64_t seed, int64_t perm_base,
                            const uint32_t* d_pi, const int32_t* direct) {
  nr::IndexSource s;
  s.mode = mode;
  s.seed = seed;
  s.perm_base = perm_base;
  s.n_null = (uint32_t)ctx->n_null;
  s.null_idx = ctx->d_null_idx;
  s.null_pos = ctx->d_null_pos;
  s.pi = d_pi;
  s.direct_idx = direct;
  return s;
}

// Network kernel scratch for modules whose per-node arrays exceed LDS: a
// persistent grid of two workgroups per CU, each with its own slot.
int prepare_net(nr_ctx* ctx, nr::NetParams& np, int64_t n_items, const Lane& ln) {
  if (!nr::net_kernel_big(np.k_max)) return NR_OK;
  int dev_cu = 256;
  (void)hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, ctx->device);
  const int64_t slots = std::max<int64_t>(1, std::min<int64_t>(n_items, 2 * (int64_t)dev_cu));
  const int64_t per = (int64_t)(nr::net_big_slot_bytes(np.k_max) / sizeof(double));
  const int rc = ensure(ctx, *ln.net_scratch, *ln.net_cap, (size_t)(per * slots));
  if (rc) return rc;
  np.big_scratch = *ln.net_scratch;
  np.big_stride = per;
  np.big_slots = (int32_t)slots;
  return NR_OK;
}

// Network-statistics launches over the size-sorted module order: modules
// whose per-node arrays do not fit LDS first (global-scratch workgroups), the
// rest in the ordinary one-workgroup-per-item launch with their own k_max.
int launch_nets(nr_ctx* ctx, nr::NetParams np, const int32_t* d_order, const std::vector<int32_t>& k_sorted,
                int64_t n_perm, const Lane& ln) {
  const int n_mod = (int)k_sorted.size();
  int n_big = 0;
  while (n_big < n_mod && nr::net_kernel_big(k_sorted[n_big])) ++n_big;
  const int first[2] = {0, n_big}, count[2] = {n_big, n_mod - n_big};
  for (int i = 0; i < 2; ++i) {
    if (count[i] == 0) continue;
    nr::NetParams q = np;
    q.mod_order = d_order + first[i];
    q.k_max = k_sorted[first[i]];
    const int64_t items = (int64_t)count[i] * n_perm;
    const int rc = prepare_net(ctx, q, items, ln);
    if (rc) return rc;
    NR_HIP(ctx, nr::launch_net(q, items, ln.st));
  }
  return NR_OK;
}

// The column sweep for one batch (sweep.hip) on the lane's buffers.
// Sub-batches of at most kSweepMaxOcc (permutation, node) occurrences (int32
// occurrence ids, bounded buffers); an item's statistics do not depend on
// the batch it runs in, so neither do the results.
constexpr int64_t kSweepMaxOcc = (int64_t)64 << 20;
// nr_debug_set test knobs (neither changes a result): a smaller sub-batch
// bound, and an injected failure of the n-th sweep buffer allocation.
std::atomic<int64_t> g_sweep_max_occ{kSweepMaxOcc};
std::atomic<int> g_fail_sweep_alloc{0};
constexpr int64_t kSweepMaxRecBytes = (int64_t)32 << 30;  // the (occurrence, chunk) records of one sub-batch

int launch_sweep_sub(nr_ctx* ctx, const nr::NetParams& np, int64_t n_perm, const Lane& ln);

int launch_sweep_batch(nr_ctx* ctx, const nr::NetParams& np, int64_t n_perm, const Lane& ln) {
  // occurrences per sub-batch: at most kSweepMaxOcc, and records of at most
  // kSweepMaxRecBytes (many column chunks at large n)
  const int64_t chunks =
      (ctx->n_nodes + nr::sweep_chunk_rows(ctx->n_nodes, np.disc_cv ? 16 : 8) - 1) /
      nr::sweep_chunk_rows(ctx->n_nodes, np.disc_cv ? 16 : 8);
  const int64_t max_occ = std::min<int64_t>(g_sweep_max_occ.load(), kSweepMaxRecBytes / (chunks * 8 * nr::kSweepRec));
  const int64_t per = std::max<int64_t>(1, max_occ / std::max<int64_t>(ctx->n_node_total, 1));
  for (int64_t p0 = 0; p0 < n_perm; p0 += per) {
    const int64_t np_sub = std::min(per, n_perm - p0);
    nr::NetParams q = np;
    q.src.perm_base = np.src.perm_base + p0;
    if (q.src.mode == nr::NR_IDX_TABLE) q.src.pi = np.src.pi + p0 * (int64_t)np.src.n_null;
    q.out = np.out + p0 * (int64_t)np.n_rows * np.n_stat;
    if (int rc = launch_sweep_sub(ctx, q, np_sub, ln)) return rc;
  }
  return NR_OK;
}

int launch_sweep_sub(nr_ctx* ctx, const nr::NetParams& np, int64_t n_perm, const Lane& ln) {
  nr_ctx::SweepBuf& b = ctx->sweep[ln.id];
  const size_t n_occ = (size_t)(n_perm * ctx->n_node_total);
  nr::SweepParams P{};
  P.chunk_rows = nr::sweep_chunk_rows(ctx->n_nodes, np.disc_cv ? 16 : 8);
  P.n_chunks = (int32_t)((ctx->n_nodes + P.chunk_rows - 1) / P.chunk_rows);
  // Every buffer of a set is freed before it is reallocated, so a set's
  // capacity is committed only once the whole chain has succeeded: after an
  // allocation failure the capacity reads 0 and the next call reallocates
  // instead of launching on the freed (null) pointers.
  auto grow = [&](auto*& ptr, size_t need, size_t per) -> int {
    dfree(ptr);
    if (g_fail_sweep_alloc.load() > 0 && g_fail_sweep_alloc.fetch_sub(1) == 1)
      return fail(ctx, NR_ERR_OOM, "sweep buffers: injected allocation failure (nr_debug_set)");
    NR_HIP(ctx, hipMalloc((void**)&ptr, std::max<size_t>(need, 1) * per));
    return NR_OK;
  };
  int rc;
  if (n_occ > b.occ_cap || P.n_chunks > b.chunk_cap) {
    b.occ_cap = 0;
    b.chunk_cap = 0;
    if ((rc = grow(b.col, n_occ, 4)) || (rc = grow(b.rank, n_occ, 4)) || (rc = grow(b.sorted, n_occ, 4)) ||
        (rc = grow(b.lrank, n_occ, 4)) || (rc = grow(b.meta, n_occ, 2 * sizeof(uint4))) ||
        (rc = grow(b.bndh, P.n_chunks > 2 ? n_occ : 0, 4 * (size_t)P.n_chunks)) ||
        (rc = grow(b.rec, n_occ, 8 * nr::kSweepRec * (size_t)P.n_chunks)))
      return rc;
    b.occ_cap = n_occ;
    b.chunk_cap = P.n_chunks;
  }
  if (!b.zs) {
    NR_HIP(ctx, hipMalloc((void**)&b.zs, (4 + 256) * sizeof(double)));
    NR_HIP(ctx, hipMemsetAsync(b.zs, 0, 4 * sizeof(double), ln.st));
  }
  const size_t n_cols = (size_t)ctx->n_nodes + 1;
  if (n_cols > b.col_cap) {
    b.col_cap = 0;
    if ((rc = grow(b.count, n_cols, 4)) || (rc = grow(b.col_off, n_cols, 4)) || (rc = grow(b.dabs, n_cols, 8)))
      return rc;
    b.col_cap = n_cols;
  }
  P.pairs = np.pairs;
  P.n_nodes = ctx->n_nodes;
  P.es = np.es;
  P.src = np.src;
  P.n_node_total = ctx->n_node_total;
  P.n_present = ctx->n_present;
  P.node_off = ctx->d_node_off;
  P.mod_order = ctx->d_mod_order;
  P.cv_off = ctx->d_cv_off;
  P.disc_cv = np.disc_cv;
  P.n_cv = ctx->n_cv_total;
  P.finite = ctx->corr_finite && ctx->disc_cv_finite;
  P.disc_wd = np.disc_wd;
  P.cv_shift = np.cv_shift;
  P.n_perm = (int32_t)n_perm;
  P.k_max = ctx->k_max;
  P.n_occ = (int64_t)n_occ;
  P.col = b.col;
  P.sorted = b.sorted;
  P.rank = b.rank;
  P.count = b.count;
  P.col_off = b.col_off;
  P.dabs = b.dabs;
  P.zero = b.zs;
  P.sink = b.zs + 4;
  P.meta = b.meta;
  P.bndh = b.bndh;
  P.lrank = b.lrank;
  P.rec = b.rec;
  P.row_of = np.row_of;
  P.n_rows = np.n_rows;
  P.n_stat = np.n_stat;
  P.slot_avg_weight = np.slot_avg_weight;
  P.slot_cor_cor = np.slot_cor_cor;
  P.slot_cor_degree = np.slot_cor_degree;
  P.slot_avg_cor = np.slot_avg_cor;
  P.out = np.out;
  NR_HIP(ctx, nr::launch_sweep(P, ln.st));
  return NR_OK;
}

// Launch the statistics kernels for n_perm permutations (or the observed /
// direct sets when src.mode == NR_IDX_DIRECT, n_perm == 1) into d_out.
int launch_batch(nr_ctx* ctx, const nr::IndexSource& src, int64_t n_perm, double* d_out, const Lane& ln) {
  const int n_stat = n_stat_of(ctx);
  const bool data = ctx->d_data != nullptr;
  NR_HIP(ctx, hipSetDevice(ctx->device));
  int rc = fill_na(ctx, d_out, (int64_t)ctx->n_rows * n_stat * n_perm, ln.st);
  if (rc) return rc;
  if (ctx->n_present == 0) return NR_OK;
  const int64_t n_items = (int64_t)ctx->n_present * n_perm;

  nr::NetParams np{};
  np.pairs = ctx->d_pairs;
  np.es = ctx->pairs_es;
  np.colsum = ctx->d_colsum;
  np.n_nodes = ctx->n_nodes;
  np.symmetric = ctx->symmetric;
  np.src = src;
  np.node_off = ctx->d_node_off;
  np.cv_off = ctx->d_cv_off;
  np.disc_cv = ctx->d_disc_cv;
  np.disc_wd = ctx->d_disc_wd;
  np.cv_shift = ctx->d_cv_shift;
  np.mod_order = ctx->d_mod_order;
  np.n_perm = (int32_t)n_perm;
  np.k_max = ctx->k_max;
  np.row_of = ctx->d_row_of;
  np.n_rows = ctx->n_rows;
  np.n_stat = n_stat;
  // slots: data path src/permutations.cpp:95-101; network-only src/permutationsNoData.cpp:82-85
  np.slot_avg_weight = 0;
  np.slot_cor_cor = data ? 2 : 1;
  np.slot_cor_degree = data ? 3 : 2;
  np.slot_avg_cor = data ? 5 : 3;
  np.out = d_out;
  // The network statistics are their own launch (module_net_kernel) ahead of
  // the summary-profile launches, on the same stream -- except with the Gram
  // table, where the packed profile launch computes them for its modules
  // from the same gathers that fill its Gram (launch_profiles reports from
  // which module on, in size order, it did). (Round 2 measured the network
  // phase fused into the profile items without the table at +0.7%, within
  // run-to-run noise, and on a concurrent stream at -11%.)
  const bool table = data && ctx->pairs_es == 2;
  // Without the Gram table the network statistics of every present module
  // come from the column sweep (sweep.hip: each test column streamed into LDS
  // once per batch) where the shapes allow it (n < 65,536, modules of at most
  // 4,096 nodes); the item-major gather kernel otherwise. The choice depends
  // on the shapes only.
  if (!table && nr::sweep_supported(ctx->n_nodes, ctx->k_max)) {
    if (ln.timed) timer_begin(ctx, 0, ln.st);
    if ((rc = launch_sweep_batch(ctx, np, n_perm, ln))) return rc;
    if (ln.timed) timer_end(ctx, 0, n_items, ln.st);
  }
  auto nets = [&](int n_mod) -> int {
    if (n_mod <= 0) return NR_OK;
    std::vector<int32_t> ks(ctx->order_k_h.begin(), ctx->order_k_h.begin() + n_mod);
    if (ln.timed) timer_begin(ctx, 0, ln.st);
    if (int r2 = launch_nets(ctx, np, ctx->d_mod_order, ks, n_perm, ln)) return r2;
    if (ln.timed) timer_end(ctx, 0, (int64_t)n_mod * n_perm, ln.st);
    return NR_OK;
  };
  if (!table && !nr::sweep_supported(ctx->n_nodes, ctx->k_max) && (rc = nets(ctx->n_present))) return rc;

  if (data) {
    nr::ProfileParams pp{};
    pp.data = ctx->d_data;
    pp.n_samples = ctx->n_samples;
    pp.ones_off = ctx->n_nodes * ctx->n_samples;
    pp.src = src;
    pp.node_off = ctx->d_node_off;
    pp.disc_nc = ctx->d_disc_nc;
    pp.n_perm = (int32_t)n_perm;
    pp.row_of = ctx->d_row_of;
    pp.n_rows = ctx->n_rows;
    pp.n_stat = n_stat;
    pp.slot_coherence = 1;
    pp.slot_cor_contrib = 4;
    pp.slot_avg_contrib = 6;
    pp.out = d_out;
    pp.queue = ln.counters;
    pp.diag = ln.counters + 1;
    pp.stamps = ln.timed ? ctx->d_stamps : nullptr;
    int fused_from = ctx->n_present;
    if (ln.timed) timer_begin(ctx, 1, ln.st);
    rc = launch_profiles(ctx, pp, ctx->d_mod_order, ctx->order_k_h, n_perm, ln, table ? &np : nullptr,
                         &fused_from);
    if (rc) return rc;
    if (ln.timed) timer_end(ctx, 1, n_items, ln.st);
    if (table && (rc = nets(fused_from))) return rc;
  }
  if (ln.timed) timer_collect(ctx);
  return NR_OK;
}

// The Gram table ("Gram table"): the data block's whole Gram
// X^T X (2 S n^2 flops on the matrix cores, once per dataset) interleaved
// with {corr, net} as {corr, net}, {gram, net^T} per element, so that a packed
// profile item reads its network values and its Gram entries in one 32-byte
// gather per pair instead of a separate network launch plus a per-item
// matrix-core Gram.
//
// The decision depends on shapes only -- never on free device memory -- so
// the numerical path of a dataset/module set is fixed (the table path and the
// per-item matrix-core Gram differ at the 1e-12 level): the table is built
// when (1) the packed-class segment (modules of <= 320 nodes) would be ONE
// fused launch of the packed kernel, i.e. launch_profiles' own rule: its
// plan is variant 2 (not the small class, min(k, S) > 112) and none of its
// modules has more nodes than samples; (2) that segment carries at least
// half of the present modules' Gram work; (3) n^2 fits kTableMaxElems (the
// build holds 56 bytes per matrix element: pairs, X^T X and the table). A
// failed allocation is NR_ERR_OOM, not a silent switch to the other path.
constexpr int64_t kTableMaxElems = (int64_t)50000 * 50000;  // n <= 50,000: 140 GB during the build

bool table_wanted(nr_ctx* ctx) {
  if (!ctx->d_data || ctx->n_present == 0) return false;
  const int64_t S = ctx->n_samples, n = ctx->n_nodes;
  if (n * n > kTableMaxElems) return false;
  double packed_w = 0.0, total_w = 0.0;
  int32_t packed_max = 0;
  for (const int32_t k : ctx->order_k_h) {
    const double kd = (double)k, Sd = (double)S;
    const double w = k <= S ? Sd * kd * kd : kd * Sd * Sd;  // the Gram's flops / 2
    total_w += w;
    if (k <= nr::kPackedLayoutK) {
      packed_w += w;
      packed_max = std::max(packed_max, k);
    }
  }
  if (packed_max == 0 || packed_max > S || packed_w < 0.5 * total_w) return false;
  // A fixed per-device bound, not the free memory (the numerical
  // path must not depend on what else holds the device): the build's peak,
  // 56 bytes per matrix element (the {corr, net} pairs, the Gram and the
  // widened table), within 60% of the device's total HBM.
  {
    size_t total = 0;
    if (hipDeviceTotalMem(&total, ctx->device) != hipSuccess) return false;
    if ((double)n * (double)n * 56.0 > 0.6 * (double)total) return false;
  }
  ProfilePlan plan;
  if (plan_profile(ctx, 1, packed_max, (int)S, &plan, (int64_t)n * S + 2 * (int64_t)S) != NR_OK) return false;
  return plan.variant == 2 &&
         nr::fused_net_fits(nr::kPackedLayoutK, std::min(nr::kPackedLayoutK, 160), nr::kTableWaves);
}

int maybe_build_table(nr_ctx* ctx) {
  if (ctx->table_checked == ctx->modules_serial) return NR_OK;
  ctx->table_checked = ctx->modules_serial;
  if (ctx->pairs_es == 2 || !table_wanted(ctx)) return NR_OK;
  const int64_t S = ctx->n_samples, n = ctx->n_nodes;
  const size_t nn = (size_t)n * (size_t)n;
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (ctx->obs_stream) NR_HIP(ctx, hipStreamSynchronize(ctx->obs_stream));
  const auto t_build = std::chrono::steady_clock::now();
  double* gram = nullptr;
  double2* tab = nullptr;
  double* cs = nullptr;
  auto drop = [&]() {
    dfree(gram);
    dfree(tab);
    dfree(cs);
  };
  if (hipMalloc((void**)&gram, nn * sizeof(double)) != hipSuccess ||
      hipMalloc((void**)&tab, 2 * nn * sizeof(double2)) != hipSuccess ||
      hipMalloc((void**)&cs, (size_t)n * sizeof(double)) != hipSuccess) {
    drop();
    (void)hipGetLastError();
    ctx->table_checked = -1;  // a later call tries again
    return fail(ctx, NR_ERR_OOM,
                "Gram table allocation failed: " + std::to_string((nn * 40) >> 20) +
                    " MiB beside the resident matrices (40 bytes per matrix element; the table path is chosen "
                    "from the shapes, DESIGN.md section 5.2)");
  }
  hipError_t e = nr::launch_gram_full(ctx->d_data, S, n, gram, cs, ctx->stream);
  if (e == hipSuccess)
    e = nr::launch_widen_pairs(ctx->d_pairs, gram, tab, n, ctx->symmetric, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    drop();
    return hip_fail(ctx, e, "Gram table");
  }
  dfree(gram);
  dfree(ctx->d_pairs);
  ctx->d_pairs = tab;
  ctx->d_colsum = cs;
  ctx->pairs_es = 2;
  ctx->table_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_build).count();
  return NR_OK;
}

int64_t auto_batch(const nr_ctx* ctx) {
  if (ctx->batch > 0) return ctx->batch;
  // Enough items to fill the 768 profile slots many times over, so the
  // launch tail (slots draining at different times) stays short: C3 at 1,024
  // permutations (51,200 items) per launch runs 3.5% faster than at 256
  // (profiles/r02/profile_variants.txt). Per-slot scratch does not depend on it.
  const int64_t items_target = ctx->d_data ? 51200 : 65536;
  int64_t b = std::max<int64_t>(1, items_target / std::max<int32_t>(ctx->n_present, 1));
  if (ctx->d_data) {
    // ... but launches of heavy modules stay short (~0.1 s), so progress and
    // interrupts keep their one-second cadence (src/thread-utils.cpp:49-82):
    // at most 2e12 Gram flops (2 S k min(S, k) per module) per launch; C3 at
    // 1,024 permutations is 1.7e12, C5 (k up to 2,000, S = 1,000) gets 66 (64 after the rounding below).
    double per_perm = 0.0;
    for (const int32_t k : ctx->order_k_h) {
      const double kk = (double)k, s = (double)ctx->n_samples;
      per_perm += 2.0 * s * kk * std::min(s, kk);
    }
    if (per_perm > 0.0) b = std::min<int64_t>(b, std::max<int64_t>(1, (int64_t)(2e12 / per_perm)));
  }
  // whole multiples of 64 (16 below 64) permutations: the one-workgroup-per-CU
  // classes then fill whole rounds of the 256 CUs more often (C5's 66 -> 64:
  // network launch 17.46 -> 15.94 ms per launch, 6% per permutation,
  // profiles/r04/c5gap/); results do not depend on the batch
  b = b >= 64 ? b / 64 * 64 : (b >= 16 ? b / 16 * 16 : b);
  return b;
}

int check_ready(nr_ctx* ctx, bool need_null) {
  if (!ctx->d_pairs) return fail(ctx, NR_ERR_INVALID, "no dataset: call nr_set_dataset first");
  if (ctx->n_rows <= 0) return fail(ctx, NR_ERR_INVALID, "no modules: call nr_set_modules first");
  if (ctx->modules_gen != ctx->data_gen)
    return fail(ctx, NR_ERR_INVALID, "the modules were set for another dataset: call nr_set_modules again");
  if (need_null && ctx->n_present > 0 && (!ctx->d_null_idx || !ctx->d_null_pos))
    return fail(ctx, NR_ERR_INVALID, "no null pool: call nr_set_null_pool and pass null_pos");
  if (need_null && ctx->n_present > 0 && ctx->null_gen != ctx->data_gen)
    return fail(ctx, NR_ERR_INVALID, "the null pool was set for another dataset: call nr_set_null_pool again");
  // Every permuted index is null_idx[pi(null_pos)]: a position outside the pool
  // would be read out of bounds on the device.
  if (need_null && ctx->n_present > 0 && ctx->null_pos_max >= ctx->n_null)
    return fail(ctx, NR_ERR_INVALID, "null_pos outside the null pool (a module node position >= n_null)");
  return NR_OK;
}

// An explicit shuffle table must hold n_perm x n_null entries, each < n_null
// (pi[p][q] is a null-pool position). Checked before anything is launched.
int check_pi_host(nr_ctx* ctx, const uint32_t* pi, int64_t n_perm) {
  const uint64_t n = (uint64_t)n_perm * (uint64_t)ctx->n_null;
  const uint32_t lim = (uint32_t)ctx->n_null;
  uint32_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) bad |= (uint32_t)(pi[i] >= lim);
  return bad ? fail(ctx, NR_ERR_INVALID, "pi holds an entry >= n_null (explicit shuffles are null-pool positions)")
             : NR_OK;
}

__global__ void pi_check_kernel(const uint32_t* __restrict__ pi, int64_t n, uint32_t lim, int* flag) {
  int bad = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    bad |= pi[i] >= lim;
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

int check_pi_device(nr_ctx* ctx, const uint32_t* d_pi, int64_t n_perm) {
  const int64_t n = n_perm * ctx->n_null;
  if (n == 0) return NR_OK;
  NR_HIP(ctx, hipMemsetAsync(ctx->d_counters + 6, 0, sizeof(int), ctx->stream));
  const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(pi_check_kernel, dim3(g), dim3(256), 0, ctx->stream, d_pi, n, (uint32_t)ctx->n_null,
                     ctx->d_counters + 6);
  NR_HIP(ctx, hipGetLastError());
  int bad = 0;
  NR_HIP(ctx, hipMemcpyAsync(&bad, ctx->d_counters + 6, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return bad ? fail(ctx, NR_ERR_INVALID, "pi holds an entry >= n_null (explicit shuffles are null-pool positions)")
             : NR_OK;
}

int run_impl(nr_ctx* ctx, int64_t b, int64_t e, uint64_t seed, const uint32_t* pi, bool pi_on_device,
             double* nulls, bool nulls_on_device) {
  int rc = check_ready(ctx, true);
  if (rc) return rc;
  if ((rc = maybe_build_table(ctx))) return rc;
  if (e < b) return fail(ctx, NR_ERR_INVALID, "perm_end < perm_begin");
  const int n_stat = n_stat_of(ctx);
  const int64_t slice = (int64_t)ctx->n_rows * n_stat;
  const int64_t batch = auto_batch(ctx);
  ctx->done = 0;
  ctx->total = e - b;
  NR_HIP(ctx, hipSetDevice(ctx->device));
  if (pi && e > b) {
    rc = pi_on_device ? check_pi_device(ctx, pi, e - b) : check_pi_host(ctx, pi, e - b);
    if (rc) return rc;
  }
  // A cancellation (nr_cancel, from any thread, before or during the run) is
  // honoured between launches: the slices not yet computed are left NA, as
  // the reference's interrupted workers leave their part of the NA-filled cube
  // (src/permutations.cpp:375-384), and the flag is consumed.
  auto cancelled = [&](int64_t p_stop) -> int {
    ctx->cancel = false;
    const double na = [] { uint64_t u = 0x7FF00000000007A2ull; double d; std::memcpy(&d, &u, 8); return d; }();
    if (nulls_on_device) {
      int r2 = fill_na(ctx, nulls + (p_stop - b) * slice, (e - p_stop) * slice);
      if (r2) return r2;
      NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    } else {
      std::fill(nulls + (p_stop - b) * slice, nulls + (e - b) * slice, na);
    }
    return fail(ctx, NR_ERR_CANCELLED, "permutation procedure cancelled");
  };
  // Host output: two batches in flight. Batch i+1 is enqueued behind batch
  // i's copy to pinned memory, so the device does not idle while the host
  // moves batch i's slices into `nulls` (drain).
  struct Pending {
    int64_t p0 = -1, np = 0;
    int slot = 0;
  } pend;
  double* h_slot[2] = {nullptr, nullptr};
  auto drain = [&]() -> int {
    if (pend.p0 < 0) return NR_OK;
    NR_HIP(ctx, hipEventSynchronize(ctx->ev_copy[pend.slot]));
    std::memcpy(nulls + (pend.p0 - b) * slice, h_slot[pend.slot], (size_t)(pend.np * slice) * sizeof(double));
    ctx->done += pend.np;
    pend.p0 = -1;
    return NR_OK;
  };
  if (!nulls_on_device)
    for (auto& ev : ctx->ev_copy)
      if (!ev) NR_HIP(ctx, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  int slot = 0;
  for (int64_t p0 = b; p0 < e; p0 += batch, slot ^= 1) {
    if (ctx->cancel.load()) {
      if ((rc = drain())) return rc;
      return cancelled(p0);
    }
    const int64_t np = std::min(batch, e - p0);
    const uint32_t* d_pi = nullptr;
    if (pi) {
      if (pi_on_device) {
        d_pi = pi + (p0 - b) * ctx->n_null;
      } else {
        rc = ensure(ctx, ctx->d_pi, ctx->pi_cap, (size_t)(np * ctx->n_null));
        if (rc) return rc;
        NR_HIP(ctx, h2d_async(ctx->d_pi, pi + (p0 - b) * ctx->n_null,
                              (size_t)(np * ctx->n_null) * sizeof(uint32_t), ctx->stream));
        d_pi = ctx->d_pi;
      }
    }
    const nr::IndexSource src =
        make_source(ctx, pi ? nr::NR_IDX_TABLE : nr::NR_IDX_PRP, seed, p0, d_pi, nullptr);
    double* d_out;
    if (nulls_on_device) {
      d_out = nulls + (p0 - b) * slice;
    } else {
      rc = slot == 0 ? ensure(ctx, ctx->d_out, ctx->out_cap, (size_t)(np * slice))
                     : ensure(ctx, ctx->d_out2, ctx->out2_cap, (size_t)(np * slice));
      if (rc) return rc;
      d_out = slot == 0 ? ctx->d_out : ctx->d_out2;
    }
    rc = launch_batch(ctx, src, np, d_out, main_lane(ctx));
    if (rc) return rc;
    if (!nulls_on_device) {
      rc = slot == 0 ? ensure_stage(ctx, ctx->h_stage, ctx->stage_cap, (size_t)(np * slice))
                     : ensure_stage(ctx, ctx->h_stage2, ctx->stage2_cap, (size_t)(np * slice));
      if (rc) return rc;
      h_slot[slot] = slot == 0 ? ctx->h_stage : ctx->h_stage2;
      NR_HIP(ctx, hipMemcpyAsync(h_slot[slot], d_out, (size_t)(np * slice) * sizeof(double),
                                 hipMemcpyDeviceToHost, ctx->stream));
      NR_HIP(ctx, hipEventRecord(ctx->ev_copy[slot], ctx->stream));
      if ((rc = drain())) return rc;   // the previous batch, while this one runs
      pend.p0 = p0;
      pend.np = np;
      pend.slot = slot;
    } else {
      NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
      ctx->done += np;
    }
  }
  if ((rc = drain())) return rc;
  ctx->cancel = false;  // a cancellation that arrives after the last launch has nothing left to stop
  return NR_OK;
}

}  // namespace

extern "C" {

int nr_device_count(int* count) {
  if (!count) return NR_ERR_INVALID;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *count = n;
  return NR_OK;
}

int nr_ctx_create(int device, nr_ctx** out) {
  if (!out) return NR_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    g_create_error = "no HIP device available (the MI355X engine has no CPU fallback)";
    return NR_ERR_HIP;
  }
  if (device < 0 || device >= n) {
    g_create_error = "device index out of range";
    return NR_ERR_INVALID;
  }
  nr_ctx* ctx = new nr_ctx();
  ctx->device = device;
  ctx->host_threads = g_host_threads.load();
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  for (int i = 0; i < 4 && e == hipSuccess; ++i) e = hipEventCreate(&ctx->ev[i]);
  if (e == hipSuccess) e = hipMalloc((void**)&ctx->d_counters, 16 * sizeof(int));
  if (e == hipSuccess) e = hipMemset(ctx->d_counters, 0, 16 * sizeof(int));
  if (e != hipSuccess) {
    g_create_error = std::string("context creation failed: ") + hipGetErrorString(e);
    nr_ctx_destroy(ctx);
    return NR_ERR_HIP;
  }
  *out = ctx;
  return NR_OK;
}

void nr_ctx_destroy(nr_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  sync_obs(ctx);
  dfree(ctx->d_pairs);
  dfree(ctx->d_data);
  dfree(ctx->d_colsum);
  dfree(ctx->d_row_of);
  dfree(ctx->d_node_off);
  dfree(ctx->d_cv_off);
  dfree(ctx->d_test_idx);
  dfree(ctx->d_null_pos);
  dfree(ctx->d_disc_cv);
  dfree(ctx->d_disc_wd);
  dfree(ctx->d_disc_nc);
  dfree(ctx->d_cv_shift);
  dfree(ctx->d_mod_order);
  for (auto& b : ctx->sweep) {
    dfree(b.col);
    dfree(b.rank);
    dfree(b.count);
    dfree(b.col_off);
    dfree(b.sorted);
    dfree(b.meta);
    dfree(b.bndh);
    dfree(b.lrank);
    dfree(b.dabs);
    dfree(b.zs);
    dfree(b.rec);
  }
  dfree(ctx->d_null_idx);
  dfree(ctx->d_out);
  dfree(ctx->d_pi);
  dfree(ctx->d_scratch);
  dfree(ctx->d_net_scratch);
  dfree(ctx->d_counters);
  dfree(ctx->d_stamps);
  dfree(ctx->d_out2);
  dfree(ctx->obs_scratch);
  dfree(ctx->obs_net_scratch);
  dfree(ctx->obs_counters);
  dfree(ctx->d_obs);
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  if (ctx->h_stage2) (void)hipHostFree(ctx->h_stage2);
  if (ctx->h_scale) (void)hipHostFree(ctx->h_scale);
  dfree(ctx->d_scale);
  for (auto& ev : ctx->ev)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& ev : ctx->ev_copy)
    if (ev) (void)hipEventDestroy(ev);
  if (ctx->obs_stream) (void)hipStreamDestroy(ctx->obs_stream);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* nr_last_error(const nr_ctx* ctx) {
  return ctx ? ctx->err.c_str() : g_create_error.c_str();
}

// Default host threads of the staging copies for contexts created later
// (process-wide); a context's own count is nr_ctx_set_host_threads (the
// reference-interface calls set it from nCores on their contexts only).
int nr_set_host_threads(int n) {
  g_host_threads = n <= 0 ? 8 : std::min(n, 16);
  return NR_OK;
}

int nr_get_host_threads(void) { return g_host_threads.load(); }

int nr_ctx_set_host_threads(nr_ctx* ctx, int n) {
  if (!ctx) return NR_ERR_INVALID;
  ctx->host_threads = n <= 0 ? 8 : std::min(n, 16);
  return NR_OK;
}

int nr_h2d_bytes(int64_t* bytes) {
  if (!bytes) return NR_ERR_INVALID;
  *bytes = g_h2d_bytes.load();
  return NR_OK;
}

// Copy n doubles with up to `threads` host threads (pageable -> pinned staging).
static void parallel_copy(double* dst, const double* src, int64_t n, int threads,
                          int64_t min_part = (int64_t)1 << 20 /* 8 MiB per thread at least */) {
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n / min_part));
  if (nt == 1) {
    std::memcpy(dst, src, (size_t)n * sizeof(double));
    return;
  }
  std::vector<std::thread> th;
  const int64_t part = (n + nt - 1) / nt;
  for (int t = 0; t < nt; ++t) {
    const int64_t a = t * part, b = std::min(n, a + part);
    if (a < b) th.emplace_back([=]() { std::memcpy(dst + a, src + a, (size_t)(b - a) * sizeof(double)); });
  }
  for (auto& x : th) x.join();
}

// Two independent copies in one fork-join, split over the threads in
// proportion to their lengths (nr_scale: one chunk in, the previous out).
static void parallel_copy2(double* d1, const double* s1, int64_t n1, double* d2, const double* s2, int64_t n2,
                           int threads, int64_t min_part) {
  const int64_t n = n1 + n2;
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n / min_part));
  if (nt == 1) {
    if (n1) std::memcpy(d1, s1, (size_t)n1 * sizeof(double));
    if (n2) std::memcpy(d2, s2, (size_t)n2 * sizeof(double));
    return;
  }
  std::vector<std::thread> th;
  const int64_t part = (n + nt - 1) / nt;
  for (int t = 0; t < nt; ++t) {
    const int64_t a = t * part, b = std::min(n, a + part);
    if (a >= b) continue;
    th.emplace_back([=]() {  // [a, b) of the concatenation of the two ranges
      if (a < n1) std::memcpy(d1 + a, s1 + a, (size_t)(std::min(b, n1) - a) * sizeof(double));
      if (b > n1) {
        const int64_t a2 = std::max(a, n1) - n1, b2 = b - n1;
        std::memcpy(d2 + a2, s2 + a2, (size_t)(b2 - a2) * sizeof(double));
      }
    });
  }
  for (auto& x : th) x.join();
}

// Host matrices to HBM through pinned, double-buffered chunks: host threads
// fill pinned buffer b with chunk i+1 (from the caller's pageable arrays)
// while the copy engine moves chunk i and, for the corr/net pair, the
// interleave kernel packs it into the {corr, net} layout. `net` NULL: a plain
// copy of `corr` into `dst_plain`. net == corr (NetProps: the network doubles
// as the unused correlation operand): the matrix crosses PCIe once and fills
// both halves of the pairs.
static int upload_pinned(nr_ctx* ctx, const double* corr, const double* net, int64_t n_elem, double2* dst_pairs,
                         double* dst_plain, hipStream_t st) {
  const bool same = net != nullptr && net == corr;
  const int parts = net && !same ? 2 : 1;
  const int threads = ctx->host_threads;
  const int64_t chunk = std::min<int64_t>(n_elem, (int64_t)1 << 23);  // 64 MiB per matrix per chunk
  double* h[2] = {nullptr, nullptr};
  double* d[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipError_t e = hipSuccess;
  for (int b = 0; b < 2 && e == hipSuccess; ++b) {
    e = hipHostMalloc((void**)&h[b], (size_t)(parts * chunk) * sizeof(double), hipHostMallocDefault);
    if (e == hipSuccess && net) e = hipMalloc((void**)&d[b], (size_t)(parts * chunk) * sizeof(double));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev[b], hipEventDisableTiming);
  }
  int64_t i = 0;
  for (int64_t o = 0; o < n_elem && e == hipSuccess; o += chunk, ++i) {
    const int b = (int)(i & 1);
    const int64_t len = std::min(chunk, n_elem - o);
    if (i >= 2) e = hipEventSynchronize(ev[b]);  // chunk i-2 has left buffer b
    if (e != hipSuccess) break;
    parallel_copy(h[b], corr + o, len, threads);
    if (parts == 2) parallel_copy(h[b] + chunk, net + o, len, threads);
    if (net) {
      e = h2d_async(d[b], h[b], (size_t)len * sizeof(double), st);
      if (e == hipSuccess && parts == 2) e = h2d_async(d[b] + chunk, h[b] + chunk, (size_t)len * sizeof(double), st);
      if (e == hipSuccess) e = nr::launch_interleave(d[b], parts == 2 ? d[b] + chunk : d[b], dst_pairs + o, len, st);
    } else {
      e = h2d_async(dst_plain + o, h[b], (size_t)len * sizeof(double), st);
    }
    if (e == hipSuccess) e = hipEventRecord(ev[b], st);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  for (int b = 0; b < 2; ++b) {
    if (h[b]) (void)hipHostFree(h[b]);
    if (d[b]) (void)hipFree(d[b]);
    if (ev[b]) (void)hipEventDestroy(ev[b]);
  }
  if (e != hipSuccess) return hip_fail(ctx, e, "dataset upload");
  return NR_OK;
}

namespace {
int set_dataset_impl(nr_ctx* ctx, const double* corr, const double* net, const double* data,
                     int64_t n_nodes, int64_t n_samples, int where, int flags);
}

int nr_set_dataset(nr_ctx* ctx, const double* corr, const double* net, const double* data,
                   int64_t n_nodes, int64_t n_samples, int where) {
  return nr_set_dataset_ex(ctx, corr, net, data, n_nodes, n_samples, where, 0);
}

int nr_set_dataset_ex(nr_ctx* ctx, const double* corr, const double* net, const double* data,
                      int64_t n_nodes, int64_t n_samples, int where, int flags) {
  if (!ctx) return NR_ERR_INVALID;
  if (flags & ~NR_SCALE_DATA) return fail(ctx, NR_ERR_INVALID, "unknown nr_set_dataset_ex flags");
  if (!corr || !net || n_nodes <= 0) return fail(ctx, NR_ERR_INVALID, "corr/net missing or n_nodes <= 0");
  if (data && n_samples < 2) return fail(ctx, NR_ERR_INVALID, "data needs n_samples >= 2");
  if (n_nodes > (int64_t)INT32_MAX) return fail(ctx, NR_ERR_UNSUPPORTED, "n_nodes exceeds 2^31-1");
  NR_HIP(ctx, hipSetDevice(ctx->device));
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  reset_dataset(ctx);
  const int rc = set_dataset_impl(ctx, corr, net, data, n_nodes, n_samples, where, flags);
  if (rc != NR_OK) {
    (void)hipStreamSynchronize(ctx->stream);
    reset_dataset(ctx);
  }
  return rc;
}

namespace {
int set_dataset_impl(nr_ctx* ctx, const double* corr, const double* net, const double* data,
                     int64_t n_nodes, int64_t n_samples, int where, int flags) {
  const int64_t n_elem = n_nodes * n_nodes;
  NR_HIP(ctx, hipMalloc((void**)&ctx->d_pairs, (size_t)n_elem * sizeof(double2)));
  if (where == NR_DEVICE) {
    NR_HIP(ctx, nr::launch_interleave(corr, net, ctx->d_pairs, n_elem, ctx->stream));
  } else {
    const int rc = upload_pinned(ctx, corr, net, n_elem, ctx->d_pairs, nullptr, ctx->stream);
    if (rc) return rc;
  }
  NR_HIP(ctx, hipMemsetAsync(ctx->d_counters + 5, 0, sizeof(int), ctx->stream));
  NR_HIP(ctx, nr::launch_symmetry(ctx->d_pairs, n_nodes, ctx->d_counters + 5, ctx->stream));
  int asym = 0;
  NR_HIP(ctx, hipMemcpyAsync(&asym, ctx->d_counters + 5, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  if (data) {
    const size_t bytes = (size_t)(n_samples * n_nodes) * sizeof(double);
    NR_HIP(ctx, hipMalloc((void**)&ctx->d_data, bytes + 2 * (size_t)n_samples * sizeof(double)));
    if (int rc = fill_virtual_columns(ctx, n_nodes, n_samples)) return rc;
    // NR_SCALE_DATA: the raw data goes to a device buffer and is scaled there
    // (Scale, src/scale.cpp:14-25) straight into the resident block
    double* raw = nullptr;
    if (flags & NR_SCALE_DATA) NR_HIP(ctx, hipMalloc((void**)&raw, bytes));
    double* dst = raw ? raw : ctx->d_data;
    int rc = NR_OK;
    if (where == NR_DEVICE) {
      const hipError_t e = hipMemcpyAsync(dst, data, bytes, hipMemcpyDeviceToDevice, ctx->stream);
      if (e != hipSuccess) rc = hip_fail(ctx, e, "data copy");
    } else {
      rc = upload_pinned(ctx, data, nullptr, n_samples * n_nodes, nullptr, dst, ctx->stream);
    }
    if (!rc && raw) {
      hipError_t e = nr::launch_scale(raw, ctx->d_data, n_samples, n_nodes, ctx->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
      if (e != hipSuccess) rc = hip_fail(ctx, e, "scale");
    }
    if (raw) (void)hipFree(raw);
    if (rc) return rc;
  }
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->symmetric = (asym & 1) ? 0 : 1;
  ctx->corr_finite = (asym & 2) ? 0 : 1;
  ctx->net_finite = (asym & 4) ? 0 : 1;
  ctx->n_nodes = n_nodes;
  ctx->n_samples = data ? n_samples : 0;
  return NR_OK;
}
}  // namespace

// File -> pinned -> HBM for one matrix payload: the host inflates / reads
// straight into pinned buffer b while the copy engine moves the previous one
// and a kernel converts it from XDR into `pairs` (half 0 / 1) or `plain`.
static int upload_file_matrix(nr_ctx* ctx, nr::RMatrixReader& rd, double2* pairs, int half, double* plain,
                              hipStream_t st) {
  const int64_t n = rd.length();
  const int64_t chunk = std::min<int64_t>(std::max<int64_t>(n, 1), (int64_t)1 << 23);  // 64 MiB
  double* h[2] = {nullptr, nullptr};
  double* d[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipError_t e = hipSuccess;
  for (int b = 0; b < 2 && e == hipSuccess; ++b) {
    e = hipHostMalloc((void**)&h[b], (size_t)chunk * sizeof(double), hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc((void**)&d[b], (size_t)chunk * sizeof(double));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev[b], hipEventDisableTiming);
  }
  bool read_ok = true;
  int64_t i = 0;
  for (int64_t o = 0; o < n && e == hipSuccess && read_ok; o += chunk, ++i) {
    const int b = (int)(i & 1);
    const int64_t len = std::min(chunk, n - o);
    if (i >= 2) e = hipEventSynchronize(ev[b]);
    if (e != hipSuccess) break;
    read_ok = rd.read_raw(h[b], len);
    if (!read_ok) break;
    e = h2d_async(d[b], h[b], (size_t)len * sizeof(double), st);
    if (e == hipSuccess) e = nr::launch_xdr(d[b], pairs ? pairs + o : nullptr, half, plain ? plain + o : nullptr, len, st);
    if (e == hipSuccess) e = hipEventRecord(ev[b], st);
  }
  const hipError_t e2 = hipStreamSynchronize(st);
  if (e == hipSuccess) e = e2;
  for (int b = 0; b < 2; ++b) {
    if (h[b]) (void)hipHostFree(h[b]);
    if (d[b]) (void)hipFree(d[b]);
    if (ev[b]) (void)hipEventDestroy(ev[b]);
  }
  if (!read_ok) return fail(ctx, NR_ERR_INVALID, rd.error());
  if (e != hipSuccess) return hip_fail(ctx, e, "file upload");
  return NR_OK;
}

namespace {
int set_dataset_files_impl(nr_ctx* ctx, const char* corr_path, const char* net_path, const char* data_path,
                           const char* corr_object, const char* net_object, const char* data_object,
                           int scale_data) {
  nr::RMatrixReader rc_, rn_;
  if (!rc_.open(corr_path, corr_object)) return fail(ctx, NR_ERR_INVALID, std::string(corr_path) + ": " + rc_.error());
  if (!rn_.open(net_path, net_object)) return fail(ctx, NR_ERR_INVALID, std::string(net_path) + ": " + rn_.error());
  const int64_t n_elem = rc_.length();
  int64_t n_nodes = (int64_t)std::llround(std::sqrt((double)n_elem));
  if (n_nodes <= 0 || n_nodes * n_nodes != n_elem) return fail(ctx, NR_ERR_INVALID, "correlation matrix is not square");
  if (rn_.length() != n_elem) return fail(ctx, NR_ERR_INVALID, "network and correlation matrices differ in size");
  if (n_nodes > (int64_t)INT32_MAX) return fail(ctx, NR_ERR_UNSUPPORTED, "n_nodes exceeds 2^31-1");
  NR_HIP(ctx, hipMalloc((void**)&ctx->d_pairs, (size_t)n_elem * sizeof(double2)));
  int rc;
  nr::RMatrixMeta mc, mn;
  if ((rc = upload_file_matrix(ctx, rc_, ctx->d_pairs, 0, nullptr, ctx->stream))) return rc;
  if (!rc_.finish(&mc)) return fail(ctx, NR_ERR_INVALID, std::string(corr_path) + ": " + rc_.error());
  if ((rc = upload_file_matrix(ctx, rn_, ctx->d_pairs, 1, nullptr, ctx->stream))) return rc;
  if (!rn_.finish(&mn)) return fail(ctx, NR_ERR_INVALID, std::string(net_path) + ": " + rn_.error());
  if (mc.nrow != n_nodes || mc.ncol != n_nodes || mn.nrow != n_nodes || mn.ncol != n_nodes)
    return fail(ctx, NR_ERR_INVALID, "correlation / network matrices must be square and of one size");
  // R/check-user-input.R:750-771: row and column names of each square matrix
  // agree, and the node order is the same in correlation, network and data
  if ((!mc.rownames.empty() && !mc.colnames.empty() && mc.rownames != mc.colnames) ||
      (!mn.rownames.empty() && !mn.colnames.empty() && mn.rownames != mn.colnames))
    return fail(ctx, NR_ERR_INVALID, "mismatch between row and column names in 'correlation' / 'network'");
  if (!mc.colnames.empty() && !mn.colnames.empty() && mc.colnames != mn.colnames)
    return fail(ctx, NR_ERR_INVALID, "mismatch in node order between 'data', 'correlation', and 'network'");
  const std::vector<std::string> names = !mn.colnames.empty() ? mn.colnames : mc.colnames;
  int64_t n_samples = 0;
  if (data_path) {
    nr::RMatrixReader rd;
    if (!rd.open(data_path, data_object)) return fail(ctx, NR_ERR_INVALID, std::string(data_path) + ": " + rd.error());
    if (rd.length() % n_nodes != 0) return fail(ctx, NR_ERR_INVALID, "data matrix columns do not match the network");
    n_samples = rd.length() / n_nodes;
    if (n_samples < 2) return fail(ctx, NR_ERR_INVALID, "data needs n_samples >= 2");
    double* raw = nullptr;
    NR_HIP(ctx, hipMalloc((void**)&raw, (size_t)rd.length() * sizeof(double)));
    rc = upload_file_matrix(ctx, rd, nullptr, 0, raw, ctx->stream);
    nr::RMatrixMeta md;
    if (!rc && !rd.finish(&md)) rc = fail(ctx, NR_ERR_INVALID, std::string(data_path) + ": " + rd.error());
    if (!rc && (md.nrow != n_samples || md.ncol != n_nodes))
      rc = fail(ctx, NR_ERR_INVALID, "data matrix must be samples x nodes");
    if (!rc && !md.colnames.empty() && !names.empty() && md.colnames != names)
      rc = fail(ctx, NR_ERR_INVALID, "mismatch in node order between 'data', 'correlation', and 'network'");
    hipError_t e = hipSuccess;
    if (!rc) e = hipMalloc((void**)&ctx->d_data, (size_t)(n_samples * (n_nodes + 2)) * sizeof(double));
    // Scale (src/scale.cpp:14-25) on the device, as the R code scales after loading
    if (!rc && e == hipSuccess)
      e = scale_data ? nr::launch_scale(raw, ctx->d_data, n_samples, n_nodes, ctx->stream)
                     : hipMemcpyAsync(ctx->d_data, raw, (size_t)(n_samples * n_nodes) * sizeof(double),
                                      hipMemcpyDeviceToDevice, ctx->stream);
    if (!rc && e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    (void)hipFree(raw);
    if (rc) return rc;
    if (e != hipSuccess) return hip_fail(ctx, e, "data upload");
    if ((rc = fill_virtual_columns(ctx, n_nodes, n_samples))) return rc;
  }
  NR_HIP(ctx, hipMemsetAsync(ctx->d_counters + 5, 0, sizeof(int), ctx->stream));
  NR_HIP(ctx, nr::launch_symmetry(ctx->d_pairs, n_nodes, ctx->d_counters + 5, ctx->stream));
  int asym = 0;
  NR_HIP(ctx, hipMemcpyAsync(&asym, ctx->d_counters + 5, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->symmetric = (asym & 1) ? 0 : 1;
  ctx->corr_finite = (asym & 2) ? 0 : 1;
  ctx->net_finite = (asym & 4) ? 0 : 1;
  // committed only once everything above has succeeded
  ctx->node_names = names;
  ctx->n_nodes = n_nodes;
  ctx->n_samples = n_samples;
  return NR_OK;
}
}  // namespace

int nr_set_dataset_files(nr_ctx* ctx, const char* corr_path, const char* net_path, const char* data_path,
                         const char* corr_object, const char* net_object, const char* data_object,
                         int scale_data) {
  if (!ctx) return NR_ERR_INVALID;
  if (!corr_path || !net_path) return fail(ctx, NR_ERR_INVALID, "corr/net file missing");
  NR_HIP(ctx, hipSetDevice(ctx->device));
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  // The old dataset is dropped first; on any failure the context is left with
  // no dataset at all (never a new buffer with the old shape), and modules
  // set for the old dataset are invalidated either way.
  reset_dataset(ctx);
  int rc;
  try {
    rc = set_dataset_files_impl(ctx, corr_path, net_path, data_path, corr_object, net_object, data_object,
                                scale_data);
  } catch (const std::bad_alloc&) {
    rc = fail(ctx, NR_ERR_OOM, "host memory allocation failed");
  } catch (const std::exception& ex) {
    rc = fail(ctx, NR_ERR_INVALID, std::string("internal error: ") + ex.what());
  }
  if (rc != NR_OK) {
    (void)hipStreamSynchronize(ctx->stream);
    reset_dataset(ctx);
  }
  return rc;
}

int nr_dataset_shape(const nr_ctx* ctx, int64_t* n_nodes, int64_t* n_samples) {
  if (!ctx) return NR_ERR_INVALID;
  if (n_nodes) *n_nodes = ctx->n_nodes;
  if (n_samples) *n_samples = ctx->n_samples;
  return NR_OK;
}

int nr_dataset_colnames(const nr_ctx* ctx, char* buf, int64_t cap, int64_t* needed) {
  if (!ctx || !needed) return NR_ERR_INVALID;
  int64_t total = 0;
  for (const std::string& s : ctx->node_names) total += (int64_t)s.size() + 1;
  *needed = total;
  if (!buf || cap < total) return NR_OK;
  for (const std::string& s : ctx->node_names) {
    std::memcpy(buf, s.c_str(), s.size() + 1);
    buf += s.size() + 1;
  }
  return NR_OK;
}

int nr_copy_dataset(nr_ctx* dst, const nr_ctx* src) {
  if (!dst || !src || dst == src) return NR_ERR_INVALID;
  if (!src->d_pairs) return fail(dst, NR_ERR_INVALID, "source context has no dataset");
  NR_HIP(dst, hipSetDevice(dst->device));
  NR_HIP(dst, hipStreamSynchronize(dst->stream));
  reset_dataset(dst);  // on a failure below dst is left with no dataset
  const size_t pair_bytes = pair_bytes_of(src);
  NR_HIP(dst, hipMalloc((void**)&dst->d_pairs, pair_bytes));
  if (src->d_colsum) NR_HIP(dst, hipMalloc((void**)&dst->d_colsum, (size_t)src->n_nodes * sizeof(double)));
  const size_t data_bytes = (size_t)(src->n_samples * (src->n_nodes + 2)) * sizeof(double);  // + virtual columns
  if (src->d_data) NR_HIP(dst, hipMalloc((void**)&dst->d_data, data_bytes));
  // Device to device: over xGMI between GPUs, an on-device copy when both
  // contexts share a GPU. The source must be idle (its upload synchronised).
  NR_HIP(dst, hipMemcpyPeerAsync(dst->d_pairs, dst->device, src->d_pairs, src->device, pair_bytes, dst->stream));
  if (src->d_data)
    NR_HIP(dst, hipMemcpyPeerAsync(dst->d_data, dst->device, src->d_data, src->device, data_bytes, dst->stream));
  if (src->d_colsum)
    NR_HIP(dst, hipMemcpyPeerAsync(dst->d_colsum, dst->device, src->d_colsum, src->device,
                                   (size_t)src->n_nodes * sizeof(double), dst->stream));
  NR_HIP(dst, hipStreamSynchronize(dst->stream));
  dst->pairs_es = src->pairs_es;
  dst->n_nodes = src->n_nodes;
  dst->n_samples = src->n_samples;
  dst->node_names = src->node_names;
  dst->symmetric = src->symmetric;
  dst->corr_finite = src->corr_finite;
  dst->net_finite = src->net_finite;
  return NR_OK;
}

// One resident dataset to n - 1 other contexts ("broadcast once
// per test dataset"), bandwidth-optimal on a full xGMI mesh: a scatter and an
// all-gather of peer copies. Each buffer is cut into n - 1 pieces. Phase 1:
// piece p goes from the source to context p + 1 (every source link busy at
// once, B / (n-1) bytes each). Phase 2: context p + 1 forwards piece p to the
// other n - 2 destinations over its own direct links, each copy behind the
// event that marks the piece's arrival. Every link carries at most
// B / (n-1) per phase: 2B / ((n-1) L) in all, against B / L for a direct
// fan-out (each destination pulls all B over its one link to the source) or
// a single pipelined ring (DESIGN.md section 7 has the arithmetic). The source
// must be idle; on failure every destination is left with no dataset.
// Peer access between every pair of distinct GPUs a broadcast uses, in both
// directions (the scatter reads GPU 0 from each destination's stream, the
// all-gather reads every destination from every other): direct copies over
// the xGMI links instead of copies staged through host memory
// (src/permutations.cpp:335-380 is the reference's one-process parallel
// section this replaces). Enabled once per ordered pair per process. A pair
// without peer access still works -- hipMemcpyPeerAsync stages it through
// host memory -- at PCIe speed; such pairs are recorded
// (nr_peer_staged_pairs) instead of failing the broadcast.
static std::mutex g_peer_mu;
static std::set<std::pair<int, int>> g_peer_on, g_peer_staged;

static int enable_peer_access(nr_ctx* err_ctx, const std::vector<int>& devs) {
  std::lock_guard<std::mutex> lk(g_peer_mu);
  for (int a : devs)
    for (int b : devs) {
      if (a == b || g_peer_on.count({a, b}) || g_peer_staged.count({a, b})) continue;
      int can = 0;
      NR_HIP(err_ctx, hipDeviceCanAccessPeer(&can, a, b));
      if (!can) {
        g_peer_staged.insert({a, b});
        continue;
      }
      NR_HIP(err_ctx, hipSetDevice(a));
      const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return hip_fail(err_ctx, e, "hipDeviceEnablePeerAccess");
      (void)hipGetLastError();  // clears hipErrorPeerAccessAlreadyEnabled
      g_peer_on.insert({a, b});
    }
  return NR_OK;
}

int nr_peer_staged_pairs(int* n) {
  if (!n) return NR_ERR_INVALID;
  std::lock_guard<std::mutex> lk(g_peer_mu);
  *n = (int)g_peer_staged.size();
  return NR_OK;
}

// The calling thread's current device, restored on every return path.
struct DeviceRestore {
  int dev = -1;
  DeviceRestore() {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  ~DeviceRestore() {
    if (dev >= 0) (void)hipSetDevice(dev);
  }
};

int nr_broadcast_dataset(nr_ctx* const* ctxs, int n) {
  if (!ctxs || n < 1) return NR_ERR_INVALID;
  DeviceRestore restore;
  nr_ctx* src = ctxs[0];
  if (!src) return NR_ERR_INVALID;
  for (int g = 1; g < n; ++g)
    for (int h = 0; h < g; ++h)
      if (!ctxs[g] || ctxs[g] == ctxs[h]) return fail(src, NR_ERR_INVALID, "broadcast: contexts must be distinct");
  if (!src->d_pairs) return fail(src, NR_ERR_INVALID, "source context has no dataset");
  if (n == 1) return NR_OK;
  {
    std::vector<int> devs;
    for (int g = 0; g < n; ++g)
      if (std::find(devs.begin(), devs.end(), ctxs[g]->device) == devs.end()) devs.push_back(ctxs[g]->device);
    if (int rc = enable_peer_access(src, devs)) return rc;
  }
  const int parts = n - 1;
  struct Buf {
    const char* s;
    std::vector<char*> d;
    size_t bytes;
  };
  std::vector<Buf> bufs;
  const size_t pair_bytes = pair_bytes_of(src);
  const size_t data_bytes = (size_t)(src->n_samples * (src->n_nodes + 2)) * sizeof(double);  // + virtual columns
  const size_t cs_bytes = (size_t)src->n_nodes * sizeof(double);
  bufs.push_back({reinterpret_cast<const char*>(src->d_pairs), std::vector<char*>(n, nullptr), pair_bytes});
  if (src->d_data) bufs.push_back({reinterpret_cast<const char*>(src->d_data), std::vector<char*>(n, nullptr), data_bytes});
  if (src->d_colsum)
    bufs.push_back({reinterpret_cast<const char*>(src->d_colsum), std::vector<char*>(n, nullptr), cs_bytes});
  auto clear_all = [&]() {
    for (int g = 1; g < n; ++g) {
      (void)hipSetDevice(ctxs[g]->device);
      (void)hipStreamSynchronize(ctxs[g]->stream);
      reset_dataset(ctxs[g]);
    }
  };
  for (int g = 1; g < n; ++g) {
    nr_ctx* d = ctxs[g];
    NR_HIP(d, hipSetDevice(d->device));
    NR_HIP(d, hipStreamSynchronize(d->stream));
    reset_dataset(d);
    hipError_t e = hipMalloc((void**)&d->d_pairs, pair_bytes);
    if (e == hipSuccess && src->d_data) e = hipMalloc((void**)&d->d_data, data_bytes);
    if (e == hipSuccess && src->d_colsum) e = hipMalloc((void**)&d->d_colsum, cs_bytes);
    if (e != hipSuccess) {
      const int rc = hip_fail(d, e, "broadcast allocation");
      clear_all();
      return fail(src, rc, d->err);
    }
    size_t b = 0;
    bufs[b++].d[g] = reinterpret_cast<char*>(d->d_pairs);
    if (src->d_data) bufs[b++].d[g] = reinterpret_cast<char*>(d->d_data);
    if (src->d_colsum) bufs[b++].d[g] = reinterpret_cast<char*>(d->d_colsum);
  }
  auto piece = [&](size_t bytes, int p, size_t* a, size_t* len) {
    const size_t per = ((bytes + parts - 1) / parts + 255) / 256 * 256;
    *a = std::min(bytes, (size_t)p * per);
    *len = std::min(bytes, *a + per) - *a;
  };
  NR_HIP(src, hipSetDevice(src->device));
  NR_HIP(src, hipStreamSynchronize(src->stream));
  std::vector<hipEvent_t> ev(parts, nullptr);
  hipError_t e = hipSuccess;
  // phase 1: the scatter
  for (int p = 0; p < parts && e == hipSuccess; ++p) {
    nr_ctx* d = ctxs[p + 1];
    e = hipSetDevice(d->device);
    for (const Buf& bf : bufs) {
      size_t a, len;
      piece(bf.bytes, p, &a, &len);
      if (e == hipSuccess && len)
        e = hipMemcpyPeerAsync(bf.d[p + 1] + a, d->device, bf.s + a, src->device, len, d->stream);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev[p], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ev[p], d->stream);
  }
  // phase 2: the all-gather among the destinations
  for (int g = 1; g < n && e == hipSuccess; ++g) {
    nr_ctx* d = ctxs[g];
    e = hipSetDevice(d->device);
    for (int p = 0; p < parts && e == hipSuccess; ++p) {
      if (p == g - 1) continue;
      e = hipStreamWaitEvent(d->stream, ev[p], 0);
      for (const Buf& bf : bufs) {
        size_t a, len;
        piece(bf.bytes, p, &a, &len);
        if (e == hipSuccess && len)
          e = hipMemcpyPeerAsync(bf.d[g] + a, d->device, bf.d[p + 1] + a, ctxs[p + 1]->device, len, d->stream);
      }
    }
  }
  for (int g = 1; g < n; ++g) {
    const hipError_t e2 = hipSetDevice(ctxs[g]->device);
    const hipError_t e3 = hipStreamSynchronize(ctxs[g]->stream);
    if (e == hipSuccess) e = e2 != hipSuccess ? e2 : e3;
  }
  for (hipEvent_t x : ev)
    if (x) (void)hipEventDestroy(x);
  if (e != hipSuccess) {
    const int rc = hip_fail(src, e, "dataset broadcast");
    clear_all();
    return rc;
  }
  for (int g = 1; g < n; ++g) {
    nr_ctx* d = ctxs[g];
    d->pairs_es = src->pairs_es;
    d->n_nodes = src->n_nodes;
    d->n_samples = src->n_samples;
    d->node_names = src->node_names;
    d->symmetric = src->symmetric;
    d->corr_finite = src->corr_finite;
    d->net_finite = src->net_finite;
    d->table_ms = src->table_ms;
  }
  return NR_OK;
}

int nr_clear_dataset(nr_ctx* ctx) {
  if (!ctx) return NR_ERR_INVALID;
  NR_HIP(ctx, hipSetDevice(ctx->device));
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  reset_dataset(ctx);
  ctx->cancel = false;  // a context cancelled after its run returned starts clean
  return NR_OK;
}

// The per-batch work buffers (the column sweep's sets, the profile slots'
// scratch, the device output and shuffle-table buffers); the next run
// reallocates what it needs. The reference-interface layer calls this when
// it pools a context, so no HBM is held between its calls (a
// sub-batch's sweep records alone may take tens of GB).
int nr_release_scratch(nr_ctx* ctx) {
  if (!ctx) return NR_ERR_INVALID;
  NR_HIP(ctx, hipSetDevice(ctx->device));
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  sync_obs(ctx);
  for (auto& b : ctx->sweep) {
    dfree(b.col);
    dfree(b.rank);
    dfree(b.count);
    dfree(b.col_off);
    dfree(b.sorted);
    dfree(b.meta);
    dfree(b.bndh);
    dfree(b.lrank);
    dfree(b.dabs);
    dfree(b.zs);
    dfree(b.rec);
    b.occ_cap = b.col_cap = 0;
    b.chunk_cap = 0;
  }
  dfree(ctx->d_out);
  ctx->out_cap = 0;
  dfree(ctx->d_scale);
  ctx->d_scale_cap = 0;
  dfree(ctx->d_out2);
  ctx->out2_cap = 0;
  dfree(ctx->d_pi);
  ctx->pi_cap = 0;
  dfree(ctx->d_scratch);
  ctx->scratch_cap = 0;
  dfree(ctx->d_net_scratch);
  ctx->net_scratch_cap = 0;
  dfree(ctx->obs_scratch);
  ctx->obs_scratch_cap = 0;
  dfree(ctx->obs_net_scratch);
  ctx->obs_net_cap = 0;
  dfree(ctx->d_obs);
  ctx->obs_cap = 0;
  return NR_OK;
}

int nr_scratch_bytes(const nr_ctx* ctx, int64_t* bytes) {
  if (!ctx || !bytes) return NR_ERR_INVALID;
  int64_t t = 0;
  for (const auto& b : ctx->sweep) {
    if (b.col) t += (int64_t)b.occ_cap * (4 * 4 + 2 * (int64_t)sizeof(uint4));
    if (b.bndh) t += (int64_t)b.occ_cap * 4 * b.chunk_cap;
    if (b.rec) t += (int64_t)b.occ_cap * 8 * nr::kSweepRec * b.chunk_cap;
    if (b.count) t += (int64_t)b.col_cap * 16;
    if (b.zs) t += (4 + 256) * 8;
  }
  if (ctx->d_out) t += (int64_t)ctx->out_cap * 8;
  if (ctx->d_out2) t += (int64_t)ctx->out2_cap * 8;
  if (ctx->d_pi) t += (int64_t)ctx->pi_cap * 4;
  if (ctx->d_scratch) t += (int64_t)ctx->scratch_cap * 8;
  if (ctx->d_net_scratch) t += (int64_t)ctx->net_scratch_cap * 8;
  if (ctx->obs_scratch) t += (int64_t)ctx->obs_scratch_cap * 8;
  if (ctx->obs_net_scratch) t += (int64_t)ctx->obs_net_cap * 8;
  if (ctx->d_obs) t += (int64_t)ctx->obs_cap * 8;
  *bytes = t;
  return NR_OK;
}

int nr_ctx_get_host_threads(const nr_ctx* ctx, int* n) {
  if (!ctx || !n) return NR_ERR_INVALID;
  *n = ctx->host_threads;
  return NR_OK;
}

int nr_debug_set(int what, int64_t value) {
  switch (what) {
    case NR_DEBUG_SWEEP_MAX_OCC:
      g_sweep_max_occ = value > 0 ? value : kSweepMaxOcc;
      return NR_OK;
    case NR_DEBUG_FAIL_SWEEP_ALLOC:
      g_fail_sweep_alloc = (int)std::max<int64_t>(0, value);
      return NR_OK;
    default:
      return NR_ERR_INVALID;
  }
}

int nr_dataset_symmetric(nr_ctx* ctx, int* symmetric) {
  if (!ctx || !symmetric) return NR_ERR_INVALID;
  if (!ctx->d_pairs) return fail(ctx, NR_ERR_INVALID, "no dataset");
  *symmetric = ctx->symmetric;
  return NR_OK;
}

int nr_gram_table(nr_ctx* ctx, int* on) {
  if (!ctx || !on) return NR_ERR_INVALID;
  *on = ctx->d_pairs && ctx->pairs_es == 2 ? 1 : 0;
  return NR_OK;
}

int nr_gram_table_ms(nr_ctx* ctx, double* ms) {
  if (!ctx || !ms) return NR_ERR_INVALID;
  *ms = ctx->d_pairs && ctx->pairs_es == 2 ? ctx->table_ms : 0.0;
  return NR_OK;
}

int nr_dataset_finite(nr_ctx* ctx, int* corr_finite, int* net_finite) {
  if (!ctx || !corr_finite || !net_finite) return NR_ERR_INVALID;
  if (!ctx->d_pairs) return fail(ctx, NR_ERR_INVALID, "no dataset");
  *corr_finite = ctx->corr_finite;
  *net_finite = ctx->net_finite;
  return NR_OK;
}

int nr_set_modules(nr_ctx* ctx, int32_t n_rows, int32_t n_present, const int32_t* row_of,
                   const int64_t* node_off, const int32_t* test_idx, const int32_t* null_pos,
                   const double* disc_corr, const double* disc_degree, const double* disc_contrib) {
  if (!ctx) return NR_ERR_INVALID;
  if (n_rows < 0 || n_present < 0 || n_present > n_rows)
    return fail(ctx, NR_ERR_INVALID, "bad n_rows / n_present");
  if (n_present > 0 && (!row_of || !node_off || !test_idx || !disc_corr || !disc_degree))
    return fail(ctx, NR_ERR_INVALID, "module arrays missing");
  NR_HIP(ctx, hipSetDevice(ctx->device));
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  sync_obs(ctx);
  ctx->modules_gen = -1;  // usable only once everything below has succeeded
  ++ctx->modules_serial;
  ctx->n_rows = n_rows;
  ctx->n_present = n_present;
  ctx->node_off_h.assign(node_off, node_off + (n_present > 0 ? n_present + 1 : 0));
  if (n_present == 0) ctx->node_off_h.assign(1, 0);
  ctx->cv_off_h.assign(n_present + 1, 0);
  int32_t kmax = 0;
  std::vector<double> shift(n_present, 0.0);
  for (int m = 0; m < n_present; ++m) {
    const int64_t k = node_off[m + 1] - node_off[m];
    if (k <= 0) return fail(ctx, NR_ERR_INVALID, "present module with no nodes");
    if (row_of[m] < 0 || row_of[m] >= n_rows) return fail(ctx, NR_ERR_INVALID, "row_of out of range");
    kmax = std::max<int32_t>(kmax, (int32_t)k);
    ctx->cv_off_h[m + 1] = ctx->cv_off_h[m] + k * (k - 1) / 2;
    for (int64_t v = 0; v < k * (k - 1) / 2; ++v) {
      const double x = disc_corr[ctx->cv_off_h[m] + v];
      if (std::isfinite(x)) {
        shift[m] = x;
        break;
      }
    }
  }
  ctx->k_max = kmax;
  ctx->n_node_total = ctx->node_off_h.back();
  ctx->n_cv_total = ctx->cv_off_h.back();
  ctx->disc_cv_finite = 1;
  for (int64_t v = 0; v < ctx->n_cv_total; ++v)
    if (!std::isfinite(disc_corr[v])) {
      ctx->disc_cv_finite = 0;
      break;
    }
  for (int64_t i = 0; i < ctx->n_node_total; ++i)
    if (test_idx[i] < 0 || test_idx[i] >= ctx->n_nodes)
      return fail(ctx, NR_ERR_INVALID, "test_idx outside the resident dataset (call nr_set_dataset first)");
  ctx->null_pos_max = -1;
  if (null_pos) {
    for (int64_t i = 0; i < ctx->n_node_total; ++i) {
      if (null_pos[i] < 0) return fail(ctx, NR_ERR_INVALID, "negative null_pos");
      ctx->null_pos_max = std::max<int64_t>(ctx->null_pos_max, null_pos[i]);
    }
  }
  std::vector<int32_t> order(n_present);
  for (int m = 0; m < n_present; ++m) order[m] = m;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    return (node_off[a + 1] - node_off[a]) > (node_off[b + 1] - node_off[b]);
  });
  int rc;
  if ((rc = upload(ctx, ctx->d_row_of, row_of, n_present))) return rc;
  if ((rc = upload(ctx, ctx->d_node_off, ctx->node_off_h.data(), ctx->node_off_h.size()))) return rc;
  if ((rc = upload(ctx, ctx->d_cv_off, ctx->cv_off_h.data(), ctx->cv_off_h.size()))) return rc;
  if ((rc = upload(ctx, ctx->d_test_idx, test_idx, (size_t)ctx->n_node_total))) return rc;
  if ((rc = upload(ctx, ctx->d_null_pos, null_pos, null_pos ? (size_t)ctx->n_node_total : 0))) return rc;
  if ((rc = upload(ctx, ctx->d_disc_cv, disc_corr, (size_t)ctx->n_cv_total))) return rc;
  if ((rc = upload(ctx, ctx->d_disc_wd, disc_degree, (size_t)ctx->n_node_total))) return rc;
  if ((rc = upload(ctx, ctx->d_disc_nc, disc_contrib, disc_contrib ? (size_t)ctx->n_node_total : 0))) return rc;
  if ((rc = upload(ctx, ctx->d_cv_shift, shift.data(), shift.size()))) return rc;
  if ((rc = upload(ctx, ctx->d_mod_order, order.data(), order.size()))) return rc;
  ctx->order_k_h.resize(n_present);
  for (int i = 0; i < n_present; ++i) ctx->order_k_h[i] = (int32_t)(node_off[order[i] + 1] - node_off[order[i]]);
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (ctx->d_data && !ctx->d_disc_nc && n_present > 0)
    return fail(ctx, NR_ERR_INVALID, "dataset has data but disc_contrib is NULL");
  ctx->modules_gen = ctx->data_gen;
  return NR_OK;
}

int nr_set_null_pool(nr_ctx* ctx, const int32_t* null_idx, int64_t n_null) {
  if (!ctx) return NR_ERR_INVALID;
  if (!null_idx || n_null <= 0 || n_null > (int64_t)UINT32_MAX / 4)
    return fail(ctx, NR_ERR_INVALID, "bad null pool");
  for (int64_t i = 0; i < n_null; ++i)
    if (null_idx[i] < 0 || null_idx[i] >= ctx->n_nodes)
      return fail(ctx, NR_ERR_INVALID, "null_idx outside the resident dataset");
  NR_HIP(ctx, hipSetDevice(ctx->device));
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  sync_obs(ctx);
  ctx->n_null = n_null;
  int rc = upload(ctx, ctx->d_null_idx, null_idx, (size_t)n_null);
  if (rc) return rc;
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->null_gen = ctx->data_gen;
  return NR_OK;
}

int nr_observed(nr_ctx* ctx, double* observed) {
  if (!ctx || !observed) return NR_ERR_INVALID;
  int rc = check_ready(ctx, false);
  if (rc) return rc;
  const int64_t slice = (int64_t)ctx->n_rows * n_stat_of(ctx);
  rc = ensure(ctx, ctx->d_out, ctx->out_cap, (size_t)slice);
  if (rc) return rc;
  if ((rc = maybe_build_table(ctx))) return rc;
  const nr::IndexSource src = make_source(ctx, nr::NR_IDX_DIRECT, 0, 0, nullptr, ctx->d_test_idx);
  rc = launch_batch(ctx, src, 1, ctx->d_out, main_lane(ctx));
  if (rc) return rc;
  NR_HIP(ctx, hipMemcpyAsync(observed, ctx->d_out, (size_t)slice * sizeof(double),
                             hipMemcpyDeviceToHost, ctx->stream));
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return NR_OK;
}

int nr_observed_async(nr_ctx* ctx) {
  if (!ctx) return NR_ERR_INVALID;
  int rc = check_ready(ctx, false);
  if (rc) return rc;
  NR_HIP(ctx, hipSetDevice(ctx->device));
  if (!ctx->obs_stream) {
    NR_HIP(ctx, hipStreamCreateWithFlags(&ctx->obs_stream, hipStreamNonBlocking));
    NR_HIP(ctx, hipMalloc((void**)&ctx->obs_counters, 16 * sizeof(int)));
    NR_HIP(ctx, hipMemset(ctx->obs_counters, 0, 16 * sizeof(int)));
  }
  sync_obs(ctx);  // a previous observed launch is done before its buffers are reused
  if ((rc = maybe_build_table(ctx))) return rc;
  const int64_t slice = (int64_t)ctx->n_rows * n_stat_of(ctx);
  rc = ensure(ctx, ctx->d_obs, ctx->obs_cap, (size_t)std::max<int64_t>(slice, 1));
  if (rc) return rc;
  const nr::IndexSource src = make_source(ctx, nr::NR_IDX_DIRECT, 0, 0, nullptr, ctx->d_test_idx);
  rc = launch_batch(ctx, src, 1, ctx->d_obs, obs_lane(ctx));
  if (rc) return rc;
  ctx->obs_pending = true;
  return NR_OK;
}

int nr_observed_wait(nr_ctx* ctx, double* observed) {
  if (!ctx || !observed) return NR_ERR_INVALID;
  if (!ctx->obs_pending)
    return fail(ctx, NR_ERR_INVALID, "no observed statistics pending (call nr_observed_async after the last "
                                     "change of dataset, modules or null pool)");
  ctx->obs_pending = false;
  const int64_t slice = (int64_t)ctx->n_rows * n_stat_of(ctx);
  NR_HIP(ctx, hipMemcpyAsync(observed, ctx->d_obs, (size_t)slice * sizeof(double), hipMemcpyDeviceToHost,
                             ctx->obs_stream));
  NR_HIP(ctx, hipStreamSynchronize(ctx->obs_stream));
  return NR_OK;
}

int nr_run(nr_ctx* ctx, int64_t perm_begin, int64_t perm_end, uint64_t seed, const uint32_t* pi,
           double* nulls) {
  if (!ctx || !nulls) return NR_ERR_INVALID;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return run_impl(ctx, perm_begin, perm_end, seed, pi, false, nulls, false);
}

int nr_run_device(nr_ctx* ctx, int64_t perm_begin, int64_t perm_end, uint64_t seed,
                  const uint32_t* pi_device, double* nulls_device) {
  if (!ctx || !nulls_device) return NR_ERR_INVALID;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return run_impl(ctx, perm_begin, perm_end, seed, pi_device, true, nulls_device, true);
}

int nr_export_indices(nr_ctx* ctx, int64_t perm_begin, int64_t perm_end, uint64_t seed,
                      int32_t* indices) {
  if (!ctx || !indices || perm_end < perm_begin) return NR_ERR_INVALID;
  int rc = check_ready(ctx, true);
  if (rc) return rc;
  const int64_t np = perm_end - perm_begin;
  if (np == 0) return NR_OK;
  int32_t* d = nullptr;
  NR_HIP(ctx, hipSetDevice(ctx->device));
  NR_HIP(ctx, hipMalloc((void**)&d, (size_t)(np * ctx->n_node_total) * sizeof(int32_t)));
  const nr::IndexSource src = make_source(ctx, nr::NR_IDX_PRP, seed, perm_begin, nullptr, nullptr);
  hipError_t e = nr::launch_export(src, ctx->n_node_total, d, np, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(indices, d, (size_t)(np * ctx->n_node_total) * sizeof(int32_t),
                       hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(ctx, e, "export indices");
  return NR_OK;
}

int nr_module_vectors(nr_ctx* ctx, int32_t n_mod, const int64_t* node_off, const int32_t* idx,
                      double* corr_vec, double* degree, double* avg_weight, double* contribution,
                      double* summary, double* coherence) {
  if (!ctx || n_mod < 0 || (n_mod > 0 && (!node_off || !idx))) return NR_ERR_INVALID;
  if (!ctx->d_pairs) return fail(ctx, NR_ERR_INVALID, "no dataset");
  if ((contribution || summary || coherence) && !ctx->d_data)
    return fail(ctx, NR_ERR_INVALID, "contribution/summary need a dataset with data");
  if (n_mod == 0) return NR_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  NR_HIP(ctx, hipSetDevice(ctx->device));
  std::vector<int64_t> cv(n_mod + 1, 0);
  int32_t kmax = 0;
  for (int m = 0; m < n_mod; ++m) {
    const int64_t k = node_off[m + 1] - node_off[m];
    if (k <= 0) return fail(ctx, NR_ERR_INVALID, "module with no nodes");
    kmax = std::max<int32_t>(kmax, (int32_t)k);
    cv[m + 1] = cv[m] + k * (k - 1) / 2;
  }
  const int64_t nodes = node_off[n_mod];
  for (int64_t i = 0; i < nodes; ++i)
    if (idx[i] < 0 || idx[i] >= ctx->n_nodes) return fail(ctx, NR_ERR_INVALID, "idx outside the dataset");
  std::vector<int32_t> order(n_mod);
  for (int m = 0; m < n_mod; ++m) order[m] = m;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    return (node_off[a + 1] - node_off[a]) > (node_off[b + 1] - node_off[b]);
  });
  int64_t *d_off = nullptr, *d_cv = nullptr;
  int32_t *d_idx = nullptr, *d_order = nullptr;
  double *d_cvo = nullptr, *d_wd = nullptr, *d_nc = nullptr, *d_sp = nullptr, *d_coh = nullptr,
         *d_aw = nullptr;
  int rc = NR_OK;
  auto cleanup = [&]() {
    dfree(d_off); dfree(d_cv); dfree(d_idx); dfree(d_order);
    dfree(d_cvo); dfree(d_wd); dfree(d_nc); dfree(d_sp); dfree(d_coh); dfree(d_aw);
  };
  const int64_t S = ctx->n_samples;
  do {
    if ((rc = upload(ctx, d_off, node_off, (size_t)n_mod + 1))) break;
    if ((rc = upload(ctx, d_cv, cv.data(), cv.size()))) break;
    if ((rc = upload(ctx, d_idx, idx, (size_t)nodes))) break;
    if ((rc = upload(ctx, d_order, order.data(), order.size()))) break;
    hipError_t e = hipMalloc((void**)&d_cvo, (size_t)std::max<int64_t>(cv.back(), 1) * sizeof(double));
    if (e == hipSuccess) e = hipMalloc((void**)&d_wd, (size_t)nodes * sizeof(double));
    if (e == hipSuccess) e = hipMalloc((void**)&d_aw, (size_t)n_mod * sizeof(double));
    if (e == hipSuccess && ctx->d_data) e = hipMalloc((void**)&d_nc, (size_t)nodes * sizeof(double));
    if (e == hipSuccess && ctx->d_data) e = hipMalloc((void**)&d_sp, (size_t)(n_mod * S) * sizeof(double));
    if (e == hipSuccess && ctx->d_data) e = hipMalloc((void**)&d_coh, (size_t)n_mod * sizeof(double));
    if (e != hipSuccess) { rc = hip_fail(ctx, e, "hipMalloc module vectors"); break; }
    nr::IndexSource src = make_source(ctx, nr::NR_IDX_DIRECT, 0, 0, nullptr, d_idx);
    nr::NetParams np{};
    np.pairs = ctx->d_pairs;
    np.es = ctx->pairs_es;
    np.colsum = ctx->d_colsum;
    np.n_nodes = ctx->n_nodes;
    np.symmetric = ctx->symmetric;
    np.src = src;
    np.node_off = d_off;
    np.cv_off = d_cv;
    np.mod_order = d_order;
    np.n_perm = 1;
    np.k_max = kmax;
    np.cv_out = d_cvo;
    np.wd_out = d_wd;
    np.avgw_out = d_aw;
    std::vector<int32_t> k_sorted(n_mod);
    for (int i = 0; i < n_mod; ++i) k_sorted[i] = (int32_t)(node_off[order[i] + 1] - node_off[order[i]]);
    if ((rc = launch_nets(ctx, np, d_order, k_sorted, 1, main_lane(ctx)))) break;
    e = hipSuccess;
    if (ctx->d_data && (contribution || summary || coherence)) {
      nr::ProfileParams pp{};
      pp.data = ctx->d_data;
      pp.n_samples = S;
      pp.ones_off = ctx->n_nodes * S;
      pp.src = src;
      pp.node_off = d_off;
      pp.n_perm = 1;
      pp.sp_out = d_sp;
      pp.nc_out = d_nc;
      pp.coh_out = d_coh;
      pp.queue = ctx->d_counters;
      pp.diag = ctx->d_counters + 1;
      if ((rc = launch_profiles(ctx, pp, d_order, k_sorted, 1, main_lane(ctx)))) break;
    }
    auto d2h = [&](double* h, const double* d, int64_t n) {
      if (e == hipSuccess && h && n > 0)
        e = hipMemcpyAsync(h, d, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
    };
    d2h(corr_vec, d_cvo, cv.back());
    d2h(degree, d_wd, nodes);
    d2h(avg_weight, d_aw, n_mod);
    d2h(contribution, d_nc, nodes);
    d2h(summary, d_sp, n_mod * S);
    d2h(coherence, d_coh, n_mod);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) rc = hip_fail(ctx, e, "module vectors");
  } while (0);
  cleanup();
  return rc;
}

// Scale (src/scale.cpp:38-45) of a host matrix: column chunks of ~16 MiB
// through the context's pinned staging buffers (kept between calls),
// double-buffered, and its device chunks (scratch: nr_release_scratch frees
// them, as a pooled context's return does). After chunk i is queued (copy in,
// scale_kernel, copy out), one fork-join of the host threads copies chunk
// i-1's result out of pinned memory and chunk i+1 into it, while the copy
// engine and the kernel work on chunk i. The caller's pageable arrays are
// never handed to the DMA engine directly (that ran at ~5 GB/s: 31 ms for
// 20k x 500, profiles/r05/props/; round 6's first pinned version, one
// fork-join per copy and a device allocation per call: 10.3 ms,
// profiles/r06/ab5/props/).
int nr_scale(nr_ctx* ctx, const double* data, int64_t n_samples, int64_t n_nodes, double* scaled) {
  if (!ctx || !data || !scaled || n_samples <= 0 || n_nodes <= 0) return NR_ERR_INVALID;
  NR_HIP(ctx, hipSetDevice(ctx->device));
  const int64_t S = n_samples;
  const int64_t cols = std::max<int64_t>(1, std::min<int64_t>(n_nodes, ((int64_t)1 << 21) / S));
  const int64_t chunk = cols * S;  // doubles per chunk
  if (int rc = ensure_stage(ctx, ctx->h_scale, ctx->scale_cap, (size_t)(4 * chunk))) return rc;
  if (int rc = ensure(ctx, ctx->d_scale, ctx->d_scale_cap, (size_t)(4 * chunk))) return rc;
  double* hin[2] = {ctx->h_scale, ctx->h_scale + chunk};
  double* hout[2] = {ctx->h_scale + 2 * chunk, ctx->h_scale + 3 * chunk};
  double* din[2] = {ctx->d_scale, ctx->d_scale + chunk};
  double* dout[2] = {ctx->d_scale + 2 * chunk, ctx->d_scale + 3 * chunk};
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipError_t e = hipSuccess;
  for (int b = 0; b < 2 && e == hipSuccess; ++b) e = hipEventCreateWithFlags(&ev[b], hipEventDisableTiming);
  const int threads = ctx->host_threads;
  const int64_t n_chunks = (n_nodes + cols - 1) / cols;
  auto len = [&](int64_t i) { return std::min(cols, n_nodes - i * cols) * S; };
  if (e == hipSuccess) parallel_copy(hin[0], data, len(0), threads, (int64_t)1 << 17);
  for (int64_t i = 0; i < n_chunks && e == hipSuccess; ++i) {
    const int b = (int)(i & 1);
    // hin[b] holds chunk i; hout[b] was drained in iteration i-1 (chunk i-2)
    e = h2d_async(din[b], hin[b], (size_t)len(i) * sizeof(double), ctx->stream);
    if (e == hipSuccess) e = nr::launch_scale(din[b], dout[b], S, len(i) / S, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(hout[b], dout[b], (size_t)len(i) * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipEventRecord(ev[b], ctx->stream);
    // chunk i-1 done (its pinned input free for chunk i+1, its result ready)
    if (e == hipSuccess && i >= 1) e = hipEventSynchronize(ev[b ^ 1]);
    if (e != hipSuccess) break;
    const bool out = i >= 1, in = i + 1 < n_chunks;
    parallel_copy2(out ? scaled + (i - 1) * cols * S : scaled, hout[b ^ 1], out ? len(i - 1) : 0, hin[b ^ 1],
                   in ? data + (i + 1) * cols * S : data, in ? len(i + 1) : 0, threads, (int64_t)1 << 17);
  }
  if (e == hipSuccess) e = hipEventSynchronize(ev[(n_chunks - 1) & 1]);
  if (e == hipSuccess)
    parallel_copy(scaled + (n_chunks - 1) * cols * S, hout[(n_chunks - 1) & 1], len(n_chunks - 1), threads,
                  (int64_t)1 << 17);
  (void)hipStreamSynchronize(ctx->stream);
  for (hipEvent_t x : ev)
    if (x) (void)hipEventDestroy(x);
  if (e != hipSuccess) return hip_fail(ctx, e, "scale");
  return NR_OK;
}

int nr_check_finite(nr_ctx* ctx, const double* mat, int64_t n_elem, int* all_finite) {
  if (!ctx || !mat || !all_finite || n_elem < 0) return NR_ERR_INVALID;
  NR_HIP(ctx, hipSetDevice(ctx->device));
  *all_finite = 1;
  if (n_elem == 0) return NR_OK;
  const int64_t chunk = std::min<int64_t>(n_elem, (int64_t)1 << 26);
  double* d = nullptr;
  NR_HIP(ctx, hipMalloc((void**)&d, (size_t)chunk * sizeof(double)));
  hipError_t e = hipMemsetAsync(ctx->d_counters + 5, 0, sizeof(int), ctx->stream);
  for (int64_t o = 0; o < n_elem && e == hipSuccess; o += chunk) {
    const int64_t len = std::min(chunk, n_elem - o);
    e = h2d_async(d, mat + o, (size_t)len * sizeof(double), ctx->stream);
    if (e == hipSuccess) e = nr::launch_finite(d, len, ctx->d_counters + 5, ctx->stream);
  }
  int bad = 0;
  if (e == hipSuccess)
    e = hipMemcpyAsync(&bad, ctx->d_counters + 5, sizeof(int), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(ctx, e, "check finite");
  *all_finite = bad ? 0 : 1;
  return NR_OK;
}

int nr_progress(nr_ctx* ctx, int64_t* done, int64_t* total) {
  if (!ctx) return NR_ERR_INVALID;
  if (done) *done = ctx->done.load();
  if (total) *total = ctx->total.load();
  return NR_OK;
}

int nr_cancel(nr_ctx* ctx) {
  if (!ctx) return NR_ERR_INVALID;
  ctx->cancel = true;
  return NR_OK;
}

int nr_set_batch(nr_ctx* ctx, int64_t perms_per_launch) {
  if (!ctx || perms_per_launch < 0) return NR_ERR_INVALID;
  ctx->batch = perms_per_launch;
  return NR_OK;
}

int nr_set_timing(nr_ctx* ctx, int enable) {
  if (!ctx) return NR_ERR_INVALID;
  ctx->timing = enable != 0;
  return NR_OK;
}

int nr_get_timing(nr_ctx* ctx, int kernel, double* total_ms, int64_t* launches, int64_t* items) {
  if (!ctx || kernel < 0 || kernel > 1) return NR_ERR_INVALID;
  if (total_ms) *total_ms = ctx->timers[kernel].ms;
  if (launches) *launches = ctx->timers[kernel].launches;
  if (items) *items = ctx->timers[kernel].items;
  return NR_OK;
}

int nr_reset_timing(nr_ctx* ctx) {
  if (!ctx) return NR_ERR_INVALID;
  ctx->timers[0] = DeviceTimer();
  ctx->timers[1] = DeviceTimer();
  NR_HIP(ctx, hipSetDevice(ctx->device));
  NR_HIP(ctx, hipMemsetAsync(ctx->d_counters + 1, 0, 4 * sizeof(int), ctx->stream));
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return NR_OK;
}

int nr_set_stamps(nr_ctx* ctx, int enable) {
  if (!ctx) return NR_ERR_INVALID;
  NR_HIP(ctx, hipSetDevice(ctx->device));
  if (enable && !ctx->d_stamps) {
    NR_HIP(ctx, hipMalloc((void**)&ctx->d_stamps, nr::NR_N_STAMPS * sizeof(unsigned long long)));
  }
  if (enable) NR_HIP(ctx, hipMemset(ctx->d_stamps, 0, nr::NR_N_STAMPS * sizeof(unsigned long long)));
  if (!enable) dfree(ctx->d_stamps);
  return NR_OK;
}

int nr_get_stamps(nr_ctx* ctx, uint64_t* cycles) {
  if (!ctx || !cycles) return NR_ERR_INVALID;
  if (!ctx->d_stamps) return fail(ctx, NR_ERR_INVALID, "stamps not enabled");
  NR_HIP(ctx, hipSetDevice(ctx->device));
  NR_HIP(ctx, hipMemcpy(cycles, ctx->d_stamps, nr::NR_N_STAMPS * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return NR_OK;
}

int nr_get_diagnostics(nr_ctx* ctx, int64_t* eig_items, int64_t* eig_steps, int64_t* eig_cap_hits,
                       int64_t* eig_reorths) {
  if (!ctx) return NR_ERR_INVALID;
  int h[4] = {0, 0, 0, 0};
  NR_HIP(ctx, hipSetDevice(ctx->device));
  NR_HIP(ctx, hipMemcpyAsync(h, ctx->d_counters + 1, 4 * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (eig_cap_hits) *eig_cap_hits = h[0];
  if (eig_items) *eig_items = h[1];
  if (eig_steps) *eig_steps = h[2];
  if (eig_reorths) *eig_reorths = h[3];
  return NR_OK;
}

int nr_synchronize(nr_ctx* ctx) {
  if (!ctx) return NR_ERR_INVALID;
  NR_HIP(ctx, hipSetDevice(ctx->device));
  NR_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return NR_OK;
}

}  // extern "C"

extern "C" {
// Host evaluation of the keyed null-pool permutation (prp.h) for tests and
// for callers that want to export the exact shuffles a run uses.
int nr_prp_table(uint64_t seed, int64_t perm_begin, int64_t perm_end, int64_t n_null,
                 uint32_t* out) {
  if (!out || perm_end < perm_begin || n_null <= 0 || n_null > (int64_t)UINT32_MAX / 4)
    return NR_ERR_INVALID;
  for (int64_t p = perm_begin; p < perm_end; ++p) {
    const nr_prp_key key = nr_prp_make_key(seed, (uint64_t)p, (uint32_t)n_null);
    for (int64_t q = 0; q < n_null; ++q)
      out[(p - perm_begin) * n_null + q] = nr_prp_permute(key, (uint32_t)q);
  }
  return NR_OK;
}
}  // extern "C"
