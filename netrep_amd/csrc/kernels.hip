// Device kernels of the MI355X NetRep permutation engine (gfx950 / CDNA4).
//
// One work item = (permutation p, module m). Two kernels cover the seven
// statistics of calculateNulls (src/permutations.cpp:71-101):
//   module_net_kernel      avg.weight, cor.cor, cor.degree, avg.cor
//                          (CorrVector + WeightedDegree gathers; HBM-bound)
//   module_profile_kernel  coherence, cor.contrib, avg.contrib
//                          (SummaryProfile + NodeContribution: fp64-MFMA Gram
//                           of the S x k data block + Lanczos top eigenpair)
// The network-only path (src/permutationsNoData.cpp:66-85) is the first kernel
// alone. Both also run in "vector" mode to produce the per-module vectors of
// IntermediateProperties (src/discProps.cpp:100-121) and NetProps
// (src/properties.cpp:155-184).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "prp.h"
#include "kernels.h"

namespace nr {

#define NR_BS 256
#define NR_WAVES (NR_BS / 64)

__device__ __forceinline__ double nr_nan() { return __longlong_as_double(0x7FF8000000000000ll); }

// R's NA_real_ (src/permutations.cpp:383-384 fills non-finite with NA_REAL).
__device__ __forceinline__ double na_fill(double x) {
  return isfinite(x) ? x : __longlong_as_double(0x7FF00000000007A2ll);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sums of N values; result broadcast to every thread. `red` must
// hold N * NR_WAVES doubles of LDS. Contains two barriers.
template <int N>
__device__ __forceinline__ void block_sums(double (&v)[N], double* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = wave_sum(v[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) red[i * NR_WAVES + wave] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NR_WAVES; ++w) s += red[i * NR_WAVES + w];
    v[i] = s;
  }
  __syncthreads();
}

// Pearson correlation from (shifted) one-pass sums over complete cases.
__device__ __forceinline__ double pearson_sums(double n, double sx, double sy,
                                               double sxx, double syy, double sxy) {
  if (n < 1.0) return nr_nan();
  const double cov = sxy - sx * sy / n;
  const double vx = sxx - sx * sx / n;
  const double vy = syy - sy * sy / n;
  return cov / (sqrt(vx) * sqrt(vy));
}

// Test column of module node c of item (p, m): GetRandomIdx
// (src/utils.cpp:193-199) under a PRP, an explicit table, or a direct set.
__device__ __forceinline__ uint32_t node_index(const IndexSource& src, const nr_prp_key& key,
                                               int64_t p_local, int64_t node) {
  if (src.mode == NR_IDX_DIRECT) return (uint32_t)src.direct_idx[node];
  const uint32_t q = (uint32_t)src.null_pos[node];
  const uint32_t s = (src.mode == NR_IDX_PRP)
                         ? nr_prp_permute(key, q)
                         : src.pi[p_local * (int64_t)src.n_null + q];
  return (uint32_t)src.null_idx[s];
}

// Decode flat CorrVector position v -> (jj, ii), ii > jj, column-major lower
// triangle (src/netStats.cpp:196-201).
__device__ __forceinline__ void decode_pair(int64_t v, int64_t k, int64_t& jj, int64_t& ii) {
  const double b = (double)(2 * k - 1);
  int64_t j = (int64_t)floor((b - sqrt(b * b - 8.0 * (double)v)) * 0.5);
  if (j < 0) j = 0;
  // off(j) = j*(2k-j-1)/2 pairs precede column j
  while (j > 0 && j * (2 * k - j - 1) / 2 > v) --j;
  while ((j + 1) * (2 * k - j - 2) / 2 <= v) ++j;
  jj = j;
  ii = v - j * (2 * k - j - 1) / 2 + j + 1;
}

// ---------------------------------------------------------------------------
// Kernel 1: module network statistics. One workgroup per item.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(NR_BS)
module_net_kernel(NetParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* red = reinterpret_cast<double*>(smem);                    // 8 * NR_WAVES
  double* wd = red + 8 * NR_WAVES;                                  // [k]
  uint32_t* idx = reinterpret_cast<uint32_t*>(wd + P.k_max);        // [k]

  const int64_t item = blockIdx.x;
  const int64_t mslot = item / P.n_perm;
  const int64_t p_local = item - mslot * P.n_perm;
  const int m = P.mod_order[mslot];
  const int64_t off = P.node_off[m];
  const int64_t k = P.node_off[m + 1] - off;
  const int tid = threadIdx.x;

  nr_prp_key key;
  if (P.src.mode == NR_IDX_PRP) key = nr_prp_make_key(P.src.seed, (uint64_t)(P.src.perm_base + p_local), P.src.n_null);

  for (int64_t c = tid; c < k; c += NR_BS) {
    idx[c] = node_index(P.src, key, p_local, off + c);
    wd[c] = 0.0;
  }
  __syncthreads();

  const int64_t npairs = k * (k - 1) / 2;
  const int64_t cvo = P.cv_off[m];
  const double2* __restrict__ pairs = P.pairs;
  const int64_t n = P.n_nodes;
  // Shifts keep the one-pass sums well conditioned and make a constant
  // vector give exactly zero variance, as the reference's two-pass stddev does.
  const double xs = P.cv_shift ? P.cv_shift[m] : 0.0;
  const double ys = npairs > 0 ? pairs[(int64_t)idx[1] + (int64_t)idx[0] * n].x : 0.0;

  double acc[7] = {0, 0, 0, 0, 0, 0, 0};  // n, sx, sy, sxx, syy, sxy, s(sign(x) y)
  constexpr int U = 4;
  for (int64_t v0 = tid; v0 < npairs; v0 += (int64_t)NR_BS * U) {
    double2 e[U];
    double e2[U];
    double x[U];
    int64_t jjs[U], iis[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = v0 + (int64_t)u * NR_BS;
      jjs[u] = -1;
      if (v < npairs) {
        int64_t jj, ii;
        decode_pair(v, k, jj, ii);
        jjs[u] = jj;
        iis[u] = ii;
        const int64_t r = idx[ii], c = idx[jj];
        e[u] = pairs[r + c * n];                      // corr(idx[ii], idx[jj]), net(idx[ii], idx[jj])
        e2[u] = P.symmetric ? e[u].y : pairs[c + r * n].y;  // net(idx[jj], idx[ii])
        x[u] = P.disc_cv ? P.disc_cv[cvo + v] : nr_nan();
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (jjs[u] < 0) continue;
      const double y = e[u].x;
      if (P.cv_out) P.cv_out[cvo + v0 + (int64_t)u * NR_BS] = y;
      atomicAdd(&wd[jjs[u]], fabs(e[u].y));     // column idx[jj] gains row idx[ii]
      atomicAdd(&wd[iis[u]], fabs(e2[u]));      // column idx[ii] gains row idx[jj]
      const double xv = x[u];
      if (isfinite(xv) && isfinite(y)) {        // CompleteCases src/netStats.cpp:43-61
        const double dx = xv - xs, dy = y - ys;
        acc[0] += 1.0;
        acc[1] += dx;
        acc[2] += dy;
        acc[3] += dx * dx;
        acc[4] += dy * dy;
        acc[5] += dx * dy;
        acc[6] += (xv > 0.0 ? y : (xv < 0.0 ? -y : 0.0));
      }
    }
  }
  block_sums<7>(acc, red);

  // Weighted degree statistics: two-pass over the k values held in LDS.
  const int64_t woff = off;
  double a1[4] = {0, 0, 0, 0};  // sum(all wd), n, sx, sy
  for (int64_t c = tid; c < k; c += NR_BS) {
    const double y = wd[c];
    const double xv = P.disc_wd ? P.disc_wd[woff + c] : nr_nan();
    a1[0] += y;
    if (isfinite(xv) && isfinite(y)) {
      a1[1] += 1.0;
      a1[2] += xv;
      a1[3] += y;
    }
  }
  block_sums<4>(a1, red);
  const double mx = a1[2] / a1[1], my = a1[3] / a1[1];
  double a2[3] = {0, 0, 0};
  for (int64_t c = tid; c < k; c += NR_BS) {
    const double y = wd[c];
    const double xv = P.disc_wd ? P.disc_wd[woff + c] : nr_nan();
    if (isfinite(xv) && isfinite(y)) {
      const double dx = xv - mx, dy = y - my;
      a2[0] += dx * dx;
      a2[1] += dy * dy;
      a2[2] += dx * dy;
    }
    if (P.wd_out) P.wd_out[woff + c] = y;
  }
  block_sums<3>(a2, red);

  // AverageEdgeWeight src/netStats.cpp:154-162: unsigned int pair count.
  const uint32_t ku = (uint32_t)k;
  const double avg_weight = a1[0] / (double)(uint32_t)(ku * ku - ku);
  if (tid == 0 && P.avgw_out) P.avgw_out[m] = avg_weight;
  if (tid == 0 && P.out) {
    const double cor_degree = a1[1] >= 1.0 ? a2[2] / (sqrt(a2[0]) * sqrt(a2[1])) : nr_nan();
    const double cor_cor = pearson_sums(acc[0], acc[1], acc[2], acc[3], acc[4], acc[5]);
    const double avg_cor = acc[0] >= 1.0 ? acc[6] / acc[0] : nr_nan();
    double* o = P.out + (int64_t)P.row_of[m] + (int64_t)P.n_rows * (int64_t)P.n_stat * p_local;
    o[(int64_t)P.n_rows * P.slot_avg_weight] = na_fill(avg_weight);
    o[(int64_t)P.n_rows * P.slot_cor_cor] = na_fill(cor_cor);
    o[(int64_t)P.n_rows * P.slot_cor_degree] = na_fill(cor_degree);
    o[(int64_t)P.n_rows * P.slot_avg_cor] = na_fill(avg_cor);
  }
}

// ---------------------------------------------------------------------------
// Kernel 2: summary-profile statistics. Persistent workgroups pull items from
// a queue; each owns a scratch slot holding G = X^T X and the Lanczos basis.
// ---------------------------------------------------------------------------
typedef double nr_f64x4 __attribute__((ext_vector_type(4)));

// Largest eigenvalue of the symmetric tridiagonal (alpha[0..n), beta[0..n-1))
// by 64-way multisection on Sturm counts; executed by one full wave.
__device__ double tri_top_eigenvalue(const double* alpha, const double* beta, int n, int lane) {
  double lo = alpha[0], hi = alpha[0];
  for (int i = 0; i < n; ++i) {
    const double r = (i > 0 ? fabs(beta[i - 1]) : 0.0) + (i < n - 1 ? fabs(beta[i]) : 0.0);
    lo = fmin(lo, alpha[i] - r);
    hi = fmax(hi, alpha[i] + r);
  }
  const double scale = fmax(fabs(lo), fabs(hi)) + 1e-300;
  lo -= 1e-14 * scale;
  hi += 1e-14 * scale;
  const double tiny = 1e-300;
  for (int it = 0; it < 12; ++it) {
    const double x = lo + (hi - lo) * (double)(lane + 1) / 65.0;
    int cnt = 0;  // eigenvalues < x
    double d = alpha[0] - x;
    if (fabs(d) < tiny) d = -tiny;
    cnt += d < 0.0;
    for (int i = 1; i < n; ++i) {
      d = alpha[i] - x - beta[i - 1] * beta[i - 1] / d;
      if (fabs(d) < tiny) d = -tiny;
      cnt += d < 0.0;
    }
    // largest x with cnt <= n-1 becomes lo; smallest x with cnt == n becomes hi
    const unsigned long long below = __ballot(cnt <= n - 1);
    // lanes are ordered by x: lanes [0, t) have cnt <= n-1, lanes [t, 64) have cnt == n
    const int t = __popcll(below);
    const double xlo = lo + (hi - lo) * (double)t / 65.0;
    const double xhi = lo + (hi - lo) * (double)(t + 1) / 65.0;
    lo = xlo;
    hi = xhi;
    if (hi - lo <= 2e-16 * scale) break;
  }
  return 0.5 * (lo + hi);
}

// Eigenvector of the tridiagonal for eigenvalue theta by two steps of inverse
// iteration; LU with partial pivoting as LAPACK dgttrf/dgtts2. Single lane.
// y[0..n) comes back normalised; work holds 5n doubles.
__device__ void tri_eigenvector(const double* alpha, const double* beta, int n, double theta,
                                double* y, double* work) {
  double* dl = work;
  double* d = work + n;
  double* du = work + 2 * n;
  double* du2 = work + 3 * n;
  double* swp = work + 4 * n;
  double scale = fabs(theta);
  for (int i = 0; i < n; ++i) {
    d[i] = alpha[i] - theta;
    scale = fmax(scale, fabs(alpha[i]));
    if (i < n - 1) {
      du[i] = beta[i];
      dl[i] = beta[i];
      scale = fmax(scale, fabs(beta[i]));
    }
    du2[i] = 0.0;
    swp[i] = 0.0;
  }
  const double floor_piv = 1e-300 + 2.2e-16 * scale;
  for (int i = 0; i < n - 1; ++i) {
    if (fabs(d[i]) >= fabs(dl[i])) {
      if (fabs(d[i]) < floor_piv) d[i] = d[i] < 0.0 ? -floor_piv : floor_piv;
      const double f = dl[i] / d[i];
      dl[i] = f;
      d[i + 1] -= f * du[i];
    } else {
      const double f = d[i] / dl[i];
      d[i] = dl[i];
      dl[i] = f;
      const double t = du[i];
      du[i] = d[i + 1];
      d[i + 1] = t - f * d[i + 1];
      if (i < n - 2) {
        du2[i] = du[i + 1];
        du[i + 1] = -f * du[i + 1];
      }
      swp[i] = 1.0;
    }
  }
  if (fabs(d[n - 1]) < floor_piv) d[n - 1] = d[n - 1] < 0.0 ? -floor_piv : floor_piv;
  for (int i = 0; i < n; ++i) y[i] = 1.0;
  for (int iter = 0; iter < 2; ++iter) {
    for (int i = 0; i < n - 1; ++i) {
      if (swp[i] == 0.0) {
        y[i + 1] -= dl[i] * y[i];
      } else {
        const double t = y[i];
        y[i] = y[i + 1];
        y[i + 1] = t - dl[i] * y[i];
      }
    }
    y[n - 1] /= d[n - 1];
    if (n > 1) y[n - 2] = (y[n - 2] - du[n - 2] * y[n - 1]) / d[n - 2];
    for (int i = n - 3; i >= 0; --i) y[i] = (y[i] - du[i] * y[i + 1] - du2[i] * y[i + 2]) / d[i];
    double mx = 0.0;
    for (int i = 0; i < n; ++i) mx = fmax(mx, fabs(y[i]));
    double nrm = 0.0;
    for (int i = 0; i < n; ++i) {
      y[i] /= mx;
      nrm += y[i] * y[i];
    }
    const double inv = 1.0 / sqrt(nrm);
    for (int i = 0; i < n; ++i) y[i] *= inv;
  }
}

__global__ void __launch_bounds__(NR_BS)
module_profile_kernel(ProfileParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int kmax = P.k_max, mmax = P.m_max, S = (int)P.n_samples;
  double* red = reinterpret_cast<double*>(smem);        // 8 * NR_WAVES
  double* q = red + 8 * NR_WAVES;                        // [kmax]
  double* w = q + kmax;                                  // [kmax]
  double* vv = w + kmax;                                 // [kmax] Ritz vector
  double* gv = vv + kmax;                                // [kmax] G v
  double* colm = gv + kmax;                              // [kmax] column means
  double* mo = colm + kmax;                              // [S] meanObs (row means)
  double* alpha = mo + S;                                // [mmax]
  double* beta = alpha + mmax;                           // [mmax]
  double* h = beta + mmax;                               // [mmax]
  double* ty = h + mmax;                                 // [mmax]
  double* twork = ty + mmax;                             // [5 * mmax]
  uint32_t* idx = reinterpret_cast<uint32_t*>(twork + 5 * mmax);  // [kmax]
  __shared__ int s_item;
  __shared__ int s_flag;
  __shared__ int s_done;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double* G = P.scratch + (int64_t)blockIdx.x * P.scratch_stride;
  const int kp = P.kp;
  double* Q = G + (int64_t)kp * kp;
  const double* __restrict__ X = P.data;

  for (;;) {
    if (tid == 0) s_item = atomicAdd(P.queue, 1);
    __syncthreads();
    const int item = s_item;
    __syncthreads();
    if (item >= P.n_items) break;

    const int64_t mslot = item / P.n_perm;
    const int64_t p_local = item - mslot * P.n_perm;
    const int m = P.mod_order[mslot];
    const int64_t off = P.node_off[m];
    const int k = (int)(P.node_off[m + 1] - off);

    nr_prp_key key;
    if (P.src.mode == NR_IDX_PRP) key = nr_prp_make_key(P.src.seed, (uint64_t)(P.src.perm_base + p_local), P.src.n_null);
    for (int c = tid; c < k; c += NR_BS) idx[c] = node_index(P.src, key, p_local, off + c);
    if (tid == 0) s_flag = 0;
    __syncthreads();

    // Column means + finiteness (svd_econ refuses non-finite input:
    // src/netStats.cpp:229-235 -> all-NaN summary).
    for (int c = tid; c < k; c += NR_BS) {
      const double* col = X + (int64_t)idx[c] * S;
      double s = 0.0;
      bool fin = true;
      for (int r = 0; r < S; ++r) {
        const double xv = col[r];
        fin &= isfinite(xv);
        s += xv;
      }
      colm[c] = s / (double)S;
      if (!fin) atomicOr(&s_flag, 1);
    }
    // Row means of the module block (meanObs, src/netStats.cpp:242).
    for (int r = tid; r < S; r += NR_BS) {
      double s = 0.0;
      for (int c = 0; c < k; ++c) s += X[(int64_t)idx[c] * S + r];
      mo[r] = s / (double)k;
    }
    __syncthreads();
    const bool bad = s_flag != 0;

    double stat_coh = nr_nan(), stat_cc = nr_nan(), stat_ac = nr_nan();
    if (!bad) {
      // ---- Gram G = X^T X with v_mfma_f64_16x16x4_f64 (lower+upper tiles) ----
      const int T = (k + 15) / 16;
      const int ntiles = T * (T + 1) / 2;
      for (int t = wave; t < ntiles; t += NR_WAVES) {
        // tile t -> (I, J), I <= J, row-major over the upper triangle
        int I = 0, rem = t;
        while (rem >= T - I) { rem -= T - I; ++I; }
        const int J = I + rem;
        const int ci = I * 16 + (lane & 15), cj = J * 16 + (lane & 15);
        const int kk = lane >> 4;
        const double* coli = ci < k ? X + (int64_t)idx[ci] * S : nullptr;
        const double* colj = cj < k ? X + (int64_t)idx[cj] * S : nullptr;
        nr_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int s0 = 0; s0 < S; s0 += 4) {
          const int s = s0 + kk;
          const double a = (coli && s < S) ? coli[s] : 0.0;
          const double b = (colj && s < S) ? colj[s] : 0.0;
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
        }
        // D[row = (lane>>4) + 4 r][col = lane & 15]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gi = I * 16 + (lane >> 4) + 4 * r;
          const int gj = J * 16 + (lane & 15);
          G[gi + (int64_t)gj * kp] = acc[r];
          G[gj + (int64_t)gi * kp] = acc[r];
        }
      }
      __syncthreads();

      // ---- Lanczos with full (two-pass classical Gram-Schmidt) reorthogonalisation ----
      const int mcap = k < mmax ? k : mmax;
      for (int c = tid; c < k; c += NR_BS) {
        const uint32_t hsh = nr_lowbias32((uint32_t)c * 0x9E3779B9u + 0x1234567u);
        q[c] = 1.0 + 0.01 * ((double)(hsh & 0xFFFF) / 65536.0 - 0.5);
      }
      __syncthreads();
      {
        double a[1] = {0.0};
        for (int c = tid; c < k; c += NR_BS) a[0] += q[c] * q[c];
        block_sums<1>(a, red);
        const double inv = 1.0 / sqrt(a[0]);
        for (int c = tid; c < k; c += NR_BS) q[c] *= inv;
      }
      if (tid == 0) s_done = 0;
      __syncthreads();
      int nsteps = 0;
      for (int j = 0; j < mcap; ++j) {
        // store q_j, w = G q_j
        for (int c = tid; c < k; c += NR_BS) Q[(int64_t)j * k + c] = q[c];
        for (int r = tid; r < k; r += NR_BS) {
          double s = 0.0;
          for (int c = 0; c < k; ++c) s += G[r + (int64_t)c * kp] * q[c];
          w[r] = s;
        }
        __syncthreads();
        double alpha_j = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
          // h_i = Q_i . w, i <= j  (one wave per dot)
          for (int i = wave; i <= j; i += NR_WAVES) {
            double s = 0.0;
            for (int c = lane; c < k; c += 64) s += Q[(int64_t)i * k + c] * w[c];
            s = wave_sum(s);
            if (lane == 0) h[i] = s;
          }
          __syncthreads();
          alpha_j += h[j];
          for (int c = tid; c < k; c += NR_BS) {
            double s = 0.0;
            for (int i = 0; i <= j; ++i) s += h[i] * Q[(int64_t)i * k + c];
            w[c] -= s;
          }
          __syncthreads();
        }
        double nb[1] = {0.0};
        for (int c = tid; c < k; c += NR_BS) nb[0] += w[c] * w[c];
        block_sums<1>(nb, red);
        const double beta_j = sqrt(nb[0]);
        if (tid == 0) {
          alpha[j] = alpha_j;
          beta[j] = beta_j;
        }
        nsteps = j + 1;
        __syncthreads();
        const bool last = (j + 1 == mcap);
        if (((j + 1) % 4 == 0) || last || beta_j <= 1e-300) {
          if (wave == 0) {
            const double theta = tri_top_eigenvalue(alpha, beta, j + 1, lane);
            if (lane == 0) {
              tri_eigenvector(alpha, beta, j + 1, theta, ty, twork);
              const double resid = beta_j * fabs(ty[j]);
              s_done = (resid <= 5e-15 * fabs(theta)) || last || beta_j <= 1e-300 * fabs(theta) ||
                        beta_j == 0.0;
              if (last && !(resid <= 5e-15 * fabs(theta)) && P.diag) atomicAdd(P.diag, 1);
            }
          }
          __syncthreads();
          if (s_done) break;
        }
        const double inv = 1.0 / beta_j;
        for (int c = tid; c < k; c += NR_BS) q[c] = w[c] * inv;
        __syncthreads();
      }
      // Ritz vector v = Q y, then G v
      for (int c = tid; c < k; c += NR_BS) {
        double s = 0.0;
        for (int i = 0; i < nsteps; ++i) s += ty[i] * Q[(int64_t)i * k + c];
        vv[c] = s;
      }
      __syncthreads();
      {
        double a[1] = {0.0};
        for (int c = tid; c < k; c += NR_BS) a[0] += vv[c] * vv[c];
        block_sums<1>(a, red);
        const double inv = 1.0 / sqrt(a[0]);
        for (int c = tid; c < k; c += NR_BS) vv[c] *= inv;
      }
      __syncthreads();
      for (int r = tid; r < k; r += NR_BS) {
        double s = 0.0;
        for (int c = 0; c < k; ++c) s += G[r + (int64_t)c * kp] * vv[c];
        gv[r] = s;
      }
      __syncthreads();
      // lambda = v.Gv, ubar = sum_j m_j v_j / sigma
      double a3[2] = {0.0, 0.0};
      for (int c = tid; c < k; c += NR_BS) {
        a3[0] += vv[c] * gv[c];
        a3[1] += colm[c] * vv[c];
      }
      block_sums<2>(a3, red);
      const double lambda = a3[0];
      const double sigma = sqrt(lambda);
      const double ubar = a3[1] / sigma;
      const double Sd = (double)S;
      const double var_u = 1.0 - Sd * ubar * ubar;  // sum (u - ubar)^2 with |u| = 1
      // orientation: sign(cor(meanObs, u)) (src/netStats.cpp:242-247)
      double a4[3] = {0.0, 0.0, 0.0};
      for (int c = tid; c < k; c += NR_BS) a4[0] += gv[c] / sigma - Sd * colm[c] * ubar;
      for (int r = tid; r < S; r += NR_BS) a4[1] += mo[r];
      block_sums<3>(a4, red);
      const double mo_mean = a4[1] / Sd;
      double a5[1] = {0.0};
      for (int r = tid; r < S; r += NR_BS) a5[0] += (mo[r] - mo_mean) * (mo[r] - mo_mean);
      block_sums<1>(a5, red);
      const bool flip = (a4[0] < 0.0) && (a5[0] > 0.0) && (var_u > 0.0);
      const double sgn = flip ? -1.0 : 1.0;
      // NC_j = cor(x_j, u) (src/netStats.cpp:279), node order = CSR order
      for (int c = tid; c < k; c += NR_BS) {
        const double gjj = G[c + (int64_t)c * kp];
        const double cov = gv[c] / sigma - Sd * colm[c] * ubar;
        const double var_x = gjj - Sd * colm[c] * colm[c];
        w[c] = sgn * cov / (sqrt(var_x) * sqrt(var_u));
      }
      if (P.sp_out) {
        for (int r = tid; r < S; r += NR_BS) {
          double s = 0.0;
          for (int c = 0; c < k; ++c) s += X[(int64_t)idx[c] * S + r] * vv[c];
          P.sp_out[(int64_t)m * S + r] = sgn * s / sigma;
        }
      }
      __syncthreads();
    } else {
      for (int c = tid; c < k; c += NR_BS) w[c] = nr_nan();
      if (P.sp_out)
        for (int r = tid; r < S; r += NR_BS) P.sp_out[(int64_t)m * S + r] = nr_nan();
      __syncthreads();
    }

    // ModuleCoherence (src/netStats.cpp:293-305), Correlation / SignAwareMean
    // against the discovery contribution (src/permutations.cpp:99,101).
    double b1[5] = {0, 0, 0, 0, 0};  // nfinite, sum nc^2, ncc, sx, sy
    for (int c = tid; c < k; c += NR_BS) {
      const double y = w[c];
      if (isfinite(y)) { b1[0] += 1.0; b1[1] += y * y; }
      if (P.disc_nc) {
        const double xv = P.disc_nc[off + c];
        if (isfinite(xv) && isfinite(y)) { b1[2] += 1.0; b1[3] += xv; b1[4] += y; }
      }
      if (P.nc_out) P.nc_out[off + c] = y;
    }
    block_sums<5>(b1, red);
    stat_coh = b1[0] >= 1.0 ? b1[1] / b1[0] : nr_nan();
    if (P.disc_nc && P.out) {
      const double mx = b1[3] / b1[2], my = b1[4] / b1[2];
      double b2[4] = {0, 0, 0, 0};
      for (int c = tid; c < k; c += NR_BS) {
        const double y = w[c], xv = P.disc_nc[off + c];
        if (isfinite(xv) && isfinite(y)) {
          const double dx = xv - mx, dy = y - my;
          b2[0] += dx * dx;
          b2[1] += dy * dy;
          b2[2] += dx * dy;
          b2[3] += (xv > 0.0 ? y : (xv < 0.0 ? -y : 0.0));
        }
      }
      block_sums<4>(b2, red);
      stat_cc = b1[2] >= 1.0 ? b2[2] / (sqrt(b2[0]) * sqrt(b2[1])) : nr_nan();
      stat_ac = b1[2] >= 1.0 ? b2[3] / b1[2] : nr_nan();
    }
    if (tid == 0) {
      if (P.out) {
        double* o = P.out + (int64_t)P.row_of[m] + (int64_t)P.n_rows * (int64_t)P.n_stat * p_local;
        o[(int64_t)P.n_rows * P.slot_coherence] = na_fill(stat_coh);
        o[(int64_t)P.n_rows * P.slot_cor_contrib] = na_fill(stat_cc);
        o[(int64_t)P.n_rows * P.slot_avg_contrib] = na_fill(stat_ac);
      }
      if (P.coh_out) P.coh_out[m] = stat_coh;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Support kernels
// ---------------------------------------------------------------------------

// {corr, net} interleave (one 16-byte element per (i, j)).
__global__ void interleave_kernel(const double* __restrict__ corr, const double* __restrict__ net,
                                  double2* __restrict__ out, int64_t n_elem) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_elem;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = make_double2(corr[i], net[i]);
}

// Exact symmetry check of the interleaved matrix via 32x32 LDS tiles: block
// (I, J), J >= I, stages A(J, I) in LDS and compares it with A(I, J); both
// reads are coalesced along rows.
__global__ void symmetry_kernel(const double2* __restrict__ a, int64_t n, int* asym) {
  __shared__ double2 tile[32][33];
  const int64_t bi = (int64_t)blockIdx.y * 32, bj = (int64_t)blockIdx.x * 32;
  if (bj < bi) return;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int64_t row = bj + tx, col = bi + r;               // tile[r][c] = A(bj + c, bi + r)
    tile[r][tx] = (row < n && col < n) ? a[row + col * n] : make_double2(0.0, 0.0);
  }
  __syncthreads();
  int bad = 0;
  for (int r = ty; r < 32; r += 8) {
    const int64_t row = bi + tx, col = bj + r;               // A(bi + c, bj + r) vs tile[c][r]
    if (row < n && col < n) {
      const double2 x = a[row + col * n];
      const double2 t = tile[tx][r];
      bad |= (x.x != t.x) | (x.y != t.y);
    }
  }
  if (bad) atomicOr(asym, 1);
}

// Scale (src/scale.cpp:14-25): one wave per column; arma mean + corrected
// two-pass variance with n-1 normalisation.
__global__ void scale_kernel(const double* __restrict__ in, double* __restrict__ out, int64_t S,
                             int64_t N) {
  const int lane = threadIdx.x & 63;
  const int64_t col = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (col >= N) return;
  const double* x = in + col * S;
  double s = 0.0;
  for (int64_t r = lane; r < S; r += 64) s += x[r];
  s = wave_sum(s);
  const double mean = s / (double)S;
  double a2 = 0.0, a3 = 0.0;
  for (int64_t r = lane; r < S; r += 64) {
    const double t = mean - x[r];
    a2 += t * t;
    a3 += t;
  }
  a2 = wave_sum(a2);
  a3 = wave_sum(a3);
  const double var = (a2 - a3 * a3 / (double)S) / (double)(S - 1);
  const double sd = sqrt(var);
  double* o = out + col * S;
  for (int64_t r = lane; r < S; r += 64) o[r] = (x[r] - mean) / sd;
}

__global__ void finite_kernel(const double* __restrict__ a, int64_t n, int* nonfinite) {
  int bad = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    bad |= !isfinite(a[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(nonfinite, 1);
}

// Exported index sets of permutations (nr_export_indices).
__global__ void export_indices_kernel(IndexSource src, int64_t n_nodes_total, int32_t* out,
                                      int64_t n_perm) {
  const int64_t p = blockIdx.y;
  if (p >= n_perm) return;
  nr_prp_key key;
  if (src.mode == NR_IDX_PRP) key = nr_prp_make_key(src.seed, (uint64_t)(src.perm_base + p), src.n_null);
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n_nodes_total;
       c += (int64_t)gridDim.x * blockDim.x)
    out[p * n_nodes_total + c] = (int32_t)node_index(src, key, p, c);
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
size_t net_kernel_lds(int k_max) { return sizeof(double) * (8 * NR_WAVES + k_max) + sizeof(uint32_t) * k_max; }

size_t profile_kernel_lds(int k_max, int m_max, int n_samples) {
  return sizeof(double) * (8 * NR_WAVES + 5 * (size_t)k_max + n_samples + 9 * (size_t)m_max) +
         sizeof(uint32_t) * k_max;
}

hipError_t launch_net(const NetParams& P, int64_t n_items, hipStream_t st) {
  const size_t lds = net_kernel_lds(P.k_max);
  hipLaunchKernelGGL(module_net_kernel, dim3((unsigned)n_items), dim3(NR_BS), lds, st, P);
  return hipGetLastError();
}

hipError_t launch_profile(const ProfileParams& P, int n_slots, hipStream_t st) {
  const size_t lds = profile_kernel_lds(P.k_max, P.m_max, (int)P.n_samples);
  hipLaunchKernelGGL(module_profile_kernel, dim3((unsigned)n_slots), dim3(NR_BS), lds, st, P);
  return hipGetLastError();
}

hipError_t launch_interleave(const double* corr, const double* net, double2* out, int64_t n_elem,
                             hipStream_t st) {
  hipLaunchKernelGGL(interleave_kernel, dim3(4096), dim3(256), 0, st, corr, net, out, n_elem);
  return hipGetLastError();
}

hipError_t launch_symmetry(const double2* a, int64_t n, int* asym, hipStream_t st) {
  const unsigned nb = (unsigned)((n + 31) / 32);
  hipLaunchKernelGGL(symmetry_kernel, dim3(nb, nb), dim3(256), 0, st, a, n, asym);
  return hipGetLastError();
}

hipError_t launch_scale(const double* in, double* out, int64_t S, int64_t N, hipStream_t st) {
  const unsigned nb = (unsigned)((N + 3) / 4);
  hipLaunchKernelGGL(scale_kernel, dim3(nb), dim3(256), 0, st, in, out, S, N);
  return hipGetLastError();
}

hipError_t launch_finite(const double* a, int64_t n, int* nonfinite, hipStream_t st) {
  hipLaunchKernelGGL(finite_kernel, dim3(2048), dim3(256), 0, st, a, n, nonfinite);
  return hipGetLastError();
}

hipError_t launch_export(const IndexSource& src, int64_t n_nodes_total, int32_t* out,
                         int64_t n_perm, hipStream_t st) {
  const unsigned gx = (unsigned)((n_nodes_total + 255) / 256 < 64 ? (n_nodes_total + 255) / 256 : 64);
  hipLaunchKernelGGL(export_indices_kernel, dim3(gx > 0 ? gx : 1, (unsigned)n_perm), dim3(256), 0, st,
                     src, n_nodes_total, out, n_perm);
  return hipGetLastError();
}

}  // namespace nr
