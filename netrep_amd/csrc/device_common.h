// Device helpers shared by the engine's kernels (kernels.hip, kernels_rg4.hip):
// wave/block reductions, R's NA_real_, the index source of a permuted module
// (GetRandomIdx, src/utils.cpp:193-199), CorrVector pair decoding, register
// butterflies on gfx950 (permlane swaps, DPP), the Lanczos tridiagonal
// helpers (top eigenvalue / residual / eigenvector, partial
// reorthogonalisation's omega recurrence) and diagnostic phase stamps.
#pragma once
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

__device__ __forceinline__ double nr_wave_sum(double v);
__device__ __forceinline__ double nr_wave_max(double v);
// Wave-wide sum (every lane active); register butterflies, see nr_wave_sum.
__device__ __forceinline__ double wave_sum(double v) { return nr_wave_sum(v); }

// Workgroup barrier of an NW-wave workgroup. One wave (the wave class): a
// wavefront-scope fence only -- a wave's LDS and vector-memory operations are
// performed in program order, so the s_barrier and the release fence's wait
// for outstanding global stores (the Lanczos basis, the cube) are not needed.
template <int NW>
__device__ __forceinline__ void nr_sync() {
  if constexpr (NW == 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// Block-wide sums of N values; result broadcast to every thread. `red` must
// hold N * NR_WAVES doubles of LDS. Contains two barriers (one with
// TRAIL = false: then `red` must not be written again before a later barrier).
template <int N, int NW = NR_WAVES, bool TRAIL = true>
__device__ __forceinline__ void block_sums(double (&v)[N], double* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = wave_sum(v[i]);
  if constexpr (NW == 1) return;  // one wave: every lane has the sums (no LDS round trip)
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) red[i * NW + wave] = v[i];
  }
  nr_sync<NW>();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[i * NW + w];
    v[i] = s;
  }
  if (TRAIL) nr_sync<NW>();
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
// Kernel 2: summary-profile statistics. Persistent workgroups pull items from
// a queue; each owns a scratch slot holding G = X^T X and the Lanczos basis.
// ---------------------------------------------------------------------------
typedef double nr_f64x4 __attribute__((ext_vector_type(4)));

// 1/d: v_rcp_f64 refined by two Newton steps as in the compiler's own
// division expansion, without its scaling/fixup (d normal, |d| >= 1e-300);
// used only in the Sturm counts of the Ritz checks.
__device__ __forceinline__ double nr_rcp(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  r = fma(r, fma(-d, r, 1.0), r);
  return r;
}

// Largest eigenvalue of the symmetric tridiagonal (alpha[0..n), beta[0..n-1))
// by 64-way multisection on Sturm counts; executed by one full wave. The
// counts use the characteristic-polynomial recurrence of the Gershgorin-
// normalised matrix, p_i = (a_i - x) p_{i-1} - b_{i-1}^2 p_{i-2} (sign changes
// of p_0..p_n = eigenvalues below x): one FMA on the dependency chain per
// step and no division; |p| is renormalised every 4 steps. Each pass puts
// lane l's point at lo + (hi - lo) (l + 1) / 64 (lane 63 on hi, an upper
// bound already counted: the division by 64 is exact, no divide on the wave's
// path) and keeps the one-64th subinterval the counts bracket.
//
// Warm start (r_prev > 0): theta_lo, a lower end of an earlier check's
// bracket of the top Ritz value, is a lower bound (Cauchy interlacing), and
// its Ritz residual r_prev bounds the distance to an eigenvalue of the grown
// matrix, so the top one lies in [theta_lo, theta_lo + 1.01 r_prev] unless
// the first pass finds eigenvalues above it; then the search continues to the
// Gershgorin bound.
//
// Two stages (round 6): sturm_init (bounds, warm bracket, the normalised
// coefficients) and sturm_passes(width) narrowing the bracket to `width`; a
// Ritz check first narrows to 1e-9 of the scale, which is all its residual
// estimate needs (tri_top_resid's relative error is O(bracket / gap of T), not
// O(bracket / residual)), and goes on to 2e-16 only where the run may stop
// (lanczos_ritz).
//
// wa, wb (n doubles of LDS each): the normalised recurrence coefficients
// alpha_i / scale and (beta_i / scale)^2, computed once by the wave instead
// of in every pass (the passes are issue-bound).
struct SturmBracket {
  double lo, hi, g_hi, scale, inv;
  bool warm;
  int passes;
};

static __device__ __forceinline__ void sturm_coeffs(const double* alpha, const double* beta, int n, int lane,
                                                    double inv, double* wa, double* wb) {
  for (int i = lane; i < n; i += 64) {
    wa[i] = alpha[i] * inv;
    if (i < n - 1) {
      const double b = beta[i] * inv;
      wb[i] = b * b;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

static __device__ __forceinline__ SturmBracket sturm_init(const double* alpha, const double* beta, int n, int lane,
                                                          double theta_lo, double r_prev, double* wa, double* wb) {
  double lo = alpha[0], hi = alpha[0];
  for (int i = lane; i < n; i += 64) {
    const double r = (i > 0 ? fabs(beta[i - 1]) : 0.0) + (i < n - 1 ? fabs(beta[i]) : 0.0);
    lo = fmin(lo, alpha[i] - r);
    hi = fmax(hi, alpha[i] + r);
  }
  lo = -nr_wave_max(-lo);  // register butterflies (DPP, permlane), no LDS round trips
  hi = nr_wave_max(hi);
  SturmBracket b;
  b.scale = fmax(fabs(lo), fabs(hi)) + 1e-300;
  b.inv = 1.0 / b.scale;
  lo -= 1e-14 * b.scale;
  hi += 1e-14 * b.scale;
  b.g_hi = hi;
  b.warm = r_prev > 0.0 && isfinite(r_prev) && theta_lo - 4e-16 * b.scale > lo &&
           theta_lo + 1.01 * r_prev + 4e-16 * b.scale < hi;
  if (b.warm) {
    lo = theta_lo - 4e-16 * b.scale;
    hi = theta_lo + 1.01 * r_prev + 4e-16 * b.scale;
  }
  b.lo = lo;
  b.hi = hi;
  b.passes = 0;
  sturm_coeffs(alpha, beta, n, lane, b.inv, wa, wb);
  return b;
}

static __device__ __forceinline__ void sturm_passes(SturmBracket& b, int n, int lane, const double* wa,
                                                    const double* wb, double width) {
  double lo = b.lo, hi = b.hi;
  const double inv = b.inv;
  const double frac = (double)(lane + 1) * 0.015625;  // (lane + 1) / 64, exact
  // (a warm bracket takes one pass whatever its width: that pass checks it)
  while (b.passes < 16 && (hi - lo > width || b.warm)) {
    ++b.passes;
    const double x = (lo + (hi - lo) * frac) * inv;
    double p0 = 1.0, p1 = wa[0] - x;
    int cnt = p1 < 0.0;  // eigenvalues < x
    // a sign change between p_{i-1} and p_i: the sign bits differ
    auto step = [&](double a, double bb) {
      const double p2 = fma(a - x, p1, -bb * p0);
      cnt += (int)((__double2hiint(p2) ^ __double2hiint(p1)) >> 31 & 1);
      p0 = p1;
      p1 = p2;
    };
    auto renorm = [&]() {
      const double mg = fabs(p1);
      const double s = mg > 1e150 ? 1e-150 : (mg < 1e-150 ? 1e150 : 1.0);
      p0 *= s;
      p1 *= s;
    };
    // 8 steps' coefficients read ahead of their recurrence steps, so the LDS
    // latency is paid once per 8 steps instead of on the dependency chain of
    // every step; whole groups of 8 carry no per-step bounds test
    int i0 = 1;
    for (; i0 + 8 <= n; i0 += 8) {
      double av[8], bv[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        av[t] = wa[i0 + t];
        bv[t] = wb[i0 + t - 1];
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        step(av[t], bv[t]);
        if ((t & 3) == 3) renorm();  // i = i0 + t with i0 = 1 mod 8: i = 0 mod 4
      }
    }
    for (int i = i0; i < n; ++i) {
      step(wa[i], wb[i - 1]);
      if ((i & 3) == 0) renorm();
    }
    // lanes are ordered by x: lanes [0, t) have cnt <= n-1, lanes [t, 64) have cnt == n
    const int t = __popcll(__ballot(cnt <= n - 1));
    if (t == 64) {  // eigenvalues above the bracket (a warm start's residual bound): search above it
      lo = hi;
      hi = b.g_hi;
      b.warm = false;
      continue;
    }
    const double xlo = lo + (hi - lo) * ((double)t * 0.015625);
    const double xhi = lo + (hi - lo) * ((double)(t + 1) * 0.015625);
    lo = xlo;
    hi = xhi;
    b.warm = false;
  }
  b.lo = lo;
  b.hi = hi;
}

// Convergence estimate of the top Ritz pair: |last component| of the unit
// eigenvector y of the tridiagonal for theta, times beta_j. y comes from the
// three-term recurrence run BACKWARDS from y_{n-1} = 1: the top eigenvector
// of an unreduced Jacobi matrix is positive and its tail decays once the
// pair converges, so upward it is the dominant (stable) solution. rb holds
// 1/beta[0..n-1), one wave fills it. Returns beta_j / |y| (every lane). The
// recurrence reads its coefficients eight steps ahead (round 6: the LDS
// latency off the dependency chain; the same arithmetic in the same order).
static __device__ __forceinline__ double tri_top_resid(const double* alpha, const double* beta, int n, double theta,
                                                       double beta_j, double* rb, int lane) {
  for (int i = lane; i < n - 1; i += 64) rb[i] = 1.0 / beta[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double y1 = 1.0, y2 = 0.0, ss = 1.0;  // y_i, y_{i+1}, sum of squares
  auto step = [&](double a, double b, double r) {
    const double y0 = fma(theta - a, y1, -b * y2) * r;
    ss = fma(y0, y0, ss);
    y2 = y1;
    y1 = y0;
  };
  // Overflow guard, every fourth step, by selects: the scale is a power of
  // two (exact), so the result is the unscaled one bit for bit. Round 6: a
  // test per step compiled to an exec-mask branch on the recurrence's chain
  // (compare, s_and_saveexec, s_or) and tripled each step's latency. After a
  // guard ss <= 2^256, so four steps may grow y by 2^384 before ss overflows.
  auto renorm = [&]() {
    const int e = ss > 0x1p256 ? -256 : 0;  // v_ldexp: no 64-bit constants to keep live
    y1 = ldexp(y1, e);
    y2 = ldexp(y2, e);
    beta_j = ldexp(beta_j, e);
    ss = ldexp(ss, 2 * e);
  };
  int i = n - 1;
  for (; i >= 8; i -= 8) {  // steps i .. i - 7, all >= 1
    double av[8], bv[8], rv[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      av[t] = alpha[i - t];
      bv[t] = i - t < n - 1 ? beta[i - t] : 0.0;
      rv[t] = rb[i - t - 1];
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      step(av[t], bv[t], rv[t]);
      if ((t & 3) == 3) renorm();
    }
  }
  for (; i > 0; --i) {
    step(alpha[i], i < n - 1 ? beta[i] : 0.0, rb[i - 1]);
    if ((i & 3) == 0) renorm();  // i is wave-uniform: a scalar branch
  }
  return beta_j / sqrt(ss);
}

// log2 of a positive double for the Ritz checks' step predictions: exponent
// plus the fp32 log2 of the mantissa (v_log_f32), ~1e-7 absolute; the library
// log's ~40 dependent instructions sat on lane 0 of a check's serial path.
static __device__ __forceinline__ double nr_log2_fast(double x) {
  const int e = __builtin_amdgcn_frexp_exp(x);
  const float m = (float)__builtin_amdgcn_frexp_mant(x);
  return (double)e + (double)__builtin_amdgcn_logf(m);
}

// Eigenvector of the tridiagonal for eigenvalue theta by two steps of inverse
// iteration; LU with partial pivoting as LAPACK dgttrf/dgtts2. Single lane.
// y[0..n) comes back normalised; work holds 5n doubles. The recurrences carry
// their running values in registers (the pivot, the super-diagonal, y_i and
// y_{i+1}) and the pivots are stored as reciprocals, so each step's
// dependency chain is one or two FMAs instead of an LDS round trip and a
// division (round 5: a single-wave item had no other wave to hide the old
// loop behind, 12% of a C2 item). The second step starts from the first
// step's result scaled by 1/max (proportional to the normalised vector the
// old loop passed on: the same direction to rounding).
// Round 6: every loop reads its operands a group of G steps ahead of the
// recurrence (the compiler had put one LDS read and its wait on each step's
// chain); the same arithmetic in the same order. G = 1 keeps the previous
// loops (the large-module kernel: with the groups its register allocation
// moved spill code into its Gram loop).
template <int G>
static __device__ __forceinline__ void tri_eigenvector(const double* __restrict__ alpha,
                                                       const double* __restrict__ beta, int n, double theta,
                                                       double* __restrict__ y, double* __restrict__ work) {
  if constexpr (G == 1) {  // the previous loops
    double* __restrict__ dl = work;
    double* __restrict__ rd = work + n;   // 1 / pivot
    double* __restrict__ du = work + 2 * n;
    double* __restrict__ du2 = work + 3 * n;
    double* __restrict__ swp = work + 4 * n;
    double scale = fabs(theta);
  #pragma unroll 4
    for (int i = 0; i < n; ++i) {
      scale = fmax(scale, fabs(alpha[i]));
      if (i < n - 1) scale = fmax(scale, fabs(beta[i]));
    }
    const double floor_piv = 1e-300 + 2.2e-16 * scale;
    double di = alpha[0] - theta;          // current pivot candidate d_i
    double dui = n > 1 ? beta[0] : 0.0;    // current super-diagonal du_i
    // branch-free steps (selects instead of the two pivoting paths), so the
    // loop unrolls and the next steps' LDS reads overlap this step's chain
  #pragma unroll 4
    for (int i = 0; i < n - 1; ++i) {
      const double bi = beta[i];                       // sub-diagonal dl_i
      const double dn = alpha[i + 1] - theta;          // d_{i+1} before this step
      const double dun = i < n - 2 ? beta[i + 1] : 0.0;  // du_{i+1} before this step
      const bool sw = !(fabs(di) >= fabs(bi));         // row interchange
      const double dc = fabs(di) < floor_piv ? (di < 0.0 ? -floor_piv : floor_piv) : di;
      const double r = 1.0 / (sw ? bi : dc);
      const double f = (sw ? di : bi) * r;
      dl[i] = f;
      rd[i] = r;
      du[i] = sw ? dn : dui;
      du2[i] = sw ? dun : 0.0;
      swp[i] = sw ? 1.0 : 0.0;
      const double ndi = sw ? dui - f * dn : dn - f * dui;
      dui = sw ? -f * dun : dun;
      di = ndi;
    }
    if (fabs(di) < floor_piv) di = di < 0.0 ? -floor_piv : floor_piv;
    rd[n - 1] = 1.0 / di;
    double sc = 1.0;  // scale of the right-hand side (1 / max of the previous iterate)
    for (int iter = 0; iter < 2; ++iter) {
      // L solve (the row interchanges applied as the factorisation made them)
      double yi = iter == 0 ? 1.0 : y[0] * sc;
  #pragma unroll 4
      for (int i = 0; i < n - 1; ++i) {
        const double yn = iter == 0 ? 1.0 : y[i + 1] * sc;
        const bool sw = swp[i] != 0.0;
        const double a = sw ? yn : yi, b = sw ? yi : yn;
        y[i] = a;
        yi = b - dl[i] * a;
      }
      // U solve (bandwidth 3)
      double y1 = yi * rd[n - 1], y2 = 0.0;
      y[n - 1] = y1;
      double mx = fabs(y1);
  #pragma unroll 4
      for (int i = n - 2; i >= 0; --i) {
        const double y0 = (y[i] - du[i] * y1 - du2[i] * y2) * rd[i];
        y[i] = y0;
        mx = fmax(mx, fabs(y0));
        y2 = y1;
        y1 = y0;
      }
      sc = 1.0 / mx;
    }
    double nrm = 0.0;
  #pragma unroll 4
    for (int i = 0; i < n; ++i) {
      const double v = y[i] * sc;
      y[i] = v;
      nrm += v * v;
    }
    const double inv = 1.0 / sqrt(nrm);
  #pragma unroll 4
    for (int i = 0; i < n; ++i) y[i] *= inv;
  } else {
    double* __restrict__ dl = work;
    double* __restrict__ rd = work + n;   // 1 / pivot
    double* __restrict__ du = work + 2 * n;
    double* __restrict__ du2 = work + 3 * n;
    double* __restrict__ swp = work + 4 * n;
    double scale = fabs(theta);
  #pragma unroll 4
    for (int i = 0; i < n; ++i) {
      scale = fmax(scale, fabs(alpha[i]));
      if (i < n - 1) scale = fmax(scale, fabs(beta[i]));
    }
    const double floor_piv = 1e-300 + 2.2e-16 * scale;
    double di = alpha[0] - theta;          // current pivot candidate d_i
    double dui = n > 1 ? beta[0] : 0.0;    // current super-diagonal du_i
    // branch-free steps (selects instead of the two pivoting paths)
    auto lu_step = [&](int i, double bi, double dn, double dun) {  // bi = dl_i, d_{i+1} and du_{i+1} before the step
      const bool sw = !(fabs(di) >= fabs(bi));         // row interchange
      const double dc = fabs(di) < floor_piv ? (di < 0.0 ? -floor_piv : floor_piv) : di;
      const double r = 1.0 / (sw ? bi : dc);
      const double f = (sw ? di : bi) * r;
      dl[i] = f;
      rd[i] = r;
      du[i] = sw ? dn : dui;
      du2[i] = sw ? dun : 0.0;
      swp[i] = sw ? 1.0 : 0.0;
      const double ndi = sw ? dui - f * dn : dn - f * dui;
      dui = sw ? -f * dun : dun;
      di = ndi;
    };
    int i = 0;
    for (; i + G <= n - 1; i += G) {
      double bv[G], dv[G], uv[G];
  #pragma unroll
      for (int t = 0; t < G; ++t) {
        bv[t] = beta[i + t];
        dv[t] = alpha[i + t + 1] - theta;
        uv[t] = i + t < n - 2 ? beta[i + t + 1] : 0.0;
      }
  #pragma unroll
      for (int t = 0; t < G; ++t) lu_step(i + t, bv[t], dv[t], uv[t]);
    }
    for (; i < n - 1; ++i) lu_step(i, beta[i], alpha[i + 1] - theta, i < n - 2 ? beta[i + 1] : 0.0);
    if (fabs(di) < floor_piv) di = di < 0.0 ? -floor_piv : floor_piv;
    rd[n - 1] = 1.0 / di;
    double sc = 1.0;  // scale of the right-hand side (1 / max of the previous iterate)
    for (int iter = 0; iter < 2; ++iter) {
      // L solve (the row interchanges applied as the factorisation made them)
      double yi = iter == 0 ? 1.0 : y[0] * sc;
      auto l_step = [&](int i, double yn, double s, double l) {
        const bool sw = s != 0.0;
        const double a = sw ? yn : yi, b = sw ? yi : yn;
        y[i] = a;
        yi = b - l * a;
      };
      i = 0;
      for (; i + G <= n - 1; i += G) {  // y[i + 1 ..] read before this group writes y[i ..]: the old values
        double yv[G], sv[G], lv[G];
  #pragma unroll
        for (int t = 0; t < G; ++t) {
          yv[t] = iter == 0 ? 1.0 : y[i + t + 1] * sc;
          sv[t] = swp[i + t];
          lv[t] = dl[i + t];
        }
  #pragma unroll
        for (int t = 0; t < G; ++t) l_step(i + t, yv[t], sv[t], lv[t]);
      }
      for (; i < n - 1; ++i) l_step(i, iter == 0 ? 1.0 : y[i + 1] * sc, swp[i], dl[i]);
      // U solve (bandwidth 3)
      double y1 = yi * rd[n - 1], y2 = 0.0;
      y[n - 1] = y1;
      double mx = fabs(y1);
      auto u_step = [&](int i, double yv, double u, double u2, double r) {
        const double y0 = (yv - u * y1 - u2 * y2) * r;
        y[i] = y0;
        mx = fmax(mx, fabs(y0));
        y2 = y1;
        y1 = y0;
      };
      i = n - 2;
      for (; i >= G - 1; i -= G) {  // steps i .. i - G + 1, all >= 0
        double yv[G], uv[G], u2[G], rv[G];
  #pragma unroll
        for (int t = 0; t < G; ++t) {
          yv[t] = y[i - t];
          uv[t] = du[i - t];
          u2[t] = du2[i - t];
          rv[t] = rd[i - t];
        }
  #pragma unroll
        for (int t = 0; t < G; ++t) u_step(i - t, yv[t], uv[t], u2[t], rv[t]);
      }
      for (; i >= 0; --i) u_step(i, y[i], du[i], du2[i], rd[i]);
      sc = 1.0 / mx;
    }
    double nrm = 0.0;
    i = 0;
    for (; i + G <= n; i += G) {
      double v[G];
  #pragma unroll
      for (int t = 0; t < G; ++t) v[t] = y[i + t] * sc;
  #pragma unroll
      for (int t = 0; t < G; ++t) {
        y[i + t] = v[t];
        nrm += v[t] * v[t];
      }
    }
    for (; i < n; ++i) {
      const double v = y[i] * sc;
      y[i] = v;
      nrm += v * v;
    }
    const double inv = 1.0 / sqrt(nrm);
  #pragma unroll 4
    for (int i = 0; i < n; ++i) y[i] *= inv;
  }
}

// Partial reorthogonalisation (Simon 1984): omega_{j+1,i} estimates q_{j+1}.q_i
// from the recurrence on T's entries; run by one wave over i = 0..j. Returns
// max_i |omega_{j+1,i}| (all lanes). om_cur = omega_{j,.}, om_prev = omega_{j-1,.}.
__device__ __forceinline__ double omega_update(const double* alpha, const double* beta, int j, double alpha_j,
                                               double beta_j,
                                               const double* om_cur, const double* om_prev, double* om_next,
                                               double anorm, int k, int lane) {
  const double eps = 2.220446049250313e-16;
  const double rbj = nr_rcp(beta_j);  // omega is an estimate: the reciprocal's last-bit error is immaterial
  const double psi = eps * anorm * rbj;
  double mx = 0.0;
  for (int i = lane; i < j; i += 64) {
    double t = beta[i] * om_cur[i + 1] + (alpha[i] - alpha_j) * om_cur[i] -
               (j > 0 ? beta[j - 1] * om_prev[i] : 0.0);
    if (i > 0) t += beta[i - 1] * om_cur[i - 1];
    t = t * rbj;
    t += t >= 0.0 ? psi : -psi;
    om_next[i] = t;
    mx = fmax(mx, fabs(t));
  }
  if (lane == 0) {
    om_next[j] = eps * sqrt((double)k) * anorm / beta_j;
    om_next[j + 1] = 1.0;
    mx = fmax(mx, fabs(om_next[j]));
  }
  return nr_wave_max(mx);
}

// Cross-lane butterfly steps without LDS (gfx950): v_permlane32_swap /
// v_permlane16_swap exchange half-waves / odd-even rows of two registers, so
// x' + y' leaves lanes [0,32) with x summed over the lane pair (l, l^32) and
// lanes [32,64) with y summed likewise (16-lane rows for the 16 variant).
__device__ __forceinline__ double nr_swap32_sum(double x, double y) {
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(y), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(y), false, false);
  return __hiloint2double((int)hi[0], (int)lo[0]) + __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ double nr_swap16_sum(double x, double y) {
  const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(y), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(y), false, false);
  return __hiloint2double((int)hi[0], (int)lo[0]) + __hiloint2double((int)hi[1], (int)lo[1]);
}
// DPP lane moves within 16-lane rows (both dwords of a double).
template <int CTRL>
__device__ __forceinline__ double nr_dpp(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
constexpr int NR_DPP_XOR1 = 0xB1;         // quad_perm [1,0,3,2]
constexpr int NR_DPP_XOR2 = 0x4E;         // quad_perm [2,3,0,1]
constexpr int NR_DPP_ROR8 = 0x128;        // row_ror:8 == lane ^ 8 within a row
constexpr int NR_DPP_HALF_MIRROR = 0x141; // lane ^ 7 within 8 lanes (flips bit 2)

// Wave-wide sum / max in registers (DPP within 16-lane rows, permlane swaps
// across rows; no LDS round trips). Every lane ends with the same value.
__device__ __forceinline__ double nr_wave_sum(double v) {
  v += nr_dpp<NR_DPP_XOR1>(v);
  v += nr_dpp<NR_DPP_XOR2>(v);
  v += nr_dpp<NR_DPP_HALF_MIRROR>(v);  // quads are uniform: lane ^ 4
  v += nr_dpp<NR_DPP_ROR8>(v);
  v = nr_swap16_sum(v, v);
  return nr_swap32_sum(v, v);
}
__device__ __forceinline__ double nr_swap16_max(double x) {
  const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(x), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(x), false, false);
  return fmax(__hiloint2double((int)hi[0], (int)lo[0]), __hiloint2double((int)hi[1], (int)lo[1]));
}
__device__ __forceinline__ double nr_swap32_max(double x) {
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(x), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(x), false, false);
  return fmax(__hiloint2double((int)hi[0], (int)lo[0]), __hiloint2double((int)hi[1], (int)lo[1]));
}
__device__ __forceinline__ double nr_wave_max(double v) {
  v = fmax(v, nr_dpp<NR_DPP_XOR1>(v));
  v = fmax(v, nr_dpp<NR_DPP_XOR2>(v));
  v = fmax(v, nr_dpp<NR_DPP_HALF_MIRROR>(v));
  v = fmax(v, nr_dpp<NR_DPP_ROR8>(v));
  return nr_swap32_max(nr_swap16_max(v));
}

// Sum over the 16 lanes of each DPP row (lanes 16r..16r+15); every lane of
// the row ends with its row's total. Fixed order: bitwise reproducible.
__device__ __forceinline__ double nr_row_sum16(double v) {
  v += nr_dpp<NR_DPP_XOR1>(v);
  v += nr_dpp<NR_DPP_XOR2>(v);
  v += nr_dpp<NR_DPP_HALF_MIRROR>(v);  // quads are uniform: lane ^ 4
  v += nr_dpp<NR_DPP_ROR8>(v);
  return v;
}

// Lane l's double, broadcast to the wave (two v_readlane_b32: SGPR result).
__device__ __forceinline__ double nr_readlane_f64(double v, int l) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// Transpose-reduce of 16 per-lane column partials up[0..16) over the 64 rows
// (lanes) of a unit: afterwards lanes with (lane & 3) == 0 hold the column
// sum of column 8*b5 + 4*b4 + 2*b3 + b2 (b = lane bits). 8 + 4 swaps, 3 + 2
// DPP-exchange levels; no LDS traffic.
__device__ __forceinline__ double nr_transpose_reduce16(const double (&up)[16], int lane) {
  double a8[8], a4[4], a2[2];
#pragma unroll
  for (int i = 0; i < 8; ++i) a8[i] = nr_swap32_sum(up[i], up[i + 8]);
#pragma unroll
  for (int i = 0; i < 4; ++i) a4[i] = nr_swap16_sum(a8[i], a8[i + 4]);
  const bool b3 = lane & 8;
#pragma unroll
  for (int i = 0; i < 2; ++i)
    a2[i] = (b3 ? a4[i + 2] : a4[i]) + nr_dpp<NR_DPP_ROR8>(b3 ? a4[i] : a4[i + 2]);
  const bool b2 = lane & 4;
  double v = (b2 ? a2[1] : a2[0]) + nr_dpp<NR_DPP_HALF_MIRROR>(b2 ? a2[0] : a2[1]);
  v += nr_dpp<NR_DPP_XOR2>(v);
  v += nr_dpp<NR_DPP_XOR1>(v);
  return v;
}

// Phase stamps (diagnostics only: active when P.stamps != NULL, a separate
// measurement run; no stamp executes otherwise). Thread 0 accumulates shader
// cycles per phase between the barriers that already delimit the phases.
__device__ __forceinline__ uint64_t nr_clock() { return __builtin_amdgcn_s_memtime(); }
// Compiled in only by a diagnostic build (make EXTRA=-DNR_STAMPS=1 OUT=...):
// the stamps' live timer and branches change the profile kernel's register
// allocation (its spills grew 212 -> 352 B/lane with four more stamp sites,
// and the kernel ran 30% slower), so the shipped library carries none.
// Each workgroup sums its phases in LDS and adds them to P.stamps once, at
// the end of the kernel (round 5: one global atomic per stamp from every
// workgroup contended on 16 addresses and inflated the per-step phases).
#ifdef NR_STAMPS
static __shared__ unsigned long long nr_stamp_acc[NR_N_STAMPS];
#define NR_STAMP(slot)                                                          \
  do {                                                                          \
    if (P.stamps && threadIdx.x == 0) {                                         \
      const uint64_t t_ = nr_clock();                                           \
      nr_stamp_acc[slot] += (unsigned long long)(t_ - t_mark);                  \
      t_mark = t_;                                                              \
    }                                                                           \
  } while (0)
#define NR_STAMP_INIT()                                                         \
  do {                                                                          \
    if (threadIdx.x < NR_N_STAMPS) nr_stamp_acc[threadIdx.x] = 0;               \
    __syncthreads();                                                            \
  } while (0)
#define NR_STAMP_FLUSH()                                                        \
  do {                                                                          \
    __syncthreads();                                                            \
    if (P.stamps && threadIdx.x < NR_N_STAMPS)                                  \
      atomicAdd((unsigned long long*)&P.stamps[threadIdx.x], nr_stamp_acc[threadIdx.x]); \
  } while (0)
#else
#define NR_STAMP(slot) \
  do {                 \
  } while (0)
#define NR_STAMP_INIT() \
  do {                  \
  } while (0)
#define NR_STAMP_FLUSH() \
  do {                   \
  } while (0)
#endif

// Sum of a[r] over lane bits 0..3 (the 16 columns of a tile); lanes with
// (lane & 3) == 0 end with the total of row group r = 2*b3 + b2, i.e. tile
// row (lane >> 4) + 4r.
__device__ __forceinline__ double rg_row_reduce(const double (&a)[4], int lane) {
  const bool b3 = lane & 8, b2 = lane & 4;
  const double v0 = (b3 ? a[2] : a[0]) + nr_dpp<NR_DPP_ROR8>(b3 ? a[0] : a[2]);
  const double v1 = (b3 ? a[3] : a[1]) + nr_dpp<NR_DPP_ROR8>(b3 ? a[1] : a[3]);
  double v = (b2 ? v1 : v0) + nr_dpp<NR_DPP_HALF_MIRROR>(b2 ? v0 : v1);
  v += nr_dpp<NR_DPP_XOR2>(v);
  v += nr_dpp<NR_DPP_XOR1>(v);
  return v;
}

// ---------------------------------------------------------------------------
// Summary-profile item pipeline pieces shared by every Gram storage scheme:
// LDS carve-out, node contributions from the Ritz vector, the statistics, and
// the persistent work queue.
// ---------------------------------------------------------------------------

// Doubles of the packed matvec's per-wave partial arrays, which double as the
// Ritz checks' work area (5 mmax).
__host__ __device__ __forceinline__ int64_t packed_part_doubles(int nw, int kvec, int mmax) {
  const int64_t a = (int64_t)nw * kvec, b = 5 * (int64_t)mmax;
  return a > b ? a : b;
}

// LDS carve-out common to all summary-profile bodies.
struct LzLds {
  double *red, *q, *qprev, *w, *vv, *gv, *colm;
  double *alpha, *beta, *h, *ty, *twork, *omg;
  uint32_t* idx;
  int mmax;
};

// Carves red, q, qprev, w, vv, gv, colm (kvec each), then `extra` doubles for
// the storage scheme (returned in *extra_out), then the Lanczos tridiagonal
// arrays and idx. Layout matches profile_kernel_lds.
template <int NW>
__device__ __forceinline__ LzLds carve_lds(unsigned char* smem, int kvec, int mmax, int64_t extra,
                                           double** extra_out, bool twork_in_extra = false) {
  LzLds L;
  L.red = reinterpret_cast<double*>(smem);  // 8 * NW
  L.q = L.red + 8 * NW;
  L.qprev = L.q + kvec;
  L.w = L.qprev + kvec;
  L.vv = L.w + kvec;
  L.gv = L.vv + kvec;
  L.colm = L.gv + kvec;
  *extra_out = L.colm + kvec;
  L.alpha = *extra_out + extra;  // [mmax]
  L.beta = L.alpha + mmax;       // [mmax]
  L.h = L.beta + mmax;           // [mmax]
  L.ty = L.h + mmax;             // [mmax]
  // [5 * mmax]; or the extra area (the packed matvec's partials, idle and zero
  // between matvecs: users zero it again)
  L.twork = twork_in_extra ? *extra_out : L.ty + mmax;
  L.omg = twork_in_extra ? L.ty + mmax : L.twork + 5 * mmax;  // [3 * (mmax + 1)] omega rows
  L.idx = reinterpret_cast<uint32_t*>(L.omg + 3 * (mmax + 1));  // [kvec]
  L.mmax = mmax;
  return L;
}

// Variant 6 (Lanczos dimensions beyond the LDS vectors): only the reduction
// scratch and the tridiagonal arrays in LDS; the six vectors (kvec each) and
// the index set in the slot's global scratch at `gvec` (the workgroup's
// barriers order them: one CU, one vector L1). Same roles as carve_lds with
// twork outside the partials.
template <int NW>
__device__ __forceinline__ LzLds carve_split(unsigned char* smem, double* gvec, int kvec, int mmax) {
  LzLds L;
  L.red = reinterpret_cast<double*>(smem);  // 8 * NW
  L.alpha = L.red + 8 * NW;
  L.beta = L.alpha + mmax;
  L.h = L.beta + mmax;
  L.ty = L.h + mmax;
  L.twork = L.ty + mmax;                    // [5 * mmax]
  L.omg = L.twork + 5 * mmax;               // [3 * (mmax + 1)]
  L.q = gvec;
  L.qprev = L.q + kvec;
  L.w = L.qprev + kvec;
  L.vv = L.w + kvec;
  L.gv = L.vv + kvec;
  L.colm = L.gv + kvec;
  L.idx = reinterpret_cast<uint32_t*>(L.colm + kvec);
  L.mmax = mmax;
  return L;
}

// Node contributions from the Ritz vector (u = X v / sigma):
//   NC_j = cor(x_j, u) = ((Gv)_j/sigma - S m_j ubar) / sqrt((G_jj - S m_j^2)(1 - S ubar^2)),
// oriented by sign(cor(rowMeans(X), u)) (src/netStats.cpp:242-247, 279); the
// result goes to L.w. diag(c) = G_cc; L.colm holds the column means.
template <int NW, class MV, class DG>
__device__ __forceinline__ void profile_contrib(const ProfileParams& P, int k, int m, const LzLds& L,
                                                const double* __restrict__ X, int S, double ones_g_ones,
                                                MV& mv, DG diag, bool gv_ready = false) {
  constexpr int BS = NW * 64;
  const int tid = threadIdx.x;
  const double Sd = (double)S;
  double* vv = L.vv;
  double* gv = L.gv;
  double* colm = L.colm;
  if (!gv_ready) mv(vv, gv, nullptr);  // else lanczos_ritz left G v in L.gv
  // lambda = v.Gv; ubar = mean of u = X v / sigma
  double a3[2] = {0.0, 0.0};
  for (int c = tid; c < k; c += BS) {
    a3[0] += vv[c] * gv[c];
    a3[1] += colm[c] * vv[c];
  }
  block_sums<2, NW>(a3, L.red);
  const double lambda = a3[0];
  const double sigma = sqrt(lambda);
  const double ubar = a3[1] / sigma;
  const double var_u = 1.0 - Sd * ubar * ubar;  // sum (u - ubar)^2 with |u| = 1
  // orientation: sign(cor(meanObs, u)) (src/netStats.cpp:242-247); the sign
  // of the covariance is that of sum_j cov(x_j, u); var(meanObs) * k^2 * (S-1)
  // = 1'G1 - (sum of all data)^2 / S.
  double a4[2] = {0.0, 0.0};
  for (int c = tid; c < k; c += BS) {
    a4[0] += gv[c] / sigma - Sd * colm[c] * ubar;
    a4[1] += colm[c];
  }
  block_sums<2, NW>(a4, L.red);
  const double var_mo = ones_g_ones - Sd * a4[1] * a4[1];
  const bool flip = (a4[0] < 0.0) && (var_mo > 0.0) && (var_u > 0.0);
  const double sgn = flip ? -1.0 : 1.0;
  // NC_j = cor(x_j, u) (src/netStats.cpp:279); node order = CSR order
  for (int c = tid; c < k; c += BS) {
    const double cov = gv[c] / sigma - Sd * colm[c] * ubar;
    const double var_x = diag(c) - Sd * colm[c] * colm[c];
    L.w[c] = sgn * cov / (sqrt(var_x) * sqrt(var_u));
  }
  if (P.sp_out) {
    for (int r = tid; r < S; r += BS) {
      double s = 0.0;
      for (int c = 0; c < k; ++c) s += X[(int64_t)L.idx[c] * S + r] * vv[c];
      P.sp_out[(int64_t)m * S + r] = sgn * s / sigma;
    }
  }
  nr_sync<NW>();
}

// The per-node sums of the dual contributions for one wave (S <= 112): the
// Gram's operand pattern -- lane (i16, kk) reads samples 16 I + i16 (I < 7)
// of nodes c0 + 4 kk + q, 28 loads per 16-node step, the next step's in
// flight -- then x_c . u, the column sum and the sum of squares per node,
// reduced over the 16 sample lanes (rg_row_reduce leaves node c0 + 4 kk + r,
// r = 2 b3 + b2, in the lanes with lane & 3 == 0). Into L.gv, L.colm (mean)
// and L.q.
__device__ __forceinline__ void contrib_dual_sums_wave(const LzLds& L, const double* __restrict__ X, int S, int k,
                                                       const double* u) {
  constexpr int NB = 7;
  const int lane = threadIdx.x & 63;
  const int i16 = lane & 15, kk = lane >> 4;
  double ul[NB];
#pragma unroll
  for (int I = 0; I < NB; ++I) ul[I] = 16 * I + i16 < S ? u[16 * I + i16] : 0.0;
  // range-checked buffer loads (out of range reads 0): no branch, so only
  // this step's loads are waited for (the engine keeps X under 2 GB here)
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, 0x7fffffff, 0x00020000);
  auto ld = [&](int c0, double (&v)[NB][4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + 4 * kk + q;
      const int base = c < k ? (int)L.idx[c] * S : 0;
#pragma unroll
      for (int I = 0; I < NB; ++I) {
        const int s = 16 * I + i16;
        const int vo = c < k && s < S ? (base + s) * 8 : (int)0x80000000;
        v[I][q] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc, vo, 0, 0));
      }
    }
  };
  const int rg = ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
  double cur[NB][4], nxt[NB][4];
  ld(0, cur);
  for (int c0 = 0; c0 < k; c0 += 16) {
    if (c0 + 16 < k) ld(c0 + 16, nxt);
    double a[4], b[4], q2[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a[q] = 0.0;
      b[q] = 0.0;
      q2[q] = 0.0;
#pragma unroll
      for (int I = 0; I < NB; ++I) {
        const double x = cur[I][q];
        a[q] = fma(x, ul[I], a[q]);
        b[q] += x;
        q2[q] = fma(x, x, q2[q]);
      }
    }
    const double sa = rg_row_reduce(a, lane), sb = rg_row_reduce(b, lane), sq = rg_row_reduce(q2, lane);
    const int c = c0 + 4 * kk + rg;
    if ((lane & 3) == 0 && c < k) {
      L.gv[c] = sa;
      L.colm[c] = sb / (double)S;
      L.q[c] = sq;
    }
#pragma unroll
    for (int I = 0; I < NB; ++I)
#pragma unroll
      for (int q = 0; q < 4; ++q) cur[I][q] = nxt[I][q];
  }
}

// Node contributions when Lanczos ran on the dual Gram (k > S): L.vv holds u
// itself (unit norm, S entries). One pass over the module's data gives, per
// node, x_c . u, the column sum and the sum of squares (one wave per node,
// lanes over samples); then NC_c = cor(x_c, u) and the orientation exactly as
// profile_contrib (src/netStats.cpp:242-247, 279). q, gv, colm are reused as
// per-node scratch (sum of squares, x_c . u, column mean).
template <int NW>
__device__ __forceinline__ void profile_contrib_dual(const ProfileParams& P, int k, int m, const LzLds& L,
                                                     const double* __restrict__ X, int S, double ones_g_ones) {
  constexpr int BS = NW * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double Sd = (double)S;
  const double* u = L.vv;
  // 16 lanes per node, 4 nodes per wave instruction, two node groups in
  // flight: the column loads of 8 nodes are issued before any is reduced (the
  // pass was one dependent global round trip per node: 14% of a C2 item)
  const int g16 = lane >> 4, l16 = lane & 15;
  if constexpr (NW == 1) {
    contrib_dual_sums_wave(L, X, S, k, u);
  } else
  for (int c0 = 8 * wave; c0 < k; c0 += 8 * NW) {
    double a[2] = {0.0, 0.0}, b[2] = {0.0, 0.0}, q[2] = {0.0, 0.0};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = c0 + 4 * h + g16;
      const double* col = X + (int64_t)L.idx[c < k ? c : k - 1] * S;
      for (int s = l16; s < S; s += 16) {
        const double x = c < k ? col[s] : 0.0;
        a[h] = fma(x, u[s], a[h]);
        b[h] += x;
        q[h] = fma(x, x, q[h]);
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      a[h] = nr_row_sum16(a[h]);
      b[h] = nr_row_sum16(b[h]);
      q[h] = nr_row_sum16(q[h]);
      const int c = c0 + 4 * h + g16;
      if (l16 == 0 && c < k) {
        L.gv[c] = a[h];
        L.colm[c] = b[h] / Sd;
        L.q[c] = q[h];
      }
    }
  }
  double a3[1] = {0.0};
  for (int s = tid; s < S; s += BS) a3[0] += u[s];
  block_sums<1, NW>(a3, L.red);  // its barriers also publish the per-node sums
  const double ubar = a3[0] / Sd;
  const double var_u = 1.0 - Sd * ubar * ubar;
  double a4[2] = {0.0, 0.0};
  for (int c = tid; c < k; c += BS) {
    a4[0] += L.gv[c] - Sd * L.colm[c] * ubar;
    a4[1] += L.colm[c];
  }
  block_sums<2, NW>(a4, L.red);
  const double var_mo = ones_g_ones - Sd * a4[1] * a4[1];
  const bool flip = (a4[0] < 0.0) && (var_mo > 0.0) && (var_u > 0.0);
  const double sgn = flip ? -1.0 : 1.0;
  for (int c = tid; c < k; c += BS) {
    const double cov = L.gv[c] - Sd * L.colm[c] * ubar;
    const double var_x = L.q[c] - Sd * L.colm[c] * L.colm[c];
    L.w[c] = sgn * cov / (sqrt(var_x) * sqrt(var_u));
  }
  if (P.sp_out)
    for (int s = tid; s < S; s += BS) P.sp_out[(int64_t)m * S + s] = sgn * u[s];
  nr_sync<NW>();
}

// svd_econ refuses non-finite input -> all-NaN summary (src/netStats.cpp:229-235).
template <int NW>
__device__ __forceinline__ void profile_nonfinite(const ProfileParams& P, int k, int m, int S, const LzLds& L) {
  constexpr int BS = NW * 64;
  for (int c = threadIdx.x; c < k; c += BS) L.w[c] = nr_nan();
  if (P.sp_out)
    for (int r = threadIdx.x; r < S; r += BS) P.sp_out[(int64_t)m * S + r] = nr_nan();
  nr_sync<NW>();
}

// ModuleCoherence (src/netStats.cpp:293-305), Correlation / SignAwareMean
// against the discovery contribution (src/permutations.cpp:99,101); node
// contributions in L.w.
template <int NW>
__device__ __forceinline__ void profile_stats(const ProfileParams& P, int k, int m, int64_t off,
                                              int64_t p_local, const LzLds& L) {
  constexpr int BS = NW * 64;
  const int tid = threadIdx.x;
  const double* w = L.w;
  double b1[5] = {0, 0, 0, 0, 0};  // nfinite, sum nc^2, ncc, sx, sy
  for (int c = tid; c < k; c += BS) {
    const double y = w[c];
    if (isfinite(y)) { b1[0] += 1.0; b1[1] += y * y; }
    if (P.disc_nc) {
      const double xv = P.disc_nc[off + c];
      if (isfinite(xv) && isfinite(y)) { b1[2] += 1.0; b1[3] += xv; b1[4] += y; }
    }
    if (P.nc_out) P.nc_out[off + c] = y;
  }
  block_sums<5, NW>(b1, L.red);
  const double stat_coh = b1[0] >= 1.0 ? b1[1] / b1[0] : nr_nan();
  double stat_cc = nr_nan(), stat_ac = nr_nan();
  if (P.disc_nc && P.out) {
    const double mx = b1[3] / b1[2], my = b1[4] / b1[2];
    double b2[4] = {0, 0, 0, 0};
    for (int c = tid; c < k; c += BS) {
      const double y = w[c], xv = P.disc_nc[off + c];
      if (isfinite(xv) && isfinite(y)) {
        const double dx = xv - mx, dy = y - my;
        b2[0] += dx * dx;
        b2[1] += dy * dy;
        b2[2] += dx * dy;
        b2[3] += (xv > 0.0 ? y : (xv < 0.0 ? -y : 0.0));
      }
    }
    block_sums<4, NW>(b2, L.red);
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
  nr_sync<NW>();
}

// Next item from the persistent queue: (module m, local permutation, CSR
// offset, k) and its index set in L.idx. Returns false when drained.
template <int NW>
__device__ __forceinline__ bool next_item(const ProfileParams& P, const LzLds& L, int* flags, int& m,
                                          int64_t& p_local, int64_t& off, int& k, int kvec = 1 << 30,
                                          uint32_t* gidx = nullptr, uint32_t** idx_used = nullptr) {
  constexpr int BS = NW * 64;
  const int tid = threadIdx.x;
  if (tid == 0) flags[0] = atomicAdd(P.queue, 1);
  nr_sync<NW>();
  const int item = flags[0];
  nr_sync<NW>();
  if (item >= P.n_items) return false;
  int64_t mslot;
  const int T = P.order_tail;
  const int64_t n_ms = P.n_items / P.n_perm;
  const int64_t head = T > 0 && T < P.n_perm ? (int64_t)(P.n_perm - T) * n_ms : 0;
  if (item < head) {  // permutation-major: every module size in flight at once
    p_local = item / n_ms;
    mslot = item - p_local * n_ms;
  } else {            // module-major, large modules first (the tail balances the slots)
    const int64_t t = item - head;
    const int64_t np = head > 0 ? T : P.n_perm;
    mslot = t / np;
    p_local = (P.n_perm - np) + (t - mslot * np);
  }
  m = P.mod_order[mslot];
  off = P.node_off[m];
  k = (int)(P.node_off[m + 1] - off);
  nr_prp_key key;
  if (P.src.mode == NR_IDX_PRP) key = nr_prp_make_key(P.src.seed, (uint64_t)(P.src.perm_base + p_local), P.src.n_null);
  // modules longer than the LDS vectors: index set in the slot's scratch
  uint32_t* dst = (k <= kvec || !gidx) ? L.idx : gidx;
  if (idx_used) *idx_used = dst;
  for (int c = tid; c < k; c += BS) dst[c] = node_index(P.src, key, p_local, off + c);
  if (tid == 0) flags[1] = 0;
  nr_sync<NW>();
  return true;
}
// Weighted-degree fixed-point helpers (the cancellation model of kernels.hip,
// shared with the column sweep, sweep.hip).
constexpr int WD_FX_BITS = 16;        // fixed-point sub-units per grid unit
constexpr int WD_NO_GRID = -100000;   // exponent sentinel: no cancellation model

// Exponent of the grid unit g = 2^e of the accumulator holding d: the ulp of
// d's binade, or of the next binade when d sits within 2^-20 below it (the
// first addition then carries the accumulator across).
__device__ __forceinline__ int wd_grid_exp(double d) {
  if (!(d >= 2.2250738585072014e-308) || !isfinite(d)) return WD_NO_GRID;
  const int e = ilogb(d);
  const double top = ldexp(1.0, e + 1);
  return (top - d <= ldexp(d, -20) ? e + 1 : e) - 52;
}

__device__ __forceinline__ unsigned long long wd_fx(double a, int ge, int extra) {
  double v = ldexp(a, extra - ge);
  v = v < 2.305843009213694e18 ? v : 2.305843009213694e18;  // 2^61: overflow is caught by the range check
  return (unsigned long long)llrint(v);
}

}  // namespace nr
