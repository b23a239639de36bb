// Probe: CU-resident Lanczos for the packed class (k <= 320), one 8-wave
// workgroup per CU, the item's packed Gram in registers (EK_R units per wave)
// + LDS (EK_L units per wave) + global (the rest). Three barriers per step;
// the reorthogonalisation decision and the convergence checks are computed
// redundantly by every wave (no broadcast barrier). Standalone: reads packed
// Grams (kernels.hip pk_at layout, side kc = k + 1) and returns theta, v.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared eig_probe.hip -o eig_probe.so
#include "../../netrep_amd/csrc/device_common.h"

namespace nr {
#ifndef EK_R
#define EK_R 4
#endif
#ifndef EK_L
#define EK_L 2
#endif
// diagnostic modes: 1 = matvec + barriers only (35 fixed steps, no control),
// 2 = everything but the matvec
#ifndef EK_MODE
#define EK_MODE 0
#endif
constexpr int EW = 8;
constexpr int EBS = EW * 64;
constexpr int ER = EK_R, EL = EK_L;
constexpr int EKV = 328;  // Lanczos dimension <= 320
constexpr int EMM = 128;  // Lanczos step cap

struct EkParams {
  const double* grams;
  const int64_t* gram_off;
  const int* kk;
  int n_items, n_real;
  int* queue;
  double* basis;  // per workgroup EKV * EMM
  double* theta_out;
  double* v_out;  // n_real x EKV
  int* steps_out;
  unsigned long long* stamps;
};

__host__ __device__ __forceinline__ int ek_units_in_group(int kc, int g) { return (kc - 16 * g + 63) >> 6; }
// the packed layout's addressing (kernels.hip pk_base / pk_at)
__host__ __device__ __forceinline__ int64_t pk_base(int g, int P) { return 16 * (int64_t)g * P - 128 * (int64_t)g * (g - 1); }
__device__ __forceinline__ int64_t pk_at(int r, int c, int kc) {
  const int g = c >> 4;
  const int rr = r - 16 * g;
  const int j = rr >> 6;
  const int h = min(64, kc - 16 * g - 64 * j);
  return pk_base(g, kc) + 1024 * (int64_t)j + (int64_t)(c & 15) * h + (rr & 63);
}

// Phase stamps (diagnostic runs only: P.stamps != NULL): thread 0 adds the
// s_memtime delta of each phase into LDS; flushed once when the workgroup
// exits (a global atomic per stamp would enter every later vmcnt wait).
#define EK_STAMP(slot)                                    \
  do {                                                    \
    if (P.stamps && threadIdx.x == 0) {                   \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
      s_st[slot] += t_ - t_mark;                          \
      t_mark = t_;                                        \
    }                                                     \
  } while (0)

// x_c of the unit's 16 columns, lane c of each 16-lane row holding x[c0 + c]:
// DPP row_newbcast gives every lane the value of lane T of its row.
template <int T>
__device__ __forceinline__ double ek_bcast16(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x150 + T, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x150 + T, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int T = 0>
__device__ __forceinline__ double ek_row_dot_rec(const double (&gb)[16], double xl, double acc) {
  if constexpr (T == 16) {
    return acc;
  } else {
    return ek_row_dot_rec<T + 1>(gb, xl, fma(gb[T], ek_bcast16<T>(xl), acc));
  }
}
__device__ __forceinline__ double ek_row_dot(const double (&gb)[16], double xl) { return ek_row_dot_rec<0>(gb, xl, 0.0); }

// Unit (cg, j) of the packed Gram at s (stride h), the lane's row, diagonal halved.
__device__ __forceinline__ void ek_load_unit(double (&gb)[16], const double* s, int h, int j, int lane, bool on) {
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const double g = (on && lane < h) ? s[t * h + lane] : 0.0;
    gb[t] = (j == 0 && lane == t) ? 0.5 * g : g;
  }
}

// One unit of the packed Gram (64 rows x 16 columns of column group cg, row
// chunk j; gb = the lane's row, 16 columns), accumulated into this wave's
// partial array: the lower part lane-locally (row r), the mirrored upper part
// into up[16] (reduced over lanes when the wave leaves the group).
struct EkMv {
  int kc, n, lane;
  int cg, j, nj;
  double xl;
  double up[16];
  const double* x;
  double* part;
  template <bool SQ>
  __device__ __forceinline__ void load_xl() {
    const int c = 16 * cg + (lane & 15);
    xl = SQ ? 0.0 : (c < n ? x[c] : 0.0);
  }
  // The stored diagonal is halved (ek_load_unit), so the lower and the
  // mirrored part each count half of G_cc x_c: no per-element mask.
  template <bool SQ>
  __device__ __forceinline__ void proc(const double (&gb)[16], bool last) {
    const int c0 = 16 * cg;
    const int r = c0 + 64 * j + lane;
    const double xr = SQ ? (r < n ? 1.0 : 0.0) : (r < n ? x[r] : 0.0);
    double acc = 0.0;
    if (SQ) {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const double g2 = gb[t] * gb[t];
        acc += c0 + t < n ? g2 : 0.0;
        up[t] = fma(g2, xr, up[t]);
      }
    } else {
      acc = ek_row_dot(gb, xl);
#pragma unroll
      for (int t = 0; t < 16; ++t) up[t] = fma(gb[t], xr, up[t]);
    }
    if (r < n) part[r] += acc;
    ++j;
    if (j == nj || last) {
      const double v = nr_transpose_reduce16(up, lane);
      if ((lane & 3) == 0) {
        const int c = c0 + ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
        if (c < n) part[c] += v;
      }
#pragma unroll
      for (int t = 0; t < 16; ++t) up[t] = 0.0;
      ++cg;
      j = 0;
      nj = ek_units_in_group(kc, cg);
      load_xl<SQ>();
    }
  }
};

template <bool SQ>
__device__ __forceinline__ void ek_matvec(const double (&greg)[ER][16], const double* lg, const double* G, int kc,
                                          int n, int nu, int cg0, int j0, const double* x, double* part) {
  EkMv m;
  m.kc = kc;
  m.n = n;
  m.lane = threadIdx.x & 63;
  m.cg = cg0;
  m.j = j0;
  m.nj = ek_units_in_group(kc, cg0);
  m.x = x;
  m.part = part;
#pragma unroll
  for (int t = 0; t < 16; ++t) m.up[t] = 0.0;
  m.load_xl<SQ>();
#pragma unroll
  for (int p = 0; p < ER; ++p)
    if (p < nu) m.proc<SQ>(greg[p], p == nu - 1);
  for (int p = ER; p < nu; ++p) {
    double gb[16];
    const int h = min(64, kc - 16 * m.cg - 64 * m.j);
    if (p < ER + EL) {
      const double* s = lg + (p - ER) * 1024;
#pragma unroll
      for (int t = 0; t < 16; ++t) gb[t] = m.lane < h ? s[t * h + m.lane] : 0.0;
    } else {
      ek_load_unit(gb, G + pk_base(m.cg, kc) + 1024 * (int64_t)m.j, h, m.j, m.lane, true);
    }
    m.proc<SQ>(gb, p == nu - 1);
  }
}

__device__ __forceinline__ double ek_wave_max(double v) { return nr_wave_max(v); }

__global__ void __launch_bounds__(EBS, 1) ek_kernel(EkParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* part = reinterpret_cast<double*>(smem);  // EW x EKV
  double* wbuf = part + EW * EKV;                  // EKV
  double* red = wbuf + EKV;                        // 64
  double* alpha = red + 64;                        // EMM
  double* beta = alpha + EMM;                      // EMM
  double* omg = beta + EMM;                        // 3 x (EMM + 1)
  double* om_num = omg + 3 * (EMM + 1);            // EMM + 1
  double* ty = om_num + (EMM + 1);                 // EMM
  double* lgram = ty + EMM;                        // EW x EL x 1024
  __shared__ int s_item;
  __shared__ unsigned long long s_st[16];
  if (threadIdx.x < 16) s_st[threadIdx.x] = 0;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* mypart = part + wave * EKV;
  double* lg = lgram + (int64_t)wave * EL * 1024;
  double* Q = P.basis + (int64_t)blockIdx.x * EKV * EMM;
  uint64_t t_mark = P.stamps && tid == 0 ? __builtin_amdgcn_s_memtime() : 0;
  for (int i = tid; i < EW * EKV; i += EBS) part[i] = 0.0;
  double greg[ER][16];

  for (;;) {
    if (tid == 0) s_item = atomicAdd(P.queue, 1);
    __syncthreads();
    const int item = s_item;
    __syncthreads();
    if (item >= P.n_items) {
      if (P.stamps && tid < 16) atomicAdd(&P.stamps[tid], s_st[tid]);
      break;
    }
    const int ri = item % P.n_real;
    const int n = P.kk[ri];
    const int kc = n + 1;
    const double* G = P.grams + P.gram_off[ri];
    // units over the matvec's column groups, contiguous per wave
    const int ncg = (n + 15) / 16;
    int U = 0;
    for (int g = 0; g < ncg; ++g) U += ek_units_in_group(kc, g);
    const int u0 = U * wave / EW, u1 = U * (wave + 1) / EW;
    const int nu = u1 - u0;
    int cg0 = 0, j0 = 0;
    {
      int first = 0;
      while (first + ek_units_in_group(kc, cg0) <= u0) {
        first += ek_units_in_group(kc, cg0);
        ++cg0;
      }
      j0 = u0 - first;
    }
    // register and LDS tiers
    {
      int cg = cg0, j = j0;
#pragma unroll
      for (int p = 0; p < ER; ++p) {
        const int h = min(64, kc - 16 * cg - 64 * j);
        const double* s = G + pk_base(cg, kc) + 1024 * (int64_t)j;
        ek_load_unit(greg[p], s, h, j, lane, p < nu);
        if (++j == ek_units_in_group(kc, cg)) {
          ++cg;
          j = 0;
        }
      }
      for (int p = ER; p < min(nu, ER + EL); ++p) {
        const int h = min(64, kc - 16 * cg - 64 * j);
        const double* s = G + pk_base(cg, kc) + 1024 * (int64_t)j;
        double* d = lg + (p - ER) * 1024;
        double gb[16];
        ek_load_unit(gb, s, h, j, lane, true);
        for (int t = 0; t < 16; ++t)
          if (lane < h) d[t * h + lane] = gb[t];
        if (++j == ek_units_in_group(kc, cg)) {
          ++cg;
          j = 0;
        }
      }
    }
    EK_STAMP(0);  // load
    // start vector: G e_c*, c* the column of largest norm (fp64 squared pass)
    ek_matvec<true>(greg, lg, G, kc, n, nu, cg0, j0, nullptr, mypart);
    __syncthreads();
    double cn = -1.0;
    if (tid < n) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < EW; ++w) {
        s += part[w * EKV + tid];
        part[w * EKV + tid] = 0.0;
      }
      cn = s;
    }
    double best = cn;
    int bi = tid < n ? tid : 0x7fffffff;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const double ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) {
        best = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      red[wave] = best;
      red[EW + wave] = (double)bi;
    }
    __syncthreads();
    best = red[0];
    bi = (int)red[EW];
#pragma unroll
    for (int w = 1; w < EW; ++w) {
      const double ov = red[w];
      const int oi = (int)red[EW + w];
      if (ov > best || (ov == best && oi < bi)) {
        best = ov;
        bi = oi;
      }
    }
    double qt = 0.0, qpt = 0.0, wt = 0.0, zt = 0.0;
    if (tid < n) qt = G[pk_at(tid > bi ? tid : bi, tid > bi ? bi : tid, kc)];
    {
      double s = wave_sum(qt * qt);
      __syncthreads();
      if (lane == 0) red[wave] = s;
      __syncthreads();
      double tot = 0.0;
#pragma unroll
      for (int w = 0; w < EW; ++w) tot += red[w];
      qt *= 1.0 / sqrt(tot);
    }
    if (tid < n) {
      wbuf[tid] = qt;
      Q[tid] = qt;
    }
    if (tid == 0) {
      omg[0] = 1.0;
    }
    __syncthreads();
    EK_STAMP(1);  // start column
    const int mcap = n < EMM ? n : EMM;
    double ib = 1.0, beta_prev = 0.0, anorm = 0.0;
    int next_check = mcap < 16 ? mcap : 16;
    int prev_j = 0;
    double prev_r = 0.0, hint_theta = 0.0, hint_r = 0.0, theta = 0.0;
    bool force_next = false;
    int nsteps = 0;
    const double sqrt_eps = 1.4901161193847656e-08;
    const double eps = 2.220446049250313e-16;
    const double eps_sqrtn = eps * sqrt((double)n);
    for (int j = 0; j < mcap; ++j) {
      // M: matvec of x = wbuf (unnormalised; y scaled by ib below)
      if (EK_MODE != 2) ek_matvec<false>(greg, lg, G, kc, n, nu, cg0, j0, wbuf, mypart);
      EK_STAMP(2);
      __syncthreads();  // B1
      EK_STAMP(3);
      // C: row threads combine
      double a = 0.0;
      if (tid < n) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < EW; ++w) {
          s += part[w * EKV + tid];
          part[w * EKV + tid] = 0.0;
        }
        if (EK_MODE == 2) s = wbuf[tid] * (1.0 + 0.37 * tid / n);  // a diagonal stand-in operator
        const double y = s * ib;
        zt = y - beta_prev * qpt;
        a = qt * zt;
      }
      a = wave_sum(a);
      if (lane == 0) red[wave] = a;
      __syncthreads();  // B2
      EK_STAMP(4);
      double alpha_j = 0.0;
#pragma unroll
      for (int w = 0; w < EW; ++w) alpha_j += red[w];
      double b = 0.0;
      if (tid < n) {
        wt = zt - alpha_j * qt;
        b = wt * wt;
        wbuf[tid] = wt;
      }
      b = wave_sum(b);
      if (lane == 0) red[16 + wave] = b;
      if (tid == 0) alpha[j] = alpha_j;
      double* om_cur = omg + (j % 3) * (EMM + 1);
      double* om_prev = omg + ((j + 2) % 3) * (EMM + 1);
      double* om_next = omg + ((j + 1) % 3) * (EMM + 1);
      if (wave == 0) {  // omega numerators (Simon's recurrence, omega_update) for i < j
        for (int i = lane; i < j; i += 64) {
          double t = beta[i] * om_cur[i + 1] + (alpha[i] - alpha_j) * om_cur[i] - (j > 0 ? beta[j - 1] * om_prev[i] : 0.0);
          if (i > 0) t += beta[i - 1] * om_cur[i - 1];
          om_num[i] = t;
        }
      }
      __syncthreads();  // B3
      EK_STAMP(5);
      double nb = 0.0;
#pragma unroll
      for (int w = 0; w < EW; ++w) nb += red[16 + w];
      double beta_j = sqrt(nb);
      double ibj = 1.0 / beta_j;
      anorm = fmax(anorm, fabs(alpha_j) + beta_j + beta_prev);
      bool reorth;
      {
        const double psi = eps * anorm * ibj;
        double mx = 0.0;
        for (int i = lane; i < j; i += 64) {
          double t = om_num[i] * ibj;
          t += t >= 0.0 ? psi : -psi;
          if (wave == 0) om_next[i] = t;
          mx = fmax(mx, fabs(t));
        }
        const double omj = eps_sqrtn * anorm * ibj;
        if (lane == 0) {
          if (wave == 0) {
            om_next[j] = omj;
            om_next[j + 1] = 1.0;
          }
          mx = fmax(mx, fabs(omj));
        }
        mx = ek_wave_max(mx);
        reorth = EK_MODE == 1 ? false : (force_next || mx > sqrt_eps);
      }
      EK_STAMP(6);
      if (reorth) {
        // CGS of w against q_0..q_j (basis in global scratch): h = Q^T w by
        // 16-vector transpose-reduces per 64-row block (wave = row block),
        // per-wave partials in part (idle), h in ty; w -= Q h; the new |w|^2
        const int ng = (j + 16) >> 4;
        for (int g = 0; g < ng; ++g) {
          double u16[16];
#pragma unroll
          for (int s2 = 0; s2 < 16; ++s2) {
            const int i = 16 * g + s2;
            u16[s2] = (i <= j && tid < n) ? Q[(int64_t)i * n + tid] * wt : 0.0;
          }
          const double v = nr_transpose_reduce16(u16, lane);
          if ((lane & 3) == 0) {
            const int i = 16 * g + ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
            if (i <= j) part[wave * EKV + i] = v;
          }
        }
        __syncthreads();
        if (tid <= j) {
          double h = 0.0;
#pragma unroll
          for (int w = 0; w < EW; ++w) {
            h += part[w * EKV + tid];
            part[w * EKV + tid] = 0.0;
          }
          ty[tid] = h;
        }
        __syncthreads();
        double bb = 0.0;
        if (tid < n) {
          double acc = 0.0;
          for (int i = 0; i <= j; ++i) acc = fma(ty[i], Q[(int64_t)i * n + tid], acc);
          wt -= acc;
          bb = wt * wt;
          wbuf[tid] = wt;
        }
        alpha_j += ty[j];
        bb = wave_sum(bb);
        if (lane == 0) red[32 + wave] = bb;
        if (tid == 0) alpha[j] = alpha_j;
        if (wave == 0)
          for (int i = lane; i <= j; i += 64) om_next[i] = eps;
        __syncthreads();
        nb = 0.0;
#pragma unroll
        for (int w = 0; w < EW; ++w) nb += red[32 + w];
        beta_j = sqrt(nb);
        ibj = 1.0 / beta_j;
        force_next = !force_next;
        EK_STAMP(10);
      }
      if (tid == 0) beta[j] = beta_j;
      nsteps = j + 1;
      ib = ibj;
      if (tid < n) {
        qpt = qt;
        qt = wt * ib;
        if (j + 1 < mcap) Q[(int64_t)(j + 1) * n + tid] = qt;
      }
      beta_prev = beta_j;
      EK_STAMP(11);
      if (EK_MODE == 1) {
        if (j + 1 == 35 || j + 1 == mcap) break;
        continue;
      }
      const bool last = j + 1 == mcap;
      if (j + 1 == next_check || last || !(beta_j > 1e-300)) {
        // every wave: the same Sturm multisection -> the same decision
        // (beta[0..j) were written before this step's barriers; beta_j is passed)
        theta = tri_top_eigenvalue(alpha, beta, j + 1, lane, hint_theta, hint_r);
        double resid;
        {  // backward recurrence (tri_top_resid) with reciprocals on the fly
          double y1 = 1.0, y2 = 0.0, ss = 1.0, bjs = beta_j;
          for (int i = j; i > 0; --i) {
            const double y0 = fma(theta - alpha[i], y1, -(i < j ? beta[i] : 0.0) * y2) * nr_rcp(beta[i - 1]);
            ss = fma(y0, y0, ss);
            y2 = y1;
            y1 = y0;
            if (ss > 1e200) {
              y1 *= 1e-100;
              y2 *= 1e-100;
              ss *= 1e-200;
              bjs *= 1e-100;
            }
          }
          resid = bjs / sqrt(ss);
        }
        hint_theta = theta;
        hint_r = resid;
        const double tol = 5e-15 * fabs(theta);
        const bool done = EK_MODE == 2 ? (j + 1 >= 35 || last) : (resid <= tol || last || !(beta_j > 1e-300 * fabs(theta)));
        int step = 8;
        if (prev_j > 0 && resid < prev_r && resid > 0.0) {
          const double rate = log(resid / prev_r) / (double)(j + 1 - prev_j);
          const double need = ceil(log(tol / resid) / rate);
          step = need < 1.0 ? 1 : (need > 8.0 ? 8 : (int)need);
        }
        prev_j = j + 1;
        prev_r = resid;
        next_check = min(j + 1 + step, mcap);
        EK_STAMP(7);
        if (done) break;
      }
    }
    // Ritz coefficients (one lane), Ritz vector v = Q y, G v from the Lanczos relation
    if (tid == 0) tri_eigenvector<8>(alpha, beta, nsteps, theta, ty, part);
    __syncthreads();
    EK_STAMP(8);
    double vt = 0.0;
    if (tid < n)
      for (int i = 0; i < nsteps; ++i) vt += ty[i] * Q[(int64_t)i * n + tid];
    {
      double s = wave_sum(vt * vt);
      if (lane == 0) red[wave] = s;
      __syncthreads();
      double tot = 0.0;
#pragma unroll
      for (int w = 0; w < EW; ++w) tot += red[w];
      vt *= 1.0 / sqrt(tot);
    }
    if (item < P.n_real) {
      if (tid < n) P.v_out[(int64_t)item * EKV + tid] = vt;
      if (tid == 0) {
        P.theta_out[item] = theta;
        P.steps_out[item] = nsteps;
      }
    }
    for (int i = tid; i < 5 * EMM; i += EBS) part[i] = 0.0;  // tri_eigenvector's work area
    __syncthreads();
    EK_STAMP(9);
  }
}

}  // namespace nr

extern "C" size_t ek_lds_bytes() {
  using namespace nr;
  return sizeof(double) * ((size_t)EW * EKV + EKV + 64 + EMM * 2 + 3 * (EMM + 1) + (EMM + 1) + EMM +
                           (size_t)EW * EL * 1024);
}

extern "C" int ek_run(const double* h_grams, int64_t n_gram_doubles, const int64_t* h_off, const int* h_k,
                      int n_real, int n_items, int reps, double* h_theta, double* h_v, int* h_steps,
                      double* ms_out, unsigned long long* h_stamps) {
  using namespace nr;
  double *d_g, *d_theta, *d_v, *d_basis;
  int64_t* d_off;
  int *d_k, *d_q, *d_steps;
  unsigned long long* d_st = nullptr;
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = ncu;
  if (hipMalloc(&d_g, n_gram_doubles * 8) != hipSuccess) return 1;
  hipMalloc(&d_off, n_real * 8);
  hipMalloc(&d_k, n_real * 4);
  hipMalloc(&d_theta, n_real * 8);
  hipMalloc(&d_v, (size_t)n_real * EKV * 8);
  hipMalloc(&d_steps, n_real * 4);
  hipMalloc(&d_q, 4);
  hipMalloc(&d_basis, (size_t)grid * EKV * EMM * 8);
  if (h_stamps) {
    hipMalloc(&d_st, 16 * 8);
    hipMemset(d_st, 0, 16 * 8);
  }
  hipMemcpy(d_g, h_grams, n_gram_doubles * 8, hipMemcpyHostToDevice);
  hipMemcpy(d_off, h_off, n_real * 8, hipMemcpyHostToDevice);
  hipMemcpy(d_k, h_k, n_real * 4, hipMemcpyHostToDevice);
  EkParams P{d_g, d_off, d_k, n_items, n_real, d_q, d_basis, d_theta, d_v, d_steps, d_st};
  const size_t lds = ek_lds_bytes();
  if (hipFuncSetAttribute((const void*)ek_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return 2;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float total = 0.f;
  for (int r = 0; r < reps + 1; ++r) {
    hipMemset(d_q, 0, 4);
    if (d_st && r == reps) hipMemset(d_st, 0, 16 * 8);
    EkParams Pr = P;
    if (r < reps) Pr.stamps = nullptr;
    hipEventRecord(e0);
    hipLaunchKernelGGL(ek_kernel, dim3(grid), dim3(EBS), lds, 0, Pr);
    hipEventRecord(e1);
    if (hipEventSynchronize(e1) != hipSuccess) return 3;
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    if (r > 0 && r < reps) total += ms;  // r = 0 warm-up, r = reps stamped
    if (reps == 1 && r == 0) total = ms;
  }
  if (hipGetLastError() != hipSuccess) return 4;
  *ms_out = reps > 1 ? total / (reps - 1) : total;
  hipMemcpy(h_theta, d_theta, n_real * 8, hipMemcpyDeviceToHost);
  hipMemcpy(h_v, d_v, (size_t)n_real * EKV * 8, hipMemcpyDeviceToHost);
  hipMemcpy(h_steps, d_steps, n_real * 4, hipMemcpyDeviceToHost);
  if (d_st) hipMemcpy(h_stamps, d_st, 16 * 8, hipMemcpyDeviceToHost);
  hipFree(d_g);
  hipFree(d_off);
  hipFree(d_k);
  hipFree(d_theta);
  hipFree(d_v);
  hipFree(d_steps);
  hipFree(d_q);
  hipFree(d_basis);
  if (d_st) hipFree(d_st);
  return 0;
}
