// Summary-profile kernel with the Gram resident in registers, one 4-wave
// workgroup per CU (one wave per SIMD, up to 512 VGPRs each).
//
// SummaryProfile + NodeContribution + ModuleCoherence (src/netStats.cpp:
// 217-305) of one (permutation, module) item with k <= 255 nodes:
//
//  1. Gram G = [X 1]^T [X 1] of the module's S x k data block plus a virtual
//     all-ones column (its row k holds the column sums) on
//     v_mfma_f64_16x16x4_f64. G is cut into 16 x 16 tiles over the upper
//     triangle (T = ceil((k+1)/16) a side, row-major tile ids); wave w owns
//     the contiguous id range [w nt/4, (w+1) nt/4) -- at most 34 tiles -- and
//     KEEPS the accumulators in registers: G never leaves the CU.
//     The data rows stream through LDS in groups of D 8-row slabs (D chosen
//     so a group is at most 1,280 16-byte pieces: one slab for the largest
//     modules, ten for k = 30); each thread holds its pieces of the next group
//     in registers while the MFMAs consume the current one.
//  2. Lanczos on G for the top eigenpair, two workgroup barriers per step:
//     the matvec runs on the unnormalised vector left by the previous step and
//     scales its result (no barrier to publish the normalised vector), and
//     alpha = x^T G x comes out of the matvec's own tile sums. The scalar work
//     (partial-reorthogonalisation omega recurrence, Sturm-multisection Ritz
//     checks) is computed redundantly and identically by every wave instead
//     of being broadcast. The Lanczos basis lives in LDS (global scratch
//     beyond what fits).
//  3. Node contributions, coherence and the statistics (device_common.h).
//
// Opt-in (NETREP_PROFILE_VARIANT=rg4; engine.hip launch_profiles): correct and
// deterministic, but with one wave per SIMD every LDS / DPP / barrier latency
// is exposed -- about 11 cycles per issued instruction -- and it measured
// 1.45x slower than the packed scratch-Gram kernel (24.4 vs 16.7 ms per 256
// permutations on C3-shaped modules of 30-255 nodes, profiles/r02/
// profile_variants.txt), although it never re-reads the Gram from memory.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "prp.h"
#include "kernels.h"
#include "device_common.h"

namespace nr {

constexpr int R4_NW = 4;                                 // waves (one per SIMD)
constexpr int R4_BS = R4_NW * 64;                        // 256 threads
constexpr int R4_TMAX = 16;                              // tiles a side: k + 1 <= 256
constexpr int R4_KP = 16 * R4_TMAX;                      // 256
constexpr int R4_NTMAX = R4_TMAX * (R4_TMAX + 1) / 2;    // 136 tiles
// Register tiles per wave: 26 x 8 accumulator registers fit the AGPR file
// with no scratch (28 spill). The tiles are accumulated in the AGPR form of
// the MFMA: the VGPR form (-mllvm -amdgpu-mfma-vgpr-form, which would hold
// more tiles) produced wrong, run-to-run varying results with ROCm 7.2.
constexpr int R4_RT = 26;
constexpr int R4_LT = 8;                                 // LDS tiles per wave (modules of > 207 nodes)
static_assert(R4_NW * (R4_RT + R4_LT) >= R4_NTMAX, "tile capacity");
// the matvec flushes its mirrored column parts four tiles at a time
constexpr int R4_TW = (R4_RT + R4_LT + 3) / 4 * 4;
constexpr int R4_MCAP = 160;                             // Lanczos step cap
constexpr int R4_LDS_BYTES = 160 * 1024;

// LDS layout: one static block (compile-time offsets; every access a ds_*
// instruction with an immediate offset, no pointer registers). A persistent
// part, then a region shared by the Gram's slab staging and the Lanczos
// partial sums + basis.
constexpr int R4_PERSIST_DOUBLES = 64 + 7 * R4_KP + 48 + 8 * R4_MCAP + 3 * (R4_MCAP + 1) + 1 + R4_NW * R4_MCAP;
constexpr int R4_PERSIST_BYTES = R4_PERSIST_DOUBLES * 8 + 2 * 4 * R4_KP + 8 * 4;
constexpr int R4_REGION = (R4_LDS_BYTES - R4_PERSIST_BYTES) / 8;

struct R4Smem {
  double red[64];        // [0,4) alpha parts, [4,8) norm parts, [8,40) block_sums, [40,44) reorth norms
  double xb[2][R4_KP + 16];  // Lanczos vectors (zero beyond k; a block of read-ahead pad)
  double vv[R4_KP + 16];     // Ritz vector (zero beyond k)
  double gv[R4_KP];      // G v
  double colm[R4_KP];    // column means
  double gdiag[R4_KP];   // diag(G)
  double ncw[R4_KP];     // node contributions
  double alpha[R4_MCAP];
  double beta[R4_MCAP];
  double ty[R4_MCAP];    // tridiagonal eigenvector / residual scratch
  double twork[5 * R4_MCAP];
  double omg[3 * (R4_MCAP + 1) + 1];  // omega rows
  double hp[R4_NW][R4_MCAP];          // reorthogonalisation partials
  uint32_t idx[R4_KP];
  int colofs[R4_KP];     // data column offset, -1 ones column, -2 zero padding
  int flags[8];
  double region[R4_REGION];
};
static_assert(sizeof(R4Smem) <= R4_LDS_BYTES, "LDS budget");


size_t rg4_kernel_lds() { return 0; }  // static LDS
int rg4_kernel_k_max() { return R4_KP - 1; }  // 255

// (I, J) of tile id t in row-major upper-triangle order.
__device__ __forceinline__ void r4_coords(int T, int t, int& I, int& J) {
  I = 0;
  while (I < T && t >= T - I) {
    t -= T - I;
    ++I;
  }
  J = I + t;
}

// A wave's tile range as wave-uniform bit masks over its tiles t = 0..cnt-1:
// `diag` marks diagonal tiles (a run of equal I starts there), `end` the last
// tile of each run (and the range's last tile). The unrolled tile loops test
// single bits instead of re-deriving the run structure per tile.
struct R4Span {
  int I0, J0;          // coordinates of tile 0
  uint64_t diag, end;  // per-tile flags
  int cnt;
};

__device__ __forceinline__ R4Span r4_span(int T, int t0, int cnt) {
  R4Span sp;
  r4_coords(T, t0, sp.I0, sp.J0);
  sp.cnt = cnt;
  sp.diag = sp.end = 0;
  int I = sp.I0, J = sp.J0;
  for (int t = 0; t < cnt; ++t) {
    if (I == J) sp.diag |= 1ull << t;
    if (J + 1 == T || t + 1 == cnt) sp.end |= 1ull << t;
    if (++J == T) {
      ++I;
      J = I;
    }
  }
  return sp;
}

// The tiles from position `from` on, as a span of their own.
__device__ __forceinline__ R4Span r4_subspan(const R4Span& a, int T, int from) {
  R4Span sp;
  int I = a.I0, J = a.J0;
  for (int t = 0; t < from; ++t) {
    if (++J == T) {
      ++I;
      J = I;
    }
  }
  sp.I0 = I;
  sp.J0 = J;
  sp.cnt = a.cnt - from;
  sp.diag = from < 64 ? a.diag >> from : 0;
  sp.end = from < 64 ? a.end >> from : 0;
  return sp;
}

// ---------------------------------------------------------------------------
// Gram: acc[t] = tile t of [X 1]^T [X 1] for this wave's cnt tiles from (I0, J0).
// Rows arrive in 8-row slabs: per tile and slab two MFMAs, lane (i16, kk)
// feeding rows 2kk and 2kk+1 (the K order is permuted identically for both
// operands). A group of D slabs (4 kp D <= 1,280 16-byte pieces, five per
// thread) is staged through LDS while the next group's pieces are in flight
// in registers.
// ---------------------------------------------------------------------------
constexpr int R4_RS = 8;      // rows per slab
constexpr int R4_SLD8 = 10;   // LDS column stride of a slab (8 rows + pad)
constexpr int R4_PIECES8 = 5; // staged 16-byte pieces per thread per group

template <int NTW>
__device__ __forceinline__ void r4_gram(nr_f64x4 (&acc)[NTW], int T, const R4Span& sp,
                                        const double* __restrict__ X, int S, R4Smem& L, int& bad) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int i16 = lane & 15, kk = lane >> 4;
  const int kp = 16 * T;
  const int cnt = sp.cnt < NTW ? sp.cnt : NTW;
#pragma unroll
  for (int t = 0; t < NTW; ++t) acc[t] = nr_f64x4{0.0, 0.0, 0.0, 0.0};
  const int nsl = (S + R4_RS - 1) / R4_RS;
  constexpr int pieces_per_col = R4_RS / 2;
  int D = (R4_PIECES8 * R4_BS) / (pieces_per_col * kp);
  D = D < 1 ? 1 : (D > nsl ? nsl : D);
  const int npg = pieces_per_col * kp * D;  // pieces per group
  double* stage = &L.region[0];
  // this thread's pieces: key = column << 8 | slab << 2 | part (part: rows 2 part, 2 part + 1)
  int key[R4_PIECES8];
#pragma unroll
  for (int u = 0; u < R4_PIECES8; ++u) {
    const int p = tid + R4_BS * u;
    if (p < npg) {
      const int d = p / (pieces_per_col * kp), rem = p - d * pieces_per_col * kp;
      key[u] = ((rem >> 2) << 8) | (d << 2) | (rem & 3);
    } else {
      key[u] = -1;
    }
  }
  double st[R4_PIECES8][2];
  auto load_group = [&](int g) {
    const int row0 = g * D * R4_RS;
#pragma unroll
    for (int u = 0; u < R4_PIECES8; ++u) {
      st[u][0] = st[u][1] = 0.0;
      if (key[u] >= 0) {
        const int r = row0 + ((key[u] >> 2) & 63) * R4_RS + 2 * (key[u] & 3);
        const int o = L.colofs[key[u] >> 8];
        if (o >= 0) {
          const double* col = X + o;
          st[u][0] = r < S ? col[r] : 0.0;
          st[u][1] = r + 1 < S ? col[r + 1] : 0.0;
        } else if (o == -1) {
          st[u][0] = r < S ? 1.0 : 0.0;
          st[u][1] = r + 1 < S ? 1.0 : 0.0;
        }
      }
    }
  };
  auto store_group = [&]() {
#pragma unroll
    for (int u = 0; u < R4_PIECES8; ++u) {
      if (key[u] >= 0) {
        const int c = key[u] >> 8, d = (key[u] >> 2) & 63, part = key[u] & 3;
        *reinterpret_cast<double2*>(stage + (d * kp + c) * R4_SLD8 + 2 * part) = make_double2(st[u][0], st[u][1]);
        // non-finite data (checked here, after the loads had the MFMAs to land)
        bad |= (int)!isfinite(st[u][0]) | (int)!isfinite(st[u][1]);
      }
    }
  };
  const int ngroups = (nsl + D - 1) / D;
  load_group(0);
  for (int g = 0; g < ngroups; ++g) {
    __syncthreads();  // the previous group is consumed
    store_group();
    __syncthreads();
    if (g + 1 < ngroups) load_group(g + 1);  // in flight during the MFMAs below
    const int nd = nsl - g * D < D ? nsl - g * D : D;
    for (int d = 0; d < nd; ++d) {
      const double* base = stage + d * kp * R4_SLD8;
      auto blk = [&](int b, double (&v)[2]) {
        const double2 x2 = *reinterpret_cast<const double2*>(base + (b * 16 + i16) * R4_SLD8 + 2 * kk);
        v[0] = x2.x;
        v[1] = x2.y;
      };
      // opaque per slab: otherwise the tile coordinates of every unrolled
      // tile are hoisted out of the slab loops and pin registers
      int I = sp.I0, J = sp.J0, nn = cnt, TT = T;
      uint64_t m_diag = sp.diag, m_end = sp.end;
      asm volatile("" : "+s"(I), "+s"(J), "+s"(nn), "+s"(TT), "+s"(m_diag), "+s"(m_end));
      double a[2], b[2], bn[2];
      blk(J, b);
      a[0] = b[0];
      a[1] = b[1];
      if (I != J) blk(I, a);
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        if (t < nn) {
          const bool e = (m_end >> t) & 1;
          const int Jn = e ? I + 1 : J + 1;
          const int In = e ? I + 1 : I;
          if (t + 1 < nn) blk(Jn, bn);
          if ((m_diag >> t) & 1) {
            a[0] = b[0];
            a[1] = b[1];
          }
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0], b[0], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[1], b[1], acc[t], 0, 0, 0);
          b[0] = bn[0];
          b[1] = bn[1];
          I = In;
          J = Jn;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

// Gram epilogue: 1'G1 over the X block (off-diagonal tiles twice), diag(G),
// column means (column k holds the column sums).
template <int NTW>
__device__ __forceinline__ void r4_epilogue(const nr_f64x4 (&acc)[NTW], int T, int I, int J, int cnt, int k,
                                            double Sd, double& g1, double* gdiag, double* colm,
                                            double* lt = nullptr) {
  const int lane = threadIdx.x & 63;
  const int i16 = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    if (t < cnt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = I * 16 + kk + 4 * r, gj = J * 16 + i16;
        const double v = acc[t][r];
        if (gi < k && gj < k) g1 += (I == J ? 1.0 : 2.0) * v;
        if (gi == gj && gi < k) gdiag[gi] = v;
        if (gj == k && gi < k) colm[gi] = v / Sd;  // column sums -> means
        if (lt) lt[t * 256 + r * 64 + lane] = v;
      }
      if (++J == T) {
        ++I;
        J = I;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Matvec from the register tiles. partials(x) writes, for w = G x:
//   rowp[wave][r]   row parts of the runs of equal I (DPP row reduction)
//   colp[id][c]     the mirrored parts G_IJ^T x_I of off-diagonal tile id
// and returns this lane's share of x^T G x. combine(r) then sums the parts of
// row r (zeroing rowp as it reads). x must be zero from k to 16 T.
// ---------------------------------------------------------------------------
struct R4Mv {
  nr_f64x4 (&acc)[R4_RT];
  const double* ltile;  // this wave's LDS tiles [LT][4][64]
  R4Span sp;            // the wave's tiles
  int T, t0;
  double* rowp;  // [NW][KP]
  double* colp;  // [NTMAX][16]

  __device__ __forceinline__ double partials(const double* x) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int i16 = lane & 15, kk = lane >> 4;
    const int b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1;
    const int rrow = kk + 4 * (2 * ((lane >> 3) & 1) + ((lane >> 2) & 1));
    int I = sp.I0, J = sp.J0, nn = sp.cnt, tt0 = t0, TT = T;
    uint64_t m_diag = sp.diag, m_end = sp.end;
    asm volatile("" : "+s"(I), "+s"(J), "+s"(nn), "+s"(tt0), "+s"(TT), "+s"(m_diag), "+s"(m_end));
    double ra[4] = {0.0, 0.0, 0.0, 0.0};
    double xi[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) xi[r] = x[I * 16 + kk + 4 * r];
    double xj = x[J * 16 + i16];
    double cx[4] = {0.0, 0.0, 0.0, 0.0};
    int cid[4] = {-1, -1, -1, -1};
    double apart = 0.0;
#pragma unroll
    for (int t = 0; t < R4_TW; ++t) {
      if (t < nn) {
        const bool e = (m_end >> t) & 1, dg = (m_diag >> t) & 1;
        // next tile: (I, J+1) inside a run, (I+1, I+1) after its end (x is
        // padded by a zero block, so the read past the last tile is harmless)
        const int Jn = e ? I + 1 : J + 1;
        const int In = e ? I + 1 : I;
        const double xjn = x[Jn * 16 + i16];
        nr_f64x4 g;
        if (t < R4_RT) {
          g = acc[t < R4_RT ? t : 0];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) g[r] = ltile[(t - R4_RT) * 256 + r * 64 + lane];
        }
        double c = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ra[r] = fma(g[r], xj, ra[r]);
          c = fma(g[r], xi[r], c);
        }
        apart = fma(dg ? c : 2.0 * c, xj, apart);
        cx[t & 3] = dg ? 0.0 : c;
        cid[t & 3] = dg ? -1 : tt0 + t;
        if (e) {  // end of a run of equal I
          const double v = rg_row_reduce(ra, lane);
          if ((lane & 3) == 0) rowp[wave * R4_KP + I * 16 + rrow] = v;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ra[r] = 0.0;
            xi[r] = x[In * 16 + kk + 4 * r];
          }
        }
        I = In;
        J = Jn;
        xj = xjn;
      } else {
        cx[t & 3] = 0.0;
        cid[t & 3] = -1;
      }
      if ((t & 3) == 3 && t - 3 < nn) {
        const double a0 = nr_swap32_sum(cx[0], cx[1]);
        const double a1 = nr_swap32_sum(cx[2], cx[3]);
        const double v = nr_swap16_sum(a0, a1);
        const int sl = 2 * b4 + b5;
        const int id = sl == 0 ? cid[0] : sl == 1 ? cid[1] : sl == 2 ? cid[2] : cid[3];
        if (id >= 0) colp[id * 16 + i16] = v;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    return apart;
  }

  // sum of the parts of row rr (rr < 16 T); zeroes its rowp entries
  __device__ __forceinline__ double combine(int rr) const {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < R4_NW; ++w) {
      s += rowp[w * R4_KP + rr];
      rowp[w * R4_KP + rr] = 0.0;
    }
    const int Jr = rr >> 4, c = rr & 15;
    int id = Jr;  // id(0, Jr)
    for (int Ii = 0; Ii < Jr; ++Ii) {
      s += colp[id * 16 + c];
      id += T - Ii - 1;
    }
    return s;
  }
};

// mv(x, out, y) for profile_contrib: out = G x (rows < k), returns y . out.
struct R4MvOp {
  R4Mv& mv;
  double* red;
  int k, kp;
  __device__ __forceinline__ double operator()(const double* x, double* out, const double* y) {
    (void)mv.partials(x);
    __syncthreads();
    double d[1] = {0.0};
    for (int rr = threadIdx.x; rr < kp; rr += R4_BS) {
      const double s = mv.combine(rr);
      if (rr < k) {
        out[rr] = s;
        if (y) d[0] += y[rr] * s;
      }
    }
    block_sums<1, R4_NW>(d, red);
    return d[0];
  }
};

// Lanczos basis column j (k doubles): LDS for j < mq, else the slot's scratch.
struct R4Basis {
  double* lds;
  double* glob;
  int mq, k;
  __device__ __forceinline__ double* col(int j) const {
    return j < mq ? lds + (size_t)j * k : glob + (size_t)(j - mq) * k;
  }
};

// ---------------------------------------------------------------------------
// Lanczos for the top eigenpair of the leading k x k block of G; leaves the
// normalised Ritz vector in L.vv (zero beyond k). Every thread owns rows
// r = tid and tid + 256.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void r4_lanczos(const ProfileParams& P, int k, int kp, R4Smem& L, R4Mv& mv,
                                           const R4Basis& Q, uint64_t& t_mark) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mcap = k < R4_MCAP ? k : R4_MCAP;
  double* red = L.red;
  // start vector (deterministic, nearly flat), normalised
  double q[2] = {0.0, 0.0}, qp[2] = {0.0, 0.0}, wp[2] = {0.0, 0.0};
  {
    double nq[1] = {0.0};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = tid + h * R4_BS;
      if (r < k) {
        const uint32_t hsh = nr_lowbias32((uint32_t)r * 0x9E3779B9u + 0x1234567u);
        q[h] = 1.0 + 0.01 * ((double)(hsh & 0xFFFF) / 65536.0 - 0.5);
        nq[0] += q[h] * q[h];
      }
    }
    block_sums<1, R4_NW>(nq, red + 8);
    const double inv = 1.0 / sqrt(nq[0]);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = tid + h * R4_BS;
      if (r < k) L.xb[0][r] = q[h] * inv;
    }
  }
  __syncthreads();
  double s = 1.0, beta_prev = 0.0, anorm = 0.0;
  const double eps = 2.220446049250313e-16, sqrt_eps = 1.4901161193847656e-08;
  double* omg = L.omg;
  if (tid == 0) omg[0] = 1.0;
  bool force_next = false;
  int next_check = mcap < 16 ? mcap : 16;
  int prev_j = 0;
  double prev_r = 0.0, prev_theta = 0.0;  // the previous check (warm start of the next)
  int nsteps = 0;
  bool done = false;
  for (int j = 0; j < mcap && !done; ++j) {
    const int cur = j & 1;
    const double* u = L.xb[cur];
    NR_STAMP(7);  // phase stamps (wave 0): 7 scalar work, 3 partials, 6 barrier A, 2 combine + barrier B
    // ---- matvec on the unnormalised u = q_j / s ----
    double ap = mv.partials(u);
    NR_STAMP(3);
    ap = wave_sum(ap);
    if (lane == 0) red[wave] = ap;
    __syncthreads();  // A: partials and alpha parts complete
    NR_STAMP(6);
    const double alpha0 = s * s * (red[0] + red[1] + red[2] + red[3]);
    double* qj = Q.col(j);
    double nb_part = 0.0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = tid + h * R4_BS;
      if (r < kp) {
        const double ws = mv.combine(r);
        if (r < k) {
          q[h] = s * u[r];
          qj[r] = q[h];
          wp[h] = s * ws - alpha0 * q[h] - beta_prev * qp[h];
          nb_part = fma(wp[h], wp[h], nb_part);
          L.xb[cur ^ 1][r] = wp[h];
        }
      }
    }
    nb_part = wave_sum(nb_part);
    if (lane == 0) red[4 + wave] = nb_part;
    __syncthreads();  // B: w' and its norm parts complete
    NR_STAMP(2);
    double nb = red[4] + red[5] + red[6] + red[7];
    double alpha_j = alpha0;
    anorm = fmax(anorm, fabs(alpha0) + sqrt(nb) + beta_prev);
    if (lane == 0) L.alpha[j] = alpha0;  // every wave writes the same value
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    // partial reorthogonalisation (Simon): omega recurrence, identical in every wave
    double* om_cur = omg + (j % 3) * (R4_MCAP + 1);
    double* om_prev = omg + ((j + 2) % 3) * (R4_MCAP + 1);
    double* om_next = omg + ((j + 1) % 3) * (R4_MCAP + 1);
    const double mx = omega_update(L.alpha, L.beta, j, L.alpha[j], sqrt(nb), om_cur, om_prev, om_next, anorm, k, lane);
    const bool reorth = force_next || mx > sqrt_eps;
    if (reorth) {
      NR_STAMP(7);
      // h = Q^T w' over q_0..q_j: per-wave partials, 16 basis vectors per burst
      const int nj = j + 1;
      for (int i0 = 0; i0 < nj; i0 += 16) {
        double up[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          double a = 0.0;
          if (i0 + t < nj) {
            const double* qc = Q.col(i0 + t);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int r = tid + h * R4_BS;
              if (r < k) a = fma(qc[r], wp[h], a);
            }
          }
          up[t] = a;
        }
        const double v = nr_transpose_reduce16(up, lane);
        if ((lane & 3) == 0) {  // these 16 lanes hold the wave's 16 sums
          const int i = i0 + ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 +
                        ((lane >> 2) & 1);
          if (i < nj) L.hp[wave][i] = v;
        }
      }
      __syncthreads();
      double nb2 = 0.0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = tid + h * R4_BS;
        if (r < k) {
          double acc = 0.0;
          for (int i = 0; i < nj; ++i) {
            const double hi = L.hp[0][i] + L.hp[1][i] + L.hp[2][i] + L.hp[3][i];
            acc = fma(hi, Q.col(i)[r], acc);
          }
          wp[h] -= acc;
          nb2 = fma(wp[h], wp[h], nb2);
          L.xb[cur ^ 1][r] = wp[h];
        }
      }
      alpha_j += L.hp[0][j] + L.hp[1][j] + L.hp[2][j] + L.hp[3][j];
      nb2 = wave_sum(nb2);
      if (lane == 0) red[40 + wave] = nb2;
      __syncthreads();
      nb = red[40] + red[41] + red[42] + red[43];
      for (int i = lane; i <= j; i += 64) om_next[i] = eps;
      force_next = !force_next;
      if (P.diag && tid == 0) atomicAdd(P.diag + 3, 1);
      NR_STAMP(4);
    }
    const double beta_j = sqrt(nb);
    if (lane == 0) {
      L.alpha[j] = alpha_j;
      L.beta[j] = beta_j;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    nsteps = j + 1;
    const bool last = (j + 1 == mcap);
    if (j + 1 == next_check || last || !(beta_j > 1e-300 * fabs(alpha_j))) {
      // every wave computes the same Ritz check (no broadcast barrier)
      const double theta = tri_top_eigenvalue(L.alpha, L.beta, j + 1, lane, prev_theta, prev_r);
      const double resid = tri_top_resid(L.alpha, L.beta, j + 1, theta, beta_j, L.ty + 0, lane);
      const double tol = 5e-15 * fabs(theta);
      const bool conv = resid <= tol;
      done = conv || last || !(beta_j > 1e-300 * fabs(theta));
      if (done) {
        __syncthreads();  // every wave is done with ty before wave 0 overwrites it
        if (tid == 0) {
          tri_eigenvector(L.alpha, L.beta, j + 1, theta, L.ty, L.twork);
          if (last && !conv && P.diag) atomicAdd(P.diag, 1);
        }
      } else {
        int step = 8;
        if (prev_j > 0 && resid < prev_r && resid > 0.0) {
          const double rate = log(resid / prev_r) / (double)(j + 1 - prev_j);
          const double need = ceil(log(tol / resid) / rate);
          step = need < 1.0 ? 1 : (need > 8.0 ? 8 : (int)need);
        }
        prev_j = j + 1;
        prev_r = resid;
        prev_theta = theta;
        next_check = min(j + 1 + step, mcap);
      }
    }
    qp[0] = q[0];
    qp[1] = q[1];
    s = 1.0 / beta_j;
    beta_prev = beta_j;
  }
  NR_STAMP(7);
  if (tid == 0 && P.diag) {
    atomicAdd(P.diag + 1, 1);
    atomicAdd(P.diag + 2, nsteps);
  }
  __syncthreads();  // ty (the Ritz coefficients) published
  // Ritz vector v = Q y, normalised
  double v[2] = {0.0, 0.0};
  double nv[1] = {0.0};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = tid + h * R4_BS;
    if (r < k) {
      double a = 0.0;
      for (int i = 0; i < nsteps; ++i) a = fma(L.ty[i], Q.col(i)[r], a);
      v[h] = a;
      nv[0] += a * a;
    }
  }
  block_sums<1, R4_NW>(nv, red + 8);
  const double inv = 1.0 / sqrt(nv[0]);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = tid + h * R4_BS;
    if (r < k) L.vv[r] = v[h] * inv;
  }
  __syncthreads();
}

__global__ void __launch_bounds__(R4_BS, 1)
module_profile_rg4_kernel(ProfileParams P) {
  uint64_t t_mark = P.stamps && threadIdx.x == 0 ? nr_clock() : 0;
  __shared__ R4Smem L;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int S = (int)P.n_samples;
  const double Sd = (double)S;
  const double* __restrict__ X = P.data;
  double* rowp = L.region;                          // [NW][KP] (Lanczos phase)
  double* colp = rowp + R4_NW * R4_KP;              // [NTMAX][16]
  double* qlds = colp + R4_NTMAX * 16;              // basis columns that fit
  const int q_doubles = R4_REGION - (R4_NW * R4_KP + R4_NTMAX * 16);
  double* qglob = P.scratch + (int64_t)blockIdx.x * P.scratch_stride;
  // the workgroup-level views next_item / profile_contrib / profile_stats expect
  LzLds Lz;
  Lz.red = L.red + 8;
  Lz.q = Lz.qprev = nullptr;
  Lz.w = L.ncw;
  Lz.vv = L.vv;
  Lz.gv = L.gv;
  Lz.colm = L.colm;
  Lz.alpha = L.alpha;
  Lz.beta = L.beta;
  Lz.h = nullptr;
  Lz.ty = L.ty;
  Lz.twork = L.twork;
  Lz.omg = L.omg;
  Lz.idx = L.idx;
  Lz.mmax = R4_MCAP;
  for (int i = tid; i < R4_NW * R4_KP; i += R4_BS) rowp[i] = 0.0;

  int m, k;
  int64_t p_local, off;
  while (next_item<R4_NW>(P, Lz, L.flags, m, p_local, off, k)) {
    NR_STAMP(0);  // queue + index derivation
    const int T = (k + 1 + 15) / 16;
    const int kp = 16 * T;
    const int nt = T * (T + 1) / 2;
    const int t0 = wave * nt / R4_NW;
    const int cnt = (wave + 1) * nt / R4_NW - t0;
    const R4Span span = r4_span(T, t0, cnt);
    for (int c = tid; c < kp; c += R4_BS) {
      L.colofs[c] = c < k ? (int)L.idx[c] * S : (c == k ? -1 : -2);
      L.xb[0][c] = 0.0;
      L.xb[1][c] = 0.0;
      L.vv[c] = 0.0;
    }
    __syncthreads();
    NR_STAMP(6);
    int bad = 0;
    double g1[1] = {0.0};
    // Modules of more than 207 nodes: the tiles beyond 26 per wave live in
    // LDS, computed by a first Gram pass (uniform over the workgroup).
    const bool lds_tiles = (nt + R4_NW - 1) / R4_NW > R4_RT;
    const int cnt_r = cnt < R4_RT ? cnt : R4_RT;
    double* ltile = colp + R4_NTMAX * 16 + wave * R4_LT * 256;
    if (lds_tiles) {
      const R4Span sl = r4_subspan(span, T, cnt_r);
      nr_f64x4 accl[R4_LT];
      r4_gram<R4_LT>(accl, T, sl, X, S, L, bad);
      r4_epilogue<R4_LT>(accl, T, sl.I0, sl.J0, sl.cnt, k, Sd, g1[0], L.gdiag, L.colm, ltile);
    }
    nr_f64x4 acc[R4_RT];
    r4_gram<R4_RT>(acc, T, span, X, S, L, bad);
    r4_epilogue<R4_RT>(acc, T, span.I0, span.J0, cnt_r, k, Sd, g1[0], L.gdiag, L.colm);
    if (bad) atomicOr(&L.flags[1], 1);
    __syncthreads();  // slab reads done before the region becomes rowp/colp
    for (int i = tid; i < R4_NW * R4_KP; i += R4_BS) rowp[i] = 0.0;
    block_sums<1, R4_NW>(g1, Lz.red);  // barriers also publish gdiag, colm, flags
    NR_STAMP(1);  // Gram
    if (L.flags[1] == 0) {
      R4Mv mv{acc, ltile, span, T, t0, rowp, colp};
      const int mq_fit = (q_doubles - (lds_tiles ? R4_NW * R4_LT * 256 : 0)) / k;
      R4Basis Q{qlds + (lds_tiles ? R4_NW * R4_LT * 256 : 0), qglob, mq_fit < R4_MCAP ? mq_fit : R4_MCAP, k};
      r4_lanczos(P, k, kp, L, mv, Q, t_mark);
      R4MvOp op{mv, Lz.red, k, kp};
      profile_contrib<R4_NW>(P, k, m, Lz, X, S, g1[0], op, [&](int c) { return L.gdiag[c]; });
    } else {
      profile_nonfinite<R4_NW>(P, k, m, S, Lz);
    }
    profile_stats<R4_NW>(P, k, m, off, p_local, Lz);
    NR_STAMP(5);  // Ritz vector, contributions, statistics
  }
}

hipError_t launch_profile_rg4(const ProfileParams& P, int n_slots, hipStream_t st) {
  hipLaunchKernelGGL(module_profile_rg4_kernel, dim3((unsigned)n_slots), dim3(R4_BS), 0, st, P);
  return hipGetLastError();
}

}  // namespace nr
