// Microbenchmark of the summary-profile kernel's packed symmetric matvec in
// isolation (GPU box): every workgroup owns one packed Gram of side k in its
// own global slot, three 4-wave workgroups per CU as in the product kernel,
// and runs dependent passes x <- G x / |G x| (the Lanczos access pattern).
// Reports the time per pass and the chip-wide byte rate of the packed Gram
// reads for the product matvec (kernels.hip packed_matvec) and candidate
// variants.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/matvec_probe.hip -o /tmp/matvec_probe
//   /tmp/matvec_probe [k] [passes] [LDS KiB per workgroup: 52 -> 3 per CU, 80 -> 2, 160 -> 1]
#include "../../netrep_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace nr {

// Variant 1: the next unit's 16 column segments are in flight while this
// unit is reduced.
template <int NW>
__device__ __forceinline__ double packed_matvec_pipe(const double* __restrict__ P, int kc, int k, const double* x,
                                                     double* out, double* part, double* upper, int ks,
                                                     const double* y, double* red) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int i = threadIdx.x; i < NW * ks; i += NW * 64) {
    part[i] = 0.0;
    upper[i] = 0.0;
  }
  __syncthreads();
  const int nrec = (kc * (kc + 1) / 2 + 1) * 8;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)P, (short)0, nrec, 0x00020000);
  const int nrb = (k + 63) / 64;
  auto ncg_of = [&](int rb) { return (min(k, (rb + 1) * 64) + 15) / 16; };
  auto load = [&](int rb, int cg, double (&g)[16]) {
    const int r = rb * 64 + lane;
    const int cmax = min(k, (rb + 1) * 64);
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int c = cg * 16 + t;
      const int colbase = c * kc - c * (c - 1) / 2 - c;
      const bool ok = c < cmax && r >= c && r < k;
      g[t] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                            rsrc, ok ? r * 8 : (int)0x80000000, colbase * 8, 0));
    }
  };
  // units of this wave in order: (row block rb, column group cg)
  auto advance = [&](int& rb, int& cg) {
    cg += NW;
    while (rb < nrb && cg >= ncg_of(rb)) {
      ++rb;
      cg = wave;
    }
  };
  double acc = 0.0;
  auto compute = [&](int rb, int cg, int rb_next, double (&g)[16]) {
    const int r = rb * 64 + lane;
    const int cmax = min(k, (rb + 1) * 64);
    const double xr = x[min(r, k - 1)];
    const int c0 = cg * 16;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int c = c0 + t;
      acc += g[t] * x[min(c, k - 1)];
      g[t] = (r > c) ? g[t] * xr : 0.0;
    }
    const double v = nr_transpose_reduce16(g, lane);
    if ((lane & 3) == 0) {
      const int c = c0 + ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
      if (c < cmax) upper[wave * ks + c] += v;
    }
    if (rb_next != rb) {
      if (r < k) part[wave * ks + r] += acc;
      acc = 0.0;
    }
  };
  int rb = 0, cg = wave - NW;
  advance(rb, cg);
  // two register sets in ping-pong: the next unit's loads are issued
  // (unconditionally: past the end every lane is out of range and reads 0)
  // before this unit is reduced
  double gA[16], gB[16];
  load(rb, cg, gA);
  while (rb < nrb) {
    int rb1 = rb, cg1 = cg;
    advance(rb1, cg1);
    load(rb1, cg1, gB);
    compute(rb, cg, rb1, gA);
    if (rb1 >= nrb) break;
    int rb2 = rb1, cg2 = cg1;
    advance(rb2, cg2);
    load(rb2, cg2, gA);
    compute(rb1, cg1, rb2, gB);
    rb = rb2;
    cg = cg2;
  }
  __syncthreads();
  double d[1] = {0.0};
  for (int rr = threadIdx.x; rr < k; rr += NW * 64) {
    double sum = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) sum += part[w * ks + rr] + upper[w * ks + rr];
    out[rr] = sum;
    if (y) d[0] += y[rr] * sum;
  }
  block_sums<1, NW>(d, red);
  return d[0];
}

// Variant 2 (ceiling): the same bytes read as a plain 16-byte-per-lane stream,
// summed, no matvec structure.
template <int NW>
__device__ __forceinline__ double stream_read(const double* __restrict__ P, int kc, double* red) {
  const int n2 = (kc * (kc + 1) / 2) / 2;
  const double2* p2 = reinterpret_cast<const double2*>(P);
  double s[1] = {0.0};
  int i = threadIdx.x;
  for (; i + 3 * NW * 64 < n2; i += 4 * NW * 64) {
    double2 a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = p2[i + u * NW * 64];
#pragma unroll
    for (int u = 0; u < 4; ++u) s[0] += a[u].x + a[u].y;
  }
  for (; i < n2; i += NW * 64) s[0] += p2[i].x + p2[i].y;
  block_sums<1, NW>(s, red);
  return s[0];
}

// Variant 3: the stream with 8-byte-per-lane loads.
template <int NW>
__device__ __forceinline__ double stream_read8(const double* __restrict__ P, int kc, double* red) {
  const int n = kc * (kc + 1) / 2;
  double s[1] = {0.0};
  int i = threadIdx.x;
  for (; i + 7 * NW * 64 < n; i += 8 * NW * 64) {
    double a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = P[i + u * NW * 64];
#pragma unroll
    for (int u = 0; u < 8; ++u) s[0] += a[u];
  }
  for (; i < n; i += NW * 64) s[0] += P[i];
  block_sums<1, NW>(s, red);
  return s[0];
}

// Variant 4: the matvec's loads (same units, addresses and masks), summed
// without the matvec arithmetic.
template <int NW>
__device__ __forceinline__ double matvec_loads_only(const double* __restrict__ P, int kc, int k, double* red) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nrec = (kc * (kc + 1) / 2 + 1) * 8;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)P, (short)0, nrec, 0x00020000);
  const int nrb = (k + 63) / 64;
  double s[1] = {0.0};
  for (int rb = 0; rb < nrb; ++rb) {
    const int r = rb * 64 + lane;
    const int cmax = min(k, (rb + 1) * 64);
    const int ncg = (cmax + 15) / 16;
    for (int cg = wave; cg < ncg; cg += NW) {
      const int c0 = cg * 16;
      double g[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int c = c0 + t;
        const int colbase = c * kc - c * (c - 1) / 2 - c;
        const bool ok = c < cmax && r >= c && r < k;
        g[t] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                              rsrc, ok ? r * 8 : (int)0x80000000, colbase * 8, 0));
      }
#pragma unroll
      for (int t = 0; t < 16; ++t) s[0] += g[t];
    }
  }
  block_sums<1, NW>(s, red);
  return s[0];
}

// Group-aligned packed layout: P = kc rounded up to 16; column c of group
// g = c / 16 holds rows 16 g .. P - 1 (rows < c stored as zero) at
// ga_base(g) + (c - 16 g) (P - 16 g), so every 64-row column segment starts on
// a 128-byte line.
__host__ __device__ __forceinline__ int ga_pad(int kc) { return (kc + 15) & ~15; }
__host__ __device__ __forceinline__ int ga_base(int g, int P) { return 16 * g * P - 128 * g * (g - 1); }
__host__ __device__ __forceinline__ int ga_total(int kc) {
  const int P = ga_pad(kc);
  return ga_base(P / 16, P);
}

// Variant 5: the matvec over the group-aligned layout: one lane mask per unit
// (rows below the group), scalar column offsets by increment, the diagonal
// compare only in units that touch the diagonal.
template <int NW>
__device__ __forceinline__ double aligned_matvec(const double* __restrict__ Ga, int kc, int k, const double* x,
                                                 double* out, double* part, double* upper, int ks,
                                                 const double* y, double* red) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int i = threadIdx.x; i < NW * ks; i += NW * 64) {
    part[i] = 0.0;
    upper[i] = 0.0;
  }
  __syncthreads();
  const int P = ga_pad(kc);
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Ga, (short)0, ga_total(kc) * 8, 0x00020000);
  const int nrb = (k + 63) / 64;
  for (int rb = 0; rb < nrb; ++rb) {
    const int r = rb * 64 + lane;
    const int cmax = min(k, (rb + 1) * 64);
    const int ncg = (cmax + 15) / 16;
    const double xr = r < k ? x[r] : 0.0;
    double acc = 0.0;
    for (int cg = wave; cg < ncg; cg += NW) {
      const int c0 = cg * 16;
      const int len = P - c0;
      const int vo = r >= c0 ? (r - c0) * 8 : (int)0x80000000;
      int so = ga_base(cg, P) * 8;
      double g[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        g[t] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc, vo, so, 0));
        so += len * 8;
      }
      double xc[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) xc[t] = c0 + t < k ? x[c0 + t] : 0.0;
#pragma unroll
      for (int t = 0; t < 16; ++t) acc += g[t] * xc[t];
      if (c0 + 15 < rb * 64) {  // every row of the block below every column of the unit
#pragma unroll
        for (int t = 0; t < 16; ++t) g[t] *= xr;
      } else {
#pragma unroll
        for (int t = 0; t < 16; ++t) g[t] = (r > c0 + t) ? g[t] * xr : 0.0;
      }
      const double v = nr_transpose_reduce16(g, lane);
      if ((lane & 3) == 0) {
        const int c = c0 + ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
        if (c < cmax) upper[wave * ks + c] += v;
      }
    }
    if (r < k) part[wave * ks + r] += acc;
  }
  __syncthreads();
  double d[1] = {0.0};
  for (int rr = threadIdx.x; rr < k; rr += NW * 64) {
    double sum = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) sum += part[w * ks + rr] + upper[w * ks + rr];
    out[rr] = sum;
    if (y) d[0] += y[rr] * sum;
  }
  block_sums<1, NW>(d, red);
  return d[0];
}

// Variant 6: the group-aligned layout walked column-group-major. The units
// (column group cg, row block rb >= the group's first row block) are
// numbered cg-major and cut into NW contiguous ranges, one per wave; the upper
// part sum_r G_rc x_r accumulates lane-locally across a wave's units of one
// column group and is reduced over the lanes once per (wave, group), the
// lower part is added to the wave's row partials per unit.
template <int NW>
__device__ __forceinline__ double aligned_matvec_cm(const double* __restrict__ Ga, int kc, int k, const double* x,
                                                    double* out, double* part, double* upper, int ks,
                                                    const double* y, double* red) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int i = threadIdx.x; i < NW * ks; i += NW * 64) {
    part[i] = 0.0;
    upper[i] = 0.0;
  }
  __syncthreads();
  const int P = ga_pad(kc);
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Ga, (short)0, ga_total(kc) * 8, 0x00020000);
  const int nrb = (k + 63) / 64;
  const int ncg = (k + 15) / 16;
  // units before column group cg: sum over cg' < cg of (nrb - cg' / 4)
  auto units_before = [&](int cg) {
    const int q = cg >> 2, rr = cg & 3;
    return cg * nrb - (4 * (q * (q - 1) / 2) + rr * q);
  };
  const int n_units = units_before(ncg);
  const int u0 = (int)((int64_t)n_units * wave / NW), u1 = (int)((int64_t)n_units * (wave + 1) / NW);
  // the first unit's (cg, rb)
  int cg = 0;
  while (cg + 1 < ncg && units_before(cg + 1) <= u0) ++cg;
  int rb = (cg >> 2) + (u0 - units_before(cg));
  double up[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) up[t] = 0.0;
  for (int u = u0; u < u1; ++u) {
    const int c0 = cg * 16;
    const int r = rb * 64 + lane;
    const double xr = r < k ? x[r] : 0.0;
    const int vo = r >= c0 ? (r - c0) * 8 : (int)0x80000000;
    const int len = P - c0;
    int so = ga_base(cg, P) * 8;
    double g[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      g[t] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc, vo, so, 0));
      so += len * 8;
    }
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < 16; ++t) acc += g[t] * (c0 + t < k ? x[c0 + t] : 0.0);
    if (c0 + 15 < rb * 64) {
#pragma unroll
      for (int t = 0; t < 16; ++t) up[t] += g[t] * xr;
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) up[t] += (r > c0 + t) ? g[t] * xr : 0.0;
    }
    if (r < k) part[wave * ks + r] += acc;
    // next unit; flush the upper part at the end of the group or the range
    ++rb;
    if (rb == nrb || u + 1 == u1) {
      const double v = nr_transpose_reduce16(up, lane);
      if ((lane & 3) == 0) {
        const int c = c0 + ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
        if (c < k) upper[wave * ks + c] += v;
      }
#pragma unroll
      for (int t = 0; t < 16; ++t) up[t] = 0.0;
      ++cg;
      rb = cg >> 2;
    }
  }
  __syncthreads();
  double d[1] = {0.0};
  for (int rr = threadIdx.x; rr < k; rr += NW * 64) {
    double sum = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) sum += part[w * ks + rr] + upper[w * ks + rr];
    out[rr] = sum;
    if (y) d[0] += y[rr] * sum;
  }
  block_sums<1, NW>(d, red);
  return d[0];
}

// Chunked group layout: column group g (columns 16 g .. 16 g + 15, rows
// 16 g .. P - 1, rows < c zero) is cut into row chunks of 64 (the last one
// h = L_g - 64 j rows); chunk j stores its 16 columns one after the other, h
// rows each, so a unit (g, j) is one contiguous run of 16 h doubles.
__host__ __device__ __forceinline__ int64_t ch_at(int r, int c, int P) {
  const int g = c >> 4, t = c & 15;
  const int L = P - 16 * g;
  const int rr = r - 16 * g;
  const int j = rr >> 6;
  const int h = min(64, L - 64 * j);
  return (int64_t)ga_base(g, P) + 1024 * j + t * h + (rr & 63);
}

// Variant 7: the matvec over the chunked layout, units (g, j) cg-major in
// NW contiguous ranges, one per wave.
template <int NW>
__device__ __forceinline__ double chunked_matvec(const double* __restrict__ Ga, int kc, int k, const double* x,
                                                 double* out, double* part, double* upper, int ks,
                                                 const double* y, double* red) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int i = threadIdx.x; i < NW * ks; i += NW * 64) {
    part[i] = 0.0;
    upper[i] = 0.0;
  }
  __syncthreads();
  const int P = ga_pad(kc);
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Ga, (short)0, ga_total(kc) * 8, 0x00020000);
  const int ncg = (k + 15) / 16;
  int n_units = 0;
  for (int g = 0; g < ncg; ++g) n_units += (P - 16 * g + 63) >> 6;
  const int u0 = (int)((int64_t)n_units * wave / NW), u1 = (int)((int64_t)n_units * (wave + 1) / NW);
  int cg = 0, first = 0;
  while (first + ((P - 16 * cg + 63) >> 6) <= u0) {
    first += (P - 16 * cg + 63) >> 6;
    ++cg;
  }
  int j = u0 - first;
  int nj = (P - 16 * cg + 63) >> 6;
  double up[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) up[t] = 0.0;
  for (int u = u0; u < u1; ++u) {
    const int c0 = cg * 16;
    const int L = P - c0;
    const int h = min(64, L - 64 * j);
    const int r = c0 + 64 * j + lane;
    const double xr = r < k ? x[r] : 0.0;
    const int vo = lane < h ? lane * 8 : (int)0x80000000;
    int so = (ga_base(cg, P) + 1024 * j) * 8;
    double g[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      g[t] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc, vo, so, 0));
      so += h * 8;
    }
    double acc = 0.0;
    const double xl = c0 + (lane & 15) < k ? x[c0 + (lane & 15)] : 0.0;  // the unit's 16 x_c, one per lane
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const uint64_t xu = __builtin_bit_cast(uint64_t, xl);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)xu, t);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(xu >> 32), t);
      const double xc = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
      acc += g[t] * xc;
    }
    if (j > 0) {
#pragma unroll
      for (int t = 0; t < 16; ++t) up[t] += g[t] * xr;
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) up[t] += (r > c0 + t) ? g[t] * xr : 0.0;
    }
    if (r < k) part[wave * ks + r] += acc;
    ++j;
    if (j == nj || u + 1 == u1) {
      const double v = nr_transpose_reduce16(up, lane);
      if ((lane & 3) == 0) {
        const int c = c0 + ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
        if (c < k) upper[wave * ks + c] += v;
      }
#pragma unroll
      for (int t = 0; t < 16; ++t) up[t] = 0.0;
      ++cg;
      j = 0;
      nj = (P - 16 * cg + 63) >> 6;
    }
  }
  __syncthreads();
  double d[1] = {0.0};
  for (int rr = threadIdx.x; rr < k; rr += NW * 64) {
    double sum = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) sum += part[w * ks + rr] + upper[w * ks + rr];
    out[rr] = sum;
    if (y) d[0] += y[rr] * sum;
  }
  block_sums<1, NW>(d, red);
  return d[0];
}

template <int V>
__global__ void __launch_bounds__(256, 3) mv_probe(double* Gall, int64_t stride, int k, int passes, double* res, int64_t ga_off) {
  const int64_t ch_off = ga_off + (ga_total(k + 1) + 31) / 32 * 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NW = 4, KS = 320;
  double* red = reinterpret_cast<double*>(smem);
  double* x = red + 32;
  double* w = x + KS;
  double* part = w + KS;
  double* upper = part + NW * KS;
  const double* G = Gall + (int64_t)blockIdx.x * stride;
  for (int c = threadIdx.x; c < k; c += 256) x[c] = 1.0 / sqrt((double)k);
  __syncthreads();
  double lam = 0.0;
  for (int p = 0; p < passes; ++p) {
    if (V == 7) {
      lam = chunked_matvec<NW>(G + ch_off, k + 1, k, x, w, part, upper, KS, x, red);
    } else if (V == 6) {
      lam = aligned_matvec_cm<NW>(G + ga_off, k + 1, k, x, w, part, upper, KS, x, red);
    } else if (V == 5) {
      lam = aligned_matvec<NW>(G + ga_off, k + 1, k, x, w, part, upper, KS, x, red);
    } else if (V >= 2) {
      const double t = V == 2 ? stream_read<NW>(G, k + 1, red)
                       : V == 3 ? stream_read8<NW>(G, k + 1, red) : matvec_loads_only<NW>(G, k + 1, k, red);
      lam = t * 1e-300 + 1.0 + x[0];
      for (int c = threadIdx.x; c < k; c += 256) w[c] = x[c];
      __syncthreads();
    } else {
      lam = V == 0 ? packed_matvec<NW>(G, k + 1, k, x, w, part, KS, x, red)
                   : packed_matvec_pipe<NW>(G, k + 1, k, x, w, part, upper, KS, x, red);
    }
    const double inv = 1.0 / fabs(lam);
    for (int c = threadIdx.x; c < k; c += 256) x[c] = w[c] * inv;
    __syncthreads();
  }
  if (threadIdx.x == 0) res[blockIdx.x] = lam;
}

}  // namespace nr

int main(int argc, char** argv) {
  const int k = argc > 1 ? atoi(argv[1]) : 300;
  const int passes = argc > 2 ? atoi(argv[2]) : 40;
  int cu = 256;
  (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  const int slots = 3 * cu;
  const int kc = k + 1;
  const int64_t tri = (int64_t)kc * (kc + 1) / 2 + 1;
  const int64_t stride = 3 * ((tri + 31) / 32 * 32 + 4096);  // three layouts of the Gram
  std::vector<double> h(tri);
  srand(7);
  for (int64_t i = 0; i < tri; ++i) h[i] = (double)rand() / RAND_MAX;
  h[tri - 1] = 0.0;
  double *G, *res;
  (void)hipMalloc(&G, stride * slots * sizeof(double));
  (void)hipMalloc(&res, slots * sizeof(double));
  // the same matrix in the group-aligned layout, behind the packed one in each slot
  const int P = nr::ga_pad(kc);
  std::vector<double> ha(nr::ga_total(kc), 0.0);
  for (int c = 0; c < kc; ++c) {
    const int g = c / 16;
    const int64_t base = nr::ga_base(g, P) + (int64_t)(c - 16 * g) * (P - 16 * g);
    const int64_t pcol = (int64_t)c * kc - (int64_t)c * (c - 1) / 2;  // pk_col
    for (int r = c; r < kc; ++r) ha[base + r - 16 * g] = h[pcol + r - c];
  }
  const int64_t ga_off = (tri + 31) / 32 * 32;
  const int64_t ch_off = ga_off + (ha.size() + 31) / 32 * 32;
  std::vector<double> hc(ha.size(), 0.0);
  for (int c = 0; c < kc; ++c) {
    const int64_t pcol = (int64_t)c * kc - (int64_t)c * (c - 1) / 2;
    for (int r = c; r < kc; ++r) hc[nr::ch_at(r, c, P)] = h[pcol + r - c];
  }
  for (int s = 0; s < slots; ++s) {
    (void)hipMemcpy(G + (int64_t)s * stride, h.data(), tri * sizeof(double), hipMemcpyHostToDevice);
    (void)hipMemcpy(G + (int64_t)s * stride + ga_off, ha.data(), ha.size() * sizeof(double), hipMemcpyHostToDevice);
    (void)hipMemcpy(G + (int64_t)s * stride + ch_off, hc.data(), hc.size() * sizeof(double), hipMemcpyHostToDevice);
  }
  const size_t lds = 52 * 1024;  // three workgroups per CU, as the product kernel's LDS
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const double bytes = (double)slots * passes * (double)(tri - 1) * 8.0;
  const size_t lds_v = argc > 3 ? (size_t)atoi(argv[3]) * 1024 : lds;
  for (int v = 0; v < 8; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(a);
      if (v == 0)
        hipLaunchKernelGGL(nr::mv_probe<0>, dim3(slots), dim3(256), lds_v, 0, G, stride, k, passes, res, ga_off);
      else if (v == 1)
        hipLaunchKernelGGL(nr::mv_probe<1>, dim3(slots), dim3(256), lds_v, 0, G, stride, k, passes, res, ga_off);
      else if (v == 2)
        hipLaunchKernelGGL(nr::mv_probe<2>, dim3(slots), dim3(256), lds_v, 0, G, stride, k, passes, res, ga_off);
      else if (v == 3)
        hipLaunchKernelGGL(nr::mv_probe<3>, dim3(slots), dim3(256), lds_v, 0, G, stride, k, passes, res, ga_off);
      else if (v == 7)
        hipLaunchKernelGGL(nr::mv_probe<7>, dim3(slots), dim3(256), lds_v, 0, G, stride, k, passes, res, ga_off);
      else if (v == 6)
        hipLaunchKernelGGL(nr::mv_probe<6>, dim3(slots), dim3(256), lds_v, 0, G, stride, k, passes, res, ga_off);
      else if (v == 5)
        hipLaunchKernelGGL(nr::mv_probe<5>, dim3(slots), dim3(256), lds_v, 0, G, stride, k, passes, res, ga_off);
      else
        hipLaunchKernelGGL(nr::mv_probe<4>, dim3(slots), dim3(256), lds_v, 0, G, stride, k, passes, res, ga_off);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, a, b);
      double r0 = 0.0;
      (void)hipMemcpy(&r0, res, sizeof(double), hipMemcpyDeviceToHost);
      if (rep == 2)
        printf("variant %d k=%d: %.3f ms, %.2f us/pass, %.2f TB/s packed-Gram reads (lambda %.6f)\n", v, k, ms,
               ms * 1e3 / passes, bytes / (ms * 1e-3) / 1e12, r0);
    }
  }
  if (hipGetLastError() != hipSuccess) return 1;
  return 0;
}
