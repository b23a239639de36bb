// Microbenchmark: v_mfma_f64_16x16x4_f64 issue rate and dependent latency on
// gfx950, plus an LDS-fed Gram slab loop shaped like the summary-profile
// kernel's. Diagnostic only (tools/probes); prints cycles per MFMA.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double f64x4 __attribute__((ext_vector_type(4)));

// CHAINS independent accumulators, ITERS rounds; each round issues one MFMA per
// chain. Cycles measured by s_memtime around the loop (wave 0 lane 0 of each WG).
template <int CHAINS>
__global__ void mfma_chain(double* out, unsigned long long* cyc, int iters) {
  f64x4 acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c) acc[c] = f64x4{0, 0, 0, 0};
  double a = 1.0 + threadIdx.x * 1e-3, b = 0.5 - threadIdx.x * 1e-4;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0;
  for (int c = 0; c < CHAINS; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int CHAINS>
void run(int waves_per_wg, int wgs, int iters) {
  const int threads = waves_per_wg * 64;
  double* d_out;
  unsigned long long* d_cyc;
  hipMalloc(&d_out, sizeof(double) * threads * wgs);
  hipMalloc(&d_cyc, sizeof(unsigned long long) * waves_per_wg * wgs);
  hipLaunchKernelGGL(mfma_chain<CHAINS>, dim3(wgs), dim3(threads), 0, 0, d_out, d_cyc, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma_chain<CHAINS>, dim3(wgs), dim3(threads), 0, 0, d_out, d_cyc, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> c(waves_per_wg * wgs);
  hipMemcpy(c.data(), d_cyc, c.size() * 8, hipMemcpyDeviceToHost);
  double mean = 0;
  for (auto v : c) mean += (double)v;
  mean /= c.size();
  const double n_mfma = (double)iters * CHAINS;
  const double flops = n_mfma * 2048.0 * waves_per_wg * wgs;
  printf("chains=%d waves/wg=%d wgs=%d: %.1f cyc per MFMA per wave; kernel %.3f ms = %.2f TF/s\n", CHAINS,
         waves_per_wg, wgs, mean / n_mfma, ms, flops / (ms * 1e-3) / 1e12);
  hipFree(d_out);
  hipFree(d_cyc);
}

int main() {
  const int it = 4096;
  // latency: one wave per CU, one chain
  run<1>(1, 256, it);
  run<2>(1, 256, it);
  run<4>(1, 256, it);
  run<8>(1, 256, it);
  // throughput: one wave per SIMD
  run<1>(4, 256, it);
  run<4>(4, 256, it);
  run<8>(4, 256, it);
  // two waves per SIMD
  run<1>(8, 256, it);
  run<4>(8, 256, it);
  run<8>(8, 256, it);
  return 0;
}
