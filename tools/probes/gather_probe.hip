// Microbenchmark: the random-access ceiling of the network-statistics gather.
// A module's pairs read corr/net(idx[ii], idx[jj]) as ONE 16-byte element of
// the interleaved N x N double2 matrix at a random (row, column): every read
// touches its own cache line. This measures, chip-wide, how many such random
// 16-byte reads per second MI355X sustains from a matrix far larger than the
// Infinity Cache (N = 20,000: 6.4 GB), for several loads in flight per
// thread, and the same for 8-byte reads (one of the two matrices alone).
// Output: reads/s and useful GB/s (the ceiling DESIGN.md quotes for the net
// kernel's roofline). The "cw" lines restrict the column to a window of cw
// columns (cw x N x 16 bytes: 82 MB at cw = 256, Infinity-Cache resident;
// 20 MB at 64; 5 MB at 16): the random-read rate a column-block pass of the
// network kernel would see.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

template <int U, typename T>
__global__ void gather(const T* __restrict__ a, int64_t n, int iters, double* out, uint32_t cw) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  double acc = 0.0;
  for (int it = 0; it < iters; ++it) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t h1 = hash32(tid * 7919u + (uint32_t)(it * U + u) * 104729u);
      const uint32_t h2 = hash32(h1 ^ 0x9E3779B9u);
      const int64_t r = h1 % (uint32_t)n, c = h2 % cw;
      v[u] = a[r + c * n];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (sizeof(T) == 16) acc += ((const double*)&v[u])[0] + ((const double*)&v[u])[1];
      else acc += (double)v[u];
    }
  }
  if (acc == 1234.5) out[tid] = acc;
}

template <int U, typename T>
void run(const void* buf, int64_t n, int blocks, int threads, int iters, double* out, const char* name,
         uint32_t cw = 0) {
  if (cw == 0) cw = (uint32_t)n;
  hipLaunchKernelGGL((gather<U, T>), dim3(blocks), dim3(threads), 0, 0, (const T*)buf, n, iters, out, cw);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((gather<U, T>), dim3(blocks), dim3(threads), 0, 0, (const T*)buf, n, iters, out, cw);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double reads = (double)blocks * threads * iters * U;
  printf("%-8s U=%2d blocks=%5d x %4d cw=%6u: %.3f ms  %.2f G reads/s  %.1f GB/s useful\n", name, U, blocks,
         threads, cw, ms, reads / (ms * 1e-3) / 1e9, reads * sizeof(T) / (ms * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
  // N = 20,000 (C3/C4: 6.4 GB) by default; 40,000 for C5's 25.6 GB footprint
  const int64_t n = argc > 1 ? atoll(argv[1]) : 20000;
  printf("N = %lld (%.1f GB interleaved)\n", (long long)n, (double)(n * n) * 16 / 1e9);
  void* buf = nullptr;
  if (hipMalloc(&buf, (size_t)(n * n) * 16) != hipSuccess) return 1;
  hipMemset(buf, 0, (size_t)(n * n) * 16);
  double* out;
  hipMalloc(&out, sizeof(double) * (1 << 24));
  // 256 CUs x 8 blocks x 256 threads
  run<4, double2>(buf, n, 2048, 256, 64, out, "16B");
  run<8, double2>(buf, n, 2048, 256, 32, out, "16B");
  run<16, double2>(buf, n, 2048, 256, 16, out, "16B");
  run<8, double2>(buf, n, 4096, 256, 16, out, "16B");
  run<8, double2>(buf, n, 1024, 256, 64, out, "16B");
  run<8, double>(buf, n, 2048, 256, 32, out, "8B");
  run<16, double>(buf, n, 2048, 256, 16, out, "8B");
  // one 512-thread block per CU, 4 in flight (the fused profile kernel's budget)
  run<4, double2>(buf, n, 256, 512, 64, out, "16B/1wg");
  run<8, double2>(buf, n, 256, 512, 32, out, "16B/1wg");
  // fewer workgroups: the parallelism of a launch tail of large modules
  // (C5's k >= 1,000 items run one or two workgroups per CU)
  run<7, double2>(buf, n, 512, 256, 64, out, "16B/2wg");
  run<7, double2>(buf, n, 256, 256, 128, out, "16B/1wg4");
  run<7, double2>(buf, n, 256, 128, 128, out, "16B/1wg2");
  for (uint32_t cw : {1024u, 512u, 256u, 128u, 64u, 16u}) run<8, double2>(buf, n, 2048, 256, 32, out, "16B", cw);
  return 0;
}
