// Keyed pseudo-random permutation of the null pool, shared by host and device.
//
// Replaces the per-permutation `nullIdx = arma::shuffle(nullIdx)` of the
// reference (src/permutations.cpp:63, src/permutationsNoData.cpp:58). A
// permutation p is the bijection pi_p of [0, n_null) given by an 8-round
// balanced Feistel network over 2h bits (2^(2h) >= n_null) with cycle walking,
// keyed by splitmix64(seed, p). Module node c at null-pool position q_c draws
// test index nullIdx[pi_p(q_c)] (GetRandomIdx, src/utils.cpp:193-199), so the
// module sets of one permutation are disjoint exactly as in the reference, and
// a permutation's index sets depend only on (seed, p): identical on 1..8 GPUs.
// oracle/prp.py restates this file for the parity tests.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define NR_HD __host__ __device__ __forceinline__
#else
#define NR_HD inline
#endif

#define NR_PRP_ROUNDS 8

struct nr_prp_key {
  uint32_t k[NR_PRP_ROUNDS];
  uint32_t h;     // half width in bits
  uint32_t mask;  // (1 << h) - 1
  uint32_t n;     // domain size
};

NR_HD uint64_t nr_mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

NR_HD uint32_t nr_lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

NR_HD uint32_t nr_prp_half_bits(uint32_t n) {
  uint32_t bits = 2;
  while ((1ull << bits) < (uint64_t)n) ++bits;
  bits += bits & 1u;
  return bits / 2;
}

NR_HD nr_prp_key nr_prp_make_key(uint64_t seed, uint64_t perm, uint32_t n) {
  nr_prp_key key;
  const uint64_t base = nr_mix64(nr_mix64(seed) ^ perm);
  for (int r = 0; r < NR_PRP_ROUNDS; ++r)
    key.k[r] = (uint32_t)(nr_mix64(base + (uint64_t)r) >> 32);
  key.h = nr_prp_half_bits(n);
  key.mask = (1u << key.h) - 1u;
  key.n = n;
  return key;
}

NR_HD uint32_t nr_prp_encrypt(const nr_prp_key& key, uint32_t x) {
  uint32_t l = x >> key.h, r = x & key.mask;
#pragma unroll
  for (int i = 0; i < NR_PRP_ROUNDS; ++i) {
    const uint32_t f = nr_lowbias32(r ^ key.k[i]) & key.mask;
    const uint32_t t = l ^ f;
    l = r;
    r = t;
  }
  return (l << key.h) | r;
}

// pi_p(x) for x in [0, n): cycle-walk the Feistel permutation of [0, 2^2h).
NR_HD uint32_t nr_prp_permute(const nr_prp_key& key, uint32_t x) {
  uint32_t y = nr_prp_encrypt(key, x);
  while (y >= key.n) y = nr_prp_encrypt(key, y);
  return y;
}
