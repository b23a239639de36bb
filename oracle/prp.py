"""Counter-based keyed permutation of the null pool (numpy restatement).

TEST INFRASTRUCTURE ONLY -- the device evaluates the same function in
``netrep_amd/csrc/prp.h``; this file exists so the oracle can derive the
identical index sets and check them bit for bit.

The reference draws one uniform shuffle of the null pool per permutation
with ``nullIdx = arma::shuffle(nullIdx)`` (src/permutations.cpp:63,
src/permutationsNoData.cpp:58) from R's RNG, whose stream is not
reproducible across thread counts. The MI355X engine
replaces the shuffle with a keyed pseudo-random permutation pi_p of
[0, n_null), keyed by (seed, global permutation index), so each module node
only needs pi_p at its own null-pool position and results are identical on
1, 2, 4 or 8 GPUs:

    idx[c] = nullIdx[pi_p(q_c)]          (GetRandomIdx, src/utils.cpp:193-199)

pi_p is an 8-round balanced Feistel network over 2*h bits (2^(2h) >= n)
with cycle walking back into [0, n). Round keys come from splitmix64 of
(seed, p); the round function is the "lowbias32" 32-bit mixer.
"""
from __future__ import annotations

import numpy as np

NROUNDS = 8
_M64 = (1 << 64) - 1


def _mix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def half_bits(n: int) -> int:
    bits = 2
    while (1 << bits) < n:
        bits += 1
    bits += bits & 1
    return bits // 2


def round_keys(seed: int, perm: int) -> np.ndarray:
    base = _mix64((_mix64(seed & _M64) ^ (perm & _M64)) & _M64)
    return np.array([_mix64((base + r) & _M64) >> 32 for r in range(NROUNDS)],
                    dtype=np.uint32)


def _lowbias32(x: np.ndarray) -> np.ndarray:
    x = x ^ (x >> np.uint32(16))
    x = x * np.uint32(0x7FEB352D)
    x = x ^ (x >> np.uint32(15))
    x = x * np.uint32(0x846CA68B)
    x = x ^ (x >> np.uint32(16))
    return x


def _encrypt(x: np.ndarray, keys: np.ndarray, h: int) -> np.ndarray:
    mask = np.uint32((1 << h) - 1)
    left = x >> np.uint32(h)
    right = x & mask
    for r in range(NROUNDS):
        f = _lowbias32(right ^ keys[r]) & mask
        left, right = right, left ^ f
    return (left << np.uint32(h)) | right


def permute(positions, n: int, seed: int, perm: int) -> np.ndarray:
    """pi_perm(positions) for positions in [0, n)."""
    with np.errstate(over="ignore"):
        x = np.asarray(positions, dtype=np.uint32).copy()
        keys = round_keys(seed, perm)
        h = half_bits(n)
        y = _encrypt(x, keys, h)
        out_of_range = y >= n
        while out_of_range.any():
            y[out_of_range] = _encrypt(y[out_of_range], keys, h)
            out_of_range = y >= n
    return y


def permutation_table(n: int, seed: int, perm_begin: int, perm_end: int) -> np.ndarray:
    """Full pi_p arrays, shape (perm_end - perm_begin, n), dtype uint32."""
    pos = np.arange(n, dtype=np.uint32)
    return np.stack([permute(pos, n, seed, p) for p in range(perm_begin, perm_end)])
