"""Offline study: passes over the Gram (block steps) that block Krylov needs
for the top eigenpair of C3 null items, against single-vector Lanczos.

Block Lanczos with full block reorthogonalisation and Rayleigh-Ritz on the
whole basis; stop when the top Ritz pair's residual |G v - theta v| is at most
TOL * theta (the engine's stop rule). The start block is
the b Gram columns of largest norm (column c* first, as the engine's start).

usage: python tools/sim_block_krylov.py N_ITEMS [b ...]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from netrep_amd import synthetic as syn  # noqa: E402

TOL = 5e-15
rng = np.random.default_rng(1)
n_nodes, S = 20000, 500
sizes = np.round(np.linspace(30, 300, 50)).astype(int)
lay = syn.make_layout(n_nodes, sizes, 7)
x = syn._gen_numpy(lay, S, np.random.default_rng(3), set(lay.modules))
x = (x - x.mean(0)) / x.std(0, ddof=1)


def block_steps(G, b, max_pass=200):
    k = G.shape[0]
    cn = np.sum(G * G, 0)
    order = np.argsort(-cn)
    V = G[:, order[:b]].copy()
    Q, _ = np.linalg.qr(V)
    basis = [Q]
    for p in range(1, max_pass + 1):
        W = G @ basis[-1]  # one pass over G for b vectors
        B = np.hstack(basis)
        # Rayleigh-Ritz over the basis (the block tridiagonal T in exact arithmetic)
        T = B.T @ (G @ B)
        ev, U = np.linalg.eigh(T)
        v = B @ U[:, -1]
        th = ev[-1]
        r = np.linalg.norm(G @ v - th * v)
        if r <= TOL * th or B.shape[1] >= k:
            return p
        W -= B @ (B.T @ W)
        W -= B @ (B.T @ W)
        Qn, R = np.linalg.qr(W)
        keep = np.abs(np.diag(R)) > 1e-10 * th
        if not keep.any():
            return p
        basis.append(Qn[:, keep])
    return max_pass


n_items = int(sys.argv[1]) if len(sys.argv) > 1 else 50
bs = [int(a) for a in sys.argv[2:]] or [1, 2, 4, 8, 16]
res = {b: [] for b in bs}
ks = []
for it in range(n_items):
    k = int(rng.choice(sizes))
    idx = rng.choice(n_nodes, k, replace=False)
    xs = x[:, idx]
    G = xs.T @ xs
    ks.append(k)
    for b in bs:
        res[b].append(block_steps(G, b))
ks = np.array(ks, dtype=float)
w = ks * ks  # a pass costs ~k^2/2 Gram entries
# Bytes per item (round 4): the Gram passes (packed fp64,
# k^2/2 x 8 B each) plus the block recurrence's vector traffic with the
# kernel's partial reorthogonalisation assumed to carry over (every step reads
# the two previous blocks and writes one, k b doubles each; a full basis pass
# -- project and update, 2 reads of the basis -- on 8% of the steps, the
# single-vector kernel's rate: 2.8 per 35 steps). G V on the matrix cores:
# 2 k^2 b flops per pass, as time at the 78.6 TF/s fp64 peak for C3's 256,000
# items per launch. LDS: six k-vectors per block column at k = 320.
base = None
for b in bs:
    v = np.array(res[b], dtype=float)
    gram = np.mean(v * ks * ks / 2 * 8)
    rec = np.mean(v * 3 * ks * b * 8)
    reo = np.mean(0.08 * v * 2 * ks * (b * v / 2) * 8)
    tot = gram + rec + reo
    base = base or tot
    mfma_ms = np.mean(v * 2 * ks * ks * b) * 256000 / 78.6e12 * 1e3
    print(f"b={b:2d}  passes mean {v.mean():6.2f}  max {v.max():4.0f}  k^2-weighted {np.sum(v * w) / w.sum():6.2f}  "
          f"bytes/item: Gram {gram / 1e6:5.2f} MB + recurrence {rec / 1e6:5.2f} + reorth {reo / 1e6:5.2f} "
          f"= {tot / base:4.2f}x b=1;  G.V at MFMA peak {mfma_ms:5.1f} ms/launch;  LDS vectors {6 * 320 * b * 8 / 1024:5.1f} KB")
