"""Offline study of a warm-started Lanczos for C3-like null items: an all-fp32
Lanczos run (matrix fl32(G)) to residual T1 * theta, whose Ritz vector starts
the kernel's relaxed fp64 run (fp64 matvecs until 1e-7 theta, then fp32) to
5e-15 theta; against the kernel's scheme from the start column G e_c*.
Prints the mean steps, fp32 steps, Gram pass-equivalents (an fp32 pass = half
a pass) and the worst / median eigenvector error. Result (40 items): 25.6 ->
21.2 pass-equivalents at T1 = 1e-6 but 32.2 -> 39.1 steps, which by the
kernel's phase split nets about -3%: not built.
Not part of the product; CPU only.

  python tools/sim_lanczos_warm.py [items]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import sim_lanczos_relax as R  # noqa: E402

def main():
    rng = np.random.default_rng(11)
    n_items = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    res = {}
    for _ in range(n_items):
        k = int(rng.choice(R.sizes))
        xs = R.x[:, rng.choice(R.n_nodes, k, replace=False)]
        G = xs.T @ xs
        G32 = G.astype(np.float32).astype(np.float64)
        vt = np.linalg.eigh(G)[1][:, -1]
        c = np.argmax((G * G).sum(0))
        q0 = G[:, c].copy()
        n, n32, v = R.lanczos_relax(G, G32, q0, 5e-15, 1e-7)
        v /= np.linalg.norm(v)
        err = min(np.linalg.norm(v - vt), np.linalg.norm(v + vt))
        res.setdefault('base', []).append((n, n32, n - 0.5 * n32, err))
        for T1 in (1e-3, 1e-4, 1e-5, 1e-6):
            n1, _, v1 = R.lanczos_relax(G32, G32, q0, T1, 0.0)   # all-fp32 phase 1 (matrix G32)
            n2, n32b, v = R.lanczos_relax(G, G32, v1, 5e-15, 1e-7)
            v /= np.linalg.norm(v)
            err = min(np.linalg.norm(v - vt), np.linalg.norm(v + vt))
            res.setdefault(T1, []).append((n1 + n2, n1 + n32b, n1 + n2 - 0.5 * (n1 + n32b), err))
    for T in res:
        a = np.array(res[T])
        print(f"{T!s:6} steps {a[:, 0].mean():6.2f} fp32 {a[:, 1].mean():6.2f} pass-eq {a[:, 2].mean():6.2f} worst err {a[:, 3].max():.2e} median {np.median(a[:, 3]):.2e}")


if __name__ == "__main__":
    main()
