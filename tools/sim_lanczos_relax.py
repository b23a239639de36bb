"""Offline study of relaxed-precision Lanczos on C3-like null items (random
gene sets of the synthetic coexpression data): fp64 matvecs until the Ritz
residual drops below T * theta, then matvecs with fl32(G) and no
reorthogonalisation. Prints, per threshold T, the mean number of steps, of
fp32 steps, the Gram pass-equivalents (an fp32 pass = half a pass) and the
worst / median distance of the final Ritz vector from LAPACK's eigenvector.
Backs the relaxed phase of the profile kernel (kernels.hip lanczos_ritz,
T = 1e-7). Not part of the product; CPU only.

  python tools/sim_lanczos_relax.py [items]
"""
import sys
import numpy as np

sys.path.insert(0, ".")
from netrep_amd import synthetic as syn  # noqa: E402

n_nodes, S = 20000, 500
sizes = np.round(np.linspace(30, 300, 50)).astype(int)
lay = syn.make_layout(n_nodes, sizes, 7)
x = syn._gen_numpy(lay, S, np.random.default_rng(3), set(lay.modules))
x = (x - x.mean(0)) / x.std(0, ddof=1)


def lanczos_relax(G, G32, q0, tol, T, mmax=200):
    k = G.shape[0]
    Q = np.zeros((k, mmax + 1))
    q = q0 / np.linalg.norm(q0)
    Q[:, 0] = q
    al, be = [], []
    qp = np.zeros(k)
    b, r, n32 = 0.0, 1.0, 0
    for j in range(min(k, mmax)):
        use32 = r <= T
        n32 += use32
        w = (G32 if use32 else G) @ q - b * qp
        a = q @ w
        w -= a * q
        if not use32:
            w -= Q[:, :j + 1] @ (Q[:, :j + 1].T @ w)
        b = np.linalg.norm(w)
        al.append(a)
        be.append(b)
        ev, evec = np.linalg.eigh(np.diag(al) + np.diag(be[:-1], 1) + np.diag(be[:-1], -1))
        y = evec[:, -1]
        r = b * abs(y[-1]) / ev[-1]
        if r <= tol or b < 1e-300 or j + 1 == k:
            return j + 1, n32, Q[:, :j + 1] @ y
        qp, q = q, w / b
        Q[:, j + 1] = q
    return mmax, n32, Q[:, :mmax] @ y


def main():
    rng = np.random.default_rng(11)
    n_items = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    res = {}
    for _ in range(n_items):
        k = int(rng.choice(sizes))
        xs = x[:, rng.choice(n_nodes, k, replace=False)]
        G = xs.T @ xs
        G32 = G.astype(np.float32).astype(np.float64)
        vt = np.linalg.eigh(G)[1][:, -1]
        q0 = np.ones(k)
        for T in (0.0, 1e-9, 1e-8, 1e-7, 1e-6):
            n, n32, v = lanczos_relax(G, G32, q0, 5e-15, T)
            v /= np.linalg.norm(v)
            err = min(np.linalg.norm(v - vt), np.linalg.norm(v + vt))
            res.setdefault(T, []).append((n, n32, n - 0.5 * n32, err))
    for T in sorted(res):
        a = np.array(res[T])
        print(f"T={T:7.0e} steps {a[:, 0].mean():6.2f} fp32 {a[:, 1].mean():6.2f} "
              f"pass-eq {a[:, 2].mean():6.2f} worst err {a[:, 3].max():.2e} median {np.median(a[:, 3]):.2e}")


if __name__ == "__main__":
    main()
