"""Offline study: a middle storage tier for the table kernel's Lanczos matvecs.

Tiers (bytes per packed Gram entry per pass):
  fp64 (8)                               while residual > T6 * theta
  fp32 + int16 correction (6)            while residual > 1e-7 * theta
  fp32 (4)                               after
The correction is c = round((G - G32) / ulp(G32) * 2^15) (|c| <= 2^14), so
G32 + c * ulp(G32) * 2^-15 carries ~2^-39 relative precision per entry.

Each switch happens at a Ritz check (the kernel only learns the residual
there); checks run at step 16, then where the residual's decay predicts
convergence (at most 8 on), plus, while a switch is pending, where the decay
predicts the crossing of its threshold (kernels.hip lanczos_ritz).

The Lanczos runs are emulated exactly in numpy with the tiered matvecs, full
reorthogonalisation, and the final Ritz vector compared with the fp64 run's
(and with eigh): a tier is safe if it leaves the eigenvector error at the
fp64 run's level. C3 null items (random gene sets of the synthetic
coexpression data). CPU only; not part of the product.

  python tools/sim_lanczos_tier6.py [items]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from netrep_amd import synthetic as syn  # noqa: E402

n_nodes, S = 20000, 500
sizes = np.round(np.linspace(30, 300, 50)).astype(int)
TOL = 5e-15


def tier_mats(G):
    G32 = G.astype(np.float32)
    g32 = G32.astype(np.float64)
    _, e = np.frexp(G32)                       # G32 = m 2^e, m in [0.5, 1)
    ulp = np.ldexp(1.0, e.astype(np.int64) - 24)
    c = np.rint((G - g32) / ulp * 32768.0)
    assert np.abs(c).max() <= 16384
    g6 = g32 + c * ulp / 32768.0
    return g32, g6


def run(G, g32, g6, t6, t7=1e-7, first=16, mmax=200, cross_checks=True):
    """Lanczos with tiered matvecs; returns (steps, bytes/entry, Ritz vector, theta)."""
    k = G.shape[0]
    c = int(np.argmax((g32 * g32).sum(0)))
    q = G[:, c].copy()
    q /= np.linalg.norm(q)
    Q = np.zeros((k, mmax + 1))
    Q[:, 0] = q
    al, be = [], []
    qp = np.zeros(k)
    b = 0.0
    tier = 0 if t6 is not None else 1  # 0 fp64, 1 six-byte, 2 fp32
    if t6 is None:
        tier = 0
    nbytes = 0
    next_check = first
    prev = (0, None)
    for j in range(min(k, mmax)):
        M = (G, g6, g32)[tier]
        nbytes += (8, 6, 4)[tier]
        w = M @ q - b * qp
        a = q @ w
        w -= a * q
        w -= Q[:, :j + 1] @ (Q[:, :j + 1].T @ w)
        b = np.linalg.norm(w)
        al.append(a)
        be.append(b)
        last = j + 1 == min(k, mmax) or b < 1e-300
        if j + 1 == next_check or last:
            T = np.diag(al) + np.diag(be[:-1], 1) + np.diag(be[:-1], -1)
            ev, evec = np.linalg.eigh(T)
            theta = ev[-1]
            r = b * abs(evec[-1, -1]) / abs(theta)
            if r <= TOL or last:
                v = Q[:, :j + 1] @ evec[:, -1]
                return j + 1, nbytes, v / np.linalg.norm(v), theta
            if tier == 0 and t6 is not None and r <= t6:
                tier = 1
            if tier <= 1 and r <= t7:
                tier = 2
            if t6 is None and tier == 0 and r <= t7:
                tier = 2
            p_j, p_r = prev
            rate = np.log(r / p_r) / (j + 1 - p_j) if p_r is not None and p_r > r > 0 else np.log(r) / (j + 1)
            step = 8
            if p_r is not None and p_r > r > 0:
                step = int(max(1, min(8, np.ceil(np.log(TOL / r) / rate))))
            if cross_checks and rate < 0:
                pend = [t for t, need in ((t6, tier == 0 and t6 is not None), (t7, tier < 2)) if need]
                for thr in pend:
                    cr = np.ceil(np.log(thr / r) / rate)
                    if 1 <= cr < step:
                        step = int(cr)
            prev = (j + 1, r)
            next_check = j + 1 + step
        qp, q = q, w / b
        Q[:, j + 1] = q
    raise RuntimeError("no convergence")


def main():
    n_items = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    lay = syn.make_layout(n_nodes, sizes, 7)
    x = syn._gen_numpy(lay, S, np.random.default_rng(3), set(lay.modules))
    x = (x - x.mean(0)) / x.std(0, ddof=1)
    rng = np.random.default_rng(11)
    schemes = [("two tiers (fp64, fp32 from 1e-7)", None), ("three tiers, 6-byte from 1e-2", 1e-2),
               ("three tiers, 6-byte from 3e-3", 3e-3), ("three tiers, 6-byte from 1e-3", 1e-3),
               ("three tiers, 6-byte from 1e-4", 1e-4)]
    acc = {n: [] for n, _ in schemes}
    wts = []
    for it in range(n_items):
        k = int(rng.choice(sizes))
        xs = x[:, rng.choice(n_nodes, k, replace=False)]
        # the Gram [X 1]^T [X 1] the kernel runs on
        xa = np.hstack([xs, np.ones((S, 1))])
        G = xa.T @ xa
        g32, g6 = tier_mats(G)
        ev, evec = np.linalg.eigh(G)
        u = evec[:, -1]
        gap = (ev[-1] - ev[-2]) / ev[-1]
        wts.append(float(k * k))
        for name, t6 in schemes:
            steps, nb, v, th = run(G, g32, g6, t6)
            err = np.linalg.norm(v - np.sign(v @ u) * u)
            acc[name].append((steps, nb, err, abs(th - ev[-1]) / ev[-1], gap))
    w = np.array(wts) / np.sum(wts)
    base = np.array(acc[schemes[0][0]])
    for name, _ in schemes:
        a = np.array(acc[name])
        print(f"{name:36s} steps {np.sum(a[:, 0] * w):6.2f}  bytes/entry {np.sum(a[:, 1] * w):7.2f}  "
              f"vec err max {a[:, 2].max():.2e} (fp64-tier run {base[:, 2].max():.2e}), "
              f"max ratio to it {np.max(a[:, 2] / np.maximum(base[:, 2], 1e-300)):.2f}, "
              f"theta err max {a[:, 3].max():.1e}")
    print(f"relative gaps: min {base[:, 4].min():.2e}, median {np.median(base[:, 4]):.2e}")


if __name__ == "__main__":
    main()
