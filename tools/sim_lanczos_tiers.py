"""Offline study: when does the table kernel's Lanczos run switch its matvecs
from the fp64 Gram to the fp32 copy, against when it could?

The kernel (kernels.hip lanczos_ritz) switches at the first Ritz check whose
residual is <= 1e-7 theta; checks run at step 16 and then where the
residual's geometric decay predicts convergence (at most 8 steps on). This
study takes C3 null items (random gene sets of the synthetic coexpression
data, start vector G e_c* as start_column), computes the fp64 residual curve
with full reorthogonalisation, and counts per item:
  - steps, fp64 steps and Gram pass-equivalents (fp32 pass = 1/2) under the
    kernel's schedule;
  - the same with the switch at the exact crossing of 1e-7 theta (ideal);
  - a three-tier scheme: fp64, then fp32 + an fp16 correction (6 B/entry,
    ~2^-35 relative) once r <= T6 theta, then fp32 once r <= 1e-7 theta.
Weights by each item's Gram bytes (k^2), as the launch's traffic is. CPU
only; not part of the product.

  python tools/sim_lanczos_tiers.py [items]
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
TOL = 5e-15


def curve(G, mmax=160):
    k = G.shape[0]
    c = int(np.argmax((G * G).sum(0)))
    q = G[:, c].copy()
    q /= np.linalg.norm(q)
    Q = np.zeros((k, mmax + 1))
    Q[:, 0] = q
    al, be, res = [], [], []
    qp = np.zeros(k)
    b = 0.0
    for j in range(min(k, mmax)):
        w = G @ q - b * qp
        a = q @ w
        w -= a * q
        w -= Q[:, :j + 1] @ (Q[:, :j + 1].T @ w)
        b = np.linalg.norm(w)
        al.append(a)
        be.append(b)
        ev, evec = np.linalg.eigh(np.diag(al) + np.diag(be[:-1], 1) + np.diag(be[:-1], -1))
        res.append(b * abs(evec[-1, -1]) / ev[-1])
        if res[-1] <= TOL or b < 1e-300:
            break
        qp, q = q, w / b
        Q[:, j + 1] = q
    return np.array(res)


def schedule(res, first=16):
    """The kernel's check points: (step, residual) of each check."""
    n = len(res)
    j = min(first, n)
    prev = None
    out = []
    while True:
        r = res[j - 1]
        out.append(j)
        if r <= TOL or j >= n:
            return out
        step = 8
        if prev is not None and prev[1] > r > 0:
            rate = np.log(r / prev[1]) / (j - prev[0])
            need = np.ceil(np.log(TOL / r) / rate)
            step = int(max(1, min(8, need)))
        prev = (j, r)
        j = min(j + step, n)


def main():
    rng = np.random.default_rng(11)
    n_items = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    rows = []
    for _ in range(n_items):
        k = int(rng.choice(sizes))
        xs = x[:, rng.choice(n_nodes, k, replace=False)]
        res = curve(xs.T @ xs)
        n = len(res)
        checks = schedule(res)
        # kernel: the switch happens after the first check with r <= 1e-7; steps
        # after that check use fp32 (the matvec of step j uses q_j, decided by
        # the checks up to j)
        sw = next((c for c in checks if res[c - 1] <= 1e-7), n)
        cross = next((j + 1 for j in range(n) if res[j] <= 1e-7), n)
        rows.append((k, n, sw, cross, res))
    w = np.array([r[0] ** 2 for r in rows], dtype=float)
    w /= w.sum()

    def report(name, f):
        v = np.array([f(r) for r in rows])
        print(f"{name:44s} bytes/entry (weighted) {np.sum(v * w):7.2f}   mean {v.mean():7.2f}")

    steps = np.array([r[1] for r in rows])
    print(f"items {len(rows)}: steps mean {steps.mean():.2f} (weighted {np.sum(steps * w):.2f})")
    sw = np.array([r[2] for r in rows])
    cr = np.array([r[3] for r in rows])
    print(f"fp64 steps: kernel schedule {np.sum(sw * w):.2f}, ideal crossing {np.sum(cr * w):.2f} (weighted)")
    report("kernel: fp64 until the check sees 1e-7", lambda r: 8 * r[2] + 4 * (r[1] - r[2]))
    report("ideal: fp64 until the crossing of 1e-7", lambda r: 8 * r[3] + 4 * (r[1] - r[3]))
    for t6 in (1e-3, 1e-4, 1e-5):
        def tier(r, t6=t6):
            n, c7 = r[1], r[3]
            c6 = next((j + 1 for j in range(n) if r[4][j] <= t6), n)
            c6 = min(c6, c7)
            return 8 * c6 + 6 * (c7 - c6) + 4 * (n - c7)
        report(f"three tiers, fp32+fp16 from {t6:.0e}, fp32 from 1e-7", tier)
    # residual at each step, the weighted median item
    for j in (4, 8, 12, 16, 20, 24, 28, 32):
        v = [r[4][j - 1] if j <= r[1] else 0.0 for r in rows]
        print(f"step {j:2d}: residual/theta median {np.median(v):.1e}  90th pct {np.quantile(v, 0.9):.1e}")


if __name__ == "__main__" and "--policies" not in sys.argv:
    main()


def policies(rows):
    """Switch policies for the fp64 -> fp32 step (and the fp64 -> 6-byte tier):
    extra checks at the predicted crossing, or a switch by extrapolation."""
    w = np.array([r[0] ** 2 for r in rows], dtype=float)
    w /= w.sum()

    def sim(r, first=16, extra=True, margin=None, t6=None):
        k, n, _, _, res = r
        j = min(first, n)
        prev = (0, 1.0)
        checks = 0
        sw7 = None
        sw6 = None if t6 else 0
        while True:
            rj = res[j - 1]
            checks += 1
            if sw7 is None and rj <= 1e-7:
                sw7 = j
            if t6 and sw6 is None and rj <= t6:
                sw6 = j
            if rj <= TOL or j >= n:
                break
            rate = np.log(rj / prev[1]) / (j - prev[0]) if prev[1] > rj > 0 else np.log(0.5)
            need = int(max(1, min(8, np.ceil(np.log(TOL / rj) / rate))))
            nxt = j + need
            # extrapolated crossings (margin: switch without a check)
            for thr, name in ((1e-7, 7), (t6, 6)):
                if not thr:
                    continue
                cur = sw7 if name == 7 else sw6
                if cur is not None:
                    continue
                steps = int(np.ceil(np.log(thr / rj) / rate))
                if margin is not None:
                    steps_m = int(np.ceil(np.log(thr / margin / rj) / rate))
                    at = j + max(1, steps_m)
                    if at < nxt:   # switch there without a check (the prediction's margin)
                        if name == 7:
                            sw7 = at
                        else:
                            sw6 = at
                elif extra and j + max(1, steps) < nxt:
                    nxt = j + max(1, steps)
            prev = (j, rj)
            j = min(nxt, n)
        sw7 = n if sw7 is None else min(sw7, n)
        if t6:
            sw6 = sw7 if sw6 is None else min(sw6, sw7)
            b = 8 * sw6 + 6 * (sw7 - sw6) + 4 * (n - sw7)
        else:
            b = 8 * sw7 + 4 * (n - sw7)
        # safety: the residual when each switch happened (must be <= its threshold)
        worst7 = res[sw7 - 1] / 1e-7 if sw7 < n else 0.0
        return b, checks, worst7

    for name, kw in [("kernel (16, predicted)", dict(extra=False)),
                     ("+ check at predicted 1e-7", dict(extra=True)),
                     ("first 12 + check at predicted", dict(first=12, extra=True)),
                     ("switch by extrapolation, margin 10", dict(extra=False, margin=10.0)),
                     ("switch by extrapolation, margin 100", dict(extra=False, margin=100.0)),
                     ("3 tiers t6=1e-4, checks at crossings", dict(extra=True, t6=1e-4)),
                     ("3 tiers t6=1e-4, first 8, checks", dict(first=8, extra=True, t6=1e-4)),
                     ("3 tiers t6=1e-4, extrapolation m10", dict(extra=False, margin=10.0, t6=1e-4))]:
        v = np.array([sim(r, **kw) for r in rows])
        print(f"{name:40s} bytes/entry {np.sum(v[:, 0] * w):7.2f}  checks {v[:, 1].mean():5.2f}  "
              f"worst r/1e-7 at the switch {v[:, 2].max():.2f}")


if __name__ == "__main__" and "--policies" in sys.argv:
    rng = np.random.default_rng(11)
    rows = []
    for _ in range(int(sys.argv[1])):
        k = int(rng.choice(sizes))
        xs = x[:, rng.choice(n_nodes, k, replace=False)]
        res = curve(xs.T @ xs)
        rows.append((k, len(res), 0, 0, res))
    policies(rows)
