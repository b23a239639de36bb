"""Offline study of the Lanczos convergence schedule of the profile kernel on
C3-like null items (random gene sets of the synthetic coexpression data).
Prints, per policy, the mean number of Lanczos steps (matvecs) and of
tridiagonal checks per item. Not part of the product; CPU only."""
import sys
import numpy as np
sys.path.insert(0, ".")
from netrep_amd import synthetic as syn

rng = np.random.default_rng(1)
n_nodes, S = 20000, 500
sizes = np.round(np.linspace(30, 300, 50)).astype(int)
lay = syn.make_layout(n_nodes, sizes, 7)
x = syn._gen_numpy(lay, S, np.random.default_rng(3), set(lay.modules))
x = (x - x.mean(0)) / x.std(0, ddof=1)

def lowbias32(h):
    h = np.uint32(h)
    h ^= h >> np.uint32(16); h = np.uint32((int(h) * 0x7FEB352D) & 0xFFFFFFFF)
    h ^= h >> np.uint32(15); h = np.uint32((int(h) * 0x846CA68B) & 0xFFFFFFFF)
    h ^= h >> np.uint32(16); return h

def start(k):
    v = np.array([1.0 + 0.01 * ((int(lowbias32((c * 0x9E3779B9 + 0x1234567) & 0xFFFFFFFF)) & 0xFFFF) / 65536.0 - 0.5) for c in range(k)])
    return v / np.linalg.norm(v)

def curve(G, mmax=160):
    k = G.shape[0]
    Q = np.zeros((k, mmax + 1)); q = start(k); Q[:, 0] = q
    al, be, res, th = [], [], [], []
    qp = np.zeros(k); b = 0.0
    for j in range(min(k, mmax)):
        w = G @ q - b * qp
        a = q @ w; w -= a * q
        w -= Q[:, :j + 1] @ (Q[:, :j + 1].T @ w)     # full reorth (the kernel's partial one is equivalent here)
        b = np.linalg.norm(w); al.append(a); be.append(b)
        T = np.diag(al) + np.diag(be[:-1], 1) + np.diag(be[:-1], -1)
        ev, evec = np.linalg.eigh(T)
        th.append(ev[-1]); res.append(b * abs(evec[-1, -1]))
        if res[-1] <= 1e-16 * ev[-1] or b < 1e-300:
            break
        qp = q; q = w / b; Q[:, j + 1] = q
    return np.array(res), np.array(th)

items = []
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 150):
    k = int(rng.choice(sizes))
    idx = rng.choice(n_nodes, k, replace=False)
    xs = x[:, idx]
    res, th = curve(xs.T @ xs)
    items.append((k, res, th))

TOL = 5e-15
def first_conv(res, th):
    ok = np.nonzero(res <= TOL * th)[0]
    return ok[0] + 1 if ok.size else len(res)

def policy_fixed(res, th, first=16, every=8):
    n = len(res); j = min(first, n); checks = 0
    while True:
        checks += 1
        if res[j - 1] <= TOL * th[j - 1] or j >= n:
            return j, checks
        j = min(j + every, n)

def policy_predict(res, th, first=16, every=8, lo=1, hi=8, slack=1.0):
    n = len(res); j = min(first, n); checks = 0; prev = None
    while True:
        checks += 1
        r = res[j - 1]; tol = TOL * th[j - 1]
        if r <= tol or j >= n:
            return j, checks
        step = every
        if prev is not None and prev[1] > r > 0:
            rho = (r / prev[1]) ** (1.0 / (j - prev[0]))
            step = int(np.ceil(slack * np.log(tol / r) / np.log(rho)))
            step = max(lo, min(hi, step))
        prev = (j, r)
        j = min(j + step, n)

need = np.array([first_conv(r, t) for _, r, t in items])
print("ideal steps", need.mean(), "max", need.max())
for name, f in [("fixed16/8", lambda r, t: policy_fixed(r, t)),
                ("fixed12/4", lambda r, t: policy_fixed(r, t, 12, 4)),
                ("pred16/8", lambda r, t: policy_predict(r, t)),
                ("pred12/8", lambda r, t: policy_predict(r, t, 12)),
                ("pred16/8 hi12", lambda r, t: policy_predict(r, t, 16, 8, 1, 12)),
                ("pred12/6 s.9", lambda r, t: policy_predict(r, t, 12, 6, 1, 12, 0.9))]:
    o = np.array([f(r, t) for _, r, t in items])
    print(f"{name:14s} steps {o[:,0].mean():6.2f}  checks {o[:,1].mean():5.2f}")
