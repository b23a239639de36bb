import sys, numpy as np
sys.path.insert(0, ".")
from netrep_amd import synthetic as syn
rng = np.random.default_rng(1)
n_nodes, S = 20000, 500
sizes = np.round(np.linspace(30, 300, 50)).astype(int)
lay = syn.make_layout(n_nodes, sizes, 7)
x = syn._gen_numpy(lay, S, np.random.default_rng(3), set(lay.modules))
x = (x - x.mean(0)) / x.std(0, ddof=1)
TOL=5e-15
def steps(G, q, mmax=200):
    k = G.shape[0]; q = q/np.linalg.norm(q)
    Q = np.zeros((k, mmax + 1)); Q[:, 0] = q
    al, be = [], []; qp = np.zeros(k); b = 0.0
    for j in range(min(k, mmax)):
        w = G @ q - b * qp
        a = q @ w; w -= a * q
        w -= Q[:, :j + 1] @ (Q[:, :j + 1].T @ w)
        b = np.linalg.norm(w); al.append(a); be.append(b)
        T = np.diag(al) + np.diag(be[:-1], 1) + np.diag(be[:-1], -1)
        ev, evec = np.linalg.eigh(T)
        if b * abs(evec[-1, -1]) <= TOL * ev[-1] or b < 1e-300: return j+1
        qp = q; q = w / b; Q[:, j + 1] = q
    return mmax
res = {}
for it in range(int(sys.argv[1])):
    k = int(rng.choice(sizes)); idx = rng.choice(n_nodes, k, replace=False)
    xs = x[:, idx]; G = xs.T @ xs
    ones = np.ones(k)
    starts = {"ones": ones, "gauss": rng.standard_normal(k), "Gabs1": np.abs(G).sum(1),
              "maxdiagcol": G[:, np.argmax(np.sum(G*G,0))],
              "topsample": xs[np.argmax((xs**2).sum(1))],
              "sketch4": np.linalg.svd(rng.standard_normal((8,S))@xs, full_matrices=False)[2][0]}
    for n, v in starts.items(): res.setdefault(n, []).append(steps(G, v))
for n, v in res.items(): print(n, np.mean(v), np.max(v))
