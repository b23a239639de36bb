import sys, numpy as np
exec(open('tools/sim_lanczos_start_base.py').read().split("res = {}")[0])
res = {}
for it in range(int(sys.argv[1])):
    k = int(rng.choice(sizes)); idx = rng.choice(n_nodes, k, replace=False)
    xs = x[:, idx]; G = xs.T @ xs
    cn = np.sum(G*G,0); order = np.argsort(-cn)
    c0 = order[0]
    top3 = G[:, c0].copy()
    for c in order[1:3]: top3 += np.sign(G[c0, c]) * G[:, c]
    starts = {"ones": np.ones(k), "maxcol": G[:, c0], "top3": top3,
              "e_c": np.eye(k)[c0], "ones+maxcol": np.ones(k)/np.sqrt(k) + G[:, c0]/np.linalg.norm(G[:, c0]),
              "signcol": np.sign(G[:, c0])}
    for n, v in starts.items(): res.setdefault(n, []).append(steps(G, v))
b = np.array(res["ones"])
for n, v in res.items():
    v = np.array(v); d = v - b
    print(f"{n:12s} mean {v.mean():6.2f} max {v.max()} diff {d.mean():+.2f} +- {d.std()/np.sqrt(len(d)):.2f}")
