"""Driver of tools/probes/eig_probe.hip: C3-shaped packed Grams (20k genes x
500 samples, null items of sizes round(linspace(30, 300, 50))), the CU-resident
Lanczos kernel's theta / v against numpy's eigh, and its time per launch of
C3's 256,000 items (5,120 permutations x 50 modules).

usage: python tools/probes/eig_probe.py [SO] [N_REAL] [N_ITEMS] [REPS]
"""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from netrep_amd import synthetic as syn  # noqa: E402

EKV = 328


def pack(G):
    """kernels.hip pk_at layout of the symmetric kc x kc matrix G."""
    kc = G.shape[0]
    ngr = (kc + 15) // 16
    base = [16 * g * kc - 128 * g * (g - 1) for g in range(ngr + 1)]
    out = np.zeros((base[ngr] + 31) // 32 * 32)
    for g in range(ngr):
        for c in range(16 * g, min(16 * g + 16, kc)):
            for j in range((kc - 16 * g + 63) // 64):
                r0 = 16 * g + 64 * j
                h = min(64, kc - r0)
                rows = np.arange(r0, r0 + h)
                vals = np.where(rows >= c, G[rows, c], 0.0)
                off = base[g] + 1024 * j + (c & 15) * h
                out[off:off + h] = vals
    return out


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else "tools/probes/eig_probe.so"
    n_real = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    n_items = int(sys.argv[3]) if len(sys.argv) > 3 else 256000
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    kmax = int(sys.argv[5]) if len(sys.argv) > 5 else 320
    t0 = time.time()
    n_nodes, S = 20000, 500
    sizes = np.round(np.linspace(30, 300, 50)).astype(int)
    lay = syn.make_layout(n_nodes, sizes, 7)
    sizes = sizes[sizes <= kmax]
    x = syn._gen_numpy(lay, S, np.random.default_rng(3), set(lay.modules))
    x = (x - x.mean(0)) / x.std(0, ddof=1)
    rng = np.random.default_rng(1)
    packs, offs, ks, gs = [], [], [], []
    off = 0
    for it in range(n_real):
        k = int(sizes[it % len(sizes)])  # the C3 size mix, every size equally often
        idx = rng.choice(n_nodes, k, replace=False)
        xs = np.hstack([x[:, idx], np.ones((S, 1))])
        G = xs.T @ xs
        p = pack(G)
        packs.append(p)
        offs.append(off)
        off += p.size
        ks.append(k)
        gs.append(G[:k, :k])
    grams = np.concatenate(packs)
    offs = np.array(offs, dtype=np.int64)
    ks = np.array(ks, dtype=np.int32)
    print(f"generated {n_real} items ({grams.nbytes / 1e6:.0f} MB) in {time.time() - t0:.1f}s", flush=True)
    lib = ctypes.CDLL(so)
    lib.ek_run.restype = ctypes.c_int
    theta = np.zeros(n_real)
    v = np.zeros((n_real, EKV))
    steps = np.zeros(n_real, dtype=np.int32)
    ms = ctypes.c_double(0)
    stamps = np.zeros(16, dtype=np.uint64)
    P = ctypes.c_void_p
    rc = lib.ek_run(grams.ctypes.data_as(P), ctypes.c_int64(grams.size), offs.ctypes.data_as(P),
                    ks.ctypes.data_as(P), ctypes.c_int(n_real), ctypes.c_int(n_items), ctypes.c_int(reps),
                    theta.ctypes.data_as(P), v.ctypes.data_as(P), steps.ctypes.data_as(P), ctypes.byref(ms),
                    stamps.ctypes.data_as(P))
    print("rc", rc)
    if rc:
        sys.exit(rc)
    worst_v, worst_t = 0.0, 0.0
    for i in range(n_real):
        w, U = np.linalg.eigh(gs[i])
        u = U[:, -1]
        k = ks[i]
        vi = v[i, :k]
        if np.dot(u, vi) < 0:
            vi = -vi
        worst_v = max(worst_v, np.abs(vi - u).max() / np.abs(u).max())
        worst_t = max(worst_t, abs(theta[i] - w[-1]) / w[-1])
    print(f"items {n_items} per launch: {ms.value:.2f} ms  ({n_items / 50 / ms.value * 1e3:.0f} C3 perms/s-equivalent)")
    for kk in (30, 96, 165, 234, 300):
        sel = np.abs(ks - kk) <= 4
        if sel.any():
            print(f"  k~{kk}: steps mean {steps[sel].mean():.1f} max {steps[sel].max()}")
    print(f"steps mean {steps.mean():.2f} max {steps.max()}; worst |dv|/|v|max {worst_v:.2e}, |dtheta|/theta {worst_t:.2e}")
    names = ["load", "start", "matvec", "B1", "combine+B2", "update+B3", "omega", "checks", "ritz coef", "ritz vec",
             "reorth", "q update"]
    tot = stamps[:12].sum()
    per_item = {nm: int(stamps[i]) // n_items for i, nm in enumerate(names)}
    print("wave-0 cycles per item:", per_item, "total", int(tot) // n_items)


if __name__ == "__main__":
    main()
