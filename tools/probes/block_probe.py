"""Driver of tools/probes/block_probe.hip: block Lanczos
b = 16 on the matrix cores for C3-shaped null items (the eig_probe.py items:
20k genes x 500 samples, sizes round(linspace(30, 300, 50))).

Per real item the host runs the offline study's block Lanczos (full
reorthogonalisation, Rayleigh-Ritz, stop at |G v - theta v| <= 5e-15 theta)
from the kernel's start block to get the item's block steps J; the kernel then
runs J steps per item over a C3 launch's 256,000 items (mode 0: no
reorthogonalisation, the lower bound; mode 1: full classical Gram-Schmidt every
step). Prints ms per launch, C3 perms/s-equivalent, the per-phase cycles, and
the top Ritz value of the kernel's block tridiagonal T against eigh(G).

usage: python tools/probes/block_probe.py SO N_REAL N_ITEMS REPS MODE
"""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from netrep_amd import synthetic as syn  # noqa: E402

B, JMAX, TOL = 16, 24, 5e-15


def pack(G):
    """kernels.hip pk_at layout of the symmetric kc x kc matrix G (kc = k here)."""
    kc = G.shape[0]
    ngr = (kc + 15) // 16
    base = [16 * g * kc - 128 * g * (g - 1) for g in range(ngr + 1)]
    out = np.zeros((base[ngr] + 31) // 32 * 32 + 1024)
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


def start_cols(G):
    d = np.diag(G).copy()
    cols = []
    for _ in range(B):
        i = int(np.argmax(d))  # first index of the maximum, as the kernel's tie rule
        cols.append(i)
        d[i] = -1.5
    return cols


def host_steps(G, max_pass=JMAX):
    k = G.shape[0]
    V = G[:, start_cols(G)].copy()
    Q, _ = np.linalg.qr(V)
    basis = [Q]
    for p in range(1, max_pass + 1):
        Bm = np.hstack(basis)
        T = Bm.T @ (G @ Bm)
        ev, U = np.linalg.eigh(T)
        v = Bm @ U[:, -1]
        th = ev[-1]
        if np.linalg.norm(G @ v - th * v) <= TOL * th or Bm.shape[1] >= k:
            return p
        W = G @ basis[-1]
        W -= Bm @ (Bm.T @ W)
        W -= Bm @ (Bm.T @ W)
        Qn, R = np.linalg.qr(W)
        basis.append(Qn)
    return max_pass


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else "tools/probes/bp_kernel.so"
    n_real = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    n_items = int(sys.argv[3]) if len(sys.argv) > 3 else 256000
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    mode = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    t0 = time.time()
    n_nodes, S = 20000, 500
    sizes = np.round(np.linspace(30, 300, 50)).astype(int)
    lay = syn.make_layout(n_nodes, sizes, 7)
    x = syn._gen_numpy(lay, S, np.random.default_rng(3), set(lay.modules))
    x = (x - x.mean(0)) / x.std(0, ddof=1)
    rng = np.random.default_rng(1)
    packs, offs, ks, js, gs = [], [], [], [], []
    off = 0
    for it in range(n_real):
        k = int(sizes[it % len(sizes)])
        idx = rng.choice(n_nodes, k, replace=False)
        G = x[:, idx].T @ x[:, idx]
        p = pack(G)
        packs.append(p)
        offs.append(off)
        off += p.size
        ks.append(k)
        js.append(host_steps(G))
        gs.append(G)
    grams = np.concatenate(packs)
    offs = np.array(offs, dtype=np.int64)
    ks = np.array(ks, dtype=np.int32)
    js = np.array(js, dtype=np.int32)
    print(f"generated {n_real} items ({grams.nbytes / 1e6:.0f} MB) in {time.time() - t0:.1f}s; block steps mean "
          f"{js.mean():.2f} max {js.max()} (item mix weighted equally per size)", flush=True)
    lib = ctypes.CDLL(so)
    lib.bp_run.restype = ctypes.c_int
    tout = np.zeros(n_real * JMAX * 2 * B * B)
    ms = ctypes.c_double(0)
    stamps = np.zeros(8, dtype=np.uint64)
    P = ctypes.c_void_p
    rc = lib.bp_run(grams.ctypes.data_as(P), ctypes.c_int64(grams.size), offs.ctypes.data_as(P),
                    ks.ctypes.data_as(P), js.ctypes.data_as(P), ctypes.c_int(n_real), ctypes.c_int(n_items),
                    ctypes.c_int(mode), ctypes.c_int(reps), tout.ctypes.data_as(P), ctypes.byref(ms),
                    stamps.ctypes.data_as(P))
    print("rc", rc, flush=True)
    if rc:
        sys.exit(rc)
    tout = tout.reshape(n_real, JMAX, 2, B, B)
    worst = 0.0
    for i in range(n_real):
        J = js[i]
        T = np.zeros((J * B, J * B))
        for j in range(J):
            T[j * B:(j + 1) * B, j * B:(j + 1) * B] = tout[i, j, 0]
            if j + 1 < J:
                R = tout[i, j, 1]
                T[(j + 1) * B:(j + 2) * B, j * B:(j + 1) * B] = R
                T[j * B:(j + 1) * B, (j + 1) * B:(j + 2) * B] = R.T
        th = np.linalg.eigvalsh(T)[-1]
        ref = np.linalg.eigvalsh(gs[i])[-1]
        worst = max(worst, abs(th - ref) / ref)
    print(f"mode {mode}: items {n_items} per launch: {ms.value:.2f} ms  "
          f"({n_items / 50 / ms.value * 1e3:.0f} C3 perms/s-equivalent); worst |theta_T - theta|/theta {worst:.2e}")
    names = ["start", "store", "G V (MFMA)", "recurrence", "reorth", "CholQR"]
    print("wave-0 cycles per item:", {nm: int(stamps[i]) // n_items for i, nm in enumerate(names)},
          "total", int(stamps[:6].sum()) // n_items)


if __name__ == "__main__":
    main()
