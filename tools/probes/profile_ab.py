"""A/B timing of builds of the summary-profile kernel on one module-size set
(GPU box): a C3-shaped dataset (20k genes x 500 samples) with the given module
sizes, 256-permutation launches, profile-kernel HIP-event time and phase
stamps per build. The library has one numerical path; alternatives are
compile-time builds (make -C netrep_amd/csrc OUT=... CXXFLAGS+=-D...), each
run in its own process.

  python tools/probes/profile_ab.py [S] [k_lo] [k_hi] [n_mod] [label=path/to/lib.so ...]
  (no builds given: the in-tree library)
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import netrep_amd as N  # noqa: E402
from netrep_amd import synthetic as S  # noqa: E402


def run_one(n_samples, k_lo, k_hi, n_mod, label):
    sizes = np.round(np.linspace(k_lo, k_hi, n_mod)).astype(int)
    lay = S.make_layout(20000, sizes, 3)
    dev = torch.device("cuda", 0)
    tx, tc, tn = S.torch_dataset(lay, n_samples, 5, preserve_all=False, device=dev)
    txs = S.scale_rows_torch(tx).contiguous()
    torch.cuda.synchronize()
    mods = lay.modules
    node_off = np.concatenate([[0], np.cumsum([lay.members[m].size for m in mods])]).astype(np.int64)
    idx = np.concatenate([lay.members[m] for m in mods]).astype(np.int32)
    k = np.diff(node_off)
    rng = np.random.default_rng(1)
    disc_cv = rng.uniform(-1, 1, int((k * (k - 1) // 2).sum()))
    disc_wd = rng.uniform(0, 1, int(node_off[-1]))
    disc_nc = rng.uniform(-1, 1, int(node_off[-1]))
    eng = N.Engine(0)
    eng.set_dataset_device(tc.data_ptr(), tn.data_ptr(), txs.data_ptr(), 20000, n_samples)
    eng.set_modules(len(mods), np.arange(len(mods)), node_off, idx, idx, disc_cv, disc_wd, disc_nc)
    eng.set_null_pool(np.arange(20000, dtype=np.int32))
    eng.set_batch(256)
    flops = (2.0 * n_samples * k.astype(np.float64) ** 2).sum() * 256
    eng.run(0, 256, 7)
    eng.synchronize()
    eng.set_timing(True)
    eng.reset_timing()
    t0 = time.perf_counter()
    out = eng.run(0, 1024, 7)
    eng.synchronize()
    wall = time.perf_counter() - t0
    tms, tl, _ = eng.timing(1)
    eng.set_timing(False)
    eng.set_stamps(True)   # separate run: the stamps' atomics cost time
    eng.run(0, 512, 7)
    eng.synchronize()
    st = eng.stamps()
    eng.set_stamps(False)
    ms = tms / max(tl, 1)
    tot = sum(st.values())
    frac = {kk: round(vv / tot, 3) for kk, vv in st.items() if vv}
    np.save(f"/tmp/profile_ab_{label}.npy", out)
    print(f"{label:8s} S={n_samples} k={k_lo}..{k_hi} x{n_mod}: profile {ms:.3f} ms/256 perms "
          f"({flops / ms / 1e9:.2f} TF/s credited), wall {wall:.2f}s/1024, diag {eng.diagnostics()}")
    per_item = {kk: round(vv / (512 * n_mod)) for kk, vv in st.items() if vv}
    print(f"   stamps {frac}")
    print(f"   wave-0 cycles per item {per_item}", flush=True)


def main():
    a = sys.argv[1:]
    if a and a[0] == "--single":
        label, lib = a[1], a[2]
        if lib != "-":
            N._lib.LIB_PATH = lib
        run_one(int(a[3]), int(a[4]), int(a[5]), int(a[6]), label)
        return
    n_samples = int(a[0]) if a else 500
    k_lo, k_hi, n_mod = (int(a[1]), int(a[2]), int(a[3])) if len(a) >= 4 else (30, 300, 50)
    builds = [x.partition("=")[::2] for x in a[4:]] or [("tree", "-")]
    import subprocess
    ref = None
    for label, lib in builds:
        subprocess.run([sys.executable, os.path.abspath(__file__), "--single", label, lib or "-",
                        str(n_samples), str(k_lo), str(k_hi), str(n_mod)], check=True)
        out = np.load(f"/tmp/profile_ab_{label}.npy")
        if ref is None:
            ref = out
        else:
            fin = np.isfinite(ref) & np.isfinite(out)
            err = float(np.max(np.where(fin, np.abs(out - ref) / np.maximum(np.abs(ref), 1e-2), 0.0)))
            print(f"   max scaled difference vs {builds[0][0]}: {err:.3e}")


if __name__ == "__main__":
    main()
