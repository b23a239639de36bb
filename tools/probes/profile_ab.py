"""A/B timing of the summary-profile kernel variants on one module-size set
(GPU box): a C3-shaped dataset (20k genes x 500 samples) with the given module
sizes, 256-permutation launches, profile-kernel HIP-event time and phase
stamps per variant.

  python tools/probes/profile_ab.py [S] [k_lo] [k_hi] [n_mod] [variants...]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import netrep_amd as N  # noqa: E402
from netrep_amd import synthetic as S  # noqa: E402


def main():
    a = sys.argv[1:]
    n_samples = int(a[0]) if a else 500
    k_lo, k_hi, n_mod = (int(a[1]), int(a[2]), int(a[3])) if len(a) >= 4 else (30, 255, 42)
    variants = a[4:] or ["rg4", "packed4"]
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
    ref = None
    flops = (2.0 * n_samples * k.astype(np.float64) ** 2).sum() * 256
    for v in variants:
        # "name:ENV=VAL,ENV=VAL" sets engine knobs for this variant only
        name, _, knobs = v.partition(":")
        os.environ["NETREP_PROFILE_VARIANT"] = name
        for kv in [x for x in knobs.split(",") if x]:
            key, _, val = kv.partition("=")
            os.environ[key] = val
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
        err = None
        if ref is None:
            ref = out
        else:
            fin = np.isfinite(ref) & np.isfinite(out)
            err = float(np.max(np.where(fin, np.abs(out - ref) / np.maximum(np.abs(ref), 1e-2), 0.0)))
        print(f"{v:8s} S={n_samples} k={k_lo}..{k_hi} x{n_mod}: profile {ms:.3f} ms/256 perms "
              f"({flops / ms / 1e9:.2f} TF/s credited), wall {wall:.2f}s/1024, max err vs first {err}, "
              f"diag {eng.diagnostics()}")
        per_item = {kk: round(vv / (512 * n_mod)) for kk, vv in st.items() if vv}
        print(f"   stamps {frac}")
        print(f"   wave-0 cycles per item {per_item}")
        for kv in [x for x in knobs.split(",") if x]:
            os.environ.pop(kv.partition("=")[0], None)


if __name__ == "__main__":
    main()
