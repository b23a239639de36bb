"""Extended parity sweep (GPU box): the metric's configuration C3 and C2 over
many more permutations than the -m gpu tests hold (they use 64 / 256), the
HIP engine against the C++ LAPACK restatement (oracle/netrep_ref.cpp) on
identical keyed shuffles. Reports, per configuration and statistic, the
largest and the 99.9th-percentile scaled error |gpu - oracle| /
max(|oracle|, 1e-2), NA-pattern agreement, and the p-value identity record
(tests/conftest.assert_pvalues_identical) over the whole sample.

  python tools/parity_sweep.py [C3 perms] [C2 perms] [C5 perms] > out.json

Test infrastructure (the oracle is the checker here, never the product)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import FLOOR, assert_pvalues_identical, assert_stats_close  # noqa: E402
from test_gpu_configs import Case  # noqa: E402

STATS7 = ["avg.weight", "coherence", "cor.cor", "cor.degree", "cor.contrib", "avg.cor", "avg.contrib"]


def sweep(cfg, seed, n_perm, chunk):
    c = Case(cfg, seed)
    p0 = 7_000_000
    got_all, exp_all, obs = [], [], None
    for b in range(p0, p0 + n_perm, chunk):
        e = min(b + chunk, p0 + n_perm)
        got_all.append(c.eng.run(b, e, seed))
        ex, ob = c.oracle(b, e, seed, True)
        exp_all.append(ex)
        obs = ob if obs is None else obs
        print(f"{cfg}: {e - p0}/{n_perm} permutations", file=sys.stderr, flush=True)
    got = np.concatenate(got_all, axis=2)
    exp = np.concatenate(exp_all, axis=2)
    gobs = c.eng.observed()
    try:   # the -m gpu tests' bar (raises past it); recorded, not fatal, here
        worst = assert_stats_close(got, exp, what=f"{cfg} nulls")
        assert_stats_close(gobs, obs, what=f"{cfg} observed")
        verdict = "within the 1e-10 bar"
    except AssertionError as e:
        worst, verdict = None, f"FAILED: {e}"
    fin = np.isfinite(exp)
    err = np.where(fin, np.abs(got - exp) / np.maximum(np.abs(exp), FLOOR), 0.0)
    per_stat = {}
    for s, name in enumerate(STATS7):
        e_s = err[:, s, :][fin[:, s, :]]
        per_stat[name] = {"max": float(e_s.max()), "p99.9": float(np.quantile(e_s, 0.999)),
                          "median": float(np.median(e_s))}
    k = np.diff(c.node_off)
    try:
        pv = assert_pvalues_identical(got, gobs, exp, obs, k, c.n, what=cfg)
    except AssertionError as e:
        pv = f"FAILED: {e}"
    c.close()
    return {"permutations": n_perm, "modules": int(got.shape[0]), "max_scaled_error": worst, "bar": verdict,
            "na_cells": int((~fin).sum()), "per_statistic": per_stat, "pvalues": pv}


def main():
    n3 = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    n2 = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    n5 = int(sys.argv[3]) if len(sys.argv) > 3 else 0   # C5 (k up to 2,000 > S = 1,000): large-module kernels
    out = {}
    if n3 > 0:
        out["C3"] = sweep("C3", 0x5EED, n3, 256)
    if n2 > 0:
        out["C2"] = sweep("C2", 0xC2C2, n2, 512)
    if n5 > 0:
        out["C5"] = sweep("C5", 0xC5C5, n5, 32)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
