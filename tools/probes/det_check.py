"""Run-to-run determinism and variant agreement of the summary-profile kernels
(GPU box): the same permutations twice with the default plan, then with
NETREP_PROFILE_VARIANT=packed4; reports bitwise differences per module and
statistic, and the largest scaled difference between the variants."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import netrep_amd as N  # noqa: E402
from netrep_amd import synthetic as S  # noqa: E402
from netrep_amd.api import RMatrix  # noqa: E402


def case(n_nodes, S_, sizes):
    lay = S.make_layout(n_nodes, np.asarray(sizes), 5)
    dx, dc, dn = S.numpy_dataset(lay, S_, 6)
    tx, tc, tn = S.numpy_dataset(lay, S_, 7, preserve_all=False)
    names = lay.names
    ma = dict(zip(names, lay.labels))
    disc = N.IntermediateProperties(N.Scale(RMatrix(dx, None, names)), RMatrix(dc, names, names),
                                    RMatrix(dn, names, names), names, ma, lay.modules)
    args = (disc, N.Scale(RMatrix(tx, None, names)), RMatrix(tc, names, names), RMatrix(tn, names, names),
            ma, lay.modules)
    return args, lay


def run(args, n_perm, seed=11):
    return N.PermutationProcedure(*args, n_perm, seed=seed)["nulls"]


def main():
    n_perm = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    for (n_nodes, S_, sizes) in ((3000, 100, np.round(np.linspace(30, 300, 10)).astype(int)),
                                 (3000, 200, [40, 120, 200, 215, 240, 255])):
        args, lay = case(n_nodes, S_, sizes)
        os.environ.pop("NETREP_PROFILE_VARIANT", None)
        a = run(args, n_perm)
        b = run(args, n_perm)
        os.environ["NETREP_PROFILE_VARIANT"] = "packed4"
        c = run(args, n_perm)
        os.environ.pop("NETREP_PROFILE_VARIANT", None)
        ab = a.view(np.uint64) != b.view(np.uint64)
        print(f"case S={S_} sizes={list(lay.module_sizes)}")
        print("  run-to-run bitwise mismatches per (module, stat):")
        print("  ", ab.sum(axis=2).tolist())
        fin = np.isfinite(a) & np.isfinite(c)
        err = np.where(fin, np.abs(a - c) / np.maximum(np.abs(c), 1e-2), 0.0)
        print("  default vs packed4 max scaled err per (module, stat):")
        print("  ", np.array2string(err.max(axis=2), precision=2))
        print("  NA pattern differs:", int((np.isfinite(a) != np.isfinite(c)).sum()))


if __name__ == "__main__":
    main()
