"""Host->HBM upload vs compute for a multi-dataset run (GPU box):
modulePreservation's loop over test datasets (R/modulePreservation.R:553-620)
run back to back with and without netrep_PrefetchTestDataset.

  python tools/probes/prefetch_overlap.py [n_nodes] [n_samples] [n_sets] [n_perm]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import netrep_amd as N  # noqa: E402
from netrep_amd import synthetic as S  # noqa: E402
from netrep_amd.api import RMatrix  # noqa: E402


def main():
    a = [int(x) for x in sys.argv[1:]]
    n_nodes, n_samples, n_sets, n_perm = (a + [12000, 300, 3, 2048][len(a):])[:4]
    lay = S.make_layout(n_nodes, np.round(np.linspace(30, 300, 30)).astype(int), 3)
    names = lay.names
    ma = dict(zip(names, lay.labels))
    t0 = time.perf_counter()
    dx, dc, dn = S.numpy_dataset(lay, n_samples, 4)
    disc = N.IntermediateProperties(N.Scale(RMatrix(dx, None, names)), RMatrix(dc, names, names),
                                    RMatrix(dn, names, names), names, ma, lay.modules)
    del dx, dc, dn
    sets = []
    for t in range(n_sets):
        tx, tc, tn = S.numpy_dataset(lay, n_samples, 10 + t, preserve_all=False)
        sets.append((N.Scale(RMatrix(np.asfortranarray(tx), None, names)),
                     RMatrix(np.asfortranarray(tc), names, names), RMatrix(np.asfortranarray(tn), names, names)))
    print(f"host datasets built in {time.perf_counter() - t0:.1f}s "
          f"({n_sets} x {2 * n_nodes * n_nodes * 8 / 1e9:.2f} GB of corr+net)", flush=True)
    # upload alone (pinned double-buffered chunks)
    eng = N.Engine(0)
    d, c, n = sets[0][0].f, sets[0][1].f, sets[0][2].f
    eng.set_dataset(c, n, d)
    t0 = time.perf_counter()
    eng.set_dataset(c, n, d)
    up = time.perf_counter() - t0
    gb = (2 * n_nodes * n_nodes + n_samples * n_nodes) * 8 / 1e9
    print(f"upload: {up:.3f} s for {gb:.2f} GB = {gb / up:.1f} GB/s", flush=True)
    eng.close()
    N.PermutationProcedure(disc, *sets[0], ma, lay.modules, 256, seed=1)  # warm
    for mode in ("sequential", "prefetch"):
        t0 = time.perf_counter()
        if mode == "prefetch":
            N.PrefetchTestDataset(*sets[0])
        for t in range(n_sets):
            if mode == "prefetch" and t + 1 < n_sets:
                N.PrefetchTestDataset(*sets[t + 1])
            N.PermutationProcedure(disc, *sets[t], ma, lay.modules, n_perm, seed=1)
        dt = time.perf_counter() - t0
        print(f"{mode}: {n_sets} datasets x {n_perm} perms in {dt:.2f} s", flush=True)


if __name__ == "__main__":
    main()
