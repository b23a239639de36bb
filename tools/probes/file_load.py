"""disk.matrix files -> HBM throughput (GPU box): writes corr/net/data of an
N-gene synthetic dataset as uncompressed and gzip RDS files, then times
nr_set_dataset_files against the in-memory upload of the same matrices.

  python tools/probes/file_load.py [n_nodes] [n_samples]
"""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import netrep_amd as N  # noqa: E402
from rds_writer import write_rds  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12000
    s = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    rng = np.random.default_rng(1)
    x = rng.standard_normal((s, n))
    xc = (x - x.mean(0)) / np.linalg.norm(x - x.mean(0), axis=0)
    corr = xc.T @ xc
    net = np.abs(corr) ** 5
    names = [f"G{i}" for i in range(n)]
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        for comp in (False, True):
            if comp and n > 8000:
                m = 4000  # gzip writing is slow in Python: a smaller matrix for the inflate rate
                sub = slice(0, m)
                c2, n2, x2, nm = corr[sub, sub], net[sub, sub], x[:, sub], names[:m]
            else:
                m, c2, n2, x2, nm = n, corr, net, x, names
            pc, pn, pd = (os.path.join(td, f"{k}{int(comp)}.rds") for k in ("c", "n", "d"))
            t0 = time.perf_counter()
            write_rds(pc, c2, None, nm, compress=comp)
            write_rds(pn, n2, None, nm, compress=comp)
            write_rds(pd, x2, None, nm, compress=comp)
            wt = time.perf_counter() - t0
            gb = (2 * m * m + s * m) * 8 / 1e9
            eng = N.Engine(0)
            t0 = time.perf_counter()
            eng.set_dataset_files(pc, pn, pd)
            ft = time.perf_counter() - t0
            t0 = time.perf_counter()
            eng.set_dataset(np.asfortranarray(c2), np.asfortranarray(n2), np.asfortranarray(x2))
            mt = time.perf_counter() - t0
            eng.close()
            print(f"{'gzip' if comp else 'plain'} RDS, {m} genes x {s} samples ({gb:.2f} GB of doubles; "
                  f"written in {wt:.1f}s): files->HBM {ft:.2f}s = {gb / ft:.2f} GB/s; "
                  f"in-memory upload {mt:.2f}s = {gb / mt:.2f} GB/s", flush=True)


if __name__ == "__main__":
    main()
