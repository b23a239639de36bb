"""CPU, world_size 2 over gloo: broadcast of the test matrices, contiguous
permutation shards, gather of null slices -- the N>1 path of bench.py. The
per-rank compute here is the C++ CPU restatement (no GPU in this container);
on the GPU box the same plumbing drives the HIP engine."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from netrep_amd.distributed import gather_nulls, perm_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_perm_range_matches_reference_chunking():
    for n_perm, world in [(10, 3), (7, 8), (100000, 8), (5, 1)]:
        ranges = [perm_range(r, world, n_perm) for r in range(world)]
        assert ranges[0][0] == 0 and ranges[-1][1] == n_perm
        assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
        sizes = [e - b for b, e in ranges]
        assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    from oracle import netrep_oracle as O, prp, ref_cpp
    g = np.load(os.path.join(ROOT, "tests", "golden", "netrep_bundled.npz"))
    e = np.load(os.path.join(ROOT, "tests", "golden", "bundled_expected.npz"))
    n = 150
    corr = torch.zeros((n, n), dtype=torch.float64)
    net = torch.zeros((n, n), dtype=torch.float64)
    if rank == 0:
        corr.copy_(torch.from_numpy(g["test_correlation"]))
        net.copy_(torch.from_numpy(g["test_network"]))
    for t in (corr, net):
        dist.broadcast(t, src=0)                      # setup-time broadcast
    mi = O.ModuleIndex(g["module_labels_names"].tolist(), g["module_labels"].tolist(),
                       g["test_network_colnames"].tolist(), ["1", "2", "3", "4"])
    mods = mi.mods_present
    node_off = np.concatenate([[0], np.cumsum([mi.test_idx[m].size for m in mods])])
    n_perm = 11
    b, end = perm_range(rank, world, n_perm)
    pis = np.stack([prp.permute(np.arange(n), n, 77, p) for p in range(b, end)])
    local, _ = ref_cpp.permutation_procedure(
        None, corr.numpy(), net.numpy(), 4, [0, 1, 2, 3], node_off,
        np.concatenate([mi.test_idx[m] for m in mods]), np.concatenate([mi.null_pos[m] for m in mods]),
        mi.null_idx, np.concatenate([e[f"disc_corr_{m}_nodata"] for m in mods]),
        np.concatenate([e[f"disc_degree_{m}_nodata"] for m in mods]), None, end - b, pi=pis,
        want_observed=False)
    full = gather_nulls(local, rank, world, n_perm)
    if rank == 0:
        np.save(out_path, full)
    dist.destroy_process_group()


def test_two_rank_shard_gather_equals_single_run(tmp_path, bundled, bundled_expected):
    from oracle import netrep_oracle as O, prp
    out = str(tmp_path / "nulls.npy")
    port = 29500 + os.getpid() % 1000
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    got = np.load(out)
    b, e = bundled, bundled_expected
    mi = O.ModuleIndex(b["module_labels_names"].tolist(), b["module_labels"].tolist(),
                       b["test_network_colnames"].tolist(), ["1", "2", "3", "4"])
    disc = {"corr": {m: e[f"disc_corr_{m}_nodata"] for m in mi.mods_present},
            "degree": {m: e[f"disc_degree_{m}_nodata"] for m in mi.mods_present}}
    pis = np.stack([prp.permute(np.arange(150), 150, 77, p) for p in range(11)]).astype(np.int64)
    exp, _ = O.permutation_procedure(disc, None, b["test_correlation"], b["test_network"], mi, pis,
                                     with_data=False)
    assert got.shape == (4, 4, 11)
    fin = np.isfinite(exp)
    assert (np.isfinite(got) == fin).all()
    assert np.max(np.abs(got[fin] - exp[fin]) / np.maximum(np.abs(exp[fin]), 1e-2)) < 1e-10
