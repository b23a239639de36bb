"""The sharded HIP path of bench.py with more than one rank (VERDICT r2 item
7): two processes, both on cuda:0, over gloo (NETREP_BENCH_BACKEND=gloo; the
driver's multi-GPU runs use RCCL), drive bench.py's own setup_dist /
build_case (rank 0 builds and broadcasts the test matrices) / time_steps
(contiguous permutation chunks, src/permutations.cpp:338-354) / gather_nulls
(combineAnalyses' abind along the permutation axis, R/multi-machine.R:114)
with the HIP engine on every rank. The gathered cube must equal a one-rank run
over the same global permutations bit for bit: each permutation is keyed by
(seed, global index), so the shard count cannot change a result."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

SEED = 4242
STEPS_2, PERMS = 3, 32   # per rank: 3 steps of 32 permutations


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _rank(rank, world, port, steps, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", NETREP_BENCH_BACKEND="gloo")
    sys.path.insert(0, ROOT)
    import numpy as np  # noqa: F811
    import torch.distributed as dist
    import bench
    w, r, local = bench.setup_dist(None)
    eng, lay, meta, tensors = bench.build_case("CT", w, r, local, SEED)
    eng.set_batch(16)
    _, chunks, total = bench.time_steps(eng, w, r, steps, 1, PERMS, SEED, 10**9)
    local_cube = np.concatenate(chunks, axis=2)
    cube = bench.gather_nulls(local_cube, r, w, total) if w > 1 else local_cube
    if r == 0:
        np.save(out, cube)
        np.save(out + ".observed.npy", eng.observed())
    if w > 1:
        dist.destroy_process_group()
    eng.close()


def test_two_ranks_gather_equals_one_rank(tmp_path):
    two = str(tmp_path / "two.npy")
    one = str(tmp_path / "one.npy")
    mp.spawn(_rank, args=(2, _free_port(), STEPS_2, two), nprocs=2, join=True)
    mp.spawn(_rank, args=(1, _free_port(), 2 * STEPS_2, one), nprocs=1, join=True)
    a, b = np.load(two), np.load(one)
    assert a.shape == b.shape == (8, 7, 2 * STEPS_2 * PERMS)
    assert np.isfinite(a).all()
    np.testing.assert_array_equal(a.view(np.uint64), b.view(np.uint64))
    np.testing.assert_array_equal(np.load(two + ".observed.npy").view(np.uint64),
                                  np.load(one + ".observed.npy").view(np.uint64))
