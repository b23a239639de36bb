"""The engine's less-travelled paths, each against a reference restatement or
against the default path bit for bit.

* The gather kernel's null cube. The network statistics come from the column
  sweep (sweep.hip) except where its packed entries cannot hold the shapes:
  modules beyond 4,096 nodes or n >= 65,536 (nr::sweep_supported). There
  module_net_kernel gathers every pair of every (permutation, module) item.
  A 4,200-node module at n = 6,000 forces that path for the whole launch; its
  null cube is compared with the C++ restatement of src/permutations.cpp:62-101
  (data) and src/permutationsNoData.cpp:57-88 (network only) on identical
  shuffles.
* Column-sweep sub-batches: a batch split into many sub-batches (a test-only
  smaller bound, nr_debug_set) is bitwise the unsplit batch.
* A failed sweep allocation leaves the context usable: the rerun with a
  smaller batch reallocates and is bitwise a clean run.
"""
import numpy as np
import pytest

import netrep_amd as N
from netrep_amd import _lib as L
from netrep_amd import synthetic as S
from oracle import netrep_oracle as O
from oracle import ref_cpp

from conftest import assert_stats_close, record, relative_error_record

pytestmark = pytest.mark.gpu

SWEEP_MAX_K = 4096   # nr::sweep_supported: modules of at most 4,096 nodes


def _setup(n, sizes, s, seed):
    lay = S.make_layout(n, list(sizes), seed)
    x, c, nt = S.numpy_dataset(lay, max(s, 2), seed + 1)
    mi = O.ModuleIndex(lay.names, lay.labels, lay.names, lay.modules)
    with_data = s > 0
    xs = O.scale(x) if with_data else None
    disc = O.intermediate_properties(xs, c, nt, mi.disc_idx(lay.names), with_data=with_data)
    # the test dataset: another draw over the same layout
    tx, tc, tn = S.numpy_dataset(lay, max(s, 2), seed + 2, preserve_all=False)
    txs = O.scale(tx) if with_data else None
    mods = mi.mods_present
    cat = lambda d: np.concatenate([d[m] for m in mods])
    m = dict(
        lay=lay, mi=mi, mods=mods, with_data=with_data,
        row_of=[mi.modules.index(m) for m in mods],
        node_off=np.concatenate([[0], np.cumsum([mi.test_idx[m].size for m in mods])]),
        idx=cat(mi.test_idx), null_pos=cat(mi.null_pos),
        dcv=cat(disc["corr"]), dwd=cat(disc["degree"]),
        dnc=cat(disc["contribution"]) if with_data else None,
        txs=txs, tc=np.asfortranarray(tc), tn=np.asfortranarray(tn))
    return m


def _engine(m):
    e = N.Engine(0)
    e.set_dataset(m["tc"], m["tn"], m["txs"])
    e.set_modules(len(m["mi"].modules), m["row_of"], m["node_off"], m["idx"], m["null_pos"], m["dcv"], m["dwd"],
                  m["dnc"])
    e.set_null_pool(m["mi"].null_idx)
    return e


@pytest.fixture(scope="module")
def wide():
    return _setup(6000, (4200, 300, 61, 7), 24, 71)


@pytest.mark.parametrize("with_data", [True, False], ids=["data", "network-only"])
def test_gather_kernel_null_cube_vs_cpp_oracle(wide, with_data):
    m = dict(wide)
    if not with_data:
        m.update(txs=None, dnc=None, with_data=False)
    assert max(np.diff(m["node_off"])) > SWEEP_MAX_K   # outside the sweep: module_net_kernel runs
    seed, p0, n_perm = 2024, 77, 16
    e = _engine(m)
    try:
        got = e.run(p0, p0 + n_perm, seed)
        gobs = e.observed()
        assert not e.gram_table()
    finally:
        e.close()
    pis = N.prp_table(seed, p0, p0 + n_perm, m["mi"].null_idx.size)
    exp, obs = ref_cpp.permutation_procedure(
        m["txs"], m["tc"], m["tn"], len(m["mi"].modules), m["row_of"], m["node_off"], m["idx"], m["null_pos"],
        m["mi"].null_idx, m["dcv"], m["dwd"], m["dnc"], n_perm, pi=pis, n_threads=16)
    e1 = assert_stats_close(gobs, obs, what="gather observed")
    e2 = assert_stats_close(got, exp, what="gather nulls")
    record(f"gather kernel nulls ({n_perm} perms, module of 4,200 nodes, "
           f"{'S=24' if with_data else 'network only'})", max(e1, e2), perms=n_perm,
           small_cells=relative_error_record(got, exp))


def test_sweep_sub_batches_bitwise():
    """One 96-permutation batch as many sub-batches (a bound of 4,000
    occurrences: ~10 permutations each) equals the unsplit batch bit for bit."""
    m = _setup(2000, (150, 90, 40, 12), 0, 81)
    e = _engine(m)
    lib = L.load()
    try:
        ref = e.run(0, 96, 5)
        assert lib.nr_debug_set(L.NR_DEBUG_SWEEP_MAX_OCC, 4000) == L.NR_OK
        try:
            got = e.run(0, 96, 5)
        finally:
            lib.nr_debug_set(L.NR_DEBUG_SWEEP_MAX_OCC, 0)
        np.testing.assert_array_equal(got.view(np.uint64), ref.view(np.uint64))
    finally:
        e.close()


def test_sweep_allocation_failure_then_smaller_batch():
    """run A sizes the sweep buffers; run B needs larger ones and
    its third allocation fails (NR_ERR_OOM); run C, with a batch smaller than
    A's, must reallocate (the set's capacity reads 0 after the failure)
    instead of launching on the freed buffers, and equals a clean run."""
    m = _setup(2000, (150, 90, 40, 12), 0, 82)
    lib = L.load()
    e = _engine(m)
    try:
        e.set_batch(64)
        e.run(0, 64, 9)                                     # A
        e.set_batch(256)
        assert lib.nr_debug_set(L.NR_DEBUG_FAIL_SWEEP_ALLOC, 3) == L.NR_OK
        try:
            with pytest.raises(L.NetRepError) as ex:
                e.run(0, 256, 9)                            # B
            assert ex.value.code == L.NR_ERR_OOM
        finally:
            lib.nr_debug_set(L.NR_DEBUG_FAIL_SWEEP_ALLOC, 0)
        e.set_batch(32)
        got = e.run(0, 96, 9)                               # C
    finally:
        e.close()
    f = _engine(m)
    try:
        ref = f.run(0, 96, 9)
    finally:
        f.close()
    np.testing.assert_array_equal(got.view(np.uint64), ref.view(np.uint64))
