"""Residency across the reference-interface calls and the
mesh broadcast of a resident dataset.

modulePreservation loads each discovery dataset once and calls
IntermediateProperties once per test dataset with it
(R/modulePreservation.R:553-590); networkProperties calls NetProps per
(discovery, test) pair (R/networkProperties.R:295-302). The library keeps
those datasets in HBM while later calls name the same host arrays and counts
every host->device byte (nr_h2d_bytes), so the tests can see what crossed
PCIe. Results must be bitwise those of a fresh upload.

nr_broadcast_dataset (scatter + all-gather of peer copies)
must give every destination a bitwise copy: runs on the copies equal the
source's run bit for bit, including sizes that do not split evenly.
"""
import numpy as np
import pytest

import netrep_amd as N
from netrep_amd import synthetic as S
from netrep_amd.api import RMatrix

pytestmark = pytest.mark.gpu

MB = 1 << 20


def _dataset(n=2500, s=120, seed=11, sizes=(200, 150, 90, 40)):
    lay = S.make_layout(n, list(sizes), seed)
    x, c, nt = S.numpy_dataset(lay, s, seed + 1)
    names = lay.names
    return lay, names, dict(zip(names, lay.labels)), np.asfortranarray(x), np.asfortranarray(c), np.asfortranarray(nt)


def _same(a, b):
    for key in a:
        if isinstance(a[key], dict):
            assert a[key].keys() == b[key].keys()
            for m in a[key]:
                _same_arr(a[key][m], b[key][m])
        else:
            _same_arr(a[key], b[key])


def _same_arr(x, y):
    x, y = np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)
    np.testing.assert_array_equal(x.view(np.uint64), y.view(np.uint64))


def test_discovery_dataset_uploaded_once_for_three_test_datasets():
    """1 discovery x 3 test datasets: the discovery matrices cross PCIe once."""
    N.ReleaseResident()
    lay, names, ma, x, c, nt = _dataset()
    dxs = N.Scale(RMatrix(x, None, names))
    dc, dn = RMatrix(c, names, names), RMatrix(nt, names, names)
    n, s = len(names), x.shape[0]
    full = 2 * n * n * 8 + s * n * 8
    rng = np.random.default_rng(3)
    t_lists = [names, [nm for nm in names if rng.random() < 0.8], names[::2]]
    outs, deltas = [], []
    for t in t_lists:
        before = N.h2d_bytes()
        outs.append(N.IntermediateProperties(dxs, dc, dn, t, ma, lay.modules))
        deltas.append(N.h2d_bytes() - before)
    assert deltas[0] >= full, deltas
    assert deltas[1] < MB and deltas[2] < MB, deltas
    # a sampled element changed in place: the fingerprint no longer matches, re-upload
    old = c[0, 0]
    c[0, 0] = 0.5
    before = N.h2d_bytes()
    N.IntermediateProperties(dxs, dc, dn, t_lists[0], ma, lay.modules)
    assert N.h2d_bytes() - before >= full
    c[0, 0] = old
    # an edit between any sampling points (one node's row and
    # column zeroed in the middle of the matrix) is seen too: every element is
    # fingerprinted
    mid = n // 2 + 7
    saved_r, saved_c = c[mid, :].copy(), c[:, mid].copy()
    c[mid, :] = 0.0
    c[:, mid] = 0.0
    before = N.h2d_bytes()
    N.IntermediateProperties(dxs, dc, dn, t_lists[0], ma, lay.modules)
    assert N.h2d_bytes() - before >= full
    c[mid, :] = saved_r
    c[:, mid] = saved_c
    # one element changed by one ulp
    c[mid + 1, 3] = np.nextafter(c[mid + 1, 3], 2.0)
    before = N.h2d_bytes()
    N.IntermediateProperties(dxs, dc, dn, t_lists[0], ma, lay.modules)
    assert N.h2d_bytes() - before >= full
    c[mid + 1, 3] = np.nextafter(c[mid + 1, 3], -2.0)
    # bitwise the results of fresh uploads
    for t, o in zip(t_lists, outs):
        N.ReleaseResident()
        _same(o, N.IntermediateProperties(dxs, dc, dn, t, ma, lay.modules))
    N.ReleaseResident()


def test_netprops_network_uploaded_once_and_kept():
    """NetProps: the network crosses PCIe once (it is also the unused
    correlation operand), the raw data once (scaled on the device), and a
    second call on the same arrays uploads neither."""
    N.ReleaseResident()
    lay, names, ma, x, c, nt = _dataset(n=1800, s=90, seed=21, sizes=(160, 70, 33))
    data, net = RMatrix(x, None, names), RMatrix(nt, names, names)
    n, s = len(names), x.shape[0]
    once = n * n * 8 + s * n * 8
    b0 = N.h2d_bytes()
    r1 = N.NetProps(data, net, ma, lay.modules)
    d1 = N.h2d_bytes() - b0
    assert once <= d1 < once + MB, (d1, once)
    b1 = N.h2d_bytes()
    r2 = N.NetProps(data, net, ma, lay.modules)
    assert N.h2d_bytes() - b1 < MB
    for m in r1:
        for key in ("degree", "summary", "contribution"):
            _same_arr(r1[m][key], r2[m][key])
    # on-device scaling gives the same statistics as host-scaled data would
    # within rounding (Scale on the device either way): compare with a fresh call
    N.ReleaseResident()
    r3 = N.NetProps(data, net, ma, lay.modules)
    for m in r1:
        _same_arr(r1[m]["summary"], r3[m]["summary"])
        _same_arr([r1[m]["coherence"]], [r3[m]["coherence"]])
    N.ReleaseResident()


def test_pooled_contexts_give_identical_permutation_results():
    """Contexts are reused across PermutationProcedure calls (no dataset
    kept): repeated calls are bitwise equal, interleaved with other calls."""
    N.ReleaseResident()
    lay, names, ma, x, c, nt = _dataset(n=1500, s=80, seed=31, sizes=(120, 60, 31))
    dxs = N.Scale(RMatrix(x, None, names))
    disc = N.IntermediateProperties(dxs, RMatrix(c, names, names), RMatrix(nt, names, names), names, ma,
                                    lay.modules)
    tx, tc, tn = S.numpy_dataset(lay, 80, 32, preserve_all=False)
    args = (disc, N.Scale(RMatrix(np.asfortranarray(tx), None, names)),
            RMatrix(np.asfortranarray(tc), names, names), RMatrix(np.asfortranarray(tn), names, names),
            ma, lay.modules, 40)
    a = N.PermutationProcedure(*args, seed=5)
    N.Scale(RMatrix(x, None, names))      # another call in between takes a pooled context too
    b = N.PermutationProcedure(*args, seed=5)
    _same_arr(a["nulls"], b["nulls"])
    _same_arr(a["observed"], b["observed"])
    N.ReleaseResident()


@pytest.mark.parametrize("n,s", [(1001, 37), (640, 0)])
def test_broadcast_dataset_three_contexts_bitwise(n, s):
    """nr_broadcast_dataset to two contexts (pieces of uneven size): each copy
    runs bitwise like the source, with and without data."""
    from oracle import netrep_oracle as O
    lay = S.make_layout(n, [120, 64, 30], 41)
    x, c, nt = S.numpy_dataset(lay, max(s, 2), 42)
    mi = O.ModuleIndex(lay.names, lay.labels, lay.names, lay.modules)
    with_data = s > 0
    disc = O.intermediate_properties(O.scale(x) if with_data else None, c, nt, mi.disc_idx(lay.names),
                                     with_data=with_data)
    mods = mi.mods_present
    node_off = np.concatenate([[0], np.cumsum([mi.test_idx[m].size for m in mods])])
    idx = np.concatenate([mi.test_idx[m] for m in mods])
    engines = [N.Engine(0) for _ in range(3)]
    try:
        engines[0].set_dataset(c, nt, O.scale(x) if with_data else None)
        engines[0].broadcast_dataset_to(engines[1:])
        outs = []
        for e in engines:
            assert e.shape() == (n, s if with_data else 0)
            e.set_modules(len(mi.modules), [mi.modules.index(m) for m in mods], node_off, idx,
                          np.concatenate([mi.null_pos[m] for m in mods]),
                          np.concatenate([disc["corr"][m] for m in mods]),
                          np.concatenate([disc["degree"][m] for m in mods]),
                          np.concatenate([disc["contribution"][m] for m in mods]) if with_data else None)
            e.set_null_pool(mi.null_idx)
            outs.append(e.run(3, 19, 8))
        for o in outs[1:]:
            _same_arr(outs[0], o)
    finally:
        for e in engines:
            e.close()


def test_cancel_after_run_does_not_stick_to_a_cleared_context():
    """a context cancelled after its run returned (the progress
    monitor cancels every context of a call) must not stop the next run once
    its dataset is cleared for the pool (nr_clear_dataset)."""
    from netrep_amd import _lib as L
    lay, names, ma, x, c, nt = _dataset(n=800, s=40, seed=51, sizes=(60, 30))
    eng = N.Engine(0)
    try:
        node_off, idx = S.csr_of(lay)
        k = node_off[1:] - node_off[:-1]
        dcv, dwd = np.zeros(int((k * (k - 1) // 2).sum())), np.zeros(int(k.sum()))

        def load():
            eng.set_dataset(c, nt, None)
            eng.set_modules(len(k), np.arange(len(k), dtype=np.int32), node_off, idx, idx, dcv, dwd)
            eng.set_null_pool(np.arange(len(names), dtype=np.int32))

        load()
        eng.run(0, 8, seed=3)
        eng.cancel()                      # after the run: nothing left to stop
        assert eng._lib.nr_clear_dataset(eng._h) == L.NR_OK
        load()
        out = eng.run(0, 8, seed=3)       # would raise NR_ERR_CANCELLED before the fix
        assert out.shape[-1] == 8
    finally:
        eng.close()


def _pool_info():
    import ctypes as C
    from netrep_amd import _lib as L
    n, b = C.c_int64(), C.c_int64()
    lo, hi = C.c_int32(), C.c_int32()
    assert L.load().netrep_PoolInfo(C.byref(n), C.byref(b), C.byref(lo), C.byref(hi)) == L.NR_OK
    return n.value, b.value, lo.value, hi.value


@pytest.mark.parametrize("n_cores", [3, 16])
def test_pooled_context_host_threads_back_to_default(n_cores):
    """a PermutationProcedure call with nCores different from
    the process default sets its contexts' host threads to nCores; once the
    call returns, every pooled context is back at the default
    (nr_get_host_threads) and holds no per-batch work buffers (its column-sweep
    sets and slot scratch are released with its dataset)."""
    from netrep_amd import _lib as L
    lib = L.load()
    default = lib.nr_get_host_threads()
    assert 1 <= default <= 16 and default != n_cores
    N.ReleaseResident()
    lay, names, ma, x, c, nt = _dataset(n=1200, s=60, seed=91, sizes=(100, 50, 20))
    disc = N.IntermediatePropertiesNoData(RMatrix(c, names, names), RMatrix(nt, names, names), names, ma,
                                          lay.modules)
    out = N.PermutationProcedureNoData(disc, RMatrix(c, names, names), RMatrix(nt, names, names), ma,
                                       lay.modules, 64, nCores=n_cores, seed=3)
    assert out["nulls"].shape[-1] == 64
    n_pooled, scratch, lo, hi = _pool_info()
    assert n_pooled >= 1
    assert lo == hi == default, (lo, hi, default)
    assert scratch == 0, scratch
    N.ReleaseResident()
    assert _pool_info()[0] == 0


def test_peer_staged_pairs_zero_on_one_device():
    """Contexts on one GPU never need peer copies: no pair is recorded as
    host-staged by a broadcast between them."""
    import ctypes as C
    from netrep_amd import _lib as L
    lay, names, ma, x, c, nt = _dataset(n=700, s=30, seed=93, sizes=(60, 20))
    with N.Engine(0) as a, N.Engine(0) as b:
        a.set_dataset(c, nt, None)
        a.broadcast_dataset_to([b])
    n = C.c_int(-1)
    assert L.load().nr_peer_staged_pairs(C.byref(n)) == L.NR_OK
    assert n.value == 0


@pytest.mark.skipif(N.device_count() < 2, reason="needs two physical GPUs")
def test_broadcast_across_two_physical_devices_bitwise():
    """nr_broadcast_dataset between two physical GPUs
    enables peer access (xGMI) and the copy runs bitwise like the source."""
    from oracle import netrep_oracle as O
    lay = S.make_layout(900, [120, 64, 30], 61)
    x, c, nt = S.numpy_dataset(lay, 40, 62)
    mi = O.ModuleIndex(lay.names, lay.labels, lay.names, lay.modules)
    disc = O.intermediate_properties(O.scale(x), c, nt, mi.disc_idx(lay.names), with_data=True)
    mods = mi.mods_present
    node_off = np.concatenate([[0], np.cumsum([mi.test_idx[m].size for m in mods])])
    with N.Engine(0) as a, N.Engine(1) as b:
        a.set_dataset(c, nt, O.scale(x))
        a.broadcast_dataset_to([b])
        outs = []
        for e in (a, b):
            e.set_modules(len(mi.modules), [mi.modules.index(m) for m in mods], node_off,
                          np.concatenate([mi.test_idx[m] for m in mods]),
                          np.concatenate([mi.null_pos[m] for m in mods]),
                          np.concatenate([disc["corr"][m] for m in mods]),
                          np.concatenate([disc["degree"][m] for m in mods]),
                          np.concatenate([disc["contribution"][m] for m in mods]))
            e.set_null_pool(mi.null_idx)
            outs.append(e.run(0, 32, seed=9))
        _same_arr(outs[0], outs[1])
