"""GPU parity: the HIP engine through the C ABI against the oracle and the
reference's known answers, on identical index sets.

Tolerance (conftest.assert_stats_close): |gpu - oracle| <= 1e-10 * max(|oracle|, 1e-2)
for every statistic; NA positions and NA_real_ bit patterns identical; index
sets and counts exact.
"""
import numpy as np
import pytest

import netrep_amd as N
from netrep_amd.api import RMatrix
from oracle import netrep_oracle as O
from oracle import prp

from conftest import assert_pvalues_identical, assert_stats_close

pytestmark = pytest.mark.gpu

MODULES = ["1", "2", "3", "4"]


def bundled_inputs(b):
    ma = dict(zip(b["module_labels_names"].tolist(), b["module_labels"].tolist()))
    d_names = b["discovery_network_colnames"].tolist()
    t_names = b["test_network_colnames"].tolist()
    d = dict(
        dData=RMatrix(b["discovery_data"], b["discovery_data_rownames"].tolist(), d_names),
        dCorr=RMatrix(b["discovery_correlation"], d_names, d_names),
        dNet=RMatrix(b["discovery_network"], d_names, d_names),
        tData=RMatrix(b["test_data"], b["test_data_rownames"].tolist(), t_names),
        tCorr=RMatrix(b["test_correlation"], t_names, t_names),
        tNet=RMatrix(b["test_network"], t_names, t_names),
    )
    return d, ma, t_names


def disc_from_golden(e, sfx, modules):
    out = {"degree": {}, "corr": {}}
    if sfx.startswith("data"):
        out["contribution"] = {}
    for key in list(out):
        for m in modules:
            k = f"disc_{key}_{m}_{sfx}"
            if k in e:
                out[key][m] = e[k]
    return out


# --------------------------------------------------------------------------
# bundled example data (C1)
# --------------------------------------------------------------------------

def test_scale_matches_oracle(bundled, bundled_expected):
    got = N.Scale(RMatrix(bundled["test_data"])).values
    assert_stats_close(got, bundled_expected["scaled_test_data"], rtol=1e-13, floor=1.0, what="Scale")


@pytest.mark.parametrize("s,n", [(37, 100_003), (500, 20_000), (1_100_000, 3), (500, 1)])
def test_scale_column_chunks_match_oracle(s, n):
    """netrep_Scale streams ~16 MiB column chunks through pinned staging, each
    fork-join of the host threads copying one chunk in and the previous one
    out: two chunks with a ragged last one, five (the metric's 20k x 500), one
    column longer than a chunk, a single column. Every column as src/scale.cpp:14-25 (numpy restatement), with a
    constant column (sd 0: NaN, as the reference gives)."""
    from oracle import netrep_oracle as O
    rng = np.random.default_rng(s + n)
    x = np.asfortranarray(rng.standard_normal((s, n)) * 3.0 + 1.5)
    x[:, n // 2] = 2.0
    got = N.Scale(RMatrix(x)).values
    exp = O.scale(x)
    # the north-star bar (a 1.1M-long column's sum rounds differently in
    # the kernel's 64 lane sums than in numpy's pairwise sum)
    assert_stats_close(got, exp, rtol=1e-10, floor=1.0, what=f"Scale {s}x{n}")


def test_check_finite():
    N.CheckFinite(np.ones((4, 3)))
    bad = np.ones((4, 3))
    bad[2, 1] = np.nan
    with pytest.raises(N.NetRepError) as ei:
        N.CheckFinite(bad)
    assert "non-finite" in str(ei.value)


@pytest.mark.parametrize("with_data", [True, False])
def test_intermediate_properties(bundled, bundled_expected, with_data):
    d, ma, t_names = bundled_inputs(bundled)
    sfx = "data" if with_data else "nodata"
    if with_data:
        got = N.IntermediateProperties(N.Scale(d["dData"]), d["dCorr"], d["dNet"], t_names, ma, MODULES)
    else:
        got = N.IntermediatePropertiesNoData(d["dCorr"], d["dNet"], t_names, ma, MODULES)
    exp = disc_from_golden(bundled_expected, sfx, MODULES)
    assert set(got) == set(exp)
    for key in exp:
        for m in MODULES:
            assert_stats_close(got[key][m], exp[key][m], what=f"{key}/{m}")


@pytest.mark.parametrize("with_data", [True, False])
def test_bundled_observed_and_nulls_explicit_pi(bundled, bundled_expected, with_data):
    d, ma, _ = bundled_inputs(bundled)
    e = bundled_expected
    sfx = "data" if with_data else "nodata"
    disc = disc_from_golden(e, sfx, MODULES)
    pis = e["pis"]
    if with_data:
        r = N.PermutationProcedure(disc, N.Scale(d["tData"]), d["tCorr"], d["tNet"], ma, MODULES,
                                   pis.shape[0], pi=pis)
    else:
        r = N.PermutationProcedureNoData(disc, d["tCorr"], d["tNet"], ma, MODULES, pis.shape[0], pi=pis)
    assert r["nulls"].shape == (4, 7 if with_data else 4, pis.shape[0])   # test1-main.R:31,41
    assert_stats_close(r["observed"], e["observed_" + sfx], what="observed")
    assert_stats_close(r["nulls"], e["nulls_" + sfx], what="nulls")
    # p-values identical to the oracle's (R/pperm.R:138-151): nVarsPresent =
    # module sizes present, totalSize = |overlapVars| (null = "overlap")
    t_names = set(bundled["test_network_colnames"].tolist())
    n_vars = [len(disc["degree"][m]) for m in MODULES]
    total = sum(1 for nm in ma if nm in t_names)
    rec = assert_pvalues_identical(r["nulls"], r["observed"], e["nulls_" + sfx], e["observed_" + sfx],
                                   n_vars, total, what=f"bundled {sfx}")
    assert rec["count_mismatches"] == 0


def test_bundled_observed_matches_vignette(bundled, bundled_expected):
    from test_oracle_golden import VIGNETTE_OBSERVED
    d, ma, _ = bundled_inputs(bundled)
    disc = disc_from_golden(bundled_expected, "data", MODULES)
    r = N.PermutationProcedure(disc, N.Scale(d["tData"]), d["tCorr"], d["tNet"], ma, MODULES, 0)
    assert np.allclose(r["observed"], VIGNETTE_OBSERVED, rtol=5e-7, atol=5e-9)
    assert "nulls" not in r


def test_prp_mode_equals_explicit_table(bundled, bundled_expected):
    """A seeded run and the same shuffles passed as a table give bit-identical cubes."""
    d, ma, _ = bundled_inputs(bundled)
    disc = disc_from_golden(bundled_expected, "data", MODULES)
    seed = 424242
    pis = N.prp_table(seed, 0, 40, 150)
    t = N.Scale(d["tData"])
    a = N.PermutationProcedure(disc, t, d["tCorr"], d["tNet"], ma, MODULES, 40, seed=seed)
    b = N.PermutationProcedure(disc, t, d["tCorr"], d["tNet"], ma, MODULES, 40, pi=pis)
    np.testing.assert_array_equal(a["nulls"].view(np.uint64), b["nulls"].view(np.uint64))


def test_netprops(bundled, bundled_expected):
    d, ma, _ = bundled_inputs(bundled)
    e = bundled_expected
    for tag, data, net in (("disc", d["dData"], d["dNet"]), ("test", d["tData"], d["tNet"])):
        got = N.NetProps(data, net, ma, MODULES)
        for m in MODULES:
            for key in ("summary", "contribution", "degree"):
                assert_stats_close(got[m][key], e[f"netprops_{tag}_{m}_{key}"], what=f"{tag}/{m}/{key}")
            assert_stats_close([got[m]["coherence"]], [e[f"netprops_{tag}_{m}_coherence"]])
            assert_stats_close([got[m]["avgWeight"]], [e[f"netprops_{tag}_{m}_avgWeight"]])
    nd = N.NetPropsNoData(d["tNet"], ma, MODULES)
    for m in MODULES:
        assert_stats_close(nd[m]["degree"], e[f"netprops_test_{m}_degree"])


# --------------------------------------------------------------------------
# the reference test's shape: unsymmetric random matrices, partial overlap
# --------------------------------------------------------------------------

@pytest.mark.parametrize("null", ["overlap", "all"])
@pytest.mark.parametrize("with_data", [True, False])
def test_unsymmetric_partial_overlap(asym, with_data, null):
    a = asym
    tag = "" if null == "overlap" else "_all"
    sfx = ("data" if with_data else "nodata") + tag
    modules = a["modules"].tolist()
    d_names, t_names = a["d_names"].tolist(), a["t_names"].tolist()
    ma = dict(zip(d_names, a["ma_labels"].tolist()))
    tCorr = RMatrix(a["t_corr"], t_names, t_names)
    tNet = RMatrix(a["t_corr"], t_names, t_names)
    disc = disc_from_golden(a, sfx, modules)
    pis = a["pis" + tag]
    if with_data:
        t = RMatrix(O.scale(a["t_data"]), None, t_names)
        r = N.PermutationProcedure(disc, t, tCorr, tNet, ma, modules, pis.shape[0], nullHypothesis=null, pi=pis)
    else:
        r = N.PermutationProcedureNoData(disc, tCorr, tNet, ma, modules, pis.shape[0], nullHypothesis=null, pi=pis)
    assert_stats_close(r["observed"], a["observed_" + sfx], what="observed")
    assert_stats_close(r["nulls"], a["nulls_" + sfx], what="nulls")
    # discovery side through the engine too
    dCorr = RMatrix(a["d_corr"], d_names, d_names)
    if with_data:
        got = N.IntermediateProperties(RMatrix(O.scale(a["d_data"]), None, d_names), dCorr, dCorr,
                                       t_names, ma, modules)
    else:
        got = N.IntermediatePropertiesNoData(dCorr, dCorr, t_names, ma, modules)
    for key in disc:
        for m in modules:
            assert_stats_close(got[key][m], disc[key][m], what=f"disc {key}/{m}")


# --------------------------------------------------------------------------
# engine layer: index export, batching, sharding, larger synthetic case
# --------------------------------------------------------------------------

def _engine_case(n_nodes=600, n_samples=40, sizes=(30, 45, 60, 80, 120), seed=7, with_data=True):
    from netrep_amd import synthetic as S
    lay = S.make_layout(n_nodes, sizes, seed)
    dx, dc, dn = S.numpy_dataset(lay, n_samples, seed + 1)
    tx, tc, tn = S.numpy_dataset(lay, n_samples, seed + 2, preserve_all=False)
    mi = O.ModuleIndex(lay.names, lay.labels, lay.names, lay.modules)
    disc = O.intermediate_properties(O.scale(dx), dc, dn, mi.disc_idx(lay.names), with_data=with_data)
    return lay, mi, disc, O.scale(tx), tc, tn


def _engine_from(mi, disc, tx, tc, tn, with_data=True):
    eng = N.Engine(0)
    eng.set_dataset(tc, tn, tx if with_data else None)
    mods = mi.mods_present
    node_off = np.concatenate([[0], np.cumsum([mi.test_idx[m].size for m in mods])])
    eng.set_modules(len(mi.modules), [mi.modules.index(m) for m in mods], node_off,
                    np.concatenate([mi.test_idx[m] for m in mods]),
                    np.concatenate([mi.null_pos[m] for m in mods]),
                    np.concatenate([disc["corr"][m] for m in mods]),
                    np.concatenate([disc["degree"][m] for m in mods]),
                    np.concatenate([disc["contribution"][m] for m in mods]) if with_data else None)
    eng.set_null_pool(mi.null_idx)
    return eng


def test_export_indices_match_oracle():
    lay, mi, disc, tx, tc, tn = _engine_case()
    eng = _engine_from(mi, disc, tx, tc, tn)
    seed = 99
    idx = eng.export_indices(10, 14, seed)
    for p in range(10, 14):
        pi = prp.permute(np.arange(mi.null_idx.size), mi.null_idx.size, seed, p)
        ref = np.concatenate([mi.random_idx(pi)[m] for m in mi.mods_present])
        np.testing.assert_array_equal(idx[p - 10], ref)


@pytest.mark.parametrize("with_data", [True, False])
def test_engine_synthetic_vs_oracle(with_data):
    lay, mi, disc, tx, tc, tn = _engine_case(with_data=with_data)
    eng = _engine_from(mi, disc, tx, tc, tn, with_data)
    assert eng.symmetric()
    seed = 1234
    nulls = eng.run(0, 6, seed)
    pis = np.stack([prp.permute(np.arange(mi.null_idx.size), mi.null_idx.size, seed, p) for p in range(6)])
    exp, obs = O.permutation_procedure(disc, tx, tc, tn, mi, pis.astype(np.int64), with_data=with_data)
    assert_stats_close(eng.observed(), obs, what="observed")
    assert_stats_close(nulls, exp, what="nulls")


def test_batching_and_sharding_are_bitwise_invariant():
    lay, mi, disc, tx, tc, tn = _engine_case()
    eng = _engine_from(mi, disc, tx, tc, tn)
    whole = eng.run(0, 24, 5)
    eng.set_batch(5)
    parts = np.concatenate([eng.run(0, 10, 5), eng.run(10, 17, 5), eng.run(17, 24, 5)], axis=2)
    np.testing.assert_array_equal(whole.view(np.uint64), parts.view(np.uint64))
    d, t = eng.progress()
    assert d == t == 7


def test_observed_async_beside_run():
    """nr_observed_async runs the observed statistics on the context's second
    stream beside the permutation batches (two batches in flight on the
    first): both results are bitwise those of the serial calls, and a pending
    result is dropped by a change of null pool."""
    lay, mi, disc, tx, tc, tn = _engine_case()
    eng = _engine_from(mi, disc, tx, tc, tn)
    obs = eng.observed()
    eng.set_batch(5)
    serial = eng.run(0, 24, 5)
    eng.observed_async()
    nulls = eng.run(0, 24, 5)
    got = eng.observed_wait()
    np.testing.assert_array_equal(got.view(np.uint64), obs.view(np.uint64))
    np.testing.assert_array_equal(nulls.view(np.uint64), serial.view(np.uint64))
    with pytest.raises(N.NetRepError):
        eng.observed_wait()            # nothing pending any more
    eng.observed_async()
    eng.set_null_pool(np.arange(eng.shape()[0], dtype=np.int32))
    with pytest.raises(N.NetRepError):
        eng.observed_wait()            # dropped by the new null pool


def test_lanczos_path_vs_oracle():
    """The one Lanczos path -- start G e_c* (kernels.hip start_column), fp32
    matvecs once the residual drops below 1e-7 theta, the Ritz vector's G v
    from the Lanczos relation -- keeps the parity bar on primal (k <= S) and
    dual (k > S) Grams in one launch, and is bitwise reproducible. (Round 2
    tested each of these on and off through run-time switches; those are gone.)"""
    lay, mi, disc, tx, tc, tn = _engine_case(n_samples=60, sizes=(30, 45, 60, 80, 120))
    eng = _engine_from(mi, disc, tx, tc, tn)
    seed = 91
    nulls = eng.run(0, 8, seed)
    pis = np.stack([prp.permute(np.arange(mi.null_idx.size), mi.null_idx.size, seed, p) for p in range(8)])
    exp, _ = O.permutation_procedure(disc, tx, tc, tn, mi, pis.astype(np.int64))
    assert_stats_close(nulls, exp, what="nulls")
    again = eng.run(0, 8, seed)
    assert np.array_equal(nulls.view(np.uint64), again.view(np.uint64))


def test_constant_column_gives_na():
    """A node with constant data scales to NaN; summary-profile stats of any module
    containing it become NA (svd_econ failure path, src/netStats.cpp:229-235)."""
    lay, mi, disc, tx, tc, tn = _engine_case()
    tx = tx.copy()
    m0 = mi.mods_present[0]
    tx[:, mi.test_idx[m0][0]] = np.nan
    eng = _engine_from(mi, disc, tx, tc, tn)
    obs = eng.observed()
    _, exp = O.permutation_procedure(disc, tx, tc, tn, mi, np.zeros((0, mi.null_idx.size), int))
    assert_stats_close(obs, exp, what="observed with NaN column")
    assert not np.isfinite(obs[0, [1, 4, 6]]).any()


@pytest.mark.parametrize("seed", [11])
def test_large_modules_vs_cpp_oracle(seed):
    """C3-like module sizes (k up to 300, S = 200) on a 4,000-node dataset:
    the Lanczos eigen-solver path at the sizes the benchmark runs, checked
    against the C++ restatement (LAPACK dgesvd) on identical shuffles."""
    from netrep_amd import synthetic as S
    from oracle import ref_cpp
    sizes = [300, 260, 200, 150, 90, 40, 31]
    lay = S.make_layout(4000, sizes, seed)
    dx, dc, dn = S.numpy_dataset(lay, 200, seed + 1)
    tx, tc, tn = S.numpy_dataset(lay, 200, seed + 2, preserve_all=False)
    mi = O.ModuleIndex(lay.names, lay.labels, lay.names, lay.modules)
    disc = O.intermediate_properties(O.scale(dx), dc, dn, mi.disc_idx(lay.names))
    txs = O.scale(tx)
    eng = _engine_from(mi, disc, txs, tc, tn)
    seed_p = 2024
    nulls = eng.run(100, 106, seed_p)
    pis = N.prp_table(seed_p, 100, 106, mi.null_idx.size)
    mods = mi.mods_present
    node_off = np.concatenate([[0], np.cumsum([mi.test_idx[m].size for m in mods])])
    exp, obs = ref_cpp.permutation_procedure(
        txs, tc, tn, len(mi.modules), [mi.modules.index(m) for m in mods], node_off,
        np.concatenate([mi.test_idx[m] for m in mods]), np.concatenate([mi.null_pos[m] for m in mods]),
        mi.null_idx, np.concatenate([disc["corr"][m] for m in mods]),
        np.concatenate([disc["degree"][m] for m in mods]),
        np.concatenate([disc["contribution"][m] for m in mods]), 6, pi=pis, n_threads=8)
    assert_stats_close(eng.observed(), obs, what="observed (large modules)")
    assert_stats_close(nulls, exp, what="nulls (large modules)")


def test_c5_sized_modules_vs_cpp_oracle():
    """C5-shaped modules (BASELINE configs[4]: up to 2,000 nodes at S = 1,000,
    so k > S): the large-module layout (full Gram, matvec partials in global
    scratch, 320-vector Lanczos basis, network statistics as their own
    kernel) against the C++ restatement (LAPACK dgesvd) on identical shuffles,
    observed values through IntermediateProperties-shaped discovery vectors."""
    from netrep_amd import synthetic as S
    from oracle import ref_cpp
    seed = 31
    sizes = [2000, 1100, 600, 250]
    lay = S.make_layout(7000, sizes, seed)
    dx, dc, dn = S.numpy_dataset(lay, 1000, seed + 1)
    tx, tc, tn = S.numpy_dataset(lay, 1000, seed + 2, preserve_all=False)
    mi = O.ModuleIndex(lay.names, lay.labels, lay.names, lay.modules)
    disc = O.intermediate_properties(O.scale(dx), dc, dn, mi.disc_idx(lay.names))
    txs = O.scale(tx)
    eng = _engine_from(mi, disc, txs, tc, tn)
    seed_p = 77
    nulls = eng.run(0, 4, seed_p)
    pis = N.prp_table(seed_p, 0, 4, mi.null_idx.size)
    mods = mi.mods_present
    node_off = np.concatenate([[0], np.cumsum([mi.test_idx[m].size for m in mods])])
    exp, obs = ref_cpp.permutation_procedure(
        txs, tc, tn, len(mi.modules), [mi.modules.index(m) for m in mods], node_off,
        np.concatenate([mi.test_idx[m] for m in mods]), np.concatenate([mi.null_pos[m] for m in mods]),
        mi.null_idx, np.concatenate([disc["corr"][m] for m in mods]),
        np.concatenate([disc["degree"][m] for m in mods]),
        np.concatenate([disc["contribution"][m] for m in mods]), 4, pi=pis, n_threads=8)
    assert_stats_close(eng.observed(), obs, what="observed (C5-sized modules)")
    assert_stats_close(nulls, exp, what="nulls (C5-sized modules)")


def test_netprops_one_node_and_absent_modules(bundled):
    """NetProps keeps AverageEdgeWeight's 0/0 = NaN for a one-node module
    (src/properties.cpp:121, no NaN->NA step for it) and leaves modules with no
    nodes present NA throughout (:86-90)."""
    d, ma, t_names = bundled_inputs(bundled)
    ma = dict(ma)
    first = t_names[0]
    ma[first] = "solo"                       # a one-node module
    ma["not_in_data_1"] = "ghost"            # a module with no node present
    ma["not_in_data_2"] = "ghost"
    mods = ["1", "solo", "ghost"]
    got = N.NetProps(d["tData"], d["tNet"], ma, mods)
    module_nodes = {m: [n for n, l in ma.items() if l == m] for m in mods}
    exp = O.net_props(d["tData"].values, d["tNet"].values, t_names, module_nodes, mods)
    for m in mods:
        for key in ("summary", "contribution", "degree"):
            assert_stats_close(got[m][key], exp[m][key], what=f"{m}/{key}")
        assert_stats_close([got[m]["coherence"]], [exp[m]["coherence"]], what=f"{m}/coherence")
        assert_stats_close([got[m]["avgWeight"]], [exp[m]["avgWeight"]], what=f"{m}/avgWeight")
    assert np.isnan(got["solo"]["avgWeight"])
    na = np.uint64(0x7FF00000000007A2)
    assert np.float64(got["solo"]["avgWeight"]).view(np.uint64) != na
    assert np.float64(got["ghost"]["avgWeight"]).view(np.uint64) == na


def test_upload_check_finite_fused():
    """CheckFinite (src/checkFinite.cpp:21-28) folded into the upload's symmetry
    pass: per-matrix flags vs numpy's isfinite, on ragged (non-multiple-of-32)
    sizes and with the bad element in either triangle or on the diagonal."""
    rng = np.random.default_rng(77)
    for n, where, what in ((45, (3, 40), "corr"), (45, (40, 3), "net"), (33, (32, 32), "net"),
                           (70, (0, 69), "corr"), (1, (0, 0), "corr"), (64, None, None)):
        a = rng.standard_normal((n, n))
        corr = (a + a.T) / 2
        net = np.abs(corr) ** 5
        bad = np.inf if what == "corr" else np.nan
        if where is not None:
            (corr if what == "corr" else net)[where] = bad
        eng = N.Engine(0)
        try:
            eng.set_dataset(corr, net)
            assert eng.finite() == (bool(np.isfinite(corr).all()), bool(np.isfinite(net).all())), (n, where)
            # exact comparison, so a NaN (even on the diagonal) reads as asymmetric
            sym = np.array_equal(corr, corr.T) and np.array_equal(net, net.T)
            assert eng.symmetric() == sym, (n, where)
        finally:
            eng.close()
