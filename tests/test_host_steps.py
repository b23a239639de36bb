"""CPU: host consumers of the nulls cube -- permutationTest/permp (R/pperm.R)
and contingencyTable (R/contingency.R)."""
import numpy as np
import pytest

from netrep_amd import contingency as CT
from netrep_amd import pvalues as PV
from oracle import netrep_oracle as O


def test_permp_vignette_floor():
    # vignettes/NetRep.md:315,318: observed beyond every null at nPerm = 10000
    p = PV.permp(0, 10000, total_nperm=1e40)
    assert f"{p:.8f}" == "0.00009999"


def test_permp_fallback_limit_and_exact():
    # large total.nperm: integral vanishes -> (x+1)/(nperm+1)
    assert PV.permp(37, 1000, 1e30) == pytest.approx(38 / 1001, rel=1e-15)
    # exact branch (total.nperm <= 10000) is a mean of binomial cdfs
    from scipy.stats import binom
    t = 50
    exp = binom.cdf(3, 100, np.arange(1, t + 1) / t).sum() / t
    assert PV.permp(3, 100, t) == pytest.approx(exp, rel=1e-14)
    # approximate branch stays below the biased estimator
    assert PV.permp(0, 100, 20000) < 1 / 101


def test_extreme_counts_drop_na_and_ties():
    nulls = np.array([[[0.1, 0.5, np.nan, 0.5, 0.9]]])
    obs = np.array([[0.5]])
    less, more, n = PV.extreme_counts(nulls, obs)
    assert (less[0, 0], more[0, 0], n[0, 0]) == (3, 3, 4)


def test_permutation_test_shapes_and_alternatives():
    rng = np.random.default_rng(3)
    nulls = rng.standard_normal((3, 7, 200))
    obs = np.array([[10.0] * 7, [-10.0] * 7, [0.0] * 7])
    obs[2, 3] = np.nan
    p_g = PV.permutationTest(nulls, obs, [20, 30, 40], 150, "greater")
    p_l = PV.permutationTest(nulls, obs, [20, 30, 40], 150, "less")
    p_2 = PV.permutationTest(nulls, obs, [20, 30, 40], 150, "two.sided")
    assert p_g.shape == (3, 7)
    assert np.allclose(p_g[0], 1 / 201) and np.allclose(p_l[1], 1 / 201)
    assert np.isnan(p_g[2, 3])
    assert np.allclose(p_2[0], 2 / 201)


def test_required_perms():
    assert PV.requiredPerms(0.05 / 4) == pytest.approx(80)
    assert PV.requiredPerms(0.01, "two.sided") == pytest.approx(200)


def test_contingency_bundled(bundled):
    b = bundled
    ma = dict(zip(b["module_labels_names"].tolist(), b["module_labels"].tolist()))
    ct = CT.contingencyTable([ma, None], ["1", "2", "3", "4"], b["test_network_colnames"].tolist())
    assert list(ct["varsPres"].items()) == [("1", 20), ("2", 25), ("3", 30), ("4", 35)]
    assert all(v == 1.0 for v in ct["propVarsPres"].values())
    assert len(ct["overlapVars"]) == 150
    assert CT.total_size("overlap", ct["overlapVars"], 150) == 150


def test_contingency_partial_overlap_and_test_modules():
    disc = {f"N_{i}": str(1 + i % 3) for i in range(1, 13)}
    test_nodes = [f"N_{i}" for i in range(1, 13, 2)] + ["X_1"]
    test = {n: ("a" if i % 2 else "b") for i, n in enumerate(test_nodes)}
    # a requested module with no discovery node: varsPres 0, propVarsPres NA
    # without test assignments; with them R fails at contingency[mods,,]
    # (R/contingency.R:95), as test_contingency_module_absent_from_discovery checks
    ct7 = CT.contingencyTable([disc, None], ["1", "2", "3", "7"], test_nodes)
    assert ct7["varsPres"]["7"] == 0 and np.isnan(ct7["propVarsPres"]["7"])
    ct = CT.contingencyTable([disc, test], ["1", "2", "3"], test_nodes)
    assert sum(ct["varsPres"].values()) == 6
    mat, rows, cols = ct["contingency"]
    assert rows[:2] == ["size", "present"] and cols[:2] == ["size", "present"]
    # every overlapping node is counted once in the body of the table
    assert np.nansum(mat[2:, 2:]) == 6


def test_bench_traffic_lookup_matches_committed_pmc():
    """bench.py reports `roofline.traffic` only from a PMC pass of the same
    config, batch and kernel (profiles/pmc_traffic.json), as a [raw, x2] range
    with the pass's kernel time next to this run's (traffic_time_ratio)."""
    import bench
    t = bench.traffic_fields("C3", 5120, "module_profile_kernel", 247.3, table=True)
    assert t["traffic"] is not None and t["traffic"] > 0
    raw, x2 = t["traffic_range"]
    assert 0 < raw <= x2 == t["traffic"]
    assert abs(t["traffic_time_ratio"] - 1.0) < 0.01     # the r06 final-tree pass: 247.90 ms
    # superseded rows (passes of kernels since replaced) are never reported
    assert bench.traffic_fields("C3", 256, "module_profile_kernel", 17.9)["traffic"] is None
    assert bench.traffic_fields("C3", 512, "module_profile_kernel", 1.0)["traffic"] is None
    assert bench.traffic_fields("C2", 256, "module_profile_kernel", 1.0)["traffic"] is None
    # a launch within 10% of a pass's size (the reference interface sizes
    # its own launches, e.g. 66 permutations at C5): the pass scaled by the
    # size, marked
    t64 = bench.traffic_fields("C5", 64, "module_profile_kernel", 50.0)   # the three-dataset pass
    t66 = bench.traffic_fields("C5", 66, "module_profile_kernel", 50.0)
    assert "traffic_scaled_from_batch" not in t64 and t66["traffic_scaled_from_batch"] == 64
    assert abs(t66["traffic"] / t64["traffic"] - 66 / 64) < 1e-12
    assert bench.traffic_fields("C5", 80, "module_profile_kernel", 50.0)["traffic"] is None  # > 10% off


def test_vars_present_aligned_by_label_from_contingency():
    """contingencyTable's varsPres (ordered by orderAsNumeric) chained
    into permutationTest with rows in another order: counts follow the labels,
    a label mismatch raises the reference's error (R/pperm.R:106-111)."""
    from netrep_amd.contingency import contingencyTable
    ma = {f"n{i}": lab for i, lab in enumerate(["10"] * 5 + ["2"] * 3 + ["0"] * 4)}
    ct = contingencyTable([ma, None], ["10", "2"], list(ma))
    assert list(ct["varsPres"]) == ["2", "10"]            # orderAsNumeric
    rng = np.random.default_rng(3)
    nulls = rng.standard_normal((2, 7, 200))
    obs = rng.standard_normal((2, 7))
    rows = ["10", "2"]
    got = PV.permutationTest(nulls, obs, ct["varsPres"], 12, "greater", modules=rows)
    exp = PV.permutationTest(nulls, obs, [5, 3], 12, "greater")
    np.testing.assert_array_equal(got, exp)
    with pytest.raises(ValueError, match="nVarsPresent"):
        PV.permutationTest(nulls, obs, ct["varsPres"], 12, "greater", modules=["10", "7"])
    with pytest.raises(ValueError, match="modules="):
        PV.permutationTest(nulls, obs, ct["varsPres"], 12, "greater")


def test_order_as_numeric_follows_r_as_integer():
    from netrep_amd.contingency import order_as_numeric
    assert order_as_numeric(["10", "2", "1.0", "1e1"]) == ["1.0", "2", "10", "1e1"]
    assert order_as_numeric(["b", "10", "a"]) == ["10", "a", "b"]      # as.integer warns -> character order


def test_contingency_module_absent_from_discovery():
    from netrep_amd.contingency import contingencyTable
    ma = {"a": "1", "b": "1", "c": "2"}
    ct = contingencyTable([ma, None], ["1", "3"], ["a", "b", "c"])
    assert ct["varsPres"]["3"] == 0 and np.isnan(ct["propVarsPres"]["3"])
    with pytest.raises(ValueError, match="subscript out of bounds"):
        contingencyTable([ma, {"a": "x", "b": "y", "c": "x"}], ["1", "3"], ["a", "b", "c"])
