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
    ct = CT.contingencyTable([disc, test], ["1", "2", "3", "7"], test_nodes)
    assert ct["varsPres"]["7"] == 0
    assert sum(ct["varsPres"].values()) == 6
    mat, rows, cols = ct["contingency"]
    assert rows[:2] == ["size", "present"] and cols[:2] == ["size", "present"]
    # every overlapping node is counted once in the body of the table
    assert np.nansum(mat[2:, 2:]) == 6


def test_bench_traffic_lookup_matches_committed_pmc():
    """bench.py reports `roofline.traffic` only from a PMC pass of the same
    config, batch and kernel (profiles/pmc_traffic.json)."""
    import bench
    t = bench.measured_traffic("C3", 256, "module_profile_kernel")
    assert t is not None and t > 0
    assert bench.measured_traffic("C3", 512, "module_profile_kernel") is None
    assert bench.measured_traffic("C2", 256, "module_profile_kernel") is None
