"""CPU tests: pin the oracle to the reference's own known answers, and check the
host-side logic (keyed permutations, index derivation) it shares with the engine."""
import numpy as np
import pytest

from oracle import netrep_oracle as O
from oracle import prp

# vignettes/NetRep.md:301-307 -- observed statistics on the bundled data
VIGNETTE_OBSERVED = np.array([
    [0.161069393, 0.6187688, 0.78448573, 0.90843993, 0.8795006, 0.550004272, 0.76084777],
    [0.001872928, 0.1359063, 0.17270312, -0.03542772, 0.5390504, 0.034040922, 0.23124826],
    [0.001957475, 0.1263280, 0.01121223, -0.17179855, -0.1074944, -0.007631867, 0.05412794],
    [0.046291489, 0.4871179, 0.32610667, 0.68122446, 0.5251965, 0.442614173, 0.68239136],
])
# vignettes/NetRep.md:913-958 -- summary profile of module 1 (first 7 samples) and coherence
VIGNETTE_SP_DISC = [-0.15173019, -0.09817810, -0.10356266, -0.21351111, -0.06424053, -0.25787365, -0.06191222]
VIGNETTE_SP_TEST = [-0.099957918, 0.061501299, 0.043541623, 0.051055323, 0.056572949, 0.136605203, 0.116491092]
VIGNETTE_COH = (0.585781, 0.6187688)


def _printed_close(a, b):
    # the vignette prints 7-9 significant digits
    return np.allclose(a, b, rtol=5e-7, atol=5e-9)


def _bundled_case(b):
    return dict(ma_names=list(b["module_labels_names"]), ma_labels=list(b["module_labels"]),
                t_names=list(b["test_network_colnames"]), d_names=list(b["discovery_network_colnames"]))


def test_vignette_observed_statistics(bundled):
    b = bundled
    c = _bundled_case(b)
    mi = O.ModuleIndex(c["ma_names"], c["ma_labels"], c["t_names"], ["1", "2", "3", "4"])
    disc = O.intermediate_properties(O.scale(b["discovery_data"]), b["discovery_correlation"],
                                     b["discovery_network"], mi.disc_idx(c["d_names"]))
    _, obs = O.permutation_procedure(disc, O.scale(b["test_data"]), b["test_correlation"],
                                     b["test_network"], mi, np.zeros((0, mi.null_idx.size), int))
    assert _printed_close(obs, VIGNETTE_OBSERVED)


def test_vignette_summary_profiles(bundled):
    b = bundled
    c = _bundled_case(b)
    mod_nodes = {"1": [n for n, lab in zip(c["ma_names"], c["ma_labels"]) if lab == "1"]}
    pd = O.net_props(b["discovery_data"], b["discovery_network"], c["d_names"], mod_nodes, ["1"])["1"]
    pt = O.net_props(b["test_data"], b["test_network"], c["t_names"], mod_nodes, ["1"])["1"]
    assert _printed_close(pd["summary"][:7], VIGNETTE_SP_DISC)
    assert _printed_close(pt["summary"][:7], VIGNETTE_SP_TEST)
    assert abs(pd["coherence"] - VIGNETTE_COH[0]) < 5e-7
    assert abs(pt["coherence"] - VIGNETTE_COH[1]) < 5e-8


def test_vignette_pvalue_floor():
    # vignettes/NetRep.md:315,318: permp(0, 10000, .) printed as 0.00009999 ~ 1/(nPerm+1)
    assert abs(1 / 10001 - 0.00009999) < 1e-8


def test_golden_fixtures_reproduce(bundled, bundled_expected):
    """The committed expected outputs are what the oracle computes from the committed inputs."""
    b, e = bundled, bundled_expected
    c = _bundled_case(b)
    mi = O.ModuleIndex(c["ma_names"], c["ma_labels"], c["t_names"], ["1", "2", "3", "4"])
    disc = O.intermediate_properties(O.scale(b["discovery_data"]), b["discovery_correlation"],
                                     b["discovery_network"], mi.disc_idx(c["d_names"]), with_data=False)
    nulls, obs = O.permutation_procedure(disc, None, b["test_correlation"], b["test_network"], mi,
                                         e["pis"][:4].astype(np.int64), with_data=False)
    np.testing.assert_array_equal(obs.view(np.uint64), e["observed_nodata"].view(np.uint64))
    np.testing.assert_array_equal(nulls.view(np.uint64), e["nulls_nodata"][:, :, :4].view(np.uint64))


@pytest.mark.parametrize("n", [1, 2, 3, 5, 150, 1000, 4097, 65537])
def test_prp_is_a_permutation(n):
    for p in (0, 1, 12345):
        y = prp.permute(np.arange(n), n, 777, p)
        assert sorted(y.tolist()) == list(range(n))


def test_prp_c_matches_python():
    from netrep_amd import prp_table
    for n in (2, 150, 20000):
        t = prp_table(0xABCDEF, 3, 6, n)
        ref = np.stack([prp.permute(np.arange(n), n, 0xABCDEF, p) for p in range(3, 6)])
        np.testing.assert_array_equal(t, ref)


def test_prp_distribution_uniform():
    """pi_p(q) for a fixed q is uniform over [0, n) across permutations (chi-square)."""
    n, P = 50, 20000
    counts = np.zeros((3, n))
    for p in range(P):
        y = prp.permute(np.array([0, 7, 49]), n, 5, p)
        counts[np.arange(3), y] += 1
    exp = P / n
    chi2 = ((counts - exp) ** 2 / exp).sum(axis=1)
    # 49 dof: 99.9th percentile ~ 85.4
    assert (chi2 < 86).all(), chi2


def test_module_sets_disjoint_and_null_pool(bundled):
    b = bundled
    c = _bundled_case(b)
    for null in ("overlap", "all"):
        mi = O.ModuleIndex(c["ma_names"], c["ma_labels"], c["t_names"], ["1", "2", "3", "4", "9"], null=null)
        assert mi.mods_present == ["1", "2", "3", "4"]
        assert mi.null_idx.size == 150
        pi = prp.permute(np.arange(150), 150, 1, 0)
        sets = mi.random_idx(pi)
        allidx = np.concatenate(list(sets.values()))
        assert np.unique(allidx).size == allidx.size          # one shuffle shared by all modules


def test_sign_and_na_semantics():
    assert np.isnan(O.correlation([1.0], [2.0]))             # n = 1 -> 0/0
    assert np.isnan(O.correlation([np.nan, 1.0], [1.0, np.nan]))  # no complete cases
    assert O.sign_aware_mean([-1.0, 0.0, 2.0], [1.0, 5.0, 3.0]) == pytest.approx((-1 + 0 + 3) / 3)
    na = O.na_fill([np.nan, np.inf, 1.0])
    assert na.view(np.uint64)[0] == O.NA_REAL_BITS and na.view(np.uint64)[1] == O.NA_REAL_BITS
    assert np.isnan(O.average_edge_weight(np.array([0.0])))  # k = 1 -> 0/0


def test_svd_driver_gesvd_agrees_with_gesdd(bundled, asym):
    """arma::svd_econ(.., "left", "dc") runs dgesvd (Armadillo uses dgesdd only
    for mode "both"); the oracle follows it. Either driver's sign-oriented top
    left singular vector -- and so every summary-profile statistic -- agrees to
    1e-12 on the golden cases, so fixtures made with dgesdd stay valid."""
    import scipy.linalg
    cases = []
    b = bundled
    for key in ("discovery_data", "test_data"):
        x = O.scale(b[key])
        rng = np.random.default_rng(1)
        for k in (20, 35, 60):
            cases.append(x[:, np.sort(rng.choice(x.shape[1], k, replace=False))])
    xa = O.scale(asym["t_data"])
    cases.append(xa[:, :14])
    for x in cases:
        us = []
        for drv in ("gesvd", "gesdd"):
            u = scipy.linalg.svd(x, full_matrices=False, lapack_driver=drv)[0][:, 0]
            c = np.corrcoef(x.mean(axis=1), u)[0, 1]
            us.append(-u if c < 0 else u)
        assert np.abs(us[0] - us[1]).max() <= 1e-12
    assert O.SVD_DRIVER == "gesvd"
