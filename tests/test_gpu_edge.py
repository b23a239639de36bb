"""Edge shapes against the numpy oracle: one-, two- and three-node modules
(CorrVector of 0 or 1 pair, AverageEdgeWeight 0/0, a 1-dimensional Lanczos),
modules larger than a tiny sample count (the dual Gram with S = 3..5), and
module sizes around the 16/32/64 tile and row-block boundaries.

Three statistics of a two-node module are rounding noise in the reference
itself and are not compared: its two node contributions are equal up to the
last bit (scaled columns of equal norm are symmetric about the first left
singular vector), so cor.contrib divides two roundoff-sized numbers, and when
the first singular vector is the columns' difference the orientation test
(cor(rowMeans, u), src/netStats.cpp:242-247) is itself roundoff, which flips
avg.contrib's sign or leaves it a difference of equal numbers; its two
weighted degrees are the same |net| entry, so cor.degree is noise too."""
import numpy as np
import pytest

from oracle import prp
from oracle import netrep_oracle as O

from conftest import assert_stats_close
from test_gpu_parity import _engine_case, _engine_from

pytestmark = pytest.mark.gpu


def _mask_two_node_noise(a, mi):
    a = a.copy()
    # cor.degree, cor.contrib, avg.contrib of two-node modules
    for m in mi.mods_present:
        if mi.test_idx[m].size == 2:
            a[mi.modules.index(m), [3, 4, 6], ...] = 0.0
    return a


@pytest.mark.parametrize("n_samples,sizes", [
    (3, (1, 2, 3, 5)),
    (4, (2, 3, 4, 9)),
    (5, (1, 4, 6, 40)),
    (40, (2, 15, 16, 17, 31, 32, 33, 63, 64, 65)),
])
def test_small_and_boundary_modules_vs_oracle(n_samples, sizes):
    lay, mi, disc, tx, tc, tn = _engine_case(n_nodes=400, n_samples=n_samples, sizes=sizes, seed=3)
    eng = _engine_from(mi, disc, tx, tc, tn)
    seed = 77
    nulls = eng.run(0, 8, seed)
    pis = np.stack([prp.permute(np.arange(mi.null_idx.size), mi.null_idx.size, seed, p) for p in range(8)])
    exp, obs = O.permutation_procedure(disc, tx, tc, tn, mi, pis.astype(np.int64))
    assert_stats_close(_mask_two_node_noise(eng.observed(), mi), _mask_two_node_noise(obs, mi),
                       what=f"observed S={n_samples} {sizes}")
    assert_stats_close(_mask_two_node_noise(nulls, mi), _mask_two_node_noise(exp, mi),
                       what=f"nulls S={n_samples} {sizes}")


@pytest.mark.parametrize("nonfinite", [False, True])
def test_wide_modules_sixteen_lane_sweep_vs_oracle(nonfinite):
    """Modules beyond kSweepWideK (1,024) nodes take the column sweep's
    sixteen-lane path (sweep.hip, the C5 shape): finite data, and with a NaN
    test correlation inside the wide module (the complete-case records)."""
    lay, mi, disc, tx, tc, tn = _engine_case(n_nodes=2600, n_samples=20, sizes=(1100, 40), seed=5)
    if nonfinite:
        m0 = max(mi.mods_present, key=lambda m: mi.test_idx[m].size)
        a, b = mi.test_idx[m0][3], mi.test_idx[m0][10]
        tc = tc.copy()
        tc[a, b] = tc[b, a] = np.nan
    eng = _engine_from(mi, disc, tx, tc, tn)
    seed = 31
    nulls = eng.run(0, 4, seed)
    pis = np.stack([prp.permute(np.arange(mi.null_idx.size), mi.null_idx.size, seed, p) for p in range(4)])
    exp, obs = O.permutation_procedure(disc, tx, tc, tn, mi, pis.astype(np.int64))
    assert_stats_close(eng.observed(), obs, what=f"observed, wide modules, nonfinite={nonfinite}")
    assert_stats_close(nulls, exp, what=f"nulls, wide modules, nonfinite={nonfinite}")
