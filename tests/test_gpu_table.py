"""The Gram table (engine.hip maybe_build_table): the data block's whole Gram
X^T X interleaved with {corr, net}, so that packed summary-profile items take
their network statistics and their Gram from one 32-byte gather per pair
(no separate network launch, no per-item matrix-core Gram). Checked against
the oracles on identical shuffles: all modules on the table path, a mix
with a module beyond the packed layout (its network statistics from the
network kernel reading the table layout), an asymmetric network (net^T from
the table's fourth slot) and a non-finite data column."""
import numpy as np
import pytest

import netrep_amd as N
from oracle import netrep_oracle as O

from conftest import assert_stats_close
from test_gpu_dual import _case, _cpp
from test_gpu_parity import _engine_from

pytestmark = pytest.mark.gpu


def _net_launch_items(eng):
    ms, launches, items = eng.timing(0)
    return launches, items


def test_table_all_packed_vs_cpp_oracle():
    """k <= 300 <= S: every module on the table path; the network kernel does
    not run at all."""
    lay, mi, disc, txs, tc, tn = _case([300, 240, 170, 120, 75, 44, 30], 320, 31, n_nodes=2500)
    eng = _engine_from(mi, disc, txs, tc, tn)
    eng.set_timing(True)
    eng.reset_timing()
    nulls = eng.run(5, 21, 13)
    assert eng.gram_table()
    assert _net_launch_items(eng) == (0, 0)
    pis = N.prp_table(13, 5, 21, mi.null_idx.size)
    exp, obs = _cpp(mi, disc, txs, tc, tn, pis)
    assert_stats_close(eng.observed(), obs, what="observed (table)")
    assert_stats_close(nulls, exp, what="nulls (table)")
    again = eng.run(5, 21, 13)
    assert np.array_equal(nulls.view(np.uint64), again.view(np.uint64))


def test_table_with_module_beyond_packed_layout():
    """A 350-node module (full-Gram launch, network kernel on the table
    layout) beside eight 130-node modules on the table path."""
    lay, mi, disc, txs, tc, tn = _case([350] + [130] * 8, 400, 37, n_nodes=2600)
    eng = _engine_from(mi, disc, txs, tc, tn)
    eng.set_timing(True)
    eng.reset_timing()
    nulls = eng.run(0, 6, 3)
    assert eng.gram_table()
    launches, items = _net_launch_items(eng)
    assert launches >= 1 and items == 6          # the 350-node module only
    pis = N.prp_table(3, 0, 6, mi.null_idx.size)
    exp, obs = _cpp(mi, disc, txs, tc, tn, pis)
    assert_stats_close(eng.observed(), obs, what="observed (table, mixed)")
    assert_stats_close(nulls, exp, what="nulls (table, mixed)")


def test_table_asymmetric_network_vs_oracle():
    """net(i, j) != net(j, i): the weighted degrees read net^T from the
    table's fourth slot."""
    lay, mi, disc, txs, tc, tn = _case([150, 60, 33], 160, 41, n_nodes=500)
    rng = np.random.default_rng(5)
    tna = tn * (1.0 + 0.05 * rng.random(tn.shape))      # no longer symmetric
    eng = _engine_from(mi, disc, txs, tc, tna)
    assert not eng.symmetric()
    eng.set_timing(True)
    eng.reset_timing()
    nulls = eng.run(0, 4, 77)
    assert _net_launch_items(eng) == (0, 0)
    pis = N.prp_table(77, 0, 4, mi.null_idx.size)
    exp, obs = O.permutation_procedure(disc, txs, tc, tna, mi, pis.astype(np.int64))
    assert_stats_close(eng.observed(), obs, what="observed (table, asymmetric)")
    assert_stats_close(nulls, exp, what="nulls (table, asymmetric)")


def test_table_nonfinite_column_gives_na():
    """A NaN data column shows on the table's diagonal: the module's
    summary-profile statistics are NA (src/netStats.cpp:229-235), its network
    statistics are not affected."""
    lay, mi, disc, txs, tc, tn = _case([130, 50, 31], 140, 43, n_nodes=500)
    txs = txs.copy()
    m0 = mi.mods_present[0]
    txs[:, mi.test_idx[m0][2]] = np.nan
    eng = _engine_from(mi, disc, txs, tc, tn)
    obs = eng.observed()
    _, exp = O.permutation_procedure(disc, txs, tc, tn, mi, np.zeros((0, mi.null_idx.size), int))
    assert_stats_close(obs, exp, what="observed with NaN column (table)")
    assert not np.isfinite(obs[0, [1, 4, 6]]).any()
    assert np.isfinite(obs[0, [0, 2, 3, 5]]).all()


def test_no_table_when_dual_items_in_packed_class():
    """S = 40 below the packed class's largest module (dual items): the
    per-item matrix-core Gram path, no table."""
    lay, mi, disc, txs, tc, tn = _case([120, 60, 30], 40, 47, n_nodes=400)
    eng = _engine_from(mi, disc, txs, tc, tn)
    eng.run(0, 2, 1)
    assert not eng.gram_table()
