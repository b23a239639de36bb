"""The small-dimension summary-profile classes. The wave class (kernels.h
kWaveDim, round 5) takes every launch whose Lanczos dimension min(k, S) is at
most 111: one wave per item, the Gram in its MFMA accumulator registers,
per-node arrays of modules longer than 112 nodes in the slot's scratch. The
small class (kSmallDim: two-wave workgroups, packed Gram in scratch) keeps a
dimension of exactly 112. Both are checked against the C++ LAPACK restatement
on identical shuffles: the wave class at S = 60 (dual items with per-node
arrays in scratch (200, 113) and in LDS (112, 61), k == S, primal items) and
through the non-finite path; the small class with a 112-node primal module at
S = 300. Also the packed 4-wave kernel's dual path at an S just above both
classes, and the large-module kernel (64 x 64 super-tile Gram) on primal and
dual modules, with non-finite columns."""
import numpy as np
import pytest

import netrep_amd as N
from oracle import netrep_oracle as O

from conftest import assert_stats_close
from test_gpu_dual import _case, _cpp
from test_gpu_parity import _engine_from

pytestmark = pytest.mark.gpu


def test_small_class_edges_vs_cpp_oracle():
    """S = 60 (the wave class): dual items with per-node arrays in scratch
    (200, 113 > 112), in LDS (112, 61), k == S and primal items (59, 7)."""
    lay, mi, disc, txs, tc, tn = _case([200, 113, 112, 61, 60, 59, 7], 60, 71, n_nodes=1500)
    eng = _engine_from(mi, disc, txs, tc, tn)
    nulls = eng.run(5, 29, 123)
    pis = N.prp_table(123, 5, 29, mi.null_idx.size)
    exp, obs = _cpp(mi, disc, txs, tc, tn, pis)
    assert_stats_close(eng.observed(), obs, what="observed (small class)")
    assert_stats_close(nulls, exp, what="nulls (small class)")


def test_small_class_primal_only_vs_cpp_oracle():
    """S = 300 with every module of at most 112 nodes: the 112-node module
    puts the launch on the small class (Lanczos dimension 112 > kWaveDim),
    primal items only."""
    lay, mi, disc, txs, tc, tn = _case([112, 96, 64, 33, 16], 300, 73, n_nodes=1200)
    eng = _engine_from(mi, disc, txs, tc, tn)
    nulls = eng.run(0, 16, 5)
    # small-class launch: no fused packed segment, so no Gram table
    assert not eng.gram_table()
    pis = N.prp_table(5, 0, 16, mi.null_idx.size)
    exp, obs = _cpp(mi, disc, txs, tc, tn, pis)
    assert_stats_close(eng.observed(), obs, what="observed (small class, primal)")
    assert_stats_close(nulls, exp, what="nulls (small class, primal)")


def test_small_class_nonfinite_column_gives_na():
    """A NaN data column of a module's node: that module's summary-profile
    statistics are NA (src/netStats.cpp:229-235) on the wave class too."""
    lay, mi, disc, txs, tc, tn = _case([150, 40, 20], 50, 75, n_nodes=600)
    txs = txs.copy()
    m0 = mi.mods_present[0]
    txs[:, mi.test_idx[m0][3]] = np.nan
    eng = _engine_from(mi, disc, txs, tc, tn)
    obs = eng.observed()
    _, exp = O.permutation_procedure(disc, txs, tc, tn, mi, np.zeros((0, mi.null_idx.size), int))
    assert_stats_close(obs, exp, what="observed with NaN column (small class)")
    assert not np.isfinite(obs[0, [1, 4, 6]]).any()


def test_packed_dual_above_small_class_vs_cpp_oracle():
    """S = 150 (> 112): dual items (k > S) stay on the packed 4-wave kernel."""
    lay, mi, disc, txs, tc, tn = _case([300, 220, 151, 150, 90], 150, 77, n_nodes=2000)
    eng = _engine_from(mi, disc, txs, tc, tn)
    nulls = eng.run(2, 14, 9)
    pis = N.prp_table(9, 2, 14, mi.null_idx.size)
    exp, obs = _cpp(mi, disc, txs, tc, tn, pis)
    assert_stats_close(eng.observed(), obs, what="observed (packed dual)")
    assert_stats_close(nulls, exp, what="nulls (packed dual)")


def test_large_module_kernel_nonfinite_column_gives_na():
    """The large-module kernel (64 x 64 super-tile Gram, one workgroup per CU
    at S = 600): a NaN data column in a dual (950-node) and in a primal
    (580-node) module gives NA summary-profile statistics for those two only."""
    lay, mi, disc, txs, tc, tn = _case([950, 580, 60], 600, 79, n_nodes=3000)
    txs = txs.copy()
    m0, m1 = mi.mods_present[0], mi.mods_present[1]
    txs[:, mi.test_idx[m0][5]] = np.nan
    txs[:, mi.test_idx[m1][7]] = np.nan
    eng = _engine_from(mi, disc, txs, tc, tn)
    obs = eng.observed()
    _, exp = O.permutation_procedure(disc, txs, tc, tn, mi, np.zeros((0, mi.null_idx.size), int))
    assert_stats_close(obs, exp, what="observed with NaN columns (large modules)")
    for m in (m0, m1):
        assert not np.isfinite(obs[mi.mods_present.index(m), [1, 4, 6]]).any()
    assert np.isfinite(obs[mi.mods_present.index(mi.mods_present[2]), [1, 4, 6]]).all()


def test_large_module_kernel_vs_cpp_oracle():
    """S = 600: primal large modules whose Gram side is not a multiple of 64
    (330, 577) and a dual one (905) on the large-module kernel."""
    lay, mi, disc, txs, tc, tn = _case([905, 577, 330, 120], 600, 81, n_nodes=3000)
    eng = _engine_from(mi, disc, txs, tc, tn)
    nulls = eng.run(0, 6, 31)
    pis = N.prp_table(31, 0, 6, mi.null_idx.size)
    exp, obs = _cpp(mi, disc, txs, tc, tn, pis)
    assert_stats_close(eng.observed(), obs, what="observed (large-module kernel)")
    assert_stats_close(nulls, exp, what="nulls (large-module kernel)")
