"""The S x S (dual) Gram for modules with more nodes than samples (k > S):
Lanczos on H = [X' 1]'[X' 1] gives the summary profile u directly
(src/netStats.cpp:229-236 takes U.col(0) of svd_econ); node contributions
from one pass over the data. Checked against the C++ LAPACK restatement
(dgesvd of the S x k block) on identical shuffles, in vector mode (NetProps'
summary profiles), through the non-finite (svd failure) path, and on the
full-Gram layouts of modules beyond the packed kernel's 320-node layout."""
import numpy as np
import pytest

import netrep_amd as N
from oracle import netrep_oracle as O

from conftest import assert_stats_close
from test_gpu_parity import _engine_from

pytestmark = pytest.mark.gpu


def _case(sizes, n_samples, seed, n_nodes=3000):
    from netrep_amd import synthetic as S
    lay = S.make_layout(n_nodes, sizes, seed)
    dx, dc, dn = S.numpy_dataset(lay, n_samples, seed + 1)
    tx, tc, tn = S.numpy_dataset(lay, n_samples, seed + 2, preserve_all=False)
    mi = O.ModuleIndex(lay.names, lay.labels, lay.names, lay.modules)
    disc = O.intermediate_properties(O.scale(dx), dc, dn, mi.disc_idx(lay.names))
    return lay, mi, disc, O.scale(tx), tc, tn


def _cpp(mi, disc, txs, tc, tn, pis):
    from oracle import ref_cpp
    mods = mi.mods_present
    node_off = np.concatenate([[0], np.cumsum([mi.test_idx[m].size for m in mods])])
    return ref_cpp.permutation_procedure(
        txs, tc, tn, len(mi.modules), [mi.modules.index(m) for m in mods], node_off,
        np.concatenate([mi.test_idx[m] for m in mods]), np.concatenate([mi.null_pos[m] for m in mods]),
        mi.null_idx, np.concatenate([disc["corr"][m] for m in mods]),
        np.concatenate([disc["degree"][m] for m in mods]),
        np.concatenate([disc["contribution"][m] for m in mods]), pis.shape[0], pi=pis, n_threads=8)


def test_dual_gram_vs_cpp_oracle():
    """S = 40 with modules of 20-260 nodes: k > S (dual), k == S and k < S
    (primal) in one launch of the packed kernel."""
    lay, mi, disc, txs, tc, tn = _case([260, 180, 64, 41, 40, 39, 20], 40, 5)
    eng = _engine_from(mi, disc, txs, tc, tn)
    nulls = eng.run(10, 22, 99)
    pis = N.prp_table(99, 10, 22, mi.null_idx.size)
    exp, obs = _cpp(mi, disc, txs, tc, tn, pis)
    assert_stats_close(eng.observed(), obs, what="observed (dual)")
    assert_stats_close(nulls, exp, what="nulls (dual)")


def test_size_classes_vs_cpp_oracle():
    """Modules beyond the packed kernel's 320-node layout run in their own
    launch on the full-Gram layout (S = 400 > k: primal, full Gram; k > S:
    dual), the rest on the packed kernel -- one cube, every statistic at the
    parity bar."""
    lay, mi, disc, txs, tc, tn = _case([520, 350, 330, 300, 120, 45], 400, 21)
    eng = _engine_from(mi, disc, txs, tc, tn)
    nulls = eng.run(3, 11, 7)
    pis = N.prp_table(7, 3, 11, mi.null_idx.size)
    exp, obs = _cpp(mi, disc, txs, tc, tn, pis)
    assert_stats_close(eng.observed(), obs, what="observed (size classes)")
    assert_stats_close(nulls, exp, what="nulls (size classes)")


def test_dual_netprops_summary():
    """Vector mode (NetProps, src/properties.cpp): summary profile, node
    contributions and coherence of modules with k > S."""
    from netrep_amd.api import RMatrix
    lay, mi, disc, txs, tc, tn = _case([150, 90, 35], 30, 13, n_nodes=600)
    names = lay.names
    ma = dict(zip(names, lay.labels))
    got = N.NetProps(RMatrix(txs, None, names), RMatrix(tn, names, names), ma, lay.modules)
    module_nodes = {m: [n for n, l in ma.items() if l == m] for m in lay.modules}
    exp = O.net_props(txs, tn, names, module_nodes, lay.modules)
    for m in lay.modules:
        for key in ("summary", "contribution"):
            assert_stats_close(got[m][key], exp[m][key], what=f"{m}/{key}")
        assert_stats_close([got[m]["coherence"]], [exp[m]["coherence"]], what=f"{m}/coherence")


def test_dual_nonfinite_column_gives_na():
    """A NaN data column inside a k > S module: svd_econ fails, the module's
    summary-profile statistics are NA (src/netStats.cpp:229-235)."""
    lay, mi, disc, txs, tc, tn = _case([90, 25], 20, 17, n_nodes=400)
    txs = txs.copy()
    m0 = mi.mods_present[0]
    txs[:, mi.test_idx[m0][3]] = np.nan
    eng = _engine_from(mi, disc, txs, tc, tn)
    obs = eng.observed()
    _, exp = O.permutation_procedure(disc, txs, tc, tn, mi, np.zeros((0, mi.null_idx.size), int))
    assert_stats_close(obs, exp, what="observed with NaN column (dual)")
    row = mi.mods_present.index(m0)
    assert not np.isfinite(obs[row, [1, 4, 6]]).any()


def test_modules_beyond_lds_vs_cpp_oracle():
    """Modules of 2,500 and 3,000 nodes at S = 1,000 (no module cap, as
    src/netStats.cpp:217-280): the 3,000-node module exceeds the LDS vectors
    (its per-node arrays go to the slot's scratch) and both exceed the network
    kernel's LDS (global-scratch workgroups). Against the C++ LAPACK
    restatement on identical shuffles."""
    lay, mi, disc, txs, tc, tn = _case([3000, 2500, 400], 1000, 21, n_nodes=7000)
    eng = _engine_from(mi, disc, txs, tc, tn)
    nulls = eng.run(5, 7, 123)
    pis = N.prp_table(123, 5, 7, mi.null_idx.size)
    exp, obs = _cpp(mi, disc, txs, tc, tn, pis)
    assert_stats_close(eng.observed(), obs, what="observed (k up to 3,000)")
    assert_stats_close(nulls, exp, what="nulls (k up to 3,000)")


def test_netprops_beyond_lds():
    """Vector mode for a 2,600-node module at S = 300: weighted degree and
    summary profile / contributions of a module beyond both kernels' LDS."""
    from netrep_amd.api import RMatrix
    lay, mi, disc, txs, tc, tn = _case([2600, 50], 300, 23, n_nodes=4000)
    names = lay.names
    ma = dict(zip(names, lay.labels))
    got = N.NetProps(RMatrix(txs, None, names), RMatrix(tn, names, names), ma, lay.modules)
    module_nodes = {m: [n for n, l in ma.items() if l == m] for m in lay.modules}
    exp = O.net_props(txs, tn, names, module_nodes, lay.modules)
    for m in lay.modules:
        for key in ("summary", "contribution", "degree"):
            assert_stats_close(got[m][key], exp[m][key], what=f"{m}/{key}")
        assert_stats_close([got[m]["coherence"]], [exp[m]["coherence"]], what=f"{m}/coherence")
        assert_stats_close([got[m]["avgWeight"]], [exp[m]["avgWeight"]], what=f"{m}/avgWeight")


@pytest.mark.parametrize("sizes,n_samples,seed,n_nodes", [([3000, 60], 3000, 93, 4500),
                                                         ([2800, 33], 2600, 95, 4000)])
def test_lanczos_dimension_beyond_lds_vectors(sizes, n_samples, seed, n_nodes):
    """a 3,000-node module at S = 3,000 (primal) and a
    2,800-node module at S = 2,600 (dual): Lanczos dimensions of 3,000 / 2,600,
    beyond the ~2,540 LDS vectors, which round 3 rejected with
    NR_ERR_UNSUPPORTED. They now run with every vector and the index set in the
    slot's scratch (variant 6); svd_econ has no size limit
    (src/netStats.cpp:217-250). Against the C++ LAPACK restatement on
    identical shuffles."""
    lay, mi, disc, txs, tc, tn = _case(sizes, n_samples, seed, n_nodes=n_nodes)
    eng = _engine_from(mi, disc, txs, tc, tn)
    nulls = eng.run(4, 5, 17)
    pis = N.prp_table(17, 4, 5, mi.null_idx.size)
    exp, obs = _cpp(mi, disc, txs, tc, tn, pis)
    assert_stats_close(eng.observed(), obs, what=f"observed (k {sizes[0]}, S {n_samples})")
    assert_stats_close(nulls, exp, what=f"nulls (k {sizes[0]}, S {n_samples})")


def test_lanczos_beyond_lds_mixed_sizes_multi_slot():
    """a variant-6 module (Lanczos dimension 2,600 > the LDS
    vectors, every vector in its slot's scratch) in a multi-permutation run
    beside a 350-node module (the runtime-layout class) and two packed-class
    modules: six permutations put six variant-6 items in flight on six slots
    of one launch. Against the C++ LAPACK restatement on identical shuffles."""
    lay, mi, disc, txs, tc, tn = _case([2700, 350, 90, 35], 2600, 97, n_nodes=4000)
    eng = _engine_from(mi, disc, txs, tc, tn)
    nulls = eng.run(0, 6, 29)
    pis = N.prp_table(29, 0, 6, mi.null_idx.size)
    exp, obs = _cpp(mi, disc, txs, tc, tn, pis)
    assert_stats_close(eng.observed(), obs, what="observed (mixed sizes, variant 6)")
    assert_stats_close(nulls, exp, what="nulls (mixed sizes, variant 6)")
