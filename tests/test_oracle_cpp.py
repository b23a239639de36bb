"""CPU: the C++ restatement (CPU baseline / large-case checker) agrees with the
numpy oracle on the golden fixtures, and its thread chunking is invariant."""
import numpy as np
import pytest

from oracle import netrep_oracle as O
from oracle import ref_cpp

from conftest import assert_stats_close


def _sets(mi, disc, with_data):
    mods = mi.mods_present
    node_off = np.concatenate([[0], np.cumsum([mi.test_idx[m].size for m in mods])])
    return dict(row_of=[mi.modules.index(m) for m in mods], node_off=node_off,
                test_idx=np.concatenate([mi.test_idx[m] for m in mods]),
                null_pos=np.concatenate([mi.null_pos[m] for m in mods]), null_idx=mi.null_idx,
                disc_cv=np.concatenate([disc["corr"][m] for m in mods]),
                disc_wd=np.concatenate([disc["degree"][m] for m in mods]),
                disc_nc=np.concatenate([disc["contribution"][m] for m in mods]) if with_data else None)


@pytest.mark.parametrize("with_data", [True, False])
def test_cpp_matches_numpy_oracle_bundled(bundled, bundled_expected, with_data):
    b, e = bundled, bundled_expected
    names, labels = b["module_labels_names"].tolist(), b["module_labels"].tolist()
    mi = O.ModuleIndex(names, labels, b["test_network_colnames"].tolist(), ["1", "2", "3", "4"])
    sfx = "data" if with_data else "nodata"
    disc = {"corr": {}, "degree": {}, "contribution": {}}
    for key in disc:
        for m in mi.mods_present:
            k = f"disc_{key}_{m}_{sfx}"
            if k in e:
                disc[key][m] = e[k]
    data = O.scale(b["test_data"]) if with_data else None
    nulls, obs = ref_cpp.permutation_procedure(data, b["test_correlation"], b["test_network"], 4,
                                               n_perm=e["pis"].shape[0], pi=e["pis"], n_threads=3,
                                               **_sets(mi, disc, with_data))
    assert_stats_close(obs, e["observed_" + sfx], what="observed")
    assert_stats_close(nulls, e["nulls_" + sfx], what="nulls")


def test_cpp_unsymmetric_all(asym):
    a = asym
    mods = a["modules"].tolist()
    mi = O.ModuleIndex(a["d_names"].tolist(), a["ma_labels"].tolist(), a["t_names"].tolist(), mods, null="all")
    disc = {key: {m: a[f"disc_{key}_{m}_data_all"] for m in mi.mods_present}
            for key in ("corr", "degree", "contribution")}
    nulls, obs = ref_cpp.permutation_procedure(O.scale(a["t_data"]), a["t_corr"], a["t_corr"], len(mods),
                                               n_perm=a["pis_all"].shape[0], pi=a["pis_all"], n_threads=2,
                                               **_sets(mi, disc, True))
    assert_stats_close(obs, a["observed_data_all"], what="observed")
    assert_stats_close(nulls, a["nulls_data_all"], what="nulls")


def test_cpp_shuffle_mode_runs_and_chunks(bundled, bundled_expected):
    b, e = bundled, bundled_expected
    mi = O.ModuleIndex(b["module_labels_names"].tolist(), b["module_labels"].tolist(),
                       b["test_network_colnames"].tolist(), ["1", "2", "3", "4"])
    disc = {key: {m: e[f"disc_{key}_{m}_nodata"] for m in mi.mods_present} for key in ("corr", "degree")}
    disc["contribution"] = {}
    nulls, _ = ref_cpp.permutation_procedure(None, b["test_correlation"], b["test_network"], 4, n_perm=37,
                                             seed=5, n_threads=4, **_sets(mi, disc, False))
    assert nulls.shape == (4, 4, 37) and np.isfinite(nulls).all()
