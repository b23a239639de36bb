"""Generate the golden fixtures under tests/golden/ (run in the build container).

Sources:
  * the reference's bundled example data ``data/NetRep.rda`` (150 nodes,
    30 samples, modules 1-4 + background "0"; R/example-data.R), decoded by
    oracle/rda.py -- a data file, converted to ``netrep_bundled.npz``;
  * a synthetic case shaped like the reference's own test
    (tests/testthat/test1-main.R:2-25: 100 nodes per dataset, 50 shared,
    unsymmetric random "correlation"/"network" matrices, 7 random modules kept
    if they have > 2 nodes present), saved with its inputs in
    ``asym_case.npz``.
Expected outputs come from the numpy oracle (oracle/netrep_oracle.py), which
tests/test_oracle_golden.py pins to the vignette's printed values first.

Usage:  python tests/golden/make_golden.py [/root/reference]
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import netrep_oracle as O  # noqa: E402
from oracle import prp  # noqa: E402
from oracle.rda import as_matrix, as_named_vector, read_rda  # noqa: E402

SEED = 20240611
N_PERM = 16


def _names(a):
    return np.array([str(x) for x in a])


def bundled(ref_root: str):
    d = read_rda(os.path.join(ref_root, "data", "NetRep.rda"))
    out = {}
    for key in ["discovery_data", "test_data", "discovery_correlation", "test_correlation",
                "discovery_network", "test_network"]:
        m, rn, cn = as_matrix(d[key])
        out[key] = m
        out[key + "_colnames"] = _names(cn)
        if key.endswith("_data"):
            out[key + "_rownames"] = _names(rn)
    lab, names = as_named_vector(d["module_labels"])
    out["module_labels"] = _names([str(int(x)) for x in lab])
    out["module_labels_names"] = _names(names)
    np.savez_compressed(os.path.join(HERE, "netrep_bundled.npz"), **out)
    return out


def expected_for(case, modules, null="overlap", tag=""):
    """Oracle outputs for one (discovery, test) pair, data and network-only."""
    names, labels = list(case["ma_names"]), list(case["ma_labels"])
    t_names = list(case["t_names"])
    mi = O.ModuleIndex(names, labels, t_names, modules, null=null)
    res = {}
    d_scaled = O.scale(case["d_data"])
    t_scaled = O.scale(case["t_data"])
    pis = np.stack([prp.permute(np.arange(mi.null_idx.size), mi.null_idx.size, SEED, p)
                    for p in range(N_PERM)]).astype(np.int64)
    for with_data in (True, False):
        disc = O.intermediate_properties(d_scaled, case["d_corr"], case["d_net"],
                                         mi.disc_idx(case["d_names"]), with_data=with_data)
        nulls, obs = O.permutation_procedure(disc, t_scaled, case["t_corr"], case["t_net"], mi, pis,
                                             with_data=with_data)
        sfx = ("data" if with_data else "nodata") + tag
        res["observed_" + sfx] = obs
        res["nulls_" + sfx] = nulls
        for key in disc:
            for m, v in disc[key].items():
                res[f"disc_{key}_{m}_{sfx}"] = v
    res["null_idx" + tag] = mi.null_idx
    res["pis" + tag] = pis.astype(np.uint32)
    return res


def bundled_expected(b):
    case = dict(d_data=b["discovery_data"], t_data=b["test_data"], d_corr=b["discovery_correlation"],
                t_corr=b["test_correlation"], d_net=b["discovery_network"], t_net=b["test_network"],
                d_names=list(b["discovery_network_colnames"]), t_names=list(b["test_network_colnames"]),
                ma_names=list(b["module_labels_names"]), ma_labels=list(b["module_labels"]))
    modules = ["1", "2", "3", "4"]
    res = expected_for(case, modules)
    # networkProperties on both datasets (src/properties.cpp)
    mod_nodes = {}
    for nm, lab in zip(case["ma_names"], case["ma_labels"]):
        mod_nodes.setdefault(lab, []).append(nm)
    for tag, data, net, names in (("disc", b["discovery_data"], b["discovery_network"], case["d_names"]),
                                  ("test", b["test_data"], b["test_network"], case["t_names"])):
        props = O.net_props(data, net, names, mod_nodes, modules)
        for m in modules:
            for key, v in props[m].items():
                res[f"netprops_{tag}_{m}_{key}"] = np.asarray(v)
    res["scaled_test_data"] = O.scale(b["test_data"])
    np.savez_compressed(os.path.join(HERE, "bundled_expected.npz"), **res)


def asym_case():
    rng = np.random.default_rng(SEED)
    gn1 = [f"N_{i}" for i in range(1, 101)]
    gn2 = [f"N_{int(v)}" for v in np.linspace(2, 200, 100)]
    sn1 = [f"S_{i}" for i in range(1, 51)]
    sn2 = [f"S_{i}" for i in range(1, 76)]
    d_corr = rng.standard_normal((100, 100))
    t_corr = rng.standard_normal((100, 100))
    d_net, t_net = d_corr.copy(), t_corr.copy()           # adjSets <- coexpSets (test1-main.R:11)
    d_data = rng.standard_normal((50, 100))
    t_data = rng.standard_normal((75, 100))
    labels = [str(v) for v in rng.integers(1, 8, size=100)]
    present = [lab for nm, lab in zip(gn1, labels) if nm in set(gn2)]
    counts = {m: present.count(m) for m in set(present)}
    modules = sorted([m for m, c in counts.items() if c > 2], key=int)
    case = dict(d_data=d_data, t_data=t_data, d_corr=d_corr, t_corr=t_corr, d_net=d_net, t_net=t_net,
                d_names=gn1, t_names=gn2, ma_names=gn1, ma_labels=labels)
    res = expected_for(case, modules)
    res.update(expected_for(case, modules, null="all", tag="_all"))
    np.savez_compressed(os.path.join(HERE, "asym_case.npz"),
                        d_data=d_data, t_data=t_data, d_corr=d_corr, t_corr=t_corr,
                        d_names=_names(gn1), t_names=_names(gn2), d_samples=_names(sn1),
                        t_samples=_names(sn2), ma_labels=_names(labels), modules=_names(modules), **res)


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    b = bundled(root)
    bundled_expected(b)
    asym_case()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
