"""Module overlap bookkeeping: contingencyTable (R/contingency.R:19-119) and the
totalSize rule of modulePreservation (R/modulePreservation.R:650-654).

Exact integer work on names; the counts feed permutationTest's total.nperm.
R semantics kept: ``table()`` sorts its levels, modules are ordered by
``orderAsNumeric`` (integer order when every label parses as an integer,
otherwise character order; R/utils.R:175-181).
"""
from __future__ import annotations

from collections import Counter, OrderedDict

import numpy as np


def _r_as_integer(x: str):
    """R's as.integer() on one character value: decimal / scientific notation
    truncated toward zero ("1.0" -> 1, "1e3" -> 1000, " 7 " -> 7); None where R
    gives NA with a warning (not a number, or outside the int32 range)."""
    try:
        v = float(x.strip())
    except ValueError:
        return None
    if not np.isfinite(v) or abs(v) >= 2**31:
        return None
    return int(v)


def order_as_numeric(labels):
    """orderAsNumeric (R/utils.R:175-181): order by as.integer(labels) (stable,
    as R's order), or -- when as.integer warns for any label -- by the labels
    as characters. R collates characters by locale; this uses code points."""
    labels = [str(x) for x in labels]
    keys = [_r_as_integer(x) for x in labels]
    if any(k is None for k in keys):
        return sorted(labels)
    return [labels[i] for i in sorted(range(len(labels)), key=lambda i: keys[i])]


def _table(values):
    c = Counter(str(v) for v in values)
    return OrderedDict((k, c[k]) for k in sorted(c))


def contingencyTable(modAssignments, mods, tiNodelist):
    """R/contingency.R:19-119.

    modAssignments: [discovery {node: label}, test {node: label} or None];
    mods: discovery modules of interest; tiNodelist: test node names.
    """
    disc = OrderedDict((str(k), str(v)) for k, v in modAssignments[0].items())
    test = None if modAssignments[1] is None else OrderedDict((str(k), str(v)) for k, v in modAssignments[1].items())
    mods = [str(m) for m in mods]
    tset = set(str(n) for n in tiNodelist)
    overlap_vars = [n for n in disc if n in tset]                      # intersect() keeps x's order
    overlap_assign = OrderedDict((n, disc[n]) for n in overlap_vars if disc[n] in set(mods))
    overlap_modules = order_as_numeric(list(OrderedDict.fromkeys(overlap_assign.values())))
    vp = _table(overlap_assign.values())
    for m in mods:
        if m not in vp:
            vp[m] = 0
    order = order_as_numeric(list(vp))
    vars_pres = OrderedDict((m, vp[m]) for m in order)
    sizes = _table(disc.values())
    # varsPres / moduleSizes[names(varsPres)]: NA for a module with no node in
    # the discovery assignments (R/contingency.R:52-53)
    prop = OrderedDict((m, vars_pres[m] / sizes[m] if m in sizes else np.nan) for m in vars_pres)
    contingency = None
    if test is not None:
        d_lab = sorted(set(disc[n] for n in overlap_vars))
        t_lab = sorted(set(test[n] for n in overlap_vars if n in test))
        cnt = Counter((disc[n], test[n]) for n in overlap_vars if n in test)
        disc_sizes, test_sizes = _table(disc.values()), _table(test.values())
        disc_present = _table(disc[n] for n in overlap_vars)
        test_present = _table(test[n] for n in overlap_vars if n in test)
        rows = d_lab + [m for m in disc_sizes if m not in d_lab]
        cols = t_lab + [m for m in test_sizes if m not in t_lab]
        missing = [m for m in mods if m not in rows]
        if missing:   # contingency[mods,, drop=FALSE] (R/contingency.R:95)
            raise ValueError("subscript out of bounds: module(s) " + ", ".join(f'"{m}"' for m in missing)
                             + " have no node in the discovery module assignments")
        rows = order_as_numeric([r for r in mods if r in rows or r in disc_sizes])
        cols = order_as_numeric(cols)
        mat = np.full((2 + len(rows), 2 + len(cols)), np.nan)
        for j, c in enumerate(cols):
            mat[0, 2 + j] = test_sizes.get(c, 0)
            mat[1, 2 + j] = test_present.get(c, 0)
        for i, r in enumerate(rows):
            mat[2 + i, 0] = disc_sizes.get(r, 0)
            mat[2 + i, 1] = disc_present.get(r, 0)
            for j, c in enumerate(cols):
                mat[2 + i, 2 + j] = cnt.get((r, c), 0)
        contingency = (mat, ["size", "present"] + rows, ["size", "present"] + cols)
    return {"contingency": contingency, "propVarsPres": prop, "overlapVars": overlap_vars,
            "varsPres": vars_pres, "overlapModules": overlap_modules,
            "overlapAssignments": overlap_assign}


def total_size(null_hypothesis, overlap_vars, n_test_nodes):
    """R/modulePreservation.R:650-654."""
    return len(overlap_vars) if null_hypothesis == "overlap" else int(n_test_nodes)
