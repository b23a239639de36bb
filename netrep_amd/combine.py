"""combineAnalyses (R/multi-machine.R:47-118): merge the null distributions of
several modulePreservation runs (e.g. one per GPU node) and recompute the
permutation p-values.

A "preservation" is the dict the R function returns per dataset comparison:
``observed`` (modules x statistics), ``nulls`` (modules x statistics x
permutations), ``p.values``, ``nVarsPresent``, ``propVarsPresent``,
``totalSize``, ``alternative`` and optionally ``contingency``. Results of
several comparisons nest as dict[test] or dict[discovery][test], as in the
reference (R/multi-machine.R:49-73).

Error behaviour follows the reference as it executes, not as its comments read
(R/multi-machine.R:89-101): ``nVarsPresent`` and the contingency presence checks
compare pres1 with itself there, so they never fire; a contingency that differs
between the two runs makes ``!all.equal(...)`` fail on a character value, which
surfaces as the "do not appear to be output" error.
"""
from __future__ import annotations

import numpy as np

from .pvalues import permutationTest

_MSG = "module preservation analyses differ between 'pres1' and 'pres2'"


def _differs(a, b) -> bool:
    """Elementwise `!=` with R's NA semantics folded in (NA vs NA is equal)."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return True
    if a.dtype.kind in "fc" and b.dtype.kind in "fc":
        both_na = np.isnan(a) & np.isnan(b)
        return bool(np.any((a != b) & ~both_na))
    return bool(np.any(a != b))


def _contingency_equal(c1, c2) -> bool:
    if c1 is None or c2 is None:
        return c1 is None and c2 is None
    a, b = np.asarray(c1), np.asarray(c2)
    return a.shape == b.shape and not _differs(a, b)


def combine_analyses_internal(pres1: dict, pres2: dict) -> dict:
    """R/multi-machine.R:87-118 (combineAnalysesInternal)."""
    try:
        o1 = np.asarray(pres1["observed"])
        o2 = np.asarray(pres2["observed"])
        bad = (o1.shape[0] != o2.shape[0] or o1.shape[1] != o2.shape[1]
               or pres1["alternative"] != pres2["alternative"]
               or _differs(pres1["totalSize"], pres2["totalSize"])
               or _differs(pres1["propVarsPresent"], pres2["propVarsPresent"]))
        c1 = pres1.get("contingency")
        if c1 is not None and not _contingency_equal(c1, pres2.get("contingency")):
            raise TypeError("all.equal returned a description of the differences")
    except (KeyError, TypeError, IndexError, AttributeError):
        raise ValueError("'pres1' and 'pres2' do not appear to be output from 'modulePreservation'")
    if bad:
        raise ValueError("module preservation analysis performed in 'pres1' and 'pres2' are not comparable")
    res = dict(pres1)
    res["nulls"] = np.concatenate([np.asarray(pres1["nulls"]), np.asarray(pres2["nulls"])], axis=2)
    res["p.values"] = permutationTest(res["nulls"], res["observed"], res["nVarsPresent"],
                                      res["totalSize"], res["alternative"],
                                      statnames=pres1.get("statnames"),
                                      modules=pres1.get("modules", pres1.get("observed_dimnames", [None])[0]))
    return res


def combineAnalyses(pres1: dict, pres2: dict) -> dict:
    """R/multi-machine.R:47-75: a single comparison, dict[test] or
    dict[discovery][test]; None entries mark comparisons that were not run."""
    if "observed" in pres1:
        return combine_analyses_internal(pres1, pres2)
    out = dict(pres1)
    for ii, v1 in pres1.items():
        v2 = pres2.get(ii)
        if v1 is not None and "observed" in v1:
            if v2 is None:
                raise ValueError(_MSG)
            out[ii] = combine_analyses_internal(v1, v2)
        elif v1 is not None:   # R: a NULL pres1[[ii]] has no names and an empty seq_along
            inner = dict(v1)
            for jj, w1 in v1.items():
                w2 = v2.get(jj) if v2 is not None else None
                if w1 is not None and w2 is not None:
                    inner[jj] = combine_analyses_internal(w1, w2)
                elif (w1 is None) != (w2 is None):
                    raise ValueError(_MSG)
            out[ii] = inner
    return out
