"""Host p-value step: permutationTest (R/pperm.R:74-167), permp (R/pperm.R:188-201)
and requiredPerms (R/pperm.R:239-250).

The reference delegates to ``statmod::permp`` (Phipson & Smyth 2010, "Permutation
p-values should never be zero"), an unvendored CRAN dependency (DESCRIPTION:17,
version unpinned). Its published algorithm is restated here:

  * total.nperm <= 10000 ("exact"): p = mean over i = 1..T of pbinom(x; nperm, i/T)
  * otherwise ("approximate"):      p = (x + 1)/(nperm + 1)
        - 0.5/T * sum_j w_j pbinom(x; nperm, z_j)
    with (z_j, w_j) the 128-point Gauss-Legendre rule on [0, 0.5/T], weights
    summing to 1 (statmod::gauss.quad.prob(128, l=0, u=0.5/T)).

Parity is pinned by the vignette's p = 0.00009999 entries (x = 0, nPerm = 10000;
vignettes/NetRep.md:315,318); beyond those it is "parity unpinned" (statmod is
not available here). The counts it consumes (#null <= obs, #null >= obs after
dropping NA, R/pperm.R:138-141) are exact integer work and are tested bit for bit.
"""
from __future__ import annotations

import math

import numpy as np

from .api import STATNAMES


def _pbinom(x, n, p):
    from scipy.stats import binom
    return binom.cdf(x, n, p)


def permp(x, nperm, total_nperm, method="auto"):
    """statmod::permp(x, nperm, total.nperm=...) restated (see module docstring)."""
    x = np.asarray(x, dtype=np.float64)
    if np.any(x < 0):
        raise ValueError("negative x values")
    if np.any(x > nperm):
        raise ValueError("x cannot exceed nperm")
    if method == "auto":
        method = "approximate" if total_nperm > 10000 else "exact"
    if method == "exact":
        t = int(round(total_nperm))
        prob = np.arange(1, t + 1, dtype=np.float64) / total_nperm
        return np.array([_pbinom(xi, nperm, prob).sum() / total_nperm for xi in x.ravel()]).reshape(x.shape)
    nodes, weights = np.polynomial.legendre.leggauss(128)
    u = 0.5 / total_nperm
    z = u / 2 * nodes + u / 2
    w = weights / 2
    integ = np.array([u * np.sum(w * _pbinom(xi, nperm, z)) for xi in x.ravel()]).reshape(x.shape)
    return (x + 1) / (nperm + 1) - integ


def _total_nperm(total_size, k, ordered):
    """R/pperm.R:131-135 (in doubles, as R computes them; may overflow to inf)."""
    if ordered:
        try:
            return float(math.prod(range(int(total_size), int(total_size - k), -1)))
        except OverflowError:
            return math.inf
    try:
        return float(math.comb(int(total_size), int(k)))
    except OverflowError:
        return math.inf


def extreme_counts(nulls, observed):
    """#(null <= obs) and #(null >= obs) per (module, statistic), NA dropped
    (R/pperm.R:138-141); also the number of non-NA null values."""
    nulls = np.asarray(nulls, dtype=np.float64)
    obs = np.asarray(observed, dtype=np.float64)[:, :, None]
    fin = np.isfinite(nulls)
    less = np.sum(fin & (nulls <= obs), axis=2)
    more = np.sum(fin & (nulls >= obs), axis=2)
    return less, more, fin.sum(axis=2)


def _align_vars_present(nVarsPresent, modules, n_rows):
    """nVarsPresent by module label (R/pperm.R:106-111 requires
    names(nVarsPresent) to match rownames(nulls)). A mapping (e.g.
    contingencyTable's ``varsPres``) is aligned to ``modules`` by label; a
    plain sequence is taken positionally."""
    from collections.abc import Mapping
    err = ValueError("expecting 'nVarsPresent' to be a numeric vector output by the "
                     "'modulePreservation' function")
    if isinstance(nVarsPresent, Mapping):
        if modules is None:
            raise ValueError("nVarsPresent given by module label: pass modules= (the row names of "
                             "'nulls'/'observed')")
        keys = [str(k) for k in nVarsPresent]
        mods = [str(m) for m in modules]
        if len(mods) != n_rows or sorted(keys) != sorted(mods):
            raise err
        lookup = {str(k): v for k, v in nVarsPresent.items()}
        return [lookup[m] for m in mods]
    vals = list(np.asarray(nVarsPresent).ravel())
    if len(vals) != n_rows:
        raise err
    return vals


def permutationTest(nulls, observed, nVarsPresent, totalSize, alternative="greater",
                    statnames=None, modules=None):
    """R/pperm.R:74-167. nulls: (modules, statistics, permutations); observed:
    (modules, statistics); nVarsPresent: per module, either a mapping
    {module label: count} (contingencyTable's varsPres), aligned by label to
    ``modules`` (the row names of nulls/observed), or a sequence in row order;
    statnames: column names of the statistics (defaults to the 7 or 4 of the
    reference)."""
    alts = ["two.sided", "less", "greater"]
    matches = [a for a in alts if a.startswith(alternative)]
    if len(matches) != 1:
        raise ValueError(f"Alternative must be one of {alts}")
    alt = matches[0]
    if not np.isscalar(totalSize) or totalSize < 1:
        raise ValueError("'totalSize' must be a single number > 0")
    nulls = np.asarray(nulls, dtype=np.float64)
    observed = np.asarray(observed, dtype=np.float64)
    if nulls.ndim != 3 or observed.ndim != 2 or nulls.shape[:2] != observed.shape:
        raise ValueError("mismatch in dimension names between 'nulls' and 'observed'")
    nVarsPresent = _align_vars_present(nVarsPresent, modules, observed.shape[0])
    if statnames is None:
        statnames = STATNAMES if observed.shape[1] == 7 else ["avg.weight", "cor.cor", "cor.degree", "avg.cor"]
    less, more, n_ok = extreme_counts(nulls, observed)
    p = np.full(observed.shape, np.nan)
    for mi in range(observed.shape[0]):
        for si in range(observed.shape[1]):
            if not np.isfinite(observed[mi, si]):
                continue
            ordered = statnames[si] not in ("avg.weight", "coherence")
            total = _total_nperm(totalSize, nVarsPresent[mi], ordered)
            n = int(n_ok[mi, si])
            lo = float(permp(less[mi, si], n, total))
            hi = float(permp(more[mi, si], n, total))
            p[mi, si] = {"two.sided": min(lo, hi) * 2, "less": lo, "greater": hi}[alt]
    return p


def requiredPerms(alpha, alternative="greater"):
    """R/pperm.R:239-250."""
    alts = ["two.sided", "less", "greater"]
    matches = [a for a in alts if a.startswith(alternative)]
    if len(matches) != 1:
        raise ValueError(f"Alternative must be one of {alts}")
    return 1 / alpha * 2 if matches[0] == "two.sided" else 1 / alpha
