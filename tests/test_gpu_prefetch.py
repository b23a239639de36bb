"""Multi-dataset pipelining (modulePreservation's loop over test datasets,
R/modulePreservation.R:553-620): the next test dataset is uploaded through
pinned double-buffered chunks while the current one's permutations run
(netrep_PrefetchTestDataset). The adopted upload must give bitwise the same
cube as an ordinary call; a mismatched prefetch is discarded."""
import numpy as np
import pytest

import netrep_amd as N
from netrep_amd.api import RMatrix

pytestmark = pytest.mark.gpu


def _datasets(n_sets, n_nodes=2500, n_samples=60, seed=3):
    from netrep_amd import synthetic as S
    lay = S.make_layout(n_nodes, [200, 120, 80, 40], seed)
    names = lay.names
    dx, dc, dn = S.numpy_dataset(lay, n_samples, seed + 1)
    disc = N.IntermediateProperties(N.Scale(RMatrix(dx, None, names)), RMatrix(dc, names, names),
                                    RMatrix(dn, names, names), names, dict(zip(names, lay.labels)),
                                    lay.modules)
    sets = []
    for t in range(n_sets):
        tx, tc, tn = S.numpy_dataset(lay, n_samples, seed + 10 + t, preserve_all=False)
        sets.append((N.Scale(RMatrix(tx, None, names)), RMatrix(tc, names, names), RMatrix(tn, names, names)))
    return lay, disc, sets


def test_prefetched_dataset_is_bitwise_equal():
    lay, disc, sets = _datasets(3)
    ma = dict(zip(lay.names, lay.labels))
    plain = [N.PermutationProcedure(disc, *st, ma, lay.modules, 64, seed=5) for st in sets]
    piped = []
    N.PrefetchTestDataset(*sets[0])
    for t, st in enumerate(sets):
        if t + 1 < len(sets):
            N.PrefetchTestDataset(*sets[t + 1])   # uploads while dataset t runs
        piped.append(N.PermutationProcedure(disc, *st, ma, lay.modules, 64, seed=5))
    for a, b in zip(plain, piped):
        np.testing.assert_array_equal(a["nulls"].view(np.uint64), b["nulls"].view(np.uint64))
        np.testing.assert_array_equal(a["observed"].view(np.uint64), b["observed"].view(np.uint64))


def test_unmatched_prefetch_stays_pending():
    """A prefetch of another dataset does not affect the call (it stays
    pending for its own call) and is adopted afterwards; DiscardPrefetch
    frees what is left."""
    lay, disc, sets = _datasets(2)
    ma = dict(zip(lay.names, lay.labels))
    ref0 = N.PermutationProcedure(disc, *sets[0], ma, lay.modules, 16, seed=9)
    ref1 = N.PermutationProcedure(disc, *sets[1], ma, lay.modules, 16, seed=9)
    N.PrefetchTestDataset(*sets[1])          # announced, but dataset 0 runs first
    got0 = N.PermutationProcedure(disc, *sets[0], ma, lay.modules, 16, seed=9)
    got1 = N.PermutationProcedure(disc, *sets[1], ma, lay.modules, 16, seed=9)
    np.testing.assert_array_equal(ref0["nulls"].view(np.uint64), got0["nulls"].view(np.uint64))
    np.testing.assert_array_equal(ref1["nulls"].view(np.uint64), got1["nulls"].view(np.uint64))
    N.PrefetchTestDataset(*sets[0])
    N.DiscardPrefetch()
