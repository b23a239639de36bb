"""disk.matrix test datasets straight to HBM (netrep_PermutationProcedureFiles,
nr_set_dataset_files): RDS files of the bundled test dataset give bitwise the
cube PermutationProcedure gives on the same matrices in RAM (tData scaled on
the device by the same kernel as Scale), with and without data."""
import numpy as np
import pytest

import netrep_amd as N
from rds_writer import write_rds
from test_gpu_parity import bundled_inputs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("with_data", [True, False])
def test_files_equal_in_memory(tmp_path, bundled, with_data):
    d, ma, t_names = bundled_inputs(bundled)
    mods = ["1", "2", "3", "4"]
    b = bundled
    paths = {}
    for key, name in (("data", "test_data"), ("corr", "test_correlation"), ("net", "test_network")):
        p = str(tmp_path / f"{key}.rds")
        rown = list(b[name + "_rownames"]) if name + "_rownames" in b else None
        write_rds(p, b[name], rown, list(b[name + "_colnames"]), compress=key != "data")
        paths[key] = p
    if with_data:
        disc = N.IntermediateProperties(N.Scale(d["dData"]), d["dCorr"], d["dNet"], t_names, ma, mods)
    else:
        disc = N.IntermediatePropertiesNoData(d["dCorr"], d["dNet"], t_names, ma, mods)
    got = N.PermutationProcedureFiles(disc, paths["data"] if with_data else None, paths["corr"], paths["net"],
                                      ma, mods, 64, seed=17)
    if with_data:
        ref = N.PermutationProcedure(disc, N.Scale(d["tData"]), d["tCorr"], d["tNet"], ma, mods, 64, seed=17)
    else:
        ref = N.PermutationProcedureNoData(disc, d["tCorr"], d["tNet"], ma, mods, 64, seed=17)
    np.testing.assert_array_equal(got["observed"].view(np.uint64), ref["observed"].view(np.uint64))
    np.testing.assert_array_equal(got["nulls"].view(np.uint64), ref["nulls"].view(np.uint64))


def test_engine_set_dataset_files_names_and_flags(tmp_path, bundled):
    b = bundled
    pc, pn = str(tmp_path / "c.rds"), str(tmp_path / "n.rds")
    write_rds(pc, b["test_correlation"], None, list(b["test_correlation_colnames"]))
    write_rds(pn, b["test_network"], None, list(b["test_network_colnames"]))
    eng = N.Engine(0)
    names = eng.set_dataset_files(pc, pn)
    assert names == list(b["test_network_colnames"])
    assert eng.symmetric()
    eng.close()


def test_files_node_order_mismatch_rejected(tmp_path, bundled):
    """R/check-user-input.R:757-771: the correlation, network and data files
    must list the nodes in one order ("mismatch in node order ..."), and each
    square matrix's row names must equal its column names."""
    b = bundled
    cols = list(b["test_network_colnames"])
    swapped = cols[1:2] + cols[:1] + cols[2:]
    pc, pn, pd = (str(tmp_path / f"{x}.rds") for x in ("c", "n", "d"))
    write_rds(pc, b["test_correlation"], None, swapped)
    write_rds(pn, b["test_network"], None, cols)
    eng = N.Engine(0)
    with pytest.raises(N.NetRepError) as ei:
        eng.set_dataset_files(pc, pn)
    assert "node order" in str(ei.value)
    write_rds(pc, b["test_correlation"], swapped, cols)   # rownames != colnames
    with pytest.raises(N.NetRepError) as ei:
        eng.set_dataset_files(pc, pn)
    assert "row and column names" in str(ei.value)
    write_rds(pc, b["test_correlation"], None, cols)
    write_rds(pd, b["test_data"], None, swapped)
    with pytest.raises(N.NetRepError) as ei:
        eng.set_dataset_files(pc, pn, pd)
    assert "node order" in str(ei.value)
    eng.close()


def test_failed_file_load_leaves_no_dataset(tmp_path, bundled):
    """A load that fails part-way (here: the data file does not match) leaves
    the context with no dataset, and modules / null pool set for the previous
    dataset are refused until set again (no stale shapes, no
    out-of-bounds kernels)."""
    from test_gpu_parity import bundled_inputs  # noqa: F401
    b = bundled
    cols = list(b["test_network_colnames"])
    pc, pn, pd = (str(tmp_path / f"{x}.rds") for x in ("c", "n", "d"))
    write_rds(pc, b["test_correlation"], None, cols)
    write_rds(pn, b["test_network"], None, cols)
    write_rds(pd, b["test_data"][:, :-1], None, cols[:-1])   # one node short
    eng = N.Engine(0)
    eng.set_dataset_files(pc, pn)
    n = len(cols)
    idx = np.arange(20, dtype=np.int32)
    eng.set_modules(1, np.arange(1), np.array([0, 20], dtype=np.int64), idx, idx,
                    np.zeros(190), np.zeros(20), None)
    eng.set_null_pool(np.arange(n, dtype=np.int32))
    eng.run(0, 4, 1)   # works on the good dataset
    with pytest.raises(N.NetRepError):
        eng.set_dataset_files(pc, pn, pd)
    assert eng.shape() == (0, 0)
    with pytest.raises(N.NetRepError) as ei:
        eng.run(0, 4, 1)
    assert "dataset" in str(ei.value)
    eng.set_dataset_files(pc, pn)      # a new load: modules must be set again
    with pytest.raises(N.NetRepError) as ei:
        eng.run(0, 4, 1)
    assert "nr_set_modules" in str(ei.value)
    eng.close()
