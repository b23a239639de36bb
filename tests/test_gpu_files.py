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
