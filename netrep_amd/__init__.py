"""netrep_amd -- MI355X-native engine for NetRep's permutation null-distribution path.

Public surface:
  * ``netrep_amd.api``    -- NetRep's Rcpp entry points (PermutationProcedure, ...)
  * ``netrep_amd.engine`` -- one GPU context over the ``nr_*`` C ABI
  * ``netrep_amd.pvalues``-- the host p-value step (permutationTest)
  * ``netrep_amd.combine``-- combineAnalyses, the multi-node merge of null cubes
The compute path is the HIP library ``netrep_amd/_lib/libnetrep_amd.so``.
"""
from ._lib import NetRepError, load  # noqa: F401
from .api import (CheckFinite, IntermediateProperties, IntermediatePropertiesNoData,  # noqa: F401
                  NetProps, NetPropsNoData, PermutationProcedure, PermutationProcedureNoData,
                  PrefetchTestDataset, DiscardPrefetch, ReleaseResident, h2d_bytes, PermutationProcedureFiles, RMatrix,
                  read_rds_matrix, Scale, STATNAMES, STATNAMES_NODATA,
                  set_interrupt_hook)
from .engine import Engine, device_count, prp_table  # noqa: F401

__all__ = ["CheckFinite", "IntermediateProperties", "IntermediatePropertiesNoData", "NetProps",
           "NetPropsNoData", "PermutationProcedure", "PermutationProcedureNoData", "RMatrix",
           "Scale", "Engine", "NetRepError", "device_count", "prp_table", "STATNAMES",
           "STATNAMES_NODATA", "set_interrupt_hook", "PrefetchTestDataset",
           "DiscardPrefetch", "ReleaseResident", "h2d_bytes", "PermutationProcedureFiles", "read_rds_matrix"]
