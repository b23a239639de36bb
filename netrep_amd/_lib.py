"""ctypes binding of the in-tree engine library ``netrep_amd/_lib/libnetrep_amd.so``.

The library is the product: there is no Python or CPU fallback. If it is
missing, or no HIP device is visible, the calls raise ``NetRepError``.
Every function declared in ``include/netrep_gpu.h`` is bound here with its
exact C signature.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# The in-tree build. A/B tools (tools/probes/profile_ab.py) point LIB_PATH at
# another build of the same library before the first load(); no environment
# variable selects the library or anything inside it.
LIB_PATH = os.path.join(_HERE, "_lib", "libnetrep_amd.so")

NR_OK = 0
NR_ERR_HIP = 1
NR_ERR_INVALID = 2
NR_ERR_OOM = 3
NR_ERR_UNSUPPORTED = 4
NR_ERR_CANCELLED = 5
NR_ERR_NONFINITE = 6
NR_HOST = 0
NR_DEVICE = 1
NR_SCALE_DATA = 1


class NetRepError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


_p = C.c_void_p
_i32 = C.c_int32
_i64 = C.c_int64
_u64 = C.c_uint64
_int = C.c_int
_dp = C.POINTER(C.c_double)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_u32p = C.POINTER(C.c_uint32)
_intp = C.POINTER(C.c_int)
_strv = C.POINTER(C.c_char_p)
INTERRUPT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p)   # netrep_interrupt_fn
PROGRESS_FN = C.CFUNCTYPE(None, C.c_int32, C.c_int64, C.c_int64, C.c_void_p)  # netrep_progress_fn
PROGRESS_BEGIN, PROGRESS_UPDATE, PROGRESS_END = 0, 1, 2


class DiscProps(C.Structure):
    """netrep_disc_props."""
    _fields_ = [("degree", C.POINTER(_dp)), ("degree_len", _i64p),
                ("corr", C.POINTER(_dp)), ("corr_len", _i64p),
                ("contribution", C.POINTER(_dp)), ("contribution_len", _i64p)]


# name -> (restype, argtypes)
SIGNATURES = {
    "nr_device_count": (_int, [_intp]),
    "nr_ctx_create": (_int, [_int, C.POINTER(_p)]),
    "nr_ctx_destroy": (None, [_p]),
    "nr_last_error": (C.c_char_p, [_p]),
    "nr_set_dataset": (_int, [_p, _dp, _dp, _dp, _i64, _i64, _int]),
    "nr_set_dataset_ex": (_int, [_p, _dp, _dp, _dp, _i64, _i64, _int, _int]),
    "nr_clear_dataset": (_int, [_p]),
    "nr_broadcast_dataset": (_int, [C.POINTER(_p), _int]),
    "nr_ctx_set_host_threads": (_int, [_p, _int]),
    "nr_h2d_bytes": (_int, [_i64p]),
    "netrep_ReleaseResident": (None, []),
    "nr_copy_dataset": (_int, [_p, _p]),
    "nr_dataset_symmetric": (_int, [_p, _intp]),
    "nr_dataset_finite": (_int, [_p, _intp, _intp]),
    "nr_set_modules": (_int, [_p, _i32, _i32, _i32p, _i64p, _i32p, _i32p, _dp, _dp, _dp]),
    "nr_set_null_pool": (_int, [_p, _i32p, _i64]),
    "nr_observed": (_int, [_p, _dp]),
    "nr_observed_async": (_int, [_p]),
    "nr_gram_table": (_int, [_p, C.POINTER(C.c_int)]),
    "nr_gram_table_ms": (_int, [_p, C.POINTER(C.c_double)]),
    "nr_observed_wait": (_int, [_p, _dp]),
    "nr_run": (_int, [_p, _i64, _i64, _u64, _u32p, _dp]),
    "nr_run_device": (_int, [_p, _i64, _i64, _u64, _p, _p]),
    "nr_prp_table": (_int, [_u64, _i64, _i64, _i64, _u32p]),
    "nr_export_indices": (_int, [_p, _i64, _i64, _u64, _i32p]),
    "nr_module_vectors": (_int, [_p, _i32, _i64p, _i32p, _dp, _dp, _dp, _dp, _dp, _dp]),
    "nr_scale": (_int, [_p, _dp, _i64, _i64, _dp]),
    "nr_check_finite": (_int, [_p, _dp, _i64, _intp]),
    "nr_progress": (_int, [_p, _i64p, _i64p]),
    "nr_cancel": (_int, [_p]),
    "nr_set_batch": (_int, [_p, _i64]),
    "nr_set_timing": (_int, [_p, _int]),
    "nr_get_timing": (_int, [_p, _int, _dp, _i64p, _i64p]),
    "nr_reset_timing": (_int, [_p]),
    "nr_get_diagnostics": (_int, [_p, _i64p, _i64p, _i64p, _i64p]),
    "nr_synchronize": (_int, [_p]),
    "nr_set_stamps": (_int, [_p, _int]),
    "nr_get_stamps": (_int, [_p, C.POINTER(C.c_uint64)]),
    "netrep_PermutationProcedure": (_int, [C.POINTER(DiscProps), _dp, _dp, _dp, _i64, _i64, _strv,
                                           _strv, _strv, _i64, _strv, _i64, _i64, _i32, C.c_char_p,
                                           _i32, _u64, _u32p, _dp, _dp]),
    "netrep_IntermediateProperties": (_int, [_dp, _dp, _dp, _i64, _i64, _strv, _strv, _i64, _strv,
                                             _strv, _i64, _strv, _i64, _dp, _i64p, _dp, _i64p, _dp,
                                             _i64p]),
    "netrep_NetProps": (_int, [_dp, _dp, _i64, _i64, _strv, _strv, _strv, _i64, _strv, _i64, _dp,
                               _dp, _dp, _dp, _dp, _i64p]),
    "netrep_Scale": (_int, [_dp, _i64, _i64, _dp]),
    "netrep_CheckFinite": (_int, [_dp, _i64, _i64]),
    "netrep_last_error": (C.c_char_p, []),
    "netrep_set_interrupt_hook": (None, [C.c_void_p, C.c_void_p]),
    "netrep_set_progress_hook": (None, [C.c_void_p, C.c_void_p]),
    "netrep_format_progress": (_int, [_i64, _i64, C.c_char_p, _i64]),
    "nr_set_host_threads": (_int, [_int]),
    "nr_get_host_threads": (_int, []),
    "netrep_PrefetchTestDataset": (_int, [_dp, _dp, _dp, _i64, _i64]),
    "nr_set_dataset_files": (_int, [_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p,
                                    C.c_char_p, _int]),
    "nr_dataset_shape": (_int, [_p, _i64p, _i64p]),
    "nr_dataset_colnames": (_int, [_p, C.c_char_p, _i64, _i64p]),
    "netrep_PermutationProcedureFiles": (_int, [C.POINTER(DiscProps), C.c_char_p, C.c_char_p, C.c_char_p,
                                                _strv, _strv, _i64, _strv, _i64, _i64, _i32, C.c_char_p,
                                                _i32, _u64, _u32p, _i64, _dp, _dp]),
    "netrep_ReadRDSMatrix": (_int, [C.c_char_p, C.c_char_p, _i64p, _i64p, _dp, C.c_char_p, _i64, _i64p]),
    "netrep_DiscardPrefetch": (None, []),
    "nr_release_scratch": (_int, [_p]),
    "nr_scratch_bytes": (_int, [_p, _i64p]),
    "nr_ctx_get_host_threads": (_int, [_p, _intp]),
    "nr_debug_set": (_int, [_int, _i64]),
    "nr_peer_staged_pairs": (_int, [_intp]),
    "netrep_PoolInfo": (_int, [_i64p, _i64p, _i32p, _i32p]),
}
NR_DEBUG_SWEEP_MAX_OCC = 1
NR_DEBUG_FAIL_SWEEP_ALLOC = 2

_lib = None


def _init_torch_runtime_first() -> None:
    """PyTorch-ROCm ships its own HIP runtime (torch/lib/libamdhip64.so, a
    different soname from /opt/rocm's libamdhip64.so.7 this library links),
    so a process that uses both holds two runtimes. Measured on MI355X: torch
    initialised AFTER the engine's runtime sees no device, the reverse order
    works (bench.py passes torch-allocated device buffers to the engine). So
    when torch is installed its runtime is initialised before the engine
    library loads; without torch this is a no-op."""
    try:
        import torch
    except ImportError:
        return
    try:
        torch.cuda.is_available()
    except Exception:  # pragma: no cover - a broken torch install must not block the engine
        pass


def load() -> C.CDLL:
    """Load (once) and return the engine library; raise if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NetRepError(NR_ERR_INVALID,
                          f"engine library not built: {LIB_PATH} (run __graft_entry__.build())")
    _init_torch_runtime_first()
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, ctx=None) -> None:
    if rc == NR_OK:
        return
    lib = load()
    msg = lib.nr_last_error(ctx).decode() if ctx is not None else lib.netrep_last_error().decode()
    raise NetRepError(rc, msg or f"engine error {rc}")


def check_api(rc: int) -> None:
    if rc != NR_OK:
        raise NetRepError(rc, load().netrep_last_error().decode() or f"engine error {rc}")
