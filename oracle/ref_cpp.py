"""ctypes driver of the C++ CPU restatement (oracle/netrep_ref.cpp).

TEST INFRASTRUCTURE ONLY (checker for large parity cases; bench.py's
cpu_baseline). Build with ``make -C oracle``.
"""
from __future__ import annotations

import ctypes as C
import glob
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libnetrep_ref.so")

_lib = None


def _openblas_path():
    import scipy
    base = os.path.dirname(os.path.dirname(scipy.__file__))
    cands = glob.glob(os.path.join(base, "scipy.libs", "libscipy_openblas*.so"))
    if not cands:
        raise RuntimeError("scipy's bundled OpenBLAS not found")
    return cands[0]


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        raise RuntimeError(f"{LIB} missing: run `make -C oracle`")
    lib = C.CDLL(LIB)
    p = C.POINTER
    lib.ref_init_lapack.argtypes = [C.c_char_p]
    lib.ref_last_error.restype = C.c_char_p
    lib.ref_permutation_procedure.argtypes = [
        p(C.c_double), p(C.c_double), p(C.c_double), C.c_int64, C.c_int64, C.c_int32, C.c_int32,
        p(C.c_int32), p(C.c_int64), p(C.c_int32), p(C.c_int32), p(C.c_int32), C.c_int64,
        p(C.c_double), p(C.c_double), p(C.c_double), C.c_int64, C.c_uint64, p(C.c_uint32), C.c_int,
        p(C.c_double), p(C.c_double)]
    if lib.ref_init_lapack(_openblas_path().encode()) != 0:
        raise RuntimeError(lib.ref_last_error().decode())
    _lib = lib
    return lib


def _p(a, t=C.c_double):
    return None if a is None else a.ctypes.data_as(C.POINTER(t))


def permutation_procedure(data, corr, net, n_rows, row_of, node_off, test_idx, null_pos, null_idx,
                          disc_cv, disc_wd, disc_nc, n_perm, seed=0, pi=None, n_threads=1,
                          want_observed=True):
    """Returns (nulls[n_rows, n_stat, n_perm] F-order, observed[n_rows, n_stat])."""
    lib = load()
    corr = np.asfortranarray(corr, dtype=np.float64)
    net = np.asfortranarray(net, dtype=np.float64)
    data = None if data is None else np.asfortranarray(data, dtype=np.float64)
    n = corr.shape[0]
    s = 0 if data is None else data.shape[0]
    n_stat = 4 if data is None else 7
    row_of = np.ascontiguousarray(row_of, dtype=np.int32)
    node_off = np.ascontiguousarray(node_off, dtype=np.int64)
    test_idx = np.ascontiguousarray(test_idx, dtype=np.int32)
    null_pos = np.ascontiguousarray(null_pos, dtype=np.int32)
    null_idx = np.ascontiguousarray(null_idx, dtype=np.int32)
    disc_cv = np.ascontiguousarray(disc_cv, dtype=np.float64)
    disc_wd = np.ascontiguousarray(disc_wd, dtype=np.float64)
    disc_nc = None if disc_nc is None else np.ascontiguousarray(disc_nc, dtype=np.float64)
    pi_arr = None if pi is None else np.ascontiguousarray(pi, dtype=np.uint32)
    nulls = np.empty((n_rows, n_stat, max(n_perm, 0)), order="F")
    obs = np.empty((n_rows, n_stat), order="F") if want_observed else None
    rc = lib.ref_permutation_procedure(
        _p(data), _p(corr), _p(net), n, s, int(n_rows), int(row_of.size), _p(row_of, C.c_int32),
        _p(node_off, C.c_int64), _p(test_idx, C.c_int32), _p(null_pos, C.c_int32),
        _p(null_idx, C.c_int32), int(null_idx.size), _p(disc_cv), _p(disc_wd), _p(disc_nc),
        int(n_perm), int(seed) & (2**64 - 1), _p(pi_arr, C.c_uint32), int(n_threads), _p(nulls), _p(obs))
    if rc != 0:
        raise RuntimeError(lib.ref_last_error().decode())
    return nulls, obs
