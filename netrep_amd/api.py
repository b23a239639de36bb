"""NetRep's Rcpp entry points, MI355X engine behind them.

Same names, argument meaning and return shapes as the functions registered in
src/RcppExports.cpp:131-146 (R wrappers R/RcppExports.R:4-35):

    Scale, CheckFinite, IntermediateProperties, IntermediatePropertiesNoData,
    PermutationProcedure, PermutationProcedureNoData, NetProps, NetPropsNoData

R values map to Python as:
  * ``NumericMatrix`` with dimnames -> ``RMatrix(values, rownames, colnames)``
    (``values`` an ``(nrow, ncol)`` array),
  * named ``CharacterVector`` moduleAssignments -> ``{node name: label}``
    (insertion order = the R vector's order),
  * ``List`` -> ``dict``; numeric arrays -> numpy (R's column-major cube layout
    for ``nulls``).
Errors raise ``NetRepError`` where the reference raises an R error.
Each call goes through the C ABI (``netrep_*``) into HIP kernels; nothing is
computed on the CPU.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict
import sys
from dataclasses import dataclass
from typing import Mapping, Optional, Sequence

import numpy as np

from . import _lib as L

STATNAMES = ["avg.weight", "coherence", "cor.cor", "cor.degree", "cor.contrib",
             "avg.cor", "avg.contrib"]                       # src/permutations.cpp:174-177
STATNAMES_NODATA = ["avg.weight", "cor.cor", "cor.degree", "avg.cor"]  # src/permutationsNoData.cpp:156-158

DEFAULT_SEED = 0x4E65745265703133  # "NetRep13"


@dataclass
class RMatrix:
    """An R numeric matrix with dimnames."""
    values: np.ndarray
    rownames: Optional[Sequence[str]] = None
    colnames: Optional[Sequence[str]] = None

    @property
    def f(self) -> np.ndarray:
        return np.asfortranarray(np.asarray(self.values, dtype=np.float64))


_STRV_CACHE: "OrderedDict[tuple, tuple]" = OrderedDict()


def _strv(names: Sequence[str]):
    """A char** of `names` (and the bytes it points into). The last few name
    lists are kept: modulePreservation passes the same node names and module
    assignments on every call (C5: 100k strings, ~60 ms to re-encode)."""
    key = tuple(str(n) for n in names)
    hit = _STRV_CACHE.get(key)
    if hit is not None:
        _STRV_CACHE.move_to_end(key)
        return hit
    enc = [n.encode() for n in key]
    arr = (C.c_char_p * max(len(enc), 1))(*enc)
    _STRV_CACHE[key] = (arr, enc)
    while len(_STRV_CACHE) > 8:
        _STRV_CACHE.popitem(last=False)
    return arr, enc


def _assignments(module_assignments):
    if isinstance(module_assignments, Mapping):
        items = list(module_assignments.items())
    else:
        items = list(module_assignments)
    names = [str(n) for n, _ in items]
    labels = [str(lab) for _, lab in items]
    return names, labels


def _dptr(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


def Scale(data) -> RMatrix:
    """Scale (src/scale.cpp:38-45): per-column (x - mean) / sd, keeping dimnames."""
    m = data if isinstance(data, RMatrix) else RMatrix(np.asarray(data))
    x = m.f
    out = np.empty_like(x, order="F")
    L.check_api(L.load().netrep_Scale(_dptr(x), x.shape[0], x.shape[1], _dptr(out)))
    return RMatrix(out, m.rownames, m.colnames)


def CheckFinite(mat) -> None:
    """CheckFinite (src/checkFinite.cpp:21-28): raise on any NA/NaN/Inf."""
    x = (mat.f if isinstance(mat, RMatrix) else np.asfortranarray(np.asarray(mat, dtype=np.float64)))
    x2 = x.reshape(x.shape[0], -1) if x.ndim > 1 else x.reshape(-1, 1)
    L.check_api(L.load().netrep_CheckFinite(_dptr(x2), x2.shape[0], x2.shape[1]))


def _intermediate(d_data, d_corr, d_net, t_node_names, module_assignments, modules):
    lib = L.load()
    names, labels = _assignments(module_assignments)
    modules = [str(m) for m in modules]
    d_names = list(d_net.colnames)
    n = len(d_names)
    corr = d_corr.f
    net = d_net.f
    data = d_data.f if d_data is not None else None
    s = data.shape[0] if data is not None else 0
    # upper bounds for the concatenated outputs: module sizes in discovery
    sizes = {}
    tset = set(map(str, t_node_names))
    for nm, lab in zip(names, labels):
        if nm in tset:
            sizes[lab] = sizes.get(lab, 0) + 1
    ks = [sizes.get(m, 0) for m in modules]
    deg = np.empty(max(sum(ks), 1))
    cv = np.empty(max(sum(k * (k - 1) // 2 for k in ks), 1))
    nc = np.empty(max(sum(ks), 1)) if data is not None else None
    nm_ = len(modules)
    deg_len = np.zeros(nm_, dtype=np.int64)
    cv_len = np.zeros(nm_, dtype=np.int64)
    nc_len = np.zeros(nm_, dtype=np.int64)
    dn, _k1 = _strv(d_names)
    tn, _k2 = _strv(t_node_names)
    an, _k3 = _strv(names)
    al, _k4 = _strv(labels)
    mo, _k5 = _strv(modules)
    i64 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int64))  # noqa: E731
    L.check_api(lib.netrep_IntermediateProperties(
        _dptr(data), _dptr(corr), _dptr(net), s, n, dn, tn, len(t_node_names), an, al, len(names),
        mo, nm_, _dptr(deg), i64(deg_len), _dptr(cv), i64(cv_len), _dptr(nc),
        i64(nc_len) if nc is not None else None))
    out = {"degree": {}, "corr": {}}
    if data is not None:
        out["contribution"] = {}
    od = oc = 0
    for i, m in enumerate(modules):
        if deg_len[i] == 0:
            continue                                     # only modsPresent (src/discProps.cpp:123-125)
        out["degree"][m] = deg[od:od + deg_len[i]].copy()
        out["corr"][m] = cv[oc:oc + cv_len[i]].copy()
        if data is not None:
            out["contribution"][m] = nc[od:od + nc_len[i]].copy()
        od += deg_len[i]
        oc += cv_len[i]
    return out


def IntermediateProperties(dData: RMatrix, dCorr: RMatrix, dNet: RMatrix, tNodeNames,
                           moduleAssignments, modules) -> dict:
    """IntermediateProperties (src/discProps.cpp:44-132). dData must be scaled."""
    return _intermediate(dData, dCorr, dNet, list(tNodeNames), moduleAssignments, modules)


def IntermediatePropertiesNoData(dCorr: RMatrix, dNet: RMatrix, tNodeNames, moduleAssignments,
                                 modules) -> dict:
    """IntermediatePropertiesNoData (src/discProps.cpp:171-244)."""
    return _intermediate(None, dCorr, dNet, list(tNodeNames), moduleAssignments, modules)


def _null_pool_size(ma_names, t_names, null_hypothesis) -> int:
    """|nullIdx| of MakeNullMap (src/utils.cpp:108-136) over validNodes
    (src/permutations.cpp:319-323)."""
    tset = set(t_names)
    if str(null_hypothesis) == "all":
        return len(tset)
    return len({nm for nm in ma_names if nm in tset})


_hook_keep = None


def set_interrupt_hook(fn) -> None:
    """Install ``fn() -> bool`` as the interrupt check polled (every 100 ms) by
    PermutationProcedure while the GPUs work (checkInterrupt,
    src/interrupt.cpp:9-11, in MonitorProgress, src/thread-utils.cpp:49-82).
    A true return cancels the run; the call then returns the partial cube
    (un-run permutations NA) with ``res["interrupted"] = True``. ``None``
    removes the hook."""
    global _hook_keep
    lib = L.load()
    if fn is None:
        lib.netrep_set_interrupt_hook(None, None)
        _hook_keep = None
        return
    cb = L.INTERRUPT_FN(lambda _user: 1 if fn() else 0)
    _hook_keep = cb
    lib.netrep_set_interrupt_hook(C.cast(cb, C.c_void_p), None)


_progress_keep = None
_progress_user_set = False


def format_progress(done: int, total: int) -> str:
    """MonitorProgress's line, "\\r%5d% completed." (src/thread-utils.cpp:66-68),
    rendered by the library (netrep_format_progress)."""
    buf = C.create_string_buffer(64)
    n = L.load().netrep_format_progress(int(done), int(total), buf, 64)
    return buf.value.decode() if n >= 0 else ""


def _install_progress(fn) -> None:
    global _progress_keep
    lib = L.load()
    if fn is None:
        lib.netrep_set_progress_hook(None, None)
        _progress_keep = None
        return
    cb = L.PROGRESS_FN(lambda ev, done, total, _user: fn(int(ev), int(done), int(total)))
    _progress_keep = cb
    lib.netrep_set_progress_hook(C.cast(cb, C.c_void_p), None)


def set_progress_hook(fn) -> None:
    """Install ``fn(event, done, total)`` as the progress report of a verbose
    PermutationProcedure (netrep_set_progress_hook; event 0 begin, 1 update
    about once a second, 2 end) -- MonitorProgress's console output
    (src/thread-utils.cpp:54-81). ``None`` restores the default, which prints
    the reference's lines to ``sys.stdout``; the library itself never writes
    to stdout."""
    global _progress_user_set
    _progress_user_set = fn is not None
    _install_progress(fn)


def _print_progress(ev: int, done: int, total: int) -> None:
    if ev == L.PROGRESS_BEGIN:
        sys.stdout.write("\n")
    elif ev == L.PROGRESS_UPDATE:
        sys.stdout.write(format_progress(done, total))
    else:
        sys.stdout.write("\n\n")
    sys.stdout.flush()


# Datasets handed to netrep_PrefetchTestDataset: their column-major arrays
# stay referenced here until the PermutationProcedure call that adopts them
# (at most two pending, as in the library).
_prefetched = []


def _prefetch_key(t_data, t_corr, t_net):
    return (id(t_data.values) if t_data is not None else None, id(t_corr.values), id(t_net.values))


def PrefetchTestDataset(tData: Optional[RMatrix], tCorr: RMatrix, tNet: RMatrix) -> None:
    """Start uploading a later test dataset to the GPU in the background
    (netrep_PrefetchTestDataset), so that its host->HBM copy overlaps the
    permutations of the current one -- modulePreservation's loop over test
    datasets (R/modulePreservation.R:553-620): prefetch dataset t+1, then run
    dataset t. The PermutationProcedure call on these same matrices adopts
    the upload."""
    lib = L.load()
    corr, net = tCorr.f, tNet.f
    data = tData.f if tData is not None else None
    s = data.shape[0] if data is not None else 0
    rc = lib.netrep_PrefetchTestDataset(_dptr(data), _dptr(corr), _dptr(net), s, corr.shape[0])
    L.check_api(rc)
    _prefetched.append((_prefetch_key(tData, tCorr, tNet), (data, corr, net), (tData, tCorr, tNet)))
    del _prefetched[:-2]


def DiscardPrefetch() -> None:
    """Drop every pending PrefetchTestDataset upload (netrep_DiscardPrefetch)."""
    L.load().netrep_DiscardPrefetch()
    _prefetched.clear()


def ReleaseResident() -> None:
    """Free the datasets kept resident between calls (IntermediateProperties'
    discovery dataset, NetProps' dataset), pending prefetches and the pooled
    contexts (netrep_ReleaseResident; the R glue calls it when
    modulePreservation / networkProperties return)."""
    L.load().netrep_ReleaseResident()
    _prefetched.clear()


def h2d_bytes() -> int:
    """Host -> device bytes the library has copied since it was loaded
    (nr_h2d_bytes): the difference across calls shows what was uploaded."""
    v = C.c_int64()
    L.check(L.load().nr_h2d_bytes(C.byref(v)))
    return int(v.value)


def _permutation(disc_props, t_data, t_corr, t_net, module_assignments, modules, n_perm, n_cores,
                 null_hypothesis, verbose, seed, pi):
    lib = L.load()
    names, labels = _assignments(module_assignments)
    modules = [str(m) for m in modules]
    with_data = t_data is not None
    t_names = list(t_net.colnames)
    n = len(t_names)
    key = _prefetch_key(t_data, t_corr, t_net)
    pre = next((p for p in _prefetched if p[0] == key), None)
    if pre is not None:
        _prefetched.remove(pre)
        data, corr, net = pre[1]   # the very arrays the upload read (same pointers)
    else:
        corr, net = t_corr.f, t_net.f
        data = t_data.f if with_data else None
    s = data.shape[0] if with_data else 0
    nm_ = len(modules)
    keep = []

    def vecs(key):
        d = disc_props.get(key, {}) if disc_props is not None else {}
        ptrs = (C.POINTER(C.c_double) * max(nm_, 1))()
        lens = np.zeros(max(nm_, 1), dtype=np.int64)
        for i, m in enumerate(modules):
            if m in d:
                v = np.ascontiguousarray(d[m], dtype=np.float64)
                keep.append(v)
                ptrs[i] = _dptr(v)
                lens[i] = v.size
        keep.append(lens)
        return ptrs, lens.ctypes.data_as(C.POINTER(C.c_int64))

    dp = L.DiscProps()
    dp.degree, dp.degree_len = vecs("degree")
    dp.corr, dp.corr_len = vecs("corr")
    if with_data:
        dp.contribution, dp.contribution_len = vecs("contribution")
    n_stat = 7 if with_data else 4
    observed = np.empty((nm_, n_stat), order="F")
    nulls = np.empty((nm_, n_stat, int(n_perm)), order="F") if n_perm > 0 else None
    pi_arr = None
    if pi is not None:
        pi_arr = np.ascontiguousarray(pi, dtype=np.uint32)
        n_null = _null_pool_size(names, t_names, null_hypothesis)
        if pi_arr.ndim != 2 or pi_arr.shape != (int(n_perm), n_null):
            raise L.NetRepError(L.NR_ERR_INVALID, f"pi must have shape (nPermutations, n_null) = "
                                                  f"({int(n_perm)}, {n_null}), got {pi_arr.shape}")
    tn, _k1 = _strv(t_names)
    an, _k2 = _strv(names)
    al, _k3 = _strv(labels)
    mo, _k4 = _strv(modules)
    if verbose and not _progress_user_set:
        _install_progress(_print_progress)  # the reference's console lines, from Python
    rc = lib.netrep_PermutationProcedure(
        C.byref(dp), _dptr(data), _dptr(corr), _dptr(net), s, n, tn, an, al, len(names), mo, nm_,
        int(n_perm), int(n_cores), str(null_hypothesis).encode(), int(bool(verbose)),
        int(seed) & (2**64 - 1), pi_arr.ctypes.data_as(C.POINTER(C.c_uint32)) if pi_arr is not None else None,
        _dptr(nulls), _dptr(observed))
    interrupted = rc == L.NR_ERR_CANCELLED
    if not interrupted:
        L.check_api(rc)
    statnames = STATNAMES if with_data else STATNAMES_NODATA
    res = {"observed": observed, "observed_dimnames": (modules, statnames)}
    if interrupted:
        # the reference returns the partial, NA-padded cube (src/permutations.cpp:375-408)
        res["interrupted"] = True
    if n_perm > 0:
        res["nulls"] = nulls
        res["nulls_dimnames"] = (modules, statnames, None)  # "permutation.i" left implicit
    return res


def PermutationProcedure(discProps: dict, tData: RMatrix, tCorr: RMatrix, tNet: RMatrix,
                         moduleAssignments, modules, nPermutations: int, nCores: int = 1,
                         nullHypothesis: str = "overlap", verbose: bool = False,
                         seed: int = DEFAULT_SEED, pi=None) -> dict:
    """PermutationProcedure (src/permutations.cpp:160-409).

    Returns ``{"nulls": (M, 7, P), "observed": (M, 7)}`` (plus dimnames).
    ``seed`` keys the per-permutation shuffle; ``pi`` ((P, n_null) uint32)
    replaces it with explicit shuffles of the null pool.
    """
    return _permutation(discProps, tData, tCorr, tNet, moduleAssignments, modules, nPermutations,
                        nCores, nullHypothesis, verbose, seed, pi)


def read_rds_matrix(path: str, object: Optional[str] = None) -> RMatrix:
    """One numeric matrix from an RDS file (saveRDS, gzip or uncompressed) or,
    by name, a save() archive -- what disk.matrix holds
    (R/disk-matrix-class.R:175-182) -- via netrep_ReadRDSMatrix (host read)."""
    lib = L.load()
    nrow, ncol, need = C.c_int64(), C.c_int64(), C.c_int64()
    p = str(path).encode()
    o = None if object is None else str(object).encode()
    L.check_api(lib.netrep_ReadRDSMatrix(p, o, C.byref(nrow), C.byref(ncol), None, None, 0, C.byref(need)))
    out = np.empty((nrow.value, ncol.value), order="F")
    buf = C.create_string_buffer(max(need.value, 1))
    L.check_api(lib.netrep_ReadRDSMatrix(p, o, C.byref(nrow), C.byref(ncol), _dptr(out), buf, need.value,
                                         C.byref(need)))
    names = [x.decode() for x in buf.raw[:need.value].split(b"\0")[:-1]] if need.value else None
    return RMatrix(out, None, names)


def PermutationProcedureFiles(discProps: dict, tData_file: Optional[str], tCorr_file: str, tNet_file: str,
                              moduleAssignments, modules, nPermutations: int, nCores: int = 1,
                              nullHypothesis: str = "overlap", verbose: bool = False,
                              seed: int = DEFAULT_SEED, pi=None) -> dict:
    """PermutationProcedure[NoData] on a test dataset held as disk.matrix files
    (netrep_PermutationProcedureFiles): the files go straight to HBM and tData
    (raw, unscaled) is scaled on the device; node names are the network file's
    column names."""
    lib = L.load()
    names, labels = _assignments(moduleAssignments)
    modules = [str(m) for m in modules]
    with_data = tData_file is not None
    nm_ = len(modules)
    keep = []

    def vecs(key):
        d = discProps.get(key, {}) if discProps is not None else {}
        ptrs = (C.POINTER(C.c_double) * max(nm_, 1))()
        lens = np.zeros(max(nm_, 1), dtype=np.int64)
        for i, m in enumerate(modules):
            if m in d:
                v = np.ascontiguousarray(d[m], dtype=np.float64)
                keep.append(v)
                ptrs[i] = _dptr(v)
                lens[i] = v.size
        keep.append(lens)
        return ptrs, lens.ctypes.data_as(C.POINTER(C.c_int64))

    dp = L.DiscProps()
    dp.degree, dp.degree_len = vecs("degree")
    dp.corr, dp.corr_len = vecs("corr")
    if with_data:
        dp.contribution, dp.contribution_len = vecs("contribution")
    n_stat = 7 if with_data else 4
    observed = np.empty((nm_, n_stat), order="F")
    nulls = np.empty((nm_, n_stat, int(nPermutations)), order="F") if nPermutations > 0 else None
    pi_arr = None if pi is None else np.ascontiguousarray(pi, dtype=np.uint32)
    an, _k2 = _strv(names)
    al, _k3 = _strv(labels)
    mo, _k4 = _strv(modules)
    enc = lambda x: None if x is None else str(x).encode()  # noqa: E731
    if pi_arr is not None and (pi_arr.ndim != 2 or pi_arr.shape[0] != int(nPermutations)):
        raise L.NetRepError(L.NR_ERR_INVALID, f"pi must have shape (nPermutations, n_null), got {pi_arr.shape}")
    if verbose and not _progress_user_set:
        _install_progress(_print_progress)
    # n_null is known only once the files' node names are read: the library
    # checks pi's length against it (pi_len)
    rc = lib.netrep_PermutationProcedureFiles(
        C.byref(dp), enc(tData_file), enc(tCorr_file), enc(tNet_file), an, al, len(names), mo, nm_,
        int(nPermutations), int(nCores), str(nullHypothesis).encode(), int(bool(verbose)),
        int(seed) & (2**64 - 1), pi_arr.ctypes.data_as(C.POINTER(C.c_uint32)) if pi_arr is not None else None,
        int(pi_arr.size) if pi_arr is not None else -1, _dptr(nulls), _dptr(observed))
    interrupted = rc == L.NR_ERR_CANCELLED
    if not interrupted:
        L.check_api(rc)
    statnames = STATNAMES if with_data else STATNAMES_NODATA
    res = {"observed": observed, "observed_dimnames": (modules, statnames)}
    if interrupted:
        res["interrupted"] = True
    if nPermutations > 0:
        res["nulls"] = nulls
        res["nulls_dimnames"] = (modules, statnames, None)
    return res


def PermutationProcedureNoData(discProps: dict, tCorr: RMatrix, tNet: RMatrix, moduleAssignments,
                               modules, nPermutations: int, nCores: int = 1,
                               nullHypothesis: str = "overlap", verbose: bool = False,
                               seed: int = DEFAULT_SEED, pi=None) -> dict:
    """PermutationProcedureNoData (src/permutationsNoData.cpp:140-375)."""
    return _permutation(discProps, None, tCorr, tNet, moduleAssignments, modules, nPermutations,
                        nCores, nullHypothesis, verbose, seed, pi)


def _netprops(data, net, module_assignments, modules):
    lib = L.load()
    names, labels = _assignments(module_assignments)
    modules = [str(m) for m in modules]
    node_names = list(net.colnames)
    netv = net.f
    x = data.f if data is not None else None
    s = x.shape[0] if x is not None else 0
    k_all = {}
    for lab in labels:
        k_all[lab] = k_all.get(lab, 0) + 1
    tot = sum(k_all.get(m, 0) for m in modules)
    nm_ = len(modules)
    deg = np.empty(max(tot, 1))
    aw = np.empty(max(nm_, 1))
    kk = np.zeros(max(nm_, 1), dtype=np.int64)
    nc = np.empty(max(tot, 1)) if x is not None else None
    sp = np.empty(max(nm_ * s, 1)) if x is not None else None
    coh = np.empty(max(nm_, 1)) if x is not None else None
    nn, _k1 = _strv(node_names)
    an, _k2 = _strv(names)
    al, _k3 = _strv(labels)
    mo, _k4 = _strv(modules)
    L.check_api(lib.netrep_NetProps(_dptr(x), _dptr(netv), s, len(node_names), nn, an, al, len(names),
                                    mo, nm_, _dptr(deg), _dptr(nc), _dptr(sp), _dptr(coh), _dptr(aw),
                                    kk.ctypes.data_as(C.POINTER(C.c_int64))))
    mod_nodes = {}
    for nm, lab in zip(names, labels):
        mod_nodes.setdefault(lab, []).append(nm)
    res = {}
    o = 0
    for i, m in enumerate(modules):
        k = int(kk[i])
        entry = {"degree": deg[o:o + k].copy(), "avgWeight": float(aw[i]),
                 "node_names": mod_nodes.get(m, [])}
        if x is not None:
            entry.update(summary=sp[i * s:(i + 1) * s].copy(), contribution=nc[o:o + k].copy(),
                         coherence=float(coh[i]))
        res[m] = entry
        o += k
    return res


def NetProps(data: RMatrix, net: RMatrix, moduleAssignments, modules) -> dict:
    """NetProps (src/properties.cpp:41-156). ``data`` is unscaled; it is scaled on the GPU."""
    return _netprops(data, net, moduleAssignments, modules)


def NetPropsNoData(net: RMatrix, moduleAssignments, modules) -> dict:
    """NetPropsNoData (src/properties.cpp:190-273)."""
    return _netprops(None, net, moduleAssignments, modules)
