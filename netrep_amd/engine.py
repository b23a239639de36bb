"""Python handle on one engine context (one GPU, one resident dataset).

Thin wrapper over the ``nr_*`` C ABI (include/netrep_gpu.h). Arrays follow R's
layout: an ``(nrow, ncol)`` matrix is passed column-major, and the nulls cube
comes back as a Fortran-ordered ``(modules, statistics, permutations)`` array,
exactly the memory layout of the reference's ``arma::cube``
(src/permutations.cpp:55, :304).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def _f64(a) -> np.ndarray:
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


def _ptr(a, ctype=C.c_double):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(ctype))


# The 16 phase-stamp slots as include/netrep_gpu.h (nr_set_stamps) lists them.
STAMP_SLOTS = ["index", "gram", "lanczos_setup", "matvec", "three_term_omega", "statistics", "q_update",
               "ritz_checks", "start_column", "reorth", "ritz_vector", "node_contributions", "ritz_coefficients",
               "check_eigenvalue", "check_residual", "s15"]


class Engine:
    """One GPU context. ``device`` is the HIP ordinal."""

    def __init__(self, device: int = 0):
        self._lib = L.load()
        h = C.c_void_p()
        rc = self._lib.nr_ctx_create(int(device), C.byref(h))
        if rc != L.NR_OK:
            raise L.NetRepError(rc, self._lib.nr_last_error(None).decode())
        self._h = h
        self.device = device
        self.n_stat = None
        self.n_rows = 0
        self.n_null = 0

    # -- lifetime ---------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.nr_ctx_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc):
        L.check(rc, self._h)

    # -- dataset ----------------------------------------------------------
    def set_dataset(self, corr, net, data=None):
        """Host numpy matrices: corr, net (N x N) and optional scaled data (S x N)."""
        corr = _f64(corr)
        net = _f64(net)
        n = corr.shape[0]
        if corr.shape != (n, n) or net.shape != (n, n):
            raise ValueError("corr and net must be square and of equal size")
        d = None
        s = 0
        if data is not None:
            d = _f64(data)
            s = d.shape[0]
            if d.shape[1] != n:
                raise ValueError("data must have one column per node")
        self._check(self._lib.nr_set_dataset(self._h, _ptr(corr), _ptr(net), _ptr(d), n, s, L.NR_HOST))
        self.n_stat = 7 if data is not None else 4
        self.n_nodes = n
        self.n_samples = s

    def set_dataset_files(self, corr_path, net_path, data_path=None, objects=(None, None, None),
                          scale_data=True):
        """disk.matrix files (saveRDS output, or objects of a save() archive)
        straight to HBM; `data` is scaled on the device. Returns the node names
        (the network file's column names)."""
        enc = lambda x: None if x is None else str(x).encode()  # noqa: E731
        self._check(self._lib.nr_set_dataset_files(self._h, enc(corr_path), enc(net_path), enc(data_path),
                                                   enc(objects[0]), enc(objects[1]), enc(objects[2]),
                                                   int(bool(scale_data))))
        n, s_ = C.c_int64(), C.c_int64()
        self._check(self._lib.nr_dataset_shape(self._h, C.byref(n), C.byref(s_)))
        need = C.c_int64()
        self._check(self._lib.nr_dataset_colnames(self._h, None, 0, C.byref(need)))
        buf = C.create_string_buffer(max(need.value, 1))
        self._check(self._lib.nr_dataset_colnames(self._h, buf, need.value, C.byref(need)))
        names = buf.raw[:need.value].split(b"\0")[:-1] if need.value else []
        self.n_stat = 7 if data_path is not None else 4
        self.n_nodes = n.value
        self.n_samples = s_.value
        return [x.decode() for x in names]

    def set_dataset_device(self, corr_ptr: int, net_ptr: int, data_ptr, n_nodes: int, n_samples: int):
        """Device pointers (e.g. torch tensors after an RCCL broadcast). The
        engine reads them on its own stream: the producer's work must be
        complete (e.g. torch.cuda.synchronize()) -- torch's streams belong to
        its own HIP runtime and are not ordered with the engine's."""
        self._check(self._lib.nr_set_dataset(self._h, C.cast(corr_ptr, L._dp), C.cast(net_ptr, L._dp),
                                             C.cast(data_ptr, L._dp) if data_ptr else None,
                                             n_nodes, n_samples, L.NR_DEVICE))
        self.n_stat = 7 if data_ptr else 4
        self.n_nodes = n_nodes
        self.n_samples = n_samples if data_ptr else 0

    def broadcast_dataset_to(self, others):
        """This context's resident dataset to every context in `others`
        (nr_broadcast_dataset: scatter + all-gather of peer copies)."""
        hs = (C.c_void_p * (1 + len(others)))(self._h.value, *[o._h.value for o in others])
        self._check(self._lib.nr_broadcast_dataset(hs, 1 + len(others)))
        for o in others:
            o.n_stat, o.n_nodes, o.n_samples = self.n_stat, self.n_nodes, self.n_samples

    def set_host_threads(self, n: int):
        """Host threads of this context's staging copies (nr_ctx_set_host_threads)."""
        self._check(self._lib.nr_ctx_set_host_threads(self._h, int(n)))

    def copy_dataset_from(self, other: "Engine"):
        """Device-to-device copy of another context's resident dataset
        (nr_copy_dataset: over xGMI between GPUs)."""
        self._check(self._lib.nr_copy_dataset(self._h, other._h))
        self.n_stat = other.n_stat
        self.n_nodes = other.n_nodes
        self.n_samples = other.n_samples

    def shape(self):
        """(n_nodes, n_samples) of the resident dataset; (0, 0) when there is none."""
        n, s_ = C.c_int64(), C.c_int64()
        self._check(self._lib.nr_dataset_shape(self._h, C.byref(n), C.byref(s_)))
        return n.value, s_.value

    def symmetric(self) -> bool:
        v = C.c_int()
        self._check(self._lib.nr_dataset_symmetric(self._h, C.byref(v)))
        return bool(v.value)

    def finite(self):
        """(corr all finite, net all finite) of the resident dataset -- CheckFinite
        (src/checkFinite.cpp:21-28) fused into the upload's symmetry pass."""
        c, n = C.c_int(), C.c_int()
        self._check(self._lib.nr_dataset_finite(self._h, C.byref(c), C.byref(n)))
        return bool(c.value), bool(n.value)

    # -- modules ----------------------------------------------------------
    def set_modules(self, n_rows, row_of, node_off, test_idx, null_pos, disc_corr, disc_degree,
                    disc_contrib=None):
        row_of = np.ascontiguousarray(row_of, dtype=np.int32)
        node_off = np.ascontiguousarray(node_off, dtype=np.int64)
        test_idx = np.ascontiguousarray(test_idx, dtype=np.int32)
        null_pos = None if null_pos is None else np.ascontiguousarray(null_pos, dtype=np.int32)
        disc_corr = np.ascontiguousarray(disc_corr, dtype=np.float64)
        disc_degree = np.ascontiguousarray(disc_degree, dtype=np.float64)
        disc_contrib = None if disc_contrib is None else np.ascontiguousarray(disc_contrib, dtype=np.float64)
        self._keep = (row_of, node_off, test_idx, null_pos, disc_corr, disc_degree, disc_contrib)
        self._check(self._lib.nr_set_modules(
            self._h, int(n_rows), int(row_of.size), _ptr(row_of, C.c_int32), _ptr(node_off, C.c_int64),
            _ptr(test_idx, C.c_int32), _ptr(null_pos, C.c_int32), _ptr(disc_corr), _ptr(disc_degree),
            _ptr(disc_contrib)))
        self.n_rows = int(n_rows)
        self.node_off = node_off

    def set_null_pool(self, null_idx):
        null_idx = np.ascontiguousarray(null_idx, dtype=np.int32)
        self._check(self._lib.nr_set_null_pool(self._h, _ptr(null_idx, C.c_int32), int(null_idx.size)))
        self.n_null = int(null_idx.size)

    # -- statistics -------------------------------------------------------
    def observed(self) -> np.ndarray:
        out = np.empty((self.n_rows, self.n_stat), dtype=np.float64, order="F")
        self._check(self._lib.nr_observed(self._h, _ptr(out)))
        return out

    def gram_table(self) -> bool:
        """Whether the resident dataset carries the Gram table (nr_gram_table)."""
        on = C.c_int()
        self._check(self._lib.nr_gram_table(self._h, C.byref(on)))
        return bool(on.value)

    def gram_table_ms(self) -> float:
        """Build time of the resident Gram table in ms (nr_gram_table_ms), 0 without one."""
        ms = C.c_double()
        self._check(self._lib.nr_gram_table_ms(self._h, C.byref(ms)))
        return float(ms.value)

    def observed_async(self):
        """Enqueue the observed statistics on the context's second stream
        (nr_observed_async); collect them with observed_wait()."""
        self._check(self._lib.nr_observed_async(self._h))

    def observed_wait(self) -> np.ndarray:
        out = np.empty((self.n_rows, self.n_stat), dtype=np.float64, order="F")
        self._check(self._lib.nr_observed_wait(self._h, _ptr(out)))
        return out

    def run(self, perm_begin: int, perm_end: int, seed: int = 0, pi=None) -> np.ndarray:
        n = perm_end - perm_begin
        out = np.empty((self.n_rows, self.n_stat, n), dtype=np.float64, order="F")
        pi_arr = None
        if pi is not None:
            pi_arr = np.ascontiguousarray(pi, dtype=np.uint32)
            if pi_arr.shape != (n, self.n_null):
                raise ValueError(f"pi must have shape ({n}, {self.n_null})")
        self._check(self._lib.nr_run(self._h, int(perm_begin), int(perm_end), int(seed) & (2**64 - 1),
                                     _ptr(pi_arr, C.c_uint32), _ptr(out)))
        return out

    def run_device(self, perm_begin: int, perm_end: int, seed: int, out_ptr: int, pi_ptr: int = 0):
        self._check(self._lib.nr_run_device(self._h, int(perm_begin), int(perm_end),
                                            int(seed) & (2**64 - 1), C.c_void_p(pi_ptr or None),
                                            C.c_void_p(out_ptr)))

    def export_indices(self, perm_begin: int, perm_end: int, seed: int) -> np.ndarray:
        nodes = int(self.node_off[-1])
        out = np.empty((perm_end - perm_begin, nodes), dtype=np.int32)
        self._check(self._lib.nr_export_indices(self._h, int(perm_begin), int(perm_end),
                                                int(seed) & (2**64 - 1), _ptr(out, C.c_int32)))
        return out

    def module_vectors(self, node_off, idx, with_data: bool):
        """Per-module vectors on explicit index sets (CSR). Returns a dict of arrays."""
        node_off = np.ascontiguousarray(node_off, dtype=np.int64)
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        n_mod = node_off.size - 1
        k = np.diff(node_off)
        cv = np.empty(max(int((k * (k - 1) // 2).sum()), 1))
        wd = np.empty(int(node_off[-1]))
        aw = np.empty(n_mod)
        nc = sp = coh = None
        if with_data:
            nc = np.empty(int(node_off[-1]))
            sp = np.empty(n_mod * self.n_samples)
            coh = np.empty(n_mod)
        self._check(self._lib.nr_module_vectors(self._h, int(n_mod), _ptr(node_off, C.c_int64),
                                                _ptr(idx, C.c_int32), _ptr(cv), _ptr(wd), _ptr(aw),
                                                _ptr(nc), _ptr(sp), _ptr(coh)))
        out = {"corr": cv[: int((k * (k - 1) // 2).sum())], "degree": wd, "avg_weight": aw}
        if with_data:
            out.update(contribution=nc, summary=sp.reshape(n_mod, self.n_samples), coherence=coh)
        return out

    def scale(self, data) -> np.ndarray:
        data = _f64(data)
        out = np.empty_like(data, order="F")
        self._check(self._lib.nr_scale(self._h, _ptr(data), data.shape[0], data.shape[1], _ptr(out)))
        return out

    # -- control / measurement -------------------------------------------
    def progress(self):
        d, t = C.c_int64(), C.c_int64()
        self._check(self._lib.nr_progress(self._h, C.byref(d), C.byref(t)))
        return d.value, t.value

    def cancel(self):
        self._check(self._lib.nr_cancel(self._h))

    def set_batch(self, perms_per_launch: int):
        self._check(self._lib.nr_set_batch(self._h, int(perms_per_launch)))

    def set_timing(self, enable: bool):
        self._check(self._lib.nr_set_timing(self._h, int(bool(enable))))

    def timing(self, kernel: int):
        ms, launches, items = C.c_double(), C.c_int64(), C.c_int64()
        self._check(self._lib.nr_get_timing(self._h, int(kernel), C.byref(ms), C.byref(launches),
                                            C.byref(items)))
        return ms.value, launches.value, items.value

    def diagnostics(self):
        a, b, c, d = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        self._check(self._lib.nr_get_diagnostics(self._h, C.byref(a), C.byref(b), C.byref(c), C.byref(d)))
        return {"eig_items": a.value, "eig_steps": b.value, "eig_cap_hits": c.value, "eig_reorths": d.value}

    def set_stamps(self, enable: bool):
        self._check(self._lib.nr_set_stamps(self._h, int(bool(enable))))

    def stamps(self):
        out = (C.c_uint64 * 16)()
        self._check(self._lib.nr_get_stamps(self._h, out))
        names = STAMP_SLOTS
        return dict(zip(names, list(out)))

    def reset_timing(self):
        self._check(self._lib.nr_reset_timing(self._h))

    def synchronize(self):
        self._check(self._lib.nr_synchronize(self._h))


def device_count() -> int:
    lib = L.load()
    n = C.c_int()
    lib.nr_device_count(C.byref(n))
    return n.value


def prp_table(seed: int, perm_begin: int, perm_end: int, n_null: int) -> np.ndarray:
    """Host evaluation of the keyed null-pool permutation (no GPU needed)."""
    lib = L.load()
    out = np.empty((perm_end - perm_begin, n_null), dtype=np.uint32)
    L.check(lib.nr_prp_table(int(seed) & (2**64 - 1), int(perm_begin), int(perm_end), int(n_null),
                             _ptr(out, C.c_uint32)))
    return out
