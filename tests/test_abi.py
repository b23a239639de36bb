"""CPU tests of the C-ABI boundary: the library loads and exports exactly what
include/netrep_gpu.h declares; without a GPU every compute entry fails loudly."""
import os
import re

import numpy as np
import pytest

import netrep_amd
from netrep_amd import _lib as L

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "netrep_gpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b((?:nr|netrep)_[A-Za-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    for name in ["netrep_PermutationProcedure", "netrep_IntermediateProperties", "netrep_NetProps",
                 "netrep_Scale", "netrep_CheckFinite", "nr_run", "nr_set_dataset", "nr_observed"]:
        assert name in fns


def test_library_exports_every_declared_symbol():
    lib = L.load()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_bindings_cover_header():
    assert set(declared_functions()) == set(L.SIGNATURES)


def test_library_is_in_tree():
    assert os.path.dirname(L.LIB_PATH).endswith(os.path.join("netrep_amd", "_lib"))


@pytest.mark.skipif(netrep_amd.device_count() > 0, reason="a GPU is visible")
def test_no_cpu_fallback_without_gpu():
    with pytest.raises(netrep_amd.NetRepError) as ei:
        netrep_amd.Engine(0)
    assert "no CPU fallback" in str(ei.value)
    with pytest.raises(netrep_amd.NetRepError):
        netrep_amd.Scale(np.ones((3, 2)))


def test_format_progress_matches_reference_line():
    """netrep_format_progress renders MonitorProgress's "\\r%5d% completed."
    with round((float)done / (float)total * 100) (src/thread-utils.cpp:66-68)."""
    from netrep_amd.api import format_progress
    assert format_progress(0, 10000) == "\r    0% completed."
    assert format_progress(5000, 10000) == "\r   50% completed."
    assert format_progress(10000, 10000) == "\r  100% completed."
    assert format_progress(1, 3) == "\r   33% completed."
    assert format_progress(2, 3) == "\r   67% completed."
    import ctypes as C
    import netrep_amd._lib as L
    buf = C.create_string_buffer(8)
    assert L.load().netrep_format_progress(1, 2, buf, 8) == -1   # too small: refused, not truncated
