"""disk.matrix loading (R/disk-matrix-class.R:175-182):
the C++ reader of R's XDR serialisation behind netrep_ReadRDSMatrix and the
file->HBM path. Round trips through a writer of the documented format, and a
pin against a file R itself wrote: the reference's data/NetRep.rda (xz, so it
is decompressed here first; the library reads gzip and uncompressed)."""
import lzma
import os

import numpy as np
import pytest

import netrep_amd as N
from netrep_amd._lib import NetRepError

from conftest import GOLDEN
from rds_writer import write_rda, write_rds


@pytest.mark.parametrize("version,compress", [(3, True), (2, False), (3, False), (2, True)])
def test_rds_round_trip(tmp_path, version, compress):
    rng = np.random.default_rng(version + 10 * compress)
    m = rng.standard_normal((7, 11))
    m[2, 3] = np.nan
    m[4, 5] = np.inf
    cols = [f"gene_{i}" for i in range(11)]
    p = str(tmp_path / "m.rds")
    write_rds(p, m, [f"s{i}" for i in range(7)], cols, version=version, compress=compress)
    got = N.read_rds_matrix(p)
    np.testing.assert_array_equal(got.values.view(np.uint64), m.view(np.uint64))
    assert got.colnames == cols


def test_rds_without_dimnames(tmp_path):
    m = np.arange(12.0).reshape(3, 4)
    p = str(tmp_path / "m.rds")
    write_rds(p, m)
    got = N.read_rds_matrix(p)
    np.testing.assert_array_equal(got.values, m)
    assert got.colnames is None


def test_rda_by_name_with_back_references(tmp_path):
    a = np.ones((2, 3))
    b = np.arange(20.0).reshape(4, 5)
    p = str(tmp_path / "x.rda")
    write_rda(p, [("labels", "strings", ["x", "y"]), ("first", "matrix", (a, None, ["p", "q", "r"])),
                  ("second", "matrix", (b, ["r1", "r2", "r3", "r4"], list("abcde")))])
    got = N.read_rds_matrix(p, "second")   # "dim"/"dimnames" are back-references here
    np.testing.assert_array_equal(got.values, b)
    assert got.colnames == list("abcde")
    first = N.read_rds_matrix(p)            # no name: the first numeric matrix
    np.testing.assert_array_equal(first.values, a)


def test_errors(tmp_path):
    p = str(tmp_path / "v.rda")
    write_rda(p, [("labels", "strings", ["x"])])
    with pytest.raises(NetRepError):
        N.read_rds_matrix(p)
    with pytest.raises(NetRepError):
        N.read_rds_matrix(str(tmp_path / "missing.rds"))
    q = str(tmp_path / "t.rds")
    with open(q, "wb") as f:
        f.write(b"X\n\x00\x00")   # truncated
    with pytest.raises(NetRepError):
        N.read_rds_matrix(q)


def test_reads_the_references_own_rda(tmp_path):
    """data/NetRep.rda as R wrote it (RDX2/3, xz): every matrix and its column
    names equal the golden arrays decoded by oracle/rda.py."""
    raw = lzma.decompress(open(os.path.join(GOLDEN, "NetRep.rda"), "rb").read())
    p = str(tmp_path / "NetRep_plain.rda")
    open(p, "wb").write(raw)
    gold = np.load(os.path.join(GOLDEN, "netrep_bundled.npz"), allow_pickle=False)
    for name in ("discovery_data", "test_data", "discovery_correlation", "test_correlation",
                 "discovery_network", "test_network"):
        got = N.read_rds_matrix(p, name)
        np.testing.assert_array_equal(got.values, gold[name])
        assert got.colnames == list(gold[name + "_colnames"])


def _forged(path, body_parts):
    import struct
    data = b"X\n" + struct.pack(">iii", 2, 0x040301, 0x020300) + b"".join(body_parts)
    with open(path, "wb") as f:
        f.write(data)


def test_forged_lengths_fail_cleanly(tmp_path):
    """lengths in an untrusted file are bounded before anything is
    allocated or skipped -- a forged long-vector length (2^60), a huge string
    length in the dimnames, and negative dims come back as NetRepError
    (NR_ERR_INVALID), never std::bad_alloc / std::terminate."""
    import struct
    p = str(tmp_path / "long.rds")
    # REALSXP with a long length of 2^60 (beyond R_XLEN_T_MAX = 2^52)
    _forged(p, [struct.pack(">iiii", 14 | (1 << 9), -1, 1 << 28, 0)])
    with pytest.raises(NetRepError) as ei:
        N.read_rds_matrix(p)
    assert ei.value.code == 2 and "limit" in str(ei.value)
    # a 1x1 matrix whose colnames CHARSXP claims 2^31-1 bytes (then EOF)
    q = str(tmp_path / "str.rds")
    parts = [struct.pack(">ii", 14 | (1 << 9), 1), struct.pack(">d", 1.0),
             struct.pack(">i", 2 | (1 << 10)), struct.pack(">i", 1), struct.pack(">ii", 0x00040009, 3), b"dim",
             struct.pack(">iiii", 13, 2, 1, 1),
             struct.pack(">i", 2 | (1 << 10)), struct.pack(">i", 1), struct.pack(">ii", 0x00040009, 8), b"dimnames",
             struct.pack(">ii", 19, 2), struct.pack(">i", 254),
             struct.pack(">ii", 16, 1), struct.pack(">ii", 0x00040009, 2**31 - 1), b"abc"]
    _forged(q, parts)
    with pytest.raises(NetRepError) as ei:
        N.read_rds_matrix(q)
    assert ei.value.code == 2
    # a character vector claiming 2^52 entries
    r = str(tmp_path / "vec.rds")
    parts2 = parts[:-2] + [struct.pack(">iiii", 16, -1, 1 << 20, 0)]
    _forged(r, parts2)
    with pytest.raises(NetRepError):
        N.read_rds_matrix(r)


def test_negative_dims_rejected(tmp_path):
    """dim = (-2, -3) with a 6-element payload is not a matrix."""
    import struct
    p = str(tmp_path / "neg.rds")
    parts = [struct.pack(">ii", 14 | (1 << 9), 6), np.arange(6.0).astype(">f8").tobytes(),
             struct.pack(">i", 2 | (1 << 10)), struct.pack(">i", 1), struct.pack(">ii", 0x00040009, 3), b"dim",
             struct.pack(">iiii", 13, 2, -2, -3), struct.pack(">i", 254)]
    _forged(p, parts)
    with pytest.raises(NetRepError):
        N.read_rds_matrix(p)


def test_altrep_dimnames_reported(tmp_path):
    """R >= 3.5 ALTREP (compact) dimnames are not decoded; the error says so."""
    import struct
    p = str(tmp_path / "alt.rds")
    parts = [struct.pack(">ii", 14 | (1 << 9), 1), struct.pack(">d", 1.0),
             struct.pack(">i", 2 | (1 << 10)), struct.pack(">i", 1), struct.pack(">ii", 0x00040009, 3), b"dim",
             struct.pack(">iiii", 13, 2, 1, 1),
             struct.pack(">i", 2 | (1 << 10)), struct.pack(">i", 1), struct.pack(">ii", 0x00040009, 8), b"dimnames",
             struct.pack(">ii", 19, 2), struct.pack(">i", 254), struct.pack(">i", 238)]
    _forged(p, parts)
    with pytest.raises(NetRepError) as ei:
        N.read_rds_matrix(p)
    assert "ALTREP" in str(ei.value)
