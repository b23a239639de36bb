"""Minimal reader for R's XDR serialisation (RDX2 / RDX3 ``.rda`` files).

TEST INFRASTRUCTURE ONLY. Used by ``tests/golden/make_golden.py`` to turn the
reference's bundled example data (``data/NetRep.rda``, documented in
R/example-data.R:1-174) into numpy fixtures. It executes nothing from the
file: it only decodes the typed value stream (reals, integers, strings,
lists, attribute pairlists).

Supported SEXP types are the ones a saved numeric matrix / named vector
uses: NILVALUE, SYMSXP, LISTSXP (pairlist), CHARSXP, LGLSXP, INTSXP,
REALSXP, STRSXP, VECSXP and back-references (REFSXP).
"""
from __future__ import annotations

import bz2
import gzip
import lzma
import struct

import numpy as np

_NILVALUE = 254
_REFSXP = 255
_GLOBALENV = 253
_EMPTYENV = 242
_BASEENV = 241
_MISSINGARG = 251
_SYMSXP = 1
_LISTSXP = 2
_CHARSXP = 9
_LGLSXP = 10
_INTSXP = 13
_REALSXP = 14
_STRSXP = 16
_VECSXP = 19
_NA_INT = -2147483648


class RObject:
    """A decoded R value plus its attributes (``names``, ``dim``, ``dimnames``)."""

    def __init__(self, value, attrs=None):
        self.value = value
        self.attrs = attrs or {}

    def __repr__(self):  # pragma: no cover - debugging aid
        return f"RObject({type(self.value).__name__}, attrs={list(self.attrs)})"


class _Reader:
    def __init__(self, buf: bytes):
        self.buf = buf
        self.pos = 0
        self.refs = []

    def _int(self) -> int:
        (v,) = struct.unpack_from(">i", self.buf, self.pos)
        self.pos += 4
        return v

    def _bytes(self, n: int) -> bytes:
        b = self.buf[self.pos:self.pos + n]
        self.pos += n
        return b

    def _length(self) -> int:
        n = self._int()
        if n == -1:  # long vector: two more ints
            hi, lo = self._int(), self._int()
            n = (hi << 32) + (lo & 0xFFFFFFFF)
        return n

    def read_item(self):
        flags = self._int()
        typ = flags & 0xFF
        has_attr = bool(flags & (1 << 9))
        has_tag = bool(flags & (1 << 10))
        if typ == _NILVALUE:
            return None
        if typ in (_GLOBALENV, _EMPTYENV, _BASEENV, _MISSINGARG):
            return None
        if typ == _REFSXP:
            idx = flags >> 8
            if idx == 0:
                idx = self._int()
            return self.refs[idx - 1]
        if typ == _SYMSXP:
            name = self.read_item()  # a CHARSXP
            self.refs.append(name)
            return name
        if typ == _LISTSXP:
            attrs = self._read_attrs() if has_attr else {}
            tag = self.read_item() if has_tag else None
            car = self.read_item()
            cdr = self.read_item()
            node = [(tag, car)]
            if isinstance(cdr, list):
                node.extend(cdr)
            return node if not attrs else node
        if typ == _CHARSXP:
            n = self._int()
            if n == -1:
                return None  # NA_character_
            return self._bytes(n).decode("utf-8", errors="replace")
        if typ in (_LGLSXP, _INTSXP):
            n = self._length()
            arr = np.frombuffer(self._bytes(4 * n), dtype=">i4").astype(np.int64)
            return self._wrap(arr, has_attr)
        if typ == _REALSXP:
            n = self._length()
            arr = np.frombuffer(self._bytes(8 * n), dtype=">f8").astype(np.float64)
            return self._wrap(arr, has_attr)
        if typ == _STRSXP:
            n = self._length()
            arr = [self.read_item() for _ in range(n)]
            return self._wrap(arr, has_attr)
        if typ == _VECSXP:
            n = self._length()
            arr = [self.read_item() for _ in range(n)]
            return self._wrap(arr, has_attr)
        raise ValueError(f"unsupported SEXP type {typ} at byte {self.pos}")

    def _wrap(self, value, has_attr):
        attrs = self._read_attrs() if has_attr else {}
        return RObject(value, attrs)

    def _read_attrs(self):
        plist = self.read_item()
        out = {}
        for tag, val in plist or []:
            out[tag] = val
        return out


def read_rda(path: str) -> dict:
    """Return ``{name: RObject}`` for every object saved in an ``.rda`` file."""
    raw = open(path, "rb").read()
    if raw[:6] == b"\xfd7zXZ\x00":
        raw = lzma.decompress(raw)
    elif raw[:2] == b"\x1f\x8b":
        raw = gzip.decompress(raw)
    elif raw[:3] == b"BZh":
        raw = bz2.decompress(raw)
    if raw[:5] not in (b"RDX2\n", b"RDX3\n"):
        raise ValueError("not an RDX2/RDX3 file")
    version3 = raw[:5] == b"RDX3\n"
    r = _Reader(raw)
    r.pos = 5
    if r._bytes(2) != b"X\n":
        raise ValueError("only XDR-format .rda files are supported")
    r._int()  # format version
    r._int()  # writer R version
    r._int()  # minimal reader R version
    if version3:
        n = r._int()
        r._bytes(n)  # native encoding name
    top = r.read_item()
    return {tag: val for tag, val in top}


def as_matrix(obj: RObject):
    """Column-major R matrix -> (np.ndarray[nrow, ncol], rownames, colnames)."""
    nrow, ncol = (int(x) for x in obj.attrs["dim"].value)
    mat = np.asarray(obj.value, dtype=np.float64).reshape((ncol, nrow)).T
    dn = obj.attrs.get("dimnames")
    rown = coln = None
    if dn is not None:
        rown = dn.value[0].value if dn.value[0] is not None else None
        coln = dn.value[1].value if dn.value[1] is not None else None
    return np.ascontiguousarray(mat), rown, coln


def as_named_vector(obj: RObject):
    """R named atomic vector -> (values, names)."""
    names = obj.attrs["names"].value if "names" in obj.attrs else None
    return obj.value, names
