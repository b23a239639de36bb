"""Writer of R's XDR serialisation for numeric matrices -- TEST INFRASTRUCTURE
for the RDS / save() reader (netrep_amd/csrc/rds_reader.cpp). Emits what
saveRDS(x) / save(...) write for a double matrix with optional dimnames:
format 2 or 3 header, REALSXP payload (big-endian), then the attribute
pairlist (dim, dimnames) with symbols and back-references (REFSXP) as R does.
The reader is also pinned against a file R itself wrote (tests/golden/NetRep.rda,
the reference's bundled data)."""
import gzip
import struct

import numpy as np


class _W:
    def __init__(self):
        self.parts = []
        self.syms = []

    def i(self, v):
        self.parts.append(struct.pack(">i", v))

    def raw(self, b):
        self.parts.append(b)

    def length(self, n):
        if n < 2**31 - 1:
            self.i(n)
        else:
            self.i(-1)
            self.i(n >> 32)
            self.i(n & 0xFFFFFFFF)

    def charsxp(self, s):
        if s is None:
            self.i(9)
            self.i(-1)
            return
        b = s.encode()
        self.i(0x00040009)  # CHARSXP, ASCII level bit as R writes it
        self.i(len(b))
        self.raw(b)

    def symbol(self, name):
        if name in self.syms:
            self.i(((self.syms.index(name) + 1) << 8) | 255)  # REFSXP
        else:
            self.syms.append(name)
            self.i(1)
            self.charsxp(name)

    def strsxp(self, names):
        if names is None:
            self.i(254)
            return
        self.i(16)
        self.length(len(names))
        for s in names:
            self.charsxp(s)

    def matrix(self, m, rownames=None, colnames=None):
        m = np.asarray(m, dtype=np.float64)
        nrow, ncol = m.shape
        self.i(14 | (1 << 9))
        self.length(m.size)
        self.raw(np.asfortranarray(m).T.astype(">f8").tobytes())
        self.i(2 | (1 << 10))
        self.symbol("dim")
        self.i(13)
        self.length(2)
        self.i(nrow)
        self.i(ncol)
        if rownames is not None or colnames is not None:
            self.i(2 | (1 << 10))
            self.symbol("dimnames")
            self.i(19)
            self.length(2)
            self.strsxp(rownames)
            self.strsxp(colnames)
        self.i(254)

    def header(self, version):
        self.raw(b"X\n")
        self.i(version)
        self.i(0x040301)
        self.i(0x030500 if version == 3 else 0x020300)
        if version == 3:
            self.i(5)
            self.raw(b"UTF-8")

    def bytes(self):
        return b"".join(self.parts)


def write_rds(path, m, rownames=None, colnames=None, version=3, compress=True):
    w = _W()
    w.header(version)
    w.matrix(m, rownames, colnames)
    data = w.bytes()
    with (gzip.open(path, "wb") if compress else open(path, "wb")) as f:
        f.write(data)


def write_rda(path, objects, version=3, compress=True):
    """objects: list of (name, kind, value) with kind 'matrix' (value = (m,
    rownames, colnames)) or 'strings' (a character vector)."""
    w = _W()
    w.raw(b"RDX3\n" if version == 3 else b"RDX2\n")
    w.header(version)
    for name, kind, value in objects:
        w.i(2 | (1 << 10))
        w.symbol(name)
        if kind == "matrix":
            w.matrix(*value)
        else:
            w.strsxp(value)
    w.i(254)
    data = w.bytes()
    with (gzip.open(path, "wb") if compress else open(path, "wb")) as f:
        f.write(data)
