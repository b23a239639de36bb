// R XDR serialisation reader for one numeric matrix (rds_reader.h).
//
// Item header: one int of flags -- type = flags & 0xFF, object bit 8,
// attribute bit 9, tag bit 10; back-references (REFSXP) carry their index in
// flags >> 8 (0: the index follows as an int). Vectors store a length (int,
// or -1 followed by two ints for long vectors) and their elements, then their
// attribute pairlist; pairlist nodes store attributes, tag, CAR, CDR in that
// order. Only the item kinds a saved numeric matrix and its neighbours in a
// save() archive use are decoded; anything else is an error, never executed.
#include "rds_reader.h"

#include <zlib.h>

#include <algorithm>
#include <cstring>

namespace nr {
namespace {

enum : int {
  kSym = 1, kList = 2, kClos = 3, kProm = 5, kLang = 6, kChar = 9, kLgl = 10, kInt = 13, kReal = 14,
  kCplx = 15, kStr = 16, kDot = 17, kVec = 19, kExpr = 20, kRaw = 24, kS4 = 25, kAltrep = 238,
  kBaseEnv = 241, kEmptyEnv = 242, kMissingArg = 251, kUnbound = 252, kGlobalEnv = 253,
  kNil = 254, kRef = 255
};

inline int32_t be32(const unsigned char* p) {
  return (int32_t)((uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | (uint32_t)p[3]);
}

}  // namespace

RMatrixReader::~RMatrixReader() {
  if (f_) gzclose((gzFile)f_);
}

bool RMatrixReader::bytes(void* dst, int64_t n) {
  unsigned char* d = static_cast<unsigned char*>(dst);
  while (n > 0) {
    const unsigned part = (unsigned)(n < (1 << 30) ? n : (1 << 30));
    const int got = gzread((gzFile)f_, d, part);
    if (got <= 0) return fail("unexpected end of the serialised stream");
    d += got;
    n -= got;
  }
  return true;
}

bool RMatrixReader::skip(int64_t n) {
  unsigned char buf[1 << 16];
  while (n > 0) {
    const int64_t part = n < (int64_t)sizeof(buf) ? n : (int64_t)sizeof(buf);
    if (!bytes(buf, part)) return false;
    n -= part;
  }
  return true;
}

bool RMatrixReader::i32(int32_t* v) {
  unsigned char b[4];
  if (!bytes(b, 4)) return false;
  *v = be32(b);
  return true;
}

bool RMatrixReader::length_field(int64_t* n) {
  int32_t a;
  if (!i32(&a)) return false;
  if (a != -1) {
    if (a < 0) return fail("negative vector length");
    *n = a;
    return true;
  }
  int32_t hi, lo;
  if (!i32(&hi) || !i32(&lo)) return false;
  *n = ((int64_t)(uint32_t)hi << 32) | (int64_t)(uint32_t)lo;
  // R_XLEN_T_MAX = 2^52: a larger long length is a corrupt or forged header
  if (*n < 0 || *n > ((int64_t)1 << 52)) return fail("vector length beyond R's limit (corrupt file)");
  return true;
}

// "X\n", format version, writer and minimal reader R versions, and (format 3)
// the native encoding; save() archives start with "RDX2\n" / "RDX3\n".
bool RMatrixReader::header() {
  unsigned char m[5];
  if (!bytes(m, 2)) return false;
  if (m[0] == 'R' && m[1] == 'D') {
    if (!bytes(m + 2, 3)) return false;
    if (m[2] != 'X' || (m[3] != '2' && m[3] != '3') || m[4] != '\n') return fail("not an RDX2/RDX3 archive");
    rda_ = true;
    if (!bytes(m, 2)) return false;
  }
  if (m[0] != 'X' || m[1] != '\n')
    return fail(m[0] == 'A' || m[0] == 'B' ? "only XDR (binary, big-endian) serialisation is supported"
                                           : "not an R serialisation stream (or bzip2/xz compressed; "
                                             "gzip and uncompressed are supported)");
  int32_t version, writer, reader;
  if (!i32(&version) || !i32(&writer) || !i32(&reader)) return false;
  if (version != 2 && version != 3) return fail("unsupported serialisation format version");
  if (version == 3) {
    int32_t n;
    if (!i32(&n)) return false;
    if (n < 0 || n > 4096) return fail("bad native-encoding field");
    if (!skip(n)) return false;
  }
  return true;
}

bool RMatrixReader::read_charsxp(std::string* s, bool* na) {
  int32_t flags;
  if (!i32(&flags)) return false;
  if ((flags & 0xFF) != kChar) return fail("expected a CHARSXP");
  int32_t n;
  if (!i32(&n)) return false;
  *na = n == -1;
  s->clear();
  if (n == -1) return true;
  if (n < 0) return fail("bad string length");
  // grown as the bytes arrive: a forged length ends at the end of the stream,
  // not in a multi-gigabyte allocation
  char buf[4096];
  for (int32_t left = n; left > 0;) {
    const int32_t part = left < (int32_t)sizeof(buf) ? left : (int32_t)sizeof(buf);
    if (!bytes(buf, part)) return false;
    s->append(buf, (size_t)part);
    left -= part;
  }
  return true;
}

// A tag: a symbol (recorded for later back-references) or a back-reference.
bool RMatrixReader::symbol_name(int32_t flags, std::string* name) {
  const int type = flags & 0xFF;
  if (type == kRef) {
    int64_t idx = (uint32_t)flags >> 8;
    if (idx == 0) {
      int32_t v;
      if (!i32(&v)) return false;
      idx = v;
    }
    if (idx < 1 || idx > (int64_t)refs_.size()) return fail("dangling back-reference");
    *name = refs_[(size_t)(idx - 1)];
    return true;
  }
  if (type != kSym) return fail("expected a symbol");
  bool na;
  if (!read_charsxp(name, &na)) return false;
  refs_.push_back(*name);
  return true;
}

bool RMatrixReader::skip_item(int depth) {
  if (depth > 64) return fail("serialised object nested too deeply");
  int32_t flags;
  if (!i32(&flags)) return false;
  const int type = flags & 0xFF;
  const bool has_attr = flags & (1 << 9), has_tag = flags & (1 << 10);
  switch (type) {
    case kNil: case kGlobalEnv: case kEmptyEnv: case kBaseEnv: case kMissingArg: case kUnbound:
      return true;
    case kRef:
      if (((uint32_t)flags >> 8) == 0) {
        int32_t v;
        return i32(&v);
      }
      return true;
    case kSym: {
      std::string nm;
      return symbol_name(flags, &nm);
    }
    case kList: case kLang: case kClos: case kProm: case kDot: {
      if (has_attr && !skip_item(depth + 1)) return false;
      if (has_tag && !skip_item(depth + 1)) return false;
      return skip_item(depth + 1) && skip_item(depth + 1);  // CAR, CDR
    }
    case kChar: {
      int32_t n;
      if (!i32(&n)) return false;
      return n <= 0 || skip(n);
    }
    case kLgl: case kInt: case kReal: case kCplx: case kRaw: {
      int64_t n;
      if (!length_field(&n)) return false;
      const int64_t w = type == kReal ? 8 : type == kCplx ? 16 : type == kRaw ? 1 : 4;
      if (!skip(n * w)) return false;  // n <= 2^52 (length_field): no overflow
      return !has_attr || skip_item(depth + 1);
    }
    case kStr: case kVec: case kExpr: {
      int64_t n;
      if (!length_field(&n)) return false;
      for (int64_t i = 0; i < n; ++i)
        if (!skip_item(depth + 1)) return false;
      return !has_attr || skip_item(depth + 1);
    }
    case kS4:
      return !has_attr || skip_item(depth + 1);
    case kAltrep:
      // R >= 3.5 compact / deferred vectors (e.g. dimnames from
      // as.character(1:n)) are not decoded: re-save with
      // saveRDS(unserialize(serialize(x, NULL, version = 2)))
      return fail("ALTREP-encoded object (R >= 3.5 compact vector) is not supported; re-save the matrix "
                  "with serialisation version 2");
    default:
      return fail("unsupported item type " + std::to_string(type) + " in the serialised stream");
  }
}

bool RMatrixReader::open(const char* path, const char* name) {
  f_ = gzopen(path, "rb");  // gzip or plain: zlib reads both
  if (!f_) return fail(std::string("cannot open ") + path);
  gzbuffer((gzFile)f_, 1 << 20);
  if (!header()) return false;
  const std::string want = name ? name : "";
  if (!rda_) {
    int32_t flags;
    if (!i32(&flags)) return false;
    if ((flags & 0xFF) != kReal) return fail("the file does not hold a numeric (double) matrix");
    has_attr_ = flags & (1 << 9);
    return length_field(&length_);
  }
  // save() archive: a pairlist of (name, object)
  for (;;) {
    int32_t flags;
    if (!i32(&flags)) return false;
    const int type = flags & 0xFF;
    if (type == kNil) return fail(want.empty() ? "no numeric matrix in the archive" : "no object '" + want + "' in the archive");
    if (type != kList || !(flags & (1 << 10))) return fail("malformed save() archive");
    if ((flags & (1 << 9)) && !skip_item(1)) return false;
    int32_t tflags;
    std::string tag;
    if (!i32(&tflags) || !symbol_name(tflags, &tag)) return false;
    int32_t cflags;
    if (!i32(&cflags)) return false;
    const bool real = (cflags & 0xFF) == kReal;
    if (real && (want.empty() || tag == want)) {
      has_attr_ = cflags & (1 << 9);
      return length_field(&length_);
    }
    if (!want.empty() && tag == want) return fail("object '" + want + "' is not a numeric matrix");
    // skip this object: its flags are already consumed
    const int ct = cflags & 0xFF;
    const bool c_attr = cflags & (1 << 9);
    if (ct == kLgl || ct == kInt || ct == kReal || ct == kCplx || ct == kRaw) {
      int64_t n;
      if (!length_field(&n)) return false;
      const int64_t w = ct == kReal ? 8 : ct == kCplx ? 16 : ct == kRaw ? 1 : 4;
      if (!skip(n * w)) return false;
      if (c_attr && !skip_item(1)) return false;
    } else if (ct == kStr || ct == kVec || ct == kExpr) {
      int64_t n;
      if (!length_field(&n)) return false;
      for (int64_t i = 0; i < n; ++i)
        if (!skip_item(1)) return false;
      if (c_attr && !skip_item(1)) return false;
    } else {
      return fail("unsupported object type " + std::to_string(ct) + " in the archive");
    }
  }
}

bool RMatrixReader::read_raw(void* dst, int64_t n) {
  if (consumed_ + n > length_) return fail("read past the matrix payload");
  if (!bytes(dst, n * 8)) return false;
  consumed_ += n;
  return true;
}

bool RMatrixReader::read_string_vector(std::vector<std::string>* out, int depth) {
  int32_t flags;
  if (!i32(&flags)) return false;
  const int type = flags & 0xFF;
  out->clear();
  if (type == kNil) return true;
  if (type == kAltrep)
    return fail("ALTREP-encoded dimnames (R >= 3.5 compact vector) are not supported; re-save the matrix "
                "with serialisation version 2");
  if (type != kStr) return fail("dimnames entry is not a character vector");
  int64_t n;
  if (!length_field(&n)) return false;
  out->reserve((size_t)(n < (1 << 16) ? n : (1 << 16)));  // grown as the strings arrive
  for (int64_t i = 0; i < n; ++i) {
    bool na;
    std::string s;
    if (!read_charsxp(&s, &na)) return false;
    out->push_back(na ? std::string("NA") : std::move(s));
  }
  return !(flags & (1 << 9)) || skip_item(depth + 1);
}

bool RMatrixReader::read_attributes(RMatrixMeta* meta, int depth) {
  for (;;) {
    int32_t flags;
    if (!i32(&flags)) return false;
    const int type = flags & 0xFF;
    if (type == kNil) return true;
    if (type != kList || !(flags & (1 << 10))) return fail("malformed attribute list");
    if ((flags & (1 << 9)) && !skip_item(depth + 1)) return false;
    int32_t tflags;
    std::string tag;
    if (!i32(&tflags) || !symbol_name(tflags, &tag)) return false;
    if (tag == "dim") {
      int32_t cflags;
      if (!i32(&cflags)) return false;
      if ((cflags & 0xFF) != kInt) return fail("dim is not an integer vector");
      int64_t n;
      if (!length_field(&n)) return false;
      if (n != 2) return fail("the object is not a matrix (dim of length " + std::to_string(n) + ")");
      int32_t r, c;
      if (!i32(&r) || !i32(&c)) return false;
      meta->nrow = r;
      meta->ncol = c;
      if ((cflags & (1 << 9)) && !skip_item(depth + 1)) return false;
    } else if (tag == "dimnames") {
      int32_t cflags;
      if (!i32(&cflags)) return false;
      if ((cflags & 0xFF) != kVec) return fail("dimnames is not a list");
      int64_t n;
      if (!length_field(&n)) return false;
      if (n != 2) return fail("dimnames of length other than 2");
      if (!read_string_vector(&meta->rownames, depth + 1) || !read_string_vector(&meta->colnames, depth + 1))
        return false;
      if ((cflags & (1 << 9)) && !skip_item(depth + 1)) return false;
    } else if (!skip_item(depth + 1)) {
      return false;
    }
  }
}

bool RMatrixReader::finish(RMatrixMeta* meta) {
  if (consumed_ != length_) return fail("matrix payload not fully read");
  *meta = RMatrixMeta();
  if (has_attr_ && !read_attributes(meta, 1)) return false;
  if (meta->nrow <= 0 || meta->ncol <= 0) return fail("the object has no (positive) dim attribute (not a matrix)");
  if (meta->nrow * meta->ncol != length_) return fail("dim does not match the payload length");
  if (!meta->rownames.empty() && (int64_t)meta->rownames.size() != meta->nrow) return fail("bad rownames length");
  if (!meta->colnames.empty() && (int64_t)meta->colnames.size() != meta->ncol) return fail("bad colnames length");
  return true;
}

bool read_matrix_host(const char* path, const char* name, RMatrixMeta* meta, std::vector<double>* values,
                      bool want_values, std::string* err) {
  RMatrixReader r;
  bool ok = r.open(path, name);
  if (ok) {
    const int64_t n = r.length();
    if (want_values) {
      try {
        values->resize((size_t)n);
      } catch (const std::exception&) {
        if (err) *err = "cannot allocate " + std::to_string(n) + " doubles for the matrix";
        return false;
      }
      ok = r.read_raw(values->data(), n);
      if (ok) {
        unsigned char* p = reinterpret_cast<unsigned char*>(values->data());
        for (int64_t i = 0; i < n; ++i, p += 8) {
          for (int b = 0; b < 4; ++b) {
            const unsigned char t = p[b];
            p[b] = p[7 - b];
            p[7 - b] = t;
          }
        }
      }
    } else {
      std::vector<double> tmp((size_t)std::min<int64_t>(n, 1 << 16));
      for (int64_t o = 0; ok && o < n; o += (int64_t)tmp.size())
        ok = r.read_raw(tmp.data(), std::min<int64_t>((int64_t)tmp.size(), n - o));
    }
  }
  if (ok) ok = r.finish(meta);
  if (!ok && err) *err = r.error();
  return ok;
}

}  // namespace nr
