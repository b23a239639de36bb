// Streaming reader for one numeric matrix in R's XDR serialisation: the
// files disk.matrix points at (R/disk-matrix-class.R:175-182 reads them back
// with readRDS), i.e. saveRDS output (gzip-compressed or plain, format
// version 2 or 3), and, by object name, save() archives (RDX2 / RDX3).
//
// The payload is handed out raw (big-endian XDR doubles) in caller-sized
// pieces, so a caller can read it straight into pinned staging buffers and
// convert on the device; the dim / dimnames attributes follow the payload in
// the stream and are read by finish(). Nothing in a file is executed: only
// the typed value stream of a numeric matrix is decoded.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace nr {

struct RMatrixMeta {
  int64_t nrow = 0, ncol = 0;
  std::vector<std::string> rownames, colnames;
};

class RMatrixReader {
 public:
  RMatrixReader() = default;
  ~RMatrixReader();
  RMatrixReader(const RMatrixReader&) = delete;
  RMatrixReader& operator=(const RMatrixReader&) = delete;

  // Opens `path` and positions the stream at the payload of the matrix: the
  // top-level object of an RDS file, or the object called `name` of a save()
  // archive (the first numeric matrix when `name` is NULL or empty).
  bool open(const char* path, const char* name);
  int64_t length() const { return length_; }  // doubles in the payload
  // Next n doubles of the payload, raw big-endian.
  bool read_raw(void* dst, int64_t n);
  // Reads the attributes (dim, dimnames); the payload must be consumed.
  bool finish(RMatrixMeta* meta);
  const std::string& error() const { return err_; }

 private:
  bool fail(const std::string& m) {
    if (err_.empty()) err_ = m;
    return false;
  }
  bool bytes(void* dst, int64_t n);
  bool skip(int64_t n);
  bool i32(int32_t* v);
  bool length_field(int64_t* n);
  bool header();
  bool skip_item(int depth);
  bool read_charsxp(std::string* s, bool* na);
  bool read_string_vector(std::vector<std::string>* out, int depth);
  bool read_attributes(RMatrixMeta* meta, int depth);
  bool symbol_name(int32_t flags, std::string* name);

  void* f_ = nullptr;  // gzFile
  bool rda_ = false;
  int64_t length_ = -1, consumed_ = 0;
  bool has_attr_ = false;
  std::vector<std::string> refs_;  // symbols seen (REFSXP targets)
  std::string err_;
};

// Whole-matrix host read (native doubles, column-major) for the C ABI's
// netrep_ReadRDSMatrix and the tests.
bool read_matrix_host(const char* path, const char* name, RMatrixMeta* meta, std::vector<double>* values,
                      bool want_values, std::string* err);

}  // namespace nr
