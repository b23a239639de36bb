// Host program that calls the C ABI exactly as the Rcpp glue would
// (INTEGRATION.md): plain C++ against include/netrep_gpu.h, linked with
// libnetrep_amd.so, no Python in between. Built by tests/abi_driver/Makefile
// (g++); driven by tests/test_abi_driver.py.
//
//   abi_driver perm <dir>       netrep_PermutationProcedure on the case in
//                               <dir> (written by the test), outputs
//                               nulls.f64 / observed.f64 / rc.txt into <dir>
//   abi_driver interrupt <dir>  same case, with an interrupt hook that fires
//                               on its 3rd poll (~200 ms in); writes the
//                               partial cube and rc
//   abi_driver progress <dir>   same case with verbose = 1 and a progress
//                               hook that records every call (progress.txt:
//                               "event done total" lines) -- the library
//                               itself must print nothing
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/netrep_gpu.h"

namespace {

template <typename T>
std::vector<T> read_bin(const std::string& path) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  if (!f) return {};
  const std::streamsize n = f.tellg();
  f.seekg(0);
  std::vector<T> v((size_t)n / sizeof(T));
  f.read(reinterpret_cast<char*>(v.data()), n);
  return v;
}

template <typename T>
void write_bin(const std::string& path, const T* p, size_t n) {
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char*>(p), (std::streamsize)(n * sizeof(T)));
}

std::vector<std::string> read_lines(const std::string& path) {
  std::ifstream f(path);
  std::vector<std::string> v;
  std::string s;
  while (std::getline(f, s)) v.push_back(s);
  return v;
}

std::vector<const char*> cstrs(const std::vector<std::string>& v) {
  std::vector<const char*> p;
  for (const auto& s : v) p.push_back(s.c_str());
  return p;
}

std::atomic<int> g_polls{0};
int interrupt_on_third_poll(void*) { return ++g_polls >= 3 ? 1 : 0; }

// The Rcpp glue would write netrep_format_progress's line to Rcpp::Rcout
// (INTEGRATION.md); here every call is recorded with the formatted line.
void record_progress(int32_t event, int64_t done, int64_t total, void* user) {
  auto* log = static_cast<std::vector<std::string>*>(user);
  char line[64] = "";
  if (event == NETREP_PROGRESS_UPDATE) netrep_format_progress(done, total, line, sizeof(line));
  std::ostringstream s;
  s << event << " " << done << " " << total << " " << (line[0] ? line + 1 : "-");  // drop the '\r'
  log->push_back(s.str());
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: abi_driver perm|interrupt|progress <dir>\n");
    return 2;
  }
  const std::string mode = argv[1], dir = std::string(argv[2]) + "/";
  // meta.txt: n_samples n_nodes n_perm seed null_hypothesis with_data use_pi
  std::ifstream mf(dir + "meta.txt");
  int64_t S = 0, N = 0, n_perm = 0;
  uint64_t seed = 0;
  std::string null_h;
  int with_data = 0, use_pi = 0;
  mf >> S >> N >> n_perm >> seed >> null_h >> with_data >> use_pi;
  const auto data = read_bin<double>(dir + "data.f64");
  const auto corr = read_bin<double>(dir + "corr.f64");
  const auto net = read_bin<double>(dir + "net.f64");
  const auto t_names = read_lines(dir + "t_names.txt");
  const auto ma_names = read_lines(dir + "ma_names.txt");
  const auto ma_labels = read_lines(dir + "ma_labels.txt");
  const auto modules = read_lines(dir + "modules.txt");
  const auto pi = read_bin<uint32_t>(dir + "pi.u32");
  if ((int64_t)corr.size() != N * N || (int64_t)t_names.size() != N) {
    std::fprintf(stderr, "bad case files\n");
    return 2;
  }
  // discovery vectors, concatenated per module in `modules` order with lengths
  const auto dwd = read_bin<double>(dir + "disc_degree.f64");
  const auto dcv = read_bin<double>(dir + "disc_corr.f64");
  const auto dnc = read_bin<double>(dir + "disc_contribution.f64");
  const auto lens = read_bin<int64_t>(dir + "disc_lens.i64");  // [M x 3]: degree, corr, contribution
  const size_t M = modules.size();
  std::vector<const double*> pwd(M, nullptr), pcv(M, nullptr), pnc(M, nullptr);
  std::vector<int64_t> lwd(M), lcv(M), lnc(M);
  size_t owd = 0, ocv = 0, onc = 0;
  for (size_t m = 0; m < M; ++m) {
    lwd[m] = lens[3 * m];
    lcv[m] = lens[3 * m + 1];
    lnc[m] = lens[3 * m + 2];
    if (lwd[m] > 0) pwd[m] = dwd.data() + owd;
    if (lcv[m] > 0 || lwd[m] == 1) pcv[m] = dcv.data() + ocv;
    if (lnc[m] > 0) pnc[m] = dnc.data() + onc;
    owd += (size_t)lwd[m];
    ocv += (size_t)lcv[m];
    onc += (size_t)lnc[m];
  }
  netrep_disc_props dp = {pwd.data(), lwd.data(), pcv.data(), lcv.data(),
                          with_data ? pnc.data() : nullptr, with_data ? lnc.data() : nullptr};
  auto tn = cstrs(t_names), an = cstrs(ma_names), al = cstrs(ma_labels), mn = cstrs(modules);
  const int n_stat = with_data ? NR_NSTAT_DATA : NR_NSTAT_NODATA;
  std::vector<double> nulls((size_t)(M * n_stat * n_perm)), observed(M * n_stat);
  if (mode == "interrupt") netrep_set_interrupt_hook(interrupt_on_third_poll, nullptr);
  std::vector<std::string> progress_log;
  if (mode == "progress") netrep_set_progress_hook(record_progress, &progress_log);
  const int rc = netrep_PermutationProcedure(
      &dp, with_data ? data.data() : nullptr, corr.data(), net.data(), S, N, tn.data(), an.data(), al.data(),
      (int64_t)an.size(), mn.data(), (int64_t)M, n_perm, 1, null_h.c_str(), mode == "progress" ? 1 : 0, seed,
      use_pi ? pi.data() : nullptr, nulls.data(), observed.data());
  netrep_set_interrupt_hook(nullptr, nullptr);
  netrep_set_progress_hook(nullptr, nullptr);
  if (mode == "progress") {
    std::ofstream pf(dir + "progress.txt");
    for (const auto& s : progress_log) pf << s << "\n";
  }
  std::ofstream(dir + "rc.txt") << rc << "\n" << netrep_last_error() << "\n";
  write_bin(dir + "nulls.f64", nulls.data(), nulls.size());
  write_bin(dir + "observed.f64", observed.data(), observed.size());
  return 0;
}
