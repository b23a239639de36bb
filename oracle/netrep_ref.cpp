// C++ CPU restatement of NetRep's permutation procedure -- TEST INFRASTRUCTURE.
//
// The reference's CPU path (src/permutations.cpp, src/permutationsNoData.cpp,
// src/netStats.cpp) restated formula by formula without Rcpp/Armadillo/Boost,
// which are absent here. Used (1) as the parity checker for
// large cases on the GPU box and (2) as bench.py's `cpu_baseline` ("port"):
// the same contiguous per-thread permutation chunks (src/permutations.cpp:
// 338-354), one Fisher-Yates shuffle of the null pool per permutation (as
// arma::shuffle, :63) when no explicit shuffle table is given, LAPACK dgesvd
// with JOBU='S', JOBVT='N' for the summary profile -- what
// arma::svd_econ(U, S, V, X, "left", "dc") (src/netStats.cpp:229) runs:
// Armadillo takes its divide-and-conquer (dgesdd) branch only for mode
// "both" -- and single-threaded LAPACK per worker
// (R/modulePreservation.R:436-437). LAPACK comes from scipy's bundled
// OpenBLAS (symbol scipy_dgesvd_), the only LAPACK in this image;
// ref_init_lapack() loads it by path.
//
// Never linked into or called by the product (netrep_amd/).
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <functional>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

typedef void (*dgesvd_t)(const char* jobu, const char* jobvt, const int* m, const int* n, double* a,
                         const int* lda, double* s, double* u, const int* ldu, double* vt,
                         const int* ldvt, double* work, const int* lwork, int* info);
dgesvd_t g_dgesvd = nullptr;
std::string g_err;

const double kNaN = std::numeric_limits<double>::quiet_NaN();

double na_real() {
  uint64_t b = 0x7FF00000000007A2ull;
  double d;
  std::memcpy(&d, &b, 8);
  return d;
}

// CorrVector src/netStats.cpp:176-204 (idx in module node order)
void corr_vector(const double* corr, int64_t n, const std::vector<int64_t>& idx, std::vector<double>& out) {
  const size_t k = idx.size();
  out.resize(k * (k - 1) / 2);
  size_t v = 0;
  for (size_t jj = 0; jj < k; ++jj)
    for (size_t ii = jj + 1; ii < k; ++ii) out[v++] = corr[idx[ii] + idx[jj] * n];
}

// SortNodes src/netStats.cpp:23-32: sorted copy + rank
void sort_nodes(const std::vector<int64_t>& idx, std::vector<int64_t>& sorted, std::vector<size_t>& rank) {
  const size_t k = idx.size();
  std::vector<size_t> order(k);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return idx[a] < idx[b]; });
  sorted.resize(k);
  rank.resize(k);
  for (size_t i = 0; i < k; ++i) {
    sorted[i] = idx[order[i]];
    rank[order[i]] = i;
  }
}

// arma::sum of a column / vector: Armadillo's arrayops::accumulate (also
// op_sum's proxy loop), two accumulators over the even and odd positions,
// returned as acc1 + acc2 (RcppArmadillo, unvendored, version unpinned:
// DESCRIPTION:28). The order matters for WeightedDegree: its column sums
// include the diagonal (src/netStats.cpp:135-141).
template <class F>
double arma_accumulate(size_t n, F at) {
  double acc1 = 0.0, acc2 = 0.0;
  size_t j = 1;
  for (; j < n; j += 2) {
    acc1 += at(j - 1);
    acc2 += at(j);
  }
  if (j - 1 < n) acc1 += at(j - 1);
  return acc1 + acc2;
}

// WeightedDegree src/netStats.cpp:124-144 on sorted indices: colsum of
// |net(srt, srt)| (diagonal included), minus |diag|; reordered by rank
// (src/permutations.cpp:81-82)
void weighted_degree(const double* net, int64_t n, const std::vector<int64_t>& srt,
                     const std::vector<size_t>& rank, std::vector<double>& wd) {
  const size_t k = srt.size();
  std::vector<double> ws(k);
  for (size_t j = 0; j < k; ++j) {
    const double* col = net + srt[j] * n;
    const double s = arma_accumulate(k, [&](size_t i) { return std::fabs(col[srt[i]]); });
    ws[j] = s - std::fabs(col[srt[j]]);
  }
  wd.resize(k);
  for (size_t c = 0; c < k; ++c) wd[c] = ws[rank[c]];
}

double average_edge_weight(const std::vector<double>& wd) {  // src/netStats.cpp:154-162
  const uint32_t k = (uint32_t)wd.size();
  const double pairs = (double)(uint32_t)(k * k - k);
  return arma_accumulate(wd.size(), [&](size_t i) { return wd[i]; }) / pairs;
}

double pearson(const double* a, const double* b, size_t n) {
  if (n == 0) return kNaN;
  double ma = 0.0, mb = 0.0;
  for (size_t i = 0; i < n; ++i) { ma += a[i]; mb += b[i]; }
  ma /= (double)n;
  mb /= (double)n;
  double sab = 0.0, saa = 0.0, sbb = 0.0;
  for (size_t i = 0; i < n; ++i) {
    const double da = a[i] - ma, db = b[i] - mb;
    sab += da * db;
    saa += da * da;
    sbb += db * db;
  }
  return sab / std::sqrt(saa * sbb);
}

// Correlation src/netStats.cpp:69-83 (complete cases)
double correlation(const double* x, const std::vector<double>& y) {
  std::vector<double> a, b;
  a.reserve(y.size());
  b.reserve(y.size());
  for (size_t i = 0; i < y.size(); ++i)
    if (std::isfinite(x[i]) && std::isfinite(y[i])) { a.push_back(x[i]); b.push_back(y[i]); }
  if (a.empty()) return kNaN;
  return pearson(a.data(), b.data(), a.size());
}

// SignAwareMean src/netStats.cpp:95-109
double sign_aware_mean(const double* x, const std::vector<double>& y) {
  double s = 0.0;
  size_t n = 0;
  for (size_t i = 0; i < y.size(); ++i)
    if (std::isfinite(x[i]) && std::isfinite(y[i])) {
      s += (x[i] > 0 ? 1.0 : (x[i] < 0 ? -1.0 : 0.0)) * y[i];
      ++n;
    }
  return n ? s / (double)n : kNaN;
}

// SummaryProfile src/netStats.cpp:217-250 + NodeContribution :265-280 (sorted
// order), returning NC in module node order.
void profile(const double* data, int64_t S, const std::vector<int64_t>& srt, const std::vector<size_t>& rank,
             std::vector<double>& nc) {
  const int m = (int)S, n = (int)srt.size();
  std::vector<double> x((size_t)m * n);
  bool finite = true;
  for (int j = 0; j < n; ++j) {
    std::memcpy(&x[(size_t)j * m], data + srt[j] * S, sizeof(double) * m);
    for (int i = 0; i < m; ++i) finite &= std::isfinite(x[(size_t)j * m + i]);
  }
  nc.assign(n, kNaN);
  if (!finite) return;  // svd_econ fails on non-finite input -> NaN summary
  std::vector<double> a = x;
  const int mn = std::min(m, n);
  std::vector<double> s(mn), u((size_t)m * mn);
  double vt_dummy = 0.0;
  const int ldvt = 1;
  int lwork = -1, info = 0;
  double wq = 0.0;
  const char jobu = 'S', jobvt = 'N';  // auxlib::svd_econ(U, S, V, A, 'l')
  g_dgesvd(&jobu, &jobvt, &m, &n, a.data(), &m, s.data(), u.data(), &m, &vt_dummy, &ldvt, &wq, &lwork, &info);
  lwork = (int)wq + 1;
  std::vector<double> work(lwork);
  g_dgesvd(&jobu, &jobvt, &m, &n, a.data(), &m, s.data(), u.data(), &m, &vt_dummy, &ldvt, work.data(), &lwork,
           &info);
  if (info != 0) return;
  std::vector<double> sp(u.begin(), u.begin() + m);
  std::vector<double> mo(m, 0.0);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) mo[i] += x[(size_t)j * m + i];
  for (int i = 0; i < m; ++i) mo[i] /= (double)n;
  const double c = pearson(mo.data(), sp.data(), m);
  if (std::isfinite(c) && c < 0) for (double& v : sp) v = -v;
  std::vector<double> ncs(n);
  for (int j = 0; j < n; ++j) ncs[j] = pearson(&x[(size_t)j * m], sp.data(), m);
  for (int c2 = 0; c2 < n; ++c2) nc[c2] = ncs[rank[c2]];
}

double coherence(const std::vector<double>& nc) {  // src/netStats.cpp:293-305
  double s = 0.0;
  size_t n = 0;
  for (double v : nc)
    if (std::isfinite(v)) { s += v * v; ++n; }
  return n ? s / (double)n : kNaN;
}

struct Problem {
  const double *data, *corr, *net;
  int64_t N, S;
  int32_t n_rows, n_present;
  const int32_t *row_of, *test_idx, *null_pos, *null_idx;
  const int64_t* node_off;
  int64_t n_null;
  const double *disc_cv, *disc_wd, *disc_nc;
  int n_stat;
  std::vector<int64_t> cv_off;
};

// Body of calculateNulls for one module (src/permutations.cpp:71-101)
void module_stats(const Problem& P, int m, const std::vector<int64_t>& idx, double* out, int64_t stride) {
  std::vector<double> tcv, twd, tnc;
  corr_vector(P.corr, P.N, idx, tcv);
  std::vector<int64_t> srt;
  std::vector<size_t> rank;
  sort_nodes(idx, srt, rank);
  weighted_degree(P.net, P.N, srt, rank, twd);
  const double* dcv = P.disc_cv + P.cv_off[m];
  const double* dwd = P.disc_wd + P.node_off[m];
  if (!P.data) {
    out[0 * stride] = average_edge_weight(twd);
    out[1 * stride] = correlation(dcv, tcv);
    out[2 * stride] = correlation(dwd, twd);
    out[3 * stride] = sign_aware_mean(dcv, tcv);
    return;
  }
  profile(P.data, P.S, srt, rank, tnc);
  const double* dnc = P.disc_nc + P.node_off[m];
  out[0 * stride] = average_edge_weight(twd);
  out[1 * stride] = coherence(tnc);
  out[2 * stride] = correlation(dcv, tcv);
  out[3 * stride] = correlation(dwd, twd);
  out[4 * stride] = correlation(dnc, tnc);
  out[5 * stride] = sign_aware_mean(dcv, tcv);
  out[6 * stride] = sign_aware_mean(dnc, tnc);
}

}  // namespace

extern "C" {

const char* ref_last_error() { return g_err.c_str(); }

int ref_init_lapack(const char* so_path) {
  void* h = dlopen(so_path, RTLD_NOW | RTLD_LOCAL);
  if (!h) { g_err = dlerror(); return 1; }
  g_dgesvd = (dgesvd_t)dlsym(h, "scipy_dgesvd_");
  if (!g_dgesvd) g_dgesvd = (dgesvd_t)dlsym(h, "dgesvd_");
  if (!g_dgesvd) { g_err = "no dgesvd symbol"; return 1; }
  typedef void (*setthreads_t)(int);
  setthreads_t st = (setthreads_t)dlsym(h, "scipy_openblas_set_num_threads");
  if (st) st(1);  // BLAS threads forced to 1 (R/modulePreservation.R:433-437)
  return 0;
}

// PermutationProcedure[NoData] on resolved index sets. nulls: n_rows x n_stat x n_perm
// (cube layout), observed: n_rows x n_stat. pi == NULL: per-thread Fisher-Yates shuffles
// seeded from `seed` (the reference's arma::shuffle); else explicit [n_perm x n_null].
int ref_permutation_procedure(const double* data, const double* corr, const double* net, int64_t N,
                              int64_t S, int32_t n_rows, int32_t n_present, const int32_t* row_of,
                              const int64_t* node_off, const int32_t* test_idx, const int32_t* null_pos,
                              const int32_t* null_idx, int64_t n_null, const double* disc_cv,
                              const double* disc_wd, const double* disc_nc, int64_t n_perm, uint64_t seed,
                              const uint32_t* pi, int n_threads, double* nulls, double* observed) {
  if (data && !g_dgesvd) { g_err = "LAPACK not initialised"; return 1; }
  Problem P{data, corr, net, N, S, n_rows, n_present, row_of, test_idx, null_pos, null_idx, node_off,
            n_null, disc_cv, disc_wd, disc_nc, data ? 7 : 4, {}};
  P.cv_off.assign(n_present + 1, 0);
  for (int m = 0; m < n_present; ++m) {
    const int64_t k = node_off[m + 1] - node_off[m];
    P.cv_off[m + 1] = P.cv_off[m] + k * (k - 1) / 2;
  }
  const double na = na_real();
  const int64_t slice = (int64_t)n_rows * P.n_stat;
  n_threads = std::max(1, n_threads);
  // Independent (permutation, module) items over threads: used for the
  // observed statistics and, with explicit shuffles and fewer permutations
  // than threads, for the nulls (checker mode; results are per item, so the
  // split does not change them).
  auto run_items = [&](int64_t n_items, const std::function<void(int64_t)>& item) {
    std::atomic<int64_t> next{0};
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t)
      th.emplace_back([&]() {
        for (int64_t i = next++; i < n_items; i = next++) item(i);
      });
    for (auto& x : th) x.join();
  };
  if (observed) {
    std::fill(observed, observed + slice, na);
    run_items(n_present, [&](int64_t m) {
      std::vector<int64_t> idx(test_idx + node_off[m], test_idx + node_off[m + 1]);
      module_stats(P, (int)m, idx, observed + row_of[m], n_rows);
    });
    for (int64_t i = 0; i < slice; ++i) if (!std::isfinite(observed[i])) observed[i] = na;
  }
  if (n_perm <= 0 || !nulls) return 0;
  std::fill(nulls, nulls + slice * n_perm, na);
  if (pi && n_perm < n_threads) {
    run_items(n_perm * n_present, [&](int64_t it) {
      const int64_t p = it / n_present;
      const int m = (int)(it % n_present);
      std::vector<int64_t> idx;
      for (int64_t c = node_off[m]; c < node_off[m + 1]; ++c) idx.push_back(null_idx[pi[p * n_null + null_pos[c]]]);
      module_stats(P, m, idx, nulls + p * slice + row_of[m], n_rows);
    });
    for (int64_t i = 0; i < slice * n_perm; ++i) if (!std::isfinite(nulls[i])) nulls[i] = na;
    return 0;
  }
  // contiguous chunks, remainder to the first threads (src/permutations.cpp:338-354)
  std::vector<int64_t> start(n_threads + 1, 0);
  for (int t = 0; t < n_threads; ++t)
    start[t + 1] = start[t] + n_perm / n_threads + (t < n_perm % n_threads ? 1 : 0);
  auto worker = [&](int t) {
    std::vector<int32_t> pool(null_idx, null_idx + n_null);
    std::mt19937_64 rng(seed + 0x9E3779B97F4A7C15ull * (uint64_t)(t + 1));
    std::vector<int64_t> idx;
    for (int64_t p = start[t]; p < start[t + 1]; ++p) {
      if (!pi) std::shuffle(pool.begin(), pool.end(), rng);  // arma::shuffle (:63)
      for (int m = 0; m < n_present; ++m) {
        idx.clear();
        for (int64_t c = node_off[m]; c < node_off[m + 1]; ++c) {
          const int64_t q = null_pos[c];
          idx.push_back(pi ? null_idx[pi[p * n_null + q]] : pool[q]);
        }
        module_stats(P, m, idx, nulls + p * slice + row_of[m], n_rows);
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < n_threads; ++t) th.emplace_back(worker, t);
  for (auto& x : th) x.join();
  for (int64_t i = 0; i < slice * n_perm; ++i) if (!std::isfinite(nulls[i])) nulls[i] = na;
  return 0;
}

}  // extern "C"
