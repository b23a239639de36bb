// Drop-in replacement of NetRep's src/discProps.cpp (IntermediateProperties,
// :44-132, and IntermediatePropertiesNoData, :171-244): the discovery
// vectors (CorrVector, weighted degree, node contribution) of every module
// with nodes in the test dataset, computed on the MI355X engine
// (netrep_IntermediateProperties). Same signatures; the R value is the named
// lists over the modules present, as the reference returns.
#include <unordered_set>

#include "netrep_glue.h"

using netrep_glue::check;

namespace {

Rcpp::List intermediate(const double* dData, int64_t nSamples, Rcpp::NumericMatrix dCorr, Rcpp::NumericMatrix dNet,
                        Rcpp::CharacterVector tNodeNames, Rcpp::CharacterVector moduleAssignments,
                        Rcpp::CharacterVector modules) {
  const bool with_data = dData != nullptr;
  const std::vector<std::string> dNames = Rcpp::as<std::vector<std::string>>(Rcpp::colnames(dNet));
  const std::vector<std::string> tNames = Rcpp::as<std::vector<std::string>>(tNodeNames);
  const std::vector<std::string> mods = Rcpp::as<std::vector<std::string>>(modules);
  const auto dn = netrep_glue::cstrs(dNames), tn = netrep_glue::cstrs(tNames), mn = netrep_glue::cstrs(mods);
  const netrep_glue::Assignments ma(moduleAssignments);
  // output sizes: the module nodes present in the test list (MakeModMap over
  // tIdxMap, src/discProps.cpp:64-67)
  const std::unordered_set<std::string> tset(tNames.begin(), tNames.end());
  int64_t sum_k = 0, sum_cv = 0;
  for (const std::string& m : mods) {
    int64_t k = 0;
    for (size_t i = 0; i < ma.labels.size(); ++i) k += ma.labels[i] == m && tset.count(ma.names[i]);
    sum_k += k;
    sum_cv += k * (k - 1) / 2;
  }
  const size_t M = mods.size();
  std::vector<double> deg((size_t)std::max<int64_t>(sum_k, 1)), cv((size_t)std::max<int64_t>(sum_cv, 1));
  std::vector<double> nc(with_data ? deg.size() : 0);
  std::vector<int64_t> deg_len(M, 0), cv_len(M, 0), nc_len(M, 0);
  check(netrep_IntermediateProperties(dData, dCorr.begin(), dNet.begin(), nSamples, dNet.ncol(), dn.data(), tn.data(),
                                      (int64_t)tn.size(), ma.n.data(), ma.l.data(), (int64_t)ma.n.size(), mn.data(),
                                      (int64_t)M, deg.data(), deg_len.data(), cv.data(), cv_len.data(),
                                      with_data ? nc.data() : nullptr, with_data ? nc_len.data() : nullptr));
  // split into the named lists; a length of 0 = a module absent from the
  // test dataset, which the reference skips (src/discProps.cpp:72-78)
  Rcpp::List degree, corr, contribution;
  std::vector<std::string> present;
  int64_t od = 0, oc = 0;
  for (size_t i = 0; i < M; ++i) {
    if (deg_len[i] == 0) continue;
    present.push_back(mods[i]);
    degree.push_back(Rcpp::NumericVector(deg.begin() + od, deg.begin() + od + deg_len[i]));
    corr.push_back(Rcpp::NumericVector(cv.begin() + oc, cv.begin() + oc + cv_len[i]));
    if (with_data) contribution.push_back(Rcpp::NumericVector(nc.begin() + od, nc.begin() + od + nc_len[i]));
    od += deg_len[i];
    oc += cv_len[i];
  }
  Rcpp::CharacterVector pn = Rcpp::wrap(present);
  degree.names() = pn;
  corr.names() = pn;
  if (!with_data) return Rcpp::List::create(Rcpp::Named("degree") = degree, Rcpp::Named("corr") = corr);
  contribution.names() = pn;
  return Rcpp::List::create(Rcpp::Named("degree") = degree, Rcpp::Named("corr") = corr,
                            Rcpp::Named("contribution") = contribution);
}

}  // namespace

// dData is scaled by the caller (R/modulePreservation.R:567 passes Scale()d data).
// [[Rcpp::export]]
Rcpp::List IntermediateProperties(Rcpp::NumericMatrix dData, Rcpp::NumericMatrix dCorr, Rcpp::NumericMatrix dNet,
                                  Rcpp::CharacterVector tNodeNames, Rcpp::CharacterVector moduleAssignments,
                                  Rcpp::CharacterVector modules) {
  return intermediate(dData.begin(), dData.nrow(), dCorr, dNet, tNodeNames, moduleAssignments, modules);
}

// [[Rcpp::export]]
Rcpp::List IntermediatePropertiesNoData(Rcpp::NumericMatrix dCorr, Rcpp::NumericMatrix dNet,
                                        Rcpp::CharacterVector tNodeNames, Rcpp::CharacterVector moduleAssignments,
                                        Rcpp::CharacterVector modules) {
  return intermediate(nullptr, 0, dCorr, dNet, tNodeNames, moduleAssignments, modules);
}
