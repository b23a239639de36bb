// Drop-in replacement of NetRep's src/properties.cpp (NetProps, :41-156, and
// NetPropsNoData, :190-273): networkProperties' per-module statistics on the
// MI355X engine (netrep_NetProps scales the data on the device, as NetProps
// scales it first, :49). Same signatures; the R value is one named list per
// module, with NA for nodes absent from the dataset (:84-91, :130-139).
#include "netrep_glue.h"

using netrep_glue::check;

namespace {

Rcpp::List netprops(Rcpp::NumericMatrix* data, Rcpp::NumericMatrix net, Rcpp::CharacterVector moduleAssignments,
                    Rcpp::CharacterVector modules) {
  const bool with_data = data != nullptr;
  const std::vector<std::string> nodeNames = Rcpp::as<std::vector<std::string>>(Rcpp::colnames(net));
  const std::vector<std::string> mods = Rcpp::as<std::vector<std::string>>(modules);
  const auto nn = netrep_glue::cstrs(nodeNames), mn = netrep_glue::cstrs(mods);
  const netrep_glue::Assignments ma(moduleAssignments);
  const int64_t S = with_data ? data->nrow() : 0;
  const size_t M = mods.size();
  std::vector<std::vector<std::string>> modNodes(M);
  int64_t tot = 0;
  for (size_t i = 0; i < M; ++i) {
    modNodes[i] = netrep_glue::module_node_names(ma, mods[i]);
    tot += (int64_t)modNodes[i].size();
  }
  std::vector<double> deg((size_t)std::max<int64_t>(tot, 1)), aw(std::max<size_t>(M, 1));
  std::vector<double> nc(with_data ? deg.size() : 0), sp(with_data ? std::max<size_t>(M * S, 1) : 0);
  std::vector<double> coh(with_data ? aw.size() : 0);
  std::vector<int64_t> k_all(std::max<size_t>(M, 1), 0);
  check(netrep_NetProps(with_data ? data->begin() : nullptr, net.begin(), S, net.ncol(), nn.data(), ma.n.data(),
                        ma.l.data(), (int64_t)ma.n.size(), mn.data(), (int64_t)M, deg.data(),
                        with_data ? nc.data() : nullptr, with_data ? sp.data() : nullptr,
                        with_data ? coh.data() : nullptr, aw.data(), k_all.data()));
  Rcpp::CharacterVector sampleNames;
  if (with_data) sampleNames = Rcpp::rownames(*data);
  Rcpp::List results;
  int64_t o = 0;
  for (size_t i = 0; i < M; ++i) {
    const int64_t k = k_all[i];
    Rcpp::CharacterVector names = Rcpp::wrap(modNodes[i]);
    Rcpp::NumericVector degree(deg.begin() + o, deg.begin() + o + k);
    degree.names() = names;
    if (with_data) {
      Rcpp::NumericVector contribution(nc.begin() + o, nc.begin() + o + k);
      contribution.names() = names;
      Rcpp::NumericVector summary(sp.begin() + (R_xlen_t)i * S, sp.begin() + (R_xlen_t)(i + 1) * S);
      summary.names() = sampleNames;
      results.push_back(Rcpp::List::create(Rcpp::Named("summary") = summary,
                                           Rcpp::Named("contribution") = contribution,
                                           Rcpp::Named("coherence") = coh[i], Rcpp::Named("degree") = degree,
                                           Rcpp::Named("avgWeight") = aw[i]));
    } else {
      results.push_back(Rcpp::List::create(Rcpp::Named("degree") = degree, Rcpp::Named("avgWeight") = aw[i]));
    }
    o += k;
  }
  results.names() = modules;
  return results;
}

}  // namespace

// data is unscaled (NetProps scales it, src/properties.cpp:49)
// [[Rcpp::export]]
Rcpp::List NetProps(Rcpp::NumericMatrix data, Rcpp::NumericMatrix net, Rcpp::CharacterVector moduleAssignments,
                    Rcpp::CharacterVector modules) {
  return netprops(&data, net, moduleAssignments, modules);
}

// [[Rcpp::export]]
Rcpp::List NetPropsNoData(Rcpp::NumericMatrix net, Rcpp::CharacterVector moduleAssignments,
                          Rcpp::CharacterVector modules) {
  return netprops(nullptr, net, moduleAssignments, modules);
}
