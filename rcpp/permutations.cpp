// Drop-in replacement of NetRep's src/permutations.cpp (PermutationProcedure,
// src/permutations.cpp:160-409): the std::thread pool of calculateNulls
// (:39-105, :335-380) becomes batched dispatch on the MI355X engine through
// netrep_PermutationProcedure (include/netrep_gpu.h). Same signature, same R
// value: list(nulls = M x 7 x nPerm with dimnames, observed = M x 7).
#include "netrep_glue.h"

using netrep_glue::check;

// [[Rcpp::export]]
Rcpp::List PermutationProcedure(Rcpp::List discProps, Rcpp::NumericMatrix tData, Rcpp::NumericMatrix tCorr,
                                Rcpp::NumericMatrix tNet, Rcpp::CharacterVector moduleAssignments,
                                Rcpp::CharacterVector modules, Rcpp::IntegerVector nPermutations,
                                Rcpp::IntegerVector nCores, Rcpp::CharacterVector nullHypothesis,
                                Rcpp::LogicalVector verbose, Rcpp::Function vCat) {
  const std::vector<std::string> tNames = Rcpp::as<std::vector<std::string>>(Rcpp::colnames(tNet));
  const std::vector<std::string> mods = Rcpp::as<std::vector<std::string>>(modules);
  const auto tn = netrep_glue::cstrs(tNames), mn = netrep_glue::cstrs(mods);
  const netrep_glue::Assignments ma(moduleAssignments);
  netrep_glue::DiscProps dp(discProps, mods, /*with_data=*/true);

  const int nPerm = nPermutations[0];
  const int M = (int)mods.size();
  Rcpp::NumericMatrix observed(M, NR_NSTAT_DATA);
  Rcpp::NumericVector nulls(nPerm > 0 ? (R_xlen_t)M * NR_NSTAT_DATA * nPerm : 0);
  vCat(verbose, 1, "Calculating observed test statistics...");
  if (nPerm > 0) vCat(verbose, 1, "Generating null distributions from", nPerm, "permutations on the GPU...");
  int rc;
  {
    const netrep_glue::Hooks hooks;  // interrupt polling + "% completed." on this thread
    rc = netrep_PermutationProcedure(&dp.dp, tData.begin(), tCorr.begin(), tNet.begin(), tData.nrow(),
                                     tData.ncol(), tn.data(), ma.n.data(), ma.l.data(), (int64_t)ma.n.size(),
                                     mn.data(), (int64_t)M, nPerm, nCores[0],
                                     Rcpp::as<std::string>(nullHypothesis[0]).c_str(), verbose[0],
                                     netrep_glue::draw_seed(), /*pi=*/nullptr,
                                     nPerm > 0 ? nulls.begin() : nullptr, observed.begin());
  }
  // NR_ERR_CANCELLED (Ctrl-C): like the reference, return the partial cube
  // (un-run permutations NA, src/permutations.cpp:375-408); R raises the
  // pending interrupt at its next check.
  if (rc != NR_ERR_CANCELLED) check(rc);
  Rcpp::CharacterVector statnames = {"avg.weight", "coherence", "cor.cor", "cor.degree",
                                     "cor.contrib", "avg.cor", "avg.contrib"};
  return netrep_glue::permutation_result(nulls, observed, modules, statnames, nPerm);
}
