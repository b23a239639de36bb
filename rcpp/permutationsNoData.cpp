// Drop-in replacement of NetRep's src/permutationsNoData.cpp
// (PermutationProcedureNoData, src/permutationsNoData.cpp:140-375): the
// network-only path, the same engine entry with tData = NULL. Same signature,
// same R value with the four statistics of :156-158.
#include "netrep_glue.h"

using netrep_glue::check;

// [[Rcpp::export]]
Rcpp::List PermutationProcedureNoData(Rcpp::List discProps, Rcpp::NumericMatrix tCorr, Rcpp::NumericMatrix tNet,
                                      Rcpp::CharacterVector moduleAssignments, Rcpp::CharacterVector modules,
                                      Rcpp::IntegerVector nPermutations, Rcpp::IntegerVector nCores,
                                      Rcpp::CharacterVector nullHypothesis, Rcpp::LogicalVector verbose,
                                      Rcpp::Function vCat) {
  const std::vector<std::string> tNames = Rcpp::as<std::vector<std::string>>(Rcpp::colnames(tNet));
  const std::vector<std::string> mods = Rcpp::as<std::vector<std::string>>(modules);
  const auto tn = netrep_glue::cstrs(tNames), mn = netrep_glue::cstrs(mods);
  const netrep_glue::Assignments ma(moduleAssignments);
  netrep_glue::DiscProps dp(discProps, mods, /*with_data=*/false);

  const int nPerm = nPermutations[0];
  const int M = (int)mods.size();
  Rcpp::NumericMatrix observed(M, NR_NSTAT_NODATA);
  Rcpp::NumericVector nulls(nPerm > 0 ? (R_xlen_t)M * NR_NSTAT_NODATA * nPerm : 0);
  vCat(verbose, 1, "Calculating observed test statistics...");
  if (nPerm > 0) vCat(verbose, 1, "Generating null distributions from", nPerm, "permutations on the GPU...");
  int rc;
  {
    const netrep_glue::Hooks hooks;
    rc = netrep_PermutationProcedure(&dp.dp, /*t_data=*/nullptr, tCorr.begin(), tNet.begin(), /*n_samples=*/0,
                                     tNet.ncol(), tn.data(), ma.n.data(), ma.l.data(), (int64_t)ma.n.size(),
                                     mn.data(), (int64_t)M, nPerm, nCores[0],
                                     Rcpp::as<std::string>(nullHypothesis[0]).c_str(), verbose[0],
                                     netrep_glue::draw_seed(), /*pi=*/nullptr,
                                     nPerm > 0 ? nulls.begin() : nullptr, observed.begin());
  }
  if (rc != NR_ERR_CANCELLED) check(rc);
  Rcpp::CharacterVector statnames = {"avg.weight", "cor.cor", "cor.degree", "avg.cor"};
  return netrep_glue::permutation_result(nulls, observed, modules, statnames, nPerm);
}
