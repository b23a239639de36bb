// Routines the MI355X engine adds beside the eight reference entry points
// (optional; `Rcpp::compileAttributes()` registers them next to the others in
// src/RcppExports.cpp): releasing the datasets kept resident between calls,
// and uploading the next test dataset while the current one's permutations run.
#include "netrep_glue.h"

// on.exit(ReleaseResident()) in modulePreservation() / networkProperties():
// the discovery dataset of IntermediateProperties, NetProps' dataset,
// pending prefetches and pooled contexts leave HBM.
// [[Rcpp::export]]
void ReleaseResident() { netrep_ReleaseResident(); }

// Upload test dataset tt + 1 before PermutationProcedure runs dataset tt
// (R/modulePreservation.R:553-620); the call that names the same three
// matrices adopts it. The matrices must stay referenced until then.
// [[Rcpp::export]]
void PrefetchTestDataset(Rcpp::NumericMatrix tData, Rcpp::NumericMatrix tCorr, Rcpp::NumericMatrix tNet) {
  netrep_glue::check(
      netrep_PrefetchTestDataset(tData.begin(), tCorr.begin(), tNet.begin(), tData.nrow(), tNet.ncol()));
}

// [[Rcpp::export]]
void DiscardPrefetch() { netrep_DiscardPrefetch(); }
