// Drop-in replacement of NetRep's src/checkFinite.cpp (CheckFinite, :21-28):
// one device pass over the matrix (finite_kernel); on any NA/NaN/Inf the
// engine returns NR_ERR_NONFINITE with the reference's message, "matrices
// cannot have non-finite or missing values" (:25-27), raised as an R error.
#include "netrep_glue.h"

// [[Rcpp::export]]
void CheckFinite(Rcpp::NumericMatrix matPtr) {
  netrep_glue::check(netrep_CheckFinite(matPtr.begin(), matPtr.nrow(), matPtr.ncol()));
}
