// Drop-in replacement of NetRep's src/scale.cpp (Scale, :38-45): per column
// (x - mean) / sd with the n - 1 normalisation (:21), on the MI355X engine
// (netrep_Scale, scale_kernel). Same signature; the dimnames are kept as the
// reference keeps them (:42-43).
#include "netrep_glue.h"

// [[Rcpp::export]]
Rcpp::NumericMatrix Scale(Rcpp::NumericMatrix data) {
  Rcpp::NumericMatrix out(data.nrow(), data.ncol());
  netrep_glue::check(netrep_Scale(data.begin(), data.nrow(), data.ncol(), out.begin()));
  Rcpp::colnames(out) = Rcpp::colnames(data);
  Rcpp::rownames(out) = Rcpp::rownames(data);
  return out;
}
