// Shared helpers of the Rcpp glue that replaces NetRep's hot-path sources
// (src/permutations.cpp, permutationsNoData.cpp, discProps.cpp,
// properties.cpp, scale.cpp, checkFinite.cpp) with calls into the MI355X
// engine's C ABI (include/netrep_gpu.h). Drop-in: the exported names,
// arguments and return shapes are those of the reference's Rcpp functions,
// registered unchanged by src/RcppExports.cpp:131-146.
#pragma once
#include <Rcpp.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "netrep_gpu.h"

namespace netrep_glue {

// R strings -> C strings whose storage lives in `keep`.
inline std::vector<const char*> cstrs(const std::vector<std::string>& keep) {
  std::vector<const char*> p;
  p.reserve(keep.size());
  for (const std::string& s : keep) p.push_back(s.c_str());
  return p;
}

// An engine error becomes an R error (BEGIN_RCPP / END_RCPP in
// src/RcppExports.cpp turn the exception into stop()).
inline void check(int rc) {
  if (rc != NR_OK) Rcpp::stop(netrep_last_error());
}

// checkInterrupt (src/interrupt.cpp:4-11): R_CheckUserInterrupt inside a
// top-level context, so an interrupt never longjmps through the engine.
inline void chk_int(void*) { R_CheckUserInterrupt(); }
inline int interrupt_hook(void*) { return R_ToplevelExec(chk_int, NULL) == FALSE; }

// MonitorProgress's console output (src/thread-utils.cpp:54-81), called by
// the library on this (R's) thread, so Rcpp::Rcout is safe here.
inline void progress_hook(int32_t event, int64_t done, int64_t total, void*) {
  if (event == NETREP_PROGRESS_BEGIN) {
    Rcpp::Rcout << std::endl;
  } else if (event == NETREP_PROGRESS_UPDATE) {
    char line[32];
    if (netrep_format_progress(done, total, line, sizeof(line)) > 0) Rcpp::Rcout << line;
  } else {
    Rcpp::Rcout << std::endl << std::endl;
  }
}

// Both hooks installed for the duration of one call.
struct Hooks {
  Hooks() {
    netrep_set_interrupt_hook(interrupt_hook, nullptr);
    netrep_set_progress_hook(progress_hook, nullptr);
  }
  ~Hooks() {
    netrep_set_interrupt_hook(nullptr, nullptr);
    netrep_set_progress_hook(nullptr, nullptr);
  }
};

// names(moduleAssignments) and its labels.
struct Assignments {
  std::vector<std::string> names, labels;
  std::vector<const char*> n, l;
  explicit Assignments(Rcpp::CharacterVector ma)
      : names(Rcpp::as<std::vector<std::string>>(ma.names())), labels(Rcpp::as<std::vector<std::string>>(ma)) {
    n = cstrs(names);
    l = cstrs(labels);
  }
};

// discProps (src/discProps.cpp:127-131): named lists over the modules present
// in the test dataset; the engine wants one pointer per requested module
// (NULL where absent).
struct DiscProps {
  std::vector<const double*> wd, cv, nc;
  std::vector<int64_t> wdl, cvl, ncl;
  netrep_disc_props dp;
  DiscProps(Rcpp::List discProps, const std::vector<std::string>& mods, bool with_data)
      : wd(mods.size(), nullptr), cv(mods.size(), nullptr), nc(mods.size(), nullptr),
        wdl(mods.size(), 0), cvl(mods.size(), 0), ncl(mods.size(), 0) {
    Rcpp::List lWD = discProps["degree"], lCV = discProps["corr"];
    Rcpp::List lNC = with_data ? Rcpp::List(discProps["contribution"]) : Rcpp::List();
    Rcpp::CharacterVector present = lWD.names();
    for (size_t i = 0; i < mods.size(); ++i) {
      if (std::find(present.begin(), present.end(), mods[i]) == present.end()) continue;
      Rcpp::NumericVector a = lWD[mods[i]], b = lCV[mods[i]];
      wd[i] = a.begin();
      wdl[i] = a.size();
      cv[i] = b.begin();
      cvl[i] = b.size();
      if (with_data) {
        Rcpp::NumericVector c = lNC[mods[i]];
        nc[i] = c.begin();
        ncl[i] = c.size();
      }
    }
    dp = {wd.data(), wdl.data(), cv.data(), cvl.data(), with_data ? nc.data() : nullptr,
          with_data ? ncl.data() : nullptr};
  }
};

// One seed per call from R's RNG (inside Rcpp's RNGScope,
// src/RcppExports.cpp:14), so set.seed() makes a run reproducible. Scaled
// BEFORE the cast: (uint64_t)unif_rand() alone is always 0.
inline uint64_t draw_seed() { return (uint64_t)(R::unif_rand() * 9007199254740992.0); }

// The permutation procedure's R value (src/permutations.cpp:387-408 and
// src/permutationsNoData.cpp:355-375): nulls M x S x P with dimnames
// (modules, statnames, "permutation.i"), observed M x S.
inline Rcpp::List permutation_result(Rcpp::NumericVector nulls, Rcpp::NumericMatrix observed,
                                     Rcpp::CharacterVector modules, Rcpp::CharacterVector statnames, int nPerm) {
  const int M = modules.size(), S = statnames.size();
  Rcpp::colnames(observed) = statnames;
  Rcpp::rownames(observed) = modules;
  if (nPerm == 0) return Rcpp::List::create(Rcpp::Named("observed") = observed);
  Rcpp::CharacterVector permNames(nPerm);
  for (int i = 0; i < nPerm; ++i) permNames[i] = "permutation." + std::to_string(i + 1);
  nulls.attr("dim") = Rcpp::IntegerVector::create(M, S, nPerm);
  nulls.attr("dimnames") = Rcpp::List::create(modules, statnames, permNames);
  return Rcpp::List::create(Rcpp::Named("nulls") = nulls, Rcpp::Named("observed") = observed);
}

// Module node names in moduleAssignments order (GetModNodeNames,
// src/utils.cpp:212-227): the names of NetProps' per-node vectors.
inline std::vector<std::string> module_node_names(const Assignments& a, const std::string& mod) {
  std::vector<std::string> out;
  for (size_t i = 0; i < a.labels.size(); ++i)
    if (a.labels[i] == mod) out.push_back(a.names[i]);
  return out;
}

}  // namespace netrep_glue
