"""The Rcpp glue under rcpp/ (drop-in replacements of NetRep's hot-path
sources) exports exactly the eight routines of the reference's CallEntries
(src/RcppExports.cpp:131-146) with their arities, and calls only functions the
C ABI header declares. (No R in this image: the glue is checked here, not
compiled; tests/abi_driver is the compiled C-ABI caller.)"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RCPP = os.path.join(ROOT, "rcpp")

# src/RcppExports.cpp:131-146 (name -> .Call arity)
CALL_ENTRIES = {
    "PermutationProcedure": 11, "PermutationProcedureNoData": 10,
    "IntermediateProperties": 6, "IntermediatePropertiesNoData": 5,
    "NetProps": 4, "NetPropsNoData": 3, "Scale": 1, "CheckFinite": 1,
}
# the reference source file each routine lives in
FILES = {
    "PermutationProcedure": "permutations.cpp", "PermutationProcedureNoData": "permutationsNoData.cpp",
    "IntermediateProperties": "discProps.cpp", "IntermediatePropertiesNoData": "discProps.cpp",
    "NetProps": "properties.cpp", "NetPropsNoData": "properties.cpp", "Scale": "scale.cpp",
    "CheckFinite": "checkFinite.cpp",
}


def exported(path):
    src = open(path).read()
    out = {}
    for m in re.finditer(r"//\s*\[\[Rcpp::export\]\]\s*\n\s*[\w:<>]+\s+(\w+)\s*\((.*?)\)\s*\{", src, re.S):
        args = [a for a in m.group(2).split(",") if a.strip()]
        out[m.group(1)] = len(args)
    return out


def test_every_call_entry_is_replaced_with_its_arity():
    found = {}
    for fn in sorted(os.listdir(RCPP)):
        if fn.endswith(".cpp"):
            for name, ar in exported(os.path.join(RCPP, fn)).items():
                found[name] = (ar, fn)
    for name, ar in CALL_ENTRIES.items():
        assert name in found, name
        assert found[name] == (ar, FILES[name]), (name, found[name])


def test_glue_calls_only_declared_abi_functions():
    hdr = open(os.path.join(ROOT, "include", "netrep_gpu.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    declared = set(re.findall(r"\b((?:nr|netrep)_[A-Za-z0-9_]+)\s*\(", hdr))
    used = set()
    for fn in os.listdir(RCPP):
        if fn.endswith((".cpp", ".h")):
            used |= set(re.findall(r"\b((?:nr|netrep)_[A-Za-z0-9_]+)\s*\(", open(os.path.join(RCPP, fn)).read()))
    assert used and used <= declared, used - declared


def test_makevars_links_the_engine_not_lapack():
    mk = open(os.path.join(RCPP, "Makevars")).read()
    assert "-lnetrep_amd" in mk and "LAPACK_LIBS" not in mk.split("PKG_LIBS", 1)[1]
