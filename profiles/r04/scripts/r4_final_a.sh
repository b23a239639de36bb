# Round 4 final tree: the whole -m gpu suite, then the C3 and C2 PMC passes
# (profiles/r04/scripts/r4_pmc_a.sh) on the same build.
set -o pipefail
D=gpurun_out/${1:-r4finA}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $D/pytest.log 2>&1 && \
bash profiles/r04/scripts/r4_pmc_a.sh r4finA_pmc
