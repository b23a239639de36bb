# Round 4, first GPU check: the whole -m gpu suite (shape-only Gram-table
# rule, residency, mesh broadcast, C3 two-context bitwise test) and a short
# default bench line.
set -o pipefail
D=gpurun_out/${1:-r4c1}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > $D/bench.json 2> $D/bench.err
