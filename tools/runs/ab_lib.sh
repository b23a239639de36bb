# A/B: the in-tree library vs netrep_amd/_lib/libnetrep_amd_prev.so, then GPU tests on the new one
set -o pipefail
D=gpurun_out/${1:-ab}; mkdir -p $D
B="python -u bench.py --steps 10 --no-secondary --no-cpu-baseline"
timeout -k 10 200 $B > $D/new.json 2> $D/new.err && \
NETREP_LIB=$PWD/netrep_amd/_lib/libnetrep_amd_prev.so timeout -k 10 200 $B > $D/prev.json 2> $D/prev.err && \
timeout -k 10 200 $B > $D/new2.json 2> $D/new2.err && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1
