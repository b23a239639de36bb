# Round 5: LDS-only barriers in the packed kernels' Lanczos steps (no wait for the basis
# stores): tests, C3 / C2-shape / large-module A/B against the previous commit.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5ldsb
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_table.py tests/test_gpu_parity.py tests/test_gpu_small.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1
timeout -k 10 300 python -u tools/probes/profile_ab.py 500 30 300 50 prev=netrep_amd/_lib/ab/prev.so ldsb=- > $D/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/probes/profile_ab.py 1000 330 2000 12 prev=netrep_amd/_lib/ab/prev.so ldsb=- > $D/ab_big.txt 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > $D/bench.json 2> $D/bench.err
