# Round 5: sixteen lanes per occurrence for modules beyond 1,024 nodes (C5): tests, C5 / C4 lines.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5sweep16
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1
timeout -k 10 500 python -u bench.py --config C5 --perms-per-step 10000 --steps 1 --warmup 0 --no-cpu-baseline > $D/C5.json 2> $D/C5.err
timeout -k 10 300 python -u bench.py --config C4 --no-cpu-baseline > $D/C4.json 2> $D/C4.err
