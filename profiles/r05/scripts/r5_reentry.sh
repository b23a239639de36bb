# Round 5 re-entry: the GPU suite and the driver's default bench on the restored tree.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5re
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1
timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline > $D/C2.json 2> $D/C2.err
