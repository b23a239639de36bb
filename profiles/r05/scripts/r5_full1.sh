# Round 5: full GPU suite on the sweep tree; C5 with the sweep; the props calls under rocprofv3.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5f1
mkdir -p $D
# a line a minute under gpurun_out while steps run silently (each step has its own time limit)
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1
timeout -k 10 400 python -u bench.py --config C5 --perms-per-step 1024 --steps 1 --warmup 1 --no-cpu-baseline > $D/C5.json 2> $D/C5.err
bash tools/props_record.sh
bash profiles/r05/scripts/r5_block.sh
