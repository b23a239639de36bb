# Round 5: the wave class (register-resident Gram, one wave per item) against the
# small class on the C2 shape; then the GPU suite and the C2 bench line.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5wave1
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 small=netrep_amd/_lib/ab/base.so wave=- > $D/ab_C2.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline > $D/C2.json 2> $D/C2.err
