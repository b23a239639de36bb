# Round 6, the committed final tree (the wave class's first Ritz check at step
# 18 through the coarse stage first, A/B 20): smoke, the GPU suite, the default bench,
# the C2 line, the C2 parity sweep at 2,048 permutations (its outputs moved
# by up to 3.9e-15 against A/B 20's base).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6final9
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 python -u bench.py --config C2 > $D/C2.json 2> $D/C2.err
timeout -k 10 400 python -u tools/parity_sweep.py 0 2048 0 > $D/parity_sweep_C2.json 2> $D/parity_sweep_C2.err
du -sh gpurun_out
