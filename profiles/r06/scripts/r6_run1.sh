# Round 6, first call of the re-entered session: smoke and the whole GPU suite on
# the committed tree, then A/B 1 (the Ritz check at the predicted crossing of the
# fp32 threshold, new, against the round-5 kernel, base), alternating on one box.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6run1
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/ || true
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
for i in 1 2; do
  timeout -k 10 300 $B --lib netrep_amd/_lib/ab/libbase.so > $D/base$i.json 2> $D/base$i.err
  timeout -k 10 300 $B > $D/new$i.json 2> $D/new$i.err
done
