# Round 6 A/B 7: the multi-wave kernels' Ritz vector with eight basis loads in
# flight (ritz, the in-tree build) against sweep2, alternating on C3; C5 once
# each; the C3 null parity test on ritz (the same sums in the same order:
# bitwise the same cube expected).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab7
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
A=netrep_amd/_lib/ab
for i in 1 2; do
  for v in sweep2 ritz; do
    timeout -k 10 300 $B --lib $A/lib$v.so > $D/${v}_C3.$i.json 2> $D/${v}_C3.$i.err
  done
done
B5="python -u bench.py --config C5 --perms-per-step 10000 --steps 1 --warmup 1 --no-secondary --no-cpu-baseline"
for v in sweep2 ritz; do
  timeout -k 10 300 $B5 --lib $A/lib$v.so > $D/${v}_C5.json 2> $D/${v}_C5.err
done
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_dual.py -m gpu -x -v --timeout 500 --timeout-method thread > $D/pytest.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
