# Round 6 A/B 6: the column sweep with the next block of entries in flight
# while a block is summed (sweep3) against sweep2 (r6_ab4), alternating on C4
# and C2; C5 once each; then sweep3 in place of the in-tree library for the
# sweep's parity tests.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab6
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
A=netrep_amd/_lib/ab
for i in 1 2; do
  for c in C4 C2; do
    for v in sweep2 sweep3; do
      timeout -k 10 300 $B --config $c --lib $A/lib$v.so > $D/${v}_$c.$i.json 2> $D/${v}_$c.$i.err
    done
  done
done
B5="python -u bench.py --config C5 --perms-per-step 10000 --steps 1 --warmup 1 --no-secondary --no-cpu-baseline"
for v in sweep2 sweep3; do
  timeout -k 10 300 $B5 --lib $A/lib$v.so > $D/${v}_C5.json 2> $D/${v}_C5.err
done
cp $A/libsweep3.so netrep_amd/_lib/libnetrep_amd.so
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_fallbacks.py tests/test_gpu_configs.py -m gpu -x -v --timeout 500 --timeout-method thread > $D/pytest.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
