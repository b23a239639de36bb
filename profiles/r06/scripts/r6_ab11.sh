# Round 6 A/B 11 on C3: the Ritz check at the predicted crossing of the fp32
# threshold again (cross), now that checks are cheaper (round 6's first try,
# r6_ab2's `new`, was neutral at the old check cost), against the final tree;
# then the C3 null parity test on cross.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab11
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
A=netrep_amd/_lib/ab
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
for i in 1 2 3; do
  for v in final cross; do
    timeout -k 10 300 $B --lib $A/lib$v.so > $D/${v}_C3.$i.json 2> $D/${v}_C3.$i.err
  done
done
cp $A/libcross.so netrep_amd/_lib/libnetrep_amd.so
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -k "c3_nulls or c3_two" --timeout 500 --timeout-method thread > $D/pytest.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
