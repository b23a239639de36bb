# Round 6 A/B 15: the Lanczos step's |w| and q-update scale 1/|w| computed
# before the omega phase, off the chain after its barrier (inv; recomputed
# when the step reorthogonalises; the large-module kernel keeps the previous
# order) against the committed final tree (f6). C3 and C2 alternating, three
# runs each; outputs compared in process pairs (tools/probes/profile_ab.py:
# max scaled difference, 0 = bitwise); then the C3 / C2 null parity tests on inv.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab15
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
A=netrep_amd/_lib/ab
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
for i in 1 2 3; do
  for v in f6 inv; do
    timeout -k 10 300 $B --lib $A/lib$v.so > $D/${v}_C3.$i.json 2> $D/${v}_C3.$i.err
    timeout -k 10 300 $B --config C2 --lib $A/lib$v.so > $D/${v}_C2.$i.json 2> $D/${v}_C2.$i.err
  done
done
timeout -k 10 300 python -u tools/probes/profile_ab.py 500 30 300 50 f6=$A/libf6.so inv=$A/libinv.so > $D/profile_ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 f6=$A/libf6.so inv=$A/libinv.so > $D/profile_ab_C2.txt 2>&1
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -k "c3_nulls or c2" --timeout 500 --timeout-method thread > $D/pytest.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
