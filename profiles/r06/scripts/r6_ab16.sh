# Round 6 A/B 16: the wave class keeps its three-term step's w and old q
# entries in registers for the q update (keep; no LDS re-read unless the step
# reorthogonalises) against the committed tree (f7). C2 only (the other
# kernels are unchanged), four runs each alternating; outputs compared in
# process pairs (tools/probes/profile_ab.py: max scaled difference, 0 =
# bitwise); then the C2 null parity test on keep.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab16
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
A=netrep_amd/_lib/ab
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
for i in 1 2 3 4; do
  for v in f7 keep; do
    timeout -k 10 300 $B --config C2 --lib $A/lib$v.so > $D/${v}_C2.$i.json 2> $D/${v}_C2.$i.err
  done
done
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 f7=$A/libf7.so keep=$A/libkeep.so > $D/profile_ab_C2.txt 2>&1
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -k "c2" --timeout 500 --timeout-method thread > $D/pytest.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
