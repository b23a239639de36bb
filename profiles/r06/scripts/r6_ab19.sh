# Round 6 A/B 19: the 4-wave kernels' first Ritz check at step 18 or 20
# instead of 16 (round 5 on the older checks: 20 -0.2%, 24 +0.9%), on C3 (the
# table kernel), three runs each alternating; Lanczos steps and outputs
# compared in process pairs (tools/probes/profile_ab.py on the C3 shape).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab19
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
A=netrep_amd/_lib/ab
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
for i in 1 2 3; do
  for v in tc16 tc18 tc20; do
    timeout -k 10 300 $B --lib $A/lib$v.so > $D/${v}_C3.$i.json 2> $D/${v}_C3.$i.err
  done
done
timeout -k 10 400 python -u tools/probes/profile_ab.py 500 30 300 50 tc16=$A/libtc16.so tc18=$A/libtc18.so tc20=$A/libtc20.so > $D/profile_ab_C3.txt 2>&1
