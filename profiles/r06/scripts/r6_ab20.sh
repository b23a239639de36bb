# Round 6 A/B 20: with the wave class's first Ritz check at step 18, that
# check through the coarse stage first (coarse) instead of full precision in
# one stage (fc18, the committed tree). C2 only, four runs each alternating;
# outputs compared in process pairs (tools/probes/profile_ab.py).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab20
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
A=netrep_amd/_lib/ab
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
for i in 1 2 3 4; do
  for v in fc18 coarse; do
    timeout -k 10 300 $B --config C2 --lib $A/lib$v.so > $D/${v}_C2.$i.json 2> $D/${v}_C2.$i.err
  done
done
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 fc18=$A/libfc18.so coarse=$A/libcoarse.so > $D/profile_ab_C2.txt 2>&1
