# Round 6 A/B 17: the wave class's first Ritz check at step 22 or 24 instead
# of 20 (round 5 moved it 16 -> 20; C2 items stop at ~24 steps). C2 only (the
# other kernels are unchanged), three runs each alternating; Lanczos steps and
# outputs compared in process pairs (tools/probes/profile_ab.py: max scaled
# difference against fc20).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab17
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
A=netrep_amd/_lib/ab
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
for i in 1 2 3; do
  for v in fc20 fc22 fc24; do
    timeout -k 10 300 $B --config C2 --lib $A/lib$v.so > $D/${v}_C2.$i.json 2> $D/${v}_C2.$i.err
  done
done
timeout -k 10 400 python -u tools/probes/profile_ab.py 100 30 300 20 fc20=$A/libfc20.so fc22=$A/libfc22.so fc24=$A/libfc24.so > $D/profile_ab_C2.txt 2>&1
