# Round 6 A/B 2 on the C3 bench command: base (round-5 kernel), new (the extra
# check at the predicted fp32 crossing, committed), tier6 (+ the six-byte
# tier: fp32 copy + 16-bit corrections, first check at step 8), alternating on
# one box; then (tier6 is the in-tree build; r6_run2.sh ran the GPU suite on it) a
# 1,024-permutation C3 parity sweep, and phase stamps of C3 and C2.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab2
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
for i in 1 2; do
  timeout -k 10 300 $B --lib netrep_amd/_lib/ab/libbase.so > $D/base$i.json 2> $D/base$i.err
  timeout -k 10 300 $B --lib netrep_amd/_lib/ab/libnew.so > $D/new$i.json 2> $D/new$i.err
  timeout -k 10 300 $B --lib netrep_amd/_lib/ab/libtier6.so > $D/tier6_$i.json 2> $D/tier6_$i.err
done
timeout -k 10 600 python -u tools/parity_sweep.py 1024 0 0 > $D/parity_sweep.json 2> $D/parity_sweep.err
S="python -u bench.py --no-secondary --no-cpu-baseline --steps 3 --stamps --lib netrep_amd/_lib/diag/libstamps.so"
timeout -k 10 300 $S > $D/stamps_C3.json 2> $D/stamps_C3.err
timeout -k 10 300 $S --config C2 > $D/stamps_C2.json 2> $D/stamps_C2.err
