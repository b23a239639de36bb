# Round 5: sweep A/B, 8 lanes per occurrence (8 occurrences per wave batch) vs 16.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5l8
mkdir -p $D
for v in def l8 def2 l82; do
  L=""; case $v in l8*) L="--lib netrep_amd/_lib/ab/l8.so";; esac
  timeout -k 10 300 python -u bench.py --config C4 --steps 4 --warmup 1 --no-cpu-baseline $L > $D/C4_$v.json 2> $D/C4_$v.err
  timeout -k 10 300 python -u bench.py --config C2 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary $L > $D/C2_$v.json 2> $D/C2_$v.err
done
