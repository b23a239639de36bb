# Round 5: PMC passes of the C2 line with the wave class (tools/collect_pmc.sh),
# summarised on the box.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5wavepmc2
mkdir -p $D
for c in C2; do
  bash tools/collect_pmc.sh $D/$c --config $c --steps 3 --warmup 1
  python3 tools/summarize_pmc.py $D/$c --json $D/$c/summary.json > $D/$c/summary.txt
  cp $D/$c/trace/run_kernel_stats.csv $D/$c/kernel_stats.csv
  find $D/$c -name 'run_*.csv' -delete
  du -sh $D/$c
done
