# Round 5 final tree (the wave class): PMC passes of the C3 line and the C4 line
# (tools/collect_pmc.sh), summarised on the box.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5final3pmc
mkdir -p $D
for c in C3 C4; do
  if [ $c = C3 ]; then X="--no-secondary"; else X=""; fi
  bash tools/collect_pmc.sh $D/$c --config $c $X --steps 3 --warmup 1
  python3 tools/summarize_pmc.py $D/$c --json $D/$c/summary.json > $D/$c/summary.txt
  cp $D/$c/trace/run_kernel_stats.csv $D/$c/kernel_stats.csv
  find $D/$c -name 'run_*.csv' -delete
  du -sh $D/$c
done
