# Round 5 final tree: PMC passes (tools/collect_pmc.sh) of the C3 line, the C4 line and the C2 line,
# summarised on the box (tools/summarize_pmc.py) so that only summaries, logs and the
# kernel statistics come back (the per-dispatch CSVs exceed gpurun_out's 64 MiB).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5pmcfinal
mkdir -p $D
for c in C3 C4 C2; do
  if [ $c = C3 ]; then X="--no-secondary"; else X=""; fi
  bash tools/collect_pmc.sh $D/$c --config $c $X --steps 3 --warmup 1
  python3 tools/summarize_pmc.py $D/$c --json $D/$c/summary.json > $D/$c/summary.txt
  cp $D/$c/trace/run_kernel_stats.csv $D/$c/kernel_stats.csv
  find $D/$c -name 'run_*.csv' -delete
  du -sh $D/$c
done
