# Round 6 final tree: PMC passes of the C3, C2, C4 and C5 lines
# (tools/collect_pmc.sh), summarised on the box (raw CSVs removed: gpurun
# copies back at most 64 MiB).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6finalpmc
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for c in C3 C2 C4 C5; do
  if [ $c = C5 ]; then X="--steps 1 --warmup 1 --perms-per-step 1920"; else X="--steps 3 --warmup 1"; fi
  bash tools/collect_pmc.sh $D/$c --config $c --no-secondary $X
  python3 tools/summarize_pmc.py $D/$c --json $D/$c/summary.json > $D/$c/summary.txt
  cp $D/$c/trace/run_kernel_stats.csv $D/$c/kernel_stats.csv
  find $D/$c -name '*.csv' ! -name 'kernel_stats.csv' -delete
  find $D/$c -name '*.db' -delete
  du -sh $D/$c
done
