# Round 6 final tree, part 2: the C3 and C5 PMC passes (the table kernel and
# the large-module kernel changed), then the C5 large-item Gram alone under
# counters (tools/runs/r6_c5gram.sh).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6final4b
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for c in C3 C5; do
  if [ $c = C5 ]; then X="--steps 1 --warmup 1 --perms-per-step 1920"; else X="--steps 3 --warmup 1"; fi
  bash tools/collect_pmc.sh $D/$c --config $c --no-secondary $X
  python3 tools/summarize_pmc.py $D/$c --json $D/$c/summary.json > $D/$c/summary.txt
  cp $D/$c/trace/run_kernel_stats.csv $D/$c/kernel_stats.csv
  find $D/$c -name '*.csv' ! -name 'kernel_stats.csv' -delete
  find $D/$c -name '*.db' -delete
done
timeout -k 10 900 bash tools/runs/r6_c5gram.sh
du -sh gpurun_out
