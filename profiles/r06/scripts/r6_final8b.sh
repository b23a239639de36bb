# Round 6 committed final tree (first Ritz check of the wave class at step 18):
# the C2 PMC passes (its profile kernel changed since r6_final5c.sh).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6final8b
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash tools/collect_pmc.sh $D/C2 --config C2 --no-secondary --steps 3 --warmup 1
python3 tools/summarize_pmc.py $D/C2 --json $D/C2/summary.json > $D/C2/summary.txt
cp $D/C2/trace/run_kernel_stats.csv $D/C2/kernel_stats.csv
find $D/C2 -name '*.csv' ! -name 'kernel_stats.csv' -delete
find $D/C2 -name '*.db' -delete
du -sh gpurun_out
