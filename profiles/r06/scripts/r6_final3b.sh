# Round 6 final tree (with the 64 x 112 dual Gram), part 2: the C5 PMC pass
# (the large-module kernel changed) and a 64-permutation C5 parity sweep.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6final3b
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash tools/collect_pmc.sh $D/C5 --config C5 --no-secondary --steps 1 --warmup 1 --perms-per-step 1920
python3 tools/summarize_pmc.py $D/C5 --json $D/C5/summary.json > $D/C5/summary.txt
cp $D/C5/trace/run_kernel_stats.csv $D/C5/kernel_stats.csv
find $D/C5 -name '*.csv' ! -name 'kernel_stats.csv' -delete
find $D/C5 -name '*.db' -delete
timeout -k 10 700 python -u tools/parity_sweep.py 0 0 64 > $D/parity_sweep_C5.json 2> $D/parity_sweep_C5.err
du -sh gpurun_out
