# Round 6 final tree (r6_final5.sh), part 2: the extended parity sweep (C3 1,024, C2 2,048,
# C5 64 permutations) against the oracle; the C2 PMC passes (its profile kernel changed).
set -e
cd $GRAFT_REPO_ROOT
D=gpurun_out/r6final5c
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u tools/parity_sweep.py 1024 2048 0 > $D/parity_sweep.json 2> $D/parity_sweep.err
timeout -k 10 500 python -u tools/parity_sweep.py 0 0 64 > $D/parity_sweep_C5.json 2> $D/parity_sweep_C5.err
export TMPDIR=/tmp
bash tools/collect_pmc.sh $D/C2 --config C2 --no-secondary --steps 3 --warmup 1
python3 tools/summarize_pmc.py $D/C2 --json $D/C2/summary.json > $D/C2/summary.txt
cp $D/C2/trace/run_kernel_stats.csv $D/C2/kernel_stats.csv
find $D/C2 -name '*.csv' ! -name 'kernel_stats.csv' -delete
find $D/C2 -name '*.db' -delete
du -sh gpurun_out
