# Round 6 final tree, part 2: the C5 line (10,000 permutations per dataset),
# the props record, the extended parity sweep (C3 1,024 and C2 2,048
# permutations).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6final2
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 500 python -u bench.py --config C5 --perms-per-step 10000 --steps 1 --warmup 0 --no-cpu-baseline > $D/C5.json 2> $D/C5.err
D0=$D
D=$D/props bash tools/props_record.sh
D=$D0
find gpurun_out/r6final2/props -name "*.csv" ! -name "*kernel_stats*" -delete
timeout -k 10 900 python -u tools/parity_sweep.py 1024 2048 > $D/parity_sweep.json 2> $D/parity_sweep.err
du -sh gpurun_out
