# Round 5: C5 A/B of the large-item Gram's super-tile order (2 x 2 blocks per four waves vs rows of four).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5g64ab
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
ARGS="--config C5 --perms-per-step 1920 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 400 python -u bench.py $ARGS > $D/blk2x2.json 2> $D/blk2x2.err
timeout -k 10 400 python -u bench.py $ARGS --lib netrep_amd/_lib/diag/g64_row.so > $D/row.json 2> $D/row.err
timeout -k 10 400 python -u bench.py $ARGS > $D/blk2x2_b.json 2> $D/blk2x2_b.err
