# Round 6 final tree, part 3: the extended parity sweep (C3 1,024, C2 2,048,
# C5 64 permutations) against the oracle.
set -e
cd $GRAFT_REPO_ROOT
D=gpurun_out/r6final4c
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u tools/parity_sweep.py 1024 2048 0 > $D/parity_sweep.json 2> $D/parity_sweep.err
timeout -k 10 500 python -u tools/parity_sweep.py 0 0 64 > $D/parity_sweep_C5.json 2> $D/parity_sweep_C5.err
du -sh gpurun_out
