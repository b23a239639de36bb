# final record: default bench command (C3 + C4 + CPU baseline) and C5 with three host datasets
set -o pipefail
D=gpurun_out/${1:-r3finalB}
mkdir -p $D
timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err && \
timeout -k 10 700 python -u bench.py --config C5 --steps 2 --warmup 1 --perms-per-step 512 > $D/C5.json 2> $D/C5.err
