# Round-3 record: the default bench command (C3 + C4 secondary + CPU baseline),
# C2, and C5 with three host datasets
set -o pipefail
D=gpurun_out/${1:-r3final}
mkdir -p $D
timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-secondary --no-cpu-baseline > $D/C2.json 2> $D/C2.err && \
timeout -k 10 900 python -u bench.py --config C5 --steps 2 --warmup 1 --perms-per-step 512 > $D/C5.json 2> $D/C5.err
