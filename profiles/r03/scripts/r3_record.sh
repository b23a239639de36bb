# Round-3 record of the default bench command (C3 + C4 secondary + CPU baseline) and C2
set -o pipefail
D=gpurun_out/${1:-r3record}
mkdir -p $D
timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-secondary --no-cpu-baseline > $D/C2.json 2> $D/C2.err
