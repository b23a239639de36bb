# Round 4: the driver's own bench command on the final tree.
set -o pipefail
D=gpurun_out/${1:-r4fin7}
mkdir -p $D
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench.json 2> $D/bench.err
