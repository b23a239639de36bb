# Network-kernel pipeline check: GPU tests, C5 (engine layer and three host
# datasets) and the default bench (C3 + the C4 network-only record)
set -o pipefail
D=gpurun_out/${1:-r3net}
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --config C5 --c5-single --steps 4 --warmup 1 --perms-per-step 512 --batch 64 --no-cpu-baseline > $D/C5s.json 2> $D/C5s.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $D/bench.json 2> $D/bench.err && \
timeout -k 10 900 python -u bench.py --config C5 --steps 2 --warmup 1 --perms-per-step 512 > $D/C5.json 2> $D/C5.err
