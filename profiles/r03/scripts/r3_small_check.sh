# GPU suite + default bench + C2 bench on the tree (small class at 2 waves)
set -o pipefail
D=gpurun_out/${1:-r3small_check}
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $D/bench.json 2> $D/bench.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-secondary --no-cpu-baseline > $D/C2.json 2> $D/C2.err
