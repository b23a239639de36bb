# GPU tests + default bench (a build already in the tree)
set -o pipefail
D=gpurun_out/${1:-r3c}
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
