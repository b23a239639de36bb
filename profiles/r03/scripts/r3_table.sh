# Gram-table path: its tests first, then the GPU suite and the default bench
set -o pipefail
D=gpurun_out/${1:-r3tab}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py -x -v --timeout 120 --timeout-method thread > $D/pytest_table.txt 2>&1 && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $D/bench.json 2> $D/bench.err
