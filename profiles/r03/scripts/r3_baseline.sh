set -o pipefail
mkdir -p gpurun_out/r3b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3b/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r3b/bench.json 2> gpurun_out/r3b/bench.err
