set -o pipefail
mkdir -p gpurun_out/s3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s3/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/s3/bench.json 2> gpurun_out/s3/bench.err
