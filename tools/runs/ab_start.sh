set -o pipefail
D=gpurun_out/s3b; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u bench.py > $D/bench_new.json 2> $D/bench_new.err && \
NETREP_START_COL=0 timeout -k 10 300 python -u bench.py > $D/bench_old.json 2> $D/bench_old.err
