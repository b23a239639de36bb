set -o pipefail
D=gpurun_out/s3e; mkdir -p $D
B="python -u bench.py --steps 10 --no-secondary --no-cpu-baseline"
timeout -k 10 200 $B > $D/d3.json 2> $D/d3.err && \
NETREP_LIB=$PWD/netrep_amd/_lib/libnetrep_amd_d2.so timeout -k 10 200 $B > $D/d2.json 2> $D/d2.err && \
timeout -k 10 200 $B > $D/d3b.json 2> $D/d3b.err && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $D/pytest.txt 2>&1
