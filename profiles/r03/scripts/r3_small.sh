set -o pipefail
D=gpurun_out/${1:-r3s}; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_dual.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --config C2 --no-secondary --no-cpu-baseline > $D/C2.json 2> $D/C2.err && \
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 > $D/ab_C2.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-secondary --no-cpu-baseline > $D/C3.json 2> $D/C3.err && \
timeout -k 10 600 python -u bench.py --config C5 --c5-single --no-secondary --no-cpu-baseline --steps 4 > $D/C5.json 2> $D/C5.err
