# Round 4: modules whose Lanczos dimension exceeds the LDS vectors (variant 6)
# against the LAPACK restatement, and the relabelled bench line.
set -o pipefail
D=gpurun_out/${1:-r4c2}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_dual.py -x -v --timeout 400 --timeout-method thread -k "beyond" > $D/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 > $D/bench.json 2> $D/bench.err
