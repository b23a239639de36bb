# Round 5: the column sweep (network statistics by test column): GPU parity
# suite on the configs it serves, then C4 / C2 bench lines.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5s1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edge.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5s1/pytest.txt 2>&1
timeout -k 10 300 python -u bench.py --config C2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r5s1/C2.json 2> gpurun_out/r5s1/C2.err
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r5s1/C3.json 2> gpurun_out/r5s1/C3.err
