# Round 5: column sweep v3 (slot-ordered occurrence metadata, sixteen lanes per
# occurrence, prefetch): parity subset, C2 / C4 bench lines, rocprofv3 kernel stats of C4.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5s3
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edge.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1
timeout -k 10 300 python -u bench.py --config C4 --steps 4 --warmup 1 --no-cpu-baseline > $D/C4.json 2> $D/C4.err
timeout -k 10 300 python -u bench.py --config C2 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $D/C2.json 2> $D/C2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o c4 --output-format csv -- python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $D/C4_prof.json 2> $D/C4_prof.err
