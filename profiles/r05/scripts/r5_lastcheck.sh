# Round 5: last check of the committed tree's build (smoke and a quick GPU subset).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5lastcheck
mkdir -p $D
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py tests/test_abi_driver.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 10 > $D/C2.json 2> $D/C2.err
