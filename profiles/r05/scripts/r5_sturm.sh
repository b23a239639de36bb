# Round 5: Sturm passes test sign alternation (one op per step) instead of counting
# sign changes: C2 / C3 shapes against the previous commit, tests.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5sturm
mkdir -p $D
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 prev=netrep_amd/_lib/ab/prev.so tree=- > $D/ab_C2.txt 2>&1
timeout -k 10 300 python -u tools/probes/profile_ab.py 500 30 300 50 prev=netrep_amd/_lib/ab/prev.so tree=- > $D/ab_C3.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_configs.py tests/test_gpu_edge.py tests/test_abi_driver.py tests/test_gpu_dual.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1
