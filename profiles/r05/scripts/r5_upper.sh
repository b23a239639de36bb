# Round 5: the wave matvec's mirrored-sum reductions without the nb branch (C2 shape).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5upper
mkdir -p $D
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 prev=netrep_amd/_lib/ab/prev.so tree=- > $D/ab_C2.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_edge.py tests/test_abi_driver.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1
