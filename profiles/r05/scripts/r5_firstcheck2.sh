# Round 5: the packed / table kernels' first Ritz check at step 20 / 24 instead of 16 (C3 shape);
# the wave class's first check at 20 (C2 shape) against the previous commit.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5firstcheck2
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 600 python -u tools/probes/profile_ab.py 500 30 300 50 t16=- t20=$L/t20.so t24=$L/t24.so > $D/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 prev=$L/prev.so tree=- > $D/ab_C2.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1
