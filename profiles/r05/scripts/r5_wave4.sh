# Round 5: wave class with burst reorthogonalisation / Ritz vector / dual sums and
# one-wave barriers: A/B vs the small class, stamps, targeted tests.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5wave4
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_abi_driver.py tests/test_gpu_small.py tests/test_gpu_dual.py -m gpu -x -v --timeout 120 --timeout-method thread > $D/pytest_small.txt 2>&1
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 small=netrep_amd/_lib/ab/base.so wave=- > $D/ab_C2.txt 2>&1
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 wave_st=netrep_amd/_lib/diag/wave_stamps.so > $D/stamps_C2.txt 2>&1
