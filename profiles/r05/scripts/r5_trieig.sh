# Round 5: branch-free, unrolled tridiagonal eigenvector: tests, C2 / C3 A/B against the
# previous commit, C2 stamps, C5 line again.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5trieig
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_table.py tests/test_gpu_parity.py tests/test_gpu_small.py tests/test_gpu_dual.py tests/test_abi_driver.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 prev=netrep_amd/_lib/ab/prev.so tree=- > $D/ab_C2.txt 2>&1
timeout -k 10 300 python -u tools/probes/profile_ab.py 500 30 300 50 prev=netrep_amd/_lib/ab/prev.so tree=- > $D/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 wave_st=netrep_amd/_lib/diag/wave_stamps.so > $D/stamps_C2.txt 2>&1
timeout -k 10 500 python -u bench.py --config C5 --perms-per-step 10000 --steps 1 --warmup 0 --no-cpu-baseline > $D/C5.json 2> $D/C5.err
