# Round 5: wave class with buffer-load operands: tests, A/B, stamps, icache/wait counters.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5wave5
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_abi_driver.py tests/test_gpu_small.py tests/test_gpu_dual.py -m gpu -x -v --timeout 120 --timeout-method thread > $D/pytest_small.txt 2>&1
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 small=netrep_amd/_lib/ab/base.so wave=- > $D/ab_C2.txt 2>&1
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 wave_st=netrep_amd/_lib/diag/wave_stamps.so > $D/stamps_C2.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $D/pmc1 -o run -- python3 tools/probes/profile_ab.py --single wave - 100 30 300 20 > $D/pmc1.log 2>&1
