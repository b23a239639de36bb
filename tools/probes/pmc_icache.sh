# Instruction-cache counters for the summary-profile kernels (GPU box).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_ic
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_ic/p1 -o run -- python3 tools/probes/profile_ab.py 500 30 255 42 rg4 packed4 > gpurun_out/pmc_ic/p1.log 2>&1 || exit 1
echo done
