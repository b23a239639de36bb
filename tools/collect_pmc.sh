#!/bin/bash
# Collect the rocprofv3 evidence for one bench configuration (run on the GPU box).
# One counter group per pass (no --pmc with tracing domains; gpurun refuses that mix).
#   tools/collect_pmc.sh <out_dir> [bench args...]
set -o pipefail
out=${1:?out dir}; shift
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- \
      python3 bench.py --no-cpu-baseline "${BENCH_ARGS[@]}" > "$out/$name.log" 2>&1 || return 1
}
BENCH_ARGS=("$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 bench.py --no-cpu-baseline "${BENCH_ARGS[@]}" > "$out/trace.log" 2>&1 || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit 1
run mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE || exit 1
echo "pmc collection done: $out"
