# Round 5: PMC passes of the block Lanczos probe (mode 1, 64,000 items per launch).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5blockpmc
mkdir -p $D
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d $D/$name -o run -- \
      python3 tools/probes/block_probe.py tools/probes/bp_kernel.so 100 64000 1 1 > $D/$name.log 2>&1 || return 1
}
run sq SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE || exit 1
run fetch FETCH_SIZE || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
echo done
