# Round 6 call 5: where C4's sweep time goes (kernel traces of check2 and
# sweep2, two SQ counter passes of each, summarised on the box and the raw
# CSVs removed), C5 at its record's size (10,000 permutations per dataset)
# for base and sweep2, and the props record (Scale through pinned chunks, the
# residency fingerprint at C5 shape) on the in-tree build (sweep2).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab5
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
A=netrep_amd/_lib/ab
C4="bench.py --config C4 --steps 3 --warmup 1 --no-secondary --no-cpu-baseline"
for v in check2 sweep2; do
  O=$D/$v
  mkdir -p $O
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $C4 --lib $A/lib$v.so > $O/trace.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- python3 $C4 --lib $A/lib$v.so > $O/sq.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $O/mfma -o run -- python3 $C4 --lib $A/lib$v.so > $O/lds.log 2>&1 || exit 1
  python3 tools/summarize_pmc.py $O --json $O/summary.json > $O/summary.txt || exit 1
  cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv || true
  rm -rf $O/trace $O/sq $O/mfma
done
B5="python -u bench.py --config C5 --perms-per-step 10000 --steps 1 --warmup 1 --no-secondary --no-cpu-baseline"
timeout -k 10 300 $B5 --lib $A/libbase.so > $D/base_C5.json 2> $D/base_C5.err || exit 1
timeout -k 10 300 $B5 --lib $A/libsweep2.so > $D/sweep2_C5.json 2> $D/sweep2_C5.err || exit 1
D=$D/props bash tools/props_record.sh
for s in trace fetch write; do
  find gpurun_out/r6ab5/props/$s -name "*.csv" ! -name "*stats*" ! -name "*counter_collection*" -delete 2>/dev/null || true
done
du -sh gpurun_out
