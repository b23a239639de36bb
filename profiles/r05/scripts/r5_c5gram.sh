# Round 5: the C5 large-item Gram alone (diagnostic build NR_GRAM_ONLY: every
# item stops after its Gram) under rocprofv3: kernel trace, MFMA/wave-state, FETCH, L2, TA/TCP passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5c5gram
mkdir -p $D
LIB=netrep_amd/_lib/diag/gram_only.so
ARGS="--config C5 --perms-per-step 1024 --steps 1 --warmup 0 --no-cpu-baseline --lib $LIB"
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -s KILL 120 rocprofv3 -L > $D/counters.txt 2>&1 || true
SEL=""
for c in TA_TA_BUSY_sum TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum; do
  grep -q "\b$c\b" $D/counters.txt && SEL="$SEL $c"
done
echo "TA/TCP counters: $SEL" > $D/tatcp_selected.txt
mkdir -p $D/trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $ARGS > $D/trace.json 2> $D/trace.err || exit 1
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 400 rocprofv3 --pmc "$@" --output-format csv -d $D/$name -o run -- python3 bench.py $ARGS > $D/$name.log 2>&1 || return 1
}
run sq SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
run fetch FETCH_SIZE || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
if [ -n "$SEL" ]; then run tatcp $SEL || exit 1; fi
python3 - $D <<'PY' > $D/summary.txt
import csv, collections, os, sys, statistics
D = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ("sq", "fetch", "tcc", "tatcp"):
    f = os.path.join(D, sub, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        if "nr::module_profile" in r["Kernel_Name"]:
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = collections.defaultdict(list)
for r in csv.DictReader(open(os.path.join(D, "trace", "run_kernel_trace.csv"))):
    if "nr::module_profile" in r["Kernel_Name"]:
        dur[r["Kernel_Name"].split("(")[0]].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:36s} n={len(v):3d} mean={statistics.mean(v):.5g} max={max(v):.5g}")
    if k in dur:
        print(f"  duration_ms n={len(dur[k])} mean={statistics.mean(dur[k]) / 1e6:.4f}")
PY
find $D -name 'run_*.csv' ! -name 'run_kernel_stats.csv' -delete
du -sh $D
