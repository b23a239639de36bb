# Round 6: the C5 large-item Gram alone on the final tree (64 x 112 dual
# super-tiles; diagnostic build NR_GRAM_ONLY: every item stops after its Gram) under rocprofv3:
# kernel trace, MFMA/wave-state, FETCH and L2 passes. Round 5's recipe (r5_c5gram.sh) without TA/TCP.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6c5gram
mkdir -p $D
LIB=netrep_amd/_lib/diag/gram_only.so
ARGS="--config C5 --perms-per-step 1024 --steps 1 --warmup 0 --no-cpu-baseline --lib $LIB"
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
mkdir -p $D/trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $ARGS > $D/trace.json 2> $D/trace.err || exit 1
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 400 rocprofv3 --pmc "$@" --output-format csv -d $D/$name -o run -- python3 bench.py $ARGS > $D/$name.log 2>&1 || return 1
}
run sq SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
run fetch FETCH_SIZE || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
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
