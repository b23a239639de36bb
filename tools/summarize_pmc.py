"""Summarise tools/collect_pmc.sh output per engine kernel (mean per full-size
dispatch: the bench's timed launches, without its one-permutation launches).

FETCH_SIZE/WRITE_SIZE are in KB. Following MI355X_MICROARCH.md (HBM section),
FETCH_SIZE reads 1/2 of the bytes of wide coalesced streams on gfx950; the
`hbm_bytes_corrected` column doubles it (exact for the wide streaming kernels,
an upper estimate for narrow random reads, whose ratio is uncalibrated).

  python tools/summarize_pmc.py <out_dir> [--json file]
"""
import csv
import json
import os
import sys
from collections import defaultdict


def load(path):
    agg = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not (name.startswith("nr::") or "nr::" in name[:60]):
            continue
        key = name.split("(")[0].replace("void ", "")
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def full_size(values):
    """Indices of the full-size dispatches: the bench's timed launches, not the
    one-permutation launches of the observed statistics and discovery vectors
    (>= 10% of the largest dispatch's count)."""
    top = max(values) if values else 0.0
    return [i for i, v in enumerate(values) if v >= 0.1 * top]


def main():
    out = sys.argv[1]
    res = defaultdict(dict)
    for sub in ("fetch", "write", "tcc", "sq", "mfma"):
        for k, cs in load(os.path.join(out, sub, "run_counter_collection.csv")).items():
            first = next(iter(cs.values()))
            keep = full_size(first)  # the pass's first counter sizes its dispatches
            for c, v in cs.items():
                kept = [v[i] for i in keep if i < len(v)]
                res[k][c] = sum(kept) / len(kept)
                res[k]["dispatches_" + sub] = len(kept)
    trace = os.path.join(out, "trace", "run_kernel_trace.csv")
    if os.path.exists(trace):
        dur = defaultdict(list)
        for r in csv.DictReader(open(trace)):
            if "nr::" in r["Kernel_Name"]:
                key = r["Kernel_Name"].split("(")[0].replace("void ", "")
                dur[key].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
        for key, v in dur.items():
            kept = [v[i] for i in full_size(v)]
            res[key]["avg_ns"] = sum(kept) / len(kept)
            res[key]["calls"] = len(kept)
    for k, d in res.items():
        if "FETCH_SIZE" in d:
            d["hbm_bytes_corrected"] = d["FETCH_SIZE"] * 1024 * 2 + d.get("WRITE_SIZE", 0.0) * 1024
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / max(d["TCC_HIT_sum"] + d["TCC_MISS_sum"], 1)
        if "GRBM_GUI_ACTIVE" in d:
            # rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs (MI355X_MICROARCH.md,
            # DVFS give-back): the kernel's own clock count is a 1/8 of it.
            d["gui_active_cycles"] = d["GRBM_GUI_ACTIVE"] / 8
            if "avg_ns" in d and d["avg_ns"] > 0:
                d["effective_clock_ghz"] = d["gui_active_cycles"] / d["avg_ns"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d:
            # busy cycles summed over the 1,024 SIMDs (256 CUs x 4)
            d["mfma_busy_pct"] = 100 * d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8 * 1024)
        if "SQ_INSTS_VALU_MFMA_MOPS_F64" in d:
            # one MOPS unit = 512 executed f64 flops (16x16x4 f64: 2,048 flops = 4 units)
            d["mfma_f64_flops_executed"] = 512 * d["SQ_INSTS_VALU_MFMA_MOPS_F64"]
            if "avg_ns" in d and d["avg_ns"] > 0:
                d["mfma_f64_tflops_executed"] = d["mfma_f64_flops_executed"] / d["avg_ns"] / 1e3
        if "SQ_WAVE_CYCLES" in d:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in d:
                    d[c + "_frac"] = d[c] / max(d["SQ_WAVE_CYCLES"], 1)
    for k in sorted(res):
        print(k)
        for c, v in sorted(res[k].items()):
            print(f"   {c:36s} {v:.6g}")
    if "--json" in sys.argv:
        json.dump(res, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
