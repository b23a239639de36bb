"""Record one logical engine kernel's PMC pass (tools/summarize_pmc.py --json
output) in profiles/pmc_traffic.json, the file bench.py reads its `traffic` /
`executed` fields from. A logical kernel may be several device kernels of one
batch (e.g. C5's profile launches: the large-module kernel + the packed one):
their per-dispatch means are summed. Older rows of the same config / batch /
kernel / table mode are marked superseded.

  python tools/pmc_to_traffic.py SUMMARY.json CONFIG BATCH KERNEL DEVICE_SUBSTR[,SUBSTR...] SOURCE [--table]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRAFFIC = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def main():
    a = [x for x in sys.argv[1:] if not x.startswith("--")]
    summary, config, batch, kernel, subs, source = a[0], a[1], int(a[2]), a[3], a[4].split(","), a[5]
    table = "--table" in sys.argv
    res = json.load(open(summary))
    names = [k for k in res if any(s in k for s in subs)]
    if not names:
        raise SystemExit(f"no kernel matching {subs} in {summary}: {sorted(res)}")

    def tot(key):
        vals = [res[n][key] for n in names if key in res[n]]
        return sum(vals) if vals else None

    row = {"config": config, "batch": batch, "kernel": kernel, "device_kernel": " + ".join(sorted(names)),
           "hbm_bytes_per_launch": tot("hbm_bytes_corrected"), "fetch_size_kb_raw": tot("FETCH_SIZE"),
           "write_size_kb": tot("WRITE_SIZE"), "avg_ns_rocprof": tot("avg_ns"), "source": source}
    if table:
        row["gram_table"] = True
    hits, misses = tot("TCC_HIT_sum"), tot("TCC_MISS_sum")
    if hits is not None and misses:
        row["l2_hit_rate"] = hits / (hits + misses)
    for key in ("mfma_f64_flops_executed", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS"):
        v = tot(key)
        if v is not None:
            row[{"SQ_LDS_BANK_CONFLICT": "lds_bank_conflict_cycles", "SQ_INSTS_LDS": "lds_instructions"}.get(key, key)] = v
    busy = [res[n]["mfma_busy_pct"] for n in names if "mfma_busy_pct" in res[n]]
    if busy and row.get("avg_ns_rocprof"):
        # time-weighted over the device kernels of the launch
        w = [res[n].get("avg_ns", 0.0) for n in names if "mfma_busy_pct" in res[n]]
        row["mfma_busy_pct"] = sum(b * x for b, x in zip(busy, w)) / max(sum(w), 1.0)
    missing = [k for k in ("hbm_bytes_per_launch", "fetch_size_kb_raw", "write_size_kb", "avg_ns_rocprof")
               if row[k] is None]
    if missing:
        raise SystemExit(f"pass incomplete: {missing}")
    rows = json.load(open(TRAFFIC))
    for r in rows:
        if (r.get("config") == config and r.get("batch") == batch and r.get("kernel") == kernel
                and bool(r.get("gram_table", False)) == table and "superseded" not in r):
            r["superseded"] = f"by {source}"
    rows.append(row)
    json.dump(rows, open(TRAFFIC, "w"), indent=1)
    print(json.dumps(row, indent=1))


if __name__ == "__main__":
    main()
