"""Per-kernel statistics from a rocprofv3 SQLite output (rocpd tables): the
kernel-trace summary when --stats' CSV is not written (rocprofv3's default
output format on this image). usage: python tools/rocpd_stats.py RESULTS.db"""
import sqlite3
import sys


def kernel_stats(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    cols = [r[1] for r in cur.execute(f"pragma table_info({disp})")]
    scol = [r[1] for r in cur.execute(f"pragma table_info({sym})")]
    name_col = "display_name" if "display_name" in scol else ("kernel_name" if "kernel_name" in scol else "name")
    q = (f"select s.{name_col}, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end - d.start), "
         f"max(d.end - d.start) from {disp} d join {sym} s on d.kernel_id = s.id group by s.{name_col} "
         f"order by sum(d.end - d.start) desc")
    return list(cur.execute(q)), cols


if __name__ == "__main__":
    rows, _ = kernel_stats(sys.argv[1])
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':70s} {'calls':>6s} {'total_ms':>10s} {'avg_ms':>9s} {'pct':>6s}")
    for name, n, s, a, mn, mx in rows:
        print(f"{name[:70]:70s} {n:6d} {s / 1e6:10.3f} {a / 1e6:9.3f} {100 * s / tot:6.2f}")
