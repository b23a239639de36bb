"""Loops of one kernel in hipcc --save-temps assembly: for every back-edge
(a branch to an earlier label) the block range it closes, with its
instruction mix (scratch spills/reloads, buffer/global loads, LDS ops, fp64
FMAs/MFMAs, barriers). Used to see whether register spills sit in hot loops.
usage: python tools/asm_loops.py file.s kernel_symbol_substring"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
want = sys.argv[2]
start = next(i for i, l in enumerate(lines) if re.match(r"^\S*" + re.escape(want) + r"\S*:", l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\S+):", l)
    if m:
        labels[m.group(1)] = i
loops = []
for i, l in enumerate(body):
    m = re.search(r"s_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        loops.append((labels[m.group(2)], i, m.group(2)))


def mix(a, b):
    c = {"scr_ld": 0, "scr_st": 0, "vmem_ld": 0, "lds": 0, "fma64": 0, "mfma": 0, "barrier": 0, "n": 0}
    for l in body[a:b + 1]:
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        c["n"] += 1
        if t.startswith("scratch_load"):
            c["scr_ld"] += 1
        elif t.startswith("scratch_store"):
            c["scr_st"] += 1
        elif t.startswith(("buffer_load", "global_load")):
            c["vmem_ld"] += 1
        elif t.startswith("ds_"):
            c["lds"] += 1
        elif t.startswith(("v_fma_f64", "v_fmac_f64")):
            c["fma64"] += 1
        elif t.startswith("v_mfma"):
            c["mfma"] += 1
        elif t.startswith("s_barrier"):
            c["barrier"] += 1
    return c


for a, b, lab in sorted(loops):
    c = mix(a, b)
    flag = "  <-- spill code in loop" if c["scr_ld"] + c["scr_st"] else ""
    print(f"loop {lab} lines {a}-{b}: " + " ".join(f"{k}={v}" for k, v in c.items()) + flag)
