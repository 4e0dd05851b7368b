"""Kernel time per category on each queue of one phase of a rocprofv3 kernel trace (forward:
the step's start to the ResNet's k_avgpool_fwd*, backward: k_ce_bwd to the first AdamW), to see
what the critical stream of that phase spends its time on.
Usage: python tools/trace_stream_mix.py <kernel_trace.csv> [step index] [forward|backward]"""
import collections
import csv
import re
import sys

STEP_MARK = re.compile(r"k_im2col_lds|k_stem_conv_x3")  # the stem: one launch per step
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
si = int(sys.argv[2]) if len(sys.argv) > 2 else 5
phase = sys.argv[3] if len(sys.argv) > 3 else "forward"
idx = [i for i, r in enumerate(rows) if STEP_MARK.search(r["Kernel_Name"])]
seg = rows[idx[si]:idx[si + 1]]
t0 = int(seg[0]["Start_Timestamp"])
pool = min(int(r["End_Timestamp"]) for r in seg if "k_avgpool_fwd" in r["Kernel_Name"])
ce = min(int(r["Start_Timestamp"]) for r in seg if "k_ce_bwd" in r["Kernel_Name"])
adam = min(int(r["Start_Timestamp"]) for r in seg if "adamw" in r["Kernel_Name"])
lo, hi = (t0, pool) if phase == "forward" else (ce, adam)


def cat(n):
    if "gemm" in n:
        return "gemm"
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:44]


for q in sorted({r["Queue_Id"] for r in seg}):
    c, k = collections.Counter(), collections.Counter()
    busy, last = 0.0, lo
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if r["Queue_Id"] != q or s < lo or s > hi:
            continue
        d = (e - s) / 1e3
        c[cat(r["Kernel_Name"])] += d
        k[cat(r["Kernel_Name"])] += 1
        busy += d
        last = max(last, e)
    if not c:
        continue
    print(f"queue {q} ({phase}): ends {(last - t0) / 1e3:.0f} us, kernel time {busy:.0f} us")
    for n, v in c.most_common(12):
        print(f"   {n:46s} {v:8.1f} us  n={k[n]}")
