"""Idle gaps of a rocprofv3 kernel trace: stretches of one step (bounded by the stem's im2col
launch) in which no kernel runs on any queue, with the kernels on each side.
Usage: python tools/trace_gaps.py <kernel_trace.csv> [step index] [min gap us]"""
import csv
import re
import sys

STEP_MARK = re.compile(r"k_im2col_lds|k_stem_conv_x3")  # the stem: one launch per step
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
si = int(sys.argv[2]) if len(sys.argv) > 2 else 5
mg = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
idx = [i for i, r in enumerate(rows) if STEP_MARK.search(r["Kernel_Name"])]
seg = rows[idx[si]:idx[si + 1]]
t0 = int(seg[0]["Start_Timestamp"])
end, last = int(seg[0]["End_Timestamp"]), seg[0]
tot = 0.0
for r in seg[1:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s > end:
        g = (s - end) / 1e3
        tot += g
        if g >= mg:
            print(f"t={(end - t0) / 1e3:8.1f} us gap {g:6.1f} us  after q{last['Queue_Id']} "
                  f"{last['Kernel_Name'][:60]}  before q{r['Queue_Id']} {r['Kernel_Name'][:60]}")
    if e > end:
        end, last = e, r
print(f"total idle {tot:.1f} us over {(end - t0) / 1e3:.1f} us")
