"""Machine fill of a rocprofv3 kernel trace over one step (bounded by the stem's im2col launch):
per phase (forward, head, backward, optimizer tail), the time with no kernel running (idle), with
only kernels of < 64 workgroups running (latency-bound: a few CUs busy), and the histogram of
idle gaps.  Usage: python tools/trace_fill.py <kernel_trace.csv> [step index]"""
import csv
import re
import sys

STEP_MARK = re.compile(r"k_im2col_lds|k_stem_conv_x3")  # the stem: one launch per step
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
si = int(sys.argv[2]) if len(sys.argv) > 2 else 5
idx = [i for i, r in enumerate(rows) if STEP_MARK.search(r["Kernel_Name"])]
seg = rows[idx[si]:idx[si + 1]]
t0 = int(seg[0]["Start_Timestamp"])
ev = []
for r in seg:
    wgs = (int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])) // max(
        1, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"]))
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    ev.append((s, e, wgs, r["Kernel_Name"]))
end = max(e for _, e, _, _ in ev)
ce = [s for s, e, w, n in ev if "k_ce_bwd" in n]
pool = [e for s, e, w, n in ev if "k_avgpool_fwd" in n]
adam = [s for s, e, w, n in ev if "adamw" in n]
marks = [("forward", 0.0, min(pool + ce)), ("head", min(pool + ce), max(ce)),
         ("backward", max(ce), min(adam)), ("tail", min(adam), end)]
step = 1.0  # us bins
nb = int(end / step) + 1
busy = [0] * nb
big = [0] * nb
for s, e, w, n in ev:
    for b in range(int(s / step), min(nb, int(e / step) + 1)):
        busy[b] += 1
        if w >= 64:
            big[b] += 1
print(f"step {end:.0f} us ({len(ev)} dispatches)")
for name, a, b in marks:
    bins = range(int(a / step), min(nb, int(b / step)))
    idle = sum(1 for k in bins if busy[k] == 0) * step
    small = sum(1 for k in bins if busy[k] and not big[k]) * step
    print(f"  {name:9s} {a:8.0f}-{b:8.0f} us: idle {idle:7.0f} us, only small kernels "
          f"{small:7.0f} us")
gaps = []
cur = None
for k in range(nb):
    if busy[k] == 0:
        cur = (cur or 0) + step
    elif cur:
        gaps.append(cur)
        cur = None
hist = {}
for g in gaps:
    key = "<5" if g < 5 else "5-10" if g < 10 else "10-20" if g < 20 else ">=20"
    hist[key] = hist.get(key, 0) + g
print("  idle gaps by length (us total):", {k: round(v) for k, v in sorted(hist.items())},
      f"count {len(gaps)}")
