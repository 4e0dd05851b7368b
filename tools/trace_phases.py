"""Phase timeline of the fusion step from a rocprofv3 kernel trace: per step (bounded by the stem's
im2col launch), when each queue's forward ends (ResNet: k_avgpool_fwd; ViT: the last kernel
before the head's first launch), when the head starts and ends (k_ce_bwd), when each queue's
backward ends and when AdamW starts.  Times in us from the step's first launch.
Usage: python tools/trace_phases.py <kernel_trace.csv>"""
import csv
import re
import sys

STEP_MARK = re.compile(r"k_im2col_lds|k_stem_conv_x3")  # the stem: one launch per step
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if STEP_MARK.search(r["Kernel_Name"])]
for a, b in zip(idx, idx[1:]):
    seg = rows[a:b]
    t0 = int(seg[0]["Start_Timestamp"])
    T = lambda r, k="End_Timestamp": (int(r[k]) - t0) / 1e3  # noqa: E731
    rq = seg[0]["Queue_Id"]
    pool = [r for r in seg if "k_avgpool_fwd" in r["Kernel_Name"]]
    ce = [r for r in seg if "k_ce_bwd" in r["Kernel_Name"]]
    adam = [r for r in seg if "adamw" in r["Kernel_Name"]]
    if not (pool and ce and adam):
        continue
    head0 = int(pool[0]["End_Timestamp"])
    vq = [q for q in {r["Queue_Id"] for r in seg} if q != rq]
    vit_fwd_end = max((T(r) for r in seg if r["Queue_Id"] in vq and int(r["Start_Timestamp"]) <
                       int(ce[0]["Start_Timestamp"])), default=0)
    bwd = [r for r in seg if int(r["Start_Timestamp"]) > int(ce[0]["End_Timestamp"])]
    res_bwd_end = max((T(r) for r in bwd if r["Queue_Id"] == rq and "adamw" not in r["Kernel_Name"]),
                      default=0)
    vit_bwd_end = max((T(r) for r in bwd if r["Queue_Id"] in vq), default=0)
    print(f"res fwd end {T(pool[0]):7.0f}  vit fwd end {vit_fwd_end:7.0f}  head end (ce_bwd) "
          f"{T(ce[0]):7.0f}  res bwd end {res_bwd_end:7.0f}  vit bwd end {vit_bwd_end:7.0f}  "
          f"adamw start {T(adam[-1], 'Start_Timestamp'):7.0f}  step end {T(seg[-1]):7.0f}")
