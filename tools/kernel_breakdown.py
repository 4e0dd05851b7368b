"""Per-kernel time per step from a rocprofv3 kernel trace (steps bounded by the stem's im2col
launch; the first two and the last are skipped), optionally per queue.
Usage: python tools/kernel_breakdown.py <kernel_trace.csv> [top] [--queues]"""
import collections
import csv
import re
import sys

STEP_MARK = re.compile(r"k_im2col_lds|k_stem_conv_x3")  # the stem: one launch per step
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
top = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 50
by_q = "--queues" in sys.argv
idx = [i for i, r in enumerate(rows) if STEP_MARK.search(r["Kernel_Name"])]
steps = list(zip(idx[2:-1], idx[3:]))
agg, cnt = collections.defaultdict(float), collections.defaultdict(int)
for a, b in steps:
    for r in rows[a:b]:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        n = re.sub(r"\(.*", "", n)[:100]
        if by_q:
            n = f"q{r['Queue_Id']} {n}"
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        agg[n] += d
        cnt[n] += 1
ns = len(steps)
print(f"steps {ns}, kernel time {sum(agg.values()) / ns / 1e3:.2f} ms/step")
for n, v in sorted(agg.items(), key=lambda kv: -kv[1])[:top]:
    print(f"{v / ns / 1e3:8.3f} ms {cnt[n] / ns:6.1f}/step {v / cnt[n]:7.1f} us  {n}")
