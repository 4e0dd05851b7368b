"""Per-step stream occupancy from a rocprofv3 kernel trace: for each step (bounded by the stem's
im2col launch), the wall span, the union of kernel busy time, and each queue's kernel time and
launch count; plus the time both queues run kernels at once.
Usage: python tools/trace_streams.py <kernel_trace.csv> [marker substring]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
mark = sys.argv[2] if len(sys.argv) > 2 else "k_stem_conv_x3"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]


def union(iv):
    iv = sorted(iv)
    tot, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + ce - cs, iv


for a, b in zip(idx, idx[1:]):
    seg = rows[a:b]
    st, en = int(seg[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in seg)
    q = collections.defaultdict(list)
    for r in seg:
        q[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    busy, _ = union([x for v in q.values() for x in v])
    per = {k: (round(union(v)[0] / 1e6, 2), len(v)) for k, v in q.items()}
    both = sum(union(v)[0] for v in q.values()) - busy
    print(f"step wall {(en - st) / 1e6:6.2f} ms  busy {busy / 1e6:6.2f}  both-queues {both / 1e6:5.2f}  "
          f"per queue (busy ms, launches) {per}")
