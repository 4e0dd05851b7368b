"""Why a kernel runs longer inside the two-stream step than alone: for every dispatch of the
kernels matching a regex in a rocprofv3 kernel trace, its duration, the part of it during which
a kernel from ANOTHER queue was running, and which kernels those were (by overlap time).
  python tools/trace_overlap.py <kernel_trace.csv> <kernel regex> [first step index]
Steps are bounded by the stem's launch; the first steps (warm-up) are skipped."""
import collections
import csv
import re
import sys

STEP_MARK = re.compile(r"k_im2col_lds|k_stem_conv_x3")  # the stem: one launch per step


def short(k):
    k = re.sub(r"\(anonymous namespace\)::", "", k)
    k = re.sub(r"\(.*$", "", k).replace("void ", "").replace("dfu::", "")
    return k.strip()[:60]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    pat = re.compile(sys.argv[2])
    first = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    marks = [i for i, r in enumerate(rows) if STEP_MARK.search(r["Kernel_Name"])]
    seg = rows[marks[first]:marks[-1]]
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"] if "Queue_Id" in r
           else r.get("Stream_Id", ""), r["Kernel_Name"]) for r in seg]
    hits = [e for e in ev if pat.search(e[3])]
    others = collections.Counter()
    table = []
    for s, t, q, _ in hits:
        cover = []
        for s2, t2, q2, k2 in ev:
            if q2 == q or t2 <= s or s2 >= t:
                continue
            a, b = max(s, s2), min(t, t2)
            cover.append((a, b))
            others[short(k2)] += b - a
        cover.sort()
        busy, cur_a, cur_b = 0, None, None
        for a, b in cover:  # union of the other queue's busy intervals
            if cur_b is None or a > cur_b:
                if cur_b is not None:
                    busy += cur_b - cur_a
                cur_a, cur_b = a, b
            else:
                cur_b = max(cur_b, b)
        if cur_b is not None:
            busy += cur_b - cur_a
        table.append(((t - s) / 1e3, busy / max(1, t - s)))
    if not table:
        print("no dispatch matches", sys.argv[2])
        return
    n = len(table)
    print(f"{n} dispatches of /{sys.argv[2]}/ from step {first}: mean {sum(d for d, _ in table) / n:.1f} us, "
          f"other queue busy {100 * sum(f for _, f in table) / n:.0f}% of their time on average")
    for lo, hi in [(0.0, 0.5), (0.5, 0.9), (0.9, 1.01)]:
        sel = [d for d, f in table if lo <= f < hi]
        if sel:
            print(f"  other queue busy {100 * lo:3.0f}-{min(100, 100 * hi):3.0f}% of the dispatch: "
                  f"{len(sel):3d} dispatches, mean {sum(sel) / len(sel):6.1f} us, "
                  f"min {min(sel):6.1f}, max {max(sel):6.1f}")
    tot = sum(others.values())
    print("kernels running beside them (share of the overlap time):")
    for k, v in others.most_common(12):
        print(f"  {100 * v / tot:5.1f}%  {k}")


if __name__ == "__main__":
    main()
