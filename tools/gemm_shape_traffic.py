"""Per-shape GEMM table of one training step: time, TFLOP/s and PMC HBM bytes per launch.

Joins tools/gemm_step_profile.py --markers <shapes.json> (run under separate rocprofv3
--pmc FETCH_SIZE and --pmc WRITE_SIZE passes) with the counter CSVs: the dispatches between two
k_argmax_rows markers belong to one distinct GEMM (its 2 + iters launches, split-K reduce
kernels included).  Bytes per launch = (FETCH_SIZE x 2 + WRITE_SIZE) KiB / launches (the gfx950
correction of MI355X_MICROARCH.md).

  python tools/gemm_shape_traffic.py shapes.json fetch.csv write.csv [times.txt] \
      > profiles/r03_gemm_shapes.md

times.txt (optional, recommended): the text output of an UNPROFILED tools/gemm_step_profile.py
run; its per-shape times replace the ones recorded in shapes.json, which were taken under the
--pmc profiler (counter collection serialises and slows every dispatch ~2-3x).
"""
import collections
import csv
import json
import sys

OPND = ["KM", "MN", "CFWD", "CDGD", "CDGW", "CWGX"]
EPI = ["BF16", "RELU", "GELU", "F32", "RESID", "DGELU", "ADD", "ACC", "ACCW", "STATS", "PATCH",
       "F32STATS", "DSTATS", "X3GELU", "F16DUAL", "F16GELU"]
TILE = ["auto", "128x128", "256x128", "128x256", "256x256", "128x128o2", "128x128w4", "256x256p8",
        "256x256ps", "192x256ps", "256x64", "128x64o2"]


def segments(path, counter):
    """Per marker segment: the summed counter value over its dispatches."""
    by_disp = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            d = int(r["Dispatch_Id"])
            name = r["Kernel_Name"]
            v = float(r["Counter_Value"])
            if d in by_disp:
                by_disp[d] = (name, by_disp[d][1] + v)
            else:
                by_disp[d] = (name, v)
    segs, cur = [], None
    for d in sorted(by_disp):
        name, v = by_disp[d]
        if "k_argmax_rows" in name:
            cur = []
            segs.append(cur)
        elif cur is not None and ("gemm" in name or "splitk" in name or "phase_fill" in name):
            cur.append(v)
    return [sum(s) for s in segs]


def clean_times(path):
    """shape name -> us from gemm_step_profile.py's table (columns: ms/step n us 1shot TF/s
    hbm_us plan shape...)."""
    t = {}
    for ln in open(path):
        f = ln.split()
        if len(f) >= 8 and f[1].isdigit():
            try:
                t[" ".join(f[7:])] = float(f[2])
            except ValueError:
                pass
    return t


def main():
    shapes = json.load(open(sys.argv[1]))
    times = clean_times(sys.argv[4]) if len(sys.argv) > 4 else {}
    fetch = segments(sys.argv[2], "FETCH_SIZE")
    write = segments(sys.argv[3], "WRITE_SIZE")
    assert len(fetch) == len(write) == len(shapes), (len(fetch), len(write), len(shapes))
    rows = []
    for s, fb, wb in zip(shapes, fetch, write):
        k = s["key"]
        rd = fb * 1024 * 2 / s["launches"]
        wr = wb * 1024 / s["launches"]
        name = f"{OPND[k[0]]}x{OPND[k[1]]}->{EPI[k[2]]} {k[3]}x{k[4]}x{k[5]}"
        if k[6]:
            name += f" conv{k[7]}x{k[8]} c{k[9]} k{k[10]} r{k[11]} s{k[13]}"
        if len(k) > 15 and k[15]:
            name += " f16"
        if times:
            key = name
            if key not in times:
                raise SystemExit(f"no clean time for {key}")
            s = dict(s, us=times[key])
        rows.append((s["per_step"] * s["us"], s, rd, wr, name))
    rows.sort(key=lambda r: -r[0])
    tot_us = sum(r[0] for r in rows)
    tot_fl = sum(r[1]["per_step"] * r[1]["flops"] for r in rows)
    tot_b = sum(r[1]["per_step"] * (r[2] + r[3]) for r in rows)
    tot_alg = sum(r[1]["per_step"] * r[1]["bytes"] for r in rows)
    n = sum(r[1]["per_step"] for r in rows)
    print("# GEMM launches of one C3 training step, by shape\n")
    print(f"{n} launches, {len(rows)} distinct; {tot_us / 1e3:.3f} ms of GEMM per step (each shape "
          f"timed back to back, HIP events{', unprofiled run' if times else ''}), "
          f"**{tot_fl / tot_us / 1e6:.0f} TFLOP/s**; PMC HBM "
          f"traffic {tot_b / n / 1e6:.1f} MB per launch vs {tot_alg / n / 1e6:.1f} MB algorithmic "
          f"(**{tot_b / tot_alg:.2f}x**).\n")
    print("| ms/step | n | us | TFLOP/s | MB/launch (PMC rd+wr) | algorithmic MB | x | plan | shape |")
    print("|---:|---:|---:|---:|---:|---:|---:|---|---|")
    for t, s, rd, wr, name in rows:
        print(f"| {t / 1e3:.3f} | {s['per_step']} | {s['us']:.1f} | "
              f"{s['flops'] / s['us'] / 1e6:.0f} | {(rd + wr) / 1e6:.1f} | {s['bytes'] / 1e6:.1f} | "
              f"{(rd + wr) / s['bytes']:.2f} | {TILE[s['plan'][0]]}/{s['plan'][1]} | `{name}` |")


if __name__ == "__main__":
    main()
