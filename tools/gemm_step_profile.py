"""Per-GEMM time breakdown of one real training step (bench.py's model and batch): records every
dfu_gemm launch, times each distinct descriptor with its library plan (HIP events, back-to-back
launches) and prints them sorted by time per step, with the plan, TFLOP/s and the HBM-bound
floor (compulsory bytes / 6 TB/s).

  python tools/gemm_step_profile.py [--batch 64] [--config fusion] [--iters 10] [--ab]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import ops  # noqa: E402

OPND = ["KM", "MN", "CFWD", "CDGD", "CDGW", "CWGX"]
EPI = ["BF16", "RELU", "GELU", "F32", "RESID", "DGELU", "ADD", "ACC", "ACCW", "STATS", "PATCH", "F32STATS",
       "DSTATS", "X3GELU", "F16DUAL", "F16GELU"]
TILE = ["auto", "128x128", "256x128", "128x256", "256x256", "128x128o2", "128x128w4", "256x256p8",
        "256x256ps", "192x256ps", "256x64", "128x64o2"]


def key(d):
    return (d.a_mode, d.b_mode, d.epilogue, d.M, d.N, d.K, d.conv_n, d.conv_h, d.conv_w, d.conv_c,
            d.conv_k, d.conv_r, d.conv_s, d.conv_stride, d.conv_pad, d.operand_type)


def time_desc(d, iters):
    lib = ops.lib()
    s = ops.stream_ptr()
    for _ in range(2):
        ops.check(lib.dfu_gemm(ctypes.byref(d), s), "dfu_gemm")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        lib.dfu_gemm(ctypes.byref(d), s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--config", default="fusion")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--precision", default="parity", help="record the step in this mode")
    ap.add_argument("--ab", action="store_true", help="also time the one-shot schedule")
    ap.add_argument("--tail-ab", action="store_true",
                    help="also time without the tail split (in the '1shot' column)")
    ap.add_argument("--markers", default=None,
                    help="PMC mode: before each distinct GEMM, launch one k_argmax_rows marker "
                         "kernel, then the GEMM 1 + iters times; write the shape list (in "
                         "launch order) to this JSON for tools/gemm_shape_traffic.py")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    from dfu_hip import nn as hnn
    from dfu_hip.optim import FusedAdamW
    model, fwd = bench.build(a.config, dev)
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=dev))
    rgb, th, y = bench.synthetic(a.batch, dev, 42)
    from dfu_hip import functional as Fn
    ops.gemm_record = []
    opt.zero_grad()
    with Fn.precision(a.precision):
        crit(fwd(model, rgb, th), y).backward()
    opt.step()
    rec, ops.gemm_record = ops.gemm_record, None
    torch.cuda.synchronize()
    uniq = {}
    for d, flops, nbytes, refs, _ in rec:
        e = uniq.setdefault(key(d), [d, flops, nbytes, refs, 0])
        e[4] += 1
    rows = []
    marks = []
    mk = torch.zeros((1, 2), device=dev)
    for d, flops, nbytes, refs, n in uniq.values():
        if a.markers:
            torch.cuda.synchronize()
            ops.argmax_rows(mk)  # segment delimiter in the dispatch trace
            marks.append({"key": list(key(d)), "per_step": n, "flops": flops, "bytes": nbytes,
                          "launches": 2 + a.iters})
        us = time_desc(d, a.iters)
        us1 = None
        if a.ab:
            old = ops.gemm_set_persistent(0)
            try:
                us1 = time_desc(d, a.iters)
            finally:
                ops.gemm_set_persistent(old)
        elif a.tail_ab:
            old = ops.gemm_set_tail_split(0)
            try:
                us1 = time_desc(d, a.iters)
            finally:
                ops.gemm_set_tail_split(old)
        t, sk = ctypes.c_int32(), ctypes.c_int32()
        ops.check(ops.lib().dfu_gemm_plan(ctypes.byref(d), ctypes.byref(t), ctypes.byref(sk)), "plan")
        rows.append((n * us, n, us, us1, flops, nbytes, d, t.value, sk.value))
    if a.markers:
        import json
        for m, r in zip(marks, rows):
            m["us"] = r[2]
            m["plan"] = [r[7], r[8]]
        with open(a.markers, "w") as f:
            json.dump(marks, f)
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    fl = sum(r[1] * r[4] for r in rows)
    print(f"{len(rec)} launches, {len(rows)} distinct; GEMM time {tot / 1e3:.3f} ms/step, "
          f"{fl / tot / 1e6:.0f} TFLOP/s")
    print(f"{'ms/step':>8} {'n':>3} {'us':>7} {'1shot':>7} {'TF/s':>5} {'hbm_us':>6}  plan  shape")
    for tot_us, n, us, us1, flops, nbytes, d, t, sk in rows:
        name = (f"{OPND[d.a_mode]}x{OPND[d.b_mode]}->{EPI[d.epilogue]} {d.M}x{d.N}x{d.K}"
                + (f" conv{d.conv_h}x{d.conv_w} c{d.conv_c} k{d.conv_k} r{d.conv_r} s{d.conv_stride}"
                   if d.conv_n else "") + (" f16" if d.operand_type else ""))
        print(f"{tot_us / 1e3:8.3f} {n:3d} {us:7.1f} {us1 if us1 is not None else 0:7.1f} "
              f"{flops / us / 1e6:5.0f} {nbytes / 6e6:6.1f}  {TILE[t]}/{sk}  {name}", flush=True)


if __name__ == "__main__":
    main()
