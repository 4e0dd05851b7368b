"""Offline GEMM plan tuning on MI355X -> dfu-multimodal_amd/csrc/gemm_tuned.inc.

Records every dfu_gemm launch of one real training step (bench.py's model and batch), and for
each distinct descriptor times every tile shape (1..5) x split-K candidate (weight gradients),
keeping the fastest.  The generated table is compiled into libdfu_hip.so and takes precedence
over the analytic cost model (csrc/gemm.hip), so plans are deterministic (no runtime tuning).

  python tools/gemm_tune.py [--batch 64] [--config fusion] [--out PATH] [--iters 10]
      [--only-wgrad --all-splits]  (the weight gradients over every split 1..32 too)
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import ops  # noqa: E402

SPLITS = [1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256]
OPND = ["KM", "MN", "CONV_FWD", "CONV_DGRAD", "CONV_DGRAD_W", "CONV_WGRAD_X"]
EPI = ["BF16", "BF16_RELU", "BF16_GELU", "F32", "F32_RESID", "BF16_DGELU", "BF16_ADD", "F32_ACC",
       "F32_ACC_CONVW", "BF16_STATS", "PATCH", "F32_STATS", "BF16_DSTATS", "X3_GELU", "F16_DUAL", "F16_GELU"]
CONV_FIELDS = ("conv_n", "conv_h", "conv_w", "conv_c", "conv_k", "conv_r", "conv_s",
               "conv_stride", "conv_pad")


def key(d):
    conv = d.a_mode >= L.OPND_CONV_FWD or d.b_mode >= L.OPND_CONV_FWD
    # the table's epilogue field is the dispatch key (| 128: interleaved bf16x3 pairs, | 64: fp16
    # operands -- whose lookup falls back to the bf16 entry of the same shape)
    e = d.epilogue | (128 if d.x3_pairs else 0) | (64 if d.operand_type == 1 else 0)
    return (d.a_mode, d.b_mode, e, d.M, d.N, d.K) + (
        tuple(getattr(d, f) for f in CONV_FIELDS) if conv else (0,) * 9)


def copy_desc(d):
    n = L.GemmDesc()
    ctypes.memmove(ctypes.byref(n), ctypes.byref(d), ctypes.sizeof(d))
    return n


def time_desc(d, iters, ws):
    lib = ops.lib()
    need = lib.dfu_gemm_workspace_bytes(ctypes.byref(d))
    if need > ws.numel():
        ws = torch.empty(need, dtype=torch.uint8, device="cuda")
    d.workspace = ws.data_ptr() if need > 0 else None
    d.workspace_bytes = int(need)
    cnt = ops.tile_counters(torch.device("cuda", 0))  # split-K / tail-split hand-off counters
    d.tile_counters, d.tile_counters_len = cnt.data_ptr(), cnt.numel()
    s = ops.stream_ptr()
    for _ in range(2):
        ops.check(lib.dfu_gemm(ctypes.byref(d), s), "dfu_gemm")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        lib.dfu_gemm(ctypes.byref(d), s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters, ws


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--config", default="fusion")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=os.path.join(ROOT, "dfu-multimodal_amd", "csrc",
                                                  "gemm_tuned.inc"))
    ap.add_argument("--append", action="store_true", help="keep entries already in --out")
    ap.add_argument("--tiles", default="1-11", help="tile ids to try, e.g. 1-11 or 6,8")
    ap.add_argument("--precision", default="bf16", help="record the step in this mode (bf16x3: "
                    "its forward GEMMs with tripled K)")
    ap.add_argument("--only-x3-pairs", action="store_true",
                    help="tune only the interleaved-pair bf16x3 GEMMs (dfu_gemm_desc.x3_pairs)")
    ap.add_argument("--only-f16", action="store_true",
                    help="tune only the fp16-operand GEMMs (dfu_gemm_desc.operand_type 1)")
    ap.add_argument("--only-wgrad", action="store_true",
                    help="tune only the split-K weight gradients (epilogue F32_ACC)")
    ap.add_argument("--all-splits", action="store_true",
                    help="weight gradients: every split 1..32 besides SPLITS (splits that fill the "
                         "CUs exactly, e.g. 36 tiles x 7 = 252 units)")
    ap.add_argument("--dump", default=None,
                    help="also write every timing (shape -> {tile/split: us}) to this JSON")
    a = ap.parse_args()
    tiles = []
    for part in a.tiles.split(","):
        lo, _, hi = part.partition("-")
        tiles += list(range(int(lo), int(hi or lo) + 1))
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
    for d, flops, _, refs, _ in rec:
        if a.only_x3_pairs and not d.x3_pairs:
            continue
        if a.only_f16 and d.operand_type != 1:
            continue
        if a.only_wgrad and d.epilogue != L.EPI_F32_ACC:
            continue
        uniq.setdefault(key(d), (d, flops, refs, []))[3].append(1)
    print(f"{len(rec)} launches, {len(uniq)} distinct GEMMs", flush=True)
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    lines, t_auto_sum, t_best_sum = [], 0.0, 0.0
    dump = {}
    t0 = time.time()
    for k, (d0, flops, refs, cnt) in uniq.items():
        n = len(cnt)
        d = copy_desc(d0)
        d.tile, d.split_k = 0, 0
        t_auto, ws = time_desc(d, a.iters, ws)
        best = (t_auto, 0, 0)
        ktiles = (d0.K + 63) // 64
        cand = sorted(set(SPLITS) | set(range(1, 33))) if a.all_splits else SPLITS
        splits = [s for s in cand if s <= ktiles] if d0.epilogue == L.EPI_F32_ACC else [1]
        for tile in tiles:
            for sk in splits:
                d = copy_desc(d0)
                d.tile, d.split_k = tile, sk
                try:
                    t, ws = time_desc(d, a.iters, ws)
                except L.DfuError:
                    break  # tile not instantiated for this combination
                dump.setdefault(",".join(map(str, k)), {"n": n, "t": {}})["t"][f"{tile}/{sk}"] = t
                if t < best[0]:
                    best = (t, tile, sk)
        t_auto_sum += n * t_auto
        t_best_sum += n * min(best[0], t_auto)
        name = (f"{OPND[d0.a_mode]}x{OPND[d0.b_mode]}->{EPI[d0.epilogue]}{'/P' if d0.x3_pairs else ''}{'/f16' if d0.operand_type == 1 else ''} "
                f"{d0.M}x{d0.N}x{d0.K} (x{n}/step)")
        print(f"{name:62s} auto {t_auto:8.1f} us  best {best[0]:8.1f} us tile {best[1]} "
              f"split {best[2]}  {flops / best[0] / 1e6:6.0f} TFLOP/s", flush=True)
        if not best[1]:  # the current plan won: record it too, so the table is complete
            d = copy_desc(d0)
            d.tile, d.split_k = 0, 0
            tt, ss = ctypes.c_int32(), ctypes.c_int32()
            ops.check(ops.lib().dfu_gemm_plan(ctypes.byref(d), ctypes.byref(tt), ctypes.byref(ss)),
                      "dfu_gemm_plan")
            best = (best[0], tt.value, ss.value if d0.epilogue == L.EPI_F32_ACC else 0)
        if best[1]:
            lines.append("    {" + ", ".join(str(v) for v in k) + f", {best[1]}, {best[2]}}},"
                         f"  // {name}: {best[0]:.1f} us (model {t_auto:.1f} us)")
    print(f"GEMM time per step: model plans {t_auto_sum / 1e3:.3f} ms -> tuned "
          f"{t_best_sum / 1e3:.3f} ms ({time.time() - t0:.0f} s tuning)")
    keep = []
    if a.append and os.path.exists(a.out):
        keep = [ln.rstrip("\n") for ln in open(a.out) if ln.startswith("    {")]
        have = {ln.split("}")[0] for ln in lines}
        keep = [ln for ln in keep if ln.split("}")[0] not in have]
    with open(a.out, "w") as f:
        f.write("// Generated by tools/gemm_tune.py on MI355X (gfx950): fastest tile/split-K per GEMM of\n"
                "// the DFU training step. Fields: a_mode, b_mode, epilogue, M, N, K, conv n,h,w,c,k,r,s,"
                "stride,pad,\n// tile (1..11), split.\n")
        for ln in keep + lines:
            f.write(ln + "\n")
    print(f"wrote {len(keep) + len(lines)} entries to {a.out}")
    if a.dump:
        import json
        with open(a.dump, "w") as f:
            json.dump(dump, f)


if __name__ == "__main__":
    main()
