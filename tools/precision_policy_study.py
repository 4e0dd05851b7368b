"""Per-stage precision study on the MI355X ("next" item 1): which stage
assignment keeps the fusion logits within north_star's 1e-3 of the fp32 oracle with margin
(target <= 5e-4 on every seed), and what does each cost?

For each seed: the fp32 CPU oracle (oracle/torch_ref.py, train-mode BN, dropout identity) at C3's
B = 64 on that seed's weights and synthetic batch, then the HIP model on the same weights under
functional.precision("mixed") for every policy; then the train step (fwd + bwd + AdamW) is timed
for every policy that passes on all seeds (and the pure modes).

  python tools/precision_policy_study.py [--seeds 0,1,2] [--grid] [--out ...json]
    --grid: also the (ResNet bf16 suffix x ViT bf16 suffix) grid of round 4's first study
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

from dfu_hip import functional as Fn  # noqa: E402
from models import precision as P  # noqa: E402
from models.fusion import MultimodalFusionModel  # noqa: E402
from oracle import torch_ref as R  # noqa: E402

RES_SUFFIX = (0, 1, 2, 3, 4, 5, 6, 7, 9, 13, 16)
VIT_SUFFIX = (0, 1, 2, 3, 4, 5, 6, 8, 12)


def policies(model, grid):
    out = {"x3": {}}
    for k in (0, 1, 2, 3, 4, 6):
        out[f"vit_fp16_after_{k}x3"] = P.parity_policy(model, k)
    if grid:
        for r in RES_SUFFIX:
            for v in VIT_SUFFIX:
                out[f"r{r}_v{v}"] = P.suffix(model, r, v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="0,1,2")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--bar", type=float, default=5e-4)
    ap.add_argument("--time-steps", type=int, default=10)
    ap.add_argument("--grid", action="store_true")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "precision_study.json"))
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    dev = torch.device("cuda", 0)
    seeds = [int(s) for s in a.seeds.split(",")]
    res = {"batch": a.batch, "bar": a.bar, "seeds": seeds, "cases": {}}
    hip = None
    for s in seeds:
        torch.manual_seed(s)
        ref = R.MultimodalFusionModel(num_classes=2, dropout=0.0).train()
        rgb, th, _ = R.synthetic_batch(a.batch, seed=42 + s)
        t0 = time.time()
        with torch.no_grad():
            want = ref(rgb, th)
        print(f"seed {s}: oracle {time.time() - t0:.1f} s, max|logit| "
              f"{want.abs().max():.4f}", flush=True)
        hip = MultimodalFusionModel(num_classes=2, dropout=0.0)
        hip.load_state_dict(ref.state_dict(), strict=True)
        hip = hip.to(dev).train()
        r_d, t_d = rgb.to(dev), th.to(dev)
        for mode in ("bf16", "bf16x3", "parity"):
            with torch.no_grad(), Fn.precision(mode):
                d = (hip(r_d, t_d).float().cpu() - want).abs().max().item()
            res["cases"].setdefault(mode, []).append(d)
            print(f"  {mode:24s}: {d:.3e}", flush=True)
        for name, pol in policies(hip, a.grid).items():
            P.apply_policy(hip, pol)
            with torch.no_grad(), Fn.precision("mixed"):
                d = (hip(r_d, t_d).float().cpu() - want).abs().max().item()
            res["cases"].setdefault(name, []).append(d)
            print(f"  {name:24s}: {d:.3e}", flush=True)
        del ref
    from dfu_hip import nn as hnn
    from dfu_hip.optim import FusedAdamW
    passing = [k for k, ds in res["cases"].items() if max(ds) <= a.bar]
    print("passing:", passing, flush=True)
    model = hip
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=dev))
    g = torch.Generator(device=dev).manual_seed(0)
    rgb = torch.randn(a.batch, 3, 224, 224, device=dev, generator=g)
    th = torch.randn(a.batch, 3, 224, 224, device=dev, generator=g)
    y = torch.randint(0, 2, (a.batch,), device=dev, generator=g)

    def step():
        opt.zero_grad()
        crit(model(rgb, th), y).backward()
        opt.step()

    def timeit():
        for _ in range(4):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.time_steps):
            step()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.time_steps

    res["step_ms"] = {}
    pols = policies(model, a.grid)
    for k in ["bf16", "bf16x3", "parity"] + [k for k in passing if k in pols]:
        if k in ("bf16", "bf16x3", "parity"):
            mode = k
        else:
            P.apply_policy(model, pols[k])
            mode = "mixed"
        with Fn.precision(mode):
            ms = timeit()
        res["step_ms"][k] = round(ms, 3)
        print(f"step {k:24s}: {ms:.3f} ms", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
