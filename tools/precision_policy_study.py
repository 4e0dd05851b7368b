"""Per-stage precision study on the MI355X ("next" item 1): which suffixes of
the two encoders can run plain bf16 while the rest runs bf16x3, with the fusion logits within
north_star's 1e-3 of the fp32 oracle (target: <= 5e-4 on every seed)?

For each seed: the fp32 CPU oracle (oracle/torch_ref.py, train-mode BN, dropout identity) at C3's
B = 64 on that seed's weights and synthetic batch, then the HIP model on the same weights under
functional.precision("mixed") for a grid of (ResNet bf16 suffix, ViT bf16 suffix) policies.
Then the train step (fwd + bwd + AdamW) is timed for every policy that passes on all seeds.

  python tools/precision_policy_study.py [--seeds 0,1,2] [--out gpurun_out/precision_study.json]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="0,1,2")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--bar", type=float, default=5e-4)
    ap.add_argument("--time-steps", type=int, default=10)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "precision_study.json"))
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    dev = torch.device("cuda", 0)
    seeds = [int(s) for s in a.seeds.split(",")]
    combos = [(r, v) for r in RES_SUFFIX for v in VIT_SUFFIX]
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
        for mode in ("bf16", "bf16x3"):
            with torch.no_grad(), Fn.precision(mode):
                d = (hip(r_d, t_d).float().cpu() - want).abs().max().item()
            res["cases"].setdefault(mode, []).append(d)
            print(f"  {mode:8s}: {d:.3e}", flush=True)
        for r, v in combos:
            P.apply_policy(hip, P.suffix(hip, r, v))
            with torch.no_grad(), Fn.precision("mixed"):
                d = (hip(r_d, t_d).float().cpu() - want).abs().max().item()
            res["cases"].setdefault(f"r{r}_v{v}", []).append(d)
            print(f"  resnet bf16 suffix {r:2d} vit bf16 suffix {v:2d}: {d:.3e}", flush=True)
        del ref
    # time the passing policies (and both pure modes) on the train step
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
        for _ in range(3):
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
    for k in ["bf16", "bf16x3"] + [k for k in passing if k.startswith("r")]:
        if k in ("bf16", "bf16x3"):
            mode = k
        else:
            r, v = (int(x[1:]) for x in k.split("_"))
            P.apply_policy(model, P.suffix(model, r, v))
            mode = "mixed"
        with Fn.precision(mode):
            ms = timeit()
        res["step_ms"][k] = round(ms, 3)
        print(f"step {k:10s}: {ms:.3f} ms", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
