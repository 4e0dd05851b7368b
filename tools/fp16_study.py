"""CPU oracle study: the fusion logits' distance from the fp32 oracle when the forward of a chosen
set of stages stores fp16 (or bf16) at the MI355X path's rounding sites and every other stage is
exact (the bf16x3 proxy).  C3 train-mode forward, B = 64 by default, seeds 0..2.
  python tools/fp16_study.py [B] [seeds]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch  # noqa: E402

from oracle import torch_ref as R  # noqa: E402

torch.set_num_threads(int(os.environ.get("THREADS", "8")))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
seeds = [int(s) for s in (sys.argv[2] if len(sys.argv) > 2 else "0,1,2").split(",")]


def run(model, rgb, th, mods, dtype):
    hs = []
    for m in mods:
        hs.append(m.register_forward_pre_hook(lambda m, i: R.set_bf16_emulation(True, dtype=dtype)))
        hs.append(m.register_forward_hook(lambda m, i, o: R.set_bf16_emulation(False)))
    try:
        with torch.no_grad():
            return model(rgb, th)
    finally:
        for h in hs:
            h.remove()
        R.set_bf16_emulation(False)


for s in seeds:
    torch.manual_seed(s)
    model = R.MultimodalFusionModel(num_classes=2, dropout=0.0).train()
    rgb, th, _ = R.synthetic_batch(B, seed=42 + s)
    t0 = time.time()
    f32 = run(model, rgb, th, [], None)
    print(f"seed {s} B={B}: max|logit| {f32.abs().max():.4f} ({time.time() - t0:.0f} s)", flush=True)
    v, r = model.vit, model.resnet
    cases = {
        "vit fp16": ([v], torch.float16),
        "vit bf16": ([v], torch.bfloat16),
        "vit blocks 4-11 fp16": (list(v.blocks)[4:], torch.float16),
        "resnet layer4 fp16": ([r.layer4], torch.float16),
        "resnet layer3+4 fp16": ([r.layer3, r.layer4], torch.float16),
        "resnet layer4 + vit fp16": ([r.layer4, v], torch.float16),
    }
    for name, (mods, dt) in cases.items():
        d = (run(model, rgb, th, mods, dt) - f32).abs().max().item()
        print(f"  {name:28s}: max|dlogit| {d:.3e}", flush=True)
