"""CPU oracle study for C2 (thermal-only ViT-B/16, train_thermal_only.py:188-205): the logits'
distance from the fp32 oracle when ViT Blocks store fp16 at the MI355X path's rounding sites
(the "parity" mode's fp16 stage), with chosen blocks exact (the bf16x3 proxy: 2^-17 products)
and chosen rounding sites exact inside the fp16 blocks.  Train-mode forward, dropout identity,
B = 64.  The emulation reproduces the GPU: all blocks fp16 gives 1.601e-3 on seed 0 here, the
HIP path 1.612e-3 (profiles/r19_thermal_bench.json).
  python tools/c2_precision_study.py [B] [seeds] [cases]      (cases: ";"-separated names, default all)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from oracle import torch_ref as R  # noqa: E402

torch.set_num_threads(int(os.environ.get("THREADS", "8")))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
seeds = [int(s) for s in (sys.argv[2] if len(sys.argv) > 2 else "0,1,2").split(",")]
SITES = ("ln1", "ln1_w", "qkv", "p", "attn_out", "attn_out_w", "ln2", "ln2_w", "gelu", "gelu_w")
W = ("ln1_w", "attn_out_w", "ln2_w", "gelu_w")


def policy(exact_blocks=(), sites=()):
    """[(block index, exact sites)] of the fp16 blocks: blocks in exact_blocks run exact."""
    return [(k, tuple(sites)) for k in range(12) if k not in exact_blocks]


CASES = {
    "all fp16": policy(),
    "block 0 exact": policy((0,)),
    "blocks 0-1 exact": policy((0, 1)),
    "blocks 0-2 exact": policy((0, 1, 2)),
    "blocks 0,11 exact": policy((0, 11)),
    "blocks 0-5 exact": policy(range(6)),
    "blocks 0-8 exact": policy(range(9)),
    "blocks 0-10 exact": policy(range(11)),
    "block 0 exact, ln1 exact": policy((0,), ("ln1",)),
    "block 0 exact, ln1+ln2 exact": policy((0,), ("ln1", "ln2")),
    "block 0 exact, weights exact": policy((0,), W),
    "weights exact": policy((), W),
}
for site in SITES:
    CASES[f"{site} exact"] = policy((), (site,))
if len(sys.argv) > 3:
    CASES = {k: v for k, v in CASES.items() if k in sys.argv[3].split(";")}


def run(vit, x, pol):
    hs = []
    for k, ex in pol:
        m = vit.blocks[k]
        hs.append(m.register_forward_pre_hook(
            lambda m, i, ex=ex: R.set_bf16_emulation(True, exact_sites=ex, dtype=torch.float16)))
        hs.append(m.register_forward_hook(lambda m, i, o: R.set_bf16_emulation(False)))
    try:
        with torch.no_grad():
            return vit(x)
    finally:
        for h in hs:
            h.remove()
        R.set_bf16_emulation(False)


res = {k: [] for k in CASES}
for s in seeds:
    torch.manual_seed(s)
    vit = R.VisionTransformer(num_classes=2)
    vit.head = nn.Sequential(nn.Dropout(0.0), nn.Linear(768, 2))
    vit.train()
    _, th, _ = R.synthetic_batch(B, seed=42 + s)
    t0 = time.time()
    f32 = run(vit, th, [])
    print(f"seed {s} B={B}: max|logit| {f32.abs().max():.4f} ({time.time() - t0:.0f} s)",
          flush=True)
    for name, pol in CASES.items():
        d = (run(vit, th, pol) - f32).abs().max().item()
        res[name].append(d)
        print(f"  {name:32s}: max|dlogit| {d:.3e}", flush=True)
print("summary (worst over seeds):")
for name, ds in res.items():
    print(f"  {name:32s}: {max(ds):.3e}  [{' '.join(f'{d:.2e}' for d in ds)}]")
