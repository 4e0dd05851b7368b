"""Which ResNet stages (and ViT block ranges) must run fp32-accurate (bf16x3) for the fusion
logits to stay within 1e-3 of the fp32 oracle?  CPU only: the oracle at C3's train-mode forward
with bf16 rounding emulated in a chosen set of stages and every other stage exact.
Usage: python tools/precision_stage_study.py [B]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch  # noqa: E402

from oracle import torch_ref as R  # noqa: E402

torch.set_num_threads(8)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
torch.manual_seed(0)
model = R.MultimodalFusionModel(num_classes=2, dropout=0.0).train()
rgb, th, _ = R.synthetic_batch(B, seed=42)


def stage_modules():
    """name -> module whose forward runs with emulation on (others off)."""
    r = model.resnet if hasattr(model, "resnet") else model.rgb_encoder
    v = model.vit if hasattr(model, "vit") else model.thermal_encoder
    out = {"l1": r.layer1, "l2": r.layer2, "l3": r.layer3, "l4": r.layer4}
    blocks = list(v.blocks)
    for i in range(0, len(blocks), 3):
        out[f"vit{i}-{i + 2}"] = torch.nn.Sequential(*blocks[i:i + 3])
    return r, v, out


r, v, stages = stage_modules()
_hooks = []


def run(emulated):
    """Forward with bf16 rounding emulated only inside the named stages ("stem": the ResNet stem;
    "vitpre": patch embed; "vitpost": final norm)."""
    hs = []

    def on(m, i):
        R.set_bf16_emulation(True)

    def off(m, i, o):
        R.set_bf16_emulation(False)
    for name in emulated:
        if name in stages:
            mods = [stages[name]] if not isinstance(stages[name], torch.nn.Sequential) or \
                name.startswith("l") else list(stages[name])
            for m in mods:
                hs.append(m.register_forward_pre_hook(on))
                hs.append(m.register_forward_hook(off))
        elif name == "stem":  # the stem calls conv() directly: on at the ResNet, off at layer1
            hs.append(r.register_forward_pre_hook(on))
            hs.append(r.layer1.register_forward_pre_hook(lambda m, i: R.set_bf16_emulation(False)))
    try:
        with torch.no_grad():
            return model(rgb, th)
    finally:
        for h in hs:
            h.remove()
        R.set_bf16_emulation(False)


f32 = run([])
print(f"B={B} max|logit| {f32.abs().max():.4f}")
cases = [["stem"], ["l1"], ["l2"], ["l3"], ["l4"], ["stem", "l1"], ["l3", "l4"],
         ["stem", "l1", "l2"], ["stem", "l1", "l2", "l3", "l4"]]
cases += [[k] for k in stages if k.startswith("vit")]
cases += [[k for k in stages if k.startswith("vit")]]
for c in cases:
    d = (run(c) - f32).abs().max().item()
    print(f"bf16 in {'+'.join(c):40s}: max|dlogit| {d:.3e}", flush=True)
