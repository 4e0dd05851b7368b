"""Which bf16 storage points of the ViT branch drive its feature error vs fp32?  CPU only:
the oracle in bf16-emulation mode with one rounding site at a time left exact."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch  # noqa: E402

from oracle import torch_ref as R  # noqa: E402

torch.set_num_threads(8)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
torch.manual_seed(0)
vit = R.VisionTransformer(num_classes=0).train()
_, th, _ = R.synthetic_batch(B, seed=42)


def feats(on, exact=()):
    R.set_bf16_emulation(on, exact)
    try:
        with torch.no_grad():
            return vit(th)
    finally:
        R.set_bf16_emulation(False)


f32 = feats(False)
rel = lambda a: ((a - f32).norm() / f32.norm()).item()  # noqa: E731
print(f"all bf16 sites: {rel(feats(True)):.3e}")
sites = ["patch", "patch_w", "ln1", "ln1_w", "qkv", "p", "attn_out", "attn_out_w", "ln2",
         "ln2_w", "gelu", "gelu_w"]
for s in sites:
    print(f"  exact {s:12s}: {rel(feats(True, [s])):.3e}")
print(f"  exact all weights: {rel(feats(True, [s for s in sites if s.endswith('_w')])):.3e}")
print(f"  exact all activations: {rel(feats(True, [s for s in sites if not s.endswith('_w')])):.3e}")
