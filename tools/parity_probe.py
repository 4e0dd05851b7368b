"""Where does the HIP-vs-oracle logit gap come from?  (GPU box; diagnostic only.)

Runs the well-conditioned fusion model (zero_init_residual) at B=8 through the HIP path, the
fp32 CPU oracle and the bf16-rounded oracle (CPU and a second realisation on the GPU), then
attributes the logit error to the RGB and thermal features by swapping features into the fp32
head one branch at a time."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

from oracle import torch_ref as R  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
zi = "--default-init" not in sys.argv


def rel(a, b):
    return ((a.float().cpu() - b.float().cpu()).norm() / b.float().cpu().norm()).item()


def maxd(a, b):
    return (a.float().cpu() - b.float().cpu()).abs().max().item()


def oracle_feats(ref, rgb, th, emu, dev="cpu"):
    m = copy.deepcopy(ref).to(dev).train()
    R.set_bf16_emulation(emu)
    try:
        with torch.no_grad():
            fr = m.resnet(rgb.to(dev))
            ft = m.vit(th.to(dev))
    finally:
        R.set_bf16_emulation(False)
    return fr.cpu(), ft.cpu()


def main():
    from models.fusion import MultimodalFusionModel
    torch.manual_seed(0)
    ref = R.MultimodalFusionModel(num_classes=2, dropout=0.0, zero_init_residual=zi)
    hip = MultimodalFusionModel(num_classes=2, dropout=0.0)
    hip.load_state_dict(ref.state_dict(), strict=False)
    hip = hip.cuda().train()
    rgb, th, y = R.synthetic_batch(B, seed=42)
    with torch.no_grad():
        fr_h = hip.resnet(rgb.cuda()).float().cpu()
        ft_h = hip.vit(th.cuda()).float().cpu()
    fr_32, ft_32 = oracle_feats(ref, rgb, th, False)
    fr_e, ft_e = oracle_feats(ref, rgb, th, True)
    fr_g, ft_g = oracle_feats(ref, rgb, th, True, "cuda")
    head = copy.deepcopy(ref.fusion).eval()
    with torch.no_grad():
        L = lambda a, b: head(a, b)  # noqa: E731
        base = L(fr_32, ft_32)
        print(f"B={B} zero_init_residual={zi} |logits|max={base.abs().max().item():.3e}")
        for name, (fr, ft) in {"HIP": (fr_h, ft_h), "bf16 oracle CPU": (fr_e, ft_e),
                               "bf16 oracle GPU": (fr_g, ft_g)}.items():
            print(f"{name:16s}: rgb feat rel {rel(fr, fr_32):.3e}  thermal feat rel "
                  f"{rel(ft, ft_32):.3e} | logits vs fp32: both {maxd(L(fr, ft), base):.3e}  "
                  f"rgb-only {maxd(L(fr, ft_32), base):.3e}  thermal-only {maxd(L(fr_32, ft), base):.3e}")
        print(f"HIP vs bf16 oracle CPU: rgb {rel(fr_h, fr_e):.3e} thermal {rel(ft_h, ft_e):.3e} "
              f"logits {maxd(L(fr_h, ft_h), L(fr_e, ft_e)):.3e}")
        print(f"GPU vs CPU bf16 oracle: rgb {rel(fr_g, fr_e):.3e} thermal {rel(ft_g, ft_e):.3e} "
              f"logits {maxd(L(fr_g, ft_g), L(fr_e, ft_e)):.3e}")


if __name__ == "__main__":
    main()
