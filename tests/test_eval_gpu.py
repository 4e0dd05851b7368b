"""Evaluation / inference path (train_multimodal_fusion.py:398-425,
extended_metrics.py:581-642): model.eval() + torch.no_grad(), BatchNorm on running statistics,
dropout off, softmax[:, 1] as the ulcer probability — against the CPU oracle in eval mode on the
same weights and running statistics.  Running statistics must not change in eval mode."""
import copy

import pytest
import torch

from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pair():
    from models.fusion import MultimodalFusionModel
    torch.manual_seed(0)
    ref = R.MultimodalFusionModel(num_classes=2, dropout=0.7, zero_init_residual=True)
    g = torch.Generator().manual_seed(7)
    with torch.no_grad():  # non-trivial running statistics
        for name, buf in ref.named_buffers():
            if name.endswith("running_mean"):
                buf.copy_(torch.randn(buf.shape, generator=g) * 0.1)
            elif name.endswith("running_var"):
                buf.copy_(torch.rand(buf.shape, generator=g) * 1.5 + 0.5)
    hip = MultimodalFusionModel(num_classes=2, dropout=0.7)
    hip.load_state_dict(ref.state_dict(), strict=True)
    return ref, hip.to(DEV)


def test_eval_logits_and_probabilities():
    from dfu_hip import functional as Fn
    B = 8
    ref, hip = _pair()
    rgb, th, _ = R.synthetic_batch(B, seed=11)
    buffers_before = {k: v.clone() for k, v in hip.state_dict().items() if "running" in k or "num_batches" in k}
    hip.eval()
    with torch.no_grad():
        outp = hip(rgb.to(DEV), th.to(DEV)).float().cpu()  # the library default: "parity"
        with Fn.precision("bf16"):
            out = hip(rgb.to(DEV), th.to(DEV)).float().cpu()
    m = copy.deepcopy(ref).eval()
    with torch.no_grad():
        f32 = m(rgb, th)
        R.set_bf16_emulation(True)
        try:
            emu = m(rgb, th)
        finally:
            R.set_bf16_emulation(False)
    d_emu = (out - emu).abs().max().item()
    d_f32 = (out - f32).abs().max().item()
    gap = (emu - f32).abs().max().item()
    print(f"\n[eval B={B}] |logits|max={f32.abs().max().item():.3e}  HIP vs bf16 oracle {d_emu:.3e}, "
          f"HIP vs fp32 oracle {d_f32:.3e}, bf16 vs fp32 oracle {gap:.3e}")
    assert torch.isfinite(out).all()
    assert d_f32 <= 5e-3  # fixed bar for bf16 (the bf16-rounded oracle's own gap is ~2e-3)
    # the default "parity" mode under eval-mode BN: the 5e-4 margin
    dp = (outp - f32).abs().max().item()
    print(f"  parity (default) eval vs fp32 oracle {dp:.3e} (bar 5e-4)")
    assert dp <= 5e-4
    assert (torch.softmax(outp, 1)[:, 1] - torch.softmax(f32, 1)[:, 1]).abs().max().item() < 5e-4
    # the fp32-accurate forward: north_star's 1e-3, fixed
    with torch.no_grad(), Fn.precision("bf16x3"):
        out3 = hip(rgb.to(DEV), th.to(DEV)).float().cpu()
    d3 = (out3 - f32).abs().max().item()
    print(f"  bf16x3 eval vs fp32 oracle {d3:.3e} (bar 1e-3)")
    assert d3 <= 1e-3
    assert (torch.softmax(out3, 1)[:, 1] - torch.softmax(f32, 1)[:, 1]).abs().max().item() < 1e-3
    p_hip = torch.softmax(out, 1)[:, 1]
    p_ref = torch.softmax(f32, 1)[:, 1]
    assert (p_hip - p_ref).abs().max().item() < 1e-3
    assert torch.equal(out.argmax(1), f32.argmax(1)) or d_f32 > (f32[:, 1] - f32[:, 0]).abs().min()
    for k, v in hip.state_dict().items():
        if k in buffers_before:
            assert torch.equal(v, buffers_before[k]), f"{k} changed in eval mode"
    assert all(p.grad is None for p in hip.parameters())  # no_grad: no backward work
