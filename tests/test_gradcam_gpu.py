"""Grad-CAM (BASELINE.json config C5; grad_cam_visualization.py:327-429, 561-632) on the MI355X
path against the CPU oracle: the stems' input-gradient kernels, the CAM / saliency kernels, and
whole-model maps through models.gradcam.GradCAM with the reference's hook protocol."""
import copy
import math

import pytest
import torch
import torch.nn.functional as F

from dfu_hip import ops
from oracle import gradcam_ref as G
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_col2im_and_unpatchify_are_adjoints():
    g = torch.Generator().manual_seed(3)
    B, C, H, W, R_, st, pad = 2, 3, 37, 29, 7, 2, 3
    P, Q = (H + 2 * pad - R_) // st + 1, (W + 2 * pad - R_) // st + 1
    Kp = 160
    dcol = torch.randn(B * P * Q, Kp, generator=g)
    ref = F.fold(dcol[:, :C * R_ * R_].view(B, P * Q, -1).transpose(1, 2), (H, W), (R_, R_),
                 padding=pad, stride=st)
    dx = ops.col2im_f32(dcol.to(DEV), B, C, H, W, R_, R_, st, pad, P, Q, Kp).cpu()
    assert (dx - ref).abs().max().item() < 1e-4
    ps = 16
    x = torch.randn(B, C, 64, 48, generator=g)
    patches = x.unfold(2, ps, ps).unfold(3, ps, ps).permute(0, 2, 3, 1, 4, 5).reshape(-1, C * ps * ps)
    back = ops.unpatchify_f32(patches.contiguous().to(DEV), B, C, 64, 48, ps).cpu()
    assert torch.equal(back, x)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("channels_last", [True, False])
@pytest.mark.parametrize("cg", [2048, 512])  # 512: the Bottleneck hook case (:418-422)
def test_gradcam_and_saliency_kernels(dtype, channels_last, cg):
    g = torch.Generator().manual_seed(5)
    B, C, h, w = 3, 2048, 7, 7
    act = torch.randn(B, C, h, w, generator=g).relu().to(dtype)
    grad = (torch.randn(B, cg, h, w, generator=g) * 1e-3).to(dtype)
    if channels_last:
        act = act.contiguous(memory_format=torch.channels_last)
        grad = grad.contiguous(memory_format=torch.channels_last)
    cam = ops.gradcam(act.to(DEV), grad.to(DEV)).cpu()
    wts = grad.float().mean(dim=(2, 3))
    ref = F.relu((wts[:, :, None, None] * act[:, :cg].float()).sum(1))
    ref = ref / ref.amax(dim=(1, 2), keepdim=True).clamp_min(1e-30)
    assert (cam - ref).abs().max().item() < 1e-4
    dx = torch.randn(B, 3, 224, 224, generator=g)
    sal = ops.saliency(dx.to(DEV)).cpu()
    s = dx.abs().mean(1)
    assert (sal - s / s.amax(dim=(1, 2), keepdim=True)).abs().max().item() < 1e-5


def _pair(zero_init_residual=True):
    from models.fusion import MultimodalFusionModel
    torch.manual_seed(0)
    ref = R.MultimodalFusionModel(num_classes=2, dropout=0.7,
                                  zero_init_residual=zero_init_residual)
    gen = torch.Generator().manual_seed(9)
    with torch.no_grad():  # non-trivial running statistics (Grad-CAM runs the model in eval mode)
        for name, buf in ref.named_buffers():
            if name.endswith("running_mean"):
                buf.copy_(torch.randn(buf.shape, generator=gen) * 0.1)
            elif name.endswith("running_var"):
                buf.copy_(torch.rand(buf.shape, generator=gen) * 1.5 + 0.5)
    hip = MultimodalFusionModel(num_classes=2, dropout=0.7)
    hip.load_state_dict(ref.state_dict(), strict=True)
    return ref, hip.to(DEV)


def _corr(a, b):
    a, b = a.flatten() - a.mean(), b.flatten() - b.mean()
    return float((a @ b) / (a.norm() * b.norm() + 1e-30))


def _input_grad(enc, x):
    x = x.clone().requires_grad_(True)
    enc(x)[:, 0].sum().backward()
    return x.grad.float().cpu()


def _rel(a, b):
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("mode", ["parity", "bf16"])
def test_input_gradients_match_oracle(mode):
    """The stems' new input gradients: d(sum_b out[b, 0]) / d input for both encoders in eval
    mode (relative L2 error).  In the bf16 mode the ResNet is held to the bf16-rounded oracle
    (rounding where the HIP path stores bf16): against the fp32 oracle ~0.1% of the ReLU masks
    flip sign under bf16 storage, and a flipped mask moves its whole gradient element, so the
    fp32-vs-bf16 ORACLES already differ by ~10% on this sparse (one-output-channel) gradient;
    measured HIP vs the bf16 oracle: 0.17%.  In the default "parity" mode the forward (and so
    every ReLU mask) is fp32-accurate and the ResNet is held to the fp32 oracle.  The ViT (GELU,
    no hard masks) is held to the fp32 oracle in both."""
    from dfu_hip import functional as Fn
    ref, hip = _pair()
    rgb, th, _ = R.synthetic_batch(2, seed=21)
    hip.eval()
    with Fn.precision(mode):
        gh = _input_grad(hip.resnet, rgb.to(DEV))
    try:
        R.set_bf16_emulation(True)
        g_bf = _input_grad(copy.deepcopy(ref.resnet).eval(), rgb)
    finally:
        R.set_bf16_emulation(False)
    g_fp = _input_grad(copy.deepcopy(ref.resnet).eval(), rgb)
    assert torch.isfinite(gh).all()
    print(f"\n[{mode}] resnet input grad: rel vs bf16 oracle {_rel(gh, g_bf):.3e}, vs fp32 "
          f"oracle {_rel(gh, g_fp):.3e} (corr {_corr(gh, g_fp):.4f})")
    if mode == "bf16":
        assert _rel(gh, g_bf) < 0.02, _rel(gh, g_bf)
        assert _rel(gh, g_fp) < 0.2 and _corr(gh, g_fp) > 0.98
    else:
        assert _rel(gh, g_fp) < 0.05 and _corr(gh, g_fp) > 0.998, _rel(gh, g_fp)
    with Fn.precision(mode):
        gh = _input_grad(hip.vit, th.to(DEV))
    g_fp = _input_grad(copy.deepcopy(ref.vit).eval(), th)
    print(f"[{mode}] vit input grad: rel vs fp32 oracle {_rel(gh, g_fp):.3e}")
    assert torch.isfinite(gh).all() and _rel(gh, g_fp) < 0.05, _rel(gh, g_fp)


@pytest.mark.parametrize("B,mode", [(3, "bf16"), (32, "bf16"), (32, "parity")])
def test_gradcam_maps_match_reference_restatement(B, mode):
    """models.gradcam.GradCAM (batched, HIP) vs the oracle's restatement of the reference's
    GradCAM run image by image (bs=1, as grad_cam_visualization.py:686): the RGB 7x7 CAM from the
    hooked 'layer4.2.relu' output and the thermal input saliency from the 'blocks' fallback.
    B = 32 is BASELINE config C5's batch; "parity" is the library's default mode (the forward
    fp32-accurate, so its maps are held to the fp32 oracle as tightly as the bf16 mode's are to
    the bf16-rounded one).  (zero_init_residual off: with bn3.weight = 0 the hooked conv1-ReLU
    gradient is exactly 0 and both maps are all-zero.)"""
    from dfu_hip import functional as Fn
    from models.gradcam import GradCAM
    Fn.set_precision(mode)  # (restored by conftest)
    ref, hip = _pair(zero_init_residual=False)
    rgb, th, _ = R.synthetic_batch(B, seed=31)
    cam_rgb = GradCAM(hip.resnet, ["layer4"])
    assert cam_rgb.target_name() == "layer4.2.relu"
    cams = cam_rgb.generate_cams(rgb.to(DEV)).cpu()
    assert cams.shape == (B, 7, 7)
    # the reference's hooks on a three-call `relu`: activation from the last call (the block
    # output), gradient from the first (conv1's 512-wide ReLU output)
    assert cam_rgb.activations["layer4.2.relu"].shape == (B, 2048, 7, 7)
    assert cam_rgb.gradients["layer4.2.relu"].shape == (B, 512, 7, 7)
    cam_th = GradCAM(hip.vit, ["blocks"])
    assert cam_th.target_name() == "blocks.11.drop_path2"
    sal = cam_th.generate_cams(th.to(DEV)).cpu()
    assert sal.shape == (B, 224, 224)
    oracle_cam = G.GradCAMRef(copy.deepcopy(ref.resnet), ["layer4"])
    rvit = copy.deepcopy(ref.vit)
    for b in range(B):
        try:  # bf16-rounded oracle (rounding where the HIP path stores bf16): the tight check
            R.set_bf16_emulation(True)
            rc_bf = oracle_cam.generate_cam(rgb[b:b + 1])
        finally:
            R.set_bf16_emulation(False)
        assert oracle_cam.gradients["layer4.2.relu"].shape == (1, 512, 7, 7)
        rc = oracle_cam.generate_cam(rgb[b:b + 1])
        assert rc.shape == (7, 7) and rc.max() > 0
        # (the HIP path also carries the gradients in bf16; the oracle's stay fp32)
        d_bf, d_fp = (cams[b] - rc_bf).abs().max().item(), (cams[b] - rc).abs().max().item()
        if b == 0:
            print(f"\n[{mode} B={B}] CAM 0: max abs vs bf16 oracle {d_bf:.3e}, vs fp32 oracle "
                  f"{d_fp:.3e} (corr {_corr(cams[b], rc):.4f})")
        if mode == "bf16":
            assert d_bf < 0.06 and _corr(cams[b], rc_bf) > 0.99, (d_bf, _corr(cams[b], rc_bf))
            assert d_fp < 0.15 and _corr(cams[b], rc) > 0.97, (d_fp, _corr(cams[b], rc))
        else:
            assert d_fp < 0.06 and _corr(cams[b], rc) > 0.99, (d_fp, _corr(cams[b], rc))
        rs = G.saliency_ref(rvit, th[b:b + 1])
        assert _corr(sal[b], rs) > 0.95, _corr(sal[b], rs)
        assert abs(sal[b].max().item() - 1.0) < 1e-6
    # the reference signature: (1, C, H, W) -> numpy map
    one = cam_rgb.generate_cam(rgb[:1].to(DEV))
    assert one.shape == (7, 7) and math.isclose(float(one.max()), 1.0, rel_tol=1e-6)


def test_gradcam_step_replays_from_a_hip_graph():
    """The C5 step (bench.py --config gradcam) captured into one HIP graph: the capture must
    succeed (every side / weight-gradient stream joined before it ends) and a replay must
    reproduce the eager maps."""
    from models.fusion import MultimodalFusionModel
    from models.gradcam import GradCAM
    torch.manual_seed(5)
    model = MultimodalFusionModel(num_classes=2, dropout=0.7).to(DEV).eval()
    rgb, th, _ = R.synthetic_batch(4, seed=41)
    rgb, th = rgb.to(DEV), th.to(DEV)
    cam_rgb, cam_th = GradCAM(model.resnet, ["layer4"]), GradCAM(model.vit, ["blocks"])
    outs = {}

    def step():
        with torch.no_grad():
            outs["pred"] = torch.softmax(model(rgb, th), dim=1).argmax(1)
        outs["cam"] = cam_rgb.generate_cams(rgb)
        outs["sal"] = cam_th.generate_cams(th)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ref = {k: v.clone() for k, v in outs.items()}
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    for k in outs:
        outs[k].zero_()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(outs["pred"], ref["pred"])
    assert torch.allclose(outs["cam"], ref["cam"], atol=1e-5)
    assert torch.allclose(outs["sal"], ref["sal"], atol=1e-5)
