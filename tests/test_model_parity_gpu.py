"""Whole-model parity on the GPU: the HIP fusion model vs the CPU oracle (oracle/torch_ref.py)
on the identical synthetic batch and weights (train-mode BN, dropout identity).

north_star: "logits match the reference CPU path within 1e-3 abs bf16 on identical synthetic
224x224 batches".  Measured at BASELINE config C3's size (B = 64), torchvision's default
ResNet initialisation, train-mode BatchNorm:

  * precision "bf16x3" (dfu_hip.functional.precision; csrc/precise.hip): the forward pass at
    fp32 accuracy on the same MFMA GEMMs (split-bf16 operands).  Asserted with the FIXED bar:
    max |logits(HIP) - logits(fp32 oracle)| <= 1e-3 (LOGIT_ATOL, train_multimodal_fusion.py:
    374-376), and the same for the loss.
  * precision "bf16" (the default, benchmarked mode): bf16 storage alone moves the logits of the
    fp32 oracle itself by 7.2e-2 at C3 with torchvision's default (zero_init_residual=False)
    initialisation -- the random-init ResNet amplifies rounding chaotically -- and
    by 2.4e-3 with zero_init_residual=True.  Held to FIXED bars: 0.1 at default init, 5e-3
    with zero-init residuals (both at B = 64).
  * gradients (the backward is bf16 in both modes): FIXED bars per parameter against the fp32
    oracle -- relative L2 error and cosine similarity -- so a wrong-sign or garbage gradient
    fails; the bf16-rounded oracle's own errors are recorded beside them.

Every measured delta is written to gpurun_out/parity_r10.json (DFU_PARITY_JSON overrides) and
committed as profiles/r10_parity.json.
"""
import copy
import json
import os

import pytest
import torch

from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
LOGIT_ATOL = 1e-3  # north_star: "logits match the reference CPU path within 1e-3 abs bf16"
# the headline ("parity") mode's own fixed bar: half the north-star bar, the margin its stage
# assignment was chosen for (profiles/r16b_precision_study.json, r17_precision_study.json: <= 5e-4 on every seed)
PARITY_ATOL = 5e-4
B_C3 = 64          # BASELINE.json C3: fusion bs=64
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PARITY_JSON = os.environ.get("DFU_PARITY_JSON",
                             os.path.join(REPO, "gpurun_out", "parity_r10.json"))


def _record(key, value):
    """Merge one measurement into the parity JSON (created on first use)."""
    os.makedirs(os.path.dirname(PARITY_JSON), exist_ok=True)
    data = {}
    if os.path.exists(PARITY_JSON):
        with open(PARITY_JSON) as f:
            data = json.load(f)
    data[key] = value
    with open(PARITY_JSON, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)


def _models(zero_init_residual=False, seed=0):
    from models.fusion import MultimodalFusionModel
    torch.manual_seed(seed)
    ref = R.MultimodalFusionModel(num_classes=2, dropout=0.0,
                                  zero_init_residual=zero_init_residual)
    hip = MultimodalFusionModel(num_classes=2, dropout=0.0)
    missing, unexpected = hip.load_state_dict(ref.state_dict(), strict=False)
    assert not unexpected and not missing, (missing, unexpected)
    return ref, hip.to(DEV)


def rel(a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp(min=1e-12)).item()


def _oracle(ref, rgb, th, y, w, emu, dev="cpu", backward=True):
    m = copy.deepcopy(ref).to(dev).train()
    R.set_bf16_emulation(emu)
    try:
        with torch.set_grad_enabled(backward):
            fr = m.resnet(rgb.to(dev))
            ft = m.vit(th.to(dev))
            out = m.fusion(fr, ft)
            loss = torch.nn.functional.cross_entropy(out, y.to(dev), weight=w.to(dev))
        if backward:
            loss.backward()
    finally:
        R.set_bf16_emulation(False)
    return dict(m=m, fr=fr.detach().cpu(), ft=ft.detach().cpu(), out=out.detach().cpu(),
                loss=loss.item())


def _hip(hip, rgb, th, y, w, precision="bf16"):
    from dfu_hip import functional as Fn
    from dfu_hip import nn as hnn
    hip.train()
    for p in hip.parameters():
        p.grad = None
    with Fn.precision(precision):
        fr = hip.resnet(rgb.to(DEV))
        ft = hip.vit(th.to(DEV))
        out = hip.fusion(fr, ft)
        loss = hnn.CrossEntropyLoss(weight=w.to(DEV))(out, y.to(DEV))
        loss.backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().cpu().clone() for n, p in hip.named_parameters()}
    return dict(fr=fr.detach().cpu(), ft=ft.detach().cpu(), out=out.detach().float().cpu(),
                loss=loss.item(), grads=grads)


def _maxd(a, b):
    return (a["out"] - b["out"]).abs().max().item()


@pytest.fixture(scope="module")
def c3():
    """C3 at B=64, default (torchvision) init: fp32 oracle (fwd+bwd), bf16-rounded oracle
    (fwd), HIP bf16x3 and HIP bf16 train steps on the identical batch and weights."""
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref, hip = _models()
    rgb, th, y = R.synthetic_batch(B_C3, seed=42)
    w = R.class_weights(y)
    res = dict(f32=_oracle(ref, rgb, th, y, w, False),
               emu=_oracle(ref, rgb, th, y, w, True),
               emu_gpu=_oracle(ref, rgb, th, y, w, True, dev=DEV, backward=False),
               x3=_hip(hip, rgb, th, y, w, "bf16x3"),
               parity=_hip(hip, rgb, th, y, w, "parity"),
               bf16=_hip(hip, rgb, th, y, w, "bf16"))
    return res


def test_state_dict_keys_match_reference_surface():
    ref, hip = _models()
    assert set(ref.state_dict().keys()) == set(hip.state_dict().keys())
    assert sum(p.numel() for p in hip.parameters()) == 110_750_018


def test_c3_logits_bf16x3_within_1e3_of_fp32_oracle(c3):
    """The north-star bar as written, at C3's batch: |logits - fp32 oracle| <= 1e-3 abs."""
    f32, h = c3["f32"], c3["x3"]
    d = _maxd(h, f32)
    dl = abs(h["loss"] - f32["loss"])
    print(f"\n[C3 B={B_C3} bf16x3] |logits|max={f32['out'].abs().max().item():.3e}  "
          f"max|d logits| vs fp32 oracle = {d:.3e} (bar {LOGIT_ATOL}); loss {h['loss']:.6f} vs "
          f"{f32['loss']:.6f}; rgb feat rel {rel(h['fr'], f32['fr']):.2e}, thermal feat rel "
          f"{rel(h['ft'], f32['ft']):.2e}")
    _record("c3_b64_bf16x3", {"max_abs_logits_vs_fp32_oracle": d, "abs_loss_vs_fp32_oracle": dl,
                              "rgb_feat_rel": rel(h["fr"], f32["fr"]),
                              "thermal_feat_rel": rel(h["ft"], f32["ft"]),
                              "max_abs_logit": f32["out"].abs().max().item(),
                              "bar": LOGIT_ATOL, "batch": B_C3, "init": "torchvision default"})
    assert d <= LOGIT_ATOL
    assert dl <= LOGIT_ATOL


def test_c3_logits_parity_mode_within_margin_of_fp32_oracle(c3):
    """The headline mode ("parity": ResNet forward bf16x3, ViT forward fp16, backward bf16) at
    C3's batch: |logits - fp32 oracle| <= 5e-4 (half north-star's 1e-3), loss likewise."""
    f32, h = c3["f32"], c3["parity"]
    d = _maxd(h, f32)
    dl = abs(h["loss"] - f32["loss"])
    print(f"\n[C3 B={B_C3} parity] max|d logits| vs fp32 oracle = {d:.3e} (bar {PARITY_ATOL}); "
          f"loss {h['loss']:.6f} vs {f32['loss']:.6f}; rgb feat rel {rel(h['fr'], f32['fr']):.2e},"
          f" thermal feat rel {rel(h['ft'], f32['ft']):.2e}")
    _record("c3_b64_parity", {"max_abs_logits_vs_fp32_oracle": d, "abs_loss_vs_fp32_oracle": dl,
                               "rgb_feat_rel": rel(h["fr"], f32["fr"]),
                               "thermal_feat_rel": rel(h["ft"], f32["ft"]),
                               "bar": PARITY_ATOL, "batch": B_C3})
    assert d <= PARITY_ATOL
    assert dl <= PARITY_ATOL


def test_c3_grads_parity_mode_vs_fp32_oracle(c3):
    """The headline mode's parameter gradients under the bf16x3 mode's fixed bars."""
    f32, h = c3["f32"], c3["parity"]
    errs = _grad_errors(h["grads"], f32["m"])
    med = errs[len(errs) // 2][0]
    _record("c3_b64_parity_grads", {"worst": [[n, e, c] for e, c, _, n in errs[:10]],
                                    "median": med, "min_cos": min(c for _, c, _, _ in errs)})
    for e, c, _, n in errs:
        assert e <= GRAD_REL_MAX and c >= GRAD_COS_MIN, (n, e, c)
    assert med <= GRAD_REL_MEDIAN, med


def _grad_errors(grads, ref_m, other_m=None):
    """[(rel L2 err, cosine, other's rel err, name)] per parameter with a non-zero reference
    gradient, worst first."""
    rp = dict(ref_m.named_parameters())
    ro = dict(other_m.named_parameters()) if other_m is not None else {}
    out = []
    for n, g in grads.items():
        r = rp[n].grad
        if r.norm().item() == 0.0:
            continue
        cos = torch.nn.functional.cosine_similarity(g.flatten().double(), r.flatten().double(),
                                                    dim=0).item()
        out.append((rel(g, r), cos, rel(ro[n].grad, r) if n in ro else None, n))
    return sorted(out, key=lambda t: t[0], reverse=True)


# fixed gradient bars (the backward is bf16): every parameter, and the median
# (round 5: tightened from 0.3 / 0.95; measured worst 0.186 / 0.983 bf16x3, 0.159 / 0.987 parity)
GRAD_REL_MAX, GRAD_COS_MIN, GRAD_REL_MEDIAN = 0.25, 0.975, 0.03


def test_c3_grads_bf16x3_vs_fp32_oracle(c3):
    """Parameter gradients of the bf16x3 step against the fp32 oracle at C3 (default init),
    FIXED bars: rel L2 <= 0.25 and cosine >= 0.975 for every parameter, median rel <= 0.03.
    (The bf16-rounded oracle itself misses these by far on the early BN parameters -- rel
    1.2-1.6: its forward is chaotic at this init -- which is why the forward is bf16x3 here.)"""
    f32, emu, h = c3["f32"], c3["emu"], c3["x3"]
    errs = _grad_errors(h["grads"], f32["m"], emu["m"])
    for e, c, b, n in errs[:6]:
        print(f"  grad vs fp32 oracle {n}: rel {e:.3e} cos {c:.5f} (bf16 oracle rel {b:.3e})")
    med = errs[len(errs) // 2][0]
    _record("c3_b64_bf16x3_grads", {"worst": [[n, e, c, b] for e, c, b, n in errs[:10]],
                                    "median": med, "min_cos": min(c for _, c, _, _ in errs),
                                    "bars": [GRAD_REL_MAX, GRAD_COS_MIN, GRAD_REL_MEDIAN],
                                    "columns": "param, HIP rel err, cosine, bf16 oracle rel err"})
    for e, c, b, n in errs:
        assert e <= GRAD_REL_MAX and c >= GRAD_COS_MIN, (n, e, c)
    assert med <= GRAD_REL_MEDIAN, med


def test_c3_logits_bf16_fixed_bar(c3):
    """Default bf16 precision at C3, default init: FIXED bar 0.1 against the fp32 oracle (the
    bf16-rounded oracle's own gap is 7.2e-2 here, see the module docstring); the
    bf16-rounded oracle's CPU-vs-GPU band is recorded beside it."""
    f32, emu, emu_gpu, h = c3["f32"], c3["emu"], c3["emu_gpu"], c3["bf16"]
    band = _maxd(emu_gpu, emu)
    d_emu, d_f32 = _maxd(h, emu), _maxd(h, f32)
    q_gap = max(_maxd(emu, f32), _maxd(emu_gpu, f32))
    print(f"\n[C3 B={B_C3} bf16] max|d logits| HIP vs bf16-rounded oracle {d_emu:.3e} (oracle "
          f"CPU-vs-GPU band {band:.3e}); HIP vs fp32 oracle {d_f32:.3e} (bf16 oracle vs fp32 "
          f"oracle {q_gap:.3e})")
    _record("c3_b64_bf16", {"max_abs_logits_vs_bf16_oracle": d_emu,
                            "max_abs_logits_vs_fp32_oracle": d_f32,
                            "oracle_bf16_cpu_vs_gpu_band": band,
                            "oracle_bf16_vs_fp32_gap": q_gap, "bar": 0.1})
    assert d_f32 <= 0.1


def test_c3_zero_init_residual_fixed_bars():
    """C3's batch (B = 64) with torchvision's zero_init_residual=True (the well-conditioned
    init): bf16x3 logits within 1e-3 of the fp32 oracle, bf16 logits within 5e-3 (the
    bf16-rounded oracle's own gap: 2.4e-3), and both modes' gradients under the fixed bars
    (bf16: rel <= 0.4, cosine >= 0.9, median <= 0.1 -- the bf16-rounded oracle's own worst is
    0.2 and median 0.05 here: the BN backward's mean subtraction amplifies bf16 rounding)."""
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref, hip = _models(zero_init_residual=True)
    rgb, th, y = R.synthetic_batch(B_C3, seed=42)
    w = R.class_weights(y)
    f32 = _oracle(ref, rgb, th, y, w, False)
    x3 = _hip(hip, rgb, th, y, w, "bf16x3")
    bf = _hip(hip, rgb, th, y, w, "bf16")
    d3, db = _maxd(x3, f32), _maxd(bf, f32)
    e3 = _grad_errors(x3["grads"], f32["m"])
    eb = _grad_errors(bf["grads"], f32["m"])
    print(f"\n[C3 B={B_C3} zero-init] logits vs fp32 oracle: bf16x3 {d3:.3e} (bar 1e-3), bf16 "
          f"{db:.3e} (bar 5e-3); grads worst rel bf16x3 {e3[0][0]:.3e} bf16 {eb[0][0]:.3e}")
    _record("c3_b64_zero_init", {"bf16x3_max_abs_logits_vs_fp32_oracle": d3,
                                 "bf16_max_abs_logits_vs_fp32_oracle": db,
                                 "bf16x3_grads_worst": [[n, e, c] for e, c, _, n in e3[:5]],
                                 "bf16_grads_worst": [[n, e, c] for e, c, _, n in eb[:5]],
                                 "bf16x3_grads_median": e3[len(e3) // 2][0],
                                 "bf16_grads_median": eb[len(eb) // 2][0]})
    assert d3 <= LOGIT_ATOL and db <= 5e-3
    for errs, rmax, cmin, med in ((e3, GRAD_REL_MAX, GRAD_COS_MIN, GRAD_REL_MEDIAN),
                                  (eb, 0.4, 0.9, 0.1)):
        for e, c, _, n in errs:
            assert e <= rmax and c >= cmin, (n, e, c)
        assert errs[len(errs) // 2][0] <= med


def test_well_conditioned_b8_grads_within_oracle_band():
    """torchvision zero_init_residual=True (every block starts as the identity), B=8, bf16:
    per-parameter gradients within the bf16 oracle's own band, BN running stats as torch."""
    B = 8
    ref, hip = _models(zero_init_residual=True)
    rgb, th, y = R.synthetic_batch(B, seed=42)
    w = R.class_weights(y)
    emu = _oracle(ref, rgb, th, y, w, True)
    emu_gpu = _oracle(ref, rgb, th, y, w, True, dev=DEV)
    f32 = _oracle(ref, rgb, th, y, w, False)
    h = _hip(hip, rgb, th, y, w)
    x3 = _hip(_models(zero_init_residual=True)[1], rgb, th, y, w, "bf16x3")
    print(f"\n[well-conditioned B={B}] bf16: vs bf16 oracle {_maxd(h, emu):.3e} (band "
          f"{_maxd(emu_gpu, emu):.3e}), vs fp32 oracle {_maxd(h, f32):.3e}; bf16x3 vs fp32 "
          f"oracle {_maxd(x3, f32):.3e}")
    _record("b8_zero_init", {"bf16_vs_bf16_oracle": _maxd(h, emu),
                             "bf16_vs_fp32_oracle": _maxd(h, f32),
                             "bf16x3_vs_fp32_oracle": _maxd(x3, f32),
                             "oracle_band": _maxd(emu_gpu, emu)})
    assert _maxd(x3, f32) <= LOGIT_ATOL
    rp = dict(emu["m"].named_parameters())
    rg = dict(emu_gpu["m"].named_parameters())
    worst = []
    for n, g in h["grads"].items():
        e, b = rel(g, rp[n].grad), rel(rg[n].grad, rp[n].grad)
        worst.append((e - 2 * b, e, b, n))
    worst.sort(reverse=True)
    for _, e, b, n in worst[:6]:
        print(f"  grad rel err vs bf16 oracle {n}: {e:.3e} (oracle band {b:.3e})")
    assert worst[0][0] <= 1e-2, worst[0]
    rb = dict(emu["m"].named_buffers())
    for n, b in hip.named_buffers():
        if n.endswith("num_batches_tracked"):
            assert b.item() == rb[n].item() == 1
        elif "running" in n:
            assert rel(b, rb[n]) < 2e-2, n


@pytest.mark.parametrize("B", [1, 3, 5])
def test_ragged_batches_parity_mode_vs_fp32_oracle(B):
    """Batches no tile divides (an epoch's last batch, Grad-CAM / TTA at bs = 1): the library
    default ("parity") train step at B = 1, 3, 5 against the fp32 oracle: logits within the
    parity margin, every parameter gradient under C3's fixed bars.  The class weights are fixed
    (B = 1 has one class)."""
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref, hip = _models(seed=B)
    rgb, th, y = R.synthetic_batch(B, seed=100 + B)
    w = torch.tensor([1.5, 0.75])
    f32 = _oracle(ref, rgb, th, y, w, False)
    h = _hip(hip, rgb, th, y, w, "parity")
    d = _maxd(h, f32)
    errs = _grad_errors(h["grads"], f32["m"])
    med = errs[len(errs) // 2][0]
    min_cos = min(c for _, c, _, _ in errs)
    print(f"\n[B={B} parity] max|d logits| {d:.3e}, loss {h['loss']:.6f} vs {f32['loss']:.6f}; "
          f"grads: median rel {med:.3e}, worst {errs[0][3]} rel {errs[0][0]:.3e}, "
          f"min cos {min_cos:.5f}")
    _record(f"ragged_b{B}_parity", {"max_abs_logits_vs_fp32_oracle": d, "grad_median_rel": med,
                                    "grad_worst": [errs[0][3], errs[0][0], errs[0][1]],
                                    "grad_min_cos": min_cos})
    assert d <= PARITY_ATOL
    assert abs(h["loss"] - f32["loss"]) <= PARITY_ATOL
    for g in h["grads"].values():
        assert torch.isfinite(g).all()
    # C3's fixed bars hold here too (measured: worst rel 0.13-0.15, min cos 0.989, median
    # 0.010-0.022 at B = 1 / 3 / 5)
    for e, c, _, n in errs:
        assert e <= GRAD_REL_MAX and c >= GRAD_COS_MIN, (n, e, c)
    assert med <= GRAD_REL_MEDIAN, med
