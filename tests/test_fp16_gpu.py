"""fp16-operand kernels of the "parity" precision mode's ViT forward (dfu_gemm operand_type 1,
dfu_attention_fwd_f16, dfu_layernorm_fwd_h16, dfu_cast_rows_f16, FusedAdamW's fp16 shadow)
against plain PyTorch fp32/fp64 on the same fp16-rounded operands: the kernels must add nothing
beyond fp32 accumulation to the operands' own fp16 rounding."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
F16 = torch.float16


def _ops():
    from dfu_hip import _lib as L
    from dfu_hip import ops
    return L, ops


@pytest.mark.parametrize("M,N,K,tile", [(12608, 2304, 768, 8), (12608, 768, 3072, 9),
                                        (1000, 520, 200, 8), (257, 264, 64, 8)])
def test_f16_gemm_f32_and_resid_epilogues(M, N, K, tile):
    L, ops = _ops()
    torch.manual_seed(1)
    A = (torch.randn(M, K, device=DEV) * 0.5).to(F16)
    B = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(F16)
    bias = torch.randn(N, device=DEV)
    res = torch.randn(M, N, device=DEV)
    ref = A.double() @ B.double().T + bias.double()
    C = torch.empty(M, N, device=DEV)
    if tile == 8:
        ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_F32, bias=bias, tile=tile,
                 operand_type=L.OPERAND_F16)
        assert ((C.double() - ref).abs().max() / ref.abs().max()).item() < 1e-5
    ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_F32_RESID, bias=bias, aux=res, ldaux=N,
             tile=tile, operand_type=L.OPERAND_F16)
    ref2 = ref + res.double()
    assert ((C.double() - ref2).abs().max() / ref2.abs().max()).item() < 1e-5
    with pytest.raises(L.DfuError):  # fp16 operands exist on the persistent tiles only
        ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_F32_RESID, bias=bias, aux=res,
                 ldaux=N, tile=1, operand_type=L.OPERAND_F16)


@pytest.mark.parametrize("M,N,K", [(12608, 2304, 768), (333, 264, 128)])
def test_f16_dual_epilogue(M, N, K):
    """qkv: fp16 C (the attention's operand) and its bf16 copy (the backward's) of the same
    fp32 value, each rounded once."""
    L, ops = _ops()
    torch.manual_seed(2)
    A = torch.randn(M, K, device=DEV).to(F16)
    B = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(F16)
    bias = torch.randn(N, device=DEV)
    C = torch.empty(M, N, dtype=F16, device=DEV)
    Cb = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_F16_DUAL, bias=bias, aux_out=Cb,
             ldaux_out=N, tile=8, operand_type=L.OPERAND_F16)
    ref = A.float() @ B.float().T + bias
    assert ((C.double() - ref.double()).abs() <= ref.double().abs() * 2.0 ** -10 + 1e-4).all()
    assert ((Cb.double() - ref.double()).abs() <= ref.double().abs() * 2.0 ** -7 + 1e-4).all()
    C1 = torch.empty_like(C)  # the bf16 copy is optional (the parity forward's qkv)
    ops.gemm(M, N, K, A, K, B, K, C1, N, epilogue=L.EPI_F16_DUAL, bias=bias, tile=8,
             operand_type=L.OPERAND_F16)
    assert torch.equal(C1, C)


@pytest.mark.parametrize("M,N,K", [(12608, 3072, 768), (1000, 520, 200)])
def test_f16_gelu_epilogue(M, N, K):
    """fc1 + GELU: [fp16 gelu | bf16 gelu] and bf16 gelu'(pre) from one fp32 pre-activation."""
    L, ops = _ops()
    torch.manual_seed(3)
    A = (torch.randn(M, K, device=DEV) * 0.5).to(F16)
    B = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(F16)
    bias = torch.randn(N, device=DEV)
    h2 = torch.empty(M, 2 * N, dtype=torch.bfloat16, device=DEV)
    dg = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.gemm(M, N, K, A, K, B, K, h2, 2 * N, epilogue=L.EPI_F16_GELU, bias=bias, aux_out=dg,
             ldaux_out=N, tile=8, operand_type=L.OPERAND_F16)
    pre = A.double() @ B.double().T + bias.double()
    g = torch.nn.functional.gelu(pre)
    h16 = h2[:, :N].contiguous().view(F16).double()
    hb = h2[:, N:].double()
    assert ((h16 - g).abs() <= g.abs() * 2.0 ** -10 + 1e-5).all()
    assert ((hb - g).abs() <= g.abs() * 2.0 ** -7 + 1e-5).all()
    dref = 0.5 * torch.erfc(-pre / math.sqrt(2)) + pre * torch.exp(-0.5 * pre * pre) / math.sqrt(2 * math.pi)
    assert ((dg.double() - dref).abs() <= 2.0 ** -7 * dref.abs() + 1e-5).all()


@pytest.mark.parametrize("N", [197, 50, 1])
def test_attention_fwd_f16_matches_sdpa(N):
    """fp16 attention vs fp64 SDPA on the same fp16 q, k, v: P rounded to fp16 and fp32
    accumulation (~2^-11 relative), the bf16 o copy is the same value rounded to bf16."""
    L, ops = _ops()
    torch.manual_seed(4)
    B, H, dh = 3, 12, 64
    D = H * dh
    qkv = (torch.randn(B * N, 3 * D, device=DEV) * 2).to(F16)
    o16, ob, lse = ops.attention_fwd_f16(qkv, B, N, H, dh, dh ** -0.5)
    q, k, v = qkv.double().view(B, N, 3, H, dh).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * dh ** -0.5
    ref = (s.softmax(-1) @ v).permute(0, 2, 1, 3).reshape(B * N, D)
    err = (o16.double() - ref).abs().max().item()
    print(f"\n[attn f16 N={N}] max abs err {err:.2e} (max |o| {ref.abs().max().item():.2f})")
    assert err < 2.0 ** -9 * ref.abs().max().item()
    assert ((ob.double() - o16.double()).abs() <= o16.double().abs() * 2.0 ** -7 + 1e-3).all()
    lref = torch.logsumexp(s, -1).reshape(B * H, N)
    assert torch.allclose(lse[:, :N].double(), lref, rtol=2.0 ** -14, atol=1e-5)


@pytest.mark.parametrize("N", [197, 50])
def test_attention_bwd_reads_fp16_qkv(N):
    """dfu_attention_bwd_qkv16 (the parity forward saves qkv in fp16 only) equals the bf16
    backward on bf16(qkv16): the kernel rounds while staging exactly as the cast does."""
    L, ops = _ops()
    torch.manual_seed(8)
    B, H, dh = 4, 12, 64
    D = H * dh
    q16 = (torch.randn(B * N, 3 * D, device=DEV) * 2).to(F16)
    qb = q16.to(torch.bfloat16)
    o, lse = ops.attention_fwd(qb, B, N, H, dh, dh ** -0.5)
    do = (torch.randn(B * N, D, device=DEV) * 0.1).to(torch.bfloat16)
    d16 = ops.attention_bwd(q16, o, do, lse, B, N, H, dh, dh ** -0.5)
    db = ops.attention_bwd(qb, o, do, lse, B, N, H, dh, dh ** -0.5)
    assert d16.dtype == torch.bfloat16 and torch.equal(d16, db)


def test_layernorm_h16_and_cast_f16():
    L, ops = _ops()
    torch.manual_seed(5)
    rows, D = 1000, 768
    x = torch.randn(rows, D, device=DEV) * 2 + 0.5
    g = torch.randn(D, device=DEV)
    b = torch.randn(D, device=DEV)
    o16 = torch.empty(rows, D, dtype=F16, device=DEV)
    ob = torch.empty(rows, D, dtype=torch.bfloat16, device=DEV)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    ops.layernorm_fwd_h16(x, D, rows, D, g, b, 1e-6, o16, ob, mean, rstd)
    ref = torch.nn.functional.layer_norm(x.double(), (D,), g.double(), b.double(), 1e-6)
    assert torch.equal(o16, ref.float().to(F16)) or \
        ((o16.double() - ref).abs() <= ref.abs() * 2.0 ** -10 + 1e-6).all()
    assert ((ob.double() - ref).abs() <= ref.abs() * 2.0 ** -7 + 1e-6).all()
    assert torch.allclose(mean.double(), x.double().mean(1), atol=1e-5)
    w = torch.randn(300, 77, device=DEV)
    assert torch.equal(ops.cast_rows_f16(w), w.to(F16))
    pad = ops.cast_rows_f16(w, ld_out=80)
    assert torch.equal(pad[:, :77], w.to(F16)) and torch.all(pad[:, 77:] == 0)


def test_adamw_keeps_the_fp16_shadow_current():
    """FusedAdamW's fp16 shadow (enabled by the first fp16-stage weight request) equals
    fp16(parameter) after every step, as the bf16 shadow equals bf16(parameter)."""
    from dfu_hip import functional as Fn
    from dfu_hip.optim import FusedAdamW
    torch.manual_seed(6)
    lin = torch.nn.Linear(768, 3072).to(DEV)
    opt = FusedAdamW(lin.parameters(), lr=1e-2, weight_decay=1e-4)
    w16 = Fn.weight_f16_rows(lin.weight)
    assert w16.dtype == F16 and torch.equal(w16, lin.weight.detach().to(F16))
    for _ in range(3):
        opt.zero_grad()
        lin.weight.grad.copy_(torch.randn_like(lin.weight))
        lin.bias.grad.copy_(torch.randn_like(lin.bias))
        opt.step()
    torch.cuda.synchronize()
    assert torch.equal(Fn.weight_f16_rows(lin.weight), lin.weight.detach().to(F16))
    assert torch.equal(lin.bias._dfu_shadow16.view(-1), lin.bias.detach().to(F16))
    with torch.no_grad():  # an outside edit is re-cast on the next request
        lin.weight.mul_(0.5)
    assert torch.equal(Fn.weight_f16_rows(lin.weight), lin.weight.detach().to(F16))


@pytest.mark.parametrize("gain", [1.0, 16.0, 128.0])
def test_fp16_vit_forward_range_at_trained_weight_scales(gain):
    """the parity mode's fp16 ViT forward saturates above 65504 (and loses bits
    below 6.1e-5), and the per-stage study that chose it used random-init weights only (DESIGN
    §4).  Trained ViT-B LayerNorm gains and activations sit well above the random init's; here
    every LayerNorm's weight and bias are scaled by `gain` and the qkv / fc1 weights that read
    its output by 1 / gain -- the same function, with the fp16 LayerNorm outputs `gain` times
    larger (up to ~1e3) and the fp16 weights `gain` times smaller (down to ~1e-4).  The fp16
    fusion-feature forward must stay finite and within fp16's own error of the bf16x3 forward.
    (Scaling the gains alone makes the random-init attention chaotic: every precision then
    diverges from every other, so that is not a range test.)"""
    from dfu_hip import functional as Fn
    from models.vit import VisionTransformer
    from oracle import torch_ref as R
    torch.manual_seed(2)
    v = VisionTransformer(num_classes=0).to(DEV).train()
    with torch.no_grad():
        for blk in v.blocks:
            for ln, lin in ((blk.norm1, blk.attn.qkv), (blk.norm2, blk.mlp.fc1)):
                ln.weight.mul_(gain)
                ln.bias.add_(0.01).mul_(gain)  # (nonzero biases: timm's are, once trained)
                lin.weight.div_(gain)
    _, th, _ = R.synthetic_batch(8, seed=3)
    th = th.to(DEV)
    with torch.no_grad():
        with Fn.precision("parity"):  # the class default: fp16 Blocks (a fusion feature extractor)
            f16 = v(th).float()
        with Fn.precision("bf16x3"):
            f32 = v(th).float()
    assert torch.isfinite(f16).all(), f"fp16 forward overflowed at gain {gain}"
    rel = ((f16 - f32).norm() / f32.norm()).item()
    print(f"\n[fp16 ViT, LayerNorm x {gain}, qkv / fc1 weights / {gain}] features rel err vs "
          f"bf16x3 {rel:.2e}")
    assert rel < 5e-3
