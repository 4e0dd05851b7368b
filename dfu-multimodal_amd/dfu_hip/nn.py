"""HIP-backed nn.Modules.

Each class subclasses its torch.nn counterpart so that parameters, buffers, initialisation,
``extra_repr`` and state_dict keys are exactly those of torchvision / timm / torch.nn (the
reference's loaders remap prefixes and call load_state_dict(strict=False),
extended_metrics.py:40-92).  Only ``forward`` differs: it runs libdfu_hip kernels.
"""
import itertools
import os

import torch
import torch.distributed as dist
import torch.nn as tnn

from . import _lib as L
from . import functional as Fn
from . import ops


class Conv2d(tnn.Conv2d):
    """Standalone convolution (bias-free, groups=1, dilation=1).  Inside ResNet the
    convolutions run fused with their BatchNorm (functional.BottleneckFn).  NHWC implicit GEMM
    when the input channels are a multiple of 64 (or a 1x1 stride-1 conv); otherwise, for
    weights stored OIHW (channels not a multiple of 8: an image stem's 1 or 3), an explicit
    im2col + GEMM as the ResNet stem runs (functional.StemFn)."""

    def forward(self, x):
        if self.bias is not None or self.groups != 1 or self.dilation != (1, 1):
            raise NotImplementedError("dfu_hip.nn.Conv2d: bias/groups/dilation unsupported")
        C = x.shape[1]
        R, S = self.kernel_size
        plain = R == 1 and S == 1 and self.stride == (1, 1) and self.padding == (0, 0)
        if C % 64 != 0 and not plain:
            if Fn._krsc_strided(self.weight):
                raise NotImplementedError(
                    "dfu_hip.nn.Conv2d: a channels-last (FusedAdamW) weight needs C % 64 == 0")
            return Conv2dIm2colFn.apply(x, self.weight, self)
        return Conv2dFn.apply(x, self.weight, self)


class Conv2dIm2colFn(torch.autograd.Function):
    """Explicit im2col (bf16 [M][Kp], K = C*R*S padded to 16, (c, r, s) order as OIHW) + GEMM;
    backward: weight gradient over the same columns, input gradient as fp32 dcol = dY W and its
    col2im adjoint."""

    @staticmethod
    def forward(ctx, x, w, mod):
        B, C, H, W = x.shape
        R, S = mod.kernel_size
        st, pad = mod.stride, mod.padding
        if st[0] != st[1] or pad[0] != pad[1]:
            raise NotImplementedError("dfu_hip.nn.Conv2d: square stride/padding only")
        Kp = ((C * R * S + 15) // 16) * 16
        xf = x.detach().float() if x.dtype != torch.float32 else x.detach()
        col, P, Q = ops.im2col_f32(xf, R, S, st[0], pad[0], Kp)
        wb = Fn.weight_bf16_rows(w, ld=Kp)
        Cout, M = w.shape[0], B * P * Q
        y = torch.empty((M, Cout), dtype=torch.bfloat16, device=x.device)
        ops.gemm(M, Cout, Kp, col, Kp, wb, Kp, y, Cout, epilogue=L.EPI_BF16)
        ctx.mod, ctx.dims, ctx.xdtype = mod, (B, C, H, W, P, Q, Kp, R, S, st[0], pad[0]), x.dtype
        ctx.save_for_backward(col, wb)
        return Fn.from_rows(y, B, P, Q, Cout)

    @staticmethod
    def backward(ctx, gy):
        col, wb = ctx.saved_tensors
        B, C, H, W, P, Q, Kp, R, S, st, pad = ctx.dims
        mod = ctx.mod
        Cout, M, K = wb.shape[0], B * P * Q, C * R * S
        dy = Fn.rows_view(Fn.nhwc_bf16(gy))
        if Fn._wants(mod.weight):
            ops.gemm(Cout, K, M, dy, Cout, col, Kp, Fn.grad_buffer(mod.weight).view(Cout, K), K,
                     a_mode=L.OPND_MNMAJOR, b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC)
            Fn.grads_done(mod.weight)
        dx = None
        if ctx.needs_input_grad[0]:
            dcol = torch.empty((M, Kp), dtype=torch.float32, device=dy.device)
            ops.gemm(M, Kp, Cout, dy, Cout, wb, Kp, dcol, Kp, b_mode=L.OPND_MNMAJOR,
                     epilogue=L.EPI_F32)
            dx = ops.col2im_f32(dcol, B, C, H, W, R, S, st, pad, P, Q, Kp)
            if ctx.xdtype != torch.float32:
                dx = dx.to(ctx.xdtype)
        return dx, None, None


class BatchNorm2d(tnn.BatchNorm2d):
    """torch.nn.BatchNorm2d.  Inside ResNet blocks the normalisation runs fused with the
    producing convolution (statistics from its GEMM epilogue, functional._BN); standalone, the
    tile statistics come from the stored input (dfu_bn_tile_stats) and the same finalize /
    apply / backward kernels run.  Output: bf16 channels_last."""

    def forward(self, x):
        return BatchNorm2dFn.apply(x, self.weight, self.bias, self)


class BatchNorm2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, mod):
        x = Fn.nhwc_bf16(x.detach())
        B, C, H, W = x.shape
        cv = C // 8  # 8-channel vectors; the backward reduce spreads min(cv, 64) over a block
        if C % 8 != 0 or (cv < 64 and cv & (cv - 1)) or (cv >= 64 and cv % 64):
            raise NotImplementedError("dfu_hip.nn.BatchNorm2d: channels must be 8, 16, 32, 64, "
                                      "128, 256 or a multiple of 512")
        M = B * H * W
        xr = Fn.rows_view(x)
        st = Fn._BN(mod, M, C, x.device)
        st.forward_coeffs(ops.bn_tile_stats(xr, M, C) if st.training else None)
        out = torch.empty((M, C), dtype=torch.bfloat16, device=x.device)
        ops.bn_apply(xr, st.scale, st.shift, None, 0, out, M, C)
        ctx.st = st
        ctx.save_for_backward(xr)
        return Fn.from_rows(out, B, H, W, C)

    @staticmethod
    def backward(ctx, gy):
        (xr,) = ctx.saved_tensors
        M, C = xr.shape
        g = Fn.rows_view(Fn.nhwc_bf16(gy))
        dx = torch.empty_like(xr)
        ctx.st.backward(g, xr, None, False, dx, None)
        B, _, H, W = gy.shape
        return Fn.from_rows(dx, B, H, W, C), None, None, None


class ReLU(tnn.ReLU):
    def forward(self, x):
        return Fn.ReLUFn.apply(x)


class MaxPool2d(tnn.MaxPool2d):
    """3x3/s2/p1 max pool on bf16 channels_last input (fused into StemFn inside ResNet)."""

    def forward(self, x):
        return MaxPoolFn.apply(x)


class MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = Fn.nhwc_bf16(x.detach())
        B, C, H, W = x.shape
        y, am, P, Q = ops.maxpool_fwd(Fn.rows_view(x), B, H, W, C)
        ctx.dims = (B, H, W, C, P, Q)
        ctx.save_for_backward(am)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, g):
        (am,) = ctx.saved_tensors
        B, H, W, C, P, Q = ctx.dims
        dx = ops.maxpool_bwd(Fn.rows_view(Fn.nhwc_bf16(g)), am, B, H, W, C, P, Q)
        return dx.permute(0, 3, 1, 2)


class AdaptiveAvgPool2d(tnn.AdaptiveAvgPool2d):
    def forward(self, x):
        if tuple(self.output_size) not in ((1, 1),) and self.output_size != 1:
            raise NotImplementedError("dfu_hip AdaptiveAvgPool2d: output size 1 only")
        return Fn.AvgPoolFn.apply(x)


class Linear(tnn.Linear):
    def forward(self, x):
        return Fn.LinearFn.apply(x, self.weight, self.bias, False)


class LayerNorm(tnn.LayerNorm):
    """fp32 LayerNorm over the last dim (the ViT blocks use it fused inside ViTBlockFn)."""

    def forward(self, x):
        return LayerNormFn.apply(x, self.weight, self.bias, self)


class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, mod):
        D = x.shape[-1]
        x2 = x.detach().float().reshape(-1, D).contiguous()
        rows = x2.shape[0]
        out = torch.empty_like(x2)
        mean = torch.empty((rows,), dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        ops.layernorm_fwd(x2, D, rows, D, mod.weight, mod.bias, mod.eps, out, D, False, mean, rstd)
        ctx.mod = mod
        ctx.shape = x.shape
        ctx.save_for_backward(x2, mean, rstd)
        return out.view(x.shape)

    @staticmethod
    def backward(ctx, g):
        x2, mean, rstd = ctx.saved_tensors
        mod = ctx.mod
        rows, D = x2.shape
        gx = torch.empty_like(x2)
        ops.zero_(gx)
        ops.layernorm_bwd(g.reshape(rows, D).float().contiguous(), D, False, x2, D, mean, rstd,
                          mod.weight, rows, D, gx, D, None,
                          Fn.grad_buffer(mod.weight) if Fn._wants(mod.weight) else None,
                          Fn.grad_buffer(mod.bias) if Fn._wants(mod.bias) else None)
        Fn.grads_done(mod.weight, mod.bias)
        return gx.view(ctx.shape), None, None, None


_M64 = (1 << 64) - 1
_dropout_instances = itertools.count()


def _splitmix64(z):
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _rank():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank()
    return int(os.environ.get("RANK", "0"))


def dropout_seed(instance, rank=None, base=None):
    """64-bit key of one Dropout instance's mask stream: torch.initial_seed(), the instance's
    creation index and the data-parallel rank, mixed by splitmix64.  The kernel's counter is
    z = seed + golden * (offset + i), so distinct well-mixed keys give unrelated streams (two
    layers of one head, or two ranks, never replay each other's masks)."""
    base = int(torch.initial_seed()) if base is None else int(base)
    rank = _rank() if rank is None else int(rank)
    return _splitmix64(_splitmix64(_splitmix64(base & _M64) ^ instance) ^ rank)


class Dropout(tnn.Dropout):
    """Inverted dropout with a counter-based device RNG (graph-replay safe).  Each instance
    draws its own stream (dropout_seed: torch seed x instance index x DP rank)."""

    def __init__(self, p=0.5, inplace=False):
        super().__init__(p, inplace)
        self.seed = dropout_seed(next(_dropout_instances))
        self.register_buffer("rng_offset", torch.zeros((), dtype=torch.int64), persistent=False)

    def forward(self, x):
        if not self.training or self.p == 0.0:
            return x
        if self.p >= 1.0:
            return x * 0.0
        return Fn.DropoutFn.apply(x, float(self.p), self.seed, self.rng_offset)


class CrossEntropyLoss(tnn.CrossEntropyLoss):
    """nn.CrossEntropyLoss(weight=w), mean reduction (train_multimodal_fusion.py:342-346)."""

    def forward(self, logits, target):
        if self.reduction != "mean" or self.label_smoothing != 0.0:
            raise NotImplementedError("dfu_hip CrossEntropyLoss: mean reduction, no smoothing")
        return Fn.CrossEntropyFn.apply(logits, target, self.weight)


Identity = tnn.Identity
Sequential = tnn.Sequential
