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

from . import functional as Fn
from . import ops


class Conv2d(tnn.Conv2d):
    """Standalone NHWC implicit-GEMM convolution (bias-free, groups=1, dilation=1).
    Inside ResNet the convolutions run fused with their BatchNorm (functional.BottleneckFn)."""

    def forward(self, x):
        if self.bias is not None or self.groups != 1 or self.dilation != (1, 1):
            raise NotImplementedError("dfu_hip.nn.Conv2d: bias/groups/dilation unsupported")
        return Conv2dFn.apply(x, self.weight, self)


class Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, mod):
        x = Fn.nhwc_bf16(x.detach())
        B, C, H, W = x.shape
        g = Fn._geom(mod, B, H, W)
        if C % 64 != 0 and not (g.r == 1 and g.s == 1 and g.stride == 1 and g.pad == 0):
            raise NotImplementedError("dfu_hip.nn.Conv2d: implicit GEMM needs C % 64 == 0")
        wk = Fn.conv_weight_bf16(w)
        M = B * g.p * g.q
        y = torch.empty((M, g.k), dtype=torch.bfloat16, device=x.device)
        stats = torch.empty((ops.stats_tiles(M), 2, g.k), dtype=torch.float32, device=x.device)
        xr = Fn.rows_view(x)
        Fn.conv_fwd(xr, g, wk, y, stats)
        ctx.g, ctx.mod = g, mod
        ctx.save_for_backward(xr, wk)
        return Fn.from_rows(y, B, g.p, g.q, g.k)

    @staticmethod
    def backward(ctx, gy):
        xr, wk = ctx.saved_tensors
        g, mod = ctx.g, ctx.mod
        dy = Fn.rows_view(Fn.nhwc_bf16(gy))
        dx = None
        if ctx.needs_input_grad[0]:
            dxr = torch.empty((g.n * g.h * g.w, g.c), dtype=torch.bfloat16, device=xr.device)
            Fn.conv_dgrad(dy, g, wk, dxr)
            dx = Fn.from_rows(dxr, g.n, g.h, g.w, g.c)
        if Fn._wants(mod.weight):
            Fn.conv_wgrad(dy, xr, g, Fn.grad_buffer(mod.weight))
            Fn.grads_done(mod.weight)
        return dx, None, None


class BatchNorm2d(tnn.BatchNorm2d):
    """Parameter/buffer holder; the normalisation runs fused into the producing convolution's
    GEMM epilogue (statistics) and its apply/backward kernels (functional._BN)."""

    def forward(self, x):
        raise NotImplementedError(
            "dfu_hip.nn.BatchNorm2d runs fused with its convolution inside ResNet blocks; "
            "standalone BatchNorm2d is not part of the hot path")


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
