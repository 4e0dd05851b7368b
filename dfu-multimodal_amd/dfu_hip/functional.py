"""autograd Functions of the DFU fusion training step, each a hand-scheduled sequence of
libdfu_hip kernels (no ATen compute on this path).

Granularity follows the reference's module tree so the nn.Module surface stays drop-in:
  StemFn         torchvision resnet conv1 + bn1 + relu + maxpool        (resnet.py _forward_impl)
  BottleneckFn   torchvision Bottleneck (v1.5, stride on the 3x3)        (resnet.py Bottleneck)
  AvgPoolFn      AdaptiveAvgPool2d(1) on NHWC -> (B, C, 1, 1) fp32
  PatchEmbedFn   timm PatchEmbed + cls token + pos_embed                 (vision_transformer.py)
  ViTBlockFn     timm Block: x += attn(norm1(x)); x += mlp(norm2(x))
  TokenNormFn    timm final norm applied to the class token rows only (global_pool='token')
  LinearFn / ReLUFn / DropoutFn / ConcatFn   fusion head (train_multimodal_fusion.py:305-324)
  CrossEntropyFn weighted CE (train_multimodal_fusion.py:342-346)

Conventions:
  * ResNet activations are bf16 tensors of logical shape (B, C, H, W) in channels_last memory
    (physically NHWC); ViT activations are the fp32 residual stream (B, T, D).
  * Parameter gradients are ACCUMULATED into persistent ``param.grad`` buffers by the
    weight-gradient GEMM epilogues (``grad_buffer``), and backward returns None for them: this
    keeps .grad addresses stable for graph replay, the fused optimizer and bucketed all-reduce.
  * ViT residual-stream gradients are fp32 and modified in place by the LayerNorm backward
    (the producer of every such tensor is a Function in this file).
"""
import math
import os
import weakref

import torch

from . import _lib as L
from . import ops

BF16 = torch.bfloat16
F32 = torch.float32

# ------------------------------------------------------------------------ precision mode
# "parity" is the library default (DEFAULT_PRECISION): a drop-in script that never names a mode
# gets logits within north_star's 1e-3 of the reference's fp32 path.
# "bf16" (opt-in): bf16 GEMM operands and activations, fp32 accumulation and statistics.
# "bf16x3": the FORWARD pass at fp32 accuracy (csrc/precise.hip): every forward contraction
#   runs on the same MFMA GEMM over split-bf16 triples (hi/lo operands, K tripled), activations
#   stay fp32 between kernels and attention runs in fp32, so the fusion logits meet north_star's
#   "within 1e-3 abs of the reference CPU path" against the fp32 oracle.  The backward pass is
#   the bf16 one (it reads the plain bf16 tensors the split kernels also write).
# "fp16" (a ViT Block stage only): the block's four Linears and its attention on fp16 MFMA
#   operands (11-bit significands, fp32 accumulate; fp32 residual stream, LayerNorm statistics
#   and softmax), writing the same bf16 tensors for the bf16 backward.
# "parity": the headline mode -- per stage the precision named by its ``dfu_parity_precision``
#   (bf16x3 where unset): every ResNet stage bf16x3; ViT Blocks as their VisionTransformer
#   assigns them per role (models/vit.py ``_parity_policy``): every Block fp16 in a ViT a
#   fusion model marks as its feature extractor, Blocks 0-8 bf16x3 and 9-11 fp16 otherwise --
#   the cheapest assignments measured to keep the logits within north_star's 1e-3 of the fp32
#   oracle with margin (profiles/r16a_precision_grid.json, profiles/r19_precision_study.json,
#   profiles/r20_c2_precision_study.txt).  A user may set ``dfu_parity_precision`` on a stage
#   instance; the ViT's policy leaves such an override alone.
# "mixed": per stage -- a ResNet Bottleneck / ViT Block (or the ResNet module itself, for the
#   stem) runs its ``dfu_precision`` attribute's mode ("bf16", "bf16x3", ViT Blocks also
#   "fp16"), bf16x3 where unset (models.precision.apply_policy sets the attributes).  A bf16 or
#   fp16 stage's output enters the next bf16x3 stage as its exact bf16 / fp32 value; a bf16x3
#   stage's output reaches a bf16 stage as the bf16 copy it also writes.
PRECISIONS = ("bf16", "bf16x3", "mixed", "parity")
STAGE_MODES = ("bf16", "bf16x3", "fp16")
DEFAULT_PRECISION = "parity"
_precision = [DEFAULT_PRECISION]


def set_precision(mode):
    """Select the forward precision ("bf16", "bf16x3", "mixed" or "parity"); returns the
    previous mode."""
    if mode not in PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}, got {mode!r}")
    old = _precision[0]
    _precision[0] = mode
    return old


def get_precision():
    return _precision[0]


class precision:
    """Context manager: ``with functional.precision("bf16x3"): logits = model(rgb, th)``."""

    def __init__(self, mode):
        self.mode = mode
        self.old = None

    def __enter__(self):
        self.old = set_precision(self.mode)
        return self

    def __exit__(self, *exc):
        set_precision(self.old)
        return False


def stage_mode(mod=None):
    """The forward precision of stage `mod` (None: a stage without a policy of its own) under
    the current mode: "bf16", "bf16x3" or "fp16"."""
    p = _precision[0]
    if p == "mixed":
        m = getattr(mod, "dfu_precision", None) or "bf16x3"
    elif p == "parity":
        m = getattr(mod, "dfu_parity_precision", None) or "bf16x3"
    else:
        return p
    if m not in STAGE_MODES:
        raise ValueError(f"stage precision must be one of {STAGE_MODES}, got {m!r}")
    return m


def _x3(mod=None):
    """Does the stage `mod` run bf16x3?"""
    return stage_mode(mod) == "bf16x3"


def _per_stage():
    return _precision[0] in ("mixed", "parity")

# ------------------------------------------------------------------------- grad plumbing
_grad_ready_hooks = []


def register_grad_ready_hook(fn):
    """fn(param) is called after a Function has finished writing param.grad (DP bucketing)."""
    _grad_ready_hooks.append(fn)
    return fn


def remove_grad_ready_hook(fn):
    if fn in _grad_ready_hooks:
        _grad_ready_hooks.remove(fn)


# Streams that wrote persistent parameter gradients since the last join.  Autograd synchronises
# only the gradients it returns; these buffers are written in place (possibly on a branch's side
# stream, see models.fusion), so consumers (FusedAdamW.step, GradAllReducer.finish) join first.
_grad_streams = {}


def grad_buffer(p):
    """Persistent fp32 gradient buffer of parameter p (zeroed on first use); notes the current
    stream as a gradient producer."""
    g = p.grad
    if g is None:
        g = torch.empty_like(p, memory_format=torch.contiguous_format)
        ops.zero_(g)
        p.grad = g
    if g.is_cuda:
        st = _current_stream_obj(g)
        _grad_streams[id(st)] = st
        # this step's producer stream of p's gradient (False: more than one), for FusedAdamW's
        # early update of parameters whose gradients are final on a side stream
        prev = getattr(p, "_dfu_grad_stream", None)
        p._dfu_grad_stream = st if prev is None or prev is st else False
    return g


def _current_stream_obj(t):
    """The current stream of t's device as one cached torch Stream object (ops.current_stream;
    called for every parameter gradient of the step)."""
    return ops.current_stream(t.get_device())


def join_grad_streams(stream=None, clear=True):
    """Make `stream` (default: the current stream) wait for every stream that wrote parameter
    gradients since the last clearing join."""
    if not _grad_streams:
        return
    cur = stream if stream is not None else ops.current_stream()
    for st in _grad_streams.values():
        if st != cur:
            ops.stream_wait(cur, st)
    if clear:
        _grad_streams.clear()


# Parameter gradients are written in place, possibly on a branch's side stream or the ViT
# weight-gradient stream, which autograd does not synchronise (it only orders the gradients it
# returns).  So that user code after loss.backward() -- torch.optim optimizers, clip_grad_norm_,
# manual reductions -- may read every p.grad on the stream that called backward, the first
# encoder-boundary backward of a graph task (arm_backward_join: the head side of TokenNormFn /
# AvgPoolFn / ConcatFn, which run on the forward's stream) queues an engine final callback that
# makes that stream wait for every gradient-producing stream once all backward nodes are
# enqueued.  Optimizers joined through join_grad_streams anyway (FusedAdamW, GradAllReducer)
# see no extra wait; any other torch.optim optimizer also joins in a step pre-hook.
_join_armed = [False]
_backward_end_hooks = []


def register_backward_end_hook(fn):
    """fn() is called when a backward pass through the HIP encoders has ended (the engine's
    final callback, after every node ran)."""
    _backward_end_hooks.append(fn)
    return fn


def remove_backward_end_hook(fn):
    if fn in _backward_end_hooks:
        _backward_end_hooks.remove(fn)


def arm_backward_join():
    if _join_armed[0] or not torch.cuda.is_available():
        return
    target = ops.current_stream()
    _join_armed[0] = True

    def _join():
        _join_armed[0] = False
        join_grad_streams(target, clear=False)
        for fn in list(_backward_end_hooks):
            fn()
    try:
        torch.autograd.Variable._execution_engine.queue_callback(_join)
    except RuntimeError:  # not inside a backward pass (a direct .backward() call of a Function)
        _join_armed[0] = False


def _optimizer_pre_hook(optimizer, args, kwargs):
    if _grad_streams and not getattr(optimizer, "_dfu_joins_itself", False):
        join_grad_streams()


try:
    from torch.optim.optimizer import register_optimizer_step_pre_hook
    register_optimizer_step_pre_hook(_optimizer_pre_hook)
except ImportError:  # torch without global optimizer hooks
    pass


_side_streams = {}
# Every library stream runs at the default HIP priority: a high-priority ViT side stream gained
# 0.3% in the eager fusion step, but a C5 Grad-CAM step whose warm-up ran with it replayed from
# a HIP graph at 49.6-54.4 ms against 22.9 ms (round 3).


def new_stream(idx, priority=0):
    """A library-owned non-blocking HIP stream (dfu_stream_create) as a torch ExternalStream.
    Never returned to torch's stream pool: a stream a failed graph capture left capturing is
    retired (dfu_hip.graphs) and this makes a fresh one."""
    import ctypes
    # hipStreamCreate is not a capturable call: under a global-mode capture it invalidates the
    # capture of every stream forked into it (dfu_hip.graphs)
    ops.refuse_in_capture("a new library stream")
    h = ctypes.c_void_p(0)
    with torch.cuda.device(idx):
        L.check(L.load().dfu_stream_create(int(priority), ctypes.byref(h)), "dfu_stream_create")
    return torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx))


def side_stream(device):
    """One persistent side stream per device for the concurrent encoder branch."""
    idx = torch.device(device).index
    if idx is None:
        idx = torch.cuda.current_device()
    st = _side_streams.get(idx)
    if st is None:
        st = _side_streams[idx] = new_stream(idx)
    return st


_wgrad_streams = {}
# DFU_VIT_WGRAD_STREAM=0: the ViT weight-gradient GEMMs stay on the backward's own stream (A/B)
_VIT_WGRAD_STREAM = os.environ.get("DFU_VIT_WGRAD_STREAM", "1") != "0"


def wgrad_stream(device):
    """One persistent stream per device for the ViT blocks' weight-gradient GEMMs: they depend
    only on tensors already produced and feed only the optimizer, so they run beside the input-
    gradient chain, whose N = 768 GEMMs fill 150 of the 256 CUs (12608 / 256 x 768 / 256 tiles)
    and whose LayerNorm / attention kernels leave the MFMAs idle."""
    idx = torch.device(device).index
    if idx is None:
        idx = torch.cuda.current_device()
    st = _wgrad_streams.get(idx)
    if st is None:
        st = _wgrad_streams[idx] = new_stream(idx)
    return st


_concurrent_encoders = [0]


class concurrent_encoders:
    """Context of a forward whose encoders run on two streams (models.fusion): there the other
    encoder's kernels already fill the CUs an N = 768 GEMM leaves idle, and a third stream of
    ViT weight gradients measured slower (18.75 -> 19.2 ms per fusion step), so ViT blocks
    built inside it keep their weight gradients inline (thermal-only: 13.66 -> 12.38 ms)."""

    def __enter__(self):
        _concurrent_encoders[0] += 1

    def __exit__(self, *exc):
        _concurrent_encoders[0] -= 1


class _Beside:
    """Runs weight-gradient work on the wgrad stream after everything already enqueued on the
    current stream (the producers of its operands); the operands are recorded on that stream so
    the allocator does not recycle them early.  Without a stream it runs inline."""

    def __init__(self, stream):
        self.ws = stream
        self.cur = ops.current_stream() if stream is not None else None

    def run(self, fn, *tensors):
        if self.ws is None:
            return fn()
        ops.stream_wait(self.ws, self.cur)
        with ops.on_stream(self.ws):
            for t in tensors:
                t.record_stream(self.ws)
            return fn()


def grads_done(*params):
    if not _grad_ready_hooks:
        return
    hooks = tuple(_grad_ready_hooks)  # (a hook may be removed meanwhile: GC)
    for p in params:
        if p is not None:
            for h in hooks:
                h(p)


def module_param(mod, name):
    """mod.<name> for a registered parameter or buffer by its dict (nn.Module.__getattr__, the
    slow path for both, costs ~0.25 us an attribute); anything else by getattr."""
    p = mod._parameters
    if name in p:
        return p[name]
    b = mod._buffers
    return b[name] if name in b else getattr(mod, name)


def _wants(p):
    return p is not None and p.requires_grad


def _empty(shape, dtype, device):
    return torch.empty(shape, dtype=dtype, device=device)


def nhwc_bf16(x):
    """Return x (B,C,H,W) as a bf16 channels_last tensor (no copy when it already is one)."""
    if x.dtype != BF16:
        x = x.to(BF16)
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    return x


def rows_view(x):
    """[B*H*W, C] view of a channels_last (B,C,H,W) tensor."""
    B, C, H, W = x.shape
    return x.permute(0, 2, 3, 1).reshape(B * H * W, C)


def from_rows(r, B, H, W, C):
    return r.view(B, H, W, C).permute(0, 3, 1, 2)


def _krsc_strided(w):
    """A 4-D OIHW-shaped tensor whose memory is KRSC (channels-last), as optim.FlatParams
    stores spatial conv weights."""
    return (w.dim() == 4 and not w.is_contiguous()
            and w.is_contiguous(memory_format=torch.channels_last))


def _rows2d(w):
    """[N, K] rows of w in its storage order (KRSC for a channels-last conv weight: a view)."""
    if _krsc_strided(w):
        return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
    return w.reshape(w.shape[0], -1)


def weight_bf16_rows(w, ld=None):
    """fp32 [N, K...] parameter -> bf16 [N, ld] GEMM operand, rows in the parameter's storage
    order.  Parameters managed by FusedAdamW have a bf16 shadow the optimizer kernel keeps
    current (optim.FlatParams): returned as a view, re-cast only if the parameter changed
    outside the optimizer (version counter)."""
    w2 = _rows2d(w.detach())
    sh = getattr(w, "_dfu_shadow", None)
    if sh is not None and (ld is None or ld == w2.shape[1]):
        if w._version != getattr(w, "_dfu_shadow_version", -1):
            ops.cast_rows_bf16(w2, out=sh)
            w._dfu_shadow_version = w._version
            w._dfu_sgen = getattr(w, "_dfu_sgen", 0) - 1  # any transposed copy is now stale
        return sh
    return ops.cast_rows_bf16(w2, ld_out=ld)


def weight_f16_rows(w):
    """fp32 [N, K...] parameter -> fp16 [N, K] GEMM operand (the "fp16" stage precision).
    FusedAdamW-managed parameters get an fp16 shadow the optimizer kernel keeps current from the
    first use on (optim.FlatParams.enable_f16; re-cast only after an outside edit); others are
    cast per call."""
    flat = getattr(w, "_dfu_flat", None)
    if flat is not None and flat.shadow is not None:
        if flat.shadow16 is None:
            flat.enable_f16()
        sh = w._dfu_shadow16
        if w._version != getattr(w, "_dfu_shadow16_version", -1):
            ops.cast_rows_f16(_rows2d(w.detach()), out=sh)
            w._dfu_shadow16_version = w._version
        return sh
    return ops.cast_rows_f16(_rows2d(w.detach()))


def weight_bf16_T(w):
    """The transposed bf16 shadow [in, out] of an FusedAdamW-managed 2-D weight (for the
    input-gradient GEMM dX = dY W, whose weight operand it makes K-contiguous), or None for a
    weight without a shadow (the caller then reads W itself as an MN-major operand).  Created
    on first use; afterwards the optimizer refreshes it with one batched launch per step
    (optim.FlatParams.shadows_rewritten) and this only re-transposes after an outside edit."""
    sh = weight_bf16_rows(w)
    flat = getattr(w, "_dfu_flat", None)
    if flat is None or sh is not getattr(w, "_dfu_shadow", None):
        return None
    if getattr(w, "_dfu_shadow_T", None) is None:
        flat.add_transposed(w)
        w._dfu_tgen = None
    if w._dfu_tgen != getattr(w, "_dfu_sgen", 0):
        ops.transpose_bf16(sh, out=w._dfu_shadow_T)
        w._dfu_tgen = getattr(w, "_dfu_sgen", 0)
    return w._dfu_shadow_T


# Stride-1 spatial conv input gradients as forward convolutions of dY with the flipped,
# channel-transposed weight (optim.FlatParams.add_flipped): K-contiguous weight operand and the
# forward's gather loader instead of the dgrad's MN-major weight view.  DFU_DGRAD_FLIP=0: the
# dgrad loaders (A/B timing).
_DGRAD_FLIP = os.environ.get("DFU_DGRAD_FLIP", "1") != "0"


def conv_weight_flipped(w):
    """W'[C][R][S][K] = W[K][R-1-r][S-1-s][C] (bf16, [C][R*S*K]) of a FusedAdamW-managed
    channels-last conv weight, or None.  Re-derived (one launch, on the current stream) on the
    first use after the optimizer rewrote the shadows or the weight was edited outside it."""
    if not _DGRAD_FLIP or not _krsc_strided(w):
        return None
    sh = weight_bf16_rows(w)
    flat = getattr(w, "_dfu_flat", None)
    if flat is None or sh is not getattr(w, "_dfu_shadow", None):
        return None
    if getattr(w, "_dfu_shadow_F", None) is None:
        flat.add_flipped(w)
    key = (flat.gen, getattr(w, "_dfu_shadow_version", None))
    if w._dfu_fkey != key:
        w._dfu_flip_jobs.launch()
        w._dfu_fkey = key
    return w._dfu_shadow_F


# 1x1 stride-1 input gradients of at most this many input channels (layer 1's 64: the N = 64
# GEMMs, which the 64-column tiles run only with a K-contiguous weight operand) on the
# transposed weight shadow (weight_bf16_T, refreshed with the optimizer's batched transposes).
# DFU_DGRAD_T1X1_MAXC=0: the MN-major weight view (A/B timing).
_DGRAD_T1X1_MAXC = int(os.environ.get("DFU_DGRAD_T1X1_MAXC", "64"))


def conv1x1_weight_T(conv, geom):
    """The transposed bf16 shadow [C][K] of a FusedAdamW-managed 1x1 stride-1 conv weight with
    at most _DGRAD_T1X1_MAXC input channels (conv_dgrad's w_t), else None."""
    if (geom.r == 1 and geom.s == 1 and geom.stride == 1 and geom.pad == 0
            and geom.c <= _DGRAD_T1X1_MAXC):
        return weight_bf16_T(conv.weight)
    return None


def conv_weight_bf16(w):
    """fp32 OIHW conv weight -> bf16 KRSC GEMM operand: the shadow view for a 1x1 conv (OIHW ==
    KRSC) and for a FusedAdamW-managed weight stored channels-last; else a packing kernel."""
    if (w.shape[2] == 1 and w.shape[3] == 1) or _krsc_strided(w):
        return weight_bf16_rows(w)
    return ops.pack_conv_weight(w.detach())


def weight_x3_rows(w, seg=None):
    """fp32 [N, K...] parameter -> bf16x3 GEMM B operand [N, 3 seg] = [hi | hi | lo]."""
    return ops.split_x3(w.detach().reshape(w.shape[0], -1), ops.X3_B, seg=seg)


# The bf16x3 ResNet forward's GEMMs on interleaved pairs (dfu_gemm_desc.x3_pairs: K = 2C, the
# three products per K-step from 2 operand tiles) instead of the tripled K; DFU_X3_PAIRS=0: the
# tripled K (A/B timing).
_X3_PAIRS = os.environ.get("DFU_X3_PAIRS", "1") != "0"


def conv_weight_x3(w):
    """fp32 OIHW conv weight -> bf16x3 KRSC' operand: C' = 2C interleaved pairs (_X3_PAIRS) or
    C' = 3C [hi | hi | lo]; 1x1: the row split.  A FusedAdamW-managed weight reads the pairs
    from the optimizer's x3 shadow (optim.FlatParams.enable_x3: written by the AdamW kernel, no
    launch here); re-split only after an edit outside the optimizer (version counter)."""
    flat = getattr(w, "_dfu_flat", None)
    if _X3_PAIRS and flat is not None:
        from .optim import x3_pair_weight
        if x3_pair_weight(w):
            if flat.shadow_x3 is None:
                flat.enable_x3()
            sh = w._dfu_shadow_x3
            if w._version != getattr(w, "_dfu_shadow_x3_version", -1):
                src = w.detach().permute(0, 2, 3, 1).reshape(-1, 32)  # KRSC rows of 32
                ops.split_x3_into(src.contiguous(), ops.X3_PAIRS, sh.view(-1, 64))
                w._dfu_shadow_x3_version = w._version
            return sh
    if _X3_PAIRS:
        if w.shape[2] == 1 and w.shape[3] == 1:
            return ops.split_x3(w.detach().reshape(w.shape[0], -1), ops.X3_PAIRS)
        return ops.pack_conv_weight_x3(w.detach(), ops.X3_PAIRS)
    if w.shape[2] == 1 and w.shape[3] == 1:
        return weight_x3_rows(w)
    return ops.pack_conv_weight_x3(w.detach())


def _take_x3(x):
    """The fp32-accurate split pair (hi, lo) of activation x, [rows][C] bf16 each: hi is x's own
    bf16 rows, lo the residual a bf16x3 producer attached (detached from x here: each one has a
    single consumer), or zeros when x came from elsewhere (a bf16 value is its own hi)."""
    hi = rows_view(nhwc_bf16(x.detach()))
    lo = getattr(x, "_dfu_lo", None)
    if lo is not None:
        try:
            del x._dfu_lo
        except AttributeError:
            pass
        return hi, lo
    return hi, torch.zeros_like(hi)


# ---------------------------------------------------------------------- BatchNorm helper
class _BN:
    """Forward/backward state of one BatchNorm2d applied to a GEMM output with stats."""

    def __init__(self, bn, M, C, device):
        self.bn = bn
        self.M, self.C = M, C
        self.training = bn.training or not bn.track_running_stats
        # one [4][C] block: rows scale, shift, mean, invstd
        self.coef4 = _empty((4, C), F32, device)
        self.scale, self.shift, self.mean, self.invstd = self.coef4.unbind(0)

    def forward_coeffs(self, stats):
        bn = self.bn
        if self.training:
            track = bn.track_running_stats and bn.training
            mom = bn.momentum if bn.momentum is not None else 0.1
            mp = module_param
            ops.bn_finalize(stats, self.M, self.C, mp(bn, "weight"), mp(bn, "bias"), bn.eps, mom,
                            mp(bn, "running_mean") if track else None,
                            mp(bn, "running_var") if track else None,
                            mp(bn, "num_batches_tracked") if track else None,
                            self.mean, self.invstd, self.scale, self.shift)
        else:
            ops.bn_eval_coeffs(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps,
                               self.scale, self.shift)
            self.mean.copy_(bn.running_mean)
            ops.bn_eval_coeffs(None, None, bn.running_mean, bn.running_var, bn.eps,
                               self.invstd, _empty((self.C,), F32, self.mean.device))

    def backward(self, dout, y, out, relu, dy, dres):
        """relu: False; True (mask from `out`, the BN + residual + ReLU case); 2 (BN + ReLU
        with no residual: the mask is recomputed from y with the forward's scale/shift, so
        `out` is not read); or 3 (`out` is the forward's ReLU bitmask, ops.bn_apply(mask=))."""
        bn = self.bn
        w, b = module_param(bn, "weight"), module_param(bn, "bias")
        dgamma = grad_buffer(w) if _wants(w) else None
        dbeta = grad_buffer(b) if _wants(b) else None
        ops.bn_bwd(dout, y, out, relu, self.mean, self.invstd, w, self.M, self.C, dy,
                   dres, dgamma, dbeta, batch_stats=self.training, scale=self.scale,
                   shift=self.shift)
        grads_done(w, b)


# --------------------------------------------------------------------------- conv helpers
def conv_fwd(x_rows, geom, w_krsc, y, stats):
    """y[M, K] = conv(x) for NHWC x with a KRSC bf16 weight; BN tile statistics into stats."""
    g = geom
    M = g.n * g.p * g.q
    if g.r == 1 and g.s == 1 and g.stride == 1 and g.pad == 0:
        ops.gemm(M, g.k, g.c, x_rows, g.c, w_krsc, g.c, y, g.k, epilogue=L.EPI_BF16_STATS,
                 stats=stats)
    else:
        K = g.r * g.s * g.c
        ops.gemm(M, g.k, K, x_rows, 0, w_krsc, K, y, g.k, a_mode=L.OPND_CONV_FWD,
                 epilogue=L.EPI_BF16_STATS, stats=stats, conv=g)


def conv_fwd_x3(x_pair, geom, w3, y, stats, y_lo=None):
    """bf16x3: y[M, K] = conv(x) over the split pair x = (hi, lo) [N*H*W, C] (the GEMM reads
    interleaved pairs, or the channel-tripled hi | lo | hi) and KRSC' weights (conv_weight_x3),
    fp32 -- or with y_lo, the split pair (y = bf16 hi, y_lo = lo) of the fp32 result; BN tile
    statistics of the unrounded outputs into stats."""
    g = geom
    hi, lo = x_pair
    M = g.n * g.p * g.q
    pairs = _X3_PAIRS
    C3 = (2 if pairs else 3) * g.c
    K3 = g.r * g.s * C3
    xk = dict(x3=True, a_lo=lo, x3_pairs=pairs)
    out = dict(aux_out=y_lo, ldaux_out=g.k if y_lo is not None else 0)
    if g.r == 1 and g.s == 1 and g.stride == 1 and g.pad == 0:
        ops.gemm(M, g.k, C3, hi, g.c, w3, C3, y, g.k, epilogue=L.EPI_F32_STATS, stats=stats,
                 **xk, **out)
    else:
        g3 = ops.ConvGeom(g.n, g.h, g.w, C3, g.k, g.r, g.s, g.stride, g.pad)
        ops.gemm(M, g.k, K3, hi, 0, w3, K3, y, g.k, a_mode=L.OPND_CONV_FWD,
                 epilogue=L.EPI_F32_STATS, stats=stats, conv=g3, **xk, **out)


def conv_dgrad(dy_rows, geom, w_krsc, dx, add=None, w_flip=None, w_t=None):
    """dx[N*H*W, C] = dgrad(dy) (+ add, bf16).  With w_flip (conv_weight_flipped; stride 1, no
    add): dx is the forward convolution of dy (K input channels, pad R-1-pad) with the flipped
    weight.  With w_t (conv1x1_weight_T; a 1x1 stride-1 conv): dx = dy W as a K-contiguous GEMM
    on the transposed [C][K] weight."""
    g = geom
    Mx = g.n * g.h * g.w
    if w_t is not None and g.r == 1 and g.s == 1 and g.stride == 1 and g.pad == 0:
        ops.gemm(Mx, g.c, g.k, dy_rows, g.k, w_t, g.k, dx, g.c,
                 epilogue=L.EPI_BF16_ADD if add is not None else L.EPI_BF16, aux=add,
                 ldaux=g.c if add is not None else 0)
        return
    if w_flip is not None and add is None and g.stride == 1:
        gd = ops.ConvGeom(g.n, g.p, g.q, g.k, g.c, g.r, g.s, 1, g.r - 1 - g.pad)
        if (gd.p, gd.q) == (g.h, g.w) and g.r - 1 - g.pad >= 0:
            K = g.r * g.s * g.k
            ops.gemm(Mx, g.c, K, dy_rows, 0, w_flip, K, dx, g.c, a_mode=L.OPND_CONV_FWD,
                     epilogue=L.EPI_BF16, conv=gd)
            return
    epi = L.EPI_BF16_ADD if add is not None else L.EPI_BF16
    aux, ld_aux = add, (g.c if add is not None else 0)
    if g.r == 1 and g.s == 1 and g.stride == 1 and g.pad == 0:
        ops.gemm(Mx, g.c, g.k, dy_rows, g.k, w_krsc, g.c, dx, g.c, b_mode=L.OPND_MNMAJOR,
                 epilogue=epi, aux=aux, ldaux=ld_aux)
    else:
        ops.gemm(Mx, g.c, g.r * g.s * g.k, dy_rows, 0, w_krsc, g.r * g.s * g.c, dx, g.c,
                 a_mode=L.OPND_CONV_DGRAD, b_mode=L.OPND_CONV_DGRAD_W, epilogue=epi, aux=aux,
                 ldaux=ld_aux, conv=g)


def conv_wgrad(dy_rows, x_rows, geom, dw):
    """dw (fp32 OIHW shape) += wgrad(dy, x).  The GEMM accumulates in KRSC order (contiguous
    n' = (r, s, c): coalesced epilogue stores): straight into dw when dw is stored KRSC (a 1x1
    conv, or optim.FlatParams' channels-last conv weights), else into a scratch buffer that is
    permute-added into the OIHW gradient."""
    g = geom
    M = g.n * g.p * g.q
    if g.r == 1 and g.s == 1 and g.stride == 1 and g.pad == 0:
        ops.gemm(g.k, g.c, M, dy_rows, g.k, x_rows, g.c, dw, g.c, a_mode=L.OPND_MNMAJOR,
                 b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC)
    elif _krsc_strided(dw):
        N = g.r * g.s * g.c
        ops.gemm(g.k, N, M, dy_rows, g.k, x_rows, 0, _rows2d(dw), N, a_mode=L.OPND_MNMAJOR,
                 b_mode=L.OPND_CONV_WGRAD_X, epilogue=L.EPI_F32_ACC, conv=g)
    else:
        N = g.r * g.s * g.c
        acc = _empty((g.k, N), F32, dy_rows.device)
        ops.zero_(acc)
        ops.gemm(g.k, N, M, dy_rows, g.k, x_rows, 0, acc, N, a_mode=L.OPND_MNMAJOR,
                 b_mode=L.OPND_CONV_WGRAD_X, epilogue=L.EPI_F32_ACC, conv=g)
        ops.conv_grad_krsc_to_oihw(acc, dw)


def _geom(conv, B, H, W):
    Cout, Cin, R, S = conv.weight.shape
    return ops.ConvGeom(B, H, W, Cin, Cout, R, S, conv.stride[0], conv.padding[0])


# ------------------------------------------------------------------------------- stem
_STEM_FUSED = os.environ.get("DFU_STEM_FUSED", "1") != "0"


class StemFn(torch.autograd.Function):
    """conv1 7x7/s2/p3 (3->64, explicit bf16 im2col, K padded 147->160) + bn1 + relu +
    maxpool 3x3/s2/p1.  Input fp32 (B,3,H,W) any strides; output bf16 channels_last."""

    KP = 160

    @staticmethod
    def forward(ctx, x, w, gamma, beta, mod):
        conv, bn = mod.conv1, mod.bn1
        B, C, H, W = x.shape
        R = S = conv.weight.shape[2]
        st, pad = conv.stride[0], conv.padding[0]
        Kp = ((C * R * S + 15) // 16) * 16
        xf = x.detach().float() if x.dtype != F32 else x.detach()
        wb = weight_bf16_rows(w, ld=Kp)
        Cout = w.shape[0]
        x3 = _x3(mod)
        # bf16x3: one implicit-GEMM kernel (dfu_stem_conv_x3: no pair im2col in HBM) where its
        # geometry allows; DFU_STEM_FUSED=0: the pair im2col + interleaved-pair GEMM (A/B)
        fused = x3 and _STEM_FUSED and Kp == 160 and ops.stem_conv_x3_ok(xf, w, st, pad)
        if fused:  # no im2col rows: the backward's weight gradient reads x (dfu_stem_wgrad_x3)
            y, y_lo, stats, col, P, Q = ops.stem_conv_x3(xf, w.detach(), st, pad, want_col=False)
        elif x3:
            (col, col_lo), P, Q = ops.im2col_f32_x3(xf, R, S, st, pad, Kp)  # split pair
        else:
            col, P, Q = ops.im2col_f32(xf, R, S, st, pad, Kp)
        M = B * P * Q
        if not fused:
            y = _empty((M, Cout), BF16, x.device)
            stats = _empty((ops.stats_tiles(M), 2, Cout), F32, x.device)
        bns = _BN(bn, M, Cout, x.device)
        if x3:
            a = _empty((M * Cout // 8,), torch.uint8, x.device)  # bn1's ReLU bitmask
            if not fused:
                y_lo = _empty((M, Cout), BF16, x.device)  # the conv output as a split pair
                if _X3_PAIRS and Kp % 32 == 0:  # interleaved pairs (conv_weight_x3)
                    w3, K3, pairs = ops.split_x3(w.detach().reshape(Cout, -1), ops.X3_PAIRS,
                                                 seg=Kp), 2 * Kp, True
                else:
                    w3, K3, pairs = weight_x3_rows(w, seg=Kp), 3 * Kp, False
                ops.gemm(M, Cout, K3, col, Kp, w3, K3, y, Cout, epilogue=L.EPI_F32_STATS,
                         stats=stats, x3=True, a_lo=col_lo, x3_pairs=pairs, aux_out=y_lo,
                         ldaux_out=Cout)
                del col_lo
            bns.forward_coeffs(stats)
            # bn1 + ReLU applied inside the pool, from the pair (no fp32 BN output stored)
            out_lo, out, am, P2, Q2 = ops.maxpool_bn_fwd_x3(y, y_lo, bns.scale, bns.shift, B, P,
                                                            Q, Cout, relu_mask=a)
            del y_lo
        else:
            ops.gemm(M, Cout, Kp, col, Kp, wb, Kp, y, Cout, epilogue=L.EPI_BF16_STATS,
                     stats=stats)
            bns.forward_coeffs(stats)
            # bn1 + relu applied inside the pool (the backward recomputes the ReLU mask from
            # y, so the BN output itself is never stored)
            a = None
            out, am, P2, Q2 = ops.maxpool_fwd(y, B, P, Q, Cout, scale=bns.scale,
                                              shift=bns.shift)
        ctx.mod = mod
        ctx.bns = bns
        ctx.x3 = x3
        ctx.dims = (B, C, H, W, P, Q, P2, Q2, Cout, Kp, R, S, st, pad)
        ctx.x_requires_grad = x.requires_grad
        ctx.fused = fused
        ctx.save_for_backward(xf if fused else col, y, a, am, wb)
        res = out.permute(0, 3, 1, 2)
        if x3:
            res._dfu_lo = out_lo
        return res

    @staticmethod
    def backward(ctx, gout):
        col, y, a, am, wb = ctx.saved_tensors
        B, C, H, W, P, Q, P2, Q2, Cout, Kp, R, S, st, pad = ctx.dims
        mod = ctx.mod
        g = rows_view(nhwc_bf16(gout))
        da = ops.maxpool_bwd(g, am, B, P, Q, Cout, P2, Q2).view(B * P * Q, Cout)
        M = B * P * Q
        dy = torch.empty_like(y)
        if ctx.x3:  # the forward's own ReLU bitmask (its pre-activation was fp32)
            ctx.bns.backward(da, y, a, 3, dy, None)
        else:
            ctx.bns.backward(da, y, None, 2, dy, None)
        w = mod.conv1.weight
        if _wants(w):
            dw = grad_buffer(w).view(Cout, -1)
            K = C * R * S
            if ctx.fused:  # from x itself (the saved tensor is xf): no im2col rows
                ops.stem_wgrad_x3(col, dy, dw, st, pad)
            else:
                # bf16 im2col rows: the col itself, or the hi rows of the bf16x3 split pair
                ops.gemm(Cout, K, M, dy, Cout, col, col.stride(0), dw, K, a_mode=L.OPND_MNMAJOR,
                         b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC)
            grads_done(w)
        dx = None
        if ctx.x_requires_grad:
            # Grad-CAM path (grad_cam_visualization.py:374): fp32 dcol = dy W (MFMA GEMM),
            # then its col2im adjoint (a gather kernel) -> fp32 NCHW input gradient.
            wkn = wb  # [Cout][Kp] viewed as B[k=cout][n=kp]
            dcol = _empty((M, Kp), F32, y.device)
            ops.gemm(M, Kp, Cout, dy, Cout, wkn, Kp, dcol, Kp, b_mode=L.OPND_MNMAJOR,
                     epilogue=L.EPI_F32)
            dx = ops.col2im_f32(dcol, B, C, H, W, R, S, st, pad, P, Q, Kp)
        return dx, None, None, None, None


# ---------------------------------------------------------------------------- Bottleneck
def _fire_grad_hooks(probe, grad):
    """Call the gradient hooks registered (Tensor.register_hook) on a probe leaf with the
    gradient the fused backward computed for the tensor it stands for."""
    for hook in list((probe._backward_hooks or {}).values()):
        hook(grad)


class BottleneckFn(torch.autograd.Function):
    """torchvision Bottleneck: relu(bn3(conv3(relu(bn2(conv2(relu(bn1(conv1 x))))))) + id)."""

    @staticmethod
    def forward(ctx, x, *params_and_mod):
        mod = params_and_mod[-1]
        mm = mod._modules  # (nn.Module attributes are slow __getattr__ lookups)
        x3mode = _x3(mod)
        xin3 = _take_x3(x) if x3mode else None
        x = nhwc_bf16(x.detach())
        B, Cin, H, W = x.shape
        dev = x.device
        xr = rows_view(x)
        g1 = _geom(mm["conv1"], B, H, W)
        g2 = _geom(mm["conv2"], B, g1.p, g1.q)
        g3 = _geom(mm["conv3"], B, g2.p, g2.q)
        w1 = conv_weight_bf16(mm["conv1"].weight)
        w2 = conv_weight_bf16(mm["conv2"].weight)
        w3 = conv_weight_bf16(mm["conv3"].weight)
        M1 = B * g1.p * g1.q
        M2 = B * g2.p * g2.q
        planes, outc = g1.k, g3.k

        def conv_bn(xrows, geom, w, bnmod, relu, residual=None, mask=None):
            M = geom.n * geom.p * geom.q
            y = _empty((M, geom.k), BF16, dev)
            stats = _empty((ops.stats_tiles(M), 2, geom.k), F32, dev)
            conv_fwd(xrows, geom, w, y, stats)
            st = _BN(bnmod, M, geom.k, dev)
            st.forward_coeffs(stats)
            out = _empty((M, geom.k), BF16, dev)
            ops.bn_apply(y, st.scale, st.shift, residual, relu, out, M, geom.k, mask=mask)
            return y, out, st

        def conv_bn_x3(xpair, geom, w3x, bnmod, relu, res=None, res_mode=0, want_pair=True,
                       want_f32=False):
            """bf16x3: fp32 conv + BN (+res) (+ReLU) -> (y bf16, out bf16 (hi), out lo, out
            fp32, BN state, ReLU bitmask); res_mode 2: res is a split pair."""
            M = geom.n * geom.p * geom.q
            # the conv output as a split pair: y (= bf16(y), what the BN backward reads) + y_lo
            y = _empty((M, geom.k), BF16, dev)
            y_lo = _empty((M, geom.k), BF16, dev)
            stats = _empty((ops.stats_tiles(M), 2, geom.k), F32, dev)
            conv_fwd_x3(xpair, geom, w3x, y, stats, y_lo=y_lo)
            st = _BN(bnmod, M, geom.k, dev)
            st.forward_coeffs(stats)
            out = _empty((M, geom.k), BF16, dev) if want_pair else None
            lo = _empty((M, geom.k), BF16, dev) if want_pair else None
            of = _empty((M, geom.k), F32, dev) if want_f32 else None
            rhi, rlo = res if res_mode == 2 else (res, None)
            mask = _empty((M * geom.k // 8,), torch.uint8, dev) if relu else None
            ops.bn_apply_x3(y, st.scale, st.shift, rhi, res_mode, relu, M, geom.k, out_lo=lo,
                            out_bf16=out, out_f32=of, residual_lo=rlo, y_lo=y_lo, relu_mask=mask)
            return y, out, lo, of, st, mask

        out_lo = None
        masks = None
        if x3mode:
            y1, a1, a1_lo, _, s1, m1 = conv_bn_x3(xin3, g1, conv_weight_x3(mm["conv1"].weight),
                                                   mm["bn1"], True)
            y2, a2, a2_lo, _, s2, m2 = conv_bn_x3((a1, a1_lo), g2,
                                                   conv_weight_x3(mm["conv2"].weight), mm["bn2"],
                                                   True)
            masks = (m1, m2)  # the BN + ReLU backward's masks (the pre-activations were fp32)
            del a1_lo
        else:
            y1, a1, s1 = conv_bn(xr, g1, w1, mm["bn1"], True)
            y2, a2, s2 = conv_bn(a1, g2, w2, mm["bn2"], True)
        if mm.get("downsample") is not None:
            dconv, dbn = mm.get("downsample")[0], mm.get("downsample")[1]
            gd = _geom(dconv, B, H, W)
            wd = conv_weight_bf16(dconv.weight)
            if x3mode:
                yd, _, _, idn, sd, _ = conv_bn_x3(xin3, gd, conv_weight_x3(dconv.weight), dbn,
                                                  False, want_pair=False, want_f32=True)
                res, res_mode = idn, 1
            else:
                yd, idn, sd = conv_bn(xr, gd, wd, dbn, False)
        else:
            gd = wd = yd = sd = None
            idn = xr
            res, res_mode = xin3, 2
        if x3mode:
            y3, out, out_lo, _, s3, mask3 = conv_bn_x3((a2, a2_lo), g3,
                                                        conv_weight_x3(mm["conv3"].weight),
                                                        mm["bn3"], True, res=res,
                                                        res_mode=res_mode)
            del a2_lo, res, xin3
        else:
            # bn3 + residual + ReLU also writes its ReLU bitmask: the backward reads M*C/8 bytes
            # instead of the block output twice (reduce and apply)
            mask3 = _empty((M2 * outc // 8,), torch.uint8, dev)
            y3, out, s3 = conv_bn(a2, g3, w3, mm["bn3"], True, residual=idn, mask=mask3)
        ctx.x3 = x3mode
        ctx.mod = mod
        ctx.geo = (g1, g2, g3, gd)
        ctx.bns = (s1, s2, s3, sd)
        ctx.shape = (B, Cin, H, W)
        ctx.x_requires_grad = ctx.needs_input_grad[0]
        ctx.probes = None
        if getattr(mod, "_probe", False):
            # Hooked `relu` (Grad-CAM): torchvision calls it after bn1 and bn2 as well, so hand
            # the block the two inner ReLU outputs as leaf tensors whose gradient hooks
            # backward fires with da2 / da1 (models/resnet.py Bottleneck.forward).
            ctx.probes = (from_rows(a1, B, g1.p, g1.q, planes).detach().requires_grad_(True),
                          from_rows(a2, B, g2.p, g2.q, planes).detach().requires_grad_(True))
            mod._probes = ctx.probes
        ctx.masks = masks
        ctx.save_for_backward(xr, y1, a1, y2, a2, y3, mask3, w1, w2,
                              w3, *( (yd, wd) if yd is not None else ()))
        res = from_rows(out, B, g3.p, g3.q, outc)
        if out_lo is not None:
            res._dfu_lo = out_lo
        return res

    @staticmethod
    def backward(ctx, gout):
        saved = ctx.saved_tensors
        xr, y1, a1, y2, a2, y3, out, w1, w2, w3 = saved[:10]
        yd, wd = (saved[10], saved[11]) if len(saved) > 10 else (None, None)
        mod = ctx.mod
        mm = mod._modules
        g1, g2, g3, gd = ctx.geo
        s1, s2, s3, sd = ctx.bns
        B, Cin, H, W = ctx.shape
        dev = xr.device
        g = rows_view(nhwc_bf16(gout))
        M1, M2 = y1.shape[0], y3.shape[0]

        def wgrad(conv, dy, x, geom):
            if _wants(conv.weight):
                conv_wgrad(dy, x, geom, grad_buffer(conv.weight))
                grads_done(conv.weight)

        # bn3 (+ residual) + relu: the ReLU bitmask its forward apply wrote
        dy3 = torch.empty_like(y3)
        dres = torch.empty_like(y3)
        s3.backward(g, y3, out, 3, dy3, dres)
        # downsample branch (its dgrad is added in place after conv1's, below)
        dyd = None
        if yd is not None:
            dyd = torch.empty_like(yd)
            sd.backward(dres, yd, None, False, dyd, None)
            wgrad(mm.get("downsample")[0], dyd, xr, gd)
        # conv3
        da2 = torch.empty_like(a2)
        conv_dgrad(dy3, g3, w3, da2, w_t=conv1x1_weight_T(mm["conv3"], g3))
        if ctx.probes is not None:
            _fire_grad_hooks(ctx.probes[1], from_rows(da2, B, g2.p, g2.q, g2.k))
        wgrad(mm["conv3"], dy3, a2, g3)
        # bn2 + relu, conv2
        # BN + ReLU masks: recomputed from y (bf16), or in bf16x3 mode (fp32 pre-activations)
        # the bitmasks the forward apply wrote
        dy2 = torch.empty_like(y2)
        m1, m2 = ctx.masks if ctx.masks is not None else (None, None)
        s2.backward(da2, y2, m2, 3 if ctx.x3 else 2, dy2, None)
        da1 = torch.empty_like(a1)
        conv_dgrad(dy2, g2, w2, da1, w_flip=None if g2.stride != 1 else
                   conv_weight_flipped(mm["conv2"].weight))
        if ctx.probes is not None:
            _fire_grad_hooks(ctx.probes[0], from_rows(da1, B, g1.p, g1.q, g1.k))
        wgrad(mm["conv2"], dy2, a1, g2)
        # bn1 + relu, conv1 (+ identity gradient fused in the dgrad epilogue)
        dy1 = torch.empty_like(y1)
        s1.backward(da1, y1, m1, 3 if ctx.x3 else 2, dy1, None)
        dx = None
        if ctx.x_requires_grad:
            dxr = _empty((M1, Cin), BF16, dev)
            w1t = conv1x1_weight_T(mm["conv1"], g1)
            if dyd is None:  # identity shortcut: its gradient rides in conv1's dgrad epilogue
                conv_dgrad(dy1, g1, w1, dxr, add=dres, w_t=w1t)
            else:  # downsample: conv1's dgrad, then the (strided) 1x1 dgrad added in place
                conv_dgrad(dy1, g1, w1, dxr, w_t=w1t)
                conv_dgrad(dyd, gd, wd, dxr, add=dxr,
                           w_t=conv1x1_weight_T(mm.get("downsample")[0], gd))
            dx = from_rows(dxr, B, H, W, Cin)
        wgrad(mm["conv1"], dy1, xr, g1)
        n_params = len(ctx.needs_input_grad) - 2
        return (dx,) + (None,) * n_params + (None,)


# ------------------------------------------------------------------------------ avgpool
class AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        # bf16x3: the split pair of the producer; per-stage modes: that pair if the last block
        # ran bf16x3 (a bf16 block's output is pooled in bf16)
        x3 = _take_x3(x) if _x3() and (not _per_stage() or hasattr(x, "_dfu_lo")) else None
        x = nhwc_bf16(x.detach())
        B, C, H, W = x.shape
        ctx.shape = (B, C, H, W)
        if x3 is not None:
            y = ops.avgpool_fwd_x3(x3[0], x3[1], B, H * W, C)
        else:
            y = ops.avgpool_fwd(rows_view(x), B, H * W, C)
        return y.view(B, C, 1, 1)

    @staticmethod
    def backward(ctx, g):
        if g.is_cuda:
            arm_backward_join()
        B, C, H, W = ctx.shape
        g = g.reshape(B, C)
        if g.dtype != F32:
            g = g.float()
        dx = ops.avgpool_bwd(g.contiguous(), B, H * W, C)
        return from_rows(dx.view(B * H * W, C), B, H, W, C)


# ------------------------------------------------------------------------ ViT embedding
class PatchEmbedFn(torch.autograd.Function):
    """timm PatchEmbed (conv16/s16 + flatten) + cat(cls_token) + pos_embed -> fp32 (B,T,D)."""

    @staticmethod
    def forward(ctx, x, w, b, cls, pos, ps):
        B, C, H, W = x.shape
        D = w.shape[0]
        xf = x.detach().float() if x.dtype != F32 else x.detach()
        T = (H // ps) * (W // ps)
        wb = weight_bf16_rows(w)
        K = wb.shape[1]
        X = _empty((B, T + 1, D), F32, x.device)
        if _x3():  # [B*T][3K] triple; the backward reads its hi segment (row stride 3K)
            patches = ops.patchify_f32_x3(xf, ps)
            A, Bop, Kg = patches, weight_x3_rows(w), 3 * K
        else:
            patches = ops.patchify_f32(xf, ps)
            A, Bop, Kg = patches, wb, K
        ops.gemm(B * T, D, Kg, A, Kg, Bop, Kg, X, D, epilogue=L.EPI_PATCH,
                 bias=b.detach() if b is not None else None, aux=pos.detach().reshape(T + 1, D),
                 ldaux=D, ep_tokens=T, x3=Kg != K)
        ops.vit_cls_rows(cls.detach().reshape(D), pos.detach().reshape(T + 1, D), X, B, T + 1, D)
        ctx.params = (w, b, cls, pos)
        ctx.dims = (B, T, D, K, C, H, W, ps)
        ctx.x_requires_grad = ctx.needs_input_grad[0]
        ctx.save_for_backward(patches, wb)
        return X

    @staticmethod
    def backward(ctx, gX):
        patches, wb = ctx.saved_tensors
        w, b, cls, pos = ctx.params
        B, T, D, K, C, H, W, ps = ctx.dims
        gX = gX.contiguous()
        gpatch = ops.vit_embed_bwd(gX, B, T + 1, D,
                                   grad_buffer(cls) if _wants(cls) else None,
                                   grad_buffer(pos) if _wants(pos) else None,
                                   grad_buffer(b) if _wants(b) else None)
        if _wants(w):
            dw = grad_buffer(w).view(D, K)
            ops.gemm(D, K, B * T, gpatch, D, patches, patches.stride(0), dw, K,
                     a_mode=L.OPND_MNMAJOR, b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC)
        grads_done(w, b, cls, pos)
        dx = None
        if ctx.x_requires_grad:
            # Grad-CAM input saliency (grad_cam_visualization.py:374, 401-413): fp32
            # d patches = gpatch W (MFMA GEMM), then the unpatchify permutation.
            dpatch = _empty((B * T, K), F32, gX.device)
            ops.gemm(B * T, K, D, gpatch, D, wb, K, dpatch, K, b_mode=L.OPND_MNMAJOR,
                     epilogue=L.EPI_F32)
            dx = ops.unpatchify_f32(dpatch, B, C, H, W, ps)
        return dx, None, None, None, None, None


# ---------------------------------------------------------------------------- ViT block
def _linear_wgrad(dy_bf, x_bf, w, rows):
    """w.grad [N, K] += dy^T x  (dy [rows, N], x [rows, K] with any row stride, both bf16)."""
    N, K = w.shape
    ops.gemm(N, K, rows, dy_bf, N, x_bf, x_bf.stride(0), grad_buffer(w), K,
             a_mode=L.OPND_MNMAJOR, b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC)


def _ln_fwd(x2d, norm, rows, D, out_bf):
    mean = _empty((rows,), F32, x2d.device)
    rstd = _empty((rows,), F32, x2d.device)
    ops.layernorm_fwd(x2d, D, rows, D, norm.weight, norm.bias, norm.eps, out_bf, D, True, mean,
                      rstd)
    return mean, rstd


def _ln_bwd(dy_bf, x2d, mean, rstd, norm, rows, D, g, g_bf, gsum=False, batch=None):
    """LayerNorm backward; dgamma / dbeta reductions go to `batch` (a PartialReductions) when
    given (the caller reports the parameters done after flushing it)."""
    gsp = ops.layernorm_bwd(dy_bf, D, True, x2d, D, mean, rstd, norm.weight, rows, D, g, D, g_bf,
                            grad_buffer(norm.weight) if _wants(norm.weight) else None,
                            grad_buffer(norm.bias) if _wants(norm.bias) else None, gsum=gsum,
                            batch=batch)
    if batch is None:
        grads_done(norm.weight, norm.bias)
    return gsp


def _colsum_of_grad(g, out, batch=None):
    """out += column sums of an fp32 residual-stream gradient: from the partial sums its
    producing LayerNorm backward emitted (stashed on the tensor), else a colsum pass."""
    gsp = getattr(g, "_dfu_colsum", None)
    if gsp is None:
        gsp = ops.colsum_partial(g.reshape(-1, g.shape[-1]))
    if batch is not None:
        batch.add(gsp, out, gsp.shape[1])
    else:
        ops.reduce_partials_add(gsp, out)


def _bf16_of_grad(g):
    """bf16 copy of an fp32 residual-stream gradient: reuse the one the producing LayerNorm
    backward emitted (stashed on the tensor) or cast."""
    gb = getattr(g, "_dfu_bf16", None)
    if gb is not None and gb.shape == g.shape:
        return gb
    return ops.cast_rows_bf16(g.reshape(-1, g.shape[-1])).view(g.shape)


def _linear_dgrad(rows, N, K, g, weight, w_rows, out, epilogue=L.EPI_BF16, **kw):
    """out[rows, N] = epilogue(g[rows, K] @ W[K, N]) for a Linear weight W [out=K][in=N] (bf16
    shadow w_rows).  With the transposed shadow (weight_bf16_T) the weight operand is
    K-contiguous (B = W^T [N][K]); otherwise W itself is read MN-major.  The same products in
    the same K order either way (bitwise equal results); the K-contiguous operand is 12-15%
    faster on the ViT-B/16 shapes (tools/gemm_one.py fc1_dgrad vs fc1_dgrad_t)."""
    wT = weight_bf16_T(weight)
    if wT is not None:
        ops.gemm(rows, N, K, g, K, wT, K, out, N, epilogue=epilogue, **kw)
    else:
        ops.gemm(rows, N, K, g, K, w_rows, N, out, N, b_mode=L.OPND_MNMAJOR, epilogue=epilogue,
                 **kw)


# Tile of the ViT's bf16x3 forward GEMMs (tripled K): 8 = the persistent phased 256x256 (with
# the fused fc1 + GELU triple epilogue, DFU_EPI_X3_GELU); DFU_X3_TILE=0: the cost model's pick
# and a separate GELU split pass (A/B).
_X3_TILE = int(os.environ.get("DFU_X3_TILE", "8"))
# The GEMMs to D = 768 columns (proj and fc2 forward, the fc1 / proj / qkv input gradients) run
# on the persistent 192 x 256 tile (tile 9: 198 tiles at M = 12608 instead of 150 of 256 rows
# for 256 CUs; 8-16 % faster standalone, tools/gpu_tile192.sh) when the ViT runs alone.  Inside
# the two-stream fusion step the 256-row tile's idle CUs run the ResNet's kernels: there tile 9
# measured 19.11 vs 18.97 ms per step (same box, three rounds), so it keeps the 256-row plan.
# (The parity mode's fp16 proj / fc2 follow their own tuned entries, tile 9: 20.79-20.85 vs
# 20.83-20.87 ms with the 256-row plan, same box.)
# DFU_GEMM_NO_T192=1: the 256-row plan everywhere (A/B).
_NO_T192 = os.environ.get("DFU_GEMM_NO_T192", "0") != "0"


def _t768():
    """Tile hint for a ViT GEMM with N = 768 output columns (0: the tuned plan)."""
    return 9 if _concurrent_encoders[0] == 0 and not _NO_T192 else 0

# fc1.bias gradient from the dGELU epilogue's column sums, in the fusion step too (round 6: 0.1 ms
# faster per step there on the final tree; DFU_DGELU_COLSUM=0: a colsum pass everywhere,
# 1: the epilogue's sums only when the ViT runs alone, the round-3 setting)
_DGELU_COLSUM = int(os.environ.get("DFU_DGELU_COLSUM", "2"))


class ViTBlockFn(torch.autograd.Function):
    """timm Block (pre-norm, qkv_bias, SDPA, exact GELU, no LayerScale, drop_path 0)."""

    @staticmethod
    def forward(ctx, x, *params_and_mod):
        blk = params_and_mod[-1]
        bm = blk._modules  # (nn.Module attributes are slow __getattr__ lookups)
        attn, mlp = bm["attn"], bm["mlp"]
        B, T, D = x.shape
        rows = B * T
        H = attn.num_heads
        dh = D // H
        dev = x.device
        x = x.detach().contiguous()
        x2 = x.view(rows, D)
        # the Linears' weights: the Function's own inputs (models.vit.Block._params order)
        wqkv = weight_bf16_rows(params_and_mod[2])
        wproj = weight_bf16_rows(params_and_mod[4])
        wfc1 = weight_bf16_rows(params_and_mod[8])
        wfc2 = weight_bf16_rows(params_and_mod[10])
        Dh = wfc1.shape[0]
        bias = lambda lin: lin.bias.detach() if lin.bias is not None else None  # noqa: E731
        mode = stage_mode(blk)
        if mode == "bf16x3":
            return ViTBlockFn._forward_x3(ctx, blk, x2, B, T, D, H, dh, rows, wqkv, wproj, wfc1,
                                          wfc2, bias)
        if mode == "fp16":
            return ViTBlockFn._forward_h16(ctx, blk, x2, B, T, D, H, dh, rows, wqkv, wproj, wfc1,
                                           wfc2, bias)
        # attention branch
        xn1 = _empty((rows, D), BF16, dev)
        m1, r1 = _ln_fwd(x2, blk.norm1, rows, D, xn1)
        qkv = _empty((rows, 3 * D), BF16, dev)
        ops.gemm(rows, 3 * D, D, xn1, D, wqkv, D, qkv, 3 * D, epilogue=L.EPI_BF16,
                 bias=bias(attn.qkv))
        o, lse = ops.attention_fwd(qkv, B, T, H, dh, attn.scale)
        xm = _empty((rows, D), F32, dev)
        t768 = _t768()
        ops.gemm(rows, D, D, o, D, wproj, D, xm, D, epilogue=L.EPI_F32_RESID, bias=bias(attn.proj),
                 aux=x2, ldaux=D, tile=t768)
        # MLP branch
        xn2 = _empty((rows, D), BF16, dev)
        m2, r2 = _ln_fwd(xm, blk.norm2, rows, D, xn2)
        dgl = _empty((rows, Dh), BF16, dev)
        h = _empty((rows, Dh), BF16, dev)
        ops.gemm(rows, Dh, D, xn2, D, wfc1, D, h, Dh, epilogue=L.EPI_BF16_GELU, bias=bias(mlp.fc1),
                 aux_out=dgl, ldaux_out=Dh)
        xo = _empty((B, T, D), F32, dev)
        ops.gemm(rows, D, Dh, h, Dh, wfc2, Dh, xo.view(rows, D), D, epilogue=L.EPI_F32_RESID,
                 bias=bias(mlp.fc2), aux=xm, ldaux=D, tile=t768)
        ctx.t768 = t768
        ctx.blk = blk
        ctx.dims = (B, T, D, H, dh, Dh)
        ctx.out_ref = weakref.ref(xo)
        ctx.beside = _VIT_WGRAD_STREAM and _concurrent_encoders[0] == 0
        ctx.save_for_backward(x2, xn1, m1, r1, qkv, o, lse, xm, xn2, m2, r2, dgl, h, wqkv,
                              wproj, wfc1, wfc2)
        return xo

    @staticmethod
    def _forward_x3(ctx, blk, x2, B, T, D, H, dh, rows, wqkv, wproj, wfc1, wfc2, bias):
        """bf16x3 forward: the four Linears on split-bf16 triples (K tripled), fp32 GEMM
        outputs, fp32-accurate attention (split-bf16 MFMA); saves the same bf16 tensors as the
        bf16 forward."""
        attn, mlp = blk.attn, blk.mlp
        dev = x2.device
        Dh = wfc1.shape[0]

        def ln_x3(xsrc, norm):
            t3 = _empty((rows, 3 * D), BF16, dev)
            tb = _empty((rows, D), BF16, dev)
            mean = _empty((rows,), F32, dev)
            rstd = _empty((rows,), F32, dev)
            ops.layernorm_fwd_x3(xsrc, D, rows, D, norm.weight, norm.bias, norm.eps, t3, tb, mean,
                                 rstd)
            return t3, tb, mean, rstd

        tl = _X3_TILE
        # the two GEMMs to D = 768 columns (proj, fc2) on the 192 x 256 persistent tile when
        # the ViT runs alone (_t768: projx3 61.6-62.6 vs 71.1-71.2 us, fc2x3 250.8-251.0 vs
        # 270.9-271.9 us standalone; in the fusion step within noise of tile 8)
        tl_d = (_t768() or tl) if tl == 8 else tl
        ctx.t768 = _t768()
        xn1_3, xn1, m1, r1 = ln_x3(x2, blk.norm1)
        qkvf = _empty((rows, 3 * D), F32, dev)
        ops.gemm(rows, 3 * D, 3 * D, xn1_3, 3 * D, weight_x3_rows(attn.qkv.weight), 3 * D, qkvf,
                 3 * D, epilogue=L.EPI_F32, bias=bias(attn.qkv), tile=tl, x3=True)
        del xn1_3
        qkv = _empty((rows, 3 * D), BF16, dev)  # written by the attention kernel
        o3, o, lse = ops.attention_fwd_f32(qkvf, B, T, H, dh, attn.scale, qkv_bf16=qkv)
        del qkvf
        xm = _empty((rows, D), F32, dev)
        ops.gemm(rows, D, 3 * D, o3, 3 * D, weight_x3_rows(attn.proj.weight), 3 * D, xm, D,
                 epilogue=L.EPI_F32_RESID, bias=bias(attn.proj), aux=x2, ldaux=D, tile=tl_d,
                 x3=True)
        del o3
        xn2_3, xn2, m2, r2 = ln_x3(xm, blk.norm2)
        dgl = _empty((rows, Dh), BF16, dev)  # bf16 gelu'(pre): the DGELU factor
        if tl == 8:
            # fc1 + GELU with the split triple written by the epilogue; the backward's bf16 h
            # is the triple's hi segment (a strided view)
            h3 = _empty((rows, 3 * Dh), BF16, dev)
            ops.gemm(rows, Dh, 3 * D, xn2_3, 3 * D, weight_x3_rows(mlp.fc1.weight), 3 * D, h3,
                     3 * Dh, epilogue=L.EPI_X3_GELU, bias=bias(mlp.fc1), aux_out=dgl,
                     ldaux_out=Dh, tile=tl, x3=True)
            h = h3[:, :Dh]
        else:
            hf = _empty((rows, Dh), F32, dev)
            ops.gemm(rows, Dh, 3 * D, xn2_3, 3 * D, weight_x3_rows(mlp.fc1.weight), 3 * D, hf,
                     Dh, epilogue=L.EPI_F32, bias=bias(mlp.fc1), tile=tl, x3=True)
            h3, h, dgl = ops.gelu_x3(hf)
            del hf
        del xn2_3
        xo = _empty((B, T, D), F32, dev)
        ops.gemm(rows, D, 3 * Dh, h3, 3 * Dh, weight_x3_rows(mlp.fc2.weight), 3 * Dh,
                 xo.view(rows, D), D, epilogue=L.EPI_F32_RESID, bias=bias(mlp.fc2), aux=xm,
                 ldaux=D, tile=tl_d, x3=True)
        ctx.blk = blk
        ctx.dims = (B, T, D, H, dh, Dh)
        ctx.out_ref = weakref.ref(xo)
        ctx.beside = _VIT_WGRAD_STREAM and _concurrent_encoders[0] == 0
        ctx.save_for_backward(x2, xn1, m1, r1, qkv, o, lse, xm, xn2, m2, r2, dgl, h, wqkv,
                              wproj, wfc1, wfc2)
        return xo

    @staticmethod
    def _forward_h16(ctx, blk, x2, B, T, D, H, dh, rows, wqkv, wproj, wfc1, wfc2, bias):
        """fp16 forward: the four Linears on fp16 operands (fp32 accumulate; persistent
        256 x 256 tile, 192 x 256 for the N = 768 GEMMs when the ViT runs alone), the fp16
        attention, fp32 residual stream; saves the same bf16 tensors as the bf16 forward (every
        fp16 producer also writes the bf16 copy)."""
        bm = blk._modules
        attn, mlp = bm["attn"], bm["mlp"]
        am, mm = attn._modules, mlp._modules
        dev = x2.device
        Dh = wfc1.shape[0]
        F16 = torch.float16

        def ln(xsrc, norm):
            t16 = _empty((rows, D), F16, dev)
            tb = _empty((rows, D), BF16, dev)
            mean = _empty((rows,), F32, dev)
            rstd = _empty((rows,), F32, dev)
            ops.layernorm_fwd_h16(xsrc, D, rows, D, norm.weight, norm.bias, norm.eps, t16, tb,
                                  mean, rstd)
            return t16, tb, mean, rstd

        h16 = L.OPERAND_F16
        ctx.t768 = _t768()
        tl_d = ctx.t768 or 8
        xn1_16, xn1, m1, r1 = ln(x2, bm["norm1"])
        # qkv in fp16 only: the attention backward rounds it to bf16 while staging
        # (same-box A/B: 21.56-21.62 vs 21.72-21.75 ms with the bf16 copy written too)
        qkv = _empty((rows, 3 * D), F16, dev)
        ops.gemm(rows, 3 * D, D, xn1_16, D, weight_f16_rows(am["qkv"].weight), D, qkv, 3 * D,
                 epilogue=L.EPI_F16_DUAL, bias=bias(am["qkv"]), tile=8, operand_type=h16)
        del xn1_16
        o16, o, lse = ops.attention_fwd_f16(qkv, B, T, H, dh, attn.scale)
        xm = _empty((rows, D), F32, dev)
        ops.gemm(rows, D, D, o16, D, weight_f16_rows(am["proj"].weight), D, xm, D,
                 epilogue=L.EPI_F32_RESID, bias=bias(am["proj"]), aux=x2, ldaux=D, tile=tl_d,
                 operand_type=h16)
        del o16
        xn2_16, xn2, m2, r2 = ln(xm, bm["norm2"])
        # fc1 + GELU: [fp16 gelu | bf16 gelu] (fc2's operand, the backward's h) + bf16 gelu'
        h2 = _empty((rows, 2 * Dh), BF16, dev)
        dgl = _empty((rows, Dh), BF16, dev)
        ops.gemm(rows, Dh, D, xn2_16, D, weight_f16_rows(mm["fc1"].weight), D, h2, 2 * Dh,
                 epilogue=L.EPI_F16_GELU, bias=bias(mm["fc1"]), aux_out=dgl, ldaux_out=Dh, tile=8,
                 operand_type=h16)
        del xn2_16
        h = h2[:, Dh:]
        xo = _empty((B, T, D), F32, dev)
        ops.gemm(rows, D, Dh, h2, 2 * Dh, weight_f16_rows(mm["fc2"].weight), Dh, xo.view(rows, D),
                 D, epilogue=L.EPI_F32_RESID, bias=bias(mm["fc2"]), aux=xm, ldaux=D, tile=tl_d,
                 operand_type=h16)
        ctx.blk = blk
        ctx.dims = (B, T, D, H, dh, Dh)
        ctx.out_ref = weakref.ref(xo)
        ctx.beside = _VIT_WGRAD_STREAM and _concurrent_encoders[0] == 0
        ctx.save_for_backward(x2, xn1, m1, r1, qkv, o, lse, xm, xn2, m2, r2, dgl, h, wqkv,
                              wproj, wfc1, wfc2)
        return xo

    @staticmethod
    def backward(ctx, gout):
        (x2, xn1, m1, r1, qkv, o, lse, xm, xn2, m2, r2, dgl, h, wqkv, wproj, wfc1,
         wfc2) = ctx.saved_tensors
        blk = ctx.blk
        # modules resolved once (each nn.Module attribute is a slow __getattr__ lookup)
        bm = blk._modules
        attn, mlp = bm["attn"], bm["mlp"]
        am, mm = attn._modules, mlp._modules
        qkv_l, proj_l, fc1_l, fc2_l = am["qkv"], am["proj"], mm["fc1"], mm["fc2"]
        norm1, norm2 = bm["norm1"], bm["norm2"]
        B, T, D, H, dh, Dh = ctx.dims
        rows = B * T
        dev = x2.device
        g = gout.contiguous()
        if g.dtype != F32:
            g = g.float()
        # The LayerNorm backwards below update the residual-stream gradient IN PLACE.  That is
        # safe for a gradient only this Function sees (another block's or TokenNormFn's
        # output); when the block output carries a tensor hook or retain_grad (Grad-CAM's
        # 'blocks.*' hooks, user code), the hook may hold that very tensor: work on a copy.
        out = ctx.out_ref()
        if g is gout and out is not None and (out.retains_grad or getattr(out, "_backward_hooks",
                                                                           None)):
            g = g.clone()
        g2 = g.view(rows, D)
        gb = _bf16_of_grad(gout if gout.dtype == F32 else g).view(rows, D)
        # the block's eight "sum per-block partials into a gradient vector" reductions (bias
        # column sums, LayerNorm dgamma / dbeta) run as one launch at the end (PartialReductions)
        red = ops.PartialReductions()
        # weight gradients (and the bias column sums of the tensors they read) on the wgrad
        # stream, beside the input-gradient chain (wgrad_stream); their reductions batch apart
        # (only when some weight gradient is wanted: a fork with no work -- Grad-CAM's backward
        # through frozen weights -- would leave the stream unjoined, which a graph capture
        # rejects; the streams that wrote gradients are joined by join_grad_streams)
        wants_w = any(_wants(lin.weight) or _wants(lin.bias)
                      for lin in (fc1_l, fc2_l, qkv_l, proj_l))
        bw = _Beside(wgrad_stream(dev) if (ctx.beside and g.is_cuda and wants_w) else None)
        red_w = ops.PartialReductions() if bw.ws is not None else red

        def wgrad(lin, dy, x, width=None, partial=None):
            def fn():
                if _wants(lin.weight):
                    _linear_wgrad(dy, x, lin.weight, rows)
                if width is not None and _wants(lin.bias):
                    red_w.add(ops.colsum_partial(dy) if partial is None else partial,
                              grad_buffer(lin.bias), width)
                grads_done(lin.weight)
            bw.run(fn, dy, x, *(() if partial is None else (partial,)))

        # ---- MLP branch: x_out = x_mid + fc2(gelu(fc1(norm2(x_mid))))
        wgrad(fc2_l, gb, h)
        dh_pre = _empty((rows, Dh), BF16, dev)
        # fc1.bias's gradient = column sums of dh_pre: reduced in the dGELU epilogue (per 128-row
        # half of each 256-row tile) where the plan is the persistent 256x256 tile, else a pass
        # (thermal-only 0.13 ms faster per step; the fusion step 0.07 ms slower in round 3 and
        # 0.1 ms faster on the round-6 tree: _DGELU_COLSUM)
        cs1 = None
        if (_DGELU_COLSUM == 2 or (_DGELU_COLSUM and ctx.beside)) and _wants(fc1_l.bias) and \
                g.is_cuda:
            cs1 = _empty((2 * ((rows + 255) // 256), Dh), F32, dev)
            try:
                _linear_dgrad(rows, Dh, D, gb, fc2_l.weight, wfc2, dh_pre,
                              epilogue=L.EPI_BF16_DGELU, aux=dgl, ldaux=Dh, stats=cs1)
            except L.DfuError as e:
                if e.code != L.DFU_E_UNSUPPORTED:
                    raise
                cs1 = None
        if cs1 is None:
            _linear_dgrad(rows, Dh, D, gb, fc2_l.weight, wfc2, dh_pre,
                          epilogue=L.EPI_BF16_DGELU, aux=dgl, ldaux=Dh)
        if _wants(fc2_l.bias):
            _colsum_of_grad(gout if gout.dtype == F32 else g, grad_buffer(fc2_l.bias), red)
        wgrad(fc1_l, dh_pre, xn2, Dh, partial=cs1)
        dxn2 = _empty((rows, D), BF16, dev)
        _linear_dgrad(rows, D, Dh, dh_pre, fc1_l.weight, wfc1, dxn2, tile=ctx.t768)
        gmb = _empty((rows, D), BF16, dev)
        gsp = _ln_bwd(dxn2, xm, m2, r2, norm2, rows, D, g2, gmb,
                      gsum=_wants(proj_l.bias), batch=red)  # g2 := g_mid (in place)
        # ---- attention branch: x_mid = x_in + proj(attn(norm1(x_in)))
        wgrad(proj_l, gmb, o)
        do = _empty((rows, D), BF16, dev)
        _linear_dgrad(rows, D, D, gmb, proj_l.weight, wproj, do, tile=ctx.t768)
        if _wants(proj_l.bias):
            red.add(gsp, grad_buffer(proj_l.bias), D)
        dqkv = ops.attention_bwd(qkv, o, do, lse, B, T, H, dh, attn.scale)
        wgrad(qkv_l, dqkv, xn1, 3 * D)
        dxn1 = _empty((rows, D), BF16, dev)
        _linear_dgrad(rows, D, 3 * D, dqkv, qkv_l.weight, wqkv, dxn1, tile=ctx.t768)
        gib = _empty((B, T, D), BF16, dev)
        gsp = _ln_bwd(dxn1, x2, m1, r1, norm1, rows, D, g2, gib.view(rows, D),
                      gsum=True, batch=red)  # g2 := g_in
        red.flush()
        if red_w is not red:
            bw.run(red_w.flush)
        grads_done(fc2_l.bias, fc1_l.bias, norm2.weight, norm2.bias,
                   proj_l.bias, qkv_l.bias, norm1.weight, norm1.bias)
        gin = g.view(B, T, D)
        gin._dfu_bf16 = gib
        gin._dfu_colsum = gsp  # the previous block's fc2.bias gradient, pre-reduced
        n_params = len(ctx.needs_input_grad) - 2
        return (gin,) + (None,) * n_params + (None,)


class TokenNormFn(torch.autograd.Function):
    """timm final LayerNorm + token pooling x[:, 0]: only the class-token rows are normalised
    (LayerNorm is per token, so this equals norm(x)[:, 0])."""

    @staticmethod
    def forward(ctx, x, gamma, beta, norm):
        B, T, D = x.shape
        x = x.detach().contiguous()
        out = _empty((B, D), F32, x.device)
        mean = _empty((B,), F32, x.device)
        rstd = _empty((B,), F32, x.device)
        ops.layernorm_fwd(x, T * D, B, D, norm.weight, norm.bias, norm.eps, out, D, False, mean,
                          rstd)
        ctx.norm = norm
        ctx.save_for_backward(x, mean, rstd)
        return out

    @staticmethod
    def backward(ctx, g):
        if g.is_cuda:  # produced on the fusion head's stream; the ViT may run on a side stream
            arm_backward_join()
            g.record_stream(ops.current_stream())
        x, mean, rstd = ctx.saved_tensors
        norm = ctx.norm
        B, T, D = x.shape
        g = g.contiguous().float()
        gx = _empty((B, T, D), F32, x.device)
        ops.zero_(gx)
        gxb = _empty((B, T, D), BF16, x.device)
        ops.zero_(gxb)
        gsp = ops.layernorm_bwd(g, D, False, x, T * D, mean, rstd, norm.weight, B, D, gx, T * D,
                                gxb, grad_buffer(norm.weight) if _wants(norm.weight) else None,
                                grad_buffer(norm.bias) if _wants(norm.bias) else None, gsum=True)
        grads_done(norm.weight, norm.bias)
        gx._dfu_bf16 = gxb
        gx._dfu_colsum = gsp  # only the class-token rows are non-zero: their sums are the total
        return gx, None, None, None


# --------------------------------------------------------------------------- fusion head
class LinearFn(torch.autograd.Function):
    """y = x W^T + b (fp32 out) for the late-fusion MLP and replaced heads.

    Small problems (the fusion head: rows = batch) run in exact fp32 (dfu_gemm_f32) — the head
    is 0.003 % of the step's FLOPs and fp32 keeps the logits free of bf16 rounding; large ones
    use the bf16 MFMA GEMM."""

    SMALL_MACS = 1 << 31

    @staticmethod
    def forward(ctx, x, w, b, relu):
        lead = x.shape[:-1]
        K = x.shape[-1]
        N = w.shape[0]
        x2 = x.detach().reshape(-1, K)
        rows = x2.shape[0]
        bias = b.detach() if b is not None else None
        small = rows * N * K <= LinearFn.SMALL_MACS
        y = _empty((rows, N), F32, x.device)
        if small:
            xf = x2.float().contiguous()
            wf = w.detach()
            ops.gemm_f32(rows, N, K, xf, K, 1, wf, K, 1, y, N, bias=bias, relu=relu)
            saved = (xf, wf)
        else:
            xb = x2.contiguous() if x2.dtype == BF16 else ops.cast_rows_bf16(x2)
            wb = weight_bf16_rows(w)
            ops.gemm(rows, N, K, xb, K, wb, K, y, N, epilogue=L.EPI_F32, bias=bias)
            if relu:
                y = ops.relu_fwd(y)
            saved = (xb, wb)
        ctx.small = small
        ctx.relu = relu
        ctx.params = (w, b)
        ctx.x_dtype = x.dtype
        ctx.lead = lead
        ctx.save_for_backward(*saved, y if relu else None)
        return y.view(*lead, N)

    @staticmethod
    def backward(ctx, gy):
        xs, ws, y = ctx.saved_tensors
        w, b = ctx.params
        rows, K = xs.shape
        N = ws.shape[0]
        g = gy.reshape(rows, N)
        if g.dtype != F32:
            g = g.float()
        g = g.contiguous()
        if ctx.relu:
            g = ops.relu_bwd(g, y)
        dx = None
        if ctx.small:
            if ctx.needs_input_grad[0]:
                dx = _empty((rows, K), F32, xs.device)
                # dX[r][k] = sum_n g[r][n] W[n][k]
                ops.gemm_f32(rows, K, N, g, N, 1, ws, 1, K, dx, K)
                if ctx.x_dtype != F32:
                    dx = dx.to(ctx.x_dtype)
                dx = dx.view(*ctx.lead, K)
            if _wants(w):
                # dW[n][k] += sum_r g[r][n] X[r][k]
                ops.gemm_f32(N, K, rows, g, 1, N, xs, 1, K, grad_buffer(w), K, accumulate=True)
        else:
            gb = ops.cast_rows_bf16(g, ld_out=max(8, (N + 7) // 8 * 8))
            if ctx.needs_input_grad[0]:
                Np = gb.shape[1]
                if Np != N:
                    wp = _empty((Np, K), BF16, xs.device)
                    ops.zero_(wp)
                    wp[:N].copy_(ws)
                else:
                    wp = ws
                out_bf = ctx.x_dtype == BF16
                dx = _empty((rows, K), BF16 if out_bf else F32, xs.device)
                ops.gemm(rows, K, Np, gb, Np, wp, K, dx, K, b_mode=L.OPND_MNMAJOR,
                         epilogue=L.EPI_BF16 if out_bf else L.EPI_F32)
                dx = dx.view(*ctx.lead, K)
            if _wants(w):
                ops.gemm(N, K, rows, gb, gb.shape[1], xs, K, grad_buffer(w), K,
                         a_mode=L.OPND_MNMAJOR, b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC)
        if _wants(b):
            ops.colsum_add(g, grad_buffer(b))
        grads_done(w, b)
        return dx, None, None, None


class ReLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = ops.relu_fwd(x.detach().contiguous())
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        return ops.relu_bwd(g.contiguous().to(y.dtype), y)


class DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed, offset):
        y, mask = ops.dropout_fwd(x.detach().contiguous(), p, seed, offset)
        ctx.p = p
        ctx.save_for_backward(mask)
        return y

    @staticmethod
    def backward(ctx, g):
        (mask,) = ctx.saved_tensors
        return ops.dropout_bwd(g.contiguous(), mask, ctx.p), None, None, None


class ConcatFn(torch.autograd.Function):
    """torch.cat([rgb_feat, thermal_feat], 1) (train_multimodal_fusion.py:321), fp32."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.dims = (a.shape[1], b.shape[1])
        ctx.dtypes = (a.dtype, b.dtype)
        return ops.concat2_f32(a.detach().float(), b.detach().float())

    @staticmethod
    def backward(ctx, g):
        if g.is_cuda:
            arm_backward_join()
        Na, Nb = ctx.dims
        ga, gb = ops.split2_f32(g, Na, Nb)
        if ctx.dtypes[0] != F32:
            ga = ga.to(ctx.dtypes[0])
        if ctx.dtypes[1] != F32:
            gb = gb.to(ctx.dtypes[1])
        return ga, gb


class CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, weight):
        z = logits.detach().contiguous().float()
        loss = _empty((1,), F32, z.device)
        dz = torch.empty_like(z)
        ops.ce_weighted_fwd(z, labels.contiguous(), weight, loss, dz)
        ctx.save_for_backward(dz)
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        (dz,) = ctx.saved_tensors
        return ops.ce_weighted_bwd(dz, g.reshape(1).float().contiguous()), None, None
