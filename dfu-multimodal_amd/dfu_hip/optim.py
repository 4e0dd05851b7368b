"""FusedAdamW: torch.optim.AdamW semantics (train_multimodal_fusion.py:347, 380:
AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4), betas (0.9, 0.999), eps 1e-8) as ONE
kernel launch over a flat fp32 parameter buffer.

At construction the parameters are moved into one contiguous fp32 buffer (``p.data`` becomes a
view) and ``p.grad`` into a matching flat gradient buffer, so:
  * the optimizer step is a single HBM-streaming kernel (5 fp32 passes over 443 MB at B=64);
  * zero_grad is one hipMemsetAsync;
  * the weight-gradient GEMM epilogues accumulate straight into the flat buffer, whose
    contiguous slices are what data-parallel all-reduce buckets send (dfu_hip.parallel);
  * the step counter lives on the device, so the whole step can be captured in a HIP graph;
  * the same kernel writes a bf16 shadow of every updated parameter (``FlatParams.shadow``):
    Linear and 1x1-conv weights are consumed by the GEMMs straight from it (no cast kernels);
    weights whose input-gradient GEMM asked for it (functional.weight_bf16_T: the ViT Linears)
    also get a transposed bf16 copy, refreshed right after the AdamW kernel by ONE batched
    transpose launch, so that GEMM reads its weight operand K-contiguous;
  * spatial conv weights (4-D, R*S > 1, C % 8 == 0) are STORED channels-last, i.e. in the
    implicit-GEMM order KRSC, while keeping their OIHW shape (``p`` is a permuted view): the
    shadow is then the 3x3 conv's bf16 weight operand as is, and the weight-gradient GEMM
    accumulates straight into ``p.grad`` (no per-step pack / zero / permute-add kernels).
    A parameter changed outside the optimizer (load_state_dict, in-place edits through the
    parameter) bumps its version counter and is re-cast on its next use
    (functional.weight_bf16_rows); edits through ``p.data`` bypass that counter — call
    ``FlatParams.refresh_shadow()`` after those.
"""
import os
import warnings
import weakref

import torch
import torch.distributed as dist

from . import functional as Fn
from . import ops

# elements: every tensor view starts 128-byte aligned, and a parameter's 32-element blocks are
# the flat buffer's (the interleaved-pair x3 shadow's blocks, enable_x3)
_ALIGN = 32


def _dp_world():
    """Whether this process is one rank of a multi-rank process group."""
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _aligned(n):
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def stores_krsc(p):
    """Whether FlatParams stores parameter p channels-last (KRSC): spatial conv weights whose
    channel count the implicit-GEMM conv takes (the stem's 3-channel 7x7 keeps OIHW)."""
    return p.dim() == 4 and p.shape[2] * p.shape[3] > 1 and p.shape[1] % 8 == 0


def x3_pair_weight(p):
    """Whether the bf16x3 ResNet forward reads conv weight p as interleaved pairs from the
    optimizer's x3 shadow (FlatParams.enable_x3): a 1x1 conv weight, or a channels-last
    spatial one, of C % 32 == 0 input channels (every ResNet-50 conv but the stem)."""
    return p.dim() == 4 and p.shape[1] % 32 == 0 and (p.shape[2] * p.shape[3] == 1
                                                        or stores_krsc(p))


def _view(flat, o, p, krsc):
    """Parameter-shaped view of flat[o:o+n]: OIHW order, or KRSC memory seen as OIHW."""
    v = flat[o:o + p.numel()]
    if krsc:
        K, C, R, S = p.shape
        return v.view(K, R, S, C).permute(0, 3, 1, 2)
    return v.view_as(p)


class FlatParams:
    """Contiguous fp32 storage for a list of parameters and their gradients."""

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("FlatParams: no trainable parameters")
        dev = self.params[0].device
        self.offsets = []
        self.krsc = [stores_krsc(p) for p in self.params]
        off = 0
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError("FusedAdamW: fp32 master parameters expected")
            self.offsets.append(off)
            off += _aligned(p.numel())
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        self.shadow = torch.zeros(off, dtype=torch.bfloat16, device=dev) if dev.type == "cuda" \
            else None
        self.shadow16 = None  # fp16 shadow, from the first fp16-stage forward on (enable_f16)
        self.shadow_x3 = None  # interleaved-pair bf16x3 conv weights (enable_x3)
        self.x3_lo = self.x3_hi = 0
        self.gen = 0         # bumped whenever every shadow is rewritten (step, refresh)
        self.t_params = []   # parameters with a transposed (p._dfu_shadow_T) or flipped
        self.t_pairs = []    # (p._dfu_shadow_F) shadow, and their (src, dst) transpose jobs
        self.t_jobs = None
        self.t_pairs_of = {}  # id(p) -> its transpose jobs
        self._range_jobs = {}  # (lo, hi) -> (jobs of the parameters inside, jobs of the rest)
        with torch.no_grad():
            for p, o, kr in zip(self.params, self.offsets, self.krsc):
                view = _view(self.data, o, p, kr)
                view.copy_(p.data)
                p.data = view
                p.grad = _view(self.grad, o, p, kr)
                if self.shadow is not None:
                    # [out][in...] rows in storage order (KRSC for channels-last conv weights)
                    p._dfu_shadow = self.shadow[o:o + p.numel()].view(p.shape[0], -1)
                    p._dfu_flat = self
        self.refresh_shadow()

    def refresh_shadow(self):
        """Re-cast every parameter into the bf16 (and fp16) shadow and mark it current."""
        if self.shadow is None:
            return
        ops.cast_rows_bf16(self.data.view(1, -1), out=self.shadow.view(1, -1))
        for p in self.params:
            p._dfu_shadow_version = p._version
        if self.shadow16 is not None:
            self._cast_f16()
        if self.shadow_x3 is not None:
            self._split_x3()
        self.shadows_rewritten()

    def _cast_f16(self):
        ops.cast_rows_f16(self.data.view(1, -1), out=self.shadow16.view(1, -1))
        for p in self.params:
            p._dfu_shadow16_version = p._version

    def enable_f16(self):
        """Keep an fp16 shadow of every parameter from now on (the "fp16" stage precision's
        GEMM operands, functional.weight_f16_rows): cast once here, then written by every AdamW
        step beside the bf16 shadow (2 B per parameter)."""
        if self.shadow16 is not None or self.shadow is None:
            return
        self.shadow16 = torch.empty(self.numel, dtype=torch.float16, device=self.data.device)
        for p, o in zip(self.params, self.offsets):
            p._dfu_shadow16 = self.shadow16[o:o + p.numel()].view(p.shape[0], -1)
        self._cast_f16()

    def enable_x3(self):
        """Keep the interleaved-pair split (dfu_gemm_desc.x3_pairs B operand: per 32 elements
        [hi 32 | lo 32]) of every conv weight x3_pair_weight accepts from now on: split once
        here, then written by every AdamW step beside the bf16 shadow for the flat span those
        weights occupy (4 B per element of it; the ResNet's 23.5M), so the bf16x3 forward
        reads its conv weights as they are instead of ~52 per-layer split / pack launches on
        its critical stream (functional.conv_weight_x3)."""
        if self.shadow_x3 is not None or self.shadow is None:
            return
        idx = [i for i, p in enumerate(self.params) if x3_pair_weight(p)]
        if not idx:
            return
        self.x3_lo = self.offsets[idx[0]]
        self.x3_hi = self.offsets[idx[-1]] + _aligned(self.params[idx[-1]].numel())
        # the span also covers any parameter registered between the first and last x3 weight
        # (contiguous in the reference ResNet: BN vectors only); report a model whose span
        # carries much more than its conv weights
        covered = sum(_aligned(self.params[i].numel()) for i in idx)
        self.x3_extra = (self.x3_hi - self.x3_lo) - covered
        if self.x3_extra > max(1 << 20, covered // 10):
            warnings.warn(f"FusedAdamW x3 shadow: the conv-weight span holds {self.x3_extra} "
                          f"elements of other parameters beside {covered} conv-weight "
                          f"elements (4 B of memory and AdamW writes each per step)")
        self.shadow_x3 =torch.empty(2 * (self.x3_hi - self.x3_lo), dtype=torch.bfloat16,
                                     device=self.data.device)
        for i in idx:
            p, o = self.params[i], self.offsets[i]
            a = 2 * (o - self.x3_lo)
            p._dfu_shadow_x3 = self.shadow_x3[a:a + 2 * p.numel()].view(p.shape[0], -1)
        self._split_x3()

    def _split_x3(self):
        ops.split_x3_into(self.data[self.x3_lo:self.x3_hi].view(-1, 32), ops.X3_PAIRS,
                          self.shadow_x3.view(-1, 64))
        for p in self.params:
            if getattr(p, "_dfu_shadow_x3", None) is not None:
                p._dfu_shadow_x3_version = p._version

    def x3_args(self, lo, hi):
        """dfu_adamw_flat's shadow_x3 arguments for the AdamW range [lo, hi): (shadow view,
        begin, end) relative to lo, or (None, 0, 0) when the range holds no x3 weights."""
        if self.shadow_x3 is None:
            return None, 0, 0
        a, b = max(lo, self.x3_lo), min(hi, self.x3_hi)
        if a >= b:
            return None, 0, 0
        return self.shadow_x3[2 * (a - self.x3_lo):], a - lo, b - lo

    def add_transposed(self, p):
        """Give parameter p a transposed bf16 shadow, kept current from now on."""
        sh = p._dfu_shadow
        p._dfu_shadow_T = torch.empty((sh.shape[1], sh.shape[0]), dtype=sh.dtype,
                                      device=sh.device)
        self._add_jobs(p, [(sh, p._dfu_shadow_T)])

    def add_flipped(self, p):
        """Give spatial conv weight p (KRSC shadow [K][R*S*C]) a flipped, channel-transposed bf16
        copy W'[C][R][S][K] = W[K][R-1-r][S-1-s][C] -- the weight of its stride-1 input gradient
        run as a forward convolution (functional.conv_dgrad) -- and its launch table (one
        transpose job per filter tap).  Derived on first use after each shadow rewrite
        (functional.conv_weight_flipped), i.e. on the ResNet's own stream in backward, not in
        the optimizer's tail: a batched refresh after AdamW measured slower in the two-stream
        step (it lengthens the step's serial end)."""
        K, C, R, S = p.shape
        sh = p._dfu_shadow.view(K, R * S, C)
        f = torch.empty((C, R * S * K), dtype=sh.dtype, device=sh.device)
        fv = f.view(C, R * S, K)
        p._dfu_shadow_F = f
        p._dfu_flip_jobs = ops.TransposeJobs([(sh[:, t, :], fv[:, R * S - 1 - t, :])
                                              for t in range(R * S)])
        p._dfu_fkey = None

    def _add_jobs(self, p, pairs):
        self.t_params.append(p)
        self.t_pairs += pairs
        self.t_pairs_of[id(p)] = pairs
        self.t_jobs = ops.TransposeJobs(self.t_pairs)
        self._range_jobs = {}

    def range_jobs(self, lo, hi):
        """(TransposeJobs of the transposed parameters inside flat range [lo, hi), those of the
        rest), either None when empty; cached per range."""
        key = (lo, hi)
        if key not in self._range_jobs:
            inside, rest = [], []
            for i, p in enumerate(self.params):
                pairs = self.t_pairs_of.get(id(p))
                if pairs:
                    (inside if lo <= self.offsets[i] < hi else rest).extend(pairs)
            self._range_jobs[key] = (ops.TransposeJobs(inside) if inside else None,
                                     ops.TransposeJobs(rest) if rest else None)
        return self._range_jobs[key]

    def shadows_rewritten(self, done=None):
        """Every shadow was just rewritten (AdamW, refresh): re-derive the transposed ones (the
        flipped conv copies follow on their next use: gen changed).  done = (lo, hi): the
        transposed parameters in that range were already re-derived (the early update)."""
        self.gen += 1
        jobs = self.t_jobs if done is None else self.range_jobs(*done)[1]
        if jobs is not None:
            jobs.launch()
        for p in self.t_params:
            p._dfu_sgen = p._dfu_tgen = self.gen

    def view(self, buf, i):
        """Parameter i's slice of a flat buffer (data, grad or an optimizer moment), shaped and
        strided like the parameter."""
        return _view(buf, self.offsets[i], self.params[i], self.krsc[i])

    def grad_view(self, i):
        return self.view(self.grad, i)

    def needs_rebind(self):
        """Host-side check: has user code replaced or cleared any p.grad?"""
        base = self.grad.data_ptr()
        for p, o in zip(self.params, self.offsets):
            g = p.grad
            if g is None or g.data_ptr() != base + 4 * o:
                return True
        return False

    def rebind_grads(self):
        """Re-attach p.grad to the flat buffer if user code replaced or cleared it (eager)."""
        for i, p in enumerate(self.params):
            v = self.grad_view(i)
            g = p.grad
            if g is None:
                ops.zero_(v)
                p.grad = v
            elif g.data_ptr() != v.data_ptr():
                v.copy_(g)
                p.grad = v


# DFU_EARLY_TRANSPOSE=0: the early-updated block's transposed shadows are re-derived in the
# step's tail with the rest (A/B)
_EARLY_T = os.environ.get("DFU_EARLY_TRANSPOSE", "1") != "0"


def _version_snapshot(wref):
    """Backward-end hook of one FusedAdamW (weakly referenced): the gradient buffer's version
    as the backward left it (see FusedAdamW._grad_version)."""
    def hook():
        o = wref()
        if o is not None:
            o._grad_version = o.flat.grad._version
    return hook


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 amsgrad=False, maximize=False):
        if amsgrad or maximize:
            raise NotImplementedError("FusedAdamW: amsgrad/maximize not supported")
        params = list(params)
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise NotImplementedError("FusedAdamW: a single param group")
        self.flat = FlatParams(self.param_groups[0]["params"])
        dev = self.flat.data.device
        self.exp_avg = torch.zeros_like(self.flat.data)
        self.exp_avg_sq = torch.zeros_like(self.flat.data)
        self.step_dev = torch.zeros((), dtype=torch.int64, device=dev)
        self.check_grads = True  # set False inside captured graphs (pointers are static)
        # update a side stream's parameter block on that stream (step); DFU_EARLY_ADAMW=0: off
        self.early_update = os.environ.get("DFU_EARLY_ADAMW", "1") != "0"
        self._dfu_joins_itself = True  # step() joins the gradient streams (functional)
        # the flat gradient buffer's autograd version at the last zero_grad / step / end of a
        # backward pass: the kernels write gradients through raw pointers (no bump), so a change
        # since means user code edited p.grad in place (clip_grad_norm_, unscaling, a manual
        # reduction) on its own stream.  Snapshotted again when a backward ends, so autograd's
        # own AccumulateGrad into a torch.nn head's gradient (the drop-in path) does not count.
        self._grad_version = self.flat.grad._version
        if dev.type == "cuda":
            hook = Fn.register_backward_end_hook(_version_snapshot(weakref.ref(self)))
            weakref.finalize(self, Fn.remove_backward_end_hook, hook)

    def zero_grad(self, set_to_none=True):
        # gradients stay bound to the flat buffer (stable addresses); one memset clears them
        ops.zero_(self.flat.grad)
        self._grad_version = self.flat.grad._version

    def _early_range(self, cur):
        """(lo, hi, stream): the largest run of parameters, contiguous in the flat buffers, whose
        gradients this step were all produced on one stream other than `cur` (the concurrent ViT
        branch's side stream in the fusion step), or None."""
        best, run = None, None
        fp = self.flat
        for i, p in enumerate(fp.params):
            st = getattr(p, "_dfu_grad_stream", None)
            st = st if st is not None and st is not False and st != cur else None
            lo, hi = fp.offsets[i], fp.offsets[i] + _aligned(p.numel())
            if st is not None and run is not None and run[2] == st and run[1] == lo:
                run = (run[0], hi, st)
            else:
                run = (lo, hi, st) if st is not None else None
            if run is not None and (best is None or run[1] - run[0] > best[1] - best[0]):
                best = run
        return best if best is not None and best[1] - best[0] >= (1 << 20) else None

    def _adamw(self, lo, hi):
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        fp = self.flat
        x3, x3b, x3e = fp.x3_args(lo, hi)
        ops.adamw_flat(fp.data[lo:hi], fp.grad[lo:hi], self.exp_avg[lo:hi],
                       self.exp_avg_sq[lo:hi], g["lr"], b1, b2, g["eps"], g["weight_decay"],
                       self.step_dev,
                       shadow=None if fp.shadow is None else fp.shadow[lo:hi],
                       shadow16=None if fp.shadow16 is None else fp.shadow16[lo:hi],
                       shadow_x3=x3, x3_begin=x3b, x3_end=x3e)

    @torch.no_grad()
    def step(self, closure=None):
        """One AdamW update of every parameter.  Where a contiguous block of parameters got its
        gradients on a side stream (the fusion step's ViT branch), that block is updated on that
        stream as soon as its backward is done -- beside the other branch's backward tail --
        and the rest after every gradient stream is joined (single process only: under data
        parallelism the gradients are final only after the all-reduce)."""
        loss = closure() if closure is not None else None
        fp = self.flat
        early = None
        # host-side check first: the rebinding copies (and their per-parameter views) only when
        # user code replaced a gradient
        rebind = self.check_grads and fp.needs_rebind()
        # the early update reads its block on the producing side stream, which does not wait for
        # the current stream: only for gradients nothing touched since backward wrote them
        touched = fp.grad._version != self._grad_version
        if (self.early_update and fp.data.is_cuda and not _dp_world() and not rebind
                and not touched):
            early = self._early_range(ops.current_stream(fp.data.get_device()))
        cur = ops.current_stream(fp.data.get_device()) if fp.data.is_cuda else None
        if early is not None:
            lo, hi, st = early
            with ops.on_stream(st):
                ops.step_increment(self.step_dev)  # the rest runs after the join: sees it
                self._adamw(lo, hi)
                # the block's transposed shadows right behind its update, beside the other
                # branch's backward tail instead of in the step's serial end
                inside = fp.range_jobs(lo, hi)[0] if fp.t_jobs is not None and _EARLY_T else None
                if inside is not None:
                    inside.launch()
            ops.stream_wait(cur, st)  # the rest, the step counter and the shadow transposes after it
        Fn.join_grad_streams()
        if rebind:
            fp.rebind_grads()
        if early is None:
            ops.step_increment(self.step_dev)
        if early is None:
            self._adamw(0, fp.numel)
        else:  # the rest: both sides of the early block
            if early[0] > 0:
                self._adamw(0, early[0])
            if early[1] < fp.numel:
                self._adamw(early[1], fp.numel)
        for p in fp.params:
            p._dfu_grad_stream = None
        self.last_early = None if early is None else early[:2]
        fp.shadows_rewritten(None if early is None or fp.t_jobs is None or not _EARLY_T
                             else early[:2])
        self._grad_version = fp.grad._version
        return loss

    def state_dict(self):
        """torch.optim.AdamW's layout: per-parameter {'step', 'exp_avg', 'exp_avg_sq'} keyed by
        parameter index, so checkpoints interchange with the reference's optimizer
        (train_multimodal_fusion.py:347, 436).  The moments are views of the flat buffers."""
        sd = super().state_dict()
        step = torch.tensor(float(self.step_dev.item()))
        index = {id(p): i for i, p in enumerate(self.param_groups[0]["params"])}
        for j, p in enumerate(self.flat.params):
            sd["state"][index[id(p)]] = {
                "step": step.clone(),
                "exp_avg": self.flat.view(self.exp_avg, j),
                "exp_avg_sq": self.flat.view(self.exp_avg_sq, j),
            }
        return sd

    def load_state_dict(self, state_dict):
        """Accepts torch.optim.AdamW state dicts (and this class's own)."""
        state = state_dict.get("state", {})
        super().load_state_dict({"state": {}, "param_groups": state_dict["param_groups"]})
        params = self.param_groups[0]["params"]
        index = {id(p): i for i, p in enumerate(params)}
        steps = set()
        with torch.no_grad():
            for j, p in enumerate(self.flat.params):
                st = state.get(index[id(p)])
                if not st:
                    continue
                self.flat.view(self.exp_avg, j).copy_(st["exp_avg"].reshape(p.shape))
                self.flat.view(self.exp_avg_sq, j).copy_(st["exp_avg_sq"].reshape(p.shape))
                steps.add(int(float(st["step"])))
        if len(steps) > 1:
            raise ValueError(f"FusedAdamW: parameters at different steps {sorted(steps)}")
        if steps:
            n = steps.pop()
            self.step_dev.fill_(n)
