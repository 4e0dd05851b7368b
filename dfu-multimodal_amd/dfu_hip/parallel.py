"""Pure data parallelism for the DFU fusion step: one process per GPU, torch.distributed with
the "nccl" backend (= RCCL on ROCm) over xGMI.

The reference has no distributed code; this adds the one exchange step the path has: the
gradient all-reduce of the 110.75M fp32 parameters.  Gradients live in the FusedAdamW flat
buffer (dfu_hip.optim.FlatParams), so buckets are contiguous slices — no packing copies.
Buckets are issued in reverse parameter order (the order backward finishes them) on a side
stream as soon as every parameter of a bucket reports grad-ready (functional.grads_done), so
the all-reduce overlaps the rest of the backward pass.  BatchNorm statistics stay per rank
(no SyncBN), as the reference's single-device BN.
"""
import os

import torch
import torch.distributed as dist

from . import functional as Fn
from . import ops


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env (RANK/WORLD_SIZE/MASTER_*).
    Rehearsal knobs (a one-GPU box running the N-rank path): DFU_DIST_BACKEND picks the backend
    (default nccl = RCCL with a GPU, else gloo) and DFU_SHARE_DEVICE=1 puts every rank on device
    0 (gloo then all-reduces the CUDA gradient buckets through host memory)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1, 0
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if os.environ.get("DFU_SHARE_DEVICE", "0") == "1":
        local = 0
    if backend is None:
        backend = os.environ.get("DFU_DIST_BACKEND") or (
            "nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return rank, world, local


def broadcast_parameters(module, src=0):
    """Same initial replica on every rank (parameters and buffers)."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src)


_AVG_OK = {}


def _supports_avg(group=None):
    """Whether all_reduce(op=AVG) works on this process group (NCCL/RCCL >= 2.10 backends do;
    gloo does not).  Probed once per group with a 1-element collective on every rank — ranks
    reach the same answer, so the collectives stay paired."""
    key = id(group)
    if key not in _AVG_OK:
        ok = False
        if dist.get_backend(group) == "nccl" and hasattr(dist.ReduceOp, "AVG"):
            t = torch.ones(1, device="cuda")
            try:
                dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group)
                torch.cuda.synchronize()
                ok = bool(abs(t.item() - 1.0) < 1e-6)
            except (RuntimeError, ValueError):
                ok = False
        _AVG_OK[key] = ok
    return _AVG_OK[key]


class GradAllReducer:
    """Bucketed all-reduce (mean over ranks) over the FusedAdamW flat gradient buffer.

    overlap=True: each bucket's collective is issued from the grad-ready notifications while
    backward still runs; call ``finish()`` before the optimizer step.  overlap=False:
    ``finish()`` issues every bucket after backward (graph-capture friendly).

    No stream of its own.  A bucket is issued asynchronously on the
    stream that produced its last gradient (the "carrier": the ViT branch's side stream or the
    backward's own stream); the process group's internal stream (PG-NCCL's) waits on that
    stream's position and runs the collective there, so the backward on the carrier is not
    held.  Gradients of the same bucket produced on another stream are covered by an event
    recorded on that stream when the bucket's producer last switched away from it (a few
    records per step, not one per parameter).  ``finish()`` makes the caller's stream wait for
    every collective.  So the fusion step at N > 1 uses the main stream, the ViT side stream and
    the process group's stream: 3 of the box's 4 hardware queues (GPU_MAX_HW_QUEUES), where a
    reducer stream of its own made 4 and any further stream would serialise the encoders."""

    def __init__(self, flat, bucket_mb=None, overlap=True, group=None):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.overlap = overlap and self.world > 1
        self.cuda = flat.grad.is_cuda
        # Buckets exist to start reducing while backward still runs.  Without overlap every
        # bucket is issued back to back after backward, so one large bucket (fewer collective
        # launches, full-size ring transfers over xGMI) is strictly better.
        if bucket_mb is None:
            bucket_mb = 32.0 if self.overlap else 1024.0
        # the mean as one collective (RCCL/NCCL ReduceOp.AVG: the 1/world scaling rides in the
        # reduction) where the backend has it; otherwise SUM, then one scaling pass at finish()
        self.avg = self.world > 1 and self.cuda and _supports_avg(group)
        cap = int(bucket_mb * (1 << 20) / 4)
        # reverse parameter order: the last parameters' gradients are produced first
        order = list(range(len(flat.params)))[::-1]
        self.buckets = []  # (start, end, set(param ids))
        cur, lo, hi = set(), None, None
        for i in order:
            p, o = flat.params[i], flat.offsets[i]
            end = o + ((p.numel() + 3) // 4 * 4)
            lo = o if lo is None else min(lo, o)
            hi = end if hi is None else max(hi, end)
            cur.add(id(p))
            if (hi - lo) >= cap:
                self.buckets.append((lo, hi, cur))
                cur, lo, hi = set(), None, None
        if cur:
            self.buckets.append((lo, hi, cur))
        self._bucket_of = {pid: k for k, b in enumerate(self.buckets) for pid in b[2]}
        self._views = None  # (flat.grad, bucket views), built on first launch
        self._pending = None
        self._issued = None
        self._hook = None
        self._works = []
        self.issue_log = []  # bucket indices in launch order (ranks must agree: RCCL pairs them)
        self.carriers = {}  # stream handle -> stream: the streams this step's collectives used
        if self.overlap:
            self._hook = Fn.register_grad_ready_hook(self._on_ready)

    def start(self):
        """Arm the per-step bucket state (call before backward)."""
        self._pending = [set(b[2]) for b in self.buckets]
        self._issued = [False] * len(self.buckets)
        # per bucket: the stream of its latest gradient, and {id: (stream, event)} of the other
        # streams it drew gradients from (event recorded when the producer switched away)
        self._last = [None] * len(self.buckets)
        self._marks = [{} for _ in self.buckets]
        # per bucket: some gradient came from several or unknown streams (its
        # producers have no event in _marks, so the bucket must join every gradient stream)
        self._unknown = [False] * len(self.buckets)
        self._works = []
        self.carriers = {}

    def _producer(self, p):
        if not self.cuda:
            return None
        st = getattr(p, "_dfu_grad_stream", None)
        return st if st else False  # False: several (or unknown) producer streams

    def _note(self, k, st):
        if st is False:
            self._unknown[k] = True
        prev = self._last[k]
        if prev is not None and prev is not st and prev is not False:
            ev = torch.cuda.Event()
            ev.record(prev)
            self._marks[k][id(prev)] = (prev, ev)
        self._last[k] = st

    def _carrier(self, k, carrier):
        """The stream bucket k's collective is issued from, or None when every gradient
        stream must join the caller's stream first: the last producer is unknown, or an
        earlier gradient of the bucket had several / unknown producers."""
        if carrier is None or carrier is False or self._unknown[k]:
            return None
        return carrier

    def _launch(self, k, carrier=None):
        g = self.flat.grad
        if self._views is None or self._views[0] is not g:
            self._views = (g, [g[lo:hi] for lo, hi, _ in self.buckets])
        view = self._views[1][k]
        if self.cuda:
            carrier = self._carrier(k, carrier)
            if carrier is None:
                carrier = ops.current_stream()
                Fn.join_grad_streams(carrier, clear=False)
            for sid, (st, ev) in self._marks[k].items():
                if st is not carrier:
                    carrier.wait_event(ev)
            self.carriers[carrier.cuda_stream] = carrier
            with ops.on_stream(carrier):
                self._works.append(self._reduce(view))
        else:
            self._works.append(self._reduce(view))
        self._issued[k] = True
        self.issue_log.append(k)

    def _reduce(self, view):
        op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
        return dist.all_reduce(view, op=op, group=self.group, async_op=True)

    def _on_ready(self, p):
        pending = self._pending
        if pending is None:
            return
        pid = id(p)
        k = self._bucket_of.get(pid)
        if k is None or pid not in pending[k]:
            return
        pend = pending[k]
        pend.discard(pid)
        st = self._producer(p) if self.cuda else None
        if st is not None:
            self._note(k, st)
        if not pend and not self._issued[k]:
            self._launch(k, st)

    def finish(self):
        Fn.join_grad_streams()
        if self.world <= 1:
            return
        if self._issued is None:
            self.start()
        for k in range(len(self.buckets)):
            if not self._issued[k]:
                self._launch(k)
        for w in self._works:
            w.wait()  # the caller's stream waits for the collective (host-blocking on gloo)
        if not self.avg:
            lo = min(b[0] for b in self.buckets)
            hi = max(b[1] for b in self.buckets)
            self.flat.grad[lo:hi].mul_(1.0 / self.world)
        self._works = []
        self._pending = None
        self._issued = None

    def close(self):
        if self._hook is not None:
            Fn.remove_grad_ready_hook(self._hook)
            self._hook = None
