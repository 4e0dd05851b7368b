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
    """Bucketed all-reduce (sum, then /world) over the FusedAdamW flat gradient buffer.

    overlap=True: buckets launch from grad-ready notifications on a side stream during
    backward; call ``finish()`` before the optimizer step.  overlap=False: ``finish()`` issues
    every bucket after backward (graph-capture friendly)."""

    def __init__(self, flat, bucket_mb=None, overlap=True, group=None):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.overlap = overlap and self.world > 1
        self.stream = torch.cuda.Stream() if flat.grad.is_cuda else None
        # Buckets exist to start reducing while backward still runs.  Without overlap every
        # bucket is issued back to back after backward, so one large bucket (fewer collective
        # launches, full-size ring transfers over xGMI) is strictly better.
        if bucket_mb is None:
            bucket_mb = 32.0 if self.overlap else 1024.0
        # the mean as one collective (RCCL/NCCL ReduceOp.AVG: the 1/world scaling rides in the
        # reduction) where the backend has it; otherwise SUM then one scaling pass per bucket
        self.avg = self.world > 1 and flat.grad.is_cuda and _supports_avg(group)
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
        self._pending = None
        self._issued = None
        self._hook = None
        self.issue_log = []  # bucket indices in launch order (ranks must agree: RCCL pairs them)
        if self.overlap:
            self._hook = Fn.register_grad_ready_hook(self._on_ready)

    def start(self):
        """Arm the per-step bucket state (call before backward)."""
        self._pending = [set(b[2]) for b in self.buckets]
        self._issued = [False] * len(self.buckets)

    def _launch(self, k):
        lo, hi, _ = self.buckets[k]
        view = self.flat.grad[lo:hi]
        if self.stream is not None:
            # a bucket may hold gradients of both encoder branches (two streams): wait for all
            self.stream.wait_stream(torch.cuda.current_stream())
            Fn.join_grad_streams(self.stream, clear=False)
            with torch.cuda.stream(self.stream):
                self._reduce(view)
        else:
            self._reduce(view)
        self._issued[k] = True
        self.issue_log.append(k)

    def _reduce(self, view):
        if self.avg:
            dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.group)
        else:
            dist.all_reduce(view, group=self.group)
            view.mul_(1.0 / self.world)

    def _on_ready(self, p):
        if self._pending is None:
            return
        pid = id(p)
        for k, pend in enumerate(self._pending):
            if pid in pend:
                pend.discard(pid)
                if not pend and not self._issued[k]:
                    self._launch(k)
                break

    def finish(self):
        Fn.join_grad_streams()
        if self.world <= 1:
            return
        if self._issued is None:
            self.start()
        for k in range(len(self.buckets)):
            if not self._issued[k]:
                self._launch(k)
        if self.stream is not None:
            torch.cuda.current_stream().wait_stream(self.stream)
        self._pending = None
        self._issued = None

    def close(self):
        if self._hook is not None:
            Fn.remove_grad_ready_hook(self._hook)
            self._hook = None
