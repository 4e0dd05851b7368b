"""HIP-graph capture of a step with a clean fallback to eager execution.

A captured step replays every kernel launch of the step from one graph launch (the host-side
enqueue cost of the ~700 launches disappears).  Capture can fail -- work forked onto a side
stream and not joined back, a host synchronisation inside the step -- and a failed capture can
leave the streams it forked into still in capture mode, so that the next eager launch or event
on them fails as well (bench.py round 2: "event last recorded in a capturing stream": the
timing event went to torch.cuda.graph's capture stream, which its __exit__ leaves current when
capture_end raises).
try_capture ends such leftover captures (dfu_streams_abort_capture over every stream the step
can touch), drops the per-stream caches that refer to them, and reports the failure, so the caller
runs eager.
"""
import ctypes
import sys

import torch

from . import _lib as L
from . import functional as Fn


def step_streams(device=None, extra=()):
    """Every stream a DFU step may enqueue on: the current one, the encoder side streams, the
    ViT weight-gradient streams, and `extra`."""
    out = [torch.cuda.current_stream(device)]
    out += list(Fn._side_streams.values()) + list(Fn._wgrad_streams.values()) + list(extra)
    seen, uniq = set(), []
    for s in out:
        if s.cuda_stream not in seen:
            seen.add(s.cuda_stream)
            uniq.append(s)
    return uniq


def abort_captures(streams):
    """End any capture left active on `streams` (dfu_streams_abort_capture); returns
    (streams that were capturing, streams still capturing afterwards)."""
    lib = L.load()
    handles = [s.cuda_stream for s in streams]
    before = 0
    for s in streams:
        with torch.cuda.stream(s):
            before += int(torch.cuda.is_current_stream_capturing())
    arr = (ctypes.c_void_p * len(handles))(*handles)
    left = ctypes.c_int32(0)
    L.check(lib.dfu_streams_abort_capture(arr, len(handles), ctypes.byref(left)),
            "dfu_streams_abort_capture")
    return before, left.value


def reset_after_failed_capture(extra=()):
    """Recover the streams and host-side stream state after a failed capture."""
    n, left = abort_captures(step_streams(extra=extra))
    if left:
        raise RuntimeError(f"dfu: {left} stream(s) still capturing after the capture abort")
    Fn._grad_streams.clear()
    Fn._join_armed[0] = False
    Fn._stream_objs.clear()
    torch.cuda.synchronize()
    return n


def try_capture(step, log=None, pool=None):
    """Capture `step()` into a torch.cuda.CUDAGraph on a fresh capture stream; returns the graph,
    or None after a failed capture (streams recovered, the failure reported through `log`,
    default stderr).  The caller warms `step` up eagerly first, as graph capture requires."""
    prev = torch.cuda.current_stream()
    cap = torch.cuda.Stream()
    cap.wait_stream(prev)
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, pool=pool, stream=cap):
            step()
        return g
    except Exception as e:  # noqa: BLE001 -- any capture failure falls back to eager
        # torch.cuda.graph.__exit__ leaves its capture stream current when capture_end raises
        torch.cuda.set_stream(prev)
        left = reset_after_failed_capture(extra=(cap,))
        msg = (f"[dfu] graph capture failed ({type(e).__name__}: {str(e).splitlines()[0]}); "
               f"{left} stream(s) left capturing were ended; running eager")
        if log is None:
            print(msg, file=sys.stderr)
        elif log:
            log(msg)
        del g
        return None
