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
from . import ops


def _seen_streams():
    """The streams library launches went to during the capture being recorded (ops.stream_ptr),
    as torch streams -- user streams the step forked onto included."""
    seen = ops._capture_seen
    if not seen:
        return []
    return [torch.cuda.ExternalStream(raw, device=torch.device("cuda", dev))
            for dev, raw in sorted(seen)]


def step_streams(device=None, extra=()):
    """Every stream a DFU step may enqueue on: the current one, the encoder side streams, the
    ViT weight-gradient streams, the streams library launches went to during the capture in
    progress, and `extra`."""
    out = [torch.cuda.current_stream(device)]
    out += list(Fn._side_streams.values()) + list(Fn._wgrad_streams.values()) + list(extra)
    out += _seen_streams()
    seen, uniq = set(), []
    for s in out:
        if s.cuda_stream not in seen:
            seen.add(s.cuda_stream)
            uniq.append(s)
    return uniq


def capture_status(stream):
    """0 none, 1 active, 2 invalidated (dfu_stream_capture_status)."""
    st = ctypes.c_int32(0)
    L.check(L.load().dfu_stream_capture_status(ctypes.c_void_p(stream.cuda_stream),
                                               ctypes.byref(st)), "dfu_stream_capture_status")
    return st.value


def join_forked(origin, extra=()):
    """Inside a capture on `origin`: make it wait for every step stream that is capturing (a
    fork of this capture), so work left on a side stream joins the graph instead of failing
    the capture as unjoined -- which HIP cannot undo: the origin's hipStreamEndCapture then
    returns hipErrorStreamCaptureUnjoined and leaves the origin and its forks capturing for
    good (a second end returns hipErrorStreamCaptureWrongThread; tools/diag).  The step streams
    include every stream a library launch went to during this capture, so a fork onto a plain
    torch stream that the step did not join back (the C5 split-graph
    attempt's crash at hipStreamEndCapture) is joined here too; only non-library work on a
    stream the library never saw can still leave a fork unjoined."""
    for s in step_streams(extra=extra):
        if s.cuda_stream != origin.cuda_stream and capture_status(s) == 1:
            origin.wait_stream(s)


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
    """Recover after a failed capture: end what HIP lets us end, retire the library-owned
    streams still capturing (HIP cannot end a capture whose origin's end already failed:
    tools/diag/capture_unjoined.py) -- the next side_stream / wgrad_stream call makes fresh
    ones -- and reset the host-side stream state.  Returns (streams that were capturing,
    streams retired)."""
    streams = step_streams(extra=extra)
    n, _ = abort_captures(streams)
    stuck = {s.cuda_stream for s in streams if capture_status(s) != 0}
    for cache in (Fn._side_streams, Fn._wgrad_streams):
        for k in [k for k, s in cache.items() if s.cuda_stream in stuck]:
            del cache[k]  # leaked on purpose: a capturing stream cannot be destroyed or reused
    cur = torch.cuda.current_stream()
    if cur.cuda_stream in stuck:
        raise RuntimeError("dfu: the caller's stream is still capturing after a failed capture")
    Fn._grad_streams.clear()
    Fn._join_armed[0] = False
    ops._stream_objs.clear()
    try:  # can the process run eager work again?  (an allocation + a kernel + a host sync)
        torch.empty(1024, device=cur.device).fill_(0.0)
        torch.cuda.synchronize()
    except RuntimeError as e:
        # HIP leaves an INVALIDATED capture that had forked streams active for good (e.g. a host
        # synchronisation inside the step): every later legacy-stream or allocation call fails
        # with hipErrorStreamCaptureImplicit.  Nothing in-process can end it.
        raise RuntimeError("dfu: a failed HIP-graph capture left this process unable to run "
                           "eager work (HIP cannot end an invalidated capture with forked "
                           "streams); rerun without graph capture") from e
    return n, len(stuck)


_capture_streams = {}


def try_capture(step, log=None, pool=None):
    """Capture `step()` into a torch.cuda.CUDAGraph on a fresh capture stream; returns the graph,
    or None after a failed capture (streams recovered, the failure reported through `log`,
    default stderr).  Work the step left on a forked stream is joined into the capture
    (join_forked).  The caller warms `step` up eagerly first, as graph capture requires."""
    prev = torch.cuda.current_stream()
    # one library-owned capture stream per device, reused by every capture (a graph does not
    # need its origin stream after the capture ends); retired, never reused, if a failure leaves
    # it capturing
    cap = _capture_streams.get(prev.device_index)
    if cap is None:
        cap = _capture_streams[prev.device_index] = Fn.new_stream(prev.device_index)
    cap.wait_stream(prev)
    # the capture stream's split-K tile counters exist before the capture: created inside it,
    # their zero-fill would be recorded into this graph and run only at its replays
    with torch.cuda.stream(cap):
        ops.tile_counters(cap.device)
    g = torch.cuda.CUDAGraph()
    ops._capture_seen = set()
    try:
        with torch.cuda.graph(g, pool=pool, stream=cap):
            try:
                step()
            finally:
                # also when step() raised (a DfuError refusing a non-capturable call): joined
                # forks let torch.cuda.graph's hipStreamEndCapture succeed, so the failure is a
                # Python exception and the streams are clean for the eager fallback
                join_forked(cap)
        return g
    except Exception as e:  # noqa: BLE001 -- any capture failure falls back to eager
        # torch.cuda.graph.__exit__ leaves its capture stream current when capture_end raises
        torch.cuda.set_stream(prev)
        n, stuck = reset_after_failed_capture(extra=(cap,))
        if capture_status(cap) != 0:
            _capture_streams.pop(prev.device_index, None)  # leaked on purpose (see above)
        msg = (f"[dfu] graph capture failed ({type(e).__name__}: {str(e).splitlines()[0]}); "
               f"{n} stream(s) were left capturing, {stuck} retired; running eager")
        if log is None:
            print(msg, file=sys.stderr)
        elif log:
            log(msg)
        del g
        return None
    finally:
        ops._capture_seen = None
