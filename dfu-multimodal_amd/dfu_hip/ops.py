"""Thin, shape-checked wrappers over the libdfu_hip C ABI (include/dfu_hip.h).

Each function takes torch tensors that already live on the GPU, passes raw pointers and the
current HIP stream, and raises DfuError on any non-zero return code.  Nothing here allocates
except where an output is documented as returned; nothing synchronises.
"""
import ctypes

import torch

from . import _lib as L
from ._lib import check

BF16 = torch.bfloat16
F32 = torch.float32
F16 = torch.float16


def lib():
    return L.load()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)


# (device, raw stream) of every launch while dfu_hip.graphs.try_capture records a graph (None
# otherwise): the capture joins each of these streams that is still capturing into its origin
# before hipStreamEndCapture, so library work a step left on a stream it forked -- a plain torch
# stream included -- becomes part of the graph instead of failing the capture as unjoined.
_capture_seen = None


def stream_ptr():
    """The current HIP stream of the current device (the raw-pointer query: torch.cuda.
    current_stream() builds a Stream object per call, ~8 us of host time x ~260 calls a step).
    Pointers go to the C ABI as plain ints (ctypes converts them for c_void_p parameters:
    0.4 us per argument less than a c_void_p object, ~2000 arguments a step)."""
    if _raw_stream is not None and _cur_device is not None:
        dev = _cur_device()
        s = _raw_stream(dev)
    else:
        st = torch.cuda.current_stream()
        dev, s = st.device_index, st.cuda_stream
    if _capture_seen is not None:
        _capture_seen.add((dev, s))
    return s


_get_cur_stream = getattr(torch._C, "_cuda_getCurrentStream", None)
_set_cur_stream = getattr(torch._C, "_cuda_setStream", None)
_stream_objs = {}


def current_stream(idx=None):
    """torch.cuda.current_stream(idx) as one cached Stream object per (device, raw HIP stream):
    torch builds a new object per call (2.7 us of host time against 0.2 us,
    tools/host_breakdown.py).  A cached object is re-validated against the raw handle, so a
    destroyed user stream whose address is reused gets a fresh object."""
    if _raw_stream is None or _cur_device is None:
        return torch.cuda.current_stream(idx)
    if idx is None:
        idx = _cur_device()
    raw = _raw_stream(idx)
    st = _stream_objs.get((idx, raw))
    if st is None or st.cuda_stream != raw:
        st = _stream_objs[(idx, raw)] = torch.cuda.current_stream(idx)
    return st


class on_stream:
    """``with torch.cuda.stream(s):`` for a stream of the current device without the Stream
    object torch's context builds on entry (5.9 us of host time per entry against ~1 us,
    tools/host_breakdown.py); any other case goes through torch's own context."""

    __slots__ = ("s", "prev")

    def __init__(self, s):
        self.s = s
        self.prev = None

    def __enter__(self):
        s = self.s
        if s is None:
            return None
        if _get_cur_stream is None or _set_cur_stream is None or _cur_device is None or \
                s.device_index != _cur_device():
            self.prev = torch.cuda.stream(s)
            self.prev.__enter__()
            return s
        dev = s.device_index
        self.prev = _get_cur_stream(dev)
        _set_cur_stream(s.stream_id, dev, s.device_type)
        return s

    def __exit__(self, *exc):
        p, self.prev = self.prev, None
        if isinstance(p, tuple):
            _set_cur_stream(p[0], p[1], p[2])
        elif p is not None:
            p.__exit__(*exc)
        return False


def stream_wait(waiter, producer):
    """waiter.wait_stream(producer) for torch streams of the current device by one C call
    (dfu_stream_wait: a pooled event instead of a torch Event object per call, 6.5 us of host
    time against ~2 us); any other case goes through torch."""
    dev = waiter.device_index
    if producer.device_index != dev or _cur_device is None or dev != _cur_device():
        waiter.wait_stream(producer)
        return
    w = waiter.cuda_stream
    if _capture_seen is not None:  # a fork into a capture: try_capture joins it at the end
        _capture_seen.add((dev, w))
    check(lib().dfu_stream_wait(w, producer.cuda_stream), "dfu_stream_wait")


def refuse_in_capture(what):
    """Raise DfuError when the current stream is recording a graph: `what` would either
    invalidate the capture (a stream creation is not a capturable call) or leave state that
    only a replay initialises (a zero-fill recorded into the graph)."""
    if torch.cuda.is_current_stream_capturing():
        stream_ptr()  # a fork with no library launch yet: join_forked must still see it
        raise L.DfuError(f"{what} requested inside a HIP-graph capture: run the step once "
                         f"eagerly on the same streams before capturing it")


def ptr(t):
    return None if t is None else t.data_ptr()


def _req(t, dtype, name):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: tensor must be on the GPU")


# ----------------------------------------------------------------------------------- GEMM
class ConvGeom:
    """Implicit-GEMM convolution geometry (NHWC input N,H,W,C; K filters of R x S)."""

    __slots__ = ("n", "h", "w", "c", "k", "r", "s", "stride", "pad", "p", "q")

    def __init__(self, n, h, w, c, k, r, s, stride, pad):
        self.n, self.h, self.w, self.c, self.k = n, h, w, c, k
        self.r, self.s, self.stride, self.pad = r, s, stride, pad
        self.p = (h + 2 * pad - r) // stride + 1
        self.q = (w + 2 * pad - s) // stride + 1


TILES = {"auto": 0, "128x128": 1, "256x128": 2, "128x256": 3, "256x256": 4, "128x128o2": 5,
         "128x128w4": 6, "256x256p8": 7, "256x256ps": 8, "192x256ps": 9, "256x64": 10,
         "128x64o2": 11}

# Optional recording of GEMM launches (bench.py's roofline): when set to a list, every
# dfu_gemm call appends (descriptor, algorithmic flops, tensors it touches) — the tensor
# references keep the buffers alive so the launches can be replayed back-to-back later.
# Never set inside graph capture.
gemm_record = None


def _algorithmic_bytes(d, conv):
    """Compulsory HBM bytes of one launch: each operand tensor read once, C written once
    (read too when accumulated), epilogue side inputs/outputs once."""
    M, N, K = d.M, d.N, d.K
    act_in = 2 * conv.n * conv.h * conv.w * conv.c if conv is not None else 0
    a = {L.OPND_CONV_FWD: act_in,
         L.OPND_CONV_DGRAD: 2 * conv.n * conv.p * conv.q * conv.k if conv is not None else 0
         }.get(d.a_mode, 2 * M * K)
    if d.a_seg and not d.x3_pairs:  # split pair: hi and lo once each (the tripled K reads hi twice)
        a = a * 2 // 3
    b = act_in if d.b_mode == L.OPND_CONV_WGRAD_X else 2 * N * K
    e = d.epilogue
    # bytes per output element: C (+ read-modify-write / side outputs)
    c = {L.EPI_F32: 4, L.EPI_F32_RESID: 8, L.EPI_F32_ACC: 8, L.EPI_PATCH: 4, L.EPI_F32_STATS: 4,
         L.EPI_BF16_GELU: 4, L.EPI_BF16_DGELU: 4, L.EPI_BF16_ADD: 4,
         L.EPI_X3_GELU: 8, L.EPI_F16_GELU: 6,
         L.EPI_F16_DUAL: 4 if d.aux_out else 2}.get(e, 2) * M * N
    return a + b + c


def gemm_replay(records, stream=None):
    """Re-issue recorded dfu_gemm launches (same descriptors) on the current stream."""
    s = stream_ptr() if stream is None else stream
    fn = lib().dfu_gemm
    for r in records:
        check(fn(ctypes.byref(r[0]), s), "dfu_gemm replay")


def gemm(M, N, K, A, lda, B, ldb, C, ldc, a_mode=L.OPND_KMAJOR, b_mode=L.OPND_KMAJOR,
         epilogue=L.EPI_BF16, alpha=1.0, bias=None, aux=None, ldaux=0, aux_out=None,
         ldaux_out=0, stats=None, split_k=0, ep_tokens=0, conv=None, tile=0, workspace=None,
         operand_type=0, x3=False, a_lo=None, x3_pairs=False):
    """C = epilogue(A @ B^T).  `split_k` (F32_ACC only): 0 = library cost model, 1 = none.
    `x3`: a bf16x3 product (K tripled): the recorded algorithmic FLOPs count K / 3.
    `a_lo`: split-pair A -- A is the hi buffer and a_lo the lo buffer ([rows][K / 3] each; the
    conv forward: NHWC with conv.c / 3 channels), read as the K-segments hi | lo | hi.
    `x3_pairs` (with a_lo): interleaved pairs instead -- K (conv.c) = 2 x the pair's width, B
    in pattern X3_PAIRS, the kernel forms the three products per K-step.
    `tile`: 0 = library cost model, else a TILES id.  Split-K partials go to fp32 slabs in
    `workspace` (allocated here from the stream-ordered caching allocator when None) and are
    reduced deterministically by a second kernel."""
    for t, name in ((A, "A"), (B, "B"), (C, "C")):
        if not t.is_cuda:
            raise ValueError(f"gemm: operand {name} must be on the GPU (there is no host path)")
    d = L.GemmDesc()
    d.M, d.N, d.K = int(M), int(N), int(K)
    d.a_mode, d.b_mode = int(a_mode), int(b_mode)
    d.A, d.lda = A.data_ptr(), int(lda)
    d.B, d.ldb = B.data_ptr(), int(ldb)
    d.C, d.ldc = C.data_ptr(), int(ldc)
    d.epilogue, d.alpha = int(epilogue), float(alpha)
    d.bias = bias.data_ptr() if bias is not None else None
    d.aux = aux.data_ptr() if aux is not None else None
    d.ldaux = int(ldaux)
    d.aux_out = aux_out.data_ptr() if aux_out is not None else None
    d.ldaux_out = int(ldaux_out)
    d.stats = stats.data_ptr() if stats is not None else None
    d.operand_type = int(operand_type)
    if a_lo is not None:
        nseg = 2 if x3_pairs else 3
        d.a_seg = int(conv.c // nseg if a_mode == L.OPND_CONV_FWD else K // nseg)
        d.a_lo = a_lo.data_ptr()
        d.x3_pairs = int(bool(x3_pairs))
    d.split_k = int(split_k)
    d.ep_tokens = int(ep_tokens)
    d.tile = int(tile)
    if conv is not None:
        d.conv_n, d.conv_h, d.conv_w, d.conv_c = conv.n, conv.h, conv.w, conv.c
        d.conv_k, d.conv_r, d.conv_s = conv.k, conv.r, conv.s
        d.conv_stride, d.conv_pad, d.conv_p, d.conv_q = conv.stride, conv.pad, conv.p, conv.q
    lb = lib()
    ref = ctypes.byref(d)
    need = lb.dfu_gemm_workspace_bytes(ref)  # split-K or tail-split slabs
    if need > 0:
        if workspace is None or workspace.numel() * workspace.element_size() < need:
            workspace = torch.empty(need, dtype=torch.uint8, device=C.device)
        d.workspace = workspace.data_ptr()
        d.workspace_bytes = int(need)
        cnt = tile_counters(C.device)
        d.tile_counters, d.tile_counters_len = cnt.data_ptr(), cnt.numel()
    rc = lb.dfu_gemm(ref, stream_ptr())
    if rc:
        check(rc, "dfu_gemm")
    if gemm_record is not None:
        # algorithmic (x3: the product, not its 3 passes)
        flops = 2.0 * M * N * (K // (2 if x3_pairs else 3) if x3 else K)
        if a_mode == L.OPND_CONV_DGRAD and conv is not None:
            flops /= conv.stride * conv.stride  # algorithmic: only the 1/stride^2 live taps
        # executed MFMA work: a bf16x3 GEMM runs three products of the real K
        executed = 3.0 * flops if x3 else 2.0 * M * N * K
        gemm_record.append((d, flops, _algorithmic_bytes(d, conv),
                            (A, B, C, bias, aux, aux_out, stats, workspace, a_lo), executed))


_COUNTERS = {}
_COUNTER_POOLS = {}  # device index -> [zeroed pool, next free slot]
TILE_COUNTERS = 1 << 16
COUNTER_SLOTS = 64  # streams per pool (64 x 256 KiB)


def tile_counters(device):
    """Per-stream zeroed int32 tile counters for the in-kernel split-K reduction (every launch
    returns them zeroed; launches on one stream never overlap).  A stream's counters are a slot
    of a per-device pool zeroed when the pool is made, so a stream first seen inside a graph
    capture takes a slot by host bookkeeping alone (a zero-fill made inside the capture would be
    recorded into the graph and run only at its replays: eager launches on that stream before
    the first replay would read uninitialised counters)."""
    idx = device.index if isinstance(device, torch.device) and device.index is not None else None
    if _raw_stream is not None and idx is not None:
        key = (idx, _raw_stream(idx))  # the raw query: ~0.3 us against ~5 us for a Stream object
        t = _COUNTERS.get(key)
        if t is not None:
            return t
    st = torch.cuda.current_stream(device)
    key = (st.device_index, st.cuda_stream)
    t = _COUNTERS.get(key)
    if t is None:
        pool = _COUNTER_POOLS.get(st.device_index)
        if pool is None or pool[1] == COUNTER_SLOTS:
            refuse_in_capture(f"a fresh pool of split-K tile counters (stream "
                              f"{st.cuda_stream:#x})")
            pool = _COUNTER_POOLS[st.device_index] = [
                torch.zeros(COUNTER_SLOTS * TILE_COUNTERS, dtype=torch.int32, device=device), 0]
        i = pool[1]
        pool[1] += 1
        t = _COUNTERS[key] = pool[0][i * TILE_COUNTERS:(i + 1) * TILE_COUNTERS]
    return t


def gemm_set_tail_split(enable):
    """Tail split of the last partial round of tiles along K (dfu_gemm_set_tail_split)."""
    return int(lib().dfu_gemm_set_tail_split(int(bool(enable))))


def gemm_set_inkernel_reduce(enable):
    """Split-K reduction inside the GEMM (1) or by the separate reduce kernel (0)."""
    return int(lib().dfu_gemm_set_inkernel_reduce(int(bool(enable))))


def _plan_desc(M, N, K, a_mode, b_mode, epilogue, split_k, tile):
    d = L.GemmDesc()
    d.M, d.N, d.K = int(M), int(N), int(K)
    d.a_mode, d.b_mode, d.epilogue = int(a_mode), int(b_mode), int(epilogue)
    d.split_k, d.tile = int(split_k), int(tile)
    return d


def gemm_workspace_bytes(M, N, K, a_mode, b_mode, epilogue=L.EPI_F32_ACC, split_k=0, tile=0):
    d = _plan_desc(M, N, K, a_mode, b_mode, epilogue, split_k, tile)
    return int(lib().dfu_gemm_workspace_bytes(ctypes.byref(d)))


def gemm_plan(M, N, K, a_mode, b_mode, epilogue, split_k=0, tile=0):
    """(tile id 1..4, split-K) the library's cost model picks."""
    d = _plan_desc(M, N, K, a_mode, b_mode, epilogue, split_k, tile)
    t, sk = ctypes.c_int32(), ctypes.c_int32()
    check(lib().dfu_gemm_plan(ctypes.byref(d), ctypes.byref(t), ctypes.byref(sk)), "dfu_gemm_plan")
    return t.value, sk.value


PERSISTENT_ALL = 3  # dfu_gemm_set_persistent: bit 0 generic tiles, bit 1 phased 256-wide tiles


def gemm_set_persistent(mode):
    """Select the GEMM schedule (dfu_gemm_set_persistent: 0 one workgroup per work unit
    everywhere, PERSISTENT_ALL persistent everywhere, 2 the default); returns the previous
    mode, which restores it exactly."""
    return int(lib().dfu_gemm_set_persistent(int(mode)))


def gemm_f32(M, N, K, A, sam, sak, B, sbn, sbk, C, ldc, bias=None, relu=False, accumulate=False):
    """Exact fp32 strided GEMM (fusion head); split-K slabs from the caching allocator."""
    need = lib().dfu_gemm_f32_workspace_bytes(int(M), int(N), int(K))
    ws = torch.empty(need, dtype=torch.uint8, device=C.device) if need > 0 else None
    check(lib().dfu_gemm_f32(int(M), int(N), int(K), ptr(A), int(sam), int(sak), ptr(B), int(sbn),
                             int(sbk), ptr(C), int(ldc), ptr(bias), int(relu), int(accumulate),
                             ptr(ws), int(need), stream_ptr()), "dfu_gemm_f32")


def stats_tiles(M):
    return lib().dfu_gemm_stats_tiles(int(M))


# ------------------------------------------------------------------------------- layouts
def pack_conv_weight(w, out=None):
    """fp32 OIHW -> bf16 KRSC."""
    _req(w, F32, "pack_conv_weight")
    K, C, R, S = w.shape
    if out is None:
        out = torch.empty((K, R, S, C), dtype=BF16, device=w.device)
    check(lib().dfu_pack_conv_weight(ptr(w.contiguous()), ptr(out), K, C, R, S, stream_ptr()),
          "dfu_pack_conv_weight")
    return out


def conv_grad_krsc_to_oihw(krsc, oihw):
    K, C, R, S = oihw.shape
    check(lib().dfu_conv_grad_krsc_to_oihw(ptr(krsc), ptr(oihw), K, C, R, S, stream_ptr()),
          "dfu_conv_grad_krsc_to_oihw")


def cast_rows_bf16(x, ld_out=None, out=None):
    """fp32 [rows, cols] -> bf16 [rows, ld_out] (zero-padded columns)."""
    _req(x, F32, "cast_rows_bf16")
    x2 = x.reshape(-1, x.shape[-1])
    if x2.stride(1) != 1:
        x2 = x2.contiguous()
    rows, cols = x2.shape
    ld_out = cols if ld_out is None else ld_out
    if out is None:
        out = torch.empty((rows, ld_out), dtype=BF16, device=x.device)
    check(lib().dfu_cast_rows_bf16(ptr(x2), x2.stride(0), ptr(out), ld_out, rows, cols,
                                   stream_ptr()), "dfu_cast_rows_bf16")
    return out


def cast_rows_f16(x, ld_out=None, out=None):
    """fp32 [rows, cols] -> fp16 [rows, ld_out] (RNE, zero-padded columns)."""
    _req(x, F32, "cast_rows_f16")
    x2 = x.reshape(-1, x.shape[-1])
    if x2.stride(1) != 1:
        x2 = x2.contiguous()
    rows, cols = x2.shape
    ld_out = cols if ld_out is None else ld_out
    if out is None:
        out = torch.empty((rows, ld_out), dtype=F16, device=x.device)
    check(lib().dfu_cast_rows_f16(ptr(x2), x2.stride(0), ptr(out), ld_out, rows, cols,
                                  stream_ptr()), "dfu_cast_rows_f16")
    return out


class TransposeJobs:
    """A device table of bf16 transposes (dfu_transpose_bf16: dst[c][r] = src[r][c]) built once
    and launched as ONE kernel each time (the transposed / flipped weight shadows,
    optim.FlatParams).  src and dst are 2-D views with unit column stride (row strides and
    sizes multiples of 8, 16-B aligned)."""

    def __init__(self, pairs):
        import struct
        raw, tile0 = bytearray(), 0
        for src, dst in pairs:
            _req(src, BF16, "transpose_bf16")
            _req(dst, BF16, "transpose_bf16")
            r, c = src.shape
            ok = (dst.shape == (c, r) and r % 8 == 0 and c % 8 == 0 and src.stride(1) == 1 and
                  dst.stride(1) == 1 and src.stride(0) % 8 == 0 and dst.stride(0) % 8 == 0 and
                  src.data_ptr() % 16 == 0 and dst.data_ptr() % 16 == 0)
            if not ok:
                raise ValueError(f"transpose_bf16: [{r}, {c}] stride {src.stride()} -> "
                                 f"{tuple(dst.shape)} stride {dst.stride()} unsupported")
            raw += struct.pack("<QQiiiiii", src.data_ptr(), dst.data_ptr(), r, c, tile0,
                               src.stride(0), dst.stride(0), 0)
            tile0 += ((r + 63) // 64) * ((c + 63) // 64)
        self.pairs = list(pairs)  # keep the buffers alive as long as the table
        self.njobs, self.ntiles = len(self.pairs), tile0
        dev = self.pairs[0][0].device
        self.table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)

    def launch(self):
        check(lib().dfu_transpose_bf16(ptr(self.table), self.njobs, self.ntiles, stream_ptr()),
              "dfu_transpose_bf16")


def transpose_bf16(src, out=None):
    """bf16 [rows, cols] -> bf16 [cols, rows] (one launch)."""
    if out is None:
        out = torch.empty((src.shape[1], src.shape[0]), dtype=BF16, device=src.device)
    TransposeJobs([(src, out)]).launch()
    return out


def cast_rows_f32(x, out=None):
    _req(x, BF16, "cast_rows_f32")
    x2 = x.reshape(-1, x.shape[-1])
    rows, cols = x2.shape
    if out is None:
        out = torch.empty((rows, cols), dtype=F32, device=x.device)
    check(lib().dfu_cast_rows_f32(ptr(x2), x2.stride(0), ptr(out), out.stride(0), rows, cols,
                                  stream_ptr()), "dfu_cast_rows_f32")
    return out


def im2col_f32(x, R, S, stride, pad, Kp):
    _req(x, F32, "im2col_f32")
    B, C, H, W = x.shape
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - S) // stride + 1
    out = torch.empty((B * P * Q, Kp), dtype=BF16, device=x.device)
    sn, sc, sh, sw = x.stride()
    check(lib().dfu_im2col_f32(ptr(x), sn, sc, sh, sw, B, C, H, W, R, S, stride, pad, P, Q,
                               ptr(out), Kp, stream_ptr()), "dfu_im2col_f32")
    return out, P, Q


def patchify_f32(x, ps):
    _req(x, F32, "patchify_f32")
    B, C, H, W = x.shape
    out = torch.empty((B * (H // ps) * (W // ps), C * ps * ps), dtype=BF16, device=x.device)
    sn, sc, sh, sw = x.stride()
    check(lib().dfu_patchify_f32(ptr(x), sn, sc, sh, sw, B, C, H, W, ps, ptr(out),
                                 stream_ptr()), "dfu_patchify_f32")
    return out


# ------------------------------------------------------------------------------ Grad-CAM
def col2im_f32(dcol, B, C, H, W, R, S, stride, pad, P, Q, Kp):
    """Adjoint of im2col_f32: fp32 [B*P*Q][Kp] column gradients -> fp32 NCHW input gradient."""
    _req(dcol, F32, "col2im_f32")
    dx = torch.empty((B, C, H, W), dtype=F32, device=dcol.device)
    check(lib().dfu_col2im_f32(ptr(dcol), B, C, H, W, R, S, stride, pad, P, Q, Kp, ptr(dx),
                               stream_ptr()), "dfu_col2im_f32")
    return dx


def unpatchify_f32(dpatch, B, C, H, W, ps):
    """Adjoint of patchify_f32: fp32 [B*(H/ps)*(W/ps)][C*ps*ps] -> fp32 NCHW."""
    _req(dpatch, F32, "unpatchify_f32")
    dx = torch.empty((B, C, H, W), dtype=F32, device=dpatch.device)
    check(lib().dfu_unpatchify_f32(ptr(dpatch), B, C, H, W, ps, ptr(dx), stream_ptr()),
          "dfu_unpatchify_f32")
    return dx


def gradcam(act, grad):
    """Grad-CAM maps (B, h, w) fp32 from a hooked activation (B, Ca, h, w) and a gradient
    (B, Cg, h, w): weights from the Cg gradient channels, the map over the first min(Ca, Cg)
    activation channels (grad_cam_visualization.py:415-429).  NCHW or channels_last views."""
    if act.dtype not in (BF16, F32) or not act.is_cuda or not grad.is_cuda:
        raise TypeError("gradcam: bf16/fp32 CUDA tensors expected")
    grad = grad.to(act.dtype)
    B, Ca, h, w = act.shape
    Bg, Cg, hg, wg = grad.shape
    if (B, h, w) != (Bg, hg, wg):
        raise ValueError(f"gradcam: activation {tuple(act.shape)} vs gradient {tuple(grad.shape)}")
    views = []
    for t in (act, grad):
        if t.stride(2) != w * t.stride(3):  # the spatial dims must be one dense position axis
            t = t.contiguous(memory_format=torch.channels_last)
        views.append((t, t.stride(0), t.stride(3), t.stride(1)))
    (a, sab, sap, sac), (g, sgb, sgp, sgc) = views
    cam = torch.empty((B, h, w), dtype=F32, device=act.device)
    check(lib().dfu_gradcam(ptr(a), Ca, sab, sap, sac, ptr(g), Cg, sgb, sgp, sgc,
                            int(a.dtype == BF16), B, h * w, ptr(cam), stream_ptr()), "dfu_gradcam")
    return cam


def saliency(dx):
    """mean_c |dx| per pixel, normalised by its per-image max: (B, H, W) fp32."""
    _req(dx, F32, "saliency")
    dx = dx.contiguous()
    B, C, H, W = dx.shape
    out = torch.empty((B, H, W), dtype=F32, device=dx.device)
    check(lib().dfu_saliency(ptr(dx), B, C, H * W, ptr(out), stream_ptr()), "dfu_saliency")
    return out


# ----------------------------------------------------------------------------- BatchNorm
def _slice_ws(nbytes, device):
    """(workspace, per-stream zeroed counters) for a sliced finalize, or (None, None)."""
    if nbytes <= 0:
        return None, None
    return torch.empty(nbytes // 8, dtype=torch.float64, device=device), tile_counters(device)


def bn_finalize(stats, M, C, gamma, beta, eps, momentum, running_mean, running_var, nbt,
                mean_out, invstd_out, scale_out, shift_out):
    tiles = stats_tiles(M)
    ws, cnt = _slice_ws(lib().dfu_bn_finalize_ws_bytes(tiles, C), stats.device)
    check(lib().dfu_bn_finalize(ptr(stats), tiles, M, C, ptr(gamma), ptr(beta), eps, momentum,
                                ptr(running_mean), ptr(running_var), ptr(nbt), ptr(mean_out),
                                ptr(invstd_out), ptr(scale_out), ptr(shift_out), ptr(ws), ptr(cnt),
                                0 if cnt is None else cnt.numel(), stream_ptr()),
          "dfu_bn_finalize")


def bn_eval_coeffs(gamma, beta, rm, rv, eps, scale_out, shift_out):
    check(lib().dfu_bn_eval_coeffs(ptr(gamma), ptr(beta), ptr(rm), ptr(rv), eps, rm.numel(),
                                   ptr(scale_out), ptr(shift_out), stream_ptr()),
          "dfu_bn_eval_coeffs")


def bn_tile_stats(x, M, C):
    """[ceil(M/128)][2][C] (sum, M2) records of bf16 rows x[M][C] (dfu_bn_finalize's input)."""
    _req(x, BF16, "bn_tile_stats")
    stats = torch.empty((stats_tiles(M), 2, C), dtype=F32, device=x.device)
    check(lib().dfu_bn_tile_stats(ptr(x), int(M), int(C), ptr(stats), stream_ptr()),
          "dfu_bn_tile_stats")
    return stats


def bn_apply(y, scale, shift, residual, relu, out, M, C, mask=None):
    """out = act(y * scale + shift (+ residual)); with `mask` (uint8 [M * C / 8]) also the bitmask
    of out > 0 that bn_bwd(relu=3) reads in place of out."""
    if mask is None:
        check(lib().dfu_bn_apply(ptr(y), ptr(scale), ptr(shift), ptr(residual), int(relu),
                                 ptr(out), M, C, stream_ptr()), "dfu_bn_apply")
    else:
        check(lib().dfu_bn_apply_mask(ptr(y), ptr(scale), ptr(shift), ptr(residual), int(relu),
                                      ptr(out), ptr(mask), M, C, stream_ptr()),
              "dfu_bn_apply_mask")


_BN_BWD_WS = {}  # (M, C) -> dfu_bn_bwd_ws_bytes


def bn_bwd(dout, y, out, relu, mean, invstd, gamma, M, C, dy, dres, dgamma, dbeta,
           batch_stats=True, scale=None, shift=None):
    """Full BN(+residual)(+ReLU) backward: reduce -> finalize -> apply, one C call (dfu_bn_bwd)
    on one workspace.  relu: False/0 none; True/1 mask from the stored output `out`; 2 mask
    recomputed from y with the forward's scale/shift (BN + ReLU without residual; `out` is not
    read); 3 mask from the bitmask bn_apply(mask=) wrote, passed as `out`."""
    relu = int(relu)
    if relu == 2 and (scale is None or shift is None):
        raise ValueError("bn_bwd: relu=2 needs the forward scale/shift")
    lb = lib()
    nb = _BN_BWD_WS.get((M, C))
    if nb is None:
        nb = _BN_BWD_WS[(M, C)] = int(lb.dfu_bn_bwd_ws_bytes(M, C))
    dev = y.device
    ws = torch.empty((nb + 7) // 8, dtype=torch.float64, device=dev)
    cnt = tile_counters(dev)
    rc = lb.dfu_bn_bwd(ptr(dout), y.data_ptr(), ptr(out), relu, ptr(scale), ptr(shift),
                       mean.data_ptr(), invstd.data_ptr(), ptr(gamma), M, C, int(batch_stats),
                       ptr(dgamma), ptr(dbeta), dy.data_ptr(), ptr(dres), ws.data_ptr(), nb,
                       cnt.data_ptr(), cnt.numel(), stream_ptr())
    if rc:
        check(rc, "dfu_bn_bwd")


# ------------------------------------------------------------------------------- pooling
def maxpool_fwd(x, B, H, W, C, scale=None, shift=None):
    """3x3/s2/p1 max pool of NHWC bf16 x; with scale/shift, of bf16(relu(x * scale + shift)) (the
    stem's bn1 + relu fused: dfu_maxpool_bn_fwd)."""
    P = (H - 1) // 2 + 1
    Q = (W - 1) // 2 + 1
    y = torch.empty((B, P, Q, C), dtype=BF16, device=x.device)
    am = torch.empty((B, P, Q, C), dtype=torch.uint8, device=x.device)
    if scale is None:
        check(lib().dfu_maxpool_fwd(ptr(x), B, H, W, C, ptr(y), ptr(am), P, Q, stream_ptr()),
              "dfu_maxpool_fwd")
    else:
        check(lib().dfu_maxpool_bn_fwd(ptr(x), ptr(scale), ptr(shift), B, H, W, C, ptr(y),
                                       ptr(am), P, Q, stream_ptr()), "dfu_maxpool_bn_fwd")
    return y, am, P, Q


def maxpool_bwd(dy, am, B, H, W, C, P, Q):
    dx = torch.empty((B, H, W, C), dtype=BF16, device=dy.device)
    check(lib().dfu_maxpool_bwd(ptr(dy), ptr(am), B, H, W, C, P, Q, ptr(dx), stream_ptr()),
          "dfu_maxpool_bwd")
    return dx


def avgpool_fwd(x, B, HW, C):
    y = torch.empty((B, C), dtype=F32, device=x.device)
    check(lib().dfu_avgpool_fwd(ptr(x), B, HW, C, ptr(y), stream_ptr()), "dfu_avgpool_fwd")
    return y


def avgpool_bwd(dy, B, HW, C):
    dx = torch.empty((B, HW, C), dtype=BF16, device=dy.device)
    check(lib().dfu_avgpool_bwd(ptr(dy), B, HW, C, ptr(dx), stream_ptr()), "dfu_avgpool_bwd")
    return dx


# ----------------------------------------------------------------------------- LayerNorm
def layernorm_fwd(x, ldx, rows, D, gamma, beta, eps, out, ldo, out_bf16, mean, rstd):
    check(lib().dfu_layernorm_fwd(ptr(x), ldx, rows, D, ptr(gamma), ptr(beta), eps, ptr(out),
                                  ldo, int(out_bf16), ptr(mean), ptr(rstd), stream_ptr()),
          "dfu_layernorm_fwd")


def layernorm_bwd(dy, lddy, dy_bf16, x, ldx, mean, rstd, gamma, rows, D, gx, ldg, gx_bf16,
                  dgamma, dbeta, gsum=False, batch=None):
    """LayerNorm backward (gx += dx).  With gsum=True also returns the [blocks][D] partial
    column sums of the updated gx (reduce with reduce_partials_add).  batch: a
    PartialReductions that takes the dgamma / dbeta reductions instead of a launch here."""
    blocks = lib().dfu_ln_bwd_blocks(rows)
    partial = torch.empty((blocks, 2, D), dtype=F32, device=x.device)
    gsp = torch.empty((blocks, D), dtype=F32, device=x.device) if gsum else None
    s = stream_ptr()
    check(lib().dfu_layernorm_bwd(ptr(dy), lddy, int(dy_bf16), ptr(x), ldx, ptr(mean), ptr(rstd),
                                  ptr(gamma), rows, D, ptr(gx), ldg, ptr(gx_bf16), ptr(partial),
                                  ptr(gsp), s), "dfu_layernorm_bwd")
    if batch is not None:
        batch.add(partial, dgamma, D, stride=2 * D, offset=0)
        batch.add(partial, dbeta, D, stride=2 * D, offset=D)
    elif dgamma is not None or dbeta is not None:
        check(lib().dfu_reduce_partials(ptr(partial), blocks, 2, D, ptr(dgamma), ptr(dbeta), s),
              "dfu_reduce_partials")
    return gsp


class PartialReductions:
    """Collects "out += sum over blocks of partial" reductions and runs them as ONE launch
    (dfu_reduce_partials_batch) per flush; the partial slabs stay referenced until then."""

    def __init__(self):
        self.entries = []
        self.keep = []

    def add(self, partial, out, D, stride=None, offset=0, blocks=None):
        if out is None:
            return
        blocks = partial.shape[0] if blocks is None else blocks
        stride = D if stride is None else stride
        self.entries.append((partial.data_ptr() + 4 * offset, stride, out.data_ptr(), blocks, D))
        self.keep.append(partial)
        if len(self.entries) == L.REDUCE_BATCH:
            self.flush()

    def flush(self):
        if not self.entries:
            return
        arr = (L.ReduceEntry * len(self.entries))()
        for i, (p, st, o, b, d) in enumerate(self.entries):
            arr[i].partial, arr[i].stride, arr[i].out, arr[i].blocks, arr[i].D = p, st, o, b, d
        check(lib().dfu_reduce_partials_batch(arr, len(self.entries), stream_ptr()),
              "dfu_reduce_partials_batch")
        self.entries = []
        self.keep = []


def colsum_partial(x, is_bf16=None):
    """Per-block partial column sums of x[rows, N] (the first half of colsum_add)."""
    x2 = x.reshape(-1, x.shape[-1])
    rows, N = x2.shape
    bf = (x.dtype == BF16) if is_bf16 is None else is_bf16
    blocks = lib().dfu_colsum_blocks(rows)
    partial = torch.empty((blocks, N), dtype=F32, device=x.device)
    check(lib().dfu_colsum(ptr(x2), int(bf), x2.stride(0), rows, N, None, ptr(partial),
                           stream_ptr()), "dfu_colsum")
    return partial


def reduce_partials_add(partial, out):
    """out[d] += sum_b partial[b][d]."""
    blocks, D = partial.shape
    check(lib().dfu_reduce_partials(ptr(partial), blocks, 1, D, ptr(out), None, stream_ptr()),
          "dfu_reduce_partials")


# ----------------------------------------------------------------------------- attention
def attention_npad(N):
    return lib().dfu_attention_npad(int(N))


def attention_fwd(qkv, B, N, H, dh, scale):
    o = torch.empty((B * N, H * dh), dtype=BF16, device=qkv.device)
    lse = torch.empty((B * H, attention_npad(N)), dtype=F32, device=qkv.device)
    check(lib().dfu_attention_fwd(ptr(qkv), B, N, H, dh, scale, ptr(o), ptr(lse), stream_ptr()),
          "dfu_attention_fwd")
    return o, lse


def attention_fwd_f16(qkv16, B, N, H, dh, scale):
    """The fp16 forward ("parity" mode): qkv fp16 [B*N][3*H*dh] -> (o fp16, o bf16, lse)."""
    _req(qkv16, F16, "attention_fwd_f16")
    assert qkv16.is_contiguous() and qkv16.shape == (B * N, 3 * H * dh)
    o16 = torch.empty((B * N, H * dh), dtype=F16, device=qkv16.device)
    o = torch.empty((B * N, H * dh), dtype=BF16, device=qkv16.device)
    lse = torch.empty((B * H, attention_npad(N)), dtype=F32, device=qkv16.device)
    check(lib().dfu_attention_fwd_f16(ptr(qkv16), B, N, H, dh, scale, ptr(o16), ptr(o), ptr(lse),
                                      stream_ptr()), "dfu_attention_fwd_f16")
    return o16, o, lse


def attention_bwd(qkv, o, dout, lse, B, N, H, dh, scale, dqkv=None):
    """dqkv (bf16) of attention; qkv bf16, or the fp16 qkv of the parity forward."""
    delta = torch.empty((B * H, attention_npad(N)), dtype=F32, device=qkv.device)
    if dqkv is None:
        dqkv = torch.empty(qkv.shape, dtype=BF16, device=qkv.device)
    fn = lib().dfu_attention_bwd_qkv16 if qkv.dtype == F16 else lib().dfu_attention_bwd
    check(fn(ptr(qkv), ptr(o), ptr(dout), ptr(lse), B, N, H, dh, scale, ptr(delta), ptr(dqkv),
             stream_ptr()), "dfu_attention_bwd")
    return dqkv


# ----------------------------------------------------------------------------- misc
def colsum_add(x, out, is_bf16=None):
    """out[n] += sum over rows of x[rows, N]."""
    x2 = x.reshape(-1, x.shape[-1])
    rows, N = x2.shape
    bf = (x.dtype == BF16) if is_bf16 is None else is_bf16
    blocks = lib().dfu_colsum_blocks(rows)
    partial = torch.empty((blocks, N), dtype=F32, device=x.device)
    check(lib().dfu_colsum(ptr(x2), int(bf), x2.stride(0), rows, N, ptr(out), ptr(partial),
                           stream_ptr()), "dfu_colsum")


def zero_(t):
    check(lib().dfu_zero(ptr(t), t.numel() * t.element_size(), stream_ptr()), "dfu_zero")
    return t


def relu_fwd(x):
    y = torch.empty_like(x)
    check(lib().dfu_relu_fwd(ptr(x), ptr(y), x.numel(), int(x.dtype == BF16), stream_ptr()),
          "dfu_relu_fwd")
    return y


def relu_bwd(dy, y):
    dx = torch.empty_like(y)
    check(lib().dfu_relu_bwd(ptr(dy), ptr(y), ptr(dx), y.numel(), int(y.dtype == BF16),
                             stream_ptr()), "dfu_relu_bwd")
    return dx


def dropout_fwd(x, p, seed, offset_dev):
    y = torch.empty_like(x)
    mask = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    check(lib().dfu_dropout_fwd(ptr(x), ptr(y), ptr(mask), x.numel(), float(p),
                                ctypes.c_uint64(int(seed)), ptr(offset_dev), int(x.dtype == BF16),
                                stream_ptr()), "dfu_dropout_fwd")
    return y, mask


def dropout_bwd(dy, mask, p):
    dx = torch.empty_like(dy)
    check(lib().dfu_dropout_bwd(ptr(dy), ptr(mask), ptr(dx), dy.numel(), float(p),
                                int(dy.dtype == BF16), stream_ptr()), "dfu_dropout_bwd")
    return dx


def concat2_f32(a, b):
    """[a | b] fp32 (rows x (Na+Nb)) by two strided row copies."""
    rows, Na = a.shape
    Nb = b.shape[1]
    out = torch.empty((rows, Na + Nb), dtype=F32, device=a.device)
    s = stream_ptr()
    check(lib().dfu_gather_rows_f32(ptr(a.contiguous()), Na, 1, 0, rows, Na, ptr(out), Na + Nb, s),
          "dfu_gather_rows_f32")
    check(lib().dfu_gather_rows_f32(ptr(b.contiguous()), Nb, 1, 0, rows, Nb, ptr(out[:, Na:]),
                                    Na + Nb, s), "dfu_gather_rows_f32")
    return out


def concat2_bf16(a, b):
    rows = a.shape[0]
    out = torch.empty((rows, a.shape[1] + b.shape[1]), dtype=BF16, device=a.device)
    check(lib().dfu_concat2_bf16(ptr(a.contiguous()), int(a.dtype == BF16), a.shape[1],
                                 ptr(b.contiguous()), int(b.dtype == BF16), b.shape[1], rows,
                                 ptr(out), stream_ptr()), "dfu_concat2_bf16")
    return out


def split2_f32(g, Na, Nb):
    rows = g.shape[0]
    ga = torch.empty((rows, Na), dtype=F32, device=g.device)
    gb = torch.empty((rows, Nb), dtype=F32, device=g.device)
    check(lib().dfu_split2_f32(ptr(g.contiguous()), int(g.dtype == BF16), rows, Na, Nb, ptr(ga),
                               ptr(gb), stream_ptr()), "dfu_split2_f32")
    return ga, gb


def vit_cls_rows(cls, pos, x, B, T, D):
    check(lib().dfu_vit_cls_rows(ptr(cls), ptr(pos), ptr(x), B, T, D, stream_ptr()),
          "dfu_vit_cls_rows")


def vit_embed_bwd(gx, B, T, D, dcls, dpos, dbias):
    gpatch = torch.empty((B * (T - 1), D), dtype=BF16, device=gx.device)
    partial = torch.empty((T, D), dtype=F32, device=gx.device)
    check(lib().dfu_vit_embed_bwd(ptr(gx), B, T, D, ptr(dcls), ptr(dpos), ptr(dbias),
                                  ptr(gpatch), ptr(partial), stream_ptr()), "dfu_vit_embed_bwd")
    return gpatch


def ce_weighted_fwd(logits, labels, weight, loss, dlogits):
    B, C = logits.shape
    check(lib().dfu_ce_weighted_fwd(ptr(logits), ptr(labels), ptr(weight), B, C, ptr(loss),
                                    ptr(dlogits), stream_ptr()), "dfu_ce_weighted_fwd")


def ce_weighted_bwd(saved, grad_loss):
    B, C = saved.shape
    out = torch.empty_like(saved)
    check(lib().dfu_ce_weighted_bwd(ptr(saved), ptr(grad_loss), B, C, ptr(out), stream_ptr()),
          "dfu_ce_weighted_bwd")
    return out


def adamw_flat(p, g, m, v, lr, b1, b2, eps, wd, step_dev, shadow=None, shadow16=None,
               shadow_x3=None, x3_begin=0, x3_end=0):
    """AdamW over the flat range p (dfu_adamw_flat); shadow_x3: the interleaved-pair split of
    elements [x3_begin, x3_end) of the range (2 (x3_end - x3_begin) bf16)."""
    if shadow_x3 is not None:
        assert shadow_x3.numel() >= 2 * (x3_end - x3_begin) and shadow_x3.dtype == BF16
    check(lib().dfu_adamw_flat(ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), lr, b1, b2, eps, wd,
                               ptr(step_dev), ptr(shadow), ptr(shadow16), ptr(shadow_x3),
                               int(x3_begin), int(x3_end), stream_ptr()), "dfu_adamw_flat")


def step_increment(step_dev):
    check(lib().dfu_step_increment(ptr(step_dev), stream_ptr()), "dfu_step_increment")


def argmax_rows(x):
    out = torch.empty((x.shape[0],), dtype=torch.int64, device=x.device)
    check(lib().dfu_argmax_rows(ptr(x), x.shape[0], x.shape[1], ptr(out), stream_ptr()),
          "dfu_argmax_rows")
    return out


def softmax_rows(x):
    """torch.softmax(x, dim=1) of fp32 [rows, C] logits (dfu_softmax_rows)."""
    _req(x, F32, "softmax_rows")
    x = x.contiguous()
    out = torch.empty_like(x)
    check(lib().dfu_softmax_rows(ptr(x), x.shape[0], x.shape[1], ptr(out), stream_ptr()),
          "dfu_softmax_rows")
    return out


# --------------------------------------------------------------- bf16x3 (split) forward
# csrc/precise.hip: a triple is bf16 [rows][3C] = [hi | lo | hi] (pattern 0, GEMM A operand)
# or [hi | hi | lo] (pattern 1, GEMM B operand / weights), hi = bf16(x), lo = bf16(x - hi).
X3_A, X3_B = 0, 1
X3_PAIRS = 2  # B operand of dfu_gemm_desc.x3_pairs: [rows][2 seg], per 32 columns [hi | lo]


def split_x3(x, pattern, seg=None, hi_out=None):
    """fp32 [rows, cols] (any row stride) -> triple [rows, 3*seg] (seg >= cols, zero-padded;
    default cols rounded up to 8), optionally also the plain bf16 hi [rows, seg]."""
    _req(x, F32, "split_x3")
    x2 = x.reshape(x.shape[0], -1) if x.dim() != 2 else x
    if x2.stride(1) != 1:
        x2 = x2.contiguous()
    rows, cols = x2.shape
    if seg is None:
        seg = (cols + 31) // 32 * 32 if pattern == X3_PAIRS else (cols + 7) // 8 * 8
    seg = int(seg)
    out = torch.empty((rows, (2 if pattern == X3_PAIRS else 3) * seg), dtype=BF16,
                      device=x.device)
    check(lib().dfu_split_x3(ptr(x2), x2.stride(0), rows, cols, seg, ptr(out), int(pattern),
                             ptr(hi_out), seg if hi_out is None else hi_out.stride(0),
                             stream_ptr()), "dfu_split_x3")
    return out


def split_x3_into(x, pattern, out):
    """split_x3 of fp32 [rows, seg] (contiguous rows, seg % 32 == 0 for pairs) into `out`."""
    _req(x, F32, "split_x3_into")
    rows, seg = x.shape
    assert x.stride(1) == 1 and out.dtype == BF16 and out.is_contiguous()
    assert out.shape == (rows, (2 if pattern == X3_PAIRS else 3) * seg)
    check(lib().dfu_split_x3(ptr(x), x.stride(0), rows, seg, seg, ptr(out), int(pattern), None,
                             seg, stream_ptr()), "dfu_split_x3")
    return out


def pack_conv_weight_x3(w, pattern=X3_B):
    """fp32 OIHW -> bf16 KRSC' (X3_B: C' = 3C [hi | hi | lo]; X3_PAIRS: C' = 2C interleaved)."""
    _req(w, F32, "pack_conv_weight_x3")
    K, C, R, S = w.shape
    nseg = 2 if pattern == X3_PAIRS else 3
    out = torch.empty((K, R, S, nseg * C), dtype=BF16, device=w.device)
    check(lib().dfu_pack_conv_weight_x3(ptr(w.contiguous()), ptr(out), K, C, R, S, int(pattern),
                                        stream_ptr()), "dfu_pack_conv_weight_x3")
    return out


def im2col_f32_x3(x, R, S, stride, pad, Kp):
    """-> ((hi, lo) split pair [B*P*Q][Kp] each, P, Q)"""
    _req(x, F32, "im2col_f32_x3")
    B, C, H, W = x.shape
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - S) // stride + 1
    hi = torch.empty((B * P * Q, Kp), dtype=BF16, device=x.device)
    lo = torch.empty((B * P * Q, Kp), dtype=BF16, device=x.device)
    sn, sc, sh, sw = x.stride()
    check(lib().dfu_im2col_f32_x3(ptr(x), sn, sc, sh, sw, B, C, H, W, R, S, stride, pad, P, Q,
                                  ptr(hi), ptr(lo), Kp, stream_ptr()), "dfu_im2col_f32_x3")
    return (hi, lo), P, Q


def patchify_f32_x3(x, ps):
    _req(x, F32, "patchify_f32_x3")
    B, C, H, W = x.shape
    out = torch.empty((B * (H // ps) * (W // ps), 3 * C * ps * ps), dtype=BF16, device=x.device)
    sn, sc, sh, sw = x.stride()
    check(lib().dfu_patchify_f32_x3(ptr(x), sn, sc, sh, sw, B, C, H, W, ps, ptr(out),
                                    stream_ptr()), "dfu_patchify_f32_x3")
    return out


def bn_apply_x3(y, scale, shift, residual, res_mode, relu, M, C, out_lo=None, out_bf16=None,
                out_f32=None, y_bf16=None, residual_lo=None, y_lo=None, relu_mask=None):
    """y fp32, or (y_lo given) the bf16 hi of a split pair; res_mode 2: residual is a split pair
    (residual = hi, residual_lo = lo); out_lo + out_bf16 write the output as a split pair
    (out_bf16 = hi); relu_mask (uint8 [M*C/8]): the ReLU bitmask for bn_bwd(relu=3)."""
    _req(y, F32 if y_lo is None else BF16, "bn_apply_x3")
    check(lib().dfu_bn_apply_x3(ptr(y), ptr(y_lo), ptr(scale), ptr(shift), ptr(residual),
                                ptr(residual_lo), int(res_mode), int(relu), ptr(out_lo),
                                ptr(out_bf16), ptr(out_f32), ptr(y_bf16), ptr(relu_mask), int(M),
                                int(C), stream_ptr()), "dfu_bn_apply_x3")


def maxpool_fwd_x3(x, B, H, W, C):
    """-> (lo [B*P*Q, C], hi = plain bf16 [B, P, Q, C], argmax, P, Q)"""
    _req(x, F32, "maxpool_fwd_x3")
    P = (H - 1) // 2 + 1
    Q = (W - 1) // 2 + 1
    lo = torch.empty((B * P * Q, C), dtype=BF16, device=x.device)
    y = torch.empty((B, P, Q, C), dtype=BF16, device=x.device)
    am = torch.empty((B, P, Q, C), dtype=torch.uint8, device=x.device)
    check(lib().dfu_maxpool_fwd_x3(ptr(x), B, H, W, C, ptr(lo), ptr(y), ptr(am), P, Q,
                                   stream_ptr()), "dfu_maxpool_fwd_x3")
    return lo, y, am, P, Q


def stem_conv_x3(x, w, stride=2, pad=3, want_col=True):
    """bf16x3 stem conv (dfu_stem_conv_x3): x fp32 (B, 3, H, W) any strides, w fp32 OIHW
    (64, 3, 7, 7) -> (y, y_lo [M, 64] bf16 split pair, stats [M / 128, 2, 64], col [M, 160] bf16
    hi im2col rows or None, P, Q)."""
    _req(x, F32, "stem_conv_x3")
    _req(w, F32, "stem_conv_x3")
    B, C, H, W = x.shape
    K, Cw, R, S = w.shape
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - S) // stride + 1
    M = B * P * Q
    y = torch.empty((M, K), dtype=BF16, device=x.device)
    y_lo = torch.empty((M, K), dtype=BF16, device=x.device)
    stats = torch.empty((max(1, M // 128), 2, K), dtype=F32, device=x.device)
    col = torch.empty((M, 160), dtype=BF16, device=x.device) if want_col else None
    sn, sc, sh, sw = x.stride()
    check(lib().dfu_stem_conv_x3(ptr(x), sn, sc, sh, sw, B, C, H, W, ptr(w.contiguous()), K, R,
                                 S, stride, pad, ptr(y), ptr(y_lo), ptr(stats), ptr(col),
                                 stream_ptr()), "dfu_stem_conv_x3")
    return y, y_lo, stats, col, P, Q


def stem_wgrad_x3(x, dy, dw, stride=2, pad=3):
    """dw [64][147] fp32 += the stem's weight gradient from x fp32 (B, 3, H, W) any strides and
    dy bf16 [B*P*Q, 64] (dfu_stem_wgrad_x3: no im2col rows)."""
    _req(x, F32, "stem_wgrad_x3")
    _req(dy, BF16, "stem_wgrad_x3")
    _req(dw, F32, "stem_wgrad_x3")
    B, C, H, W = x.shape
    if not (dw.is_contiguous() and dw.numel() == 64 * C * 49 and dy.is_contiguous()):
        raise ValueError("stem_wgrad_x3: dw [64][3*7*7] and dy [M][64] contiguous")
    nbytes = int(lib().dfu_stem_wgrad_ws_bytes(B, H, W))
    slab = torch.empty((max(1, nbytes // 4),), dtype=F32, device=x.device)
    sn, sc, sh, sw = x.stride()
    check(lib().dfu_stem_wgrad_x3(ptr(x), sn, sc, sh, sw, B, C, H, W, ptr(dy), 64, 7, 7, stride,
                                  pad, ptr(dw), ptr(slab), nbytes, stream_ptr()),
          "dfu_stem_wgrad_x3")


def stem_conv_x3_ok(x, w, stride, pad):
    """Whether dfu_stem_conv_x3 takes this stem (its geometry checks, host side)."""
    B, C, H, W = x.shape
    K, _, R, S = w.shape
    if (C, K, R, S, stride, pad) != (3, 64, 7, 7, 2, 3) or H < 7 or W < 7 or W > 250:
        return False
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - S) // stride + 1
    return ((P * Q) % 128 == 0 and Q >= 64 and Q % 16 == 0 and Q <= 112 and P % 2 == 0 and
            B * P * Q < (1 << 31))


def maxpool_bn_fwd_x3(y, y_lo, scale, shift, B, H, W, C, relu_mask=None):
    """bn + ReLU + maxpool 3x3/s2/p1 of the split pair (y, y_lo) [B*H*W, C] (dfu_maxpool_bn_fwd_x3)
    -> (lo [B*P*Q, C], hi = plain bf16 [B, P, Q, C], argmax, P, Q); relu_mask (uint8
    [B*H*W*C / 8]) receives the BN output's ReLU bitmask."""
    _req(y, BF16, "maxpool_bn_fwd_x3")
    _req(y_lo, BF16, "maxpool_bn_fwd_x3")
    assert y.is_contiguous() and y_lo.is_contiguous() and y.numel() == B * H * W * C
    assert relu_mask is None or relu_mask.numel() * 8 == y.numel()
    P = (H - 1) // 2 + 1
    Q = (W - 1) // 2 + 1
    lo = torch.empty((B * P * Q, C), dtype=BF16, device=y.device)
    out = torch.empty((B, P, Q, C), dtype=BF16, device=y.device)
    am = torch.empty((B, P, Q, C), dtype=torch.uint8, device=y.device)
    check(lib().dfu_maxpool_bn_fwd_x3(ptr(y), ptr(y_lo), ptr(scale), ptr(shift), B, H, W, C,
                                      ptr(lo), ptr(out), ptr(am), ptr(relu_mask), P, Q,
                                      stream_ptr()), "dfu_maxpool_bn_fwd_x3")
    return lo, out, am, P, Q


def avgpool_fwd_x3(hi, lo, B, HW, C):
    y = torch.empty((B, C), dtype=F32, device=hi.device)
    check(lib().dfu_avgpool_fwd_x3(ptr(hi), ptr(lo), B, HW, C, ptr(y), stream_ptr()),
          "dfu_avgpool_fwd_x3")
    return y


def layernorm_fwd_x3(x, ldx, rows, D, gamma, beta, eps, out3, out_bf16, mean, rstd):
    check(lib().dfu_layernorm_fwd_x3(ptr(x), ldx, rows, D, ptr(gamma), ptr(beta), eps, ptr(out3),
                                     ptr(out_bf16), ptr(mean), ptr(rstd), stream_ptr()),
          "dfu_layernorm_fwd_x3")


def layernorm_fwd_h16(x, ldx, rows, D, gamma, beta, eps, out16, out_bf16, mean, rstd):
    _req(out16, F16, "layernorm_fwd_h16")
    check(lib().dfu_layernorm_fwd_h16(ptr(x), ldx, rows, D, ptr(gamma), ptr(beta), eps,
                                      ptr(out16), ptr(out_bf16), ptr(mean), ptr(rstd),
                                      stream_ptr()), "dfu_layernorm_fwd_h16")


def gelu_x3(hpre):
    rows, N = hpre.shape
    h3 = torch.empty((rows, 3 * N), dtype=BF16, device=hpre.device)
    h = torch.empty((rows, N), dtype=BF16, device=hpre.device)
    hp = torch.empty((rows, N), dtype=BF16, device=hpre.device)
    check(lib().dfu_gelu_x3(ptr(hpre), rows, N, ptr(h3), ptr(h), ptr(hp), stream_ptr()),
          "dfu_gelu_x3")
    return h3, h, hp


def attention_fwd_f32(qkv, B, N, H, dh, scale, qkv_bf16=None):
    """fp32-accurate attention (bf16x3 MFMA) on fp32 qkv -> (o triple, o bf16, lse); also fills
    qkv_bf16 (the plain bf16 copy of qkv) when given."""
    _req(qkv, F32, "attention_fwd_f32")
    D = H * dh
    if qkv_bf16 is not None:
        _req(qkv_bf16, BF16, "attention_fwd_f32")
        assert qkv_bf16.shape == qkv.shape and qkv_bf16.is_contiguous()
    o3 = torch.empty((B * N, 3 * D), dtype=BF16, device=qkv.device)
    o = torch.empty((B * N, D), dtype=BF16, device=qkv.device)
    npad = attention_npad(N)
    lse = torch.empty((B * H, npad), dtype=F32, device=qkv.device)
    check(lib().dfu_attention_fwd_f32(ptr(qkv), B, N, H, dh, scale, npad, ptr(qkv_bf16), ptr(o3),
                                      ptr(o), ptr(lse), stream_ptr()), "dfu_attention_fwd_f32")
    return o3, o, lse


def metrics_accumulate(logits, labels, loss, confusion, loss_sum, batches):
    """Device-side per-step metrics (dfu_metrics_accumulate): confusion int64 [C, C] (label,
    argmax) counts, fp64 loss sum, int64 batch count; no host synchronisation."""
    lg = logits.detach()
    if lg.dtype != F32 or not lg.is_contiguous():
        lg = lg.float().contiguous()
    rows, C = lg.shape
    lf = None
    if loss is not None:
        lf = loss.detach().reshape(1)
        if lf.dtype != F32:
            lf = lf.float()
    check(lib().dfu_metrics_accumulate(ptr(lg), ptr(labels.contiguous()), rows, C, ptr(lf),
                                       ptr(confusion), ptr(loss_sum), ptr(batches),
                                       stream_ptr()), "dfu_metrics_accumulate")
