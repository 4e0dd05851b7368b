"""a HIP-graph capture whose step forks work onto a plain torch stream.

Round 5's C5 split-graph attempt (DESIGN.md experiment log) captured the ViT's pieces forked onto
a plain torch stream and crashed in hipStreamEndCapture.  Reading the capture path gives three
ways such a fork breaks a capture, each handled now:
  * library work left on the fork, not joined back: dfu_hip.graphs.join_forked only knew the
    library's own streams, so the origin's hipStreamEndCapture failed as unjoined -- which HIP
    cannot undo.  try_capture now records every stream a library launch goes to while it
    captures (ops.stream_ptr) and joins each one still capturing;
  * per-stream state first created inside the capture: the split-K tile counters of a stream
    never used before (their zero-fill was recorded into the graph, so eager launches on that
    stream before the first replay read uninitialised counters) -- now a slot of a per-device
    pool zeroed beforehand, taken by host bookkeeping; and a new library stream
    (hipStreamCreate is not capturable: it invalidates the capture of every fork) -- now
    refused with DfuError before the call: the capture joins its forks, ends cleanly, and
    try_capture returns None (eager fallback);
  * non-library work on a fork the step leaves unjoined: the library cannot see it; the capture
    fails and try_capture recovers (or raises a RuntimeError naming the condition).
Each case runs in a child process, so a crash fails this test instead of the test session."""
import json
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

CHILD = textwrap.dedent(r'''
    import json, sys
    import torch
    from dfu_hip import _lib as L, graphs, ops
    DEV = "cuda"
    res = {}
    torch.manual_seed(0)
    M, N, K = 768, 768, 12608
    A = torch.randn(K, M, device=DEV).to(torch.bfloat16)
    B = torch.randn(K, N, device=DEV).to(torch.bfloat16)

    def wgrad(C, split=8):  # split-K through slabs, tile counters of the current stream
        ops.gemm(M, N, K, A, M, B, N, C, N, a_mode=L.OPND_MNMAJOR, b_mode=L.OPND_MNMAJOR,
                 epilogue=L.EPI_F32_ACC, split_k=split)

    # 1. library work forked onto a plain torch stream, never joined by the step
    fork = torch.cuda.Stream()
    C1 = torch.zeros(M, N, device=DEV)
    C2 = torch.zeros(M, N, device=DEV)

    def step1():
        C1.zero_()
        C2.zero_()
        cur = torch.cuda.current_stream()
        fork.wait_stream(cur)
        with torch.cuda.stream(fork):
            wgrad(C2)      # left on the fork: no cur.wait_stream(fork)
        wgrad(C1)
    step1()                # eager warm-up (also creates the fork's tile counters)
    torch.cuda.synchronize()
    ref1, ref2 = C1.clone(), C2.clone()
    msgs = []
    g = graphs.try_capture(step1, log=msgs.append)
    res["unjoined_library_fork"] = dict(captured=g is not None, log=msgs)
    if g is not None:
        C1.fill_(7.0)
        C2.fill_(7.0)
        g.replay()
        torch.cuda.synchronize()
        res["unjoined_library_fork"]["replay_equal"] = bool(torch.equal(C1, ref1) and
                                                            torch.equal(C2, ref2))

    # 2. a stream first used inside the capture needs split-K counters: a slot of the zeroed
    #    per-device pool (host bookkeeping, nothing recorded); eager work on that stream BEFORE
    #    any replay is right, and so is the replay
    cold = torch.cuda.Stream()

    def step2():
        C2.zero_()
        cur = torch.cuda.current_stream()
        cold.wait_stream(cur)
        with torch.cuda.stream(cold):
            wgrad(C2)
        cur.wait_stream(cold)
    msgs = []
    g = graphs.try_capture(step2, log=msgs.append)
    step2()                # eager on the cold stream first
    torch.cuda.synchronize()
    r = dict(captured=g is not None, log=msgs, eager_equal=bool(torch.equal(C2, ref2)))
    if g is not None:
        C2.fill_(7.0)
        g.replay()
        torch.cuda.synchronize()
        r["replay_equal"] = bool(torch.equal(C2, ref2))
    res["cold_stream_counters"] = r

    # 4. a library stream first created inside the capture (hipStreamCreate is not capturable):
    #    refused with DfuError before the call, the capture ends cleanly, eager fallback
    from dfu_hip import functional as Fn

    def step4():
        ws = Fn.wgrad_stream(torch.device(DEV))
        ws.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(ws):
            wgrad(C2)
        torch.cuda.current_stream().wait_stream(ws)
    msgs = []
    g = graphs.try_capture(step4, log=msgs.append)
    C2.zero_()
    step4()                # the eager fallback creates the stream
    torch.cuda.synchronize()
    res["stream_created_in_capture"] = dict(captured=g is not None, log=msgs,
                                            eager_equal=bool(torch.equal(C2, ref2)))

    # 3. non-library work on a fork the step leaves unjoined
    other = torch.cuda.Stream()
    x = torch.zeros(1 << 20, device=DEV)

    def step3():
        cur = torch.cuda.current_stream()
        other.wait_stream(cur)
        with torch.cuda.stream(other):
            x.add_(1.0)    # torch's own kernel: invisible to the library
        wgrad(C1)
    msgs = []
    try:
        g = graphs.try_capture(step3, log=msgs.append)
        C1.zero_()
        wgrad(C1)
        torch.cuda.synchronize()
        res["unjoined_torch_fork"] = dict(captured=g is not None, log=msgs,
                                          eager_equal=bool(torch.equal(C1, ref1)))
    except RuntimeError as e:
        res["unjoined_torch_fork"] = dict(captured=False, log=msgs,
                                          error=str(e).splitlines()[0])
    print("RESULT " + json.dumps(res))
''')


def test_capture_fork_onto_plain_torch_stream():
    import os
    env = dict(os.environ)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(root, "dfu-multimodal_amd"), root,
                                         env.get("PYTHONPATH", "")])
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                       timeout=240)
    line = [s for s in p.stdout.splitlines() if s.startswith("RESULT ")]
    print(p.stdout[-3000:], p.stderr[-3000:])
    assert p.returncode == 0 and line, f"child exited {p.returncode} (a crash, not an exception)"
    res = json.loads(line[0][len("RESULT "):])
    for k, v in res.items():
        print(f"  {k}: {v}")
    r1 = res["unjoined_library_fork"]
    assert r1["captured"] and r1["replay_equal"], r1
    r2 = res["cold_stream_counters"]
    assert r2["captured"] and r2["eager_equal"] and r2["replay_equal"], r2
    r4 = res["stream_created_in_capture"]
    assert not r4["captured"] and r4["eager_equal"], r4
    assert any("DfuError" in m and "inside a HIP-graph capture" in m for m in r4["log"]), r4
    r3 = res["unjoined_torch_fork"]
    # the library cannot join work it never saw: a Python-level failure, never a crash
    assert not r3["captured"], r3
