"""The encoders run on two streams (models.fusion: ViT on a side stream).  Every kernel of the
step is deterministic (split-K through fp32 slabs, BN statistics by fixed-order merges), so two
training steps with concurrent branches must match two serialized steps BITWISE — logits, loss,
every gradient and every updated parameter.  A missing stream join or a buffer reused across
streams shows up here as a mismatch."""
import pytest
import torch

from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(concurrent, steps=2):
    from dfu_hip import nn as hnn
    from dfu_hip.optim import FusedAdamW
    from models.fusion import MultimodalFusionModel
    torch.manual_seed(0)
    ref = R.MultimodalFusionModel(num_classes=2, dropout=0.0)
    m = MultimodalFusionModel(num_classes=2, dropout=0.0, concurrent_branches=concurrent)
    m.load_state_dict(ref.state_dict())
    m = m.to(DEV).train()
    opt = FusedAdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
    rgb, th, y = R.synthetic_batch(16, seed=3)
    rgb, th, y = rgb.to(DEV), th.to(DEV), y.to(DEV)
    crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=DEV))
    outs, grads = [], None
    for _ in range(steps):
        opt.zero_grad()
        out = m(rgb, th)
        loss = crit(out, y)
        loss.backward()
        if grads is None:
            torch.cuda.synchronize()
            grads = {n: p.grad.clone() for n, p in m.named_parameters()}
        opt.step()
        outs.append((out.detach().clone(), loss.detach().clone()))
    torch.cuda.synchronize()
    return outs, grads, {n: p.detach().clone() for n, p in m.named_parameters()}


def test_concurrent_branches_bitwise_equal_to_serial(monkeypatch):
    # fc1.bias by the colsum pass in both modes (the serial ViT, running alone, would otherwise
    # take the dGELU epilogue's column sums: the same sums in another order)
    from dfu_hip import functional as Fn
    monkeypatch.setattr(Fn, "_DGELU_COLSUM", False)
    o1, g1, p1 = _run(True)
    o0, g0, p0 = _run(False)
    for (a, la), (b, lb) in zip(o1, o0):
        assert torch.equal(a, b) and torch.equal(la, lb)
    bad = [n for n in g0 if not torch.equal(g0[n], g1[n])]
    assert not bad, f"gradients differ: {bad[:5]}"
    bad = [n for n in p0 if not torch.equal(p0[n], p1[n])]
    assert not bad, f"parameters differ after two steps: {bad[:5]}"


def _capture_setup():
    from dfu_hip import functional as Fn
    from dfu_hip import nn as hnn
    from models.fusion import MultimodalFusionModel
    torch.manual_seed(0)
    m = MultimodalFusionModel(num_classes=2, dropout=0.0).to(DEV).train()
    rgb, th, y = R.synthetic_batch(4, seed=3)
    rgb, th, y = rgb.to(DEV), th.to(DEV), y.to(DEV)
    crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=DEV))
    out = {}

    def step():
        m.zero_grad(set_to_none=False)
        loss = crit(m(rgb, th), y)
        loss.backward()
        Fn.join_grad_streams()
        out["loss"] = loss
        return loss
    ref = step().detach().clone()
    torch.cuda.synchronize()
    return step, ref, out


def test_failed_capture_recovers_to_eager():
    """A failed HIP-graph capture -- here an error raised inside the captured step after its
    forward and backward were enqueued (e.g. a DfuError from an unsupported launch, or the
    bench's replay check) -- must leave a process that runs eager steps and HIP-event timing
    normally (bench.py crashed in elapsed_time after a failed capture: the
    capture stream stayed current), with the same results as before the attempt, and a good
    step must still capture afterwards."""
    from dfu_hip import graphs
    step, ref, out = _capture_setup()

    def bad():
        step()
        raise ValueError("forced failure inside the capture")

    msgs = []
    prev = torch.cuda.current_stream()
    g = graphs.try_capture(bad, log=msgs.append)
    assert g is None and msgs and "graph capture failed" in msgs[0]
    assert torch.cuda.current_stream() == prev
    assert not torch.cuda.is_current_stream_capturing()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    got = step().detach().clone()
    e1.record()
    torch.cuda.synchronize()
    assert e0.elapsed_time(e1) > 0
    assert torch.equal(got, ref)
    g = graphs.try_capture(step, log=msgs.append)
    assert g is not None
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out["loss"], ref)


def test_capture_joins_work_left_on_a_side_stream():
    """Work a step leaves on the encoder side stream (never joined back: the round-2 Grad-CAM
    bug) is joined into the capture by try_capture instead of failing it as unjoined -- HIP
    cannot end such a capture, so the streams would stay capturing for the rest of the
    process.  The replay then performs that work too."""
    from dfu_hip import functional as Fn
    from dfu_hip import graphs
    step, ref, out = _capture_setup()
    scratch = torch.zeros(1024, device=DEV)

    def forking():
        step()
        side = Fn.side_stream(DEV)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            scratch.add_(1.0)  # not joined by the step itself

    msgs = []
    g = graphs.try_capture(forking, log=msgs.append)
    assert g is not None and not msgs
    torch.cuda.synchronize()
    scratch.zero_()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(scratch, torch.full_like(scratch, 2.0))
    assert torch.equal(out["loss"], ref)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    step()
    e1.record()
    torch.cuda.synchronize()
    assert e0.elapsed_time(e1) > 0
