"""The host-side stream helpers of the hot path (dfu_hip.ops): dfu_stream_wait (a pooled event
per join instead of a torch Event object), the cached current-stream objects and the stream
context without a Stream object per entry -- each against torch's own behaviour."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_stream_wait_orders_a_consumer_after_a_producer():
    from dfu_hip import ops
    dev = torch.device("cuda", 0)
    prod, cons = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    n = 1 << 24
    x = torch.zeros(n, device=dev)
    out = []
    torch.cuda.synchronize()
    for it in range(300):  # more joins than the event ring holds (256): re-recorded events
        # both directions: the producer's next fill must also wait for the consumer's read
        ops.stream_wait(prod, cons)
        with torch.cuda.stream(prod):
            x.fill_(float(it))
            for _ in range(3):  # keep the producer busy so an unordered read would see old data
                x.mul_(1.0)
        ops.stream_wait(cons, prod)
        with ops.on_stream(cons):
            out.append(x[-1:].clone())
    ops.stream_wait(torch.cuda.current_stream(dev), cons)
    torch.cuda.synchronize()
    got = torch.cat(out).cpu()
    assert torch.equal(got, torch.arange(300, dtype=torch.float32))


def test_stream_wait_on_itself_is_a_no_op():
    from dfu_hip import ops
    s = torch.cuda.Stream()
    ops.stream_wait(s, s)
    torch.cuda.synchronize()


def test_on_stream_sets_and_restores_like_torch():
    from dfu_hip import ops
    dev = torch.device("cuda", 0)
    before = torch.cuda.current_stream(dev)
    s = torch.cuda.Stream(dev)
    with ops.on_stream(s) as got:
        assert got is s
        assert torch.cuda.current_stream(dev) == s
        assert ops.stream_ptr() == s.cuda_stream
        inner = torch.cuda.Stream(dev)
        with ops.on_stream(inner):
            assert torch.cuda.current_stream(dev) == inner
        assert torch.cuda.current_stream(dev) == s
    assert torch.cuda.current_stream(dev) == before
    with ops.on_stream(None):
        assert torch.cuda.current_stream(dev) == before
    # an exception inside restores the caller's stream too
    with pytest.raises(RuntimeError):
        with ops.on_stream(s):
            raise RuntimeError("x")
    assert torch.cuda.current_stream(dev) == before


def test_current_stream_is_cached_and_follows_the_context():
    from dfu_hip import ops
    dev = torch.device("cuda", 0)
    a = ops.current_stream()
    assert a is ops.current_stream(0)
    assert a == torch.cuda.current_stream(dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        b = ops.current_stream()
        assert b == s and b.cuda_stream == s.cuda_stream
    assert ops.current_stream() is a
