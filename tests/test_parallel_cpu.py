"""Data-parallel gradient exchange (dfu_hip.parallel) with world_size 2 over
gloo on CPU: bucketed all-reduce of the flat gradient buffer, launched from grad-ready
notifications in reverse parameter order (overlap) or all at finish(), equals the mean of the
per-rank gradients; parameters are broadcast from rank 0."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2
SHAPES = [(64, 32), (32,), (300,), (17, 5), (2,), (1000,)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _grads(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return [torch.randn(s, generator=g) for s in SHAPES]


def _worker(rank, port, overlap, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank))
    try:
        from dfu_hip import functional as Fn
        from dfu_hip import parallel
        from dfu_hip.optim import FlatParams
        r, w, _ = parallel.init_from_env(backend="gloo")
        assert (r, w) == (rank, WORLD)
        torch.manual_seed(rank)  # different replicas before the broadcast
        mod = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(s)) for s in SHAPES])
        parallel.broadcast_parameters(mod)
        flat = FlatParams(list(mod))
        # ~1 KiB buckets: several buckets, some holding one parameter, some several
        red = parallel.GradAllReducer(flat, bucket_mb=1.0 / 1024, overlap=overlap)
        assert len(red.buckets) >= 3
        # no stream of its own (the step's streams must fit the box's
        # 4 hardware queues): collectives ride the producing stream, asynchronously
        assert not any(isinstance(v, torch.cuda.Stream) for v in vars(red).values())
        for p, g in zip(flat.params, _grads(rank)):
            p.grad.copy_(g)
        red.start()
        if overlap:
            for p in reversed(flat.params):  # the order backward produces them
                Fn.grads_done(p)
            assert all(red._issued), "every bucket must launch from grad-ready hooks"
        red.finish()
        red.close()
        data = torch.cat([p.detach().reshape(-1) for p in flat.params])
        grads = torch.cat([p.grad.reshape(-1) for p in flat.params])
        # numpy arrays travel pickled by value (a tensor would pass a shared-memory handle that
        # dies with this process if it exits before the parent has read it)
        q.put((rank, data.numpy(), grads.numpy(), None))
    except Exception as e:  # report to the parent instead of hanging it
        q.put((rank, None, None, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [True, False])
def test_grad_allreduce_world2(overlap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, overlap, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        rank, data, grads, err = q.get(timeout=120)
        assert err is None, f"rank {rank}: {err}"
        res[rank] = (torch.from_numpy(data), torch.from_numpy(grads))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = torch.stack([torch.cat([g.reshape(-1) for g in _grads(r)])
                          for r in range(WORLD)]).mean(0)
    for r in range(WORLD):
        torch.testing.assert_close(res[r][1], expect, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(res[0][0], res[1][0], rtol=0, atol=0)  # broadcast replicas
