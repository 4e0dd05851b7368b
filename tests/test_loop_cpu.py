"""Host logic of the data-parallel epoch loop (no GPU): the sharded samplers, the metric
formulas from confusion counts, and the cross-rank metric reduction over gloo at world 2."""
import os

import pytest
import torch

from data.sharding import ShardedSequentialSampler, ShardedWeightedSampler
from training.loop import DeviceMetrics, metrics_from_confusion


@pytest.mark.parametrize("n,world", [(32, 2), (33, 2), (10, 4), (7, 1)])
def test_sharded_samplers_cover_one_draw(n, world):
    w = [1.0 / 3 if i % 3 == 0 else 1.0 / 7 for i in range(n)]
    shards = [ShardedWeightedSampler(w, rank=r, world_size=world, seed=5) for r in range(world)]
    for e in (1, 2):
        for s in shards:
            s.set_epoch(e)
        full = shards[0].full_draw()
        assert all(s.full_draw() == full for s in shards)  # every rank makes the same draw
        parts = [list(s) for s in shards]
        assert len({len(p) for p in parts}) == 1 and len(parts[0]) == len(shards[0])
        per = len(parts[0])
        padded = full + full[:per * world - n]
        assert sorted(sum(parts, [])) == sorted(padded)
        # interleaved: rank r holds draws r, r + world, ...
        assert [parts[k % world][k // world] for k in range(per * world)] == padded
    # the draw is the weighted sampler's: torch.multinomial with replacement
    g = torch.Generator().manual_seed(5 + 2)
    assert shards[0].full_draw() == torch.multinomial(torch.tensor(w, dtype=torch.double), n, True,
                                                      generator=g).tolist()
    for B in (1, 3, 4):
        seq = [ShardedSequentialSampler(n, r, world, batch_size=B) for r in range(world)]
        parts = [list(s) for s in seq]
        # every sample exactly once (no wrap padding), batches of the single-process walk
        assert sorted(sum(parts, [])) == list(range(n))
        assert seq[0].global_indices() == sum(parts, [])
        assert [len(p) for p in parts] == [len(s) for s in seq]
        for r, p in enumerate(parts):
            for k in range(0, len(p), B):
                blk = p[k:k + B]
                j = blk[0] // B
                assert j % world == r and blk == list(range(j * B, min(n, (j + 1) * B)))


def test_sequential_sampler_batch_size_required_and_checked():
    """the val/test shard must split by the loader's batch size."""
    from training.loop import run_epoch
    with pytest.raises(TypeError):
        ShardedSequentialSampler(10, 0, 2)  # batch_size is keyword-only and required

    class _Loader:
        batch_size = 4
        sampler = ShardedSequentialSampler(10, 0, 2, batch_size=3)

        def __iter__(self):
            return iter(())
    with pytest.raises(ValueError, match="batch_size"):
        run_epoch(torch.nn.Identity(), _Loader(), None, train=False, device="cpu")


def test_metrics_from_confusion_matches_sklearn():
    from sklearn.metrics import accuracy_score, f1_score
    g = torch.Generator().manual_seed(0)
    for C in (2, 3):
        L = torch.randint(0, C, (200,), generator=g)
        P = torch.randint(0, C, (200,), generator=g)
        conf = torch.zeros(C, C, dtype=torch.int64)
        for a, b in zip(L.tolist(), P.tolist()):
            conf[a, b] += 1
        r = metrics_from_confusion(conf, 12.5, 5)
        assert r["acc"] == accuracy_score(L, P) and r["loss"] == 2.5
        avg = "binary" if C == 2 else "macro"
        assert abs(r["f1"] - f1_score(L, P, average=avg)) < 1e-12
    assert metrics_from_confusion(torch.zeros(2, 2, dtype=torch.int64), 0.0, 0)["f1"] == 0.0


def _reduce_worker(rank, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        met = DeviceMetrics(2, "cpu")
        met.confusion += torch.tensor([[3, 1], [2, 4]]) * (rank + 1)
        met.loss_sum += 0.5 + rank
        met.batches += 2 + rank
        met.all_reduce()
        q.put((rank, met.result()))
    finally:
        dist.destroy_process_group()


def _order_worker(rank, port, q):
    import torch.distributed as dist

    from training.loop import gather_in_order
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        n, B = 11, 3  # 4 batches, the last short: rank 0 runs batches 0, 2; rank 1 runs 1, 3

        class _L:
            sampler = ShardedSequentialSampler(n, rank, 2, batch_size=B)
        mine = torch.tensor(list(_L.sampler), dtype=torch.int64)
        got, sq = gather_in_order((mine, (mine * mine).float()), _L)
        q.put((rank, got.tolist(), sq.tolist()))
    finally:
        dist.destroy_process_group()


def test_gather_in_order_world2_ragged():
    """val / test under DP with n % world != 0 -- every sample once, in order."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_order_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, got, sq = q.get(timeout=120)
        res[r] = (got, sq)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in (0, 1):
        assert res[r][0] == list(range(11))
        assert res[r][1] == [float(i * i) for i in range(11)]


def test_device_metrics_all_reduce_world2():
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_reduce_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    want = metrics_from_confusion(torch.tensor([[9, 3], [6, 12]]), 2.0, 5)
    assert res[0] == res[1] == want
