"""RCCL pieces of the data-parallel path that one GPU can exercise (the N-rank runs are the
driver's): the ReduceOp.AVG probe and an AVG all-reduce on an nccl (= RCCL) process group."""
import pytest
import torch
import torch.distributed as dist

from dfu_hip import parallel

pytestmark = pytest.mark.gpu


def test_rccl_avg_allreduce_world1():
    assert not dist.is_initialized()
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert parallel._supports_avg() is True
        x = torch.arange(1 << 20, dtype=torch.float32, device="cuda")
        ref = x.clone()
        dist.all_reduce(x, op=dist.ReduceOp.AVG)
        torch.cuda.synchronize()
        assert torch.equal(x, ref)
    finally:
        dist.destroy_process_group()
        parallel._AVG_OK.clear()


def test_bucket_ready_points_are_final():
    """Overlapped all-reduce launches a bucket from the gradient-ready hooks while backward is
    still running.  On the real fusion model, stop the device at each bucket's launch point and
    snapshot its gradients: none may change afterwards (a launch before the last write to its
    slice would all-reduce a partial gradient), and every bucket must launch from the hooks."""
    import bench
    from dfu_hip import functional as Fn
    from dfu_hip import nn as hnn
    from dfu_hip.optim import FusedAdamW
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model, fwd = bench.build("fusion", dev)
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=dev))
    rgb, th, y = bench.synthetic(8, dev, seed=1)
    red = parallel.GradAllReducer(opt.flat, bucket_mb=32.0, overlap=False)  # world 1
    snaps = {}

    def launch(k):
        lo, hi, _ = red.buckets[k]
        torch.cuda.synchronize()
        snaps[k] = opt.flat.grad[lo:hi].clone()
        red._issued[k] = True
    red._launch = launch
    red.overlap = True
    hook = Fn.register_grad_ready_hook(red._on_ready)
    try:
        for _ in range(2):  # the second step runs on warm persistent buffers
            snaps.clear()
            opt.zero_grad()
            red.start()
            loss = crit(fwd(model, rgb, th), y)
            loss.backward()
            Fn.join_grad_streams()
            torch.cuda.synchronize()
            assert len(red.buckets) > 4
            missing = [k for k in range(len(red.buckets)) if k not in snaps]
            assert not missing, f"buckets never launched from the hooks: {missing}"
            for k, s in snaps.items():
                lo, hi, _ = red.buckets[k]
                assert torch.equal(s, opt.flat.grad[lo:hi]), f"bucket {k} changed after launch"
            red._pending = red._issued = None
    finally:
        Fn.remove_grad_ready_hook(hook)
