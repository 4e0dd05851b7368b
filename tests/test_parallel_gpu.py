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
