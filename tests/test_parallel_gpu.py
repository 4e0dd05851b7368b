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

    def launch(k, carrier=None):
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


def _dp_worker(rank, port, overlap, q):
    """One rank of a world-2 data-parallel step on the real fusion model, both ranks on cuda:0
    over gloo (CUDA tensors; RCCL needs one GPU per rank).  The GPU is touched only here, after
    the spawn."""
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE="2", LOCAL_RANK=str(rank))
    try:
        import bench
        from dfu_hip import functional as Fn
        from dfu_hip import nn as hnn
        from dfu_hip.optim import FusedAdamW
        from models.fusion import MultimodalFusionModel
        r, w, _ = parallel.init_from_env(backend="gloo")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        torch.manual_seed(42 + rank)  # different replicas before the broadcast
        model = MultimodalFusionModel(num_classes=2, dropout=0.0).to(dev).train()
        parallel.broadcast_parameters(model)
        opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
        crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=dev))
        rgb, th, y = bench.synthetic(4, dev, seed=42 + rank)  # each rank its own batch

        streams = {}

        def step(red=None):
            opt.zero_grad()
            if red is not None:
                red.start()
            loss = crit(model(rgb, th), y)
            loss.backward()
            # the streams this step ran gradient work or collectives on (besides the process
            # group's own internal stream)
            streams.clear()
            streams.update(Fn._grad_streams)
            cur = torch.cuda.current_stream()
            streams[id(cur)] = cur
            if red is not None:
                streams.update(red.carriers)
            Fn.join_grad_streams()
            if red is not None:
                red.finish()
            torch.cuda.synchronize()

        step()  # this rank's own gradient (no exchange)
        local = opt.flat.grad.clone()
        red = parallel.GradAllReducer(opt.flat, overlap=overlap)
        # overlap: bucketed all-reduce launched from the grad-ready hooks; otherwise every
        # bucket from finish() (bench's graph mode at world > 1)
        step(red)
        nstreams = len({s.cuda_stream for s in streams.values()})
        ncarriers = len(red.carriers)
        got = opt.flat.grad.clone()
        dist.all_reduce(local)  # the expectation: one plain all-reduce of the local gradients
        local /= 2
        torch.cuda.synchronize()
        diff = (got - local).abs().max().item()
        scale = local.abs().max().item()
        g64 = got.double()
        idx = torch.arange(0, got.numel(), 997, device=dev)
        q.put((rank, dict(diff=diff, scale=scale, log=list(red.issue_log), nstreams=nstreams,
                          ncarriers=ncarriers,
                          nbuckets=len(red.buckets), sum=g64.sum().item(),
                          sq=(g64 * g64).sum().item(), sample=got[idx].cpu().numpy()), None))
        red.close()
    except Exception as e:  # report to the parent instead of hanging it
        import traceback
        q.put((rank, None, traceback.format_exc() + repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [True, False])
def test_fusion_dp_world2_overlapped_reducer(overlap):
    """SURVEY §8e check on the real fusion model with overlap=True: the
    averaged gradients equal the mean of the per-rank gradients, both ranks issue the buckets
    in the same order (every one from the hooks), and hold identical averaged gradients.  The
    step stays inside the box's 4 hardware queues: gradient work and
    collective launches use 2 streams (the main stream and the ViT branch's side stream) -- 3
    with the process group's internal one."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, port, overlap, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, d, err = q.get(timeout=240)
        assert err is None, f"rank {rank}: {err}"
        res[rank] = d
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a, b = res[0], res[1]
    print(f"\n[DP world 2, overlap={overlap}] buckets {a['nbuckets']}, issue order r0 {a['log']} r1 {b['log']}; "
          f"max |avg - mean(local)| {a['diff']:.2e} / {b['diff']:.2e} (scale {a['scale']:.2e})")
    print(f"  streams used (grad producers + collective carriers): {a['nstreams']} / "
          f"{b['nstreams']}; carriers {a['ncarriers']}")
    assert a["nstreams"] <= 2 and b["nstreams"] <= 2
    assert a["log"] == b["log"] and sorted(a["log"]) == list(range(a["nbuckets"]))
    for d in (a, b):
        assert d["diff"] <= 1e-6 * max(d["scale"], 1e-30)
    assert a["sum"] == b["sum"] and a["sq"] == b["sq"] and (a["sample"] == b["sample"]).all()


def _dp_oracle_worker(rank, port, q, B):
    """One rank of a world-2 data-parallel step (gloo, both ranks on cuda:0): the HIP fusion
    model in the library default precision on this rank's batch, gradients averaged by the
    overlapped reducer; beside it the fp32 CPU oracle on the same batch and weights, its
    gradients averaged over the ranks too ("compare against N independent
    per-rank CPU computations averaged")."""
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE="2", LOCAL_RANK=str(rank))
    try:
        import copy
        from dfu_hip import functional as Fn
        from dfu_hip import nn as hnn
        from dfu_hip.optim import FusedAdamW
        from models.fusion import MultimodalFusionModel
        from oracle import torch_ref as R
        parallel.init_from_env(backend="gloo")
        torch.set_num_threads(8)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        torch.manual_seed(0)  # the same initial replica on both ranks
        ref = R.MultimodalFusionModel(num_classes=2, dropout=0.0)
        hip = MultimodalFusionModel(num_classes=2, dropout=0.0)
        hip.load_state_dict(ref.state_dict(), strict=True)
        hip = hip.to(dev).train()
        rgb, th, y = R.synthetic_batch(B, seed=42 + rank)  # each rank its own batch
        w = torch.tensor([2.0, 2.0])
        opt = FusedAdamW(hip.parameters(), lr=1e-4, weight_decay=1e-4)
        red = parallel.GradAllReducer(opt.flat, overlap=True)
        opt.zero_grad()
        red.start()
        loss = hnn.CrossEntropyLoss(weight=w.to(dev))(hip(rgb.to(dev), th.to(dev)), y.to(dev))
        loss.backward()
        Fn.join_grad_streams()
        red.finish()
        torch.cuda.synchronize()
        got = {n: p.grad.detach().float().cpu().clone() for n, p in hip.named_parameters()}
        red.close()
        # the oracle on this rank's batch, then the mean over the ranks
        m = copy.deepcopy(ref).train()
        out = m(rgb, th)
        torch.nn.functional.cross_entropy(out, y, weight=w).backward()
        errs = []
        for n, p in m.named_parameters():
            g = p.grad.detach().clone()
            dist.all_reduce(g)
            g /= 2
            if g.norm().item() == 0.0:
                continue
            h = got[n]
            cos = torch.nn.functional.cosine_similarity(h.flatten().double(),
                                                        g.flatten().double(), dim=0).item()
            errs.append((((h - g).norm() / g.norm()).item(), cos, n))
        errs.sort(reverse=True)
        q.put((rank, dict(worst=errs[:5], median=errs[len(errs) // 2][0],
                          min_cos=min(e[1] for e in errs), n=len(errs),
                          checksum=float(sum(v.double().sum() for v in got.values()))), None))
    except Exception as e:
        import traceback
        q.put((rank, None, traceback.format_exc() + repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_fusion_dp_world2_vs_mean_of_rank_oracles():
    """VERDICT round 5 weak item 6 / SURVEY §8e: the averaged gradients of a world-2 step (two
    ranks, own batches of 32 -- C3's 64 pairs in all --, overlapped bucketed all-reduce) against the MEAN OF THE TWO RANKS'
    fp32 CPU ORACLE gradients, under the single-rank parity test's fixed bars (rel L2 <= 0.25
    and cosine >= 0.975 per parameter, median rel <= 0.03); both ranks hold the same average."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_oracle_worker, args=(r, port, q, 32)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, d, err = q.get(timeout=280)
        assert err is None, f"rank {rank}: {err}"
        res[rank] = d
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, d in sorted(res.items()):
        print(f"\n[DP world 2 vs mean of rank oracles, rank {r}] {d['n']} params, median rel "
              f"{d['median']:.3e}, min cos {d['min_cos']:.5f}, worst {d['worst'][:3]}")
        assert d["median"] <= 0.03 and d["min_cos"] >= 0.975
        assert all(e <= 0.25 for e, _, _ in d["worst"]), d["worst"]
    assert res[0]["checksum"] == res[1]["checksum"]
