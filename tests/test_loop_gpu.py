"""The reference's epoch loop under data parallelism and its test-set phase (VERDICT round 2,
items 6 and 7):

  * training.loop.evaluate (train_multimodal_fusion.py:457-504) against the CPU oracle in eval
    mode: bf16x3 logits within 1e-3, softmax[:, 1] probabilities, argmax predictions, the mean
    batch loss, and test_results.pt with the reference's six keys;
  * training.loop.fit (:360-451) as a world-2 data-parallel run of the real fusion model (two
    ranks sharing cuda:0 over gloo; RCCL needs one GPU per rank): both ranks report the same
    history, that history equals a recomputation over the union of the two ranks' batches,
    exactly one best_model.pt is written (by rank 0), the replicas stay identical, and the
    sharded weighted draws of the two ranks make up one draw.
"""
import os

import numpy as np
import pytest
import torch

from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


class _TensorLoader:
    """A DataLoader over in-HBM tensors in the order of `sampler` (batches of batch_size)."""

    def __init__(self, tensors, batch_size, sampler):
        self.tensors = tensors
        self.batch_size = batch_size
        self.sampler = sampler

    def __iter__(self):
        order = list(self.sampler)
        for s in range(0, len(order), self.batch_size):
            idx = torch.tensor(order[s:s + self.batch_size], device=self.tensors[0].device)
            yield tuple(t.index_select(0, idx) for t in self.tensors)

    def __len__(self):
        return -(-len(self.sampler) // self.batch_size)


def _union_metrics(recs):
    """Accuracy / binary F1 / mean batch loss over (logits, labels, loss) batch records, as the
    reference computes them from its per-step lists (sklearn on the whole epoch)."""
    from sklearn.metrics import accuracy_score, f1_score
    P = np.concatenate([np.asarray(r[0]).argmax(1) for r in recs])
    L = np.concatenate([np.asarray(r[1]) for r in recs])
    return (accuracy_score(L, P), f1_score(L, P, average="binary", zero_division=0),
            float(np.mean([r[2] for r in recs])))


def test_evaluate_test_phase_against_oracle(tmp_path):
    import copy

    from dfu_hip import functional as Fn
    from dfu_hip import nn as hnn
    from models import checkpoint as ck
    from models.fusion import MultimodalFusionModel
    from training import loop
    torch.manual_seed(0)
    ref = R.MultimodalFusionModel(num_classes=2, dropout=0.7)
    g = torch.Generator().manual_seed(4)
    with torch.no_grad():  # non-trivial running statistics
        for name, buf in ref.named_buffers():
            if name.endswith("running_mean"):
                buf.copy_(torch.randn(buf.shape, generator=g) * 0.1)
            elif name.endswith("running_var"):
                buf.copy_(torch.rand(buf.shape, generator=g) * 1.5 + 0.5)
    hip = MultimodalFusionModel(num_classes=2, dropout=0.7)
    hip.load_state_dict(ref.state_dict(), strict=True)
    hip = hip.to(DEV)
    N, B = 20, 8  # a ragged last batch, as the reference's test loader has
    rgb, th, y = R.synthetic_batch(N, seed=21)
    w = R.class_weights(y)
    loader = _TensorLoader((rgb.to(DEV), th.to(DEV), y.to(DEV)), B, range(N))
    path = tmp_path / "test_results.pt"
    with Fn.precision("bf16x3"):
        res = loop.evaluate(hip, loader, hnn.CrossEntropyLoss(weight=w.to(DEV)),
                            results_path=str(path), log=None, device=DEV)
    # the oracle's test phase on the same batches
    m = copy.deepcopy(ref).eval()
    logits, losses = [], []
    with torch.no_grad():
        for s in range(0, N, B):
            o = m(rgb[s:s + B], th[s:s + B])
            logits.append(o)
            losses.append(torch.nn.functional.cross_entropy(o, y[s:s + B], weight=w).item())
    logits = torch.cat(logits)
    probs = torch.softmax(logits, 1)[:, 1]
    preds = logits.argmax(1)
    got_p = torch.tensor(np.array(res["test_probs"]))
    dp = (got_p - probs).abs().max().item()
    print(f"\n[test phase] max |prob - oracle| {dp:.2e}, loss {res['test_loss']:.6f} vs "
          f"{np.mean(losses):.6f}")
    assert set(res) == {"test_preds", "test_labels", "test_probs", "test_acc", "test_f1",
                        "test_loss"}
    assert len(res["test_preds"]) == len(res["test_labels"]) == len(res["test_probs"]) == N
    assert [int(v) for v in res["test_labels"]] == y.tolist()
    assert dp <= 1e-3
    margin = (logits[:, 1] - logits[:, 0]).abs()
    sure = margin > 2e-3  # where the oracle's decision is not within the parity bar
    assert torch.equal(torch.tensor(np.array(res["test_preds"]))[sure], preds[sure])
    assert abs(res["test_loss"] - float(np.mean(losses))) <= 1e-3
    from sklearn.metrics import accuracy_score, f1_score
    P = [int(v) for v in res["test_preds"]]
    assert res["test_acc"] == accuracy_score(y.tolist(), P)
    assert res["test_f1"] == f1_score(y.tolist(), P, average="binary", zero_division=0)
    saved = ck.load_checkpoint(str(path))  # weights-only load (numpy scalars allow-listed)
    assert set(saved) == set(res) and saved["test_f1"] == res["test_f1"]
    assert isinstance(saved["test_probs"][0], np.floating)
    assert isinstance(saved["test_preds"][0], np.integer)
    assert np.allclose(np.array(saved["test_probs"]), got_p.numpy())


def _fit_worker(rank, port, ckdir, q):
    """One rank of a world-2 data-parallel fit on the real fusion model (both ranks on cuda:0
    over gloo).  The GPU is touched only here, after the spawn."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE="2", LOCAL_RANK=str(rank))
    import torch.distributed as dist
    try:
        from data.sharding import ShardedSequentialSampler, ShardedWeightedSampler
        from data.multimodal import sample_weights
        from dfu_hip import nn as hnn
        from dfu_hip import parallel
        from dfu_hip.optim import FusedAdamW
        from models.fusion import MultimodalFusionModel
        from training import loop
        parallel.init_from_env(backend="gloo")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        torch.manual_seed(42 + rank)  # different replicas before the broadcast
        model = MultimodalFusionModel(num_classes=2, dropout=0.0).to(dev).train()
        parallel.broadcast_parameters(model)
        opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
        red = parallel.GradAllReducer(opt.flat, overlap=True)
        NT, NV, B = 32, 16, 4
        rgb, th, y = R.synthetic_batch(NT + NV, seed=77)  # the same dataset on every rank
        y[:NT] = (torch.arange(NT) % 3 == 0).long()  # imbalanced: the sampler reweights
        tr = (rgb[:NT].to(dev), th[:NT].to(dev), y[:NT].to(dev))
        va = (rgb[NT:].to(dev), th[NT:].to(dev), y[NT:].to(dev))
        wsamp = ShardedWeightedSampler(sample_weights(y[:NT].tolist()), rank=rank, world_size=2,
                                       seed=42)
        train_loader = _TensorLoader(tr, B, wsamp)
        val_loader = _TensorLoader(va, B, ShardedSequentialSampler(NV, rank, 2, batch_size=B))
        recs = []

        class _Rec(hnn.CrossEntropyLoss):
            def forward(self, logits, target):
                loss = super().forward(logits, target)
                # by value (numpy): tensors through the queue would share memory with a
                # process that may have exited by the time the parent reads them
                recs.append((logits.detach().float().cpu().numpy(), target.cpu().numpy(),
                             loss.item()))
                return loss
        crit = _Rec(weight=torch.tensor([1.5, 3.0], device=dev))
        saves = []
        real_save = loop.save_checkpoint

        def counting_save(*a, **k):
            saves.append(a[1])
            return real_save(*a, **k)
        loop.save_checkpoint = counting_save
        draws = []
        for e in (1, 2, 3):
            wsamp.set_epoch(e)
            draws.append((list(wsamp), wsamp.full_draw()))
        hist, best, path = loop.fit(model, train_loader, val_loader, crit, opt, num_epochs=3,
                                    checkpoint_dir=ckdir, save_best_after=1, reducer=red,
                                    log=None, device=dev)
        torch.cuda.synchronize()
        p64 = opt.flat.data.double()
        bsum = sum(b.double().sum().item() for b in model.buffers() if b.is_floating_point())
        q.put((rank, dict(hist=hist, best=best, path=path, saves=saves, recs=recs, draws=draws,
                          psum=p64.sum().item(), psq=(p64 * p64).sum().item(), bsum=bsum), None))
        red.close()
    except Exception as e:  # report to the parent instead of hanging it
        import traceback
        q.put((rank, None, traceback.format_exc() + repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_fit_world2_data_parallel(tmp_path):
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ckdir = str(tmp_path / "ck")
    os.makedirs(ckdir)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fit_worker, args=(r, port, ckdir, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, d, err = q.get(timeout=300)
        assert err is None, f"rank {rank}: {err}"
        res[rank] = d
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a, b = res[0], res[1]
    print(f"\n[fit DP world 2] history {a['hist']}\n  saves r0 {a['saves']} r1 {b['saves']}")
    assert a["hist"] == b["hist"] and a["best"] == b["best"] and a["path"] == b["path"]
    assert a["psum"] == b["psum"] and a["psq"] == b["psq"]  # identical replicas
    # exactly one checkpoint, written by rank 0 only
    assert b["saves"] == [] and len(a["saves"]) >= 1
    assert os.listdir(os.path.join(str(tmp_path), "ck")) == ["best_model.pt"]
    # the two shards of every epoch's draw make up the shared weighted draw
    for (da, fa), (db, fb) in zip(a["draws"], b["draws"]):
        assert fa == fb and sorted(da + db) == sorted(fa)
    assert a["draws"][0][1] != a["draws"][1][1]  # a fresh draw per epoch
    # metrics = a recomputation over the union of both ranks' batches; per epoch each rank ran
    # 4 train batches (16 draws / B 4) then 2 val batches (8 samples)
    per = 6
    for e in range(3):
        tr = a["recs"][per * e:per * e + 4] + b["recs"][per * e:per * e + 4]
        va = a["recs"][per * e + 4:per * (e + 1)] + b["recs"][per * e + 4:per * (e + 1)]
        for split, recs in (("train", tr), ("val", va)):
            acc, f1, loss = _union_metrics(recs)
            assert a["hist"][f"{split}_acc"][e] == acc
            assert abs(a["hist"][f"{split}_f1"][e] - f1) < 1e-12
            assert abs(a["hist"][f"{split}_loss"][e] - loss) < 1e-6
    # eval on one model: rank 0's buffers were broadcast before every val phase, so both ranks'
    # val logits of the SAME model differ only in their samples (checked via the union above)
    assert a["bsum"] == b["bsum"]
