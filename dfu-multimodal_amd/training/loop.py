"""The reference's training / validation epoch loop and test-set evaluation on the HIP modules,
with the per-step metrics kept on the device, data-parallel aware.

Reference loop shape (notebooks/train_multimodal_fusion.py:360-451; the single-modality twins
train_rgb_only.py:241-328, train_thermal_only.py:233-320):
  for epoch in 1..NUM_EPOCHS:
      model.train(); for batch: zero_grad, forward, weighted CE, backward, AdamW step,
          loss.item(), torch.max(outputs, 1), .cpu()          <- 3 host syncs per step (:383-386)
      train_loss = sum(loss.item()) / len(loader); accuracy_score, f1_score(average='binary')
      model.eval(); no_grad: the same metrics over the val loader
      history[...].append(...)
      if epoch >= SAVE_BEST_AFTER_EPOCH (3) and val_f1 > best: delete the old best, torch.save
          {'epoch', 'model_state_dict', 'optimizer_state_dict', 'val_f1', 'history'}
  test phase (:457-504): eval, no_grad; per batch the loss, softmax(outputs, 1)[:, 1] and the
      argmax; test_loss = sum / len(loader), accuracy, binary F1; torch.save of
      {'test_preds', 'test_labels', 'test_probs', 'test_acc', 'test_f1', 'test_loss'}.

Here the per-step metrics never leave the GPU: DeviceMetrics accumulates a confusion matrix
(argmax vs label) and the loss sum with dfu_metrics_accumulate, and the host reads them ONCE
per epoch; accuracy and binary F1 (positive class 1, 0 when undefined, as sklearn's
zero_division default reports) come from the confusion counts, so they equal the reference's
sklearn values on the same predictions.

Data parallelism (one process per GPU; the reference has none): with a process
group of world > 1 the loop
  * sums the confusion counts, loss sums and batch counts over ranks before reading them, so
    every rank reports the metrics of the union of the ranks' batches (what one process running
    all of them would report);
  * broadcasts rank 0's buffers (BatchNorm running statistics, updated per rank by the train
    phase's per-rank batches) before every eval phase, as DistributedDataParallel's
    broadcast_buffers does, so the replicas evaluate one model;
  * writes checkpoints and test results on rank 0 only, followed by a barrier;
  * calls set_epoch(epoch) on samplers that have it (data.sharding: every rank draws the same
    weighted sample per epoch and keeps its own shard).
"""
import os

import torch
import torch.distributed as dist

from dfu_hip import functional as Fn
from dfu_hip import ops
from models.checkpoint import save_checkpoint

SAVE_BEST_AFTER_EPOCH = 3  # train_multimodal_fusion.py:46


def _dp_group_size(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


def _is_rank0(group=None):
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank(group) == 0


def _barrier(group=None):
    if _dp_group_size(group) > 1:
        dist.barrier(group)


class DeviceMetrics:
    """Epoch accumulators in HBM: confusion int64 [C][C] (row = label, column = prediction),
    fp64 loss sum, int64 batch count.  update() enqueues one tiny kernel; result() syncs once."""

    def __init__(self, num_classes=2, device="cuda"):
        self.C = num_classes
        self.confusion = torch.zeros((num_classes, num_classes), dtype=torch.int64, device=device)
        self.loss_sum = torch.zeros((1,), dtype=torch.float64, device=device)
        self.batches = torch.zeros((1,), dtype=torch.int64, device=device)

    def update(self, logits, labels, loss=None):
        ops.metrics_accumulate(logits, labels, loss, self.confusion, self.loss_sum, self.batches)

    def all_reduce(self, group=None):
        """Sum every rank's counts (exact: integer counts, fp64 loss sums of fp32 losses)."""
        if _dp_group_size(group) > 1:
            for t in (self.confusion, self.loss_sum, self.batches):
                dist.all_reduce(t, group=group)

    def result(self):
        conf = self.confusion.cpu()  # the epoch's one device->host synchronisation
        loss_sum = float(self.loss_sum.cpu()[0])
        nb = int(self.batches.cpu()[0])
        return metrics_from_confusion(conf, loss_sum, nb)


def metrics_from_confusion(conf, loss_sum, batches):
    """loss = loss_sum / batches (the reference's sum of loss.item() / len(loader)), accuracy,
    and F1: binary F1 of class 1 for two classes (f1_score(average='binary')), macro F1 over
    the classes otherwise (the reference is binary; 'binary' is undefined for more classes)."""
    conf = torch.as_tensor(conf)
    C = conf.shape[0]
    n = int(conf.sum())
    correct = int(conf.diagonal().sum())
    out = {"loss": loss_sum / batches if batches else 0.0, "acc": correct / n if n else 0.0,
           "n": n, "batches": batches, "confusion": conf.tolist()}

    def f1_of(c):
        tp = int(conf[c, c])
        fp = int(conf[:, c].sum()) - tp
        fn = int(conf[c, :].sum()) - tp
        den = 2 * tp + fp + fn
        return 2 * tp / den if den else 0.0
    out["f1"] = f1_of(1) if C == 2 else sum(f1_of(c) for c in range(C)) / C
    return out


def _forward_fn(model):
    """model(rgb, thermal) for the fusion model, model(x) otherwise."""
    def fwd(m, *inputs):
        return m(*inputs)
    return fwd


def _set_epoch(loader, epoch):
    for obj in (loader, getattr(loader, "sampler", None)):
        if obj is not None and hasattr(obj, "set_epoch"):
            obj.set_epoch(epoch)


def broadcast_buffers(model, src=0, group=None):
    """Rank src's buffers (BatchNorm running mean / var / batches tracked) on every rank."""
    if _dp_group_size(group) > 1:
        with torch.no_grad():
            for b in model.buffers():
                dist.broadcast(b.data, src, group=group)


def _check_batch_split(loader):
    """A sampler that splits the sample order by whole batches (data.sharding.
    ShardedSequentialSampler) must split by the loader's own batch size, or the ranks' batches
    are not batches of the single-process run (and the batch-mean losses differ from it)."""
    sampler = getattr(loader, "sampler", None)
    sb, lb = getattr(sampler, "batch_size", None), getattr(loader, "batch_size", None)
    if sb is not None and lb is not None and sb != lb:
        raise ValueError(f"sampler batch_size {sb} != loader batch_size {lb}: pass "
                         f"ShardedSequentialSampler(..., batch_size=<the loader's>)")


def run_epoch(model, loader, criterion, optimizer=None, train=True, reducer=None,
              forward=None, num_classes=2, device="cuda", group=None, collect=None):
    """One pass over `loader` (batches (*inputs, labels) on the GPU).  train=True runs the
    reference's step (zero_grad, forward, criterion, backward, optimizer.step; the DP reducer
    brackets backward when given); train=False runs under no_grad in eval mode.  Metrics are
    summed over the ranks of `group` (data parallelism).  collect: a list that receives
    (logits, labels) per batch (the test phase)."""
    forward = forward or _forward_fn(model)
    _check_batch_split(loader)
    model.train(train)
    met = DeviceMetrics(num_classes, device)
    with torch.set_grad_enabled(train):
        for batch in loader:
            *inputs, labels = batch
            if train:
                optimizer.zero_grad()
                if reducer is not None and reducer.overlap:
                    reducer.start()
            out = forward(model, *inputs)
            loss = criterion(out, labels)
            if train:
                loss.backward()
                Fn.join_grad_streams()
                if reducer is not None:
                    reducer.finish()
                optimizer.step()
            met.update(out.detach(), labels, loss.detach())
            if collect is not None:
                collect.append((out.detach(), labels))
    met.all_reduce(group)
    return met.result()


def fit(model, train_loader, val_loader, criterion, optimizer, num_epochs, checkpoint_dir=None,
        save_best_after=SAVE_BEST_AFTER_EPOCH, reducer=None, forward=None, log=print,
        device="cuda", num_classes=2, group=None):
    """The reference's epoch loop (train_multimodal_fusion.py:360-451).  Returns (history,
    best_val_f1, best_path or None).  Under data parallelism every rank returns the same
    history (metrics of the union of the ranks' batches) and only rank 0 writes checkpoints."""
    history = {"train_loss": [], "train_acc": [], "train_f1": [],
               "val_loss": [], "val_acc": [], "val_f1": []}
    best_val_f1 = 0.0
    best_path = None
    rank0 = _is_rank0(group)
    log = log if rank0 else None
    for epoch in range(1, num_epochs + 1):
        _set_epoch(train_loader, epoch)
        tr = run_epoch(model, train_loader, criterion, optimizer, True, reducer, forward,
                       num_classes, device, group)
        broadcast_buffers(model, group=group)
        va = run_epoch(model, val_loader, criterion, None, False, None, forward, num_classes,
                       device, group)
        for split, r in (("train", tr), ("val", va)):
            history[f"{split}_loss"].append(r["loss"])
            history[f"{split}_acc"].append(r["acc"])
            history[f"{split}_f1"].append(r["f1"])
        if log:
            log(f"[Epoch {epoch}/{num_epochs}] Train Loss: {tr['loss']:.4f}, Acc: {tr['acc']:.4f}, "
                f"F1: {tr['f1']:.4f} | Val Loss: {va['loss']:.4f}, Acc: {va['acc']:.4f}, "
                f"F1: {va['f1']:.4f}")
        if checkpoint_dir is not None and epoch >= save_best_after and va["f1"] > best_val_f1:
            best_val_f1 = va["f1"]
            best_path = os.path.join(str(checkpoint_dir), "best_model.pt")
            if rank0:
                try:
                    if os.path.exists(best_path):
                        os.unlink(best_path)
                except OSError:
                    pass
                save_checkpoint(best_path, epoch, model, optimizer, va["f1"], history)
                if log:
                    log(f"  Saved BEST model (Val F1: {va['f1']:.4f})")
            _barrier(group)
    return history, best_val_f1, best_path


def _gather_rows(t, group=None):
    """Concatenate a per-rank [rows, ...] tensor over the ranks in rank order (rows may differ)."""
    world = _dp_group_size(group)
    if world <= 1:
        return t
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x) for x in ns]
    pad = torch.zeros((max(ns),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[:t.shape[0]] = t
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[:k] for p, k in zip(parts, ns)])


def gather_in_order(tensors, loader, group=None):
    """Every rank's per-sample rows of each tensor, concatenated over the ranks; when the
    loader's sampler knows the shards' sample indices (data.sharding.ShardedSequentialSampler
    .global_indices), the rows are put back at their sample index (the reference's sequential
    order, every sample exactly once)."""
    out = [_gather_rows(t, group) for t in tensors]
    order = getattr(getattr(loader, "sampler", None), "global_indices", None)
    if order is None or _dp_group_size(group) <= 1:
        return out
    idx = torch.tensor(order(), dtype=torch.int64, device=out[0].device)
    if idx.numel() != out[0].shape[0]:
        raise RuntimeError(f"gather_in_order: {out[0].shape[0]} rows for {idx.numel()} samples")
    inv = torch.empty_like(idx)
    inv[idx] = torch.arange(idx.numel(), device=idx.device)
    return [t[inv] for t in out]


def evaluate(model, loader, criterion, forward=None, num_classes=2, device="cuda",
             results_path=None, group=None, log=print):
    """The reference's test phase (train_multimodal_fusion.py:457-504): eval mode, no_grad;
    test_loss = mean of the batch losses, accuracy / binary F1 from the predictions,
    test_probs = softmax(outputs, 1)[:, 1] (dfu_softmax_rows), test_preds = argmax
    (dfu_argmax_rows, torch.max's first maximum).  Returns the reference's result dict; with
    `results_path`, rank 0 also saves it there (torch.save, as :497-504: lists of numpy scalars
    for preds / labels / probs).  Under data parallelism each rank evaluates its shard and the
    dict holds every sample once, in the reference's order when the loader's sampler is a
    data.sharding.ShardedSequentialSampler (its global_indices)."""
    collect = []
    broadcast_buffers(model, group=group)
    r = run_epoch(model, loader, criterion, None, False, None, forward, num_classes, device,
                  group, collect=collect)
    if collect:
        logits = torch.cat([o.float() for o, _ in collect])
        labels = torch.cat([y for _, y in collect])
        probs = ops.softmax_rows(logits)[:, 1].contiguous()
        preds = ops.argmax_rows(logits.contiguous())
    else:
        logits = torch.zeros((0, num_classes), dtype=torch.float32, device=device)
        probs = torch.zeros((0,), dtype=torch.float32, device=device)
        preds = labels = torch.zeros((0,), dtype=torch.int64, device=device)
    preds, labels, probs = gather_in_order((preds, labels, probs), loader, group)
    res = {"test_preds": list(preds.cpu().numpy()), "test_labels": list(labels.cpu().numpy()),
           "test_probs": list(probs.cpu().numpy()), "test_acc": r["acc"], "test_f1": r["f1"],
           "test_loss": r["loss"]}
    if _is_rank0(group):
        if log:
            log(f"Test Loss: {r['loss']:.4f}\nTest Acc:  {r['acc']:.4f}\nTest F1:   {r['f1']:.4f}")
        if results_path is not None:
            torch.save(res, results_path)
    if results_path is not None:
        _barrier(group)
    return res
