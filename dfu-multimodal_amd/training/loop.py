"""The reference's training / validation epoch loop on the HIP modules, with the per-step
metrics kept on the device.

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

Here the per-step metrics never leave the GPU: DeviceMetrics accumulates a confusion matrix
(argmax vs label) and the loss sum with dfu_metrics_accumulate, and the host reads them ONCE
per epoch; accuracy and binary F1 (positive class 1, 0 when undefined, as sklearn's
zero_division default reports) come from the confusion counts, so they equal the reference's
sklearn values on the same predictions.  The steps themselves are the same calls the
reference's loop makes (model(...), criterion, backward, optimizer.step) on dfu_hip modules.
"""
import os

import torch

from dfu_hip import functional as Fn
from dfu_hip import ops
from models.checkpoint import save_checkpoint

SAVE_BEST_AFTER_EPOCH = 3  # train_multimodal_fusion.py:46


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

    def result(self):
        conf = self.confusion.cpu()  # the epoch's one device->host synchronisation
        loss_sum = float(self.loss_sum.cpu()[0])
        nb = int(self.batches.cpu()[0])
        n = int(conf.sum())
        correct = int(conf.diagonal().sum())
        out = {"loss": loss_sum / nb if nb else 0.0, "acc": correct / n if n else 0.0,
               "n": n, "batches": nb, "confusion": conf.tolist()}
        if self.C == 2:  # sklearn f1_score(average='binary', pos_label=1)
            tp, fp, fn = int(conf[1, 1]), int(conf[0, 1]), int(conf[1, 0])
            den = 2 * tp + fp + fn
            out["f1"] = 2 * tp / den if den else 0.0
        return out


def _forward_fn(model):
    """model(rgb, thermal) for the fusion model, model(x) otherwise."""
    def fwd(m, *inputs):
        return m(*inputs)
    return fwd


def run_epoch(model, loader, criterion, optimizer=None, train=True, reducer=None,
              forward=None, num_classes=2, device="cuda"):
    """One pass over `loader` (batches (*inputs, labels) on the GPU).  train=True runs the
    reference's step (zero_grad, forward, criterion, backward, optimizer.step; the DP reducer
    brackets backward when given); train=False runs under no_grad in eval mode."""
    forward = forward or _forward_fn(model)
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
    return met.result()


def fit(model, train_loader, val_loader, criterion, optimizer, num_epochs, checkpoint_dir=None,
        save_best_after=SAVE_BEST_AFTER_EPOCH, reducer=None, forward=None, log=print,
        device="cuda"):
    """The reference's epoch loop (train_multimodal_fusion.py:360-451).  Returns (history,
    best_val_f1, best_path or None)."""
    history = {"train_loss": [], "train_acc": [], "train_f1": [],
               "val_loss": [], "val_acc": [], "val_f1": []}
    best_val_f1 = 0.0
    best_path = None
    for epoch in range(1, num_epochs + 1):
        tr = run_epoch(model, train_loader, criterion, optimizer, True, reducer, forward,
                       device=device)
        va = run_epoch(model, val_loader, criterion, None, False, None, forward, device=device)
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
            try:
                if os.path.exists(best_path):
                    os.unlink(best_path)
            except OSError:
                pass
            save_checkpoint(best_path, epoch, model, optimizer, va["f1"], history)
            if log:
                log(f"  Saved BEST model (Val F1: {va['f1']:.4f})")
    return history, best_val_f1, best_path
