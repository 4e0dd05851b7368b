"""Checkpoint format compatibility.

The reference saves ``best_model.pt`` as ``{'epoch', 'model_state_dict', 'optimizer_state_dict',
'val_f1', 'history'}`` (notebooks/train_multimodal_fusion.py:433-451), and its evaluation
scripts load checkpoints with a flexible loader that maps the training scripts' ``backbone.*``
prefix onto ``resnet.*`` / ``vit.*`` and skips shape-mismatched heads
(notebooks/extended_metrics.py:40-92, notebooks/fix_checkpoint_keys.py:15-56).  The models of
this package keep torchvision/timm state-dict keys and shapes, so those files load unchanged in
either direction; FusedAdamW's ``state_dict`` uses torch.optim.AdamW's layout.

Loading uses ``torch.load(..., weights_only=True)``: a checkpoint holds tensors, numbers,
lists and dicts only, and nothing in it is executed.  The reference stores sklearn metric
results (numpy.float64 scalars, train_multimodal_fusion.py:428-439) in ``val_f1`` and
``history``; the weights-only unpickler is told about exactly the numpy scalar types that
needs (numpy's scalar reconstructor and dtypes), nothing else.
"""
import numpy as np
import torch

CHECKPOINT_KEYS = ("epoch", "model_state_dict", "optimizer_state_dict", "val_f1", "history")


def make_checkpoint(epoch, model, optimizer, val_f1, history):
    """The reference's checkpoint dict (train_multimodal_fusion.py:433-439)."""
    return {
        "epoch": epoch,
        "model_state_dict": model.state_dict(),
        "optimizer_state_dict": optimizer.state_dict(),
        "val_f1": val_f1,
        "history": history,
    }


def save_checkpoint(path, epoch, model, optimizer, val_f1, history):
    ckpt = make_checkpoint(epoch, model, optimizer, val_f1, history)
    torch.save(ckpt, path)
    return ckpt


def _numpy_scalar_globals():
    """The globals a weights-only load needs for pickled numpy scalars (np.float64(...),
    np.int64(...)): numpy's scalar reconstructor, np.dtype and the concrete dtype classes."""
    try:
        from numpy._core.multiarray import scalar
    except ImportError:  # numpy < 2
        from numpy.core.multiarray import scalar
    allowed = [scalar, np.dtype]
    for t in (np.float64, np.float32, np.int64, np.int32, np.bool_):
        allowed.append(type(np.dtype(t)))
    return allowed


def _load(path, map_location):
    with torch.serialization.safe_globals(_numpy_scalar_globals()):
        return torch.load(path, map_location=map_location, weights_only=True)


def load_checkpoint(path, map_location="cpu"):
    return _load(path, map_location)


def remap_backbone_keys(state_dict, model):
    """``backbone.X`` -> ``resnet.X`` if the model has ``resnet``, else ``vit.X`` if it has
    ``vit`` (extended_metrics.py:52-66); other keys unchanged."""
    out = {}
    for key, value in state_dict.items():
        if key.startswith("backbone."):
            rest = key[len("backbone."):]
            if hasattr(model, "resnet"):
                key = "resnet." + rest
            elif hasattr(model, "vit"):
                key = "vit." + rest
            else:
                key = rest
        out[key] = value
    return out


def remap_multimodal_keys(state_dict):
    """The multimodal evaluation's fix (extended_metrics.py:803-813): ``backbone.X`` ->
    ``resnet.X`` (the RGB branch) and ``vit_backbone.X`` -> ``vit.X`` (the thermal branch);
    other keys unchanged."""
    out = {}
    for key, value in state_dict.items():
        if key.startswith("backbone."):
            key = "resnet." + key[len("backbone."):]
        elif key.startswith("vit_backbone."):
            key = "vit." + key[len("vit_backbone."):]
        out[key] = value
    return out


def load_multimodal_checkpoint(model, checkpoint_path, device="cuda"):
    """extended_metrics.py:795-815: torch.load the multimodal best_model.pt, remap its keys
    (remap_multimodal_keys) and load_state_dict(strict=False).  Returns (missing, unexpected)."""
    ckpt = _load(checkpoint_path, device)
    return model.load_state_dict(remap_multimodal_keys(ckpt["model_state_dict"]), strict=False)


class LoadReport:
    """What load_checkpoint_flexible did: loaded keys and shape-mismatched skips."""

    def __init__(self, loaded, skipped):
        self.loaded = loaded
        self.skipped = skipped

    def __bool__(self):
        return True

    def __repr__(self):
        return f"LoadReport(loaded={len(self.loaded)}, skipped={len(self.skipped)})"


def load_checkpoint_flexible(model, checkpoint_path, device="cuda", verbose=True):
    """extended_metrics.py:40-92: remap ``backbone.*``, load every key present in the model with
    a matching shape, skip shape mismatches (heads of another class count), ``strict=False``.
    Returns False if the file has no ``model_state_dict``, else a (truthy) LoadReport."""
    ckpt = _load(checkpoint_path, device)
    state_dict = ckpt.get("model_state_dict", {}) if isinstance(ckpt, dict) else {}
    if not state_dict:
        return False
    model_state = model.state_dict()
    loaded, skipped = [], []
    for key, value in remap_backbone_keys(state_dict, model).items():
        if key not in model_state:
            continue
        if value.shape != model_state[key].shape:
            if "fc" in key or "head" in key or "classifier" in key:
                skipped.append(f"{key}: {tuple(value.shape)} vs {tuple(model_state[key].shape)}")
            continue
        model_state[key] = value
        loaded.append(key)
    model.load_state_dict(model_state, strict=False)
    if verbose:
        print(f"  Loaded {len(loaded)} layers from checkpoint")
        if skipped:
            print(f"  Skipped {len(skipped)} layers due to shape mismatch")
    return LoadReport(loaded, skipped)


def fix_checkpoint_keys(checkpoint_path, output_path=None):
    """fix_checkpoint_keys.py:15-56: rewrite ``backbone.*`` keys as ``resnet.*`` in place (or
    into output_path).  Returns the checkpoint, or None without a model_state_dict."""
    ckpt = _load(checkpoint_path, "cpu")
    sd = ckpt.get("model_state_dict", {})
    if not sd:
        return None
    if "backbone" in next(iter(sd)):
        sd = {k.replace("backbone.", "resnet."): v for k, v in sd.items()}
    ckpt["model_state_dict"] = sd
    torch.save(ckpt, output_path or checkpoint_path)
    return ckpt
