"""Single-modality datasets and split-leakage guards of the reference's RGB-only and
thermal-only training scripts (BASELINE configs C1 / C2), as a drop-in module.

Semantics kept:
  * RGBDataset(data_dir, split, transform) (notebooks/train_rgb_only.py:55-97) and
    ThermalDataset (notebooks/train_thermal_only.py:56-98): ImageFolder-style walk of
    <data_dir>/<split>/healthy (label 0) then <data_dir>/<split>/ulcer (label 1), each by
    Path.rglob('*') in the filesystem's order (NOT sorted, unlike the paired dataset), suffixes
    .jpg .jpeg .png .bmp .tif .tiff case-insensitive; no shuffle.  Items:
    (transform(PIL RGB image), int64 label).  `image_paths` / `labels` are lists, as the scripts
    read them.
  * check_split_hash_leakage (train_rgb_only.py:128-167) and check_split_hash_leakage_modality
    (train_thermal_only.py:128-168): SHA-256 of every file per split; any exact duplicate
    across train/val/test raises RuntimeError (unreadable files are skipped).
  * the training sampler (train_rgb_only.py:181-193, train_thermal_only.py:172-181): weight
    1 / count of the sample's class, len(dataset) draws with replacement; class weights of the
    weighted CE total / count_c (train_rgb_only.py:170-176).
Parity: tests/test_single_modality_cpu.py against fixtures produced by running the reference's
own classes and functions on a synthetic tree (oracle/gen_single_golden.py).
"""
from pathlib import Path

import torch
from torch.utils.data import Dataset, WeightedRandomSampler

from .multimodal import IMAGE_EXTS, class_weights, compute_sha256, sample_weights  # noqa: F401


def walk_class(root):
    """Image files under `root` in Path.rglob order; [] when it does not exist."""
    root = Path(root)
    if not root.exists():
        return []
    return [p for p in root.rglob("*") if p.suffix.lower() in IMAGE_EXTS]


class _SingleModalityDataset(Dataset):
    MODALITY = ""

    def __init__(self, data_dir, split="train", transform=None, verbose=True):
        self.data_dir = Path(data_dir) / split
        self.transform = transform
        self.image_paths = []
        self.labels = []
        for label, cls in enumerate(("healthy", "ulcer")):
            paths = walk_class(self.data_dir / cls)
            self.image_paths += paths
            self.labels += [label] * len(paths)
        if verbose:
            print(f"  {split.upper()}: {len(self.image_paths)} images "
                  f"({self.labels.count(0)} healthy, {self.labels.count(1)} ulcer)")

    def __len__(self):
        return len(self.image_paths)

    def __getitem__(self, idx):
        from PIL import Image
        image = Image.open(self.image_paths[idx]).convert("RGB")
        if self.transform:
            image = self.transform(image)
        return image, torch.tensor(self.labels[idx], dtype=torch.long)


class RGBDataset(_SingleModalityDataset):
    """train_rgb_only.py:55 RGBDataset."""
    MODALITY = "rgb"


class ThermalDataset(_SingleModalityDataset):
    """train_thermal_only.py:56 ThermalDataset."""
    MODALITY = "thermal"


def split_hash_overlaps(train_ds, val_ds, test_ds):
    """(train/val, train/test, val/test) exact-duplicate hash counts; unreadable files are
    left out, as the reference's hashes_for does."""
    def hashes(ds):
        return {h for h in (compute_sha256(p) for p in ds.image_paths) if h}
    a, b, c = hashes(train_ds), hashes(val_ds), hashes(test_ds)
    return len(a & b), len(a & c), len(b & c)


def check_split_hash_leakage(train_ds, val_ds, test_ds, max_samples=5, verbose=True):
    """train_rgb_only.py:128: raise RuntimeError on any exact-image overlap between splits."""
    ov = split_hash_overlaps(train_ds, val_ds, test_ds)
    if verbose:
        print(f"  Overlaps - train/val: {ov[0]}, train/test: {ov[1]}, val/test: {ov[2]}")
    if sum(ov) > 0:
        raise RuntimeError("Image leakage detected across splits - aborting training")


def check_split_hash_leakage_modality(train_ds, val_ds, test_ds, max_samples=5, verbose=True):
    """train_thermal_only.py:128 (the thermal script's copy of the same guard)."""
    ov = split_hash_overlaps(train_ds, val_ds, test_ds)
    if verbose:
        print(f"  Overlaps - train/val: {ov[0]}, train/test: {ov[1]}, val/test: {ov[2]}")
    if sum(ov) > 0:
        raise RuntimeError("Image leakage detected across thermal splits")


def make_weighted_sampler(dataset, generator=None):
    """The single-modality training loader's sampler (train_rgb_only.py:185-193)."""
    w = sample_weights(dataset.labels)
    return WeightedRandomSampler(w, num_samples=len(w), replacement=True, generator=generator)
