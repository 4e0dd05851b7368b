"""Paired RGB + thermal dataset, class-balanced sampling and the split-leakage guard of the
reference training script (notebooks/train_multimodal_fusion.py), as a drop-in module.

Semantics kept (what a training script and its checkpoints depend on):
  * MultimodalDataset(rgb_dir, thermal_dir, split, transform_rgb, transform_thermal)
    (:60-165): images under <dir>/<split>/{healthy,ulcer}/ (recursive, suffixes .jpg .jpeg .png
    .bmp .tif .tiff, case-insensitive), sorted per class; per class the two modalities are paired
    cyclically up to the longer list (pair i = (rgb[i % n_rgb], thermal[i % n_th])), healthy
    pairs (label 0) before ulcer pairs (label 1); a class missing in either modality is skipped;
    then random.shuffle on the module-level `random` state (the script seeds it with 42).
    Items: (rgb, thermal, label) with the transforms applied to PIL RGB images.
  * compute_sha256 / check_multimodal_leakage (:224-257): exact-duplicate images across the
    three splits, per modality, raise RuntimeError.
  * the WeightedRandomSampler of the paired training loader (:259-268): weight 1 / count of
    the pair's class, num_samples = len(pairs), replacement=True.
  * the class weights of the weighted cross-entropy (:341-345): total / count_c (0 for an
    empty class).
Parity: tests/test_data_cpu.py against fixtures produced by running the reference's own class
and functions on a synthetic directory tree (oracle/gen_data_golden.py).
"""
import hashlib
import random
from collections import Counter
from pathlib import Path

import torch
from torch.utils.data import Dataset, WeightedRandomSampler

IMAGE_EXTS = frozenset({".jpg", ".jpeg", ".png", ".bmp", ".tif", ".tiff"})
CLASSES = ("healthy", "ulcer")  # label 0, 1


def scan_images(root):
    """Sorted image paths under `root` (recursive); [] when it does not exist."""
    root = Path(root)
    if not root.exists():
        return []
    return sorted(p for p in root.rglob("*") if p.suffix.lower() in IMAGE_EXTS)


def cyclic_pairs(rgb, thermal, label):
    """(rgb[i % len(rgb)], thermal[i % len(thermal)], label) for i < max(len): the shorter
    modality is cycled; no pairs when either list is empty."""
    if not rgb or not thermal:
        return []
    n = max(len(rgb), len(thermal))
    return [(rgb[i % len(rgb)], thermal[i % len(thermal)], label) for i in range(n)]


class MultimodalDataset(Dataset):
    """train_multimodal_fusion.py:60 MultimodalDataset."""

    def __init__(self, rgb_dir, thermal_dir, split="train", transform_rgb=None,
                 transform_thermal=None, verbose=True):
        self.rgb_dir = Path(rgb_dir) / split
        self.thermal_dir = Path(thermal_dir) / split
        self.transform_rgb = transform_rgb
        self.transform_thermal = transform_thermal
        self.rgb_healthy = scan_images(self.rgb_dir / "healthy")
        self.rgb_ulcer = scan_images(self.rgb_dir / "ulcer")
        self.thermal_healthy = scan_images(self.thermal_dir / "healthy")
        self.thermal_ulcer = scan_images(self.thermal_dir / "ulcer")
        self.pairs = (cyclic_pairs(self.rgb_healthy, self.thermal_healthy, 0)
                      + cyclic_pairs(self.rgb_ulcer, self.thermal_ulcer, 1))
        for name, r, t in (("healthy", self.rgb_healthy, self.thermal_healthy),
                           ("ulcer", self.rgb_ulcer, self.thermal_ulcer)):
            if verbose and not (r and t):
                missing = "RGB" if not r else "Thermal"
                print(f"  Warning: no {missing} {name} images found; skipping {name} pairing")
        random.shuffle(self.pairs)
        if verbose:
            n0 = sum(1 for *_, y in self.pairs if y == 0)
            print(f"  {split.upper()}: {len(self.pairs)} pairs ({n0} healthy, "
                  f"{len(self.pairs) - n0} ulcer)")
            print(f"    RGB: {len(self.rgb_healthy)} healthy, {len(self.rgb_ulcer)} ulcer")
            print(f"    Thermal: {len(self.thermal_healthy)} healthy, "
                  f"{len(self.thermal_ulcer)} ulcer")

    def __len__(self):
        return len(self.pairs)

    def labels(self):
        return [y for *_, y in self.pairs]

    def __getitem__(self, idx):
        from PIL import Image
        rgb_path, thermal_path, label = self.pairs[idx]
        rgb = Image.open(rgb_path).convert("RGB")
        thermal = Image.open(thermal_path).convert("RGB")
        if self.transform_rgb:
            rgb = self.transform_rgb(rgb)
        if self.transform_thermal:
            thermal = self.transform_thermal(thermal)
        return rgb, thermal, torch.tensor(label, dtype=torch.long)


def compute_sha256(path, block_size=65536):
    """SHA-256 of a file's bytes (None when unreadable), train_multimodal_fusion.py:224."""
    h = hashlib.sha256()
    try:
        with open(path, "rb") as f:
            for block in iter(lambda: f.read(block_size), b""):
                h.update(block)
        return h.hexdigest()
    except OSError:
        return None


def split_overlaps(train_ds, val_ds, test_ds):
    """Exact-duplicate counts between the splits' image sets, per modality:
    {"rgb": (tr/val, tr/test, val/test), "thermal": (...)}."""
    out = {}
    for m, key in (("rgb", 0), ("thermal", 1)):
        hashes = [{compute_sha256(p[key]) for p in ds.pairs} for ds in (train_ds, val_ds, test_ds)]
        out[m] = (len(hashes[0] & hashes[1]), len(hashes[0] & hashes[2]),
                  len(hashes[1] & hashes[2]))
    return out


def check_multimodal_leakage(train_ds, val_ds, test_ds, verbose=True):
    """Raise RuntimeError on any exact-image overlap between splits (:233-257)."""
    ov = split_overlaps(train_ds, val_ds, test_ds)
    if verbose:
        for m in ("rgb", "thermal"):
            a, b, c = ov[m]
            print(f"  {m} overlaps tr/val: {a}, tr/test: {b}, val/test: {c}")
    if sum(ov["rgb"]) + sum(ov["thermal"]) > 0:
        raise RuntimeError("Exact-image leakage detected across multimodal splits")


def sample_weights(labels):
    """1 / (count of the sample's class) for each sample (:261-265)."""
    counts = Counter(labels)
    cc = [counts.get(0, 0), counts.get(1, 0)]
    return [1.0 / cc[y] if cc[y] > 0 else 0.0 for y in labels]


def make_weighted_sampler(dataset, generator=None):
    """The paired training loader's sampler (:266): replacement, len(dataset) draws."""
    w = sample_weights(dataset.labels())
    return WeightedRandomSampler(w, num_samples=len(w), replacement=True, generator=generator)


def class_weights(labels):
    """Weighted-CE class weights total / count_c, 0 for an empty class (:341-345)."""
    counts = Counter(labels)
    cc = [counts.get(0, 0), counts.get(1, 0)]
    total = sum(cc) if sum(cc) > 0 else 1
    return torch.tensor([total / c if c > 0 else 0.0 for c in cc], dtype=torch.float)
