"""GPU input pipeline (csrc/augment.hip through data/gpu_transforms.py) against the PIL-backed
oracle (oracle/transforms_ref.py): bit-exact fp32 output for the reference's four Compose
pipelines (train_multimodal_fusion.py:172-205) over ragged image sizes and forced parameters
covering every op and op order."""
import itertools
import os
import random
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import data_inputs as DI  # noqa: E402
import transforms_ref as TR  # noqa: E402

from data import gpu_transforms as GT  # noqa: E402
from data import multimodal as MM  # noqa: E402

pytestmark = pytest.mark.gpu

SIZES = [(1, 1), (224, 224), (240, 320), (480, 640), (713, 389), (1000, 30), (31, 900),
         (3000, 2000)]


def _img(h, w, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    a = np.stack([128 + 100 * np.sin(x / (5 + 3 * c) + c) * np.cos(y / (11 + c))
                  for c in range(3)], -1)
    return np.clip(a + rng.normal(0, 12, a.shape), 0, 255).astype(np.uint8)


def _oracle(img, spec, p):
    return TR.reference_transform(img, spec.size, spec.mean, spec.std, p.hflip, p.vflip,
                                  p.angle if spec.rotation else None, p.ops, p.affine)


def _check(imgs, spec, params):
    out = GT.GpuPreprocessor(spec)(imgs, params).cpu()
    assert out.shape == (len(imgs), 3) + tuple(spec.size) and out.dtype == torch.float32
    for i, (im, p) in enumerate(zip(imgs, params)):
        ref = _oracle(im, spec, p)
        bad = (out[i] != ref).sum().item()
        assert bad == 0, f"image {i} {im.shape} {p}: {bad} values differ, " \
                         f"max {(out[i] - ref).abs().max().item()}"


@pytest.mark.parametrize("spec", ["rgb", "thermal"])
def test_eval_transform_bitwise(spec):
    s = GT.rgb_val_test_transform if spec == "rgb" else GT.thermal_val_test_transform
    imgs = [_img(h, w, i) for i, (h, w) in enumerate(SIZES)]
    _check(imgs, s, [GT.AugParams() for _ in imgs])


@pytest.mark.parametrize("spec", ["rgb", "thermal"])
def test_train_transform_sampled_params_bitwise(spec):
    s = GT.rgb_train_transform if spec == "rgb" else GT.thermal_train_transform
    g = torch.Generator().manual_seed(11)
    imgs = [_img(h, w, 50 + i) for i, (h, w) in enumerate(SIZES * 3)]
    _check(imgs, s, [GT.sample_params(s, g) for _ in imgs])


def test_every_colour_op_order_bitwise():
    s = GT.rgb_train_transform
    imgs, params = [], []
    for k, order in enumerate(itertools.permutations([0, 1, 2])):
        for f in ((0.7, 1.3, 0.95), (1.2999, 0.7001, 1.0), (0.0, 1.0, 0.5)):
            imgs.append(_img(180 + 7 * k, 260, len(imgs)))
            params.append(GT.AugParams(hflip=k % 2 == 0, vflip=k % 3 == 0,
                                       angle=(-1) ** k * 4.0 * k,
                                       ops=[(op, f[j]) for j, op in enumerate(order)],
                                       affine=(3.0 * k - 7, (k - 3, 2 - k), 0.85 + 0.05 * k,
                                               (0.0, 0.0)) if k % 2 else None))
    _check(imgs, s, params)


def test_pair_loader_matches_oracle(tmp_path):
    rgb_dir, th_dir = DI.build_tree(str(tmp_path))
    random.seed(42)
    ds = MM.MultimodalDataset(rgb_dir, th_dir, "train", verbose=False)
    torch.manual_seed(3)
    sampler = MM.make_weighted_sampler(ds)
    idx = list(iter(torch.utils.data.BatchSampler(list(sampler), 6, False)))
    torch.manual_seed(3)
    g = torch.Generator().manual_seed(7)
    loader = GT.GpuPairLoader(ds, 6, sampler=MM.make_weighted_sampler(ds), train=True,
                              generator=g, num_threads=3)
    batches = list(loader)
    assert len(batches) == len(loader) == len(idx)
    g = torch.Generator().manual_seed(7)
    for (rgb, th, y), b in zip(batches, idx):
        assert rgb.is_cuda and rgb.shape == (len(b), 3, 224, 224) and th.shape == rgb.shape
        assert y.tolist() == [ds.pairs[i][2] for i in b]
        for j, i in enumerate(b):
            pr = GT.sample_params(GT.rgb_train_transform, g)
            pt = GT.sample_params(GT.thermal_train_transform, g)
            r = _oracle(GT.decode_rgb(ds.pairs[i][0]), GT.rgb_train_transform, pr)
            t = _oracle(GT.decode_rgb(ds.pairs[i][1]), GT.thermal_train_transform, pt)
            assert torch.equal(rgb[j].cpu(), r) and torch.equal(th[j].cpu(), t)
