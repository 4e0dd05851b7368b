"""GPU input pipeline, host side (no GPU): the resize taps computed by the native library, the
16.16 inverse maps and the blend arithmetic, each against PIL itself through the numpy
restatements in oracle/transforms_ref.py (which mirror the HIP kernels' integer arithmetic).
Reference: notebooks/train_multimodal_fusion.py:172-205."""
import os
import sys

import numpy as np
import pytest
import torch
from PIL import Image, ImageEnhance

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import transforms_ref as TR  # noqa: E402

from data import gpu_transforms as GT  # noqa: E402


def _img(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def _smooth(h, w, seed):
    """Low-frequency content: the blends and contrast means see realistic histograms."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    a = np.stack([128 + 100 * np.sin(x / (7 + c) + rng.uniform(0, 6)) * np.cos(y / (9 + c))
                  for c in range(3)], -1)
    return np.clip(a + rng.normal(0, 8, a.shape), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("n_in,n_out", [(1, 224), (7, 224), (224, 224), (225, 224), (300, 224),
                                        (448, 224), (640, 224), (1000, 224), (3024, 224),
                                        (97, 13)])
def test_native_taps_match_restatement(n_in, n_out):
    k, b, kk = GT.resize_taps(n_in, n_out)
    rb, rk = TR.taps_np(n_in, n_out)
    assert k == rk.shape[1]
    np.testing.assert_array_equal(b, rb)
    np.testing.assert_array_equal(kk, rk)


@pytest.mark.parametrize("h,w", [(1, 1), (5, 300), (224, 224), (240, 320), (480, 640),
                                 (713, 389), (1000, 30)])
def test_resample_with_native_taps_is_pil_resize(h, w):
    img = _img(h, w, h * 7 + w)

    def taps(i, o):
        _, b, kk = GT.resize_taps(i, o)
        return b, kk
    ours = TR.resample_np(img, 224, 224, taps)
    ref = np.asarray(Image.fromarray(img).resize((224, 224), Image.BILINEAR))
    np.testing.assert_array_equal(ours, ref)


@pytest.mark.parametrize("angle", [-30.0, -17.25, -0.3, 0.5, 12.0, 29.999])
def test_rotation_fixed_map_is_pil_rotate(angle):
    img = _img(224, 224, 3)
    a = GT.fixed_map(GT.rotate_matrix(angle, 224, 224), 224, 224)
    ref = np.asarray(Image.fromarray(img).rotate(angle, Image.NEAREST, fillcolor=(0, 0, 0)))
    np.testing.assert_array_equal(TR.fixed_gather_np(img, a), ref)


@pytest.mark.parametrize("params", [(-20.0, (-22, 3), 0.8), (7.5, (0, 0), 1.0),
                                    (19.9, (22, -22), 1.2), (-3.1, (5, 11), 0.93)])
def test_affine_fixed_map_is_pil_transform(params):
    img = _img(224, 224, 4)
    angle, tr, sc = params
    m = GT.affine_matrix(angle, tr, sc, (0.0, 0.0), 224, 224)
    assert m == TR.inverse_affine_matrix([112.0, 112.0], angle, tr, sc, (0.0, 0.0))
    a = GT.fixed_map(m, 224, 224)
    ref = np.asarray(Image.fromarray(img).transform((224, 224), Image.AFFINE, m, Image.NEAREST,
                                                    fillcolor=(0, 0, 0)))
    np.testing.assert_array_equal(TR.fixed_gather_np(img, a), ref)


@pytest.mark.parametrize("op", [0, 1, 2])
@pytest.mark.parametrize("f", [0.0, 0.7, 0.7312345, 1.0, 1.05, 1.3])
def test_enhance_arithmetic_is_pil(op, f):
    img = _smooth(224, 224, op)
    cls = {0: ImageEnhance.Brightness, 1: ImageEnhance.Contrast, 2: ImageEnhance.Color}[op]
    f = float(np.float32(f))
    ref = np.asarray(cls(Image.fromarray(img)).enhance(f))
    np.testing.assert_array_equal(TR.enhance_np(img, op, f), ref)


def test_grey_is_pil_convert_L():
    img = _img(64, 64, 9)
    np.testing.assert_array_equal(TR.grey_np(img), np.asarray(Image.fromarray(img).convert("L")))


def test_param_draw_order_and_ranges():
    g = torch.Generator().manual_seed(0)
    ps = [GT.sample_params(GT.rgb_train_transform, g) for _ in range(400)]
    assert any(p.hflip for p in ps) and not all(p.hflip for p in ps)
    assert all(-30 <= p.angle <= 30 for p in ps)
    jit = [p for p in ps if p.ops]
    aff = [p for p in ps if p.affine]
    assert 0.45 < len(jit) / len(ps) < 0.75 and 0.45 < len(aff) / len(ps) < 0.75
    for p in jit:
        assert sorted(op for op, _ in p.ops) == [0, 1, 2]
        assert all(0.7 <= f <= 1.3 for _, f in p.ops)
    for p in aff:
        ang, (tx, ty), s, sh = p.affine
        assert -20 <= ang <= 20 and -22 <= tx <= 22 and -22 <= ty <= 22 and 0.8 <= s <= 1.2
        assert sh == (0.0, 0.0) and isinstance(tx, int)
    # thermal: no colour jitter; same seed -> same draws
    g1, g2 = torch.Generator().manual_seed(5), torch.Generator().manual_seed(5)
    a = [GT.sample_params(GT.thermal_train_transform, g1) for _ in range(20)]
    b = [GT.sample_params(GT.thermal_train_transform, g2) for _ in range(20)]
    assert a == b and not any(p.ops for p in a)
    assert not GT.rgb_val_test_transform.random and GT.thermal_val_test_transform.mean == (0.5,) * 3


def test_pack_params_layout():
    p = GT.AugParams(hflip=True, angle=10.0, ops=[(1, 0.8), (0, 1.2)],
                     affine=(5.0, (1, 2), 1.1, (0.0, 0.0)))
    r = GT.pack_params([p, GT.AugParams()], GT.rgb_train_transform)
    assert r.itemsize == 92 and r["hflip"][0] == 1 and r["rotate"][0] == 1
    assert r["affine"][0] == 1 and r["n_ops"][0] == 2 and list(r["op"][0][:2]) == [1, 0]
    assert r["rotate"][1] == 0 and r["affine"][1] == 0 and r["n_ops"][1] == 0
    assert np.float32(r["factor"][0][0]) == np.float32(0.8)
