"""ORACLE — test infrastructure only.  CPU restatement of the reference's per-sample transforms
(notebooks/train_multimodal_fusion.py:172-205) as torchvision's PIL backend executes them, for
explicit random parameters.  The pixel operations are PIL's own (PIL 12.2 is in the image, the
library torchvision calls for PIL inputs), so the GPU pipeline is pinned against the real code:
  Resize((224, 224))       torchvision F.resize -> img.resize((W, H), BILINEAR), skipped when
                           the size already matches
  RandomHorizontalFlip     img.transpose(FLIP_LEFT_RIGHT);  RandomVerticalFlip: FLIP_TOP_BOTTOM
  RandomRotation(30)       img.rotate(angle, NEAREST, expand=False, center=None, fillcolor=0)
  ColorJitter              ImageEnhance.Brightness / Contrast / Color(img).enhance(factor) in
                           the drawn order
  RandomAffine             img.transform(size, AFFINE, torchvision's inverse matrix about
                           (W/2, H/2), NEAREST, fillcolor=0)
  ToTensor + Normalize     from_numpy(..).permute(2, 0, 1).float().div(255); sub_(mean).div_(std)
torchvision itself is not installed: the inverse-matrix formula (_get_inverse_affine_matrix)
and the parameter draws are restated from its published source ("parity unpinned" for those).

Also: numpy restatements of PIL's resample and of the ImageEnhance blends, checked against
PIL in tests/test_augment_cpu.py (they pin the formulas the HIP kernels implement).
"""
import math

import numpy as np
import torch
from PIL import Image, ImageEnhance

PREC = 22


def inverse_affine_matrix(center, angle, translate, scale, shear):
    """torchvision.transforms.functional._get_inverse_affine_matrix (inverted=True)."""
    rot = math.radians(angle)
    sx, sy = math.radians(shear[0]), math.radians(shear[1])
    cx, cy = center
    tx, ty = translate
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    m = [d, -b, 0.0, -c, a, 0.0]
    m = [x / scale for x in m]
    m[2] += m[0] * (-cx - tx) + m[1] * (-cy - ty)
    m[5] += m[3] * (-cx - tx) + m[4] * (-cy - ty)
    m[2] += cx
    m[5] += cy
    return m


def reference_transform(img, size, mean, std, hflip=False, vflip=False, rotation=None,
                        ops=(), affine=None):
    """img: H x W x 3 uint8.  rotation: angle (the RandomRotation is present) or None;
    ops: [(0 brightness | 1 contrast | 2 saturation, factor)]; affine: (angle, (tx, ty), scale,
    shear) or None.  Returns fp32 (3, H, W)."""
    H, W = size
    im = Image.fromarray(np.ascontiguousarray(img, np.uint8), "RGB")
    if im.size != (W, H):
        im = im.resize((W, H), Image.BILINEAR)
    if hflip:
        im = im.transpose(Image.FLIP_LEFT_RIGHT)
    if vflip:
        im = im.transpose(Image.FLIP_TOP_BOTTOM)
    if rotation is not None:
        im = im.rotate(rotation, Image.NEAREST, expand=False, center=None, fillcolor=(0, 0, 0))
    enh = {0: ImageEnhance.Brightness, 1: ImageEnhance.Contrast, 2: ImageEnhance.Color}
    for op, f in ops:
        im = enh[op](im).enhance(f)
    if affine is not None:
        angle, tr, scale, shear = affine
        m = inverse_affine_matrix([W * 0.5, H * 0.5], angle, tr, scale, shear)
        im = im.transform((W, H), Image.AFFINE, m, Image.NEAREST, fillcolor=(0, 0, 0))
    t = torch.from_numpy(np.array(im, np.uint8, copy=True)).permute(2, 0, 1).contiguous()
    t = t.float().div(255)
    return t.sub_(torch.as_tensor(mean, dtype=torch.float32).view(-1, 1, 1)).div_(
        torch.as_tensor(std, dtype=torch.float32).view(-1, 1, 1))


# ------------------------------------------------------------ numpy restatements of PIL C code
def taps_np(in_size, out_size):
    """Resample.c precompute_coeffs (bilinear, support 1) + normalize_coeffs_8bpc."""
    scale = in_size / out_size
    fs = max(scale, 1.0)
    support = fs
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [max(0.0, 1.0 - abs((x + xmin - center + 0.5) / fs)) for x in range(xmax)]
        ww = sum(w)  # left-to-right, as the C loop accumulates
        for x in range(xmax):
            v = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + v * (1 << PREC)) if v < 0 else int(0.5 + v * (1 << PREC))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def resample_np(img, out_w, out_h, taps=taps_np):
    """Two-pass fixed-point resample (horizontal, then vertical), u8 between passes."""
    def one_pass(a, out, axis):
        bounds, kk = taps(a.shape[axis], out)
        a = np.moveaxis(a.astype(np.int64), axis, 0)
        res = np.empty((out,) + a.shape[1:], np.int64)
        for o in range(out):
            xmin, cnt = bounds[o]
            s = np.full(a.shape[1:], 1 << (PREC - 1), np.int64)
            for j in range(cnt):
                s += a[xmin + j] * int(kk[o, j])
            res[o] = np.clip(s >> PREC, 0, 255)
        return np.moveaxis(res, 0, axis).astype(np.uint8)
    return one_pass(one_pass(np.asarray(img), out_w, 1), out_h, 0)


def grey_np(a):
    a = a.astype(np.int64)
    return (a[..., 0] * 19595 + a[..., 1] * 38470 + a[..., 2] * 7471 + 0x8000) >> 16


def blend_np(deg, img, alpha):
    """ImagingBlend in float32 with truncation and clipping."""
    if alpha == 0.0:
        return deg.astype(np.uint8)
    if alpha == 1.0:
        return img.astype(np.uint8)
    a = np.float32(alpha)
    d = deg.astype(np.float32)
    t = d + a * (img.astype(np.int64) - deg.astype(np.int64)).astype(np.float32)
    return np.clip(np.trunc(t), 0, 255).astype(np.uint8)


def enhance_np(img, op, f):
    if op == 0:
        deg = np.zeros_like(img)
    elif op == 1:
        g = grey_np(img)
        n = g.size
        mean = (2 * int(g.sum()) + n) // (2 * n)
        deg = np.full_like(img, mean)
    else:
        deg = np.repeat(grey_np(img)[..., None], 3, axis=2)
    return blend_np(deg, img, f)


def fixed_gather_np(img, a):
    """Geometry.c affine_fixed with 16.16 coefficients a0 a1 a2' a3 a4 a5', fill 0."""
    H, W = img.shape[:2]
    y, x = np.meshgrid(np.arange(H, dtype=np.int64), np.arange(W, dtype=np.int64), indexing="ij")
    xs = (a[2] + y * a[1] + x * a[0]) >> 16
    ys = (a[5] + y * a[4] + x * a[3]) >> 16
    ok = (xs >= 0) & (xs < W) & (ys >= 0) & (ys < H)
    out = np.zeros_like(img)
    out[ok] = img[ys[ok], xs[ok]]
    return out
