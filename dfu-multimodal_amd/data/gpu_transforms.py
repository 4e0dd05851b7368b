"""GPU input pipeline: the reference's torchvision transforms (train_multimodal_fusion.py:172-205)
run as two HIP launches per modality per batch (csrc/augment.hip), bit-exact with torchvision's
PIL backend for the same random parameters.

Division of labour (MI355X-first): the host decodes (PIL, exactly as the reference's DataLoader
workers do), draws the per-sample random parameters in torchvision's order, and packs one
pinned staging buffer per batch — descriptors, parameters, resize taps and the decoded bytes —
which crosses PCIe as ONE copy.  Resize, flips, rotation, colour jitter, affine, ToTensor and
Normalize then run on the GPU and the batch lands in HBM as the fp32 NCHW tensors the
reference's model receives.

Parameter draws follow torchvision's transforms (version pinned by the reference's
requirements, not installed here): RandomHorizontalFlip / RandomVerticalFlip
`torch.rand(1) < p`; RandomRotation `uniform_(-deg, deg)`; RandomApply `p < torch.rand(1)`
skips; ColorJitter `randperm(4)` then brightness, contrast, saturation factors
`uniform_(1 - 0.3, 1 + 0.3)`; RandomAffine angle, tx, ty (`int(round(uniform_(-0.1 W, 0.1 W)))`),
scale.  The pixel arithmetic given those parameters is pinned against PIL itself
(tests/test_augment_gpu.py); the draw order is "parity unpinned" (torchvision absent).
"""
import ctypes
import math
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from functools import lru_cache

import numpy as np
import torch

from dfu_hip import _lib as L
from dfu_hip._lib import check

AUG_PROB = 0.6  # train_multimodal_fusion.py:37
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
THERMAL_MEAN = (0.5, 0.5, 0.5)
THERMAL_STD = (0.5, 0.5, 0.5)

BRIGHTNESS, CONTRAST, SATURATION = 0, 1, 2  # enum dfu_aug_op

RESIZE_DESC = np.dtype([("src_off", "<i8"), ("tmp_off", "<i8"), ("coef_off", "<i8"),
                        ("w", "<i4"), ("h", "<i4"), ("ksh", "<i4"), ("ksv", "<i4")])
AUG_PARAMS = np.dtype([("hflip", "<i4"), ("vflip", "<i4"), ("rotate", "<i4"), ("rot", "<i4", 6),
                       ("affine", "<i4"), ("aff", "<i4", 6), ("n_ops", "<i4"), ("op", "<i4", 3),
                       ("factor", "<f4", 3)])
assert RESIZE_DESC.itemsize == 40 and AUG_PARAMS.itemsize == 92  # the C structs


@dataclass(frozen=True)
class TransformSpec:
    """One of the reference's Compose pipelines (resize -> random ops -> normalize)."""
    size: tuple = (224, 224)                 # (H, W) of transforms.Resize
    hflip_p: float = 0.0
    vflip_p: float = 0.0
    rotation: float = 0.0                     # RandomRotation(degrees); 0 = absent
    jitter: tuple = None                      # ColorJitter(brightness, contrast, saturation)
    jitter_p: float = 0.0
    affine: tuple = None                      # RandomAffine(degrees, translate, scale)
    affine_p: float = 0.0
    mean: tuple = IMAGENET_MEAN
    std: tuple = IMAGENET_STD

    @property
    def random(self):
        return bool(self.hflip_p or self.vflip_p or self.rotation or self.jitter or self.affine)


# train_multimodal_fusion.py:172-205
rgb_train_transform = TransformSpec(hflip_p=0.5, vflip_p=0.5, rotation=30,
                                    jitter=(0.3, 0.3, 0.3), jitter_p=AUG_PROB,
                                    affine=(20, (0.1, 0.1), (0.8, 1.2)), affine_p=AUG_PROB)
rgb_val_test_transform = TransformSpec()
thermal_train_transform = TransformSpec(hflip_p=0.5, vflip_p=0.5, rotation=30,
                                        affine=(20, (0.1, 0.1), (0.8, 1.2)), affine_p=AUG_PROB,
                                        mean=THERMAL_MEAN, std=THERMAL_STD)
thermal_val_test_transform = TransformSpec(mean=THERMAL_MEAN, std=THERMAL_STD)


@dataclass
class AugParams:
    """Random parameters of one sample, as torchvision would have drawn them."""
    hflip: bool = False
    vflip: bool = False
    angle: float = 0.0                        # RandomRotation
    ops: list = field(default_factory=list)   # [(op, factor)] ColorJitter, in applied order
    affine: tuple = None                      # (angle, (tx, ty), scale, (shear_x, shear_y))


def _uniform(a, b, g):
    return float(torch.empty(1).uniform_(a, b, generator=g).item())


def sample_params(spec, generator=None):
    """Draw one sample's parameters in the order torchvision's Compose consumes the torch RNG
    (generator None = the global RNG, as the reference's transforms use)."""
    g = generator
    p = AugParams()
    H, W = spec.size
    if spec.hflip_p:
        p.hflip = bool(torch.rand(1, generator=g) < spec.hflip_p)
    if spec.vflip_p:
        p.vflip = bool(torch.rand(1, generator=g) < spec.vflip_p)
    if spec.rotation:
        p.angle = _uniform(-float(spec.rotation), float(spec.rotation), g)
    if spec.jitter is not None and not (spec.jitter_p < torch.rand(1, generator=g)):
        order = torch.randperm(4, generator=g).tolist()
        f = [_uniform(max(0.0, 1 - v), 1 + v, g) for v in spec.jitter]
        p.ops = [(k, f[k]) for k in order if k < 3]   # hue (3) is None in the reference
    if spec.affine is not None and not (spec.affine_p < torch.rand(1, generator=g)):
        deg, (tr_x, tr_y), (s0, s1) = spec.affine
        angle = _uniform(-float(deg), float(deg), g)
        max_dx, max_dy = float(tr_x * W), float(tr_y * H)
        tx = int(round(_uniform(-max_dx, max_dx, g)))
        ty = int(round(_uniform(-max_dy, max_dy, g)))
        scale = _uniform(s0, s1, g)
        p.affine = (angle, (tx, ty), scale, (0.0, 0.0))
    return p


# ------------------------------------------------------------------ inverse maps (host)
def rotate_matrix(angle, W, H):
    """PIL Image.rotate(angle, expand=False, center=None) inverse affine matrix, or None when
    PIL copies the image (angle % 360 == 0).  angle % 360 in {90, 180, 270} takes PIL's
    transpose fast paths, which this pipeline does not model (never drawn by +-30 degrees)."""
    angle = angle % 360.0
    if angle == 0:
        return None
    if angle == 180 or (angle in (90, 270) and W == H):
        raise NotImplementedError("rotation by a multiple of 90 degrees")
    cx, cy = W / 2, H / 2
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0,
         round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]
    m2 = m[0] * -cx + m[1] * -cy + m[2]
    m5 = m[3] * -cx + m[4] * -cy + m[5]
    m[2], m[5] = m2 + cx, m5 + cy
    return m


def affine_matrix(angle, translate, scale, shear, W, H):
    """torchvision F.affine for PIL images: _get_inverse_affine_matrix about the centre
    (W * 0.5, H * 0.5)."""
    cx, cy = W * 0.5, H * 0.5
    tx, ty = translate
    rot = math.radians(angle)
    sx, sy = math.radians(shear[0]), math.radians(shear[1])
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    m = [x / scale for x in (d, -b, 0.0, -c, a, 0.0)]
    m[2] += m[0] * (-cx - tx) + m[1] * (-cy - ty)
    m[5] += m[3] * (-cx - tx) + m[4] * (-cy - ty)
    m[2] += cx
    m[5] += cy
    return m


def fixed_map(m, W, H):
    """PIL Geometry.c affine_fixed: 16.16 coefficients with the pixel-centre terms folded in.
    Raises when PIL would take another path (ImagingScaleAffine for a pure scale, the float
    path when a coordinate leaves +-32768) — neither is reachable by the reference's ranges."""
    if m[1] == 0 and m[3] == 0:
        raise NotImplementedError("pure scaling affine (PIL ImagingScaleAffine)")
    for x, y in ((0, 0), (W, H), (0, H), (W, 0)):
        if abs(m[0] * x + m[1] * y + m[2]) >= 32768.0 or abs(m[3] * x + m[4] * y + m[5]) >= 32768.0:
            raise NotImplementedError("affine map outside PIL's fixed-point range")

    def fix(v):
        v = v * 65536.0 + 0.5
        return int(math.floor(v)) if v < 0 else int(v)
    return [fix(m[0]), fix(m[1]), fix(m[2] + m[0] * 0.5 + m[1] * 0.5),
            fix(m[3]), fix(m[4]), fix(m[5] + m[3] * 0.5 + m[4] * 0.5)]


def pack_params(params, spec):
    """AugParams list -> dfu_aug_params records."""
    H, W = spec.size
    rec = np.zeros(len(params), AUG_PARAMS)
    for i, p in enumerate(params):
        rec["hflip"][i], rec["vflip"][i] = int(p.hflip), int(p.vflip)
        m = rotate_matrix(p.angle, W, H) if p.angle else None
        if m is not None:
            rec["rotate"][i] = 1
            rec["rot"][i] = fixed_map(m, W, H)
        if p.affine is not None:
            rec["affine"][i] = 1
            rec["aff"][i] = fixed_map(affine_matrix(*p.affine, W, H), W, H)
        rec["n_ops"][i] = len(p.ops)
        for k, (op, f) in enumerate(p.ops):
            rec["op"][i][k], rec["factor"][i][k] = op, f
    return rec


# ------------------------------------------------------------------------- resize taps
@lru_cache(maxsize=4096)
def resize_taps(in_size, out_size):
    """(ksize, bounds int32 [out][2], weights int32 [out][ksize]) from the native host code."""
    lib = L.load()
    k = lib.dfu_resize_ksize(in_size, out_size)
    if k <= 0:
        raise ValueError(f"resize {in_size} -> {out_size}")
    bounds = np.empty((out_size, 2), np.int32)
    kk = np.empty((out_size, k), np.int32)
    check(lib.dfu_resize_coeffs(in_size, out_size, bounds.ctypes.data_as(ctypes.c_void_p),
                                kk.ctypes.data_as(ctypes.c_void_p)), "dfu_resize_coeffs")
    return k, bounds, kk


def _align(n, a=256):
    return (n + a - 1) // a * a


class GpuPreprocessor:
    """Applies one TransformSpec to a batch of decoded H x W x 3 uint8 images on the GPU."""

    def __init__(self, spec, device="cuda"):
        self.spec = spec
        self.device = torch.device(device)
        self._mean = (ctypes.c_float * 3)(*spec.mean)
        self._std = (ctypes.c_float * 3)(*spec.std)

    def __call__(self, images, params=None):
        return self.run(self.stage(images, params))

    def stage(self, images, params=None):
        """Host side of one batch: pack descriptors, parameters, resize taps and pixels into one
        pinned buffer and start its single H2D copy on the current stream."""
        spec = self.spec
        OH, OW = spec.size
        n = len(images)
        if n == 0:
            return _Staged(None, 0, 0, 0, 0, 0)
        if params is None:
            params = [AugParams() for _ in range(n)]
        if len(params) != n:
            raise ValueError("one AugParams per image")
        imgs = [np.ascontiguousarray(im, dtype=np.uint8) for im in images]
        for im in imgs:
            if im.ndim != 3 or im.shape[2] != 3 or im.shape[0] < 1 or im.shape[1] < 1:
                raise ValueError(f"expected H x W x 3 uint8 images, got {im.shape}")
        desc = np.zeros(n, RESIZE_DESC)
        taps, coef_len, src_len, tmp_len = [], 0, 0, 0
        for i, im in enumerate(imgs):
            h, w = im.shape[:2]
            kh, bh, wh = resize_taps(w, OW)
            kv, bv, wv = resize_taps(h, OH)
            desc[i] = (src_len, tmp_len, coef_len, w, h, kh, kv)
            taps.append((bh, wh, bv, wv))
            coef_len += bh.size + wh.size + bv.size + wv.size
            src_len += im.size
            tmp_len += h * OW * 3
        rec = pack_params(params, spec)
        # one staging buffer: [descs | params | taps | pixels], 256-byte aligned sections
        o_par = _align(desc.nbytes)
        o_coef = o_par + _align(rec.nbytes)
        o_src = o_coef + _align(coef_len * 4)
        total = o_src + src_len + 4  # the resize reads whole dwords of the last row
        stage = torch.empty(total, dtype=torch.uint8, pin_memory=self.device.type == "cuda")
        buf = stage.numpy()
        buf[:desc.nbytes] = desc.view(np.uint8)
        buf[o_par:o_par + rec.nbytes] = rec.view(np.uint8)
        cv = buf[o_coef:o_coef + coef_len * 4].view(np.int32)
        at = 0
        for t in taps:
            for a in t:
                cv[at:at + a.size] = a.ravel()
                at += a.size
        at = o_src
        for im in imgs:
            buf[at:at + im.size] = im.ravel()
            at += im.size
        return _Staged(stage.to(self.device, non_blocking=True), n, o_par, o_coef, o_src,
                       tmp_len)

    def run(self, st):
        """Device side: resize + augment + normalise a staged batch (4 launches)."""
        OH, OW = self.spec.size
        if st.n == 0:
            return torch.empty((0, 3, OH, OW), dtype=torch.float32, device=self.device)
        lib = L.load()
        base = st.dev.data_ptr()
        tmp = torch.empty(st.tmp_len, dtype=torch.uint8, device=self.device)
        resized = torch.empty(st.n * OH * OW * 3, dtype=torch.uint8, device=self.device)
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        check(lib.dfu_resize_batch(ctypes.c_void_p(base + st.o_src), ctypes.c_void_p(base),
                                   ctypes.c_void_p(base + st.o_coef), st.n, OW, OH,
                                   ctypes.c_void_p(tmp.data_ptr()),
                                   ctypes.c_void_p(resized.data_ptr()), stream),
              "dfu_resize_batch")
        out = torch.empty((st.n, 3, OH, OW), dtype=torch.float32, device=self.device)
        means = torch.empty(st.n, dtype=torch.int32, device=self.device)
        check(lib.dfu_augment_normalize(ctypes.c_void_p(resized.data_ptr()),
                                        ctypes.c_void_p(base + st.o_par), st.n, OH, OW,
                                        self._mean, self._std, ctypes.c_void_p(means.data_ptr()),
                                        ctypes.c_void_p(out.data_ptr()), stream),
              "dfu_augment_normalize")
        return out


@dataclass
class _Staged:
    dev: torch.Tensor      # the batch's staging buffer in HBM
    n: int
    o_par: int
    o_coef: int
    o_src: int
    tmp_len: int


def decode_rgb(path):
    """MultimodalDataset.__getitem__'s decode: Image.open(path).convert('RGB') as H x W x 3."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"))


class GpuPairLoader:
    """DataLoader replacement for MultimodalDataset (train_multimodal_fusion.py:259-275): yields
    (rgb, thermal, label) batches already on the GPU, fp32 NCHW as the reference's loader
    produces them after pin_memory + .to(DEVICE).  Decode runs on `num_threads` host threads
    one batch ahead of the GPU; per sample the RGB parameters are drawn before the thermal
    ones, as __getitem__ applies the two transforms."""

    def __init__(self, dataset, batch_size, sampler=None, shuffle=False, train=False,
                 rgb_spec=None, thermal_spec=None, device="cuda", num_threads=4, generator=None,
                 drop_last=False):
        self.dataset = dataset
        self.batch_size = batch_size
        self.sampler = sampler
        self.shuffle = shuffle
        self.generator = generator
        self.drop_last = drop_last
        rgb_spec = rgb_spec or (rgb_train_transform if train else rgb_val_test_transform)
        thermal_spec = thermal_spec or (thermal_train_transform if train
                                        else thermal_val_test_transform)
        self.rgb = GpuPreprocessor(rgb_spec, device)
        self.thermal = GpuPreprocessor(thermal_spec, device)
        self.device = torch.device(device)
        self.num_threads = num_threads

    def _batches(self):
        if self.sampler is not None:
            order = list(self.sampler)
        elif self.shuffle:
            order = torch.randperm(len(self.dataset), generator=self.generator).tolist()
        else:
            order = list(range(len(self.dataset)))
        bs = self.batch_size
        for s in range(0, len(order), bs):
            b = order[s:s + bs]
            if len(b) < bs and self.drop_last:
                return
            yield b

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else len(self.dataset)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def _decode(self, pool, idx):
        pairs = [self.dataset.pairs[i] for i in idx]
        rgb = pool.map(decode_rgb, [p[0] for p in pairs])
        th = pool.map(decode_rgb, [p[1] for p in pairs])
        return list(rgb), list(th), [p[2] for p in pairs]

    def __iter__(self):
        # one thread orchestrates the next batch's decode on the pool (a pool task waiting on
        # its own pool could starve it)
        with ThreadPoolExecutor(self.num_threads) as pool, ThreadPoolExecutor(1) as ahead:
            pending = None
            for idx in self._batches():
                nxt = ahead.submit(self._decode, pool, idx)
                if pending is not None:
                    yield self._finish(*pending.result())
                pending = nxt
            if pending is not None:
                yield self._finish(*pending.result())

    def _finish(self, rgb, th, labels):
        rp, tp = [], []
        for _ in labels:
            rp.append(sample_params(self.rgb.spec, self.generator) if self.rgb.spec.random
                      else AugParams())
            tp.append(sample_params(self.thermal.spec, self.generator) if self.thermal.spec.random
                      else AugParams())
        y = torch.tensor(labels, dtype=torch.long).to(self.device, non_blocking=True)
        return self.rgb(rgb, rp), self.thermal(th, tp), y


class GpuImageLoader:
    """DataLoader replacement for the single-modality datasets (data.single_modality:
    RGBDataset, train_rgb_only.py:181-197; ThermalDataset): yields (images, labels) already on
    the GPU, fp32 NCHW, through the same decode-ahead threads and HIP transform kernels as
    GpuPairLoader.  `spec` defaults to the RGB train / val-test transform of
    train_rgb_only.py:102-118 (the fusion script's RGB transforms, identical); the thermal-only
    script's train transform adds a GaussianBlur this pipeline does not implement, so a thermal
    loader takes `thermal_val_test_transform` (or a spec without blur)."""

    def __init__(self, dataset, batch_size, sampler=None, shuffle=False, train=False,
                 spec=None, device="cuda", num_threads=4, generator=None, drop_last=False):
        self.dataset = dataset
        self.batch_size = batch_size
        self.sampler = sampler
        self.shuffle = shuffle
        self.generator = generator
        self.drop_last = drop_last
        spec = spec or (rgb_train_transform if train else rgb_val_test_transform)
        self.pre = GpuPreprocessor(spec, device)
        self.device = torch.device(device)
        self.num_threads = num_threads

    _batches = GpuPairLoader._batches
    __len__ = GpuPairLoader.__len__

    def _decode(self, pool, idx):
        imgs = pool.map(decode_rgb, [self.dataset.image_paths[i] for i in idx])
        return list(imgs), [self.dataset.labels[i] for i in idx]

    def __iter__(self):
        with ThreadPoolExecutor(self.num_threads) as pool, ThreadPoolExecutor(1) as ahead:
            pending = None
            for idx in self._batches():
                nxt = ahead.submit(self._decode, pool, idx)
                if pending is not None:
                    yield self._finish(*pending.result())
                pending = nxt
            if pending is not None:
                yield self._finish(*pending.result())

    def _finish(self, imgs, labels):
        params = [sample_params(self.pre.spec, self.generator) if self.pre.spec.random
                  else AugParams() for _ in labels]
        y = torch.tensor(labels, dtype=torch.long).to(self.device, non_blocking=True)
        return self.pre(imgs, params), y
