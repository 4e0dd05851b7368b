"""ORACLE — test infrastructure only.  Deterministic synthetic RGB/thermal directory tree for
the dataset / sampler / leakage fixtures (oracle/gen_data_golden.py, tests/test_data_cpu.py).

The tree exercises what the reference's MultimodalDataset scan and pairing depend on
(notebooks/train_multimodal_fusion.py:60-142): unequal modality counts per class (cyclic
pairing), nested sub-directories (rglob), mixed-case suffixes of every accepted kind, files
that must be skipped, and a split with one class missing in one modality.
"""
import os

import numpy as np

# split -> modality -> class -> list of relative file names (under <modality>/<split>/<class>/)
LAYOUT = {
    "train": {
        "rgb": {"healthy": ["h%02d.png" % i for i in range(7)] + ["sub/x1.JPG", "sub/deep/x2.jpeg"],
                "ulcer": ["u%02d.png" % i for i in range(4)] + ["u_b.bmp"]},
        "thermal": {"healthy": ["t%02d.png" % i for i in range(3)] + ["t_t.tif"],
                    "ulcer": ["tu%02d.png" % i for i in range(11)] + ["tu_x.TIFF"]},
    },
    "val": {
        "rgb": {"healthy": ["vh%d.png" % i for i in range(3)],
                "ulcer": ["vu%d.png" % i for i in range(2)]},
        "thermal": {"healthy": ["vth%d.png" % i for i in range(2)],
                    "ulcer": ["vtu%d.png" % i for i in range(5)]},
    },
    "test": {
        "rgb": {"healthy": ["eh%d.png" % i for i in range(2)],
                "ulcer": ["eu%d.png" % i for i in range(3)]},
        "thermal": {"healthy": ["eth%d.png" % i for i in range(4)],
                    "ulcer": []},           # no thermal ulcer: the class is skipped
    },
}
# files every split gets that the scan must ignore
IGNORED = ["notes.txt", "thumbs.db", "img.gif"]


def _write_image(path, seed):
    from PIL import Image
    rng = np.random.default_rng(seed)
    arr = rng.integers(0, 256, size=(8 + seed % 5, 6 + seed % 3, 3), dtype=np.uint8)
    ext = os.path.splitext(path)[1].lower()
    fmt = {".png": "PNG", ".jpg": "PNG", ".jpeg": "PNG", ".bmp": "BMP",
           ".tif": "TIFF", ".tiff": "TIFF"}[ext]
    # JPEG-suffixed files are written as PNG bytes: PIL sniffs content, and lossless bytes keep
    # the tree (and its SHA-256s) identical across PIL versions.
    Image.fromarray(arr).save(path, format=fmt)


def build_tree(root, leak=False, leak_thermal=False):
    """Create the tree under root/{rgb,thermal}/<split>/<class>/.  Every image has distinct
    content; with leak=True one train RGB image is copied byte-for-byte into val (renamed), with
    leak_thermal=True one val thermal image into test.  Returns (rgb_dir, thermal_dir)."""
    seed = 1
    for split, mods in LAYOUT.items():
        for mod, classes in mods.items():
            for cls, names in classes.items():
                d = os.path.join(root, mod, split, cls)
                os.makedirs(d, exist_ok=True)
                for n in names:
                    p = os.path.join(d, n)
                    os.makedirs(os.path.dirname(p), exist_ok=True)
                    _write_image(p, seed)
                    seed += 1
                for n in IGNORED:
                    with open(os.path.join(d, n), "wb") as f:
                        f.write(b"not an image %d" % seed)
                    seed += 1
    if leak:
        src = os.path.join(root, "rgb", "train", "ulcer", "u02.png")
        dst = os.path.join(root, "rgb", "val", "healthy", "copied.png")
        with open(src, "rb") as f, open(dst, "wb") as g:
            g.write(f.read())
    if leak_thermal:
        src = os.path.join(root, "thermal", "val", "ulcer", "vtu3.png")
        dst = os.path.join(root, "thermal", "test", "healthy", "dup", "again.PNG")
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        with open(src, "rb") as f, open(dst, "wb") as g:
            g.write(f.read())
    return os.path.join(root, "rgb"), os.path.join(root, "thermal")
