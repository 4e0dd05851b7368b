"""ORACLE — test infrastructure only.  Deterministic inputs for the golden fixtures in
tests/golden/: shared by oracle/gen_golden.py (which runs the reference's own code on them, in
the build container) and by the tests (which regenerate the same inputs on any machine and
compare against the stored outputs).  numpy's PCG64 stream is version-stable, so only outputs
need committing.

Each head case is one fusion-head training iteration of the reference loop
(notebooks/train_multimodal_fusion.py:374-380): forward, weighted CE (:341-346), backward,
AdamW(lr=1e-4, weight_decay=1e-4) (:347), repeated STEPS times on the same batch, in eval mode
(dropout = identity, SURVEY.md §8(d) "dropout forced to identity").
"""
import numpy as np

STEPS = 3
LR = 1e-4
WEIGHT_DECAY = 1e-4

# name -> (kind, dims, batch, seed)
#   mlp2:    MLPFusion, grad_cam_visualization.py:289-302   dims = (rgb, thermal, hidden, classes)
#   mlp3:    train-script head, train_multimodal_fusion.py:305-313  dims = (rgb, thermal, classes)
#   sigmoid: models/models.py:24-40 MultimodalFusion       dims = (rgb, thermal, hidden)
#   gated:   models/fusion.py:4-17 GatedFusion              dims = (feat,)
HEAD_CASES = {
    "mlp2_small": ("mlp2", (64, 32, 16, 2), 8, 1),
    "mlp2_full": ("mlp2", (2048, 768, 512, 2), 64, 2),
    "mlp2_ragged": ("mlp2", (40, 24, 24, 2), 5, 3),
    "mlp3_small": ("mlp3", (64, 32, 2), 8, 4),
    "sigmoid_small": ("sigmoid", (64, 32, 16), 8, 5),
    "gated_small": ("gated", (32,), 6, 6),
}

# label vectors for the class-weight formula (:341-345), incl. an absent class
WEIGHT_LABELS = {
    "balanced": [0, 1, 0, 1, 1, 0],
    "skewed": [1, 1, 1, 0, 1, 1, 1, 1],
    "absent": [1, 1, 1],
    "empty": [],
}


def layer_dims(kind, dims):
    """Ordered (out, in) shapes of the Linear layers of a head case."""
    if kind == "mlp2":
        r, t, h, c = dims
        return [(h, r + t), (c, h)]
    if kind == "mlp3":
        r, t, c = dims
        return [(512, r + t), (256, 512), (c, 256)]
    if kind == "sigmoid":
        r, t, h = dims
        return [(h, r + t), (1, h)]
    if kind == "gated":
        (f,) = dims
        return [(f, 2 * f), (f, f)]
    raise ValueError(kind)


def head_inputs(name):
    """-> dict(weights=[(W, b), ...] float32, rgb (B,R), th (B,T), labels (B,) int64)."""
    kind, dims, B, seed = HEAD_CASES[name]
    rng = np.random.default_rng(seed)
    weights = []
    for out_f, in_f in layer_dims(kind, dims):
        bound = 1.0 / np.sqrt(in_f)
        W = rng.uniform(-bound, bound, size=(out_f, in_f)).astype(np.float32)
        b = rng.uniform(-bound, bound, size=(out_f,)).astype(np.float32)
        weights.append((W, b))
    if kind == "gated":
        R = T = dims[0]
    else:
        R, T = dims[0], dims[1]
    # encoder features are post-ReLU pooled (rgb, >= 0) and LayerNorm'd tokens (thermal)
    rgb = np.abs(rng.standard_normal((B, R))).astype(np.float32)
    th = rng.standard_normal((B, T)).astype(np.float32)
    labels = rng.integers(0, 2, size=(B,)).astype(np.int64)
    return dict(kind=kind, dims=dims, weights=weights, rgb=rgb, th=th, labels=labels)


def summarize(a):
    """Size-independent digest of a large array: row sums, column sums, 64 fixed samples."""
    a = np.asarray(a, dtype=np.float64)
    if a.ndim == 1:
        a = a[:, None]
    flat = a.reshape(-1)
    idx = np.linspace(0, flat.size - 1, num=min(64, flat.size)).astype(np.int64)
    return dict(rows=a.sum(1), cols=a.sum(0), samples=flat[idx], idx=idx)
