"""Paired dataset, weighted sampler, class weights and the SHA-256 split-leakage guard
against fixtures from the reference's own code (oracle/gen_data_golden.py ->
tests/golden/data_pairs.json), on the synthetic tree of oracle/data_inputs.py.
Reference: notebooks/train_multimodal_fusion.py:60-165, :224-268, :341-345."""
import json
import os
import random
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import data_inputs as DI  # noqa: E402

from data import multimodal as MM  # noqa: E402

with open(os.path.join(HERE, "golden", "data_pairs.json")) as f:
    GOLD = json.load(f)


def _build(tmp_path, leak):
    root = str(tmp_path)
    rgb, th = DI.build_tree(root, leak=leak)
    random.seed(42)
    dss = {s: MM.MultimodalDataset(rgb, th, s, verbose=False) for s in ("train", "val", "test")}
    return root, dss


@pytest.mark.parametrize("case", ["clean", "leak"])
def test_pairs_match_reference(tmp_path, case):
    root, dss = _build(tmp_path, case == "leak")
    g = GOLD[case]
    for s, ds in dss.items():
        got = [[os.path.relpath(str(r), root), os.path.relpath(str(t), root), y]
               for r, t, y in ds.pairs]
        assert got == g["splits"][s], s
    if g["leakage_raises"]:
        with pytest.raises(RuntimeError, match="leakage"):
            MM.check_multimodal_leakage(dss["train"], dss["val"], dss["test"], verbose=False)
    else:
        MM.check_multimodal_leakage(dss["train"], dss["val"], dss["test"], verbose=False)


def test_sha256_match_reference(tmp_path):
    root, _ = _build(tmp_path, False)
    g = GOLD["clean"]
    for rel, h in g["sha256"].items():
        assert MM.compute_sha256(os.path.join(root, rel)) == h, rel
    assert MM.compute_sha256(os.path.join(root, "does_not_exist.png")) is g["sha256_missing"]


def test_sampler_and_class_weights_match_reference(tmp_path):
    _, dss = _build(tmp_path, False)
    g = GOLD["clean"]
    labels = dss["train"].labels()
    assert MM.sample_weights(labels) == g["sample_weights"]
    torch.manual_seed(42)
    assert list(MM.make_weighted_sampler(dss["train"])) == g["sampler_draws"]
    cw = MM.class_weights(labels)
    assert cw.dtype == torch.float32
    assert cw.tolist() == g["class_weights"]


def test_class_weights_edge_cases():
    assert MM.class_weights([]).tolist() == [0.0, 0.0]
    assert MM.class_weights([1, 1]).tolist() == [0.0, 1.0]
    assert MM.sample_weights([1, 1, 0]) == [0.5, 0.5, 1.0]


def test_getitem_loads_rgb_and_applies_transforms(tmp_path):
    _, dss = _build(tmp_path, False)
    ds = dss["train"]
    seen = []
    ds.transform_rgb = lambda im: (seen.append(("rgb", im.mode)), torch.zeros(1))[1]
    ds.transform_thermal = lambda im: (seen.append(("th", im.mode)), torch.ones(1))[1]
    for i in range(len(ds)):
        r, t, y = ds[i]
        assert r.item() == 0 and t.item() == 1
        assert y.dtype == torch.long and y.item() == ds.pairs[i][2]
    assert seen.count(("rgb", "RGB")) == len(ds) and seen.count(("th", "RGB")) == len(ds)
    ds.transform_rgb = ds.transform_thermal = None
    r, t, _ = ds[0]
    assert r.mode == "RGB" and t.mode == "RGB"


def test_missing_split_dir_is_empty(tmp_path):
    random.seed(0)
    ds = MM.MultimodalDataset(str(tmp_path / "a"), str(tmp_path / "b"), "train", verbose=False)
    assert len(ds) == 0 and ds.labels() == []
