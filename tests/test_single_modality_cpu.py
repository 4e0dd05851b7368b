"""Single-modality datasets (C1 RGB-only, C2 thermal-only), split-hash leakage guards, sampler
and class weights against fixtures from the reference's own code (oracle/gen_single_golden.py
-> tests/golden/single_modality.json), on the synthetic tree of oracle/data_inputs.py.
Reference: notebooks/train_rgb_only.py:55-97, 117-193; notebooks/train_thermal_only.py:56-98,
117-181."""
import json
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import data_inputs as DI  # noqa: E402

from data import single_modality as SM  # noqa: E402

with open(os.path.join(HERE, "golden", "single_modality.json")) as f:
    GOLD = json.load(f)

CASES = {"clean": (False, False), "leak_rgb": (True, False), "leak_thermal": (False, True)}
CLS = {"rgb": (SM.RGBDataset, SM.check_split_hash_leakage),
       "thermal": (SM.ThermalDataset, SM.check_split_hash_leakage_modality)}


def _build(tmp_path, modality, case):
    root = str(tmp_path)
    rgb, th = DI.build_tree(root, *CASES[case])
    ds_cls, _ = CLS[modality]
    d = rgb if modality == "rgb" else th
    return root, {s: ds_cls(d, s, verbose=False) for s in ("train", "val", "test")}


@pytest.mark.parametrize("modality", ["rgb", "thermal"])
@pytest.mark.parametrize("case", list(CASES))
def test_walk_and_guard_match_reference(tmp_path, modality, case):
    root, dss = _build(tmp_path, modality, case)
    g = GOLD[f"{modality}/{case}"]
    for s, ds in dss.items():
        got = [[os.path.relpath(str(p), root), y] for p, y in zip(ds.image_paths, ds.labels)]
        assert got == g["splits"][s], s  # same items, same (rglob) order
    guard = CLS[modality][1]
    if g["leakage_raises"]:
        with pytest.raises(RuntimeError) as e:
            guard(dss["train"], dss["val"], dss["test"], verbose=False)
        assert str(e.value) == g["leakage_raises"]
    else:
        guard(dss["train"], dss["val"], dss["test"], verbose=False)


@pytest.mark.parametrize("modality", ["rgb", "thermal"])
def test_sampler_and_class_weights_match_reference(tmp_path, modality):
    _, dss = _build(tmp_path, modality, "clean")
    g = GOLD[f"{modality}/clean"]
    labels = dss["train"].labels
    assert SM.sample_weights(labels) == g["sample_weights"]
    torch.manual_seed(42)
    assert list(SM.make_weighted_sampler(dss["train"])) == g["sampler_draws"]
    if "class_weights" in g and g["class_weights"] is not None:
        assert SM.class_weights(labels).tolist() == g["class_weights"]


def test_getitem_and_missing_dirs(tmp_path):
    _, dss = _build(tmp_path, "rgb", "clean")
    ds = dss["train"]
    seen = []
    ds.transform = lambda im: (seen.append(im.mode), torch.zeros(1))[1]
    for i in range(len(ds)):
        x, y = ds[i]
        assert y.dtype == torch.long and y.item() == ds.labels[i]
    assert seen == ["RGB"] * len(ds)
    empty = SM.ThermalDataset(str(tmp_path / "nowhere"), "train", verbose=False)
    assert len(empty) == 0 and empty.labels == [] and empty.image_paths == []
