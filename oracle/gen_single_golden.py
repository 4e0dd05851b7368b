"""ORACLE — test infrastructure only.  Generates tests/golden/single_modality.json by running the
REFERENCE's own single-modality dataset, leakage-guard, sampler and class-weight code on the
synthetic tree of oracle/data_inputs.py, in this build container (the reference is absent on
the GPU box).

Executed from /root/reference (extracted by `ast`, run with only the names it uses in scope;
the scripts train at import time, so they are not imported whole):
  * notebooks/train_rgb_only.py      RGBDataset :55-97, compute_sha256 / check_split_hash_leakage
                                     :117-167, class-weight statements :170-176, sampler-weight
                                     statements inside `if len(train_labels) > 0:` :184-190
  * notebooks/train_thermal_only.py  ThermalDataset :56-98, check_split_hash_leakage_modality
                                     :128-168, sampler-weight statements :173-179
Cases: a clean tree, an RGB train->val duplicate, a thermal val->test duplicate (nested, upper-
case suffix).  The walk order is Path.rglob's on this container's /tmp filesystem (the tests
rebuild the tree under pytest's tmp_path, on the same filesystem).

Usage:  python oracle/gen_single_golden.py     (writes tests/golden/single_modality.json)
"""
import ast
import hashlib
import json
import os
import sys
import tempfile
from collections import Counter
from pathlib import Path

import torch
from PIL import Image
from torch.utils.data import Dataset, WeightedRandomSampler

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import data_inputs as DI  # noqa: E402

REF = "/root/reference/notebooks"
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden", "single_modality.json")
SCRIPTS = {"rgb": ("train_rgb_only.py", "RGBDataset", "check_split_hash_leakage"),
           "thermal": ("train_thermal_only.py", "ThermalDataset",
                       "check_split_hash_leakage_modality")}


def _tree(script):
    path = os.path.join(REF, script)
    with open(path) as f:
        return ast.parse(f.read(), path), path


def extract(script, names):
    tree, path = _tree(script)
    ns = {"torch": torch, "Path": Path, "Dataset": Dataset, "Image": Image, "hashlib": hashlib,
          "Counter": Counter}
    body = [n for n in tree.body if isinstance(n, (ast.ClassDef, ast.FunctionDef))
            and n.name in names]
    assert len(body) == len(names), [n.name for n in body]
    exec(compile(ast.Module(body=body, type_ignores=[]), path, "exec"), ns)
    return ns


def sampler_stmts(script):
    """The sample-weight assignments of the `if len(train_labels) > 0:` block."""
    tree, path = _tree(script)
    for n in tree.body:
        if (isinstance(n, ast.If) and "train_labels" in ast.unparse(n.test)
                and "sample_weights" in ast.unparse(n)):
            body = [s for s in n.body if isinstance(s, ast.Assign)
                    and s.targets[0].id in ("counts", "class_counts", "sample_weights")]
            assert len(body) == 3
            return compile(ast.Module(body=body, type_ignores=[]), path, "exec")
    raise AssertionError("sampler block not found")


def class_weight_stmts(script):
    tree, path = _tree(script)
    want = {"train_counts", "class_counts", "total", "class_weights"}
    body = [n for n in tree.body if isinstance(n, ast.Assign)
            and any(isinstance(t, ast.Name) and t.id in want for t in n.targets)]
    body = [n for n in body if "sample_weights" not in ast.unparse(n)]
    return compile(ast.Module(body=body, type_ignores=[]), path, "exec")


def run_reference(root, modality, leak, leak_thermal):
    script, cls, guard = SCRIPTS[modality]
    ns = extract(script, [cls, "compute_sha256", guard])
    rgb_dir, th_dir = DI.build_tree(root, leak=leak, leak_thermal=leak_thermal)
    data_dir = rgb_dir if modality == "rgb" else th_dir
    dss = {s: ns[cls](data_dir, s) for s in ("train", "val", "test")}
    rel = lambda p: os.path.relpath(str(p), root)  # noqa: E731
    out = {"splits": {s: [[rel(p), y] for p, y in zip(ds.image_paths, ds.labels)]
                      for s, ds in dss.items()}}
    try:
        ns[guard](dss["train"], dss["val"], dss["test"])
        out["leakage_raises"] = None
    except RuntimeError as e:
        out["leakage_raises"] = str(e)
    g = {"Counter": Counter, "torch": torch, "train_labels": dss["train"].labels,
         "WeightedRandomSampler": WeightedRandomSampler}
    exec(sampler_stmts(script), g)
    out["sample_weights"] = g["sample_weights"]
    torch.manual_seed(42)
    out["sampler_draws"] = list(WeightedRandomSampler(g["sample_weights"],
                                                      num_samples=len(g["sample_weights"]),
                                                      replacement=True))
    if modality == "rgb":
        g2 = {"Counter": Counter, "torch": torch, "train_dataset": dss["train"]}
        exec(class_weight_stmts(script), g2)
        out["class_weights"] = g2["class_weights"].tolist()
    return out


def main():
    res = {}
    for modality in ("rgb", "thermal"):
        for case, (leak, leak_th) in (("clean", (False, False)), ("leak_rgb", (True, False)),
                                      ("leak_thermal", (False, True))):
            with tempfile.TemporaryDirectory() as root:
                res[f"{modality}/{case}"] = run_reference(root, modality, leak, leak_th)
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
