"""ORACLE — test infrastructure only.  Generates tests/golden/data_pairs.json by running the
REFERENCE's own dataset, leakage and sampler code on the synthetic tree of
oracle/data_inputs.py, in this build container (the reference is absent on the GPU box).

Executed from /root/reference (extracted by `ast`, run with only the names it uses in scope;
the script is not imported as a whole because it trains at import time):
  * class MultimodalDataset           notebooks/train_multimodal_fusion.py:60-165
  * compute_sha256, check_multimodal_leakage                             :224-257
  * the sampler-weight statements inside `if len(train_labels) > 0:`     :261-265
  * the class-weight statements                                          :341-345
The splits are built in the script's order (train, val, test) after random.seed(42) (:40-42);
the sampler's draws are WeightedRandomSampler's under torch.manual_seed(42).

Usage:  python oracle/gen_data_golden.py     (writes tests/golden/data_pairs.json)
"""
import ast
import hashlib
import json
import os
import random
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

REF = "/root/reference"
REL = "notebooks/train_multimodal_fusion.py"
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden", "data_pairs.json")


def _tree():
    path = os.path.join(REF, REL)
    with open(path) as f:
        return ast.parse(f.read(), path), path


def extract(names):
    tree, path = _tree()
    ns = {"torch": torch, "Path": Path, "Dataset": Dataset, "Image": Image, "random": random,
          "hashlib": hashlib, "Counter": Counter}
    body = [n for n in tree.body if isinstance(n, (ast.ClassDef, ast.FunctionDef))
            and n.name in names]
    assert len(body) == len(names), [n.name for n in body]
    exec(compile(ast.Module(body=body, type_ignores=[]), path, "exec"), ns)
    return ns


def extract_weight_stmts():
    """(sampler-weight statements, class-weight statements) as code objects."""
    tree, path = _tree()
    samp = None
    for n in tree.body:
        if (isinstance(n, ast.If) and "train_labels" in ast.unparse(n.test)
                and "sample_weights" in ast.unparse(n)):
            samp = [s for s in n.body if isinstance(s, ast.Assign)
                    and s.targets[0].id in ("counts", "class_counts", "sample_weights")]
    assert samp and len(samp) == 3
    want = {"train_counts", "class_counts", "total", "class_weights"}
    cw = [n for n in tree.body if isinstance(n, ast.Assign)
          and any(isinstance(t, ast.Name) and t.id in want for t in n.targets)]
    assert len(cw) == 4
    mk = lambda b: compile(ast.Module(body=b, type_ignores=[]), path, "exec")  # noqa: E731
    return mk(samp), mk(cw)


def run_reference(root, leak):
    ns = extract(["MultimodalDataset", "compute_sha256", "check_multimodal_leakage"])
    rgb_dir, th_dir = DI.build_tree(root, leak=leak)
    random.seed(42)
    dss = {s: ns["MultimodalDataset"](rgb_dir, th_dir, s) for s in ("train", "val", "test")}
    rel = lambda p: os.path.relpath(str(p), root)  # noqa: E731
    out = {"splits": {s: [[rel(r), rel(t), y] for r, t, y in ds.pairs] for s, ds in dss.items()}}
    try:
        ns["check_multimodal_leakage"](dss["train"], dss["val"], dss["test"])
        out["leakage_raises"] = False
    except RuntimeError:
        out["leakage_raises"] = True
    out["sha256"] = {rel(p): ns["compute_sha256"](p)
                     for ds in dss.values() for pr in ds.pairs for p in pr[:2]}
    out["sha256_missing"] = ns["compute_sha256"](os.path.join(root, "does_not_exist.png"))
    samp, cw = extract_weight_stmts()
    train_labels = [label for _, _, label in dss["train"].pairs]
    g = {"Counter": Counter, "torch": torch, "train_labels": train_labels}
    exec(samp, g)
    out["sample_weights"] = g["sample_weights"]
    torch.manual_seed(42)
    out["sampler_draws"] = list(WeightedRandomSampler(g["sample_weights"],
                                                      num_samples=len(g["sample_weights"]),
                                                      replacement=True))
    exec(cw, g)
    out["class_weights"] = g["class_weights"].tolist()
    return out


def main():
    res = {}
    for leak in (False, True):
        with tempfile.TemporaryDirectory() as root:
            res["leak" if leak else "clean"] = run_reference(root, leak)
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
