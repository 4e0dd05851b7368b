"""ORACLE — test infrastructure only.  Generates the golden fixtures in tests/golden/ by running
the REFERENCE's own pure-torch code in this build container (the reference is not present on
the GPU box; only the .npz outputs travel).

What is executed from /root/reference (classes and statements extracted by `ast`, executed with
nothing but torch / torch.nn / collections.Counter in scope — no reference module is imported
as a whole, because the notebooks train at import time and the encoders need torchvision/timm,
which are absent):
  * MLPFusion                 notebooks/grad_cam_visualization.py:289-302
  * the 3-layer fusion head   notebooks/train_multimodal_fusion.py:305-313 (the `self.fusion =
                              nn.Sequential(...)` expression inside MultimodalFusionModel)
  * MultimodalFusion          models/models.py:24-40 (sigmoid head)
  * GatedFusion               models/fusion.py:4-17
  * class-weight statements   notebooks/train_multimodal_fusion.py:341-345
The loss and optimizer are the ones the reference instantiates (:346-347):
nn.CrossEntropyLoss(weight=class_weights) and torch.optim.AdamW(lr=1e-4, weight_decay=1e-4).

Usage:  python oracle/gen_golden.py        (writes tests/golden/*.npz; deterministic)
"""
import ast
import collections
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import golden_inputs as GI  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def _src(rel):
    path = os.path.join(REF, rel)
    with open(path) as f:
        return f.read(), path


def extract_class(rel, name):
    src, path = _src(rel)
    tree = ast.parse(src, path)
    for node in tree.body:
        if isinstance(node, ast.ClassDef) and node.name == name:
            ns = {"torch": torch, "nn": nn}
            exec(compile(ast.Module(body=[node], type_ignores=[]), path, "exec"), ns)
            return ns[name], node.lineno
    raise LookupError(f"{name} not found in {rel}")


def extract_fusion_expr(rel, cls):
    """The value expression of `self.fusion = ...` inside class `cls`."""
    src, path = _src(rel)
    tree = ast.parse(src, path)
    for node in ast.walk(tree):
        if isinstance(node, ast.ClassDef) and node.name == cls:
            for sub in ast.walk(node):
                if (isinstance(sub, ast.Assign) and len(sub.targets) == 1
                        and isinstance(sub.targets[0], ast.Attribute)
                        and sub.targets[0].attr == "fusion"):
                    return compile(ast.Expression(body=sub.value), path, "eval"), sub.lineno
    raise LookupError(f"self.fusion assignment not found in {rel}:{cls}")


def extract_class_weight_stmts(rel):
    """Module-level statements that define train_counts .. class_weights."""
    src, path = _src(rel)
    tree = ast.parse(src, path)
    want = {"train_counts", "class_counts", "total", "class_weights"}
    body = [n for n in tree.body if isinstance(n, ast.Assign)
            and any(isinstance(t, ast.Name) and t.id in want for t in n.targets)]
    assert len(body) == 4, [ast.dump(b)[:60] for b in body]
    return compile(ast.Module(body=body, type_ignores=[]), path, "exec"), body[0].lineno


def build_module(name, inp):
    kind, dims = inp["kind"], inp["dims"]
    if kind == "mlp2":
        cls, line = extract_class("notebooks/grad_cam_visualization.py", "MLPFusion")
        r, t, h, c = dims
        m = cls(rgb_feat_dim=r, thermal_feat_dim=t, hidden_dim=h, num_classes=c)
        linears = [m.classifier[0], m.classifier[3]]
    elif kind == "mlp3":
        expr, line = extract_fusion_expr("notebooks/train_multimodal_fusion.py", "MultimodalFusionModel")
        r, t, c = dims
        seq = eval(expr, {"nn": nn, "torch": torch, "rgb_feat_dim": r, "thermal_feat_dim": t,
                          "dropout": 0.5, "num_classes": c})

        class Head(nn.Module):  # the reference forward (:318-326): cat then self.fusion
            def __init__(self):
                super().__init__()
                self.fusion = seq

            def forward(self, a, b):
                return self.fusion(torch.cat([a, b], dim=1))
        m = Head()
        linears = [seq[0], seq[3], seq[6]]
    elif kind == "sigmoid":
        cls, line = extract_class("models/models.py", "MultimodalFusion")
        r, t, h = dims
        m = cls(rgb_dim=r, thermal_dim=t, hidden_dim=h)
        linears = [m.classifier[0], m.classifier[3]]
    elif kind == "gated":
        cls, line = extract_class("models/fusion.py", "GatedFusion")
        m = cls(feat_dim=dims[0])
        linears = [m.gate[0], m.gate[2]]
    else:
        raise ValueError(kind)
    with torch.no_grad():
        for lin, (W, b) in zip(linears, inp["weights"]):
            assert tuple(lin.weight.shape) == W.shape, (name, lin.weight.shape, W.shape)
            lin.weight.copy_(torch.from_numpy(W))
            lin.bias.copy_(torch.from_numpy(b))
    return m, linears


def class_weights_ref(labels):
    code, _ = extract_class_weight_stmts("notebooks/train_multimodal_fusion.py")
    ns = {"Counter": collections.Counter, "torch": torch, "train_labels": list(labels)}
    exec(code, ns)
    return ns["class_weights"].numpy()


def run_head_case(name):
    inp = GI.head_inputs(name)
    m, linears = build_module(name, inp)
    m.eval()  # dropout = identity
    rgb = torch.from_numpy(inp["rgb"])
    th = torch.from_numpy(inp["th"])
    labels = torch.from_numpy(inp["labels"])
    out = {}
    with torch.no_grad():
        out["out0"] = m(rgb, th).numpy()
    if inp["kind"] in ("mlp2", "mlp3"):
        w = torch.from_numpy(class_weights_ref(inp["labels"].tolist()))
        crit = nn.CrossEntropyLoss(weight=w)
        out["class_weights"] = w.numpy()
        opt = torch.optim.AdamW(m.parameters(), lr=GI.LR, weight_decay=GI.WEIGHT_DECAY)
        for s in range(GI.STEPS):
            opt.zero_grad()
            logits = m(rgb, th)
            loss = crit(logits, labels)
            loss.backward()
            out[f"loss{s}"] = np.float64(loss.item())
            if s == 0:
                for i, lin in enumerate(linears):
                    for pn, p in (("w", lin.weight), ("b", lin.bias)):
                        g = p.grad.numpy()
                        if g.size <= 65536:
                            out[f"grad{i}{pn}"] = g.copy()
                        else:
                            for k, v in GI.summarize(g).items():
                                out[f"grad{i}{pn}_{k}"] = v
            opt.step()
        with torch.no_grad():
            out["out_final"] = m(rgb, th).numpy()
        for i, lin in enumerate(linears):
            for pn, p in (("w", lin.weight), ("b", lin.bias)):
                a = p.detach().numpy()
                if a.size <= 65536:
                    out[f"param{i}{pn}"] = a.copy()
                else:
                    for k, v in GI.summarize(a).items():
                        out[f"param{i}{pn}_{k}"] = v
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(1)  # deterministic reduction order on the CPU
    for name in GI.HEAD_CASES:
        res = run_head_case(name)
        np.savez_compressed(os.path.join(OUT, f"head_{name}.npz"), **res)
        print(f"head_{name}.npz: {len(res)} arrays")
    cw = {k: class_weights_ref(v) for k, v in GI.WEIGHT_LABELS.items()}
    np.savez_compressed(os.path.join(OUT, "class_weights.npz"), **cw)
    print("class_weights.npz:", {k: v.tolist() for k, v in cw.items()})


if __name__ == "__main__":
    main()
