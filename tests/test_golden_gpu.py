"""The MI355X fusion head (dfu_hip Linear/ReLU/Dropout/concat, weighted CE, FusedAdamW — all
HIP kernels) against the golden fixtures made from the reference's own head code
(oracle/gen_golden.py).  The head runs in exact fp32 (dfu_gemm_f32), so tolerances are fp32
reassociation-level: rtol 1e-5 on logits/grads.  Parameters after AdamW: Adam normalises each
gradient element (m / (sqrt(v) + eps)), so where a gradient is ~0 its reassociation noise can
change that element's update by a visible fraction of one step (at most lr); parameters are
bounded at 1% of one step, atol = 0.01 * lr."""
import numpy as np
import pytest
import torch

import oracle.golden_inputs as GI
from golden_util import check_array, load

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _load_linears(lins, inp):
    with torch.no_grad():
        for lin, (W, b) in zip(lins, inp["weights"]):
            lin.weight.copy_(torch.from_numpy(W))
            lin.bias.copy_(torch.from_numpy(b))


def _product_head(inp):
    from dfu_hip import nn as hnn
    from models.fusion import GatedFusion, MLPFusion
    from models.models import MultimodalFusion
    kind, dims = inp["kind"], inp["dims"]
    if kind == "mlp2":
        r, t, h, c = dims
        m = MLPFusion(r, t, h, c)
    elif kind == "mlp3":
        r, t, c = dims
        m = MLPFusion(r, t, num_classes=c, hidden_dims=(512, 256), dropout=0.5)
    elif kind == "sigmoid":
        r, t, h = dims
        m = MultimodalFusion(r, t, h)
    else:
        m = GatedFusion(dims[0])
    lins = [l for l in m.modules() if isinstance(l, hnn.Linear)]
    _load_linears(lins, inp)
    return m.to(DEV), lins


@pytest.mark.parametrize("case", list(GI.HEAD_CASES))
def test_head_forward(case):
    fx = load(f"head_{case}.npz")
    inp = GI.head_inputs(case)
    m, _ = _product_head(inp)
    m.eval()
    rgb, th = torch.from_numpy(inp["rgb"]).to(DEV), torch.from_numpy(inp["th"]).to(DEV)
    with torch.no_grad():
        out = m(rgb, th)
    np.testing.assert_allclose(out.cpu().numpy(), fx["out0"], rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("case", ["mlp2_small", "mlp2_full", "mlp2_ragged", "mlp3_small"])
def test_head_train_steps(case):
    from dfu_hip.nn import CrossEntropyLoss
    from dfu_hip.optim import FusedAdamW
    fx = load(f"head_{case}.npz")
    inp = GI.head_inputs(case)
    m, lins = _product_head(inp)
    m.eval()  # dropout = identity, as the fixtures
    rgb, th = torch.from_numpy(inp["rgb"]).to(DEV), torch.from_numpy(inp["th"]).to(DEV)
    labels = torch.from_numpy(inp["labels"]).to(DEV)
    w = torch.from_numpy(fx["class_weights"]).to(DEV)
    crit = CrossEntropyLoss(weight=w)
    opt = FusedAdamW(m.parameters(), lr=GI.LR, weight_decay=GI.WEIGHT_DECAY)
    for s in range(GI.STEPS):
        opt.zero_grad()
        loss = crit(m(rgb, th), labels)
        loss.backward()
        if s == 0:
            for i, lin in enumerate(lins):
                check_array(fx, f"grad{i}w", lin.weight.grad.cpu().numpy(), 1e-5, 1e-7)
                check_array(fx, f"grad{i}b", lin.bias.grad.cpu().numpy(), 1e-5, 1e-7)
        opt.step()
        assert abs(loss.item() - float(fx[f"loss{s}"])) < 1e-5, (s, loss.item(), fx[f"loss{s}"])
    for i, lin in enumerate(lins):
        check_array(fx, f"param{i}w", lin.weight.detach().cpu().numpy(), 1e-6, 0.01 * GI.LR)
        check_array(fx, f"param{i}b", lin.bias.detach().cpu().numpy(), 1e-6, 0.01 * GI.LR)
    with torch.no_grad():
        np.testing.assert_allclose(m(rgb, th).cpu().numpy(), fx["out_final"], rtol=1e-5, atol=2e-6)
