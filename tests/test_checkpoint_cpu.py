"""Checkpoint compatibility, CPU only: the reference's checkpoint dict,
its flexible loader semantics (backbone.* remap, shape-mismatch skips), the key fixer, and a
FusedAdamW state dict that interchanges with torch.optim.AdamW."""
import torch
import torch.nn as nn

from models import checkpoint as ck


class _Head(nn.Module):
    def __init__(self, attr, classes=2):
        super().__init__()
        setattr(self, attr, nn.Sequential(nn.Linear(8, 4), nn.ReLU(), nn.Linear(4, 4)))
        self.classifier = nn.Sequential(nn.Linear(4, classes))


def test_backbone_prefix_remap_and_head_skip(tmp_path):
    src = _Head("backbone_tmp")
    sd = {k.replace("backbone_tmp.", "backbone."): v for k, v in src.state_dict().items()}
    sd["classifier.0.weight"] = torch.randn(3, 4)  # a 3-class head: shape mismatch -> skipped
    sd["classifier.0.bias"] = torch.randn(3)
    path = tmp_path / "best_model.pt"
    torch.save({"epoch": 3, "model_state_dict": sd}, path)
    for attr in ("resnet", "vit"):
        m = _Head(attr)
        rep = ck.load_checkpoint_flexible(m, path, device="cpu", verbose=False)
        assert rep and len(rep.loaded) == 4 and len(rep.skipped) == 2
        for k, v in src.state_dict().items():
            if k.startswith("backbone_tmp."):
                assert torch.equal(m.state_dict()[k.replace("backbone_tmp.", attr + ".")], v)
    torch.save({"epoch": 0}, path)
    assert ck.load_checkpoint_flexible(_Head("vit"), path, device="cpu", verbose=False) is False


def test_fix_checkpoint_keys(tmp_path):
    path = tmp_path / "c.pt"
    torch.save({"model_state_dict": {"backbone.conv1.weight": torch.ones(2)}, "epoch": 1}, path)
    out = ck.fix_checkpoint_keys(path)
    assert list(out["model_state_dict"]) == ["resnet.conv1.weight"]
    assert list(ck.load_checkpoint(path)["model_state_dict"]) == ["resnet.conv1.weight"]


def test_fused_adamw_state_dict_interchanges_with_torch_adamw():
    from dfu_hip.optim import FusedAdamW
    torch.manual_seed(0)
    ref = nn.Sequential(nn.Linear(6, 5), nn.ReLU(), nn.Linear(5, 3))
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-4, weight_decay=1e-4)
    for _ in range(3):
        opt.zero_grad()
        ref(torch.randn(4, 6)).sum().backward()
        opt.step()
    sd = opt.state_dict()
    mine = nn.Sequential(nn.Linear(6, 5), nn.ReLU(), nn.Linear(5, 3))
    mine.load_state_dict(ref.state_dict())
    fopt = FusedAdamW(mine.parameters(), lr=1e-4, weight_decay=1e-4)
    fopt.load_state_dict(sd)
    assert int(fopt.step_dev) == 3
    out = fopt.state_dict()
    assert set(out["state"]) == set(sd["state"])
    for i, st in sd["state"].items():
        assert torch.equal(out["state"][i]["exp_avg"], st["exp_avg"])
        assert torch.equal(out["state"][i]["exp_avg_sq"], st["exp_avg_sq"])
        assert float(out["state"][i]["step"]) == float(st["step"])
    # and back into torch's AdamW
    opt2 = torch.optim.AdamW(ref.parameters(), lr=1e-4, weight_decay=1e-4)
    opt2.load_state_dict(out)
    for i, st in opt2.state_dict()["state"].items():
        assert torch.equal(st["exp_avg"], sd["state"][i]["exp_avg"])


def test_fusion_checkpoint_round_trip_with_reference_layout(tmp_path):
    """The MI355X model's checkpoint loads strictly into the CPU restatement of the reference
    model (torchvision/timm keys) and back."""
    from models.fusion import MultimodalFusionModel
    from oracle import torch_ref as R
    torch.manual_seed(1)
    hip = MultimodalFusionModel(num_classes=2)
    path = tmp_path / "best_model.pt"
    torch.save({"epoch": 1, "model_state_dict": hip.state_dict(), "val_f1": 0.5,
                "history": {"val_f1": [0.5]}}, path)
    ckpt = ck.load_checkpoint(path)
    assert set(ckpt) >= {"epoch", "model_state_dict", "val_f1", "history"}
    ref = R.MultimodalFusionModel(num_classes=2)
    ref.load_state_dict(ckpt["model_state_dict"], strict=True)
    back = MultimodalFusionModel(num_classes=2)
    rep = ck.load_checkpoint_flexible(back, path, device="cpu", verbose=False)
    assert len(rep.loaded) == len(hip.state_dict()) and not rep.skipped
    for k, v in hip.state_dict().items():
        assert torch.equal(back.state_dict()[k], v)


def test_reference_numpy_metrics_load_weights_only(tmp_path):
    """The reference saves sklearn results (numpy.float64) in val_f1 / history
    (train_multimodal_fusion.py:428-439); all three loaders read them with weights_only."""
    import numpy as np
    path = tmp_path / "best_model.pt"
    hist = {"train_loss": [0.7, 0.6], "train_acc": [np.float64(0.5), np.float64(0.625)],
            "train_f1": [np.float64(0.4), np.float64(0.5)], "val_f1": [np.float64(0.55)],
            "n": [np.int64(3)]}
    sd = {"backbone.conv1.weight": torch.ones(2), "fc.weight": torch.zeros(1)}
    torch.save({"epoch": 4, "model_state_dict": sd, "optimizer_state_dict": {},
                "val_f1": np.float64(0.7142857), "history": hist}, path)
    c = ck.load_checkpoint(path)
    assert isinstance(c["val_f1"], np.float64) and c["val_f1"] == np.float64(0.7142857)
    assert c["history"]["train_acc"][1] == 0.625 and c["history"]["n"][0] == 3
    m = _Head("resnet")
    assert ck.load_checkpoint_flexible(m, path, device="cpu", verbose=False)
    assert ck.fix_checkpoint_keys(path)["val_f1"] == np.float64(0.7142857)


def test_multimodal_vit_backbone_remap(tmp_path):
    """extended_metrics.py:803-813: backbone.* -> resnet.*, vit_backbone.* -> vit.*."""
    sd = {"backbone.conv1.weight": torch.ones(1), "vit_backbone.cls_token": torch.zeros(1),
          "fusion.0.weight": torch.ones(2)}
    assert ck.remap_multimodal_keys(sd) == {"resnet.conv1.weight": sd["backbone.conv1.weight"],
                                            "vit.cls_token": sd["vit_backbone.cls_token"],
                                            "fusion.0.weight": sd["fusion.0.weight"]}

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.resnet = nn.Linear(3, 2)
            self.vit = nn.Linear(2, 2)
    src = M()
    path = tmp_path / "mm.pt"
    torch.save({"model_state_dict": {("backbone." + k[7:] if k.startswith("resnet.")
                                      else "vit_backbone." + k[4:]): v
                                     for k, v in src.state_dict().items()}}, path)
    dst = M()
    missing, unexpected = ck.load_multimodal_checkpoint(dst, path, device="cpu")
    assert not missing and not unexpected
    for k, v in src.state_dict().items():
        assert torch.equal(dst.state_dict()[k], v)
