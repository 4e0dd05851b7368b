"""Per-stage forward precision of the HIP encoders.

A stage is the ResNet stem ("resnet.stem"), a ResNet Bottleneck ("resnet.layer<i>.<j>") or a
ViT Block ("vit.blocks.<k>").  Its forward runs in one of functional.STAGE_MODES: "bf16" (bf16
operands and activations), "bf16x3" (fp32-accurate split-bf16 operands) or, for a ViT Block,
"fp16" (fp16 operands, fp32 accumulation and residual stream).  The backward is bf16 in every
mode.

  * functional.precision("parity") -- the headline mode and the library default -- runs each
    stage at its ``dfu_parity_precision``: ResNet stages bf16x3; ViT Blocks fp16 when a fusion
    model marks the ViT as its feature extractor (mark_feature_extractor), Blocks 0-8 bf16x3
    and 9-11 fp16 otherwise (models/vit.py _parity_policy).  The fusion assignment is the
    cheapest the per-stage study found to keep the fusion logits within half of
    north_star's 1e-3 of the fp32 oracle on every seed (profiles/r16a_precision_grid.json,
    profiles/r16b_precision_study.json, profiles/r19_precision_study.json,
    tools/precision_policy_study.py): the random-init ResNet amplifies rounding ~30x more than
    the ViT, so its forward needs ~2^-17 products while the ViT's holds the bar with fp16's
    2^-11 -- and bf16 anywhere, even in the last ResNet block or ViT Block alone, costs 4-7e-4.
  * functional.precision("mixed") runs each stage at its ``dfu_precision`` attribute (bf16x3
    where unset), which apply_policy sets -- the study's tool.
"""


def encoders(model):
    """(resnet or None, vit or None) inside a fusion / single-modality model or an encoder."""
    from .resnet import ResNet
    from .vit import VisionTransformer
    r = v = None
    for m in model.modules():
        if r is None and isinstance(m, ResNet):
            r = m
        elif v is None and isinstance(m, VisionTransformer):
            v = m
    return r, v


def stages(model):
    """Ordered {name: module} of every stage a policy can name."""
    r, v = encoders(model)
    out = {}
    if r is not None:
        out["resnet.stem"] = r
        for i, layer in enumerate((r.layer1, r.layer2, r.layer3, r.layer4), 1):
            for j, blk in enumerate(layer):
                out[f"resnet.layer{i}.{j}"] = blk
    if v is not None:
        for k, blk in enumerate(v.blocks):
            out[f"vit.blocks.{k}"] = blk
    return out


def apply_policy(model, policy):
    """Set every stage's ``dfu_precision`` (effective under functional.precision("mixed")):
    `policy` maps stage names to modes (every other stage bf16x3), or is an iterable of stage
    names that run bf16.  Unknown names or modes raise; returns the model."""
    from dfu_hip.functional import STAGE_MODES
    st = stages(model)
    pol = dict(policy) if isinstance(policy, dict) else {n: "bf16" for n in policy}
    bad = set(pol) - set(st)
    if bad:
        raise ValueError(f"unknown stages {sorted(bad)}; known: {list(st)}")
    for name, mode in pol.items():
        if mode not in STAGE_MODES or (mode == "fp16" and not name.startswith("vit.")):
            raise ValueError(f"stage {name}: unsupported precision {mode!r}")
    for name, m in st.items():
        m.dfu_precision = pol.get(name, "bf16x3")
    return model


def suffix(model, resnet_blocks=0, vit_blocks=0):
    """The bf16 policy that runs the last `resnet_blocks` Bottlenecks and the last `vit_blocks`
    ViT Blocks in bf16."""
    names = list(stages(model))
    rn = [n for n in names if n.startswith("resnet.layer")]
    vn = [n for n in names if n.startswith("vit.")]
    return tuple((rn[len(rn) - resnet_blocks:] if resnet_blocks else []) +
                 (vn[len(vn) - vit_blocks:] if vit_blocks else []))


def parity_policy(model, vit_x3_blocks=0):
    """The "parity" assignment as an explicit policy (ViT Blocks fp16, ResNet bf16x3), with the
    first `vit_x3_blocks` ViT Blocks bf16x3 instead (the study's variants)."""
    names = [n for n in stages(model) if n.startswith("vit.")]
    return {n: ("bf16x3" if k < vit_x3_blocks else "fp16") for k, n in enumerate(names)}


def mark_feature_extractor(model, on=True):
    """Mark the ViT inside `model` (or `model` itself) as a fusion feature extractor: its
    features reach the logits only through a late-fusion head beside the ResNet's 2048
    (train_multimodal_fusion.py:305-313, grad_cam_visualization.py:289-302), so the "parity"
    mode runs every Block fp16 (models/vit.py _parity_policy).  Unmarked, a ViT runs Blocks 0-8
    bf16x3 -- the safe assignment for a ViT whose features feed a head directly.
    models.fusion.MultimodalFusionModel marks its own ViT; a script that builds the fusion from
    models.encoders.create_model(num_classes=0) and torch.cat may call this.  Returns the
    model."""
    _, v = encoders(model)
    if v is None:
        raise ValueError("mark_feature_extractor: no VisionTransformer in the model")
    v.dfu_feature_extractor = bool(on)
    return model


def clear_policy(model):
    for m in stages(model).values():
        if "dfu_precision" in m.__dict__:
            del m.dfu_precision
    return model


__all__ = ["apply_policy", "clear_policy", "encoders", "mark_feature_extractor", "parity_policy",
           "stages", "suffix"]
