"""Per-stage forward precision of the HIP encoders (functional.set_precision("mixed")).

A stage is the ResNet stem ("resnet.stem"), a ResNet Bottleneck ("resnet.layer<i>.<j>") or a
ViT Block ("vit.blocks.<k>").  A *policy* names the stages whose forward runs in plain bf16;
every other stage runs bf16x3 (fp32-accurate).  Rounding introduced late in an encoder is
amplified by fewer layers than rounding introduced early, so the cheapest policy that keeps the
fusion logits within north_star's 1e-3 of the fp32 oracle runs a suffix of each encoder in bf16.
The shipped policy (PARITY_POLICY) and the study it comes from are in DESIGN.md §4 and
profiles/r16_precision_study.{json,md} (tools/precision_policy_study.py).
"""
# The policy the bench's headline mode runs ("parity": the cheapest stage assignment measured to
# hold max |logits - fp32 oracle| <= 5e-4 at C3 B = 64 on every seed of the study).
PARITY_POLICY = ()


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
    """Ordered {name: module} of every stage the policy can name."""
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


def apply_policy(model, bf16_stages):
    """Mark the named stages bf16 and every other stage bf16x3 (effective under
    functional.precision("mixed")).  Unknown names raise; returns the model."""
    st = stages(model)
    names = set(bf16_stages)
    bad = names - set(st)
    if bad:
        raise ValueError(f"unknown stages {sorted(bad)}; known: {list(st)}")
    for name, m in st.items():
        m.dfu_precision = "bf16" if name in names else "bf16x3"
    return model


def suffix(model, resnet_blocks=0, vit_blocks=0):
    """The policy that runs the last `resnet_blocks` Bottlenecks and the last `vit_blocks` ViT
    Blocks in bf16."""
    names = list(stages(model))
    rn = [n for n in names if n.startswith("resnet.layer")]
    vn = [n for n in names if n.startswith("vit.")]
    return tuple((rn[len(rn) - resnet_blocks:] if resnet_blocks else []) +
                 (vn[len(vn) - vit_blocks:] if vit_blocks else []))


def clear_policy(model):
    for m in stages(model).values():
        if "dfu_precision" in m.__dict__:
            del m.dfu_precision
    return model


__all__ = ["PARITY_POLICY", "apply_policy", "clear_policy", "encoders", "stages", "suffix"]
