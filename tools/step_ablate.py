"""Step-level timing ablation of the C3 fusion step: how long the step would take if one family
of kernels were free.  One process: the library-default fusion step (bench.py's model, batch and
optimizer), timed with HIP events over K steps, alternating the baseline with variants that skip
the named C-ABI launches (their outputs keep the previous step's values, so the data the other
kernels see stays realistic; results are wrong by design: timing only).  In the two-stream step a
kernel's own duration says little about what it costs the step (the other encoder fills the CUs
it leaves idle); this measures the step instead.

  python tools/step_ablate.py [--steps 10] [--rounds 3] [--variants bn_fin,attn_bwd,...]
      [--config rgb]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import functional as Fn  # noqa: E402
from dfu_hip import nn as hnn  # noqa: E402
from dfu_hip.optim import FusedAdamW  # noqa: E402

EPI_BF16, EPI_F32_RESID, EPI_BF16_DGELU, EPI_F32_ACC, EPI_F16_GELU = 0, 4, 5, 7, 15
# variant -> C-ABI symbols skipped, or ("gemm", predicate on the descriptor)
VARIANTS = {
    "bn_fin": ["dfu_bn_finalize", "dfu_bn_bwd_finalize"],
    "bn_apply_x3": ["dfu_bn_apply_x3"],
    "bn_bwd": ["dfu_bn_bwd", "dfu_bn_bwd_reduce", "dfu_bn_bwd_finalize", "dfu_bn_bwd_apply"],
    "attn_bwd": ["dfu_attention_bwd", "dfu_attention_bwd_qkv16"],
    "attn": ["dfu_attention_fwd", "dfu_attention_fwd_f16", "dfu_attention_bwd",
             "dfu_attention_bwd_qkv16"],
    "ln": ["dfu_layernorm_fwd", "dfu_layernorm_fwd_x3", "dfu_layernorm_fwd_h16",
           "dfu_layernorm_bwd"],
    "adamw": ["dfu_adamw_flat", "dfu_transpose_bf16"],
    "colsum": ["dfu_colsum", "dfu_reduce_partials", "dfu_reduce_partials_batch"],
    "gemm_wgrad": ("gemm", lambda d: d.epilogue == EPI_F32_ACC),
    # the ViT's weight gradients reduce over its 64 x 197 = 12608 token rows
    "gemm_wgrad_vit": ("gemm", lambda d: d.epilogue == EPI_F32_ACC and d.K == 12608),
    "gemm_wgrad_resnet": ("gemm", lambda d: d.epilogue == EPI_F32_ACC and d.K != 12608),
    "gemm_x3pairs": ("gemm", lambda d: bool(d.x3_pairs)),
    "gemm_dgrad_strided": ("gemm", lambda d: d.a_mode == 3),  # OPND_CONV_DGRAD (stride 2)
    "gemm_resnet_dgrad": ("gemm", lambda d: d.M != 12608 and not d.x3_pairs and
                          d.epilogue in (EPI_BF16, 6)),  # BF16 / BF16_ADD input gradients
    "gemm_x3_layer1": ("gemm", lambda d: bool(d.x3_pairs) and d.M == 200704),
    "gemm_x3_deep": ("gemm", lambda d: bool(d.x3_pairs) and d.M < 200704),
    "gemm_f16_gelu": ("gemm", lambda d: d.operand_type == 1 and d.epilogue == EPI_F16_GELU),
    "gemm_f16_resid": ("gemm", lambda d: d.operand_type == 1 and d.epilogue == EPI_F32_RESID),
    "gemm_vit_dgrad": ("gemm", lambda d: d.M == 12608 and d.epilogue in (EPI_BF16, EPI_BF16_DGELU)),
    "gemm_f16": ("gemm", lambda d: d.operand_type == 1),
    "gemm_all": ("gemm", lambda d: True),
}


class _Proxy:
    """The loaded library with some symbols replaced by no-ops (rc 0)."""

    def __init__(self, real):
        self._real = real
        self.skip = set()
        self.gemm_pred = None

    def __getattr__(self, name):
        fn = getattr(self._real, name)
        if name in self.skip:
            return lambda *a, **k: 0
        if name == "dfu_gemm" and self.gemm_pred is not None:
            pred = self.gemm_pred

            def gemm(dref, stream):
                return 0 if pred(dref._obj) else fn(dref, stream)
            return gemm
        return fn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--config", default="fusion", help="fusion | rgb | thermal (bench.build)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    proxy = _Proxy(L.load())
    L._lib = proxy  # every L.load() / ops.lib() from here on returns the proxy
    torch.manual_seed(42)
    model, fwd = bench.build(a.config, dev)
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=dev))
    rgb, th, y = bench.synthetic(64, dev, seed=42)

    def step():
        opt.zero_grad()
        loss = crit(fwd(model, rgb, th), y)
        loss.backward()
        Fn.join_grad_streams()
        opt.step()

    def timed(n):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            step()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    for _ in range(5):
        step()
    names = [v for v in a.variants.split(",") if v]
    res = {v: [] for v in ["baseline"] + names}
    for r in range(a.rounds):
        for v in names:
            proxy.skip, proxy.gemm_pred = set(), None
            timed(2)
            res["baseline"].append(timed(a.steps))
            spec = VARIANTS[v]
            if isinstance(spec, tuple):
                proxy.gemm_pred = spec[1]
            else:
                proxy.skip = set(spec)
            timed(2)
            res[v].append(timed(a.steps))
            proxy.skip, proxy.gemm_pred = set(), None
            print(f"round {r} {v:14s} {res[v][-1]:7.3f} ms  (baseline {res['baseline'][-1]:7.3f})",
                  flush=True)
    base = sorted(res["baseline"])[len(res["baseline"]) // 2]
    print(f"\nbaseline median {base:.3f} ms/step over {len(res['baseline'])} runs")
    for v in names:
        med = sorted(res[v])[len(res[v]) // 2]
        print(f"  without {v:14s} {med:7.3f} ms  ({100 * (base - med) / base:5.1f}% of the step)")


if __name__ == "__main__":
    main()
