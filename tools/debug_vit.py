"""Stage-by-stage ViT block forward: HIP saved intermediates vs torch fp32 on the GPU fed the
same (bf16-rounded) inputs (debug tool)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch
import torch.nn.functional as F
from models.vit import VisionTransformer

def rel(a, b):
    a = a.detach().float(); b = b.detach().float()
    return ((a - b).norm() / b.norm().clamp(min=1e-12)).item()
rb = lambda t: t.to(torch.bfloat16).float()
torch.manual_seed(0)
v = VisionTransformer(num_classes=0, depth=1).cuda()
B = 2
th = torch.randn(B, 3, 224, 224, device="cuda")
X = v._embed(th)
pe = v.patch_embed
ref_X = torch.cat([v.cls_token.expand(B, -1, -1), F.conv2d(rb(th), rb(pe.proj.weight), pe.proj.bias, stride=16).flatten(2).transpose(1, 2)], 1) + v.pos_embed
print("embed", rel(X, ref_X))
blk = v.blocks[0]
xo = blk(X)
ctx = xo.grad_fn
(x2, xn1, m1, r1, qkv, o, lse, xm, xn2, m2, r2, hpre, h, wqkv, wproj, wfc1, wfc2) = ctx.saved_tensors
T = 197; D = 768
x2r = X.reshape(-1, D)
ln1 = F.layer_norm(x2r, (D,), blk.norm1.weight, blk.norm1.bias, 1e-6)
print("ln1", rel(xn1, ln1), "mean", rel(m1, x2r.mean(-1)))
qkv_r = F.linear(xn1.float(), rb(blk.attn.qkv.weight), blk.attn.qkv.bias)
print("qkv", rel(qkv, qkv_r))
q, k, vv = qkv.float().view(B, T, 3, 12, 64).permute(2, 0, 3, 1, 4).unbind(0)
s = (q @ k.transpose(-1, -2)) * 0.125
p = torch.exp(s - s.amax(-1, keepdim=True))
o_r = ((rb(p) @ vv) / p.sum(-1, keepdim=True)).transpose(1, 2).reshape(B * T, D)
o_exact = F.scaled_dot_product_attention(q, k, vv).transpose(1, 2).reshape(B * T, D)
print("attn o vs emu", rel(o, o_r), " vs exact", rel(o, o_exact), " emu vs exact", rel(o_r, o_exact))
print("lse", rel(lse.view(B, 12, -1)[:, :, :T], torch.logsumexp(s, -1)))
xm_r = x2r + F.linear(o.float(), rb(blk.attn.proj.weight), blk.attn.proj.bias)
print("x_mid", rel(xm, xm_r))
ln2 = F.layer_norm(xm, (D,), blk.norm2.weight, blk.norm2.bias, 1e-6)
print("ln2", rel(xn2, ln2))
hp_r = F.linear(xn2.float(), rb(blk.mlp.fc1.weight), blk.mlp.fc1.bias)
print("fc1 pre", rel(hpre, hp_r), "gelu", rel(h, F.gelu(hpre.float())))
xo_r = xm + F.linear(h.float(), rb(blk.mlp.fc2.weight), blk.mlp.fc2.bias)
print("x_out", rel(xo.reshape(-1, D), xo_r))
