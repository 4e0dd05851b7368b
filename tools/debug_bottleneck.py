"""Stage-by-stage check of BottleneckFn.backward against torch fp32 autograd on the GPU,
fed with the Function's own saved intermediates (debug tool)."""
import sys, os
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dfu-multimodal_amd")]
import torch
import torch.nn.functional as F
from models.resnet import Bottleneck
from dfu_hip import functional as Fn, ops

def rel(a, b):
    a = a.detach().float(); b = b.detach().float()
    return ((a - b).norm() / b.norm().clamp(min=1e-12)).item()

torch.manual_seed(0)
dev = "cuda"
blk = Bottleneck(256, 64).to(dev)
with torch.no_grad():
    for m in blk.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.uniform_(0.5, 1.5); m.bias.uniform_(-0.5, 0.5)
B, H = 2, 56
x = torch.randn(B, 256, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
out = blk(x)
g = torch.randn_like(out.float()).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
# grab ctx via grad_fn
ctx = out.grad_fn
saved = ctx.saved_tensors
xr, y1, a1, y2, a2, y3, o, w1, w2, w3 = saved[:10]
s1, s2, s3, sd = ctx.bns
out.backward(g)
torch.cuda.synchronize()
M = y3.shape[0]
gr = Fn.rows_view(g).float()

def bn_ref(y, st, bn, relu_out, dout, res=None):
    yf = y.float().clone().requires_grad_(True)
    gam = bn.weight.detach().clone().requires_grad_(True)
    bet = bn.bias.detach().clone().requires_grad_(True)
    z = F.batch_norm(yf, None, None, gam, bet, training=True, eps=bn.eps)
    if res is not None:
        z = z + res.float()
    # mask from the HIP forward output (same rounding)
    z = z * (relu_out.float() > 0).float() if relu_out is not None else z
    z.backward(dout.float())
    return yf.grad, gam.grad, bet.grad

# bn3 with residual + relu
dy3_ref, dg3, db3 = bn_ref(y3, s3, blk.bn3, o, gr, res=xr)
dy3 = torch.empty_like(y3); dres = torch.empty_like(y3)
s3.backward(Fn.rows_view(g), y3, o, True, dy3, dres)
print("bn3 dy", rel(dy3, dy3_ref))
# conv3 dgrad
da2_ref = dy3.float() @ blk.conv3.weight.detach().view(256, 64).float()
da2 = torch.empty_like(a2)
Fn.conv_dgrad(dy3, ctx.geo[2], w3, da2)
print("conv3 dgrad", rel(da2, da2_ref))
dy2_ref, _, _ = bn_ref(y2, s2, blk.bn2, a2, da2)
dy2 = torch.empty_like(y2)
s2.backward(da2, y2, a2, True, dy2, None)
print("bn2 dy", rel(dy2, dy2_ref))
# conv2 dgrad 3x3
dy2_nchw = dy2.float().view(B, H, H, 64).permute(0, 3, 1, 2)
da1_ref = torch.nn.grad.conv2d_input((B, 64, H, H), blk.conv2.weight.detach().float(), dy2_nchw, padding=1)
da1 = torch.empty_like(a1)
Fn.conv_dgrad(dy2, ctx.geo[1], w2, da1)
print("conv2 dgrad", rel(da1.view(B, H, H, 64).permute(0, 3, 1, 2), da1_ref))
dy1_ref, dg1, db1 = bn_ref(y1, s1, blk.bn1, a1, da1)
dy1 = torch.empty_like(y1)
s1.backward(da1, y1, a1, True, dy1, None)
print("bn1 dy", rel(dy1, dy1_ref))
dx_ref = dy1.float() @ blk.conv1.weight.detach().view(64, 256).float() + dres.float()
print("dx total (from ctx path)", rel(Fn.rows_view(x.grad), dx_ref))
# pure fp32 reference of the whole block from the same x
xf = x.detach().float().requires_grad_(True)
def blockf(xx):
    o1 = F.relu(F.batch_norm(F.conv2d(xx, blk.conv1.weight.float()), None, None, blk.bn1.weight, blk.bn1.bias, True))
    o2 = F.relu(F.batch_norm(F.conv2d(o1, blk.conv2.weight.float(), padding=1), None, None, blk.bn2.weight, blk.bn2.bias, True))
    o3 = F.batch_norm(F.conv2d(o2, blk.conv3.weight.float()), None, None, blk.bn3.weight, blk.bn3.bias, True)
    return F.relu(o3 + xx)
of = blockf(xf)
of.backward(g.float())
print("block out vs fp32", rel(out, of), "dx vs fp32", rel(x.grad, xf.grad))
print("dres vs masked g", rel(dres, gr * (o.float() > 0)))
