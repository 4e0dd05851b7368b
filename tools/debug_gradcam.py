"""Debug: eval-mode ResNet input gradients vs the oracle, stage by stage (the gradient arriving at
each layerN input), and the stem alone driven by the oracle's own layer1-input gradient."""
import copy, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gradcam_gpu import _pair
from oracle import torch_ref as R


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def grab(model):
    store = {}
    for n in ("layer1", "layer2", "layer3", "layer4"):
        def pre(mod, args, n=n):
            t = args[0]
            t.retain_grad()
            store[n] = t
        getattr(model, n).register_forward_pre_hook(pre)
    return store


ref, hip = _pair()
rgb, th, _ = R.synthetic_batch(2, seed=21)
eh, er = hip.resnet.eval(), copy.deepcopy(ref.resnet).eval()
sh, sr = grab(eh), grab(er)
xh = rgb.cuda().requires_grad_(True)
eh(xh)[:, 0].sum().backward()
xr = rgb.clone().requires_grad_(True)
er(xr)[:, 0].sum().backward()
for n in ("layer4", "layer3", "layer2", "layer1"):
    print(n, "act rel", rel(sh[n].detach(), sr[n].detach()), "grad rel", rel(sh[n].grad, sr[n].grad),
          "zeros", (sh[n].grad == 0).float().mean().item(), (sr[n].grad == 0).float().mean().item())
print("input grad rel", rel(xh.grad, xr.grad))
# stem alone, same upstream gradient
g = sr["layer1"].grad
xh2 = rgb.cuda().requires_grad_(True)
Rm = eh
import dfu_hip.functional as Fn
out_h = Fn.StemFn.apply(xh2, Rm.conv1.weight, Rm.bn1.weight, Rm.bn1.bias, Rm)
out_h.backward(g.cuda().to(out_h.dtype).contiguous(memory_format=torch.channels_last))
xr2 = rgb.clone().requires_grad_(True)
er2 = er
out_r = er2.maxpool(R.rb(er2.relu(er2.bn1(R.rb(R.conv(xr2, er2.conv1.weight, 2, 3))))))
out_r.backward(g)
print("stem out rel", rel(out_h.detach(), out_r.detach()), "stem dx rel", rel(xh2.grad, xr2.grad))
# ties in the pooled windows
a = R.rb(er2.relu(er2.bn1(R.rb(R.conv(rgb, er2.conv1.weight, 2, 3))))).detach()
u = torch.nn.functional.unfold(a.flatten(0, 1)[:, None], 3, padding=1, stride=2)
mx = u.max(1, keepdim=True).values
ties = ((u == mx).sum(1) > 1) & (mx[:, 0] > 0)
print("windows with a positive tied max:", ties.float().mean().item())
for n in ("layer1", "layer2", "layer3", "layer4"):
    a, b = sh[n].detach().float().cpu() > 0, sr[n].detach() > 0
    print(n, "relu-mask flips", (a != b).float().mean().item())
# against the bf16-rounded oracle (rounding at the same storage points as the HIP path)
R.set_bf16_emulation(True)
er3 = copy.deepcopy(ref.resnet).eval()
xr3 = rgb.clone().requires_grad_(True)
er3(xr3)[:, 0].sum().backward()
print("input grad rel vs bf16 oracle", rel(xh.grad, xr3.grad), "fp32 vs bf16 oracle", rel(xr.grad, xr3.grad))
