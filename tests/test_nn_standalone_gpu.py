"""dfu_hip.nn modules used outside the fused ResNet blocks:
a standalone BatchNorm2d (train and eval) and a Conv2d whose input channels are not a multiple
of 64 (explicit im2col + GEMM, as an image stem), each against torch.nn on the same bf16-rounded
operands (fp32 arithmetic): outputs, running statistics, input and parameter gradients."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _bf(t):
    return t.to(torch.bfloat16).float()


@pytest.mark.parametrize("C,H", [(64, 28), (32, 15), (8, 7)])
def test_batchnorm2d_standalone_train_and_eval(C, H):
    from dfu_hip import nn as hnn
    torch.manual_seed(0)
    B = 6  # M = B*H*W: ragged last 128-row tile for H = 15 and 7
    bn = hnn.BatchNorm2d(C).to(DEV)
    ref = torch.nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        ref.weight.copy_(bn.weight)
        ref.bias.copy_(bn.bias)
    x = (torch.randn(B, C, H, H, device=DEV) * 2 + 0.7).requires_grad_(True)
    xr = _bf(x.detach()).requires_grad_(True)
    for step in range(2):
        y = bn(x)
        yr = ref(xr)
        assert y.dtype == torch.bfloat16 and y.shape == (B, C, H, H)
        assert rel(y, yr) < 1e-2, (step, rel(y, yr))
        assert torch.allclose(bn.running_mean, ref.running_mean, rtol=1e-4, atol=1e-5)
        assert torch.allclose(bn.running_var, ref.running_var, rtol=1e-4, atol=1e-5)
        assert int(bn.num_batches_tracked) == int(ref.num_batches_tracked) == step + 1
        g = torch.randn(y.shape, device=DEV)
        (y.float() * g).sum().backward()
        (yr * _bf(g)).sum().backward()
        assert rel(x.grad, xr.grad) < 2e-2, rel(x.grad, xr.grad)
        assert rel(bn.weight.grad, ref.weight.grad) < 1e-2
        assert rel(bn.bias.grad, ref.bias.grad) < 1e-2
        for t in (x, xr, bn.weight, bn.bias, ref.weight, ref.bias):
            t.grad = None
    bn.eval()
    ref.eval()
    with torch.no_grad():
        assert rel(bn(x), ref(xr)) < 1e-2


def test_batchnorm2d_standalone_rejects_unsupported_channels():
    from dfu_hip import nn as hnn
    with pytest.raises(NotImplementedError, match="channels"):
        hnn.BatchNorm2d(24).to(DEV)(torch.randn(2, 24, 4, 4, device=DEV))


@pytest.mark.parametrize("C,K,R,stride,pad", [(3, 64, 7, 2, 3), (1, 32, 3, 1, 1), (20, 48, 3, 2, 1)])
def test_conv2d_standalone_any_channel_count(C, K, R, stride, pad):
    from dfu_hip import nn as hnn
    torch.manual_seed(1)
    conv = hnn.Conv2d(C, K, R, stride=stride, padding=pad, bias=False).to(DEV)
    ref = torch.nn.Conv2d(C, K, R, stride=stride, padding=pad, bias=False).to(DEV)
    with torch.no_grad():
        ref.weight.copy_(_bf(conv.weight))
    x = torch.randn(4, C, 33, 31, device=DEV).requires_grad_(True)
    xr = _bf(x.detach()).requires_grad_(True)
    y = conv(x)
    yr = ref(xr)
    assert y.shape == yr.shape and y.dtype == torch.bfloat16
    assert rel(y, yr) < 1e-2
    g = torch.randn(y.shape, device=DEV)
    (y.float() * g).sum().backward()
    (yr * _bf(g)).sum().backward()
    assert x.grad.dtype == torch.float32 and x.grad.shape == x.shape
    assert rel(x.grad, xr.grad) < 1e-2, rel(x.grad, xr.grad)
    assert rel(conv.weight.grad, ref.weight.grad) < 1e-2, rel(conv.weight.grad, ref.weight.grad)


def test_conv2d_channels_last_weight_needs_c64():
    """A FusedAdamW-managed spatial weight is stored KRSC; the explicit (c, r, s) im2col cannot
    read it, so a channel count the implicit GEMM cannot take raises a clear error."""
    from dfu_hip import nn as hnn
    from dfu_hip.optim import FusedAdamW
    conv = hnn.Conv2d(32, 32, 3, padding=1, bias=False).to(DEV)
    FusedAdamW(conv.parameters())
    with pytest.raises(NotImplementedError, match="C % 64"):
        conv(torch.randn(2, 32, 8, 8, device=DEV))
