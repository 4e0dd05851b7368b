"""ORACLE — test infrastructure only (imported by tests/; never by dfu-multimodal_amd/).

CPU restatement of the reference's Grad-CAM (notebooks/grad_cam_visualization.py:327-429) on the
plain-PyTorch oracle models (oracle/torch_ref.py), for the config-C5 parity tests:
  * forward hooks on every module whose name contains a target string store the output and
    register a tensor hook for its gradient (:339-357);
  * generate_cam: eval mode, input cloned with requires_grad, score output[0, 0] backpropagated
    (:370-386); the target is the last matching module name (:389-392);
  * 4-D target: weights = grad.mean((2, 3)); cam = sum_i w_i * A_i over the first
    min(C_act, C_grad) channels (in channel order), ReLU, / max if max > 0 (:415-429); otherwise
    |input grad|.mean(1) / max (:401-413).
  * the hook protocol on a ResNet Bottleneck, whose single `relu` module runs three times per
    block: the stored activation is the last call's output (the 2048-channel block output); the
    tensor hooks fire in reverse order in backward, so the stored gradient is the FIRST call's
    (the 512-channel conv1/bn1 ReLU output) — the channel-mismatch branch (:418-422) is the one
    the reference actually runs for 'layer4'.  Reproduced here by the same module calls.
Parity status: the reference file cannot run here (it needs timm/torchvision/cv2 and pretrained
weights), so this restatement is checked only against the reference's source text; the CAM
arithmetic is four torch ops and the hook protocol is plain nn.Module API.
"""
import torch
import torch.nn.functional as F


class GradCAMRef:
    def __init__(self, model, target_layers):
        self.model = model
        self.target_layers = target_layers if isinstance(target_layers, list) else [target_layers]
        self.activations, self.gradients = {}, {}
        for name, module in model.named_modules():
            if any(t in name for t in self.target_layers):
                module.register_forward_hook(self._hook(name))

    def _hook(self, name):
        def hook(module, inputs, output):
            self.activations[name] = output
            if isinstance(output, torch.Tensor) and output.requires_grad:
                output.register_hook(lambda g: self.gradients.__setitem__(name, g))
        return hook

    def target_name(self):
        last = None
        for n, _ in self.model.named_modules():
            if any(t in n for t in self.target_layers):
                last = n
        return last

    def generate_cam(self, x):
        """x: (1, C, H, W) -> fp32 (h, w) CAM (or (H, W) input saliency)."""
        self.model.eval()
        xi = x.clone().detach().requires_grad_(True)
        with torch.enable_grad():
            out = self.model(xi)
            self.model.zero_grad()
            out[0, 0].backward()
        name = self.target_name()
        act, grad = self.activations[name], self.gradients.get(name)
        if act.ndim != 4 or grad is None or grad.ndim != 4:
            sal = xi.grad.detach().abs().mean(dim=1)[0]
            return sal / sal.max() if sal.max() > 0 else sal
        w = grad.mean(dim=(2, 3))
        cam = torch.zeros(act.shape[2:])
        for i in range(min(act.shape[1], w.shape[1])):
            cam = cam + w[0, i] * act[0, i].detach()
        cam = F.relu(cam)
        return cam / cam.max() if cam.max() > 0 else cam


def saliency_ref(model, x):
    """The ViT branch of generate_cam (timm's last 'blocks' module is 3-D, so :401-413 applies):
    |d output[0, 0] / d input|.mean(channel) / max, for a (1, C, H, W) input.  (The oracle ViT
    has no timm Identity submodules to hook, so the fallback is computed directly.)"""
    model.eval()
    xi = x.clone().detach().requires_grad_(True)
    with torch.enable_grad():
        model(xi)[0, 0].backward()
    sal = xi.grad.detach().abs().mean(dim=1)[0]
    return sal / sal.max() if sal.max() > 0 else sal
