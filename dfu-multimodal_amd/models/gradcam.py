"""Grad-CAM on the MI355X path (BASELINE.json config C5): the reference's GradCAM
(notebooks/grad_cam_visualization.py:327-429) with its hook protocol unchanged, and the map
arithmetic on HIP kernels (dfu_gradcam, dfu_saliency).

The protocol (what callers and checkpoints rely on):
  * a forward hook on EVERY module whose name contains one of the target strings (:355-357),
    each storing its output and registering a tensor hook that stores that output's gradient
    (:341-351);
  * the target layer is the LAST matching name in named_modules() (:389-392): 'layer4.2.relu' for
    a ResNet-50 with ['layer4'] (a (B, 2048, 7, 7) block output), 'blocks.11.drop_path2' for the
    ViT with ['blocks'] (a 3-D (B, 197, 768) token tensor);
  * 4-D activation and gradient: weights = grad.mean((2, 3)), cam = ReLU(sum_c w_c A_c) / max
    over the first min(C_act, C_grad) channels (:415-429); otherwise input-gradient saliency
    |dx|.mean(channel) / max (:401-413);
  * a Bottleneck's `relu` runs three times per block in torchvision, so for 'layer4.2.relu' the
    stored activation is the block output (2048 channels) and the stored gradient the first
    call's, conv1's ReLU output (512 channels: hooks fire in reverse in backward) — the
    reference's map is the 512-channel mismatch case, and models.resnet replays the two inner
    calls to the hooks (with their gradients from the fused backward) to give the same map;
  * generate_cam runs the model in eval mode with the input requiring grad and backpropagates
    output[0, 0] (:370-386).
models.resnet / models.vit keep those module names and call `layer4[-1].relu` and
`blocks[-1].drop_path2` when hooked, and the stems return input gradients, so this runs the
reference's algorithm end to end on device.  `generate_cams` is the batched form (one backward of
sum_b output[b, 0]; in eval mode the images are independent, so each map equals the bs=1 one).
"""
import torch

from dfu_hip import functional as Fn
from dfu_hip import ops


class GradCAM:
    """grad_cam_visualization.py:327 GradCAM(model, target_layers)."""

    def __init__(self, model, target_layers):
        self.model = model
        self.target_layers = target_layers if isinstance(target_layers, list) else [target_layers]
        self.activations = {}
        self.gradients = {}
        self.handles = []
        self._register_hooks()

    def _register_hooks(self):
        def get_activation(name):
            def hook(module, inputs, output):
                self.activations[name] = output
                if isinstance(output, torch.Tensor) and output.requires_grad:
                    def save_grad(grad):
                        self.gradients[name] = grad
                    output.register_hook(save_grad)
            return hook

        for name, module in self.model.named_modules():
            if any(layer in name for layer in self.target_layers):
                self.handles.append(module.register_forward_hook(get_activation(name)))

    def remove(self):
        """Detach the hooks (the reference leaks them; this is opt-in)."""
        for h in self.handles:
            h.remove()
        self.handles = []

    def target_name(self):
        """The LAST module name matching a target string (:389-392)."""
        name = None
        for n, _ in self.model.named_modules():
            if any(layer in n for layer in self.target_layers):
                name = n
        return name

    def generate_cams(self, inputs, class_idx=None):
        """Batched Grad-CAM: (B, h, w) fp32 maps on the device (4-D target) or (B, H, W) input
        saliency (other targets), for the score output[:, 0] of every image."""
        self.model.eval()
        x = inputs.detach().clone().requires_grad_(True)
        with torch.enable_grad():
            out = self.model(x)
            self.model.zero_grad()
            out[:, 0].sum().backward()
        # the ViT blocks' weight gradients may run on the wgrad stream: join it (a graph capture
        # rejects unjoined work, and the next forward's weight reads must follow it)
        Fn.join_grad_streams()
        name = self.target_name()
        if name is None:
            return None
        act = self.activations.get(name)
        grad = self.gradients.get(name)
        if act is None or act.ndim != 4 or grad is None or grad.ndim != 4:
            if x.grad is None:
                return torch.zeros((x.shape[0],) + tuple(x.shape[2:]), device=x.device)
            return ops.saliency(x.grad.detach().float())
        return ops.gradcam(act.detach(), grad.detach())

    def generate_cam(self, input_tensor, class_idx=None):
        """Reference signature: (1, C, H, W) input -> numpy (h, w) map, or None."""
        if self.target_name() is None:
            print(f"Warning: Could not find layer {self.target_layers}")
            return None
        cams = self.generate_cams(input_tensor[:1], class_idx)
        return cams[0].cpu().numpy()
