"""Drop-in replacement of the reference's ``fused_ssim`` package
(submodules/fused-ssim/fused_ssim/__init__.py): same names, arguments and behaviour,
over ``fused_ssim_cuda`` (libgsr.so, csrc/ssim.hip).  train.py:34-39 imports
``fused_ssim`` and uses it at :157 when it is available.
"""
import torch

from fused_ssim_cuda import fusedssim, fusedssim_backward

allowed_padding = ["same", "valid"]


class FusedSSIMMap(torch.autograd.Function):
    """fused_ssim/__init__.py:8-33 of the reference."""

    @staticmethod
    def forward(ctx, C1, C2, img1, img2, padding="same", train=True):
        ssim_map, dm_dmu1, dm_dsigma1_sq, dm_dsigma12 = fusedssim(C1, C2, img1, img2, train)
        if padding == "valid":
            ssim_map = ssim_map[:, :, 5:-5, 5:-5]
        ctx.save_for_backward(img1.detach(), img2, dm_dmu1, dm_dsigma1_sq, dm_dsigma12)
        ctx.C1 = C1
        ctx.C2 = C2
        ctx.padding = padding
        return ssim_map

    @staticmethod
    def backward(ctx, opt_grad):
        img1, img2, dm_dmu1, dm_dsigma1_sq, dm_dsigma12 = ctx.saved_tensors
        C1, C2, padding = ctx.C1, ctx.C2, ctx.padding
        dL_dmap = opt_grad
        if padding == "valid":
            dL_dmap = torch.zeros_like(img1)
            dL_dmap[:, :, 5:-5, 5:-5] = opt_grad
        grad = fusedssim_backward(C1, C2, img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12)
        return None, None, grad, None, None, None


def fused_ssim(img1, img2, padding="same", train=True):
    """fused_ssim/__init__.py:35-41: mean SSIM with C1 = 0.01^2, C2 = 0.03^2."""
    C1 = 0.01 ** 2
    C2 = 0.03 ** 2
    assert padding in allowed_padding
    map = FusedSSIMMap.apply(C1, C2, img1, img2, padding, train)
    return map.mean()
