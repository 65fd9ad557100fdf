"""Generate the golden fixtures under tests/golden/ (run in the build container only).

    python tests/golden/make_golden.py [--reference /root/reference]

Two kinds of vectors, both small .npz files of inputs and expected outputs:

1. REFERENCE vectors -- produced by importing the reference's own Python functions
   (they run on CPU; SURVEY.md section 8c lists them):
     camera.npz   utils/graphics_utils.py:38-71 getWorld2View2 / getProjectionMatrix composed as
                  scene/cameras.py:86-89 (world_view_transform, full_proj_transform, camera_center)
     sh_eval.npz  utils/sh_utils.py:57-112 eval_sh, composed as gaussian_renderer/__init__.py:86-96
                  (convert_SHs_python: colours = clamp_min(eval_sh(...) + 0.5, 0))
     l1_grad.npz  utils/loss_utils.py:16-19 l1_loss, its autograd gradient (the upstream-gradient
                  convention of train.py:155)
     ssim.npz     utils/loss_utils.py ssim/_ssim (conv2d SSIM), mean and autograd gradient: pins
                  oracle/ssim.py, the oracle of the fused-SSIM kernels
     cov3d.npz    scene/gaussian_model.py:32-42 build_covariance_from_scaling_rotation with
                  utils/general_utils.py:65-110 (build_rotation, build_scaling_rotation,
                  strip_symmetric) -- GaussianModel.get_covariance, the cov3D_precomp input of
                  compute_cov3D_python (gaussian_renderer/__init__.py:86-87); compiled from the
                  reference's source with "cuda" read as "cpu".  Pins the oracle's computeCov3D
                  and the HIP cov3D_precomp path
   These pin the camera conventions, the SH polynomial and the loss-gradient convention of the
   oracle and the HIP path.  The reference's rasterizer itself cannot run here (CUDA source,
   no nvcc, and BACKWARD::render is missing from the source).

2. RASTERIZER vectors -- raster_<case>.npz: inputs and the float64 oracle's outputs
   (oracle/gsr_oracle.c, the C restatement, which tests/test_oracle_autograd.py pins against
   torch autograd of an independent restatement and tests/test_golden.py against the vectors
   above).  The GPU parity tests compare the HIP path with these on the box, where neither the
   reference nor (by design) any generator runs.

Nothing from the reference is copied into the fixtures except these input/output arrays.
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

# (W, H, focal, yaw_deg) cameras; the geometry (camera yawed about +y around (0,0,7)) is
# gaussian_splatting_amd/synthetic.py's, the matrix conventions are the reference's.
CAMERAS = [(64, 48, 60.0, 0.0), (37, 23, 30.0, 15.0), (1920, 1080, 1600.0, 5.0), (256, 256, 213.0, -35.0)]

RASTER_CASES = ["sh3_scalerot", "ragged_37x23", "sh1_of_16", "colors_precomp", "cov3d_precomp", "antialiasing",
                "background", "scale_modifier", "yawed_view"]


def camera_pose(yaw_deg: float, pivot_z: float = 7.0):
    th = math.radians(yaw_deg)
    c, s = math.cos(th), math.sin(th)
    R = np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])
    center = np.array([0.0, 0.0, pivot_z]) + R @ np.array([0.0, 0.0, -pivot_z])
    return R, -R.T @ center


def make_camera_vectors(gu):
    out = {}
    for i, (W, H, f, yaw) in enumerate(CAMERAS):
        R, T = camera_pose(yaw)
        fovx, fovy = gu.focal2fov(f, W), gu.focal2fov(f, H)
        wv = torch.tensor(gu.getWorld2View2(R, T)).transpose(0, 1)
        pm = gu.getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fovx, fovY=fovy).transpose(0, 1)
        full = wv.unsqueeze(0).bmm(pm.unsqueeze(0)).squeeze(0)
        campos = wv.inverse()[3, :3]
        out[f"cam{i}_inputs"] = np.array([W, H, f, yaw, fovx, fovy], np.float64)
        out[f"cam{i}_R"], out[f"cam{i}_T"] = R, T
        out[f"cam{i}_viewmatrix"] = wv.numpy()
        out[f"cam{i}_projmatrix"] = full.numpy()
        out[f"cam{i}_campos"] = campos.numpy()
    np.savez_compressed(os.path.join(HERE, "camera.npz"), **out)


def make_sh_vectors(sh_utils):
    """A small synthetic scene seen by a yawed camera; colours from the reference's eval_sh for every
    degree.  Rendering with shs= must equal rendering with colors_precomp= these colours."""
    from gaussian_splatting_amd import synthetic as syn

    cam = syn.make_camera(64, 48, 60.0, 10.0)
    sc = syn.make_scene(96, syn.make_camera(64, 48, 60.0, 0.0), sh_degree=3, seed=11, scale_range=(0.02, 0.25),
                        z_range=(2.0, 8.0))
    feats = sc.shs * 6.0  # larger higher-order terms than the benchmark scene, so every degree matters
    P = sc.P
    out = dict(means3D=sc.means3D.numpy(), scales=sc.scales.numpy(), rotations=sc.rotations.numpy(),
               opacities=sc.opacities.numpy(), features=feats.numpy(), viewmatrix=cam.viewmatrix.numpy(),
               projmatrix=cam.projmatrix.numpy(), campos=cam.campos.numpy(),
               camera=np.array([cam.width, cam.height, cam.tanfovx, cam.tanfovy], np.float64))
    for deg in range(4):
        # gaussian_renderer/__init__.py:86-96 (convert_SHs_python branch)
        shs_view = feats.transpose(1, 2).view(-1, 3, 16)
        dir_pp = sc.means3D - cam.campos.repeat(P, 1)
        dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
        sh2rgb = sh_utils.eval_sh(deg, shs_view, dir_pp_normalized)
        out[f"colors_deg{deg}"] = torch.clamp_min(sh2rgb + 0.5, 0.0).numpy()
    out["rgb2sh_in"] = np.linspace(0, 1, 7, dtype=np.float32)
    out["rgb2sh_out"] = sh_utils.RGB2SH(torch.tensor(out["rgb2sh_in"])).numpy()
    np.savez_compressed(os.path.join(HERE, "sh_eval.npz"), **out)


def make_l1_vectors(loss_utils):
    g = torch.Generator().manual_seed(5)
    img = torch.rand(3, 12, 10, generator=g, requires_grad=True)
    gt = torch.rand(3, 12, 10, generator=g)
    loss = loss_utils.l1_loss(img, gt)
    loss.backward()
    np.savez_compressed(os.path.join(HERE, "l1_grad.npz"), image=img.detach().numpy(), gt=gt.numpy(),
                        loss=np.array(loss.item()), grad=img.grad.numpy())


def make_ssim_vectors(loss_utils):
    """utils/loss_utils.py ssim (conv2d, 11x11 window, sigma 1.5) -- the function the reference's
    fused-ssim test compares its kernels against (submodules/fused-ssim/tests/test.py:23-52,78-87) --
    evaluated in float64 on CPU: the mean SSIM and its autograd gradient w.r.t. img1."""
    out = {}
    g = torch.Generator().manual_seed(9)
    for i, shape in enumerate([(1, 3, 37, 53), (2, 2, 40, 45), (1, 1, 16, 9)]):
        img1 = torch.rand(shape, generator=g, dtype=torch.float64)
        img2 = (0.7 * img1 + 0.3 * torch.rand(shape, generator=g, dtype=torch.float64)).clamp(0, 1)
        x = img1.clone().requires_grad_(True)
        val = loss_utils.ssim(x, img2)
        val.backward()
        out[f"img1_{i}"], out[f"img2_{i}"] = img1.numpy(), img2.numpy()
        out[f"value_{i}"], out[f"grad_{i}"] = np.array(val.item()), x.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "ssim.npz"), **out)


class _CudaToCpu(__import__("ast").NodeTransformer):
    """Reads the device literal "cuda" as "cpu" -- the only change made to the reference's code."""

    def visit_Constant(self, node):
        if node.value == "cuda":
            node.value = "cpu"
        return node


def _reference_covariance(reference):
    """GaussianModel.get_covariance's function (scene/gaussian_model.py:32-42, built by setup_functions)
    with build_scaling_rotation / build_rotation / strip_symmetric (utils/general_utils.py:65-110),
    compiled from the reference's source with the device literal "cuda" read as "cpu" so it runs here.
    (scene/ does not import in this container: cameras.py needs cv2.)"""
    import ast

    ns = {"torch": torch, "np": np}
    gu = ast.parse(open(os.path.join(reference, "utils/general_utils.py")).read())
    funcs = [n for n in gu.body if isinstance(n, ast.FunctionDef)]
    exec(compile(_CudaToCpu().visit(ast.Module(body=funcs, type_ignores=[])), "general_utils", "exec"), ns)
    gm = ast.parse(open(os.path.join(reference, "scene/gaussian_model.py")).read())
    cls = next(n for n in gm.body if isinstance(n, ast.ClassDef) and n.name == "GaussianModel")
    setup = next(n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name == "setup_functions")
    inner = next(n for n in setup.body if isinstance(n, ast.FunctionDef)
                 and n.name == "build_covariance_from_scaling_rotation")
    exec(compile(_CudaToCpu().visit(ast.Module(body=[inner], type_ignores=[])), "gaussian_model", "exec"), ns)
    return ns["build_covariance_from_scaling_rotation"], ns["build_rotation"]


def make_cov3d_vectors(reference):
    """cov3d.npz: the reference's own covariance (GaussianModel.get_covariance =
    build_covariance_from_scaling_rotation(get_scaling, modifier, _rotation), the cov3D_precomp input of
    compute_cov3D_python, gaussian_renderer/__init__.py:86-87) on the scene of the cov3d_precomp case, with
    un-normalised raw quaternions (get_covariance passes _rotation; build_rotation normalises), plus the
    normalised quaternion get_rotation would give (the rasterizer's scales/rotations input)."""
    from tests import common as C

    cov_fn, build_rotation = _reference_covariance(reference)
    case = next(c for c in C.SMALL_CASES if c.name == "cov3d_precomp")
    inp = C.build(C.Case(case.name, P=case.P, W=case.W, H=case.H, seed=case.seed))  # scales/rotations form
    g = torch.Generator().manual_seed(21)
    raw_rot = inp["rotations"] * (0.5 + 2.0 * torch.rand(case.P, 1, generator=g))  # as stored in _rotation
    out = {}
    for tag, mod in (("", 1.0), ("_mod", 0.7)):
        cov = cov_fn(inp["scales"], mod, raw_rot)
        out["cov3D" + tag] = cov.numpy().astype(np.float32)
        out["modifier" + tag] = np.array(mod)
    out["scales"] = inp["scales"].numpy()
    out["raw_rotations"] = raw_rot.numpy()
    out["rotations"] = torch.nn.functional.normalize(raw_rot).numpy()  # get_rotation (rotation_activation)
    out["R"] = build_rotation(raw_rot).numpy()
    np.savez_compressed(os.path.join(HERE, "cov3d.npz"), **out)


def make_raster_vectors():
    from tests import common as C
    from gaussian_splatting_amd import synthetic as syn

    cases = {c.name: c for c in C.SMALL_CASES}
    for name in RASTER_CASES:
        inp = C.build(cases[name])
        save_raster(name, inp, C, with_backward=True)
    # the reference's CPU-runnable config (BASELINE.json configs[0]): 10k Gaussians, 256x256, SH0, forward only
    scene, cam = syn.config_scene("10k_256_sh0", seed=0)
    inp = dict(bg=torch.zeros(3), means3D=scene.means3D, opacities=scene.opacities, shs=scene.shs, sh_degree=0,
               scales=scene.scales, rotations=scene.rotations, colors_precomp=None, cov3D_precomp=None,
               viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix, campos=cam.campos, tanfovx=cam.tanfovx,
               tanfovy=cam.tanfovy, H=cam.height, W=cam.width, scale_modifier=1.0, antialiasing=False)
    save_raster("10k_256_sh0", inp, C, with_backward=False)


def save_raster(name, inp, C, with_backward):
    ref = C.run_oracle(inp, precision="f64", nthreads=os.cpu_count())
    out = {}
    for k, v in inp.items():
        if v is None:
            continue
        out["in_" + k] = v.numpy() if torch.is_tensor(v) else np.array(v)
    out["out_color"] = ref.color.astype(np.float32)
    out["out_invdepth"] = ref.invdepth.astype(np.float32)
    out["out_radii"] = ref.radii.astype(np.int32)
    out["out_num_rendered"] = np.array(ref.num_rendered)
    if with_backward:
        gc, gd = C.unit_grads(inp["H"], inp["W"])
        out["grad_color"], out["grad_invdepth"] = gc.numpy(), gd.numpy()
        g = ref.handle.backward(gc.double().numpy(), gd.double().numpy(), nthreads=os.cpu_count())
        for k in C.GRAD_NAMES:
            out["out_" + k] = g[k].astype(np.float32)
    np.savez_compressed(os.path.join(HERE, f"raster_{name}.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    sys.path.insert(0, args.reference)
    from utils import graphics_utils as gu, loss_utils, sh_utils  # the reference's own Python

    make_camera_vectors(gu)
    make_l1_vectors(loss_utils)
    make_ssim_vectors(loss_utils)
    sys.path.remove(args.reference)
    make_cov3d_vectors(args.reference)
    make_sh_vectors(sh_utils)
    make_raster_vectors()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f"{f:32s} {os.path.getsize(os.path.join(HERE, f)):>9d} B")


if __name__ == "__main__":
    main()
