"""Build libgsr.so (HIP, gfx950) in-tree with hipcc.

    python -m gaussian_splatting_amd.build [--force] [--jobs N]

Each .hip translation unit is compiled to an object in parallel, then linked
into ``gaussian_splatting_amd/lib/libgsr.so``.  No torch headers are involved:
the library is a plain C ABI (include/gsr.h).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build")
LIB_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIB_DIR, "libgsr.so")
SOURCES = ["api.hip", "preprocess.hip", "binning.hip", "render.hip", "backward.hip", "knn.hip", "ssim.hip", "adam.hip", "densify.hip", "ply.cpp"]
HEADERS = ["gsr_common.h", "kernels.h", "footprint.h"]
ARCH = os.environ.get("GSR_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result",
            "-I", os.path.join(ROOT, "include"), "-I", CSRC]


def _newest_input_mtime() -> float:
    files = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", h) for h in
                                                                  ("gsr.h", "gsr_knn.h", "gsr_ssim.h", "gsr_adam.h", "gsr_densify.h", "gsr_ply.h")] + [__file__]
    return max(os.path.getmtime(f) for f in files)


# Per-file flags.  The SLP vectorizer packs adjacent fp32 ops into v_pk_*_f32 plus
# v_mov shuffles; on gfx950 packed fp32 is not faster than two plain ops
# (MI355X_MICROARCH.md, "price of one filler"), so the VALU-bound kernels opt out.
# preprocess.hip is compiled without FMA contraction: every integer it derives from floats
# (radius, getRect's tile rectangle, tiles_touched, hence num_rendered and the tile lists) then
# comes from the same individually rounded operations as the reference's and the oracle's
# (oracle/Makefile builds with -ffp-contract=off), so those integers are identical, not close.
# backward.hip: contraction inside each expression only (-ffp-contract=on, not HIP's default
# "fast", which fuses a multiply into an add wherever the backend's DAG sees both) and no SLP
# vectorisation (it also splits fmuladd pairs into a packed multiply plus a scalar add): an
# expression then rounds the same way whatever code surrounds it, so the split and combined SH
# layouts' kernels give bitwise-equal gradients (tests/test_separate_sh.py).
FILE_FLAGS = {"render.hip": ["-fno-slp-vectorize"],
              "backward.hip": ["-fno-slp-vectorize", "-ffp-contract=on"],
              "preprocess.hip": ["-fno-slp-vectorize", "-ffp-contract=off"]}


def _compile(src: str, objdir: str = OBJ, extra=()) -> str:
    obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
    cmd = [HIPCC, *CXXFLAGS, *FILE_FLAGS.get(src, []), *extra, "-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 5, verbose: bool = True, variant: str = "", extra=()) -> str:
    """Compile every HIP source for gfx950 and link libgsr.so; returns the library path.

    ``variant``/``extra`` build a side library ``libgsr_<variant>.so`` with extra compiler
    flags (for A/B measurements; select it at run time with GSR_LIBRARY)."""
    lib = LIB if not variant else os.path.join(LIB_DIR, f"libgsr_{variant}.so")
    objdir = OBJ if not variant else os.path.join(OBJ, variant)
    if not force and os.path.exists(lib) and os.path.getmtime(lib) >= _newest_input_mtime():
        return lib
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda f: _compile(f, objdir, extra), SOURCES))
    LIB_OUT = lib
    tmp = os.path.join(os.path.dirname(LIB_OUT), "tmp_" + os.path.basename(LIB_OUT))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB_OUT)
    # the offload bundler may leave per-object device images next to the output; nothing loads them
    import glob

    for stray in glob.glob(os.path.join(os.path.dirname(LIB_OUT), "*.hipv4-amdgcn-*")) + \
            glob.glob(os.path.join(os.path.dirname(LIB_OUT), "*.host-x86_64-*")):
        os.remove(stray)
    if verbose:
        print(f"[gsr] built {LIB_OUT}")
    return LIB_OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=5)
    ap.add_argument("--variant", default="")
    ap.add_argument("--cflags", default="")
    args = ap.parse_args()
    try:
        build(force=args.force, jobs=args.jobs, variant=args.variant, extra=tuple(args.cflags.split()))
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
