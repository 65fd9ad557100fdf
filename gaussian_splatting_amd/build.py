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


ABI_HEADERS = ("gsr.h", "gsr_knn.h", "gsr_ssim.h", "gsr_adam.h", "gsr_densify.h", "gsr_ply.h")


# Per-file flags.  The SLP vectorizer packs adjacent fp32 ops into v_pk_*_f32 plus
# v_mov shuffles; on gfx950 packed fp32 is not faster than two plain ops
# (MI355X_MICROARCH.md, "price of one filler"), so the VALU-bound kernels opt out.
# preprocess.hip is compiled without FMA contraction: every integer it derives from floats
# (radius, getRect's tile rectangle, tiles_touched, hence num_rendered and the tile lists) then
# comes from the same individually rounded operations as the oracle's (oracle/Makefile builds
# with -ffp-contract=off), so those integers are identical to the oracle's, not close.
# (That is the uncontracted ORACLE's rounding.  The reference itself is built by nvcc with its default
# --fmad=true -- RI/setup.py passes only -I -- so its radius and getRect decisions may come from
# contracted multiply-adds; DESIGN.md section 6 gives the measured difference between a contracted and
# an uncontracted oracle on the full-size frames.)
# backward.hip: contraction inside each expression only (-ffp-contract=on, not HIP's default
# "fast", which fuses a multiply into an add wherever the backend's DAG sees both) and no SLP
# vectorisation (it also splits fmuladd pairs into a packed multiply plus a scalar add): an
# expression then rounds the same way whatever code surrounds it, so the split and combined SH
# layouts' kernels give bitwise-equal gradients (tests/test_separate_sh.py).
FILE_FLAGS = {"render.hip": ["-fno-slp-vectorize"],
              "backward.hip": ["-fno-slp-vectorize", "-ffp-contract=on"],
              "preprocess.hip": ["-fno-slp-vectorize", "-ffp-contract=off"]}


def input_hash(extra=()) -> str:
    """sha256 over everything the library is compiled from: each source and header (name + bytes),
    the compiler flags (global, per file, extra) and the target.  Stored beside the library
    (``libgsr.so.inputs``) and compiled into it (``gsr_build_id``): the library is rebuilt whenever
    this changes, and the loader refuses a library whose id differs from the tree's (_lib.load)."""
    import hashlib
    import json

    h = hashlib.sha256()
    files = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", f) for f in ABI_HEADERS]
    for path in files:
        with open(path, "rb") as f:
            data = f.read()
        h.update(os.path.basename(path).encode() + b"\0" + str(len(data)).encode() + b"\0" + data)
    # (the compiler's path is not part of the identity: a library built with HIPCC=/custom/hipcc must load in a
    # shell without that variable; the target is)
    h.update(json.dumps([CXXFLAGS[:-4], FILE_FLAGS, list(extra), ARCH], sort_keys=True).encode())
    return h.hexdigest()


def _stamp_path(lib: str) -> str:
    return lib + ".inputs"


def _compile(src: str, objdir: str = OBJ, extra=(), build_id: str = "", verbose: bool = False) -> str:
    import time

    obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
    ident = [f'-DGSR_BUILD_ID="{build_id}"'] if build_id and src == "api.hip" else []
    cmd = [HIPCC, *CXXFLAGS, *FILE_FLAGS.get(src, []), *extra, *ident, "-c", os.path.join(CSRC, src), "-o", obj]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:  # one line per compiled file: the build log shows that hipcc ran, and for how long
        print(f"[gsr] hipcc {src} -> {os.path.basename(obj)} {time.perf_counter() - t0:.1f}s", flush=True)
    return obj


def build(force: bool = False, jobs: int = 5, verbose: bool = True, variant: str = "", extra=()) -> str:
    """Compile every HIP source for gfx950 and link libgsr.so; returns the library path.

    ``variant``/``extra`` build a side library ``libgsr_<variant>.so`` with extra compiler
    flags (for A/B measurements; select it at run time with GSR_LIBRARY)."""
    lib = LIB if not variant else os.path.join(LIB_DIR, f"libgsr_{variant}.so")
    objdir = OBJ if not variant else os.path.join(OBJ, variant)
    ident = input_hash(extra)
    stamp = _stamp_path(lib)
    if not force and os.path.exists(lib) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == ident:
                if verbose:
                    print(f"[gsr] {lib} is up to date (inputs sha256 {ident[:16]})")
                return lib
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    if verbose:
        print(f"[gsr] compiling {len(SOURCES)} sources with {HIPCC} --offload-arch={ARCH} (inputs sha256 {ident[:16]})",
              flush=True)
    if os.path.exists(stamp):
        os.remove(stamp)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda f: _compile(f, objdir, extra, ident, verbose), SOURCES))
    LIB_OUT = lib
    tmp = os.path.join(os.path.dirname(LIB_OUT), "tmp_" + os.path.basename(LIB_OUT))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB_OUT)
    with open(stamp, "w") as f:
        f.write(ident + "\n")
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
