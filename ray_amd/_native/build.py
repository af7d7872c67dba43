"""In-tree native build for ray_amd.

Produces (all git-ignored, all travel with the gpurun snapshot):
  ray_amd/_native/libray_amd_hip.so   HIP/CDNA4 kernels + HBM arena glue (hipcc, gfx950)
  ray_amd/_native/_core*.so           C++ runtime core: shm object store, frame I/O loop,
                                      resource scheduler (CPython extension, g++)
  ray_amd/_native/raylet_bin           (optional) native helper binaries

Usage: python -m ray_amd._native.build [--force] [--only hip|core]
"""

from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
HIP_SRC = os.path.join(PKG, "ops", "csrc")
CORE_SRC = os.path.join(HERE, "src")
BUILD_DIR = os.path.join(HERE, "build")
HIP_LIB = os.path.join(HERE, "libray_amd_hip.so")
ARCH = os.environ.get("RAY_AMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
NO_SLP_SOURCES = {"attn.hip", "layernorm.hip", "gelu.hip"}


def _newer(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build_hip(force: bool = False, jobs: int = 8) -> str:
    os.makedirs(BUILD_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(HIP_SRC, "*.hip")))
    headers = glob.glob(os.path.join(HIP_SRC, "*.h"))
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(BUILD_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + headers):
            todo.append((s, o))

    def cc(so):
        s, o = so
        # VGPR-form MFMA: accumulators live in arch VGPRs, so the softmax / epilogue VALU
        # work on them needs no v_accvgpr_read/write round trips (gfx950 unified RF)
        vgpr_form = ["-mllvm", "-amdgpu-mfma-vgpr-form"]
        # attention: no SLP vectorisation — it pairs the softmax / dS multiplies into
        # v_pk_mul_f32 whose even-aligned operand pairs cost v_mov / v_alignbit / v_perm
        # shuffles of the MFMA accumulators (and packed f32 VALU is slower beside MFMAs:
        # MI355X_MICROARCH.md, 'price of one filler'): -10% / -14% VALU in dK/dV / dQ
        extra = ["-fno-slp-vectorize"] if os.path.basename(s) in NO_SLP_SOURCES else []
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
              "-munsafe-fp-atomics", "-Wno-unused-result"] + vgpr_form + extra +
             ["-c", s, "-o", o])

    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(cc, todo))
    if force or _newer(HIP_LIB, objs):
        tmp = HIP_LIB + ".tmp"
        # hipBLASLt (fp32-output GEMM selection, ops/csrc/gemm_lt.hip): SONAME
        # libhipblaslt.so.1, resolved to the copy torch already loaded when imported after it
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs +
             ["-L/opt/rocm/lib", "-lhipblaslt"])
        os.replace(tmp, HIP_LIB)
    return HIP_LIB


def core_lib_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(HERE, "_core" + suffix)


def build_core(force: bool = False) -> str:
    target = core_lib_path()
    srcs = sorted(glob.glob(os.path.join(CORE_SRC, "*.cc")))
    headers = glob.glob(os.path.join(CORE_SRC, "*.h"))
    if not srcs:
        return ""
    if not (force or _newer(target, srcs + headers)):
        return target
    import pybind11

    inc = [sysconfig.get_paths()["include"], pybind11.get_include()]
    os.makedirs(BUILD_DIR, exist_ok=True)
    objs = []

    def cc(s):
        o = os.path.join(BUILD_DIR, os.path.basename(s) + ".o")
        cmd = ["g++", "-O2", "-g", "-fPIC", "-std=c++17", "-fvisibility=hidden", "-Wall",
               "-Wno-unused-function", "-c", s, "-o", o]
        for i in inc:
            cmd += ["-I", i]
        _run(cmd)
        return o

    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(cc, srcs))
    tmp = target + ".tmp"
    _run(["g++", "-shared", "-o", tmp] + objs + ["-lpthread", "-lrt"])
    os.replace(tmp, target)
    return target


def build_all(force: bool = False) -> None:
    build_core(force)
    build_hip(force)


if __name__ == "__main__":
    force = "--force" in sys.argv
    only = None
    if "--only" in sys.argv:
        only = sys.argv[sys.argv.index("--only") + 1]
    if only in (None, "core"):
        print("core:", build_core(force))
    if only in (None, "hip"):
        print("hip:", build_hip(force))
