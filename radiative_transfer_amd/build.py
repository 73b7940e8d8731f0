"""Build the HIP/C++ library (liblvg_amd.so) for gfx950, in-tree.

hipcc cross-compiles without a GPU, so this runs in the CPU container as well
as on the GPU box. The .so lands in radiative_transfer_amd/_lib/ and travels
with the repository snapshot (git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "_lib")
LIB = os.path.join(LIB_DIR, "liblvg_amd.so")
SOURCES = ["lvg_kernels.hip", "lvg_kernels_big.hip", "lvg_kernels_wide.hip", "lvg_wave.hip", "lvg_transitions.hip", "lvg_sched.hip", "lvg_abi.cpp"]
HEADERS = ["lvg_device.h", "lvg_common.h", "lvg_lu256.h", "lvg_kernels.hip", os.path.join("..", "..", "include", "lvg_amd.h"),
           os.path.join("..", "..", "include", "lvg_math.h")]
ARCH = os.environ.get("LVG_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, lib: str = LIB, defines=(), obj_sub: str = "obj") -> str:
    """Compile every source to an object in parallel (hipcc per file), then link.
    `defines` / `lib` / `obj_sub` build a diagnostic variant of the same sources (build_checked)."""
    if not force and lib == LIB and not _stale():
        return LIB
    from concurrent.futures import ThreadPoolExecutor
    obj_dir = os.path.join(LIB_DIR, obj_sub)
    os.makedirs(obj_dir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall",
             "-Wno-unused-function"] + ["-D" + d for d in defines]
    objs = [os.path.join(obj_dir, os.path.splitext(f)[0] + ".o") for f in SOURCES]

    def compile_one(i):
        cmd = [HIPCC] + flags + ["-c", os.path.join(CSRC, SOURCES[i]), "-o", objs[i]]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)

    with ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 1)) as ex:
        list(ex.map(compile_one, range(len(SOURCES))))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(lib + ".tmp", lib)
    return lib


CHECKED_LIB = os.path.join(LIB_DIR, "liblvg_amd_checked.so")


def build_checked(verbose: bool = False) -> str:
    """The product sources with -DLVG_CHECKED_GLB: every glb() cast traps on an LDS or scratch
    pointer (lvg_common.h, the HBM-only rule). Run the GPU suite on it with
    LVG_LIB_PATH=radiative_transfer_amd/_lib/liblvg_amd_checked.so."""
    return build(force=True, verbose=verbose, lib=CHECKED_LIB, defines=("LVG_CHECKED_GLB",), obj_sub="obj_checked")


HOST_SRCS = [os.path.join(PKG, "host", f) for f in ("lvg_host.cpp", "lvg_ingest.cpp")]
HOST_HDRS = [os.path.join(PKG, "host", f) for f in ("lvg_host.hpp", "lvg_ingest.hpp")]
HOST_LIB = os.path.join(LIB_DIR, "liblvg_host.so")
CXX = os.environ.get("CXX", "g++")


def build_host(force: bool = False, verbose: bool = False) -> str:
    """The C++ host surface (host/lvg_host.{hpp,cpp}) over the C ABI: liblvg_host.so,
    linked against liblvg_amd.so in the same directory (rpath $ORIGIN)."""
    lib = build(verbose=verbose)
    deps = HOST_SRCS + HOST_HDRS + [os.path.join(ROOT, "include", "lvg_amd.h"), lib]
    if not force and os.path.exists(HOST_LIB) and all(os.path.getmtime(d) <= os.path.getmtime(HOST_LIB) for d in deps):
        return HOST_LIB
    cmd = [CXX, "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall", "-o", HOST_LIB + ".tmp"] + HOST_SRCS + [
           "-L" + LIB_DIR, "-llvg_amd", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(HOST_LIB + ".tmp", HOST_LIB)
    return HOST_LIB


if __name__ == "__main__":
    if "--checked" in sys.argv:
        print(build_checked(verbose=True))
        sys.exit(0)
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_host(force="--force" in sys.argv, verbose=True))
