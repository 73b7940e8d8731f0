"""Register / scratch / LDS usage of every gfx950 kernel in a hipcc object (.o) or in the
built library: the code object is unbundled from the object's .hip_fatbin section and its
AMDGPU metadata notes are read with llvm-readelf (no GPU needed).

    python tools/kernel_notes.py [radiative_transfer_amd/_lib/obj/lvg_kernels.o ...]

Prints one line per kernel: VGPRs, VGPR spills, SGPRs, SGPR spills, scratch bytes per lane,
LDS bytes. Diagnostic and test helper (tests/test_kernel_resources_cpu.py)."""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
FIELDS = {
    ".vgpr_count": "vgpr",
    ".vgpr_spill_count": "vgpr_spill",
    ".sgpr_count": "sgpr",
    ".sgpr_spill_count": "sgpr_spill",
    ".private_segment_fixed_size": "scratch",
    ".group_segment_fixed_size": "lds",
    ".agpr_count": "agpr",
}


def _demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                             text=True, check=True).stdout.split("\n")
        return [o.split("(")[0] for o in out[:len(names)]]
    except (OSError, subprocess.CalledProcessError):
        return names


def kernel_notes(obj: str) -> dict:
    """{demangled kernel name: {vgpr, vgpr_spill, sgpr, sgpr_spill, scratch, lds, agpr}}"""
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.co")
        with open(obj, "rb") as f:
            bundle = f.read(24) == b"__CLANG_OFFLOAD_BUNDLE__"   # hipcc --offload-device-only -c output
        if bundle:
            fb = obj
        else:
            subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", obj,
                            os.path.join(d, "x.o")], check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fb}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                             text=True).stdout
    kernels, cur = [], {}
    # one metadata map per kernel: the entries of the amdhsa.kernels list start at indent 2
    for line in txt.splitlines():
        s = line.strip()
        if line.startswith("  - ."):
            if cur:
                kernels.append(cur)
            cur = {}
            s = s[2:]
        m = re.match(r"(\.[a-z_]+):\s+(\S+)", s)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == ".name":
            cur["name"] = v
        elif k in FIELDS:
            cur[FIELDS[k]] = int(v)
    if cur:
        kernels.append(cur)
    kernels = [k for k in kernels if "name" in k]
    names = _demangle([k["name"] for k in kernels])
    return {n: {f: k.get(f, 0) for f in FIELDS.values()} for n, k in zip(names, kernels)}


def main(argv):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    objs = argv or [os.path.join(root, "radiative_transfer_amd", "_lib", "obj", f)
                    for f in ("lvg_kernels.o", "lvg_kernels_wide.o", "lvg_kernels_big.o", "lvg_wave.o")]
    for o in objs:
        print(f"== {os.path.relpath(o, root)}")
        for n, k in kernel_notes(o).items():
            print(f"  {n:60s} vgpr {k['vgpr']:3d} (+{k['agpr']} agpr) spill {k['vgpr_spill']:3d} | sgpr {k['sgpr']:3d} "
                  f"spill {k['sgpr_spill']:4d} | scratch {k['scratch']:4d} B/lane | lds {k['lds']}")


if __name__ == "__main__":
    main(sys.argv[1:])
