"""Per-kernel resource metadata of the built libp3d.so's gfx950 code object (no GPU needed).

Extracts the .hip_fatbin section (llvm-objcopy), unbundles the gfx950 code object
(clang-offload-bundler) and reads its AMDGPU metadata note (llvm-readelf --notes):
VGPR / AGPR / SGPR counts, spill counts and the private (scratch) segment size of every kernel,
names demangled with c++filt.  Used by tests/test_kernel_resources.py (a kernel that starts
spilling to scratch fails in the build container, not on the box) and for the AGPR comparisons
DESIGN.md 6 asks for before any k_serve6 measurement.

    python tools/kernel_resources.py [libp3d.so] [--filter SUBSTRING]
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "3d-pose-baseline_amd", "libp3d.so")
KEYS = ("agpr_count", "vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
        "private_segment_fixed_size", "group_segment_fixed_size", "uses_dynamic_stack")


def kernel_resources(lib=LIB, arch="gfx950"):
    """{demangled kernel name: {key: value}} for every kernel of `lib`'s `arch` code object."""
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "co.o")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, lib, os.devnull],
                       check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + fat,
                        "--targets=hipv4-amdgcn-amd-amdhsa--" + arch, "--output=" + co], check=True, capture_output=True)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    out = {}
    # each kernel record is a "  - .agpr_count:" list item of amdhsa.kernels; its keys are indented
    for block in re.split(r"\n\s*- \.agpr_count:", notes)[1:]:
        block = ".agpr_count:" + block
        rec = {}
        m = re.search(r"\.name:\s+(\S+)", block)
        if not m:
            continue
        for k in KEYS:
            km = re.search(r"\." + k + r":\s+(\S+)", block)
            if km:
                v = km.group(1)
                rec[k] = (v == "true") if v in ("true", "false") else int(v)
        out[m.group(1)] = rec
    names = list(out)
    filt = shutil.which("c++filt") or os.path.join(LLVM, "llvm-cxxfilt")
    dem = subprocess.run([filt], input="\n".join(names), capture_output=True, text=True,
                         check=True).stdout.splitlines() if os.path.exists(filt) else names
    return {dm: dict(out[n], mangled=n) for n, dm in zip(names, dem)}


def kernel_isa(name_prefix, lib=LIB, arch="gfx950"):
    """Disassembly lines of the first kernel of `lib` whose demangled name starts with
    `name_prefix` (llvm-objdump of the unbundled gfx950 code object), from its symbol to the next
    kernel symbol."""
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "co.o")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, lib, os.devnull],
                       check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + fat,
                        "--targets=hipv4-amdgcn-amd-amdhsa--" + arch, "--output=" + co], check=True, capture_output=True)
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--symbolize-operands", co], check=True,
                             capture_output=True, text=True).stdout.split("\n")
    sym = re.compile(r"^[0-9a-f]{16} <(_Z\w+)>:$")
    mangled = [(i, m.group(1)) for i, line in enumerate(dis) for m in [sym.match(line)] if m]
    filt = shutil.which("c++filt") or os.path.join(LLVM, "llvm-cxxfilt")
    dem = subprocess.run([filt], input="\n".join(n for _, n in mangled), capture_output=True, text=True,
                         check=True).stdout.splitlines()
    for k, ((i, _), dm) in enumerate(zip(mangled, dem)):
        if dm.startswith(name_prefix):
            end = mangled[k + 1][0] if k + 1 < len(mangled) else len(dis)
            return dis[i:end]
    raise KeyError(name_prefix)


def main(argv):
    lib = next((a for a in argv if a.endswith(".so")), LIB)
    flt = argv[argv.index("--filter") + 1] if "--filter" in argv else ""
    res = kernel_resources(lib)
    for name in sorted(res):
        if flt and flt not in name:
            continue
        r = res[name]
        print("%-4s v%-3d a%-3d s%-3d spill v%d s%d scratch %-5d lds %-6d %s" % (
            "!!" if r.get("private_segment_fixed_size") else "", r.get("vgpr_count", 0), r.get("agpr_count", 0),
            r.get("sgpr_count", 0), r.get("vgpr_spill_count", 0), r.get("sgpr_spill_count", 0),
            r.get("private_segment_fixed_size", 0), r.get("group_segment_fixed_size", 0), name))


if __name__ == "__main__":
    main(sys.argv[1:])
