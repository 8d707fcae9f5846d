"""Builds libmcs.so in-tree.

Two steps:
  1. hipcc compiles each device source device-only for gfx950 into a code object
     (csrc/mcs_kernels.hip: the stitch path; csrc/mcs_features.hip: matching/estimation);
  2. g++ compiles the host side (plan builder, HIP runtime binding, C ABI) and embeds those code
     objects (.incbin) into libmcs.so.  libmcs links no HIP runtime: it binds to the one the process
     already has (PyTorch's) or to ROCm's (csrc/hip_rt.h explains why).

The library is the product path: the Python drop-in refuses to run without it.
Usage: python -m multicamera_stitching_amd.build [--force]
"""
from __future__ import annotations

import hashlib
import os
import struct
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmcs.so")
ARCH = os.environ.get("MCS_OFFLOAD_ARCH", "gfx950")
# device sources -> embedded code objects (blob symbol mcs_hsaco_<name>_start)
DEVICE = {"stitch": "mcs_kernels.hip", "features": "mcs_features.hip", "sweep": "mcs_sweep.hip"}
HSACO = os.path.join(HERE, f"mcs_kernels.{ARCH}.hsaco")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.environ.get("HIPCC", os.path.join(ROCM, "bin", "hipcc"))
CXX = os.environ.get("CXX", "g++")
HOST_SRC = ["mcs_plan.cpp", "hip_rt.cpp", "mcs_runtime.cpp", "mcs_capi.cpp", "mcs_features.cpp",
            "mcs_stream.cpp", "mcs_seam.cpp", "mcs_refine.cpp", "mcs_group.cpp", "mcs_rig.cpp",
            "mcs_chain.cpp"]
HEADERS = ["mcs_kparams.h", "mcs_dev.h", "mcs_fparams.h", "mcs_common.h", "hip_rt.h", "mcs_blend.h", "mcs_ransac_core.h",
           "mcs_orb_core.h", "mcs_orb_pattern.h", "mcs_feat_int.h"]
INC = ["-I" + os.path.join(ROOT, "include"), "-I" + CSRC]

DEVICE_FLAGS = [
    f"--offload-arch={ARCH}", "--offload-device-only", "--no-gpu-bundle-output",
    "-O3", "-std=c++17",
    # bit-exact OpenCV arithmetic: no FMA contraction of the FP64 coordinate map
    "-ffp-contract=off", "-fno-fast-math", "-Wall",
]
HOST_FLAGS = [
    "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra", "-Wno-unused-parameter",
    # cv::invert must be bit-identical: no FMA contraction on the host either
    "-ffp-contract=off", "-fno-fast-math",
    "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(ROCM, "include"),
]


def _elf_sections(path: str) -> dict:
    """{name: bytes} of an ELF64 little-endian file's sections (NOBITS sections: b"")."""
    with open(path, "rb") as f:
        b = f.read()
    if b[:4] != b"\x7fELF" or b[4] != 2 or b[5] != 1:
        raise ValueError(f"{path}: not an ELF64 little-endian object")
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    names = hdrs[shstrndx]
    strtab = b[names[4]:names[4] + names[5]]
    out = {}
    for h in hdrs:
        name = strtab[h[0]:strtab.index(b"\0", h[0])].decode()
        out[name] = b"" if h[1] == 8 else b[h[4]:h[4] + h[5]]
    return out


# The sections that define what runs: machine code, kernel descriptors (.rodata) and the kernel
# metadata note (names, argument layout, register and LDS counts).  The symbol/string tables are
# left out: they carry names derived from the output path, so a rebuild of the same sources at
# another path keeps its id.
CODE_SECTIONS = (".text", ".rodata", ".note")


def code_id(paths) -> str:
    """16-hex build id of code objects, from their code sections only (see CODE_SECTIONS)."""
    digest = hashlib.sha256()
    for p in paths:
        secs = _elf_sections(p)
        for name in CODE_SECTIONS:
            data = secs.get(name, b"")
            digest.update(name.encode() + struct.pack("<Q", len(data)) + data)
    return digest.hexdigest()[:16]


def _stale() -> bool:
    if not (os.path.exists(LIB) and os.path.exists(HSACO)):
        return True
    t = os.path.getmtime(LIB)   # (each code object is checked against its own sources: _fresh)
    deps = [os.path.join(CSRC, s) for s in [*DEVICE.values(), *HOST_SRC, *HEADERS]]
    deps += [os.path.join(ROOT, "include", "mcs.h"), __file__]
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build(force: bool = False, verbose: bool = False, lib: str = None, defines=()) -> str:
    """Builds libmcs.so (or, for kernel experiments, a variant at `lib` with extra -D defines)."""
    if lib is not None:
        return _build_to(lib, HSACO + "." + os.path.basename(lib), list(defines), verbose)
    if not force and not _stale():
        return LIB
    return _build_to(LIB, HSACO, [], verbose)


def _fresh(out: str, src: str) -> bool:
    """out is newer than its device source and every header (incremental main builds)"""
    if not os.path.exists(out):
        return False
    deps = [os.path.join(CSRC, src)] + [os.path.join(CSRC, h) for h in HEADERS]
    deps += [os.path.join(ROOT, "include", "mcs.h"), __file__]
    return all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps)


def _build_to(LIB: str, HSACO: str, defines, verbose: bool) -> str:
    objs = {}
    for name, src in DEVICE.items():
        out = HSACO if name == "stitch" else HSACO.replace("mcs_kernels", "mcs_" + name)
        if defines or not _fresh(out, src):
            _run([HIPCC, *DEVICE_FLAGS, *["-D" + d for d in defines], *INC, "-o", out + ".tmp",
                  os.path.join(CSRC, src)], verbose)
            os.replace(out + ".tmp", out)
        objs[name] = out
    build_id = code_id([objs[name] for name in sorted(objs)])
    blob = LIB + ".blob.S"
    with open(blob, "w") as f:
        f.write("    .section .rodata\n")
        for name, path in objs.items():
            f.write('    .balign 4096\n    .globl mcs_hsaco_%s_start\nmcs_hsaco_%s_start:\n'
                    '    .incbin "%s"\n    .byte 0\n' % (name, name, path))
        f.write('    .section .note.GNU-stack,"",@progbits\n')
    try:
        _run([CXX, *HOST_FLAGS, *["-D" + d for d in defines], f'-DMCS_BUILD_ID="{build_id}"',
              *INC, "-o", LIB + ".tmp",
              *[os.path.join(CSRC, s) for s in HOST_SRC], blob, "-ldl", "-lpthread"], verbose)
    finally:
        os.remove(blob)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
