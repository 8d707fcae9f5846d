"""Builds a kernel-experiment variant of libmcs.so: variants/<name>.so with extra -D defines,
optionally from the sources with patches applied.

    python tools/build_variant.py <name> [--patch FILE ...] [DEFINE[=VALUE] ...]

Variants are timing experiments only (tools/gpu_var_bench.sh runs bench lines with
MCS_LIBRARY=variants/<name>.so); the product library is multicamera_stitching_amd/libmcs.so and
its sources carry only numeric tuning defaults (`#ifndef MCS_<knob>`), no experiment code paths.
The experiment forms removed from the product sources in round 6 (the round-4 streaming loop,
row-job DMA, the decomposition hooks, the band-pass / blend phase skips, the band diagnostics,
the serial multi-band launch) are kept as tools/variant_patches/r05_experiments.patch: with
`--patch` the sources are copied to a scratch directory, patched (`patch -p1` from the repo
root) and built from there.
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from multicamera_stitching_amd import build  # noqa: E402


def main(argv):
    name, rest = argv[0], argv[1:]
    patches, defines = [], []
    while rest:
        a = rest.pop(0)
        if a == "--patch":
            patches.append(os.path.abspath(rest.pop(0)))
        else:
            defines.append(a)
    os.makedirs(os.path.join(ROOT, "variants"), exist_ok=True)
    lib = os.path.join(ROOT, "variants", name + ".so")
    if not patches:
        return build.build(lib=lib, defines=defines)
    with tempfile.TemporaryDirectory() as tmp:
        rel = os.path.relpath(build.CSRC, ROOT)
        shutil.copytree(build.CSRC, os.path.join(tmp, rel))
        for p in patches:
            subprocess.check_call(["patch", "-s", "-p1", "-d", tmp, "-i", p])
        csrc = os.path.join(tmp, rel)
        build.CSRC = csrc
        build.INC = ["-I" + os.path.join(ROOT, "include"), "-I" + csrc]
        return build.build(lib=lib, defines=defines)


if __name__ == "__main__":
    print(main(sys.argv[1:]))
