"""Builds a kernel-experiment variant of libmcs.so: variants/<name>.so with extra -D defines.

    python tools/build_variant.py <name> [DEFINE[=VALUE] ...]

Variants are timing experiments only (tools/gpu_var_bench.sh runs bench lines with
MCS_LIBRARY=variants/<name>.so); the product library is multicamera_stitching_amd/libmcs.so.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from multicamera_stitching_amd import build  # noqa: E402

if __name__ == "__main__":
    name, defines = sys.argv[1], sys.argv[2:]
    os.makedirs(os.path.join(ROOT, "variants"), exist_ok=True)
    print(build.build(lib=os.path.join(ROOT, "variants", name + ".so"), defines=defines))
