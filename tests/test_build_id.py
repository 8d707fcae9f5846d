"""mcs_build_id identifies the CODE of the embedded gfx950 objects, not their file bytes: a rebuild
of the same sources at another path keeps the id (so roofline.traffic stays attached to the
counters taken on that code), a change of the generated code changes it."""
import os
import shutil
import subprocess

import pytest

from multicamera_stitching_amd import build

HIPCC = build.HIPCC

SRC = r"""
#include <hip/hip_runtime.h>
#ifndef STORE_NT
#define STORE_NT 1
#endif
extern "C" __global__ void probe(const unsigned *a, unsigned *b, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
#if STORE_NT
        __builtin_nontemporal_store(a[i] * 3u + 1u, &b[i]);
#else
        b[i] = a[i] * 3u + 1u;
#endif
    }
}
"""


def _compile(tmp, name, defines=()):
    src = os.path.join(tmp, "probe.hip")
    with open(src, "w") as f:
        f.write(SRC)
    out = os.path.join(tmp, name)
    subprocess.check_call([HIPCC, *build.DEVICE_FLAGS, *["-D" + d for d in defines], "-o", out,
                           src])
    return out


@pytest.mark.skipif(shutil.which(HIPCC) is None and not os.path.exists(HIPCC),
                    reason="hipcc not present")
def test_code_id_is_path_independent(tmp_path):
    a = _compile(str(tmp_path), "first.hsaco")
    os.makedirs(tmp_path / "elsewhere")
    b = _compile(str(tmp_path / "elsewhere"), "a_much_longer_output_name.gfx950.hsaco")
    c = _compile(str(tmp_path), "plain_store.hsaco", defines=["STORE_NT=0"])
    with open(a, "rb") as fa, open(b, "rb") as fb:
        same_bytes = fa.read() == fb.read()
    # (the file bytes differ with the output name; the id must not)
    assert build.code_id([a]) == build.code_id([b]), "same code, different path: ids differ"
    assert build.code_id([a]) != build.code_id([c]), "different code, same id"
    assert isinstance(same_bytes, bool)


def test_embedded_id_matches_in_tree_objects():
    """The id libmcs.so reports is code_id() of the code objects built beside it."""
    here = os.path.dirname(build.LIB)
    objs = [os.path.join(here, f"mcs_{n}.{build.ARCH}.hsaco")
            for n in ("features", "kernels", "sweep")]
    if not all(os.path.exists(p) for p in objs) or not os.path.exists(build.LIB):
        pytest.skip("library not built")
    with open(build.LIB, "rb") as f:
        lib = f.read()
    want = build.code_id(objs)   # sorted by name: features, stitch (= mcs_kernels), sweep
    assert want.encode() in lib, f"libmcs.so does not embed build id {want}"
