"""The C-ABI library: loads without a GPU, exports every symbol include/mcs.h declares, embeds the
gfx950 code object, links no HIP runtime, and validates plans on the host."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from multicamera_stitching_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mcs.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mcs_[a-z_0-9]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_functions() == sorted(_capi.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = _capi.load()
    for name in declared_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for name in declared_functions():
        assert re.search(r"\bT %s\b" % name, out), name


def test_no_hip_runtime_linked_and_code_object_embedded():
    out = subprocess.run(["readelf", "-d", _capi.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert "amdhip64" not in out          # bound at run time (csrc/hip_rt.h)
    blob = open(_capi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for k in (b"mcs_stream_c3", b"mcs_prepare_c3_i1", b"mcs_direct_c3_i1_o32", b"mcs_resize_c3",
              b"mcs_hamming_knn2"):
        assert k in blob
    assert blob.count(b"amdgcn-amd-amdhsa--gfx950") >= 2   # stitch + features code objects


def test_version_and_abi():
    L = _capi.load()
    assert L.mcs_abi_version() == _capi.ABI_VERSION
    assert b"gfx950" in L.mcs_version()


def _desc(**kw):
    d = _capi.StageDesc()
    d.H[:] = [1, 0, 10, 0, 1, 0, 0, 0, 1]
    d.calibrated = 1
    d.canvas_w, d.canvas_h = 74, 48
    d.b_x, d.b_y, d.b_w, d.b_h = 0, 0, 64, 48
    d.a_w, d.a_h = 64, 48
    for k, v in kw.items():
        setattr(d, k, v)
    return d


def test_plan_create_host_only_and_describe():
    p = _capi.Plan([_desc()], 64, 48, 3)
    assert p.out_shape() == (48, 74, 3)
    fl = p.describe()
    assert fl["n_stages"] == 1 and fl["rect"] == [[0, 0, 64, 48]] and fl["bw0"] == [64]
    assert fl["minv"][0] == [1.0, -0.0, -10.0, 0.0, 1.0, -0.0, 0.0, -0.0, 1.0]
    p.close()


@pytest.mark.parametrize("kw,code", [
    ({"b_w": 60}, _capi.MCS_E_SHAPE),              # B size differs from the chain (resize)
    ({"b_x": 20}, _capi.MCS_E_SHAPE),              # paste would overflow the canvas
    ({"canvas_w": 0}, _capi.MCS_E_SHAPE),
    ({"a_w": 0}, _capi.MCS_E_SHAPE),
])
def test_plan_create_rejects_inconsistent_geometry(kw, code):
    with pytest.raises(_capi.McsError) as e:
        _capi.Plan([_desc(**kw)], 64, 48, 3)
    assert e.value.code == code
    assert _capi.load().mcs_last_error()


def test_plan_create_rejects_unsupported():
    with pytest.raises(_capi.McsError) as e:
        _capi.Plan([_desc()], 64, 48, 5)
    assert e.value.code == _capi.MCS_E_UNSUPPORTED
    with pytest.raises(_capi.McsError) as e:
        _capi.Plan([_desc()] * 16, 64, 48, 3)
    assert e.value.code == _capi.MCS_E_UNSUPPORTED


def test_null_arguments_return_status_not_crash():
    L = _capi.load()
    assert L.mcs_plan_create(None, 1, 1, 1, 3, 1, 0, None) == _capi.MCS_E_INVALID
    assert L.mcs_stitch_host(None, None, None) == _capi.MCS_E_INVALID
    assert L.mcs_plan_destroy(None) == _capi.MCS_OK


def test_passthrough_stages_flatten_away():
    un = _capi.StageDesc()
    un.calibrated = 0
    un.a_w, un.a_h = 64, 48
    p = _capi.Plan([un, _desc()], 64, 48, 1)
    fl = p.describe()
    assert fl["n_stages"] == 1 and fl["cam"] == [2]
    p2 = _capi.Plan([un], 64, 48, 1)
    assert p2.out_shape() == (48, 64)


def test_rig_job_host_validation():
    """mcs_rig_job: creation touches no GPU; bad shapes and a wait with nothing submitted are
    status codes, not crashes."""
    L = _capi.load()
    j = _capi.RigJob(4, 640, 480, 3)
    with pytest.raises(_capi.McsError) as e:
        j.wait()
    assert e.value.code == _capi.MCS_E_INVALID
    j.close()
    for bad in ({"n_cams": 1}, {"channels": 2}, {"nfeatures": 0}, {"iters": 0}):
        kw = dict(n_cams=4, w=640, h=480, channels=3)
        kw.update(bad)
        with pytest.raises(_capi.McsError) as e:
            _capi.RigJob(**kw)
        assert e.value.code == _capi.MCS_E_INVALID
    assert L.mcs_rig_job_submit(None, None, None) == _capi.MCS_E_INVALID
    assert L.mcs_rig_job_destroy(None) == _capi.MCS_OK
