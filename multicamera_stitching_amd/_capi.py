"""ctypes binding of libmcs.so (include/mcs.h).

This is the only route to pixels in the product path: there is no CPU fallback.  If the HIP
library is missing the import of the drop-in fails loudly with instructions to build it.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MCS_LIBRARY", os.path.join(_HERE, "libmcs.so"))

MCS_OK = 0
MCS_E_INVALID = -1
MCS_E_HIP = -2
MCS_E_NOMEM = -3
MCS_E_SHAPE = -4
MCS_E_UNSUPPORTED = -5
MCS_INTER_NEAREST = 0
MCS_INTER_LINEAR = 1
MCS_BLEND_NONE = 0
MCS_BLEND_FEATHER = 1
MCS_BLEND_MULTIBAND = 2
MCS_BLEND_SEAM = 3
MCS_SEAM_DISTANCE = 0
MCS_SEAM_GRAPHCUT = 1
MCS_MAX_STAGES = 15
MCS_MAX_CAMS = MCS_MAX_STAGES + 1
ABI_VERSION = 1

# every symbol include/mcs.h declares (checked by tests/test_capi_exports.py)
EXPORTS = (
    "mcs_version", "mcs_abi_version", "mcs_last_error", "mcs_device_count", "mcs_hip_runtime",
    "mcs_plan_create", "mcs_plan_destroy", "mcs_plan_out_shape", "mcs_plan_describe",
    "mcs_stitch_host", "mcs_stitch_device", "mcs_plan_footprint", "mcs_plan_prepare",
    "mcs_plan_stats", "mcs_stitch_host_sized", "mcs_resize_linear_device",
    "mcs_match_hamming_knn2", "mcs_match_hamming_knn2_host", "mcs_plan_set_blend",
    "mcs_ransac_homography_host", "mcs_stream_create", "mcs_stream_input", "mcs_stream_next_slot",
    "mcs_stream_copy_workers",
    "mcs_stream_submit", "mcs_stream_wait", "mcs_stream_destroy", "mcs_orb_detect_host",
    "mcs_plan_create_cylindrical", "mcs_plan_find_seams", "mcs_plan_seam_labels",
    "mcs_seam_graphcut_host", "mcs_plan_create_warp", "mcs_plan_create_undistort",
    "mcs_undistort_map_host", "mcs_match_l2_knn2", "mcs_match_l2_knn2_host",
    "mcs_stream_submit_strided", "mcs_build_id", "mcs_homography_refine_host", "mcs_stream_output",
    "mcs_stitch_direct", "mcs_orb_detect_device", "mcs_group_unique_id", "mcs_group_create",
    "mcs_group_gather", "mcs_group_destroy", "mcs_rccl_library", "mcs_rig_job_create",
    "mcs_rig_job_submit", "mcs_rig_job_wait", "mcs_rig_job_counts", "mcs_rig_job_destroy",
    "mcs_seam_graphcut_device", "mcs_plan_seam_stats", "mcs_chain_stages",
    "mcs_rig_job_wait_stitch", "mcs_rig_job_create_batch", "mcs_rig_job_wait_stitch_batch",
)
MCS_GROUP_ID_BYTES = 128


class McsError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libmcs error {code}: {msg}")
        self.code = code


class StageDesc(ctypes.Structure):
    _fields_ = [
        ("H", ctypes.c_double * 9),
        ("calibrated", ctypes.c_int),
        ("canvas_w", ctypes.c_int),
        ("canvas_h", ctypes.c_int),
        ("b_x", ctypes.c_int),
        ("b_y", ctypes.c_int),
        ("b_w", ctypes.c_int),
        ("b_h", ctypes.c_int),
        ("a_w", ctypes.c_int),
        ("a_h", ctypes.c_int),
        ("super_mode", ctypes.c_int),
        ("x_lim0", ctypes.c_int),
        ("x_lim1", ctypes.c_int),
        ("y_lim0", ctypes.c_int),
        ("y_lim1", ctypes.c_int),
    ]


class FlatStage(ctypes.Structure):
    _fields_ = [
        ("minv", ctypes.c_double * 9),
        ("rect", ctypes.c_int * 4),
        ("off_x", ctypes.c_int),
        ("off_y", ctypes.c_int),
        ("bw0", ctypes.c_int),
        ("cam", ctypes.c_int),
    ]


class FlatDesc(ctypes.Structure):
    _fields_ = [
        ("n_stages", ctypes.c_int),
        ("out_w", ctypes.c_int),
        ("out_h", ctypes.c_int),
        ("channels", ctypes.c_int),
        ("interp", ctypes.c_int),
        ("cam0_off_x", ctypes.c_int),
        ("cam0_off_y", ctypes.c_int),
        ("n_cams", ctypes.c_int),
        ("cam_w", ctypes.c_int * MCS_MAX_CAMS),
        ("cam_h", ctypes.c_int * MCS_MAX_CAMS),
        ("st", FlatStage * MCS_MAX_STAGES),
    ]


_lib = None
_lib_lock = threading.Lock()


def _preload_hip_runtime():
    """Make sure the process will hold ONE HIP runtime, shared with PyTorch when it is installed.

    libmcs links no HIP runtime; it binds to the libamdhip64 already in the process.  PyTorch-ROCm
    bundles its own (torch/lib/libamdhip64.so); a second runtime (ROCm's libamdhip64.so.7) in the
    same process fails to initialise.  So when torch is installed its runtime is loaded first
    (without importing torch); torch, if imported later, then reuses it.  $MCS_HIP_RUNTIME
    overrides the choice (handled inside libmcs).
    """
    if os.environ.get("MCS_HIP_RUNTIME"):
        return
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.submodule_search_locations:
        return
    for loc in spec.submodule_search_locations:
        cand = os.path.join(loc, "lib", "libamdhip64.so")
        if os.path.exists(cand):
            ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)
            return


def load() -> ctypes.CDLL:
    """Load libmcs.so once.  Raises ImportError (loudly) when it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libmcs.so not found at {LIB_PATH}: the MI355X stitch path has no CPU fallback. "
                "Build it with `python -m multicamera_stitching_amd.build` (hipcc, gfx950).")
        _preload_hip_runtime()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        I = ctypes.c_int
        L.mcs_version.restype = ctypes.c_char_p
        L.mcs_version.argtypes = []
        L.mcs_abi_version.restype = I
        L.mcs_abi_version.argtypes = []
        L.mcs_build_id.restype = ctypes.c_char_p
        L.mcs_build_id.argtypes = []
        L.mcs_hip_runtime.restype = ctypes.c_char_p
        L.mcs_hip_runtime.argtypes = []
        L.mcs_last_error.restype = ctypes.c_char_p
        L.mcs_last_error.argtypes = []
        L.mcs_device_count.argtypes = [ctypes.POINTER(I)]
        L.mcs_device_count.restype = I
        L.mcs_plan_create.argtypes = [ctypes.POINTER(StageDesc), I, I, I, I, I, I,
                                      ctypes.POINTER(P)]
        L.mcs_plan_create.restype = I
        L.mcs_plan_destroy.argtypes = [P]
        L.mcs_plan_destroy.restype = I
        L.mcs_plan_out_shape.argtypes = [P, ctypes.POINTER(I), ctypes.POINTER(I),
                                         ctypes.POINTER(I)]
        L.mcs_plan_out_shape.restype = I
        L.mcs_plan_describe.argtypes = [P, ctypes.POINTER(FlatDesc)]
        L.mcs_plan_describe.restype = I
        L.mcs_stitch_host.argtypes = [P, ctypes.POINTER(P), P]
        L.mcs_stitch_host.restype = I
        L.mcs_stitch_host_sized.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(I),
                                            ctypes.POINTER(I), P]
        L.mcs_stitch_host_sized.restype = I
        i64 = ctypes.c_int64
        L.mcs_resize_linear_device.argtypes = [P, I, I, i64, i64, P, I, I, i64, i64, I, I, I, P]
        L.mcs_resize_linear_device.restype = I
        L.mcs_ransac_homography_host.argtypes = [P, P, I, ctypes.c_double, I, ctypes.c_uint32,
                                                 P, P, ctypes.POINTER(I), I]
        L.mcs_ransac_homography_host.restype = I
        L.mcs_homography_refine_host.argtypes = [P, P, I, P, P]
        L.mcs_homography_refine_host.restype = I
        L.mcs_stream_create.argtypes = [P, I, I, ctypes.POINTER(P)]
        L.mcs_stream_create.restype = I
        L.mcs_stream_copy_workers.argtypes = []
        L.mcs_stream_copy_workers.restype = I
        L.mcs_stream_input.argtypes = [P, I, I]
        L.mcs_stream_input.restype = P
        L.mcs_stream_output.argtypes = [P, I]
        L.mcs_stream_output.restype = P
        L.mcs_stream_next_slot.argtypes = [P]
        L.mcs_stream_next_slot.restype = I
        L.mcs_stream_submit.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(I)]
        L.mcs_stream_submit.restype = I
        L.mcs_stream_submit_strided.argtypes = [P, ctypes.POINTER(P), P, ctypes.POINTER(I)]
        L.mcs_stream_submit_strided.restype = I
        L.mcs_stream_wait.argtypes = [P, I, P]
        L.mcs_stream_wait.restype = I
        L.mcs_stream_destroy.argtypes = [P]
        L.mcs_stream_destroy.restype = I
        L.mcs_orb_detect_host.argtypes = [P, I, I, I, I, I, ctypes.c_float, I, P, P, P, P, P,
                                          ctypes.POINTER(I), I]
        L.mcs_orb_detect_host.restype = I
        L.mcs_orb_detect_device.argtypes = L.mcs_orb_detect_host.argtypes
        L.mcs_orb_detect_device.restype = I
        L.mcs_rig_job_create.argtypes = [I, I, I, I, I, I, ctypes.c_float, I, ctypes.c_float,
                                         ctypes.c_double, I, ctypes.c_uint32, I,
                                         ctypes.POINTER(P)]
        L.mcs_rig_job_create.restype = I
        L.mcs_rig_job_create_batch.argtypes = [I] + L.mcs_rig_job_create.argtypes
        L.mcs_rig_job_create_batch.restype = I
        L.mcs_rig_job_submit.argtypes = [P, P, P]
        L.mcs_rig_job_submit.restype = I
        L.mcs_rig_job_wait.argtypes = [P, P, P, P, P, P]
        L.mcs_rig_job_wait.restype = I
        L.mcs_rig_job_wait_stitch.argtypes = [P, P, P, I, I, P, ctypes.c_int64, ctypes.c_int64,
                                              P, P, P, P, P, P]
        L.mcs_rig_job_wait_stitch.restype = I
        L.mcs_rig_job_wait_stitch_batch.argtypes = L.mcs_rig_job_wait_stitch.argtypes
        L.mcs_rig_job_wait_stitch_batch.restype = I
        L.mcs_chain_stages.argtypes = [I, P, P, P, P, I, ctypes.POINTER(StageDesc)]
        L.mcs_chain_stages.restype = I
        L.mcs_seam_graphcut_device.argtypes = [I, I, I, P, P, P, I, I, P]
        L.mcs_seam_graphcut_device.restype = I
        L.mcs_plan_seam_stats.argtypes = [P, P]
        L.mcs_plan_seam_stats.restype = I
        L.mcs_rig_job_counts.argtypes = [P, P, P]
        L.mcs_rig_job_counts.restype = I
        L.mcs_rig_job_destroy.argtypes = [P]
        L.mcs_rig_job_destroy.restype = I
        L.mcs_plan_set_blend.argtypes = [P, I]
        L.mcs_plan_create_cylindrical.argtypes = [ctypes.POINTER(CylCamera), I, I, I,
                                                  ctypes.c_double, ctypes.c_double,
                                                  ctypes.c_double, I, I, I, ctypes.POINTER(P)]
        L.mcs_plan_create_cylindrical.restype = I
        L.mcs_plan_find_seams.argtypes = [P, P, I, I]
        L.mcs_plan_find_seams.restype = I
        L.mcs_plan_seam_labels.argtypes = [P, P, ctypes.POINTER(I), ctypes.POINTER(I)]
        L.mcs_plan_seam_labels.restype = I
        L.mcs_seam_graphcut_host.argtypes = [I, I, I, P, P, P, I]
        L.mcs_seam_graphcut_host.restype = I
        L.mcs_plan_create_warp.argtypes = [P, I, I, I, I, I, I, I, ctypes.POINTER(P)]
        L.mcs_plan_create_warp.restype = I
        L.mcs_plan_create_undistort.argtypes = [P, P, I, I, I, I, I, ctypes.POINTER(P)]
        L.mcs_plan_create_undistort.restype = I
        L.mcs_undistort_map_host.argtypes = [P, P, I, I, I, P]
        L.mcs_undistort_map_host.restype = I
        L.mcs_match_l2_knn2.argtypes = [P, I, P, I, I, P, P, P, I, P]
        L.mcs_match_l2_knn2.restype = I
        L.mcs_match_l2_knn2_host.argtypes = [P, I, P, I, I, P, P, P, I]
        L.mcs_match_l2_knn2_host.restype = I
        L.mcs_plan_set_blend.restype = I
        L.mcs_match_hamming_knn2.argtypes = [P, I, P, I, P, P, I, P]
        L.mcs_match_hamming_knn2.restype = I
        L.mcs_match_hamming_knn2_host.argtypes = [P, I, P, I, P, P, I]
        L.mcs_match_hamming_knn2_host.restype = I
        L.mcs_stitch_device.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_int64), P,
                                        ctypes.c_int64, ctypes.c_int64, I, P]
        L.mcs_stitch_device.restype = I
        L.mcs_stitch_direct.argtypes = L.mcs_stitch_device.argtypes
        L.mcs_stitch_direct.restype = I
        L.mcs_group_unique_id.argtypes = [P]
        L.mcs_group_unique_id.restype = I
        L.mcs_group_create.argtypes = [I, I, P, I, ctypes.POINTER(P)]
        L.mcs_group_create.restype = I
        L.mcs_group_gather.argtypes = [P, P, ctypes.c_int64, P, I, P]
        L.mcs_group_gather.restype = I
        L.mcs_group_destroy.argtypes = [P]
        L.mcs_group_destroy.restype = I
        L.mcs_rccl_library.argtypes = []
        L.mcs_rccl_library.restype = ctypes.c_char_p
        L.mcs_plan_prepare.argtypes = [P, P]
        L.mcs_plan_prepare.restype = I
        L.mcs_plan_stats.argtypes = [P, ctypes.POINTER(ctypes.c_int64), I]
        L.mcs_plan_stats.restype = I
        L.mcs_plan_footprint.argtypes = [P, ctypes.POINTER(ctypes.c_int64), I]
        L.mcs_plan_footprint.restype = I
        L.mcs__force_off64.argtypes = [I]   # test hook (not part of mcs.h)
        L.mcs__force_off64.restype = None
        if L.mcs_abi_version() != ABI_VERSION:
            raise ImportError(f"libmcs ABI {L.mcs_abi_version()} != expected {ABI_VERSION}")
        _lib = L
    return _lib


def check(rc: int):
    if rc != MCS_OK:
        msg = load().mcs_last_error()
        raise McsError(rc, msg.decode() if msg else "")


def build_id() -> str:
    """SHA-256 prefix of the embedded gfx950 code objects (mcs_build_id)."""
    return load().mcs_build_id().decode()


def hip_runtime() -> str:
    return load().mcs_hip_runtime().decode()


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = load().mcs_device_count(ctypes.byref(n))
    return n.value if rc == MCS_OK else 0


class CylCamera(ctypes.Structure):
    """include/mcs.h mcs_cyl_camera: rig -> camera rotation R (row-major), f, cx, cy, w, h."""
    _fields_ = [
        ("R", ctypes.c_double * 9),
        ("f", ctypes.c_double),
        ("cx", ctypes.c_double),
        ("cy", ctypes.c_double),
        ("w", ctypes.c_int),
        ("h", ctypes.c_int),
    ]


class Plan:
    """Owning handle of an mcs_plan (flattened geometry of one calibrated chain, or of a
    cylindrical rig: Plan.cylindrical)."""

    def __init__(self, stages, cam0_w: int, cam0_h: int, channels: int,
                 interp: int = MCS_INTER_LINEAR, device: int = 0, _handle=None):
        L = load()
        if _handle is None:
            arr = (StageDesc * max(1, len(stages)))()
            for i, s in enumerate(stages):
                arr[i] = s
            h = ctypes.c_void_p()
            check(L.mcs_plan_create(arr, len(stages), int(cam0_w), int(cam0_h), int(channels),
                                    int(interp), int(device), ctypes.byref(h)))
        else:
            h = _handle
        self._h = h
        self._lib = L
        w, hh, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(L.mcs_plan_out_shape(h, ctypes.byref(w), ctypes.byref(hh), ctypes.byref(c)))
        self.out_w, self.out_h, self.channels = w.value, hh.value, c.value
        self.interp = int(interp)
        self.device = int(device)
        fd = FlatDesc()
        check(L.mcs_plan_describe(h, ctypes.byref(fd)))
        self.flat = fd
        self.n_cams = fd.n_cams
        self.cam_shapes = [(fd.cam_h[i], fd.cam_w[i]) for i in range(fd.n_cams)]

    @classmethod
    def cylindrical(cls, cams, out_w: int, out_h: int, f_cyl: float, u0: float, v0: float,
                    channels: int, interp: int = MCS_INTER_LINEAR, device: int = 0):
        """mcs_plan_create_cylindrical: cams = [dict(R=3x3, f=, cx=, cy=, w=, h=)]; the plan
        blends with MCS_BLEND_MULTIBAND until set_blend changes it."""
        L = load()
        arr = (CylCamera * max(1, len(cams)))()
        for i, c in enumerate(cams):
            arr[i].R = (ctypes.c_double * 9)(*[float(v) for v in
                                               np.asarray(c["R"], np.float64).reshape(9)])
            arr[i].f, arr[i].cx, arr[i].cy = float(c["f"]), float(c["cx"]), float(c["cy"])
            arr[i].w, arr[i].h = int(c["w"]), int(c["h"])
        h = ctypes.c_void_p()
        check(L.mcs_plan_create_cylindrical(arr, len(cams), int(out_w), int(out_h),
                                            ctypes.c_double(f_cyl), ctypes.c_double(u0),
                                            ctypes.c_double(v0), int(channels), int(interp),
                                            int(device), ctypes.byref(h)))
        return cls(None, 0, 0, channels, interp, device, _handle=h)

    @classmethod
    def warp(cls, M, src_w: int, src_h: int, dst_w: int, dst_h: int, channels: int,
             interp: int = MCS_INTER_LINEAR, device: int = 0):
        """mcs_plan_create_warp: cv2.warpPerspective(src, M, (dst_w, dst_h)) as a plan."""
        L = load()
        m = np.ascontiguousarray(np.asarray(M, np.float64).reshape(9))
        h = ctypes.c_void_p()
        check(L.mcs_plan_create_warp(m.ctypes.data_as(ctypes.c_void_p), int(src_w), int(src_h),
                                     int(dst_w), int(dst_h), int(channels), int(interp),
                                     int(device), ctypes.byref(h)))
        return cls(None, 0, 0, channels, interp, device, _handle=h)

    @classmethod
    def undistort(cls, K, dist, w: int, h: int, channels: int, device: int = 0):
        """mcs_plan_create_undistort: cv2.undistort(src, K, dist) as a plan."""
        L = load()
        k = np.ascontiguousarray(np.asarray(K, np.float64).reshape(9))
        d = np.ascontiguousarray(np.asarray(dist if dist is not None else [], np.float64)
                                 .reshape(-1))
        hd = ctypes.c_void_p()
        check(L.mcs_plan_create_undistort(k.ctypes.data_as(ctypes.c_void_p),
                                          d.ctypes.data_as(ctypes.c_void_p) if d.size else None,
                                          int(d.size), int(w), int(h), int(channels),
                                          int(device), ctypes.byref(hd)))
        return cls(None, 0, 0, channels, MCS_INTER_LINEAR, device, _handle=hd)

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.mcs_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def out_shape(self):
        if self.channels == 1:
            return (self.out_h, self.out_w)
        return (self.out_h, self.out_w, self.channels)

    def describe(self) -> dict:
        fd = self.flat
        n = fd.n_stages
        return {
            "n_stages": n,
            "out_w": fd.out_w, "out_h": fd.out_h, "channels": fd.channels,
            "off_x": [fd.st[j].off_x for j in range(n)] + [fd.cam0_off_x],
            "off_y": [fd.st[j].off_y for j in range(n)] + [fd.cam0_off_y],
            "rect": [list(fd.st[j].rect) for j in range(n)],
            "minv": [list(fd.st[j].minv) for j in range(n)],
            "bw0": [fd.st[j].bw0 for j in range(n)],
            "cam": [fd.st[j].cam for j in range(n)],
            "cam_w": [fd.cam_w[i] for i in range(fd.n_cams)],
            "cam_h": [fd.cam_h[i] for i in range(fd.n_cams)],
        }

    def stitch_host(self, cams, sizes=None) -> np.ndarray:
        """cams: dense u8 arrays in sorted-label order.  sizes: their (w, h) when some differ
        from the calibrated ones (those are resized on the device first, :226-233)."""
        cams = [np.ascontiguousarray(c, dtype=np.uint8) for c in cams]
        out = np.empty(self.out_shape(), np.uint8)
        ptrs = (ctypes.c_void_p * len(cams))(*[c.ctypes.data for c in cams])
        outp = out.ctypes.data_as(ctypes.c_void_p)
        fd = self.flat
        if sizes is None or all((w, h) == (fd.cam_w[i], fd.cam_h[i])
                                for i, (w, h) in enumerate(sizes)):
            check(self._lib.mcs_stitch_host(self._h, ptrs, outp))
        else:
            ws = (ctypes.c_int * len(sizes))(*[int(w) for w, _ in sizes])
            hs = (ctypes.c_int * len(sizes))(*[int(h) for _, h in sizes])
            check(self._lib.mcs_stitch_host_sized(self._h, ptrs, ws, hs, outp))
        return out

    def find_seams(self, cams=None, method: int = MCS_SEAM_GRAPHCUT, scale_log2: int = 2):
        """mcs_plan_find_seams: graph-cut seams from one capture (host frames, calibrated
        sizes), or back to distance seams (method=MCS_SEAM_DISTANCE)."""
        if cams is None:
            check(self._lib.mcs_plan_find_seams(self._h, None, int(method), int(scale_log2)))
            return
        cams = [np.ascontiguousarray(c, dtype=np.uint8) for c in cams]
        ptrs = (ctypes.c_void_p * len(cams))(*[c.ctypes.data for c in cams])
        check(self._lib.mcs_plan_find_seams(self._h, ptrs, int(method), int(scale_log2)))

    def seam_labels(self):
        """The graph-cut seam grid (camera per point, 255 = none), or None."""
        w, h = ctypes.c_int(), ctypes.c_int()
        check(self._lib.mcs_plan_seam_labels(self._h, None, ctypes.byref(w), ctypes.byref(h)))
        if w.value == 0:
            return None
        out = np.empty((h.value, w.value), np.uint8)
        check(self._lib.mcs_plan_seam_labels(self._h, out.ctypes.data_as(ctypes.c_void_p),
                                             ctypes.byref(w), ctypes.byref(h)))
        return out

    def seam_stats(self):
        """The device max-flow's counts of the last find_seams: (pairs with a graph, push
        launches, relabel launches, global relabels, microseconds of the max-flows)."""
        st = np.zeros(5, np.int64)
        check(self._lib.mcs_plan_seam_stats(self._h, st.ctypes.data_as(ctypes.c_void_p)))
        return tuple(int(v) for v in st)

    def stitch_device(self, cam_ptrs, cam_frame_strides, out_ptr: int, out_pitch: int,
                      out_frame_stride: int, n_frames: int, stream: int = 0):
        """Device-resident batch (raw device pointers, e.g. torch tensor data_ptr())."""
        n = len(cam_ptrs)
        ptrs = (ctypes.c_void_p * n)(*[int(p) for p in cam_ptrs])
        strides = (ctypes.c_int64 * n)(*[int(s) for s in cam_frame_strides])
        check(self._lib.mcs_stitch_device(self._h, ptrs, strides, ctypes.c_void_p(int(out_ptr)),
                                          int(out_pitch), int(out_frame_stride), int(n_frames),
                                          ctypes.c_void_p(int(stream))))

    def stitch_direct(self, cam_ptrs, cam_frame_strides, out_ptr: int, out_pitch: int,
                      out_frame_stride: int, n_frames: int, stream: int = 0):
        """mcs_stitch_direct: the same pixels as stitch_device without prepared tables (the
        exact map evaluated per pixel in the kernel) -- for a plan built for one capture, e.g.
        from per-frame homographies.  Paste / seam plans."""
        n = len(cam_ptrs)
        ptrs = (ctypes.c_void_p * n)(*[int(p) for p in cam_ptrs])
        strides = (ctypes.c_int64 * n)(*[int(s) for s in cam_frame_strides])
        check(self._lib.mcs_stitch_direct(self._h, ptrs, strides, ctypes.c_void_p(int(out_ptr)),
                                          int(out_pitch), int(out_frame_stride), int(n_frames),
                                          ctypes.c_void_p(int(stream))))

    def prepare(self, stream: int = 0):
        """Evaluate and store the plan's map tables on its device (once)."""
        check(self._lib.mcs_plan_prepare(self._h, ctypes.c_void_p(int(stream))))

    def stats(self) -> dict:
        arr = (ctypes.c_int64 * 20)()
        check(self._lib.mcs_plan_stats(self._h, arr, 20))
        return {"prepared": bool(arr[0]), "tiles": arr[1], "lds_tiles": arr[2],
                "direct_tiles": arr[3], "table_bytes": arr[4], "blend": arr[5],
                "blend_tiles": arr[6], "mb_owners": arr[7], "mb_degraded_tiles": arr[8],
                "mb_bands": arr[9], "mb_bands_lds": arr[10], "big_tiles": arr[11],
                "mb_mixed_px": arr[12], "mb_r1_entries": arr[13],
                "dma_bytes_per_capture": arr[14], "box_bytes_per_capture": arr[15],
                "mb_sweep_strips": arr[16], "mb_sweep_px": arr[17],
                "mb_sweep_threads": arr[18], "mb_sweep_desc_rows": arr[19]}

    def set_blend(self, mode: int):
        """MCS_BLEND_NONE (reference paste), MCS_BLEND_FEATHER, MCS_BLEND_MULTIBAND or
        MCS_BLEND_SEAM (owner only)."""
        check(self._lib.mcs_plan_set_blend(self._h, int(mode)))
        return self

    def footprint(self):
        arr = (ctypes.c_int64 * MCS_MAX_CAMS)()
        check(self._lib.mcs_plan_footprint(self._h, arr, MCS_MAX_CAMS))
        return [int(arr[i]) for i in range(self.n_cams)]


def resize_linear_device(src_ptr: int, src_w: int, src_h: int, dst_ptr: int, dst_w: int,
                         dst_h: int, channels: int, n_frames: int = 1, src_pitch: int = 0,
                         dst_pitch: int = 0, src_frame_stride: int = 0,
                         dst_frame_stride: int = 0, device: int = 0, stream: int = 0):
    """cv2.resize(..., interpolation=INTER_LINEAR) of device-resident u8 images (mcs.h)."""
    L = load()
    check(L.mcs_resize_linear_device(
        src_ptr, src_w, src_h, src_pitch or src_w * channels, src_frame_stride, dst_ptr, dst_w,
        dst_h, dst_pitch or dst_w * channels, dst_frame_stride, channels, n_frames, device,
        stream or None))


def match_hamming_knn2(query, train, device: int = 0):
    """BFMatcher(NORM_HAMMING).knnMatch(query, train, k=2) on the GPU for host arrays of
    N x 32-byte descriptors: (idx (nq, 2), dist (nq, 2)) int32, -1 where no candidate."""
    L = load()
    q = np.ascontiguousarray(query, dtype=np.uint8).reshape(-1, 32)
    t = np.ascontiguousarray(train, dtype=np.uint8).reshape(-1, 32)
    idx = np.empty((q.shape[0], 2), np.int32)
    dist = np.empty((q.shape[0], 2), np.int32)
    check(L.mcs_match_hamming_knn2_host(q.ctypes.data, q.shape[0], t.ctypes.data, t.shape[0],
                                        idx.ctypes.data, dist.ctypes.data, device))
    return idx, dist


def match_hamming_knn2_device(q_ptr: int, nq: int, t_ptr: int, nt: int, idx_ptr: int,
                              dist_ptr: int, device: int = 0, stream: int = 0):
    """Device-pointer form (enqueued on `stream`)."""
    check(load().mcs_match_hamming_knn2(q_ptr, nq, t_ptr, nt, idx_ptr, dist_ptr, device,
                                        stream or None))


def homography_refine(src, dst, mask, H):
    """findHomography's post-RANSAC refinement (mcs_homography_refine_host, host FP64):
    normalised DLT on the inliers + 10 Levenberg-Marquardt iterations from the model H."""
    L = load()
    src = np.ascontiguousarray(src, np.float32).reshape(-1, 2)
    dst = np.ascontiguousarray(dst, np.float32).reshape(-1, 2)
    m = np.ascontiguousarray(np.asarray(mask).reshape(-1), np.uint8)
    h = np.ascontiguousarray(np.asarray(H, np.float64).reshape(9)).copy()
    check(L.mcs_homography_refine_host(src.ctypes.data, dst.ctypes.data, src.shape[0],
                                       m.ctypes.data, h.ctypes.data))
    return h.reshape(3, 3)


def ransac_homography(src, dst, thresh: float, iters: int = 2000, seed: int = 0,
                      device: int = 0):
    """RANSAC homography on the GPU (mcs.h): (H 3x3 or None, status mask (n, 1) uint8), the
    return shape of cv2.findHomography(src, dst, cv2.RANSAC, thresh)."""
    L = load()
    src = np.ascontiguousarray(src, np.float32).reshape(-1, 2)
    dst = np.ascontiguousarray(dst, np.float32).reshape(-1, 2)
    n = src.shape[0]
    H = np.zeros(9, np.float64)
    mask = np.zeros(n, np.uint8)
    ninl = ctypes.c_int(0)
    check(L.mcs_ransac_homography_host(src.ctypes.data, dst.ctypes.data, n, float(thresh),
                                       int(iters), int(seed) & 0xffffffff, H.ctypes.data,
                                       mask.ctypes.data, ctypes.byref(ninl), device))
    return (H.reshape(3, 3) if ninl.value > 0 else None), mask.reshape(-1, 1)


class StreamPipeline:
    """Host-frame pipeline over a plan (mcs_stream_*): submit() returns a slot, wait(slot) the
    mosaic.  Keep at most `depth` captures in flight."""

    def __init__(self, plan: "Plan", depth: int = 3, use_graphs: bool = True):
        self._lib = load()
        self.plan = plan
        self.depth = depth
        h = ctypes.c_void_p()
        check(self._lib.mcs_stream_create(plan._h, depth, 1 if use_graphs else 0,
                                          ctypes.byref(h)))
        self._h = h

    def _check_frames(self, cams):
        """The pipeline copies cam_w * C * cam_h bytes per camera from each frame: refuse
        anything that is not exactly the plan's camera (count, (h, w[, C]), uint8).  Frames off
        their calibrated size go through Stitcher.stitch, which resizes them like the reference
        (StitcherClass.py:226-233)."""
        C = self.plan.channels
        if len(cams) != self.plan.n_cams:
            raise ValueError(f"{len(cams)} frames for a plan of {self.plan.n_cams} cameras")
        out = []
        for i, (c, (h, w)) in enumerate(zip(cams, self.plan.cam_shapes)):
            c = np.asarray(c)
            if c.dtype != np.uint8:
                raise ValueError(f"camera {i}: dtype {c.dtype}, expected uint8")
            want = (h, w) if C == 1 and c.ndim == 2 else (h, w, C)
            if tuple(c.shape) != want:
                raise ValueError(f"camera {i}: frame shape {c.shape}, the plan expects {want}")
            out.append(np.ascontiguousarray(c))
        return out

    def submit(self, cams) -> int:
        cams = self._check_frames(cams)
        ptrs = (ctypes.c_void_p * len(cams))(*[c.ctypes.data for c in cams])
        slot = ctypes.c_int(-1)
        check(self._lib.mcs_stream_submit(self._h, ptrs, ctypes.byref(slot)))
        return slot.value

    def submit_concat(self, frame) -> int:
        """One frame of the reference's memmap bus layout: the cameras side by side on axis 1
        (np.concatenate(images, axis=1), video_mapping_node.py:140), in the plan's camera
        order; gathered into the pinned slot without an intermediate copy per camera."""
        frame = np.asarray(frame)
        C = self.plan.channels
        if frame.dtype != np.uint8:
            raise ValueError(f"bus frame dtype {frame.dtype}, expected uint8")
        if (frame.ndim == 3 and frame.shape[2] != C) or (frame.ndim == 2 and C != 1) or \
                frame.ndim not in (2, 3):
            raise ValueError(f"bus frame shape {frame.shape} for a {C}-channel plan")
        if frame.strides[-1] != 1 or (frame.ndim == 3 and frame.strides[1] != frame.shape[2]):
            frame = np.ascontiguousarray(frame)
        pitch = frame.strides[0]
        ptrs, pitches, x = [], [], 0
        for (h, w) in self.plan.cam_shapes:
            if frame.shape[0] < h or frame.shape[1] < x + w:
                raise ValueError(f"frame {frame.shape} too small for cameras {self.plan.cam_shapes}")
            ptrs.append(frame.ctypes.data + x * C)
            pitches.append(pitch)
            x += w
        if frame.shape[1] != x:
            raise ValueError(f"frame width {frame.shape[1]} != sum of camera widths {x}")
        pp = (ctypes.c_void_p * len(ptrs))(*ptrs)
        rp = (ctypes.c_int64 * len(pitches))(*pitches)
        slot = ctypes.c_int(-1)
        check(self._lib.mcs_stream_submit_strided(self._h, pp, rp, ctypes.byref(slot)))
        return slot.value

    def next_slot(self) -> int:
        """The slot the next submit fills (McsError if it has not been collected yet)."""
        r = self._lib.mcs_stream_next_slot(self._h)
        if r < 0:
            check(r)
        return r

    def input_views(self, slot: int):
        """Zero-copy producer side: numpy views of `slot`'s pinned input buffers, one per
        camera ((h, w[, C]) uint8), to be filled in place before submit_inplace()."""
        C = self.plan.channels
        views = []
        for i, (h, w) in enumerate(self.plan.cam_shapes):
            p = self._lib.mcs_stream_input(self._h, int(slot), i)
            if not p:
                raise McsError(MCS_E_INVALID, f"no input buffer for slot {slot} camera {i}")
            buf = (ctypes.c_uint8 * (h * w * C)).from_address(p)
            views.append(np.frombuffer(buf, np.uint8).reshape((h, w) if C == 1 else (h, w, C)))
        return views

    def submit_inplace(self) -> int:
        """Submit the next slot with the frames already written into its input_views()."""
        slot = ctypes.c_int(-1)
        check(self._lib.mcs_stream_submit(self._h, None, ctypes.byref(slot)))
        return slot.value

    def output_view(self, slot: int) -> np.ndarray:
        """Zero-copy consumer side: the pinned mosaic of `slot` (valid after wait(slot,
        copy=False) until the slot is submitted again)."""
        p = self._lib.mcs_stream_output(self._h, int(slot))
        if not p:
            raise McsError(MCS_E_INVALID, f"no output buffer for slot {slot}")
        shape = self.plan.out_shape()
        buf = (ctypes.c_uint8 * int(np.prod(shape))).from_address(p)
        return np.frombuffer(buf, np.uint8).reshape(shape)

    def wait(self, slot: int, out=None, copy: bool = True) -> np.ndarray:
        if not copy:
            check(self._lib.mcs_stream_wait(self._h, slot, None))
            return self.output_view(slot)
        if out is None:
            out = np.empty(self.plan.out_shape(), np.uint8)
        elif not (isinstance(out, np.ndarray) and out.dtype == np.uint8 and
                  out.flags.c_contiguous and out.flags.writeable and
                  tuple(out.shape) == self.plan.out_shape()):
            raise ValueError(f"out must be a writeable C-contiguous uint8 array of shape "
                             f"{self.plan.out_shape()}")
        check(self._lib.mcs_stream_wait(self._h, slot, out.ctypes.data))
        return out

    def close(self):
        if getattr(self, "_h", None):
            self._lib.mcs_stream_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def orb_detect(image, nfeatures: int = 2000, nlevels: int = 8, scale_factor: float = 1.2,
               fast_threshold: int = 20, device: int = 0):
    """ORB on the GPU (mcs_orb_detect_host): image u8 gray (h, w) or BGR (h, w, 3).  Returns a
    dict of xy (n, 2) float32 level-0 pixels, response (n,) float32, angle (n,) degrees,
    level (n,) int32, desc (n, 32) uint8."""
    L = load()
    img = np.ascontiguousarray(image, np.uint8)
    ch = 1 if img.ndim == 2 else img.shape[2]
    h, w = img.shape[:2]
    xy = np.zeros((max(nfeatures, 1), 2), np.float32)
    resp = np.zeros(max(nfeatures, 1), np.float32)
    ang = np.zeros(max(nfeatures, 1), np.float32)
    lvl = np.zeros(max(nfeatures, 1), np.int32)
    desc = np.zeros((max(nfeatures, 1), 32), np.uint8)
    n = ctypes.c_int(0)
    check(L.mcs_orb_detect_host(img.ctypes.data, w, h, ch, nfeatures, nlevels,
                                float(scale_factor), fast_threshold, xy.ctypes.data,
                                resp.ctypes.data, ang.ctypes.data, lvl.ctypes.data,
                                desc.ctypes.data, ctypes.byref(n), device))
    k = n.value
    return dict(xy=xy[:k], response=resp[:k], angle=ang[:k], level=lvl[:k], desc=desc[:k])


class Group:
    """mcs_group: RCCL communicator of one process per GPU (include/mcs.h) for
    the final mosaic gather.  Group.unique_id() on rank 0, passed to every rank; then
    Group(n_ranks, rank, uid, device) on each (collective)."""

    @staticmethod
    def unique_id() -> bytes:
        L = load()
        buf = (ctypes.c_uint8 * MCS_GROUP_ID_BYTES)()
        check(L.mcs_group_unique_id(buf))
        return bytes(buf)

    def __init__(self, n_ranks: int, rank: int, uid: bytes, device: int = 0):
        L = load()
        if len(uid) != MCS_GROUP_ID_BYTES:
            raise ValueError("uid must be %d bytes" % MCS_GROUP_ID_BYTES)
        buf = (ctypes.c_uint8 * MCS_GROUP_ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        check(L.mcs_group_create(int(n_ranks), int(rank), buf, int(device), ctypes.byref(h)))
        self._h, self._lib = h, L
        self.n_ranks, self.rank, self.device = int(n_ranks), int(rank), int(device)

    def gather(self, src_ptr: int, nbytes: int, recv_ptr: int = 0, root: int = 0,
               stream: int = 0):
        """Every rank's nbytes at src_ptr to `root`'s recv_ptr + rank * nbytes (enqueued)."""
        check(self._lib.mcs_group_gather(self._h, ctypes.c_void_p(int(src_ptr)), int(nbytes),
                                         ctypes.c_void_p(int(recv_ptr)) if recv_ptr else None,
                                         int(root), ctypes.c_void_p(int(stream))))

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.mcs_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def stream_copy_workers() -> int:
    """Helper threads of this process's host copy pool (mcs_stream_copy_workers): the CPUs it
    may use, shared by the node's LOCAL_WORLD_SIZE ranks."""
    return int(load().mcs_stream_copy_workers())


def rccl_library() -> str:
    return (load().mcs_rccl_library() or b"").decode()


def orb_detect_device(ptr: int, w: int, h: int, channels: int, nfeatures: int = 2000,
                      nlevels: int = 8, scale_factor: float = 1.2, fast_threshold: int = 20,
                      device: int = 0):
    """mcs_orb_detect_device: ORB of a dense u8 frame already in device memory (e.g. a torch
    tensor's data_ptr(), its producer finished).  Same dict as orb_detect."""
    L = load()
    xy = np.zeros((max(nfeatures, 1), 2), np.float32)
    resp = np.zeros(max(nfeatures, 1), np.float32)
    ang = np.zeros(max(nfeatures, 1), np.float32)
    lvl = np.zeros(max(nfeatures, 1), np.int32)
    desc = np.zeros((max(nfeatures, 1), 32), np.uint8)
    n = ctypes.c_int(0)
    check(L.mcs_orb_detect_device(ctypes.c_void_p(int(ptr)), w, h, channels, nfeatures, nlevels,
                                  float(scale_factor), fast_threshold, xy.ctypes.data,
                                  resp.ctypes.data, ang.ctypes.data, lvl.ctypes.data,
                                  desc.ctypes.data, ctypes.byref(n), device))
    k = n.value
    return dict(xy=xy[:k], response=resp[:k], angle=ang[:k], level=lvl[:k], desc=desc[:k])


class RigJob:
    """mcs_rig_job: the per-capture estimation of config 3 (ORB of every camera, then BF Hamming
    kNN-2 + ratio + RANSAC/LM per adjacent pair) on libmcs's worker threads.  submit() returns at
    once; wait() gives (H list with None for failed pairs, stats dict).  captures > 1
    (mcs_rig_job_create_batch): one launch chain over that many captures' cameras; submit takes
    captures x n_cams pointers, wait() returns one (H list, stats) per capture."""

    def __init__(self, n_cams: int, w: int, h: int, channels: int = 3, nfeatures: int = 2000,
                 nlevels: int = 8, scale_factor: float = 1.2, fast_threshold: int = 20,
                 ratio: float = 0.75, reproj_thresh: float = 3.0, iters: int = 2000,
                 seed: int = 0, device: int = 0, captures: int = 1):
        self._lib = load()
        self.n, self.q = n_cams, captures
        h_ = ctypes.c_void_p()
        check(self._lib.mcs_rig_job_create_batch(n_cams, captures, w, h, channels, nfeatures,
                                                 nlevels, float(scale_factor), fast_threshold,
                                                 float(ratio), float(reproj_thresh), iters,
                                                 int(seed) & 0xffffffff, device, ctypes.byref(h_)))
        self._h = h_
        self._H = np.zeros((captures * (n_cams - 1), 9), np.float64)
        self._ok = np.zeros(captures * (n_cams - 1), np.int32)
        self._kp = np.zeros(captures * n_cams, np.int32)
        self._m = np.zeros(captures * (n_cams - 1), np.int32)
        self._inl = np.zeros(captures * (n_cams - 1), np.int32)

    def submit(self, frame_ptrs, wait_event: int = 0):
        if len(frame_ptrs) != self.n * self.q:
            raise McsError(MCS_E_INVALID, f"rig job: {self.n * self.q} frames expected, "
                           f"{len(frame_ptrs)} given")
        arr = (ctypes.c_void_p * (self.n * self.q))(*[int(p) for p in frame_ptrs])
        check(self._lib.mcs_rig_job_submit(self._h, arr, ctypes.c_void_p(int(wait_event)) if
                                           wait_event else None))

    def _stats(self, q):
        n, m = self.n, self.n - 1
        return {"keypoints": self._kp[q * n:(q + 1) * n].tolist(),
                "matches": self._m[q * m:(q + 1) * m].tolist(),
                "inliers": self._inl[q * m:(q + 1) * m].tolist()}

    def wait(self):
        check(self._lib.mcs_rig_job_wait(self._h, self._H.ctypes.data, self._ok.ctypes.data,
                                         self._kp.ctypes.data, self._m.ctypes.data,
                                         self._inl.ctypes.data))
        m = self.n - 1
        res = [([self._H[q * m + k].reshape(3, 3).copy() if self._ok[q * m + k] else None
                 for k in range(m)], self._stats(q)) for q in range(self.q)]
        return res[0] if self.q == 1 else res

    def wait_stitch(self, H_io, ok_io, out_ptr, out_pitch: int, out_capacity: int,
                    stream: int = 0, super_mode: bool = False, interp: int = MCS_INTER_LINEAR):
        """wait() + the capture's chain geometry, plan and stitch in libmcs
        (mcs_rig_job_wait_stitch[_batch]): H_io ((n - 1, 9) float64) / ok_io ((n - 1,) int32)
        hold the pairs' homographies, updated in place capture by capture (a failed pair keeps
        its entry); the mosaic goes to out_ptr (device, rows out_pitch bytes apart; a list of
        `captures` pointers for a batch job) on `stream`.  Returns ((out_h, out_w), stats), or a
        list of them for a batch job."""
        ptrs = list(out_ptr) if self.q > 1 else [out_ptr]
        if len(ptrs) != self.q:
            raise McsError(MCS_E_INVALID, f"rig job: {self.q} outputs expected")
        # libmcs reads and writes 9 (n - 1) doubles and (n - 1) int32 through these pointers
        n1 = self.n - 1
        if not (isinstance(H_io, np.ndarray) and H_io.dtype == np.float64 and
                H_io.shape == (n1, 9) and H_io.flags.c_contiguous and H_io.flags.writeable):
            raise McsError(MCS_E_INVALID, f"rig job: H_io must be a writable C-contiguous "
                                          f"float64 array of shape ({n1}, 9)")
        if not (isinstance(ok_io, np.ndarray) and ok_io.dtype == np.int32 and
                ok_io.shape == (n1,) and ok_io.flags.c_contiguous and ok_io.flags.writeable):
            raise McsError(MCS_E_INVALID, f"rig job: ok_io must be a writable C-contiguous "
                                          f"int32 array of shape ({n1},)")
        outs = (ctypes.c_void_p * self.q)(*[int(p) for p in ptrs])
        w, h = (ctypes.c_int * self.q)(), (ctypes.c_int * self.q)()
        check(self._lib.mcs_rig_job_wait_stitch_batch(
            self._h, H_io.ctypes.data, ok_io.ctypes.data, 1 if super_mode else 0, int(interp),
            outs, int(out_pitch), int(out_capacity),
            ctypes.c_void_p(int(stream)) if stream else None, w, h,
            self._kp.ctypes.data, self._m.ctypes.data, self._inl.ctypes.data))
        res = [((h[q], w[q]), self._stats(q)) for q in range(self.q)]
        return res[0] if self.q == 1 else res

    def counts(self):
        """(captures finished on the device path, on the per-call path)."""
        a, b = ctypes.c_int(), ctypes.c_int()
        check(self._lib.mcs_rig_job_counts(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def close(self):
        if self._h:
            self._lib.mcs_rig_job_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def chain_stages(pair_H, pair_ok, cam_shapes, super_mode: bool = False):
    """mcs_chain_stages: the StageDesc of every stage of a chain from its adjacent-pair
    homographies (pair_H (n - 1, 9) float64, pair_ok (n - 1,) flags; cam_shapes (h, w[, C]) per
    camera) -- libmcs's restatement of estimate.chain_stages (host arithmetic, no GPU)."""
    L = load()
    n = len(cam_shapes)
    H = np.ascontiguousarray(np.asarray(pair_H, np.float64).reshape(max(n - 1, 0), 9))
    ok = np.ascontiguousarray(np.asarray(pair_ok, np.int32).reshape(max(n - 1, 0)))
    cw = np.array([s[1] for s in cam_shapes], np.int32)
    ch = np.array([s[0] for s in cam_shapes], np.int32)
    out = (StageDesc * max(1, n - 1))()
    check(L.mcs_chain_stages(n, cw.ctypes.data, ch.ctypes.data, H.ctypes.data, ok.ctypes.data,
                             1 if super_mode else 0, out))
    return [out[k] for k in range(n - 1)]


def seam_graphcut_host(labels, cover, samples):
    """mcs_seam_graphcut_host: labels (gh, gw) u8 (distance owners' cameras), cover (gh, gw)
    u16 camera masks, samples (n_cams, gh, gw, C) u8 -> the cut labels (new array)."""
    L = load()
    lab = np.ascontiguousarray(labels, np.uint8).copy()
    cov = np.ascontiguousarray(cover, np.uint16)
    smp = np.ascontiguousarray(samples, np.uint8)
    n, gh, gw = smp.shape[0], lab.shape[0], lab.shape[1]
    C = 1 if smp.ndim == 3 else smp.shape[3]
    check(L.mcs_seam_graphcut_host(n, gw, gh, lab.ctypes.data_as(ctypes.c_void_p),
                                   cov.ctypes.data_as(ctypes.c_void_p),
                                   smp.ctypes.data_as(ctypes.c_void_p), C))
    return lab


def seam_graphcut_device(labels, cover, samples, device: int = 0, with_stats: bool = False):
    """mcs_seam_graphcut_device: the cut of seam_graphcut_host by push-relabel on the GPU
    (same arrays); with_stats: also (pairs, push launches, relabel launches, global relabels,
    microseconds)."""
    L = load()
    lab = np.ascontiguousarray(labels, np.uint8).copy()
    cov = np.ascontiguousarray(cover, np.uint16)
    smp = np.ascontiguousarray(samples, np.uint8)
    n, gh, gw = smp.shape[0], lab.shape[0], lab.shape[1]
    C = 1 if smp.ndim == 3 else smp.shape[3]
    st = np.zeros(5, np.int64)
    check(L.mcs_seam_graphcut_device(n, gw, gh, lab.ctypes.data, cov.ctypes.data,
                                     smp.ctypes.data, C, device, st.ctypes.data))
    return (lab, tuple(int(v) for v in st)) if with_stats else lab


def undistort_map_host(K, dist, w: int, h: int) -> np.ndarray:
    """mcs_undistort_map_host: (h, w, 2) int32 fixed-point map (x, y in 1/32 px)."""
    L = load()
    k = np.ascontiguousarray(np.asarray(K, np.float64).reshape(9))
    d = np.ascontiguousarray(np.asarray(dist if dist is not None else [], np.float64).reshape(-1))
    out = np.empty((h, w, 2), np.int32)
    check(L.mcs_undistort_map_host(k.ctypes.data_as(ctypes.c_void_p),
                                   d.ctypes.data_as(ctypes.c_void_p) if d.size else None,
                                   int(d.size), int(w), int(h),
                                   out.ctypes.data_as(ctypes.c_void_p)))
    return out


def match_l2_knn2(query, train, device: int = 0):
    """mcs_match_l2_knn2_host: BFMatcher(NORM_L2).knnMatch(k=2) of float descriptors ->
    (idx (nq, 2) int32, dist (nq, 2) float32, exact: bool)."""
    L = load()
    q = np.ascontiguousarray(query, np.float32)
    t = np.ascontiguousarray(train, np.float32)
    nq = q.shape[0]
    nt = t.shape[0] if t.size else 0
    dim = q.shape[1] if q.ndim == 2 else (t.shape[1] if t.ndim == 2 else 1)
    idx = np.empty((nq, 2), np.int32)
    dist = np.empty((nq, 2), np.float32)
    ex = ctypes.c_int(0)
    check(L.mcs_match_l2_knn2_host(q.ctypes.data_as(ctypes.c_void_p), nq,
                                   t.ctypes.data_as(ctypes.c_void_p) if nt else None, nt, dim,
                                   idx.ctypes.data_as(ctypes.c_void_p),
                                   dist.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ex),
                                   int(device)))
    return idx, dist, bool(ex.value)

