"""Calibration-time feature matching behind StitcherBase.detectAndDescribe / matchKeypoints.

Reference (StitcherClass.py:356-448): OpenCV SIFT keypoints + float descriptors, BruteForce L2
kNN-2, Lowe ratio (strict <), more than 4 matches, findHomography(RANSAC, reprojThresh).  This
runs once per calibration (a keypress, video_mapping_node.py:187-188), not per frame.

Backends (MCS_FEATURES = auto | sift | orb): "sift" is OpenCV contrib SIFT when cv2 is
importable (the reference's own algorithm; its float L2 kNN-2 runs on the GPU unless
MCS_L2_MATCHER=cv2, exact for SIFT's integer-valued descriptors, and so does findHomography's
RANSAC + LM refinement unless MCS_HOMOGRAPHY=cv2); "orb" is the GPU path of
SURVEY.md 8 NS-3..5 -- ORB (mcs_orb_detect_host), brute-force Hamming kNN-2
(mcs_match_hamming_knn2_host), the same ratio test, RANSAC (mcs_ransac_homography_host).  "auto"
prefers SIFT (reference behaviour) and falls back to ORB when a GPU is present.  With neither,
calibrate_stitcher logs an error and returns, exactly like the reference without opencv-contrib
(:87-93), unless the caller passes precomputed homographies.
"""
from __future__ import annotations

import os

import numpy as np

from ._debugger import DEBUG_LEVEL_0

ORB_NFEATURES = int(os.environ.get("MCS_ORB_NFEATURES", "2000"))


def _cv2():
    try:
        import cv2
        return cv2
    except ImportError:
        return None


def _sift_available() -> bool:
    cv2 = _cv2()
    if cv2 is None:
        return False
    try:
        if int(cv2.__version__.split(".")[0]) == 3:
            cv2.xfeatures2d.SIFT_create()
            return True
        return hasattr(cv2, "SIFT_create") or hasattr(cv2, "FeatureDetector_create")
    except Exception:
        return False


def _orb_available() -> bool:
    try:
        from . import _capi
        return _capi.device_count() > 0
    except Exception:
        return False


def backend():
    """"sift", "orb" or None (MCS_FEATURES selects; "auto" = SIFT, else ORB on the GPU)."""
    want = os.environ.get("MCS_FEATURES", "auto").lower()
    if want in ("auto", "sift") and _sift_available():
        return "sift"
    if want in ("auto", "orb") and _orb_available():
        return "orb"
    return None


def available() -> bool:
    return backend() is not None


def detect_and_describe(owner, image):
    b = backend()
    if b == "orb":
        from . import _capi
        r = _capi.orb_detect(np.ascontiguousarray(image), nfeatures=ORB_NFEATURES)
        return r["xy"], r["desc"]
    cv2 = _cv2()
    if cv2 is None or b is None:
        owner.debugger(DEBUG_LEVEL_0, "OpenCV is not a contrib version, check for the module "
                       "xfeatures2d", log_type="err")
        return None, None
    major = int(cv2.__version__.split(".")[0])
    if major == 3:
        kps, features = cv2.xfeatures2d.SIFT_create().detectAndCompute(image, None)
    elif hasattr(cv2, "SIFT_create"):
        kps, features = cv2.SIFT_create().detectAndCompute(image, None)
    else:
        gray = cv2.cvtColor(image, cv2.COLOR_BGR2GRAY)
        kps = cv2.FeatureDetector_create("SIFT").detect(gray)
        kps, features = cv2.DescriptorExtractor_create("SIFT").compute(gray, kps)
    return np.float32([kp.pt for kp in kps]), features


def match_keypoints(owner, kpsA, kpsB, featuresA, featuresB, ratio=0.75, reprojThresh=4.0):
    if np.asarray(featuresA).dtype == np.uint8:     # binary (ORB) descriptors: the GPU path
        from . import _capi
        idx, dist = _capi.match_hamming_knn2(featuresA, featuresB)
        matches = ratio_matches(idx, dist, ratio)
        H = status = None
        if len(matches) > 4:
            ptsA = np.float32([kpsA[i] for (_, i) in matches])
            ptsB = np.float32([kpsB[i] for (i, _) in matches])
            H, status = _capi.ransac_homography(ptsA, ptsB, reprojThresh)
        return H, matches, status
    cv2 = _cv2()
    if os.environ.get("MCS_L2_MATCHER", "gpu") == "gpu":
        # BruteForce L2 kNN-2 on MFMA: SIFT's integer-valued descriptors are
        # matched exactly as OpenCV's float arithmetic does (mcs_match_l2_knn2_host)
        from . import _capi
        idx, dist, _ = _capi.match_l2_knn2(featuresA, featuresB)
        matches = ratio_matches(idx, dist, ratio)
    else:
        raw = cv2.DescriptorMatcher_create("BruteForce").knnMatch(featuresA, featuresB, 2)
        matches = [(m[0].trainIdx, m[0].queryIdx) for m in raw
                   if len(m) == 2 and m[0].distance < m[1].distance * ratio]
    H = status = None
    if len(matches) > 4:
        ptsA = np.float32([kpsA[i] for (_, i) in matches])
        ptsB = np.float32([kpsB[i] for (i, _) in matches])
        if os.environ.get("MCS_HOMOGRAPHY", "gpu") == "cv2" and cv2 is not None:
            H, status = cv2.findHomography(ptsA, ptsB, cv2.RANSAC, reprojThresh)
        else:
            # findHomography(RANSAC) on the GPU + its LM refinement (mcs_ransac_homography_host):
            # calibration needs no cv2 once the descriptors exist
            from . import _capi
            H, status = _capi.ransac_homography(ptsA, ptsB, reprojThresh)
    return H, matches, status


def ratio_matches(idx, dist, ratio=0.75):
    """Lowe's ratio test over knnMatch(k=2) results, as StitcherClass.py:427-433: query q is kept
    as (trainIdx, queryIdx) when it has two candidates and d0 < d1 * ratio (strict), in query
    order.  idx/dist: (nq, 2) arrays as returned by _capi.match_hamming_knn2."""
    idx = np.asarray(idx)
    dist = np.asarray(dist)
    ok = (idx[:, 1] >= 0) & (dist[:, 0].astype(np.float64) < dist[:, 1].astype(np.float64) * ratio)
    q = np.nonzero(ok)[0]
    return [(int(idx[i, 0]), int(i)) for i in q]
