// mcs_common.h -- host-side declarations shared by the plan builder, the runtime binding and the
// C ABI (all compiled with g++; the kernels are a separate gfx950 code object).
#pragma once

#include <stdint.h>

#include "hip_rt.h"
#include "mcs.h"
#include "mcs_kparams.h"

// Returns MCS_E_HIP with the HIP error text when `expr` fails (needs `A`, the bound runtime).
#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return mcs::fail(MCS_E_HIP, "%s failed: %s", #expr, A->hipGetErrorString(e_));   \
    } while (0)

namespace mcs {

int fail(int code, const char *fmt, ...);
const char *last_error();
void clear_error();

void invert3x3_cv(const double *m, double *out);
int build_flat(const mcs_stage_desc *stages, int n_stages, int cam0_w, int cam0_h, int channels,
               int interp, mcs_flat_desc *fd);
void fill_kparams(const mcs_flat_desc &fd, KParams *kp);
int block_width(int W, int H);
bool undistort_map(const double *K, const double *dist, int n_dist, int w, int h, int32_t *tab);
// Pairwise graph-cut seam labels over the seam grid (mcs_seam.cpp; spec: oracle/orc_seam.c).
int seam_graphcut(int n_cams, int gw, int gh, uint8_t *lab, const uint16_t *cov,
                  const uint8_t *smp, int cn);

// Embedded gfx950 code objects (one per device source, see build.py) and their kernels.
enum Module { kModStitch = 0, kModFeatures = 1, kModSweep = 2, kNumModules = 3 };
constexpr int kMaxDevices = 64;
// Loads module `m` on `device` once (the device must be current) and looks up `name`.
int module_function(const rt::Api *A, int device, Module m, const char *name, hipFunction_t *out);
// findHomography's post-RANSAC stage (mcs_refine.cpp): normalised DLT on the inliers of `mask`
// + 10 Levenberg-Marquardt iterations; H (9 doubles) holds the RANSAC model on entry.
void homography_refine(const float *src_xy, const float *dst_xy, int n, const uint8_t *mask,
                       double *H);
// The same cut on the device (push-relabel, mcs_features.hip mcs_seam_flow_*): labels / cov /
// samples already in device memory (d_lab updated in place, on stream s, synchronised); cov is
// the host copy of d_cov (the pairs' boxes).  stats (may be NULL): [0] pairs with a graph, [1]
// push launches, [2] relabel launches, [3] global relabels, [4] microseconds.
int seam_graphcut_device(int device, hipStream_t s, int n_cams, int gw, int gh, uint8_t *d_lab,
                         const uint16_t *d_cov, const uint8_t *d_smp, int cn, const uint16_t *cov,
                         int64_t *stats);
// Orders the calling thread's feature-workspace stream on `device` (the stream its ORB / match /
// RANSAC calls run on, mcs_features.cpp) after `event`: a GPU-side wait, no host round trip.
int features_stream_wait(int device, void *event);
// The HIP device a plan was created for (its tables, buffers and side streams live there).
int plan_device(const mcs_plan *plan);

// Makes `dev` current for the duration of a call and restores the caller's device.
struct DeviceGuard {
    const rt::Api *A;
    int prev = -1;
    hipError_t err = hipSuccess;
    DeviceGuard(const rt::Api *a, int dev) : A(a)
    {
        err = A->hipGetDevice(&prev);
        if (err == hipSuccess && prev != dev) err = A->hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)A->hipSetDevice(prev);
    }
};

}  // namespace mcs
