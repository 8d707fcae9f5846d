// mcs_feat_int.h -- internals of the estimation module shared by its host files
// (mcs_features.cpp: the per-call entry points; mcs_rig.cpp: a whole rig capture per launch
// chain).  Not part of the C ABI.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "mcs_common.h"
#include "mcs_fparams.h"

namespace mcs {
namespace feat {

// The feature code object's kernels on one device (looked up once).
struct FeatureKernels {
    bool loaded = false;
    hipFunction_t knn2 = nullptr, knn2_finalize = nullptr;
    hipFunction_t ransac_score = nullptr, ransac_mask = nullptr;
    hipFunction_t orb_gray = nullptr, orb_level = nullptr, orb_describe = nullptr;
    hipFunction_t orb_pyramid = nullptr;
    hipFunction_t orb_select = nullptr;
    hipFunction_t l2_prep = nullptr, l2_i8 = nullptr, l2_f32 = nullptr, l2_finalize = nullptr;
    hipFunction_t rig_knn2 = nullptr, rig_match = nullptr, rig_ransac = nullptr,
                  rig_best = nullptr, rig_hyp = nullptr;
    hipFunction_t seam_init = nullptr, seam_hinit = nullptr, seam_relabel = nullptr,
                  seam_push = nullptr, seam_active = nullptr, seam_label = nullptr,
                  seam_relabel_lds = nullptr;
};
int feature_kernels(const rt::Api *A, int device, const FeatureKernels **out);
// hipModuleLaunchKernel with the argument block passed by value (grid gx x gy x gz).
int launch(const rt::Api *A, hipFunction_t f, unsigned gx, unsigned gy, unsigned bx, void *args,
           size_t sz, hipStream_t s, unsigned gz = 1, unsigned lds = 0);

// ORB's level geometry, as OpenCV's ORB computes it (float arithmetic): level sizes, scales and
// per-level keypoint quotas; the level images' pixel offsets (256-aligned) and the candidate
// buffer's per-level capacity / offset.
struct OrbGeom {
    int nlevels = 0;
    int lw[12] = {0}, lh[12] = {0}, quota[12] = {0};
    float lscale[12] = {0};
    size_t off[13] = {0};
    size_t cap[12] = {0}, coff[13] = {0}, cap_total = 0;
    int n_bound = 0;   // sum of the quotas: keypoints per frame at most
};
int orb_geom(int w, int h, int nfeatures, int nlevels, float scale_factor, OrbGeom *g);
// mcs_orb_pyramid's arguments for the levels of `g` (level images at lvl + off[l]); the block
// count, 0 when the one-launch pyramid does not apply (the per-level resize chain then does).
unsigned pyramid_args(const OrbGeom &g, uint8_t *lvl, KOrbBuildArgs &a);

}  // namespace feat
}  // namespace mcs
