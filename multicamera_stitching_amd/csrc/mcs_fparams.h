// mcs_fparams.h -- kernel argument blocks of the feature/estimation module (mcs_features.hip),
// shared by the host (g++) and the device compile.
#pragma once

#include <stdint.h>

namespace mcs {

// Brute-force Hamming kNN-2 over 256-bit descriptors (BFMatcher(NORM_HAMMING).knnMatch(k=2),
// the per-frame matcher of SURVEY.md 8 NS-4; reference counterpart StitcherClass.py:405-448).
constexpr int kDescBytes = 32;
constexpr int kKnnQueriesPerBlock = 64;   // one query per lane
constexpr int kKnnKeyShift = 23;          // key = distance << 23 | train index
constexpr int kKnnMaxTrain = 1 << kKnnKeyShift;
struct KHammingArgs {
    const uint32_t *query;   // nq x 8 words
    const uint32_t *train;   // nt x 8 words
    uint32_t *keys;          // nq x 2 (best, second) -> finalised into idx
    int32_t *dist;           // nq x 2
    int nq, nt, per_chunk, pad_;
};

// RANSAC homography (mcs_ransac_core.h): one block per hypothesis scores it
// over all correspondences; a second launch writes the best hypothesis' inlier mask.
constexpr int kRansacBlock = 256;
struct KRansacArgs {
    const double *pts;    // n x 4: x, y (source), u, v (destination)
    double *hyps;         // iters x 8: h0..h7 (h33 = 1); NaN for a rejected hypothesis
    int32_t *scores;      // iters: inlier count, -1 for a rejected hypothesis
    uint8_t *mask;        // n: inliers of hypothesis `best`
    double t2;            // threshold^2
    int n, iters, best;
    uint32_t seed;
};

// ORB (mcs_orb_core.h).
struct OrbCand {
    int x, y;
    double response;
};
struct KOrbLevelArgs {
    const uint8_t *img;    // level image (w x h, dense)
    uint16_t *hblur;       // horizontal blur pass
    uint8_t *blur;         // blurred level
    uint8_t *score;        // FAST scores of corners (0 elsewhere)
    OrbCand *cand;         // NMS survivors with their Harris response
    int *ncand;
    int w, h, threshold, cap;
};
struct KOrbDescArgs {
    const uint8_t *img[12], *blur[12];
    int w[12];
    const int *kp;         // n x 3: level, x, y
    uint8_t *desc;         // n x 32
    double *orient;        // n x 2: cos, sin
    int n, pad_;
};
struct KGrayArgs {
    const uint8_t *bgr;
    uint8_t *gray;
    int n, pad_;
};

}  // namespace mcs
