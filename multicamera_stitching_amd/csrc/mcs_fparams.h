// mcs_fparams.h -- kernel argument blocks of the feature/estimation module (mcs_features.hip),
// shared by the host (g++) and the device compile.
#pragma once

#include <stdint.h>

namespace mcs {

// Brute-force Hamming kNN-2 over 256-bit descriptors (BFMatcher(NORM_HAMMING).knnMatch(k=2),
// the per-frame matcher of SURVEY.md 8 NS-4; reference counterpart StitcherClass.py:405-448).
constexpr int kDescBytes = 32;
#ifndef MCS_KNN_QPL
#define MCS_KNN_QPL 1
#endif
constexpr int kKnnLanes = 64;                               // one wave per block
constexpr int kKnnQueriesPerLane = MCS_KNN_QPL;             // each staged train descriptor
constexpr int kKnnQueriesPerBlock = kKnnLanes * kKnnQueriesPerLane;   // serves this many
constexpr int kKnnKeyShift = 23;          // key = distance << 23 | train index
constexpr int kKnnMaxTrain = 1 << kKnnKeyShift;
#ifndef MCS_KNN_TARGET_BLOCKS
#define MCS_KNN_TARGET_BLOCKS 65536
#endif
constexpr int kKnnTargetBlocks = MCS_KNN_TARGET_BLOCKS;   // (query wave, train chunk) blocks
struct KHammingArgs {
    const uint32_t *query;   // nq x 8 words
    const uint32_t *train;   // nt x 8 words
    uint32_t *keys;          // nq x 2 (best, second) -> finalised into idx
    int32_t *dist;           // nq x 2
    int nq, nt, per_chunk, pad_;
};

// Brute-force L2 kNN-2 over float descriptors (BFMatcher(NORM_L2) / "BruteForce"
// .knnMatch(k=2), the reference's SIFT matcher, StitcherClass.py:423-424).
// Integer-valued descriptors in [0, 255] (OpenCV's SIFT output) take the exact path: int8 MFMA
// on (d - 128), |a - b|^2 = |a|^2 + |b|^2 - 2 a.b in int32, distance = float(sqrt(double)) --
// the same float OpenCV computes (its float sums are exact for such data); anything else takes
// the f32-MFMA path (float |a|^2 + |b|^2 - 2 a.b).  Keys: float bits << 32 | train index.
constexpr int kL2QueriesPerBlock = 64;   // 4 waves x one 16-query MFMA row tile
constexpr int kL2MaxDim = 256;
constexpr unsigned long long kL2KeyNone = ~0ull;
struct KL2PrepArgs {
    const float *desc;   // n x dim
    int8_t *i8;          // n x dimp: d - 128 (padding: d = 0)
    int32_t *norm_i;     // sum d^2 (exact path)
    int32_t *sum_i;      // sum (d - 128)
    float *norm_f;       // sum d^2 in float (f32 path)
    uint32_t *flag;      // |= 1 when a value is not an integer in [0, 255]
    int n, dim, dimp, pad_;
};
struct KL2Args {
    const int8_t *q8, *t8;
    const float *qf, *tf;
    const int32_t *qn, *tn, *qs, *ts;
    const float *qnf, *tnf;
    const uint32_t *flag;
    unsigned long long *keys;   // nq x 2
    int32_t *idx;               // nq x 2 (finalised)
    float *dist;                // nq x 2
    int nq, nt, dim, dimp, per_chunk, pad_;
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
// mcs_orb_level's tile: kOrbTileW x kOrbTileH pixels of a level per block (MCS_ORB_TILE_H: 16, 32
// or 64 rows).  64: the 4-pixel halo and the five barrier phases shared by four times the pixels
// of round 5's 64 x 16 tile, 52 KB of LDS, 3 blocks per CU (C3 resident estimate + stitch, same
// boxes: 16 rows 2,860-2,865, 32 rows 2,957-2,984, 64 rows 3,131-3,236 captures/s;
// profiles/r06_orb_tile_ab.txt)
#ifndef MCS_ORB_TILE_H
#define MCS_ORB_TILE_H 64
#endif
constexpr int kOrbTileW = 64, kOrbTileH = MCS_ORB_TILE_H;
// threads of an mcs_orb_level block (8 waves: with 4 blocks of 36 KB per CU, 32 waves in flight)
#ifndef MCS_ORB_LEVEL_THREADS
#define MCS_ORB_LEVEL_THREADS 512
#endif
constexpr int kOrbLevelThreads = MCS_ORB_LEVEL_THREADS;
// All levels of one frame in one launch (mcs_orb_level): grid (bstart[nlevels]) blocks of 256
// threads, level l owning blocks [bstart[l], bstart[l + 1]), one block per 64 x 16 tile (row-major
// over the level).  Level buffers are the bases + off[l] (pixels) and cand + coff[l].
// Every ORB kernel also runs over a batch of frames (the cameras of a rig capture, grid.y =
// camera c): camera c's level images at + c * stride pixels, its candidates at + c * cstride,
// its counts at ncand + c * kOrbMaxLevels, its keypoints (kp, resp, desc, orient) at
// + c * kstride keypoints, its sel at + 2 c.  Single-frame launches: grid.y = 1.
constexpr int kOrbMaxCams = 16;
struct KOrbPyrArgs {
    const uint8_t *img;
    uint8_t *blur;
    OrbCand *cand;
    int *ncand;                 // [nlevels]
    int64_t off[12];
    int coff[12], w[12], h[12], cap[12], bstart[13];
    int nlevels, threshold;
    int64_t stride;
    int cstride, pad_;
};
// The ORB pyramid in one launch (mcs_orb_pyramid): levels 1 .. nlevels-1, each OpenCV's
// resize(INTER_LINEAR) of the level before it.  One block per tw x th tile of the LAST level;
// the block derives, top down, the region of every level that tile depends on (a level-l
// region = the source span of the level-(l+1) region), then computes them bottom up in LDS
// (ping-pong buffers of lds_w x lds_h bytes), writing every computed pixel to its level image.
// Neighbouring blocks' regions overlap by a pixel or two: those pixels are written twice with
// the same value.  Level l lives at lvl + off[l]; sx / sy = OpenCV's 1 / (dst / src) per level.
struct KOrbBuildArgs {
    uint8_t *lvl;
    int64_t off[12];
    double sx[12], sy[12];
    int w[12], h[12];
    int nlevels, tw, th, gx, lds_w, lds_h;
    int64_t stride;
};
struct KOrbDescArgs {
    const uint8_t *img[12], *blur[12];
    int w[12];
    const int *kp;         // n x 3: level, x, y
    uint8_t *desc;         // n x 32
    double *orient;        // n x 2: cos, sin
    const int *sel;        // mcs_orb_select's [n, overflow] (grid = the n bound), or NULL: n
    int n, kstride;
    int64_t stride;
};
// Per-level ranking on the device (mcs_orb_select): one block per level sorts the level's
// candidates (<= kOrbSelMax, else the host ranks every level) and writes its quota's
// keypoints, levels in order.  sel[0] = total keypoints, sel[1] = overflow flag.
constexpr int kOrbSelMax = 4096;
constexpr int kOrbSelThreads = 1024;
struct KOrbSelArgs {
    const OrbCand *cand;
    const int *ncand;      // [nlevels]
    int *kp;               // n x 3: level, x, y
    double *resp;          // n
    int *sel;              // [2]: n, overflow
    int coff[12], cap[12], quota[12];
    int nlevels, cstride, kstride, pad_;
};
struct KGrayArgs {
    const uint8_t *bgr[kOrbMaxCams];   // camera c = grid.y
    uint8_t *gray;                     // camera c at gray + c * stride
    int64_t stride;
    int n, pad_;
};

// A whole rig capture's estimation on the device (mcs_rig.cpp): after the batched ORB, per
// adjacent pair p (query camera p + 1, train camera p) the Hamming kNN-2 (mcs_rig_knn2), Lowe's
// ratio with the matched positions compacted in query order (mcs_rig_match), the RANSAC
// hypotheses (mcs_rig_ransac) and the best one with its inlier mask (mcs_rig_best) -- counts read
// from the device, so the chain needs no host round trip.
struct KRigArgs {
    const int *kp;          // camera c: kp + 3 c kstride (level, x, y)
    const uint8_t *desc;    // camera c: desc + 32 c kstride
    const int *sel;         // camera c: sel[2 c] keypoints, sel[2 c + 1] overflow
    uint32_t *keys;         // pair p: keys + 2 p kstride (kNN-2 keys, 0xffffffff on entry)
    double *pts;            // pair p: pts + 4 p kstride: x, y (camera p + 1), u, v (camera p)
    int *info;              // pair p: info[4 p ..]: matches, best hypothesis, its score, 0
    double *hyps;           // pair p: hyps + 8 p iters
    int32_t *scores;        // pair p: scores + p iters
    uint8_t *mask;          // pair p: mask + p kstride
    double *hbest;          // pair p: hbest + 8 p
    float lscale[12];       // level -> level-0 scale ((float)scale_factor^level)
    double ratio, t2;
    int kstride, iters, per_chunk;
    uint32_t seed;
};

// Graph-cut seams on the device (mcs_seam.cpp; spec oracle/orc_seam.c): the
// maximum flow of one camera pair's 4-connected overlap graph on the 2^k seam grid by
// push-relabel, run on the REVERSED graph (source = the b-side terminal, sink = the a side), so
// that the nodes which can still reach its sink in the residual graph of a maximum preflow are
// exactly the source side of the original graph's minimal minimum cut (the host Dinic's
// residual-reachable set, unique for every maximum flow).  Per grid point q of the pair's box:
// in[q] (node of this pair's graph), cap[d * np + q] the residual capacity toward neighbour d
// (0 +x, 1 -x, 2 +y, 3 -y), snk[q] toward the sink, ex[q] the excess, h[q] the height
// (kSeamHInf: cannot reach the sink).  Heights come from global relabels (Bellman-Ford
// relaxation from the sink to a fixpoint); pushes follow Hong's lock-free rule (push to the
// lowest residual neighbour when higher than it, else relabel), all updates atomic.
constexpr int kSeamTile = 16;                 // 16 x 16 grid points per block
constexpr int32_t kSeamHInf = 1 << 30;
constexpr long long kSeamBig = 1LL << 40;     // terminal capacity (the host Dinic's kBig)
struct KSeamFlowArgs {
    uint8_t *lab;             // gw x gh labels (camera index; 255 = none)
    const uint16_t *cov;      // covering cameras per point
    const uint8_t *smp;       // n_cams x np x cn samples
    uint8_t *in;
    int32_t *cap;             // 4 x np
    long long *snk, *ex;      // np
    int32_t *h;               // np
    int32_t *flag;            // [0] a height changed / [1] active nodes
    long long np;
    int gw, gh, cn, a, b;
    int x0, y0, bw, bh;       // the pair's box on the grid
    int iters, hmax;          // inner rounds per launch; heights >= hmax cannot reach the sink
};

}  // namespace mcs
