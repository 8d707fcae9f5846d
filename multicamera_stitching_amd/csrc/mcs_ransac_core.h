// mcs_ransac_core.h -- the per-hypothesis arithmetic of RANSAC homography estimation
// (SURVEY.md section 8 NS-5), shared by the gfx950 kernels (mcs_features.hip) and the host
// refit (mcs_features.cpp).  Semantics of cv2.findHomography(src, dst, cv2.RANSAC, thresh) as
// the reference calls it (StitcherClass.py:440-441); OpenCV's own RNG, solver and LM refinement
// are not reproduced (third-party, version unpinned): the algorithm is specified here and
// restated independently in oracle/orc_ransac.c.
//
//   hypothesis k: 4 distinct point indices from a counter-based hash of (seed, k, draw, retry);
//     rejected when a point triple flips orientation between src and dst (a mirrored or
//     degenerate subset, as OpenCV's checkSubset) or the 8x8 system is singular;
//   model: h (h33 = 1) from the 8x8 DLT system, Gaussian elimination with partial pivoting, FP64;
//   score: points with (h.src projected - dst)^2 <= thresh^2 (FP64, explicit operation order);
//   best: most inliers, ties to the lower k; refit: least squares over the best hypothesis'
//   inliers (8x8 normal equations, same solver); mask: the best hypothesis' inliers.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define MCS_HD __host__ __device__ __forceinline__
#else
#define MCS_HD static inline
#endif

namespace mcs {

constexpr int kRansacMaxRetry = 64;

MCS_HD uint32_t rs_fmix(uint32_t a)
{
    a ^= a >> 16;
    a *= 0x85ebca6bu;
    a ^= a >> 13;
    a *= 0xc2b2ae35u;
    a ^= a >> 16;
    return a;
}

// Index of draw m (0..3) of hypothesis k, retry c.
MCS_HD uint32_t rs_draw(uint32_t seed, uint32_t k, uint32_t m, uint32_t c, uint32_t n)
{
    const uint32_t base = rs_fmix(seed + 0x9e3779b9u * (k + 1u));
    return rs_fmix(base ^ (m * 0x632be5abu + c * 0x85157af5u)) % n;
}

// 4 distinct indices of hypothesis k; false if the retries run out.
MCS_HD bool rs_subset(uint32_t seed, uint32_t k, uint32_t n, int *idx)
{
    for (int m = 0; m < 4; m++) {
        bool ok = false;
        for (uint32_t c = 0; c < (uint32_t)kRansacMaxRetry && !ok; c++) {
            const int v = (int)rs_draw(seed, k, (uint32_t)m, c, n);
            ok = true;
            for (int q = 0; q < m; q++) ok = ok && idx[q] != v;
            if (ok) idx[m] = v;
        }
        if (!ok) return false;
    }
    return true;
}

MCS_HD double rs_cross(const double *p, int a, int b, int c)
{
    return (p[2 * b] - p[2 * a]) * (p[2 * c + 1] - p[2 * a + 1]) -
           (p[2 * b + 1] - p[2 * a + 1]) * (p[2 * c] - p[2 * a]);
}

// Every triple of the 4 points keeps its orientation (no mirroring, no collinear triple).
MCS_HD bool rs_check_subset(const double *s, const double *d)
{
    const int tri[4][3] = {{0, 1, 2}, {0, 1, 3}, {0, 2, 3}, {1, 2, 3}};
    for (int t = 0; t < 4; t++) {
        const double a = rs_cross(s, tri[t][0], tri[t][1], tri[t][2]);
        const double b = rs_cross(d, tri[t][0], tri[t][1], tri[t][2]);
        if (!(a * b > 0.0)) return false;
    }
    return true;
}

// Solves the 8x8 system M h = r in place (M row-major, 8 x 9 augmented: column 8 = r).
// Partial pivoting (first maximum |a| wins), FP64, fixed order.  false if a pivot is < 1e-12.
MCS_HD bool rs_solve8(double (&M)[8][9], double *h)
{
    for (int c = 0; c < 8; c++) {
        int p = c;
        double best = M[c][c] < 0 ? -M[c][c] : M[c][c];
        for (int r = c + 1; r < 8; r++) {
            const double v = M[r][c] < 0 ? -M[r][c] : M[r][c];
            if (v > best) best = v, p = r;
        }
        if (!(best >= 1e-12)) return false;
        if (p != c)
            for (int j = 0; j < 9; j++) {
                const double t = M[c][j];
                M[c][j] = M[p][j];
                M[p][j] = t;
            }
        for (int r = c + 1; r < 8; r++) {
            const double f = M[r][c] / M[c][c];
            for (int j = c; j < 9; j++) M[r][j] = M[r][j] - f * M[c][j];
        }
    }
    for (int r = 7; r >= 0; r--) {
        double acc = M[r][8];
        for (int j = r + 1; j < 8; j++) acc = acc - M[r][j] * h[j];
        h[r] = acc / M[r][r];
    }
    return true;
}

// DLT rows of correspondence (x, y) -> (u, v).
MCS_HD void rs_rows(double x, double y, double u, double v, double *ru, double *rv)
{
    ru[0] = x, ru[1] = y, ru[2] = 1.0, ru[3] = 0.0, ru[4] = 0.0, ru[5] = 0.0;
    ru[6] = -u * x, ru[7] = -u * y, ru[8] = u;
    rv[0] = 0.0, rv[1] = 0.0, rv[2] = 0.0, rv[3] = x, rv[4] = y, rv[5] = 1.0;
    rv[6] = -v * x, rv[7] = -v * y, rv[8] = v;
}

// Model of 4 correspondences (s, d: 4 x 2 doubles).
MCS_HD bool rs_model4(const double *s, const double *d, double *h)
{
    if (!rs_check_subset(s, d)) return false;
    double M[8][9];
    for (int i = 0; i < 4; i++)
        rs_rows(s[2 * i], s[2 * i + 1], d[2 * i], d[2 * i + 1], M[2 * i], M[2 * i + 1]);
    return rs_solve8(M, h);
}

// Squared reprojection error of (x, y) -> (u, v) under h; negative when w == 0.
MCS_HD double rs_err2(const double *h, double x, double y, double u, double v)
{
    const double w = (h[6] * x + h[7] * y) + 1.0;
    if (w == 0.0) return -1.0;
    const double px = ((h[0] * x + h[1] * y) + h[2]) / w;
    const double py = ((h[3] * x + h[4] * y) + h[5]) / w;
    const double ex = px - u, ey = py - v;
    return ex * ex + ey * ey;
}

MCS_HD bool rs_inlier(const double *h, double x, double y, double u, double v, double t2)
{
    const double e = rs_err2(h, x, y, u, v);
    return e >= 0.0 && e <= t2;
}

}  // namespace mcs
