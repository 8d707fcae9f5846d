// mcs_orb_core.h -- ORB feature detection/description: the
// specification shared by the gfx950 kernels (mcs_features.hip) and the host orchestration
// (mcs_features.cpp); restated independently in oracle/orc_orb.c.  Structure of OpenCV 3.4's
// ORB (nlevels pyramid by INTER_LINEAR resize of the previous level, FAST-9 + 3x3 non-maximum
// suppression, Harris ranking, intensity-centroid orientation over a radius-15 disk, 256-bit
// rBRIEF on a 7x7-blurred level with OpenCV's bit_pattern_31_), with the details defined here so
// that every value is an integer or a correctly rounded IEEE double (no atan2/sin/cos):
//   FAST score   max over the 16 arcs of 9 contiguous circle pixels of
//                max(min(I_c - I_p), min(I_p - I_c)); corner iff score > threshold;
//   NMS          a corner survives iff its score is > each of its 8 neighbours' (0 if not one);
//   border       keypoints only with edge <= x < w - edge (edge = 31) on their level;
//   Harris       a, b, c = sums over the 7x7 block of Ix^2, Iy^2, IxIy (3x3 Sobel, integers),
//                response = (double)(a b - c^2) - 0.04 ((double)(a + b))^2;
//   ranking      per level by response (desc), then y, then x; the per-level quota is
//                OpenCV's geometric split of nfeatures (float arithmetic as OpenCV);
//   orientation  m10, m01 over OpenCV's umax disk (integers); r = sqrt(m10^2 + m01^2),
//                (cos, sin) = (m10 / r, m01 / r) ((1, 0) when r = 0);
//   blur         7-tap integer kernel [18 34 49 54 49 34 18] / 256 (sigma ~2), horizontal then
//                vertical, rounding once: (sum + 32768) >> 16, reflect-101 borders;
//   descriptor   bit j of byte i (pair p = 8 i + j): B(q1) < B(q2), q = (rint(x c - y s),
//                rint(x s + y c)) for the pattern point (x, y), B the blurred level;
//   keypoint     (x, y) * (float)1.2^level in level-0 pixels.
#pragma once

#include <math.h>
#include <stdint.h>

#include "mcs_orb_pattern.h"

#if defined(__HIPCC__)
#define MCS_ORB_HD __host__ __device__ __forceinline__
#else
#define MCS_ORB_HD static inline
#endif

namespace mcs {

constexpr int kOrbEdge = 31;
constexpr int kOrbHalfPatch = 15;
constexpr int kOrbMaxLevels = 12;
constexpr int kOrbBlur[7] = {18, 34, 49, 54, 49, 34, 18};
// OpenCV's ORB u_max for HALF_PATCH_SIZE 15 (circle of the orientation patch)
constexpr int kOrbUmax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
// FAST-9 circle (x, y), OpenCV's order
constexpr int kFastCircle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1},
                                    {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                    {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

// FAST score of the pixel at p (row stride `step`): the arcs' minima by doubling windows
// (2, 4, 8, then the ninth pixel) over the circle unrolled to 24 entries -- the same values as
// the 16 x 9 scan, in a quarter of the operations.
MCS_ORB_HD int orb_fast_score(const uint8_t *p, int step)
{
    int d[24], lo[23], hi[23];
    const int c = p[0];
    for (int i = 0; i < 16; i++) d[i] = (int)p[kFastCircle[i][1] * step + kFastCircle[i][0]] - c;
    for (int i = 16; i < 24; i++) d[i] = d[i - 16];
    // lo: min of d (I_p - I_c) over the window, hi: max of d (so min(I_c - I_p) = -hi)
    for (int i = 0; i < 23; i++) {
        lo[i] = d[i] < d[i + 1] ? d[i] : d[i + 1];
        hi[i] = d[i] > d[i + 1] ? d[i] : d[i + 1];
    }
    for (int i = 0; i < 21; i++) {                       // windows of 4
        lo[i] = lo[i] < lo[i + 2] ? lo[i] : lo[i + 2];
        hi[i] = hi[i] > hi[i + 2] ? hi[i] : hi[i + 2];
    }
    int best = -255;
    for (int s = 0; s < 16; s++) {                       // windows of 8, then 9
        int l = lo[s] < lo[s + 4] ? lo[s] : lo[s + 4];
        int h = hi[s] > hi[s + 4] ? hi[s] : hi[s + 4];
        l = l < d[s + 8] ? l : d[s + 8];
        h = h > d[s + 8] ? h : d[s + 8];
        const int m = l > -h ? l : -h;
        best = m > best ? m : best;
    }
    return best;
}

// FAST segment test: some arc of 9 contiguous circle pixels is entirely brighter than
// I_c + t or entirely darker than I_c - t.  Exactly orb_fast_score(p) > t (an arc's
// max(min(I_c - I_p), min(I_p - I_c)) exceeds t iff every pixel of it is beyond t on one side),
// in bit operations: bit i of the masks per circle pixel, runs of 9 found on the mask doubled
// to 32 bits (a & a >> 1: runs of 2, then 4, 8, and the ninth).
MCS_ORB_HD bool orb_fast_test(const uint8_t *p, int step, int t)
{
    const int c = p[0];
    uint32_t br = 0, dk = 0;
    for (int i = 0; i < 16; i++) {
        const int v = p[kFastCircle[i][1] * step + kFastCircle[i][0]];
        br |= (uint32_t)(v > c + t) << i;
        dk |= (uint32_t)(v < c - t) << i;
    }
    br |= br << 16;
    dk |= dk << 16;
    uint32_t a = br & (br >> 1), b = dk & (dk >> 1);
    a &= a >> 2;
    b &= b >> 2;
    a &= a >> 4;
    b &= b >> 4;
    a &= br >> 8;
    b &= dk >> 8;
    return ((a | b) & 0xffffu) != 0;
}

// Necessary condition for orb_fast_test: any 9 contiguous circle positions hold two cyclically
// adjacent cardinal positions (0, 4, 8, 12 -- spacing 4), so a corner has such a pair both
// brighter than I_c + t or both darker than I_c - t.  A cheap filter ahead of the full test.
MCS_ORB_HD bool orb_fast_pretest(const uint8_t *p, int step, int t)
{
    const int c = p[0];
    const int v0 = p[3 * step], v4 = p[3], v8 = p[-3 * step], v12 = p[-3];
    const uint32_t br = (uint32_t)(v0 > c + t) | (uint32_t)(v4 > c + t) << 1 |
                        (uint32_t)(v8 > c + t) << 2 | (uint32_t)(v12 > c + t) << 3;
    const uint32_t dk = (uint32_t)(v0 < c - t) | (uint32_t)(v4 < c - t) << 1 |
                        (uint32_t)(v8 < c - t) << 2 | (uint32_t)(v12 < c - t) << 3;
    // adjacent pairs (0,4) (4,8) (8,12) (12,0): bit k and bit (k + 1) mod 4
    const uint32_t rb = br & ((br >> 1) | (br << 3)), rd = dk & ((dk >> 1) | (dk << 3));
    return ((rb | rd) & 15u) != 0;
}

// 3x3 Sobel gradients at p.
MCS_ORB_HD void orb_sobel(const uint8_t *p, int step, int &ix, int &iy)
{
    ix = ((int)p[-step + 1] + 2 * p[1] + p[step + 1]) -
         ((int)p[-step - 1] + 2 * p[-1] + p[step - 1]);
    iy = ((int)p[step - 1] + 2 * p[step] + p[step + 1]) -
         ((int)p[-step - 1] + 2 * p[-step] + p[-step + 1]);
}

// |Ix|, |Iy| <= 4 * 255, so each of the 49-term sums stays below 49 * 1020^2 < 2^31: 32-bit
// accumulators are exact (the products of the final combination need 64 bits).
MCS_ORB_HD double orb_harris(const uint8_t *p, int step)
{
    int32_t a = 0, b = 0, c = 0;
    for (int v = -3; v <= 3; v++)
        for (int u = -3; u <= 3; u++) {
            int ix, iy;
            orb_sobel(p + v * step + u, step, ix, iy);
            a += ix * ix;
            b += iy * iy;
            c += ix * iy;
        }
    const double t = (double)((int64_t)a + b);
    return (double)((int64_t)a * b - (int64_t)c * c) - 0.04 * (t * t);
}

// (cos, sin) of the intensity-centroid orientation at p (level image, unblurred).
MCS_ORB_HD void orb_orientation(const uint8_t *p, int step, double &cs, double &sn)
{
    int64_t m10 = 0, m01 = 0;
    for (int u = -kOrbHalfPatch; u <= kOrbHalfPatch; u++) m10 += u * (int)p[u];
    for (int v = 1; v <= kOrbHalfPatch; v++) {
        int64_t vs = 0;
        const int d = kOrbUmax[v];
        for (int u = -d; u <= d; u++) {
            const int a = p[u + v * step], b = p[u - v * step];
            vs += a - b;
            m10 += (int64_t)u * (a + b);
        }
        m01 += v * vs;
    }
    const double x = (double)m10, y = (double)m01;
    const double r = sqrt(x * x + y * y);
    cs = r > 0.0 ? x / r : 1.0;
    sn = r > 0.0 ? y / r : 0.0;
}

// Rotated offset of a pattern point.
MCS_ORB_HD int orb_rot_off(int px, int py, double cs, double sn, int step)
{
    const int ix = (int)rint((double)px * cs - (double)py * sn);
    const int iy = (int)rint((double)px * sn + (double)py * cs);
    return iy * step + ix;
}

}  // namespace mcs
