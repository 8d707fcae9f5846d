// mcs_dev.h -- device helpers shared by the gfx950 code objects of the stitch path
// (mcs_kernels.hip: streaming / prepare / blend kernels; mcs_sweep.hip: the multi-band sweep):
// the OpenCV-exact warpPerspective map, window loads and the fixed-point bilinear tap.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "mcs_kparams.h"

namespace mcs {

__device__ __forceinline__ int sat_i16(int v) { return min(max(v, -32768), 32767); }

// std::max(INT_MIN, std::min(INT_MAX, v)) then cvRound (round half to even).
__device__ __forceinline__ int cv_round_clamped(double v)
{
    const double a = 2147483647.0, b = -2147483648.0;
    v = (v < a) ? v : a;
    v = (b < v) ? v : b;
    return (int)__builtin_rint(v);
}

// WarpPerspectiveInvoker arithmetic for canvas pixel (X, Y) of a stage.  Returns the
// fixed-point source coordinate (1/32 px units for bilinear, whole px for nearest).
template <int INTERP>
__device__ __forceinline__ void map_exact(const KStage &S, int X, int Y, int &xo, int &yo)
{
    const int xb = S.bw_shift >= 0 ? ((X >> S.bw_shift) << S.bw_shift) : (X / S.bw0) * S.bw0;
    const int x1 = X - xb;
    const double dxb = (double)xb, dy = (double)Y, dx1 = (double)x1;
    const double X0 = S.m[0] * dxb + S.m[1] * dy + S.m[2];
    const double Y0 = S.m[3] * dxb + S.m[4] * dy + S.m[5];
    const double W0 = S.m[6] * dxb + S.m[7] * dy + S.m[8];
    double W = W0 + S.m[6] * dx1;
    if (INTERP == MCS_INTER_LINEAR) W = (W != 0.0) ? 32.0 / W : 0.0;
    else W = (W != 0.0) ? 1.0 / W : 0.0;
    xo = cv_round_clamped((X0 + S.m[0] * dx1) * W);
    yo = cv_round_clamped((Y0 + S.m[3] * dx1) * W);
}

// Source coordinate of output pixel (x, y) under stage S, in map_exact's units.  Cylinder
// stages (mcs_plan_create_cylindrical): ray (sin t, h, cos t) of the panorama column/row, rotated
// into the camera (d = R ray, explicit summation order), projected x = f dx / dz + cx; rays
// behind the camera map far outside every frame.
template <int INTERP>
__device__ __forceinline__ void stage_map(const KParams &P, const KStage &S, int x, int y,
                                          int &xo, int &yo)
{
    if (S.kind == kStageHomography) {
        map_exact<INTERP>(S, x + S.offx, y + S.offy, xo, yo);
        return;
    }
    if (S.kind == kStageTable) {
        const int64_t p = 2 * ((int64_t)y * P.out_w + x);
        xo = P.map_tab[p];
        yo = P.map_tab[p + 1];
        return;
    }
    const double sn = P.cyl_tab[2 * x], cs = P.cyl_tab[2 * x + 1];
    const double hv = P.cyl_tab[2 * P.out_w + y];
    const double dx = (S.m[0] * sn + S.m[1] * hv) + S.m[2] * cs;
    const double dy = (S.m[3] * sn + S.m[4] * hv) + S.m[5] * cs;
    const double dz = (S.m[6] * sn + S.m[7] * hv) + S.m[8] * cs;
    if (!(dz > 0.0)) {
        xo = yo = INTERP == MCS_INTER_LINEAR ? -(1 << 25) : -(1 << 20);
        return;
    }
    const double sx = (S.f * dx) / dz + S.cx, sy = (S.f * dy) / dz + S.cy;
    const double k = INTERP == MCS_INTER_LINEAR ? 32.0 : 1.0;
    xo = cv_round_clamped(sx * k);
    yo = cv_round_clamped(sy * k);
}

// 8 bytes starting at byte offset o of a frame of `fbytes` bytes (only the first NB are used).
// Unaligned dwordx2 in the common case; an in-bounds dword path at the very end of a frame.
template <int NB>
__device__ __forceinline__ uint2 load8(const uint8_t *fb, int64_t o, int64_t fbytes)
{
    uint2 r;
    if (o + 8 <= fbytes) {
        __builtin_memcpy(&r, fb + o, 8);
    } else {
        const uint32_t *p = reinterpret_cast<const uint32_t *>(fb + (o & ~int64_t(3)));
        const uint32_t sh = (uint32_t)o & 3u;
        const uint32_t last = (sh + NB - 1) >> 2;
        const uint32_t w0 = p[0];
        const uint32_t w1 = p[last < 1 ? last : 1];
        const uint32_t w2 = p[last < 2 ? last : 2];
        r.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
        r.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
    }
    return r;
}

__device__ __forceinline__ uint32_t byte_of(uint2 v, int i)
{
    return ((i < 4 ? v.x : v.y) >> (8 * (i & 3))) & 0xffu;
}

// remapBilinear / remapNearest for one pixel, BORDER_CONSTANT 0.  Returns the CN channel bytes
// packed little-endian in one uint32 (byte k = channel k).  (A per-channel uint32 array here was
// turned into <3 x i32> phis with poison lanes, which the ROCm 7.2 gfx950 backend miscompiled:
// the fully-outside branch returned a stale register instead of 0.  One scalar avoids that.)
template <int CN, int INTERP>
__device__ __forceinline__ uint32_t sample(const uint8_t *fb, int sw, int sh, int64_t fbytes,
                                           int X, int Y)
{
    const int64_t pitch = (int64_t)sw * CN;
    if (INTERP == MCS_INTER_NEAREST) {
        const int sx = sat_i16(X), sy = sat_i16(Y);
        if ((unsigned)sx < (unsigned)sw && (unsigned)sy < (unsigned)sh) {
            const uint2 v = load8<CN>(fb, sy * pitch + (int64_t)sx * CN, fbytes);
            return CN == 4 ? v.x : (v.x & ((1u << (8 * CN)) - 1u));
        }
        return 0u;
    }
    const int sx = sat_i16(X >> 5), sy = sat_i16(Y >> 5);
    const int fx = X & 31, fy = Y & 31;
    // 15-bit weights of initInterTab2D: 32*(32-fx)*(32-fy) ... (sum 32768; the (0,0) entry's
    // 32767/0/0/1 table quirk gives the same u8 result, see tests/test_oracle_known_answers.py)
    const int w00 = (32 - fx) * (32 - fy) * 32, w01 = fx * (32 - fy) * 32;
    const int w10 = (32 - fx) * fy * 32, w11 = fx * fy * 32;
    uint32_t r = 0;
    if ((unsigned)sx < (unsigned)(sw - 1) && (unsigned)sy < (unsigned)(sh - 1)) {
        const int64_t o = sy * pitch + (int64_t)sx * CN;
        const uint2 r0 = load8<2 * CN>(fb, o, fbytes);
        const uint2 r1 = load8<2 * CN>(fb, o + pitch, fbytes);
#pragma unroll
        for (int k = 0; k < CN; k++) {
            const int s = (int)byte_of(r0, k) * w00 + (int)byte_of(r0, CN + k) * w01 +
                          (int)byte_of(r1, k) * w10 + (int)byte_of(r1, CN + k) * w11;
            r |= (uint32_t)((s + 16384) >> 15) << (8 * k);
        }
    } else if (sx < sw && sx + 1 >= 0 && sy < sh && sy + 1 >= 0) {
        // partial border: the taps outside the image read the border value 0
        const bool x0ok = sx >= 0, x1ok = sx + 1 < sw, y0ok = sy >= 0, y1ok = sy + 1 < sh;
        const uint8_t *r0 = fb + sy * pitch, *r1 = r0 + pitch;
#pragma unroll
        for (int k = 0; k < CN; k++) {
            const int v0 = (x0ok && y0ok) ? r0[sx * CN + k] : 0;
            const int v1 = (x1ok && y0ok) ? r0[(sx + 1) * CN + k] : 0;
            const int v2 = (x0ok && y1ok) ? r1[sx * CN + k] : 0;
            const int v3 = (x1ok && y1ok) ? r1[(sx + 1) * CN + k] : 0;
            r |= (uint32_t)((v0 * w00 + v1 * w01 + v2 * w10 + v3 * w11 + 16384) >> 15) << (8 * k);
        }
    }
    return r;   // all four taps outside: the border value 0
}

// Stage that owns output pixel (x, y): the outermost stage whose paste rect does not contain
// it (-1 = camera 0, reached through every rect).
__device__ __forceinline__ int owner(const KParams &P, int x, int y)
{
    int sel = -1;
    bool in = true;
    for (int s = P.n_stages - 1; s >= 0; --s) {
        const KStage &S = P.st[s];
        const bool r = x >= S.rx0 && x < S.rx1 && y >= S.ry0 && y < S.ry1;
        sel = (in && !r) ? s : sel;
        in = in && r;
    }
    return sel;
}

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// 8 bytes of LDS starting at byte a (any alignment): three dword reads + v_alignbyte.  (An
// unaligned ds_read_b64 is legal on gfx950 but measured 2.5x slower in the streaming kernel.)
__device__ __forceinline__ uint2 lds_window(const uint8_t *smem, uint32_t a)
{
    const lds_u32 *d = (const lds_u32 *)(((const lds_u8 *)smem) + (a & ~3u));
    const uint32_t sh = a & 3u;
    const uint32_t x0 = d[0], x1 = d[1], x2 = d[2];
    uint2 r;
    r.x = __builtin_amdgcn_alignbyte(x1, x0, sh);
    r.y = __builtin_amdgcn_alignbyte(x2, x1, sh);
    return r;
}

// Bilinear weights of the stitch kernels as u16 pairs: remapBilinear's 15-bit weight w (the four
// sum to 32768) is stored doubled, min(2 w, 65535), so that a channel's sum
// s = sum p (2 w) + 32768 carries (sum p w + 2^14) >> 15 -- remapBilinear's value -- in its
// byte 2.  (Only fx = fy = 0 gives w = 32768, all on one tap: 65535 p + 32768 still has p in
// byte 2.)  pack_b2 then assembles output bytes with v_perm instead of shift + or per byte.
__device__ __forceinline__ uint32_t w2x(uint32_t w) { return w >= 32768u ? 65535u : 2u * w; }

// Channel k of a pixel from its two row windows (v_perm_b32 + 2 x v_dot2_u32_u16): the result
// byte is byte 2 of the returned sum (bits 24+ are 0).
template <int CN>
__device__ __forceinline__ uint32_t blend(uint2 r0, uint2 r1, uint32_t w0, uint32_t w1, int k)
{
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const uint32_t sel = (uint32_t)k | (0x0cu << 8) | ((uint32_t)(CN + k) << 16) | (0x0cu << 24);
    const uint32_t a0 = __builtin_amdgcn_perm(r0.y, r0.x, sel);
    const uint32_t a1 = __builtin_amdgcn_perm(r1.y, r1.x, sel);
    uint32_t s = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, a0), __builtin_bit_cast(us2, w0),
                                        32768u, false);
    s = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, a1), __builtin_bit_cast(us2, w1), s, false);
    return s;
}

// Byte 2 of a, b, c, d as the bytes 0..3 of one word (two v_perm + or).
__device__ __forceinline__ uint32_t pack_b2(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    return __builtin_amdgcn_perm(b, a, 0x0c0c0602u) | __builtin_amdgcn_perm(d, c, 0x06020c0cu);
}

}  // namespace mcs
