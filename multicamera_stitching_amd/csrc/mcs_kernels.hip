// mcs_kernels.hip -- gfx950 kernels of the stitch hot path.
//
// stitch_gather: renders the FINAL mosaic of the reference chain
// (PostScripts/Stitcher/StitcherClass.py:114-136 -> :211-256) in one pass, one output pixel
// once.  Per pixel: (1) ownership walk through the nested paste rectangles (integer compares
// against wave-uniform kernargs), (2) OpenCV-exact projective map of its canvas coordinate
// (FP64 in OpenCV's operation order, 64-column block start, round-half-even -- Appendix A of
// SURVEY.md), (3) 4-tap 15-bit fixed-point bilinear (or nearest) gather from that camera, border
// 0.  Layout: each lane owns 4 consecutive pixels of one row (12 B for BGR -> one dwordx3
// store), a wave owns 256 contiguous pixels of a row, a 256-thread block 256 x 16 pixels of one
// frame; grid.z walks the frames of a batch.
//
// Built device-only (hipcc --offload-device-only --no-gpu-bundle-output) into a gfx950 code
// object embedded in libmcs.so; the host launches the extern "C" entry points at the bottom
// through hipModuleLaunchKernel.  -ffp-contract=off: no FMA contraction, like OpenCV's
// SSE2/SSE4.1 x86 code.
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

// The lane's 4*CN output bytes as four scalar words (scalars, not an array: small arrays become
// <N x i32> vectors whose poison-lane phis the gfx950 backend has miscompiled, see sample()).
struct OutWords {
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    __device__ __forceinline__ void or_at(int i, uint32_t v)
    {
        if (i == 0) w0 |= v;
        else if (i == 1) w1 |= v;
        else if (i == 2) w2 |= v;
        else w3 |= v;
    }
    __device__ __forceinline__ uint32_t at(int i) const
    {
        return i == 0 ? w0 : (i == 1 ? w1 : (i == 2 ? w2 : w3));
    }
};

// Inserts pixel p's packed bytes (channel k = byte k of v) into the lane's output words.
template <int CN>
__device__ __forceinline__ void put_px(OutWords &w, int p, uint32_t v)
{
#pragma unroll
    for (int k = 0; k < CN; k++) {
        const int b = p * CN + k;   // compile-time after unrolling
        w.or_at(b >> 2, ((v >> (8 * k)) & 0xffu) << (8 * (b & 3)));
    }
}

// ---------------------------------------------------------------------------------------------
// Batched gather.  The geometry is frame-invariant (the reference re-warps every frame with the
// same cachedAH), so each lane evaluates the exact OpenCV map of its 4 pixels ONCE per launch
// into a compact descriptor and then streams every capture of the batch through it.
//
// Every pixel -- bilinear inside the image, bilinear on its border, a paste copy, a nearest
// sample, or outside everything -- is expressed in ONE form: two row windows of 2*CN bytes
// (row 0 at off0, row 1 at off1) and 15-bit weights packed as u16 pairs W0 = (w00, w01),
// W1 = (w10, w11), so that per channel k
//     out_k = dot2(row1_k, W1, dot2(row0_k, W0, 16384)) >> 15            (v_dot2_u32_u16)
// which is remapBilinear's sum(p * w) + 2^14 >> 15 exactly.  A copy is W0 = (32768, 0),
// W1 = 0; a pixel outside every camera has W0 = W1 = 0; taps outside the image get weight 0
// and their window is moved onto valid bytes (so nothing outside a frame is ever read, see
// place_window()).  No per-pixel branching remains in the frame loop except the rare
// "window would end past the frame" case (last pixels of a frame), flagged in `slow`.
template <bool OFF32>
struct Desc {
    typedef typename std::conditional<OFF32, uint32_t, uint64_t>::type off_t;
    off_t off0, off1;      // window byte offsets from the launch base (or absolute addresses)
    uint32_t w0, w1;       // packed u16 weight pairs (w00, w01), (w10, w11)
    uint32_t shift;        // bits 0-3 / 4-7: bytes row 0 / row 1 were moved left to end in-frame
};

// Column placement of one row's tap pair (sx, sx+1) with weights (wl, wr): returns the window's
// first column cx (the window covers cx, cx+1) and the weights as seen from the window.
__device__ __forceinline__ int place_cols(int sx, int sw, uint32_t wl, uint32_t wr, uint32_t &wa,
                                          uint32_t &wb)
{
    const bool l_in = sx >= 0 && sx < sw, r_in = sx + 1 >= 0 && sx + 1 < sw;
    if (l_in && r_in) {
        wa = wl;
        wb = wr;
        return sx;
    }
    if (l_in) {                  // sx = sw - 1: its right neighbour is outside the image
        if (sw >= 2) {
            wa = 0u;
            wb = wl;
            return sx - 1;
        }
        wa = wl;
        wb = 0u;
        return sx;
    }
    if (r_in) {                  // sx = -1: only column 0 contributes
        wa = wr;
        wb = 0u;
        return 0;
    }
    wa = wb = 0u;                // both taps outside: weight 0, any in-image window
    return 0;
}

// Geometry of one output pixel: the camera it samples, its two row windows (in-image row and
// byte column of each window's first tap) and the packed u16 weight pairs seen from them.
struct Geo {
    int cam, r0, c0, r1, c1;
    uint32_t w0, w1;
};

template <int CN, int INTERP>
__device__ __forceinline__ Geo describe_geo(const KParams &P, int x, int y)
{
    Geo g;
    const int s = owner(P, x, y);
    int sw, sh, X, Y;
    if (s < 0) {                 // camera 0 pasted whole: a copy (weights 32768, 0, 0, 0)
        g.cam = 0;
        sw = P.cam0_w;
        sh = P.cam0_h;
        X = (x + P.cam0_offx) << 5;
        Y = (y + P.cam0_offy) << 5;
    } else {
        const KStage &S = P.st[s];
        g.cam = S.cam;
        sw = S.src_w;
        sh = S.src_h;
        map_exact<INTERP>(S, x + S.offx, y + S.offy, X, Y);
        if (INTERP == MCS_INTER_NEAREST) {   // remapNearest: a copy of (X, Y) or the border value
            X = sat_i16(X);
            Y = sat_i16(Y);
            const bool in = (unsigned)X < (unsigned)sw && (unsigned)Y < (unsigned)sh;
            X = in ? X * 32 : -(1 << 20);
            Y = in ? Y * 32 : -(1 << 20);
        }
    }
    const int sx = sat_i16(X >> 5), sy = sat_i16(Y >> 5), fx = X & 31, fy = Y & 31;
    const uint32_t w00 = (32 - fx) * (32 - fy) * 32, w01 = fx * (32 - fy) * 32;
    const uint32_t w10 = (32 - fx) * fy * 32, w11 = fx * fy * 32;
    const bool y0_in = sy >= 0 && sy < sh, y1_in = sy + 1 >= 0 && sy + 1 < sh;
    uint32_t a0, b0, a1, b1;
    g.c0 = place_cols(sx, sw, y0_in ? w00 : 0u, y0_in ? w01 : 0u, a0, b0) * CN;
    g.c1 = place_cols(sx, sw, y1_in ? w10 : 0u, y1_in ? w11 : 0u, a1, b1) * CN;
    g.r0 = y0_in ? sy : 0;
    g.r1 = y1_in ? sy + 1 : 0;
    g.w0 = a0 | (b0 << 16);
    g.w1 = a1 | (b1 << 16);
    if (g.w0 == 0u) {            // no live tap in row 0: reuse row 1's window
        g.r0 = g.r1;
        g.c0 = g.c1;
    }
    if (g.w1 == 0u) {
        g.r1 = g.r0;
        g.c1 = g.c0;
    }
    return g;
}

// Global-gather form of a pixel (tiles whose footprint does not fit the LDS budget).
template <int CN, int INTERP, bool OFF32>
__device__ __forceinline__ Desc<OFF32> describe(const KParams &P, int x, int y)
{
    const Geo g = describe_geo<CN, INTERP>(P, x, y);
    Desc<OFF32> d;
    const int64_t pitch = (int64_t)P.cam_w[g.cam] * CN, fbytes = pitch * P.cam_h[g.cam];
    const int64_t o0 = (int64_t)g.r0 * pitch + g.c0, o1 = (int64_t)g.r1 * pitch + g.c1;
    // an 8-byte window must end inside the frame: move it left, remember by how much
    const int64_t sh0 = o0 + 8 > fbytes ? o0 + 8 - fbytes : 0;
    const int64_t sh1 = o1 + 8 > fbytes ? o1 + 8 - fbytes : 0;
    const uint64_t cam_off = (uint64_t)(uintptr_t)P.cams[g.cam] - (uint64_t)(uintptr_t)P.base;
    d.off0 = (typename Desc<OFF32>::off_t)(cam_off + (uint64_t)(o0 - sh0));
    d.off1 = (typename Desc<OFF32>::off_t)(cam_off + (uint64_t)(o1 - sh1));
    d.w0 = g.w0;
    d.w1 = g.w1;
    d.shift = (uint32_t)sh0 | ((uint32_t)sh1 << 4);
    return d;
}

// Channel k of a pixel from its two row windows: v_perm_b32 + 2 x v_dot2_u32_u16.
template <int CN>
__device__ __forceinline__ uint32_t blend(uint2 r0, uint2 r1, uint32_t w0, uint32_t w1, int k)
{
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const uint32_t sel = (uint32_t)k | (0x0cu << 8) | ((uint32_t)(CN + k) << 16) | (0x0cu << 24);
    const uint32_t a0 = __builtin_amdgcn_perm(r0.y, r0.x, sel);
    const uint32_t a1 = __builtin_amdgcn_perm(r1.y, r1.x, sel);
    uint32_t s = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, a0), __builtin_bit_cast(us2, w0),
                                        16384u, false);
    s = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, a1), __builtin_bit_cast(us2, w1), s, false);
    return s >> 15;
}

__device__ __forceinline__ uint2 shr_bytes(uint2 v, uint32_t n)
{
    uint64_t t;
    __builtin_memcpy(&t, &v, 8);
    t >>= 8 * n;
    __builtin_memcpy(&v, &t, 8);
    return v;
}

// Direct global-gather path for the 4 pixels at (xg, y): descriptors once, then every capture
// (frame stride P.cam_fstride[0] for all cameras; the host splits batches that differ).
template <int CN, int INTERP, bool OFF32>
__device__ __forceinline__ void stitch_direct(const KParams &P, int n_frames, int xg, int y)
{
    const int npx = min(kPx, P.out_w - xg);
    Desc<OFF32> d[kPx];
    uint32_t any_shift = 0;
#pragma unroll
    for (int p = 0; p < kPx; p++) {
        d[p] = describe<CN, INTERP, OFF32>(P, min(xg + p, P.out_w - 1), y);
        any_shift |= d[p].shift;
    }
    const int64_t fstride = P.cam_fstride[0];
    uint8_t *dst = P.out + (int64_t)y * P.out_pitch + (int64_t)xg * CN;
    const bool wide = npx == kPx && (((uintptr_t)dst | (uintptr_t)P.out_fstride) & 3) == 0;
    for (int f = 0; f < n_frames; f++) {
        const uint8_t *bf = P.base + (int64_t)f * fstride;
        uint2 r0[kPx], r1[kPx];
#pragma unroll
        for (int p = 0; p < kPx; p++) {
            __builtin_memcpy(&r0[p], bf + d[p].off0, 8);
            __builtin_memcpy(&r1[p], bf + d[p].off1, 8);
        }
        if (any_shift) {         // windows moved left at a frame's end (last pixels only)
#pragma unroll
            for (int p = 0; p < kPx; p++) {
                r0[p] = shr_bytes(r0[p], d[p].shift & 15u);
                r1[p] = shr_bytes(r1[p], d[p].shift >> 4);
            }
        }
        OutWords w;
#pragma unroll
        for (int p = 0; p < kPx; p++)
#pragma unroll
            for (int k = 0; k < CN; k++) {
                const int b = p * CN + k;
                w.or_at(b >> 2, blend<CN>(r0[p], r1[p], d[p].w0, d[p].w1, k) << (8 * (b & 3)));
            }
        uint8_t *o = dst + (int64_t)f * P.out_fstride;
        if (wide) {
            uint32_t *o32 = reinterpret_cast<uint32_t *>(o);
#pragma unroll
            for (int i = 0; i < CN; i++) o32[i] = w.at(i);
        } else {
            for (int b = 0; b < npx * CN; b++) o[b] = (uint8_t)(w.at(b >> 2) >> (8 * (b & 3)));
        }
    }
}

// ---------------------------------------------------------------------------------------------
// LDS-staged gather (the main path).  Per launch, every block (256 x 8 output pixels, 8 waves)
// evaluates its pixels' exact maps, reduces them to one source footprint per camera (rows x
// 16-byte chunks, the union of all its row windows) and lays the footprints out in LDS.  Per
// capture, each footprint row is ONE global_load_lds_dwordx4 wave instruction (LDS-DMA: wide,
// contiguous, no registers), double-buffered across captures; pixels then read their 8-byte
// windows from LDS with aligned ds_read2_b32 + ds_read_b32 and v_alignbyte.  Blocks whose
// footprint exceeds kLdsBuf (steep perspective, 3+ cameras in one tile) take the direct path.
struct LdsHeader {
    int rmin[MCS_MAX_CAMS], rmax[MCS_MAX_CAMS], cmin[MCS_MAX_CAMS], cmax[MCS_MAX_CAMS];
    int base[MCS_MAX_CAMS], stride[MCS_MAX_CAMS], cal[MCS_MAX_CAMS];
    int jobstart[MCS_MAX_CAMS + 1];
    int fits, njobs;
};
static_assert(sizeof(LdsHeader) <= kLdsHeader, "LDS header");

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

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

// Issues the LDS-DMA loads of capture f's footprint rows into buffer `buf` (rows split over the
// block's waves; lanes = 16-byte chunks of a row).  Chunks that would cross the end of a camera
// frame are copied byte by byte instead (only the bytes inside the frame).
template <int CN>
__device__ __forceinline__ void stage_capture(const KParams &P, const LdsHeader *h, uint8_t *buf,
                                              int f, int lane, int wave)
{
    const int njobs = h->njobs;
    for (int j = wave; j < njobs; j += kWavesPerBlock) {
        int c = 0;
        while (j >= h->jobstart[c + 1]) c++;
        c = __builtin_amdgcn_readfirstlane(c);
        const int row = j - h->jobstart[c];
        const int stride = __builtin_amdgcn_readfirstlane(h->stride[c]);
        const int64_t pitch = (int64_t)P.cam_w[c] * CN;
        const int64_t fbytes = pitch * P.cam_h[c];
        const int64_t goff = (int64_t)(h->rmin[c] + row) * pitch + h->cal[c] + 16 * lane;
        const uint8_t *src = P.cams[c] + (int64_t)f * P.cam_fstride[0];
        const uint32_t lds_row = (uint32_t)(h->base[c] + row * stride);
        lds_u8 *dst = ((lds_u8 *)buf) + __builtin_amdgcn_readfirstlane(lds_row);
        if (16 * lane < stride) {
            if (goff + 16 <= fbytes) {
                __builtin_amdgcn_global_load_lds(src + goff, dst, 16, 0, 0);
            } else {
                for (int b = 0; b < 16; b++)
                    if (goff + b < fbytes) dst[16 * lane + b] = src[goff + b];
            }
        }
    }
}

template <int CN, int INTERP, bool OFF32>
__device__ __forceinline__ void stitch_lds(const KParams &P, int n_frames, uint8_t *smem)
{
    const int lane = threadIdx.x, wave = threadIdx.y;
    const int tid = wave * kWave + lane;
    const int xg = (blockIdx.x * kWave + lane) * kPx;
    const int y = blockIdx.y * kTileH + wave;
    const bool live = xg < P.out_w && y < P.out_h;
    const int npx = live ? min(kPx, P.out_w - xg) : 0;
    LdsHeader *h = reinterpret_cast<LdsHeader *>(smem);
    if (tid < MCS_MAX_CAMS) {
        h->rmin[tid] = 0x7fffffff;
        h->rmax[tid] = -0x7fffffff;
        h->cmin[tid] = 0x7fffffff;
        h->cmax[tid] = -0x7fffffff;
    }
    __syncthreads();

    // 1. exact map of this lane's pixels, then the per-camera footprint of the block
    Geo g[kPx];
#pragma unroll
    for (int p = 0; p < kPx; p++) {
        g[p] = describe_geo<CN, INTERP>(P, min(xg + p, P.out_w - 1), min(y, P.out_h - 1));
        if (p >= npx) g[p].w0 = g[p].w1 = 0u;
    }
    {
        int cam = -1, rmin = 0x7fffffff, rmax = -0x7fffffff, cmin = 0x7fffffff, cmax = -0x7fffffff;
#pragma unroll
        for (int p = 0; p < kPx; p++) {
            if ((g[p].w0 | g[p].w1) == 0u) continue;
            if (cam < 0) cam = g[p].cam;
            const int r_lo = min(g[p].r0, g[p].r1), r_hi = max(g[p].r0, g[p].r1);
            const int c_lo = min(g[p].c0, g[p].c1), c_hi = max(g[p].c0, g[p].c1);
            if (g[p].cam == cam) {
                rmin = min(rmin, r_lo);
                rmax = max(rmax, r_hi);
                cmin = min(cmin, c_lo);
                cmax = max(cmax, c_hi);
            } else {
                atomicMin(&h->rmin[g[p].cam], r_lo);
                atomicMax(&h->rmax[g[p].cam], r_hi);
                atomicMin(&h->cmin[g[p].cam], c_lo);
                atomicMax(&h->cmax[g[p].cam], c_hi);
            }
        }
        if (cam >= 0) {
            atomicMin(&h->rmin[cam], rmin);
            atomicMax(&h->rmax[cam], rmax);
            atomicMin(&h->cmin[cam], cmin);
            atomicMax(&h->cmax[cam], cmax);
        }
    }
    __syncthreads();
    if (tid == 0) {
        int total = 0, jobs = 0, fits = 1;
        for (int c = 0; c < MCS_MAX_CAMS; c++) {
            h->jobstart[c] = jobs;
            if (h->rmin[c] > h->rmax[c]) continue;
            const int cal = h->cmin[c] & ~15;
            const int stride = (h->cmax[c] + 8 - cal + 15) & ~15;
            const int rows = h->rmax[c] - h->rmin[c] + 1;
            h->cal[c] = cal;
            h->stride[c] = stride;
            h->base[c] = total;
            total += rows * stride;
            jobs += rows;
            if (stride > 16 * kWave) fits = 0;
        }
        h->jobstart[MCS_MAX_CAMS] = jobs;
        h->njobs = jobs;
        h->fits = fits && total <= kLdsBuf;
    }
    __syncthreads();
    if (!h->fits) {              // block-uniform: footprint too large for the LDS budget
        if (live) stitch_direct<CN, INTERP, OFF32>(P, n_frames, xg, y);
        return;
    }

    // 2. LDS window addresses of every pixel (buffer-relative)
    uint32_t win[kPx], w0[kPx], w1[kPx];
#pragma unroll
    for (int p = 0; p < kPx; p++) {
        const int c = g[p].cam;
        const int st = h->stride[c], rm = h->rmin[c], ca = h->cal[c], bs = h->base[c];
        uint32_t a0 = (uint32_t)(bs + (g[p].r0 - rm) * st + (g[p].c0 - ca));
        uint32_t a1 = (uint32_t)(bs + (g[p].r1 - rm) * st + (g[p].c1 - ca));
        if ((g[p].w0 | g[p].w1) == 0u) a0 = a1 = 0u;
        win[p] = a0 | (a1 << 16);
        w0[p] = g[p].w0;
        w1[p] = g[p].w1;
    }

    uint8_t *bufs[2] = {smem + kLdsHeader, smem + kLdsHeader + kLdsBuf + kLdsSlack};
    uint8_t *dst = P.out + (int64_t)min(y, P.out_h - 1) * P.out_pitch + (int64_t)xg * CN;
    const bool wide = npx == kPx && (((uintptr_t)dst | (uintptr_t)P.out_fstride) & 3) == 0;

    // 3. stream the captures: DMA(f+1) || gather(f), one barrier per capture
    stage_capture<CN>(P, h, bufs[0], 0, lane, wave);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int f = 0; f < n_frames; f++) {
        if (f + 1 < n_frames) stage_capture<CN>(P, h, bufs[(f + 1) & 1], f + 1, lane, wave);
        const uint8_t *b = bufs[f & 1];
        if (live) {
            OutWords w;
#pragma unroll
            for (int p = 0; p < kPx; p++) {
                const uint2 r0 = lds_window(b, win[p] & 0xffffu);
                const uint2 r1 = lds_window(b, win[p] >> 16);
#pragma unroll
                for (int k = 0; k < CN; k++) {
                    const int bb = p * CN + k;
                    w.or_at(bb >> 2, blend<CN>(r0, r1, w0[p], w1[p], k) << (8 * (bb & 3)));
                }
            }
            uint8_t *o = dst + (int64_t)f * P.out_fstride;
            if (wide) {
                uint32_t *o32 = reinterpret_cast<uint32_t *>(o);
#pragma unroll
                for (int i = 0; i < CN; i++) o32[i] = w.at(i);
            } else {
                for (int bb = 0; bb < npx * CN; bb++)
                    o[bb] = (uint8_t)(w.at(bb >> 2) >> (8 * (bb & 3)));
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

// Footprint marking: sets mask[cam][pixel] = 1 for every source pixel the mosaic reads with a
// non-zero weight; counts[cam] += number of newly marked pixels.
template <int CN, int INTERP>
__device__ __forceinline__ void footprint_mark(const KParams &P, uint8_t *const *masks,
                                               unsigned long long *counts)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= P.out_w || y >= P.out_h) return;
    const int s = owner(P, x, y);
    auto mark = [&](int cam, int sx, int sy, int w, int h) {
        if ((unsigned)sx < (unsigned)w && (unsigned)sy < (unsigned)h) {
            uint8_t *m = masks[cam] + (int64_t)sy * w + sx;
            if (*m == 0) {
                unsigned int *word = reinterpret_cast<unsigned int *>((uintptr_t)m & ~uintptr_t(3));
                const unsigned int bit = 1u << (8 * ((uintptr_t)m & 3));
                const unsigned int old = atomicOr(word, bit);
                if (!(old & bit)) atomicAdd(&counts[cam], 1ull);
            }
        }
    };
    if (s < 0) {
        mark(0, x + P.cam0_offx, y + P.cam0_offy, P.cam0_w, P.cam0_h);
        return;
    }
    const KStage &S = P.st[s];
    int X, Y;
    map_exact<INTERP>(S, x + S.offx, y + S.offy, X, Y);
    if (INTERP == MCS_INTER_NEAREST) {
        mark(S.cam, sat_i16(X), sat_i16(Y), S.src_w, S.src_h);
    } else {
        const int sx = sat_i16(X >> 5), sy = sat_i16(Y >> 5), fx = X & 31, fy = Y & 31;
        mark(S.cam, sx, sy, S.src_w, S.src_h);
        if (fx) mark(S.cam, sx + 1, sy, S.src_w, S.src_h);
        if (fy) mark(S.cam, sx, sy + 1, S.src_w, S.src_h);
        if (fx && fy) mark(S.cam, sx + 1, sy + 1, S.src_w, S.src_h);
    }
}

}  // namespace mcs

// ---------------------------------------------------------------------------------------------
// Entry points (names looked up by mcs_capi.cpp).  Block shapes: stitch (64, 8, 1) with grid
// (ceil(out_w/256), ceil(out_h/8)) and kLdsBytes of dynamic LDS; footprint (256, 1, 1) with grid
// (ceil(out_w/256), out_h).
#define MCS_STITCH_ENTRY(CN, IN, O32)                                                          \
    extern "C" __global__ __launch_bounds__(512) void mcs_stitch_c##CN##_i##IN##_o##O32(       \
        const mcs::KParams P, int n_frames)                                                    \
    {                                                                                          \
        extern __shared__ __attribute__((aligned(16))) uint8_t smem[];                         \
        mcs::stitch_lds<CN, IN, O32 == 32>(P, n_frames, smem);                                 \
    }
#define MCS_STITCH_ENTRIES(CN)                                                                 \
    MCS_STITCH_ENTRY(CN, 0, 32)                                                                \
    MCS_STITCH_ENTRY(CN, 1, 32)                                                                \
    MCS_STITCH_ENTRY(CN, 0, 64)                                                                \
    MCS_STITCH_ENTRY(CN, 1, 64)
MCS_STITCH_ENTRIES(1)
MCS_STITCH_ENTRIES(2)
MCS_STITCH_ENTRIES(3)
MCS_STITCH_ENTRIES(4)

extern "C" __global__ __launch_bounds__(256) void mcs_footprint_i0(const mcs::KParams P,
                                                                   uint8_t *const *masks,
                                                                   unsigned long long *counts)
{
    mcs::footprint_mark<1, 0>(P, masks, counts);
}

extern "C" __global__ __launch_bounds__(256) void mcs_footprint_i1(const mcs::KParams P,
                                                                   uint8_t *const *masks,
                                                                   unsigned long long *counts)
{
    mcs::footprint_mark<1, 1>(P, masks, counts);
}

// Diagnostic: per output pixel of frame 0, {owner stage, X, Y, packed sampled bytes}.
extern "C" __global__ __launch_bounds__(256) void mcs_debug_pixels_c3(const mcs::KParams P,
                                                                      int *dbg)
{
    using namespace mcs;
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= P.out_w || y >= P.out_h) return;
    const int s = owner(P, x, y);
    int X = 0, Y = 0;
    uint32_t v = 0;
    if (s >= 0) {
        const KStage &S = P.st[s];
        map_exact<MCS_INTER_LINEAR>(S, x + S.offx, y + S.offy, X, Y);
        v = sample<3, MCS_INTER_LINEAR>(P.cams[S.cam], S.src_w, S.src_h,
                                        (int64_t)S.src_w * S.src_h * 3, X, Y);
    }
    int *d = dbg + 4 * ((int64_t)y * P.out_w + x);
    d[0] = s;
    d[1] = X;
    d[2] = Y;
    d[3] = (int)v;
}

// Diagnostic: copies the parameter block as the device sees it (kernarg transport check).
extern "C" __global__ __launch_bounds__(64) void mcs_echo_kparams(const mcs::KParams P,
                                                                  uint8_t *out)
{
    const uint8_t *src = reinterpret_cast<const uint8_t *>(&P);
    for (int i = threadIdx.x; i < (int)sizeof(mcs::KParams); i += 64) out[i] = src[i];
}
