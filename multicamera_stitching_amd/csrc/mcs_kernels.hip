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
#include "mcs_dev.h"

#include "mcs_blend.h"

namespace mcs {

// Stage sampled by output pixel (x, y): the paste rule (owner()) or, in the blended modes, the
// blend owner; -1 = camera 0, -2 = no camera (blended modes only).
template <int INTERP>
__device__ __forceinline__ int pixel_stage(const KParams &P, int x, int y)
{
    if (P.blend == MCS_BLEND_NONE) return owner(P, x, y);
    const int s = blend_owner<INTERP>(P, x, y, nullptr);
    return s == kBlendNone ? -2 : s - 1;
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

// The lane's 4 * CN output bytes from the blend sums of its 4 pixels (channel-interleaved).
template <int CN>
__device__ __forceinline__ OutWords pack_words(const uint32_t (&r)[kPx * CN])
{
    OutWords w;
    w.w0 = pack_b2(r[0], r[1], r[2], r[3]);
    if (CN > 1) w.w1 = pack_b2(r[4 % (kPx * CN)], r[5 % (kPx * CN)], r[6 % (kPx * CN)], r[7 % (kPx * CN)]);
    if (CN > 2) w.w2 = pack_b2(r[8 % (kPx * CN)], r[9 % (kPx * CN)], r[10 % (kPx * CN)], r[11 % (kPx * CN)]);
    if (CN > 3) w.w3 = pack_b2(r[12 % (kPx * CN)], r[13 % (kPx * CN)], r[14 % (kPx * CN)], r[15 % (kPx * CN)]);
    return w;
}

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
// (row 0 at off0, row 1 at off1) and remapBilinear's 15-bit weights stored DOUBLED as u16 pairs
// W0 = (w2x(w00), w2x(w01)), W1 = (w2x(w10), w2x(w11)) (w2x above), so that per channel k
//     s_k = dot2(row1_k, W1, dot2(row0_k, W0, 32768))                    (v_dot2_u32_u16)
// carries remapBilinear's (sum(p * w) + 2^14) >> 15 exactly in its byte 2 (pack_b2 extracts
// it).  A copy is W0 = (65535, 0), W1 = 0; a pixel outside every camera has W0 = W1 = 0; taps
// outside the image get weight 0 and their window is moved onto valid bytes (so nothing outside
// a frame is ever read, see place_cols()).  No per-pixel branching remains in the frame loop
// except the rare "window would end past the frame" case (last pixels of a frame), flagged in
// `shift`.
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
    int cw, ch;                  // the camera's frame size
    const uint8_t *frame;        // its frame 0 (P.cams[cam])
    uint32_t w0, w1;
    int fx, fy;                  // the bilinear fraction (1/32 px)
    bool plain;                  // all four taps in the image (or fy = 0 and both row-0 taps):
                                 // the weights follow from (fx, fy), row 1 = row 0 + 1, c1 = c0
};

template <int CN, int INTERP>
__device__ __forceinline__ Geo describe_geo(const KParams &P, int x, int y)
{
    Geo g;
    const int s = pixel_stage<INTERP>(P, x, y);
    int sw, sh, X, Y;
    g.cam = 0;
    g.cw = P.cam_w[0];
    g.ch = P.cam_h[0];
    g.frame = P.cams[0];
    if (s == -2) {               // no camera: all weights 0 (the border value)
        sw = P.cam0_w;
        sh = P.cam0_h;
        X = Y = -(1 << 20);
    } else if (s < 0) {          // camera 0 pasted whole: a copy (weights 32768, 0, 0, 0)
        sw = P.cam0_w;
        sh = P.cam0_h;
        X = (x + P.cam0_offx) << 5;
        Y = (y + P.cam0_offy) << 5;
    } else {
        sw = sh = X = Y = 0;
    }
    // The stages of the wave's pixels one at a time, each with its parameters read by scalar loads:
    // P.st or P.cams indexed by a per-lane stage are vector loads from the kernel arguments (~40 per
    // wave in the direct stitch).  (P is always a kernel argument here, i.e. in the constant
    // address space, which is what makes the uniform-address reads scalar.)
    typedef __attribute__((address_space(4))) const KParams ckp;
    const ckp *P4 = (const ckp *)&P;
    bool pending = s >= 0;
    for (uint64_t m = __builtin_amdgcn_ballot_w64(pending); m != 0;
         m = __builtin_amdgcn_ballot_w64(pending)) {
        const int s0 = __builtin_amdgcn_readlane(s, (int)__builtin_ctzll(m));
        // (read before the branch: inside it the compiler would address them by the lane's own s,
        // equal to s0 there, with vector loads)
        const KStage S = P4->st[s0];
        const int cw = P4->cam_w[S.cam], ch = P4->cam_h[S.cam];
        const uint8_t *frame = P4->cams[S.cam];
        if (pending && s == s0) {
            g.cam = S.cam;
            g.cw = cw;
            g.ch = ch;
            g.frame = frame;
            sw = S.src_w;
            sh = S.src_h;
            stage_map<INTERP>(P, S, x, y, X, Y);
            if (INTERP == MCS_INTER_NEAREST) {   // remapNearest: a copy of (X, Y) or the border
                X = sat_i16(X);
                Y = sat_i16(Y);
                const bool in = (unsigned)X < (unsigned)sw && (unsigned)Y < (unsigned)sh;
                X = in ? X * 32 : -(1 << 20);
                Y = in ? Y * 32 : -(1 << 20);
            }
            pending = false;
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
    g.w0 = w2x(a0) | (w2x(b0) << 16);
    g.w1 = w2x(a1) | (w2x(b1) << 16);
    g.fx = fx;
    g.fy = fy;
    g.plain = sx >= 0 && sx + 1 < sw && y0_in && (y1_in || fy == 0);
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
    const int64_t pitch = (int64_t)g.cw * CN, fbytes = pitch * g.ch;
    const int64_t o0 = (int64_t)g.r0 * pitch + g.c0, o1 = (int64_t)g.r1 * pitch + g.c1;
    // an 8-byte window must end inside the frame: move it left, remember by how much
    const int64_t sh0 = o0 + 8 > fbytes ? o0 + 8 - fbytes : 0;
    const int64_t sh1 = o1 + 8 > fbytes ? o1 + 8 - fbytes : 0;
    const uint64_t cam_off = (uint64_t)(uintptr_t)g.frame - (uint64_t)(uintptr_t)P.base;
    d.off0 = (typename Desc<OFF32>::off_t)(cam_off + (uint64_t)(o0 - sh0));
    d.off1 = (typename Desc<OFF32>::off_t)(cam_off + (uint64_t)(o1 - sh1));
    d.w0 = g.w0;
    d.w1 = g.w1;
    d.shift = (uint32_t)sh0 | ((uint32_t)sh1 << 4);
    return d;
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
__device__ __forceinline__ void stitch_direct(const KParams &P, int f0, int n_frames, int xg,
                                              int y)
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
    for (int f = f0; f < n_frames; f++) {
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
        uint32_t rr[kPx * CN];
#pragma unroll
        for (int p = 0; p < kPx; p++)
#pragma unroll
            for (int k = 0; k < CN; k++) rr[p * CN + k] = blend<CN>(r0[p], r1[p], d[p].w0, d[p].w1, k);
        const OutWords w = pack_words<CN>(rr);
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
// LDS-staged gather (the main path), in two kernels.
//
// prepare (once per plan): every 256 x 8 tile evaluates its pixels' exact maps, reduces them to
// one source footprint per camera (rows x 16-byte chunks: the union of all its row windows),
// lays the footprints out as one LDS slot, and stores a TileHdr plus each pixel's LDS window
// addresses and weights.  Tiles that do not fit (more than kTileCams cameras, a slot larger than
// half the ring, rows wider than 1 KiB) are listed for the direct-gather kernel instead.
//
// stream (every launch): per capture, each footprint row is ONE global_load_lds_dwordx4 wave
// instruction (LDS-DMA: wide, contiguous, no registers) into a ring of slots, several captures in
// flight; pixels read their 8-byte windows from LDS with aligned ds_read2_b32 + ds_read_b32 and
// v_alignbyte, blend with v_dot2_u32_u16, and store 12 contiguous bytes per lane.

// Output pixel group of (lane, wave) in tile (bx, by): first pixel column xg, row y.
__device__ __forceinline__ void tile_pixel(int bx, int by, int lane, int wave, int &xg, int &y)
{
    xg = (bx * kLanesPerRow + lane % kLanesPerRow) * kPx;
    y = by * kTileH + wave * kRowsPerWave + lane / kLanesPerRow;
}


struct FootprintLds {
    int rmin[MCS_MAX_CAMS], rmax[MCS_MAX_CAMS], cmin[MCS_MAX_CAMS], cmax[MCS_MAX_CAMS];
};

template <int CN, int INTERP>
__device__ __forceinline__ void prepare_tile(const KParams &P, TileHdr *tiles, uint32_t *desc,
                                             uint32_t *desc4, int *fallback, int *big,
                                             uint16_t *spans)
{
    __shared__ FootprintLds fl;
    __shared__ TileHdr th;
    // per footprint row (DMA job): the LDS byte span [lo, hi) the tile's windows read
    __shared__ int span_lo[kMaxTileJobs], span_hi[kMaxTileJobs];
    const int lane = threadIdx.x, wave = threadIdx.y;
    const int tid = wave * kWave + lane;
    const int tile = blockIdx.y * gridDim.x + blockIdx.x;
    int xg, y;
    tile_pixel(blockIdx.x, blockIdx.y, lane, wave, xg, y);
    const bool live = xg < P.out_w && y < P.out_h;
    const int npx = live ? min(kPx, P.out_w - xg) : 0;
    if (tid < MCS_MAX_CAMS) {
        fl.rmin[tid] = 0x7fffffff;
        fl.rmax[tid] = -0x7fffffff;
        fl.cmin[tid] = 0x7fffffff;
        fl.cmax[tid] = -0x7fffffff;
    }
    if (tid < kMaxTileJobs) {
        span_lo[tid] = 0x7fffffff;
        span_hi[tid] = -0x7fffffff;
    }
    __syncthreads();
    Geo g[kPx];
    // (a lane whose pixels the multi-band sweep writes: no footprint, no store -- kCwSkip)
    const bool swept = P.skip && live && P.skip[(int64_t)y * P.out_w + xg];
#pragma unroll
    for (int p = 0; p < kPx; p++) {
        g[p] = describe_geo<CN, INTERP>(P, min(xg + p, P.out_w - 1), min(y, P.out_h - 1));
        if (p >= npx || swept) g[p].w0 = g[p].w1 = 0u;
    }
#pragma unroll
    for (int p = 0; p < kPx; p++) {
        if ((g[p].w0 | g[p].w1) == 0u) continue;
        const int c = g[p].cam;
        atomicMin(&fl.rmin[c], min(g[p].r0, g[p].r1));
        atomicMax(&fl.rmax[c], max(g[p].r0, g[p].r1));
        atomicMin(&fl.cmin[c], min(g[p].c0, g[p].c1));
        atomicMax(&fl.cmax[c], max(g[p].c0, g[p].c1));
    }
    __syncthreads();
    if (tid == 0) {
        int total = 0, jobs = 0, n = 0, fits = 1, shifts = 0;
        for (int c = 0; c < MCS_MAX_CAMS; c++) {
            if (fl.rmin[c] > fl.rmax[c]) continue;
            if (n == kTileCams) {
                fits = 0;
                break;
            }
            const int cal = fl.cmin[c] & ~15;
            const int stride = (fl.cmax[c] + 8 - cal + 15) & ~15;   // DMA bytes per row
            const int lpitch = lds_row_pitch(stride);                 // LDS row spacing
            const int rows = fl.rmax[c] - fl.rmin[c] + 1;
            th.cam[n] = c;
            th.rmin[n] = fl.rmin[c];
            th.cal[n] = cal;
            th.stride[n] = lpitch | ((stride >> 4) << 16);
            th.base[n] = total;
            th.jobstart[n] = jobs;
            total += rows * lpitch;
            jobs += rows;
            if (stride > 16 * kWave) fits = 0;
            // DMA chunks must end inside the camera frame: the frame's last row is fetched from
            // `e` bytes earlier (the bytes it needs end before the frame end, so they are all
            // still covered); the preceding bytes must exist
            const int pitch = P.cam_w[c] * CN;
            if (fl.rmax[c] == P.cam_h[c] - 1 && cal + stride > pitch) {
                const int e = cal + stride - pitch;
                if (e > 255 || (int64_t)fl.rmax[c] * pitch + cal - e < 0) fits = 0;
                else shifts |= e << (8 * n);
            }
            n++;
        }
        for (int k = n; k < kTileCams; k++) {
            th.cam[k] = th.rmin[k] = th.cal[k] = th.stride[k] = th.base[k] = 0;
            th.jobstart[k] = jobs;
        }
        th.jobstart[kTileCams] = jobs;
        th.ncam = n;
        th.njobs = jobs;
        const int buf = (total + kLdsSlack + 15) & ~15;
        th.buf_bytes = buf;
        th.ring = min(kMaxRing, lds_ring_bytes(CN) / buf);
        const bool ok = fits && total < 65536 - kLdsSlack;
        th.fits = ok && th.ring >= 2 && jobs <= kJobsPerWave * kWavesPerBlock;
        if (!th.fits && ok && min(kMaxRing, big_ring_bytes() / buf) >= 2 &&
            jobs <= kBigJobsPerWave * kWavesPerBlock) {
            th.fits = 2;
            th.ring = min(kMaxRing, big_ring_bytes() / buf);
        }
        th.last_shift = shifts;
        th.pad_ = 0;
        tiles[tile] = th;
        if (th.fits == 0) fallback[1 + atomicAdd(&fallback[0], 1)] = tile;
        if (th.fits == 2) big[1 + atomicAdd(&big[0], 1)] = tile;
    }
    __syncthreads();
    uint32_t d[kPx * kDescWords], cw[kPx];
#pragma unroll
    for (int p = 0; p < kPx; p++) {
        int k = 0;
        while (k < th.ncam - 1 && th.cam[k] != g[p].cam) k++;
        const int st = th.stride[k] & 0xffff, rm = th.rmin[k], ca = th.cal[k], bs = th.base[k];
        const int last = P.cam_h[g[p].cam] - 1, e = (th.last_shift >> (8 * k)) & 255;
        uint32_t a0 = (uint32_t)(bs + (g[p].r0 - rm) * st + (g[p].c0 - ca) +
                                 (g[p].r0 == last ? e : 0));
        uint32_t a1 = (uint32_t)(bs + (g[p].r1 - rm) * st + (g[p].c1 - ca) +
                                 (g[p].r1 == last ? e : 0));
        const bool zero = (g[p].w0 | g[p].w1) == 0u || !th.fits;
        if (zero) a0 = a1 = 0u;
        if (!zero) {
            // the row spans: this pixel's two windows (2 CN bytes each) in LDS row coordinates
            const int j0 = th.jobstart[k] + g[p].r0 - rm, j1 = th.jobstart[k] + g[p].r1 - rm;
            const int q0 = (int)a0 - bs - (g[p].r0 - rm) * st;
            const int q1 = (int)a1 - bs - (g[p].r1 - rm) * st;
            if (j0 >= 0 && j0 < kMaxTileJobs) {
                atomicMin(&span_lo[j0], q0);
                atomicMax(&span_hi[j0], q0 + 2 * CN);
            }
            if (j1 >= 0 && j1 < kMaxTileJobs) {
                atomicMin(&span_lo[j1], q1);
                atomicMax(&span_hi[j1], q1 + 2 * CN);
            }
        }
        d[p * kDescWords + 0] = (a0 & 0xffffu) | (a1 << 16);
        d[p * kDescWords + 1] = g[p].w0;
        d[p * kDescWords + 2] = g[p].w1;
        // compact form (kCw*): a plain bilinear pixel is its row-0 window, (fx, fy) and its
        // camera's footprint slot; row 1 is one footprint row further (plus the last-row shift
        // when row 1 is the frame's last row)
        if (swept)
            cw[p] = kCwSkip;
        else if (zero)
            cw[p] = kCwZero;
        else if (!g[p].plain)
            cw[p] = kCwFull;
        else
            cw[p] = (a0 & 0xffffu) | ((uint32_t)g[p].fx << 16) | ((uint32_t)g[p].fy << 21) |
                    ((uint32_t)k << 26) | (g[p].fy == 0 ? kCwOneRow : 0u) |
                    (g[p].fy != 0 && g[p].r1 == last && e ? kCwLastRow1 : 0u);
    }
    reinterpret_cast<uint4 *>(desc4)[(int64_t)tile * (kTilePx / kPx) + tid] =
        make_uint4(cw[0], cw[1], cw[2], cw[3]);
    __syncthreads();
    if (tid < kMaxTileJobs) {
        // first chunk | chunk count (>= 1: a row no window reads still issues its one DMA
        // instruction, of one chunk, so every job counts in the streaming kernel's vmcnt waits)
        int lo = span_lo[tid], hi = span_hi[tid];
        const int c0 = lo <= hi ? lo >> 4 : 0, c1 = lo <= hi ? (hi + 15) >> 4 : 1;
        spans[(int64_t)tile * kMaxTileJobs + tid] = (uint16_t)(c0 | (max(c1 - c0, 1) << 8));
    }
    uint4 *o = reinterpret_cast<uint4 *>(desc + ((int64_t)tile * kTilePx + (int64_t)tid * kPx) *
                                                    kDescWords);
#pragma unroll
    for (int i = 0; i < kPx * kDescWords / 4; i++)
        o[i] = make_uint4(d[4 * i], d[4 * i + 1], d[4 * i + 2], d[4 * i + 3]);
}

// Cache policy of the footprint DMA: default (aux 0; nontemporal measured 12 % slower: vertically
// adjacent tiles re-read footprint rows from L2).  The mosaic stores are nontemporal: the mosaic
// is written once and never re-read by this launch (same-box A/B paste 0.62 -> 0.60 ms,
// multi-band 0.978 -> 0.951 ms).
constexpr int kDmaAux = 0;


// Block-uniform value read from LDS (broadcast read + readfirstlane -> SGPR).
__device__ __forceinline__ int uni(const int &v) { return __builtin_amdgcn_readfirstlane(v); }

// The LDS-DMA jobs of one wave, resolved once per block.  Every chunk lies inside its camera frame
// (TileHdr::last_shift).
//   BUF (every byte of every capture of every used camera within 4 GiB of P.base): offsets from
//   P.base, read through one buffer resource (buffer_load_dwordx4 ... offen lds), the capture's
//   offset f * fstride in the instruction's scalar offset -- no per-row 64-bit address math;
//   otherwise 64-bit frame-0 addresses for global_load_lds_dwordx4.
// Jobs are 1 KiB LDS windows: a camera's footprint rows lie in LDS at a
// uniform pitch (a multiple of 128 B), so the 64 lanes of one LDS-DMA instruction -- lane L writes
// 16 bytes at M0 + 16 L -- can cover 1 KiB of consecutive rows: lane L takes row
// (16 L + 1024 w) / pitch, chunk ((16 L + 1024 w) % pitch) / 16, and is enabled only where that
// chunk lies in its row's span.  A 512-B pitch (C2's 128-pixel tiles) moves 2 rows per
// instruction instead of 1, a 256-B pitch 4: half the DMA instructions per capture or fewer, and
// the same bytes.  Every window issues its instruction (a window no span reaches enables lane 0,
// whose 16 bytes land outside every span: no pixel reads them), so the counted vmcnt waits hold.
constexpr int kDmaWindow = 16 * kWave;     // bytes of LDS one window job fills

template <bool BUF, int NJ>
struct WaveWins {
    typedef typename std::conditional<BUF, uint32_t, const uint8_t *>::type src_t;
    src_t src[NJ];       // per lane: frame-0 offset (BUF) / address of its 16 bytes
    uint32_t lds[NJ];    // LDS offset of the window in slot 0 (wave-uniform)
    bool on[NJ];         // per lane: the chunk is in its row's span
    int n;               // windows of this wave
    int total;           // windows of the tile
};

template <int CN, bool BUF, int NJ>
__device__ __forceinline__ WaveWins<BUF, NJ> wave_windows(const KParams &P, const TileHdr &h,
                                                          int wave, const uint16_t *spans, int lane)
{
    WaveWins<BUF, NJ> J;
    const int ncam = uni(h.ncam);
    int wst[kTileCams + 1];
    wst[0] = 0;
#pragma unroll
    for (int k = 0; k < kTileCams; k++) {
        const int rows = uni(h.jobstart[k + 1]) - uni(h.jobstart[k]);
        const int pitch = uni(h.stride[k]) & 0xffff;
        wst[k + 1] = wst[k] + (k < ncam ? (rows * pitch + kDmaWindow - 1) / kDmaWindow : 0);
    }
    J.total = wst[kTileCams];
    J.n = 0;
#pragma unroll
    for (int jj = 0; jj < NJ; jj++) {
        const int j = wave + jj * kWavesPerBlock;
        J.src[jj] = 0;
        J.lds[jj] = 0;
        J.on[jj] = false;
        if (j < J.total) {
            int k = 0;
            while (k < kTileCams - 1 && j >= wst[k + 1]) k++;
            const int c = uni(h.cam[k]);
            const int pitch = uni(h.stride[k]) & 0xffff;
            const int rows = uni(h.jobstart[k + 1]) - uni(h.jobstart[k]);
            const int off = (j - wst[k]) * kDmaWindow + 16 * lane;
            const int ri = off / pitch, ch = (off - ri * pitch) >> 4;
            const uint32_t sp = ri < rows ? (uint32_t)spans[uni(h.jobstart[k]) + ri] : 0u;
            const int lo = (int)(sp & 0xffu), n = (int)((sp >> 8) & 0xffu);
            bool on = ri < rows && ch >= lo && ch < lo + n;
            // (a window no span reaches still issues its instruction: lane 0, row ri's chunk 0)
            const bool none = __builtin_amdgcn_ballot_w64(on) == 0;
            const int cch = none ? 0 : ch;
            on = on || (none && lane == 0);
            const int r = uni(h.rmin[k]) + min(ri, rows - 1);
            const int64_t pitch_f = (int64_t)P.cam_w[c] * CN;
            const int e = r == P.cam_h[c] - 1 ? (uni(h.last_shift) >> (8 * k)) & 255 : 0;
            const int64_t in_frame = (int64_t)r * pitch_f + uni(h.cal[k]) - e + 16 * cch;
            if constexpr (BUF)
                J.src[jj] = (uint32_t)((uint64_t)(uintptr_t)P.cams[c] -
                                       (uint64_t)(uintptr_t)P.base + (uint64_t)in_frame);
            else
                J.src[jj] = P.cams[c] + in_frame;
            // (LDS offset from the block's LDS base: the ring follows the tile header)
            J.lds[jj] = (uint32_t)(sizeof(TileHdr) + uni(h.base[k]) + (j - wst[k]) * kDmaWindow);
            J.on[jj] = on;
            J.n = jj + 1;
        }
    }
    return J;
}

// Issues capture f's footprint windows into `slot`: one LDS-DMA wave instruction per window,
// windows JJ .. n-1 of the wave (a uniform exit after the last: no mask test per absent window).
template <int JJ, bool BUF, int NJ>
__device__ __forceinline__ void stage_windows_from(const WaveWins<BUF, NJ> &J,
                                                   __amdgpu_buffer_rsrc_t rs, uint8_t *slot,
                                                   int64_t foff)
{
    if constexpr (JJ < NJ) {
        if (JJ >= J.n) return;
        if (J.on[JJ]) {
            if constexpr (BUF)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, ((lds_u8 *)slot) + J.lds[JJ], 16,
                                                         J.src[JJ], (int)(uint32_t)foff, 0,
                                                         kDmaAux);
            else
                __builtin_amdgcn_global_load_lds(J.src[JJ] + foff, ((lds_u8 *)slot) + J.lds[JJ],
                                                 16, 0, kDmaAux);
        }
        stage_windows_from<JJ + 1, BUF, NJ>(J, rs, slot, foff);
    }
}
template <bool BUF, int NJ>
__device__ __forceinline__ void stage_windows(const WaveWins<BUF, NJ> &J,
                                              __amdgpu_buffer_rsrc_t rs, uint8_t *slot,
                                              int64_t foff)
{
    stage_windows_from<0, BUF, NJ>(J, rs, slot, foff);
}

// s_waitcnt vmcnt(n) + lgkmcnt(0) for a block-uniform run-time n (0 <= n <= 15; waiting for fewer
// outstanding operations is always safe), as a computed jump: `entry` = 8 n + 12 selects entry n of a table of
// `s_waitcnt vmcnt(n) lgkmcnt(0); s_branch end` pairs (8 bytes each) that starts 12 bytes past
// the s_getpc_b64 result (the address of the instruction after it: s_add_u32, s_addc_u32 and
// s_setpc_b64 are 4 bytes each).  5 scalar instructions per wait instead of the switch's compare
// tree of a switch (~25); vcc is the 64-bit temporary.
__device__ __forceinline__ uint32_t vmcnt_entry(int n) { return 8u * (uint32_t)n + 12u; }
__device__ __forceinline__ void wait_vmcnt_jump(uint32_t entry)
{
    asm volatile("s_getpc_b64 vcc\n\t"
                 "s_add_u32 vcc_lo, vcc_lo, %0\n\t"
                 "s_addc_u32 vcc_hi, vcc_hi, 0\n\t"
                 "s_setpc_b64 vcc\n\t"
                 "s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(1) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(3) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(5) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(7) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(9) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(10) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(11) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(12) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(13) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(14) lgkmcnt(0)\n\ts_branch .Lmcs_vm_end%=\n\t"
                 "s_waitcnt vmcnt(15) lgkmcnt(0)\n\t"
                 ".Lmcs_vm_end%=:" ::"s"(entry)
                 : "vcc", "memory");
}

// grid (8 * ceil(n_order / 8)), block (64, 8); the launch streams tiles order[0, n_order) (or
// tiles 0 .. n_order - 1).  XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs
// (b % 8 share one), so XCD x gets the contiguous band of list entries [x * per, (x+1) * per),
// walked in list (row-major) order; vertically adjacent tiles, whose footprints overlap
// by a few source rows, then run at about the same time on the same L2.  (Placement affects
// speed only.)
template <int CN, bool BUF, int FITS = 1>
__device__ __forceinline__ void stream_tile(const KParams &P, const TileHdr *tiles,
                                            const uint32_t *desc, const uint32_t *desc4,
                                            const uint16_t *spans, int n_frames, int parts,
                                            const int *order, int n_order, uint8_t *smem)
{
    // FITS 1: the tiles of the main launch; 2: the large-footprint tiles (kBigJobsPerWave rows per
    // wave, kBigStreamLds bytes of LDS)
    constexpr int NJ = FITS == 2 ? kBigJobsPerWave : kJobsPerWave;
    const int lane = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const int tid = wave * kWave + lane;
    const int gx = (P.out_w + kTileW - 1) / kTileW;
    const int per = (n_order * parts + 7) >> 3;
    const int item = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (item >= n_order * parts) return;
    // launch-list entry: a tile (-1 = padding); the block streams the captures of its part of
    // the batch through it (parts > 1: the large-footprint launch, whose few tiles would
    // otherwise each hold one CU for the whole batch -- the launch's tail)
    const int idx = item / parts, part = item - idx * parts;
    const int tile = order ? __builtin_amdgcn_readfirstlane(order[idx]) : idx;
    if (tile < 0) return;
    const int f_beg = (int)((int64_t)part * n_frames / parts);
    const int f_end = (int)((int64_t)(part + 1) * n_frames / parts);
    if (f_beg >= f_end) return;
    const int bx = tile % gx, by = tile / gx;
    // the tile header, copied once into LDS (the kernel also stores to global memory, so the
    // compiler cannot serve `tiles` from the scalar cache)
    TileHdr &h = *reinterpret_cast<TileHdr *>(smem);
    uint8_t *const ring0 = smem + sizeof(TileHdr);
    if (tid < (int)(sizeof(TileHdr) / 4))
        reinterpret_cast<int *>(&h)[tid] = reinterpret_cast<const int *>(&tiles[tile])[tid];
    __syncthreads();
    if (uni(h.fits) != FITS) return;           // handled by another launch of the plan
    int xg, y;
    tile_pixel(bx, by, lane, wave, xg, y);
    bool live = xg < P.out_w && y < P.out_h;
    const int npx = live ? min(kPx, P.out_w - xg) : 0;
    // the lane's 4 pixel descriptors: one 16-byte load of their compact words (4 B per pixel
    // per launch instead of 12), expanded here; pixels off the plain bilinear form (frame edges)
    // read their full 12-byte form
    uint32_t d[kPx * kDescWords];
    {
        const uint4 c4 = reinterpret_cast<const uint4 *>(desc4)[(int64_t)tile * (kTilePx / kPx) +
                                                                 tid];
        const uint32_t cw[kPx] = {c4.x, c4.y, c4.z, c4.w};
        // (pixels of the multi-band sweep's regions: the sweep kernel writes them)
        const bool skip_lane = c4.x == kCwSkip;
        live = live && !skip_lane;
        const uint32_t *full = desc + ((int64_t)tile * kTilePx + (int64_t)tid * kPx) * kDescWords;
#pragma unroll
        for (int p = 0; p < kPx; p++) {
            const uint32_t w = cw[p];
            uint32_t d0, d1, d2;
            if (skip_lane) {
                d0 = d1 = d2 = 0u;
            } else if (w & kCwFull) {
                d0 = full[p * kDescWords];
                d1 = full[p * kDescWords + 1];
                d2 = full[p * kDescWords + 2];
            } else {
                const uint32_t a0 = w & 0xffffu, fx = (w >> 16) & 31u, fy = (w >> 21) & 31u;
                const int k = (int)((w >> 26) & 3u);
                const uint32_t e = (w & kCwLastRow1) ? ((uint32_t)h.last_shift >> (8 * k)) & 255u
                                                     : 0u;
                const uint32_t a1 =
                    (w & kCwOneRow) ? a0 : a0 + ((uint32_t)h.stride[k] & 0xffffu) + e;
                d0 = a0 | (a1 << 16);
                d1 = w2x((32u - fx) * (32u - fy) * 32u) | (w2x(fx * (32u - fy) * 32u) << 16);
                d2 = w2x((32u - fx) * fy * 32u) | (w2x(fx * fy * 32u) << 16);
                if (w & kCwZero) d0 = d1 = d2 = 0u;
            }
            d[p * kDescWords] = d0;
            d[p * kDescWords + 1] = d1;
            d[p * kDescWords + 2] = d2;
        }
    }
    const WaveWins<BUF, NJ> J =
        wave_windows<CN, BUF, NJ>(P, h, wave, spans + (int64_t)tile * kMaxTileJobs, lane);
#define MCS_STAGE(slot, foff) stage_windows<BUF, NJ>(J, rs, (slot) - sizeof(TileHdr), (foff))
    const int njobs = J.total;   // DMA instructions per capture of the block
    // (BUF: raw buffer over [P.base, P.base + 4 GiB); no range clamping needed, every chunk is
    // inside a frame)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(BUF ? P.base : P.out), 0, 0xffffffff, 0x00020000);
    const int ring = uni(h.ring), buf_bytes = uni(h.buf_bytes);
    const int d_min = njobs / kWavesPerBlock;
    const int waitn = min((ring - 2) * d_min, 15);
    uint8_t *dst = P.out + (int64_t)min(y, P.out_h - 1) * P.out_pitch + (int64_t)xg * CN;
    const bool wide = npx == kPx && (((uintptr_t)dst | (uintptr_t)P.out_fstride) & 3) == 0;
    const int64_t fstride = P.cam_fstride[0];
    for (int q = 0; q < ring - 1 && f_beg + q < f_end; q++)
        MCS_STAGE(ring0 + q * buf_bytes, (int64_t)(f_beg + q) * fstride);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // Capture f's pixels from its ring slot at LDS offset `sf`, stored to the mosaic at byte
    // offset `of` = f * out_fstride.  Every lane computes (a lane past the mosaic edge holds zero
    // descriptors and reads slot byte 0); only the stores are per lane.  A wave whose lanes all
    // store 12 aligned bytes (every interior tile) takes one branch-free store.
    const bool all_wide =
        __builtin_amdgcn_ballot_w64(live && wide) == __builtin_amdgcn_read_exec();
    auto emit = [&](uint32_t sf, int64_t of) __attribute__((always_inline)) {
        const uint8_t *b = ring0 + sf;
        uint32_t rr[kPx * CN];
        uint32_t raw[kPx][6];
#pragma unroll
        for (int p = 0; p < kPx; p++) {
            const uint32_t win = d[p * kDescWords];
            const lds_u32 *w0 = (const lds_u32 *)(((const lds_u8 *)b) + ((win & 0xffffu) & ~3u));
            const lds_u32 *w1 = (const lds_u32 *)(((const lds_u8 *)b) + ((win >> 16) & ~3u));
            raw[p][0] = w0[0], raw[p][1] = w0[1], raw[p][2] = w0[2];
            raw[p][3] = w1[0], raw[p][4] = w1[1], raw[p][5] = w1[2];
        }
#pragma unroll
        for (int p = 0; p < kPx; p++) {
            const uint32_t win = d[p * kDescWords], s0 = win & 3u, s1 = (win >> 16) & 3u;
            const uint2 r0 = make_uint2(__builtin_amdgcn_alignbyte(raw[p][1], raw[p][0], s0),
                                        __builtin_amdgcn_alignbyte(raw[p][2], raw[p][1], s0));
            const uint2 r1 = make_uint2(__builtin_amdgcn_alignbyte(raw[p][4], raw[p][3], s1),
                                        __builtin_amdgcn_alignbyte(raw[p][5], raw[p][4], s1));
#pragma unroll
            for (int k = 0; k < CN; k++)
                rr[p * CN + k] = blend<CN>(r0, r1, d[p * kDescWords + 1], d[p * kDescWords + 2], k);
        }
        const OutWords w = pack_words<CN>(rr);
        uint32_t *o32 = reinterpret_cast<uint32_t *>(dst + of);
        if (all_wide) {
#pragma unroll
            for (int i = 0; i < CN; i++) __builtin_nontemporal_store(w.at(i), &o32[i]);
        } else if (live) {
            if (wide) {
#pragma unroll
                for (int i = 0; i < CN; i++) __builtin_nontemporal_store(w.at(i), &o32[i]);
            } else {
                // (a frame-edge lane: byte stores through a buffer resource over this capture's
                // mosaic -- 32-bit offsets instead of a 64-bit address per byte)
                const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
                    (void *)(P.out + of), 0, 0x7fffffff, 0x00020000);
                const uint32_t lo = (uint32_t)(dst - P.out);
                for (int bb = 0; bb < npx * CN; bb++)
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(w.at(bb >> 2) >> (8 * (bb & 3))),
                                                         ro, lo + (uint32_t)bb, 0, 0);
            }
        }
    };
    // Steady state (captures whose iteration stages capture f + ring - 1): the wait leaves
    // `waitn` DMA instructions outstanding -- those this wave issued after capture f + 1's
    // ((ring - 2) later captures x D_min rows).  The DMAs (loads) complete in issue order among
    // themselves, so with at most waitn VMEM operations of any kind outstanding, capture f + 1
    // has landed for this wave (stores are not counted: loads and stores may complete out of
    // order with respect to each other); the barrier makes it so for the block.  The last
    // ring - 1 captures stage nothing and wait for everything.  Slots as LDS byte offsets,
    // capture offsets as running sums: no multiplies in the loop.  (One loop body: a separate
    // tail loop, a second copy of emit, costs 8 VGPRs.)
    const uint32_t slot_end = (uint32_t)(ring * buf_bytes);
    uint32_t sf = 0, sa = (uint32_t)((ring - 1) * buf_bytes);
    int64_t of = (int64_t)f_beg * P.out_fstride, fa = (int64_t)(f_beg + ring - 1) * fstride;
    const int n = f_end - f_beg, n_steady = max(0, n - (ring - 1));
    const uint32_t wait_steady = vmcnt_entry(waitn), wait_all = vmcnt_entry(0);
    for (int i = 0; i < n; i++) {
        const bool steady = i < n_steady;
        if (steady) MCS_STAGE(ring0 + sa, fa);
        emit(sf, of);
        wait_vmcnt_jump(steady ? wait_steady : wait_all);
        __builtin_amdgcn_s_barrier();
        sf += (uint32_t)buf_bytes;
        sf = sf == slot_end ? 0u : sf;
        sa += (uint32_t)buf_bytes;
        sa = sa == slot_end ? 0u : sa;
        fa += fstride;
        of += P.out_fstride;
    }
#undef MCS_STAGE
}

// Direct global gather for the tiles prepare could not fit in LDS (list in fallback[1..]):
// grid (tiles, ceil(frames / kDirectFrames)), launched on a side stream next to the streaming
// kernel, so these few tiles cost no extra time on the critical path.
template <int CN, int INTERP, bool OFF32>
__device__ __forceinline__ void direct_tile(const KParams &P, const int *fallback, int n_frames)
{
    const int tile = fallback ? fallback[1 + blockIdx.x] : (int)blockIdx.x;   // NULL: every tile
    const int f0 = blockIdx.y * kDirectFrames;
    const int gx = (P.out_w + kTileW - 1) / kTileW;
    const int tx = tile % gx, ty = tile / gx;
    int xg, y;
    tile_pixel(tx, ty, threadIdx.x, threadIdx.y, xg, y);
    if (xg < P.out_w && y < P.out_h && !(P.skip && P.skip[(int64_t)y * P.out_w + xg]))
        stitch_direct<CN, INTERP, OFF32>(P, f0, min(n_frames, f0 + kDirectFrames), xg, y);
}

// Footprint marking: mask[cam][pixel] = 1 for every source pixel the mosaic reads with a
// non-zero weight; counts[cam] += newly marked pixels (algorithmic bytes of the roofline).
template <int CN, int INTERP>
__device__ __forceinline__ void footprint_mark(const KParams &P, uint8_t *const *masks,
                                               unsigned long long *counts)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= P.out_w || y >= P.out_h) return;
    const int s = pixel_stage<INTERP>(P, x, y);
    if (s == -2) return;
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
    stage_map<INTERP>(P, S, x, y, X, Y);
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

// ---------------------------------------------------------------------------------------------
// cv2.resize(src, (dw, dh), interpolation=INTER_LINEAR) for u8 images: the reference's pre-warp
// resize of frames that do not have their calibrated shape (StitcherClass.py:226-233).  OpenCV
// 3.4 resize.cpp arithmetic (restated in oracle/orc_resize.c): per-axis source index and 11-bit
// coefficients from float coordinates (computed here exactly as on the host: IEEE double, then
// float, no contraction), horizontal taps into int, vertical pass
// ((b0 * (D0 >> 4)) >> 16) + ((b1 * (D1 >> 4)) >> 16) + 2 >> 2.  An exact 2x downscale is
// OpenCV's INTER_AREA fast path.  HBM-bound (reads each source byte ~once through L2, writes
// the destination once); one thread per destination pixel, all channels.
__device__ __forceinline__ void resize_axis(int d, double scale, int ssize, bool is_x, int &s,
                                            int &c0, int &c1)
{
    float f = (float)((d + 0.5) * scale - 0.5);
    int si = (int)floorf(f);
    f -= (float)si;
    if (is_x) {
        if (si < 0) f = 0.f, si = 0;
        if (si >= ssize - 1) f = 0.f, si = ssize - 1;
    }
    s = si;
    c0 = __float2int_rn((1.f - f) * 2048.f);
    c1 = __float2int_rn(f * 2048.f);
}

template <int CN>
__device__ __forceinline__ void resize_px(const KResizeArgs &a)
{
    const int x = blockIdx.x * kResizeBlock + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
    if (x >= a.dw) return;
    const uint8_t *src = a.src + (int64_t)f * a.src_fstride;
    uint8_t *dst = a.dst + (int64_t)f * a.dst_fstride + (int64_t)y * a.dst_pitch + (int64_t)x * CN;
    if (a.area2x) {
        const uint8_t *s0 = src + (int64_t)(2 * y) * a.src_pitch + (int64_t)(2 * x) * CN;
        const uint8_t *s1 = s0 + a.src_pitch;
#pragma unroll
        for (int k = 0; k < CN; k++) {
            const int sum = s0[k] + s0[CN + k] + s1[k] + s1[CN + k];
            dst[k] = (uint8_t)(CN == 2 ? __float2int_rn((float)sum * 0.25f) : (sum + 2) >> 2);
        }
        return;
    }
    int sx, a0, a1, sy, b0, b1;
    resize_axis(x, a.scale_x, a.sw, true, sx, a0, a1);
    resize_axis(y, a.scale_y, a.sh, false, sy, b0, b1);
    const int r0 = min(max(sy, 0), a.sh - 1), r1 = min(max(sy + 1, 0), a.sh - 1);
    const uint8_t *p0 = src + (int64_t)r0 * a.src_pitch + (int64_t)sx * CN;
    const uint8_t *p1 = src + (int64_t)r1 * a.src_pitch + (int64_t)sx * CN;
    const bool one = sx >= a.sw - 1;
#pragma unroll
    for (int k = 0; k < CN; k++) {
        const int d0 = one ? p0[k] * 2048 : p0[k] * a0 + p0[CN + k] * a1;
        const int d1 = one ? p1[k] * 2048 : p1[k] * a0 + p1[CN + k] * a1;
        dst[k] = (uint8_t)((((b0 * (d0 >> 4)) >> 16) + ((b1 * (d1 >> 4)) >> 16) + 2) >> 2);
    }
}

}  // namespace mcs

// ---------------------------------------------------------------------------------------------
// Entry points (names looked up by mcs_capi.cpp).  Block shapes: prepare (64, 8, 1) over the tile
// grid (ceil(out_w/256), ceil(out_h/8)); stream (64, 8, 1) over 8 * ceil(tiles / 8) blocks with
// lds_stream_bytes(CN) of dynamic LDS; direct (64, 8, 1) over the fallback tile list; footprint
// (256, 1, 1) with grid
// (ceil(out_w/256), out_h).
#define MCS_PREPARE_ENTRY(CN, IN)                                                              \
    extern "C" __global__ __launch_bounds__(512) void mcs_prepare_c##CN##_i##IN(               \
        const mcs::KParams P, mcs::TileHdr *tiles, uint32_t *desc, uint32_t *desc4,            \
        int *fallback, int *big, uint16_t *spans)                                              \
    {                                                                                          \
        mcs::prepare_tile<CN, IN>(P, tiles, desc, desc4, fallback, big, spans);                \
    }
#define MCS_STREAM_ENTRY(CN, SUF, BUF)                                                         \
    extern "C" __global__ __launch_bounds__(512) void mcs_stream_c##CN##SUF(         \
        const mcs::KParams P, const mcs::TileHdr *tiles, const uint32_t *desc,                \
        const uint32_t *desc4, const uint16_t *spans, int n_frames, int parts,                \
        const int *order, int n_order)                                                         \
    {                                                                                          \
        extern __shared__ __attribute__((aligned(16))) uint8_t smem[];                         \
        mcs::stream_tile<CN, BUF>(P, tiles, desc, desc4, spans, n_frames, parts, order,        \
                                  n_order, smem);                                              \
    }                                                                                          \
    extern "C" __global__ __launch_bounds__(512) void mcs_stream_big_c##CN##SUF(               \
        const mcs::KParams P, const mcs::TileHdr *tiles, const uint32_t *desc,                \
        const uint32_t *desc4, const uint16_t *spans, int n_frames, int parts,                \
        const int *order, int n_order)                                                         \
    {                                                                                          \
        extern __shared__ __attribute__((aligned(16))) uint8_t smem[];                         \
        mcs::stream_tile<CN, BUF, 2>(P, tiles, desc, desc4, spans, n_frames, parts, order,     \
                                     n_order, smem);                                           \
    }
#define MCS_DIRECT_ENTRY(CN, IN, O32)                                                          \
    extern "C" __global__ __launch_bounds__(512) void mcs_direct_c##CN##_i##IN##_o##O32(       \
        const mcs::KParams P, const int *fallback, int n_frames)                              \
    {                                                                                          \
        mcs::direct_tile<CN, IN, O32 == 32>(P, fallback, n_frames);                            \
    }
#define MCS_ENTRIES(CN)                                                                        \
    MCS_PREPARE_ENTRY(CN, 0)                                                                   \
    MCS_PREPARE_ENTRY(CN, 1)                                                                   \
    MCS_STREAM_ENTRY(CN, , false)                                                              \
    MCS_STREAM_ENTRY(CN, _b32, true)                                                           \
    MCS_DIRECT_ENTRY(CN, 0, 32)                                                                \
    MCS_DIRECT_ENTRY(CN, 1, 32)                                                                \
    MCS_DIRECT_ENTRY(CN, 0, 64)                                                                \
    MCS_DIRECT_ENTRY(CN, 1, 64)
MCS_ENTRIES(1)
MCS_ENTRIES(2)
MCS_ENTRIES(3)
MCS_ENTRIES(4)

// Blended modes (mcs_blend.h).  Prepare: owner map + tile info over the 32-px blend grid, then
// the classification into the per-frame tile list; per frame: feather / multiband over it.
#define MCS_BLEND_PREP_ENTRY(IN)                                                               \
    extern "C" __global__ __launch_bounds__(256) void mcs_blend_owner_i##IN(                  \
        const mcs::KBlendPrepArgs a)                                                           \
    {                                                                                          \
        mcs::blend_owner_tile<IN>(a.P, a.owner, a.info);                                       \
    }
MCS_BLEND_PREP_ENTRY(0)
MCS_BLEND_PREP_ENTRY(1)
#define MCS_SEAM_ENTRY(CN, IN)                                                                 \
    extern "C" __global__ __launch_bounds__(256) void mcs_seam_sample_c##CN##_i##IN(           \
        const mcs::KSeamArgs a)                                                                \
    {                                                                                          \
        mcs::seam_sample<CN, IN>(a);                                                           \
    }
MCS_SEAM_ENTRY(1, 0)
MCS_SEAM_ENTRY(1, 1)
MCS_SEAM_ENTRY(2, 0)
MCS_SEAM_ENTRY(2, 1)
MCS_SEAM_ENTRY(3, 0)
MCS_SEAM_ENTRY(3, 1)
MCS_SEAM_ENTRY(4, 0)
MCS_SEAM_ENTRY(4, 1)
extern "C" __global__ __launch_bounds__(256) void mcs_blend_classify(const mcs::KBlendPrepArgs a)
{
    mcs::blend_classify(a.P, a.mode, a.owner, a.info, a.list, a.overflow, a.list2);
}
#define MCS_BLEND_ENTRY(CN, IN)                                                                \
    extern "C" __global__ __launch_bounds__(256) void mcs_feather_c##CN##_i##IN(               \
        const mcs::KBlendArgs a)                                                               \
    {                                                                                          \
        mcs::feather_tile<CN, IN>(a);                                                          \
    }                                                                                          \
    extern "C" __global__ __launch_bounds__(256) void mcs_mb_prep_c##CN##_i##IN(               \
        const mcs::KMbArgs a)                                                                  \
    {                                                                                          \
        mcs::mb_prep<CN, IN>(a);                                                               \
    }                                                                                          \
    extern "C" __global__ __launch_bounds__(256) void mcs_mb_bdesc_c##CN##_i##IN(              \
        const mcs::KMbBandArgs a)                                                              \
    {                                                                                          \
        mcs::mb_bdesc<CN, IN>(a);                                                              \
    }
#ifndef MCS_MB_WAVES
#define MCS_MB_WAVES 4
#endif
// band pass entry points: interior, bottom / right edge, both in one grid; SFX _a = the
// dword-aligned window form (mb_bands AL).  Up to 3 channels at most 128 VGPRs: 4 waves per SIMD.
// (3 waves per SIMD: 129 VGPRs and no scratch; at 4 the register cap spilled 3 dwords whose
// reloads in the global-form store path drained every load in flight, s_waitcnt vmcnt(0) --
// C4 launch -1 %, C2 unchanged, profiles/r04_band_wpe_ab.txt)
#ifndef MCS_MB_BAND_WPE
#define MCS_MB_BAND_WPE 3
#endif
#define MCS_MB_BAND_ATTR(CN) __attribute__((amdgpu_waves_per_eu(MCS_MB_BAND_WPE)))
// (the aligned entries hold the LDS ring of mode 2; the others none)
#define MCS_MB_BAND_RING(AL)                                                                   \
    __shared__ __attribute__((aligned(16))) uint8_t ring_[(AL) ? mcs::kMbLdsBytes : 16];       \
    mcs::lds_u8 *const ring = (mcs::lds_u8 *)ring_
#define MCS_MB_BANDS_ENTRY(CN, SFX, AL)                                                        \
    extern "C" __global__ __launch_bounds__(64) MCS_MB_BAND_ATTR(CN) void                     \
        mcs_mb_bands##SFX##_c##CN(                                                             \
        const mcs::KMbBandArgs a)                                                              \
    {                                                                                          \
        MCS_MB_BAND_RING(AL);                                                                  \
        int bl, pr;                                                                            \
        if (!mcs::xcd_unit(a.nb, (a.nf + mcs::kMbBandFrames - 1) / mcs::kMbBandFrames, bl, pr)) \
            return;                                                                            \
        mcs::mb_bands<CN, mcs::kMbBandFrames, false, AL>(a, a.band0 + bl, ring, pr);          \
    }                                                                                          \
    extern "C" __global__ __launch_bounds__(64) MCS_MB_BAND_ATTR(CN) void                     \
        mcs_mb_bands_br##SFX##_c##CN(                                                          \
        const mcs::KMbBandArgs a)                                                              \
    {                                                                                          \
        MCS_MB_BAND_RING(AL);                                                                  \
        int bl, pr;                                                                            \
        if (!mcs::xcd_unit(a.nb, (a.nf + mcs::kMbBandFrames - 1) / mcs::kMbBandFrames, bl, pr)) \
            return;                                                                            \
        mcs::mb_bands<CN, mcs::kMbBandFrames, true, AL>(a, a.band0 + bl, ring, pr);           \
    }                                                                                          \
    extern "C" __global__ __launch_bounds__(64) MCS_MB_BAND_ATTR(CN) void                     \
        mcs_mb_bands_all##SFX##_c##CN(                                                         \
        const mcs::KMbBandArgs a)                                                              \
    {                                                                                          \
        MCS_MB_BAND_RING(AL);                                                                  \
        int bl, pr;                                                                            \
        if (!mcs::xcd_unit(a.nb, (a.nf + mcs::kMbBandFrames - 1) / mcs::kMbBandFrames, bl, pr)) \
            return;                                                                            \
        if (bl < a.n_in)                                                                       \
            mcs::mb_bands<CN, mcs::kMbBandFrames, false, AL>(a, a.band0 + bl, ring, pr);      \
        else mcs::mb_bands<CN, mcs::kMbBandFrames, true, AL>(a, a.band1 + bl - a.n_in, ring, pr); \
    }
#define MCS_MB_ENTRY(CN)                                                                       \
    extern "C" __global__ __launch_bounds__(MCS_MB_LV_THREADS) __attribute__((amdgpu_waves_per_eu(MCS_MB_WAVES))) \
    void mcs_mb_levels_c##CN(const mcs::KMbArgs a)                                             \
    {                                                                                          \
        __shared__ mcs::MbLvLds<CN> lds;                                                       \
        mcs::mb_levels<CN>(a, lds);                                                            \
    }                                                                                          \
    MCS_MB_BANDS_ENTRY(CN, , false)                                                            \
    MCS_MB_BANDS_ENTRY(CN, _a, true)                                                           \
    extern "C" __global__ __launch_bounds__(MCS_MB_BL_THREADS) void                            \
        mcs_mb_blend_c##CN##_s2(                                                               \
        const mcs::KMbArgs a)                                                                  \
    {                                                                                          \
        __shared__ mcs::MbBlLds<CN, 2> lds;                                                    \
        mcs::mb_blend<CN, 2>(a, lds);                                                          \
    }                                                                                          \
    extern "C" __global__ __launch_bounds__(MCS_MB_BL_THREADS) void                            \
        mcs_mb_blend_c##CN##_s4(                                                               \
        const mcs::KMbArgs a)                                                                  \
    {                                                                                          \
        __shared__ mcs::MbBlLds<CN, 4> lds;                                                    \
        mcs::mb_blend<CN, 4>(a, lds);                                                          \
    }                                                                                          \
    extern "C" __global__ __launch_bounds__(MCS_MB_BL_THREADS) void                            \
        mcs_mb_blend_c##CN##_s8(                                                               \
        const mcs::KMbArgs a)                                                                  \
    {                                                                                          \
        __shared__ mcs::MbBlLds<CN, 8> lds;                                                    \
        mcs::mb_blend<CN, 8>(a, lds);                                                          \
    }
MCS_MB_ENTRY(1)
MCS_MB_ENTRY(2)
MCS_MB_ENTRY(3)
MCS_MB_ENTRY(4)
MCS_BLEND_ENTRY(1, 0)
MCS_BLEND_ENTRY(1, 1)
MCS_BLEND_ENTRY(2, 0)
MCS_BLEND_ENTRY(2, 1)
MCS_BLEND_ENTRY(3, 0)
MCS_BLEND_ENTRY(3, 1)
MCS_BLEND_ENTRY(4, 0)
MCS_BLEND_ENTRY(4, 1)

// grid (ceil(dw / kResizeBlock), dh, n_frames), block (kResizeBlock)
#define MCS_RESIZE_ENTRY(CN)                                                                   \
    extern "C" __global__ __launch_bounds__(256) void mcs_resize_c##CN(const mcs::KResizeArgs a) \
    {                                                                                          \
        mcs::resize_px<CN>(a);                                                                 \
    }
MCS_RESIZE_ENTRY(1)
MCS_RESIZE_ENTRY(2)
MCS_RESIZE_ENTRY(3)
MCS_RESIZE_ENTRY(4)

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
