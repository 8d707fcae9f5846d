// mcs_blend.h -- device code of the blended stitch modes,
// included by mcs_kernels.hip (one code object).  The arithmetic is specified, and restated on
// the CPU, in oracle/orc_blend.c; this file reproduces it bit for bit (integers and IEEE
// doubles in the same order, no contraction).
//
// Layout: the stitch kernels first write every pixel from its "owner" camera (the covering
// camera farthest from its own image edge); then only the tiles where blending changes pixels
// are recomputed here, 32 x 32 output pixels per block:
//   feather   -- tiles with a pixel covered by two cameras at positive edge distance;
//   multiband -- tiles whose neighbourhood (the 3-level pyramid's reach, 16 px halo)
//                holds two owners (the seam band).  Per tile: the owners' warped images over the
//                neighbourhood (replicate border) -> integer Gaussian/Laplacian pyramids in LDS
//                -> mask-weighted blend per level (double) -> collapse -> bytes.
// Both are a few percent of the mosaic's tiles for a linear rig.
#pragma once

namespace mcs {

// Camera slot s of the plan: 0 = camera 0 (integer offset), j+1 = stage j's camera.
template <int INTERP>
__device__ __forceinline__ void slot_xy(const KParams &P, int s, int x, int y, int &x32, int &y32,
                                        int &cam, int &w, int &h)
{
    if (s == 0) {
        cam = 0;
        w = P.cam0_w;
        h = P.cam0_h;
        x32 = (x + P.cam0_offx) * 32;
        y32 = (y + P.cam0_offy) * 32;
        return;
    }
    const KStage &S = P.st[s - 1];
    cam = S.cam;
    w = S.src_w;
    h = S.src_h;
    int X, Y;
    stage_map<INTERP>(P, S, x, y, X, Y);
    if (INTERP == MCS_INTER_NEAREST) {
        x32 = sat_i16(X) * 32;
        y32 = sat_i16(Y) * 32;
    } else {
        x32 = sat_i16(X >> 5) * 32 + (X & 31);
        y32 = sat_i16(Y >> 5) * 32 + (Y & 31);
    }
}

// Distance to the image edge in 1/32 px, -1 when the position is not covered.
__device__ __forceinline__ int slot_dist(int x32, int y32, int w, int h)
{
    const int xm = 32 * (w - 1) - x32, ym = 32 * (h - 1) - y32;
    if (x32 < 0 || y32 < 0 || xm < 0 || ym < 0) return -1;
    return min(min(x32, y32), min(xm, ym));
}

// Owner slot of output pixel (x, y) (largest edge distance, ties to the lower camera index),
// kBlendNone when no camera covers it.  *pos_mask: slots covering it at positive distance.
template <int INTERP>
__device__ __forceinline__ int blend_owner(const KParams &P, int x, int y, uint32_t *pos_mask)
{
    int best = kBlendNone, bestd = -1, bestcam = 0;
    // graph-cut seams: the label's camera owns the pixel when it covers it
    const int hcam = P.seam_hint ? (int)P.seam_hint[(int64_t)(y >> P.seam_shift) * P.seam_w +
                                                    (x >> P.seam_shift)]
                                 : (int)kBlendNone;
    int hslot = -1;
    uint32_t pm = 0;
    for (int s = 0; s <= P.n_stages; s++) {
        int x32, y32, cam, w, h;
        slot_xy<INTERP>(P, s, x, y, x32, y32, cam, w, h);
        const int d = slot_dist(x32, y32, w, h);
        if (d > 0) pm |= 1u << s;
        if (d >= 0 && cam == hcam) hslot = s;
        if (d >= 0 && (d > bestd || (d == bestd && cam < bestcam))) {
            best = s;
            bestd = d;
            bestcam = cam;
        }
    }
    if (pos_mask) *pos_mask = pm;
    return hslot >= 0 ? hslot : best;
}

// Bilinear sample at (x32, y32) with the taps clamped into the image (BORDER_REPLICATE), the
// remapBilinear fixed point; channel k in byte k.  One 8-byte window load per tap row.
template <int CN>
__device__ __forceinline__ uint32_t sample_replicate(const uint8_t *fb, int w, int h, int x32,
                                                     int y32)
{
    const int sx = x32 >> 5, sy = y32 >> 5, fx = x32 & 31, fy = y32 & 31;
    const int cx = w >= 2 ? min(max(sx, 0), w - 2) : 0;
    const int oa = (min(max(sx, 0), w - 1) - cx) * CN, ob = (min(max(sx + 1, 0), w - 1) - cx) * CN;
    const int ya = min(max(sy, 0), h - 1), yb = min(max(sy + 1, 0), h - 1);
    const int w00 = (32 - fx) * (32 - fy) * 32, w01 = fx * (32 - fy) * 32;
    const int w10 = (32 - fx) * fy * 32, w11 = fx * fy * 32;
    const int64_t pitch = (int64_t)w * CN, fbytes = pitch * h;
    const uint2 r0 = load8<2 * CN>(fb, ya * pitch + (int64_t)cx * CN, fbytes);
    const uint2 r1 = load8<2 * CN>(fb, yb * pitch + (int64_t)cx * CN, fbytes);
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < CN; k++) {
        const int s = (int)byte_of(r0, oa + k) * w00 + (int)byte_of(r0, ob + k) * w01 +
                      (int)byte_of(r1, oa + k) * w10 + (int)byte_of(r1, ob + k) * w11;
        r |= (uint32_t)((s + 16384) >> 15) << (8 * k);
    }
    return r;
}

// Camera, size of slot s (uniform).
__device__ __forceinline__ void slot_info(const KParams &P, int s, int &cam, int &w, int &h)
{
    cam = s == 0 ? 0 : P.st[s - 1].cam;
    w = s == 0 ? P.cam0_w : P.st[s - 1].src_w;
    h = s == 0 ? P.cam0_h : P.st[s - 1].src_h;
}

__device__ __forceinline__ int refl(int i, int n)
{
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

// ---- seam finder inputs (mcs_plan_find_seams) ------------------------------------------------
// One thread per point of the 2^k grid (P.seam_hint must be NULL: the distance owner).
template <int CN, int INTERP>
__device__ __forceinline__ void seam_sample(const KSeamArgs &a)
{
    const KParams &P = a.P;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.gw * a.gh) return;
    const int x = (q % a.gw) << a.k, y = (q / a.gw) << a.k;
    const int64_t np = (int64_t)a.gw * a.gh;
    const int o = blend_owner<INTERP>(P, x, y, nullptr);
    uint32_t cov = 0;
    for (int s = 0; s <= P.n_stages; s++) {
        int x32, y32, cam, w, h;
        slot_xy<INTERP>(P, s, x, y, x32, y32, cam, w, h);
        if (slot_dist(x32, y32, w, h) < 0) continue;
        cov |= 1u << cam;
        const uint8_t *fb = P.cams[cam];
        const uint32_t v = sample_replicate<CN>(fb, w, h, x32, y32);
        uint8_t *d = a.samples + ((int64_t)cam * np + q) * CN;
#pragma unroll
        for (int k = 0; k < CN; k++) d[k] = (uint8_t)(v >> (8 * k));
    }
    a.cov[q] = (uint16_t)cov;
    int ocam = kBlendNone;
    if (o != kBlendNone) {
        int c, w, h;
        slot_info(P, o, c, w, h);
        ocam = c;
    }
    a.label[q] = (uint8_t)ocam;
}

// ---- prepare (once per plan) -----------------------------------------------------------------
// grid (ceil(W / 32), ceil(H / 32)), block 256: owner map, and per blend tile the owners it holds
// (info[2t]) and the slots covering any of its pixels at positive distance when two do
// (info[2t+1], the feather set).
template <int INTERP>
__device__ __forceinline__ void blend_owner_tile(const KParams &P, uint8_t *owner_map,
                                                 uint32_t *info)
{
    __shared__ uint32_t s_own, s_feather;
    if (threadIdx.x == 0) s_own = s_feather = 0;
    __syncthreads();
    const int X0 = blockIdx.x * kBlendTileW, Y0 = blockIdx.y * kBlendTileH;
    uint32_t own = 0, fea = 0;
    for (int i = threadIdx.x; i < kMbTilePx; i += blockDim.x) {
        const int x = X0 + (i % kBlendTileW), y = Y0 + i / kBlendTileW;
        if (x >= P.out_w || y >= P.out_h) continue;
        uint32_t pm;
        const int o = blend_owner<INTERP>(P, x, y, &pm);
        owner_map[(int64_t)y * P.out_w + x] = (uint8_t)o;
        if (o != kBlendNone) own |= 1u << o;
        if (__popc(pm) >= 2) fea |= pm;
    }
    atomicOr(&s_own, own);
    atomicOr(&s_feather, fea);
    __syncthreads();
    if (threadIdx.x == 0) {
        const int t = blockIdx.y * gridDim.x + blockIdx.x;
        info[2 * t] = s_own;
        info[2 * t + 1] = s_feather;
    }
}

// grid (tiles), block 256: appends (tile, slot mask) to list[1 + 2i] for the tiles the mode
// recomputes; list[0] = count.  multiband: the owners in the tile's neighbourhood (the tile grown
// by kBlendHalo, clipped to the mosaic: reflected positions land inside it), when there are two
// or more.  A neighbourhood with more than kBlendSlots owners (more than the blend kernels hold)
// degrades its tile to the feather rule (orc_blend.c "dense seams"): the tile goes to list2 with
// its feather slot set (none when no pixel has two cameras at positive distance: the owner
// sample the streaming kernel writes IS the feather value there), counted in overflow[0];
// overflow[1] = the most owners any multi-band-listed tile has.
__device__ __forceinline__ void blend_classify(const KParams &P, int mode, const uint8_t *owner,
                                               const uint32_t *info, int *list, int *overflow,
                                               int *list2)
{
    __shared__ uint32_t s_mask;
    const int gx = (P.out_w + kBlendTileW - 1) / kBlendTileW;
    const int t = blockIdx.x, tx = t % gx, ty = t / gx;
    uint32_t mask;
    if (mode == MCS_BLEND_FEATHER) {
        mask = info[2 * t + 1];
    } else {
        if (threadIdx.x == 0) s_mask = 0;
        __syncthreads();
        const int x0 = max(tx * kBlendTileW - kBlendHalo, 0);
        const int x1 = min(tx * kBlendTileW + kBlendTileW + kBlendHalo, P.out_w);
        const int y0 = max(ty * kBlendTileH - kBlendHalo, 0);
        const int y1 = min(ty * kBlendTileH + kBlendTileH + kBlendHalo, P.out_h);
        const int rw = x1 - x0, n = rw * (y1 - y0);
        uint32_t m = 0;
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const int o = owner[(int64_t)(y0 + i / rw) * P.out_w + x0 + i % rw];
            if (o != kBlendNone) m |= 1u << o;
        }
        atomicOr(&s_mask, m);
        __syncthreads();
        mask = s_mask;
        if (__popc(mask) < 2) mask = 0;
    }
    if (threadIdx.x == 0 && mode == MCS_BLEND_MULTIBAND && __popc(mask) > kBlendSlots) {
        atomicAdd(overflow, 1);
        const uint32_t fea = info[2 * t + 1];
        if (fea) {
            const int i = atomicAdd(&list2[0], 1);
            list2[1 + 2 * i] = t;
            list2[2 + 2 * i] = (int)fea;
        }
        return;
    }
    if (threadIdx.x == 0 && mask) {
        atomicMax(overflow + 1, __popc(mask));
        const int i = atomicAdd(&list[0], 1);
        list[1 + 2 * i] = t;
        list[2 + 2 * i] = (int)mask;
    }
}

// ---- per frame ---------------------------------------------------------------------------------
// Feather: grid (listed tiles, frames), block 256.
template <int CN, int INTERP>
__device__ __forceinline__ void feather_tile(const KBlendArgs &a)
{
    const KParams &P = a.P;
    const int gx = (P.out_w + kBlendTileW - 1) / kBlendTileW;
    const int t = a.list[1 + 2 * blockIdx.x];
    const uint32_t mask = (uint32_t)a.list[2 + 2 * blockIdx.x];
    const int X0 = (t % gx) * kBlendTileW, Y0 = (t / gx) * kBlendTileH, f = blockIdx.y;
    for (int i = threadIdx.x; i < kMbTilePx; i += blockDim.x) {
        const int x = X0 + (i % kBlendTileW), y = Y0 + i / kBlendTileW;
        if (x >= P.out_w || y >= P.out_h) continue;
        int den = 0, num[CN];
#pragma unroll
        for (int k = 0; k < CN; k++) num[k] = 0;
        for (uint32_t m = mask; m; m &= m - 1) {
            const int s = __ffs(m) - 1;
            int x32, y32, cam, w, h;
            slot_xy<INTERP>(P, s, x, y, x32, y32, cam, w, h);
            const int d = slot_dist(x32, y32, w, h);
            if (d <= 0) continue;
            const uint32_t v = sample_replicate<CN>(P.cams[cam] + (int64_t)f * P.cam_fstride[cam],
                                                    w, h, x32, y32);
            den += d;
#pragma unroll
            for (int k = 0; k < CN; k++) num[k] += d * (int)((v >> (8 * k)) & 0xffu);
        }
        if (den == 0) continue;   // the stitch kernel already wrote the owner's sample
        uint8_t *o = P.out + (int64_t)f * P.out_fstride + (int64_t)y * P.out_pitch + x * CN;
#pragma unroll
        for (int k = 0; k < CN; k++) o[k] = (uint8_t)((num[k] + den / 2) / den);
    }
}

// ---- multi-band (3 levels) -------------------------------------------------------------------
// Per listed tile (a 32 x 32 output tile whose 64 x 64 neighbourhood holds two or more owners)
// the pyramid needs, per owner slot: level 0 over [X0-14, X0+42] (57 of the 64 px), level 1
// g1 over [X0/2-6, X0/2+20] (27), level 2 g2 over [X0/4-2, X0/4+9] (12), and the collapsed
// level 1 R1 over [X0/2-1, X0/2+16] (18, "the R1 region").  Entries at coordinates outside the
// mosaic hold the reflected coordinate's value, so reflected lookups land in range.  Three
// kernels, all with small LDS footprints (many blocks per CU) and no FP64 map in the capture
// loop:
//   mcs_mb_prep_c*_i*   once per plan: per (tile, owner) the source window + folded bilinear
//                       weights of every level-0 sample (mb_desc), and per tile the seam masks
//                       m1 (R1 region), m2, and their sums over the owners (the denominators);
//   mcs_mb_levels_c*    per (tile, owner, 4 captures): samples -> level 0 (LDS) -> separable
//                       5-tap reduces -> g1 (R1 region, u16) and g2 to a scratch buffer;
//   mcs_mb_blend_c*     per (tile, capture): B2, R1 = B1 + up(B2), R0 = L0_owner + up(R1) over
//                       the tile's pixels; level 0 of the owner is the owner sample the stitch
//                       kernel already wrote (equal to the replicate-border sample wherever the
//                       owner covers the pixel, which it always does).
// Long launches run in chunks of captures so the scratch stays a few tens of MB.
constexpr int kMbO1 = 6, kMbO2 = 2, kMbOR = 1;       // array origins: O/2 - 6, O/4 - 2, O/2 - 1
constexpr int kMbU = kMbUsedX * kMbUsedY;             // level-0 samples per owner
constexpr int kMbFoot = 28672;      // bytes of one LDS footprint buffer
constexpr int kMbFootBufs = 1;      // 2: double buffer, 1: refilled during the reduces
constexpr int kMbRS = kMbO1 - kMbOR;                  // R1 region origin in the level-1 array (5)
// Level scratch of one (tile, owner, capture), row-major (a band's lanes, adjacent columns,
// store contiguous bytes): g1 (R1 region, 8 B entries) at row * kMbNRX + col, g2 with the
// channels of an entry together at (row * kMbN2X + col) * CN + channel.
__device__ __forceinline__ int mb_g1_at(int col, int row) { return row * kMbNRX + col; }
template <int CN>
__device__ __forceinline__ int mb_g2_at(int col, int row, int k)
{
    return (row * kMbN2X + col) * CN + k;
}

// Expand taps of fine index x into a coarse level of size n (IN: no reflection needed).
template <bool IN>
__device__ __forceinline__ void exp_taps(int x, int n, int *idx, int *wt)
{
    if ((x & 1) == 0) {
        idx[0] = IN ? x / 2 - 1 : refl(x / 2 - 1, n), wt[0] = 1;
        idx[1] = IN ? x / 2 : refl(x / 2, n), wt[1] = 6;
        idx[2] = IN ? x / 2 + 1 : refl(x / 2 + 1, n), wt[2] = 1;
        return;
    }
    idx[0] = IN ? (x - 1) / 2 : refl((x - 1) / 2, n), wt[0] = 4;
    idx[1] = IN ? (x + 1) / 2 : refl((x + 1) / 2, n), wt[1] = 4;
    idx[2] = idx[1], wt[2] = 0;   // padding tap: adds an exact 0, keeps the trip count fixed
}

// Parity class of a fine position's expand taps: bit 0 = odd column (2 taps), bit 1 = odd row.
// (Reflection at the level's borders keeps parity: refl(-i) = i, refl(n - 1 + i) = n - 1 - i.)
__device__ __forceinline__ int mb_cls(int x, int y) { return (x & 1) | ((y & 1) << 1); }

// Geometry of one multi-band tile: level sizes and the origins of the arrays held per level.
struct MbGeo {
    int W, H, w1, h1, w2, h2;
    int X0, Y0, RX, RY, X1, Y1, X2, Y2, XR, YR;
    bool interior;
};

__device__ __forceinline__ MbGeo mb_geo(const KParams &P, int t)
{
    MbGeo G;
    G.W = P.out_w;
    G.H = P.out_h;
    G.w1 = (G.W + 1) / 2, G.h1 = (G.H + 1) / 2, G.w2 = (G.w1 + 1) / 2, G.h2 = (G.h1 + 1) / 2;
    const int gx = (G.W + kBlendTileW - 1) / kBlendTileW;
    G.X0 = (t % gx) * kBlendTileW, G.Y0 = (t / gx) * kBlendTileH;
    G.RX = G.X0 - kBlendHalo, G.RY = G.Y0 - kBlendHalo;         // level-0 origin
    G.X1 = G.X0 / 2 - kMbO1, G.Y1 = G.Y0 / 2 - kMbO1;             // level-1 origin
    G.X2 = G.X0 / 4 - kMbO2, G.Y2 = G.Y0 / 4 - kMbO2;             // level-2 origin
    G.XR = G.X0 / 2 - kMbOR, G.YR = G.Y0 / 2 - kMbOR;             // R1 origin
    G.interior = G.RX >= 0 && G.RY >= 0 && G.RX + kBlendTileW + 2 * kBlendHalo <= G.W &&
                 G.RY + kBlendTileH + 2 * kBlendHalo <= G.H;
    return G;
}

// Level coordinate -> reflected coordinate.  IN (interior tile): every coordinate the tile
// touches lies inside its level, so the reflection is the identity and index arithmetic folds.
template <bool IN>
__device__ __forceinline__ int rf(int i, int n) { return IN ? i : refl(i, n); }
template <bool IN>
__device__ __forceinline__ int ix2(int c, int o, int n)
{
    return IN ? c - o : min(max(c - o, 0), n - 1);
}

// Replicate-border bilinear sample of slot s at output (x, y) (sample_replicate): tap rows ya,
// yb, the window's first pixel c, meta = fx' | fy << 6, where fx' is the horizontal fraction
// with the replicate border folded in: both taps on the window's pixel 0 -> 0, both on pixel 1
// -> 32 (the weights then sum onto one pixel, as the clamped taps do).
struct MbSrc {
    int ya, yb, c;
    uint32_t meta;
};

template <int INTERP>
__device__ __forceinline__ MbSrc mb_src(const KParams &P, int s, int x, int y)
{
    int x32, y32, cam, w, h;
    slot_xy<INTERP>(P, s, x, y, x32, y32, cam, w, h);
    const int sx = x32 >> 5, sy = y32 >> 5;
    MbSrc r;
    r.c = w >= 2 ? min(max(sx, 0), w - 2) : 0;
    const bool a_hi = min(max(sx, 0), w - 1) > r.c;       // left tap on pixel 1
    const bool b_hi = min(max(sx + 1, 0), w - 1) > r.c;   // right tap on pixel 1
    const uint32_t fx = a_hi ? 32u : (b_hi ? (uint32_t)(x32 & 31) : 0u);
    r.ya = min(max(sy, 0), h - 1);
    r.yb = min(max(sy + 1, 0), h - 1);
    r.meta = fx | ((uint32_t)(y32 & 31) << 6);
    return r;
}

// Global-memory window descriptor of a sample (frame of w x h x CN): .x = byte offset of tap row
// a in the frame (bit 31: tap row b is the next row, else the same row); .y = meta | d << 12,
// where d = bytes both windows start earlier so that row b's window ends inside the frame (the
// taps then sit at bytes d and d + CN).  Every capture's load is then unconditional.  Frames
// with (h - 1) * w * CN < 16 bytes take load8's guarded path instead.
// Bits 15..18 of .y: the band pass's dword-aligned form (mb_bands<.., AL>): both tap rows read as
// 12-byte windows starting sh bytes before tap a, at a 4-byte boundary (sh <= 12 - 2 CN: the
// taps' 2 CN bytes inside the window; chosen so that row b's window ends inside the frame);
// 15 = no such window.  Valid wherever the host enables
// that form (band_aligned: pitch and frame bytes multiples of 4, frames of >= pitch + 12 bytes).
template <int CN>
__device__ __forceinline__ uint2 mb_desc(const MbSrc &q, int w, int h)
{
    const int64_t pitch = (int64_t)w * CN, fbytes = pitch * h;
    const int64_t oa = q.ya * pitch + (int64_t)q.c * CN, ob = oa + (q.yb > q.ya ? pitch : 0);
    const uint32_t d = (uint32_t)min(max(ob + 8 - fbytes, (int64_t)0), (int64_t)7);
    const int64_t e = fbytes - (ob - oa) - 12;   // last start of row a's window
    int64_t o4 = oa & ~(int64_t)3;
    if (o4 > e) o4 = e & ~(int64_t)3;
    const uint32_t sh = (e >= 0 && oa - o4 <= 12 - 2 * CN) ? (uint32_t)(oa - o4) : 15u;
    return make_uint2((uint32_t)oa | (q.yb > q.ya ? 0x80000000u : 0u),
                      q.meta | (d << 12) | (sh << 15));
}

// The 8 bytes starting sh (<= 10) bytes into a 12-byte window, zero past its end (v_alignbyte
// funnel shifts).
// 6 a + b for packed u16 pairs whose product does not fit 24 bits, as two full-rate shift-adds
// (the compiler otherwise emits the multiply as a v_mad_u64_u32)
__device__ __forceinline__ uint32_t mad6_u32(uint32_t a, uint32_t b)
{
    uint32_t t, r;
    asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(t) : "v"(a), "v"(b));
    asm("v_lshl_add_u32 %0, %1, 2, %2" : "=v"(r) : "v"(a), "v"(t));
    return r;
}

// The LDS-ring window (mb_bands_body mode 2): 4-byte aligned in the ring, byte shift sh < 4, so
// the 8 bytes are two alignbytes (no third dword's select as in mb_win_shift).
__device__ __forceinline__ uint2 mb_win_shift4(uint3 v, uint32_t sh)
{
    return make_uint2(__builtin_amdgcn_alignbyte(v.y, v.x, sh & 3u),
                      __builtin_amdgcn_alignbyte(v.z, v.y, sh & 3u));
}

template <int CN>
__device__ __forceinline__ uint2 mb_win_shift(uint3 v, uint32_t sh)
{
    const uint32_t s = sh & 3u;
    const uint32_t a = __builtin_amdgcn_alignbyte(v.y, v.x, s);
    const uint32_t b = __builtin_amdgcn_alignbyte(v.z, v.y, s);
    const uint32_t c = __builtin_amdgcn_alignbyte(0u, v.z, s);
    if (CN <= 2 && (sh & 8u)) return make_uint2(c, 0u);   // (sh > 6 only for 1 or 2 channels)
    return (sh & 4u) ? make_uint2(b, c) : make_uint2(a, b);
}

// Source footprint of one (tile, owner) staged in LDS per capture (mb_levels): rows
// [rmin, rmin + rows), bytes [cal, cal + stride) of each (cal 16-byte aligned, stride a multiple
// of 16), rows `stride` bytes apart in LDS.  The frame's last row is fetched `e` bytes earlier so
// that no 16-byte chunk crosses the frame end.  A sample's LDS descriptor: .x = LDS offsets of
// its two tap-row windows (16 bits each), .y = meta.
struct MbFoot {
    int rmin, rows, cal, stride, e, fits, pad0, pad1;
};

__device__ __forceinline__ uint32_t mb_foot_off(const MbFoot &F, int row, int byte, int h)
{
    return (uint32_t)((row - F.rmin) * F.stride + byte - F.cal + (row == h - 1 ? F.e : 0));
}

// The descriptor's 15-bit weights as u16 pairs on the window's pixels 0 / 1, row a and row b:
// (32 - fx', fx') * 32 (32 - fy) and * 32 fy (each lane <= 32768: no carry between lanes), so
// that mb_tap() gives sample_replicate's (sum p w + 2^14) >> 15 exactly.
__device__ __forceinline__ void mb_weights(uint32_t meta, uint32_t &wa, uint32_t &wb)
{
    const uint32_t fx = meta & 63u, fy = (meta >> 6) & 31u;
    const uint32_t wx = (32u - fx) | (fx << 16);
    wa = wx * ((32u - fy) << 5);
    wb = wx * (fy << 5);
}

// mb_weights with every weight doubled, min(2 w, 65535) (the stitch kernels' w2x): a channel's
// mb_tap2 sum then carries mb_tap's (sum p w + 2^14) >> 15 in its byte 2 -- s = 2 sum p w + 2^15
// < 2^24; the one weight 2 w = 65536 (fx' = 0 or 32 with fy = 0: all on one pixel) clamps to
// 65535, and 65535 p + 2^15 still has p in byte 2 -- so the band pass packs channels with one
// v_perm instead of shifting, masking and or-ing each.
__device__ __forceinline__ void mb_weights2(uint32_t meta, uint32_t &wa, uint32_t &wb)
{
    const uint32_t fx = meta & 63u, fy = (meta >> 6) & 31u;
    const uint32_t ya = (32u - fy) << 6, yb = fy << 6;
    wa = min((32u - fx) * ya, 65535u) | (min(fx * ya, 65535u) << 16);
    wb = min((32u - fx) * yb, 65535u) | (min(fx * yb, 65535u) << 16);
}

// Channel k of a descriptor's sample from its two (shifted) row windows.
template <int CN>
__device__ __forceinline__ uint32_t mb_tap(uint2 r0, uint2 r1, uint32_t wa, uint32_t wb, int k,
                                           uint32_t d)
{
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const uint32_t sel = ((uint32_t)k | (0x0cu << 8) | ((uint32_t)(CN + k) << 16) | (0x0cu << 24)) +
                         d * 0x00010001u;
    const uint32_t a0 = __builtin_amdgcn_perm(r0.y, r0.x, sel);
    const uint32_t a1 = __builtin_amdgcn_perm(r1.y, r1.x, sel);
    uint32_t v = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, a0), __builtin_bit_cast(us2, wa),
                                        16384u, false);
    v = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, a1), __builtin_bit_cast(us2, wb), v, false);
    return v >> 15;
}

// Channel k of a sample with mb_weights2's doubled weights: the value is byte 2 of the result.
template <int CN>
__device__ __forceinline__ uint32_t mb_tap2(uint2 r0, uint2 r1, uint32_t wa, uint32_t wb, int k,
                                            uint32_t d)
{
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const uint32_t sel = ((uint32_t)k | (0x0cu << 8) | ((uint32_t)(CN + k) << 16) | (0x0cu << 24)) +
                         d * 0x00010001u;
    const uint32_t a0 = __builtin_amdgcn_perm(r0.y, r0.x, sel);
    const uint32_t a1 = __builtin_amdgcn_perm(r1.y, r1.x, sel);
    const uint32_t v = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, a0),
                                              __builtin_bit_cast(us2, wa), 32768u, false);
    return __builtin_amdgcn_udot2(__builtin_bit_cast(us2, a1), __builtin_bit_cast(us2, wb), v,
                                  false);
}

// Makes a register array opaque to the optimiser (one asm per capture): values derived from it
// are then recomputed per capture instead of being hoisted out of the capture loop and held.
template <int N>
__device__ __forceinline__ void mb_opaque(uint32_t (&v)[N])
{
#pragma unroll
    for (int i = 0; i < N; i += 4) {
        if (i + 3 < N) asm volatile("" : "+v"(v[i]), "+v"(v[i + 1]), "+v"(v[i + 2]), "+v"(v[i + 3]));
        else if (i + 2 < N) asm volatile("" : "+v"(v[i]), "+v"(v[i + 1]), "+v"(v[i + 2]));
        else if (i + 1 < N) asm volatile("" : "+v"(v[i]), "+v"(v[i + 1]));
        else asm volatile("" : "+v"(v[i]));
    }
}

// e / D for 0 <= e < 2^16 / D (multiply-shift, exact in that range: D = 12, 18 here)
template <int D>
__device__ __forceinline__ int div_small(int e)
{
    return (int)(__umul24((unsigned)e, (65536u + D - 1) / D) >> 16);
}

// Sample e of a tile's compacted level-0 columns [a0, a0 + w0) -> its 57 x 57 array index.
__device__ __forceinline__ int mb_sample_index(int e, int a0, int w0)
{
    const int r = e / w0;
    return r * kMbUsedX + a0 + (e - r * w0);
}

// Local slot j (0 .. popc(mask) - 1) -> plan slot: the j-th set bit of mask.
__device__ __forceinline__ int mb_slot(uint32_t mask, int j)
{
    for (int q = 0; q < j; q++) mask &= mask - 1;
    return __ffs(mask) - 1;
}

// ---- prep (once per plan): grid (listed tiles), block kMbPrepThreads ---------------------------
template <int CN, int INTERP>
__device__ __forceinline__ void mb_prep(const KMbArgs &a)
{
    __shared__ uint8_t own[kMbU];
    __shared__ int32_t m1[kBlendSlots][kMbN1X * kMbN1Y];
    __shared__ int32_t m2[kBlendSlots][kMbN2X * kMbN2Y];
    const KParams &P = a.P;
    const int bt = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    const uint32_t mask = (uint32_t)a.list[2 + 2 * bt];
    const int ns = __popc(mask);
    const MbGeo G = mb_geo(P, a.list[1 + 2 * bt]);
    const int w5[5] = {1, 4, 6, 4, 1};
    // owner map of the used neighbourhood as local slot indices (bit rank in `mask`)
    for (int i = tid; i < kMbU; i += nt) {
        const int cx = refl(G.RX + kMbFirst + i % kMbUsedX, G.W);
        const int cy = refl(G.RY + kMbFirst + i / kMbUsedX, G.H);
        const int o = a.owner[(int64_t)cy * G.W + cx];
        own[i] = (uint8_t)((o != kBlendNone && ((mask >> o) & 1u))
                               ? __popc(mask & ((1u << o) - 1u)) : kBlendNone);
    }
    const int RX2 = G.RX + kMbFirst, RY2 = G.RY + kMbFirst;
    // m1 = reduce(owner == slot) over the level-1 array (25-tap form with reflection)
    for (int i = tid; i < kMbN1X * kMbN1Y * ns; i += nt) {
        const int j = i / (kMbN1X * kMbN1Y), e = i % (kMbN1X * kMbN1Y);
        const int qx = refl(G.X1 + e % kMbN1X, G.w1), qy = refl(G.Y1 + e / kMbN1X, G.h1);
        int macc = 0;
        for (int u = 0; u < 5; u++) {
            const int cy = refl(2 * qy + u - 2, G.H);
            for (int v = 0; v < 5; v++) {
                const int cx = refl(2 * qx + v - 2, G.W);
                const int p = ix2<false>(cy, RY2, kMbUsedY) * kMbUsedX + ix2<false>(cx, RX2, kMbUsedX);
                macc += own[p] == j ? w5[u] * w5[v] : 0;
            }
        }
        m1[j][e] = macc;
    }
    __syncthreads();
    // m2 = reduce(m1)
    for (int i = tid; i < kMbN2X * kMbN2Y * ns; i += nt) {
        const int j = i / (kMbN2X * kMbN2Y), e = i % (kMbN2X * kMbN2Y);
        const int zx = refl(G.X2 + e % kMbN2X, G.w2), zy = refl(G.Y2 + e / kMbN2X, G.h2);
        int macc = 0;
        for (int u = 0; u < 5; u++) {
            const int qy = refl(2 * zy + u - 2, G.h1);
            for (int v = 0; v < 5; v++) {
                const int qx = refl(2 * zx + v - 2, G.w1);
                const int p = ix2<false>(qy, G.Y1, kMbN1Y) * kMbN1X + ix2<false>(qx, G.X1, kMbN1X);
                macc += w5[u] * w5[v] * m1[j][p];
            }
        }
        m2[j][e] = macc;
    }
    __syncthreads();
    // table: m1 (R1 region) [slots], m2 [slots], d1 (R1 region), d2
    int32_t *tab = a.tab + (int64_t)bt * mb_tab_words(a.slots);
    int32_t *t_m1 = tab, *t_m2 = tab + a.slots * kMbNRX * kMbNRY;
    int32_t *t_d1 = t_m2 + a.slots * kMbN2X * kMbN2Y, *t_d2 = t_d1 + kMbNRX * kMbNRY;
    for (int e = tid; e < kMbNRX * kMbNRY; e += nt) {
        const int p = (e / kMbNRX + kMbRS) * kMbN1X + e % kMbNRX + kMbRS;
        int d = 0;
        for (int j = 0; j < a.slots; j++) {
            const int v = j < ns ? m1[j][p] : 0;
            t_m1[j * kMbNRX * kMbNRY + e] = v;
            d += v;
        }
        t_d1[e] = d;
    }
    for (int e = tid; e < kMbN2X * kMbN2Y; e += nt) {
        int d = 0;
        for (int j = 0; j < a.slots; j++) {
            const int v = j < ns ? m2[j][e] : 0;
            t_m2[j * kMbN2X * kMbN2Y + e] = v;
            d += v;
        }
        t_d2[e] = d;
    }
    // The blend work lists.  A pixel's collapse equals its owner's sample exactly (bit for bit)
    // when no other owner's level-2 mask reaches a level-2 tap of its level-1 taps: B1 and B2 are
    // then the owner's own l1 / 2^22 and g2 / 2^16 (one-term quotients of exact integers), R1 =
    // g1 / 256 and R0 = g0 exactly (all dyadic, no rounding).  The stitch kernel has written that
    // sample (or the border 0 where no camera covers the pixel), so the blend kernel computes only
    // the other ("mixed") pixels and the R1 entries they read.
    __shared__ int need_r1[kMbNRX * kMbNRY];
    __shared__ int n_px, n_r1;
    // Both lists are stored grouped by the parity class of their expand taps (mb_cls: row
    // parity, column parity -> 3 or 2 taps per axis), so the blend kernel's waves run one
    // fixed-count tap body each (4, 6 or 9 taps instead of 9 with zero-weight padding)
    __shared__ uint8_t px_cls[kMbTilePx];
    __shared__ int cls_n[2][4], cls_at[2][4];
    // per owner slot: mosaic level-1 / level-2 columns the blend reads from it (band pass)
    __shared__ int nq1lo[kBlendSlots], nq1hi[kBlendSlots], nz2lo[kBlendSlots], nz2hi[kBlendSlots];
    int32_t *t_cnt = t_d2 + kMbN2X * kMbN2Y;
    uint16_t *t_px = reinterpret_cast<uint16_t *>(t_cnt + kMbTabCounts);
    uint16_t *t_r1 = t_px + kMbTilePx;
    for (int e = tid; e < kMbNRX * kMbNRY; e += nt) need_r1[e] = 0;
    for (int i = tid; i < kMbTilePx; i += nt) px_cls[i] = 255;
    if (tid < 8) cls_n[tid >> 2][tid & 3] = 0;
    if (tid == 0) n_px = n_r1 = 0;
    if (tid < kBlendSlots) {
        nq1lo[tid] = nz2lo[tid] = 1 << 30;
        nq1hi[tid] = nz2hi[tid] = -(1 << 30);
    }
    __syncthreads();
    for (int i = tid; i < kMbTilePx; i += nt) {
        const int x = G.X0 + i % kBlendTileW, y = G.Y0 + i / kBlendTileW;
        if (x >= G.W || y >= G.H) continue;
        const int o = a.owner[(int64_t)y * G.W + x];
        if (o == kBlendNone) continue;
        const int s = __popc(mask & ((1u << o) - 1u));
        int iy[3], wy[3], ix[3], wx[3];
        exp_taps<false>(y, G.h1, iy, wy);
        exp_taps<false>(x, G.w1, ix, wx);
        bool mixed = false;
        for (int u = 0; u < 3; u++)
            for (int v = 0; v < 3; v++) {
                int zy[3], uy[3], zx[3], ux[3];
                exp_taps<false>(iy[u], G.h2, zy, uy);
                exp_taps<false>(ix[v], G.w2, zx, ux);
                for (int b = 0; b < 3; b++)
                    for (int c = 0; c < 3; c++) {
                        const int e2 = ix2<false>(zy[b], G.Y2, kMbN2Y) * kMbN2X +
                                       ix2<false>(zx[c], G.X2, kMbN2X);
                        for (int j = 0; j < ns; j++)
                            mixed = mixed || (j != s && m2[j][e2] > 0);
                    }
            }
        if (!mixed) continue;
        atomicAdd(&n_px, 1);
        px_cls[i] = (uint8_t)mb_cls(x, y);
        atomicAdd(&cls_n[0][px_cls[i]], 1);
        for (int u = 0; u < 3; u++)
            for (int v = 0; v < 3; v++)
                need_r1[ix2<false>(iy[u], G.YR, kMbNRY) * kMbNRX + ix2<false>(ix[v], G.XR, kMbNRX)] =
                    1;
        // R0 reads the owner's g1 at the pixel's level-1 taps
        atomicMin(&nq1lo[s], min(ix[0], ix[1]));
        atomicMax(&nq1hi[s], max(ix[1], ix[2]));
    }
    __syncthreads();
    for (int e = tid; e < kMbNRX * kMbNRY; e += nt)
        if (need_r1[e]) {
            atomicAdd(&n_r1, 1);
            atomicAdd(&cls_n[1][mb_cls(G.XR + e % kMbNRX, G.YR + e / kMbNRX)], 1);
        }
    __syncthreads();
    if (tid < 2) {
        int at = 0;
        for (int c = 0; c < 4; c++) cls_at[tid][c] = at, at += cls_n[tid][c];
    }
    __syncthreads();
    for (int i = tid; i < kMbTilePx; i += nt)
        if (px_cls[i] != 255) t_px[atomicAdd(&cls_at[0][px_cls[i]], 1)] = (uint16_t)i;
    for (int e = tid; e < kMbNRX * kMbNRY; e += nt)
        if (need_r1[e])
            t_r1[atomicAdd(&cls_at[1][mb_cls(G.XR + e % kMbNRX, G.YR + e / kMbNRX)], 1)] =
                (uint16_t)e;
    // R1 at a listed entry reads owner j's g1 there and g2 at its level-2 taps where m1_j > 0,
    // and B2 at those taps reads g2_j where m2_j > 0 (positions in the mosaic: reflected, as the
    // blend kernel addresses them)
    for (int e = tid; e < kMbNRX * kMbNRY; e += nt) {
        if (!need_r1[e]) continue;
        const int ey = e / kMbNRX, ex = e % kMbNRX;
        const int p = (ey + kMbRS) * kMbN1X + ex + kMbRS;
        const int qx = G.XR + ex, qy = G.YR + ey;
        int zy[3], uy[3], zx[3], ux[3];
        exp_taps<false>(qy, G.h2, zy, uy);
        exp_taps<false>(qx, G.w2, zx, ux);
        for (int j = 0; j < ns; j++) {
            if (m1[j][p] > 0) {
                atomicMin(&nq1lo[j], qx);
                atomicMax(&nq1hi[j], qx);
            }
            for (int b = 0; b < 3; b++)
                for (int c = 0; c < 3; c++)
                    if (m2[j][ix2<false>(zy[b], G.Y2, kMbN2Y) * kMbN2X +
                              ix2<false>(zx[c], G.X2, kMbN2X)] > 0) {
                        atomicMin(&nz2lo[j], zx[c]);
                        atomicMax(&nz2hi[j], zx[c]);
                    }
        }
    }
    __syncthreads();
    // Column ranges of the level arrays the mixed pixels depend on (interior tiles; mosaic-border
    // tiles keep the full arrays): R1 entries -> their level-2 taps -> the level-1 entries the R1
    // region and those taps reduce from -> the level-0 samples.  mb_levels computes only these.
    __shared__ int r1lo, r1hi, rng[6];
    if (tid == 0) r1lo = kMbNRX, r1hi = -1;
    __syncthreads();
    for (int e = tid; e < kMbNRX * kMbNRY; e += nt)
        if (need_r1[e]) {
            atomicMin(&r1lo, e % kMbNRX);
            atomicMax(&r1hi, e % kMbNRX);
        }
    __syncthreads();
    if (tid == 0) {
        int a0_ = 0, b0_ = kMbUsedX - 1, a1_ = 0, b1_ = kMbN1X - 1, a2_ = 0, b2_ = kMbN2X - 1;
        if (n_px == 0) {
            a0_ = a1_ = a2_ = 0;
            b0_ = b1_ = b2_ = -1;
        } else if (G.interior) {
            int zlo = 1 << 30, zhi = -(1 << 30);
            for (int q = G.XR + r1lo; q <= G.XR + r1hi; q++) {
                int zi[3], zw[3];
                exp_taps<true>(q, G.w2, zi, zw);
                zlo = min(zlo, min(zi[0], zi[1]));
                zhi = max(zhi, max(zi[1], zi[2]));
            }
            a2_ = max(zlo - G.X2, 0);
            b2_ = min(zhi - G.X2, kMbN2X - 1);
            a1_ = max(min(G.XR + r1lo, 2 * zlo - 2) - G.X1, 0);
            b1_ = min(max(G.XR + r1hi, 2 * zhi + 2) - G.X1, kMbN1X - 1);
            a0_ = max(2 * (a1_ + G.X1) - 2 - (G.RX + kMbFirst), 0);
            b0_ = min(2 * (b1_ + G.X1) + 2 - (G.RX + kMbFirst), kMbUsedX - 1);
        }
        rng[0] = a0_, rng[1] = b0_, rng[2] = a1_, rng[3] = b1_, rng[4] = a2_, rng[5] = b2_;
        t_cnt[0] = n_px;
        t_cnt[1] = n_r1;
        for (int q = 0; q < 6; q++) t_cnt[2 + q] = rng[q];
        for (int j = 0; j < kBlendSlots; j++) {
            int q1lo = nq1lo[j], q1hi = nq1hi[j], z2lo = nz2lo[j], z2hi = nz2hi[j];
            if (n_px == 0 || j >= ns) {
                q1lo = z2lo = 1 << 30;
                q1hi = z2hi = -(1 << 30);
            } else if (q1lo <= q1hi) {
                // the level-2 taps of those g1 entries (L1 = 16384 g1 - E(g2))
                z2lo = min(z2lo, (q1lo - 1) >> 1);
                z2hi = max(z2hi, (q1hi >> 1) + 1);
            }
            t_cnt[kMbTabRanges + 4 * j + 0] = q1lo;
            t_cnt[kMbTabRanges + 4 * j + 1] = q1hi;
            t_cnt[kMbTabRanges + 4 * j + 2] = z2lo;
            t_cnt[kMbTabRanges + 4 * j + 3] = z2hi;
        }
    }
    __syncthreads();
    const int a0 = rng[0], w0 = rng[1] - rng[0] + 1, n_s = kMbUsedY * w0;
    // every owner's source footprint (bounding box of its taps) ...
    __shared__ int f_rmin[kBlendSlots], f_rmax[kBlendSlots], f_bmin[kBlendSlots],
        f_bmax[kBlendSlots];
    __shared__ MbFoot foot[kBlendSlots];
    if (tid < kBlendSlots) {
        f_rmin[tid] = f_bmin[tid] = 0x7fffffff;
        f_rmax[tid] = f_bmax[tid] = -1;
    }
    __syncthreads();
    for (int i = tid; i < n_s * ns; i += nt) {
        const int j = i / n_s, e = i % n_s;
        const int g = mb_sample_index(e, a0, w0);
        const int cx = refl(G.RX + kMbFirst + g % kMbUsedX, G.W);
        const int cy = refl(G.RY + kMbFirst + g / kMbUsedX, G.H);
        const MbSrc q = mb_src<INTERP>(P, mb_slot(mask, j), cx, cy);
        atomicMin(&f_rmin[j], q.ya);
        atomicMax(&f_rmax[j], q.yb);
        atomicMin(&f_bmin[j], q.c * CN);
        atomicMax(&f_bmax[j], q.c * CN + 2 * CN);
    }
    __syncthreads();
    if (tid < ns) {
        int cam, w, h;
        slot_info(P, mb_slot(mask, tid), cam, w, h);
        const int64_t pitch = (int64_t)w * CN;
        MbFoot F;
        F.rmin = f_rmin[tid];
        F.rows = f_rmax[tid] - f_rmin[tid] + 1;
        F.cal = f_bmin[tid] & ~15;
        F.stride = (f_bmax[tid] - F.cal + 15) & ~15;
        F.e = 0;
        // (rows above the last one may run into the next row, never past the frame)
        F.fits = F.rows * F.stride + kLdsSlack <= kMbFoot &&
                 F.stride <= 16 * kWave && F.cal + F.stride <= 2 * pitch;
        if (f_rmax[tid] == h - 1 && F.cal + F.stride > pitch) {
            F.e = (int)(F.cal + F.stride - pitch);
            if ((int64_t)(h - 1) * pitch + F.cal - F.e < 0) F.fits = 0;
        }
        F.pad0 = F.pad1 = 0;
        foot[tid] = F;
        reinterpret_cast<MbFoot *>(a.foot)[(int64_t)bt * a.slots + tid] = F;
    }
    __syncthreads();
    // ... and every needed level-0 sample's windows: LDS offsets in the footprint, or frame
    // offsets; .y bits 16-27 = its index in the 57 x 57 level-0 array
    for (int i = tid; i < n_s * ns; i += nt) {
        const int j = i / n_s, e = i % n_s;
        const int g = mb_sample_index(e, a0, w0);
        const int cx = refl(G.RX + kMbFirst + g % kMbUsedX, G.W);
        const int cy = refl(G.RY + kMbFirst + g / kMbUsedX, G.H);
        const int sj = mb_slot(mask, j);
        const MbSrc q = mb_src<INTERP>(P, sj, cx, cy);
        int cam, w, h;
        slot_info(P, sj, cam, w, h);
        const MbFoot &F = foot[j];
        uint2 v;
        if (F.fits) {
            v.x = mb_foot_off(F, q.ya, q.c * CN, h) | (mb_foot_off(F, q.yb, q.c * CN, h) << 16);
            v.y = q.meta;
        } else {
            v = mb_desc<CN>(q, w, h);
        }
        v.y |= (uint32_t)g << 16;
        a.desc[((int64_t)bt * a.slots + j) * kMbU + e] = (uint64_t)v.x | ((uint64_t)v.y << 32);
    }
}

// ---- levels: grid (listed tiles, slots, ceil(nf / kMbLvFrames)), block kMbLvThreads -------------
template <int CN>
struct MbLvLds {
    uint8_t foot[kMbFootBufs][kMbFoot] __attribute__((aligned(16)));   // source footprints
    // (one spare entry past each array: the branch-free stores of out-of-range items land there)
    uint32_t g0[kMbU + 1];             // level 0: channel k in byte k
    uint2 g1[kMbN1X * kMbN1Y + 1];     // 256 G1 <= 65280 as u16 lanes: x = (c0, c2), y = (c1, c3)
    union {
        uint2 hs[kMbUsedY * kMbN1X + 1];   // horizontal pass of level 1 (<= 4080), lanes as g1
        int4 hs2[kMbN1Y * kMbN2X];     // horizontal pass of level 2, one int per channel
    };
};

// u16 lane of channel k in a packed level-1 entry (x = (c0, c2), y = (c1, c3))
__device__ __forceinline__ int ch16(uint2 v, int k)
{
    return (int)((((k & 1) ? v.y : v.x) >> ((k & 2) ? 16 : 0)) & 0xffffu);
}

template <int CN>
__device__ __forceinline__ void mb_levels(const KMbArgs &a, MbLvLds<CN> &L)
{
    constexpr int NT = kMbLvThreads, KJ = (kMbU + NT - 1) / NT;
    const KParams &P = a.P;
    const int bt = blockIdx.x, j = blockIdx.y, tid = threadIdx.x;
    const uint32_t mask = (uint32_t)a.list[2 + 2 * bt];
    if (j >= __popc(mask)) return;   // uniform: the whole block leaves before any barrier
    const MbGeo G = mb_geo(P, a.list[1 + 2 * bt]);
    // the column ranges the tile's mixed pixels depend on (mb_prep): level 0 [a0, a0 + w0),
    // level 1 [a1, a1 + w1), level 2 [a2, a2 + w2); all rows
    const int32_t *rg = a.tab + (int64_t)bt * mb_tab_words(a.slots) +
                        a.slots * (kMbNRX * kMbNRY + kMbN2X * kMbN2Y) + kMbNRX * kMbNRY +
                        kMbN2X * kMbN2Y + 2;
    const int w0 = rg[1] - rg[0] + 1, a1 = rg[2], w1 = rg[3] - rg[2] + 1;
    const int a2 = rg[4], w2 = rg[5] - rg[4] + 1;
    const int n_s = kMbUsedY * w0;                   // level-0 samples (compacted columns)
    if (n_s <= 0) return;                            // no mixed pixel: nothing to do (uniform)
    const unsigned d1m = (65536u + w1 - 1) / w1, d2m = (65536u + w2 - 1) / w2;   // / w1, / w2
    int cam, w, h;
    slot_info(P, mb_slot(mask, j), cam, w, h);
    const int64_t pitch = (int64_t)w * CN, fbytes = pitch * h;
    const MbFoot F = reinterpret_cast<const MbFoot *>(a.foot)[(int64_t)bt * a.slots + j];
    const bool staged = F.fits;                      // footprint through LDS (else global loads)
    const bool shifted = (h - 1) * pitch >= 16;
    // this owner's sample windows, once for the block's captures (global path with frames of
    // (h - 1) * pitch < 16 bytes: re-read per capture, load8's guarded path)
    uint32_t doff[KJ], dmeta[KJ];
    const uint64_t *dsc = a.desc + ((int64_t)bt * a.slots + j) * kMbU;
#pragma unroll
    for (int kk = 0; kk < KJ; kk++) {
        const int i = tid + kk * NT;
        const uint64_t v = ((staged || shifted) && i < n_s) ? dsc[i] : 0ull;
        doff[kk] = (uint32_t)v;
        dmeta[kk] = (uint32_t)(v >> 32);
    }
    const int w5[5] = {1, 4, 6, 4, 1};
    const int fl0 = blockIdx.z * kMbLvFrames, fl1 = min(a.nf, fl0 + kMbLvFrames);
    // LDS-DMA of capture fl's footprint into buffer b: row r by wave r % 8, lane = 16-byte chunk
    const int wave = __builtin_amdgcn_readfirstlane(tid / kWave), lane = tid % kWave;
    auto stage = [&](int fl, int b) {
        const uint8_t *fb = P.cams[cam] + (int64_t)(a.f0 + fl) * P.cam_fstride[cam];
        for (int r = wave; r < F.rows; r += NT / kWave) {
            const int row = F.rmin + r;
            const uint8_t *src = fb + (int64_t)row * pitch + F.cal - (row == h - 1 ? F.e : 0);
            if (lane < (F.stride >> 4))
                __builtin_amdgcn_global_load_lds(src + 16 * lane,
                                                 ((lds_u8 *)L.foot[b]) + r * F.stride, 16, 0, 0);
        }
    };
    if (staged && fl0 < fl1) stage(fl0, 0);
    for (int fl = fl0; fl < fl1; fl++) {
        const uint8_t *fb = P.cams[cam] + (int64_t)(a.f0 + fl) * P.cam_fstride[cam];
        // level 0.  The descriptors are made opaque per capture so that the compiler does not
        // hoist their decoding out of the loop (which would hold ~5 registers per sample).
        if (staged) {
            // this capture's footprint has landed (every wave's DMA: wait + barrier); the next
            // one streams in while this one is processed
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (kMbFootBufs == 2 && fl + 1 < fl1) stage(fl + 1, (fl + 1 - fl0) & 1);
            const uint8_t *buf = L.foot[kMbFootBufs == 2 ? (fl - fl0) & 1 : 0];
            // all samples into registers first: a level-0 store between them would order the
            // next sample's LDS reads behind it (the compiler cannot tell the arrays apart)
            uint32_t px[KJ];
            mb_opaque(doff);
            mb_opaque(dmeta);
#pragma unroll
            for (int kk = 0; kk < KJ; kk++) {
                const uint2 r0 = lds_window(buf, doff[kk] & 0xffffu);
                const uint2 r1 = lds_window(buf, doff[kk] >> 16);
                uint32_t wa, wb;
                mb_weights(dmeta[kk], wa, wb);
                px[kk] = 0;
#pragma unroll
                for (int k = 0; k < CN; k++) px[kk] |= mb_tap<CN>(r0, r1, wa, wb, k, 0u) << (8 * k);
            }
#pragma unroll
            for (int kk = 0; kk < KJ; kk++)
                L.g0[tid + kk * NT < n_s ? (dmeta[kk] >> 16) & 0x1fffu : (uint32_t)kMbU] = px[kk];
        } else if (shifted) {
            struct __attribute__((packed)) U2 {
                uint32_t x, y;
            };
            typedef __attribute__((address_space(1))) const uint8_t gu8;
            typedef __attribute__((address_space(1))) const U2 gu2;
            const gu8 *gfb = (const gu8 *)fb;
            uint32_t px[KJ];
            mb_opaque(doff);
            mb_opaque(dmeta);
#pragma unroll
            for (int kk = 0; kk < KJ; kk++) {
                const uint32_t d = (dmeta[kk] >> 12) & 7u;
                const uint32_t o = (doff[kk] & 0x7fffffffu) - d;
                const uint32_t ob = o + ((doff[kk] >> 31) ? (uint32_t)pitch : 0u);
                const U2 ra = *(const gu2 *)(gfb + o), rb = *(const gu2 *)(gfb + ob);
                const uint2 r0 = make_uint2(ra.x, ra.y), r1 = make_uint2(rb.x, rb.y);
                uint32_t wa, wb;
                mb_weights(dmeta[kk], wa, wb);
                px[kk] = 0;
#pragma unroll
                for (int k = 0; k < CN; k++) px[kk] |= mb_tap<CN>(r0, r1, wa, wb, k, d) << (8 * k);
            }
#pragma unroll
            for (int kk = 0; kk < KJ; kk++)
                L.g0[tid + kk * NT < n_s ? (dmeta[kk] >> 16) & 0x1fffu : (uint32_t)kMbU] = px[kk];
        } else {
            for (int i = tid; i < n_s; i += NT) {
                const uint64_t v = dsc[i];
                const uint32_t o = (uint32_t)v & 0x7fffffffu;
                const uint32_t ob = o + (((uint32_t)v >> 31) ? (uint32_t)pitch : 0u);
                const uint2 r0 = load8<2 * CN>(fb, o, fbytes), r1 = load8<2 * CN>(fb, ob, fbytes);
                uint32_t wa, wb, px = 0;
                mb_weights((uint32_t)(v >> 32), wa, wb);
#pragma unroll
                for (int k = 0; k < CN; k++) px |= mb_tap<CN>(r0, r1, wa, wb, k, 0u) << (8 * k);
                L.g0[(uint32_t)(v >> 48) & 0x1fffu] = px;
            }
        }
        __syncthreads();
        // single buffer: the next capture's footprint streams in during this one's reduces
        if (kMbFootBufs == 1 && staged && fl + 1 < fl1) stage(fl + 1, 0);
        const int64_t job = ((int64_t)bt * a.slots + j) * a.chunk + fl;
        uint2 *og1 = reinterpret_cast<uint2 *>(a.g1) + job * (kMbNRX * kMbNRY);
        int32_t *og2 = a.g2 + job * (kMbN2X * kMbN2Y * CN);
        if (G.interior) {
            // separable 5-tap reduces, all channels at once in 16-bit lanes up to level 1 (the
            // sums stay below 2^16: exact), then per channel.  Level-1 entry e reads level-0
            // offsets 2e + [0, 5); level-2 entry z reads level-1 entries 2z + [0, 5).
            // (each thread's items are computed before any is stored, so that their LDS reads
            // are not ordered behind the stores; only the needed columns, all rows)
            {
                constexpr int IT = (kMbUsedY * kMbN1X + NT - 1) / NT;
                const int n = kMbUsedY * w1;
                uint2 res[IT];
#pragma unroll
                for (int q = 0; q < IT; q++) {
                    const int i = min(tid + q * NT, n - 1);
                    const int r = (int)(__umul24((unsigned)i, d1m) >> 16);
                    const int e = a1 + i - (int)__umul24((unsigned)r, (unsigned)w1);
                    const uint32_t *g = &L.g0[r * kMbUsedX + 2 * e];
                    uint32_t lo = 0, hi = 0;
#pragma unroll
                    for (int v = 0; v < 5; v++) {
                        const uint32_t t = g[v];
                        lo += (uint32_t)w5[v] * (t & 0x00ff00ffu);
                        hi += (uint32_t)w5[v] * ((t >> 8) & 0x00ff00ffu);
                    }
                    res[q] = make_uint2(lo, hi);
                }
#pragma unroll
                for (int q = 0; q < IT; q++) {
                    const int i = tid + q * NT;
                    const int r = (int)(__umul24((unsigned)i, d1m) >> 16);
                    L.hs[i < n ? r * kMbN1X + a1 + i - (int)__umul24((unsigned)r, (unsigned)w1)
                               : kMbUsedY * kMbN1X] = res[q];
                }
            }
            __syncthreads();
            {
                constexpr int IT = (kMbN1Y * kMbN1X + NT - 1) / NT;
                const int n = kMbN1Y * w1;
                uint2 res[IT];
#pragma unroll
                for (int q = 0; q < IT; q++) {
                    const int i = min(tid + q * NT, n - 1);
                    const int ey = (int)(__umul24((unsigned)i, d1m) >> 16);
                    const int ex = a1 + i - (int)__umul24((unsigned)ey, (unsigned)w1);
                    uint32_t lo = 0, hi = 0;
#pragma unroll
                    for (int u = 0; u < 5; u++) {
                        const uint2 t = L.hs[(2 * ey + u) * kMbN1X + ex];
                        lo += (uint32_t)w5[u] * t.x;
                        hi += (uint32_t)w5[u] * t.y;
                    }
                    res[q] = make_uint2(lo, hi);
                }
#pragma unroll
                for (int q = 0; q < IT; q++) {
                    const int i = tid + q * NT;
                    const int ey = (int)(__umul24((unsigned)i, d1m) >> 16);
                    L.g1[i < n ? ey * kMbN1X + a1 + i - (int)__umul24((unsigned)ey, (unsigned)w1)
                               : kMbN1X * kMbN1Y] = res[q];
                }
            }
            __syncthreads();
            for (int i = tid; i < kMbN1Y * w2; i += NT) {
                const int r = (int)(__umul24((unsigned)i, d2m) >> 16);
                const int e = a2 + i - (int)__umul24((unsigned)r, (unsigned)w2);
                int acc[4] = {0, 0, 0, 0};
#pragma unroll
                for (int v = 0; v < 5; v++) {
                    const uint2 t = L.g1[r * kMbN1X + 2 * e + v];
#pragma unroll
                    for (int k = 0; k < CN; k++) acc[k] += w5[v] * ch16(t, k);
                }
                L.hs2[r * kMbN2X + e] = make_int4(acc[0], acc[1], acc[2], acc[3]);
            }
            __syncthreads();
            for (int i = tid; i < kMbN2Y * w2; i += NT) {
                const int ey = (int)(__umul24((unsigned)i, d2m) >> 16);
                const int ex = a2 + i - (int)__umul24((unsigned)ey, (unsigned)w2);
                int acc[4] = {0, 0, 0, 0};
#pragma unroll
                for (int u = 0; u < 5; u++) {
                    const int4 t = L.hs2[(2 * ey + u) * kMbN2X + ex];
                    acc[0] += w5[u] * t.x;
                    acc[1] += w5[u] * t.y;
                    acc[2] += w5[u] * t.z;
                    acc[3] += w5[u] * t.w;
                }
#pragma unroll
                for (int k = 0; k < CN; k++) og2[mb_g2_at<CN>(ex, ey, k)] = acc[k];
            }
        } else {
            // mosaic-border tiles: 25-tap form with reflection at every level
            const int RX2 = G.RX + kMbFirst, RY2 = G.RY + kMbFirst;
            for (int e = tid; e < kMbN1X * kMbN1Y; e += NT) {
                const int qx = refl(G.X1 + e % kMbN1X, G.w1), qy = refl(G.Y1 + e / kMbN1X, G.h1);
                uint32_t lo = 0, hi = 0;
                for (int u = 0; u < 5; u++) {
                    const int cy = ix2<false>(refl(2 * qy + u - 2, G.H), RY2, kMbUsedY);
#pragma unroll
                    for (int v = 0; v < 5; v++) {
                        const int cx = ix2<false>(refl(2 * qx + v - 2, G.W), RX2, kMbUsedX);
                        const uint32_t t = L.g0[cy * kMbUsedX + cx], wt = w5[u] * w5[v];
                        lo += wt * (t & 0x00ff00ffu);
                        hi += wt * ((t >> 8) & 0x00ff00ffu);
                    }
                }
                L.g1[e] = make_uint2(lo, hi);
            }
            __syncthreads();
            for (int e = tid; e < kMbN2X * kMbN2Y; e += NT) {
                const int zx = refl(G.X2 + e % kMbN2X, G.w2), zy = refl(G.Y2 + e / kMbN2X, G.h2);
                int acc[4] = {0, 0, 0, 0};
                for (int u = 0; u < 5; u++) {
                    const int qy = ix2<false>(refl(2 * zy + u - 2, G.h1), G.Y1, kMbN1Y);
#pragma unroll
                    for (int v = 0; v < 5; v++) {
                        const int qx = ix2<false>(refl(2 * zx + v - 2, G.w1), G.X1, kMbN1X);
                        const uint2 t = L.g1[qy * kMbN1X + qx];
                        const int wt = w5[u] * w5[v];
#pragma unroll
                        for (int k = 0; k < CN; k++) acc[k] += wt * ch16(t, k);
                    }
                }
#pragma unroll
                for (int k = 0; k < CN; k++) og2[mb_g2_at<CN>(e % kMbN2X, e / kMbN2X, k)] = acc[k];
            }
        }
        // the R1 region of g1 (level-1 entries from kMbRS on, both axes)
        for (int e = tid; e < kMbNRX * kMbNRY; e += NT)
            og1[mb_g1_at(e % kMbNRX, e / kMbNRX)] =
                L.g1[(e / kMbNRX + kMbRS) * kMbN1X + e % kMbNRX + kMbRS];
        __syncthreads();   // the next capture overwrites level 0 and the pass arrays
    }
}

// ---- band pass: descriptors once per plan, then per chunk of captures ------------------------
// Band descriptors: grid (bands), block 256.  Per (array row r, lane l) the global-memory window
// descriptor (mb_desc) of the band's owner at mosaic (c0 + l, Y0 - 14 + r), positions reflected
// into the mosaic as mb_prep does (BORDER_DEFAULT: a lane or row past a mosaic edge holds the
// sample of its reflected position).
template <int CN, int INTERP>
__device__ __forceinline__ void mb_bdesc(const KMbBandArgs &a)
{
    const KParams &P = a.P;
    const MbBand B = a.bands[blockIdx.x];
    int cam, w, h;
    slot_info(P, B.slot, cam, w, h);
    const int y0 = B.row * kBlendTileH - kBlendHalo + kMbFirst;
    uint64_t *o = a.bdesc + (int64_t)blockIdx.x * kMbBandDescRows * kMbBandLanes;
    for (int i = threadIdx.x; i < kMbBandDescRows * kMbBandLanes; i += blockDim.x) {
        const int r = i / kMbBandLanes, l = i % kMbBandLanes;
        const int x = refl(B.c0 + l, P.out_w), y = refl(y0 + r, P.out_h);
        const uint2 v = mb_desc<CN>(mb_src<INTERP>(P, B.slot, x, y), w, h);
        o[i] = (uint64_t)v.x | ((uint64_t)v.y << 32);
    }
}

// Value of lane l + 1 / l - 1 of the wave (DPP wave_shl:1 / wave_shr:1; the end lanes get 0).
// (bound_ctrl: a lane without a source reads 0 -- the edge lanes' value -- so no `old` register
// has to be zeroed before every DPP move)
__device__ __forceinline__ uint32_t lane_next(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t lane_prev(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, true);
}
// Value of lane `src` (byte address src * 4: ds_bpermute).
__device__ __forceinline__ int lane_at(int v, int src4)
{
    return __builtin_amdgcn_ds_bpermute(src4, v);
}

// f(std::integral_constant<int, 0>()) .. f(std::integral_constant<int, N - 1>()), in order.
template <int I, int N, class F>
__device__ __forceinline__ void static_for_(F &&f)
{
    if constexpr (I < N) {
        f(std::integral_constant<int, I>());
        static_for_<I + 1, N>(f);
    }
}
template <int N, class F>
__device__ __forceinline__ void static_for(F &&f) { static_for_<0, N>(f); }

// CN consecutive ints (one wide store: 4-byte aligned).
template <int CN>
__device__ __forceinline__ void mb_store_ch(__attribute__((address_space(1))) uint8_t *p,
                                            const int (&v)[CN])
{
    typedef __attribute__((address_space(1))) int gi;
    typedef int i3 __attribute__((ext_vector_type(3), aligned(4)));
    typedef int i4 __attribute__((ext_vector_type(4), aligned(4)));
    if (CN == 3) {
        i3 t;
        t.x = v[0], t.y = v[CN > 1 ? 1 : 0], t.z = v[CN > 2 ? 2 : 0];
        *(__attribute__((address_space(1))) i3 *)p = t;
    } else if (CN == 4) {
        i4 t;
        t.x = v[0], t.y = v[CN > 1 ? 1 : 0], t.z = v[CN > 2 ? 2 : 0], t.w = v[CN > 3 ? 3 : 0];
        *(__attribute__((address_space(1))) i4 *)p = t;
    } else {
#pragma unroll
        for (int k = 0; k < CN; k++) ((gi *)p)[k] = v[k];
    }
}

// Scratch targets of one emitted entry: up to two listed tiles of the band's row whose arrays
// hold the column (base = (list index * slots + local slot) * chunk, col = column in the tile's
// array); base -1 = none.
struct MbTarget {
    int base[2], col[2];
};
static_assert(kBlendTileW == 32, "mb_bands: tile columns are found by shifts");

__device__ __forceinline__ void mb_target(const KMbBandArgs &a, int s, int row, int tx, int col,
                                          MbTarget &T, int k)
{
    T.base[k] = -1;
    T.col[k] = 0;
    if (tx < 0 || tx >= a.gxb) return;
    const int bt = a.tile_bt[row * a.gxb + tx];
    if (bt < 0) return;
    const uint32_t mask = (uint32_t)a.list[2 + 2 * bt];
    if (!((mask >> s) & 1u)) return;
    const int j = __popc(mask & ((1u << s) - 1u));
    T.base[k] = (bt * a.slots + j) * a.chunk;
    T.col[k] = col;
}

// One band, FR captures: grid (bands, ceil(nf / FR)), block 64 (one wave).  Per level-0 row: the
// lane's replicate-border sample (the owner's frame through L1/L2; descriptors three rows ahead,
// windows two rows ahead), unpacked to 16-bit lanes and accumulated into the vertical 5-tap sums
// of the level-1 rows it feeds (three rolling accumulators).  Per finished level-1 row: the
// horizontal 5-tap over the neighbour lanes (DPP), giving level 1 at the even lanes; its
// R1-region entries go to the scratch, and the row is accumulated per channel into the vertical
// sums of level 2.  Per finished level-2 row: the horizontal 5-tap over lanes 2 and 4 apart
// (ds_bpermute), level 2 at every fourth lane.  Only entries at real mosaic positions are stored
// (the blend reads no others).  Integer sums, exact: the values of mb_levels' LDS passes.
// Rows and columns of a unit past the top / left mosaic edge hold reflected level-0 samples, and
// the reduces computed there are the reflected entries (reflect-101 about 0 commutes with the
// 2x decimation).  At the bottom / right edges it does not (for even level sizes), so BR units
// give level 2 the reflected level-1 rows (a history of four) and columns (source lanes).
// XCD-grouped 1-D launch of nx * ny units (x: a band or blend tile, y: its captures): block b
// runs on XCD b % 8 (the dispatcher deals blocks round-robin), and XCD k takes the contiguous
// unit range [k * per, (k + 1) * per), x-major -- so all captures of one band / tile run on one
// XCD one after another, and the band's descriptors (101 KB, the same for every capture) or the
// tile's tables come from that XCD's L2 after the first wave instead of being fetched again by
// every capture (round 3: 0.58 GB of descriptor reads per C2 launch, every band's 32 waves spread
// over the whole launch and over the XCDs).  False past the launch's units.
__device__ __forceinline__ bool xcd_unit(int nx, int ny, int &x, int &y)
{
    const int n = nx * ny, per = (n + 7) >> 3;
    const int u = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (u >= n) return false;
    x = u / ny;
    y = u - x * ny;
    return true;
}

// CN consecutive ints by one buffer store (offset past the range: nothing written).
template <int CN>
__device__ __forceinline__ void mb_buffer_store_ch(__amdgpu_buffer_rsrc_t rs, uint32_t off,
                                                   const int (&v)[CN])
{
    typedef unsigned int u2v __attribute__((ext_vector_type(2)));
    typedef unsigned int u3v __attribute__((ext_vector_type(3)));
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    if constexpr (CN == 1) {
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v[0], rs, off, 0, 0);
    } else if constexpr (CN == 2) {
        const u2v t = {(uint32_t)v[0], (uint32_t)v[CN > 1 ? 1 : 0]};
        __builtin_amdgcn_raw_buffer_store_b64(t, rs, off, 0, 0);
    } else if constexpr (CN == 3) {
        const u3v t = {(uint32_t)v[0], (uint32_t)v[CN > 1 ? 1 : 0], (uint32_t)v[CN > 2 ? 2 : 0]};
        __builtin_amdgcn_raw_buffer_store_b96(t, rs, off, 0, 0);
    } else {
        const u4v t = {(uint32_t)v[0], (uint32_t)v[CN > 1 ? 1 : 0], (uint32_t)v[CN > 2 ? 2 : 0],
                       (uint32_t)v[CN > 3 ? 3 : 0]};
        __builtin_amdgcn_raw_buffer_store_b128(t, rs, off, 0, 0);
    }
}

// LDS band pass: vector memory operations issued at body row ph (after its LDS reads): the
// stores of the entries finished by the previous row (2 targets per capture: level 1 after odd
// rows, level 2 after rows 4j + 1), the group DMAs (rows 4j, one per capture), the descriptor DMA.
template <int FR>
constexpr int mb_lds_ops(int ph)
{
    return ((ph & 1) ? 2 * FR : 0) + (ph % 4 == 1 ? 2 * FR : 0) + (ph % 4 == 0 ? FR : 0) + 1;
}
// The vmcnt bound before row ph's LDS reads: no more operations outstanding than were issued after
// the latest one that row needs -- its descriptor (issued NL rows earlier, last in that row) and
// its source groups (issued >= kMbLdsGLead rows earlier, before that row's descriptor).  First
// body pass, ph < NL: the descriptor came in the prologue, followed by the prologue's later
// descriptors and this pass's rows (the groups those rows may read are all prologue groups).
template <int FR, int NL>
constexpr int mb_lds_wait(int ph, bool first)
{
    int d = 0, g = 1;
    for (int j = 1; j < NL; j++) d += mb_lds_ops<FR>((ph - j + 12) % 12);
    for (int j = 1; j < kMbLdsGLead; j++) g += mb_lds_ops<FR>((ph - j + 12) % 12);
    int w = d < g ? d : g;
    if (first) {
        int w0 = NL - 1 - ph;
        for (int j = 0; j < ph; j++) w0 += mb_lds_ops<FR>(j);
        w = w0 < w ? w0 : w;
    }
    return w > 63 ? 63 : w;
}

// Window modes (WM): 0 = unaligned 8-byte global loads; 1 (AL) = dword-aligned 12-byte global
// loads (mb_desc's sh), funnel-shifted in registers (the texture addresser splits unaligned
// loads: serial band pass 270 -> ~220 us, tools/experiments/gpu_r03_bandalign.sh); 2 = the
// band's source rows staged in an LDS ring by LDS-DMA, 4 rows per wave instruction (KMbBandArgs
// bgrp), the windows read from LDS (descriptor .x = the two windows' ring offsets): one 16-byte
// chunk per lane instead of four 12-byte gathers per lane and row.  Mode 2 needs a band whose
// source rows advance with its rows (mcs_capi.cpp band_lds_tables checks the ring schedule);
// the other bands of an aligned launch take mode 1.  In mode 2 the descriptors come by LDS-DMA
// too (16 B per lane and row: windows, meta, the offset of the group issued after that row), so
// the loop holds no ordinary global load: the compiler's own vmcnt waits for ordinary loads
// would otherwise drain the LDS-DMAs every row.
template <int CN, int FR, bool BR, int WM>
__device__ __forceinline__ void mb_bands_body(const KMbBandArgs &a, int bi, lds_u8 *ring, int pr)
{
    constexpr bool AL = WM >= 1, LD = WM == 2;
    typedef __attribute__((address_space(1))) const uint8_t gu8;
    struct __attribute__((packed)) U2 {
        uint32_t x, y;
    };
    struct U3 {
        uint32_t x, y, z;
    };
    typedef __attribute__((address_space(1))) const U2 gu2;
    typedef __attribute__((address_space(1))) const U3 gu3;
    typedef std::conditional_t<AL, uint3, uint2> Win;
    typedef __attribute__((address_space(1))) uint2 g2u;
    const KParams &P = a.P;
    const int l = threadIdx.x;
    const MbBand B = a.bands[bi];
    const int fl0 = pr * FR;
    if (fl0 >= a.nf) return;
    int cam, w, h;
    slot_info(P, B.slot, cam, w, h);
    const uint32_t pitch = (uint32_t)(w * CN);
    const gu8 *fb[FR];
#pragma unroll
    for (int i = 0; i < FR; i++)
        fb[i] = (const gu8 *)(P.cams[cam] +
                              (int64_t)(a.f0 + min(fl0 + i, a.nf - 1)) * P.cam_fstride[cam]);
    const int W = P.out_w, H = P.out_h;
    const int w1 = (W + 1) / 2, h1 = (H + 1) / 2, w2 = (w1 + 1) / 2, h2 = (h1 + 1) / 2;
    const int Y0 = B.row * kBlendTileH, Y1 = Y0 / 2 - kMbO1, Y2 = Y0 / 4 - kMbO2;
    const int x = B.c0 + l;
    // level-1 column x / 2 on even lanes 2..60, level-2 column x / 4 on lanes 8, 12, .., 56
    // (complete there), stored when inside the mosaic
    MbTarget T1, T2;
    T1.base[0] = T1.base[1] = T2.base[0] = T2.base[1] = -1;
    T1.col[0] = T1.col[1] = T2.col[0] = T2.col[1] = 0;
    if ((l & 1) == 0 && l >= 2 && l <= 61 && x >= 0 && (x >> 1) < w1) {
        // R1 region of tile tx: columns [16 tx - 1, 16 tx + 16]
        const int qx = x >> 1, tx = (qx + kMbOR) >> 4;
        mb_target(a, B.slot, B.row, tx, qx - (tx * (kBlendTileW / 2) - kMbOR), T1, 0);
        if (((qx + kMbOR) & 15) < kMbNRX - 16)
            mb_target(a, B.slot, B.row, tx - 1, qx - ((tx - 1) * (kBlendTileW / 2) - kMbOR), T1, 1);
    }
    if ((l & 3) == 0 && l >= 8 && l <= 56 && x >= 0 && (x >> 2) < w2) {
        // level-2 array of tile tx: columns [8 tx - 2, 8 tx + 9]
        const int z = x >> 2, tx = (z + kMbO2) >> 3;
        mb_target(a, B.slot, B.row, tx, z - (tx * (kBlendTileW / 4) - kMbO2), T2, 0);
        if (((z + kMbO2) & 7) < kMbN2X - 8)
            mb_target(a, B.slot, B.row, tx - 1, z - ((tx - 1) * (kBlendTileW / 4) - kMbO2), T2, 1);
    }
    // level-2 horizontal sources: level-1 columns qx - 2 .. qx + 2 (lanes 2 apart), reflected
    // at the right mosaic edge (BR)
    int src[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        int q = (x >> 1) + (t < 2 ? t - 2 : t - 1);
        if (BR && q >= w1) q = 2 * w1 - 2 - q;
        src[t] = min(max(2 * q - B.c0, 0), kMbBandLanes - 1) * 4;
    }
    // scratch byte offsets (32-bit: the scratch is < 4 GiB) of this lane's targets, capture fl0,
    // array row 0
    uint32_t o1[2], o2[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
        o1[k] = T1.base[k] < 0 ? 0u : (uint32_t)((T1.base[k] + fl0) * (kMbNRX * kMbNRY) +
                                                 mb_g1_at(T1.col[k], 0)) * 8u;
        o2[k] = T2.base[k] < 0 ? 0u : (uint32_t)((T2.base[k] + fl0) * (kMbN2X * kMbN2Y * CN) +
                                                 mb_g2_at<CN>(T2.col[k], 0, 0)) * 4u;
    }
    typedef __attribute__((address_space(1))) uint8_t g8;
    g8 *const g1b = (g8 *)a.g1, *const g2b = (g8 *)a.g2;
    const uint64_t *dsc = a.bdesc + (int64_t)bi * kMbBandDescRows * kMbBandLanes + l;
    const int nst = min(FR, a.nf - fl0);
    // Rolling vertical sums, indexed by row % 3 (compile-time inside the 12-row body): level-1
    // rows (packed u16: lo = channels 0, 2; hi = 1, 3), level-2 rows (one int per channel).  A
    // row's sum starts with '=' at its first input row, so the rows before the array (and the
    // padding rows after it) only ever feed rows that are not stored.
    uint32_t Vl[FR][3], Vh[FR][3];
    int V2[FR][3][CN];
    uint32_t hl[FR][BR ? 4 : 1], hh[FR][BR ? 4 : 1];   // BR: the last four level-1 rows
#pragma unroll
    for (int i = 0; i < FR; i++)
#pragma unroll
        for (int q = 0; q < 3; q++) {
            Vl[i][q] = Vh[i][q] = 0u;
#pragma unroll
            for (int k = 0; k < CN; k++) V2[i][q][k] = 0;
            if (q < (BR ? 4 : 1)) hl[i][q] = hh[i][q] = 0u;
        }
    if (BR) {
#pragma unroll
        for (int i = 0; i < FR; i++) hl[i][BR ? 3 : 0] = hh[i][BR ? 3 : 0] = 0u;
    }
    auto load_win = [&](uint64_t dv, Win (&r0)[FR], Win (&r1)[FR]) {
        if constexpr (LD) return;
        const uint32_t dx = (uint32_t)dv;
        const uint32_t d = AL ? (uint32_t)(dv >> 47) & 15u : (uint32_t)(dv >> 44) & 7u;
        uint32_t o = (dx & 0x7fffffffu) - d, ob = o + ((dx >> 31) ? pitch : 0u);
#pragma unroll
        for (int i = 0; i < FR; i++) {
            if constexpr (AL) {
                const U3 ra = *(const gu3 *)(fb[i] + o), rb = *(const gu3 *)(fb[i] + ob);
                r0[i] = make_uint3(ra.x, ra.y, ra.z);
                r1[i] = make_uint3(rb.x, rb.y, rb.z);
            } else {
                const U2 ra = *(const gu2 *)(fb[i] + o), rb = *(const gu2 *)(fb[i] + ob);
                r0[i] = make_uint2(ra.x, ra.y);
                r1[i] = make_uint2(rb.x, rb.y);
            }
        }
    };
    // Finished entries wait one row in registers before they are stored: gfx9 counts stores
    // in vmcnt, so the wait for a row's window loads also waits for every store issued after
    // those loads -- a store issued early in the next row has that row's work to complete.
    int pend1 = -1, pend2 = -1;   // array row of the pending level-1 / level-2 entries (-1: none)
    uint32_t p1l[FR], p1h[FR];
    int p2[FR][CN];
    // LDS mode: the entries of every level-1 / level-2 row are stored, at fixed rows of the body
    // (level 1 after odd rows, level 2 after rows 4j + 1), as buffer stores whose lanes without a
    // target (or rows outside the arrays: ok1 / ok2 false) carry an out-of-range offset and write
    // nothing -- so every row issues a fixed number of vector memory operations and the waits
    // before its LDS reads can count them (mb_lds_wait)
    bool ok1 = false, ok2 = false;
    const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void *)a.g1, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs2 = __builtin_amdgcn_make_buffer_rsrc((void *)a.g2, 0, 0x7fffffff, 0x00020000);
    auto flush_ld = [&](auto PHc) {
        constexpr int ph = decltype(PHc)::value;
        constexpr uint32_t none = 0xfffffff0u;
        if constexpr (ph & 1) {
#pragma unroll
            for (int f = 0; f < FR; f++) {
                const uint32_t ro =
                    (uint32_t)(f * (kMbNRX * kMbNRY) + mb_g1_at(0, pend1 - kMbRS)) * 8u;
                typedef unsigned int u2v __attribute__((ext_vector_type(2)));
                const u2v v = {p1l[f], p1h[f]};
#pragma unroll
                for (int k = 0; k < 2; k++)
                    __builtin_amdgcn_raw_buffer_store_b64(
                        v, rs1, (ok1 && f < nst && T1.base[k] >= 0) ? o1[k] + ro : none, 0, 0);
            }
        }
        if constexpr (ph % 4 == 1) {
#pragma unroll
            for (int f = 0; f < FR; f++) {
                const uint32_t ro =
                    (uint32_t)(f * (kMbN2X * kMbN2Y * CN) + mb_g2_at<CN>(0, pend2, 0)) * 4u;
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    const uint32_t off = (ok2 && f < nst && T2.base[q] >= 0) ? o2[q] + ro : none;
                    mb_buffer_store_ch<CN>(rs2, off, p2[f]);
                }
            }
        }
    };
    auto flush = [&]() {
        if (pend1 >= 0) {
#pragma unroll
            for (int f = 0; f < FR; f++) {
                if (f >= nst) break;
                const uint32_t ro =
                    (uint32_t)(f * (kMbNRX * kMbNRY) + mb_g1_at(0, pend1 - kMbRS)) * 8u;
#pragma unroll
                for (int k = 0; k < 2; k++)
                    if (T1.base[k] >= 0) *(g2u *)(g1b + (o1[k] + ro)) = make_uint2(p1l[f], p1h[f]);
            }
            pend1 = -1;
        }
        if (pend2 >= 0) {
#pragma unroll
            for (int f = 0; f < FR; f++) {
                if (f >= nst) break;
                const uint32_t ro =
                    (uint32_t)(f * (kMbN2X * kMbN2Y * CN) + mb_g2_at<CN>(0, pend2, 0)) * 4u;
#pragma unroll
                for (int q = 0; q < 2; q++)
                    if (T2.base[q] >= 0) mb_store_ch<CN>(g2b + (o2[q] + ro), p2[f]);
            }
            pend2 = -1;
        }
    };
    // finished level-1 vertical sums (vl, vh) of array row i = 2m + P2 (m % 3 = M3), capture f
    auto level1_done = [&](int i, auto P2c, auto M3c, int f, uint32_t vl, uint32_t vh) {
        constexpr int P2 = decltype(P2c)::value, M3 = decltype(M3c)::value;
        // horizontal: level-1 entry at lane x = 2 qx reads lanes x - 2 .. x + 2
        const uint32_t l1 = lane_prev(vl), l2 = lane_prev(l1), r1 = lane_next(vl),
                       r2 = lane_next(r1);
        const uint32_t h1_ = lane_prev(vh), h2_ = lane_prev(h1_), s1 = lane_next(vh),
                       s2 = lane_next(s1);
        uint32_t gl = mad6_u32(vl, (l2 + r2) + 4u * (l1 + r1));
        uint32_t gh = mad6_u32(vh, (h2_ + s2) + 4u * (h1_ + s1));
        const int qy = Y1 + i;
        if constexpr (LD) {
            pend1 = i;
            ok1 = qy >= 0 && qy < h1 && i >= kMbRS && i < kMbRS + kMbNRY;
            p1l[f] = gl;
            p1h[f] = gh;
        } else if (qy >= 0 && qy < h1 && i >= kMbRS && i < kMbRS + kMbNRY) {
            pend1 = i;   // (stored at the next row, see flush)
            p1l[f] = gl;
            p1h[f] = gh;
        }
        if (BR) {
            // rows past the bottom edge feed level 2 as their reflections: h1 -> h1 - 2 (two
            // rows back), h1 + 1 -> h1 - 3 (four back); deeper rows feed no stored entry
            if (qy >= h1) {
                const bool d0 = qy == h1;
                gl = d0 ? hl[f][1] : hl[f][BR ? 3 : 0];
                gh = d0 ? hh[f][1] : hh[f][BR ? 3 : 0];
            }
#pragma unroll
            for (int q = (BR ? 3 : 0); q > 0; q--) hl[f][q] = hl[f][q - 1], hh[f][q] = hh[f][q - 1];
            hl[f][0] = gl, hh[f][0] = gh;
        }
        int g[CN];
#pragma unroll
        for (int k = 0; k < CN; k++)
            g[k] = (int)((((k & 1) ? gh : gl) >> ((k & 2) ? 16 : 0)) & 0xffffu);
        // vertical: level-2 array row e reads level-1 rows 2e .. 2e + 4
        if (P2 == 0) {
#pragma unroll
            for (int k = 0; k < CN; k++) V2[f][(M3 + 1) % 3][k] += g[k];   // row m - 2 done
            const int e = (i >> 1) - 2, zy = Y2 + e;
            if (LD) {
                pend2 = e;
                ok2 = e >= 0 && e < kMbN2Y && zy < h2;
            }
            if (LD || (e >= 0 && e < kMbN2Y && zy < h2)) {
                pend2 = e;
#pragma unroll
                for (int k = 0; k < CN; k++) {
                    const int v = V2[f][(M3 + 1) % 3][k];
                    p2[f][k] = (lane_at(v, src[0]) + lane_at(v, src[3])) +
                               4 * (lane_at(v, src[1]) + lane_at(v, src[2])) + 6 * v;
                }
            }
#pragma unroll
            for (int k = 0; k < CN; k++) {
                V2[f][(M3 + 2) % 3][k] += 6 * g[k];
                V2[f][M3][k] = g[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < CN; k++) {
                V2[f][(M3 + 2) % 3][k] += 4 * g[k];
                V2[f][M3][k] += 4 * g[k];
            }
        }
    };
    // Pipeline over rows: at row r the windows of rows r + 1 .. r + A and the descriptor of row
    // r + A + 1 are in flight (A = kMbBandAhead), A + 1 buffers each indexed by row % (A + 1).
    // The 12-row body makes every buffer and accumulator index a compile-time constant, so no
    // register copy ever reads an in-flight load (such a copy makes the compiler drain all loads
    // at the loop's back edge).
    constexpr int NB = kMbBandBufs, A = kMbBandAhead, ND = kMbBandDescRing;
    uint64_t dq[ND];
    Win wq0[NB][FR], wq1[NB][FR];
    // LDS mode: group g = the band's source rows 4g .. 4g + 3 (from its first) into ring rows
    // (4g .. 4g + 3) mod kMbLdsRows of every capture's ring, one LDS-DMA instruction per capture
    // (lane = 16-byte chunk, byte offsets in the frame from bgrp); groups 0 .. kMbLdsLead / 4 before
    // the loop, group r / 4 + kMbLdsLead / 4 + 1 after row r (r % 4 == 0); descriptor row r + NL
    // after row r.  No ordinary global load in the loop: `s_waitcnt vmcnt(mb_lds_wait)` before a
    // row's LDS reads counts the fixed operations issued after everything that row reads.
    const uint32_t *grp = a.bgrp + (int64_t)bi * kMbLdsGroups * kMbBandLanes + l;
    typedef __attribute__((address_space(3))) const uint32_t lu32;
    lds_u8 *const dring = ring + kMbLdsDescOff;
    constexpr int NL = kMbLdsDescRing;
    const uint4 *d16 = a.bdesc16 + (int64_t)bi * kMbLdsDescRows * kMbBandLanes + l;
    auto issue_desc = [&](int row) {   // descriptor row `row` into ring slot row % NL
        __builtin_amdgcn_global_load_lds(d16 + row * kMbBandLanes,
                                         dring + (row % NL) * kMbBandLanes * 16, 16, 0, 0);
        asm volatile("" ::: "memory");
    };
    // (one buffer resource per capture frame: the chunks a row's samples do not read carry an
    // out-of-range offset and fetch nothing, while the instruction count stays fixed)
    __amdgpu_buffer_rsrc_t rsf[FR];
#pragma unroll
    for (int f = 0; f < FR; f++)
        rsf[f] = __builtin_amdgcn_make_buffer_rsrc((void *)fb[f], 0, (int)(pitch * (uint32_t)h),
                                                   0x00020000);
    auto issue_group = [&](int g, uint32_t off) {
#pragma unroll
        for (int f = 0; f < FR; f++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rsf[f], ring + f * kMbLdsRingBytes + ((4 * g) % kMbLdsRows) * kMbLdsSpan, 16, off, 0,
                0, 0);
        asm volatile("" ::: "memory");   // (the next row's descriptor load stays after the DMAs)
    };
    if constexpr (LD) {
        uint32_t go[kMbLdsLead / 4 + 1];
#pragma unroll
        for (int g = 0; g <= kMbLdsLead / 4; g++) go[g] = grp[g * kMbBandLanes];
#pragma unroll
        for (int g = 0; g <= kMbLdsLead / 4; g++) issue_group(g, go[g]);
#pragma unroll
        for (int i = 0; i < NL; i++) issue_desc(i);
    } else {
#pragma unroll
        for (int i = 0; i < ND; i++) dq[i] = dsc[i * kMbBandLanes];
    }
#pragma unroll
    for (int i = 0; i < A; i++) load_win(dq[i], wq0[i], wq1[i]);
    for (int r12 = 0; r12 < kMbBandRows; r12 += 12) {
        static_for<12>([&](auto PHc) {
            constexpr int ph = decltype(PHc)::value;
            const int r = r12 + ph;
            constexpr int b0 = ph % NB, bA = (ph + A) % NB, d0 = ph % ND, dA = (ph + A) % ND;
            uint32_t wa, wb, meta, dxr;
            if constexpr (LD) {
                if (ph < NL && r12 == 0)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(mb_lds_wait<FR, NL>(ph, true)) : "memory");
                else
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(mb_lds_wait<FR, NL>(ph, false)) : "memory");
                // (ring descriptor: windows + shift, and the doubled weights precomputed on the
                // host, band_lds_tables)
                const lu32 *dd = (const lu32 *)(dring + (ph % NL) * kMbBandLanes * 16 + l * 16);
                dxr = dd[0];
                wa = dd[1];
                wb = dd[3];
                meta = 0u;
            } else {
                dxr = (uint32_t)dq[d0];
                meta = (uint32_t)(dq[d0] >> 32);
                mb_weights2(meta, wa, wb);
            }
            const uint32_t dd = AL ? 0u : (meta >> 12) & 7u;
            // per capture the sample's channels as packed u16 pairs: pl = (ch 0, ch 2), ph = (ch
            // 1, ch 3), each channel from byte 2 of its mb_tap2 sum
            uint32_t pls[FR], phs[FR];
#pragma unroll
            for (int f = 0; f < FR; f++) {
                uint2 r0, r1;
                if constexpr (LD) {
                    const uint32_t dx = dxr, sh = (dx >> 14) & 3u;
                    const lu32 *pa = (const lu32 *)(ring + f * kMbLdsRingBytes + (dx & 0x3fffu));
                    const lu32 *pb = (const lu32 *)(ring + f * kMbLdsRingBytes + (dx >> 16));
                    r0 = mb_win_shift4(make_uint3(pa[0], pa[1], pa[2]), sh);
                    r1 = mb_win_shift4(make_uint3(pb[0], pb[1], pb[2]), sh);
                } else if constexpr (AL) {
                    const uint32_t sh = (meta >> 15) & 15u;
                    r0 = mb_win_shift<CN>(wq0[b0][f], sh);
                    r1 = mb_win_shift<CN>(wq1[b0][f], sh);
                } else {
                    r0 = wq0[b0][f];
                    r1 = wq1[b0][f];
                }
                uint32_t t[4];
#pragma unroll
                for (int c = 0; c < 4; c++) t[c] = c < CN ? mb_tap2<CN>(r0, r1, wa, wb, c, dd) : 0u;
                if constexpr (CN >= 3) pls[f] = __builtin_amdgcn_perm(t[2], t[0], 0x0c060c02u);
                else pls[f] = (t[0] >> 16) & 0xffu;
                if constexpr (CN >= 4) phs[f] = __builtin_amdgcn_perm(t[3], t[1], 0x0c060c02u);
                else if constexpr (CN == 2 || CN == 3) phs[f] = (t[1] >> 16) & 0xffu;
                else phs[f] = 0u;
            }
            // the previous row's finished entries (after this row's window wait), then the loads:
            // windows of row r + A (its descriptor arrived a row ago), descriptor of row r + A + 1
            if constexpr (LD) flush_ld(PHc);
            else flush();
            load_win(dq[dA], wq0[bA], wq1[bA]);
            if constexpr (LD) {
                // this row's descriptor slot is refilled below (issue_desc(r + NL)): its LDS reads
                // must have completed -- in the schedule and in hardware -- before that DMA is
                // issued (without this the compiler sank the weight reads past it: a race)
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if constexpr (ph % 4 == 0) {
                    const lu32 *dd = (const lu32 *)(dring + (ph % NL) * kMbBandLanes * 16 + l * 16);
                    issue_group(r / 4 + kMbLdsLead / 4 + 1, dd[2]);
                }
                issue_desc(r + NL);
            } else {
                dq[d0] = dsc[(r + ND) * kMbBandLanes];
            }
            // level-0 row r = 2k + (ph & 1), k % 3 = K3; level-1 row k - 2 = 2m + P2, m % 3 = M3
            constexpr int K3 = (ph / 2) % 3;
            constexpr int q = ph / 2 - 2, P2 = q & 1, M3 = ((q - P2) / 2 + 3) % 3;
            const int k = r >> 1;
#pragma unroll
            for (int f = 0; f < FR; f++) {
                const uint32_t pl = pls[f], ph_ = phs[f];
                // vertical: level-1 array row i reads level-0 rows 2i .. 2i + 4
                if ((ph & 1) == 0) {
                    Vl[f][(K3 + 1) % 3] += pl;   // row k - 2 done
                    Vh[f][(K3 + 1) % 3] += ph_;
                    level1_done(k - 2, std::integral_constant<int, P2>(),
                                std::integral_constant<int, M3>(), f, Vl[f][(K3 + 1) % 3],
                                Vh[f][(K3 + 1) % 3]);
                    // (pl, ph_ <= 0x00ff00ff < 2^24: a full-rate 24-bit multiply)
                    Vl[f][(K3 + 2) % 3] += __umul24(pl, 6u);
                    Vh[f][(K3 + 2) % 3] += __umul24(ph_, 6u);
                    Vl[f][K3] = pl;
                    Vh[f][K3] = ph_;
                } else {
                    Vl[f][(K3 + 2) % 3] += 4u * pl;
                    Vh[f][(K3 + 2) % 3] += 4u * ph_;
                    Vl[f][K3] += 4u * pl;
                    Vh[f][K3] += 4u * ph_;
                }
            }
        });
    }
    if constexpr (!LD) flush();   // (LD: the last row stored everything pending)
}

// The band pass of band bi: the aligned launch (AL) runs bands flagged for the LDS ring (MbBand
// pad_ bit 0, band_lds_tables) in mode 2, the others in mode 1.
template <int CN, int FR, bool BR, bool AL>
__device__ __forceinline__ void mb_bands(const KMbBandArgs &a, int bi, lds_u8 *ring, int pr)
{
    if constexpr (AL) {
        const int lds = __builtin_amdgcn_readfirstlane(a.bands[bi].pad_) & 1;
        if (lds) mb_bands_body<CN, FR, BR, 2>(a, bi, ring, pr);
        else mb_bands_body<CN, FR, BR, 1>(a, bi, ring, pr);
    } else {
        mb_bands_body<CN, FR, BR, 0>(a, bi, ring, pr);
    }
}

// ---- blend: grid (listed tiles, nf), block kMbBlThreads ------------------------------------------
template <int CN, int S>
struct MbBlLds {
    uint2 g1[S][kMbNRX * kMbNRY];      // packed as in mb_levels
    int32_t g2[S][CN][kMbN2X * kMbN2Y];   // channel-planar: indices need no * CN
    double b2[CN][kMbN2X * kMbN2Y];
    double r1[CN][kMbNRX * kMbNRY];
};

constexpr int kMbPQ = kMbTilePx / kMbBlThreads;   // tile pixels per thread
template <int CN>
struct MbPix {
    int i[kMbPQ];            // the thread's mixed pixels (tile index, -1: none)
    int own[kMbPQ];          // owner slot of each of the thread's pixels (kBlendNone: none)
    uint32_t v[kMbPQ];       // its owner sample (the stitch kernel's output), channel k in byte k
};

template <int CN, int S, bool IN>
__device__ __forceinline__ void mb_blend_tile(const KMbArgs &a, const MbGeo &G, MbBlLds<CN, S> &L,
                                              const MbPix<CN> &px, uint32_t mask, int ns, int f,
                                              int bt)
{
    const KParams &P = a.P;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int32_t *tab = a.tab + (int64_t)bt * mb_tab_words(a.slots);
    const int32_t *t_m1 = tab, *t_m2 = tab + a.slots * kMbNRX * kMbNRY;
    const int32_t *t_d1 = t_m2 + a.slots * kMbN2X * kMbN2Y, *t_d2 = t_d1 + kMbNRX * kMbNRY;
    // (24-bit multiplies: full-rate v_mul_u32_u24 instead of quarter-rate v_mul_lo_u32)
    auto i2 = [&](int cx, int cy) {
        return (int)__umul24((unsigned)ix2<IN>(cy, G.Y2, kMbN2Y), kMbN2X) + ix2<IN>(cx, G.X2, kMbN2X);
    };
    auto ir = [&](int cx, int cy) {   // the R1 region (g1, m1, d1, r1)
        return (int)__umul24((unsigned)ix2<IN>(cy, G.YR, kMbNRY), kMbNRX) + ix2<IN>(cx, G.XR, kMbNRX);
    };
    const int n_r1 = t_d2[kMbN2X * kMbN2Y + 1];
    const uint16_t *t_r1 =
        reinterpret_cast<const uint16_t *>(t_d2 + kMbN2X * kMbN2Y + kMbTabCounts) + kMbTilePx;
    // B2 = sum m2 g2 / (sum m2 * 65536)
    for (int e = tid; e < kMbN2X * kMbN2Y; e += nt) {
        // (integer sums in double: every product < 2^41, every sum < 2^43 -- exact)
        double num[CN];
#pragma unroll
        for (int k = 0; k < CN; k++) num[k] = 0.0;
        for (int j = 0; j < ns; j++) {
            const double m = (double)t_m2[__umul24((unsigned)j, kMbN2X * kMbN2Y) + e];
#pragma unroll
            for (int k = 0; k < CN; k++) num[k] += m * (double)L.g2[j][k][e];
        }
        const int den = t_d2[e];
#pragma unroll
        for (int k = 0; k < CN; k++)
            L.b2[k][e] = den ? num[k] / ((double)den * 65536.0) : 0.0;
    }
    __syncthreads();
    // R1 = B1 + up(B2), B1 = sum m1 (16384 g1 - E(g2)) / (sum m1 * 4194304)
    // (the list is grouped by parity class, mb_prep: the zero-weight third taps of odd
    // coordinates are skipped by whole waves)
    for (int l = tid; l < n_r1; l += nt) {
        const int e = t_r1[l];
        const int ey = div_small<kMbNRX>(e), ex = e - (int)__umul24((unsigned)ey, kMbNRX);
        const int qx = rf<IN>(G.XR + ex, G.w1), qy = rf<IN>(G.YR + ey, G.h1);
        int iy[3], wy[3], ix[3], wx[3];
        exp_taps<IN>(qy, G.h2, iy, wy);
        exp_taps<IN>(qx, G.w2, ix, wx);
        const bool y3 = wy[2] != 0, x3 = wx[2] != 0;
        int tp[9], tw[9];
#pragma unroll
        for (int u = 0; u < 3; u++)
#pragma unroll
            for (int v = 0; v < 3; v++) {
                tp[3 * u + v] = i2(ix[v], iy[u]);
                tw[3 * u + v] = wy[u] * wx[v];
            }
        const int p1 = ir(qx, qy);
        // (integer sums in double: every product < 2^39, every sum < 2^41 -- exact)
        double num[CN];
#pragma unroll
        for (int k = 0; k < CN; k++) num[k] = 0.0;
        for (int j = 0; j < ns; j++) {
            int e2[CN];   // <= 64 * 65536 * 255 < 2^31: exact in int32
#pragma unroll
            for (int k = 0; k < CN; k++) e2[k] = 0;
#pragma unroll
            for (int t = 0; t < 9; t++) {
                if ((t >= 6 && !y3) || (t % 3 == 2 && !x3)) continue;   // zero-weight taps
#pragma unroll
                for (int k = 0; k < CN; k++)   // (tw <= 36, g2 < 2^24: a 24-bit multiply)
                    e2[k] += (int)__umul24((unsigned)tw[t], (unsigned)L.g2[j][k][tp[t]]);
            }
            const uint2 g1 = L.g1[j][p1];
            const double m = (double)t_m1[__umul24((unsigned)j, kMbNRX * kMbNRY) + p1];
#pragma unroll
            for (int k = 0; k < CN; k++) num[k] += m * (double)(16384 * ch16(g1, k) - e2[k]);
        }
        const int den = t_d1[p1];
        double acc[CN];
#pragma unroll
        for (int k = 0; k < CN; k++) acc[k] = 0.0;
#pragma unroll
        for (int t = 0; t < 9; t++) {
            if ((t >= 6 && !y3) || (t % 3 == 2 && !x3)) continue;   // (adds of an exact 0)
            const double wt = (double)tw[t];
#pragma unroll
            for (int k = 0; k < CN; k++) acc[k] += wt * L.b2[k][tp[t]];
        }
#pragma unroll
        for (int k = 0; k < CN; k++) {
            const double b1 = den ? num[k] / ((double)den * 4194304.0) : 0.0;
            L.r1[k][e] = b1 + acc[k] / 64.0;
        }
    }
    __syncthreads();
    // R0 = L0_owner / 16384 + up(R1) over the tile's own pixels; L0 = 16384 g0 - E(g1), g0 = the
    // owner sample already in the mosaic
#pragma unroll
    for (int q = 0; q < kMbPQ; q++) {
        const int i = px.i[q];
        if (i < 0) continue;
        const int x = G.X0 + (i % kBlendTileW), y = G.Y0 + i / kBlendTileW;
        // (global address space: the stores cannot alias the LDS arrays read by later pixels)
        typedef __attribute__((address_space(1))) uint8_t gu8;
        gu8 *po = (gu8 *)(P.out + (int64_t)f * P.out_fstride + (int64_t)y * P.out_pitch + x * CN);
        const int o = px.own[q];
        if (o == kBlendNone) {
#pragma unroll
            for (int k = 0; k < CN; k++) po[k] = 0;
            continue;
        }
        const int s = __popc(mask & ((1u << o) - 1u));
        int iy[3], wy[3], ix[3], wx[3];
        exp_taps<IN>(y, G.h1, iy, wy);
        exp_taps<IN>(x, G.w1, ix, wx);
        int e1[CN];   // <= 64 * 256 * 255: exact in int32
        double acc[CN];
#pragma unroll
        for (int k = 0; k < CN; k++) e1[k] = 0, acc[k] = 0.0;
        // the taps in the restatement's order (rows outer); an odd coordinate's third tap has
        // weight 0 and is skipped (it would add an exact 0) -- the list is grouped by parity
        // class (mb_prep), so a wave skips it together
#pragma unroll
        for (int u = 0; u < 3; u++) {
            if (u == 2 && wy[2] == 0) break;
#pragma unroll
            for (int v = 0; v < 3; v++) {
                if (v == 2 && wx[2] == 0) break;
                const int p = ir(ix[v], iy[u]), wt = wy[u] * wx[v];
                const uint2 g1 = L.g1[s][p];
                const double wd = (double)wt;
#pragma unroll
                for (int k = 0; k < CN; k++) {
                    e1[k] += wt * ch16(g1, k);
                    acc[k] += wd * L.r1[k][p];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < CN; k++) {
            const int l0 = 16384 * (int)((px.v[q] >> (8 * k)) & 0xffu) - e1[k];
            const double r0 = (double)l0 / 16384.0 + acc[k] / 64.0;
            const double vf = floor(r0 + 0.5);
            po[k] = (uint8_t)(vf < 0.0 ? 0.0 : (vf > 255.0 ? 255.0 : vf));
        }
    }
}

template <int CN, int S>
__device__ __forceinline__ void mb_blend(const KMbArgs &a, MbBlLds<CN, S> &L)
{
    typedef __attribute__((address_space(1))) const uint8_t cgu8;
    typedef __attribute__((address_space(1))) const uint2 cgu2;
    typedef __attribute__((address_space(1))) const int32_t cgi32;
    const KParams &P = a.P;
    // (tile, capture) units dealt XCD-grouped: a tile's captures share its tables in one L2
    int ux, fl;
    if (!xcd_unit(a.n_list, a.nf, ux, fl)) return;   // (block-uniform, before any barrier)
    const int bt = a.list0 + ux, tid = threadIdx.x;
    const uint32_t mask = (uint32_t)a.list[2 + 2 * bt];
    const int ns = __popc(mask), f = a.f0 + fl;
    const MbGeo G = mb_geo(P, a.list[1 + 2 * bt]);
    // every global read of the block issued up front (one memory round trip): the tile pixels'
    // owners and owner samples, and the owners' level scratch
    MbPix<CN> px;
    int n_px;
    {
        const cgi32 *tc = (const cgi32 *)a.tab + (int64_t)bt * mb_tab_words(a.slots) +
                          a.slots * (kMbNRX * kMbNRY + kMbN2X * kMbN2Y) + kMbNRX * kMbNRY +
                          kMbN2X * kMbN2Y;
        typedef __attribute__((address_space(1))) const uint16_t cgu16;
        n_px = tc[0];
        const cgu16 *lp = (const cgu16 *)(tc + kMbTabCounts);
#pragma unroll
        for (int q = 0; q < kMbPQ; q++) {
            const int l = tid + q * kMbBlThreads;
            px.i[q] = l < n_px ? (int)lp[l] : -1;
        }
    }
    if (n_px == 0) return;   // uniform: no mixed pixel in this tile (before any barrier)
#pragma unroll
    for (int q = 0; q < kMbPQ; q++) {
        const int i = px.i[q];
        const int x = G.X0 + (i % kBlendTileW), y = G.Y0 + i / kBlendTileW;
        px.own[q] = kBlendNone;
        px.v[q] = 0;
        if (i >= 0) {
            px.own[q] = ((cgu8 *)a.owner)[(int64_t)y * G.W + x];
            const cgu8 *po = (const cgu8 *)(P.out + (int64_t)f * P.out_fstride +
                                            (int64_t)y * P.out_pitch + x * CN);
#pragma unroll
            for (int k = 0; k < CN; k++) px.v[q] |= (uint32_t)po[k] << (8 * k);
        }
    }
    constexpr int N1 = (kMbNRX * kMbNRY + kMbBlThreads - 1) / kMbBlThreads;
    constexpr int N2 = (kMbN2X * kMbN2Y * CN + kMbBlThreads - 1) / kMbBlThreads;
    uint2 r1[S][N1];
    int32_t r2[S][N2];
#pragma unroll
    for (int j = 0; j < S; j++) {
        if (j >= ns) break;
        const int64_t job = ((int64_t)bt * a.slots + j) * a.chunk + fl;
        const cgu2 *s1 = (const cgu2 *)a.g1 + job * (kMbNRX * kMbNRY);
        const cgi32 *s2 = (const cgi32 *)a.g2 + job * (kMbN2X * kMbN2Y * CN);
#pragma unroll
        for (int q = 0; q < N1; q++)
            r1[j][q] = s1[min(tid + q * kMbBlThreads, kMbNRX * kMbNRY - 1)];
#pragma unroll
        for (int q = 0; q < N2; q++)
            r2[j][q] = s2[min(tid + q * kMbBlThreads, kMbN2X * kMbN2Y * CN - 1)];
    }
    // (the scratch holds an entry's channels together, mb_g2_at; LDS is channel-planar)
#pragma unroll
    for (int j = 0; j < S; j++) {
        if (j >= ns) break;
#pragma unroll
        for (int q = 0; q < N1; q++)
            if (tid + q * kMbBlThreads < kMbNRX * kMbNRY) L.g1[j][tid + q * kMbBlThreads] = r1[j][q];
#pragma unroll
        for (int q = 0; q < N2; q++) {
            const int e = tid + q * kMbBlThreads;
            if (e < kMbN2X * kMbN2Y * CN) L.g2[j][e % CN][e / CN] = r2[j][q];
        }
    }
    __syncthreads();
    if (G.interior) mb_blend_tile<CN, S, true>(a, G, L, px, mask, ns, f, bt);
    else mb_blend_tile<CN, S, false>(a, G, L, px, mask, ns, f, bt);
}

}  // namespace mcs
