// mcs_blend.h -- device code of the blended stitch modes,
// included by mcs_kernels.hip (one code object).  The arithmetic is specified, and restated on
// the CPU, in oracle/orc_blend.c; this file reproduces it bit for bit (integers and IEEE
// doubles in the same order, no contraction).
//
// Layout: the stitch kernels first write every pixel from its "owner" camera (the covering
// camera farthest from its own image edge); then only the tiles where blending changes pixels
// are recomputed here, 32 x 32 output pixels per block:
//   feather   -- tiles with a pixel covered by two cameras at positive edge distance;
//   multiband -- tiles whose 64 x 64 neighbourhood (the 3-level pyramid's reach, 16 px halo)
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
    const int X0 = blockIdx.x * kBlendTile, Y0 = blockIdx.y * kBlendTile;
    uint32_t own = 0, fea = 0;
    for (int i = threadIdx.x; i < kBlendTile * kBlendTile; i += blockDim.x) {
        const int x = X0 + (i % kBlendTile), y = Y0 + i / kBlendTile;
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
// recomputes; list[0] = count.  multiband: the owners in the tile's 64 x 64 neighbourhood
// (clipped to the mosaic: reflected positions land inside it), when there are two or more;
// more than kBlendSlots owners in one neighbourhood is counted in overflow[0] (prepare fails);
// overflow[1] = the most owners any listed tile has.
__device__ __forceinline__ void blend_classify(const KParams &P, int mode, const uint8_t *owner,
                                               const uint32_t *info, int *list, int *overflow)
{
    __shared__ uint32_t s_mask;
    const int gx = (P.out_w + kBlendTile - 1) / kBlendTile;
    const int t = blockIdx.x, tx = t % gx, ty = t / gx;
    uint32_t mask;
    if (mode == MCS_BLEND_FEATHER) {
        mask = info[2 * t + 1];
    } else {
        if (threadIdx.x == 0) s_mask = 0;
        __syncthreads();
        const int x0 = max(tx * kBlendTile - kBlendHalo, 0);
        const int x1 = min(tx * kBlendTile + kBlendTile + kBlendHalo, P.out_w);
        const int y0 = max(ty * kBlendTile - kBlendHalo, 0);
        const int y1 = min(ty * kBlendTile + kBlendTile + kBlendHalo, P.out_h);
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
    if (threadIdx.x == 0 && mask) {
        if (mode == MCS_BLEND_MULTIBAND && __popc(mask) > kBlendSlots) atomicAdd(overflow, 1);
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
    const int gx = (P.out_w + kBlendTile - 1) / kBlendTile;
    const int t = a.list[1 + 2 * blockIdx.x];
    const uint32_t mask = (uint32_t)a.list[2 + 2 * blockIdx.x];
    const int X0 = (t % gx) * kBlendTile, Y0 = (t / gx) * kBlendTile, f = blockIdx.y;
    for (int i = threadIdx.x; i < kBlendTile * kBlendTile; i += blockDim.x) {
        const int x = X0 + (i % kBlendTile), y = Y0 + i / kBlendTile;
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

// Multi-band (3 levels): grid (listed tiles, ceil(frames / kMbFrames)), block kMbThreads2/4, the
// source positions computed once per block and reused for its kMbFrames captures.  Level ranges
// held per tile
// (origin of the 32-px tile X0): level 0 [X0-16, X0+48), level 1 [X0/2-6, X0/2+20] (g1, m1),
// level 2 [X0/4-2, X0/4+9] (g2, m2, B2), collapsed level 1 [X0/2-1, X0/2+16] (R1).  Entries at
// coordinates outside the mosaic hold the reflected coordinate's value, so reflected lookups
// (always inside the mosaic) land in range.
constexpr int kMbR0 = kBlendTile + 2 * kBlendHalo;   // 64
constexpr int kMbN1 = 27, kMbO1 = 6;                  // level 1: [X0/2 - 6, X0/2 + 20]
constexpr int kMbN2 = 12, kMbO2 = 2;                  // level 2: [X0/4 - 2, X0/4 + 9]
constexpr int kMbNR = 18, kMbOR = 1;                  // R1:      [X0/2 - 1, X0/2 + 16]
constexpr int kMbFirst = 2, kMbUsed = 57;             // level-0 offsets the pyramid reads

__device__ __forceinline__ int exp_taps(int x, int n, int *idx, int *wt)
{
    if ((x & 1) == 0) {
        idx[0] = refl(x / 2 - 1, n), wt[0] = 1;
        idx[1] = refl(x / 2, n), wt[1] = 6;
        idx[2] = refl(x / 2 + 1, n), wt[2] = 1;
        return 3;
    }
    idx[0] = refl((x - 1) / 2, n), wt[0] = 4;
    idx[1] = refl((x + 1) / 2, n), wt[1] = 4;
    idx[2] = idx[1], wt[2] = 0;   // padding tap: adds an exact 0, keeps the trip count fixed
    return 3;
}

// LDS of one multi-band block for up to S owner slots.  Level-0 arrays hold the 57 x 57 part of
// the 64 x 64 neighbourhood the pyramid reads (offsets [2, 58]); hs/hm: the horizontal passes of
// the separable 5-tap reduces, aliased with the blend arrays of the later phases.
template <int CN, int S>
struct MbLds {
    static constexpr int HS = S <= 2 ? S : 1;   // slots per separable-pass group
    uint8_t g0[S][kMbUsed * kMbUsed * CN];
    int32_t g1[S][kMbN1 * kMbN1 * CN];
    int32_t g2[S][kMbN2 * kMbN2 * CN];
    uint16_t m1[S][kMbN1 * kMbN1];
    int32_t m2[S][kMbN2 * kMbN2];
    uint8_t own[kMbUsed * kMbUsed];
    union {
        struct {   // phases 2-3 (separable reduce passes)
            uint16_t hs[HS][kMbUsed * kMbN1 * CN];
            uint8_t hm[HS][kMbUsed * kMbN1];
            int32_t hs2[HS][kMbN1 * kMbN2 * CN];
            int32_t hm2[HS][kMbN1 * kMbN2];
        };
        struct {   // phases 4-6
            double b2[kMbN2 * kMbN2 * CN];
            double r1[kMbNR * kMbNR * CN];
        };
    };
};

// Geometry of one multi-band tile: level sizes and the origins of the arrays held per level.
struct MbGeo {
    int W, H, w1, h1, w2, h2;
    int X0, Y0, RX, RY, X1, Y1, X2, Y2, XR, YR;
};

// Level coordinate -> reflected coordinate.  IN (interior tile): every coordinate the tile
// touches lies inside its level, so the reflection is the identity and index arithmetic folds.
template <bool IN>
__device__ __forceinline__ int rf(int i, int n) { return IN ? i : refl(i, n); }
template <bool IN>
__device__ __forceinline__ int ix2(int c, int o, int n)
{
    return IN ? c - o : min(max(c - o, 0), n - 1);
}

// One capture through the pyramid phases 2-6 (g0 and the owner map already in LDS).
template <int CN, int S, bool IN>
__device__ __forceinline__ void mb_phases(const KParams &P, const MbGeo &G, MbLds<CN, S> &L,
                                          int ns, int f)
{
    const int tid = threadIdx.x, nt = blockDim.x;
    const int w5[5] = {1, 4, 6, 4, 1};
    const int RX2 = G.RX + kMbFirst, RY2 = G.RY + kMbFirst;   // origin of the level-0 arrays
    auto i0 = [&](int cx, int cy) {
        return ix2<IN>(cy, RY2, kMbUsed) * kMbUsed + ix2<IN>(cx, RX2, kMbUsed);
    };
    auto i1 = [&](int cx, int cy) {
        return ix2<IN>(cy, G.Y1, kMbN1) * kMbN1 + ix2<IN>(cx, G.X1, kMbN1);
    };
    auto i2 = [&](int cx, int cy) {
        return ix2<IN>(cy, G.Y2, kMbN2) * kMbN2 + ix2<IN>(cx, G.X2, kMbN2);
    };
    auto ir = [&](int cx, int cy) {
        return ix2<IN>(cy, G.YR, kMbNR) * kMbNR + ix2<IN>(cx, G.XR, kMbNR);
    };
    if (IN) {
        // 2-3, interior tiles: separable 5-tap reduces (integer sums: the same values as the
        // 25-tap form).  Level-1 entry e reads level-0 offsets 2e + [0, 5) of the 57-wide
        // arrays; level-2 entry z reads level-1 entries 2z + [0, 5).
        constexpr int HS = MbLds<CN, S>::HS;
        for (int jg = 0; jg < ns; jg += HS) {
            for (int i = tid; i < kMbUsed * kMbN1 * HS; i += nt) {
                const int jl = i / (kMbUsed * kMbN1), e0 = i % (kMbUsed * kMbN1), j = jg + jl;
                if (j >= ns) break;
                const int r = e0 / kMbN1, e = e0 % kMbN1;
                const uint8_t *g = &L.g0[j][(r * kMbUsed + 2 * e) * CN];
                const uint8_t *ow = &L.own[r * kMbUsed + 2 * e];
                int acc[CN], macc = 0;
#pragma unroll
                for (int k = 0; k < CN; k++) acc[k] = 0;
#pragma unroll
                for (int v = 0; v < 5; v++) {
                    macc += ow[v] == j ? w5[v] : 0;
#pragma unroll
                    for (int k = 0; k < CN; k++) acc[k] += w5[v] * g[v * CN + k];
                }
                L.hm[jl][e0] = (uint8_t)macc;
#pragma unroll
                for (int k = 0; k < CN; k++) L.hs[jl][e0 * CN + k] = (uint16_t)acc[k];
            }
            __syncthreads();
            for (int i = tid; i < kMbN1 * kMbN1 * HS; i += nt) {
                const int jl = i / (kMbN1 * kMbN1), e0 = i % (kMbN1 * kMbN1), j = jg + jl;
                if (j >= ns) break;
                const int ey = e0 / kMbN1, ex = e0 % kMbN1;
                int acc[CN], macc = 0;
#pragma unroll
                for (int k = 0; k < CN; k++) acc[k] = 0;
#pragma unroll
                for (int u = 0; u < 5; u++) {
                    const int q = (2 * ey + u) * kMbN1 + ex;
                    macc += w5[u] * L.hm[jl][q];
#pragma unroll
                    for (int k = 0; k < CN; k++) acc[k] += w5[u] * L.hs[jl][q * CN + k];
                }
                L.m1[j][e0] = (uint16_t)macc;
#pragma unroll
                for (int k = 0; k < CN; k++) L.g1[j][e0 * CN + k] = acc[k];
            }
            __syncthreads();
            for (int i = tid; i < kMbN1 * kMbN2 * HS; i += nt) {
                const int jl = i / (kMbN1 * kMbN2), e0 = i % (kMbN1 * kMbN2), j = jg + jl;
                if (j >= ns) break;
                const int r = e0 / kMbN2, e = e0 % kMbN2;
                int acc[CN], macc = 0;
#pragma unroll
                for (int k = 0; k < CN; k++) acc[k] = 0;
#pragma unroll
                for (int v = 0; v < 5; v++) {
                    const int q = r * kMbN1 + 2 * e + v;
                    macc += w5[v] * L.m1[j][q];
#pragma unroll
                    for (int k = 0; k < CN; k++) acc[k] += w5[v] * L.g1[j][q * CN + k];
                }
                L.hm2[jl][e0] = macc;
#pragma unroll
                for (int k = 0; k < CN; k++) L.hs2[jl][e0 * CN + k] = acc[k];
            }
            __syncthreads();
            for (int i = tid; i < kMbN2 * kMbN2 * HS; i += nt) {
                const int jl = i / (kMbN2 * kMbN2), e0 = i % (kMbN2 * kMbN2), j = jg + jl;
                if (j >= ns) break;
                const int ey = e0 / kMbN2, ex = e0 % kMbN2;
                int acc[CN], macc = 0;
#pragma unroll
                for (int k = 0; k < CN; k++) acc[k] = 0;
#pragma unroll
                for (int u = 0; u < 5; u++) {
                    const int q = (2 * ey + u) * kMbN2 + ex;
                    macc += w5[u] * L.hm2[jl][q];
#pragma unroll
                    for (int k = 0; k < CN; k++) acc[k] += w5[u] * L.hs2[jl][q * CN + k];
                }
                L.m2[j][e0] = macc;
#pragma unroll
                for (int k = 0; k < CN; k++) L.g2[j][e0 * CN + k] = acc[k];
            }
            __syncthreads();
        }
    } else {
        // 2. level 1: g1 = reduce(g0), m1 = reduce(owner == slot)
        for (int i = tid; i < kMbN1 * kMbN1 * S; i += nt) {
            const int j = i / (kMbN1 * kMbN1), e = i % (kMbN1 * kMbN1);
            if (j >= ns) break;
            const int qx = refl(G.X1 + e % kMbN1, G.w1), qy = refl(G.Y1 + e / kMbN1, G.h1);
            int macc = 0, acc[CN];
#pragma unroll
            for (int k = 0; k < CN; k++) acc[k] = 0;
#pragma unroll
            for (int u = 0; u < 5; u++) {
                const int cy = refl(2 * qy + u - 2, G.H);
#pragma unroll
                for (int v = 0; v < 5; v++) {
                    const int cx = refl(2 * qx + v - 2, G.W), wt = w5[u] * w5[v];
                    const int p = i0(cx, cy);
                    macc += L.own[p] == j ? wt : 0;
#pragma unroll
                    for (int k = 0; k < CN; k++) acc[k] += wt * L.g0[j][p * CN + k];
                }
            }
            L.m1[j][e] = (uint16_t)macc;
#pragma unroll
            for (int k = 0; k < CN; k++) L.g1[j][e * CN + k] = acc[k];
        }
        __syncthreads();
        // 3. level 2: g2 = reduce(g1), m2 = reduce(m1)
        for (int i = tid; i < kMbN2 * kMbN2 * S; i += nt) {
            const int j = i / (kMbN2 * kMbN2), e = i % (kMbN2 * kMbN2);
            if (j >= ns) break;
            const int zx = refl(G.X2 + e % kMbN2, G.w2), zy = refl(G.Y2 + e / kMbN2, G.h2);
            int macc = 0, acc[CN];
#pragma unroll
            for (int k = 0; k < CN; k++) acc[k] = 0;
#pragma unroll
            for (int u = 0; u < 5; u++) {
                const int qy = refl(2 * zy + u - 2, G.h1);
#pragma unroll
                for (int v = 0; v < 5; v++) {
                    const int qx = refl(2 * zx + v - 2, G.w1), wt = w5[u] * w5[v];
                    const int p = i1(qx, qy);
                    macc += wt * L.m1[j][p];
#pragma unroll
                    for (int k = 0; k < CN; k++) acc[k] += wt * L.g1[j][p * CN + k];
                }
            }
            L.m2[j][e] = macc;
#pragma unroll
            for (int k = 0; k < CN; k++) L.g2[j][e * CN + k] = acc[k];
        }
        __syncthreads();
    }
    // 4. B2 = sum m2 g2 / (sum m2 * 65536)
    for (int i = tid; i < kMbN2 * kMbN2 * CN; i += nt) {
        const int e = i / CN, k = i % CN;
        int64_t num = 0, den = 0;
        for (int j = 0; j < ns; j++) {
            num += (int64_t)L.m2[j][e] * L.g2[j][e * CN + k];
            den += L.m2[j][e];
        }
        L.b2[i] = den ? (double)num / ((double)den * 65536.0) : 0.0;
    }
    __syncthreads();
    // 5. R1 = B1 + up(B2), B1 = sum m1 (16384 g1 - E(g2)) / (sum m1 * 4194304)
    for (int i = tid; i < kMbNR * kMbNR * CN; i += nt) {
        const int e = i / CN, k = i % CN;
        const int qx = rf<IN>(G.XR + e % kMbNR, G.w1), qy = rf<IN>(G.YR + e / kMbNR, G.h1);
        int iy[3], wy[3], ix[3], wx[3];
        exp_taps(qy, G.h2, iy, wy);
        exp_taps(qx, G.w2, ix, wx);
        int64_t num = 0, den = 0;
        const int p1 = i1(qx, qy);
        for (int j = 0; j < ns; j++) {
            int e2 = 0;   // <= 64 * 65536 * 255 < 2^31: exact in int32
#pragma unroll
            for (int u = 0; u < 3; u++)
#pragma unroll
                for (int v = 0; v < 3; v++)
                    e2 += wy[u] * wx[v] * L.g2[j][i2(ix[v], iy[u]) * CN + k];
            const int l1 = 16384 * L.g1[j][p1 * CN + k] - e2;
            num += (int64_t)L.m1[j][p1] * l1;
            den += L.m1[j][p1];
        }
        const double b1 = den ? (double)num / ((double)den * 4194304.0) : 0.0;
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < 3; u++)
#pragma unroll
            for (int v = 0; v < 3; v++)
                acc += (double)(wy[u] * wx[v]) * L.b2[i2(ix[v], iy[u]) * CN + k];
        L.r1[i] = b1 + acc / 64.0;
    }
    __syncthreads();
    // 6. R0 = L0_owner / 16384 + up(R1) over the tile's own pixels
    for (int i = tid; i < kBlendTile * kBlendTile; i += nt) {
        const int x = G.X0 + (i % kBlendTile), y = G.Y0 + i / kBlendTile;
        if (!IN && (x >= G.W || y >= G.H)) continue;
        const int p0 = i0(x, y), s = L.own[p0];
        uint8_t *o = P.out + (int64_t)f * P.out_fstride + (int64_t)y * P.out_pitch + x * CN;
        if (s == kBlendNone) {
#pragma unroll
            for (int k = 0; k < CN; k++) o[k] = 0;
            continue;
        }
        int iy[3], wy[3], ix[3], wx[3];
        exp_taps(y, G.h1, iy, wy);
        exp_taps(x, G.w1, ix, wx);
#pragma unroll
        for (int k = 0; k < CN; k++) {
            int e1 = 0;   // <= 64 * 256 * 255: exact in int32
            double acc = 0.0;
#pragma unroll
            for (int u = 0; u < 3; u++)
#pragma unroll
                for (int v = 0; v < 3; v++) {
                    e1 += wy[u] * wx[v] * L.g1[s][i1(ix[v], iy[u]) * CN + k];
                    acc += (double)(wy[u] * wx[v]) * L.r1[ir(ix[v], iy[u]) * CN + k];
                }
            const int l0 = 16384 * (int)L.g0[s][p0 * CN + k] - e1;
            const double r0 = (double)l0 / 16384.0 + acc / 64.0;
            const double vf = floor(r0 + 0.5);
            o[k] = (uint8_t)(vf < 0.0 ? 0.0 : (vf > 255.0 ? 255.0 : vf));
        }
    }
    __syncthreads();   // the next capture overwrites the level arrays
}

template <int CN, int INTERP, int S>
__device__ __forceinline__ void multiband_tile(const KBlendArgs &a, MbLds<CN, S> &L)
{
    const KParams &P = a.P;
    MbGeo G;
    G.W = P.out_w;
    G.H = P.out_h;
    G.w1 = (G.W + 1) / 2, G.h1 = (G.H + 1) / 2, G.w2 = (G.w1 + 1) / 2, G.h2 = (G.h1 + 1) / 2;
    const int gx = (G.W + kBlendTile - 1) / kBlendTile;
    const int t = a.list[1 + 2 * blockIdx.x];
    const uint32_t mask = (uint32_t)a.list[2 + 2 * blockIdx.x];
    G.X0 = (t % gx) * kBlendTile, G.Y0 = (t / gx) * kBlendTile;
    G.RX = G.X0 - kBlendHalo, G.RY = G.Y0 - kBlendHalo;         // level-0 origin
    G.X1 = G.X0 / 2 - kMbO1, G.Y1 = G.Y0 / 2 - kMbO1;             // level-1 origin
    G.X2 = G.X0 / 4 - kMbO2, G.Y2 = G.Y0 / 4 - kMbO2;             // level-2 origin
    G.XR = G.X0 / 2 - kMbOR, G.YR = G.Y0 / 2 - kMbOR;             // R1 origin
    const bool interior = G.RX >= 0 && G.RY >= 0 && G.RX + kMbR0 <= G.W && G.RY + kMbR0 <= G.H;
    const int ns = __popc(mask);
    const int tid = threadIdx.x, nt = blockDim.x;
    // owner map of the used neighbourhood as local slot indices (bit rank in `mask`)
    for (int i = tid; i < kMbUsed * kMbUsed; i += nt) {
        const int cx = refl(G.RX + kMbFirst + i % kMbUsed, G.W);
        const int cy = refl(G.RY + kMbFirst + i / kMbUsed, G.H);
        const int o = a.owner[(int64_t)cy * G.W + cx];
        L.own[i] = (uint8_t)((o != kBlendNone && ((mask >> o) & 1u))
                                 ? __popc(mask & ((1u << o) - 1u)) : kBlendNone);
    }
    const int f1 = min(a.n_frames, (int)(blockIdx.y + 1) * kMbFrames);
    for (int f = blockIdx.y * kMbFrames; f < f1; f++) {
        // 1. the owners' warped images over the used neighbourhood, capture f
        uint32_t mrem = mask;
        for (int j = 0; j < ns; j++) {
            const int s = __ffs(mrem) - 1;
            mrem &= mrem - 1;
            int cam, w, h;
            slot_info(P, s, cam, w, h);
            const uint8_t *fb = P.cams[cam] + (int64_t)f * P.cam_fstride[cam];
            for (int i = tid; i < kMbUsed * kMbUsed; i += nt) {
                const int cx = refl(G.RX + kMbFirst + i % kMbUsed, G.W);
                const int cy = refl(G.RY + kMbFirst + i / kMbUsed, G.H);
                int x32, y32, c_, w_, h_;
                slot_xy<INTERP>(P, s, cx, cy, x32, y32, c_, w_, h_);
                const uint32_t v = sample_replicate<CN>(fb, w, h, x32, y32);
#pragma unroll
                for (int k = 0; k < CN; k++) L.g0[j][i * CN + k] = (uint8_t)(v >> (8 * k));
            }
        }
        __syncthreads();
        if (interior) mb_phases<CN, S, true>(P, G, L, ns, f);
        else mb_phases<CN, S, false>(P, G, L, ns, f);
    }
}

}  // namespace mcs
