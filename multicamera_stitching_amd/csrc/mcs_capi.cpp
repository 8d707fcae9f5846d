// mcs_capi.cpp -- the extern "C" boundary of libmcs.so (declared in include/mcs.h).
//
// Replaces, for a calibrated chain, the per-frame work of Stitcher.stitch
// (PostScripts/Stitcher/StitcherClass.py:114-136).  No exception crosses this boundary: every
// entry point returns an MCS_* status and leaves a message in mcs_last_error().
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "hip_rt.h"
#include "mcs_common.h"

struct mcs_plan {
    mcs_flat_desc fd;
    mcs::KParams kp;
    int device = 0;
    hipStream_t stream = nullptr;
    // device buffers for the host-array path (allocated on first use)
    uint8_t *d_cams[MCS_MAX_CAMS] = {};
    uint8_t *d_out = nullptr;
    int64_t out_pitch = 0;
    // prepared tables (mcs_plan_prepare): tile headers, per-pixel LDS descriptors, fallback list
    bool prepared = false;
    int gx = 0, gy = 0, n_fallback = 0;
    int n_big = 0;                    // large-footprint tiles (mcs_stream_big, listed in d_big)
    int *d_big = nullptr;             // (the second half of d_fallback's allocation)
    mcs::TileHdr *d_tiles = nullptr;
    uint32_t *d_desc = nullptr;
    uint32_t *d_desc4 = nullptr;      // compact per-pixel words (the streaming kernel reads these)
    uint16_t *d_spans = nullptr;      // per tile footprint row: the chunks its windows read
    int *d_fallback = nullptr;
    // side stream for the direct-gather tiles, forked from / joined to the caller's stream
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // second side stream: the multi-band level pyramids (concurrent with both of the above)
    hipStream_t side2 = nullptr;
    hipEvent_t ev_join2 = nullptr;
    // multi-band: the streaming tiles under mixed blend pixels run first (d_order[0, n_early)),
    // then the multi-band blend starts on side2 (ev_early) beside the rest of the streaming tiles
    hipEvent_t ev_early = nullptr;
    int *d_order = nullptr;
    int n_early = 0;              // launch-list items of the early launch (multi-band split)
    int n_list = 0;               // items of the whole list (d_order; 0: none, grid order)
    // host path with frames off their calibrated size: upload buffers for the resize pre-pass
    uint8_t *d_raw[MCS_MAX_CAMS] = {};
    size_t raw_bytes[MCS_MAX_CAMS] = {};
    // blended modes (mcs_plan_set_blend): owner map, 32-px tile info, per-frame tile list
    int blend = MCS_BLEND_NONE;
    int n_blend = 0, mb_slots = 0;
    // multi-band: tiles degraded to the feather rule (d_blist + 2 * blend tiles + 3: count, then
    // (tile, feather mask) pairs)
    int n_dense = 0, n_degraded = 0;
    int *d_dense = nullptr;
    uint8_t *d_owner = nullptr;
    uint32_t *d_binfo = nullptr;
    int *d_blist = nullptr;
    // multi-band: per (tile, owner) sample windows, per-tile masks, level scratch per chunk
    uint64_t *d_mbdesc = nullptr;
    int32_t *d_mbtab = nullptr;
    int32_t *d_mbfoot = nullptr;
    uint16_t *d_mbg1 = nullptr;
    int32_t *d_mbg2 = nullptr;
    int mb_chunk = 0;
    // multi-band band pass: bands (the first n_bands_in reach no bottom / right mosaic edge),
    // blend-tile grid -> list index, descriptors; without bands mb_levels computes the levels
    int n_bands = 0, n_bands_in = 0, gxb = 0;
    mcs::MbBand *d_bands = nullptr;
    int *d_tile_bt = nullptr;
    uint64_t *d_bdesc = nullptr;
    uint32_t *d_bgrp = nullptr;    // LDS-ring band pass: group source offsets (band_lds_tables)
    uint4 *d_bdesc16 = nullptr;    // LDS-ring band pass: descriptors + group offsets per row
    int n_bands_lds = 0;
    int64_t mb_mixed_px = 0, mb_r1 = 0;   // per capture: blend pixels computed, R1 entries
    // multi-band sweep (mcs_sweep.hip, prepare_sweep): strips, their output regions (one int per
    // output row), window descriptors, the per-pixel skip map of the stitch kernels; n_strips = 0:
    // the band pass + blend kernels instead
    int n_strips = 0, sw_jb = 0;
    mcs::MbStrip *d_strips = nullptr;
    int *d_region = nullptr;
    uint64_t *d_sdesc = nullptr;
    uint8_t *d_skip = nullptr;
    int64_t sw_px = 0, sw_desc_rows = 0;   // per capture: pixels the sweep writes; descriptor rows
    // per capture, streaming tiles: bytes the footprint DMAs read (row spans, 16-byte chunks) and
    // the bytes of the footprint boxes (every row at its camera's full box width)
    int64_t dma_bytes = 0, box_bytes = 0;
    // cylindrical plans: per-column (sin, cos) and per-row h, host copy and device table
    bool cyl = false;
    std::vector<double> cyl_tab;
    double *d_cyl = nullptr;
    // graph-cut seam labels (mcs_plan_find_seams): host copy and device grid
    std::vector<uint8_t> seam_lab;
    int seam_w = 0, seam_h = 0, seam_k = 0;
    // device max-flow: pairs, push / relabel launches, global relabels, microseconds
    int64_t seam_stats[5] = {0, 0, 0, 0, 0};
    uint8_t *d_seam = nullptr;
    // single-camera remap plans (warp / undistort): blend modes refused; table plans' map
    bool single = false;
    std::vector<int32_t> map_tab;
    int32_t *d_map = nullptr;
};

int mcs::plan_device(const mcs_plan *plan) { return plan ? plan->device : 0; }

#define MCS_VERSION_STRING "mcs 0.1.0 (gfx950 code object, HIP module launch)"


namespace {

using mcs::DeviceGuard;
using mcs::kMaxDevices;
using mcs::rt::Api;

struct Kernels {
    bool loaded = false;
    hipFunction_t prepare[5][2] = {};     // [channels][interp]
    hipFunction_t stream[5][2] = {};      // [channels][buffer-resource DMA]
    hipFunction_t stream_big[5][2] = {};  // large-footprint tiles, as stream
    hipFunction_t direct[5][2][2] = {};   // [channels][interp][32-bit offsets]
    hipFunction_t footprint[2] = {};
    hipFunction_t resize[5] = {};         // [channels]
    hipFunction_t blend_owner[2] = {};    // [interp]
    hipFunction_t blend_classify = nullptr;
    hipFunction_t seam_sample[5][2] = {};  // [channels][interp]
    hipFunction_t feather[5][2] = {};     // [channels][interp]
    hipFunction_t mb_prep[5][2] = {};     // [channels][interp]
    hipFunction_t mb_levels[5] = {};      // [channels]
    hipFunction_t mb_blend[5][3] = {};    // [channels][<= 2 owners, <= 4, <= 8]
    // [channels][unaligned / dword-aligned windows][interior, bottom / right edge, both]
    hipFunction_t mb_bands[5][2][3] = {};
    hipFunction_t mb_bdesc[5][2] = {};    // [channels][interp]
    // multi-band sweep (module kModSweep): [channels][dword-aligned windows][2 / 4 owners]
    hipFunction_t mb_sweep[4][2][2] = {};
    hipFunction_t mb_sweep_desc[4][2] = {};   // [channels][interp]
};
Kernels g_k[kMaxDevices];
std::mutex g_k_mu;

// The stitch module's kernels on `device` (looked up once per device).
int kernels(const Api *A, int device, const Kernels **out)
{
    if (device < 0 || device >= kMaxDevices) return mcs::fail(MCS_E_INVALID, "device %d", device);
    std::lock_guard<std::mutex> lk(g_k_mu);
    Kernels &k = g_k[device];
    if (!k.loaded) {
        auto fn = [&](const char *name, hipFunction_t *f) {
            return mcs::module_function(A, device, mcs::kModStitch, name, f);
        };
        char name[64];
        int rc = MCS_OK;
        for (int c = 1; c <= 4 && rc == MCS_OK; c++) {
            snprintf(name, sizeof(name), "mcs_stream_c%d", c);
            rc = fn(name, &k.stream[c][0]);
            snprintf(name, sizeof(name), "mcs_stream_c%d_b32", c);
            if (rc == MCS_OK) rc = fn(name, &k.stream[c][1]);
            snprintf(name, sizeof(name), "mcs_stream_big_c%d", c);
            if (rc == MCS_OK) rc = fn(name, &k.stream_big[c][0]);
            snprintf(name, sizeof(name), "mcs_stream_big_c%d_b32", c);
            if (rc == MCS_OK) rc = fn(name, &k.stream_big[c][1]);
            snprintf(name, sizeof(name), "mcs_resize_c%d", c);
            if (rc == MCS_OK) rc = fn(name, &k.resize[c]);
            snprintf(name, sizeof(name), "mcs_mb_levels_c%d", c);
            if (rc == MCS_OK) rc = fn(name, &k.mb_levels[c]);
            for (int al = 0; al < 2; al++) {
                const char *sfx = al ? "_a" : "";
                snprintf(name, sizeof(name), "mcs_mb_bands%s_c%d", sfx, c);
                if (rc == MCS_OK) rc = fn(name, &k.mb_bands[c][al][0]);
                snprintf(name, sizeof(name), "mcs_mb_bands_br%s_c%d", sfx, c);
                if (rc == MCS_OK) rc = fn(name, &k.mb_bands[c][al][1]);
                snprintf(name, sizeof(name), "mcs_mb_bands_all%s_c%d", sfx, c);
                if (rc == MCS_OK) rc = fn(name, &k.mb_bands[c][al][2]);
            }
            snprintf(name, sizeof(name), "mcs_mb_blend_c%d_s2", c);
            if (rc == MCS_OK) rc = fn(name, &k.mb_blend[c][0]);
            snprintf(name, sizeof(name), "mcs_mb_blend_c%d_s4", c);
            if (rc == MCS_OK) rc = fn(name, &k.mb_blend[c][1]);
            snprintf(name, sizeof(name), "mcs_mb_blend_c%d_s8", c);
            if (rc == MCS_OK) rc = fn(name, &k.mb_blend[c][2]);
            for (int i = 0; i < 2 && rc == MCS_OK; i++) {
                snprintf(name, sizeof(name), "mcs_prepare_c%d_i%d", c, i);
                rc = fn(name, &k.prepare[c][i]);
                snprintf(name, sizeof(name), "mcs_feather_c%d_i%d", c, i);
                if (rc == MCS_OK) rc = fn(name, &k.feather[c][i]);
                snprintf(name, sizeof(name), "mcs_mb_prep_c%d_i%d", c, i);
                if (rc == MCS_OK) rc = fn(name, &k.mb_prep[c][i]);
                snprintf(name, sizeof(name), "mcs_mb_bdesc_c%d_i%d", c, i);
                if (rc == MCS_OK) rc = fn(name, &k.mb_bdesc[c][i]);
                snprintf(name, sizeof(name), "mcs_seam_sample_c%d_i%d", c, i);
                if (rc == MCS_OK) rc = fn(name, &k.seam_sample[c][i]);
                for (int o = 0; o < 2 && rc == MCS_OK; o++) {
                    snprintf(name, sizeof(name), "mcs_direct_c%d_i%d_o%d", c, i, o ? 32 : 64);
                    rc = fn(name, &k.direct[c][i][o]);
                }
            }
        }
        for (int c = 1; c <= 3 && rc == MCS_OK; c++)
            for (int al = 0; al < 2 && rc == MCS_OK; al++) {
                for (int jb = 0; jb < 2 && rc == MCS_OK; jb++) {
                    snprintf(name, sizeof(name), "mcs_mb_sweep%s_c%d_j%d", al ? "_a" : "", c,
                             jb ? 4 : 2);
                    rc = mcs::module_function(A, device, mcs::kModSweep, name,
                                              &k.mb_sweep[c][al][jb]);
                }
                snprintf(name, sizeof(name), "mcs_mb_sweep_desc_c%d_i%d", c, al);
                if (rc == MCS_OK)
                    rc = mcs::module_function(A, device, mcs::kModSweep, name,
                                              &k.mb_sweep_desc[c][al]);
            }
        if (rc == MCS_OK) rc = fn("mcs_footprint_i0", &k.footprint[0]);
        if (rc == MCS_OK) rc = fn("mcs_footprint_i1", &k.footprint[1]);
        if (rc == MCS_OK) rc = fn("mcs_blend_owner_i0", &k.blend_owner[0]);
        if (rc == MCS_OK) rc = fn("mcs_blend_owner_i1", &k.blend_owner[1]);
        if (rc == MCS_OK) rc = fn("mcs_blend_classify", &k.blend_classify);
        if (rc) return rc;
        k.loaded = true;
    }
    *out = &k;
    return MCS_OK;
}

int ensure_stream(const Api *A, mcs_plan *p)
{
    if (!p->stream) HIP_TRY(A->hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
    return MCS_OK;
}

int ensure_host_buffers(const Api *A, mcs_plan *p)
{
    const int C = p->fd.channels;
    for (int i = 0; i < p->fd.n_cams; i++) {
        if (p->d_cams[i]) continue;
        const size_t bytes = (size_t)p->fd.cam_w[i] * p->fd.cam_h[i] * C;
        HIP_TRY(A->hipMalloc((void **)&p->d_cams[i], bytes > 0 ? bytes : 1));
    }
    if (!p->d_out && p->fd.out_w > 0 && p->fd.out_h > 0) {
        p->out_pitch = ((int64_t)p->fd.out_w * C + 63) / 64 * 64;
        HIP_TRY(A->hipMalloc((void **)&p->d_out, (size_t)p->out_pitch * p->fd.out_h));
    }
    return MCS_OK;
}

void need_mask(const mcs_flat_desc &fd, bool *need)
{
    for (int i = 0; i < MCS_MAX_CAMS; i++) need[i] = false;
    need[0] = true;
    for (int j = 0; j < fd.n_stages; j++) need[fd.st[j].cam] = true;
}

// Lowest used camera address for frame 0 of `kp`, and whether every used byte of that frame lies
// within 4 GiB above it (then the kernel addresses taps as SGPR base + 32-bit offsets).
int g_force_off64 = 0;   // test hook: exercise the 64-bit-address kernels

bool offset_base(const mcs_plan *p, const mcs::KParams &kp, const uint8_t **base)
{
    bool need[MCS_MAX_CAMS];
    need_mask(p->fd, need);
    uintptr_t lo = UINTPTR_MAX, hi = 0;
    for (int i = 0; i < p->fd.n_cams; i++) {
        if (!need[i]) continue;
        const uintptr_t a = (uintptr_t)kp.cams[i];
        const uintptr_t e = a + (uintptr_t)p->fd.cam_w[i] * p->fd.cam_h[i] * p->fd.channels;
        lo = a < lo ? a : lo;
        hi = e > hi ? e : hi;
    }
    const bool off32 = !g_force_off64 && hi - lo < (uintptr_t(1) << 32);
    *base = off32 ? (const uint8_t *)lo : nullptr;
    return off32;
}

// The streaming kernel's DMA base: when every byte of every capture of every used camera lies in
// [base, base + 4 GiB) the footprint rows are read through one buffer resource with 32-bit
// offsets (mcs_stream_c*_b32).  Captures are fstride = cam_fstride[0] apart (the stream kernel's
// layout).
bool stream_base(const mcs_plan *p, const mcs::KParams &kp, int n_frames, const uint8_t **base)
{
    bool need[MCS_MAX_CAMS];
    need_mask(p->fd, need);
    uintptr_t lo = UINTPTR_MAX, hi = 0;
    const uintptr_t span = (uintptr_t)(n_frames > 0 ? n_frames - 1 : 0) * kp.cam_fstride[0];
    for (int i = 0; i < p->fd.n_cams; i++) {
        if (!need[i]) continue;
        const uintptr_t a = (uintptr_t)kp.cams[i];
        const uintptr_t e = a + span + (uintptr_t)p->fd.cam_w[i] * p->fd.cam_h[i] * p->fd.channels;
        lo = a < lo ? a : lo;
        hi = e > hi ? e : hi;
    }
    const bool b32 = !g_force_off64 && lo <= hi && hi - lo < (uintptr_t(1) << 32);
    *base = b32 ? (const uint8_t *)lo : kp.base;
    return b32;
}

int launch_args(const Api *A, hipFunction_t f, unsigned gx, unsigned gy, unsigned bx,
                unsigned by, void *args, size_t sz, hipStream_t s)
{
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                   HIP_LAUNCH_PARAM_END};
    HIP_TRY(A->hipModuleLaunchKernel(f, gx, gy, 1, bx, by, 1, 0, s, nullptr, cfg));
    return MCS_OK;
}

void mb_args(const mcs_plan *p, const mcs::KParams &P, mcs::KMbArgs &a)
{
    a.P = P;
    a.owner = p->d_owner;
    a.list = p->d_blist;
    a.desc = p->d_mbdesc;
    a.tab = p->d_mbtab;
    a.foot = p->d_mbfoot;
    a.g1 = p->d_mbg1;
    a.g2 = p->d_mbg2;
    a.slots = p->mb_slots;
    a.chunk = p->mb_chunk;
    a.f0 = 0;
    a.nf = 0;
    a.list0 = 0;
    a.n_list = p->n_blend;
}

void band_args(const mcs_plan *p, const mcs::KParams &P, mcs::KMbBandArgs &a)
{
    a.P = P;
    a.list = p->d_blist;
    a.tile_bt = p->d_tile_bt;
    a.bands = p->d_bands;
    a.bdesc = p->d_bdesc;
    a.bgrp = p->d_bgrp;
    a.bdesc16 = p->d_bdesc16;
    a.g1 = p->d_mbg1;
    a.g2 = p->d_mbg2;
    a.slots = p->mb_slots;
    a.chunk = p->mb_chunk;
    a.f0 = 0;
    a.nf = 0;
    a.gxb = p->gxb;
    a.band0 = 0;
    a.n_in = p->n_bands_in;
    a.band1 = p->n_bands_in;
    a.nb = p->n_bands;
}

// 1-D grid of an XCD-grouped launch of n units (mcs_blend.h xcd_unit): 8 * ceil(n / 8) blocks.
unsigned xcd_grid(int64_t n) { return 8u * (unsigned)((n + 7) / 8); }

// The band pass's dword-aligned window form (mb_bands AL, mb_desc's sh) applies when every used
// camera's rows and frames are multiples of 4 bytes, its frames start at 4-byte boundaries and hold
// at least pitch + 12 bytes; otherwise the unaligned 8-byte form.
int band_form(const mcs_plan *p, const mcs::KParams &P)
{
    bool need[MCS_MAX_CAMS];
    need_mask(p->fd, need);
    const int C = p->fd.channels;
    for (int i = 0; i < p->fd.n_cams; i++) {
        if (!need[i]) continue;
        const int64_t pitch = (int64_t)p->fd.cam_w[i] * C, fb = pitch * p->fd.cam_h[i];
        if (pitch % 4 || fb % 4 || fb < pitch + 12 || P.cam_fstride[i] % 4 ||
            (uintptr_t)P.cams[i] % 4)
            return 0;
    }
    return 1;
}

// Launch list of the streaming kernel for tiles in launch order: stream_tile deals a list to the
// 8 XCDs in equal contiguous slices (XCD x: entries [x * per, (x + 1) * per)), each walked in
// order, so an XCD holds a band of whole tile rows (horizontal neighbours share its L2; measured
// faster than vertical strips, round 3); slices padded to one length with -1.
std::vector<int> launch_list(const std::vector<int> &tiles)
{
    const size_t n = tiles.size(), per = (n + 7) / 8;
    std::vector<int> out(8 * per, -1);
    for (size_t i = 0; i < n; i++) out[i] = tiles[i];
    return out;
}

// The band pass of a multi-band plan (after mb_prep): per (owner slot, blend-tile row) the
// level-1 / level-2 mosaic columns the tiles of that row read from that owner (mb_prep's per-slot
// ranges), merged where they overlap and covered by 64-column windows kMbBandStride apart; then
// the windows' sample descriptors (once).  Mosaics under 128 px a side (a unit would reach past
// two opposite edges) and plans whose camera frames are too small for the 8-byte window loads
// stay with mb_levels.
int band_lds_tables(const Api *A, mcs_plan *p, std::vector<mcs::MbBand> &bands, hipStream_t s);

int prepare_bands(const Api *A, mcs_plan *p, const Kernels *k, hipStream_t s)
{
    const int n = p->n_blend, S = p->mb_slots, C = p->fd.channels;
    const int W = p->fd.out_w, H = p->fd.out_h;
    p->gxb = (W + mcs::kBlendTileW - 1) / mcs::kBlendTileW;
    const int gyb = (H + mcs::kBlendTileH - 1) / mcs::kBlendTileH;
    const mcs::KParams &P = p->kp;
    for (int c = 0; c <= P.n_stages; c++) {
        if (c == 0 && P.cam0_w == 0) continue;     // (cylindrical plans: no slot-0 camera)
        const int64_t w = c == 0 ? P.cam0_w : P.st[c - 1].src_w;
        const int64_t h = c == 0 ? P.cam0_h : P.st[c - 1].src_h;
        if ((h - 1) * w * C < 16) return MCS_OK;   // (mb_levels' guarded window loads)
    }
    if (W < 128 || H < 128) return MCS_OK;
    std::vector<int> list(1 + 2 * (size_t)n);
    std::vector<int> cnt((size_t)n * mcs::kMbTabCounts);
    const size_t words = (size_t)mcs::mb_tab_words(S);
    const size_t cnt_at = (size_t)S * (mcs::kMbNRX * mcs::kMbNRY + mcs::kMbN2X * mcs::kMbN2Y) +
                          mcs::kMbNRX * mcs::kMbNRY + mcs::kMbN2X * mcs::kMbN2Y;
    HIP_TRY(A->hipMemcpyAsync(list.data(), p->d_blist, list.size() * sizeof(int),
                              hipMemcpyDeviceToHost, s));
    HIP_TRY(A->hipMemcpy2DAsync(cnt.data(), mcs::kMbTabCounts * sizeof(int), p->d_mbtab + cnt_at,
                                words * sizeof(int), mcs::kMbTabCounts * sizeof(int), (size_t)n,
                                hipMemcpyDeviceToHost, s));
    HIP_TRY(A->hipStreamSynchronize(s));
    // per (plan slot, tile row): the level-1 / level-2 column intervals of its tiles
    struct Need { int q1lo, q1hi, z2lo, z2hi; };
    constexpr int kSlots = 32;   // plan slots: bits of a tile's owner mask
    std::vector<std::vector<Need>> need((size_t)kSlots * gyb);
    std::vector<int> tile_bt((size_t)p->gxb * gyb, -1);
    for (int i = 0; i < n; i++) {
        const int t = list[1 + 2 * i];
        const uint32_t mask = (uint32_t)list[2 + 2 * i];
        tile_bt[t] = i;
        const int Y0 = (t / p->gxb) * mcs::kBlendTileH;
        const int *c = cnt.data() + (size_t)i * mcs::kMbTabCounts + mcs::kMbTabRanges;
        uint32_t m = mask;
        for (int j = 0; m; j++, m &= m - 1) {
            const int slot = __builtin_ctz(m);
            Need q{c[4 * j], c[4 * j + 1], c[4 * j + 2], c[4 * j + 3]};
            if (q.q1lo > q.q1hi && q.z2lo > q.z2hi) continue;
            need[(size_t)slot * gyb + Y0 / mcs::kBlendTileH].push_back(q);
        }
    }
    // per capture: the blend pixels and R1 entries the blend kernel computes (counted before the
    // band list: a plan whose tiles need no band still blends its mixed pixels)
    p->mb_mixed_px = p->mb_r1 = 0;
    for (int i = 0; i < n; i++) {
        p->mb_mixed_px += cnt[(size_t)i * mcs::kMbTabCounts];
        p->mb_r1 += cnt[(size_t)i * mcs::kMbTabCounts + 1];
    }
    std::vector<mcs::MbBand> bands;
    const int big = 1 << 30;
    for (int slot = 0; slot < kSlots; slot++)
        for (int row = 0; row < gyb; row++) {
            std::vector<Need> &v = need[(size_t)slot * gyb + row];
            if (v.empty()) continue;
            // (a column interval in level-0 terms: its lowest needed level-0 column)
            auto lo0 = [&](const Need &q) {
                return std::min(q.z2lo <= q.z2hi ? 4 * q.z2lo : big,
                                q.q1lo <= q.q1hi ? 2 * q.q1lo : big);
            };
            std::sort(v.begin(), v.end(), [&](const Need &a, const Need &b) {
                return lo0(a) < lo0(b);
            });
            size_t i = 0;
            while (i < v.size()) {
                Need u = v[i++];
                auto hi0 = [&](const Need &q) {
                    return std::max(q.z2lo <= q.z2hi ? 4 * q.z2hi : -big,
                                    q.q1lo <= q.q1hi ? 2 * q.q1hi : -big);
                };
                // merge intervals that overlap or nearly touch (one window covers the gap)
                while (i < v.size() && lo0(v[i]) <= hi0(u) + 2 * mcs::kMbBandStride) {
                    const Need &q = v[i++];
                    if (q.q1lo <= q.q1hi)
                        u.q1lo = std::min(u.q1lo, q.q1lo), u.q1hi = std::max(u.q1hi, q.q1hi);
                    if (q.z2lo <= q.z2hi)
                        u.z2lo = std::min(u.z2lo, q.z2lo), u.z2hi = std::max(u.z2hi, q.z2hi);
                }
                // windows: c0 emits level-1 columns [c0/2 + 1, c0/2 + 30] and level-2 columns
                // [c0/4 + 2, c0/4 + 14] (mb_bands' complete lanes)
                int c0 = std::min(u.z2lo <= u.z2hi ? 4 * (u.z2lo - 2) : big,
                                  u.q1lo <= u.q1hi ? 2 * (u.q1lo - 1) : big);
                c0 = c0 >= 0 ? c0 & ~3 : -((-c0 + 3) & ~3);
                for (;;) {
                    bands.push_back(mcs::MbBand{slot, row, c0, 0});
                    const bool z_ok = u.z2lo > u.z2hi || c0 / 4 + 14 >= u.z2hi;
                    const bool q_ok = u.q1lo > u.q1hi || c0 / 2 + 30 >= u.q1hi;
                    if (z_ok && q_ok) break;
                    c0 += mcs::kMbBandStride;
                }
            }
        }
    if (bands.empty()) return MCS_OK;
    {
        // streaming tiles under the blend tiles that have mixed pixels: launched first, so the
        // blend (which overwrites those pixels) can run beside the other streaming tiles
        std::vector<char> early((size_t)p->gx * p->gy, 0);
        for (int i = 0; i < n; i++) {
            if (cnt[(size_t)i * mcs::kMbTabCounts] == 0) continue;
            const int t = list[1 + 2 * i];
            const int X0 = (t % p->gxb) * mcs::kBlendTileW, Y0 = (t / p->gxb) * mcs::kBlendTileH;
            const int x1 = std::min(X0 + mcs::kBlendTileW, W) - 1;
            const int y1 = std::min(Y0 + mcs::kBlendTileH, H) - 1;
            for (int ty = Y0 / mcs::kTileH; ty <= y1 / mcs::kTileH; ty++)
                for (int tx = X0 / mcs::kTileW; tx <= x1 / mcs::kTileW; tx++)
                    early[(size_t)ty * p->gx + tx] = 1;
        }
        std::vector<int> first, late;
        for (size_t t = 0; t < early.size(); t++)
            (early[t] ? first : late).push_back((int)t);
        std::vector<int> order = launch_list(first);
        p->n_early = (int)order.size();
        const std::vector<int> rest = launch_list(late);
        order.insert(order.end(), rest.begin(), rest.end());
        p->n_list = (int)order.size();
        if (p->d_order) (void)A->hipFree(p->d_order);
        HIP_TRY(A->hipMalloc((void **)&p->d_order, order.size() * sizeof(int)));
        HIP_TRY(A->hipMemcpyAsync(p->d_order, order.data(), order.size() * sizeof(int),
                                  hipMemcpyHostToDevice, s));
    }
    // bands whose rows or columns reach past the bottom / right mosaic edge: the _br kernel
    auto br = [&](const mcs::MbBand &b) {
        return b.row * mcs::kBlendTileH - mcs::kBlendHalo + mcs::kMbFirst + mcs::kMbUsedY > H ||
               b.c0 + mcs::kMbBandLanes > W;
    };
    std::stable_sort(bands.begin(), bands.end(),
                     [](const mcs::MbBand &a, const mcs::MbBand &b) { return a.row < b.row; });
    std::stable_partition(bands.begin(), bands.end(), [&](const mcs::MbBand &b) { return !br(b); });
    p->n_bands_in = (int)(std::find_if(bands.begin(), bands.end(), br) - bands.begin());
    const size_t nb = bands.size();
    HIP_TRY(A->hipMalloc((void **)&p->d_bands, nb * sizeof(mcs::MbBand)));
    HIP_TRY(A->hipMalloc((void **)&p->d_tile_bt, tile_bt.size() * sizeof(int)));
    HIP_TRY(A->hipMalloc((void **)&p->d_bdesc,
                         nb * mcs::kMbBandDescRows * mcs::kMbBandLanes * sizeof(uint64_t)));
    HIP_TRY(A->hipMemcpyAsync(p->d_bands, bands.data(), nb * sizeof(mcs::MbBand),
                              hipMemcpyHostToDevice, s));
    HIP_TRY(A->hipMemcpyAsync(p->d_tile_bt, tile_bt.data(), tile_bt.size() * sizeof(int),
                              hipMemcpyHostToDevice, s));
    p->n_bands = (int)nb;
    mcs::KMbBandArgs a;
    band_args(p, p->kp, a);
    int rc = launch_args(A, k->mb_bdesc[C][p->fd.interp], (unsigned)nb, 1, 256, 1, &a, sizeof(a),
                         s);
    if (rc) return rc;
    rc = band_lds_tables(A, p, bands, s);
    if (rc) return rc;
    // the band pass writes only the entries the blend reads: the rest of the scratch holds
    // zeros (or an earlier capture's value of the same entry), never stale garbage
    HIP_TRY(A->hipMemsetAsync(p->d_mbg1, 0,
                              (size_t)n * S * p->mb_chunk * mcs::kMbNRX * mcs::kMbNRY * 8, s));
    HIP_TRY(A->hipMemsetAsync(p->d_mbg2, 0,
                              (size_t)n * S * p->mb_chunk * mcs::kMbN2X * mcs::kMbN2Y * C * 4, s));
    HIP_TRY(A->hipStreamSynchronize(s));
    return MCS_OK;
}

// LDS-ring form of the band pass (mb_bands_body mode 2), once per plan: from the device-built
// window descriptors (mb_bdesc) of every band, the band's source rows [y0, y1] (both taps of
// every lane and row), per row the byte span its samples read and the 256-byte window of the row
// staged for it (16-byte aligned, moved back to end inside the frame), the group table (LDS-DMA
// source offsets of rows 4g .. 4g + 3 per lane) and the descriptors rewritten to ring offsets.
// A band takes the ring only when its rows fit the schedule of mb_bands_body: every row's groups
// issued >= kMbLdsGLead rows before it and still resident (rows advancing with the band's rows, at
// most kMbLdsRows in flight); the rest keep the global-window form.
int band_lds_tables(const Api *A, mcs_plan *p, std::vector<mcs::MbBand> &bands, hipStream_t s)
{
    const size_t nb = bands.size();
    const int C = p->fd.channels, R = mcs::kMbBandRows, DR = mcs::kMbBandDescRows;
    const int L = mcs::kMbBandLanes, NG = mcs::kMbLdsGroups, K = mcs::kMbLdsRows;
    const int SP = mcs::kMbLdsSpan, D4 = mcs::kMbLdsLead / 4;
    p->n_bands_lds = 0;
    std::vector<uint64_t> desc(nb * DR * L);
    HIP_TRY(A->hipMemcpyAsync(desc.data(), p->d_bdesc, desc.size() * sizeof(uint64_t),
                              hipMemcpyDeviceToHost, s));
    HIP_TRY(A->hipStreamSynchronize(s));
    std::vector<uint32_t> grp(nb * NG * L, 0u);
    const int DL = mcs::kMbLdsDescRows;
    std::vector<uint4> d16(nb * DL * L, make_uint4(0u, 0u, 0u, 0u));
    // row r's loop position at which group g is issued (prologue groups: the kMbLdsDescRing
    // descriptor DMAs of the prologue follow them before row 0)
    auto issue = [&](int g) { return g <= D4 ? -mcs::kMbLdsDescRing : 4 * (g - D4 - 1); };
    for (size_t i = 0; i < nb; i++) {
        const int slot = bands[i].slot;
        const int w = slot == 0 ? p->kp.cam0_w : p->kp.st[slot - 1].src_w;
        const int h = slot == 0 ? p->kp.cam0_h : p->kp.st[slot - 1].src_h;
        const int64_t pitch = (int64_t)w * C, fb = pitch * h;
        if (pitch % 4 || pitch < SP) continue;
        uint64_t *d = desc.data() + i * DR * L;
        int y0 = INT32_MAX, y1 = -1;
        bool ok = true;
        for (int e = 0; e < R * L && ok; e++) {
            const uint32_t dx = (uint32_t)d[e], sh = (uint32_t)(d[e] >> 47) & 15u;
            const int64_t oa = dx & 0x7fffffffu;
            const int ya = (int)(oa / pitch), yb = ya + (int)(dx >> 31);
            ok = sh != 15u && yb < h;
            y0 = std::min(y0, ya);
            y1 = std::max(y1, yb);
        }
        if (!ok || y1 - y0 + 1 > 4 * (NG - 2)) continue;
        const int nr = y1 - y0 + 1;
        std::vector<int64_t> lo(nr, INT64_MAX), hi(nr, -1), bs(nr, 0);
        std::vector<int> glo(R, INT32_MAX), ghi(R, -1);
        for (int r = 0; r < R; r++)
            for (int l = 0; l < L; l++) {
                const uint32_t dx = (uint32_t)d[r * L + l];
                const int64_t oa = dx & 0x7fffffffu, cb = oa % pitch;
                const int ya = (int)(oa / pitch) - y0, yb = ya + (int)(dx >> 31);
                for (int y : {ya, yb}) {
                    lo[y] = std::min(lo[y], cb);
                    hi[y] = std::max(hi[y], cb + 2 * C);
                }
                glo[r] = std::min(glo[r], ya / 4);
                ghi[r] = std::max(ghi[r], yb / 4);
            }
        // staged window of every row: 16-byte aligned at its first byte, moved back so that its
        // 256 bytes end inside the frame (4-byte steps: pitch is a multiple of 4)
        for (int y = 0; y < nr && ok; y++) {
            const int64_t room = fb - (int64_t)(y0 + y) * pitch - SP;
            bs[y] = std::min(hi[y] < 0 ? 0 : lo[y] & ~(int64_t)15, room);
            ok = bs[y] >= 0 && (hi[y] < 0 || hi[y] - bs[y] <= SP);
        }
        if (!ok) continue;
        for (int r = 0; r < R && ok; r++)
            ok = issue(ghi[r]) <= r - mcs::kMbLdsGLead && issue(glo[r] + K / 4) >= r;
        if (!ok) continue;
       
        // group table: lane l loads chunk l % 16 of row 4g + l / 16; chunks no sample of the row
        // reads, rows no sample reads and rows past the band: an offset past the frame (the
        // kernel's buffer load fetches nothing for them)
        uint32_t *gt = grp.data() + i * NG * L;
        for (int g = 0; g < NG; g++)
            for (int l = 0; l < L; l++) {
                const int y = 4 * g + l / 16, c = l % 16;
                const bool need = y < nr && hi[y] >= 0 && 16 * c < hi[y] - bs[y];
                gt[g * L + l] = need ? (uint32_t)((int64_t)(y0 + y) * pitch + bs[y] + 16 * c)
                                     : 0xfffffff0u;
            }
        // descriptors: .x = ring offsets of the tap-a / tap-b windows (4-byte aligned), .y keeps
        // the weights and takes the window shift sh = tap byte & 3
        for (int r = 0; r < DR; r++)
            for (int l = 0; l < L; l++) {
                const uint64_t v = d[std::min(r, R - 1) * L + l];
                const uint32_t dx = (uint32_t)v, dy = (uint32_t)(v >> 32);
                const int64_t oa = dx & 0x7fffffffu, cb = oa % pitch;
                const int ya = (int)(oa / pitch) - y0, yb = ya + (int)(dx >> 31);
                const uint32_t wa = (uint32_t)((ya % K) * SP + ((cb & ~(int64_t)3) - bs[ya]));
                const uint32_t wb = (uint32_t)((yb % K) * SP + ((cb & ~(int64_t)3) - bs[yb]));
                const uint32_t ny = (dy & ~(15u << 15)) | ((uint32_t)(cb & 3) << 15);
                d[r * L + l] = (uint64_t)(wa | (wb << 16)) | ((uint64_t)ny << 32);
            }
        // the 16-byte descriptors the kernel stages by LDS-DMA: .x = the windows' ring offsets
        // (12 bits each) with the byte shift in bits 14-15, .y / .w = the doubled bilinear
        // weights of rows a / b as u16 pairs (mb_weights2, precomputed here once per plan
        // instead of per row and wave), .z on rows r % 4 == 0 the lane's source offset of the
        // group issued after row r
        for (int r = 0; r < DL; r++)
            for (int l = 0; l < L; l++) {
                const uint64_t v = d[std::min(r, R - 1) * L + l];
                const uint32_t x = (uint32_t)v, meta = (uint32_t)(v >> 32);
                const uint32_t sh = (meta >> 15) & 3u, fx = meta & 63u, fy = (meta >> 6) & 31u;
                const uint32_t ya = (32u - fy) << 6, yb = fy << 6;
                const uint32_t wa = std::min((32u - fx) * ya, 65535u) |
                                    (std::min(fx * ya, 65535u) << 16);
                const uint32_t wb = std::min((32u - fx) * yb, 65535u) |
                                    (std::min(fx * yb, 65535u) << 16);
                const int g = r / 4 + D4 + 1;
                const uint32_t z = (r < R && r % 4 == 0 && g < NG) ? gt[g * L + l] : 0u;
                d16[(i * DL + r) * L + l] = make_uint4(x | (sh << 14), wa, z, wb);
            }
        bands[i].pad_ |= 1;
        p->n_bands_lds++;
    }
    if (p->n_bands_lds == 0) return MCS_OK;
    HIP_TRY(A->hipMalloc((void **)&p->d_bgrp, grp.size() * sizeof(uint32_t)));
    HIP_TRY(A->hipMemcpyAsync(p->d_bgrp, grp.data(), grp.size() * sizeof(uint32_t),
                              hipMemcpyHostToDevice, s));
    // (d_bdesc keeps the frame-offset descriptors: the ring offsets live only in d_bdesc16, so
    // a launch that takes the unaligned form -- band_form() == 0, decided per launch from the
    // frame pointers and strides -- reads valid descriptors for every band)
    HIP_TRY(A->hipMalloc((void **)&p->d_bdesc16, d16.size() * sizeof(uint4)));
    HIP_TRY(A->hipMemcpyAsync(p->d_bdesc16, d16.data(), d16.size() * sizeof(uint4),
                              hipMemcpyHostToDevice, s));
    HIP_TRY(A->hipMemcpyAsync(p->d_bands, bands.data(), nb * sizeof(mcs::MbBand),
                              hipMemcpyHostToDevice, s));
    HIP_TRY(A->hipStreamSynchronize(s));
    return MCS_OK;
}

// The multi-band sweep of a plan (mcs_sweep.hip), once, after mb_prep: from the mixed pixels mb_prep
// listed per 32 x 64 blend tile,
//   1. per blend-tile row, segments: the listed tiles with mixed pixels, merged where their mixed
//      column hulls lie within 32 px; per output row of a segment its region = the 4-aligned
//      span of that row's mixed pixels;
//   2. runs: a segment continues the run of the row above whose column hull, with it, still fits
//      the window's 100 output columns and whose owners (every owner within 16 px of the run's
//      regions: the masks the blend reads there) stay <= kSwMaxOwners; otherwise it starts one;
//   3. per run a strip (window c0 centred on the hull, rows from ya - 16), the R1 / B2 column
//      ranges its regions read, checked against the columns the window computes;
//   4. the skip map (stitch kernels) and the window descriptors (mcs_mb_sweep_desc).
// Plans the sweep cannot take -- 4 channels, narrow mosaics, a run past the ranges, a region in a
// tile degraded to the feather rule (more than 8 owners near it), MCS_MB_SWEEP=0 -- keep the band
// pass + blend kernels (n_strips = 0).
int prepare_sweep(const Api *A, mcs_plan *p, const Kernels *k, hipStream_t s)
{
    p->n_strips = 0;
    // opt-in (MCS_MB_SWEEP=1): bit-exact, but measured 3x slower than the band pass + blend on
    // the C2 / C4 launches -- latency-bound at ~1 workgroup per CU
    const char *e = getenv("MCS_MB_SWEEP");
    if (!e || e[0] != '1') return MCS_OK;
    const int n = p->n_blend, S = p->mb_slots, C = p->fd.channels;
    const int W = p->fd.out_w, H = p->fd.out_h;
    if (n == 0 || C > 3 || W < 128 || H < 128 || W >= 32768 || H >= 32768) return MCS_OK;
    const mcs::KParams &P = p->kp;
    for (int c = 0; c <= P.n_stages; c++) {
        if (c == 0 && P.cam0_w == 0) continue;     // (cylindrical plans: no slot-0 camera)
        const int64_t w = c == 0 ? P.cam0_w : P.st[c - 1].src_w;
        const int64_t h = c == 0 ? P.cam0_h : P.st[c - 1].src_h;
        if ((h - 1) * w * C < 16 || w < 2 || h < 2) return MCS_OK;
    }
    const int TW = mcs::kBlendTileW, TH = mcs::kBlendTileH;
    const int gxb = (W + TW - 1) / TW, gyb = (H + TH - 1) / TH;
    // the tile list, per tile its pixel count and mixed-pixel list (mb_prep), the owner map
    const size_t words = (size_t)mcs::mb_tab_words(S);
    const size_t cnt_at = (size_t)S * (mcs::kMbNRX * mcs::kMbNRY + mcs::kMbN2X * mcs::kMbN2Y) +
                          mcs::kMbNRX * mcs::kMbNRY + mcs::kMbN2X * mcs::kMbN2Y;
    const size_t rec = mcs::kMbTabCounts + mcs::kMbTilePx / 2;   // counts + pixel list (words)
    std::vector<int> list(1 + 2 * (size_t)n);
    std::vector<int32_t> tab((size_t)n * rec);
    std::vector<uint8_t> own((size_t)W * H);
    HIP_TRY(A->hipMemcpyAsync(list.data(), p->d_blist, list.size() * sizeof(int),
                              hipMemcpyDeviceToHost, s));
    HIP_TRY(A->hipMemcpy2DAsync(tab.data(), rec * 4, p->d_mbtab + cnt_at, words * 4, rec * 4,
                                (size_t)n, hipMemcpyDeviceToHost, s));
    HIP_TRY(A->hipMemcpyAsync(own.data(), p->d_owner, own.size(), hipMemcpyDeviceToHost, s));
    HIP_TRY(A->hipStreamSynchronize(s));
    auto owners_in = [&](int x0, int x1, int y0, int y1) -> uint32_t {
        x0 = std::max(x0, 0), x1 = std::min(x1, W), y0 = std::max(y0, 0), y1 = std::min(y1, H);
        uint32_t m = 0;
        for (int y = y0; y < y1; y++) {
            const uint8_t *r = own.data() + (size_t)y * W;
            for (int x = x0; x < x1; x++)
                if (r[x] != mcs::kBlendNone) m |= 1u << r[x];
        }
        return m;
    };
    // tiles degraded to the feather rule (more than kBlendSlots owners in tile + 16 px)
    std::vector<char> dense((size_t)gxb * gyb, 0);
    for (int ty = 0; ty < gyb; ty++)
        for (int tx = 0; tx < gxb; tx++)
            dense[(size_t)ty * gxb + tx] =
                __builtin_popcount(owners_in(tx * TW - mcs::kBlendHalo, tx * TW + TW + mcs::kBlendHalo,
                                             ty * TH - mcs::kBlendHalo,
                                             ty * TH + TH + mcs::kBlendHalo)) > mcs::kBlendSlots;
    // 1. segments per tile row: per output row of the segment [lo, hi] of its mixed pixels
    struct Seg {
        int x0, x1;                 // 4-aligned column hull
        std::vector<int> lo, hi;    // per row of the tile row (lo > hi: none)
    };
    std::vector<std::vector<Seg>> segs((size_t)gyb);
    int64_t n_mixed = 0, n_r1 = 0;
    for (int i = 0; i < n; i++) {
        const int32_t *c = tab.data() + (size_t)i * rec;
        const int npx = c[0];
        n_mixed += npx;
        n_r1 += c[1];
        if (npx == 0) continue;
        const int t = list[1 + 2 * i], tx = t % gxb, ty = t / gxb;
        const uint16_t *px = reinterpret_cast<const uint16_t *>(c + mcs::kMbTabCounts);
        Seg g;
        g.lo.assign(TH, 1 << 30);
        g.hi.assign(TH, -1);
        for (int q = 0; q < npx; q++) {
            const int r = px[q] / TW, x = tx * TW + px[q] % TW;
            g.lo[r] = std::min(g.lo[r], x);
            g.hi[r] = std::max(g.hi[r], x);
        }
        int mn = 1 << 30, mx = -1;
        for (int r = 0; r < TH; r++)
            if (g.lo[r] <= g.hi[r]) mn = std::min(mn, g.lo[r]), mx = std::max(mx, g.hi[r]);
        g.x0 = mn & ~3;
        g.x1 = std::min((mx + 4) & ~3, W);
        std::vector<Seg> &row = segs[(size_t)ty];
        // (the list is in tile order; merged hulls stay within one window's output columns)
        if (!row.empty() && g.x0 <= row.back().x1 + 32 &&
            std::max(row.back().x1, g.x1) - row.back().x0 <= mcs::kSwValid) {
            Seg &b = row.back();
            b.x1 = std::max(b.x1, g.x1);
            for (int r = 0; r < TH; r++)
                b.lo[r] = std::min(b.lo[r], g.lo[r]), b.hi[r] = std::max(b.hi[r], g.hi[r]);
        } else {
            row.push_back(std::move(g));
        }
    }
    p->mb_mixed_px = n_mixed;
    p->mb_r1 = n_r1;
    // 2. runs of segments down the tile rows
    struct Run {
        int x0, x1, ty0, ty1;
        std::vector<int> seg;       // segment index per tile row ty0 .. ty1
        uint32_t owners;
    };
    std::vector<Run> runs;
    std::vector<int> open;          // runs that reached the previous tile row
    auto run_owners = [&](int x0, int x1, int ty0, int ty1) {
        return owners_in(x0 - 16, x1 + 16, ty0 * TH - 16, std::min(ty1 * TH + TH, H) + 16);
    };
    for (int ty = 0; ty < gyb; ty++) {
        std::vector<int> next;
        for (size_t gi = 0; gi < segs[(size_t)ty].size(); gi++) {
            const Seg &g = segs[(size_t)ty][gi];
            int pick = -1;
            for (size_t oi = 0; oi < open.size() && pick < 0; oi++) {
                Run &r = runs[(size_t)open[oi]];
                const int x0 = std::min(r.x0, g.x0), x1 = std::max(r.x1, g.x1);
                if (x1 - x0 > mcs::kSwValid) continue;
                if (std::max(r.x0, g.x0) > std::min(r.x1, g.x1) + 32) continue;
                const uint32_t ow = run_owners(x0, x1, r.ty0, ty);
                if (__builtin_popcount(ow) > mcs::kSwMaxOwners) continue;
                pick = open[oi];
                open.erase(open.begin() + (long)oi);
                r.x0 = x0, r.x1 = x1, r.ty1 = ty, r.owners = ow;
                r.seg.push_back((int)gi);
            }
            if (pick < 0) {
                Run r;
                r.x0 = g.x0, r.x1 = g.x1, r.ty0 = r.ty1 = ty;
                r.seg.push_back((int)gi);
                r.owners = run_owners(g.x0, g.x1, ty, ty);
                if (g.x1 - g.x0 > mcs::kSwValid || __builtin_popcount(r.owners) > mcs::kSwMaxOwners)
                    return MCS_OK;   // (a segment the window cannot hold: band pass + blend)
                runs.push_back(std::move(r));
                pick = (int)runs.size() - 1;
            }
            next.push_back(pick);
        }
        open = next;
    }
    if (runs.empty()) return MCS_OK;
    // 3. strips
    const int w1 = (W + 1) / 2, h1 = (H + 1) / 2, w2 = (w1 + 1) / 2;
    (void)h1;
    auto rf = [](int i, int n_) {
        i = i < 0 ? -i : i;
        return i >= n_ ? 2 * n_ - 2 - i : i;
    };
    auto taps = [&](int x, int n_, int *idx) {   // expand taps (reflected), count
        if ((x & 1) == 0) {
            idx[0] = rf((x >> 1) - 1, n_), idx[1] = rf(x >> 1, n_), idx[2] = rf((x >> 1) + 1, n_);
            return 3;
        }
        idx[0] = rf((x - 1) >> 1, n_), idx[1] = rf((x + 1) >> 1, n_);
        return 2;
    };
    std::vector<mcs::MbStrip> strips;
    std::vector<int> region;
    std::vector<uint8_t> skip((size_t)W * H, 0);
    int64_t desc_rows = 0, sw_px = 0;
    int max_ns = 0;
    for (const Run &r : runs) {
        mcs::MbStrip st;
        memset(&st, 0, sizeof(st));
        const int width = r.x1 - r.x0;
        st.c0 = r.x0 - mcs::kSwMargin - (((mcs::kSwValid - width) / 2) & ~3);
        st.ya = r.ty0 * TH;
        st.yb = std::min(r.ty1 * TH + TH, H);
        st.r0 = st.ya - mcs::kSwLead;
        // R0 of output row y runs in step s = (y - ya + 34) / 4 (mcs_sweep.hip phase A)
        const int last = (st.yb - 1 - st.ya + 34) / 4;
        st.nsteps = (last + 1 + 2) / 3 * 3;
        st.ns = 0;
        for (uint32_t m = r.owners; m; m &= m - 1) st.slot[st.ns++] = __builtin_ctz(m);
        if (st.ns == 0) continue;
        max_ns = std::max(max_ns, st.ns);
        st.reg = (int)region.size();
        st.dsc = (int)desc_rows;
        desc_rows += (int64_t)st.ns * (4 * st.nsteps + mcs::kSwDescPad);
        int e1lo = 1 << 30, e1hi = -1;
        for (int y = st.ya; y < st.yb; y++) {
            const Seg &g = segs[(size_t)(y / TH)][(size_t)r.seg[(size_t)(y / TH - r.ty0)]];
            const int lo = g.lo[(size_t)(y % TH)], hi = g.hi[(size_t)(y % TH)];
            int xa = 0, xb = 0;
            if (lo <= hi) {
                xa = lo & ~3;
                xb = std::min((hi + 4) & ~3, W);
            }
            region.push_back(xa | (xb << 16));
            for (int x = xa; x < xb; x++) {
                if (dense[(size_t)(y / TH) * gxb + x / TW]) return MCS_OK;
                skip[(size_t)y * W + x] = 1;
                int ix[3];
                const int nt = taps(x, w1, ix);
                for (int q = 0; q < nt; q++) e1lo = std::min(e1lo, ix[q]), e1hi = std::max(e1hi, ix[q]);
            }
            sw_px += xb - xa;
        }
        if (e1hi < 0) continue;
        int z2lo = 1 << 30, z2hi = -1;
        for (int E = e1lo; E <= e1hi; E++) {
            int iz[3];
            const int nt = taps(E, w2, iz);
            for (int q = 0; q < nt; q++) z2lo = std::min(z2lo, iz[q]), z2hi = std::max(z2hi, iz[q]);
        }
        st.e1lo = e1lo, st.e1n = e1hi - e1lo + 1, st.z2lo = z2lo, st.z2n = z2hi - z2lo + 1;
        // the window computes level-1 columns c0/2 + [1, 62] and level-2 columns c0/4 + [2, 30]
        bool ok = st.e1n <= mcs::kSwMaxR1 && st.z2n <= mcs::kSwMaxB2;
        const int c1 = st.c0 >> 1, c2 = st.c0 >> 2;
        for (int E = e1lo; E <= e1hi && ok; E++) ok = E - c1 >= 1 && E - c1 <= 62;
        for (int Z = z2lo; Z <= z2hi && ok; Z++) {
            ok = Z - c2 >= 2 && Z - c2 <= 30;
            for (int v = 0; v < 5 && ok; v++) {
                const int q = rf(2 * Z - 2 + v, w1) - c1;
                ok = q >= 1 && q <= 62;
            }
        }
        if (!ok) return MCS_OK;
        strips.push_back(st);
    }
    if (strips.empty()) return MCS_OK;
    // 4. device tables, descriptors
    const size_t ns_ = strips.size();
    HIP_TRY(A->hipMalloc((void **)&p->d_strips, ns_ * sizeof(mcs::MbStrip)));
    HIP_TRY(A->hipMalloc((void **)&p->d_region, region.size() * sizeof(int)));
    HIP_TRY(A->hipMalloc((void **)&p->d_sdesc, (size_t)desc_rows * mcs::kSwCols * 8));
    HIP_TRY(A->hipMalloc((void **)&p->d_skip, skip.size()));
    HIP_TRY(A->hipMemcpyAsync(p->d_strips, strips.data(), ns_ * sizeof(mcs::MbStrip),
                              hipMemcpyHostToDevice, s));
    HIP_TRY(A->hipMemcpyAsync(p->d_region, region.data(), region.size() * sizeof(int),
                              hipMemcpyHostToDevice, s));
    HIP_TRY(A->hipMemcpyAsync(p->d_skip, skip.data(), skip.size(), hipMemcpyHostToDevice, s));
    mcs::KMbSweepArgs a;
    memset(&a, 0, sizeof(a));
    a.P = p->kp;
    a.strips = p->d_strips;
    a.sdesc = p->d_sdesc;
    a.region = p->d_region;
    a.owner = p->d_owner;
    a.n_strips = (int)ns_;
    int rc = launch_args(A, k->mb_sweep_desc[C][p->fd.interp], (unsigned)ns_, mcs::kSwMaxOwners, 256,
                         1, &a, sizeof(a), s);
    if (rc) return rc;
    HIP_TRY(A->hipStreamSynchronize(s));
    p->kp.skip = p->d_skip;
    p->n_strips = (int)ns_;
    // (the band pass + blend's level scratch and per-tile sample windows are not used)
    for (void **q : {(void **)&p->d_mbg1, (void **)&p->d_mbg2, (void **)&p->d_mbdesc}) {
        if (*q) (void)A->hipFree(*q);
        *q = nullptr;
    }
    p->sw_jb = max_ns <= 2 ? 2 : 4;
    p->sw_px = sw_px;
    p->sw_desc_rows = desc_rows;
    return MCS_OK;
}

// Multi-band: per (tile, owner) level-0 sample windows and per-tile masks (once), and the level
// scratch for chunks of mb_chunk captures (budget kMbScratchBytes).
int prepare_multiband(const Api *A, mcs_plan *p, const Kernels *k, hipStream_t s)
{
    const int n = p->n_blend, S = p->mb_slots, C = p->fd.channels;
    const mcs::KParams &P = p->kp;
    for (int c = 0; c <= P.n_stages; c++) {
        const int64_t w = c == 0 ? P.cam0_w : P.st[c - 1].src_w;
        const int64_t h = c == 0 ? P.cam0_h : P.st[c - 1].src_h;
        if (w * h * C >= (int64_t(1) << 31))
            return mcs::fail(MCS_E_UNSUPPORTED, "multi-band: camera frames must be < 2 GiB");
    }
    const int64_t per_f = (int64_t)n * S * (mcs::kMbNRX * mcs::kMbNRY * 8 +
                                            mcs::kMbN2X * mcs::kMbN2Y * C * 4);
    int chunk = (int)std::max<int64_t>(1, std::min<int64_t>(64, mcs::kMbScratchBytes / per_f));
    if (chunk > mcs::kMbLvFrames) chunk -= chunk % mcs::kMbLvFrames;
    const int64_t samples = (int64_t)mcs::kMbUsedX * mcs::kMbUsedY;
    HIP_TRY(A->hipMalloc((void **)&p->d_mbdesc, (size_t)(n * S * samples) * sizeof(uint64_t)));
    HIP_TRY(A->hipMalloc((void **)&p->d_mbtab, (size_t)n * mcs::mb_tab_words(S) * sizeof(int32_t)));
    HIP_TRY(A->hipMalloc((void **)&p->d_mbfoot, (size_t)n * S * 8 * sizeof(int32_t)));
    HIP_TRY(A->hipMalloc((void **)&p->d_mbg1,
                         (size_t)n * S * chunk * mcs::kMbNRX * mcs::kMbNRY * 8));
    HIP_TRY(A->hipMalloc((void **)&p->d_mbg2,
                         (size_t)n * S * chunk * mcs::kMbN2X * mcs::kMbN2Y * C * 4));
    p->mb_chunk = chunk;
    mcs::KMbArgs a;
    mb_args(p, p->kp, a);
    int rc = launch_args(A, k->mb_prep[C][p->fd.interp], (unsigned)n, 1,
                         mcs::kMbPrepThreads, 1, &a, sizeof(a), s);
    if (rc) return rc;
    rc = prepare_sweep(A, p, k, s);
    if (rc || p->n_strips > 0) return rc;
    return prepare_bands(A, p, k, s);
}

// Blended modes: the owner map and the list of 32-px tiles the blend kernels recompute.
int prepare_blend(const Api *A, mcs_plan *p, const Kernels *k, hipStream_t s)
{
    const int W = p->fd.out_w, H = p->fd.out_h;
    const int bx = (W + mcs::kBlendTileW - 1) / mcs::kBlendTileW;
    const int by = (H + mcs::kBlendTileH - 1) / mcs::kBlendTileH;
    const size_t nt = (size_t)bx * by;
    HIP_TRY(A->hipMalloc((void **)&p->d_owner, (size_t)W * H));
    HIP_TRY(A->hipMalloc((void **)&p->d_binfo, nt * 2 * sizeof(uint32_t)));
    HIP_TRY(A->hipMalloc((void **)&p->d_blist, (4 * nt + 4) * sizeof(int)));
    HIP_TRY(A->hipMemsetAsync(p->d_blist, 0, (4 * nt + 4) * sizeof(int), s));
    mcs::KBlendPrepArgs a;
    a.P = p->kp;
    a.owner = p->d_owner;
    a.info = p->d_binfo;
    a.list = p->d_blist;
    a.overflow = p->d_blist + 2 * nt + 1;
    a.list2 = p->d_blist + 2 * nt + 3;
    a.mode = p->blend;
    a.pad_ = 0;
    int rc = launch_args(A, k->blend_owner[p->fd.interp], bx, by, 256, 1, &a, sizeof(a), s);
    if (rc == MCS_OK) rc = launch_args(A, k->blend_classify, (unsigned)nt, 1, 256, 1, &a,
                                       sizeof(a), s);
    if (rc) return rc;
    int n = 0, tail[3] = {0, 0, 0};
    HIP_TRY(A->hipMemcpyAsync(&n, p->d_blist, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(A->hipMemcpyAsync(tail, p->d_blist + 2 * nt + 1, 3 * sizeof(int),
                              hipMemcpyDeviceToHost, s));
    HIP_TRY(A->hipStreamSynchronize(s));
    // tail[0]: multi-band tiles with more than kBlendSlots owners (degraded to the feather rule),
    // tail[2]: those of them with pixels to feather (listed in d_dense)
    if (n > 1) {
        // the list in tile order (classify appends in arrival order)
        std::vector<int> l(1 + 2 * (size_t)n);
        HIP_TRY(A->hipMemcpyAsync(l.data(), p->d_blist, l.size() * sizeof(int),
                                  hipMemcpyDeviceToHost, s));
        HIP_TRY(A->hipStreamSynchronize(s));
        std::vector<std::pair<int, int>> e((size_t)n);
        for (int i = 0; i < n; i++) e[i] = {l[1 + 2 * i], l[2 + 2 * i]};
        std::sort(e.begin(), e.end());
        for (int i = 0; i < n; i++) l[1 + 2 * i] = e[i].first, l[2 + 2 * i] = e[i].second;
        HIP_TRY(A->hipMemcpyAsync(p->d_blist, l.data(), l.size() * sizeof(int),
                                  hipMemcpyHostToDevice, s));
        HIP_TRY(A->hipStreamSynchronize(s));
    }
    p->mb_slots = tail[1];
    p->n_degraded = p->blend == MCS_BLEND_MULTIBAND ? tail[0] : 0;
    p->n_dense = tail[2];
    p->d_dense = p->d_blist + 2 * nt + 3;
    p->n_blend = n;
    if (p->blend == MCS_BLEND_MULTIBAND && n > 0) return prepare_multiband(A, p, k, s);
    return MCS_OK;
}

// Frees the prepared tables (after a blend-mode change they are rebuilt on next use).
void release_tables(const Api *A, mcs_plan *p)
{
    if (p->stream) (void)A->hipStreamSynchronize(p->stream);
    if (p->side) (void)A->hipStreamSynchronize(p->side);
    if (p->side2) (void)A->hipStreamSynchronize(p->side2);
    for (void *q : {(void *)p->d_tiles, (void *)p->d_desc, (void *)p->d_desc4,
                    (void *)p->d_spans, (void *)p->d_fallback,
                    (void *)p->d_owner, (void *)p->d_binfo, (void *)p->d_blist,
                    (void *)p->d_mbdesc, (void *)p->d_mbtab, (void *)p->d_mbfoot, (void *)p->d_mbg1,
                    (void *)p->d_mbg2, (void *)p->d_bands, (void *)p->d_tile_bt,
                    (void *)p->d_bdesc, (void *)p->d_bgrp, (void *)p->d_bdesc16,
                    (void *)p->d_order, (void *)p->d_strips, (void *)p->d_region,
                    (void *)p->d_sdesc, (void *)p->d_skip})
        if (q) (void)A->hipFree(q);
    p->d_strips = nullptr;
    p->d_region = nullptr;
    p->d_sdesc = nullptr;
    p->d_skip = nullptr;
    p->kp.skip = nullptr;
    p->n_strips = p->sw_jb = 0;
    p->sw_px = p->sw_desc_rows = 0;
    p->d_bgrp = nullptr;
    p->d_bdesc16 = nullptr;
    p->n_bands_lds = 0;
    p->d_order = nullptr;
    p->n_early = p->n_list = 0;
    p->d_bands = nullptr;
    p->d_tile_bt = nullptr;
    p->d_bdesc = nullptr;
    p->n_bands = p->n_bands_in = p->gxb = 0;
    p->mb_mixed_px = p->mb_r1 = 0;
    p->dma_bytes = p->box_bytes = 0;
    p->d_mbdesc = nullptr;
    p->d_mbtab = nullptr;
    p->d_mbfoot = nullptr;
    p->d_mbg1 = nullptr;
    p->d_mbg2 = nullptr;
    p->mb_chunk = 0;
    p->d_tiles = nullptr;
    p->d_desc = nullptr;
    p->d_desc4 = nullptr;
    p->d_spans = nullptr;
    p->d_fallback = nullptr;
    p->d_big = nullptr;
    p->n_big = 0;
    p->d_owner = nullptr;
    p->d_binfo = nullptr;
    p->d_blist = nullptr;
    p->d_dense = nullptr;
    p->n_dense = p->n_degraded = 0;
    p->prepared = false;
    p->n_fallback = p->n_blend = 0;
}

// Cylindrical plans: the per-column / per-row table on the plan's device (once).
int ensure_cyl(const Api *A, mcs_plan *p, hipStream_t s)
{
    if (!p->map_tab.empty() && !p->d_map) {
        const size_t bytes = p->map_tab.size() * sizeof(int32_t);
        HIP_TRY(A->hipMalloc((void **)&p->d_map, bytes));
        HIP_TRY(A->hipMemcpyAsync(p->d_map, p->map_tab.data(), bytes, hipMemcpyHostToDevice, s));
        HIP_TRY(A->hipStreamSynchronize(s));
        p->kp.map_tab = p->d_map;
    }
    if (!p->cyl || p->d_cyl) return MCS_OK;
    const size_t bytes = p->cyl_tab.size() * sizeof(double);
    HIP_TRY(A->hipMalloc((void **)&p->d_cyl, bytes));
    HIP_TRY(A->hipMemcpyAsync(p->d_cyl, p->cyl_tab.data(), bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(A->hipStreamSynchronize(s));
    p->kp.cyl_tab = p->d_cyl;
    return MCS_OK;
}

// Prepared tables of a plan: one prepare launch, then the fallback-tile count is read back.
// Allocates and synchronises: call before graph capture (the stitch entry points call it lazily).
int prepare(const Api *A, mcs_plan *p, hipStream_t s)
{
    if (p->prepared) return MCS_OK;
    const Kernels *k = nullptr;
    int rc = kernels(A, p->device, &k);
    if (rc) return rc;
    p->gx = (p->fd.out_w + mcs::kTileW - 1) / mcs::kTileW;
    p->gy = (p->fd.out_h + mcs::kTileH - 1) / mcs::kTileH;
    const size_t tiles = (size_t)p->gx * p->gy;
    if (tiles == 0) {
        p->prepared = true;
        return MCS_OK;
    }
    rc = ensure_cyl(A, p, s);
    if (rc) return rc;
    if (p->blend == MCS_BLEND_FEATHER || p->blend == MCS_BLEND_MULTIBAND) {
        rc = prepare_blend(A, p, k, s);
        if (rc) return rc;
    }
    HIP_TRY(A->hipMalloc((void **)&p->d_tiles, tiles * sizeof(mcs::TileHdr)));
    HIP_TRY(A->hipMalloc((void **)&p->d_desc, tiles * mcs::kTilePx * mcs::kDescWords * 4));
    HIP_TRY(A->hipMalloc((void **)&p->d_desc4, tiles * mcs::kTilePx * 4));
    HIP_TRY(A->hipMalloc((void **)&p->d_spans, tiles * mcs::kMaxTileJobs * sizeof(uint16_t)));
    HIP_TRY(A->hipMalloc((void **)&p->d_fallback, 2 * (tiles + 1) * sizeof(int)));
    p->d_big = p->d_fallback + tiles + 1;
    HIP_TRY(A->hipMemsetAsync(p->d_fallback, 0, sizeof(int), s));
    HIP_TRY(A->hipMemsetAsync(p->d_big, 0, sizeof(int), s));
    mcs::KPrepareArgs args;
    args.P = p->kp;
    args.tiles = p->d_tiles;
    args.desc = p->d_desc;
    args.desc4 = p->d_desc4;
    args.fallback = p->d_fallback;
    args.big = p->d_big;
    args.spans = p->d_spans;
    size_t sz = sizeof(args);
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, (void *)&args, HIP_LAUNCH_PARAM_BUFFER_SIZE,
                   &sz, HIP_LAUNCH_PARAM_END};
    HIP_TRY(A->hipModuleLaunchKernel(k->prepare[p->fd.channels][p->fd.interp], p->gx, p->gy, 1,
                                     mcs::kWave, mcs::kWavesPerBlock, 1, 0, s, nullptr, cfg));
    int nf = 0, nb = 0;
    HIP_TRY(A->hipMemcpyAsync(&nf, p->d_fallback, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(A->hipMemcpyAsync(&nb, p->d_big, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(A->hipStreamSynchronize(s));
    p->n_fallback = nf;
    p->n_big = nb;
    {
        // the streaming launch's read volume per capture, from the tables just built (once)
        std::vector<mcs::TileHdr> th(tiles);
        std::vector<uint16_t> sp(tiles * mcs::kMaxTileJobs);
        HIP_TRY(A->hipMemcpyAsync(th.data(), p->d_tiles, tiles * sizeof(mcs::TileHdr),
                                  hipMemcpyDeviceToHost, s));
        HIP_TRY(A->hipMemcpyAsync(sp.data(), p->d_spans, sp.size() * sizeof(uint16_t),
                                  hipMemcpyDeviceToHost, s));
        HIP_TRY(A->hipStreamSynchronize(s));
        p->dma_bytes = p->box_bytes = 0;
        for (size_t t = 0; t < tiles; t++) {
            const mcs::TileHdr &h = th[t];
            if (h.fits == 0) continue;
            for (int k = 0; k < h.ncam; k++) {
                const int rows = h.jobstart[k + 1] - h.jobstart[k];
                p->box_bytes += (int64_t)rows * 16 * ((h.stride[k] >> 16) & 0xff);
            }
            for (int j = 0; j < h.njobs && j < mcs::kMaxTileJobs; j++)
                p->dma_bytes += 16 * (int64_t)((sp[t * mcs::kMaxTileJobs + j] >> 8) & 0xff);
        }
    }
    if (!p->d_order) {
        // one launch list of every tile (the multi-band split builds its own, early tiles first)
        std::vector<int> tl(tiles);
        for (size_t t = 0; t < tiles; t++) tl[t] = (int)t;
        const std::vector<int> order = launch_list(tl);
        HIP_TRY(A->hipMalloc((void **)&p->d_order, order.size() * sizeof(int)));
        HIP_TRY(A->hipMemcpyAsync(p->d_order, order.data(), order.size() * sizeof(int),
                                  hipMemcpyHostToDevice, s));
        HIP_TRY(A->hipStreamSynchronize(s));
        p->n_early = 0;
        p->n_list = (int)order.size();
    }
    p->prepared = true;
    return MCS_OK;
}

// Multi-band level pyramids of captures [f0, f0 + nf) on stream s: the band pass when the plan
// has one (interior and bottom / right edge bands in ONE launch, blocks below n_in interior, so
// the edge bands run beside the interior ones), else mb_levels.
int launch_mb_levels(const Api *A, const mcs_plan *p, const Kernels *k, mcs::KMbArgs &m, int f0,
                     int nf, hipStream_t s)
{
    m.f0 = f0;
    m.nf = nf;
    if (p->n_bands > 0) {
        mcs::KMbBandArgs b;
        band_args(p, m.P, b);
        b.f0 = f0;
        b.nf = nf;
        const unsigned gy = (unsigned)((nf + mcs::kMbBandFrames - 1) / mcs::kMbBandFrames);
        const int form = band_form(p, b.P);
        const int kind = p->n_bands_in == 0 ? 1 : (p->n_bands > p->n_bands_in ? 2 : 0);
        if (kind == 1) b.band0 = 0;
        return launch_args(A, k->mb_bands[p->fd.channels][form][kind],
                           xcd_grid((int64_t)p->n_bands * gy), 1, mcs::kMbBandLanes, 1, &b,
                           sizeof(b), s);
    }
    const unsigned gz = (unsigned)((nf + mcs::kMbLvFrames - 1) / mcs::kMbLvFrames);
    size_t sz = sizeof(m);
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, (void *)&m, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                   HIP_LAUNCH_PARAM_END};
    HIP_TRY(A->hipModuleLaunchKernel(k->mb_levels[p->fd.channels], (unsigned)p->n_blend,
                                     (unsigned)p->mb_slots, gz, mcs::kMbLvThreads, 1, 1, 0, s,
                                     nullptr, cfg));
    return MCS_OK;
}

// Multi-band tiles degraded to the feather rule (more than kBlendSlots owners in their
// neighbourhood): the feather kernel over d_dense, on stream s after the mosaic is written.
int launch_dense(const Api *A, const mcs_plan *p, const Kernels *k, const mcs::KParams &P,
                 int n_frames, hipStream_t s)
{
    if (p->blend != MCS_BLEND_MULTIBAND || p->n_dense <= 0) return MCS_OK;
    mcs::KBlendArgs b;
    b.P = P;
    b.owner = p->d_owner;
    b.list = p->d_dense;
    b.n_frames = n_frames;
    b.pad_ = 0;
    return launch_args(A, k->feather[p->fd.channels][p->fd.interp], p->n_dense, n_frames, 256, 1,
                       &b, sizeof(b), s);
}

// The multi-band blend kernel for the plan's owner count (<= 2, <= 4, <= 8 per neighbourhood).
int launch_mb_blend(const Api *A, const mcs_plan *p, const Kernels *k, mcs::KMbArgs &m, int f0,
                    int nf, hipStream_t s)
{
    m.f0 = f0;
    m.nf = nf;
    const int v = p->mb_slots <= 2 ? 0 : (p->mb_slots <= 4 ? 1 : 2);
    m.list0 = 0;
    m.n_list = p->n_blend;
    return launch_args(A, k->mb_blend[p->fd.channels][v], xcd_grid((int64_t)p->n_blend * nf), 1,
                       mcs::kMbBlThreads, 1, &m, sizeof(m), s);
}

// One launch (stream over all tiles, + direct over the fallback tiles, + the blend passes) for
// n_frames captures that share one frame stride.  Work that does not read the mosaic -- the
// direct-gather tiles and the first multi-band chunk's level pyramids -- runs on two side streams,
// concurrently with the HBM-bound streaming kernel.
// Capture ranges per large-footprint tile (mcs_stream_big).  Same-box C4 A/B over 1 / 2 / 4 / 8
// parts (profiles/r06_big_parts_ab.txt): the paste launch gains with more parts (0.734 -> 0.720
// ms at 8), the multi-band launch loses (1.297 -> 1.349 ms: the extra blocks take CUs from the
// band pass and blend running beside them).  MCS_BIG_PARTS overrides both.
int big_parts(bool multiband)
{
    static const int v = [] {
        const char *e = getenv("MCS_BIG_PARTS");
        const int n = e ? atoi(e) : 0;
        return n >= 1 && n <= 64 ? n : 0;
    }();
    return v ? v : multiband ? 1 : 8;
}

int launch_pair(const Api *A, const mcs_plan *p, const Kernels *k, mcs::KParams &P, int n_frames,
                hipStream_t s)
{
    // multi-band: the sweep (strips) or the band pass + blend
    const bool sweep = p->blend == MCS_BLEND_MULTIBAND && p->n_strips > 0;
    const bool mb = !sweep && p->blend == MCS_BLEND_MULTIBAND && p->n_blend > 0;
    // side work beside the main streaming launch: the large-footprint tiles and the
    // direct-gather tiles (tiles the main launch skips), on p->side
    const bool aside = p->n_fallback > 0 || p->n_big > 0;
    const bool fork = aside || mb || sweep;
    mcs::KMbArgs m;
    if (mb) mb_args(p, P, m);
    mcs::KStreamArgs args;
    args.P = P;
    const bool b32 = stream_base(p, P, n_frames, &args.P.base);
    args.tiles = p->d_tiles;
    args.desc = p->d_desc;
    args.desc4 = p->d_desc4;
    args.spans = p->d_spans;
    args.n_frames = n_frames;
    args.parts = 1;
    args.pad2_ = 0;
    if (fork) HIP_TRY(A->hipEventRecord(p->ev_fork, s));
    if (aside) HIP_TRY(A->hipStreamWaitEvent(p->side, p->ev_fork, 0));
    auto big_launch = [&](hipStream_t q) -> int {
        mcs::KStreamArgs bg = args;
        bg.order = p->d_big + 1;
        bg.n_order = p->n_big;
        // each large-footprint tile as `parts` blocks over capture ranges: one block per CU per
        // tile otherwise streams the whole batch and sets the launch's tail (C4: 31 tiles)
        bg.parts = std::max(1, std::min(big_parts(mb || sweep), n_frames));
        size_t sz = sizeof(bg);
        void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, (void *)&bg, HIP_LAUNCH_PARAM_BUFFER_SIZE,
                       &sz, HIP_LAUNCH_PARAM_END};
        HIP_TRY(A->hipModuleLaunchKernel(k->stream_big[p->fd.channels][b32 ? 1 : 0],
                                         8u * (((unsigned)(p->n_big * bg.parts) + 7u) / 8u), 1, 1,
                                         mcs::kWave,
                                         mcs::kWavesPerBlock, 1, (unsigned)mcs::kBigStreamLds, q,
                                         nullptr, cfg));
        return MCS_OK;
    };
    if (p->n_big > 0) {
        const int rc = big_launch(p->side);
        if (rc) return rc;
    }
    if (p->n_fallback > 0) {
        mcs::KDirectArgs da;
        da.P = P;
        const bool off32 = offset_base(p, da.P, &da.P.base);
        da.fallback = p->d_fallback;
        da.n_frames = n_frames;
        da.pad_ = 0;
        size_t sz = sizeof(da);
        void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, (void *)&da, HIP_LAUNCH_PARAM_BUFFER_SIZE,
                       &sz, HIP_LAUNCH_PARAM_END};
        const unsigned gy = (unsigned)((n_frames + mcs::kDirectFrames - 1) / mcs::kDirectFrames);
        HIP_TRY(A->hipModuleLaunchKernel(k->direct[p->fd.channels][p->fd.interp][off32 ? 1 : 0],
                                         p->n_fallback, gy, 1, mcs::kWave, mcs::kWavesPerBlock, 1,
                                         0, p->side, nullptr, cfg));
    }
    if (aside) HIP_TRY(A->hipEventRecord(p->ev_join, p->side));
    // split (multi-band, one scratch chunk): streaming tiles under mixed pixels first, then the
    // blend on side2 (after the band pass, those tiles and the side tiles) beside the remaining
    // streaming tiles (same-box A/B, round 2: C2 1.009 -> 0.985 ms)
    const bool split = mb && p->d_order && p->n_early > 0 && n_frames <= p->mb_chunk;
    if (sweep) {
        // the sweep writes only its regions' pixels, the streaming tiles every other pixel: the
        // two run side by side from the start, no ordering between them
        HIP_TRY(A->hipStreamWaitEvent(p->side2, p->ev_fork, 0));
        mcs::KMbSweepArgs a;
        a.P = P;
        a.strips = p->d_strips;
        a.sdesc = p->d_sdesc;
        a.region = p->d_region;
        a.owner = p->d_owner;
        a.n_strips = p->n_strips;
        a.f0 = 0;
        a.nf = n_frames;
        a.pad_ = 0;
        const int al = band_form(p, P);
        int rc = launch_args(A, k->mb_sweep[p->fd.channels][al][p->sw_jb == 4 ? 1 : 0],
                             xcd_grid((int64_t)p->n_strips * n_frames), 1,
                             (unsigned)(mcs::kSwCols * p->sw_jb), 1, &a, sizeof(a), p->side2);
        if (rc) return rc;
        HIP_TRY(A->hipEventRecord(p->ev_join2, p->side2));
    }
    if (mb) {
        HIP_TRY(A->hipStreamWaitEvent(p->side2, p->ev_fork, 0));
        int rc = launch_mb_levels(A, p, k, m, 0, std::min(p->mb_chunk, n_frames), p->side2);
        if (rc) return rc;
        if (!split) HIP_TRY(A->hipEventRecord(p->ev_join2, p->side2));
    }
    // 1-D grid dealt over the 8 XCDs; the kernel maps block -> tile (XCD-contiguous bands)
    const unsigned lds = (unsigned)mcs::lds_stream_bytes(p->fd.channels);
    auto stream_launch = [&](const int *order, int n_items) -> int {
        args.order = order;
        args.n_order = n_items;
        size_t sz = sizeof(args);
        void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, (void *)&args, HIP_LAUNCH_PARAM_BUFFER_SIZE,
                       &sz, HIP_LAUNCH_PARAM_END};
        const unsigned grid = 8u * (((unsigned)n_items + 7u) / 8u);
        HIP_TRY(A->hipModuleLaunchKernel(k->stream[p->fd.channels][b32 ? 1 : 0], grid, 1, 1,
                                         mcs::kWave, mcs::kWavesPerBlock, 1,
                                         lds, s, nullptr, cfg));
        return MCS_OK;
    };
    if (split) {
        int rc = stream_launch(p->d_order, p->n_early);
        if (rc) return rc;
        HIP_TRY(A->hipEventRecord(p->ev_early, s));
        HIP_TRY(A->hipStreamWaitEvent(p->side2, p->ev_early, 0));
        if (aside) HIP_TRY(A->hipStreamWaitEvent(p->side2, p->ev_join, 0));
        rc = launch_mb_blend(A, p, k, m, 0, n_frames, p->side2);
        if (rc) return rc;
        HIP_TRY(A->hipEventRecord(p->ev_join2, p->side2));
        if (p->n_list > p->n_early) {
            rc = stream_launch(p->d_order + p->n_early, p->n_list - p->n_early);
            if (rc) return rc;
        }
        if (aside) HIP_TRY(A->hipStreamWaitEvent(s, p->ev_join, 0));
        HIP_TRY(A->hipStreamWaitEvent(s, p->ev_join2, 0));
        return launch_dense(A, p, k, P, n_frames, s);
    }
    {
        // (d_order: the tile order of prepare / prepare_bands; NULL: row-major grid order)
        const int rc = p->d_order ? stream_launch(p->d_order, p->n_list)
                                  : stream_launch(nullptr, p->gx * p->gy);
        if (rc) return rc;
    }
    if (aside) HIP_TRY(A->hipStreamWaitEvent(s, p->ev_join, 0));
    if (mb || sweep) HIP_TRY(A->hipStreamWaitEvent(s, p->ev_join2, 0));
    if (p->n_blend > 0 && !sweep) {
        // recompute the blended tiles over the owner-sampled mosaic (same stream: ordered)
        int rc = MCS_OK;
        if (p->blend == MCS_BLEND_FEATHER) {
            mcs::KBlendArgs b;
            b.P = P;
            b.owner = p->d_owner;
            b.list = p->d_blist;
            b.n_frames = n_frames;
            b.pad_ = 0;
            rc = launch_args(A, k->feather[p->fd.channels][p->fd.interp], p->n_blend, n_frames,
                             256, 1, &b, sizeof(b), s);
        } else {
            // multi-band: per chunk of captures (scratch stride mb_chunk) levels (chunk 0's
            // already ran on the side stream) then blend
            for (int f0 = 0; f0 < n_frames && rc == MCS_OK; f0 += p->mb_chunk) {
                const int nf = std::min(p->mb_chunk, n_frames - f0);
                if (f0 > 0) rc = launch_mb_levels(A, p, k, m, f0, nf, s);
                if (rc == MCS_OK) rc = launch_mb_blend(A, p, k, m, f0, nf, s);
            }
        }
        if (rc) return rc;
    }
    return launch_dense(A, p, k, P, n_frames, s);
}

// Side streams + fork/join events for the direct-gather tiles and the multi-band levels (created
// once per plan, when needed).
int ensure_side(const Api *A, mcs_plan *p)
{
    const bool mb = p->blend == MCS_BLEND_MULTIBAND && p->n_blend > 0;
    const bool aside = p->n_fallback > 0 || p->n_big > 0;
    int least = 0, greatest = 0;
    if (aside && !p->side) HIP_TRY(A->hipDeviceGetStreamPriorityRange(&least, &greatest));
    if ((aside || mb) && !p->ev_fork)
        HIP_TRY(A->hipEventCreateWithFlags(&p->ev_fork, hipEventDisableTiming));
    if (aside && !p->side) {
        HIP_TRY(A->hipEventCreateWithFlags(&p->ev_join, hipEventDisableTiming));
        // (the least priority: a stream of its own priority level does not share a hardware
        // queue with side2, whose band pass otherwise waited behind the large-footprint tiles --
        // C4 multi-band launch 1.345-1.352 -> 1.315-1.317 ms same box, round 5)
        HIP_TRY(A->hipStreamCreateWithPriority(&p->side, hipStreamNonBlocking, least));
    }
    if (mb && !p->side2) {
        HIP_TRY(A->hipEventCreateWithFlags(&p->ev_join2, hipEventDisableTiming));
        HIP_TRY(A->hipEventCreateWithFlags(&p->ev_early, hipEventDisableTiming));
        HIP_TRY(A->hipStreamCreateWithFlags(&p->side2, hipStreamNonBlocking));
    }
    return MCS_OK;
}

// cv2.resize(INTER_LINEAR) of n_frames device images (same size: OpenCV copies).
int launch_resize(const Api *A, const Kernels *k, const uint8_t *src, int sw, int sh,
                  int64_t src_pitch, int64_t src_fstride, uint8_t *dst, int dw, int dh,
                  int64_t dst_pitch, int64_t dst_fstride, int C, int n_frames, hipStream_t s)
{
    if (sw == dw && sh == dh) {
        for (int f = 0; f < n_frames; f++)
            HIP_TRY(A->hipMemcpy2DAsync(dst + f * dst_fstride, (size_t)dst_pitch,
                                        src + f * src_fstride, (size_t)src_pitch, (size_t)dw * C,
                                        dh, hipMemcpyDeviceToDevice, s));
        return MCS_OK;
    }
    mcs::KResizeArgs a;
    a.src = src;
    a.dst = dst;
    a.src_pitch = src_pitch;
    a.src_fstride = src_fstride;
    a.dst_pitch = dst_pitch;
    a.dst_fstride = dst_fstride;
    a.scale_x = 1. / ((double)dw / sw);
    a.scale_y = 1. / ((double)dh / sh);
    a.sw = sw;
    a.sh = sh;
    a.dw = dw;
    a.dh = dh;
    a.n_frames = n_frames;
    a.area2x = a.scale_x == 2. && a.scale_y == 2.;
    size_t sz = sizeof(a);
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, (void *)&a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                   HIP_LAUNCH_PARAM_END};
    HIP_TRY(A->hipModuleLaunchKernel(k->resize[C], (dw + mcs::kResizeBlock - 1) / mcs::kResizeBlock,
                                     dh, n_frames, mcs::kResizeBlock, 1, 1, 0, s, nullptr, cfg));
    return MCS_OK;
}

int launch_stitch(const Api *A, mcs_plan *p, const mcs::KParams &kp, int n_frames, hipStream_t s)
{
    if (kp.out_w <= 0 || kp.out_h <= 0 || n_frames <= 0) return MCS_OK;
    const Kernels *k = nullptr;
    int rc = kernels(A, p->device, &k);
    if (rc) return rc;
    rc = prepare(A, p, s);
    if (rc) return rc;
    rc = ensure_side(A, p);
    if (rc) return rc;
    // the kernels walk the batch with one frame stride for every camera: split otherwise
    bool uniform = true;
    for (int j = 0; j < p->fd.n_stages; j++)
        uniform = uniform && kp.cam_fstride[p->fd.st[j].cam] == kp.cam_fstride[0];
    mcs::KParams P = kp;
    P.cyl_tab = p->kp.cyl_tab;   // set by prepare on a cylindrical plan's first use
    P.map_tab = p->kp.map_tab;   // (table plans)
    P.skip = p->kp.skip;         // (multi-band sweep plans: set by prepare)
    if (uniform) return launch_pair(A, p, k, P, n_frames, s);
    for (int f = 0; f < n_frames; f++) {
        for (int i = 0; i < p->fd.n_cams; i++)
            P.cams[i] = kp.cams[i] ? kp.cams[i] + (int64_t)f * kp.cam_fstride[i] : nullptr;
        P.out = kp.out + (int64_t)f * kp.out_fstride;
        rc = launch_pair(A, p, k, P, 1, s);
        if (rc) return rc;
    }
    return MCS_OK;
}

}  // namespace

extern "C" {

const char *mcs_version(void) { return MCS_VERSION_STRING; }

int mcs_abi_version(void) { return MCS_ABI_VERSION; }

#ifndef MCS_BUILD_ID
#define MCS_BUILD_ID "unknown"
#endif
const char *mcs_build_id(void) { return MCS_BUILD_ID; }

const char *mcs_hip_runtime(void)
{
    (void)mcs::rt::api();
    return mcs::rt::runtime_name();
}

const char *mcs_last_error(void) { return mcs::last_error(); }

int mcs_device_count(int *n)
{
    if (!n) return mcs::fail(MCS_E_INVALID, "n is NULL");
    *n = 0;
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    int c = 0;
    hipError_t e = A->hipGetDeviceCount(&c);
    if (e != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipGetDeviceCount: %s", A->hipGetErrorString(e));
    *n = c;
    return MCS_OK;
}

int mcs_plan_create(const mcs_stage_desc *stages, int n_stages, int cam0_w, int cam0_h,
                    int channels, int interp, int device, mcs_plan **out)
{
    mcs::clear_error();
    if (!stages || !out) return mcs::fail(MCS_E_INVALID, "NULL stages/out");
    *out = nullptr;
    if (device < 0 || device >= kMaxDevices) return mcs::fail(MCS_E_INVALID, "device=%d", device);
    mcs_plan *p = new (std::nothrow) mcs_plan();
    if (!p) return mcs::fail(MCS_E_NOMEM, "plan allocation");
    int rc = mcs::build_flat(stages, n_stages, cam0_w, cam0_h, channels, interp, &p->fd);
    if (rc != MCS_OK) {
        delete p;
        return rc;
    }
    mcs::fill_kparams(p->fd, &p->kp);
    p->device = device;
    *out = p;
    return MCS_OK;
}

int mcs_plan_create_cylindrical(const mcs_cyl_camera *cams, int n_cams, int out_w, int out_h,
                                double f_cyl, double u0, double v0, int channels, int interp,
                                int device, mcs_plan **out)
{
    mcs::clear_error();
    if (!cams || !out) return mcs::fail(MCS_E_INVALID, "NULL cams/out");
    *out = nullptr;
    if (device < 0 || device >= kMaxDevices) return mcs::fail(MCS_E_INVALID, "device=%d", device);
    if (n_cams < 1 || n_cams > MCS_MAX_STAGES)
        return mcs::fail(MCS_E_INVALID, "n_cams %d (1..%d)", n_cams, MCS_MAX_STAGES);
    if (channels < 1 || channels > 4) return mcs::fail(MCS_E_INVALID, "channels %d", channels);
    if (interp != MCS_INTER_NEAREST && interp != MCS_INTER_LINEAR)
        return mcs::fail(MCS_E_INVALID, "interp %d", interp);
    if (out_w < 1 || out_h < 1 || (int64_t)out_w * out_h * channels > ((int64_t)1 << 31))
        return mcs::fail(MCS_E_SHAPE, "panorama %dx%d", out_w, out_h);
    if (!(f_cyl > 0.0) || !std::isfinite(u0) || !std::isfinite(v0))
        return mcs::fail(MCS_E_INVALID, "f_cyl / u0 / v0");
    for (int c = 0; c < n_cams; c++) {
        const mcs_cyl_camera &k = cams[c];
        if (k.w < 1 || k.h < 1 || k.w > 32767 || k.h > 32767)
            return mcs::fail(MCS_E_SHAPE, "camera %d: %dx%d", c, k.w, k.h);
        bool fin = std::isfinite(k.f) && k.f > 0.0 && std::isfinite(k.cx) && std::isfinite(k.cy);
        for (double r : k.R) fin = fin && std::isfinite(r);
        if (!fin) return mcs::fail(MCS_E_INVALID, "camera %d: R / f / cx / cy", c);
    }
    mcs_plan *p = new (std::nothrow) mcs_plan();
    if (!p) return mcs::fail(MCS_E_NOMEM, "plan allocation");
    mcs_flat_desc &fd = p->fd;
    memset(&fd, 0, sizeof(fd));
    fd.n_stages = n_cams;
    fd.out_w = out_w;
    fd.out_h = out_h;
    fd.channels = channels;
    fd.interp = interp;
    fd.n_cams = n_cams;
    for (int c = 0; c < n_cams; c++) {
        fd.cam_w[c] = cams[c].w;
        fd.cam_h[c] = cams[c].h;
        mcs_flat_stage &st = fd.st[c];
        memcpy(st.minv, cams[c].R, sizeof(st.minv));   // the rotation (describe: R, not H^-1)
        st.rect[2] = out_w;
        st.rect[3] = out_h;
        st.bw0 = 1;
        st.cam = c;
    }
    mcs::fill_kparams(fd, &p->kp);
    p->kp.cam0_w = p->kp.cam0_h = 0;   // no integer-placed camera: every camera is a stage
    for (int c = 0; c < n_cams; c++) {
        mcs::KStage &k = p->kp.st[c];
        k.kind = mcs::kStageCylinder;
        k.f = cams[c].f;
        k.cx = cams[c].cx;
        k.cy = cams[c].cy;
    }
    p->cyl = true;
    p->cyl_tab.resize(2 * (size_t)out_w + out_h);
    for (int u = 0; u < out_w; u++) {
        const double t = ((double)u - u0) / f_cyl;
        p->cyl_tab[2 * u] = std::sin(t);
        p->cyl_tab[2 * u + 1] = std::cos(t);
    }
    for (int v = 0; v < out_h; v++) p->cyl_tab[2 * (size_t)out_w + v] = ((double)v - v0) / f_cyl;
    p->blend = MCS_BLEND_MULTIBAND;
    p->kp.blend = MCS_BLEND_MULTIBAND;
    p->device = device;
    *out = p;
    return MCS_OK;
}

namespace {

// Single-camera plan: stage 0 samples camera 0 everywhere (empty paste rect, paste rule).
mcs_plan *single_plan(int src_w, int src_h, int dst_w, int dst_h, int channels, int interp,
                      int device, const double *minv, int kind)
{
    mcs_plan *p = new (std::nothrow) mcs_plan();
    if (!p) return nullptr;
    mcs_flat_desc &fd = p->fd;
    memset(&fd, 0, sizeof(fd));
    fd.n_stages = 1;
    fd.out_w = dst_w;
    fd.out_h = dst_h;
    fd.channels = channels;
    fd.interp = interp;
    fd.n_cams = 1;
    fd.cam_w[0] = src_w;
    fd.cam_h[0] = src_h;
    if (minv) memcpy(fd.st[0].minv, minv, sizeof(fd.st[0].minv));
    fd.st[0].bw0 = mcs::block_width(dst_w, dst_h);
    fd.st[0].cam = 0;
    mcs::fill_kparams(fd, &p->kp);
    p->kp.cam0_w = p->kp.cam0_h = 0;
    p->kp.st[0].kind = kind;
    p->single = true;
    p->device = device;
    return p;
}

int check_single_args(int src_w, int src_h, int dst_w, int dst_h, int channels, int device)
{
    if (device < 0 || device >= kMaxDevices) return mcs::fail(MCS_E_INVALID, "device=%d", device);
    if (channels < 1 || channels > 4) return mcs::fail(MCS_E_INVALID, "channels %d", channels);
    if (src_w < 1 || src_h < 1 || src_w > 32767 || src_h > 32767)
        return mcs::fail(MCS_E_SHAPE, "source %dx%d", src_w, src_h);
    if (dst_w < 1 || dst_h < 1 || (int64_t)dst_w * dst_h * channels > ((int64_t)1 << 31))
        return mcs::fail(MCS_E_SHAPE, "destination %dx%d", dst_w, dst_h);
    return MCS_OK;
}

}  // namespace

int mcs_plan_create_warp(const double *M, int src_w, int src_h, int dst_w, int dst_h,
                         int channels, int interp, int device, mcs_plan **out)
{
    mcs::clear_error();
    if (!M || !out) return mcs::fail(MCS_E_INVALID, "NULL M/out");
    *out = nullptr;
    int rc = check_single_args(src_w, src_h, dst_w, dst_h, channels, device);
    if (rc) return rc;
    if (interp != MCS_INTER_NEAREST && interp != MCS_INTER_LINEAR)
        return mcs::fail(MCS_E_INVALID, "interp %d", interp);
    for (int i = 0; i < 9; i++)
        if (!std::isfinite(M[i])) return mcs::fail(MCS_E_INVALID, "M[%d] not finite", i);
    double minv[9];
    mcs::invert3x3_cv(M, minv);   // warpPerspective inverts M (no WARP_INVERSE_MAP)
    mcs_plan *p = single_plan(src_w, src_h, dst_w, dst_h, channels, interp, device, minv,
                              mcs::kStageHomography);
    if (!p) return mcs::fail(MCS_E_NOMEM, "plan allocation");
    *out = p;
    return MCS_OK;
}

int mcs_plan_create_undistort(const double *K, const double *dist, int n_dist, int w, int h,
                              int channels, int device, mcs_plan **out)
{
    mcs::clear_error();
    if (!K || !out || (n_dist > 0 && !dist)) return mcs::fail(MCS_E_INVALID, "NULL K/dist/out");
    *out = nullptr;
    int rc = check_single_args(w, h, w, h, channels, device);
    if (rc) return rc;
    for (int i = 0; i < 9; i++)
        if (!std::isfinite(K[i])) return mcs::fail(MCS_E_INVALID, "K[%d] not finite", i);
    std::vector<int32_t> tab(2 * (size_t)w * h);
    if (!mcs::undistort_map(K, dist, n_dist, w, h, tab.data()))
        return mcs::fail(MCS_E_UNSUPPORTED, "distortion vector of %d coefficients (0, 4, 5, 8, "
                         "12 or 14 with tau = 0)", n_dist);
    mcs_plan *p = single_plan(w, h, w, h, channels, MCS_INTER_LINEAR, device, nullptr,
                              mcs::kStageTable);
    if (!p) return mcs::fail(MCS_E_NOMEM, "plan allocation");
    p->map_tab.swap(tab);
    *out = p;
    return MCS_OK;
}

int mcs_undistort_map_host(const double *K, const double *dist, int n_dist, int w, int h,
                           int32_t *map)
{
    mcs::clear_error();
    if (!K || !map || (n_dist > 0 && !dist)) return mcs::fail(MCS_E_INVALID, "NULL K/dist/map");
    if (w < 1 || h < 1 || w > 32767 || h > 32767) return mcs::fail(MCS_E_SHAPE, "%dx%d", w, h);
    if (!mcs::undistort_map(K, dist, n_dist, w, h, map))
        return mcs::fail(MCS_E_UNSUPPORTED, "distortion vector of %d coefficients", n_dist);
    return MCS_OK;
}

int mcs_plan_destroy(mcs_plan *p)
{
    if (!p) return MCS_OK;
    bool touched = p->stream || p->d_out || p->d_tiles || p->side || p->side2;
    for (int i = 0; i < MCS_MAX_CAMS; i++) touched = touched || p->d_cams[i];
    if (touched) {
        const Api *A = mcs::rt::api();
        if (A) {
            DeviceGuard g(A, p->device);
            if (p->stream) (void)A->hipStreamSynchronize(p->stream);
            for (int i = 0; i < MCS_MAX_CAMS; i++)
                if (p->d_cams[i]) (void)A->hipFree(p->d_cams[i]);
            if (p->d_out) (void)A->hipFree(p->d_out);
            for (int i = 0; i < MCS_MAX_CAMS; i++)
                if (p->d_raw[i]) (void)A->hipFree(p->d_raw[i]);
            // every prepared table (stream, blend, multi-band, band pass, launch order): one list,
            // shared with the blend-mode change
            release_tables(A, p);
            if (p->d_cyl) (void)A->hipFree(p->d_cyl);
            if (p->d_seam) (void)A->hipFree(p->d_seam);
            if (p->d_map) (void)A->hipFree(p->d_map);
            if (p->side) (void)A->hipStreamSynchronize(p->side);
            if (p->side2) (void)A->hipStreamSynchronize(p->side2);
            if (p->stream) (void)A->hipStreamDestroy(p->stream);
            if (p->side) (void)A->hipStreamDestroy(p->side);
            if (p->side2) (void)A->hipStreamDestroy(p->side2);
            if (p->ev_fork) (void)A->hipEventDestroy(p->ev_fork);
            if (p->ev_join) (void)A->hipEventDestroy(p->ev_join);
            if (p->ev_join2) (void)A->hipEventDestroy(p->ev_join2);
            if (p->ev_early) (void)A->hipEventDestroy(p->ev_early);
        }
    }
    delete p;
    return MCS_OK;
}

int mcs_plan_out_shape(const mcs_plan *p, int *w, int *h, int *channels)
{
    if (!p) return mcs::fail(MCS_E_INVALID, "NULL plan");
    if (w) *w = p->fd.out_w;
    if (h) *h = p->fd.out_h;
    if (channels) *channels = p->fd.channels;
    return MCS_OK;
}

int mcs_plan_describe(const mcs_plan *p, mcs_flat_desc *out)
{
    if (!p || !out) return mcs::fail(MCS_E_INVALID, "NULL plan/out");
    *out = p->fd;
    return MCS_OK;
}

int mcs_stitch_host(mcs_plan *p, const uint8_t *const *cams, uint8_t *out)
{
    return mcs_stitch_host_sized(p, cams, nullptr, nullptr, out);
}

int mcs_stitch_host_sized(mcs_plan *p, const uint8_t *const *cams, const int *cam_w,
                          const int *cam_h, uint8_t *out)
{
    mcs::clear_error();
    if (!p || !cams || !out) return mcs::fail(MCS_E_INVALID, "NULL plan/cams/out");
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    const int C = p->fd.channels;
    DeviceGuard g(A, p->device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", p->device, A->hipGetErrorString(g.err));
    int rc = ensure_stream(A, p);
    if (rc) return rc;
    rc = ensure_host_buffers(A, p);
    if (rc) return rc;
    if (p->fd.out_w <= 0 || p->fd.out_h <= 0) return MCS_OK;
    const Kernels *k = nullptr;
    rc = kernels(A, p->device, &k);
    if (rc) return rc;
    // only cameras that contribute are uploaded (a passthrough stage's A is never read); a frame
    // off its calibrated size is resized on the device first (StitcherClass.py:226-233)
    bool need[MCS_MAX_CAMS];
    need_mask(p->fd, need);
    for (int i = 0; i < p->fd.n_cams; i++) {
        if (!need[i]) continue;
        if (!cams[i]) return mcs::fail(MCS_E_INVALID, "cams[%d] NULL", i);
        const int cw = p->fd.cam_w[i], ch = p->fd.cam_h[i];
        const int w = cam_w ? cam_w[i] : cw, h = cam_h ? cam_h[i] : ch;
        if (w <= 0 || h <= 0) return mcs::fail(MCS_E_INVALID, "cams[%d] size %dx%d", i, w, h);
        if (w == cw && h == ch) {
            HIP_TRY(A->hipMemcpyAsync(p->d_cams[i], cams[i], (size_t)cw * ch * C,
                                      hipMemcpyHostToDevice, p->stream));
            continue;
        }
        const size_t bytes = (size_t)w * h * C;
        if (p->raw_bytes[i] < bytes) {
            if (p->d_raw[i]) {
                HIP_TRY(A->hipStreamSynchronize(p->stream));
                HIP_TRY(A->hipFree(p->d_raw[i]));
                p->d_raw[i] = nullptr;
                p->raw_bytes[i] = 0;
            }
            HIP_TRY(A->hipMalloc((void **)&p->d_raw[i], bytes));
            p->raw_bytes[i] = bytes;
        }
        HIP_TRY(A->hipMemcpyAsync(p->d_raw[i], cams[i], bytes, hipMemcpyHostToDevice, p->stream));
        rc = launch_resize(A, k, p->d_raw[i], w, h, (int64_t)w * C, 0, p->d_cams[i], cw, ch,
                           (int64_t)cw * C, 0, C, 1, p->stream);
        if (rc) return rc;
    }
    mcs::KParams kp = p->kp;
    for (int i = 0; i < p->fd.n_cams; i++) {
        kp.cams[i] = p->d_cams[i];
        kp.cam_fstride[i] = 0;
    }
    kp.out = p->d_out;
    kp.out_pitch = p->out_pitch;
    kp.out_fstride = 0;
    rc = launch_stitch(A, p, kp, 1, p->stream);
    if (rc) return rc;
    const size_t row = (size_t)p->fd.out_w * C;
    HIP_TRY(A->hipMemcpy2DAsync(out, row, p->d_out, (size_t)p->out_pitch, row, p->fd.out_h,
                                hipMemcpyDeviceToHost, p->stream));
    HIP_TRY(A->hipStreamSynchronize(p->stream));
    return MCS_OK;
}

int mcs_resize_linear_device(const uint8_t *d_src, int src_w, int src_h, int64_t src_pitch,
                             int64_t src_frame_stride, uint8_t *d_dst, int dst_w, int dst_h,
                             int64_t dst_pitch, int64_t dst_frame_stride, int channels,
                             int n_frames, int device, void *stream)
{
    mcs::clear_error();
    if (!d_src || !d_dst) return mcs::fail(MCS_E_INVALID, "NULL src/dst");
    if (channels < 1 || channels > 4) return mcs::fail(MCS_E_UNSUPPORTED, "channels=%d", channels);
    if (src_w <= 0 || src_h <= 0 || dst_w <= 0 || dst_h <= 0)
        return mcs::fail(MCS_E_INVALID, "sizes %dx%d -> %dx%d", src_w, src_h, dst_w, dst_h);
    if (dst_h > 65535 || n_frames < 0 || n_frames > 65535)
        return mcs::fail(MCS_E_INVALID, "dst_h=%d n_frames=%d", dst_h, n_frames);
    if (src_pitch < (int64_t)src_w * channels || dst_pitch < (int64_t)dst_w * channels)
        return mcs::fail(MCS_E_INVALID, "pitch smaller than a row");
    if (n_frames == 0) return MCS_OK;
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    DeviceGuard g(A, device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", device, A->hipGetErrorString(g.err));
    const Kernels *k = nullptr;
    int rc = kernels(A, device, &k);
    if (rc) return rc;
    const int64_t sfs = src_frame_stride ? src_frame_stride : src_pitch * src_h;
    const int64_t dfs = dst_frame_stride ? dst_frame_stride : dst_pitch * dst_h;
    return launch_resize(A, k, d_src, src_w, src_h, src_pitch, sfs, d_dst, dst_w, dst_h, dst_pitch,
                         dfs, channels, n_frames, (hipStream_t)stream);
}

// Kernel parameters of a device-resident batch (mcs_stitch_device / mcs_stitch_direct).
static int device_kparams(const mcs_plan *p, const uint8_t *const *d_cams,
                          const int64_t *cam_frame_stride, uint8_t *d_out, int64_t out_pitch,
                          int64_t out_frame_stride, int n_frames, mcs::KParams *kp)
{
    if (!p || !d_cams || !d_out) return mcs::fail(MCS_E_INVALID, "NULL plan/d_cams/d_out");
    if (n_frames < 0 || n_frames > 65535) return mcs::fail(MCS_E_INVALID, "n_frames=%d", n_frames);
    const int C = p->fd.channels;
    if (out_pitch < (int64_t)p->fd.out_w * C)
        return mcs::fail(MCS_E_INVALID, "out_pitch %lld < row bytes %lld", (long long)out_pitch,
                         (long long)p->fd.out_w * C);
    *kp = p->kp;
    bool need[MCS_MAX_CAMS];
    need_mask(p->fd, need);
    for (int i = 0; i < p->fd.n_cams; i++) {
        if (need[i] && !d_cams[i]) return mcs::fail(MCS_E_INVALID, "d_cams[%d] NULL", i);
        kp->cams[i] = d_cams[i];
        kp->cam_fstride[i] = cam_frame_stride ? cam_frame_stride[i]
                                              : (int64_t)p->fd.cam_w[i] * p->fd.cam_h[i] * C;
    }
    kp->out = d_out;
    kp->out_pitch = out_pitch;
    kp->out_fstride = out_frame_stride ? out_frame_stride : out_pitch * p->fd.out_h;
    return MCS_OK;
}

int mcs_stitch_device(mcs_plan *p, const uint8_t *const *d_cams, const int64_t *cam_frame_stride,
                      uint8_t *d_out, int64_t out_pitch, int64_t out_frame_stride, int n_frames,
                      void *stream)
{
    mcs::KParams kp;
    int rc = device_kparams(p, d_cams, cam_frame_stride, d_out, out_pitch, out_frame_stride,
                            n_frames, &kp);
    if (rc) return rc;
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    DeviceGuard g(A, p->device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", p->device, A->hipGetErrorString(g.err));
    return launch_stitch(A, p, kp, n_frames, (hipStream_t)stream);
}

int mcs_stitch_direct(mcs_plan *p, const uint8_t *const *d_cams, const int64_t *cam_frame_stride,
                      uint8_t *d_out, int64_t out_pitch, int64_t out_frame_stride, int n_frames,
                      void *stream)
{
    mcs::KParams kp;
    int rc = device_kparams(p, d_cams, cam_frame_stride, d_out, out_pitch, out_frame_stride,
                            n_frames, &kp);
    if (rc) return rc;
    if (p->blend != MCS_BLEND_NONE && p->blend != MCS_BLEND_SEAM)
        return mcs::fail(MCS_E_UNSUPPORTED, "mcs_stitch_direct renders paste / seam plans; "
                         "blended plans need their prepared tables (mcs_stitch_device)");
    if (kp.out_w <= 0 || kp.out_h <= 0 || n_frames == 0) return MCS_OK;
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    DeviceGuard g(A, p->device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", p->device, A->hipGetErrorString(g.err));
    const Kernels *k = nullptr;
    rc = kernels(A, p->device, &k);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    rc = ensure_cyl(A, p, s);   // (cylinder / table plans: their device tables, once)
    if (rc) return rc;
    kp.cyl_tab = p->kp.cyl_tab;
    kp.map_tab = p->kp.map_tab;
    kp.seam_hint = p->kp.seam_hint;
    const int gx = (p->fd.out_w + mcs::kTileW - 1) / mcs::kTileW;
    const int gy = (p->fd.out_h + mcs::kTileH - 1) / mcs::kTileH;
    // one frame stride for every camera per launch (the kernel's walk), else frame by frame
    bool uniform = true;
    for (int j = 0; j < p->fd.n_stages; j++)
        uniform = uniform && kp.cam_fstride[p->fd.st[j].cam] == kp.cam_fstride[0];
    const int runs = uniform ? 1 : n_frames;
    for (int f = 0; f < runs; f++) {
        mcs::KDirectArgs args;
        args.P = kp;
        if (!uniform) {
            for (int i = 0; i < p->fd.n_cams; i++)
                args.P.cams[i] = kp.cams[i] ? kp.cams[i] + (int64_t)f * kp.cam_fstride[i] : nullptr;
            args.P.out = kp.out + (int64_t)f * kp.out_fstride;
        }
        const bool off32 = offset_base(p, args.P, &args.P.base);
        args.fallback = nullptr;   // every tile
        args.n_frames = uniform ? n_frames : 1;
        args.pad_ = 0;
        const unsigned fy = (unsigned)((args.n_frames + mcs::kDirectFrames - 1) / mcs::kDirectFrames);
        size_t sz = sizeof(args);
        void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, (void *)&args, HIP_LAUNCH_PARAM_BUFFER_SIZE,
                       &sz, HIP_LAUNCH_PARAM_END};
        HIP_TRY(A->hipModuleLaunchKernel(k->direct[p->fd.channels][p->fd.interp][off32 ? 1 : 0],
                                         (unsigned)(gx * gy), fy, 1, mcs::kWave,
                                         mcs::kWavesPerBlock, 1, 0, s, nullptr, cfg));
    }
    return MCS_OK;
}

int mcs_plan_prepare(mcs_plan *p, void *stream)
{
    if (!p) return mcs::fail(MCS_E_INVALID, "NULL plan");
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    if (p->fd.out_w <= 0 || p->fd.out_h <= 0) return MCS_OK;
    DeviceGuard g(A, p->device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", p->device, A->hipGetErrorString(g.err));
    hipStream_t s = (hipStream_t)stream;
    if (!s) {
        int rc = ensure_stream(A, p);
        if (rc) return rc;
        s = p->stream;
    }
    return prepare(A, p, s);
}

int mcs_plan_set_blend(mcs_plan *p, int mode)
{
    mcs::clear_error();
    if (!p) return mcs::fail(MCS_E_INVALID, "NULL plan");
    if (mode != MCS_BLEND_NONE && mode != MCS_BLEND_FEATHER && mode != MCS_BLEND_MULTIBAND &&
        mode != MCS_BLEND_SEAM)
        return mcs::fail(MCS_E_INVALID, "blend mode %d", mode);
    if (p->single && mode != MCS_BLEND_NONE)
        return mcs::fail(MCS_E_INVALID, "a single-camera remap plan (warp / undistort) has "
                         "nothing to blend: blend mode NONE only");
    if (p->cyl && mode == MCS_BLEND_NONE)
        return mcs::fail(MCS_E_INVALID, "a cylindrical plan has no paste order: blend mode "
                         "NONE is not defined for it (use SEAM, FEATHER or MULTIBAND)");
    if (mode == p->blend) return MCS_OK;
    if (p->prepared) {
        const Api *A = mcs::rt::api();
        if (!A) return MCS_E_HIP;
        DeviceGuard g(A, p->device);
        release_tables(A, p);
    }
    p->blend = mode;
    p->kp.blend = mode;
    return MCS_OK;
}

int mcs_plan_find_seams(mcs_plan *p, const uint8_t *const *cams, int method, int scale_log2)
{
    mcs::clear_error();
    if (!p) return mcs::fail(MCS_E_INVALID, "NULL plan");
    for (int64_t &v : p->seam_stats) v = 0;   // (only the device max-flow fills them in)
    if (method != MCS_SEAM_DISTANCE && method != MCS_SEAM_GRAPHCUT)
        return mcs::fail(MCS_E_INVALID, "seam method %d", method);
    if (method == MCS_SEAM_GRAPHCUT && (!cams || scale_log2 < 0 || scale_log2 > 4))
        return mcs::fail(MCS_E_INVALID, "graph-cut seams need cams and scale_log2 in 0..4");
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    DeviceGuard g(A, p->device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", p->device, A->hipGetErrorString(g.err));
    release_tables(A, p);
    if (p->d_seam) (void)A->hipFree(p->d_seam);
    p->d_seam = nullptr;
    p->kp.seam_hint = nullptr;
    p->seam_lab.clear();
    p->seam_w = p->seam_h = p->seam_k = 0;
    if (method == MCS_SEAM_DISTANCE || p->fd.out_w <= 0 || p->fd.out_h <= 0) return MCS_OK;
    int rc = ensure_stream(A, p);
    if (rc == MCS_OK) rc = ensure_host_buffers(A, p);
    if (rc == MCS_OK) rc = ensure_cyl(A, p, p->stream);
    const Kernels *k = nullptr;
    if (rc == MCS_OK) rc = kernels(A, p->device, &k);
    if (rc) return rc;
    const int C = p->fd.channels, n = p->fd.n_cams;
    for (int i = 0; i < n; i++) {
        if (!cams[i]) return mcs::fail(MCS_E_INVALID, "NULL cams[%d]", i);
        HIP_TRY(A->hipMemcpyAsync(p->d_cams[i], cams[i],
                                  (size_t)p->fd.cam_w[i] * p->fd.cam_h[i] * C,
                                  hipMemcpyHostToDevice, p->stream));
    }
    const int kk = scale_log2;
    const int gw = (p->fd.out_w + (1 << kk) - 1) >> kk, gh = (p->fd.out_h + (1 << kk) - 1) >> kk;
    const size_t np = (size_t)gw * gh;
    mcs::KSeamArgs a;
    memset(&a, 0, sizeof(a));
    a.P = p->kp;
    for (int i = 0; i < n; i++) {
        a.P.cams[i] = p->d_cams[i];
        a.P.cam_fstride[i] = 0;
    }
    a.gw = gw;
    a.gh = gh;
    a.k = kk;
    std::vector<uint8_t> lab(np), smp;   // (smp: host Dinic only)
    std::vector<uint16_t> cov(np);
    hipError_t e = A->hipMalloc((void **)&a.label, np);
    if (e == hipSuccess) e = A->hipMalloc((void **)&a.cov, np * sizeof(uint16_t));
    if (e == hipSuccess) e = A->hipMalloc((void **)&a.samples, np * C * n);
    if (e == hipSuccess) e = A->hipMemsetAsync(a.samples, 0, np * C * n, p->stream);
    if (e == hipSuccess) {
        rc = launch_args(A, k->seam_sample[C][p->fd.interp], (unsigned)((np + 255) / 256), 1,
                         256, 1, &a, sizeof(a), p->stream);
        if (rc) e = hipErrorLaunchFailure;
    }
    // the pairwise cuts: push-relabel on the device (default), or the host Dinic
    // (MCS_SEAM_FLOW=host; the checker of the device path)
    static const bool host_flow =
        getenv("MCS_SEAM_FLOW") && !strcmp(getenv("MCS_SEAM_FLOW"), "host");
    if (e == hipSuccess)
        e = A->hipMemcpyAsync(cov.data(), a.cov, np * 2, hipMemcpyDeviceToHost, p->stream);
    if (host_flow) {
        if (e == hipSuccess)
            e = A->hipMemcpyAsync(lab.data(), a.label, np, hipMemcpyDeviceToHost, p->stream);
        smp.resize(np * C * n);
        if (e == hipSuccess)
            e = A->hipMemcpyAsync(smp.data(), a.samples, np * C * n, hipMemcpyDeviceToHost,
                                  p->stream);
    }
    if (e == hipSuccess) e = A->hipStreamSynchronize(p->stream);
    if (e == hipSuccess && rc == MCS_OK) {
        if (host_flow) {
            rc = mcs::seam_graphcut(n, gw, gh, lab.data(), cov.data(), smp.data(), C);
            if (rc == MCS_OK)
                e = A->hipMemcpyAsync(a.label, lab.data(), np, hipMemcpyHostToDevice, p->stream);
        } else {
            rc = mcs::seam_graphcut_device(p->device, p->stream, n, gw, gh, a.label, a.cov,
                                           a.samples, C, cov.data(), p->seam_stats);
            if (rc == MCS_OK)
                e = A->hipMemcpyAsync(lab.data(), a.label, np, hipMemcpyDeviceToHost, p->stream);
        }
        if (e == hipSuccess) e = A->hipStreamSynchronize(p->stream);
    }
    for (void *q : {(void *)a.cov, (void *)a.samples})
        if (q) (void)A->hipFree(q);
    if (rc || e != hipSuccess) {
        if (a.label) (void)A->hipFree(a.label);
        if (rc) return rc;
        return mcs::fail(MCS_E_HIP, "seam finding: %s", A->hipGetErrorString(e));
    }
    p->d_seam = a.label;   // the device labels (the seam grid the stitch kernels read)
    p->seam_lab.swap(lab);
    p->seam_w = gw;
    p->seam_h = gh;
    p->seam_k = kk;
    p->kp.seam_hint = p->d_seam;
    p->kp.seam_w = gw;
    p->kp.seam_shift = kk;
    return MCS_OK;
}

int mcs_seam_graphcut_host(int n_cams, int gw, int gh, uint8_t *labels, const uint16_t *cover,
                           const uint8_t *samples, int channels)
{
    mcs::clear_error();
    if (!labels || !cover || !samples) return mcs::fail(MCS_E_INVALID, "NULL input");
    if (n_cams < 1 || n_cams > 16 || gw < 1 || gh < 1 || channels < 1 || channels > 4 ||
        (int64_t)gw * gh > (int64_t)1 << 28)
        return mcs::fail(MCS_E_INVALID, "n_cams %d, grid %dx%d, channels %d", n_cams, gw, gh,
                         channels);
    return mcs::seam_graphcut(n_cams, gw, gh, labels, cover, samples, channels);
}

int mcs_seam_graphcut_device(int n_cams, int gw, int gh, uint8_t *labels, const uint16_t *cover,
                             const uint8_t *samples, int channels, int device, int64_t *stats)
{
    mcs::clear_error();
    if (!labels || !cover || !samples) return mcs::fail(MCS_E_INVALID, "NULL input");
    if (n_cams < 1 || n_cams > 16 || gw < 1 || gh < 1 || channels < 1 || channels > 4 ||
        (int64_t)gw * gh > (int64_t)1 << 28)
        return mcs::fail(MCS_E_INVALID, "n_cams %d, grid %dx%d, channels %d", n_cams, gw, gh,
                         channels);
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    DeviceGuard g(A, device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", device, A->hipGetErrorString(g.err));
    const size_t np = (size_t)gw * gh, sb = np * n_cams * channels;
    uint8_t *buf = nullptr;
    hipStream_t s = nullptr;
    HIP_TRY(A->hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipError_t e = A->hipMalloc((void **)&buf, np * 3 + sb + 16);
    uint8_t *d_lab = buf, *d_smp = buf + np * 3 + 16;
    uint16_t *d_cov = reinterpret_cast<uint16_t *>(buf + ((np + 7) & ~(size_t)7));
    if (e == hipSuccess) e = A->hipMemcpyAsync(d_lab, labels, np, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = A->hipMemcpyAsync(d_cov, cover, np * 2, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = A->hipMemcpyAsync(d_smp, samples, sb, hipMemcpyHostToDevice, s);
    int rc = MCS_OK;
    if (e == hipSuccess)
        rc = mcs::seam_graphcut_device(device, s, n_cams, gw, gh, d_lab, d_cov, d_smp, channels,
                                       cover, stats);
    if (e == hipSuccess && rc == MCS_OK)
        e = A->hipMemcpyAsync(labels, d_lab, np, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = A->hipStreamSynchronize(s);
    (void)A->hipStreamSynchronize(s);
    if (buf) (void)A->hipFree(buf);
    (void)A->hipStreamDestroy(s);
    if (rc) return rc;
    if (e != hipSuccess) return mcs::fail(MCS_E_HIP, "seam graph cut: %s", A->hipGetErrorString(e));
    return MCS_OK;
}

int mcs_plan_seam_stats(const mcs_plan *p, int64_t *stats)
{
    if (!p || !stats) return mcs::fail(MCS_E_INVALID, "NULL plan/stats");
    for (int j = 0; j < 5; j++) stats[j] = p->seam_stats[j];
    return MCS_OK;
}

int mcs_plan_seam_labels(const mcs_plan *p, uint8_t *out, int *w, int *h)
{
    if (!p) return mcs::fail(MCS_E_INVALID, "NULL plan");
    if (w) *w = p->seam_w;
    if (h) *h = p->seam_h;
    if (out && !p->seam_lab.empty()) memcpy(out, p->seam_lab.data(), p->seam_lab.size());
    return MCS_OK;
}

int mcs_plan_stats(const mcs_plan *p, int64_t *stats, int n)
{
    if (!p || !stats) return mcs::fail(MCS_E_INVALID, "NULL plan/stats");
    const int64_t tiles = (int64_t)p->gx * p->gy;
    const int64_t v[20] = {p->prepared ? 1 : 0, tiles, tiles - p->n_fallback, p->n_fallback,
                           tiles * (int64_t)(sizeof(mcs::TileHdr) +
                                             mcs::kTilePx * (mcs::kDescWords + 1) * 4),
                           p->blend, p->n_blend, p->mb_slots, p->n_degraded, p->n_bands,
                           p->n_bands_lds, p->n_big, p->mb_mixed_px, p->mb_r1,
                           p->dma_bytes, p->box_bytes, p->n_strips, p->sw_px,
                           (int64_t)mcs::kSwCols * p->sw_jb, p->sw_desc_rows};
    for (int i = 0; i < n; i++) stats[i] = i < 20 ? v[i] : 0;
    return MCS_OK;
}

int mcs_plan_footprint(mcs_plan *p, int64_t *touched_px, int n_cams)
{
    if (!p || !touched_px) return mcs::fail(MCS_E_INVALID, "NULL plan/touched_px");
    if (n_cams < p->fd.n_cams)
        return mcs::fail(MCS_E_INVALID, "n_cams %d < %d", n_cams, p->fd.n_cams);
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    DeviceGuard g(A, p->device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", p->device, A->hipGetErrorString(g.err));
    int rc = ensure_stream(A, p);
    if (rc) return rc;
    const Kernels *k = nullptr;
    rc = kernels(A, p->device, &k);
    if (rc) return rc;
    rc = ensure_cyl(A, p, p->stream);
    if (rc) return rc;
    const int n = p->fd.n_cams;
    uint8_t *masks[MCS_MAX_CAMS] = {};
    uint8_t **d_masks = nullptr;
    unsigned long long *d_counts = nullptr;
    unsigned long long counts[MCS_MAX_CAMS] = {};
    hipError_t e = hipSuccess;
    for (int i = 0; i < n && e == hipSuccess; i++) {
        const size_t bytes = ((size_t)p->fd.cam_w[i] * p->fd.cam_h[i] + 3) / 4 * 4;
        e = A->hipMalloc((void **)&masks[i], bytes > 0 ? bytes : 4);
        if (e == hipSuccess) e = A->hipMemsetAsync(masks[i], 0, bytes > 0 ? bytes : 4, p->stream);
    }
    if (e == hipSuccess) e = A->hipMalloc((void **)&d_masks, sizeof(masks));
    if (e == hipSuccess) e = A->hipMalloc((void **)&d_counts, sizeof(counts));
    if (e == hipSuccess)
        e = A->hipMemcpyAsync(d_masks, masks, sizeof(masks), hipMemcpyHostToDevice, p->stream);
    if (e == hipSuccess) e = A->hipMemsetAsync(d_counts, 0, sizeof(counts), p->stream);
    if (e == hipSuccess && p->fd.out_w > 0 && p->fd.out_h > 0) {
        mcs::KFootprintArgs args;
        args.P = p->kp;
        args.masks = d_masks;
        args.counts = d_counts;
        size_t sz = sizeof(args);
        void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, (void *)&args, HIP_LAUNCH_PARAM_BUFFER_SIZE,
                       &sz, HIP_LAUNCH_PARAM_END};
        e = A->hipModuleLaunchKernel(k->footprint[p->fd.interp], (p->fd.out_w + 255) / 256,
                                     p->fd.out_h, 1, 256, 1, 1, 0, p->stream, nullptr, cfg);
    }
    if (e == hipSuccess)
        e = A->hipMemcpyAsync(counts, d_counts, sizeof(counts), hipMemcpyDeviceToHost, p->stream);
    if (e == hipSuccess) e = A->hipStreamSynchronize(p->stream);
    for (int i = 0; i < n; i++)
        if (masks[i]) (void)A->hipFree(masks[i]);
    if (d_masks) (void)A->hipFree(d_masks);
    if (d_counts) (void)A->hipFree(d_counts);
    if (e != hipSuccess) return mcs::fail(MCS_E_HIP, "footprint: %s", A->hipGetErrorString(e));
    for (int i = 0; i < n_cams; i++) touched_px[i] = i < n ? (int64_t)counts[i] : 0;
    return MCS_OK;
}

// Test hook (not in mcs.h): force the 64-bit-address kernel variants.
void mcs__force_off64(int on) { g_force_off64 = on; }

}  // extern "C"
