// mcs_kparams.h -- kernel parameter block shared by the host code (g++) and the gfx950 kernels
// (hipcc, device-only).  Plain C++: no HIP headers.
#pragma once

#include <stdint.h>

#include "mcs.h"

namespace mcs {

// One calibrated stage of the flattened chain (see mcs_plan.cpp).  Passed by value in the
// kernarg segment, so every field is read with wave-uniform scalar loads.
struct KStage {
    double m[9];              // OpenCV-inverted stage matrix
    int rx0, ry0, rx1, ry1;   // paste rect of B in output coords
    int offx, offy;           // output -> canvas coords
    int bw0;                  // OpenCV WarpPerspectiveInvoker block width
    int bw_shift;             // log2(bw0) when bw0 is a power of two, else -1
    int cam;                  // camera sampled by this stage
    int src_w, src_h;         // its size
    int kind;                 // kStageHomography (m = inverted H), kStageCylinder (m = R),
                              // kStageTable (map_tab)
    double f, cx, cy;         // kStageCylinder: pinhole intrinsics of the camera
};

constexpr int kStageHomography = 0;
constexpr int kStageCylinder = 1;
constexpr int kStageTable = 2;    // per-output-pixel map (KParams.map_tab), e.g. undistortion

struct KParams {
    int n_stages;
    int out_w, out_h;
    int cam0_offx, cam0_offy;
    int cam0_w, cam0_h;
    int blend;                     // MCS_BLEND_*: which camera owns a pixel (paste or blend rule)
    // Cylinder plans: (sin theta, cos theta) per output column, then h per output row (computed
    // once on the host, so that device and oracle share every transcendental value bit for bit)
    const double *cyl_tab;
    // Graph-cut seam labels (mcs_plan_find_seams): camera per point of the 2^seam_shift grid,
    // 255 = none; NULL = distance seams only
    const uint8_t *seam_hint;
    int seam_w, seam_shift;
    // kStageTable plans: map value (bilinear fixed point) of every output pixel, x then y
    const int32_t *map_tab;
    // Multi-band sweep plans (mcs_sweep.hip): 1 for every mosaic pixel the sweep kernel writes --
    // the streaming / direct kernels skip those pixels (no footprint, no store); NULL = none
    const uint8_t *skip;
    const uint8_t *cams[MCS_MAX_CAMS];
    int64_t cam_fstride[MCS_MAX_CAMS];
    uint8_t *out;
    int64_t out_pitch;
    int64_t out_fstride;
    // Common base of the used camera buffers: when every byte of frame 0 of every used camera
    // lies in [base, base + 4 GiB), pixels address their taps as base + f*fstride + u32 offset
    // (SGPR base, VGPR offset); otherwise base is NULL and offsets are full 64-bit addresses.
    const uint8_t *base;
    int cam_w[MCS_MAX_CAMS], cam_h[MCS_MAX_CAMS];   // sizes of every camera (sorted-label order)
    KStage st[MCS_MAX_STAGES];
};

// Kernarg block of the footprint kernel: (KParams, uint8_t* const* masks, u64* counts).
struct KFootprintArgs {
    KParams P;
    uint8_t *const *masks;
    unsigned long long *counts;
};

// Tiling of the stitch kernel (host and device share it): a block is 8 waves; a wave covers
// kRowsPerWave output rows of kWave / kRowsPerWave lanes, 4 consecutive pixels per lane.  Taller
// tiles re-fetch fewer source rows (the footprints of vertically adjacent tiles overlap by the
// bilinear row and the homography's slant); tools/footprint_model.py.
#ifndef MCS_ROWS_PER_WAVE
#define MCS_ROWS_PER_WAVE 2
#endif
constexpr int kPx = 4;             // output pixels per lane
constexpr int kWave = 64;
constexpr int kWavesPerBlock = 8;
constexpr int kRowsPerWave = MCS_ROWS_PER_WAVE;
constexpr int kLanesPerRow = kWave / kRowsPerWave;
constexpr int kTileW = kPx * kLanesPerRow;
constexpr int kTileH = kWavesPerBlock * kRowsPerWave;

// Prepared per-plan tables (mcs_plan_prepare): one TileHdr per tile, and per pixel of the
// tile three u32 -- the LDS byte addresses of its two row windows (16 bits each) and the packed
// u16 weight pairs (w00, w01), (w10, w11) -- stored thread-major so each lane loads its 4 pixels
// as 48 contiguous bytes.
constexpr int kTileCams = 4;       // cameras one LDS tile may draw from
constexpr int kTilePx = kTileW * kTileH;
constexpr int kDescWords = 3;

// Compact per-pixel word the streaming kernel loads (4 B instead of 12): bits 0-15 the row-0
// window's LDS address, 16-20 fx, 21-25 fy, 26-27 the camera's footprint slot in the tile header;
// flags below.  A "plain" pixel (all taps in the image) has the weights of (fx, fy) and its row-1
// window one footprint row further; other pixels (frame edges) read the full 12-byte form.
constexpr uint32_t kCwLastRow1 = 1u << 28;   // row 1 is the frame's last row (+ its DMA shift)
constexpr uint32_t kCwZero = 1u << 29;       // no live tap (no camera): output 0
constexpr uint32_t kCwFull = 1u << 30;       // read the full form
constexpr uint32_t kCwOneRow = 1u << 31;     // fy = 0: row 1 unused (= row 0)
constexpr uint32_t kCwSkip = 0xffffffffu;    // (all four words) the lane's pixels belong to the
                                             // multi-band sweep: no footprint, no store
struct TileHdr {
    int fits;                      // 1: LDS path, 2: the large-footprint LDS path (mcs_stream_big),
                                   // 0: listed for the direct-gather launch
    int ncam, njobs, ring, buf_bytes;
    // stride[k]: LDS row pitch (bits 0-15) | 16-byte DMA chunks per row (bits 16-23)
    int cam[kTileCams], rmin[kTileCams], cal[kTileCams], stride[kTileCams], base[kTileCams];
    int jobstart[kTileCams + 1];
    // per camera slot k, byte k: how far the DMA of the camera frame's LAST row starts earlier
    // than cal, so its last 16-byte chunk ends at the frame end (0: no shift); pixels reading
    // that row add it to their LDS window address
    int last_shift;
    int pad_;
};
static_assert(sizeof(TileHdr) == 128, "TileHdr layout");

// Kernarg blocks.
// Per footprint row (DMA job j of a tile, kMaxTileJobs per tile): the 16-byte chunks of its LDS
// row that any pixel window reads -- first chunk (bits 0-7) | chunk count (bits 8-15, >= 1: every
// job issues exactly one DMA instruction, which the counted vmcnt waits rely on).  A footprint is
// the box of its rows x the union of their byte spans; where the map curves (a cylinder's rows
// through a camera) each row needs only part of the box's width.
constexpr int kMaxTileJobs = 128;
struct KPrepareArgs {
    KParams P;
    TileHdr *tiles;
    uint32_t *desc;
    uint32_t *desc4;               // compact words (kCw*), 4 per lane
    int *fallback;                 // [0] = count, then tile indices (direct-gather tiles)
    int *big;                      // [0] = count, then tile indices (large-footprint tiles)
    uint16_t *spans;               // [tiles][kMaxTileJobs] row spans
};
struct KStreamArgs {
    KParams P;
    const TileHdr *tiles;
    const uint32_t *desc;
    const uint32_t *desc4;
    const uint16_t *spans;         // [tiles][kMaxTileJobs] row spans
    int n_frames;
    int parts;                     // launch-list item = (tile, capture range 1 / parts of the batch)
    const int *order;              // tiles to stream (NULL: all, in grid order)
    int n_order;                   // tiles in this launch
    int pad2_;
};
struct KDirectArgs {
    KParams P;
    const int *fallback;
    int n_frames;
    int pad_;
};

// cv2.resize(INTER_LINEAR) pre-pass (StitcherClass.py:226-233): n_frames images per launch.
struct KResizeArgs {
    const uint8_t *src;
    uint8_t *dst;
    int64_t src_pitch, src_fstride, dst_pitch, dst_fstride;
    double scale_x, scale_y;       // 1. / ((double)dst / src), as OpenCV computes them
    int sw, sh, dw, dh;
    int n_frames;
    int area2x;                    // exact 2x downscale: OpenCV switches to INTER_AREA's 2x2 mean
};
constexpr int kResizeBlock = 256;

// Blended modes (mcs_blend.h): 32 x 64 output tiles (tall: the seams of a horizontal rig run
// vertically, so a tall tile shares its pyramid rows), 16-px pyramid halo, <= 4 owners per
// multi-band neighbourhood (more: the tile takes the feather rule), owner map byte 255 = no
// camera.
#ifndef MCS_BLEND_TILE_H
#define MCS_BLEND_TILE_H 64
#endif
constexpr int kBlendTileW = 32;
constexpr int kBlendTileH = MCS_BLEND_TILE_H;
constexpr int kBlendHalo = 16;
// most owners in one multi-band neighbourhood (blend kernels for <= 2, <= 4 and <= 8)
constexpr int kBlendSlots = 8;
constexpr int kBlendNone = 255;
// multi-band kernels (mcs_blend.h): prep once per plan, then per chunk of captures levels + blend
constexpr int kMbPrepThreads = 256;
#ifndef MCS_MB_LV_THREADS
#define MCS_MB_LV_THREADS 512
#endif
constexpr int kMbLvThreads = MCS_MB_LV_THREADS;
#ifndef MCS_MB_LV_FRAMES
#define MCS_MB_LV_FRAMES 8
#endif
constexpr int kMbLvFrames = MCS_MB_LV_FRAMES;   // captures per levels block (sample windows held
                                                // in registers)
#ifndef MCS_MB_BL_THREADS
#define MCS_MB_BL_THREADS 256
#endif
constexpr int kMbBlThreads = MCS_MB_BL_THREADS;
constexpr int64_t kMbScratchBytes = 1ll << 30;    // level scratch budget per plan (<= 64 captures)
// The pyramid arrays a tile holds, per axis (tile side T): level 0 [O - 14, O + T + 10]
// (T + 25), level 1 [O/2 - 6, O/2 + T/2 + 4] (T/2 + 11), level 2 [O/4 - 2, O/4 + T/4 + 1]
// (T/4 + 4), the collapsed level 1 ("R1 region") [O/2 - 1, O/2 + T/2] (T/2 + 2).
constexpr int kMbUsedX = kBlendTileW + 25, kMbUsedY = kBlendTileH + 25;
constexpr int kMbFirst = 2;        // level-0 array origin: O - kBlendHalo + kMbFirst
constexpr int kMbN1X = kBlendTileW / 2 + 11, kMbN1Y = kBlendTileH / 2 + 11;
constexpr int kMbN2X = kBlendTileW / 4 + 4, kMbN2Y = kBlendTileH / 4 + 4;
constexpr int kMbNRX = kBlendTileW / 2 + 2, kMbNRY = kBlendTileH / 2 + 2;
constexpr int kMbTilePx = kBlendTileW * kBlendTileH;
// per-tile table (int32 words): m1 (R1 region) [slots], m2 [slots], d1 (R1 region), d2, then
// the work lists: n_px, n_r1, the level-0 / level-1 / level-2 column ranges (first, last) the
// mixed pixels depend on, per owner slot the level-1 and level-2 mosaic columns (first, last,
// first, last) of the entries the blend reads from that owner (the band pass computes only
// these), the tile pixels to blend (u16, one per tile pixel) and the R1 entries
// they read (u16, one per R1 entry)
constexpr int kMbTabRanges = 8;
constexpr int kMbTabCounts = kMbTabRanges + 4 * kBlendSlots;
constexpr int kMbTabLists = kMbTabCounts + kMbTilePx / 2 + (kMbNRX * kMbNRY + 1) / 2;
constexpr int mb_tab_words(int slots)
{
    return slots * (kMbNRX * kMbNRY + kMbN2X * kMbN2Y) + kMbNRX * kMbNRY + kMbN2X * kMbN2Y +
           kMbTabLists;
}
struct KBlendPrepArgs {
    KParams P;
    uint8_t *owner;
    uint32_t *info;
    int *list;
    int *overflow;
    // multi-band: tiles whose neighbourhood holds more than kBlendSlots owners take the feather
    // rule instead (list2[0] = count, then (tile, feather slot mask) pairs); overflow[0] counts them
    int *list2;
    int mode, pad_;
};
struct KMbArgs {
    KParams P;
    const uint8_t *owner;          // owner map of the mosaic
    const int *list;               // blend tile list: list[1 + 2i] = tile, list[2 + 2i] = mask
    uint64_t *desc;                // [tiles][slots][kMbUsedX * kMbUsedY] level-0 samples (prep)
    int32_t *tab;                  // [tiles][mb_tab_words(slots)] masks + denominators (prep)
    int32_t *foot;                 // [tiles][slots][8] source footprint per owner (prep)
    uint16_t *g1;                  // scratch [tiles][slots][chunk][R1 region][4] (u16 lanes)
    int32_t *g2;                   // scratch [tiles][slots][chunk][CN][level 2]
    int slots;                     // owners per tile (the tables' slot dimension)
    int chunk;                     // scratch capture stride
    int f0, nf;                    // captures [f0, f0 + nf) of this launch
    int list0;                     // blend: first list entry of this launch
    int n_list;                    // blend: list entries in this launch (xcd_unit's nx)
};

// Band pass of the multi-band levels (mcs_mb_bands_c*): one wave per (band, kMbBandFrames
// captures).  A band is one owner slot's pyramid over a 64-column window of the mosaic and the
// level-0 rows of one blend-tile row (its 89-row array): lane = level-0 column, rows walked top
// to bottom with the 5-tap reduces rolling in registers (no LDS, no barriers); the finished level-1
// / level-2 entries go to the per-(tile, owner) scratch of every listed blend tile of that row
// whose arrays contain them.  Windows start at multiples of 4 columns, so even lanes hold
// level-1 columns and every fourth lane a level-2 column.  Bands reaching past the bottom or
// right mosaic edge run the _br variant (reflected level-1 inputs of level 2).
struct MbBand {
    int slot, row, c0, pad_;
};
constexpr int kMbBandLanes = 64;
// rows walked per band: the 89-row level-0 array padded to the 12-row unrolled body (the extra
// rows feed no stored entry), and descriptor rows for the 3-row lookahead past it, so that no
// load in the loop needs a guard
constexpr int kMbBandRows = (kMbUsedY + 11) / 12 * 12;
// rows of window loads the band pass keeps in flight ahead of the row it computes (+1 buffer;
// the buffer count divides the 12-row body)
#ifndef MCS_MB_BAND_AHEAD
#define MCS_MB_BAND_AHEAD 2
#endif
constexpr int kMbBandAhead = MCS_MB_BAND_AHEAD;
constexpr int kMbBandBufs = kMbBandAhead + 1;
static_assert(12 % kMbBandBufs == 0, "band pass: buffers must divide the 12-row body");
// descriptor ring of the band pass: the descriptor of row r + kMbBandDescRing - 1 is loaded at row
// r and first used at row r + kMbBandDescRing - 1 - kMbBandAhead (to issue that row's window
// loads), so a ring deeper than the window buffers gives the dependent descriptor -> window
// loads more than one row of slack
#ifndef MCS_MB_DESC_RING
#define MCS_MB_DESC_RING 3
#endif
constexpr int kMbBandDescRing = MCS_MB_DESC_RING;
static_assert(12 % kMbBandDescRing == 0 && kMbBandDescRing >= kMbBandBufs,
              "band pass: descriptor ring must divide the 12-row body and hold the window rows");
constexpr int kMbBandDescRows = kMbBandRows + kMbBandDescRing;
constexpr int kMbBandStride = 52;  // window step: consecutive windows' level-2 outputs abut
#ifndef MCS_MB_BAND_FRAMES
#define MCS_MB_BAND_FRAMES 2
#endif
constexpr int kMbBandFrames = MCS_MB_BAND_FRAMES;
// LDS-ring band pass (mb_bands_body mode 2): per capture a ring of kMbLdsRows source rows of
// kMbLdsSpan bytes each; groups of 4 rows, kMbLdsLead rows loaded before the first row; counted
// vmcnt waits before each row's LDS reads (mb_lds_wait)
#define MCS_STR_(x) #x
#define MCS_STR(x) MCS_STR_(x)
#ifndef MCS_MB_LDS_DESC
#define MCS_MB_LDS_DESC 3
#endif
#ifndef MCS_MB_LDS_GLEAD
#define MCS_MB_LDS_GLEAD 3
#endif
constexpr int kMbLdsSpan = 256;
#ifndef MCS_MB_LDS_ROWS
#define MCS_MB_LDS_ROWS 16
#endif
#ifndef MCS_MB_LDS_LEAD
#define MCS_MB_LDS_LEAD 4
#endif
constexpr int kMbLdsRows = MCS_MB_LDS_ROWS;
constexpr int kMbLdsLead = MCS_MB_LDS_LEAD;
constexpr int kMbLdsGLead = MCS_MB_LDS_GLEAD;   // rows between a group's DMA and its first reader
constexpr int kMbLdsRingBytes = kMbLdsRows * kMbLdsSpan;
// (the ring descriptor keeps window a's ring offset in 14 bits, its byte shift in bits 14-15:
// mcs_capi.cpp band_lds_tables, decoded with & 0x3fff in mb_bands_body)
static_assert(kMbLdsRingBytes <= (1 << 14), "LDS band ring: offsets must fit the 14-bit field");
// per wave: the captures' rings, then the descriptor ring (kMbLdsDescRing rows of 16 B per
// lane: the descriptor of row r + kMbLdsDescRing is staged after row r, so the kMbLdsDescRing - 1
// descriptor DMAs after it bound the wait)
constexpr int kMbLdsDescRing = MCS_MB_LDS_DESC;
constexpr int kMbLdsDescRows = kMbBandRows + kMbLdsDescRing;
constexpr int kMbLdsDescOff = kMbBandFrames * kMbLdsRingBytes;
constexpr int kMbLdsBytes = kMbLdsDescOff + kMbLdsDescRing * kMbBandLanes * 16 + 16;
static_assert(12 % kMbLdsDescRing == 0 && kMbLdsGLead >= 1 && kMbLdsGLead <= kMbLdsDescRing,
              "LDS band ring: descriptor ring divides the 12-row body; groups led by <= its rows");
constexpr int kMbLdsGroups = kMbBandRows / 4 + kMbLdsLead / 4 + 3;  // group offsets per band
static_assert(kMbLdsRows % 4 == 0 && kMbLdsLead % 4 == 0 && kMbLdsRows / 4 > kMbLdsLead / 4 + 1,
              "LDS band ring: whole groups, the prologue's groups never evicted by the loop's first");
struct KMbBandArgs {
    KParams P;
    const int *list;               // blend tile list (tile, mask)
    const int *tile_bt;            // blend-tile grid -> list index (-1: not listed)
    const MbBand *bands;
    uint64_t *bdesc;               // [bands][kMbBandDescRows][kMbBandLanes] window descriptors
    uint16_t *g1;                  // scratch, as KMbArgs
    int32_t *g2;
    const uint32_t *bgrp;          // [bands][kMbLdsGroups][kMbBandLanes] LDS-ring group offsets
    const uint4 *bdesc16;          // [bands][kMbLdsDescRows][kMbBandLanes] LDS-ring descriptors
    int slots, chunk, f0, nf;
    int gxb;                       // blend tiles per mosaic row
    int band0;                     // first band of this launch
    int n_in;                      // mcs_mb_bands_all: blocks below n_in take the interior path
                                   // (band band0 + block), the others the _br path (band
                                   // band1 + block - n_in)
    int band1;
    int nb;                        // bands in this launch (xcd_unit's nx)
};
struct KBlendArgs {
    KParams P;
    const uint8_t *owner;
    const int *list;
    int n_frames, pad_;
};

// Multi-band sweep (mcs_sweep.hip): the band pass and the blend fused into one kernel.  A strip
// is a 128-column window of the mosaic over a run of blend-tile rows around one seam region; one
// workgroup per (strip, capture) walks it top to bottom, 4 level-0 rows per step: the owners'
// replicate-border samples -> level-1 / level-2 rows (5-tap reduces: vertical in registers,
// horizontal through LDS) -> B2 / R1 / R0 of the blend from LDS rings, and writes every pixel of
// its output region (mixed pixels blended, the others their owner sample; the streaming kernel
// skips them).  No level scratch in HBM, no second launch.
constexpr int kSwCols = 128;         // level-0 columns of a strip window (2 waves per owner)
constexpr int kSwMaxOwners = 4;      // owners per strip (workgroup of 128 x 2 or 128 x 4 threads)
constexpr int kSwMargin = 16;        // output columns [c0 + 16, c0 + 116) of a window (interior)
constexpr int kSwValid = 100;
constexpr int kSwLead = 16;          // first level-0 row sampled: ya - 16
constexpr int kSwDescPad = 12;       // descriptor rows past the last step (12-row prefetch)
// LDS rings (rows): level-0 owner samples, level 1, level 2, B2, R1
constexpr int kSwNG0 = 24, kSwNG1 = 10, kSwNG2 = 4, kSwNB2 = 4, kSwNR1 = 4;
constexpr int kSwMaxR1 = 64, kSwMaxB2 = 32;   // R1 / B2 columns of a strip
struct MbStrip {
    int c0;                  // first level-0 column of the window (multiple of 4)
    int r0;                  // first level-0 row sampled (ya - kSwLead)
    int nsteps;              // steps of 4 rows (a multiple of 3)
    int ya, yb;              // output rows [ya, yb)
    int ns;                  // owners (<= kSwMaxOwners)
    int reg;                 // region table entry of row ya (one per output row: xa | xb << 16)
    int dsc;                 // descriptor block: rows of kSwCols u64 from sdesc
    int e1lo, e1n, z2lo, z2n;   // R1 / B2 columns (mosaic level-1 / level-2 coordinates)
    int slot[kSwMaxOwners];  // plan slots of the owners
};
static_assert(sizeof(MbStrip) == 64, "MbStrip layout");
struct KMbSweepArgs {
    KParams P;
    const MbStrip *strips;
    uint64_t *sdesc;         // per strip [ns][4 nsteps + kSwDescPad][kSwCols] window descriptors
    const int *region;
    const uint8_t *owner;    // owner map (descriptor kernel)
    int n_strips, f0, nf, pad_;
};

constexpr int kDirectFrames = 4;    // captures per direct-gather block
// Footprint rows per wave per capture (a tile needing more goes to the direct path).  8 x 8 = 64
// rows covers every tile of the C4 cylinder rig, whose top and bottom tiles' footprints curve
// over ~40 source rows per camera (6 per wave left 215 of its 3672 tiles on the direct path:
// C4 launch 1.94 -> 1.82 ms; the C2 launch is unchanged, 80 VGPRs keep 6 waves per SIMD).
#ifndef MCS_JOBS_PER_WAVE
#define MCS_JOBS_PER_WAVE 8
#endif
constexpr int kJobsPerWave = MCS_JOBS_PER_WAVE;
constexpr int kLdsSlack = 16;      // window reads run up to 8 bytes past a row's last byte
constexpr int kMaxRing = 6;
// LDS of a streaming block: the tile header, then a ring of capture footprints, as many slots
// (2..kMaxRing) as fit.  3 blocks per CU (the kernel's registers allow 3 x 8 waves) at 40 KiB
// each leave 40 KiB of the CU's 160 KiB for a multi-band blend block beside them (same-box A/B
// against 52 KiB: paste launch 0.612 -> 0.605 ms, multi-band 0.963 -> 0.957 ms; round 3).
#ifndef MCS_STREAM_LDS
#define MCS_STREAM_LDS 40960
#endif
constexpr int lds_stream_bytes(int cn) { return cn >= 3 ? MCS_STREAM_LDS : 40960; }
constexpr int lds_ring_bytes(int cn) { return lds_stream_bytes(cn) - (int)sizeof(TileHdr); }
// Large-footprint tiles (TileHdr::fits == 2): the tiles whose footprints exceed the streaming
// block's budget -- the C4 cylinder's top and bottom tiles, whose rows curve over ~45 source rows
// per camera, two cameras at a seam -- run the same streaming code with 16 footprint rows per
// wave and a 120 KiB ring (one block per CU) over their own list, on the side stream beside the
// main launch (round 3 sent these 39 C4 tiles to the direct-gather kernel).
constexpr int kBigJobsPerWave = 16;
static_assert(kBigJobsPerWave * kWavesPerBlock <= kMaxTileJobs, "row spans per tile");
constexpr int kBigStreamLds = 120 * 1024;
constexpr int big_ring_bytes() { return kBigStreamLds - (int)sizeof(TileHdr); }
// LDS row pitch of a footprint row of `bytes` DMA bytes.  The 32 lanes of an output row read
// dwords ~3 apart (C = 3, 4 pixels per lane: a permutation of the 32 ds_read_b32 banks); where
// the source row changes inside the lane group (a rotated map), the lanes past the change read
// one pitch further -- conflict-free only when the pitch is a multiple of 128 bytes (32 banks).
constexpr int lds_row_pitch(int bytes) { return (bytes + 127) & ~127; }


// Seam-finder inputs (mcs_plan_find_seams): per point of the 2^k grid the distance owner's
// camera, the covering cameras and every covering camera's sample (samples[cam][point][CN]).
struct KSeamArgs {
    KParams P;
    uint8_t *label;
    uint16_t *cov;
    uint8_t *samples;
    int gw, gh, k, pad_;
};

}  // namespace mcs
