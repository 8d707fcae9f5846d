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
    int pad_;
};

struct KParams {
    int n_stages;
    int out_w, out_h;
    int cam0_offx, cam0_offy;
    int cam0_w, cam0_h;
    int pad_;
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

// Tiling of the stitch kernel (must match the kernel): a block is 256 px x 8 rows, one row per
// wave, 4 consecutive pixels per lane.
constexpr int kPx = 4;             // output pixels per lane
constexpr int kWave = 64;
constexpr int kWavesPerBlock = 8;  // one row per wave
constexpr int kTileW = kPx * kWave;
constexpr int kTileH = kWavesPerBlock;

// Prepared per-plan tables (mcs_plan_prepare): one TileHdr per 256 x 8 tile, and per pixel of the
// tile three u32 -- the LDS byte addresses of its two row windows (16 bits each) and the packed
// u16 weight pairs (w00, w01), (w10, w11) -- stored thread-major so each lane loads its 4 pixels
// as 48 contiguous bytes.
constexpr int kTileCams = 4;       // cameras one LDS tile may draw from
constexpr int kTilePx = kTileW * kTileH;
constexpr int kDescWords = 3;
struct TileHdr {
    int fits;                      // 1: LDS path, 0: listed for the direct-gather launch
    int ncam, njobs, ring, buf_bytes;
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
struct KPrepareArgs {
    KParams P;
    TileHdr *tiles;
    uint32_t *desc;
    int *fallback;                 // [0] = count, then tile indices
};
struct KStreamArgs {
    KParams P;
    const TileHdr *tiles;
    const uint32_t *desc;
    int n_frames;
    int pad_;
};
struct KDirectArgs {
    KParams P;
    const int *fallback;
    int n_frames;
    int pad_;
};

// LDS of a streaming block: the tile header, then a ring of capture footprints, as many slots (up
// to kMaxRing, at least 2) as fit in kLdsRing bytes.
constexpr int kLdsRing = 40832;
constexpr int kDirectFrames = 4;    // captures per direct-gather block
constexpr int kJobsPerWave = 4;     // footprint rows per wave per capture (more rows -> direct path)
constexpr int kLdsSlack = 16;      // window reads run up to 8 bytes past a row's last byte
constexpr int kMaxRing = 4;
constexpr int kLdsStream = (int)sizeof(TileHdr) + kLdsRing;   // 40960 bytes: 4 blocks per CU

}  // namespace mcs
