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

// Kernarg block of the stitch kernels: (KParams, int n_frames).
struct KStitchArgs {
    KParams P;
    int n_frames;
    int pad_;
};

// Tiling of the stitch kernel (must match the kernel): a block is 256 px x 8 rows, one row per
// wave, 4 consecutive pixels per lane.
constexpr int kPx = 4;             // output pixels per lane
constexpr int kWave = 64;
constexpr int kWavesPerBlock = 8;  // one row per wave
constexpr int kTileW = kPx * kWave;
constexpr int kTileH = kWavesPerBlock;

// LDS of one block: a header (per-camera footprint and layout) and two staging buffers.
constexpr int kLdsHeader = 1024;
constexpr int kLdsBuf = 19456;     // bytes of source footprint one capture may occupy
constexpr int kLdsSlack = 16;      // window reads run up to 8 bytes past a row's last byte
constexpr int kLdsBytes = kLdsHeader + 2 * (kLdsBuf + kLdsSlack);

}  // namespace mcs
