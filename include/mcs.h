/*
 * mcs.h -- C ABI of libmcs.so, the MI355X (gfx950) multi-camera stitch hot path.
 *
 * The reference (kiwicampus/multicamera_stitching) is Python 2 glue around OpenCV; it has no
 * FFI of its own.  Its per-frame hot path is
 *     Stitcher.stitch(images_dic)                PostScripts/Stitcher/StitcherClass.py:114-136
 *       -> N-1 x StitcherBase.stitch((B, A))                                    :211-256
 *            cv2.warpPerspective(A, cachedAH, ABSize)                            :239
 *            dst[By:By+hB, Bx:Bx+wB] = B                                         :240-241
 *            dst = dst[y_limits[0]:y_limits[1], x_limits[0]:x_limits[1]]  (super) :248-251
 * The entry points below replace exactly that chain: the Python drop-in
 * (multicamera_stitching_amd/StitcherClass.py, module name `StitcherClass`) marshals the
 * calibrated StitcherBase fields into mcs_stage_desc[] once, and each Stitcher.stitch call
 * becomes one mcs_stitch_host (or mcs_stitch_device) call.  The ctypes binding a maintainer
 * adds on the reference side is shown in INTEGRATION.md.
 *
 * Conventions: plain pointers and sizes only; every function returns an int status
 * (MCS_OK = 0, negative = error) and never throws; mcs_last_error() returns a thread-local
 * message for the last failure on the calling thread.  A plan is bound to one device and is
 * not re-entrant (callers serialise per plan; distinct plans are independent).
 */
#ifndef MCS_H_
#define MCS_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MCS_ABI_VERSION 1

enum {
    MCS_OK = 0,
    MCS_E_INVALID = -1,     /* bad argument / null pointer */
    MCS_E_HIP = -2,         /* HIP runtime failure (no device, launch error, ...) */
    MCS_E_NOMEM = -3,       /* host or device allocation failed */
    MCS_E_SHAPE = -4,       /* stage geometry inconsistent (reference would resize / raise) */
    MCS_E_UNSUPPORTED = -5  /* channels / stage count outside what the kernels handle */
};

enum { MCS_INTER_NEAREST = 0, MCS_INTER_LINEAR = 1 };
/* How overlapping cameras combine (mcs_plan_set_blend).  NONE is the reference: B pasted over
 * the warped A (StitcherClass.py:240-241).  FEATHER / MULTIBAND (no
 * reference implementation; specified in oracle/orc_blend.c): every pixel belongs to the
 * covering camera farthest from its own image edge; FEATHER averages the covering cameras
 * weighted by that edge distance, MULTIBAND blends a 3-level Laplacian pyramid across those
 * ownership seams, SEAM copies the owner's sample (the seam without blending). */
enum { MCS_BLEND_NONE = 0, MCS_BLEND_FEATHER = 1, MCS_BLEND_MULTIBAND = 2, MCS_BLEND_SEAM = 3 };

#define MCS_MAX_STAGES 15
#define MCS_MAX_CAMS (MCS_MAX_STAGES + 1)

/* One StitcherBase of the chain, in sorted-label order (StitcherClass.py:61-75). */
typedef struct mcs_stage_desc {
    double H[9];        /* cachedAH, row-major, FORWARD (A -> canvas) exactly as handed to
                           cv2.warpPerspective (:239); inverted inside like OpenCV (LU, n=3) */
    int calibrated;     /* cachedAH is not None (:223); 0 -> stage passes B through (:255-256) */
    int canvas_w;       /* ABSize[0] (:238) */
    int canvas_h;       /* ABSize[1] */
    int b_x, b_y;       /* int(Bpts[0][0]), int(Bpts[0][1]) (:237) */
    int b_w, b_h;       /* BimgSize[1], BimgSize[0]: calibrated size of B (:226) */
    int a_w, a_h;       /* AimgSize[1], AimgSize[0]: calibrated size of A (:230) */
    int super_mode;     /* (:248) */
    int x_lim0, x_lim1; /* x_limits (:251), Python-slice semantics */
    int y_lim0, y_lim1; /* y_limits (:250) */
} mcs_stage_desc;

/* Flattened geometry of a plan (what the single-pass gather kernel consumes). */
typedef struct mcs_flat_stage {
    double minv[9];     /* OpenCV-inverted H (cv::invert DECOMP_LU closed form) */
    int rect[4];        /* B paste rect of this stage in OUTPUT coords: x0, y0, x1, y1 */
    int off_x, off_y;   /* output coords -> this stage's canvas coords */
    int bw0;            /* OpenCV WarpPerspectiveInvoker block width of the canvas */
    int cam;            /* camera index (sorted-label order) warped by this stage */
} mcs_flat_stage;

typedef struct mcs_flat_desc {
    int n_stages;                  /* calibrated stages only, innermost first */
    int out_w, out_h, channels, interp;
    int cam0_off_x, cam0_off_y;    /* output coords -> camera-0 coords */
    int n_cams;
    int cam_w[MCS_MAX_CAMS], cam_h[MCS_MAX_CAMS];
    mcs_flat_stage st[MCS_MAX_STAGES];
} mcs_flat_desc;

typedef struct mcs_plan mcs_plan;

/* Library / device info. */
const char *mcs_version(void);
int mcs_abi_version(void);
/* Identity of the kernels this library runs: the first 16 hex digits of the SHA-256 of its
 * embedded gfx950 code objects (profiles/ PMC summaries record it, and bench.py reports their
 * HBM traffic only for the same build). */
const char *mcs_build_id(void);
const char *mcs_last_error(void);
int mcs_device_count(int *n);
/* The HIP runtime libmcs bound to (it links none: it uses the process's, e.g. PyTorch's). */
const char *mcs_hip_runtime(void);

/* Build a plan from the calibrated chain (replaces the per-stage state the reference keeps in
 * StitcherBase, :190-209).  cam0_w/cam0_h: calibrated size of the first camera (B of stage 0).
 * channels: 1..4 (interleaved u8, e.g. BGR = 3).  interp: MCS_INTER_LINEAR is the reference
 * default (:239); MCS_INTER_NEAREST is the north-star C1 variant.  device: HIP ordinal.
 * Host-side only: no device memory is touched until the first stitch call. */
int mcs_plan_create(const mcs_stage_desc *stages, int n_stages, int cam0_w, int cam0_h,
                    int channels, int interp, int device, mcs_plan **out);
/* A camera of a rotation-only rig projected onto a cylinder (SURVEY.md section 8 NS-6 / C4:
 * 8 cameras at 45 degree yaw steps around one centre, f = 1100).  R: rig -> camera rotation,
 * row-major (a rig ray d maps to R d in camera coordinates, z forward, y down); f, cx, cy:
 * pinhole intrinsics in pixels; w, h: frame size.  Undistorted frames (see mcs_undistort_*). */
typedef struct mcs_cyl_camera {
    double R[9];
    double f, cx, cy;
    int w, h;
} mcs_cyl_camera;

/* Plan of a cylindrical panorama: output pixel (u, v) is the rig ray (sin t, h, cos t) with
 * t = (u - u0) / f_cyl, h = (v - v0) / f_cyl; every camera is warped through it and the cameras
 * meet at the blend seam (largest edge distance, ties to the lower camera index), blended by the
 * plan's blend mode: MCS_BLEND_MULTIBAND by default, FEATHER or SEAM (MCS_BLEND_NONE is
 * refused: there is no paste order).  The same fixed-point bilinear / nearest sampling as the
 * homography plans; the per-column sin/cos and per-row h are computed once on the host. */
int mcs_plan_create_cylindrical(const mcs_cyl_camera *cams, int n_cams, int out_w, int out_h,
                                double f_cyl, double u0, double v0, int channels, int interp,
                                int device, mcs_plan **out);
/* cv2.warpPerspective(src, M, (dst_w, dst_h)) as a plan (flags INTER_LINEAR / INTER_NEAREST,
 * BORDER_CONSTANT 0): the extrinsic bird's-eye view of the reference's display path
 * (MediaPlayer/view.py:387-388, PostScripts/Calibration_Utils/Extrinsic.py:99).  One camera of
 * src_w x src_h; stitch calls take one camera pointer.  Blend mode NONE only. */
int mcs_plan_create_warp(const double *M, int src_w, int src_h, int dst_w, int dst_h,
                         int channels, int interp, int device, mcs_plan **out);
/* cv2.undistort(src, K, dist) as a plan (OpenCV 3.4 stripes + initUndistortRectifyMap + remap
 * INTER_LINEAR, BORDER_CONSTANT): the per-frame undistortion before stitching
 * (video_mapping_node.py:157-158, MediaPlayer/view.py:380-381, Intrinsic.py:234-235).  K: 3x3
 * row-major; dist: 0, 4, 5, 8, 12 or 14 coefficients (tilt tau_x = tau_y = 0).  The map is
 * computed once on the host; per frame it is the plan's remap.  Blend mode NONE only. */
int mcs_plan_create_undistort(const double *K, const double *dist, int n_dist, int w, int h,
                              int channels, int device, mcs_plan **out);
/* The undistortion map of mcs_plan_create_undistort on the host (no device): map[2 p], map[2 p+1]
 * = cv::initUndistortRectifyMap's CV_16SC2 + CV_16UC1 pair of output pixel p as one fixed-point
 * value per axis, (short)(i >> 5) * 32 + (i & 31) with i = cvRound(32 u). */
int mcs_undistort_map_host(const double *K, const double *dist, int n_dist, int w, int h,
                           int32_t *map);
int mcs_plan_destroy(mcs_plan *plan);
int mcs_plan_out_shape(const mcs_plan *plan, int *w, int *h, int *channels);
int mcs_plan_describe(const mcs_plan *plan, mcs_flat_desc *out);

/* Evaluates the plan's exact OpenCV coordinate map once on its device and stores it as per-tile
 * LDS layouts + per-pixel window descriptors (the fixed-point remap tables of this plan; OpenCV's
 * own remap path uses the same idea, cv::convertMaps).  Allocates device memory and
 * synchronises: call it before capturing stitch calls into a HIP graph.  The stitch entry points
 * call it on first use.  stream: hipStream_t or NULL for the plan's own stream. */
int mcs_plan_prepare(mcs_plan *plan, void *stream);

/* stats[0..15] = prepared, tiles, tiles on the LDS path, tiles on the direct path, table bytes,
 * blend mode, 32 x 64 tiles the blend kernels recompute per frame, the most owners any
 * multi-band tile blends (<= 8), multi-band tiles degraded to the feather rule (their
 * neighbourhood -- the tile grown by 16 px -- holds more than 8 owners), multi-band bands of the
 * level pass, of those the bands whose source rows are staged in the LDS ring (the rest read
 * their windows from global memory), and of the LDS-path tiles those whose footprints need the
 * large-footprint streaming launch (16 rows per wave, 120 KiB ring), then per capture the
 * multi-band blend's computed ("mixed") pixels and R1 entries, then per capture the bytes the
 * LDS-path tiles' footprint DMAs read (each row's span in 16-byte chunks) and the bytes of their
 * footprint boxes (every row at the box width); stats[16..19] = the multi-band sweep's strips
 * (MCS_MB_SWEEP=1 plans; 0 otherwise), the mosaic pixels they write per capture, threads per
 * sweep workgroup, and the rows of its precomputed sample descriptors.  Entries past 19 read 0. */
int mcs_plan_stats(const mcs_plan *plan, int64_t *stats, int n);

/* Blend mode of the plan (MCS_BLEND_*; default NONE = the reference's paste).  Changing it drops
 * the prepared tables (rebuilt by mcs_plan_prepare or the next stitch).  FEATHER / MULTIBAND
 * replace the reference's paste with the blends of SURVEY.md 8 NS-2 / NS-1.  MULTIBAND blends up
 * to 8 owners per 32 x 64 tile neighbourhood (the tile grown by 16 px); a tile with more takes
 * the FEATHER rule instead, on the GPU (counted in mcs_plan_stats[8]; oracle/orc_blend.c "dense
 * seams").  Cylindrical plans refuse NONE. */
int mcs_plan_set_blend(mcs_plan *plan, int mode);

/* Seams.  MCS_SEAM_DISTANCE: the owner is the covering camera farthest from
 * its image edge (the default).  MCS_SEAM_GRAPHCUT: pairwise minimum cuts through the overlaps
 * (cost: colour difference of the two cameras, OpenCV GraphCutSeamFinder COST_COLOR style) on
 * the 2^scale_log2-subsampled panorama of this capture (cams: host frames at calibrated sizes),
 * then every pixel takes its grid point's camera when that camera covers it.  Once per plan
 * (calibration time: device sampling + device push-relabel max-flows, MCS_SEAM_FLOW=host: the
 * host Dinic; both give the same cut); drops the prepared tables.  The exact rules:
 * oracle/orc_seam.c.  scale_log2: 0..4. */
enum { MCS_SEAM_DISTANCE = 0, MCS_SEAM_GRAPHCUT = 1 };
int mcs_plan_find_seams(mcs_plan *plan, const uint8_t *const *cams, int method, int scale_log2);
/* The current seam labels (camera per grid point, 255 = none): *w, *h = grid size (0 when the
 * plan uses distance seams); out (w*h bytes) may be NULL to query the size. */
int mcs_plan_seam_labels(const mcs_plan *plan, uint8_t *out, int *w, int *h);
/* The host half of mcs_plan_find_seams on caller-supplied inputs (no device): labels (in: the
 * distance owners' cameras, 255 = none; out: the cut), cover (bit c: camera c covers the point),
 * samples [camera][point][channels].  grid gw x gh, up to 16 cameras. */
int mcs_seam_graphcut_host(int n_cams, int gw, int gh, uint8_t *labels, const uint16_t *cover,
                           const uint8_t *samples, int channels);
/* The same pairwise cuts on the device (push-relabel, the path mcs_plan_find_seams takes by
 * default; MCS_SEAM_FLOW=host selects the host Dinic there): host arrays in, labels updated in
 * place.  stats (5, may be NULL): pairs with a graph, push launches, relabel launches, global
 * relabels, microseconds of the max-flows. */
int mcs_seam_graphcut_device(int n_cams, int gw, int gh, uint8_t *labels, const uint16_t *cover,
                             const uint8_t *samples, int channels, int device, int64_t *stats);
/* The device max-flow's counts of the plan's last mcs_plan_find_seams (as above). */
int mcs_plan_seam_stats(const mcs_plan *plan, int64_t *stats);

/* Stitcher.stitch on host arrays (drop-in path, :114-136): cams[i] is the i-th camera in
 * sorted-label order, dense HxWxC u8 of the calibrated size; out is a dense out_h x out_w x C
 * buffer.  Synchronous: H2D -> kernel -> D2H on the plan's stream. */
int mcs_stitch_host(mcs_plan *plan, const uint8_t *const *cams, uint8_t *out);

/* The same with the frames' actual sizes (cam_w[i] x cam_h[i], same channel count): a frame off
 * its calibrated size is first resized to it on the device with cv2.resize(INTER_LINEAR)
 * arithmetic, as StitcherBase.stitch does before warping (StitcherClass.py:226-233).  NULL
 * cam_w/cam_h = calibrated sizes (== mcs_stitch_host). */
int mcs_stitch_host_sized(mcs_plan *plan, const uint8_t *const *cams, const int *cam_w,
                          const int *cam_h, uint8_t *out);

/* cv2.resize(src, (dst_w, dst_h), interpolation=cv2.INTER_LINEAR) (replaces the call at
 * StitcherClass.py:229,233) on n_frames device-resident u8 images of `channels` interleaved
 * channels; frame f of src starts at d_src + f*src_frame_stride (0 = src_pitch*src_h), rows at
 * src_pitch; likewise dst.  Same size = copy (as OpenCV).  Enqueued on `stream` of `device`. */
int mcs_resize_linear_device(const uint8_t *d_src, int src_w, int src_h, int64_t src_pitch,
                             int64_t src_frame_stride, uint8_t *d_dst, int dst_w, int dst_h,
                             int64_t dst_pitch, int64_t dst_frame_stride, int channels,
                             int n_frames, int device, void *stream);

/* Device-resident batch: n_frames rigs.  d_cams[i] + f*cam_frame_stride[i] is frame f of camera
 * i (dense rows, pitch = w*C); d_out + f*out_frame_stride + y*out_pitch is output row y of frame
 * f.  Enqueued on `stream` (a hipStream_t of the process's HIP runtime; NULL = the null
 * stream); does not synchronise. */
int mcs_stitch_device(mcs_plan *plan, const uint8_t *const *d_cams,
                      const int64_t *cam_frame_stride, uint8_t *d_out, int64_t out_pitch,
                      int64_t out_frame_stride, int n_frames, void *stream);

/* mcs_stitch_device without prepared tables: every output pixel maps through the exact FP64
 * OpenCV map in the kernel itself (the direct-gather kernel over all tiles), so a plan is
 * usable the moment mcs_plan_create returns (host flattening only, microseconds) -- the path for
 * geometry that changes every capture (per-frame homographies, SURVEY.md 8 C3: estimate ->
 * stitch).  Paste (MCS_BLEND_NONE) and MCS_BLEND_SEAM plans; the same pixels as
 * mcs_stitch_device.  Replaces, per capture, StitcherBase.calibrate (:258-354) followed by
 * StitcherBase.stitch (:211-256). */
int mcs_stitch_direct(mcs_plan *plan, const uint8_t *const *d_cams,
                      const int64_t *cam_frame_stride, uint8_t *d_out, int64_t out_pitch,
                      int64_t out_frame_stride, int n_frames, void *stream);

/* Source pixels each camera actually contributes to the mosaic (for the roofline's algorithmic
 * byte count): touched_px[i] for i < n_cams.  Runs a one-off marking kernel. */
int mcs_plan_footprint(mcs_plan *plan, int64_t *touched_px, int n_cams);

/* ---- Streaming (host frames in, host mosaics out) ---------------------
 * `depth` capture slots, each with pinned host staging and device buffers.  submit: the camera
 * frames (sorted-label order, calibrated sizes, or NULL after filling mcs_stream_input() in
 * place) are uploaded on a copy stream, stitched on a compute stream (one hipGraph per slot when
 * use_graphs), and the mosaic downloaded on a second copy stream -- so consecutive captures
 * overlap upload, stitch and download.  wait: blocks for that slot's mosaic and copies it to
 * `out` (out_h x out_w x C, dense; NULL: no copy, read mcs_stream_output instead); a slot must
 * be collected before it is reused.  The plan (blend mode included) is fixed for the stream's
 * lifetime; the stream lives on the plan's device.  Zero-copy use: the producer writes the next
 * slot's frames into mcs_stream_input(mcs_stream_next_slot()) and submits NULL, the consumer
 * reads mcs_stream_output(slot) after mcs_stream_wait(slot, NULL) until that slot's next
 * submit -- the pipeline then moves bytes only over PCIe. */
typedef struct mcs_stream mcs_stream;
int mcs_stream_create(mcs_plan *plan, int depth, int use_graphs, mcs_stream **out);
/* Helper threads of this process's host copy pool (caller frames -> pinned slots, slots ->
 * caller mosaics): half of the CPUs it may use (affinity, cgroup quota) divided among the
 * LOCAL_WORLD_SIZE ranks of the node, minus one, at most 7.  Host only (no device). */
int mcs_stream_copy_workers(void);
uint8_t *mcs_stream_input(mcs_stream *stream, int slot, int cam);
/* The pinned host mosaic of `slot` (out_h x out_w x C, dense), NULL for a bad slot. */
const uint8_t *mcs_stream_output(const mcs_stream *stream, int slot);
int mcs_stream_next_slot(const mcs_stream *stream);
int mcs_stream_submit(mcs_stream *stream, const uint8_t *const *cams, int *slot);
/* mcs_stream_submit with a row pitch (bytes) per camera: camera c is cam_h rows of
 * cam_w * channels bytes starting at cams[c], rows row_pitch[c] apart -- e.g. one frame of the
 * reference's memmap bus, np.concatenate(images, axis=1) (video_mapping_node.py:140), with
 * cams[c] = frame + c * cam_w * channels and row_pitch = the frame's row bytes.  NULL row_pitch
 * = dense cameras. */
int mcs_stream_submit_strided(mcs_stream *s, const uint8_t *const *cams,
                              const int64_t *row_pitch, int *slot);
int mcs_stream_wait(mcs_stream *stream, int slot, uint8_t *out);
int mcs_stream_destroy(mcs_stream *stream);

/* ---- Matching (per-frame estimation path) -------------------------------
 * Brute-force k=2 nearest neighbours of each query descriptor among the train descriptors under
 * the Hamming distance, as cv2.BFMatcher(cv2.NORM_HAMMING).knnMatch(query, train, k=2) (the
 * reference's matcher is the float-L2 BFMatcher at StitcherClass.py:405-448; with binary ORB
 * descriptors it becomes this).  Descriptors: 32 bytes (256 bits) each, dense.  Output per query
 * q: idx2[2q], idx2[2q+1] = train indices of the best and second best, dist2[...] their
 * distances (ties: the lower train index first, as OpenCV); -1/-1 where n_train < 2 leaves no
 * candidate.  n_train < 2^23.  Device pointers, enqueued on `stream` of `device`. */
int mcs_match_hamming_knn2(const uint8_t *d_query, int n_query, const uint8_t *d_train,
                           int n_train, int32_t *d_idx2, int32_t *d_dist2, int device,
                           void *stream);
/* The same on host buffers (synchronous; allocates and frees its device buffers). */
int mcs_match_hamming_knn2_host(const uint8_t *query, int n_query, const uint8_t *train,
                                int n_train, int32_t *idx2, int32_t *dist2, int device);

/* ---- Features -----------------------------------------------------------
 * ORB keypoints + 256-bit descriptors of one image (u8, channels 1 = gray or 3 = BGR, dense),
 * the per-frame replacement of detectAndDescribe (StitcherClass.py:356-403, SIFT there):
 * nlevels pyramid (scale_factor, INTER_LINEAR), FAST-9 (fast_threshold) + NMS, Harris ranking
 * with OpenCV's per-level quota of nfeatures, intensity-centroid orientation, rBRIEF (OpenCV's
 * 31x31 pattern).  Specified in csrc/mcs_orb_core.h.  Outputs (capacity nfeatures): kp_xy
 * (level-0 pixels), kp_response, kp_angle (degrees), kp_level (may be NULL), desc (32 B each),
 * *n_out.  w, h <= 65535.  Synchronous: one upload, one copy back (levels ranked on the device;
 * a level with more than 4096 candidates is ranked on the host, same result). */
int mcs_orb_detect_host(const uint8_t *image, int w, int h, int channels, int nfeatures,
                        int nlevels, float scale_factor, int fast_threshold, float *kp_xy,
                        float *kp_response, float *kp_angle, int *kp_level, uint8_t *desc,
                        int *n_out, int device);

/* The same on a frame already in device memory (d_image, dense, on `device`; its producer must
 * have finished -- the call runs on the calling thread's own stream): no upload, e.g. when the
 * frame is also stitched (mcs_stitch_direct).  Same outputs, same result. */
int mcs_orb_detect_device(const uint8_t *d_image, int w, int h, int channels, int nfeatures,
                          int nlevels, float scale_factor, int fast_threshold, float *kp_xy,
                          float *kp_response, float *kp_angle, int *kp_level, uint8_t *desc,
                          int *n_out, int device);

/* BFMatcher(NORM_L2) ("BruteForce").knnMatch(query, train, k=2) for float descriptors (the
 * reference's SIFT matcher, StitcherClass.py:423-424) on MFMA.  Descriptors that
 * are all integers in [0, 255] (OpenCV SIFT's) are matched exactly (int8 MFMA, integer squared
 * distances, float(sqrt) -- OpenCV's own float result for such data, ordered by (distance,
 * index) as its batchDistance); other data on f32 MFMA (|a|^2 + |b|^2 - 2 a.b in float).
 * *exact (optional) reports which.  idx2 / dist2: n_query x 2, -1 / -1.0f where fewer than two
 * train descriptors exist.  dim 1..256.  Allocates scratch and synchronises (calibration-time). */
int mcs_match_l2_knn2(const float *d_query, int n_query, const float *d_train, int n_train,
                      int dim, int32_t *d_idx2, float *d_dist2, int *exact, int device,
                      void *stream);
int mcs_match_l2_knn2_host(const float *query, int n_query, const float *train, int n_train,
                           int dim, int32_t *idx2, float *dist2, int *exact, int device);

/* ---- Homography estimation ----------------------------------------------
 * RANSAC homography of n correspondences src_xy[i] -> dst_xy[i] (float x, y pairs), the role of
 * cv2.findHomography(ptsA, ptsB, cv2.RANSAC, reprojThresh) at StitcherClass.py:443-444.  `iters`
 * hypotheses (4-point DLT, FP64) are scored in parallel on the GPU (one workgroup each); the
 * most-supported one (ties: lowest index) gives the inlier mask; then, as findHomography does
 * after its RANSAC loop (n > 4), the model is re-estimated on its inliers (Hartley-normalised
 * DLT, Jacobi eigenvector) and refined by 10 Levenberg-Marquardt iterations
 * (mcs_homography_refine_host).  H: row-major 3x3.  Deterministic for a given seed; hypothesis
 * algorithm specified in csrc/mcs_ransac_core.h, refinement in csrc/mcs_refine.cpp.  *n_inliers = 0 and H = 0 when no model (n < 4 or no
 * hypothesis with >= 4 inliers), like the reference's H = None.  mask may be NULL. */
int mcs_ransac_homography_host(const float *src_xy, const float *dst_xy, int n, double thresh,
                               int iters, uint32_t seed, double *H, uint8_t *mask,
                               int *n_inliers, int device);
/* findHomography's post-RANSAC stage alone (host FP64, no GPU): H (9 doubles) holds the RANSAC
 * model on entry and the refined one on return; mask[i] != 0 marks the inliers.  n <= 4 or no
 * inlier: H unchanged. */
int mcs_homography_refine_host(const float *src_xy, const float *dst_xy, int n,
                               const uint8_t *mask, double *H);

/* ---- Chain geometry of one capture -----------------------------------------
 * Stage descriptors of a left-to-right chain from its adjacent-pair homographies: pair k
 * (pair_H + 9 k, row-major, used when pair_ok[k]) maps camera k+1 into camera k; stage k's A ->
 * mosaic homography is T(o_k) . H_0 ... H_k with o_k camera 0's origin in the mosaic so far, and
 * its fields follow StitcherBase.calibrate (StitcherClass.py:293-351: corners projected and
 * truncated, the translation patched into H, ABSize, super-mode limits) in one fixed FP64 order
 * (estimate.chain_stages restates it).  The first pair without a homography leaves its stage and
 * every later one uncalibrated.  out: n_cams - 1 descriptors (mcs_plan_create's input).
 * Replaces the per-capture numpy geometry of estimate.chain_stages / geometry.stage_geometry. */
int mcs_chain_stages(int n_cams, const int *cam_w, const int *cam_h, const double *pair_H,
                     const int *pair_ok, int super_mode, mcs_stage_desc *out);

/* ---- A whole rig capture ---------------------------------------------------
 * Per capture, detectAndDescribe + matchKeypoints (StitcherClass.py:356-448) of every adjacent
 * camera pair, made per-frame by config 3: ORB of the n_cams device frames (dense w x h x
 * channels, sorted-label order), then per pair k (camera k+1 -> camera k: query k+1, train k)
 * BF Hamming kNN-2, Lowe's ratio (m0 < ratio * m1, strict), more than 4 matches, RANSAC + LM
 * (mcs_ransac_homography_host with thresh / iters / seed).  A job runs on libmcs's worker
 * threads: the whole capture as one launch chain on the job's stream (ORB batched over the
 * cameras, the pairs' matching, ratio test, RANSAC and best model batched over the pairs, one
 * copy back; the host runs only the LM refinement), or per-call steps for a capture whose ORB
 * ranking overflowed on the device.  submit returns at once, wait blocks for the result, so a
 * caller with several jobs overlaps one capture's estimation with another's.  wait_event (a
 * hipEvent_t or NULL): the frames' producer; the job's streams wait for it on the GPU.  Replaces the per-capture
 * Python loop over StitcherBase.detectAndDescribe / matchKeypoints (StitcherClass.py:356-448)
 * for config 3.  Results: H (n_cams - 1) x 9 row-major (0 where ok[k] = 0: the reference's
 * H = None), per camera keypoints, per pair ratio-test matches and RANSAC inliers (each may be
 * NULL).  A job holds one capture at a time; destroy waits for a running one. */
typedef struct mcs_rig_job mcs_rig_job;
int mcs_rig_job_create(int n_cams, int w, int h, int channels, int nfeatures, int nlevels,
                       float scale_factor, int fast_threshold, float ratio, double reproj_thresh,
                       int iters, uint32_t seed, int device, mcs_rig_job **out);
int mcs_rig_job_submit(mcs_rig_job *job, const uint8_t *const *d_frames, void *wait_event);
int mcs_rig_job_wait(mcs_rig_job *job, double *H, int *ok, int *n_keypoints, int *n_matches,
                     int *n_inliers);
/* wait + the capture's stitch, issued from libmcs (config 3 end to end, no caller code per
 * capture): the pairs the job estimated replace H_io / ok_io (n_cams - 1 pairs, in/out: a pair
 * whose estimate failed keeps the caller's -- the previous capture's -- homography, ok 0 and no
 * previous one: uncalibrated from that pair on), the chain geometry of mcs_chain_stages, a plan,
 * and mcs_stitch_direct of the submitted frames into d_out (rows out_pitch bytes apart, at most
 * out_capacity bytes) on `stream` (enqueued; the frames and d_out must stay valid until it has
 * run).  out_w / out_h: the mosaic's size.  Replaces estimate.CaptureEstimator.collect + stitch
 * (chain geometry and plan built per capture in Python). */
int mcs_rig_job_wait_stitch(mcs_rig_job *job, double *H_io, int *ok_io, int super_mode,
                            int interp, uint8_t *d_out, int64_t out_pitch, int64_t out_capacity,
                            void *stream, int *out_w, int *out_h, int *n_keypoints,
                            int *n_matches, int *n_inliers);
/* A job of n_captures captures at once (n_cams x n_captures <= MCS_MAX_CAMS): one launch chain
 * over all their cameras, so each launch carries n_captures times the work (the rig's captures
 * are independent; the results equal n_captures single-capture jobs bit for bit: no kernel of
 * the chain depends on a pair's index).  submit takes n_captures x n_cams frames, capture q's
 * cameras at q n_cams; wait returns capture-major arrays (H n_captures x (n_cams - 1) x 9,
 * n_keypoints n_captures x n_cams, ...); wait_stitch_batch stitches capture q into d_out[q]
 * (out_w / out_h per capture) with H_io / ok_io carried from capture to capture in order.
 * mcs_rig_job_create is create_batch with n_captures = 1; mcs_rig_job_wait_stitch refuses a
 * batch job. */
int mcs_rig_job_create_batch(int n_cams, int n_captures, int w, int h, int channels,
                             int nfeatures, int nlevels, float scale_factor, int fast_threshold,
                             float ratio, double reproj_thresh, int iters, uint32_t seed,
                             int device, mcs_rig_job **out);
int mcs_rig_job_wait_stitch_batch(mcs_rig_job *job, double *H_io, int *ok_io, int super_mode,
                                  int interp, uint8_t *const *d_out, int64_t out_pitch,
                                  int64_t out_capacity, void *stream, int *out_w, int *out_h,
                                  int *n_keypoints, int *n_matches, int *n_inliers);
/* Captures the job finished on the device path (one launch chain) and on the per-call path (a
 * device ranking overflow, or MCS_RIG_PATH=calls). */
int mcs_rig_job_counts(const mcs_rig_job *job, int *device_captures, int *call_captures);
int mcs_rig_job_destroy(mcs_rig_job *job);

/* ---- Multi-GPU group ---------------------------------------------------
 * One process per GPU of a node.  Rig captures are independent (capture f -> rank f mod N, each
 * rank stitching with its own plan, no collective in the stitch itself); the one collective is
 * the final mosaic gather to the consumer's rank, over RCCL (xGMI point-to-point links).  RCCL
 * is bound at run time like the HIP runtime: the librccl beside the runtime in the process
 * (PyTorch-ROCm's), else $MCS_RCCL_LIBRARY, else ROCm's.
 * unique_id: rank 0 creates the id (MCS_GROUP_ID_BYTES bytes) and hands it to every rank by any
 * means (a file, a socket, torch.distributed.broadcast_object_list); create: every rank, with
 * the same n_ranks and id, its own rank and device (collective: blocks until all joined).
 * gather: every rank's `bytes` contiguous bytes at d_mosaics (e.g. its F finished mosaics) to
 * rank `root`, which receives rank r's at d_recv + r * bytes (its own copied on the device);
 * non-roots pass d_recv = NULL.  One grouped send/recv, enqueued on `stream`. */
#define MCS_GROUP_ID_BYTES 128
typedef struct mcs_group mcs_group;
int mcs_group_unique_id(uint8_t *id);
int mcs_group_create(int n_ranks, int rank, const uint8_t *id, int device, mcs_group **out);
int mcs_group_gather(mcs_group *group, const uint8_t *d_mosaics, int64_t bytes, uint8_t *d_recv,
                     int root, void *stream);
int mcs_group_destroy(mcs_group *group);
/* Path (or soname) of the bound RCCL ("" when none was found). */
const char *mcs_rccl_library(void);

#ifdef __cplusplus
}
#endif

#endif /* MCS_H_ */
