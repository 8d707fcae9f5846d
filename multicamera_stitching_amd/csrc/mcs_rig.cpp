// mcs_rig.cpp -- config 3 estimation of a whole rig capture in libmcs:
// ORB of every camera frame, then per adjacent pair (camera k+1 -> camera k, k = 0 .. n-2)
// BF Hamming kNN-2, Lowe's ratio (strict, StitcherClass.py:432), more than 4 matches
// (:437), findHomography's RANSAC + LM (:440-441, mcs_ransac_homography_host).  The reference
// runs detectAndDescribe + matchKeypoints once at calibration (:356-448); config 3 runs them per
// capture.
//
// Device path (default): the whole capture is ONE launch chain on the job's own stream, with
// one host round trip -- the ORB kernels batched over the cameras (grid.y = camera), the pairs'
// kNN-2, ratio test + compaction, RANSAC hypotheses and best-model selection batched over the
// pairs (mcs_rig_* kernels, every count read on the device), then one copy back of the counts,
// best models, inlier masks and matched positions; the host only runs findHomography's LM
// refinement (mcs_refine.cpp) per pair.  The same kernels and arithmetic as the per-call entry
// points, so the same homographies, bit for bit.  The chain is captured once as a hipGraph and
// replayed while the job is fed the same frame pointers (one graph launch per capture; a new
// frame set re-captures it; MCS_RIG_GRAPH=0: plain launches).
//
// Per-call path (a capture whose ORB ranking overflowed on the device -- more than kOrbSelMax
// candidates on a level --, or MCS_RIG_PATH=calls): the C-ABI's own steps
// (mcs_orb_detect_device, mcs_match_hamming_knn2_host, mcs_ransac_homography_host -- each with
// its thread's device workspace and stream) issued from libmcs's worker threads: a job's camera
// ORBs side by side, a pair queued as soon as both of its cameras' ORBs are done, the last pair
// marks the job done.
//
// Either way a job runs on libmcs's worker threads and mcs_rig_job_submit returns at once, so a
// caller that keeps several jobs in flight overlaps one capture's estimation with another's.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <memory>
#include <functional>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "hip_rt.h"
#include "mcs_common.h"
#include "mcs_feat_int.h"
#include "mcs_orb_core.h"

namespace {

// Worker threads of libmcs (created on first use, never joined: they sleep on the queue).
class Pool {
public:
    static Pool &get()
    {
        // (sized for three captures in flight: one job's pairs beside two jobs' camera ORBs)
        static Pool *p = new Pool(12);
        return *p;
    }
    void run(std::function<void()> f)
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(std::move(f));
        }
        cv_.notify_one();
    }

private:
    explicit Pool(int n)
    {
        for (int i = 0; i < n; i++) std::thread([this] { loop(); }).detach();
    }
    void loop()
    {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [this] { return !q_.empty(); });
                f = std::move(q_.front());
                q_.pop_front();
            }
            f();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
};

struct Feat {
    std::vector<float> xy;
    std::vector<uint8_t> desc;
    int n = 0;
    int rc = MCS_OK;
    char err[256] = {0};
};

// Device state of the one-launch-chain path (allocated on the job's first capture).
struct RigDevice {
    bool ready = false;
    hipStream_t s = nullptr;
    uint8_t *buf = nullptr;      // device: every per-capture buffer
    uint8_t *host = nullptr;     // pinned: the copy-back blob
    size_t blob_bytes = 0;
    mcs::feat::OrbGeom geo;
    int K = 0;                   // keypoints per camera at most (the quotas' sum)
    unsigned pyr_blocks = 0, knn_qblocks = 0, knn_chunks = 0;
    size_t o_cnt = 0, cnt_bytes = 0, o_keys = 0, keys_bytes = 0, o_blob = 0;
    size_t o_sel = 0, o_info = 0, o_hbest = 0, o_mask = 0, o_pts = 0;   // within the blob
    mcs::KGrayArgs ga;
    mcs::KOrbBuildArgs ba;
    mcs::KOrbPyrArgs pa;
    mcs::KOrbSelArgs sa;
    mcs::KOrbDescArgs da;
    mcs::KRigArgs ra;
    // the chain captured as a hipGraph for the frame pointers it was captured with (a job is
    // usually fed the same frame set every time: one per capture slot in flight)
    hipGraphExec_t exec = nullptr;
    std::vector<const uint8_t *> graph_frames;
};

}  // namespace

struct mcs_rig_job {
    int n_cams, w, h, channels;
    // captures per job (mcs_rig_job_create_batch): the chain runs over ci = n_cams x n_caps
    // cameras, capture q's at q n_cams ..; the pairs across a capture boundary are computed with
    // the others and never reported
    int n_caps = 1, ci = 0;
    int nfeatures, nlevels, fast_threshold, iters;
    float scale_factor, ratio;
    double thresh;
    uint32_t seed;
    int device;
    // per submitted capture
    std::vector<const uint8_t *> frames;
    void *wait_event = nullptr;
    std::vector<Feat> feat;
    std::vector<double> H;            // (ci - 1) x 9
    std::vector<int> ok, n_matches, n_inliers;
    std::vector<int> prc;             // per pair status
    std::vector<std::string> perr;
    std::atomic<int> left{0};             // pairs not finished
    std::unique_ptr<std::atomic<int>[]> need;   // per pair: cameras whose ORB is still running
    std::mutex mu;
    std::condition_variable cv;
    bool busy = false, done = true;
    RigDevice dev;
    int captures_device = 0, captures_calls = 0;   // captures finished by each path
};

namespace {

void finish(mcs_rig_job *j)
{
    std::lock_guard<std::mutex> lk(j->mu);
    j->done = true;
    j->cv.notify_all();
}

// Pair k: camera k+1 (query, matchKeypoints' A) against camera k (train, B).
void pair_task(mcs_rig_job *j, int k)
{
    const Feat &fa = j->feat[k + 1], &fb = j->feat[k];
    double *H = j->H.data() + 9 * k;
    for (int i = 0; i < 9; i++) H[i] = 0.0;
    j->ok[k] = 0;
    j->n_matches[k] = j->n_inliers[k] = 0;
    int rc = fa.rc ? fa.rc : fb.rc;
    if (rc == MCS_OK && fa.n > 0 && fb.n > 0) {
        std::vector<int32_t> idx((size_t)fa.n * 2), dist((size_t)fa.n * 2);
        rc = mcs_match_hamming_knn2_host(fa.desc.data(), fa.n, fb.desc.data(), fb.n, idx.data(),
                                         dist.data(), j->device);
        std::vector<float> src, dst;
        if (rc == MCS_OK) {
            // Lowe's ratio, m0.distance < ratio * m1.distance (strict), in double as the
            // reference's Python float compare
            for (int q = 0; q < fa.n; q++) {
                if (idx[2 * q + 1] < 0) continue;
                if (!((double)dist[2 * q] < (double)dist[2 * q + 1] * (double)j->ratio)) continue;
                const int t = idx[2 * q];
                src.push_back(fa.xy[2 * q]);
                src.push_back(fa.xy[2 * q + 1]);
                dst.push_back(fb.xy[2 * t]);
                dst.push_back(fb.xy[2 * t + 1]);
            }
            j->n_matches[k] = (int)src.size() / 2;
        }
        if (rc == MCS_OK && j->n_matches[k] > 4) {
            int ninl = 0;
            rc = mcs_ransac_homography_host(src.data(), dst.data(), j->n_matches[k], j->thresh,
                                            j->iters, j->seed, H, nullptr, &ninl, j->device);
            if (rc == MCS_OK) {
                j->n_inliers[k] = ninl;
                j->ok[k] = ninl > 0;
            }
        }
    }
    j->prc[k] = rc;
    if (rc != MCS_OK) {
        const char *m = mcs_last_error();
        j->perr[k] = m ? m : "";
    }
    if (j->left.fetch_sub(1) == 1) finish(j);
}

void orb_task(mcs_rig_job *j, int c)
{
    Feat &f = j->feat[c];
    f.rc = MCS_OK;
    f.err[0] = 0;
    const int cap = std::max(j->nfeatures, 1);
    f.xy.resize((size_t)cap * 2);
    f.desc.resize((size_t)cap * 32);
    // the frames' producer (e.g. an upload on the caller's stream): ordered before this
    // thread's ORB stream on the GPU
    if (j->wait_event) f.rc = mcs::features_stream_wait(j->device, j->wait_event);
    if (f.rc == MCS_OK)
        f.rc = mcs_orb_detect_device(j->frames[c], j->w, j->h, j->channels, j->nfeatures,
                                     j->nlevels, j->scale_factor, j->fast_threshold, f.xy.data(),
                                     nullptr, nullptr, nullptr, f.desc.data(), &f.n, j->device);
    if (f.rc != MCS_OK) {
        const char *m = mcs_last_error();
        snprintf(f.err, sizeof(f.err), "%s", m ? m : "");
        f.n = 0;
    }
    // a pair starts as soon as both of its cameras' features are in (pair c - 1 and pair c use
    // camera c)
    for (int k = c - 1; k <= c; k++)
        if (k >= 0 && k < j->ci - 1 && j->need[k].fetch_sub(1) == 1)
            Pool::get().run([j, k] { pair_task(j, k); });
}

const mcs::rt::Api *api_for(int device, int *rc)
{
    const mcs::rt::Api *A = mcs::rt::api();
    *rc = A ? MCS_OK : MCS_E_HIP;
    return A;
}

// Sizes, offsets, stream and buffers of the device path; the argument blocks that do not change
// between captures.
int device_setup(mcs_rig_job *j)
{
    RigDevice &d = j->dev;
    int rc = MCS_OK;
    const mcs::rt::Api *A = api_for(j->device, &rc);
    if (rc) return rc;
    rc = mcs::feat::orb_geom(j->w, j->h, j->nfeatures, j->nlevels, j->scale_factor, &d.geo);
    if (rc) return rc;
    const mcs::feat::OrbGeom &g = d.geo;
    const int C = j->ci, P = j->ci - 1, L = j->nlevels;
    const int K = d.K = std::max(g.n_bound, 1);
    const size_t pix = g.off[L];
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += (bytes + 255) & ~(size_t)255;
        return at;
    };
    const size_t o_lvl = take(C * pix), o_blur = take(C * pix);
    const size_t o_cand = take(C * g.cap_total * sizeof(mcs::OrbCand));
    d.cnt_bytes = (size_t)C * mcs::kOrbMaxLevels * sizeof(int);
    d.o_cnt = take(d.cnt_bytes);
    const size_t o_kp = take((size_t)C * K * 3 * sizeof(int));
    const size_t o_resp = take((size_t)C * K * sizeof(double));
    const size_t o_desc = take((size_t)C * K * 32);
    const size_t o_or = take((size_t)C * K * 2 * sizeof(double));
    d.keys_bytes = (size_t)P * K * 2 * sizeof(uint32_t);
    d.o_keys = take(d.keys_bytes);
    const size_t o_hyps = take((size_t)P * j->iters * 8 * sizeof(double));
    const size_t o_scores = take((size_t)P * j->iters * sizeof(int32_t));
    // the copy-back blob, contiguous
    d.o_blob = o;
    size_t b = 0;
    auto btake = [&](size_t bytes) {
        const size_t at = b;
        b += (bytes + 255) & ~(size_t)255;
        return at;
    };
    d.o_sel = btake((size_t)C * 2 * sizeof(int));
    d.o_info = btake((size_t)P * 4 * sizeof(int));
    d.o_hbest = btake((size_t)P * 8 * sizeof(double));
    d.o_mask = btake((size_t)P * K);
    d.o_pts = btake((size_t)P * K * 4 * sizeof(double));
    d.blob_bytes = b;
    o += b;
    mcs::DeviceGuard dg(A, j->device);
    if (dg.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", j->device, A->hipGetErrorString(dg.err));
    HIP_TRY(A->hipStreamCreateWithFlags(&d.s, hipStreamNonBlocking));
    HIP_TRY(A->hipMalloc((void **)&d.buf, o));
    HIP_TRY(A->hipHostMalloc((void **)&d.host, d.blob_bytes, 0));
    uint8_t *B = d.buf, *blob = d.buf + d.o_blob;
    int *sel = reinterpret_cast<int *>(blob + d.o_sel);

    std::memset(&d.ga, 0, sizeof(d.ga));
    d.ga.gray = B + o_lvl;
    d.ga.stride = (int64_t)pix;
    d.ga.n = j->w * j->h;
    d.pyr_blocks = mcs::feat::pyramid_args(g, B + o_lvl, d.ba);
    d.ba.stride = (int64_t)pix;

    std::memset(&d.pa, 0, sizeof(d.pa));
    d.pa.img = B + o_lvl;
    d.pa.blur = B + o_blur;
    d.pa.cand = reinterpret_cast<mcs::OrbCand *>(B + o_cand);
    d.pa.ncand = reinterpret_cast<int *>(B + d.o_cnt);
    d.pa.nlevels = L;
    d.pa.threshold = j->fast_threshold;
    d.pa.stride = (int64_t)pix;
    d.pa.cstride = (int)g.cap_total;
    for (int l = 0; l < L; l++) {
        d.pa.off[l] = (int64_t)g.off[l];
        d.pa.coff[l] = (int)g.coff[l];
        d.pa.w[l] = g.lw[l];
        d.pa.h[l] = g.lh[l];
        d.pa.cap[l] = (int)g.cap[l];
        d.pa.bstart[l + 1] = d.pa.bstart[l] + (g.lw[l] + mcs::kOrbTileW - 1) / mcs::kOrbTileW *
                                                ((g.lh[l] + mcs::kOrbTileH - 1) / mcs::kOrbTileH);
    }

    std::memset(&d.sa, 0, sizeof(d.sa));
    d.sa.cand = d.pa.cand;
    d.sa.ncand = d.pa.ncand;
    d.sa.kp = reinterpret_cast<int *>(B + o_kp);
    d.sa.resp = reinterpret_cast<double *>(B + o_resp);
    d.sa.sel = sel;
    for (int l = 0; l < L; l++) {
        d.sa.coff[l] = (int)g.coff[l];
        d.sa.cap[l] = (int)g.cap[l];
        d.sa.quota[l] = g.quota[l];
    }
    d.sa.nlevels = L;
    d.sa.cstride = (int)g.cap_total;
    d.sa.kstride = K;

    std::memset(&d.da, 0, sizeof(d.da));
    for (int l = 0; l < mcs::kOrbMaxLevels; l++) {
        const int ll = l < L ? l : 0;
        d.da.img[l] = B + o_lvl + g.off[ll];
        d.da.blur[l] = B + o_blur + g.off[ll];
        d.da.w[l] = g.lw[ll];
    }
    d.da.kp = d.sa.kp;
    d.da.desc = B + o_desc;
    d.da.orient = reinterpret_cast<double *>(B + o_or);
    d.da.sel = sel;
    d.da.n = g.n_bound;
    d.da.kstride = K;
    d.da.stride = (int64_t)pix;

    std::memset(&d.ra, 0, sizeof(d.ra));
    d.ra.kp = d.sa.kp;
    d.ra.desc = B + o_desc;
    d.ra.sel = sel;
    d.ra.keys = reinterpret_cast<uint32_t *>(B + d.o_keys);
    d.ra.pts = reinterpret_cast<double *>(blob + d.o_pts);
    d.ra.info = reinterpret_cast<int *>(blob + d.o_info);
    d.ra.hyps = reinterpret_cast<double *>(B + o_hyps);
    d.ra.scores = reinterpret_cast<int32_t *>(B + o_scores);
    d.ra.mask = blob + d.o_mask;
    d.ra.hbest = reinterpret_cast<double *>(blob + d.o_hbest);
    for (int l = 0; l < L; l++) d.ra.lscale[l] = g.lscale[l];
    d.ra.ratio = (double)j->ratio;
    d.ra.t2 = j->thresh * j->thresh;
    d.ra.kstride = K;
    d.ra.iters = j->iters;
    d.ra.seed = j->seed;
    // kNN-2 blocks: query waves x train chunks x pairs, enough to fill the chip (as the per-call
    // matcher sizes them; the result does not depend on the chunking)
    d.knn_qblocks = (unsigned)((K + mcs::kKnnQueriesPerBlock - 1) / mcs::kKnnQueriesPerBlock);
    int chunks = (int)((mcs::kKnnTargetBlocks + d.knn_qblocks * P - 1) / (d.knn_qblocks * P));
    chunks = std::max(1, std::min(chunks, (K + 63) / 64));
    d.ra.per_chunk = (K + chunks - 1) / chunks;
    d.knn_chunks = (unsigned)((K + d.ra.per_chunk - 1) / d.ra.per_chunk);
    d.ready = true;
    return MCS_OK;
}

void device_release(mcs_rig_job *j)
{
    RigDevice &d = j->dev;
    const mcs::rt::Api *A = mcs::rt::api();
    if (!A) return;
    mcs::DeviceGuard dg(A, j->device);
    if (d.s) (void)A->hipStreamSynchronize(d.s);
    if (d.exec) (void)A->hipGraphExecDestroy(d.exec);
    if (d.buf) (void)A->hipFree(d.buf);
    if (d.host) (void)A->hipHostFree(d.host);
    if (d.s) (void)A->hipStreamDestroy(d.s);
    d = RigDevice();
}

// The per-capture resets (candidate counts, kNN-2 keys): stream-ordered memsets issued before
// the chain or its graph (measured: memset nodes captured into the graph did not reset the counts
// on replay -- the ranking then overflowed and every capture fell back to the per-call path).
int enqueue_resets(mcs_rig_job *j, const mcs::rt::Api *A, hipStream_t s)
{
    RigDevice &d = j->dev;
    HIP_TRY(A->hipMemsetAsync(d.buf + d.o_cnt, 0, d.cnt_bytes, s));
    HIP_TRY(A->hipMemsetAsync(d.buf + d.o_keys, 0xff, d.keys_bytes, s));
    return MCS_OK;
}

// The capture's launch chain on stream s (its one copy back included; after enqueue_resets):
// issued directly or recorded into the job's graph.  Every argument block lives in the job (a
// graph's kernel nodes keep their arguments for replays).
int enqueue_chain(mcs_rig_job *j, const mcs::rt::Api *A, const mcs::feat::FeatureKernels *k,
                  hipStream_t s)
{
    RigDevice &d = j->dev;
    using mcs::feat::launch;
    const int C = j->ci, P = j->ci - 1, L = j->nlevels;
    const mcs::feat::OrbGeom &g = d.geo;
    const size_t pix = g.off[L];
    int rc = MCS_OK;
    if (j->channels == 3) {
        for (int c = 0; c < C; c++) d.ga.bgr[c] = j->frames[c];
        rc = launch(A, k->orb_gray, (unsigned)((j->w * j->h + 1023) / 1024), C, 256, &d.ga,
                    sizeof(d.ga), s);
    } else {
        for (int c = 0; c < C; c++)
            HIP_TRY(A->hipMemcpyAsync(d.ga.gray + c * pix, j->frames[c], (size_t)j->w * j->h,
                                      hipMemcpyDeviceToDevice, s));
    }
    if (rc == MCS_OK && L > 1) {
        if (d.pyr_blocks > 0) {
            rc = launch(A, k->orb_pyramid, d.pyr_blocks, C, 256, &d.ba, sizeof(d.ba), s, 1,
                        (unsigned)(2 * d.ba.lds_w * d.ba.lds_h + 16));
        } else {
            for (int l = 1; l < L && rc == MCS_OK; l++)
                rc = mcs_resize_linear_device(d.ga.gray + g.off[l - 1], g.lw[l - 1], g.lh[l - 1],
                                              g.lw[l - 1], (int64_t)pix, d.ga.gray + g.off[l],
                                              g.lw[l], g.lh[l], g.lw[l], (int64_t)pix, 1, C,
                                              j->device, s);
        }
    }
    if (rc == MCS_OK)
        rc = launch(A, k->orb_level, (unsigned)d.pa.bstart[L], C, mcs::kOrbLevelThreads, &d.pa,
                    sizeof(d.pa), s);
    if (rc == MCS_OK)
        rc = launch(A, k->orb_select, (unsigned)L, C, mcs::kOrbSelThreads, &d.sa, sizeof(d.sa), s);
    if (rc == MCS_OK && g.n_bound > 0)
        rc = launch(A, k->orb_describe, (unsigned)g.n_bound, C, 64, &d.da, sizeof(d.da), s);
    if (rc == MCS_OK)
        rc = launch(A, k->rig_knn2, d.knn_qblocks, d.knn_chunks, mcs::kKnnLanes, &d.ra,
                    sizeof(d.ra), s, (unsigned)P);
    if (rc == MCS_OK) rc = launch(A, k->rig_match, (unsigned)P, 1, 1024, &d.ra, sizeof(d.ra), s);
    if (rc == MCS_OK)
        rc = launch(A, k->rig_hyp, (unsigned)((j->iters + 63) / 64), (unsigned)P, 64, &d.ra,
                    sizeof(d.ra), s);
    if (rc == MCS_OK)
        rc = launch(A, k->rig_ransac, (unsigned)j->iters, (unsigned)P, mcs::kRansacBlock, &d.ra,
                    sizeof(d.ra), s);
    if (rc == MCS_OK) rc = launch(A, k->rig_best, (unsigned)P, 1, 1024, &d.ra, sizeof(d.ra), s);
    if (rc == MCS_OK)
        HIP_TRY(A->hipMemcpyAsync(d.host, d.buf + d.o_blob, d.blob_bytes, hipMemcpyDeviceToHost,
                                  s));
    return rc;
}

// The capture's launch chain and its one copy back (see the file comment).  Returns MCS_OK
// with *overflow set when a camera's device ranking overflowed (nothing else is valid then).
int device_capture(mcs_rig_job *j, bool *overflow)
{
    *overflow = false;
    int rc = MCS_OK;
    const mcs::rt::Api *A = api_for(j->device, &rc);
    if (rc) return rc;
    if (!j->dev.ready && (rc = device_setup(j)) != MCS_OK) {
        device_release(j);   // (a partial setup: the next capture starts from clean state)
        return rc;
    }
    RigDevice &d = j->dev;
    const mcs::feat::FeatureKernels *k = nullptr;
    mcs::DeviceGuard dg(A, j->device);
    if (dg.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", j->device, A->hipGetErrorString(dg.err));
    if ((rc = mcs::feat::feature_kernels(A, j->device, &k)) != MCS_OK) return rc;
    const int C = j->ci, P = j->ci - 1;
    hipStream_t s = d.s;
    if (j->wait_event) HIP_TRY(A->hipStreamWaitEvent(s, (hipEvent_t)j->wait_event, 0));
    hipError_t e = hipSuccess;
    if ((rc = enqueue_resets(j, A, s)) != MCS_OK) return rc;
    if (d.pyr_blocks > 0) {
        if (!d.exec || d.graph_frames != j->frames) {
            if (d.exec) (void)A->hipGraphExecDestroy(d.exec);
            d.exec = nullptr;
            hipGraph_t graph = nullptr;
            HIP_TRY(A->hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            rc = enqueue_chain(j, A, k, s);
            const hipError_t ec = A->hipStreamEndCapture(s, &graph);
            if (rc == MCS_OK && ec != hipSuccess)
                rc = mcs::fail(MCS_E_HIP, "rig capture graph: %s", A->hipGetErrorString(ec));
            if (rc == MCS_OK) {
                const hipError_t ei =
                    A->hipGraphInstantiate(&d.exec, graph, nullptr, nullptr, 0);
                if (ei != hipSuccess) {
                    d.exec = nullptr;
                    rc = mcs::fail(MCS_E_HIP, "rig graph instantiate: %s",
                                   A->hipGetErrorString(ei));
                }
            }
            if (graph) (void)A->hipGraphDestroy(graph);
            if (rc) return rc;
            d.graph_frames = j->frames;
        }
        e = A->hipGraphLaunch(d.exec, s);
    } else {
        rc = enqueue_chain(j, A, k, s);
    }
    const hipError_t e2 = A->hipStreamSynchronize(s);   // (drains the queued work on error too)
    if (rc) return rc;
    if (e != hipSuccess || e2 != hipSuccess)
        return mcs::fail(MCS_E_HIP, "rig capture: %s",
                         A->hipGetErrorString(e != hipSuccess ? e : e2));
    const int *sel = reinterpret_cast<const int *>(d.host + d.o_sel);
    for (int c = 0; c < C; c++)
        if (sel[2 * c + 1]) {
            *overflow = true;
            return MCS_OK;
        }
    const int *info = reinterpret_cast<const int *>(d.host + d.o_info);
    const double *hbest = reinterpret_cast<const double *>(d.host + d.o_hbest);
    for (int c = 0; c < C; c++) j->feat[c].n = sel[2 * c], j->feat[c].rc = MCS_OK;
    std::vector<float> src, dst;
    for (int p = 0; p < P; p++) {
        double *H = j->H.data() + 9 * p;
        for (int i = 0; i < 9; i++) H[i] = 0.0;
        const int nm = info[4 * p], score = info[4 * p + 2];
        j->n_matches[p] = nm;
        j->n_inliers[p] = 0;
        j->ok[p] = 0;
        j->prc[p] = MCS_OK;
        if (nm <= 4 || score < 4) continue;
        // findHomography's refinement of the chosen model on its inliers (as
        // mcs_ransac_homography_host): the positions are floats carried as doubles
        const double *pts = reinterpret_cast<const double *>(d.host + d.o_pts) + 4 * (size_t)p * d.K;
        src.resize(2 * (size_t)nm);
        dst.resize(2 * (size_t)nm);
        for (int i = 0; i < nm; i++) {
            src[2 * i] = (float)pts[4 * i], src[2 * i + 1] = (float)pts[4 * i + 1];
            dst[2 * i] = (float)pts[4 * i + 2], dst[2 * i + 1] = (float)pts[4 * i + 3];
        }
        for (int i = 0; i < 8; i++) H[i] = hbest[8 * p + i];
        H[8] = 1.0;
        mcs::homography_refine(src.data(), dst.data(), nm, d.host + d.o_mask + (size_t)p * d.K, H);
        j->n_inliers[p] = score;
        j->ok[p] = 1;
    }
    return MCS_OK;
}

void start_calls(mcs_rig_job *j)
{
    j->left.store(j->ci - 1);
    for (int k = 0; k < j->ci - 1; k++) j->need[k].store(2);
    for (int c = 0; c < j->ci; c++) Pool::get().run([j, c] { orb_task(j, c); });
}

void capture_task(mcs_rig_job *j)
{
    bool overflow = false;
    const int rc = device_capture(j, &overflow);
    if (rc == MCS_OK && !overflow) {
        j->captures_device++;
        finish(j);
        return;
    }
    if (rc != MCS_OK) {
        // report through the pairs' status, as the per-call path does
        const char *m = mcs_last_error();
        for (int p = 0; p < j->ci - 1; p++) {
            j->prc[p] = rc;
            j->perr[p] = m ? m : "";
            j->ok[p] = 0;
        }
        for (auto &f : j->feat) f.rc = MCS_OK, f.n = 0;
        finish(j);
        return;
    }
    j->captures_calls++;
    start_calls(j);   // a ranking overflowed: the per-call path (host ranking) for this capture
}

}  // namespace

extern "C" {

int mcs_rig_job_create_batch(int n_cams, int n_captures, int w, int h, int channels,
                             int nfeatures, int nlevels, float scale_factor, int fast_threshold,
                             float ratio, double reproj_thresh, int iters, uint32_t seed,
                             int device, mcs_rig_job **out)
{
    mcs::clear_error();
    if (!out) return mcs::fail(MCS_E_INVALID, "NULL out");
    *out = nullptr;
    if (n_cams < 2 || n_cams > MCS_MAX_CAMS || n_captures < 1 ||
        n_cams * n_captures > MCS_MAX_CAMS || w < 1 || h < 1 ||
        (channels != 1 && channels != 3) || nfeatures < 1 || nlevels < 1 ||
        nlevels > mcs::kOrbMaxLevels || iters < 1 || iters > (1 << 20) ||
        !(ratio > 0.f) || !(reproj_thresh >= 0.0))
        return mcs::fail(MCS_E_INVALID, "n_cams %d x %d captures, %dx%dx%d, nfeatures %d, iters %d",
                         n_cams, n_captures, w, h, channels, nfeatures, iters);
    mcs_rig_job *j = new (std::nothrow) mcs_rig_job();
    if (!j) return mcs::fail(MCS_E_NOMEM, "rig job");
    const int ci = n_cams * n_captures;
    j->n_cams = n_cams, j->n_caps = n_captures, j->ci = ci;
    j->w = w, j->h = h, j->channels = channels;
    j->nfeatures = nfeatures, j->nlevels = nlevels, j->fast_threshold = fast_threshold;
    j->iters = iters, j->scale_factor = scale_factor, j->ratio = ratio;
    j->thresh = reproj_thresh, j->seed = seed, j->device = device;
    j->feat.resize(ci);
    j->H.assign(9 * (size_t)(ci - 1), 0.0);
    j->ok.assign(ci - 1, 0);
    j->n_matches.assign(ci - 1, 0);
    j->n_inliers.assign(ci - 1, 0);
    j->prc.assign(ci - 1, MCS_OK);
    j->perr.assign(ci - 1, std::string());
    j->need.reset(new (std::nothrow) std::atomic<int>[ci - 1]);
    if (!j->need) {
        delete j;
        return mcs::fail(MCS_E_NOMEM, "rig job");
    }
    *out = j;
    return MCS_OK;
}

int mcs_rig_job_create(int n_cams, int w, int h, int channels, int nfeatures, int nlevels,
                       float scale_factor, int fast_threshold, float ratio, double reproj_thresh,
                       int iters, uint32_t seed, int device, mcs_rig_job **out)
{
    return mcs_rig_job_create_batch(n_cams, 1, w, h, channels, nfeatures, nlevels, scale_factor,
                                    fast_threshold, ratio, reproj_thresh, iters, seed, device, out);
}

int mcs_rig_job_submit(mcs_rig_job *j, const uint8_t *const *d_frames, void *wait_event)
{
    mcs::clear_error();
    if (!j || !d_frames) return mcs::fail(MCS_E_INVALID, "NULL job/frames");
    {
        std::lock_guard<std::mutex> lk(j->mu);
        if (j->busy && !j->done) return mcs::fail(MCS_E_INVALID, "job still running");
        j->busy = true;
        j->done = false;
    }
    j->frames.assign(d_frames, d_frames + j->ci);
    j->wait_event = wait_event;
    Pool::get().run([j] { capture_task(j); });
    return MCS_OK;
}

int mcs_rig_job_wait(mcs_rig_job *j, double *H, int *ok, int *n_keypoints, int *n_matches,
                     int *n_inliers)
{
    mcs::clear_error();
    if (!j) return mcs::fail(MCS_E_INVALID, "NULL job");
    {
        std::unique_lock<std::mutex> lk(j->mu);
        if (!j->busy) return mcs::fail(MCS_E_INVALID, "no capture submitted");
        j->cv.wait(lk, [j] { return j->done; });
        j->busy = false;
    }
    // capture q's pair k is chain pair q n_cams + k (the pair across the boundary is skipped)
    const int N = j->n_cams, np = N - 1;
    for (int q = 0; q < j->n_caps; q++)
        for (int k = 0; k < np; k++) {
            const int p = q * N + k, o = q * np + k;
            if (H) std::memcpy(H + 9 * o, j->H.data() + 9 * p, sizeof(double) * 9);
            if (ok) ok[o] = j->ok[p];
            if (n_matches) n_matches[o] = j->n_matches[p];
            if (n_inliers) n_inliers[o] = j->n_inliers[p];
        }
    for (int c = 0; c < j->ci; c++) {
        if (n_keypoints) n_keypoints[c] = j->feat[c].n;
        if (j->feat[c].rc) return mcs::fail(j->feat[c].rc, "camera %d ORB: %s", c, j->feat[c].err);
    }
    for (int q = 0; q < j->n_caps; q++)
        for (int k = 0; k < np; k++) {
            const int p = q * N + k;
            if (j->prc[p]) return mcs::fail(j->prc[p], "pair %d: %s", p, j->perr[p].c_str());
        }
    return MCS_OK;
}

int mcs_rig_job_wait_stitch_batch(mcs_rig_job *j, double *H_io, int *ok_io, int super_mode,
                                  int interp, uint8_t *const *d_out, int64_t out_pitch,
                                  int64_t out_capacity, void *stream, int *out_w, int *out_h,
                                  int *n_keypoints, int *n_matches, int *n_inliers)
{
    mcs::clear_error();
    if (!j || !H_io || !ok_io || !d_out || !out_w || !out_h)
        return mcs::fail(MCS_E_INVALID, "mcs_rig_job_wait_stitch: NULL argument");
    const int N = j->n_cams, np = N - 1;
    std::vector<double> H(9 * (size_t)np * j->n_caps);
    std::vector<int> ok((size_t)np * j->n_caps);
    int rc = mcs_rig_job_wait(j, H.data(), ok.data(), n_keypoints, n_matches, n_inliers);
    if (rc) return rc;
    for (int q = 0; q < j->n_caps; q++) {
        if (!d_out[q]) return mcs::fail(MCS_E_INVALID, "mcs_rig_job_wait_stitch: NULL output %d", q);
        // a pair whose estimate failed keeps the caller's -- the previous capture's -- homography
        for (int k = 0; k < np; k++)
            if (ok[q * np + k]) {
                std::memcpy(H_io + 9 * k, H.data() + 9 * ((size_t)q * np + k), sizeof(double) * 9);
                ok_io[k] = 1;
            }
        mcs_stage_desc st[MCS_MAX_CAMS];
        int cw[MCS_MAX_CAMS], ch[MCS_MAX_CAMS];
        for (int c = 0; c < N; c++) cw[c] = j->w, ch[c] = j->h;
        rc = mcs_chain_stages(N, cw, ch, H_io, ok_io, super_mode, st);
        if (rc) return rc;
        mcs_plan *plan = nullptr;
        rc = mcs_plan_create(st, np, j->w, j->h, j->channels, interp, j->device, &plan);
        if (rc) return rc;
        int w = 0, h = 0, c = 0;
        rc = mcs_plan_out_shape(plan, &w, &h, &c);
        if (rc == MCS_OK && ((int64_t)w * c > out_pitch || (int64_t)h * out_pitch > out_capacity))
            rc = mcs::fail(MCS_E_SHAPE, "mosaic %d x %d does not fit the output (pitch %lld, "
                           "%lld bytes)", w, h, (long long)out_pitch, (long long)out_capacity);
        if (rc == MCS_OK) {
            int64_t fs[MCS_MAX_CAMS];
            for (int i = 0; i < N; i++) fs[i] = (int64_t)j->w * j->h * j->channels;
            // (the plan's geometry travels in the kernel arguments: it may go right after the
            // launch)
            rc = mcs_stitch_direct(plan, j->frames.data() + (size_t)q * N, fs, d_out[q], out_pitch,
                                   out_pitch * h, 1, stream);
        }
        mcs_plan_destroy(plan);
        out_w[q] = w;
        out_h[q] = h;
        if (rc) return rc;
    }
    return MCS_OK;
}

int mcs_rig_job_wait_stitch(mcs_rig_job *j, double *H_io, int *ok_io, int super_mode, int interp,
                            uint8_t *d_out, int64_t out_pitch, int64_t out_capacity, void *stream,
                            int *out_w, int *out_h, int *n_keypoints, int *n_matches,
                            int *n_inliers)
{
    if (j && j->n_caps != 1)
        return mcs::fail(MCS_E_INVALID, "mcs_rig_job_wait_stitch: a %d-capture job needs "
                         "mcs_rig_job_wait_stitch_batch", j->n_caps);
    return mcs_rig_job_wait_stitch_batch(j, H_io, ok_io, super_mode, interp, &d_out, out_pitch,
                                         out_capacity, stream, out_w, out_h, n_keypoints,
                                         n_matches, n_inliers);
}

int mcs_rig_job_counts(const mcs_rig_job *j, int *device_captures, int *call_captures)
{
    mcs::clear_error();
    if (!j) return mcs::fail(MCS_E_INVALID, "NULL job");
    if (device_captures) *device_captures = j->captures_device;
    if (call_captures) *call_captures = j->captures_calls;
    return MCS_OK;
}

int mcs_rig_job_destroy(mcs_rig_job *j)
{
    if (!j) return MCS_OK;
    {
        std::unique_lock<std::mutex> lk(j->mu);
        j->cv.wait(lk, [j] { return j->done; });   // never free a job the workers still use
    }
    device_release(j);
    delete j;
    return MCS_OK;
}

}  // extern "C"
