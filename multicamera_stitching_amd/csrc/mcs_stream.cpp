// mcs_stream.cpp -- host-frame streaming pipeline over a plan:
// double-(or deeper-)buffered pinned staging, H2D on one copy stream, the stitch (captured once
// per slot into a hipGraph) on the compute stream, D2H on a second copy stream, so that the
// upload of capture i+1, the stitch of capture i and the download of capture i-1 overlap.  Uses
// only the public plan API (mcs_stitch_device) plus the bound HIP runtime.
#include <sched.h>

#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "mcs_common.h"

namespace {
constexpr int kMaxDepth = 8;

// Host staging copies (caller frames -> pinned slot, pinned slot -> caller mosaic) split over a
// few worker threads: one thread's memcpy into pinned memory runs at ~30 GB/s, under the PCIe
// link it feeds (round 3: the non-zero-copy C5 path reached 0.27 of the link), so the
// double-buffered H2D pipeline needs several.  Chunks of >= kCopyChunk bytes.
constexpr size_t kCopyChunk = 2u << 20;

class CopyPool {
public:
    static CopyPool &get()
    {
        static CopyPool *p = new (std::nothrow) CopyPool(workers());
        static CopyPool serial(0);   // (the pool itself could not be allocated)
        return p ? *p : serial;
    }
    int size() const { return n_; }
    // Runs every copy job -- `rows` rows of `row` bytes, dense at dst, src_pitch apart at src --
    // the calling thread taking a share, and returns when all are done.
    struct Job {
        uint8_t *dst;
        const uint8_t *src;
        size_t row, rows, src_pitch;
    };
    // Never throws (it runs inside extern "C" entry points): when the chunk list or a helper
    // cannot be allocated, the jobs the helpers did not take are copied on the calling thread.
    void copy(const Job *jobs, int n_jobs) noexcept
    {
        std::vector<Job> chunks;   // pieces of about kCopyChunk bytes
        try {
            for (int k = 0; k < n_jobs; k++) {
                const Job &j = jobs[k];
                if (j.src_pitch == j.row) {
                    const size_t bytes = j.row * j.rows;
                    for (size_t o = 0; o < bytes; o += kCopyChunk)
                        chunks.push_back({j.dst + o, j.src + o, std::min(kCopyChunk, bytes - o),
                                          1, 0});
                    continue;
                }
                const size_t per = std::max<size_t>(1, kCopyChunk / std::max<size_t>(j.row, 1));
                for (size_t r = 0; r < j.rows; r += per)
                    chunks.push_back({j.dst + r * j.row, j.src + r * j.src_pitch, j.row,
                                      std::min(per, j.rows - r), j.src_pitch});
            }
        } catch (...) {
            for (int k = 0; k < n_jobs; k++) one(jobs[k]);
            return;
        }
        if (chunks.size() <= 1 || n_ == 0) {
            for (const Job &c : chunks) one(c);
            return;
        }
        std::atomic<size_t> next{0};
        int left = 0;
        std::mutex m;
        std::condition_variable done;
        auto work = [&] {
            for (size_t i; (i = next.fetch_add(1)) < chunks.size();) one(chunks[i]);
        };
        const int helpers = (int)std::min<size_t>((size_t)n_, chunks.size() - 1);
        for (int h = 0; h < helpers; h++) {
            {
                std::lock_guard<std::mutex> lk(m);
                left++;
            }
            if (!run([&] {
                    work();
                    std::lock_guard<std::mutex> lk(m);
                    if (--left == 0) done.notify_one();
                })) {
                std::lock_guard<std::mutex> lk(m);
                left--;
                break;
            }
        }
        work();   // (takes whatever the helpers have not)
        std::unique_lock<std::mutex> lk(m);
        done.wait(lk, [&] { return left == 0; });
    }

private:
    static void one(const Job &c)
    {
        for (size_t r = 0; r < c.rows; r++)
            memcpy(c.dst + r * c.row, c.src + r * c.src_pitch, c.row);
    }
public:
    static int workers()
    {
        // the CPUs this process may run on: the affinity set, bounded by the cgroup's CPU quota
        // (the GPU box reports an affinity of every CPU of the machine but a quota of 16), shared
        // by the ranks of this node (LOCAL_WORLD_SIZE, set by torch.distributed.run: one process
        // per GPU, every rank with its own pool), capped at 7 helpers -- a handful of memcpy
        // threads saturate the host memory the link reads
        cpu_set_t set;
        int cpus = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 1;
        if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = {};
            long period = 0;
            if (fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
                const long quota = (atol(q) + period / 2) / period;
                if (quota >= 1 && quota < cpus) cpus = (int)quota;
            }
            fclose(f);
        }
        if (const char *e = getenv("LOCAL_WORLD_SIZE")) {
            const int ranks = atoi(e);
            if (ranks > 1) cpus = std::max(1, cpus / ranks);
        }
        return std::max(0, std::min(7, cpus / 2 - 1));
    }

private:
    // helper threads that could be started (a failed std::thread leaves the pool smaller)
    explicit CopyPool(int n) : n_(0)
    {
        for (int i = 0; i < n; i++) {
            try {
                std::thread([this] { loop(); }).detach();
                n_++;
            } catch (...) {
                break;
            }
        }
    }
    // (the std::function is built inside the try: a capturing lambda larger than its small
    // buffer allocates, and a bad_alloc must not escape this noexcept path)
    template <class F>
    bool run(F &&fn) noexcept
    {
        try {
            std::function<void()> f(std::forward<F>(fn));
            {
                std::lock_guard<std::mutex> lk(mu_);
                q_.push_back(std::move(f));
            }
            cv_.notify_one();
            return true;
        } catch (...) {
            return false;
        }
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
    int n_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
};
}

struct mcs_stream {
    mcs_plan *plan = nullptr;
    int device = 0, depth = 0, channels = 0, n_cams = 0, next = 0;
    bool graphs = false;
    int cam_w[MCS_MAX_CAMS] = {}, cam_h[MCS_MAX_CAMS] = {};
    size_t cam_off[MCS_MAX_CAMS] = {};
    size_t in_bytes = 0, out_bytes = 0;
    int out_w = 0, out_h = 0;
    hipStream_t up = nullptr, compute = nullptr, down = nullptr;
    struct Slot {
        uint8_t *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
        hipEvent_t ev_in = nullptr, ev_k = nullptr, ev_out = nullptr;
        hipGraphExec_t exec = nullptr;
        bool busy = false;
    } slot[kMaxDepth];
};

namespace {

using mcs::rt::Api;

int stitch_slot(mcs_stream *s, int i, hipStream_t st)
{
    const uint8_t *cams[MCS_MAX_CAMS];
    int64_t strides[MCS_MAX_CAMS];
    for (int c = 0; c < s->n_cams; c++) {
        cams[c] = s->slot[i].d_in + s->cam_off[c];
        strides[c] = (int64_t)s->cam_w[c] * s->cam_h[c] * s->channels;
    }
    const int64_t pitch = (int64_t)s->out_w * s->channels;
    return mcs_stitch_device(s->plan, cams, strides, s->slot[i].d_out, pitch,
                             pitch * s->out_h, 1, st);
}

void release(const Api *A, mcs_stream *s)
{
    for (void *q : {(void *)s->up, (void *)s->compute, (void *)s->down})
        if (q) (void)A->hipStreamSynchronize((hipStream_t)q);
    for (int i = 0; i < kMaxDepth; i++) {
        mcs_stream::Slot &sl = s->slot[i];
        if (sl.exec) (void)A->hipGraphExecDestroy(sl.exec);
        if (sl.h_in) (void)A->hipHostFree(sl.h_in);
        if (sl.h_out) (void)A->hipHostFree(sl.h_out);
        if (sl.d_in) (void)A->hipFree(sl.d_in);
        if (sl.d_out) (void)A->hipFree(sl.d_out);
        for (hipEvent_t e : {sl.ev_in, sl.ev_k, sl.ev_out})
            if (e) (void)A->hipEventDestroy(e);
    }
    for (hipStream_t q : {s->up, s->compute, s->down})
        if (q) (void)A->hipStreamDestroy(q);
}

int build(const Api *A, mcs_stream *s)
{
    HIP_TRY(A->hipStreamCreateWithFlags(&s->up, hipStreamNonBlocking));
    HIP_TRY(A->hipStreamCreateWithFlags(&s->compute, hipStreamNonBlocking));
    HIP_TRY(A->hipStreamCreateWithFlags(&s->down, hipStreamNonBlocking));
    for (int i = 0; i < s->depth; i++) {
        mcs_stream::Slot &sl = s->slot[i];
        HIP_TRY(A->hipHostMalloc((void **)&sl.h_in, s->in_bytes, 0));
        HIP_TRY(A->hipHostMalloc((void **)&sl.h_out, s->out_bytes, 0));
        HIP_TRY(A->hipMalloc((void **)&sl.d_in, s->in_bytes));
        HIP_TRY(A->hipMalloc((void **)&sl.d_out, s->out_bytes));
        HIP_TRY(A->hipEventCreateWithFlags(&sl.ev_in, hipEventDisableTiming));
        HIP_TRY(A->hipEventCreateWithFlags(&sl.ev_k, hipEventDisableTiming));
        HIP_TRY(A->hipEventCreateWithFlags(&sl.ev_out, hipEventDisableTiming));
    }
    // tables, modules and side streams exist before any capture: one plain run
    int rc = mcs_plan_prepare(s->plan, s->compute);
    if (rc == MCS_OK) rc = stitch_slot(s, 0, s->compute);
    if (rc) return rc;
    HIP_TRY(A->hipStreamSynchronize(s->compute));
    if (!s->graphs) return MCS_OK;
    for (int i = 0; i < s->depth; i++) {
        hipGraph_t g = nullptr;
        HIP_TRY(A->hipStreamBeginCapture(s->compute, hipStreamCaptureModeThreadLocal));
        rc = stitch_slot(s, i, s->compute);
        const hipError_t e = A->hipStreamEndCapture(s->compute, &g);
        if (rc) {
            if (g) (void)A->hipGraphDestroy(g);
            return rc;
        }
        if (e != hipSuccess)
            return mcs::fail(MCS_E_HIP, "stream capture: %s", A->hipGetErrorString(e));
        const hipError_t e2 = A->hipGraphInstantiate(&s->slot[i].exec, g, nullptr, nullptr, 0);
        (void)A->hipGraphDestroy(g);
        if (e2 != hipSuccess)
            return mcs::fail(MCS_E_HIP, "graph instantiate: %s", A->hipGetErrorString(e2));
    }
    return MCS_OK;
}

}  // namespace

extern "C" {

int mcs_stream_copy_workers(void) { return CopyPool::workers(); }

int mcs_stream_create(mcs_plan *plan, int depth, int use_graphs, mcs_stream **out)
{
    mcs::clear_error();
    if (!plan || !out) return mcs::fail(MCS_E_INVALID, "NULL plan/out");
    *out = nullptr;
    if (depth < 1 || depth > kMaxDepth)
        return mcs::fail(MCS_E_INVALID, "depth %d (1..%d)", depth, kMaxDepth);
    mcs_flat_desc fd;
    int rc = mcs_plan_describe(plan, &fd);
    if (rc) return rc;
    if (fd.out_w <= 0 || fd.out_h <= 0) return mcs::fail(MCS_E_SHAPE, "empty mosaic");
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    // streams, pinned slots and device buffers live on the plan's device, whatever device the
    // caller has current (the stitch itself switches to plan->device)
    const int dev = mcs::plan_device(plan);
    mcs::DeviceGuard g(A, dev);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "device %d: %s", dev, A->hipGetErrorString(g.err));
    mcs_stream *s = new (std::nothrow) mcs_stream();
    if (!s) return mcs::fail(MCS_E_NOMEM, "stream");
    s->device = dev;
    s->plan = plan;
    s->depth = depth;
    s->graphs = use_graphs != 0;
    s->channels = fd.channels;
    s->n_cams = fd.n_cams;
    for (int c = 0; c < fd.n_cams; c++) {
        s->cam_w[c] = fd.cam_w[c];
        s->cam_h[c] = fd.cam_h[c];
        s->cam_off[c] = s->in_bytes;
        s->in_bytes += ((size_t)fd.cam_w[c] * fd.cam_h[c] * fd.channels + 255) & ~(size_t)255;
    }
    s->out_w = fd.out_w;
    s->out_h = fd.out_h;
    s->out_bytes = (size_t)fd.out_w * fd.out_h * fd.channels;
    rc = build(A, s);
    if (rc) {
        release(A, s);
        delete s;
        return rc;
    }
    *out = s;
    return MCS_OK;
}

uint8_t *mcs_stream_input(mcs_stream *s, int slot, int cam)
{
    if (!s || slot < 0 || slot >= s->depth || cam < 0 || cam >= s->n_cams) return nullptr;
    return s->slot[slot].h_in + s->cam_off[cam];
}

const uint8_t *mcs_stream_output(const mcs_stream *s, int slot)
{
    if (!s || slot < 0 || slot >= s->depth) return nullptr;
    return s->slot[slot].h_out;
}

int mcs_stream_next_slot(const mcs_stream *s)
{
    if (!s) return mcs::fail(MCS_E_INVALID, "NULL stream");
    return s->slot[s->next].busy ? mcs::fail(MCS_E_INVALID, "slot %d not yet collected (call "
                                             "mcs_stream_wait)", s->next)
                                 : s->next;
}

int mcs_stream_submit(mcs_stream *s, const uint8_t *const *cams, int *slot_out)
{
    return mcs_stream_submit_strided(s, cams, nullptr, slot_out);
}

int mcs_stream_submit_strided(mcs_stream *s, const uint8_t *const *cams,
                              const int64_t *row_pitch, int *slot_out)
{
    mcs::clear_error();
    if (!s) return mcs::fail(MCS_E_INVALID, "NULL stream");
    if (cams && row_pitch)
        for (int c = 0; c < s->n_cams; c++)
            if (cams[c] && row_pitch[c] < (int64_t)s->cam_w[c] * s->channels)
                return mcs::fail(MCS_E_INVALID, "camera %d: row pitch %lld < %d", c,
                                 (long long)row_pitch[c], s->cam_w[c] * s->channels);
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    const int i = s->next;
    mcs_stream::Slot &sl = s->slot[i];
    if (sl.busy)
        return mcs::fail(MCS_E_INVALID, "slot %d not yet collected (call mcs_stream_wait)", i);
    mcs::DeviceGuard g(A, s->device);
    if (cams) {   // else: the caller filled mcs_stream_input() buffers in place
        // (a camera inside a wider frame, e.g. the main_stream layout with cameras side by side
        // on axis 1, is gathered row by row into its dense staging slot)
        CopyPool::Job jobs[MCS_MAX_CAMS];
        int n_jobs = 0;
        for (int c = 0; c < s->n_cams; c++) {
            if (!cams[c]) continue;
            const size_t row = (size_t)s->cam_w[c] * s->channels;
            jobs[n_jobs++] = {sl.h_in + s->cam_off[c], cams[c], row, (size_t)s->cam_h[c],
                              row_pitch ? (size_t)row_pitch[c] : row};
        }
        CopyPool::get().copy(jobs, n_jobs);
    }
    HIP_TRY(A->hipMemcpyAsync(sl.d_in, sl.h_in, s->in_bytes, hipMemcpyHostToDevice, s->up));
    HIP_TRY(A->hipEventRecord(sl.ev_in, s->up));
    HIP_TRY(A->hipStreamWaitEvent(s->compute, sl.ev_in, 0));
    if (s->graphs) {
        HIP_TRY(A->hipGraphLaunch(sl.exec, s->compute));
    } else {
        const int rc = stitch_slot(s, i, s->compute);
        if (rc) return rc;
    }
    HIP_TRY(A->hipEventRecord(sl.ev_k, s->compute));
    HIP_TRY(A->hipStreamWaitEvent(s->down, sl.ev_k, 0));
    HIP_TRY(A->hipMemcpyAsync(sl.h_out, sl.d_out, s->out_bytes, hipMemcpyDeviceToHost, s->down));
    HIP_TRY(A->hipEventRecord(sl.ev_out, s->down));
    sl.busy = true;
    s->next = (i + 1) % s->depth;
    if (slot_out) *slot_out = i;
    return MCS_OK;
}

int mcs_stream_wait(mcs_stream *s, int slot, uint8_t *out)
{
    mcs::clear_error();
    if (!s || slot < 0 || slot >= s->depth) return mcs::fail(MCS_E_INVALID, "stream/slot");
    mcs_stream::Slot &sl = s->slot[slot];
    if (!sl.busy) return mcs::fail(MCS_E_INVALID, "slot %d has no capture in flight", slot);
    const Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    mcs::DeviceGuard g(A, s->device);
    HIP_TRY(A->hipEventSynchronize(sl.ev_out));
    if (out) {
        const CopyPool::Job job = {out, sl.h_out, s->out_bytes, 1, s->out_bytes};
        CopyPool::get().copy(&job, 1);
    }
    sl.busy = false;
    return MCS_OK;
}

int mcs_stream_destroy(mcs_stream *s)
{
    if (!s) return MCS_OK;
    const Api *A = mcs::rt::api();
    if (A) {
        mcs::DeviceGuard g(A, s->device);
        release(A, s);
    }
    delete s;
    return MCS_OK;
}

}  // extern "C"
