// mcs_group.cpp -- the multi-GPU boundary (include/mcs.h "Multi-GPU group"): an RCCL
// communicator over the GPUs of one node, one process per GPU, and the final mosaic gather of
// SURVEY.md 8e -- rig captures are independent (capture f -> rank f mod N), so the only
// collective on the path delivers the finished mosaics to the consumer's rank.
//
// Like the HIP runtime (hip_rt.h), RCCL is bound at run time, never linked: the librccl that
// belongs to the HIP runtime already in the process (PyTorch-ROCm ships both side by side), else
// $MCS_RCCL_LIBRARY, else ROCm's.  Only the handful of entry points below are used, with their
// C types restated (RCCL's ABI: ncclResult_t / ncclDataType_t are ints, ncclComm_t a pointer,
// ncclUniqueId 128 bytes).
#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>

#include "hip_rt.h"
#include "mcs_common.h"

namespace {

typedef int nccl_result;            // ncclResult_t: 0 = ncclSuccess
typedef void *nccl_comm;            // ncclComm_t
struct nccl_id {                    // ncclUniqueId
    char internal[MCS_GROUP_ID_BYTES];
};
constexpr int kNcclUint8 = 1;       // ncclDataType_t ncclUint8

struct Rccl {
    nccl_result (*GetUniqueId)(nccl_id *);
    nccl_result (*CommInitRank)(nccl_comm *, int, nccl_id, int);
    nccl_result (*CommDestroy)(nccl_comm);
    nccl_result (*Send)(const void *, size_t, int, int, nccl_comm, hipStream_t);
    nccl_result (*Recv)(void *, size_t, int, int, nccl_comm, hipStream_t);
    nccl_result (*GroupStart)();
    nccl_result (*GroupEnd)();
    const char *(*GetErrorString)(nccl_result);
};

Rccl g_rccl;
bool g_rccl_ok = false;
std::once_flag g_rccl_once;
std::string g_rccl_err, g_rccl_name;

void *open_rccl(const mcs::rt::Api *A)
{
    // 1. already in the process (e.g. torch.distributed's nccl backend)
    for (const char *n : {"librccl.so", "librccl.so.1"})
        if (void *h = dlopen(n, RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL)) {
            g_rccl_name = n;
            return h;
        }
    // 2. explicit choice
    if (const char *p = getenv("MCS_RCCL_LIBRARY")) {
        if (void *h = dlopen(p, RTLD_NOW | RTLD_GLOBAL)) {
            g_rccl_name = p;
            return h;
        }
        g_rccl_err = std::string("dlopen($MCS_RCCL_LIBRARY=") + p + "): " + dlerror();
        return nullptr;
    }
    // 3. next to the bound HIP runtime (the RCCL built against it), then ROCm's
    Dl_info info;
    if (A && dladdr(reinterpret_cast<void *>(A->hipGetDevice), &info) && info.dli_fname) {
        std::string dir(info.dli_fname);
        const size_t slash = dir.rfind('/');
        if (slash != std::string::npos) {
            const std::string path = dir.substr(0, slash) + "/librccl.so";
            if (void *h = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL)) {
                g_rccl_name = path;
                return h;
            }
        }
    }
    for (const char *n : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "/opt/rocm/lib/librccl.so"})
        if (void *h = dlopen(n, RTLD_NOW | RTLD_GLOBAL)) {
            g_rccl_name = n;
            return h;
        }
    g_rccl_err = std::string("no RCCL found (librccl): ") + dlerror();
    return nullptr;
}

void bind_rccl(const mcs::rt::Api *A)
{
    void *h = open_rccl(A);
    if (!h) return;
    auto sym = [&](const char *name) {
        void *f = dlsym(h, name);
        if (!f && g_rccl_err.empty()) g_rccl_err = g_rccl_name + " lacks " + name;
        return f;
    };
    g_rccl.GetUniqueId = reinterpret_cast<decltype(g_rccl.GetUniqueId)>(sym("ncclGetUniqueId"));
    g_rccl.CommInitRank = reinterpret_cast<decltype(g_rccl.CommInitRank)>(sym("ncclCommInitRank"));
    g_rccl.CommDestroy = reinterpret_cast<decltype(g_rccl.CommDestroy)>(sym("ncclCommDestroy"));
    g_rccl.Send = reinterpret_cast<decltype(g_rccl.Send)>(sym("ncclSend"));
    g_rccl.Recv = reinterpret_cast<decltype(g_rccl.Recv)>(sym("ncclRecv"));
    g_rccl.GroupStart = reinterpret_cast<decltype(g_rccl.GroupStart)>(sym("ncclGroupStart"));
    g_rccl.GroupEnd = reinterpret_cast<decltype(g_rccl.GroupEnd)>(sym("ncclGroupEnd"));
    g_rccl.GetErrorString =
        reinterpret_cast<decltype(g_rccl.GetErrorString)>(sym("ncclGetErrorString"));
    g_rccl_ok = g_rccl_err.empty();
}

const Rccl *rccl(const mcs::rt::Api *A)
{
    std::call_once(g_rccl_once, bind_rccl, A);
    if (!g_rccl_ok) {
        mcs::fail(MCS_E_HIP, "%s", g_rccl_err.c_str());
        return nullptr;
    }
    return &g_rccl;
}

}  // namespace

struct mcs_group {
    nccl_comm comm = nullptr;
    int n_ranks = 0, rank = 0, device = 0;
};

#define RCCL_TRY(expr)                                                                         \
    do {                                                                                       \
        const nccl_result r_ = (expr);                                                         \
        if (r_ != 0)                                                                           \
            return mcs::fail(MCS_E_HIP, "%s failed: %s", #expr, R->GetErrorString(r_));       \
    } while (0)

extern "C" {

const char *mcs_rccl_library(void)
{
    // only a caller with a bound runtime triggers the one-time bind (the search for the librccl
    // beside the HIP runtime needs it; a failed bind is cached for the life of the process)
    const mcs::rt::Api *A = mcs::rt::api();
    if (!A) return "";
    (void)rccl(A);
    return g_rccl_name.c_str();
}

int mcs_group_unique_id(uint8_t *id)
{
    mcs::clear_error();
    if (!id) return mcs::fail(MCS_E_INVALID, "NULL id");
    const mcs::rt::Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    const Rccl *R = rccl(A);
    if (!R) return MCS_E_HIP;
    nccl_id u;
    RCCL_TRY(R->GetUniqueId(&u));
    std::memcpy(id, u.internal, MCS_GROUP_ID_BYTES);
    return MCS_OK;
}

int mcs_group_create(int n_ranks, int rank, const uint8_t *id, int device, mcs_group **out)
{
    mcs::clear_error();
    if (!id || !out) return mcs::fail(MCS_E_INVALID, "NULL id/out");
    *out = nullptr;
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks || device < 0 || device >= mcs::kMaxDevices)
        return mcs::fail(MCS_E_INVALID, "n_ranks=%d rank=%d device=%d", n_ranks, rank, device);
    const mcs::rt::Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    const Rccl *R = rccl(A);
    if (!R) return MCS_E_HIP;
    mcs::DeviceGuard g(A, device);
    if (g.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", device, A->hipGetErrorString(g.err));
    mcs_group *grp = new (std::nothrow) mcs_group();
    if (!grp) return mcs::fail(MCS_E_NOMEM, "group allocation");
    nccl_id u;
    std::memcpy(u.internal, id, MCS_GROUP_ID_BYTES);
    const nccl_result r = R->CommInitRank(&grp->comm, n_ranks, u, rank);
    if (r != 0) {
        delete grp;
        return mcs::fail(MCS_E_HIP, "ncclCommInitRank(%d of %d): %s", rank, n_ranks,
                         R->GetErrorString(r));
    }
    grp->n_ranks = n_ranks;
    grp->rank = rank;
    grp->device = device;
    *out = grp;
    return MCS_OK;
}

int mcs_group_gather(mcs_group *g, const uint8_t *d_mosaics, int64_t bytes, uint8_t *d_recv,
                     int root, void *stream)
{
    mcs::clear_error();
    if (!g || (!d_mosaics && bytes > 0)) return mcs::fail(MCS_E_INVALID, "NULL group/d_mosaics");
    if (root < 0 || root >= g->n_ranks || bytes < 0)
        return mcs::fail(MCS_E_INVALID, "root=%d bytes=%lld", root, (long long)bytes);
    if (g->rank == root && !d_recv && bytes > 0) return mcs::fail(MCS_E_INVALID, "NULL d_recv");
    if (bytes == 0) return MCS_OK;
    const mcs::rt::Api *A = mcs::rt::api();
    if (!A) return MCS_E_HIP;
    const Rccl *R = rccl(A);
    if (!R) return MCS_E_HIP;
    mcs::DeviceGuard dg(A, g->device);
    if (dg.err != hipSuccess)
        return mcs::fail(MCS_E_HIP, "hipSetDevice(%d): %s", g->device,
                         A->hipGetErrorString(dg.err));
    hipStream_t s = (hipStream_t)stream;
    // one grouped call: every peer's batch arrives over its own xGMI link concurrently
    RCCL_TRY(R->GroupStart());
    nccl_result r = 0;
    if (g->rank == root) {
        for (int p = 0; p < g->n_ranks && r == 0; p++)
            if (p != root) r = R->Recv(d_recv + (int64_t)p * bytes, (size_t)bytes, kNcclUint8, p,
                                       g->comm, s);
    } else {
        r = R->Send(d_mosaics, (size_t)bytes, kNcclUint8, root, g->comm, s);
    }
    const nccl_result r2 = R->GroupEnd();
    if (r != 0) return mcs::fail(MCS_E_HIP, "ncclSend/Recv: %s", R->GetErrorString(r));
    if (r2 != 0) return mcs::fail(MCS_E_HIP, "ncclGroupEnd: %s", R->GetErrorString(r2));
    if (g->rank == root && d_recv + (int64_t)root * bytes != d_mosaics)
        HIP_TRY(A->hipMemcpyAsync(d_recv + (int64_t)root * bytes, d_mosaics, (size_t)bytes,
                                  hipMemcpyDeviceToDevice, s));
    return MCS_OK;
}

int mcs_group_destroy(mcs_group *g)
{
    if (!g) return MCS_OK;
    const mcs::rt::Api *A = mcs::rt::api();
    const Rccl *R = A ? rccl(A) : nullptr;
    int rc = MCS_OK;
    if (R && g->comm) {
        const nccl_result r = R->CommDestroy(g->comm);
        if (r != 0) rc = mcs::fail(MCS_E_HIP, "ncclCommDestroy: %s", R->GetErrorString(r));
    }
    delete g;
    return rc;
}

}  // extern "C"
