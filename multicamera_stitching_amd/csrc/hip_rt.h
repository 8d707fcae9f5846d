// hip_rt.h -- the HIP runtime entry points libmcs uses, bound at run time.
//
// libmcs does not link a HIP runtime.  A process must hold exactly one HIP runtime: PyTorch-ROCm
// ships its own libamdhip64.so, ROCm installs libamdhip64.so.7, and a second runtime in the same
// process fails to initialise.  So libmcs binds to the runtime already loaded in the process
// (torch's, when torch is imported), else to $MCS_HIP_RUNTIME, else to ROCm's.  Streams, events
// and device pointers are then shared with the host framework.  Kernels come from the gfx950
// code object embedded in the library (hipModuleLoadData + hipModuleLaunchKernel).
#pragma once

#include <hip/hip_runtime_api.h>

namespace mcs {
namespace rt {

#define MCS_HIP_API(X)                                                                         \
    X(hipGetDeviceCount, hipError_t, (int *))                                                  \
    X(hipGetDevice, hipError_t, (int *))                                                       \
    X(hipSetDevice, hipError_t, (int))                                                         \
    X(hipGetErrorString, const char *, (hipError_t))                                           \
    X(hipMalloc, hipError_t, (void **, size_t))                                                \
    X(hipFree, hipError_t, (void *))                                                           \
    X(hipHostMalloc, hipError_t, (void **, size_t, unsigned int))                              \
    X(hipHostFree, hipError_t, (void *))                                                       \
    X(hipMemcpyAsync, hipError_t, (void *, const void *, size_t, hipMemcpyKind, hipStream_t)) \
    X(hipMemcpy2DAsync, hipError_t,                                                            \
      (void *, size_t, const void *, size_t, size_t, size_t, hipMemcpyKind, hipStream_t))      \
    X(hipMemsetAsync, hipError_t, (void *, int, size_t, hipStream_t))                         \
    X(hipStreamCreateWithFlags, hipError_t, (hipStream_t *, unsigned int))                    \
    X(hipStreamCreateWithPriority, hipError_t, (hipStream_t *, unsigned int, int))            \
    X(hipDeviceGetStreamPriorityRange, hipError_t, (int *, int *))                             \
    X(hipStreamDestroy, hipError_t, (hipStream_t))                                             \
    X(hipStreamSynchronize, hipError_t, (hipStream_t))                                         \
    X(hipEventCreate, hipError_t, (hipEvent_t *))                                              \
    X(hipEventCreateWithFlags, hipError_t, (hipEvent_t *, unsigned int))                       \
    X(hipStreamWaitEvent, hipError_t, (hipStream_t, hipEvent_t, unsigned int))                 \
    X(hipEventDestroy, hipError_t, (hipEvent_t))                                               \
    X(hipEventRecord, hipError_t, (hipEvent_t, hipStream_t))                                   \
    X(hipEventSynchronize, hipError_t, (hipEvent_t))                                           \
    X(hipEventElapsedTime, hipError_t, (float *, hipEvent_t, hipEvent_t))                      \
    X(hipModuleLoadData, hipError_t, (hipModule_t *, const void *))                            \
    X(hipModuleUnload, hipError_t, (hipModule_t))                                              \
    X(hipStreamBeginCapture, hipError_t, (hipStream_t, hipStreamCaptureMode))                  \
    X(hipStreamEndCapture, hipError_t, (hipStream_t, hipGraph_t *))                            \
    X(hipGraphInstantiate, hipError_t, (hipGraphExec_t *, hipGraph_t, hipGraphNode_t *, char *, \
                                        size_t))                                               \
    X(hipGraphLaunch, hipError_t, (hipGraphExec_t, hipStream_t))                               \
    X(hipGraphExecDestroy, hipError_t, (hipGraphExec_t))                                       \
    X(hipGraphDestroy, hipError_t, (hipGraph_t))                                               \
    X(hipModuleGetFunction, hipError_t, (hipFunction_t *, hipModule_t, const char *))         \
    X(hipModuleLaunchKernel, hipError_t,                                                       \
      (hipFunction_t, unsigned int, unsigned int, unsigned int, unsigned int, unsigned int,   \
       unsigned int, unsigned int, hipStream_t, void **, void **))

struct Api {
#define MCS_DECL_FN(name, ret, args) ret(*name) args;
    MCS_HIP_API(MCS_DECL_FN)
#undef MCS_DECL_FN
};

// Binds on first call (thread-safe).  nullptr on failure, with mcs_last_error() set.
const Api *api();
// Path (or soname) of the bound runtime, "" before binding.
const char *runtime_name();

}  // namespace rt
}  // namespace mcs
