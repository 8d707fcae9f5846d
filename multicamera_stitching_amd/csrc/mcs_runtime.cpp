// mcs_runtime.cpp -- loading of the embedded gfx950 code objects (one per device source; the
// build embeds them with .incbin, see build.py) and kernel lookup, per device.
#include <mutex>

#include "mcs_common.h"

extern "C" const unsigned char mcs_hsaco_stitch_start[];
extern "C" const unsigned char mcs_hsaco_features_start[];
extern "C" const unsigned char mcs_hsaco_sweep_start[];

namespace mcs {

namespace {
hipModule_t g_mod[kMaxDevices][kNumModules];
std::mutex g_mod_mu;

const unsigned char *blob(Module m)
{
    return m == kModStitch ? mcs_hsaco_stitch_start
                           : (m == kModSweep ? mcs_hsaco_sweep_start : mcs_hsaco_features_start);
}
}  // namespace

int module_function(const rt::Api *A, int device, Module m, const char *name, hipFunction_t *out)
{
    if (device < 0 || device >= kMaxDevices) return fail(MCS_E_INVALID, "device %d", device);
    hipModule_t mod;
    {
        std::lock_guard<std::mutex> lk(g_mod_mu);
        if (!g_mod[device][m]) HIP_TRY(A->hipModuleLoadData(&g_mod[device][m], blob(m)));
        mod = g_mod[device][m];
    }
    HIP_TRY(A->hipModuleGetFunction(out, mod, name));
    return MCS_OK;
}

}  // namespace mcs
