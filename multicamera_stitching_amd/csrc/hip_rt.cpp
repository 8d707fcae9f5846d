// hip_rt.cpp -- run-time binding of the HIP runtime (see hip_rt.h for why).
#include "hip_rt.h"

#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "mcs_common.h"

namespace mcs {
namespace rt {

static Api g_api;
static bool g_ok = false;
static std::once_flag g_once;
static std::string g_name;
static std::string g_err;

static void *open_runtime()
{
    // 1. a runtime already in the process (torch's soname first, then ROCm's)
    const char *loaded[] = {"libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"};
    for (const char *n : loaded) {
        if (void *h = dlopen(n, RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL)) {
            g_name = n;
            return h;
        }
    }
    // 2. explicit choice
    if (const char *p = getenv("MCS_HIP_RUNTIME")) {
        if (void *h = dlopen(p, RTLD_NOW | RTLD_GLOBAL)) {
            g_name = p;
            return h;
        }
        g_err = std::string("dlopen($MCS_HIP_RUNTIME=") + p + "): " + dlerror();
        return nullptr;
    }
    // 3. ROCm's runtime
    const char *paths[] = {"libamdhip64.so.7", "/opt/rocm/lib/libamdhip64.so.7",
                           "/opt/rocm/lib/libamdhip64.so"};
    for (const char *n : paths) {
        if (void *h = dlopen(n, RTLD_NOW | RTLD_GLOBAL)) {
            g_name = n;
            return h;
        }
    }
    g_err = std::string("no HIP runtime found (libamdhip64): ") + dlerror();
    return nullptr;
}

static void bind()
{
    void *h = open_runtime();
    if (!h) return;
#define MCS_BIND_FN(name, ret, args)                                                           \
    g_api.name = reinterpret_cast<ret(*) args>(dlsym(h, #name));                               \
    if (!g_api.name) {                                                                         \
        g_err = std::string("HIP runtime ") + g_name + " lacks " #name;                       \
        return;                                                                                \
    }
    MCS_HIP_API(MCS_BIND_FN)
#undef MCS_BIND_FN
    g_ok = true;
}

const Api *api()
{
    std::call_once(g_once, bind);
    if (!g_ok) {
        fail(MCS_E_HIP, "%s", g_err.c_str());
        return nullptr;
    }
    return &g_api;
}

const char *runtime_name() { return g_name.c_str(); }

}  // namespace rt
}  // namespace mcs
