// ABI housekeeping: version and thread-local error text.
#include <cstring>

#include "gm_common.h"

namespace gm {

static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return (int)e;
    }
    return GM_OK;
}

static unsigned g_spin_limit = 0;  // 0: default

unsigned spin_limit() { return g_spin_limit ? g_spin_limit : (1u << 24); }

}  // namespace gm

extern "C" int gm_abi_version(void) { return GM_ABI_VERSION; }

extern "C" int gm_device_faults(unsigned* out, int clear) {
    GM_REQUIRE(out, "gm_device_faults: null out");
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        gm::set_error("gm_device_faults: %s", hipGetErrorString(e));
        return (int)e;
    }
    *out = gm::bn_faults_read(clear != 0) | gm::conv_faults_read(clear != 0);
    return GM_OK;
}

extern "C" int gm_set_spin_limit(unsigned polls) {
    gm::g_spin_limit = polls;
    return GM_OK;
}
extern "C" const char* gm_last_error(void) { return gm::g_err; }
