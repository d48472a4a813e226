// ABI housekeeping: version and thread-local error text.
#include <cstdlib>
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

static Residency g_res = {2, 1, 0};  // two trunk streams, one process, nothing reserved

const Residency& residency() { return g_res; }

int usable_cus(int cus) {
    const int u = cus - g_res.reserved_cus;
    return u > cus / 4 ? u : cus / 4;
}

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

extern "C" int gm_set_residency(int streams, int sharers, int reserved_cus) {
    GM_REQUIRE(streams >= 1 && streams <= 64, "gm_set_residency: streams must be in [1, 64] (got %d)", streams);
    GM_REQUIRE(sharers >= 1 && sharers <= 64, "gm_set_residency: sharers must be in [1, 64] (got %d)", sharers);
    GM_REQUIRE(reserved_cus >= 0 && reserved_cus <= 4096, "gm_set_residency: reserved_cus out of range (%d)",
               reserved_cus);
    gm::g_res = gm::Residency{streams, sharers, reserved_cus};
    return GM_OK;
}

extern "C" int gm_get_residency(int* streams, int* sharers, int* reserved_cus) {
    GM_REQUIRE(streams && sharers && reserved_cus, "gm_get_residency: null output");
    *streams = gm::g_res.streams;
    *sharers = gm::g_res.sharers;
    *reserved_cus = gm::g_res.reserved_cus;
    return GM_OK;
}
