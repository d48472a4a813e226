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

}  // namespace gm

extern "C" int gm_abi_version(void) { return GM_ABI_VERSION; }
extern "C" const char* gm_last_error(void) { return gm::g_err; }
