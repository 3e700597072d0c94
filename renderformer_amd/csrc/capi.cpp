// Error plumbing shared by every entry point of librfhip (thread-local last error).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/rf.h"

namespace rf {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return RF_ERR_LAUNCH;
    }
    return RF_OK;
}
}  // namespace rf

extern "C" const char* rf_last_error(void) { return rf::g_err; }
extern "C" int rf_abi_version(void) { return RF_ABI_VERSION; }
