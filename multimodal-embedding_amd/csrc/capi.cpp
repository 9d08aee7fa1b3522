// Error plumbing of the libmme C ABI (include/mme.h).
//
// The reference reports failures as Python exceptions caught per model
// (main.py:822-824, 839-842); the ABI returns an int status and keeps the
// message in a thread-local buffer that the Python shim turns into RuntimeError.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/mme.h"

static thread_local char g_err[512] = "";

int mme_set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int mme_check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return mme_set_error(MME_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    return MME_OK;
}

extern "C" const char* mme_last_error(void) { return g_err; }
extern "C" int mme_abi_version(void) { return MME_ABI_VERSION; }
extern "C" int mme_build_flags(void) {
#ifdef MME_DEV
    return MME_BUILD_DEV;
#else
    return 0;
#endif
}
