// C-ABI plumbing: version, thread-local error reporting, launch checks.
#include "cmt_common.h"

static thread_local std::string g_last_error;

void cmt_set_error(const std::string& msg) { g_last_error = msg; }

int cmt_fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int cmt_check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_last_error = std::string(what) + ": " + hipGetErrorString(e);
        return (int)e;
    }
    return 0;
}

extern "C" int cmt_abi_version(void) { return CMT_ABI_VERSION; }

extern "C" const char* cmt_last_error(void) { return g_last_error.c_str(); }
