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

// sizeof of every argument struct, so a binding (ctypes / cffi) can assert its
// mirror against the library it loaded instead of trusting the header copy
extern "C" int64_t cmt_gemm_args_size(void) { return (int64_t)sizeof(cmt_gemm_args); }
extern "C" int64_t cmt_attn_args_size(void) { return (int64_t)sizeof(cmt_attn_args); }
extern "C" int64_t cmt_ln_args_size(void) { return (int64_t)sizeof(cmt_ln_args); }
extern "C" int64_t cmt_chain_args_size(void) { return (int64_t)sizeof(cmt_chain_args); }

extern "C" int64_t cmt_chain_ws_bytes(int rows) {
    if (rows <= 0) return 0;
    return (int64_t)4 * cdiv(rows, 32) * 32 * 256 * (int64_t)sizeof(float);
}
extern "C" int64_t cmt_gemm_ex_args_size(void) { return (int64_t)sizeof(cmt_gemm_ex_args); }
extern "C" int64_t cmt_attn_train_args_size(void) { return (int64_t)sizeof(cmt_attn_train_args); }
extern "C" int64_t cmt_ln_train_args_size(void) { return (int64_t)sizeof(cmt_ln_train_args); }
extern "C" int64_t cmt_bn_args_size(void) { return (int64_t)sizeof(cmt_bn_args); }
extern "C" int64_t cmt_det_loss_args_size(void) { return (int64_t)sizeof(cmt_det_loss_args); }
extern "C" int64_t cmt_match_cost_args_size(void) { return (int64_t)sizeof(cmt_match_cost_args); }
extern "C" int64_t cmt_adamw_args_size(void) { return (int64_t)sizeof(cmt_adamw_args); }
