// The C ABI's context object and the error helpers shared by the host-side translation units
// (cmpc_api.hip, rounds_api.hip).  Not part of the public header: cmpc.h keeps cmpc_ctx opaque.
#pragma once
#include <string>

#include <rccl/rccl.h>

#include "internal.h"

struct cmpc_ctx {
    int device = 0;
    hipStream_t stream = nullptr;  // private stream for the host-pointer entry points
    char* ws = nullptr;            // device arena
    size_t ws_bytes = 0;
    ncclComm_t comm = nullptr;     // RCCL communicator of cmpc_comm_init (multi-GPU exchange)
    int nranks = 1, rank = 0;      // of that communicator
    std::string err;
};

inline int fail(cmpc_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

inline int hip_fail(cmpc_ctx* c, hipError_t e, const char* where) {
    return fail(c, CMPC_ERR_DEVICE, std::string(where) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr)                                              \
    do {                                                           \
        hipError_t e_ = (expr);                                    \
        if (e_ != hipSuccess) return hip_fail(ctx, e_, #expr);     \
    } while (0)
