// common.hpp -- error plumbing shared by the C-ABI entry points.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>

#include "../../include/ldpc_amd.h"

namespace ldpc {

void set_error(const std::string &msg);

inline int fail(int code, const std::string &msg) {
    set_error(msg);
    return code;
}

}  // namespace ldpc

#define LDPC_HIP(call)                                                                        \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return ::ldpc::fail(LDPC_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define LDPC_CHECK_LAUNCH(what)                                                                  \
    do {                                                                                         \
        hipError_t e_ = hipGetLastError();                                                       \
        if (e_ != hipSuccess)                                                                    \
            return ::ldpc::fail(LDPC_EHIP, std::string(what) + " launch: " + hipGetErrorString(e_)); \
    } while (0)
