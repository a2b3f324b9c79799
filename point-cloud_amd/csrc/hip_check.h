#pragma once
#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>

namespace pcc {
struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
}  // namespace pcc

#define HIP_CHECK(expr)                                                                                   \
    do {                                                                                                  \
        hipError_t e_ = (expr);                                                                           \
        if (e_ != hipSuccess)                                                                             \
            throw ::pcc::HipError(std::string(#expr) + " failed: " + hipGetErrorString(e_) + " at " +    \
                                  __FILE__ + ":" + std::to_string(__LINE__));                             \
    } while (0)
