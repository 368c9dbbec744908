// hip_util.hpp — error handling and small device helpers.
#pragma once
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "gtfv3.hpp"

#define HIP_CHECK(x)                                                                  \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess)                                                             \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) +   \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__));   \
  } while (0)

#define HIP_LAUNCH_CHECK() HIP_CHECK(hipGetLastError())

namespace gtfv3 {

// plane offset of local (i,j); i,j may be negative down to -NG
__host__ __device__ inline long pidx(const Dims& d, int i, int j) {
  return (long)(j + NG) * d.pitch + (i + NG);
}

inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

}  // namespace gtfv3
