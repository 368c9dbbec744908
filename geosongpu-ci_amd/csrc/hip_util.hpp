// hip_util.hpp — error handling and small device helpers.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
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

// Optional per-kernel timing: when enabled, every GT_LAUNCH brackets its kernel
// with a pair of HIP events on the launch stream; ktimer_flush() (after a stream
// sync) folds them into per-kernel totals.  Off by default: zero cost then.
struct KernelStat {
  double ms = 0.0;
  long launches = 0;
  double bytes = 0.0;  // algorithmic HBM bytes of the timed launches (0: no formula)
};
bool ktimer_enabled();
void ktimer_enable(bool on);
void ktimer_begin(const char* name, hipStream_t s);
void ktimer_end(hipStream_t s);
// algorithmic bytes of the launch just issued (DESIGN.md §4 formulas); no-op when off
void ktimer_bytes(double bytes);
void ktimer_flush();
void ktimer_reset();
const std::map<std::string, KernelStat>& ktimer_stats();

struct KScope {
  bool on;
  hipStream_t s;
  KScope(const char* n, hipStream_t st) : on(ktimer_enabled()), s(st) {
    if (on) ktimer_begin(n, s);
  }
  ~KScope() {
    if (on) ktimer_end(s);
  }
};

#define GT_LAUNCH(kern, grid, block, shm, st, ...)        \
  do {                                                    \
    ::gtfv3::KScope kscope_(#kern, st);                   \
    hipLaunchKernelGGL(kern, grid, block, shm, st, __VA_ARGS__); \
  } while (0)

}  // namespace gtfv3
