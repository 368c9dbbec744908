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
#ifdef GTFV3_BOUNDS
// debugging build (make BOUNDS=1): report and clamp plane indices outside the padded plane
__host__ __device__ inline long pidx(const Dims& d, int i, int j) {
  if (i < -NG || i > d.pitch - NG - 1 || j < -NG || j > d.nj - NG - 1) {
#ifdef __HIP_DEVICE_COMPILE__
    printf("GTFV3_BOUNDS pidx(%d, %d) outside plane pitch %d nj %d (block %d %d %d thread %d %d)\n", i, j, d.pitch,
           d.nj, blockIdx.x, blockIdx.y, blockIdx.z, threadIdx.x, threadIdx.y);
#endif
    i = i < -NG ? -NG : (i > d.pitch - NG - 1 ? d.pitch - NG - 1 : i);
    j = j < -NG ? -NG : (j > d.nj - NG - 1 ? d.nj - NG - 1 : j);
  }
  return (long)(j + NG) * d.pitch + (i + NG);
}
#else
__host__ __device__ inline long pidx(const Dims& d, int i, int j) {
  return (long)(j + NG) * d.pitch + (i + NG);
}
#endif

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
// Restrict timing to one kernel family: `name` is the kernel's name without template
// arguments (e.g. "tp_march" times every tp_march<...> instantiation); empty or null:
// every kernel.  Untimed launches cost nothing.
void ktimer_filter(const char* name);
bool ktimer_wants(const char* name);
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
  KScope(const char* n, hipStream_t st) : on(ktimer_enabled() && ktimer_wants(n)), s(st) {
    if (on) ktimer_begin(n, s);
  }
  ~KScope() {
    if (on) ktimer_end(s);
  }
};

// GTFV3_SYNC_LAUNCH=1 (debugging): synchronise after every launch and name the kernel
// in the error, so an asynchronous fault is attributed to the launch that caused it.
bool debug_sync_launch();
void debug_sync_check(const char* kern, hipStream_t st);
// Debug mode only: register device bytes that must not change (checked after every launch).
void debug_canary(const char* what, const void* d, const void* h, size_t bytes);
void debug_canary_drop(const void* d);

// GT_LAUNCH_N: the same with an explicit (string literal) timer name, for launch sites
// whose template arguments are not spelled out at the call
#define GT_LAUNCH_N(name, kern, grid, block, shm, st, ...)                 \
  do {                                                                   \
    {                                                                    \
      ::gtfv3::KScope kscope_(name, st);                                 \
      hipLaunchKernelGGL(kern, grid, block, shm, st, __VA_ARGS__);       \
    }                                                                    \
    if (::gtfv3::debug_sync_launch()) ::gtfv3::debug_sync_check(name, st); \
  } while (0)

#define GT_LAUNCH(kern, grid, block, shm, st, ...)                       \
  do {                                                                   \
    {                                                                    \
      ::gtfv3::KScope kscope_(#kern, st);                                \
      hipLaunchKernelGGL(kern, grid, block, shm, st, __VA_ARGS__);       \
    }                                                                    \
    if (::gtfv3::debug_sync_launch()) ::gtfv3::debug_sync_check(#kern, st); \
  } while (0)

}  // namespace gtfv3
