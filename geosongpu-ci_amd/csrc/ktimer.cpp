// ktimer.cpp — per-kernel HIP event timing behind GT_LAUNCH (hip_util.hpp).
#include <vector>

#include "hip_util.hpp"

namespace gtfv3 {
namespace {

struct Pending {
  const char* name;
  hipEvent_t b, e;
  double bytes;
};

struct KTimer {
  bool on = false;
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  std::vector<Pending> pending;
  std::map<std::string, KernelStat> stats;

  hipEvent_t take() {
    if (used == pool.size()) {
      hipEvent_t e;
      HIP_CHECK(hipEventCreate(&e));
      pool.push_back(e);
    }
    return pool[used++];
  }
};

KTimer& kt() {
  static KTimer t;
  return t;
}

}  // namespace

bool ktimer_enabled() { return kt().on; }
void ktimer_enable(bool on) { kt().on = on; }

void ktimer_begin(const char* name, hipStream_t s) {
  KTimer& t = kt();
  hipEvent_t b = t.take();
  HIP_CHECK(hipEventRecord(b, s));
  t.pending.push_back({name, b, nullptr, 0.0});
}

void ktimer_end(hipStream_t s) {
  KTimer& t = kt();
  hipEvent_t e = t.take();
  HIP_CHECK(hipEventRecord(e, s));
  t.pending.back().e = e;
}

void ktimer_bytes(double bytes) {
  KTimer& t = kt();
  if (t.on && !t.pending.empty()) t.pending.back().bytes = bytes;
}

void ktimer_flush() {
  KTimer& t = kt();
  for (auto& p : t.pending) {
    if (!p.e) continue;
    HIP_CHECK(hipEventSynchronize(p.e));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, p.b, p.e));
    KernelStat& k = t.stats[p.name];
    k.ms += ms;
    k.launches += 1;
    k.bytes += p.bytes;
  }
  t.pending.clear();
  t.used = 0;
}

void ktimer_reset() {
  ktimer_flush();
  kt().stats.clear();
}

const std::map<std::string, KernelStat>& ktimer_stats() { return kt().stats; }

}  // namespace gtfv3
