// ktimer.cpp — per-kernel HIP event timing behind GT_LAUNCH (hip_util.hpp).
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
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
  std::string only;       // timed kernel (empty: all)
  bool last_timed = false;  // the launch just issued was bracketed
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
void ktimer_filter(const char* name) { kt().only = name ? name : ""; }
// the filter names a kernel family: "tp_march" matches "(tp_march<6, true, false>)"
bool ktimer_wants(const char* name) {
  KTimer& t = kt();
  if (t.only.empty()) {
    t.last_timed = true;
    return true;
  }
  const char* n = name[0] == '(' ? name + 1 : name;
  const size_t L = t.only.size();
  t.last_timed = std::strncmp(n, t.only.c_str(), L) == 0 && (n[L] == '\0' || n[L] == '<' || n[L] == ')');
  return t.last_timed;
}

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
  if (t.on && t.last_timed && !t.pending.empty()) t.pending.back().bytes = bytes;
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

bool debug_sync_launch() {
  static const bool on = [] {
    const char* e = std::getenv("GTFV3_SYNC_LAUNCH");
    return e && e[0] == '1';
  }();
  return on;
}

namespace {
struct Canary {
  std::string what;
  const void* d;
  std::vector<unsigned char> h;
};
std::mutex g_canary_m;
std::vector<Canary> g_canaries;
}  // namespace

void debug_canary(const char* what, const void* d, const void* h, size_t bytes) {
  if (!debug_sync_launch() || !d || !bytes) return;
  std::lock_guard<std::mutex> lk(g_canary_m);
  const unsigned char* hb = static_cast<const unsigned char*>(h);
  g_canaries.push_back({what, d, std::vector<unsigned char>(hb, hb + bytes)});
}

void debug_canary_drop(const void* d) {
  std::lock_guard<std::mutex> lk(g_canary_m);
  for (size_t i = 0; i < g_canaries.size();)
    if (g_canaries[i].d == d) g_canaries.erase(g_canaries.begin() + i);
    else ++i;
}

void debug_sync_check(const char* kern, hipStream_t st) {
  const hipError_t e = hipStreamSynchronize(st);
  if (e != hipSuccess) throw std::runtime_error(std::string("kernel ") + kern + ": " + hipGetErrorString(e));
  // every registered read-only table / guard zone must still hold its bytes
  std::lock_guard<std::mutex> lk(g_canary_m);
  std::vector<unsigned char> tmp;
  for (const Canary& c : g_canaries) {
    tmp.resize(c.h.size());
    HIP_CHECK(hipMemcpy(tmp.data(), c.d, tmp.size(), hipMemcpyDeviceToHost));
    if (std::memcmp(tmp.data(), c.h.data(), tmp.size()) != 0) {
      size_t i = 0;
      while (tmp[i] == c.h[i]) ++i;
      throw std::runtime_error(std::string("after kernel ") + kern + ": canary '" + c.what + "' overwritten at byte " +
                               std::to_string(i) + " of " + std::to_string(tmp.size()));
    }
  }
}

}  // namespace gtfv3
