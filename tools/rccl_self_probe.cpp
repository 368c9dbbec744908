// rccl_self_probe.cpp — does RCCL run a size-1 communicator with point-to-point messages to
// itself and an allreduce on one GPU?  (the NcclTransport path of
// comm.cpp has never executed; this pool gives one GPU per box.)  Prints one JSON line.
//   build: hipcc -O2 --offload-arch=gfx950 tools/rccl_self_probe.cpp -lrccl -o tools/bin/rccl_self_probe
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    auto _r = (x);                                                              \
    if (_r != 0) {                                                              \
      std::printf("{\"ok\": false, \"call\": \"%s\", \"code\": %d}\n", #x, (int)_r); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main() {
  CK(hipSetDevice(0));
  ncclUniqueId id;
  CK(ncclGetUniqueId(&id));
  ncclComm_t comm;
  CK(ncclCommInitRank(&comm, 1, id, 0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const size_t n = 1 << 20;
  double *a, *b, *c;
  CK(hipMalloc(&a, n * sizeof(double)));
  CK(hipMalloc(&b, n * sizeof(double)));
  CK(hipMalloc(&c, 8 * sizeof(double)));
  std::vector<double> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = 0.5 * (double)i - 3.0;
  CK(hipMemcpy(a, h.data(), n * sizeof(double), hipMemcpyHostToDevice));
  CK(hipMemset(b, 0, n * sizeof(double)));
  // two messages to self in one group, as the halo exchange posts them (several per peer)
  CK(ncclGroupStart());
  CK(ncclSend(a, n / 2, ncclDouble, 0, comm, st));
  CK(ncclRecv(b, n / 2, ncclDouble, 0, comm, st));
  CK(ncclSend(a + n / 2, n / 2, ncclDouble, 0, comm, st));
  CK(ncclRecv(b + n / 2, n / 2, ncclDouble, 0, comm, st));
  CK(ncclGroupEnd());
  std::vector<double> hc(8, 0.0);
  for (int i = 0; i < 8; ++i) hc[i] = i * 1.5;
  CK(hipMemcpyAsync(c, hc.data(), 8 * sizeof(double), hipMemcpyHostToDevice, st));
  CK(ncclAllReduce(c, c, 8, ncclDouble, ncclMax, comm, st));
  CK(hipStreamSynchronize(st));
  std::vector<double> hb(n), hr(8);
  CK(hipMemcpy(hb.data(), b, n * sizeof(double), hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), c, 8 * sizeof(double), hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < n; ++i) bad += hb[i] != h[i];
  for (int i = 0; i < 8; ++i) bad += hr[i] != hc[i];
  // time a group of 18 self messages of 64 KB (a halo exchange's size class at C180)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  for (int it = 0; it < 20; ++it) {
    CK(ncclGroupStart());
    for (int m = 0; m < 18; ++m) {
      CK(ncclSend(a + m * 8192, 8192, ncclDouble, 0, comm, st));
      CK(ncclRecv(b + m * 8192, 8192, ncclDouble, 0, comm, st));
    }
    CK(ncclGroupEnd());
  }
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  int ver = 0;
  ncclGetVersion(&ver);
  std::printf("{\"ok\": %s, \"mismatches\": %zu, \"rccl_version\": %d, \"group18x64KB_us\": %.1f}\n",
              bad ? "false" : "true", bad, ver, 1000.0 * ms / 20);
  CK(ncclCommDestroy(comm));
  return bad ? 1 : 0;
}
