// pmc_calib.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths the dycore kernels use (MI355X_MICROARCH.md, HBM section: only 16-B-per-lane
// streaming reads are calibrated there, at 1/2).  Each kernel streams a known number of
// bytes through 1 GiB buffers (4x the 256 MiB Infinity Cache, so nothing is re-served
// on-die), one launch per kernel; the counter value per launch divided by the known byte
// count is the correction factor tools/pmc_summary.py applies.
//
//   hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/bin/pmc_calib
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d D -o run -- tools/bin/pmc_calib
//
// Kernels (bytes per launch printed by the program, "name bytes_read bytes_written"):
//   rd4 / rd8 / rd16   global loads of 4, 8 (dwordx2, the fp64 stencils) and 16 B per lane
//   brd8               raw buffer loads of 8 B per lane (tp_march / a2b_march / riem)
//   cp8                8-B load + 8-B store per lane (the plane stencils' read-modify-write)
//   wr8 / bwr8         global / buffer stores of 8 B per lane
//   pl8                a plane stencil's pattern: rows of pitch 192 doubles, 181 read per row
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                           \
    }                                                                         \
  } while (0)

template <typename T>
__global__ void rd_k(const T* __restrict__ a, long n, double* __restrict__ sink) {
  double acc = 0.0;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < n; t += (long)gridDim.x * blockDim.x) {
    const T v = a[t];
    const double* pv = reinterpret_cast<const double*>(&v);
    for (unsigned q = 0; q < (sizeof(T) + 7) / 8; ++q) acc += sizeof(T) >= 8 ? pv[q] : (double)*(const float*)&v;
  }
  if (acc == 1.2345e300) sink[0] = acc;  // never true for the zero-filled input; keeps the loads
}

__global__ void brd8_k(const double* __restrict__ a, long n, double* __restrict__ sink) {
  // one descriptor per 2^28-byte window (32-bit offsets), as the stencils form per plane
  double acc = 0.0;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < n; t += (long)gridDim.x * blockDim.x) {
    const long win = t >> 25;  // 2^25 doubles = 256 MiB
    auto r = __builtin_amdgcn_make_buffer_rsrc((void*)(a + (win << 25)), 0, 1u << 28, 0x00020000);
    acc += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)((t & ((1 << 25) - 1)) * 8), 0, 0));
  }
  if (acc == 1.2345e300) sink[0] = acc;
}

__global__ void cp8_k(const double* __restrict__ a, double* __restrict__ b, long n) {
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < n; t += (long)gridDim.x * blockDim.x) b[t] = a[t] + 1.0;
}

__global__ void wr8_k(double* __restrict__ b, long n) {
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < n; t += (long)gridDim.x * blockDim.x) b[t] = (double)t;
}

typedef unsigned int U2 __attribute__((ext_vector_type(2)));
__global__ void bwr8_k(double* __restrict__ b, long n) {
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < n; t += (long)gridDim.x * blockDim.x) {
    const long win = t >> 25;
    auto r = __builtin_amdgcn_make_buffer_rsrc((void*)(b + (win << 25)), 0, 1u << 28, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(U2, (double)t), r, (uint32_t)((t & ((1 << 25) - 1)) * 8), 0, 0);
  }
}

// plane pattern: nrow rows of pitch 192 doubles, 181 of them read (the C180 cell rows)
__global__ void pl8_k(const double* __restrict__ a, long nrow, double* __restrict__ sink) {
  double acc = 0.0;
  const long n = nrow * 181;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < n; t += (long)gridDim.x * blockDim.x) {
    const long row = t / 181, col = t - row * 181;
    acc += a[row * 192 + col];
  }
  if (acc == 1.2345e300) sink[0] = acc;
}

int main() {
  const long bytes = 1L << 30;
  const long n8 = bytes / 8;
  double *a, *b, *sink;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  CK(hipDeviceSynchronize());
  const dim3 grid(256 * 32), blk(256);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, double rb, double wbytes, auto launch) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("%s %.0f %.0f %.3f ms %.2f TB/s\n", name, rb, wbytes, ms, (rb + wbytes) / (ms * 1e-3) / 1e12);
  };
  run("rd4", bytes, 0, [&] { rd_k<float><<<grid, blk>>>((const float*)a, bytes / 4, sink); });
  run("rd8", bytes, 0, [&] { rd_k<double><<<grid, blk>>>(a, n8, sink); });
  run("rd16", bytes, 0, [&] { rd_k<double2><<<grid, blk>>>((const double2*)a, bytes / 16, sink); });
  run("brd8", bytes, 0, [&] { brd8_k<<<grid, blk>>>(a, n8, sink); });
  run("cp8", bytes, bytes, [&] { cp8_k<<<grid, blk>>>(a, b, n8); });
  run("wr8", 0, bytes, [&] { wr8_k<<<grid, blk>>>(b, n8); });
  run("bwr8", 0, bytes, [&] { bwr8_k<<<grid, blk>>>(b, n8); });
  const long nrow = n8 / 192;
  run("pl8", (double)nrow * 181 * 8, 0, [&] { pl8_k<<<grid, blk>>>(a, nrow, sink); });
  CK(hipDeviceSynchronize());
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(sink));
  return 0;
}
