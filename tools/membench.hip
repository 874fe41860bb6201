// membench.hip — HBM write/copy ceilings on this box for the emission's shape (3 u32 columns of n
// rows written, one read stream): what k_emit_lists can reach at most. Not part of the product.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/_membench tools/membench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__global__ void k_write3(uint32_t *a, uint32_t *b, uint32_t *c, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    a[i] = (uint32_t)i;
    b[i] = (uint32_t)i ^ 7u;
    c[i] = (uint32_t)i + 3u;
  }
}
__global__ void k_write3x4(uint4 *a, uint4 *b, uint4 *c, uint64_t n4) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t x = (uint32_t)i;
    a[i] = make_uint4(x, x + 1, x + 2, x + 3);
    b[i] = make_uint4(x ^ 1, x, x, x);
    c[i] = make_uint4(x + 5, x, x, x);
  }
}
// the emission's shape: one read stream (a small, L2-resident table) + 3 write streams
__global__ void k_read1_write3(const uint32_t *src, uint64_t mask, uint32_t *a, uint32_t *b, uint32_t *c, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = src[i & mask];
    a[i] = v;
    b[i] = (uint32_t)(i >> 8);
    c[i] = (uint32_t)(i >> 10);
  }
}
// blocked: each block writes a contiguous window of W rows per iteration (the emission's order)
template <int IPT>
__global__ __launch_bounds__(256) void k_win_write3(uint32_t *a, uint32_t *b, uint32_t *c, uint64_t n) {
  constexpr uint64_t W = 256 * IPT;
  for (uint64_t w = blockIdx.x; w * W < n; w += gridDim.x) {
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const uint64_t p = w * W + k * 256 + threadIdx.x;
      if (p < n) {
        a[p] = (uint32_t)p;
        b[p] = (uint32_t)w;
        c[p] = (uint32_t)k;
      }
    }
  }
}

int main(int argc, char **argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1027370460ull;
  uint32_t *a, *b, *c, *s;
  CK(hipMalloc((void **)&a, n * 4));
  CK(hipMalloc((void **)&b, n * 4));
  CK(hipMalloc((void **)&c, n * 4));
  CK(hipMalloc((void **)&s, (1u << 22) * 4));
  CK(hipMemset(s, 1, (1u << 22) * 4));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char *name, double bytes, auto launch) {
    for (int i = 0; i < 2; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int reps = 5;
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    std::printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  const double wb = 12.0 * n;
  for (int bpc : {4, 8, 16, 32}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "write3 dword grid=%dx%d", cus, bpc);
    run(nm, wb, [&] { hipLaunchKernelGGL(k_write3, dim3(cus * bpc), dim3(256), 0, 0, a, b, c, n); });
  }
  run("write3 dword grid=n/256", wb, [&] { hipLaunchKernelGGL(k_write3, dim3((n + 255) / 256), dim3(256), 0, 0, a, b, c, n); });
  run("write3 dwordx4 grid=cus*16", wb, [&] {
    hipLaunchKernelGGL(k_write3x4, dim3(cus * 16), dim3(256), 0, 0, (uint4 *)a, (uint4 *)b, (uint4 *)c, n / 4);
  });
  run("read1(L2)+write3 grid=cus*16", 16.0 * n, [&] {
    hipLaunchKernelGGL(k_read1_write3, dim3(cus * 16), dim3(256), 0, 0, s, (uint64_t)(1u << 22) - 1, a, b, c, n);
  });
  run("win_write3 ipt4 grid=cus*7", wb, [&] { hipLaunchKernelGGL(k_win_write3<4>, dim3(cus * 7), dim3(256), 0, 0, a, b, c, n); });
  run("win_write3 ipt16 grid=cus*8", wb, [&] { hipLaunchKernelGGL(k_win_write3<16>, dim3(cus * 8), dim3(256), 0, 0, a, b, c, n); });
  run("memset 12n", wb, [&] {
    CK(hipMemsetAsync(a, 0, n * 4));
    CK(hipMemsetAsync(b, 0, n * 4));
    CK(hipMemsetAsync(c, 0, n * 4));
  });
  return 0;
}
