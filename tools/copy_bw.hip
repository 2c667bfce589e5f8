// copy_bw.hip -- HBM ceiling probe for this box: float4 stream copy (R+W),
// read-only and write-only, a few unroll / grid shapes.  Establishes the
// practical read+write roofline the one-hot gather (a copy with a random
// source) is compared against in DESIGN.md.  Not part of the product.
//   hipcc -O3 --offload-arch=gfx950 tools/copy_bw.hip -o tools/copy_bw
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * 256 * U;
  for (; i < n; i += stride) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t k = i + (size_t)u * 256;
      if (k < n) v[u] = a[k];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t k = i + (size_t)u * 256;
      if (k < n) {
        if (NT) __builtin_nontemporal_store(v[u].x, &b[k].x), __builtin_nontemporal_store(v[u].y, &b[k].y),
                __builtin_nontemporal_store(v[u].z, &b[k].z), __builtin_nontemporal_store(v[u].w, &b[k].w);
        else b[k] = v[u];
      }
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void read_k(const float4* __restrict__ a, float* out, size_t n) {
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * 256 * U;
  float s = 0.f;
  for (; i < n; i += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t k = i + (size_t)u * 256;
      if (k < n) { float4 v = a[k]; s += v.x + v.y + v.z + v.w; }
    }
  }
  if (s == 12345.f) out[0] = s;
}

__global__ __launch_bounds__(256) void write_k(float4* __restrict__ b, size_t n) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * 256;
  for (; i < n; i += stride) b[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

template <class F>
static float timeit(F f, int iters) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < iters; ++i) f();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / iters;
}

int main() {
  const size_t bytes = (size_t)1 << 31;  // 2 GiB per buffer (far beyond the 256 MiB MALL)
  const size_t n = bytes / 16;
  float4 *a, *b;
  float* o;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&o, 64));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int iters = 10;
  for (int wpc : {4, 8, 16, 32}) {
    const int grid = cus * wpc;
    float ms;
    ms = timeit([&] { hipLaunchKernelGGL((copy_k<1, false>), dim3(grid), dim3(256), 0, 0, a, b, n); }, iters);
    printf("{\"kernel\":\"copy U1\",\"blocks_per_cu\":%d,\"us\":%.1f,\"GBps\":%.1f}\n", wpc, ms * 1e3, 2.0 * bytes / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL((copy_k<4, false>), dim3(grid), dim3(256), 0, 0, a, b, n); }, iters);
    printf("{\"kernel\":\"copy U4\",\"blocks_per_cu\":%d,\"us\":%.1f,\"GBps\":%.1f}\n", wpc, ms * 1e3, 2.0 * bytes / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL((copy_k<4, true>), dim3(grid), dim3(256), 0, 0, a, b, n); }, iters);
    printf("{\"kernel\":\"copy U4 nt-store\",\"blocks_per_cu\":%d,\"us\":%.1f,\"GBps\":%.1f}\n", wpc, ms * 1e3, 2.0 * bytes / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL((read_k<4>), dim3(grid), dim3(256), 0, 0, a, o, n); }, iters);
    printf("{\"kernel\":\"read U4\",\"blocks_per_cu\":%d,\"us\":%.1f,\"GBps\":%.1f}\n", wpc, ms * 1e3, 1.0 * bytes / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL(write_k, dim3(grid), dim3(256), 0, 0, b, n); }, iters);
    printf("{\"kernel\":\"write\",\"blocks_per_cu\":%d,\"us\":%.1f,\"GBps\":%.1f}\n", wpc, ms * 1e3, 1.0 * bytes / ms / 1e6);
  }
  // one-shot (non-persistent) copy: one float4 per thread
  {
    const int grid = (int)(n / 256);
    float ms = timeit([&] { hipLaunchKernelGGL((copy_k<1, false>), dim3(grid), dim3(256), 0, 0, a, b, n); }, iters);
    printf("{\"kernel\":\"copy one-shot\",\"us\":%.1f,\"GBps\":%.1f}\n", ms * 1e3, 2.0 * bytes / ms / 1e6);
  }
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(o));
  return 0;
}
