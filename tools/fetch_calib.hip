// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE on gfx950 for the access
// widths the EV lookup issues (MI355X_MICROARCH.md: FETCH_SIZE is exact / 2
// only for wide coalesced streams; "other access widths are uncalibrated").
// One launch per kernel, each over a KNOWN number of accesses:
//   stream      1 GiB read in order with 16 B per lane (the known-x2 case)
//   rand<W>     NACC accesses of W bytes at uniformly random W-aligned
//               offsets of an 8 GiB table (far past the 256 MiB Infinity
//               Cache): W = 8 (one lane, like a key), 16 (one lane: the hash
//               slot probe), 64 / 128 / 512 (W/16 lanes, dwordx4 each: rows)
//   keys_tb     the lookup's key read in output-slot order from a [T, B]
//               id matrix (T = 26, B = 65536): slot s = b*T + t reads
//               keys[t*B + b], 8 B per slot
//   keys_bt     the same slots from a [B, T] matrix: keys[b*T + t]
// Compare FETCH_SIZE (KB) per dispatch against NACC * W (the requested bytes)
// and against the line counts.  Not part of the product.
//   hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__);               \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void stream_k(const float4* __restrict__ a, float* out, size_t n) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  float s = 0.f;
  for (; i < n; i += (size_t)gridDim.x * 256) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[0] = s;
}

// W-byte random accesses: L = max(1, W/16) lanes per access
template <int W>
__global__ __launch_bounds__(256) void rand_k(const char* __restrict__ t, size_t tbytes, float* out,
                                              size_t nacc) {
  constexpr int L = W >= 16 ? W / 16 : 1;
  const size_t g = ((size_t)blockIdx.x * 256 + threadIdx.x) / L;
  const int lane = threadIdx.x % L;
  if (g >= nacc) return;
  const size_t off = (mix(g) % (tbytes / W)) * W;
  float s;
  if (W == 8) {
    s = (float)*reinterpret_cast<const uint64_t*>(t + off);
  } else {
    const float4 v = *reinterpret_cast<const float4*>(t + off + 16 * lane);
    s = v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[0] = s;
}

// 32 slots per 256-thread block, as the D = 128 lookup (8 groups x NB = 4)
__global__ __launch_bounds__(256) void keys_k(const int64_t* __restrict__ k, int T, int B, int bt,
                                              int64_t* out) {
  if (threadIdx.x >= 32) return;
  const int64_t s = (int64_t)blockIdx.x * 32 + threadIdx.x;
  if (s >= (int64_t)T * B) return;
  const int64_t b = s / T, tt = s - b * T;
  const int64_t v = bt ? k[b * T + tt] : k[tt * B + b];
  if (v == 0x7fffffffffffll) out[0] = v;
}

int main() {
  const size_t tbytes = 8ull << 30, sbytes = 1ull << 30;
  const size_t nacc = 16u << 20;
  char* t;
  float* out;
  int64_t* kk;
  CK(hipMalloc(&t, tbytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(t, 1, tbytes));
  const int T = 26, B = 65536;
  CK(hipMalloc(&kk, (size_t)T * B * 8));
  CK(hipMemset(kk, 0, (size_t)T * B * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms;
  auto rep = [&](const char* name, double req_bytes) {
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-10s requested %12.0f B  %8.3f ms  %7.1f GB/s requested\n", name, req_bytes, ms,
           req_bytes / (ms * 1e-3) / 1e9);
  };
  // evict: one pass over a second 1 GiB region between launches
  auto evict = [&]() {
    hipLaunchKernelGGL(stream_k, dim3(4096), dim3(256), 0, 0, (const float4*)(t + sbytes),
                       out, sbytes / 16);
  };
  for (int rep_i = 0; rep_i < 2; ++rep_i) {
    evict();
    hipEventRecord(e0);
    hipLaunchKernelGGL(stream_k, dim3(8192), dim3(256), 0, 0, (const float4*)t, out, sbytes / 16);
    hipEventRecord(e1);
    CK(hipEventSynchronize(e1));
    rep("stream", (double)sbytes);
#define RAND(W)                                                                               \
    evict();                                                                                  \
    hipEventRecord(e0);                                                                       \
    hipLaunchKernelGGL(rand_k<W>, dim3((unsigned)((nacc * (W >= 16 ? W / 16 : 1) + 255) / 256)), \
                       dim3(256), 0, 0, t, tbytes, out, nacc);                                \
    hipEventRecord(e1);                                                                       \
    CK(hipEventSynchronize(e1));                                                              \
    rep("rand" #W, (double)nacc * W);
    RAND(8) RAND(16) RAND(64) RAND(128) RAND(512)
    for (int bt = 0; bt < 2; ++bt) {
      evict();
      hipEventRecord(e0);
      hipLaunchKernelGGL(keys_k, dim3((T * B + 31) / 32), dim3(256), 0, 0, kk, T, B, bt,
                         (int64_t*)out);
      hipEventRecord(e1);
      CK(hipEventSynchronize(e1));
      rep(bt ? "keys_bt" : "keys_tb", (double)T * B * 8);
    }
  }
  CK(hipGetLastError());
  return 0;
}
