// Serial fp32 add-chain rate on gfx950: one wave walks N dependent
// v_add_f32 (a) from registers, (b) through the LDS walk the long-run
// gradient kernels use (chain_walk: 16-B reads 16 positions ahead, counted
// waits), (c) as (b) with 15 other waves of the block writing the LDS.
// Prints cycles per add from s_memtime around the walk.  hipcc
// --offload-arch=gfx950 -O3 -I../deeprec-1_amd/csrc tools/chain_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "dr_rows.h"

using namespace dr;

__global__ __launch_bounds__(64) void reg_chain(const float* x, int n, float* out, long long* cyc) {
  float a = x[threadIdx.x], b = x[64 + threadIdx.x];
  float acc = 0.f;
  const long long t0 = clock64();
  for (int i = 0; i < n; i += 8) {
    acc = acc + a; acc = acc + b; acc = acc + a; acc = acc + b;
    acc = acc + a; acc = acc + b; acc = acc + a; acc = acc + b;
  }
  const long long t1 = clock64();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <bool BUSY>
__global__ __launch_bounds__(1024) void lds_chain(const float* x, int reps, float* out,
                                                  long long* cyc) {
  constexpr int S = 960, SP = S + 4;
  __shared__ __attribute__((aligned(16))) float st[2 * 16 * SP];
  for (int i = threadIdx.x; i < 2 * 16 * SP; i += blockDim.x) st[i] = x[i & 1023];
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  float acc = 0.f;
  bool fresh = true;
  long long t0 = 0, t1 = 0;
  if (wave == 0) {
    __builtin_amdgcn_s_setprio(3);
    t0 = clock64();
    for (int r = 0; r < reps; ++r)
      acc = chain_walk(st + (r & 1) * 16 * SP + (lane & 15) * SP, S, fresh, acc);
    t1 = clock64();
  } else if (BUSY) {   // the loaders' transposed stage writes, continuously
    for (int r = 0; r < reps; ++r) {
      float* c = st + (r & 1) * 16 * SP + ((threadIdx.x & 7) * 2) * SP + (threadIdx.x >> 3);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        c[q * 120] = acc + q;
        c[SP + q * 120] = acc - q;
      }
    }
  }
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  float *x, *out;
  long long* cyc;
  hipMalloc(&x, 4096 * 4);
  hipMalloc(&out, 4096 * 4);
  hipMalloc(&cyc, 8);
  std::vector<float> h(4096);
  for (int i = 0; i < 4096; ++i) h[i] = 1e-3f * (i % 97);
  hipMemcpy(x, h.data(), 4096 * 4, hipMemcpyHostToDevice);
  long long c = 0;
  const int n = 1 << 20;
  hipLaunchKernelGGL(reg_chain, dim3(1), dim3(64), 0, 0, x, n, out, cyc);
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("{\"probe\":\"chain\",\"form\":\"registers\",\"adds\":%d,\"cycles_per_add\":%.2f}\n", n,
         (double)c / n);
  const int reps = 2000;
  hipLaunchKernelGGL((lds_chain<false>), dim3(1), dim3(1024), 0, 0, x, reps, out, cyc);
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("{\"probe\":\"chain\",\"form\":\"lds walk, idle block\",\"adds\":%d,\"cycles_per_add\":%.2f}\n",
         reps * 960, (double)c / (reps * 960.0));
  hipLaunchKernelGGL((lds_chain<true>), dim3(1), dim3(1024), 0, 0, x, reps, out, cyc);
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("{\"probe\":\"chain\",\"form\":\"lds walk, 15 waves writing LDS\",\"adds\":%d,\"cycles_per_add\":%.2f}\n",
         reps * 960, (double)c / (reps * 960.0));
  hipDeviceSynchronize();
  return 0;
}
