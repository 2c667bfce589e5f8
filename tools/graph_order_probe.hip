// Round 6: are the nodes of a replayed hipGraph ordered and coherent?
// (The captured DIN step is right on its first replay and wrong from the
// second on unless DEBUG_CLR_GRAPH_PACKET_CAPTURE=0; tools/graph_piece_probe.py
// narrows it to lookups -> a torch reduction -> din_pool_kernel.)
//
// One graph, captured on one stream, replayed R times:
//   produce_kernel  x[i] = epoch * 1000003 + i, epoch read from device memory
//                   (slow: spins first, so an overlapping consumer would see
//                   the previous replay's x)
//   [optional memset / memcpy node, as torch's zeros / clone put in a graph]
//   consume_kernel  dynamic LDS like din_pool_kernel; counts x[i] that do not
//                   hold this epoch's value, then bumps the epoch
// Eager launches of an unrelated kernel run between replays.
//
// build: hipcc --offload-arch=gfx950 -O2 tools/graph_order_probe.hip -o tools/graph_order_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void produce_kernel(int* x, int n, const int* epoch) {
  for (int k = 0; k < 50; ++k) __builtin_amdgcn_s_sleep(20);
  const int e = *epoch;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    x[i] = e * 1000003 + i;
}

__global__ __launch_bounds__(64) void consume_kernel(const int* x, const int* y, int n,
                                                     int per, int* epoch, unsigned* errors) {
  extern __shared__ int lds[];
  const int e = *epoch;
  const int b0 = blockIdx.x * per;
  for (int j = threadIdx.x; j < per; j += 64) lds[j] = b0 + j < n ? x[b0 + j] : 0;
  __syncthreads();
  unsigned bad = 0;
  for (int j = threadIdx.x; j < per && b0 + j < n; j += 64) {
    bad += lds[j] != e * 1000003 + b0 + j;
    if (y) bad += y[b0 + j] != e * 1000003 + b0 + j;
  }
  if (bad) atomicAdd(errors, bad);
}

__global__ void bump_kernel(int* epoch) { *epoch += 1; }

__global__ void busy_kernel(float* x, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] * 0.5f + 1.0f;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "plain";   // plain | memset | memcpy
  const int n = 1 << 22, per = 1024, grid = n / per;
  int *x, *y, *epoch, *scratch;
  unsigned* err;
  float* junk;
  CK(hipMalloc(&x, n * sizeof(int)));
  CK(hipMalloc(&y, n * sizeof(int)));
  CK(hipMalloc(&scratch, n * sizeof(int)));
  CK(hipMalloc(&epoch, sizeof(int)));
  CK(hipMalloc(&err, sizeof(unsigned)));
  CK(hipMalloc(&junk, (1 << 20) * sizeof(float)));
  CK(hipMemset(epoch, 0, sizeof(int)));
  CK(hipMemset(err, 0, sizeof(unsigned)));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const bool cp = !strcmp(mode, "memcpy"), ms = !strcmp(mode, "memset");
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  if (ms) CK(hipMemsetAsync(scratch, 0, n * sizeof(int), st));
  hipLaunchKernelGGL(produce_kernel, dim3(1024), dim3(256), 0, st, x, n, epoch);
  if (cp) CK(hipMemcpyAsync(y, x, n * sizeof(int), hipMemcpyDeviceToDevice, st));
  hipLaunchKernelGGL(consume_kernel, dim3(grid), dim3(64), per * sizeof(int), st, x,
                     cp ? y : nullptr, n, per, epoch, err);
  hipLaunchKernelGGL(bump_kernel, dim3(1), dim3(1), 0, st, epoch);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  unsigned total = 0;
  for (int r = 0; r < 6; ++r) {
    CK(hipGraphLaunch(ge, st));
    unsigned h = 0;
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(&h, err, sizeof(h), hipMemcpyDeviceToHost));
    CK(hipMemset(err, 0, sizeof(unsigned)));
    printf("%-7s replay %d: %u stale values\n", mode, r, h);
    total += h;
    for (int k = 0; k < 1000; ++k)
      hipLaunchKernelGGL(busy_kernel, dim3(1 << 12), dim3(256), 0, st, junk, 1 << 20);
  }
  printf("graph_order_probe %s: %s\n", mode, total ? "STALE READS" : "ok");
  return total ? 2 : 0;
}
