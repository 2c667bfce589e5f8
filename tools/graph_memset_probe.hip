// Round 6: a memset node followed by a kernel that counts on it being zero,
// the pattern of torch's multi-block reductions (Reduce.cuh: semaphores
// zeroed with cudaMemsetAsync, the last block to arrive -- atomicAdd ==
// gridDim - 1 -- folds the partial sums).  In a replayed hipGraph the
// counter must start from zero every replay; if it does not, no block sees
// itself last and the result is never written (or is written early).
//
// Graph: [memset sem] -> reduce_kernel (partials + arrival count; the last
// block writes the total) -> check.  Replayed R times, eager kernels between.
//
// build: hipcc --offload-arch=gfx950 -O2 tools/graph_memset_probe.hip -o tools/graph_memset_probe
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

__global__ void reduce_kernel(const float* x, int n, float* partial, unsigned* sem, float* out) {
  __shared__ float s[256];
  __shared__ bool last;
  float v = 0.f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) v += x[i];
  s[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = s[0];
    __threadfence();
    last = atomicAdd(sem, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) {
    __threadfence();
    float t = 0.f;
    for (unsigned b = 0; b < gridDim.x; ++b) t += __hip_atomic_load(&partial[b], __ATOMIC_RELAXED,
                                                                     __HIP_MEMORY_SCOPE_AGENT);
    *out = t;
  }
}

__global__ void poison_kernel(float* out) { *out = -1.f; }

__global__ void busy_kernel(float* x, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] * 0.5f + 1.0f;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "memset";   // memset | kernelzero
  const int n = 1 << 20, grid = 512;
  float *x, *partial, *out, *junk;
  unsigned* sem;
  CK(hipMalloc(&x, n * sizeof(float)));
  CK(hipMalloc(&partial, grid * sizeof(float)));
  CK(hipMalloc(&out, sizeof(float)));
  CK(hipMalloc(&sem, 64));
  CK(hipMalloc(&junk, (1 << 20) * sizeof(float)));
  float* h = (float*)malloc(n * sizeof(float));
  for (int i = 0; i < n; ++i) h[i] = 1.0f;
  CK(hipMemcpy(x, h, n * sizeof(float), hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(poison_kernel, dim3(1), dim3(1), 0, st, out);
  if (!strcmp(mode, "memset"))
    CK(hipMemsetAsync(sem, 0, sizeof(unsigned), st));
  else
    CK(hipMemsetD32Async((hipDeviceptr_t)sem, 0, 1, st));
  hipLaunchKernelGGL(reduce_kernel, dim3(grid), dim3(256), 0, st, x, n, partial, sem, out);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  int bad = 0;
  for (int r = 0; r < 6; ++r) {
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    float o = 0.f;
    unsigned sv = 0;
    CK(hipMemcpy(&o, out, sizeof(o), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&sv, sem, sizeof(sv), hipMemcpyDeviceToHost));
    printf("%-10s replay %d: sum %.1f (want %d), counter after %u (want %d)\n", mode, r, o, n, sv,
           grid);
    bad += o != (float)n;
    for (int k = 0; k < 1000; ++k)
      hipLaunchKernelGGL(busy_kernel, dim3(1 << 12), dim3(256), 0, st, junk, 1 << 20);
  }
  printf("graph_memset_probe %s: %s\n", mode, bad ? "WRONG" : "ok");
  return bad ? 2 : 0;
}
