// Round 6: does a hipGraph replay give a kernel the dynamic LDS it was
// captured with?  (tools/graph_piece_probe.py: the captured DIN step goes
// wrong from its second replay on, only through the kernels that take
// dynamic LDS -- din_pool_kernel -- and not with DEBUG_CLR_GRAPH_PACKET_
// CAPTURE=0.)
//
// Every workgroup fills its whole dynamic LDS region with a word pattern of
// its own, spins a while (so that workgroups sharing a CU overlap in time),
// and counts the words that no longer hold its pattern.  A launch that
// allocates less LDS than asked lets co-resident workgroups alias, and the
// count goes non-zero.  The kernel is launched eagerly, then captured into a
// graph and replayed; between replays, eager launches of an unrelated
// kernel (the allocator churn of the Python probe did the same).
//
// build: hipcc --offload-arch=gfx950 -O2 tools/dynlds_graph_probe.hip -o tools/dynlds_graph_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ __launch_bounds__(64) void fill_check_kernel(int words, unsigned* errors) {
  extern __shared__ unsigned lds[];
  const unsigned tag = 0x9E3779B9u * (blockIdx.x + 1);
  for (int i = threadIdx.x; i < words; i += 64) lds[i] = tag ^ (unsigned)i;
  __syncthreads();
  for (int k = 0; k < 200; ++k) __builtin_amdgcn_s_sleep(10);
  __syncthreads();
  unsigned bad = 0;
  for (int i = threadIdx.x; i < words; i += 64) bad += lds[i] != (tag ^ (unsigned)i);
  if (bad) atomicAdd(errors, bad);
}

__global__ void busy_kernel(float* x, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] * 0.5f + 1.0f;
}

int main(int argc, char** argv) {
  const int words = argc > 1 ? atoi(argv[1]) : 612;   // din_pool_kernel at T = 100: 2448 B
  const int grid = argc > 2 ? atoi(argv[2]) : 4096;
  unsigned* err = nullptr;
  float* junk = nullptr;
  CK(hipMalloc(&err, sizeof(unsigned)));
  CK(hipMalloc(&junk, (1 << 20) * sizeof(float)));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const size_t lds = (size_t)words * 4;
  auto result = [&](const char* what) {
    unsigned h = 0;
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(&h, err, sizeof(h), hipMemcpyDeviceToHost));
    printf("%-28s words %d grid %d: %u LDS words overwritten\n", what, words, grid, h);
    CK(hipMemsetAsync(err, 0, sizeof(unsigned), st));
    CK(hipStreamSynchronize(st));
    return h;
  };
  CK(hipMemsetAsync(err, 0, sizeof(unsigned), st));
  hipLaunchKernelGGL(fill_check_kernel, dim3(grid), dim3(64), lds, st, words, err);
  unsigned bad = result("eager launch");
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(fill_check_kernel, dim3(grid), dim3(64), lds, st, words, err);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int r = 0; r < 4; ++r) {
    CK(hipGraphLaunch(ge, st));
    char name[64];
    snprintf(name, sizeof(name), "graph replay %d", r);
    bad += result(name);
    for (int k = 0; k < 1000; ++k)
      hipLaunchKernelGGL(busy_kernel, dim3(1 << 12), dim3(256), 0, st, junk, 1 << 20);
  }
  printf("dynlds_graph_probe: %s\n", bad ? "LDS ALIASED" : "ok");
  return bad ? 2 : 0;
}
