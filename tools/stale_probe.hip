// stale_probe.hip -- does a GPU read return stale data for memory that was
// re-written by a DMA copy / memset / another kernel after this GPU's L2s
// cached its previous contents?  (Diagnosis aid for the EV grow / create
// paths)
//
//   hipcc --offload-arch=gfx950 -O3 tools/stale_probe.hip -o tools/stale_probe
//
// For each writer W in {kernel fill, hipMemsetAsync, hipMemcpyAsync D2D,
// hipMemcpyAsync H2D} and reader policy R in {plain, nontemporal}:
//   1. kernel writes pattern A to buffer X and every block reads it back
//      (pulls X into all 8 XCD L2s), repeated twice;
//   2. W writes pattern B to X;
//   3. a kernel on all XCDs reads X with policy R and counts words != B.
// Also the re-allocation variant: free X, malloc Y of the same size (same
// address in practice), write B with W, read.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__global__ void fill_k(unsigned* p, size_t n, unsigned v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

__global__ void touch_k(const unsigned* p, size_t n, unsigned* sink) {
  unsigned acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    acc += p[i];
  if (acc == 0x12345678u) *sink = acc;
}

template <bool NT>
__global__ void check_k(const unsigned* p, size_t n, unsigned v, unsigned long long* bad) {
  unsigned long long b = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const unsigned x = NT ? __builtin_nontemporal_load(p + i) : p[i];
    b += x != v;
  }
  if (b) atomicAdd(bad, b);
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 8) << 20;  // MiB
  const size_t n = bytes / 4;
  unsigned *sink, *src;
  unsigned long long* bad;
  CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&bad, 8));
  CK(hipMalloc(&src, bytes));
  std::vector<unsigned> host(n, 0xBBBBBBBBu);
  hipStream_t s;
  CK(hipStreamCreate(&s));
  fill_k<<<1024, 256, 0, s>>>(src, n, 0xBBBBBBBBu);
  const char* wname[] = {"kernel fill", "hipMemsetAsync", "hipMemcpyAsync D2D",
                         "hipMemcpyAsync H2D"};
  for (int realloc_ = 0; realloc_ < 2; ++realloc_)
    for (int w = 0; w < 4; ++w)
      for (int nt = 0; nt < 2; ++nt) {
        unsigned long long total = 0;
        for (int rep = 0; rep < 20; ++rep) {
          unsigned* x;
          CK(hipMalloc(&x, bytes));
          fill_k<<<2048, 256, 0, s>>>(x, n, 0xAAAAAAAAu);
          for (int k = 0; k < 2; ++k) touch_k<<<2048, 256, 0, s>>>(x, n, sink);
          CK(hipStreamSynchronize(s));
          if (realloc_) {
            CK(hipFree(x));
            CK(hipMalloc(&x, bytes));
          }
          if (w == 0) fill_k<<<2048, 256, 0, s>>>(x, n, 0xBBBBBBBBu);
          if (w == 1) CK(hipMemsetAsync(x, 0xBB, bytes, s));
          if (w == 2) CK(hipMemcpyAsync(x, src, bytes, hipMemcpyDeviceToDevice, s));
          if (w == 3) CK(hipMemcpyAsync(x, host.data(), bytes, hipMemcpyHostToDevice, s));
          fill_k<<<1, 64, 0, s>>>((unsigned*)bad, 2, 0u);
          if (nt)
            check_k<true><<<2048, 256, 0, s>>>(x, n, 0xBBBBBBBBu, bad);
          else
            check_k<false><<<2048, 256, 0, s>>>(x, n, 0xBBBBBBBBu, bad);
          unsigned long long b = 0;
          CK(hipMemcpyAsync(&b, bad, 8, hipMemcpyDeviceToHost, s));
          CK(hipStreamSynchronize(s));
          total += b;
          CK(hipFree(x));
        }
        printf("{\"realloc\": %d, \"writer\": \"%s\", \"reader\": \"%s\", \"stale_words\": %llu, "
               "\"words_checked\": %zu}\n",
               realloc_, wname[w], nt ? "nontemporal" : "plain", total, n * 20);
        fflush(stdout);
      }
  // Uncached round trip (xgmi.hip dr_ipc_alloc history):
  // cached X warmed into every XCD L2 with pattern A -> hipFree -> an
  // UNCACHED allocation U (hipDeviceMallocUncached) written B by a kernel
  // (its stores bypass L2) -> hipFree -> a cached hipMalloc Y written C by
  // writer w -> every XCD reads Y.  Counts words != C, and how many of those
  // read A (a stale L2 line of the first cached use) or B.
  for (int w = 0; w < 2; ++w)
    for (int nt = 0; nt < 2; ++nt) {
      unsigned long long total = 0, same_u = 0, same_y = 0;
      for (int rep = 0; rep < 20; ++rep) {
        unsigned *x, *u, *y;
        CK(hipMalloc(&x, bytes));
        fill_k<<<2048, 256, 0, s>>>(x, n, 0xAAAAAAAAu);
        for (int k = 0; k < 2; ++k) touch_k<<<2048, 256, 0, s>>>(x, n, sink);
        CK(hipStreamSynchronize(s));
        CK(hipFree(x));
        CK(hipExtMallocWithFlags((void**)&u, bytes, hipDeviceMallocUncached));
        same_u += u == x;
        fill_k<<<2048, 256, 0, s>>>(u, n, 0xBBBBBBBBu);
        for (int k = 0; k < 2; ++k) touch_k<<<2048, 256, 0, s>>>(u, n, sink);
        CK(hipStreamSynchronize(s));
        CK(hipFree(u));
        CK(hipMalloc(&y, bytes));
        same_y += y == u;
        if (w == 0) fill_k<<<2048, 256, 0, s>>>(y, n, 0xCCCCCCCCu);
        if (w == 1) CK(hipMemsetAsync(y, 0xCC, bytes, s));
        fill_k<<<1, 64, 0, s>>>((unsigned*)bad, 2, 0u);
        if (nt)
          check_k<true><<<2048, 256, 0, s>>>(y, n, 0xCCCCCCCCu, bad);
        else
          check_k<false><<<2048, 256, 0, s>>>(y, n, 0xCCCCCCCCu, bad);
        unsigned long long b = 0;
        CK(hipMemcpyAsync(&b, bad, 8, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        total += b;
        CK(hipFree(y));
      }
      printf("{\"uncached_round_trip\": 1, \"writer\": \"%s\", \"reader\": \"%s\", "
             "\"stale_words\": %llu, \"words_checked\": %zu, \"u_reused_x_va\": %llu, "
             "\"y_reused_u_va\": %llu}\n",
             wname[w], nt ? "nontemporal" : "plain", total, n * 20, same_u, same_y);
      fflush(stdout);
    }
  return 0;
}
