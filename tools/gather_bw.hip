// gather_bw.hip -- shape study for the one-hot gather-copy (pool_onehot_kernel):
// out[j] = table[idx[j]] for 512-byte rows, varying rows in flight per lane
// group (NB), cache policy (default / nontemporal) and the index pattern
// (sequential = a plain copy through the indirection, random).  Not part of
// the product; results feed DESIGN.md.
//   hipcc -O3 --offload-arch=gfx950 tools/gather_bw.hip -o tools/gather_bw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int NB, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void gather_k(const f4* __restrict__ table, const int64_t* __restrict__ idx,
                                                f4* __restrict__ out, int64_t n) {
  constexpr int G = 32;  // 32 lanes x 16 B = one 512-byte row
  const int64_t j0 = ((int64_t)blockIdx.x * (256 / G) + threadIdx.x / G) * NB;
  const int lg = threadIdx.x % G;
  f4 x[NB];
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int64_t j = j0 + k;
    if (j < n) {
      const f4* p = table + idx[j] * G + lg;
      x[k] = NTL ? __builtin_nontemporal_load(p) : *p;
    }
  }
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int64_t j = j0 + k;
    if (j < n) {
      f4* q = out + j * G + lg;
      if (NTS) __builtin_nontemporal_store(x[k], q); else *q = x[k];
    }
  }
}

__global__ void fill_idx(int64_t* idx, int64_t n, int64_t rows, int mode, uint64_t seed) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  if (mode == 0) { idx[j] = j % rows; return; }
  uint64_t z = seed + (uint64_t)j * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  idx[j] = (int64_t)(z % (uint64_t)rows);
}

template <int NB, bool NTL, bool NTS>
static float run(const f4* table, const int64_t* idx, f4* out, int64_t n, int iters) {
  const unsigned blocks = (unsigned)((n + NB * 8 - 1) / (NB * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((gather_k<NB, NTL, NTS>), dim3(blocks), dim3(256), 0, 0, table, idx, out, n);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((gather_k<NB, NTL, NTS>), dim3(blocks), dim3(256), 0, 0, table, idx, out, n);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main(int argc, char** argv) {
  const int64_t rows = (int64_t)(argc > 1 ? atof(argv[1]) : 32.0) * (1ll << 30) / 512;  // table GiB
  const int64_t n = 26ll * 65536;  // lookups per launch (bench shape)
  f4 *table, *out;
  int64_t* idx;
  CK(hipMalloc(&table, rows * 512));
  CK(hipMalloc(&out, n * 512));
  CK(hipMalloc(&idx, n * 8));
  CK(hipMemset(table, 0, rows * 512));
  const int iters = 20;
  const double bytes = (double)n * (512 + 512 + 8);
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(fill_idx, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, idx, n, rows, mode, 7ull);
    CK(hipDeviceSynchronize());
    const char* m = mode == 0 ? "sequential" : "random";
#define R(NB, L, S, NAME)                                                                          \
  {                                                                                                \
    float ms = run<NB, L, S>(table, idx, out, n, iters);                                           \
    printf("{\"idx\":\"%s\",\"kernel\":\"%s\",\"us\":%.1f,\"GBps\":%.1f}\n", m, NAME, ms * 1e3,     \
           bytes / ms / 1e6);                                                                      \
  }
    R(1, false, false, "NB1 default");
    R(1, true, true, "NB1 nt");
    R(2, false, false, "NB2 default");
    R(2, true, true, "NB2 nt");
    R(4, false, false, "NB4 default");
    R(4, true, true, "NB4 nt");
    R(4, true, false, "NB4 ntload");
    R(4, false, true, "NB4 ntstore");
    R(8, true, true, "NB8 nt");
  }
  return 0;
}
