// uncached_reuse_probe.hip -- targeted probe of the round-2 hazard "coarse-
// grained hipMalloc reusing memory freed from a hipDeviceMallocUncached
// allocation returned corrupted rows" (VERDICT r02 #7).  Not part of the
// product (the library never frees uncached blocks, dr_ipc_free); results
// feed DESIGN.md.
//
// Each trial: allocate an uncached block U (hipExtMallocWithFlags(
// hipDeviceMallocUncached)), write it with a kernel (pattern A) and read it
// from every XCD, hipFree it, then hipMalloc the same size (reports whether
// the VA came back), and exercise the new block the way an EV pool is used:
//   1. plain kernel stores of pattern B from blocks spread over all XCDs,
//      then a second kernel reading every word (plain loads) and counting
//      words != B                                        -> "stale_after_write"
//   2. device-scope atomicAdd on 4096 counters from every block (the EV
//      row counter / CAS pattern), totals checked          -> "atomic_errors"
//   3. write in one kernel, read with nontemporal loads in the next
//                                                         -> "stale_nt"
// A control trial reallocates after freeing a COARSE-grained block.
//   hipcc -O3 --offload-arch=gfx950 tools/uncached_reuse_probe.hip -o tools/uncached_reuse_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__);                \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void fill_k(uint32_t* p, int64_t n, uint32_t salt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)(i * 2654435761u) ^ salt;
}

__global__ void check_k(const uint32_t* p, int64_t n, uint32_t salt, unsigned long long* bad,
                        int nt) {
  unsigned long long b = 0;
  // read in a different block -> address mapping than fill_k (reverse order)
  for (int64_t i = (int64_t)(gridDim.x - 1 - blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t v = nt ? __builtin_nontemporal_load(p + i) : p[i];
    b += v != ((uint32_t)(i * 2654435761u) ^ salt);
  }
  if (b) atomicAdd(bad, b);
}

__global__ void atomics_k(unsigned int* ctr, int nctr, int reps) {
  for (int r = 0; r < reps; ++r)
    atomicAdd(ctr + ((blockIdx.x * 131 + threadIdx.x + r * 17) % nctr), 1u);
}

__global__ void sum_k(const unsigned int* ctr, int nctr, unsigned long long* tot) {
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < nctr; i += blockDim.x) s += ctr[i];
  atomicAdd(tot, s);
}

static void trial(int uncached_first, size_t bytes, int t) {
  const int64_t n = (int64_t)(bytes / 4);
  void* u = nullptr;
  if (uncached_first)
    CK(hipExtMallocWithFlags(&u, bytes, hipDeviceMallocUncached));
  else
    CK(hipMalloc(&u, bytes));
  hipLaunchKernelGGL(fill_k, dim3(2048), dim3(256), 0, 0, (uint32_t*)u, n, 0xA5A5A5A5u);
  unsigned long long* bad;
  CK(hipMalloc(&bad, 16));
  CK(hipMemset(bad, 0, 16));
  hipLaunchKernelGGL(check_k, dim3(2048), dim3(256), 0, 0, (const uint32_t*)u, n, 0xA5A5A5A5u,
                     bad, 0);
  CK(hipDeviceSynchronize());
  CK(hipFree(u));
  void* c = nullptr;
  CK(hipMalloc(&c, bytes));
  const int same_va = c == u;
  unsigned long long h[2] = {0, 0};
  // 1. plain stores then plain loads from other blocks / XCDs
  CK(hipMemset(bad, 0, 16));
  hipLaunchKernelGGL(fill_k, dim3(2048), dim3(256), 0, 0, (uint32_t*)c, n, 0x5A5A0000u + t);
  hipLaunchKernelGGL(check_k, dim3(2048), dim3(256), 0, 0, (const uint32_t*)c, n,
                     0x5A5A0000u + t, bad, 0);
  // 3. nontemporal reads of the same words
  hipLaunchKernelGGL(check_k, dim3(2048), dim3(256), 0, 0, (const uint32_t*)c, n,
                     0x5A5A0000u + t, bad + 1, 1);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost));
  // 2. device-scope atomics on counters at the start of the block
  const int nctr = 4096, reps = 64;
  CK(hipMemset(c, 0, nctr * 4));
  hipLaunchKernelGGL(atomics_k, dim3(2048), dim3(256), 0, 0, (unsigned int*)c, nctr, reps);
  unsigned long long* tot;
  CK(hipMalloc(&tot, 8));
  CK(hipMemset(tot, 0, 8));
  hipLaunchKernelGGL(sum_k, dim3(1), dim3(256), 0, 0, (const unsigned int*)c, nctr, tot);
  unsigned long long ht = 0;
  CK(hipMemcpy(&ht, tot, 8, hipMemcpyDeviceToHost));
  const unsigned long long want = 2048ull * 256 * reps;
  printf("{\"trial\":%d,\"freed\":\"%s\",\"bytes\":%zu,\"same_va\":%d,\"stale_after_write\":%llu,"
         "\"stale_nt\":%llu,\"atomic_errors\":%lld}\n",
         t, uncached_first ? "uncached" : "coarse", bytes, same_va, h[0], h[1],
         (long long)(want - ht));
  CK(hipFree(c));
  CK(hipFree(bad));
  CK(hipFree(tot));
}

// Small blocks (sub-allocated): many uncached blocks zero-filled by a kernel
// and freed, then small hipMalloc blocks written by a HOST-TO-DEVICE copy and
// read by a kernel ("stale_h2d": words the kernel does not see as written).
static void small_h2d_trial(size_t bytes, int nblk) {
  void* u[64];
  for (int i = 0; i < nblk; ++i) {
    CK(hipExtMallocWithFlags(&u[i], bytes, hipDeviceMallocUncached));
    hipLaunchKernelGGL(fill_k, dim3(64), dim3(256), 0, 0, (uint32_t*)u[i], (int64_t)(bytes / 4), 0u);
  }
  CK(hipDeviceSynchronize());
  for (int i = 0; i < nblk; ++i) CK(hipFree(u[i]));
  const int64_t n = (int64_t)(bytes / 4);
  uint32_t* h = (uint32_t*)malloc(bytes);
  for (int64_t i = 0; i < n; ++i) h[i] = (uint32_t)(i * 2654435761u) ^ 0x77u;
  unsigned long long* bad;
  CK(hipMalloc(&bad, 8));
  CK(hipMemset(bad, 0, 8));
  int reused = 0;
  void* c[64];
  for (int i = 0; i < nblk; ++i) {
    CK(hipMalloc(&c[i], bytes));
    for (int j = 0; j < nblk; ++j) reused += c[i] == u[j];
    CK(hipMemcpy(c[i], h, bytes, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(check_k, dim3(64), dim3(256), 0, 0, (const uint32_t*)c[i], n, 0x77u, bad, 0);
  }
  unsigned long long hb = 0;
  CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  printf("{\"small_h2d\":1,\"bytes\":%zu,\"blocks\":%d,\"same_va\":%d,\"stale_h2d\":%llu}\n",
         bytes, nblk, reused, hb);
  for (int i = 0; i < nblk; ++i) CK(hipFree(c[i]));
  CK(hipFree(bad));
  free(h);
}

int main(int argc, char** argv) {
  if (argc > 2 && atoi(argv[2]) == 1) {
    const size_t sz[4] = {512, 4096, 65536, 1 << 20};
    for (int i = 0; i < 4; ++i) small_h2d_trial(sz[i], 32);
    return 0;
  }
  const int trials = argc > 1 ? atoi(argv[1]) : 6;
  const size_t sizes[3] = {(size_t)64 << 20, (size_t)1 << 30, (size_t)4 << 30};
  for (int t = 0; t < trials; ++t) {
    const size_t b = sizes[t % 3];
    trial(1, b, t);
    trial(0, b, t);
  }
  return 0;
}
