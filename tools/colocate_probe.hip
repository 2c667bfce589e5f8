// colocate_probe.hip -- is a key co-located with its row cheaper than a
// separate 16-B hash slot?  (VERDICT r02 "next" #3: "a hash-placed, bucketed
// row arena whose first 16 B per row hold the key, so the probe's line is the
// row's first line".)  Not part of the product; results feed DESIGN.md.
//
// Same shape as the bench's dominant kernel: 26 x 65 536 one-hot lookups of
// D = 128 fp32 rows, output in slot order (b*T + t), 32 lanes per row, 4 rows
// in flight per lane group, nontemporal loads / stores, keys read from a
// record-major id matrix.  Four variants, each over 4 rotating batches:
//   gather     pre-resolved row ids -> 512-B row -> out   (pool_onehot shape)
//   separate   key -> 16-B slot {key, row} at mix(key) -> row -> out
//              (ev_lookup_onehot shape: two dependent HBM round trips)
//   colocated  key -> arena row at mix(key) with stride 528 B: the 16-B
//              {key, meta} header and the 512-B row read TOGETHER (one round
//              trip; the key is checked after the loads), 5 lines touched
//   coloc640   the same with rows padded to 640 B (5 aligned lines)
//   tail640    640-B rows with the 512-B data line-aligned at offset 0 and
//              the header in the fifth line (4 full lines + one 16-B read,
//              like `separate`, but with no dependent round trip)
// Every probe hits at its home position (no collisions): the best case for
// both hashed layouts.
//   hipcc -O3 --offload-arch=gfx950 tools/colocate_probe.hip -o tools/colocate_probe
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

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u2v __attribute__((ext_vector_type(2)));

static constexpr int T = 26;
static constexpr int64_t B = 65536;
static constexpr int64_t N = T * B;
static constexpr int G = 32;   // lanes per row
static constexpr int NB = 4;   // rows in flight per lane group

__device__ __host__ inline uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

// MODE 0 gather (ids = row ids), 1 separate slots, 2 colocated (stride S
// floats), all with the same lane layout and store path.
template <int MODE, int S>
__global__ __launch_bounds__(256) void lookup_k(const int64_t* __restrict__ ids,
                                                const u2v* __restrict__ slots, uint64_t smask,
                                                const float* __restrict__ arena, uint64_t amod,
                                                f4* __restrict__ out, int* __restrict__ bad) {
  const int64_t s0 = ((int64_t)blockIdx.x * (256 / G) + threadIdx.x / G) * NB;
  if (s0 >= N) return;
  const int lg = threadIdx.x % G;
  const int base = (int)(threadIdx.x % 64) - lg;
  // lanes 0..NB-1 of the group resolve one slot each
  const float* mine = nullptr;
  uint64_t key = 0;
  if (lg < NB) {
    key = (uint64_t)__builtin_nontemporal_load(ids + s0 + lg);
    if (MODE == 0) {
      mine = arena + (int64_t)key * S;
    } else if (MODE == 1) {
      const u2v sv = slots[mix64(key) & smask];
      if (sv.x != key) atomicAdd(bad, 1);
      mine = arena + (int64_t)sv.y * S;
    } else {  // MODE 2 / 3: home row of the hashed arena
      mine = arena + (int64_t)(mix64(key) % amod) * S;
    }
  }
  const float* p[NB];
  uint64_t kq[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const uint64_t u = (uint64_t)(uintptr_t)mine;
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)u, base + q, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(u >> 32), base + q, 64);
    p[q] = reinterpret_cast<const float*>((uintptr_t)(((uint64_t)hi << 32) | lo));
    const uint32_t klo = (uint32_t)__shfl((int)(uint32_t)key, base + q, 64);
    const uint32_t khi = (uint32_t)__shfl((int)(uint32_t)(key >> 32), base + q, 64);
    kq[q] = ((uint64_t)khi << 32) | klo;
  }
  f4 x[NB];
  u2v hd[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const float* row = MODE == 2 ? p[q] + 4 : p[q];   // colocated: data after the header
    x[q] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(row) + lg);
    if (MODE == 2 && lg == 0) hd[q] = __builtin_nontemporal_load(reinterpret_cast<const u2v*>(p[q]));
    if (MODE == 3 && lg == 0)
      hd[q] = __builtin_nontemporal_load(reinterpret_cast<const u2v*>(p[q] + 128));
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if ((MODE == 2 || MODE == 3) && lg == 0 && hd[q].x != kq[q]) atomicAdd(bad, 1);
    const int64_t s = s0 + q;
    __builtin_nontemporal_store(x[q], out + s * G + lg);
  }
}

__global__ void make_keys(int64_t* keys, int64_t n, uint64_t seed) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  keys[j] = (int64_t)(mix64(seed * 0x9E3779B97F4A7C15ull + (uint64_t)j) >> 1);
}

// slot table / arena headers for the keys used (home position, no collision
// handling needed for a timing probe: a later key overwrites an earlier one
// at the same position, counted as `bad` by the kernels and reported)
__global__ void place(const int64_t* keys, int64_t n, u2v* slots, uint64_t smask, float* arena,
                      uint64_t amod, int S, uint64_t rows, int mode) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t k = (uint64_t)keys[j];
  if (mode == 1) {
    u2v v;
    v.x = k;
    v.y = mix64(k ^ 0x5555) % rows;
    slots[mix64(k) & smask] = v;
  } else if (mode >= 2) {
    u2v v;
    v.x = k;
    v.y = 0;
    *reinterpret_cast<u2v*>(arena + (int64_t)(mix64(k) % amod) * S + (mode == 3 ? 128 : 0)) = v;
  }
}

__global__ void to_rows(const int64_t* keys, int64_t n, int64_t* rows, uint64_t nrows) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) rows[j] = (int64_t)(mix64((uint64_t)keys[j] ^ 0x5555) % nrows);
}

template <int MODE, int S>
static double run(int64_t* const* batch, const u2v* slots, uint64_t smask, const float* arena,
                  uint64_t amod, f4* out, int* bad, int iters) {
  const unsigned blocks = (unsigned)((N / NB + (256 / G) - 1) / (256 / G));
  for (int i = 0; i < 4; ++i)
    hipLaunchKernelGGL((lookup_k<MODE, S>), dim3(blocks), dim3(256), 0, 0, batch[i], slots, smask,
                       arena, amod, out, bad);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  double tot = 0;
  for (int i = 0; i < iters; ++i) {
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((lookup_k<MODE, S>), dim3(blocks), dim3(256), 0, 0, batch[i % 4], slots,
                       smask, arena, amod, out, bad);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  return tot / iters;
}

int main(int argc, char** argv) {
  const double arena_gib = argc > 1 ? atof(argv[1]) : 96.0;
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  int64_t* keys[4];
  int64_t* rowids[4];
  for (int i = 0; i < 4; ++i) {
    CK(hipMalloc(&keys[i], N * 8));
    CK(hipMalloc(&rowids[i], N * 8));
    hipLaunchKernelGGL(make_keys, dim3((unsigned)(N / 256)), dim3(256), 0, 0, keys[i], N,
                       (uint64_t)(1000 + i));
  }
  f4* out;
  int* bad;
  CK(hipMalloc(&out, N * 512));
  CK(hipMalloc(&bad, 4));
  // slot table: 26 tables x 2^24 slots x 16 B (the bench's EVs: cap 2^24)
  const uint64_t nslots = 26ull << 24;
  uint64_t smask = 1;
  while (smask < nslots) smask <<= 1;
  smask -= 1;  // power-of-two table covering 26 x 2^24
  const double bytes_sep = (double)N * (8 + 16 + 512 + 512);
  printf("{\"lookups\":%lld,\"algorithmic_B_per_lookup\":1048}\n", (long long)N);
  // ---- gather + separate share one row arena of 512-B rows
  {
    const uint64_t rows = (uint64_t)(arena_gib * (1ull << 30) / 512);
    float* arena;
    u2v* slots;
    CK(hipMalloc(&arena, rows * 512));
    CK(hipMalloc(&slots, (smask + 1) * 16));
    CK(hipMemset(arena, 0, rows * 512));
    CK(hipMemset(slots, 0xFF, (smask + 1) * 16));
    for (int i = 0; i < 4; ++i) {
      hipLaunchKernelGGL(place, dim3((unsigned)(N / 256)), dim3(256), 0, 0, keys[i], N, slots,
                         smask, arena, 1, 128, rows, 1);
      hipLaunchKernelGGL(to_rows, dim3((unsigned)(N / 256)), dim3(256), 0, 0, keys[i], N,
                         rowids[i], rows);
    }
    CK(hipMemset(bad, 0, 4));
    CK(hipDeviceSynchronize());
    double g = run<0, 128>(rowids, nullptr, 0, arena, 0, out, bad, iters);
    double sp = run<1, 128>(keys, slots, smask, arena, 0, out, bad, iters);
    int nb = 0;
    CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
    printf("{\"variant\":\"gather\",\"us\":%.1f,\"frac_1032B\":%.4f}\n", g * 1e3,
           (double)N * 1032 / (g * 1e-3) / 8e12);
    printf("{\"variant\":\"separate\",\"us\":%.1f,\"frac_1048B\":%.4f,\"slot_collisions_seen\":%d}\n",
           sp * 1e3, bytes_sep / (sp * 1e-3) / 8e12, nb);
    CK(hipFree(arena));
    CK(hipFree(slots));
  }
  // ---- colocated arenas (528-B and 640-B row stride)
  for (int v = 0; v < 3; ++v) {
    const int S = v == 0 ? 132 : 160;  // floats per row incl. the 16-B header
    const uint64_t rows = (uint64_t)(arena_gib * (1ull << 30) / (S * 4));
    float* arena;
    CK(hipMalloc(&arena, rows * S * 4));
    CK(hipMemset(arena, 0, rows * S * 4));
    for (int i = 0; i < 4; ++i)
      hipLaunchKernelGGL(place, dim3((unsigned)(N / 256)), dim3(256), 0, 0, keys[i], N, nullptr,
                         0, arena, rows, S, rows, v == 2 ? 3 : 2);
    CK(hipMemset(bad, 0, 4));
    CK(hipDeviceSynchronize());
    double c = v == 0   ? run<2, 132>(keys, nullptr, 0, arena, rows, out, bad, iters)
               : v == 1 ? run<2, 160>(keys, nullptr, 0, arena, rows, out, bad, iters)
                        : run<3, 160>(keys, nullptr, 0, arena, rows, out, bad, iters);
    int nb = 0;
    CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
    printf("{\"variant\":\"%s\",\"us\":%.1f,\"frac_1048B\":%.4f,\"home_collisions_seen\":%d}\n",
           v == 0 ? "colocated528" : (v == 1 ? "coloc640" : "tail640"), c * 1e3, bytes_sep / (c * 1e-3) / 8e12, nb);
    CK(hipFree(arena));
  }
  return 0;
}
