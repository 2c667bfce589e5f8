// xgmi.hip -- requester side of the peer-mapped sharded lookup, and the HIP
// IPC helpers that map the peers' buffers once.
//
// The reference (SOK, all2all_input_dispatcher.cu:74,256-268) buckets keys by
// owner = key % world, exchanges counts, and copies keys through NCCL send /
// recv buffers.  Here the requester writes every (key, slot) pair straight
// into the owner's inbox over xGMI: no send buffer, no host read of counts.
#include <map>
#include <stdio.h>
#include <vector>
#include <mutex>
#include <stdlib.h>

#include "dr_common.h"

namespace dr {

struct XgmiArgs {
  int32_t world, rank;
  int64_t cap;
  int64_t* inbox_keys[DR_MAX_PEERS];
  int32_t* inbox_slot[DR_MAX_PEERS];
  int64_t* inbox_cnt[DR_MAX_PEERS];
};

// Ids are visited in OUTPUT (slot) order, slot j = b*T + t, so each owner's
// inbox region is near-sorted by slot and the owner's row writes stream
// through the requester's [B, T*D] output.  A block takes RT_ITEMS x 256
// consecutive slots: wave-ballot-aggregated LDS atomics give each id its
// offset within (block, owner); one global atomic per (block, owner) places
// the block's run in the owner's region.
constexpr int RT_ITEMS = 8;

// n_dev (nullable, DEVICE [T]): only ids b < n_dev[t] of table t are routed
// -- the deduplicating requester routes each table's first-occurrence unique
// keys (u = b < U_t) and expands the rows it gets back locally.
__global__ __launch_bounds__(256) void xgmi_route_kernel(XgmiArgs a, const int64_t* __restrict__ keys,
                                                         int T, int64_t B,
                                                         const int64_t* __restrict__ n_dev,
                                                         unsigned long long* __restrict__ cnt) {
  __shared__ unsigned int lcnt[DR_MAX_PEERS];
  __shared__ unsigned long long lbase[DR_MAX_PEERS];
  if (threadIdx.x < DR_MAX_PEERS) lcnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t n = (int64_t)T * B;
  const int64_t j0 = (int64_t)blockIdx.x * 256 * RT_ITEMS + threadIdx.x;
  const int lane = lane_id();
  int own[RT_ITEMS];
  unsigned int off[RT_ITEMS];
#pragma unroll
  for (int it = 0; it < RT_ITEMS; ++it) {
    const int64_t j = j0 + (int64_t)it * 256;
    int owner = -1;
    if (j < n) {
      const int64_t b = j / T;
      const int t = (int)(j - b * T);
      if (!n_dev || b < n_dev[t]) {
        int64_t o = keys[(int64_t)t * B + b] % a.world;
        if (o < 0) o += a.world;
        owner = (int)o;
      }
    }
    own[it] = owner;
    off[it] = 0;
    for (int o = 0; o < a.world; ++o) {
      const uint64_t m = __ballot(owner == o);
      if (!m) continue;
      const int leader = __ffsll((unsigned long long)m) - 1;
      unsigned int base = 0;
      if (lane == leader) base = atomicAdd(&lcnt[o], (unsigned int)__popcll(m));
      base = __shfl(base, leader, 64);
      if (owner == o) off[it] = base + (unsigned int)__popcll(m & lanemask_lt());
    }
  }
  __syncthreads();
  if (threadIdx.x < a.world)
    lbase[threadIdx.x] = lcnt[threadIdx.x]
                             ? atomicAdd(&cnt[threadIdx.x], (unsigned long long)lcnt[threadIdx.x])
                             : 0ull;
  __syncthreads();
#pragma unroll
  for (int it = 0; it < RT_ITEMS; ++it) {
    const int o = own[it];
    if (o < 0) continue;
    const int64_t j = j0 + (int64_t)it * 256;
    const int64_t b = j / T;
    const int t = (int)(j - b * T);
    const int64_t at = (int64_t)a.rank * a.cap + (int64_t)lbase[o] + off[it];
    __builtin_nontemporal_store(keys[(int64_t)t * B + b], a.inbox_keys[o] + at);
    __builtin_nontemporal_store((int32_t)j, a.inbox_slot[o] + at);
  }
  // no per-block system fence (one per block cost more than the kernel):
  // xgmi_counts_kernel flushes every XCD's L2 right after this launch
}

// Runs after the route kernel: every block issues a system-scope release
// (L2 write-back of the XCD it runs on; 64 blocks cover the 8 XCDs), and
// block 0 publishes this rank's per-owner counts.
__global__ void xgmi_counts_kernel(XgmiArgs a, const unsigned long long* __restrict__ cnt) {
  __threadfence_system();
  const int p = threadIdx.x;
  if (blockIdx.x == 0 && p < a.world) {
    __hip_atomic_store(a.inbox_cnt[p] + a.rank, (int64_t)cnt[p], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __threadfence_system();
}


// ---- backward (owner side): pull the requesters' gradient rows ---------------
// The inbox entries of source s (positions [0, cnt[s]) of region s) are
// compacted to e = prefix[s] + i, sorted by (table, source, slot) -- slot is
// unique per source, so the order is canonical whatever order the route
// kernel's atomics placed them in -- and each sorted entry copies its key and
// the requester's gradient row gin[s][slot] (read over xGMI) into the output.
struct XgmiPullArgs {
  int32_t world;
  int64_t cap;
  int64_t prefix[DR_MAX_PEERS + 1];
  const float* gin[DR_MAX_PEERS];
};

__device__ __forceinline__ int pull_source(const XgmiPullArgs& a, int64_t e) {
  int s = 0;
  while (s + 1 < a.world && e >= a.prefix[s + 1]) ++s;
  return s;
}

__global__ void xgmi_grad_keys_kernel(XgmiPullArgs a, const int32_t* __restrict__ inbox_slot,
                                      int T, int64_t TB, int64_t R, uint64_t* __restrict__ kin,
                                      int32_t* __restrict__ vin) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= R) return;
  const int s = pull_source(a, e);
  const int64_t slot = inbox_slot[(int64_t)s * a.cap + (e - a.prefix[s])];
  const int64_t t = slot % T;
  kin[e] = (uint64_t)(t * a.world + s) * (uint64_t)TB + (uint64_t)slot;
  vin[e] = (int32_t)e;
}

// one 64-lane wave per sorted entry, 4 per block
__global__ __launch_bounds__(256) void xgmi_grad_pull_kernel(
    XgmiPullArgs a, const int64_t* __restrict__ inbox_keys, const int32_t* __restrict__ inbox_slot,
    const int32_t* __restrict__ perm, int64_t R, int dim, int64_t row_stride,
    int64_t* __restrict__ keys_out, float* __restrict__ grads_out) {
  const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= R) return;
  const int lane = threadIdx.x & 63;
  const int64_t e = perm[p];
  const int s = pull_source(a, e);
  const int64_t at = (int64_t)s * a.cap + (e - a.prefix[s]);
  const int64_t slot = inbox_slot[at];
  if (lane == 0) keys_out[p] = inbox_keys[at];
  // slot j = b*T + t of the requester's [B, T*dim] gradient: row b, column t*dim
  const int64_t T = row_stride / dim;
  const int64_t b = slot / T, t = slot - b * T;
  const float* g = a.gin[s] + b * row_stride + t * dim;
  float* o = grads_out + p * (int64_t)dim;
  if ((dim & 3) == 0) {
    const float4* g4 = reinterpret_cast<const float4*>(g);
    float4* o4 = reinterpret_cast<float4*>(o);
    for (int c = lane; c < dim / 4; c += 64) o4[c] = g4[c];
  } else {
    for (int c = lane; c < dim; c += 64) o[c] = g[c];
  }
}

// table_start[t] = first sorted position of table t (lower bound), t <= T
__global__ void xgmi_table_start_kernel(const uint64_t* __restrict__ kout, int64_t R, int T,
                                        int world, int64_t TB, int64_t* __restrict__ tstart) {
  const int t = threadIdx.x;
  if (t > T) return;
  const uint64_t lo_key = (uint64_t)t * (uint64_t)world * (uint64_t)TB;
  int64_t lo = 0, hi = R;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (kout[mid] < lo_key)
      lo = mid + 1;
    else
      hi = mid;
  }
  tstart[t] = lo;
}

// ---- the same pull with device-side counts (no host read) -------------------
// prefix[s] = entries of sources < s in this rank's inbox (clamped to cap);
// prefix[W] = R, the device element count of the sort and the pull.
__global__ void xgmi_pull_prefix_kernel(const int64_t* __restrict__ inbox_cnt, int world,
                                        int64_t cap, int64_t* __restrict__ prefix, int* st) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t acc = 0;
  prefix[0] = 0;
  for (int s = 0; s < world; ++s) {
    int64_t c = inbox_cnt[s];
    if (c < 0 || c > cap) {
      latch(st, DR_INTERNAL);
      c = c < 0 ? 0 : cap;
    }
    acc += c;
    prefix[s + 1] = acc;
  }
}

__device__ __forceinline__ int pull_source_dev(const int64_t* prefix, int world, int64_t e) {
  int s = 0;
  while (s + 1 < world && e >= prefix[s + 1]) ++s;
  return s;
}

__global__ void xgmi_grad_keys_dev_kernel(const int64_t* __restrict__ prefix, int world,
                                          int64_t cap, const int32_t* __restrict__ inbox_slot,
                                          int T, int64_t TB, uint64_t* __restrict__ kin,
                                          int32_t* __restrict__ vin) {
  const int64_t R = prefix[world];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < R;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int s = pull_source_dev(prefix, world, e);
    const int64_t slot = inbox_slot[(int64_t)s * cap + (e - prefix[s])];
    const int64_t t = slot % T;
    kin[e] = (uint64_t)(t * world + s) * (uint64_t)TB + (uint64_t)slot;
    vin[e] = (int32_t)e;
  }
}

// tstart[t] = first sorted position of table t; counts[t] = its entry count
__global__ void xgmi_table_start_dev_kernel(const uint64_t* __restrict__ kout,
                                            const int64_t* __restrict__ prefix, int T, int world,
                                            int64_t TB, int64_t* __restrict__ tstart,
                                            int64_t* __restrict__ counts) {
  __shared__ int64_t ts[1025];
  const int64_t R = prefix[world];
  for (int t = threadIdx.x; t <= T; t += blockDim.x) {
    const uint64_t lo_key = (uint64_t)t * (uint64_t)world * (uint64_t)TB;
    int64_t lo = 0, hi = R;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (kout[mid] < lo_key)
        lo = mid + 1;
      else
        hi = mid;
    }
    ts[t] = lo;
    tstart[t] = lo;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += blockDim.x) counts[t] = ts[t + 1] - ts[t];
}

// one 64-lane wave per sorted entry (grid-stride over the device count):
// table t's entries land at t * tcap + (p - tstart[t]), tcap = world * batch
// (every requester sends at most `batch` ids of a table)
__global__ __launch_bounds__(256) void xgmi_grad_pull_dev_kernel(
    const int64_t* __restrict__ prefix, int world, int64_t cap, XgmiPullArgs a, const int64_t* __restrict__ inbox_keys,
    const int32_t* __restrict__ inbox_slot, const uint64_t* __restrict__ kout,
    const int32_t* __restrict__ perm, const int64_t* __restrict__ tstart, int64_t TB,
    int64_t tcap, int dim, int64_t row_stride, int64_t* __restrict__ keys_out,
    float* __restrict__ grads_out) {
  const int64_t R = prefix[world];
  const int lane = threadIdx.x & 63;
  const int64_t T = row_stride / dim;
  for (int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); p < R;
       p += (int64_t)gridDim.x * 4) {
    const int64_t e = perm[p];
    const int s = pull_source_dev(prefix, world, e);
    const int64_t at = (int64_t)s * cap + (e - prefix[s]);
    const int64_t slot = inbox_slot[at];
    const int64_t tt = (int64_t)(kout[p] / ((uint64_t)world * (uint64_t)TB));
    const int64_t q = tt * tcap + (p - tstart[tt]);
    if (lane == 0) keys_out[q] = inbox_keys[at];
    // slot j = b*T + t of the requester's [B, T*dim] gradient: row b, column t*dim
    const int64_t b = slot / T, t = slot - b * T;
    const float* g = a.gin[s] + b * row_stride + t * dim;
    float* o = grads_out + q * (int64_t)dim;
    if ((dim & 3) == 0) {
      const float4* g4 = reinterpret_cast<const float4*>(g);
      float4* o4 = reinterpret_cast<float4*>(o);
      for (int c = lane; c < dim / 4; c += 64) o4[c] = g4[c];
    } else {
      for (int c = lane; c < dim; c += 64) o[c] = g[c];
    }
  }
}

}  // namespace dr

namespace {
struct UcFree {
  std::mutex mu;
  std::multimap<std::pair<int, size_t>, void*> free;  // (device, bytes) -> ptr
  std::map<void*, std::pair<int, size_t>> size_of;
};
UcFree& uc_pool() {
  static UcFree* p = new UcFree();  // never destroyed (process lifetime)
  return *p;
}
}  // namespace

extern "C" {

int dr_ipc_export(const void* ptr, void* handle_out, int64_t* offset_out) {
  DR_REQUIRE(ptr && handle_out && offset_out, DR_INVALID_ARGUMENT, "null argument");
  static_assert(sizeof(hipIpcMemHandle_t) <= DR_IPC_HANDLE_BYTES, "IPC handle size");
  hipIpcMemHandle_t h;
  DR_HIP(hipIpcGetMemHandle(&h, const_cast<void*>(ptr)));
  void* base = nullptr;
  size_t size = 0;
  DR_HIP(hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr)));
  memset(handle_out, 0, DR_IPC_HANDLE_BYTES);
  memcpy(handle_out, &h, sizeof(h));
  *offset_out = (int64_t)((const char*)ptr - (const char*)base);
  return DR_OK;
}

int dr_ipc_import(const void* handle, int64_t offset, void** ptr_out, void** base_out) {
  DR_REQUIRE(handle && ptr_out && base_out && offset >= 0, DR_INVALID_ARGUMENT,
             "bad argument");
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  void* base = nullptr;
  DR_HIP(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess));
  *base_out = base;
  *ptr_out = (char*)base + offset;
  return DR_OK;
}

int dr_ipc_close(void* base) {
  DR_REQUIRE(base, DR_INVALID_ARGUMENT, "null base");
  DR_HIP(hipIpcCloseMemHandle(base));
  return DR_OK;
}

// Buffers that other GPUs write over xGMI (inboxes, outputs) or read
// (gradients): uncached device memory, so no XCD L2 of the owning GPU can
// hold a line a peer has since rewritten -- per-XCD L2s are not coherent
// with writes arriving from another agent (MI355X_MICROARCH.md "Correctness
// boundaries"; the DMA-memset staleness of DESIGN.md section 6 is the same
// effect).  Zero-filled, synchronously (allocation time only).
//
// Uncached buffers are never handed back to the HIP allocator: measured on
// MI355X / ROCm 7.2, a coarse-grained hipMalloc that reuses memory freed
// from a hipDeviceMallocUncached allocation of the same process returned
// corrupted rows (tests/test_gpu_sharded.py::test_xgmi_serve_grows_small_
// tables after the peer-write tests).  Freed buffers go
// to a per-device free list keyed by size and are reused by the next
// allocation of that size.

int dr_ipc_alloc(size_t bytes, void** ptr_out) {
  using namespace dr;
  DR_REQUIRE(ptr_out, DR_INVALID_ARGUMENT, "null ptr_out");
  const size_t n = bytes > 0 ? (bytes + 255) & ~size_t(255) : 256;
  int dev = 0;
  DR_HIP(hipGetDevice(&dev));
  void* p = nullptr;
  {
    UcFree& u = uc_pool();
    std::lock_guard<std::mutex> g(u.mu);
    auto it = u.free.find({dev, n});
    if (it != u.free.end()) {
      p = it->second;
      u.free.erase(it);
    }
  }
  if (p) {
    // Reuse is ordered after every stream's work issued before the free:
    // dr_ipc_free runs from a DLPack deleter as soon as the framework drops
    // the tensor, while kernels on its (non-blocking) streams may still read
    // or write the buffer.  A device-wide sync here (allocation time only)
    // covers all of them.  Peer GPUs' writes are the caller's contract: every
    // peer closes its IPC mapping (after a barrier) before the owner frees.
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
      UcFree& u = uc_pool();
      std::lock_guard<std::mutex> g(u.mu);
      u.free.insert({{dev, n}, p});
      set_error("dr_ipc_alloc: %s", hipGetErrorString(e));
      return DR_INTERNAL;
    }
  } else {
    DR_HIP(hipExtMallocWithFlags(&p, n, hipDeviceMallocUncached));
    UcFree& u = uc_pool();
    std::lock_guard<std::mutex> g(u.mu);
    u.size_of[p] = {dev, n};
  }
  int rc = fill_bytes(p, 0, n, nullptr);
  if (rc == DR_OK) {
    hipError_t e = hipStreamSynchronize(nullptr);
    if (e != hipSuccess) {
      set_error("dr_ipc_alloc: %s", hipGetErrorString(e));
      rc = DR_INTERNAL;
    }
  }
  if (rc) {
    (void)dr_ipc_free(p);
    return rc;
  }
  *ptr_out = p;
  return DR_OK;
}

#ifdef DR_UC_DIAG
}  // extern "C" (the diagnostics have C++ linkage)
namespace dr {
// Diagnostic (DR_IPC_RELEASE=3/4 below): a system-scope fence from blocks on
// every XCD -- an L2 write-back and invalidate of each XCD's L2.
__global__ void uc_l2_flush_kernel() { __threadfence_system(); }

// Ranges of uncached blocks handed back to hipFree, and a check of a small
// buffer a later allocation wrote by DMA: the bytes as a D2H copy reads them
// and as a kernel reads them (plain loads, stored to pinned host memory).
static std::mutex g_diag_mu;
static std::vector<std::pair<uintptr_t, size_t>> g_freed;

void uc_diag_freed(void* p, size_t n) {
  std::lock_guard<std::mutex> g(g_diag_mu);
  g_freed.push_back({(uintptr_t)p, n});
  fprintf(stderr, "[uc-diag] hipFree uncached [%p, +%zu)\n", p, n);
}

__global__ void uc_diag_read_kernel(const uint32_t* __restrict__ src, int64_t n,
                                    uint32_t* __restrict__ dst) {
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}

void uc_diag_check(const char* what, const void* dev, const void* expect, size_t bytes) {
  const size_t nw = bytes / 4;
  if (nw == 0) return;
  std::vector<uint32_t> dma(nw);
  uint32_t* kh = nullptr;
  if (hipHostMalloc(&kh, nw * 4) != hipSuccess) return;
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(dma.data(), dev, nw * 4, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL(uc_diag_read_kernel, dim3(1), dim3(256), 0, nullptr,
                     static_cast<const uint32_t*>(dev), (int64_t)nw, kh);
  (void)hipDeviceSynchronize();
  const uint32_t* ex = static_cast<const uint32_t*>(expect);
  size_t bad_dma = 0, bad_k = 0;
  for (size_t i = 0; i < nw; ++i) {
    bad_dma += dma[i] != ex[i];
    bad_k += kh[i] != ex[i];
  }
  bool recycled = false;
  {
    std::lock_guard<std::mutex> g(g_diag_mu);
    for (auto& r : g_freed)
      if ((uintptr_t)dev < r.first + r.second && (uintptr_t)dev + bytes > r.first) recycled = true;
  }
  fprintf(stderr,
          "[uc-diag] %s %p +%zu: on a freed uncached range %d, D2H mismatches %zu, "
          "kernel-read mismatches %zu (word 0: expect %08x D2H %08x kernel %08x)\n",
          what, dev, bytes, (int)recycled, bad_dma, bad_k, ex[0], dma[0], kh[0]);
  (void)hipHostFree(kh);
}

// An acquire at system scope on every XCD: invalidates each XCD's L2 lines of
// memory that is not local-coherent (and the vector L1s).
__global__ void uc_inv_kernel() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }
// L2 write-back of every XCD at agent scope (buffer_wbl2 sc1, what a
// kernel-end release does for coarse-grained memory) or system scope
// (buffer_wbl2 sc0 sc1 + buffer_inv sc0 sc1).
__global__ void uc_wb_agent_kernel() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent"); }

void uc_diag_writeback(int system) {
  if (system)
    hipLaunchKernelGGL(uc_l2_flush_kernel, dim3(2048), dim3(64), 0, nullptr);
  else
    hipLaunchKernelGGL(uc_wb_agent_kernel, dim3(2048), dim3(64), 0, nullptr);
  (void)hipDeviceSynchronize();
}

// The same read from 64 blocks spread over the XCDs: block b records its XCD
// (HW_REG_XCC_ID) and how many words differ from `expect` -- a stale
// translation of a recycled VA would show on some XCDs only.
__global__ void uc_diag_xcd_kernel(const uint32_t* __restrict__ src, int64_t n,
                                   uint32_t expect_fill, const uint32_t* __restrict__ expect,
                                   uint32_t* __restrict__ res) {
  __shared__ uint32_t bad, zeros;
  if (threadIdx.x == 0) {
    bad = 0;
    zeros = 0;
  }
  __syncthreads();
  uint32_t b = 0, z = 0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t v = __builtin_nontemporal_load(src + i);
    const uint32_t e = expect ? expect[i] : expect_fill;
    b += v != e;
    z += v == 0;
  }
  atomicAdd(&bad, b);
  atomicAdd(&zeros, z);
  __syncthreads();
  if (threadIdx.x == 0) {
    res[3 * blockIdx.x] = (uint32_t)__builtin_amdgcn_s_getreg(0x1814);   // XCC_ID[3:0]
    res[3 * blockIdx.x + 1] = bad;
    res[3 * blockIdx.x + 2] = zeros;
  }
}

bool uc_diag_check_xcd(const char* what, const void* dev, uint32_t fill, size_t bytes) {
  const size_t nw = bytes / 4;
  if (nw == 0) return false;
  uint32_t* res = nullptr;
  if (hipHostMalloc(&res, 64 * 3 * 4) != hipSuccess) return false;
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(uc_diag_xcd_kernel, dim3(64), dim3(256), 0, nullptr,
                     static_cast<const uint32_t*>(dev), (int64_t)nw, fill, nullptr, res);
  (void)hipDeviceSynchronize();
  // the bytes as DMA reads them (no GPU L2 on the path), and the per-block
  // view again after an L2 invalidate on every XCD
  size_t dz = 0, dbad = 0;
  {
    std::vector<uint32_t> h(nw);
    (void)hipMemcpy(h.data(), dev, nw * 4, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < nw; ++i) {
      dz += h[i] == 0;
      dbad += h[i] != fill;
    }
  }
  uint32_t* res2 = nullptr;
  if (hipHostMalloc(&res2, 64 * 3 * 4) != hipSuccess) return false;
  hipLaunchKernelGGL(uc_inv_kernel, dim3(2048), dim3(64), 0, nullptr);
  hipLaunchKernelGGL(uc_diag_xcd_kernel, dim3(64), dim3(256), 0, nullptr,
                     static_cast<const uint32_t*>(dev), (int64_t)nw, fill, nullptr, res2);
  (void)hipDeviceSynchronize();
  bool recycled = false;
  {
    std::lock_guard<std::mutex> g(g_diag_mu);
    for (auto& r : g_freed)
      if ((uintptr_t)dev < r.first + r.second && (uintptr_t)dev + bytes > r.first) recycled = true;
  }
  uint32_t badx[16] = {0}, zx[16] = {0}, seen[16] = {0};
  for (int b = 0; b < 64; ++b) {
    const uint32_t x = res[3 * b] & 15;
    seen[x] = 1;
    badx[x] += res[3 * b + 1];
    zx[x] += res[3 * b + 2];
  }
  char line[1024];
  int o = snprintf(line, sizeof(line), "[uc-diag] %s %p +%zu: recycled-uncached %d, per XCD "
                   "bad/zero words:", what, dev, bytes, (int)recycled);
  for (int x = 0; x < 16 && o < (int)sizeof(line) - 24; ++x)
    if (seen[x]) o += snprintf(line + o, sizeof(line) - o, " %d:%u/%u", x, badx[x], zx[x]);
  if (o < (int)sizeof(line) - 64)
    o += snprintf(line + o, sizeof(line) - o, "; D2H bad/zero %zu/%zu; blocks 0-7 zero", dbad, dz);
  for (int b = 0; b < 8 && o < (int)sizeof(line) - 24; ++b)
    o += snprintf(line + o, sizeof(line) - o, " x%u:%u", res[3 * b] & 15, res[3 * b + 2]);
  if (o < (int)sizeof(line) - 40)
    o += snprintf(line + o, sizeof(line) - o, "; after L2 inv blocks 0-7 zero");
  for (int b = 0; b < 8 && o < (int)sizeof(line) - 24; ++b)
    o += snprintf(line + o, sizeof(line) - o, " x%u:%u", res2[3 * b] & 15, res2[3 * b + 2]);
  fprintf(stderr, "%s\n", line);
  (void)hipHostFree(res);
  (void)hipHostFree(res2);
  return dbad != 0;
}
}  // namespace dr
extern "C" {
#endif

// Returns the buffer to the uncached free list (never to hipFree, see
// above).  Cheap and safe to call from a DLPack deleter: the next
// dr_ipc_alloc that reuses it synchronises the device first.
int dr_ipc_free(void* ptr) {
  using namespace dr;
  if (!ptr) return DR_OK;
  UcFree& u = uc_pool();
  std::lock_guard<std::mutex> g(u.mu);
  auto it = u.size_of.find(ptr);
  DR_REQUIRE(it != u.size_of.end(), DR_INVALID_ARGUMENT,
             "dr_ipc_free: %p was not allocated by dr_ipc_alloc", ptr);
#ifdef DR_UC_DIAG
  // Diagnostic build only (make ab AB_FLAGS=-DDR_UC_DIAG; tools/gpu_uc_reuse.sh):
  // DR_IPC_RELEASE=1 hands the block back to hipFree at once (the round-2
  // behaviour), =2 after a device-wide synchronisation, =3 / 4 with the L2
  // flush kernel after (and before) the free.  The product library has no
  // such switch: freed uncached blocks only ever go to the free list.
  static const int release = [] {
    const char* e = getenv("DR_IPC_RELEASE");
    return e ? atoi(e) : 0;
  }();
  if (release >= 1 && release <= 4) {
    // 3: L2 flushed on every XCD after the free, 4: before and after
    uc_diag_freed(ptr, it->second.second);
    u.size_of.erase(it);
    if (release >= 2) DR_HIP(hipDeviceSynchronize());
    if (release == 4) {
      hipLaunchKernelGGL(uc_l2_flush_kernel, dim3(512), dim3(64), 0, nullptr);
      DR_HIP(hipDeviceSynchronize());
    }
    DR_HIP(hipFree(ptr));
    if (release >= 3) {
      hipLaunchKernelGGL(uc_l2_flush_kernel, dim3(512), dim3(64), 0, nullptr);
      DR_HIP(hipDeviceSynchronize());
    }
    return DR_OK;
  }
#endif
  u.free.insert({it->second, ptr});
  return DR_OK;
}

// DLPack (v0.8 DLManagedTensor) view of a dr_ipc_alloc buffer, so a framework
// can own it as a tensor (torch.utils.dlpack.from_dlpack); the deleter is C,
// independent of the interpreter's lifetime.
namespace {
struct DlDevice {
  int32_t device_type, device_id;
};
struct DlDataType {
  uint8_t code, bits;
  uint16_t lanes;
};
struct DlTensor {
  void* data;
  DlDevice device;
  int32_t ndim;
  DlDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DlManaged {
  DlTensor t;
  void* ctx;
  void (*deleter)(DlManaged*);
  int64_t shape[8];
};
void dl_delete(DlManaged* m) {
  if (!m) return;
  (void)dr_ipc_free(m->t.data);
  free(m);
}
void dl_delete_view(DlManaged* m) { free(m); }   // a view: the memory is not ours
}  // namespace

int dr_dlpack_view(void* data, int ndim, const int64_t* shape, int dtype_code, int dtype_bits,
                   int device_id, void** managed_out) {
  using namespace dr;
  DR_REQUIRE(data && ndim >= 1 && ndim <= 8 && shape && managed_out && dtype_bits % 8 == 0 &&
                 dtype_bits > 0,
             DR_INVALID_ARGUMENT, "dr_dlpack_view: bad argument");
  DlManaged* m = static_cast<DlManaged*>(calloc(1, sizeof(DlManaged)));
  DR_REQUIRE(m, DR_RESOURCE_EXHAUSTED, "dr_dlpack_view: out of host memory");
  for (int i = 0; i < ndim; ++i) m->shape[i] = shape[i];
  m->t.data = data;
  m->t.device.device_type = 10;  // kDLROCM
  m->t.device.device_id = device_id;
  m->t.ndim = ndim;
  m->t.dtype.code = (uint8_t)dtype_code;
  m->t.dtype.bits = (uint8_t)dtype_bits;
  m->t.dtype.lanes = 1;
  m->t.shape = m->shape;
  m->t.strides = nullptr;
  m->t.byte_offset = 0;
  m->deleter = dl_delete_view;
  *managed_out = m;
  return DR_OK;
}

int dr_ipc_alloc_dlpack(int ndim, const int64_t* shape, int dtype_code, int dtype_bits,
                        int device_id, void** managed_out) {
  using namespace dr;
  DR_REQUIRE(ndim >= 1 && ndim <= 8 && shape && managed_out && dtype_bits % 8 == 0 &&
                 dtype_bits > 0,
             DR_INVALID_ARGUMENT, "dr_ipc_alloc_dlpack: bad shape / dtype");
  size_t n = (size_t)(dtype_bits / 8);
  for (int i = 0; i < ndim; ++i) {
    DR_REQUIRE(shape[i] >= 0, DR_INVALID_ARGUMENT, "negative dim");
    n *= (size_t)shape[i];
  }
  int cur = 0;
  DR_HIP(hipGetDevice(&cur));
  DR_REQUIRE(cur == device_id, DR_INVALID_ARGUMENT, "device %d is not current (%d)", device_id,
             cur);
  void* p = nullptr;
  int rc = dr_ipc_alloc(n, &p);
  if (rc) return rc;
  DlManaged* m = static_cast<DlManaged*>(calloc(1, sizeof(DlManaged)));
  if (!m) {
    (void)dr_ipc_free(p);  // uncached blocks never go back to hipFree
    set_error("dr_ipc_alloc_dlpack: out of host memory");
    return DR_RESOURCE_EXHAUSTED;
  }
  for (int i = 0; i < ndim; ++i) m->shape[i] = shape[i];
  m->t.data = p;
  m->t.device.device_type = 10;  // kDLROCM
  m->t.device.device_id = device_id;
  m->t.ndim = ndim;
  m->t.dtype.code = (uint8_t)dtype_code;
  m->t.dtype.bits = (uint8_t)dtype_bits;
  m->t.dtype.lanes = 1;
  m->t.shape = m->shape;
  m->t.strides = nullptr;  // compact row-major
  m->t.byte_offset = 0;
  m->ctx = nullptr;
  m->deleter = dl_delete;
  *managed_out = m;
  return DR_OK;
}

int dr_xgmi_route_ex(const dr_xgmi_peers* peers, const int64_t* keys, int num_tables,
                     int64_t batch, const int64_t* n_dev, int64_t* cnt_ws, void* stream) {
  using namespace dr;
  DR_REQUIRE(peers && cnt_ws && num_tables >= 1 && batch >= 0, DR_INVALID_ARGUMENT,
             "bad argument");
  const int W = peers->world;
  DR_REQUIRE(W >= 1 && W <= DR_MAX_PEERS && peers->rank >= 0 && peers->rank < W,
             DR_INVALID_ARGUMENT, "bad world/rank");
  const int64_t n = (int64_t)num_tables * batch;
  DR_REQUIRE(n <= peers->cap && n < (1ll << 31), DR_INVALID_ARGUMENT,
             "T*B = %lld exceeds the inbox capacity %lld", (long long)n, (long long)peers->cap);
  XgmiArgs a;
  memset(&a, 0, sizeof(a));
  a.world = W;
  a.rank = peers->rank;
  a.cap = peers->cap;
  for (int p = 0; p < W; ++p) {
    DR_REQUIRE(peers->inbox_keys[p] && peers->inbox_slot[p] && peers->inbox_cnt[p],
               DR_INVALID_ARGUMENT, "peer %d not mapped", p);
    a.inbox_keys[p] = peers->inbox_keys[p];
    a.inbox_slot[p] = peers->inbox_slot[p];
    a.inbox_cnt[p] = peers->inbox_cnt[p];
  }
  hipStream_t st = S(stream);
  int rc = fill_bytes(cnt_ws, 0, (size_t)W * sizeof(int64_t), st);
  if (rc) return rc;
  if (n > 0) {
    DR_REQUIRE(keys, DR_INVALID_ARGUMENT, "null keys");
    hipLaunchKernelGGL(xgmi_route_kernel, dim3((unsigned)ceil_div(n, 256 * RT_ITEMS)), dim3(256),
                       0, st, a, keys, num_tables, batch, n_dev, (unsigned long long*)cnt_ws);
  }
  hipLaunchKernelGGL(xgmi_counts_kernel, dim3(64), dim3(64), 0, st, a,
                     (const unsigned long long*)cnt_ws);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_xgmi_route(const dr_xgmi_peers* peers, const int64_t* keys, int num_tables,
                  int64_t batch, int64_t* cnt_ws, void* stream) {
  return dr_xgmi_route_ex(peers, keys, num_tables, batch, nullptr, cnt_ws, stream);
}


size_t dr_xgmi_grad_pull_workspace_size(int world, int64_t cap) {
  using namespace dr;
  const int64_t n = (int64_t)(world > 0 ? world : 1) * (cap > 0 ? cap : 1);
  Carver c(nullptr);
  c.take<uint64_t>(n);
  c.take<int32_t>(n);
  c.take<uint64_t>(n);
  c.take<int32_t>(n);
  c.take<char>(dr_sort_pairs_workspace_size(n));
  return c.used + 256;
}

int dr_xgmi_grad_pull(const dr_xgmi_peers* peers, const float* const* grad_in,
                      const int64_t* cnt_host, int num_tables, int64_t batch, int dim,
                      int64_t* keys_out, float* grads_out, int64_t* table_start, void* ws,
                      size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(peers && grad_in && cnt_host && table_start && num_tables >= 1 && batch >= 0 &&
                 dim > 0,
             DR_INVALID_ARGUMENT, "bad argument");
  const int W = peers->world;
  DR_REQUIRE(W >= 1 && W <= DR_MAX_PEERS && peers->rank >= 0 && peers->rank < W,
             DR_INVALID_ARGUMENT, "bad world/rank");
  DR_REQUIRE(num_tables < 1024, DR_INVALID_ARGUMENT, "too many tables");
  DR_REQUIRE(ws_bytes >= dr_xgmi_grad_pull_workspace_size(W, peers->cap), DR_INVALID_ARGUMENT,
             "workspace too small");
  const int64_t TB = (int64_t)num_tables * batch;
  XgmiPullArgs a;
  memset(&a, 0, sizeof(a));
  a.world = W;
  a.cap = peers->cap;
  a.prefix[0] = 0;
  for (int s = 0; s < W; ++s) {
    DR_REQUIRE(cnt_host[s] >= 0 && cnt_host[s] <= peers->cap, DR_INVALID_ARGUMENT,
               "inbox count %lld of source %d out of range", (long long)cnt_host[s], s);
    DR_REQUIRE(grad_in[s], DR_INVALID_ARGUMENT, "peer %d gradient buffer not mapped", s);
    a.prefix[s + 1] = a.prefix[s] + cnt_host[s];
    a.gin[s] = grad_in[s];
  }
  const int64_t R = a.prefix[W];
  DR_REQUIRE(R < (1ll << 31), DR_INVALID_ARGUMENT, "too many entries");
  hipStream_t st = S(stream);
  const int me = peers->rank;
  const int64_t* ikeys = peers->inbox_keys[me];
  const int32_t* islot = peers->inbox_slot[me];
  DR_REQUIRE(ikeys && islot, DR_INVALID_ARGUMENT, "own inbox not mapped");
  Carver c(ws);
  const int64_t n = (int64_t)W * (peers->cap > 0 ? peers->cap : 1);
  uint64_t* kin = c.take<uint64_t>(n);
  int32_t* vin = c.take<int32_t>(n);
  uint64_t* kout = c.take<uint64_t>(n);
  int32_t* perm = c.take<int32_t>(n);
  const size_t sb = dr_sort_pairs_workspace_size(n);
  void* sws = c.take<char>(sb);
  if (R > 0) {
    hipLaunchKernelGGL(xgmi_grad_keys_kernel, dim3((unsigned)ceil_div(R, 256)), dim3(256), 0, st,
                       a, islot, num_tables, TB, R, kin, vin);
    DR_LAUNCH_CHECK();
    int bits = 1;
    while (bits < 64 && ((uint64_t)num_tables * (uint64_t)W * (uint64_t)TB) >> bits) ++bits;
    int rc = dr_sort_pairs(kin, vin, kout, perm, R, 0, bits, sws, sb, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(xgmi_grad_pull_kernel, dim3((unsigned)ceil_div(R, 4)), dim3(256), 0, st, a,
                       ikeys, islot, perm, R, dim, (int64_t)num_tables * dim, keys_out,
                       grads_out);
    DR_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(xgmi_table_start_kernel, dim3(1), dim3(1024), 0, st, kout, R, num_tables, W,
                     TB, table_start);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

size_t dr_xgmi_grad_pull_dev_workspace_size(int world, int64_t cap) {
  using namespace dr;
  const int64_t n = (int64_t)(world > 0 ? world : 1) * (cap > 0 ? cap : 1);
  Carver c(nullptr);
  c.take<int64_t>(DR_MAX_PEERS + 1);
  c.take<int64_t>(1025);
  c.take<uint64_t>(n);
  c.take<int32_t>(n);
  c.take<uint64_t>(n);
  c.take<int32_t>(n);
  c.take<char>(dr_sort_pairs_workspace_size(n));
  return c.used + 256;
}

int dr_xgmi_grad_pull_dev(const dr_xgmi_peers* peers, const float* const* grad_in,
                          int num_tables, int64_t batch, int dim, int64_t* keys_out,
                          float* grads_out, int64_t* counts_out, void* ws, size_t ws_bytes,
                          void* stream) {
  using namespace dr;
  DR_REQUIRE(peers && grad_in && keys_out && grads_out && counts_out && num_tables >= 1 &&
                 batch >= 0 && dim > 0,
             DR_INVALID_ARGUMENT, "bad argument");
  const int W = peers->world;
  DR_REQUIRE(W >= 1 && W <= DR_MAX_PEERS && peers->rank >= 0 && peers->rank < W,
             DR_INVALID_ARGUMENT, "bad world/rank");
  DR_REQUIRE(num_tables < 1024, DR_INVALID_ARGUMENT, "too many tables");
  DR_REQUIRE(ws_bytes >= dr_xgmi_grad_pull_dev_workspace_size(W, peers->cap),
             DR_INVALID_ARGUMENT, "workspace too small");
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  const int64_t TB = (int64_t)num_tables * batch;
  XgmiPullArgs a;
  memset(&a, 0, sizeof(a));
  a.world = W;
  a.cap = peers->cap;
  for (int q = 0; q < W; ++q) {
    DR_REQUIRE(grad_in[q], DR_INVALID_ARGUMENT, "peer %d gradient buffer not mapped", q);
    a.gin[q] = grad_in[q];
  }
  hipStream_t s = S(stream);
  const int me = peers->rank;
  const int64_t* ikeys = peers->inbox_keys[me];
  const int32_t* islot = peers->inbox_slot[me];
  const int64_t* icnt = peers->inbox_cnt[me];
  DR_REQUIRE(ikeys && islot && icnt, DR_INVALID_ARGUMENT, "own inbox not mapped");
  const int64_t n = (int64_t)W * (peers->cap > 0 ? peers->cap : 1);
  DR_REQUIRE(n < (1ll << 31), DR_INVALID_ARGUMENT, "inbox too large");
  Carver c(ws);
  int64_t* prefix = c.take<int64_t>(DR_MAX_PEERS + 1);
  int64_t* tstart = c.take<int64_t>(1025);
  uint64_t* kin = c.take<uint64_t>(n);
  int32_t* vin = c.take<int32_t>(n);
  uint64_t* kout = c.take<uint64_t>(n);
  int32_t* perm = c.take<int32_t>(n);
  void* sws = c.take<char>(dr_sort_pairs_workspace_size(n));
  hipLaunchKernelGGL(xgmi_pull_prefix_kernel, dim3(1), dim3(64), 0, s, icnt, W, peers->cap,
                     prefix, st);
  const unsigned kb = (unsigned)std::min<int64_t>(ceil_div(n, 256), 4096);
  hipLaunchKernelGGL(xgmi_grad_keys_dev_kernel, dim3(kb), dim3(256), 0, s, prefix, W, peers->cap,
                     islot, num_tables, TB, kin, vin);
  DR_LAUNCH_CHECK();
  int bits = 1;
  while (bits < 64 && ((uint64_t)num_tables * (uint64_t)W * (uint64_t)TB) >> bits) ++bits;
  int rc = sort_pairs_u64_dev(kin, vin, kout, perm, n, prefix + W, bits, sws, s);
  if (rc) return rc;
  hipLaunchKernelGGL(xgmi_table_start_dev_kernel, dim3(1), dim3(1024), 0, s, kout, prefix,
                     num_tables, W, TB, tstart, counts_out);
  const unsigned pb = (unsigned)std::min<int64_t>(ceil_div(n, 4), 16384);
  hipLaunchKernelGGL(xgmi_grad_pull_dev_kernel, dim3(pb), dim3(256), 0, s, prefix, W, peers->cap,
                     a, ikeys, islot, kout, perm, tstart, TB, (int64_t)W * batch, dim,
                     (int64_t)num_tables * dim, keys_out, grads_out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // extern "C"
