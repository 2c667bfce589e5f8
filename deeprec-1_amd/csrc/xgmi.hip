// xgmi.hip -- requester side of the peer-mapped sharded lookup, and the HIP
// IPC helpers that map the peers' buffers once.
//
// The reference (SOK, all2all_input_dispatcher.cu:74,256-268) buckets keys by
// owner = key % world, exchanges counts, and copies keys through NCCL send /
// recv buffers.  Here the requester writes every (key, slot) pair straight
// into the owner's inbox over xGMI: no send buffer, no host read of counts.
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

__global__ __launch_bounds__(256) void xgmi_route_kernel(XgmiArgs a, const int64_t* __restrict__ keys,
                                                         int T, int64_t B,
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
      int64_t o = keys[(int64_t)t * B + b] % a.world;
      if (o < 0) o += a.world;
      owner = (int)o;
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

}  // namespace dr

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

int dr_xgmi_route(const dr_xgmi_peers* peers, const int64_t* keys, int num_tables,
                  int64_t batch, int64_t* cnt_ws, void* stream) {
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
                       0, st, a, keys, num_tables, batch, (unsigned long long*)cnt_ws);
  }
  hipLaunchKernelGGL(xgmi_counts_kernel, dim3(64), dim3(64), 0, st, a,
                     (const unsigned long long*)cnt_ws);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // extern "C"
