// unique.hip -- Unique / UniqueWithCounts in first-occurrence order.
//
// Replaces UniqueAliOp (core/kernels/unique_ali_op.cc:46-180); the order
// contract is SerialComputeV1 (unique_ali_op_util.h:192-222): y lists keys
// in order of first appearance, idx[i] = position of x[i] in y.
//
// GPU algorithm (no host sync, integer-exact):
//   1. open-addressing table (capacity pow2 >= 2n) in the workspace; each
//      position i CAS-inserts its key and atomicMin's its position into the
//      slot -> slot holds the FIRST position of that key;
//   2. flag[i] = (slot.minpos == i); exclusive scan of flags gives the
//      unique id of every first occurrence (= first-occurrence order);
//   3. idx[i] = uid(slot(i)); counts by integer atomics (order-free, exact).
// Key -1 is the table's empty pattern; it is routed to a dedicated slot.
#include "dr_common.h"

namespace dr {

static constexpr uint64_t kEmpty = ~0ull;

struct UniqueWs {
  uint64_t* tkeys;   // [cap]
  uint32_t* minpos;  // [cap + 1]
  int32_t* tuid;     // [cap + 1]
  int32_t* slot_of;  // [n]
  int32_t* flags;    // [n] scan output
  void* scan_ws;
  int64_t cap;
};

static UniqueWs carve_unique(void* ws, int64_t n, size_t* used = nullptr) {
  Carver c(ws);
  UniqueWs u;
  u.cap = next_pow2(2 * (n > 32 ? n : 32));
  u.tkeys = c.take<uint64_t>(u.cap);
  u.minpos = c.take<uint32_t>(u.cap + 1);
  u.tuid = c.take<int32_t>(u.cap + 1);
  u.slot_of = c.take<int32_t>(n > 0 ? n : 1);
  u.flags = c.take<int32_t>(n > 0 ? n : 1);
  u.scan_ws = c.take<char>(scan_ws_bytes(n));
  if (used) *used = c.used;
  return u;
}

__global__ void unique_insert_kernel(const int64_t* __restrict__ keys, int64_t n,
                                     uint64_t* __restrict__ tkeys, uint32_t* __restrict__ minpos,
                                     int32_t* __restrict__ slot_of, int64_t cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = (uint64_t)keys[i];
  int64_t s;
  if (k == kEmpty) {
    s = cap;
  } else {
    const uint64_t mask = (uint64_t)cap - 1;
    uint64_t h = mix64(k) & mask;
    for (;;) {
      uint64_t cur = tkeys[h];
      if (cur == k) break;
      if (cur == kEmpty) {
        uint64_t old = atomicCAS((unsigned long long*)&tkeys[h], (unsigned long long)kEmpty,
                                 (unsigned long long)k);
        if (old == kEmpty || old == k) break;
      }
      h = (h + 1) & mask;
    }
    s = (int64_t)h;
  }
  atomicMin(&minpos[s], (uint32_t)i);
  slot_of[i] = (int32_t)s;
}

__global__ void unique_flag_kernel(int64_t n, const uint32_t* __restrict__ minpos,
                                   const int32_t* __restrict__ slot_of,
                                   int32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flags[i] = minpos[slot_of[i]] == (uint32_t)i ? 1 : 0;
}

// After the scan flags[] holds exclusive prefix sums.
__global__ void unique_emit_kernel(const int64_t* __restrict__ keys, int64_t n,
                                   const uint32_t* __restrict__ minpos,
                                   const int32_t* __restrict__ slot_of,
                                   const int32_t* __restrict__ prefix, int64_t* __restrict__ uniq,
                                   int32_t* __restrict__ tuid) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t s = slot_of[i];
  if (minpos[s] == (uint32_t)i) {
    const int32_t u = prefix[i];
    uniq[u] = keys[i];
    tuid[s] = u;
  }
}

__global__ void unique_expand_kernel(int64_t n, const int32_t* __restrict__ slot_of,
                                     const int32_t* __restrict__ tuid, int32_t* __restrict__ idx,
                                     int32_t* __restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t u = tuid[slot_of[i]];
  idx[i] = u;
  if (counts) atomicAdd(&counts[u], 1);
}

}  // namespace dr

extern "C" size_t dr_unique_workspace_size(int64_t n) {
  size_t used = 0;
  dr::carve_unique(nullptr, n, &used);
  return used + 256;
}

extern "C" int dr_unique(const int64_t* keys, int64_t n, int64_t* uniq_out, int32_t* idx_out,
                         int32_t* counts_out, int64_t* num_unique, void* ws, size_t ws_bytes,
                         void* stream) {
  using namespace dr;
  DR_REQUIRE(n >= 0 && n < (int64_t)0x7fffffff, DR_INVALID_ARGUMENT, "dr_unique: bad n");
  DR_REQUIRE(ws_bytes >= dr_unique_workspace_size(n), DR_INVALID_ARGUMENT,
             "dr_unique: workspace too small");
  hipStream_t st = S(stream);
  if (n == 0) {
    DR_HIP(hipMemsetAsync(num_unique, 0, sizeof(int64_t), st));
    return DR_OK;
  }
  UniqueWs u = carve_unique(ws, n);
  DR_HIP(hipMemsetAsync(u.tkeys, 0xFF, u.cap * sizeof(uint64_t), st));
  DR_HIP(hipMemsetAsync(u.minpos, 0xFF, (u.cap + 1) * sizeof(uint32_t), st));
  if (counts_out) DR_HIP(hipMemsetAsync(counts_out, 0, n * sizeof(int32_t), st));
  const unsigned blocks = (unsigned)ceil_div(n, 256);
  hipLaunchKernelGGL(unique_insert_kernel, dim3(blocks), dim3(256), 0, st, keys, n, u.tkeys,
                     u.minpos, u.slot_of, u.cap);
  hipLaunchKernelGGL(unique_flag_kernel, dim3(blocks), dim3(256), 0, st, n, u.minpos, u.slot_of,
                     u.flags);
  DR_LAUNCH_CHECK();
  int rc = scan_exclusive_i32(u.flags, u.flags, n, nullptr, num_unique, u.scan_ws, st);
  if (rc) return rc;
  hipLaunchKernelGGL(unique_emit_kernel, dim3(blocks), dim3(256), 0, st, keys, n, u.minpos,
                     u.slot_of, u.flags, uniq_out, u.tuid);
  hipLaunchKernelGGL(unique_expand_kernel, dim3(blocks), dim3(256), 0, st, n, u.slot_of, u.tuid,
                     idx_out, counts_out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}
