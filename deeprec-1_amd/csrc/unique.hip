// unique.hip -- Unique / UniqueWithCounts in first-occurrence order, for one
// table or for all T tables of a step in one pass (grouped).
//
// Replaces UniqueAliOp (core/kernels/unique_ali_op.cc:46-180); the order
// contract is SerialComputeV1 (unique_ali_op_util.h:192-222): y lists keys
// in order of first appearance, idx[i] = position of x[i] in y.
//
// GPU algorithm (no host sync, integer-exact):
//   1. open-addressing table per feature (capacity pow2 >= 2 n_t) in the
//      workspace whose 4-byte slots hold a POSITION, not a key: a slot is
//      claimed by CAS-ing its first inserter's position in, and a probe
//      matches when keys[slot value] == k (the input is immutable, so the
//      position identifies the key).  A later, smaller position of the same
//      key lowers the slot with atomicMin -- only when it is smaller, which
//      the roughly ascending launch order makes rare -- so the slot ends
//      at the key's FIRST position with one returning atomic per key
//      instead of a key CAS plus a position atomicMin (memory-side atomics
//      are the insert's bound: one 64-B request per lane);
//   2. flag[i] = (slot == i); one exclusive scan over all features;
//      the local unique id is prefix[i] - prefix[first position of table t]
//      (a table's first position is always a first occurrence);
//   3. idx[i] = prefix[slot value] - prefix[table start] in the same pass
//      that writes the unique keys; counts by integer atomics (order-free,
//      exact).
// Every key value (-1 included) is an ordinary key: the empty pattern is a
// position (0xFFFFFFFF), never a key.
// Outputs keep the input layout: table t's uniques / counts sit at
// [koff[t], koff[t] + U_t) and U_t goes to num_unique[t] (device int64).
#include "dr_common.h"

namespace dr {

static constexpr uint32_t kEmptyPos = ~0u;

struct UniqGroup {
  int64_t koff[DR_MAX_GROUP + 1];   // input offsets
  int64_t hbase[DR_MAX_GROUP];      // hash region base (slots)
  int64_t hcap[DR_MAX_GROUP];       // region capacity (pow2)
};

struct UniqueWs {
  uint32_t* minpos;  // [hash_total] first position of the slot's key
  int32_t* slot_of;  // [n]
  int32_t* flags;    // [n] scan output
  int64_t* total;    // [1]
  void* scan_ws;
};

static int64_t build_group(const int64_t* koff, int T, UniqGroup* g) {
  int64_t base = 0;
  for (int t = 0; t < T; ++t) {
    const int64_t n = koff[t + 1] - koff[t];
    g->koff[t] = koff[t];
    g->hbase[t] = base;
    g->hcap[t] = next_pow2(2 * (n > 32 ? n : 32));
    base += g->hcap[t];
  }
  g->koff[T] = koff[T];
  return base;
}

static UniqueWs carve_unique(void* ws, int64_t n, int64_t hash_total, size_t* used) {
  Carver c(ws);
  UniqueWs u;
  u.minpos = c.take<uint32_t>(hash_total);
  u.slot_of = c.take<int32_t>(n > 0 ? n : 1);
  u.flags = c.take<int32_t>(n > 0 ? n : 1);
  u.total = c.take<int64_t>(1);
  u.scan_ws = c.take<char>(scan_ws_bytes(n));
  if (used) *used = c.used + 256;
  return u;
}

// (all callers index elements as blockIdx.x * blockDim.x + threadIdx.x)
__device__ __forceinline__ int group_table(const UniqGroup& g, int T, int64_t i) {
  return table_of(g.koff, T, i, (int64_t)blockIdx.x * blockDim.x);
}

__global__ void unique_insert_kernel(UniqGroup g, int T, const int64_t* __restrict__ keys,
                                     uint32_t* __restrict__ minpos,
                                     int32_t* __restrict__ slot_of) {
  __shared__ int64_t shcap[DR_MAX_GROUP], shbase[DR_MAX_GROUP];  // per-lane table: LDS
  if (threadIdx.x < T) {
    shcap[threadIdx.x] = g.hcap[threadIdx.x];
    shbase[threadIdx.x] = g.hbase[threadIdx.x];
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.koff[T]) return;  // (exited lanes are the wave's tail: never a run head)
  const int t = group_table(g, T, i);
  const int64_t k = keys[i];
  // Runs of one key in consecutive positions of a wave (a padded history
  // batch, a hot id) insert once: only the run's first lane -- the smallest
  // position -- touches the slot; the rest take its slot by a shuffle.
  const int lane = __lane_id();
  const uint32_t klo = (uint32_t)k, khi = (uint32_t)((uint64_t)k >> 32);
  const uint32_t plo = (uint32_t)__shfl_up((int)klo, 1, 64);
  const uint32_t phi = (uint32_t)__shfl_up((int)khi, 1, 64);
  const int pt = __shfl_up(t, 1, 64);
  const bool head = lane == 0 || plo != klo || phi != khi || pt != t;
  const uint64_t heads = __ballot(head);
  int64_t s = 0;
  if (head) {
    const int64_t cap = shcap[t];
    uint32_t* mp = minpos + shbase[t];
    const uint64_t mask = (uint64_t)cap - 1;
    uint64_t h = mix64((uint64_t)k) & mask;
    const uint32_t me = (uint32_t)i;
    // The CAS result (performed at the memory side) is the only truth used
    // to skip a slot; the table holds at most half its capacity.
    for (int64_t probes = 0; probes <= cap; ++probes) {
      const uint32_t old = atomicCAS(&mp[h], kEmptyPos, me);
      if (old == kEmptyPos) break;
      if (keys[old] == k) {
        if (me < old) atomicMin(&mp[h], me);
        break;
      }
      h = (h + 1) & mask;
    }
    s = (int64_t)h + shbase[t];
  }
  const uint64_t le = heads & (lanemask_lt() | (1ull << lane));
  const int src = 63 - __clzll((long long)le);
  s = (int64_t)(uint32_t)__shfl((int)(uint32_t)s, src, 64);
  slot_of[i] = (int32_t)s;
}

__global__ void unique_flag_kernel(int64_t n, const uint32_t* __restrict__ minpos,
                                   const int32_t* __restrict__ slot_of,
                                   int32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flags[i] = minpos[slot_of[i]] == (uint32_t)i ? 1 : 0;
}

// After the scan flags[] holds exclusive prefix sums.  One pass writes idx
// (the uid of the key's first position, read through the slot) and, at first
// positions, the unique key; no per-slot uid table is written or gathered.
__global__ void unique_emit_kernel(UniqGroup g, int T, const int64_t* __restrict__ keys,
                                   const uint32_t* __restrict__ minpos,
                                   const int32_t* __restrict__ slot_of,
                                   const int32_t* __restrict__ prefix, int64_t* __restrict__ uniq,
                                   int32_t* __restrict__ idx, int32_t* __restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.koff[T]) return;
  const int t = group_table(g, T, i);
  const int64_t kt = g.koff[t];
  const uint32_t m = minpos[slot_of[i]];
  const int32_t u = prefix[m] - prefix[kt];
  idx[i] = u;
  if (m == (uint32_t)i) uniq[kt + u] = keys[i];
  if (counts) atomicAdd(&counts[kt + u], 1);
}

__global__ void unique_counts_kernel(UniqGroup g, int T, const int32_t* __restrict__ prefix,
                                     const int64_t* __restrict__ total,
                                     int64_t* __restrict__ num_unique) {
  const int t = threadIdx.x;
  if (t >= T) return;
  const int64_t n = g.koff[T];
  const int64_t a = g.koff[t] < n ? prefix[g.koff[t]] : *total;
  const int64_t b = g.koff[t + 1] < n ? prefix[g.koff[t + 1]] : *total;
  num_unique[t] = g.koff[t + 1] > g.koff[t] ? b - a : 0;
}

}  // namespace dr

extern "C" size_t dr_unique_grouped_workspace_size(const int64_t* koff_host, int num_tables) {
  if (num_tables < 1 || num_tables > DR_MAX_GROUP) return 0;
  dr::UniqGroup g;
  const int64_t ht = dr::build_group(koff_host, num_tables, &g);
  size_t used = 0;
  dr::carve_unique(nullptr, koff_host[num_tables], ht, &used);
  return used;
}

extern "C" int dr_unique_grouped(const int64_t* keys, const int64_t* koff_host, int num_tables,
                                 int64_t* uniq_out, int32_t* idx_out, int32_t* counts_out,
                                 int64_t* num_unique, void* ws, size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(num_tables >= 1 && num_tables <= DR_MAX_GROUP, DR_INVALID_ARGUMENT,
             "dr_unique_grouped: 1..%d tables", DR_MAX_GROUP);
  const int T = num_tables;
  const int64_t n = koff_host[T];
  DR_REQUIRE(n >= 0 && n < (int64_t)0x7fffffff, DR_INVALID_ARGUMENT, "dr_unique: bad n");
  for (int t = 0; t < T; ++t)
    DR_REQUIRE(koff_host[t + 1] >= koff_host[t], DR_INVALID_ARGUMENT, "koff must be sorted");
  DR_REQUIRE(ws_bytes >= dr_unique_grouped_workspace_size(koff_host, T), DR_INVALID_ARGUMENT,
             "dr_unique: workspace too small");
  hipStream_t st = S(stream);
  if (n == 0) {
    return fill_bytes(num_unique, 0, T * sizeof(int64_t), st);
  }
  UniqGroup g;
  const int64_t ht = build_group(koff_host, T, &g);
  UniqueWs u = carve_unique(ws, n, ht, nullptr);
  int frc = fill_bytes(u.minpos, 0xFF, ht * sizeof(uint32_t), st);
  if (!frc && counts_out) frc = fill_bytes(counts_out, 0, n * sizeof(int32_t), st);
  if (frc) return frc;
  const unsigned blocks = (unsigned)ceil_div(n, 256);
  hipLaunchKernelGGL(unique_insert_kernel, dim3(blocks), dim3(256), 0, st, g, T, keys, u.minpos,
                     u.slot_of);
  hipLaunchKernelGGL(unique_flag_kernel, dim3(blocks), dim3(256), 0, st, n, u.minpos, u.slot_of,
                     u.flags);
  DR_LAUNCH_CHECK();
  int rc = scan_exclusive_i32(u.flags, u.flags, n, nullptr, u.total, u.scan_ws, st);
  if (rc) return rc;
  hipLaunchKernelGGL(unique_emit_kernel, dim3(blocks), dim3(256), 0, st, g, T, keys, u.minpos,
                     u.slot_of, u.flags, uniq_out, idx_out, counts_out);
  hipLaunchKernelGGL(unique_counts_kernel, dim3(1), dim3(64), 0, st, g, T, u.flags, u.total,
                     num_unique);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

extern "C" size_t dr_unique_workspace_size(int64_t n) {
  const int64_t koff[2] = {0, n > 0 ? n : 0};
  return dr_unique_grouped_workspace_size(koff, 1);
}

extern "C" int dr_unique(const int64_t* keys, int64_t n, int64_t* uniq_out, int32_t* idx_out,
                         int32_t* counts_out, int64_t* num_unique, void* ws, size_t ws_bytes,
                         void* stream) {
  const int64_t koff[2] = {0, n};
  return dr_unique_grouped(keys, koff, 1, uniq_out, idx_out, counts_out, num_unique, ws, ws_bytes,
                           stream);
}
