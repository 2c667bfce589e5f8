// fused.hip -- FusedEmbeddingLocalSparseLookUp[Grad] and the owner partition /
// row exchange helpers of the row-sharded all-to-all.
#include <climits>

#include "dr_common.h"

extern "C" int dr_bag_offsets_strided(const int64_t* seg, int64_t stride, int64_t n, int64_t batch,
                                      int32_t* bag_off, void* stream);

namespace dr {

// values_offset[b] = first nnz of row b (INT_MAX when empty), the
// SetToIntMaxSTG128 + CalcPerElementRowInBatchValuesOffset result
// (fused_embedding_local_ops_gpu.cu.cc:18-39).
__global__ void values_offset_kernel(const int32_t* __restrict__ off, int64_t B,
                                     int32_t* __restrict__ vo) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  vo[b] = off[b + 1] > off[b] ? off[b] : INT_MAX;
}

// DoEmbeddingGrad (fused_embedding_local_ops_gpu.cu.cc:86-122): one wave per bag.
__global__ void fused_grad_kernel(const float* __restrict__ top, const float* __restrict__ table,
                                  int64_t rows, int D, const int64_t* __restrict__ values,
                                  const int32_t* __restrict__ vo, int64_t nnz, int64_t B,
                                  int combiner, float max_norm, float* __restrict__ gout,
                                  int* st) {
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  const int64_t off = vo[b];
  const int64_t cnt = (b == B - 1 ? nnz : (int64_t)vo[b + 1]) - off;
  for (int64_t k = 0; k < cnt; ++k) {
    const int64_t v = values[off + k];
    const bool ok = v >= 0 && v < rows;
    if (!ok && lane == 0) latch(st, DR_INVALID_ARGUMENT);
    float f = 1.f;
    bool clip = false;
    if (max_norm > 0.f && ok) {
      float s = 0.f;
      for (int d = lane; d < D; d += 64) {
        const float e = table[v * D + d];
        s += e * e;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      const float l2 = sqrtf(s);
      if (l2 > max_norm) {
        clip = true;
        f = max_norm / l2;
      }
    }
    for (int d = lane; d < D; d += 64) {
      float g = top[b * D + d];
      if (combiner == DR_COMBINER_SQRTN)
        g = g / sqrtf((float)cnt);
      else if (combiner == DR_COMBINER_MEAN)
        g = g / (float)cnt;
      if (clip) g = g * f;
      gout[(off + k) * D + d] = g;
    }
  }
}

// owner = key mod world (non-negative), sentinel bucket `world` past n_eff.
// premod > 0: owner = floormod(floormod(key, premod), world) (EV partitions).
__global__ void owner_keys_kernel(const int64_t* __restrict__ keys, int64_t n, const int64_t* n_dev,
                                  int world, int64_t premod, uint64_t* __restrict__ okey,
                                  int32_t* __restrict__ pos, unsigned long long* __restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t ne = eff_n(n, n_dev);
  int64_t o = world;
  if (i < ne) {
    int64_t k = keys[i];
    if (premod > 0) {
      k %= premod;
      if (k < 0) k += premod;
    }
    o = k % world;
    if (o < 0) o += world;
    atomicAdd(&counts[o], 1ull);
  }
  okey[i] = (uint64_t)o;
  pos[i] = (int32_t)i;
}

__global__ void permute_keys_kernel(const int64_t* __restrict__ keys, const int32_t* __restrict__ perm,
                                    int64_t n, const int64_t* n_dev, int64_t* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= eff_n(n, n_dev)) return;
  out[j] = keys[perm[j]];
}

// rows: one wave per row, dwordx4 when dim % 4 == 0.
template <bool SCATTER>
__global__ void rows_move_kernel(const float* __restrict__ src, const int32_t* __restrict__ perm,
                                 int64_t n, const int64_t* n_dev, int dim,
                                 float* __restrict__ dst) {
  const int64_t j = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (j >= eff_n(n, n_dev)) return;
  const int lane = threadIdx.x & 63;
  const int64_t p = perm[j];
  const float* s = SCATTER ? src + j * dim : src + p * dim;
  float* d = SCATTER ? dst + p * dim : dst + j * dim;
  if ((dim & 3) == 0) {
    for (int c = lane; c < dim / 4; c += 64)
      reinterpret_cast<float4*>(d)[c] = reinterpret_cast<const float4*>(s)[c];
  } else {
    for (int c = lane; c < dim; c += 64) d[c] = s[c];
  }
}

struct RouteGroup {
  int64_t koff[DR_MAX_GROUP + 1];
};

// sort key = owner * T + feature for valid uniques, world * T otherwise.
// num_unique == nullptr: every key of a feature is valid (raw ids, no dedup).
// The [world*T] histogram is built in LDS per block (one global atomic per
// bin per block instead of one per key onto ~200 hot addresses).
constexpr int kRouteLdsBins = 4096;
__global__ __launch_bounds__(256) void route_keys_kernel(RouteGroup g, int T,
                                                         const int64_t* __restrict__ uniq,
                                                         const int64_t* __restrict__ num_unique,
                                                         int world, uint64_t* __restrict__ skey,
                                                         int32_t* __restrict__ pos,
                                                         unsigned long long* __restrict__ counts) {
  __shared__ unsigned int hist[kRouteLdsBins];
  const int bins = world * T;
  const bool lds = bins <= kRouteLdsBins;
  if (lds)
    for (int b = threadIdx.x; b < bins; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < g.koff[T]) {
    const int t = table_of(g.koff, T, i, (int64_t)blockIdx.x * blockDim.x);
    uint64_t k = (uint64_t)bins;
    if (!num_unique || i - g.koff[t] < num_unique[t]) {
      int64_t o = uniq[i] % world;
      if (o < 0) o += world;
      k = (uint64_t)o * T + t;
      if (lds)
        atomicAdd(&hist[k], 1u);
      else
        atomicAdd(&counts[k], 1ull);
    }
    skey[i] = k;
    pos[i] = (int32_t)i;
  }
  if (!lds) return;
  __syncthreads();
  for (int b = threadIdx.x; b < bins; b += blockDim.x)
    if (hist[b]) atomicAdd(&counts[b], (unsigned long long)hist[b]);
}

__global__ void route_emit_kernel(const int64_t* __restrict__ uniq, const uint64_t* __restrict__ skey,
                                  const int32_t* __restrict__ perm, int64_t n, int T, int world,
                                  int64_t* __restrict__ keys_out, int32_t* __restrict__ tags_out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t k = skey[j];
  if (k >= (uint64_t)world * T) return;
  keys_out[j] = uniq[perm[j]];
  tags_out[j] = (int32_t)(k % (uint64_t)T);
}

}  // namespace dr

extern "C" {

size_t dr_route_workspace_size(int64_t n, int world, int num_tables) {
  (void)world;
  (void)num_tables;
  dr::Carver c(nullptr);
  c.take<uint64_t>(n > 0 ? n : 1);
  c.take<int32_t>(n > 0 ? n : 1);
  c.take<uint64_t>(n > 0 ? n : 1);
  c.take<char>(dr_sort_pairs_workspace_size(n));
  return c.used + 256;
}

int dr_route_by_owner(const int64_t* uniq, const int64_t* koff_host, int num_tables,
                      const int64_t* num_unique, int world, int64_t* keys_out, int32_t* tags_out,
                      int32_t* perm_out, int64_t* counts, void* ws, size_t ws_bytes,
                      void* stream) {
  using namespace dr;
  const int T = num_tables;
  DR_REQUIRE(T >= 1 && T <= DR_MAX_GROUP && world >= 1 && world <= 1024, DR_INVALID_ARGUMENT,
             "dr_route_by_owner: bad T/world");
  const int64_t n = koff_host[T];
  DR_REQUIRE(ws_bytes >= dr_route_workspace_size(n, world, T), DR_INVALID_ARGUMENT,
             "workspace too small");
  hipStream_t st = S(stream);
  int frc = fill_bytes(counts, 0, (size_t)world * T * sizeof(int64_t), st);
  if (frc) return frc;
  if (n == 0) return DR_OK;
  RouteGroup g;
  for (int t = 0; t <= T; ++t) g.koff[t] = koff_host[t];
  Carver c(ws);
  uint64_t* skey = c.take<uint64_t>(n);
  int32_t* pos = c.take<int32_t>(n);
  uint64_t* skey2 = c.take<uint64_t>(n);
  const size_t sb = dr_sort_pairs_workspace_size(n);
  void* sws = c.take<char>(sb);
  const unsigned blocks = (unsigned)ceil_div(n, 256);
  hipLaunchKernelGGL(route_keys_kernel, dim3(blocks), dim3(256), 0, st, g, T, uniq, num_unique,
                     world, skey, pos, (unsigned long long*)counts);
  DR_LAUNCH_CHECK();
  int bits = 0;
  while (((int64_t)1 << bits) <= (int64_t)world * T) ++bits;
  int rc = dr_sort_pairs(skey, pos, skey2, perm_out, n, 0, bits, sws, sb, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(route_emit_kernel, dim3(blocks), dim3(256), 0, st, uniq, skey2, perm_out, n,
                     T, world, keys_out, tags_out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

size_t dr_fused_local_workspace_size(int64_t batch) {
  return (size_t)(batch + 2) * sizeof(int32_t) + 256;
}

int dr_fused_local_lookup(const float* table, int64_t rows, int dim, const int64_t* sp_values,
                          const int64_t* sp_indices, int64_t nnz, int64_t batch, int combiner,
                          float max_norm, float* out, int32_t* values_offset, void* ws,
                          size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(ws_bytes >= dr_fused_local_workspace_size(batch), DR_INVALID_ARGUMENT,
             "workspace too small");
  if (batch == 0) return DR_OK;
  int32_t* off = static_cast<int32_t*>(ws);
  int rc = dr_bag_offsets_strided(sp_indices, 2, nnz, batch, off, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(values_offset_kernel, dim3((unsigned)ceil_div(batch, 256)), dim3(256), 0,
                     S(stream), off, batch, values_offset);
  DR_LAUNCH_CHECK();
  dr_pool_desc d;
  memset(&d, 0, sizeof(d));
  d.pool = table;
  d.pool_rows = rows;
  d.ids = sp_values;
  d.bag_off = off;
  d.out = out;
  d.out_stride = dim;
  d.combiner = combiner;
  d.max_norm = max_norm;  // enabled iff >= 0, fused-kernel semantics
  return dr_pool_grouped(&d, 1, batch, dim, DR_ORDER_SEQ, stream);
}

int dr_fused_local_lookup_grad(const float* top_grad, const float* table, int64_t rows, int dim,
                               const int64_t* sp_values, const int32_t* values_offset,
                               int64_t nnz, int64_t batch, int combiner, float max_norm,
                               float* grad_out, void* stream) {
  using namespace dr;
  if (batch == 0 || nnz == 0) return DR_OK;
  hipLaunchKernelGGL(fused_grad_kernel, dim3((unsigned)ceil_div(batch, 4)), dim3(256), 0,
                     S(stream), top_grad, table, rows, dim, sp_values, values_offset, nnz, batch,
                     combiner, max_norm, grad_out, status_word());
  DR_LAUNCH_CHECK();
  return DR_OK;
}

size_t dr_partition_workspace_size(int64_t n) {
  dr::Carver c(nullptr);
  c.take<uint64_t>(n > 0 ? n : 1);
  c.take<int32_t>(n > 0 ? n : 1);
  c.take<uint64_t>(n > 0 ? n : 1);
  c.take<char>(dr_sort_pairs_workspace_size(n));
  return c.used + 256;
}

int dr_partition_by_owner(const int64_t* keys, int64_t n, const int64_t* n_dev, int world,
                          int64_t* keys_out, int32_t* perm_out, int64_t* send_counts, void* ws,
                          size_t ws_bytes, void* stream) {
  return dr_partition_by_owner_mod(keys, n, n_dev, world, 0, keys_out, perm_out, send_counts, ws,
                                   ws_bytes, stream);
}

int dr_partition_by_owner_mod(const int64_t* keys, int64_t n, const int64_t* n_dev, int world,
                              int64_t premod, int64_t* keys_out, int32_t* perm_out,
                              int64_t* send_counts, void* ws, size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(world >= 1 && world <= 4096, DR_INVALID_ARGUMENT, "bad world size");
  DR_REQUIRE(ws_bytes >= dr_partition_workspace_size(n), DR_INVALID_ARGUMENT,
             "workspace too small");
  hipStream_t st = S(stream);
  int frc = fill_bytes(send_counts, 0, world * sizeof(int64_t), st);
  if (frc) return frc;
  if (n == 0) return DR_OK;
  Carver c(ws);
  uint64_t* okey = c.take<uint64_t>(n);
  int32_t* pos = c.take<int32_t>(n);
  uint64_t* okey2 = c.take<uint64_t>(n);
  const size_t sb = dr_sort_pairs_workspace_size(n);
  void* sws = c.take<char>(sb);
  const unsigned blocks = (unsigned)ceil_div(n, 256);
  hipLaunchKernelGGL(owner_keys_kernel, dim3(blocks), dim3(256), 0, st, keys, n, n_dev, world,
                     premod, okey, pos, (unsigned long long*)send_counts);
  DR_LAUNCH_CHECK();
  int bits = 0;
  while ((1 << bits) <= world) ++bits;
  int rc = dr_sort_pairs(okey, pos, okey2, perm_out, n, 0, bits, sws, sb, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(permute_keys_kernel, dim3(blocks), dim3(256), 0, st, keys, perm_out, n, n_dev,
                     keys_out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_rows_scatter(const float* src, const int32_t* perm, int64_t n, const int64_t* n_dev,
                    int dim, float* dst, void* stream) {
  using namespace dr;
  if (n == 0) return DR_OK;
  hipLaunchKernelGGL(rows_move_kernel<true>, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0,
                     S(stream), src, perm, n, n_dev, dim, dst);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_rows_pack(const float* src, const int32_t* perm, int64_t n, const int64_t* n_dev, int dim,
                 float* dst, void* stream) {
  using namespace dr;
  if (n == 0) return DR_OK;
  hipLaunchKernelGGL(rows_move_kernel<false>, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0,
                     S(stream), src, perm, n, n_dev, dim, dst);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // extern "C"
