// partitioned.hip -- the partitioned fused lookup of python/ops/fused_embedding_ops.py:45-67:
// FusedEmbeddingSparsePreLookUp -> per-partition Gather -> FusedEmbeddingSparsePostLookUp
// (+ PostLookUpGrad), core/kernels/fused_embedding/fused_embedding_ops_gpus.cu.cc:150-519.
//
// PreLookUp: one stable LSD radix sort of (id, position) pairs over the
// bits of the id range (the reference sorts all 64 bits of (id, (row, col)));
// one emit pass rebases each id to its partition and copies its (row, col)
// pair; partition boundaries are lower bounds in the sorted ids.
//
// PostLookUp: the reference scatters every entry into its bag with float
// atomics (SumUpEmbeddingShard), so its sums have no fixed order.  Here the
// entries of all partitions are sorted by (row, col) -- the SparseTensor's
// canonical order -- and each bag is summed from 0 in that order by one lane
// group, rows clipped on the fly: deterministic, and bit-identical to
// FusedEmbeddingLocalSparseLookUp (fused_embedding_local_ops_gpu.cu.cc:41-84)
// on the same ids.  Row reads are the HBM-bound part: nnz * dim * 4 B.
#include "dr_common.h"
#include "dr_rows.h"

namespace dr {

struct PartAcc {
  int64_t acc[DR_MAX_PARTITIONS];  // prefix sums of partition rows
};

// key = id for ids in range, `total` (sorted last, left out) otherwise
__global__ void pre_keys_kernel(const int64_t* __restrict__ vals, int64_t n, int64_t total,
                                uint64_t* __restrict__ key, int32_t* __restrict__ pos, int* st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t v = vals[i];
  if (v < 0 || v >= total) {
    latch(st, DR_INVALID_ARGUMENT);
    v = total;
  }
  key[i] = (uint64_t)v;
  pos[i] = (int32_t)i;
}

__device__ __forceinline__ int partition_of(const PartAcc& a, int P, int64_t v) {
  int lo = 0, hi = P - 1;  // first p with v < acc[p]
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (v < a.acc[mid])
      hi = mid;
    else
      lo = mid + 1;
  }
  return lo;
}

__global__ void pre_emit_kernel(PartAcc a, int P, const uint64_t* __restrict__ skey,
                                const int32_t* __restrict__ perm,
                                const int64_t* __restrict__ ind, int64_t n, int64_t total,
                                int64_t* __restrict__ vout, int64_t* __restrict__ iout) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int64_t v = (int64_t)skey[j];
  if (v >= total) return;  // out of range: not in any partition
  const int p = partition_of(a, P, v);
  vout[j] = v - (p == 0 ? 0 : a.acc[p - 1]);
  const int64_t s = perm[j];
  iout[2 * j] = ind[2 * s];
  iout[2 * j + 1] = ind[2 * s + 1];
}

// part_off[p] = first sorted position with id >= acc[p - 1] (part_off[0] = 0)
__global__ void pre_offsets_kernel(PartAcc a, int P, const uint64_t* __restrict__ skey, int64_t n,
                                   int64_t* __restrict__ part_off) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p > P) return;
  if (p == 0) {
    part_off[0] = 0;
    return;
  }
  const uint64_t target = (uint64_t)a.acc[p - 1];
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (skey[mid] < target)
      lo = mid + 1;
    else
      hi = mid;
  }
  part_off[p] = lo;
}

struct PostGroup {
  const float* shard[DR_MAX_PARTITIONS];
  const int64_t* ind[DR_MAX_PARTITIONS];
  int64_t koff[DR_MAX_PARTITIONS + 1];
};

// entry e (partitions back to back) -> key row * cols + col
__global__ void post_keys_kernel(PostGroup g, int P, int64_t B, int64_t cols,
                                 uint64_t* __restrict__ key, int32_t* __restrict__ pos, int* st) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= g.koff[P]) return;
  const int p = table_of(g.koff, P, e, (int64_t)blockIdx.x * blockDim.x);
  const int64_t k = e - g.koff[p];
  const int64_t r = g.ind[p][2 * k], c = g.ind[p][2 * k + 1];
  uint64_t kk;
  if (r < 0 || r >= B || c < 0 || c >= cols) {
    latch(st, DR_INVALID_ARGUMENT);
    kk = (uint64_t)B * (uint64_t)cols;  // past every bag
  } else {
    kk = (uint64_t)r * (uint64_t)cols + (uint64_t)c;
  }
  key[e] = kk;
  pos[e] = (int32_t)e;
}

// off[b] = first sorted position of bag >= b, b in [0, B]
__global__ void post_bags_kernel(const uint64_t* __restrict__ skey, int64_t N, int64_t B,
                                 int64_t cols, int32_t* __restrict__ off) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j > N) return;
  const int64_t bj = j < N ? (int64_t)(skey[j] / (uint64_t)cols) : B;
  const int64_t bp = j > 0 ? (int64_t)(skey[j - 1] / (uint64_t)cols) : -1;
  for (int64_t b = bp + 1; b <= bj && b <= B; ++b) off[b] = (int32_t)j;
}

template <int VEC, int G, int CPL>
__device__ __forceinline__ void seq_clip(Row<VEC, G, CPL>& x, float max_norm) {
  // emb_element *= max_norm / l2_norm when l2_norm > max_norm (SumUpEmbeddingShard)
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) s += vdot(x.v[c]);
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float l2 = sqrtf(s);
  if (l2 > max_norm) {
    const float f = max_norm / l2;
#pragma unroll
    for (int c = 0; c < CPL; ++c) x.v[c] = vmul(x.v[c], f);
  }
}

__device__ __forceinline__ const float* post_row(const PostGroup& g, int P, int64_t e, int dim) {
  int lo = 0, hi = P - 1;  // last p with koff[p] <= e
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (g.koff[mid] <= e)
      lo = mid;
    else
      hi = mid - 1;
  }
  return g.shard[lo] + (e - g.koff[lo]) * (int64_t)dim;
}

// One lane group per bag: out = 0; out += clip(e_k) in (row, col) order;
// Combine (fused_embedding_common.cu.h:11-33); 4 rows in flight.
template <int VEC, int G, int CPL>
__global__ __launch_bounds__(256) void post_pool_kernel(PostGroup g, int P, int64_t B, int dim,
                                                        const int32_t* __restrict__ off,
                                                        const int32_t* __restrict__ perm,
                                                        int combiner, float max_norm,
                                                        float* __restrict__ out,
                                                        int32_t* __restrict__ fnum) {
  using R = Row<VEC, G, CPL>;
  constexpr int GPB = 256 / G;
  const int64_t b = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
  if (b >= B) return;
  const int lg = threadIdx.x % G;
  const int dv = dim / VEC;
  const int64_t k0 = off[b], num = (int64_t)off[b + 1] - k0;
  R acc;
#pragma unroll
  for (int c = 0; c < CPL; ++c) acc.v[c] = vzero<typename VecT<VEC>::T>();
  constexpr int NB = 4;
  for (int64_t k = 0; k < num; k += NB) {
    R x[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int64_t kk = k + j < num ? k + j : num - 1;
      load_row_u<VEC, G, CPL>(x[j], post_row(g, P, perm[k0 + kk], dim), lg, dv);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (k + j >= num) break;
      if (max_norm >= 0.f) seq_clip<VEC, G, CPL>(x[j], max_norm);
      acc_add(acc, x[j]);
    }
  }
  if (combiner != DR_COMBINER_SUM) {
    const float q = combiner == DR_COMBINER_SQRTN ? sqrtf((float)num) : (float)num;
#pragma unroll
    for (int c = 0; c < CPL; ++c) acc.v[c] = vdiv(acc.v[c], q);
  }
  store_row<VEC, G, CPL>(acc, out + b * (int64_t)dim, lg, dv);
  if (lg == 0) fnum[b] = (int32_t)num;
}

struct GradShards {
  float* grad[DR_MAX_PARTITIONS];
};

// DistributeGradToShard: one lane group per entry.
template <int VEC, int G, int CPL>
__global__ __launch_bounds__(256) void post_grad_kernel(PostGroup g, GradShards o, int P, int64_t B,
                                                        int dim, const float* __restrict__ top,
                                                        const int32_t* __restrict__ fnum,
                                                        int combiner, float max_norm, int* st) {
  using R = Row<VEC, G, CPL>;
  constexpr int GPB = 256 / G;
  const int64_t e = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
  if (e >= g.koff[P]) return;
  const int lg = threadIdx.x % G;
  const int dv = dim / VEC;
  const int p = table_of(g.koff, P, e, (int64_t)blockIdx.x * GPB);
  const int64_t k = e - g.koff[p];
  int64_t r = g.ind[p][2 * k];
  if (r < 0 || r >= B) {
    if (lg == 0) latch(st, DR_INVALID_ARGUMENT);
    r = 0;
  }
  R x;
  load_row_u<VEC, G, CPL>(x, top + r * (int64_t)dim, lg, dv);
  const int n = fnum[r];
  if (combiner != DR_COMBINER_SUM) {
    const float q = combiner == DR_COMBINER_SQRTN ? sqrtf((float)n) : (float)n;
#pragma unroll
    for (int c = 0; c < CPL; ++c) x.v[c] = vdiv(x.v[c], q);
  }
  if (max_norm >= 0.f) {
    R v;
    load_row_u<VEC, G, CPL>(v, g.shard[p] + k * (int64_t)dim, lg, dv);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) s += vdot(v.v[c]);
#pragma unroll
    for (int o2 = G / 2; o2 > 0; o2 >>= 1) s += __shfl_xor(s, o2, 64);
    const float l2 = sqrtf(s);
    if (l2 > max_norm) {
      const float f = max_norm / l2;
#pragma unroll
      for (int c = 0; c < CPL; ++c) x.v[c] = vmul(x.v[c], f);
    }
  }
  store_row<VEC, G, CPL>(x, o.grad[p] + k * (int64_t)dim, lg, dv);
}

static int bits_above(int64_t x) {  // bits to hold values 0..x
  int b = 1;
  while (b < 63 && ((int64_t)1 << b) <= x) ++b;
  return b;
}

}  // namespace dr

extern "C" {

size_t dr_fused_pre_lookup_workspace_size(int64_t nnz) {
  dr::Carver c(nullptr);
  const int64_t n = nnz > 0 ? nnz : 1;
  c.take<uint64_t>(n);
  c.take<int32_t>(n);
  c.take<uint64_t>(n);
  c.take<int32_t>(n);
  c.take<char>(dr_sort_pairs_workspace_size(n));
  return c.used + 256;
}

int dr_fused_pre_lookup(const int64_t* sp_values, const int64_t* sp_indices, int64_t nnz,
                        const int64_t* partition_rows, int num_partitions, int64_t* values_out,
                        int64_t* indices_out, int64_t* part_off, void* ws, size_t ws_bytes,
                        void* stream) {
  using namespace dr;
  const int P = num_partitions;
  DR_REQUIRE(P >= 1 && P <= DR_MAX_PARTITIONS && partition_rows && part_off, DR_INVALID_ARGUMENT,
             "dr_fused_pre_lookup: num_partitions must be in [1, %d]", DR_MAX_PARTITIONS);
  DR_REQUIRE(nnz >= 0 && nnz < (1ll << 31), DR_INVALID_ARGUMENT, "bad nnz");
  DR_REQUIRE(ws_bytes >= dr_fused_pre_lookup_workspace_size(nnz), DR_INVALID_ARGUMENT,
             "workspace too small");
  PartAcc a;
  int64_t tot = 0;
  for (int p = 0; p < P; ++p) {
    DR_REQUIRE(partition_rows[p] >= 0, DR_INVALID_ARGUMENT, "negative partition size");
    tot += partition_rows[p];
    a.acc[p] = tot;
  }
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  hipStream_t s = S(stream);
  if (nnz == 0) return fill_bytes(part_off, 0, (size_t)(P + 1) * sizeof(int64_t), s);
  Carver c(ws);
  uint64_t* key = c.take<uint64_t>(nnz);
  int32_t* pos = c.take<int32_t>(nnz);
  uint64_t* skey = c.take<uint64_t>(nnz);
  int32_t* perm = c.take<int32_t>(nnz);
  const size_t sb = dr_sort_pairs_workspace_size(nnz);
  void* sws = c.take<char>(sb);
  const unsigned blocks = (unsigned)ceil_div(nnz, 256);
  hipLaunchKernelGGL(pre_keys_kernel, dim3(blocks), dim3(256), 0, s, sp_values, nnz, tot, key, pos,
                     st);
  DR_LAUNCH_CHECK();
  int rc = dr_sort_pairs(key, pos, skey, perm, nnz, 0, bits_above(tot), sws, sb, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(pre_emit_kernel, dim3(blocks), dim3(256), 0, s, a, P, skey, perm, sp_indices,
                     nnz, tot, values_out, indices_out);
  DR_LAUNCH_CHECK();
  hipLaunchKernelGGL(pre_offsets_kernel, dim3((unsigned)ceil_div(P + 1, 64)), dim3(64), 0, s, a, P,
                     skey, nnz, part_off);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

size_t dr_fused_post_lookup_workspace_size(int64_t total_entries, int64_t batch) {
  dr::Carver c(nullptr);
  const int64_t n = total_entries > 0 ? total_entries : 1;
  c.take<uint64_t>(n);
  c.take<int32_t>(n);
  c.take<uint64_t>(n);
  c.take<int32_t>(n);
  c.take<int32_t>(batch + 2);
  c.take<char>(dr_sort_pairs_workspace_size(n));
  return c.used + 256;
}

static int post_group(const float* const* shards, const int64_t* const* ind,
                      const int64_t* shard_rows, int P, dr::PostGroup* g) {
  DR_REQUIRE(P >= 1 && P <= DR_MAX_PARTITIONS && shards && ind && shard_rows, DR_INVALID_ARGUMENT,
             "num_partitions must be in [1, %d]", DR_MAX_PARTITIONS);
  memset(g, 0, sizeof(*g));
  for (int p = 0; p < P; ++p) {
    DR_REQUIRE(shard_rows[p] >= 0 && (shard_rows[p] == 0 || (shards[p] && ind[p])),
               DR_INVALID_ARGUMENT, "partition %d: missing pointers", p);
    g->shard[p] = shards[p];
    g->ind[p] = ind[p];
    g->koff[p + 1] = g->koff[p] + shard_rows[p];
  }
  DR_REQUIRE(g->koff[P] < (1ll << 31), DR_INVALID_ARGUMENT, "too many entries");
  return DR_OK;
}

#define DR_ROWS_DISPATCH(dim, aligned, LAUNCH)          \
  do {                                                  \
    if (aligned) {                                      \
      const int d4_ = (dim) / 4;                        \
      if (d4_ <= 8) LAUNCH(4, 8, 1);                    \
      else if (d4_ <= 16) LAUNCH(4, 16, 1);             \
      else if (d4_ <= 32) LAUNCH(4, 32, 1);             \
      else if (d4_ <= 64) LAUNCH(4, 64, 1);             \
      else LAUNCH(4, 64, 4);                            \
    } else if ((dim) <= 64) {                           \
      LAUNCH(1, 64, 1);                                 \
    } else if ((dim) <= 256) {                          \
      LAUNCH(1, 64, 4);                                 \
    } else {                                            \
      LAUNCH(1, 64, 16);                                \
    }                                                   \
  } while (0)

int dr_fused_post_lookup(const float* const* emb_shards, const int64_t* const* partitioned_indices,
                         const int64_t* shard_rows, int num_partitions, int64_t batch,
                         int64_t dense_cols, int dim, int combiner, float max_norm,
                         float* emb_vectors, int32_t* feature_nums, void* ws, size_t ws_bytes,
                         void* stream) {
  using namespace dr;
  const int P = num_partitions;
  PostGroup g;
  int rc = post_group(emb_shards, partitioned_indices, shard_rows, P, &g);
  if (rc) return rc;
  const int64_t N = g.koff[P];
  DR_REQUIRE(batch >= 0 && dense_cols >= 1 && dim > 0 && dim <= 1024, DR_INVALID_ARGUMENT,
             "bad batch / dense shape / dim");
  DR_REQUIRE(batch <= ((int64_t)1 << 62) / dense_cols, DR_INVALID_ARGUMENT,
             "batch * dense_cols must be < 2^62");
  DR_REQUIRE(ws_bytes >= dr_fused_post_lookup_workspace_size(N, batch), DR_INVALID_ARGUMENT,
             "workspace too small");
  if (batch == 0) return DR_OK;
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  hipStream_t s = S(stream);
  Carver c(ws);
  const int64_t n1 = N > 0 ? N : 1;
  uint64_t* key = c.take<uint64_t>(n1);
  int32_t* pos = c.take<int32_t>(n1);
  uint64_t* skey = c.take<uint64_t>(n1);
  int32_t* perm = c.take<int32_t>(n1);
  int32_t* off = c.take<int32_t>(batch + 2);
  const size_t sb = dr_sort_pairs_workspace_size(n1);
  void* sws = c.take<char>(sb);
  if (N > 0) {
    hipLaunchKernelGGL(post_keys_kernel, dim3((unsigned)ceil_div(N, 256)), dim3(256), 0, s, g, P,
                       batch, dense_cols, key, pos, st);
    DR_LAUNCH_CHECK();
    rc = dr_sort_pairs(key, pos, skey, perm, N, 0, bits_above(batch * dense_cols), sws, sb,
                       stream);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(post_bags_kernel, dim3((unsigned)ceil_div(N + 1, 256)), dim3(256), 0, s, skey,
                     N, batch, dense_cols, off);
  DR_LAUNCH_CHECK();
  bool aligned = dim % 4 == 0 && ((uintptr_t)emb_vectors & 15) == 0;
  for (int p = 0; p < P; ++p) aligned = aligned && ((uintptr_t)emb_shards[p] & 15) == 0;
#define DR_POST(V, G, C)                                                                       \
  hipLaunchKernelGGL((post_pool_kernel<V, G, C>), dim3((unsigned)ceil_div(batch, 256 / G)),   \
                     dim3(256), 0, s, g, P, batch, dim, off, perm, combiner, max_norm,         \
                     emb_vectors, feature_nums)
  DR_ROWS_DISPATCH(dim, aligned, DR_POST);
#undef DR_POST
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_fused_post_lookup_grad(const float* top_grad, const float* const* emb_shards,
                              const int64_t* const* partitioned_indices,
                              const int64_t* shard_rows, int num_partitions, int64_t batch,
                              int dim, const int32_t* feature_nums, int combiner, float max_norm,
                              float* const* grad_shards, void* stream) {
  using namespace dr;
  const int P = num_partitions;
  PostGroup g;
  int rc = post_group(emb_shards, partitioned_indices, shard_rows, P, &g);
  if (rc) return rc;
  DR_REQUIRE(dim > 0 && dim <= 1024 && batch >= 0 && grad_shards, DR_INVALID_ARGUMENT,
             "bad arguments");
  const int64_t N = g.koff[P];
  if (N == 0) return DR_OK;
  DR_REQUIRE(top_grad && feature_nums, DR_INVALID_ARGUMENT, "missing top_grad / feature_nums");
  GradShards o;
  memset(&o, 0, sizeof(o));
  bool aligned = dim % 4 == 0 && ((uintptr_t)top_grad & 15) == 0;
  for (int p = 0; p < P; ++p) {
    DR_REQUIRE(shard_rows[p] == 0 || grad_shards[p], DR_INVALID_ARGUMENT,
               "partition %d: missing grad shard", p);
    o.grad[p] = grad_shards[p];
    aligned = aligned && ((uintptr_t)emb_shards[p] & 15) == 0 && ((uintptr_t)o.grad[p] & 15) == 0;
  }
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  hipStream_t s = S(stream);
#define DR_PGRAD(V, G, C)                                                                      \
  hipLaunchKernelGGL((post_grad_kernel<V, G, C>), dim3((unsigned)ceil_div(N, 256 / G)),       \
                     dim3(256), 0, s, g, o, P, batch, dim, top_grad, feature_nums, combiner,   \
                     max_norm, st)
  DR_ROWS_DISPATCH(dim, aligned, DR_PGRAD);
#undef DR_PGRAD
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // extern "C"
