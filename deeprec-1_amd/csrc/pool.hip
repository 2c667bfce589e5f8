// pool.hip -- the hot path: grouped fused lookup + segment pooling, dense row
// gather, CSR bag offsets, deterministic segment-sum backward.
//
// Layout: a row of `dim` fp32 values is covered by a lane group of G lanes,
// each lane owning CPL chunks of VEC (4 -> dwordx4) consecutive floats, so a
// wave64 moves 64 x 16 B = 1 KiB per load instruction.  D=128 fp32: G=32,
// CPL=1 (two rows per wave instruction); D=64: G=16 (four rows).  A group
// owns NB consecutive bags of one table and issues all their row loads
// before the first store (memory-level parallelism for the random row
// reads, which are the HBM-bound part: SURVEY.md section 8d "row gather").
//
// Pooling replays the reference association order exactly:
//  ORDER_ALI: SparseSegmentReduction::Reduce
//             (core/kernels/segment_reduction_ali_ops_util.h:193-318)
//  ORDER_SEQ: FusedEmbeddingLocalSparseLookUp EmbeddingLookUp
//             (core/kernels/fused_embedding/fused_embedding_local_ops_gpu.cu.cc:41-84)
// fp32 adds are separate roundings (built with -ffp-contract=off).
#include "dr_common.h"
#include "dr_rows.h"

namespace dr {

struct PoolArgs {
  dr_pool_desc d[DR_MAX_GROUP];
};

// Sum over the G lanes of a group (xor butterfly stays inside the group).
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Pointer to the row selected by nnz position k (nullptr -> zero row).
__device__ __forceinline__ const float* select_row(const dr_pool_desc& d, int64_t k, int dim,
                                                   int* st) {
  int64_t r;
  // (descriptors are read from LDS: gld keeps these global, not flat, loads)
  if (d.ids) {
    r = gld(d.ids + k);
    // pre-resolved EV rows (dr_rows_per_nnz): negative = filtered -> default
    if (r < 0 && d.default_rows) return d.default_rows + (-r - 1) * d.default_stride;
  } else if (!d.rows) {
    r = gld(d.idx + k);
  } else {
    r = gld(d.rows + gld(d.idx + k));
    if (r < 0) return d.default_rows + (-r - 1) * d.default_stride;
    return d.pool + r * (int64_t)dim;
  }
  if (r < 0 || r >= d.pool_rows) {
    latch(st, DR_INVALID_ARGUMENT);
    return nullptr;
  }
  return d.pool + r * (int64_t)dim;
}

// clip_by_norm (embedding_ops._clip -> clip_ops.clip_by_norm) for ORDER_ALI,
// and the fused kernel's `emb *= max_norm / l2` (fused_embedding_local_ops_gpu.
// cu.cc:59-71) for ORDER_SEQ.  Enabled iff max_norm >= 0.
template <int VEC, int G, int CPL, int ORDER>
__device__ __forceinline__ void clip_row(Row<VEC, G, CPL>& x, float max_norm) {
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) s += vdot(x.v[c]);
  s = group_sum<G>(s);
  if (ORDER == DR_ORDER_ALI) {
    const float l2 = s > 0.f ? sqrtf(s) : s;
    const float den = l2 > max_norm ? l2 : max_norm;
#pragma unroll
    for (int c = 0; c < CPL; ++c) x.v[c] = vdiv(vmul(x.v[c], max_norm), den);
  } else {
    const float l2 = sqrtf(s);
    if (l2 > max_norm) {
      const float f = max_norm / l2;
#pragma unroll
      for (int c = 0; c < CPL; ++c) x.v[c] = vmul(x.v[c], f);
    }
  }
}

// BF: the rows hold bf16 values (bf16 EV / table), widened to fp32 on load;
// `dim` passed to select_row then counts float words (D / 2).
template <int VEC, int G, int CPL, bool BF>
__device__ __forceinline__ void load_any(Row<VEC, G, CPL>& x, const float* p, int lg, int dv) {
  if constexpr (BF)
    load_row_bf16<VEC, G, CPL>(x, p, lg, dv);
  else
    load_row<VEC, G, CPL>(x, p, lg, dv);
}
template <int VEC, int G, int CPL, bool BF>
__device__ __forceinline__ void store_any(const Row<VEC, G, CPL>& x, float* p, int lg, int dv) {
  if constexpr (BF)  // (BF here: a bf16 OUTPUT)
    store_row_bf16<VEC, G, CPL>(x, p, lg, dv);
  else
    store_row<VEC, G, CPL>(x, p, lg, dv);
}

template <int VEC, int G, int CPL, int ORDER, bool BF = false>
__device__ __forceinline__ void fetch(Row<VEC, G, CPL>& x, const dr_pool_desc& d, int64_t k,
                                      int dim, int lg, int dv, int* st) {
  load_any<VEC, G, CPL, BF>(x, select_row(d, k, dim, st), lg, dv);
  if (d.max_norm >= 0.f) clip_row<VEC, G, CPL, ORDER>(x, d.max_norm);
}

template <int VEC, int G, int CPL, int ORDER, bool BF = false>
__device__ __forceinline__ void fetch_p(Row<VEC, G, CPL>& x, const float* p, float max_norm,
                                        int lg, int dv) {
  load_any<VEC, G, CPL, BF>(x, p, lg, dv);
  if (max_norm >= 0.f) clip_row<VEC, G, CPL, ORDER>(x, max_norm);
}

// Row pointers of up to 4G bag positions, one per lane and window, fetched
// in parallel by the G lanes of a group before any row load (the idx -> row
// chain is paid once per bag instead of once per 8-row chunk); position k is
// read back with a shuffle inside the group.
template <int G>
struct BagPtrs {
  const float* p[4];
  int base;  // first lane of the group
  __device__ __forceinline__ const float* at(int64_t k) const {
    const int w = (int)(k / G), j = (int)(k % G);
    const float* q = w == 0 ? p[0] : (w == 1 ? p[1] : (w == 2 ? p[2] : p[3]));
    const uint64_t u = (uint64_t)(uintptr_t)q;
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)u, base + j, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(u >> 32), base + j, 64);
    return reinterpret_cast<const float*>((uintptr_t)(((uint64_t)hi << 32) | lo));
  }
};

// Unweighted bag of `num` rows, P(k) = row pointer of position k, summed in
// the reference association order.
template <int VEC, int G, int CPL, int ORDER, bool BF, bool OB, class PtrAt>
__device__ __forceinline__ void pool_bag_rows(const dr_pool_desc& d, int64_t num, float* out,
                                              int lg, int dv, const PtrAt& P) {
  using R = Row<VEC, G, CPL>;
  R acc;
#pragma unroll
  for (int c = 0; c < CPL; ++c) acc.v[c] = vzero<typename VecT<VEC>::T>();
  if (ORDER == DR_ORDER_SEQ) {
    // out = 0; out += e_k ...; Combine: / sqrtf(n) or / n
    int64_t k = 0;
    for (; k + 4 <= num; k += 4) {
      R x0, x1, x2, x3;
      fetch_p<VEC, G, CPL, ORDER, BF>(x0, P(k), d.max_norm, lg, dv);
      fetch_p<VEC, G, CPL, ORDER, BF>(x1, P(k + 1), d.max_norm, lg, dv);
      fetch_p<VEC, G, CPL, ORDER, BF>(x2, P(k + 2), d.max_norm, lg, dv);
      fetch_p<VEC, G, CPL, ORDER, BF>(x3, P(k + 3), d.max_norm, lg, dv);
      acc_add(acc, x0);
      acc_add(acc, x1);
      acc_add(acc, x2);
      acc_add(acc, x3);
    }
    for (; k < num; ++k) {
      R x;
      fetch_p<VEC, G, CPL, ORDER, BF>(x, P(k), d.max_norm, lg, dv);
      acc_add(acc, x);
    }
    if (d.combiner != DR_COMBINER_SUM) {
      const float q = d.combiner == DR_COMBINER_SQRTN ? sqrtf((float)num) : (float)num;
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc.v[c] = vdiv(acc.v[c], q);
    }
    store_any<VEC, G, CPL, OB>(acc, out, lg, dv);
    return;
  }
  // ORDER_ALI
  if (num == 1) {
    fetch_p<VEC, G, CPL, ORDER, BF>(acc, P(0), d.max_norm, lg, dv);
    store_any<VEC, G, CPL, OB>(acc, out, lg, dv);
    return;
  }
  int64_t r = num % 8;
  if (r == 0) r = 8;
  if (r == 1) r = 9;
  {
    R x[9];
#pragma unroll
    for (int j = 0; j < 9; ++j)
      if (j < r) fetch_p<VEC, G, CPL, ORDER, BF>(x[j], P(j), d.max_norm, lg, dv);
    acc = x[0];
#pragma unroll
    for (int j = 1; j < 9; ++j)
      if (j < r) acc_add(acc, x[j]);
  }
  if (num < 10 && d.combiner != DR_COMBINER_SUM) {
    const float m = d.combiner == DR_COMBINER_MEAN ? (float)num : (float)sqrt((double)num);
#pragma unroll
    for (int c = 0; c < CPL; ++c) acc.v[c] = vdiv(acc.v[c], m);
  }
  for (int64_t g = r; g < num; g += 8) {
    R x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) fetch_p<VEC, G, CPL, ORDER, BF>(x[j], P(g + j), d.max_norm, lg, dv);
    R s = x[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) acc_add(s, x[j]);
    acc_add(acc, s);
  }
  if (num >= 10 && d.combiner != DR_COMBINER_SUM) {
    const float q = d.combiner == DR_COMBINER_MEAN ? (float)num : (float)sqrt((double)num);
#pragma unroll
    for (int c = 0; c < CPL; ++c) acc.v[c] = vdiv(acc.v[c], q);
  }
  store_any<VEC, G, CPL, OB>(acc, out, lg, dv);
}

// One bag, general length, in the reference association order.  Called by
// every lane of a group together (the shuffles of BagPtrs need that).
template <int VEC, int G, int CPL, int ORDER, bool BF = false, bool OB = false>
__device__ void pool_bag(const dr_pool_desc& d, int64_t b, int dim, int lg, int dv, int* st) {
  using R = Row<VEC, G, CPL>;
  const int64_t k0 = d.bag_off[b];
  const int64_t num = (int64_t)d.bag_off[b + 1] - k0;
  float* out = d.out + b * d.out_stride;
  // an empty bag is a zero row -- except with weights and mean / sqrtn,
  // where the reference divides the zero segment_sum by a zero weight sum
  // (embedding_ops.py:636-645): 0 / 0 = NaN, which the weights branch
  // below reproduces
  if (num <= 0 && !(d.weights && d.combiner != DR_COMBINER_SUM)) {
    R z;
#pragma unroll
    for (int c = 0; c < CPL; ++c) z.v[c] = vzero<typename VecT<VEC>::T>();
    store_any<VEC, G, CPL, OB>(z, out, lg, dv);
    return;
  }
  if (d.weights) {
    // embedding_ops.py:609-651: gather * w, segment_sum, / sum(w) or sqrt(sum(w^2))
    R acc;
#pragma unroll
    for (int c = 0; c < CPL; ++c) acc.v[c] = vzero<typename VecT<VEC>::T>();
    float wsum = 0.f;
    for (int64_t k = 0; k < num; ++k) {
      R x;
      fetch<VEC, G, CPL, ORDER, BF>(x, d, k0 + k, dim, lg, dv, st);
      const float w = d.weights[k0 + k];
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc.v[c] = vadd(acc.v[c], vmul(x.v[c], w));
      wsum = wsum + (d.combiner == DR_COMBINER_SQRTN ? w * w : w);
    }
    if (d.combiner != DR_COMBINER_SUM) {
      const float q = d.combiner == DR_COMBINER_SQRTN ? sqrtf(wsum) : wsum;
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc.v[c] = vdiv(acc.v[c], q);
    }
    store_any<VEC, G, CPL, OB>(acc, out, lg, dv);
    return;
  }
  if (G >= 8 && num <= 4 * G) {
    BagPtrs<G> bp;
    bp.base = (int)(threadIdx.x % 64) - lg;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int64_t k = (int64_t)w * G + lg;
      bp.p[w] = k < num ? select_row(d, k0 + k, dim, st) : nullptr;
    }
    pool_bag_rows<VEC, G, CPL, ORDER, BF, OB>(d, num, out, lg, dv,
                                      [&](int64_t k) { return bp.at(k); });
    return;
  }
  pool_bag_rows<VEC, G, CPL, ORDER, BF, OB>(d, num, out, lg, dv,
                                    [&](int64_t k) { return select_row(d, k0 + k, dim, st); });
}

// Pooling kernels:
//  * pool_onehot_kernel (DR_POOL_ONEHOT: bag b is nnz b): a pure row copy in
//    OUTPUT order -- group g covers slots j = g*NB .. g*NB+NB-1 of the [B, T]
//    slot grid (slot j = bag j / T of table j % T), so consecutive groups
//    write consecutive NB*D-float pieces of the [B, T*D] concat; row reads
//    are random.  Nontemporal loads and stores (each row byte is touched once
//    per launch).  Measured on MI355X (tools/pool_probe.py): this
//    shape 5.08 TB/s vs 4.25 for table-major NB=8 default-policy copies.
//  * pool_fast_kernel: without the one-hot guarantee, chunks of NB bags of one
//    table whose bags each hold exactly one id, with no weights / clipping.
//  * pool_general_kernel: every other chunk (multi-hot bags, weights,
//    max_norm), replaying the reference association order.  It skips the
//    chunks the fast kernel took, by the same predicate.
template <int NB>
__device__ __forceinline__ bool chunk_is_fast(const dr_pool_desc& d, int64_t b0, int64_t B,
                                              int (&off)[NB + 1]) {
  if (b0 + NB > B || d.weights || d.max_norm >= 0.f) return false;
#pragma unroll
  for (int j = 0; j <= NB; ++j) off[j] = gld(d.bag_off + b0 + j);
  bool fast = true;
#pragma unroll
  for (int j = 0; j < NB; ++j) fast = fast && (off[j + 1] - off[j] == 1);
  return fast;
}

template <int VEC, int G, int CPL, int ORDER>
__device__ __forceinline__ void seq_zero_add(Row<VEC, G, CPL>& x) {
  // fused op (ORDER_SEQ): out = 0 + e, which turns -0.0 into +0.0 exactly
  if (ORDER == DR_ORDER_SEQ) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) x.v[c] = vadd(vzero<typename VecT<VEC>::T>(), x.v[c]);
  }
}

// WIDEN: bf16 rows widened into an fp32 output (a bf16 EV's pooled lookup,
// embedding_ops.py:606-607 casts bf16 embeddings to float32); `dim` counts
// values, rows are dim / 2 float words apart.
template <int VEC, int G, int CPL, int ORDER, int NB, bool WIDEN = false>
__global__ __launch_bounds__(256) void pool_onehot_kernel(PoolArgs args, int T, int64_t B, int dim,
                                                          int* st) {
  // The slot -> table mapping differs per lane, so the descriptors are
  // staged in LDS once per block: a per-lane descriptor read from
  // kernel-argument memory would put one more dependent memory round trip
  // ahead of every row load (measured: ~25% of the kernel time).
  __shared__ dr_pool_desc sd[DR_MAX_GROUP];
  if (threadIdx.x < T) sd[threadIdx.x] = args.d[threadIdx.x];
  __syncthreads();
  constexpr int GPB = 256 / G;
  const int64_t slots = (int64_t)T * B;
  // (an XCD-contiguous renumbering of the blocks measured 2-3 % slower:
  // profiles/r02_ab_xcd_swizzle.log)
  const int64_t s0 = ((int64_t)blockIdx.x * GPB + threadIdx.x / G) * NB;
  if (s0 >= slots) return;
  const int lg = threadIdx.x % G;
  const int dv = dim / VEC;
  Row<VEC, G, CPL> x[NB];
  float* o[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int64_t s = s0 + j;
    const float* p = nullptr;
    o[j] = nullptr;
    if (s < slots) {
      // slots < 2^31 (checked on the host): 32-bit division
      const int64_t b = (int64_t)((uint32_t)s / (uint32_t)T);
      const dr_pool_desc& d = sd[(int)(s - b * T)];
      p = select_row(d, b, WIDEN ? dim / 2 : dim, st);
      o[j] = d.out + b * d.out_stride;
    }
    load_row_copy<VEC, G, CPL, WIDEN>(x[j], p, lg, dv);
  }
  wait_loads();
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    seq_zero_add<VEC, G, CPL, ORDER>(x[j]);
    if (o[j]) store_row_nt<VEC, G, CPL>(x[j], o[j], lg, dv);
  }
}

template <int VEC, int G, int CPL, int ORDER, int NB, bool WIDEN = false>
__global__ __launch_bounds__(256) void pool_fast_kernel(PoolArgs args, int T, int64_t B, int dim,
                                                        int64_t chunks_per_table, int* st) {
  __shared__ dr_pool_desc sd[DR_MAX_GROUP];  // per-group table index: stage in LDS
  if (threadIdx.x < T) sd[threadIdx.x] = args.d[threadIdx.x];
  __syncthreads();
  constexpr int GPB = 256 / G;
  const int64_t item = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
  if (item >= (int64_t)T * chunks_per_table) return;
  const int t = (int)(item / chunks_per_table);
  const int64_t b0 = (item - (int64_t)t * chunks_per_table) * NB;
  const int lg = threadIdx.x % G;
  const int dv = dim / VEC;
  const dr_pool_desc& d = sd[t];
  int off[NB + 1];
  if (!chunk_is_fast<NB>(d, b0, B, off)) return;
  Row<VEC, G, CPL> x[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j)
    load_row_copy<VEC, G, CPL, WIDEN>(x[j], select_row(d, off[j], WIDEN ? dim / 2 : dim, st), lg,
                                      dv);
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    seq_zero_add<VEC, G, CPL, ORDER>(x[j]);
    store_row_nt<VEC, G, CPL>(x[j], d.out + (b0 + j) * d.out_stride, lg, dv);
  }
}

// One bag per lane group (multi-hot bags need the parallelism: a group per
// chunk of NB bags left most of the chip idle), over a capped grid that
// strides through the bags so the per-block descriptor staging and the
// early exits of fast chunks stay cheap.
// BF: bf16 rows and output; `dim` = float words per row (D / 2), the lane
// layout covers D values in chunks of VEC (dv = 2 * dim / VEC).
template <int VEC, int G, int CPL, int ORDER, int NB, bool BF = false, bool OB = false>
__global__ __launch_bounds__(256) void pool_general_kernel(PoolArgs args, int T, int64_t B,
                                                           int dim, int* st) {
  __shared__ dr_pool_desc sd[DR_MAX_GROUP];  // per-group table index: stage in LDS
  if (threadIdx.x < T) sd[threadIdx.x] = args.d[threadIdx.x];
  __syncthreads();
  constexpr int GPB = 256 / G;
  const int lg = threadIdx.x % G;
  const int dv = (BF ? 2 * dim : dim) / VEC;
  const int64_t total = (int64_t)T * B;
  for (int64_t item = (int64_t)blockIdx.x * GPB + threadIdx.x / G; item < total;
       item += (int64_t)gridDim.x * GPB) {
    const int t = (int)(item / B);
    const int64_t b = item - (int64_t)t * B;
    const dr_pool_desc& d = sd[t];
    int off[NB + 1];
    if (chunk_is_fast<NB>(d, b - b % NB, B, off)) continue;  // taken by pool_fast_kernel
    pool_bag<VEC, G, CPL, ORDER, BF, OB>(d, b, dim, lg, dv, st);
  }
}

enum { POOL_ONEHOT = 1 };
static constexpr int kOneHotNB = 4;  // rows in flight per lane group (probe optimum)
static constexpr int kChunkNB = 8;   // bags per chunk, fast/general split
static constexpr int64_t kGeneralBlocks = 256 * 16;  // general-kernel grid cap (16 per CU)

template <int VEC, int G, int CPL, int ORDER, bool WIDEN = false>
static int launch_pool(const PoolArgs& a, int T, int64_t B, int dim, int flags, hipStream_t s,
                       int* st) {
  if (flags & POOL_ONEHOT) {
    const int64_t items = ceil_div((int64_t)T * B, kOneHotNB);
    timing_mark(DR_TIME_POOL_ONEHOT, s, true);
    hipLaunchKernelGGL((pool_onehot_kernel<VEC, G, CPL, ORDER, kOneHotNB, WIDEN>),
                       dim3((unsigned)ceil_div(items, 256 / G)), dim3(256), 0, s, a, T, B, dim,
                       st);
    timing_mark(DR_TIME_POOL_ONEHOT, s, false);
  } else {
    const int64_t cpt = ceil_div(B, kChunkNB);
    const unsigned blocks = (unsigned)ceil_div((int64_t)T * cpt, 256 / G);
    hipLaunchKernelGGL((pool_fast_kernel<VEC, G, CPL, ORDER, kChunkNB, WIDEN>), dim3(blocks),
                       dim3(256), 0, s, a, T, B, dim, cpt, st);
    if (!(flags & 2)) {  // (2: fast kernel only -- the bf16 dispatcher's copies)
      const int64_t gblocks = std::min<int64_t>(ceil_div((int64_t)T * B, 256 / G), kGeneralBlocks);
      hipLaunchKernelGGL((pool_general_kernel<VEC, G, CPL, ORDER, kChunkNB>),
                         dim3((unsigned)gblocks), dim3(256), 0, s, a, T, B, dim, st);
    }
  }
  DR_LAUNCH_CHECK();
  return DR_OK;
}

// bf16 rows (DR_POOL_BF16).  bf16 output (DR_POOL_OUT_BF16): one-hot slots
// and single-id chunks are bitwise copies of D / 2 float words (the fp32
// kernels on words), multi-hot bags / weights / max_norm pool in fp32 and
// round each bag once.  fp32 output (the reference's cast of bf16
// embeddings to float32 before pooling, embedding_ops.py:606-607): the
// copies widen each value, bags pool in fp32.
template <int G, int CPL, bool OB>
static int launch_pool_bf16_general(const PoolArgs& a, int T, int64_t B, int words, hipStream_t s,
                                    int* st) {
  const int64_t gblocks = std::min<int64_t>(ceil_div((int64_t)T * B, 256 / G), kGeneralBlocks);
  hipLaunchKernelGGL((pool_general_kernel<4, G, CPL, DR_ORDER_ALI, kChunkNB, true, OB>),
                     dim3((unsigned)gblocks), dim3(256), 0, s, a, T, B, words, st);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

template <int ORDER>
static int dispatch_pool(const PoolArgs& a, int T, int64_t B, int dim, int flags, hipStream_t s,
                         int* st);

template <int G, int CPL>
static int launch_bf16(const PoolArgs& a, int T, int64_t B, int D, int flags, bool out_bf16,
                       hipStream_t s, int* st) {
  const int words = D / 2;
  if (out_bf16) {
    if (flags & POOL_ONEHOT) return dispatch_pool<DR_ORDER_ALI>(a, T, B, words, flags, s, st);
    int rc = dispatch_pool<DR_ORDER_ALI>(a, T, B, words, flags | 2 /* fast only */, s, st);
    if (rc) return rc;
    return launch_pool_bf16_general<G, CPL, true>(a, T, B, words, s, st);
  }
  int rc = launch_pool<4, G, CPL, DR_ORDER_ALI, true>(a, T, B, D, flags | 2, s, st);
  if (rc || (flags & POOL_ONEHOT)) return rc;
  return launch_pool_bf16_general<G, CPL, false>(a, T, B, words, s, st);
}

static int dispatch_pool_bf16(const PoolArgs& a, int T, int64_t B, int D, int flags, bool out_bf16,
                              hipStream_t s, int* st) {
  const int d4 = D / 4;
  if (d4 <= 4) return launch_bf16<4, 1>(a, T, B, D, flags, out_bf16, s, st);
  if (d4 <= 8) return launch_bf16<8, 1>(a, T, B, D, flags, out_bf16, s, st);
  if (d4 <= 16) return launch_bf16<16, 1>(a, T, B, D, flags, out_bf16, s, st);
  if (d4 <= 32) return launch_bf16<32, 1>(a, T, B, D, flags, out_bf16, s, st);
  if (d4 <= 64) return launch_bf16<64, 1>(a, T, B, D, flags, out_bf16, s, st);
  if (d4 <= 128) return launch_bf16<64, 2>(a, T, B, D, flags, out_bf16, s, st);
  if (d4 <= 256) return launch_bf16<64, 4>(a, T, B, D, flags, out_bf16, s, st);
  set_error("bf16 dim %d unsupported (max 1024)", D);
  return DR_INVALID_ARGUMENT;
}

template <int ORDER>
static int dispatch_pool(const PoolArgs& a, int T, int64_t B, int dim, int flags, hipStream_t s,
                         int* st) {
#define DR_POOL(V, G, C) return launch_pool<V, G, C, ORDER>(a, T, B, dim, flags, s, st)
  if (dim % 4 == 0) {
    const int d4 = dim / 4;
    if (d4 <= 1) DR_POOL(4, 1, 1);
    if (d4 <= 2) DR_POOL(4, 2, 1);
    if (d4 <= 4) DR_POOL(4, 4, 1);
    if (d4 <= 8) DR_POOL(4, 8, 1);
    if (d4 <= 16) DR_POOL(4, 16, 1);
    if (d4 <= 32) DR_POOL(4, 32, 1);
    if (d4 <= 64) DR_POOL(4, 64, 1);
    if (d4 <= 128) DR_POOL(4, 64, 2);
    if (d4 <= 256) DR_POOL(4, 64, 4);
  } else {
    if (dim <= 4) DR_POOL(1, 4, 1);
    if (dim <= 8) DR_POOL(1, 8, 1);
    if (dim <= 16) DR_POOL(1, 16, 1);
    if (dim <= 32) DR_POOL(1, 32, 1);
    if (dim <= 64) DR_POOL(1, 64, 1);
    if (dim <= 256) DR_POOL(1, 64, 4);
  }
#undef DR_POOL
  set_error("dim %d unsupported (max 1024 fp32 / 256 unaligned)", dim);
  return DR_INVALID_ARGUMENT;
}

// ---------------------------------------------------------------------------
// CSR bag offsets from sorted segment ids.
// ---------------------------------------------------------------------------
template <class TI>
__global__ void bag_offsets_kernel(const TI* __restrict__ seg, int64_t stride, int64_t n,
                                   const int64_t* n_dev, int64_t B, int32_t* __restrict__ off,
                                   int* st) {
  const int64_t ne = eff_n(n, n_dev);
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > ne) return;
  if (ne == 0) {
    for (int64_t r = 0; r <= B; ++r) off[r] = 0;
    return;
  }
  if (k == ne) return;
  int64_t s = (int64_t)seg[k * stride];
  int64_t prev = k > 0 ? (int64_t)seg[(k - 1) * stride] : -1;
  if (s < prev || s < 0 || s >= B) {
    latch(st, DR_INVALID_ARGUMENT);
    s = s < 0 ? 0 : (s >= B ? B - 1 : s);
    prev = prev < -1 ? -1 : (prev >= B ? B - 1 : prev);  // keep the window in [0, B]
    if (s < prev) return;
  }
  for (int64_t r = prev + 1; r <= s; ++r) off[r] = (int32_t)k;
  if (k == ne - 1)
    for (int64_t r = s + 1; r <= B; ++r) off[r] = (int32_t)ne;
}

// Grouped form: blockIdx.y = feature.
struct BagGroup {
  const int64_t* seg[DR_MAX_GROUP];
  int64_t stride[DR_MAX_GROUP];
  int64_t n[DR_MAX_GROUP];
  int32_t* off[DR_MAX_GROUP];
};

__global__ void bag_offsets_grouped_kernel(BagGroup g, int64_t B, int* st) {
  const int t = blockIdx.y;
  const int64_t ne = g.n[t];
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > ne) return;
  const int64_t* seg = g.seg[t];
  const int64_t stride = g.stride[t];
  int32_t* off = g.off[t];
  if (ne == 0) {
    for (int64_t r = k; r <= B; r += blockDim.x) off[r] = 0;
    return;
  }
  if (k == ne) return;
  int64_t s = seg[k * stride];
  int64_t prev = k > 0 ? seg[(k - 1) * stride] : -1;
  if (s < prev || s < 0 || s >= B) {
    latch(st, DR_INVALID_ARGUMENT);
    s = s < 0 ? 0 : (s >= B ? B - 1 : s);
    // an out-of-range predecessor must not move the write window outside
    // [0, B] (seg = [-5, 0] would otherwise write off[-4..0])
    prev = prev < -1 ? -1 : (prev >= B ? B - 1 : prev);
    if (s < prev) return;
  }
  for (int64_t r = prev + 1; r <= s; ++r) off[r] = (int32_t)k;
  if (k == ne - 1)
    for (int64_t r = s + 1; r <= B; ++r) off[r] = (int32_t)ne;
}

// Zero-fill of every table's offsets ahead of bag_offsets_grouped_kernel
// (see launch_bag_offsets: positions skipped for bad input leave no garbage).
__global__ void bag_zero_grouped_kernel(BagGroup g, int64_t B) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r <= B) g.off[blockIdx.y][r] = 0;
}

// rowsel[i] = rows[koff[t] + idx[i]] for i in feature t: the EV row of every
// nnz, resolved once so the pool kernel's load chain is bag_off -> row id ->
// row data (one dependent load fewer).
struct KoffGroup {
  int64_t koff[DR_MAX_GROUP + 1];
};

__global__ void rows_per_nnz_kernel(KoffGroup g, int T, const int64_t* __restrict__ rows,
                                    const int32_t* __restrict__ idx, int64_t* __restrict__ rowsel) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.koff[T]) return;
  const int t = table_of(g.koff, T, i, (int64_t)blockIdx.x * blockDim.x);
  rowsel[i] = rows[g.koff[t] + idx[i]];
}

// Caller-supplied segment ids may be unsorted or out of range: the kernel
// latches INVALID_ARGUMENT, but the positions it skips would leave entries
// of `off` unwritten, and a pool launched behind it (no host sync in
// between) would follow garbage offsets.  So `off` is zero-filled first:
// every entry then lies in [0, n] and a bad bag reads as empty or as a
// range of valid positions.  Internal, sorted-by-construction keys skip it.
template <class TI>
static int launch_bag_offsets(const TI* seg, int64_t stride, int64_t n, const int64_t* n_dev,
                              int64_t B, int32_t* off, hipStream_t s, bool trusted = false) {
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  if (!trusted) {
    int rc = fill_bytes(off, 0, (size_t)(B + 1) * sizeof(int32_t), s);
    if (rc) return rc;
  }
  const unsigned blocks = (unsigned)ceil_div(n + 1, 256);
  hipLaunchKernelGGL(bag_offsets_kernel<TI>, dim3(blocks), dim3(256), 0, s, seg, stride, n, n_dev,
                     B, off, st);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

// ---------------------------------------------------------------------------
// Row gather (ResourceGather): group per index, NB indices per group.
// ---------------------------------------------------------------------------
// EV mode (dr_ev_gather copy-out): ids are resolved rows, a negative row
// takes default row i of `defaults` [n, dim] or, without it, the EV default.
template <int VEC, int G, int CPL, bool EV>
__global__ __launch_bounds__(256) void gather_kernel(const float* __restrict__ table, int64_t rows,
                                                     int dim, const int64_t* __restrict__ ids,
                                                     int64_t n, float* __restrict__ out, int* st,
                                                     const float* __restrict__ defaults,
                                                     const float* __restrict__ dflt) {
  constexpr int GPB = 256 / G;
  constexpr int NB = 4;
  const int64_t i0 = ((int64_t)blockIdx.x * GPB + threadIdx.x / G) * NB;
  const int lg = threadIdx.x % G;
  const int dv = dim / VEC;
  Row<VEC, G, CPL> x[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const float* p = nullptr;
    if (i0 + j < n) {
      const int64_t r = ids[i0 + j];
      if (EV)
        p = r >= 0 ? table + r * (int64_t)dim : (defaults ? defaults + (i0 + j) * dim : dflt);
      else if (r >= 0 && r < rows)
        p = table + r * (int64_t)dim;
      else
        latch(st, DR_INVALID_ARGUMENT);
    }
    load_row_nt<VEC, G, CPL>(x[j], p, lg, dv);
  }
#pragma unroll
  for (int j = 0; j < NB; ++j)
    if (i0 + j < n) store_row_nt<VEC, G, CPL>(x[j], out + (i0 + j) * (int64_t)dim, lg, dv);
}

template <int VEC, int G, int CPL, bool EV>
static int launch_gather(const float* table, int64_t rows, int dim, const int64_t* ids,
                         int64_t n, float* out, hipStream_t s, int* st, const float* defaults,
                         const float* dflt) {
  const int64_t blocks = ceil_div(ceil_div(n, 4), 256 / G);
  hipLaunchKernelGGL((gather_kernel<VEC, G, CPL, EV>), dim3((unsigned)blocks), dim3(256), 0, s,
                     table, rows, dim, ids, n, out, st, defaults, dflt);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

template <bool EV>
static int gather_dispatch(const float* table, int64_t rows, int d, const int64_t* ids, int64_t n,
                           float* out, hipStream_t s, int* st, const float* defaults,
                           const float* dflt) {
  const bool al = ((((uintptr_t)table) | ((uintptr_t)out) | ((uintptr_t)defaults) |
                    ((uintptr_t)dflt)) & 15) == 0;
#define DR_G(VEC, G, CPL) \
  return launch_gather<VEC, G, CPL, EV>(table, rows, d, ids, n, out, s, st, defaults, dflt)
  if (d % 4 == 0 && al) {
    const int d4 = d / 4;
    if (d4 <= 4) DR_G(4, 4, 1);
    if (d4 <= 8) DR_G(4, 8, 1);
    if (d4 <= 16) DR_G(4, 16, 1);
    if (d4 <= 32) DR_G(4, 32, 1);
    if (d4 <= 64) DR_G(4, 64, 1);
    DR_G(4, 64, 4);
  }
  if (d <= 8) DR_G(1, 8, 1);
  if (d <= 32) DR_G(1, 32, 1);
  if (d <= 64) DR_G(1, 64, 1);
  if (d <= 256) DR_G(1, 64, 4);
#undef DR_G
  set_error("dim %d unsupported", d);
  return DR_INVALID_ARGUMENT;
}

// dr_ev_gather's copy-out (ev.hip): out[i] = rows[i] >= 0 ? pool[rows[i]]
// : (defaults ? defaults[i] : dflt).
int gather_ev_rows(const float* pool, int64_t dim, const int64_t* rows, int64_t n,
                   const float* defaults, const float* dflt, float* out, hipStream_t s) {
  DR_REQUIRE(dim > 0 && dim <= 1024, DR_INVALID_ARGUMENT, "bad gather dim");
  if (n == 0) return DR_OK;
  return gather_dispatch<true>(pool, 0, (int)dim, rows, n, out, s, status_word(), defaults, dflt);
}

// ---------------------------------------------------------------------------
// Deterministic CSR segment sum: out[u] = init + sum_{j in [off[u],off[u+1])}
// src[srow(j)] * scale(j), j ascending.  Used for SparseSegment*Grad,
// UnsortedSegmentSum and the pooled-lookup backward.
//   mode 0: sum from 0.0f             (UnsortedSegmentSum, Sum grad)
//   mode 1: ali mean grad (first assigns, scale = float(1/double(cnt)))
//   mode 2: ali sqrtn grad (scale = float(1/sqrt(double(cnt))))
// srow(j) = seg_of_pos ? seg_of_pos[perm[j]] : perm[j]; cnt from bag_off.
// ---------------------------------------------------------------------------
// A group of G lanes owns CSR_SB consecutive segments, whose positions form
// one contiguous window [off[u0], off[u0 + CSR_SB]) of the sorted order: it
// loads CSR_NB rows of the window at a time (independent loads, however
// the segment boundaries fall) and sums them into ONE running row in
// ascending j, storing each segment's row when the window passes its end
// (empty segments get zeros).  Per segment the association order is the
// serial one; the window gives every load batch CSR_NB useful rows where a
// group per segment (1.6 positions on average for an all-distinct batch)
// kept about 2 of 4 loads useful behind a chain of dependent loads.
static constexpr int CSR_SB = 4, CSR_NB = 8;

template <int VEC, int G, int CPL>
__global__ __launch_bounds__(256) void csr_sum_kernel(
    const float* __restrict__ src, int64_t src_stride, int64_t src_rows,
    const int32_t* __restrict__ perm, const int32_t* __restrict__ seg_of_pos,
    const int32_t* __restrict__ off, const int32_t* __restrict__ bag_off, int64_t U,
    const int64_t* U_dev, int dim, int mode, float* __restrict__ out, int* st) {
  constexpr int GPB = 256 / G;
  const int64_t ue = eff_n(U, U_dev);
  const int64_t u0 = ((int64_t)blockIdx.x * GPB + threadIdx.x / G) * CSR_SB;
  if (u0 >= ue) return;
  const int lg = threadIdx.x % G;
  const int dv = dim / VEC;
  using R = Row<VEC, G, CPL>;
  using V = typename VecT<VEC>::T;
  const int ns = ue - u0 < CSR_SB ? (int)(ue - u0) : CSR_SB;
  // window bounds: o0 .. o4 (segments past ns are empty, never stored)
  const int32_t o0 = gld(off + u0);
  const int32_t o1 = gld(off + u0 + (ns > 1 ? 1 : ns));
  const int32_t o2 = gld(off + u0 + (ns > 2 ? 2 : ns));
  const int32_t o3 = gld(off + u0 + (ns > 3 ? 3 : ns));
  const int32_t o4 = gld(off + u0 + ns);
  auto bound = [&](int s) -> int32_t {  // end of segment s (s < CSR_SB)
    return s == 0 ? o1 : (s == 1 ? o2 : (s == 2 ? o3 : o4));
  };
  R cur;
#pragma unroll
  for (int c = 0; c < CPL; ++c) cur.v[c] = vzero<V>();
  bool started = false;
  int s = 0;
  int32_t nxt = o1;
  auto finish = [&]() {  // store segment s, move to s + 1
    store_row_nt<VEC, G, CPL>(cur, out + (u0 + s) * (int64_t)dim, lg, dv);
#pragma unroll
    for (int c = 0; c < CPL; ++c) cur.v[c] = vzero<V>();
    started = false;
    ++s;
    nxt = bound(s < CSR_SB ? s : CSR_SB - 1);
  };
  for (int32_t jb = o0; jb < o4; jb += CSR_NB) {
    R x[CSR_NB];
    int64_t rr[CSR_NB];
#pragma unroll
    for (int q = 0; q < CSR_NB; ++q) {  // unconditional, clamped loads (load_row_u)
      const int32_t jq = jb + q < o4 ? jb + q : o4 - 1;
      rr[q] = gld(perm + jq);
    }
    if (seg_of_pos) {
#pragma unroll
      for (int q = 0; q < CSR_NB; ++q) rr[q] = gld(seg_of_pos + rr[q]);
    }
    bool bad = false;
#pragma unroll
    for (int q = 0; q < CSR_NB; ++q) {
      const bool okr = (rr[q] >= 0) & (rr[q] < src_rows);
      bad |= (jb + q < o4) & !okr;
      rr[q] = okr ? rr[q] : -1;
      load_row_u<VEC, G, CPL>(x[q], src + (okr ? rr[q] : 0) * src_stride, lg, dv);
    }
    wait_loads();
#pragma unroll
    for (int q = 0; q < CSR_NB; ++q)
      if (rr[q] < 0) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) x[q].v[c] = vzero<V>();
      }
    if (bad) latch(st, DR_INVALID_ARGUMENT);
#pragma unroll
    for (int q = 0; q < CSR_NB; ++q) {
      const int32_t j = jb + q;
      if (j >= o4) break;
      while (j >= nxt) finish();  // (empty segments in between get zeros)
      if (mode == 0) {
        acc_add(cur, x[q]);
      } else {
        const int32_t cnt = (rr[q] >= 0 && bag_off) ? bag_off[rr[q] + 1] - bag_off[rr[q]] : 1;
        if (cnt != 1) {
          const float sc = mode == 2 ? (float)(1.0 / sqrt((double)cnt)) : (float)(1.0 / (double)cnt);
#pragma unroll
          for (int c = 0; c < CPL; ++c) x[q].v[c] = vmul(x[q].v[c], sc);
        }
        if (!started)
          cur = x[q];
        else
          acc_add(cur, x[q]);
        started = true;
      }
    }
  }
  while (s < ns) finish();
}

template <int VEC, int G, int CPL>
static int launch_csr_sum(const float* src, int64_t src_stride, int64_t src_rows,
                          const int32_t* perm, const int32_t* seg_of_pos, const int32_t* off,
                          const int32_t* bag_off, int64_t U, const int64_t* U_dev, int dim,
                          int mode, float* out, hipStream_t s, int* st) {
  const int64_t blocks = ceil_div(ceil_div(U > 0 ? U : 1, CSR_SB), 256 / G);
  hipLaunchKernelGGL((csr_sum_kernel<VEC, G, CPL>), dim3((unsigned)blocks), dim3(256), 0, s, src,
                     src_stride, src_rows, perm, seg_of_pos, off, bag_off, U, U_dev, dim, mode,
                     out, st);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

static int dispatch_csr_sum(const float* src, int64_t src_stride, int64_t src_rows,
                            const int32_t* perm, const int32_t* seg_of_pos, const int32_t* off,
                            const int32_t* bag_off, int64_t U, const int64_t* U_dev, int dim,
                            int mode, float* out, hipStream_t s, int* st) {
#define DR_CSR(V, G, C) \
  return launch_csr_sum<V, G, C>(src, src_stride, src_rows, perm, seg_of_pos, off, bag_off, U, U_dev, dim, mode, out, s, st)
  if (dim % 4 == 0 && (src_stride % 4) == 0) {
    const int d4 = dim / 4;
    if (d4 <= 2) DR_CSR(4, 2, 1);
    if (d4 <= 4) DR_CSR(4, 4, 1);
    if (d4 <= 8) DR_CSR(4, 8, 1);
    if (d4 <= 16) DR_CSR(4, 16, 1);
    if (d4 <= 32) DR_CSR(4, 32, 1);
    if (d4 <= 64) DR_CSR(4, 64, 1);
    if (d4 <= 256) DR_CSR(4, 64, 4);
  } else {
    if (dim <= 8) DR_CSR(1, 8, 1);
    if (dim <= 32) DR_CSR(1, 32, 1);
    if (dim <= 64) DR_CSR(1, 64, 1);
    if (dim <= 256) DR_CSR(1, 64, 4);
  }
#undef DR_CSR
  set_error("dim %d unsupported", dim);
  return DR_INVALID_ARGUMENT;
}

// seg (int32) -> sort keys; negatives go to a sentinel bucket past `limit`.
__global__ void keys_from_i32_kernel(const int32_t* __restrict__ seg, int64_t n, int64_t limit,
                                     uint64_t* __restrict__ keys, int32_t* __restrict__ vals,
                                     int* st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t s = seg[i];
  if (s >= limit) {
    latch(st, DR_INVALID_ARGUMENT);
    s = limit;
  }
  keys[i] = (uint64_t)(s < 0 ? limit : s);
  vals[i] = (int32_t)i;
}

static int bits_for(int64_t x) {
  int b = 0;
  while (b < 63 && ((int64_t)1 << b) <= x) ++b;
  return b;
}

struct SegSumWs {
  uint64_t* kin;
  int32_t* vin;
  uint64_t* kout;
  int32_t* perm;
  int32_t* off;
  void* sort_ws;
  size_t sort_bytes;
};

static SegSumWs carve_segsum(void* ws, int64_t n, int64_t num_out, size_t* used) {
  Carver c(ws);
  SegSumWs w;
  const int64_t nn = n > 0 ? n : 1;
  w.kin = c.take<uint64_t>(nn);
  w.vin = c.take<int32_t>(nn);
  w.kout = c.take<uint64_t>(nn);
  w.perm = c.take<int32_t>(nn);
  w.off = c.take<int32_t>(num_out + 2);
  w.sort_bytes = dr_sort_pairs_workspace_size(n);
  w.sort_ws = c.take<char>(w.sort_bytes);
  if (used) *used = c.used + 256;
  return w;
}

// Shared driver: group positions by seg (stable), then CSR-sum.
static int segsum_driver(const int32_t* keyseg, int64_t n, int64_t num_out, const int64_t* U_dev,
                         const float* src, int64_t src_stride, int64_t src_rows,
                         const int32_t* seg_of_pos, const int32_t* bag_off, int dim, int mode,
                         float* out, void* ws, hipStream_t s) {
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  size_t used = 0;
  SegSumWs w = carve_segsum(ws, n, num_out, &used);
  if (num_out == 0) return DR_OK;
  if (n == 0) return fill_bytes(out, 0, (size_t)num_out * dim * sizeof(float), s);
  // (rows are loaded through clamped indices: a row 0 must exist)
  DR_REQUIRE(src_rows > 0, DR_INVALID_ARGUMENT, "segment ids given for an empty data tensor");
  hipLaunchKernelGGL(keys_from_i32_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s,
                     keyseg, n, num_out, w.kin, w.vin, st);
  DR_LAUNCH_CHECK();
  int rc = dr_sort_pairs(w.kin, w.vin, w.kout, w.perm, n, 0, bits_for(num_out), w.sort_ws,
                         w.sort_bytes, s);
  if (rc) return rc;
  // offsets over num_out + 1 buckets (the last one collects skipped positions)
  rc = launch_bag_offsets<uint64_t>(w.kout, 1, n, nullptr, num_out + 1, w.off, s, true);
  if (rc) return rc;
  return dispatch_csr_sum(src, src_stride, src_rows, w.perm, seg_of_pos, w.off, bag_off, num_out,
                          U_dev, dim, mode, out, s, st);
}

// ---- grouped pooling backward (dr_pool_grad_grouped) -----------------------
// One stable radix sort of all features' nnz by global unique row
// (koff[t] + idx[k]) replaces T per-feature sorts; one CSR pass sums them.
struct GradGroup {
  dr_pool_grad_desc d[DR_MAX_GROUP];
  int64_t koff[DR_MAX_GROUP + 1];
};

__device__ __forceinline__ int grad_table(const GradGroup& g, int T, int64_t i,
                                          int64_t block_first) {
  return table_of(g.koff, T, i, block_first);
}

__global__ void grad_keys_kernel(GradGroup g, int T, uint64_t* __restrict__ kin,
                                 int32_t* __restrict__ vin, int* st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.koff[T]) return;
  const int t = grad_table(g, T, i, (int64_t)blockIdx.x * blockDim.x);
  const int64_t k = i - g.koff[t];
  int64_t u = g.d[t].idx[k];
  if (u < 0 || u >= g.d[t].nnz) {
    latch(st, DR_INVALID_ARGUMENT);
    u = g.koff[T] - g.koff[t];  // sentinel bucket past the end
  }
  kin[i] = (uint64_t)(g.koff[t] + u);
  vin[i] = (int32_t)i;
}

// Position-driven over the sorted (global unique row, nnz) pairs: a group
// owns NB consecutive sorted positions.  Runs (all nnz of one unique row)
// are cut into chunks of kGradChunk positions counted from the run's start;
// a position that starts a chunk sums it in ascending nnz order (the sort is
// stable), every other position is skipped.  A run that fits one chunk --
// every run in practice, and every run of the parity tests -- is therefore
// summed exactly in the serial order of the reference's CPU loops
// (UnsortedSegmentSum / SparseSegmentReductionGrad).  A longer run (a
// padding id repeated over a whole DIN history batch, a hot Zipf key) is
// the ordered sum of its chunk partials, ((c_0 + c_1) + c_2) + ...: fixed
// association, deterministic run to run, no atomics, and no single wave
// walking a run of 10^5 positions.  The common one-element run costs two
// independent sequential loads (key, nnz) and one row load.
static constexpr int64_t kGradChunk = 256;

// Scratch of the chunked pass: run_start = the segsum workspace's off[0, n)
// (unused by the grouped path), long-run count = off[n + 1]; the long-run
// list (2 int32 per run) and the chunk partials (dim <= kGradMaxDim floats per
// chunk) follow the segsum workspace (dr_pool_grad_grouped_workspace_size).
static constexpr int64_t kGradMaxDim = 1024;
static size_t grad_chunk_ws_bytes(int64_t n) {
  const int64_t chunks = n / kGradChunk + 2;
  return (size_t)(2 * chunks * sizeof(int32_t) + 256 + chunks * kGradMaxDim * sizeof(float) + 256);
}
struct GradWs {
  int32_t* run_start;
  int32_t* nlong;
  int32_t* longs;
  float* part;
};
static constexpr int kGradChain = 4;         // positions of a chunk fetched per step (80 VGPRs: 6 waves/SIMD)
static constexpr int kGradFinishChain = 32;  // chunk partials of a long run fetched per step

// run_start[u] = first sorted position of row u; clears the long-run count.
__global__ void grad_run_start_kernel(const uint64_t* __restrict__ skey, int64_t N,
                                      int32_t* __restrict__ run_start, int32_t* __restrict__ nlong) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p == 0) *nlong = 0;
  if (p >= N) return;
  const uint64_t u = skey[p];
  if (u < (uint64_t)N && (p == 0 || skey[p - 1] != u)) run_start[u] = (int32_t)p;
}

// W: some feature of the group is weighted (dr_pool_grad_desc.weights): a
// separate instantiation, so the unweighted kernel keeps its register budget.
template <int VEC, int G, int CPL, int NB, bool W>
__global__ __launch_bounds__(256) void grad_seg_kernel(GradGroup g, int T, int64_t B,
                                                       const uint64_t* __restrict__ skey,
                                                       const int32_t* __restrict__ perm,
                                                       const int32_t* __restrict__ run_start,
                                                       int dim, float* __restrict__ out,
                                                       float* __restrict__ part,
                                                       int32_t* __restrict__ longs,
                                                       int32_t* __restrict__ nlong, int chunked,
                                                       int* st) {
  __shared__ dr_pool_grad_desc sd[DR_MAX_GROUP];  // per-lane table index: stage in LDS
  if (threadIdx.x < T) sd[threadIdx.x] = g.d[threadIdx.x];
  __syncthreads();
  constexpr int GPB = 256 / G;
  const int64_t N = g.koff[T];
  const int64_t p0 = ((int64_t)blockIdx.x * GPB + threadIdx.x / G) * NB;
  if (p0 >= N) return;
  const int64_t pf = (int64_t)blockIdx.x * GPB * NB;  // block's first position
  const int64_t ufirst = (int64_t)skey[pf];           // uniform: its row, for table_of
  const int lg = threadIdx.x % G;
  const int dv = dim / VEC;
  using R = Row<VEC, G, CPL>;
  using V = typename VecT<VEC>::T;
  // -- keys of the NB positions and their neighbours: unconditional loads --
  int64_t uk[NB + 2];
#pragma unroll
  for (int q = -1; q <= NB; ++q) {
    int64_t pp = p0 + q;
    pp = pp < 0 ? 0 : (pp >= N ? N - 1 : pp);
    uk[q + 1] = (int64_t)skey[pp];
  }
  // run starts are needed only by positions inside a run (chunk alignment);
  // a wave with none (all-distinct ids, the common case) skips that
  // dependent load -- the chain key -> start -> source -> row is the
  // kernel's latency bound
  int64_t rsq[NB];
  bool inner = false;
#pragma unroll
  for (int q = 0; q < NB; ++q) inner |= (p0 + q) > 0 && uk[q] == uk[q + 1];
  if (chunked && __ballot(inner)) {
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int64_t u = uk[q + 1];
      rsq[q] = run_start[u < N ? u : 0];
    }
  } else {
#pragma unroll
    for (int q = 0; q < NB; ++q) rsq[q] = p0 + q;
  }
  bool head[NB], single[NB];
  int64_t uq[NB], sq[NB];
  int tq[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int64_t p = p0 + q;
    const int64_t u = uk[q + 1];
    const bool in = p < N && u < N;  // u == N: sentinel for out-of-range idx
    const bool rhead = p == 0 || uk[q] != u;
    sq[q] = rhead ? p : rsq[q];
    // exact (default): only run heads; a run longer than kGradChunk is queued
    // whole for grad_long_kernel.  chunked (A/B): chunk heads too.
    head[q] = in && (rhead || (chunked && (p - sq[q]) % kGradChunk == 0));
    single[q] = p + 1 >= N || uk[q + 2] != u;
    uq[q] = u;
    tq[q] = head[q] ? table_of(g.koff, T, u, ufirst < N ? ufirst : 0) : 0;
  }
  // -- source rows of the head positions: one batch of unconditional loads --
  int64_t rq[NB];
  int64_t kq[W ? NB : 1];  // feature-local position (weight index)
  bool bad = false;
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    int64_t pp = p0 + q;
    pp = pp >= N ? N - 1 : pp;
    const int64_t k = (int64_t)perm[pp] - g.koff[tq[q]];
    rq[q] = head[q] && k >= 0 && k < sd[tq[q]].nnz ? k : 0;
    if (W) kq[W ? q : 0] = rq[q];
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int64_t* segp = sd[tq[q]].seg;
    if (segp) rq[q] = segp[rq[q] * sd[tq[q]].seg_stride];
  }
  R x[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const bool okr = rq[q] >= 0 && rq[q] < B;
    bad |= head[q] && !okr;
    if (!okr) rq[q] = -1;
    load_row_u<VEC, G, CPL>(x[q], sd[tq[q]].top_grad + (okr ? rq[q] : 0) * sd[tq[q]].top_stride,
                            lg, dv);
  }
#pragma unroll
  for (int q = 0; q < NB; ++q)
    if (rq[q] < 0) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) x[q].v[c] = vzero<V>();
    }
  if (bad) latch(st, DR_INVALID_ARGUMENT);
  // UnsortedSegmentSum order 0 + x_0 + x_1 ... (sum); x_0 * s + ... (mean/sqrtn);
  // a later chunk's partial starts at its first element
  auto scaled = [&](R& y, const dr_pool_grad_desc& d, int mode, int64_t r) {
    if (mode == 0) return;
    const int32_t cnt = (r >= 0 && d.bag_off) ? d.bag_off[r + 1] - d.bag_off[r] : 1;
    if (cnt != 1) {
      const float sc = mode == 2 ? (float)(1.0 / sqrt((double)cnt)) : (float)(1.0 / (double)cnt);
#pragma unroll
      for (int c = 0; c < CPL; ++c) y.v[c] = vmul(y.v[c], sc);
    }
  };
  auto mode_of = [](const dr_pool_grad_desc& d) {
    return d.combiner == DR_COMBINER_SUM ? 0 : (d.combiner == DR_COMBINER_MEAN ? 1 : 2);
  };
  // weighted: (g / bag_scale[bag]) * w[k]  (RealDiv grad, then Mul grad)
  auto wscaled = [&](R& y, const dr_pool_grad_desc& d, int64_t r, int64_t k) {
    if (d.bag_scale) {
      const float q = d.bag_scale[r >= 0 ? r : 0];
#pragma unroll
      for (int c = 0; c < CPL; ++c) y.v[c] = vdiv(y.v[c], q);
    }
    const float w = d.weights[k];
#pragma unroll
    for (int c = 0; c < CPL; ++c) y.v[c] = vmul(y.v[c], w);
  };
  // the weighted gradient reaches the rows as IndexedSlices -> dense, an
  // UnsortedSegmentSum (0 + x_0 + ...) whatever the combiner
  auto zero_start = [&](const dr_pool_grad_desc& d, int mode) {
    return mode == 0 || (W && d.weights);
  };
  // -- one-position runs (every run of all-distinct ids): the row is loaded.
  // A one-position LAST chunk of a long run is not one of them: it is a
  // partial, left to the chunk path below --
  unsigned multi = 0;
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if (!head[q]) continue;
    if (!single[q] || sq[q] != p0 + q) {
      multi |= 1u << q;
      continue;
    }
    const dr_pool_grad_desc& d = sd[tq[q]];
    const int mode = mode_of(d);
    if (W && d.weights)
      wscaled(x[q], d, rq[q], kq[W ? q : 0]);
    else
      scaled(x[q], d, mode, rq[q]);
    R acc;
    if (zero_start(d, mode)) {   // 0 + x_0 (a chunk head of a one-position run is its run head)
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc.v[c] = vzero<V>();
      acc_add(acc, x[q]);
    } else {
      acc = x[q];
    }
    store_row<VEC, G, CPL>(acc, out + uq[q] * (int64_t)dim, lg, dv);
  }
  // -- chunk heads of longer runs: state re-read from memory so that the
  // per-position arrays above are dead here (register pressure, occupancy) --
  while (multi) {
    const int q = __builtin_ctz(multi);
    multi &= multi - 1;
    const int64_t c0 = p0 + q;          // chunk's first position
    const int64_t u = (int64_t)skey[c0];
    const int t = table_of(g.koff, T, u, ufirst < N ? ufirst : 0);
    const dr_pool_grad_desc& d = sd[t];
    const int mode = mode_of(d);
    const bool first_chunk = c0 == 0 || (int64_t)skey[c0 - 1] != u;
    if (!chunked) {
      // a run longer than one chunk: one serial chain in grad_long_kernel
      if (c0 + kGradChunk < N && (int64_t)skey[c0 + kGradChunk] == u) {
        if (lg == 0) {
          const int32_t at = atomicAdd(nlong, 1);
          longs[2 * at] = (int32_t)u;
          longs[2 * at + 1] = (int32_t)c0;
        }
        continue;
      }
    }
    R acc;
#pragma unroll
    for (int c = 0; c < CPL; ++c) acc.v[c] = vzero<V>();
    bool fresh = !(first_chunk && zero_start(d, mode));
    const int64_t lim = c0 + kGradChunk < N ? c0 + kGradChunk : N;
    const float* tg = d.top_grad;
    const int64_t ts = d.top_stride;
    const int64_t* segp = d.seg;
    const int64_t sst = d.seg_stride;
    const int64_t kt0 = g.koff[t];
    const int64_t nnz_t = d.nnz;
    bool cbad = false;
    for (int64_t p = c0; p < lim; p += kGradChain) {
      R y[kGradChain];
      int64_t ry[kGradChain];
      int64_t ky[W ? kGradChain : 1];
      bool ok[kGradChain];
#pragma unroll
      for (int j = 0; j < kGradChain; ++j) {  // keys and sources: unconditional, clamped
        const int64_t pj = p + j < N ? p + j : N - 1;
        const int64_t kj = (int64_t)skey[pj];
        ok[j] = (p + j < lim) & (kj == u);  // monotone: sorted keys
        const int64_t k = (int64_t)perm[pj] - kt0;
        ry[j] = ((k >= 0) & (k < nnz_t)) ? k : 0;
        if (W) ky[W ? j : 0] = ry[j];
      }
      if (segp) {
#pragma unroll
        for (int j = 0; j < kGradChain; ++j) ry[j] = segp[ry[j] * sst];
      }
#pragma unroll
      for (int j = 0; j < kGradChain; ++j) {
        const bool okr = (ry[j] >= 0) & (ry[j] < B);
        cbad |= ok[j] & !okr;
        ry[j] = okr ? ry[j] : -1;
        load_row_u<VEC, G, CPL>(y[j], tg + (okr ? ry[j] : 0) * ts, lg, dv);
      }
#pragma unroll
      for (int j = 0; j < kGradChain; ++j) {
        if (!ok[j]) break;
        if (ry[j] < 0) {
#pragma unroll
          for (int c = 0; c < CPL; ++c) y[j].v[c] = vzero<V>();
        }
        if (W && d.weights)
          wscaled(y[j], d, ry[j], ky[W ? j : 0]);
        else
          scaled(y[j], d, mode, ry[j]);
        if (fresh) {
          acc = y[j];
          fresh = false;
        } else {
          acc_add(acc, y[j]);
        }
      }
      if (!ok[kGradChain - 1]) break;
    }
    if (cbad) latch(st, DR_INVALID_ARGUMENT);
    if (first_chunk) {
      store_row<VEC, G, CPL>(acc, out + u * (int64_t)dim, lg, dv);
      // (chunked) a run longer than one chunk: queue it for grad_finish_kernel
      if (chunked && lg == 0 && c0 + kGradChunk < N && (int64_t)skey[c0 + kGradChunk] == u) {
        const int32_t at = atomicAdd(nlong, 1);
        longs[2 * at] = (int32_t)u;
        longs[2 * at + 1] = (int32_t)c0;
      }
    } else {
      store_row<VEC, G, CPL>(acc, part + (c0 / kGradChunk) * (int64_t)dim, lg, dv);
    }
  }
}

// out[u] = ((c_0 + c_1) + c_2) + ... for the queued long runs: c_0 is already
// in out[u]; c_k sits in part[start / chunk + k] (consecutive slots).
template <int VEC, int G, int CPL>
__global__ __launch_bounds__(256) void grad_finish_kernel(const uint64_t* __restrict__ skey,
                                                          int64_t N, int dim,
                                                          float* __restrict__ out,
                                                          const float* __restrict__ part,
                                                          const int32_t* __restrict__ longs,
                                                          const int32_t* __restrict__ nlong,
                                                          int64_t nslots) {
  constexpr int GPB = 256 / G;
  const int n = *nlong;
  const int lg = threadIdx.x % G;
  const int dv = dim / VEC;
  using R = Row<VEC, G, CPL>;
  for (int64_t i = (int64_t)blockIdx.x * GPB + threadIdx.x / G; i < n;
       i += (int64_t)gridDim.x * GPB) {
    const int64_t u = longs[2 * i], c0 = longs[2 * i + 1];
    R acc;
    load_row_u<VEC, G, CPL>(acc, out + u * (int64_t)dim, lg, dv);
    const int64_t s0 = c0 / kGradChunk;  // c0's slot; chunk k of the run -> slot s0 + k
    // <= 128 floats of rows in flight per lane
    constexpr int FC = 128 / (VEC * CPL) < 8 ? 8
                       : (128 / (VEC * CPL) > kGradFinishChain ? kGradFinishChain
                                                               : 128 / (VEC * CPL));
    for (int64_t c = c0 + kGradChunk; c < N; c += FC * kGradChunk) {
      R y[FC];
      bool ok[FC];
#pragma unroll
      for (int j = 0; j < FC; ++j) {  // unconditional, clamped loads
        const int64_t cj = c + j * kGradChunk;
        const int64_t kj = (int64_t)skey[cj < N ? cj : N - 1];
        ok[j] = (cj < N) & (kj == u);
        int64_t sl = s0 + 1 + (c - c0 - kGradChunk) / kGradChunk + j;
        sl = sl < nslots ? sl : nslots - 1;
        load_row_u<VEC, G, CPL>(y[j], part + sl * (int64_t)dim, lg, dv);
      }
#pragma unroll
      for (int j = 0; j < FC; ++j)
        if (ok[j]) acc_add(acc, y[j]);
      if (!ok[FC - 1]) break;
    }
    store_row<VEC, G, CPL>(acc, out + u * (int64_t)dim, lg, dv);
  }
}

// Exact long runs of the grouped backward (the default): one block per
// (queued run, column slice of SW columns) sums the WHOLE run in ascending
// position order -- the reference's serial UnsortedSegmentSum /
// SparseSegmentReductionGrad chain (segment_reduction_ops.cc:391-404,
// segment_reduction_ali_ops_util.h:331-458), bit-exact at any length.  The
// run's end is found by 256-way probing of the sorted keys; then stages of S
// positions: all 256 threads load the terms' row slices (the next stage's
// rows in flight while this one is summed), scale them exactly as
// grad_seg_kernel does (mean / sqrtn bag scale, weights) and write them to
// LDS transposed ([column][position]); wave 0 walks each column's chain (one
// lane per column, chain_walk).
template <int VEC, int SW, bool W>
__global__ __launch_bounds__(256) void grad_long_kernel(GradGroup g, int T, int64_t B,
                                                        const uint64_t* __restrict__ skey,
                                                        const int32_t* __restrict__ perm, int dim,
                                                        float* __restrict__ out,
                                                        const int32_t* __restrict__ longs,
                                                        const int32_t* __restrict__ nlong,
                                                        int* st) {
  using V = typename VecT<VEC>::T;
  constexpr int SV = SW / VEC;             // vectors of a position's slice
  constexpr int PI = 256 / SV;             // positions per load instruction
  constexpr int R = VEC == 4 ? 16 : 32;    // loads in flight per thread
  constexpr int S = PI * R;                // positions per stage
  constexpr int SP = S + 4;                // column stride of the transposed stage
  static_assert(SV >= 1 && 256 % SV == 0 && S % 4 == 0, "slice shape");
  __shared__ __attribute__((aligned(16))) float stage[SW * SP];
  __shared__ int smin;
  const int64_t N = g.koff[T];
  const int nsl = (dim + SW - 1) / SW;
  const int64_t total = (int64_t)(*nlong) * nsl;
  const int tid = threadIdx.x;
  const int pv = tid / SV, cv = tid % SV;
  const int lane = tid & 63;
  const int lc = lane < SW ? lane : 0;
  const bool walker = __builtin_amdgcn_readfirstlane(tid >> 6) == 0;
  for (int64_t wi = blockIdx.x; wi < total; wi += gridDim.x) {   // block-uniform
    const int i = (int)(wi / nsl), slice = (int)(wi % nsl);
    const int64_t u = __builtin_amdgcn_readfirstlane(longs[2 * i]);
    const int64_t c0 = __builtin_amdgcn_readfirstlane(longs[2 * i + 1]);
    // run end: lo in the run, hi = N or a position past it (the run is a
    // prefix of [c0, N)); 256 probes per round cover (lo, hi]
    int64_t lo = c0, hi = N;
    while (hi - lo > 1) {
      const int64_t step = (hi - lo - 1 + 255) / 256;
      if (tid == 0) smin = 255;
      __syncthreads();
      const int64_t q = lo + step * (int64_t)(tid + 1);
      if (q >= hi || (int64_t)skey[q] != u) atomicMin(&smin, tid);
      __syncthreads();
      const int m = smin;   // first probe past the run (q_255 >= hi: one exists)
      __syncthreads();
      const int64_t nh = lo + step * (int64_t)(m + 1);
      hi = nh < hi ? nh : hi;
      lo = lo + step * (int64_t)m;
    }
    const int64_t pe = lo + 1;   // one past the run's last position
    const int t = __builtin_amdgcn_readfirstlane(table_of(g.koff, T, u, u));
    const dr_pool_grad_desc& d = g.d[t];
    const int mode = d.combiner == DR_COMBINER_SUM ? 0 : (d.combiner == DR_COMBINER_MEAN ? 1 : 2);
    const bool wt = W && d.weights != nullptr;
    const bool zs = mode == 0 || wt;                  // 0 + x_0 + x_1 ...
    const int colv = slice * SV + cv;                 // this thread's vector column
    const bool colok = colv * VEC < dim;
    const float* tg = d.top_grad + (colok ? colv * VEC : 0);
    const int64_t ts = d.top_stride;
    const int64_t* segp = d.seg;
    const int64_t sst = d.seg_stride;
    const int64_t kt0 = g.koff[t];
    const int64_t nnz_t = d.nnz;
    // bag rows one stage ahead of the row loads; loads clamped to the run
    int64_t rq[R];
    int64_t kk[W ? R : 1];
    bool bad = false;
    auto load_idx = [&](int64_t b0) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        int64_t q = b0 + r * PI + pv;
        q = q < pe ? q : pe - 1;
        const int64_t k = (int64_t)perm[q] - kt0;
        rq[r] = ((k >= 0) & (k < nnz_t)) ? k : 0;
        if (W) kk[W ? r : 0] = rq[r];
      }
      if (segp) {
#pragma unroll
        for (int r = 0; r < R; ++r) rq[r] = segp[rq[r] * sst];
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const bool okr = (rq[r] >= 0) & (rq[r] < B);
        bad |= !okr;
        rq[r] = okr ? rq[r] : -1;
      }
    };
    V y[R];
    int64_t ry[R];
    int64_t ky[W ? R : 1];
    auto load_rows = [&]() {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        ry[r] = rq[r];
        if (W) ky[W ? r : 0] = kk[W ? r : 0];
        y[r] = gld(reinterpret_cast<const V*>(tg + (rq[r] >= 0 ? rq[r] : 0) * ts));
      }
    };
    float acc = 0.f;
    bool fresh = !zs;   // first term: 0 + y (zero-started sum) or y
    load_idx(c0);
    load_rows();
    load_idx(c0 + S);
    for (int64_t b0 = c0; b0 < pe; b0 += S) {
      // y: this stage's rows in flight; rq: the next stage's bag rows
#pragma unroll
      for (int r = 0; r < R; ++r) {
        V x = ry[r] >= 0 ? y[r] : vzero<V>();
        if (wt) {   // (g / bag_scale[bag]) * w[k]
          if (d.bag_scale) x = vdiv(x, d.bag_scale[ry[r] >= 0 ? ry[r] : 0]);
          x = vmul(x, d.weights[ky[W ? r : 0]]);
        } else if (mode != 0) {   // * 1/cnt or 1/sqrt(cnt), scale computed in double
          const int64_t rr = ry[r];
          const int32_t cnt = (rr >= 0 && d.bag_off) ? d.bag_off[rr + 1] - d.bag_off[rr] : 1;
          if (cnt != 1)
            x = vmul(x, mode == 2 ? (float)(1.0 / sqrt((double)cnt)) : (float)(1.0 / (double)cnt));
        }
        // transposed, [column][position]: the walker's column is contiguous
        float* c = stage + (cv * VEC) * SP + r * PI + pv;
        if constexpr (VEC == 4) {
          c[0] = x.x;
          c[SP] = x.y;
          c[2 * SP] = x.z;
          c[3 * SP] = x.w;
        } else if constexpr (VEC == 2) {
          c[0] = x.x;
          c[SP] = x.y;
        } else {
          c[0] = x;
        }
      }
      __syncthreads();
      load_rows();              // the next stage's rows: in flight while wave 0 sums this one
      load_idx(b0 + 2 * S);
      if (walker) {             // wave 0 (an SGPR test: a scalar-controlled walk)
        const int nv = (int)(pe - b0 < S ? pe - b0 : S);
        acc = chain_walk(stage + lc * SP, nv, fresh, acc);
      }
      __syncthreads();   // the stage is rewritten next
    }
    if (bad) latch(st, DR_INVALID_ARGUMENT);
    const int col = slice * SW + lane;
    if (tid < 64 && lane < SW && col < dim) out[u * (int64_t)dim + col] = acc;
  }
}

template <int VEC, int G, int CPL>
static void launch_grad_csr(const GradGroup& g, int T, int64_t B, const uint64_t* skey,
                            const int32_t* perm, int dim, float* out, const GradWs& w,
                            hipStream_t s, int* st) {
  constexpr int NB = 4;
  const int64_t N = g.koff[T];
  hipLaunchKernelGGL(grad_run_start_kernel, dim3((unsigned)ceil_div(N > 0 ? N : 1, 256)),
                     dim3(256), 0, s, skey, N, w.run_start, w.nlong);
  const int64_t blocks = ceil_div(ceil_div(N > 0 ? N : 1, NB), 256 / G);
  bool weighted = false;
  for (int t = 0; t < T; ++t) weighted = weighted || g.d[t].weights;
  // DR_GRAD_CHUNKED=1 (A/B switch): long runs as ordered 256-position chunk
  // partials (deterministic, fp32 tolerance); default: one exact serial chain
  static const int chunked = getenv("DR_GRAD_CHUNKED") ? atoi(getenv("DR_GRAD_CHUNKED")) : 0;
  if (weighted)
    hipLaunchKernelGGL((grad_seg_kernel<VEC, G, CPL, NB, true>), dim3((unsigned)blocks), dim3(256),
                       0, s, g, T, B, skey, perm, w.run_start, dim, out, w.part, w.longs, w.nlong,
                       chunked, st);
  else
    hipLaunchKernelGGL((grad_seg_kernel<VEC, G, CPL, NB, false>), dim3((unsigned)blocks),
                       dim3(256), 0, s, g, T, B, skey, perm, w.run_start, dim, out, w.part,
                       w.longs, w.nlong, chunked, st);
  if (N <= kGradChunk) return;
  if (chunked) {
    hipLaunchKernelGGL((grad_finish_kernel<VEC, G, CPL>), dim3(64), dim3(256), 0, s, skey, N, dim,
                       out, w.part, w.longs, w.nlong, N / kGradChunk + 2);
    return;
  }
  // one block per (long run, slice); an empty list costs one load per block
  constexpr int SWC = 32;
  const int nsl = (dim + SWC - 1) / SWC;
  int64_t gb = (N / (kGradChunk + 1) + 1) * nsl;
  if (gb > 512) gb = 512;
  if (weighted)
    hipLaunchKernelGGL((grad_long_kernel<VEC, SWC, true>), dim3((unsigned)gb), dim3(256), 0, s, g,
                       T, B, skey, perm, dim, out, w.longs, w.nlong, st);
  else
    hipLaunchKernelGGL((grad_long_kernel<VEC, SWC, false>), dim3((unsigned)gb), dim3(256), 0, s,
                       g, T, B, skey, perm, dim, out, w.longs, w.nlong, st);
}

// ---- weighted-lookup divisor and clip_by_norm backward ----------------------
// q[b] = 0 + w_0 + w_1 ... (mean) or sqrtf(0 + w_0^2 + ...) (sqrtn), in the
// weighted forward's order (pool_bag's weighted branch).
__global__ void bag_weight_scale_kernel(const float* __restrict__ w,
                                        const int32_t* __restrict__ off, int64_t B, int combiner,
                                        float* __restrict__ q) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float s = 0.f;
  for (int64_t k = off[b]; k < off[b + 1]; ++k) {
    const float x = w[k];
    s = s + (combiner == DR_COMBINER_SQRTN ? x * x : x);
  }
  q[b] = combiner == DR_COMBINER_SQRTN ? sqrtf(s) : s;
}

// One lane group per row: TF's chain rule through clip_by_norm's ops
// (clip_ops.py:169-179), see dr_clip_by_norm_grad in the header.
template <int VEC, int G, int CPL>
__global__ __launch_bounds__(256) void clip_grad_kernel(const float* __restrict__ pool,
                                                        int64_t pool_rows,
                                                        const int64_t* __restrict__ rows,
                                                        const float* __restrict__ dflt,
                                                        int64_t dstride, const int64_t* n_dev,
                                                        int64_t n, int dim, float c,
                                                        float* __restrict__ grad, int* st) {
  using R = Row<VEC, G, CPL>;
  constexpr int GPB = 256 / G;
  const int64_t i = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
  const bool live = i < eff_n(n, n_dev);
  const int lg = threadIdx.x % G;
  const int dv = dim / VEC;
  const int64_t r = live ? rows[i] : 0;
  const float* src;
  if (r < 0) {
    src = dflt ? dflt + (-r - 1) * dstride : nullptr;
  } else if (r < pool_rows) {
    src = pool + r * (int64_t)dim;
  } else {
    src = nullptr;
  }
  if (live && !src) latch(st, DR_INVALID_ARGUMENT);
  R v, g;
  load_row<VEC, G, CPL>(v, live ? src : nullptr, lg, dv);
  load_row<VEC, G, CPL>(g, live ? grad + i * (int64_t)dim : nullptr, lg, dv);
  // l2sum = reduce_sum(v * v); l2norm = l2sum > 0 ? sqrt(l2sum) : l2sum
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < CPL; ++k) s += vdot(v.v[k]);
  s = group_sum<G>(s);
  const bool pred = s > 0.f;
  const float l2 = pred ? sqrtf(s) : s;
  const float m = l2 > c ? l2 : c;
  // dL/dm = sum_d g * ((-(v * c)) / m) / m   (RealDiv's grad w.r.t. y)
  float gm = 0.f;
  const float* gp = reinterpret_cast<const float*>(&g.v[0]);
  const float* vp = reinterpret_cast<const float*>(&v.v[0]);
#pragma unroll
  for (int k = 0; k < VEC * CPL; ++k) gm += gp[k] * ((-(vp[k] * c) / m) / m);
  gm = group_sum<G>(gm);
  const float gl2 = l2 >= c ? gm : 0.f;             // Maximum: x >= y takes the grad
  const float gs = pred ? (0.5f * gl2) / l2 : 0.f;  // Sqrt grad, where(pred, ...)
  R o;
  float* op = reinterpret_cast<float*>(&o.v[0]);
#pragma unroll
  for (int k = 0; k < VEC * CPL; ++k) {
    const float a = (gp[k] / m) * c;  // values * clip_norm path
    const float b = gs * vp[k];       // values * values path, both factors
    op[k] = (a + b) + b;
  }
  if (live) store_row<VEC, G, CPL>(o, grad + i * (int64_t)dim, lg, dv);
}

}  // namespace dr

// ===========================================================================
extern "C" {

int dr_pool_grouped(const dr_pool_desc* descs_host, int num_tables, int64_t batch, int dim,
                    int order, void* stream) {
  return dr_pool_grouped_ex(descs_host, num_tables, batch, dim, order, 0, stream);
}

int dr_pool_grouped_ex(const dr_pool_desc* descs_host, int num_tables, int64_t batch, int dim,
                       int order, int flags, void* stream) {
  using namespace dr;
  DR_REQUIRE(num_tables >= 1 && num_tables <= DR_MAX_GROUP, DR_INVALID_ARGUMENT,
             "num_tables must be in [1, %d]", DR_MAX_GROUP);
  DR_REQUIRE(batch >= 0 && dim > 0, DR_INVALID_ARGUMENT, "bad batch/dim");
  DR_REQUIRE((flags & ~(DR_POOL_ONEHOT | DR_POOL_BF16 | DR_POOL_OUT_BF16)) == 0,
             DR_INVALID_ARGUMENT, "unknown flags 0x%x", flags);
  if (batch == 0) return DR_OK;
  const bool onehot = flags & DR_POOL_ONEHOT;
  const bool bf16 = flags & DR_POOL_BF16;
  const bool out_bf16 = flags & DR_POOL_OUT_BF16;
  DR_REQUIRE(!bf16 || (dim % 8 == 0 && order == DR_ORDER_ALI), DR_INVALID_ARGUMENT,
             "DR_POOL_BF16 needs dim %% 8 == 0 and the ALI order");
  DR_REQUIRE(!out_bf16 || bf16, DR_INVALID_ARGUMENT, "DR_POOL_OUT_BF16 needs DR_POOL_BF16");
  DR_REQUIRE(!onehot || (int64_t)num_tables * batch < (1ll << 31), DR_INVALID_ARGUMENT,
             "DR_POOL_ONEHOT: tables x batch must be < 2^31");
  PoolArgs a;
  memset(&a, 0, sizeof(a));
  for (int t = 0; t < num_tables; ++t) {
    const dr_pool_desc& d = descs_host[t];
    DR_REQUIRE(d.pool && (d.bag_off || onehot) && d.out && (d.ids || d.idx),
               DR_INVALID_ARGUMENT, "table %d: missing pointers", t);
    DR_REQUIRE(!onehot || (!d.weights && d.max_norm < 0.f), DR_INVALID_ARGUMENT,
               "table %d: DR_POOL_ONEHOT excludes weights and max_norm", t);
    if (dim % 4 == 0)
      DR_REQUIRE(((uintptr_t)d.pool & 15) == 0 && ((uintptr_t)d.out & 15) == 0 &&
                     d.out_stride % 4 == 0 &&
                     (!d.default_rows || ((uintptr_t)d.default_rows & 15) == 0),
                 DR_INVALID_ARGUMENT, "table %d: pool/out must be 16B aligned with stride %% 4", t);
    a.d[t] = d;
    if (bf16) {
      // strides arrive in elements of their type; rows move as float words
      DR_REQUIRE(d.default_stride % 2 == 0 && (!out_bf16 || d.out_stride % 2 == 0),
                 DR_INVALID_ARGUMENT, "table %d: bf16 strides must be even", t);
      a.d[t].default_stride = d.default_stride / 2;
      if (out_bf16) a.d[t].out_stride = d.out_stride / 2;
    }
  }
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  hipStream_t s = S(stream);
  if (bf16)
    return dispatch_pool_bf16(a, num_tables, batch, dim, flags & DR_POOL_ONEHOT, out_bf16, s, st);
  if (order == DR_ORDER_SEQ)
    return dispatch_pool<DR_ORDER_SEQ>(a, num_tables, batch, dim, flags, s, st);
  return dispatch_pool<DR_ORDER_ALI>(a, num_tables, batch, dim, flags, s, st);
}

int dr_bag_offsets(const int64_t* seg, int64_t n, int64_t batch, int32_t* bag_off,
                   void* stream) {
  return dr::launch_bag_offsets<int64_t>(seg, 1, n, nullptr, batch, bag_off, dr::S(stream));
}

int dr_bag_offsets_i32(const int32_t* seg, int64_t n, int64_t batch, int32_t* bag_off,
                       void* stream) {
  return dr::launch_bag_offsets<int32_t>(seg, 1, n, nullptr, batch, bag_off, dr::S(stream));
}

int dr_bag_offsets_grouped(const int64_t* const* seg, const int64_t* stride,
                           const int64_t* n, int num_tables, int64_t batch,
                           int32_t* const* bag_off, void* stream) {
  using namespace dr;
  DR_REQUIRE(num_tables >= 1 && num_tables <= DR_MAX_GROUP, DR_INVALID_ARGUMENT,
             "bad table count");
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  BagGroup g;
  memset(&g, 0, sizeof(g));
  int64_t mx = 0;
  for (int t = 0; t < num_tables; ++t) {
    g.seg[t] = seg[t];
    g.stride[t] = stride[t];
    g.n[t] = n[t];
    g.off[t] = bag_off[t];
    mx = n[t] > mx ? n[t] : mx;
  }
  hipLaunchKernelGGL(bag_zero_grouped_kernel, dim3((unsigned)ceil_div(batch + 1, 256),
                                                   (unsigned)num_tables), dim3(256), 0,
                     S(stream), g, batch);
  dim3 grid((unsigned)ceil_div(mx + 1, 256), (unsigned)num_tables);
  hipLaunchKernelGGL(bag_offsets_grouped_kernel, grid, dim3(256), 0, S(stream), g, batch, st);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_rows_per_nnz(const int64_t* rows, const int32_t* idx, const int64_t* koff_host,
                    int num_tables, int64_t* rowsel, void* stream) {
  using namespace dr;
  DR_REQUIRE(num_tables >= 1 && num_tables <= DR_MAX_GROUP, DR_INVALID_ARGUMENT,
             "bad table count");
  KoffGroup g;
  for (int t = 0; t <= num_tables; ++t) g.koff[t] = koff_host[t];
  const int64_t n = koff_host[num_tables];
  if (n == 0) return DR_OK;
  hipLaunchKernelGGL(rows_per_nnz_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0,
                     S(stream), g, num_tables, rows, idx, rowsel);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

// Strided variant for sp_indices[:, 0] (stride 2), used by the fused ops.
int dr_bag_offsets_strided(const int64_t* seg, int64_t stride, int64_t n, int64_t batch,
                           int32_t* bag_off, void* stream) {
  return dr::launch_bag_offsets<int64_t>(seg, stride, n, nullptr, batch, bag_off, dr::S(stream));
}

int dr_bag_offsets_strided_dev(const int64_t* seg, int64_t stride, int64_t n_cap,
                               const int64_t* n_dev, int64_t batch, int32_t* bag_off,
                               void* stream) {
  return dr::launch_bag_offsets<int64_t>(seg, stride, n_cap, n_dev, batch, bag_off,
                                         dr::S(stream));
}

int dr_gather(const float* table, int64_t rows, int64_t dim, const int64_t* ids, int64_t n,
              float* out, void* stream) {
  using namespace dr;
  DR_REQUIRE(n >= 0 && dim > 0 && dim <= 1024, DR_INVALID_ARGUMENT, "bad gather shape");
  if (n == 0) return DR_OK;
  return gather_dispatch<false>(table, rows, (int)dim, ids, n, out, S(stream), status_word(),
                                nullptr, nullptr);
}

size_t dr_segment_workspace_size(int64_t num_segments) {
  return (size_t)(num_segments + 2) * sizeof(int32_t) + 512;
}

int dr_sparse_segment_reduce(const float* data, int64_t data_rows, int64_t dim,
                             const int32_t* idx, const int32_t* seg, int64_t n,
                             int64_t num_segments, int combiner, float* out, void* ws,
                             size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(ws_bytes >= dr_segment_workspace_size(num_segments), DR_INVALID_ARGUMENT,
             "workspace too small");
  DR_REQUIRE(num_segments >= 0 && dim > 0, DR_INVALID_ARGUMENT, "bad shape");
  if (num_segments == 0) return DR_OK;
  int32_t* off = static_cast<int32_t*>(ws);
  int rc = launch_bag_offsets<int32_t>(seg, 1, n, nullptr, num_segments, off, S(stream));
  if (rc) return rc;
  dr_pool_desc d;
  memset(&d, 0, sizeof(d));
  d.pool = data;
  d.pool_rows = data_rows;
  d.idx = idx;
  d.bag_off = off;
  d.out = out;
  d.out_stride = dim;
  d.combiner = combiner;
  d.max_norm = -1.0f;
  return dr_pool_grouped(&d, 1, num_segments, (int)dim, DR_ORDER_ALI, stream);
}

size_t dr_segment_grad_workspace_size(int64_t n, int64_t grad_rows, int64_t out_rows) {
  size_t used = 0;
  dr::carve_segsum(nullptr, n, out_rows, &used);
  return used + (size_t)(grad_rows + 2) * sizeof(int32_t) + 512;
}

int dr_sparse_segment_reduce_grad(const float* grad, int64_t grad_rows, int64_t dim,
                                  const int32_t* idx, const int32_t* seg, int64_t n,
                                  int64_t out_rows, int combiner, float* out, void* ws,
                                  size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(ws_bytes >= dr_segment_grad_workspace_size(n, grad_rows, out_rows),
             DR_INVALID_ARGUMENT, "workspace too small");
  size_t used = 0;
  carve_segsum(nullptr, n, out_rows, &used);
  int32_t* bag_off = reinterpret_cast<int32_t*>(static_cast<char*>(ws) + ((used + 255) & ~255ul));
  int rc = DR_OK;
  if (combiner != DR_COMBINER_SUM) {
    rc = launch_bag_offsets<int32_t>(seg, 1, n, nullptr, grad_rows, bag_off, S(stream));
    if (rc) return rc;
  }
  const int mode = combiner == DR_COMBINER_SUM ? 0 : (combiner == DR_COMBINER_MEAN ? 1 : 2);
  return segsum_driver(idx, n, out_rows, nullptr, grad, dim, grad_rows, seg,
                       combiner == DR_COMBINER_SUM ? nullptr : bag_off, (int)dim, mode, out, ws,
                       S(stream));
}

size_t dr_unsorted_segment_sum_workspace_size(int64_t n, int64_t num_segments) {
  size_t used = 0;
  dr::carve_segsum(nullptr, n, num_segments, &used);
  return used;
}

int dr_unsorted_segment_sum(const float* data, int64_t n, int64_t dim, const int32_t* seg,
                            int64_t num_segments, float* out, void* ws, size_t ws_bytes,
                            void* stream) {
  using namespace dr;
  DR_REQUIRE(ws_bytes >= dr_unsorted_segment_sum_workspace_size(n, num_segments),
             DR_INVALID_ARGUMENT, "workspace too small");
  return segsum_driver(seg, n, num_segments, nullptr, data, dim, n, nullptr, nullptr, (int)dim, 0,
                       out, ws, S(stream));
}

size_t dr_pool_grad_workspace_size(int64_t n) {
  size_t used = 0;
  dr::carve_segsum(nullptr, n, n, &used);
  return used;
}

size_t dr_pool_grad_grouped_workspace_size(int64_t total_nnz) {
  return ((dr_pool_grad_workspace_size(total_nnz) + 255) & ~size_t(255)) +
         dr::grad_chunk_ws_bytes(total_nnz);
}

int dr_pool_grad_grouped(const dr_pool_grad_desc* descs_host, int num_tables, int64_t batch,
                         int dim, float* grad_unique, void* ws, size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(descs_host && num_tables >= 1 && num_tables <= DR_MAX_GROUP && dim > 0 &&
                 batch >= 0 && grad_unique,
             DR_INVALID_ARGUMENT, "bad argument");
  GradGroup g;
  memset(&g, 0, sizeof(g));
  g.koff[0] = 0;
  bool aligned = dim % 4 == 0 && ((uintptr_t)grad_unique & 15) == 0;
  for (int t = 0; t < num_tables; ++t) {
    const dr_pool_grad_desc& d = descs_host[t];
    DR_REQUIRE(d.top_grad && d.idx && d.num_unique && d.nnz >= 0, DR_INVALID_ARGUMENT,
               "table %d: missing pointers", t);
    DR_REQUIRE(d.combiner == DR_COMBINER_SUM || d.bag_off || !d.seg, DR_INVALID_ARGUMENT,
               "table %d: mean/sqrtn of multi-hot bags need bag_off", t);
    DR_REQUIRE(!d.weights || d.combiner == DR_COMBINER_SUM || d.bag_scale, DR_INVALID_ARGUMENT,
               "table %d: weighted mean/sqrtn needs bag_scale (dr_bag_weight_scale)", t);
    g.d[t] = d;
    g.koff[t + 1] = g.koff[t] + d.nnz;
    aligned = aligned && ((uintptr_t)d.top_grad & 15) == 0 && d.top_stride % 4 == 0;
  }
  const int64_t n = g.koff[num_tables];
  DR_REQUIRE(n < (1ll << 31), DR_INVALID_ARGUMENT, "too many nnz");
  DR_REQUIRE(batch > 0 || n == 0, DR_INVALID_ARGUMENT, "nnz without a batch");
  DR_REQUIRE(ws_bytes >= dr_pool_grad_grouped_workspace_size(n), DR_INVALID_ARGUMENT,
             "workspace too small");
  if (n == 0) return DR_OK;
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  hipStream_t s = S(stream);
  SegSumWs w = carve_segsum(ws, n, n, nullptr);
  GradWs gw;
  gw.run_start = w.off;
  gw.nlong = w.off + n + 1;
  {
    size_t seg_used = 0;
    carve_segsum(nullptr, n, n, &seg_used);
    Carver c(static_cast<char*>(ws) + ((seg_used + 255) & ~size_t(255)));
    const int64_t chunks = n / kGradChunk + 2;
    gw.longs = c.take<int32_t>(2 * chunks);
    gw.part = c.take<float>(chunks * kGradMaxDim);
  }
  DR_REQUIRE(dim <= kGradMaxDim, DR_INVALID_ARGUMENT, "dim %d unsupported", dim);
  hipLaunchKernelGGL(grad_keys_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, g,
                     num_tables, w.kin, w.vin, st);
  DR_LAUNCH_CHECK();
  int rc = dr_sort_pairs(w.kin, w.vin, w.kout, w.perm, n, 0, bits_for(n), w.sort_ws,
                         w.sort_bytes, stream);
  if (rc) return rc;
  if (aligned) {
    const int d4 = dim / 4;
    if (d4 <= 8)
      launch_grad_csr<4, 8, 1>(g, num_tables, batch, w.kout, w.perm, dim, grad_unique, gw, s,
                                st);
    else if (d4 <= 16)
      launch_grad_csr<4, 16, 1>(g, num_tables, batch, w.kout, w.perm, dim, grad_unique, gw, s,
                                st);
    else if (d4 <= 32)
      launch_grad_csr<4, 32, 1>(g, num_tables, batch, w.kout, w.perm, dim, grad_unique, gw, s,
                                st);
    else if (d4 <= 64)
      launch_grad_csr<4, 64, 1>(g, num_tables, batch, w.kout, w.perm, dim, grad_unique, gw, s,
                                st);
    else if (d4 <= 256)
      launch_grad_csr<4, 64, 4>(g, num_tables, batch, w.kout, w.perm, dim, grad_unique, gw, s,
                                st);
    else
      DR_REQUIRE(false, DR_INVALID_ARGUMENT, "dim %d unsupported", dim);
  } else {
    if (dim <= 64)
      launch_grad_csr<1, 64, 1>(g, num_tables, batch, w.kout, w.perm, dim, grad_unique, gw, s,
                                st);
    else if (dim <= 256)
      launch_grad_csr<1, 64, 4>(g, num_tables, batch, w.kout, w.perm, dim, grad_unique, gw, s,
                                st);
    else
      DR_REQUIRE(false, DR_INVALID_ARGUMENT, "dim %d unsupported", dim);
  }
  DR_LAUNCH_CHECK();
  return DR_OK;
}

// Backward of dr_pool_grouped (ORDER_ALI / TF grad semantics) for one table:
// gradient per unique row, deterministic.  seg[k] = bag of position k,
// idx[k] = unique position; rows past *num_unique are not written.
int dr_pool_grad(const float* top_grad, int64_t top_stride, int64_t batch, int dim,
                 const int32_t* bag_off, const int32_t* seg, const int32_t* idx, int64_t n,
                 const int64_t* num_unique, int combiner, float* grad_unique, void* ws,
                 size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(ws_bytes >= dr_pool_grad_workspace_size(n), DR_INVALID_ARGUMENT,
             "workspace too small");
  const int mode = combiner == DR_COMBINER_SUM ? 0 : (combiner == DR_COMBINER_MEAN ? 1 : 2);
  return segsum_driver(idx, n, n, num_unique, top_grad, top_stride, batch, seg,
                       combiner == DR_COMBINER_SUM ? nullptr : bag_off, dim, mode, grad_unique,
                       ws, S(stream));
}

int dr_bag_weight_scale(const float* weights, const int32_t* bag_off, int64_t batch, int combiner,
                        float* bag_scale, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && (batch == 0 || (weights && bag_off && bag_scale)), DR_INVALID_ARGUMENT,
             "dr_bag_weight_scale: missing pointers");
  if (batch == 0) return DR_OK;
  hipLaunchKernelGGL(bag_weight_scale_kernel, dim3((unsigned)ceil_div(batch, 256)), dim3(256), 0,
                     S(stream), weights, bag_off, batch, combiner, bag_scale);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_clip_by_norm_grad(const float* pool, int64_t pool_rows, const int64_t* rows,
                         const float* default_rows, int64_t default_stride, const int64_t* n_dev,
                         int64_t n, int dim, float max_norm, float* grad, void* stream) {
  using namespace dr;
  DR_REQUIRE(n >= 0 && dim > 0 && dim <= 1024 && (n == 0 || (pool && rows && grad)),
             DR_INVALID_ARGUMENT, "dr_clip_by_norm_grad: bad arguments");
  if (n == 0) return DR_OK;
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  hipStream_t s = S(stream);
  const bool al = dim % 4 == 0 && ((uintptr_t)grad & 15) == 0 && ((uintptr_t)pool & 15) == 0 &&
                  (!default_rows || (((uintptr_t)default_rows & 15) == 0 && default_stride % 4 == 0));
#define DR_CLIPG(V, G, C)                                                                      \
  do {                                                                                         \
    hipLaunchKernelGGL((clip_grad_kernel<V, G, C>), dim3((unsigned)ceil_div(n, 256 / G)),    \
                       dim3(256), 0, s, pool, pool_rows, rows, default_rows, default_stride,  \
                       n_dev, n, dim, max_norm, grad, st);                                     \
    DR_LAUNCH_CHECK();                                                                         \
    return DR_OK;                                                                              \
  } while (0)
  if (al) {
    const int d4 = dim / 4;
    if (d4 <= 8) DR_CLIPG(4, 8, 1);
    if (d4 <= 16) DR_CLIPG(4, 16, 1);
    if (d4 <= 32) DR_CLIPG(4, 32, 1);
    if (d4 <= 64) DR_CLIPG(4, 64, 1);
    DR_CLIPG(4, 64, 4);
  }
  if (dim <= 64) DR_CLIPG(1, 64, 1);
  if (dim <= 256) DR_CLIPG(1, 64, 4);
  DR_CLIPG(1, 64, 16);
#undef DR_CLIPG
}

}  // extern "C"
