/*
 * deeprec_amd.h -- C ABI of the MI355X-native sharded-embedding engine.
 *
 * This is the drop-in boundary for DeepRec's EmbeddingVariable /
 * embedding_lookup_sparse hot path.  Each entry point
 * names the reference op/kernel it replaces (paths relative to the DeepRec
 * reference root).  Conventions:
 *   - every buffer argument is a caller-owned DEVICE pointer unless its name
 *     ends in `_host`; `stream` is a hipStream_t passed as void*;
 *   - EmbeddingVariables are library-owned, refcounted opaque handles
 *     (ResourceMgr + core::ScopedUnref in the reference);
 *   - return value is a TF error::Code (DR_OK == 0); dr_last_error() returns
 *     a thread-local message for the last failure on this thread;
 *   - data-dependent errors found on the device (index out of range,
 *     unsorted segment ids, table full) are latched in a device status word
 *     and reported by dr_status_check() (which synchronises the stream), so
 *     that the hot entry points never block the host;
 *   - no call aborts the process;
 *   - entry points taking `ws`/`ws_bytes` need a device workspace of at least
 *     the size returned by the matching *_workspace_size() query;
 *   - nothing here allocates device memory or synchronises except the
 *     functions documented as such (create/reserve/size/export/status), so
 *     the per-step calls can be captured into a hipGraph.
 */
#ifndef DEEPREC_AMD_H_
#define DEEPREC_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* TF error::Code values (tensorflow/core/lib/core/error_codes.proto). */
enum {
  DR_OK = 0,
  DR_INVALID_ARGUMENT = 3,
  DR_NOT_FOUND = 5,
  DR_ALREADY_EXISTS = 6,
  DR_RESOURCE_EXHAUSTED = 8,
  DR_INTERNAL = 13
};

/* Combiners of embedding_lookup_sparse / SparseSegment{Sum,Mean,SqrtN}. */
enum { DR_COMBINER_SUM = 0, DR_COMBINER_MEAN = 1, DR_COMBINER_SQRTN = 2 };

/* Pooling association order.
 * DR_ORDER_ALI  : SparseSegmentReduction::Reduce CPU order
 *                 (core/kernels/segment_reduction_ali_ops_util.h:193-318)
 * DR_ORDER_SEQ  : left-to-right then combiner, FusedEmbeddingLocalSparseLookUp
 *                 (core/kernels/fused_embedding/fused_embedding_local_ops_gpu.cu.cc:41-84) */
enum { DR_ORDER_ALI = 0, DR_ORDER_SEQ = 1 };

int dr_abi_version(void);
const char* dr_last_error(void);
/* Synchronises `stream`, returns and clears the device status word
 * (DR_OK or the first DR_* code latched by a kernel since the last check). */
int dr_status_check(void* stream);

/* ------------------------------------------------------------------------ */
/* Unique / UniqueWithCounts, first-occurrence order.                        */
/* Replaces UniqueAliOp (core/kernels/unique_ali_op.cc:46-180,               */
/* unique_ali_op_util.h:192-222).  num_unique is a DEVICE int64.             */
/* ------------------------------------------------------------------------ */
size_t dr_unique_workspace_size(int64_t n);
int dr_unique(const int64_t* keys, int64_t n, int64_t* uniq_out, int32_t* idx_out,
              int32_t* counts_out /* nullable */, int64_t* num_unique,
              void* ws, size_t ws_bytes, void* stream);
/* The same for T features in one pass: feature t owns keys                 */
/* [koff_host[t], koff_host[t+1]); its uniques / counts are written at the  */
/* same offset, idx is feature-local, num_unique[t] (DEVICE) = U_t.         */
size_t dr_unique_grouped_workspace_size(const int64_t* koff_host, int num_tables);
int dr_unique_grouped(const int64_t* keys, const int64_t* koff_host, int num_tables,
                      int64_t* uniq_out, int32_t* idx_out, int32_t* counts_out,
                      int64_t* num_unique, void* ws, size_t ws_bytes, void* stream);
/* Test hook: bound of the per-bucket LDS hash walk before a key goes to the */
/* bucket's global overflow region (default and maximum 2048; a smaller     */
/* value makes small inputs take the overflow path).  Results never change. */
int dr_unique_set_lds_probes(int probes);

/* Measurement hook (bench.py): dr_kernel_timing(which) clears the record and */
/* brackets every later launch of one kernel with a pair of HIP events on the */
/* launch's stream (1: the fused lookup kernel of dr_ev_lookup_onehot*, 2: the */
/* one-hot pooling kernel of dr_pool_grouped_ex; 0: off).  Not for use inside */
/* graph capture.  dr_kernel_timing_result syncs and returns the summed        */
/* kernel time (ms) and the number of bracketed launches.                     */
int dr_kernel_timing(int which);
int dr_kernel_timing_result(double* total_ms, int64_t* launches);

/* ------------------------------------------------------------------------ */
/* Stable radix sort of (uint64 key, int32 value) pairs on bits [lo, hi).    */
/* Replaces cub::DeviceRadixSort::SortPairs in FusedEmbeddingSparsePreLookUp */
/* (core/kernels/fused_embedding/fused_embedding_ops_gpus.cu.cc:192-212).    */
/* ------------------------------------------------------------------------ */
size_t dr_sort_pairs_workspace_size(int64_t n);
int dr_sort_pairs(const uint64_t* keys_in, const int32_t* vals_in, uint64_t* keys_out,
                  int32_t* vals_out, int64_t n, int bit_lo, int bit_hi,
                  void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------ */
/* Dense-table row gather: ResourceGather / GatherV2                         */
/* (core/kernels/resource_variable_ops.cc:628, gather_functor.h:36-115).     */
/* Out-of-range ids latch DR_INVALID_ARGUMENT and write zeros.               */
/* ------------------------------------------------------------------------ */
int dr_gather(const float* table, int64_t rows, int64_t dim, const int64_t* ids,
              int64_t n, float* out, void* stream);

/* ------------------------------------------------------------------------ */
/* SparseSegment{Sum,Mean,SqrtN}[WithNumSegments] over a materialised       */
/* [data_rows, dim] input (segment_reduction_ali_ops.cc:141-250).  seg must */
/* be sorted; missing segments are 0.                                        */
/* ------------------------------------------------------------------------ */
size_t dr_segment_workspace_size(int64_t num_segments);
int dr_sparse_segment_reduce(const float* data, int64_t data_rows, int64_t dim,
                             const int32_t* idx, const int32_t* seg, int64_t n,
                             int64_t num_segments, int combiner, float* out,
                             void* ws, size_t ws_bytes, void* stream);

/* SparseSegment{Sum,Mean,SqrtN}Grad in the CPU order (ascending i per       */
/* output row; segment_reduction_ali_ops_util.h:331-458, and for Sum the    */
/* math_grad.py:321-327 unsorted_segment_sum composition).  Deterministic.   */
size_t dr_segment_grad_workspace_size(int64_t n, int64_t grad_rows, int64_t out_rows);
int dr_sparse_segment_reduce_grad(const float* grad, int64_t grad_rows, int64_t dim,
                                  const int32_t* idx, const int32_t* seg, int64_t n,
                                  int64_t out_rows, int combiner, float* out,
                                  void* ws, size_t ws_bytes, void* stream);

/* UnsortedSegmentSum (segment_reduction_ops.cc:377-405): serial ascending-i */
/* order per output row, seg < 0 skipped.  Deterministic (no float atomics). */
size_t dr_unsorted_segment_sum_workspace_size(int64_t n, int64_t num_segments);
int dr_unsorted_segment_sum(const float* data, int64_t n, int64_t dim, const int32_t* seg,
                            int64_t num_segments, float* out, void* ws, size_t ws_bytes,
                            void* stream);

/* ------------------------------------------------------------------------ */
/* Grouped fused lookup + pooling: one launch for up to DR_MAX_GROUP tables  */
/* (features).  For table t, bag b of batch B: rows L_k = pool[row(k)] for   */
/* k in [bag_off[b], bag_off[b+1]), reduced in `order` with `combiner` (and */
/* per-row clip_by_norm when max_norm > 0), written to                       */
/* out[b * out_stride + d].  Row selection per nnz k:                        */
/*   idx == NULL : row = ids[k]              (dense table, bounds-checked)   */
/*   idx != NULL : row = rows[idx[k]]        (EV resolved unique rows);      */
/*                 row < 0 -> default_rows[-row-1] (filtered / not admitted) */
/* Empty bags are 0 (gap fill), or zero_empty==0 keeps the same.             */
/* This is the fused embedding_lookup_sparse forward                        */
/* (python/ops/embedding_ops.py:480-675) minus the dedup/resolve steps.      */
/* ------------------------------------------------------------------------ */
#define DR_MAX_GROUP 32
typedef struct {
  const float* pool;          /* table or EV value pool base, [rows, dim]  */
  int64_t pool_rows;          /* bounds for dense ids                       */
  const int64_t* ids;         /* dense: [nnz] row ids                       */
  const int32_t* idx;         /* EV: [nnz] -> unique position (or NULL)     */
  const int64_t* rows;        /* EV: [U] resolved row per unique key        */
  const float* default_rows;  /* EV: rows for negative selections           */
  int64_t default_stride;     /* elements between default rows (0: one row) */
  const int32_t* bag_off;     /* [B+1] CSR offsets of the bags              */
  const float* weights;       /* [nnz] sp_weights or NULL                   */
  float* out;                 /* [B, out_stride] output                     */
  int64_t out_stride;
  int32_t combiner;
  float max_norm;             /* >= 0: clip rows (clip_by_norm for ALI order,
                                 fused `*= max_norm/l2` for SEQ); -1: off     */
} dr_pool_desc;

int dr_pool_grouped(const dr_pool_desc* descs_host, int num_tables, int64_t batch,
                    int dim, int order, void* stream);
/* Same with flags.  DR_POOL_ONEHOT: the caller guarantees bag b holds      */
/* exactly nnz b (one id per row, nnz == batch, e.g. Criteo categorical      */
/* features); bag_off may be NULL and is not read; weights must be NULL and  */
/* max_norm < 0.  Results are identical to dr_pool_grouped on such input.    */
#define DR_POOL_ONEHOT 1
/* DR_POOL_BF16: the pools (and default rows) hold bf16 values (a bf16 EV,  */
/* value_bits 16); `dim` counts values (multiple of 8); default_stride      */
/* counts bf16 elements.  The output is fp32 (the reference casts bf16      */
/* embeddings to float32 before pooling, embedding_ops.py:606-607) unless   */
/* DR_POOL_OUT_BF16, when it is bf16 (out_stride in bf16 elements): bags of */
/* one id are then bitwise copies, longer bags / weights / max_norm pool in */
/* fp32 (ALI order) and round once to nearest even.  ALI order only.        */
#define DR_POOL_BF16 2
#define DR_POOL_OUT_BF16 4
int dr_pool_grouped_ex(const dr_pool_desc* descs_host, int num_tables, int64_t batch,
                       int dim, int order, int flags, void* stream);

/* CSR bag offsets from sorted segment ids (sp_indices[:,0]):               */
/* bag_off[s] = first k with seg[k] >= s, bag_off[B] = n.  Unsorted or out  */
/* of range ids latch DR_INVALID_ARGUMENT.                                   */
int dr_bag_offsets(const int64_t* seg, int64_t n, int64_t batch, int32_t* bag_off,
                   void* stream);
int dr_bag_offsets_i32(const int32_t* seg, int64_t n, int64_t batch, int32_t* bag_off,
                       void* stream);
/* Grouped over T features in one launch (seg[t] read with stride[t]).      */
int dr_bag_offsets_grouped(const int64_t* const* seg, const int64_t* stride,
                           const int64_t* n, int num_tables, int64_t batch,
                           int32_t* const* bag_off, void* stream);
/* rowsel[i] = rows[koff[t] + idx[i]] for nnz i of feature t (grouped-unique */
/* layout): pre-resolves every nnz to its EV row for dr_pool_grouped (set   */
/* desc.ids = rowsel, desc.default_rows for negative = filtered rows).       */
int dr_rows_per_nnz(const int64_t* rows, const int32_t* idx, const int64_t* koff_host,
                    int num_tables, int64_t* rowsel, void* stream);
/* Same over sp_indices[:, 0] read with a stride (2 for [nnz, 2] indices).   */
int dr_bag_offsets_strided(const int64_t* seg, int64_t stride, int64_t n, int64_t batch,
                           int32_t* bag_off, void* stream);
/* The same over a DEVICE count n_dev (<= n_cap), e.g. the filled output of */
/* dr_sparse_prune_fill: no host read of the entry count.                   */
int dr_bag_offsets_strided_dev(const int64_t* seg, int64_t stride, int64_t n_cap,
                               const int64_t* n_dev, int64_t batch, int32_t* bag_off,
                               void* stream);

/* Backward of dr_pool_grouped over T features in one pass (the features of */
/* one dr_unique_grouped call): grad_unique row koff[t] + u (koff = prefix  */
/* sums of nnz) = sum over nnz k of feature t with idx[k] == u, ascending k, */
/* of top_grad_t[bag(k)] scaled like dr_pool_grad.  bag(k) = seg[k *         */
/* seg_stride] (sp_indices[:, 0] read in place), or k when seg == NULL       */
/* (one-hot).  Rows u >= num_unique[t] are not written.  Deterministic; the  */
/* per-feature math equals dr_pool_grad / SparseSegment*Grad.                */
typedef struct {
  const float* top_grad;      /* feature t's [B, dim] slice of the pooled grad */
  int64_t top_stride;
  const int32_t* bag_off;     /* [B+1]; NULL for one-hot                      */
  const int64_t* seg;         /* NULL for one-hot                             */
  int64_t seg_stride;
  const int32_t* idx;         /* [nnz] feature-local unique position          */
  int64_t nnz;
  const int64_t* num_unique;  /* DEVICE U_t                                   */
  int32_t combiner;
  /* Weighted lookups (embedding_ops.py:609-651: gather * w -> segment_sum   */
  /* -> / weight_sum): NULL, or sp_weights [nnz].  Position k contributes    */
  /* (top_grad[bag] / bag_scale[bag]) * weights[k] (mean / sqrtn; bag_scale  */
  /* from dr_bag_weight_scale) or top_grad[bag] * weights[k] (sum), summed    */
  /* from 0 in ascending k (the IndexedSlices -> dense unsorted_segment_sum). */
  const float* weights;
  const float* bag_scale;     /* [B] per-bag divisor, NULL for sum          */
} dr_pool_grad_desc;

/* bag_scale[b] = sum of weights (mean) or sqrtf(sum of weights^2) (sqrtn)  */
/* over bag b, accumulated from 0 in ascending position (math_ops.          */
/* segment_sum(weights) / segment_sum(pow(weights, 2)), embedding_ops.py:    */
/* 636-645); the divisor of the weighted forward and of its backward.        */
int dr_bag_weight_scale(const float* weights, const int32_t* bag_off, int64_t batch, int combiner,
                        float* bag_scale, void* stream);

/* Backward of clip_by_norm (embedding_ops._clip -> clip_ops.py:164-184),    */
/* in place on grad [n, dim] (n_dev: DEVICE row count or NULL): row i of the */
/* clipped values came from v = pool[rows[i]] (rows[i] < 0: default_rows +   */
/* (-rows[i]-1) * default_stride, an EV default).  With m = max(l2, c):      */
/* grad = (g / m) * c + 2 * (s * v), s = (0.5 * sum_d(g * ((-(v * c)) / m) / */
/* m)) / l2 when l2 >= c and l2 > 0, else 0 -- TF's op-by-op chain rule     */
/* (RealDiv, Maximum(x >= y), Sqrt, Mul).  Row sums in wave order: fp32     */
/* tolerance, not bit-exact.                                                */
int dr_clip_by_norm_grad(const float* pool, int64_t pool_rows, const int64_t* rows,
                         const float* default_rows, int64_t default_stride, const int64_t* n_dev,
                         int64_t n, int dim, float max_norm, float* grad, void* stream);
size_t dr_pool_grad_grouped_workspace_size(int64_t total_nnz);
int dr_pool_grad_grouped(const dr_pool_grad_desc* descs_host, int num_tables, int64_t batch,
                         int dim, float* grad_unique, void* ws, size_t ws_bytes, void* stream);

/* Grouped backward keyed by the forward's rows (filter-free EVs resolved    */
/* without Unique: dr_ev_resolve_grouped with counts == NULL).  rowsel[i] =  */
/* the row of nnz i (koff order, every row < row_limit; a negative row -- a  */
/* default served on an exhausted pool -- gets no gradient), keys[i] its id. */
/* Same results as dr_unique_grouped -> dr_pool_grad_grouped: uniq_out[koff  */
/* [t] + u] = table t's unique ids in first-occurrence order (Unique's       */
/* order), num_unique[t] (DEVICE) = U_t, and the gradient of unique u is     */
/* the ascending-position SparseSegment*Grad sum (bit-exact for runs of up   */
/* to 256 positions; longer runs: ordered chunk partials, fp32 tolerance).   */
/* The gradient is returned BY ADDRESS: grad_ptr[koff[t] + u] = address of   */
/* its fp32 row, bit 0 = use as 0.0f + g.  defer != 0: an unscaled           */
/* one-position gradient points straight into top_grad (nothing written);   */
/* every other row is written to grad_unique[koff[t] + u] and points there.  */
/* desc.idx / desc.num_unique are unused.  grad_unique 16-byte aligned when  */
/* dim % 4 == 0.  dr_rows_from_ptr materialises the values.                  */
size_t dr_pool_grad_rows_workspace_size(int64_t total_nnz);
int dr_pool_grad_rows_grouped(const dr_pool_grad_desc* descs_host, int num_tables, int64_t batch,
                              int dim, const int64_t* rowsel, int64_t row_limit,
                              const int64_t* keys, int defer, int64_t* uniq_out,
                              int64_t* num_unique, uint64_t* grad_ptr, float* grad_unique,
                              void* ws, size_t ws_bytes, void* stream);
/* The same, also writing uniq_rows[o] = the row the forward resolved unique */
/* id o to (rowsel at its first position; NULL: not written).               */
int dr_pool_grad_rows_grouped_ex(const dr_pool_grad_desc* descs_host, int num_tables,
                                 int64_t batch, int dim, const int64_t* rowsel, int64_t row_limit,
                                 const int64_t* keys, int defer, int64_t* uniq_out,
                                 int64_t* uniq_rows, int64_t* num_unique, uint64_t* grad_ptr,
                                 float* grad_unique, void* ws, size_t ws_bytes, void* stream);
/* rows_record = 1: rowsel is the record-major [batch, T] of a one-hot      */
/* training lookup with DR_LOOKUP_ROWS_RECORD (every feature nnz == batch). */
int dr_pool_grad_rows_grouped_ex2(const dr_pool_grad_desc* descs_host, int num_tables,
                                  int64_t batch, int dim, const int64_t* rowsel, int rows_record,
                                  int64_t row_limit, const int64_t* keys, int defer,
                                  int64_t* uniq_out, int64_t* uniq_rows, int64_t* num_unique,
                                  uint64_t* grad_ptr, float* grad_unique, void* ws,
                                  size_t ws_bytes, void* stream);
/* out[i] = row at grad_ptr[i] (+0.0f first when bit 0 is set) for i <      */
/* min(n, *n_dev) (n_dev DEVICE or NULL); later rows are not written.        */
int dr_rows_from_ptr(const uint64_t* grad_ptr, int64_t n, const int64_t* n_dev, int dim,
                     float* out, void* stream);

/* Backward of the grouped pooling for one table, deterministic:             */
/* grad_unique[u] = sum over k with idx[k]==u (ascending k) of               */
/*   top_grad[bag(k)] * scale(bag)  (scale: 1, 1/n, 1/sqrt(n) as the         */
/* reference grad kernels compute it).  = SparseSegment*Grad on the unique  */
/* rows.  num_unique is a DEVICE int64 (upper bound n).                      */
size_t dr_pool_grad_workspace_size(int64_t n);
int dr_pool_grad(const float* top_grad, int64_t top_stride, int64_t batch, int dim,
                 const int32_t* bag_off, const int32_t* seg, const int32_t* idx, int64_t n,
                 const int64_t* num_unique, int combiner, float* grad_unique,
                 void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------ */
/* EmbeddingVariable (core/framework/embedding/embedding_var.h:50-363).      */
/* ------------------------------------------------------------------------ */
typedef struct dr_ev dr_ev;

typedef struct {
  int64_t dim;                       /* value_len                           */
  int64_t capacity;                  /* initial key capacity (grows)        */
  int64_t steps_to_live;             /* >0: versions kept                   */
  int64_t filter_freq;               /* >0: Counter (or Bloom) admission    */
  int64_t max_element_size;          /* Bloom sizing (with fpp)             */
  float false_positive_probability;  /* -1: Counter filter                  */
  int32_t counter_bits;              /* Bloom counter width 8/16/32/64      */
  int32_t layout;                    /* 0 light, 1 normal (informational)   */
  int32_t value_bits;                /* 32 (float, default when 0) or 64:    */
                                     /* double EVs (KvResourceGather's V =   */
                                     /* double, kv_variable_ops.cc:368-388)  */
                                     /* support gather / insert / export;   */
                                     /* default rows / values / outputs are */
                                     /* doubles; the applies and pooled     */
                                     /* lookups are float-only (INVALID_ARG) */
                                     /* or 16: bf16 EV (build-defined, the  */
                                     /* BASELINE configs[4] DCN-v2 tables;  */
                                     /* the reference registers float and   */
                                     /* double only): the primary column    */
                                     /* holds bf16 rows (default_row_host is */
                                     /* fp32, rounded to nearest even); slot */
                                     /* columns (optimizer state) stay fp32; */
                                     /* gather / insert / export values and  */
                                     /* one-hot lookup outputs are bf16;     */
                                     /* applies (SGD / Adagrad / Adam /      */
                                     /* AdamAsync / AdagradDecay, not FTRL)  */
                                     /* take fp32 gradients and round the    */
                                     /* updated value once to bf16           */
} dr_ev_config;

/* InitializeKvVariableOp primary branch (kernels/kv_variable_ops.cc:173-193). */
int dr_ev_create(const dr_ev_config* cfg, const float* default_row_host, dr_ev** out);
/* Slot EV sharing the primary's key space (kv_variable_ops.cc:212-226).    */
int dr_ev_create_slot(dr_ev* primary, int slot_index, const float* default_row_host,
                      dr_ev** out);
int dr_ev_retain(dr_ev* ev);
int dr_ev_release(dr_ev* ev);
/* 16 (bf16 primary column), 32 (float) or 64 (double) */
int dr_ev_value_bits(dr_ev* ev);
/* use_locking = true of the KV applies (training_ali_ops.cc:104,141,161,   */
/* 198,217; MaybeLockEmbeddingVariableInputMutexesInOrder, training_ali_op_ */
/* helpers.h:85-118): bracket the apply calls.  lock takes the EVs' update  */
/* mutexes in address order and makes `stream` wait for the previous locked */
/* update of each EV (on any stream); unlock records this stream's point    */
/* and releases them.  Without them updates from several streams race, as  */
/* the reference's use_locking = false.                                     */
int dr_ev_lock_updates(dr_ev* const* vars, int n, void* stream);
int dr_ev_unlock_updates(dr_ev* const* vars, int n, void* stream);

/* int32-key forms of the key-taking entry points (the reference registers  */
/* KvResourceGather / Import / Export and Unique for int32 and int64 keys,  */
/* kv_variable_ops.cc:368-388, unique_ali_op.cc): keys are widened on the  */
/* device (the key value is the same), outputs narrowed back.  defaults /   */
/* values / out are float or double per the EV's value_bits.                */
size_t dr_ev_gather_i32_workspace_size(int64_t n);
int dr_ev_gather_i32(dr_ev* ev, const int32_t* keys, int64_t n, const void* defaults,
                     const int32_t* counts, void* out, void* ws, size_t ws_bytes, void* stream);
int dr_ev_insert_i32(dr_ev* ev, const int32_t* keys, int64_t n, const void* values,
                     const int64_t* versions, const int64_t* freqs, int64_t partition_id,
                     int64_t partition_num, void* stream);
int dr_ev_export_i32(dr_ev* ev, int32_t* keys_out, void* values_out, int64_t* versions_out,
                     int64_t* freqs_out, int64_t capacity, int64_t* m_host, void* stream);
size_t dr_unique_i32_workspace_size(int64_t n);
int dr_unique_i32(const int32_t* keys, int64_t n, int32_t* uniq_out, int32_t* idx_out,
                  int32_t* counts_out /* nullable */, int64_t* num_unique, void* ws,
                  size_t ws_bytes, void* stream);
/* KvVariableShapeOp (kv_variable_ops.cc:58-75): number of keys.  Syncs.   */
int dr_ev_size(dr_ev* ev, int64_t* size_host, void* stream);
/* Save-time eviction EmbeddingVar::Shrink (embedding_var.h:264-313), as     */
/* DumpEv runs it before a save (save_restore_v2_ops.cc:128-131):            */
/* l2_weight_threshold != -1 drops keys with 0.5 * |row|^2 < threshold; else  */
/* with steps_to_live > 0, version -1 becomes global_step and keys with      */
/* global_step - version > steps_to_live are dropped.  Synchronises;         */
/* *removed_host (nullable) = keys dropped.                                   */
int dr_ev_shrink(dr_ev* ev, int64_t global_step, float l2_weight_threshold,
                 int64_t* removed_host, void* stream);
int64_t dr_ev_dim(dr_ev* ev);
/* filter_freq of the EV's Counter / Bloom admission filter (0: none).        */
int64_t dr_ev_filter_freq(dr_ev* ev);
/* Row-pool capacity of the EV's key space (host value, no sync): every row  */
/* index the EV has handed out is below it (the row_limit of                 */
/* dr_pool_grad_rows_grouped).                                               */
int64_t dr_ev_row_capacity(dr_ev* ev);
/* Ensures room for `extra` new keys (may rehash/grow; syncs when it must). */
int dr_ev_reserve(dr_ev* ev, int64_t extra, void* stream);

/* Resolve keys to value-pool rows with insert-on-miss and the filter,       */
/* initialising first-touch rows from `defaults` ([n,dim], or NULL = the EV */
/* default).  rows_out[i] = row, or -(i+1) when the key is filtered (the    */
/* caller then reads defaults[i]).  n_dev: optional DEVICE count <= n.       */
/* This is the per-key part of KvResourceGather[V1]                          */
/* (kv_variable_ops.cc:314-449 -> EmbeddingVar::LookupOrCreate).             */
size_t dr_ev_resolve_workspace_size(int64_t n);
int dr_ev_resolve(dr_ev* ev, const int64_t* keys, int64_t n, const int64_t* n_dev,
                  const float* defaults, const int32_t* counts, int64_t* rows_out,
                  void* ws, size_t ws_bytes, void* stream);
/* Grouped resolve over T EVs of equal dim (one per feature) in one launch: */
/* keys/counts/rows_out concatenated, table t at [koff_host[t],             */
/* koff_host[t+1]), optional per-table DEVICE counts; defaults = EV default. */
int dr_ev_resolve_grouped(dr_ev* const* evs, int num_tables, const int64_t* keys,
                          const int64_t* koff_host, const int64_t* const* n_dev_per_table,
                          const int32_t* counts, int64_t* rows_out, void* ws, size_t ws_bytes,
                          void* stream);
/* Fused one-hot forward lookup: KvResourceGather + SparseSegmentSum of     */
/* embedding_lookup_sparse (embedding_ops.py:480-675, kv_variable_ops.cc:   */
/* 314-366) for T filter-free EVs of equal dim when every bag holds exactly */
/* one id (a [B, 1] SparseTensor per feature): keys [T, batch] (table t's   */
/* id of bag b at t*batch + b) -> out[b*out_stride + t*dim + c].  Insert-on-*/
/* miss with the EV default row, as resolve + pool.  order: DR_ORDER_ALI    */
/* (embedding_lookup_sparse) or DR_ORDER_SEQ (fused op: 0 + e).  Requires   */
/* dim % 4 == 0, dim <= 256, 16-B aligned out, T*batch < 2^31.              */
size_t dr_ev_lookup_onehot_workspace_size(int num_tables, int64_t batch);
int dr_ev_lookup_onehot(dr_ev* const* evs, int num_tables, const int64_t* keys, int64_t batch,
                        float* out, int64_t out_stride, int order, void* ws, size_t ws_bytes,
                        void* stream);
/* The same, also writing the row each id was served from (rows_out[t*batch */
/* + b]; -1 = the EV default, served when the pool was exhausted): the       */
/* training forward of filter-free EVs, whose backward regroups by these     */
/* rows (dr_pool_grad_rows_grouped) instead of by a Unique.                  */
int dr_ev_lookup_onehot_rows(dr_ev* const* evs, int num_tables, const int64_t* keys,
                             int64_t batch, float* out, int64_t out_stride, int order,
                             int64_t* rows_out, void* ws, size_t ws_bytes, void* stream);
/* The same with the ids read through strides: id of (bag b, table t) =    */
/* keys[b*key_stride_bag + t*key_stride_table].  (1, batch) is the [T,      */
/* batch] layout above; (T, 1) reads a record-major [batch, T] id matrix in */
/* place -- one Criteo record of T categorical ids per row, the input of     */
/* the SOK/DLRM Criteo-TB pipeline (modelzoo/SOK/DLRM) -- so the kernel,    */
/* which visits (b, t) in output order, reads its ids as one contiguous run  */
/* instead of one 128-B line per table.  rows_out (nullable) is written at  */
/* rows_out[t*batch + b] in either layout.                                   */
int dr_ev_lookup_onehot_strided(dr_ev* const* evs, int num_tables, const int64_t* keys,
                                int64_t key_stride_bag, int64_t key_stride_table, int64_t batch,
                                float* out, int64_t out_stride, int order, int64_t* rows_out,
                                void* ws, size_t ws_bytes, void* stream);
/* The strided form with flags.  bf16 EVs (value_bits 16): by default the  */
/* output is fp32, each value widened (the reference casts bf16 embeddings */
/* to float32 before pooling, embedding_ops.py:606-607; out_stride in       */
/* floats); DR_LOOKUP_OUT_BF16 copies the rows bitwise into a bf16 output   */
/* (out_stride in bf16 elements, even; dim % 8 == 0): 8 + 16 + 2*2*D bytes  */
/* per lookup.  ALI order only for bf16 EVs.  The entries above are this    */
/* one with flags 0.                                                         */
#define DR_LOOKUP_OUT_BF16 1
/* DR_LOOKUP_TABLE_ORDER: visit the ids table by table (t, b) instead of in */
/* output order (b, t) -- the same results; with feature-major [T, B] ids   */
/* (key_stride_table = B) the id reads and the rows_out records ([T, B])    */
/* become contiguous instead of one 8-byte access per 128-byte line.        */
#define DR_LOOKUP_TABLE_ORDER 2
/* DR_LOOKUP_ROWS_RECORD: rows_out record-major, rows_out[b*T + t] -- the     */
/* slots of a wave are consecutive in output order, so the records leave as  */
/* whole 64-byte writes instead of one partial line per table; pass          */
/* rows_record = 1 to the row-grouped backward (_ex2 / _sgd_ex) with them.   */
#define DR_LOOKUP_ROWS_RECORD 4
int dr_ev_lookup_onehot_ex(dr_ev* const* evs, int num_tables, const int64_t* keys,
                           int64_t key_stride_bag, int64_t key_stride_table, int64_t batch,
                           void* out, int64_t out_stride, int order, int flags, int64_t* rows_out,
                           void* ws, size_t ws_bytes, void* stream);
/* Tagged resolve (owner side of the sharded exchange): keys of all T EVs  */
/* (equal dim) in one array, table of key i = tags[i]; n_dev: optional      */
/* DEVICE count.  Filtered keys give -(i+1) (read table t's default row).   */
/* per_table_host: optional HOST count of keys per table (capacity          */
/* accounting; NULL assumes all n keys may be new to every table).          */
int dr_ev_resolve_tagged(dr_ev* const* evs, int num_tables, const int64_t* keys,
                         const int32_t* tags, int64_t n, const int64_t* n_dev,
                         const int64_t* per_table_host, const int32_t* counts,
                         int64_t* rows_out, void* ws, size_t ws_bytes, void* stream);
/* Owner-side row pack: out[i] = resolved row of key i of table tags[i]     */
/* (the table's default row when filtered).                                  */
int dr_ev_gather_tagged(dr_ev* const* evs, int num_tables, const int32_t* tags,
                        const int64_t* rows, int64_t n, const int64_t* n_dev, float* out,
                        void* stream);
/* Value-pool base of this EV's column (primary or slot).                   */
const float* dr_ev_pool(dr_ev* ev);
/* Device pointer of this EV's default row (dim floats).                    */
const float* dr_ev_default_row(dr_ev* ev);

/* KvResourceGather (counts == NULL) / KvResourceGatherV1.                   */
size_t dr_ev_gather_workspace_size(int64_t n);
int dr_ev_gather(dr_ev* ev, const int64_t* keys, int64_t n, const float* defaults,
                 const int32_t* counts, float* out, void* ws, size_t ws_bytes,
                 void* stream);

/* KvResourceInsert / KvResourceImportV2 with EmbeddingVar::Import semantics */
/* (embedding_var.h:187-219): partition_num <= 0 disables the               */
/* key % 1000 % partition_num == partition_id filter.                        */
int dr_ev_insert(dr_ev* ev, const int64_t* keys, int64_t n, const float* values,
                 const int64_t* versions, const int64_t* freqs, int64_t partition_id,
                 int64_t partition_num, void* stream);

/* Bulk insert of keys key_begin + i * key_stride, i in [0, n), whose rows  */
/* are synth(seed, key, col) (dr_synth_value): populates synthetic tables   */
/* (stride = world for the key % world shard a rank owns).                   */
int dr_ev_insert_synthetic(dr_ev* ev, int64_t key_begin, int64_t key_stride, int64_t n,
                           uint64_t seed,
                           void* stream);

/* KvResourceExport (kv_variable_ops.cc:786-835), keys ascending.  Syncs.   */
/* Pass NULL outputs to query the count into *m_host first.                 */
int dr_ev_export(dr_ev* ev, int64_t* keys_out, float* values_out, int64_t* versions_out,
                 int64_t* freqs_out, int64_t capacity, int64_t* m_host, void* stream);

/* Per-key freq / version of the primary, host-side, syncs (tests/debug).   */
int dr_ev_key_meta(dr_ev* ev, const int64_t* keys_host, int64_t n, int64_t* freq_host,
                   int64_t* version_host, int32_t* has_row_host, void* stream);

/* Sparse applies: keys must be distinct within one call (rows are updated   */
/* in parallel).  Repeated indices are handled by the caller the way DeepRec */
/* does: summed first (optimizer.py:68-83), or for GradientDescent applied  */
/* one occurrence-round after another (gradient_descent.py:71-76).          */
/* KvResourceSparseApplyGradientDescent (training_ali_ops.cc:1597-1678).     */
int dr_ev_apply_sgd(dr_ev* var, float lr, const float* grad, const int64_t* keys,
                    int64_t n, const int64_t* n_dev, int64_t global_step, void* stream);
/* KvSparseApplyAdagrad (training_ali_ops.cc:61-145).                        */
int dr_ev_apply_adagrad(dr_ev* var, dr_ev* accum, float lr, const float* grad,
                        const int64_t* keys, int64_t n, const int64_t* n_dev,
                        int64_t global_step, void* stream);
/* KvSparseApplyAdam (training_ali_ops.cc:848-975).                          */
int dr_ev_apply_adam(dr_ev* var, dr_ev* m, dr_ev* v, float beta1_power, float beta2_power,
                     float lr, float beta1, float beta2, float epsilon, const float* grad,
                     const int64_t* keys, int64_t n, const int64_t* n_dev,
                     int64_t global_step, void* stream);
/* The same applies over T EVs of equal dim in few launches (16 tables per  */
/* launch): table t gets grads[t] [n_host[t], dim] for keys[t], optional     */
/* DEVICE count n_dev[t]; slot1/slot2: Adagrad accumulator / Adam m, v (or  */
/* NULL).  Scalars as in the single-table calls.                             */
/* DR_OPT_ADAM_ASYNC[_RMSPROP]: KvResourceSparseApplyAdamAsync               */
/* (training_ali_ops.cc:1404-1575; apply_sparse_rmsprop selects the second);  */
/* beta1_power / beta2_power are the variable's beta power slots (key 0), the */
/* caller advances them after the apply (:1558-1559).                        */
enum {
  DR_OPT_SGD = 0,
  DR_OPT_ADAGRAD = 1,
  DR_OPT_ADAM = 2,
  DR_OPT_ADAM_ASYNC = 3,
  DR_OPT_ADAM_ASYNC_RMSPROP = 4
};
int dr_ev_apply_grouped(int optimizer, dr_ev* const* vars, dr_ev* const* slot1,
                        dr_ev* const* slot2, int num_tables, const float* const* grads,
                        const int64_t* const* keys, const int64_t* n_host,
                        const int64_t* const* n_dev, float lr, float beta1_power,
                        float beta2_power, float beta1, float beta2, float epsilon,
                        int64_t global_step, void* stream);
/* The same with each gradient row given BY ADDRESS: grad_ptrs[t][i] is the */
/* address of key i's [dim] fp32 gradient row; bit 0 set = the row is used  */
/* as 0.0f + g (the reference's unsorted segment sum starting from 0).  The  */
/* grad_ptr output of dr_pool_grad_rows_grouped: the optimizer reads the     */
/* pooled gradient in place (no [U, dim] gradient written and read back).   */
/* Rows must be 16-byte aligned when dim % 4 == 0.                           */
int dr_ev_apply_grouped_ptr(int optimizer, dr_ev* const* vars, dr_ev* const* slot1,
                            dr_ev* const* slot2, int num_tables, const uint64_t* const* grad_ptrs,
                            const int64_t* const* keys, const int64_t* n_host,
                            const int64_t* const* n_dev, float lr, float beta1_power,
                            float beta2_power, float beta1, float beta2, float epsilon,
                            int64_t global_step, void* stream);
/* KvResourceSparseApplyGradientDescent by address with the keys' rows      */
/* KNOWN (rows[t][i], the uniq_rows output of dr_pool_grad_rows_grouped_ex): */
/* the forward of a filter-free EV resolved and initialised every key, so   */
/* LookupOrCreate would return exactly that row -- the key table is not     */
/* probed again (versions still stamped).  SGD only: the other optimizers   */
/* need the slot-column first-touch bits of the key's hash slot.            */
int dr_ev_apply_grouped_ptr_rows(int optimizer, dr_ev* const* vars, int num_tables,
                                 const uint64_t* const* grad_ptrs, const int64_t* const* keys,
                                 const int64_t* const* rows, const int64_t* n_host,
                                 const int64_t* const* n_dev, float lr, int64_t global_step,
                                 void* stream);
/* The row-grouped lookup backward and KvResourceSparseApplyGradientDescent  */
/* (training_ali_ops.cc:1597-1678) fused: the composition                    */
/*   dr_pool_grad_rows_grouped_ex(descs, ..., rowsel, defer = 1) ->          */
/*   dr_ev_apply_grouped_ptr_rows(DR_OPT_SGD, vars, ...)                     */
/* when the optimizer is the gradient's only consumer (the training graph   */
/* of embedding_ops.py:592-675 -> optimizer.apply_gradients).  Every         */
/* (table, row) run gets the same sum (ascending positions, the same chunk   */
/* association for runs > 256) and the same v -= lr * g rounding, the same   */
/* version stamp (steps_to_live EVs, global_step != -1); the runs are        */
/* applied in row order and the IndexedSlices are never formed.  vars[t]:    */
/* distinct filter-free primary EVs (fp32 or bf16) of dim `dim`, dim % 4 ==  */
/* 0, descs' top_grad slices 16-byte aligned with top_stride % 4 == 0.       */
/* Workspace: dr_ev_pool_grad_rows_sgd_workspace_size(total nnz, dim).       */
size_t dr_ev_pool_grad_rows_sgd_workspace_size(int64_t total_nnz, int dim);
int dr_ev_pool_grad_rows_apply_sgd(dr_ev* const* vars, const dr_pool_grad_desc* descs,
                                   int num_tables, int64_t batch, int dim, const int64_t* rowsel,
                                   float lr, int64_t global_step, void* ws, size_t ws_bytes,
                                   void* stream);
/* The same with record-major rows (rows_record = 1, DR_LOOKUP_ROWS_RECORD). */
int dr_ev_pool_grad_rows_apply_sgd_ex(dr_ev* const* vars, const dr_pool_grad_desc* descs,
                                      int num_tables, int64_t batch, int dim,
                                      const int64_t* rowsel, int rows_record, float lr,
                                      int64_t global_step, void* ws, size_t ws_bytes,
                                      void* stream);
/* KvResourceSparseApplyAdamAsync (training_ali_ops.cc:1404-1575) with the  */
/* beta powers DEVICE-resident, as the reference keeps them in an EV (key 0,  */
/* :1523-1526): powers[t] is table t's float[2] {beta1_power, beta2_power}.   */
/* The kernel forms alpha = lr sqrt(1 - b2p) / (1 - b1p) from them and a      */
/* follow-up kernel multiplies them by beta1 / beta2 only for tables whose    */
/* effective N (min(n_host, *n_dev)) is > 0 (:1482 `if (N > 0)`) -- no host   */
/* read of a device count, so the step can be graph-captured.  rmsprop != 0:  */
/* apply_sparse_rmsprop (:1483-1519), powers unused (may be NULL).  grads[t]:  */
/* a [n, dim] float block, or (by_address) uint64 row addresses.             */
int dr_ev_apply_adam_async_grouped(int rmsprop, int by_address, dr_ev* const* vars,
                                   dr_ev* const* m, dr_ev* const* v, int num_tables,
                                   const void* const* grads, const int64_t* const* keys,
                                   const int64_t* n_host, const int64_t* const* n_dev,
                                   float* const* powers, float lr, float beta1, float beta2,
                                   float epsilon, int64_t global_step, void* stream);
/* KvSparseApplyAdam (training_ali_ops.cc:848-975) with the beta powers     */
/* read from HBM: powers is ONE device float[2] {beta1_power, beta2_power}   */
/* shared by the tables (the optimizer's non-slot variables, adam.py          */
/* _create_slots); every table's kernel forms alpha = lr sqrt(1 - b2p) /     */
/* (1 - b1p) in float from it, as dr_ev_apply_grouped does on the host.      */
/* The powers are NOT advanced here (the optimizer's _finish does it once    */
/* per apply_gradients, after every table): with no host scalar that        */
/* changes per step, the apply can sit in a captured hipGraph.  grads[t]: a  */
/* [n, dim] float block, or (by_address) uint64 row addresses.               */
int dr_ev_apply_adam_grouped_dev(int by_address, dr_ev* const* vars, dr_ev* const* m,
                                 dr_ev* const* v, int num_tables, const void* const* grads,
                                 const int64_t* const* keys, const int64_t* n_host,
                                 const int64_t* const* n_dev, const float* powers, float lr,
                                 float beta1, float beta2, float epsilon, int64_t global_step,
                                 void* stream);
/* KvResourceSparseApplyAdagradDecay (training_ali_ops.cc:703-823; op def    */
/* core/ops/training_ali_ops.cc): accum and accum_decay_power are slot EVs   */
/* of var (var-shaped; the decay count is element 0 of a row, as the         */
/* optimizer's slot, adagrad_decay.py:104-124).  A row whose count is below  */
/* global_step / decay_step decays first: accum = max(accum * decay_rate,    */
/* decay_baseline), count += 1; then accum += g^2, var -= lr g rsqrt(accum).  */
/* grads[t]: a [n, dim] float block, or (grad_by_address) the uint64 row     */
/* addresses of dr_pool_grad_rows_grouped.  decay_step must be > 0.          */
int dr_ev_apply_adagrad_decay_grouped(dr_ev* const* vars, dr_ev* const* accums,
                                      dr_ev* const* decay_powers, int num_tables,
                                      const void* const* grads, int grad_by_address,
                                      const int64_t* const* keys, const int64_t* n_host,
                                      const int64_t* const* n_dev, float lr, int64_t decay_step,
                                      float decay_rate, float decay_baseline,
                                      int64_t global_step, void* stream);
/* KvResourceSparseApplyFtrl / FtrlV2 (training_ali_ops.cc:167-331; op defs  */
/* core/ops/training_ali_ops.cc): accum / linear are slot EVs of var;        */
/* l2_shrinkage 0 = Ftrl, > 0 = FtrlV2.  The row norm of `linear` is an fp32 */
/* reduction (Eigen's order is not reproducible: parity within 1e-5 rel).    */
int dr_ev_apply_ftrl(dr_ev* var, dr_ev* accum, dr_ev* linear, float lr, float l1, float l2,
                     float lr_power, float l2_shrinkage, const float* grad, const int64_t* keys,
                     int64_t n, const int64_t* n_dev, int64_t global_step, void* stream);
int dr_ev_apply_ftrl_grouped(dr_ev* const* vars, dr_ev* const* accums, dr_ev* const* linears,
                             int num_tables, const float* const* grads,
                             const int64_t* const* keys, const int64_t* n_host,
                             const int64_t* const* n_dev, float lr, float l1, float l2,
                             float lr_power, float l2_shrinkage, int64_t global_step,
                             void* stream);
int dr_ev_apply_ftrl_grouped_ptr(dr_ev* const* vars, dr_ev* const* accums,
                                 dr_ev* const* linears, int num_tables,
                                 const uint64_t* const* grad_ptrs, const int64_t* const* keys,
                                 const int64_t* n_host, const int64_t* const* n_dev, float lr,
                                 float l1, float l2, float lr_power, float l2_shrinkage,
                                 int64_t global_step, void* stream);

/* ------------------------------------------------------------------------ */
/* FusedEmbeddingLocalSparseLookUp[Grad]                                     */
/* (core/ops/fused_embedding_ops.cc:12-58, kernels in                        */
/* fused_embedding_local_ops_gpu.cu.cc:18-122).  sp_indices [nnz,2].         */
/* ------------------------------------------------------------------------ */
size_t dr_fused_local_workspace_size(int64_t batch);
int dr_fused_local_lookup(const float* table, int64_t rows, int dim, const int64_t* sp_values,
                          const int64_t* sp_indices, int64_t nnz, int64_t batch,
                          int combiner, float max_norm, float* out, int32_t* values_offset,
                          void* ws, size_t ws_bytes, void* stream);
int dr_fused_local_lookup_grad(const float* top_grad, const float* table, int64_t rows,
                               int dim, const int64_t* sp_values, const int32_t* values_offset,
                               int64_t nnz, int64_t batch, int combiner, float max_norm,
                               float* grad_out, void* stream);

/* ------------------------------------------------------------------------ */
/* Partitioned fused lookup: FusedEmbeddingSparsePreLookUp / PostLookUp /    */
/* PostLookUpGrad (core/ops/fused_embedding_ops.cc:60-198, kernels           */
/* core/kernels/fused_embedding/fused_embedding_ops_gpus.cu.cc:150-519),     */
/* the path python/ops/fused_embedding_ops.py:45-67 runs for a list of       */
/* partitioned dense tables ("div" strategy over partition_shapes[i][0]).    */
/* At most DR_MAX_PARTITIONS partitions.                                     */
/* ------------------------------------------------------------------------ */
#define DR_MAX_PARTITIONS 64
/* PreLookUp: ids are stably sorted by value (ties keep input order, as the  */
/* reference's cub radix sort of (value, (row, col)) pairs), partition p     */
/* holds the ids in [acc[p-1], acc[p]) (acc = prefix sums of partition_rows, */
/* host int64 [P]) rebased to the partition, with their (row, col) pairs.    */
/* Outputs are the partitions back to back: values_out [nnz], indices_out    */
/* [nnz, 2], and part_off (DEVICE int64 [P+1]) partition p = [part_off[p],   */
/* part_off[p+1]).  Ids outside [0, acc[P-1]) latch DR_INVALID_ARGUMENT and  */
/* are left out (the reference drops ids >= acc[P-1] silently and hands      */
/* negative ids to partition 0, where its Gather fails).  Partition          */
/* boundaries are exact lower bounds (the reference's CalcElementsOffset-    */
/* PerPartition dichotomy returns a wrong offset when exactly one sorted id  */
/* lies below a boundary, or when nnz <= 2).                   */
size_t dr_fused_pre_lookup_workspace_size(int64_t nnz);
int dr_fused_pre_lookup(const int64_t* sp_values, const int64_t* sp_indices, int64_t nnz,
                        const int64_t* partition_rows, int num_partitions, int64_t* values_out,
                        int64_t* indices_out, int64_t* part_off, void* ws, size_t ws_bytes,
                        void* stream);
/* PostLookUp: emb_vectors[b] = combiner over the entries (e, p) whose      */
/* partitioned_indices[p][e] row is b of (clip(emb_shards[p][e])), clip =    */
/* `*= max_norm / l2` when max_norm >= 0 and l2 > max_norm (SumUpEmbedding-  */
/* Shard).  The reference adds with float atomics (order unspecified); here  */
/* a bag is summed from 0 in ascending column order (sp_indices order), so   */
/* PostLookUp(PreLookUp(x)) equals FusedEmbeddingLocalSparseLookUp bit for   */
/* bit.  Combiner: sum; mean / n; sqrtn / sqrtf(n) (ApplyCombiner), so an    */
/* empty bag is 0 for sum and 0/0 (NaN) for mean / sqrtn, as the reference.  */
/* feature_nums[b] = n (int32).  emb_shards[p] / partitioned_indices[p] are  */
/* device pointers held in host arrays; shard_rows[p] = entries of p.        */
/* dense_cols = sp_dense_shape[1] (batch * dense_cols < 2^62).               */
size_t dr_fused_post_lookup_workspace_size(int64_t total_entries, int64_t batch);
int dr_fused_post_lookup(const float* const* emb_shards, const int64_t* const* partitioned_indices,
                         const int64_t* shard_rows, int num_partitions, int64_t batch,
                         int64_t dense_cols, int dim, int combiner, float max_norm,
                         float* emb_vectors, int32_t* feature_nums, void* ws, size_t ws_bytes,
                         void* stream);
/* PostLookUpGrad (DistributeGradToShard): grad_shards[p][e] =               */
/* CombineGrad(top_grad[row], feature_nums[row]) scaled by max_norm / l2 of  */
/* emb_shards[p][e] when max_norm >= 0 and l2 > max_norm.                    */
int dr_fused_post_lookup_grad(const float* top_grad, const float* const* emb_shards,
                              const int64_t* const* partitioned_indices,
                              const int64_t* shard_rows, int num_partitions, int64_t batch,
                              int dim, const int32_t* feature_nums, int combiner, float max_norm,
                              float* const* grad_shards, void* stream);

/* ------------------------------------------------------------------------ */
/* Owner partition for the row-sharded all-to-all (SOK selectKernel,         */
/* sparse_operation_kit/.../all2all_input_dispatcher.cu:36-126, and the EV   */
/* partition rule embedding_ops.py:207-209): stable bucket of keys by        */
/* owner = key % world; perm_out[j] = source position; send_counts[world]   */
/* (device int64).                                                           */
/* ------------------------------------------------------------------------ */
size_t dr_partition_workspace_size(int64_t n);
int dr_partition_by_owner(const int64_t* keys, int64_t n, const int64_t* n_dev, int world,
                          int64_t* keys_out, int32_t* perm_out, int64_t* send_counts,
                          void* ws, size_t ws_bytes, void* stream);
/* Same with owner = floormod(floormod(key, premod), world) when premod > 0: */
/* premod = 1000 is the EmbeddingVariable partition rule                     */
/* `ids % 1000 % np` of embedding_lookup (python/ops/embedding_ops.py:       */
/* 207-209; TF `%` is FloorMod), which differs from key % np when np does    */
/* not divide 1000.                                                          */
int dr_partition_by_owner_mod(const int64_t* keys, int64_t n, const int64_t* n_dev, int world,
                              int64_t premod, int64_t* keys_out, int32_t* perm_out,
                              int64_t* send_counts, void* ws, size_t ws_bytes, void* stream);
/* Request routing of a grouped unique (dr_unique_grouped layout): the      */
/* valid uniques of all T features are stably ordered by (owner, feature),  */
/* owner = key % world, giving the [peer][feature]-blocked send buffer of    */
/* the key all-to-all: keys_out/tags_out (feature id)/perm_out (source      */
/* position) and counts[world * T] (DEVICE int64, peer-major).               */
/* num_unique == NULL routes every key (raw ids of a forward-only one-hot   */
/* lookup: the owner's insert-on-miss dedups, SOK all2all_input_dispatcher).*/
size_t dr_route_workspace_size(int64_t n, int world, int num_tables);
int dr_route_by_owner(const int64_t* uniq, const int64_t* koff_host, int num_tables,
                      const int64_t* num_unique, int world, int64_t* keys_out,
                      int32_t* tags_out, int32_t* perm_out, int64_t* counts, void* ws,
                      size_t ws_bytes, void* stream);
/* Row exchange helpers: dst[perm[j]] = src[j] (scatter back) / dst[j] =     */
/* src[perm[j]] (pack), rows of `dim` floats; n_dev optional.                */
int dr_rows_scatter(const float* src, const int32_t* perm, int64_t n, const int64_t* n_dev,
                    int dim, float* dst, void* stream);
int dr_rows_pack(const float* src, const int32_t* perm, int64_t n, const int64_t* n_dev,
                 int dim, float* dst, void* stream);

/* ------------------------------------------------------------------------ */
/* Peer-mapped sharded one-hot lookup over xGMI (no staging copies).         */
/* The reference's SOK all2all dispatcher moves keys to owners and rows     */
/* back through NCCL buffers (all2all_input_dispatcher.cu:74,256-268,       */
/* forward_functions.cuh); here every rank exposes, once, through HIP IPC:  */
/*   inbox_keys [world][cap] int64, inbox_slot [world][cap] int32,          */
/*   inbox_cnt [world] int64 (region src is written by requester src),      */
/*   out [B, T*dim] fp32 (the pooled one-hot result, written by owners).    */
/* A step is dr_xgmi_route (requester: owner = key % world; writes           */
/* (key, slot = b*T + t) straight into the owner's inbox over xGMI) ->       */
/* a cross-rank barrier on the stream -> dr_xgmi_serve (owner: insert-on-    */
/* miss resolve of its inbox in its EVs, then writes each row straight into  */
/* out[slot] of the requester) -> barrier.  Filter-free EVs, forward only.   */
/* Outputs are position-addressed, so they equal the single-GPU lookup bit   */
/* for bit.  EVs are not grown by serve: dr_ev_reserve beforehand; overflow  */
/* latches DR_RESOURCE_EXHAUSTED.                                             */
/* ------------------------------------------------------------------------ */
#define DR_MAX_PEERS 16
#define DR_IPC_HANDLE_BYTES 64
/* handle of the allocation holding ptr (+ ptr's offset in it).              */
int dr_ipc_export(const void* ptr, void* handle_out, int64_t* offset_out);
/* maps a peer's allocation; *ptr_out = base + offset, *base_out for close.  */
int dr_ipc_import(const void* handle, int64_t offset, void** ptr_out, void** base_out);
int dr_ipc_close(void* base);
/* Allocation for buffers peers access over xGMI (the exchange inboxes,    */
/* outputs and gradients): UNCACHED device memory (hipDeviceMallocUncached), */
/* zero-filled, synchronous.  A coarse-grained hipMalloc buffer can keep a  */
/* stale line in one of its own GPU's per-XCD L2s after a peer rewrote it.  */
/* dr_ipc_free recycles the buffer for the next dr_ipc_alloc of the same    */
/* size (uncached memory is never returned to the HIP allocator).           */
int dr_ipc_alloc(size_t bytes, void** ptr_out);
int dr_ipc_free(void* ptr);
/* The same buffer as a DLPack v0.8 DLManagedTensor (device kDLROCM, compact */
/* row-major; dtype_code: 0 int, 1 uint, 2 float) whose C deleter frees it, */
/* for frameworks to own (torch.utils.dlpack.from_dlpack of a "dltensor"    */
/* capsule).  device_id must be the current device.                         */
int dr_ipc_alloc_dlpack(int ndim, const int64_t* shape, int dtype_code, int dtype_bits,
                        int device_id, void** managed_out);
/* A DLPack view (no ownership: the deleter frees the descriptor only) of   */
/* device memory the library owns, e.g. an engine buffer (dr_sharded_output). */
int dr_dlpack_view(void* data, int ndim, const int64_t* shape, int dtype_code, int dtype_bits,
                   int device_id, void** managed_out);

typedef struct {
  int32_t world, rank;
  int64_t cap;                        /* keys per (requester, owner) region */
  int64_t* inbox_keys[DR_MAX_PEERS];  /* rank p's inbox, mapped here         */
  int32_t* inbox_slot[DR_MAX_PEERS];
  int64_t* inbox_cnt[DR_MAX_PEERS];
  float* out[DR_MAX_PEERS];           /* rank p's [B, T*dim] output          */
} dr_xgmi_peers;

/* keys [T, B] int64 (feature-major, bag b of feature t = keys[t*B + b]);   */
/* cnt_ws: DEVICE int64[world] scratch.  Requires T*B <= cap.                */
int dr_xgmi_route(const dr_xgmi_peers* peers, const int64_t* keys, int num_tables,
                  int64_t batch, int64_t* cnt_ws, void* stream);
/* The same routing only ids b < n_dev[t] of each table t (n_dev: DEVICE   */
/* int64[num_tables], nullable = all): the deduplicating requester routes   */
/* each table's first-occurrence unique keys (dr_unique_grouped output laid */
/* out [T, batch], u = b < U_t) -- SOK's per-destination dedup before the   */
/* key exchange (all2all_input_dispatcher.cu:36-126) -- and expands the     */
/* rows it gets back (slot u*T + t) over its bags locally.                  */
int dr_xgmi_route_ex(const dr_xgmi_peers* peers, const int64_t* keys, int num_tables,
                     int64_t batch, const int64_t* n_dev, int64_t* cnt_ws, void* stream);
size_t dr_xgmi_serve_workspace_size(int world, int64_t cap);
int dr_xgmi_serve(const dr_xgmi_peers* peers, dr_ev* const* evs, int num_tables,
                  int64_t batch, void* ws, size_t ws_bytes, void* stream);
/* Backward of the peer-write lookup, owner side: this rank's inbox entries  */
/* (cnt_host[s] of source s, read by the caller from its inbox counts),      */
/* sorted by (table, source, slot), each pulling the requester's gradient    */
/* row grad_in[s][slot] ([B, T*dim] per peer, mapped like the outputs) over  */
/* xGMI: keys_out [R], grads_out [R, dim], table_start [T+1] (DEVICE; table  */
/* t's entries are [table_start[t], table_start[t+1])).  R = sum cnt_host.   */
size_t dr_xgmi_grad_pull_workspace_size(int world, int64_t cap);
int dr_xgmi_grad_pull(const dr_xgmi_peers* peers, const float* const* grad_in,
                      const int64_t* cnt_host, int num_tables, int64_t batch, int dim,
                      int64_t* keys_out, float* grads_out, int64_t* table_start, void* ws,
                      size_t ws_bytes, void* stream);
/* The same without any host read: the inbox counts are read on the device,  */
/* and table t's entries (sorted by (source, slot)) land in its fixed region */
/* keys_out[t*W*batch ...], grads_out[t*W*batch ...] (every requester sends  */
/* at most `batch` ids of a table); counts_out[t] (DEVICE int64) = how many. */
/* The optimizer takes the region with counts_out[t] as its device count.    */
size_t dr_xgmi_grad_pull_dev_workspace_size(int world, int64_t cap);
int dr_xgmi_grad_pull_dev(const dr_xgmi_peers* peers, const float* const* grad_in,
                          int num_tables, int64_t batch, int dim, int64_t* keys_out,
                          float* grads_out, int64_t* counts_out, void* ws, size_t ws_bytes,
                          void* stream);

/* ------------------------------------------------------------------------ */
/* Sharded lookup as C entries (SURVEY 8b "sharded variants taking a         */
/* dr_comm*"): the index all-to-all -> owner gather -> row all-to-all        */
/* engine of the reference's multi-GPU embedding plugin, the SOK C++ entry   */
/* (sparse_operation_kit/kit_cc/framework/kernels/dense_fprop.cc:193-212 ->  */
/* kit_cc_infra/src/embeddings/embedding_layer.cc:52-72, NCCL send / recv in */
/* kit_cc_impl/embedding/dispatcher/all2all_input_dispatcher.cu:241-286),    */
/* and the EV partition rule owner = key % world (embedding_ops.py:207-209;  */
/* = key % 1000 % world for world | 1000).                                    */
/*                                                                            */
/* A dr_comm carries the collective: RCCL over xGMI (dr_comm_init with an    */
/* ncclUniqueId from dr_comm_rccl_unique_id, distributed by the caller), or  */
/* a caller-supplied callback table (a host framework's own collectives;     */
/* tests drive it with gloo).  All device buffers, stream-ordered.           */
/* ------------------------------------------------------------------------ */
typedef struct dr_comm dr_comm;
typedef struct {
  void* user;
  /* Variable all-to-all: send_counts[p] elements of elem_bytes from send    */
  /* (peer-major, consecutive) to rank p; recv_counts[p] from rank p into    */
  /* recv (peer-major).  Counts are HOST arrays of world entries.  Return 0. */
  int (*all_to_all_v)(void* user, const void* send, const int64_t* send_counts, void* recv,
                      const int64_t* recv_counts, int64_t elem_bytes, void* stream);
  /* All-gather of `bytes` HOST bytes from every rank into recv, rank-major  */
  /* (world * bytes).  Engine setup only (the IPC handle exchange of the     */
  /* XGMI kind).  NULL: no XGMI engine on this comm.                         */
  int (*all_gather)(void* user, const void* send, int64_t bytes, void* recv);
  /* Stream-ordered cross-rank barrier: all work queued on `stream` before it */
  /* on every rank completes before work queued after it on any rank.  The   */
  /* XGMI kind calls it twice per step.  NULL: no XGMI engine on this comm.  */
  int (*barrier)(void* user, void* stream);
} dr_comm_ops;
#define DR_RCCL_UNIQUE_ID_BYTES 128
/* ncclGetUniqueId (rank 0 calls it and hands the bytes to every rank).      */
int dr_comm_rccl_unique_id(void* out, int64_t bytes);
/* Exactly one of rccl_unique_id / ops.  The RCCL form binds the calling    */
/* thread's current HIP device (ncclCommInitRank).                           */
int dr_comm_init(const void* rccl_unique_id, int rank, int world, const dr_comm_ops* ops,
                 dr_comm** out);
int dr_comm_destroy(dr_comm* comm);
int dr_comm_rank(const dr_comm* comm);
int dr_comm_world(const dr_comm* comm);
/* The comm's variable all-to-all (exported for callers and tests).          */
int dr_comm_all_to_all_v(dr_comm* comm, const void* send, const int64_t* send_counts,
                         void* recv, const int64_t* recv_counts, int64_t elem_bytes,
                         void* stream);

/* The sharded lookup engine over this rank's T EV shards (filter-free EVs  */
/* of one dim and value type; rank r holds the keys with key % world == r). */
/* Buffers are owned by the engine and grown on demand.                      */
typedef struct dr_sharded dr_sharded;
int dr_sharded_create(dr_comm* comm, dr_ev* const* evs, int num_tables, dr_sharded** out);
int dr_sharded_destroy(dr_sharded* s);
/* Forward: ids int64, this rank's batch in the grouped layout -- table t   */
/* owns ids[koff_host[t], koff_host[t+1]) (koff_host: HOST T+1 offsets; NULL */
/* = t * bags, one-hot).  bag_off NULL = one-hot (every table holds `bags`   */
/* ids, bag b = id b), else T pointers to int32 [bags + 1] CSR offsets over  */
/* the table's ids (bag_off[t][bags] = its id count: every id is in a bag).  */
/* out [bags, T*dim]: fp32 (bf16 EVs widened, the                            */
/* reference's cast, embedding_ops.py:606-607) or bf16 with                  */
/* DR_SHARDED_OUT_BF16.  Per-bag association = the single-GPU lookup's (ALI  */
/* order by position), so the output equals one GPU's bit for bit.           */
/* need_grad keeps the exchange state for dr_sharded_backward; a forward-   */
/* only one-hot lookup routes the raw ids (the owner's insert-on-miss        */
/* dedups, SOK's all2all_input_dispatcher), otherwise the grouped Unique     */
/* runs first (embedding_ops.py:592-596).  One host read of the split sizes */
/* per direction (SOK syncs there too, all2all_input_dispatcher.cu:256-268). */
#define DR_SHARDED_OUT_BF16 1
int dr_sharded_forward(dr_sharded* s, const int64_t* ids, const int64_t* koff_host,
                       const int32_t* const* bag_off, int64_t bags, int combiner, int need_grad,
                       int flags, void* out, void* stream);
/* Backward of the last need_grad forward: grad [bags, T*dim] fp32 -> per   */
/* local unique id its SparseSegment*Grad row (math_grad.py:321-368) -> the  */
/* rows all-to-all to the owners -> this rank's IndexedSlices per table,     */
/* source-rank-major (what the optimizer's _deduplicate_indexed_slices,     */
/* optimizer.py:68-83, then sums in order).  keys_out[t] / grads_out[t]      */
/* point into the engine's buffers (valid until its next call); counts_out  */
/* [t] (HOST) = rows of table t.                                             */
int dr_sharded_backward(dr_sharded* s, const float* grad, const int64_t** keys_out,
                        const float** grads_out, int64_t* counts_out, void* stream);
/* Keys exchanged by the last forward: sent to peers / received from them   */
/* (-1 for the kinds below, which keep the counts on the device).            */
int dr_sharded_last_stats(const dr_sharded* s, int64_t* sent, int64_t* received);

/* Engine kinds (dr_sharded_create_ex).                                      */
/* DR_SHARDED_RCCL: the engine above (dr_sharded_create): exact-size         */
/*   all-to-alls, one host read of the split sizes per direction.            */
/* DR_SHARDED_XGMI: the peer-write exchange (dr_xgmi_* above) run inside the */
/*   library -- route -> barrier -> serve -> barrier; backward: the gradient */
/*   into the shared buffer -> barrier -> owner pull -> barrier.  Buffers    */
/*   (uncached, dr_ipc_alloc) are mapped across ranks once at create time    */
/*   through the comm's all_gather (IPC handles); the barriers are the       */
/*   comm's (RCCL: a one-float all-reduce).  One-hot sum over `batch` bags;  */
/*   no host read, so a step captures into a hipGraph.                       */
/* DR_SHARDED_RCCL_FIXED: the all-to-all engine at fixed capacity: every     */
/*   rank sends each peer a region of tables * max_ids keys (and the rows   */
/*   back in the same layout), the [world, tables] counts in a header; every */
/*   size after the exchange is a device count, so no host read and the step */
/*   captures into a hipGraph.  It moves world x the keys of the variable    */
/*   exchange at worst -- the price of the capture.  A block past its region */
/*   latches DR_RESOURCE_EXHAUSTED (dr_status_check).                        */
/* Outputs of every kind equal the single-GPU lookup bit for bit.            */
#define DR_SHARDED_RCCL 0
#define DR_SHARDED_XGMI 1
#define DR_SHARDED_RCCL_FIXED 2
typedef struct {
  int32_t kind;
  int32_t reserved;  /* 0 */
  int64_t batch;     /* XGMI: bags per table (one-hot), the same on every rank */
  int64_t max_ids;   /* RCCL_FIXED: most ids one table holds on one rank in a step */
} dr_sharded_config;
int dr_sharded_create_ex(dr_comm* comm, dr_ev* const* evs, int num_tables,
                         const dr_sharded_config* cfg, dr_sharded** out);
/* XGMI: the engine buffer holding the last forward's [batch, T*dim] result  */
/* (the EVs' value type; valid until the next forward).  dr_sharded_forward  */
/* with out == NULL leaves it there instead of copying it out.               */
int dr_sharded_output(dr_sharded* s, void** out);
/* Backward of the XGMI / RCCL_FIXED kinds with device counts: table t's    */
/* IndexedSlices are keys_out[t][0, n_t) / grads_out[t][0, n_t) with n_t =   */
/* *counts_dev_out[t] (DEVICE int64), inside a fixed region of *region_rows */
/* rows (world x batch, or world x max_ids).  Order: table-major, source-   */
/* rank-major (source-slot order within a source for XGMI, the source's     */
/* first-occurrence Unique order for RCCL_FIXED).  Valid until the next     */
/* call.  dr_sharded_backward works for these kinds too (one host read).    */
int dr_sharded_backward_dev(dr_sharded* s, const float* grad, const int64_t** keys_out,
                            const float** grads_out, const int64_t** counts_dev_out,
                            int64_t* region_rows, void* stream);
/* Byte copy between any host / device buffers on `stream` (hipMemcpyDefault); */
/* sync != 0 waits for it.  For host frameworks' dr_comm callbacks that stage */
/* device buffers through host memory (e.g. a CPU collective).               */
int dr_memcpy(void* dst, const void* src, int64_t bytes, int sync, void* stream);

/* ------------------------------------------------------------------------ */
/* Interactions (callers of the path).                                       */
/* ------------------------------------------------------------------------ */
/* FM 2nd order (modelzoo/DeepFM/train.py:205-209): emb [B,F,D] -> [B,D].   */
int dr_fm2(const float* emb, int64_t batch, int fields, int dim, float* out, void* stream);
int dr_fm2_grad(const float* emb, const float* top_grad, int64_t batch, int fields, int dim,
                float* grad_emb, void* stream);
/* DeepFM --bf16 (train.py:186-189: the dnn input cast to bf16): dr_fm2 that  */
/* also writes emb_bf16 [B, F*D] = bf16(emb) from the same loads, and the FM  */
/* backward that adds the bf16 gradient of that copy (row stride add_stride) */
/* after the FM term -- the single fp32 add where the two uses meet.         */
int dr_fm2_bf16_copy(const float* emb, int64_t batch, int fields, int dim, float* out,
                     uint16_t* emb_bf16, void* stream);
int dr_fm2_grad_add_bf16(const float* emb, const float* top_grad, const uint16_t* add,
                         int64_t add_stride, int64_t batch, int fields, int dim, float* grad_emb,
                         void* stream);
/* DLRM dot (modelzoo/DLRM/train.py:150-163): X [B,F,D] -> [B, F(F-1)/2].   */
int dr_dot_interaction(const float* x, int64_t batch, int fields, int dim, float* out,
                       void* stream);
/* Its backward: grad_x [B,F,D] = S X with S the symmetric completion of    */
/* top_grad [B, F(F-1)/2] (autodiff of the reference's matmul + mask).       */
int dr_dot_interaction_grad(const float* x, const float* top_grad, int64_t batch, int fields,
                            int dim, float* grad_x, void* stream);
/* The DLRM dot layer with its concat and --bf16 cast fused                   */
/* (modelzoo/DLRM/train.py:211-226: concat([dense_inputs, dot_op(stack)], 1), */
/* then tf.cast(net, bf16)), X[b, 0, :] = dense_inputs: row b of out [B,      */
/* out_stride] bf16 = bf16(X[b,0,:]) | bf16(dot) | zeros to out_stride (the   */
/* top MLP's K padding).  2 <= fields <= 32, dim in {16, 32, 64, 128},        */
/* out_stride even.  Same fp32 products as dr_dot_interaction, one RNE.      */
int dr_dot_interaction_concat_bf16(const float* x, int64_t batch, int fields, int dim,
                                   uint16_t* out, int64_t out_stride, void* stream);
/* Its backward from the bf16 gradient of that matrix: grad_x = S X + (the     */
/* dense_inputs columns 0..dim-1 added to row 0), S from columns dim...       */
int dr_dot_interaction_concat_grad_bf16(const float* x, const uint16_t* grad, int64_t grad_stride,
                                        int64_t batch, int fields, int dim, float* grad_x,
                                        void* stream);
/* DCN-v2 cross layer (absent in the reference): out = x0 * (xl W^T + b) + xl */
/* x0/xl/out [B,d] bf16 (uint16 storage), W [d,d] bf16 row-major (out,in),   */
/* b [d] f32; bf16 MFMA with fp32 accumulation.                              */
int dr_crossnet_layer_bf16(const uint16_t* x0, const uint16_t* xl, const uint16_t* W,
                           const float* bias, int64_t batch, int d, uint16_t* out,
                           void* stream);
/* CrossNet backward, elementwise part of one layer in one pass (dx_l = u W  */
/* + g: dr_crossnet_dx_bf16; dW = u^T x_l a library GEMM): u = bf16(g * x0), */
/* acc_out = (acc_in or 0) + g * lin in fp32 (dx0 summed over the layers),  */
/* db = column sums of u (fixed order).  g, x0, lin, u bf16 [batch, d];     */
/* acc_in may be NULL or equal acc_out.  Workspace: per-row-block partials.  */
/* The layer's input gradient on the forward's 256 x 256 MFMA schedule:     */
/* dx = u W + g = u wt^T + g, wt = W^T [d, d] bf16 (row k = column k of W),   */
/* u, g, dx [batch, d] bf16; fp32 accumulate, one rounding of (u W + g) --    */
/* what torch.addmm(g, u, W) computes in bf16.  d % 64 == 0, 16-B aligned.   */
int dr_crossnet_dx_bf16(const uint16_t* u, const uint16_t* wt, const uint16_t* g, int64_t batch,
                        int d, uint16_t* dx, void* stream);
size_t dr_crossnet_backward_workspace_size(int64_t batch, int d);
int dr_crossnet_backward_elem_bf16(const uint16_t* g, const uint16_t* x0, const uint16_t* lin,
                                   const float* acc_in, float* acc_out, uint16_t* u, float* db,
                                   int64_t batch, int d, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------ */
/* Dense towers on the pooled output: bf16 MFMA GEMMs of the DLRM top /     */
/* bottom MLPs (modelzoo/DLRM/train.py:183-221 with --bf16; north_star:     */
/* "MFMA ... for the dense CrossNet / top-MLP contraction").                */
/*   C[M, N] = act(A[M, K] . B[N, K]^T + bias[N])                            */
/* A, B bf16 row-major with row strides lda, ldb (elements); fp32           */
/* accumulate; C bf16 (c_fp32 = 0) or fp32, row stride ldc.  K % 64 == 0,    */
/* N % 8 == 0, strides % 8 == 0, 16-B aligned pointers (pad with zeros).     */
/* split_k > 1 cuts K into split_k chunks (fp32 partials in ws, summed in    */
/* chunk order: deterministic) -- for the weight gradient dW = g^T x, whose  */
/* K is the batch.  bias nullable; act DR_ACT_NONE / DR_ACT_RELU.           */
#define DR_ACT_NONE 0
#define DR_ACT_RELU 1
#define DR_ACT_MASK 2  /* _ex only: C = result where aux > 0, else 0 (no split) */
size_t dr_gemm_nt_workspace_size(int64_t M, int64_t N, int split_k);
int dr_gemm_nt_bf16(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, int64_t M,
                    int64_t N, int64_t K, const float* bias, int act, void* C, int64_t ldc,
                    int c_fp32, int split_k, void* ws, size_t ws_bytes, void* stream);
/* With an aux operand: act DR_ACT_MASK zeroes C where the bf16 aux[M, N]  */
/* (row stride ld_aux) is not > 0 -- the ReLU mask of the layer below,      */
/* applied to the input gradient of the layer above in the same pass.       */
int dr_gemm_nt_bf16_ex(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, int64_t M,
                       int64_t N, int64_t K, const float* bias, int act, const uint16_t* aux,
                       int64_t ld_aux, void* C, int64_t ldc, int c_fp32, int split_k, void* ws,
                       size_t ws_bytes, void* stream);
/* Weight-gradient GEMM without operand transposes: C[n][k] (fp32, ldc) =    */
/* sum_b G[b][n] X[b][k] over rows b, G [rows, N] and X [rows, K] bf16       */
/* row-major (the gradient and the input of a Linear layer: dW = g^T x).     */
/* rows % 64 == 0, N and K % 8 == 0.  colsum (nullable) [N] fp32 = the       */
/* column sums of G (the layer's bias gradient).  split_k > 1 splits the     */
/* rows into fp32 partials summed in split order (deterministic); workspace: */
/* dr_gemm_tn_workspace_size(N, K, split_k, colsum != NULL).                 */
size_t dr_gemm_tn_workspace_size(int64_t N, int64_t K, int split_k, int with_colsum);
int dr_gemm_tn_bf16(const uint16_t* G, int64_t ldg, const uint16_t* X, int64_t ldx, int64_t rows,
                    int64_t N, int64_t K, float* C, int64_t ldc, float* colsum, int split_k,
                    void* ws, size_t ws_bytes, void* stream);
/* out[c][r] = in[r][c], bf16; rows, cols and strides multiples of 8.        */
int dr_transpose_bf16(const uint16_t* in, int64_t rows, int64_t cols, int64_t ld_in,
                      uint16_t* out, int64_t ld_out, void* stream);
/* Same, also writing col_partials [ceil(rows/64), cols] fp32: each 64-row   */
/* tile's column sums (8 rows in order, then a fixed butterfly), so a layer's */
/* bias gradient db = col_partials summed over tiles comes with the dW       */
/* operand transpose instead of another pass over g.                         */
int dr_transpose_bf16_colsum(const uint16_t* in, int64_t rows, int64_t cols, int64_t ld_in,
                             uint16_t* out, int64_t ld_out, float* col_partials, void* stream);
/* ReLU layer backward entry: out = bf16(grad) where the bf16 ReLU output y */
/* is > 0, else 0; grad fp32 (row stride ld_grad, a multiple of 4), cols and */
/* the bf16 strides multiples of 8, pointers 16-B aligned.                   */
int dr_relu_grad_bf16(const float* grad, int64_t ld_grad, const uint16_t* y, int64_t ld_y,
                      int64_t rows, int64_t cols, uint16_t* out, int64_t ld_out, void* stream);
/* The DLRM output layer under --bf16 (modelzoo/DLRM/train.py:241-249:       */
/* dense(units=1) on the bf16 top MLP): z[b] = bf16(sum_k h[b,k] w[k] + bias) */
/* as fp32, h [batch, k] bf16 (row stride ldh), w [k] bf16, bias a device   */
/* fp32 scalar (nullable), fp32 sum in a fixed order.  k in {64,128,256,512}.*/
/* w_fp32 = 1: the fp32 output layer on a bf16 tower (DeepFM --bf16,        */
/* train.py:213-221): w fp32, the logit (and, backward, gz) not rounded.     */
int dr_mlp_head_forward_bf16(const uint16_t* h, int64_t ldh, int64_t batch, int k,
                             const void* w, int w_fp32, const float* bias, float* z,
                             void* stream);
/* Its backward from grad_z [batch] fp32 (rounded to bf16 first, as the bf16 */
/* layer sees it): grad_h = bf16(gz w) where h > 0, else 0 (the top layer's   */
/* ReLU derivative in the same pass); dw_partials [P, k] and db_partials [P]  */
/* fp32 = per-block sums of gz h and gz, P = dr_mlp_head_grad_partials(batch) */
/* (the caller sums them over P: deterministic).                              */
size_t dr_mlp_head_grad_partials(int64_t batch);
int dr_mlp_head_backward_bf16(const uint16_t* h, int64_t ldh, int64_t batch, int k,
                              const void* w, int w_fp32, const float* grad_z, uint16_t* grad_h,
                              int64_t ld_grad_h, float* dw_partials, float* db_partials,
                              void* stream);
/* Same layer, also writing lin_out = xl W^T + b (bf16, nullable; needs      */
/* d % 64 == 0) for the backward pass.  d % 64 == 0 selects the pipelined    */
/* kernel (global_load_lds staging, double-buffered K steps of 64).          */
int dr_crossnet_forward_bf16(const uint16_t* x0, const uint16_t* xl, const uint16_t* W,
                             const float* bias, int64_t batch, int d, uint16_t* out,
                             uint16_t* lin_out, void* stream);

/* CrossNet weight gradient dW = u^T x_l, fp32 [d, d] (u, x_l [batch, d]    */
/* bf16 row-major; d and batch multiples of 64): the forward's 256^2         */
/* four-phase MFMA schedule in TN form (transposing LDS reads), the batch     */
/* split into slices whose fp32 partials (workspace) are summed in slice     */
/* order -- deterministic.                                                    */
size_t dr_crossnet_dw_workspace_size(int64_t batch, int d);
int dr_crossnet_dw_bf16(const uint16_t* u, const uint16_t* xl, int64_t batch, int d, float* dw,
                        void* ws, size_t ws_bytes, void* stream);

/* DIN user-behaviour attention (modelzoo/DIN/script/utils.py:264-309,      */
/* din_attention mode 'SUM'; script/model.py:94-98,381-390).  query [B,H],  */
/* facts [B,T,H] (the gathered history, H = 2 x EMBEDDING_DIM), fp32.        */
/* hidden <= 64, or a multiple of 4 <= 256 with 16-B aligned operands.       */
/* din_all [B,T,4H] = [q, f, q - f, q * f] (utils.py:280-282).              */
int dr_din_attention_input(const float* query, const float* facts, int64_t batch, int64_t seq_len,
                           int hidden, float* out, void* stream);
/* Its backward: grad_query [B,H] = sum over t; grad_facts [B,T,H] is        */
/* written (accumulate = 0) or added to (accumulate = 1).                     */
int dr_din_attention_input_grad(const float* query, const float* facts, const float* top_grad,
                                int64_t batch, int64_t seq_len, int hidden, float* grad_query,
                                float* grad_facts, int accumulate, void* stream);
/* scores [B,T] (attention-MLP output), mask [B,T] (1.0 = valid,             */
/* tf.equal(mask, 1)): s = mask ? scores : float(-2^32+1); alphas = softmax  */
/* over t; att_out [B,H] = sum_t alpha_t f_t; sum_out [B,H] (nullable) =     */
/* sum_t f_t over every position (item_his_eb_sum, model.py:98).             */
int dr_din_attention_pool(const float* scores, const float* mask, const float* facts,
                          int64_t batch, int64_t seq_len, int hidden, float* att_out,
                          float* sum_out, float* alphas, void* stream);
/* Its backward: grad_scores [B,T] (0 where masked), grad_facts [B,T,H] =    */
/* alpha_t grad_att + grad_sum (grad_sum nullable).                          */
int dr_din_attention_pool_grad(const float* alphas, const float* mask, const float* facts,
                               const float* grad_att, const float* grad_sum, int64_t batch,
                               int64_t seq_len, int hidden, float* grad_scores,
                               float* grad_facts, void* stream);

/* The attention MLP of din_attention (utils.py:284-289: din_all -> 80      */
/* sigmoid -> 40 sigmoid -> 1 -> scores), fused: din_all is never written    */
/* (W1 = [A|Bm|C|Dm]: a1 = (A + C) q + b1 + [Bm - C | Dm] [f ; q f]) and only */
/* the valid (mask != 0) positions run it -- a padded position's score is     */
/* replaced by the padding value before the softmax.  Weights are the torch  */
/* Linear layouts: w1 [n1, 4H], w2 [n2, n1], w3 [n2] (f3_att.weight[0]),      */
/* b3 [1]; n1 = 80, n2 = 40; hidden 16, 32, 36 or 64.  Caller-owned buffers   */
/* (cap = batch * seq_len); forward fills pos / cnt / off / w1p / w2t / cq /  */
/* h1t / h2t and writes scores at the valid positions (others untouched);    */
/* the backward reads them and grad_scores, adds the MLP's part to           */
/* grad_facts and fills the per-position / per-sample buffers from which the  */
/* caller forms the weight gradients:                                         */
/*   dW1 = [Gq | Gf | Gq - Gf | Gqf], Gq = s1^T q, [Gf | Gqf] = da1t xt^T,    */
/*   db1 = column sums of s1, dW2 = da2t h1t^T, db2 = row sums of da2t,       */
/*   dw3 = h2t dsc, db3 = sum dsc, grad_query += s1 (A + C) + dq2.            */
typedef struct dr_din_mlp_buf {
  int32_t* pos;   /* [cap] valid positions b*T + t, sample-major, ascending   */
  int32_t* cnt;   /* [batch] valid positions per sample                      */
  int32_t* off;   /* [batch + 1] exclusive prefix of cnt (off[batch] = P)    */
  float* w1p;     /* [n1, 2H] = [Bm - C | Dm]                                */
  float* w2t;     /* [n1, n2] = w2^T                                         */
  float* cq;      /* [batch, n1] = (A + C) q + b1                            */
  float* h1t;     /* [n1, cap] sigmoid outputs (columns p < P)               */
  float* h2t;     /* [n2, cap]                                               */
  float* da1t;    /* [n1, cap] backward: d a1 (zero columns p >= P)          */
  float* da2t;    /* [n2, cap] d a2                                          */
  float* xt;      /* [2H, cap] [f ; q f]                                     */
  float* dsc;     /* [cap] d score per valid position                        */
  float* dqp;     /* [H, cap] f * d(q f)                                     */
  float* s1;      /* [batch, n1] per-sample sum of d a1 (ascending positions) */
  float* dq2;     /* [batch, H] per-sample sum of f * d(q f)                 */
} dr_din_mlp_buf;
int dr_din_mlp_forward(const float* query, const float* facts, const float* mask, int64_t batch,
                       int64_t seq_len, int hidden, const float* w1, const float* b1, int n1,
                       const float* w2, const float* b2, int n2, const float* w3, const float* b3,
                       float* scores, const dr_din_mlp_buf* buf, void* stream);
/* The attention MLP's weight gradients from dr_din_mlp_backward's buffers   */
/* in one split-K pass over the cap positions: out = [G = da1 x^T (n1 x 2H),  */
/* dW2 = da2 h1^T (n2 x n1), db2 = sum da2 (n2), dw3 = h2 dsc (n2), db3 =     */
/* sum dsc (1)], fp32 partials summed in block order (deterministic).  The    */
/* buffers are the dr_din_mlp_buf fields da1t, xt, da2t, h1t, h2t, dsc        */
/* (feature-major, columns past the valid count zero).  n1 = 80, n2 = 40.     */
size_t dr_din_mlp_wgrad_workspace_size(int n1, int hidden2, int n2);
int dr_din_mlp_wgrad(const float* da1t, const float* xt, const float* da2t, const float* h1t,
                     const float* h2t, const float* dsc, int64_t cap, int n1, int hidden2, int n2,
                     float* out, void* ws, size_t ws_bytes, void* stream);
/* The same over the valid positions only: valid = a device int32 (the       */
/* buffer's off[batch] = P), read on the device, so the columns p >= P need  */
/* not be zero (dr_din_mlp_backward_tail with zero_tail = 0 skips them).      */
int dr_din_mlp_wgrad_valid(const float* da1t, const float* xt, const float* da2t,
                           const float* h1t, const float* h2t, const float* dsc, int64_t cap,
                           const int32_t* valid, int n1, int hidden2, int n2, float* out, void* ws,
                           size_t ws_bytes, void* stream);
int dr_din_mlp_backward(const float* query, const float* facts, int64_t batch, int64_t seq_len,
                        int hidden, int n1, int n2, const float* w3, const float* grad_scores,
                        float* grad_facts, const dr_din_mlp_buf* buf, void* stream);
/* dr_din_mlp_backward with the zeroing of the buffers' columns p >= P       */
/* optional (zero_tail = 0: only dr_din_mlp_wgrad_valid reads them after).    */
int dr_din_mlp_backward_tail(const float* query, const float* facts, int64_t batch,
                             int64_t seq_len, int hidden, int n1, int n2, const float* w3,
                             const float* grad_scores, float* grad_facts,
                             const dr_din_mlp_buf* buf, int zero_tail, void* stream);

/* DIN's Dice activation (modelzoo/DIN/script/utils.py:12-35, the batch      */
/* statistics form Model_DIN's fcn uses, model.py:130-134), fp32 x [batch, n] */
/* row-major: mean and std = sqrt(mean((x - mean)^2 + eps)) per column over   */
/* the batch, p = sigmoid((x - mean) / (std + eps)), y = alpha (1 - p) x +   */
/* p x.  stats [2, n] (mean, std) is written for the backward.  Column sums   */
/* in a fixed order (deterministic).                                          */
int dr_din_dice_forward(const float* x, const float* alpha, int64_t batch, int n, float epsilon,
                        float* y, float* stats, void* stream);
/* Its backward through the batch statistics: grad_x [batch, n], grad_alpha  */
/* [n] (written).                                                             */
int dr_din_dice_backward(const float* x, const float* grad_y, const float* alpha,
                         const float* stats, int64_t batch, int n, float epsilon, float* grad_x,
                         float* grad_alpha, void* stream);

/* Model_DIN's fcn input (model.py:118-124): inp = [uid (uid_dim), item,    */
/* his_sum, item * his_sum, att (hidden each)] per sample, then the           */
/* inference-form batch_normalization out = (inp * scale) * gamma + beta     */
/* (scale = 1 / sqrt(1 + 1e-3); gamma / beta [uid_dim + 4 hidden]); fp32,    */
/* out [batch, uid_dim + 4 hidden].  The backward writes the four inputs'    */
/* gradients and gamma / beta's (batch sums in a fixed order).               */
int dr_din_fcn_input_forward(const float* uid, const float* item, const float* his_sum,
                             const float* att, const float* gamma, const float* beta,
                             int64_t batch, int uid_dim, int hidden, float scale, float* out,
                             void* stream);
int dr_din_fcn_input_backward(const float* grad, const float* uid, const float* item,
                              const float* his_sum, const float* att, const float* gamma,
                              int64_t batch, int uid_dim, int hidden, float scale, float* g_uid,
                              float* g_item, float* g_his_sum, float* g_att, float* g_gamma,
                              float* g_beta, void* stream);

/* ------------------------------------------------------------------------ */
/* String -> id, the step before the lookup.  Strings are one byte buffer    */
/* plus int64 offsets[n+1] (string i = bytes[offsets[i] .. offsets[i+1])).   */
/* ------------------------------------------------------------------------ */
/* farmhash Fingerprint64 (core/platform/fingerprint.h:80-88; the Fingerprint */
/* op's per-string value, core/kernels/fingerprint_op.cc:55-64).             */
int dr_fingerprint64(const uint8_t* bytes, const int64_t* offsets, int64_t n, uint64_t* out,
                     void* stream);
/* StringToHashBucketFast (core/kernels/string_to_hash_bucket_ali_op.h:33-63, */
/* op def core/ops/string_ops.cc:77): out[i] = Fingerprint64(s_i) %          */
/* num_buckets.  EV string columns pass INT64_MAX                            */
/* (python/feature_column/feature_column_v2.py:5954-5957).                   */
int dr_string_to_hash_bucket_fast(const uint8_t* bytes, const int64_t* offsets, int64_t n,
                                  int64_t num_buckets, int64_t* out, void* stream);

/* SparseTensor preparation of safe_embedding_lookup_sparse                  */
/* (python/ops/embedding_ops.py:1289-1310) in one call: prune = 0 none,      */
/* 1 _prune_invalid_ids (ids < 0), 2 also _prune_invalid_weights (w <= 0),   */
/* then SparseFillEmptyRows (core/kernels/sparse_fill_empty_rows_op_util.h:  */
/* 17-128): rows ascending, a row's entries in input order, each empty row   */
/* one [row, 0..] entry = default_value (weight default_weight).  indices    */
/* [nnz, rank]; outputs sized for nnz + dense_rows entries, the used count   */
/* in *out_nnz (DEVICE int64).  reverse_index_map[i] = output position of    */
/* input i or -1 when pruned (nullable); empty_row [dense_rows] (nullable).  */
/* weights / out_weights both NULL or both set.  Rows out of range latch     */
/* INVALID_ARGUMENT.                                                         */
size_t dr_sparse_fill_workspace_size(int64_t nnz, int64_t dense_rows);
int dr_sparse_prune_fill(const int64_t* indices, int rank, const int64_t* values,
                         const float* weights, int64_t nnz, int64_t dense_rows, int prune,
                         int64_t default_value, float default_weight, int64_t* out_indices,
                         int64_t* out_values, float* out_weights, int64_t* reverse_index_map,
                         uint8_t* empty_row, int64_t* out_nnz, void* ws, size_t ws_bytes,
                         void* stream);

/* ------------------------------------------------------------------------ */
/* embedding_lookup_sparse / safe_embedding_lookup_sparse as ONE call        */
/* (python/ops/embedding_ops.py:480-675 and :1209-1344; the composition a TF */
/* custom-op kernel binds).  params: exactly one of `ev` (an */
/* EmbeddingVariable, insert-on-miss; a Counter/Bloom EV goes through         */
/* UniqueWithCounts -> KvResourceGatherV1 as :592-596 do) or a dense fp32     */
/* `table` [table_rows, dim] (ids bounds-checked).  sp_indices [nnz, 2]       */
/* int64 rows-sorted (SparseTensor canonical order), sp_values [nnz] int64,   */
/* sp_weights [nnz] or NULL.  combiner DR_COMBINER_*; max_norm >= 0 clips     */
/* each gathered row (clip_by_norm, :183-190), < 0 = None.                    */
/* safe != 0: safe_embedding_lookup_sparse: prune != 0 drops ids < 0 (and     */
/* weights <= 0 when weighted and combiner != sum), empty rows get           */
/* default_id (default_id < 0 = None: filled with id 0, their outputs zeroed */
/* at the end).  out [batch, out_stride] fp32: row b = bag b (bags past the   */
/* last non-empty one are 0; the reference's plain embedding_lookup_sparse   */
/* returns last_row + 1 rows, callers slice).  No host synchronisation        */
/* except for a filter EV with safe != 0 (the Unique's length).  Errors found */
/* on the device (unsorted rows, OOB dense ids) latch into dr_status_check.  */
/* ------------------------------------------------------------------------ */
size_t dr_embedding_lookup_sparse_workspace_size(int64_t nnz, int64_t batch);
int dr_embedding_lookup_sparse(dr_ev* ev, const float* table, int64_t table_rows, int dim,
                               const int64_t* sp_indices, const int64_t* sp_values,
                               const float* sp_weights, int64_t nnz, int64_t batch, int combiner,
                               float max_norm, int safe, int64_t default_id, int prune,
                               float* out, int64_t out_stride, void* ws, size_t ws_bytes,
                               void* stream);

/* ------------------------------------------------------------------------ */
/* Checkpoint support (host function, no device work): crc32c::Extend of    */
/* core/lib/hash/crc32c.h, used for TensorBundle entry and SSTable block     */
/* checksums (core/util/tensor_bundle/tensor_bundle.cc:435-455).             */
/* ------------------------------------------------------------------------ */
uint32_t dr_crc32c_extend(uint32_t init_crc, const void* data, size_t n);

/* ------------------------------------------------------------------------ */
/* Synthetic data (bench/tests): table[r, c] = hash-derived uniform [-1, 1)  */
/* of (seed, r, c), regenerable on host (dr_synth_value).                     */
/* ------------------------------------------------------------------------ */
int dr_fill_synthetic(float* table, int64_t rows, int dim, uint64_t seed, void* stream);
float dr_synth_value(uint64_t seed, int64_t row, int64_t col);

#ifdef __cplusplus
}
#endif
#endif /* DEEPREC_AMD_H_ */
