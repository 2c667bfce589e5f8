// lookup_sparse.hip -- the embedding_lookup_sparse / safe_embedding_lookup_
// sparse composition as ONE C entry (dr_embedding_lookup_sparse), so a TF
// custom-op kernel binds a single call instead of
// re-implementing python/ops/embedding_ops.py:480-675 and :1209-1344.
//
// Steps, all on `stream`, in the reference's order:
//   safe:  _prune_invalid_ids (id < 0) [+ _prune_invalid_weights (w <= 0)
//          when weighted and combiner != sum] -> SparseFillEmptyRows(default_id
//          or 0)   (:1289-1310; dr_sparse_prune_fill, DEVICE entry count)
//   seg = indices[:, 0] -> CSR bag offsets            (:587-589)
//   ids -> rows:  dense table: the ids themselves (bounds-checked, :94-342);
//                 EV without a filter: LookupOrCreate of every id (the CAS
//                 insert is the dedup; outputs equal unique -> gather);
//                 EV with a Counter / Bloom filter: UniqueWithCounts ->
//                 KvResourceGatherV1 with counts (:592-596, kv_variable_ops.cc
//                 :395-449) -> row of every id
//   gather + [clip_by_norm(max_norm)] + [* w] + SparseSegment{Sum,Mean,SqrtN}
//          in the reference's association order          (:600-675);
//          bf16 EVs: every row widened to float32 first  (:606-607)
//   safe, default_id None: rows that were empty come out 0   (:1330-1337)
//
// Every step takes device counts: no host synchronisation, except the
// filter-EV case after a prune/fill, where the Unique needs the entry count
// on the host (TF's own Unique has a data-dependent output shape there too).
#include <hip/hip_runtime.h>

#include "dr_common.h"

namespace dr {

__global__ void zero_empty_rows_kernel(float* __restrict__ out, int64_t stride, int64_t batch,
                                       int dim, const uint8_t* __restrict__ empty) {
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (b >= batch || !empty[b]) return;
  for (int c = threadIdx.x % 64; c < dim; c += 64) out[b * stride + c] = 0.f;
}

struct LsWs {
  int64_t *ind, *val, *n_dev, *rowsel, *uniq, *urows, *U;
  float* w;
  uint8_t* empty;
  int32_t *bag_off, *idx, *cnt;
  void* sub;  // workspace of the largest sub-call
  size_t sub_bytes;
};

static size_t sub_ws_bytes(int64_t cap, int64_t batch) {
  size_t m = dr_sparse_fill_workspace_size(cap, batch);
  m = m > dr_ev_resolve_workspace_size(cap) ? m : dr_ev_resolve_workspace_size(cap);
  m = m > dr_unique_workspace_size(cap) ? m : dr_unique_workspace_size(cap);
  return m;
}

static LsWs carve_ls(void* ws, int64_t nnz, int64_t batch, size_t* used) {
  Carver c(ws);
  const int64_t cap = nnz + batch > 0 ? nnz + batch : 1;
  LsWs w;
  w.ind = c.take<int64_t>(2 * cap);
  w.val = c.take<int64_t>(cap);
  w.w = c.take<float>(cap);
  w.empty = c.take<uint8_t>(batch > 0 ? batch : 1);
  w.n_dev = c.take<int64_t>(1);
  w.bag_off = c.take<int32_t>(batch + 1);
  w.rowsel = c.take<int64_t>(cap);
  w.uniq = c.take<int64_t>(cap);
  w.idx = c.take<int32_t>(cap);
  w.cnt = c.take<int32_t>(cap);
  w.urows = c.take<int64_t>(cap);
  w.U = c.take<int64_t>(1);
  w.sub_bytes = sub_ws_bytes(cap, batch > 0 ? batch : 1);
  w.sub = c.take<char>(w.sub_bytes);
  if (used) *used = c.used + 256;
  return w;
}

}  // namespace dr

extern "C" {

size_t dr_embedding_lookup_sparse_workspace_size(int64_t nnz, int64_t batch) {
  size_t used = 0;
  dr::carve_ls(nullptr, nnz, batch, &used);
  return used;
}

int dr_embedding_lookup_sparse(dr_ev* ev, const float* table, int64_t table_rows, int dim,
                               const int64_t* sp_indices, const int64_t* sp_values,
                               const float* sp_weights, int64_t nnz, int64_t batch, int combiner,
                               float max_norm, int safe, int64_t default_id, int prune,
                               float* out, int64_t out_stride, void* ws, size_t ws_bytes,
                               void* stream) {
  using namespace dr;
  DR_REQUIRE((ev != nullptr) != (table != nullptr), DR_INVALID_ARGUMENT,
             "exactly one of ev / table must be given");
  // the resolve and the pooling that reads the EV's pool are one call on it
  EvGuardRef guard_(ev);
  DR_REQUIRE(nnz >= 0 && batch >= 0 && dim > 0 && out && out_stride >= dim,
             DR_INVALID_ARGUMENT, "bad shape");
  DR_REQUIRE(nnz == 0 || (sp_indices && sp_values), DR_INVALID_ARGUMENT, "null sparse input");
  DR_REQUIRE(combiner >= DR_COMBINER_SUM && combiner <= DR_COMBINER_SQRTN, DR_INVALID_ARGUMENT,
             "combiner must be sum, mean or sqrtn");
  DR_REQUIRE(nnz + batch < (1ll << 31), DR_INVALID_ARGUMENT, "nnz + batch must be < 2^31");
  DR_REQUIRE(ws_bytes >= dr_embedding_lookup_sparse_workspace_size(nnz, batch),
             DR_INVALID_ARGUMENT, "workspace too small");
  if (ev) {
    DR_REQUIRE(dr_ev_dim(ev) == dim, DR_INVALID_ARGUMENT, "dim %d != the EV's %lld", dim,
               (long long)dr_ev_dim(ev));
    // bf16 EVs (BASELINE configs[4]): rows widened to float32 before the
    // pooling, as the reference casts bf16 embeddings (embedding_ops.py:606-607)
    const int vb = dr_ev_value_bits(ev);
    DR_REQUIRE(vb == 32 || (vb == 16 && dim % 8 == 0), DR_INVALID_ARGUMENT,
               "embedding lookups pool float32 EVs, or bf16 EVs with dim %% 8 == 0");
  } else {
    DR_REQUIRE(table_rows >= 0, DR_INVALID_ARGUMENT, "bad table_rows");
  }
  if (batch == 0) return DR_OK;
  hipStream_t st = S(stream);
  LsWs w = carve_ls(ws, nnz, batch, nullptr);
  const int64_t* ind = sp_indices;
  const int64_t* val = sp_values;
  const float* wts = sp_weights;
  const int64_t* n_dev = nullptr;
  int64_t n_cap = nnz;
  int rc;
  if (safe) {
    // _prune_invalid_weights only for weighted non-sum lookups (:1296-1299)
    const int mode = !prune ? 0 : (sp_weights && combiner != DR_COMBINER_SUM ? 2 : 1);
    rc = dr_sparse_prune_fill(sp_indices, 2, sp_values, sp_weights, nnz, batch, mode,
                              default_id >= 0 ? default_id : 0, 1.0f, w.ind, w.val,
                              sp_weights ? w.w : nullptr, nullptr, w.empty, w.n_dev, w.sub,
                              w.sub_bytes, stream);
    if (rc) return rc;
    ind = w.ind;
    val = w.val;
    wts = sp_weights ? w.w : nullptr;
    n_dev = w.n_dev;
    n_cap = nnz + batch;
  }
  rc = n_dev ? dr_bag_offsets_strided_dev(ind, 2, n_cap, n_dev, batch, w.bag_off, stream)
             : dr_bag_offsets_strided(ind, 2, n_cap, batch, w.bag_off, stream);
  if (rc) return rc;
  dr_pool_desc d;
  memset(&d, 0, sizeof(d));
  if (ev) {
    const bool filtered = dr_ev_filter_freq(ev) > 0;
    if (!filtered) {
      rc = dr_ev_resolve(ev, val, n_cap, n_dev, nullptr, nullptr, w.rowsel, w.sub, w.sub_bytes,
                         stream);
      if (rc) return rc;
    } else {
      int64_t n = n_cap;
      if (n_dev) {  // the Unique's input length (see the header comment)
        DR_HIP(hipMemcpyAsync(&n, n_dev, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        DR_HIP(hipStreamSynchronize(st));
      }
      rc = dr_unique(val, n, w.uniq, w.idx, w.cnt, w.U, w.sub, w.sub_bytes, stream);
      if (rc) return rc;
      rc = dr_ev_resolve(ev, w.uniq, n, w.U, nullptr, w.cnt, w.urows, w.sub, w.sub_bytes, stream);
      if (rc) return rc;
      const int64_t koff[2] = {0, n};
      rc = dr_rows_per_nnz(w.urows, w.idx, koff, 1, w.rowsel, stream);
      if (rc) return rc;
    }
    d.pool = dr_ev_pool(ev);  // after the resolve: a growth may have moved it
    d.pool_rows = 1ll << 62;
    d.ids = w.rowsel;
    d.default_rows = dr_ev_default_row(ev);
    d.default_stride = 0;
  } else {
    d.pool = table;
    d.pool_rows = table_rows;
    d.ids = val;
  }
  d.bag_off = w.bag_off;
  d.weights = wts;
  d.out = out;
  d.out_stride = out_stride;
  d.combiner = combiner;
  d.max_norm = max_norm >= 0.f ? max_norm : -1.f;
  const int flags = (ev && dr_ev_value_bits(ev) == 16) ? DR_POOL_BF16 : 0;
  rc = dr_pool_grouped_ex(&d, 1, batch, dim, DR_ORDER_ALI, flags, stream);
  if (rc) return rc;
  if (safe && default_id < 0) {
    hipLaunchKernelGGL(zero_empty_rows_kernel, dim3((unsigned)ceil_div(batch, 4)), dim3(256), 0,
                       st, out, out_stride, batch, dim, w.empty);
    DR_LAUNCH_CHECK();
  }
  return DR_OK;
}

}  // extern "C"
