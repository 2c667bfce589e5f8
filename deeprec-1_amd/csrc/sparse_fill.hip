// sparse_fill.hip -- the SparseTensor preparation of
// safe_embedding_lookup_sparse (python/ops/embedding_ops.py:1289-1310) on the
// GPU in one call: _prune_invalid_ids / _prune_invalid_weights, then
// SparseFillEmptyRows (core/kernels/sparse_fill_empty_rows_op_util.h:17-128).
//
// Output order is the reference's: rows ascending, a row's surviving entries
// in input order, an empty row gets one entry [row, 0, ...] = default.  The
// reference places entry i at scratch[row-1] + filled_count[row]++ in a
// serial loop; here a stable radix sort of (row, i) gives every entry its
// rank inside its row, two scans give the row starts, and the placement is
// one parallel scatter.  No host synchronisation: the output count is
// written to a device word.
#include "dr_common.h"

namespace dr {

// keep flag + row histogram + sort key (row, or `rows` for dropped entries).
__global__ void fill_mark_kernel(const int64_t* __restrict__ ind, int rank,
                                 const int64_t* __restrict__ val, const float* __restrict__ w,
                                 int64_t n, int64_t rows, int prune, int32_t* __restrict__ cnt,
                                 uint64_t* __restrict__ skey, int32_t* __restrict__ pos,
                                 int64_t* __restrict__ rev, int* st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = ind[i * rank];
  bool keep = true;
  if (prune >= 1 && val[i] < 0) keep = false;             // _prune_invalid_ids
  if (prune >= 2 && w && !(w[i] > 0.f)) keep = false;     // _prune_invalid_weights
  if (keep && (r < 0 || r >= rows)) {                     // OP_REQUIRES row in range
    latch(st, DR_INVALID_ARGUMENT);
    keep = false;
  }
  if (keep) atomicAdd(&cnt[r], 1);
  skey[i] = keep ? (uint64_t)r : (uint64_t)rows;
  pos[i] = (int32_t)i;
  if (rev) rev[i] = -1;
}

__global__ void fill_rows_kernel(const int32_t* __restrict__ cnt, int64_t rows,
                                 int32_t* __restrict__ nout, uint8_t* __restrict__ empty) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const int32_t c = cnt[r];
  nout[r] = c > 0 ? c : 1;
  if (empty) empty[r] = c == 0;
}

// sorted position j -> output position row_off[row] + (j - kept_off[row]).
__global__ void fill_place_kernel(const uint64_t* __restrict__ skey, const int32_t* __restrict__ spos,
                                  int64_t n, int64_t rows, const int32_t* __restrict__ kept_off,
                                  const int32_t* __restrict__ row_off,
                                  const int64_t* __restrict__ ind, int rank,
                                  const int64_t* __restrict__ val, const float* __restrict__ w,
                                  int64_t* __restrict__ oind, int64_t* __restrict__ oval,
                                  float* __restrict__ ow, int64_t* __restrict__ rev) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t r = skey[j];
  if (r >= (uint64_t)rows) return;  // dropped entries sort last
  const int64_t i = spos[j];
  const int64_t o = (int64_t)row_off[r] + (j - (int64_t)kept_off[r]);
  for (int c = 0; c < rank; ++c) oind[o * rank + c] = ind[i * rank + c];
  oval[o] = val[i];
  if (ow) ow[o] = w[i];
  if (rev) rev[i] = o;
}

__global__ void fill_empty_kernel(const int32_t* __restrict__ cnt, const int32_t* __restrict__ row_off,
                                  int64_t rows, int rank, int64_t default_value,
                                  float default_weight, int64_t* __restrict__ oind,
                                  int64_t* __restrict__ oval, float* __restrict__ ow) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows || cnt[r] != 0) return;
  const int64_t o = row_off[r];
  oind[o * rank] = r;
  for (int c = 1; c < rank; ++c) oind[o * rank + c] = 0;
  oval[o] = default_value;
  if (ow) ow[o] = default_weight;
}

struct FillWs {
  int32_t* cnt;
  int32_t* nout;
  int32_t* kept_off;
  int32_t* row_off;
  int64_t* totals;  // [2]
  uint64_t* skey;
  uint64_t* skey2;
  int32_t* pos;
  int32_t* pos2;
  void* sort_ws;
  size_t sort_bytes;
  void* scan_ws;
};

static FillWs carve_fill(void* ws, int64_t n, int64_t rows, size_t* used) {
  Carver c(ws);
  FillWs w;
  const int64_t nn = n > 0 ? n : 1, rr = rows > 0 ? rows : 1;
  w.cnt = c.take<int32_t>(rr);
  w.nout = c.take<int32_t>(rr);
  w.kept_off = c.take<int32_t>(rr);
  w.row_off = c.take<int32_t>(rr);
  w.totals = c.take<int64_t>(2);
  w.skey = c.take<uint64_t>(nn);
  w.skey2 = c.take<uint64_t>(nn);
  w.pos = c.take<int32_t>(nn);
  w.pos2 = c.take<int32_t>(nn);
  w.sort_bytes = dr_sort_pairs_workspace_size(nn);
  w.sort_ws = c.take<char>(w.sort_bytes);
  w.scan_ws = c.take<char>(scan_ws_bytes(rr));
  if (used) *used = c.used + 256;
  return w;
}

}  // namespace dr

extern "C" size_t dr_sparse_fill_workspace_size(int64_t nnz, int64_t dense_rows) {
  size_t used = 0;
  dr::carve_fill(nullptr, nnz, dense_rows, &used);
  return used;
}

extern "C" int dr_sparse_prune_fill(const int64_t* indices, int rank, const int64_t* values,
                                    const float* weights, int64_t nnz, int64_t dense_rows,
                                    int prune, int64_t default_value, float default_weight,
                                    int64_t* out_indices, int64_t* out_values, float* out_weights,
                                    int64_t* reverse_index_map, uint8_t* empty_row,
                                    int64_t* out_nnz, void* ws, size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(rank >= 1 && rank <= 8 && nnz >= 0 && dense_rows >= 0 && prune >= 0 && prune <= 2,
             DR_INVALID_ARGUMENT, "dr_sparse_prune_fill: bad argument");
  DR_REQUIRE(nnz < (1ll << 31) && dense_rows < (1ll << 31) && nnz + dense_rows < (1ll << 31),
             DR_INVALID_ARGUMENT, "dr_sparse_prune_fill: sizes must be < 2^31");
  DR_REQUIRE(dense_rows > 0 || nnz == 0, DR_INVALID_ARGUMENT,
             "Received SparseTensor with dense_shape[0] = 0 but indices.shape[0] = %lld",
             (long long)nnz);
  DR_REQUIRE((weights == nullptr) == (out_weights == nullptr), DR_INVALID_ARGUMENT,
             "weights and out_weights go together");
  DR_REQUIRE(ws_bytes >= dr_sparse_fill_workspace_size(nnz, dense_rows), DR_INVALID_ARGUMENT,
             "workspace too small");
  hipStream_t st = S(stream);
  int* stw = status_word();
  DR_REQUIRE(stw, DR_INTERNAL, "status word unavailable");
  if (dense_rows == 0) return fill_bytes(out_nnz, 0, sizeof(int64_t), st);
  FillWs w = carve_fill(ws, nnz, dense_rows, nullptr);
  int rc = fill_bytes(w.cnt, 0, dense_rows * sizeof(int32_t), st);
  if (rc) return rc;
  const unsigned bn = (unsigned)ceil_div(nnz > 0 ? nnz : 1, 256);
  const unsigned br = (unsigned)ceil_div(dense_rows, 256);
  if (nnz > 0) {
    hipLaunchKernelGGL(fill_mark_kernel, dim3(bn), dim3(256), 0, st, indices, rank, values,
                       weights, nnz, dense_rows, prune, w.cnt, w.skey, w.pos, reverse_index_map,
                       stw);
    DR_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(fill_rows_kernel, dim3(br), dim3(256), 0, st, w.cnt, dense_rows, w.nout,
                     empty_row);
  DR_LAUNCH_CHECK();
  rc = scan_exclusive_i32(w.cnt, w.kept_off, dense_rows, nullptr, w.totals, w.scan_ws, st);
  if (rc) return rc;
  rc = scan_exclusive_i32(w.nout, w.row_off, dense_rows, nullptr, out_nnz, w.scan_ws, st);
  if (rc) return rc;
  if (nnz > 0) {
    int bits = 0;
    while (bits < 63 && (1ll << bits) <= dense_rows) ++bits;
    rc = dr_sort_pairs(w.skey, w.pos, w.skey2, w.pos2, nnz, 0, bits, w.sort_ws, w.sort_bytes,
                       stream);
    if (rc) return rc;
    hipLaunchKernelGGL(fill_place_kernel, dim3(bn), dim3(256), 0, st, w.skey2, w.pos2, nnz,
                       dense_rows, w.kept_off, w.row_off, indices, rank, values, weights,
                       out_indices, out_values, out_weights, reverse_index_map);
    DR_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(fill_empty_kernel, dim3(br), dim3(256), 0, st, w.cnt, w.row_off, dense_rows,
                     rank, default_value, default_weight, out_indices, out_values, out_weights);
  DR_LAUNCH_CHECK();
  return DR_OK;
}
