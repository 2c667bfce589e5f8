// dtypes.hip -- the int32-key forms of the key-taking entry points
// (KvResourceGather / Import / Export and Unique are registered for int32
// and int64 keys in the reference: core/kernels/kv_variable_ops.cc:368-388,
// core/kernels/unique_ali_op.cc).  An int32 key is the same key value as its
// sign-extended int64: the keys are widened on the device into the
// workspace, the int64 path runs, and key outputs are narrowed back.
#include "dr_common.h"

namespace dr {

__global__ void widen_i32_kernel(const int32_t* __restrict__ in, int64_t n,
                                 int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int64_t)in[i];
}

__global__ void narrow_i64_kernel(const int64_t* __restrict__ in, int64_t n,
                                  const int64_t* n_dev, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < eff_n(n, n_dev)) out[i] = (int32_t)in[i];
}

static int widen(const int32_t* in, int64_t n, int64_t* out, hipStream_t st) {
  if (n == 0) return DR_OK;
  hipLaunchKernelGGL(widen_i32_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, in, n,
                     out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

static int narrow(const int64_t* in, int64_t n, const int64_t* n_dev, int32_t* out,
                  hipStream_t st) {
  if (n == 0) return DR_OK;
  hipLaunchKernelGGL(narrow_i64_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, in, n,
                     n_dev, out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // namespace dr

extern "C" {

size_t dr_ev_gather_i32_workspace_size(int64_t n) {
  dr::Carver c(nullptr);
  c.take<int64_t>(n > 0 ? n : 1);
  c.take<char>(dr_ev_gather_workspace_size(n));
  return c.used + 256;
}

int dr_ev_gather_i32(dr_ev* ev, const int32_t* keys, int64_t n, const void* defaults,
                     const int32_t* counts, void* out, void* ws, size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(ev && n >= 0, DR_INVALID_ARGUMENT, "bad argument");
  DR_REQUIRE(ws_bytes >= dr_ev_gather_i32_workspace_size(n), DR_INVALID_ARGUMENT,
             "workspace too small");
  if (n == 0) return DR_OK;
  Carver c(ws);
  int64_t* k = c.take<int64_t>(n);
  const size_t gb = dr_ev_gather_workspace_size(n);
  void* gws = c.take<char>(gb);
  int rc = widen(keys, n, k, S(stream));
  if (rc) return rc;
  return dr_ev_gather(ev, k, n, static_cast<const float*>(defaults), counts,
                      static_cast<float*>(out), gws, gb, stream);
}

int dr_ev_insert_i32(dr_ev* ev, const int32_t* keys, int64_t n, const void* values,
                     const int64_t* versions, const int64_t* freqs, int64_t partition_id,
                     int64_t partition_num, void* stream) {
  using namespace dr;
  DR_REQUIRE(ev && n >= 0, DR_INVALID_ARGUMENT, "bad argument");
  if (n == 0) return DR_OK;
  hipStream_t st = S(stream);
  int64_t* k = nullptr;
  DR_HIP(hipMallocAsync((void**)&k, n * sizeof(int64_t), st));
  int rc = widen(keys, n, k, st);
  if (!rc)
    rc = dr_ev_insert(ev, k, n, static_cast<const float*>(values), versions, freqs, partition_id,
                      partition_num, stream);
  (void)hipFreeAsync(k, st);
  return rc;
}

int dr_ev_export_i32(dr_ev* ev, int32_t* keys_out, void* values_out, int64_t* versions_out,
                     int64_t* freqs_out, int64_t capacity, int64_t* m_host, void* stream) {
  using namespace dr;
  DR_REQUIRE(ev && m_host, DR_INVALID_ARGUMENT, "null argument");
  hipStream_t st = S(stream);
  int64_t* k = nullptr;
  if (keys_out && capacity > 0) DR_HIP(hipMallocAsync((void**)&k, capacity * sizeof(int64_t), st));
  int rc = dr_ev_export(ev, k, static_cast<float*>(values_out), versions_out, freqs_out, capacity,
                        m_host, stream);
  if (!rc && k) rc = narrow(k, *m_host, nullptr, keys_out, st);
  if (k) (void)hipFreeAsync(k, st);
  return rc;
}

size_t dr_unique_i32_workspace_size(int64_t n) {
  dr::Carver c(nullptr);
  const int64_t m = n > 0 ? n : 1;
  c.take<int64_t>(m);
  c.take<int64_t>(m);
  c.take<char>(dr_unique_workspace_size(n));
  return c.used + 256;
}

int dr_unique_i32(const int32_t* keys, int64_t n, int32_t* uniq_out, int32_t* idx_out,
                  int32_t* counts_out, int64_t* num_unique, void* ws, size_t ws_bytes,
                  void* stream) {
  using namespace dr;
  DR_REQUIRE(n >= 0 && num_unique, DR_INVALID_ARGUMENT, "bad argument");
  DR_REQUIRE(ws_bytes >= dr_unique_i32_workspace_size(n), DR_INVALID_ARGUMENT,
             "workspace too small");
  Carver c(ws);
  const int64_t m = n > 0 ? n : 1;
  int64_t* k = c.take<int64_t>(m);
  int64_t* y = c.take<int64_t>(m);
  const size_t ub = dr_unique_workspace_size(n);
  void* uws = c.take<char>(ub);
  hipStream_t st = S(stream);
  int rc = widen(keys, n, k, st);
  if (rc) return rc;
  rc = dr_unique(k, n, y, idx_out, counts_out, num_unique, uws, ub, stream);
  if (rc) return rc;
  return narrow(y, n, num_unique, uniq_out, st);
}

}  // extern "C"
