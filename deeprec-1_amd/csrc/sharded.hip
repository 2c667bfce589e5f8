// sharded.hip -- the row-sharded lookup engine as C entries (dr_comm_*,
// dr_sharded_*): what a DeepRec / TF integration binds to drive the
// multi-GPU path through the library, as the reference's multi-GPU
// embedding is a C++ plugin entry (SOK: sparse_operation_kit/kit_cc/
// framework/kernels/dense_fprop.cc:193-212 -> kit_cc_infra/src/embeddings/
// embedding_layer.cc:52-72; NCCL send / recv of the index and row exchange in
// kit_cc_impl/embedding/dispatcher/all2all_input_dispatcher.cu:241-286).
//
// One forward step on `stream` (this rank's T EV shards, owner = key % world):
//   1. grouped first-occurrence Unique of the local ids (skipped for
//      a forward-only one-hot lookup: the raw ids are routed and the owner's
//      insert-on-miss resolve dedups)
//   2. dr_route_by_owner: (owner, table)-blocked send order, counts [G, T]
//   3. counts all-to-all, one host read of the split sizes
//   4. keys all-to-all
//   5. owner: tagged insert-on-miss resolve + row pack of the received keys
//   6. rows all-to-all back (bf16 EVs: bf16 rows, half the link bytes)
//   7. requester: rowsel[perm[j]] = j, then the grouped ALI-order pooling
//      straight from the received rows -- position-ordered, so the result
//      equals the single-GPU lookup bit for bit.
// Backward: per local unique id the SparseSegment*Grad row, packed into the
// forward's send order, all-to-all to the owners, regrouped table-major /
// source-rank-major into the owner's IndexedSlices.
//
// The collective is a dr_comm: RCCL over xGMI (ncclSend / ncclRecv inside
// one group per exchange; librccl is opened on first use), or a callback
// table a host framework supplies.
#include <dlfcn.h>

#include <mutex>
#include <vector>

#include <rccl/rccl.h>

#include "dr_common.h"

struct dr_comm {
  int rank = 0, world = 1;
  int kind = 0;  // 1 = RCCL, 2 = callbacks
  dr_comm_ops ops{};
  ncclComm_t nc = nullptr;
  float* bar = nullptr;  // RCCL: the one-float all-reduce of the stream barrier
};

namespace dr {

// ---- RCCL, opened on first use ----------------------------------------------
struct RcclApi {
  bool ok = false;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) =
      nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                            hipStream_t) = nullptr;
  const char* (*ErrorString)(ncclResult_t) = nullptr;
};

static RcclApi* rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
#define DR_SYM(f, n) api.f = reinterpret_cast<decltype(api.f)>(dlsym(h, n))
    DR_SYM(GetUniqueId, "ncclGetUniqueId");
    DR_SYM(CommInitRank, "ncclCommInitRank");
    DR_SYM(CommDestroy, "ncclCommDestroy");
    DR_SYM(Send, "ncclSend");
    DR_SYM(Recv, "ncclRecv");
    DR_SYM(GroupStart, "ncclGroupStart");
    DR_SYM(GroupEnd, "ncclGroupEnd");
    DR_SYM(ErrorString, "ncclGetErrorString");
    DR_SYM(AllReduce, "ncclAllReduce");
    DR_SYM(AllGather, "ncclAllGather");
#undef DR_SYM
    api.ok = api.GetUniqueId && api.CommInitRank && api.CommDestroy && api.Send && api.Recv &&
             api.GroupStart && api.GroupEnd && api.ErrorString && api.AllReduce && api.AllGather;
  });
  return api.ok ? &api : nullptr;
}

#define DR_NCCL(x)                                                                   \
  do {                                                                               \
    ncclResult_t r_ = (x);                                                           \
    if (r_ != ncclSuccess) {                                                         \
      ::dr::set_error("%s failed: %s", #x, ::dr::rccl()->ErrorString(r_));           \
      return DR_INTERNAL;                                                            \
    }                                                                                \
  } while (0)

static int a2a_v(dr_comm* c, const void* send, const int64_t* sc, void* recv, const int64_t* rc,
                 int64_t eb, hipStream_t st) {
  if (c->kind == 2) {
    const int r = c->ops.all_to_all_v(c->ops.user, send, sc, recv, rc, eb, (void*)st);
    DR_REQUIRE(r == 0, DR_INTERNAL, "dr_comm callback all_to_all_v failed (%d)", r);
    return DR_OK;
  }
  RcclApi* api = rccl();
  DR_REQUIRE(api, DR_INTERNAL, "librccl is not available");
  const char* sp = static_cast<const char*>(send);
  char* rp = static_cast<char*>(recv);
  int64_t so = 0, ro = 0;
  // the self block is a local copy; the others one ncclSend / ncclRecv pair
  // per peer inside one group (all xGMI links at once).  Any failure inside
  // the group still closes it (GroupEnd), or every later collective on this
  // thread's communicator would run inside the dangling group.
  DR_NCCL(api->GroupStart());
  int err = DR_OK;
  for (int p = 0; p < c->world && err == DR_OK; ++p) {
    if (p == c->rank) {
      if (sc[p]) {
        const hipError_t e = hipMemcpyAsync(rp + ro * eb, sp + so * eb, (size_t)(sc[p] * eb),
                                            hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) {
          set_error("self block copy failed: %s", hipGetErrorString(e));
          err = DR_INTERNAL;
        }
      }
    } else {
      int r = 0;
      if (sc[p]) r = api->Send(sp + so * eb, (size_t)(sc[p] * eb), ncclUint8, p, c->nc, st);
      if (r == 0 && rc[p]) r = api->Recv(rp + ro * eb, (size_t)(rc[p] * eb), ncclUint8, p, c->nc, st);
      if (r != 0) {
        set_error("ncclSend/ncclRecv to peer %d failed (%d)", p, r);
        err = DR_INTERNAL;
      }
    }
    so += sc[p];
    ro += rc[p];
  }
  const int ge = api->GroupEnd();
  if (err) return err;
  DR_REQUIRE(ge == 0, DR_INTERNAL, "ncclGroupEnd failed (%d)", ge);
  return DR_OK;
}

// Stream-ordered cross-rank barrier: everything queued on `st` before it, on
// every rank, completes before anything queued after it on any rank (RCCL:
// a one-float all-reduce, which a hipGraph captures; callbacks: ops.barrier).
static int comm_barrier(dr_comm* c, hipStream_t st) {
  if (c->world == 1) return DR_OK;
  if (c->kind == 2) {
    DR_REQUIRE(c->ops.barrier, DR_INVALID_ARGUMENT, "dr_comm_ops.barrier is required");
    const int r = c->ops.barrier(c->ops.user, (void*)st);
    DR_REQUIRE(r == 0, DR_INTERNAL, "dr_comm callback barrier failed (%d)", r);
    return DR_OK;
  }
  RcclApi* api = rccl();
  DR_REQUIRE(api && c->bar, DR_INTERNAL, "librccl is not available");
  DR_NCCL(api->AllReduce(c->bar, c->bar, 1, ncclFloat32, ncclSum, c->nc, st));
  return DR_OK;
}

// All-gather of `bytes` HOST bytes per rank into recv [world][bytes] (setup
// only: synchronous).
static int comm_all_gather_host(dr_comm* c, const void* send, int64_t bytes, void* recv) {
  char* rv = static_cast<char*>(recv);
  if (c->world == 1) {
    memcpy(rv, send, (size_t)bytes);
    return DR_OK;
  }
  if (c->kind == 2) {
    DR_REQUIRE(c->ops.all_gather, DR_INVALID_ARGUMENT, "dr_comm_ops.all_gather is required");
    const int r = c->ops.all_gather(c->ops.user, send, bytes, recv);
    DR_REQUIRE(r == 0, DR_INTERNAL, "dr_comm callback all_gather failed (%d)", r);
    return DR_OK;
  }
  RcclApi* api = rccl();
  DR_REQUIRE(api, DR_INTERNAL, "librccl is not available");
  char* d = nullptr;
  DR_HIP(hipMalloc(&d, (size_t)bytes * (c->world + 1)));
  int rc = DR_OK;
  if (hipMemcpy(d, send, (size_t)bytes, hipMemcpyHostToDevice) != hipSuccess ||
      api->AllGather(d, d + bytes, (size_t)bytes, ncclUint8, c->nc, nullptr) != ncclSuccess ||
      hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(rv, d + bytes, (size_t)bytes * c->world, hipMemcpyDeviceToHost) != hipSuccess) {
    set_error("RCCL all-gather of the engine setup failed");
    rc = DR_INTERNAL;
  }
  (void)hipFree(d);
  return rc;
}

// ---- engine buffers ------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t b) {
    if (b <= bytes) return DR_OK;
    if (p) {
      // an earlier step's kernels may still read it: hipFree synchronises
      DR_HIP(hipFree(p));
      p = nullptr;
      bytes = 0;
    }
    size_t nb = b < 256 ? 256 : b;
    nb += nb / 4;   // grow ahead
    DR_HIP(hipMalloc(&p, nb));
    bytes = nb;
    return DR_OK;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

// tags_r[i] = table of received key i: blocks (peer p, table t) of
// rc[p][t] keys in peer-major order (boff: prefix offsets, G*T + 1)
__global__ void sh_tags_kernel(const int64_t* __restrict__ boff, int GT, int T, int64_t R,
                               int32_t* __restrict__ tags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R) return;
  int lo = 0, hi = GT - 1;   // last block with boff <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (boff[mid] <= i)
      lo = mid;
    else
      hi = mid - 1;
  }
  tags[i] = (int32_t)(lo % T);
}

// rowsel[perm[j]] = j: the received row of each routed position
__global__ void sh_rowsel_kernel(const int32_t* __restrict__ perm, int64_t S,
                                 int64_t* __restrict__ rowsel) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < S) rowsel[perm[j]] = j;
}

// seg[k] = bag of position k (CSR bag offsets -> per-position bag ids)
__global__ void sh_seg_kernel(const int32_t* __restrict__ off, int64_t bags,
                              int64_t* __restrict__ seg) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= bags) return;
  for (int32_t k = off[b]; k < off[b + 1]; ++k) seg[k] = b;
}

// Received grads are [peer][table] blocks; the owner's slices are table-major,
// source-rank-major inside a table: dst = dbase[p*T + t] + (i - boff[p*T + t]).
__global__ void sh_regroup_kernel(const int64_t* __restrict__ boff,
                                  const int64_t* __restrict__ dbase, int GT, int64_t R,
                                  const int64_t* __restrict__ keys_r, int64_t* __restrict__ keys_t,
                                  int32_t* __restrict__ permt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R) return;
  int lo = 0, hi = GT - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (boff[mid] <= i)
      lo = mid;
    else
      hi = mid - 1;
  }
  const int64_t d = dbase[lo] + (i - boff[lo]);
  keys_t[d] = keys_r[i];
  permt[d] = (int32_t)i;
}

// ---- fixed-capacity exchange (DR_SHARDED_RCCL_FIXED): no host read ---------
// Every rank sends each peer a region of `cap` keys (the first c_q hold the
// keys it routes there), the [G, T] counts travel in a header, and every
// kernel after the all-to-all takes its sizes from those device counts.
constexpr int kFxMaxGT = DR_MAX_PEERS * DR_MAX_GROUP;

// blocks' shared view of a [G, T] count matrix: per-peer totals and their
// exclusive prefix (off[G] = total)
struct FxCounts {
  int64_t tot[DR_MAX_PEERS];
  int64_t off[DR_MAX_PEERS + 1];
};
__device__ void fx_load(const int64_t* __restrict__ c, int G, int T, FxCounts& f) {
  if (threadIdx.x == 0) {
    int64_t a = 0;
    for (int q = 0; q < G; ++q) {
      int64_t v = 0;
      for (int t = 0; t < T; ++t) v += c[q * T + t];
      f.tot[q] = v;
      f.off[q] = a;
      a += v;
    }
    f.off[G] = a;
  }
  __syncthreads();
}

// sender: keys / tags of owner q's block into region q, the header, an
// overflow latch when a block exceeds the region
__global__ void fx_pack_kernel(const int64_t* __restrict__ keys_s, const int32_t* __restrict__ tags_s,
                               const int64_t* __restrict__ counts, int G, int T, int64_t cap,
                               int64_t* __restrict__ kf, int32_t* __restrict__ tf,
                               int64_t* __restrict__ hf, int* st) {
  __shared__ FxCounts f;
  fx_load(counts, G, T, f);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (int64_t)G * T) hf[i] = counts[i];
  if (i >= (int64_t)G * cap) return;
  const int q = (int)(i / cap);
  const int64_t j = i - (int64_t)q * cap;
  if (j == 0 && f.tot[q] > cap) latch(st, DR_RESOURCE_EXHAUSTED);
  const bool v = j < f.tot[q];
  kf[i] = v ? keys_s[f.off[q] + j] : 0;
  tf[i] = v ? tags_s[f.off[q] + j] : 0;
}

// owner: the valid keys of every received region, compacted peer-major
__global__ void fx_compact_kernel(const int64_t* __restrict__ kr, const int32_t* __restrict__ tr,
                                  const int64_t* __restrict__ hr, int G, int T, int64_t cap,
                                  int64_t* __restrict__ kc, int32_t* __restrict__ tc,
                                  int64_t* __restrict__ rtot) {
  __shared__ FxCounts f;
  fx_load(hr, G, T, f);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) rtot[0] = f.off[G];
  if (i >= (int64_t)G * cap) return;
  const int q = (int)(i / cap);
  const int64_t j = i - (int64_t)q * cap;
  if (j < f.tot[q] && j < cap) {
    kc[f.off[q] + j] = kr[i];
    tc[f.off[q] + j] = tr[i];
  }
}

// owner: resolved rows back into the fixed region layout (padding: row -1,
// table 0 -- a default row, never read by the requester)
__global__ void fx_expand_kernel(const int64_t* __restrict__ rows_c, const int32_t* __restrict__ tr,
                                 const int64_t* __restrict__ hr, int G, int T, int64_t cap,
                                 int64_t* __restrict__ rows_f, int32_t* __restrict__ tags_f) {
  __shared__ FxCounts f;
  fx_load(hr, G, T, f);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)G * cap) return;
  const int q = (int)(i / cap);
  const int64_t j = i - (int64_t)q * cap;
  const bool v = j < f.tot[q];
  rows_f[i] = v ? rows_c[f.off[q] + j] : -1;
  tags_f[i] = v ? tr[i] : 0;
}

// requester: rowsel[perm[j]] = the received row of routed position j
// (owner q's block [off_q, off_q + c_q) came back at region q)
__global__ void fx_rowsel_kernel(const int32_t* __restrict__ perm, const int64_t* __restrict__ counts,
                                 int G, int T, int64_t cap, int64_t n, int64_t* __restrict__ rowsel) {
  __shared__ FxCounts f;
  fx_load(counts, G, T, f);
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || j >= f.off[G]) return;
  int q = 0;
  while (q + 1 < G && j >= f.off[q + 1]) ++q;
  rowsel[perm[j]] = (int64_t)q * cap + (j - f.off[q]);
}

// requester: gradient rows into the fixed regions (perm: send position ->
// grouped-unique row of gu); padding rows zero.  One 64-lane wave per row.
__global__ void fx_grad_pack_kernel(const float* __restrict__ gu, const int32_t* __restrict__ perm,
                                    const int64_t* __restrict__ counts, int G, int T, int64_t cap,
                                    int D, float* __restrict__ gf) {
  __shared__ FxCounts f;
  fx_load(counts, G, T, f);
  const int64_t i = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (i >= (int64_t)G * cap) return;
  const int q = (int)(i / cap);
  const int64_t j = i - (int64_t)q * cap;
  float* dst = gf + i * D;
  if (j < f.tot[q]) {
    const float* src = gu + (int64_t)perm[f.off[q] + j] * D;
    for (int c = lane; c < D; c += 64) dst[c] = src[c];
  } else {
    for (int c = lane; c < D; c += 64) dst[c] = 0.f;
  }
}

// owner: received gradient rows regrouped table-major, source-rank-major
// into fixed per-table regions of tcap rows; cnt_t[t] = rows of table t
__global__ void fx_regroup_kernel(const int64_t* __restrict__ kr, const int32_t* __restrict__ tr,
                                  const float* __restrict__ gr, const int64_t* __restrict__ hr,
                                  int G, int T, int64_t cap, int64_t tcap, int D,
                                  int64_t* __restrict__ keys_t, float* __restrict__ grads_t,
                                  int64_t* __restrict__ cnt_t) {
  __shared__ FxCounts f;
  __shared__ int64_t inreg[kFxMaxGT];   // region q: start of table t's block
  __shared__ int64_t pre[kFxMaxGT];     // table t's region: start of source q's rows
  fx_load(hr, G, T, f);
  if (threadIdx.x == 0) {
    for (int q = 0; q < G; ++q) {
      int64_t a = 0;
      for (int t = 0; t < T; ++t) {
        inreg[q * T + t] = a;
        a += hr[q * T + t];
      }
    }
    for (int t = 0; t < T; ++t) {
      int64_t a = 0;
      for (int q = 0; q < G; ++q) {
        pre[q * T + t] = a;
        a += hr[q * T + t];
      }
      if (blockIdx.x == 0) cnt_t[t] = a;
    }
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (i >= (int64_t)G * cap) return;
  const int q = (int)(i / cap);
  const int64_t j = i - (int64_t)q * cap;
  if (j >= f.tot[q]) return;
  const int t = tr[i];
  const int64_t d = (int64_t)t * tcap + pre[q * T + t] + (j - inreg[q * T + t]);
  if (lane == 0) keys_t[d] = kr[i];
  for (int c = lane; c < D; c += 64) grads_t[d * D + c] = gr[i * D + c];
}

// plain row copies between engine buffers (kernels, not DMA: graph-safe);
// bf16 -> fp32 widening of the XGMI kind's bf16 output
__global__ void fx_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
__global__ void fx_widen_kernel(const uint16_t* __restrict__ src, float* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = __uint_as_float((uint32_t)src[i] << 16);
}

static int copy_bytes(void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (!bytes) return DR_OK;
  DR_REQUIRE(bytes % 16 == 0 && ((uintptr_t)dst | (uintptr_t)src) % 16 == 0, DR_INVALID_ARGUMENT,
             "engine copies need 16-B aligned, 16-B multiple buffers");
  const int64_t n16 = (int64_t)(bytes / 16);
  hipLaunchKernelGGL(fx_copy_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n16, 256), 8192)),
                     dim3(256), 0, st, static_cast<const uint4*>(src), static_cast<uint4*>(dst),
                     n16);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // namespace dr

struct dr_sharded {
  dr_comm* comm = nullptr;
  std::vector<dr_ev*> evs;
  int T = 0;
  int64_t dim = 0;
  int bf16 = 0;
  int kind = DR_SHARDED_RCCL;
  // DR_SHARDED_XGMI: peer-write exchange over IPC-mapped buffers
  int64_t batch = 0;
  dr_xgmi_peers peers{};
  void* own[5] = {};            // inbox_keys, inbox_slot, inbox_cnt, out, gin (dr_ipc_alloc)
  std::vector<void*> bases;     // peers' mappings (dr_ipc_import)
  const float* gin_peer[DR_MAX_PEERS] = {};
  // DR_SHARDED_RCCL_FIXED: per-peer regions of `cap` keys, counts in a header
  int64_t max_ids = 0, cap = 0;
  dr::DevBuf xcnt, xws, pkeys, pgrads, pcounts, kf, tf, hf, kr, tr, hr, kc, tc, rtot, rows_c,
      rows_f, tags_f;
  bool fx_saved = false;
  int64_t fx_n = 0;
  dr::DevBuf uniq, idx, U, keys_s, tags_s, perm, counts, keys_r, tags_r, rows, rows_s, rows_r,
      rowsel, ws, seg, gu, grads_s, grads_r, keys_t, grads_t, permt, blk;
  int64_t* host = nullptr;   // pinned: counts [G*T], received counts [G*T], offsets
  hipEvent_t up_ev = nullptr;  // the last upload of the offsets has been read
  // the last need_grad forward
  bool saved = false;
  std::vector<int64_t> koff;
  int64_t bags = 0, S = 0, R = 0;
  int combiner = 0;
  std::vector<const int32_t*> bag_off;
  std::vector<int64_t> send, recv, rc;
  int64_t last_sent = 0, last_recv = 0;
};

namespace dr {

// boff (prefix of rc, peer-major, G*T + 1) and, for the backward, the
// table-major destination base of every (p, t) block, into the device block
// buffer: [boff | dbase]
static int upload_blocks(dr_sharded* s, const std::vector<int64_t>& rc, hipStream_t st) {
  const int G = s->comm->world, T = s->T, GT = G * T;
  // the previous upload (possibly on another stream) has left the staging area
  DR_HIP(hipEventSynchronize(s->up_ev));
  int64_t* h = s->host + 2 * GT;
  h[0] = 0;
  for (int i = 0; i < GT; ++i) h[i + 1] = h[i] + rc[i];
  std::vector<int64_t> toff(T + 1, 0);
  for (int t = 0; t < T; ++t) {
    int64_t n = 0;
    for (int p = 0; p < G; ++p) n += rc[p * T + t];
    toff[t + 1] = toff[t] + n;
  }
  int64_t* db = h + GT + 1;
  for (int t = 0; t < T; ++t) {
    int64_t a = toff[t];
    for (int p = 0; p < G; ++p) {
      db[p * T + t] = a;
      a += rc[p * T + t];
    }
  }
  int rc_ = s->blk.ensure((size_t)(2 * GT + 1) * sizeof(int64_t));
  if (rc_) return rc_;
  DR_HIP(hipMemcpyAsync(s->blk.p, h, (size_t)(2 * GT + 1) * sizeof(int64_t),
                        hipMemcpyHostToDevice, st));
  DR_HIP(hipEventRecord(s->up_ev, st));
  return DR_OK;
}

// ---- DR_SHARDED_XGMI: the peer-write exchange inside the library ----------
// (the orchestration of sharded.py XgmiShardedLookup: route -> barrier ->
// serve -> barrier; backward: gradient into the shared buffer -> barrier ->
// owner pull -> barrier), the IPC handle exchange and the barriers through
// the dr_comm.
static int xgmi_setup(dr_sharded* s) {
  dr_comm* c = s->comm;
  const int G = c->world, T = s->T;
  const int64_t B = s->batch, cap = (int64_t)T * B;
  const size_t vb = s->bf16 ? 2 : 4;
  const size_t bytes[5] = {(size_t)G * cap * 8, (size_t)G * cap * 4, (size_t)G * 8,
                           (size_t)B * T * s->dim * vb, (size_t)B * T * s->dim * 4};
  int rc = DR_OK;
  for (int k = 0; k < 5 && rc == DR_OK; ++k) rc = dr_ipc_alloc(bytes[k], &s->own[k]);
  // the handle exchange runs on every rank even after a local failure (the
  // failure travels in the record), so no rank waits on another
  struct Rec {
    int32_t ok, pad;
    int64_t off[5];
    char h[5][DR_IPC_HANDLE_BYTES];
  };
  Rec mine;
  memset(&mine, 0, sizeof(mine));
  mine.ok = rc == DR_OK;
  if (G > 1)
    for (int k = 0; k < 5 && mine.ok; ++k)
      mine.ok = dr_ipc_export(s->own[k], mine.h[k], &mine.off[k]) == DR_OK;
  std::vector<Rec> all(G);
  int arc = comm_all_gather_host(c, &mine, sizeof(Rec), all.data());
  if (arc) return arc;
  for (int q = 0; q < G; ++q)
    DR_REQUIRE(all[q].ok, DR_INTERNAL, "xgmi engine setup failed on rank %d", q);
  void* ptrs[DR_MAX_PEERS][5];
  for (int q = 0; q < G; ++q)
    for (int k = 0; k < 5; ++k) {
      if (q == c->rank) {
        ptrs[q][k] = s->own[k];
        continue;
      }
      void* base = nullptr;
      int irc = dr_ipc_import(all[q].h[k], all[q].off[k], &ptrs[q][k], &base);
      if (irc) return irc;
      s->bases.push_back(base);
    }
  s->peers.world = G;
  s->peers.rank = c->rank;
  s->peers.cap = cap;
  for (int q = 0; q < G; ++q) {
    s->peers.inbox_keys[q] = static_cast<int64_t*>(ptrs[q][0]);
    s->peers.inbox_slot[q] = static_cast<int32_t*>(ptrs[q][1]);
    s->peers.inbox_cnt[q] = static_cast<int64_t*>(ptrs[q][2]);
    s->peers.out[q] = static_cast<float*>(ptrs[q][3]);
    s->gin_peer[q] = static_cast<const float*>(ptrs[q][4]);
  }
  int e = s->xcnt.ensure((size_t)G * 8);
  if (!e) e = s->xws.ensure(std::max(dr_xgmi_serve_workspace_size(G, cap),
                                     dr_xgmi_grad_pull_dev_workspace_size(G, cap)));
  if (!e) e = s->pkeys.ensure((size_t)T * G * B * 8);
  if (!e) e = s->pgrads.ensure((size_t)T * G * B * s->dim * 4);
  if (!e) e = s->pcounts.ensure((size_t)T * 8);
  return e;
}

static int xgmi_forward(dr_sharded* s, const int64_t* ids, const int64_t* koff_host,
                        const int32_t* const* bag_off, int64_t bags, int combiner, int need_grad,
                        int flags, void* out, void* stream) {
  const int T = s->T;
  const int64_t B = s->batch;
  DR_REQUIRE(!bag_off && bags == B && combiner == DR_COMBINER_SUM, DR_INVALID_ARGUMENT,
             "the XGMI kind takes one-hot ids, bags == the engine's batch (%lld), sum",
             (long long)B);
  for (int t = 0; koff_host && t <= T; ++t)
    DR_REQUIRE(koff_host[t] == (int64_t)t * B, DR_INVALID_ARGUMENT, "one-hot koff_host expected");
  DR_REQUIRE(ids, DR_INVALID_ARGUMENT, "null ids");
  hipStream_t st = S(stream);
  int rc = dr_xgmi_route_ex(&s->peers, ids, T, B, nullptr, s->xcnt.as<int64_t>(), stream);
  if (!rc) rc = comm_barrier(s->comm, st);
  if (!rc) rc = dr_xgmi_serve(&s->peers, s->evs.data(), T, B, s->xws.p, s->xws.bytes, stream);
  if (!rc) rc = comm_barrier(s->comm, st);
  if (rc) return rc;
  s->saved = need_grad != 0;
  s->last_sent = s->last_recv = -1;   // (device counts: not read back)
  if (!out) return DR_OK;   // the result stays in the engine buffer (dr_sharded_output)
  const int64_t nv = B * T * s->dim;
  if (s->bf16 && !(flags & DR_SHARDED_OUT_BF16)) {
    hipLaunchKernelGGL(fx_widen_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(nv, 256), 8192)),
                       dim3(256), 0, st, static_cast<const uint16_t*>(s->own[3]),
                       static_cast<float*>(out), nv);
    DR_LAUNCH_CHECK();
    return DR_OK;
  }
  return copy_bytes(out, s->own[3], (size_t)nv * (s->bf16 ? 2 : 4), st);
}

static int xgmi_backward(dr_sharded* s, const float* grad, void* stream) {
  hipStream_t st = S(stream);
  int rc = copy_bytes(s->own[4], grad, (size_t)s->batch * s->T * s->dim * 4, st);
  if (!rc) rc = comm_barrier(s->comm, st);
  if (!rc)
    rc = dr_xgmi_grad_pull_dev(&s->peers, s->gin_peer, s->T, s->batch, (int)s->dim,
                               s->pkeys.as<int64_t>(), s->pgrads.as<float>(),
                               s->pcounts.as<int64_t>(), s->xws.p, s->xws.bytes, stream);
  // no peer's next route may overwrite the inbox before this pull
  if (!rc) rc = comm_barrier(s->comm, st);
  return rc;
}

// ---- DR_SHARDED_RCCL_FIXED: the all-to-all engine without a host read ----
static int fixed_forward(dr_sharded* s, const int64_t* ids, const int64_t* koff_host,
                         const int32_t* const* bag_off, int64_t bags, int combiner, int need_grad,
                         int flags, void* out, void* stream) {
  const int T = s->T, G = s->comm->world, GT = G * T;
  const int64_t D = s->dim, cap = s->cap;
  DR_REQUIRE(out && bags >= 0, DR_INVALID_ARGUMENT, "bad argument");
  DR_REQUIRE(!(flags & DR_SHARDED_OUT_BF16) || s->bf16, DR_INVALID_ARGUMENT,
             "a bf16 output needs bf16 EVs");
  std::vector<int64_t> koff(T + 1);
  for (int t = 0; t <= T; ++t) koff[t] = koff_host ? koff_host[t] : (int64_t)t * bags;
  DR_REQUIRE(koff[0] == 0, DR_INVALID_ARGUMENT, "koff_host[0] must be 0");
  for (int t = 0; t < T; ++t) {
    DR_REQUIRE(koff[t + 1] >= koff[t] && koff[t + 1] - koff[t] <= s->max_ids, DR_INVALID_ARGUMENT,
               "table %d: %lld ids, the engine's max_ids is %lld", t,
               (long long)(koff[t + 1] - koff[t]), (long long)s->max_ids);
    DR_REQUIRE(bag_off || koff[t + 1] - koff[t] == bags, DR_INVALID_ARGUMENT,
               "table %d: one-hot ids need `bags` ids", t);
  }
  const int64_t n = koff[T], nn = n > 0 ? n : 1;
  DR_REQUIRE(ids || n == 0, DR_INVALID_ARGUMENT, "null ids");
  hipStream_t st = S(stream);
  const bool direct = !need_grad && !bag_off;
  const size_t vrow = (size_t)D * (s->bf16 ? 2 : 4);
  int rc;
#define DR_ENS(buf, bytes)             \
  do {                                 \
    rc = (buf).ensure((size_t)(bytes)); \
    if (rc) return rc;                 \
  } while (0)
  DR_ENS(s->keys_s, nn * 8);
  DR_ENS(s->tags_s, nn * 4);
  DR_ENS(s->perm, nn * 4);
  DR_ENS(s->counts, (size_t)GT * 8);
  DR_ENS(s->rowsel, nn * 8);
  const int64_t GC = (int64_t)G * cap;
  DR_ENS(s->kf, GC * 8);
  DR_ENS(s->tf, GC * 4);
  DR_ENS(s->hf, (size_t)GT * 8);
  DR_ENS(s->kr, GC * 8);
  DR_ENS(s->tr, GC * 4);
  DR_ENS(s->hr, (size_t)GT * 8);
  DR_ENS(s->kc, GC * 8);
  DR_ENS(s->tc, GC * 4);
  DR_ENS(s->rtot, 8);
  DR_ENS(s->rows_c, GC * 8);
  DR_ENS(s->rows_f, GC * 8);
  DR_ENS(s->tags_f, GC * 4);
  DR_ENS(s->rows_s, GC * vrow);
  DR_ENS(s->rows_r, GC * vrow);
  size_t wsb = std::max(dr_route_workspace_size(n, G, T), dr_ev_resolve_workspace_size(GC));
  if (!direct) {
    wsb = std::max(wsb, dr_unique_grouped_workspace_size(koff.data(), T));
    DR_ENS(s->uniq, nn * 8);
    DR_ENS(s->idx, nn * 4);
    DR_ENS(s->U, (size_t)T * 8);
  }
  DR_ENS(s->ws, wsb);
  const int64_t* src = ids;
  const int64_t* nu = nullptr;
  if (!direct) {
    rc = dr_unique_grouped(ids, koff.data(), T, s->uniq.as<int64_t>(), s->idx.as<int32_t>(),
                           nullptr, s->U.as<int64_t>(), s->ws.p, s->ws.bytes, stream);
    if (rc) return rc;
    src = s->uniq.as<int64_t>();
    nu = s->U.as<int64_t>();
  }
  rc = dr_route_by_owner(src, koff.data(), T, nu, G, s->keys_s.as<int64_t>(),
                         s->tags_s.as<int32_t>(), s->perm.as<int32_t>(), s->counts.as<int64_t>(),
                         s->ws.p, s->ws.bytes, stream);
  if (rc) return rc;
  int* stw = status_word();
  DR_REQUIRE(stw, DR_INTERNAL, "status word unavailable");
  const unsigned gb = (unsigned)ceil_div(std::max<int64_t>(GC, GT), 256);
  hipLaunchKernelGGL(fx_pack_kernel, dim3(gb), dim3(256), 0, st, s->keys_s.as<int64_t>(),
                     s->tags_s.as<int32_t>(), s->counts.as<int64_t>(), G, T, cap,
                     s->kf.as<int64_t>(), s->tf.as<int32_t>(), s->hf.as<int64_t>(), stw);
  DR_LAUNCH_CHECK();
  // fixed sizes: header T, keys / tags cap per peer
  std::vector<int64_t> hT(G, T), hC(G, cap);
  rc = a2a_v(s->comm, s->hf.p, hT.data(), s->hr.p, hT.data(), 8, st);
  if (!rc) rc = a2a_v(s->comm, s->kf.p, hC.data(), s->kr.p, hC.data(), 8, st);
  if (!rc) rc = a2a_v(s->comm, s->tf.p, hC.data(), s->tr.p, hC.data(), 4, st);
  if (rc) return rc;
  // owner: compact, resolve (device count), rows back into region layout
  hipLaunchKernelGGL(fx_compact_kernel, dim3((unsigned)ceil_div(GC, 256)), dim3(256), 0, st,
                     s->kr.as<int64_t>(), s->tr.as<int32_t>(), s->hr.as<int64_t>(), G, T, cap,
                     s->kc.as<int64_t>(), s->tc.as<int32_t>(), s->rtot.as<int64_t>());
  DR_LAUNCH_CHECK();
  // capacity accounting: at most G * max_ids keys of a table arrive per step
  std::vector<int64_t> per_table(T, (int64_t)G * s->max_ids);
  rc = dr_ev_resolve_tagged(s->evs.data(), T, s->kc.as<int64_t>(), s->tc.as<int32_t>(), GC,
                            s->rtot.as<int64_t>(), per_table.data(), nullptr,
                            s->rows_c.as<int64_t>(), s->ws.p, s->ws.bytes, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(fx_expand_kernel, dim3((unsigned)ceil_div(GC, 256)), dim3(256), 0, st,
                     s->rows_c.as<int64_t>(), s->tr.as<int32_t>(), s->hr.as<int64_t>(), G, T, cap,
                     s->rows_f.as<int64_t>(), s->tags_f.as<int32_t>());
  DR_LAUNCH_CHECK();
  rc = dr_ev_gather_tagged(s->evs.data(), T, s->tags_f.as<int32_t>(), s->rows_f.as<int64_t>(), GC,
                           nullptr, s->rows_s.as<float>(), stream);
  if (!rc) rc = a2a_v(s->comm, s->rows_s.p, hC.data(), s->rows_r.p, hC.data(), (int64_t)vrow, st);
  if (rc) return rc;
  // requester: pool straight from the received regions
  if (n > 0) {
    hipLaunchKernelGGL(fx_rowsel_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st,
                       s->perm.as<int32_t>(), s->counts.as<int64_t>(), G, T, cap, n,
                       s->rowsel.as<int64_t>());
    DR_LAUNCH_CHECK();
  }
  if (bags > 0) {
    std::vector<dr_pool_desc> d(T);
    const size_t ob = (flags & DR_SHARDED_OUT_BF16) ? 2 : 4;
    for (int t = 0; t < T; ++t) {
      memset(&d[t], 0, sizeof(dr_pool_desc));
      d[t].pool = s->rows_r.as<float>();
      if (direct) {
        d[t].ids = s->rowsel.as<int64_t>() + koff[t];
        d[t].pool_rows = GC;
      } else {
        d[t].idx = s->idx.as<int32_t>() + koff[t];
        d[t].rows = s->rowsel.as<int64_t>() + koff[t];
      }
      d[t].default_rows = s->rows_r.as<float>();
      d[t].default_stride = 0;
      d[t].bag_off = bag_off ? bag_off[t] : nullptr;
      d[t].out = reinterpret_cast<float*>(static_cast<char*>(out) + ob * (size_t)t * D);
      d[t].out_stride = (int64_t)T * D;
      d[t].combiner = combiner;
      d[t].max_norm = -1.f;
    }
    const int pf = (bag_off ? 0 : DR_POOL_ONEHOT) | (s->bf16 ? DR_POOL_BF16 : 0) |
                   ((flags & DR_SHARDED_OUT_BF16) ? DR_POOL_OUT_BF16 : 0);
    rc = dr_pool_grouped_ex(d.data(), T, bags, (int)D, DR_ORDER_ALI, pf, stream);
    if (rc) return rc;
  }
  s->last_sent = s->last_recv = -1;   // (device counts: not read back)
  s->fx_saved = need_grad != 0;
  if (need_grad) {
    s->koff = koff;
    s->bags = bags;
    s->combiner = combiner;
    s->bag_off.assign(T, nullptr);
    if (bag_off)
      for (int t = 0; t < T; ++t) s->bag_off[t] = bag_off[t];
  }
  return DR_OK;
#undef DR_ENS
}

static int fixed_backward(dr_sharded* s, const float* grad, void* stream) {
  hipStream_t st = S(stream);
  const int T = s->T, G = s->comm->world;
  const std::vector<int64_t>& koff = s->koff;
  const int64_t D = s->dim, n = koff[T], nn = n > 0 ? n : 1, cap = s->cap;
  const int64_t GC = (int64_t)G * cap, tcap = (int64_t)G * s->max_ids;
  int rc;
#define DR_ENS(buf, bytes)             \
  do {                                 \
    rc = (buf).ensure((size_t)(bytes)); \
    if (rc) return rc;                 \
  } while (0)
  DR_ENS(s->gu, (size_t)nn * D * 4);
  DR_ENS(s->grads_s, (size_t)GC * D * 4);
  DR_ENS(s->grads_r, (size_t)GC * D * 4);
  DR_ENS(s->pkeys, (size_t)T * tcap * 8);
  DR_ENS(s->pgrads, (size_t)T * tcap * D * 4);
  DR_ENS(s->pcounts, (size_t)T * 8);
  const bool multi = s->bag_off[0] != nullptr;
  if (multi) DR_ENS(s->seg, nn * 8);
  const size_t wsb = dr_pool_grad_grouped_workspace_size(n);
  if (wsb > s->ws.bytes) DR_ENS(s->ws, wsb);
#undef DR_ENS
  if (n > 0 && s->bags > 0) {
    std::vector<dr_pool_grad_desc> d(T);
    for (int t = 0; t < T; ++t) {
      memset(&d[t], 0, sizeof(dr_pool_grad_desc));
      d[t].top_grad = grad + (size_t)t * D;
      d[t].top_stride = (int64_t)T * D;
      if (multi) {
        int64_t* sg = s->seg.as<int64_t>() + koff[t];
        hipLaunchKernelGGL(sh_seg_kernel, dim3((unsigned)ceil_div(s->bags, 256)), dim3(256), 0,
                           st, s->bag_off[t], s->bags, sg);
        DR_LAUNCH_CHECK();
        d[t].bag_off = s->bag_off[t];
        d[t].seg = sg;
        d[t].seg_stride = 1;
      }
      d[t].idx = s->idx.as<int32_t>() + koff[t];
      d[t].nnz = koff[t + 1] - koff[t];
      d[t].num_unique = s->U.as<int64_t>() + t;
      d[t].combiner = s->combiner;
    }
    rc = dr_pool_grad_grouped(d.data(), T, s->bags, (int)D, s->gu.as<float>(), s->ws.p,
                              s->ws.bytes, stream);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(fx_grad_pack_kernel, dim3((unsigned)ceil_div(GC, 4)), dim3(256), 0, st,
                     s->gu.as<float>(), s->perm.as<int32_t>(), s->counts.as<int64_t>(), G, T, cap,
                     (int)D, s->grads_s.as<float>());
  DR_LAUNCH_CHECK();
  std::vector<int64_t> hC(G, cap);
  rc = a2a_v(s->comm, s->grads_s.p, hC.data(), s->grads_r.p, hC.data(), D * 4, st);
  if (rc) return rc;
  hipLaunchKernelGGL(fx_regroup_kernel, dim3((unsigned)ceil_div(GC, 4)), dim3(256), 0, st,
                     s->kr.as<int64_t>(), s->tr.as<int32_t>(), s->grads_r.as<float>(),
                     s->hr.as<int64_t>(), G, T, cap, tcap, (int)D, s->pkeys.as<int64_t>(),
                     s->pgrads.as<float>(), s->pcounts.as<int64_t>());
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // namespace dr

extern "C" {

int dr_comm_rccl_unique_id(void* out, int64_t bytes) {
  using namespace dr;
  DR_REQUIRE(out && bytes >= (int64_t)sizeof(ncclUniqueId), DR_INVALID_ARGUMENT,
             "need %d bytes", (int)sizeof(ncclUniqueId));
  RcclApi* api = rccl();
  DR_REQUIRE(api, DR_INTERNAL, "librccl is not available");
  ncclUniqueId id;
  DR_NCCL(api->GetUniqueId(&id));
  memcpy(out, &id, sizeof(id));
  return DR_OK;
}

int dr_comm_init(const void* rccl_unique_id, int rank, int world, const dr_comm_ops* ops,
                 dr_comm** out) {
  using namespace dr;
  DR_REQUIRE(out && world >= 1 && world <= DR_MAX_PEERS && rank >= 0 && rank < world,
             DR_INVALID_ARGUMENT, "bad rank / world");
  DR_REQUIRE((rccl_unique_id != nullptr) != (ops != nullptr), DR_INVALID_ARGUMENT,
             "exactly one of rccl_unique_id / ops");
  DR_REQUIRE(!ops || ops->all_to_all_v, DR_INVALID_ARGUMENT, "ops.all_to_all_v is required");
  dr_comm* c = new (std::nothrow) dr_comm();
  DR_REQUIRE(c, DR_RESOURCE_EXHAUSTED, "out of host memory");
  c->rank = rank;
  c->world = world;
  if (ops) {
    c->kind = 2;
    c->ops = *ops;
  } else {
    RcclApi* api = rccl();
    if (!api) {
      delete c;
      set_error("librccl is not available");
      return DR_INTERNAL;
    }
    ncclUniqueId id;
    memcpy(&id, rccl_unique_id, sizeof(id));
    const ncclResult_t r = api->CommInitRank(&c->nc, world, id, rank);
    if (r != ncclSuccess) {
      delete c;
      set_error("ncclCommInitRank failed: %s", api->ErrorString(r));
      return DR_INTERNAL;
    }
    c->kind = 1;
    if (hipMalloc(&c->bar, sizeof(float)) != hipSuccess ||
        hipMemset(c->bar, 0, sizeof(float)) != hipSuccess) {
      api->CommDestroy(c->nc);
      delete c;
      set_error("hipMalloc of the barrier word failed");
      return DR_INTERNAL;
    }
  }
  *out = c;
  return DR_OK;
}

int dr_comm_destroy(dr_comm* comm) {
  if (!comm) return DR_OK;
  if (comm->kind == 1 && comm->nc && dr::rccl()) dr::rccl()->CommDestroy(comm->nc);
  if (comm->bar) (void)hipFree(comm->bar);
  delete comm;
  return DR_OK;
}

int dr_comm_rank(const dr_comm* comm) { return comm ? comm->rank : -1; }
int dr_comm_world(const dr_comm* comm) { return comm ? comm->world : -1; }

int dr_comm_all_to_all_v(dr_comm* comm, const void* send, const int64_t* send_counts, void* recv,
                         const int64_t* recv_counts, int64_t elem_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(comm && send_counts && recv_counts && elem_bytes > 0, DR_INVALID_ARGUMENT,
             "bad argument");
  return a2a_v(comm, send, send_counts, recv, recv_counts, elem_bytes, S(stream));
}

int dr_memcpy(void* dst, const void* src, int64_t bytes, int sync, void* stream) {
  using namespace dr;
  DR_REQUIRE(bytes >= 0 && (bytes == 0 || (dst && src)), DR_INVALID_ARGUMENT, "bad argument");
  if (bytes == 0) return DR_OK;
  DR_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, S(stream)));
  if (sync) DR_HIP(hipStreamSynchronize(S(stream)));
  return DR_OK;
}

int dr_sharded_create(dr_comm* comm, dr_ev* const* evs, int num_tables, dr_sharded** out) {
  using namespace dr;
  DR_REQUIRE(comm && evs && out && num_tables >= 1 && num_tables <= DR_MAX_GROUP,
             DR_INVALID_ARGUMENT, "bad argument");
  for (int t = 0; t < num_tables; ++t) {
    DR_REQUIRE(evs[t], DR_INVALID_ARGUMENT, "table %d: null EV", t);
    DR_REQUIRE(dr_ev_filter_freq(evs[t]) == 0, DR_INVALID_ARGUMENT,
               "table %d: the sharded engine takes filter-free EVs", t);
    DR_REQUIRE(dr_ev_dim(evs[t]) == dr_ev_dim(evs[0]) &&
                   dr_ev_value_bits(evs[t]) == dr_ev_value_bits(evs[0]),
               DR_INVALID_ARGUMENT, "table %d: EVs of one dim and value type", t);
  }
  const int vb = dr_ev_value_bits(evs[0]);
  DR_REQUIRE(vb == 32 || (vb == 16 && dr_ev_dim(evs[0]) % 8 == 0), DR_INVALID_ARGUMENT,
             "float32 EVs, or bf16 EVs with dim %% 8 == 0");
  dr_sharded* s = new (std::nothrow) dr_sharded();
  DR_REQUIRE(s, DR_RESOURCE_EXHAUSTED, "out of host memory");
  s->comm = comm;
  s->T = num_tables;
  s->dim = dr_ev_dim(evs[0]);
  s->bf16 = vb == 16;
  const int GT = comm->world * num_tables;
  if (hipHostMalloc(&s->host, (size_t)(4 * GT + 2) * sizeof(int64_t)) != hipSuccess ||
      hipEventCreateWithFlags(&s->up_ev, hipEventDisableTiming) != hipSuccess) {
    if (s->host) (void)hipHostFree(s->host);
    delete s;
    set_error("hipHostMalloc / hipEventCreate failed");
    return DR_INTERNAL;
  }
  for (int t = 0; t < num_tables; ++t) {
    dr_ev_retain(evs[t]);
    s->evs.push_back(evs[t]);
  }
  *out = s;
  return DR_OK;
}

int dr_sharded_create_ex(dr_comm* comm, dr_ev* const* evs, int num_tables,
                         const dr_sharded_config* cfg, dr_sharded** out) {
  using namespace dr;
  DR_REQUIRE(cfg && out, DR_INVALID_ARGUMENT, "bad argument");
  DR_REQUIRE(cfg->kind >= DR_SHARDED_RCCL && cfg->kind <= DR_SHARDED_RCCL_FIXED,
             DR_INVALID_ARGUMENT, "unknown engine kind %d", cfg->kind);
  DR_REQUIRE(cfg->kind != DR_SHARDED_XGMI || cfg->batch > 0, DR_INVALID_ARGUMENT,
             "the XGMI kind needs batch > 0");
  DR_REQUIRE(cfg->kind != DR_SHARDED_RCCL_FIXED || cfg->max_ids > 0, DR_INVALID_ARGUMENT,
             "the fixed kind needs max_ids > 0");
  DR_REQUIRE(cfg->kind != DR_SHARDED_XGMI || !comm || comm->world == 1 || comm->kind == 1 ||
                 (comm->ops.all_gather && comm->ops.barrier),
             DR_INVALID_ARGUMENT, "the XGMI kind needs dr_comm_ops.all_gather and .barrier");
  dr_sharded* s = nullptr;
  int rc = dr_sharded_create(comm, evs, num_tables, &s);
  if (rc) return rc;
  s->kind = cfg->kind;
  if (cfg->kind == DR_SHARDED_XGMI) {
    s->batch = cfg->batch;
    DR_REQUIRE((int64_t)num_tables * cfg->batch < (1ll << 31), DR_INVALID_ARGUMENT,
               "tables x batch must be < 2^31");
    rc = xgmi_setup(s);
  } else if (cfg->kind == DR_SHARDED_RCCL_FIXED) {
    s->max_ids = cfg->max_ids;
    s->cap = (int64_t)num_tables * cfg->max_ids;   // a rank's ids, all to one owner at worst
    DR_REQUIRE(s->cap * comm->world < (1ll << 31), DR_INVALID_ARGUMENT,
               "world x tables x max_ids must be < 2^31");
  }
  if (rc) {
    dr_sharded_destroy(s);
    return rc;
  }
  *out = s;
  return DR_OK;
}

int dr_sharded_output(dr_sharded* s, void** out) {
  using namespace dr;
  DR_REQUIRE(s && out, DR_INVALID_ARGUMENT, "bad argument");
  DR_REQUIRE(s->kind == DR_SHARDED_XGMI, DR_INVALID_ARGUMENT,
             "only the XGMI kind keeps its output in an engine buffer");
  *out = s->own[3];
  return DR_OK;
}

int dr_sharded_backward_dev(dr_sharded* s, const float* grad, const int64_t** keys_out,
                            const float** grads_out, const int64_t** counts_dev_out,
                            int64_t* region_rows, void* stream) {
  using namespace dr;
  DR_REQUIRE(s && keys_out && grads_out && counts_dev_out && region_rows, DR_INVALID_ARGUMENT,
             "bad argument");
  DR_REQUIRE(s->kind != DR_SHARDED_RCCL, DR_INVALID_ARGUMENT,
             "the RCCL kind returns host counts: dr_sharded_backward");
  int rc;
  int64_t region;
  if (s->kind == DR_SHARDED_XGMI) {
    DR_REQUIRE(s->saved, DR_INVALID_ARGUMENT,
               "dr_sharded_backward needs a dr_sharded_forward(need_grad=1) first");
    DR_REQUIRE(grad, DR_INVALID_ARGUMENT, "null gradient");
    s->saved = false;
    rc = xgmi_backward(s, grad, stream);
    region = (int64_t)s->comm->world * s->batch;
  } else {
    DR_REQUIRE(s->fx_saved, DR_INVALID_ARGUMENT,
               "dr_sharded_backward needs a dr_sharded_forward(need_grad=1) first");
    DR_REQUIRE(grad || s->bags == 0, DR_INVALID_ARGUMENT, "null gradient");
    s->fx_saved = false;
    rc = fixed_backward(s, grad, stream);
    region = (int64_t)s->comm->world * s->max_ids;
  }
  if (rc) return rc;
  for (int t = 0; t < s->T; ++t) {
    keys_out[t] = s->pkeys.as<int64_t>() + (size_t)t * region;
    grads_out[t] = s->pgrads.as<float>() + (size_t)t * region * s->dim;
    counts_dev_out[t] = s->pcounts.as<int64_t>() + t;
  }
  *region_rows = region;
  return DR_OK;
}

int dr_sharded_destroy(dr_sharded* s) {
  if (!s) return DR_OK;
  (void)hipDeviceSynchronize();   // no kernel of a step may still use the buffers
  for (void* b : s->bases) (void)dr_ipc_close(b);
  for (void* p : s->own)
    if (p) (void)dr_ipc_free(p);
  for (dr_ev* e : s->evs) dr_ev_release(e);
  if (s->host) (void)hipHostFree(s->host);
  if (s->up_ev) (void)hipEventDestroy(s->up_ev);
  delete s;
  return DR_OK;
}

int dr_sharded_last_stats(const dr_sharded* s, int64_t* sent, int64_t* received) {
  using namespace dr;
  DR_REQUIRE(s, DR_INVALID_ARGUMENT, "bad argument");
  if (sent) *sent = s->last_sent;
  if (received) *received = s->last_recv;
  return DR_OK;
}

int dr_sharded_forward(dr_sharded* s, const int64_t* ids, const int64_t* koff_host,
                       const int32_t* const* bag_off, int64_t bags, int combiner, int need_grad,
                       int flags, void* out, void* stream) {
  using namespace dr;
  DR_REQUIRE(s && bags >= 0, DR_INVALID_ARGUMENT, "bad argument");
  DR_REQUIRE(combiner >= DR_COMBINER_SUM && combiner <= DR_COMBINER_SQRTN, DR_INVALID_ARGUMENT,
             "combiner must be sum, mean or sqrtn");
  DR_REQUIRE(!(flags & DR_SHARDED_OUT_BF16) || s->bf16, DR_INVALID_ARGUMENT,
             "a bf16 output needs bf16 EVs");
  // (XGMI: out may be NULL -- the result stays in the engine buffer)
  if (s->kind == DR_SHARDED_XGMI)
    return xgmi_forward(s, ids, koff_host, bag_off, bags, combiner, need_grad, flags, out, stream);
  DR_REQUIRE(out, DR_INVALID_ARGUMENT, "null output");
  if (s->kind == DR_SHARDED_RCCL_FIXED)
    return fixed_forward(s, ids, koff_host, bag_off, bags, combiner, need_grad, flags, out, stream);
  const int T = s->T, G = s->comm->world, GT = G * T;
  const int64_t D = s->dim;
  std::vector<int64_t> koff(T + 1);
  for (int t = 0; t <= T; ++t) koff[t] = koff_host ? koff_host[t] : (int64_t)t * bags;
  DR_REQUIRE(koff[0] == 0, DR_INVALID_ARGUMENT, "koff_host[0] must be 0");
  for (int t = 0; t < T; ++t) {
    DR_REQUIRE(koff[t + 1] >= koff[t], DR_INVALID_ARGUMENT, "koff_host must not decrease");
    DR_REQUIRE(bag_off || koff[t + 1] - koff[t] == bags, DR_INVALID_ARGUMENT,
               "table %d: one-hot ids need `bags` ids", t);
  }
  const int64_t n = koff[T];
  DR_REQUIRE(n < (1ll << 31), DR_INVALID_ARGUMENT, "total ids must be < 2^31");
  DR_REQUIRE(ids || n == 0, DR_INVALID_ARGUMENT, "null ids");
  hipStream_t st = S(stream);
  s->saved = false;
  const bool direct = !need_grad && !bag_off;
  const int64_t nn = n > 0 ? n : 1;
  const size_t vrow = (size_t)D * (s->bf16 ? 2 : 4);   // bytes of one exchanged row
  int rc;
#define DR_ENS(buf, bytes)             \
  do {                                 \
    rc = (buf).ensure((size_t)(bytes)); \
    if (rc) return rc;                 \
  } while (0)
  DR_ENS(s->keys_s, nn * 8);
  DR_ENS(s->tags_s, nn * 4);
  DR_ENS(s->perm, nn * 4);
  DR_ENS(s->counts, (size_t)2 * GT * 8);
  DR_ENS(s->rowsel, nn * 8);
  size_t wsb = dr_route_workspace_size(n, G, T);
  if (!direct) {
    const size_t u = dr_unique_grouped_workspace_size(koff.data(), T);
    wsb = u > wsb ? u : wsb;
    DR_ENS(s->uniq, nn * 8);
    DR_ENS(s->idx, nn * 4);
    DR_ENS(s->U, (size_t)T * 8);
  }
  DR_ENS(s->ws, wsb);
  const int64_t* src = ids;
  const int64_t* nu = nullptr;
  if (!direct) {
    rc = dr_unique_grouped(ids, koff.data(), T, s->uniq.as<int64_t>(), s->idx.as<int32_t>(),
                           nullptr, s->U.as<int64_t>(), s->ws.p, s->ws.bytes, stream);
    if (rc) return rc;
    src = s->uniq.as<int64_t>();
    nu = s->U.as<int64_t>();
  }
  rc = dr_route_by_owner(src, koff.data(), T, nu, G, s->keys_s.as<int64_t>(),
                         s->tags_s.as<int32_t>(), s->perm.as<int32_t>(), s->counts.as<int64_t>(),
                         s->ws.p, s->ws.bytes, stream);
  if (rc) return rc;
  // 3. counts exchange (T per peer), one host read of the splits
  std::vector<int64_t> tcnt(G, T);
  int64_t* cs = s->counts.as<int64_t>();
  rc = a2a_v(s->comm, cs, tcnt.data(), cs + GT, tcnt.data(), 8, st);
  if (rc) return rc;
  DR_HIP(hipMemcpyAsync(s->host, cs, (size_t)2 * GT * 8, hipMemcpyDeviceToHost, st));
  DR_HIP(hipStreamSynchronize(st));
  std::vector<int64_t> send(G, 0), recv(G, 0), rcv(GT), per_table(T, 0);
  for (int p = 0; p < G; ++p)
    for (int t = 0; t < T; ++t) {
      send[p] += s->host[p * T + t];
      recv[p] += s->host[GT + p * T + t];
      rcv[p * T + t] = s->host[GT + p * T + t];
      per_table[t] += s->host[GT + p * T + t];
    }
  int64_t S = 0, R = 0;
  for (int p = 0; p < G; ++p) {
    S += send[p];
    R += recv[p];
  }
  const int64_t RR = R > 0 ? R : 1, SS = S > 0 ? S : 1;
  DR_ENS(s->keys_r, RR * 8);
  DR_ENS(s->tags_r, RR * 4);
  DR_ENS(s->rows, RR * 8);
  DR_ENS(s->rows_s, (size_t)RR * vrow);
  DR_ENS(s->rows_r, (size_t)SS * vrow);
  const size_t rws = dr_ev_resolve_workspace_size(RR);
  if (rws > s->ws.bytes) DR_ENS(s->ws, rws);
  // 4. keys to the owners
  rc = a2a_v(s->comm, s->keys_s.p, send.data(), s->keys_r.p, recv.data(), 8, st);
  if (rc) return rc;
  // 5. owner: tags of the received keys, resolve (insert-on-miss), row pack
  rc = upload_blocks(s, rcv, st);
  if (rc) return rc;
  if (R > 0) {
    hipLaunchKernelGGL(sh_tags_kernel, dim3((unsigned)ceil_div(R, 256)), dim3(256), 0, st,
                       s->blk.as<int64_t>(), GT, T, R, s->tags_r.as<int32_t>());
    DR_LAUNCH_CHECK();
    rc = dr_ev_resolve_tagged(s->evs.data(), T, s->keys_r.as<int64_t>(), s->tags_r.as<int32_t>(),
                              R, nullptr, per_table.data(), nullptr, s->rows.as<int64_t>(),
                              s->ws.p, s->ws.bytes, stream);
    if (rc) return rc;
    rc = dr_ev_gather_tagged(s->evs.data(), T, s->tags_r.as<int32_t>(), s->rows.as<int64_t>(), R,
                             nullptr, s->rows_s.as<float>(), stream);
    if (rc) return rc;
  }
  // 6. rows back to the requesters
  rc = a2a_v(s->comm, s->rows_s.p, recv.data(), s->rows_r.p, send.data(), (int64_t)vrow, st);
  if (rc) return rc;
  // 7. requester: pool straight from the received rows
  if (S > 0) {
    hipLaunchKernelGGL(sh_rowsel_kernel, dim3((unsigned)ceil_div(S, 256)), dim3(256), 0, st,
                       s->perm.as<int32_t>(), S, s->rowsel.as<int64_t>());
    DR_LAUNCH_CHECK();
  }
  if (bags > 0) {
    std::vector<dr_pool_desc> d(T);
    const size_t ob = (flags & DR_SHARDED_OUT_BF16) ? 2 : 4;
    for (int t = 0; t < T; ++t) {
      memset(&d[t], 0, sizeof(dr_pool_desc));
      d[t].pool = s->rows_r.as<float>();
      if (direct) {
        d[t].ids = s->rowsel.as<int64_t>() + koff[t];
        d[t].pool_rows = SS;
      } else {
        d[t].idx = s->idx.as<int32_t>() + koff[t];
        d[t].rows = s->rowsel.as<int64_t>() + koff[t];
      }
      d[t].default_rows = s->rows_r.as<float>();
      d[t].default_stride = 0;
      d[t].bag_off = bag_off ? bag_off[t] : nullptr;
      d[t].out = reinterpret_cast<float*>(static_cast<char*>(out) + ob * (size_t)t * D);
      d[t].out_stride = (int64_t)T * D;
      d[t].combiner = combiner;
      d[t].max_norm = -1.f;
    }
    const int pf = (bag_off ? 0 : DR_POOL_ONEHOT) | (s->bf16 ? DR_POOL_BF16 : 0) |
                   ((flags & DR_SHARDED_OUT_BF16) ? DR_POOL_OUT_BF16 : 0);
    rc = dr_pool_grouped_ex(d.data(), T, bags, (int)D, DR_ORDER_ALI, pf, stream);
    if (rc) return rc;
  }
  s->last_sent = S;
  s->last_recv = R;
  if (need_grad) {
    s->saved = true;
    s->koff = koff;
    s->bags = bags;
    s->S = S;
    s->R = R;
    s->combiner = combiner;
    s->bag_off.assign(T, nullptr);
    if (bag_off)
      for (int t = 0; t < T; ++t) s->bag_off[t] = bag_off[t];
    s->send = send;
    s->recv = recv;
    s->rc = rcv;
  }
  return DR_OK;
#undef DR_ENS
}

int dr_sharded_backward(dr_sharded* s, const float* grad, const int64_t** keys_out,
                        const float** grads_out, int64_t* counts_out, void* stream) {
  using namespace dr;
  DR_REQUIRE(s && keys_out && grads_out && counts_out, DR_INVALID_ARGUMENT, "bad argument");
  if (s->kind != DR_SHARDED_RCCL) {   // device counts -> host (one read)
    const int64_t* cd[DR_MAX_GROUP];
    int64_t region = 0;
    int rc = dr_sharded_backward_dev(s, grad, keys_out, grads_out, cd, &region, stream);
    if (rc) return rc;
    DR_HIP(hipMemcpyAsync(counts_out, cd[0], (size_t)s->T * 8, hipMemcpyDeviceToHost,
                          S(stream)));
    DR_HIP(hipStreamSynchronize(S(stream)));
    return DR_OK;
  }
  DR_REQUIRE(s->saved, DR_INVALID_ARGUMENT,
             "dr_sharded_backward needs a dr_sharded_forward(need_grad=1) first");
  DR_REQUIRE(grad || s->bags == 0, DR_INVALID_ARGUMENT, "null gradient");
  s->saved = false;
  hipStream_t st = S(stream);
  const int T = s->T, G = s->comm->world, GT = G * T;
  const std::vector<int64_t>& koff = s->koff;
  const int64_t D = s->dim, n = koff[T], nn = n > 0 ? n : 1;
  const int64_t Sn = s->S, R = s->R, SS = Sn > 0 ? Sn : 1, RR = R > 0 ? R : 1;
  int rc;
#define DR_ENS(buf, bytes)             \
  do {                                 \
    rc = (buf).ensure((size_t)(bytes)); \
    if (rc) return rc;                 \
  } while (0)
  DR_ENS(s->gu, (size_t)nn * D * 4);
  DR_ENS(s->grads_s, (size_t)SS * D * 4);
  DR_ENS(s->grads_r, (size_t)RR * D * 4);
  DR_ENS(s->grads_t, (size_t)RR * D * 4);
  DR_ENS(s->keys_t, RR * 8);
  DR_ENS(s->permt, RR * 4);
  const bool multi = s->bag_off[0] != nullptr;
  if (multi) DR_ENS(s->seg, nn * 8);
  const size_t wsb = dr_pool_grad_grouped_workspace_size(n);
  if (wsb > s->ws.bytes) DR_ENS(s->ws, wsb);
  // 1. per local unique id its SparseSegment*Grad row (grouped-unique layout)
  if (n > 0 && s->bags > 0) {
    std::vector<dr_pool_grad_desc> d(T);
    for (int t = 0; t < T; ++t) {
      memset(&d[t], 0, sizeof(dr_pool_grad_desc));
      d[t].top_grad = grad + (size_t)t * D;
      d[t].top_stride = (int64_t)T * D;
      if (multi) {
        int64_t* sg = s->seg.as<int64_t>() + koff[t];
        hipLaunchKernelGGL(sh_seg_kernel, dim3((unsigned)ceil_div(s->bags, 256)), dim3(256), 0,
                           st, s->bag_off[t], s->bags, sg);
        DR_LAUNCH_CHECK();
        d[t].bag_off = s->bag_off[t];
        d[t].seg = sg;
        d[t].seg_stride = 1;
      }
      d[t].idx = s->idx.as<int32_t>() + koff[t];
      d[t].nnz = koff[t + 1] - koff[t];
      d[t].num_unique = s->U.as<int64_t>() + t;
      d[t].combiner = s->combiner;
    }
    rc = dr_pool_grad_grouped(d.data(), T, s->bags, (int)D, s->gu.as<float>(), s->ws.p,
                              s->ws.bytes, stream);
    if (rc) return rc;
  }
  // 2. packed into the forward's send order, 3. to the owners
  if (Sn > 0) {
    rc = dr_rows_pack(s->gu.as<float>(), s->perm.as<int32_t>(), Sn, nullptr, (int)D,
                      s->grads_s.as<float>(), stream);
    if (rc) return rc;
  }
  rc = a2a_v(s->comm, s->grads_s.p, s->send.data(), s->grads_r.p, s->recv.data(), D * 4, st);
  if (rc) return rc;
  // 4. table-major, source-rank-major slices (the block layout the forward
  // uploaded: the same received counts)
  if (R > 0) {
    const int64_t* bo = s->blk.as<int64_t>();
    hipLaunchKernelGGL(sh_regroup_kernel, dim3((unsigned)ceil_div(R, 256)), dim3(256), 0, st, bo,
                       bo + GT + 1, GT, R, s->keys_r.as<int64_t>(), s->keys_t.as<int64_t>(),
                       s->permt.as<int32_t>());
    DR_LAUNCH_CHECK();
    rc = dr_rows_pack(s->grads_r.as<float>(), s->permt.as<int32_t>(), R, nullptr, (int)D,
                      s->grads_t.as<float>(), stream);
    if (rc) return rc;
  }
  int64_t off = 0;
  for (int t = 0; t < T; ++t) {
    int64_t c = 0;
    for (int p = 0; p < G; ++p) c += s->rc[p * T + t];
    keys_out[t] = s->keys_t.as<int64_t>() + off;
    grads_out[t] = s->grads_t.as<float>() + (size_t)off * D;
    counts_out[t] = c;
    off += c;
  }
  return DR_OK;
#undef DR_ENS
}

}  // extern "C"
