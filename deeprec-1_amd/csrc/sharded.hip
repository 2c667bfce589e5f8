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
#undef DR_SYM
    api.ok = api.GetUniqueId && api.CommInitRank && api.CommDestroy && api.Send && api.Recv &&
             api.GroupStart && api.GroupEnd && api.ErrorString;
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

}  // namespace dr

struct dr_sharded {
  dr_comm* comm = nullptr;
  std::vector<dr_ev*> evs;
  int T = 0;
  int64_t dim = 0;
  int bf16 = 0;
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
  }
  *out = c;
  return DR_OK;
}

int dr_comm_destroy(dr_comm* comm) {
  if (!comm) return DR_OK;
  if (comm->kind == 1 && comm->nc && dr::rccl()) dr::rccl()->CommDestroy(comm->nc);
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

int dr_sharded_destroy(dr_sharded* s) {
  if (!s) return DR_OK;
  (void)hipDeviceSynchronize();   // no kernel of a step may still use the buffers
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
  DR_REQUIRE(s && out && bags >= 0, DR_INVALID_ARGUMENT, "bad argument");
  DR_REQUIRE(combiner >= DR_COMBINER_SUM && combiner <= DR_COMBINER_SQRTN, DR_INVALID_ARGUMENT,
             "combiner must be sum, mean or sqrtn");
  DR_REQUIRE(!(flags & DR_SHARDED_OUT_BF16) || s->bf16, DR_INVALID_ARGUMENT,
             "a bf16 output needs bf16 EVs");
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
