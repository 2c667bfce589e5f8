// ev.hip -- GPU EmbeddingVariable: open-addressing key -> row table in HBM,
// value pools per column (primary + optimizer slots), DeepRec filters,
// insert-on-miss resolve, import/export and sparse-apply optimizers.
//
// Reference semantics (paths relative to the DeepRec root):
//   EmbeddingVar            core/framework/embedding/embedding_var.h:50-363
//   LookupOrCreateKeyInternal  embedding_var.h:320-339
//   ValuePtr::GetOrAllocate value_ptr.h:145-170 (per-column default copy)
//   Nullable/Counter/Bloom  embedding_filter.h:27-396
//   KvResourceGather[V1]    core/kernels/kv_variable_ops.cc:314-449
//   Import / GetSnapshot    embedding_var.h:187-243
//   KvSparseApply*          core/kernels/training_ali_ops.cc
//
// HBM layout (one key space shared by a primary EV and its slot EVs, as the
// reference shares kv_ between them, kv_variable_ops.cc:232-238):
//   slots[cap + 1]  16 B {key, rc}: rc = row (bits 0..47) | column-init
//                   bitset (bits 48..63); key -1 lives in slots[cap].
//   pool[c]         [row_cap, dim] fp32 rows of column c (0 = primary).
//   freq/version    [row_cap] int64, only when filter / steps_to_live on.
// A key owns one row id for all columns; a column's row is initialised from
// that column's default the first time it is touched, exactly like the
// reference's lazily allocated per-emb_index rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <atomic>
#include <cmath>
#include <mutex>
#include <new>
#include <vector>

#include "dr_common.h"
#include "dr_rows.h"

namespace dr {

static constexpr int kMaxCols = 16;
static constexpr uint64_t kEmptyKey = ~0ull;
static constexpr uint64_t kUnset = ~0ull;
static constexpr uint64_t kRowMask = (1ull << 48) - 1;
static constexpr uint64_t kRowDead = kRowMask;  // allocation failed

struct __attribute__((aligned(16))) Slot {
  uint64_t key;
  uint64_t rc;
};

struct EvShared {
  std::atomic<int> refs{1};
  int device = 0;
  int64_t dim = 0;
  int64_t filter_freq = 0, steps_to_live = 0;
  int64_t k_hash = 0, num_counter = 0;
  int counter_bits = 64;
  Slot* slots = nullptr;
  int64_t cap = 0;  // power of two (+1 special slot allocated)
  int64_t* top = nullptr;
  int64_t row_cap = 0;
  int64_t* freq = nullptr;
  int64_t* version = nullptr;
  float* pools[kMaxCols] = {nullptr};
  float* defaults[kMaxCols] = {nullptr};
  void* bloom = nullptr;
  uint64_t* seeds = nullptr;
  // host-side capacity accounting (no sync on the steady-state path)
  std::mutex mu;
  int64_t known = 0, adds_since_known = 0, adds_since_copy = 0;
  bool copy_pending = false;
  // which streams reserved adds since `known` was exact (adds) and since the
  // pending mirror copy was issued (copy_adds): a copy or a sync on stream X
  // only covers the adds of other streams once they have run
  struct Streams {
    bool any = false, mixed = false;
    hipStream_t st = nullptr;
    void note(hipStream_t x) {
      if (!any) {
        any = true;
        st = x;
      } else if (st != x) {
        mixed = true;
      }
    }
    bool only(hipStream_t x) const { return !mixed && (!any || st == x); }
  };
  Streams adds, copy_adds;
  bool copy_exact = false;
  hipEvent_t copy_ev = nullptr;
  int64_t* pinned_top = nullptr;
  int64_t removed = 0;  // keys removed by dr_ev_shrink (rows are not recycled)
  // value dtype: 1 = float, 2 = double (a double row is stored as 2 * dim
  // float words and moved bitwise; `dim` counts float words)
  int value_words = 1;
  // bf16 EV (value_bits 16): the primary column holds bf16 rows of D values
  // (D/2 float words, moved bitwise by the copy kernels); `dim` = D counts
  // the fp32 words of the optimizer slot columns, which stay fp32.
  int bf16 = 0;
  // use_locking applies (dr_ev_lock_updates): exclusive updates across
  // host threads and streams
  std::mutex update_mu;
  hipEvent_t update_ev = nullptr;
  // host side of every call on this EV (EvGuard below)
  std::recursive_mutex api_mu;
};

// float words per row of column `col`
inline int64_t col_words(const EvShared* s, int col) {
  return (s->bf16 && col == 0) ? s->dim / 2 : s->dim;
}

}  // namespace dr

struct dr_ev {
  dr::EvShared* sh;
  int col;
  std::atomic<int> refs{1};
};

namespace dr {

// Host-side serialisation of the calls on one EV.  The reference runs ops on
// one EmbeddingVar concurrently from inter-op threads; here a call reads the
// EV's table / pool pointers and enqueues kernels, and a growth (reserve ->
// grow) rehashes and frees them.  A call holds the api_mu of every EV it
// touches (distinct shared states, address order: no lock-order cycle) from
// its first read of an EV pointer to its last launch, and grow() synchronises
// the device before reading the old buffers, so every kernel another stream
// enqueued on them earlier has finished.  The kernels of different streams
// still overlap on the device -- the CAS insert arbitrates there, as the
// lockless map's CAS does -- and a launch is asynchronous, so the lock costs
// launch time only.  dr_ev_lock_updates (use_locking) is a separate mutex
// taken around whole calls and never inside one.
class EvGuard {
 public:
  EvGuard(dr_ev* const* evs, int64_t n) {
    if (evs)
      for (int64_t i = 0; i < n; ++i)
        if (evs[i]) v_.push_back(evs[i]->sh);
    std::sort(v_.begin(), v_.end());
    v_.erase(std::unique(v_.begin(), v_.end()), v_.end());
    for (EvShared* e : v_) e->api_mu.lock();
  }
  explicit EvGuard(dr_ev* ev) : EvGuard(&ev, 1) {}
  ~EvGuard() {
    for (auto it = v_.rbegin(); it != v_.rend(); ++it) (*it)->api_mu.unlock();
  }
  EvGuard(const EvGuard&) = delete;
  EvGuard& operator=(const EvGuard&) = delete;

 private:
  std::vector<EvShared*> v_;
};

void* ev_guard_acquire(dr_ev* const* evs, int64_t n) { return new EvGuard(evs, n); }
void ev_guard_release(void* g) { delete static_cast<EvGuard*>(g); }

// Per-table view passed to kernels by value.
struct EvDesc {
  Slot* slots;
  int64_t cap;
  int64_t* top;
  int64_t row_cap;
  int64_t* freq;
  int64_t* version;
  void* bloom;
  const uint64_t* seeds;
  int64_t filter_freq;
  int64_t num_counter;
  int32_t k_hash;
  int32_t counter_bits;
  int32_t col;
  int32_t primary;
};

static EvDesc make_desc(const dr_ev* ev) {
  const EvShared* s = ev->sh;
  EvDesc d;
  d.slots = s->slots;
  d.cap = s->cap;
  d.top = s->top;
  d.row_cap = s->row_cap;
  d.freq = s->freq;
  d.version = s->version;
  d.bloom = s->bloom;
  d.seeds = s->seeds;
  d.filter_freq = s->filter_freq;
  d.num_counter = s->num_counter;
  d.k_hash = (int32_t)s->k_hash;
  d.counter_bits = s->counter_bits;
  d.col = ev->col;
  d.primary = ev->col == 0;
  return d;
}

// ---- device helpers --------------------------------------------------------
// Bucket-local linear probing.  The table is cut into 128-B lines of 8 slots;
// the i-th probe of a key whose home slot is h0 visits line (h0 / 8 + i / 8)
// at offset (h0 + i) % 8, i.e. a key's probe sequence wraps inside its home
// line before it moves on.  At the tables' load (<= 3/4, 3/8 at the bench's
// sizing) a key is found or ruled out inside its home line ~99.5 % of the
// time, so one line-wide load of 8 lanes (ev_line_probe) settles a lookup in a
// single memory round trip.  Every probe / insert / rehash uses this one
// sequence (cap is a power of two >= 1024, so lines never straddle the end).
__device__ __forceinline__ uint64_t probe_slot(uint64_t h0, uint64_t i, uint64_t mask) {
  return (((h0 & ~7ull) + (i & ~7ull)) & mask) | ((h0 + i) & 7ull);
}

__device__ __forceinline__ uint64_t atomic_read_u64(uint64_t* p) {
  return __hip_atomic_fetch_or(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Find (or, with insert, create) the slot of `key`.  Returns nullptr when not
// found (insert == false).  *rc receives the published rc word.
__device__ Slot* ev_find(const EvDesc& e, uint64_t key, bool insert, bool* created,
                         uint64_t* rc, int* st) {
  *created = false;
  Slot* s = nullptr;
  uint64_t rc_seen = kUnset;  // rc read together with a matching key
  if (key == kEmptyKey) {
    s = e.slots + e.cap;
    uint64_t cur = s->key;
    if (cur != 0ull) {
      if (!insert) {
        cur = atomic_read_u64(&s->key);
        if (cur != 0ull) return nullptr;
      } else {
        uint64_t old = atomicCAS((unsigned long long*)&s->key, (unsigned long long)kEmptyKey, 0ull);
        if (old == kEmptyKey) *created = true;
      }
    }
  } else {
    const uint64_t mask = (uint64_t)e.cap - 1;
    const uint64_t h0 = mix64(key) & mask;
    for (int64_t probes = 0;; ++probes) {
      if (probes > e.cap) {
        latch(st, DR_RESOURCE_EXHAUSTED);
        return nullptr;
      }
      Slot* c = e.slots + probe_slot(h0, (uint64_t)probes, mask);
      // one 16-byte load brings key and rc: a hit needs no second round trip
      typedef unsigned long long slot_v __attribute__((ext_vector_type(2)));
      const slot_v sv = *reinterpret_cast<const slot_v*>(c);
      uint64_t cur = sv.x;
      if (cur == key) {
        s = c;
        rc_seen = sv.y;
        break;
      }
      if (cur == kEmptyKey) {
        if (!insert) {
          cur = atomic_read_u64(&c->key);  // rule out a stale empty
          if (cur == kEmptyKey) return nullptr;
          if (cur == key) {
            s = c;
            break;
          }
        } else {
          uint64_t old =
              atomicCAS((unsigned long long*)&c->key, (unsigned long long)kEmptyKey,
                        (unsigned long long)key);
          if (old == kEmptyKey) {
            s = c;
            *created = true;
            break;
          }
          if (old == key) {
            s = c;
            break;
          }
        }
      }
    }
  }
  // The creator publishes the row BEFORE any lane waits for one: with
  // duplicate keys in one call, creator and waiter can share a wavefront,
  // and a divergent spin ahead of the creator's store would never end
  // (lanes of a wave do not progress independently).  Two sequential ifs
  // reconverge in between, so the store is issued first.
  if (*created) {
    const int64_t row = (int64_t)atomicAdd((unsigned long long*)e.top, 1ull);
    uint64_t v;
    if (row >= e.row_cap) {
      latch(st, DR_RESOURCE_EXHAUSTED);
      v = kRowDead;
    } else {
      v = (uint64_t)row;  // freq/version rows were zeroed at allocation
    }
    __hip_atomic_store(&s->rc, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *rc = v;
  }
  __builtin_amdgcn_wave_barrier();  // convergent: keeps the two ifs apart
  if (*created) return s;
  uint64_t v = rc_seen != kUnset ? rc_seen : s->rc;
  if (v == kUnset) {
    for (int spin = 0; spin < (1 << 22); ++spin) {
      v = atomic_read_u64(&s->rc);
      if (v != kUnset) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (v == kUnset) {
      latch(st, DR_INTERNAL);
      v = kRowDead;
    }
  }
  *rc = v;
  return s;
}

// ---- Bloom counters (embedding_filter.h:97-250) -----------------------------
__device__ __forceinline__ uint64_t fasthash64(uint64_t key, uint64_t seed) {
  const uint64_t m = 0x880355f21e6d1965ULL;
  uint64_t h = seed ^ (8 * m);
  uint64_t v = key;
  v ^= v >> 23;
  v *= 0x2127599bf4325c37ULL;
  v ^= v >> 47;
  h ^= v;
  h *= m;
  v = 0;
  v ^= v >> 23;
  v *= 0x2127599bf4325c37ULL;
  v ^= v >> 47;
  h ^= v;
  h *= m;
  h ^= h >> 23;
  h *= 0x2127599bf4325c37ULL;
  h ^= h >> 47;
  return h;
}

__device__ __forceinline__ uint64_t bloom_get(const EvDesc& e, int64_t c) {
  switch (e.counter_bits) {
    case 8: return ((const uint8_t*)e.bloom)[c];
    case 16: return ((const uint16_t*)e.bloom)[c];
    case 32: return ((const uint32_t*)e.bloom)[c];
    default: return ((const uint64_t*)e.bloom)[c];
  }
}

__device__ __forceinline__ void bloom_add(const EvDesc& e, int64_t c, uint64_t cnt) {
  if (e.counter_bits == 64) {
    atomicAdd((unsigned long long*)e.bloom + c, (unsigned long long)cnt);
  } else if (e.counter_bits == 32) {
    atomicAdd((unsigned int*)e.bloom + c, (unsigned int)cnt);
  } else {
    // 8/16-bit counters: add into the containing aligned 32-bit word (wraps
    // in-field like the reference's __sync_fetch_and_add on uint8/16).
    const int bytes = e.counter_bits / 8;
    char* base = (char*)e.bloom + c * bytes;
    unsigned int* w = (unsigned int*)((uintptr_t)base & ~(uintptr_t)3);
    const int sh = (int)(((uintptr_t)base & 3) * 8);
    const unsigned int fmask = (bytes == 1 ? 0xFFu : 0xFFFFu) << sh;
    unsigned int old = *w, assumed;
    do {
      assumed = old;
      unsigned int f = ((assumed & fmask) >> sh) + (unsigned int)cnt;
      unsigned int nv = (assumed & ~fmask) | ((f << sh) & fmask);
      old = atomicCAS(w, assumed, nv);
    } while (old != assumed);
  }
}

__device__ int64_t bloom_min_freq(const EvDesc& e, uint64_t key) {
  uint64_t mn = 0;
  for (int i = 0; i < e.k_hash; ++i) {
    const int64_t c = (int64_t)(fasthash64(key, e.seeds[i]) % (uint64_t)e.num_counter);
    const uint64_t v = bloom_get(e, c);
    if (i == 0 || v < mn) mn = v;
  }
  return (int64_t)mn;
}

__device__ void bloom_addfreq(const EvDesc& e, uint64_t key, int64_t cnt) {
  for (int i = 0; i < e.k_hash; ++i) {
    const int64_t c = (int64_t)(fasthash64(key, e.seeds[i]) % (uint64_t)e.num_counter);
    if ((int64_t)bloom_get(e, c) < e.filter_freq) bloom_add(e, c, (uint64_t)cnt);
  }
}

// ---------------------------------------------------------------------------
// Resolve (gather): lane per key.  rows_out[i] = row or -(i+1) (default);
// init[i] = 1 when this lane claimed the column's first touch of the row;
// badd[i] = count to add to Bloom counters in the follow-up pass.
// Grouped over tables: table t owns keys [koff[t], koff[t+1]) and the device
// count n_dev[t] (nullable) bounds it.
// ---------------------------------------------------------------------------
// Tagged mode (tags != nullptr): one array holds keys of all T tables with a
// per-key table id tags[i]; n_dev[0] bounds it.  This is the owner side of
// the sharded exchange, where keys of every feature arrive interleaved.
struct EvGroup {
  EvDesc e[DR_MAX_GROUP];
  int64_t koff[DR_MAX_GROUP + 1];
  const int64_t* n_dev[DR_MAX_GROUP];
  const int32_t* tags;
};

__device__ __forceinline__ bool locate(const EvGroup& g, int T, int64_t i,
                                       const int64_t* __restrict__ keys, int* t, int64_t* li,
                                       uint64_t* key) {
  if (i >= g.koff[T]) return false;
  if (g.tags) {
    if (g.n_dev[0] && i >= *g.n_dev[0]) return false;
    *t = g.tags[i];
    *key = (uint64_t)keys[i];
    *li = i;
    return true;
  }
  const int tt = table_of(g.koff, T, i, (int64_t)blockIdx.x * blockDim.x);
  *t = tt;
  *li = i - g.koff[tt];
  if (g.n_dev[tt] && *li >= *g.n_dev[tt]) return false;
  *key = (uint64_t)keys[i];
  return true;
}

__global__ void ev_resolve_kernel(EvGroup g, int T, const int64_t* __restrict__ keys,
                                  const int32_t* __restrict__ counts, int64_t* __restrict__ rows_out,
                                  uint8_t* __restrict__ init, int32_t* __restrict__ badd, int* st) {
  // per-lane table index: descriptors staged in LDS (see pool_onehot_kernel)
  __shared__ EvDesc se[DR_MAX_GROUP];
  if (threadIdx.x < T) se[threadIdx.x] = g.e[threadIdx.x];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int t;
  int64_t li;
  uint64_t key;
  if (!locate(g, T, i, keys, &t, &li, &key)) return;
  const EvDesc& e = se[t];
  init[i] = 0;
  if (badd) badd[i] = 0;
  const int64_t cnt = counts ? counts[i] : 1;
  if (e.k_hash > 0) {  // BloomFilter::LookupOrCreate (embedding_filter.h:56-82)
    if (bloom_min_freq(e, key) < e.filter_freq) {
      badd[i] = (int32_t)cnt;
      rows_out[i] = -(li + 1);
      return;
    }
  }
  bool created;
  uint64_t rc;
  Slot* s = ev_find(e, key, true, &created, &rc, st);
  if (!s || (rc & kRowMask) == kRowDead) {
    rows_out[i] = -(li + 1);
    return;
  }
  const int64_t row = (int64_t)(rc & kRowMask);
  if (e.filter_freq > 0 && e.k_hash == 0) {  // CounterFilter (embedding_filter.h:296-320)
    unsigned long long* f = (unsigned long long*)(e.freq + row);
    unsigned long long old = __hip_atomic_fetch_add(f, 0ull, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
    bool admitted = false;
    for (;;) {
      if ((int64_t)old >= e.filter_freq) {
        admitted = true;
        break;
      }
      unsigned long long prev = atomicCAS(f, old, old + (unsigned long long)cnt);
      if (prev == old) break;
      old = prev;
    }
    if (!admitted) {
      rows_out[i] = -(li + 1);
      return;
    }
  }
  const uint64_t bit = 1ull << (48 + e.col);
  if (!(rc & bit)) {
    const uint64_t old = atomicOr((unsigned long long*)&s->rc, (unsigned long long)bit);
    if (!(old & bit)) init[i] = 1;
  }
  rows_out[i] = row;
}

__global__ void ev_bloom_add_kernel(EvGroup g, int T, const int64_t* __restrict__ keys,
                                    const int32_t* __restrict__ badd) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int t;
  int64_t li;
  uint64_t key;
  if (!locate(g, T, i, keys, &t, &li, &key)) return;
  if (badd[i] > 0) bloom_addfreq(g.e[t], key, badd[i]);
}

// Copy the first-touch rows: pool[col][row_i] = src(i), group of 64 lanes
// per key, lane-strided floats.  src(i) = src_rows[li*dim] or src_default.
struct InitGroup {
  float* pool[DR_MAX_GROUP];
  const float* src[DR_MAX_GROUP];      // per-key rows ([n,dim]) or nullptr
  const float* dflt[DR_MAX_GROUP];     // column default (dim)
  int64_t koff[DR_MAX_GROUP + 1];
  const int64_t* n_dev[DR_MAX_GROUP];
  const int32_t* tags;
  int64_t* mtop[DR_MAX_GROUP];  // row counters to mirror (nullptr: none)
  int64_t* mdst[DR_MAX_GROUP];  // pinned host mirrors
};

// Wave-cooperative: each lane tests one key's flag, the wave ballots and then
// copies every flagged row with all 64 lanes.  In steady state (no new keys)
// this is one coalesced byte load per key.
__global__ void ev_init_rows_kernel(InitGroup g, int T, int64_t dim,
                                    const int64_t* __restrict__ rows,
                                    const uint8_t* __restrict__ init) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  if (blockIdx.x == 0 && threadIdx.x < T && g.mdst[threadIdx.x]) {
    // the resolve kernel before this one has finished: the counter is final
    const int64_t top = __hip_atomic_load(g.mtop[threadIdx.x], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(g.mdst[threadIdx.x], top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  bool need = false;
  int t = 0;
  int64_t li = i;
  if (i < g.koff[T]) {
    bool live = true;
    if (g.tags) {
      if (g.n_dev[0] && i >= *g.n_dev[0]) live = false;
      else t = g.tags[i];
    } else {
      t = table_of(g.koff, T, i, (int64_t)blockIdx.x * blockDim.x);
      li = i - g.koff[t];
      if (g.n_dev[t] && li >= *g.n_dev[t]) live = false;
    }
    need = live && init[i];
  }
  uint64_t mask = __ballot(need);
  while (mask) {
    const int src_lane = __ffsll((unsigned long long)mask) - 1;
    mask &= mask - 1;
    const int tt = __shfl(t, src_lane, 64);
    const int64_t ll = __shfl(li, src_lane, 64);
    const int64_t ii = __shfl(i, src_lane, 64);
    const int64_t row = rows[ii];
    const float* src = g.src[tt] ? g.src[tt] + ll * dim : g.dflt[tt];
    float* dst = g.pool[tt] + row * dim;
    for (int64_t c = lane; c < dim; c += 64) dst[c] = src[c];
  }
}

// Owner-side row pack of the sharded exchange: out[i] = pool_t[row_i] (or the
// table's default row when filtered), t from the composite key.  G lanes per
// row, dwordx4.
struct PoolGroup {
  const float* pool[DR_MAX_GROUP];
  const float* dflt[DR_MAX_GROUP];
};

template <int G>
__global__ __launch_bounds__(256) void ev_gather_tagged_kernel(
    PoolGroup pg, int T, int64_t dim, const int32_t* __restrict__ tags,
    const int64_t* __restrict__ rows, int64_t n, const int64_t* n_dev, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G;
  if (i >= eff_n(n, n_dev)) return;
  const int t = tags[i];
  const int64_t r = rows[i];
  const float* src = r >= 0 ? pg.pool[t] + r * dim : pg.dflt[t];
  const int lg = threadIdx.x % G;
  if ((dim & 3) == 0) {
    for (int64_t c = lg; c < dim / 4; c += G)
      reinterpret_cast<float4*>(out + i * dim)[c] = reinterpret_cast<const float4*>(src)[c];
  } else {
    for (int64_t c = lg; c < dim; c += G) out[i * dim + c] = src[c];
  }
}

// ---------------------------------------------------------------------------
// Import (EmbeddingVar::Import, embedding_var.h:187-219).
// ---------------------------------------------------------------------------
__global__ void ev_import_kernel(EvDesc e, const int64_t* __restrict__ keys, int64_t n,
                                 const int64_t* __restrict__ versions,
                                 const int64_t* __restrict__ freqs, int64_t partition_id,
                                 int64_t partition_num, int64_t steps_to_live,
                                 int64_t* __restrict__ rows_out, uint8_t* __restrict__ init,
                                 int* st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  init[i] = 0;
  rows_out[i] = -1;
  const int64_t key = keys[i];
  if (partition_num > 0 && key % 1000 % partition_num != partition_id) return;
  bool created;
  uint64_t rc;
  Slot* s = ev_find(e, (uint64_t)key, true, &created, &rc, st);
  if (!s || (rc & kRowMask) == kRowDead) return;
  const int64_t row = (int64_t)(rc & kRowMask);
  if (e.primary) {
    if (e.filter_freq != 0 && e.freq) {
      const int64_t f = freqs ? freqs[i] : 0;
      e.freq[row] = f <= e.filter_freq ? e.filter_freq : f;
    }
    if (steps_to_live != 0 && e.version) e.version[row] = versions ? versions[i] : 0;
  }
  const uint64_t bit = 1ull << (48 + e.col);
  if (!(rc & bit)) {
    const uint64_t old = atomicOr((unsigned long long*)&s->rc, (unsigned long long)bit);
    if (!(old & bit)) init[i] = 1;
  }
  rows_out[i] = row;
}

// Synthetic bulk insert of keys [begin, begin + n) (bench / test tables):
// rows are filled with synth(seed, key, col) by ev_synth_rows_kernel.
__global__ void ev_insert_range_kernel(EvDesc e, int64_t begin, int64_t stride, int64_t n,
                                       int64_t* __restrict__ rows_out, uint8_t* __restrict__ init,
                                       int* st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  init[i] = 0;
  rows_out[i] = -1;
  bool created;
  uint64_t rc;
  Slot* s = ev_find(e, (uint64_t)(begin + i * stride), true, &created, &rc, st);
  if (!s || (rc & kRowMask) == kRowDead) return;
  const uint64_t bit = 1ull << (48 + e.col);
  if (!(rc & bit)) {
    const uint64_t old = atomicOr((unsigned long long*)&s->rc, (unsigned long long)bit);
    if (!(old & bit)) init[i] = 1;
  }
  rows_out[i] = (int64_t)(rc & kRowMask);
}

__global__ void ev_synth_rows_kernel(float* __restrict__ pool, int64_t dim, int bf16,
                                     int64_t begin, int64_t stride, int64_t n,
                                     const int64_t* __restrict__ rows,
                                     const uint8_t* __restrict__ init, uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (i >= n || !init[i]) return;
  const int64_t key = begin + i * stride;
  if (bf16) {  // bf16(synth) pairs, element 2k in the low half
    uint32_t* dst = reinterpret_cast<uint32_t*>(pool) + rows[i] * (dim / 2);
    for (int64_t c = threadIdx.x % 64; c < dim / 2; c += 64)
      dst[c] = f2_to_bf16x2(synth(seed, key, 2 * c), synth(seed, key, 2 * c + 1));
    return;
  }
  float* dst = pool + rows[i] * dim;
  for (int64_t c = threadIdx.x % 64; c < dim; c += 64) dst[c] = synth(seed, key, c);
}

// Lookup without insert (export helpers / key_meta).
__global__ void ev_lookup_kernel(EvDesc e, const int64_t* __restrict__ keys, int64_t n,
                                 int64_t* __restrict__ rows_out, uint64_t* __restrict__ rc_out,
                                 int* st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool created;
  uint64_t rc = kUnset;
  Slot* s = ev_find(e, (uint64_t)keys[i], false, &created, &rc, st);
  rows_out[i] = s ? (int64_t)(rc & kRowMask) : -1;
  rc_out[i] = s ? rc : 0;
}

// ---------------------------------------------------------------------------
// Sparse apply: group of G lanes per key; the leader probes, sets version
// and column bits, the group initialises first-touch rows from the column
// defaults (var->flat / accum->flat in training_ali_ops.cc) and updates.
// ---------------------------------------------------------------------------
struct ApplyCols {
  float* pool[3];
  const float* dflt[3];
  int ncol;
  int cols[3];
};

enum {
  OPT_SGD = 0,
  OPT_ADAGRAD = 1,
  OPT_ADAM = 2,
  OPT_FTRL = 3,
  OPT_ADAM_ASYNC = 4,     // KvSparseApplyAdamAsync (training_ali_ops.cc:1404-1575)
  OPT_ADAM_RMSPROP = 5,   //   ... with apply_sparse_rmsprop (:1483-1519)
  OPT_ADAGRAD_DECAY = 6   // KvSparseApplyAdagradDecay (training_ali_ops.cc:703-823)
};
// var + two slot columns (m / v, or accum / accum_decay_power)
__host__ __device__ constexpr bool opt_three_cols(int opt) {
  return opt == OPT_ADAM || opt == OPT_ADAM_ASYNC || opt == OPT_ADAM_RMSPROP ||
         opt == OPT_ADAGRAD_DECAY;
}

struct OptScalars {
  float lr, beta1, beta2, eps, alpha;
  float l1, l2, lr_power, l2_shrinkage;  // FTRL
  float decay_rate, decay_baseline;      // AdagradDecay
  int64_t decay_step;
};

// Two phases per wave of 64 keys.  Phase 1, lane per key: LookupOrCreate
// with the global step / filter admission / first-touch column mask (the
// dependent hash probes of 64 keys overlap).  Phase 2: groups of G lanes
// update 64/G rows at a time with VEC-wide loads/stores; every element is
// the reference's scalar formula with separate fp32 roundings.
template <int OPT, int VEC, int G>
__device__ __forceinline__ float apply_one(float gv, float w, float* a1, float* a2,
                                           const OptScalars& sc) {
  if (OPT == OPT_SGD) {
    const float p = sc.lr * gv;  // v -= lr * g  (training_ali_ops.cc:1663)
    return w - p;
  } else if (OPT == OPT_ADAGRAD) {  // training_ali_ops.cc:131-132
    float a = *a1;
    const float g2 = gv * gv;
    a = a + g2;
    const float lg_ = sc.lr * gv;
    const float rs = 1.0f / sqrtf(a);
    const float up = lg_ * rs;
    *a1 = a;
    return w - up;
  } else if (OPT == OPT_ADAM_ASYNC) {  // training_ali_ops.cc:1552-1554
    float m = *a1;
    float v = *a2;
    const float mt = m * sc.beta1;
    const float mg = gv * (1.0f - sc.beta1);
    m = mt + mg;
    const float vt = v * sc.beta2;
    const float g2 = gv * gv;
    const float vg = g2 * (1.0f - sc.beta2);
    v = vt + vg;
    const float num = m * sc.alpha;
    const float den = sqrtf(v) + sc.eps;
    *a1 = m;
    *a2 = v;
    return w - num / den;
  } else if (OPT == OPT_ADAM_RMSPROP) {  // training_ali_ops.cc:1506-1513
    float m = *a1;
    float v = *a2;
    const float vt = v * sc.beta2;
    const float g2 = gv * gv;
    const float vg = g2 * (1.0f - sc.beta2);
    v = vt + vg;
    const float rs = 1.0f / sqrtf(v + sc.eps);
    const float step = (rs * sc.lr) * gv;
    const float mt = m * sc.beta1;
    m = mt + step;
    *a1 = m;
    *a2 = v;
    return w - m;
  } else {  // OPT_ADAM, training_ali_ops.cc:952-958
    float m = *a1;
    float v = *a2;
    float t1 = gv - m;
    t1 = t1 * (1.0f - sc.beta1);
    m = m + t1;
    float t2 = gv * gv;
    t2 = t2 - v;
    t2 = t2 * (1.0f - sc.beta2);
    v = v + t2;
    const float num = m * sc.alpha;
    const float den = sqrtf(v) + sc.eps;
    *a1 = m;
    *a2 = v;
    return w - num / den;
  }
}

// AdagradDecay element (training_ali_ops.cc:802-808): when the row decays
// this step, a = max(a * rate, baseline) (cwiseMax: a < b ? b : a), then
// a += g^2; v -= (lr * g) * rsqrt(a).
__device__ __forceinline__ float adagrad_decay_one(float gv, float w, float* a1, bool dec,
                                                   const OptScalars& sc) {
  float a = *a1;
  if (dec) {
    a = a * sc.decay_rate;
    a = a < sc.decay_baseline ? sc.decay_baseline : a;
  }
  const float g2 = gv * gv;
  a = a + g2;
  const float lg_ = sc.lr * gv;
  const float rs = 1.0f / sqrtf(a);
  const float up = lg_ * rs;
  *a1 = a;
  return w - up;
}

// One table of a grouped apply launch (blockIdx.y selects it).
struct ApplyTable {
  EvDesc e;
  ApplyCols cols;
  const int64_t* keys;
  const float* grad;
  int64_t n;
  const int64_t* n_dev;
  int64_t steps_to_live;
  const int64_t* rows;  // known rows of the keys (SGD of a row-grouped backward) or nullptr
  // AdamAsync: this variable's device-resident {beta1_power, beta2_power}
  // (the reference keeps them in an EV of their own, training_ali_ops.cc
  // :1523-1526); alpha is formed from them in the kernel, and
  // ev_adam_powers_kernel advances them after the apply when N > 0
  const float* powers;
};
static constexpr int kApplyGroup = 16;  // keeps the kernel arguments < 4 KiB
struct ApplyGroup {
  ApplyTable t[kApplyGroup];
};
static_assert(sizeof(ApplyGroup) + 64 <= 4096, "apply kernel arguments exceed 4 KiB");

// Phase 1 of a sparse apply, lane per key: LookupOrCreate with the global
// step / filter admission / first-touch column mask (training_ali_ops.cc
// LookupOrCreateKey + is_filter).  row = -1 when not admitted.
__device__ __forceinline__ void apply_probe(const ApplyTable& at, int64_t i, int64_t ne,
                                            int64_t gs, int64_t* row_out, int* initmask_out,
                                            int* st) {
  const EvDesc& e = at.e;
  const ApplyCols& cols = at.cols;
  const int64_t* __restrict__ keys = at.keys;
  const int64_t steps_to_live = at.steps_to_live;
  int64_t row = -1;
  int initmask = 0;
  if (i < ne && at.rows) {
    // Rows known (dr_ev_apply_grouped_ptr_rows: SGD of a filter-free EV whose
    // forward resolved -- and initialised -- every key's row): what
    // LookupOrCreate would return, without probing the key table again.
    row = gld(at.rows + i);
    if (steps_to_live != 0 && gs != -1 && e.version) e.version[row] = gs;
  } else if (i < ne) {
    const uint64_t key = (uint64_t)keys[i];
    bool ok = true;
    if (e.k_hash > 0 && bloom_min_freq(e, key) < e.filter_freq) ok = false;
    if (ok) {
      bool created;
      uint64_t rc;
      Slot* s = ev_find(e, key, true, &created, &rc, st);
      if (s && (rc & kRowMask) != kRowDead) {
        row = (int64_t)(rc & kRowMask);
        if (steps_to_live != 0 && gs != -1 && e.version) e.version[row] = gs;
        if (e.filter_freq > 0 && e.k_hash == 0) {
          const int64_t f = (int64_t)__hip_atomic_fetch_add(
              (unsigned long long*)(e.freq + row), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (f < e.filter_freq) row = -1;
        }
        if (row >= 0) {
          uint64_t bits = 0;
          for (int c = 0; c < cols.ncol; ++c) bits |= 1ull << (48 + cols.cols[c]);
          if ((rc & bits) != bits) {
            const uint64_t old = atomicOr((unsigned long long*)&s->rc, (unsigned long long)bits);
            for (int c = 0; c < cols.ncol; ++c)
              if (!(old & (1ull << (48 + cols.cols[c])))) initmask |= 1 << c;
          }
        }
      }
    }
  }
  *row_out = row;
  *initmask_out = initmask;
}

// Row traffic of the apply: every gradient / weight / slot row is read once
// and written once per launch -- nontemporal policy unless DR_APPLY_NO_NT
// (A/B switch).
__device__ __forceinline__ float4 apply_ld(const float4* p) {
#ifdef DR_APPLY_NO_NT
  return *p;
#else
  return nt_load(p);
#endif
}
__device__ __forceinline__ float apply_ld(const float* p) {
#ifdef DR_APPLY_NO_NT
  return *p;
#else
  return nt_load(p);
#endif
}
__device__ __forceinline__ void apply_st(float4* p, float4 v) {
#ifdef DR_APPLY_NO_NT
  *p = v;
#else
  nt_store(v, p);
#endif
}
__device__ __forceinline__ void apply_st(float* p, float v) {
#ifdef DR_APPLY_NO_NT
  *p = v;
#else
  nt_store(v, p);
#endif
}

// Gradient row of apply entry i: row i of a dense [n, dim] block, or (gind)
// the address grad_ptr[i] handed on by dr_pool_grad_rows_grouped, whose bit
// 0 asks for the reference's 0 + x (-0.0f -> +0.0f) before use.
__device__ __forceinline__ uint64_t apply_grad_addr(const float* grad, int gind, int64_t i,
                                                    int64_t dim) {
  return gind ? reinterpret_cast<const uint64_t*>(grad)[i]
              : (uint64_t)(uintptr_t)(grad + i * dim);
}
// bf16 var rows of a bf16 EV: 4 values (8 B) per float4 lane chunk, or one
// value; widened to fp32 for the update and stored rounded to nearest even.
typedef unsigned int ab_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 apply_ldw(const ab_u2* p) {
#ifdef DR_APPLY_NO_NT
  const ab_u2 v = *gp(p);
#else
  const ab_u2 v = __builtin_nontemporal_load(gp(p));
#endif
  const float2 a = bf16x2_to_f2(v.x), b = bf16x2_to_f2(v.y);
  return make_float4(a.x, a.y, b.x, b.y);
}
__device__ __forceinline__ float apply_ldw(const uint16_t* p) { return bf16_to_f32(gld(p)); }
__device__ __forceinline__ void apply_stw(ab_u2* p, float4 w) {
  const ab_u2 v = {f2_to_bf16x2(w.x, w.y), f2_to_bf16x2(w.z, w.w)};
#ifdef DR_APPLY_NO_NT
  *gp(p) = v;
#else
  __builtin_nontemporal_store(v, gp(p));
#endif
}
__device__ __forceinline__ void apply_stw(uint16_t* p, float w) { gst(p, bf16_rne(w)); }

template <class V>
__device__ __forceinline__ V apply_grad_load(uint64_t a, int64_t c) {
  const V g = reinterpret_cast<const V*>((uintptr_t)(a & ~(uint64_t)1))[c];
  return (a & 1) ? vadd(vzero<V>(), g) : g;
}

// WB: the var column holds bf16 values (bf16 EV); gradients and optimizer
// slots stay fp32, the updated value is rounded to bf16 once per step.
template <int OPT, int VEC, int G, bool WB = false>
__global__ __launch_bounds__(256) void ev_apply_kernel(ApplyGroup ag, int64_t dim, int64_t gs,
                                                       OptScalars sc_arg, int gind, int* st) {
  const ApplyTable& at = ag.t[blockIdx.y];
  OptScalars sc = sc_arg;
  if ((OPT == OPT_ADAM_ASYNC || OPT == OPT_ADAM) && at.powers) {
    // alpha = lr * sqrt(1 - beta2_power) / (1 - beta1_power) in T = float
    // (training_ali_ops.cc:1529-1531; Adam :935-937), from the powers as they
    // stand in HBM
    const float b1p = gld(at.powers), b2p = gld(at.powers + 1);
    sc.alpha = sc.lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
  }
  const ApplyCols& cols = at.cols;
  const float* __restrict__ grad = at.grad;
  const int lane = threadIdx.x & 63;
  const int64_t base = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63);
  const int64_t ne = eff_n(at.n, at.n_dev);
  if (base >= ne) return;  // wave-uniform
  int64_t row;
  int initmask;
  apply_probe(at, base + lane, ne, gs, &row, &initmask, st);
  constexpr int P = 64 / G;                          // rows updated together
  constexpr bool C3 = opt_three_cols(OPT);
  constexpr int U = C3 ? 2 : 4;                      // row batches in flight
  const int sub = lane / G;
  const int lg = lane % G;
  const int64_t dv = dim / VEC;
  using V = typename std::conditional<VEC == 4, float4, float>::type;
  using WT = typename std::conditional<WB, typename std::conditional<VEC == 4, ab_u2, uint16_t>::type,
                                       V>::type;
  const WT* d0 = reinterpret_cast<const WT*>(cols.dflt[0]);
  const V* dg = reinterpret_cast<const V*>(cols.dflt[WB ? 1 : 0]);  // any readable row
  const V* d1 = reinterpret_cast<const V*>(cols.dflt[1]);
  const V* d2 = reinterpret_cast<const V*>(cols.dflt[2]);
  for (int k0 = 0; k0 < 64; k0 += P * U) {
    // cross-lane reads with every lane active (a disabled source lane reads 0)
    int64_t rr[U];
    // Row pointers chosen once per row, outside the column loop, and always
    // valid (a skipped row reads the default row): the loads of all U rows
    // issue back to back.  A "pointer or default" select inside the loop
    // makes hipcc branch around every load and wait for it.
    const V* gp[U];
    const WT* wp[U];
    const V* ap1[U];
    const V* ap2[U];
    bool zs[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int k = k0 + q * P + sub;
      rr[q] = __shfl(row, k, 64);
      const int im = __shfl(initmask, k, 64);
      if (base + k >= ne) rr[q] = -1;
      const bool ok = rr[q] >= 0;
      const uint64_t ga = ok ? apply_grad_addr(grad, gind, base + k, dim) : 0;
      zs[q] = ga & 1;
      gp[q] = ok ? reinterpret_cast<const V*>((uintptr_t)(ga & ~(uint64_t)1))
                 : (WB && OPT == OPT_SGD ? reinterpret_cast<const V*>(cols.dflt[0]) : dg);
      wp[q] = (ok && !(im & 1)) ? reinterpret_cast<const WT*>(cols.pool[0] + rr[q] * (WB ? dim / 2 : dim))
                                : d0;
      ap1[q] = (OPT != OPT_SGD && ok && !(im & 2))
                   ? reinterpret_cast<const V*>(cols.pool[1] + rr[q] * dim) : d1;
      ap2[q] = (C3 && ok && !(im & 4))
                   ? reinterpret_cast<const V*>(cols.pool[2] + rr[q] * dim) : d2;
    }
    // AdagradDecay: the row's decay count is element 0 of its
    // accum_decay_power row (a var-shaped slot, adagrad_decay.py:104-124);
    // the row decays when global_step / decay_step > that count (Tstep
    // division, compared as T)
    bool dec[U];
    float pw[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      dec[q] = false;
      pw[q] = 0.f;
      if (OPT == OPT_ADAGRAD_DECAY) {
        pw[q] = gld(reinterpret_cast<const float*>(ap2[q]));
        dec[q] = (float)(gs / sc.decay_step) > pw[q];
      }
    }
    for (int64_t c = lg; c < dv; c += G) {
      V gv[U], w[U], a1[U], a2[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {  // all loads of U rows first, unconditional
        if constexpr (WB) {
          // a skipped row of an SGD apply reads the (bf16) default for its
          // gradient too: half a row of bytes, always readable
          gv[q] = (OPT == OPT_SGD && rr[q] < 0) ? V{} : apply_ld(gp[q] + c);
          w[q] = apply_ldw(wp[q] + c);
        } else {
          gv[q] = apply_ld(gp[q] + c);
          w[q] = apply_ld(wp[q] + c);
        }
        if (OPT != OPT_SGD) a1[q] = apply_ld(ap1[q] + c);
        if (C3) a2[q] = apply_ld(ap2[q] + c);
      }
#pragma unroll
      for (int q = 0; q < U; ++q) {
        if (rr[q] < 0) continue;
        if (zs[q]) gv[q] = vadd(vzero<V>(), gv[q]);
        if constexpr (OPT == OPT_ADAGRAD_DECAY) {
          if constexpr (VEC == 4) {
            w[q].x = adagrad_decay_one(gv[q].x, w[q].x, &a1[q].x, dec[q], sc);
            w[q].y = adagrad_decay_one(gv[q].y, w[q].y, &a1[q].y, dec[q], sc);
            w[q].z = adagrad_decay_one(gv[q].z, w[q].z, &a1[q].z, dec[q], sc);
            w[q].w = adagrad_decay_one(gv[q].w, w[q].w, &a1[q].w, dec[q], sc);
            if (c == 0 && dec[q]) a2[q].x = pw[q] + 1.0f;   // accum_decay_power(0) += 1
          } else {
            w[q] = adagrad_decay_one(gv[q], w[q], &a1[q], dec[q], sc);
            if (c == 0 && dec[q]) a2[q] = pw[q] + 1.0f;
          }
        } else if constexpr (VEC == 4) {
          w[q].x = apply_one<OPT, VEC, G>(gv[q].x, w[q].x, &a1[q].x, &a2[q].x, sc);
          w[q].y = apply_one<OPT, VEC, G>(gv[q].y, w[q].y, &a1[q].y, &a2[q].y, sc);
          w[q].z = apply_one<OPT, VEC, G>(gv[q].z, w[q].z, &a1[q].z, &a2[q].z, sc);
          w[q].w = apply_one<OPT, VEC, G>(gv[q].w, w[q].w, &a1[q].w, &a2[q].w, sc);
        } else {
          w[q] = apply_one<OPT, VEC, G>(gv[q], w[q], &a1[q], &a2[q], sc);
        }
        if (OPT != OPT_SGD) apply_st(reinterpret_cast<V*>(cols.pool[1] + rr[q] * dim) + c, a1[q]);
        if (C3) apply_st(reinterpret_cast<V*>(cols.pool[2] + rr[q] * dim) + c, a2[q]);
        if constexpr (WB)
          apply_stw(reinterpret_cast<WT*>(cols.pool[0] + rr[q] * (dim / 2)) + c, w[q]);
        else
          apply_st(reinterpret_cast<V*>(cols.pool[0] + rr[q] * dim) + c, w[q]);
      }
    }
  }
}

// KvResourceSparseApplyFtrl[V2] (training_ali_ops.cc:167-331, COMPUTE_FTRL
// :279-307).  Phase 1 as above (columns var, accum, linear).  Phase 2, G
// lanes per row, two passes: (1) linear += gu - (new_accum^p - accum^p) / lr
// * var, stored, with the row's sum of squares reduced over the group by
// xor shuffles; (2) var = norm > l1 ? (l1 - norm) / ((new_accum^p / lr + 2
// l2) norm) * linear : 0, accum += g^2 (plain g, :307).  gu = g + 2 l2_shr
// var for V2.  p = 1/2 (sqrt) when lr_power == -0.5, else -lr_power (powf).
template <int VEC, int G>
__device__ __forceinline__ float ftrl_pow(float x, const OptScalars& sc) {
  return sc.lr_power == -0.5f ? sqrtf(x) : powf(x, -sc.lr_power);
}

template <int VEC, int G>
__global__ __launch_bounds__(256) void ev_apply_ftrl_kernel(ApplyGroup ag, int64_t dim,
                                                            int64_t gs, OptScalars sc, int gind,
                                                            int* st) {
  const ApplyTable& at = ag.t[blockIdx.y];
  const ApplyCols& cols = at.cols;
  const float* __restrict__ grad = at.grad;
  const int lane = threadIdx.x & 63;
  const int64_t base = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63);
  const int64_t ne = eff_n(at.n, at.n_dev);
  if (base >= ne) return;  // wave-uniform
  int64_t row;
  int initmask;
  apply_probe(at, base + lane, ne, gs, &row, &initmask, st);
  constexpr int P = 64 / G;
  const int sub = lane / G;
  const int lg = lane % G;
  const int64_t dv = dim / VEC;
  using V = typename std::conditional<VEC == 4, float4, float>::type;
  const bool shrink = sc.l2_shrinkage > 0.f;
  for (int k0 = 0; k0 < 64; k0 += P) {
    const int k = k0 + sub;
    int64_t r = __shfl(row, k, 64);  // every lane active for the shuffles
    const int im = __shfl(initmask, k, 64);
    if (base + k >= ne) r = -1;
    float ss = 0.f;
    const uint64_t ga = r >= 0 ? apply_grad_addr(grad, gind, base + k, dim) : 0;
    if (r >= 0) {
      V* wp = reinterpret_cast<V*>(cols.pool[0] + r * dim);
      V* ap = reinterpret_cast<V*>(cols.pool[1] + r * dim);
      V* lp = reinterpret_cast<V*>(cols.pool[2] + r * dim);
      const V* d0 = reinterpret_cast<const V*>(cols.dflt[0]);
      const V* d1 = reinterpret_cast<const V*>(cols.dflt[1]);
      const V* d2 = reinterpret_cast<const V*>(cols.dflt[2]);
      for (int64_t c = lg; c < dv; c += G) {
        const V gv = apply_grad_load<V>(ga, c);
        const V w = (im & 1) ? d0[c] : wp[c];
        const V a = (im & 2) ? d1[c] : ap[c];
        V l = (im & 4) ? d2[c] : lp[c];
        const float* gf = reinterpret_cast<const float*>(&gv);
        const float* wf = reinterpret_cast<const float*>(&w);
        const float* af = reinterpret_cast<const float*>(&a);
        float* lf = reinterpret_cast<float*>(&l);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float gu = shrink ? gf[j] + 2.0f * sc.l2_shrinkage * wf[j] : gf[j];
          const float na = af[j] + gu * gu;
          const float dp = ftrl_pow<VEC, G>(na, sc) - ftrl_pow<VEC, G>(af[j], sc);
          const float t = dp / sc.lr * wf[j];
          lf[j] = lf[j] + (gu - t);
          ss += lf[j] * lf[j];
        }
        lp[c] = l;
      }
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
    if (r < 0) continue;
    const float norm = sqrtf(ss);
    V* wp = reinterpret_cast<V*>(cols.pool[0] + r * dim);
    V* ap = reinterpret_cast<V*>(cols.pool[1] + r * dim);
    const V* lp = reinterpret_cast<const V*>(cols.pool[2] + r * dim);
    const V* d0 = reinterpret_cast<const V*>(cols.dflt[0]);
    const V* d1 = reinterpret_cast<const V*>(cols.dflt[1]);
    for (int64_t c = lg; c < dv; c += G) {
      const V gv = apply_grad_load<V>(ga, c);
      V w = (im & 1) ? d0[c] : wp[c];
      V a = (im & 2) ? d1[c] : ap[c];
      const V l = lp[c];
      const float* gf = reinterpret_cast<const float*>(&gv);
      float* wf = reinterpret_cast<float*>(&w);
      float* af = reinterpret_cast<float*>(&a);
      const float* lf = reinterpret_cast<const float*>(&l);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float gu = shrink ? gf[j] + 2.0f * sc.l2_shrinkage * wf[j] : gf[j];
        const float na = af[j] + gu * gu;
        if (norm > sc.l1) {
          const float eta_rec = ftrl_pow<VEC, G>(na, sc) / sc.lr;
          const float coef = (sc.l1 - norm) / ((eta_rec + 2.0f * sc.l2) * norm);
          wf[j] = coef * lf[j];
        } else {
          wf[j] = 0.f;
        }
        af[j] = af[j] + gf[j] * gf[j];
      }
      wp[c] = w;
      ap[c] = a;
    }
  }
}

// ---------------------------------------------------------------------------
// Save-time eviction, EmbeddingVar::Shrink (embedding_var.h:264-313), called
// by DumpEv before DumpEmbeddingValues (save_restore_v2_ops.cc:128-131):
//   l2_weight_threshold != -1 : drop keys whose 0.5 * sum_j v_j^2 (primary
//                               row, ascending j in fp32) < threshold
//   else, steps_to_live > 0   : version == -1 -> version = gs; drop keys
//                               with gs - version > steps_to_live
// Marking is one thread per slot; the kept slots are rehashed into a fresh
// table (linear probing has no tombstones).  Rows of dropped keys are not
// recycled ("TODO memory recycle" in the reference too).
// ---------------------------------------------------------------------------
__global__ void ev_shrink_mark_kernel(Slot* __restrict__ slots, int64_t cap, const float* pool,
                                      const float* dflt, int64_t dim, int bf16,
                                      int64_t* __restrict__ version,
                                      int mode, float l2_threshold, int64_t gs,
                                      int64_t steps_to_live, uint8_t* __restrict__ keep,
                                      unsigned long long* __restrict__ nremoved) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > cap) return;
  const Slot sl = slots[i];
  const bool occupied = i < cap ? sl.key != kEmptyKey : sl.key == 0ull;
  uint8_t k = 1;
  if (occupied && sl.rc != kUnset && (sl.rc & kRowMask) != kRowDead) {
    const int64_t row = (int64_t)(sl.rc & kRowMask);
    if (mode == 1) {
      float l2 = 0.f;
      if (bf16) {  // dim bf16 values, widened (fp32 sum in element order)
        const uint16_t* v = reinterpret_cast<const uint16_t*>(
            (sl.rc & (1ull << 48)) ? pool + row * (dim / 2) : dflt);
        for (int64_t j = 0; j < dim; ++j) {
          const float x = bf16_to_f32(v[j]);
          l2 += x * x;
        }
      } else {
        const float* v = (sl.rc & (1ull << 48)) ? pool + row * dim : dflt;
        for (int64_t j = 0; j < dim; ++j) l2 += v[j] * v[j];
      }
      l2 *= 0.5f;
      if (l2 < l2_threshold) k = 0;
    } else if (mode == 2 && version) {
      const int64_t ver = version[row];
      if (ver == -1)
        version[row] = gs;
      else if (gs - ver > steps_to_live)
        k = 0;
    }
  }
  keep[i] = k;
  if (!k) atomicAdd(nremoved, 1ull);
}

__global__ void ev_rehash_kept_kernel(const Slot* __restrict__ old_slots, int64_t cap,
                                      const uint8_t* __restrict__ keep,
                                      Slot* __restrict__ new_slots) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > cap) return;
  const Slot s = old_slots[i];
  if (i == cap) {  // the key -1 slot
    if (keep[i]) new_slots[cap] = s;
    return;
  }
  if (s.key == kEmptyKey || !keep[i]) return;
  const uint64_t mask = (uint64_t)cap - 1;
  const uint64_t h0 = mix64(s.key) & mask;
  for (uint64_t i = 0;; ++i) {
    const uint64_t h = probe_slot(h0, i, mask);
    uint64_t old = atomicCAS((unsigned long long*)&new_slots[h].key, (unsigned long long)kEmptyKey,
                             (unsigned long long)s.key);
    if (old == kEmptyKey) {
      new_slots[h].rc = s.rc;
      return;
    }
  }
}

// ---------------------------------------------------------------------------
// Rehash into a larger slot table (growth).
// ---------------------------------------------------------------------------
__global__ void ev_rehash_kernel(const Slot* __restrict__ old_slots, int64_t old_cap,
                                 Slot* __restrict__ new_slots, int64_t new_cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= old_cap) return;
  const Slot s = old_slots[i];
  if (s.key == kEmptyKey) return;
  const uint64_t mask = (uint64_t)new_cap - 1;
  const uint64_t h0 = mix64(s.key) & mask;
  for (uint64_t i = 0;; ++i) {
    const uint64_t h = probe_slot(h0, i, mask);
    uint64_t old = atomicCAS((unsigned long long*)&new_slots[h].key, (unsigned long long)kEmptyKey,
                             (unsigned long long)s.key);
    if (old == kEmptyKey) {
      new_slots[h].rc = s.rc;
      return;
    }
  }
}

// ---- host helpers ------------------------------------------------------------
static void bloom_params(int64_t max_element_size, float fpp, int64_t* k, int64_t* nc) {
  // EmbeddingConfig::calc_num_hash_func / calc_num_counter (embedding_config.h:63-70)
  float loghpp = fabsf((float)(log(fpp) / log(2)));
  *k = (int64_t)ceil(loghpp);
  float loghpp2 = fabsf((float)log(fpp));
  float factor = (float)(log(2) * log(2));
  *nc = (int64_t)ceil(loghpp2 / factor * max_element_size);
}

static void bloom_seeds(int64_t k, std::vector<uint64_t>* out) {
  // BloomFilter::GenerateSeed (embedding_filter.h:252-279)
  static const int64_t defaults[25] = {2,  3,  5,  7,  11, 13, 17, 19, 23, 29, 31, 37, 41,
                                       43, 47, 53, 59, 61, 67, 71, 73, 79, 83, 89, 97};
  out->clear();
  for (int64_t i = 0; i < k && i < 25; ++i) out->push_back((uint64_t)defaults[i]);
  int64_t last = 98;
  for (int64_t i = 25; i < k; ++i) {
    for (int64_t j = last;; ++j) {
      if (j % 2 == 0) continue;
      bool prime = true;
      for (int64_t q = 2; q <= (int64_t)std::sqrt((double)j) + 1; ++q)
        if (j % q == 0) {
          prime = false;
          break;
        }
      if (prime) {
        out->push_back((uint64_t)j);
        last = j;
        break;
      }
    }
  }
}

static int alloc_pool(EvShared* s, int col, const float* default_row_host) {
  const int64_t w = col_words(s, col);
  DR_HIP(hipMalloc(&s->pools[col], (size_t)s->row_cap * w * sizeof(float)));
  DR_HIP(hipMalloc(&s->defaults[col], (size_t)w * sizeof(float)));
#ifdef DR_UC_DIAG
  // poison: a 0xFF word read later was never written by the init / copy;
  // a 0 word came from stale backing (the uncached blocks were zero-filled)
  {
    int frc = fill_bytes(s->pools[col], 0xFF, (size_t)s->row_cap * w * sizeof(float), nullptr);
    if (!frc) frc = fill_bytes(s->defaults[col], 0xFF, (size_t)w * sizeof(float), nullptr);
    if (frc) return frc;
    DR_HIP(hipDeviceSynchronize());
    const size_t cb = (size_t)std::min<int64_t>(s->row_cap * w, 1 << 18) * sizeof(float);
    if (uc_diag_check_xcd("new pool (poisoned)", s->pools[col], 0xFFFFFFFFu, cb)) {
      uc_diag_writeback(0);
      if (uc_diag_check_xcd("  after an agent-scope L2 write-back", s->pools[col], 0xFFFFFFFFu, cb)) {
        uc_diag_writeback(1);
        uc_diag_check_xcd("  after a system-scope L2 write-back", s->pools[col], 0xFFFFFFFFu, cb);
      }
    }
  }
#endif
  if (w != s->dim) {
    // bf16 column: the fp32 default row rounded to nearest even
    std::vector<uint16_t> b((size_t)s->dim);
    for (int64_t c = 0; c < s->dim; ++c) b[(size_t)c] = bf16_rne_host(default_row_host[c]);
    DR_HIP(hipMemcpy(s->defaults[col], b.data(), b.size() * sizeof(uint16_t),
                     hipMemcpyHostToDevice));
#ifdef DR_UC_DIAG
    uc_diag_check("default row (bf16)", s->defaults[col], b.data(), b.size() * 2);
#endif
  } else {
    DR_HIP(hipMemcpy(s->defaults[col], default_row_host, s->dim * sizeof(float),
                     hipMemcpyHostToDevice));
#ifdef DR_UC_DIAG
    uc_diag_check("default row", s->defaults[col], default_row_host, s->dim * sizeof(float));
#endif
  }
  return DR_OK;
}

static void free_shared(EvShared* s) {
  (void)hipFree(s->slots);
  (void)hipFree(s->top);
  (void)hipFree(s->freq);
  (void)hipFree(s->version);
  for (int c = 0; c < kMaxCols; ++c) {
    (void)hipFree(s->pools[c]);
    (void)hipFree(s->defaults[c]);
  }
  (void)hipFree(s->bloom);
  (void)hipFree(s->seeds);
  if (s->copy_ev) (void)hipEventDestroy(s->copy_ev);
  if (s->update_ev) (void)hipEventDestroy(s->update_ev);
  if (s->pinned_top) (void)hipHostFree(s->pinned_top);
  delete s;
}

// Grow the slot table and/or the row arrays so that `need` keys fit.
// Diagnostic (tools/gpu_uc_reuse.sh): DR_GROW_KERNEL_COPY=1 copies the
// pools with a kernel instead of hipMemcpyAsync (the DMA copy path).
__global__ void grow_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                 int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

static hipError_t grow_copy(void* dst, const void* src, size_t bytes, hipStream_t st) {
  static const bool kcopy = getenv("DR_GROW_KERNEL_COPY") != nullptr;
  if (!kcopy || bytes % 16 || ((uintptr_t)dst | (uintptr_t)src) % 16)
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st);
  const int64_t n16 = (int64_t)(bytes / 16);
  const int64_t blocks = std::min<int64_t>(std::max<int64_t>(ceil_div(n16, 256), 1), 4096);
  hipLaunchKernelGGL(grow_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     static_cast<const uint4*>(src), static_cast<uint4*>(dst), n16);
  return hipGetLastError();
}

static int grow(EvShared* s, int64_t need, hipStream_t st) {
  // kernels other streams enqueued on the old table / pools must be done
  // before they are copied and freed (EvGuard keeps new ones from starting)
  DR_HIP(hipDeviceSynchronize());
  if (need > s->cap * 3 / 4) {
    int64_t ncap = next_pow2(need * 2);
    Slot* ns = nullptr;
    DR_HIP(hipMalloc(&ns, (size_t)(ncap + 1) * sizeof(Slot)));
    int frc = fill_bytes(ns, 0xFF, (size_t)(ncap + 1) * sizeof(Slot), st);
    if (frc) return frc;
    hipLaunchKernelGGL(ev_rehash_kernel, dim3((unsigned)ceil_div(s->cap, 256)), dim3(256), 0, st,
                       s->slots, s->cap, ns, ncap);
    DR_LAUNCH_CHECK();
    DR_HIP(hipMemcpyAsync(ns + ncap, s->slots + s->cap, sizeof(Slot), hipMemcpyDeviceToDevice, st));
    DR_HIP(hipStreamSynchronize(st));
    DR_HIP(hipFree(s->slots));
    s->slots = ns;
    s->cap = ncap;
  }
  if (need > s->row_cap) {
    int64_t nrc = std::max(need, s->row_cap * 2);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess &&
        (size_t)nrc * col_words(s, 0) * sizeof(float) > fr) {
      set_error("EV row pool growth %lld -> %lld rows (need %lld) needs %zu bytes, %zu free",
                (long long)s->row_cap, (long long)nrc, (long long)need,
                (size_t)nrc * col_words(s, 0) * sizeof(float), fr);
      return DR_RESOURCE_EXHAUSTED;
    }
    for (int c = 0; c < kMaxCols; ++c) {
      if (!s->pools[c]) continue;
      const int64_t w = col_words(s, c);
      float* np = nullptr;
      DR_HIP(hipMalloc(&np, (size_t)nrc * w * sizeof(float)));
#ifdef DR_UC_DIAG
      {
        int frc = fill_bytes(np, 0xFF, (size_t)nrc * w * sizeof(float), st);
        if (frc) return frc;
      }
#endif
      DR_HIP(grow_copy(np, s->pools[c], (size_t)s->row_cap * w * sizeof(float), st));
      DR_HIP(hipStreamSynchronize(st));
#ifdef DR_UC_DIAG
      {
        const size_t cb = (size_t)std::min<int64_t>(s->row_cap * w, 4096) * sizeof(float);
        std::vector<float> old(cb / 4);
        DR_HIP(hipMemcpy(old.data(), s->pools[c], cb, hipMemcpyDeviceToHost));
        uc_diag_check("grown pool (head)", np, old.data(), cb);
      }
#endif
      DR_HIP(hipFree(s->pools[c]));
      s->pools[c] = np;
    }
    int64_t** arrs[2] = {&s->freq, &s->version};
    for (auto a : arrs) {
      if (!*a) continue;
      int64_t* np = nullptr;
      DR_HIP(hipMalloc(&np, (size_t)nrc * sizeof(int64_t)));
      int frc = fill_bytes(np, 0, (size_t)nrc * sizeof(int64_t), st);
      if (frc) return frc;
      DR_HIP(grow_copy(np, *a, (size_t)s->row_cap * sizeof(int64_t), st));
      DR_HIP(hipStreamSynchronize(st));
      DR_HIP(hipFree(*a));
      *a = np;
    }
    s->row_cap = nrc;
  }
  return DR_OK;
}

// Make sure `n` more keys fit.  Steady state: no host sync (the device key
// count is mirrored asynchronously into pinned memory after every call).
static int reserve(EvShared* s, int64_t n, hipStream_t st) {
  std::lock_guard<std::mutex> g(s->mu);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(st, &cs);
  const bool capturing = cs != hipStreamCaptureStatusNone;
  // (event queries are illegal while a global-mode capture is open)
  if (!capturing && s->copy_pending && hipEventQuery(s->copy_ev) == hipSuccess) {
    // a mirror taken on stream X holds every add reserved before it only if
    // all of those were issued on X (EvGuard keeps each call's reserve and
    // launch together); otherwise it is dropped and the count stays an
    // over-estimate
    if (s->copy_exact) {
      s->known = *s->pinned_top;
      s->adds_since_known = s->adds_since_copy;
      s->adds = s->copy_adds;
    }
    s->copy_pending = false;
  }
  const int64_t limit = std::min(s->row_cap, s->cap * 3 / 4);
  if (s->known + s->adds_since_known + n > limit) {
    DR_REQUIRE(!capturing, DR_RESOURCE_EXHAUSTED,
               "EV capacity may be exceeded inside stream capture; dr_ev_reserve first");
    // every reserved add must have run before `top` is read: other streams'
    // too (no new launch on this EV can start: the caller holds its EvGuard)
    if (s->adds.only(st))
      DR_HIP(hipStreamSynchronize(st));
    else
      DR_HIP(hipDeviceSynchronize());
    int64_t actual = 0;
    DR_HIP(hipMemcpy(&actual, s->top, sizeof(int64_t), hipMemcpyDeviceToHost));
    s->known = actual;
    s->adds_since_known = 0;
    s->adds = EvShared::Streams();
    s->copy_pending = false;
    if (actual + n > limit) {
      int rc = grow(s, actual + n, st);
      if (rc) return rc;
    }
  }
  s->adds_since_known += n;
  s->adds.note(st);
  if (s->copy_pending) {
    s->adds_since_copy += n;
    s->copy_adds.note(st);
  }
  return DR_OK;
}

// Mirror of the device row counter into pinned host memory (capacity
// accounting without syncs).  want_mirror() says whether a fresh copy should
// be issued now; the copy is either a DMA (post_call) or written by the
// stream's next init kernel (resolve paths), followed by mirrored().
static bool want_mirror(EvShared* s, hipStream_t st) {
  static const bool no_mirror = getenv("DR_NO_MIRROR") != nullptr;
  if (no_mirror || s->copy_pending) return false;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(st, &cs);
  return cs == hipStreamCaptureStatusNone;
}

static void mirrored(EvShared* s, hipStream_t st) {
  if (hipEventRecord(s->copy_ev, st) != hipSuccess) return;
  s->copy_pending = true;
  s->copy_exact = s->adds.only(st);
  s->adds_since_copy = 0;
  s->copy_adds = EvShared::Streams();
}

static void post_call(EvShared* s, hipStream_t st) {
  std::lock_guard<std::mutex> g(s->mu);
  if (!want_mirror(s, st)) return;
  if (hipMemcpyAsync(s->pinned_top, s->top, sizeof(int64_t), hipMemcpyDeviceToHost, st) !=
      hipSuccess)
    return;
  mirrored(s, st);
}

struct ResolveWs {
  uint8_t* init;
  int32_t* badd;
};
static ResolveWs carve_resolve(void* ws, int64_t n, size_t* used) {
  Carver c(ws);
  ResolveWs w;
  w.init = c.take<uint8_t>(n > 0 ? n : 1);
  w.badd = c.take<int32_t>(n > 0 ? n : 1);
  if (used) *used = c.used + 256;
  return w;
}

static int resolve_grouped(dr_ev* const* evs, int T, const int64_t* keys, const int64_t* koff,
                           const int64_t* const* n_dev, const float* const* defaults,
                           const int32_t* counts, int64_t* rows_out, void* ws, size_t ws_bytes,
                           hipStream_t st, const int32_t* tags = nullptr,
                           const int64_t* per_table_host = nullptr) {
  EvGuard guard_(evs, T);
  const bool composite = tags != nullptr;
  DR_REQUIRE(T >= 1 && T <= DR_MAX_GROUP, DR_INVALID_ARGUMENT, "bad table count");
  const int64_t total = koff[T];
  size_t need = 0;
  carve_resolve(nullptr, total, &need);
  DR_REQUIRE(ws_bytes >= need, DR_INVALID_ARGUMENT, "resolve workspace too small");
  if (total == 0) return DR_OK;
  int* stw = status_word();
  DR_REQUIRE(stw, DR_INTERNAL, "status word unavailable");
  for (int t = 0; t < T; ++t) {
    const int64_t nt = composite ? (per_table_host ? per_table_host[t] : total)
                                 : koff[t + 1] - koff[t];
    int rc = reserve(evs[t]->sh, nt, st);
    if (rc) return rc;
  }
  ResolveWs w = carve_resolve(ws, total, nullptr);
  EvGroup g;
  memset(&g, 0, sizeof(g));
  InitGroup ig;
  memset(&ig, 0, sizeof(ig));
  bool any_bloom = false;
  g.tags = tags;
  ig.tags = tags;
  for (int t = 0; t < T; ++t) {
    g.e[t] = make_desc(evs[t]);
    g.koff[t] = composite ? 0 : koff[t];
    g.n_dev[t] = n_dev ? n_dev[composite ? 0 : t] : nullptr;
    ig.pool[t] = evs[t]->sh->pools[evs[t]->col];
    ig.src[t] = defaults ? defaults[t] : nullptr;
    ig.dflt[t] = evs[t]->sh->defaults[evs[t]->col];
    ig.koff[t] = g.koff[t];
    ig.n_dev[t] = g.n_dev[t];
    any_bloom |= g.e[t].k_hash > 0;
    DR_REQUIRE(col_words(evs[t]->sh, evs[t]->col) == col_words(evs[0]->sh, evs[0]->col) &&
                   evs[t]->sh->dim == evs[0]->sh->dim && evs[t]->sh->bf16 == evs[0]->sh->bf16,
               DR_INVALID_ARGUMENT, "grouped EVs must share dim and value type");
  }
  g.koff[T] = total;
  ig.koff[T] = total;
  const unsigned blocks = (unsigned)ceil_div(total, 256);
  hipLaunchKernelGGL(ev_resolve_kernel, dim3(blocks), dim3(256), 0, st, g, T, keys, counts,
                     rows_out, w.init, any_bloom ? w.badd : nullptr, stw);
  if (any_bloom)
    hipLaunchKernelGGL(ev_bloom_add_kernel, dim3(blocks), dim3(256), 0, st, g, T, keys, w.badd);
  // counter mirrors ride on the init kernel (no extra copy launches)
  EvShared* mir[DR_MAX_GROUP];
  int nmir = 0;
  for (int t = 0; t < T; ++t) {
    EvShared* sh = evs[t]->sh;
    bool seen = false;
    for (int q = 0; q < nmir; ++q) seen = seen || mir[q] == sh;
    if (seen) continue;
    sh->mu.lock();
    if (want_mirror(sh, st)) {
      ig.mtop[t] = sh->top;
      ig.mdst[t] = sh->pinned_top;
      mir[nmir++] = sh;
    } else {
      sh->mu.unlock();
    }
  }
  hipLaunchKernelGGL(ev_init_rows_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, st, ig,
                     T, col_words(evs[0]->sh, evs[0]->col), rows_out, w.init);
  const hipError_t le = hipGetLastError();
  for (int q = 0; q < nmir; ++q) {
    if (le == hipSuccess) mirrored(mir[q], st);
    mir[q]->mu.unlock();
  }
  if (le != hipSuccess) {
    set_error("kernel launch failed: %s", hipGetErrorString(le));
    return DR_INTERNAL;
  }
  return DR_OK;
}

// AdamAsync beta powers, after the apply (training_ali_ops.cc:1558-1559):
// beta1_power *= beta1, beta2_power *= beta2 -- only for tables whose
// gradient had rows (the op's `if (N > 0)`, :1482; N = the device count when
// one is given, so a fixed-capacity slice with no valid row leaves them).
struct PowersArgs {
  float* p[DR_MAX_GROUP];
  int64_t n[DR_MAX_GROUP];
  const int64_t* n_dev[DR_MAX_GROUP];
};
__global__ void ev_adam_powers_kernel(PowersArgs a, int T, float beta1, float beta2) {
  const int t = threadIdx.x;
  if (t >= T || !a.p[t]) return;
  if (eff_n(a.n[t], a.n_dev[t]) <= 0) return;
  a.p[t][0] = a.p[t][0] * beta1;
  a.p[t][1] = a.p[t][1] * beta2;
}

// Grouped sparse apply: T tables (same dim) per launch, blockIdx.y = table,
// in chunks of kApplyGroup.  A single-table apply is a group of one.
static int apply_grouped(int opt, dr_ev* const* vars, dr_ev* const* s1, dr_ev* const* s2, int T,
                         OptScalars sc, const float* const* grads, const int64_t* const* keys,
                         const int64_t* n_host, const int64_t* const* n_dev, int64_t gs,
                         hipStream_t st, int gind = 0, const int64_t* const* rows = nullptr,
                         float* const* powers = nullptr, bool advance_powers = true) {
  EvGuard guard_(vars, T);
  DR_REQUIRE(!rows || opt == OPT_SGD, DR_INVALID_ARGUMENT,
             "known rows skip the slot-column first-touch check: SGD only");
  DR_REQUIRE(T >= 1 && vars && grads && keys && n_host, DR_INVALID_ARGUMENT, "bad argument");
  int* stw = status_word();
  DR_REQUIRE(stw, DR_INTERNAL, "status word unavailable");
  const int64_t dim = vars[0] ? vars[0]->sh->dim : 0;
  const int ncol = opt == OPT_SGD ? 1 : (opt_three_cols(opt) || opt == OPT_FTRL ? 3 : 2);
  // Capacity first: a reserve may grow (reallocate) the slot table and the
  // row pools, so no pointer may be read into a descriptor before it.
  for (int t = 0; t < T; ++t) {
    DR_REQUIRE(vars[t] && vars[t]->col == 0, DR_INVALID_ARGUMENT,
               "table %d: var must be a primary EV", t);
    DR_REQUIRE(vars[t]->sh->value_words == 1, DR_INVALID_ARGUMENT,
               "table %d: the KvResourceSparseApply* kernels are registered for float values "
               "only (training_ali_ops.cc)", t);
    DR_REQUIRE(!vars[t]->sh->bf16 || opt != OPT_FTRL, DR_INVALID_ARGUMENT,
               "table %d: FTRL is not built for bf16 EVs", t);
    if (n_host[t] > 0) {
      int rc = reserve(vars[t]->sh, n_host[t], st);
      if (rc) return rc;
    }
  }
  for (int c0 = 0; c0 < T; c0 += kApplyGroup) {
    const int tn = std::min(kApplyGroup, T - c0);
    ApplyGroup ag;
    memset(&ag, 0, sizeof(ag));
    int64_t nmax = 0;
    bool aligned = dim % 4 == 0;
    for (int j = 0; j < tn; ++j) {
      const int t = c0 + j;
      dr_ev* var = vars[t];
      EvShared* s = var->sh;
      DR_REQUIRE(s->dim == dim && s->bf16 == vars[0]->sh->bf16, DR_INVALID_ARGUMENT,
                 "grouped apply needs equal dims and value types");
      dr_ev* cv[3] = {var, s1 ? s1[t] : nullptr, s2 ? s2[t] : nullptr};
      ApplyTable& a = ag.t[j];
      a.cols.ncol = ncol;
      for (int c = 0; c < ncol; ++c) {
        DR_REQUIRE(cv[c] && cv[c]->sh == s, DR_INVALID_ARGUMENT,
                   "table %d: slot EV missing or not sharing the primary's keys", t);
        a.cols.cols[c] = cv[c]->col;
        a.cols.pool[c] = s->pools[cv[c]->col];
        a.cols.dflt[c] = s->defaults[cv[c]->col];
        aligned = aligned && ((((uintptr_t)a.cols.pool[c]) | ((uintptr_t)a.cols.dflt[c])) & 15) == 0;
      }
      // by-address rows (gind) are 16-byte aligned when dim % 4 == 0
      // (dr_pool_grad_rows_grouped defers only aligned rows)
      aligned = aligned && (gind || (((uintptr_t)grads[t]) & 15) == 0);
      a.e = make_desc(var);
      a.keys = keys[t];
      a.grad = grads[t];
      a.n = n_host[t];
      a.n_dev = n_dev ? n_dev[t] : nullptr;
      a.steps_to_live = s->steps_to_live;
      if (rows) {
        DR_REQUIRE(rows[t] && s->filter_freq == 0 && s->k_hash == 0, DR_INVALID_ARGUMENT,
                   "table %d: known rows need a filter-free EV and a rows array", t);
        a.rows = rows[t];
      }
      if (powers) a.powers = powers[t];
      nmax = std::max(nmax, a.n);
    }
    if (nmax == 0) continue;
    const dim3 grid((unsigned)ceil_div(nmax, 256), (unsigned)tn);
#define DR_APPLY(VEC, G, WB)                                                                    \
  do {                                                                                     \
    if (opt == OPT_SGD)                                                                    \
      hipLaunchKernelGGL((ev_apply_kernel<OPT_SGD, VEC, G, WB>), grid, dim3(256), 0, st, ag,    \
                         dim, gs, sc, gind, stw);                                           \
    else if (opt == OPT_ADAGRAD)                                                           \
      hipLaunchKernelGGL((ev_apply_kernel<OPT_ADAGRAD, VEC, G, WB>), grid, dim3(256), 0, st, ag,\
                         dim, gs, sc, gind, stw);                                           \
    else if (opt == OPT_FTRL)                                                              \
      hipLaunchKernelGGL((ev_apply_ftrl_kernel<VEC, G>), grid, dim3(256), 0, st, ag, dim,   \
                         gs, sc, gind, stw);                                                \
    else if (opt == OPT_ADAM_ASYNC)                                                        \
      hipLaunchKernelGGL((ev_apply_kernel<OPT_ADAM_ASYNC, VEC, G, WB>), grid, dim3(256), 0, st, \
                         ag, dim, gs, sc, gind, stw);                                       \
    else if (opt == OPT_ADAM_RMSPROP)                                                      \
      hipLaunchKernelGGL((ev_apply_kernel<OPT_ADAM_RMSPROP, VEC, G, WB>), grid, dim3(256), 0,   \
                         st, ag, dim, gs, sc, gind, stw);                                   \
    else if (opt == OPT_ADAGRAD_DECAY)                                                     \
      hipLaunchKernelGGL((ev_apply_kernel<OPT_ADAGRAD_DECAY, VEC, G, WB>), grid, dim3(256), 0,  \
                         st, ag, dim, gs, sc, gind, stw);                                   \
    else                                                                                   \
      hipLaunchKernelGGL((ev_apply_kernel<OPT_ADAM, VEC, G, WB>), grid, dim3(256), 0, st, ag,   \
                         dim, gs, sc, gind, stw);                                           \
  } while (0)
    const bool wb = vars[c0]->sh->bf16 != 0;
    if (wb && aligned && dim / 4 <= 8)
      DR_APPLY(4, 8, true);
    else if (wb && aligned && dim / 4 <= 16)
      DR_APPLY(4, 16, true);
    else if (wb && aligned && dim / 4 <= 32)
      DR_APPLY(4, 32, true);
    else if (wb && aligned)
      DR_APPLY(4, 64, true);
    else if (wb)
      DR_APPLY(1, 64, true);
    else if (aligned && dim / 4 <= 8)
      DR_APPLY(4, 8, false);
    else if (aligned && dim / 4 <= 16)
      DR_APPLY(4, 16, false);
    else if (aligned && dim / 4 <= 32)
      DR_APPLY(4, 32, false);
    else if (aligned)
      DR_APPLY(4, 64, false);
    else if (dim <= 4)    // narrow unaligned rows (a linear model's dim 1): 16 rows per pass
      DR_APPLY(1, 4, false);
    else if (dim <= 32)   // DIN's D = 18
      DR_APPLY(1, 32, false);
    else
      DR_APPLY(1, 64, false);
#undef DR_APPLY
    DR_LAUNCH_CHECK();
  }
  if (powers && advance_powers) {
    for (int c0 = 0; c0 < T; c0 += DR_MAX_GROUP) {
      const int tn = std::min(DR_MAX_GROUP, T - c0);
      PowersArgs pa;
      memset(&pa, 0, sizeof(pa));
      for (int j = 0; j < tn; ++j) {
        pa.p[j] = powers[c0 + j];
        pa.n[j] = n_host[c0 + j];
        pa.n_dev[j] = n_dev ? n_dev[c0 + j] : nullptr;
      }
      hipLaunchKernelGGL(ev_adam_powers_kernel, dim3(1), dim3(64), 0, st, pa, tn, sc.beta1,
                         sc.beta2);
      DR_LAUNCH_CHECK();
    }
  }
  // no counter mirror here: the step's next resolve refreshes it
  return DR_OK;
}

// DR_OPT_* of dr_ev_apply_grouped[_ptr] -> kernel optimizer + scalars.
// Adam / AdamAsync: alpha = lr * sqrt(1 - beta2^t) / (1 - beta1^t)
// (training_ali_ops.cc:935-937, :1529-1531).
static int grouped_opt(int optimizer, float lr, float beta1_power, float beta2_power, float beta1,
                       float beta2, float epsilon, int* opt, OptScalars* sc) {
  DR_REQUIRE(optimizer >= DR_OPT_SGD && optimizer <= DR_OPT_ADAM_ASYNC_RMSPROP,
             DR_INVALID_ARGUMENT, "unknown optimizer %d", optimizer);
  *sc = OptScalars{};
  sc->lr = lr;
  sc->beta1 = beta1;
  sc->beta2 = beta2;
  sc->eps = epsilon;
  if (optimizer == DR_OPT_ADAM || optimizer == DR_OPT_ADAM_ASYNC)
    sc->alpha = lr * sqrtf(1.0f - beta2_power) / (1.0f - beta1_power);
  static const int map[] = {OPT_SGD, OPT_ADAGRAD, OPT_ADAM, OPT_ADAM_ASYNC, OPT_ADAM_RMSPROP};
  *opt = map[optimizer];
  return DR_OK;
}

static int apply_common(int opt, dr_ev* var, dr_ev* s1, dr_ev* s2, OptScalars sc,
                        const float* grad, const int64_t* keys, int64_t n, const int64_t* n_dev,
                        int64_t gs, hipStream_t st) {
  DR_REQUIRE(var && var->col == 0, DR_INVALID_ARGUMENT, "var must be a primary EV");
  if (n == 0) return DR_OK;
  dr_ev* v[1] = {var};
  dr_ev* a[1] = {s1};
  dr_ev* b[1] = {s2};
  const float* g[1] = {grad};
  const int64_t* k[1] = {keys};
  const int64_t nh[1] = {n};
  const int64_t* nd[1] = {n_dev};
  return apply_grouped(opt, v, a, b, 1, sc, g, k, nh, nd, gs, st);
}


// ---------------------------------------------------------------------------
// Fused one-hot forward lookup (dr_ev_lookup_onehot): filter-free EVs, bag b
// of table t = id t*B + b, output [B, T*D] concat.  One kernel probes the key
// table and copies the row straight into the output, in output-slot order
// (slot j = b*T + t, the pool_onehot_kernel layout); the resolve pass and
// its row-index array disappear from the step.  The probe is read-only: a
// key that is absent, still being created, or whose column has not been
// initialised is appended to a miss list, and one small kernel finishes
// those slots exactly as resolve -> init -> copy would (insert-on-miss with
// the creator-first protocol of ev_find, first-touch default row, copy).
// In steady state the list is empty and it exits at once.
// ---------------------------------------------------------------------------
struct LkDesc {
  const Slot* slots;
  int64_t cap;
  const float* pool;
  uint64_t colbit;
};

struct LookupArgs {
  LkDesc d[DR_MAX_GROUP];
  const int64_t* keys;  // id of (bag b, table t) = keys[b * ksb + t * kst]
  int64_t ksb, kst;     // [T, B] feature-major: (1, B); [B, T] record-major: (T, 1)
  float* out;
  int64_t out_stride;
  int64_t* rows;        // [T, B] row served per id (-1: default), or nullptr
  int tmaj;             // visit slots table by table (s = t * B + b), not in output order
  int rrec;             // rows record-major: rows[b * T + t] (DR_LOOKUP_ROWS_RECORD)
};

// Row of `key` when present with this column initialised, else -1.
__device__ __forceinline__ int64_t ev_probe_row(const LkDesc& e, uint64_t key) {
  uint64_t rc;
  typedef unsigned long long slot_v __attribute__((ext_vector_type(2)));
  if (key == kEmptyKey) {
    const slot_v sv = gld(reinterpret_cast<const slot_v*>(e.slots + e.cap));
    if (sv.x != 0ull) return -1;
    rc = sv.y;
  } else {
    const uint64_t mask = (uint64_t)e.cap - 1;
    const uint64_t h0 = mix64(key) & mask;
    for (int64_t probes = 0;; ++probes) {
      if (probes > e.cap) return -1;
      const slot_v sv =
          gld(reinterpret_cast<const slot_v*>(e.slots + probe_slot(h0, (uint64_t)probes, mask)));
      if (sv.x == key) {
        rc = sv.y;
        break;
      }
      if (sv.x == kEmptyKey) return -1;  // (a stale empty only sends it to the miss path)
    }
  }
  if (rc == kUnset || !(rc & e.colbit)) return -1;
  const int64_t row = (int64_t)(rc & kRowMask);
  return row == (int64_t)kRowDead ? -1 : row;
}

// WIDEN: bf16 rows (a bf16 EV) widened into an fp32 output -- `dim` counts
// values, rows are dim / 2 float words apart.  (A bf16 output is the plain
// kernel on float words.)
template <int VEC, int G, int CPL, int ORDER, int NB, bool WIDEN = false>
__global__ __launch_bounds__(256) void ev_lookup_onehot_kernel(LookupArgs a, int T, int64_t B,
                                                               int dim, int32_t* __restrict__ mlist,
                                                               unsigned long long* __restrict__ mcnt) {
  __shared__ LkDesc sd[DR_MAX_GROUP];  // per-lane table index: stage in LDS
  constexpr int GPB = 256 / G;
  const int64_t slots = (int64_t)T * B;
  const int64_t s0 = ((int64_t)blockIdx.x * GPB + threadIdx.x / G) * NB;
  const int lg = threadIdx.x % G;
  // The probing lanes' ids are loaded BEFORE the descriptor staging and its
  // barrier: the id's memory round trip overlaps them (the ids are read
  // once: nontemporal).
  const bool prober = lg < NB && s0 + lg < slots;
  int64_t pb = 0;
  int pt = 0;
  uint64_t pkey = 0;
  if (prober) {
    const int64_t s = s0 + lg;
    if (a.tmaj) {   // slots < 2^31 (host check)
      pt = (int)((uint32_t)s / (uint32_t)B);
      pb = s - (int64_t)pt * B;
    } else {
      pb = (int64_t)((uint32_t)s / (uint32_t)T);
      pt = (int)(s - pb * T);
    }
    pkey = (uint64_t)__builtin_nontemporal_load(gp(a.keys + pb * a.ksb + (int64_t)pt * a.kst));
  }
  if (threadIdx.x < T) sd[threadIdx.x] = a.d[threadIdx.x];
  __syncthreads();
  if (s0 >= slots) return;
  const int dv = dim / VEC;
  const int base = (int)(threadIdx.x % 64) - lg;
  // lanes 0..NB-1 of the group probe one slot each
  const float* mine = nullptr;
  bool missed = false;
  if (prober) {
    const int64_t b = pb;
    const int t = pt;
    const LkDesc& e = sd[t];
    const int64_t row = ev_probe_row(e, pkey);
    if (row >= 0) {
      mine = e.pool + row * (int64_t)(WIDEN ? dim / 2 : dim);
      if (a.rows) a.rows[a.rrec ? b * T + t : (int64_t)t * B + b] = row;
    } else {
      missed = true;
    }
  }
  // wave-aggregated append of the misses
  const uint64_t mm = __ballot(missed);
  if (mm) {
    const int lane = (int)(threadIdx.x % 64);
    const int leader = __ffsll((unsigned long long)mm) - 1;
    unsigned long long at = 0;
    if (lane == leader) at = atomicAdd(mcnt, (unsigned long long)__popcll(mm));
    at = __shfl(at, leader, 64);
    // (the miss list holds output-order slots b * T + t in either visiting order)
    if (missed) mlist[at + __popcll(mm & lanemask_lt())] = (int32_t)(pb * T + pt);
  }
  // every row address first (the shuffles' LDS waits then precede the row
  // loads), then the NB row loads back to back as global (not flat) loads
  const float* p[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const uint64_t u = (uint64_t)(uintptr_t)mine;
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)u, base + q, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(u >> 32), base + q, 64);
    p[q] = reinterpret_cast<const float*>((uintptr_t)(((uint64_t)hi << 32) | lo));
  }
  Row<VEC, G, CPL> x[NB];
  float* o[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int64_t s = s0 + q;
    o[q] = nullptr;
    if (p[q] && s < slots) {
      int64_t b, t;
      if (a.tmaj) {
        t = (int64_t)((uint32_t)s / (uint32_t)B);
        b = s - t * B;
      } else {
        b = (int64_t)((uint32_t)s / (uint32_t)T);
        t = s - b * T;
      }
      o[q] = a.out + b * a.out_stride + t * (int64_t)dim;
    }
    load_row_copy<VEC, G, CPL, WIDEN>(x[q], p[q], lg, dv);
  }
  wait_loads();
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if (ORDER == DR_ORDER_SEQ) {  // fused op: out = 0 + e (-0.0 -> +0.0)
#pragma unroll
      for (int c = 0; c < CPL; ++c) x[q].v[c] = vadd(vzero<typename VecT<VEC>::T>(), x[q].v[c]);
    }
    if (o[q]) store_row_nt<VEC, G, CPL>(x[q], o[q], lg, dv);
  }
}

// ---------------------------------------------------------------------------
// Line-wide probes (bucket-local probing, probe_slot): the 8 lanes that share
// a key load the 8 slots of its home line in one instruction (one 128-B
// request), and two ballots settle the lookup -- no dependent second probe
// for the keys displaced from their home slot (a quarter of them at the
// bench's load), which the slot-by-slot walk paid as an extra L2 round trip
// in most waves.
// ---------------------------------------------------------------------------
typedef unsigned long long slot_v2 __attribute__((ext_vector_type(2)));

// Issue half: lane j (= lane % 8) of the key's 8 lanes loads slot j of the
// home line (key -1: its special slot, on all 8 lanes).  Branch-free: the
// address is a select, the load is unconditional.
__device__ __forceinline__ slot_v2 line_probe_issue(const Slot* slots, int64_t cap, uint64_t key,
                                                    int j) {
  const uint64_t line = (mix64(key) & (uint64_t)(cap - 1)) & ~7ull;
  const uint64_t at = key == kEmptyKey ? (uint64_t)cap : line + (uint64_t)j;
  return gld(reinterpret_cast<const slot_v2*>(slots + at));
}

// Resolve half: every lane of the wave calls it (ballots, shuffles).  Each
// group of 8 lanes gets its key's row, or -1 (absent, column not initialised,
// dead row: the miss path).  A key neither found nor ruled out in its home
// line (a full line, ~0.5 % at the bench's load) walks on from probe 8.
__device__ __forceinline__ int64_t line_probe_resolve(const Slot* slots, int64_t cap,
                                                      uint64_t colbit, uint64_t key, slot_v2 sv,
                                                      int lane) {
  const int j = lane & 7;
  const bool special = key == kEmptyKey;
  const uint64_t mask = (uint64_t)cap - 1;
  const uint64_t h0 = mix64(key) & mask;
  const int o = special ? 0 : (int)(h0 & 7);
  // key -1's slot holds 0 when present, -1 when absent; its 8 lanes loaded
  // the same slot, lane 0 speaks for them (selects, no branches)
  const bool speaks = !special || j == 0;
  const bool hit = speaks && sv.x == (special ? 0ull : key);
  const bool emp = speaks && sv.x == kEmptyKey;
  const uint64_t hm = __ballot(hit), em = __ballot(emp);
  const int sh = lane & ~7;
  const uint32_t h8 = (uint32_t)(hm >> sh) & 0xffu, e8 = (uint32_t)(em >> sh) & 0xffu;
  // bit i = probe i of the key (offset (o + i) % 8 of the line)
  const uint32_t rh = ((h8 >> o) | (h8 << (8 - o))) & 0xffu;
  const uint32_t re = ((e8 >> o) | (e8 << (8 - o))) & 0xffu;
  const uint32_t any = rh | re;
  const int f = any ? __builtin_ctz(any) : 0;
  const int src = sh + ((o + f) & 7);
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)sv.y, src, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(sv.y >> 32), src, 64);
  uint64_t rc = ((uint64_t)hi << 32) | lo;
  if (!((rh >> f) & 1u)) rc = kUnset;  // an empty slot comes first, or nothing settled
  if (!any) {  // the home line holds 8 other keys: continue the sequence
    for (uint64_t i = 8; i <= (uint64_t)cap; ++i) {
      const slot_v2 w = gld(reinterpret_cast<const slot_v2*>(slots + probe_slot(h0, i, mask)));
      if (w.x == key) {
        rc = w.y;
        break;
      }
      if (w.x == kEmptyKey) break;  // (a stale empty only sends it to the miss path)
    }
  }
  if (rc == kUnset || !(rc & colbit)) return -1;
  const int64_t row = (int64_t)(rc & kRowMask);
  return row == (int64_t)kRowDead ? -1 : row;
}

// One-hot row load / store with no branch around the memory operation: the
// address is always valid (lanes past the row read its last chunk, rows that
// are not stored read row 0), the store target a select (rows that must not
// be written go to a junk line of the workspace).  A branch around a load
// makes hipcc wait for it right there; a branch around a store makes the
// counted waits of a software pipeline path-dependent (vmcnt(0)).
template <int VEC, int G, int CPL, bool WIDEN>
__device__ __forceinline__ void load_row_copy_u(Row<VEC, G, CPL>& x, const float* p, int lg,
                                                int dv) {
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    int col = lg + c * G;
    col = col < dv ? col : dv - 1;
    if constexpr (WIDEN) {
      typedef unsigned int u2 __attribute__((ext_vector_type(2)));
      const u2 w = __builtin_nontemporal_load(gp(reinterpret_cast<const u2*>(p) + col));
      const float2 a = bf16x2_to_f2(w.x), b = bf16x2_to_f2(w.y);
      x.v[c] = make_float4(a.x, a.y, b.x, b.y);
    } else {
      x.v[c] = nt_load(reinterpret_cast<const typename VecT<VEC>::T*>(p) + col);
    }
  }
}

template <int VEC, int G, int CPL, int ORDER>
__device__ __forceinline__ void store_row_sel(Row<VEC, G, CPL>& x, float* p, float* junk, int lg,
                                              int dv) {
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int col = lg + c * G;
    if (ORDER == DR_ORDER_SEQ) x.v[c] = vadd(vzero<typename VecT<VEC>::T>(), x.v[c]);  // 0 + e
    float* dst = col < dv ? p + (int64_t)col * VEC : junk + 2048 + (int64_t)(lg % 64) * VEC;
    nt_store(x.v[c], reinterpret_cast<typename VecT<VEC>::T*>(dst));
  }
}

// Output-order lookup with line-wide probes: a wave owns 8 consecutive
// output slots (key k of the wave on lanes 8k..8k+7); each group of G = 8 NB
// lanes then copies NB of the 8 rows (row q of group g = the key on lane
// g G + 8 q).  One-shot: key -> line -> rows -> stores per wave.
template <int VEC, int G, int CPL, int ORDER, bool WIDEN = false>
__global__ __launch_bounds__(256) void ev_lookup_line_kernel(LookupArgs a, int T, int64_t B,
                                                             int dim, int32_t* __restrict__ mlist,
                                                             unsigned long long* __restrict__ mcnt,
                                                             float* __restrict__ junk) {
  constexpr int NB = G / 8;
  static_assert(NB * 8 == G, "8 lanes per key, 8 keys per wave");
  __shared__ LkDesc sd[DR_MAX_GROUP];
  const int64_t slots = (int64_t)T * B;
  const int lane = (int)(threadIdx.x & 63);
  const int64_t ws0 = ((int64_t)blockIdx.x * 4 + threadIdx.x / 64) * 8;  // wave's first slot
  const int64_t s = ws0 + (lane >> 3);
  const bool valid = s < slots;
  const int64_t sc = valid ? s : slots - 1;
  const int64_t b = (int64_t)((uint32_t)sc / (uint32_t)T);
  const int t = (int)(sc - b * T);
  // the id's round trip overlaps the descriptor staging (ids read once)
  const uint64_t key =
      (uint64_t)__builtin_nontemporal_load(gp(a.keys + b * a.ksb + (int64_t)t * a.kst));
  if (threadIdx.x < T) sd[threadIdx.x] = a.d[threadIdx.x];
  __syncthreads();
  if (ws0 >= slots) return;  // whole waves
  const Slot* tsl = sd[t].slots;
  const int64_t tcap = sd[t].cap;
  const int64_t row = line_probe_resolve(tsl, tcap, sd[t].colbit, key,
                                         line_probe_issue(tsl, tcap, key, lane & 7), lane);
  const bool head = (lane & 7) == 0 && valid;
  const bool missed = head && row < 0;
  if (head && row >= 0 && a.rows) a.rows[a.rrec ? s : (int64_t)t * B + b] = row;
  const uint64_t mm = __ballot(missed);
  if (mm) {
    const int leader = __ffsll((unsigned long long)mm) - 1;
    unsigned long long at = 0;
    if (lane == leader) at = atomicAdd(mcnt, (unsigned long long)__popcll(mm));
    at = __shfl(at, leader, 64);
    if (missed) mlist[at + __popcll(mm & lanemask_lt())] = (int32_t)s;
  }
  const int64_t rstride = WIDEN ? dim / 2 : dim;
  const uint64_t mine = (uint64_t)(uintptr_t)(sd[t].pool + (row >= 0 ? row : 0) * rstride);
  const uint64_t okm = __ballot(valid && row >= 0);
  const int lg = lane % G, base = lane - lg;
  const int dv = dim / VEC;
  const float* p[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)mine, base + 8 * q, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(mine >> 32), base + 8 * q, 64);
    p[q] = reinterpret_cast<const float*>((uintptr_t)(((uint64_t)hi << 32) | lo));
  }
  Row<VEC, G, CPL> x[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) load_row_copy_u<VEC, G, CPL, WIDEN>(x[q], p[q], lg, dv);
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int64_t sq = ws0 + (base / G) * NB + q;
    const int64_t bq = (int64_t)((uint32_t)sq / (uint32_t)T);
    const int64_t tq = sq - bq * T;
    float* dst = ((okm >> (base + 8 * q)) & 1ull) ? a.out + bq * a.out_stride + tq * (int64_t)dim
                                                  : junk + q * 256;
    store_row_sel<VEC, G, CPL, ORDER>(x[q], dst, junk, lg, dv);
  }
}

// Software-pipelined persistent form of the same lookup: each wave walks its
// items (8 output slots each) with the keys of item k+2 and the home-line
// probes of item k+1 in flight while the rows of item k load and the rows of
// item k-1 are stored -- the probe's dependent round trip leaves the row
// stream's critical path.  Issue order per iteration: rows(k), probes(k+1),
// keys(k+2), then the NB stores of k-1; every one of them unconditional, so
// the wait at the loop top for probes(k+1) is vmcnt(1 + NB stores) on every
// path and never waits for the stores just issued.  XCD-major item ranges
// (blocks b, b + 8, ... run on one XCD: speed only, any placement is correct).
template <int VEC, int G, int CPL, int ORDER, bool WIDEN = false>
__global__ __launch_bounds__(256) void ev_lookup_pipe_kernel(LookupArgs a, int T, int64_t B,
                                                             int dim, int32_t* __restrict__ mlist,
                                                             unsigned long long* __restrict__ mcnt,
                                                             float* __restrict__ junk) {
  constexpr int NB = G / 8;
  static_assert(NB * 8 == G, "8 lanes per key, 8 keys per wave");
  __shared__ LkDesc sd[DR_MAX_GROUP];
  if (threadIdx.x < T) sd[threadIdx.x] = a.d[threadIdx.x];
  __syncthreads();
  const uint32_t slots = (uint32_t)((int64_t)T * B);  // < 2^31 (host check)
  const uint32_t items = (slots + 7) / 8;
  const int lane = (int)(threadIdx.x & 63);
  const int kq = lane >> 3, j = lane & 7;
  const int lg = lane % G, base = lane - lg;
  const int dv = dim / VEC;
  const int64_t rstride = WIDEN ? dim / 2 : dim;
  const uint32_t LW = (gridDim.x / 8) * 4;  // waves per XCD (grid % 8 == 0)
  const uint32_t per = (items + 7) / 8;
  const uint32_t i0 = (blockIdx.x % 8) * per;
  const uint32_t i1 = i0 + per < items ? i0 + per : items;
  uint32_t it = i0 + (blockIdx.x / 8) * 4 + threadIdx.x / 64;
  if (it >= i1) return;  // whole waves
  const uint32_t T32 = (uint32_t)T;
  // slot of this lane's key in item `item` (clamped: reads past the range
  // are harmless and keep the loop free of branches)
  auto slot_of = [&](uint32_t item) -> uint32_t {
    const uint32_t s = item * 8 + kq;
    return s < slots ? s : slots - 1;
  };
  auto key_at = [&](uint32_t s) -> uint64_t {
    const uint32_t b = s / T32, t = s - b * T32;
    return (uint64_t)__builtin_nontemporal_load(
        gp(a.keys + (int64_t)b * a.ksb + (int64_t)t * a.kst));
  };
  uint32_t sA = slot_of(it);
  uint64_t kA = key_at(sA);
  uint32_t tA = sA % T32;
  slot_v2 svA = line_probe_issue(sd[tA].slots, sd[tA].cap, kA, j);
  uint32_t sB = slot_of(it + LW);
  uint64_t kB = key_at(sB);
  // rows in flight / being stored ping-pong between X0 and X1 (the loop is
  // unrolled twice: no register copy of a pending load)
  Row<VEC, G, CPL> X0[NB], X1[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q)
#pragma unroll
    for (int c = 0; c < CPL; ++c) X1[q].v[c] = vzero<typename VecT<VEC>::T>();
  uint64_t okp = 0;  // which rows of the previous item to store (bit = key lane)
  uint32_t itp = it;
  auto store_item = [&](Row<VEC, G, CPL>(&xs)[NB]) {
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const uint32_t sq = itp * 8 + (uint32_t)((base / G) * NB + q);
      const uint32_t bq = sq / T32, tq = sq - bq * T32;
      float* dst = ((okp >> (base + 8 * q)) & 1ull)
                       ? a.out + (int64_t)bq * a.out_stride + (int64_t)tq * dim
                       : junk + q * 256;  // distinct lines: no store merged away
      store_row_sel<VEC, G, CPL, ORDER>(xs[q], dst, junk, lg, dv);
    }
  };
  // the loop's shape on entry too: NB (junk) stores after the first probes
  store_item(X1);
  // one item: settle its probes, issue its rows into xl, the probes of the
  // next item and the keys of the one after, then store xs (previous item)
  auto step = [&](Row<VEC, G, CPL>(&xl)[NB], Row<VEC, G, CPL>(&xs)[NB]) {
    const int64_t row = line_probe_resolve(sd[tA].slots, sd[tA].cap, sd[tA].colbit, kA, svA, lane);
    const uint32_t s = it * 8 + kq;
    const bool valid = s < slots;
    const bool head = j == 0 && valid;
    const bool missed = head && row < 0;
    if (a.rows && head && row >= 0) a.rows[a.rrec ? (int64_t)s : (int64_t)tA * B + s / T32] = row;
    const uint64_t mm = __ballot(missed);
    if (mm) {
      const int leader = __ffsll((unsigned long long)mm) - 1;
      unsigned long long at = 0;
      if (lane == leader) at = atomicAdd(mcnt, (unsigned long long)__popcll(mm));
      at = __shfl(at, leader, 64);
      if (missed) mlist[at + __popcll(mm & lanemask_lt())] = (int32_t)s;
    }
    const uint64_t mine = (uint64_t)(uintptr_t)(sd[tA].pool + (row >= 0 ? row : 0) * rstride);
    const uint64_t okc = __ballot(valid && row >= 0);
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)mine, base + 8 * q, 64);
      const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(mine >> 32), base + 8 * q, 64);
      load_row_copy_u<VEC, G, CPL, WIDEN>(
          xl[q], reinterpret_cast<const float*>((uintptr_t)(((uint64_t)hi << 32) | lo)), lg, dv);
    }
    kA = kB;
    tA = sB % T32;
    svA = line_probe_issue(sd[tA].slots, sd[tA].cap, kA, j);
    sB = slot_of(it + 2 * LW);
    kB = key_at(sB);
    store_item(xs);
    okp = okc;
    itp = it;
    it += LW;
  };
  for (;;) {
    step(X0, X1);
    if (it >= i1) {
      store_item(X0);
      break;
    }
    step(X1, X0);
    if (it >= i1) {
      store_item(X1);
      break;
    }
  }
}

struct MissArgs {
  EvDesc e[DR_MAX_GROUP];
  float* pool[DR_MAX_GROUP];
  const float* dflt[DR_MAX_GROUP];
  int64_t* mtop[DR_MAX_GROUP];  // row counters to mirror (nullptr: none)
  int64_t* mdst[DR_MAX_GROUP];
  const int64_t* keys;
  int64_t ksb, kst;
  float* out;
  int64_t out_stride;
  int64_t* rows;
  int rrec;
};

// Grid-wide barrier of the miss kernel.  The grid is small enough to be
// co-resident (kMissBlocks, ~2 blocks per CU), the spin is bounded (latches
// INTERNAL instead of hanging), and the agent-scope fences write back /
// invalidate the XCD-local L2s around it.
__device__ __forceinline__ void miss_grid_sync(unsigned* bar, unsigned target, int* st) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    atomicAdd(bar, 1u);
    for (unsigned spin = 0;
         __hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target; ++spin) {
      if (spin > (1u << 24)) {
        latch(st, DR_INTERNAL);
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
    __threadfence();
  }
  __syncthreads();
}

// The listed slots, in three grid-synchronised phases (what resolve -> init
// -> copy do in three launches): (1) insert-on-miss resolve, creator-first
// (ev_find), claiming each row's first touch of the column; (2) default rows
// for the claims, one wave per row, and block 0 refreshes the capacity
// mirrors (the counter is final); (3) copy each slot's row (or the default
// when allocation failed) into the output.  Steady state: the list is empty
// and every block returns after one load.
template <int ORDER>
__global__ __launch_bounds__(256) void ev_miss_kernel(MissArgs a, int T, int64_t B, int64_t dim,
                                                      int widen,
                                                      const int32_t* __restrict__ mlist,
                                                      const unsigned long long* __restrict__ mcnt,
                                                      unsigned* __restrict__ bar,
                                                      int64_t* __restrict__ mrow,
                                                      uint8_t* __restrict__ minit, int* st) {
  const int64_t n = (int64_t)*mcnt;
  if (n == 0) return;  // uniform over the grid
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthreads) {
    const int64_t s = mlist[i];
    const int64_t b = s / T;
    const int t = (int)(s - b * T);
    const EvDesc& e = a.e[t];
    bool created;
    uint64_t rc;
    Slot* sl = ev_find(e, (uint64_t)a.keys[b * a.ksb + (int64_t)t * a.kst], true, &created, &rc,
                       st);
    uint8_t claim = 0;
    int64_t row = -1;
    if (sl && (rc & kRowMask) != kRowDead) {
      row = (int64_t)(rc & kRowMask);
      const uint64_t bit = 1ull << (48 + e.col);
      if (!(rc & bit)) {
        const uint64_t old = atomicOr((unsigned long long*)&sl->rc, (unsigned long long)bit);
        if (!(old & bit)) claim = 1;
      }
    }
    mrow[i] = row;
    minit[i] = claim;
  }
  miss_grid_sync(bar, gridDim.x, st);
  if (blockIdx.x == 0 && threadIdx.x < T && a.mdst[threadIdx.x]) {
    const int64_t top = __hip_atomic_load(a.mtop[threadIdx.x], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.mdst[threadIdx.x], top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / 64);
  const int64_t w0 = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  for (int64_t i = w0; i < n; i += waves) {
    if (!minit[i]) continue;
    const int t = (int)(mlist[i] % T);
    float* dst = a.pool[t] + mrow[i] * dim;
    for (int64_t c = lane; c < dim; c += 64) dst[c] = a.dflt[t][c];
  }
  miss_grid_sync(bar, 2 * gridDim.x, st);
  for (int64_t i = w0; i < n; i += waves) {
    const int64_t s = mlist[i];
    const int64_t b = s / T;
    const int t = (int)(s - b * T);
    const float* src = mrow[i] >= 0 ? a.pool[t] + mrow[i] * dim : a.dflt[t];
    if (a.rows && lane == 0)
      a.rows[a.rrec ? b * T + t : (int64_t)t * B + b] = mrow[i] >= 0 ? mrow[i] : -1;
    if (widen) {  // bf16 row (dim float words) -> 2 * dim fp32 values
      const uint16_t* h = reinterpret_cast<const uint16_t*>(src);
      float* dst = a.out + b * a.out_stride + (int64_t)t * 2 * dim;
      for (int64_t c = lane; c < 2 * dim; c += 64) dst[c] = bf16_to_f32(h[c]);
      continue;
    }
    float* dst = a.out + b * a.out_stride + (int64_t)t * dim;
    for (int64_t c = lane; c < dim; c += 64) dst[c] = ORDER == DR_ORDER_SEQ ? 0.f + src[c] : src[c];
  }
}

// 2 blocks per CU of the current device: co-resident by construction
static unsigned miss_blocks() {
  static std::atomic<int> cached[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 64;
  int cus = cached[dev].load(std::memory_order_relaxed);
  if (cus <= 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 32;
    cached[dev].store(cus, std::memory_order_relaxed);
  }
  return (unsigned)(2 * cus);
}

struct LookupWs {
  float* junk;  // 16 KB sink of the branch-free stores (line / pipe kernels)
  int32_t* mlist;
  unsigned long long* mcnt;  // [2]: miss count, grid-barrier counter
  int64_t* mrow;
  uint8_t* minit;
};
static LookupWs carve_lookup(void* ws, int64_t n, size_t* used) {
  Carver c(ws);
  LookupWs w;
  const int64_t nn = n > 0 ? n : 1;
  w.junk = c.take<float>(4096);
  w.mlist = c.take<int32_t>(nn);
  w.mcnt = c.take<unsigned long long>(2);
  w.mrow = c.take<int64_t>(nn);
  w.minit = c.take<uint8_t>(nn);
  if (used) *used = c.used + 256;
  return w;
}

template <int VEC, int G, int CPL, int ORDER, int NB, bool WIDEN = false>
static void launch_lookup_nb(const LookupArgs& a, int T, int64_t B, int dim, const LookupWs& w,
                             hipStream_t st) {
  const int64_t items = ceil_div((int64_t)T * B, NB);
  timing_mark(DR_TIME_LOOKUP, st, true);
  hipLaunchKernelGGL((ev_lookup_onehot_kernel<VEC, G, CPL, ORDER, NB, WIDEN>),
                     dim3((unsigned)ceil_div(items, 256 / G)), dim3(256), 0, st, a, T, B, dim,
                     w.mlist, w.mcnt);
  timing_mark(DR_TIME_LOOKUP, st, false);
}

// DR_LOOKUP_KERNEL (A/B switch): 0 = slot-by-slot one-shot kernel (NB rows
// per lane group), 1 = line probes, one-shot (ev_lookup_line_kernel), 2 =
// line probes, software-pipelined persistent waves (ev_lookup_pipe_kernel).
static int lookup_kernel_kind() {   // read per launch (host only): tests cover each kernel
  const char* e = getenv("DR_LOOKUP_KERNEL");
  return e ? atoi(e) : 1;
}

// Persistent grid of a 256-thread kernel: resident blocks per CU x CUs,
// a multiple of 8 (XCD-major item ranges), at most `want`.
template <class K>
static unsigned persistent_grid(K kernel, int64_t want) {
  // resident blocks of this kernel on this device, asked once
  static std::mutex mu;
  static std::vector<std::pair<std::pair<const void*, int>, int64_t>> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  const void* key = reinterpret_cast<const void*>(kernel);
  int64_t g = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    for (auto& e : cache)
      if (e.first.first == key && e.first.second == dev) g = e.second;
  }
  if (g == 0) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 256, 0) != hipSuccess ||
        per <= 0)
      per = 1;
    g = (int64_t)per * cus;
    std::lock_guard<std::mutex> lk(mu);
    cache.push_back({{key, dev}, g});
  }
  want = ceil_div(want, 8) * 8;
  if (g > want) g = want;
  g = std::max<int64_t>(8, g / 8 * 8);
  return (unsigned)g;
}

// Line-probe lookups (8 lanes per key: G = 8 NB); false when the shape or
// the switch leaves it to the slot-by-slot kernel.
template <int VEC, int G, int CPL, int ORDER, bool WIDEN>
static bool launch_lookup_line(const LookupArgs& a, int T, int64_t B, int dim, const LookupWs& w,
                               hipStream_t st) {
  if constexpr (G % 8 != 0) {
    return false;
  } else {
    const int kind = lookup_kernel_kind();
    if (kind == 0 || a.tmaj) return false;
    const int64_t waves = ceil_div((int64_t)T * B, 8);
    timing_mark(DR_TIME_LOOKUP, st, true);
    if (kind == 1) {
      hipLaunchKernelGGL((ev_lookup_line_kernel<VEC, G, CPL, ORDER, WIDEN>),
                         dim3((unsigned)ceil_div(waves, 4)), dim3(256), 0, st, a, T, B, dim,
                         w.mlist, w.mcnt, w.junk);
    } else {
      const unsigned grid =
          persistent_grid(ev_lookup_pipe_kernel<VEC, G, CPL, ORDER, WIDEN>, ceil_div(waves, 4));
      hipLaunchKernelGGL((ev_lookup_pipe_kernel<VEC, G, CPL, ORDER, WIDEN>), dim3(grid), dim3(256),
                         0, st, a, T, B, dim, w.mlist, w.mcnt, w.junk);
    }
    timing_mark(DR_TIME_LOOKUP, st, false);
    return true;
  }
}

template <int VEC, int G, int CPL, int ORDER>
static void launch_lookup_onehot(const LookupArgs& a, int T, int64_t B, int dim, const LookupWs& w,
                                 hipStream_t st) {
  if (launch_lookup_line<VEC, G, CPL, ORDER, false>(a, T, B, dim, w, st)) return;
  // rows in flight per lane group: 2 for rows of <= 64 floats (D = 64:
  // 0.194 against 0.200 ms for 4, profiles/r04_lookup_ab_nb2.log -- more,
  // smaller groups hide the dependent slot probe better), 4 above (D = 128:
  // the step, not the kernel alone, is 0.7 % slower with 2)
  static const int nb_env = getenv("DR_LOOKUP_NB") ? atoi(getenv("DR_LOOKUP_NB")) : 0;
  const int nb = nb_env ? nb_env : (G <= 16 ? 2 : 4);
  if (nb == 8 && G >= 8)
    launch_lookup_nb<VEC, G, CPL, ORDER, 8>(a, T, B, dim, w, st);
  else if (nb == 2)
    launch_lookup_nb<VEC, G, CPL, ORDER, 2>(a, T, B, dim, w, st);
  else
    launch_lookup_nb<VEC, G, CPL, ORDER, 4>(a, T, B, dim, w, st);
}

static int lookup_onehot(dr_ev* const* evs, int T, const int64_t* keys, int64_t ksb, int64_t kst,
                         int64_t B, float* out, int64_t out_stride, int order, int64_t* rows_out,
                         void* ws, size_t ws_bytes, hipStream_t st, int flags = 0) {
  EvGuard guard_(evs, T);
  DR_REQUIRE(evs && T >= 1 && T <= DR_MAX_GROUP && B >= 0 && out_stride >= 0, DR_INVALID_ARGUMENT,
             "bad argument");
  DR_REQUIRE(ksb >= 0 && kst >= 0, DR_INVALID_ARGUMENT, "key strides must be >= 0");
  DR_REQUIRE(order == DR_ORDER_ALI || order == DR_ORDER_SEQ, DR_INVALID_ARGUMENT, "bad order");
  const int64_t n = (int64_t)T * B;
  DR_REQUIRE(n < (1ll << 31), DR_INVALID_ARGUMENT, "T*B must be < 2^31");
  size_t need = 0;
  carve_lookup(nullptr, n, &need);
  DR_REQUIRE(ws_bytes >= need, DR_INVALID_ARGUMENT, "lookup workspace too small");
  // bf16 EVs (value_bits 16): an fp32 output widens each value (the
  // reference casts bf16 embeddings to float32, embedding_ops.py:606-607);
  // with DR_LOOKUP_OUT_BF16 the rows are copied bitwise as D / 2 float words
  // into a bf16 output.  out_stride counts elements of the output type.
  DR_REQUIRE((flags & ~(DR_LOOKUP_OUT_BF16 | DR_LOOKUP_TABLE_ORDER | DR_LOOKUP_ROWS_RECORD)) == 0,
             DR_INVALID_ARGUMENT, "unknown flags 0x%x", flags);
  const bool bf16 = evs[0]->sh->bf16 && evs[0]->col == 0;
  const bool out_bf16 = flags & DR_LOOKUP_OUT_BF16;
  const bool widen = bf16 && !out_bf16;
  DR_REQUIRE(!out_bf16 || bf16, DR_INVALID_ARGUMENT, "DR_LOOKUP_OUT_BF16 needs bf16 EVs");
  DR_REQUIRE(!bf16 || order == DR_ORDER_ALI, DR_INVALID_ARGUMENT,
             "bf16 EV lookups pool in the ALI order");
  DR_REQUIRE(!out_bf16 || out_stride % 2 == 0, DR_INVALID_ARGUMENT,
             "bf16 output stride must be even");
  if (out_bf16) out_stride /= 2;                       // float words from here on
  // floats per output row segment (and per row, except when widening, where
  // a row is dim / 2 words)
  const int64_t dim = bf16 && !widen ? col_words(evs[0]->sh, 0) : evs[0]->sh->dim;
  DR_REQUIRE(dim % 4 == 0 && dim <= 256, DR_INVALID_ARGUMENT,
             "fused one-hot lookup needs dim %% 4 == 0 (bf16: %% 8) and <= 256 words");
  DR_REQUIRE(out_stride >= (int64_t)T * dim && (out_stride % 4) == 0 &&
                 ((uintptr_t)out & 15) == 0,
             DR_INVALID_ARGUMENT, "out must be 16-B aligned with stride >= T*dim (multiple of 4)");
  if (n == 0) return DR_OK;
  int* stw = status_word();
  DR_REQUIRE(stw, DR_INTERNAL, "status word unavailable");
  for (int t = 0; t < T; ++t) {
    const EvShared* s = evs[t]->sh;
    DR_REQUIRE(s->dim == evs[0]->sh->dim && (s->bf16 && evs[t]->col == 0) == bf16,
               DR_INVALID_ARGUMENT, "tables must share dim and value type");
    DR_REQUIRE(s->value_words == 1, DR_INVALID_ARGUMENT,
               "table %d: pooled lookups are fp32 / bf16 (double EVs: dr_ev_gather)", t);
    DR_REQUIRE(s->filter_freq == 0 && s->k_hash == 0, DR_INVALID_ARGUMENT,
               "table %d: the fused lookup is for filter-free EVs", t);
    DR_REQUIRE(((uintptr_t)s->pools[evs[t]->col] & 15) == 0, DR_INVALID_ARGUMENT,
               "pool alignment");
  }
  // capacity before any pointer is read (a reserve may grow the tables)
  for (int t = 0; t < T; ++t) {
    int rc = reserve(evs[t]->sh, B, st);
    if (rc) return rc;
  }
  LookupWs w = carve_lookup(ws, n, nullptr);
  int rc = fill_bytes(w.mcnt, 0, 2 * sizeof(unsigned long long), st);
  if (rc) return rc;
  LookupArgs la;
  memset(&la, 0, sizeof(la));
  MissArgs ma;
  memset(&ma, 0, sizeof(ma));
  for (int t = 0; t < T; ++t) {
    const EvShared* s = evs[t]->sh;
    la.d[t].slots = s->slots;
    la.d[t].cap = s->cap;
    la.d[t].pool = s->pools[evs[t]->col];
    la.d[t].colbit = 1ull << (48 + evs[t]->col);
    ma.e[t] = make_desc(evs[t]);
    ma.pool[t] = s->pools[evs[t]->col];
    ma.dflt[t] = s->defaults[evs[t]->col];
  }
  la.keys = ma.keys = keys;
  la.ksb = ma.ksb = ksb;
  la.kst = ma.kst = kst;
  la.rows = ma.rows = rows_out;
  la.out = ma.out = out;
  la.out_stride = ma.out_stride = out_stride;
  la.tmaj = (flags & DR_LOOKUP_TABLE_ORDER) ? 1 : 0;
  la.rrec = ma.rrec = (flags & DR_LOOKUP_ROWS_RECORD) ? 1 : 0;
  const int d4 = (int)(dim / 4);
#define DR_LK(G, C)                                                             \
  do {                                                                          \
    if (widen) {                                                                \
      if (!launch_lookup_line<4, G, C, DR_ORDER_ALI, true>(la, T, B, (int)dim, w, st)) \
        launch_lookup_nb<4, G, C, DR_ORDER_ALI, 4, true>(la, T, B, (int)dim, w, st); \
    }                                                                           \
    else if (order == DR_ORDER_ALI)                                             \
      launch_lookup_onehot<4, G, C, DR_ORDER_ALI>(la, T, B, (int)dim, w, st);   \
    else                                                                        \
      launch_lookup_onehot<4, G, C, DR_ORDER_SEQ>(la, T, B, (int)dim, w, st);   \
  } while (0)
  // DR_LOOKUP_SPLIT=2 (A/B switch): half the lanes per row, two float4 per
  // lane -- twice the rows (and probes) per wave in flight
  static const int split = getenv("DR_LOOKUP_SPLIT") ? atoi(getenv("DR_LOOKUP_SPLIT")) : 1;
  if (split == 2 && d4 > 8 && d4 <= 16) DR_LK(8, 2);
  else if (split == 2 && d4 > 16 && d4 <= 32) DR_LK(16, 2);
  else if (d4 <= 4) DR_LK(4, 1);
  else if (d4 <= 8) DR_LK(8, 1);
  else if (d4 <= 16) DR_LK(16, 1);
  else if (d4 <= 32) DR_LK(32, 1);
  else DR_LK(64, 1);
#undef DR_LK
  // capacity mirrors ride on the miss kernel (as on resolve_grouped's init)
  EvShared* mir[DR_MAX_GROUP];
  int nmir = 0;
  for (int t = 0; t < T; ++t) {
    EvShared* sh = evs[t]->sh;
    bool seen = false;
    for (int q = 0; q < nmir; ++q) seen = seen || mir[q] == sh;
    if (seen) continue;
    sh->mu.lock();
    if (want_mirror(sh, st)) {
      ma.mtop[t] = sh->top;
      ma.mdst[t] = sh->pinned_top;
      mir[nmir++] = sh;
    } else {
      sh->mu.unlock();
    }
  }
  unsigned* bar = reinterpret_cast<unsigned*>(w.mcnt + 1);
  const unsigned kMissBlocks = miss_blocks();
  if (order == DR_ORDER_ALI)
    hipLaunchKernelGGL(ev_miss_kernel<DR_ORDER_ALI>, dim3(kMissBlocks), dim3(256), 0, st, ma, T, B,
                       widen ? dim / 2 : dim, (int)widen, w.mlist, w.mcnt, bar, w.mrow, w.minit,
                       stw);
  else
    hipLaunchKernelGGL(ev_miss_kernel<DR_ORDER_SEQ>, dim3(kMissBlocks), dim3(256), 0, st, ma, T, B,
                       dim, 0, w.mlist, w.mcnt, bar, w.mrow, w.minit, stw);
  const hipError_t le = hipGetLastError();
  for (int q = 0; q < nmir; ++q) {
    if (le == hipSuccess) mirrored(mir[q], st);
    mir[q]->mu.unlock();
  }
  if (le != hipSuccess) {
    set_error("kernel launch failed: %s", hipGetErrorString(le));
    return DR_INTERNAL;
  }
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // namespace dr

// ===========================================================================
extern "C" {

int dr_ev_create(const dr_ev_config* cfg, const float* default_row_host, dr_ev** out) {
  using namespace dr;
  DR_REQUIRE(cfg && out && default_row_host, DR_INVALID_ARGUMENT, "null argument");
  DR_REQUIRE(cfg->dim > 0, DR_INVALID_ARGUMENT, "dim must be > 0");
  DR_REQUIRE(cfg->steps_to_live >= 0, DR_INVALID_ARGUMENT, "steps_to_live must >= 0");
  DR_REQUIRE(cfg->value_bits == 0 || cfg->value_bits == 16 || cfg->value_bits == 32 ||
                 cfg->value_bits == 64,
             DR_INVALID_ARGUMENT, "value_bits must be 16 (bf16), 32 (float) or 64 (double)");
  DR_REQUIRE(cfg->value_bits != 16 || cfg->dim % 2 == 0, DR_INVALID_ARGUMENT,
             "bf16 EVs need an even dim (rows are moved as float words)");
  EvShared* s = new (std::nothrow) EvShared();
  DR_REQUIRE(s, DR_RESOURCE_EXHAUSTED, "host allocation failed");
  (void)hipGetDevice(&s->device);
  s->value_words = cfg->value_bits == 64 ? 2 : 1;
  s->bf16 = cfg->value_bits == 16;
  s->dim = cfg->dim * s->value_words;
  s->filter_freq = cfg->filter_freq < 0 ? 0 : cfg->filter_freq;
  s->steps_to_live = cfg->steps_to_live;
  const int64_t capacity = cfg->capacity > 0 ? cfg->capacity : 1024;
  s->cap = next_pow2(std::max<int64_t>(1024, capacity * 2));
  s->row_cap = std::max<int64_t>(1024, capacity);
  int rc = DR_OK;
#define DR_TRY(x)                        \
  do {                                   \
    if ((x) != hipSuccess) {             \
      set_error("%s failed", #x);        \
      free_shared(s);                    \
      return DR_RESOURCE_EXHAUSTED;      \
    }                                    \
  } while (0)
  DR_TRY(hipMalloc(&s->slots, (size_t)(s->cap + 1) * sizeof(Slot)));
  DR_TRY(hipMemset(s->slots, 0xFF, (size_t)(s->cap + 1) * sizeof(Slot)));
  DR_TRY(hipMalloc(&s->top, sizeof(int64_t)));
  DR_TRY(hipMemset(s->top, 0, sizeof(int64_t)));
  if (s->filter_freq > 0) {
    DR_TRY(hipMalloc(&s->freq, (size_t)s->row_cap * sizeof(int64_t)));
    DR_TRY(hipMemset(s->freq, 0, (size_t)s->row_cap * sizeof(int64_t)));
  }
  if (s->steps_to_live != 0) {
    DR_TRY(hipMalloc(&s->version, (size_t)s->row_cap * sizeof(int64_t)));
    DR_TRY(hipMemset(s->version, 0, (size_t)s->row_cap * sizeof(int64_t)));
  }
  if (s->filter_freq > 0 && cfg->max_element_size != 0 && cfg->false_positive_probability != -1.0f) {
    bloom_params(cfg->max_element_size, cfg->false_positive_probability, &s->k_hash,
                 &s->num_counter);
    s->counter_bits = cfg->counter_bits ? cfg->counter_bits : 64;
    if (s->counter_bits != 8 && s->counter_bits != 16 && s->counter_bits != 32)
      s->counter_bits = 64;
    const size_t bytes = ((size_t)s->num_counter * (s->counter_bits / 8) + 7) & ~(size_t)7;
    DR_TRY(hipMalloc(&s->bloom, bytes));
    DR_TRY(hipMemset(s->bloom, 0, bytes));
    std::vector<uint64_t> seeds;
    bloom_seeds(s->k_hash, &seeds);
    DR_TRY(hipMalloc(&s->seeds, seeds.size() * sizeof(uint64_t) + 8));
    DR_TRY(hipMemcpy(s->seeds, seeds.data(), seeds.size() * sizeof(uint64_t),
                     hipMemcpyHostToDevice));
  }
  DR_TRY(hipEventCreateWithFlags(&s->copy_ev, hipEventDisableTiming));
  DR_TRY(hipEventCreateWithFlags(&s->update_ev, hipEventDisableTiming));
  DR_TRY(hipHostMalloc(&s->pinned_top, sizeof(int64_t)));
#undef DR_TRY
  rc = alloc_pool(s, 0, default_row_host);
  if (rc) {
    free_shared(s);
    return rc;
  }
  dr_ev* ev = new dr_ev();
  ev->sh = s;
  ev->col = 0;
  *out = ev;
  return DR_OK;
}

int dr_ev_create_slot(dr_ev* primary, int slot_index, const float* default_row_host, dr_ev** out) {
  using namespace dr;
  DR_REQUIRE(primary && out && default_row_host, DR_INVALID_ARGUMENT, "null argument");
  DR_REQUIRE(primary->col == 0, DR_INVALID_ARGUMENT, "slots attach to a primary EV");
  DR_REQUIRE(slot_index >= 1 && slot_index < kMaxCols, DR_INVALID_ARGUMENT,
             "slot_index must be in [1, %d)", kMaxCols);
  EvShared* s = primary->sh;
  std::lock_guard<std::mutex> g(s->mu);
  DR_REQUIRE(!s->pools[slot_index], DR_ALREADY_EXISTS, "slot %d already exists", slot_index);
  int rc = alloc_pool(s, slot_index, default_row_host);
  if (rc) return rc;
  s->refs.fetch_add(1);
  dr_ev* ev = new dr_ev();
  ev->sh = s;
  ev->col = slot_index;
  *out = ev;
  return DR_OK;
}

int dr_ev_retain(dr_ev* ev) {
  DR_REQUIRE(ev, DR_INVALID_ARGUMENT, "null ev");
  ev->refs.fetch_add(1);
  return DR_OK;
}

int dr_ev_release(dr_ev* ev) {
  DR_REQUIRE(ev, DR_INVALID_ARGUMENT, "null ev");
  if (ev->refs.fetch_sub(1) == 1) {
    dr::EvShared* s = ev->sh;
    if (s->refs.fetch_sub(1) == 1) dr::free_shared(s);
    delete ev;
  }
  return DR_OK;
}

int64_t dr_ev_dim(dr_ev* ev) { return ev ? ev->sh->dim / ev->sh->value_words : -1; }

int64_t dr_ev_row_capacity(dr_ev* ev) { return ev ? ev->sh->row_cap : -1; }

int64_t dr_ev_filter_freq(dr_ev* ev) { return ev ? ev->sh->filter_freq : -1; }

int dr_ev_value_bits(dr_ev* ev) {
  return ev ? (ev->sh->bf16 && ev->col == 0 ? 16 : 32 * ev->sh->value_words) : -1;
}

// MaybeLockEmbeddingVariableInputMutexesInOrder (training_ali_op_helpers.h:
// 85-118) for stream-ordered updates: the host mutexes are taken in address
// order, and the stream waits for the previous locked update of each EV.
int dr_ev_lock_updates(dr_ev* const* vars, int n, void* stream) {
  using namespace dr;
  DR_REQUIRE(vars && n >= 0, DR_INVALID_ARGUMENT, "bad argument");
  std::vector<EvShared*> v;
  for (int i = 0; i < n; ++i)
    if (vars[i]) v.push_back(vars[i]->sh);
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  for (EvShared* s : v) s->update_mu.lock();
  for (EvShared* s : v) {
    hipError_t e = hipStreamWaitEvent(S(stream), s->update_ev, 0);
    if (e != hipSuccess) {
      for (EvShared* u : v) u->update_mu.unlock();
      set_error("hipStreamWaitEvent: %s", hipGetErrorString(e));
      return DR_INTERNAL;
    }
  }
  return DR_OK;
}

int dr_ev_unlock_updates(dr_ev* const* vars, int n, void* stream) {
  using namespace dr;
  DR_REQUIRE(vars && n >= 0, DR_INVALID_ARGUMENT, "bad argument");
  std::vector<EvShared*> v;
  for (int i = 0; i < n; ++i)
    if (vars[i]) v.push_back(vars[i]->sh);
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  int rc = DR_OK;
  for (EvShared* s : v) {
    if (hipEventRecord(s->update_ev, S(stream)) != hipSuccess) rc = DR_INTERNAL;
    s->update_mu.unlock();
  }
  if (rc) set_error("dr_ev_unlock_updates: hipEventRecord failed");
  return rc;
}

const float* dr_ev_pool(dr_ev* ev) { return ev ? ev->sh->pools[ev->col] : nullptr; }

int dr_ev_size(dr_ev* ev, int64_t* size_host, void* stream) {
  dr::EvGuard guard_(ev);
  DR_REQUIRE(ev && size_host, DR_INVALID_ARGUMENT, "null argument");
  DR_HIP(hipStreamSynchronize(dr::S(stream)));
  DR_HIP(hipMemcpy(size_host, ev->sh->top, sizeof(int64_t), hipMemcpyDeviceToHost));
  *size_host -= ev->sh->removed;
  return DR_OK;
}

int dr_ev_shrink(dr_ev* ev, int64_t global_step, float l2_weight_threshold,
                 int64_t* removed_host, void* stream) {
  dr::EvGuard guard_(ev);
  using namespace dr;
  DR_REQUIRE(ev && ev->col == 0, DR_INVALID_ARGUMENT, "shrink needs a primary EV");
  EvShared* s = ev->sh;
  hipStream_t st = S(stream);
  const int mode = l2_weight_threshold != -1.0f ? 1 : (s->steps_to_live > 0 ? 2 : 0);
  if (removed_host) *removed_host = 0;
  if (mode == 0) return DR_OK;
  DR_REQUIRE(mode == 2 || s->value_words == 1, DR_INVALID_ARGUMENT,
             "l2-weight shrink is for float / bf16 EVs");
  std::lock_guard<std::mutex> g(s->mu);
  const int64_t n = s->cap + 1;
  uint8_t* keep = nullptr;
  unsigned long long* cnt = nullptr;
  Slot* ns = nullptr;
  DR_HIP(hipMalloc(&keep, (size_t)n));
  if (hipMalloc(&cnt, sizeof(unsigned long long)) != hipSuccess) {
    (void)hipFree(keep);
    DR_REQUIRE(false, DR_RESOURCE_EXHAUSTED, "shrink: out of device memory");
  }
  if (hipMalloc(&ns, (size_t)n * sizeof(Slot)) != hipSuccess) {
    (void)hipFree(keep);
    (void)hipFree(cnt);
    DR_REQUIRE(false, DR_RESOURCE_EXHAUSTED, "shrink: out of device memory");
  }
  int rc = fill_bytes(cnt, 0, sizeof(unsigned long long), st);
  if (!rc) rc = fill_bytes(ns, 0xFF, (size_t)n * sizeof(Slot), st);
  unsigned long long removed = 0;
  if (!rc) {
    const unsigned blocks = (unsigned)ceil_div(n, 256);
    hipLaunchKernelGGL(ev_shrink_mark_kernel, dim3(blocks), dim3(256), 0, st, s->slots, s->cap,
                       s->pools[0], s->defaults[0], s->dim, s->bf16, s->version, mode,
                       l2_weight_threshold, global_step, s->steps_to_live, keep, cnt);
    hipLaunchKernelGGL(ev_rehash_kept_kernel, dim3(blocks), dim3(256), 0, st, s->slots, s->cap,
                       keep, ns);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpy(&removed, cnt, sizeof(removed), hipMemcpyDeviceToHost) != hipSuccess)
      rc = DR_INTERNAL;
  }
  (void)hipFree(keep);
  (void)hipFree(cnt);
  if (rc) {
    (void)hipFree(ns);
    set_error("dr_ev_shrink failed");
    return rc;
  }
  (void)hipFree(s->slots);
  s->slots = ns;
  s->removed += (int64_t)removed;
  if (removed_host) *removed_host = (int64_t)removed;
  return DR_OK;
}

int dr_ev_reserve(dr_ev* ev, int64_t extra, void* stream) {
  dr::EvGuard guard_(ev);
  DR_REQUIRE(ev && extra >= 0, DR_INVALID_ARGUMENT, "bad argument");
  dr::EvShared* s = ev->sh;
  hipStream_t st = dr::S(stream);
  std::lock_guard<std::mutex> g(s->mu);
  if (s->adds.only(st))
    DR_HIP(hipStreamSynchronize(st));
  else
    DR_HIP(hipDeviceSynchronize());   // adds reserved on other streams must have run
  int64_t actual = 0;
  DR_HIP(hipMemcpy(&actual, s->top, sizeof(int64_t), hipMemcpyDeviceToHost));
  s->known = actual;
  s->adds_since_known = 0;
  s->adds = dr::EvShared::Streams();
  s->copy_pending = false;
  return dr::grow(s, actual + extra, st);
}

size_t dr_ev_resolve_workspace_size(int64_t n) {
  size_t used = 0;
  dr::carve_resolve(nullptr, n, &used);
  return used;
}

int dr_ev_resolve(dr_ev* ev, const int64_t* keys, int64_t n, const int64_t* n_dev,
                  const float* defaults, const int32_t* counts, int64_t* rows_out, void* ws,
                  size_t ws_bytes, void* stream) {
  DR_REQUIRE(ev && n >= 0, DR_INVALID_ARGUMENT, "bad argument");
  int64_t koff[2] = {0, n};
  const int64_t* nd[1] = {n_dev};
  const float* df[1] = {defaults};
  return dr::resolve_grouped(&ev, 1, keys, koff, nd, defaults ? df : nullptr, counts, rows_out, ws,
                             ws_bytes, dr::S(stream));
}

// Grouped resolve over T EVs (one per feature); keys/counts/rows_out are
// concatenated with table t at [koff_host[t], koff_host[t+1]).
int dr_ev_resolve_grouped(dr_ev* const* evs, int num_tables, const int64_t* keys,
                          const int64_t* koff_host, const int64_t* const* n_dev_per_table,
                          const int32_t* counts, int64_t* rows_out, void* ws, size_t ws_bytes,
                          void* stream) {
  return dr::resolve_grouped(evs, num_tables, keys, koff_host, n_dev_per_table, nullptr, counts,
                             rows_out, ws, ws_bytes, dr::S(stream));
}

// Fused one-hot forward lookup over T filter-free EVs (see lookup_onehot).
size_t dr_ev_lookup_onehot_workspace_size(int num_tables, int64_t batch) {
  size_t used = 0;
  dr::carve_lookup(nullptr, (int64_t)num_tables * batch, &used);
  return used;
}

int dr_ev_lookup_onehot(dr_ev* const* evs, int num_tables, const int64_t* keys, int64_t batch,
                        float* out, int64_t out_stride, int order, void* ws, size_t ws_bytes,
                        void* stream) {
  return dr::lookup_onehot(evs, num_tables, keys, 1, batch, batch, out, out_stride, order, nullptr,
                           ws, ws_bytes, dr::S(stream));
}

int dr_ev_lookup_onehot_strided(dr_ev* const* evs, int num_tables, const int64_t* keys,
                                int64_t key_stride_bag, int64_t key_stride_table, int64_t batch,
                                float* out, int64_t out_stride, int order, int64_t* rows_out,
                                void* ws, size_t ws_bytes, void* stream) {
  return dr::lookup_onehot(evs, num_tables, keys, key_stride_bag, key_stride_table, batch, out,
                           out_stride, order, rows_out, ws, ws_bytes, dr::S(stream));
}

int dr_ev_lookup_onehot_ex(dr_ev* const* evs, int num_tables, const int64_t* keys,
                           int64_t key_stride_bag, int64_t key_stride_table, int64_t batch,
                           void* out, int64_t out_stride, int order, int flags, int64_t* rows_out,
                           void* ws, size_t ws_bytes, void* stream) {
  return dr::lookup_onehot(evs, num_tables, keys, key_stride_bag, key_stride_table, batch,
                           static_cast<float*>(out), out_stride, order, rows_out, ws, ws_bytes,
                           dr::S(stream), flags);
}

int dr_ev_lookup_onehot_rows(dr_ev* const* evs, int num_tables, const int64_t* keys,
                             int64_t batch, float* out, int64_t out_stride, int order,
                             int64_t* rows_out, void* ws, size_t ws_bytes, void* stream) {
  if (!rows_out) {
    dr::set_error("rows_out is required");
    return DR_INVALID_ARGUMENT;
  }
  return dr::lookup_onehot(evs, num_tables, keys, 1, batch, batch, out, out_stride, order,
                           rows_out, ws, ws_bytes, dr::S(stream));
}

// Tagged resolve: keys of all T tables in one array, table of key i =
// tags[i] (n_dev: optional DEVICE count).  Filtered keys give -(i+1) and
// read table t's EV default.
int dr_ev_resolve_tagged(dr_ev* const* evs, int num_tables, const int64_t* keys,
                         const int32_t* tags, int64_t n, const int64_t* n_dev,
                         const int64_t* per_table_host, const int32_t* counts,
                         int64_t* rows_out, void* ws, size_t ws_bytes, void* stream) {
  dr::EvGuard guard_(evs, num_tables);
  DR_REQUIRE(num_tables >= 1 && num_tables <= DR_MAX_GROUP, DR_INVALID_ARGUMENT,
             "bad table count");
  int64_t koff[DR_MAX_GROUP + 1];
  for (int t = 0; t < num_tables; ++t) koff[t] = 0;
  koff[num_tables] = n;
  const int64_t* nd[1] = {n_dev};
  DR_REQUIRE(tags, DR_INVALID_ARGUMENT, "tags required");
  return dr::resolve_grouped(evs, num_tables, keys, koff, nd, nullptr, counts, rows_out, ws,
                             ws_bytes, dr::S(stream), tags, per_table_host);
}

// Owner-side pack for the row exchange: out[i] = resolved row of key i of
// table tags[i] (table default when filtered).
int dr_ev_gather_tagged(dr_ev* const* evs, int num_tables, const int32_t* tags,
                        const int64_t* rows, int64_t n, const int64_t* n_dev, float* out,
                        void* stream) {
  dr::EvGuard guard_(evs, num_tables);
  using namespace dr;
  DR_REQUIRE(num_tables >= 1 && num_tables <= DR_MAX_GROUP, DR_INVALID_ARGUMENT,
             "bad table count");
  if (n == 0) return DR_OK;
  PoolGroup pg;
  memset(&pg, 0, sizeof(pg));
  const int64_t dim = col_words(evs[0]->sh, evs[0]->col);  // float words (bf16: D / 2)
  for (int t = 0; t < num_tables; ++t) {
    DR_REQUIRE(col_words(evs[t]->sh, evs[t]->col) == dim && evs[t]->sh->value_words == 1 &&
                   evs[t]->sh->bf16 == evs[0]->sh->bf16,
               DR_INVALID_ARGUMENT, "tables must be float (or bf16) EVs sharing dim");
    pg.pool[t] = evs[t]->sh->pools[evs[t]->col];
    pg.dflt[t] = evs[t]->sh->defaults[evs[t]->col];
  }
  constexpr int G = 32;
  hipLaunchKernelGGL(ev_gather_tagged_kernel<G>, dim3((unsigned)ceil_div(n, 256 / G)),
                     dim3(256), 0, S(stream), pg, num_tables, dim, tags, rows, n, n_dev, out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

const float* dr_ev_default_row(dr_ev* ev) {
  return ev ? ev->sh->defaults[ev->col] : nullptr;
}

int dr_ev_gather(dr_ev* ev, const int64_t* keys, int64_t n, const float* defaults,
                 const int32_t* counts, float* out, void* ws, size_t ws_bytes, void* stream) {
  dr::EvGuard guard_(ev);
  using namespace dr;
  DR_REQUIRE(ev && n >= 0, DR_INVALID_ARGUMENT, "bad argument");
  if (n == 0) return DR_OK;
  Carver c(ws);
  int64_t* rows = c.take<int64_t>(n);
  size_t rneed = dr_ev_resolve_workspace_size(n);
  void* rws = c.take<char>(rneed);
  DR_REQUIRE(ws_bytes >= c.used, DR_INVALID_ARGUMENT, "workspace too small");
  int rc = dr_ev_resolve(ev, keys, n, nullptr, defaults, counts, rows, rws, rneed, stream);
  if (rc) return rc;
  return gather_ev_rows(ev->sh->pools[ev->col], col_words(ev->sh, ev->col), rows, n, defaults,
                        ev->sh->defaults[ev->col], out, S(stream));
}

size_t dr_ev_gather_workspace_size(int64_t n) {
  dr::Carver c(nullptr);
  c.take<int64_t>(n > 0 ? n : 1);
  c.take<char>(dr_ev_resolve_workspace_size(n));
  return c.used + 256;
}

int dr_ev_insert(dr_ev* ev, const int64_t* keys, int64_t n, const float* values,
                 const int64_t* versions, const int64_t* freqs, int64_t partition_id,
                 int64_t partition_num, void* stream) {
  dr::EvGuard guard_(ev);
  using namespace dr;
  DR_REQUIRE(ev && n >= 0, DR_INVALID_ARGUMENT, "bad argument");
  if (n == 0) return DR_OK;
  hipStream_t st = S(stream);
  int rc = reserve(ev->sh, n, st);
  if (rc) return rc;
  int64_t* rows = nullptr;
  uint8_t* init = nullptr;
  DR_HIP(hipMallocAsync((void**)&rows, n * sizeof(int64_t), st));
  DR_HIP(hipMallocAsync((void**)&init, n, st));
  EvDesc e = make_desc(ev);
  const unsigned blocks = (unsigned)ceil_div(n, 256);
  hipLaunchKernelGGL(ev_import_kernel, dim3(blocks), dim3(256), 0, st, e, keys, n, versions, freqs,
                     partition_id, partition_num, ev->sh->steps_to_live, rows, init,
                     status_word());
  InitGroup ig;
  memset(&ig, 0, sizeof(ig));
  ig.pool[0] = ev->sh->pools[ev->col];
  ig.src[0] = values;
  ig.dflt[0] = ev->sh->defaults[ev->col];
  ig.koff[0] = 0;
  ig.koff[1] = n;
  hipLaunchKernelGGL(ev_init_rows_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, ig, 1,
                     col_words(ev->sh, ev->col), rows, init);
  DR_LAUNCH_CHECK();
  DR_HIP(hipFreeAsync(rows, st));
  DR_HIP(hipFreeAsync(init, st));
  post_call(ev->sh, st);
  return DR_OK;
}

// Bulk insert of keys [key_begin, key_begin + n) with synthetic rows
// synth(seed, key, col) -- populates bench/test tables without a host copy.
int dr_ev_insert_synthetic(dr_ev* ev, int64_t key_begin, int64_t key_stride, int64_t n,
                           uint64_t seed, void* stream) {
  dr::EvGuard guard_(ev);
  using namespace dr;
  DR_REQUIRE(ev && n >= 0 && key_stride >= 1, DR_INVALID_ARGUMENT, "bad argument");
  if (n == 0) return DR_OK;
  hipStream_t st = S(stream);
  int rc = reserve(ev->sh, n, st);
  if (rc) return rc;
  const int64_t chunk = std::min<int64_t>(n, 1 << 24);
  int64_t* rows = nullptr;
  uint8_t* init = nullptr;
  DR_HIP(hipMallocAsync((void**)&rows, chunk * sizeof(int64_t), st));
  DR_HIP(hipMallocAsync((void**)&init, chunk, st));
  EvDesc e = make_desc(ev);
  for (int64_t b = 0; b < n; b += chunk) {
    const int64_t m = std::min(chunk, n - b);
    hipLaunchKernelGGL(ev_insert_range_kernel, dim3((unsigned)ceil_div(m, 256)), dim3(256), 0, st,
                       e, key_begin + b * key_stride, key_stride, m, rows, init, status_word());
    hipLaunchKernelGGL(ev_synth_rows_kernel, dim3((unsigned)ceil_div(m, 4)), dim3(256), 0, st,
                       ev->sh->pools[ev->col], ev->sh->dim, ev->sh->bf16 && ev->col == 0,
                       key_begin + b * key_stride,
                       key_stride, m, rows, init, seed);
    DR_LAUNCH_CHECK();
  }
  DR_HIP(hipFreeAsync(rows, st));
  DR_HIP(hipFreeAsync(init, st));
  post_call(ev->sh, st);
  return DR_OK;
}

// Export: keys whose own column and primary rows exist (GetSnapshot,
// embedding_var.h:221-243), ascending key order.
int dr_ev_export(dr_ev* ev, int64_t* keys_out, float* values_out, int64_t* versions_out,
                 int64_t* freqs_out, int64_t capacity, int64_t* m_host, void* stream) {
  dr::EvGuard guard_(ev);
  using namespace dr;
  DR_REQUIRE(ev && m_host, DR_INVALID_ARGUMENT, "null argument");
  hipStream_t st = S(stream);
  EvShared* s = ev->sh;
  DR_HIP(hipStreamSynchronize(st));
  std::vector<Slot> slots((size_t)s->cap + 1);
  DR_HIP(hipMemcpy(slots.data(), s->slots, slots.size() * sizeof(Slot), hipMemcpyDeviceToHost));
  const uint64_t need = (1ull << 48) | (1ull << (48 + ev->col));
  std::vector<std::pair<int64_t, int64_t>> kr;  // (key, row)
  for (size_t i = 0; i < slots.size(); ++i) {
    const Slot& x = slots[i];
    const bool occupied = (i < (size_t)s->cap) ? x.key != kEmptyKey : x.key == 0ull;
    if (!occupied || x.rc == kUnset || (x.rc & kRowMask) == kRowDead) continue;
    if ((x.rc & need) != need) continue;
    const int64_t key = i < (size_t)s->cap ? (int64_t)x.key : -1;
    kr.emplace_back(key, (int64_t)(x.rc & kRowMask));
  }
  std::sort(kr.begin(), kr.end());
  const int64_t m = (int64_t)kr.size();
  *m_host = m;
  if (!keys_out && !values_out && !versions_out && !freqs_out) return DR_OK;
  DR_REQUIRE(capacity >= m, DR_INVALID_ARGUMENT, "export capacity %lld < %lld",
             (long long)capacity, (long long)m);
  if (m == 0) return DR_OK;
  std::vector<int64_t> keys(m), rows(m), vers(m, 0), frqs(m, 0);
  for (int64_t i = 0; i < m; ++i) {
    keys[i] = kr[i].first;
    rows[i] = kr[i].second;
  }
  int64_t top = 0;
  DR_HIP(hipMemcpy(&top, s->top, sizeof(int64_t), hipMemcpyDeviceToHost));
  if ((versions_out && s->version) || (freqs_out && s->freq)) {
    std::vector<int64_t> hv(top > 0 ? top : 1), hf(top > 0 ? top : 1);
    if (s->version && top > 0)
      DR_HIP(hipMemcpy(hv.data(), s->version, top * sizeof(int64_t), hipMemcpyDeviceToHost));
    if (s->freq && top > 0)
      DR_HIP(hipMemcpy(hf.data(), s->freq, top * sizeof(int64_t), hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < m; ++i) {
      if (s->version) vers[i] = hv[rows[i]];
      if (s->freq) frqs[i] = hf[rows[i]];
    }
  }
  if (keys_out) DR_HIP(hipMemcpy(keys_out, keys.data(), m * sizeof(int64_t), hipMemcpyHostToDevice));
  if (versions_out)
    DR_HIP(hipMemcpy(versions_out, vers.data(), m * sizeof(int64_t), hipMemcpyHostToDevice));
  if (freqs_out) {
    if (s->k_hash > 0) {
      // Bloom: freq is the counters' minimum (GetFreq -> GetBloomFreq)
      const size_t bytes = ((size_t)s->num_counter * (s->counter_bits / 8) + 7) & ~(size_t)7;
      std::vector<uint8_t> hb(bytes);
      DR_HIP(hipMemcpy(hb.data(), s->bloom, bytes, hipMemcpyDeviceToHost));
      std::vector<uint64_t> seeds;
      bloom_seeds(s->k_hash, &seeds);
      for (int64_t i = 0; i < m; ++i) {
        uint64_t mn = 0;
        for (int64_t h = 0; h < s->k_hash; ++h) {
          uint64_t key = (uint64_t)keys[i];
          const uint64_t mm = 0x880355f21e6d1965ULL;
          uint64_t hh = seeds[h] ^ (8 * mm), v = key;
          v ^= v >> 23; v *= 0x2127599bf4325c37ULL; v ^= v >> 47; hh ^= v; hh *= mm;
          v = 0; v ^= v >> 23; v *= 0x2127599bf4325c37ULL; v ^= v >> 47; hh ^= v; hh *= mm;
          hh ^= hh >> 23; hh *= 0x2127599bf4325c37ULL; hh ^= hh >> 47;
          const int64_t c = (int64_t)(hh % (uint64_t)s->num_counter);
          uint64_t val = 0;
          switch (s->counter_bits) {
            case 8: val = hb[c]; break;
            case 16: val = ((uint16_t*)hb.data())[c]; break;
            case 32: val = ((uint32_t*)hb.data())[c]; break;
            default: val = ((uint64_t*)hb.data())[c]; break;
          }
          if (h == 0 || val < mn) mn = val;
        }
        frqs[i] = (int64_t)mn;
      }
    }
    DR_HIP(hipMemcpy(freqs_out, frqs.data(), m * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  if (values_out) {
    int64_t* drows = nullptr;
    DR_HIP(hipMalloc(&drows, m * sizeof(int64_t)));
    DR_HIP(hipMemcpy(drows, rows.data(), m * sizeof(int64_t), hipMemcpyHostToDevice));
    int rc = dr_gather(s->pools[ev->col], top, col_words(s, ev->col), drows, m, values_out, stream);
    (void)hipStreamSynchronize(st);
    (void)hipFree(drows);
    if (rc) return rc;
  }
  return DR_OK;
}

int dr_ev_key_meta(dr_ev* ev, const int64_t* keys_host, int64_t n, int64_t* freq_host,
                   int64_t* version_host, int32_t* has_row_host, void* stream) {
  dr::EvGuard guard_(ev);
  using namespace dr;
  DR_REQUIRE(ev && keys_host && n >= 0, DR_INVALID_ARGUMENT, "bad argument");
  if (n == 0) return DR_OK;
  hipStream_t st = S(stream);
  EvShared* s = ev->sh;
  int64_t *dk = nullptr, *dr_ = nullptr;
  uint64_t* drc = nullptr;
  DR_HIP(hipMalloc(&dk, n * sizeof(int64_t)));
  DR_HIP(hipMalloc(&dr_, n * sizeof(int64_t)));
  DR_HIP(hipMalloc(&drc, n * sizeof(uint64_t)));
  DR_HIP(hipMemcpy(dk, keys_host, n * sizeof(int64_t), hipMemcpyHostToDevice));
  EvDesc e = make_desc(ev);
  hipLaunchKernelGGL(ev_lookup_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, e, dk,
                     n, dr_, drc, status_word());
  DR_HIP(hipStreamSynchronize(st));
  std::vector<int64_t> rows(n);
  std::vector<uint64_t> rcs(n);
  DR_HIP(hipMemcpy(rows.data(), dr_, n * sizeof(int64_t), hipMemcpyDeviceToHost));
  DR_HIP(hipMemcpy(rcs.data(), drc, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
  (void)hipFree(dk);
  (void)hipFree(dr_);
  (void)hipFree(drc);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t r = rows[i];
    if (freq_host) {
      freq_host[i] = 0;
      if (r >= 0 && s->freq) DR_HIP(hipMemcpy(&freq_host[i], s->freq + r, 8, hipMemcpyDeviceToHost));
    }
    if (version_host) {
      version_host[i] = r >= 0 ? 0 : -1;
      if (r >= 0 && s->version)
        DR_HIP(hipMemcpy(&version_host[i], s->version + r, 8, hipMemcpyDeviceToHost));
    }
    if (has_row_host) has_row_host[i] = r >= 0 && ((rcs[i] >> (48 + ev->col)) & 1);
  }
  return DR_OK;
}

int dr_ev_apply_sgd(dr_ev* var, float lr, const float* grad, const int64_t* keys, int64_t n,
                    const int64_t* n_dev, int64_t global_step, void* stream) {
  dr::OptScalars sc = {lr, 0, 0, 0, 0, 0, 0, 0, 0};
  return dr::apply_common(dr::OPT_SGD, var, nullptr, nullptr, sc, grad, keys, n, n_dev,
                          global_step, dr::S(stream));
}

int dr_ev_apply_adagrad(dr_ev* var, dr_ev* accum, float lr, const float* grad,
                        const int64_t* keys, int64_t n, const int64_t* n_dev, int64_t global_step,
                        void* stream) {
  dr::OptScalars sc = {lr, 0, 0, 0, 0, 0, 0, 0, 0};
  return dr::apply_common(dr::OPT_ADAGRAD, var, accum, nullptr, sc, grad, keys, n, n_dev,
                          global_step, dr::S(stream));
}

int dr_ev_apply_grouped(int optimizer, dr_ev* const* vars, dr_ev* const* slot1,
                        dr_ev* const* slot2, int num_tables, const float* const* grads,
                        const int64_t* const* keys, const int64_t* n_host,
                        const int64_t* const* n_dev, float lr, float beta1_power,
                        float beta2_power, float beta1, float beta2, float epsilon,
                        int64_t global_step, void* stream) {
  using namespace dr;
  int opt;
  OptScalars sc;
  int rc = grouped_opt(optimizer, lr, beta1_power, beta2_power, beta1, beta2, epsilon, &opt, &sc);
  if (rc) return rc;
  return apply_grouped(opt, vars, slot1, slot2, num_tables, sc, grads, keys, n_host, n_dev,
                       global_step, S(stream));
}

int dr_ev_apply_adam_async_grouped(int rmsprop, int by_address, dr_ev* const* vars,
                                   dr_ev* const* m, dr_ev* const* v, int num_tables,
                                   const void* const* grads, const int64_t* const* keys,
                                   const int64_t* n_host, const int64_t* const* n_dev,
                                   float* const* powers, float lr, float beta1, float beta2,
                                   float epsilon, int64_t global_step, void* stream) {
  using namespace dr;
  DR_REQUIRE(grads && (rmsprop || powers), DR_INVALID_ARGUMENT,
             "bad argument (AdamAsync needs the device beta powers)");
  DR_REQUIRE(num_tables >= 1, DR_INVALID_ARGUMENT, "num_tables must be >= 1");
  if (!rmsprop)
    for (int t = 0; t < num_tables; ++t)
      DR_REQUIRE(powers[t] && ((uintptr_t)powers[t] & 3) == 0, DR_INVALID_ARGUMENT,
                 "table %d: powers must be a device float[2]", t);
  int opt;
  OptScalars sc;
  int rc = grouped_opt(rmsprop ? DR_OPT_ADAM_ASYNC_RMSPROP : DR_OPT_ADAM_ASYNC, lr, 0.f, 0.f,
                       beta1, beta2, epsilon, &opt, &sc);
  if (rc) return rc;
  return apply_grouped(opt, vars, m, v, num_tables, sc,
                       reinterpret_cast<const float* const*>(grads), keys, n_host, n_dev,
                       global_step, S(stream), by_address ? 1 : 0, nullptr,
                       rmsprop ? nullptr : powers);
}

int dr_ev_apply_adam_grouped_dev(int by_address, dr_ev* const* vars, dr_ev* const* m,
                                 dr_ev* const* v, int num_tables, const void* const* grads,
                                 const int64_t* const* keys, const int64_t* n_host,
                                 const int64_t* const* n_dev, const float* powers, float lr,
                                 float beta1, float beta2, float epsilon, int64_t global_step,
                                 void* stream) {
  using namespace dr;
  DR_REQUIRE(grads && powers && ((uintptr_t)powers & 3) == 0 && num_tables >= 1,
             DR_INVALID_ARGUMENT, "bad argument (powers: a device float[2])");
  DR_REQUIRE(num_tables <= 4096, DR_INVALID_ARGUMENT, "too many tables");
  int opt;
  OptScalars sc;
  int rc = grouped_opt(DR_OPT_ADAM, lr, 0.f, 0.f, beta1, beta2, epsilon, &opt, &sc);
  if (rc) return rc;
  float* pw[4096];
  for (int t = 0; t < num_tables; ++t) pw[t] = const_cast<float*>(powers);
  return apply_grouped(opt, vars, m, v, num_tables, sc,
                       reinterpret_cast<const float* const*>(grads), keys, n_host, n_dev,
                       global_step, S(stream), by_address ? 1 : 0, nullptr, pw, false);
}

int dr_ev_apply_grouped_ptr(int optimizer, dr_ev* const* vars, dr_ev* const* slot1,
                            dr_ev* const* slot2, int num_tables, const uint64_t* const* grad_ptrs,
                            const int64_t* const* keys, const int64_t* n_host,
                            const int64_t* const* n_dev, float lr, float beta1_power,
                            float beta2_power, float beta1, float beta2, float epsilon,
                            int64_t global_step, void* stream) {
  using namespace dr;
  DR_REQUIRE(grad_ptrs, DR_INVALID_ARGUMENT, "bad argument");
  int opt;
  OptScalars sc;
  int rc = grouped_opt(optimizer, lr, beta1_power, beta2_power, beta1, beta2, epsilon, &opt, &sc);
  if (rc) return rc;
  return apply_grouped(opt, vars, slot1, slot2, num_tables, sc,
                       reinterpret_cast<const float* const*>(grad_ptrs), keys, n_host, n_dev,
                       global_step, S(stream), 1);
}

int dr_ev_apply_grouped_ptr_rows(int optimizer, dr_ev* const* vars, int num_tables,
                                 const uint64_t* const* grad_ptrs, const int64_t* const* keys,
                                 const int64_t* const* rows, const int64_t* n_host,
                                 const int64_t* const* n_dev, float lr, int64_t global_step,
                                 void* stream) {
  using namespace dr;
  DR_REQUIRE(optimizer == DR_OPT_SGD, DR_INVALID_ARGUMENT,
             "dr_ev_apply_grouped_ptr_rows: SGD only (slot columns need the key probe)");
  DR_REQUIRE(grad_ptrs && rows, DR_INVALID_ARGUMENT, "bad argument");
  OptScalars sc = {lr, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  return apply_grouped(OPT_SGD, vars, nullptr, nullptr, num_tables, sc,
                       reinterpret_cast<const float* const*>(grad_ptrs), keys, n_host, n_dev,
                       global_step, S(stream), 1, rows);
}

size_t dr_ev_pool_grad_rows_sgd_workspace_size(int64_t total_nnz, int dim) {
  (void)dim;   // (the long-run piece partials live in the backward's own workspace)
  return dr_pool_grad_rows_workspace_size(total_nnz);
}

int dr_ev_pool_grad_rows_apply_sgd(dr_ev* const* vars, const dr_pool_grad_desc* descs,
                                   int num_tables, int64_t batch, int dim, const int64_t* rowsel,
                                   float lr, int64_t global_step, void* ws, size_t ws_bytes,
                                   void* stream) {
  return dr_ev_pool_grad_rows_apply_sgd_ex(vars, descs, num_tables, batch, dim, rowsel, 0, lr,
                                           global_step, ws, ws_bytes, stream);
}

int dr_ev_pool_grad_rows_apply_sgd_ex(dr_ev* const* vars, const dr_pool_grad_desc* descs,
                                      int num_tables, int64_t batch, int dim,
                                      const int64_t* rowsel, int rows_record, float lr,
                                      int64_t global_step, void* ws, size_t ws_bytes,
                                      void* stream) {
  dr::EvGuard guard_(vars, num_tables);
  using namespace dr;
  DR_REQUIRE(vars && descs && num_tables >= 1 && num_tables <= DR_MAX_GROUP, DR_INVALID_ARGUMENT,
             "bad argument");
  RowsSgd sg;
  memset(&sg, 0, sizeof(sg));
  sg.lr = lr;
  sg.gs = global_step;
  int64_t limit = 1;
  for (int t = 0; t < num_tables; ++t) {
    dr_ev* var = vars[t];
    DR_REQUIRE(var && var->col == 0, DR_INVALID_ARGUMENT, "table %d: var must be a primary EV", t);
    EvShared* s = var->sh;
    DR_REQUIRE(s->value_words == 1 && s->dim == dim && s->bf16 == vars[0]->sh->bf16,
               DR_INVALID_ARGUMENT, "table %d: float / bf16 EVs of one dim and value type", t);
    DR_REQUIRE(s->filter_freq == 0 && s->k_hash == 0, DR_INVALID_ARGUMENT,
               "table %d: the forward's rows stand for LookupOrCreate only without a filter", t);
    for (int j = 0; j < t; ++j)
      DR_REQUIRE(vars[j]->sh != s, DR_INVALID_ARGUMENT,
                 "tables %d and %d share an EV (their updates are sequential rounds)", j, t);
    sg.pool[t] = s->pools[0];
    sg.version[t] = (s->steps_to_live != 0 && global_step != -1) ? s->version : nullptr;
    limit = std::max(limit, s->row_cap);
  }
  sg.bf16 = vars[0]->sh->bf16;
  return rows_apply_sgd(descs, num_tables, batch, dim, rowsel, limit, sg, ws, ws_bytes,
                        S(stream), rows_record);
}

int dr_ev_apply_adagrad_decay_grouped(dr_ev* const* vars, dr_ev* const* accums,
                                      dr_ev* const* decay_powers, int num_tables,
                                      const void* const* grads, int grad_by_address,
                                      const int64_t* const* keys, const int64_t* n_host,
                                      const int64_t* const* n_dev, float lr, int64_t decay_step,
                                      float decay_rate, float decay_baseline,
                                      int64_t global_step, void* stream) {
  using namespace dr;
  // the op's scalar checks and the optimizer's constructor checks
  // (adagrad_decay.py:64-72): a zero decay_step would divide by zero
  DR_REQUIRE(decay_step > 0, DR_INVALID_ARGUMENT, "accumulator_decay_step must be positive");
  DR_REQUIRE(grads, DR_INVALID_ARGUMENT, "bad argument");
  OptScalars sc{};
  sc.lr = lr;
  sc.decay_step = decay_step;
  sc.decay_rate = decay_rate;
  sc.decay_baseline = decay_baseline;
  return apply_grouped(OPT_ADAGRAD_DECAY, vars, accums, decay_powers, num_tables, sc,
                       reinterpret_cast<const float* const*>(grads), keys, n_host, n_dev,
                       global_step, S(stream), grad_by_address ? 1 : 0);
}

static int ftrl_grouped(dr_ev* const* vars, dr_ev* const* accums, dr_ev* const* linears,
                        int num_tables, const float* const* grads, const int64_t* const* keys,
                        const int64_t* n_host, const int64_t* const* n_dev, float lr, float l1,
                        float l2, float lr_power, float l2_shrinkage, int64_t global_step,
                        void* stream, int grad_by_address) {
  using namespace dr;
  // the op's OP_REQUIRES (training_ali_ops.cc:189-246)
  DR_REQUIRE(lr > 0.f, DR_INVALID_ARGUMENT, "lr is not a positive scalar");
  DR_REQUIRE(l1 >= 0.f && l2 >= 0.f && l2_shrinkage >= 0.f, DR_INVALID_ARGUMENT,
             "l1 / l2 / l2_shrinkage regularization strength must be non-negative");
  DR_REQUIRE(lr_power <= 0.f, DR_INVALID_ARGUMENT, "lr_power is not a non-positive scalar");
  OptScalars sc = {lr, 0.f, 0.f, 0.f, 0.f, l1, l2, lr_power, l2_shrinkage};
  return apply_grouped(OPT_FTRL, vars, accums, linears, num_tables, sc, grads, keys, n_host,
                       n_dev, global_step, S(stream), grad_by_address);
}

int dr_ev_apply_ftrl_grouped(dr_ev* const* vars, dr_ev* const* accums, dr_ev* const* linears,
                             int num_tables, const float* const* grads,
                             const int64_t* const* keys, const int64_t* n_host,
                             const int64_t* const* n_dev, float lr, float l1, float l2,
                             float lr_power, float l2_shrinkage, int64_t global_step,
                             void* stream) {
  return ftrl_grouped(vars, accums, linears, num_tables, grads, keys, n_host, n_dev, lr, l1, l2,
                      lr_power, l2_shrinkage, global_step, stream, 0);
}

int dr_ev_apply_ftrl_grouped_ptr(dr_ev* const* vars, dr_ev* const* accums,
                                 dr_ev* const* linears, int num_tables,
                                 const uint64_t* const* grad_ptrs, const int64_t* const* keys,
                                 const int64_t* n_host, const int64_t* const* n_dev, float lr,
                                 float l1, float l2, float lr_power, float l2_shrinkage,
                                 int64_t global_step, void* stream) {
  if (!grad_ptrs) return DR_INVALID_ARGUMENT;
  return ftrl_grouped(vars, accums, linears, num_tables,
                      reinterpret_cast<const float* const*>(grad_ptrs), keys, n_host, n_dev, lr,
                      l1, l2, lr_power, l2_shrinkage, global_step, stream, 1);
}

int dr_ev_apply_ftrl(dr_ev* var, dr_ev* accum, dr_ev* linear, float lr, float l1, float l2,
                     float lr_power, float l2_shrinkage, const float* grad, const int64_t* keys,
                     int64_t n, const int64_t* n_dev, int64_t global_step, void* stream) {
  if (n == 0) return DR_OK;
  dr_ev* v[1] = {var};
  dr_ev* a[1] = {accum};
  dr_ev* l[1] = {linear};
  const float* g[1] = {grad};
  const int64_t* k[1] = {keys};
  const int64_t nh[1] = {n};
  const int64_t* nd[1] = {n_dev};
  return dr_ev_apply_ftrl_grouped(v, a, l, 1, g, k, nh, nd, lr, l1, l2, lr_power, l2_shrinkage,
                                  global_step, stream);
}

int dr_ev_apply_adam(dr_ev* var, dr_ev* m, dr_ev* v, float beta1_power, float beta2_power,
                     float lr, float beta1, float beta2, float epsilon, const float* grad,
                     const int64_t* keys, int64_t n, const int64_t* n_dev, int64_t global_step,
                     void* stream) {
  // alpha = lr * sqrt(1 - beta2^t) / (1 - beta1^t)  (training_ali_ops.cc:935-937)
  const float alpha = lr * sqrtf(1.0f - beta2_power) / (1.0f - beta1_power);
  dr::OptScalars sc = {lr, beta1, beta2, epsilon, alpha, 0, 0, 0, 0};
  return dr::apply_common(dr::OPT_ADAM, var, m, v, sc, grad, keys, n, n_dev, global_step,
                          dr::S(stream));
}

}  // extern "C"

// ===========================================================================
// Owner side of the peer-mapped sharded lookup (dr_xgmi_serve).
// The inbox region of requester src holds cnt[src] (key, slot) pairs written
// over xGMI by src's dr_xgmi_route; a cross-rank barrier separates the two.
// Three launches, each a (grid.x, grid.y = src) grid-stride loop:
//   resolve: insert-on-miss of every inbox key in EV (slot % T)
//   init   : first-touch default rows (kernel boundary: before any read)
//   emit   : row -> out[src][slot * dim] of the requester, over xGMI
//            (1-D grid, destinations interleaved block by block)
// ===========================================================================
namespace dr {

struct XgmiResolveArgs {
  EvDesc e[DR_MAX_GROUP];
  const int64_t* keys;  // local inbox [world][cap]
  const int32_t* slot;
  const int64_t* cnt;   // local [world], written by the requesters
  int64_t cap;
  int T;
};

__device__ __forceinline__ int64_t inbox_count(const int64_t* cnt, int src) {
  return __hip_atomic_load(cnt + src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void xgmi_resolve_kernel(XgmiResolveArgs a,
                                                           int64_t* __restrict__ rows,
                                                           uint8_t* __restrict__ init, int* st) {
  __shared__ EvDesc se[DR_MAX_GROUP];  // per-lane table index: stage in LDS
  if (threadIdx.x < a.T) se[threadIdx.x] = a.e[threadIdx.x];
  __syncthreads();
  const int src = blockIdx.y;
  const int64_t n = inbox_count(a.cnt, src);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t j = (int64_t)src * a.cap + i;
    const uint64_t key = (uint64_t)a.keys[j];
    const int t = a.slot[j] % a.T;
    const EvDesc& e = se[t];
    bool created;
    uint64_t rc;
    Slot* s = ev_find(e, key, true, &created, &rc, st);
    uint8_t flag = 0;
    int64_t row = -1;
    if (s && (rc & kRowMask) != kRowDead) {
      row = (int64_t)(rc & kRowMask);
      const uint64_t bit = 1ull << (48 + e.col);
      if (!(rc & bit)) {
        const uint64_t old = atomicOr((unsigned long long*)&s->rc, (unsigned long long)bit);
        if (!(old & bit)) flag = 1;
      }
    }
    rows[j] = row;
    init[j] = flag;
  }
}

struct XgmiRowArgs {
  float* pool[DR_MAX_GROUP];
  const float* dflt[DR_MAX_GROUP];
  float* out[DR_MAX_PEERS];   // requesters' outputs (peer-mapped)
  const int32_t* slot;
  const int64_t* cnt;
  int64_t cap;
  int64_t dim;
  int T;
  int world;
  int64_t* mtop[DR_MAX_GROUP];   // row counters to mirror (nullptr: none)
  int64_t* mdst[DR_MAX_GROUP];   // their pinned host mirrors
};

// Wave-cooperative first-touch copy (steady state: one byte per key); block
// (0, 0) also mirrors the tables' row counters to the host (the resolve
// before it has finished: the counters are final) -- no per-table copy launch.
__global__ __launch_bounds__(256) void xgmi_init_kernel(XgmiRowArgs a,
                                                        const int64_t* __restrict__ rows,
                                                        const uint8_t* __restrict__ init) {
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < a.T && a.mdst[threadIdx.x]) {
    const int64_t top = __hip_atomic_load(a.mtop[threadIdx.x], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.mdst[threadIdx.x], top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const int src = blockIdx.y;
  const int64_t n = inbox_count(a.cnt, src);
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t base = wave * 64; base < n; base += waves * 64) {
    const int64_t i = base + lane;
    const int64_t j = (int64_t)src * a.cap + i;
    const bool need = i < n && init[j];
    uint64_t mask = __ballot(need);
    while (mask) {
      const int l = __ffsll((unsigned long long)mask) - 1;
      mask &= mask - 1;
      const int64_t jj = __shfl(j, l, 64);
      const int t = a.slot[jj] % a.T;
      float* dst = a.pool[t] + rows[jj] * a.dim;
      const float* src_row = a.dflt[t];
      for (int64_t c = lane; c < a.dim; c += 64) dst[c] = src_row[c];
    }
  }
}

typedef float xf4 __attribute__((ext_vector_type(4)));

// G lanes per row (dim/4 <= G), NB rows in flight per group, nontemporal
// (each row byte crosses once); the stores land in the requester's HBM.
template <int G, int NB>
__global__ __launch_bounds__(256) void xgmi_emit_kernel(XgmiRowArgs a,
                                                        const int64_t* __restrict__ rows) {
  __shared__ const float* spool[DR_MAX_GROUP];  // per-lane table index: stage in LDS
  __shared__ const float* sdflt[DR_MAX_GROUP];
  if (threadIdx.x < a.T) {
    spool[threadIdx.x] = a.pool[threadIdx.x];
    sdflt[threadIdx.x] = a.dflt[threadIdx.x];
  }
  __syncthreads();
  // Destinations interleaved over consecutive blocks (src = block % world):
  // the blocks resident at any moment write to every peer at once, so all
  // xGMI links carry rows together.  A src-major grid would keep most of
  // the chip writing to one peer (one link) at a time.
  const int W = a.world;
  const int src = (int)(blockIdx.x % (unsigned)W);
  const int64_t bx = blockIdx.x / (unsigned)W;
  const int64_t nbx = gridDim.x / (unsigned)W;
  const int64_t n = inbox_count(a.cnt, src);
  constexpr int GPB = 256 / G;
  const int lg = threadIdx.x % G;
  const int dv = (int)(a.dim / 4);
  const int64_t grp = bx * GPB + threadIdx.x / G;
  const int64_t ngrp = nbx * GPB;
  float* out = a.out[src];
  for (int64_t i0 = grp * NB; i0 < n; i0 += ngrp * NB) {
    xf4 x[NB];
    float* dst[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      dst[k] = nullptr;
      x[k] = xf4{0.f, 0.f, 0.f, 0.f};
      const int64_t i = i0 + k;
      if (i < n && lg < dv) {
        const int64_t j = (int64_t)src * a.cap + i;
        const int32_t sl = a.slot[j];
        const int t = sl % a.T;
        const int64_t r = rows[j];
        const float* row = r >= 0 ? spool[t] + r * a.dim : sdflt[t];
        x[k] = __builtin_nontemporal_load(reinterpret_cast<const xf4*>(row) + lg);
        dst[k] = out + (int64_t)sl * a.dim;
      }
    }
#pragma unroll
    for (int k = 0; k < NB; ++k)
      if (dst[k]) __builtin_nontemporal_store(x[k], reinterpret_cast<xf4*>(dst[k]) + lg);
  }
  // no per-block system fence here: xgmi_flush_kernel follows the launch
}

// System-scope release on every XCD (blocks are dispatched round-robin over
// the 8 XCDs; 64 blocks cover each several times): writes back whatever the
// previous kernel left in the XCDs' L2 for the peers' memory.
__global__ void xgmi_flush_kernel() { __threadfence_system(); }

struct XgmiWs {
  int64_t* rows;
  uint8_t* init;
};
static XgmiWs carve_xgmi(void* ws, int world, int64_t cap, size_t* used) {
  Carver c(ws);
  XgmiWs w;
  w.rows = c.take<int64_t>((int64_t)world * cap);
  w.init = c.take<uint8_t>((int64_t)world * cap);
  if (used) *used = c.used + 256;
  return w;
}

}  // namespace dr

extern "C" {

size_t dr_xgmi_serve_workspace_size(int world, int64_t cap) {
  size_t used = 0;
  dr::carve_xgmi(nullptr, world > 0 ? world : 1, cap > 0 ? cap : 1, &used);
  return used;
}

int dr_xgmi_serve(const dr_xgmi_peers* peers, dr_ev* const* evs, int num_tables,
                  int64_t batch, void* ws, size_t ws_bytes, void* stream) {
  dr::EvGuard guard_(evs, num_tables);
  using namespace dr;
  DR_REQUIRE(peers && evs && num_tables >= 1 && num_tables <= DR_MAX_GROUP && batch >= 0,
             DR_INVALID_ARGUMENT, "bad argument");
  const int W = peers->world;
  const int r = peers->rank;
  DR_REQUIRE(W >= 1 && W <= DR_MAX_PEERS && r >= 0 && r < W && peers->cap > 0,
             DR_INVALID_ARGUMENT, "bad world/rank/cap");
  DR_REQUIRE(ws_bytes >= dr_xgmi_serve_workspace_size(W, peers->cap), DR_INVALID_ARGUMENT,
             "serve workspace too small");
  // float words per row (bf16 EVs: D / 2 words, rows moved bitwise -- the
  // bf16 wire format halves the link bytes)
  const int64_t dim = col_words(evs[0]->sh, evs[0]->col);
  DR_REQUIRE(dim % 4 == 0 && dim <= 256, DR_INVALID_ARGUMENT,
             "xgmi serve needs row words %% 4 == 0 and <= 256 (got %lld)", (long long)dim);
  XgmiResolveArgs ra;
  memset(&ra, 0, sizeof(ra));
  XgmiRowArgs wa;
  memset(&wa, 0, sizeof(wa));
  for (int t = 0; t < num_tables; ++t) {
    const EvShared* s = evs[t]->sh;
    DR_REQUIRE(col_words(s, evs[t]->col) == dim && s->bf16 == evs[0]->sh->bf16,
               DR_INVALID_ARGUMENT, "tables must share dim and value type");
    DR_REQUIRE(s->filter_freq == 0 && s->k_hash == 0 && s->value_words == 1,
               DR_INVALID_ARGUMENT, "table %d: xgmi serve is for filter-free fp32 / bf16 EVs", t);
    ra.e[t] = make_desc(evs[t]);
    wa.pool[t] = s->pools[evs[t]->col];
    wa.dflt[t] = s->defaults[evs[t]->col];
  }
  DR_REQUIRE(peers->inbox_keys[r] && peers->inbox_slot[r] && peers->inbox_cnt[r],
             DR_INVALID_ARGUMENT, "own inbox not set");
  ra.keys = peers->inbox_keys[r];
  ra.slot = peers->inbox_slot[r];
  ra.cnt = peers->inbox_cnt[r];
  ra.cap = peers->cap;
  ra.T = num_tables;
  for (int p = 0; p < W; ++p) {
    DR_REQUIRE(peers->out[p], DR_INVALID_ARGUMENT, "peer %d output not mapped", p);
    wa.out[p] = peers->out[p];
  }
  wa.slot = ra.slot;
  wa.cnt = ra.cnt;
  wa.cap = peers->cap;
  wa.dim = dim;
  wa.T = num_tables;
  wa.world = W;
  XgmiWs w = carve_xgmi(ws, W, peers->cap, nullptr);
  int* stw = status_word();
  DR_REQUIRE(stw, DR_INTERNAL, "status word unavailable");
  hipStream_t st = S(stream);
  // Insert-on-miss of up to W * batch new keys per table (every source may
  // send `batch` keys of table t): grow the key table / row pools first,
  // like every other insert path (no host sync while the mirrored row count
  // leaves room).
  for (int t = 0; t < num_tables; ++t) {
    int rc = reserve(evs[t]->sh, (int64_t)W * batch, st);
    if (rc) return rc;
    ra.e[t] = make_desc(evs[t]);   // grow() may have moved the table / pools
    wa.pool[t] = evs[t]->sh->pools[evs[t]->col];
    wa.dflt[t] = evs[t]->sh->defaults[evs[t]->col];
  }
  // One-shot grids sized for 1.25x the keys a source sends on average
  // (T*B / W for keys spread over owners); the kernels' grid-stride loops
  // take any excess (skewed keys) in a second pass.  Small grids with long
  // grid-stride loops measured ~30% slower on the emit.
  const int64_t per_src = std::max<int64_t>(1, (int64_t)num_tables * batch / W);
  const int64_t expect = per_src + per_src / 4 + 256;
  const unsigned gx = (unsigned)ceil_div(expect, 256);
  hipLaunchKernelGGL(xgmi_resolve_kernel, dim3(gx, W), dim3(256), 0, st, ra, w.rows, w.init, stw);
  // counter mirrors ride on the init kernel (as resolve_grouped's)
  EvShared* mir[DR_MAX_GROUP];
  int nmir = 0;
  for (int t = 0; t < num_tables; ++t) {
    EvShared* sh = evs[t]->sh;
    bool seen = false;
    for (int q = 0; q < nmir; ++q) seen = seen || mir[q] == sh;
    if (seen) continue;
    sh->mu.lock();
    if (want_mirror(sh, st)) {
      wa.mtop[t] = sh->top;
      wa.mdst[t] = sh->pinned_top;
      mir[nmir++] = sh;
    } else {
      sh->mu.unlock();
    }
  }
  hipLaunchKernelGGL(xgmi_init_kernel, dim3(gx, W), dim3(256), 0, st, wa, w.rows, w.init);
  {
    const hipError_t le = hipGetLastError();
    for (int q = 0; q < nmir; ++q) {
      if (le == hipSuccess) mirrored(mir[q], st);
      mir[q]->mu.unlock();
    }
    if (le != hipSuccess) {
      set_error("kernel launch failed: %s", hipGetErrorString(le));
      return DR_INTERNAL;
    }
  }
  for (int t = 0; t < num_tables; ++t) wa.mtop[t] = wa.mdst[t] = nullptr;   // (emit: unused)
  const int dv = (int)(dim / 4);
  auto ge = [&](int G) { return dim3((unsigned)(ceil_div(expect, (256 / G) * 4) * W)); };
  if (dv <= 8)
    hipLaunchKernelGGL((xgmi_emit_kernel<8, 4>), ge(8), dim3(256), 0, st, wa, w.rows);
  else if (dv <= 16)
    hipLaunchKernelGGL((xgmi_emit_kernel<16, 4>), ge(16), dim3(256), 0, st, wa, w.rows);
  else if (dv <= 32)
    hipLaunchKernelGGL((xgmi_emit_kernel<32, 4>), ge(32), dim3(256), 0, st, wa, w.rows);
  else
    hipLaunchKernelGGL((xgmi_emit_kernel<64, 4>), ge(64), dim3(256), 0, st, wa, w.rows);
  // (one rank: the rows stay on this device, whose next kernels see them
  // after the kernel boundary -- no system-scope release needed)
  if (W > 1) hipLaunchKernelGGL(xgmi_flush_kernel, dim3(64), dim3(64), 0, st);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // extern "C"
