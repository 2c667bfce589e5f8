// unique.hip -- Unique / UniqueWithCounts in first-occurrence order, for one
// table or for all T tables of a step in one pass (grouped).
//
// Replaces UniqueAliOp (core/kernels/unique_ali_op.cc:46-180); the order
// contract is SerialComputeV1 (unique_ali_op_util.h:192-222): y lists keys
// in order of first appearance, idx[i] = position of x[i] in y.
//
// GPU algorithm: hash-partition, then LDS dedup per bucket (no host sync,
// integer-exact, no global atomics on the common path).
//   1. count: table t's keys are cut into tiles of UQ_TILE positions; each
//      tile histograms its keys over the table's nb_t hash buckets (high
//      bits of mix64(key), nb_t ~ n_t / UQ_TARGET) in LDS;
//   2. an exclusive scan of the [table][bucket][tile] count matrix gives
//      every (bucket, tile) its output range (table t's buckets land at
//      [koff[t], koff[t+1]), in bucket order);
//   3. scatter: each tile writes (key, position) pairs into those ranges (LDS
//      cursors; a wave whose 64 keys share one bucket reserves once);
//   4. dedup: one workgroup per bucket builds an LDS hash of the bucket's
//      distinct keys.  A slot holds the bucket-local index of the key's
//      first inserter (the key itself is compared in the immutable
//      partitioned array), plus LDS atomicMin of the position (= the key's
//      FIRST occurrence, order-free) and LDS atomicAdd of the count.  Runs
//      of one key in consecutive lanes (a hot id, padded histories) are
//      reduced in registers first and touch the slot once.  A bucket with
//      more distinct keys than the LDS table holds continues in a global
//      hash region of its own (same protocol, global atomics).
//      Per distinct key: flag[first] = 1, cnt_at[first] = count; per
//      element (bucket order): its key's first position;
//   5. exclusive scan of flag over positions: rank of each first occurrence;
//   6. emit (bucket order): idx[p] = rank(first(p)) - rank(table start), and
//      at first positions uniq[..] = key, counts[..] = count.
// Every key value (-1 included) is an ordinary key: empty is an index
// (0xFFFFFFFF), never a key.  Outputs keep the input layout: table t's
// uniques / counts sit at [koff[t], koff[t] + U_t) and U_t goes to
// num_unique[t] (device int64).
#include "dr_common.h"

namespace dr {

static constexpr uint32_t kEmptyIx = ~0u;
static constexpr int UQ_TILE = 4096;     // positions per count / scatter block (256 x 16)
static constexpr int UQ_TARGET = 1024;   // keys per bucket aimed at
static constexpr int UQ_MAXB = 1024;     // buckets per table (LDS histogram)
static constexpr int UQ_LCAP = 2048;     // LDS hash slots per bucket (24 KB)
static constexpr int UQ_ESLOT = 4096;    // elements whose slot is kept in LDS (16 KB)

struct UqGroup {
  int64_t koff[DR_MAX_GROUP + 1];   // input offsets
  int64_t tbase[DR_MAX_GROUP + 1];  // first tile of table t
  int64_t cbase[DR_MAX_GROUP + 1];  // first count-matrix entry of table t
  int64_t bbase[DR_MAX_GROUP + 1];  // first global bucket of table t
  int32_t nb[DR_MAX_GROUP];         // buckets of table t (pow2; 0 when empty)
};

struct UqWs {
  int32_t* cnt;     // [ncnt] count matrix, scanned in place
  int64_t* pkey;    // [n] partitioned keys
  int32_t* ppos;    // [n] their positions
  int32_t* pfirst;  // [n] first position of each partitioned element's key
  int32_t* flags;   // [n] first-occurrence flags, scanned in place
  int32_t* cnt_at;  // [n] count of the key whose first position this is
  uint32_t* gidx;   // [2n] overflow hash regions (bucket b: [2 start, 2 end))
  uint32_t* gmin;   // [2n]
  int32_t* gcnt;    // [2n]
  int64_t* total;   // [2] scan totals
  void* scan_ws;
};

static void build_group(const int64_t* koff, int T, UqGroup* g, int64_t* ncnt, int64_t* nbk,
                        int64_t* ntiles) {
  int64_t tb = 0, cb = 0, bb = 0;
  for (int t = 0; t < T; ++t) {
    const int64_t n = koff[t + 1] - koff[t];
    g->koff[t] = koff[t];
    g->tbase[t] = tb;
    g->cbase[t] = cb;
    g->bbase[t] = bb;
    int64_t nb = 0, tiles = 0;
    if (n > 0) {
      nb = next_pow2(ceil_div(n, UQ_TARGET));
      if (nb > UQ_MAXB) nb = UQ_MAXB;
      tiles = ceil_div(n, UQ_TILE);
    }
    g->nb[t] = (int32_t)nb;
    tb += tiles;
    cb += nb * tiles;
    bb += nb;
  }
  g->koff[T] = koff[T];
  g->tbase[T] = tb;
  g->cbase[T] = cb;
  g->bbase[T] = bb;
  *ncnt = cb;
  *nbk = bb;
  *ntiles = tb;
}

static UqWs carve_unique(void* ws, int64_t n, int64_t ncnt, size_t* used) {
  Carver c(ws);
  UqWs u;
  const int64_t nn = n > 0 ? n : 1;
  u.cnt = c.take<int32_t>(ncnt > 0 ? ncnt : 1);
  u.pkey = c.take<int64_t>(nn);
  u.ppos = c.take<int32_t>(nn);
  u.pfirst = c.take<int32_t>(nn);
  u.flags = c.take<int32_t>(nn);
  u.cnt_at = c.take<int32_t>(nn);
  u.gidx = c.take<uint32_t>(2 * nn);
  u.gmin = c.take<uint32_t>(2 * nn);
  u.gcnt = c.take<int32_t>(2 * nn);
  u.total = c.take<int64_t>(2);
  const int64_t sn = ncnt > nn ? ncnt : nn;
  u.scan_ws = c.take<char>(scan_ws_bytes(sn));
  if (used) *used = c.used + 256;
  return u;
}

// overflow-region words after their atomics: read at device scope (past L1)
__device__ __forceinline__ uint32_t uq_ld(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int uq_bucket(uint64_t h, int nb) {
  return nb > 1 ? (int)((h >> 40) & (uint64_t)(nb - 1)) : 0;
}

// Block g of the tile grid: its table, tile index and position range.
__device__ __forceinline__ void uq_tile(const UqGroup& g, int T, int64_t blk, int* t, int64_t* j,
                                        int64_t* p0, int64_t* p1) {
  const int tt = table_of(g.tbase, T, blk, blk);
  *t = tt;
  *j = blk - g.tbase[tt];
  *p0 = g.koff[tt] + *j * UQ_TILE;
  const int64_t e = *p0 + UQ_TILE;
  *p1 = e < g.koff[tt + 1] ? e : g.koff[tt + 1];
}

__global__ __launch_bounds__(256) void uq_count_kernel(UqGroup g, int T,
                                                       const int64_t* __restrict__ keys,
                                                       int32_t* __restrict__ cnt) {
  __shared__ int hist[UQ_MAXB];
  int t;
  int64_t j, p0, p1;
  uq_tile(g, T, blockIdx.x, &t, &j, &p0, &p1);
  const int nb = g.nb[t];
  for (int d = threadIdx.x; d < nb; d += 256) hist[d] = 0;
  __syncthreads();
  const int lane = __lane_id();
  for (int64_t i = p0 + threadIdx.x; i - threadIdx.x < p1; i += 256) {
    const bool in = i < p1;
    const int d = in ? uq_bucket(mix64((uint64_t)gld(keys + i)), nb) : -1;
    // a wave whose live lanes all hit one bucket (a hot id) adds once
    const int d0 = __shfl(d, 0, 64);
    const uint64_t live = __ballot(in);
    if (__ballot(in && d == d0) == live) {
      if (lane == 0) atomicAdd(&hist[d0], (int)__popcll(live));
    } else if (in) {
      atomicAdd(&hist[d], 1);
    }
  }
  __syncthreads();
  const int64_t tiles = g.tbase[t + 1] - g.tbase[t];
  for (int d = threadIdx.x; d < nb; d += 256) cnt[g.cbase[t] + (int64_t)d * tiles + j] = hist[d];
}

__global__ __launch_bounds__(256) void uq_scatter_kernel(UqGroup g, int T,
                                                         const int64_t* __restrict__ keys,
                                                         const int32_t* __restrict__ cnt,
                                                         int64_t* __restrict__ pkey,
                                                         int32_t* __restrict__ ppos) {
  __shared__ int cur[UQ_MAXB];
  int t;
  int64_t j, p0, p1;
  uq_tile(g, T, blockIdx.x, &t, &j, &p0, &p1);
  const int nb = g.nb[t];
  const int64_t tiles = g.tbase[t + 1] - g.tbase[t];
  for (int d = threadIdx.x; d < nb; d += 256) cur[d] = cnt[g.cbase[t] + (int64_t)d * tiles + j];
  __syncthreads();
  const int lane = __lane_id();
  for (int64_t i = p0 + threadIdx.x; i - threadIdx.x < p1; i += 256) {
    const bool in = i < p1;
    const int64_t k = in ? gld(keys + i) : 0;
    const int d = in ? uq_bucket(mix64((uint64_t)k), nb) : -1;
    const int d0 = __shfl(d, 0, 64);
    const uint64_t live = __ballot(in);
    int slot;
    if (__ballot(in && d == d0) == live) {
      int base = 0;
      if (lane == 0) base = atomicAdd(&cur[d0], (int)__popcll(live));
      base = __shfl(base, 0, 64);
      slot = base + (int)__popcll(live & lanemask_lt());
    } else {
      slot = in ? atomicAdd(&cur[d], 1) : 0;
    }
    if (in) {
      gst(pkey + slot, k);
      gst(ppos + slot, (int32_t)i);
    }
  }
}

// Segmented (by runs of equal keys in consecutive lanes) min / sum to the run
// head.  head: this lane starts a run.
__device__ __forceinline__ void run_reduce(bool head, uint32_t* pmin, int* pcnt) {
  const uint64_t heads = __ballot(head);
  const int lane = __lane_id();
  // run end (exclusive) of this lane's run
  const uint64_t after = heads & ~((2ull << lane) - 1);  // heads strictly after lane
  const int end = after ? __ffsll((unsigned long long)after) - 1 : 64;
  uint32_t m = *pmin;
  int c = *pcnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t om = (uint32_t)__shfl_down((int)m, off, 64);
    const int oc = __shfl_down(c, off, 64);
    if (lane + off < end) {
      m = om < m ? om : m;
      c += oc;
    }
  }
  *pmin = m;
  *pcnt = c;
}

__global__ __launch_bounds__(256) void uq_dedup_kernel(
    UqGroup g, int T, const int32_t* __restrict__ cnt, const int64_t* __restrict__ pkey,
    const int32_t* __restrict__ ppos, int32_t* __restrict__ pfirst, int32_t* __restrict__ flags,
    int32_t* __restrict__ cnt_at, uint32_t* __restrict__ gidx, uint32_t* __restrict__ gmin,
    int32_t* __restrict__ gcnt, int lprobes, int* st) {
  // one LDS array: [idx | min | cnt] x UQ_LCAP, then the overflow flag
  __shared__ uint32_t lds[3 * UQ_LCAP + 1 + UQ_ESLOT];
  uint32_t* lidx = lds;
  uint32_t* lmin = lds + UQ_LCAP;
  int* lcnt = reinterpret_cast<int*>(lds + 2 * UQ_LCAP);
  int* lover = reinterpret_cast<int*>(lds + 3 * UQ_LCAP);
  // slot of element e < UQ_ESLOT (kEmptyIx: not in the LDS table)
  uint32_t* eslot = lds + 3 * UQ_LCAP + 1;
  const int64_t gb = blockIdx.x;
  const int t = table_of(g.bbase, T, gb, gb);
  const int d = (int)(gb - g.bbase[t]);
  const int64_t tiles = g.tbase[t + 1] - g.tbase[t];
  const int64_t start = cnt[g.cbase[t] + (int64_t)d * tiles];
  const int64_t end = d + 1 < g.nb[t] ? (int64_t)cnt[g.cbase[t] + (int64_t)(d + 1) * tiles]
                                      : g.koff[t + 1];
  const int64_t m = end - start;
  for (int s = threadIdx.x; s < UQ_LCAP; s += 256) {
    lidx[s] = kEmptyIx;
    lmin[s] = kEmptyIx;
    lcnt[s] = 0;
  }
  if (threadIdx.x == 0) *lover = 0;
  __syncthreads();
  if (m <= 0) return;
  const int64_t* bk = pkey + start;
  const int lane = __lane_id();
  const int64_t gcap = 2 * m;
  uint32_t* gi = gidx + 2 * start;
  uint32_t* gm = gmin + 2 * start;
  int* gc = gcnt + 2 * start;
  // Pass 1 inserts.  e runs over the bucket in 256-element chunks, so the
  // lanes of a wave see consecutive partitioned elements (runs of one key:
  // the scatter wrote a hot id's wave-runs contiguously); the run's min
  // position and count are reduced in registers and its head touches the
  // slot once.  A key lives in the LDS table iff the CAS walk of its first
  // inserter found a free slot within UQ_LCAP / 2 probes; slots are never
  // freed, so every later walk of the key meets it.  Walks that fail mark
  // the bucket overflowed, and (round b) go to the bucket's global region,
  // filled first by the block: a key sits in exactly one of the two tables.
  auto chunk_key = [&](int64_t e0, int64_t* k, uint32_t* p, int* c, bool* head) {
    const int64_t e = e0 + threadIdx.x;
    const bool in = e < m;
    *k = in ? gld(bk + e) : 0;
    *p = in ? (uint32_t)gld(ppos + start + e) : kEmptyIx;
    *c = in ? 1 : 0;
    const uint32_t klo = (uint32_t)*k, khi = (uint32_t)((uint64_t)*k >> 32);
    const uint32_t plo = (uint32_t)__shfl_up((int)klo, 1, 64);
    const uint32_t phi = (uint32_t)__shfl_up((int)khi, 1, 64);
    *head = in && (lane == 0 || plo != klo || phi != khi);
    run_reduce(*head || !in, p, c);
  };
  auto lds_find = [&](int64_t k, uint64_t h) -> int {  // slot of k, or -1
    uint32_t s = (uint32_t)h & (UQ_LCAP - 1);
    for (int probes = 0; probes < lprobes; ++probes) {
      const uint32_t cur = lidx[s];
      if (cur == kEmptyIx) return -1;
      if (gld(bk + cur) == k) return (int)s;
      s = (s + 1) & (UQ_LCAP - 1);
    }
    return -1;
  };
  for (int64_t e0 = 0; e0 < m; e0 += 256) {
    int64_t k;
    uint32_t p;
    int c;
    bool head;
    chunk_key(e0, &k, &p, &c, &head);
    uint32_t mys = kEmptyIx;
    if (head) {
      uint32_t s = (uint32_t)mix64((uint64_t)k) & (UQ_LCAP - 1);
      for (int probes = 0; probes < lprobes; ++probes) {
        const uint32_t old = atomicCAS(&lidx[s], kEmptyIx, (uint32_t)(e0 + threadIdx.x));
        if (old == kEmptyIx || gld(bk + old) == k) {
          atomicMin(&lmin[s], p);
          atomicAdd(&lcnt[s], c);
          mys = s;
          break;
        }
        s = (s + 1) & (UQ_LCAP - 1);
      }
      if (mys == kEmptyIx) *lover = 1;
    }
    // run members take their head's slot (the nearest head at or below)
    const uint64_t hb = __ballot(head);
    const uint64_t le = hb & (lanemask_lt() | (1ull << lane));
    const int src = le ? 63 - __clzll((long long)le) : lane;
    mys = (uint32_t)__shfl((int)mys, src, 64);
    const int64_t e = e0 + threadIdx.x;
    if (e < m && e < UQ_ESLOT) eslot[e] = mys;
  }
  __syncthreads();
  if (*lover) {  // round b (rare): the keys whose walk failed, into the global region
    for (int64_t q = threadIdx.x; q < gcap; q += 256) {
      gi[q] = kEmptyIx;
      gm[q] = kEmptyIx;
      gc[q] = 0;
    }
    __syncthreads();
    for (int64_t e0 = 0; e0 < m; e0 += 256) {
      int64_t k;
      uint32_t p;
      int c;
      bool head;
      chunk_key(e0, &k, &p, &c, &head);
      if (!head) continue;
      const uint64_t h = mix64((uint64_t)k);
      if (lds_find(k, h) >= 0) continue;  // counted in round a
      uint64_t q = h % (uint64_t)gcap;
      bool done = false;
      for (int64_t probes = 0; probes < gcap; ++probes) {
        const uint32_t old = atomicCAS(&gi[q], kEmptyIx, (uint32_t)(e0 + threadIdx.x));
        if (old == kEmptyIx || gld(bk + old) == k) {
          atomicMin(&gm[q], p);
          atomicAdd(&gc[q], c);
          done = true;
          break;
        }
        q = q + 1 == (uint64_t)gcap ? 0 : q + 1;
      }
      if (!done) latch(st, DR_INTERNAL);
    }
    __syncthreads();
  }
  const bool over = *lover != 0;
  // pass 2: per element its key's first position (bucket order); per distinct
  // key flag + count at the first position
  for (int64_t e = threadIdx.x; e < m; e += 256) {
    uint32_t f = kEmptyIx;
    int64_t k = 0;
    uint64_t h = 0;
    if (e < UQ_ESLOT) {
      const uint32_t es = eslot[e];
      if (es != kEmptyIx) f = lmin[es];
    } else {
      k = gld(bk + e);
      h = mix64((uint64_t)k);
      const int ls = lds_find(k, h);
      if (ls >= 0) f = lmin[ls];
    }
    if (f == kEmptyIx && over && e < UQ_ESLOT) {
      k = gld(bk + e);
      h = mix64((uint64_t)k);
    }
    if (f == kEmptyIx && over) {
      uint64_t q = h % (uint64_t)gcap;
      for (int64_t probes = 0; probes < gcap; ++probes) {
        const uint32_t cur = uq_ld(gi + q);
        if (cur == kEmptyIx) break;
        if (gld(bk + cur) == k) {
          f = uq_ld(gm + q);
          break;
        }
        q = q + 1 == (uint64_t)gcap ? 0 : q + 1;
      }
    }
    if (f == kEmptyIx) {
      latch(st, DR_INTERNAL);
      f = (uint32_t)gld(ppos + start + e);
    }
    gst(pfirst + start + e, (int32_t)f);
  }
  for (int s = threadIdx.x; s < UQ_LCAP; s += 256) {
    if (lidx[s] != kEmptyIx) {
      gst(flags + lmin[s], 1);
      gst(cnt_at + lmin[s], lcnt[s]);
    }
  }
  if (over) {
    for (int64_t q = threadIdx.x; q < gcap; q += 256) {
      if (uq_ld(gi + q) != kEmptyIx) {
        const uint32_t f = uq_ld(gm + q);
        gst(flags + f, 1);
        gst(cnt_at + f, (int32_t)uq_ld(reinterpret_cast<uint32_t*>(gc) + q));
      }
    }
  }
}

// After the scan flags[] holds exclusive prefix sums.  Bucket order: each
// element's idx (scattered by position), and at first positions the unique
// key and its count.
__global__ void uq_emit_kernel(UqGroup g, int T, int64_t n, const int64_t* __restrict__ pkey,
                               const int32_t* __restrict__ ppos,
                               const int32_t* __restrict__ pfirst,
                               const int32_t* __restrict__ prefix,
                               const int32_t* __restrict__ cnt_at, int64_t* __restrict__ uniq,
                               int32_t* __restrict__ idx, int32_t* __restrict__ counts) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  // partitioned element e belongs to the table whose range holds it
  const int t = table_of(g.koff, T, e, (int64_t)blockIdx.x * blockDim.x);
  const int64_t kt = g.koff[t];
  const int32_t p = ppos[e];
  const int32_t f = pfirst[e];
  const int32_t u = prefix[f] - prefix[kt];
  gst(idx + p, u);
  if (f == p) {
    gst(uniq + kt + u, pkey[e]);
    if (counts) gst(counts + kt + u, cnt_at[p]);
  }
}

__global__ void uq_num_unique_kernel(UqGroup g, int T, const int32_t* __restrict__ prefix,
                                     const int64_t* __restrict__ total,
                                     int64_t* __restrict__ num_unique) {
  const int t = threadIdx.x;
  if (t >= T) return;
  const int64_t n = g.koff[T];
  const int64_t a = g.koff[t] < n ? prefix[g.koff[t]] : *total;
  const int64_t b = g.koff[t + 1] < n ? prefix[g.koff[t + 1]] : *total;
  num_unique[t] = g.koff[t + 1] > g.koff[t] ? b - a : 0;
}

// LDS walk bound (UQ_LCAP / 2); dr_unique_set_lds_probes lowers it so tests
// can drive the overflow path with small inputs
static int g_uq_lds_probes = UQ_LCAP / 2;

}  // namespace dr

extern "C" int dr_unique_set_lds_probes(int probes) {
  if (probes < 1 || probes > dr::UQ_LCAP / 2) probes = dr::UQ_LCAP / 2;
  dr::g_uq_lds_probes = probes;
  return DR_OK;
}

extern "C" size_t dr_unique_grouped_workspace_size(const int64_t* koff_host, int num_tables) {
  if (num_tables < 1 || num_tables > DR_MAX_GROUP) return 0;
  dr::UqGroup g;
  int64_t ncnt, nbk, ntiles;
  dr::build_group(koff_host, num_tables, &g, &ncnt, &nbk, &ntiles);
  size_t used = 0;
  dr::carve_unique(nullptr, koff_host[num_tables], ncnt, &used);
  return used;
}

extern "C" int dr_unique_grouped(const int64_t* keys, const int64_t* koff_host, int num_tables,
                                 int64_t* uniq_out, int32_t* idx_out, int32_t* counts_out,
                                 int64_t* num_unique, void* ws, size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(num_tables >= 1 && num_tables <= DR_MAX_GROUP, DR_INVALID_ARGUMENT,
             "dr_unique_grouped: 1..%d tables", DR_MAX_GROUP);
  const int T = num_tables;
  const int64_t n = koff_host[T];
  DR_REQUIRE(n >= 0 && n < (int64_t)0x3fffffff, DR_INVALID_ARGUMENT, "dr_unique: bad n");
  for (int t = 0; t < T; ++t)
    DR_REQUIRE(koff_host[t + 1] >= koff_host[t], DR_INVALID_ARGUMENT, "koff must be sorted");
  DR_REQUIRE(ws_bytes >= dr_unique_grouped_workspace_size(koff_host, T), DR_INVALID_ARGUMENT,
             "dr_unique: workspace too small");
  hipStream_t st = S(stream);
  if (n == 0) {
    return fill_bytes(num_unique, 0, T * sizeof(int64_t), st);
  }
  int* sw = status_word();
  DR_REQUIRE(sw, DR_INTERNAL, "status word unavailable");
  UqGroup g;
  int64_t ncnt, nbk, ntiles;
  build_group(koff_host, T, &g, &ncnt, &nbk, &ntiles);
  UqWs u = carve_unique(ws, n, ncnt, nullptr);
  // (a bucket's overflow region is initialised by that bucket's block, and
  // only when it overflows)
  int frc = fill_bytes(u.flags, 0, n * sizeof(int32_t), st);
  if (frc) return frc;
  hipLaunchKernelGGL(uq_count_kernel, dim3((unsigned)ntiles), dim3(256), 0, st, g, T, keys, u.cnt);
  DR_LAUNCH_CHECK();
  int rc = scan_exclusive_i32(u.cnt, u.cnt, ncnt, nullptr, u.total + 1, u.scan_ws, st);
  if (rc) return rc;
  hipLaunchKernelGGL(uq_scatter_kernel, dim3((unsigned)ntiles), dim3(256), 0, st, g, T, keys,
                     u.cnt, u.pkey, u.ppos);
  hipLaunchKernelGGL(uq_dedup_kernel, dim3((unsigned)nbk), dim3(256), 0, st, g, T, u.cnt, u.pkey,
                     u.ppos, u.pfirst, u.flags, u.cnt_at, u.gidx, u.gmin, u.gcnt,
                     g_uq_lds_probes, sw);
  DR_LAUNCH_CHECK();
  rc = scan_exclusive_i32(u.flags, u.flags, n, nullptr, u.total, u.scan_ws, st);
  if (rc) return rc;
  hipLaunchKernelGGL(uq_emit_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, g, T, n,
                     u.pkey, u.ppos, u.pfirst, u.flags, u.cnt_at, uniq_out, idx_out, counts_out);
  hipLaunchKernelGGL(uq_num_unique_kernel, dim3(1), dim3(64), 0, st, g, T, u.flags, u.total,
                     num_unique);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

extern "C" size_t dr_unique_workspace_size(int64_t n) {
  const int64_t koff[2] = {0, n > 0 ? n : 0};
  return dr_unique_grouped_workspace_size(koff, 1);
}

extern "C" int dr_unique(const int64_t* keys, int64_t n, int64_t* uniq_out, int32_t* idx_out,
                         int32_t* counts_out, int64_t* num_unique, void* ws, size_t ws_bytes,
                         void* stream) {
  const int64_t koff[2] = {0, n};
  return dr_unique_grouped(keys, koff, 1, uniq_out, idx_out, counts_out, num_unique, ws, ws_bytes,
                           stream);
}
