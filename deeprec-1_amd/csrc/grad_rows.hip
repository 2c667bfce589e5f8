// grad_rows.hip -- backward of a grouped pooled EV lookup keyed by the rows
// the forward resolved (dr_pool_grad_rows_grouped).
//
// The reference's training lookup is Unique -> gather -> SparseSegmentSum
// (python/ops/embedding_ops.py:592-675); its gradient is IndexedSlices over
// the unique ids in first-occurrence order, each value the SparseSegment*Grad
// sum of that id's positions in ascending order (segment_reduction_ali_ops_
// util.h:331-458 / math_grad.py:321-368).  For filter-free EVs the forward
// here skips the Unique (every nnz is resolved straight into the EV: the CAS
// insert is the dedup), so the backward regroups by the resolved row
// instead of by a unique index:
//
//   1. (row of nnz i, i) pairs, stable radix sort by row.  Positions are
//      table-major and the sort is stable, so the positions of one (table,
//      row) are contiguous and ascending: a run.
//   2. mark[first position of each run] = its sorted index; exclusive scan
//      of the marks over positions
//      -> the first-occurrence rank of every unique id of table t, i.e. the
//      index Unique would have given it; U_t from the scan.
//   3. one position pass emits the unique ids in that order.
//   4. per run, the gradient (rows_emit_kernel, position order): a
//      one-position run whose value needs no arithmetic is handed on BY
//      ADDRESS (grad_ptr[o] = the pooled-grad row, bit 0 = "add +0.0f", the
//      0 + x of the reference's unsorted sum), so the optimizer reads the
//      pooled gradient directly and no [U, D] gradient is written and read
//      back; every other run goes to a worklist that rows_work_kernel (G
//      lanes per entry) sums into grad_unique[o] (grad_ptr[o] points there).
//
// A run of at most kRowsChunk positions is summed serially in ascending
// order by one lane group (rows_work_kernel) -- bit-exact to the reference
// loops.  Longer runs (hot ids) go to the long-run kernels: rows_expand_kernel
// measures each run (two rounds of parallel probes) and cuts it into pieces
// of serial_max() positions counted from the RUN's first position (default:
// unbounded, one piece per run); every piece is summed in ascending position order by rows_serial_kernel (one
// block per piece and column slice: all threads stage the piece's gradient
// rows through LDS, one wave walks each column's serial chain), and a run of
// several pieces is the ordered sum of its piece partials
// (rows_combine_kernel).  So every run (any length, by default) is the
// reference's exact serial sum (segment_reduction_ops.cc:391-404), and every
// association depends only on the run's own position order -- never on the
// key -> row numbering that racing first-touch inserts assign, nor on where
// the run lands in the sorted array.
#include "dr_repadd.h"
#include "dr_rows.h"

namespace dr {

struct RowsGroup {
  dr_pool_grad_desc d[DR_MAX_GROUP];
  int64_t koff[DR_MAX_GROUP + 1];
};

static constexpr int64_t kRowsChunk = 256;    // longest run of the lane-group path
// Longest exact-serial piece of a long run.  Default: unbounded -- every run,
// however long (a hot id over a whole batch), is ONE serial chain in the
// reference's ascending order, bit-exact (segment_reduction_ops.cc:391-404).
// DR_GRAD_SERIAL_MAX=n (A/B switch) cuts runs into pieces of n positions
// summed in parallel and combined in order (deterministic, fp32-tolerance).
static int64_t serial_max() {
  static const int64_t v = [] {
    const char* e = getenv("DR_GRAD_SERIAL_MAX");
    const long long n = e ? atoll(e) : 0;
    // (pieces share the run list's capacity: at least kRowsChunk + 1 long)
    return n > 0 ? (int64_t)(n > 8192 ? n : 8192) : (int64_t)(1ll << 40);
  }();
  return v;
}
#ifndef DR_ROWS_CHAIN
#define DR_ROWS_CHAIN 8
#endif
static constexpr int kRowsChain = DR_ROWS_CHAIN;  // positions of a run fetched per step
static constexpr int64_t kRowsMaxDim = 1024;
// Zero-term skipping on long serial chains.  A zero-started chain
// (0 + x_0 + x_1 ..., the sum combiner or a weighted lookup) is never -0.0,
// so adding a term that is +0.0 or -0.0 leaves it bit-for-bit unchanged
// (round-to-nearest: s + 0 = s for every s != -0; NaN / Inf terms are not
// zero and are kept).  Runs longer than zero_scan() positions are first
// scanned in parallel (rows_nz_kernel: chunks of kRowsChunk positions, each
// compacted to its nonzero terms in ascending order) and the serial walk
// visits only those -- e.g. a padding id whose positions are masked out
// downstream.  A run that is mostly nonzero (DIN's padding id: its history
// positions feed the unmasked his_sum, model.py:98, so they all carry
// gradient) is walked whole instead (run_sparse()).  Opt-in:
// DR_GRAD_ZERO_SKIP=1 (zero_scan()).
// Plain-sum runs (no weights, no mean / sqrtn scale, not walked compacted)
// go to rows_serial_plain_kernel (1, default) or rows_serial_dma_kernel (2,
// A/B); DR_GRAD_SERIAL_PLAIN=0 keeps them in rows_serial_kernel.
static int serial_dma() {   // read per call (host, once per backward): tests cover each walker
  const char* e = getenv("DR_GRAD_SERIAL_PLAIN");
  return e ? atoi(e) : 1;
}

// Segment scan of the plain long runs (A/B, opt-in): a one-piece plain-sum
// run longer than seg_scan() positions is first split (rows_seg_kernel, in
// parallel) into segments of bitwise-identical consecutive terms -- DIN's
// padding id: each sample's padded history positions all carry that
// sample's his_sum gradient -- and, when its segments average at least
// kSegMin terms, walked one segment at a time (rows_serial_seg_kernel): k
// additions of one term in closed form (rep_add, dr_repadd.h), bit-equal to
// k plain adds.  Off by default: a closed-form segment costs ~600 cycles
// of branchy integer work against 8.5 per position for the plain chain, so
// it only pays for segments of ~70+ terms; DIN's average 50 (4 050 segments
// over 203 800 padding positions) walked 4x slower (profiles/r05_seg_walk.log).
// Read per call (DR_GRAD_SEG_SCAN=n positions; 0 = off).  Round 6: the
// segment step is two fp32 adds then the rest in closed form on the sum's
// grid (serial_seg_walk, dr_repadd.h seg_walk2: 93-97 % of DIN's segments),
// every value wave-uniform, one walker wave per SIMD, segments of >= 16
// terms on average: ~450 cycles per segment measured (clock64, ~10 cycles
// per dependent instruction of a lone wave), 0.83-1.19 ms for DIN's chain
// against the plain walk's 1.0 -- still opt-in (profiles/r06_seg_rounds_walk.log).
// Round 6: DR_GRAD_SEG_ROUNDS=1 (opt-in) walks the segments by a whole wave
// in rounds (wave_rounds_walk: every segment of a window on the running
// sum's grid at once, an integer prefix over the lanes, the segment where the
// grid changes added exactly by seg_add), scanning runs longer than 4 096
// positions and walking them by segments when they average >= 8 terms.  Its
// cost is data-dependent: a round per grid change.  DIN's padding chain at
// the first step (sums growing steadily to ~0.06) takes ~100 rounds per
// column, 0.48 ms against the plain walk's 1.0; after training the column
// sums wander around 1e-5, every few segments change the grid (200-350
// rounds per column, tools/din_term_probe.py DTP_STEPS + tools/
// repadd_check.cpp file mode) and the walk takes 0.3-1.6 ms per step, 1.0 on
// average -- no better than the plain walk, which stays the default
// (profiles/r06_seg_rounds_walk.log).
static bool seg_rounds_host();
static constexpr int64_t kSegPlainMax = 256;   // seg_add: plain adds up to this many
static int64_t seg_scan() {
  const char* e = getenv("DR_GRAD_SEG_SCAN");
  if (e) return (int64_t)atoll(e);
  return seg_rounds_host() ? (int64_t)4096 : (int64_t)0;
}
static int32_t seg_min() { return seg_rounds_host() ? 8 : 16; }

static int64_t zero_scan() {
  // read per call (host only, once per backward): tests switch it on around
  // one call.  Off by default: none of the measured workloads has exact-zero
  // terms (DIN's padding positions carry his_sum's gradient), where the scan
  // only adds a pass over every long run's terms (127 us at configs[3])
  const char* e = getenv("DR_GRAD_ZERO_SKIP");
  return (e && atoi(e) != 0) ? (int64_t)2048 : (int64_t)0;
}

// Long-run state (the workspace arrays of RowsWs, passed as one argument).
struct RowsLong {
  const uint32_t* skey;
  const int32_t* perm;
  const int32_t* ex;       // unfused: first-occurrence ranks (output index)
  const int32_t* base;
  int32_t* srow;           // per sorted position in a multi-position run: bag row (-1 invalid)
  float* smul;             //   weight, or the mean / sqrtn scale (1: none)
  float* sdiv;             //   bag_scale of a weighted mean / sqrtn
  const int32_t* longs;    // sorted head of each run longer than kRowsChunk
  const int32_t* nlong;
  int32_t* rlen;           // its length (rows_expand_kernel)
  int32_t* rfirst;         // its first piece item
  int32_t* items;          // pieces: (run, piece index)
  int32_t* nitems;
  uint64_t* gptr;
  float* gu;
  float* part;             // [item][dim] piece partials of multi-piece runs
  int64_t smax;            // piece length (serial_max())
  int64_t zscan;           // zero-scan runs longer than this (0: never)
  int32_t* cfirst;         // per long run: its first zero-scan chunk (-1: not scanned)
  int32_t* crun;           // per chunk: (run, chunk index)
  int32_t* nchunk;
  int32_t* ccnt;           // per chunk: its nonzero terms
  int32_t* kpos;           // [N] chunk k of run c0: nonzero positions at c0 + k*kRowsChunk ..
  int32_t* rnz;            // per long run: its nonzero terms (zero scan)
  float* zrow;             // 64 zeros (rows_expand_kernel): the term of an invalid bag
  int dma;                 // who takes the plain-sum runs (serial_dma()): 1 plain, 2 dma
  int32_t* rseg;           // per long run: its segment count (seg scan; -1: not scanned)
  int64_t sscan;           // seg-scan plain runs longer than this (0: never)
  int32_t segmin;          // walk a seg-scanned run by segments from this mean length
  int32_t srounds;         // segment walk in wave rounds (wave_rounds_walk)
};

// A zero-scanned run is walked compacted only when at most half its terms
// are nonzero (the same test in both serial kernels, so they split the runs
// between them exactly).
__device__ __forceinline__ bool run_sparse(const RowsLong& L, int i, int np, int64_t len) {
  return np == 1 && L.cfirst[i] >= 0 && L.rseg[i] < 0 && 2 * (int64_t)L.rnz[i] <= len;
}

// A seg-scanned run is walked by segments when they average at least kSegMin
// terms (every walker applies the same test, so they split the runs exactly).
__device__ __forceinline__ bool run_seg(const RowsLong& L, int i, int np, int64_t len) {
  return np == 1 && L.cfirst[i] >= 0 && L.rseg[i] >= 0 && (int64_t)L.segmin * L.rseg[i] <= len;
}

// Table of global position i (lane-varying; koff staged in LDS).
__device__ __forceinline__ int tab_of(const int64_t* koff, int T, int64_t i) {
  int lo = 0, hi = T - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (koff[mid] <= i)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

// The forward's row of global position i: position order (rec_t == 0), or
// the record-major [batch, T] rows of a one-hot training lookup
// (DR_LOOKUP_ROWS_RECORD: rows[b * T + t], written as whole lines in output
// order) -- position i = t * batch + b.
__device__ __forceinline__ int64_t rowsel_at(const int64_t* rowsel, int64_t i, int rec_t,
                                             int64_t rec_b) {
  if (!rec_t) return rowsel[i];
  const int64_t t = i / rec_b;
  return rowsel[(i - t * rec_b) * rec_t + t];
}

// (also zeroes the worklist / long-run counters: they are first used after
// the sort, two launches later)
__global__ void rows_keys_kernel(const int64_t* __restrict__ rowsel, int64_t N, int64_t row_limit,
                                 uint32_t sentinel, uint32_t* __restrict__ kin,
                                 int32_t* __restrict__ vin, int32_t* __restrict__ flags,
                                 int32_t* __restrict__ nlong, int32_t* __restrict__ nwork,
                                 int32_t* __restrict__ nitems, int32_t* __restrict__ nchunk,
                                 int rec_t, int64_t rec_b) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    *nlong = 0;
    *nwork = 0;
    *nitems = 0;
    *nchunk = 0;
  }
  if (i >= N) return;
  const int64_t r = rowsel_at(rowsel, i, rec_t, rec_b);
  // a negative row is an EV default served because the pool was exhausted
  // (RESOURCE_EXHAUSTED already latched by the resolve): no gradient row
  kin[i] = (r >= 0 && r < row_limit) ? (uint32_t)r : sentinel;
  vin[i] = (int32_t)i;
  if (flags) flags[i] = -1;
}

// v -= lr * g on one row of a var column (KvResourceSparseApplyGradientDescent,
// training_ali_ops.cc:1663: one fp32 product, one fp32 difference -- the
// build keeps -ffp-contract=off, as ev_apply_kernel's apply_one).  bf16 var
// rows (4 values = 8 B per lane chunk) are widened, updated and rounded to
// nearest even once, as ev_apply_kernel<OPT_SGD, 4, G, true>.
__device__ __forceinline__ float4 sgd4(float4 w, float4 g, float lr) {
  const float4 p = make_float4(lr * g.x, lr * g.y, lr * g.z, lr * g.w);
  return make_float4(w.x - p.x, w.y - p.y, w.z - p.z, w.w - p.w);
}
typedef unsigned int sg_u2 __attribute__((ext_vector_type(2)));
template <bool WB>
__device__ __forceinline__ float4 sgd_ld(const float* row, int c) {
  if constexpr (WB) {
    const sg_u2 v = __builtin_nontemporal_load(gp(reinterpret_cast<const sg_u2*>(row) + c));
    const float2 a = bf16x2_to_f2(v.x), b = bf16x2_to_f2(v.y);
    return make_float4(a.x, a.y, b.x, b.y);
  } else {
    return nt_load(reinterpret_cast<const float4*>(row) + c);
  }
}
template <bool WB>
__device__ __forceinline__ void sgd_st(float* row, int c, float4 w) {
  if constexpr (WB) {
    const sg_u2 v = {f2_to_bf16x2(w.x, w.y), f2_to_bf16x2(w.z, w.w)};
    __builtin_nontemporal_store(v, gp(reinterpret_cast<sg_u2*>(row) + c));
  } else {
    nt_store(w, reinterpret_cast<float4*>(row) + c);
  }
}
// Row u of table t += -lr * (the G-lane row gr); version stamped by lane 0.
template <int G, int CPL, bool WB>
__device__ __forceinline__ void sgd_row(const Row<4, G, CPL>& gr, void* pool, int64_t* version,
                                        int64_t u, int dim, float lr, int64_t gs, int lg, int dv) {
  float* row = static_cast<float*>(pool) + u * (int64_t)(WB ? dim / 2 : dim);
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int col = lg + c * G;
    if (col < dv) sgd_st<WB>(row, col, sgd4(sgd_ld<WB>(row, col), gr.v[c], lr));
  }
  if (version && lg == 0) version[u] = gs;
}

// Block-aggregated append (256-thread blocks, every thread of the block
// reaching it): one counter atomic per block instead of one per wave --
// a 1.7 M-position pass with many pushes made ~26 K atomics on one address
// (rows_heads 160 us per call on WDL's small-bucket columns).
__device__ __forceinline__ void work_push_block(bool push, int64_t p, int32_t* __restrict__ work,
                                                int32_t* __restrict__ nwork) {
  __shared__ int wcnt[4];
  __shared__ int bbase;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t m = __ballot(push);
  if (lane == 0) wcnt[wv] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    bbase = tot ? atomicAdd(nwork, tot) : 0;
  }
  __syncthreads();
  if (push) {
    int off = bbase;
    for (int w = 0; w < wv; ++w) off += wcnt[w];
    work[off + __popcll(m & lanemask_lt())] = (int32_t)p;
  }
}

// Two block-aggregated appends at once (same contract as work_push_block).
__device__ __forceinline__ void push2_block(bool pa, int32_t va, int32_t* __restrict__ la,
                                            int32_t* __restrict__ na, bool pb, int32_t vb,
                                            int32_t* __restrict__ lb, int32_t* __restrict__ nb) {
  __shared__ int wc[2][4];
  __shared__ int bb[2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t ma = __ballot(pa), mb = __ballot(pb);
  if (lane == 0) {
    wc[0][wv] = __popcll(ma);
    wc[1][wv] = __popcll(mb);
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const int x = threadIdx.x;
    const int tot = wc[x][0] + wc[x][1] + wc[x][2] + wc[x][3];
    bb[x] = tot ? atomicAdd(x ? nb : na, tot) : 0;
  }
  __syncthreads();
  if (pa) {
    int off = bb[0];
    for (int w = 0; w < wv; ++w) off += wc[0][w];
    la[off + __popcll(ma & lanemask_lt())] = va;
  }
  if (pb) {
    int off = bb[1];
    for (int w = 0; w < wv; ++w) off += wc[1][w];
    lb[off + __popcll(mb & lanemask_lt())] = vb;
  }
}

// The term of sorted position p of a multi-position run (feature-local
// position k of table descriptor d), for the long-run kernels: its bag row
// (-1: an invalid bag, a zero term, latched here) and factors -- smul = the
// weight (weighted) or the mean / sqrtn scale of its bag (1: none), sdiv =
// the weighted mean / sqrtn divisor -- the arithmetic of rows_work_kernel's
// scaled / wscaled, precomputed in the fully parallel classification pass so
// that the serial pass streams one contiguous index per position.
__device__ __forceinline__ void rows_term(const dr_pool_grad_desc& d, int64_t k, int64_t B,
                                          int64_t p, const RowsLong& L, int* st) {
  const int64_t r = d.seg ? d.seg[k * d.seg_stride] : k;
  const bool okr = r >= 0 && r < B;
  if (!okr) latch(st, DR_INVALID_ARGUMENT);
  float m = 1.f, q = 1.f;
  if (okr && d.weights) {
    m = d.weights[k];
    if (d.bag_scale) q = d.bag_scale[r];
  } else if (okr && d.combiner != DR_COMBINER_SUM && d.bag_off) {
    const int32_t cnt = d.bag_off[r + 1] - d.bag_off[r];
    if (cnt != 1)
      m = d.combiner == DR_COMBINER_SQRTN ? (float)(1.0 / sqrt((double)cnt))
                                          : (float)(1.0 / (double)cnt);
  }
  L.srow[p] = okr ? (int32_t)r : -1;
  L.smul[p] = m;
  L.sdiv[p] = q;
}

// Sorted order, lane per position: mark[i] = p (| 1 << 31 for a one-position
// run) at the run head's original position i; heads of runs of 2 ..
// kRowsChunk positions go to the worklist of rows_work_kernel, heads of
// longer runs to the long-run list; every position of a multi-position run
// records its term (rows_term).
__global__ __launch_bounds__(256) void rows_heads_kernel(RowsGroup g, int T, int64_t B,
                                                         const uint32_t* __restrict__ skey,
                                                         const int32_t* __restrict__ perm,
                                                         uint32_t sentinel,
                                                         int32_t* __restrict__ mark,
                                                         int32_t* __restrict__ work,
                                                         int32_t* __restrict__ nwork, RowsLong L,
                                                         int32_t* __restrict__ longs,
                                                         int32_t* __restrict__ nlong, int* st) {
  __shared__ dr_pool_grad_desc sd[DR_MAX_GROUP];
  __shared__ int64_t sk[DR_MAX_GROUP + 1];
  if (threadIdx.x < T) sd[threadIdx.x] = g.d[threadIdx.x];
  if (threadIdx.x <= T) sk[threadIdx.x] = g.koff[threadIdx.x];
  __syncthreads();
  const int64_t N = sk[T];
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool push = false, plong = false;
  if (p < N) {
    const int64_t pm = p > 0 ? p - 1 : 0, pn = p + 1 < N ? p + 1 : N - 1;
    const uint32_t u = skey[p], um = skey[pm], un = skey[pn];
    const int32_t i = perm[p], im = perm[pm], in = perm[pn];
    const int t = tab_of(sk, T, i);
    const bool valid = u != sentinel;
    const bool head = valid && (p == 0 || um != u || tab_of(sk, T, im) != t);
    const bool last = p + 1 >= N || un != u || tab_of(sk, T, in) != t;
    if (head) mark[i] = (int32_t)p | (last ? (int32_t)0x80000000 : 0);
    if (valid && !(head && last)) {
      rows_term(sd[t], i - sk[t], B, p, L, st);
      if (head) {
        const int64_t q = p + kRowsChunk;
        plong = q < N && skey[q] == u && tab_of(sk, T, perm[q]) == t;
        push = !plong;
      }
    }
  }
  push2_block(push, (int32_t)p, work, nwork, plong, (int32_t)p, longs, nlong);
}

// Fused SGD, sorted order, lane per position (dr_ev_pool_grad_rows_apply_sgd):
// the run classification of rows_heads_kernel, and a one-position run whose
// gradient needs no arithmetic -- the rows the unfused backward hands on by
// address (rows_emit_kernel's rule) -- is applied right here: v -= lr * (0 +
// g) read from the pooled gradient, the same bytes and roundings as
// ev_apply_kernel on that address.  Runs of 2 .. kRowsChunk positions and
// the other one-position runs go to rows_work_kernel's worklist, longer runs
// to the long-run list (rows_heads_kernel's rule).  No mark, scan or emit:
// the optimizer is the gradient's only consumer, so the IndexedSlices order
// (first occurrence) is never formed.
template <int G, bool WB>
__global__ __launch_bounds__(256) void rows_sgd_kernel(RowsGroup g, RowsSgd sg, int T, int64_t B,
                                                       const uint32_t* __restrict__ skey,
                                                       const int32_t* __restrict__ perm,
                                                       uint32_t sentinel, int dim,
                                                       int32_t* __restrict__ work,
                                                       int32_t* __restrict__ nwork, RowsLong L,
                                                       int32_t* __restrict__ longs,
                                                       int32_t* __restrict__ nlong, int* st) {
  __shared__ dr_pool_grad_desc sd[DR_MAX_GROUP];
  __shared__ int64_t sk[DR_MAX_GROUP + 1];
  __shared__ void* spool[DR_MAX_GROUP];
  __shared__ int64_t* sver[DR_MAX_GROUP];
  if (threadIdx.x < T) {
    sd[threadIdx.x] = g.d[threadIdx.x];
    spool[threadIdx.x] = sg.pool[threadIdx.x];
    sver[threadIdx.x] = sg.version[threadIdx.x];
  }
  if (threadIdx.x <= T) sk[threadIdx.x] = g.koff[threadIdx.x];
  __syncthreads();
  const int64_t N = sk[T];
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool push = false, plong = false, direct = false;
  int64_t u = -1;
  uint64_t ga = 0;
  int t = 0;
  if (p < N) {
    const int64_t pm = p > 0 ? p - 1 : 0, pn = p + 1 < N ? p + 1 : N - 1;
    const uint32_t uk = skey[p], um = skey[pm], un = skey[pn];
    const int32_t i = perm[p], im = perm[pm], in = perm[pn];
    t = tab_of(sk, T, i);
    const bool valid = uk != sentinel;
    const bool head = valid && (p == 0 || um != uk || tab_of(sk, T, im) != t);
    const bool last = p + 1 >= N || un != uk || tab_of(sk, T, in) != t;
    if (head && last) {
      const dr_pool_grad_desc& d = sd[t];
      const int64_t k = i - sk[t];
      const int64_t r = d.seg ? d.seg[k * d.seg_stride] : k;
      const bool okr = r >= 0 && r < B;
      const int mode = d.combiner == DR_COMBINER_SUM ? 0 : 1;
      bool dfr = okr && !d.weights;
      if (dfr && mode != 0) dfr = !d.bag_off || d.bag_off[r + 1] - d.bag_off[r] == 1;
      if (dfr) {
        direct = true;
        u = (int64_t)uk;
        ga = (uint64_t)(uintptr_t)(d.top_grad + r * d.top_stride) | (mode == 0 ? 1u : 0u);
      } else {
        push = true;   // (an invalid bag latches in rows_work_kernel)
      }
    } else if (valid) {
      rows_term(sd[t], i - sk[t], B, p, L, st);
      if (head) {
        const int64_t q = p + kRowsChunk;
        plong = q < N && skey[q] == uk && tab_of(sk, T, perm[q]) == t;
        push = !plong;
      }
    }
  }
  push2_block(push, (int32_t)p, work, nwork, plong, (int32_t)p, longs, nlong);
  if (!__ballot(direct)) return;   // wave-uniform
  // the wave's direct rows, P at a time, U batches of loads in flight
  constexpr int P = 64 / G, U = 4;
  const int lane = threadIdx.x & 63;
  const int sub = lane / G, lg = lane % G;
  const int dv = dim / 4;
  const int64_t stride = WB ? dim / 2 : dim;
  const float lr = sg.lr;
  for (int k0 = 0; k0 < 64; k0 += P * U) {
    int64_t rq[U];
    const float4* gq[U];
    float* wq[U];
    bool zq[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int k = k0 + q * P + sub;
      rq[q] = __shfl(u, k, 64);
      const uint64_t a = (uint64_t)__shfl((long long)ga, k, 64);
      const int tq = __shfl(t, k, 64);
      const bool ok = rq[q] >= 0;
      zq[q] = a & 1;
      // always-valid pointers (a skipped row reads table 0's row 0): the
      // loads of all U rows issue back to back (dr_rows.h load_row_u)
      gq[q] = reinterpret_cast<const float4*>(ok ? (uintptr_t)(a & ~(uint64_t)1)
                                                 : (uintptr_t)sd[0].top_grad);
      wq[q] = static_cast<float*>(spool[ok ? tq : 0]) + (ok ? rq[q] : 0) * stride;
      if (ok && lg == 0 && sver[tq]) sver[tq][rq[q]] = sg.gs;
    }
    for (int c = lg; c < dv; c += G) {
      float4 gv[U], w[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        gv[q] = nt_load(gq[q] + c);
        w[q] = sgd_ld<WB>(wq[q], c);
      }
#pragma unroll
      for (int q = 0; q < U; ++q) {
        if (rq[q] < 0) continue;
        if (zq[q]) gv[q] = vadd(vzero<float4>(), gv[q]);
        sgd_st<WB>(wq[q], c, sgd4(w[q], gv[q], lr));
      }
    }
  }
}

// Position order: unique ids in first-occurrence order per table, U_t, the
// scan base of every table, and the gradient of each one-position run: by
// address when its value needs no arithmetic (sum, or mean/sqrtn of a
// one-id bag, unweighted: grad_ptr[o] = the pooled-grad row, bit 0 = "add
// +0.0f", the 0 + x of the reference's unsorted sum), else a worklist
// entry.  All-distinct sum lookups (the Criteo shape) leave the worklist
// empty and the backward moves no embedding-row bytes at all.
__global__ __launch_bounds__(256) void rows_emit_kernel(
    RowsGroup g, int T, int64_t B, const int64_t* __restrict__ keys,
    const int32_t* __restrict__ mark, const int32_t* __restrict__ ex,
    const int64_t* __restrict__ total, int defer, int64_t* __restrict__ uniq_out,
    int64_t* __restrict__ num_unique, int32_t* __restrict__ base, uint64_t* __restrict__ gptr,
    int32_t* __restrict__ work, int32_t* __restrict__ nwork, const int64_t* __restrict__ rowsel,
    int64_t* __restrict__ urows, int* st, int dim, float* __restrict__ gu, int rec_t) {
  __shared__ dr_pool_grad_desc sd[DR_MAX_GROUP];
  if (threadIdx.x < T) sd[threadIdx.x] = g.d[threadIdx.x];
  __syncthreads();
  const int64_t N = g.koff[T];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= T) {   // base[t] = first-occurrence count before table t
    const int64_t o = g.koff[i];
    base[i] = o < N ? ex[o] : (int32_t)*total;
  }
  if (blockIdx.x == 0 && threadIdx.x < T) {
    const int t = threadIdx.x;
    const int64_t a = g.koff[t], b = g.koff[t + 1];
    const int64_t ba = a < N ? ex[a] : *total;
    const int64_t bb = b < N ? ex[b] : *total;
    num_unique[t] = bb - ba;
  }
  const int32_t mk = i < N ? mark[i] : -1;
  bool push = false;
  if (mk != -1) {
    const int t = table_of(g.koff, T, i, (int64_t)blockIdx.x * blockDim.x);
    const int64_t a = g.koff[t];
    const int64_t o = a + ex[i] - ex[a];
    uniq_out[o] = keys[i];
    if (urows) urows[o] = rowsel_at(rowsel, i, rec_t, B);  // the row the forward resolved
    if (mk < 0) {   // one-position run
      const dr_pool_grad_desc& d = sd[t];
      const int64_t k = i - a;
      const int64_t r = d.seg ? d.seg[k * d.seg_stride] : k;
      const bool okr = r >= 0 && r < B;
      const int mode = d.combiner == DR_COMBINER_SUM ? 0 : 1;
      bool dfr = defer && okr && !d.weights;
      if (dfr && mode != 0) dfr = !d.bag_off || d.bag_off[r + 1] - d.bag_off[r] == 1;
      if (dfr) {
        gptr[o] = (uint64_t)(uintptr_t)(d.top_grad + r * d.top_stride) | (mode == 0 ? 1u : 0u);
      } else if (dim <= 4 && okr) {
        // narrow rows (wide / linear tables): the run's value formed right
        // here, with rows_work_kernel's single-row arithmetic (the 0 + x of
        // a zero-started sum, the mean / sqrtn scale, weights / bag scale),
        // instead of one worklist entry (one contended counter atomic per
        // wave and a lane group) per position
        const int m3 = d.combiner == DR_COMBINER_SUM ? 0 : (d.combiner == DR_COMBINER_MEAN ? 1 : 2);
        const bool zero_start = m3 == 0 || d.weights;
        float sc = 1.f, q = 1.f, w = 1.f;
        if (d.weights) {
          if (d.bag_scale) q = d.bag_scale[r];
          w = d.weights[k];
        } else if (m3 != 0) {
          const int32_t cnt = d.bag_off ? d.bag_off[r + 1] - d.bag_off[r] : 1;
          if (cnt != 1)
            sc = m3 == 2 ? (float)(1.0 / sqrt((double)cnt)) : (float)(1.0 / (double)cnt);
        }
        float* dst = gu + o * (int64_t)dim;
        for (int c = 0; c < dim; ++c) {
          float y = d.top_grad[r * d.top_stride + c];
          if (d.weights) {
            if (d.bag_scale) y = y / q;
            y = y * w;
          } else if (m3 != 0 && sc != 1.f) {
            y = y * sc;
          }
          dst[c] = zero_start ? 0.f + y : y;
        }
        gptr[o] = (uint64_t)(uintptr_t)dst;
      } else {
        push = true;   // (an invalid bag latches there)
      }
    }
  }
  work_push_block(push, (int64_t)(mk & 0x7FFFFFFF), work, nwork);
}

// G lanes per worklist entry (a sorted run head c0 of a run of at most
// kRowsChunk positions, or a one-position run whose value needs arithmetic):
// the run summed in ascending position order into grad_unique[o].
//
// SGD (the fused dr_ev_pool_grad_rows_apply_sgd): the run's sum is applied
// to its var row (v -= lr * sum) instead of stored.
template <int VEC, int G, int CPL, bool W, bool SGD = false, bool WB = false>
__global__ __launch_bounds__(256) void rows_work_kernel(
    RowsGroup g, int T, int64_t B, const uint32_t* __restrict__ skey,
    const int32_t* __restrict__ perm, const int32_t* __restrict__ ex,
    const int32_t* __restrict__ base, int dim, const int32_t* __restrict__ work,
    const int32_t* __restrict__ nwork, uint64_t* __restrict__ gptr, float* __restrict__ gu, int* st,
    RowsSgd sg) {
  const int nw = *nwork;
  if ((int64_t)blockIdx.x * (256 / G) >= nw) return;   // block-uniform (empty list: one load)
  __shared__ dr_pool_grad_desc sd[DR_MAX_GROUP];
  __shared__ int64_t sk[DR_MAX_GROUP + 1];
  __shared__ int32_t sb[DR_MAX_GROUP + 1];
  __shared__ void* spool[SGD ? DR_MAX_GROUP : 1];
  __shared__ int64_t* sver[SGD ? DR_MAX_GROUP : 1];
  if (threadIdx.x < T) {
    sd[threadIdx.x] = g.d[threadIdx.x];
    if constexpr (SGD) {
      spool[threadIdx.x] = sg.pool[threadIdx.x];
      sver[threadIdx.x] = sg.version[threadIdx.x];
    }
  }
  if (threadIdx.x <= T) {
    sk[threadIdx.x] = g.koff[threadIdx.x];
    if constexpr (!SGD) sb[threadIdx.x] = base[threadIdx.x];
  }
  __syncthreads();
  constexpr int GPB = 256 / G;
  // positions of a run fetched per step: the serial sum's loads are issued
  // CH at a time -- deeper for scalar rows (one register per row chunk), so
  // a 256-position run is 16 dependent steps instead of 32
  constexpr int CH = VEC * CPL <= 1 ? 16 : kRowsChain;
  const int64_t N = sk[T];
  const int lg = threadIdx.x % G;
  const int dv = dim / VEC;
  using R = Row<VEC, G, CPL>;
  using V = typename VecT<VEC>::T;
  auto scaled = [&](R& y, const dr_pool_grad_desc& d, int mode, int64_t r) {
    if (mode == 0) return;
    const int32_t cnt = (r >= 0 && d.bag_off) ? d.bag_off[r + 1] - d.bag_off[r] : 1;
    if (cnt != 1) {
      const float sc = mode == 2 ? (float)(1.0 / sqrt((double)cnt)) : (float)(1.0 / (double)cnt);
#pragma unroll
      for (int c = 0; c < CPL; ++c) y.v[c] = vmul(y.v[c], sc);
    }
  };
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
  for (int64_t e = (int64_t)blockIdx.x * GPB + threadIdx.x / G; e < nw;
       e += (int64_t)gridDim.x * GPB) {
    const int64_t c0 = work[e];
    const uint32_t u = skey[c0];
    const int32_t pc = perm[c0];
    const int t = tab_of(sk, T, pc);
    const int64_t lim = c0 + kRowsChunk < N ? c0 + kRowsChunk : N;
    // a one-position run (the common case under uniform keys when the
    // run's value needs arithmetic, e.g. unaligned rows): one row load
    // instead of a CH-position speculative chunk
    const bool single =
        c0 + 1 >= N || skey[c0 + 1] != u || tab_of(sk, T, perm[c0 + 1]) != t;
    const dr_pool_grad_desc& d = sd[t];
    const int mode = d.combiner == DR_COMBINER_SUM ? 0 : (d.combiner == DR_COMBINER_MEAN ? 1 : 2);
    const bool zero_start = mode == 0 || (W && d.weights);
    R acc;
#pragma unroll
    for (int c = 0; c < CPL; ++c) acc.v[c] = vzero<V>();
    bool fresh = !zero_start;
    const float* tg = d.top_grad;
    const int64_t ts = d.top_stride;
    const int64_t* segp = d.seg;
    const int64_t sst = d.seg_stride;
    const int64_t kt0 = sk[t];
    const int64_t nnz_t = d.nnz;
    bool cbad = false;
    if (single) {
      const int64_t k = (int64_t)perm[c0] - kt0;
      int64_t r = segp ? segp[k * sst] : k;
      const bool okr = (r >= 0) & (r < B);
      cbad = !okr;
      r = okr ? r : -1;
      R y;
      load_row_u<VEC, G, CPL>(y, tg + (okr ? r : 0) * ts, lg, dv);
      if (r < 0) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) y.v[c] = vzero<V>();
      }
      if (W && d.weights)
        wscaled(y, d, r, k);
      else
        scaled(y, d, mode, r);
      if (fresh)
        acc = y;
      else
        acc_add(acc, y);
    }
    for (int64_t p = c0; !single && p < lim; p += CH) {
      R y[CH];
      int64_t ry[CH];
      int64_t ky[W ? CH : 1];
      bool ok[CH];
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int64_t pj = p + j < N ? p + j : N - 1;
        const int64_t k = (int64_t)perm[pj] - kt0;
        // positions of one (table, row) are contiguous; a position of the same
        // row in another table has k outside [0, nnz_t)
        ok[j] = (p + j < lim) & (skey[pj] == u) & (k >= 0) & (k < nnz_t);
        ry[j] = ok[j] ? k : 0;
        if (W) ky[W ? j : 0] = ry[j];
      }
      if (segp) {
#pragma unroll
        for (int j = 0; j < CH; ++j) ry[j] = segp[ry[j] * sst];
      }
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const bool okr = (ry[j] >= 0) & (ry[j] < B);
        cbad |= ok[j] & !okr;
        ry[j] = okr ? ry[j] : -1;
        load_row_u<VEC, G, CPL>(y[j], tg + (okr ? ry[j] : 0) * ts, lg, dv);
      }
      // ok[] is a prefix (a run's positions are contiguous): predicated, not
      // an early exit, so the loop unrolls and y[] stays in registers
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        if (ok[j]) {
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
      }
      if (!ok[CH - 1]) break;
    }
    if (cbad) latch(st, DR_INVALID_ARGUMENT);
    if constexpr (SGD) {
      static_assert(!SGD || VEC == 4, "fused SGD takes 16-byte rows");
      sgd_row<G, CPL, WB>(acc, spool[t], sver[t], (int64_t)u, dim, sg.lr, sg.gs, lg, dv);
    } else {
      const int64_t o = kt0 + (int64_t)ex[pc] - sb[t];
      float* dst = gu + o * (int64_t)dim;
      store_row<VEC, G, CPL>(acc, dst, lg, dv);
      if (lg == 0) gptr[o] = (uint64_t)(uintptr_t)dst;
    }
  }
}

// ---- long runs (more than kRowsChunk positions) ------------------------------

// Columns c, c + 1 (c + 1 < dim or ignored) of a finished run: the
// IndexedSlices row o (unfused), or v -= lr * sum on the var row u of table
// t (SGD: one fp32 product, one fp32 difference per value, as sgd4; bf16 rows
// widened, updated and rounded once per packed pair, as sgd_ld / sgd_st).
template <bool SGD, bool WB>
__device__ __forceinline__ void rows_fin_pair(const RowsSgd& sg, int t, uint32_t u, int64_t o,
                                              int dim, int c, float a, float b, float* gu) {
  if constexpr (SGD) {
    if constexpr (WB) {
      uint32_t* row = static_cast<uint32_t*>(sg.pool[t]) + (int64_t)u * (dim / 2);
      const float2 w = bf16x2_to_f2(row[c / 2]);
      const float pa = sg.lr * a, pb = sg.lr * b;
      row[c / 2] = f2_to_bf16x2(w.x - pa, w.y - pb);
    } else {
      float* row = static_cast<float*>(sg.pool[t]) + (int64_t)u * dim;
      const float pa = sg.lr * a;
      row[c] = row[c] - pa;
      if (c + 1 < dim) {
        const float pb = sg.lr * b;
        row[c + 1] = row[c + 1] - pb;
      }
    }
  } else {
    float* dst = gu + o * (int64_t)dim;
    dst[c] = a;
    if (c + 1 < dim) dst[c + 1] = b;
  }
}

// Once per finished run: the steps_to_live version (SGD) or the by-address
// gradient pointer of IndexedSlices row o (unfused).
template <bool SGD>
__device__ __forceinline__ void rows_fin_run(const RowsSgd& sg, int t, uint32_t u, int64_t o,
                                             int dim, const RowsLong& L) {
  if constexpr (SGD) {
    if (sg.version[t]) sg.version[t][u] = sg.gs;
  } else {
    L.gptr[o] = (uint64_t)(uintptr_t)(L.gu + o * (int64_t)dim);
  }
}

// Is sorted position q in the run of (u, table slice [lo, hi) of positions)?
__device__ __forceinline__ bool in_run(const RowsLong& L, int64_t N, int64_t q, uint32_t u,
                                       int64_t lo, int64_t hi) {
  const int64_t qc = q < N ? q : N - 1;
  const uint32_t kq = L.skey[qc];
  const int32_t pq = L.perm[qc];
  return (q < N) & (kq == u) & (pq >= lo) & (pq < hi);
}

// One block per long run: its end (two rounds of parallel probes -- every
// kRowsChunk-th position past the head, then the 256 positions of the window
// the run ends in: a run's positions are contiguous, so in_run is a prefix),
// then its pieces of serial_max() positions as work items.
__global__ __launch_bounds__(256) void rows_expand_kernel(RowsGroup g, int T, RowsLong L) {
  if (blockIdx.x == 0 && threadIdx.x < 64) L.zrow[threadIdx.x] = 0.f;
  __shared__ int64_t sk[DR_MAX_GROUP + 1];
  __shared__ int smin;
  __shared__ int sfirst;
  if (threadIdx.x <= T) sk[threadIdx.x] = g.koff[threadIdx.x];
  __syncthreads();
  const int64_t N = sk[T];
  const int n = *L.nlong;
  for (int i = blockIdx.x; i < n; i += gridDim.x) {   // block-uniform
    const int64_t c0 = L.longs[i];
    const uint32_t u = L.skey[c0];
    const int t = tab_of(sk, T, L.perm[c0]);
    const int64_t lo = sk[t], hi = sk[t + 1];
    int64_t a = c0;   // a position known to be in the run
    int64_t w0 = 0;   // last in-run probe of the coarse round
    for (;;) {        // one probe per thread: rounds of 256 x kRowsChunk positions
      if (threadIdx.x == 0) smin = 0x7FFFFFFF;
      __syncthreads();
      const int m = 1 + threadIdx.x;
      if (!in_run(L, N, a + kRowsChunk * (int64_t)m, u, lo, hi)) atomicMin(&smin, m);
      __syncthreads();
      const int mm = smin;
      __syncthreads();
      if (mm != 0x7FFFFFFF) {
        w0 = a + kRowsChunk * (int64_t)(mm - 1);
        break;
      }
      a += kRowsChunk * 256;   // (runs of more than 2^16 positions: another round)
    }
    if (threadIdx.x == 0) smin = 0x7FFFFFFF;
    __syncthreads();
    // the end lies in (w0, w0 + kRowsChunk]: one probe per thread
    if (!in_run(L, N, w0 + 1 + threadIdx.x, u, lo, hi)) atomicMin(&smin, (int)threadIdx.x);
    __syncthreads();
    const int64_t len = w0 + 1 + smin - c0;
    const int np = (int)((len + L.smax - 1) / L.smax);
    // zero-scan chunks: one-piece runs of a zero-started chain (sum combiner
    // or weighted: rows_serial_kernel's fresh start is then 0 + x_0)
    const bool zs = g.d[t].combiner == DR_COMBINER_SUM || g.d[t].weights != nullptr;
    const bool zscan = np == 1 && zs && L.zscan > 0 && len > L.zscan;
    // plain-sum runs not zero-scanned: segment scan (seg_scan())
    const bool plain = g.d[t].combiner == DR_COMBINER_SUM && g.d[t].weights == nullptr;
    const bool sscan = !zscan && np == 1 && plain && L.sscan > 0 && len > L.sscan;
    const int nch = (zscan || sscan) ? (int)((len + kRowsChunk - 1) / kRowsChunk) : 0;
    if (threadIdx.x == 0) {
      const int fi = atomicAdd(L.nitems, np);
      L.rlen[i] = (int32_t)len;
      L.rfirst[i] = fi;
      sfirst = fi;
      const int cf = nch ? atomicAdd(L.nchunk, nch) : -1;
      L.cfirst[i] = cf;
      L.rnz[i] = 0;
      L.rseg[i] = sscan ? 0 : -1;
      smin = cf;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < np; k += 256) {
      L.items[2 * (sfirst + k)] = i;
      L.items[2 * (sfirst + k) + 1] = k;
    }
    const int cf = smin;
    for (int k = threadIdx.x; k < nch; k += 256) {
      L.crun[2 * (cf + k)] = i;
      L.crun[2 * (cf + k) + 1] = k;
    }
    __syncthreads();   // smin / sfirst are rewritten by the next run
  }
}

// Zero scan of the long runs' chunks (zero_scan()): one block per chunk of
// kRowsChunk positions, one thread per position computes its term exactly as
// rows_serial_kernel stages it (bag row or zero, weights / mean scale) and
// tests every column for != 0; the chunk's nonzero positions are compacted in
// ascending order into kpos[chunk start ..] and counted in ccnt.
template <int VEC>
__global__ __launch_bounds__(256) void rows_nz_kernel(RowsGroup g, int T, int dim, RowsLong L) {
  __shared__ int64_t sk[DR_MAX_GROUP + 1];
  __shared__ int wc[4];
  using V = typename VecT<VEC>::T;
  if (threadIdx.x <= T) sk[threadIdx.x] = g.koff[threadIdx.x];
  __syncthreads();
  const int n = *L.nchunk;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int c = blockIdx.x; c < n; c += gridDim.x) {   // block-uniform
    const int i = L.crun[2 * c], k = L.crun[2 * c + 1];
    if (L.rseg[i] >= 0) continue;   // a seg-scanned run's chunk (rows_seg_kernel)
    const int64_t c0 = L.longs[i];
    const int64_t len = L.rlen[i];
    const int64_t cs = c0 + (int64_t)k * kRowsChunk;
    const int64_t ce = c0 + len < cs + kRowsChunk ? c0 + len : cs + kRowsChunk;
    const int t = tab_of(sk, T, L.perm[c0]);
    const dr_pool_grad_desc& d = g.d[t];
    const bool wt = d.weights != nullptr;
    const bool qs = wt && d.bag_scale;
    const bool ms = !wt && d.combiner != DR_COMBINER_SUM;
    const int64_t q = cs + tid;
    bool nz = false;
    if (q < ce) {
      const int32_t rq = L.srow[q];
      const float mf = (wt || ms) ? L.smul[q] : 1.f;
      const float df = qs ? L.sdiv[q] : 1.f;
      const float* row = d.top_grad + (int64_t)(rq >= 0 ? rq : 0) * d.top_stride;
      for (int cv = 0; cv * VEC < dim; ++cv) {
        V x = rq >= 0 ? gld(reinterpret_cast<const V*>(row) + cv) : vzero<V>();
        if (wt) {
          if (qs) x = vdiv(x, df);
          x = vmul(x, mf);
        } else if (ms && mf != 1.f) {
          x = vmul(x, mf);
        }
        if constexpr (VEC == 4)
          nz |= (x.x != 0.f) | (x.y != 0.f) | (x.z != 0.f) | (x.w != 0.f);
        else
          nz |= x != 0.f;
      }
    }
    const uint64_t bm = __ballot(nz);
    if (lane == 0) wc[wv] = __popcll(bm);
    __syncthreads();
    int before = 0;
    for (int w = 0; w < wv; ++w) before += wc[w];
    if (nz) L.kpos[cs + before + __popcll(bm & lanemask_lt())] = (int32_t)q;
    if (tid == 0) {
      const int nzc = wc[0] + wc[1] + wc[2] + wc[3];
      L.ccnt[c] = nzc;
      if (nzc) atomicAdd(&L.rnz[i], nzc);
    }
    __syncthreads();   // wc is rewritten by the next chunk
  }
}

// Segment scan of the seg-scanned runs' chunks (seg_scan()): one block per
// chunk of kRowsChunk positions, one thread per position q: q ends a segment
// when it is the run's last position or its term differs, bitwise in any
// column, from position q + 1's (the same bag row always gives the same
// term; an invalid bag's term is the zero row).  The chunk's segment ends are
// compacted in ascending order into kpos[chunk start ..], counted in ccnt
// and summed per run into rseg.
template <int VEC>
__global__ __launch_bounds__(256) void rows_seg_kernel(RowsGroup g, int T, int dim, RowsLong L) {
  __shared__ int64_t sk[DR_MAX_GROUP + 1];
  __shared__ int wc[4];
  using V = typename VecT<VEC>::T;
  if (threadIdx.x <= T) sk[threadIdx.x] = g.koff[threadIdx.x];
  __syncthreads();
  const int n = *L.nchunk;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int c = blockIdx.x; c < n; c += gridDim.x) {   // block-uniform
    const int i = L.crun[2 * c], k = L.crun[2 * c + 1];
    if (L.rseg[i] < 0) continue;   // a zero-scanned run's chunk (rows_nz_kernel)
    const int64_t c0 = L.longs[i];
    const int64_t len = L.rlen[i];
    const int64_t cs = c0 + (int64_t)k * kRowsChunk;
    const int64_t ce = c0 + len < cs + kRowsChunk ? c0 + len : cs + kRowsChunk;
    const int t = tab_of(sk, T, L.perm[c0]);
    const dr_pool_grad_desc& d = g.d[t];
    const int64_t q = cs + tid;
    bool end = false;
    if (q < ce) {
      end = q + 1 >= c0 + len;
      if (!end) {
        const int32_t r0 = L.srow[q], r1 = L.srow[q + 1];
        if (r0 != r1) {
          const float* p0 = d.top_grad + (int64_t)(r0 >= 0 ? r0 : 0) * d.top_stride;
          const float* p1 = d.top_grad + (int64_t)(r1 >= 0 ? r1 : 0) * d.top_stride;
          for (int cv = 0; cv * VEC < dim && !end; ++cv) {
            const V x0 = r0 >= 0 ? gld(reinterpret_cast<const V*>(p0) + cv) : vzero<V>();
            const V x1 = r1 >= 0 ? gld(reinterpret_cast<const V*>(p1) + cv) : vzero<V>();
            if constexpr (VEC == 4)
              end = (__float_as_uint(x0.x) != __float_as_uint(x1.x)) ||
                    (__float_as_uint(x0.y) != __float_as_uint(x1.y)) ||
                    (__float_as_uint(x0.z) != __float_as_uint(x1.z)) ||
                    (__float_as_uint(x0.w) != __float_as_uint(x1.w));
            else if constexpr (VEC == 2)
              end = (__float_as_uint(x0.x) != __float_as_uint(x1.x)) ||
                    (__float_as_uint(x0.y) != __float_as_uint(x1.y));
            else
              end = __float_as_uint(x0) != __float_as_uint(x1);
          }
        }
      }
    }
    const uint64_t bm = __ballot(end);
    if (lane == 0) wc[wv] = __popcll(bm);
    __syncthreads();
    int before = 0;
    for (int w = 0; w < wv; ++w) before += wc[w];
    if (end) L.kpos[cs + before + __popcll(bm & lanemask_lt())] = (int32_t)q;
    if (tid == 0) {
      const int ns = wc[0] + wc[1] + wc[2] + wc[3];
      L.ccnt[c] = ns;
      if (ns) atomicAdd(&L.rseg[i], ns);
    }
    __syncthreads();   // wc is rewritten by the next chunk
  }
}

// Inclusive prefix sum over the 64 lanes of a wave: DPP row shifts inside
// each 16-lane row (out-of-row sources read 0), then the row totals added
// from lanes 15 / 31 / 47 by readlane (VALU + SALU, no LDS permute).
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
  const int r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31),
            r2 = __builtin_amdgcn_readlane(v, 47);
  const int row = lane >> 4;
  return v + (row >= 1 ? r0 : 0) + (row >= 2 ? r1 : 0) + (row >= 3 ? r2 : 0);
}

// k adds of x to acc, exactly: the plain adds themselves for a short
// segment (one dependent v_add_f32 each, ~8.5 cycles -- a DIN segment's ~50
// cost less than rep_add's double-precision closed form, ~2-4 k cycles of
// dependent instructions), rep_add for a long one.
__device__ __forceinline__ float seg_add(float acc, float x, int64_t k) {
  if (k > kSegPlainMax) return rep_add(acc, x, k);
  for (int q = 0; q < (int)k; ++q) acc = acc + x;
  return acc;
}

// One column's segments [0, nv) walked one at a time by a wave, every value
// wave-uniform (readfirstlane): per segment of k terms the first two adds
// on the fp32 adder, then the other k - 2 in closed form when the sum stays
// on one grid (dr_repadd.h seg_walk2 / seg_tail_fits: a few scalar integer
// ops; 93-97 % of DIN's padding segments), else plainly.  The next
// segment's term and end are read from LDS while this one is added.
__device__ __forceinline__ float serial_seg_walk(float acc, const float* sp, const int32_t* qe,
                                                int nv_, int64_t pe0) {
  const int nv = __builtin_amdgcn_readfirstlane(nv_);
  int32_t pe = __builtin_amdgcn_readfirstlane((int32_t)pe0);
  float a = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(acc)));
  float xv = sp[0];
  int32_t qv = qe[0];
  for (int e = 0; e < nv; ++e) {
    const float x = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(xv)));
    const int32_t q = __builtin_amdgcn_readfirstlane(qv);
    if (e + 1 < nv) {
      xv = sp[e + 1];
      qv = qe[e + 1];
    }
    const int32_t k = q - pe;
    pe = q;
    const float a1 = a + x;
    if (k == 1) {
      a = a1;
      continue;
    }
    const float a2 = a1 + x;
    if (k == 2) {
      a = a2;
      continue;
    }
    uint32_t bk;
    const uint32_t b0 = __builtin_amdgcn_readfirstlane(__float_as_uint(a));
    const uint32_t b1 = __builtin_amdgcn_readfirstlane(__float_as_uint(a1));
    const uint32_t b2 = __builtin_amdgcn_readfirstlane(__float_as_uint(a2));
    if (seg_tail_fits(b0, b1, b2, k - 2, &bk)) {
      a = __uint_as_float(bk);
      continue;
    }
    a = a2;
    if (k - 2 > kSegPlainMax)
      a = rep_add(a, x, k - 2);
    else
      for (int j = 0; j < k - 2; ++j) a = a + x;
  }
  return a;
}

// One column's segments [0, nv) walked by a whole wave in rounds
// (dr_repadd.h "many segments at once"): each round, lane l takes segment
// i + l -- its term's step on the current sum's grid, an exclusive prefix of
// k * D over the lanes, whether its adds stay on the grid from there -- and
// the wave moves the sum past every segment before the first lane that does
// not fit in one step; that segment is added exactly by rep_add and the next
// round starts on the new grid.  A zero / subnormal sum: one rep_add.
// sp: the column's terms, qe: segment end positions (LDS), pe0: the end of
// the segment before the first.  Bit-equal to rep_add segment by segment.
#ifdef DR_SEG_DEBUG
__device__ unsigned long long g_dbg[4096][3];   // (measurement build) per wave: rounds, rep_add, walk cycles
#endif
__device__ __noinline__ float wave_rounds_walk(float acc, const float* sp, const int32_t* qe, int nv,
                                               int64_t pe0, int lane) {
  int i = 0;
  int64_t pe = pe0;
#ifdef DR_SEG_DEBUG
  int nr = 0;
  uint64_t t_rep = 0;
  const uint64_t t_all = clock64();
#endif
  while (i < nv) {   // wave-uniform
#ifdef DR_SEG_DEBUG
    ++nr;
#endif
    SegGrid g;
    int64_t a;
    if (!seg_grid_of(acc, &g, &a)) {
      const int64_t q = qe[i];
      acc = seg_add(acc, sp[i], q - pe);
      pe = q;
      ++i;
      continue;
    }
    const int j = i + lane;
    const bool in = j < nv;
    const float x = in ? sp[j] : 0.f;
    const int32_t q = in ? qe[j] : 0;
    const int32_t qp = lane == 0 ? (int32_t)pe : (in ? qe[j - 1] : 0);
    const int32_t k = in ? q - qp : 0;
    const SegTerm t = seg_grid_term(g, x);
    // the lane's move k * D, clamped to +-(2^24 + 1) ulps: a clamped lane
    // leaves the binade itself (its own fits test below uses k * D
    // unclamped), so it or an earlier lane is the first stop and every prefix
    // before it is exact; 64 clamped values cannot overflow int32
    int64_t c64 = (in && t.ok) ? (int64_t)k * t.D : 0;
    c64 = c64 > 0x1000001 ? 0x1000001 : (c64 < -0x1000001 ? -0x1000001 : c64);
    const int c = (int)c64;
    const int incl = wave_incl_scan(c, lane);
    const int excl = incl - c;
    const bool stop = !in || !seg_grid_fits(a + excl, k, t);
    const uint64_t sm = __ballot(stop);
    const int f = sm ? __builtin_ctzll(sm) : 64;   // segments i .. i + f - 1 fit (wave-uniform)
    const int64_t af = a + (f < 64 ? __builtin_amdgcn_readlane(excl, f)
                                   : __builtin_amdgcn_readlane(incl, 63));
    acc = seg_grid_value(g, af);
    if (f < 64 && i + f < nv) {   // segment i + f: one exact rep_add
      const int32_t kf = __builtin_amdgcn_readlane(k, f);
      const float xf = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), f));
#ifdef DR_SEG_DEBUG
      const uint64_t t0 = clock64();
#endif
      acc = seg_add(acc, xf, kf);
#ifdef DR_SEG_DEBUG
      t_rep += clock64() - t0;
#endif
      i += f + 1;
    } else {
      i += f < 64 ? f : 64;
    }
    pe = qe[i - 1];
  }
#ifdef DR_SEG_DEBUG
  if (lane == 0) {
    const int slot = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    g_dbg[slot][0] += nr;
    g_dbg[slot][1] += t_rep;
    g_dbg[slot][2] += clock64() - t_all;
  }
#endif
  return acc;
}

// DR_GRAD_SEG_ROUNDS (default 0): 1 = the segment walk takes segments in
// rounds of a wave (wave_rounds_walk, and the scan on from 4 096 positions);
// 0 = one rep_add per segment where DR_GRAD_SEG_SCAN asks for a scan
static bool seg_rounds_host() {
  const char* e = getenv("DR_GRAD_SEG_ROUNDS");
  return e && atoi(e) != 0;
}

// The runs walked by segments (run_seg()): one block per (run, slice of 16
// columns).  Windows of up to 256 chunks: the chunks' segment ends (kpos)
// in ascending order, prefix of their counts in LDS; stages of up to 1024
// segments: every thread stages segments' terms (the term at the segment's
// end, = every term of it) transposed [column][segment] and their lengths
// (end - previous end); then lanes 0..15 of wave 0 each walk one column:
// acc = rep_add(acc, term, length) per segment, in order.  The chain starts
// at 0 (the sum combiner), so the first segment's first add is 0 + x, as in
// the plain walk.
// SW columns per slice, NT threads: (16, 1024) for the one-wave-per-column
// rep_add walk (16 walker waves on one CU); (4, 256) for the wave-rounds
// walk, whose whole-wave rounds are VALU work: one column per SIMD, the
// slices spread over CUs.
template <int VEC, bool SGD, bool WB, int SW, int NT>
__global__ __launch_bounds__(NT) void rows_serial_seg_kernel(RowsGroup g, int T, int dim,
                                                             RowsLong L, RowsSgd sg) {
  using V = typename VecT<VEC>::T;
  constexpr int SV = SW / VEC;     // vectors of a term's slice
  constexpr int S = 1024;          // segments per stage
  constexpr int WCH = NT;          // chunks per window (one per thread)
  static_assert(SW % VEC == 0 && SW % 2 == 0 && SW <= NT / 64, "slice shape");
  __shared__ __attribute__((aligned(16))) float stage[SW * S];
  __shared__ int32_t qend[S];
  __shared__ int64_t sk[DR_MAX_GROUP + 1];
  __shared__ int32_t cpre[WCH + 1];
  __shared__ int32_t wsum[NT / 64];
  __shared__ float accs[SW];
  if (threadIdx.x <= T) sk[threadIdx.x] = g.koff[threadIdx.x];
  __syncthreads();
  const int nsl = (dim + SW - 1) / SW;
  const int64_t total = (int64_t)(*L.nitems) * nsl;
  const int tid = threadIdx.x, lane = tid & 63;
  // wave w walks column w of the slice, all 64 lanes on the same values:
  // the closed form branches per column, and one column per wave keeps each
  // wave on its own path (16 columns on the lanes of one wave ran the union
  // of their paths: 2-3x slower than the plain walk, profiles/r05_seg_walk.log)
  const int wcol = __builtin_amdgcn_readfirstlane(tid >> 6);
  // the chains are the backward's critical path: ahead of co-resident waves
  // of other kernels (the DIN step runs this on a side stream beside them)
  __builtin_amdgcn_s_setprio(3);
  for (int64_t wi = blockIdx.x; wi < total; wi += gridDim.x) {   // block-uniform
    const int j = (int)(wi / nsl), slice = (int)(wi % nsl);
    const int i = L.items[2 * j];
    const int64_t len = L.rlen[i];
    const int np = (int)((len + L.smax - 1) / L.smax);
    if (!run_seg(L, i, np, len)) continue;
    const int64_t c0 = L.longs[i];
    const int32_t pc = L.perm[c0];
    const uint32_t u = L.skey[c0];
    const int t = tab_of(sk, T, pc);
    const dr_pool_grad_desc& d = g.d[t];
    const int cf = L.cfirst[i];
    const int64_t nch = (len + kRowsChunk - 1) / kRowsChunk;
    const int64_t ts = d.top_stride;
    float acc = 0.f;
    int64_t prev = c0 - 1;   // the end of the segment before the stage's first
#ifdef DR_SEG_DEBUG
    uint64_t t_pre = 0, t_stage = 0, t_walk = 0, tc = clock64();
    int nseg = 0;
#endif
    for (int64_t w0 = 0; w0 < nch; w0 += WCH) {
      const int nw = (int)(nch - w0 < WCH ? nch - w0 : WCH);
      // exclusive prefix of the window's chunk counts (one chunk per thread)
      const int cnt = tid < nw ? L.ccnt[cf + w0 + tid] : 0;
      int incl = cnt;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
      }
      if (lane == 63) wsum[tid >> 6] = incl;
      __syncthreads();
      int before = incl - cnt;
      for (int w = 0; w < (tid >> 6); ++w) before += wsum[w];
      if (tid < nw) cpre[tid] = before;
      if (tid == nw - 1) cpre[nw] = before + cnt;
      __syncthreads();
      const int K = cpre[nw];
#ifdef DR_SEG_DEBUG
      { const uint64_t t = clock64(); t_pre += t - tc; tc = t; }
#endif
      for (int b0 = 0; b0 < K; b0 += S) {
        const int nv = K - b0 < S ? K - b0 : S;
        for (int e = tid; e < nv; e += NT) {
          int lo = 0, hi = nw - 1;   // last chunk with cpre <= b0 + e
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (cpre[mid] <= b0 + e)
              lo = mid;
            else
              hi = mid - 1;
          }
          const int32_t q = L.kpos[c0 + (w0 + lo) * kRowsChunk + (b0 + e - cpre[lo])];
          qend[e] = q;
          const int32_t rq = L.srow[q];
          const float* row = d.top_grad + (int64_t)(rq >= 0 ? rq : 0) * ts;
#pragma unroll
          for (int cv = 0; cv < SV; ++cv) {
            const int col = slice * SW + cv * VEC;
            V x = (rq >= 0 && col < dim) ? gld(reinterpret_cast<const V*>(row + col)) : vzero<V>();
            if constexpr (VEC == 4) {
              stage[(cv * 4 + 0) * S + e] = x.x;
              stage[(cv * 4 + 1) * S + e] = x.y;
              stage[(cv * 4 + 2) * S + e] = x.z;
              stage[(cv * 4 + 3) * S + e] = x.w;
            } else if constexpr (VEC == 2) {
              stage[(cv * 2 + 0) * S + e] = x.x;
              stage[(cv * 2 + 1) * S + e] = x.y;
            } else {
              stage[cv * S + e] = x;
            }
          }
        }
        __syncthreads();
#ifdef DR_SEG_DEBUG
        { const uint64_t t = clock64(); t_stage += t - tc; tc = t; nseg += nv; }
#endif
        if (wcol < SW && slice * SW + wcol < dim) {   // (columns past dim: idle)
          const float* sp = stage + wcol * S;
          if (L.srounds)
            acc = wave_rounds_walk(acc, sp, qend, nv, prev, lane);
          else
            acc = serial_seg_walk(acc, sp, qend, nv, prev);
        }
        prev = qend[nv - 1];
        __syncthreads();   // the stage and qend are rewritten next
#ifdef DR_SEG_DEBUG
        { const uint64_t t = clock64(); t_walk += t - tc; tc = t; }
#endif
      }
    }
#ifdef DR_SEG_DEBUG
    if (lane == 0 && wcol == 0)
      printf("segwalk run %d slice %d: segs %d chunks %lld pre %llu stage %llu walk %llu cycles\n",
             i, slice, nseg, (long long)nch, (unsigned long long)t_pre, (unsigned long long)t_stage,
             (unsigned long long)t_walk);
    if (lane == 0 && L.srounds) {
      const int slot = blockIdx.x * 4 + wcol;
      printf("roundswalk run %d slice %d col %d: rounds %llu rep_add %llu walk %llu cycles\n", i,
             slice, wcol, g_dbg[slot][0], g_dbg[slot][1], g_dbg[slot][2]);
      g_dbg[slot][0] = g_dbg[slot][1] = g_dbg[slot][2] = 0;
    }
#endif
    if (wcol < SW && lane == 0) accs[wcol] = acc;
    __syncthreads();
    if (wcol == 0) {
      const int col = slice * SW + lane;
      const float a0 = accs[lane < SW ? lane : 0];
      const float nx = __shfl_down(a0, 1, 64);
      const int64_t o = SGD ? 0 : sk[t] + (int64_t)L.ex[pc] - L.base[t];
      if (lane < SW && (lane & 1) == 0 && col < dim)
        rows_fin_pair<SGD, WB>(sg, t, u, o, dim, col, a0, nx, L.gu);
      if (slice == 0 && lane == 0) rows_fin_run<SGD>(sg, t, u, o, dim, L);
    }
    __syncthreads();   // accs is rewritten by the next item
  }
}

// One block per (piece, column slice of SW columns): the piece's terms in
// ascending position order.  Wave 0 walks the serial chain of each column
// (one lane per column, at raised priority); waves 1..15 load the gradient-row
// slices S positions at a time (R loads in flight per thread, bag rows one
// stage ahead of the row loads), scale them and write them into LDS.  The
// stage is double-buffered: while the walker sums stage n out of one buffer
// the loaders write stage n + 1 into the other and issue the loads of stage
// n + 2, one barrier per stage -- the walk and the fill overlap.  A one-piece
// run is finished here; a piece of a longer run stores its partial for
// rows_combine_kernel.
template <int VEC, int SW, bool SGD, bool WB>
__global__ __launch_bounds__(1024) void rows_serial_kernel(RowsGroup g, int T, int dim, RowsLong L,
                                                           RowsSgd sg) {
  using V = typename VecT<VEC>::T;
  constexpr int NT = 1024;                 // threads: wave 0 walks, waves 1..15 load
  constexpr int NL = NT - 64;              // loader threads
  constexpr int SV = SW / VEC;             // vectors of a position's slice
  constexpr int PI = NL / SV;              // positions per load instruction
  constexpr int R = VEC == 4 ? 4 : 6;      // loads in flight per thread (<= 128 VGPRs, no spill)
  static_assert(VEC == 1 || VEC == 2 || VEC == 4, "vector width");
  constexpr int S = PI * R;                // positions per stage (S * SW <= 15 K floats)
  constexpr int SP = S + 4;                // column stride of the transposed stage
  constexpr int WCH = 1024;                // zero-scan chunks per window (prefix in LDS)
  static_assert(SV >= 1 && NL % SV == 0 && S % 4 == 0, "slice shape");
  // two stages, each TRANSPOSED, [column][position] (stride S + 4: the
  // loaders' column writes spread over the banks, the walker's 16-B reads
  // stay aligned): a lane walks its column 4 positions per LDS read
  __shared__ __attribute__((aligned(16))) float stage[2 * SW * SP];
  __shared__ int64_t sk[DR_MAX_GROUP + 1];
  __shared__ int32_t cpre[WCH + 1];
  __shared__ int32_t wsum[NT / 64];
  if (threadIdx.x <= T) sk[threadIdx.x] = g.koff[threadIdx.x];
  __syncthreads();
  const int nsl = (dim + SW - 1) / SW;
  const int64_t total = (int64_t)(*L.nitems) * nsl;
  const int tid = threadIdx.x;
  // wave-uniform, and known so to the compiler (readfirstlane): the walk
  // below then compiles as a scalar-controlled loop, not an exec-masked one
  const bool walker = __builtin_amdgcn_readfirstlane(tid >> 6) == 0;
  const int lt = walker ? 0 : tid - 64;    // loader index
  const int pv = lt / SV, cv = lt % SV;
  const int lane = tid & 63;
  const int lc = lane < SW ? lane : 0;
  if (walker) __builtin_amdgcn_s_setprio(3);   // the chain is the critical path
  for (int64_t wi = blockIdx.x; wi < total; wi += gridDim.x) {   // block-uniform
    const int j = (int)(wi / nsl), slice = (int)(wi % nsl);
    const int i = __builtin_amdgcn_readfirstlane(L.items[2 * j]);
    const int k = __builtin_amdgcn_readfirstlane(L.items[2 * j + 1]);
    const int64_t c0 = __builtin_amdgcn_readfirstlane(L.longs[i]);
    const int64_t len = __builtin_amdgcn_readfirstlane(L.rlen[i]);
    const int64_t smax = L.smax;
    const int np = (int)((len + smax - 1) / smax);
    const int64_t ps = c0 + (int64_t)k * smax;
    const int64_t pe = c0 + len < ps + smax ? c0 + len : ps + smax;
    const int32_t pc = __builtin_amdgcn_readfirstlane(L.perm[c0]);
    const uint32_t u = (uint32_t)__builtin_amdgcn_readfirstlane((int)L.skey[c0]);
    const int t = __builtin_amdgcn_readfirstlane(tab_of(sk, T, pc));
    const dr_pool_grad_desc& d = g.d[t];
    const bool wt = d.weights != nullptr;
    const bool qs = wt && d.bag_scale;
    const bool ms = !wt && d.combiner != DR_COMBINER_SUM;
    const bool zs = d.combiner == DR_COMBINER_SUM || wt;
    const int colv = slice * SV + cv;                 // this thread's vector column
    const float* src = d.top_grad + (colv * VEC < dim ? colv * VEC : 0);
    const int64_t ts = d.top_stride;
    // zero-scanned run (rows_nz_kernel): walk only its nonzero terms, chunk by
    // chunk in ascending order; a zero-started chain is unchanged by the
    // skipped +-0.0 terms (zero_scan()).  Otherwise entry e = position ps + e.
    if (run_seg(L, i, np, len)) continue;       // rows_serial_seg_kernel's run
    const bool zc = run_sparse(L, i, np, len);
    if (L.dma && !wt && !ms && !zc) continue;   // the plain / dma kernel's run
    const int cf = zc ? __builtin_amdgcn_readfirstlane(L.cfirst[i]) : -1;
    const int64_t nch = zc ? (len + kRowsChunk - 1) / kRowsChunk : 1;
    float acc = 0.f;
    bool fresh = !(k == 0 && zs);   // first term: 0 + y (zero-started sum) or y
    for (int64_t w0 = 0; w0 < nch; w0 += WCH) {   // windows of chunks (plain: one)
      int64_t K;
      int nw = 1;
      if (zc) {
        nw = (int)(nch - w0 < WCH ? nch - w0 : WCH);
        // exclusive prefix of the window's chunk counts (one chunk per
        // thread): wave scan by shuffles, wave totals through LDS
        const int cnt = tid < nw ? L.ccnt[cf + w0 + tid] : 0;
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int v = __shfl_up(incl, o, 64);
          if (lane >= o) incl += v;
        }
        if (lane == 63) wsum[tid >> 6] = incl;
        __syncthreads();
        int before = incl - cnt;
        for (int w = 0; w < (tid >> 6); ++w) before += wsum[w];
        if (tid < nw) cpre[tid] = before;
        if (tid == nw - 1) cpre[nw] = before + cnt;
        __syncthreads();
        K = cpre[nw];
      } else {
        K = pe - ps;
      }
      // sorted position of entry e (0 <= e < K)
      auto posmap = [&](int64_t e) -> int64_t {
        if (!zc) return ps + e;
        int lo = 0, hi = nw - 1;   // last chunk with cpre <= e
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (cpre[mid] <= e)
            lo = mid;
          else
            hi = mid - 1;
        }
        return L.kpos[c0 + (w0 + lo) * kRowsChunk + (e - cpre[lo])];
      };
      // bag rows one stage ahead of the row loads; every load is clamped to
      // the entries, so the batches issue unconditionally (a branch around a
      // batch would make the compiler wait for it at the join)
      int32_t rq[R];
      auto load_idx = [&](int64_t b0) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          int64_t e = b0 + r * PI + pv;
          e = e < K ? e : K - 1;
          rq[r] = L.srow[posmap(e)];
        }
      };
      uint32_t zmask = 0;   // invalid bags among the rows in flight (zero terms)
      auto take = [&]() {
        zmask = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) zmask |= (rq[r] < 0 ? 1u : 0u) << r;
      };
      V y[R];
      auto load_rows = [&]() {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int64_t rr = rq[r] >= 0 ? rq[r] : 0;
          y[r] = gld(reinterpret_cast<const V*>(src + rr * ts));
        }
      };
      auto put = [&](float* stg, int r, V x) {   // term (r, pv) -> its column rows of the stage
        const int pos = r * PI + pv;
        if constexpr (VEC == 4) {
          float* c = stg + (cv * 4) * SP + pos;
          c[0] = x.x;
          c[SP] = x.y;
          c[2 * SP] = x.z;
          c[3 * SP] = x.w;
        } else if constexpr (VEC == 2) {
          float* c = stg + (cv * 2) * SP + pos;
          c[0] = x.x;
          c[SP] = x.y;
        } else {
          stg[cv * SP + pos] = x;
        }
      };
      // the rows in flight (y) -> stage buffer stg, scaled (entries from b0)
      auto fill = [&](float* stg, int64_t b0) {
        if (wt || ms) {   // block-uniform: the terms' factors (rows_term), then scaled
          float mf[R], df[R];
#pragma unroll
          for (int r = 0; r < R; ++r) {
            int64_t e = b0 + r * PI + pv;
            e = e < K ? e : K - 1;
            const int64_t q = posmap(e);
            mf[r] = L.smul[q];
            df[r] = qs ? L.sdiv[q] : 1.f;
          }
#pragma unroll
          for (int r = 0; r < R; ++r) {
            V x = y[r];
            if ((zmask >> r) & 1u) x = vzero<V>();
            if (wt) {
              if (qs) x = vdiv(x, df[r]);
              x = vmul(x, mf[r]);
            } else if (mf[r] != 1.f) {
              x = vmul(x, mf[r]);
            }
            put(stg, r, x);
          }
        } else {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            V x = y[r];
            if ((zmask >> r) & 1u) x = vzero<V>();
            put(stg, r, x);
          }
        }
      };
      if (!walker && K > 0) {   // stage 0 into buffer 0; stage 1's rows in flight
        load_idx(0);
        take();
        load_rows();
        load_idx(S);
        fill(stage, 0);
        take();
        load_rows();
        load_idx(2 * S);
      }
      __syncthreads();
      int sb = 0;   // the buffer holding the stage at b0
      for (int64_t b0 = 0; b0 < K; b0 += S, sb ^= 1) {
        if (walker) {             // wave-uniform: lane lc walks column lc
          const int nv = (int)(K - b0 < S ? K - b0 : S);
          const float* sp = stage + sb * (SW * SP) + lc * SP;
          acc = chain_walk(sp, nv, fresh, acc);
        } else if (b0 + S < K) {  // the next stage into the other buffer, then its successor's loads
          fill(stage + (sb ^ 1) * (SW * SP), b0 + S);
          take();
          load_rows();
          load_idx(b0 + 3 * S);
        }
        __syncthreads();   // the next stage is in place; this one may be rewritten
      }
    }
    if (tid < 64) {
      const int col = slice * SW + lane;
      const float nxt = __shfl_down(acc, 1, 64);
      if (np == 1) {
        const int64_t o = SGD ? 0 : sk[t] + (int64_t)L.ex[pc] - L.base[t];
        if (lane < SW && (lane & 1) == 0 && col < dim)
          rows_fin_pair<SGD, WB>(sg, t, u, o, dim, col, acc, nxt, L.gu);
        if (slice == 0 && lane == 0) rows_fin_run<SGD>(sg, t, u, o, dim, L);
      } else if (lane < SW && col < dim) {
        L.part[(int64_t)j * dim + col] = acc;
      }
    }
  }
}

// The plain-sum runs (rows_serial_kernel's terms with no scale: the sum
// combiner, unweighted, not walked compacted), one block per (piece, slice of
// 16 columns): rows_serial_kernel's double-buffered walk without the scaling,
// compaction and window machinery, whose registers capped it at 6 loads in
// flight per thread -- here 8 (float2 / float) or 4 (float4) with a 16-column
// slice, so a stage is 960 positions (2.7 x the general kernel's 360 at DIN's
// dim 18): the loads of a stage have the walk of a whole stage to land.
template <int VEC, bool SGD, bool WB>
__global__ __launch_bounds__(1024) void rows_serial_plain_kernel(RowsGroup g, int T, int dim,
                                                                 RowsLong L, RowsSgd sg) {
  using V = typename VecT<VEC>::T;
  constexpr int SW = 16;                   // columns per slice
  constexpr int NL = 960;                  // loader threads (waves 1..15)
  constexpr int SV = SW / VEC;             // vectors of a position's slice
  constexpr int PI = NL / SV;              // positions per load instruction
  constexpr int R = VEC == 4 ? 4 : 8;      // loads in flight per thread
  constexpr int S = PI * R;                // positions per stage (480 / 960)
  constexpr int SP = S + 4;                // column stride of the transposed stage
  static_assert(NL % SV == 0 && S % 4 == 0, "slice shape");
  __shared__ __attribute__((aligned(16))) float stage[2 * SW * SP];
  __shared__ int64_t sk[DR_MAX_GROUP + 1];
  if (threadIdx.x <= T) sk[threadIdx.x] = g.koff[threadIdx.x];
  __syncthreads();
  const int nsl = (dim + SW - 1) / SW;
  const int64_t total = (int64_t)(*L.nitems) * nsl;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const bool walker = wave == 0;           // wave-uniform (an SGPR: scalar-controlled walk)
  const int lt = walker ? 0 : tid - 64;
  const int pv = lt / SV, cv = lt % SV;
  const int lc = lane < SW ? lane : 0;
  if (walker) __builtin_amdgcn_s_setprio(3);   // the chain is the critical path
  for (int64_t wi = blockIdx.x; wi < total; wi += gridDim.x) {   // block-uniform
    const int j = (int)(wi / nsl), slice = (int)(wi % nsl);
    const int i = __builtin_amdgcn_readfirstlane(L.items[2 * j]);
    const int k = __builtin_amdgcn_readfirstlane(L.items[2 * j + 1]);
    const int64_t c0 = __builtin_amdgcn_readfirstlane(L.longs[i]);
    const int64_t len = __builtin_amdgcn_readfirstlane(L.rlen[i]);
    const int64_t smax = L.smax;
    const int np = (int)((len + smax - 1) / smax);
    const int64_t ps = c0 + (int64_t)k * smax;
    const int64_t pe = c0 + len < ps + smax ? c0 + len : ps + smax;
    const int32_t pc = __builtin_amdgcn_readfirstlane(L.perm[c0]);
    const uint32_t u = (uint32_t)__builtin_amdgcn_readfirstlane((int)L.skey[c0]);
    const int t = __builtin_amdgcn_readfirstlane(tab_of(sk, T, pc));
    const dr_pool_grad_desc& d = g.d[t];
    const bool wt = d.weights != nullptr;
    const bool ms = !wt && d.combiner != DR_COMBINER_SUM;
    if (wt || ms || run_sparse(L, i, np, len)) continue;   // rows_serial_kernel's run
    if (run_seg(L, i, np, len)) continue;                  // rows_serial_seg_kernel's run
    const int64_t K = pe - ps;
    const int colv = slice * SV + cv;
    const float* src = d.top_grad + (colv * VEC < dim ? colv * VEC : 0);
    const int64_t ts = d.top_stride;
    const int32_t* srow = L.srow + ps;
    int32_t rq[R];
    auto load_idx = [&](int64_t b0) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        int64_t e = b0 + r * PI + pv;
        e = e < K ? e : K - 1;
        rq[r] = srow[e];
      }
    };
    V y[R];
    auto load_rows = [&]() {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int64_t rr = rq[r] >= 0 ? rq[r] : 0;
        y[r] = gld(reinterpret_cast<const V*>(src + rr * ts));
      }
    };
    uint32_t zmask = 0;
    auto take = [&]() {
      zmask = 0;
#pragma unroll
      for (int r = 0; r < R; ++r) zmask |= (rq[r] < 0 ? 1u : 0u) << r;
    };
    auto fill = [&](float* stg) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        V x = y[r];
        if ((zmask >> r) & 1u) x = vzero<V>();
        float* c = stg + (cv * VEC) * SP + r * PI + pv;
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
    };
    if (!walker) {   // stage 0 into buffer 0; stage 1's rows in flight
      load_idx(0);
      take();
      load_rows();
      load_idx(S);
      fill(stage);
      take();
      load_rows();
      load_idx(2 * S);
    }
    __syncthreads();
    float acc = 0.f;
    bool fresh = !(k == 0);   // first term: 0 + y (the sum combiner is zero-started) or y
    int sb = 0;
    for (int64_t b0 = 0; b0 < K; b0 += S, sb ^= 1) {
      if (walker) {
        const int nv = (int)(K - b0 < S ? K - b0 : S);
        acc = chain_walk(stage + sb * (SW * SP) + lc * SP, nv, fresh, acc);
      } else if (b0 + S < K) {
        fill(stage + (sb ^ 1) * (SW * SP));
        take();
        load_rows();
        load_idx(b0 + 3 * S);
      }
      __syncthreads();
    }
    if (walker) {
      const int col = slice * SW + lane;
      const float nx = __shfl_down(acc, 1, 64);
      if (np == 1) {
        const int64_t o = SGD ? 0 : sk[t] + (int64_t)L.ex[pc] - L.base[t];
        if (lane < SW && (lane & 1) == 0 && col < dim)
          rows_fin_pair<SGD, WB>(sg, t, u, o, dim, col, acc, nx, L.gu);
        if (slice == 0 && lane == 0) rows_fin_run<SGD>(sg, t, u, o, dim, L);
      } else if (lane < SW && col < dim) {
        L.part[(int64_t)j * dim + col] = acc;
      }
    }
  }
}

// The plain-sum runs (rows_serial_kernel's terms with no scale: the sum
// combiner, unweighted, not walked compacted), one block per (piece, slice of
// 16 columns).  Waves 1..15 stage the terms by LDS-DMA instead of through
// registers: loader wave w owns positions [64 w, 64 w + 64) of each stage of
// 960 and issues, per column, one global_load_lds of 4 B per lane (the term's
// column c lands at stage[c][position], the walker's transposed layout, with
// no register round trip and no LDS write instructions); an invalid bag reads
// the zero row.  Two stages in the ring: stage n + 1 lands while wave 0
// walks stage n, the loaders' bag rows one stage further ahead; one raw
// barrier per stage after each loader's counted vmcnt (its DMAs landed).
template <bool SGD, bool WB>
__global__ __launch_bounds__(1024) void rows_serial_dma_kernel(RowsGroup g, int T, int dim,
                                                               RowsLong L, RowsSgd sg) {
  constexpr int SW = 16;                   // columns per slice
  constexpr int S = 64 * 15;               // positions per stage: 64 per loader wave
  constexpr int SP = S + 4;                // column stride (16-B walker reads, banks spread)
  __shared__ __attribute__((aligned(16))) float stage[2 * SW * SP];
  __shared__ int64_t sk[DR_MAX_GROUP + 1];
  if (threadIdx.x <= T) sk[threadIdx.x] = g.koff[threadIdx.x];
  __syncthreads();
  const int nsl = (dim + SW - 1) / SW;
  const int64_t total = (int64_t)(*L.nitems) * nsl;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const bool walker = wave == 0;           // wave-uniform (an SGPR: scalar-controlled walk)
  const int lw = walker ? 0 : wave - 1;    // loader wave: its 64 positions of a stage
  const int lc = lane < SW ? lane : 0;
  if (walker) __builtin_amdgcn_s_setprio(3);   // the chain is the critical path
  for (int64_t wi = blockIdx.x; wi < total; wi += gridDim.x) {   // block-uniform
    const int j = (int)(wi / nsl), slice = (int)(wi % nsl);
    const int i = __builtin_amdgcn_readfirstlane(L.items[2 * j]);
    const int k = __builtin_amdgcn_readfirstlane(L.items[2 * j + 1]);
    const int64_t c0 = __builtin_amdgcn_readfirstlane(L.longs[i]);
    const int64_t len = __builtin_amdgcn_readfirstlane(L.rlen[i]);
    const int64_t smax = L.smax;
    const int np = (int)((len + smax - 1) / smax);
    const int64_t ps = c0 + (int64_t)k * smax;
    const int64_t pe = c0 + len < ps + smax ? c0 + len : ps + smax;
    const int32_t pc = __builtin_amdgcn_readfirstlane(L.perm[c0]);
    const uint32_t u = (uint32_t)__builtin_amdgcn_readfirstlane((int)L.skey[c0]);
    const int t = __builtin_amdgcn_readfirstlane(tab_of(sk, T, pc));
    const dr_pool_grad_desc& d = g.d[t];
    const bool wt = d.weights != nullptr;
    const bool ms = !wt && d.combiner != DR_COMBINER_SUM;
    if (wt || ms || run_sparse(L, i, np, len)) continue;   // rows_serial_kernel's run
    if (run_seg(L, i, np, len)) continue;                  // rows_serial_seg_kernel's run
    const int64_t K = pe - ps;
    const int64_t nst = (K + S - 1) / S;
    const int c0l = slice * SW;
    const int ncol = dim - c0l < SW ? dim - c0l : SW;
    const int64_t ts = d.top_stride;
    // this lane's bag row for the stage at entry b0 (clamped to the piece),
    // and the term source it gives -- split, so the row load is waited for
    // only where the next stage's DMAs use it
    auto rowof = [&](int64_t b0) -> int32_t {
      int64_t e = b0 + 64 * lw + lane;
      e = e < K ? e : K - 1;
      return L.srow[ps + e];
    };
    auto srcof = [&](int32_t r) -> const float* {
      return r >= 0 ? d.top_grad + (int64_t)r * ts + c0l : L.zrow;
    };
    auto dma = [&](const float* src, int slot) {
      char* base = reinterpret_cast<char*>(stage + slot * (SW * SP) + 64 * lw);
      for (int c = 0; c < ncol; ++c)   // uniform trip count
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + c),
                                         (__attribute__((address_space(3))) void*)(base + c * SP * 4),
                                         4, 0, 0);
    };
    int32_t nxt = 0;
    if (!walker) {   // stage 0 into slot 0, stage 1's bag rows in flight
      dma(srcof(rowof(0)), 0);
      asm volatile("" ::: "memory");   // the row load below stays behind the DMAs
      nxt = rowof(S);
      asm volatile("s_waitcnt vmcnt(1)" ::: "memory");   // this wave's stage-0 DMAs landed
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    float acc = 0.f;
    bool fresh = !(k == 0);   // first term: 0 + y (the sum combiner is zero-started) or y
    for (int64_t st = 0; st < nst; ++st) {
      if (walker) {
        const int64_t b0 = st * S;
        const int nv = (int)(K - b0 < S ? K - b0 : S);
        const float* sp = stage + (st & 1) * (SW * SP) + lc * SP;
        acc = chain_walk(sp, nv, fresh, acc);
      } else if (st + 1 < nst) {
        dma(srcof(nxt), (int)((st + 1) & 1));   // stage st+1 into the slot stage st-1 left
        asm volatile("" ::: "memory");
        nxt = rowof((st + 2) * S);       // (clamped past the end: one load, always)
        asm volatile("s_waitcnt vmcnt(1)" ::: "memory");   // stage st+1's DMAs landed
      }
      __builtin_amdgcn_s_barrier();   // stage st+1 in place (all loaders); stage st walked
      asm volatile("" ::: "memory");
    }
    if (walker) {
      const int col = c0l + lane;
      const float nx = __shfl_down(acc, 1, 64);
      if (np == 1) {
        const int64_t o = SGD ? 0 : sk[t] + (int64_t)L.ex[pc] - L.base[t];
        if (lane < SW && (lane & 1) == 0 && col < dim)
          rows_fin_pair<SGD, WB>(sg, t, u, o, dim, col, acc, nx, L.gu);
        if (slice == 0 && lane == 0) rows_fin_run<SGD>(sg, t, u, o, dim, L);
      } else if (lane < SW && col < dim) {
        L.part[(int64_t)j * dim + col] = acc;
      }
    }
  }
}

// Runs of several pieces: ((p_0 + p_1) + p_2) + ... of the piece partials in
// piece order (deterministic, independent of which block summed which
// piece), then finished as in rows_serial_kernel.
template <bool SGD, bool WB>
__global__ __launch_bounds__(256) void rows_combine_kernel(RowsGroup g, int T, int dim, RowsLong L,
                                                           RowsSgd sg) {
  __shared__ int64_t sk[DR_MAX_GROUP + 1];
  if (threadIdx.x <= T) sk[threadIdx.x] = g.koff[threadIdx.x];
  __syncthreads();
  const int n = *L.nlong;
  for (int i = blockIdx.x; i < n; i += gridDim.x) {   // block-uniform
    const int64_t len = L.rlen[i];
    const int np = (int)((len + L.smax - 1) / L.smax);
    if (np <= 1) continue;
    const int64_t fi = L.rfirst[i];
    const int64_t c0 = L.longs[i];
    const int32_t pc = L.perm[c0];
    const uint32_t u = L.skey[c0];
    const int t = tab_of(sk, T, pc);
    const int64_t o = SGD ? 0 : sk[t] + (int64_t)L.ex[pc] - L.base[t];
    for (int c = 2 * threadIdx.x; c < dim; c += 512) {
      const bool two = c + 1 < dim;
      float a = L.part[fi * dim + c];
      float b = two ? L.part[fi * dim + c + 1] : 0.f;
      for (int q = 1; q < np; ++q) {
        a = a + L.part[(fi + q) * dim + c];
        if (two) b = b + L.part[(fi + q) * dim + c + 1];
      }
      rows_fin_pair<SGD, WB>(sg, t, u, o, dim, c, a, b, L.gu);
    }
    if (threadIdx.x == 0) rows_fin_run<SGD>(sg, t, u, o, dim, L);
  }
}

// out[i] = *grad_ptr[i] (+0.0f first when bit 0 is set), i < min(n, *n_dev):
// the IndexedSlices values of a by-address gradient, materialised.
template <int VEC, int G, int CPL>
__global__ __launch_bounds__(256) void rows_from_ptr_kernel(const uint64_t* __restrict__ gptr,
                                                            int64_t n, const int64_t* n_dev,
                                                            int dim, float* __restrict__ out) {
  constexpr int GPB = 256 / G;
  const int64_t ne = eff_n(n, n_dev);
  const int64_t i = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
  if (i >= ne) return;
  const int lg = threadIdx.x % G;
  const int dv = dim / VEC;
  using R = Row<VEC, G, CPL>;
  using V = typename VecT<VEC>::T;
  const uint64_t p = gptr[i];
  R x;
  load_row_u<VEC, G, CPL>(x, reinterpret_cast<const float*>((uintptr_t)(p & ~(uint64_t)1)), lg,
                          dv);
  if (p & 1) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) x.v[c] = vadd(vzero<V>(), x.v[c]);
  }
  store_row<VEC, G, CPL>(x, out + i * (int64_t)dim, lg, dv);
}

struct RowsWs {
  uint32_t* kin;
  int32_t* vin;
  uint32_t* kout;
  int32_t* perm;
  int32_t* flags;
  int32_t* ex;
  int32_t* base;
  int64_t* total;
  int32_t* nlong;
  int32_t* nwork;
  int32_t* nitems;
  int32_t* work;
  int32_t* srow;
  float* smul;
  float* sdiv;
  int32_t* longs;
  int32_t* rlen;
  int32_t* rfirst;
  int32_t* items;
  float* part;
  int32_t* cfirst;
  int32_t* crun;
  int32_t* nchunk;
  int32_t* ccnt;
  int32_t* kpos;
  int32_t* rnz;
  int32_t* rseg;
  float* zrow;
  void* sort_ws;
  size_t sort_bytes;
  void* scan_ws;
  RowsLong longrun(uint64_t* gptr, float* gu) const {
    return RowsLong{kout, perm, ex, base, srow, smul, sdiv, longs, nlong, rlen, rfirst, items,
                    nitems, gptr, gu, part, serial_max(), zero_scan(), cfirst, crun, nchunk,
                    ccnt, kpos, rnz, zrow, serial_dma(), rseg, seg_scan(), seg_min(),
                    (int32_t)seg_rounds_host()};
  }
};

static RowsWs carve_rows(void* ws, int64_t n, size_t* used) {
  Carver c(ws);
  RowsWs w;
  const int64_t nn = n > 0 ? n : 1;
  w.kin = c.take<uint32_t>(nn);
  w.vin = c.take<int32_t>(nn);
  w.kout = c.take<uint32_t>(nn);
  w.perm = c.take<int32_t>(nn);
  w.flags = c.take<int32_t>(nn);
  w.ex = c.take<int32_t>(nn);
  w.base = c.take<int32_t>(DR_MAX_GROUP + 1);
  w.total = c.take<int64_t>(1);
  w.nlong = c.take<int32_t>(1);
  w.nwork = c.take<int32_t>(1);
  w.nitems = c.take<int32_t>(1);
  w.work = c.take<int32_t>(nn);
  w.srow = c.take<int32_t>(nn);
  w.smul = c.take<float>(nn);
  w.sdiv = c.take<float>(nn);
  // runs longer than kRowsChunk, and their pieces: at most one per
  // kRowsChunk + 1 positions each
  const int64_t runs = nn / (kRowsChunk + 1) + 2;
  w.longs = c.take<int32_t>(runs);
  w.rlen = c.take<int32_t>(runs);
  w.rfirst = c.take<int32_t>(runs);
  w.items = c.take<int32_t>(2 * runs);
  w.part = c.take<float>(runs * kRowsMaxDim);
  // zero scan: chunks of kRowsChunk positions of the long runs (at most one
  // per kRowsChunk positions plus one per run), compacted positions [N]
  const int64_t chunks = nn / kRowsChunk + runs + 1;
  w.cfirst = c.take<int32_t>(runs);
  w.crun = c.take<int32_t>(2 * chunks);
  w.nchunk = c.take<int32_t>(1);
  w.ccnt = c.take<int32_t>(chunks);
  w.kpos = c.take<int32_t>(nn);
  w.rnz = c.take<int32_t>(runs);
  w.rseg = c.take<int32_t>(runs);
  w.zrow = c.take<float>(64);
  w.sort_bytes = sort_pairs_u32_ws_bytes(nn);
  w.sort_ws = c.take<char>(w.sort_bytes);
  w.scan_ws = c.take<char>(scan_ws_bytes(nn));
  if (used) *used = c.used + 256;
  return w;
}

// The long-run kernels (expand, serial pieces, combine); empty lists cost one
// load per block.  Slices of at most 32 columns: a stage of S positions is
// 64 KiB (fp32 rows) / 32 KiB (unaligned) of LDS.
template <int VEC, bool SGD, bool WB>
static void launch_long(const RowsGroup& g, int T, int dim, const RowsLong& L, const RowsSgd& sg,
                        hipStream_t s, bool aligned2 = false) {
  const int64_t N = g.koff[T];
  if (N <= kRowsChunk) return;
  const int64_t runs = N / (kRowsChunk + 1) + 1;
  hipLaunchKernelGGL(rows_expand_kernel, dim3((unsigned)(runs < 1024 ? runs : 1024)), dim3(256), 0,
                     s, g, T, L);
  if (L.zscan > 0 && N > L.zscan) {
    const int64_t chunks = N / kRowsChunk + 1;
    hipLaunchKernelGGL((rows_nz_kernel<VEC>), dim3((unsigned)(chunks < 2048 ? chunks : 2048)),
                       dim3(256), 0, s, g, T, dim, L);
  }
  const bool segs = L.sscan > 0 && N > L.sscan;
  if (segs) {
    const int64_t chunks = N / kRowsChunk + 1;
    // (8-byte rows when every slice is: as the walk below)
    if (VEC == 1 && aligned2 && dim % 2 == 0)
      hipLaunchKernelGGL((rows_seg_kernel<2>), dim3((unsigned)(chunks < 2048 ? chunks : 2048)),
                         dim3(256), 0, s, g, T, dim, L);
    else
      hipLaunchKernelGGL((rows_seg_kernel<VEC>), dim3((unsigned)(chunks < 2048 ? chunks : 2048)),
                         dim3(256), 0, s, g, T, dim, L);
  }
  int sw = 1;
  while (sw < dim && sw < 32) sw <<= 1;
  if (VEC == 4 && sw < 4) sw = 4;
  const int64_t nsl = ceil_div(dim, sw);
  int64_t sb = runs * nsl;
  if (sb > 1024) sb = 1024;
  const dim3 grid((unsigned)sb);
#define DR_SERIAL(SWC)                                                                         \
  hipLaunchKernelGGL((rows_serial_kernel<VEC, SWC, SGD, WB>), grid, dim3(1024), 0, s, g, T, dim, L, \
                     sg)
  if constexpr (VEC == 4) {
    switch (sw) {
      case 4: DR_SERIAL(4); break;
      case 8: DR_SERIAL(8); break;
      case 16: DR_SERIAL(16); break;
      default: DR_SERIAL(32); break;
    }
  } else if (aligned2 && dim % 2 == 0) {
    // 8-byte rows (an even dim such as DIN's 18 at 8-byte offsets): the
    // serial walk loads float2 -- twice the bytes per load in flight
#define DR_SERIAL2(SWC)                                                                       \
  hipLaunchKernelGGL((rows_serial_kernel<2, SWC, SGD, WB>), grid, dim3(1024), 0, s, g, T, dim, L, \
                     sg)
    switch (sw < 2 ? 2 : sw) {
      case 2: DR_SERIAL2(2); break;
      case 4: DR_SERIAL2(4); break;
      case 8: DR_SERIAL2(8); break;
      case 16: DR_SERIAL2(16); break;
      default: DR_SERIAL2(32); break;
    }
#undef DR_SERIAL2
  } else {
    switch (sw) {
      case 1: DR_SERIAL(1); break;
      case 2: DR_SERIAL(2); break;
      case 4: DR_SERIAL(4); break;
      case 8: DR_SERIAL(8); break;
      case 16: DR_SERIAL(16); break;
      default: DR_SERIAL(32); break;
    }
  }
#undef DR_SERIAL
  if (L.dma) {
    const int64_t nsl16 = ceil_div(dim, 16);
    int64_t db = runs * nsl16;
    if (db > 1024) db = 1024;
    if (L.dma == 2)
      hipLaunchKernelGGL((rows_serial_dma_kernel<SGD, WB>), dim3((unsigned)db), dim3(1024), 0, s,
                         g, T, dim, L, sg);
    else if (VEC == 4)
      hipLaunchKernelGGL((rows_serial_plain_kernel<VEC, SGD, WB>), dim3((unsigned)db), dim3(1024),
                         0, s, g, T, dim, L, sg);
    else if (aligned2 && dim % 2 == 0)
      hipLaunchKernelGGL((rows_serial_plain_kernel<2, SGD, WB>), dim3((unsigned)db), dim3(1024), 0,
                         s, g, T, dim, L, sg);
    else
      hipLaunchKernelGGL((rows_serial_plain_kernel<1, SGD, WB>), dim3((unsigned)db), dim3(1024), 0,
                         s, g, T, dim, L, sg);
  }
  if (segs) {   // 4 columns per 256-thread block: one walker wave per SIMD
    int64_t sb2 = runs * ceil_div(dim, 4);
    if (sb2 > 1024) sb2 = 1024;
    if (VEC == 4)
      hipLaunchKernelGGL((rows_serial_seg_kernel<VEC, SGD, WB, 4, 256>), dim3((unsigned)sb2),
                         dim3(256), 0, s, g, T, dim, L, sg);
    else if (aligned2 && dim % 2 == 0)
      hipLaunchKernelGGL((rows_serial_seg_kernel<2, SGD, WB, 4, 256>), dim3((unsigned)sb2),
                         dim3(256), 0, s, g, T, dim, L, sg);
    else
      hipLaunchKernelGGL((rows_serial_seg_kernel<1, SGD, WB, 4, 256>), dim3((unsigned)sb2),
                         dim3(256), 0, s, g, T, dim, L, sg);
  }
  if (N > L.smax) {
    const int64_t big = N / (L.smax + 1) + 1;
    hipLaunchKernelGGL((rows_combine_kernel<SGD, WB>), dim3((unsigned)(big < 256 ? big : 256)),
                       dim3(256), 0, s, g, T, dim, L, sg);
  }
}

template <int VEC, int G, int CPL>
static void launch_rows(const RowsGroup& g, int T, int64_t B, const RowsWs& w, int dim,
                        bool weighted, uint64_t* gptr, float* gu, hipStream_t s, int* st) {
  const int64_t N = g.koff[T];
  // the worklist is at most N entries; a grid-stride pass over its device
  // count (an empty list costs one load per block)
  int64_t blocks = ceil_div(N, 256 / G);
  if (blocks > 1024) blocks = 1024;   // grid-stride: an idle block still costs its dispatch
  if (weighted)
    hipLaunchKernelGGL((rows_work_kernel<VEC, G, CPL, true>), dim3((unsigned)blocks), dim3(256),
                       0, s, g, T, B, w.kout, w.perm, w.ex, w.base, dim, w.work, w.nwork, gptr,
                       gu, st, RowsSgd{});
  else
    hipLaunchKernelGGL((rows_work_kernel<VEC, G, CPL, false>), dim3((unsigned)blocks), dim3(256),
                       0, s, g, T, B, w.kout, w.perm, w.ex, w.base, dim, w.work, w.nwork, gptr,
                       gu, st, RowsSgd{});
  bool aligned2 = dim % 2 == 0;
  for (int t = 0; t < T; ++t)
    aligned2 = aligned2 && ((uintptr_t)g.d[t].top_grad & 7) == 0 && g.d[t].top_stride % 2 == 0;
  launch_long<VEC, false, false>(g, T, dim, w.longrun(gptr, gu), RowsSgd{}, s, aligned2);
}

// The fused SGD tail: direct rows + worklist (rows_sgd_kernel), runs of 2 ..
// kRowsChunk positions (rows_work_kernel<SGD>), long runs (launch_long).
template <int G, int CPL, bool WB>
static void launch_rows_sgd(const RowsGroup& g, int T, int64_t B, const RowsWs& w, int dim,
                            bool weighted, uint32_t sentinel, const RowsSgd& sg, hipStream_t s,
                            int* st) {
  const int64_t N = g.koff[T];
  const RowsLong L = w.longrun(nullptr, nullptr);
  hipLaunchKernelGGL((rows_sgd_kernel<G, WB>), dim3((unsigned)ceil_div(N, 256)), dim3(256), 0, s,
                     g, sg, T, B, w.kout, w.perm, sentinel, dim, w.work, w.nwork, L, w.longs,
                     w.nlong, st);
  int64_t blocks = ceil_div(N, 256 / G);
  if (blocks > 1024) blocks = 1024;   // grid-stride: an idle block still costs its dispatch
  if (weighted)
    hipLaunchKernelGGL((rows_work_kernel<4, G, CPL, true, true, WB>), dim3((unsigned)blocks),
                       dim3(256), 0, s, g, T, B, w.kout, w.perm, nullptr, nullptr, dim, w.work,
                       w.nwork, nullptr, nullptr, st, sg);
  else
    hipLaunchKernelGGL((rows_work_kernel<4, G, CPL, false, true, WB>), dim3((unsigned)blocks),
                       dim3(256), 0, s, g, T, B, w.kout, w.perm, nullptr, nullptr, dim, w.work,
                       w.nwork, nullptr, nullptr, st, sg);
  launch_long<4, true, WB>(g, T, dim, L, sg, s);
}

// rows_record: the forward's rows are record-major [batch, T] (every feature
// one-hot, nnz == batch); validated here
static int rec_tables(const dr_pool_grad_desc* descs, int T, int64_t batch, int rows_record,
                      int* rec_t) {
  *rec_t = 0;
  if (!rows_record) return DR_OK;
  for (int t = 0; t < T; ++t)
    DR_REQUIRE(descs[t].nnz == batch && !descs[t].seg, DR_INVALID_ARGUMENT,
               "record-major rows need one-hot features of nnz == batch (table %d)", t);
  *rec_t = T;
  return DR_OK;
}

// Fused row-grouped backward + KV SGD (ev.hip dr_ev_pool_grad_rows_apply_sgd
// validates the EVs and fills sg).  Same sort and run sums as
// dr_pool_grad_rows_grouped_ex, applied in sorted order.  Needs 16-byte rows
// (dim % 4 == 0, aligned top_grad slices with top_stride % 4 == 0).
int rows_apply_sgd(const dr_pool_grad_desc* descs_host, int num_tables, int64_t batch, int dim,
                   const int64_t* rowsel, int64_t row_limit, const RowsSgd& sg, void* ws,
                   size_t ws_bytes, hipStream_t s, int rows_record) {
  DR_REQUIRE(descs_host && num_tables >= 1 && num_tables <= DR_MAX_GROUP && dim > 0 &&
                 dim <= kRowsMaxDim && dim % 4 == 0 && batch >= 0 && row_limit > 0 && rowsel,
             DR_INVALID_ARGUMENT, "bad argument (the fused SGD needs dim %% 4 == 0)");
  RowsGroup g;
  memset(&g, 0, sizeof(g));
  bool weighted = false;
  for (int t = 0; t < num_tables; ++t) {
    const dr_pool_grad_desc& d = descs_host[t];
    DR_REQUIRE(d.top_grad && d.nnz >= 0, DR_INVALID_ARGUMENT, "table %d: missing pointers", t);
    DR_REQUIRE(d.combiner == DR_COMBINER_SUM || d.bag_off || !d.seg, DR_INVALID_ARGUMENT,
               "table %d: mean/sqrtn of multi-hot bags need bag_off", t);
    DR_REQUIRE(!d.weights || d.combiner == DR_COMBINER_SUM || d.bag_scale, DR_INVALID_ARGUMENT,
               "table %d: weighted mean/sqrtn needs bag_scale (dr_bag_weight_scale)", t);
    DR_REQUIRE(((uintptr_t)d.top_grad & 15) == 0 && d.top_stride % 4 == 0, DR_INVALID_ARGUMENT,
               "table %d: the fused SGD reads 16-byte gradient rows", t);
    g.d[t] = d;
    g.koff[t + 1] = g.koff[t] + d.nnz;
    weighted = weighted || d.weights;
  }
  const int64_t n = g.koff[num_tables];
  DR_REQUIRE(n < (1ll << 31), DR_INVALID_ARGUMENT, "too many nnz");
  DR_REQUIRE(batch > 0 || n == 0, DR_INVALID_ARGUMENT, "nnz without a batch");
  DR_REQUIRE(batch < (1ll << 31), DR_INVALID_ARGUMENT, "batch must be < 2^31");
  DR_REQUIRE(ws_bytes >= dr_pool_grad_rows_workspace_size(n), DR_INVALID_ARGUMENT,
             "workspace too small");
  if (n == 0) return DR_OK;
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  RowsWs w = carve_rows(ws, n, nullptr);
  DR_REQUIRE(row_limit < ((int64_t)1 << 32) - 1, DR_INVALID_ARGUMENT,
             "row_limit must be < 2^32 - 1");
  int rb = 1;
  while (rb < 32 && ((int64_t)1 << rb) <= row_limit) ++rb;
  const uint32_t sentinel = (uint32_t)(((uint64_t)1 << rb) - 1);
  int rec_t = 0;
  int rrc = rec_tables(descs_host, num_tables, batch, rows_record, &rec_t);
  if (rrc) return rrc;
  hipLaunchKernelGGL(rows_keys_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, rowsel,
                     n, row_limit, sentinel, w.kin, w.vin, (int32_t*)nullptr, w.nlong, w.nwork,
                     w.nitems, w.nchunk, rec_t, batch);
  DR_LAUNCH_CHECK();
  int rc = sort_pairs_u32(w.kin, w.vin, w.kout, w.perm, n, rb, w.sort_ws, s);
  if (rc) return rc;
  const int d4 = dim / 4;
#define DR_ROWS_SGD(G, CPL)                                                                  \
  (sg.bf16 ? launch_rows_sgd<G, CPL, true>(g, num_tables, batch, w, dim, weighted, sentinel, sg, \
                                           s, st)                                              \
           : launch_rows_sgd<G, CPL, false>(g, num_tables, batch, w, dim, weighted, sentinel, sg, \
                                            s, st))
  if (d4 <= 8)
    DR_ROWS_SGD(8, 1);
  else if (d4 <= 16)
    DR_ROWS_SGD(16, 1);
  else if (d4 <= 32)
    DR_ROWS_SGD(32, 1);
  else if (d4 <= 64)
    DR_ROWS_SGD(64, 1);
  else
    DR_ROWS_SGD(64, 4);
#undef DR_ROWS_SGD
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // namespace dr

extern "C" {

size_t dr_pool_grad_rows_workspace_size(int64_t total_nnz) {
  size_t used = 0;
  dr::carve_rows(nullptr, total_nnz, &used);
  return used;
}

int dr_pool_grad_rows_grouped(const dr_pool_grad_desc* descs_host, int num_tables, int64_t batch,
                              int dim, const int64_t* rowsel, int64_t row_limit,
                              const int64_t* keys, int defer, int64_t* uniq_out,
                              int64_t* num_unique, uint64_t* grad_ptr, float* grad_unique,
                              void* ws, size_t ws_bytes, void* stream) {
  return dr_pool_grad_rows_grouped_ex(descs_host, num_tables, batch, dim, rowsel, row_limit, keys,
                                      defer, uniq_out, nullptr, num_unique, grad_ptr, grad_unique,
                                      ws, ws_bytes, stream);
}

int dr_pool_grad_rows_grouped_ex(const dr_pool_grad_desc* descs_host, int num_tables,
                                 int64_t batch, int dim, const int64_t* rowsel, int64_t row_limit,
                                 const int64_t* keys, int defer, int64_t* uniq_out,
                                 int64_t* uniq_rows, int64_t* num_unique, uint64_t* grad_ptr,
                                 float* grad_unique, void* ws, size_t ws_bytes, void* stream) {
  return dr_pool_grad_rows_grouped_ex2(descs_host, num_tables, batch, dim, rowsel, 0, row_limit,
                                       keys, defer, uniq_out, uniq_rows, num_unique, grad_ptr,
                                       grad_unique, ws, ws_bytes, stream);
}

int dr_pool_grad_rows_grouped_ex2(const dr_pool_grad_desc* descs_host, int num_tables,
                                  int64_t batch, int dim, const int64_t* rowsel, int rows_record,
                                  int64_t row_limit, const int64_t* keys, int defer,
                                  int64_t* uniq_out, int64_t* uniq_rows, int64_t* num_unique,
                                  uint64_t* grad_ptr, float* grad_unique, void* ws,
                                  size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(descs_host && num_tables >= 1 && num_tables <= DR_MAX_GROUP && dim > 0 &&
                 dim <= kRowsMaxDim && batch >= 0 && row_limit > 0 && rowsel && keys &&
                 uniq_out && num_unique && grad_ptr && grad_unique,
             DR_INVALID_ARGUMENT, "bad argument");
  RowsGroup g;
  memset(&g, 0, sizeof(g));
  bool aligned = dim % 4 == 0 && ((uintptr_t)grad_unique & 15) == 0;
  bool weighted = false;
  for (int t = 0; t < num_tables; ++t) {
    const dr_pool_grad_desc& d = descs_host[t];
    DR_REQUIRE(d.top_grad && d.nnz >= 0, DR_INVALID_ARGUMENT, "table %d: missing pointers", t);
    DR_REQUIRE(d.combiner == DR_COMBINER_SUM || d.bag_off || !d.seg, DR_INVALID_ARGUMENT,
               "table %d: mean/sqrtn of multi-hot bags need bag_off", t);
    DR_REQUIRE(!d.weights || d.combiner == DR_COMBINER_SUM || d.bag_scale, DR_INVALID_ARGUMENT,
               "table %d: weighted mean/sqrtn needs bag_scale (dr_bag_weight_scale)", t);
    g.d[t] = d;
    g.koff[t + 1] = g.koff[t] + d.nnz;
    aligned = aligned && ((uintptr_t)d.top_grad & 15) == 0 && d.top_stride % 4 == 0;
    weighted = weighted || d.weights;
  }
  const int64_t n = g.koff[num_tables];
  DR_REQUIRE(n < (1ll << 31), DR_INVALID_ARGUMENT, "too many nnz");
  DR_REQUIRE(batch > 0 || n == 0, DR_INVALID_ARGUMENT, "nnz without a batch");
  DR_REQUIRE(batch < (1ll << 31), DR_INVALID_ARGUMENT, "batch must be < 2^31");
  DR_REQUIRE(ws_bytes >= dr_pool_grad_rows_workspace_size(n), DR_INVALID_ARGUMENT,
             "workspace too small");
  hipStream_t s = S(stream);
  if (n == 0) return fill_bytes(num_unique, 0, sizeof(int64_t) * num_tables, s);
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  DR_REQUIRE(dim % 4 != 0 || ((uintptr_t)grad_unique & 15) == 0, DR_INVALID_ARGUMENT,
             "grad_unique must be 16-byte aligned");
  if (!aligned) defer = 0;   // by-address rows must share grad_unique's alignment
  RowsWs w = carve_rows(ws, n, nullptr);
  DR_REQUIRE(row_limit < ((int64_t)1 << 32) - 1, DR_INVALID_ARGUMENT,
             "row_limit must be < 2^32 - 1");
  int rb = 1;
  while (rb < 32 && ((int64_t)1 << rb) <= row_limit) ++rb;   // rows < 2^rb - 1
  const uint32_t sentinel = (uint32_t)(((uint64_t)1 << rb) - 1);
  const unsigned nb = (unsigned)ceil_div(n, 256);
  int rec_t = 0;
  int rrc = rec_tables(descs_host, num_tables, batch, rows_record, &rec_t);
  if (rrc) return rrc;
  hipLaunchKernelGGL(rows_keys_kernel, dim3(nb), dim3(256), 0, s, rowsel, n, row_limit, sentinel,
                     w.kin, w.vin, w.flags, w.nlong, w.nwork, w.nitems, w.nchunk, rec_t, batch);
  DR_LAUNCH_CHECK();
  int rc = sort_pairs_u32(w.kin, w.vin, w.kout, w.perm, n, rb, w.sort_ws, s);
  if (rc) return rc;
  hipLaunchKernelGGL(rows_heads_kernel, dim3(nb), dim3(256), 0, s, g, num_tables, batch, w.kout,
                     w.perm, sentinel, w.flags, w.work, w.nwork, w.longrun(grad_ptr, grad_unique),
                     w.longs, w.nlong, st);
  rc = scan_exclusive_marks(w.flags, w.ex, n, w.total, w.scan_ws, s);
  if (rc) return rc;
  hipLaunchKernelGGL(rows_emit_kernel, dim3(nb), dim3(256), 0, s, g, num_tables, batch, keys,
                     w.flags, w.ex, w.total, defer, uniq_out, num_unique, w.base, grad_ptr, w.work,
                     w.nwork, rowsel, uniq_rows, st, dim, grad_unique, rec_t);
  DR_LAUNCH_CHECK();
  if (aligned) {
    const int d4 = dim / 4;
    if (d4 <= 8)
      launch_rows<4, 8, 1>(g, num_tables, batch, w, dim, weighted, grad_ptr, grad_unique, s, st);
    else if (d4 <= 16)
      launch_rows<4, 16, 1>(g, num_tables, batch, w, dim, weighted, grad_ptr, grad_unique, s, st);
    else if (d4 <= 32)
      launch_rows<4, 32, 1>(g, num_tables, batch, w, dim, weighted, grad_ptr, grad_unique, s, st);
    else if (d4 <= 64)
      launch_rows<4, 64, 1>(g, num_tables, batch, w, dim, weighted, grad_ptr, grad_unique, s, st);
    else
      launch_rows<4, 64, 4>(g, num_tables, batch, w, dim, weighted, grad_ptr, grad_unique, s, st);
  } else {
    if (dim <= 4)   // wide (linear) tables: dim 1
      launch_rows<1, 4, 1>(g, num_tables, batch, w, dim, weighted, grad_ptr, grad_unique, s, st);
    else if (dim <= 32)
      launch_rows<1, 32, 1>(g, num_tables, batch, w, dim, weighted, grad_ptr, grad_unique, s, st);
    else if (dim <= 64)
      launch_rows<1, 64, 1>(g, num_tables, batch, w, dim, weighted, grad_ptr, grad_unique, s, st);
    else if (dim <= 256)
      launch_rows<1, 64, 4>(g, num_tables, batch, w, dim, weighted, grad_ptr, grad_unique, s, st);
    else
      launch_rows<1, 64, 16>(g, num_tables, batch, w, dim, weighted, grad_ptr, grad_unique, s,
                             st);
  }
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_rows_from_ptr(const uint64_t* grad_ptr, int64_t n, const int64_t* n_dev, int dim,
                     float* out, void* stream) {
  using namespace dr;
  DR_REQUIRE(n >= 0 && dim > 0 && dim <= kRowsMaxDim && (n == 0 || (grad_ptr && out)),
             DR_INVALID_ARGUMENT, "bad argument");
  if (n == 0) return DR_OK;
  hipStream_t s = S(stream);
  // by-address rows are 16-byte aligned whenever dim % 4 == 0 (the producer
  // only defers when every top_grad slice is)
  if (dim % 4 == 0 && ((uintptr_t)out & 15) == 0) {
    const int d4 = dim / 4;
    if (d4 <= 32)
      hipLaunchKernelGGL((rows_from_ptr_kernel<4, 32, 1>), dim3((unsigned)ceil_div(n, 8)),
                         dim3(256), 0, s, grad_ptr, n, n_dev, dim, out);
    else
      hipLaunchKernelGGL((rows_from_ptr_kernel<4, 64, 4>), dim3((unsigned)ceil_div(n, 4)),
                         dim3(256), 0, s, grad_ptr, n, n_dev, dim, out);
  } else if (dim <= 4) {
    hipLaunchKernelGGL((rows_from_ptr_kernel<1, 4, 1>), dim3((unsigned)ceil_div(n, 64)),
                       dim3(256), 0, s, grad_ptr, n, n_dev, dim, out);
  } else if (dim <= 32) {
    hipLaunchKernelGGL((rows_from_ptr_kernel<1, 32, 1>), dim3((unsigned)ceil_div(n, 8)),
                       dim3(256), 0, s, grad_ptr, n, n_dev, dim, out);
  } else if (dim <= 64) {
    hipLaunchKernelGGL((rows_from_ptr_kernel<1, 64, 1>), dim3((unsigned)ceil_div(n, 4)),
                       dim3(256), 0, s, grad_ptr, n, n_dev, dim, out);
  } else {
    hipLaunchKernelGGL((rows_from_ptr_kernel<1, 64, 16>), dim3((unsigned)ceil_div(n, 4)),
                       dim3(256), 0, s, grad_ptr, n, n_dev, dim, out);
  }
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // extern "C"
