// scan_sort.hip -- device-wide exclusive scan and stable LSD radix sort.
//
// Scan: reduce-then-scan over 2048-item tiles (256 threads x 8 items), wave64
// shuffles + LDS across the 4 waves of a block.  Sort: 8-bit digits, per-tile
// LDS histograms, stable in-tile ranking by wave64 ballot matching and an
// LDS regroup so each digit's run leaves the tile as one coalesced store (the
// CDNA4 replacement for cub::DeviceRadixSort::SortPairs used by
// FusedEmbeddingSparsePreLookUp, fused_embedding_ops_gpus.cu.cc:192-212).
#include "dr_common.h"

namespace dr {

static constexpr int kScanThreads = 256;
static constexpr int kScanItems = 8;
static constexpr int kScanTile = kScanThreads * kScanItems;

// Block-wide exclusive scan of one int per thread; returns the block total.
__device__ __forceinline__ int block_exclusive_scan(int v, int* lds /*[4]*/, int* total) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds[wave] = x;
  __syncthreads();
  int wprefix = 0, t = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / 64; ++w) {
    int s = lds[w];
    if (w < wave) wprefix += s;
    t += s;
  }
  __syncthreads();
  *total = t;
  return wprefix + x - v;
}

// FLAG: the scanned value of element i is (in[i] != -1) -- a count of the
// set entries of a "-1 = empty" marker array.
template <bool FLAG>
__device__ __forceinline__ int scan_val(int32_t v) {
  return FLAG ? (v != -1) : v;
}

template <bool FLAG>
__global__ void scan_reduce_kernel(const int32_t* __restrict__ in, int64_t n,
                                   const int64_t* n_dev, int32_t* __restrict__ bsum) {
  __shared__ int lds[4];
  const int64_t ne = eff_n(n, n_dev);
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  int s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < ne) s += scan_val<FLAG>(in[base + k]);
  int tot;
  block_exclusive_scan(s, lds, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// One block scans the block sums in place (exclusive) and writes the total.
__global__ void scan_bsum_kernel(int32_t* __restrict__ bsum, int64_t nb, int64_t* total) {
  __shared__ int lds[4];
  int carry = 0;
  for (int64_t base = 0; base < nb; base += kScanThreads) {
    const int64_t i = base + threadIdx.x;
    int v = i < nb ? bsum[i] : 0;
    int tot;
    int ex = block_exclusive_scan(v, lds, &tot);
    if (i < nb) bsum[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

template <bool FLAG>
__global__ void scan_apply_kernel(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                  int64_t n, const int64_t* n_dev,
                                  const int32_t* __restrict__ bsum) {
  __shared__ int lds[4];
  const int64_t ne = eff_n(n, n_dev);
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  int v[kScanItems];
  int s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = (base + k < ne) ? scan_val<FLAG>(in[base + k]) : 0;
    s += v[k];
  }
  int tot;
  int run = block_exclusive_scan(s, lds, &tot) + bsum[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (base + k < ne) out[base + k] = run;
    run += v[k];
  }
}

// Small inputs (n <= kSmallScan): ONE block of 1024 threads scans the whole
// array in chunks of 8192 (coalesced loads staged through LDS, each thread
// scans 8 consecutive items, a carry runs across chunks) -- one launch
// instead of reduce / block sums / apply, whose cost at this size is the
// three launch latencies.
static constexpr int kSmallScanThreads = 1024;
static constexpr int kSmallScanChunk = kSmallScanThreads * 8;
static constexpr int64_t kSmallScan = 65536;

template <bool FLAG>
__global__ __launch_bounds__(1024) void scan_small_kernel(const int32_t* __restrict__ in,
                                                          int32_t* __restrict__ out, int64_t n,
                                                          const int64_t* n_dev, int64_t* total) {
  __shared__ int buf[kSmallScanChunk];
  __shared__ int wsum[kSmallScanThreads / 64];
  const int64_t ne = eff_n(n, n_dev);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int carry = 0;
  for (int64_t c0 = 0; c0 < ne; c0 += kSmallScanChunk) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t i = c0 + k * kSmallScanThreads + threadIdx.x;
      buf[k * kSmallScanThreads + threadIdx.x] = i < ne ? scan_val<FLAG>(in[i]) : 0;
    }
    __syncthreads();
    int v[8], s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] = buf[threadIdx.x * 8 + k];
      s += v[k];
    }
    int x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kSmallScanThreads / 64; ++w) {
      const int ws = wsum[w];
      pre += w < wave ? ws : 0;
      tot += ws;
    }
    int run = carry + pre + x - s;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      buf[threadIdx.x * 8 + k] = run;
      run += v[k];
    }
    carry += tot;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t i = c0 + k * kSmallScanThreads + threadIdx.x;
      if (i < ne) out[i] = buf[k * kSmallScanThreads + threadIdx.x];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

size_t scan_ws_bytes(int64_t n) {
  return (size_t)((ceil_div(n > 0 ? n : 1, kScanTile) + 64) * sizeof(int32_t)) + 256;
}

template <bool FLAG>
static int scan_exclusive(const int32_t* in, int32_t* out, int64_t n, const int64_t* n_dev,
                          int64_t* total, void* ws, hipStream_t st) {
  if (n <= 0) {
    if (total) return fill_bytes(total, 0, sizeof(int64_t), st);
    return DR_OK;
  }
  if (n <= kSmallScan) {
    hipLaunchKernelGGL(scan_small_kernel<FLAG>, dim3(1), dim3(kSmallScanThreads), 0, st, in, out,
                       n, n_dev, total);
    DR_LAUNCH_CHECK();
    return DR_OK;
  }
  const int64_t nb = ceil_div(n, kScanTile);
  int32_t* bsum = static_cast<int32_t*>(ws);
  hipLaunchKernelGGL(scan_reduce_kernel<FLAG>, dim3((unsigned)nb), dim3(kScanThreads), 0, st, in,
                     n, n_dev, bsum);
  hipLaunchKernelGGL(scan_bsum_kernel, dim3(1), dim3(kScanThreads), 0, st, bsum, nb, total);
  hipLaunchKernelGGL(scan_apply_kernel<FLAG>, dim3((unsigned)nb), dim3(kScanThreads), 0, st, in,
                     out, n, n_dev, bsum);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int scan_exclusive_i32(const int32_t* in, int32_t* out, int64_t n, const int64_t* n_dev,
                       int64_t* total, void* ws, hipStream_t st) {
  return scan_exclusive<false>(in, out, n, n_dev, total, ws, st);
}

int scan_exclusive_marks(const int32_t* in, int32_t* out, int64_t n, int64_t* total, void* ws,
                         hipStream_t st) {
  return scan_exclusive<true>(in, out, n, nullptr, total, ws, st);
}

// ---------------------------------------------------------------------------
// Stable LSD radix sort, 8-bit digits, 3 launches per pass:
//   hist    per-tile digit counts, layout [digit][tile];
//   rowscan one block per digit: exclusive scan of its row over the tiles,
//           and the digit's total;
//   scatter ranks the tile stably in LDS (wave64 ballot matching, 16 rounds
//           of 256 keys), regroups the tile by digit in LDS, then writes
//           every digit's run of the tile to consecutive global positions --
//           consecutive lanes hit consecutive addresses, so the stores
//           coalesce instead of landing one 8-byte key per digit per round.
// Global position = exclusive prefix of the digit totals (scanned in each
// scatter block, 256 entries) + the digit's row prefix + the tile-local
// offset inside the digit's run.
// ---------------------------------------------------------------------------
// Tile = 256 threads x R rounds of keys.  R = 16 (4096-key tiles) left a
// 1.7 M-pair sort with 416 blocks, every one of them resident at once and
// the pass bound by one block's 16 serial ranking rounds; R = 8 halves that
// chain at the same residency (DR_SORT_ROUNDS: 16 / 8 / 4 A/B switch).
static constexpr int kSortThreads = 256;
static int sort_rounds() {
  static const int r = [] {
    const char* e = getenv("DR_SORT_ROUNDS");
    const int v = e ? atoi(e) : 8;
    return (v == 4 || v == 16) ? v : 8;
  }();
  return r;
}

// n_dev (optional DEVICE count <= n): the grid is sized for n, tiles past
// the device count contribute empty histograms and scatter nothing.
template <class K, int kSortRounds>
__global__ __launch_bounds__(256) void sort_hist_kernel(const K* __restrict__ keys, int64_t n,
                                                        const int64_t* n_dev, int shift,
                                                        int dmask, int32_t* __restrict__ hist,
                                                        int64_t nblocks) {
  constexpr int kSortTile = kSortThreads * kSortRounds;
  __shared__ int cnt[256];
  cnt[threadIdx.x] = 0;
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
  const int64_t ne = eff_n(n, n_dev);
  const int c = ne <= base ? 0 : (int)(ne - base < kSortTile ? ne - base : kSortTile);
  int d[kSortRounds];
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {       // all loads in flight before the atomics
    const int i = r * kSortThreads + threadIdx.x;
    d[r] = i < c ? (int)((keys[base + i] >> shift) & dmask) : -1;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r)
    if (d[r] >= 0) atomicAdd(&cnt[d[r]], 1);
  __syncthreads();
  hist[(int64_t)threadIdx.x * nblocks + blockIdx.x] = cnt[threadIdx.x];
}

__global__ __launch_bounds__(256) void sort_rowscan_kernel(int32_t* __restrict__ hist,
                                                           int64_t nblocks,
                                                           int32_t* __restrict__ digit_tot) {
  __shared__ int lds[4];
  int32_t* row = hist + (int64_t)blockIdx.x * nblocks;
  int carry = 0;
  for (int64_t b0 = 0; b0 < nblocks; b0 += kSortThreads) {
    const int64_t i = b0 + threadIdx.x;
    const int v = i < nblocks ? row[i] : 0;
    int tot;
    const int ex = block_exclusive_scan(v, lds, &tot);
    if (i < nblocks) row[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) digit_tot[blockIdx.x] = carry;
}

// Each wave ranks its own contiguous quarter of the tile (16 rounds of 64
// keys) against wave-private LDS digit counters: within one wave the LDS
// read of a counter and the group leader's update are ordered, so the loop
// needs no block barrier.  Tile offset of (wave w, digit d) =
// exclusive-over-digits(total) + sum over w' < w of the wave counts.
template <class K, int kSortRounds>
__global__ __launch_bounds__(256) void sort_scatter_kernel(
    const K* __restrict__ kin, const int32_t* __restrict__ vin, K* __restrict__ kout,
    int32_t* __restrict__ vout, int64_t n, const int64_t* n_dev, int shift, int dmask,
    const int32_t* __restrict__ row_scanned, const int32_t* __restrict__ digit_tot,
    int64_t nblocks) {
  constexpr int kSortTile = kSortThreads * kSortRounds;
  __shared__ K sk[kSortTile];
  __shared__ int32_t sv[kSortTile];
  __shared__ int wcnt[4][256];
  __shared__ int toff[256];
  __shared__ int gbase[256];
  __shared__ int lds[4];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
  const int64_t ne = eff_n(n, n_dev);
  if (ne <= base) return;   // block-uniform: a tile past the device count
  const int cnt = (int)(ne - base < kSortTile ? ne - base : kSortTile);
  const int wbase = wave * (kSortTile / 4);
  K key[kSortRounds];
  int32_t val[kSortRounds];
  int rk[kSortRounds];
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = wbase + r * 64 + lane;
    const bool valid = i < cnt;
    key[r] = valid ? kin[base + i] : 0;
    val[r] = valid ? vin[base + i] : 0;
  }
  wcnt[0][tid] = 0;
  wcnt[1][tid] = 0;
  wcnt[2][tid] = 0;
  wcnt[3][tid] = 0;
  int tot;
  const int dex = block_exclusive_scan(digit_tot[tid], lds, &tot);   // has barriers
  gbase[tid] = dex + row_scanned[(int64_t)tid * nblocks + blockIdx.x];
  int* mycnt = wcnt[wave];
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const bool valid = wbase + r * 64 + lane < cnt;
    const int d = (int)((key[r] >> shift) & dmask);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1;
      const uint64_t bb = __ballot(valid && bit);
      peers &= bit ? bb : ~bb;
    }
    const int rank = __popcll(peers & lanemask_lt());
    const int gsize = __popcll(peers);
    const int old = valid ? mycnt[d] : 0;
    rk[r] = old + rank;
    if (valid && rank == 0) mycnt[d] = old + gsize;
  }
  __syncthreads();
  const int c0 = wcnt[0][tid], c1 = wcnt[1][tid], c2 = wcnt[2][tid], c3 = wcnt[3][tid];
  const int dt = block_exclusive_scan(c0 + c1 + c2 + c3, lds, &tot);
  toff[tid] = dt;
  wcnt[0][tid] = dt;                 // per-wave tile offsets of digit tid
  wcnt[1][tid] = dt + c0;
  wcnt[2][tid] = dt + c0 + c1;
  wcnt[3][tid] = dt + c0 + c1 + c2;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    if (wbase + r * 64 + lane < cnt) {
      const int d = (int)((key[r] >> shift) & dmask);
      const int at = mycnt[d] + rk[r];
      sk[at] = key[r];
      sv[at] = val[r];
    }
  }
  __syncthreads();
#pragma unroll 4
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = r * kSortThreads + tid;
    if (i < cnt) {
      const K k = sk[i];
      const int d = (int)((k >> shift) & dmask);
      const int64_t pos = (int64_t)gbase[d] + (i - toff[d]);
      kout[pos] = k;
      vout[pos] = sv[i];
    }
  }
}

}  // namespace dr

namespace dr {

template <class K>
static size_t sort_ws_bytes(int64_t n) {
  Carver c(nullptr);
  c.take<K>(n > 0 ? n : 1);
  c.take<int32_t>(n > 0 ? n : 1);
  // sized for the smallest tile any switch setting uses
  c.take<int32_t>((size_t)256 * ceil_div(n > 0 ? n : 1, kSortThreads * 4));
  c.take<int32_t>(256);
  return c.used + 256;
}

template <class K>
static int sort_pairs(const K* keys_in, const int32_t* vals_in, K* keys_out, int32_t* vals_out,
                      int64_t n, int bit_lo, int bit_hi, void* ws, hipStream_t st,
                      const int64_t* n_dev = nullptr) {
  if (n == 0) return DR_OK;
  Carver c(ws);
  K* ktmp = c.take<K>(n);
  int32_t* vtmp = c.take<int32_t>(n);
  const int rounds = sort_rounds();
  const int64_t nblocks = ceil_div(n, (int64_t)kSortThreads * rounds);
  int32_t* hist = c.take<int32_t>((size_t)256 * ceil_div(n, (int64_t)kSortThreads * 4));
  int32_t* dtot = c.take<int32_t>(256);
  int passes = (bit_hi - bit_lo + 7) / 8;
  if (passes == 0) {
    DR_HIP(hipMemcpyAsync(keys_out, keys_in, n * sizeof(K), hipMemcpyDeviceToDevice, st));
    DR_HIP(hipMemcpyAsync(vals_out, vals_in, n * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    return DR_OK;
  }
  const K* ks = keys_in;
  const int32_t* vs = vals_in;
  for (int p = 0; p < passes; ++p) {
    const bool to_out = ((passes - 1 - p) % 2) == 0;
    K* kd = to_out ? keys_out : ktmp;
    int32_t* vd = to_out ? vals_out : vtmp;
    const int shift = bit_lo + 8 * p;
    const int dbits = bit_hi - shift < 8 ? bit_hi - shift : 8;   // bits >= bit_hi are ignored
    const int dmask = (1 << dbits) - 1;
#define DR_SORT_PASS(R)                                                                      \
  do {                                                                                       \
    hipLaunchKernelGGL((sort_hist_kernel<K, R>), dim3((unsigned)nblocks), dim3(kSortThreads), \
                       0, st, ks, n, n_dev, shift, dmask, hist, nblocks);                    \
    hipLaunchKernelGGL(sort_rowscan_kernel, dim3(256), dim3(kSortThreads), 0, st, hist,      \
                       nblocks, dtot);                                                       \
    hipLaunchKernelGGL((sort_scatter_kernel<K, R>), dim3((unsigned)nblocks),                 \
                       dim3(kSortThreads), 0, st, ks, vs, kd, vd, n, n_dev, shift, dmask, hist, \
                       dtot, nblocks);                                                       \
  } while (0)
    if (rounds == 16)
      DR_SORT_PASS(16);
    else if (rounds == 4)
      DR_SORT_PASS(4);
    else
      DR_SORT_PASS(8);
#undef DR_SORT_PASS
    DR_LAUNCH_CHECK();
    ks = kd;
    vs = vd;
  }
  return DR_OK;
}

size_t sort_pairs_u32_ws_bytes(int64_t n) { return sort_ws_bytes<uint32_t>(n); }

int sort_pairs_u64_dev(const uint64_t* keys_in, const int32_t* vals_in, uint64_t* keys_out,
                       int32_t* vals_out, int64_t n_cap, const int64_t* n_dev, int bits,
                       void* ws, hipStream_t st) {
  DR_REQUIRE(n_cap >= 0 && n_cap < ((int64_t)1 << 31) && bits >= 0 && bits <= 64 && n_dev,
             DR_INVALID_ARGUMENT, "sort_pairs_u64_dev: bad arguments");
  // the pass count is fixed on the host: an even count keeps the result in
  // keys_out whatever n turns out to be
  return sort_pairs<uint64_t>(keys_in, vals_in, keys_out, vals_out, n_cap, 0, bits, ws, st,
                              n_dev);
}

int sort_pairs_u32(const uint32_t* keys_in, const int32_t* vals_in, uint32_t* keys_out,
                   int32_t* vals_out, int64_t n, int bits, void* ws, hipStream_t st) {
  DR_REQUIRE(n >= 0 && n < ((int64_t)1 << 31) && bits >= 0 && bits <= 32, DR_INVALID_ARGUMENT,
             "sort_pairs_u32: bad arguments");
  return sort_pairs<uint32_t>(keys_in, vals_in, keys_out, vals_out, n, 0, bits, ws, st);
}

}  // namespace dr

extern "C" size_t dr_sort_pairs_workspace_size(int64_t n) {
  return dr::sort_ws_bytes<uint64_t>(n);
}

extern "C" int dr_sort_pairs(const uint64_t* keys_in, const int32_t* vals_in, uint64_t* keys_out,
                             int32_t* vals_out, int64_t n, int bit_lo, int bit_hi, void* ws,
                             size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(n >= 0 && bit_lo >= 0 && bit_hi <= 64 && bit_lo <= bit_hi, DR_INVALID_ARGUMENT,
             "dr_sort_pairs: bad arguments");
  DR_REQUIRE(n < ((int64_t)1 << 31), DR_INVALID_ARGUMENT, "dr_sort_pairs: n >= 2^31");
  DR_REQUIRE(ws_bytes >= dr_sort_pairs_workspace_size(n), DR_INVALID_ARGUMENT,
             "dr_sort_pairs: workspace too small");
  return sort_pairs<uint64_t>(keys_in, vals_in, keys_out, vals_out, n, bit_lo, bit_hi, ws,
                              S(stream));
}
