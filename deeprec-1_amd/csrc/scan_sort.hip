// scan_sort.hip -- device-wide exclusive scan and stable LSD radix sort.
//
// Scan: reduce-then-scan over 2048-item tiles (256 threads x 8 items), wave64
// shuffles + LDS across the 4 waves of a block.  Sort: 8-bit digits, per-tile
// LDS histograms, stable in-tile ranking by wave64 ballot matching (the
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

__global__ void scan_reduce_kernel(const int32_t* __restrict__ in, int64_t n,
                                   const int64_t* n_dev, int32_t* __restrict__ bsum) {
  __shared__ int lds[4];
  const int64_t ne = eff_n(n, n_dev);
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  int s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < ne) s += in[base + k];
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
    v[k] = (base + k < ne) ? in[base + k] : 0;
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

size_t scan_ws_bytes(int64_t n) {
  return (size_t)((ceil_div(n > 0 ? n : 1, kScanTile) + 64) * sizeof(int32_t)) + 256;
}

int scan_exclusive_i32(const int32_t* in, int32_t* out, int64_t n, const int64_t* n_dev,
                       int64_t* total, void* ws, hipStream_t st) {
  if (n <= 0) {
    if (total) return fill_bytes(total, 0, sizeof(int64_t), st);
    return DR_OK;
  }
  const int64_t nb = ceil_div(n, kScanTile);
  int32_t* bsum = static_cast<int32_t*>(ws);
  hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(kScanThreads), 0, st, in, n,
                     n_dev, bsum);
  hipLaunchKernelGGL(scan_bsum_kernel, dim3(1), dim3(kScanThreads), 0, st, bsum, nb, total);
  hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nb), dim3(kScanThreads), 0, st, in, out,
                     n, n_dev, bsum);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

// ---------------------------------------------------------------------------
// Stable LSD radix sort, 8-bit digits.  Tile = 256 threads x 16 rounds.
// hist layout: [digit][block] so one exclusive scan yields scatter bases.
// ---------------------------------------------------------------------------
static constexpr int kSortThreads = 256;
static constexpr int kSortRounds = 16;
static constexpr int kSortTile = kSortThreads * kSortRounds;

__global__ void sort_hist_kernel(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                 int32_t* __restrict__ hist, int64_t nblocks) {
  __shared__ int cnt[256];
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
  for (int r = 0; r < kSortRounds; ++r) {
    const int64_t i = base + (int64_t)r * kSortThreads + threadIdx.x;
    if (i < n) atomicAdd(&cnt[(keys[i] >> shift) & 255], 1);
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * nblocks + blockIdx.x] = cnt[threadIdx.x];
}

__global__ void sort_scatter_kernel(const uint64_t* __restrict__ kin,
                                    const int32_t* __restrict__ vin, uint64_t* __restrict__ kout,
                                    int32_t* __restrict__ vout, int64_t n, int shift,
                                    const int32_t* __restrict__ hist_scanned, int64_t nblocks) {
  __shared__ int run[256];
  __shared__ int wcnt[4][256];
  run[threadIdx.x] = hist_scanned[(int64_t)threadIdx.x * nblocks + blockIdx.x];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
  for (int r = 0; r < kSortRounds; ++r) {
    wcnt[0][threadIdx.x] = 0;
    wcnt[1][threadIdx.x] = 0;
    wcnt[2][threadIdx.x] = 0;
    wcnt[3][threadIdx.x] = 0;
    __syncthreads();
    const int64_t i = base + (int64_t)r * kSortThreads + threadIdx.x;
    const bool valid = i < n;
    uint64_t key = valid ? kin[i] : 0;
    int32_t val = valid ? vin[i] : 0;
    const int d = (int)((key >> shift) & 255);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1;
      const uint64_t bb = __ballot(valid && bit);
      peers &= bit ? bb : ~bb;
    }
    const int rank = __popcll(peers & lanemask_lt());
    const int gsize = __popcll(peers);
    if (valid && rank == gsize - 1) wcnt[wave][d] = gsize;
    __syncthreads();
    int pos = 0;
    if (valid) {
      pos = run[d] + rank;
      for (int w = 0; w < wave; ++w) pos += wcnt[w][d];
    }
    __syncthreads();
    run[threadIdx.x] += wcnt[0][threadIdx.x] + wcnt[1][threadIdx.x] + wcnt[2][threadIdx.x] +
                        wcnt[3][threadIdx.x];
    if (valid) {
      kout[pos] = key;
      vout[pos] = val;
    }
    (void)lane;
  }
}

static size_t sort_hist_elems(int64_t n) { return (size_t)256 * ceil_div(n > 0 ? n : 1, kSortTile); }

}  // namespace dr

extern "C" size_t dr_sort_pairs_workspace_size(int64_t n) {
  dr::Carver c(nullptr);
  c.take<uint64_t>(n > 0 ? n : 1);
  c.take<int32_t>(n > 0 ? n : 1);
  size_t he = dr::sort_hist_elems(n);
  c.take<int32_t>(he);
  c.take<char>(dr::scan_ws_bytes((int64_t)he));
  c.take<int64_t>(1);
  return c.used + 256;
}

extern "C" int dr_sort_pairs(const uint64_t* keys_in, const int32_t* vals_in, uint64_t* keys_out,
                             int32_t* vals_out, int64_t n, int bit_lo, int bit_hi, void* ws,
                             size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(n >= 0 && bit_lo >= 0 && bit_hi <= 64 && bit_lo <= bit_hi, DR_INVALID_ARGUMENT,
             "dr_sort_pairs: bad arguments");
  DR_REQUIRE(ws_bytes >= dr_sort_pairs_workspace_size(n), DR_INVALID_ARGUMENT,
             "dr_sort_pairs: workspace too small");
  hipStream_t st = S(stream);
  if (n == 0) return DR_OK;
  Carver c(ws);
  uint64_t* ktmp = c.take<uint64_t>(n);
  int32_t* vtmp = c.take<int32_t>(n);
  const size_t he = sort_hist_elems(n);
  int32_t* hist = c.take<int32_t>(he);
  void* sws = c.take<char>(scan_ws_bytes((int64_t)he));
  int64_t* tot = c.take<int64_t>(1);
  const int64_t nblocks = ceil_div(n, kSortTile);
  int passes = (bit_hi - bit_lo + 7) / 8;
  if (passes == 0) {
    DR_HIP(hipMemcpyAsync(keys_out, keys_in, n * sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
    DR_HIP(hipMemcpyAsync(vals_out, vals_in, n * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    return DR_OK;
  }
  const uint64_t* ks = keys_in;
  const int32_t* vs = vals_in;
  for (int p = 0; p < passes; ++p) {
    const bool to_out = ((passes - 1 - p) % 2) == 0;
    uint64_t* kd = to_out ? keys_out : ktmp;
    int32_t* vd = to_out ? vals_out : vtmp;
    const int shift = bit_lo + 8 * p;
    hipLaunchKernelGGL(sort_hist_kernel, dim3((unsigned)nblocks), dim3(kSortThreads), 0, st, ks,
                       n, shift, hist, nblocks);
    int rc = scan_exclusive_i32(hist, hist, (int64_t)he, nullptr, tot, sws, st);
    if (rc) return rc;
    hipLaunchKernelGGL(sort_scatter_kernel, dim3((unsigned)nblocks), dim3(kSortThreads), 0, st,
                       ks, vs, kd, vd, n, shift, hist, nblocks);
    DR_LAUNCH_CHECK();
    ks = kd;
    vs = vd;
  }
  return DR_OK;
}
