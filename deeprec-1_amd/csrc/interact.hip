// interact.hip -- feature interactions fed by the pooled embeddings.
//   FM second order   modelzoo/DeepFM/train.py:205-209   (HBM-bound)
//   DLRM dot          modelzoo/DLRM/train.py:150-163     (LDS-tiled, per sample)
//   DCN-v2 CrossNet   (absent from the reference)        (bf16 MFMA GEMM)
#include "dr_common.h"

#include <algorithm>
#include <stdlib.h>

namespace dr {

// out[b, d] = 0.5 * ((sum_f e)^2 - sum_f e^2); thread per (b, 4 columns).
// ecopy (nullable): also the bf16 copy of emb [B, F*D] -- DeepFM's --bf16
// dnn input (train.py:186-189) written from the loads the sum already makes.
__global__ void fm2_kernel(const float* __restrict__ emb, int64_t B, int F, int D,
                           float* __restrict__ out, uint16_t* __restrict__ ecopy = nullptr) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int D4 = D / 4;
  if (t >= B * D4) return;
  const int64_t b = t / D4;
  const int c = (int)(t % D4);
  const float4* p = reinterpret_cast<const float4*>(emb + b * (int64_t)F * D) + c;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
  uint2* cp = ecopy ? reinterpret_cast<uint2*>(ecopy + b * (int64_t)F * D) + c : nullptr;
  for (int f = 0; f < F; ++f) {
    const float4 e = p[(int64_t)f * D4];
    s.x += e.x; s.y += e.y; s.z += e.z; s.w += e.w;
    q.x += e.x * e.x; q.y += e.y * e.y; q.z += e.z * e.z; q.w += e.w * e.w;
    if (cp) cp[(int64_t)f * D4] = make_uint2(f2_to_bf16x2(e.x, e.y), f2_to_bf16x2(e.z, e.w));
  }
  float4 o;
  o.x = 0.5f * (s.x * s.x - q.x);
  o.y = 0.5f * (s.y * s.y - q.y);
  o.z = 0.5f * (s.z * s.z - q.z);
  o.w = 0.5f * (s.w * s.w - q.w);
  reinterpret_cast<float4*>(out + b * (int64_t)D)[c] = o;
}

// d fm / d e_f = (sum_f' e_f' - e_f) * g.  Thread per (b, 4 columns); the F
// field vectors stay in registers between the sum and the write (a second
// read pass went back to HBM: the in-flight working set outgrows L2).
// add (nullable): a bf16 gradient of the same [B, F*D] embedding from its
// other use (DeepFM's bf16 dnn input), added after the FM term -- the one
// fp32 add autograd does where the two uses meet.
template <int FM>
__global__ __launch_bounds__(256) void fm2_grad_kernel(const float* __restrict__ emb,
                                                       const float* __restrict__ g, int64_t B,
                                                       int F, int D, float* __restrict__ ge,
                                                       const uint16_t* __restrict__ add = nullptr,
                                                       int64_t add_stride = 0) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int D4 = D / 4;
  if (t >= B * D4) return;
  const int64_t b = t / D4;
  const int c = (int)(t - b * D4);
  const float4* p = reinterpret_cast<const float4*>(emb + b * (int64_t)F * D) + c;
  float4 e[FM];
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int f = 0; f < FM; ++f)
    if (f < F) e[f] = nt_load(p + (int64_t)f * D4);
#pragma unroll
  for (int f = 0; f < FM; ++f)
    if (f < F) {
      s.x += e[f].x; s.y += e[f].y; s.z += e[f].z; s.w += e[f].w;
    }
  const float4 gv = reinterpret_cast<const float4*>(g + b * (int64_t)D)[c];
  float4* q = reinterpret_cast<float4*>(ge + b * (int64_t)F * D) + c;
  const uint2* ap = add ? reinterpret_cast<const uint2*>(add + b * add_stride) + c : nullptr;
  uint2 av[FM];
  if (ap) {
#pragma unroll
    for (int f = 0; f < FM; ++f)
      if (f < F) av[f] = ap[(int64_t)f * D4];
  }
#pragma unroll
  for (int f = 0; f < FM; ++f)
    if (f < F) {
      float4 o;
      o.x = (s.x - e[f].x) * gv.x;
      o.y = (s.y - e[f].y) * gv.y;
      o.z = (s.z - e[f].z) * gv.z;
      o.w = (s.w - e[f].w) * gv.w;
      if (ap) {
        const float2 a0 = bf16x2_to_f2(av[f].x), a1 = bf16x2_to_f2(av[f].y);
        o.x = o.x + a0.x;
        o.y = o.y + a0.y;
        o.z = o.z + a1.x;
        o.w = o.w + a1.y;
      }
      nt_store(o, q + (int64_t)f * D4);
    }
}

// Any shape: scalar, two passes.
__global__ void fm2_grad_any_kernel(const float* __restrict__ emb, const float* __restrict__ g,
                                    int64_t B, int F, int D, float* __restrict__ ge) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * D) return;
  const int64_t b = t / D;
  const int d = (int)(t % D);
  const float* p = emb + b * (int64_t)F * D + d;
  float s = 0.f;
  for (int f = 0; f < F; ++f) s += p[(int64_t)f * D];
  const float gv = g[b * D + d];
  for (int f = 0; f < F; ++f) ge[b * (int64_t)F * D + (int64_t)f * D + d] = (s - p[(int64_t)f * D]) * gv;
}

// DLRM dot, register-tiled: one wave per sample, X [F, D] staged in LDS
// (rows padded to a multiple of 4, row stride D+4 floats).  The lower
// triangle of X X^T is cut into 4x4 tiles (nb = ceil(F/4) row blocks,
// nb(nb+1)/2 <= 32 tiles); lane = 2*tile + khalf accumulates its tile's 16
// dot products over alternate 4-float K slices with dwordx4 LDS reads (8
// reads per 64 FMAs), and one xor-shuffle adds the two partial sums.  LDS traffic per sample ~ tiles x 8
// rows x D floats instead of 2 rows x D per pair.
// Any shape: one block per sample: X [F, D] staged in LDS (row stride D+1 to break bank
// conflicts), thread per lower-triangle pair (i > j), row-major pair order.
__global__ void dot_kernel(const float* __restrict__ x, int F, int D, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int64_t b = blockIdx.x;
  const int ld = D + 1;
  const float* src = x + b * (int64_t)F * D;
  for (int e = threadIdx.x; e < F * D; e += blockDim.x) xs[(e / D) * ld + e % D] = src[e];
  __syncthreads();
  const int P = F * (F - 1) / 2;
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    // invert p = i(i-1)/2 + j
    int i = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)p)) * 0.5f);
    while (i * (i - 1) / 2 > p) --i;
    while ((i + 1) * i / 2 <= p) ++i;
    const int j = p - i * (i - 1) / 2;
    const float* a = xs + i * ld;
    const float* c = xs + j * ld;
    float s = 0.f;
    for (int d = 0; d < D; ++d) s += a[d] * c[d];
    out[b * (int64_t)P + p] = s;
  }
}

static constexpr int DOT_WAVES = 4;
static constexpr int DOT_MAXE = 16;  // float4 per lane when staging: F_pad * D / 4 <= 1024

__device__ __forceinline__ void dot_load(float4 (&v)[DOT_MAXE], const float* x, int64_t b,
                                         int64_t B, int nv, int FD, int lane) {
  const float4* src = reinterpret_cast<const float4*>(x + b * (int64_t)FD);
#pragma unroll
  for (int q = 0; q < DOT_MAXE; ++q) {
    const int e = lane + q * 64;
    v[q] = (b < B && e < nv) ? nt_load(src + e) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// Persistent: block i handles samples (i + it*grid)*DOT_WAVES + wave, and
// the loads of a wave's next sample are issued before it computes the
// current one (their registers are free once the sample sits in LDS), so
// HBM latency hides behind the LDS/FMA work at 2 blocks per CU.
__global__ __launch_bounds__(256) void dot_tile_kernel(const float* __restrict__ x, int64_t B,
                                                       int F, int D, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float xs_all[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int Fp = (F + 3) & ~3;
  const int ld = D + 4;
  const int D4 = D / 4;
  const int n4 = Fp * D4, nv = F * D4;
  float* xs = xs_all + (size_t)wave * Fp * ld;
  const int nb = Fp / 4;
  const int tiles = nb * (nb + 1) / 2;
  const int tile = lane >> 1, kh = lane & 1;
  int bi = 0, bj = 0;
  if (tile < tiles) {
    // tile -> (bi >= bj), row-major over the lower block triangle
    while ((bi + 1) * (bi + 2) / 2 <= tile) ++bi;
    bj = tile - bi * (bi + 1) / 2;
  }
  const int64_t P = (int64_t)F * (F - 1) / 2;
  const int64_t step = (int64_t)gridDim.x * DOT_WAVES;
  int64_t b = (int64_t)blockIdx.x * DOT_WAVES + wave;
  const int64_t b_first_of_block = (int64_t)blockIdx.x * DOT_WAVES;
  float4 v[DOT_MAXE];
  dot_load(v, x, b, B, nv, F * D, lane);
  for (int64_t bb = b_first_of_block; bb < B; bb += step, b += step) {
    // (the trip count is uniform over the block: bb is the block's first sample)
#pragma unroll
    for (int q = 0; q < DOT_MAXE; ++q) {
      const int e = lane + q * 64;
      if (e < n4) {
        const int r = e / D4, c = e - r * D4;
        *reinterpret_cast<float4*>(xs + r * ld + c * 4) = v[q];
      }
    }
    __syncthreads();
    dot_load(v, x, b + step, B, nv, F * D, lane);  // next sample, in flight during compute
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    if (tile < tiles) {
      const float* A = xs + (bi * 4) * ld;
      const float* Bm = xs + (bj * 4) * ld;
      // lanes 2t, 2t+1 take alternate 4-float slices of K (adjacent banks)
      for (int k = kh * 4; k < D; k += 8) {
        float4 a4[4], c4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a4[i] = *reinterpret_cast<const float4*>(A + i * ld + k);
#pragma unroll
        for (int j = 0; j < 4; ++j) c4[j] = *reinterpret_cast<const float4*>(Bm + j * ld + k);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[i][j] = fmaf(a4[i].x, c4[j].x, acc[i][j]);
            acc[i][j] = fmaf(a4[i].y, c4[j].y, acc[i][j]);
            acc[i][j] = fmaf(a4[i].z, c4[j].z, acc[i][j]);
            acc[i][j] = fmaf(a4[i].w, c4[j].w, acc[i][j]);
          }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] += __shfl_xor(acc[i][j], 1, 64);
    if (b < B && tile < tiles && !kh) {
      float* o = out + b * P;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int gi = bi * 4 + i, gj = bj * 4 + j;
          if (gi < F && gj < gi) o[gi * (gi - 1) / 2 + gj] = acc[i][j];
        }
    }
    __syncthreads();  // LDS is rewritten next iteration
  }
}

// ---------------------------------------------------------------------------
// DLRM dot on the f32-input MFMA (v_mfma_f32_16x16x4_f32: exact f32, one
// rounding per product, a k-ordered fmaf chain per 4-k step).  One wave per
// sample, no LDS: the Gram matrix X X^T of a sample is at most 32 x 32 =
// 2 x 2 blocks of 16 rows, of which the lower three are formed:
// (0,0) = mfma(a0, a0), (1,0) = mfma(a1, a0), (1,1) = mfma(a1, a1).
// The A and B operand maps of 16x16x4 (A[i = l&15][k = l>>4], B[k = l>>4]
// [j = l&15]) ask each lane for the SAME value X[l&15 (+16)][k], so one
// register per row block feeds both operands.  The k order is free as long
// as A and B agree: lane (r = l&15, q = l>>4) loads float4 i of its rows at
// columns i*16 + q*4 .. +3 (each row's 64 B per load instruction are
// contiguous), and MFMA step (i, c) takes component c.
// Per sample: 2 * KI float4 loads per lane, NT * 4 * KI MFMAs (NT = 1 when
// F <= 16, 3 otherwise), the strict lower triangle stored from the C/D map
// (col = l&15, row = (l>>4)*4 + reg).  HBM-bound: X read once, out written
// once; the LDS-tiled VALU kernel above was LDS-read bound (8 ds_read_b128
// per 64 FMAs).
// ---------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(4))) float dot_f4;
template <int KI, int NT>
struct DotRows {
  float4 a0[KI], a1[KI];
};
// Rows >= F are loaded from a clamped (valid) address and left as they are:
// Gram entry (i, j) depends on rows i and j only, and entries with i or j >=
// F are never stored.  No predicated loads: a branch per load made hipcc
// fall back to vmcnt(0), which also waited for the prefetched next sample.
template <int KI, int NT>
__device__ __forceinline__ void dot_rows_load(DotRows<KI, NT>& v, const float* x, int64_t b, int F,
                                              int r, int q) {
  constexpr int D = KI * 16;
  const float4* base = reinterpret_cast<const float4*>(x + b * F * (int64_t)D) + q;
  const float4* p0 = base + (r < F ? r : F - 1) * (D / 4);
#pragma unroll
  for (int i = 0; i < KI; ++i) v.a0[i] = gld(p0 + i * 4);
  if (NT > 1) {
    const float4* p1 = base + (r + 16 < F ? r + 16 : F - 1) * (D / 4);
#pragma unroll
    for (int i = 0; i < KI; ++i) v.a1[i] = gld(p1 + i * 4);
  }
}
// One sample per wave, 40 VGPRs, so 8 waves per SIMD overlap one another's
// loads and MFMAs (persistent waves prefetching their next sample, 188 VGPRs
// at 2 waves per SIMD, measured slower: 209 vs 196 us in the DLRM step).
// The C/D map scatters a lane's results over the sample's output row (4
// segments of <= 64 B per store instruction): the row is assembled in the
// wave's LDS slice and written out as contiguous 256-B instructions (the
// scattered dword stores cost ~25 % of the kernel; nontemporal stores 201-206
// vs 195 us).  LDS ops of one wave complete in order, so the reads see the
// writes.
// CAT: the DLRM top-MLP input instead (modelzoo/DLRM/train.py:211-226:
// concat([dense_inputs, dot], 1), cast to bf16 under --bf16): row b of a
// bf16 [B, ostride] matrix = bf16(X[b, 0, :]) | bf16(dot) | zeros up to
// ostride (the MFMA tower's K padding), two values per lane and store.
template <int KI, int NT, bool CAT>
__global__ __launch_bounds__(256) void dot_mfma_kernel(const float* __restrict__ x, int64_t B,
                                                       int F, void* __restrict__ out,
                                                       int64_t ostride) {
  constexpr int D = KI * 16;
  __shared__ float rows_lds[4][CAT ? 640 : 512];   // (x0 |) the pairs (<= 496) per wave
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  if (b >= B) return;   // wave-uniform; no barriers below
  DotRows<KI, NT> v;
  dot_rows_load<KI, NT>(v, x, b, F, r, q);
  dot_f4 c00 = {0.f, 0.f, 0.f, 0.f}, c10 = c00, c11 = c00;
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const float p0[4] = {v.a0[i].x, v.a0[i].y, v.a0[i].z, v.a0[i].w};
    const float p1[4] = {v.a1[i].x, v.a1[i].y, v.a1[i].z, v.a1[i].w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      c00 = __builtin_amdgcn_mfma_f32_16x16x4f32(p0[c], p0[c], c00, 0, 0, 0);
      if (NT > 1) {
        c10 = __builtin_amdgcn_mfma_f32_16x16x4f32(p1[c], p0[c], c10, 0, 0, 0);
        c11 = __builtin_amdgcn_mfma_f32_16x16x4f32(p1[c], p1[c], c11, 0, 0, 0);
      }
    }
  }
  float* row = rows_lds[wave];
  float* pr = row + (CAT ? D : 0);   // the pairs
  if (CAT && r == 0) {               // lanes 0, 16, 32, 48 hold X[b, 0, :]
#pragma unroll
    for (int i = 0; i < KI; ++i) *reinterpret_cast<float4*>(row + i * 16 + q * 4) = v.a0[i];
  }
  const int gj = lane & 15;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int gi = q * 4 + e;
    if (gi < F && gj < gi) pr[gi * (gi - 1) / 2 + gj] = c00[e];
    if (NT > 1) {
      const int hi = gi + 16;
      if (hi < F) {
        pr[hi * (hi - 1) / 2 + gj] = c10[e];
        if (gj + 16 < hi) pr[hi * (hi - 1) / 2 + gj + 16] = c11[e];
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  const int P = F * (F - 1) / 2;
  if (!CAT) {
    float* o = static_cast<float*>(out) + b * (int64_t)P;
    for (int e = lane; e < P; e += 64) o[e] = row[e];
  } else {
    uint32_t* o = reinterpret_cast<uint32_t*>(static_cast<uint16_t*>(out) + b * ostride);
    const int n = D + P;
    for (int e2 = lane; e2 < ostride / 2; e2 += 64) {
      const int e = 2 * e2;
      const float lo = e < n ? row[e] : 0.f, hi = e + 1 < n ? row[e + 1] : 0.f;
      o[e2] = (uint32_t)bf16_rne(lo) | ((uint32_t)bf16_rne(hi) << 16);
    }
  }
}

// ---------------------------------------------------------------------------
// Dot interaction backward: dX[b,i,:] = sum_{j != i} S[i,j] X[b,j,:] with S
// the symmetric completion of the pair grads (S[i,j] = S[j,i] = g[b, p(i,j)],
// p(i,j) = i(i-1)/2 + j for i > j) -- the autodiff of DLRM's dot_op
// (modelzoo/DLRM/train.py:150-163: matmul(X, X^T) then the strictly-lower
// boolean mask).  A half-wave owns one sample, a lane one float4 column:
// the column of X stays in registers (F float4), the sample's S sits in LDS
// and is read as 16-B broadcasts.  HBM bound: X read + dX written once.
// ---------------------------------------------------------------------------
// CAT: the gradient arrives as the bf16 top-MLP input gradient [B, gstride]
// of dot_mfma_kernel<CAT> (x0 | pairs | padding): the pair coefficients are
// read from columns D.., and columns 0..D-1 (the concat's dense_inputs
// slot, i.e. X[b, 0, :] itself) are added to dX[b, 0, :] after the sum --
// the one fp32 add autograd does when the two uses of x0 meet.
template <int FM, bool CAT = false>
__global__ __launch_bounds__(256) void dot_grad_kernel(const float* __restrict__ x,
                                                       const void* __restrict__ gv, int64_t B,
                                                       int F, int D, float* __restrict__ dx,
                                                       int64_t gstride = 0) {
  // S of the half-wave's sample, zero-padded to FM x FM (row i = the
  // coefficients of dX[i]): no branches in the FMA loop, 16-B LDS reads.
  __shared__ __attribute__((aligned(16))) float ss_all[8][FM * FM];
  const int P = F * (F - 1) / 2;
  const int half = threadIdx.x >> 5, hl = threadIdx.x & 31;
  float* ss = ss_all[half];
  const int64_t b = (int64_t)blockIdx.x * 8 + half;
  const bool live = b < B;
  const float* gb = static_cast<const float*>(gv) + b * (int64_t)P;
  const uint16_t* gh = static_cast<const uint16_t*>(gv) + b * gstride;   // CAT
  for (int e = hl; e < FM * FM; e += 32) {
    const int i = e / FM, j = e - i * FM;
    float v = 0.f;
    if (live && i < F && j < F && i != j) {
      const int p = i > j ? i * (i - 1) / 2 + j : j * (j - 1) / 2 + i;
      v = CAT ? bf16_to_f32(gh[D + p]) : gb[p];
    }
    ss[e] = v;
  }
  __syncthreads();
  if (!live) return;
  const int D4 = D / 4;
  const float4* xb = reinterpret_cast<const float4*>(x + b * (int64_t)F * D);
  float4* ob = reinterpret_cast<float4*>(dx + b * (int64_t)F * D);
  for (int c = hl; c < D4; c += 32) {
    float4 xr[FM];
#pragma unroll
    for (int j = 0; j < FM; ++j)
      xr[j] = j < F ? nt_load(xb + j * D4 + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = 0; i < F; ++i) {
      const float4* srow = reinterpret_cast<const float4*>(ss + i * FM);
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int j4 = 0; j4 < FM / 4; ++j4) {
        const float4 s4 = srow[j4];
        const float sj[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 xv = xr[j4 * 4 + q];
          acc.x = fmaf(sj[q], xv.x, acc.x);
          acc.y = fmaf(sj[q], xv.y, acc.y);
          acc.z = fmaf(sj[q], xv.z, acc.z);
          acc.w = fmaf(sj[q], xv.w, acc.w);
        }
      }
      if (CAT && i == 0) {
        const uint2 h = *reinterpret_cast<const uint2*>(gh + c * 4);
        const float2 a = bf16x2_to_f2(h.x), d = bf16x2_to_f2(h.y);
        acc.x += a.x;
        acc.y += a.y;
        acc.z += d.x;
        acc.w += d.y;
      }
      nt_store(acc, ob + i * D4 + c);
    }
  }
}

// ---------------------------------------------------------------------------
// CrossNet layer: out[b,o] = x0[b,o] * (sum_k xl[b,k] W[o,k] + bias[o]) + xl[b,o]
// bf16 operands, fp32 accumulate, v_mfma_f32_16x16x32_bf16.
// Block tile 128 (rows of the batch) x 128 (output features), 4 waves as
// 2x2, each wave 64x64 = 4x4 MFMA tiles; K step 32 staged through LDS with
// rows padded to 80 B.  A = xl [B, d] and W [d, d] are both K-contiguous,
// so every fragment is one 16-B LDS read (lane l: row l&15, k 8(l>>4)..+7).
// ---------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  // round-to-nearest-even; NaN stays NaN
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffff) > 0x7f800000) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

static constexpr int CN_BM = 128, CN_BN = 128, CN_BK = 32, CN_LDS_ROW = 40;  // 40 shorts = 80 B

__global__ __launch_bounds__(256) void crossnet_kernel(const uint16_t* __restrict__ x0,
                                                       const uint16_t* __restrict__ xl,
                                                       const uint16_t* __restrict__ W,
                                                       const float* __restrict__ bias, int64_t M,
                                                       int d, uint16_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[CN_BM * CN_LDS_ROW];
  __shared__ __attribute__((aligned(16))) uint16_t sB[CN_BN * CN_LDS_ROW];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.y * CN_BM;
  const int n0 = blockIdx.x * CN_BN;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < d; k0 += CN_BK) {
    // stage: 128 rows x 4 chunks of 8 bf16 per operand = 512 chunks, 2 per thread
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + r * 256;
      const int row = c >> 2, kc = (c & 3) * 8;
      bf16x8 va = bf16x8{0, 0, 0, 0, 0, 0, 0, 0}, vb = va;
      const int64_t gm = m0 + row;
      const int gn = n0 + row;
      const int gk = k0 + kc;
      if (gm < M && gk < d) va = *reinterpret_cast<const bf16x8*>(xl + gm * d + gk);
      if (gn < d && gk < d) vb = *reinterpret_cast<const bf16x8*>(W + (int64_t)gn * d + gk);
      *reinterpret_cast<bf16x8*>(sA + row * CN_LDS_ROW + kc) = va;
      *reinterpret_cast<bf16x8*>(sB + row * CN_LDS_ROW + kc) = vb;
    }
    __syncthreads();
    bf16x8 fa[4], fb[4];
    const int fr = lane & 15, fk = (lane >> 4) * 8;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      fa[i] = *reinterpret_cast<const bf16x8*>(sA + (wm * 64 + i * 16 + fr) * CN_LDS_ROW + fk);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      fb[j] = *reinterpret_cast<const bf16x8*>(sB + (wn * 64 + j * 16 + fr) * CN_LDS_ROW + fk);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
  // epilogue: C/D map col = lane&15, row = (lane>>4)*4 + reg
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wn * 64 + j * 16 + (lane & 15);
      if (col >= d) continue;
      const float bv = bias ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (row >= M) continue;
        const float lin = acc[i][j][r] + bv;
        const float v = bf2f(x0[row * d + col]) * lin + bf2f(xl[row * d + col]);
        out[row * d + col] = f2bf(v);
      }
    }
}


// ---------------------------------------------------------------------------
// CrossNet layer, pipelined (d % 64 == 0): same 128 x 128 tile and 2 x 2 waves
// of 4 x 4 v_mfma_f32_16x16x32_bf16, K step 64, operands staged global -> LDS
// by global_load_lds_dwordx4 (no VGPR round trip) into two LDS buffers, so the
// DMA of K tile k+1 is in flight while tile k is multiplied.  One counted
// s_waitcnt vmcnt + one raw s_barrier per K step (a __syncthreads() would
// drain the prefetch with a vmcnt(0)), one s_barrier before a buffer is
// restaged.  LDS image: [128 rows][8 chunks of 16 B], chunk c of row r stored
// at c ^ ((r >> 1) & 7) (the swizzle is applied to the per-lane global source
// address; the DMA destination is wave base + lane * 16), so the 16 lanes of
// a fragment read hit 16 distinct 16-B bank slots.  Blocks are remapped so
// that the 8 XCDs each own a contiguous range of tiles (row tile major): the
// 27+ column tiles of one xl row panel share an XCD's L2.
// Optionally writes lin = xl W^T + b (bf16) for the backward pass.
// ---------------------------------------------------------------------------
static constexpr int CG_BM = 128, CG_BN = 128, CG_BK = 64;
static constexpr int CG_TILE_BYTES = CG_BM * CG_BK * 2;  // 16 KB per operand per buffer

template <int NI>
__device__ __forceinline__ void cg_stage_n(const uint16_t* __restrict__ X, int64_t rows_valid,
                                           int64_t row0, int d, int k0, char* lds_tile, int wave,
                                           int lane) {
  // NI wave instructions of 8 rows x 128 B per wave cover waves * NI * 8 rows
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r0 = (wave * NI + i) * 8;
    const int r = r0 + (lane >> 3);
    const int pc = lane & 7;
    const int lc = pc ^ ((r >> 1) & 7);
    int64_t gr = row0 + r;
    if (gr >= rows_valid) gr = rows_valid - 1;  // rows past the end feed discarded outputs
    const uint16_t* src = X + gr * (int64_t)d + k0 + lc * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(lds_tile + r0 * 128),
                                     16, 0, 0);
  }
}

__device__ __forceinline__ void cg_stage(const uint16_t* __restrict__ X, int64_t rows_valid,
                                         int64_t row0, int d, int k0, char* lds_tile, int wave,
                                         int lane) {
  cg_stage_n<4>(X, rows_valid, row0, d, k0, lds_tile, wave, lane);
}

__device__ __forceinline__ bf16x8 cg_frag(const char* lds_tile, int r, int lc) {
  return *reinterpret_cast<const bf16x8*>(lds_tile + r * 128 + ((lc ^ ((r >> 1) & 7)) << 4));
}

__global__ __launch_bounds__(256, 2) void crossnet_glds_kernel(
    const uint16_t* __restrict__ x0, const uint16_t* __restrict__ xl,
    const uint16_t* __restrict__ W, const float* __restrict__ bias, int64_t M, int d,
    int n_base, uint16_t* __restrict__ out, uint16_t* __restrict__ lin_out) {
  // output columns [n_base, d)
  __shared__ __attribute__((aligned(1024))) char lds[2 * 2 * CG_TILE_BYTES];  // [buf][A|B]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-contiguous tile order (bijective for any grid size)
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t orig = blockIdx.x;
  const int64_t xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t tile = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = (d - n_base) / CG_BN + ((d - n_base) % CG_BN ? 1 : 0);
  const int64_t m0 = (tile / ntn) * CG_BM;
  const int n0 = n_base + (int)(tile % ntn) * CG_BN;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = d / CG_BK;
  cg_stage(xl, M, m0, d, 0, lds, wave, lane);
  cg_stage(W, d, n0, d, 0, lds + CG_TILE_BYTES, wave, lane);
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = lds + (kt & 1) * 2 * CG_TILE_BYTES;
    if (kt + 1 < nk) {
      char* nxt = lds + ((kt + 1) & 1) * 2 * CG_TILE_BYTES;
      cg_stage(xl, M, m0, d, (kt + 1) * CG_BK, nxt, wave, lane);
      cg_stage(W, d, n0, d, (kt + 1) * CG_BK, nxt + CG_TILE_BYTES, wave, lane);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's tile-kt DMAs landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // ... and every other wave's
    asm volatile("" ::: "memory");
    const char* sA = cur;
    const char* sB = cur + CG_TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[4], fb[4];
      const int lc = kk * 4 + fq;
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = cg_frag(sA, wm * 64 + i * 16 + fr, lc);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = cg_frag(sB, wn * 64 + j * 16 + fr, lc);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // buffer kt&1 is restaged by iteration kt+1's DMA
    asm volatile("" ::: "memory");
  }
  // Epilogue through LDS (free after the loop's last barrier): each wave puts
  // its 64 x 64 fp32 accumulator tile into its own 16 KB region (C/D map col =
  // lane&15, row = (lane>>4)*4 + reg; columns XOR-swizzled by (row>>2)&3 x 16
  // so the four row groups of one store hit different banks), then reads it
  // back 8 columns per lane: x0 / xl / out / lin move as 16-B vectors, 8
  // lanes per 128-B row segment.
  float* ct = reinterpret_cast<float*>(lds) + wave * 64 * 64;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * 16 + fq * 4 + r;
        const int col = (j * 16 + fr) ^ (((row >> 2) & 3) << 4);
        ct[row * 64 + col] = acc[i][j][r];
      }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = it * 64 + lane;
    const int row = idx >> 3, cc = (idx & 7) * 8;
    const int64_t grow = m0 + wm * 64 + row;
    const int gcol = n0 + wn * 64 + cc;
    if (grow >= M || gcol >= d) continue;
    const int pc = cc ^ (((row >> 2) & 3) << 4);
    const float4 l0 = *reinterpret_cast<const float4*>(ct + row * 64 + pc);
    const float4 l1 = *reinterpret_cast<const float4*>(ct + row * 64 + pc + 4);
    float lin[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
    if (bias) {
      const float4 b0 = *reinterpret_cast<const float4*>(bias + gcol);
      const float4 b1 = *reinterpret_cast<const float4*>(bias + gcol + 4);
      lin[0] += b0.x; lin[1] += b0.y; lin[2] += b0.z; lin[3] += b0.w;
      lin[4] += b1.x; lin[5] += b1.y; lin[6] += b1.z; lin[7] += b1.w;
    }
    const int64_t o = grow * d + gcol;
    const u32x4 a0 = *reinterpret_cast<const u32x4*>(x0 + o);
    const u32x4 al = *reinterpret_cast<const u32x4*>(xl + o);
    u32x4 ov, lv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t p0 = a0[e], pl = al[e];
      const float v0 = bf2f((uint16_t)(p0 & 0xffff)) * lin[2 * e] + bf2f((uint16_t)(pl & 0xffff));
      const float v1 = bf2f((uint16_t)(p0 >> 16)) * lin[2 * e + 1] + bf2f((uint16_t)(pl >> 16));
      ov[e] = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
      lv[e] = (uint32_t)f2bf(lin[2 * e]) | ((uint32_t)f2bf(lin[2 * e + 1]) << 16);
    }
    *reinterpret_cast<u32x4*>(out + o) = ov;
    if (lin_out) *reinterpret_cast<u32x4*>(lin_out + o) = lv;
  }
}

// The same layer with a 256 x 128 tile, 8 waves (4 x 2, each 64 x 64) and
// three LDS stages (3 x 48 KB, one block per CU): two K tiles stay in
// flight, and a K step needs ONE barrier -- wait for this wave's DMAs of
// tile kt (vmcnt(6): tile kt+1's six may remain), s_barrier (every wave's
// landed, and every wave is done reading tile kt-1's buffer), then issue
// tile kt+2 into that buffer and multiply tile kt.
static constexpr int C3_BM = 256, C3_BN = 128, C3_BK = 64;
static constexpr int C3_A_BYTES = C3_BM * C3_BK * 2, C3_B_BYTES = C3_BN * C3_BK * 2;
static constexpr int C3_STAGE = C3_A_BYTES + C3_B_BYTES;  // 48 KB

__global__ __launch_bounds__(512, 1) void crossnet_glds3_kernel(
    const uint16_t* __restrict__ x0, const uint16_t* __restrict__ xl,
    const uint16_t* __restrict__ W, const float* __restrict__ bias, int64_t M, int d,
    uint16_t* __restrict__ out, uint16_t* __restrict__ lin_out) {
  __shared__ __attribute__((aligned(1024))) char lds[3 * C3_STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;  // 4 x 2 waves
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t orig = blockIdx.x;
  const int64_t xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t tile = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = d / C3_BN + (d % C3_BN ? 1 : 0);
  const int64_t m0 = (tile / ntn) * C3_BM;
  const int n0 = (int)(tile % ntn) * C3_BN;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = d / C3_BK;
  // prologue: tiles 0 and 1 in flight (6 DMAs per wave per tile)
  cg_stage_n<4>(xl, M, m0, d, 0, lds, wave, lane);
  cg_stage_n<2>(W, d, n0, d, 0, lds + C3_A_BYTES, wave, lane);
  if (nk > 1) {
    cg_stage_n<4>(xl, M, m0, d, C3_BK, lds + C3_STAGE, wave, lane);
    cg_stage_n<2>(W, d, n0, d, C3_BK, lds + C3_STAGE + C3_A_BYTES, wave, lane);
  }
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // tile kt landed (this wave)
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // ... every wave's, and tile kt-1's buffer is free
    asm volatile("" ::: "memory");
    if (kt + 2 < nk) {
      char* nxt = lds + ((kt + 2) % 3) * C3_STAGE;
      cg_stage_n<4>(xl, M, m0, d, (kt + 2) * C3_BK, nxt, wave, lane);
      cg_stage_n<2>(W, d, n0, d, (kt + 2) * C3_BK, nxt + C3_A_BYTES, wave, lane);
    }
    const char* sA = lds + (kt % 3) * C3_STAGE;
    const char* sB = sA + C3_A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[4], fb[4];
      const int lc = kk * 4 + fq;
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = cg_frag(sA, wm * 64 + i * 16 + fr, lc);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = cg_frag(sB, wn * 64 + j * 16 + fr, lc);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // every wave done with the last tile before LDS is reused
  asm volatile("" ::: "memory");
  // epilogue through LDS, as crossnet_glds_kernel (a 16 KB region per wave)
  float* ct = reinterpret_cast<float*>(lds) + wave * 64 * 64;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * 16 + fq * 4 + r;
        const int col = (j * 16 + fr) ^ (((row >> 2) & 3) << 4);
        ct[row * 64 + col] = acc[i][j][r];
      }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = it * 64 + lane;
    const int row = idx >> 3, cc = (idx & 7) * 8;
    const int64_t grow = m0 + wm * 64 + row;
    const int gcol = n0 + wn * 64 + cc;
    if (grow >= M || gcol >= d) continue;
    const int pc = cc ^ (((row >> 2) & 3) << 4);
    const float4 l0 = *reinterpret_cast<const float4*>(ct + row * 64 + pc);
    const float4 l1 = *reinterpret_cast<const float4*>(ct + row * 64 + pc + 4);
    float lin[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
    if (bias) {
      const float4 b0 = *reinterpret_cast<const float4*>(bias + gcol);
      const float4 b1 = *reinterpret_cast<const float4*>(bias + gcol + 4);
      lin[0] += b0.x; lin[1] += b0.y; lin[2] += b0.z; lin[3] += b0.w;
      lin[4] += b1.x; lin[5] += b1.y; lin[6] += b1.z; lin[7] += b1.w;
    }
    const int64_t o = grow * d + gcol;
    const u32x4 a0 = *reinterpret_cast<const u32x4*>(x0 + o);
    const u32x4 al = *reinterpret_cast<const u32x4*>(xl + o);
    u32x4 ov, lv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t p0 = a0[e], pl = al[e];
      const float v0 = bf2f((uint16_t)(p0 & 0xffff)) * lin[2 * e] + bf2f((uint16_t)(pl & 0xffff));
      const float v1 = bf2f((uint16_t)(p0 >> 16)) * lin[2 * e + 1] + bf2f((uint16_t)(pl >> 16));
      ov[e] = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
      lv[e] = (uint32_t)f2bf(lin[2 * e]) | ((uint32_t)f2bf(lin[2 * e + 1]) << 16);
    }
    *reinterpret_cast<u32x4*>(out + o) = ov;
    if (lin_out) *reinterpret_cast<u32x4*>(lin_out + o) = lv;
  }
}

// The same layer with a 256 x 256 tile: 8 waves as 2 (M) x 4 (N), each
// wave 128 x 64 (8 x 4 v_mfma_f32_16x16x32_bf16 accumulators), K step 64,
// both operands staged by global_load_lds_dwordx4 into two 64 KB LDS
// buffers (tile k+1's DMA in flight while tile k is multiplied; one counted
// vmcnt + s_barrier before the reads, one s_barrier before a buffer is
// restaged).  Why 256^2: the 128-wide tiles above read 8 fragments per 16
// MFMAs from LDS, which at 8 waves per CU is the LDS's whole bandwidth (the
// 824 TF ceiling measured in round 1); a 128 x 64 wave tile reads 12 per 32.
static constexpr int C4_BM = 256, C4_BN = 256, C4_BK = 64;
static constexpr int C4_OP_BYTES = C4_BM * C4_BK * 2;     // 32 KB per operand per buffer
static constexpr int C4_STAGE = 2 * C4_OP_BYTES;          // 64 KB

__global__ __launch_bounds__(512, 1) void crossnet_256_kernel(
    const uint16_t* __restrict__ x0, const uint16_t* __restrict__ xl,
    const uint16_t* __restrict__ W, const float* __restrict__ bias, int64_t M, int d,
    uint16_t* __restrict__ out, uint16_t* __restrict__ lin_out) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * C4_STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t orig = blockIdx.x;
  const int64_t xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t tile = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = d / C4_BN + (d % C4_BN ? 1 : 0);
  const int64_t m0 = (tile / ntn) * C4_BM;
  const int n0 = (int)(tile % ntn) * C4_BN;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = d / C4_BK;
  cg_stage_n<4>(xl, M, m0, d, 0, lds, wave, lane);
  cg_stage_n<4>(W, d, n0, d, 0, lds + C4_OP_BYTES, wave, lane);
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = lds + (kt & 1) * C4_STAGE;
    if (kt + 1 < nk) {
      char* nxt = lds + ((kt + 1) & 1) * C4_STAGE;
      cg_stage_n<4>(xl, M, m0, d, (kt + 1) * C4_BK, nxt, wave, lane);
      cg_stage_n<4>(W, d, n0, d, (kt + 1) * C4_BK, nxt + C4_OP_BYTES, wave, lane);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's tile-kt DMAs landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // ... and every other wave's
    asm volatile("" ::: "memory");
    const char* sA = cur;
    const char* sB = cur + C4_OP_BYTES;
#ifndef DR_C4_BATCHED_FRAGS
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[8], fb[4];
      const int lc = kk * 4 + fq;
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = cg_frag(sB, wc * 64 + j * 16 + fr, lc);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = cg_frag(sA, wr * 128 + i * 16 + fr, lc);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
#else
    // all 24 fragment reads of the K step issued up front: the second k
    // half's reads overlap the first half's MFMAs (224 VGPRs)
    bf16x8 fa[2][8], fb[2][4];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int lc = kk * 4 + fq;
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[kk][j] = cg_frag(sB, wc * 64 + j * 16 + fr, lc);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[kk][i] = cg_frag(sA, wr * 128 + i * 16 + fr, lc);
    }
    // keep the reads ahead of the MFMAs: left alone, the scheduler sinks
    // each read to its first use and waits lgkmcnt(0) every 8 MFMAs
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][i], fb[kk][j], acc[i][j], 0, 0, 0);
#endif
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // buffer kt&1 is restaged by iteration kt+1's DMA
    asm volatile("" ::: "memory");
  }
  // Epilogue in two row halves of the wave tile (LDS: 8 waves x 16 KB), each
  // as in crossnet_glds_kernel: accumulators -> swizzled fp32 image -> 8
  // columns per lane, so x0 / xl / out / lin move as 16-B vectors.
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
  float* ct = reinterpret_cast<float*>(lds) + wave * 64 * 64;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();   // this wave's region is free again
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + fq * 4 + r;
          const int col = (j * 16 + fr) ^ (((row >> 2) & 3) << 4);
          ct[row * 64 + col] = acc[h * 4 + i][j][r];
        }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int idx = it * 64 + lane;
      const int row = idx >> 3, cc = (idx & 7) * 8;
      const int64_t grow = m0 + wr * 128 + h * 64 + row;
      const int gcol = n0 + wc * 64 + cc;
      if (grow >= M || gcol >= d) continue;
      const int pc = cc ^ (((row >> 2) & 3) << 4);
      const float4 l0 = *reinterpret_cast<const float4*>(ct + row * 64 + pc);
      const float4 l1 = *reinterpret_cast<const float4*>(ct + row * 64 + pc + 4);
      float lin[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
      if (bias) {
        const float4 b0 = *reinterpret_cast<const float4*>(bias + gcol);
        const float4 b1 = *reinterpret_cast<const float4*>(bias + gcol + 4);
        lin[0] += b0.x; lin[1] += b0.y; lin[2] += b0.z; lin[3] += b0.w;
        lin[4] += b1.x; lin[5] += b1.y; lin[6] += b1.z; lin[7] += b1.w;
      }
      const int64_t o = grow * d + gcol;
      const u32x4 a0 = *reinterpret_cast<const u32x4*>(x0 + o);
      const u32x4 al = *reinterpret_cast<const u32x4*>(xl + o);
      u32x4 ov, lv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t p0 = a0[e], pl = al[e];
        const float v0 = bf2f((uint16_t)(p0 & 0xffff)) * lin[2 * e] + bf2f((uint16_t)(pl & 0xffff));
        const float v1 = bf2f((uint16_t)(p0 >> 16)) * lin[2 * e + 1] + bf2f((uint16_t)(pl >> 16));
        ov[e] = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
        lv[e] = (uint32_t)f2bf(lin[2 * e]) | ((uint32_t)f2bf(lin[2 * e + 1]) << 16);
      }
      *reinterpret_cast<u32x4*>(out + o) = ov;
      if (lin_out) *reinterpret_cast<u32x4*>(lin_out + o) = lv;
    }
  }
}

// The 256 x 256 layer with the two wave groups STAGGERED by one barrier, so
// that on every SIMD one wave multiplies while its partner stages and waits
// (waves w and w+4 share a SIMD; group g = w / 4 owns output rows
// g*128..+127).  Per K step each wave runs  [issue DMAs of tile k+1; counted
// vmcnt for tile k] barrier [24 fragment reads + 64 MFMAs] barrier,  group 1
// one barrier behind group 0, so the MFMA windows of the two groups
// alternate.  The stagger moves a shared buffer's last read one window later,
// so: the A half-tiles are group-private (each group stages its own 128 rows,
// 2 buffers), and B -- read by both groups -- is staged by group 0 alone into
// 3 buffers (2 x 32 KB + 3 x 32 KB = 160 KB).  Ordering, windows n between
// barriers n and n+1 (group 0 computes tile k in window 2k, group 1 in 2k+1):
//   RAW  B(k+1), A_top(k+1): issued by group 0 in window 2k-1, vmcnt-retired
//        before barrier 2k+2, read in windows 2k+2 / 2k+3;  A_bot(k+1): issued
//        by group 1 in window 2k, retired before barrier 2k+3, read in 2k+3.
//   WAR  B buffer (k+1)%3 last held tile k-2, whose last reads (group 1, window
//        2k-3) retired before barrier 2k-2; A buffers: the owner group's last
//        reads of tile k-1 retired one barrier before its next DMA.
static constexpr int CS_A_BYTES = 256 * 128;   // one A tile (two 128-row halves)
static constexpr int CS_B_BYTES = 256 * 128;
static constexpr int CS_LDS = 2 * CS_A_BYTES + 3 * CS_B_BYTES;  // 160 KB

__global__ __launch_bounds__(512, 1) void crossnet_stag_kernel(
    const uint16_t* __restrict__ x0, const uint16_t* __restrict__ xl,
    const uint16_t* __restrict__ W, const float* __restrict__ bias, int64_t M, int d,
    uint16_t* __restrict__ out, uint16_t* __restrict__ lin_out) {
  __shared__ __attribute__((aligned(1024))) char lds[CS_LDS];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const bool g1 = wr != 0;
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t orig = blockIdx.x;
  const int64_t xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t tile = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = d / 256 + (d % 256 ? 1 : 0);
  const int64_t m0 = (tile / ntn) * 256;
  const int n0 = (int)(tile % ntn) * 256;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = d / 64;
  char* const bbase = lds + 2 * CS_A_BYTES;
  auto stage = [&](int kt) {
    const int k0 = kt * 64;
    char* a = lds + (kt & 1) * CS_A_BYTES;
    if (!g1) {
      cg_stage_n<4>(xl, M, m0, d, k0, a, wc, lane);
      cg_stage_n<8>(W, d, n0, d, k0, bbase + (kt % 3) * CS_B_BYTES, wc, lane);
    } else {
      cg_stage_n<4>(xl, M, m0 + 128, d, k0, a + 128 * 128, wc, lane);
    }
  };
  stage(0);
  if (g1) __builtin_amdgcn_s_barrier();  // the stagger: group 1 one barrier behind
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) {
      stage(kt + 1);
      if (!g1)
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // tile kt's 12 DMAs of this wave
      else
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const char* sA = lds + (kt & 1) * CS_A_BYTES;
    const char* sB = bbase + (kt % 3) * CS_B_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[8], fb[4];
      const int lc = kk * 4 + fq;
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = cg_frag(sB, wc * 64 + j * 16 + fr, lc);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = cg_frag(sA, wr * 128 + i * 16 + fr, lc);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if (!g1) __builtin_amdgcn_s_barrier();  // matches group 1's extra barrier
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
  float* ct = reinterpret_cast<float*>(lds) + wave * 64 * 64;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + fq * 4 + r;
          const int col = (j * 16 + fr) ^ (((row >> 2) & 3) << 4);
          ct[row * 64 + col] = acc[h * 4 + i][j][r];
        }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int idx = it * 64 + lane;
      const int row = idx >> 3, cc = (idx & 7) * 8;
      const int64_t grow = m0 + wr * 128 + h * 64 + row;
      const int gcol = n0 + wc * 64 + cc;
      if (grow >= M || gcol >= d) continue;
      const int pc = cc ^ (((row >> 2) & 3) << 4);
      const float4 l0 = *reinterpret_cast<const float4*>(ct + row * 64 + pc);
      const float4 l1 = *reinterpret_cast<const float4*>(ct + row * 64 + pc + 4);
      float lin[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
      if (bias) {
        const float4 b0 = *reinterpret_cast<const float4*>(bias + gcol);
        const float4 b1 = *reinterpret_cast<const float4*>(bias + gcol + 4);
        lin[0] += b0.x; lin[1] += b0.y; lin[2] += b0.z; lin[3] += b0.w;
        lin[4] += b1.x; lin[5] += b1.y; lin[6] += b1.z; lin[7] += b1.w;
      }
      const int64_t o = grow * d + gcol;
      const u32x4 a0 = *reinterpret_cast<const u32x4*>(x0 + o);
      const u32x4 al = *reinterpret_cast<const u32x4*>(xl + o);
      u32x4 ov, lv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t p0 = a0[e], pl = al[e];
        const float v0 = bf2f((uint16_t)(p0 & 0xffff)) * lin[2 * e] + bf2f((uint16_t)(pl & 0xffff));
        const float v1 = bf2f((uint16_t)(p0 >> 16)) * lin[2 * e + 1] + bf2f((uint16_t)(pl >> 16));
        ov[e] = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
        lv[e] = (uint32_t)f2bf(lin[2 * e]) | ((uint32_t)f2bf(lin[2 * e + 1]) << 16);
      }
      *reinterpret_cast<u32x4*>(out + o) = ov;
      if (lin_out) *reinterpret_cast<u32x4*>(lin_out + o) = lv;
    }
  }
}

// ---------------------------------------------------------------------------
// The 256 x 256 layer with four phases per K tile (the guide's 8-phase
// schedule, two K tiles per 8 phases).  Each wave owns 128 x 64 outputs as
// four 64 x 32 quadrants; a phase multiplies ONE quadrant over K = 64 (16
// MFMAs).  The LDS tile is cut into half-tiles that each phase reads once:
//   A_h0 = the first 64 rows of both wave groups' 128-row halves,
//   A_h1 = their last 64 rows, B_h0 / B_h1 = the first / last 32 of every
//   wave's 64 output columns (W rows),
// so phase 1 reads A_h0 + B_h0 (quadrant m0n0), phase 2 B_h1 (m0n1), phase 3
// A_h1 (m1n0, B_h0 still in registers), phase 4 nothing (m1n1).  One
// half-tile is staged per phase (2 global_load_lds per thread):
//   p1: A_h1(t+1)   p2: A_h0(t+2)   p3: B_h0(t+2)   p4: B_h1(t+2)
// each into a half that was last read at least one phase earlier, and
// s_waitcnt vmcnt(6) in p4 retires tile t+1 while tile t+2's three halves
// stay in flight across the barriers.  The two wave groups (waves w, w+4
// share a SIMD) run staggered by one barrier: between two barriers one group
// multiplies (s_setprio 1) while the other issues its LDS reads and DMAs.
// Ordering (window n = between barriers n and n+1; group g reads phase p in
// window 2p+g and multiplies it in 2p+1+g):
//   WAR  every wave retires its reads with lgkmcnt(0) BEFORE the barrier
//        that closes its read window, so a DMA issued one phase later (by
//        either group) cannot overtake them;
//   RAW  every wave retires its own DMAs with the counted vmcnt before the
//        barrier that closes its p4 read window; reads of that tile start in
//        the next phase, after a barrier every wave passed behind its wait.
// ---------------------------------------------------------------------------
static constexpr int C8_HALF = 128 * 128;  // one half-tile image: 128 rows x 64 bf16
static constexpr int C8_BUF = 4 * C8_HALF;  // [A_h0 | A_h1 | B_h0 | B_h1]

// Stage one half-tile: image row r (0..127) <- global row row0 + map(r),
// 2 wave instructions of 8 rows x 128 B per wave.  AH: A half (image row r ->
// tile row (r >> 6) * 128 + h * 64 + (r & 63)); otherwise B half (r -> tile
// col (r >> 5) * 64 + h * 32 + (r & 31)).
template <bool AH>
__device__ __forceinline__ void c8_stage(const uint16_t* __restrict__ X, int64_t rows_valid,
                                         int64_t row0, int h, int d, int k0, char* img, int wave,
                                         int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r0 = (wave * 2 + i) * 8;
    const int r = r0 + (lane >> 3);
    const int lc = (lane & 7) ^ ((r >> 1) & 7);
    const int tr = AH ? ((r >> 6) * 128 + h * 64 + (r & 63)) : ((r >> 5) * 64 + h * 32 + (r & 31));
    int64_t gr = row0 + tr;
    if (gr >= rows_valid) gr = rows_valid - 1;  // rows past the end feed discarded outputs
    const uint16_t* src = X + gr * (int64_t)d + k0 + lc * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(img + r0 * 128),
                                     16, 0, 0);
  }
}

// MODE 1: the cross layer, out = x0 * (xl W^T + b) + xl (lin_out = xl W^T + b);
// MODE 2: the layer's input gradient, out = xl W^T + x0 -- called with A = u,
// W = the transposed weight and x0 = g, it is dx_l = u W + g (no bias);
// MODE 0: the loop alone (timing build, no outputs).
template <int MODE, int GM, bool PIPE>
__global__ __launch_bounds__(512, 1) void crossnet_8ph_kernel(
    const uint16_t* __restrict__ x0, const uint16_t* __restrict__ xl,
    const uint16_t* __restrict__ W, const float* __restrict__ bias, int64_t M, int d,
    int ncols, uint16_t* __restrict__ out, uint16_t* __restrict__ lin_out) {
  // output columns [0, ncols) (ncols <= d; K and the row stride are d)
  __shared__ __attribute__((aligned(1024))) char lds[2 * C8_BUF];  // 128 KB
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const bool g1 = wr != 0;
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t orig = blockIdx.x;
  const int64_t xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t tile = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = ncols / 256 + (ncols % 256 ? 1 : 0);
  int64_t m0;
  int n0;
  if (GM <= 1) {  // row-major: an XCD's running tiles span ~2 row panels x all columns
    m0 = (tile / ntn) * 256;
    n0 = (int)(tile % ntn) * 256;
  } else {  // groups of GM row panels walked column-major: GM x (32 / GM) running tiles
    const int64_t ntm = (M + 255) / 256;
    const int64_t g = tile / ((int64_t)GM * ntn), idx = tile % ((int64_t)GM * ntn);
    const int64_t rows = ntm - g * GM < GM ? ntm - g * GM : GM;
    m0 = (g * GM + idx % rows) * 256;
    n0 = (int)(idx / rows) * 256;
  }
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = d / 64;
  auto img = [&](int t, int part) -> char* { return lds + (t & 1) * C8_BUF + part * C8_HALF; };
  auto st_a = [&](int t, int h) { c8_stage<true>(xl, M, m0, h, d, t * 64, img(t, h), wave, lane); };
  auto st_b = [&](int t, int h) {
    c8_stage<false>(W, d, n0, h, d, t * 64, img(t, 2 + h), wave, lane);
  };
  // prologue: tile 0 whole, tile 1 but its A_h1 (issued in tile 0's p1)
  st_a(0, 0); st_b(0, 0); st_b(0, 1); st_a(0, 1);
  if (nk > 1) {
    st_a(1, 0); st_b(1, 0); st_b(1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (g1) __builtin_amdgcn_s_barrier();  // the stagger
  asm volatile("" ::: "memory");
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];  // [frag][kk]
  auto read_a = [&](const char* s) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[i][kk] = cg_frag(s, wr * 64 + i * 16 + fr, kk * 4 + fq);
  };
  auto read_b = [&](const char* s, bf16x8 (&fb)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb[j][kk] = cg_frag(s, wc * 32 + j * 16 + fr, kk * 4 + fq);
  };
  auto close_read = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto mma = [&](int mi, bf16x8 (&fb)[2][2], int nj) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mi + i][nj + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][kk], fb[j][kk], acc[mi + i][nj + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  for (int t = 0; t < nk; ++t) {
    const bool pf1 = t + 1 < nk, pf2 = t + 2 < nk;
    // p1: m0n0
    read_b(img(t, 2), fb0);
    read_a(img(t, 0));
    if (pf1) st_a(t + 1, 1);
    close_read();
    mma(0, fb0, 0);
    // p2: m0n1
    read_b(img(t, 3), fb1);
    if (pf2) st_a(t + 2, 0);
    close_read();
    mma(0, fb1, 2);
    // p3: m1n0
    read_a(img(t, 1));
    if (pf2) st_b(t + 2, 0);
    close_read();
    mma(4, fb0, 0);
    // p4: m1n1
    if (pf2) {
      st_b(t + 2, 1);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // tile t+1 landed (this wave's DMAs)
    } else if (pf1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    close_read();
    mma(4, fb1, 2);
  }
  if (!g1) __builtin_amdgcn_s_barrier();  // matches group 1's extra barrier
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if (MODE == 0) {  // loop-only timing build: keep the MFMAs alive, store nothing
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sum == 1234.5678f) out[0] = 0;
    return;
  }
  // Epilogue: per 64-row half, this wave's x0 / xl vectors are requested
  // first (addresses clamped, stores predicated), the accumulators go
  // through LDS (C/D map -> 8 columns per lane), then out / lin are formed
  // and stored as 16-B vectors.
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
  float* ct = reinterpret_cast<float*>(lds) + wave * 64 * 64;
  const int cc = (lane & 7) * 8;
  const int gcol = n0 + wc * 64 + cc;
  const bool col_ok = gcol < ncols;
  const int gcol_c = col_ok ? gcol : d - 8;
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(bias + gcol_c);
    const float4 b1 = *reinterpret_cast<const float4*>(bias + gcol_c + 4);
    bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w;
    bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
  }
  // x0 / xl vectors of rows [h*64, h*64+64) of this wave's 128 (addresses
  // clamped; stores are predicated instead)
  auto load_half = [&](int h, u32x4 (&a0)[8], u32x4 (&al)[8]) {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      int64_t grow = m0 + wr * 128 + h * 64 + it * 8 + (lane >> 3);
      if (grow >= M) grow = M - 1;
      const int64_t o = grow * d + gcol_c;
      a0[it] = *reinterpret_cast<const u32x4*>(x0 + o);
      if (MODE == 1) al[it] = *reinterpret_cast<const u32x4*>(xl + o);
    }
  };
  auto acc_to_lds = [&](int h) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + fq * 4 + r;
          const int col = (j * 16 + fr) ^ (((row >> 2) & 3) << 4);
          ct[row * 64 + col] = acc[h * 4 + i][j][r];
        }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto finish_half = [&](int h, const u32x4 (&a0)[8], const u32x4 (&al)[8]) {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int row = it * 8 + (lane >> 3);
      const int64_t grow = m0 + wr * 128 + h * 64 + row;
      const int pc = cc ^ (((row >> 2) & 3) << 4);
      const float4 l0 = *reinterpret_cast<const float4*>(ct + row * 64 + pc);
      const float4 l1 = *reinterpret_cast<const float4*>(ct + row * 64 + pc + 4);
      float lin[8] = {l0.x + bv[0], l0.y + bv[1], l0.z + bv[2], l0.w + bv[3],
                      l1.x + bv[4], l1.y + bv[5], l1.z + bv[6], l1.w + bv[7]};
      u32x4 ov, lv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t p0 = a0[it][e];
        if (MODE == 1) {
          const uint32_t pl = al[it][e];
          const float v0 = bf2f((uint16_t)(p0 & 0xffff)) * lin[2 * e] + bf2f((uint16_t)(pl & 0xffff));
          const float v1 = bf2f((uint16_t)(p0 >> 16)) * lin[2 * e + 1] + bf2f((uint16_t)(pl >> 16));
          ov[e] = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
          lv[e] = (uint32_t)f2bf(lin[2 * e]) | ((uint32_t)f2bf(lin[2 * e + 1]) << 16);
        } else {  // one fp32 sum of the product and the addend, one rounding
          const float v0 = lin[2 * e] + bf2f((uint16_t)(p0 & 0xffff));
          const float v1 = lin[2 * e + 1] + bf2f((uint16_t)(p0 >> 16));
          ov[e] = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
        }
      }
      if (grow < M && col_ok) {
        const int64_t o = grow * d + gcol;
        *reinterpret_cast<u32x4*>(out + o) = ov;
        if (MODE == 1 && lin_out) *reinterpret_cast<u32x4*>(lin_out + o) = lv;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ct reads done before it is rewritten
    __builtin_amdgcn_wave_barrier();
  };
  if (PIPE) {  // h = 1's loads in flight while h = 0 is formed and stored
    u32x4 a00[8], al0[8], a01[8], al1[8];
    load_half(0, a00, al0);
    acc_to_lds(0);
    load_half(1, a01, al1);
    finish_half(0, a00, al0);
    acc_to_lds(1);
    finish_half(1, a01, al1);
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      u32x4 a0[8], al[8];
      load_half(h, a0, al);
      acc_to_lds(h);
      finish_half(h, a0, al);
    }
  }
}

// ---------------------------------------------------------------------------
// The 256 x 256 layer at ONE wave per SIMD (crossnet_w4_kernel): 4 waves of
// 128 x 128 outputs each (8 x 8 v_mfma_f32_16x16x32_bf16 tiles = 256
// accumulator registers per lane).  The accumulators are pinned in AGPRs by
// issuing the MFMAs as inline asm with "+a" operands (written with the
// builtin, the register allocator rotated them through VGPRs: ~440 accvgpr
// moves per 128 MFMAs, round 4).  No barrier-locked pairing of two waves per
// SIMD: each wave keeps its matrix pipe busy on its own, 64 MFMAs (1024
// cycles) per K step of 32 between two barriers.
//   * LDS: a ring of 4 K-32 stages [A 256 x 64 B | B 256 x 64 B] (128 KB),
//     filled by global_load_lds three stages ahead; 16-B chunk c of image row
//     r stored at c ^ (((r >> 2) & 1) << 1) -- the four ds_read_b128 lane
//     groups of a fragment read hit 16 distinct slots (conflict-free);
//   * fragments one stage ahead: the 16 reads of stage s + 1 are issued
//     before the 64 MFMAs of stage s, which use registers filled one
//     iteration earlier;
//   * ordering per iteration s: counted vmcnt (this wave's DMAs of stage s+1
//     landed) then s_barrier (every wave's), then the DMA of stage s+3 into
//     the slot stage s-1 left -- whose fragments every wave consumed (its
//     MFMAs waited for them) before it reached this barrier.
// ---------------------------------------------------------------------------
static constexpr int W4_IMG = 256 * 64;        // one operand's K-32 stage image
static constexpr int W4_BUF = 2 * W4_IMG;      // [A | B]

__device__ __forceinline__ int w4_sw(int r) { return ((r >> 2) & 1) << 1; }

// image rows [wave * 64, wave * 64 + 64) <- global rows row0 + r, k0..k0+31:
// 4 wave instructions of 16 rows x 64 B
__device__ __forceinline__ void w4_stage(const uint16_t* __restrict__ X, int64_t rows_valid,
                                         int64_t row0, int d, int k0, char* img, int wave,
                                         int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r0 = (wave * 4 + i) * 16;
    const int r = r0 + (lane >> 2);
    const int c = (lane & 3) ^ w4_sw(r);
    int64_t gr = row0 + r;
    if (gr >= rows_valid) gr = rows_valid - 1;  // rows past the end feed discarded outputs
    const uint16_t* src = X + gr * (int64_t)d + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(img + r0 * 64),
                                     16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 w4_frag(const char* img, int r, int c) {
  return *reinterpret_cast<const bf16x8*>(img + r * 64 + ((c ^ w4_sw(r)) << 4));
}

#define W4_MFMA(C, A, B) \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(C) : "v"(A), "v"(B))

// MODE 1: out = x0 * (xl W^T + b) + xl (lin_out = xl W^T + b); MODE 2: out =
// xl W^T + x0 (the input gradient, as crossnet_8ph_kernel); MODE 0: the loop
// alone (timing build).
template <int MODE, int GM, bool IL>
__global__ __launch_bounds__(256, 1) void crossnet_w4_kernel(
    const uint16_t* __restrict__ x0, const uint16_t* __restrict__ xl,
    const uint16_t* __restrict__ W, const float* __restrict__ bias, int64_t M, int d,
    int ncols, uint16_t* __restrict__ out, uint16_t* __restrict__ lin_out) {
  __shared__ __attribute__((aligned(1024))) char lds[4 * W4_BUF];  // 128 KB
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t orig = blockIdx.x;
  const int64_t xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t tile = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = ncols / 256 + (ncols % 256 ? 1 : 0);
  int64_t m0;
  int n0;
  {  // groups of GM row panels walked column-major (crossnet_8ph_kernel)
    const int64_t ntm = (M + 255) / 256;
    const int64_t g = tile / ((int64_t)GM * ntn), idx = tile % ((int64_t)GM * ntn);
    const int64_t rows = ntm - g * GM < GM ? ntm - g * GM : GM;
    m0 = (g * GM + idx % rows) * 256;
    n0 = (int)(idx / rows) * 256;
  }
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = d / 32;
  auto img = [&](int s) -> char* { return lds + (s & 3) * W4_BUF; };
  auto stage = [&](int s) {
    w4_stage(xl, M, m0, d, s * 32, img(s), wave, lane);
    w4_stage(W, d, n0, d, s * 32, img(s) + W4_IMG, wave, lane);
  };
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 F0[16], F1[16];   // [0, 8): A fragments (rows), [8, 16): B fragments (columns)
  auto read = [&](int s, bf16x8 (&F)[16]) {
    const char* a = img(s);
    const char* b = a + W4_IMG;
#pragma unroll
    for (int i = 0; i < 8; ++i) F[i] = w4_frag(a, wr * 128 + i * 16 + fr, fq);
#pragma unroll
    for (int j = 0; j < 8; ++j) F[8 + j] = w4_frag(b, wc * 128 + j * 16 + fr, fq);
  };
  auto mma = [&](bf16x8 (&F)[16]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) W4_MFMA(acc[i][j], F[i], F[8 + j]);
  };
  // IL: the 16 fragment reads (inline asm, so they keep their place) and the
  // 8 DMA pieces of stage s + 3 spread over the 64 MFMAs -- a read after
  // every 4th MFMA, a DMA piece after every 8th -- instead of issued in a
  // block in front of them.  The DMAs are unconditional (past the last stage
  // they reload stage nk - 1 into the slot stage s - 1 left: dead data), so
  // vmcnt(8) always means "stage s + 1 landed".
  typedef __attribute__((address_space(3))) char lds_t;
  const uint32_t lb = (uint32_t)(fr * 64 + ((fq ^ w4_sw(fr)) << 4));
  auto dma_piece = [&](int s3, int p) {
    const int k0 = s3 * 32;
    const int i = p & 3;
    const int r0 = (wave * 4 + i) * 16;
    const int r = r0 + (lane >> 2);
    const int c = (lane & 3) ^ w4_sw(r);
    char* dst = img(s3) + (p >> 2) * W4_IMG + r0 * 64;
    const uint16_t* X = (p >> 2) ? W : xl;
    const int64_t rv = (p >> 2) ? (int64_t)d : M;
    int64_t gr = ((p >> 2) ? (int64_t)n0 : m0) + r;
    if (gr >= rv) gr = rv - 1;
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(X + gr * (int64_t)d + k0 + c * 8),
        (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  };
  // The fragment reads are inline asm, so the compiler takes their
  // registers as written at issue: a read whose result it deems dead (the
  // last iteration's Fn) or copies early lets it recycle the register while
  // the LDS return is in flight.  Every wait on them therefore names them
  // ("+v"), keeping them live and in place up to it.
  auto tie16 = [&](bf16x8 (&F)[16]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(F[0]), "+v"(F[1]), "+v"(F[2]), "+v"(F[3]), "+v"(F[4]), "+v"(F[5]),
                   "+v"(F[6]), "+v"(F[7])::"memory");
    asm volatile(""
                 : "+v"(F[8]), "+v"(F[9]), "+v"(F[10]), "+v"(F[11]), "+v"(F[12]), "+v"(F[13]),
                   "+v"(F[14]), "+v"(F[15])::"memory");
  };
  auto iter_il = [&](int s, bf16x8 (&Fc)[16], bf16x8 (&Fn)[16]) {
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): Fc complete
    tie16(Fc);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // stage s+1 landed (this wave's DMAs)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int s1 = s + 1 < nk ? s + 1 : s;
    const int s3 = s + 3 < nk ? s + 3 : nk - 1;
    const uint32_t ra = (uint32_t)(size_t)(lds_t*)img(s1) + lb + wr * 8192;
    const uint32_t rb = (uint32_t)(size_t)(lds_t*)img(s1) + W4_IMG + lb + wc * 8192;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        W4_MFMA(acc[i][j], Fc[i], Fc[8 + j]);
        const int m = i * 8 + j;
        if ((m & 3) == 3) {
          const int k = m >> 2;   // 0..15
          if (k < 8)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(Fn[k]) : "v"(ra), "i"(k * 1024));
          else
            asm volatile("ds_read_b128 %0, %1 offset:%2"
                         : "=v"(Fn[k]) : "v"(rb), "i"((k - 8) * 1024));
        }
        if ((m & 7) == 1) dma_piece(s3, m >> 3);
      }
  };
  auto iter = [&](int s, bf16x8 (&Fc)[16], bf16x8 (&Fn)[16]) {
    // Fc (read one iteration ago) complete -- as a real s_waitcnt the
    // compiler's wait pass sees, so it puts no lgkmcnt(0) behind this
    // iteration's reads in front of the MFMAs
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
    tie16(Fc);
    if (s + 2 < nk)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // stage s+1 landed (this wave's DMAs)
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + 3 < nk) stage(s + 3);
    read(s + 1 < nk ? s + 1 : s, Fn);   // unconditional (a branch would end in a wait)
    mma(Fc);
  };
  if (IL) {   // prologue: stages 0..2 (clamped), stage 0 landed
    for (int p = 0; p < 8; ++p) dma_piece(0, p);
    for (int p = 0; p < 8; ++p) dma_piece(1 < nk ? 1 : nk - 1, p);
    for (int p = 0; p < 8; ++p) dma_piece(2 < nk ? 2 : nk - 1, p);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
  stage(0);
  if (nk > 1) stage(1);
  if (nk > 2) stage(2);
  if (nk > 2)
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (nk > 1)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read(0, F0);
  int s = 0;
  if (IL) {
    for (; s + 1 < nk; s += 2) {
      iter_il(s, F0, F1);
      iter_il(s + 1, F1, F0);
    }
    if (s < nk) iter_il(s, F0, F1);
  } else {
    for (; s + 1 < nk; s += 2) {
      iter(s, F0, F1);
      iter(s + 1, F1, F0);
    }
    if (s < nk) iter(s, F0, F1);
  }
  tie16(F0);
  tie16(F1);
  // the last MFMAs' results are read below (AGPR -> VGPR): cover their latency
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();   // every wave's last fragment reads done: the ring is reused below
  if (MODE == 0) {
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sum == 1234.5678f) out[0] = 0;
    return;
  }
  // Epilogue by 64 x 64 quarters (row half h, column half g): this wave's x0
  // / xl vectors requested first, the accumulators through LDS (C/D map -> 8
  // columns per lane), then out / lin formed and stored as 16-B vectors.
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
  float* ct = reinterpret_cast<float*>(lds) + wave * 64 * 64;
  const int cc = (lane & 7) * 8;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int gcol = n0 + wc * 128 + g * 64 + cc;
    const bool col_ok = gcol < ncols;
    const int gcol_c = col_ok ? gcol : d - 8;
    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (MODE == 1 && bias) {
      const float4 b0 = *reinterpret_cast<const float4*>(bias + gcol_c);
      const float4 b1 = *reinterpret_cast<const float4*>(bias + gcol_c + 4);
      bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w;
      bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      u32x4 a0[8], al[8];
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        int64_t grow = m0 + wr * 128 + h * 64 + it * 8 + (lane >> 3);
        if (grow >= M) grow = M - 1;
        const int64_t o = grow * d + gcol_c;
        a0[it] = *reinterpret_cast<const u32x4*>(x0 + o);
        if (MODE == 1) al[it] = *reinterpret_cast<const u32x4*>(xl + o);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = i * 16 + fq * 4 + r;
            const int col = (j * 16 + fr) ^ (((row >> 2) & 3) << 4);
            ct[row * 64 + col] = acc[h * 4 + i][g * 4 + j][r];
          }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int row = it * 8 + (lane >> 3);
        const int64_t grow = m0 + wr * 128 + h * 64 + row;
        const int pc = cc ^ (((row >> 2) & 3) << 4);
        const float4 l0 = *reinterpret_cast<const float4*>(ct + row * 64 + pc);
        const float4 l1 = *reinterpret_cast<const float4*>(ct + row * 64 + pc + 4);
        float lin[8] = {l0.x + bv[0], l0.y + bv[1], l0.z + bv[2], l0.w + bv[3],
                        l1.x + bv[4], l1.y + bv[5], l1.z + bv[6], l1.w + bv[7]};
        u32x4 ov, lv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t p0 = a0[it][e];
          if (MODE == 1) {
            const uint32_t pl = al[it][e];
            const float v0 = bf2f((uint16_t)(p0 & 0xffff)) * lin[2 * e] + bf2f((uint16_t)(pl & 0xffff));
            const float v1 = bf2f((uint16_t)(p0 >> 16)) * lin[2 * e + 1] + bf2f((uint16_t)(pl >> 16));
            ov[e] = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
            lv[e] = (uint32_t)f2bf(lin[2 * e]) | ((uint32_t)f2bf(lin[2 * e + 1]) << 16);
          } else {  // one fp32 sum of the product and the addend, one rounding
            const float v0 = lin[2 * e] + bf2f((uint16_t)(p0 & 0xffff));
            const float v1 = lin[2 * e + 1] + bf2f((uint16_t)(p0 >> 16));
            ov[e] = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
          }
        }
        if (grow < M && col_ok) {
          const int64_t o = grow * d + gcol;
          *reinterpret_cast<u32x4*>(out + o) = ov;
          if (MODE == 1 && lin_out) *reinterpret_cast<u32x4*>(lin_out + o) = lv;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ct reads done before it is rewritten
      __builtin_amdgcn_wave_barrier();
    }
  }
}
#undef W4_MFMA

// ---------------------------------------------------------------------------
// CrossNet weight gradient dW = u^T x_l (TN: the contraction runs down the
// rows of both [B, d] operands), on the forward's 256 x 256, four-phase
// schedule (crossnet_8ph_kernel): the same waves / quadrants / half-tiles,
// barriers and counted waits, with two changes --
//   * a half-tile is 64 contraction rows x 128 output columns staged as they
//     lie in memory (global_load_lds, 256-B image rows, 32-B slots XOR-
//     swizzled by dw_h(r)), A_h holding columns {wr*128 + h*64 + [0, 64)} of
//     u and B_h columns {wc*64 + h*32 + [0, 32)} of x_l;
//   * the MFMA fragments (8 consecutive contraction rows of one column per
//     lane, for both operands) come from ds_read_b64_tr_b16, the transposing
//     LDS read (gemm_tn_kernel's fragment, mlp.hip).
// The 14 x 14 output tiles of d = 3 392 are fewer than the CUs: the batch is
// split into S slices (grid = tiles x S) whose fp32 partials
// crossnet_dw_reduce_kernel sums in slice order (deterministic).
// ---------------------------------------------------------------------------
typedef short dw_v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int dw_h(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

// half-tile h of u (AH) or x_l: 64 rows from k0, 128 logical columns; 2 wave
// instructions of 4 rows x 256 B per wave
template <bool AH>
__device__ __forceinline__ void dw_stage(const uint16_t* __restrict__ X, int d, int64_t k0,
                                         int c0, int h, char* img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rb = (wave * 2 + i) * 4;
    const int r = rb + (lane >> 4), sl = lane & 15;
    const int c = (((sl >> 1) ^ dw_h(r)) << 1) | (sl & 1);   // logical 16-B chunk
    const int col = AH ? ((c >> 3) * 128 + h * 64 + (c & 7) * 8)
                       : ((c >> 2) * 64 + h * 32 + (c & 3) * 8);
    int gc = c0 + col;
    if (gc >= d) gc = c0;   // columns past the end feed discarded outputs
    const uint16_t* src = X + (k0 + r) * (int64_t)d + gc;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(img + rb * 256),
                                     16, 0, 0);
  }
}

// 16 logical columns at slot m (0..7) for the 32-row step kk
__device__ __forceinline__ bf16x8 dw_frag(const char* img, int kk, int m, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r1 = kk * 32 + 8 * g + q, r2 = r1 + 4;
  const dw_v4s a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) dw_v4s*)(img + r1 * 256 + ((m ^ dw_h(r1)) << 5) + 8 * p));
  const dw_v4s b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) dw_v4s*)(img + r2 * 256 + ((m ^ dw_h(r2)) << 5) + 8 * p));
  return bf16x8{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
}

__global__ __launch_bounds__(512, 1) void crossnet_dw_kernel(
    const uint16_t* __restrict__ u, const uint16_t* __restrict__ xl, int64_t K, int d, int S,
    float* __restrict__ part) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * C8_BUF];  // 128 KB
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const bool g1 = wr != 0;
  // XCD-contiguous work items, then (output tile, batch slice), slices of a
  // tile adjacent (they read different rows of the same columns)
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t orig = blockIdx.x;
  const int64_t xcd = orig % 8, q8 = nwg / 8, rr = nwg % 8;
  const int64_t item = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + orig / 8;
  const int64_t tile = item / S;
  const int z = (int)(item % S);
  const int nt = d / 256 + (d % 256 ? 1 : 0);
  const int m0 = (int)(tile / nt) * 256, n0 = (int)(tile % nt) * 256;
  const int64_t kt = K / 64;                           // 64-row steps (K % 64 == 0)
  const int64_t ks = (kt * z) / S, ke = (kt * (z + 1)) / S;
  const int nk = (int)(ke - ks);
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto img = [&](int t, int part_) -> char* { return lds + (t & 1) * C8_BUF + part_ * C8_HALF; };
  auto st_a = [&](int t, int h) {
    dw_stage<true>(u, d, (ks + t) * 64, m0, h, img(t, h), wave, lane);
  };
  auto st_b = [&](int t, int h) {
    dw_stage<false>(xl, d, (ks + t) * 64, n0, h, img(t, 2 + h), wave, lane);
  };
  if (nk > 0) {
    st_a(0, 0); st_b(0, 0); st_b(0, 1); st_a(0, 1);
    if (nk > 1) {
      st_a(1, 0); st_b(1, 0); st_b(1, 1);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __builtin_amdgcn_s_barrier();
  if (g1) __builtin_amdgcn_s_barrier();  // the stagger
  asm volatile("" ::: "memory");
  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];  // [frag][kk]
  auto read_a = [&](const char* sm) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[i][kk] = dw_frag(sm, kk, wr * 4 + i, lane);
  };
  auto read_b = [&](const char* sm, bf16x8 (&fb)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb[j][kk] = dw_frag(sm, kk, wc * 2 + j, lane);
  };
  auto close_read = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto mma = [&](int mi, bf16x8 (&fb)[2][2], int nj) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mi + i][nj + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][kk], fb[j][kk], acc[mi + i][nj + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  for (int t = 0; t < nk; ++t) {
    const bool pf1 = t + 1 < nk, pf2 = t + 2 < nk;
    read_b(img(t, 2), fb0);
    read_a(img(t, 0));
    if (pf1) st_a(t + 1, 1);
    close_read();
    mma(0, fb0, 0);
    read_b(img(t, 3), fb1);
    if (pf2) st_a(t + 2, 0);
    close_read();
    mma(0, fb1, 2);
    read_a(img(t, 1));
    if (pf2) st_b(t + 2, 0);
    close_read();
    mma(4, fb0, 0);
    if (pf2) {
      st_b(t + 2, 1);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else if (pf1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    close_read();
    mma(4, fb1, 2);
  }
  if (!g1) __builtin_amdgcn_s_barrier();  // matches group 1's extra barrier
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // accumulators -> LDS (C/D map), then 2 x 16-B fp32 stores of 8 columns
  const int fr = lane & 15, fq = lane >> 4;
  float* ct = reinterpret_cast<float*>(lds) + wave * 64 * 64;
  float* pz = part + (int64_t)z * d * d;
  const int cc = (lane & 7) * 8;
  const int gcol = n0 + wc * 64 + cc;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + fq * 4 + r;
          const int col = (j * 16 + fr) ^ (((row >> 2) & 3) << 4);
          ct[row * 64 + col] = acc[h * 4 + i][j][r];
        }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int row = it * 8 + (lane >> 3);
      const int grow = m0 + wr * 128 + h * 64 + row;
      const int pc = cc ^ (((row >> 2) & 3) << 4);
      const float4 l0 = *reinterpret_cast<const float4*>(ct + row * 64 + pc);
      const float4 l1 = *reinterpret_cast<const float4*>(ct + row * 64 + pc + 4);
      if (grow < d && gcol < d) {
        float* dst = pz + (int64_t)grow * d + gcol;
        reinterpret_cast<float4*>(dst)[0] = l0;
        reinterpret_cast<float4*>(dst)[1] = l1;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
}

// dW = u^T x_l on the one-wave-per-SIMD schedule (crossnet_w4_kernel) in TN
// form (the default; DR_CROSSNET_DW_KERNEL=8ph the A/B): 4 waves of 128 x 128 outputs, the 64
// accumulators per lane pinned in AGPRs by inline-asm MFMAs; a 4-deep ring
// of K-32 stages, each operand 32 contraction rows x 256 output columns as
// they lie in memory (512-B image rows, 32-B slots XOR-swizzled by dw_h(r),
// global_load_lds three stages ahead, unconditional: past the slice's last
// stage the pieces reload it into the dead slot); fragments by
// ds_read_b64_tr_b16 (two per fragment, one stage ahead); batch slices as
// crossnet_dw_kernel, fp32 partials stored straight from the accumulators.
static constexpr int W4D_IMG = 32 * 512;   // one operand's K-32 stage: 32 rows x 256 bf16

#define W4D_MFMA(C, A, B) \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(C) : "v"(A), "v"(B))

// LDS ring [u slots 0..3 | x_l slots 0..3]; the stage loop is unrolled 4x so
// a stage's ring slot is a compile-time offset on per-lane fragment
// addresses computed once (16 VGPRs): with the slot at run time the
// compiler held 32 live addresses and spilled.
// XCD-region work order (grp == -2): the nt x nt tiles in Hilbert-curve
// order cut into 8 compact regions, region x the tiles of XCD x; XCD x walks
// slice 0's region, then slice 1's, ...  All 8 XCDs thus work on the same
// slice at once (its operands, K / S rows of u and x_l, fit the MALL: fetched
// from HBM about once), each on a compact block of tiles (its L2 shares the
// block's operand columns).
struct DwOrder {
  int16_t tile[256];   // tile ids (row * nt + col) in region order
  int16_t start[9];    // region x = tile[start[x] .. start[x + 1])
};

__global__ __launch_bounds__(256, 1) void crossnet_dw_w4_kernel(
    const uint16_t* __restrict__ u, const uint16_t* __restrict__ xl, int64_t K, int d, int S,
    float* __restrict__ part, int grp, DwOrder ord) {
  __shared__ __attribute__((aligned(1024))) char lds[8 * W4D_IMG];  // 128 KB
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t orig = blockIdx.x;
  const int64_t xcd = orig % 8, q8 = nwg / 8, rr = nwg % 8;
  const int64_t item = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + orig / 8;
  const int nt = d / 256 + (d % 256 ? 1 : 0);
  int z, m0, n0;
  if (grp == -2) {
    const int x = (int)(orig % 8);
    const int64_t k = orig / 8;
    const int n = ord.start[x + 1] - ord.start[x];
    if (k >= (int64_t)S * n) return;   // (XCDs with a smaller region: idle blocks)
    z = (int)(k / n);
    const int t = ord.tile[ord.start[x] + (int)(k % n)];
    m0 = (t / nt) * 256;
    n0 = (t % nt) * 256;
  } else if (grp > 0) {
    // slice-major, tiles in groups of grp tile rows walked column by column:
    // the ~32 work-groups an XCD runs at once share one K slice and cover a
    // grp x (32 / grp) block of tiles, so its L2 fetches each operand block
    // once for grp (or 32 / grp) tiles instead of once per tile
    const int64_t tiles = (int64_t)nt * nt;
    z = (int)(item / tiles);
    const int t = (int)(item % tiles);
    const int g0 = (t / (grp * nt)) * grp;
    const int gm = nt - g0 < grp ? nt - g0 : grp;
    const int tr = t - g0 * nt;
    m0 = (g0 + tr % gm) * 256;
    n0 = (tr / gm) * 256;
  } else {
    const int64_t tile = item / S;
    z = (int)(item % S);
    m0 = (int)(tile / nt) * 256;
    n0 = (int)(tile % nt) * 256;
  }
  const int64_t kt = K / 32;                           // 32-row stages (K % 64 == 0)
  const int64_t ks = (kt * z) / S, ke = (kt * (z + 1)) / S;
  const int nk = (int)(ke - ks);
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // DMA piece p of a stage: operand p >> 2 (u / x_l), image rows r0, r0 + 1
  const uint16_t* psrc[8];
  int pdst[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int r0 = (wave * 4 + (p & 3)) * 2;
    const int r = r0 + (lane >> 5), sl = lane & 31;
    const int c = (((sl >> 1) ^ dw_h(r)) << 1) | (sl & 1);   // logical 16-B chunk
    const int cb = (p >> 2) ? n0 : m0;
    int gc = cb + c * 8;
    if (gc >= d) gc = cb;   // columns past the end feed discarded outputs
    psrc[p] = ((p >> 2) ? xl : u) + (ks * 32 + r) * (int64_t)d + gc;
    pdst[p] = (p >> 2) * 4 * W4D_IMG + r0 * 512;
  }
  auto dma = [&](int stage, int slot) {
#pragma unroll
    for (int p = 0; p < 8; ++p)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(psrc[p] + (int64_t)stage * 32 * d),
          (__attribute__((address_space(3))) void*)(lds + pdst[p] + slot * W4D_IMG), 16, 0, 0);
  };
  // fragment f (0..7 u rows, 8..15 x_l columns): its first row's address in
  // slot 0; the second read is 4 rows (2048 B) on (same swizzle)
  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int r1 = 8 * g + qq;
  int fa[16];
#pragma unroll
  for (int f = 0; f < 16; ++f) {
    const int slot = f < 8 ? wr * 8 + f : wc * 8 + (f - 8);
    fa[f] = (f < 8 ? 0 : 4 * W4D_IMG) + r1 * 512 + ((slot ^ dw_h(r1)) << 5) + 8 * pp;
  }
  bf16x8 F0[16], F1[16];
  // the transposing reads as inline asm: written with the builtin, the
  // compiler (which cannot tell the ring slots apart) put a vmcnt(0) in
  // front of them for the LDS-DMA pieces just issued -- a wait for stage
  // s + 3 in every stage.  Completion is the lgkmcnt(0) at the next stage's
  // top, before any MFMA reads these registers.
  typedef __attribute__((address_space(3))) char lds_c;
  const uint32_t lbase = (uint32_t)(size_t)(lds_c*)lds;
  auto tie_compose = [&](dw_v4s (&hx)[16], dw_v4s (&hy)[16], bf16x8 (&F)[16]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(hx[0]), "+v"(hx[1]), "+v"(hx[2]), "+v"(hx[3]), "+v"(hx[4]), "+v"(hx[5]),
                   "+v"(hx[6]), "+v"(hx[7]), "+v"(hy[0]), "+v"(hy[1]), "+v"(hy[2]), "+v"(hy[3]),
                   "+v"(hy[4]), "+v"(hy[5]), "+v"(hy[6]), "+v"(hy[7])::"memory");
    asm volatile(""
                 : "+v"(hx[8]), "+v"(hx[9]), "+v"(hx[10]), "+v"(hx[11]), "+v"(hx[12]),
                   "+v"(hx[13]), "+v"(hx[14]), "+v"(hx[15]), "+v"(hy[8]), "+v"(hy[9]),
                   "+v"(hy[10]), "+v"(hy[11]), "+v"(hy[12]), "+v"(hy[13]), "+v"(hy[14]),
                   "+v"(hy[15])::"memory");
#pragma unroll
    for (int f = 0; f < 16; ++f)
      F[f] = bf16x8{hx[f].x, hx[f].y, hx[f].z, hx[f].w, hy[f].x, hy[f].y, hy[f].z, hy[f].w};
  };
  auto read = [&](int slot, bf16x8 (&F)[16]) {
    dw_v4s hx[16], hy[16];
#pragma unroll
    for (int f = 0; f < 16; ++f) {
      const uint32_t a = lbase + (uint32_t)(fa[f] + slot * W4D_IMG);
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hx[f]) : "v"(a));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(hy[f]) : "v"(a));
    }
    tie_compose(hx, hy, F);
  };
  // one stage: s at ring slot Q (compile time); the next stage's fragments
  // from slot Q + 1, stage s + 3's pieces into slot Q + 3 (= the slot stage
  // s - 1 left), clamped to the slice's last stage
  // interleaved form: the 32 transposing reads after the stage's first 32
  // MFMAs, the 8 DMA pieces after every 4th of the last 32; the halves are
  // tied through the closing lgkmcnt(0) ("+v") so the compiler neither
  // copies nor reuses their registers while the LDS returns are in flight
  // (without the tie it recycled one for an address: an illegal access)
  auto stage_il = [&](int Q, int s, bf16x8 (&FC)[16], bf16x8 (&FN)[16]) {
    const int s3 = s + 3 < nk ? s + 3 : nk - 1;
    const int rslot = s + 1 < nk ? ((Q + 1) & 3) : Q;
    const int dslot = (Q + 3) & 3;
    dw_v4s hx[16], hy[16];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        W4D_MFMA(acc[i][j], FC[i], FC[8 + j]);
        const int m = i * 8 + j;
        if (m < 32) {
          const int f = m >> 1;
          const uint32_t a = lbase + (uint32_t)(fa[f] + rslot * W4D_IMG);
          if (m & 1)
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(hy[f]) : "v"(a));
          else
            asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hx[f]) : "v"(a));
        } else if ((m & 3) == 2) {
          const int p = (m - 34) >> 2;
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(psrc[p] + (int64_t)s3 * 32 * d),
              (__attribute__((address_space(3))) void*)(lds + pdst[p] + dslot * W4D_IMG), 16, 0, 0);
        }
      }
    tie_compose(hx, hy, FN);
  };
#define W4D_ITER(Q, FC, FN)                                                               \
  do {                                                                                    \
    __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): FC complete */                    \
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); /* stage s+1 landed (this wave) */  \
    __builtin_amdgcn_s_barrier();                                                         \
    asm volatile("" ::: "memory");                                                        \
    stage_il((Q), s, FC, FN);                                                             \
    ++s;                                                                                  \
  } while (0)
  if (nk > 0) {
    dma(0, 0);
    dma(1 < nk ? 1 : nk - 1, 1);
    dma(2 < nk ? 2 : nk - 1, 2);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read(0, F0);
    int s = 0;
    while (s + 4 <= nk) {
      W4D_ITER(0, F0, F1);
      W4D_ITER(1, F1, F0);
      W4D_ITER(2, F0, F1);
      W4D_ITER(3, F1, F0);
    }
    if (s < nk) W4D_ITER(0, F0, F1);
    if (s < nk) W4D_ITER(1, F1, F0);
    if (s < nk) W4D_ITER(2, F0, F1);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  }
#undef W4D_ITER
  // fp32 partials straight from the accumulators (C/D map: row fq * 4 + r,
  // column fr of each 16 x 16 tile; 16 lanes write 64 contiguous bytes)
  const int fr = lane & 15, fq = lane >> 4;
  float* pz = part + (int64_t)z * d * d;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = n0 + wc * 128 + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 128 + i * 16 + fq * 4 + r;
        if (m < d && n < d) pz[(int64_t)m * d + n] = acc[i][j][r];
      }
    }
}
#undef W4D_MFMA

// dW = sum over slices z of part[z], in slice order (deterministic)
__global__ void crossnet_dw_reduce_kernel(const float* __restrict__ part, int S, int64_t n4,
                                          int64_t zstride, float* __restrict__ dw) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n4) return;
  float4 s = reinterpret_cast<const float4*>(part)[q];
  for (int z = 1; z < S; ++z) {
    const float4 p = reinterpret_cast<const float4*>(part + (int64_t)z * zstride)[q];
    s.x += p.x;
    s.y += p.y;
    s.z += p.z;
    s.w += p.w;
  }
  reinterpret_cast<float4*>(dw)[q] = s;
}

// ---------------------------------------------------------------------------
// CrossNet backward, the elementwise part of one layer in ONE pass over HBM
// (the GEMMs dW = u^T x_l and dx_l = u W + g stay library calls):
//   u   = bf16(g * x0)                         [B, d] bf16
//   acc = (acc_in ? acc_in : 0) + g * lin      [B, d] fp32 (dx0 over layers)
//   dbp[blk][c] = sum over this block's rows of u[r][c]   (fp32 partials)
// A thread owns 8 consecutive columns (one 16-B bf16 vector) and walks the
// block's rows; the 4 waves of a block take rows r0 + w, r0 + w + 4, ...
// and their column partials are added in wave order through LDS, so the
// partials, and db = crossnet_db_kernel's fixed-order sum of them, are
// deterministic.
// ---------------------------------------------------------------------------
static constexpr int CB_ROWS = 256;  // rows per block

__global__ __launch_bounds__(256) void crossnet_bwd_elem_kernel(
    const uint16_t* __restrict__ g, const uint16_t* __restrict__ x0,
    const uint16_t* __restrict__ lin, const float* acc_in, float* acc_out,
    uint16_t* __restrict__ u, float* __restrict__ dbp, int64_t B, int d) {
  __shared__ float part[3][64][8 + 1];
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = (blockIdx.x * 64 + lane) * 8;
  const int64_t r0 = (int64_t)blockIdx.y * CB_ROWS;
  const bool col_ok = c0 < d;
  float db[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col_ok) {
    for (int64_t r = r0 + wave; r < r0 + CB_ROWS && r < B; r += 4) {
      const int64_t o = r * d + c0;
      const u32x4 gv = *reinterpret_cast<const u32x4*>(g + o);
      const u32x4 xv = *reinterpret_cast<const u32x4*>(x0 + o);
      const u32x4 lv = *reinterpret_cast<const u32x4*>(lin + o);
      float a[8];
      if (acc_in) {
        const float4 a0 = *reinterpret_cast<const float4*>(acc_in + o);
        const float4 a1 = *reinterpret_cast<const float4*>(acc_in + o + 4);
        a[0] = a0.x; a[1] = a0.y; a[2] = a0.z; a[3] = a0.w;
        a[4] = a1.x; a[5] = a1.y; a[6] = a1.z; a[7] = a1.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] = 0.f;
      }
      u32x4 uv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g0 = bf2f((uint16_t)(gv[e] & 0xffff)), g1 = bf2f((uint16_t)(gv[e] >> 16));
        const uint16_t u0 = f2bf(g0 * bf2f((uint16_t)(xv[e] & 0xffff)));
        const uint16_t u1 = f2bf(g1 * bf2f((uint16_t)(xv[e] >> 16)));
        uv[e] = (uint32_t)u0 | ((uint32_t)u1 << 16);
        db[2 * e] += bf2f(u0);
        db[2 * e + 1] += bf2f(u1);
        a[2 * e] += g0 * bf2f((uint16_t)(lv[e] & 0xffff));
        a[2 * e + 1] += g1 * bf2f((uint16_t)(lv[e] >> 16));
      }
      *reinterpret_cast<u32x4*>(u + o) = uv;
      *reinterpret_cast<float4*>(acc_out + o) = make_float4(a[0], a[1], a[2], a[3]);
      *reinterpret_cast<float4*>(acc_out + o + 4) = make_float4(a[4], a[5], a[6], a[7]);
    }
  }
  // column partials of the 4 waves, added in wave order
  if (wave > 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) part[wave - 1][lane][e] = db[e];
  }
  __syncthreads();
  if (wave == 0 && col_ok) {
#pragma unroll
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int e = 0; e < 8; ++e) db[e] += part[w][lane][e];
    float* dst = dbp + (int64_t)blockIdx.y * d + c0;
    *reinterpret_cast<float4*>(dst) = make_float4(db[0], db[1], db[2], db[3]);
    *reinterpret_cast<float4*>(dst + 4) = make_float4(db[4], db[5], db[6], db[7]);
  }
}

// db[c] = sum over row blocks of dbp[blk][c], in block order
__global__ void crossnet_db_kernel(const float* __restrict__ dbp, int64_t nblk, int d,
                                   float* __restrict__ db) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d) return;
  float s = 0.f;
  for (int64_t k = 0; k < nblk; ++k) s += dbp[k * d + c];
  db[c] = s;
}

}  // namespace dr

namespace dr {
static bool dot_mfma_ok(int fields, int dim) {
  return fields >= 2 && fields <= 32 && (dim == 16 || dim == 32 || dim == 64 || dim == 128);
}
template <bool CAT>
static int dot_mfma_launch(const float* x, int64_t batch, int fields, int dim, void* out,
                           int64_t ostride, hipStream_t st) {
  const unsigned grid = (unsigned)ceil_div(batch, 4);
#define DR_DOT_MFMA(KI)                                                                         \
  do {                                                                                          \
    if (fields <= 16)                                                                           \
      hipLaunchKernelGGL((dot_mfma_kernel<KI, 1, CAT>), dim3(grid), dim3(256), 0, st, x, batch,  \
                         fields, out, ostride);                                                 \
    else                                                                                        \
      hipLaunchKernelGGL((dot_mfma_kernel<KI, 3, CAT>), dim3(grid), dim3(256), 0, st, x, batch,  \
                         fields, out, ostride);                                                 \
  } while (0)
  if (dim == 16)
    DR_DOT_MFMA(1);
  else if (dim == 32)
    DR_DOT_MFMA(2);
  else if (dim == 64)
    DR_DOT_MFMA(4);
  else
    DR_DOT_MFMA(8);
#undef DR_DOT_MFMA
  DR_LAUNCH_CHECK();
  return DR_OK;
}
}  // namespace dr

extern "C" {

int dr_fm2(const float* emb, int64_t batch, int fields, int dim, float* out, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && fields > 0 && dim > 0 && dim % 4 == 0, DR_INVALID_ARGUMENT,
             "dr_fm2: dim must be a multiple of 4");
  if (batch == 0) return DR_OK;
  const int64_t n = batch * (dim / 4);
  hipLaunchKernelGGL(fm2_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, S(stream), emb,
                     batch, fields, dim, out, (uint16_t*)nullptr);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_fm2_bf16_copy(const float* emb, int64_t batch, int fields, int dim, float* out,
                     uint16_t* emb_bf16, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && fields > 0 && dim > 0 && dim % 4 == 0 && emb_bf16, DR_INVALID_ARGUMENT,
             "dr_fm2_bf16_copy: dim must be a multiple of 4");
  DR_REQUIRE(((((uintptr_t)emb) | ((uintptr_t)out)) & 15) == 0 && ((uintptr_t)emb_bf16 & 7) == 0,
             DR_INVALID_ARGUMENT, "dr_fm2_bf16_copy: emb / out 16-B, emb_bf16 8-B aligned");
  if (batch == 0) return DR_OK;
  const int64_t n = batch * (dim / 4);
  hipLaunchKernelGGL(fm2_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, S(stream), emb,
                     batch, fields, dim, out, emb_bf16);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_fm2_grad_add_bf16(const float* emb, const float* top_grad, const uint16_t* add,
                         int64_t add_stride, int64_t batch, int fields, int dim, float* grad_emb,
                         void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && fields > 0 && fields <= 32 && dim > 0 && dim % 4 == 0 && add &&
                 add_stride >= (int64_t)fields * dim && add_stride % 4 == 0,
             DR_INVALID_ARGUMENT,
             "dr_fm2_grad_add_bf16: fields <= 32, dim %% 4 == 0, add_stride >= fields*dim, %% 4");
  DR_REQUIRE(((((uintptr_t)emb) | ((uintptr_t)top_grad) | ((uintptr_t)grad_emb)) & 15) == 0 &&
                 ((uintptr_t)add & 7) == 0,
             DR_INVALID_ARGUMENT, "dr_fm2_grad_add_bf16: pointers 16-B (add: 8-B) aligned");
  if (batch == 0) return DR_OK;
  const unsigned blocks = (unsigned)ceil_div(batch * (dim / 4), 256);
  if (fields <= 8)
    hipLaunchKernelGGL(fm2_grad_kernel<8>, dim3(blocks), dim3(256), 0, S(stream), emb, top_grad,
                       batch, fields, dim, grad_emb, add, add_stride);
  else if (fields <= 16)
    hipLaunchKernelGGL(fm2_grad_kernel<16>, dim3(blocks), dim3(256), 0, S(stream), emb, top_grad,
                       batch, fields, dim, grad_emb, add, add_stride);
  else
    hipLaunchKernelGGL(fm2_grad_kernel<32>, dim3(blocks), dim3(256), 0, S(stream), emb, top_grad,
                       batch, fields, dim, grad_emb, add, add_stride);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_fm2_grad(const float* emb, const float* top_grad, int64_t batch, int fields, int dim,
                float* grad_emb, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && fields > 0 && dim > 0, DR_INVALID_ARGUMENT, "bad shape");
  if (batch == 0) return DR_OK;
  const bool al = ((((uintptr_t)emb) | ((uintptr_t)top_grad) | ((uintptr_t)grad_emb)) & 15) == 0;
  if (dim % 4 == 0 && al && fields <= 32) {
    const unsigned blocks = (unsigned)ceil_div(batch * (dim / 4), 256);
    if (fields <= 8)
      hipLaunchKernelGGL(fm2_grad_kernel<8>, dim3(blocks), dim3(256), 0, S(stream), emb, top_grad,
                         batch, fields, dim, grad_emb, (const uint16_t*)nullptr, (int64_t)0);
    else if (fields <= 16)
      hipLaunchKernelGGL(fm2_grad_kernel<16>, dim3(blocks), dim3(256), 0, S(stream), emb,
                         top_grad, batch, fields, dim, grad_emb, (const uint16_t*)nullptr,
                         (int64_t)0);
    else
      hipLaunchKernelGGL(fm2_grad_kernel<32>, dim3(blocks), dim3(256), 0, S(stream), emb,
                         top_grad, batch, fields, dim, grad_emb, (const uint16_t*)nullptr,
                         (int64_t)0);
  } else {
    hipLaunchKernelGGL(fm2_grad_any_kernel, dim3((unsigned)ceil_div(batch * dim, 256)), dim3(256),
                       0, S(stream), emb, top_grad, batch, fields, dim, grad_emb);
  }
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_dot_interaction(const float* x, int64_t batch, int fields, int dim, float* out,
                       void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && fields > 1 && dim > 0, DR_INVALID_ARGUMENT, "bad shape");
  const size_t lds = (size_t)fields * (dim + 1) * sizeof(float);
  DR_REQUIRE(lds <= 64 * 1024, DR_INVALID_ARGUMENT, "fields*dim too large for one block");
  if (batch == 0) return DR_OK;
  // f32 MFMA path (dot_mfma_kernel): F <= 32, D in {16, 32, 64, 128}
  static const bool dot_valu = getenv("DR_DOT_VALU") != nullptr;   // A/B: LDS-tiled VALU kernel
  if (!dot_valu && dot_mfma_ok(fields, dim) && ((uintptr_t)x & 15) == 0)
    return dot_mfma_launch<false>(x, batch, fields, dim, out, 0, S(stream));
  const int nb = (fields + 3) / 4;
  const size_t tlds = (size_t)DOT_WAVES * nb * 4 * (dim + 4) * sizeof(float);
  if (nb * (nb + 1) / 2 <= 32 && dim % 8 == 0 && ((uintptr_t)x & 15) == 0 && tlds <= 64 * 1024 &&
      nb * 4 * (dim / 4) <= DOT_MAXE * 64) {
    // grid: what fits at once (LDS-limited blocks per CU x 256 CUs)
    const int per_cu = std::max<int>(1, (int)((160 * 1024) / tlds));
    const int64_t grid = std::min<int64_t>(ceil_div(batch, DOT_WAVES), (int64_t)per_cu * 256);
    hipLaunchKernelGGL(dot_tile_kernel, dim3((unsigned)grid), dim3(256), tlds, S(stream), x, batch,
                       fields, dim, out);
    DR_LAUNCH_CHECK();
    return DR_OK;
  }
  hipLaunchKernelGGL(dot_kernel, dim3((unsigned)batch), dim3(256), lds, S(stream), x, fields, dim,
                     out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_dot_interaction_grad(const float* x, const float* top_grad, int64_t batch, int fields,
                            int dim, float* grad_x, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && fields > 1 && fields <= 32 && dim > 0 && dim % 4 == 0,
             DR_INVALID_ARGUMENT, "dr_dot_interaction_grad: need 2 <= fields <= 32, dim %% 4 == 0");
  DR_REQUIRE((((uintptr_t)x) | ((uintptr_t)grad_x)) % 16 == 0, DR_INVALID_ARGUMENT,
             "x / grad_x must be 16-B aligned");
  if (batch == 0) return DR_OK;
  const unsigned grid = (unsigned)ceil_div(batch, 8);
  if (fields <= 16)
    hipLaunchKernelGGL(dot_grad_kernel<16>, dim3(grid), dim3(256), 0, S(stream), x, top_grad,
                       batch, fields, dim, grad_x);
  else if (fields <= 28)
    hipLaunchKernelGGL(dot_grad_kernel<28>, dim3(grid), dim3(256), 0, S(stream), x, top_grad,
                       batch, fields, dim, grad_x);
  else
    hipLaunchKernelGGL(dot_grad_kernel<32>, dim3(grid), dim3(256), 0, S(stream), x, top_grad,
                       batch, fields, dim, grad_x);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_dot_interaction_concat_bf16(const float* x, int64_t batch, int fields, int dim,
                                   uint16_t* out, int64_t out_stride, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && dot_mfma_ok(fields, dim), DR_INVALID_ARGUMENT,
             "dr_dot_interaction_concat_bf16: need 2 <= fields <= 32, dim in {16, 32, 64, 128}");
  DR_REQUIRE(out_stride % 2 == 0 && out_stride >= dim + (int64_t)fields * (fields - 1) / 2,
             DR_INVALID_ARGUMENT, "out_stride must be even and >= dim + fields*(fields-1)/2");
  DR_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 3) == 0, DR_INVALID_ARGUMENT,
             "x must be 16-B and out 4-B aligned");
  if (batch == 0) return DR_OK;
  return dot_mfma_launch<true>(x, batch, fields, dim, out, out_stride, S(stream));
}

int dr_dot_interaction_concat_grad_bf16(const float* x, const uint16_t* grad, int64_t grad_stride,
                                        int64_t batch, int fields, int dim, float* grad_x,
                                        void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && fields > 1 && fields <= 32 && dim > 0 && dim % 4 == 0,
             DR_INVALID_ARGUMENT,
             "dr_dot_interaction_concat_grad_bf16: need 2 <= fields <= 32, dim %% 4 == 0");
  DR_REQUIRE(grad_stride >= dim + (int64_t)fields * (fields - 1) / 2 && grad_stride % 4 == 0,
             DR_INVALID_ARGUMENT, "grad_stride must be a multiple of 4 and >= dim + pairs");
  DR_REQUIRE((((uintptr_t)x) | ((uintptr_t)grad_x)) % 16 == 0 && ((uintptr_t)grad & 7) == 0,
             DR_INVALID_ARGUMENT, "x / grad_x must be 16-B and grad 8-B aligned");
  if (batch == 0) return DR_OK;
  const unsigned grid = (unsigned)ceil_div(batch, 8);
  if (fields <= 16)
    hipLaunchKernelGGL((dot_grad_kernel<16, true>), dim3(grid), dim3(256), 0, S(stream), x, grad,
                       batch, fields, dim, grad_x, grad_stride);
  else if (fields <= 28)
    hipLaunchKernelGGL((dot_grad_kernel<28, true>), dim3(grid), dim3(256), 0, S(stream), x, grad,
                       batch, fields, dim, grad_x, grad_stride);
  else
    hipLaunchKernelGGL((dot_grad_kernel<32, true>), dim3(grid), dim3(256), 0, S(stream), x, grad,
                       batch, fields, dim, grad_x, grad_stride);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_crossnet_forward_bf16(const uint16_t* x0, const uint16_t* xl, const uint16_t* W,
                             const float* bias, int64_t batch, int d, uint16_t* out,
                             uint16_t* lin_out, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && d > 0 && d % 8 == 0, DR_INVALID_ARGUMENT,
             "dr_crossnet_layer_bf16: d must be a multiple of 8 (pad features)");
  DR_REQUIRE(((uintptr_t)x0 | (uintptr_t)xl | (uintptr_t)W) % 16 == 0, DR_INVALID_ARGUMENT,
             "operands must be 16B aligned");
  if (batch == 0) return DR_OK;
  static const bool legacy = getenv("DR_CROSSNET_LEGACY") != nullptr;
  const bool al16 = (((uintptr_t)bias | (uintptr_t)out | (uintptr_t)lin_out) & 15) == 0;
  // 8 = crossnet_8ph_kernel (default); the others are kept for A/B runs
  // (tools/gpu_crossnet_v.sh): 5 stag, 4 256^2, 3 glds3, 6/9/10 8ph with other
  // tile orders / epilogue, 7 the 8ph loop alone (no outputs: timing only).
  // (Round 4, removed: 13, desynchronised epilogues -- half the CUs starting
  // with a half tile so the two halves' epilogue bursts alternate --
  // measured 3-5 % slower, profiles/r04_crossnet_desync_ab.log; a one-wave-
  // per-SIMD 128 x 128-per-wave form did not compile to a usable loop: with
  // 256 accumulators the register allocator rotated them through VGPRs,
  // ~440 accvgpr moves per 128 MFMAs.)
  static const int variant = getenv("DR_CROSSNET_VARIANT") ? atoi(getenv("DR_CROSSNET_VARIANT"))
                                                           : 8;
  if (d % 64 == 0 && !legacy && al16 && variant >= 14 && variant <= 17) {
    // 14: crossnet_w4_kernel (one wave per SIMD, AGPR accumulators); 15 its
    // loop alone (timing only); 16 / 17 the same with reads and DMAs
    // interleaved with the MFMAs
    const int64_t tiles = ceil_div(batch, 256) * ceil_div(d, 256);
    DR_REQUIRE(tiles < (1ll << 31), DR_INVALID_ARGUMENT, "batch too large");
#define DR_W4(E, IL)                                                                        \
  hipLaunchKernelGGL((crossnet_w4_kernel<E, 4, IL>), dim3((unsigned)tiles), dim3(256), 0,      \
                     S(stream), x0, xl, W, bias, batch, d, d, out, lin_out)
    if (variant == 14) DR_W4(1, false);
    else if (variant == 15) DR_W4(0, false);
    else if (variant == 16) DR_W4(1, true);
    else DR_W4(0, true);
#undef DR_W4
    DR_LAUNCH_CHECK();
    return DR_OK;
  }
  if (d % 64 == 0 && !legacy && al16 && (variant >= 6 && variant <= 12)) {
    // variant 12 (A/B only): the 8-phase kernel covers the whole 256-column
    // tiles and the 128 x 128 glds kernel the d % 256 strip, instead of one
    // ragged 256-column tile -- measured 1.43 vs 1.42 ms at d = 3392, i.e. no
    // gain, so the default keeps the ragged tile
    const bool split = variant == 12 && d > 256 && d % 256 != 0;
    const int ncols = split ? d - d % 256 : d;
    const int64_t tiles = ceil_div(batch, 256) * ceil_div(ncols, 256);
    DR_REQUIRE(tiles < (1ll << 31), DR_INVALID_ARGUMENT, "batch too large");
#define DR_C8(E, G, P)                                                                     \
  hipLaunchKernelGGL((crossnet_8ph_kernel<E, G, P>), dim3((unsigned)tiles), dim3(512), 0,   \
                     S(stream), x0, xl, W, bias, batch, d, ncols, out, lin_out)
    if (variant == 6) DR_C8(1, 1, false);
    else if (variant == 8) DR_C8(1, 4, false);
    else if (variant == 9) DR_C8(1, 8, false);
    else if (variant == 10) DR_C8(1, 4, true);
    else if (variant == 11 || variant == 12) DR_C8(1, 4, false);
    else DR_C8(0, 4, false);  // 7: loop-only timing build (no outputs; measurement only)
#undef DR_C8
    if (split) {
      const int64_t st = ceil_div(batch, CG_BM) * ceil_div(d - ncols, CG_BN);
      hipLaunchKernelGGL(crossnet_glds_kernel, dim3((unsigned)st), dim3(256), 0, S(stream), x0, xl,
                         W, bias, batch, d, ncols, out, lin_out);
    }
    DR_LAUNCH_CHECK();
    return DR_OK;
  }
  if (d % 64 == 0 && !legacy && al16 && variant == 5) {
    const int64_t tiles = ceil_div(batch, 256) * ceil_div(d, 256);
    DR_REQUIRE(tiles < (1ll << 31), DR_INVALID_ARGUMENT, "batch too large");
    hipLaunchKernelGGL(crossnet_stag_kernel, dim3((unsigned)tiles), dim3(512), 0, S(stream), x0,
                       xl, W, bias, batch, d, out, lin_out);
    DR_LAUNCH_CHECK();
    return DR_OK;
  }
  if (d % C4_BK == 0 && !legacy && al16 && variant == 4) {
    const int64_t tiles = ceil_div(batch, C4_BM) * ceil_div(d, C4_BN);
    DR_REQUIRE(tiles < (1ll << 31), DR_INVALID_ARGUMENT, "batch too large");
    hipLaunchKernelGGL(crossnet_256_kernel, dim3((unsigned)tiles), dim3(512), 0, S(stream), x0,
                       xl, W, bias, batch, d, out, lin_out);
    DR_LAUNCH_CHECK();
    return DR_OK;
  }
  if (d % C3_BK == 0 && !legacy && al16 && variant == 3) {
    const int64_t tiles = ceil_div(batch, C3_BM) * ceil_div(d, C3_BN);
    DR_REQUIRE(tiles < (1ll << 31), DR_INVALID_ARGUMENT, "batch too large");
    hipLaunchKernelGGL(crossnet_glds3_kernel, dim3((unsigned)tiles), dim3(512), 0, S(stream), x0,
                       xl, W, bias, batch, d, out, lin_out);
    DR_LAUNCH_CHECK();
    return DR_OK;
  }
  if (d % CG_BK == 0 && !legacy && al16) {
    const int64_t tiles = ceil_div(batch, CG_BM) * ceil_div(d, CG_BN);
    DR_REQUIRE(tiles < (1ll << 31), DR_INVALID_ARGUMENT, "batch too large");
    hipLaunchKernelGGL(crossnet_glds_kernel, dim3((unsigned)tiles), dim3(256), 0, S(stream), x0,
                       xl, W, bias, batch, d, 0, out, lin_out);
    DR_LAUNCH_CHECK();
    return DR_OK;
  }
  DR_REQUIRE(!lin_out, DR_INVALID_ARGUMENT,
             "lin_out needs d %% 64 == 0 and 16-B aligned bias / out / lin_out");
  dim3 grid((unsigned)ceil_div(d, CN_BN), (unsigned)ceil_div(batch, CN_BM));
  hipLaunchKernelGGL(crossnet_kernel, grid, dim3(256), 0, S(stream), x0, xl, W, bias, batch, d,
                     out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_crossnet_dx_bf16(const uint16_t* u, const uint16_t* wt, const uint16_t* g, int64_t batch,
                        int d, uint16_t* dx, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && d > 0 && d % 64 == 0, DR_INVALID_ARGUMENT,
             "dr_crossnet_dx_bf16: d must be a multiple of 64 (pad features)");
  DR_REQUIRE(u && wt && g && dx, DR_INVALID_ARGUMENT, "null operand");
  DR_REQUIRE((((uintptr_t)u | (uintptr_t)wt | (uintptr_t)g | (uintptr_t)dx) & 15) == 0,
             DR_INVALID_ARGUMENT, "operands must be 16-B aligned");
  if (batch == 0) return DR_OK;
  const int64_t tiles = ceil_div(batch, 256) * ceil_div(d, 256);
  DR_REQUIRE(tiles < (1ll << 31), DR_INVALID_ARGUMENT, "batch too large");
  // the forward's 256^2 schedule with A = u, B = W^T and the addend g
  static const int variant = getenv("DR_CROSSNET_VARIANT") ? atoi(getenv("DR_CROSSNET_VARIANT"))
                                                           : 8;
  if (variant == 14 || variant == 15)
    hipLaunchKernelGGL((crossnet_w4_kernel<2, 4, false>), dim3((unsigned)tiles), dim3(256), 0,
                       S(stream), g, u, wt, (const float*)nullptr, batch, d, d, dx,
                       (uint16_t*)nullptr);
  else if (variant >= 16 && variant <= 17)
    hipLaunchKernelGGL((crossnet_w4_kernel<2, 4, true>), dim3((unsigned)tiles), dim3(256), 0,
                       S(stream), g, u, wt, (const float*)nullptr, batch, d, d, dx,
                       (uint16_t*)nullptr);
  else
    hipLaunchKernelGGL((crossnet_8ph_kernel<2, 4, false>), dim3((unsigned)tiles), dim3(512), 0,
                       S(stream), g, u, wt, (const float*)nullptr, batch, d, d, dx,
                       (uint16_t*)nullptr);
  DR_LAUNCH_CHECK();
  return DR_OK;
}


// CrossNet weight gradient dW = u^T x_l (fp32 [d, d]); the batch split into
// crossnet_dw_slices() slices whose partials live in the workspace.
static int crossnet_dw_slices(int64_t batch, int d) {
  const int64_t tiles = (int64_t)dr::ceil_div(d, 256) * dr::ceil_div(d, 256);
  // one block per CU (128 KB of LDS): S slices fill whole rounds of 256 CUs
  // best; each slice >= 1024 rows
  int best = 1;
  double best_eff = 0.0;
  for (int s = 1; s <= 16; ++s) {
    if (batch / s < 1024) break;
    const int64_t items = tiles * s;
    const int64_t rounds = (items + 255) / 256;
    const double eff = (double)items / (double)(rounds * 256);
    if (eff > best_eff + 0.02) {
      best_eff = eff;
      best = s;
    }
  }
  return best;
}

size_t dr_crossnet_dw_workspace_size(int64_t batch, int d) {
  if (batch <= 0 || d <= 0) return 256;
  return (size_t)crossnet_dw_slices(batch, d) * (size_t)d * (size_t)d * sizeof(float) + 256;
}

int dr_crossnet_dw_bf16(const uint16_t* u, const uint16_t* xl, int64_t batch, int d, float* dw,
                        void* ws, size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && d > 0 && d % 64 == 0 && batch % 64 == 0, DR_INVALID_ARGUMENT,
             "dr_crossnet_dw_bf16: d and batch must be multiples of 64");
  DR_REQUIRE(u && xl && dw && ws, DR_INVALID_ARGUMENT, "null operand");
  DR_REQUIRE((((uintptr_t)u | (uintptr_t)xl | (uintptr_t)dw | (uintptr_t)ws) & 15) == 0,
             DR_INVALID_ARGUMENT, "operands must be 16-B aligned");
  DR_REQUIRE(ws_bytes >= dr_crossnet_dw_workspace_size(batch, d), DR_INVALID_ARGUMENT,
             "workspace too small");
  const int64_t n4 = (int64_t)d * d / 4;
  if (batch == 0) return fill_bytes(dw, 0, (size_t)d * d * sizeof(float), S(stream));
  const int Sl = crossnet_dw_slices(batch, d);
  const int64_t tiles = (int64_t)ceil_div(d, 256) * ceil_div(d, 256);
  float* part = static_cast<float*>(ws);
  // the one-wave-per-SIMD form by default (1.35-1.37 ms at B = 65536, d =
  // 3392 against 2.16 for the 8-phase kernel and 1.43-1.64 for hipBLASLt,
  // profiles/r05_cross_dw_w4.log); DR_CROSSNET_DW_KERNEL=8ph (read per call)
  // selects the 8-phase kernel (A/B)
  const char* kern = getenv("DR_CROSSNET_DW_KERNEL");
  const bool w4 = !(kern && strcmp(kern, "8ph") == 0);
  // DR_CROSSNET_DW_ORDER (read per call): the w4 work order, 0 = tile-major
  // (an XCD's concurrent work-groups are the slices of a few tiles), g > 0 =
  // slice-major in groups of g tile rows (default 4)
  // ("xcd": the XCD-region order, DwOrder)
  const char* ord = getenv("DR_CROSSNET_DW_ORDER");
  const bool xcd = ord && strcmp(ord, "xcd") == 0;
  const int grp = xcd ? -2 : (ord ? atoi(ord) : 4);
  DwOrder wo;
  memset(&wo, 0, sizeof(wo));
  int64_t blocks = tiles * Sl;
  if (xcd) {
    const int nt = (int)ceil_div(d, 256);
    DR_REQUIRE(nt <= 16, DR_INVALID_ARGUMENT, "xcd dW order: d <= 4096");
    int n = 0;
    for (int h = 0; h < 256; ++h) {   // Hilbert curve over a 16 x 16 grid
      int x = 0, y = 0, t = h;
      for (int sq = 1; sq < 16; sq *= 2) {
        const int rx = 1 & (t / 2), ry = 1 & (t ^ rx);
        if (ry == 0) {
          if (rx == 1) {
            x = sq - 1 - x;
            y = sq - 1 - y;
          }
          std::swap(x, y);
        }
        x += sq * rx;
        y += sq * ry;
        t /= 4;
      }
      if (x < nt && y < nt) wo.tile[n++] = (int16_t)(y * nt + x);
    }
    int most = 0;
    for (int r = 0; r <= 8; ++r) wo.start[r] = (int16_t)((int64_t)n * r / 8);
    for (int r = 0; r < 8; ++r) most = std::max(most, wo.start[r + 1] - wo.start[r]);
    blocks = 8ll * Sl * most;
  }
  if (w4)
    hipLaunchKernelGGL(crossnet_dw_w4_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       S(stream), u, xl, batch, d, Sl, part, grp == -2 ? -2 : (grp < 0 ? 0 : grp),
                       wo);
  else
    hipLaunchKernelGGL(crossnet_dw_kernel, dim3((unsigned)(tiles * Sl)), dim3(512), 0, S(stream),
                       u, xl, batch, d, Sl, part);
  hipLaunchKernelGGL(crossnet_dw_reduce_kernel, dim3((unsigned)ceil_div(n4, 256)), dim3(256), 0,
                     S(stream), part, Sl, n4, (int64_t)d * d, dw);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

size_t dr_crossnet_backward_workspace_size(int64_t batch, int d) {
  return (size_t)dr::ceil_div(batch > 0 ? batch : 1, dr::CB_ROWS) * (size_t)d * sizeof(float) + 256;
}

int dr_crossnet_backward_elem_bf16(const uint16_t* g, const uint16_t* x0, const uint16_t* lin,
                                   const float* acc_in, float* acc_out, uint16_t* u, float* db,
                                   int64_t batch, int d, void* ws, size_t ws_bytes,
                                   void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && d > 0 && d % 8 == 0, DR_INVALID_ARGUMENT,
             "dr_crossnet_backward_elem_bf16: d must be a multiple of 8");
  DR_REQUIRE(g && x0 && lin && acc_out && u && db, DR_INVALID_ARGUMENT, "null operand");
  DR_REQUIRE((((uintptr_t)g | (uintptr_t)x0 | (uintptr_t)lin | (uintptr_t)acc_in |
               (uintptr_t)acc_out | (uintptr_t)u | (uintptr_t)db) & 15) == 0,
             DR_INVALID_ARGUMENT, "operands must be 16-B aligned");
  DR_REQUIRE(ws && ws_bytes >= dr_crossnet_backward_workspace_size(batch, d), DR_INVALID_ARGUMENT,
             "workspace too small");
  if (batch == 0) return fill_bytes(db, 0, (size_t)d * sizeof(float), S(stream));
  const int64_t nblk = ceil_div(batch, CB_ROWS);
  DR_REQUIRE(nblk < 65536, DR_INVALID_ARGUMENT, "batch too large");
  float* dbp = static_cast<float*>(ws);
  dim3 grid((unsigned)ceil_div(d, 8 * 64), (unsigned)nblk);
  hipLaunchKernelGGL(crossnet_bwd_elem_kernel, grid, dim3(256), 0, S(stream), g, x0, lin, acc_in,
                     acc_out, u, dbp, batch, d);
  hipLaunchKernelGGL(crossnet_db_kernel, dim3((unsigned)ceil_div(d, 256)), dim3(256), 0, S(stream),
                     dbp, nblk, d, db);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_crossnet_layer_bf16(const uint16_t* x0, const uint16_t* xl, const uint16_t* W,
                           const float* bias, int64_t batch, int d, uint16_t* out,
                           void* stream) {
  return dr_crossnet_forward_bf16(x0, xl, W, bias, batch, d, out, nullptr, stream);
}

}  // extern "C"
