// mlp.hip -- bf16 MFMA GEMMs of the dense towers that sit on the embedding
// path's output: the DLRM top / bottom MLPs (modelzoo/DLRM/train.py:183-221,
// the reference's --bf16 switch) -- north_star: "MFMA used only for the
// dense CrossNet / top-MLP contraction".
//
//   C = act(A B^T + bias),  A [M, K], B [N, K] bf16 row-major (lda, ldb),
//   fp32 accumulate (v_mfma_f32_16x16x32_bf16), C bf16 or fp32.
//
// One "NT" form serves a Linear layer's three GEMMs: forward y = x W^T (A =
// x, B = W), input gradient dx = g W (A = g, B = W^T, a tiny transpose), and
// weight gradient dW = g^T x (A = g^T, B = x^T: both operands transposed by
// dr_transpose_bf16, then a GEMM whose K is the batch).  That last GEMM has
// an output of only N_out x K_in (512 x 512) over K = 65 536: a library GEMM
// runs it on a few dozen workgroups (DESIGN §6 "Huge-K weight gradients"),
// here it is split over K (grid.y = split) into fp32 partials that a second
// kernel sums in split order -- deterministic.
//
// Tile: 128 x 128 per block, 4 waves as 2 x 2 of 64 x 64 (4 x 4 MFMA 16x16
// tiles each), K step 64; operands staged global -> LDS by
// global_load_lds_dwordx4 into two LDS buffers (the DMA of K tile k+1 in
// flight while tile k is multiplied), XOR-swizzled image (conflict-free
// fragment reads), one counted vmcnt + one barrier per K step; blocks remapped
// so each XCD owns a contiguous range of tiles; 2 blocks per CU.  Epilogue
// through LDS: 8 columns per lane, bias + ReLU, 16-B (bf16) / 32-B (fp32)
// stores.
#include "dr_common.h"

namespace dr {
namespace {

typedef __attribute__((ext_vector_type(8))) short mbf16x8;
typedef __attribute__((ext_vector_type(4))) float mf32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int mu32x4;

constexpr int GM_BM = 128, GM_BN = 128, GM_BK = 64;
constexpr int GM_TILE = GM_BM * GM_BK * 2;  // 16 KB per operand per buffer

// 128 rows x 64 bf16 of X starting at (row0, k0): 4 wave instructions of 8
// rows x 128 B per wave; chunk c of row r lands at c ^ ((r >> 1) & 7).
__device__ __forceinline__ void gm_stage(const uint16_t* __restrict__ X, int64_t rows_valid,
                                         int64_t row0, int64_t ld, int64_t k0, char* tile,
                                         int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r0 = (wave * 4 + i) * 8;
    const int r = r0 + (lane >> 3);
    const int lc = (lane & 7) ^ ((r >> 1) & 7);
    int64_t gr = row0 + r;
    if (gr >= rows_valid) gr = rows_valid - 1;  // rows past the end feed discarded outputs
    const uint16_t* src = X + gr * ld + k0 + lc * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(tile + r0 * 128),
                                     16, 0, 0);
  }
}

__device__ __forceinline__ mbf16x8 gm_frag(const char* tile, int r, int lc) {
  return *reinterpret_cast<const mbf16x8*>(tile + r * 128 + ((lc ^ ((r >> 1) & 7)) << 4));
}

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  return (uint32_t)bf16_rne(a) | ((uint32_t)bf16_rne(b) << 16);
}

// EPI 0: fp32 partial of split z at C + z * M * ldc; 1: bf16 act(acc + bias);
// 2: fp32 act(acc + bias).  act DR_ACT_MASK: the result is zeroed where the
// bf16 aux [M, N] (ld_aux) is not > 0 -- the ReLU mask of the layer below
// applied to its input gradient (dx of the layer above) in the same pass.
template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(
    const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
    int64_t M, int64_t N, int64_t K, int64_t kchunk, const float* __restrict__ bias, int act,
    void* __restrict__ C, int64_t ldc, const uint16_t* __restrict__ aux, int64_t ld_aux) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * 2 * GM_TILE];  // [buf][A|B], 64 KB
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t orig = blockIdx.x;
  const int64_t xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t tile = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int64_t ntn = (N + GM_BN - 1) / GM_BN;
  const int64_t m0 = (tile / ntn) * GM_BM;
  const int64_t n0 = (tile % ntn) * GM_BN;
  const int64_t kb = (int64_t)blockIdx.y * kchunk;
  const int64_t ke = kb + kchunk < K ? kb + kchunk : K;
  const int nk = ke > kb ? (int)((ke - kb) / GM_BK) : 0;
  mf32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = mf32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  if (nk > 0) {
    gm_stage(A, M, m0, lda, kb, lds, wave, lane);
    gm_stage(B, N, n0, ldb, kb, lds + GM_TILE, wave, lane);
  }
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = lds + (kt & 1) * 2 * GM_TILE;
    if (kt + 1 < nk) {
      char* nxt = lds + ((kt + 1) & 1) * 2 * GM_TILE;
      gm_stage(A, M, m0, lda, kb + (int64_t)(kt + 1) * GM_BK, nxt, wave, lane);
      gm_stage(B, N, n0, ldb, kb + (int64_t)(kt + 1) * GM_BK, nxt + GM_TILE, wave, lane);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's tile-kt DMAs landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // ... and every other wave's
    asm volatile("" ::: "memory");
    const char* sA = cur;
    const char* sB = cur + GM_TILE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      mbf16x8 fa[4], fb[4];
      const int lc = kk * 4 + fq;
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = gm_frag(sA, wm * 64 + i * 16 + fr, lc);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = gm_frag(sB, wn * 64 + j * 16 + fr, lc);
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
  __syncthreads();
  // accumulators -> this wave's 16 KB LDS region (C/D map: col = lane & 15,
  // row = (lane >> 4) * 4 + reg; columns XOR-swizzled by (row >> 2) & 3)
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
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = it * 64 + lane;
    const int row = idx >> 3, cc = (idx & 7) * 8;
    const int64_t grow = m0 + wm * 64 + row;
    const int64_t gcol = n0 + wn * 64 + cc;
    if (grow >= M || gcol >= N) continue;
    const int pc = cc ^ (((row >> 2) & 3) << 4);
    const float4 l0 = *reinterpret_cast<const float4*>(ct + row * 64 + pc);
    const float4 l1 = *reinterpret_cast<const float4*>(ct + row * 64 + pc + 4);
    float v[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
    if (EPI == 0) {
      float* dst = reinterpret_cast<float*>(C) + (int64_t)blockIdx.y * M * ldc + grow * ldc + gcol;
      reinterpret_cast<float4*>(dst)[0] = make_float4(v[0], v[1], v[2], v[3]);
      reinterpret_cast<float4*>(dst)[1] = make_float4(v[4], v[5], v[6], v[7]);
      continue;
    }
    if (bias) {
      const float4 b0 = *reinterpret_cast<const float4*>(bias + gcol);
      const float4 b1 = *reinterpret_cast<const float4*>(bias + gcol + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
      v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    }
    if (act == DR_ACT_RELU) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
    } else if (act == DR_ACT_MASK) {
      const mu32x4 m = *reinterpret_cast<const mu32x4*>(aux + grow * ld_aux + gcol);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // bf16 > 0: sign bit clear and not +0 (the bits of a positive value)
        const uint32_t lo = m[e] & 0xffffu, hi = m[e] >> 16;
        if (!(lo != 0u && lo < 0x8000u && lo <= 0x7f80u)) v[2 * e] = 0.f;
        if (!(hi != 0u && hi < 0x8000u && hi <= 0x7f80u)) v[2 * e + 1] = 0.f;
      }
    }
    if (EPI == 1) {
      mu32x4 o = {pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]), pack_bf16(v[4], v[5]),
                  pack_bf16(v[6], v[7])};
      *reinterpret_cast<mu32x4*>(reinterpret_cast<uint16_t*>(C) + grow * ldc + gcol) = o;
    } else {
      float* dst = reinterpret_cast<float*>(C) + grow * ldc + gcol;
      reinterpret_cast<float4*>(dst)[0] = make_float4(v[0], v[1], v[2], v[3]);
      reinterpret_cast<float4*>(dst)[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

// ---------------------------------------------------------------------------
// Weight-gradient GEMM in "TN" form, no operand transposes:
//   C[n][k] = sum_b G[b][n] X[b][k]    (dW = g^T x of a Linear layer)
// G [rows, N], X [rows, K] bf16 row-major: the contraction runs down the rows
// of both.  Tile 128 (n) x 128 (k), 4 waves of 64 x 64 (v_mfma_f32_16x16x32_
// bf16), 64 contraction rows per step.  Each step stages a 64 x 128 chunk of
// G and of X into LDS as they lie in memory (global_load_lds_dwordx4, 256-B
// rows, 32-B slots XOR-swizzled by h(r) = (r & 3) | ((r >> 3) & 1) << 2),
// and the MFMA fragments -- 8 consecutive rows of one column per lane, for
// the A and the B operand alike -- come from ds_read_b64_tr_b16, the CDNA4
// transposing LDS read (4 rows x 16 columns per 16-lane group, column i to
// lane i): the two 8-row halves of a 32-row MFMA step are two such reads.
// With the swizzle the 8 rows a 32-lane half reads ({0..3, 8..11} + 16 h,
// {4..7, 12..15} + 16 h) sit in 8 distinct 32-B slots: conflict-free.
// Split over the rows (grid.y): fp32 partials summed in split order by
// gemm_splitk_reduce_kernel (deterministic); S = 1 writes C directly.
// colsum (optional): the column sums of G over each split, from the A
// fragments already in registers (blocks of the first k tile, waves wn = 0):
// a layer's bias gradient without another pass over g.
// Replaces transpose(g) + transpose(x) + an NT GEMM (3 passes).
// ---------------------------------------------------------------------------
typedef short tn_v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int tn_h(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

// 64 rows x 128 columns of X from (row0, col0) into img (64 x 256 B): 4 wave
// instructions of 4 rows each per wave.
__device__ __forceinline__ void tn_stage(const uint16_t* __restrict__ X, int64_t ld, int64_t row0,
                                         int64_t col0, int64_t cols, char* img, int wave,
                                         int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rb = (wave * 4 + i) * 4;
    const int r = rb + (lane >> 4), sl = lane & 15;
    const int c = (((sl >> 1) ^ tn_h(r)) << 1) | (sl & 1);   // logical 16-B chunk
    int64_t gc = col0 + c * 8;
    if (gc >= cols) gc = col0;  // columns past the end feed discarded outputs
    const uint16_t* src = X + (row0 + r) * ld + gc;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(img + rb * 256),
                                     16, 0, 0);
  }
}

// The fragment of 16 columns starting at slot m (16 bf16 = one 32-B slot)
// for the 32-row step kk: lane (g, 4q + p) reads rows kk*32 + 8g + q (+ 4).
__device__ __forceinline__ mbf16x8 tn_frag(const char* img, int kk, int m, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r1 = kk * 32 + 8 * g + q, r2 = r1 + 4;
  const tn_v4s a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) tn_v4s*)(img + r1 * 256 + ((m ^ tn_h(r1)) << 5) + 8 * p));
  const tn_v4s b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) tn_v4s*)(img + r2 * 256 + ((m ^ tn_h(r2)) << 5) + 8 * p));
  return mbf16x8{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
}

__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(
    const uint16_t* __restrict__ G, int64_t ldg, const uint16_t* __restrict__ X, int64_t ldx,
    int64_t N, int64_t K, int64_t bchunk, int64_t rows, float* __restrict__ C, int64_t ldc,
    int64_t split_stride, float* __restrict__ colsum) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * 2 * GM_TILE];  // [buf][G|X], 64 KB
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t orig = blockIdx.x;
  const int64_t xcd = orig % 8, qq = nwg / 8, rr = nwg % 8;
  const int64_t tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  const int64_t ntk = (K + 127) / 128;
  const int64_t m0 = (tile / ntk) * 128;   // n
  const int64_t n0 = (tile % ntk) * 128;   // k
  const int64_t b0 = (int64_t)blockIdx.y * bchunk;
  const int64_t be = b0 + bchunk < rows ? b0 + bchunk : rows;
  const int nk = be > b0 ? (int)((be - b0) / 64) : 0;
  const bool sums = colsum && n0 == 0 && wn == 0;
  mf32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = mf32x4{0.f, 0.f, 0.f, 0.f};
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  if (nk > 0) {
    tn_stage(G, ldg, b0, m0, N, lds, wave, lane);
    tn_stage(X, ldx, b0, n0, K, lds + GM_TILE, wave, lane);
  }
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = lds + (kt & 1) * 2 * GM_TILE;
    if (kt + 1 < nk) {
      char* nxt = lds + ((kt + 1) & 1) * 2 * GM_TILE;
      tn_stage(G, ldg, b0 + (int64_t)(kt + 1) * 64, m0, N, nxt, wave, lane);
      tn_stage(X, ldx, b0 + (int64_t)(kt + 1) * 64, n0, K, nxt + GM_TILE, wave, lane);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's step-kt DMAs landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // ... and every other wave's
    asm volatile("" ::: "memory");
    const char* sG = cur;
    const char* sX = cur + GM_TILE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      mbf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = tn_frag(sG, kk, wm * 4 + i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = tn_frag(sX, kk, wn * 4 + j, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      if (sums) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[i] += bf16_to_f32((uint16_t)fa[i][e]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // buffer kt&1 is restaged by iteration kt+1's DMA
    asm volatile("" ::: "memory");
  }
  if (sums) {
    // lane (g, li) summed rows 8g..8g+7 of each 32-row step for column li:
    // the 4 groups in a fixed butterfly
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      cs[i] += __shfl_xor(cs[i], 16, 64);
      cs[i] += __shfl_xor(cs[i], 32, 64);
      const int64_t col = m0 + wm * 64 + i * 16 + (lane & 15);
      if (lane < 16 && col < N) colsum[(int64_t)blockIdx.y * N + col] = cs[i];
    }
  }
  __syncthreads();
  // accumulators -> LDS (C/D map: col = lane & 15 = k, row = (lane >> 4) * 4
  // + reg = n), then 32-B fp32 row stores, as gemm_nt_kernel's epilogue
  const int fr = lane & 15, fq = lane >> 4;
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
  float* Cz = C + (int64_t)blockIdx.y * split_stride;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = it * 64 + lane;
    const int row = idx >> 3, cc = (idx & 7) * 8;
    const int64_t grow = m0 + wm * 64 + row;
    const int64_t gcol = n0 + wn * 64 + cc;
    if (grow >= N || gcol >= K) continue;
    const int pc = cc ^ (((row >> 2) & 3) << 4);
    const float4 l0 = *reinterpret_cast<const float4*>(ct + row * 64 + pc);
    const float4 l1 = *reinterpret_cast<const float4*>(ct + row * 64 + pc + 4);
    float* dst = Cz + grow * ldc + gcol;
    reinterpret_cast<float4*>(dst)[0] = l0;
    reinterpret_cast<float4*>(dst)[1] = l1;
  }
}

// Split-K reduction in split order: C = act(sum_z ws[z] + bias), 4 columns
// per thread.
__global__ void gemm_splitk_reduce_kernel(const float* __restrict__ ws, int S, int64_t M,
                                          int64_t N, const float* __restrict__ bias, int act,
                                          void* __restrict__ C, int64_t ldc, int out_bf16) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nq = N / 4;
  if (q >= M * nq) return;
  const int64_t m = q / nq, n = (q - m * nq) * 4;
  float4 s = reinterpret_cast<const float4*>(ws + m * N + n)[0];
  for (int z = 1; z < S; ++z) {
    const float4 p = reinterpret_cast<const float4*>(ws + (int64_t)z * M * N + m * N + n)[0];
    s.x += p.x;
    s.y += p.y;
    s.z += p.z;
    s.w += p.w;
  }
  if (bias) {
    s.x += bias[n];
    s.y += bias[n + 1];
    s.z += bias[n + 2];
    s.w += bias[n + 3];
  }
  if (act == DR_ACT_RELU) {
    s.x = s.x > 0.f ? s.x : 0.f;
    s.y = s.y > 0.f ? s.y : 0.f;
    s.z = s.z > 0.f ? s.z : 0.f;
    s.w = s.w > 0.f ? s.w : 0.f;
  }
  if (out_bf16) {
    uint2 o = {pack_bf16(s.x, s.y), pack_bf16(s.z, s.w)};
    *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(C) + m * ldc + n) = o;
  } else {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + m * ldc + n) = s;
  }
}

// gemm_tn's two split reductions in ONE launch: threads [0, nq_c) sum the
// dW partials (C = sum_z part[z], split order), threads [nq_c, nq_c + N/4)
// the column-sum partials (colsum = sum_z csp[z]) -- one launch per layer
// instead of two (a DLRM step runs five such layers).
__global__ void gemm_tn_reduce_kernel(const float* __restrict__ part, int S, int64_t N,
                                      int64_t K, float* __restrict__ C, int64_t ldc,
                                      const float* __restrict__ csp, float* __restrict__ colsum,
                                      int64_t nq_c) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const float* src;
  float* dst;
  int64_t stride;
  if (q < nq_c) {
    const int64_t kq = K / 4;
    const int64_t n = q / kq, k = (q - n * kq) * 4;
    src = part + n * K + k;
    stride = N * K;
    dst = C + n * ldc + k;
  } else {
    const int64_t c = (q - nq_c) * 4;
    if (!colsum || c >= N) return;
    src = csp + c;
    stride = N;
    dst = colsum + c;
  }
  float4 s = reinterpret_cast<const float4*>(src)[0];
  for (int z = 1; z < S; ++z) {
    const float4 p = reinterpret_cast<const float4*>(src + (int64_t)z * stride)[0];
    s.x += p.x;
    s.y += p.y;
    s.z += p.z;
    s.w += p.w;
  }
  *reinterpret_cast<float4*>(dst) = s;
}

// out[c][r] = in[r][c] (bf16), 64 x 64 tiles through LDS: each thread loads
// two 16-B row vectors and stores two 16-B column vectors.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const uint16_t* __restrict__ in,
                                                             int64_t rows, int64_t cols,
                                                             int64_t ld_in,
                                                             uint16_t* __restrict__ out,
                                                             int64_t ld_out,
                                                             float* __restrict__ colsum) {
  __shared__ uint16_t t[64][66];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int v = tid + h * 256;  // 512 vectors of 8: row v / 8, column chunk v % 8
    const int r = v >> 3, cc = (v & 7) * 8;
    mu32x4 x = {0u, 0u, 0u, 0u};
    if (r0 + r < rows && c0 + cc < cols)
      x = *reinterpret_cast<const mu32x4*>(in + (r0 + r) * ld_in + c0 + cc);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      t[r][cc + 2 * e] = (uint16_t)(x[e] & 0xffff);
      t[r][cc + 2 * e + 1] = (uint16_t)(x[e] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int v = tid + h * 256;  // output row c = v / 8 (an input column), rows chunk v % 8
    const int c = v >> 3, rc = (v & 7) * 8;
    mu32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      o[e] = (uint32_t)t[rc + 2 * e][c] | ((uint32_t)t[rc + 2 * e + 1][c] << 16);
    if (colsum) {
      // column c's sum over this tile's 64 rows (rows past the end are 0):
      // 8 rows in order per lane, then the 8 lanes of the column (v & 7 =
      // consecutive lanes) by a fixed xor butterfly -- deterministic
      float sum = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += bf16_to_f32(t[rc + e][c]);
      sum += __shfl_xor(sum, 1, 64);
      sum += __shfl_xor(sum, 2, 64);
      sum += __shfl_xor(sum, 4, 64);
      if ((v & 7) == 0 && c0 + c < cols) colsum[(int64_t)blockIdx.y * cols + c0 + c] = sum;
    }
    if (c0 + c >= cols || r0 + rc >= rows) continue;
    *reinterpret_cast<mu32x4*>(out + (c0 + c) * ld_out + r0 + rc) = o;
  }
}


// ---------------------------------------------------------------------------
// The DLRM output layer on top of the bf16 top MLP (modelzoo/DLRM/train.py:
// 241-249 under --bf16: dense(units=1) in bf16, then sigmoid): a GEMV with
// N = 1 that a library GEMM runs as three kernels (forward, dx, and a
// K = 65 536 dW on few workgroups: 15 + 19 + 70 us per DLRM step) plus the
// casts around them and the top layer's ReLU-mask multiply.
//   forward  z[b] = bf16( sum_k h[b,k] * bf16(w[k]) + bias )   (fp32 sum)
//   backward with gz = bf16(dL/dz):
//            dh[b,k] = h[b,k] > 0 ? bf16(gz[b] * bf16(w[k])) : 0   (the
//                      top layer's ReLU derivative applied in the same pass)
//            dw_part[blk][k] = sum over the block's rows of gz[b] * h[b,k]
//            db_part[blk]    = sum over the block's rows of gz[b]
// K in {64, 128, 256, 512}: L = K / 8 lanes per row, 8 bf16 per lane; every
// sum is in a fixed order (8 columns per lane, then an xor butterfly; rows
// of a block in a fixed lane / LDS order), so results are deterministic.
// ---------------------------------------------------------------------------
// F32: the fp32 output layer on a bf16-computed tower (DeepFM --bf16,
// train.py:213-221: the tower output cast to fp32, then dense(units=1) in
// fp32): w fp32, the logit and gz unrounded.  h is read as bf16 either way
// (its fp32 widening is exact).
template <bool F32>
__device__ __forceinline__ void head_w8(const void* w, int lc, float (&wf)[8]) {
  if constexpr (F32) {
    const float4 a = reinterpret_cast<const float4*>(w)[lc * 2];
    const float4 b = reinterpret_cast<const float4*>(w)[lc * 2 + 1];
    wf[0] = a.x; wf[1] = a.y; wf[2] = a.z; wf[3] = a.w;
    wf[4] = b.x; wf[5] = b.y; wf[6] = b.z; wf[7] = b.w;
  } else {
    const mu32x4 wv = *reinterpret_cast<const mu32x4*>(static_cast<const uint16_t*>(w) + lc * 8);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float2 c = bf16x2_to_f2(wv[e]);
      wf[2 * e] = c.x;
      wf[2 * e + 1] = c.y;
    }
  }
}

template <int L, bool F32>
__global__ __launch_bounds__(256) void head_fwd_kernel(const uint16_t* __restrict__ h, int64_t ldh,
                                                       int64_t B, const void* __restrict__ w,
                                                       const float* __restrict__ bias,
                                                       float* __restrict__ z) {
  constexpr int RPB = 256 / L;  // rows per block
  const int tid = threadIdx.x;
  const int lc = tid % L;
  const int64_t b = (int64_t)blockIdx.x * RPB + tid / L;
  const bool ok = b < B;
  const mu32x4 hv = *reinterpret_cast<const mu32x4*>(h + (ok ? b : 0) * ldh + lc * 8);
  float wf[8];
  head_w8<F32>(w, lc, wf);
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float2 a = bf16x2_to_f2(hv[e]);
    s = fmaf(a.x, wf[2 * e], s);
    s = fmaf(a.y, wf[2 * e + 1], s);
  }
#pragma unroll
  for (int m = 1; m < L; m <<= 1) s += __shfl_xor(s, m, 64);
  const float zz = bias ? s + *bias : s;
  if (ok && lc == 0) z[b] = F32 ? zz : bf16_to_f32(bf16_rne(zz));
}

template <int L, bool F32>
__global__ __launch_bounds__(256) void head_bwd_kernel(const uint16_t* __restrict__ h, int64_t ldh,
                                                       int64_t B, const void* __restrict__ w,
                                                       const float* __restrict__ gz,
                                                       uint16_t* __restrict__ dh, int64_t lddh,
                                                       int rows_per_block,
                                                       float* __restrict__ dw_part,
                                                       float* __restrict__ db_part) {
  constexpr int RPS = 256 / L;  // rows per sweep of the block
  constexpr int K = L * 8;
  __shared__ float red[RPS][K + 4];
  __shared__ float redb[RPS];
  const int tid = threadIdx.x;
  const int lc = tid % L, rs = tid / L;
  float wf[8];
  head_w8<F32>(w, lc, wf);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float accb = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  // rows_per_block / RPS rows per thread, all of them loaded before use
  // (the loads of one thread are independent: unrolled, they are in flight
  // together instead of one latency per row)
#pragma unroll 8
  for (int i = rs; i < rows_per_block; i += RPS) {
    const int64_t b = r0 + i;
    if (b >= B) break;
    const float g = F32 ? gz[b] : bf16_to_f32(bf16_rne(gz[b]));
    const mu32x4 hv = *reinterpret_cast<const mu32x4*>(h + b * ldh + lc * 8);
    mu32x4 ov;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float2 a = bf16x2_to_f2(hv[e]);
      acc[2 * e] = fmaf(g, a.x, acc[2 * e]);
      acc[2 * e + 1] = fmaf(g, a.y, acc[2 * e + 1]);
      const float d0 = a.x > 0.f ? g * wf[2 * e] : 0.f;
      const float d1 = a.y > 0.f ? g * wf[2 * e + 1] : 0.f;
      ov[e] = (uint32_t)bf16_rne(d0) | ((uint32_t)bf16_rne(d1) << 16);
    }
    *reinterpret_cast<mu32x4*>(dh + b * lddh + lc * 8) = ov;
    accb += g;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rs][lc * 8 + e] = acc[e];
  if (lc == 0) redb[rs] = accb;
  __syncthreads();
  // column sums over the RPS row sweeps, in sweep order
  for (int c = tid; c < K; c += 256) {
    float t = 0.f;
    for (int r = 0; r < RPS; ++r) t += red[r][c];
    dw_part[(int64_t)blockIdx.x * K + c] = t;
  }
  if (tid == 0) {
    float t = 0.f;
    for (int r = 0; r < RPS; ++r) t += redb[r];
    db_part[blockIdx.x] = t;
  }
}


// dL/dy of a ReLU layer's bf16 output y, from an fp32 gradient (row stride
// ldg): out = bf16(g) where y > 0, else 0 -- the MFMA tower's entry when
// its output was widened to fp32 for the layer above (one pass instead of
// a cast, a compare and a multiply).  8 columns per thread.
__global__ __launch_bounds__(256) void relu_grad_bf16_kernel(const float* __restrict__ g,
                                                             int64_t ldg,
                                                             const uint16_t* __restrict__ y,
                                                             int64_t ldy, int64_t rows,
                                                             int64_t cols,
                                                             uint16_t* __restrict__ out,
                                                             int64_t ldo) {
  const int64_t c8 = cols / 8;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * c8) return;
  const int64_t r = i / c8, c = (i - r * c8) * 8;
  const float4 g0 = *reinterpret_cast<const float4*>(g + r * ldg + c);
  const float4 g1 = *reinterpret_cast<const float4*>(g + r * ldg + c + 4);
  const mu32x4 yv = *reinterpret_cast<const mu32x4*>(y + r * ldy + c);
  const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
  mu32x4 ov;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float2 yy = bf16x2_to_f2(yv[e]);
    const uint32_t lo = yy.x > 0.f ? bf16_rne(gv[2 * e]) : 0u;
    const uint32_t hi = yy.y > 0.f ? bf16_rne(gv[2 * e + 1]) : 0u;
    ov[e] = lo | (hi << 16);
  }
  *reinterpret_cast<mu32x4*>(out + r * ldo + c) = ov;
}

}  // namespace
}  // namespace dr

extern "C" {

size_t dr_gemm_nt_workspace_size(int64_t M, int64_t N, int split_k) {
  if (split_k <= 1) return 0;
  return (size_t)split_k * (size_t)(M > 0 ? M : 1) * (size_t)(N > 0 ? N : 1) * sizeof(float) + 256;
}

int dr_gemm_nt_bf16_ex(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, int64_t M,
                       int64_t N, int64_t K, const float* bias, int act, const uint16_t* aux,
                       int64_t ld_aux, void* C, int64_t ldc, int c_fp32, int split_k, void* ws,
                       size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(A && B && C && M >= 0 && N >= 0 && K >= 0, DR_INVALID_ARGUMENT, "bad argument");
  DR_REQUIRE(K % 64 == 0 && N % 8 == 0, DR_INVALID_ARGUMENT,
             "dr_gemm_nt_bf16: K must be a multiple of 64 and N of 8 (pad with zeros)");
  DR_REQUIRE(lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 && lda >= K && ldb >= K && ldc >= N,
             DR_INVALID_ARGUMENT, "dr_gemm_nt_bf16: strides must be multiples of 8 and >= K / N");
  DR_REQUIRE((((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) == 0 &&
                 (!bias || ((uintptr_t)bias & 15) == 0),
             DR_INVALID_ARGUMENT, "dr_gemm_nt_bf16: pointers must be 16-B aligned");
  DR_REQUIRE(act == DR_ACT_NONE || act == DR_ACT_RELU || act == DR_ACT_MASK, DR_INVALID_ARGUMENT,
             "unknown act %d", act);
  DR_REQUIRE(act != DR_ACT_MASK || (aux && ld_aux >= N && ld_aux % 8 == 0 &&
                                    ((uintptr_t)aux & 15) == 0),
             DR_INVALID_ARGUMENT, "DR_ACT_MASK needs a 16-B aligned aux with ld_aux >= N, %% 8");
  if (M == 0 || N == 0) return DR_OK;
  hipStream_t st = S(stream);
  const int64_t tiles = ((M + GM_BM - 1) / GM_BM) * ((N + GM_BN - 1) / GM_BN);
  DR_REQUIRE(tiles < (1ll << 31), DR_INVALID_ARGUMENT, "dr_gemm_nt_bf16: too many tiles");
  const int64_t ksteps = K / GM_BK;
  int S_ = split_k < 1 ? 1 : split_k;
  if (S_ > ksteps && ksteps > 0) S_ = (int)ksteps;
  const int64_t kchunk = (ksteps > 0 ? (ksteps + S_ - 1) / S_ : 1) * GM_BK;
  if (S_ == 1) {
    if (c_fp32)
      hipLaunchKernelGGL(gemm_nt_kernel<2>, dim3((unsigned)tiles, 1), dim3(256), 0, st, A, lda, B,
                         ldb, M, N, K, kchunk, bias, act, C, ldc, aux, ld_aux);
    else
      hipLaunchKernelGGL(gemm_nt_kernel<1>, dim3((unsigned)tiles, 1), dim3(256), 0, st, A, lda, B,
                         ldb, M, N, K, kchunk, bias, act, C, ldc, aux, ld_aux);
    DR_LAUNCH_CHECK();
    return DR_OK;
  }
  DR_REQUIRE(act != DR_ACT_MASK, DR_INVALID_ARGUMENT, "DR_ACT_MASK is not built for split-K");
  DR_REQUIRE(ws && ws_bytes >= dr_gemm_nt_workspace_size(M, N, S_), DR_INVALID_ARGUMENT,
             "dr_gemm_nt_bf16: split-K workspace too small");
  DR_REQUIRE(((uintptr_t)ws & 15) == 0, DR_INVALID_ARGUMENT, "workspace must be 16-B aligned");
  hipLaunchKernelGGL(gemm_nt_kernel<0>, dim3((unsigned)tiles, (unsigned)S_), dim3(256), 0, st, A,
                     lda, B, ldb, M, N, K, kchunk, (const float*)nullptr, 0, ws, N,
                     (const uint16_t*)nullptr, (int64_t)0);
  const int64_t quads = M * (N / 4);
  hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3((unsigned)ceil_div(quads, 256)), dim3(256),
                     0, st, (const float*)ws, S_, M, N, bias, act, C, ldc, c_fp32 ? 0 : 1);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_gemm_nt_bf16(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, int64_t M,
                    int64_t N, int64_t K, const float* bias, int act, void* C, int64_t ldc,
                    int c_fp32, int split_k, void* ws, size_t ws_bytes, void* stream) {
  return dr_gemm_nt_bf16_ex(A, lda, B, ldb, M, N, K, bias, act, nullptr, 0, C, ldc, c_fp32,
                            split_k, ws, ws_bytes, stream);
}

int dr_transpose_bf16(const uint16_t* in, int64_t rows, int64_t cols, int64_t ld_in,
                      uint16_t* out, int64_t ld_out, void* stream) {
  return dr_transpose_bf16_colsum(in, rows, cols, ld_in, out, ld_out, nullptr, stream);
}

int dr_transpose_bf16_colsum(const uint16_t* in, int64_t rows, int64_t cols, int64_t ld_in,
                             uint16_t* out, int64_t ld_out, float* col_partials, void* stream) {
  using namespace dr;
  DR_REQUIRE(in && out && rows >= 0 && cols >= 0, DR_INVALID_ARGUMENT, "bad argument");
  DR_REQUIRE(rows % 8 == 0 && cols % 8 == 0 && ld_in % 8 == 0 && ld_out % 8 == 0 &&
                 ld_in >= cols && ld_out >= rows,
             DR_INVALID_ARGUMENT, "dr_transpose_bf16: rows, cols and strides multiples of 8");
  DR_REQUIRE(((((uintptr_t)in) | ((uintptr_t)out)) & 15) == 0, DR_INVALID_ARGUMENT,
             "dr_transpose_bf16: pointers must be 16-B aligned");
  if (rows == 0 || cols == 0) return DR_OK;
  const dim3 grid((unsigned)ceil_div(cols, 64), (unsigned)ceil_div(rows, 64));
  hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, S(stream), in, rows, cols, ld_in,
                     out, ld_out, col_partials);
  DR_LAUNCH_CHECK();
  return DR_OK;
}


static constexpr int kHeadRows = 64;    // rows per backward block (1024 blocks at B = 65 536)

size_t dr_mlp_head_grad_partials(int64_t batch) {
  return (size_t)(batch > 0 ? dr::ceil_div(batch, kHeadRows) : 0);
}

int dr_mlp_head_forward_bf16(const uint16_t* h, int64_t ldh, int64_t batch, int k,
                             const void* w, int w_fp32, const float* bias, float* z,
                             void* stream) {
  using namespace dr;
  DR_REQUIRE(h && w && z && batch >= 0 && (k == 64 || k == 128 || k == 256 || k == 512) &&
                 ldh >= k && ldh % 8 == 0,
             DR_INVALID_ARGUMENT, "dr_mlp_head_forward_bf16: k in {64,128,256,512}, ldh % 8 == 0");
  DR_REQUIRE(((((uintptr_t)h) | ((uintptr_t)w)) & 15) == 0, DR_INVALID_ARGUMENT,
             "dr_mlp_head_forward_bf16: h and w must be 16-B aligned");
  if (batch == 0) return DR_OK;
  const int L = k / 8;
  const unsigned grid = (unsigned)ceil_div(batch, 256 / L);
#define DR_HEAD_F(LL)                                                                          \
  do {                                                                                         \
    if (w_fp32)                                                                                \
      hipLaunchKernelGGL((head_fwd_kernel<LL, true>), dim3(grid), dim3(256), 0, S(stream), h,   \
                         ldh, batch, w, bias, z);                                              \
    else                                                                                       \
      hipLaunchKernelGGL((head_fwd_kernel<LL, false>), dim3(grid), dim3(256), 0, S(stream), h,  \
                         ldh, batch, w, bias, z);                                              \
  } while (0)
  if (L == 8) DR_HEAD_F(8);
  else if (L == 16) DR_HEAD_F(16);
  else if (L == 32) DR_HEAD_F(32);
  else DR_HEAD_F(64);
#undef DR_HEAD_F
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_mlp_head_backward_bf16(const uint16_t* h, int64_t ldh, int64_t batch, int k,
                              const void* w, int w_fp32, const float* grad_z, uint16_t* grad_h,
                              int64_t ld_grad_h, float* dw_partials, float* db_partials,
                              void* stream) {
  using namespace dr;
  DR_REQUIRE(h && w && grad_z && grad_h && dw_partials && db_partials && batch >= 0 &&
                 (k == 64 || k == 128 || k == 256 || k == 512) && ldh >= k && ldh % 8 == 0 &&
                 ld_grad_h >= k && ld_grad_h % 8 == 0,
             DR_INVALID_ARGUMENT, "dr_mlp_head_backward_bf16: bad shape");
  DR_REQUIRE(((((uintptr_t)h) | ((uintptr_t)w) | ((uintptr_t)grad_h)) & 15) == 0,
             DR_INVALID_ARGUMENT, "dr_mlp_head_backward_bf16: h, w, grad_h must be 16-B aligned");
  if (batch == 0) return DR_OK;
  const int L = k / 8;
  const unsigned grid = (unsigned)ceil_div(batch, kHeadRows);
#define DR_HEAD_B(LL)                                                                          \
  do {                                                                                         \
    if (w_fp32)                                                                                \
      hipLaunchKernelGGL((head_bwd_kernel<LL, true>), dim3(grid), dim3(256), 0, S(stream), h,   \
                         ldh, batch, w, grad_z, grad_h, ld_grad_h, kHeadRows, dw_partials,     \
                         db_partials);                                                         \
    else                                                                                       \
      hipLaunchKernelGGL((head_bwd_kernel<LL, false>), dim3(grid), dim3(256), 0, S(stream), h,  \
                         ldh, batch, w, grad_z, grad_h, ld_grad_h, kHeadRows, dw_partials,     \
                         db_partials);                                                         \
  } while (0)
  if (L == 8) DR_HEAD_B(8);
  else if (L == 16) DR_HEAD_B(16);
  else if (L == 32) DR_HEAD_B(32);
  else DR_HEAD_B(64);
#undef DR_HEAD_B
  DR_LAUNCH_CHECK();
  return DR_OK;
}


int dr_relu_grad_bf16(const float* grad, int64_t ld_grad, const uint16_t* y, int64_t ld_y,
                      int64_t rows, int64_t cols, uint16_t* out, int64_t ld_out, void* stream) {
  using namespace dr;
  DR_REQUIRE(grad && y && out && rows >= 0 && cols >= 0 && cols % 8 == 0 && ld_grad % 4 == 0 &&
                 ld_y % 8 == 0 && ld_out % 8 == 0 && ld_grad >= cols && ld_y >= cols &&
                 ld_out >= cols,
             DR_INVALID_ARGUMENT, "dr_relu_grad_bf16: cols and strides multiples of 8 (grad: 4)");
  DR_REQUIRE(((((uintptr_t)grad) | ((uintptr_t)y) | ((uintptr_t)out)) & 15) == 0,
             DR_INVALID_ARGUMENT, "dr_relu_grad_bf16: pointers must be 16-B aligned");
  if (rows == 0 || cols == 0) return DR_OK;
  const int64_t n = rows * (cols / 8);
  hipLaunchKernelGGL(relu_grad_bf16_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0,
                     S(stream), grad, ld_grad, y, ld_y, rows, cols, out, ld_out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}


size_t dr_gemm_tn_workspace_size(int64_t N, int64_t K, int split_k, int with_colsum) {
  if (split_k <= 1 && !with_colsum) return 0;
  const size_t s = (size_t)(split_k > 1 ? split_k : 1);
  size_t b = split_k > 1 ? s * (size_t)(N > 0 ? N : 1) * (size_t)(K > 0 ? K : 1) * sizeof(float) : 0;
  b = (b + 255) & ~size_t(255);
  if (with_colsum) b += s * (size_t)(N > 0 ? N : 1) * sizeof(float);
  return b + 256;
}

int dr_gemm_tn_bf16(const uint16_t* G, int64_t ldg, const uint16_t* X, int64_t ldx, int64_t rows,
                    int64_t N, int64_t K, float* C, int64_t ldc, float* colsum, int split_k,
                    void* ws, size_t ws_bytes, void* stream) {
  using namespace dr;
  DR_REQUIRE(G && X && C && rows >= 0 && N >= 0 && K >= 0, DR_INVALID_ARGUMENT, "bad argument");
  DR_REQUIRE(rows % 64 == 0 && N % 8 == 0 && K % 8 == 0, DR_INVALID_ARGUMENT,
             "dr_gemm_tn_bf16: rows must be a multiple of 64, N and K of 8");
  DR_REQUIRE(ldg % 8 == 0 && ldx % 8 == 0 && ldc % 4 == 0 && ldg >= N && ldx >= K && ldc >= K,
             DR_INVALID_ARGUMENT, "dr_gemm_tn_bf16: strides must be multiples of 8 (ldc: 4)");
  DR_REQUIRE((((uintptr_t)G | (uintptr_t)X | (uintptr_t)C) & 15) == 0 &&
                 (!colsum || ((uintptr_t)colsum & 15) == 0),
             DR_INVALID_ARGUMENT, "dr_gemm_tn_bf16: pointers must be 16-B aligned");
  if (N == 0 || K == 0) return DR_OK;
  hipStream_t st = S(stream);
  if (rows == 0) {
    for (int64_t n = 0; n < N; ++n) {
      int rc = fill_bytes(C + n * ldc, 0, (size_t)K * sizeof(float), st);
      if (rc) return rc;
    }
    return colsum ? fill_bytes(colsum, 0, (size_t)N * sizeof(float), st) : DR_OK;
  }
  const int64_t tiles = ((N + 127) / 128) * ((K + 127) / 128);
  DR_REQUIRE(tiles < (1ll << 31), DR_INVALID_ARGUMENT, "dr_gemm_tn_bf16: too many tiles");
  const int64_t steps = rows / 64;
  int S_ = split_k < 1 ? 1 : split_k;
  if (S_ > steps) S_ = (int)steps;
  const int64_t bchunk = ((steps + S_ - 1) / S_) * 64;
  S_ = (int)((rows + bchunk - 1) / bchunk);
  const bool direct = S_ == 1;
  const bool need_ws = !direct || colsum;
  DR_REQUIRE(!need_ws || (ws && ws_bytes >= dr_gemm_tn_workspace_size(N, K, S_, colsum != nullptr)),
             DR_INVALID_ARGUMENT, "dr_gemm_tn_bf16: workspace too small");
  DR_REQUIRE(!need_ws || ((uintptr_t)ws & 15) == 0, DR_INVALID_ARGUMENT,
             "workspace must be 16-B aligned");
  float* part = direct ? C : static_cast<float*>(ws);
  size_t off = direct ? 0 : (((size_t)S_ * N * K * sizeof(float)) + 255) & ~size_t(255);
  float* csp = colsum ? reinterpret_cast<float*>(static_cast<char*>(ws) + off) : nullptr;
  hipLaunchKernelGGL(gemm_tn_kernel, dim3((unsigned)tiles, (unsigned)S_), dim3(256), 0, st, G, ldg,
                     X, ldx, N, K, bchunk, rows, part, direct ? ldc : K,
                     direct ? (int64_t)0 : N * K, csp);
  // (K % 8 == 0 and N % 8 == 0: whole float4 quads on both sides)
  const int64_t nq_c = direct ? 0 : N * (K / 4);
  const int64_t nq = nq_c + (colsum ? N / 4 : 0);
  if (nq > 0)
    hipLaunchKernelGGL(gemm_tn_reduce_kernel, dim3((unsigned)ceil_div(nq, 256)), dim3(256), 0, st,
                       (const float*)part, S_, N, K, C, ldc, (const float*)csp, colsum, nq_c);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // extern "C"
