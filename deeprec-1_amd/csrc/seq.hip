// seq.hip -- user-behaviour sequence ops of DIN (BASELINE configs[3]; SURVEY.md
// 8d config 4 and 8f #4): the attention over a sample's behaviour history.
//   dr_din_attention_input   din_all = [q, f, q-f, q*f]
//                            (modelzoo/DIN/script/utils.py:280-282)
//   dr_din_attention_pool    masked softmax of the scores + weighted sum of
//                            the facts (utils.py:286-303, mode 'SUM'), and the
//                            plain history sum item_his_eb_sum (script/model.py:98)
//                            from the same pass over the facts
//   and their backward passes.
// All four are HBM-bound (the facts [B, T, H] and the attention-MLP input
// [B, T, 4H] dominate the bytes); the MLP itself (144 -> 80 -> 40 -> 1) is a
// plain library GEMM.  Rows are moved in float4 chunks when H % 4 == 0.  A
// per-sample pass uses one 64-lane block, so its LDS exchanges are ordered by
// s_barrier alone; lane (r, c) owns chunk c of rows r, r + R, r + 2R, ... with
// R = 64 / (H / VEC), and partial sums are combined through LDS in a fixed
// order (deterministic, run to run).
#include "dr_common.h"

#include <math.h>

#include <type_traits>

namespace dr {

// tf.ones_like(scores) * (-2 ** 32 + 1) in float32 (utils.py:291)
static constexpr float kDinPad = -4294967296.0f;

template <int VEC>
__device__ __forceinline__ void ldv(float (&v)[VEC], const float* p) {
  if constexpr (VEC == 4) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  } else {
#pragma unroll
    for (int k = 0; k < VEC; ++k) v[k] = p[k];
  }
}

template <int VEC>
__device__ __forceinline__ void stv(float* p, const float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    nt_store(make_float4(v[0], v[1], v[2], v[3]), reinterpret_cast<float4*>(p));
  } else {
#pragma unroll
    for (int k = 0; k < VEC; ++k) p[k] = v[k];
  }
}

__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// din_all[b, t] = [q_b, f_bt, q_b - f_bt, q_b * f_bt]; thread per (b, t, chunk).
template <int VEC>
__global__ __launch_bounds__(256) void din_input_kernel(const float* __restrict__ q,
                                                        const float* __restrict__ f, int64_t B,
                                                        int64_t T, int H, float* __restrict__ out) {
  const int n4 = H / VEC;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * T * n4) return;
  const int64_t bt = i / n4;
  const int c = (int)(i - bt * n4) * VEC;
  const int64_t b = bt / T;
  float qv[VEC], fv[VEC], dv[VEC], pv[VEC];
  ldv<VEC>(qv, q + b * H + c);
  ldv<VEC>(fv, f + bt * H + c);
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    dv[k] = qv[k] - fv[k];
    pv[k] = qv[k] * fv[k];
  }
  float* o = out + bt * 4 * H + c;
  stv<VEC>(o, qv);
  stv<VEC>(o + H, fv);
  stv<VEC>(o + 2 * H, dv);
  stv<VEC>(o + 3 * H, pv);
}

// Backward of din_input (autodiff of tile + concat + sub + mul):
//   grad_f[b, t] (=|+=) g_f - g_d + g_p * q_b
//   grad_q[b]    = sum_t (g_q + g_d) + g_p * f_bt
// One 64-lane block per sample.
template <int VEC>
__global__ __launch_bounds__(64) void din_input_grad_kernel(
    const float* __restrict__ q, const float* __restrict__ f, const float* __restrict__ g,
    int64_t T, int H, float* __restrict__ gq, float* __restrict__ gf, int accumulate) {
  __shared__ float part[64 * VEC];
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const int n4 = H / VEC;
  const int R = 64 / n4;
  const int r = lane / n4;
  const int c = (lane - r * n4) * VEC;
  if (r < R) {
    float qv[VEC], acc[VEC];
    ldv<VEC>(qv, q + b * H + c);
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
    for (int64_t t = r; t < T; t += R) {
      const int64_t bt = b * T + t;
      const float* gp = g + bt * 4 * H + c;
      float g0[VEC], g1[VEC], g2[VEC], g3[VEC], fv[VEC], o[VEC];
      ldv<VEC>(g0, gp);
      ldv<VEC>(g1, gp + H);
      ldv<VEC>(g2, gp + 2 * H);
      ldv<VEC>(g3, gp + 3 * H);
      ldv<VEC>(fv, f + bt * H + c);
      float* dst = gf + bt * H + c;
      float prev[VEC];
      if (accumulate) ldv<VEC>(prev, dst);
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        acc[k] += (g0[k] + g2[k]) + g3[k] * fv[k];
        o[k] = (g1[k] - g2[k]) + g3[k] * qv[k];
        if (accumulate) o[k] = prev[k] + o[k];
      }
      stv<VEC>(dst, o);
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) part[r * H + c + k] = acc[k];
  }
  __syncthreads();
  for (int cc = lane; cc < H; cc += 64) {
    float s = 0.f;
    for (int rr = 0; rr < R; ++rr) s += part[rr * H + cc];
    gq[b * H + cc] = s;
  }
}

// Masked softmax attention pooling, one 64-lane block per sample:
//   s_t = mask_t == 1 ? scores_t : float(-2^32 + 1)
//   alpha = softmax_t(s)             (exp(s - max) / sum, Eigen's order)
//   att[b] = sum_t alpha_t f_bt      (tf.matmul(scores, facts), mode SUM)
//   hsum[b] = sum_t f_bt             (reduce_sum over every position, padding
//                                     included, script/model.py:98)
// Dynamic LDS: T alphas + 2 x 64*VEC partial sums.
template <int VEC>
__global__ __launch_bounds__(64) void din_pool_kernel(const float* __restrict__ scores,
                                                      const float* __restrict__ mask,
                                                      const float* __restrict__ f, int64_t T,
                                                      int H, float* __restrict__ att,
                                                      float* __restrict__ hsum,
                                                      float* __restrict__ alphas) {
  extern __shared__ float lds[];
  float* al = lds;
  float* pa = lds + ((T + 3) & ~3ll);
  float* ps = pa + 64 * VEC;
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  float m = -INFINITY;
  for (int64_t t = lane; t < T; t += 64) {
    const float s = mask[b * T + t] == 1.f ? scores[b * T + t] : kDinPad;
    al[t] = s;
    m = fmaxf(m, s);
  }
  m = wave_max(m);
  float z = 0.f;
  for (int64_t t = lane; t < T; t += 64) {
    const float e = expf(al[t] - m);
    al[t] = e;
    z += e;
  }
  z = wave_sum(z);
  for (int64_t t = lane; t < T; t += 64) {
    const float a = al[t] / z;
    al[t] = a;
    alphas[b * T + t] = a;
  }
  __syncthreads();
  const int n4 = H / VEC;
  const int R = 64 / n4;
  const int r = lane / n4;
  const int c = (lane - r * n4) * VEC;
  if (r < R) {
    float aa[VEC], as[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) aa[k] = as[k] = 0.f;
    for (int64_t t = r; t < T; t += R) {
      float fv[VEC];
      ldv<VEC>(fv, f + (b * T + t) * H + c);
      const float a = al[t];
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        aa[k] += a * fv[k];
        as[k] += fv[k];
      }
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      pa[r * H + c + k] = aa[k];
      ps[r * H + c + k] = as[k];
    }
  }
  __syncthreads();
  for (int cc = lane; cc < H; cc += 64) {
    float sa = 0.f, ss = 0.f;
    for (int rr = 0; rr < R; ++rr) {
      sa += pa[rr * H + cc];
      ss += ps[rr * H + cc];
    }
    att[b * H + cc] = sa;
    if (hsum) hsum[b * H + cc] = ss;
  }
}

// Its backward (one 64-lane block per sample):
//   da_t      = g_att . f_bt
//   gscore_t  = mask_t == 1 ? (da_t - sum_t' da_t' alpha_t') alpha_t : 0
//               (softmax grad; tf.where routes nothing to the padding)
//   grad_f_bt = alpha_t g_att + g_sum
// Dynamic LDS: T alphas + T da + 64 partial dots.
template <int VEC>
__global__ __launch_bounds__(64) void din_pool_grad_kernel(
    const float* __restrict__ alphas, const float* __restrict__ mask, const float* __restrict__ f,
    const float* __restrict__ g_att, const float* __restrict__ g_sum, int64_t T, int H,
    float* __restrict__ gscore, float* __restrict__ gf) {
  extern __shared__ float lds[];
  const int64_t Tp = (T + 3) & ~3ll;
  float* al = lds;
  float* da = lds + Tp;
  float* pb = da + Tp;
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  for (int64_t t = lane; t < T; t += 64) al[t] = alphas[b * T + t];
  const int n4 = H / VEC;
  const int R = 64 / n4;
  const int r = lane / n4;
  const int c = (lane - r * n4) * VEC;
  const bool act = r < R;
  float ga[VEC], gs[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) ga[k] = gs[k] = 0.f;
  if (act) {
    ldv<VEC>(ga, g_att + b * H + c);
    if (g_sum) ldv<VEC>(gs, g_sum + b * H + c);
  }
  __syncthreads();
  for (int64_t t0 = 0; t0 < T; t0 += R) {  // uniform trip count
    const int64_t t = t0 + r;
    float p = 0.f;
    if (act && t < T) {
      float fv[VEC];
      ldv<VEC>(fv, f + (b * T + t) * H + c);
#pragma unroll
      for (int k = 0; k < VEC; ++k) p += ga[k] * fv[k];
    }
    pb[lane] = p;
    __syncthreads();
    if (lane < R && t0 + lane < T) {
      float s = 0.f;
      for (int j = 0; j < n4; ++j) s += pb[lane * n4 + j];
      da[t0 + lane] = s;
    }
    __syncthreads();
  }
  float S = 0.f;
  for (int64_t t = lane; t < T; t += 64) S += da[t] * al[t];
  S = wave_sum(S);
  for (int64_t t = lane; t < T; t += 64)
    gscore[b * T + t] = mask[b * T + t] == 1.f ? (da[t] - S) * al[t] : 0.f;
  if (act) {
    for (int64_t t = r; t < T; t += R) {
      const float a = al[t];
      float o[VEC];
#pragma unroll
      for (int k = 0; k < VEC; ++k) o[k] = a * ga[k] + gs[k];
      stv<VEC>(gf + (b * T + t) * H + c, o);
    }
  }
}

// VEC = 4 when H % 4 == 0, H / 4 <= 64 and the operands are 16-B aligned;
// VEC = 1 for H <= 64; else 0 (unsupported).
static int seq_vec(int H, uintptr_t ptrs) {
  if (H % 4 == 0 && H / 4 <= 64 && (ptrs & 15) == 0) return 4;
  if (H <= 64) return 1;
  return 0;
}


// ---------------------------------------------------------------------------
// DIN attention MLP, fused (utils.py:284-289: din_all -> f1_att 80 sigmoid ->
// f2_att 40 sigmoid -> f3_att 1).  With W1 = [A | Bm | C | Dm] over din_all =
// [q, f, q - f, q * f]:
//   a1 = (A + C) q + b1  +  [Bm - C | Dm] [f ; q * f]
// the first term is per SAMPLE (cq, computed once), the second per position
// with the 80 x 2H matrix W1p -- half the multiply-adds of din_all's 4H, and
// din_all [B, T, 4H] is never written.  Only the valid (mask != 0) history
// positions run the MLP: a padded position's score is replaced by the
// padding value before the softmax (utils.py:290-292), so its MLP output and
// gradient are dead (about half of a batch padded to its longest history).
// One lane per position, the weights uniform across the wave (scalar loads);
// activations stored feature-major ([unit][cap]: coalesced) for the
// backward and the weight-gradient GEMMs.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// W1p = [Bm - C | Dm] [n1][2H], W2T = W2^T [n1][n2], cq = (A + C) q + b1 [B][n1]
__global__ void din_mlp_prep_kernel(const float* __restrict__ w1, const float* __restrict__ b1,
                                    const float* __restrict__ w2, const float* __restrict__ q,
                                    int64_t B, int H, int n1, int n2, float* __restrict__ w1p,
                                    float* __restrict__ w2t, float* __restrict__ cq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t np = (int64_t)n1 * 2 * H, nt = (int64_t)n1 * n2;
  if (i < np) {
    const int j = (int)(i / (2 * H)), k = (int)(i % (2 * H));
    const float* r = w1 + (int64_t)j * 4 * H;
    w1p[i] = k < H ? r[H + k] - r[2 * H + k] : r[3 * H + (k - H)];
  } else if (i < np + nt) {
    const int64_t e = i - np;
    const int j = (int)(e / n2), m = (int)(e % n2);
    w2t[e] = w2[(int64_t)m * n1 + j];
  } else if (i < np + nt + B * n1) {
    const int64_t e = i - np - nt;
    const int64_t b = e / n1;
    const int j = (int)(e % n1);
    const float* r = w1 + (int64_t)j * 4 * H;
    const float* qb = q + b * H;
    float acc = b1[j];
    // the loads run ahead of the chain (a rolled loop waited for each pair)
#pragma unroll 12
    for (int k = 0; k < H; ++k) acc = fmaf(r[k] + r[2 * H + k], qb[k], acc);
    cq[e] = acc;
  }
}

// valid positions per sample (one wave per sample): cnt[b]
__global__ void din_mlp_count_kernel(const float* __restrict__ mask, int64_t B, int64_t T,
                                     int32_t* __restrict__ cnt) {
  const int64_t b = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  int c = 0;
  for (int64_t t = lane; t < T; t += 64) c += mask[b * T + t] != 0.f;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane == 0) cnt[b] = c;
}

// off = exclusive scan of cnt (off[B] = P); one block, serial over its
// 1024-sample windows (B is a batch: thousands)
__global__ __launch_bounds__(1024) void din_mlp_scan_kernel(const int32_t* __restrict__ cnt,
                                                             int64_t B, int32_t* __restrict__ off) {
  __shared__ int32_t ws[16];
  __shared__ int32_t carry;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < B; b0 += 1024) {
    const int64_t b = b0 + tid;
    const int v = b < B ? cnt[b] : 0;
    int incl = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) ws[wv] = incl;
    __syncthreads();
    int before = carry;
    for (int w = 0; w < wv; ++w) before += ws[w];
    if (b < B) off[b] = before + incl - v;
    __syncthreads();
    if (tid == 1023) carry = before + incl;
    __syncthreads();
  }
  if (tid == 0) off[B] = carry;
}

// pos[off[b] + r] = b * T + t for the r-th valid position t of sample b
__global__ void din_mlp_pos_kernel(const float* __restrict__ mask, int64_t B, int64_t T,
                                   const int32_t* __restrict__ off, int32_t* __restrict__ pos) {
  const int64_t b = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  int base = off[b];
  for (int64_t t0 = 0; t0 < T; t0 += 64) {
    const int64_t t = t0 + lane;
    const bool v = t < T && mask[b * T + t] != 0.f;
    const uint64_t m = __ballot(v);
    if (v) pos[base + __popcll(m & lanemask_lt())] = (int32_t)(b * T + t);
    base += __popcll(m);
  }
}

// The attention MLP's weights (W1p [N1][2H] then W2^T [N1][N2], 36 KB at H =
// 36) staged in LDS once per block: every lane reads the same word, so the
// reads broadcast.  Read through scalar loads instead, the 35 KB stream
// overflowed the scalar cache and every unit pair waited on an L2 round
// trip (SQ_WAIT_ANY 62 % of the forward's wave cycles, profiles/r05_din_pmc.json).
template <int H, int N1, int N2>
__device__ __forceinline__ void din_stage_weights(float* sw, const float* __restrict__ w1p,
                                                  const float* __restrict__ w2t) {
  constexpr int A = N1 * 2 * H, Bn = N1 * N2;
  for (int i = threadIdx.x; i < (A + Bn) / 4; i += blockDim.x) {
    const int e = 4 * i;
    const float4 v = e < A ? *reinterpret_cast<const float4*>(w1p + e)
                           : *reinterpret_cast<const float4*>(w2t + (e - A));
    *reinterpret_cast<float4*>(sw + e) = v;
  }
  __syncthreads();
}

// forward: one lane per valid position p < P (= off[B]); lanes past P exit
template <int H, int N1, int N2>
__global__ __launch_bounds__(256) void din_mlp_fwd_kernel(
    const int32_t* __restrict__ pos, const int32_t* __restrict__ off, int64_t B, int64_t T,
    int64_t cap, const float* __restrict__ facts, const float* __restrict__ q,
    const float* __restrict__ cq, const float* __restrict__ w1p, const float* __restrict__ w2t,
    const float* __restrict__ b2, const float* __restrict__ w3, const float* __restrict__ b3,
    float* __restrict__ scores, float* __restrict__ h1t, float* __restrict__ h2t) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t P = off[B];
  if ((int64_t)blockIdx.x * blockDim.x >= P) return;   // whole blocks past the count
  static_assert((N1 * 2 * H) % 4 == 0 && N2 % 4 == 0, "16-B weight rows");
  __shared__ __attribute__((aligned(16))) float sw[N1 * 2 * H + N1 * N2];
  din_stage_weights<H, N1, N2>(sw, w1p, w2t);
  const int64_t pc = p < P ? p : P - 1;                 // (clamped: loads stay valid)
  const int64_t bt = pos[pc];
  const int64_t b = bt / T;
  float x[2 * H];
  const float* fr = facts + bt * H;
  const float* qr = q + b * H;
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const float f = fr[k];
    x[k] = f;
    x[H + k] = qr[k] * f;
  }
  float a2[N2];
#pragma unroll
  for (int m = 0; m < N2; ++m) a2[m] = 0.f;
  const float* cqb = cq + b * N1;
  // two hidden units per pass: two independent 72-term chains interleave
  static_assert(N1 % 2 == 0, "unit pairs");
  // the per-sample bias pair one iteration ahead (a load per pair waited
  // for at once was most of the forward's SQ_WAIT_ANY, r05_din_pmc.json)
  float cn0 = cqb[0], cn1 = cqb[1];
  for (int j = 0; j < N1; j += 2) {
    float acc0 = cn0, acc1 = cn1;
    const int jn = j + 2 < N1 ? j + 2 : N1 - 2;
    cn0 = cqb[jn];
    cn1 = cqb[jn + 1];
    const float* wr0 = sw + j * 2 * H;
    const float* wr1 = wr0 + 2 * H;
#pragma unroll
    for (int k = 0; k < 2 * H; ++k) {
      acc0 = fmaf(wr0[k], x[k], acc0);
      acc1 = fmaf(wr1[k], x[k], acc1);
    }
    const float h0 = sigm(acc0), h1 = sigm(acc1);
    if (p < P) {
      h1t[(int64_t)j * cap + p] = h0;
      h1t[(int64_t)(j + 1) * cap + p] = h1;
    }
    const float* vr0 = sw + N1 * 2 * H + j * N2;
    const float* vr1 = vr0 + N2;
#pragma unroll
    for (int m = 0; m < N2; ++m) a2[m] = fmaf(vr1[m], h1, fmaf(vr0[m], h0, a2[m]));
  }
  float s = b3[0];
#pragma unroll
  for (int m = 0; m < N2; ++m) {
    const float h = sigm(a2[m] + b2[m]);
    if (p < P) h2t[(int64_t)m * cap + p] = h;
    s = fmaf(w3[m], h, s);
  }
  if (p < P) scores[bt] = s;
}

// backward: one lane per position p < cap.  p < P: the MLP backward from the
// score gradient; the facts gradient (already holding the pool's) gains
// d f + q * d(q f); per-position buffers for the weight-gradient GEMMs and the
// per-sample sums.  P <= p < cap, when zero_tail: zero columns of every buffer
// the library weight-gradient GEMMs read (they run over cap; the forward wrote
// only p < P) -- 1.25 KB per position the hand pass (bounded by P) skips.
template <int H, int N1, int N2>
__global__ __launch_bounds__(256) void din_mlp_bwd_kernel(
    const int32_t* __restrict__ pos, const int32_t* __restrict__ off, int64_t B, int64_t T,
    int64_t cap, const float* __restrict__ facts, const float* __restrict__ q,
    const float* __restrict__ w1p, const float* __restrict__ w2t, const float* __restrict__ w3,
    const float* __restrict__ gscores, float* __restrict__ h1t,
    float* __restrict__ h2t, float* __restrict__ gfacts, float* __restrict__ da1t,
    float* __restrict__ da2t, float* __restrict__ xt, float* __restrict__ dsc,
    float* __restrict__ dqp, int zero_tail) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t P = off[B];
  __shared__ __attribute__((aligned(16))) float sw[N1 * 2 * H + N1 * N2];
  if ((int64_t)blockIdx.x * blockDim.x < P)   // block-uniform: the block has valid positions
    din_stage_weights<H, N1, N2>(sw, w1p, w2t);
  if (p >= cap) return;
  if (p >= P) {
    if (!zero_tail) return;   // the hand weight-gradient pass stops at P itself
#pragma unroll 8
    for (int j = 0; j < N1; ++j) da1t[(int64_t)j * cap + p] = h1t[(int64_t)j * cap + p] = 0.f;
#pragma unroll 8
    for (int m = 0; m < N2; ++m) da2t[(int64_t)m * cap + p] = h2t[(int64_t)m * cap + p] = 0.f;
#pragma unroll 8
    for (int k = 0; k < 2 * H; ++k) xt[(int64_t)k * cap + p] = 0.f;
    dsc[p] = 0.f;
    return;
  }
  const int64_t bt = pos[p];
  const int64_t b = bt / T;
  const float ds = gscores[bt];
  dsc[p] = ds;
  float da2[N2];
#pragma unroll
  for (int m = 0; m < N2; ++m) {
    const float h = h2t[(int64_t)m * cap + p];
    da2[m] = ds * w3[m] * (1.f - h) * h;
    da2t[(int64_t)m * cap + p] = da2[m];
  }
  float dx[2 * H];
#pragma unroll
  for (int k = 0; k < 2 * H; ++k) dx[k] = 0.f;
  // the h1 activations four units ahead of their use: a load per unit inside
  // the loop was waited for right away, ~80 exposed global-load latencies
  // per position (the kernel took 280-300 us at configs[3])
  static_assert(N1 % 4 == 0, "unit groups of 4");
  float hn[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) hn[q] = h1t[(int64_t)q * cap + p];
  for (int j0 = 0; j0 < N1; j0 += 4) {
    float hc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      hc[q] = hn[q];
      const int jn = j0 + 4 + q < N1 ? j0 + 4 + q : N1 - 1;
      hn[q] = h1t[(int64_t)jn * cap + p];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = j0 + q;
      const float* vr = sw + N1 * 2 * H + j * N2;
      float dh = 0.f;
#pragma unroll
      for (int m = 0; m < N2; ++m) dh = fmaf(vr[m], da2[m], dh);
      const float h = hc[q];
      const float da = dh * (1.f - h) * h;
      da1t[(int64_t)j * cap + p] = da;
      const float* wr = sw + j * 2 * H;
#pragma unroll
      for (int k = 0; k < 2 * H; ++k) dx[k] = fmaf(wr[k], da, dx[k]);
    }
  }
  const float* fr = facts + bt * H;
  const float* qr = q + b * H;
  float* gr = gfacts + bt * H;
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const float f = fr[k], qk = qr[k];
    xt[(int64_t)k * cap + p] = f;
    xt[(int64_t)(H + k) * cap + p] = qk * f;
    gr[k] = gr[k] + (dx[k] + qk * dx[H + k]);
    dqp[(int64_t)k * cap + p] = f * dx[H + k];
  }
}

// per sample b: s1[b] = sum of da1 over its positions, dq2[b] = sum of the
// q-side terms f * d(q f); one wave per sample, lanes over its positions (a
// coalesced 256-B load per unit and 64 positions), each lane's partial over
// the position chunks then a fixed xor-shuffle tree (deterministic).  (The
// per-lane-unit form -- 64 units' rows per load instruction, 64 lines each --
// took 173 us at configs[3].)
template <int H, int N1>
__global__ void din_mlp_sample_kernel(const int32_t* __restrict__ off, int64_t B, int64_t cap,
                                      const float* __restrict__ da1t,
                                      const float* __restrict__ dqp, float* __restrict__ s1,
                                      float* __restrict__ dq2) {
  const int64_t b = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (b >= B) return;   // wave-uniform
  const int64_t p0 = off[b], p1 = off[b + 1];
  constexpr int NU = N1 + H;
  for (int jb = 0; jb < NU; jb += 8) {   // 8 units' loads in flight together
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.f;
    for (int64_t p = p0 + lane; p < p1; p += 64) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int j = jb + q < NU ? jb + q : NU - 1;
        const float* src = j < N1 ? da1t + (int64_t)j * cap : dqp + (int64_t)(j - N1) * cap;
        acc[q] += src[p];
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) acc[q] += __shfl_xor(acc[q], o, 64);
    }
    if (lane < 8 && jb + lane < NU) {
      float v = acc[0];
#pragma unroll
      for (int q = 1; q < 8; ++q) v = lane == q ? acc[q] : v;
      const int j = jb + lane;
      if (j < N1)
        s1[b * N1 + j] = v;
      else
        dq2[b * H + (j - N1)] = v;
    }
  }
}

// The attention MLP's weight gradients in one pass over the per-position
// buffers (dr_din_mlp_wgrad): G = da1 x^T [N1 x H2] (dW1's four blocks are
// formed from it), dW2 = da2 h1^T [N2 x N1], db2 = sum da2, dw3 = h2 dsc,
// db3 = sum dsc -- reductions over the cap positions, which the library did
// as two batched split-K GEMMs, a GEMV and three reductions (≈ 0.25-0.3 ms at
// DIN's cap = 409 600).  Split-K: block b sums positions [b*per, (b+1)*per)
// in chunks of 64 staged through LDS position-major ([p][row]: a thread's 4
// or CW rows at one position are contiguous), fp32 partials per block;
// din_wgrad_reduce_kernel sums them in block order (deterministic).
// Threads 0..20*(H2/CW)-1: a 4 x CW tile of G; threads 0..199: a 4 x 4 tile
// of dW2; threads 200..239: db2 / dw3 of one row; thread 240: db3.
static constexpr int DW_CH = 64;
template <int H2, int CW, int N1, int N2>
__global__ __launch_bounds__(256) void din_wgrad_kernel(
    const float* __restrict__ da1t, const float* __restrict__ xt, const float* __restrict__ da2t,
    const float* __restrict__ h1t, const float* __restrict__ h2t, const float* __restrict__ dsc,
    int64_t cap, int64_t per, const int32_t* __restrict__ valid, float* __restrict__ part) {
  static_assert(N1 == 80 && N2 == 40 && H2 % CW == 0 && 20 * (H2 / CW) <= 256, "tile shape");
  constexpr int GOUT = N1 * H2, WOUT = N2 * N1, OUT = GOUT + WOUT + 2 * N2 + 1;
  constexpr int RA = N1, RX = H2, RD = N2, RH = N1, RG = N2;     // rows per position
  constexpr int OA = 0, OX = OA + RA, OD = OX + RX, OH = OD + RD, OG = OH + RH, OS = OG + RG;
  constexpr int ROW = (OS + 1 + 3) / 4 * 4;                       // floats per staged position (16-B rows)
  __shared__ __attribute__((aligned(16))) float st[DW_CH * ROW];
  const int tid = threadIdx.x;
  // positions [0, lim): cap, or the valid count P read on the device (the
  // blocks then split P in whole chunks; no host read, capturable)
  int64_t lim = cap;
  if (valid) {
    lim = *valid;
    per = ((lim + gridDim.x - 1) / gridDim.x + DW_CH - 1) / DW_CH * DW_CH;
  }
  const int64_t p0 = (int64_t)blockIdx.x * per;
  const int64_t p1 = p0 + per < lim ? p0 + per : lim;
  constexpr int NG = 20 * (H2 / CW);
  const bool tg = tid < NG;
  const int gi = (tid / (H2 / CW)) * 4, gj = (tid % (H2 / CW)) * CW;
  const bool tw = tid < 200;
  const int wi = (tid / 20) * 4, wj = (tid % 20) * 4;
  const bool tb = tid >= 200 && tid < 200 + N2;
  const int bk = tid - 200;
  float g[4][CW], w[4][4], db2 = 0.f, dw3 = 0.f, db3 = 0.f;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
#pragma unroll
    for (int c = 0; c < CW; ++c) g[a][c] = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) w[a][c] = 0.f;
  }
  for (int64_t c0 = p0; c0 < p1; c0 += DW_CH) {
    const int nc = (int)(p1 - c0 < DW_CH ? p1 - c0 : DW_CH);
    // stage: row r of matrix M, positions c0 .. c0 + 63 as 16-B vectors
    // (coalesced along p), into st[p][offset + r]; positions past nc are
    // zero.  Four vector loads in flight per thread, from clamped (always
    // valid) addresses, so none is branched around (rows are 16-B aligned:
    // cap % 4 == 0, c0 % 64 == 0)
    auto stage_mat = [&](const float* __restrict__ M, int R, int off) {
      const int nv = R * (DW_CH / 4);
      for (int e0 = 0; e0 < nv; e0 += 256 * 4) {
        float4 v[4];
        int ee[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          int e = e0 + u * 256 + tid;
          ee[u] = e;
          e = e < nv ? e : nv - 1;
          const int r = e / (DW_CH / 4), p4 = (e % (DW_CH / 4)) * 4;
          const int pc = p4 < nc ? p4 : 0;
          v[u] = *reinterpret_cast<const float4*>(M + (int64_t)r * cap + c0 + pc);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = ee[u];
          if (e < nv) {
            const int r = e / (DW_CH / 4), p4 = (e % (DW_CH / 4)) * 4;
            float* d = st + p4 * ROW + off + r;
            d[0] = p4 < nc ? v[u].x : 0.f;
            d[ROW] = p4 + 1 < nc ? v[u].y : 0.f;
            d[2 * ROW] = p4 + 2 < nc ? v[u].z : 0.f;
            d[3 * ROW] = p4 + 3 < nc ? v[u].w : 0.f;
          }
        }
      }
    };
    stage_mat(da1t, RA, OA);
    stage_mat(xt, RX, OX);
    stage_mat(da2t, RD, OD);
    stage_mat(h1t, RH, OH);
    stage_mat(h2t, RG, OG);
    if (tid < DW_CH) st[tid * ROW + OS] = tid < nc ? dsc[c0 + tid] : 0.f;
    __syncthreads();
    for (int p = 0; p < nc; ++p) {
      const float* sp = st + p * ROW;
      if (tg) {
        float a[4], x[CW];
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] = sp[OA + gi + k];
#pragma unroll
        for (int k = 0; k < CW; ++k) x[k] = sp[OX + gj + k];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int c = 0; c < CW; ++c) g[k][c] = fmaf(a[k], x[c], g[k][c]);
      }
      if (tw) {
        float a[4], h[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] = sp[OD + wi + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) h[k] = sp[OH + wj + k];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int c = 0; c < 4; ++c) w[k][c] = fmaf(a[k], h[c], w[k][c]);
      } else if (tb) {
        db2 += sp[OD + bk];
        dw3 = fmaf(sp[OG + bk], sp[OS], dw3);
      } else if (tid == 240) {
        db3 += sp[OS];
      }
    }
    __syncthreads();   // the stage is rewritten next
  }
  float* pb = part + (int64_t)blockIdx.x * OUT;
  if (tg)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int c = 0; c < CW; ++c) pb[(gi + k) * H2 + gj + c] = g[k][c];
  if (tw)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int c = 0; c < 4; ++c) pb[GOUT + (wi + k) * N1 + wj + c] = w[k][c];
  if (tb) {
    pb[GOUT + WOUT + bk] = db2;
    pb[GOUT + WOUT + N2 + bk] = dw3;
  }
  if (tid == 240) pb[GOUT + WOUT + 2 * N2] = db3;
}

__global__ __launch_bounds__(1024) void din_wgrad_reduce_kernel(const float* __restrict__ part,
                                                                int nb, int out_n,
                                                                float* __restrict__ out) {
  // 64 outputs per block; wave w of 16 sums blocks [w*q, (w+1)*q) in order,
  // then the sixteen wave sums are added in wave order (deterministic)
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int o = blockIdx.x * 64 + lane;
  const int q = (nb + 15) / 16;
  const int b0 = w * q, b1 = b0 + q < nb ? b0 + q : nb;
  float a = 0.f;
  if (o < out_n)
#pragma unroll 8
    for (int b = b0; b < b1; ++b) a += part[(int64_t)b * out_n + o];
  red[w][lane] = a;
  __syncthreads();
  if (w == 0 && o < out_n) {
    float t = red[0][lane];
#pragma unroll
    for (int k = 1; k < 16; ++k) t += red[k][lane];
    out[o] = t;
  }
}

// The same reductions on the matrix cores (the default of DR_DIN_WGRAD=hand;
// DR_DIN_WGRAD_VALU=1 the kernel above): every output is a 16 x 16 tile of
// v_mfma_f32_16x16x4f32 over K = 4 positions at a time -- G (5 x NT tiles,
// columns past H2 discarded), dW2 (3 x 5, rows past N2 discarded) and 5
// tiles whose B operand is [dsc, 1, 0, ...] over the rows [da2 ; h2]
// (column 1 of the da2 rows = db2, column 0 of the h2 rows = dw3); db3 by
// wave 0's lanes.  Tiles dealt round-robin to the 4 waves; fragments read
// from the same position-major LDS stage (lane l: row l % 16 of the tile at
// position p + l / 16).
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <int H2, int N1, int N2, int CH>
__global__ __launch_bounds__(256, 3) void din_wgrad_mfma_kernel(
    const float* __restrict__ da1t, const float* __restrict__ xt, const float* __restrict__ da2t,
    const float* __restrict__ h1t, const float* __restrict__ h2t, const float* __restrict__ dsc,
    int64_t cap, int64_t per, const int32_t* __restrict__ valid, float* __restrict__ part) {
  static_assert(N1 == 80 && N2 == 40, "tile shape");
  constexpr int NT = (H2 + 15) / 16;
  constexpr int GT = 5 * NT, WT = 15, XT = 5, TT = GT + WT + XT;
  constexpr int TPW = (TT + 3) / 4;                                // tiles per wave
  constexpr int GOUT = N1 * H2, WOUT = N2 * N1, OUT = GOUT + WOUT + 2 * N2 + 1;
  constexpr int RA = N1, RX = H2, RD = N2, RH = N1, RG = N2;
  constexpr int OA = 0, OX = OA + RA, OD = OX + RX, OH = OD + RD, OG = OH + RH, OS = OG + RG;
  // floats per staged position: ROW = 17 (mod 64), so the stage's transposing
  // stores (16 positions 4 apart x 4 rows per wave) hit 64 distinct banks and
  // the fragment reads (4 positions x 16 rows) overlap in at most 3 banks
  constexpr int ROW = OS + 1 + ((17 - (OS + 1) % 64) % 64 + 64) % 64;
  static_assert(OX + 16 * NT <= ROW && OD + 48 <= ROW, "padded fragment reads stay in the row");
  __shared__ __attribute__((aligned(16))) float st[CH * ROW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // positions [0, lim): cap, or the valid count P read on the device (the
  // blocks then split P in whole chunks; no host read, capturable)
  int64_t lim = cap;
  if (valid) {
    lim = *valid;
    per = ((lim + gridDim.x - 1) / gridDim.x + CH - 1) / CH * CH;
  }
  const int64_t p0 = (int64_t)blockIdx.x * per;
  const int64_t p1 = p0 + per < lim ? p0 + per : lim;
  const int li = lane & 15, lk = lane >> 4;
  f32x4v acc[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = f32x4v{0.f, 0.f, 0.f, 0.f};
  float db3 = 0.f;
  for (int64_t c0 = p0; c0 < p1; c0 += CH) {
    const int nc = (int)(p1 - c0 < CH ? p1 - c0 : CH);
    // stage: the six operands as one list of rows (da1, x, da2, h1, h2, dsc:
    // row q lands at st[p][q], the LDS offsets OA.. OS follow the same
    // order), positions c0 .. c0 + CH - 1 as 16-B vectors coalesced along p;
    // positions past nc are zero.  SU vector loads in flight per thread, from
    // clamped (always valid) addresses, so none is branched around (rows are
    // 16-B aligned: cap % 4 == 0, c0 % 4 == 0) -- two round trips to HBM per
    // 64-position chunk, not one per operand and 1024 vectors
    {
      constexpr int NQ = OS + 1, NV = NQ * (CH / 4), SU = CH == 32 ? 10 : 8;
      for (int e0 = 0; e0 < NV; e0 += 256 * SU) {
        float4 v[SU];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          int e = e0 + u * 256 + tid;
          e = e < NV ? e : NV - 1;
          const int q = e / (CH / 4), p4 = (e % (CH / 4)) * 4;
          const int pc = p4 < nc ? p4 : 0;
          const float* M = q < OX ? da1t + (int64_t)q * cap
                         : q < OD ? xt + (int64_t)(q - OX) * cap
                         : q < OH ? da2t + (int64_t)(q - OD) * cap
                         : q < OG ? h1t + (int64_t)(q - OH) * cap
                         : q < OS ? h2t + (int64_t)(q - OG) * cap
                                  : dsc;
          v[u] = *reinterpret_cast<const float4*>(M + c0 + pc);
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int e = e0 + u * 256 + tid;
          if (e < NV) {
            const int q = e / (CH / 4), p4 = (e % (CH / 4)) * 4;
            float* d = st + p4 * ROW + q;
            d[0] = p4 < nc ? v[u].x : 0.f;
            d[ROW] = p4 + 1 < nc ? v[u].y : 0.f;
            d[2 * ROW] = p4 + 2 < nc ? v[u].z : 0.f;
            d[3 * ROW] = p4 + 3 < nc ? v[u].w : 0.f;
          }
        }
      }
    }
    __syncthreads();
    if (wave == 0 && lane < CH) db3 += st[lane * ROW + OS];   // (zero past nc)
    // the wave's tiles as compile-time indices (one instantiation per wave),
    // so the fragment reads of all its tiles are issued together and shared
    // reads are merged, rather than a branch and a read-wait before each MFMA
    auto mma = [&](auto w_) {
      constexpr int W = decltype(w_)::value;
#pragma unroll 2
      for (int p = 0; p < CH; p += 4) {        // zero-padded past nc: a full chunk
        const float* sp = st + (p + lk) * ROW;
        const float ds = sp[OS];
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          const int t = W + 4 * j;
          if (t >= TT) break;
          float a, b;
          if (t < GT) {
            a = sp[OA + (t / NT) * 16 + li];
            b = sp[OX + (t % NT) * 16 + li];
          } else if (t < GT + WT) {
            const int q = t - GT;
            a = sp[OD + (q / 5) * 16 + li];
            b = sp[OH + (q % 5) * 16 + li];
          } else {
            const int r = (t - GT - WT) * 16 + li;    // virtual rows [da2 ; h2]
            a = r < N2 ? sp[OD + r] : sp[OG + (r - N2)];
            b = li == 0 ? ds : (li == 1 ? 1.f : 0.f);
          }
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
        }
      }
    };
    if (wave == 0) mma(std::integral_constant<int, 0>{});
    else if (wave == 1) mma(std::integral_constant<int, 1>{});
    else if (wave == 2) mma(std::integral_constant<int, 2>{});
    else mma(std::integral_constant<int, 3>{});
    __syncthreads();   // the stage is rewritten next
  }
  float* pb = part + (int64_t)blockIdx.x * OUT;
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + 4 * j;
    if (t >= TT) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * lk + r, col = li;      // C/D map: rows 4 (l / 16) + r, column l % 16
      const float v = acc[j][r];
      if (t < GT) {
        const int gi = (t / NT) * 16 + row, gj = (t % NT) * 16 + col;
        if (gj < H2) pb[gi * H2 + gj] = v;
      } else if (t < GT + WT) {
        const int q = t - GT;
        const int wi = (q / 5) * 16 + row, wj = (q % 5) * 16 + col;
        if (wi < N2) pb[GOUT + wi * N1 + wj] = v;
      } else {
        const int vr = (t - GT - WT) * 16 + row;
        if (vr < N2 && col == 1) pb[GOUT + WOUT + vr] = v;                 // db2
        if (vr >= N2 && vr < 2 * N2 && col == 0) pb[GOUT + WOUT + vr] = v;  // dw3 (N2 + k)
      }
    }
  }
  if (wave == 0) {
    for (int o = 32; o > 0; o >>= 1) db3 += __shfl_down(db3, o, 64);
    if (lane == 0) pb[GOUT + WOUT + 2 * N2] = db3;
  }
}

static constexpr int kWgradBlocks = 1024;

// ---- Dice (modelzoo/DIN/script/utils.py:12-35, batch statistics) ----------
// One block per 4 columns, 256 row groups (1024 threads; 50 blocks for a
// 200-wide layer -- with 16 columns per block the 13 blocks' dependent load
// chains set the time): each thread sums its rows rg, rg + 256, ... (loops
// unrolled 8 deep), then a fixed LDS tree over the row groups -- a column's
// statistics do not depend on timing.
static constexpr int kDiceCols = 4, kDiceRg = 256;

__device__ __forceinline__ float dice_col_sum(float v, float (*red)[kDiceCols], int rg, int cl) {
  red[rg][cl] = v;
  __syncthreads();
#pragma unroll
  for (int st = kDiceRg / 2; st > 0; st >>= 1) {
    if (rg < st) red[rg][cl] += red[rg + st][cl];
    __syncthreads();
  }
  const float t = red[0][cl];
  __syncthreads();
  return t;
}

// y = alpha (1 - p) x + p x, p = sigmoid((x - mean) / (std + eps)), mean and
// std = sqrt(mean((x - mean)^2 + eps)) over the batch; stats [2, n] = mean,
// std for the backward.
__global__ __launch_bounds__(1024) void dice_fwd_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ alpha, int64_t B,
                                                       int n, float eps, float* __restrict__ y,
                                                       float* __restrict__ stats) {
  __shared__ float red[kDiceRg][kDiceCols];
  const int cl = threadIdx.x % kDiceCols, rg = threadIdx.x / kDiceCols;
  const int col = blockIdx.x * kDiceCols + cl;
  const bool ok = col < n;
  const float inv = 1.f / (float)B;
  float s = 0.f;
  if (ok)
#pragma unroll 8
    for (int i = rg; i < (int)B; i += kDiceRg) s += x[(int64_t)i * n + col];
  const float mean = dice_col_sum(s, red, rg, cl) * inv;
  float v = 0.f;
  if (ok)
#pragma unroll 8
    for (int i = rg; i < (int)B; i += kDiceRg) {
      const float c = x[(int64_t)i * n + col] - mean;
      v += c * c + eps;
    }
  const float sd = sqrtf(dice_col_sum(v, red, rg, cl) * inv);
  if (!ok) return;
  const float a = alpha[col], den = sd + eps;
#pragma unroll 8
  for (int i = rg; i < (int)B; i += kDiceRg) {
    const float xv = x[(int64_t)i * n + col];
    const float p = 1.f / (1.f + expf(-((xv - mean) / den)));
    y[(int64_t)i * n + col] = a * (1.f - p) * xv + p * xv;
  }
  if (rg == 0) {
    stats[col] = mean;
    stats[n + col] = sd;
  }
}

// Its backward: with c = x - mean, s = std + eps, p = sigmoid(c / s),
// gz = gy (1 - alpha) x p (1 - p), g_std = -sum(gz c) / s^2, g_var =
// g_std / (2 std), gc = gz / s + g_var 2 c / B:  gx = gy (alpha + (1 - alpha)
// p) + gc - mean(gc);  g_alpha = sum gy (1 - p) x.
__global__ __launch_bounds__(1024) void dice_bwd_kernel(
    const float* __restrict__ x, const float* __restrict__ gy, const float* __restrict__ alpha,
    const float* __restrict__ stats, int64_t B, int n, float eps, float* __restrict__ gx,
    float* __restrict__ galpha) {
  __shared__ float red[kDiceRg][kDiceCols];
  const int cl = threadIdx.x % kDiceCols, rg = threadIdx.x / kDiceCols;
  const int col = blockIdx.x * kDiceCols + cl;
  const bool ok = col < n;
  const float inv = 1.f / (float)B;
  const float mean = ok ? stats[col] : 0.f, sd = ok ? stats[n + col] : 1.f;
  const float a = ok ? alpha[col] : 0.f, den = sd + eps;
  float sgc = 0.f, sga = 0.f;
  if (ok)
#pragma unroll 8
    for (int i = rg; i < (int)B; i += kDiceRg) {
      const float xv = x[(int64_t)i * n + col], g = gy[(int64_t)i * n + col];
      const float c = xv - mean;
      const float p = 1.f / (1.f + expf(-(c / den)));
      const float gz = g * (1.f - a) * xv * (p * (1.f - p));
      sgc += gz * c;
      sga += g * (1.f - p) * xv;
    }
  const float gs = -dice_col_sum(sgc, red, rg, cl) / (den * den);
  const float ga = dice_col_sum(sga, red, rg, cl);
  const float gv2 = gs / (2.f * sd) * 2.f * inv;   // g_var * 2 / B
  float sc = 0.f;
  if (ok)
#pragma unroll 8
    for (int i = rg; i < (int)B; i += kDiceRg) {
      const float xv = x[(int64_t)i * n + col], g = gy[(int64_t)i * n + col];
      const float c = xv - mean;
      const float p = 1.f / (1.f + expf(-(c / den)));
      const float gz = g * (1.f - a) * xv * (p * (1.f - p));
      sc += gz / den + gv2 * c;
    }
  const float mgc = dice_col_sum(sc, red, rg, cl) * inv;
  if (!ok) return;
#pragma unroll 8
  for (int i = rg; i < (int)B; i += kDiceRg) {
    const float xv = x[(int64_t)i * n + col], g = gy[(int64_t)i * n + col];
    const float c = xv - mean;
    const float p = 1.f / (1.f + expf(-(c / den)));
    const float gz = g * (1.f - a) * xv * (p * (1.f - p));
    // (the centring first: gc and its mean can be far larger than the
    // direct term when std is tiny, e.g. a batch of one)
    gx[(int64_t)i * n + col] = g * (a + (1.f - a) * p) + ((gz / den + gv2 * c) - mgc);
  }
  if (rg == 0) galpha[col] = ga;
}


// ---- the fcn input of Model_DIN (model.py:118-124) -----------------------
// inp = [uid, item, his_sum, item * his_sum, att] ([B, Du + 4H]), then the
// inference-form batch_normalization bn = (inp * c) * gamma + beta (c =
// 1 / sqrt(1 + 1e-3)): one elementwise pass instead of a concat and three
// broadcast ops.
__device__ __forceinline__ float fcn_in(const float* uid, const float* item, const float* hs,
                                        const float* att, int64_t b, int j, int Du, int H) {
  if (j < Du) return uid[b * Du + j];
  const int k = j - Du, piece = k / H, h = k - piece * H;
  const int64_t o = b * H + h;
  switch (piece) {
    case 0: return item[o];
    case 1: return hs[o];
    case 2: return item[o] * hs[o];
    default: return att[o];
  }
}

__global__ __launch_bounds__(256) void fcn_input_fwd_kernel(
    const float* __restrict__ uid, const float* __restrict__ item, const float* __restrict__ hs,
    const float* __restrict__ att, const float* __restrict__ gamma, const float* __restrict__ beta,
    int64_t B, int Du, int H, float c, float* __restrict__ out) {
  const int n = Du + 4 * H;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * n) return;
  const int64_t b = e / n;
  const int j = (int)(e - b * n);
  const float v = fcn_in(uid, item, hs, att, b, j, Du, H);
  out[e] = (v * c) * gamma[j] + beta[j];
}

// Its backward, per (sample, column of a piece): gi = (g gamma) c for each
// inp column; g_uid = gi_uid, g_item = gi_item + gi_prod his_sum, g_his_sum
// = gi_hs + gi_prod item, g_att = gi_att.
__global__ __launch_bounds__(256) void fcn_input_bwd_kernel(
    const float* __restrict__ g, const float* __restrict__ item, const float* __restrict__ hs,
    const float* __restrict__ gamma, int64_t B, int Du, int H, float c, float* __restrict__ g_uid,
    float* __restrict__ g_item, float* __restrict__ g_hs, float* __restrict__ g_att) {
  const int n = Du + 4 * H, w = Du + H;   // per sample: Du uid columns, H (item, hs, prod, att)
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * w) return;
  const int64_t b = e / w;
  const int j = (int)(e - b * w);
  const float* gr = g + b * n;
  if (j < Du) {
    g_uid[b * Du + j] = (gr[j] * gamma[j]) * c;
    return;
  }
  const int h = j - Du;
  const int ji = Du + h, jh = Du + H + h, jp = Du + 2 * H + h, ja = Du + 3 * H + h;
  const float gi = (gr[ji] * gamma[ji]) * c, gh = (gr[jh] * gamma[jh]) * c;
  const float gp = (gr[jp] * gamma[jp]) * c, ga = (gr[ja] * gamma[ja]) * c;
  const int64_t o = b * H + h;
  g_item[o] = gi + gp * hs[o];
  g_hs[o] = gh + gp * item[o];
  g_att[o] = ga;
}

// g_gamma[j] = sum_b g (inp c), g_beta[j] = sum_b g: one block per 16
// columns, fixed-order sums (dice_col_sum).
__global__ __launch_bounds__(1024) void fcn_input_param_grad_kernel(
    const float* __restrict__ g, const float* __restrict__ uid, const float* __restrict__ item,
    const float* __restrict__ hs, const float* __restrict__ att, int64_t B, int Du, int H, float c,
    float* __restrict__ g_gamma, float* __restrict__ g_beta) {
  __shared__ float red[kDiceRg][kDiceCols];
  const int n = Du + 4 * H;
  const int cl = threadIdx.x % kDiceCols, rg = threadIdx.x / kDiceCols;
  const int col = blockIdx.x * kDiceCols + cl;
  const bool ok = col < n;
  float sg = 0.f, sb = 0.f;
  if (ok)
#pragma unroll 8
    for (int i = rg; i < (int)B; i += kDiceRg) {
      const float gv = g[(int64_t)i * n + col];
      sg += gv * (fcn_in(uid, item, hs, att, i, col, Du, H) * c);
      sb += gv;
    }
  const float tg = dice_col_sum(sg, red, rg, cl);
  const float tb = dice_col_sum(sb, red, rg, cl);
  if (ok && rg == 0) {
    g_gamma[col] = tg;
    g_beta[col] = tb;
  }
}
}  // namespace dr

extern "C" {

int dr_din_attention_input(const float* query, const float* facts, int64_t batch, int64_t seq_len,
                           int hidden, float* out, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && seq_len >= 0 && hidden > 0, DR_INVALID_ARGUMENT, "bad shape");
  if (batch * seq_len == 0) return DR_OK;
  DR_REQUIRE(query && facts && out, DR_INVALID_ARGUMENT, "null operand");
  const int vec = seq_vec(hidden, (uintptr_t)query | (uintptr_t)facts | (uintptr_t)out);
  DR_REQUIRE(vec > 0, DR_INVALID_ARGUMENT,
             "dr_din_attention_input: hidden must be <= 64, or a multiple of 4 <= 256");
  const int64_t n = batch * seq_len * (hidden / vec);
  if (n == 0) return DR_OK;
  const unsigned blocks = (unsigned)ceil_div(n, 256);
  if (vec == 4)
    hipLaunchKernelGGL(din_input_kernel<4>, dim3(blocks), dim3(256), 0, S(stream), query, facts,
                       batch, seq_len, hidden, out);
  else
    hipLaunchKernelGGL(din_input_kernel<1>, dim3(blocks), dim3(256), 0, S(stream), query, facts,
                       batch, seq_len, hidden, out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_din_attention_input_grad(const float* query, const float* facts, const float* top_grad,
                                int64_t batch, int64_t seq_len, int hidden, float* grad_query,
                                float* grad_facts, int accumulate, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && seq_len >= 0 && hidden > 0, DR_INVALID_ARGUMENT, "bad shape");
  DR_REQUIRE(batch < (1ll << 31), DR_INVALID_ARGUMENT, "batch must be < 2^31");
  if (batch == 0) return DR_OK;
  DR_REQUIRE(query && facts && top_grad && grad_query && grad_facts, DR_INVALID_ARGUMENT,
             "null operand");
  const int vec = seq_vec(hidden, (uintptr_t)query | (uintptr_t)facts | (uintptr_t)top_grad |
                                      (uintptr_t)grad_facts);
  DR_REQUIRE(vec > 0, DR_INVALID_ARGUMENT,
             "dr_din_attention_input_grad: hidden must be <= 64, or a multiple of 4 <= 256");
  if (vec == 4)
    hipLaunchKernelGGL(din_input_grad_kernel<4>, dim3((unsigned)batch), dim3(64), 0, S(stream),
                       query, facts, top_grad, seq_len, hidden, grad_query, grad_facts,
                       accumulate);
  else
    hipLaunchKernelGGL(din_input_grad_kernel<1>, dim3((unsigned)batch), dim3(64), 0, S(stream),
                       query, facts, top_grad, seq_len, hidden, grad_query, grad_facts,
                       accumulate);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_din_attention_pool(const float* scores, const float* mask, const float* facts,
                          int64_t batch, int64_t seq_len, int hidden, float* att_out,
                          float* sum_out, float* alphas, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && seq_len >= 1 && hidden > 0, DR_INVALID_ARGUMENT,
             "bad shape (seq_len must be >= 1)");
  DR_REQUIRE(batch < (1ll << 31) && seq_len <= 8192, DR_INVALID_ARGUMENT,
             "batch must be < 2^31 and seq_len <= 8192");
  if (batch == 0) return DR_OK;
  DR_REQUIRE(scores && mask && facts && att_out && alphas, DR_INVALID_ARGUMENT, "null operand");
  const int vec = seq_vec(hidden, (uintptr_t)facts);
  DR_REQUIRE(vec > 0, DR_INVALID_ARGUMENT,
             "dr_din_attention_pool: hidden must be <= 64, or a multiple of 4 <= 256");
  const size_t lds = (size_t)(((seq_len + 3) & ~3ll) + 2 * 64 * vec) * sizeof(float);
  if (vec == 4)
    hipLaunchKernelGGL(din_pool_kernel<4>, dim3((unsigned)batch), dim3(64), lds, S(stream),
                       scores, mask, facts, seq_len, hidden, att_out, sum_out, alphas);
  else
    hipLaunchKernelGGL(din_pool_kernel<1>, dim3((unsigned)batch), dim3(64), lds, S(stream),
                       scores, mask, facts, seq_len, hidden, att_out, sum_out, alphas);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_din_attention_pool_grad(const float* alphas, const float* mask, const float* facts,
                               const float* grad_att, const float* grad_sum, int64_t batch,
                               int64_t seq_len, int hidden, float* grad_scores,
                               float* grad_facts, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && seq_len >= 1 && hidden > 0, DR_INVALID_ARGUMENT,
             "bad shape (seq_len must be >= 1)");
  DR_REQUIRE(batch < (1ll << 31) && seq_len <= 8192, DR_INVALID_ARGUMENT,
             "batch must be < 2^31 and seq_len <= 8192");
  if (batch == 0) return DR_OK;
  DR_REQUIRE(alphas && mask && facts && grad_att && grad_scores && grad_facts,
             DR_INVALID_ARGUMENT, "null operand");
  const int vec = seq_vec(hidden, (uintptr_t)facts | (uintptr_t)grad_att | (uintptr_t)grad_sum |
                                      (uintptr_t)grad_facts);
  DR_REQUIRE(vec > 0, DR_INVALID_ARGUMENT,
             "dr_din_attention_pool_grad: hidden must be <= 64, or a multiple of 4 <= 256");
  const size_t lds = (size_t)(2 * ((seq_len + 3) & ~3ll) + 64) * sizeof(float);
  if (vec == 4)
    hipLaunchKernelGGL(din_pool_grad_kernel<4>, dim3((unsigned)batch), dim3(64), lds, S(stream),
                       alphas, mask, facts, grad_att, grad_sum, seq_len, hidden, grad_scores,
                       grad_facts);
  else
    hipLaunchKernelGGL(din_pool_grad_kernel<1>, dim3((unsigned)batch), dim3(64), lds, S(stream),
                       alphas, mask, facts, grad_att, grad_sum, seq_len, hidden, grad_scores,
                       grad_facts);
  DR_LAUNCH_CHECK();
  return DR_OK;
}


// ---- fused DIN attention MLP -------------------------------------------------
#define DR_DIN_MLP_SHAPES(X) X(16) X(32) X(36) X(64)

int dr_din_mlp_forward(const float* query, const float* facts, const float* mask, int64_t batch,
                       int64_t seq_len, int hidden, const float* w1, const float* b1, int n1,
                       const float* w2, const float* b2, int n2, const float* w3, const float* b3,
                       float* scores, const dr_din_mlp_buf* buf, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && seq_len >= 1 && hidden > 0 && buf, DR_INVALID_ARGUMENT, "bad shape");
  DR_REQUIRE(n1 == 80 && n2 == 40, DR_INVALID_ARGUMENT,
             "dr_din_mlp_forward: the reference's 80 / 40 attention units");
  DR_REQUIRE(hidden == 16 || hidden == 32 || hidden == 36 || hidden == 64, DR_INVALID_ARGUMENT,
             "dr_din_mlp_forward: hidden %d not built (16, 32, 36, 64)", hidden);
  DR_REQUIRE(batch * seq_len < (1ll << 31), DR_INVALID_ARGUMENT, "batch * seq_len must be < 2^31");
  if (batch == 0) return DR_OK;
  DR_REQUIRE(query && facts && mask && w1 && b1 && w2 && b2 && w3 && b3 && scores && buf->pos &&
                 buf->off && buf->cnt && buf->w1p && buf->w2t && buf->cq && buf->h1t && buf->h2t,
             DR_INVALID_ARGUMENT, "null operand");
  hipStream_t st = S(stream);
  const int64_t cap = batch * seq_len;
  const int64_t prep = (int64_t)n1 * 2 * hidden + (int64_t)n1 * n2 + batch * n1;
  hipLaunchKernelGGL(din_mlp_prep_kernel, dim3((unsigned)ceil_div(prep, 256)), dim3(256), 0, st,
                     w1, b1, w2, query, batch, hidden, n1, n2, buf->w1p, buf->w2t, buf->cq);
  const unsigned sb = (unsigned)ceil_div(batch, 4);
  hipLaunchKernelGGL(din_mlp_count_kernel, dim3(sb), dim3(256), 0, st, mask, batch, seq_len,
                     buf->cnt);
  hipLaunchKernelGGL(din_mlp_scan_kernel, dim3(1), dim3(1024), 0, st, buf->cnt, batch, buf->off);
  hipLaunchKernelGGL(din_mlp_pos_kernel, dim3(sb), dim3(256), 0, st, mask, batch, seq_len,
                     buf->off, buf->pos);
  const unsigned pb = (unsigned)ceil_div(cap, 256);
#define DR_FWD(HH)                                                                            \
  if (hidden == HH)                                                                           \
    hipLaunchKernelGGL((din_mlp_fwd_kernel<HH, 80, 40>), dim3(pb), dim3(256), 0, st, buf->pos, \
                       buf->off, batch, seq_len, cap, facts, query, buf->cq, buf->w1p,        \
                       buf->w2t, b2, w3, b3, scores, buf->h1t, buf->h2t);
  DR_DIN_MLP_SHAPES(DR_FWD)
#undef DR_FWD
  DR_LAUNCH_CHECK();
  return DR_OK;
}

size_t dr_din_mlp_wgrad_workspace_size(int n1, int hidden2, int n2) {
  return (size_t)dr::kWgradBlocks * (size_t)(n1 * hidden2 + n2 * n1 + 2 * n2 + 1) * sizeof(float) +
         256;
}

int dr_din_mlp_wgrad(const float* da1t, const float* xt, const float* da2t, const float* h1t,
                     const float* h2t, const float* dsc, int64_t cap, int n1, int hidden2, int n2,
                     float* out, void* ws, size_t ws_bytes, void* stream) {
  return dr_din_mlp_wgrad_valid(da1t, xt, da2t, h1t, h2t, dsc, cap, nullptr, n1, hidden2, n2, out,
                                ws, ws_bytes, stream);
}

int dr_din_mlp_wgrad_valid(const float* da1t, const float* xt, const float* da2t,
                           const float* h1t, const float* h2t, const float* dsc, int64_t cap,
                           const int32_t* valid, int n1, int hidden2, int n2, float* out, void* ws,
                           size_t ws_bytes, void* stream) {
  using namespace dr;
  // the matrix-core form unless DR_DIN_WGRAD_VALU=1 (read per call)
  const char* ve = getenv("DR_DIN_WGRAD_VALU");
  const bool mfma = !(ve && atoi(ve) != 0);
  // positions staged per chunk by the matrix-core form: 32 (three blocks per
  // CU, so one block's loads overlap the others' MFMAs) or 64 (24: 0.184 ms
  // against 32's 0.160, profiles/r05_din_wgrad.log)
  const char* ce = getenv("DR_DIN_WGRAD_CH");
  const int ch = ce && atoi(ce) == 64 ? 64 : 32;
  DR_REQUIRE(cap >= 1 && n1 == 80 && n2 == 40 &&
                 (hidden2 == 32 || hidden2 == 64 || hidden2 == 72 || hidden2 == 128),
             DR_INVALID_ARGUMENT, "dr_din_mlp_wgrad: n1 = 80, n2 = 40, 2H in {32, 64, 72, 128}");
  DR_REQUIRE(da1t && xt && da2t && h1t && h2t && dsc && out && ws, DR_INVALID_ARGUMENT,
             "null operand");
  DR_REQUIRE(ws_bytes >= dr_din_mlp_wgrad_workspace_size(n1, hidden2, n2), DR_INVALID_ARGUMENT,
             "workspace too small");
  DR_REQUIRE(cap % 4 == 0 && ((uintptr_t)da1t | (uintptr_t)xt | (uintptr_t)da2t | (uintptr_t)h1t |
                              (uintptr_t)h2t) % 16 == 0,
             DR_INVALID_ARGUMENT, "dr_din_mlp_wgrad: cap % 4 == 0 and 16-B aligned buffers");
  const int out_n = n1 * hidden2 + n2 * n1 + 2 * n2 + 1;
  // split-K blocks: kWgradBlocks (1024, the workspace's size) for the VALU
  // form; the matrix-core form runs 3 blocks per CU (DR_DIN_WGRAD_BLOCKS)
  const char* be = getenv("DR_DIN_WGRAD_BLOCKS");
  int nbk = mfma ? 768 : 512;
  if (be && atoi(be) > 0) nbk = atoi(be) < kWgradBlocks ? atoi(be) : kWgradBlocks;
  int64_t per = (cap + nbk - 1) / nbk;
  const int pr = mfma ? ch : DW_CH;   // whole chunks per block
  per = (per + pr - 1) / pr * pr;
  const int nb = (int)((cap + per - 1) / per);
  float* part = static_cast<float*>(ws);
  hipStream_t s = S(stream);
#define DR_WG(H2, CW)                                                                         \
  do {                                                                                        \
    if (mfma && ch == 32)                                                                     \
      hipLaunchKernelGGL((din_wgrad_mfma_kernel<H2, 80, 40, 32>), dim3((unsigned)nb), dim3(256),  \
                         0, s, da1t, xt, da2t, h1t, h2t, dsc, cap, per, valid, part);                \
    else if (mfma)                                                                            \
      hipLaunchKernelGGL((din_wgrad_mfma_kernel<H2, 80, 40, 64>), dim3((unsigned)nb), dim3(256),  \
                         0, s, da1t, xt, da2t, h1t, h2t, dsc, cap, per, valid, part);                \
    else                                                                                      \
      hipLaunchKernelGGL((din_wgrad_kernel<H2, CW, 80, 40>), dim3((unsigned)nb), dim3(256), 0, \
                         s, da1t, xt, da2t, h1t, h2t, dsc, cap, per, valid, part);                   \
  } while (0)
  if (hidden2 == 72) DR_WG(72, 6);
  else if (hidden2 == 64) DR_WG(64, 8);
  else if (hidden2 == 32) DR_WG(32, 4);
  else DR_WG(128, 16);
#undef DR_WG
  hipLaunchKernelGGL(din_wgrad_reduce_kernel, dim3((unsigned)ceil_div((int64_t)out_n, 64)),
                     dim3(1024), 0, s, part, nb, out_n, out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_din_mlp_backward(const float* query, const float* facts, int64_t batch, int64_t seq_len,
                        int hidden, int n1, int n2, const float* w3, const float* grad_scores,
                        float* grad_facts, const dr_din_mlp_buf* buf, void* stream) {
  return dr_din_mlp_backward_tail(query, facts, batch, seq_len, hidden, n1, n2, w3, grad_scores,
                                  grad_facts, buf, 1, stream);
}

int dr_din_mlp_backward_tail(const float* query, const float* facts, int64_t batch,
                             int64_t seq_len, int hidden, int n1, int n2, const float* w3,
                             const float* grad_scores, float* grad_facts,
                             const dr_din_mlp_buf* buf, int zero_tail, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && seq_len >= 1 && buf && n1 == 80 && n2 == 40 &&
                 (hidden == 16 || hidden == 32 || hidden == 36 || hidden == 64),
             DR_INVALID_ARGUMENT, "bad shape");
  if (batch == 0) return DR_OK;
  DR_REQUIRE(query && facts && w3 && grad_scores && grad_facts && buf->da1t && buf->da2t &&
                 buf->xt && buf->dsc && buf->dqp && buf->s1 && buf->dq2,
             DR_INVALID_ARGUMENT, "null operand");
  hipStream_t st = S(stream);
  const int64_t cap = batch * seq_len;
  const unsigned pb = (unsigned)ceil_div(cap, 256);
  const unsigned sb = (unsigned)ceil_div(batch, 4);
#define DR_BWD(HH)                                                                              \
  if (hidden == HH) {                                                                           \
    hipLaunchKernelGGL((din_mlp_bwd_kernel<HH, 80, 40>), dim3(pb), dim3(256), 0, st, buf->pos,   \
                       buf->off, batch, seq_len, cap, facts, query, buf->w1p, buf->w2t, w3,     \
                       grad_scores, buf->h1t, buf->h2t, grad_facts, buf->da1t, buf->da2t,       \
                       buf->xt, buf->dsc, buf->dqp, zero_tail);                                 \
    hipLaunchKernelGGL((din_mlp_sample_kernel<HH, 80>), dim3(sb), dim3(256), 0, st, buf->off,    \
                       batch, cap, buf->da1t, buf->dqp, buf->s1, buf->dq2);                     \
  }
  DR_DIN_MLP_SHAPES(DR_BWD)
#undef DR_BWD
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_din_dice_forward(const float* x, const float* alpha, int64_t batch, int n, float epsilon,
                        float* y, float* stats, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 1 && n >= 0, DR_INVALID_ARGUMENT, "bad shape (batch >= 1)");
  if (n == 0) return DR_OK;
  DR_REQUIRE(x && alpha && y && stats, DR_INVALID_ARGUMENT, "null operand");
  DR_REQUIRE(batch < (1ll << 31), DR_INVALID_ARGUMENT, "batch must be < 2^31");
  hipLaunchKernelGGL(dice_fwd_kernel, dim3((unsigned)ceil_div(n, kDiceCols)), dim3(1024), 0,
                     S(stream), x, alpha, batch, n, epsilon, y, stats);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_din_dice_backward(const float* x, const float* grad_y, const float* alpha,
                         const float* stats, int64_t batch, int n, float epsilon, float* grad_x,
                         float* grad_alpha, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 1 && n >= 0, DR_INVALID_ARGUMENT, "bad shape (batch >= 1)");
  if (n == 0) return DR_OK;
  DR_REQUIRE(x && grad_y && alpha && stats && grad_x && grad_alpha, DR_INVALID_ARGUMENT,
             "null operand");
  DR_REQUIRE(batch < (1ll << 31), DR_INVALID_ARGUMENT, "batch must be < 2^31");
  hipLaunchKernelGGL(dice_bwd_kernel, dim3((unsigned)ceil_div(n, kDiceCols)), dim3(1024), 0,
                     S(stream), x, grad_y, alpha, stats, batch, n, epsilon, grad_x, grad_alpha);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_din_fcn_input_forward(const float* uid, const float* item, const float* his_sum,
                             const float* att, const float* gamma, const float* beta,
                             int64_t batch, int uid_dim, int hidden, float scale, float* out,
                             void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && uid_dim >= 0 && hidden > 0, DR_INVALID_ARGUMENT, "bad shape");
  const int64_t total = batch * (uid_dim + 4 * (int64_t)hidden);
  if (total == 0) return DR_OK;
  DR_REQUIRE(item && his_sum && att && gamma && beta && out && (uid || !uid_dim),
             DR_INVALID_ARGUMENT, "null operand");
  hipLaunchKernelGGL(fcn_input_fwd_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0,
                     S(stream), uid, item, his_sum, att, gamma, beta, batch, uid_dim, hidden, scale,
                     out);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

int dr_din_fcn_input_backward(const float* grad, const float* uid, const float* item,
                              const float* his_sum, const float* att, const float* gamma,
                              int64_t batch, int uid_dim, int hidden, float scale, float* g_uid,
                              float* g_item, float* g_his_sum, float* g_att, float* g_gamma,
                              float* g_beta, void* stream) {
  using namespace dr;
  DR_REQUIRE(batch >= 0 && uid_dim >= 0 && hidden > 0, DR_INVALID_ARGUMENT, "bad shape");
  DR_REQUIRE(batch < (1ll << 31), DR_INVALID_ARGUMENT, "batch must be < 2^31");
  const int n = uid_dim + 4 * hidden;
  DR_REQUIRE(grad && item && his_sum && att && gamma && g_item && g_his_sum && g_att && g_gamma &&
                 g_beta && (!uid_dim || (uid && g_uid)),
             DR_INVALID_ARGUMENT, "null operand");
  if (batch == 0) {
    int rc = fill_bytes(g_gamma, 0, (size_t)n * 4, S(stream));
    return rc ? rc : fill_bytes(g_beta, 0, (size_t)n * 4, S(stream));
  }
  const int64_t rows = batch * (uid_dim + (int64_t)hidden);
  hipLaunchKernelGGL(fcn_input_bwd_kernel, dim3((unsigned)ceil_div(rows, 256)), dim3(256), 0,
                     S(stream), grad, item, his_sum, gamma, batch, uid_dim, hidden, scale, g_uid,
                     g_item, g_his_sum, g_att);
  hipLaunchKernelGGL(fcn_input_param_grad_kernel, dim3((unsigned)ceil_div(n, kDiceCols)),
                     dim3(1024), 0, S(stream), grad, uid, item, his_sum, att, batch, uid_dim,
                     hidden, scale, g_gamma, g_beta);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // extern "C"
