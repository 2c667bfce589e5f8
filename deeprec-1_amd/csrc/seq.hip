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

}  // extern "C"
