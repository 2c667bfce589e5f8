// dr_rows.h -- one embedding row held by a group of G lanes (VEC floats per
// lane per column chunk, CPL chunks): loads / stores (default or
// nontemporal policy) and elementwise helpers shared by the pooling, gather
// and EV kernels.
#pragma once
#include "dr_common.h"

namespace dr {

template <int VEC>
struct VecT;
template <>
struct VecT<4> {
  using T = float4;
};
template <>
struct VecT<2> {
  using T = float2;
};
template <>
struct VecT<1> {
  using T = float;
};

__device__ __forceinline__ float4 vadd(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float2 vadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float vadd(float a, float b) { return a + b; }
__device__ __forceinline__ float2 vdiv(float2 a, float q) { return make_float2(a.x / q, a.y / q); }
__device__ __forceinline__ float2 vmul(float2 a, float q) { return make_float2(a.x * q, a.y * q); }
__device__ __forceinline__ float4 vdiv(float4 a, float q) {
  return make_float4(a.x / q, a.y / q, a.z / q, a.w / q);
}
__device__ __forceinline__ float vdiv(float a, float q) { return a / q; }
__device__ __forceinline__ float4 vmul(float4 a, float q) {
  return make_float4(a.x * q, a.y * q, a.z * q, a.w * q);
}
__device__ __forceinline__ float vmul(float a, float q) { return a * q; }
__device__ __forceinline__ float vdot(float4 a) { return a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w; }
__device__ __forceinline__ float vdot(float a) { return a * a; }
template <class V>
__device__ __forceinline__ V vzero();
template <>
__device__ __forceinline__ float4 vzero<float4>() {
  return make_float4(0.f, 0.f, 0.f, 0.f);
}
template <>
__device__ __forceinline__ float2 vzero<float2>() {
  return make_float2(0.f, 0.f);
}
template <>
__device__ __forceinline__ float vzero<float>() {
  return 0.f;
}

template <int VEC, int G, int CPL>
struct Row {
  typename VecT<VEC>::T v[CPL];
};

template <int VEC, int G, int CPL>
__device__ __forceinline__ void load_row(Row<VEC, G, CPL>& x, const float* p, int lg, int dv) {
  using V = typename VecT<VEC>::T;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int col = lg + c * G;
    x.v[c] = (p && col < dv) ? gld(reinterpret_cast<const V*>(p) + col) : vzero<V>();
  }
}

// Rows read exactly once per launch: nontemporal hint (no L2 retention).
template <int VEC, int G, int CPL>
__device__ __forceinline__ void load_row_nt(Row<VEC, G, CPL>& x, const float* p, int lg, int dv) {
  using V = typename VecT<VEC>::T;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int col = lg + c * G;
    x.v[c] = (p && col < dv) ? nt_load(reinterpret_cast<const V*>(p) + col) : vzero<V>();
  }
}

template <int VEC, int G, int CPL>
__device__ __forceinline__ void store_row_nt(const Row<VEC, G, CPL>& x, float* p, int lg, int dv) {
  using V = typename VecT<VEC>::T;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int col = lg + c * G;
    if (col < dv) nt_store(x.v[c], reinterpret_cast<V*>(p) + col);
  }
}

template <int VEC, int G, int CPL>
__device__ __forceinline__ void store_row(const Row<VEC, G, CPL>& x, float* p, int lg, int dv) {
  using V = typename VecT<VEC>::T;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int col = lg + c * G;
    if (col < dv) gst(reinterpret_cast<V*>(p) + col, x.v[c]);
  }
}

template <int VEC, int G, int CPL>
__device__ __forceinline__ void acc_add(Row<VEC, G, CPL>& a, const Row<VEC, G, CPL>& b) {
#pragma unroll
  for (int c = 0; c < CPL; ++c) a.v[c] = vadd(a.v[c], b.v[c]);
}

// bf16 rows (bf16 EVs): lane chunk c covers VEC consecutive bf16 values
// (VEC * 2 bytes) of a row whose float-word pointer is p; widened to fp32.
template <int VEC, int G, int CPL>
__device__ __forceinline__ void load_row_bf16(Row<VEC, G, CPL>& x, const float* p, int lg, int dv) {
  static_assert(VEC == 4, "bf16 rows use 4-value chunks");
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int col = lg + c * G;
    if (p && col < dv) {
      const u2 w = gld(reinterpret_cast<const u2*>(p) + col);
      const float2 a = bf16x2_to_f2(w.x), b = bf16x2_to_f2(w.y);
      x.v[c] = make_float4(a.x, a.y, b.x, b.y);
    } else {
      x.v[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// The same with the nontemporal policy (rows read once per launch).
template <int VEC, int G, int CPL>
__device__ __forceinline__ void load_row_bf16_nt(Row<VEC, G, CPL>& x, const float* p, int lg,
                                                 int dv) {
  static_assert(VEC == 4, "bf16 rows use 4-value chunks");
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int col = lg + c * G;
    if (p && col < dv) {
      const u2 w = __builtin_nontemporal_load(gp(reinterpret_cast<const u2*>(p) + col));
      const float2 a = bf16x2_to_f2(w.x), b = bf16x2_to_f2(w.y);
      x.v[c] = make_float4(a.x, a.y, b.x, b.y);
    } else {
      x.v[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// Row load of a one-hot copy: fp32 rows, or (WIDEN) bf16 rows widened.
template <int VEC, int G, int CPL, bool WIDEN>
__device__ __forceinline__ void load_row_copy(Row<VEC, G, CPL>& x, const float* p, int lg, int dv) {
  if constexpr (WIDEN)
    load_row_bf16_nt<VEC, G, CPL>(x, p, lg, dv);
  else
    load_row_nt<VEC, G, CPL>(x, p, lg, dv);
}

// fp32 row -> bf16 (round to nearest even) at the float-word pointer p.
template <int VEC, int G, int CPL>
__device__ __forceinline__ void store_row_bf16(const Row<VEC, G, CPL>& x, float* p, int lg, int dv) {
  static_assert(VEC == 4, "bf16 rows use 4-value chunks");
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int col = lg + c * G;
    if (col < dv) {
      const u2 w = {f2_to_bf16x2(x.v[c].x, x.v[c].y), f2_to_bf16x2(x.v[c].z, x.v[c].w)};
      gst(reinterpret_cast<u2*>(p) + col, w);
    }
  }
}

// Row load with an always-valid pointer (only the lane's column predicate):
// a per-row "pointer or zero" select makes hipcc branch around every load
// and wait for it before the next one, so batches of independent loads
// serialise into dependent round trips.  Callers clamp indices instead and
// discard invalid rows after the loads.
template <int VEC, int G, int CPL>
__device__ __forceinline__ void load_row_u(Row<VEC, G, CPL>& x, const float* p, int lg, int dv) {
  using V = typename VecT<VEC>::T;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int col = lg + c * G;
    x.v[c] = col < dv ? gld(reinterpret_cast<const V*>(p) + col) : vzero<V>();
  }
}

// One column's serial chain over the LDS stage sp[0, nv) (16-B aligned):
// acc = acc + sp[0] + sp[1] + ... in order (fresh: the chain starts at
// sp[0]).  The 16-B reads run 64 positions ahead of the adds in 16 fixed
// registers (the lgkmcnt limit), one counted wait per 8 registers (32
// positions), each group reloaded right after its adds -- as inline asm,
// because the compiler otherwise re-issued the reads and waited for them
// every 4 positions.  The wait takes the registers it guards as operands, so
// the adds cannot be scheduled above it.  The s_waitcnt itself was the cost:
// DIN's padding chain (2 x 10^5 positions) took 1.00 ms with a wait per 4
// positions and 4 registers, 0.90 with 16 registers, 0.74 / 0.65 / 0.62 ms
// with a wait per 8 / 16 / 32 positions (7.4 cycles per position;
// profiles/r06_seg_rounds_walk.log).
#define DR_LDS4(R, A, OFF) \
  asm volatile("ds_read_b128 %0, %1 offset:" #OFF : "=v"(R) : "v"(A))
#define DR_LGKM(N, R) asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(R))
#define DR_LGKM2(N, R, Q) asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(R), "+v"(Q))
__device__ __forceinline__ float chain_walk(const float* sp, int nv, bool& fresh, float acc) {
  int jj = 0;
  if (fresh) {
    acc = sp[0];
    fresh = false;
    jj = 1;
  }
  for (; jj < nv && (jj & 3); ++jj) acc = acc + sp[jj];
  if (jj + 64 <= nv) {
    typedef __attribute__((address_space(3))) const float lds_f;
    uint32_t a = (uint32_t)(size_t)(lds_f*)(sp + jj);
    // nothing of the compiler's own in flight: its wait pass then puts no
    // lgkmcnt(0) inside the loop (it does not see the asm reads)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v r0, r1, r2, r3, r4, r5, r6, r7, r8, r9, r10, r11, r12, r13, r14, r15;
    DR_LDS4(r0, a, 0);
    DR_LDS4(r1, a, 16);
    DR_LDS4(r2, a, 32);
    DR_LDS4(r3, a, 48);
    DR_LDS4(r4, a, 64);
    DR_LDS4(r5, a, 80);
    DR_LDS4(r6, a, 96);
    DR_LDS4(r7, a, 112);
    DR_LDS4(r8, a, 128);
    DR_LDS4(r9, a, 144);
    DR_LDS4(r10, a, 160);
    DR_LDS4(r11, a, 176);
    DR_LDS4(r12, a, 192);
    DR_LDS4(r13, a, 208);
    DR_LDS4(r14, a, 224);
    DR_LDS4(r15, a, 240);
    auto add4 = [&](const f4v& v) {
      acc = acc + v.x; acc = acc + v.y; acc = acc + v.z; acc = acc + v.w;
    };
    for (; jj + 128 <= nv; jj += 64) {
      asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)); add4(r0); add4(r1); add4(r2); add4(r3); add4(r4); add4(r5); add4(r6); add4(r7); DR_LDS4(r0, a, 256); DR_LDS4(r1, a, 272); DR_LDS4(r2, a, 288); DR_LDS4(r3, a, 304); DR_LDS4(r4, a, 320); DR_LDS4(r5, a, 336); DR_LDS4(r6, a, 352); DR_LDS4(r7, a, 368);
      asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(r8), "+v"(r9), "+v"(r10), "+v"(r11), "+v"(r12), "+v"(r13), "+v"(r14), "+v"(r15)); add4(r8); add4(r9); add4(r10); add4(r11); add4(r12); add4(r13); add4(r14); add4(r15); DR_LDS4(r8, a, 384); DR_LDS4(r9, a, 400); DR_LDS4(r10, a, 416); DR_LDS4(r11, a, 432); DR_LDS4(r12, a, 448); DR_LDS4(r13, a, 464); DR_LDS4(r14, a, 480); DR_LDS4(r15, a, 496);
      a += 256;
    }
    asm volatile("s_waitcnt lgkmcnt(15)" : "+v"(r0)); add4(r0);
    asm volatile("s_waitcnt lgkmcnt(14)" : "+v"(r1)); add4(r1);
    asm volatile("s_waitcnt lgkmcnt(13)" : "+v"(r2)); add4(r2);
    asm volatile("s_waitcnt lgkmcnt(12)" : "+v"(r3)); add4(r3);
    asm volatile("s_waitcnt lgkmcnt(11)" : "+v"(r4)); add4(r4);
    asm volatile("s_waitcnt lgkmcnt(10)" : "+v"(r5)); add4(r5);
    asm volatile("s_waitcnt lgkmcnt(9)" : "+v"(r6)); add4(r6);
    asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(r7)); add4(r7);
    asm volatile("s_waitcnt lgkmcnt(7)" : "+v"(r8)); add4(r8);
    asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(r9)); add4(r9);
    asm volatile("s_waitcnt lgkmcnt(5)" : "+v"(r10)); add4(r10);
    asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(r11)); add4(r11);
    asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(r12)); add4(r12);
    asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(r13)); add4(r13);
    asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(r14)); add4(r14);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r15)); add4(r15);
    jj += 64;
  }
  for (; jj < nv; ++jj) acc = acc + sp[jj];
  return acc;
}
#undef DR_LDS4
#undef DR_LGKM
#undef DR_LGKM2

}  // namespace dr
