// strings.hip -- string -> id on the GPU: farmhash Fingerprint64 and
// StringToHashBucketFast (the step before the lookup).
//
// Reference: StringToHashBucketAliOp (core/kernels/string_to_hash_bucket_ali_op.h:
// 33-63) computes bucket = Fingerprint64(s) % num_buckets per string on CPU
// threads (Shard); EV string columns use num_buckets = INT64_MAX
// (python/feature_column/feature_column_v2.py:5954-5957).  Fingerprint64 is
// farmhash::Fingerprint64 = farmhashna::Hash64 (core/platform/fingerprint.h:
// 80-88; google/farmhash @816a4ae6, tensorflow/workspace.bzl:275-282).
//
// Layout: strings arrive Arrow-style -- one byte buffer plus int64 offsets
// [n+1] -- resident in HBM.  One lane hashes one string.  Byte work, HBM
// bound: per string 8 B offset + len bytes read + 8 B id written.  Unaligned
// 8-/4-byte fetches are assembled from naturally aligned loads; an aligned
// word that contains at least one byte of the string lies inside the same
// page as that byte, so it can never fault even at the buffer's ends.
#include "dr_common.h"

namespace dr {

namespace fh {
constexpr uint64_t k0 = 0xc3a5c85c97cb3127ULL;
constexpr uint64_t k1 = 0xb492b66fbe98f273ULL;
constexpr uint64_t k2 = 0x9ae16a3b2f90404fULL;

__device__ __forceinline__ uint64_t fetch64(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p & ~(uintptr_t)7;
  const unsigned sh = (unsigned)((uintptr_t)p & 7) * 8;
  const uint64_t lo = *reinterpret_cast<const uint64_t*>(a);
  if (sh == 0) return lo;
  const uint64_t hi = *reinterpret_cast<const uint64_t*>(a + 8);
  return (lo >> sh) | (hi << (64 - sh));
}
__device__ __forceinline__ uint64_t fetch32(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p & ~(uintptr_t)3;
  const unsigned sh = (unsigned)((uintptr_t)p & 3) * 8;
  const uint32_t lo = *reinterpret_cast<const uint32_t*>(a);
  if (sh == 0) return lo;
  const uint32_t hi = *reinterpret_cast<const uint32_t*>(a + 4);
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh);
}
__device__ __forceinline__ uint64_t rot(uint64_t v, int s) {
  return s == 0 ? v : (v >> s) | (v << (64 - s));
}
__device__ __forceinline__ uint64_t smix(uint64_t v) { return v ^ (v >> 47); }
__device__ __forceinline__ uint64_t len16(uint64_t u, uint64_t v, uint64_t mul) {
  uint64_t a = (u ^ v) * mul;
  a ^= a >> 47;
  uint64_t b = (v ^ a) * mul;
  b ^= b >> 47;
  return b * mul;
}
__device__ __forceinline__ void weak32(const uint8_t* s, uint64_t a, uint64_t b, uint64_t& o1,
                                       uint64_t& o2) {
  const uint64_t w = fetch64(s), x = fetch64(s + 8), y = fetch64(s + 16), z = fetch64(s + 24);
  a += w;
  b = rot(b + a + z, 21);
  const uint64_t c = a;
  a += x;
  a += y;
  b += rot(a, 44);
  o1 = a + z;
  o2 = b + c;
}

__device__ uint64_t hash64(const uint8_t* s, uint64_t len) {
  if (len <= 16) {
    if (len >= 8) {
      const uint64_t mul = k2 + len * 2;
      const uint64_t a = fetch64(s) + k2;
      const uint64_t b = fetch64(s + len - 8);
      const uint64_t c = rot(b, 37) * mul + a;
      const uint64_t d = (rot(a, 25) + b) * mul;
      return len16(c, d, mul);
    }
    if (len >= 4) {
      const uint64_t mul = k2 + len * 2;
      const uint64_t a = fetch32(s);
      return len16(len + (a << 3), fetch32(s + len - 4), mul);
    }
    if (len > 0) {
      const uint32_t a = s[0], b = s[len >> 1], c = s[len - 1];
      const uint32_t y = a + (b << 8);
      const uint32_t z = (uint32_t)len + (c << 2);
      return smix(y * k2 ^ z * k0) * k2;
    }
    return k2;
  }
  if (len <= 32) {
    const uint64_t mul = k2 + len * 2;
    const uint64_t a = fetch64(s) * k1;
    const uint64_t b = fetch64(s + 8);
    const uint64_t c = fetch64(s + len - 8) * mul;
    const uint64_t d = fetch64(s + len - 16) * k2;
    return len16(rot(a + b, 43) + rot(c, 30) + d, a + rot(b + k2, 18) + c, mul);
  }
  if (len <= 64) {
    const uint64_t mul = k2 + len * 2;
    const uint64_t a = fetch64(s) * k2;
    const uint64_t b = fetch64(s + 8);
    const uint64_t c = fetch64(s + len - 8) * mul;
    const uint64_t d = fetch64(s + len - 16) * k2;
    const uint64_t y = rot(a + b, 43) + rot(c, 30) + d;
    const uint64_t z = len16(y, a + rot(b + k2, 18) + c, mul);
    const uint64_t e = fetch64(s + 16) * mul;
    const uint64_t f = fetch64(s + 24);
    const uint64_t g = (y + fetch64(s + len - 32)) * mul;
    const uint64_t h = (z + fetch64(s + len - 24)) * mul;
    return len16(rot(e + f, 43) + rot(g, 30) + h, e + rot(f + a, 18) + g, mul);
  }
  const uint64_t seed = 81;
  uint64_t x = seed, y = seed * k1 + 113, z = smix(y * k2 + 113) * k2;
  uint64_t v1 = 0, v2 = 0, w1 = 0, w2 = 0, t;
  x = x * k2 + fetch64(s);
  const uint8_t* end = s + ((len - 1) / 64) * 64;
  const uint8_t* last64 = end + ((len - 1) & 63) - 63;
  do {
    x = rot(x + y + v1 + fetch64(s + 8), 37) * k1;
    y = rot(y + v2 + fetch64(s + 48), 42) * k1;
    x ^= w2;
    y += v1 + fetch64(s + 40);
    z = rot(z + w1, 33) * k1;
    weak32(s, v2 * k1, x + w1, v1, v2);
    weak32(s + 32, z + w2, y + fetch64(s + 16), w1, w2);
    t = z;
    z = x;
    x = t;
    s += 64;
  } while (s != end);
  const uint64_t mul = k1 + ((z & 0xff) << 1);
  s = last64;
  w1 += ((len - 1) & 63);
  v1 += w1;
  w1 += v1;
  x = rot(x + y + v1 + fetch64(s + 8), 37) * mul;
  y = rot(y + v2 + fetch64(s + 48), 42) * mul;
  x ^= w2 * 9;
  y += v1 * 9 + fetch64(s + 40);
  z = rot(z + w1, 33) * mul;
  weak32(s, v2 * mul, x + w1, v1, v2);
  weak32(s + 32, z + w2, y + fetch64(s + 16), w1, w2);
  t = z;
  z = x;
  x = t;
  return len16(len16(v1, w1, mul) + smix(y) * k0 + z, len16(v2, w2, mul) + x, mul);
}
}  // namespace fh

// MODE 0: raw fingerprint; 1: % num_buckets.  Offsets must be non-decreasing
// (a negative length latches INVALID_ARGUMENT and writes 0).
template <int MODE>
__global__ __launch_bounds__(256) void hash_strings_kernel(const uint8_t* __restrict__ bytes,
                                                           const int64_t* __restrict__ off,
                                                           int64_t n, uint64_t nb,
                                                           uint64_t* __restrict__ out, int* st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t b = off[i], e = off[i + 1];
  if (e < b || b < 0) {
    latch(st, DR_INVALID_ARGUMENT);
    out[i] = 0;
    return;
  }
  const uint64_t h = fh::hash64(bytes + b, (uint64_t)(e - b));
  out[i] = MODE == 0 ? h : h % nb;
}

template <int MODE>
static int hash_strings(const uint8_t* bytes, const int64_t* offsets, int64_t n, uint64_t nb,
                        uint64_t* out, void* stream) {
  DR_REQUIRE(n >= 0 && (n == 0 || (offsets && out)), DR_INVALID_ARGUMENT, "bad argument");
  if (n == 0) return DR_OK;
  int* st = status_word();
  DR_REQUIRE(st, DR_INTERNAL, "status word unavailable");
  hipLaunchKernelGGL(hash_strings_kernel<MODE>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0,
                     S(stream), bytes, offsets, n, nb, out, st);
  DR_LAUNCH_CHECK();
  return DR_OK;
}

}  // namespace dr

extern "C" int dr_fingerprint64(const uint8_t* bytes, const int64_t* offsets, int64_t n,
                                uint64_t* out, void* stream) {
  return dr::hash_strings<0>(bytes, offsets, n, 0, out, stream);
}

extern "C" int dr_string_to_hash_bucket_fast(const uint8_t* bytes, const int64_t* offsets,
                                             int64_t n, int64_t num_buckets, int64_t* out,
                                             void* stream) {
  DR_REQUIRE(num_buckets > 0, DR_INVALID_ARGUMENT,
             "num_buckets must be positive (StringToHashBucketFast attr)");
  return dr::hash_strings<1>(bytes, offsets, n, (uint64_t)num_buckets,
                             reinterpret_cast<uint64_t*>(out), stream);
}
