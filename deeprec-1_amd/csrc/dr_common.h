// dr_common.h -- shared helpers of the MI355X engine (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "deeprec_amd.h"

namespace dr {

// Global-address-space views.  A pointer read from memory (a descriptor in
// LDS or a kernel-argument struct, a shuffled row address) is generic, and
// hipcc then emits FLAT loads / stores: those count on lgkmcnt as well as
// vmcnt and complete out of order, so every later LDS wait (a shuffle's
// lgkmcnt(0)) also waits for them and a batch of row loads serialises.  Row
// data always lives in device memory, so the hot helpers cast to
// address_space(1) and get global_load / global_store.
#if defined(__HIP_DEVICE_COMPILE__)
#define DR_GLOBAL __attribute__((address_space(1)))
#else
#define DR_GLOBAL  // (host pass: the device-only helpers below are never emitted)
#endif
template <class T>
__device__ __forceinline__ const DR_GLOBAL T* gp(const T* p) {
  return (const DR_GLOBAL T*)p;
}
template <class T>
__device__ __forceinline__ DR_GLOBAL T* gp(T* p) {
  return (DR_GLOBAL T*)p;
}
template <class T>
__device__ __forceinline__ T gld(const T* p) {
  return *gp(p);
}
template <class T>
__device__ __forceinline__ void gst(T* p, const T& v) {
  *gp(p) = v;
}

// Every vector-memory load of this wave has returned (s_waitcnt vmcnt(0),
// expcnt / lgkmcnt left alone).  Placed between a batch of row loads and
// the conditional stores of those rows: the compiler's own wait before a
// store inside a branch is vmcnt(0) again, which then also waits for the
// PREVIOUS store -- the stores of a batch serialise on their write
// acknowledgements.  After this wait no load is outstanding and the stores
// issue back to back.
__device__ __forceinline__ void wait_loads() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Nontemporal (stream-once) loads / stores of float / float4.
typedef float nf4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 nt_load(const float4* p) {
  const nf4 v = __builtin_nontemporal_load(gp(reinterpret_cast<const nf4*>(p)));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float nt_load(const float* p) { return __builtin_nontemporal_load(gp(p)); }
__device__ __forceinline__ void nt_store(float4 v, float4* p) {
  nf4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, gp(reinterpret_cast<nf4*>(p)));
}
__device__ __forceinline__ void nt_store(float v, float* p) { __builtin_nontemporal_store(v, gp(p)); }

void set_error(const char* fmt, ...);
// Device status word of the current device (latched by kernels).
int* status_word();

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// core.hip: measurement hook (dr_kernel_timing) -- events around one kernel
enum { DR_TIME_LOOKUP = 1, DR_TIME_POOL_ONEHOT = 2 };
void timing_mark(int which, hipStream_t st, bool begin);

// pool.hip: EV copy-out, out[i] = rows[i] >= 0 ? pool[rows[i]] : (defaults ?
// defaults[i] : dflt); the gather-copy kernel (dwordx4, nontemporal).
int gather_ev_rows(const float* pool, int64_t dim, const int64_t* rows, int64_t n,
                   const float* defaults, const float* dflt, float* out, hipStream_t s);

#define DR_HIP(x)                                                              \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      ::dr::set_error("%s failed: %s", #x, hipGetErrorString(e_));            \
      return DR_INTERNAL;                                                      \
    }                                                                          \
  } while (0)

#define DR_REQUIRE(cond, code, ...)                                            \
  do {                                                                         \
    if (!(cond)) {                                                             \
      ::dr::set_error(__VA_ARGS__);                                            \
      return code;                                                             \
    }                                                                          \
  } while (0)

#define DR_LAUNCH_CHECK()                                                      \
  do {                                                                         \
    hipError_t e_ = hipGetLastError();                                         \
    if (e_ != hipSuccess) {                                                    \
      ::dr::set_error("kernel launch failed: %s", hipGetErrorString(e_));     \
      return DR_INTERNAL;                                                      \
    }                                                                          \
  } while (0)

// Latch the first error code into the device status word.
__device__ __forceinline__ void latch(int* st, int code) { atomicCAS(st, 0, code); }

// Workspace carving: every piece 256-byte aligned.
struct Carver {
  char* p;
  size_t used;
  explicit Carver(void* base) : p(static_cast<char*>(base)), used(0) {}
  template <class T>
  T* take(size_t n) {
    size_t off = (used + 255) & ~size_t(255);
    used = off + n * sizeof(T);
    return p ? reinterpret_cast<T*>(p + off) : nullptr;
  }
};

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t next_pow2(int64_t x) {
  int64_t c = 1;
  while (c < x) c <<= 1;
  return c;
}

__device__ __forceinline__ uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

// SplitMix64 of (seed, row, col) -> uniform [-1, 1).  Host and device share it
// (synthetic tables: dr_fill_synthetic, dr_ev_insert_synthetic).
__host__ __device__ __forceinline__ float synth(uint64_t seed, int64_t row, int64_t col) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ULL + (uint64_t)row * 0xBF58476D1CE4E5B9ULL +
               (uint64_t)col * 0x94D049BB133111EBULL;
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return (float)(int32_t)(uint32_t)(z >> 32) * (1.0f / 2147483648.0f);
}

// ---- bf16 rows (bf16 EVs) --------------------------------------------------
// fp32 -> bf16 round-to-nearest-even; NaN -> 0x7FC0 (torch's c10::BFloat16
// conversion, so bf16 results compare bitwise with torch.bfloat16 casts).
__host__ __device__ __forceinline__ uint16_t bf16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7FFFFFFFu) > 0x7F800000u) return 0x7FC0;
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline uint16_t bf16_rne_host(float f) { return bf16_rne(f); }
__host__ __device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
// two packed bf16 (low half = element 2k) <-> float2
__device__ __forceinline__ float2 bf16x2_to_f2(uint32_t w) {
  return make_float2(__uint_as_float(w << 16), __uint_as_float(w & 0xFFFF0000u));
}
__device__ __forceinline__ uint32_t f2_to_bf16x2(float a, float b) {
  return (uint32_t)bf16_rne(a) | ((uint32_t)bf16_rne(b) << 16);
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int l = __lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Effective element count: min(n, *n_dev) when a device count is supplied.
__device__ __forceinline__ int64_t eff_n(int64_t n, const int64_t* n_dev) {
  if (!n_dev) return n;
  int64_t m = *n_dev;
  return m < n ? m : n;
}

// Table holding element i of a grouped launch (koff: T+1 prefix offsets in
// kernel-argument memory).  The binary search for the block's first element
// is uniform (scalar loads); each lane then steps over the few table
// boundaries inside its block.  A per-lane linear walk over koff would be up
// to T dependent loads per element.
__device__ __forceinline__ int table_of(const int64_t* koff, int T, int64_t i,
                                        int64_t block_first) {
  int lo = 0, hi = T - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (koff[mid] <= block_first)
      lo = mid;
    else
      hi = mid - 1;
  }
  int t = lo;
  while (t + 1 < T && i >= koff[t + 1]) ++t;
  return t;
}

// Byte-pattern fill by a kernel (stream-ordered, graph-capturable).  Used
// instead of hipMemsetAsync for workspace state that later kernels probe:
// a captured memset node is serviced by a DMA engine and in hipGraph replay
// the next kernel may still see the previous contents in another XCD's L2.
int fill_bytes(void* p, unsigned char value, size_t bytes, hipStream_t st);

// ev.hip: host-side serialisation of the calls on EVs (EvGuard) for
// composite entries outside ev.hip that read EV pointers across calls
void* ev_guard_acquire(dr_ev* const* evs, int64_t n);
void ev_guard_release(void* g);
struct EvGuardRef {
  void* g;
  explicit EvGuardRef(dr_ev* ev) : g(ev_guard_acquire(&ev, 1)) {}
  ~EvGuardRef() { ev_guard_release(g); }
  EvGuardRef(const EvGuardRef&) = delete;
  EvGuardRef& operator=(const EvGuardRef&) = delete;
};

// ---- row-grouped lookup backward fused with KV SGD (grad_rows.hip; the C
// entry dr_ev_pool_grad_rows_apply_sgd is in ev.hip, which owns the EVs) ----
// Per table of the group: the var column's rows (fp32, or bf16 pairs when
// bf16), and the version array to stamp with gs (steps_to_live EVs) or null.
struct RowsSgd {
  void* pool[DR_MAX_GROUP];
  int64_t* version[DR_MAX_GROUP];
  float lr;
  int bf16;
  int64_t gs;
};
int rows_apply_sgd(const dr_pool_grad_desc* descs_host, int num_tables, int64_t batch, int dim,
                   const int64_t* rowsel, int64_t row_limit, const RowsSgd& sg, void* ws,
                   size_t ws_bytes, hipStream_t s, int rows_record);

#ifdef DR_UC_DIAG
// xgmi.hip, diagnostic build only: uncached blocks freed to hipFree, and a
// D2H-vs-kernel read check of a buffer against the bytes expected in it
void uc_diag_freed(void* p, size_t n);
void uc_diag_check(const char* what, const void* dev, const void* expect, size_t bytes);
bool uc_diag_check_xcd(const char* what, const void* dev, uint32_t fill, size_t bytes);
void uc_diag_writeback(int system);
#endif

// ---- scan / sort primitives (scan_sort.hip) --------------------------------
size_t scan_ws_bytes(int64_t n);
// Exclusive scan of int32 values into int32 out; *total (device int64) = sum.
int scan_exclusive_i32(const int32_t* in, int32_t* out, int64_t n, const int64_t* n_dev,
                       int64_t* total, void* ws, hipStream_t st);
// Exclusive scan of the marks (in[i] != -1) of a "-1 = empty" array.
int scan_exclusive_marks(const int32_t* in, int32_t* out, int64_t n, int64_t* total, void* ws,
                         hipStream_t st);

// Stable LSD radix sort of (uint32 key, int32 value) pairs on bits [0, bits).
size_t sort_pairs_u32_ws_bytes(int64_t n);
int sort_pairs_u32(const uint32_t* keys_in, const int32_t* vals_in, uint32_t* keys_out,
                   int32_t* vals_out, int64_t n, int bits, void* ws, hipStream_t st);

// The same for uint64 keys over the first *n_dev of n_cap pairs (DEVICE
// count; the grid is sized for n_cap, no host sync).  Workspace:
// dr_sort_pairs_workspace_size(n_cap).
int sort_pairs_u64_dev(const uint64_t* keys_in, const int32_t* vals_in, uint64_t* keys_out,
                       int32_t* vals_out, int64_t n_cap, const int64_t* n_dev, int bits,
                       void* ws, hipStream_t st);

}  // namespace dr
