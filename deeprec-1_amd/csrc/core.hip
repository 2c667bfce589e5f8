// core.hip -- error reporting, device status word, synthetic table fill.
#include <stdarg.h>
#include <stdio.h>

#include <mutex>
#include <vector>

#include "dr_common.h"

__device__ int g_dr_status;

namespace dr {

static thread_local char t_err[1024];

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(t_err, sizeof(t_err), fmt, ap);
  va_end(ap);
}

int* status_word() {
  static std::mutex mu;
  static int* cache[64] = {nullptr};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  if (!cache[dev]) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_dr_status)) != hipSuccess) return nullptr;
    cache[dev] = static_cast<int*>(p);
  }
  return cache[dev];
}

__global__ void fill_u32_kernel(uint32_t* __restrict__ p, int64_t n4, uint32_t v) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) p[i] = v;
}

__global__ void fill_u8_kernel(unsigned char* __restrict__ p, int64_t n, unsigned char v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

int fill_bytes(void* p, unsigned char value, size_t bytes, hipStream_t st) {
  if (bytes == 0) return DR_OK;
  const uintptr_t a = (uintptr_t)p;
  const uint32_t v4 = 0x01010101u * value;
  if ((a & 3) == 0) {
    const int64_t n4 = (int64_t)(bytes / 4);
    if (n4 > 0) {
      int64_t blocks = ceil_div(n4, 256);
      if (blocks > 4096) blocks = 4096;
      hipLaunchKernelGGL(fill_u32_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                         static_cast<uint32_t*>(p), n4, v4);
    }
    const int64_t tail = (int64_t)(bytes - (size_t)n4 * 4);
    if (tail > 0)
      hipLaunchKernelGGL(fill_u8_kernel, dim3(1), dim3(256), 0, st,
                         static_cast<unsigned char*>(p) + n4 * 4, tail, value);
  } else {
    hipLaunchKernelGGL(fill_u8_kernel, dim3((unsigned)ceil_div((int64_t)bytes, 256)), dim3(256), 0,
                       st, static_cast<unsigned char*>(p), (int64_t)bytes, value);
  }
  DR_LAUNCH_CHECK();
  return DR_OK;
}

__global__ void fill_synth_kernel(float* __restrict__ t, int64_t rows, int dim, uint64_t seed) {
  const int64_t total4 = rows * dim / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += stride) {
    const int64_t e = i * 4;
    float4 v;
    v.x = synth(seed, (e + 0) / dim, (e + 0) % dim);
    v.y = synth(seed, (e + 1) / dim, (e + 1) % dim);
    v.z = synth(seed, (e + 2) / dim, (e + 2) % dim);
    v.w = synth(seed, (e + 3) / dim, (e + 3) % dim);
    reinterpret_cast<float4*>(t)[i] = v;
  }
}

__global__ void fill_synth_tail_kernel(float* __restrict__ t, int64_t begin, int64_t end,
                                       int dim, uint64_t seed) {
  const int64_t e = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < end) t[e] = synth(seed, e / dim, e % dim);
}


// ---- measurement hook: HIP events around one kernel's launches ------------
// dr_kernel_timing(which) arms it (DR_TIME_LOOKUP: ev_lookup_onehot_kernel,
// DR_TIME_POOL_ONEHOT: pool_onehot_kernel); every such launch on any stream
// is then bracketed by a pair of events recorded on that launch's stream,
// and dr_kernel_timing_result sums their elapsed times -- the kernel's own
// duration, not the surrounding helper launches.  Off: one branch per launch.
static std::mutex g_tmu;
static int g_time_which = 0;
static std::vector<std::pair<hipEvent_t, hipEvent_t>> g_tev;

bool timing_on(int which) { return g_time_which == which; }

void timing_mark(int which, hipStream_t st, bool begin) {
  if (g_time_which != which) return;
  std::lock_guard<std::mutex> g(g_tmu);
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return;
  if (hipEventRecord(e, st) != hipSuccess) {
    (void)hipEventDestroy(e);
    return;
  }
  if (begin)
    g_tev.push_back({e, nullptr});
  else if (!g_tev.empty() && g_tev.back().second == nullptr)
    g_tev.back().second = e;
  else
    (void)hipEventDestroy(e);
}

}  // namespace dr

extern "C" {

int dr_kernel_timing(int which) {
  using namespace dr;
  std::lock_guard<std::mutex> g(g_tmu);
  for (auto& p : g_tev) {
    if (p.first) (void)hipEventDestroy(p.first);
    if (p.second) (void)hipEventDestroy(p.second);
  }
  g_tev.clear();
  g_time_which = which;
  return DR_OK;
}

int dr_kernel_timing_result(double* total_ms, int64_t* launches) {
  using namespace dr;
  DR_REQUIRE(total_ms && launches, DR_INVALID_ARGUMENT, "null output");
  std::lock_guard<std::mutex> g(g_tmu);
  double t = 0.0;
  int64_t n = 0;
  for (auto& p : g_tev) {
    if (!p.first || !p.second) continue;
    DR_HIP(hipEventSynchronize(p.second));
    float ms = 0.f;
    DR_HIP(hipEventElapsedTime(&ms, p.first, p.second));
    t += ms;
    ++n;
  }
  *total_ms = t;
  *launches = n;
  return DR_OK;
}

int dr_abi_version(void) { return 2; }

const char* dr_last_error(void) { return dr::t_err; }

int dr_status_check(void* stream) {
  int* st = dr::status_word();
  DR_REQUIRE(st != nullptr, DR_INTERNAL, "no device status word");
  DR_HIP(hipStreamSynchronize(dr::S(stream)));
  int v = 0;
  DR_HIP(hipMemcpy(&v, st, sizeof(int), hipMemcpyDeviceToHost));
  if (v != 0) {
    int z = 0;
    DR_HIP(hipMemcpy(st, &z, sizeof(int), hipMemcpyHostToDevice));
    dr::set_error("device kernel latched status %d", v);
  }
  return v;
}

int dr_fill_synthetic(float* table, int64_t rows, int dim, uint64_t seed, void* stream) {
  DR_REQUIRE(rows >= 0 && dim > 0, DR_INVALID_ARGUMENT, "bad table shape");
  DR_REQUIRE(((uintptr_t)table & 15) == 0, DR_INVALID_ARGUMENT, "table must be 16B aligned");
  const int64_t total = rows * dim;
  const int64_t total4 = total / 4;
  if (total4 > 0) {
    int64_t blocks = dr::ceil_div(total4, 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(dr::fill_synth_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       dr::S(stream), table, rows, dim, seed);
    DR_LAUNCH_CHECK();
  }
  if (total4 * 4 < total) {
    hipLaunchKernelGGL(dr::fill_synth_tail_kernel, dim3(1), dim3(256), 0, dr::S(stream), table,
                       total4 * 4, total, dim, seed);
    DR_LAUNCH_CHECK();
  }
  return DR_OK;
}

float dr_synth_value(uint64_t seed, int64_t row, int64_t col) { return dr::synth(seed, row, col); }

}  // extern "C"
