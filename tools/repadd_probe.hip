// Device timing of dr::rep_add (dr_repadd.h): one wave, lanes 0..15 each walk
// one column over DIN-like segments (4050 segments of 1..99 identical terms,
// terms ~N(0, 1e-5)), against the same walk by plain adds; both checked
// bit-equal to the host loop.  Prints cycles per segment / per position.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <random>
#include <vector>
#include "dr_repadd.h"

constexpr int NS = 4050, NC = 16;

// mode 0: plain adds, lane = column; 1: rep_add, lane = column (16 lanes of
// one wave); 2: rep_add, wave = column (all 64 lanes of wave w on column w)
__global__ void walk(const float* x, const int* k, int mode, float* out, long long* cyc) {
  const int lane = mode == 2 ? (int)(threadIdx.x >> 6) : (int)threadIdx.x;
  if (lane >= NC || (mode != 2 && threadIdx.x >= 64)) return;
  float s = 0.f;
  const long long t0 = clock64();
  for (int i = 0; i < NS; ++i) {
    const float xi = x[i * NC + lane];
    const int ki = k[i];
    if (mode) {
      s = dr::rep_add(s, xi, ki);
    } else {
      for (int j = 0; j < ki; ++j) s = s + xi;
    }
  }
  const long long t1 = clock64();
  if (mode != 2 || (threadIdx.x & 63) == 0) out[lane] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  std::mt19937 g(1);
  std::normal_distribution<float> nd(0.f, 1e-5f);
  std::uniform_int_distribution<int> ud(1, 99);
  std::vector<float> x(NS * NC);
  std::vector<int> k(NS);
  long pos = 0;
  for (int i = 0; i < NS; ++i) {
    k[i] = ud(g);
    pos += k[i];
    for (int c = 0; c < NC; ++c) x[i * NC + c] = nd(g);
  }
  std::vector<float> ref(NC, 0.f);
  for (int c = 0; c < NC; ++c)
    for (int i = 0; i < NS; ++i)
      for (int j = 0; j < k[i]; ++j) ref[c] = ref[c] + x[i * NC + c];
  float *dx, *dout;
  int* dk;
  long long* dc;
  hipMalloc(&dx, x.size() * 4);
  hipMalloc(&dk, k.size() * 4);
  hipMalloc(&dout, NC * 4);
  hipMalloc(&dc, 8);
  hipMemcpy(dx, x.data(), x.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dk, k.data(), k.size() * 4, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep)
      hipLaunchKernelGGL(walk, dim3(1), dim3(mode == 2 ? 1024 : 64), 0, 0, dx, dk, mode, dout, dc);
    hipDeviceSynchronize();
    float out[NC];
    long long cyc;
    hipMemcpy(out, dout, NC * 4, hipMemcpyDeviceToHost);
    hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
    int same = 0;
    for (int c = 0; c < NC; ++c) same += dr::f32_bits(out[c]) == dr::f32_bits(ref[c]);
    printf("%s: %lld cycles, %.1f per segment, %.2f per position; %d/%d columns bit-equal\n",
           mode == 0 ? "plain adds" : mode == 1 ? "rep_add, 16 columns per wave" : "rep_add, one column per wave", cyc, (double)cyc / NS, (double)cyc / pos, same, NC);
  }
  return 0;
}
