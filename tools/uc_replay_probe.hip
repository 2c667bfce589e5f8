// uc_replay_probe.hip -- standalone replay of the round-4 uncached-reuse
// failure: no torch, no library.  The sequence of
// tests/test_gpu_sharded.py -k xgmi under DR_IPC_RELEASE=1 as the r04
// diagnostic build logged it (profiles/r04_uc_reuse_xcd_views.log):
//   * groups of five uncached IPC buffers (hipExtMallocWithFlags(
//     hipDeviceMallocUncached); the sizes and free order of the log: inbox
//     keys / slots / counts / output / gradient per engine), each zero-filled
//     by a kernel + stream sync (dr_ipc_alloc), written by kernels spread over
//     every XCD (the peer-write engine's route / serve / pull), with ordinary
//     hipMalloc blocks (EV pools, torch segments) allocated between them,
//     then hipFree'd in the logged order;
//   * then 92 EV pools of 256 KiB (hipMalloc), each poisoned 0xFF by a fill
//     kernel, device-synchronised and read three ways: 64 blocks spread over
//     the XCDs (each records HW_REG_XCC_ID and counts words != 0xFFFFFFFF),
//     a D2H copy (SDMA), and the 64 blocks again after an agent-scope
//     acquire.  The r04 library run showed 4 of 92 pools with stale words
//     (per-XCD views disagreeing).
//   hipcc -O3 --offload-arch=gfx950 tools/uc_replay_probe.hip -o tools/uc_replay_probe
//   tools/uc_replay_probe [rounds] [control] [ipc]   (control: coarse hipMalloc for the IPC
//   buffers; ipc: export every buffer with hipIpcGetMemHandle, open it again in this same
//   process -- as the ranks-as-threads engines of test_gpu_sharded.py do for their peers --
//   write through that second mapping, close it before hipFree)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__);                \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

// uncached block sizes in the order the r04 log freed them
static const size_t kFree[] = {
    16384, 8192, 256, 524288, 524288, 32768, 16384, 256, 524288, 524288, 32768, 16384, 256,
    524288, 524288, 49152, 24576, 256, 524288, 524288, 49152, 24576, 256, 524288, 524288, 49152,
    24576, 256, 524288, 524288, 16384, 8192, 256, 524288, 524288, 32768, 16384, 256, 524288,
    524288, 32768, 16384, 256, 524288, 524288, 49152, 24576, 256, 524288, 524288, 49152, 24576,
    256, 524288, 524288, 49152, 24576, 256, 524288, 524288, 65536, 32768, 256, 2097152, 2097152,
    131072, 65536, 256, 2097152, 2097152, 131072, 65536, 256, 2097152, 2097152, 196608, 98304,
    256, 2097152, 2097152, 196608, 98304, 256, 2097152, 2097152, 196608, 98304, 256, 2097152,
    2097152, 131072, 65536, 256, 2097152, 2097152, 131072, 65536, 256, 2097152, 2097152, 16384,
    8192, 256, 524288, 524288, 32768, 16384, 256, 524288, 524288, 32768, 16384, 256, 524288,
    524288};

__global__ void fill_k(uint32_t* p, int64_t n, uint32_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// scattered writes from every block (the peer-write engine's row stores)
__global__ void scatter_k(uint32_t* p, int64_t n, uint32_t salt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t j = (i * 2654435761ll) % n;
  if (i < n) p[j] = (uint32_t)j ^ salt;
}

// res[3 b] = XCC id of block b, res[3 b + 1] = words != expect it saw
__global__ void view_k(const uint32_t* p, int64_t n, uint32_t expect, uint32_t* res, int acquire) {
  if (acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  uint32_t bad = 0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) bad += p[i] != expect;
  __shared__ uint32_t sb[256];
  sb[threadIdx.x] = bad;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < (int)blockDim.x; ++k) t += sb[k];
    res[3 * blockIdx.x] = (uint32_t)__builtin_amdgcn_s_getreg(0x1814) & 0xF;
    res[3 * blockIdx.x + 1] = t;
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 3;
  const int control = argc > 2 ? atoi(argv[2]) : 0;
  const int ipc = argc > 3 ? atoi(argv[3]) : 0;
  const size_t nfree = sizeof(kFree) / sizeof(kFree[0]);
  uint32_t* res;
  CK(hipMalloc(&res, 64 * 3 * sizeof(uint32_t)));
  int bad_pools = 0, pools = 0;
  for (int r = 0; r < rounds; ++r) {
    std::vector<void*> keep;
    // groups of 5 (one engine's IPC buffers): alloc, zero, use, then free
    for (size_t g = 0; g + 5 <= nfree; g += 5) {
      void* u[5];
      void* m[5];   // the buffer written by the engine: u, or its IPC mapping
      for (int k = 0; k < 5; ++k) {
        if (control)
          CK(hipMalloc(&u[k], kFree[g + k]));
        else
          CK(hipExtMallocWithFlags(&u[k], kFree[g + k], hipDeviceMallocUncached));
        hipLaunchKernelGGL(fill_k, dim3(64), dim3(256), 0, 0, (uint32_t*)u[k],
                           (int64_t)(kFree[g + k] / 4), 0u);
        CK(hipStreamSynchronize(nullptr));
        m[k] = u[k];
        if (ipc) {
          hipIpcMemHandle_t h;
          CK(hipIpcGetMemHandle(&h, u[k]));
          CK(hipIpcOpenMemHandle(&m[k], h, hipIpcMemLazyEnablePeerAccess));
        }
      }
      // the engine's cached neighbours: EV pools / torch segments
      void* c = nullptr;
      CK(hipMalloc(&c, (size_t)256 << 10));
      keep.push_back(c);
      for (int k = 0; k < 5; ++k) {
        const int64_t n = (int64_t)(kFree[g + k] / 4);
        hipLaunchKernelGGL(scatter_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0,
                           (uint32_t*)m[k], n, 0x1234u + (uint32_t)k);
      }
      CK(hipDeviceSynchronize());
      for (int k = 0; k < 5; ++k) {
        if (ipc) CK(hipIpcCloseMemHandle(m[k]));
        CK(hipFree(u[k]));
      }
    }
    // the EV pools of the next test: poison, sync, three views
    for (int pidx = 0; pidx < 92; ++pidx) {
      const size_t bytes = (size_t)256 << 10;
      const int64_t n = (int64_t)(bytes / 4);
      uint32_t* p = nullptr;
      CK(hipMalloc(&p, bytes));
      keep.push_back(p);
      hipLaunchKernelGGL(fill_k, dim3(256), dim3(256), 0, 0, p, n, 0xFFFFFFFFu);
      CK(hipDeviceSynchronize());
      hipLaunchKernelGGL(view_k, dim3(64), dim3(256), 0, 0, p, n, 0xFFFFFFFFu, res, 0);
      std::vector<uint32_t> h(64 * 3), h2(64 * 3), w((size_t)n);
      CK(hipMemcpy(h.data(), res, h.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(w.data(), p, bytes, hipMemcpyDeviceToHost));
      hipLaunchKernelGGL(view_k, dim3(64), dim3(256), 0, 0, p, n, 0xFFFFFFFFu, res, 1);
      CK(hipMemcpy(h2.data(), res, h2.size() * 4, hipMemcpyDeviceToHost));
      uint64_t d2h = 0, xb = 0, xb2 = 0;
      for (int64_t i = 0; i < n; ++i) d2h += w[(size_t)i] != 0xFFFFFFFFu;
      for (int b = 0; b < 64; ++b) {
        xb += h[3 * b + 1];
        xb2 += h2[3 * b + 1];
      }
      ++pools;
      if (d2h || xb || xb2) {
        ++bad_pools;
        printf("round %d pool %d %p: D2H stale %llu, per-XCD views:", r, pidx, (void*)p,
               (unsigned long long)d2h);
        for (int b = 0; b < 8; ++b) printf(" xcc%u:%u", h[3 * b], h[3 * b + 1]);
        printf("; after acquire %llu\n", (unsigned long long)xb2);
      }
    }
    for (void* p : keep) CK(hipFree(p));
    printf("round %d done: %d / %d pools stale so far\n", r, bad_pools, pools);
    fflush(stdout);
  }
  printf("{\"probe\":\"uc_replay\",\"control\":%d,\"ipc\":%d,\"rounds\":%d,\"pools\":%d,"
         "\"stale_pools\":%d}\n", control, ipc, rounds, pools, bad_pools);
  CK(hipFree(res));
  return 0;
}
