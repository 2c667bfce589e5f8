// crc32c.hip -- host-side CRC-32C (Castagnoli) for the checkpoint writer /
// reader (deeprec_amd/checkpoint.py).  TensorBundle checksums every tensor's
// bytes and every SSTable block with crc32c (core/lib/hash/crc32c.h,
// core/util/tensor_bundle/tensor_bundle.cc:435-455, core/lib/io/
// table_builder.cc); EV values tensors reach hundreds of GB, so the checksum
// runs natively (SSE4.2 crc32 instructions, table fallback).
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "dr_common.h"

namespace {

struct Table {
  uint32_t t[256];
  Table() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82f63b78u : c >> 1;
      t[i] = c;
    }
  }
};

uint32_t crc_sw(uint32_t crc, const uint8_t* p, size_t n) {
  static const Table tab;  // thread-safe one-time init
  for (size_t i = 0; i < n; ++i) crc = tab.t[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return crc;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t crc_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc;
  while (n && ((uintptr_t)p & 7)) {
    c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
    --n;
  }
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  while (n--) c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
  return (uint32_t)c;
}
#endif

}  // namespace

// crc32c::Extend(init_crc, data, n) (core/lib/hash/crc32c.h): the
// un-inverted running value in, the finished value out.
extern "C" uint32_t dr_crc32c_extend(uint32_t init_crc, const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t crc = init_crc ^ 0xffffffffu;
#if defined(__x86_64__)
  if (__builtin_cpu_supports("sse4.2"))
    crc = crc_hw(crc, p, n);
  else
#endif
    crc = crc_sw(crc, p, n);
  return crc ^ 0xffffffffu;
}
