// count_pack.h -- the sharded-index count exchange's wire format (SURVEY.md
// 8(e)3): every shard saturates a k-mer's count at max_count + 1, and two of
// those counts travel as the 16-bit halves of one ncclUint32.  A sum over
// n_ranks shards stays below 2^16 in each half when
// n_ranks * (max_count + 1) < 65536, so ncclSum on the packed words never
// carries from the low half into the high one, and the all-reduce moves 2 B a
// read base instead of 4.  Outside that range the counts travel as plain u32.
// Header-only, host and device (the CPU test compiles it with g++).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define PBGPU_HD __host__ __device__ inline
#else
#define PBGPU_HD inline
#endif

namespace pbgpu {

PBGPU_HD bool counts_pack16_ok(uint32_t n_ranks, uint32_t max_count) {
  return (uint64_t)n_ranks * ((uint64_t)max_count + 1) < 65536u;
}
PBGPU_HD uint64_t counts_packed_words(uint64_t n) { return (n + 1) / 2; }
// word w of the packed form of c[0, n): c[2w] in the low half, c[2w + 1] (0 past n) in the high
PBGPU_HD uint32_t counts_pack16(const uint32_t* c, uint64_t n, uint64_t w) {
  const uint32_t lo = c[2 * w], hi = 2 * w + 1 < n ? c[2 * w + 1] : 0u;
  return (lo & 0xFFFFu) | (hi << 16);
}
PBGPU_HD void counts_unpack16(uint32_t v, uint32_t* c, uint64_t n, uint64_t w) {
  c[2 * w] = v & 0xFFFFu;
  if (2 * w + 1 < n) c[2 * w + 1] = v >> 16;
}

}  // namespace pbgpu
