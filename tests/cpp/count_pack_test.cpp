// CPU check of the sharded-index count exchange's wire format (count_pack.h):
// every rank packs its saturated counts two per u32, the words are summed as
// u32 (what ncclSum does), and the unpacked sum must equal the per-base sum.
// Usage: count_pack_test RANKS MAX_COUNT N SEED  ->  prints "ok PACKED" or
// "mismatch PACKED i", PACKED = counts_pack16_ok(RANKS, MAX_COUNT).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../pacbio_amd/csrc/count_pack.h"

int main(int argc, char** argv) {
  if (argc < 5) return 2;
  const uint32_t R = (uint32_t)atoi(argv[1]), mc = (uint32_t)atoi(argv[2]);
  const uint64_t n = strtoull(argv[3], nullptr, 10);
  std::mt19937_64 rng(strtoull(argv[4], nullptr, 10));
  const uint32_t sat = mc + 1;
  std::vector<uint64_t> want(n, 0);
  const uint64_t nw = pbgpu::counts_packed_words(n);
  std::vector<uint32_t> wire(nw, 0), c(n);
  for (uint32_t r = 0; r < R; ++r) {
    for (uint64_t i = 0; i < n; ++i) {
      // mostly saturated counts: the worst case for a carry between the halves
      const uint64_t x = rng();
      c[i] = (x & 3) ? sat : (uint32_t)((x >> 8) % (sat + 1));
      want[i] += c[i];
    }
    for (uint64_t w = 0; w < nw; ++w) wire[w] += pbgpu::counts_pack16(c.data(), n, w);  // u32 ncclSum
  }
  std::vector<uint32_t> got(n + 1, 0xDEADBEEFu);
  for (uint64_t w = 0; w < nw; ++w) pbgpu::counts_unpack16(wire[w], got.data(), n, w);
  const bool ok16 = pbgpu::counts_pack16_ok(R, mc);
  if (got[n] != 0xDEADBEEFu) { printf("overrun %d\n", ok16); return 0; }
  for (uint64_t i = 0; i < n; ++i)
    if (got[i] != want[i]) { printf("mismatch %d %llu\n", ok16, (unsigned long long)i); return 0; }
  printf("ok %d\n", ok16);
  return 0;
}
