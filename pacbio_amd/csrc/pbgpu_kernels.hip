// pbgpu_kernels.hip -- MI355X (gfx950) kernels of the jf_aligner hot path.
//
//   index build : k_build_keys -> radix sort (hipcub) -> k_runs/k_occ_fill/k_headers
//   per batch   : k_seed   (one workgroup per read: 2-bit k-mers, SSR, toggle,
//                           hash probe, max-count filter, 99% threshold, hit count)
//                 k_group  (one workgroup per read: LDS hash of super-reads,
//                           two-pass enumeration -> (read, SR) chains)
//                 k_chain  (one wave per chain: LDS bitonic sort, order-exact
//                           LIS, least-squares fit, filters, --max-match)
//                 k_rec_*  (records grouped per read and sorted by (rs, re, ql))
//
// Every floating-point expression restates the reference's operation order;
// the file is compiled with -ffp-contract=off and the critical expressions
// use explicit __dadd_rn / __dmul_rn so that no FMA is ever formed.
#include <hip/hip_runtime.h>

#include <atomic>
#include <stdint.h>
#include <algorithm>
#include <cstdio>
#include <type_traits>
#include "pbgpu.h"
#include "pbgpu_internal.h"
#include "count_pack.h"

namespace pbgpu {

#define DEV __device__ __forceinline__

// Optional phase profiling of k_lis (build with -DPBGPU_PROF; tools/prof_lis.py):
// per-wave s_memtime deltas summed into g_prof.
#ifdef PBGPU_PROF
constexpr int PROF_SLOTS = 160;
__device__ unsigned long long g_prof[PROF_SLOTS];
#define PROF_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define PROF_ADD(slot, v) do { if (lane_id() == 0) atomicAdd(&g_prof[slot], (unsigned long long)(v)); } while (0)
#else
#define PROF_T(v)
#define PROF_ADD(slot, v)
#endif

// ------------------------------------------------------------------ utils
DEV uint64_t fmix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
  return k;
}
DEV uint64_t mer_mask(uint32_t k) { return k >= 32 ? ~0ull : ((1ull << (2 * k)) - 1); }
// reverse complement of an MSB-first k-mer code (word_reverse, mer_sa_imp.hpp:60-68)
DEV uint64_t revcomp(uint64_t m, uint32_t k) {
  uint64_t w = ~m;
  w = ((w >> 2) & 0x3333333333333333ULL) | ((w & 0x3333333333333333ULL) << 2);
  w = ((w >> 4) & 0x0F0F0F0F0F0F0F0FULL) | ((w & 0x0F0F0F0F0F0F0F0FULL) << 4);
  w = ((w >> 8) & 0x00FF00FF00FF00FFULL) | ((w & 0x00FF00FF00FF00FFULL) << 8);
  w = ((w >> 16) & 0x0000FFFF0000FFFFULL) | ((w & 0x0000FFFF0000FFFFULL) << 16);
  w = (w >> 32) | (w << 32);
  return w >> (64 - 2 * k);
}
// k-mer starting at text position x (MSB-first packed text, padded by 1 word)
DEV uint64_t text_kmer(const uint64_t* text, uint64_t x, uint32_t k) {
  const uint64_t w = x >> 5;
  const uint32_t sh = (uint32_t)(x & 31) * 2;
  uint64_t v = text[w];
  if (sh) v = (v << sh) | (text[w + 1] >> (64 - sh));
  return v >> (64 - 2 * k);
}
DEV int base_code(uint8_t c) {
  switch (c) {
  case 'A': case 'a': return 0;
  case 'C': case 'c': return 1;
  case 'G': case 'g': return 2;
  case 'T': case 't': return 3;
  default: return -1;
  }
}
// is_ssr (coarse_aligner.cc:8-15): two cyclic right rotations by one base
DEV bool is_ssr(uint64_t m, uint32_t k) {
  const uint32_t hs = 2 * (k - 1);
  uint64_t n1 = (m >> 2) | ((m & 3) << hs);
  uint64_t n2 = (n1 >> 2) | ((n1 & 3) << hs);
  return (n1 == m) | (n2 == m);
}
// Branch-free base decoding for the seeding loops: ACGT/acgt -> 0..3
// (((c >> 1) ^ (c >> 2)) & 3), and validity by an exact compare of the
// upper-cased byte (every other byte resets the k-mer, as base_code's -1).
DEV bool base_valid(uint8_t c) {
  const uint32_t u = c & 0xDFu;
  return (u == 'A') | (u == 'C') | (u == 'G') | (u == 'T');
}
DEV uint32_t base_code2(uint8_t c) { return ((c >> 1) ^ (c >> 2)) & 3u; }
DEV int lane_id() { return threadIdx.x & 63; }
DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
DEV uint64_t wave_min_u64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}
DEV uint64_t wave_sum_u64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide exclusive scan of one u32 per thread (BLOCK a multiple of 64).
template <int BLOCK>
DEV uint32_t block_excl_scan(uint32_t v, uint32_t* s_tmp, uint32_t& total) {
  constexpr int NW = BLOCK / 64;
  const int lane = lane_id(), w = threadIdx.x >> 6;
  uint32_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_tmp[w] = x;
  __syncthreads();
  uint32_t wbase = 0, tot = 0;
  for (int i = 0; i < NW; ++i) { uint32_t t = s_tmp[i]; if (i < w) wbase += t; tot += t; }
  __syncthreads();
  total = tot;
  return wbase + x - v;
}
template <int BLOCK>
DEV uint64_t block_sum_u64(uint64_t v, uint64_t* s_tmp) {
  constexpr int NW = BLOCK / 64;
  v = wave_sum_u64(v);
  if (lane_id() == 0) s_tmp[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
  for (int i = 0; i < NW; ++i) t += s_tmp[i];
  __syncthreads();
  return t;
}

// Bucketized probe: 64-byte bucket of 4 {key, payload} slots.
DEV bool table_lookup(const IndexView& ix, uint64_t key, uint64_t& payload, uint32_t& probes) {
  uint64_t b = fmix64(key) & ix.bucket_mask;
  for (;;) {
    ++probes;
    const ulonglong2* bk = ix.table + 4 * b;
    ulonglong2 s0 = bk[0], s1 = bk[1], s2 = bk[2], s3 = bk[3];
    if (s0.x == key) { payload = s0.y; return true; }
    if (s0.x == EMPTY_KEY) return false;
    if (s1.x == key) { payload = s1.y; return true; }
    if (s1.x == EMPTY_KEY) return false;
    if (s2.x == key) { payload = s2.y; return true; }
    if (s2.x == EMPTY_KEY) return false;
    if (s3.x == key) { payload = s3.y; return true; }
    if (s3.x == EMPTY_KEY) return false;
    b = (b + 1) & ix.bucket_mask;
  }
}

// Presence filter in front of the table: one 64-bit word per key, FILT_HASHES
// bits set in it (a register-blocked Bloom filter, 16 bits per key).  ~90% of
// a CLR read's k-mers are absent from the index; their 8-byte filter word sits
// in L2 / MALL (16 MB on C2) instead of a 64-byte HBM bucket probe.  No false
// negatives, so results do not depend on it.
constexpr int FILT_HASHES = 5;
DEV uint64_t filt_hash(uint64_t key) { return fmix64(key * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull); }
DEV uint64_t filt_bits(uint64_t h) {
  uint64_t m = 0;
#pragma unroll
  for (int i = 0; i < FILT_HASHES; ++i) m |= 1ull << ((h >> (6 * i)) & 63);
  return m;
}
DEV bool filt_test(const IndexView& ix, uint64_t key) {
  const uint64_t h = filt_hash(key);
  const uint64_t m = filt_bits(h);
  return (__ldg(ix.filt + (h >> ix.filt_shift)) & m) == m;
}

// ============================================================ index build
// Sort keys, one per text position x in [0, N), N = n - km + 1:
//   (canonical km-mer << 1 | orientation) << ebits | extension
// ebits = 0 for the coarse index (km = k: occurrences in descending x, the SA
// tie-break of mer_sa_imp.hpp:363).  The fine (-F) sub-index (km = fine_k < K
// = k) appends the K - km bases after the occurrence, zero-padded past n, and
// a "full" bit (x + K <= n): the SA order of a pattern shorter than max_size
// (sort_one_mer, mer_sa_imp.hpp:351-364: extension lexicographic, a truncated
// one first, then x descending).  Positions are enumerated in descending
// order so the stable radix sort keeps x descending among equal keys.
// Partitioned build (indexes too large to sort at once, e.g. C4's 10 Gbp):
// sel lists the enumeration indices i of one partition (ascending, so the
// order among equal keys is still x descending); key j of the output is
// position N - 1 - sel[j].  sel == nullptr: every position, Nsel == N.
__global__ void k_build_keys(IndexView ix, uint32_t km, uint32_t K, uint32_t ebits, uint64_t N, const uint64_t* sel,
                             uint64_t Nsel, uint64_t* keys, uint64_t* vals) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < Nsel; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = sel ? sel[j] : j;
    const uint64_t x = N - 1 - i;
    const uint64_t f = text_kmer(ix.text, x, km);
    const uint64_t r = revcomp(f, km);
    const uint64_t canon = f < r ? f : r;
    const uint64_t obit = f > r ? 1 : 0;
    // SR holding x: upper_bound(sr_start, x) - 1 (pos_iterator, superread_parser.hpp:110-140)
    uint32_t lo = 0, hi = ix.n_sr + 1;
    while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (ix.sr_start[m] <= x) lo = m + 1; else hi = m; }
    const uint32_t s = lo - 1;
    const bool cross = x + km > ix.sr_start[s + 1];
    uint64_t key = (canon << 1) | obit;
    if (ebits) {
      const uint64_t ext = K > km ? text_kmer(ix.text, x + km, K - km) : 0;  // text is zero past n
      key = (key << ebits) | (ext << 1) | (x + K <= ix.n ? 1u : 0u);
    }
    keys[j] = key;
    vals[j] = cross ? ~0ull : (((uint64_t)s << 32) | (uint32_t)(x - ix.sr_start[s] + 1));
  }
}

// partition of the canonical km-mer at enumeration index i (x = N - 1 - i): all
// occurrences of a km-mer fall in one partition, so its list stays contiguous
DEV uint32_t kmer_part(uint64_t canon, uint32_t P) { return (uint32_t)(((fmix64(canon) >> 32) * P) >> 32); }
__global__ void k_part_ids(IndexView ix, uint32_t km, uint64_t N, uint32_t P, uint8_t* pid,
                           unsigned long long* hist) {
  __shared__ unsigned long long s_h[256];
  for (uint32_t t = threadIdx.x; t < P; t += blockDim.x) s_h[t] = 0;
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = N - 1 - i;
    const uint64_t f = text_kmer(ix.text, x, km);
    const uint64_t r = revcomp(f, km);
    const uint32_t p = kmer_part(f < r ? f : r, P);
    pid[i] = (uint8_t)p;
    atomicAdd(&s_h[p], 1ull);
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < P; t += blockDim.x) if (s_h[t]) atomicAdd(&hist[t], s_h[t]);
}

// the table entries of a partition's k-mers (k_headers with kh != null), moved to
// the final occurrence array at base: payload += base << 24
__global__ void k_table_insert(const ulonglong2* kh, uint64_t U, uint64_t base, ulonglong2* table, uint64_t bucket_mask,
                               unsigned long long* filt, uint32_t filt_shift);

__global__ void k_runs(const uint64_t* keys, const uint64_t* uidx, uint64_t N, uint32_t sh, uint64_t* run_start) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const bool head = i == 0 || (keys[i] >> sh) != (keys[i - 1] >> sh);
    if (head) run_start[uidx[i] - 1] = i;
  }
}

__global__ void k_occ_fill(const uint64_t* vals, const uint64_t* uidx, const uint64_t* kpos, uint64_t N, uint64_t* occ) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t v = vals[i];
    if (v != ~0ull) occ[2 * uidx[i] + kpos[i]] = v;
  }
}

DEV void table_put(ulonglong2* table, uint64_t bucket_mask, uint64_t canon, uint64_t payload, unsigned long long* filt,
                   uint32_t filt_shift) {
  if (filt) {
    const uint64_t h = filt_hash(canon);
    atomicOr(filt + (h >> filt_shift), (unsigned long long)filt_bits(h));
  }
  uint64_t b = fmix64(canon) & bucket_mask;
  for (;;) {
    for (int sl = 0; sl < 4; ++sl) {
      unsigned long long* kp = (unsigned long long*)&table[4 * b + sl].x;
      const unsigned long long old = atomicCAS(kp, (unsigned long long)EMPTY_KEY, (unsigned long long)canon);
      if (old == EMPTY_KEY) { table[4 * b + sl].y = payload; return; }
    }
    b = (b + 1) & bucket_mask;
  }
}

__global__ void k_table_insert(const ulonglong2* kh, uint64_t U, uint64_t base, ulonglong2* table, uint64_t bucket_mask,
                               unsigned long long* filt, uint32_t filt_shift) {
  for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < U; u += (uint64_t)gridDim.x * blockDim.x) {
    const ulonglong2 e = kh[u];
    table_put(table, bucket_mask, e.x, e.y + (base << 24), filt, filt_shift);
  }
}

// kh != null (partitioned build): {canon, payload} per k-mer instead of the table insert
__global__ void k_headers(const uint64_t* keys, const uint64_t* kpos, const uint64_t* run_start, uint64_t U,
                          uint64_t* occ, ulonglong2* table, uint64_t bucket_mask, uint32_t k, uint32_t ebits,
                          unsigned long long* filt, uint32_t filt_shift, ulonglong2* kh) {
  for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < U; u += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s = run_start[u], e = run_start[u + 1];
    const uint64_t canon = keys[s] >> (ebits + 1);
    const bool pal = canon == revcomp(canon, k);
    uint64_t lo = s, hi = e;  // first index with orientation bit set
    while (lo < hi) { uint64_t m = (lo + hi) >> 1; if ((keys[m] >> ebits) & 1) hi = m; else lo = m + 1; }
    const uint64_t nA = kpos[lo] - kpos[s], nB = kpos[e] - kpos[lo];
    const uint64_t hb = 2 * u + kpos[s];
    const uint64_t count = (e - s) * (pal ? 2 : 1);
    const uint64_t cnt32 = count > 0xFFFFFFFFull ? 0xFFFFFFFFull : count;
    occ[hb] = cnt32 | ((uint64_t)pal << 32);
    occ[hb + 1] = nA | (nB << 32);
    const uint64_t payload = (hb << 24) | (count < SAT_COUNT ? count : SAT_COUNT);
    if (kh) kh[u] = make_ulonglong2(canon, payload);
    else table_put(table, bucket_mask, canon, payload, filt, filt_shift);
  }
}

// Unitig length of every name entry of the index (sr_uids), for kmers_info:
// ulen(id) = ul[id], unusable (INT32_MIN) for an invalid id or one past the table
// SrMeta of every super-read of the index (AlignParamsDev::sr_meta), from its text starts,
// name offsets and the resolved unitig lengths
__global__ void k_sr_meta(const uint64_t* sr_start, const uint32_t* sr_uoff, uint64_t n_sr, const int32_t* sr_ul,
                          SrMeta* out) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < n_sr; s += (uint64_t)gridDim.x * blockDim.x) {
    SrMeta m;
    m.ql = (uint32_t)(sr_start[s + 1] - sr_start[s]);
    m.u0 = sr_uoff[s];
    m.nsz = sr_uoff[s + 1] - m.u0;
#pragma unroll
    for (uint32_t i = 0; i < SR_META_UL; ++i) m.ul[i] = i < m.nsz ? sr_ul[m.u0 + i] : INT32_MIN;
    out[s] = m;
  }
}
void launch_sr_meta(const uint64_t* sr_start, const uint32_t* sr_uoff, uint64_t n_sr, const int32_t* sr_ul, SrMeta* out,
                    hipStream_t st) {
  if (n_sr) hipLaunchKernelGGL(k_sr_meta, dim3(1024), dim3(256), 0, st, sr_start, sr_uoff, n_sr, sr_ul, out);
}
__global__ void k_sr_ul(const uint32_t* ids, uint64_t n, const int32_t* ul, uint64_t n_ul, int32_t* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t id = ids[i];
    out[i] = (id == INVALID_UNITIG || id >= n_ul) ? INT32_MIN : ul[id];
  }
}

// ================================================================== seed
// One workgroup per read.  fetch_super_reads (coarse_aligner.cc:81-125).
// MODE (index sharded by super-read range):
//   SEED_WHOLE   the index holds every super-read: counts come from the table;
//   SEED_COUNTS  this shard's count of every looked-up k-mer, saturated at
//                max_count + 1, goes to gcount[read offset + position] (then
//                summed over the shards by the caller: RCCL all-reduce) -- a sum
//                of per-shard counts saturated at max_count + 1 decides every
//                use of the count (skip, histogram, threshold) exactly;
//   SEED_FINISH  the summed counts drive the filter and the 99% threshold, so
//                every shard keeps the same k-mers; hits come from this shard's
//                occurrence lists (a k-mer absent here points at the index's
//                empty header).
enum { SEED_WHOLE = 0, SEED_COUNTS = 1, SEED_FINISH = 2 };
template <int BLOCK, int PER, int MODE>
__global__ __launch_bounds__(BLOCK) void k_seed(IndexView ix, const uint8_t* __restrict__ seq,
                                                const uint64_t* __restrict__ roff, uint32_t n_reads,
                                                AlignParamsDev P, KRec* __restrict__ krec,
                                                uint32_t* __restrict__ n_kept_out, uint32_t* __restrict__ thr_out,
                                                uint64_t* __restrict__ nhits_out, unsigned long long* stats,
                                                uint32_t* __restrict__ gcount, uint64_t null_ptr) {
  constexpr int TILE = BLOCK * PER;
  constexpr int LOOK = 32;
  __shared__ uint8_t s_seq[TILE + LOOK];
  __shared__ uint32_t s_tmp[BLOCK / 64];
  __shared__ uint64_t s_tmp64[BLOCK / 64];
  __shared__ uint32_t s_hist[256];
  __shared__ uint32_t s_sel[2];
  const uint32_t r = blockIdx.x;
  if (r >= n_reads) return;
  const int tid = threadIdx.x;
  const uint64_t base = roff[r];
  const int64_t L = (int64_t)(roff[r + 1] - base);
  const uint32_t k = P.k;
  const uint64_t mask = mer_mask(k);
  const uint32_t hs = 2 * (k - 1);
  uint32_t cand_carry = 0, kept_carry = 0;
  uint64_t my_kmers = 0, my_probes = 0, my_fchecks = 0;

  for (int64_t t0 = 0; t0 < L; t0 += TILE) {
    for (int i = tid; i < TILE + LOOK; i += BLOCK) {
      const int64_t p = t0 - LOOK + i;
      s_seq[i] = (p >= 0 && p < L) ? seq[base + p] : (uint8_t)'N';
    }
    __syncthreads();
    const int64_t p0 = t0 + (int64_t)tid * PER;
    // history needed before p0: the k - 1 bases of the first k-mer, and 17 to tell a
    // run of <= 17 valid bases (the toggle) from a longer one; LOOK (32) bounds both
    const int64_t lb = k - 1 > 17 ? (int64_t)k - 1 : 17;
    const int64_t s = p0 - lb > 0 ? p0 - lb : 0;
    uint64_t m = 0, rm = 0;
    uint32_t rl = s > 0 ? 1000u : 0u;  // unknown history before s counts as a long valid run
    for (int64_t q = s; q < p0; ++q) {  // branch-free: an invalid base resets the run
      const uint8_t ch = s_seq[q - t0 + LOOK];
      const bool v = base_valid(ch);
      const uint64_t c = base_code2(ch);
      rl = v ? rl + 1 : 0u;
      m = v ? ((m << 2) | c) & mask : m;
      rm = v ? (rm >> 2) | ((3ull - c) << hs) : rm;
    }
    uint64_t mm[PER], rr[PER];
    uint32_t fl[PER];  // bit0 valid&!ssr (candidate for lookup), bit1 toggle candidate
    uint32_t ncand = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      // branch-free; positions past the read end hold 'N' in the tile
      const int64_t p = p0 + q;
      const uint8_t ch = s_seq[p - t0 + LOOK];
      const bool v = base_valid(ch);
      const uint64_t c = base_code2(ch);
      rl = v ? rl + 1 : 0u;
      m = v ? ((m << 2) | c) & mask : m;
      rm = v ? (rm >> 2) | ((3ull - c) << hs) : rm;
      const bool km = v & (rl >= k);
      my_kmers += km ? 1u : 0u;
      const bool cand = km & !is_ssr(m, k);
      const bool tog = cand & (rl <= 17u);  // coarse_aligner.cc:96-102
      fl[q] = (cand ? 1u : 0u) | (tog ? 2u : 0u);
      ncand += tog ? 1u : 0u;
      mm[q] = km ? m : 0; rr[q] = km ? rm : 0;
      (void)p;
    }
    // toggle: candidate number c (1-based, whole read) is processed iff c is odd
    uint32_t ctot;
    uint32_t cidx = cand_carry + block_excl_scan<BLOCK>(ncand, s_tmp, ctot);
    uint32_t nkept = 0;
    uint64_t kp_ptr[PER];
    uint32_t kp_cnt[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      bool go = fl[q] & 1;
      if (fl[q] & 2) { ++cidx; go = (cidx & 1) != 0; }
      fl[q] = 0;
      if (go) {
        const uint64_t canon = mm[q] < rr[q] ? mm[q] : rr[q];
        uint64_t payload = 0; uint32_t pr = 0;
        bool found = false;
        if (ix.filt) ++my_fchecks;
        if (!ix.filt || filt_test(ix, canon)) found = table_lookup(ix, canon, payload, pr);
        my_probes += pr;
        uint32_t cnt = 0;
        uint64_t ptr = null_ptr;
        if (found) {
          cnt = (uint32_t)(payload & SAT_COUNT);
          ptr = payload >> 24;
          if (cnt == SAT_COUNT) cnt = (uint32_t)(ix.occ[ptr] & 0xFFFFFFFFull);
        }
        const uint64_t gi = base + (uint64_t)(p0 + q);
        if (MODE == SEED_COUNTS) {
          const uint32_t sat = (uint32_t)P.max_count + 1u;
          gcount[gi] = cnt < sat ? cnt : sat;
        } else {
          if (MODE == SEED_FINISH) cnt = gcount[gi];
          if (cnt != 0 && cnt < (uint32_t)P.max_count) {
            fl[q] = 1; ++nkept;
            kp_ptr[q] = ptr | ((mm[q] < rr[q]) ? (1ull << 63) : 0ull);
            kp_cnt[q] = cnt;
          }
        }
      }
    }
    cand_carry += ctot;
    uint32_t ktot;
    uint32_t kidx = kept_carry + block_excl_scan<BLOCK>(nkept, s_tmp, ktot);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      if (fl[q]) {
        KRec kr;
        kr.pb_off = (int32_t)(p0 + q - (int64_t)k + 2);  // parser.offset<0>(), 1-based
        kr.count = kp_cnt[q];
        kr.occ_ptr = kp_ptr[q];
        krec[base + kidx] = kr;
        ++kidx;
      }
    }
    kept_carry += ktot;
    __syncthreads();
  }

  if (MODE == SEED_COUNTS) {
    const uint64_t kmers = block_sum_u64<BLOCK>(my_kmers, s_tmp64);
    const uint64_t probes = block_sum_u64<BLOCK>(my_probes, s_tmp64);
    const uint64_t fchecks = block_sum_u64<BLOCK>(my_fchecks, s_tmp64);
    if (tid == 0) {
      atomicAdd(&stats[ST_KMERS], (unsigned long long)kmers);
      atomicAdd(&stats[ST_PROBES], (unsigned long long)probes);
      atomicAdd(&stats[ST_FILTER], (unsigned long long)fchecks);
    }
    return;
  }
  // ---- 99% threshold (coarse_aligner.cc:117-125) via block radix select
  const uint32_t n_kept = kept_carry;
  const uint32_t sum_thresh = (uint32_t)round((double)n_kept * 0.99);
  uint32_t thr;
  if (n_kept > sum_thresh) {
    __threadfence_block();
    __syncthreads();
    uint32_t prefix = 0, pmask = 0, rank = sum_thresh;
    const uint32_t mc = (uint32_t)P.max_count;
    int top = mc <= 0xFFu ? 0 : mc <= 0xFFFFu ? 8 : mc <= 0xFFFFFFu ? 16 : 24;
    for (int shift = top; shift >= 0; shift -= 8) {
      for (int i = tid; i < 256; i += BLOCK) s_hist[i] = 0;
      __syncthreads();
      for (uint32_t i = tid; i < n_kept; i += BLOCK) {
        const uint32_t v = krec[base + i].count;
        if ((v & pmask) == prefix) atomicAdd(&s_hist[(v >> shift) & 255], 1u);
      }
      __syncthreads();
      {  // the digit whose bin holds the rank-th count: one block scan, not 256 serial steps
        static_assert(BLOCK == 256, "one histogram bin per thread");
        const uint32_t hv = s_hist[tid];
        uint32_t tot;
        const uint32_t ex = block_excl_scan<BLOCK>(hv, s_tmp, tot);
        if (ex <= rank && rank < ex + hv) { s_sel[0] = tid; s_sel[1] = rank - ex; }
      }
      __syncthreads();
      prefix |= s_sel[0] << shift; pmask |= 255u << shift; rank = s_sel[1];
      __syncthreads();
    }
    thr = prefix;
  } else {
    thr = (uint32_t)P.max_count + 1u;
  }
  // ---- hits of the kept k-mers with count <= threshold
  uint64_t my_hits = 0;
  for (uint32_t i = tid; i < n_kept; i += BLOCK) {
    const KRec kr = krec[base + i];
    if (kr.count > thr) continue;
    const uint64_t ptr = kr.occ_ptr & ~(1ull << 63);
    const uint64_t h0 = ix.occ[ptr], h1 = ix.occ[ptr + 1];
    const uint64_t nA = h1 & 0xFFFFFFFFull, nB = h1 >> 32;
    my_hits += ((h0 >> 32) & 1) ? 2 * nA : nA + nB;
  }
  const uint64_t hits = block_sum_u64<BLOCK>(my_hits, s_tmp64);
  const uint64_t kmers = block_sum_u64<BLOCK>(my_kmers, s_tmp64);
  const uint64_t probes = block_sum_u64<BLOCK>(my_probes, s_tmp64);
  const uint64_t fchecks = block_sum_u64<BLOCK>(my_fchecks, s_tmp64);
  if (tid == 0) {
    atomicAdd(&stats[ST_FILTER], (unsigned long long)fchecks);
    n_kept_out[r] = n_kept;
    thr_out[r] = thr;
    nhits_out[r] = hits;
    atomicAdd(&stats[ST_KMERS], (unsigned long long)kmers);
    atomicAdd(&stats[ST_PROBES], (unsigned long long)probes);
    atomicAdd(&stats[ST_KEPT], (unsigned long long)n_kept);
    atomicAdd(&stats[ST_HITS], (unsigned long long)hits);
  }
}

// ================================================================= group
// Workgroup barrier that orders LDS only: outstanding global loads (prefetched
// occurrences) stay in flight, where __syncthreads() would wait for them.
DEV void table_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// One workgroup (4 waves) per read: enumerate the read's hits exactly in the reference's
// append order (kept k-mers in read order; per k-mer occ(m) then occ(rm),
// each in descending text position == pos_iterator, superread_parser.hpp:
// 110-140), group them by super-read in an open-addressing table (LDS, or a
// global region for reads touching more super-reads than the LDS table
// holds), and scatter every hit to its (read, SR, strand) list with an
// order-preserving multisplit.  Each list comes out in exactly the
// reference's frags_pos order (coarse_aligner.cc:128-140) -- no sort needed.
// 4 waves share one read's table; reads touching many super-reads use a
// 16-wave block over the largest LDS table.
#ifndef PBGPU_GROUP_BLOCK
#define PBGPU_GROUP_BLOCK 256
#endif
#ifndef PBGPU_GROUP_BLOCK_BIG
#define PBGPU_GROUP_BLOCK_BIG 1024
#endif
constexpr uint32_t GROUP_BLOCK = PBGPU_GROUP_BLOCK, GROUP_BLOCK_BIG = PBGPU_GROUP_BLOCK_BIG;
#ifndef PBGPU_GROUP_U
#define PBGPU_GROUP_U 4
#endif
#ifndef PBGPU_GROUP_U_BIG
#define PBGPU_GROUP_U_BIG 4
#endif
constexpr int GROUP_U = PBGPU_GROUP_U, GROUP_U_BIG = PBGPU_GROUP_U_BIG;  // 64-hit windows per wave and step (their occurrence loads are in flight together)

#ifndef PBGPU_GROUP_MINW
#define PBGPU_GROUP_MINW 1
#endif
#ifndef PBGPU_GROUP_BUCKET
#define PBGPU_GROUP_BUCKET 1  // bucketed LDS-table probing (4 slots a 16-byte read); 0 = slot by slot
#endif
// MODE 0: a work item enumerates its read's hits from the index (k-mer records ->
// occurrence lists).  MODE 1 (split): one item per bucketed read (P0 partitions) enumerates
// them once and writes them to the read's P0 buckets (GroupOut::stage_*); no table, no
// chains.  MODE 2: a partition item of a bucketed read streams its bucket (for a refined
// item, partition q of Q = P0 f: bucket q / f, its entries filtered by partition).
template <bool GLOBAL_TABLE, uint32_t B, int MODE>
__global__ __launch_bounds__(B, B == GROUP_BLOCK ? PBGPU_GROUP_MINW : 1) void k_group(IndexView ix, const KRec* __restrict__ krec,
                                                       const uint64_t* __restrict__ roff, const uint32_t* __restrict__ n_kept,
                                                       const uint32_t* __restrict__ thr_in, const uint64_t* __restrict__ hit_off,
                                                       uint64_t node_base, uint32_t r0, const uint2* __restrict__ items,
                                                       uint32_t n_list, uint32_t hcap_log2, uint32_t* gtable, GroupOut O,
                                                       unsigned long long* stats) {
  extern __shared__ uint32_t s_dyn[];
  // static LDS kept under 8 KiB: with the 2048-slot table a 4-wave block then
  // needs < 32 KiB, and 5 blocks fit a CU instead of 4
  // per k-mer record of the current group: {fwd list count, pb offset} and the
  // occurrence addresses {fwd list, bwd list - fwd count}, read together by locate()
  __shared__ uint32_t s_off[B], s_scan[B / 64];
  __shared__ uint2 s_np[B];
  __shared__ ulonglong2 s_ptr[B];
  __shared__ uint32_t s_flag, s_used, s_cbase, s_pbase;
  if (blockIdx.x >= n_list) return;
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = tid >> 6;
  constexpr uint32_t NW = B / 64;
  constexpr int GU = B == GROUP_BLOCK ? GROUP_U : GROUP_U_BIG;  // windows per wave and step
  // work item: read r, hash partition `part` of P of its super-reads (group_item)
  const uint2 item = items ? items[blockIdx.x] : make_uint2(r0 + blockIdx.x, 1u << 16);
  const uint32_t r = item.x, part = item.y & 0xFFFFu, P = item.y >> 16;
  const uint32_t hcap = 1u << hcap_log2;
  // table: key (sr + 1, 0 = empty), fwd count/cursor, bwd count/cursor
  uint32_t* tkey = GLOBAL_TABLE ? gtable + (uint64_t)blockIdx.x * (3u * hcap) : s_dyn;
  uint32_t* tcf = tkey + hcap;
  uint32_t* tcb = tcf + hcap;
  const uint64_t kbase = roff[r];
  const uint64_t hbase = hit_off[r] - node_base;
  // MODE 2: the item's bucket [b_lo, b_lo + nk) of the read's staged hits
  uint32_t b_lo = 0;
  uint32_t nk = n_kept[r];
  if constexpr (MODE == 2) {
    const uint2 bm = O.bmeta[r];
    const uint32_t p0 = part / (P / bm.y);
    b_lo = O.boff[bm.x + p0];
    nk = O.boff[bm.x + p0 + 1] - b_lo;
  }
  const uint32_t thr = thr_in[r];
  // the group loop's step: k-mer records (MODE 0 / 1), or staged hits (MODE 2: 16 windows a wave)
  constexpr uint32_t GSTEP = MODE == 2 ? B * 16 : B;
#ifndef PBGPU_GROUP_BIG_FILL8
#define PBGPU_GROUP_BIG_FILL8 6  // the LDS tables' fill limit in eighths (the 8192-slot tier's below)
#endif
  const uint32_t used_limit = (B == GROUP_BLOCK || GLOBAL_TABLE) ? hcap - hcap / 4 : hcap / 8 * PBGPU_GROUP_BIG_FILL8;
  // Reads touching many super-reads are grouped over P hash partitions of the
  // super-read ids, one block a partition (each scans the read's k-mers and keeps
  // its partition's super-reads); a partition's lists go to the read's next free
  // hit range (an atomic cursor per read, O.rcur), so every list is still
  // contiguous and in reference order.  (Round 4 ran a read's partitions one
  // after the other in one block: with a sub-batch's few hundred long reads
  // the longest read's block was the launch.)
  uint32_t read_chains = 0, part_hits = 0;
  uint32_t g_stop = nk;  // pass 0 over the k-mers [0, g_stop) when the table overflowed
  uint32_t p0x = 0;  // PBGPU_EXP_P0_NOTABLE: keeps the loads live
  auto part_of = [&](uint32_t sr) -> uint32_t {
    return P == 1 ? 0u : (uint32_t)(((uint64_t)(sr * 0x85EBCA77u) * P) >> 32);
  };
#ifdef PBGPU_PROF
  uint64_t pr_setup[2] = {0, 0}, pr_steps[2] = {0, 0}, pr_compact = 0;
  const uint64_t pr_t0 = __builtin_amdgcn_s_memtime();
#endif
  {
  for (uint32_t i = tid; i < hcap; i += B) { tkey[i] = 0; tcf[i] = 0; tcb[i] = 0; }
  if (tid == 0) { s_flag = 0; s_used = 0; }
  if (GLOBAL_TABLE) __threadfence_block();
  __syncthreads();

#ifdef PBGPU_EXP_SKIP_PASS1  // experiment (with PBGPU_EXP_GROUP_ONLY): pass 0 alone
  constexpr int n_pass = 1;
#else
  constexpr int n_pass = 2;
#endif
  for (int pass_rt = 0; pass_rt < n_pass; ++pass_rt) {
    // the group loop, compiled once per pass: with a run-time pass the stores of
    // pass 1 sit behind a branch, and the compiler then cannot count the loads in
    // flight and waits for all of them
    auto groups = [&](auto pass_c) {
    constexpr int pass = decltype(pass_c)::value;
    for (uint32_t g0 = 0; g0 < nk; g0 += GSTEP) {
      if (s_flag) { g_stop = g0; break; }  // uniform (written before the last barrier)
#ifdef PBGPU_PROF
      const uint64_t pr_a = __builtin_amdgcn_s_memtime();
#endif
      const uint32_t i = g0 + tid;
      uint32_t nf = 0, nb = 0;
      int32_t pbv = 0;
      if (MODE != 2 && i < nk) {
        const KRec kr = krec[kbase + i];
        if (kr.count <= thr) {
          const uint64_t ptr = kr.occ_ptr & ~(1ull << 63);
          const bool canon = kr.occ_ptr >> 63;
          const uint64_t h0 = ix.occ[ptr], h1 = ix.occ[ptr + 1];
          const uint32_t nA = (uint32_t)(h1 & 0xFFFFFFFFull), nB = (uint32_t)(h1 >> 32);
          const uint64_t A = ptr + 2, Bp = ptr + 2 + nA;
          // occ(m) -> fwd list (+off), occ(rm) -> bwd list (-off)    
          uint64_t pf, pbk;
          if ((h0 >> 32) & 1) { nf = nb = nA; pf = A; pbk = A; }
          else if (canon) { nf = nA; pf = A; nb = nB; pbk = Bp; }
          else { nf = nB; pf = Bp; nb = nA; pbk = A; }
          s_ptr[tid] = make_ulonglong2(pf, pbk - nf);
          pbv = kr.pb_off;
        }
      }
      uint32_t total;
      if constexpr (MODE == 2) {
        total = nk - g0 < GSTEP ? nk - g0 : GSTEP;
      } else {
        s_np[tid] = make_uint2(nf, (uint32_t)pbv);
        s_off[tid] = block_excl_scan<B>(nf + nb, s_scan, total);
        __syncthreads();
      }
#ifdef PBGPU_PROF
      const uint64_t pr_b = __builtin_amdgcn_s_memtime();
      pr_setup[pass] += pr_b - pr_a;
#endif
      // ---- the group's hits in 64-hit windows: a wave takes GU consecutive
      // windows per step, the waves of a step in order (pass 1 takes its cursors
      // wave by wave, so the step's hits are placed in enumeration order).  Lane l
      // of the window at h0 holds hit h0 + l; its k-mer record is the last one
      // starting at or before it (a fixed-depth search; k-mers without hits tie
      // with the next start and are skipped, as the reference's enumeration does).
      // Measured against a ballot walk over record starts held in registers
      // (one LDS read per 64 records instead of 8 per hit): the walk's readlane
      // chain was slower (pass 0 7.7 vs 6.9 ms, 25k C2 reads).
      const uint32_t lane = tid & 63;
      const uint32_t n_win = (total + 63) >> 6;
      // pass 0's super-read ids: the packed copy when the index has one, else the high
      // words of the entries (a pointer and stride, not a branch around the load)
      const uint32_t* sr_base = ix.occ_sr ? ix.occ_sr : reinterpret_cast<const uint32_t*>(ix.occ) + 1;
      const uint64_t sr_stride = ix.occ_sr ? 1 : 2;
      // locate + load of the wave's GU windows of step ws, one step ahead of
      // their use, so the occurrence loads overlap the table work of the step before
      auto fetch = [&](uint32_t ws, uint64_t (&e_o)[GU], int32_t (&pb_o)[GU], bool (&fwd_o)[GU],
                       bool (&val_o)[GU]) {
#pragma unroll
        for (int u = 0; u < GU; ++u) {
          const uint32_t h = ((ws + wave * GU + (uint32_t)u) << 6) + lane;
          if constexpr (MODE == 2) {
            // a staged hit (the bucket's entries past the group's end reload its first)
            const bool valid = h < total;
            const uint64_t at = hbase + b_lo + g0 + (valid ? h : 0u);
            const uint32_t w = O.stage_sr[at];
            val_o[u] = valid;
            fwd_o[u] = (w >> 31) == 0;
            if constexpr (pass == 0) {
              e_o[u] = (uint64_t)(w & 0x7FFFFFFFu) << 32;
              pb_o[u] = 0;
            } else {
              const int2 x = O.stage_x[at];
              e_o[u] = ((uint64_t)(w & 0x7FFFFFFFu) << 32) | (uint32_t)x.y;
              pb_o[u] = x.x;
            }
            continue;
          }
          // no branch around the load (windows past the group's end load occ[0]): the
          // compiler counts the loads in flight only when every path issues them
          uint32_t lo = 0;  // s_off[0] = 0: fixed depth, branch-free
#pragma unroll
          for (uint32_t stp = B / 2; stp >= 1; stp >>= 1) lo = s_off[lo + stp] <= h ? lo + stp : lo;
          const uint32_t local = h - s_off[lo];
          const uint2 np = s_np[lo];
          const ulonglong2 pp = s_ptr[lo];
          const bool valid = h < total;
          const bool fwd = local < np.x;
          fwd_o[u] = fwd;
          pb_o[u] = (int32_t)np.y;
          val_o[u] = valid;
          const uint64_t at = valid ? (fwd ? pp.x : pp.y) + local : 0;
          // pass 0 needs the super-read id alone: a 4-byte load of the high word (an
          // 8-byte one leaves a dead half whose register the compiler reuses, which
          // again drains the loads in flight)
          if constexpr (pass == 0) e_o[u] = (uint64_t)sr_base[sr_stride * at] << 32;
          else e_o[u] = ix.occ[at];
        }
      };
      // the hits of step ws from register set e_q (loaded one step earlier)
      auto process = [&](const uint64_t (&e_q)[GU], const int32_t (&pb_q)[GU],
                         const bool (&fwd_q)[GU], const bool (&val_q)[GU]) {
        uint32_t sr_q[GU], slot_q[GU];
        int32_t so_q[GU], pbx_q[GU];
        bool mine_q[GU], fwdx_q[GU];
#pragma unroll
        for (int u = 0; u < GU; ++u) {
          sr_q[u] = (uint32_t)(e_q[u] >> 32);
          so_q[u] = (int32_t)(uint32_t)(e_q[u] & 0xFFFFFFFFull);
          slot_q[u] = (sr_q[u] * 0x9E3779B1u) >> (32 - hcap_log2);
          mine_q[u] = val_q[u] && part_of(sr_q[u]) == part;
          pbx_q[u] = pb_q[u];
          fwdx_q[u] = fwd_q[u];
        }
        if constexpr (MODE == 1) {
          // split: every hit to its partition's bucket -- pass 0 counts (tkey[p]), pass 1
          // takes the bucket cursor (tcf[p]) in wave turn order, as pass 1 below does
          if constexpr (pass == 0) {
#pragma unroll
            for (int u = 0; u < GU; ++u)
              if (val_q[u]) atomicAdd(&tkey[part_of(sr_q[u])], 1u);
          } else {
            uint32_t pos_q[GU];
#pragma unroll
            for (int u = 0; u < GU; ++u) pos_q[u] = 0;
            for (uint32_t w = 0; w < NW; ++w) {
              if (wave == w) {
#pragma unroll
                for (int u = 0; u < GU; ++u)
                  if (val_q[u]) pos_q[u] = atomicAdd(&tcf[part_of(sr_q[u])], 1u);
              }
              table_barrier();
            }
            uint32_t* const sink32 = reinterpret_cast<uint32_t*>(O.sink);
#pragma unroll
            for (int u = 0; u < GU; ++u) {
              (val_q[u] ? O.stage_sr[hbase + pos_q[u]] : sink32[(blockIdx.x + wave) & (GROUP_SINKS - 1)]) =
                  sr_q[u] | (fwdx_q[u] ? 0u : 0x80000000u);
              (val_q[u] ? O.stage_x[hbase + pos_q[u]] : O.sink[(blockIdx.x + wave) & (GROUP_SINKS - 1)]) =
                  make_int2(pbx_q[u], so_q[u]);
            }
          }
          return;
        }
        // The first table probe of every window is issued together (one LDS round trip
        // for the step), then the rare collisions are walked one window at a time.  A
        // wave's LDS operations execute in order, so a later window of a lane sees
        // what an earlier one inserted.
        uint32_t first[GU];
#ifdef PBGPU_EXP_P0_NOTABLE  // experiment (with GROUP_ONLY + SKIP_PASS1): pass 0's loads without the table
        if constexpr (pass == 0) {
#pragma unroll
          for (int u = 0; u < GU; ++u) p0x ^= mine_q[u] ? sr_q[u] : 0u;
          return;
        }
#endif
#ifdef PBGPU_PROF
        const uint64_t gp_t0 = __builtin_amdgcn_s_memtime();
#endif
#if PBGPU_GROUP_BUCKET
        // Bucketed probing (LDS tables): a key lives in the first bucket of 4 slots, from its
        // home bucket on, that holds it or had room when it was inserted; one 16-byte LDS read
        // tests 4 slots.  Every window's home bucket is read together; a lane then inserts
        // into its bucket's first empty slot by compare-and-swap (re-reading the bucket when
        // another key took that slot) or walks on to the next bucket.  (Round 4's linear
        // probing walked slot by slot, one LDS round trip each, the wave waiting for its
        // longest walk; on C4r-shaped reads the table work was ~38 of the 43 ms of pass 0.)
        uint4 fb_q[GU];
#pragma unroll
        for (int u = 0; u < GU; ++u) {
          fb_q[u] = make_uint4(0u, 0u, 0u, 0u);
          if (mine_q[u] && !GLOBAL_TABLE) fb_q[u] = *reinterpret_cast<const uint4*>(&tkey[slot_q[u] & ~3u]);
        }
        if (!GLOBAL_TABLE) {
#pragma unroll
          for (int u = 0; u < GU; ++u) {
            if (!mine_q[u]) continue;
            const uint32_t key = sr_q[u] + 1;
            uint32_t b = slot_q[u] & ~3u, slot = 0;
            uint4 kk = fb_q[u];
            bool ok = true;
            for (uint32_t walk = 0;; ++walk) {
              const int pos = kk.x == key ? 0 : kk.y == key ? 1 : kk.z == key ? 2 : kk.w == key ? 3 : -1;
              if (pos >= 0) { slot = b + (uint32_t)pos; break; }
              if (pass == 1) {  // (present: pass 0 inserted every key of the partition)
                b = (b + 4) & (hcap - 1);
                kk = *reinterpret_cast<const uint4*>(&tkey[b]);
                continue;
              }
              const int e = kk.x == 0 ? 0 : kk.y == 0 ? 1 : kk.z == 0 ? 2 : kk.w == 0 ? 3 : -1;
              if (e < 0) {
                if (walk >= 8 && (walk >= hcap / 4 || __hip_atomic_load(&s_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) {
                  s_flag = 1; ok = false; break;
                }
                b = (b + 4) & (hcap - 1);
                kk = *reinterpret_cast<const uint4*>(&tkey[b]);
                continue;
              }
              const uint32_t old = atomicCAS(&tkey[b + (uint32_t)e], 0u, key);
              if (old == 0) {
                slot = b + (uint32_t)e;
                if (atomicAdd(&s_used, 1u) >= used_limit) { s_flag = 1; ok = false; }
                break;
              }
              if (old == key) { slot = b + (uint32_t)e; break; }
              kk = *reinterpret_cast<const uint4*>(&tkey[b]);  // another key took it: look again
            }
            if (pass == 0) { if (ok) atomicAdd(fwdx_q[u] ? &tcf[slot] : &tcb[slot], 1u); }
            else slot_q[u] = slot;
          }
        }
#endif
#pragma unroll
        for (int u = 0; u < GU; ++u) {
          first[u] = 0;
          if (mine_q[u] && (GLOBAL_TABLE || !PBGPU_GROUP_BUCKET))
            first[u] = pass == 0 ? atomicCAS(&tkey[slot_q[u]], 0u, sr_q[u] + 1) : tkey[slot_q[u]];
        }
#ifdef PBGPU_PROF
        __builtin_amdgcn_s_waitcnt(0xc07f);
        const uint64_t gp_t1 = __builtin_amdgcn_s_memtime();
        uint32_t gp_mine = 0, gp_walk = 0;
#pragma unroll
        for (int u = 0; u < GU; ++u) {
          gp_mine += mine_q[u];
          gp_walk += __ballot(mine_q[u] && first[u] != sr_q[u] + 1 && !(pass == 0 && first[u] == 0)) != 0;
        }
#endif
#pragma unroll
        for (int u = 0; u < GU; ++u) {
          if (!mine_q[u] || (!GLOBAL_TABLE && PBGPU_GROUP_BUCKET)) continue;
          const uint32_t key = sr_q[u] + 1;
          uint32_t slot = slot_q[u], old = first[u];
          if (pass == 0) {
            // order-free: distinct super-reads and per-strand list lengths
            // Once the table is over its fill limit the read is abandoned (it resumes in
            // a larger tier), but the rest of this k-mer group still runs and may fill
            // the table: long probe sequences give up once the flag is set (or after
            // hcap probes), so a full table can never trap a thread.
            bool ok = true;
            if (old == 0) {
              if (atomicAdd(&s_used, 1u) >= used_limit) { s_flag = 1; ok = false; }
            } else if (old != key) {
              for (uint32_t probe = 1;; ++probe) {
                slot = (slot + 1) & (hcap - 1);
                if (probe >= 8 && (probe == hcap || __hip_atomic_load(&s_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) {
                  s_flag = 1; ok = false; break;
                }
                old = atomicCAS(&tkey[slot], 0u, key);
                if (old == 0) { if (atomicAdd(&s_used, 1u) >= used_limit) { s_flag = 1; ok = false; } break; }
                if (old == key) break;
              }
            }
            if (ok) atomicAdd(fwdx_q[u] ? &tcf[slot] : &tcb[slot], 1u);
          } else {
            while (old != key) { slot = (slot + 1) & (hcap - 1); old = tkey[slot]; }
            slot_q[u] = slot;
          }
        }
#ifdef PBGPU_PROF
        __builtin_amdgcn_s_waitcnt(0xc07f);
        if (B == GROUP_BLOCK_BIG && !GLOBAL_TABLE) {  // slots 112..118: the 8192-slot tier's table work
          const uint64_t gp_t2 = __builtin_amdgcn_s_memtime();
          PROF_ADD(112 + 3 * pass, gp_t1 - gp_t0);  // first probes
          PROF_ADD(113 + 3 * pass, gp_t2 - gp_t1);  // collision walks + count atomics (pass 0)
          PROF_ADD(114 + 3 * pass, gp_walk);        // windows with a collision walk
          for (int o = 32; o > 0; o >>= 1) gp_mine += (uint32_t)__shfl_xor((int)gp_mine, o, 64);
          if (pass == 0) PROF_ADD(118, gp_mine);
        }
#endif
        if constexpr (pass == 1) {
          // Scatter: each hit takes the next slot of its (super-read, strand) list.  The
          // waves take their cursors in wave order (one barrier each) and a wave its
          // windows in order, so a list's run inside this step is out of order only
          // where the LDS unit does not serve one instruction's same-address atomics in
          // lane order; the consumers restore the reference order (pb offset ascending,
          // then |sr offset| descending) with a transposition pass bounded by the run
          // lengths (k_lis_w, k_strand_order, k_order_tiny).  The turn barriers order
          // the table's memory only (LDS; the HBM table's atomics return before them),
          // so the next step's occurrence loads stay in flight across them.
          uint32_t pos_q[GU];
#pragma unroll
          for (int u = 0; u < GU; ++u) pos_q[u] = 0;
#ifdef PBGPU_EXP_GROUP_NOTURN  // experiment (with PBGPU_EXP_GROUP_ONLY): cursors in any order, no turn barriers
          for (uint32_t w = wave; w == wave; ++w) {
#else
          for (uint32_t w = 0; w < NW; ++w) {
#endif
            if (wave == w) {
#pragma unroll
              for (int u = 0; u < GU; ++u)
                if (mine_q[u]) pos_q[u] = atomicAdd(fwdx_q[u] ? &tcf[slot_q[u]] : &tcb[slot_q[u]], 1u);
            }
#ifndef PBGPU_EXP_GROUP_NOTURN
            if (GLOBAL_TABLE) __syncthreads();
            else table_barrier();
#endif
          }
          // every lane stores (lanes without a hit to the sink entry), for the same reason
#ifndef PBGPU_EXP_GROUP_NOSTORE  // experiment (with PBGPU_EXP_GROUP_ONLY): no list stores
#pragma unroll
          for (int u = 0; u < GU; ++u)
            (mine_q[u] ? O.X[hbase + pos_q[u]] : O.sink[(blockIdx.x + wave) & (GROUP_SINKS - 1)]) =
                make_int2(pbx_q[u], fwdx_q[u] ? so_q[u] : -so_q[u]);
#else
          if (pos_q[0] == 0xFFFFFFFFu) O.X[0] = make_int2(pbx_q[0], so_q[0]);
#endif
        }
      };
      // Two register sets, each loaded in place one step ahead of its use: with one
      // set the compiler copies the new loads into it at the loop's back edge and
      // waits there for them and for the step's stores.
      uint64_t eA[GU], eB[GU];
      int32_t pbA[GU], pbB[GU];
      bool fwdA[GU], fwdB[GU], valA[GU], valB[GU];
      constexpr uint32_t S = NW * GU;  // windows per block step
      fetch(0, eA, pbA, fwdA, valA);
      for (uint32_t ws = 0; ws < n_win; ws += 2 * S) {  // block-uniform trip count
        fetch(ws + S, eB, pbB, fwdB, valB);
        process(eA, pbA, fwdA, valA);
        if (ws + S >= n_win) break;  // block-uniform
        fetch(ws + 2 * S, eA, pbA, fwdA, valA);
        process(eB, pbB, fwdB, valB);
      }
      __syncthreads();
#ifdef PBGPU_PROF
      pr_steps[pass] += __builtin_amdgcn_s_memtime() - pr_b;
#endif
    }
    };
    const int pass = pass_rt;
    if (pass == 0) groups(std::integral_constant<int, 0>{});
    else groups(std::integral_constant<int, 1>{});
    if (MODE == 1 && pass == 0) {
      // the buckets: an exclusive scan of the P partition counts (<= 4096, hcap), written as
      // the read's bucket offsets and kept as pass 1's cursors
      const uint32_t per = (P + B - 1) / B;
      uint32_t sum = 0;
      for (uint32_t j = 0; j < per; ++j) {
        const uint32_t pj = tid * per + j;
        sum += pj < P ? tkey[pj] : 0u;
      }
      uint32_t tot;
      uint32_t b0 = block_excl_scan<B>(sum, s_scan, tot);
      const uint32_t ob = O.bmeta[r].x;
      for (uint32_t j = 0; j < per; ++j) {
        const uint32_t pj = tid * per + j;
        if (pj < P) {
          O.boff[ob + pj] = b0;
          tcf[pj] = b0;
          b0 += tkey[pj];
        }
      }
      if (tid == 0) O.boff[ob + P] = tot;
      __syncthreads();
      continue;
    }
    if (MODE == 1) break;
    if (pass == 0) {
#ifdef PBGPU_PROF
      const uint64_t pr_c = __builtin_amdgcn_s_memtime();
#endif
      if (s_flag) {  // table too full: the item goes again, split or with a larger table
        if (tid == 0) {
          const uint32_t o = atomicAdd(O.n_overflow, 1u);
          // (an item overflows once a launch and the list holds every item of it: the
          // guard never drops one; the host checks the count against the cap)
          if (o < O.overflow_cap) {
          O.overflow_items[o] = item;
          // the table filled over the first g_stop k-mers of nk: nk / g_stop estimates how much
          // larger the item is (the host splits it that many ways; too few only costs a round)
          const uint32_t grow = g_stop ? (nk + g_stop - 1) / g_stop : nk;
          O.overflow_grow[o] = (grow < 0xFFFFFFu ? grow : 0xFFFFFFu) | (hcap_log2 << 24);  // | the table it filled
          }
        }
        return;
      }
      // chain descriptors, slot order; cursors become read-local list starts
      const uint32_t per = hcap / B;
      uint32_t sum = 0, nn = 0;
      for (uint32_t j = 0; j < per; ++j) {
        const uint32_t sl = tid * per + j;
        if (tkey[sl]) { sum += tcf[sl] + tcb[sl]; ++nn; }
      }
      uint32_t tsum, tn;
      const uint32_t esum = block_excl_scan<B>(sum, s_scan, tsum);
      part_hits = tsum;
      const uint32_t enn = block_excl_scan<B>(nn, s_scan, tn);
      read_chains += tn;
      if (tid == 0) {
        s_cbase = atomicAdd(O.chain_count, tn);
        s_pbase = P == 1 ? 0u : atomicAdd(&O.rcur[r], tsum);
        atomicAdd(&stats[ST_CHAINS], (unsigned long long)tn);
      }
      __syncthreads();
      uint32_t b0 = s_pbase + esum, ci = s_cbase + enn;
      for (uint32_t j = 0; j < per; ++j) {
        const uint32_t sl = tid * per + j;
        if (!tkey[sl]) continue;
        const uint32_t cf = tcf[sl], cb = tcb[sl];
        if (ci < O.chain_cap) {
          ChainDesc d;
          d.read = r; d.sr = tkey[sl] - 1; d.nf = cf; d.nb = cb; d.hit_base = hbase + b0;
          O.chains[ci] = d;
        }
        ++ci;
        tcf[sl] = b0;        // fwd cursor (read-local)
        tcb[sl] = b0 + cf;   // bwd cursor
        b0 += cf + cb;
      }
      if (GLOBAL_TABLE) __threadfence_block();
      __syncthreads();
#ifdef PBGPU_PROF
      pr_compact += __builtin_amdgcn_s_memtime() - pr_c;
#endif
    }
  }
  }  // the partition
  if (p0x == 0x9E3779B9u) O.sink[0] = make_int2((int)p0x, 0);  // practically never
  if (MODE == 0 && !GLOBAL_TABLE && B == GROUP_BLOCK && tid == 0) {  // per-launch algorithmic counters (bench roofline)
    atomicAdd(&stats[ST_G0_KEPT], (unsigned long long)nk);
    atomicAdd(&stats[ST_G0_HITS], (unsigned long long)part_hits);
    atomicAdd(&stats[ST_G0_CHAINS], (unsigned long long)read_chains);
  }
#ifdef PBGPU_PROF
  if (tid == 0 && !GLOBAL_TABLE) {
    const int sb = B == GROUP_BLOCK ? 8 : 14;
    atomicAdd(&g_prof[sb + 0], (unsigned long long)pr_setup[0] + pr_setup[1]);
    atomicAdd(&g_prof[sb + 1], (unsigned long long)pr_steps[0]);
    atomicAdd(&g_prof[sb + 2], (unsigned long long)pr_steps[1]);
    atomicAdd(&g_prof[sb + 3], (unsigned long long)pr_compact);
    atomicAdd(&g_prof[sb + 4], (unsigned long long)(__builtin_amdgcn_s_memtime() - pr_t0));
    atomicAdd(&g_prof[sb + 5], 1ull);
  }
#endif
}

// Work ordering for the lane-per-item kernels: items by descending length
// class so the lanes of a wave get items of nearly equal length (exact below
// 128, 16 classes per octave above).
constexpr uint32_t NLB = 528;
DEV uint32_t len_bucket(uint32_t n) {
  if (n < 128) return n;
  const uint32_t l = 31u - (uint32_t)__clz(n);
  return 128u + 16u * (l - 7u) + ((n >> (l - 4u)) & 15u);
}
struct StrandLen {  // item = chain << 1 | strand (0 fwd, 1 bwd)
  using Info = uint2;
  const uint32_t* slen;
  const ChainDesc* chains;  // (info(): the strand's hit range, for the permuted {base, n} array)
  DEV uint32_t operator()(uint32_t i) const { return slen[i]; }
  DEV uint2 info(uint32_t i, uint32_t n) const {
    const ChainDesc d = chains[i >> 1];
    return make_uint2((uint32_t)(d.hit_base + ((i & 1) ? d.nf : 0)), n);
  }
};
struct ChainLisLen {  // item = chain; the longer of its two lis
  using Info = uint2;
  const uint32_t* lisl;
  DEV uint32_t operator()(uint32_t c) const { const uint32_t a = lisl[2 * c], b = lisl[2 * c + 1]; return a > b ? a : b; }
  DEV uint2 info(uint32_t, uint32_t) const { return make_uint2(0u, 0u); }
};
// sums (optional): [0] += number of non-empty items, [1] += their total length
// (one atomic pair per block: the work counters of the kernel that consumes them)
template <typename F>
__global__ __launch_bounds__(256) void k_len_hist(F f, uint32_t n, uint32_t* hist, unsigned long long* sums) {
  __shared__ uint32_t h[NLB];
  __shared__ uint64_t s_red[4];
  for (uint32_t i = threadIdx.x; i < NLB; i += 256) h[i] = 0;
  __syncthreads();
  uint64_t cnt = 0, len = 0;
  for (uint32_t c = blockIdx.x * 256 + threadIdx.x; c < n; c += gridDim.x * 256) {
    const uint32_t v = f(c);
    atomicAdd(&h[len_bucket(v)], 1u);
    cnt += v != 0; len += v;
  }
  if (sums) {
    cnt = block_sum_u64<256>(cnt, s_red);
    len = block_sum_u64<256>(len, s_red);
    if (threadIdx.x == 0 && cnt) { atomicAdd(&sums[0], (unsigned long long)cnt); atomicAdd(&sums[1], (unsigned long long)len); }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < NLB; i += 256) if (h[i]) atomicAdd(&hist[i], h[i]);
}
// block-aggregated over LEN_PERM_ITEMS items a thread: one global atomic per
// (block, bucket) -- the few hot buckets (the shortest lengths) see one atomic
// per 4096 items; zero-length items are dropped
constexpr uint32_t LEN_PERM_ITEMS = 16;
template <typename F>
// pinfo (optional, StrandLen): beside perm, each placed item's {first hit, hits}, so the
// lane-per-strand LIS reads its strand's range coalesced instead of item -> chain -> range
__global__ __launch_bounds__(256) void k_len_perm(F f, uint32_t n, uint32_t* cursor, uint32_t* perm,
                                                  typename F::Info* pinfo) {
  __shared__ uint32_t cnt[NLB], base[NLB];
  for (uint32_t i = threadIdx.x; i < NLB; i += 256) cnt[i] = 0;
  __syncthreads();
  const uint32_t c0 = blockIdx.x * 256 * LEN_PERM_ITEMS + threadIdx.x;
  uint32_t b[LEN_PERM_ITEMS], loc[LEN_PERM_ITEMS], len[LEN_PERM_ITEMS];
#pragma unroll
  for (uint32_t q = 0; q < LEN_PERM_ITEMS; ++q) {
    const uint32_t c = c0 + q * 256;
    len[q] = c < n ? f(c) : 0u;
    b[q] = c < n ? len_bucket(len[q]) : 0u;
    loc[q] = b[q] ? atomicAdd(&cnt[b[q]], 1u) : 0u;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < NLB; i += 256) if (cnt[i]) base[i] = atomicAdd(&cursor[i], cnt[i]);
  __syncthreads();
#pragma unroll
  for (uint32_t q = 0; q < LEN_PERM_ITEMS; ++q)
    if (b[q]) {
      const uint32_t at = base[b[q]] + loc[q];
      perm[at] = c0 + q * 256;
      if (pinfo) pinfo[at] = f.info(c0 + q * 256, len[q]);
    }
}

// ================================================================= lis / fit
// Lane-per-item kernels whose per-lane streams are staged through LDS: a wave
// owns 64 items of similar length and walks them in chunks of CH elements.
// Each chunk's rows (CH consecutive elements of one item = one 128-byte
// segment) are loaded / stored cooperatively, CH lanes per row, into a
// transposed LDS tile, so every HBM access is a whole coalesced segment and
// the serial per-lane work reads and writes LDS.
constexpr uint32_t RS = 65;  // LDS tile row stride (elements): one padding column

// all of this wave's LDS and memory operations complete and visible to its lanes
DEV void wave_drain() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
}
DEV uint64_t shfl_u64(uint64_t v, int src) {
  const uint32_t lo = __shfl((uint32_t)v, src, 64), hi = __shfl((uint32_t)(v >> 32), src, 64);
  return (uint64_t)hi << 32 | lo;
}
DEV uint32_t wave_max_u32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) { const uint32_t y = __shfl_xor(v, o, 64); v = y > v ? y : v; }
  return v;
}
// tile[e][l] = src[row_l + e] for lo_l <= e < hi_l (every lane passes its own row)
template <int CH, typename T>
DEV void rows_load(T* tile, const T* __restrict__ src, uint64_t row, uint32_t lo, uint32_t hi) {
  const int lane = lane_id();
#pragma unroll
  for (int g = 0; g < 64; g += 64 / CH) {
    const int l = g + lane / CH, e = lane % CH;
    const uint64_t rl = shfl_u64(row, l);
    const uint32_t lol = __shfl(lo, l, 64), hil = __shfl(hi, l, 64);
    if ((uint32_t)e >= lol && (uint32_t)e < hil) tile[e * RS + l] = src[rl + e];
  }
}
template <int CH, typename T>
DEV void rows_store(const T* tile, T* __restrict__ dst, uint64_t row, uint32_t lo, uint32_t hi) {
  const int lane = lane_id();
#pragma unroll
  for (int g = 0; g < 64; g += 64 / CH) {
    const int l = g + lane / CH, e = lane % CH;
    const uint64_t rl = shfl_u64(row, l);
    const uint32_t lol = __shfl(lo, l, 64), hil = __shfl(hi, l, 64);
    if ((uint32_t)e >= lol && (uint32_t)e < hil) dst[rl + e] = tile[e * RS + l];
  }
}
// Software-pipelined row load: issue() starts the global loads of one chunk
// into registers (each lane holds 64/CH elements of the transposed tile),
// commit() writes them to the LDS tile -- so the HBM latency of chunk j+1
// overlaps the serial work on chunk j.
template <int CH, typename T>
struct RowPipe {
  static constexpr int NG = CH;        // load instructions per chunk
  static constexpr int SPG = 64 / CH;  // rows (items) per instruction
  T v[NG];
  uint32_t mask;
  DEV void issue(const T* __restrict__ src, uint64_t row, uint32_t lo, uint32_t hi) {
    const int lane = lane_id();
    mask = 0;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int l = g * SPG + lane / CH, e = lane % CH;
      const uint64_t rl = shfl_u64(row, l);
      const uint32_t lol = __shfl(lo, l, 64), hil = __shfl(hi, l, 64);
      if ((uint32_t)e >= lol && (uint32_t)e < hil) { v[g] = src[rl + e]; mask |= 1u << g; }
    }
  }
  DEV void commit(T* tile) const {
    const int lane = lane_id();
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int l = g * SPG + lane / CH, e = lane % CH;
      if (mask & (1u << g)) tile[e * RS + l] = v[g];
    }
  }
};
DEV void lds_fence() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS traffic done
  __builtin_amdgcn_wave_barrier();
}

template <int CH>
struct ChunkGrid;
// Streams every lane's item through the LDS tile chunk by chunk, the next
// chunk's rows in flight while f() consumes the current one.
template <int CH, typename T, typename F>
DEV void stream_rows(const T* __restrict__ src, const ChunkGrid<CH>& G, uint32_t nch, T* tile, F&& f);

// A lane's item occupies [b, b + n) of a per-hit array; chunks follow the
// absolute CH-aligned grid so that every row is one aligned segment.
template <int CH>
struct ChunkGrid {
  uint64_t b, a0;   // item start, aligned start of chunk 0
  uint32_t n;
  DEV void init(uint64_t b_, uint32_t n_) { b = b_; n = n_; a0 = b_ & ~(uint64_t)(CH - 1); }
  DEV uint32_t chunks() const { return n ? (uint32_t)((b - a0 + n + CH - 1) / CH) : 0; }
  DEV uint64_t row(uint32_t j) const { return a0 + (uint64_t)j * CH; }
  // valid element slots [lo, hi) of chunk j
  DEV uint32_t lo(uint32_t j) const { const uint64_t r = row(j); return r >= b ? 0u : (uint32_t)(b - r); }
  DEV uint32_t hi(uint32_t j) const {
    const uint64_t r = row(j), e = b + n;
    if (!n || r >= e) return 0u;
    return e - r < CH ? (uint32_t)(e - r) : (uint32_t)CH;
  }
};

// Row pipe for 64-byte rows (CH * sizeof(T) == 64) loaded 16 bytes a lane:
// 4 lanes per row, 16 rows per load instruction, every lane loading (a lane
// with no row in the chunk re-reads row 0 of src).  The rows are CH-aligned
// 64-byte segments: src must be readable up to the next 64-byte boundary.
template <int CH, typename T>
struct RowPipe16 {
  static_assert(CH * sizeof(T) == 64, "64-byte rows");
  static constexpr int E = 16 / sizeof(T);  // elements per 16-byte piece
  uint4 v[4];
  DEV void issue(const T* __restrict__ src, uint64_t row, bool has) {
    const int lane = lane_id();
    const uint64_t r = has ? row : 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint64_t rl = shfl_u64(r, g * 16 + lane / 4);
      v[g] = *(const uint4*)(src + rl + (lane % 4) * E);
    }
  }
  DEV void commit(T* tile) const {
    const int lane = lane_id();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const T* p = (const T*)&v[g];
#pragma unroll
      for (int q = 0; q < E; ++q) tile[((lane % 4) * E + q) * RS + g * 16 + lane / 4] = p[q];
    }
  }
};

template <int CH, typename T, typename F>
DEV void stream_rows(const T* __restrict__ src, const ChunkGrid<CH>& G, uint32_t nch, T* tile, F&& f) {
  const int lane = lane_id();
  if constexpr (CH * sizeof(T) == 64) {
    RowPipe16<CH, T> pp;
    if (nch) pp.issue(src, G.row(0), G.hi(0) > G.lo(0));
    for (uint32_t j = 0; j < nch; ++j) {
      const uint32_t lo = G.lo(j), hi = G.hi(j);
      pp.commit(tile);
      if (j + 1 < nch) pp.issue(src, G.row(j + 1), G.hi(j + 1) > G.lo(j + 1));
      lds_fence();
      for (uint32_t e = lo; e < hi; ++e) f(tile[e * RS + lane]);
      lds_fence();
    }
    return;
  }
  RowPipe<CH, T> pp;
  if (nch) pp.issue(src, G.row(0), G.lo(0), G.hi(0));
  for (uint32_t j = 0; j < nch; ++j) {
    const uint32_t lo = G.lo(j), hi = G.hi(j);
    pp.commit(tile);
    if (j + 1 < nch) pp.issue(src, G.row(j + 1), G.lo(j + 1), G.hi(j + 1));
    lds_fence();
    for (uint32_t e = lo; e < hi; ++e) f(tile[e * RS + lane]);
    lds_fence();
  }
}

// The conjunctions are evaluated in full (bitwise &, no short circuit): every
// operand is a side-effect-free compare, and a short circuit costs a divergent
// branch (exec-mask save / restore) per operand in the wave-wide scans.
DEV bool affine_ok(double a, double b, double C, double df, double ds) {
  // (s.first <= b + a*s.second) && (s.second <= b + a*s.first) && s.first <= C && s.second <= C
  return (df <= __dadd_rn(b, __dmul_rn(a, ds))) & (ds <= __dadd_rn(b, __dmul_rn(a, df))) & (df <= C) & (ds <= C);
}
DEV bool linear_ok(double a, double df, double ds) {
  return (df <= __dmul_rn(a, ds)) & (ds <= __dmul_rn(a, df));
}

// k_lis chunk rows (elements a row) for 16- / 32-bit nodes; k_coords' rows
#ifndef PBGPU_FIT_CH
#define PBGPU_FIT_CH 8
#endif
constexpr int LIS_CH16 = 8, LIS_CH32 = 8, FIT_CH = PBGPU_FIT_CH;
// lis_align::compute_L_P (lis_align.hpp:139-182) + indices (:190-204),
// restated literally, one strand per lane: singly linked list L, first
// acceptable predecessor in list order, insertion after the first node of
// minimal length seen before it.  The window test uses X[i] - X[anc_{W-1}(j)],
// which equals sum_buffer::test_sum exactly (all values are small integers);
// span_full is X[i] - X[root].  The list head stays in registers (the typical
// scan stops there); older nodes are read from the chunk tile or from HBM.
// Forward pass, then a reverse chunk sweep along P writes the lis points
// pts[0..len) (and, with keep_idx, the lis indices into N[t].nxt).
template <typename I, int CH>
__global__ __launch_bounds__(64) void k_lis(const ChainDesc* __restrict__ chains, const uint32_t* __restrict__ items,
                                            uint32_t n_items, const uint32_t* __restrict__ slen,
                                            const int2* __restrict__ X, LNode<I>* __restrict__ N,
                                            int2* __restrict__ pts, uint32_t* __restrict__ lisl, LisParams lp,
                                            int keep_idx, unsigned long long* stats,
                                            const uint32_t* __restrict__ nshift) {
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  constexpr I INONE = (I)~(I)0;
  __shared__ int2 xs[CH * RS];
  __shared__ LNode<I> ns[CH * RS];
  const int lane = lane_id();
  const uint32_t w = blockIdx.x * 64 + lane;
  const bool act = w < n_items;
  uint32_t item = 0, n = 0;
  uint64_t base = 0;
  if (act) {
    item = items[w];
    const ChainDesc d = chains[item >> 1];
    base = d.hit_base + ((item & 1) ? d.nf : 0);
    n = slen[item];
  }
  ChunkGrid<CH> G;
  G.init(base, n);
  // nshift (32-bit nodes): the strand's nodes live in a compact array of the long
  // strands alone, from chunk nshift[item] on (k_node32_place): node index = hit
  // index + sh, sh a multiple of CH so the node rows stay CH-aligned (unsigned
  // wrap-around arithmetic)
  const uint64_t sh = (act && nshift) ? (uint64_t)nshift[item] * CH - (base & ~(uint64_t)(CH - 1)) : 0;
  const int2* Xl = X + base;
  LNode<I>* Nl = N + (base + sh);
  const uint32_t nch = wave_max_u32(G.chunks());
  auto wide = [](I v) -> uint32_t { return v == INONE ? NONE : (uint32_t)v; };
  uint64_t tests = 0;
  uint32_t head = NONE, hlen = 0, hnxt = NONE, hroot = 0, longest = 0, longest_ind = 0;
  int2 hx = make_int2(0, 0), hrootx = make_int2(0, 0);
  int32_t xmn = INT32_MAX, xmx = INT32_MIN, ymn = INT32_MAX, ymx = INT32_MIN;  // hit spans: lis layout
  PROF_T(t_start);
#ifdef PBGPU_PROF
  uint64_t p_load = 0, p_fetch = 0, p_elem = 0, p_store = 0;
#endif
  RowPipe<CH, int2> px;
  if (nch) px.issue(X, G.row(0), G.lo(0), G.hi(0));
  for (uint32_t j = 0; j < nch; ++j) {
    const uint32_t lo = G.lo(j), hi = G.hi(j);
    const uint64_t row = G.row(j);
    PROF_T(t0);
    px.commit(xs);
    if (j + 1 < nch) px.issue(X, G.row(j + 1), G.lo(j + 1), G.hi(j + 1));
    PROF_T(t1);
    lds_fence();
    int2 xr[CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) xr[e] = xs[e * RS + lane];
    lds_fence();
    PROF_T(t2);
#ifdef PBGPU_PROF
    p_load += t1 - t0; p_fetch += t2 - t1;
#endif
    // local index of slot 0 of this chunk (wraps for the first chunk; only c0 + e with e >= lo is used)
    const uint32_t c0 = (uint32_t)(row - base);
    const uint32_t first = hi > lo ? c0 + lo : 0u;  // smallest local index held in the tile
    auto in_tile = [&](uint32_t q) -> bool { return hi > lo && q >= first; };
    // Older elements live in HBM.  Those reads are rare (deep list scans) but
    // each one must drain vmcnt; the drain stays inside the rare branch so that
    // the common path never waits on the row prefetch or the row stores.
    auto getX = [&](uint32_t q) -> int2 {
      int2 v;
      if (in_tile(q)) {
        v = xs[(q - c0) * RS + lane];
      } else {
        v = Xl[q];
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
      }
      return v;
    };
    auto getN = [&](uint32_t q) -> LNode<I> {
      LNode<I> v;
      if (in_tile(q)) {
        v = ns[(q - c0) * RS + lane];
      } else {
        v = Nl[q];
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
      }
      return v;
    };
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      if ((uint32_t)e < lo || (uint32_t)e >= hi) continue;
      const uint32_t i = c0 + e;
      const int2 xi = xr[e];
      xmn = min(xmn, xi.x); xmx = max(xmx, xi.x); ymn = min(ymn, xi.y); ymx = max(ymx, xi.y);
      uint32_t prev = NONE, prev_len = 0, prev_nxt = NONE, found = NONE, f_len = 0, f_root = 0;
      int2 f_rootx = hrootx;
      if (head != NONE) {
        uint32_t it = head, lj = hlen, nx = hnxt, jroot = hroot;
        int2 xj = hx;
        bool at_head = true;
        for (;;) {
          ++tests;
          if (xi.y > xj.y) {
            bool ok;
            if (lp.mer_all) ok = true;
            else if (lp.W == 1) ok = affine_ok(lp.a, lp.b, lp.C, (double)(xi.x - xj.x), (double)(xi.y - xj.y));
            else if (lp.W == 0 || lj < lp.W) ok = true;  // !will_be_filled()
            else {
              uint32_t anc = it;
              for (uint32_t q = 1; q < lp.W; ++q) anc = wide(getN(anc).P);
              const int2 xa = getX(anc);
              ok = affine_ok(lp.a, lp.b, lp.C, (double)(xi.x - xa.x), (double)(xi.y - xa.y));
            }
            if (ok) {
              found = it; f_len = lj; f_root = jroot;
              if (!at_head) f_rootx = getX(jroot);  // the head's root is cached in registers
              break;
            }
          }
          if (prev == NONE || lj < prev_len) { prev = it; prev_len = lj; prev_nxt = nx; }
          it = nx;
          if (it == NONE) break;
          const LNode<I> nd = getN(it);
          xj = getX(it); lj = nd.len; nx = wide(nd.nxt); jroot = nd.root; at_head = false;
        }
      }
      LNode<I> en;
      uint32_t elen, eroot;
      int2 erootx;
      if (found != NONE) {
        elen = f_len + 1; eroot = f_root; en.P = (I)found; erootx = f_rootx;
      } else {
        elen = 1; eroot = i; en.P = INONE; erootx = xi;
      }
      en.len = (I)elen; en.root = (I)eroot;
      if (prev == NONE) {  // insert at the head
        en.nxt = head == NONE ? INONE : (I)head;
        hnxt = head; head = i; hx = xi; hlen = elen; hroot = eroot; hrootx = erootx;
      } else {
        en.nxt = prev_nxt == NONE ? INONE : (I)prev_nxt;
        if (in_tile(prev)) ns[(prev - c0) * RS + lane].nxt = (I)i;
        else Nl[prev].nxt = (I)i;
        if (prev == head) hnxt = i;
      }
      ns[e * RS + lane] = en;
      if (longest < elen) {
        if (lp.seq_all || linear_ok(lp.a, (double)(xi.x - erootx.x), (double)(xi.y - erootx.y))) {
          longest = elen; longest_ind = i;
        }
      }
    }
    lds_fence();
    PROF_T(t3);
    rows_store<CH>(ns, N, row + sh, lo, hi);
    lds_fence();  // tile rows read before the next chunk overwrites them
    PROF_T(t4);
#ifdef PBGPU_PROF
    p_elem += t3 - t2; p_store += t4 - t3;
#endif
  }
  PROF_T(t_fwd);
  // reverse sweep along P: lis points in ascending order
  uint32_t s = longest_ind, t = 0;
  bool need = longest > 0;
  int2* Pl = pts + base;
  // compact layout when every hit of the strand lies within 65535 of every other
  uint32_t* Pw = (uint32_t*)Pl + 2;
  const bool cmp = longest >= 2 && (uint32_t)(xmx - xmn) < 65536u && (uint32_t)(ymx - ymn) < 65536u;
  const int2 last = cmp ? Xl[longest_ind] : make_int2(0, 0);
  auto sweep_rows = [&](int64_t j, uint32_t& lo, uint32_t& hi) {
    const bool here = need && (uint64_t)base + s >= G.row((uint32_t)j);
    lo = here ? G.lo((uint32_t)j) : 0; hi = here ? G.hi((uint32_t)j) : 0;
  };
  RowPipe<CH, LNode<I>> pn;
  int64_t j = (int64_t)nch - 1;
  uint32_t lo_n = 0, hi_n = 0;
  if (j >= 0) {
    sweep_rows(j, lo_n, hi_n);
    px.issue(X, G.row((uint32_t)j), lo_n, hi_n);
    pn.issue(N, G.row((uint32_t)j) + sh, lo_n, hi_n);
  }
  for (; j >= 0; --j) {
    if (!__ballot(need)) break;
    const uint64_t row = G.row((uint32_t)j);
    const uint32_t c0 = (uint32_t)(row - base);
    px.commit(xs);
    pn.commit(ns);
    // the next chunk down: every lane still needing points reaches into it
    if (j >= 1) {
      const bool later = need;  // conservative: rows of lanes whose walk may continue below this chunk
      const uint64_t r1 = G.row((uint32_t)(j - 1));
      const uint32_t lo1 = later ? G.lo((uint32_t)(j - 1)) : 0, hi1 = later ? G.hi((uint32_t)(j - 1)) : 0;
      (void)r1;
      px.issue(X, r1, lo1, hi1);
      pn.issue(N, r1 + sh, lo1, hi1);
    }
    lds_fence();
    if (need && (uint64_t)base + s >= row) {
      while (need && (uint64_t)base + s >= row) {
        const uint32_t o = longest - 1 - t;
        const int2 p = xs[(s - c0) * RS + lane];
        if (cmp) Pw[o] = pt_word(last, p);
        else Pl[o] = p;
        const uint32_t ps = wide(ns[(s - c0) * RS + lane].P);
        if (keep_idx) Nl[o].nxt = (I)s;  // nxt is dead after the forward pass; the sweep reads only P
        s = ps;
        if (++t == longest) need = false;
      }
    }
    lds_fence();
  }
  (void)lo_n; (void)hi_n;
  if (cmp) { Pw[-2] = (uint32_t)last.x | PT_COMPACT; Pw[-1] = (uint32_t)last.y; }
  PROF_T(t_end);
  PROF_ADD(0, p_load); PROF_ADD(1, p_fetch); PROF_ADD(2, p_elem); PROF_ADD(3, p_store);
  PROF_ADD(4, t_end - t_fwd); PROF_ADD(5, t_end - t_start); PROF_ADD(6, nch); PROF_ADD(7, 1);
  if (act) lisl[item] = longest;
  tests = wave_sum_u64(tests);
  if (lane == 0 && tests) atomicAdd(&stats[ST_LIS_TESTS], (unsigned long long)tests);
}

// ------------------------------------------------------------------------
// k_lis_w: one WAVE per strand, the whole strand (X and the list nodes) in
// LDS.  Same algorithm (compute_L_P, lis_align.hpp:139-182), evaluated with
// the wave's 64 lanes on 64 consecutive elements at a time:
//  * "clean" step: element i's first test is against the current list head.
//    If every element of a run passes that test, each is found at the head
//    and inserted at the head (prev stays before_begin), so for the run
//    head(i) = i-1, len(i) = len(head)+1+(i-start), root(i) = root(head),
//    P(i) = i-1.  Lanes test their element against X[i-1] (lane 0 against
//    the real head) and a ballot finds the first element that is not clean;
//    the clean prefix is committed in parallel, including the longest update
//    (len grows by one per element, so the last lane whose span passes
//    `linear` with len > longest wins, exactly as the sequential loop).
//  * any other element runs the literal list scan, wave-uniformly.
// Backtracking (indices, :190-204) walks maximal runs with P(e) = e-1 at
// once: run starts are kept per node.  Only the default window (W = 1,
// accept_mer = affine_capped) takes the clean step; other windows and the
// test-only accept_all variants use the literal scan for every element.
// HBM traffic: X once (coalesced, prefetched for the next strand while the
// current one is processed), the lis points (and, for --max-match, the lis
// indices) once.
// List order of a strand (coarse_aligner.cc:128-140): pb offset
// ascending, then occurrence order, which within one super-read and strand is
// |sr offset| descending.  (pb, |so|) pairs are unique within a list.
DEV bool hit_after(int2 a, int2 b) {  // branch-free (a select compiled to an if / else)
  return (a.x > b.x) | ((a.x == b.x) & (abs(a.y) < abs(b.y)));
}

// Restores list order for strands too long for k_lis_w's LDS (one block per
// strand, in place): odd-even transposition rounds until one swaps nothing.
// k_group leaves only short unordered runs, so a few rounds suffice.
__global__ __launch_bounds__(256) void k_strand_order(const ChainDesc* __restrict__ chains,
                                                      const uint32_t* __restrict__ items, uint32_t n_items,
                                                      const uint32_t* __restrict__ slen, int2* X) {
  __shared__ uint32_t s_sw[2];
  for (uint32_t w = blockIdx.x; w < n_items; w += gridDim.x) {
    const uint32_t item = items[w];
    const ChainDesc d = chains[item >> 1];
    int2* x = X + d.hit_base + ((item & 1) ? d.nf : 0);
    const uint32_t n = slen[item];
    for (uint32_t round = 0;; ++round) {
      if (threadIdx.x == 0) s_sw[round & 1] = 0;  // the other flag is still being read
      bool sw = false;
      for (uint32_t par = 0; par < 2; ++par) {
        for (uint32_t j = 2 * threadIdx.x + par; j + 1 < n; j += 512) {
          const int2 a = x[j], b = x[j + 1];
          if (hit_after(a, b)) { x[j] = b; x[j + 1] = a; sw = true; }
        }
        __threadfence_block();
        __syncthreads();
      }
      if (sw) s_sw[round & 1] = 1;
      __syncthreads();
      if (!s_sw[round & 1]) break;
    }
    __syncthreads();
  }
}

// List order of strands of at most NMAX hits, one strand per lane: an odd-even
// transposition network over registers (NMAX rounds sort any NMAX elements),
// written back only when something moved.  These strands then go to the
// lane-per-strand k_lis: a wave-per-strand kernel would spend a whole wave on
// a handful of hits (on C2 30% of the non-empty strands have <= 8 hits).
template <int NMAX>
__global__ __launch_bounds__(256) void k_order_tiny(const ChainDesc* __restrict__ chains,
                                                    const uint32_t* __restrict__ items, uint32_t n_items,
                                                    const uint32_t* __restrict__ slen, int2* X) {
  const uint32_t w = blockIdx.x * 256 + threadIdx.x;
  if (w >= n_items) return;
  const uint32_t item = items[w];
  const ChainDesc d = chains[item >> 1];
  const uint64_t base = d.hit_base + ((item & 1) ? d.nf : 0);
  const uint32_t n = slen[item];
  int2 v[NMAX];
#pragma unroll
  for (int j = 0; j < NMAX; ++j) v[j] = (uint32_t)j < n ? X[base + j] : make_int2(0, 0);
  bool moved = false;
#pragma unroll
  for (int r = 0; r < NMAX; ++r) {
#pragma unroll
    for (int j = r & 1; j + 1 < NMAX; j += 2) {
      if ((uint32_t)(j + 1) < n && hit_after(v[j], v[j + 1])) {
        const int2 t = v[j]; v[j] = v[j + 1]; v[j + 1] = t;
        moved = true;
      }
    }
  }
  if (moved) {
#pragma unroll
    for (int j = 0; j < NMAX; ++j) if ((uint32_t)j < n) X[base + j] = v[j];
  }
}

// Strands of at most NMAX (<= 15) hits, one per lane, entirely in registers: the list order
// restored by the odd-even network of k_order_tiny (X written back when it moved), then
// lis_align::compute_L_P (lis_align.hpp:139-182) and indices (:190-204) restated literally
// -- the singly linked list L walked from its head, the first acceptable predecessor, the
// insertion after the first node of minimal length seen before it -- with the nodes packed
// 16 bits each ({nxt, P, len, root} 4 bits apiece, 15 = none) in two 64-bit registers and
// a node's hit picked from registers by index.  The generic lane-per-strand k_lis staged
// these strands through LDS rows, stored every node to HBM and read hits and nodes back
// for the reverse sweep (C4: 1 chain per 9 hits, most strands <= 8 hits: k_lis 13.9 +
// k_order_tiny 3.2 ms of a 92-ms sub-batch).  Default window only (W = 1, affine
// step test), no kept lis indices (--max-match takes the generic kernel).
template <int NMAX>
__global__ __launch_bounds__(256) void k_lis_tiny(const ChainDesc* __restrict__ chains,
                                                  const uint32_t* __restrict__ items, const uint2* __restrict__ pinfo,
                                                  uint32_t n_items, const uint32_t* __restrict__ slen, int2* X,
                                                  int2* __restrict__ pts, uint32_t* __restrict__ lisl, LisParams lp,
                                                  unsigned long long* stats) {
  static_assert(NMAX <= 15, "4-bit node fields (15 = none)");
  constexpr uint32_t NONE = 15;
  const uint32_t w = blockIdx.x * 256 + threadIdx.x;
  const bool act = w < n_items;
  uint32_t item = 0, n = 0;
  uint64_t base = 0;
  if (act) {
    item = items[w];
    if (pinfo) {  // the strand's range from the permutation pass: no dependent loads
      const uint2 pi = pinfo[w];
      base = pi.x; n = pi.y;
    } else {
      const ChainDesc d = chains[item >> 1];
      base = d.hit_base + ((item & 1) ? d.nf : 0);
      n = slen[item];
    }
  }
  int2 v[NMAX];
#pragma unroll
  for (int j = 0; j < NMAX; ++j) v[j] = (uint32_t)j < n ? X[base + j] : make_int2(0, 0);
  if (!lp.ordered) {
    bool moved = false;
#pragma unroll
    for (int r = 0; r < NMAX; ++r) {
#pragma unroll
      for (int j = r & 1; j + 1 < NMAX; j += 2) {
        if ((uint32_t)(j + 1) < n && hit_after(v[j], v[j + 1])) {
          const int2 t = v[j]; v[j] = v[j + 1]; v[j + 1] = t;
          moved = true;
        }
      }
    }
    if (moved) {
#pragma unroll
      for (int j = 0; j < NMAX; ++j) if ((uint32_t)j < n) X[base + j] = v[j];
    }
  }
  auto xat = [&](uint32_t q) -> int2 {  // v[q], q < NMAX, by selects
    int2 r = v[0];
#pragma unroll
    for (int j = 1; j < NMAX; ++j) r = q == (uint32_t)j ? v[j] : r;
    return r;
  };
  // node q: bits [16 (q & 3), +16) of nd[q >> 2]: nxt | P << 4 | len << 8 | root << 12
  constexpr int NW = (NMAX + 3) / 4;
  uint64_t nd[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) nd[j] = 0;
  auto word = [&](uint32_t q) -> uint64_t {
    uint64_t r = nd[0];
#pragma unroll
    for (int j = 1; j < NW; ++j) r = (q >> 2) == (uint32_t)j ? nd[j] : r;
    return r;
  };
  auto node = [&](uint32_t q) -> uint32_t { return (uint32_t)((word(q) >> (16 * (q & 3))) & 0xFFFFu); };
  auto set_node = [&](uint32_t q, uint32_t val) {
    const uint32_t sh = 16 * (q & 3);
    const uint64_t m = ~(0xFFFFull << sh), x = (uint64_t)val << sh;
#pragma unroll
    for (int j = 0; j < NW; ++j) nd[j] = (q >> 2) == (uint32_t)j ? ((nd[j] & m) | x) : nd[j];
  };
  auto set_nxt = [&](uint32_t q, uint32_t nx) { set_node(q, (node(q) & ~15u) | nx); };
  uint64_t tests = 0;
  uint32_t head = NONE, longest = 0, longest_ind = 0;
  int32_t xmn = INT32_MAX, xmx = INT32_MIN, ymn = INT32_MAX, ymx = INT32_MIN;
  for (uint32_t i = 0; i < n; ++i) {
    const int2 xi = xat(i);
    xmn = min(xmn, xi.x); xmx = max(xmx, xi.x); ymn = min(ymn, xi.y); ymx = max(ymx, xi.y);
    uint32_t prev = NONE, prev_len = 0, found = NONE, f_len = 0, f_root = 0;
    for (uint32_t it = head; it != NONE;) {
      ++tests;
      const uint32_t nv = node(it), lj = (nv >> 8) & 15u;
      const int2 xj = xat(it);
      if ((xi.y > xj.y) && affine_ok(lp.a, lp.b, lp.C, (double)(xi.x - xj.x), (double)(xi.y - xj.y))) {
        found = it; f_len = lj; f_root = nv >> 12;
        break;
      }
      if (prev == NONE || lj < prev_len) { prev = it; prev_len = lj; }
      it = nv & 15u;
    }
    const uint32_t elen = found != NONE ? f_len + 1 : 1u, eroot = found != NONE ? f_root : i;
    uint32_t enxt;
    if (prev == NONE) { enxt = head; head = i; }
    else { enxt = node(prev) & 15u; set_nxt(prev, i); }
    set_node(i, enxt | (found << 4) | (elen << 8) | (eroot << 12));
    if (longest < elen) {
      const int2 xr = xat(eroot);
      if (lp.seq_all || linear_ok(lp.a, (double)(xi.x - xr.x), (double)(xi.y - xr.y))) {
        longest = elen; longest_ind = i;
      }
    }
  }
  if (act) {
    // the lis points in ascending order along P (indices, lis_align.hpp:190-204)
    int2* Pl = pts + base;
    uint32_t* Pw = (uint32_t*)Pl + 2;
    const bool cmp = longest >= 2 && (uint32_t)(xmx - xmn) < 65536u && (uint32_t)(ymx - ymn) < 65536u;
    const int2 last = xat(longest_ind);
    uint32_t sidx = longest_ind;
    for (uint32_t t = 0; t < longest; ++t) {
      const uint32_t o = longest - 1 - t;
      const int2 p = xat(sidx);
      if (cmp) Pw[o] = pt_word(last, p);
      else Pl[o] = p;
      sidx = (node(sidx) >> 4) & 15u;
    }
    if (cmp) { Pw[-2] = (uint32_t)last.x | PT_COMPACT; Pw[-1] = (uint32_t)last.y; }
    lisl[item] = longest;
  }
  tests = wave_sum_u64(tests);
  if ((threadIdx.x & 63) == 0 && tests) atomicAdd(&stats[ST_LIS_TESTS], (unsigned long long)tests);
}

constexpr int LISW_TINY_N = 255;  // SMAX of the timed tier-0 k_lis_w
#ifndef PBGPU_LISW_WAVES
#define PBGPU_LISW_WAVES 0  // experiment: waves per SIMD asked of the compiler (0 = its choice)
#endif
template <int SMAX, int WPB>
__global__ __launch_bounds__(64 * WPB)
#if PBGPU_LISW_WAVES
__attribute__((amdgpu_waves_per_eu(PBGPU_LISW_WAVES, PBGPU_LISW_WAVES)))
#endif
void k_lis_w(const ChainDesc* __restrict__ chains,
                                                    const uint32_t* __restrict__ items, uint32_t n_items,
                                                    const uint32_t* __restrict__ slen, int2* X,
                                                    LNode<uint16_t>* __restrict__ N16, int2* __restrict__ pts,
                                                    uint32_t* __restrict__ lisl, LisParams lp, int keep_idx,
                                                    unsigned long long* stats) {
  constexpr uint32_t NONE = 0xFFFFu;
  constexpr int PF = (SMAX + 63) / 64;  // prefetch registers per lane
  __shared__ int2 s_x[WPB][SMAX];
  // s_ord: the list L (lis_align.hpp:146) as an array in reverse order -- after i
  // elements, s_ord[i - 1] is the head and the node the reference's walk reaches after s
  // steps is s_ord[i - 1 - s] (every element is inserted, so the list holds all of them)
  __shared__ uint16_t s_ord[WPB][SMAX], s_len[WPB][SMAX], s_P[WPB][SMAX], s_root[WPB][SMAX], s_rs[WPB][SMAX];
  const int lane = lane_id();
  const uint32_t wv = threadIdx.x >> 6;
  int2* sx = s_x[wv];
  uint16_t *sord = s_ord[wv], *sln = s_len[wv], *sP = s_P[wv], *sroot = s_root[wv], *srs = s_rs[wv];
  const uint32_t nwaves = gridDim.x * WPB;
  const bool fast = lp.W == 1 && !lp.mer_all;
  uint64_t tests = 0, my_hits = 0, my_strands = 0, my_points = 0;
  auto desc = [&](uint32_t item, uint64_t& base, uint32_t& n) {
    const ChainDesc d = chains[item >> 1];
    base = d.hit_base + ((item & 1) ? d.nf : 0);
    n = slen[item];
  };
  // Software pipeline over this wave's strands w, w + nwaves, ...: while strand
  // w is processed, the X rows of w + nwaves (small SMAX: into registers), the
  // descriptor of w + 2 nwaves and the item id of w + 3 nwaves are in flight,
  // so the dependent item -> descriptor -> rows chain never stalls a strand.
  constexpr bool PREFETCH = PF <= 8;
  uint32_t w = blockIdx.x * WPB + wv;
  int2 pf[PREFETCH ? PF : 1];
  uint64_t nbase = 0, nbase2 = 0;
  uint32_t nn = 0, nitem = 0, nn2 = 0, nitem2 = 0, nitem3 = 0;
  if (w < n_items) {
    nitem = items[w];
    desc(nitem, nbase, nn);
    if constexpr (PREFETCH) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {  // clamped, not branched: lanes past the strand reload its last hit
        const uint32_t j = q * 64 + lane;
        pf[q] = X[nbase + (j < nn ? j : nn - 1)];
      }
    }
    if (w + nwaves < n_items) { nitem2 = items[w + nwaves]; desc(nitem2, nbase2, nn2); }
    if (w + 2 * nwaves < n_items) nitem3 = items[w + 2 * nwaves];
  }
  for (; w < n_items; w += nwaves) {
    const uint64_t base = nbase;
    const uint32_t n = nn, item = nitem;
    my_hits += n; ++my_strands;
    int2 xv[PREFETCH ? PF : 1];
    if constexpr (PREFETCH) {
#pragma unroll
      for (int q = 0; q < PF; ++q) xv[q] = pf[q];
    }
    // advance the pipeline: rows of w + nwaves, descriptor of w + 2 nwaves, item of w + 3 nwaves
    nbase = nbase2; nn = nn2; nitem = nitem2;
    if (w + nwaves < n_items) {
      if constexpr (PREFETCH) {
#pragma unroll
        for (int q = 0; q < PF; ++q) {  // clamped, not branched: lanes past the strand reload its last hit
        const uint32_t j = q * 64 + lane;
        pf[q] = X[nbase + (j < nn ? j : nn - 1)];
      }
      }
      if (w + 2 * nwaves < n_items) {
        nitem2 = nitem3;
        desc(nitem2, nbase2, nn2);
        if (w + 3 * nwaves < n_items) nitem3 = items[w + 3 * nwaves];
      }
    }
    if constexpr (PREFETCH) {
      // Register path: a strand already in list order whose every element is
      // clean (passes the test against its predecessor, see below) is one run
      // P(e) = e-1 from element 0; the forward pass then only picks the last
      // element whose span from element 0 passes `linear`, and the lis is
      // elements 0..top.  Same result as the LDS path, no LDS traffic.
#ifdef PBGPU_EXP_NO_LISW_REG
      if (false) {
#else
      if (fast) {
#endif
        // broadcasts by v_readlane and the predecessor by a DPP wave shift (wave_shr:1), no
        // ds_bpermute round trips; every lane is active here, so every source is valid
        // (LIS stage -0.3 ms, r04)
        const int2 x0 = make_int2(__builtin_amdgcn_readlane(xv[0].x, 0), __builtin_amdgcn_readlane(xv[0].y, 0));
        bool bad = false;
        int32_t top = -1;
#pragma unroll
        for (int q = 0; q < PF; ++q) {
          if ((uint32_t)q * 64 >= n) break;  // wave-uniform
          const uint32_t i = q * 64 + lane;
          int2 pv = make_int2(__builtin_amdgcn_update_dpp(0, xv[q].x, 0x138, 0xf, 0xf, false),  // wave_shr:1
                              __builtin_amdgcn_update_dpp(0, xv[q].y, 0x138, 0xf, 0xf, false));
          const int qp = q > 0 ? q - 1 : 0;
          const int2 plast = make_int2(__builtin_amdgcn_readlane(xv[qp].x, 63), __builtin_amdgcn_readlane(xv[qp].y, 63));
          if (q > 0 && lane == 0) pv = plast;
          const int2 xi = xv[q];
          {  // branch-free: the lanes past n compute on stale values and are masked out
            const bool clean = (xi.y > pv.y) & affine_ok(lp.a, lp.b, lp.C, (double)(xi.x - pv.x), (double)(xi.y - pv.y));
            bad |= (i < n) & (i > 0) & (!clean | ((lp.ordered == 0) & hit_after(pv, xi)));
          }
          const bool lin = (i < n) & ((lp.seq_all != 0) | linear_ok(lp.a, (double)(xi.x - x0.x), (double)(xi.y - x0.y)));
          const uint64_t lb = __ballot(lin);
          if (lb) top = q * 64 + 63 - (int32_t)__clzll((long long)lb);
        }
        if (!__ballot(bad)) {
          const uint32_t longest = (uint32_t)(top + 1);  // element 0 always passes
          int2 last = make_int2(0, 0);
#pragma unroll
          for (int q = 0; q < PF; ++q)
            if (top >> 6 == q) last = make_int2(__builtin_amdgcn_readlane(xv[q].x, top & 63),
                                                __builtin_amdgcn_readlane(xv[q].y, top & 63));
          bool far = false;
#pragma unroll
          for (int q = 0; q < PF; ++q) {
            const int32_t i = q * 64 + lane;
            if (i <= top) far |= !pt_fits(last, xv[q]);
          }
          const bool cmp = longest >= 2 && !__ballot(far);
          int2* Pl = pts + base;
          uint32_t* Pw = (uint32_t*)Pl + 2;
#pragma unroll
          for (int q = 0; q < PF; ++q) {
            const int32_t i = q * 64 + lane;
            if (i <= top) {
              if (cmp) Pw[i] = pt_word(last, xv[q]);
              else Pl[i] = xv[q];
              if (keep_idx) N16[base + i].nxt = (uint16_t)i;
            }
          }
          if (lane == 0) {
            if (cmp) { Pw[-2] = (uint32_t)last.x | PT_COMPACT; Pw[-1] = (uint32_t)last.y; }
            lisl[item] = longest;
          }
          tests += n - 1;
          continue;
        }
      }
#pragma unroll
      for (int q = 0; q < PF; ++q) { const uint32_t j = q * 64 + lane; if (j < n) sx[j] = xv[q]; }
    } else {
      for (uint32_t j = lane; j < n; j += 64) sx[j] = X[base + j];
    }
    lds_fence();
#ifdef PBGPU_PROF
    const uint64_t pw_t0 = __builtin_amdgcn_s_memtime();
    uint64_t pw_rounds = 0;
#endif
    // ---- list order: k_group leaves each 256-hit step's run of a list unordered.
    // Odd-even transposition in LDS until a round swaps nothing (an ordered strand
    // costs one compare per element); written back to X when anything moved, for
    // k_discard and the --max-match redo rounds.  The fine aligner's lists come in
    // order (and follow another order rule), so they skip this.
    if (!lp.ordered) {
      bool moved = false;
      for (;;) {
        bool sw = false;
        for (uint32_t par = 0; par < 2; ++par) {
          for (uint32_t j = 2 * lane + par; j + 1 < n; j += 128) {
            const int2 a = sx[j], b = sx[j + 1];
            if (hit_after(a, b)) { sx[j] = b; sx[j + 1] = a; sw = true; }
          }
          lds_fence();
        }
        if (!__ballot(sw)) break;
        moved = true;
#ifdef PBGPU_PROF
        ++pw_rounds;
#endif
      }
      if (moved)
        for (uint32_t j = lane; j < n; j += 64) X[base + j] = sx[j];
    }
#ifdef PBGPU_PROF
    const uint64_t pw_t1 = __builtin_amdgcn_s_memtime();
#endif
    // ---- forward pass (compute_L_P)
    uint32_t head = NONE, longest = 0, longest_ind = 0;
    uint32_t cur = 0;
    while (cur < n) {
      const uint32_t pend = cur + 64 < n ? cur + 64 : n;
      uint32_t m = 0;
      if (fast) {
        // The strand's first element (empty list) is clean too: no scan, len 1,
        // P = NONE, its own root, inserted at the head (what the literal step does).
        const bool empty = head == NONE;
        const uint32_t i = cur + lane;
        bool clean = false;
        int2 xi = make_int2(0, 0);
        if (i < pend) {
          xi = sx[i];
          if (lane == 0 && empty) {
            clean = true;
          } else {
            const int2 xj = sx[lane == 0 ? head : i - 1];
            clean = (xi.y > xj.y) & affine_ok(lp.a, lp.b, lp.C, (double)(xi.x - xj.x), (double)(xi.y - xj.y));
          }
        }
        const uint64_t bad = __ballot((i < pend) & !clean);
        m = bad ? (uint32_t)__ffsll((unsigned long long)bad) - 1 : pend - cur;
        if (m) {
          const uint32_t hl = empty ? 0u : sln[head], hr = empty ? cur : sroot[head];
          const uint32_t rsr = !empty && head + 1 == cur ? srs[head] : cur;  // run of P(e) = e-1 links
          const int2 hrx = sx[hr];
          bool cand = false;
          if ((uint32_t)lane < m) {
            const uint32_t elen = hl + 1 + lane;
            const uint32_t P = lane == 0 ? head : i - 1;
            sord[i] = (uint16_t)i; sln[i] = (uint16_t)elen; sP[i] = (uint16_t)P; sroot[i] = (uint16_t)hr;
            srs[i] = (uint16_t)(P + 1 == i ? rsr : i);
            cand = (elen > longest) &
                   ((lp.seq_all != 0) | linear_ok(lp.a, (double)(xi.x - hrx.x), (double)(xi.y - hrx.y)));
          }
          const uint64_t cb = __ballot(cand);
          if (cb) {
            const uint32_t top = 63u - (uint32_t)__clzll((long long)cb);
            longest = hl + 1 + top; longest_ind = cur + top;
          }
          head = cur + m - 1;
          tests += m - (empty ? 1u : 0u);  // the first element tests nothing
          cur += m;
          PROF_ADD(21, 1);
          PROF_ADD(22, m);
          lds_fence();
        }
      }
      if (cur < pend) {
        // ---- literal step for element cur (wave-uniform): the reference's walk down L
        // (lis_align.hpp:156-171) evaluated 64 nodes at a time.  Lane l of chunk c0 holds
        // the node at walk step s = c0 + l; the node that takes i is the first set lane of
        // a ballot, and `prev` (the first node of the smallest length met before it: the
        // last strict decrease of the walk's running minimum) is a min-reduction of
        // (len, s) over the nodes before it.  On repeat-rich strands the walks are long
        // (C4r: 76 nodes a step on average), which a serial pointer chase paid node by node.
        const uint32_t i = cur;
        const int2 xi = sx[i];
        uint32_t found = NONE, found_s = 0, best = 0xFFFFFFFFu;  // best: len << 16 | s (lane-local)
        bool hit = false;
#ifdef PBGPU_PROF
        PROF_ADD(20, 1);
#endif
        for (uint32_t c0 = 0; c0 < i; c0 += 64) {
          const uint32_t s = c0 + lane;
          const bool valid = s < i;
          const uint32_t j = sord[valid ? i - 1 - s : 0];
          const uint32_t lj = sln[j];
          const int2 xj = sx[j];
          bool ok = valid & (xi.y > xj.y);
          if (lp.mer_all) {
          } else if (lp.W == 1) {
            ok &= affine_ok(lp.a, lp.b, lp.C, (double)(xi.x - xj.x), (double)(xi.y - xj.y));
          } else if (lp.W == 0) {
          } else if (ok & (lj >= lp.W)) {  // will_be_filled(): the window's oldest add
            uint32_t anc = j;
            for (uint32_t q = 1; q < lp.W; ++q) anc = sP[anc];
            const int2 xa = sx[anc];
            ok = affine_ok(lp.a, lp.b, lp.C, (double)(xi.x - xa.x), (double)(xi.y - xa.y));
          }
          const uint64_t fb = __ballot(ok);
          const uint32_t lim = fb ? (uint32_t)__ffsll((unsigned long long)fb) - 1 : 64u;
          const uint32_t key = lj << 16 | s;
          if (valid & (lane < lim) & (key < best)) best = key;
#ifdef PBGPU_PROF
          PROF_ADD(23, 1);
#endif
          if (fb) {
            found_s = c0 + lim; hit = true;
            found = (uint32_t)__builtin_amdgcn_readlane((int)j, (int)lim);
            break;
          }
        }
        tests += hit ? found_s + 1 : i;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const uint32_t y = (uint32_t)__shfl_xor((int)best, o, 64);
          best = y < best ? y : best;
        }
        uint32_t elen, eroot, P;
        if (hit) { elen = sln[found] + 1u; eroot = sroot[found]; P = found; }
        else { elen = 1; eroot = i; P = NONE; }
        if (best == 0xFFFFFFFFu) {  // nothing met before the taker: insert at the head
          if (lane == 0) sord[i] = (uint16_t)i;
          head = i;
        } else {  // insert after prev (walk step ps): shift positions [a, i) up by one
          const uint32_t a = i - 1 - (best & 0xFFFFu);
          for (int32_t t0 = (int32_t)i - 1; t0 >= (int32_t)a; t0 -= 64) {
            const int32_t q = t0 - lane;
            const bool mv = q >= (int32_t)a;
            const uint16_t v = sord[mv ? q : 0];
            if (mv) sord[q + 1] = v;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
          }
          if (lane == 0) sord[a] = (uint16_t)i;
        }
        if (lane == 0) {
          sln[i] = (uint16_t)elen; sP[i] = (uint16_t)P; sroot[i] = (uint16_t)eroot;
          srs[i] = (uint16_t)(P + 1 == i ? srs[i - 1] : i);
        }
        if (elen > longest) {
          const int2 xr = sx[eroot];
          if (lp.seq_all || linear_ok(lp.a, (double)(xi.x - xr.x), (double)(xi.y - xr.y))) {
            longest = elen; longest_ind = i;
          }
        }
        ++cur;
        lds_fence();
      }
    }
#ifdef PBGPU_PROF
    const uint64_t pw_t2 = __builtin_amdgcn_s_memtime();
#endif
    // ---- backtracking (indices): whole P(e) = e-1 runs at a time, lis points in ascending order
    // compact layout unless a point lies too far from the last one: then once
    // more in the wide layout (rare: spans beyond 64 kb)
    int2* Pl = pts + base;
    uint32_t* Pw = (uint32_t*)Pl + 2;
    const int2 last = longest ? sx[longest_ind] : make_int2(0, 0);
    for (int wide = longest < 2; wide < 2; ++wide) {
      uint32_t t = longest, s = longest_ind;
      bool far = false;
      while (t > 0) {
        const uint32_t r = srs[s];
        const uint32_t run = s - r + 1, cnt = run < t ? run : t;
        for (uint32_t j = lane; j < cnt; j += 64) {
          const int2 p = sx[s - j];
          if (wide) Pl[t - 1 - j] = p;
          else { Pw[t - 1 - j] = pt_word(last, p); far |= !pt_fits(last, p); }
          if (keep_idx) N16[base + t - 1 - j].nxt = (uint16_t)(s - j);
        }
        t -= cnt;
        if (t) s = cnt == run ? sP[r] : s - cnt;
      }
      if (!wide && !__ballot(far)) {
        if (lane == 0) { Pw[-2] = (uint32_t)last.x | PT_COMPACT; Pw[-1] = (uint32_t)last.y; }
        break;
      }
    }
    if (lane == 0) lisl[item] = longest;
    my_points += longest;
    lds_fence();  // LDS reads of this strand done before the next strand's commit
#ifdef PBGPU_PROF
    {  // per tier (255: slots 24.., 511: 28..): order ticks, order rounds, forward ticks, strand ticks
      const uint64_t pw_t3 = __builtin_amdgcn_s_memtime();
      const int sb = SMAX == 255 ? 24 : 28;
      if (SMAX == 255 || SMAX == 511) {
        PROF_ADD(sb + 0, pw_t1 - pw_t0); PROF_ADD(sb + 1, pw_rounds); PROF_ADD(sb + 2, pw_t2 - pw_t1);
        PROF_ADD(sb + 3, pw_t3 - pw_t0);
      }
    }
#endif
  }
  tests = lane == 0 ? tests : 0;
  tests = wave_sum_u64(tests);
  if (lane == 0 && tests) atomicAdd(&stats[ST_LIS_TESTS], (unsigned long long)tests);
  if (SMAX <= LISW_TINY_N && lane == 0 && my_strands) {  // per-launch work of the timed tier (bench roofline)
    atomicAdd(&stats[ST_L0_HITS], (unsigned long long)my_hits);
    atomicAdd(&stats[ST_L0_STRANDS], (unsigned long long)my_strands);
    atomicAdd(&stats[ST_L0_POINTS], (unsigned long long)my_points);
  }
}

// compute_kmers_info (pb_aligner.cc:84-143) along one lis, one point at a
// time.  lens: unitig lengths along the fwd name (P.sr_ul, resolved once per
// aligner, so no dependent id -> length gather per chain); rev => bwd name
// (reversed list).
// Any error leaves n_info == 0 (the reference clears both vectors).
// T: the arrays' element type, int32_t (global) or lds_i32 (LDS): an LDS
// array must not be reached through a flat pointer, whose accesses wait for
// every outstanding global load (the row prefetch).
typedef __attribute__((address_space(3))) int32_t lds_i32;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;
// k_coords caches the unitig lengths of names of at most INFO_LDS_UNITIGS unitigs in LDS
constexpr uint32_t INFO_LDS_UNITIGS = 8, INFO_LDS = 2 * INFO_LDS_UNITIGS - 1;
// CT: the unitig-length cache's element type (lds_i32 in k_coords)
template <typename T, typename CT = T>
struct KmersInfo {
  const int32_t* lens;
  uint32_t nsz;
  bool rev, ok;
  int32_t k, uk;
  T* mers;    // element i at mers[i * stride]
  T* bases;
  uint32_t stride;
  CT* cl;  // optional cache: length of unitig i at cl[i * cstride]
  uint32_t cstride;
  uint32_t cunitig;
  int32_t cend, prev_pos;
  // Pending increments kept in registers: element 2c (pm, pb: the current
  // unitig c), 2c+1 (om, ob: its overlap with c+1) and 2c+2 (nm, nb: unitig
  // c+1), and nlen = ulen(c+1).  Points inside one unitig, and k-mers reaching
  // into the next one, touch no memory; moving to the next unitig writes 2c
  // and 2c+1 and makes 2c+2 the current element.  Overlaps reaching further
  // than the next unitig (unitigs shorter than a k-mer) update memory directly.
  int32_t pm, pb, om, ob, nm, nb, nlen;
  static constexpr int32_t UL_INVALID = INT32_MIN;
  DEV int32_t ulen_direct(uint32_t i) const { return i >= nsz ? UL_INVALID : lens[rev ? nsz - 1 - i : i]; }
  DEV int32_t ulen(uint32_t i) const {
    if (cl) return i < nsz ? cl[i * cstride] : UL_INVALID;
    return ulen_direct(i);
  }
  DEV T& M(uint32_t i) { return mers[i * stride]; }
  DEV T& B(uint32_t i) { return bases[i * stride]; }
  // x[i] += v as a no-return atomic add (each lane owns its elements): no read to
  // wait for -- the arrays are not read back here
  DEV void acc(T* x, uint32_t i, int32_t v) {
    if constexpr (std::is_same<T, lds_i32>::value) __atomic_fetch_add(x + i * stride, v, __ATOMIC_RELAXED);
    else __hip_atomic_fetch_add(x + i * stride, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  DEV void init(const AlignParamsDev& P, const int32_t* lens_, uint32_t nsz_, bool rev_, T* m, T* b,
                uint32_t stride_, CT* cache = nullptr, uint32_t cstride_ = 0) {
    lens = lens_; nsz = nsz_; rev = rev_; k = (int32_t)P.k; uk = (int32_t)P.unitigs_k;
    mers = m; bases = b; stride = stride_; cl = nullptr; cstride = cstride_;
    if (cache) {  // nsz <= INFO_LDS_UNITIGS: independent loads, issued together
      int32_t v[INFO_LDS_UNITIGS];
#pragma unroll
      for (uint32_t i = 0; i < INFO_LDS_UNITIGS; ++i) v[i] = i < nsz ? ulen_direct(i) : 0;
#pragma unroll
      for (uint32_t i = 0; i < INFO_LDS_UNITIGS; ++i) if (i < nsz) cache[i * cstride] = v[i];
      cl = cache;
    }
    start();
  }
  // the same with the name's lengths given (fwd order, SrMeta::ul) for nsz <= SR_META_UL:
  // the cache filled from registers, no loads
  DEV void init_pre(const AlignParamsDev& P, const int32_t (&f)[SR_META_UL], uint32_t nsz_, bool rev_, T* m, T* b,
                    uint32_t stride_, CT* cache, uint32_t cstride_) {
    lens = nullptr; nsz = nsz_; rev = rev_; k = (int32_t)P.k; uk = (int32_t)P.unitigs_k;
    mers = m; bases = b; stride = stride_; cl = cache; cstride = cstride_;
#pragma unroll
    for (uint32_t i = 0; i < SR_META_UL; ++i) {
      const uint32_t q = rev ? nsz - 1 - i : i;
      int32_t v = f[0];
#pragma unroll
      for (uint32_t j = 1; j < SR_META_UL; ++j) v = q == j ? f[j] : v;
      if (i < nsz) cache[i * cstride] = v;
    }
    start();
  }
  DEV void start() {
    const int32_t l0 = ulen(0);
    ok = l0 != UL_INVALID;
    if (!ok) return;
    for (uint32_t i = 0; i < 2 * nsz - 1; ++i) { M(i) = 0; B(i) = 0; }
    cunitig = 0;
    cend = l0;
    prev_pos = (int32_t)(0u - (uint32_t)k);
    pm = pb = om = ob = nm = nb = 0;
    nlen = ulen(1);
  }
  DEV void flush() {
    acc(mers, 2 * cunitig, pm); acc(bases, 2 * cunitig, pb);
    if (cunitig + 1 < nsz) {
      acc(mers, 2 * cunitig + 1, om); acc(bases, 2 * cunitig + 1, ob);
      acc(mers, 2 * cunitig + 2, nm); acc(bases, 2 * cunitig + 2, nb);
    }
    pm = pb = om = ob = nm = nb = 0;
  }
  // The same steps with no return: a lane whose name failed (!ok) keeps computing on
  // its stale state (its arrays are discarded) but never advances, so every memory
  // update stays inside its own 2 nsz - 1 elements; the advance is entered only when
  // a lane of the wave needs it.
  DEV void add(int32_t sr_pos) {
    const int32_t new_bases = k < sr_pos - prev_pos ? k : sr_pos - prev_pos;
    bool adv = ok & (sr_pos + k > cend + 1);
    if (__builtin_expect(__ballot(adv) != 0, 0)) {
      while (adv) {
        const bool part = cend >= sr_pos;  // the k-mer starts inside unitig c
        const bool bad = (part & (cunitig >= nsz - 1)) | (nlen == UL_INVALID);
        if (bad) { ok = false; break; }
        const int32_t mx = sr_pos > prev_pos + k ? sr_pos : prev_pos + k;
        const int32_t nbb = part ? cend - mx + 1 : 0;
        pb += nbb; ob += nbb;
        acc(mers, 2 * cunitig, pm); acc(bases, 2 * cunitig, pb);
        if (cunitig + 1 < nsz) { acc(mers, 2 * cunitig + 1, om); acc(bases, 2 * cunitig + 1, ob); }
        pm = nm; pb = nb; om = ob = nm = nb = 0;
        ++cunitig;
        cend = (int32_t)((uint32_t)cend + (uint32_t)nlen - (uint32_t)uk + 1u);
        nlen = ulen(cunitig + 1);
        adv = sr_pos + k > cend + 1;
      }
    }
    ++pm;
    pb += new_bases;
    const bool in_ov = ok & (cunitig < nsz - 1) & ((uint32_t)sr_pos + (uint32_t)k > (uint32_t)cend - (uint32_t)uk + 1u);
    const int32_t full_mer = (in_ov & (sr_pos + uk > cend + 1)) ? 1 : 0;
    const int32_t tt0 = sr_pos + k - cend + uk - 2;
    const int32_t nbb0 = in_ov ? (new_bases < tt0 ? new_bases : tt0) : 0;
    om += full_mer; nm += full_mer;
    ob += nbb0; nb += nbb0;
    int32_t cendi = (int32_t)((uint32_t)cend + (uint32_t)nlen - (uint32_t)uk + 1u);
    if (in_ov & ((nlen == UL_INVALID) |
                 ((cunitig + 1 < nsz - 1) & ((uint32_t)sr_pos + (uint32_t)k > (uint32_t)cendi - (uint32_t)uk + 1u)))) {
      if (nlen == UL_INVALID) {
        ok = false;
      } else {
        for (uint32_t i = cunitig + 1; (i < nsz - 1) && ((uint32_t)sr_pos + (uint32_t)k > (uint32_t)cendi - (uint32_t)uk + 1u); ++i) {
          const int32_t fm = sr_pos + uk > cendi + 1;
          acc(mers, 2 * i + 1, fm); acc(mers, 2 * i + 2, fm);
          const int32_t tt = sr_pos + k - cendi + uk - 2;
          const int32_t nbb = new_bases < tt ? new_bases : tt;
          acc(bases, 2 * i + 1, nbb); acc(bases, 2 * i + 2, nbb);
          const int32_t l = ulen(i + 1);
          if (l == UL_INVALID) { ok = false; break; }
          cendi = (int32_t)((uint32_t)cendi + (uint32_t)l - (uint32_t)uk + 1u);
        }
      }
    }
    prev_pos = sr_pos;
  }
};

// a / b correctly rounded from y = RN(1 / b): one correction makes q faithful,
// whose residual is then exact, and Markstein's step rounds it correctly
// (Handbook of Floating-Point Arithmetic, thm. "Markstein"); no over- or
// underflow here.  The sign of a zero quotient may differ from a / b, which
// no sum below can see (the accumulators are never -0).
DEV double div_rcp(double a, double b, double y) {
  const double q0 = __dmul_rn(a, y);
  const double q1 = __fma_rn(__fma_rn(-b, q0, a), y, q0);
  return __fma_rn(__fma_rn(-b, q1, a), y, q1);
}

// least_square_2d::add (least_square_2d.hpp:47-67), x = sr offset, y = pb offset;
// the four divisions by n share one correctly rounded reciprocal
// RN(1 / d) for an integer 1 <= d < 2^32: the compiler's __ddiv_rn(1.0, d) less the
// operand scaling (v_div_scale) and special-case fixup (v_div_fixup), which change
// nothing for such d -- the same reciprocal and Newton steps and the same final
// correction fma(1 - d y, y, y) (v_div_fmas without scaling).  7 instructions
// instead of 11; checked against __ddiv_rn for every d < 2^24 on the device
// (pbgpu_check_reciprocal, tests/test_gpu_edge.py).
DEV double recip_int(double d) {
  double y = __builtin_amdgcn_rcp(d);
  double e = __fma_rn(-d, y, 1.0);
  y = __fma_rn(y, e, y);
  e = __fma_rn(-d, y, 1.0);
  y = __fma_rn(y, e, y);
  const double r = __fma_rn(-d, y, 1.0);
  return __fma_rn(r, y, y);
}
__global__ void k_check_recip(uint32_t n_max, unsigned long long* bad) {
  unsigned long long nb = 0;
  for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x + 1; d <= n_max; d += gridDim.x * blockDim.x) {
    const double dd = (double)d;
    nb += __double_as_longlong(recip_int(dd)) != __double_as_longlong(__ddiv_rn(1.0, dd));
  }
  if (nb) atomicAdd(bad, nb);
}
void launch_check_recip(uint32_t n_max, unsigned long long* bad, hipStream_t st) {
  hipLaunchKernelGGL(k_check_recip, dim3(1024), dim3(256), 0, st, n_max, bad);
}
// (n as a 32-bit count with its double kept beside it, dn + 1 exact: the 64-bit long of
// the reference converts to double in five instructions a point)
struct Lsq {
  double EX = 0, EY = 0, EXX = 0, EXY = 0, VX = 0, CXY = 0, NB = 0, dn = 0;
  uint32_t n = 0;
  DEV void add(double x, double y) {
    ++n;
    dn = __dadd_rn(dn, 1.0);
    const double rn = recip_int(dn);
    const double deltaX = __dadd_rn(x, -EX);
    EX = __dadd_rn(EX, div_rcp(deltaX, dn, rn));
    const double ndeltaX = __dadd_rn(x, -EX);
    VX = __dadd_rn(VX, __dmul_rn(deltaX, ndeltaX));
    const double deltaY = __dadd_rn(y, -EY);
    EY = __dadd_rn(EY, div_rcp(deltaY, dn, rn));
    const double ndeltaY = __dadd_rn(y, -EY);
    const double deltaXX = __dadd_rn(__dmul_rn(x, x), -EXX);
    EXX = __dadd_rn(EXX, div_rcp(deltaXX, dn, rn));
    const double deltaXY = __dadd_rn(__dmul_rn(x, y), -EXY);
    EXY = __dadd_rn(EXY, div_rcp(deltaXY, dn, rn));
    CXY = __dadd_rn(CXY, __dmul_rn(deltaX, ndeltaY));
    NB = __dadd_rn(NB, __dadd_rn(__dmul_rn(deltaXY, ndeltaX), -__dmul_rn(deltaXX, ndeltaY)));
  }
};

// coords_info::canonicalize (pb_aligner.hpp:151-167) and the filters of
// align_sequence_max (coarse_aligner.cc:46-54): fabs(stretch)==0, min_mers
// (-M), min_bases (-B) (pb_aligner.hpp:169-174).  Returns true if kept.
DEV bool coords_finish(const AlignParamsDev& P, uint32_t rl, Rec& R) {
  const uint32_t k = P.k, ql = R.ql;
  if (R.qs < 0) {
    if (P.forward) {
      R.qs = (int32_t)(uint32_t)((uint64_t)ql + (uint64_t)(int64_t)R.qs - (uint64_t)k + 2ull);
      R.qe = (int32_t)(uint32_t)((uint64_t)ql + (uint64_t)(int64_t)R.qe + 1ull);
      R.flags |= 1u;
      R.offset = __dadd_rn(R.offset, -__dadd_rn(__dmul_rn(R.stretch, (double)((uint64_t)ql + 1ull)), -(double)k));
    } else {
      R.qs = (int32_t)((uint32_t)(-R.qs) + k - 1u);
      R.qe = -R.qe;
      R.stretch = -R.stretch;
      R.offset = __dadd_rn(R.offset, (double)(k - 1u));
    }
  } else {
    R.qe = (int32_t)((uint32_t)R.qe + k - 1u);
  }
  if (P.fine) return true;  // fine_aligner.cc:47-48 pushes every window's info unfiltered
  if (fabs(R.stretch) == 0.0) return false;
  const double drl = (double)rl;
  double vs = __dadd_rn(R.stretch, R.offset);
  double ims = drl < vs ? drl : vs; ims = 1.0 > ims ? 1.0 : ims;
  double ve = __dadd_rn(__dmul_rn(R.stretch, (double)ql), R.offset);
  double ime = drl < ve ? drl : ve; ime = 1.0 > ime ? 1.0 : ime;
  const long lr = (long)rint(__dadd_rn(ime, -ims));
  const int32_t imp_len = (int32_t)((lr < 0 ? -lr : lr) + 1);
  if (P.mers_factor != 0.0 &&
      !(__dmul_rn(P.mers_factor, (double)((uint32_t)imp_len - k + 1u)) <= (double)R.nb_mers)) return false;
  if (P.bases_factor > 0.0 &&
      !(__dmul_rn(P.bases_factor, (double)(imp_len - 2 * (int32_t)k)) <= (double)R.pb_cover)) return false;
  return true;
}

// One lane per chain: coarse_aligner::align_sequence_max's loop body
// (coarse_aligner.cc:42-60) for one emission -- pick the strand
// (pb_aligner.cc:15, |fwd.lis| >= |bwd.lis|), compute_coords_info
// (pb_aligner.cc:11-82) over its lis points (staged through LDS in aligned
// chunks), filters, kmers_info.  kmers_info of super-reads with at most
// INFO_LDS_UNITIGS unitigs is accumulated in LDS during the first pass and
// written once if the record is kept; longer names use a third pass that
// updates the arrays in HBM.  With --max-match, kept chains go to the redo list.
// One lane's lis (pt_get's two layouts) streamed in order through the LDS
// tile: the compact lanes' words in 2*CH-word rows, then the wide lanes'
// points in CH-point rows (a lane takes part in one of the two loops).
template <int CH>
struct LisStream {
  int2 last;
  bool cmp;
  uint64_t base;
  DEV void init(const int2* pts, uint64_t base_, uint32_t nl) {
    base = base_; cmp = false; last = make_int2(0, 0);
    if (nl) {
      const uint2 h = *(const uint2*)(pts + base);
      cmp = (h.x & PT_COMPACT) != 0;
      last = make_int2((int32_t)(h.x & ~PT_COMPACT), (int32_t)h.y);
    }
  }
  template <typename F>
  DEV void run(const int2* pts, uint32_t n, int2* tile, F&& f) const {
    ChunkGrid<2 * CH> gc;
    gc.init(2 * base + 2, cmp ? n : 0);
    ChunkGrid<CH> gw;
    gw.init(base, cmp ? 0 : n);
    const uint32_t ncc = wave_max_u32(gc.chunks()), ncw = wave_max_u32(gw.chunks());
    const int2 l = last;
    stream_rows<2 * CH>((const uint32_t*)pts, gc, ncc, (uint32_t*)tile, [&](const uint32_t w) { f(pt_decode(l, w)); });
    stream_rows<CH>(pts, gw, ncw, tile, f);
  }
};
template <int CH>
__global__ __launch_bounds__(64) void k_coords(IndexView ix, AlignParamsDev P, const ChainDesc* __restrict__ chains,
                                               const uint32_t* __restrict__ list, uint32_t n,
                                               const uint64_t* __restrict__ roff, uint32_t emit, ChainOut O) {
  __shared__ int2 ps[CH * RS];
  __shared__ int32_t im[INFO_LDS * 64], ib[INFO_LDS * 64], iul[INFO_LDS_UNITIGS * 64];
  const int lane = lane_id();
  PROF_T(kc_t0);
  const uint32_t w = blockIdx.x * 64 + lane;
  const bool act = w < n;
  uint32_t c = 0, nl = 0;
  uint64_t base = 0;
  bool fwd_align = true;
  ChainDesc d{};
  if (act) {
    c = list[w];
    d = chains[c];
    const uint32_t lf = O.lisl[2 * c], lb = O.lisl[2 * c + 1];
    fwd_align = lf >= lb;
    nl = fwd_align ? lf : lb;
    base = d.hit_base + (fwd_align ? 0 : d.nf);
  }
  LisStream<CH> LS;
  LS.init(O.pts, base, act ? nl : 0);
  const uint32_t k = P.k;
  Rec R;
  R.nb_mers = (int32_t)nl; R.pb_cons = 0; R.sr_cons = 0; R.pb_cover = k; R.sr_cover = k;
  // the super-read's length, name range and first unitig lengths: one 32-byte SrMeta line
  // (kmers_info runs) instead of sr_start, sr_uoff and sr_ul, three random sectors a chain
  SrMeta sm{};
  if (act && P.sr_meta) {
    const uint4* mp = reinterpret_cast<const uint4*>(P.sr_meta + d.sr);
    const uint4 m0 = mp[0], m1 = mp[1];
    sm.ql = m0.x; sm.u0 = m0.y; sm.nsz = m0.z;
    sm.ul[0] = (int32_t)m0.w; sm.ul[1] = (int32_t)m1.x; sm.ul[2] = (int32_t)m1.y; sm.ul[3] = (int32_t)m1.z;
    sm.ul[4] = (int32_t)m1.w;
  }
  R.ql = !act ? 0u : P.sr_meta ? sm.ql : (uint32_t)(ix.sr_start[d.sr + 1] - ix.sr_start[d.sr]);
  // the read length is needed only by the filters at the end: loaded here, with the other
  // descriptor-dependent loads, so it does not stall the wave after the passes
  const uint32_t rl = act ? (uint32_t)(roff[d.read + 1] - roff[d.read]) : 0;
  R.sr = d.sr; R.read = d.read; R.flags = (P.forward && !fwd_align) ? 2u : 0u;
  R.n_info = 0; R.reserved = 0; R.info_off = 0; R.emit = O.emit_of ? (act ? O.emit_of[c] : 0u) : emit;
  R.stretch = 0; R.offset = 0; R.avg_err = 0;
  // kmers_info setup (pb_aligner.cc:62-81): unitig list of the name used for the record
  uint32_t u0 = 0, nsz = 0;
  if (act && nl && P.unitigs_k) {
    if (P.sr_meta) { u0 = sm.u0; nsz = sm.nsz; }
    else { u0 = ix.sr_uoff[d.sr]; nsz = ix.sr_uoff[d.sr + 1] - u0; }
  }
  const bool info_lds = nsz && nsz <= INFO_LDS_UNITIGS;
  KmersInfo<lds_i32> KI;
  if (info_lds) {
    if (P.sr_meta && nsz <= SR_META_UL)
      KI.init_pre(P, sm.ul, nsz, (R.flags & 2u) != 0, (lds_i32*)(im + lane), (lds_i32*)(ib + lane), 64,
                  (lds_i32*)(iul + lane), 64);
    else
      KI.init(P, P.sr_ul + u0, nsz, (R.flags & 2u) != 0, (lds_i32*)(im + lane), (lds_i32*)(ib + lane), 64,
              (lds_i32*)(iul + lane), 64);
  }
  auto info_pos = [&](int32_t so) -> int32_t {
    const int32_t pos = fwd_align ? so : (int32_t)(R.ql + (uint32_t)so - k + 2u);
    return pos < 0 ? -pos : pos;
  };
  // pass 1: cons / cover and the least-squares fit (pb_aligner.cc:19-47)
  Lsq L;
  int2 prev = make_int2(0, 0), first = make_int2(0, 0);
  PROF_T(kc_t1);
#ifdef PBGPU_EXP_NO_PASS1
  LS.run(O.pts, 0, ps, [&](const int2 p) {
#else
  LS.run(O.pts, nl, ps, [&](const int2 p) {
#endif
    // consecutive / covered counts against the previous point, branch-free (the first
    // point adds nothing: its diffs are masked)
    const bool later = L.n != 0;
    first = later ? first : p;
    const uint32_t pb_diff = (uint32_t)(p.x - prev.x), sr_diff = (uint32_t)(p.y - prev.y);
    R.pb_cons += (later & (pb_diff == 1u)) ? 1u : 0u;
    R.pb_cover += later ? (k < pb_diff ? k : pb_diff) : 0u;
    R.sr_cons += (later & (sr_diff == 1u)) ? 1u : 0u;
    R.sr_cover += later ? (k < sr_diff ? k : sr_diff) : 0u;
#ifndef PBGPU_EXP_NO_LSQ
    L.add((double)p.y, (double)p.x);
#else
    ++L.n; L.EX += p.y;
#endif
    prev = p;
  });
  // pass 2: average error of the fit (least_square_2d.hpp:70-80 + pb_aligner.cc:49-60) and kmers_info
  PROF_T(kc_t2);
  double a = 0, b = 0;
  if (L.n == 1) {
    R.stretch = 1.0; R.offset = __dadd_rn(L.EY, -L.EX); R.avg_err = 0;
  } else if (L.n > 1) {
    a = __ddiv_rn(L.CXY, L.VX); b = __ddiv_rn(L.NB, L.VX);
    R.stretch = a; R.offset = b;
  }
  R.rs = first.x;
  R.re = (int32_t)((uint32_t)prev.x + k - 1u);
  R.qs = first.y; R.qe = prev.y;
  // the filters read neither the average error nor kmers_info (coords_finish), so they run
  // before pass 2 and a dropped chain skips it
  const bool keep = act && nl > 0 && coords_finish(P, rl, R);
  double err = 0;
  // kmers_info (LDS case) rides this pass, not the fit's: the fit's registers are dead
  // here, and the pass then also runs for single-point chains (-0.6 ms, r04b).  (Round 5
  // tried the arrays in HBM, allocated before this pass, to free the 7.7 KB of LDS a wave
  // that limits the kernel's occupancy: 21.0 -> 23.9 ms, the atomics cost more.)
#ifdef PBGPU_EXP_NO_PASS2
  LS.run(O.pts, 0, ps, [&](const int2 p) {
#else
  LS.run(O.pts, (keep && (L.n > 1 || info_lds)) ? nl : 0, ps, [&](const int2 p) {
#endif
#ifndef PBGPU_EXP_NO_INFO
    if (info_lds) KI.add(info_pos(p.y));
#endif
    err = __dadd_rn(err, fabs(__dadd_rn(__dadd_rn(__dmul_rn(a, (double)p.y), b), -(double)p.x)));
  });
  if (L.n > 1) R.avg_err = __ddiv_rn(err, L.dn);
  PROF_T(kc_t3);
  // info arrays: allocate for kept records, copy the LDS case, or run pass 3 in HBM
  bool info_ok = true, pass3 = false;
  KmersInfo<int32_t> KG;  // pass 3: the arrays in HBM
  if (keep && nsz) {
    const uint32_t need = 2 * nsz - 1;
    const unsigned long long io = atomicAdd(O.info_count, (unsigned long long)need);
    if (io + need <= O.info_cap) {
      R.info_off = io;
      if (info_lds) {
        if (KI.ok) {
          KI.flush();
          for (uint32_t q = 0; q < need; ++q) { O.info_m[io + q] = im[q * 64 + lane]; O.info_b[io + q] = ib[q * 64 + lane]; }
          R.n_info = need;
        }
      } else {
        KG.init(P, P.sr_ul + u0, nsz, (R.flags & 2u) != 0, O.info_m + io, O.info_b + io, 1);
        pass3 = KG.ok;
      }
    } else {
      info_ok = false;
    }
  }
  PROF_T(kc_t4);
  LS.run(O.pts, pass3 ? nl : 0, ps, [&](const int2 p) { KG.add(info_pos(p.y)); });
  if (pass3 && KG.ok) { KG.flush(); R.n_info = 2 * nsz - 1; }
  PROF_T(kc_t5);
  if (keep) {
    const uint32_t ri = atomicAdd(O.rec_count, 1u);
    if (ri < O.rec_cap && info_ok) {
      O.recs[ri] = R; O.rec_read[ri] = R.read;
      if (O.per_read) O.rec_slot[ri] = atomicAdd(&O.per_read[R.read], 1u);
    } else {
      atomicAdd(&O.stats[ST_REC_OVERFLOW], 1ull);
    }
    if (P.max_match) O.redo[atomicAdd(O.n_redo, 1u)] = c;
  }
#ifdef PBGPU_PROF
  {  // slots 32..: waves, total, prologue, pass 1, pass 2, gap, pass 3, chunks; per-log2(chunks) ticks / waves
    PROF_T(kc_t6);
    const uint32_t lane_ch = (nl + CH - 1) / CH;
    unsigned long long sum_ch = lane_ch;
    for (int o = 32; o > 0; o >>= 1) sum_ch += __shfl_xor(sum_ch, o, 64);
    const uint32_t nch = wave_max_u32(lane_ch);
    const uint32_t bk = nch ? 32 - __builtin_clz(nch) : 0;
    PROF_ADD(32, 1); PROF_ADD(33, kc_t6 - kc_t0); PROF_ADD(34, kc_t1 - kc_t0); PROF_ADD(35, kc_t2 - kc_t1);
    PROF_ADD(36, kc_t3 - kc_t2); PROF_ADD(37, kc_t4 - kc_t3); PROF_ADD(38, kc_t5 - kc_t4); PROF_ADD(39, nch);
    PROF_ADD(40, sum_ch); PROF_ADD(41, __ballot(pass3) ? 1 : 0); PROF_ADD(42, kc_t6 - kc_t5);
    PROF_ADD(48 + (bk > 15 ? 15 : bk), kc_t6 - kc_t0); PROF_ADD(64 + (bk > 15 ? 15 : bk), 1);
  }
#endif
}

// --max-match: mer_lists::discard_update_LIS (pb_aligner.hpp:86-92) drops the
// longer lis (bwd on ties) from its strand; off_lis::discard_LIS
// (pb_aligner.hpp:47-61) keeps the remaining offsets in order.  The strand
// goes to the small- or big-node k_lis list for the next round.
__global__ void k_discard(const ChainDesc* __restrict__ chains, const uint32_t* __restrict__ list, uint32_t n,
                          const uint32_t* __restrict__ lisl, uint32_t* __restrict__ slen, int2* __restrict__ X,
                          const LNode<uint16_t>* __restrict__ N16, const LNode<uint32_t>* __restrict__ N32,
                          const uint32_t* __restrict__ nshift, uint32_t* items_small, uint32_t* n_small,
                          uint32_t* items_big, uint32_t* n_big) {
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < n; w += gridDim.x * blockDim.x) {
    const uint32_t c = list[w];
    const ChainDesc d = chains[c];
    const uint32_t lf = lisl[2 * c], lb = lisl[2 * c + 1];
    const bool dF = lf > lb;
    const uint32_t item = 2 * c + (dF ? 0u : 1u);
    const uint64_t base = d.hit_base + (dF ? 0 : d.nf);
    const uint32_t nD = slen[item], lD = dF ? lf : lb;
    int2* XD = X + base;
    // k_node32_place's layout: chunk nshift[item] holds the strand's first CH-aligned row
    const uint64_t base32 = nD <= LIS_U16_MAX ? 0 : (uint64_t)nshift[item] * LIS_CH32 + (base & (LIS_CH32 - 1));
    auto lis_at = [&](uint32_t t) -> uint32_t { return nD <= LIS_U16_MAX ? N16[base + t].nxt : N32[base32 + t].nxt; };
    uint32_t wpos = 0, li = 0, next = lD ? lis_at(0) : 0xFFFFFFFFu;
    for (uint32_t rpos = 0; rpos < nD; ++rpos) {
      if (rpos == next) { ++li; next = li < lD ? lis_at(li) : 0xFFFFFFFFu; continue; }
      XD[wpos++] = XD[rpos];
    }
    const uint32_t nn = nD - lD;
    slen[item] = nn;
    if (nn <= LIS_U16_MAX) items_small[atomicAdd(n_small, 1u)] = item;
    else items_big[atomicAdd(n_big, 1u)] = item;
  }
}

// 32-bit LIS nodes for the strands of more than LIS_U16_MAX hits only: each
// such strand gets the CH-aligned chunks its hit range spans, at an offset from
// one atomic counter (placement order is immaterial), so the node array holds
// those strands' hits, not the sub-batch's (it was 16 B per hit of the whole
// sub-batch: a multi-GB late allocation on the first batch with a long strand).
template <int CH>
__global__ void k_node32_place(const ChainDesc* __restrict__ chains, const uint32_t* __restrict__ items, uint32_t n,
                               const uint32_t* __restrict__ slen, uint32_t* __restrict__ nshift,
                               unsigned long long* __restrict__ total_chunks) {
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < n; w += gridDim.x * blockDim.x) {
    const uint32_t item = items[w];
    const ChainDesc d = chains[item >> 1];
    const uint64_t base = d.hit_base + ((item & 1) ? d.nf : 0);
    const uint64_t a0 = base & ~(uint64_t)(CH - 1);
    const uint64_t nchunks = (base - a0 + slen[item] + CH - 1) / CH;
    nshift[item] = (uint32_t)atomicAdd(total_chunks, (unsigned long long)nchunks);
  }
}
__global__ void k_init_slen(const ChainDesc* __restrict__ chains, uint32_t n, uint32_t* slen) {
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
    const ChainDesc d = chains[c];
    slen[2 * c] = d.nf; slen[2 * c + 1] = d.nb;
  }
}

// ============================================================= fine (-F)
// fine_aligner::thread::align_sequence (fine_aligner.cc:38-51): one window per
// coarse record (prime_frags_pos, fine_aligner.hpp:50-58), every fine_k-mer of
// the read looked up in the fine sub-index with no SSR / toggle / count
// filter, each occurrence kept in every window of its super-read whose
// [begin, end] holds the k-mer's pb offset (fetch_local_super_reads,
// fine_aligner.cc:7-36).  The windowed hits then go through the same LIS
// (accept_all) and k_coords (forward, no filters) as the coarse chains.

// windows sorted by (read, super-read): keys, then FineWin records
__global__ void k_fine_win_keys(const Rec* __restrict__ recs, uint32_t n, uint64_t* keys, uint32_t* idx) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    keys[i] = (uint64_t)recs[i].read << 32 | recs[i].sr;
    idx[i] = i;
  }
}
__global__ void k_fine_win_fill(const Rec* __restrict__ recs, const uint32_t* __restrict__ idx, uint32_t n,
                                const uint64_t* __restrict__ roff, uint32_t fk, FineWin* __restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t w = idx[i];
    const Rec R = recs[w];
    const double rl = (double)(roff[R.read + 1] - roff[R.read]);
    // begin = max(0, stretch + offset - avg_err); end = min(rl, stretch * ql + offset + avg_err - align_k)
    const double b = __dadd_rn(__dadd_rn(R.stretch, R.offset), -R.avg_err);
    const double e = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(R.stretch, (double)R.ql), R.offset), R.avg_err), -(double)fk);
    FineWin W;
    W.sr = R.sr; W.w = w;
    W.begin = 0.0 < b ? b : 0.0;
    W.end = e < rl ? e : rl;
    out[i] = W;
  }
}

constexpr int FINE_BLOCK = 256;
constexpr uint32_t FINE_LDS_WIN = 4096, FINE_BITS = 1u << 16;
DEV uint32_t fine_hash(uint32_t sr) { return (sr * 0x9E3779B1u) >> 16; }

// One workgroup per read, one fine_k-mer per thread and step.  EMIT = false:
// the read's windowed hit count.  EMIT = true: each step counts its threads'
// hits, scans, and writes them in (k-mer, occurrence) order -- the list
// order of fetch_local_super_reads -- as (list key, (pb offset, sr offset)),
// list key = 2 * window + (bwd).  A stable sort by key then yields every
// window's fwd and bwd lists in order.
template <bool EMIT>
__global__ __launch_bounds__(FINE_BLOCK) void k_fine_hits(IndexView fx, const uint8_t* __restrict__ seq,
                                                          const uint64_t* __restrict__ roff, uint32_t r0,
                                                          const FineWin* __restrict__ win,
                                                          const uint64_t* __restrict__ woff,
                                                          uint64_t* __restrict__ read_hits,
                                                          const uint64_t* __restrict__ hit_off, uint64_t w_sub0,
                                                          uint32_t* __restrict__ keys, int2* __restrict__ vals,
                                                          unsigned long long* stats) {
  __shared__ uint32_t s_bits[FINE_BITS / 32];
  __shared__ uint32_t s_sr[FINE_LDS_WIN];
  __shared__ uint32_t s_tmp[FINE_BLOCK / 64];
  __shared__ uint64_t s_tmp64[FINE_BLOCK / 64];
  const uint32_t r = r0 + blockIdx.x;
  const int tid = threadIdx.x;
  const uint64_t w0 = woff[r];
  const uint32_t nw = (uint32_t)(woff[r + 1] - w0);
  if (nw == 0) {
    if (!EMIT && tid == 0) read_hits[r] = 0;
    return;
  }
  for (uint32_t i = tid; i < FINE_BITS / 32; i += FINE_BLOCK) s_bits[i] = 0;
  __syncthreads();
  const bool lds = nw <= FINE_LDS_WIN;
  for (uint32_t i = tid; i < nw; i += FINE_BLOCK) {
    const uint32_t sr = win[w0 + i].sr, h = fine_hash(sr);
    atomicOr(&s_bits[h >> 5], 1u << (h & 31));
    if (lds) s_sr[i] = sr;
  }
  __syncthreads();
  auto sr_at = [&](uint32_t i) -> uint32_t { return lds ? s_sr[i] : win[w0 + i].sr; };
  const uint64_t base = roff[r];
  const int64_t L = (int64_t)(roff[r + 1] - base);
  const uint32_t k = fx.k;
  const uint32_t hs = 2 * (k - 1);
  uint64_t out = EMIT ? hit_off[r] : 0, total = 0;
  for (int64_t t0 = 0; t0 < L; t0 += FINE_BLOCK) {
    const int64_t p = t0 + tid;  // k-mer start, 0-based
    bool valid = p + (int64_t)k <= L;
    uint64_t m = 0, rm = 0;
    if (valid) {
      for (uint32_t j = 0; j < k; ++j) {
        const int c = base_code(seq[base + p + j]);
        if (c < 0) { valid = false; break; }
        m = (m << 2) | (uint64_t)c;
        rm = (rm >> 2) | ((uint64_t)(3 - c) << hs);
      }
    }
    uint64_t ptr = 0;
    bool found = false;
    if (valid) {
      uint64_t payload; uint32_t pr = 0;
      found = table_lookup(fx, m < rm ? m : rm, payload, pr);
      ptr = payload >> 24;
    }
    const int32_t o = (int32_t)(p + 1);  // parser.offset<0>(), 1-based
    const bool canon = m < rm;
    // occ(a) then occ(b), a = the canonical k-mer (find_pos_size, superread_parser.hpp:183-192)
    auto walk = [&](auto&& emit) {
      if (!found) return;
      const uint64_t h0 = fx.occ[ptr], h1 = fx.occ[ptr + 1];
      const bool pal = (h0 >> 32) & 1;
      const uint32_t nA = (uint32_t)h1, nB = (uint32_t)(h1 >> 32);
      for (int half = 0; half < 2; ++half) {
        const bool useB = half && !pal;
        const uint64_t lst = ptr + 2 + (useB ? nA : 0);
        const uint32_t nl = useB ? nB : nA;
        for (uint32_t j = 0; j < nl; ++j) {
          const uint64_t v = fx.occ[lst + j];
          const uint32_t sr = (uint32_t)(v >> 32), h = fine_hash(sr);
          if (!((s_bits[h >> 5] >> (h & 31)) & 1u)) continue;
          uint32_t lo = 0, hi = nw;
          while (lo < hi) { const uint32_t md = (lo + hi) >> 1; if (sr_at(md) < sr) lo = md + 1; else hi = md; }
          if (lo == nw || sr_at(lo) != sr) continue;
          const int32_t off = (int32_t)(uint32_t)v;
          const int32_t it_off = half ? -off : off;
          const int32_t fin = canon ? it_off : -it_off;
          for (uint32_t q = lo; q < nw && sr_at(q) == sr; ++q) {
            const FineWin W = win[w0 + q];
            if ((double)o >= W.begin && (double)o <= W.end) emit(W.w, fin);
          }
        }
      }
    };
    uint32_t cnt = 0;
    walk([&](uint32_t, int32_t) { ++cnt; });
    if constexpr (EMIT) {
      uint32_t tot;
      uint64_t at = out + block_excl_scan<FINE_BLOCK>(cnt, s_tmp, tot);
      walk([&](uint32_t w, int32_t fin) {
        keys[at] = 2u * (uint32_t)(w - w_sub0) + (fin < 0 ? 1u : 0u);
        vals[at] = make_int2(o, fin);
        ++at;
      });
      out += tot;
      total += tot;
    } else {
      total += cnt;
    }
  }
  if constexpr (EMIT) {
    if (tid == 0 && total) atomicAdd(&stats[ST_FINE_HITS], (unsigned long long)total);
  } else {
    const uint64_t t = block_sum_u64<FINE_BLOCK>(total, s_tmp64);
    if (tid == 0) read_hits[r] = t;
  }
}

// first / one-past-last position of every list key in the sorted hits
__global__ void k_list_bounds(const uint32_t* __restrict__ keys, uint64_t G, uint32_t* lstart, uint32_t* lend) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < G; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t key = keys[i];
    if (i == 0 || keys[i - 1] != key) lstart[key] = (uint32_t)i;
    if (i + 1 == G || keys[i + 1] != key) lend[key] = (uint32_t)(i + 1);
  }
}

// one chain per window (its coarse record): lists, emission index, kmers_info capacity
__global__ void k_fine_desc(IndexView ix, const Rec* __restrict__ recs, uint64_t w_sub0, uint32_t nwin,
                            const uint32_t* __restrict__ lstart, const uint32_t* __restrict__ lend, int with_info,
                            ChainDesc* chains, uint32_t* emit_of, unsigned long long* info_need) {
  uint64_t need = 0;
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < nwin; c += gridDim.x * blockDim.x) {
    const Rec R = recs[w_sub0 + c];
    const uint32_t nf = lend[2 * c] - lstart[2 * c], nb = lend[2 * c + 1] - lstart[2 * c + 1];
    ChainDesc d;
    d.read = R.read; d.sr = R.sr; d.nf = nf; d.nb = nb;
    d.hit_base = nf ? lstart[2 * c] : lstart[2 * c + 1];
    chains[c] = d;
    emit_of[c] = R.emit;
    const uint32_t nsz = ix.sr_uoff[R.sr + 1] - ix.sr_uoff[R.sr];
    if (with_info && nsz && (nf || nb)) need += 2 * nsz - 1;
  }
  need = wave_sum_u64(need);
  if (lane_id() == 0 && need) atomicAdd(info_need, (unsigned long long)need);
}

// windows without a hit: compute_coords_info returns right after the ctor
// (pb_aligner.cc:27) and the record is still pushed (fine_aligner.cc:47).  Its
// rs/re/qs/qe are uninitialized upstream; they are 0 here (as in the oracle).
__global__ void k_fine_empty(IndexView ix, uint32_t k, const ChainDesc* __restrict__ chains, uint32_t n,
                             const uint32_t* __restrict__ lisl, const uint32_t* __restrict__ emit_of, ChainOut O) {
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
    if (lisl[2 * c] | lisl[2 * c + 1]) continue;
    const ChainDesc d = chains[c];
    Rec R;
    R.rs = R.re = R.qs = R.qe = 0; R.nb_mers = 0;
    R.pb_cons = R.sr_cons = 0; R.pb_cover = R.sr_cover = k;
    R.ql = (uint32_t)(ix.sr_start[d.sr + 1] - ix.sr_start[d.sr]);
    R.sr = d.sr; R.read = d.read; R.emit = emit_of[c]; R.flags = 0; R.n_info = 0; R.reserved = 0; R.info_off = 0;
    R.stretch = 0; R.offset = 0; R.avg_err = 0;
    const uint32_t ri = atomicAdd(O.rec_count, 1u);
    if (ri < O.rec_cap) { O.recs[ri] = R; O.rec_read[ri] = R.read; }
    else atomicAdd(&O.stats[ST_REC_OVERFLOW], 1ull);
  }
}

// =============================================================== records
__global__ void k_rec_hist(const uint32_t* rec_read, uint32_t n, uint32_t* per_read) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    atomicAdd(&per_read[rec_read[i]], 1u);
}
__global__ void k_rec_place(const uint32_t* __restrict__ rec_read, const uint32_t* __restrict__ rec_slot, uint32_t n,
                            const uint64_t* __restrict__ rec_off, uint32_t* __restrict__ order) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    order[rec_off[rec_read[i]] + rec_slot[i]] = i;
}
__global__ void k_rec_scatter(const uint32_t* rec_read, uint32_t n, const uint64_t* rec_off, uint32_t* cursor,
                              uint32_t* order) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t r = rec_read[i];
    order[rec_off[r] + atomicAdd(&cursor[r], 1u)] = i;
  }
}

// Sort key of a record within its read: (rs, re, ql, sr, emit) as two u64 words
// plus a tie word (emit, then the read-local slot, which never decides since
// (sr, emit) is unique per read).  Signed rs/re are biased so u64 order = int order.
DEV uint64_t rec_key_hi(const Rec& r) {
  return ((uint64_t)((uint32_t)r.rs ^ 0x80000000u) << 32) | (uint32_t)((uint32_t)r.re ^ 0x80000000u);
}
DEV uint64_t rec_key_lo(const Rec& r) { return ((uint64_t)r.ql << 32) | r.sr; }

// Bitonic network over staged keys: pair p -> (i, i + j), all threads busy.
template <int BLOCK, typename EX>
DEV void bitonic_keys(uint64_t* hi, uint64_t* lo, EX* ex, uint32_t np2) {
  for (uint32_t kk = 2; kk <= np2; kk <<= 1) {
    for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
      for (uint32_t p = threadIdx.x; p < (np2 >> 1); p += BLOCK) {
        const uint32_t i = ((p & ~(j - 1)) << 1) | (p & (j - 1)), l = i + j;
        const uint64_t h0 = hi[i], h1 = hi[l], l0 = lo[i], l1 = lo[l];
        const EX e0 = ex[i], e1 = ex[l];
        const bool gt = (h0 > h1) | ((h0 == h1) & ((l0 > l1) | ((l0 == l1) & (e0 > e1))));
        if (gt == ((i & kk) == 0)) { hi[i] = h1; hi[l] = h0; lo[i] = l1; lo[l] = l0; ex[i] = e1; ex[l] = e0; }
      }
      __syncthreads();
    }
  }
}

// One block per read of at most LCAP records: stage the sort keys of the read's
// records in LDS, sort them with a bitonic network, then gather the records in that
// order (padding entries carry all-ones keys and sort last).  A read of more records
// is only registered here: its ceil(n / LCAP) tiles go to a list (tiles[], counted in
// ctr[0], the largest such read in ctr[1]) for k_rec_tile_sort / k_rec_merge /
// k_rec_gather.  (Round 5 sorted such a read with one block running the bitonic network
// over HBM scratch padded to a power of two: 136 global passes at 65536 records, 0.04
// of HBM peak on C4-shaped reads.)
template <int BLOCK, int LCAP>
__global__ __launch_bounds__(BLOCK) void k_rec_sort(const Rec* __restrict__ recs, const uint64_t* __restrict__ rec_off,
                                                    const uint32_t* __restrict__ order_in, uint32_t n_reads,
                                                    Rec* __restrict__ out, uint2* __restrict__ tiles,
                                                    uint32_t* __restrict__ ctr) {
  static_assert(LCAP <= 4096, "LDS tie word holds a 12-bit slot");
  __shared__ uint64_t s_hi[LCAP], s_lo[LCAP];
  __shared__ uint32_t s_ex[LCAP];
  const uint32_t r = blockIdx.x;
  if (r >= n_reads) return;
  const uint64_t b = rec_off[r];
  const uint32_t n = (uint32_t)(rec_off[r + 1] - b);
  if (n == 0) return;
  if (n > LCAP) {
    const uint32_t t = (n + LCAP - 1) / LCAP;
    __shared__ uint32_t s_base;
    if (threadIdx.x == 0) {
      s_base = atomicAdd(&ctr[0], t);
      atomicMax(&ctr[1], n);
    }
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < t; c += BLOCK) tiles[s_base + c] = make_uint2(r, c);
    return;
  }
  uint32_t np2 = 1;
  while (np2 < n) np2 <<= 1;
  for (uint32_t i = threadIdx.x; i < np2; i += BLOCK) {
    if (i < n) {
      const Rec& R = recs[order_in[b + i]];
      s_hi[i] = rec_key_hi(R); s_lo[i] = rec_key_lo(R); s_ex[i] = (R.emit << 12) | i;
    } else {
      s_hi[i] = ~0ull; s_lo[i] = ~0ull; s_ex[i] = ~0u;
    }
  }
  __syncthreads();
  bitonic_keys<BLOCK>(s_hi, s_lo, s_ex, np2);
  for (uint32_t i = threadIdx.x; i < n; i += BLOCK) out[b + i] = recs[order_in[b + (s_ex[i] & 0xFFFu)]];
}

// The keys of a long read in HBM, two buffers of {hi[n], lo[n], ex[n]} per read at its
// record offset (A: 3 b words on, B: 3 nrec + 3 b on; 6 words a record in all); ex =
// emit << 32 | the record's read-local index, so keys are unique within a read.
struct RecKeys {
  uint64_t *hi, *lo, *ex;
};
DEV RecKeys rec_keys(uint64_t* scratch, uint64_t b, uint32_t n, uint64_t buf_off) {
  uint64_t* h = scratch + buf_off + 3 * b;
  return RecKeys{h, h + n, h + 2 * (uint64_t)n};
}
DEV bool key_lt(uint64_t h0, uint64_t l0, uint64_t e0, uint64_t h1, uint64_t l1, uint64_t e1) {
  return (h0 < h1) | ((h0 == h1) & ((l0 < l1) | ((l0 == l1) & (e0 < e1))));
}
// merge passes a read of n records needs after its tiles are sorted: ceil(log2(tiles))
DEV uint32_t rec_merge_passes(uint32_t n, uint32_t lcap) {
  uint32_t p = 0;
  while (((uint64_t)lcap << p) < n) ++p;
  return p;
}

// Tile c of a long read: its <= LCAP keys sorted in LDS, written to buffer A
template <int BLOCK, int LCAP>
__global__ __launch_bounds__(BLOCK) void k_rec_tile_sort(const Rec* __restrict__ recs,
                                                         const uint64_t* __restrict__ rec_off,
                                                         const uint32_t* __restrict__ order_in,
                                                         const uint2* __restrict__ tiles, const uint32_t* ctr,
                                                         uint64_t* scratch) {
  __shared__ uint64_t s_hi[LCAP], s_lo[LCAP], s_ex[LCAP];
  const uint32_t n_items = ctr[0];
  for (uint32_t it = blockIdx.x; it < n_items; it += gridDim.x) {
    const uint2 tc = tiles[it];
    const uint64_t b = rec_off[tc.x];
    const uint32_t n = (uint32_t)(rec_off[tc.x + 1] - b);
    const uint32_t i0 = tc.y * LCAP, cnt = min((uint32_t)LCAP, n - i0);
    uint32_t np2 = 1;
    while (np2 < cnt) np2 <<= 1;
    for (uint32_t i = threadIdx.x; i < np2; i += BLOCK) {
      if (i < cnt) {
        const Rec& R = recs[order_in[b + i0 + i]];
        s_hi[i] = rec_key_hi(R); s_lo[i] = rec_key_lo(R); s_ex[i] = ((uint64_t)R.emit << 32) | (i0 + i);
      } else {
        s_hi[i] = ~0ull; s_lo[i] = ~0ull; s_ex[i] = ~0ull;
      }
    }
    __syncthreads();
    bitonic_keys<BLOCK>(s_hi, s_lo, s_ex, np2);
    const RecKeys A = rec_keys(scratch, b, n, 0);
    for (uint32_t i = threadIdx.x; i < cnt; i += BLOCK) {
      A.hi[i0 + i] = s_hi[i]; A.lo[i0 + i] = s_lo[i]; A.ex[i0 + i] = s_ex[i];
    }
    __syncthreads();  // (LDS reused by the next item)
  }
}

// Merge pass p of the long reads: sorted runs of w = LCAP << p keys merged pairwise
// from one buffer into the other.  Work item (read, c) produces the merged outputs
// [c LCAP, (c + 1) LCAP) of its read: the merge-path split of the chunk's two ends (a
// binary search each), the two input ranges (<= LCAP keys together) staged in LDS,
// then each key's output rank = its index + the count of the other range's keys below
// it (an LDS binary search; keys are unique).  Items of reads already in one run
// (n <= w) are skipped: their keys stay in the buffer their last pass wrote.
template <int BLOCK, int LCAP>
__global__ __launch_bounds__(BLOCK) void k_rec_merge(const uint64_t* __restrict__ rec_off,
                                                     const uint2* __restrict__ tiles, const uint32_t* ctr,
                                                     uint64_t* scratch, uint64_t nrec, uint32_t p) {
  __shared__ uint64_t s_hi[LCAP], s_lo[LCAP], s_ex[LCAP];
  __shared__ uint32_t s_split[2];
  const uint64_t w = (uint64_t)LCAP << p;
  if (w >= ctr[1]) return;  // every long read is one run already
  const uint32_t n_items = ctr[0];
  const uint64_t src_off = (p & 1) ? 3 * nrec : 0, dst_off = (p & 1) ? 0 : 3 * nrec;
  for (uint32_t it = blockIdx.x; it < n_items; it += gridDim.x) {
    const uint2 tc = tiles[it];
    const uint64_t b = rec_off[tc.x];
    const uint32_t n = (uint32_t)(rec_off[tc.x + 1] - b);
    if (n <= w) continue;  // (uniform over the block)
    const RecKeys S = rec_keys(scratch, b, n, src_off), D = rec_keys(scratch, b, n, dst_off);
    const uint64_t o0 = (uint64_t)tc.y * LCAP;
    const uint64_t s = o0 / (2 * w) * (2 * w);  // the pair's first key
    const uint32_t la = (uint32_t)min<uint64_t>(w, n - s);
    const uint32_t lb = (uint32_t)(n - s - la < w ? n - s - la : w);
    const uint32_t d0 = (uint32_t)(o0 - s), d1 = min(d0 + (uint32_t)LCAP, la + lb);
    if (threadIdx.x < 2) {
      // merge path: a = left keys among the first d merged
      const uint32_t d = threadIdx.x ? d1 : d0;
      uint32_t lo = d > lb ? d - lb : 0, hi = min(d, la);
      while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        const uint64_t ia = s + m, ib = s + la + (d - m - 1);
        if (key_lt(S.hi[ia], S.lo[ia], S.ex[ia], S.hi[ib], S.lo[ib], S.ex[ib])) lo = m + 1;
        else hi = m;
      }
      s_split[threadIdx.x] = lo;
    }
    __syncthreads();
    const uint32_t a0 = s_split[0], a1 = s_split[1];
    const uint32_t na = a1 - a0, nb = (d1 - d0) - na, b0 = d0 - a0;
    for (uint32_t i = threadIdx.x; i < na + nb; i += BLOCK) {
      const uint64_t g = i < na ? s + a0 + i : s + la + b0 + (i - na);
      s_hi[i] = S.hi[g]; s_lo[i] = S.lo[g]; s_ex[i] = S.ex[g];
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < na + nb; i += BLOCK) {
      const uint64_t h = s_hi[i], l = s_lo[i], e = s_ex[i];
      // the other range: [ob, ob + on) in LDS
      const uint32_t ob = i < na ? na : 0, on = i < na ? nb : na;
      uint32_t lo = 0, hi = on;
      while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (key_lt(s_hi[ob + m], s_lo[ob + m], s_ex[ob + m], h, l, e)) lo = m + 1;
        else hi = m;
      }
      const uint64_t o = s + d0 + (i < na ? i : i - na) + lo;
      D.hi[o] = h; D.lo[o] = l; D.ex[o] = e;
    }
    __syncthreads();  // (LDS reused by the next item)
  }
}

// The long reads' records in their sorted order, from the buffer their last pass wrote
template <int LCAP>
__global__ void k_rec_gather(const Rec* __restrict__ recs, const uint64_t* __restrict__ rec_off,
                             const uint32_t* __restrict__ order_in, const uint2* __restrict__ tiles,
                             const uint32_t* ctr, const uint64_t* __restrict__ scratch, uint64_t nrec,
                             Rec* __restrict__ out) {
  const uint32_t n_items = ctr[0];
  for (uint32_t it = blockIdx.x; it < n_items; it += gridDim.x) {
    const uint2 tc = tiles[it];
    const uint64_t b = rec_off[tc.x];
    const uint32_t n = (uint32_t)(rec_off[tc.x + 1] - b);
    const uint64_t* ex = scratch + ((rec_merge_passes(n, LCAP) & 1) ? 3 * nrec : 0) + 3 * b + 2 * (uint64_t)n;
    const uint32_t i0 = tc.y * LCAP, cnt = min((uint32_t)LCAP, n - i0);
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x)
      out[b + i0 + i] = recs[order_in[b + (uint32_t)ex[i0 + i]]];
  }
}

}  // namespace pbgpu

// ====================================================== launch wrappers
namespace pbgpu {

void launch_build_keys(IndexView ix, uint32_t km, uint32_t K, uint32_t ebits, uint64_t N, const uint64_t* sel,
                       uint64_t Nsel, uint64_t* keys, uint64_t* vals, hipStream_t st) {
  hipLaunchKernelGGL(k_build_keys, dim3(4096), dim3(256), 0, st, ix, km, K, ebits, N, sel, Nsel, keys, vals);
}
void launch_part_ids(IndexView ix, uint32_t km, uint64_t N, uint32_t P, uint8_t* pid, unsigned long long* hist,
                     hipStream_t st) {
  hipLaunchKernelGGL(k_part_ids, dim3(4096), dim3(256), 0, st, ix, km, N, P, pid, hist);
}
void launch_table_insert(const ulonglong2* kh, uint64_t U, uint64_t base, ulonglong2* table, uint64_t bucket_mask,
                         uint64_t* filt, uint32_t filt_shift, hipStream_t st) {
  hipLaunchKernelGGL(k_table_insert, dim3(4096), dim3(256), 0, st, kh, U, base, table, bucket_mask,
                     (unsigned long long*)filt, filt_shift);
}
void launch_runs(const uint64_t* keys, const uint64_t* uidx, uint64_t N, uint32_t sh, uint64_t* run_start, hipStream_t st) {
  hipLaunchKernelGGL(k_runs, dim3(4096), dim3(256), 0, st, keys, uidx, N, sh, run_start);
}
void launch_occ_fill(const uint64_t* vals, const uint64_t* uidx, const uint64_t* kpos, uint64_t N, uint64_t* occ,
                     hipStream_t st) {
  hipLaunchKernelGGL(k_occ_fill, dim3(4096), dim3(256), 0, st, vals, uidx, kpos, N, occ);
}
void launch_headers(const uint64_t* keys, const uint64_t* kpos, const uint64_t* run_start, uint64_t U, uint64_t* occ,
                    ulonglong2* table, uint64_t bucket_mask, uint32_t k, uint32_t ebits, uint64_t* filt,
                    uint32_t filt_shift, ulonglong2* kh, hipStream_t st) {
  hipLaunchKernelGGL(k_headers, dim3(4096), dim3(256), 0, st, keys, kpos, run_start, U, occ, table, bucket_mask, k, ebits,
                     (unsigned long long*)filt, filt_shift, kh);
}

#ifndef PBGPU_SEED_PER
#define PBGPU_SEED_PER 8
#endif
constexpr int SEED_BLOCK = 256, SEED_PER = PBGPU_SEED_PER;
// mode: SEED_WHOLE / SEED_COUNTS / SEED_FINISH (gcount: per read position, indexed like seq)
void launch_seed(int mode, IndexView ix, const uint8_t* seq, const uint64_t* roff, uint32_t n_reads, AlignParamsDev P,
                 KRec* krec, uint32_t* n_kept, uint32_t* thr, uint64_t* nhits, unsigned long long* stats,
                 uint32_t* gcount, uint64_t null_ptr, hipStream_t st) {
  if (mode == SEED_COUNTS)
    hipLaunchKernelGGL((k_seed<SEED_BLOCK, SEED_PER, SEED_COUNTS>), dim3(n_reads), dim3(SEED_BLOCK), 0, st, ix, seq, roff,
                       n_reads, P, krec, n_kept, thr, nhits, stats, gcount, null_ptr);
  else if (mode == SEED_FINISH)
    hipLaunchKernelGGL((k_seed<SEED_BLOCK, SEED_PER, SEED_FINISH>), dim3(n_reads), dim3(SEED_BLOCK), 0, st, ix, seq, roff,
                       n_reads, P, krec, n_kept, thr, nhits, stats, gcount, null_ptr);
  else
    hipLaunchKernelGGL((k_seed<SEED_BLOCK, SEED_PER, SEED_WHOLE>), dim3(n_reads), dim3(SEED_BLOCK), 0, st, ix, seq, roff,
                       n_reads, P, krec, n_kept, thr, nhits, stats, gcount, null_ptr);
}

// mode: k_group's MODE (0: enumerate from the index; 1: split bucketed reads, 16-wave blocks,
// hcap_log2 12 for the partition counters; 2: partition items of bucketed reads)
void launch_group(IndexView ix, const KRec* krec, const uint64_t* roff, const uint32_t* n_kept, const uint32_t* thr,
                  const uint64_t* hit_off, uint64_t node_base, uint32_t r0, const uint2* read_list, uint32_t n_list,
                  uint32_t hcap_log2, uint32_t* gtable, GroupOut O, unsigned long long* stats, hipStream_t st,
                  int mode) {
  if (!n_list) return;
#define PBGPU_GROUP_ARGS ix, krec, roff, n_kept, thr, hit_off, node_base, r0, read_list, n_list, hcap_log2, gtable, O, stats
  if (!gtable) {  // LDS table: hcap_log2 <= 13; the 8192-slot table gets a 16-wave block
    // PBGPU_GROUP_LDS_PAD (experiment): extra dynamic LDS for the 4-wave tier, so fewer of
    // its blocks share a CU (fewer reads' lists open at once)
    static const size_t pad = getenv("PBGPU_GROUP_LDS_PAD") ? (size_t)atol(getenv("PBGPU_GROUP_LDS_PAD")) : 0;
#ifndef PBGPU_GROUP_BIG_LOG2
#define PBGPU_GROUP_BIG_LOG2 13
#endif
    const size_t lds = ((size_t)3 << hcap_log2) * sizeof(uint32_t) + (hcap_log2 < PBGPU_GROUP_BIG_LOG2 ? pad : 0);
    // the 96 KiB dynamic-LDS attribute, set once per device (function attributes are per device)
    static std::atomic<uint64_t> attr_done(0);
    int dev = 0;
    (void)hipGetDevice(&dev);
    const uint64_t bit = 1ull << (dev & 63);
    if (!(attr_done.load(std::memory_order_acquire) & bit)) {
      for (const void* f : {(const void*)k_group<false, GROUP_BLOCK, 0>, (const void*)k_group<false, GROUP_BLOCK_BIG, 0>,
                            (const void*)k_group<false, GROUP_BLOCK_BIG, 1>, (const void*)k_group<false, GROUP_BLOCK_BIG, 2>,
                            (const void*)k_group<false, GROUP_BLOCK, 2>, (const void*)k_group<false, GROUP_BLOCK, 1>})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024);
      attr_done.fetch_or(bit, std::memory_order_acq_rel);
    }
    // the split in 8-wave blocks: per 50k C4 reads its group stage 103.3 -> 93.0 ms against
    // 16-wave blocks (2 reads a CU at a time), 94.5 with 4 waves, 119 with 2
    // (profiles/r06sp_split_block.txt; PBGPU_SPLIT_BLOCK 128 / 256 / 512 / 1024)
    static const int split_b = getenv("PBGPU_SPLIT_BLOCK") ? atoi(getenv("PBGPU_SPLIT_BLOCK")) : 512;
    if (mode == 1) {
      static std::atomic<uint64_t> sattr(0);
      if (!(sattr.load(std::memory_order_acquire) & bit)) {
        for (const void* f : {(const void*)k_group<false, 128, 1>, (const void*)k_group<false, 512, 1>})
          (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024);
        sattr.fetch_or(bit, std::memory_order_acq_rel);
      }
    }
    if (mode == 1 && split_b == 128)
      hipLaunchKernelGGL((k_group<false, 128, 1>), dim3(n_list), dim3(128), lds, st, PBGPU_GROUP_ARGS);
    else if (mode == 1 && split_b == 512)
      hipLaunchKernelGGL((k_group<false, 512, 1>), dim3(n_list), dim3(512), lds, st, PBGPU_GROUP_ARGS);
    else if (mode == 1 && split_b == (int)GROUP_BLOCK)
      hipLaunchKernelGGL((k_group<false, GROUP_BLOCK, 1>), dim3(n_list), dim3(GROUP_BLOCK), lds, st, PBGPU_GROUP_ARGS);
    else if (mode == 1)
      hipLaunchKernelGGL((k_group<false, GROUP_BLOCK_BIG, 1>), dim3(n_list), dim3(GROUP_BLOCK_BIG), lds, st, PBGPU_GROUP_ARGS);
    else if (mode == 2 && hcap_log2 >= PBGPU_GROUP_BIG_LOG2)
      hipLaunchKernelGGL((k_group<false, GROUP_BLOCK_BIG, 2>), dim3(n_list), dim3(GROUP_BLOCK_BIG), lds, st, PBGPU_GROUP_ARGS);
    else if (mode == 2)
      hipLaunchKernelGGL((k_group<false, GROUP_BLOCK, 2>), dim3(n_list), dim3(GROUP_BLOCK), lds, st, PBGPU_GROUP_ARGS);
    else if (hcap_log2 >= PBGPU_GROUP_BIG_LOG2)
      hipLaunchKernelGGL((k_group<false, GROUP_BLOCK_BIG, 0>), dim3(n_list), dim3(GROUP_BLOCK_BIG), lds, st, PBGPU_GROUP_ARGS);
    else
      hipLaunchKernelGGL((k_group<false, GROUP_BLOCK, 0>), dim3(n_list), dim3(GROUP_BLOCK), lds, st, PBGPU_GROUP_ARGS);
  } else if (mode == 2) {
    hipLaunchKernelGGL((k_group<true, GROUP_BLOCK_BIG, 2>), dim3(n_list), dim3(GROUP_BLOCK_BIG), 0, st, PBGPU_GROUP_ARGS);
  } else {
    hipLaunchKernelGGL((k_group<true, GROUP_BLOCK_BIG, 0>), dim3(n_list), dim3(GROUP_BLOCK_BIG), 0, st, PBGPU_GROUP_ARGS);
  }
#undef PBGPU_GROUP_ARGS
}
// IndexView::occ_sr: the high word of every occ word (headers included, unused)
__global__ void k_occ_sr(const uint64_t* __restrict__ occ, uint64_t n, uint32_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = (uint32_t)(occ[i] >> 32);
}
void launch_occ_sr(const uint64_t* occ, uint64_t n, uint32_t* out, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_occ_sr, dim3(4096), dim3(256), 0, st, occ, n, out);
}

// sharded-index count exchange: two saturated counts per u32 (count_pack.h)
__global__ void k_counts_pack16(const uint32_t* __restrict__ c, uint64_t n, uint32_t* __restrict__ out) {
  const uint64_t nw = counts_packed_words(n);
  for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * blockDim.x)
    out[w] = counts_pack16(c, n, w);
}
__global__ void k_counts_unpack16(const uint32_t* __restrict__ in, uint64_t n, uint32_t* __restrict__ c) {
  const uint64_t nw = counts_packed_words(n);
  for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * blockDim.x)
    counts_unpack16(in[w], c, n, w);
}
void launch_counts_pack16(bool unpack, const uint32_t* src, uint64_t n, uint32_t* dst, hipStream_t st) {
  if (!n) return;
  if (unpack) hipLaunchKernelGGL(k_counts_unpack16, dim3(2048), dim3(256), 0, st, src, n, dst);
  else hipLaunchKernelGGL(k_counts_pack16, dim3(2048), dim3(256), 0, st, src, n, dst);
}

void launch_sr_ul(const uint32_t* ids, uint64_t n, const int32_t* ul, uint64_t n_ul, int32_t* out, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_sr_ul, dim3(1024), dim3(256), 0, st, ids, n, ul, n_ul, out);
}
uint64_t group_table_words(uint32_t hcap_log2) { return (uint64_t)3 << hcap_log2; }

static uint32_t grid_for(uint32_t n, uint32_t block, uint32_t cap = 65536) {
  uint64_t g = ((uint64_t)n + block - 1) / block;
  return (uint32_t)(g < 1 ? 1 : (g > cap ? cap : g));
}
void launch_init_slen(const ChainDesc* chains, uint32_t n_chains, uint32_t* slen, hipStream_t st) {
  if (!n_chains) return;
  hipLaunchKernelGGL(k_init_slen, dim3(grid_for(n_chains, 256)), dim3(256), 0, st, chains, n_chains, slen);
}
void launch_strand_order(const uint32_t* slen, uint32_t n_items, uint32_t* hist, uint32_t* cursor, uint32_t* perm,
                         int phase, hipStream_t st, const ChainDesc* chains, uint2* pinfo) {
  if (!n_items) return;
  StrandLen f{slen, chains};
  if (phase == 0)
    hipLaunchKernelGGL((k_len_hist<StrandLen>), dim3(grid_for(n_items, 256, 2048)), dim3(256), 0, st, f, n_items, hist,
                       (unsigned long long*)nullptr);
  else hipLaunchKernelGGL((k_len_perm<StrandLen>), dim3((n_items + 256 * LEN_PERM_ITEMS - 1) / (256 * LEN_PERM_ITEMS)), dim3(256), 0,
                          st, f, n_items, cursor, perm, chains ? pinfo : nullptr);
}
void launch_chain_order(const uint32_t* lisl, uint32_t n, uint32_t* hist, uint32_t* cursor, uint32_t* perm, int phase,
                        unsigned long long* sums, hipStream_t st) {
  if (!n) return;
  ChainLisLen f{lisl};
  if (phase == 0)
    hipLaunchKernelGGL((k_len_hist<ChainLisLen>), dim3(grid_for(n, 256, 2048)), dim3(256), 0, st, f, n, hist, sums);
  else hipLaunchKernelGGL((k_len_perm<ChainLisLen>), dim3((n + 256 * LEN_PERM_ITEMS - 1) / (256 * LEN_PERM_ITEMS)), dim3(256), 0,
                          st, f, n, cursor, perm, (uint2*)nullptr);
}
void launch_lis(bool big_nodes, const ChainDesc* chains, const uint32_t* items, uint32_t n_items, const uint32_t* slen,
                const int2* X, void* N, int2* pts, uint32_t* lisl, LisParams lp, int keep_idx,
                unsigned long long* stats, hipStream_t st, const uint32_t* nshift) {
  if (!n_items) return;
  const dim3 grid((n_items + 63) / 64);
  if (big_nodes)
    hipLaunchKernelGGL((k_lis<uint32_t, LIS_CH32>), grid, dim3(64), 0, st, chains, items, n_items, slen, X,
                       (LNode<uint32_t>*)N, pts, lisl, lp, keep_idx, stats, nshift);
  else
    hipLaunchKernelGGL((k_lis<uint16_t, LIS_CH16>), grid, dim3(64), 0, st, chains, items, n_items, slen, X,
                       (LNode<uint16_t>*)N, pts, lisl, lp, keep_idx, stats, (const uint32_t*)nullptr);
}
// returns the chunk count through *total (device); node index = hit index + nshift[item]
void launch_node32_place(const ChainDesc* chains, const uint32_t* items, uint32_t n, const uint32_t* slen,
                         uint32_t* nshift, unsigned long long* total, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_node32_place<LIS_CH32>, dim3(grid_for(n, 256)), dim3(256), 0, st, chains, items, n, slen,
                     nshift, total);
}
uint32_t node32_chunk() { return LIS_CH32; }
constexpr uint32_t LISW_TINY = LISW_TINY_N, LISW_SMALL = 511, LISW_LARGE = 4095;
#ifndef PBGPU_LIS_LANE_MAX
#define PBGPU_LIS_LANE_MAX 8
#endif
// strands of <= LIS_LANE_MAX hits: order restored lane-per-strand, then k_lis (lane per strand)
void launch_lis_lane(const ChainDesc* chains, const uint32_t* items, uint32_t n_items, const uint32_t* slen, int2* X,
                     void* N16, int2* pts, uint32_t* lisl, LisParams lp, int keep_idx, unsigned long long* stats,
                     hipStream_t st, const uint2* pinfo) {
  if (!n_items) return;
  // the register kernel: default window, no kept lis indices (PBGPU_LIS_TINY=0: the generic path)
  static const bool tiny_on = !(getenv("PBGPU_LIS_TINY") && !atoi(getenv("PBGPU_LIS_TINY")));
  if (tiny_on && !keep_idx && lp.W == 1 && !lp.mer_all) {
    hipLaunchKernelGGL((k_lis_tiny<PBGPU_LIS_LANE_MAX>), dim3((n_items + 255) / 256), dim3(256), 0, st, chains, items,
                       pinfo, n_items, slen, X, pts, lisl, lp, stats);
    return;
  }
  if (!lp.ordered)
    hipLaunchKernelGGL((k_order_tiny<PBGPU_LIS_LANE_MAX>), dim3((n_items + 255) / 256), dim3(256), 0, st, chains, items,
                       n_items, slen, X);
  launch_lis(false, chains, items, n_items, slen, X, N16, pts, lisl, lp, keep_idx, stats, st, nullptr);
}
uint32_t lis_lane_max() { return PBGPU_LIS_LANE_MAX; }
// CU count of the current device, cached per device (aligners on several
// devices and host threads call this concurrently: atomics, no lock)
static int device_cus() {
  static std::atomic<int> cache[64];
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  int c = cache[dev].load(std::memory_order_relaxed);
  if (!c) {
    hipDeviceProp_t pr;
    c = hipGetDeviceProperties(&pr, dev) == hipSuccess ? pr.multiProcessorCount : 256;
    cache[dev].store(c, std::memory_order_relaxed);
  }
  return c;
}
static uint32_t resident_blocks(const void* fn, int block) {
  const int cus = device_cus();
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, block, 0) != hipSuccess || per < 1) per = 1;
  return (uint32_t)(per * cus);
}
template <int SMAX, int WPB>
static void launch_lis_w(const ChainDesc* chains, const uint32_t* items, uint32_t n_items, const uint32_t* slen,
                         int2* X, void* N16, int2* pts, uint32_t* lisl, LisParams lp, int keep_idx,
                         unsigned long long* stats, hipStream_t st) {
  const void* fn = (const void*)k_lis_w<SMAX, WPB>;
  const uint32_t g = std::min<uint32_t>(resident_blocks(fn, 64 * WPB), (n_items + WPB - 1) / WPB);
  hipLaunchKernelGGL((k_lis_w<SMAX, WPB>), dim3(g), dim3(64 * WPB), 0, st, chains, items, n_items, slen, X,
                     (LNode<uint16_t>*)N16, pts, lisl, lp, keep_idx, stats);
}
// tier 0: n <= 255 (8 waves per block), 1: n <= 511 (4 waves), 2: n <= 4095 (1 wave)
void launch_lis_wave(int tier, const ChainDesc* chains, const uint32_t* items, uint32_t n_items, const uint32_t* slen,
                     int2* X, void* N16, int2* pts, uint32_t* lisl, LisParams lp, int keep_idx,
                     unsigned long long* stats, hipStream_t st) {
  if (!n_items) return;
  if (tier == 2) launch_lis_w<LISW_LARGE, 1>(chains, items, n_items, slen, X, N16, pts, lisl, lp, keep_idx, stats, st);
  else if (tier == 1) launch_lis_w<LISW_SMALL, 4>(chains, items, n_items, slen, X, N16, pts, lisl, lp, keep_idx, stats, st);
  else launch_lis_w<LISW_TINY, 8>(chains, items, n_items, slen, X, N16, pts, lisl, lp, keep_idx, stats, st);
}
// length classes (len_bucket) at the kernel boundaries
uint32_t lis_class_bounds(int which) {  // first class of: 0 = > LISW_SMALL, 1 = > LISW_LARGE, 2 = > LIS_U16_MAX, 3 = > LISW_TINY
  return which == 0 ? 128u + 16u * (9u - 7u) : which == 1 ? 128u + 16u * (12u - 7u)
       : which == 2 ? 128u + 16u * (16u - 7u) : 128u + 16u * (8u - 7u);
}
void launch_coords(IndexView ix, AlignParamsDev P, const ChainDesc* chains, const uint32_t* list, uint32_t n,
                   const uint64_t* roff, uint32_t emit, ChainOut O, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL((k_coords<FIT_CH>), dim3((n + 63) / 64), dim3(64), 0, st, ix, P, chains, list, n, roff, emit, O);
}
void launch_discard(const ChainDesc* chains, const uint32_t* list, uint32_t n, const uint32_t* lisl, uint32_t* slen,
                    int2* X, const void* N16, const void* N32, const uint32_t* nshift, uint32_t* items_small,
                    uint32_t* n_small, uint32_t* items_big, uint32_t* n_big, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_discard, dim3(grid_for(n, 256)), dim3(256), 0, st, chains, list, n, lisl, slen, X,
                     (const LNode<uint16_t>*)N16, (const LNode<uint32_t>*)N32, nshift, items_small, n_small,
                     items_big, n_big);
}
uint32_t len_buckets() { return NLB; }
void launch_strand_order(const ChainDesc* chains, const uint32_t* items, uint32_t n_items, const uint32_t* slen, int2* X,
                         hipStream_t st) {
  if (!n_items) return;
  hipLaunchKernelGGL(k_strand_order, dim3(std::min<uint32_t>(n_items, 2048)), dim3(256), 0, st, chains, items, n_items,
                     slen, X);
}
#ifdef PBGPU_PROF
extern "C" int pbgpu_debug_prof(unsigned long long* out, int n, int reset) {
  if (n > PROF_SLOTS) n = PROF_SLOTS;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), n * sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[PROF_SLOTS] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif
uint32_t big_bucket() {  // first length class whose items all exceed LIS_U16_MAX
  static_assert(LIS_U16_MAX == 65535u, "len_bucket(65536) starts a class");
  return 128u + 16u * (16u - 7u);
}

void launch_rec_hist(const uint32_t* rec_read, uint32_t n, uint32_t* per_read, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_rec_hist, dim3(1024), dim3(256), 0, st, rec_read, n, per_read);
}
void launch_rec_place(const uint32_t* rec_read, const uint32_t* rec_slot, uint32_t n, const uint64_t* rec_off,
                      uint32_t* order, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_rec_place, dim3(std::min<uint32_t>((n + 255) / 256, 16384)), dim3(256), 0, st, rec_read, rec_slot,
                     n, rec_off, order);
}
void launch_rec_scatter(const uint32_t* rec_read, uint32_t n, const uint64_t* rec_off, uint32_t* cursor, uint32_t* order,
                        hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_rec_scatter, dim3(1024), dim3(256), 0, st, rec_read, n, rec_off, cursor, order);
}
constexpr int REC_BLOCK = 256, REC_LCAP = 2048;
int rec_sort_lcap() { return REC_LCAP; }
// tiles of the reads past REC_LCAP records: a read of n > LCAP records has ceil(n / LCAP) < 2 n / LCAP
uint64_t rec_sort_max_tiles(uint64_t nrec) { return 2 * nrec / REC_LCAP + 1; }
// Records sorted per read: the LDS kernel for reads of <= REC_LCAP records; the longer
// reads' tiles sorted in LDS, then merged pairwise over the scratch's two key buffers
// (6 words a record, nrec records), then gathered.  ctr: 2 words, zeroed by the caller.
// max_passes: a bound on the merge passes (the longest read is not known on the host):
// passes past the longest read's exit at once on the device.
void launch_rec_sort(const Rec* recs, const uint64_t* rec_off, const uint32_t* order, uint64_t* gscratch,
                     uint32_t n_reads, uint64_t nrec, uint2* tiles, uint32_t* ctr, Rec* out, hipStream_t st) {
  if (!n_reads) return;
  hipLaunchKernelGGL((k_rec_sort<REC_BLOCK, REC_LCAP>), dim3(n_reads), dim3(REC_BLOCK), 0, st, recs, rec_off, order,
                     n_reads, out, tiles, ctr);
  if (nrec <= (uint64_t)REC_LCAP) return;
  const uint64_t max_tiles = rec_sort_max_tiles(nrec);
  const uint32_t grid = (uint32_t)std::min<uint64_t>(max_tiles, 8192);
  hipLaunchKernelGGL((k_rec_tile_sort<REC_BLOCK, REC_LCAP>), dim3(grid), dim3(REC_BLOCK), 0, st, recs, rec_off, order,
                     tiles, ctr, gscratch);
  uint32_t passes = 0;
  while (((uint64_t)REC_LCAP << passes) < nrec) ++passes;
  for (uint32_t p = 0; p < passes; ++p)
    hipLaunchKernelGGL((k_rec_merge<REC_BLOCK, REC_LCAP>), dim3(grid), dim3(REC_BLOCK), 0, st, rec_off, tiles, ctr,
                       gscratch, nrec, p);
  hipLaunchKernelGGL((k_rec_gather<REC_LCAP>), dim3(grid), dim3(256), 0, st, recs, rec_off, order, tiles, ctr,
                     gscratch, nrec, out);
}

// ------------------------------------------------------------ fine launchers
// The coarse records of each read (recs_sorted, grouped by read) as fine windows in
// (super-read, record) order -- the (read, super-read) order of the windows'
// std::map lookup (fine_aligner.hpp:50-58), ties in record order as a stable sort
// leaves them: a bitonic sort per read of (sr, record) keys, in LDS, or in the
// records-stage scratch (6 words a record) for reads of more than LCAP records.
template <int BLOCK, int LCAP>
__global__ __launch_bounds__(BLOCK) void k_fine_win_sort(const Rec* __restrict__ recs, const uint64_t* __restrict__ rec_off,
                                                         uint32_t n_reads, uint64_t* gscratch, uint32_t* __restrict__ idx) {
  __shared__ uint64_t s_hi[LCAP], s_lo[LCAP];
  __shared__ uint32_t s_ex[LCAP];
  const uint32_t r = blockIdx.x;
  if (r >= n_reads) return;
  const uint64_t b = rec_off[r];
  const uint32_t n = (uint32_t)(rec_off[r + 1] - b);
  if (n == 0) return;
  uint32_t np2 = 1;
  while (np2 < n) np2 <<= 1;
  if (np2 <= LCAP) {
    for (uint32_t i = threadIdx.x; i < np2; i += BLOCK) {
      s_hi[i] = i < n ? (uint64_t)recs[b + i].sr : ~0ull;
      s_lo[i] = 0;
      s_ex[i] = i < n ? i : ~0u;
    }
    __syncthreads();
    bitonic_keys<BLOCK>(s_hi, s_lo, s_ex, np2);
    for (uint32_t i = threadIdx.x; i < n; i += BLOCK) idx[b + i] = (uint32_t)b + s_ex[i];
  } else {
    uint64_t* hi = gscratch + 6 * b;
    uint64_t* lo = hi + np2;
    uint64_t* ex = lo + np2;
    for (uint32_t i = threadIdx.x; i < np2; i += BLOCK) {
      hi[i] = i < n ? (uint64_t)recs[b + i].sr : ~0ull;
      lo[i] = 0;
      ex[i] = i < n ? i : ~0ull;
    }
    __threadfence_block();
    __syncthreads();
    bitonic_keys<BLOCK>(hi, lo, ex, np2);
    for (uint32_t i = threadIdx.x; i < n; i += BLOCK) idx[b + i] = (uint32_t)(b + ex[i]);
  }
}
void launch_fine_win_sort(const Rec* recs, const uint64_t* rec_off, uint32_t n_reads, uint64_t* gscratch, uint32_t* idx,
                          hipStream_t st) {
  if (n_reads) hipLaunchKernelGGL((k_fine_win_sort<256, 2048>), dim3(n_reads), dim3(256), 0, st, recs, rec_off, n_reads,
                                  gscratch, idx);
}

// The fine hits of a sub-batch (k_fine_hits: each read's hits contiguous, in
// (k-mer, occurrence) order, keyed 2 (window - w_sub0) + strand, a read's keys
// contiguous) stable-sorted by key, so every window's fwd and bwd lists come out in
// the reference's order, contiguous: one wave per read, a counting sort -- the
// read's key counts (LDS, or a global region for reads with more than KCAP keys),
// their exclusive scan, then the hits placed 64 at a time in order, equal keys of a
// tile ranked by lane.
template <uint32_t KCAP>
__global__ __launch_bounds__(64) void k_fine_sort(const uint32_t* __restrict__ keys, const int2* __restrict__ vals,
                                                  const uint64_t* __restrict__ woff, const uint64_t* __restrict__ hit_off,
                                                  uint32_t r0, uint32_t nr, uint64_t w_sub0, uint32_t* gcount,
                                                  uint32_t* __restrict__ okeys, int2* __restrict__ ovals) {
  __shared__ uint32_t s_cnt[KCAP];
  if (blockIdx.x >= nr) return;
  const uint32_t r = r0 + blockIdx.x, lane = threadIdx.x;
  const uint64_t h0 = hit_off[r], nh = hit_off[r + 1] - h0;
  if (nh == 0) return;
  const uint32_t kb = (uint32_t)(2 * (woff[r] - w_sub0)), nk = (uint32_t)(2 * (woff[r + 1] - woff[r]));
  uint32_t* cnt = nk <= KCAP ? s_cnt : gcount + kb;
  for (uint32_t x = lane; x < nk; x += 64) cnt[x] = 0;
  __threadfence_block();
  __syncthreads();
  for (uint64_t i = lane; i < nh; i += 64) atomicAdd(&cnt[keys[h0 + i] - kb], 1u);
  __threadfence_block();
  __syncthreads();
  uint32_t carry = 0;  // counts -> read-relative list starts (the cursors)
  for (uint32_t x0 = 0; x0 < nk; x0 += 64) {
    const uint32_t x = x0 + lane;
    const uint32_t v = x < nk ? cnt[x] : 0u;
    uint32_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if ((int)lane >= o) inc += y;
    }
    if (x < nk) cnt[x] = carry + inc - v;
    carry += (uint32_t)__shfl((int)inc, 63, 64);
  }
  __threadfence_block();
  __syncthreads();
  for (uint64_t t0 = 0; t0 < nh; t0 += 64) {
    const uint64_t i = t0 + lane;
    const bool act = i < nh;
    const uint32_t k = act ? keys[h0 + i] - kb : 0xFFFFFFFFu;
    const int2 v = act ? vals[h0 + i] : make_int2(0, 0);
    uint32_t dest = 0;
    for (uint64_t rem = __ballot(act); rem;) {
      const uint32_t leader = (uint32_t)__ffsll((long long)rem) - 1;
      const uint32_t kl = (uint32_t)__builtin_amdgcn_readlane((int)k, (int)leader);
      const uint64_t m = __ballot(act && k == kl);
      uint32_t base = lane == leader ? cnt[kl] : 0u;
      base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)leader);
      if (lane == leader) cnt[kl] = base + (uint32_t)__builtin_popcountll(m);
      if (act && k == kl) dest = base + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1));
      rem &= ~m;
    }
    if (act) { okeys[h0 + dest] = k + kb; ovals[h0 + dest] = v; }
  }
}
void launch_fine_sort(const uint32_t* keys, const int2* vals, const uint64_t* woff, const uint64_t* hit_off, uint32_t r0,
                      uint32_t nr, uint64_t w_sub0, uint32_t* gcount, uint32_t* okeys, int2* ovals, hipStream_t st) {
  if (nr) hipLaunchKernelGGL((k_fine_sort<8192>), dim3(nr), dim3(64), 0, st, keys, vals, woff, hit_off, r0, nr, w_sub0,
                             gcount, okeys, ovals);
}
void launch_fine_windows(const Rec* recs, uint32_t n, uint64_t* keys, uint32_t* idx, int phase, const uint64_t* roff,
                         uint32_t fk, FineWin* out, hipStream_t st) {
  const uint32_t g = std::max<uint32_t>(1, std::min<uint32_t>(4096, (n + 255) / 256));
  if (phase == 0) hipLaunchKernelGGL(k_fine_win_keys, dim3(g), dim3(256), 0, st, recs, n, keys, idx);
  else hipLaunchKernelGGL(k_fine_win_fill, dim3(g), dim3(256), 0, st, recs, idx, n, roff, fk, out);
}
void launch_fine_hits(bool emit, IndexView fx, const uint8_t* seq, const uint64_t* roff, uint32_t r0, uint32_t nr,
                      const FineWin* win, const uint64_t* woff, uint64_t* read_hits, const uint64_t* hit_off,
                      uint64_t w_sub0, uint32_t* keys, int2* vals, unsigned long long* stats, hipStream_t st) {
  if (!nr) return;
  if (emit)
    hipLaunchKernelGGL(k_fine_hits<true>, dim3(nr), dim3(FINE_BLOCK), 0, st, fx, seq, roff, r0, win, woff, read_hits,
                       hit_off, w_sub0, keys, vals, stats);
  else
    hipLaunchKernelGGL(k_fine_hits<false>, dim3(nr), dim3(FINE_BLOCK), 0, st, fx, seq, roff, r0, win, woff, read_hits,
                       hit_off, w_sub0, keys, vals, stats);
}
void launch_list_bounds(const uint32_t* keys, uint64_t G, uint32_t* lstart, uint32_t* lend, hipStream_t st) {
  if (!G) return;
  const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(8192, (G + 255) / 256));
  hipLaunchKernelGGL(k_list_bounds, dim3(g), dim3(256), 0, st, keys, G, lstart, lend);
}
void launch_fine_desc(IndexView ix, const Rec* recs, uint64_t w_sub0, uint32_t nwin, const uint32_t* lstart,
                      const uint32_t* lend, int with_info, ChainDesc* chains, uint32_t* emit_of,
                      unsigned long long* info_need, hipStream_t st) {
  if (!nwin) return;
  const uint32_t g = std::max<uint32_t>(1, std::min<uint32_t>(4096, (nwin + 255) / 256));
  hipLaunchKernelGGL(k_fine_desc, dim3(g), dim3(256), 0, st, ix, recs, w_sub0, nwin, lstart, lend, with_info, chains,
                     emit_of, info_need);
}
void launch_fine_empty(IndexView ix, uint32_t k, const ChainDesc* chains, uint32_t n, const uint32_t* lisl,
                       const uint32_t* emit_of, ChainOut O, hipStream_t st) {
  if (!n) return;
  const uint32_t g = std::max<uint32_t>(1, std::min<uint32_t>(4096, (n + 255) / 256));
  hipLaunchKernelGGL(k_fine_empty, dim3(g), dim3(256), 0, st, ix, k, chains, n, lisl, emit_of, O);
}

// ================================================================= scans
// Exclusive scan of per-item counts into offsets (the per-batch hit, record and
// text offsets): reduce per 2048-item tile, scan the tile sums in one block,
// rescan each tile from its base.  Item n is a zero, so out[n] is the total.
constexpr uint32_t SCAN_BLOCK = 256, SCAN_ITEMS = 8, SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;
DEV uint64_t scan_item(const uint32_t* in32, const uint64_t* in64, uint64_t n, uint64_t i) {
  if (i >= n) return 0;
  return in32 ? (uint64_t)in32[i] : in64[i];
}
// inclusive scan of one u64 per thread over the block, block total in tot
template <uint32_t BLOCK>
DEV uint64_t block_incl_scan_u64(uint64_t v, uint64_t* s_w, uint64_t& tot) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  if (lane == 63) s_w[w] = v;
  __syncthreads();
  uint64_t base = 0, t = 0;
  for (uint32_t j = 0; j < BLOCK / 64; ++j) {
    const uint64_t x = s_w[j];
    base += j < w ? x : 0;
    t += x;
  }
  __syncthreads();
  tot = t;
  return base + v;
}
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_reduce(const uint32_t* __restrict__ in32,
                                                            const uint64_t* __restrict__ in64, uint64_t n,
                                                            uint64_t* __restrict__ tile_sum) {
  __shared__ uint64_t s_w[SCAN_BLOCK / 64];
  const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_TILE + threadIdx.x;
  uint64_t v = 0;
#pragma unroll
  for (uint32_t j = 0; j < SCAN_ITEMS; ++j) v += scan_item(in32, in64, n, i0 + (uint64_t)j * SCAN_BLOCK);
  uint64_t tot;
  block_incl_scan_u64<SCAN_BLOCK>(v, s_w, tot);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}
// one block: the tile sums, scanned exclusive in place
__global__ __launch_bounds__(1024) void k_scan_tiles(uint64_t* __restrict__ tile_sum, uint64_t nt) {
  __shared__ uint64_t s_w[1024 / 64];
  uint64_t carry = 0;
  for (uint64_t c = 0; c < nt; c += 1024) {
    const uint64_t i = c + threadIdx.x;
    const uint64_t v = i < nt ? tile_sum[i] : 0;
    uint64_t tot;
    const uint64_t inc = block_incl_scan_u64<1024>(v, s_w, tot);
    if (i < nt) tile_sum[i] = carry + inc - v;
    carry += tot;
  }
}
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_apply(const uint32_t* __restrict__ in32,
                                                           const uint64_t* __restrict__ in64, uint64_t n,
                                                           const uint64_t* __restrict__ tile_base,
                                                           uint64_t* __restrict__ out) {
  __shared__ uint64_t s_w[SCAN_BLOCK / 64];
  // thread t takes items [t * SCAN_ITEMS, (t + 1) * SCAN_ITEMS) of the tile
  const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
  uint64_t v[SCAN_ITEMS], sum = 0;
#pragma unroll
  for (uint32_t j = 0; j < SCAN_ITEMS; ++j) { v[j] = scan_item(in32, in64, n, i0 + j); sum += v[j]; }
  uint64_t tot;
  uint64_t run = tile_base[blockIdx.x] + block_incl_scan_u64<SCAN_BLOCK>(sum, s_w, tot) - sum;
#pragma unroll
  for (uint32_t j = 0; j < SCAN_ITEMS; ++j) {
    if (i0 + j <= n) out[i0 + j] = run;
    run += v[j];
  }
}
uint64_t excl_scan_scratch_words(uint64_t n) { return (n + 1 + SCAN_TILE - 1) / SCAN_TILE; }
void launch_excl_scan(const uint32_t* in32, const uint64_t* in64, uint64_t n, uint64_t* out, uint64_t* scratch,
                      hipStream_t st) {
  const uint64_t nt = excl_scan_scratch_words(n);
  hipLaunchKernelGGL(k_scan_reduce, dim3((uint32_t)nt), dim3(SCAN_BLOCK), 0, st, in32, in64, n, scratch);
  hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(1024), 0, st, scratch, nt);
  hipLaunchKernelGGL(k_scan_apply, dim3((uint32_t)nt), dim3(SCAN_BLOCK), 0, st, in32, in64, n, scratch, out);
}

// ========================================================== overlap graph
#ifdef PBGPU_GRAPH_CHECK
// Bounds-checking build (tools/r06/graph_check.sh, never the product): every far node k_graph_edges
// reads, its name offset and prefix-sum index, and every edge target the relaxations read,
// checked against the batch's arrays; violations counted (and the access redirected to a
// valid index), reported at process exit.  [0] far j outside (q, qe) / n_recs, [1] name
// units past the batch's units, [2] prefix sums past them, [3] edge target outside its read,
// [4] checks made.
__device__ unsigned long long g_graph_check[5];
#define GCHECK(ok, slot) do { if (!(ok)) atomicAdd(&g_graph_check[slot], 1ull); } while (0)
#endif
// create_mega_reads' per-read overlap graph (overlap_graph.cc:7-59,
// overlap_graph::traverse, with node_info::reset, overlap_graph.hpp:24-34, and
// union_find.cc) on the records of recs_sorted: the host then only collects the
// components, tiles and prints (create_mega_reads.cc:79-89).  The double
// arithmetic restates the reference's operation order with _rn intrinsics (no
// contraction); the record order and the stable sort by implied position are
// the host's.
DEV uint32_t graph_unit(const GraphDev& G, uint32_t sr, uint32_t nsz, bool rev, uint32_t u) {
  // super_read_name of the record's orientation: the bwd name is the fwd one reversed,
  // each unitig flipped (super_read_name.cc:38-47)
  const uint64_t o = G.noff[sr];
  return rev ? G.units[o + nsz - 1 - u] ^ 1u : G.units[o + u];
}
DEV uint32_t graph_nsz(const GraphDev& G, uint32_t sr) { return (uint32_t)(G.noff[sr + 1] - G.noff[sr]); }
// node p of a read (record b + i) as k_graph_edges reads it (k_graph_prep wrote its units)
DEV void graph_write_desc(const GraphDev& G, uint64_t at, uint64_t b, uint32_t i) {
  const Rec& R = G.recs[b + i];
  const double2 m = G.imp[b + i];
  const uint64_t po = G.poff[b + i];
  const uint32_t ns = graph_nsz(G, R.sr);
  GDesc d;
  d.imp_s = m.x; d.imp_e = m.y; d.err = R.avg_err;
  d.idx = (uint16_t)i; d.nsz = (uint16_t)ns;
  d.lp_add = G.bases ? R.sr_cover : (uint32_t)R.nb_mers;
#pragma unroll
  for (uint32_t u = 0; u < GRAPH_U; ++u) d.u[u] = u < ns ? G.ounits[po + u] : 0u;
  G.desc[at] = d;
  G.spo[at] = (uint32_t)po;  // (< 2^32: host check)
  G.fis[at] = m.x; G.fie[at] = m.y; G.fer[at] = R.avg_err; G.fu0[at] = d.u[0];
}
constexpr uint32_t GRAPH_PREP_U = 8;  // names of at most this many unitigs: loads batched in registers
__global__ void k_graph_sizes(GraphDev G, uint64_t n, uint32_t* sizes) {
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < n; q += (uint64_t)gridDim.x * blockDim.x)
    sizes[q] = graph_nsz(G, G.recs[q].sr) + 1;
}
// the most records of a read in the batch (a wave's max, one atomic a wave)
__global__ void k_graph_max_n(GraphDev G, uint32_t n_reads) {
  uint32_t mx = 0;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n_reads; r += gridDim.x * blockDim.x) {
    const uint32_t nr = (uint32_t)(G.rec_off[r + 1] - G.rec_off[r]);
    mx = nr > mx ? nr : mx;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t v = (uint32_t)__shfl_xor((int)mx, o, 64);
    mx = v > mx ? v : mx;
  }
  if ((threadIdx.x & 63) == 0 && mx) atomicMax(G.max_n, mx);
}
// per record: implied start / end (overlap_graph.hpp:24-34), its name's unitigs in
// its orientation, and the prefix sums over them of the unitig lengths (ulen: 0 past
// the lengths, as the host's) and of info[2u] - info[2u - 1] (kmers_info, or
// bases_info with -b; 0 past n_info)
__global__ void k_graph_prep(GraphDev G, uint64_t n) {
  const uint32_t* __restrict__ units = G.units;
  const int32_t* __restrict__ ul = G.ul;
  uint32_t* __restrict__ ounits = G.ounits;
  uint2* __restrict__ pp = G.pp;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < n; q += (uint64_t)gridDim.x * blockDim.x) {
    const Rec R = G.recs[q];
    G.imp[q] = make_double2(__dadd_rn(R.stretch, R.offset), __dadd_rn(__dmul_rn(R.stretch, (double)R.ql), R.offset));
    const uint64_t o = G.noff[R.sr];
    const uint32_t nsz = (uint32_t)(G.noff[R.sr + 1] - o);
    const bool rev = (R.flags & 2u) != 0;
    const int32_t* __restrict__ info = (G.bases ? G.info_b : G.info_m) + R.info_off;
    const uint32_t ni = R.n_info;
    auto info_at = [&](uint32_t i) -> uint32_t { return i < ni ? (uint32_t)info[i] : 0u; };
    const uint64_t po = G.poff[q];
    pp[po] = make_uint2(0u, 0u);
    if (nsz <= GRAPH_PREP_U) {
      // the name's unitigs, their lengths and info words as independent loads issued
      // together (the loop below waits for each unitig's id before its length, and
      // for its stores before the next loads)
      uint32_t un[GRAPH_PREP_U], len[GRAPH_PREP_U], ia[GRAPH_PREP_U], ib[GRAPH_PREP_U];
#pragma unroll
      for (uint32_t u = 0; u < GRAPH_PREP_U; ++u)
        un[u] = u < nsz ? (rev ? units[o + nsz - 1 - u] ^ 1u : units[o + u]) : 0u;
#pragma unroll
      for (uint32_t u = 0; u < GRAPH_PREP_U; ++u) {
        const uint32_t id = un[u] >> 1;
        len[u] = (u < nsz && id < G.n_ul) ? (uint32_t)ul[id] : 0u;
        ia[u] = u < nsz ? info_at(2 * u) : 0u;
        ib[u] = (u < nsz && u > 0) ? info_at(2 * u - 1) : 0u;
      }
      uint32_t a = 0, c = 0;
#pragma unroll
      for (uint32_t u = 0; u < GRAPH_PREP_U; ++u) {
        if (u < nsz) {
          a += len[u];
          c += ia[u] - ib[u];
          ounits[po + u] = un[u];
          pp[po + u + 1] = make_uint2(a, c);
        }
      }
      continue;
    }
    uint32_t a = 0, c = 0;
    for (uint32_t u = 0; u < nsz; ++u) {
      const uint32_t un = rev ? units[o + nsz - 1 - u] ^ 1u : units[o + u];
      ounits[po + u] = un;
      const uint32_t id = un >> 1;
      a += id < G.n_ul ? (uint32_t)ul[id] : 0u;
      c += info_at(2 * u) - (u > 0 ? info_at(2 * u - 1) : 0u);
      pp[po + u + 1] = make_uint2(a, c);
    }
  }
}
// order-preserving key of a double (finite; -0 sorts as +0, as operator< sees them)
DEV uint64_t graph_dkey(double x) {
  const uint64_t b = (uint64_t)__double_as_longlong(__dadd_rn(x, 0.0));
  return (b >> 63) ? ~b : b | (1ull << 63);
}
// per read: records by (imp_s, imp_e), ties in record order (the host's stable_sort of
// sort_nodes), written out as descriptors in that order
// Three tiers by the read's record count (LDS sized to the tier, so the common
// reads of <= GRAPH_NM_SMALL records run many blocks a CU): NM = GRAPH_NM_SMALL
// takes those, NM = GRAPH_NM_MID the reads up to it, NM = GRAPH_NMAX the rest.
#ifndef PBGPU_RELAX_PF
#define PBGPU_RELAX_PF 6
#endif
constexpr uint32_t GRAPH_SORT_BLOCK = 256, GRAPH_NM_SMALL = 1024, GRAPH_NM_MID = 4096, GRAPH_RELAX_MIN = 512,
                   GRAPH_RELAX_PF = PBGPU_RELAX_PF;
static_assert(GRAPH_EBLK >= 1 && GRAPH_EBLK <= 64, "k_graph_relax takes a node's block with one 64-lane load");
template <uint32_t NM>
DEV bool graph_tier(const GraphDev& G, uint32_t n) {
  if (n == 0 || n > G.nmax || n > GRAPH_NMAX) return false;
  return n <= NM && (NM == GRAPH_NM_SMALL || n > (NM == GRAPH_NM_MID ? GRAPH_NM_SMALL : GRAPH_NM_MID));
}
template <uint32_t NM>
__global__ __launch_bounds__(GRAPH_SORT_BLOCK) void k_graph_sort(GraphDev G, uint32_t n_reads) {
  __shared__ uint64_t s_hi[NM], s_lo[NM];
  __shared__ uint16_t s_ex[NM];
  const uint32_t r = blockIdx.x;
  if (r >= n_reads) return;
  const uint64_t b = G.rec_off[r];
  const uint32_t n = (uint32_t)(G.rec_off[r + 1] - b);
  if (!graph_tier<NM>(G, n)) return;
  uint32_t np2 = 1;
  while (np2 < n) np2 <<= 1;
  for (uint32_t i = threadIdx.x; i < np2; i += GRAPH_SORT_BLOCK) {
    if (i < n) {
      const double2 m = G.imp[b + i];
      s_hi[i] = graph_dkey(m.x); s_lo[i] = graph_dkey(m.y); s_ex[i] = (uint16_t)i;
    } else {
      s_hi[i] = ~0ull; s_lo[i] = ~0ull; s_ex[i] = 0xFFFFu;
    }
  }
  __syncthreads();
  bitonic_keys<GRAPH_SORT_BLOCK>(s_hi, s_lo, s_ex, np2);
  for (uint32_t p = threadIdx.x; p < n; p += GRAPH_SORT_BLOCK) {
    graph_write_desc(G, b + p, b, s_ex[p]);
  }
}
// The traversal (overlap_graph.cc:7-59) in two phases.  Everything the reference
// tests for a pair (i, j) -- the 5' / not-advancing skips, the break, the names'
// dovetail overlap, the same-name case, the play / error bounds, and the edge's
// path increment (nb_mers or sr_cover minus the common k-mers) and unitig count --
// reads only static node data, so it runs for every node at once
// (k_graph_edges); only the longest-path relaxation and the unions, in the
// reference's (i, then j) order, are serial per read (k_graph_relax).
//
// k_graph_edges: a block per window of GE_NODES consecutive sorted positions of
// the batch; the window's nodes and the GE_SLOTS - GE_NODES positions after them
// (implied span, error, name size, first GRAPH_U unitigs, read bounds) are staged
// in LDS; a wave per node i, lanes j = i + 1 + lane, ... 64 at a time until the
// reference's break (past the staged positions, a prefilter over per-field arrays in HBM
// queues the positions that can break or be an edge, tested 64 at a time).  Each node
// writes its first GRAPH_EBLK edges, in j order, as {j's record index | (unitigs
// added) << 16, path increment} into a block of its own, and its exact count
// (ecnt); a node with more (2 in 28k on C2) is listed, with its region past the
// block.  OVF: a wave per listed node runs its scan again (from HBM) and writes the
// edges past its block there.
constexpr uint32_t GRAPH_NMAX_K = GRAPH_NMAX;  // reads of more records: k_graph_relax_big (state in HBM)
constexpr uint32_t GRAPH_ROOT_BITS = 13;  // k_graph_relax matches roots by this many bits
static_assert(GRAPH_NMAX_K <= (1u << GRAPH_ROOT_BITS) && GRAPH_NMAX_K < 0x8000u,
              "k_graph_relax matches roots by GRAPH_ROOT_BITS and keeps 15-bit indices");
static_assert(GRAPH_NMAX_BIG <= 0xFFFFu, "an edge holds its node j in 16 bits");
#ifndef PBGPU_GE_SLOTS
#define PBGPU_GE_SLOTS 192  // (round 5: 384 -> 192 with 8 waves a SIMD, below)
#endif
#ifndef PBGPU_GE_DIRECT_FAR
#define PBGPU_GE_DIRECT_FAR 0
#endif
// GE_DIRECT_FAR: chunks past the staged window a scan still tests directly before it turns
// to the prefilter queue (short scans, C2's, end within them)
constexpr uint32_t GE_NODES = 64, GE_SLOTS = PBGPU_GE_SLOTS, GE_BLOCK = 256, GE_DIRECT_FAR = PBGPU_GE_DIRECT_FAR;

DEV bool graph_on_device(const GraphDev& G, uint32_t n) { return n > 0 && n <= G.nmax && n <= GRAPH_NMAX_BIG; }
// super_read_name::overlap (super_read_name.cc:49-72) in registers for a name i of SA
// unitigs (wave-uniform: the wave's node): the smallest t >= max(SA - sb + 1, 1) with
// name_i[t..SA) == name_j[0..SA - t) (0: none), and whether the names are the same
template <int SA>
DEV void name_overlap_reg(const uint32_t (&a)[GRAPH_U], const uint32_t (&bu)[GRAPH_U], uint32_t sb, int32_t& nb,
                          bool& same) {
  const int t0 = SA - (int)sb + 1;
  nb = 0;
#pragma unroll
  for (int t = SA - 1; t >= 1; --t) {
    bool m = (t >= t0) & (a[t] == bu[0]);
#pragma unroll
    for (int qq = t + 1; qq < SA; ++qq) m &= a[qq] == bu[qq - t];
    nb = m ? SA - t : nb;
  }
  same = sb == (uint32_t)SA;
#pragma unroll
  for (int u = 0; u < SA; ++u) same &= a[u] == bu[u];
}
// G.bmax: a wave per 64 sorted positions.  Positions of reads left to the host hold an
// earlier batch's descriptors; they are never scanned, and a stale value can only raise
// a block's maximum (or make it +inf), which skips less, never more.
__global__ __launch_bounds__(256) void k_graph_bmax(GraphDev G, uint64_t n_recs) {
  const uint64_t blk = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if ((blk << 6) >= n_recs) return;
  const uint64_t q = (blk << 6) + lane;
  double v = -INFINITY;
  if (q < n_recs) {
    const double is = G.desc[q].imp_s, ie = G.desc[q].imp_e;
    if (!(is <= 1.0)) v = ie != ie ? INFINITY : ie;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  if (lane == 0) G.bmax[blk] = v;
}
// Waves per SIMD asked of the compiler (0: its choice).  The scans wait on memory (64% of
// their wave cycles on C4r), so occupancy pays: 8 waves (64 VGPRs, no spills) with a
// 192-slot staged window (≈14 KB of LDS a block) against 5 (100 VGPRs, 384 slots): graph
// stage C4r 155 -> 148 ms, C2 36.1 -> 32.2 (profiles/r05ze_edges_occupancy_ab.txt)
#ifndef PBGPU_GE_WAVES
#define PBGPU_GE_WAVES 8
#endif
template <bool OVF>
#if PBGPU_GE_WAVES
__attribute__((amdgpu_waves_per_eu(PBGPU_GE_WAVES, PBGPU_GE_WAVES)))
#endif
__global__ __launch_bounds__(GE_BLOCK) void k_graph_edges(GraphDev G, uint64_t n_recs, uint64_t n_ovf) {
  __shared__ double s_is[GE_SLOTS], s_ie[GE_SLOTS], s_er[GE_SLOTS];
  __shared__ uint32_t s_meta[GE_SLOTS], s_lpa[GE_SLOTS], s_po[GE_SLOTS];
  __shared__ double s_rl[GE_NODES];    // node i's read length and scan end: the
  __shared__ uint32_t s_end[GE_NODES];  // window's nodes only (OVF: WAVES <= GE_NODES slots)
  __shared__ uint32_t s_u[GRAPH_U * GE_SLOTS];  // [u * GE_SLOTS + slot]
  constexpr uint32_t WAVES = GE_BLOCK / 64;
  __shared__ uint32_t s_q[WAVES * 128];  // a wave's queue of positions to test in full
  uint32_t* const sq = s_q + (threadIdx.x >> 6) * 128;
  // OVF: slot t holds listed node blockIdx.x * WAVES + t; nothing else is staged
  const uint64_t q0 = (uint64_t)blockIdx.x * (OVF ? WAVES : GE_NODES);
  if (q0 >= (OVF ? n_ovf : n_recs)) return;
  const uint64_t lim = OVF ? n_ovf : n_recs;
  const uint32_t ns = (uint32_t)(lim - q0 < (OVF ? WAVES : GE_SLOTS) ? lim - q0 : (OVF ? WAVES : GE_SLOTS));
  for (uint32_t t = threadIdx.x; t < ns; t += GE_BLOCK) {
    const uint64_t q = OVF ? G.ovf_list[q0 + t] : q0 + t;
    const uint32_t r = G.recs[q].read;  // records are grouped per read
    const uint64_t e = G.rec_off[r + 1];
    const uint32_t n = (uint32_t)(e - G.rec_off[r]);
    // a read left to the host has no descriptors (k_graph_sort skipped it: G.desc holds an
    // earlier batch's words there), so nothing of it is read; its slots are never a j of a
    // device read's scan (scans stop at their read's end) and its nodes scan nothing
    const bool dev = graph_on_device(G, n);
    GDesc d{};
    if (dev) d = G.desc[q];
    s_is[t] = d.imp_s; s_ie[t] = d.imp_e; s_er[t] = d.err;
    s_meta[t] = d.idx | ((uint32_t)d.nsz << 16); s_lpa[t] = d.lp_add;
    s_po[t] = dev ? G.spo[q] : 0u;
    if (t < GE_NODES) {
      s_rl[t] = (double)(G.roff[r + 1] - G.roff[r]);
      s_end[t] = dev ? (uint32_t)e : (uint32_t)(q + 1);  // a read left to the host: no scan
    }
#pragma unroll
    for (uint32_t u = 0; u < GRAPH_U; ++u) s_u[u * GE_SLOTS + t] = d.u[u];
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const double play = G.play, kd = (double)G.k;
  const uint32_t km1 = G.k - 1;
  for (uint32_t ti = threadIdx.x >> 6; ti < (OVF ? WAVES : GE_NODES) && ti < ns; ti += WAVES) {
    const uint64_t q = OVF ? G.ovf_list[q0 + ti] : q0 + ti;
    const uint32_t qe = s_end[ti];
    const double ie_i = s_ie[ti], err_i = s_er[ti];
    uint32_t cnt = 0;
#ifdef PBGPU_PROF
    uint64_t ge_seen = 0, ge_far = 0, ge_cand = 0;
#endif
    if ((q + 1 < qe) & !(ie_i >= s_rl[ti])) {  // (imp_e >= rl: hanging off the 3' end)
      const uint32_t sa = s_meta[ti] >> 16, po_i = s_po[ti];
      const uint32_t sa_u = (uint32_t)__builtin_amdgcn_readfirstlane((int)sa);  // (uniform: the wave's node i)
      uint32_t a[GRAPH_U];
#pragma unroll
      for (uint32_t u = 0; u < GRAPH_U; ++u) a[u] = s_u[u * GE_SLOTS + ti];
      auto unit_i = [&](uint32_t t) -> uint32_t { return G.ounits[po_i + t]; };
      uint2* const out = OVF ? G.eovf : G.edges;
      const uint64_t ob = OVF ? G.eoff[q] - GRAPH_EBLK : q * GRAPH_EBLK;  // (mod 2^64)
      // the skip bits of blocks [ck_b0, ck_b0 + 64) for node i (set: not skippable), kept
      // across chunks: a test is one bmax load a lane, needed again only past those blocks
      uint64_t ck_b0 = 0, ck_m = 0;
      bool ck_set = false;
      // Fast-forward over whole 64-position blocks in which every node is skipped for node i
      // (imp_s <= 1, or not advancing: imp_e_i > imp_e_j + 31): none of them can give an
      // edge or the break.  On repeat-rich reads most of a long node's scan is nodes it
      // contains (C4r: 73% of 252 G scanned positions were skips).  Returns the position
      // the chunk at j0 really starts at (>= qe: the scan is over).
      auto next_pos = [&](uint64_t j0) -> uint64_t {
        if (j0 >= qe) return j0;
        uint64_t b0 = j0 >> 6;
        for (;;) {
          if (!ck_set || b0 - ck_b0 >= 64) {  // (b0 never decreases)
            ck_set = true;
            ck_b0 = b0;
            const uint64_t bb = b0 + lane;
            const bool in = (bb << 6) < qe;
            const double m = in ? G.bmax[bb] : 0.0;
            ck_m = __ballot(!(in & (ie_i > __dadd_rn(m, 31.0))));
          }
          const uint64_t nsk = ck_m >> (b0 - ck_b0);
          if (nsk & 1ull) break;  // block b0 is scanned
          if (!nsk) { b0 = ck_b0 + 64; continue; }  // all 64 skipped: test the next 64
          b0 += (uint64_t)__ffsll((unsigned long long)nsk) - 1;  // the first block that is not
          break;
        }
        return (b0 << 6) > j0 ? b0 << 6 : j0;
      };
      // The prefilter of the chunk [j0, j0 + 64): the positions that can be the reference's
      // break or an edge of node i, a superset of both -- not skipped, and the break test
      // itself or j's first unitig among i's unitigs 1 .. sa - 1 (super_read_name::overlap
      // matches name_j[0] at some t >= 1 of name_i; every position for names longer than
      // GRAPH_U).  Four fields a position, staged or from the per-field arrays (coalesced);
      // positions past the first break are dropped.  brk: the chunk holds the break.
      auto pre = [&](uint64_t j0, bool& brk) -> uint64_t {
        const uint64_t j = j0 + lane;
        const bool act = j < qe;
        const uint64_t jj = act ? j : q;
        const uint32_t sj = (uint32_t)(jj - q0);
        const bool staged = !OVF && sj < ns;
        double is_j, ie_j, er_j;
        uint32_t u0;
        if (staged) {
          is_j = s_is[sj]; ie_j = s_ie[sj]; er_j = s_er[sj]; u0 = s_u[sj];
        } else {
#ifndef PBGPU_GE_FLAT
          // (global loads spelled out: the compiler made these four flat loads, which also
          // count against the LDS counter the queue's waits use)
          typedef const __attribute__((address_space(1))) double gdbl;
          typedef const __attribute__((address_space(1))) uint32_t gu32;
          is_j = ((gdbl*)G.fis)[jj]; ie_j = ((gdbl*)G.fie)[jj]; er_j = ((gdbl*)G.fer)[jj]; u0 = ((gu32*)G.fu0)[jj];
#else
          is_j = G.fis[jj]; ie_j = G.fie[jj]; er_j = G.fer[jj]; u0 = G.fu0[jj];
#endif
        }
        const bool skip = (is_j <= 1.0) | (ie_i > __dadd_rn(ie_j, 31.0));
        const double position_len = __dadd_rn(ie_i, -is_j);
        const double error = __dmul_rn(G.nb_errors, __dadd_rn(err_i, er_j));
        const bool b = act & !skip & (__dadd_rn(__dmul_rn(position_len, play), error) < kd);
        bool m = sa_u > GRAPH_U;
#pragma unroll
        for (uint32_t t = 1; t < GRAPH_U; ++t) m |= (t < sa_u) & (a[t] == u0);
        uint64_t pm = __ballot(act & !skip & (b | m));
        const uint64_t bm = __ballot(b);
        brk = bm != 0;
        if (brk) pm &= bm ^ (bm - 1);  // through the first break
#ifdef PBGPU_PROF
        ge_seen += (uint64_t)__builtin_popcountll(__ballot(act));
        ge_far += (uint64_t)__builtin_popcountll(__ballot(act & !staged));
#endif
        return pm;
      };
      // node i's tests on the chunk [x, x + 64) (direct) or on the queued positions sq[0 .. x),
      // in j order; true at the reference's break
      auto chunk = [&](uint64_t x, auto direct_c) -> bool {
        constexpr bool direct = decltype(direct_c)::value;  // (two instantiations)
        const bool act = direct ? x + lane < qe : lane < x;
        const uint64_t j = direct ? x + lane : (act ? (uint64_t)sq[lane] : q);
        const uint32_t sj = (uint32_t)((act ? j : q) - q0);
#ifdef PBGPU_GRAPH_CHECK
        if (act) GCHECK(j > q && j < qe && j < n_recs, 0);
        {
          const uint64_t am = __ballot(act);
          if (lane == 0 && am) atomicAdd(&g_graph_check[4], (unsigned long long)__builtin_popcountll(am));
        }
#endif
        // node j: staged, or (a scan past the window) one 64-byte line from HBM.  Every load
        // is issued before the tests (measured: loading the name only where the name test
        // runs, after the skip / break ballot, made the C4r graph stage 240 -> 316 ms: a
        // second round trip on the critical path costs more than the loads it saves; and
        // loading the next chunk's lines one chunk ahead, two register sets, was slower
        // too: C4r 159 -> 178 ms, C2 36.5 -> 38.8 at 5 waves a SIMD; against the 8-wave
        // kernel, 149 -> 162 / 298 / 562 ms at 5 / 6 / 8 waves, its registers spilling)
        double is_j, ie_j, er_j;
        uint32_t mj, lpa_j, bu[GRAPH_U], po_j;
        const bool staged = !OVF && sj < ns;
        if (staged) {
          is_j = s_is[sj]; ie_j = s_ie[sj]; er_j = s_er[sj]; mj = s_meta[sj]; lpa_j = s_lpa[sj]; po_j = 0;
#pragma unroll
          for (uint32_t u = 0; u < GRAPH_U; ++u) bu[u] = s_u[u * GE_SLOTS + sj];
        } else {
          const GDesc dj = G.desc[act ? j : q];
          po_j = G.spo[act ? j : q];  // (coalesced, issued with the node: no second round trip)
#ifdef PBGPU_GRAPH_CHECK
          if (act) GCHECK((uint64_t)po_j + dj.nsz <= G.units_total, 1);
#endif
          is_j = dj.imp_s; ie_j = dj.imp_e; er_j = dj.err; mj = dj.idx | ((uint32_t)dj.nsz << 16); lpa_j = dj.lp_add;
#pragma unroll
          for (uint32_t u = 0; u < GRAPH_U; ++u) bu[u] = dj.u[u];
        }
        const bool skip = (is_j <= 1.0) | (ie_i > __dadd_rn(ie_j, 31.0));  // off the 5' end | not advancing
        const double position_len = __dadd_rn(ie_i, -is_j);
        const double error = __dmul_rn(G.nb_errors, __dadd_rn(err_i, er_j));
        const bool brk = act & !skip & (__dadd_rn(__dmul_rn(position_len, play), error) < kd);
        const uint64_t bm = __ballot(brk);
        const uint32_t fb = bm ? (uint32_t)__ffsll((long long)bm) - 1 : 64u;
        const uint32_t sb = mj >> 16;
        const bool cand = act & !skip & (lane < fb) & (sa >= 2) & (sb >= 2);
        bool edge = false;
        int32_t nb = 0, common = 0;
        // j's name offset (its prefix sums, and its units past GRAPH_U): staged, or loaded
        // with the node.  (Round 5: the far nodes' offset came from G.poff by j's record
        // index, a second dependent round trip; G.spo holds it by sorted position.)
        auto po_of_j = [&]() -> uint32_t { return staged ? s_po[sj] : po_j; };
        if (cand) {
          bool same;
          if ((sa <= GRAPH_U) & (sb <= GRAPH_U)) {
            // specialized by the wave-uniform name size of node i: the compare network
            // of SA unitigs, not of GRAPH_U (names are mostly 2-5 unitigs)
            switch (sa_u) {
              case 2: name_overlap_reg<2>(a, bu, sb, nb, same); break;
              case 3: name_overlap_reg<3>(a, bu, sb, nb, same); break;
              case 4: name_overlap_reg<4>(a, bu, sb, nb, same); break;
              case 5: name_overlap_reg<5>(a, bu, sb, nb, same); break;
              case 6: name_overlap_reg<6>(a, bu, sb, nb, same); break;
              case 7: name_overlap_reg<7>(a, bu, sb, nb, same); break;
              default: name_overlap_reg<8>(a, bu, sb, nb, same); break;
            }
          } else {
            const uint32_t po_j = po_of_j();
            auto unit_j = [&](uint32_t qq) -> uint32_t { return G.ounits[po_j + qq]; };
            const uint32_t u0 = unit_j(0);
            const int t0 = (int)sa - (int)sb + 1;
            for (uint32_t t = t0 > 1 ? (uint32_t)t0 : 1u; t < sa; ++t) {
              if (unit_i(t) != u0) continue;
              uint32_t qq = t + 1;
              while (qq < sa && unit_i(qq) == unit_j(qq - t)) ++qq;
              if (qq == sa) { nb = (int32_t)(sa - t); break; }
            }
            same = false;
            if (nb && sb == sa) {  // the same super-read name
              same = true;
              for (uint32_t u = 0; u < sa && same; ++u) same = unit_i(u) == unit_j(u);
            }
          }
          if (nb && !same) {
#ifdef PBGPU_GRAPH_CHECK
            GCHECK((uint64_t)po_of_j() + (uint32_t)nb < G.units_total, 2);
#endif
            const uint2 v = G.pp[po_of_j() + (uint32_t)nb];
            const int32_t uol = (int32_t)(v.x - (uint32_t)(nb - 1) * km1);
            common = (int32_t)v.y;
            const double duol = (double)uol;
            edge = !((duol > __dadd_rn(__dmul_rn(play, position_len), error)) |
                     (position_len > __dmul_rn(play, __dadd_rn(duol, error))));
          }
        }
        const uint64_t em = __ballot(edge);
        const uint32_t at = cnt + (uint32_t)__builtin_popcountll(em & ((1ull << lane) - 1));
        if (edge & (OVF ? at >= GRAPH_EBLK : at < GRAPH_EBLK)) {
          // the edge's path increment (nb_mers or sr_cover of j minus the common k-mers) and
          // the unitigs it adds (overlap_graph.cc:47-53)
          out[ob + at] = make_uint2((mj & 0xFFFFu) | ((sb - (uint32_t)nb) << 16), lpa_j - (uint32_t)common);
        }
        cnt += (uint32_t)__builtin_popcountll(em);
#ifdef PBGPU_PROF
        ge_cand += (uint64_t)__builtin_popcountll(__ballot(cand));
        if (direct) ge_seen += (uint64_t)__builtin_popcountll(__ballot(act & (lane < fb)));
#endif
        return bm != 0;
      };
      // Chunks inside the staged window are tested directly (LDS loads are cheap).  Past it,
      // the prefilter's positions are queued in j order (sq, up to 127) and tested in full
      // 64 at a time: on repeat-rich reads few of the positions a long scan passes are
      // candidates (C4r: 23 of 940 a node, 88% of them past the window), and a chunk with
      // one cost a whole chunk of 64-byte node loads and tests.  A chunk holding the break
      // ends the scan, the queue tested through it.  (C4r edges 97.5 -> 63.5 ms, 55.1 with the
      // prefilter's global loads; C2 9.0 -> 10.3; the queue for the staged chunks too made C2 11.7 ms, and testing 2 or 5 chunks
      // past the window directly first was slower on both: profiles/r05zw_*, r05zx_*.)
      uint32_t qn = 0;
      bool done = false;
      uint64_t j0 = next_pos(q + 1);
      const uint64_t win_end = OVF ? 0 : q0 + ns;
      for (uint32_t nfar = 0; j0 < qe; j0 = next_pos(j0 + 64)) {
        const bool far = (j0 + 64 < qe ? j0 + 64 : qe) > win_end;
        if (far && nfar >= GE_DIRECT_FAR) break;  // a long scan: the queue from here
        nfar += far ? 1u : 0u;
        if (chunk(j0, std::true_type{})) { done = true; break; }
      }
      for (; j0 < qe && !done; j0 = next_pos(j0 + 64)) {
        bool brk;
        const uint64_t pm = pre(j0, brk);
        if ((pm >> lane) & 1ull)
          sq[qn + (uint32_t)__builtin_popcountll(pm & ((1ull << lane) - 1))] = (uint32_t)(j0 + lane);
        qn += (uint32_t)__builtin_popcountll(pm);
        if (qn >= 64 || brk) {
          lds_fence();
          done = chunk(qn < 64 ? qn : 64, std::false_type{});
          if (qn > 64) {  // the rest to the front
            const uint32_t v = lane + 64 < qn ? sq[lane + 64] : 0u;
            lds_fence();
            sq[lane] = v;
            lds_fence();
            qn -= 64;
            if (!done && brk) done = chunk(qn, std::false_type{});
          } else {
            qn = 0;
          }
          done |= brk;
        }
      }
      if (!done && qn) {
        lds_fence();
        chunk(qn, std::false_type{});
      }
    }
#ifdef PBGPU_PROF
    if (!OVF) {  // slots 128..130: positions scanned, of them past the staged window, candidates (name test)
      PROF_ADD(128, ge_seen); PROF_ADD(129, ge_far); PROF_ADD(130, ge_cand);
    }
#endif
    if (!OVF && lane == 0) {
      G.ecnt[q] = cnt;
      if (cnt > GRAPH_EBLK) {  // its region past the block, and listed
        G.eoff[q] = atomicAdd((unsigned long long*)&G.ovf[1], (unsigned long long)(cnt - GRAPH_EBLK));
        G.ovf_list[atomicAdd((unsigned long long*)&G.ovf[0], 1ull)] = q;
      }
    }
  }
}

// k_graph_relax: a block of two waves per read, both streaming the read's edges
// node by node in sorted order (each node's block, GRAPH_RELAX_PF nodes ahead in
// flight; the rare edges past a block as they come).  Wave 0 relaxes
// the longest paths: node i's edges update their own node j each (distinct j per
// lane, as the reference's updates for one i are independent).  Wave 1 unites them
// in j order (union_find.cc:13-23): the pre-scan roots are found in parallel (path
// halving; a root never changes by compression, and the roots are what the output
// needs), a root already met, or i's own, is a no-op, the rest are merged in
// registers with the reference's rank rule.  The unions never read the paths and
// the paths never read the sets, so the two waves run unsynchronized until the end.
// Node state lives in LDS by record index, 18 B a node (four blocks a CU at NM =
// 2048); tiers by records a read (NM).  Each node's record index and edge count come
// from HBM, 64 positions a load, one load ahead.  The start node's implied start
// (lstart_imp_s), which the reference compares as a double, is kept as its rank key:
// the first sorted position of its imp_s value (the nodes are sorted by imp_s, so
// a > b exactly when their keys are), NaN as RANK_NAN, which compares false.
template <uint32_t NM>
DEV bool graph_relax_tier(const GraphDev& G, uint32_t n) {
  if (!graph_on_device(G, n) || n > G.relax_big_min) return false;
  return (n <= NM && n > NM / 2) || (NM == GRAPH_RELAX_MIN && n <= NM);
}
template <uint32_t NM>
__global__ __launch_bounds__(128) void k_graph_relax(GraphDev G, uint32_t n_reads) {
  __shared__ int32_t s_lp[NM], s_lun[NM];
  __shared__ int16_t s_lst[NM], s_lpv[NM];
  __shared__ uint16_t s_lsk[NM], s_par[NM];
  __shared__ uint8_t s_rank[NM], s_fl[NM];  // s_fl: 1 an edge into it, 2 an edge out of it
  __shared__ uint64_t s_head[NM / 64];       // sorted positions starting an imp_s value
  constexpr uint32_t RANK_NAN = 0xFFFFu;
  const uint32_t r = blockIdx.x;
  if (r >= n_reads) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint64_t b = G.rec_off[r];
  const uint32_t n = (uint32_t)(G.rec_off[r + 1] - b);
  if (n == 0) return;
  if (!graph_on_device(G, n)) {  // the host traverses this read (marked by the top tier)
    if (NM == GRAPH_NMAX)
      for (uint32_t i = tid; i < n; i += 128) G.out[b + i] = GraphNode{0, -1, -1, 0, i, GRAPH_HOST};
    return;
  }
  if (!graph_relax_tier<NM>(G, n)) return;
  // node_info::reset (overlap_graph.hpp:24-34) of every node; the imp_s value heads
  for (uint32_t p0 = 0; p0 < n; p0 += 128) {
    const uint32_t p = p0 + tid;
    bool head = false;
    if (p < n) {
      const GDesc d = G.desc[b + p];
      const uint32_t it = d.idx;
      head = p == 0 || !(G.desc[b + p - 1].imp_s == d.imp_s);  // (-0 == +0; a NaN heads its own)
      s_lp[it] = (int32_t)d.lp_add; s_lun[it] = (int32_t)d.nsz; s_lst[it] = -1; s_lpv[it] = -1;
      s_fl[it] = G.ecnt[b + p] ? 2 : 0;
      s_par[it] = (uint16_t)it; s_rank[it] = 0;
    }
    const uint64_t hm = __ballot(head);
    if (lane == 0 && p < NM) s_head[p >> 6] = hm;
  }
  __syncthreads();
  for (uint32_t p = tid; p < n; p += 128) {  // rank key: the last head at or before p
    const GDesc d = G.desc[b + p];
    uint32_t w = p >> 6;
    uint64_t m = s_head[w] & (~0ull >> (63 - (p & 63)));
    while (!m) m = s_head[--w];  // position 0 is a head
    s_lsk[d.idx] = d.imp_s != d.imp_s ? RANK_NAN : w * 64 + 63 - (uint32_t)__builtin_clzll(m);
  }
  __syncthreads();
  const bool paths = tid < 64;
  // per sorted position: record index | edge count << 16; cur holds [c0, c0 + 64), nxt the
  // next 64 (in flight)
  auto ldw = [&](uint32_t p) -> uint32_t {
    return p < n ? (G.desc[b + p].idx | (G.ecnt[b + p] << 16)) : 0u;
  };
  uint32_t c0 = 0, cur = ldw(lane), nxt = ldw(64 + lane);
  auto wd = [&](uint32_t x) -> uint32_t {  // x wave-uniform, in [c0, c0 + 128)
    const uint32_t o = x - c0;
    return (uint32_t)__builtin_amdgcn_readlane((int)(o < 64 ? cur : nxt), (int)(o & 63));
  };
  // the nodes' edge blocks: pf[d] holds node p + d's (lanes past its count zero)
  const uint2* EB = G.edges + b * GRAPH_EBLK;
  auto ldb = [&](uint32_t p, uint32_t ec) -> uint2 {
    return lane < (ec < GRAPH_EBLK ? ec : GRAPH_EBLK) ? EB[(uint64_t)p * GRAPH_EBLK + lane] : make_uint2(0u, 0u);
  };
  uint2 pf[GRAPH_RELAX_PF];
#pragma unroll
  for (uint32_t d = 0; d < GRAPH_RELAX_PF; ++d) pf[d] = ldb(d, wd(d) >> 16);

#ifdef PBGPU_PROF
  uint64_t pr_find = 0, pr_merge = 0, pr_paths = 0, pr_chunks = 0;
  const uint64_t pr0 = __builtin_amdgcn_s_memtime();
#endif
  for (uint32_t p = 0; p < n; ++p) {
    if (p - c0 == 64) {
      c0 += 64; cur = nxt;
      nxt = ldw(c0 + 64 + lane);
    }
    const uint32_t w = wd(p), ec = w >> 16, it_i = w & 0xFFFFu;
    const uint2 blk = pf[0];
#pragma unroll
    for (uint32_t d = 0; d + 1 < GRAPH_RELAX_PF; ++d) pf[d] = pf[d + 1];
    pf[GRAPH_RELAX_PF - 1] = ldb(p + GRAPH_RELAX_PF, wd(p + GRAPH_RELAX_PF) >> 16);
    if (ec == 0) continue;
    int32_t lp_i = 0, lun_i = 0, lst_i = 0;
    uint32_t lsk_i = 0;
    if (paths) { lp_i = s_lp[it_i]; lun_i = s_lun[it_i]; lst_i = s_lst[it_i]; lsk_i = s_lsk[it_i]; }
    for (uint32_t k0 = 0; k0 < ec; k0 += 64) {
      const bool edge = k0 + lane < ec;
      // past the block: the node's overflow region (G.eoff)
      // the first GRAPH_EBLK edges from the node's block (prefetched), the rest from its region past it
      const uint2 ce = k0 + lane < GRAPH_EBLK ? blk
                                              : (edge ? G.eovf[G.eoff[b + p] + (k0 + lane - GRAPH_EBLK)] : make_uint2(0u, 0u));
      const uint32_t it_j = ce.x & 0xFFFFu;
#ifdef PBGPU_GRAPH_CHECK
      if (edge) GCHECK(it_j < n, 3);
#endif
      PROF_T(pa);
#ifdef PBGPU_PROF
      ++pr_chunks;
#endif
      if (paths) {
        if (edge) {  // node_info update (overlap_graph.cc:41-56); this lane owns node j
          s_fl[it_j] |= 1;  // an edge into j: not a start node
          const int32_t nlpath = (int32_t)((uint32_t)lp_i + ce.y);
          const int32_t lp_j = s_lp[it_j];
          bool upd = nlpath > lp_j;
          if (!upd && nlpath == lp_j) {  // (lstart_imp_s: lsk_i > lsk_j, neither NaN)
            const uint32_t lsk_j = s_lsk[it_j];
            upd = s_lst[it_j] == -1 || ((lsk_i != RANK_NAN) & (lsk_j != RANK_NAN) & (lsk_i > lsk_j));
          }
          if (upd) {
            s_lp[it_j] = nlpath;
            s_lst[it_j] = (int16_t)(lst_i == -1 ? (int32_t)it_i : lst_i);
            s_lsk[it_j] = (uint16_t)lsk_i;
            s_lpv[it_j] = (int16_t)it_i;
            s_lun[it_j] = lun_i + (int32_t)(ce.x >> 16);
          }
        }
#ifdef PBGPU_PROF
        lds_fence();
        pr_paths += __builtin_amdgcn_s_memtime() - pa;
#endif
      } else {
        // union_sets(it_i, it_j) for this chunk's edges in j order
        // both roots in one walk (path halving on each): the two chains' LDS round trips
        // overlap instead of following one another
        uint32_t r1 = it_i, R = edge ? it_j : it_i;
        for (;;) {
          const uint32_t p1 = s_par[r1], p2 = s_par[R];
          if ((p1 == r1) & (p2 == R)) break;
          const uint32_t g1 = s_par[p1], g2 = s_par[p2];
          if (p1 != r1) { s_par[r1] = (uint16_t)g1; r1 = g1; }
          if (p2 != R) { s_par[R] = (uint16_t)g2; R = g2; }
        }
        if (!edge) R = r1;
        // most edges join nodes already in i's set: nothing to merge then
        const uint64_t fo = __ballot(edge & (R != r1));
        PROF_T(pb);
#ifdef PBGPU_PROF
        pr_find += pb - pa;
#endif
        uint64_t fm = fo;
        if (fo & (fo - 1)) {  // two or more foreign edges: the first lane of each root
          // the edge lanes holding the same root: a ballot per bit of R (node indices < 2^13)
          uint64_t same = fo;
#pragma unroll
          for (uint32_t bit = 0; bit < GRAPH_ROOT_BITS; ++bit) {
            const uint64_t bb = __ballot((R >> bit) & 1u);
            same &= ((R >> bit) & 1u) ? bb : ~bb;
          }
          fm = __ballot(((fo >> lane) & 1) && (same & ((1ull << lane) - 1)) == 0);
        }
        const uint32_t rk = fm ? s_rank[R] : 0u;
        uint32_t cr = r1, crank = fm ? s_rank[r1] : 0u;
        for (; fm; fm &= fm - 1) {
          const uint32_t l = (uint32_t)__ffsll((long long)fm) - 1;
          const uint32_t vv = (uint32_t)__builtin_amdgcn_readlane((int)R, (int)l);
          const uint32_t vr = (uint32_t)__builtin_amdgcn_readlane((int)rk, (int)l);
          if (crank > vr) {
            if (lane == 0) s_par[vv] = (uint16_t)cr;
          } else if (crank < vr) {
            if (lane == 0) s_par[cr] = (uint16_t)vv;
            cr = vv; crank = vr;
          } else {
            ++crank;
            if (lane == 0) { s_par[vv] = (uint16_t)cr; s_rank[cr] = (uint8_t)crank; }
          }
        }
#ifdef PBGPU_PROF
        lds_fence();
        pr_merge += __builtin_amdgcn_s_memtime() - pb;
#endif
      }
      // a wave's LDS operations execute in order, so the next chunk's reads see this one's
      // writes; the fence keeps the compiler from moving memory operations across
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
#ifdef PBGPU_PROF
  // slots 80..: [paths wave] chunk ticks, chunks, total; [union wave] find ticks, merge ticks,
  // total; nodes; blocks (NM = 4096 / 2048 tiers at +16)
  {
    const uint32_t sl = 80 + (NM > GRAPH_NM_SMALL ? 16 : 0);
    const uint64_t tot = __builtin_amdgcn_s_memtime() - pr0;
    if (paths) { PROF_ADD(sl + 0, pr_paths); PROF_ADD(sl + 1, pr_chunks); PROF_ADD(sl + 2, tot); PROF_ADD(sl + 6, n); PROF_ADD(sl + 7, 1); }
    else { PROF_ADD(sl + 3, pr_find); PROF_ADD(sl + 4, pr_merge); PROF_ADD(sl + 5, tot); }
  }
#endif
  __syncthreads();
  for (uint32_t i = tid; i < n; i += 128) {
    uint32_t q = i;
    while (s_par[q] != q) q = s_par[q];
    // start node: no edge into it; end node: no edge out of it
    const uint32_t fl = (s_fl[i] & 1 ? 0u : GRAPH_START) | (s_fl[i] & 2 ? 0u : GRAPH_END);
    G.out[b + i] = GraphNode{s_lp[i], s_lst[i], s_lpv[i], s_lun[i], q, fl};
  }
}
// Reads of more than GRAPH_NMAX records (up to GRAPH_NMAX_BIG; on C4r-shaped reads 1.8%
// of the reads, round 4 left them to the host graph at ~10 ms of a core each): the same
// two steps with their keys and node state in the read's region of G.scratch (6 words a
// record) instead of LDS, one block per such read.
constexpr uint32_t GRAPH_BIG_BLOCK = 1024;
DEV bool graph_big(const GraphDev& G, uint32_t n) { return n > GRAPH_NMAX && graph_on_device(G, n); }
// the relaxation with its state in HBM: the reads past the LDS tiers, and those past
// G.relax_big_min (their blocks, no LDS, share a CU where an LDS tier's block takes it)
DEV bool graph_relax_big(const GraphDev& G, uint32_t n) { return n > G.relax_big_min && graph_on_device(G, n); }
// k_graph_sort for one big read: the bitonic network over np2 <= 2n entries of {hi, lo, ex}
__global__ __launch_bounds__(GRAPH_BIG_BLOCK) void k_graph_sort_big(GraphDev G, uint32_t n_reads) {
  const uint32_t r = blockIdx.x;
  if (r >= n_reads) return;
  const uint64_t b = G.rec_off[r];
  const uint32_t n = (uint32_t)(G.rec_off[r + 1] - b);
  if (!graph_big(G, n)) return;
  uint32_t np2 = 1;
  while (np2 < n) np2 <<= 1;
  uint64_t* hi = G.scratch + 6 * b;
  uint64_t* lo = hi + np2;
  uint64_t* ex = lo + np2;
  for (uint32_t i = threadIdx.x; i < np2; i += GRAPH_BIG_BLOCK) {
    if (i < n) {
      const double2 m = G.imp[b + i];
      hi[i] = graph_dkey(m.x); lo[i] = graph_dkey(m.y); ex[i] = i;
    } else {
      hi[i] = ~0ull; lo[i] = ~0ull; ex[i] = ~0ull;
    }
  }
  __syncthreads();
  bitonic_keys<GRAPH_BIG_BLOCK>(hi, lo, ex, np2);
  for (uint32_t p = threadIdx.x; p < n; p += GRAPH_BIG_BLOCK) {
    graph_write_desc(G, b + p, b, (uint32_t)ex[p]);
  }
}
// k_graph_relax for one big read, node state in HBM (a 16-byte path record per node, the
// union-find's parent and rank as u32 arrays, then the imp_s head bitmap): the same two
// waves, the same order of updates and unions.  The state is this block's alone and both
// waves run on one CU, so plain loads and stores with a workgroup fence after each chunk
// (its stores complete before the next chunk's loads) order it as the LDS kernel's in-order
// LDS does.  A node's path fields are one record so that a node j's test and update are one
// load and one store (round 5: five arrays, two dependent round trips and the flag's
// read-modify-write a node).
struct alignas(16) RelaxPath {
  int32_t lp, lun;       // longest path, its unitigs
  uint16_t lst, lpv;     // start and previous node (0xFFFF: -1)
  uint16_t lsk, fl;      // the start's implied-start key (0xFFFF: NaN), flags (1 an edge in, 2 out)
};
// (Measured: the union-find's parent and rank in LDS for reads of <= 8192 records, 3 B a
// node, gained nothing -- C4r graph stage 154.2 vs 154.7 ms -- and <= 16384 lost 10 ms.
// Round 6, again with the union-find 2 B a node in LDS (a root's word holding its rank) in
// tiers of 4096 / 8192 / 16384 / 32768 records on three streams: the union wave 4699 -> 1893
// cycles a node, the paths wave, 2159-2541, then bounds it; the longest launch 26.5 -> 18.1 ms
// and the resident graph stage of 20k C4r reads 107.3 -> 106.2 ms, but create_mega_reads on
// them 0.35 -> 0.38 s: blocks that hold LDS for 10-18 ms take it from the other aligner's
// k_group tables.  profiles/r06y_relax_uf_lds_tried.txt.)
__global__ __launch_bounds__(128) void k_graph_relax_big(GraphDev G, uint32_t n_reads) {
  constexpr uint32_t RANK_NAN = 0xFFFFu, NONE = 0xFFFFu;
  const uint32_t r = blockIdx.x;
  if (r >= n_reads) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint64_t b = G.rec_off[r];
  const uint32_t n = (uint32_t)(G.rec_off[r + 1] - b);
  if (!graph_relax_big(G, n)) return;
  RelaxPath* S = reinterpret_cast<RelaxPath*>(G.scratch + 6 * b);  // 16 n bytes
  uint32_t* const s_par = reinterpret_cast<uint32_t*>(S + n);      // the union-find: 8 n bytes
  uint32_t* const s_rank = s_par + n;
  uint64_t* s_head = G.scratch + 6 * b + 4 * (uint64_t)n;     // (n + 63) / 64 words: within 6n
  static_assert(sizeof(RelaxPath) == 16, "path record");
  for (uint32_t p0 = 0; p0 < n; p0 += 128) {
    const uint32_t p = p0 + tid;
    bool head = false;
    if (p < n) {
      const GDesc d = G.desc[b + p];
      const uint32_t it = d.idx;
      head = p == 0 || !(G.desc[b + p - 1].imp_s == d.imp_s);  // (-0 == +0; a NaN heads its own)
      RelaxPath ps;
      ps.lp = (int32_t)d.lp_add; ps.lun = (int32_t)d.nsz; ps.lst = 0xFFFFu; ps.lpv = 0xFFFFu;
      ps.lsk = 0; ps.fl = G.ecnt[b + p] ? 2 : 0;
      S[it] = ps;
      s_par[it] = it; s_rank[it] = 0;
    }
    const uint64_t hm = __ballot(head);
    if (lane == 0 && p < n) s_head[p >> 6] = hm;
  }
  __syncthreads();
  for (uint32_t p = tid; p < n; p += 128) {  // rank key: the last head at or before p
    const GDesc d = G.desc[b + p];
    uint32_t w = p >> 6;
    uint64_t m = s_head[w] & (~0ull >> (63 - (p & 63)));
    while (!m) m = s_head[--w];  // position 0 is a head
    S[d.idx].lsk = (uint16_t)(d.imp_s != d.imp_s ? RANK_NAN : w * 64 + 63 - (uint32_t)__builtin_clzll(m));
  }
  __syncthreads();
  const bool paths = tid < 64;
  auto ldw = [&](uint32_t p) -> uint32_t {
    return p < n ? (G.desc[b + p].idx | (G.ecnt[b + p] << 16)) : 0u;
  };
  // (a node's edges go to later nodes of its read: at most n - 1 <= 65534, so the count fits
  // the packed word's 16 bits)
  static_assert(GRAPH_NMAX_BIG <= 0xFFFFu, "edge counts fit 16 bits");
  uint32_t c0 = 0, cur = ldw(lane), nxt = ldw(64 + lane);
  auto wd = [&](uint32_t x) -> uint32_t {
    const uint32_t o = x - c0;
    return (uint32_t)__builtin_amdgcn_readlane((int)(o < 64 ? cur : nxt), (int)(o & 63));
  };
  const uint2* EB = G.edges + b * GRAPH_EBLK;
  auto ldb = [&](uint32_t p, uint32_t ec) -> uint2 {
    return lane < (ec < GRAPH_EBLK ? ec : GRAPH_EBLK) ? EB[(uint64_t)p * GRAPH_EBLK + lane] : make_uint2(0u, 0u);
  };
  uint2 pf[GRAPH_RELAX_PF];
#pragma unroll
  for (uint32_t d = 0; d < GRAPH_RELAX_PF; ++d) pf[d] = ldb(d, wd(d) >> 16);
  PROF_T(rb_t0);
  for (uint32_t p = 0; p < n; ++p) {
    if (p - c0 == 64) {
      c0 += 64; cur = nxt;
      nxt = ldw(c0 + 64 + lane);
    }
    const uint32_t w = wd(p), ec = w >> 16, it_i = w & 0xFFFFu;  // (round 5: ec was a load a node)
    const uint2 blk = pf[0];
#pragma unroll
    for (uint32_t d = 0; d + 1 < GRAPH_RELAX_PF; ++d) pf[d] = pf[d + 1];
    pf[GRAPH_RELAX_PF - 1] = ldb(p + GRAPH_RELAX_PF, wd(p + GRAPH_RELAX_PF) >> 16);
    if (ec == 0) continue;
    RelaxPath si{};
    if (paths) si = S[it_i];
    const int32_t lp_i = si.lp, lun_i = si.lun;
    const uint32_t lst_i = si.lst, lsk_i = si.lsk;
    for (uint32_t k0 = 0; k0 < ec; k0 += 64) {
      const bool edge = k0 + lane < ec;
      // the first GRAPH_EBLK edges from the node's block (prefetched), the rest from its region past it
      const uint2 ce = k0 + lane < GRAPH_EBLK ? blk
                                              : (edge ? G.eovf[G.eoff[b + p] + (k0 + lane - GRAPH_EBLK)] : make_uint2(0u, 0u));
      const uint32_t it_j = ce.x & 0xFFFFu;
#ifdef PBGPU_GRAPH_CHECK
      if (edge) GCHECK(it_j < n, 3);
#endif
      if (paths) {
        if (edge) {  // node_info update (overlap_graph.cc:41-56); this lane owns node j
          RelaxPath sj = S[it_j];
          sj.fl |= 1;  // an edge into j: not a start node
          const int32_t nlpath = (int32_t)((uint32_t)lp_i + ce.y);
          bool upd = nlpath > sj.lp;
          if (!upd && nlpath == sj.lp)  // (lstart_imp_s: lsk_i > lsk_j, neither NaN)
            upd = sj.lst == NONE || ((lsk_i != RANK_NAN) & (sj.lsk != RANK_NAN) & (lsk_i > sj.lsk));
          if (upd) {
            sj.lp = nlpath;
            sj.lst = (uint16_t)(lst_i == NONE ? it_i : lst_i);
            sj.lsk = (uint16_t)lsk_i;
            sj.lpv = (uint16_t)it_i;
            sj.lun = lun_i + (int32_t)(ce.x >> 16);
          }
          S[it_j] = sj;
        }
      } else {
        // union_sets(it_i, it_j) for this chunk's edges in j order (union_find.cc:13-23)
        uint32_t r1 = it_i, R = edge ? it_j : it_i;
        for (;;) {
          const uint32_t p1 = s_par[r1], p2 = s_par[R];
          if ((p1 == r1) & (p2 == R)) break;
          const uint32_t g1 = s_par[p1], g2 = s_par[p2];
          if (p1 != r1) { s_par[r1] = g1; r1 = g1; }
          if (p2 != R) { s_par[R] = g2; R = g2; }
        }
        if (!edge) R = r1;
        const uint64_t fo = __ballot(edge & (R != r1));
        uint64_t fm = fo;
        if (fo & (fo - 1)) {  // the first lane of each foreign root: a ballot per bit of R (< 2^16)
          uint64_t same = fo;
#pragma unroll
          for (uint32_t bit = 0; bit < 16; ++bit) {
            const uint64_t bb = __ballot((R >> bit) & 1u);
            same &= ((R >> bit) & 1u) ? bb : ~bb;
          }
          fm = __ballot(((fo >> lane) & 1) && (same & ((1ull << lane) - 1)) == 0);
        }
        const uint32_t rk = fm ? s_rank[R] : 0u;
        uint32_t cr = r1, crank = fm ? s_rank[r1] : 0u;
        for (; fm; fm &= fm - 1) {
          const uint32_t l = (uint32_t)__ffsll((long long)fm) - 1;
          const uint32_t vv = (uint32_t)__builtin_amdgcn_readlane((int)R, (int)l);
          const uint32_t vr = (uint32_t)__builtin_amdgcn_readlane((int)rk, (int)l);
          if (crank > vr) {
            if (lane == 0) s_par[vv] = cr;
          } else if (crank < vr) {
            if (lane == 0) s_par[cr] = vv;
            cr = vv; crank = vr;
          } else {
            ++crank;
            if (lane == 0) { s_par[vv] = cr; s_rank[cr] = crank; }
          }
        }
      }
      // this chunk's stores complete before the next chunk's (or node's) loads
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
    }
  }
  (void)NONE;
  PROF_T(rb_t1);
  // slots 140..: [paths wave] ticks, [union wave] ticks, nodes, blocks
  PROF_ADD(paths ? 140 : 141, rb_t1 - rb_t0);
  if (paths) { PROF_ADD(142, n); PROF_ADD(143, 1); }
  __syncthreads();
  for (uint32_t i = tid; i < n; i += 128) {
    uint32_t q = i;
    while (s_par[q] != q) q = s_par[q];
    const RelaxPath si = S[i];
    const uint32_t fl = (si.fl & 1 ? 0u : GRAPH_START) | (si.fl & 2 ? 0u : GRAPH_END);
    G.out[b + i] = GraphNode{si.lp, si.lst == NONE ? -1 : (int32_t)si.lst, si.lpv == NONE ? -1 : (int32_t)si.lpv,
                             si.lun, q, fl};
  }
}
// ====================================================== mega-reads (device)
// The rest of create_mega_reads' per-read work after the traversal, on the
// device: overlap_graph::mega_reads_per_comp (overlap_graph.cc:116-161) with
// make / trim_match (:61-114), tile_greedy / tile_maximal (:163-252) and the
// path and numbers of every printed mega-read (print_mega_reads, :254-299); the
// host only formats them.  One wave per read: the candidates (end nodes passing
// the density and length filters) lane-parallel, the rest -- a handful of
// candidates a read -- by lane 0, in the reference's order, with per-read
// scratch regions in HBM.  std::min / std::max are restated as their
// definitions (b < a ? b : a, a < b ? b : a).
DEV double std_min(double a, double b) { return b < a ? b : a; }
DEV uint32_t rl_u32(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }
DEV double rl_f64(double v, uint32_t l) {  // lane l's value, l wave-uniform
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return __longlong_as_double((long long)(((uint64_t)rl_u32((uint32_t)(u >> 32), l) << 32) | rl_u32((uint32_t)u, l)));
}
DEV uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DEV double std_max(double a, double b) { return a < b ? b : a; }
DEV int32_t graph_ulen(const GraphDev& G, uint32_t id) { return id < G.n_ul ? G.ul[id] : 0; }  // ReadGraph::ulen
constexpr uint32_t UNIT_INVALID = 0x7fffffffu;  // super_read_name::invalid_id
__global__ __launch_bounds__(64) void k_mega(GraphDev G, uint32_t n_reads) {
  const uint32_t r = blockIdx.x;
  if (r >= n_reads) return;
  const uint32_t lane = threadIdx.x;
  const uint64_t b = G.rec_off[r];
  const uint32_t n = (uint32_t)(G.rec_off[r + 1] - b);
  if (n == 0) {
    if (lane == 0) { G.mcount[r] = 0; G.mhost[r] = 0; }
    return;
  }
  if (G.out[b].flags & GRAPH_HOST) {
    if (lane == 0) { G.mcount[r] = 0; G.mhost[r] = 1; atomicAdd(G.n_host, 1u); }
    return;
  }
  const uint32_t k = G.k;
  const double rl = (double)(G.roff[r + 1] - G.roff[r]);
  MegaTmp* cand = G.cand + b;
  PROF_T(km0);
  // ---- candidates, in node order (mega_reads_per_comp's loop body up to the filter)
  uint32_t nc = 0;
  for (uint32_t i0 = 0; i0 < n; i0 += 64) {
    const uint32_t i = i0 + lane;
    bool keep = false;
    MegaTmp m{};
    if (i < n) {
      const GraphNode g = G.out[b + i];
      const uint32_t sn = g.lstart == -1 ? i : (uint32_t)g.lstart;
      const Rec& Rs = G.recs[b + sn];
      const Rec& Re = G.recs[b + i];
      m.start_node = (int32_t)sn; m.end_node = (int32_t)i; m.start_unitig = 0;
      m.nb_unitigs = g.lunitigs; m.end_unitig = (int32_t)(Re.n_info / 2);
      m.imp_s = __dadd_rn(Rs.stretch, Rs.offset);
      m.imp_e = __dadd_rn(__dmul_rn(Re.stretch, (double)Re.ql), Re.offset);
      m.tiling_start = (double)Rs.rs; m.tiling_end = (double)Re.re;
      m.start_offset = 0; m.end_offset = 0; m.lpath = g.lpath; m.root = g.root;
      if (G.trim) {  // overlap_graph::trim_match (overlap_graph.cc:78-114)
        if (G.imp[b + sn].x < 1) {
          const uint32_t nsz = graph_nsz(G, Rs.sr);
          const uint32_t* un = G.ounits + G.poff[b + sn];
          int32_t offset = 0, su;
          for (su = 0; su < (int32_t)Rs.n_info; su += 2) {
            if (G.info_m[Rs.info_off + (uint32_t)su]) break;
            const int32_t u = su / 2;
            offset += graph_ulen(G, u < (int32_t)nsz ? un[u] >> 1 : UNIT_INVALID);
          }
          su /= 2;
          m.start_unitig = su;
          m.nb_unitigs -= su;
          offset = (int32_t)((uint32_t)offset - (k - 1) * (uint32_t)su);
          m.start_offset = offset;
          m.imp_s = __dadd_rn(__dmul_rn(Rs.stretch, (double)(offset + 1)), Rs.offset);
        }
        if (G.imp[b + i].y > (double)Re.ql) {
          const uint32_t nsz = graph_nsz(G, Re.sr);
          const uint32_t* un = G.ounits + G.poff[b + i];
          int32_t offset = 0, eu;
          for (eu = (int32_t)Re.n_info - 1; eu >= 0; eu -= 2) {
            if (G.info_m[Re.info_off + (uint32_t)eu]) break;
            const int32_t u = eu / 2;
            offset += graph_ulen(G, u < (int32_t)nsz ? un[u] >> 1 : UNIT_INVALID);
          }
          eu /= 2;
          m.end_unitig = eu;
          const int32_t removed = (int32_t)(Re.n_info / 2) - eu;
          m.nb_unitigs -= removed;
          offset = (int32_t)((uint32_t)offset - (k - 1) * (uint32_t)removed);
          m.end_offset = offset;
          m.imp_e = __dadd_rn(__dmul_rn(Re.stretch, (double)((uint64_t)Re.ql - (uint64_t)(int64_t)offset)), Re.offset);
        }
      }
      const double imp_len = __dadd_rn(std_min(__dadd_rn(rl, 0.5), m.tiling_end), -std_max(0.5, m.tiling_start));
      m.density = __ddiv_rn((double)g.lpath, imp_len);
      keep = (g.flags & GRAPH_END) && !(m.density < G.min_density) &&
             !(__dadd_rn(m.tiling_end, -m.tiling_start) < G.min_len);
    }
    const uint64_t km = __ballot(keep);
    if (keep) cand[nc + (uint32_t)__builtin_popcountll(km & ((1ull << lane) - 1))] = m;
    nc += (uint32_t)__builtin_popcountll(km);
  }
  __threadfence_block();
  __syncthreads();
  PROF_T(km1);
  // ---- components (per union-find root, in root order, the best terminal node), the
  // tiling order and tile_greedy / weighted with every lane: each of the reference's
  // O(m^2) comparison loops as 64-wide register rows broadcast by readlane, the interval
  // sets in LDS.  A NaN density or weight makes the reference's comparison chains
  // order-dependent; such a read runs the serial lane-0 restatement instead.
  int32_t* comp = G.ord + b;           // candidate index per component, sorted by root
  int32_t* order = G.ord + G.n_recs + b;
  int32_t* tiled = G.ord + 2 * G.n_recs + b;
  auto M = [&](int32_t t) -> const MegaTmp& { return cand[comp[t]]; };  // mega_reads_[t]
  auto weight = [&](const MegaTmp& q) -> double {  // weights_[t] (tile_weighted)
    const int32_t span = G.recs[b + q.end_node].re - G.recs[b + q.start_node].rs + 1;
    return __dmul_rn(__dmul_rn(q.density, q.density), (double)span);
  };
  const double play = G.play;
  const double kplay = __dmul_rn((double)k, play);
  uint32_t m = 0, nt = 0;  // components, tiled_mr_
  auto stable_sort = [&](int32_t* a, uint32_t cnt, auto less) {  // insertion sort: stable
    for (uint32_t x = 1; x < cnt; ++x) {
      const int32_t v = a[x];
      uint32_t y = x;
      while (y > 0 && less(v, a[y - 1])) { a[y] = a[y - 1]; --y; }
      a[y] = v;
    }
  };
  bool odd = false;
  for (uint32_t c = lane; c < nc; c += 64) {
    const MegaTmp& q = cand[c];
    odd |= isnan(q.density) | ((G.tiling == PBGPU_TILING_WEIGHTED) && isnan(weight(q)));
  }
  const bool serial = __ballot(odd) != 0;
  if (!serial) {
    constexpr uint32_t RW = GRAPH_NMAX / 64 / 64;  // root words a lane: lane * RW ...
    static_assert(GRAPH_NMAX == 64 * 64 * RW, "whole root words a lane");
    __shared__ uint64_t s_roots[GRAPH_NMAX / 64];  // the winners' roots (node indices)
    __shared__ uint32_t s_rpre[GRAPH_NMAX / 64];
    // the root bitmap and its prefix counts: in LDS, or for a read of more than GRAPH_NMAX
    // records in its region of G.scratch (free after the relaxation)
    auto components = [&](auto* roots, auto* rpre, uint32_t rw, uint64_t* ra) {
    for (uint32_t t = 0; t < rw; ++t) roots[lane * rw + t] = 0;
    // A candidate wins its root if no candidate of the root has a larger (lpath, density)
    // and none before it an equal one: where the reference's fold (replace on strictly
    // better, in candidate order) ends.  Per root, three atomic passes in the read's
    // scratch (ra: lpath max, density key max, index min; a root is a node index < n):
    // the best lpath, then the best density among those, then the first candidate
    // among those.  (Round 4 compared every pair of candidates: O(nc^2) readlanes, the
    // whole k_mega time on C4r reads with thousands of candidates.)  No NaN density here
    // (those reads take the serial path), so the key order is the double order, and
    // graph_dkey maps -0 and +0 to one key, as == sees them.
    int32_t* lpmax = reinterpret_cast<int32_t*>(ra);
    uint32_t* imin = reinterpret_cast<uint32_t*>(ra) + n;
    unsigned long long* dmax = reinterpret_cast<unsigned long long*>(ra) + n;
    for (uint32_t c = lane; c < nc; c += 64) {
      const uint32_t rt = cand[c].root;
      lpmax[rt] = INT32_MIN; imin[rt] = 0xFFFFFFFFu; dmax[rt] = 0ull;
    }
    __threadfence_block();
    __syncthreads();
    for (uint32_t c = lane; c < nc; c += 64) atomicMax(&lpmax[cand[c].root], cand[c].lpath);
    __threadfence_block();
    __syncthreads();
    for (uint32_t c = lane; c < nc; c += 64) {
      const uint32_t rt = cand[c].root;
      if (cand[c].lpath == __hip_atomic_load(&lpmax[rt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMax(&dmax[rt], (unsigned long long)graph_dkey(cand[c].density));
    }
    __threadfence_block();
    __syncthreads();
    for (uint32_t c = lane; c < nc; c += 64) {
      const uint32_t rt = cand[c].root;
      if (cand[c].lpath == __hip_atomic_load(&lpmax[rt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &&
          (unsigned long long)graph_dkey(cand[c].density) ==
              __hip_atomic_load(&dmax[rt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMin(&imin[rt], c);
    }
    __threadfence_block();
    __syncthreads();
    for (uint32_t c = lane; c < nc; c += 64) {
      const uint32_t rt = cand[c].root;
      const bool win = __hip_atomic_load(&imin[rt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == c;
      if (win) __atomic_fetch_or(&roots[rt >> 6], 1ull << (rt & 63), __ATOMIC_RELAXED);
      tiled[c] = win ? 1 : 0;  // (scratch until the tiling)
    }
    __threadfence_block();
    __syncthreads();
    // a winner's component index = its root's rank among the winners' roots
    uint32_t pc = 0;
    for (uint32_t t = 0; t < rw; ++t) pc += (uint32_t)__builtin_popcountll(__atomic_load_n(&roots[lane * rw + t], __ATOMIC_RELAXED));
    uint32_t incl = pc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o, 64);
      if (lane >= (uint32_t)o) incl += v;
    }
    for (uint32_t t = 0, acc = incl - pc; t < rw; ++t) {
      rpre[lane * rw + t] = acc;
      acc += (uint32_t)__builtin_popcountll(__atomic_load_n(&roots[lane * rw + t], __ATOMIC_RELAXED));
    }
    m = (uint32_t)__shfl(incl, 63, 64);
    __threadfence_block();
    __syncthreads();
    for (uint32_t c = lane; c < nc; c += 64)
      if (tiled[c]) {
        const uint32_t rt = cand[c].root;
        comp[rpre[rt >> 6] + (uint32_t)__builtin_popcountll(__atomic_load_n(&roots[rt >> 6], __ATOMIC_RELAXED) &
                                                           ((1ull << (rt & 63)) - 1))] = (int32_t)c;
      }
    __threadfence_block();
    __syncthreads();
    };
    // the read's region of G.scratch, 6 words a record: [the root bitmap and its prefix
    // counts (reads past GRAPH_NMAX records)], then the per-root arrays (2 words a node)
    if (n > GRAPH_NMAX) {
      const uint32_t rwb = (n + 4095) / 4096;  // n <= GRAPH_NMAX_BIG: 64 * rwb words of each
      uint64_t* groots = G.scratch + 6 * b;
      components(groots, reinterpret_cast<uint32_t*>(groots + 64 * rwb), rwb, groots + 128 * rwb);
    } else {
      components((lds_u64*)s_roots, (lds_u32*)s_rpre, RW, G.scratch + 6 * b);
    }
    // the tiling order, the reference's stable insertion sorts as ranks: lpath
    // descending (greedy), weight descending (weighted), tiling_end ascending
    // (maximal); none keeps component order.  key: ascending, exact (negation).
    auto key = [&](uint32_t t) -> double {
      const MegaTmp& q = M((int32_t)t);
      return G.tiling == PBGPU_TILING_GREEDY ? -(double)q.lpath
             : G.tiling == PBGPU_TILING_WEIGHTED ? -weight(q) : q.tiling_end;
    };
    for (uint32_t t0 = 0; t0 < m; t0 += 64) {
      const uint32_t t = t0 + lane;
      const bool ok = t < m;
      uint32_t rank = t;
      if (G.tiling != PBGPU_TILING_NONE) {
        const double kt = ok ? key(t) : 0.0;
        rank = 0;
        for (uint32_t u0 = 0; u0 < m; u0 += 64) {
          const double ku = u0 + lane < m ? key(u0 + lane) : 0.0;
          const uint32_t cnt = m - u0 < 64 ? m - u0 : 64;
          for (uint32_t x = 0; x < cnt; ++x) {
            const double k2 = rl_f64(ku, x);
            rank += (uint32_t)((k2 < kt) | ((k2 == kt) & (u0 + x < t)));
          }
        }
      }
      if (ok) order[rank] = (int32_t)t;
    }
    __threadfence_block();
    __syncthreads();
    if (G.tiling == PBGPU_TILING_GREEDY || G.tiling == PBGPU_TILING_WEIGHTED) {
      // tile_greedy (overlap_graph.cc:163-197) in component order: the overlap and
      // containment tests over every lane, the joined right-open interval set kept
      // sorted with strict gaps, so an insert [lo, hi) merges exactly the intervals
      // [s0, e) with s0 = #{y < lo}, e = #{x <= hi}
      constexpr uint32_t GCAP = 256;  // (128 and 64, for more waves a CU, measured the same)
      __shared__ double2 s_cov[GCAP], s_pl[GCAP], s_tile[GCAP];
      __shared__ int32_t s_it[GCAP];
      const bool in_lds = m <= GCAP;
      double2* cov = in_lds ? s_cov : G.ivs + b;
      double2* placed = in_lds ? s_pl : G.ivs + G.n_recs + b;
      if (in_lds) {  // the components' [tiling_start, tiling_end) in tiling order
        for (uint32_t t = lane; t < m; t += 64) {
          const int32_t it = order[t];
          const MegaTmp& q = M(it);
          s_it[t] = it; s_tile[t] = make_double2(q.tiling_start, q.tiling_end);
        }
        __syncthreads();
      }
      uint32_t ncov = 0, npl = 0;
      for (uint32_t t = 0; t < m; ++t) {
        const int32_t it = in_lds ? s_it[t] : order[t];
        const double2 tl = in_lds ? s_tile[t] : make_double2(M(it).tiling_start, M(it).tiling_end);
        const double lo = tl.x, hi = tl.y;
        const double span = hi > lo ? __dadd_rn(hi, -lo) : 0.0;
        const double max_overlap = std_max(kplay, __dmul_rn(span, __dadd_rn(play, -0.9)));
        bool large = false;
        for (uint32_t c = lane; c < ncov; c += 64) {
          const double2 v = cov[c];
          const double a = std_max(lo, v.x), bb = std_min(hi, v.y);
          large |= a < bb && __dadd_rn(bb, -a) >= max_overlap;
        }
        if (__ballot(large)) continue;
        bool contains = false;
        for (uint32_t c = lane; c < npl; c += 64) {
          const double2 v = placed[c];
          contains |= !(lo < hi) || (v.x < v.y && v.x <= lo && hi <= v.y);
        }
        if (__ballot(contains)) continue;
        if (lo < hi) {  // IntervalSet::add
          uint32_t s0 = 0, e = 0;
          for (uint32_t c = lane; c < ncov; c += 64) {
            const double2 v = cov[c];
            s0 += v.y < lo; e += v.x <= hi;
          }
          s0 = wave_sum_u32(s0); e = wave_sum_u32(e);
          double l2 = lo, h2 = hi;
          if (e > s0) { l2 = std_min(lo, cov[s0].x); h2 = std_max(hi, cov[e - 1].y); }
          // cov[e, ncov) moves to s0 + 1: from the back when it moves right
          const uint32_t len = ncov - e, dst = s0 + 1;
          if (dst > e) {
            for (int32_t c0 = len ? (int32_t)((len - 1) & ~63u) : -64; c0 >= 0; c0 -= 64) {
              const uint32_t c = (uint32_t)c0 + lane;
              double2 v = make_double2(0.0, 0.0);
              if (c < len) v = cov[e + c];
              if (c < len) cov[dst + c] = v;
              __threadfence_block();
            }
          } else if (dst < e) {
            for (uint32_t c0 = 0; c0 < len; c0 += 64) {
              const uint32_t c = c0 + lane;
              double2 v = make_double2(0.0, 0.0);
              if (c < len) v = cov[e + c];
              if (c < len) cov[dst + c] = v;
              __threadfence_block();
            }
          }
          __threadfence_block();
          if (lane == 0) cov[s0] = make_double2(l2, h2);
          ncov = dst + len;
        }
        if (lane == 0) { placed[npl] = make_double2(lo, hi); tiled[nt] = it; }
        ++npl; ++nt;
        __threadfence_block();
        __syncthreads();
      }
    }
    if (G.tiling == PBGPU_TILING_MAXIMAL && lane == 0) {
      // tile_maximal (overlap_graph.cc:199-252): info {score, pos, node, previous, length}
      double* ipos = (double*)(G.ivs + b);               // pos
      int4* ilink = (int4*)(G.ivs + G.n_recs + b);     // {previous, length, score, node}
      uint32_t ni = 0;
      if (m) {
        ipos[0] = M(order[0]).tiling_end;
        ilink[0] = make_int4(-1, 1, M(order[0]).lpath, order[0]);
        ni = 1;
        for (uint32_t t = 1; t < m; ++t) {
          const MegaTmp& q = M(order[t]);
          const double lstart = q.tiling_start;
          const double key = std_min(__dadd_rn(lstart, kplay), q.tiling_end);
          uint32_t lo = 0, hi = ni;  // upper_bound: the first info with key < pos
          while (lo < hi) { const uint32_t mid = (lo + hi) / 2; if (key < ipos[mid]) hi = mid; else lo = mid + 1; }
          int32_t x = (int32_t)lo - 1;
          while (x >= 0 && M(ilink[x].w).tiling_start >= lstart) x = ilink[x].x;
          const int32_t nscore = (x >= 0 ? ilink[x].z : 0) + q.lpath;
          if (nscore > ilink[ni - 1].z) {
            ipos[ni] = q.tiling_end;
            ilink[ni] = make_int4(x, (x >= 0 ? ilink[x].y : 0) + 1, nscore, order[t]);
            ++ni;
          }
        }
        nt = (uint32_t)ilink[ni - 1].y;
        int32_t ptr = (int32_t)ni - 1;
        for (int32_t q = (int32_t)nt - 1; q >= 0; --q) { tiled[q] = ilink[ptr].w; ptr = ilink[ptr].x; }
      }
    }
  } else if (lane == 0) {
    for (uint32_t c = 0; c < nc; ++c) {
      const uint32_t root = cand[c].root;
      uint32_t lo = 0, hi = m;  // lower_bound by root
      while (lo < hi) { const uint32_t mid = (lo + hi) / 2; if (cand[comp[mid]].root < root) lo = mid + 1; else hi = mid; }
      if (lo == m || cand[comp[lo]].root != root) {
        for (uint32_t q = m; q > lo; --q) comp[q] = comp[q - 1];
        comp[lo] = (int32_t)c; ++m;
      } else {
        const MegaTmp& cur = cand[comp[lo]];
        if (cand[c].lpath > cur.lpath || (cand[c].lpath == cur.lpath && cand[c].density > cur.density)) comp[lo] = (int32_t)c;
      }
    }
    for (uint32_t t = 0; t < m; ++t) order[t] = (int32_t)t;
    if (G.tiling == PBGPU_TILING_GREEDY || G.tiling == PBGPU_TILING_WEIGHTED) {
      if (G.tiling == PBGPU_TILING_GREEDY) {
        stable_sort(order, m, [&](int32_t x, int32_t y) { return M(y).lpath < M(x).lpath; });
      } else {
        double* w = (double*)(G.ivs + b);  // weights_[t]
        for (uint32_t t = 0; t < m; ++t) {
          const MegaTmp& q = M((int32_t)t);
          const int32_t span = G.recs[b + q.end_node].re - G.recs[b + q.start_node].rs + 1;
          w[t] = __dmul_rn(__dmul_rn(q.density, q.density), (double)span);
        }
        stable_sort(order, m, [&](int32_t x, int32_t y) { return w[y] < w[x]; });
      }
      // tile_greedy (overlap_graph.cc:163-197): covered = joined right-open intervals
      double2* cov = G.ivs + b;                 // (weights are read before this)
      double2* placed = G.ivs + G.n_recs + b;
      uint32_t ncov = 0, npl = 0;
      for (uint32_t t = 0; t < m; ++t) {
        const int32_t it = order[t];
        const MegaTmp& q = M(it);
        const double lo = q.tiling_start, hi = q.tiling_end;
        const double span = hi > lo ? __dadd_rn(hi, -lo) : 0.0;
        const double max_overlap = std_max(kplay, __dmul_rn(span, __dadd_rn(play, -0.9)));
        bool large = false;
        for (uint32_t c = 0; c < ncov && !large; ++c) {
          const double a = std_max(lo, cov[c].x), bb = std_min(hi, cov[c].y);
          large = a < bb && __dadd_rn(bb, -a) >= max_overlap;
        }
        if (large) continue;
        bool contains = false;
        for (uint32_t c = 0; c < npl && !contains; ++c)
          contains = !(lo < hi) || (placed[c].x < placed[c].y && placed[c].x <= lo && hi <= placed[c].y);
        if (contains) continue;
        if (lo < hi) {  // IntervalSet::add
          uint32_t s0 = 0;
          while (s0 < ncov && cov[s0].y < lo) ++s0;
          uint32_t e = s0;
          double l2 = lo, h2 = hi;
          while (e < ncov && cov[e].x <= h2) { l2 = std_min(l2, cov[e].x); h2 = std_max(h2, cov[e].y); ++e; }
          const uint32_t rem = e - s0;  // replaced by one interval at s0
          if (rem == 0) {
            for (uint32_t q2 = ncov; q2 > s0; --q2) cov[q2] = cov[q2 - 1];
            ++ncov;
          } else {
            for (uint32_t q2 = s0 + 1; q2 + rem - 1 < ncov; ++q2) cov[q2] = cov[q2 + rem - 1];
            ncov -= rem - 1;
          }
          cov[s0] = make_double2(l2, h2);
        }
        placed[npl++] = make_double2(lo, hi);
        tiled[nt++] = it;
      }
    } else if (G.tiling == PBGPU_TILING_MAXIMAL) {
      stable_sort(order, m, [&](int32_t x, int32_t y) { return M(x).tiling_end < M(y).tiling_end; });
      // tile_maximal (overlap_graph.cc:199-252): info {score, pos, node, previous, length}
      double* ipos = (double*)(G.ivs + b);               // pos
      int4* ilink = (int4*)(G.ivs + G.n_recs + b);     // {previous, length, score, node}
      uint32_t ni = 0;
      if (m) {
        ipos[0] = M(order[0]).tiling_end;
        ilink[0] = make_int4(-1, 1, M(order[0]).lpath, order[0]);
        ni = 1;
        for (uint32_t t = 1; t < m; ++t) {
          const MegaTmp& q = M(order[t]);
          const double lstart = q.tiling_start;
          const double key = std_min(__dadd_rn(lstart, kplay), q.tiling_end);
          uint32_t lo = 0, hi = ni;  // upper_bound: the first info with key < pos
          while (lo < hi) { const uint32_t mid = (lo + hi) / 2; if (key < ipos[mid]) hi = mid; else lo = mid + 1; }
          int32_t x = (int32_t)lo - 1;
          while (x >= 0 && M(ilink[x].w).tiling_start >= lstart) x = ilink[x].x;
          const int32_t nscore = (x >= 0 ? ilink[x].z : 0) + q.lpath;
          if (nscore > ilink[ni - 1].z) {
            ipos[ni] = q.tiling_end;
            ilink[ni] = make_int4(x, (x >= 0 ? ilink[x].y : 0) + 1, nscore, order[t]);
            ++ni;
          }
        }
        nt = (uint32_t)ilink[ni - 1].y;
        int32_t ptr = (int32_t)ni - 1;
        for (int32_t q = (int32_t)nt - 1; q >= 0; --q) { tiled[q] = ilink[ptr].w; ptr = ilink[ptr].x; }
      }
    }
  }
  PROF_T(km2);
  __threadfence_block();
  __syncthreads();
  m = (uint32_t)__shfl((int)m, 0, 64);
  nt = (uint32_t)__shfl((int)nt, 0, 64);
  PROF_T(km3);
  // the tiled mega-reads in print order: the reference's stable sort by (imp_s, imp_e)
  // (overlap_graph.cc:254-260).  As ranks over every lane -- #{smaller} + #{equal, earlier}
  // -- written into `order`, which the tiling has consumed; lane 0's insertion sort took
  // ~nt^2 / 4 dependent HBM compares, tens of ms for a C4r read with hundreds of tiles.
  // A NaN key makes the comparison chain order-dependent: then the serial sort, as before.
  const int32_t* tiled_sorted = tiled;
  if (G.tiling != PBGPU_TILING_NONE && nt > 1) {
    bool nan_key = false;
    for (uint32_t t = lane; t < nt; t += 64) {
      const MegaTmp& q = M(tiled[t]);
      nan_key |= isnan(q.imp_s) | isnan(q.imp_e);
    }
    if (__ballot(nan_key)) {
      if (lane == 0)
        stable_sort(tiled, nt, [&](int32_t x, int32_t y) {
          return M(x).imp_s < M(y).imp_s || (M(x).imp_s == M(y).imp_s && M(x).imp_e < M(y).imp_e);
        });
    } else {
      for (uint32_t t0 = 0; t0 < nt; t0 += 64) {
        const uint32_t t = t0 + lane;
        const bool ok = t < nt;
        const int32_t it = ok ? tiled[t] : 0;
        const double ks = ok ? M(it).imp_s : 0.0, ke = ok ? M(it).imp_e : 0.0;
        uint32_t rank = 0;
        for (uint32_t u0 = 0; u0 < nt; u0 += 64) {
          const bool uk = u0 + lane < nt;
          const int32_t iu = uk ? tiled[u0 + lane] : 0;
          const double us = uk ? M(iu).imp_s : 0.0, ue = uk ? M(iu).imp_e : 0.0;
          const uint32_t cnt = nt - u0 < 64 ? nt - u0 : 64;
          for (uint32_t x = 0; x < cnt; ++x) {
            const double s2 = rl_f64(us, x), e2 = rl_f64(ue, x);
            rank += (uint32_t)((s2 < ks) | ((s2 == ks) & ((e2 < ke) | ((e2 == ke) & (u0 + x < t)))));
          }
        }
        if (ok) order[rank] = it;
      }
      tiled_sorted = order;
    }
  }
  __threadfence_block();
  __syncthreads();
  // ---- print_mega_reads: what each printed mega-read needs (overlap_graph.cc:254-299),
  // the wave walking each path together (lane-parallel copies and sums).  A node's
  // name size and unitigs come from its prefix-sum offsets (poff[q + 1] - poff[q] =
  // size + 1), so a path step waits on one load, and the next node's is issued first.
  PROF_T(km4);
  const int32_t* pr = nt ? tiled_sorted : order;
  const uint32_t npr = nt ? nt : m;  // print(tiled_mr_.empty() ? sort_tiling_ : tiled_mr_)
  uint32_t done = 0;
  bool host = false;
  for (uint32_t t = 0; t < npr; ++t) {
    const MegaTmp& q = M(pr[t]);
    const GraphNode ge = G.out[b + (uint32_t)q.end_node];
    const Rec& Re = G.recs[b + (uint32_t)q.end_node];
    const Rec& Rs = G.recs[b + (uint32_t)q.start_node];
    const uint64_t nu = ge.lunitigs > 0 ? (uint64_t)ge.lunitigs : 0ull;
    unsigned long long uo = 0;
    if (lane == 0) uo = atomicAdd(G.units_used, (unsigned long long)nu);
    uo = (unsigned long long)__shfl((long long)uo, 0, 64);
    if (uo + nu > G.units_cap) { host = true; break; }
    uint32_t* sr = G.munits + uo;
    for (uint64_t x = lane; x < nu; x += 64) sr[x] = 0;
    __threadfence_block();
    // super_read_name::prepend (super_read_name.cc:29-36) of node's name, whose unitigs
    // start at un and number sz
    auto prepend = [&](uint64_t offset, const uint32_t* un, uint64_t sz, uint64_t first, uint64_t last) -> uint64_t {
      if (first > last || first >= sz) return offset;
      const uint64_t to_copy = (last < sz - 1 ? last : sz - 1) - first + 1;
      if (to_copy > offset) return offset;
      const uint64_t no = offset - to_copy;
      for (uint64_t x = lane; x < to_copy; x += 64) sr[no + x] = un[first + x];
      return no;
    };
    const uint64_t pe0 = G.poff[b + (uint32_t)q.end_node], nsze = G.poff[b + (uint32_t)q.end_node + 1] - pe0 - 1;
    int32_t node_i = ge.lprev;
    int32_t prev_i = 0, lun_i = 0;  // node i's lprev, lunitigs
    if (node_i >= 0) { prev_i = G.out[b + (uint32_t)node_i].lprev; lun_i = G.out[b + (uint32_t)node_i].lunitigs; }
    uint64_t offset = prepend(nu, G.ounits + pe0, nsze, 0, nsze - 1);
    int32_t lun_j = ge.lunitigs;
    uint64_t nszj = nsze;
    while (node_i >= 0) {
      const uint64_t p0 = G.poff[b + (uint32_t)node_i], nszi = G.poff[b + (uint32_t)node_i + 1] - p0 - 1;
      const int32_t nxt = prev_i;
      int32_t prev_n = 0, lun_n = 0;
      if (nxt >= 0) { prev_n = G.out[b + (uint32_t)nxt].lprev; lun_n = G.out[b + (uint32_t)nxt].lunitigs; }
      const uint64_t overlap = (uint64_t)(int64_t)lun_i + nszj - (uint64_t)(int64_t)lun_j;
      offset = prepend(offset, G.ounits + p0, nszi, 0, nszi - 1 - overlap);
      lun_j = lun_i; nszj = nszi;
      node_i = nxt; prev_i = prev_n; lun_i = lun_n;
    }
    __threadfence_block();
    __syncthreads();
    uint32_t sl = 0;  // sr_len: the unitig lengths summed modulo 2^32, as the int32 sum
    for (int64_t x = (int64_t)q.start_unitig + lane; x < (int64_t)q.start_unitig + q.nb_unitigs; x += 64)
      sl += (uint32_t)graph_ulen(G, x >= 0 && (uint64_t)x < nu ? sr[x] >> 1 : UNIT_INVALID);
    sl = wave_sum_u32(sl);
    const int32_t sr_len = (int32_t)(sl - (uint32_t)(q.nb_unitigs - 1) * (k - 1));
    if (lane == 0) {
      MegaOut o;
      o.imp_s = q.imp_s; o.imp_e = q.imp_e; o.density = q.density;
      o.rs = Rs.rs; o.re = Re.re; o.qs = Rs.qs - q.start_offset; o.lpath = ge.lpath;
      o.sr_len = sr_len; o.start_unitig = q.start_unitig; o.nb_unitigs = q.nb_unitigs; o.n_units = (uint32_t)nu;
      o.qend = (uint64_t)(int64_t)(sr_len + q.end_offset) - ((uint64_t)Re.ql - (uint64_t)(int64_t)Re.qe);
      o.unit_offset = uo;
      G.mo[b + done] = o;
    }
    ++done;
  }
  if (lane != 0) return;
  G.mcount[r] = host ? 0u : done;
  G.mhost[r] = host ? 1 : 0;
  if (host) atomicAdd(G.n_host, 1u);
#ifdef PBGPU_PROF
  {  // slots 88..: candidates, components, sort + tiling, final sort, paths, waves, max wave, candidates / comps
    PROF_T(km5);
    atomicAdd(&g_prof[88], km1 - km0); atomicAdd(&g_prof[89], km2 - km1); atomicAdd(&g_prof[90], km3 - km2);
    atomicAdd(&g_prof[91], km4 - km3); atomicAdd(&g_prof[92], km5 - km4); atomicAdd(&g_prof[93], 1ull);
    atomicMax(&g_prof[94], km5 - km0); atomicAdd(&g_prof[95], ((unsigned long long)nc << 32) | m);
  }
#endif
}
__global__ void k_mega_pack(GraphDev G, uint32_t n_reads, const uint64_t* __restrict__ moff, MegaOut* __restrict__ mc) {
  const uint32_t r = blockIdx.x;
  if (r >= n_reads) return;
  const uint64_t b = G.rec_off[r], o = moff[r];
  const uint32_t c = G.mcount[r];
  for (uint32_t t = threadIdx.x; t < c; t += blockDim.x) mc[o + t] = G.mo[b + t];
}
// sizes for the host's share: per read its record count if left to the host (rsize),
// per record its info length if its read is (isize)
__global__ void k_host_sizes(GraphDev G, uint32_t n_reads, uint32_t* __restrict__ rsize, uint32_t* __restrict__ isize) {
  const uint32_t r = blockIdx.x;
  if (r >= n_reads) return;
  const uint64_t b = G.rec_off[r];
  const uint32_t n = (uint32_t)(G.rec_off[r + 1] - b);
  const bool h = G.mhost[r] != 0;
  if (threadIdx.x == 0) rsize[r] = h ? n : 0u;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) isize[b + i] = h ? G.recs[b + i].n_info : 0u;
}
__global__ void k_host_pack(GraphDev G, uint32_t n_reads, const uint64_t* __restrict__ hroff,
                            const uint64_t* __restrict__ hioff, Rec* __restrict__ hrec, GraphNode* __restrict__ hgraph,
                            int32_t* __restrict__ hinfo_m, int32_t* __restrict__ hinfo_b) {
  const uint32_t r = blockIdx.x;
  if (r >= n_reads || !G.mhost[r]) return;
  const uint64_t b = G.rec_off[r];
  const uint32_t n = (uint32_t)(G.rec_off[r + 1] - b);
  const uint64_t o = hroff[r];
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    Rec R = G.recs[b + i];
    const uint64_t io = hioff[b + i];
    for (uint32_t x = 0; x < R.n_info; ++x) { hinfo_m[io + x] = G.info_m[R.info_off + x]; hinfo_b[io + x] = G.info_b[R.info_off + x]; }
    R.info_off = io;
    hrec[o + i] = R;
    hgraph[o + i] = G.out[b + i];
  }
}
void launch_host_sizes(const GraphDev& G, uint32_t n_reads, uint32_t* rsize, uint32_t* isize, hipStream_t st) {
  if (n_reads) hipLaunchKernelGGL(k_host_sizes, dim3(n_reads), dim3(64), 0, st, G, n_reads, rsize, isize);
}
void launch_host_pack(const GraphDev& G, uint32_t n_reads, const uint64_t* hroff, const uint64_t* hioff, Rec* hrec,
                      GraphNode* hgraph, int32_t* hinfo_m, int32_t* hinfo_b, hipStream_t st) {
  if (n_reads)
    hipLaunchKernelGGL(k_host_pack, dim3(n_reads), dim3(64), 0, st, G, n_reads, hroff, hioff, hrec, hgraph, hinfo_m, hinfo_b);
}
void launch_mega(const GraphDev& G, uint32_t n_reads, hipStream_t st) {
  if (!n_reads) return;
  hipLaunchKernelGGL(k_mega, dim3(n_reads), dim3(64), 0, st, G, n_reads);
}
void launch_mega_pack(const GraphDev& G, uint32_t n_reads, const uint64_t* moff, MegaOut* mc, hipStream_t st) {
  if (!n_reads) return;
  hipLaunchKernelGGL(k_mega_pack, dim3(n_reads), dim3(64), 0, st, G, n_reads, moff, mc);
}
void launch_graph_sizes(const GraphDev& G, uint32_t n_reads, uint64_t n_recs, uint32_t* sizes, uint64_t* scan_scratch,
                        hipStream_t st) {
  if (n_reads)
    hipLaunchKernelGGL(k_graph_max_n, dim3(std::min<uint32_t>((n_reads + 255) / 256, 1024)), dim3(256), 0, st, G, n_reads);
  if (n_recs) hipLaunchKernelGGL(k_graph_sizes, dim3((uint32_t)std::min<uint64_t>((n_recs + 255) / 256, 65535)), dim3(256),
                                 0, st, G, n_recs, sizes);
  launch_excl_scan(sizes, nullptr, n_recs, G.poff, scan_scratch, st);
}
hipError_t launch_graph(const GraphDev& G, uint32_t n_reads, uint64_t n_recs, uint32_t max_n, hipStream_t st,
                        hipStream_t side, hipEvent_t fork, hipEvent_t join, uint64_t* ovf) {
  ovf[0] = ovf[1] = 0;
  if (!n_recs || !n_reads) return hipSuccess;
  hipError_t e = hipMemsetAsync(G.ovf, 0, 16, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_graph_prep, dim3((uint32_t)std::min<uint64_t>((n_recs + 255) / 256, 65535)), dim3(256), 0, st,
                     G, n_recs);
  // the per-read sorts: the long reads' tiers on the side stream, beside the short one.  A
  // failed fork or join would let a kernel read what the other stream still writes, so
  // each is checked (the caller raises)
  if ((e = hipEventRecord(fork, st)) == hipSuccess) e = hipStreamWaitEvent(side, fork, 0);
  if (e != hipSuccess) return e;
  // (a tier above the batch's longest read is not launched: an empty 8192-record block
  // still takes a CU's LDS while it starts and exits, 1.4 ms a launch of 50k of them)
  if (max_n > GRAPH_NMAX)
    hipLaunchKernelGGL(k_graph_sort_big, dim3(n_reads), dim3(GRAPH_BIG_BLOCK), 0, side, G, n_reads);
  if (max_n > GRAPH_NM_MID)
    hipLaunchKernelGGL(k_graph_sort<GRAPH_NMAX>, dim3(n_reads), dim3(GRAPH_SORT_BLOCK), 0, side, G, n_reads);
  if (max_n > GRAPH_NM_SMALL)
    hipLaunchKernelGGL(k_graph_sort<GRAPH_NM_MID>, dim3(n_reads), dim3(GRAPH_SORT_BLOCK), 0, side, G, n_reads);
  if ((e = hipEventRecord(join, side)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_graph_sort<GRAPH_NM_SMALL>, dim3(n_reads), dim3(GRAPH_SORT_BLOCK), 0, st, G, n_reads);
  if ((e = hipStreamWaitEvent(st, join, 0)) != hipSuccess) return e;
  // the blocks' largest implied ends (the scans' fast-forward), then every node's edges (its
  // first GRAPH_EBLK) and the nodes with more
  hipLaunchKernelGGL(k_graph_bmax, dim3((uint32_t)((n_recs + 255) / 256)), dim3(256), 0, st, G, n_recs);
  const uint32_t eg = (uint32_t)((n_recs + GE_NODES - 1) / GE_NODES);
  hipLaunchKernelGGL(k_graph_edges<false>, dim3(eg), dim3(GE_BLOCK), 0, st, G, n_recs, 0ull);
  if ((e = hipMemcpyAsync(ovf, G.ovf, 16, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
  return hipStreamSynchronize(st);
}
hipError_t launch_graph_relax(const GraphDev& G, uint32_t n_reads, uint64_t n_recs, uint32_t max_n, uint64_t n_ovf,
                              hipStream_t st, hipStream_t side, hipStream_t side2, hipEvent_t fork, hipEvent_t join,
                              hipEvent_t join2) {
  if (!n_recs || !n_reads) return hipSuccess;
  constexpr uint32_t W = GE_BLOCK / 64;
  if (n_ovf) hipLaunchKernelGGL(k_graph_edges<true>, dim3((uint32_t)((n_ovf + W - 1) / W)), dim3(GE_BLOCK), 0, st, G,
                                n_recs, n_ovf);
  // the long reads' relaxations on side streams (their blocks are the longest: > 4096
  // records then > 2048 on one, > 1024 on the other), beside the short reads' on st
  hipError_t e = hipEventRecord(fork, st);
  if (e == hipSuccess) e = hipStreamWaitEvent(side, fork, 0);
  if (e == hipSuccess) e = hipStreamWaitEvent(side2, fork, 0);
  if (e != hipSuccess) return e;
  // (tiers above the longest read are not launched; the top one also marks the reads
  // left to the host, so it runs whenever a read is past the device cap)
  if (max_n > G.relax_big_min && G.nmax > G.relax_big_min)
    hipLaunchKernelGGL(k_graph_relax_big, dim3(n_reads), dim3(128), 0, side, G, n_reads);
  // an LDS tier runs when it has reads: some read past NM / 2 records and not past
  // relax_big_min (an empty launch of a tier's blocks still costs ~1.4 ms per 50k reads)
  auto tier_has = [&](uint32_t nm) { return max_n > nm / 2 && G.relax_big_min > nm / 2; };
  if (tier_has(GRAPH_NMAX) || max_n > G.nmax)
    hipLaunchKernelGGL(k_graph_relax<GRAPH_NMAX>, dim3(n_reads), dim3(128), 0, side, G, n_reads);
  if (tier_has(GRAPH_NMAX / 2))
    hipLaunchKernelGGL(k_graph_relax<GRAPH_NMAX / 2>, dim3(n_reads), dim3(128), 0, side, G, n_reads);
  if (tier_has(GRAPH_NMAX / 4))
    hipLaunchKernelGGL(k_graph_relax<GRAPH_NMAX / 4>, dim3(n_reads), dim3(128), 0, side2, G, n_reads);
  if ((e = hipEventRecord(join, side)) != hipSuccess) return e;
  if ((e = hipEventRecord(join2, side2)) != hipSuccess) return e;
  if (tier_has(GRAPH_NM_SMALL))
    hipLaunchKernelGGL(k_graph_relax<GRAPH_NM_SMALL>, dim3(n_reads), dim3(128), 0, st, G, n_reads);
  hipLaunchKernelGGL(k_graph_relax<GRAPH_RELAX_MIN>, dim3(n_reads), dim3(128), 0, st, G, n_reads);
  if ((e = hipStreamWaitEvent(st, join, 0)) != hipSuccess) return e;
  return hipStreamWaitEvent(st, join2, 0);
}

}  // namespace pbgpu

#ifdef PBGPU_GRAPH_CHECK
// the check counters so far, printed to stderr by every aligner with a graph at its free
// (the CLIs run the variant through LD_LIBRARY_PATH and print nothing of their own)
namespace pbgpu {
void graph_check_report() {
  unsigned long long h[5] = {};
  const hipError_t e = hipMemcpyFromSymbol(h, HIP_SYMBOL(g_graph_check), sizeof(h));
  fprintf(stderr, "pbgpu graph-check: far_j %llu name_units %llu prefix_sums %llu edge_targets %llu checks %llu%s\n",
          h[0], h[1], h[2], h[3], h[4], e == hipSuccess ? "" : " (counters unreadable)");
}
}  // namespace pbgpu
#endif
