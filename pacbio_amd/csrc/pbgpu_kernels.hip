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
#include <stdint.h>
#include "pbgpu_internal.h"

namespace pbgpu {

#define DEV __device__ __forceinline__

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
  if (n1 == m) return true;
  uint64_t n2 = (n1 >> 2) | ((n1 & 3) << hs);
  return n2 == m;
}
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

// ============================================================ index build
__global__ void k_build_keys(IndexView ix, uint64_t N, uint64_t* keys, uint64_t* vals) {
  const uint32_t k = ix.k;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = N - 1 - i;  // descending positions => stable sort keeps x desc
    const uint64_t f = text_kmer(ix.text, x, k);
    const uint64_t r = revcomp(f, k);
    const uint64_t canon = f < r ? f : r;
    const uint64_t obit = f > r ? 1 : 0;
    // SR holding x: upper_bound(sr_start, x) - 1 (pos_iterator, superread_parser.hpp:110-140)
    uint32_t lo = 0, hi = ix.n_sr + 1;
    while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (ix.sr_start[m] <= x) lo = m + 1; else hi = m; }
    const uint32_t s = lo - 1;
    const bool cross = x + k > ix.sr_start[s + 1];
    keys[i] = (canon << 1) | obit;
    vals[i] = cross ? ~0ull : (((uint64_t)s << 32) | (uint32_t)(x - ix.sr_start[s] + 1));
  }
}

__global__ void k_runs(const uint64_t* keys, const uint64_t* uidx, uint64_t N, uint64_t* run_start) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const bool head = i == 0 || (keys[i] >> 1) != (keys[i - 1] >> 1);
    if (head) run_start[uidx[i] - 1] = i;
  }
}

__global__ void k_occ_fill(const uint64_t* vals, const uint64_t* uidx, const uint64_t* kpos, uint64_t N, uint64_t* occ) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t v = vals[i];
    if (v != ~0ull) occ[2 * uidx[i] + kpos[i]] = v;
  }
}

__global__ void k_headers(const uint64_t* keys, const uint64_t* kpos, const uint64_t* run_start, uint64_t U,
                          uint64_t* occ, ulonglong2* table, uint64_t bucket_mask, uint32_t k) {
  for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < U; u += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s = run_start[u], e = run_start[u + 1];
    const uint64_t canon = keys[s] >> 1;
    const bool pal = canon == revcomp(canon, k);
    uint64_t lo = s, hi = e;  // first index with orientation bit set
    while (lo < hi) { uint64_t m = (lo + hi) >> 1; if (keys[m] & 1) hi = m; else lo = m + 1; }
    const uint64_t nA = kpos[lo] - kpos[s], nB = kpos[e] - kpos[lo];
    const uint64_t hb = 2 * u + kpos[s];
    const uint64_t count = (e - s) * (pal ? 2 : 1);
    const uint64_t cnt32 = count > 0xFFFFFFFFull ? 0xFFFFFFFFull : count;
    occ[hb] = cnt32 | ((uint64_t)pal << 32);
    occ[hb + 1] = nA | (nB << 32);
    const uint64_t payload = (hb << 24) | (count < SAT_COUNT ? count : SAT_COUNT);
    uint64_t b = fmix64(canon) & bucket_mask;
    for (;;) {
      bool done = false;
      for (int sl = 0; sl < 4; ++sl) {
        unsigned long long* kp = (unsigned long long*)&table[4 * b + sl].x;
        unsigned long long old = atomicCAS(kp, (unsigned long long)EMPTY_KEY, (unsigned long long)canon);
        if (old == EMPTY_KEY) { table[4 * b + sl].y = payload; done = true; break; }
      }
      if (done) break;
      b = (b + 1) & bucket_mask;
    }
  }
}

// ================================================================== seed
// One workgroup per read.  fetch_super_reads (coarse_aligner.cc:81-125).
template <int BLOCK, int PER>
__global__ __launch_bounds__(BLOCK) void k_seed(IndexView ix, const uint8_t* __restrict__ seq,
                                                const uint64_t* __restrict__ roff, uint32_t n_reads,
                                                AlignParamsDev P, KRec* __restrict__ krec,
                                                uint32_t* __restrict__ n_kept_out, uint32_t* __restrict__ thr_out,
                                                uint64_t* __restrict__ nhits_out, unsigned long long* stats) {
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
  uint64_t my_kmers = 0, my_probes = 0;

  for (int64_t t0 = 0; t0 < L; t0 += TILE) {
    for (int i = tid; i < TILE + LOOK; i += BLOCK) {
      const int64_t p = t0 - LOOK + i;
      s_seq[i] = (p >= 0 && p < L) ? seq[base + p] : (uint8_t)'N';
    }
    __syncthreads();
    const int64_t p0 = t0 + (int64_t)tid * PER;
    const int64_t s = p0 - LOOK > 0 ? p0 - LOOK : 0;
    uint64_t m = 0, rm = 0;
    uint32_t rl = s > 0 ? 1000u : 0u;  // unknown history before s counts as a long valid run
    for (int64_t q = s; q < p0; ++q) {
      const int c = base_code(s_seq[q - t0 + LOOK]);
      if (c < 0) { rl = 0; continue; }
      ++rl;
      m = ((m << 2) | (uint64_t)c) & mask;
      rm = (rm >> 2) | ((uint64_t)(3 - c) << hs);
    }
    uint64_t mm[PER], rr[PER];
    uint32_t fl[PER];  // bit0 valid&!ssr (candidate for lookup), bit1 toggle candidate
    uint32_t ncand = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int64_t p = p0 + q;
      fl[q] = 0;
      mm[q] = 0; rr[q] = 0;
      if (p < L) {
        const int c = base_code(s_seq[p - t0 + LOOK]);
        if (c < 0) rl = 0;
        else {
          ++rl;
          m = ((m << 2) | (uint64_t)c) & mask;
          rm = (rm >> 2) | ((uint64_t)(3 - c) << hs);
          if (rl >= k) {
            ++my_kmers;
            if (!is_ssr(m, k)) {
              fl[q] = 1;
              if (rl <= 17) { fl[q] |= 2; ++ncand; }  // coarse_aligner.cc:96-102
            }
            mm[q] = m; rr[q] = rm;
          }
        }
      }
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
        uint64_t payload; uint32_t pr = 0;
        const bool found = table_lookup(ix, canon, payload, pr);
        my_probes += pr;
        if (found) {
          uint32_t cnt = (uint32_t)(payload & SAT_COUNT);
          const uint64_t ptr = payload >> 24;
          if (cnt == SAT_COUNT) cnt = (uint32_t)(ix.occ[ptr] & 0xFFFFFFFFull);
          if (cnt < (uint32_t)P.max_count) {  // count >= 1 here
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
      if (tid == 0) {
        uint32_t cum = 0, d = 0;
        for (; d < 256; ++d) { if (cum + s_hist[d] > rank) break; cum += s_hist[d]; }
        s_sel[0] = d; s_sel[1] = rank - cum;
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
  if (tid == 0) {
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
// One workgroup per read: enumerate hits (pos_iterator order), group them by
// super-read in an open-addressing table (LDS, or a global region for reads
// with too many super-reads), emit one ChainDesc per (read, SR).

template <int BLOCK, bool GLOBAL_TABLE>
__global__ __launch_bounds__(BLOCK) void k_group(IndexView ix, const KRec* __restrict__ krec,
                                                 const uint64_t* __restrict__ roff, const uint32_t* __restrict__ n_kept,
                                                 const uint32_t* __restrict__ thr_in, const uint64_t* __restrict__ hit_off,
                                                 const uint32_t* __restrict__ read_list, uint32_t n_list,
                                                 uint32_t hcap_log2, uint32_t* gtable, GroupOut O,
                                                 unsigned long long* stats) {
  extern __shared__ uint32_t s_dyn[];
  __shared__ uint32_t s_nf[BLOCK], s_nb[BLOCK], s_off[BLOCK + 1];
  __shared__ int32_t s_pb[BLOCK];
  __shared__ uint64_t s_pf[BLOCK], s_pbk[BLOCK];
  __shared__ uint32_t s_tmp[BLOCK / 64];
  __shared__ uint32_t s_flag[8];
  if (blockIdx.x >= n_list) return;
  const uint32_t r = read_list ? read_list[blockIdx.x] : blockIdx.x;
  const int tid = threadIdx.x;
  const uint32_t hcap = 1u << hcap_log2;
  uint32_t* tkey = GLOBAL_TABLE ? gtable + (uint64_t)blockIdx.x * 4 * hcap : s_dyn;
  uint32_t* tcf = tkey + hcap;
  uint32_t* tcb = tcf + hcap;
  uint32_t* tbase = tcb + hcap;
  for (uint32_t i = tid; i < hcap; i += BLOCK) { tkey[i] = 0; tcf[i] = 0; tcb[i] = 0; }
  if (tid < 8) s_flag[tid] = 0;
  __syncthreads();
  const uint64_t kbase = roff[r];
  const uint32_t nk = n_kept[r], thr = thr_in[r];
  const uint64_t hbase = hit_off[r];

  for (int pass = 0; pass < 2; ++pass) {
    for (uint32_t c0 = 0; c0 < nk; c0 += BLOCK) {
      const uint32_t i = c0 + tid;
      uint32_t nf = 0, nb = 0;
      if (i < nk) {
        const KRec kr = krec[kbase + i];
        if (kr.count <= thr) {
          const uint64_t ptr = kr.occ_ptr & ~(1ull << 63);
          const bool canon = kr.occ_ptr >> 63;
          const uint64_t h0 = ix.occ[ptr], h1 = ix.occ[ptr + 1];
          const uint32_t nA = (uint32_t)(h1 & 0xFFFFFFFFull), nB = (uint32_t)(h1 >> 32);
          const uint64_t A = ptr + 2, B = ptr + 2 + nA;
          // occ(m) -> fwd list (+off), occ(rm) -> bwd list (-off)   (A.3)
          if ((h0 >> 32) & 1) { nf = nb = nA; s_pf[tid] = A; s_pbk[tid] = A; }
          else if (canon) { nf = nA; s_pf[tid] = A; nb = nB; s_pbk[tid] = B; }
          else { nf = nB; s_pf[tid] = B; nb = nA; s_pbk[tid] = A; }
          s_pb[tid] = kr.pb_off;
        }
      }
      s_nf[tid] = nf; s_nb[tid] = nb;
      uint32_t total;
      const uint32_t off = block_excl_scan<BLOCK>(nf + nb, s_tmp, total);
      s_off[tid] = off;
      if (tid == 0) s_off[BLOCK] = total;
      __syncthreads();
      for (uint32_t h = tid; h < total; h += BLOCK) {
        uint32_t lo = 0, hi = BLOCK;  // last ri with s_off[ri] <= h
        while (hi - lo > 1) { uint32_t md = (lo + hi) >> 1; if (s_off[md] <= h) lo = md; else hi = md; }
        const uint32_t ri = lo;
        const uint32_t local = h - s_off[ri];
        const bool fwd = local < s_nf[ri];
        const uint64_t e = ix.occ[fwd ? s_pf[ri] + local : s_pbk[ri] + (local - s_nf[ri])];
        const uint32_t sr = (uint32_t)(e >> 32);
        const int32_t so = (int32_t)(uint32_t)(e & 0xFFFFFFFFull);
        uint32_t slot = (sr * 0x9E3779B1u) >> (32 - hcap_log2);
        if (pass == 0) {
          uint32_t probe = 0;
          for (;;) {
            const uint32_t old = atomicCAS(&tkey[slot], 0u, sr + 1);
            if (old == 0 || old == sr + 1) break;
            slot = (slot + 1) & (hcap - 1);
            if (++probe >= hcap) { s_flag[0] = 1; slot = ~0u; break; }
          }
          if (slot != ~0u) atomicAdd(fwd ? &tcf[slot] : &tcb[slot], 1u);
        } else {
          while (tkey[slot] != sr + 1) slot = (slot + 1) & (hcap - 1);
          const uint32_t pos = atomicAdd(fwd ? &tcf[slot] : &tcb[slot], 1u);
          O.hits[hbase + pos] = make_int2(s_pb[ri], fwd ? so : -so);
        }
      }
      __syncthreads();
    }
    if (pass == 0) {
      if (s_flag[0]) {  // too many super-reads for the table: retry this read with a global table
        if (tid == 0) { uint32_t o = atomicAdd(O.n_overflow, 1u); O.overflow_reads[o] = r; }
        return;
      }
      // chain bases: scan (cf+cb) over the slots; classify; reserve descriptors
      const uint32_t per = hcap / BLOCK;  // hcap >= BLOCK
      uint32_t sum = 0, nsm = 0, nlg = 0, nhg = 0;
      uint64_t hg_elems = 0;
      for (uint32_t j = 0; j < per; ++j) {
        const uint32_t sl = tid * per + j;
        if (tkey[sl]) {
          const uint32_t cf = tcf[sl], cb = tcb[sl], mx = cf > cb ? cf : cb;
          sum += cf + cb;
          if (mx <= O.cap_small) ++nsm; else if (mx <= O.cap_large) ++nlg; else { ++nhg; hg_elems += cf + cb; }
        }
      }
      uint32_t tsum, tsm, tlg, thg;
      uint32_t b0 = block_excl_scan<BLOCK>(sum, s_tmp, tsum);
      uint32_t i_sm = block_excl_scan<BLOCK>(nsm, s_tmp, tsm);
      uint32_t i_lg = block_excl_scan<BLOCK>(nlg, s_tmp, tlg);
      uint32_t i_hg = block_excl_scan<BLOCK>(nhg, s_tmp, thg);
      uint32_t hg_e32 = (uint32_t)hg_elems, thg_e;
      uint32_t e_hg = block_excl_scan<BLOCK>(hg_e32, s_tmp, thg_e);
      if (tid == 0) {
        s_flag[1] = tsm ? atomicAdd(&O.chain_count[0], tsm) : 0;
        s_flag[2] = tlg ? atomicAdd(&O.chain_count[1], tlg) : 0;
        s_flag[3] = thg ? atomicAdd(&O.chain_count[2], thg) : 0;
        unsigned long long hb = thg_e ? atomicAdd((unsigned long long*)O.huge_elems, (unsigned long long)thg_e) : 0ull;
        s_flag[4] = (uint32_t)hb; s_flag[5] = (uint32_t)(hb >> 32);
        atomicAdd(&stats[ST_CHAINS], (unsigned long long)(tsm + tlg + thg));
      }
      __syncthreads();
      const uint64_t hgb = (uint64_t)s_flag[4] | ((uint64_t)s_flag[5] << 32);
      i_sm += s_flag[1]; i_lg += s_flag[2]; i_hg += s_flag[3];
      uint64_t e_cur = hgb + e_hg;
      for (uint32_t j = 0; j < per; ++j) {
        const uint32_t sl = tid * per + j;
        if (!tkey[sl]) continue;
        const uint32_t cf = tcf[sl], cb = tcb[sl], mx = cf > cb ? cf : cb;
        ChainDesc d;
        d.read = r; d.sr = tkey[sl] - 1; d.nf = cf; d.nb = cb; d.hit_base = hbase + b0; d.scratch = 0;
        if (mx <= O.cap_small) { if (i_sm < O.chain_cap[0]) O.chains[0][i_sm] = d; ++i_sm; }
        else if (mx <= O.cap_large) { if (i_lg < O.chain_cap[1]) O.chains[1][i_lg] = d; ++i_lg; }
        else { d.scratch = e_cur; e_cur += cf + cb; if (i_hg < O.chain_cap[2]) O.chains[2][i_hg] = d; ++i_hg; }
        tcf[sl] = b0;        // fwd cursor
        tcb[sl] = b0 + cf;   // bwd cursor
        b0 += cf + cb;
      }
      __syncthreads();
    }
  }
}

// ================================================================= chain
// lis_align::compute_L_P (lis_align.hpp:139-182) for one wave.
// The forward_list L is kept as an array in REVERSED list order (head at
// the end) so that the common "extend the head" insertion is an append.
// Node fields (SoA): j (element index), len, root (first element of its
// chain: span_full == X[i] - X[root] exactly, all values are small ints).

template <typename IDX>
struct ListStore {
  IDX* j; IDX* len; IDX* root; IDX* P;
};

DEV bool affine_ok(double a, double b, double C, double df, double ds) {
  // (s.first <= b + a*s.second) && (s.second <= b + a*s.first) && s.first <= C && s.second <= C
  return (df <= __dadd_rn(b, __dmul_rn(a, ds))) && (ds <= __dadd_rn(b, __dmul_rn(a, df))) && df <= C && ds <= C;
}
DEV bool linear_ok(double a, double df, double ds) {
  return (df <= __dmul_rn(a, ds)) && (ds <= __dmul_rn(a, df));
}

// returns LIS length; writes ascending indices to out[0..len)
template <typename IDX>
DEV uint32_t wave_lis(const int2* X, uint32_t n, ListStore<IDX> S, IDX* out, const LisParams& lp,
                      uint64_t& tests) {
  const int lane = lane_id();
  uint32_t L = 0, longest = 0, longest_ind = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const int2 xi = X[i];
    int found = -1;
    uint32_t best_len = 0xFFFFFFFFu;
    int best_t = -1;
    for (uint32_t t0 = 0; t0 < L; t0 += 64) {
      const uint32_t t = t0 + lane;
      const bool valid = t < L;
      uint32_t nl = 0xFFFFFFFFu;
      bool cond = false;
      if (valid) {
        const uint32_t idx = L - 1 - t;
        nl = S.len[idx];
        const uint32_t j = S.j[idx];
        const int2 xj = X[j];
        if (xi.y > xj.y) {
          if (lp.mer_all) cond = true;
          else if (lp.W == 1) cond = affine_ok(lp.a, lp.b, lp.C, (double)(xi.x - xj.x), (double)(xi.y - xj.y));
          else if (lp.W == 0 || nl < lp.W) cond = true;  // !will_be_filled()
          else {
            uint32_t anc = j;  // test_sum == X[i] - X[anc_{W-1}(j)]
            for (uint32_t w = 1; w < lp.W; ++w) anc = S.P[anc];
            const int2 xa = X[anc];
            cond = affine_ok(lp.a, lp.b, lp.C, (double)(xi.x - xa.x), (double)(xi.y - xa.y));
          }
        }
      }
      const uint64_t mk = __ballot(cond);
      const uint32_t lim = mk ? (uint32_t)(__ffsll((unsigned long long)mk) - 1) : 64u;
      tests += (uint64_t)(lim < 64 ? lim + 1 : (L - t0 < 64 ? L - t0 : 64));
      const uint64_t key = (valid && (uint32_t)lane < lim) ? (((uint64_t)nl << 32) | t) : ~0ull;
      const uint64_t mn = wave_min_u64(key);
      if (mn != ~0ull && (uint32_t)(mn >> 32) < best_len) { best_len = (uint32_t)(mn >> 32); best_t = (int)(uint32_t)mn; }
      if (mk) { found = (int)(t0 + lim); break; }
    }
    uint32_t e_len, e_root, Pi;
    if (found >= 0) {
      const uint32_t idx = L - 1 - (uint32_t)found;
      e_len = (uint32_t)S.len[idx] + 1; Pi = S.j[idx]; e_root = S.root[idx];
    } else {
      e_len = 1; Pi = n; e_root = i;
    }
    uint32_t dst;
    if (best_t < 0) {
      dst = L;  // insert at the list head
    } else {
      // insert after list position q: move R[L-1-q .. L-1] up by one
      const int64_t lo = (int64_t)L - 1 - best_t;
      for (int64_t top = (int64_t)L - 1; top >= lo; top -= 64) {
        const int64_t sidx = top - lane;
        IDX vj = 0, vl = 0, vr = 0;
        const bool act = sidx >= lo;
        if (act) { vj = S.j[sidx]; vl = S.len[sidx]; vr = S.root[sidx]; }
        wave_sync();
        if (act) { S.j[sidx + 1] = vj; S.len[sidx + 1] = vl; S.root[sidx + 1] = vr; }
        wave_sync();
      }
      dst = (uint32_t)lo;
    }
    if (lane == 0) {
      S.j[dst] = (IDX)i; S.len[dst] = (IDX)e_len; S.root[dst] = (IDX)e_root; S.P[i] = (IDX)Pi;
    }
    wave_sync();
    ++L;
    if (longest < e_len) {
      const int2 xr = X[e_root];
      if (lp.seq_all || linear_ok(lp.a, (double)(xi.x - xr.x), (double)(xi.y - xr.y))) { longest = e_len; longest_ind = i; }
    }
  }
  if (lane == 0) {
    uint32_t s = longest_ind;
    for (uint32_t t = 0; t < longest; ++t) { out[longest - 1 - t] = (IDX)s; s = S.P[s]; }
  }
  wave_sync();
  return longest;
}

// wave-level bitonic sort of np2 (power of two) u64 keys, ascending
DEV void wave_bitonic(uint64_t* a, uint32_t np2) {
  const int lane = lane_id();
  for (uint32_t kk = 2; kk <= np2; kk <<= 1) {
    for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
      for (uint32_t i = lane; i < np2; i += 64) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const uint64_t x = a[i], y = a[l];
          const bool up = (i & kk) == 0;
          if ((x > y) == up) { a[i] = y; a[l] = x; }
        }
      }
      wave_sync();
    }
  }
}

// per-chain list: (pb_off asc, |sr_off| desc) == append order of
// fetch_super_reads (PB k-mer order, then pos_iterator's descending SA order)
DEV void load_sort_strand(const int2* src, uint32_t n, bool bwd, uint64_t* keys) {
  const int lane = lane_id();
  uint32_t np2 = 1;
  while (np2 < n) np2 <<= 1;
  for (uint32_t i = lane; i < np2; i += 64) {
    uint64_t kk = ~0ull;
    if (i < n) {
      const int2 h = src[i];
      const uint32_t a = (uint32_t)(h.y < 0 ? -h.y : h.y);
      kk = ((uint64_t)(uint32_t)h.x << 32) | (uint64_t)(0xFFFFFFFFu - a);
    }
    keys[i] = kk;
  }
  wave_sync();
  if (n > 1) wave_bitonic(keys, np2);
  int2* X = (int2*)keys;
  for (uint32_t i = lane; i < n; i += 64) {
    const uint64_t kk = keys[i];
    const int32_t a = (int32_t)(0xFFFFFFFFu - (uint32_t)kk);
    X[i] = make_int2((int32_t)(kk >> 32), bwd ? -a : a);
  }
  wave_sync();
}


// compute_kmers_info (pb_aligner.cc:84-143) for one lis, on lane 0.
// ids: unitig ids of the fwd name; rev => bwd name (reversed list).
DEV uint32_t kmers_info_run(const uint32_t* ids, uint32_t nsz, bool rev, const AlignParamsDev& P,
                            const int2* X, const uint32_t* lisv, uint32_t nlis, bool fwd_align, uint32_t ql,
                            int32_t* mers, int32_t* bases) {
  const int32_t k = (int32_t)P.k, uk = (int32_t)P.unitigs_k;
  auto uid = [&](uint32_t i) -> uint32_t { return i >= nsz ? INVALID_UNITIG : (rev ? ids[nsz - 1 - i] : ids[i]); };
  const uint32_t id0 = uid(0);
  if (!(id0 != INVALID_UNITIG && id0 < P.n_ul)) return 0;
  const uint32_t size = 2 * nsz - 1;
  for (uint32_t i = 0; i < size; ++i) { mers[i] = 0; bases[i] = 0; }
  uint32_t cunitig = 0;
  int32_t cend = P.ul[id0];
  int32_t prev_pos = (int32_t)(0u - P.k);
  for (uint32_t t = 0; t < nlis; ++t) {
    const int32_t so = X[lisv[t]].y;
    const int32_t pos = fwd_align ? so : (int32_t)(ql + (uint32_t)so - P.k + 2u);
    const int32_t sr_pos = pos < 0 ? -pos : pos;
    const int32_t new_bases = k < sr_pos - prev_pos ? k : sr_pos - prev_pos;
    while (sr_pos + k > cend + 1) {
      if (cend >= sr_pos) {
        if (cunitig >= nsz - 1) return 0;
        const int32_t mx = sr_pos > prev_pos + k ? sr_pos : prev_pos + k;
        const int32_t nbb = cend - mx + 1;
        bases[2 * cunitig] += nbb; bases[2 * cunitig + 1] += nbb;
      }
      const uint32_t id = uid(++cunitig);
      if (id == INVALID_UNITIG || id >= P.n_ul) return 0;
      cend = (int32_t)((uint32_t)cend + (uint32_t)P.ul[id] - (uint32_t)uk + 1u);
    }
    ++mers[2 * cunitig];
    bases[2 * cunitig] += new_bases;
    int32_t cendi = cend;
    for (uint32_t i = cunitig; (i < nsz - 1) && ((uint32_t)sr_pos + (uint32_t)k > (uint32_t)cendi - (uint32_t)uk + 1u); ++i) {
      const int32_t full_mer = sr_pos + uk > cendi + 1;
      mers[2 * i + 1] += full_mer; mers[2 * i + 2] += full_mer;
      const int32_t tt = sr_pos + k - cendi + uk - 2;
      const int32_t nbb = new_bases < tt ? new_bases : tt;
      bases[2 * i + 1] += nbb; bases[2 * i + 2] += nbb;
      const uint32_t id = uid(i + 1);
      if (id != INVALID_UNITIG && id < P.n_ul) cendi = (int32_t)((uint32_t)cendi + (uint32_t)P.ul[id] - (uint32_t)uk + 1u);
      else return 0;
    }
    prev_pos = sr_pos;
  }
  return size;
}

// compute_coords_info (pb_aligner.cc:11-82) + filters of align_sequence_max
// (coarse_aligner.cc:46-54), lane 0. Returns true if the record is kept.
DEV bool coords_record(const IndexView& ix, const AlignParamsDev& P, const ChainDesc& d, uint32_t rl,
                       const int2* X, const uint32_t* lisv, uint32_t nlis, bool fwd_align, Rec& R) {
  const uint32_t k = P.k;
  const uint32_t ql = (uint32_t)(ix.sr_start[d.sr + 1] - ix.sr_start[d.sr]);
  R.nb_mers = (int32_t)nlis; R.pb_cons = 0; R.sr_cons = 0; R.pb_cover = k; R.sr_cover = k;
  R.ql = ql; R.sr = d.sr; R.read = d.read; R.flags = (P.forward && !fwd_align) ? 2u : 0u;
  R.n_info = 0; R.reserved = 0; R.info_off = 0;
  R.stretch = 0; R.offset = 0; R.avg_err = 0;
  if (nlis == 0) return false;
  // least_square_2d (least_square_2d.hpp:47-67)
  double EX = 0, EY = 0, EXX = 0, EXY = 0, VX = 0, CXY = 0, NB = 0;
  long n = 0;
  int2 prev = X[lisv[0]];
  for (uint32_t t = 0; t < nlis; ++t) {
    const int2 c = X[lisv[t]];
    if (t) {
      const uint32_t pb_diff = (uint32_t)(c.x - prev.x);
      R.pb_cons += pb_diff == 1u;
      R.pb_cover += k < pb_diff ? k : pb_diff;
      const uint32_t sr_diff = (uint32_t)(c.y - prev.y);
      R.sr_cons += sr_diff == 1u;
      R.sr_cover += k < sr_diff ? k : sr_diff;
    }
    const double x = (double)c.y, y = (double)c.x;
    ++n;
    const double dn = (double)n;
    const double deltaX = __dadd_rn(x, -EX);
    EX = __dadd_rn(EX, __ddiv_rn(deltaX, dn));
    const double ndeltaX = __dadd_rn(x, -EX);
    VX = __dadd_rn(VX, __dmul_rn(deltaX, ndeltaX));
    const double deltaY = __dadd_rn(y, -EY);
    EY = __dadd_rn(EY, __ddiv_rn(deltaY, dn));
    const double ndeltaY = __dadd_rn(y, -EY);
    const double deltaXX = __dadd_rn(__dmul_rn(x, x), -EXX);
    EXX = __dadd_rn(EXX, __ddiv_rn(deltaXX, dn));
    const double deltaXY = __dadd_rn(__dmul_rn(x, y), -EXY);
    EXY = __dadd_rn(EXY, __ddiv_rn(deltaXY, dn));
    CXY = __dadd_rn(CXY, __dmul_rn(deltaX, ndeltaY));
    NB = __dadd_rn(NB, __dadd_rn(__dmul_rn(deltaXY, ndeltaX), -__dmul_rn(deltaXX, ndeltaY)));
    prev = c;
  }
  if (n == 1) {
    R.stretch = 1.0; R.offset = __dadd_rn(EY, -EX); R.avg_err = 0;
  } else {
    const double a = __ddiv_rn(CXY, VX), b = __ddiv_rn(NB, VX);
    R.stretch = a; R.offset = b;
    double e = 0;
    for (uint32_t t = 0; t < nlis; ++t) {
      const int2 c = X[lisv[t]];
      e = __dadd_rn(e, fabs(__dadd_rn(__dadd_rn(__dmul_rn(a, (double)c.y), b), -(double)c.x)));
    }
    R.avg_err = __ddiv_rn(e, (double)n);
  }
  const int2 first = X[lisv[0]], last = X[lisv[nlis - 1]];
  R.rs = first.x;
  R.re = (int32_t)((uint32_t)last.x + k - 1u);
  R.qs = first.y; R.qe = last.y;
  // canonicalize (pb_aligner.hpp:151-167)
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
  // filters
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

// off_lis::discard_LIS (pb_aligner.hpp:47-61): in-place ordered compaction
// of X without the lis elements. `mark` is scratch (>= n entries).
template <typename IDX>
DEV uint32_t wave_discard(int2* X, uint32_t n, const IDX* lisv, uint32_t nlis, IDX* mark) {
  const int lane = lane_id();
  for (uint32_t i = lane; i < n; i += 64) mark[i] = 0;
  wave_sync();
  for (uint32_t t = lane; t < nlis; t += 64) mark[lisv[t]] = 1;
  wave_sync();
  uint32_t w = 0;
  for (uint32_t c0 = 0; c0 < n; c0 += 64) {
    const uint32_t i = c0 + lane;
    const bool keep = i < n && !mark[i];
    const uint64_t bm = __ballot(keep);
    const uint32_t rank = __popcll(bm & ((1ull << lane) - 1ull));
    int2 v = make_int2(0, 0);
    if (keep) v = X[i];
    wave_sync();
    if (keep) X[w + rank] = v;
    wave_sync();
    w += (uint32_t)__popcll(bm);
  }
  return w;
}

template <typename IDX>
struct ChainMem {
  int2* Xf; int2* Xb;          // sorted strands (sort keys live here first)
  IDX* lisf; IDX* lisb;
  ListStore<IDX> S;            // list arrays + P (capacity >= max(nf, nb))
  uint32_t* lis32;             // lane-0 view of the chosen lis as u32 (capacity >= max)
};

template <typename IDX>
DEV void process_chain(const IndexView& ix, const AlignParamsDev& P, const LisParams& lp, const ChainDesc& d,
                       const int2* hits, const uint64_t* roff, ChainMem<IDX> M, const ChainOut& O,
                       uint64_t& tests) {
  const int lane = lane_id();
  load_sort_strand(hits + d.hit_base, d.nf, false, (uint64_t*)M.Xf);
  load_sort_strand(hits + d.hit_base + d.nf, d.nb, true, (uint64_t*)M.Xb);
  uint32_t nf = d.nf, nb = d.nb;
  uint32_t lf = wave_lis<IDX>(M.Xf, nf, M.S, M.lisf, lp, tests);
  uint32_t lb = wave_lis<IDX>(M.Xb, nb, M.S, M.lisb, lp, tests);
  const uint32_t rl = (uint32_t)(roff[d.read + 1] - roff[d.read]);
  uint32_t emit = 0;
  for (;;) {
    const bool fwd_align = lf >= lb;
    const uint32_t nl = fwd_align ? lf : lb;
    if (nl == 0) break;
    const int2* X = fwd_align ? M.Xf : M.Xb;
    const IDX* lis = fwd_align ? M.lisf : M.lisb;
    for (uint32_t t = lane; t < nl; t += 64) M.lis32[t] = (uint32_t)lis[t];
    wave_sync();
    int keep = 0;
    if (lane == 0) {
      Rec R;
      keep = coords_record(ix, P, d, rl, X, M.lis32, nl, fwd_align, R);
      if (keep) {
        R.emit = emit;
        if (P.unitigs_k) {
          const uint32_t u0 = ix.sr_uoff[d.sr], nsz = ix.sr_uoff[d.sr + 1] - u0;
          const uint32_t need = nsz ? 2 * nsz - 1 : 0;
          if (need) {
            const unsigned long long io = atomicAdd(O.info_count, (unsigned long long)need);
            if (io + need <= O.info_cap) {
              const uint32_t got = kmers_info_run(ix.sr_uids + u0, nsz, (R.flags & 2u) != 0, P, X, M.lis32, nl,
                                                  fwd_align, R.ql, O.info_m + io, O.info_b + io);
              R.n_info = got; R.info_off = io;
            } else {
              atomicAdd(&O.stats[ST_REC_OVERFLOW], 1ull);
            }
          }
        }
        const uint32_t ri = atomicAdd(O.rec_count, 1u);
        if (ri < O.rec_cap) O.recs[ri] = R;
        else atomicAdd(&O.stats[ST_REC_OVERFLOW], 1ull);
      }
    }
    keep = __shfl(keep, 0, 64);
    if (!keep) break;
    ++emit;
    if (!P.max_match) break;
    // mer_lists::discard_update_LIS (pb_aligner.hpp:86-92): larger lis, bwd on ties
    if (lf > lb) {
      nf = wave_discard<IDX>(M.Xf, nf, M.lisf, lf, M.S.P);
      lf = wave_lis<IDX>(M.Xf, nf, M.S, M.lisf, lp, tests);
    } else {
      nb = wave_discard<IDX>(M.Xb, nb, M.lisb, lb, M.S.P);
      lb = wave_lis<IDX>(M.Xb, nb, M.S, M.lisb, lp, tests);
    }
  }
}

// LDS path: WAVES waves per block, each with its own CAP-element slice.
template <int WAVES, int CAP>
__global__ __launch_bounds__(WAVES * 64) void k_chain_lds(IndexView ix, AlignParamsDev P, LisParams lp,
                                                          const ChainDesc* __restrict__ chains, uint32_t n_chains,
                                                          const int2* __restrict__ hits, const uint64_t* __restrict__ roff,
                                                          ChainOut O) {
  // per wave: Xf, Xb (8B), lisf, lisb, j, len, root, P (2B) , lis32 (4B)
  constexpr int BYTES = CAP * (8 + 8 + 2 * 6 + 4);
  extern __shared__ __align__(16) uint8_t s_mem[];
  const int w = threadIdx.x >> 6;
  uint8_t* base = s_mem + (size_t)w * BYTES;
  ChainMem<uint16_t> M;
  M.Xf = (int2*)base; M.Xb = (int2*)(base + 8 * CAP);
  uint16_t* p16 = (uint16_t*)(base + 16 * CAP);
  M.lisf = p16; M.lisb = p16 + CAP; M.S.j = p16 + 2 * CAP; M.S.len = p16 + 3 * CAP; M.S.root = p16 + 4 * CAP;
  M.S.P = p16 + 5 * CAP;
  M.lis32 = (uint32_t*)(base + 28 * CAP);
  uint64_t tests = 0;
  for (uint32_t c = blockIdx.x * WAVES + w; c < n_chains; c += gridDim.x * WAVES) {
    const ChainDesc d = chains[c];
    process_chain<uint16_t>(ix, P, lp, d, hits, roff, M, O, tests);
  }
  tests = wave_sum_u64(tests);
  if (lane_id() == 0 && tests) atomicAdd(&O.stats[ST_LIS_TESTS], (unsigned long long)tests);
}

// Global-memory path for chains longer than the LDS capacities.  Scratch
// per chain at d.scratch (elements): Xf/Xb sort keys (8B x np2), lis (4B),
// list arrays (4 x 4B) -- all sized by the chain's element counts.
__global__ __launch_bounds__(64) void k_chain_global(IndexView ix, AlignParamsDev P, LisParams lp,
                                                     const ChainDesc* __restrict__ chains, uint32_t n_chains,
                                                     const int2* __restrict__ hits, const uint64_t* __restrict__ roff,
                                                     uint8_t* scratch, ChainOut O) {
  uint64_t tests = 0;
  for (uint32_t c = blockIdx.x; c < n_chains; c += gridDim.x) {
    const ChainDesc d = chains[c];
    const uint32_t mx = d.nf > d.nb ? d.nf : d.nb;
    uint32_t np2 = 1;
    while (np2 < mx) np2 <<= 1;
    // region size: 2*8*np2 + 8*4*np2 bytes, reserved as 48*np2 per chain by the host
    uint8_t* base = scratch + d.scratch * 48;  // d.scratch counts elements of np2 granularity
    ChainMem<uint32_t> M;
    M.Xf = (int2*)base; M.Xb = (int2*)(base + 8ull * np2);
    uint32_t* p32 = (uint32_t*)(base + 16ull * np2);
    M.lisf = p32; M.lisb = p32 + np2; M.S.j = p32 + 2 * np2; M.S.len = p32 + 3 * np2; M.S.root = p32 + 4 * np2;
    M.S.P = p32 + 5 * np2; M.lis32 = p32 + 6 * np2;
    process_chain<uint32_t>(ix, P, lp, d, hits, roff, M, O, tests);
  }
  tests = wave_sum_u64(tests);
  if (lane_id() == 0 && tests) atomicAdd(&O.stats[ST_LIS_TESTS], (unsigned long long)tests);
}

// =============================================================== records
__global__ void k_rec_hist(const Rec* recs, uint32_t n, uint32_t* per_read) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    atomicAdd(&per_read[recs[i].read], 1u);
}
__global__ void k_rec_scatter(const Rec* recs, uint32_t n, const uint64_t* rec_off, uint32_t* cursor, uint32_t* order) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t r = recs[i].read;
    order[rec_off[r] + atomicAdd(&cursor[r], 1u)] = i;
  }
}

DEV bool rec_less(const Rec& a, const Rec& b) {
  if (a.rs != b.rs) return a.rs < b.rs;
  if (a.re != b.re) return a.re < b.re;
  if (a.ql != b.ql) return a.ql < b.ql;
  if (a.sr != b.sr) return a.sr < b.sr;
  return a.emit < b.emit;
}

// One block per read: sort the read's record indices by (rs, re, ql, sr, emit)
// with an odd-even merge (bitonic) network over LDS (or global for big reads),
// then gather the records in that order.
template <int BLOCK, int LCAP>
__global__ __launch_bounds__(BLOCK) void k_rec_sort(const Rec* __restrict__ recs, const uint64_t* __restrict__ rec_off,
                                                    const uint32_t* __restrict__ order_in, uint32_t* gscratch,
                                                    uint32_t n_reads, Rec* __restrict__ out) {
  __shared__ uint32_t s_idx[LCAP];
  const uint32_t r = blockIdx.x;
  if (r >= n_reads) return;
  const uint64_t b = rec_off[r];
  const uint32_t n = (uint32_t)(rec_off[r + 1] - b);
  if (n == 0) return;
  uint32_t np2 = 1;
  while (np2 < n) np2 <<= 1;
  uint32_t* a = np2 <= LCAP ? s_idx : gscratch + 2 * b;  // host reserves 2x per read for the global case
  for (uint32_t i = threadIdx.x; i < np2; i += BLOCK) a[i] = i < n ? order_in[b + i] : 0xFFFFFFFFu;
  __syncthreads();
  for (uint32_t kk = 2; kk <= np2; kk <<= 1) {
    for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < np2; i += BLOCK) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const uint32_t x = a[i], y = a[l];
          bool gt;  // x > y ?
          if (x == 0xFFFFFFFFu) gt = y != 0xFFFFFFFFu;
          else if (y == 0xFFFFFFFFu) gt = false;
          else gt = rec_less(recs[y], recs[x]);
          const bool up = (i & kk) == 0;
          if (gt == up) { a[i] = y; a[l] = x; }
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t i = threadIdx.x; i < n; i += BLOCK) out[b + i] = recs[a[i]];
}

}  // namespace pbgpu

// ====================================================== launch wrappers
namespace pbgpu {

void launch_build_keys(IndexView ix, uint64_t N, uint64_t* keys, uint64_t* vals, hipStream_t st) {
  hipLaunchKernelGGL(k_build_keys, dim3(4096), dim3(256), 0, st, ix, N, keys, vals);
}
void launch_runs(const uint64_t* keys, const uint64_t* uidx, uint64_t N, uint64_t* run_start, hipStream_t st) {
  hipLaunchKernelGGL(k_runs, dim3(4096), dim3(256), 0, st, keys, uidx, N, run_start);
}
void launch_occ_fill(const uint64_t* vals, const uint64_t* uidx, const uint64_t* kpos, uint64_t N, uint64_t* occ,
                     hipStream_t st) {
  hipLaunchKernelGGL(k_occ_fill, dim3(4096), dim3(256), 0, st, vals, uidx, kpos, N, occ);
}
void launch_headers(const uint64_t* keys, const uint64_t* kpos, const uint64_t* run_start, uint64_t U, uint64_t* occ,
                    ulonglong2* table, uint64_t bucket_mask, uint32_t k, hipStream_t st) {
  hipLaunchKernelGGL(k_headers, dim3(4096), dim3(256), 0, st, keys, kpos, run_start, U, occ, table, bucket_mask, k);
}

constexpr int SEED_BLOCK = 256, SEED_PER = 8;
void launch_seed(IndexView ix, const uint8_t* seq, const uint64_t* roff, uint32_t n_reads, AlignParamsDev P,
                 KRec* krec, uint32_t* n_kept, uint32_t* thr, uint64_t* nhits, unsigned long long* stats, hipStream_t st) {
  hipLaunchKernelGGL((k_seed<SEED_BLOCK, SEED_PER>), dim3(n_reads), dim3(SEED_BLOCK), 0, st, ix, seq, roff, n_reads, P,
                     krec, n_kept, thr, nhits, stats);
}

constexpr int GROUP_BLOCK = 256;
void launch_group(IndexView ix, const KRec* krec, const uint64_t* roff, const uint32_t* n_kept, const uint32_t* thr,
                  const uint64_t* hit_off, const uint32_t* read_list, uint32_t n_list, uint32_t hcap_log2,
                  uint32_t* gtable, GroupOut O, unsigned long long* stats, hipStream_t st) {
  if (!gtable) {
    const size_t lds = (size_t)4 * sizeof(uint32_t) << hcap_log2;
    hipLaunchKernelGGL((k_group<GROUP_BLOCK, false>), dim3(n_list), dim3(GROUP_BLOCK), lds, st, ix, krec, roff, n_kept,
                       thr, hit_off, read_list, n_list, hcap_log2, gtable, O, stats);
  } else {
    hipLaunchKernelGGL((k_group<GROUP_BLOCK, true>), dim3(n_list), dim3(GROUP_BLOCK), 0, st, ix, krec, roff, n_kept,
                       thr, hit_off, read_list, n_list, hcap_log2, gtable, O, stats);
  }
}

constexpr int CH_SMALL_WAVES = 4, CH_SMALL_CAP = 512;
constexpr int CH_LARGE_WAVES = 1, CH_LARGE_CAP = 4096;
int chain_cap_small() { return CH_SMALL_CAP; }
int chain_cap_large() { return CH_LARGE_CAP; }

void launch_chain_small(IndexView ix, AlignParamsDev P, LisParams lp, const ChainDesc* chains, uint32_t n,
                        const int2* hits, const uint64_t* roff, ChainOut O, hipStream_t st) {
  if (!n) return;
  constexpr size_t lds = (size_t)CH_SMALL_WAVES * CH_SMALL_CAP * (8 + 8 + 2 * 6 + 4);
  uint32_t grid = (n + CH_SMALL_WAVES - 1) / CH_SMALL_WAVES;
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL((k_chain_lds<CH_SMALL_WAVES, CH_SMALL_CAP>), dim3(grid), dim3(CH_SMALL_WAVES * 64), lds, st, ix, P,
                     lp, chains, n, hits, roff, O);
}
void launch_chain_large(IndexView ix, AlignParamsDev P, LisParams lp, const ChainDesc* chains, uint32_t n,
                        const int2* hits, const uint64_t* roff, ChainOut O, hipStream_t st) {
  if (!n) return;
  constexpr size_t lds = (size_t)CH_LARGE_WAVES * CH_LARGE_CAP * (8 + 8 + 2 * 6 + 4);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_chain_lds<CH_LARGE_WAVES, CH_LARGE_CAP>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  uint32_t grid = n < 4096 ? n : 4096;
  hipLaunchKernelGGL((k_chain_lds<CH_LARGE_WAVES, CH_LARGE_CAP>), dim3(grid), dim3(CH_LARGE_WAVES * 64), lds, st, ix, P,
                     lp, chains, n, hits, roff, O);
}
void launch_chain_huge(IndexView ix, AlignParamsDev P, LisParams lp, const ChainDesc* chains, uint32_t n,
                       const int2* hits, const uint64_t* roff, uint8_t* scratch, ChainOut O, hipStream_t st) {
  if (!n) return;
  uint32_t grid = n < 1024 ? n : 1024;
  hipLaunchKernelGGL(k_chain_global, dim3(grid), dim3(64), 0, st, ix, P, lp, chains, n, hits, roff, scratch, O);
}

void launch_rec_hist(const Rec* recs, uint32_t n, uint32_t* per_read, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_rec_hist, dim3(1024), dim3(256), 0, st, recs, n, per_read);
}
void launch_rec_scatter(const Rec* recs, uint32_t n, const uint64_t* rec_off, uint32_t* cursor, uint32_t* order,
                        hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_rec_scatter, dim3(1024), dim3(256), 0, st, recs, n, rec_off, cursor, order);
}
constexpr int REC_BLOCK = 256, REC_LCAP = 4096;
int rec_sort_lcap() { return REC_LCAP; }
void launch_rec_sort(const Rec* recs, const uint64_t* rec_off, const uint32_t* order, uint32_t* gscratch,
                     uint32_t n_reads, Rec* out, hipStream_t st) {
  if (!n_reads) return;
  hipLaunchKernelGGL((k_rec_sort<REC_BLOCK, REC_LCAP>), dim3(n_reads), dim3(REC_BLOCK), 0, st, recs, rec_off, order,
                     gscratch, n_reads, out);
}

}  // namespace pbgpu
