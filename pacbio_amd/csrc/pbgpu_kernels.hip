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
// One workgroup (4 waves) per read: enumerate the read's hits exactly in the reference's
// append order (kept k-mers in read order; per k-mer occ(m) then occ(rm),
// each in descending text position == pos_iterator, superread_parser.hpp:
// 110-140), group them by super-read in an open-addressing table (LDS, or a
// global region for reads touching more super-reads than the LDS table
// holds), and scatter every hit to its (read, SR, strand) list with an
// order-preserving multisplit.  Each list comes out in exactly the
// reference's frags_pos order (coarse_aligner.cc:128-140) -- no sort needed.
constexpr uint32_t GROUP_BLOCK = 256;  // 4 waves share one read's table

template <bool GLOBAL_TABLE>
__global__ __launch_bounds__(GROUP_BLOCK) void k_group(IndexView ix, const KRec* __restrict__ krec,
                                                       const uint64_t* __restrict__ roff, const uint32_t* __restrict__ n_kept,
                                                       const uint32_t* __restrict__ thr_in, const uint64_t* __restrict__ hit_off,
                                                       uint64_t node_base, uint32_t r0, const uint32_t* __restrict__ read_list,
                                                       uint32_t n_list, uint32_t hcap_log2, uint32_t* gtable, GroupOut O,
                                                       unsigned long long* stats) {
  constexpr uint32_t B = GROUP_BLOCK;
  extern __shared__ uint32_t s_dyn[];
  __shared__ uint32_t s_nf[B], s_nb[B], s_off[B + 1], s_scan[8];
  __shared__ int32_t s_pb[B];
  __shared__ uint64_t s_pf[B], s_pbk[B];
  __shared__ uint32_t s_flag, s_used, s_cbase;
  if (blockIdx.x >= n_list) return;
  const uint32_t tid = threadIdx.x;
  const int lane = lane_id();
  const uint32_t wave = tid >> 6;
  const uint32_t r = read_list ? read_list[blockIdx.x] : r0 + blockIdx.x;
  const uint32_t hcap = 1u << hcap_log2;
  // table: key (sr + 1, 0 = empty), fwd count/cursor, bwd count/cursor, 2*hcap byte tags
  uint32_t* tkey = GLOBAL_TABLE ? gtable + (uint64_t)blockIdx.x * (7u * hcap / 2) : s_dyn;
  uint32_t* tcf = tkey + hcap;
  uint32_t* tcb = tcf + hcap;
  uint8_t* tag = (uint8_t*)(tcb + hcap);
  if (!GLOBAL_TABLE)  // the global variant is zeroed by hipMemsetAsync
    for (uint32_t i = tid; i < hcap; i += B) { tkey[i] = 0; tcf[i] = 0; tcb[i] = 0; }
  if (tid == 0) { s_flag = 0; s_used = 0; }
  __syncthreads();
  const uint64_t kbase = roff[r];
  const uint32_t nk = n_kept[r], thr = thr_in[r];
  const uint64_t hbase = hit_off[r] - node_base;
  const uint32_t used_limit = hcap - hcap / 4;
  const uint64_t lt_mask = (1ull << lane) - 1ull;

  for (int pass = 0; pass < 2; ++pass) {
    for (uint32_t g0 = 0; g0 < nk; g0 += B) {
      if (s_flag) break;  // uniform (written before the last barrier)
      const uint32_t i = g0 + tid;
      uint32_t nf = 0, nb = 0;
      if (i < nk) {
        const KRec kr = krec[kbase + i];
        if (kr.count <= thr) {
          const uint64_t ptr = kr.occ_ptr & ~(1ull << 63);
          const bool canon = kr.occ_ptr >> 63;
          const uint64_t h0 = ix.occ[ptr], h1 = ix.occ[ptr + 1];
          const uint32_t nA = (uint32_t)(h1 & 0xFFFFFFFFull), nB = (uint32_t)(h1 >> 32);
          const uint64_t A = ptr + 2, Bp = ptr + 2 + nA;
          // occ(m) -> fwd list (+off), occ(rm) -> bwd list (-off)    
          if ((h0 >> 32) & 1) { nf = nb = nA; s_pf[tid] = A; s_pbk[tid] = A; }
          else if (canon) { nf = nA; s_pf[tid] = A; nb = nB; s_pbk[tid] = Bp; }
          else { nf = nB; s_pf[tid] = Bp; nb = nA; s_pbk[tid] = A; }
          s_pb[tid] = kr.pb_off;
        }
      }
      s_nf[tid] = nf; s_nb[tid] = nb;
      uint32_t total;
      s_off[tid] = block_excl_scan<B>(nf + nb, s_scan, total);
      if (tid == 0) s_off[B] = total;
      __syncthreads();
      for (uint32_t h0 = 0; h0 < total; h0 += B) {
        const uint32_t h = h0 + tid;
        const bool valid = h < total;
        uint32_t sr = 0, slot = 0, rec = 0xFFFFFFFFu;
        int32_t so = 0, pb = 0;
        bool fwd = true;
        if (valid) {
          uint32_t lo = 0, hi = B;  // last record with s_off <= h
          while (hi - lo > 1) { const uint32_t md = (lo + hi) >> 1; if (s_off[md] <= h) lo = md; else hi = md; }
          rec = lo;
          const uint32_t local = h - s_off[lo];
          fwd = local < s_nf[lo];
          const uint64_t e = ix.occ[fwd ? s_pf[lo] + local : s_pbk[lo] + (local - s_nf[lo])];
          sr = (uint32_t)(e >> 32);
          so = (int32_t)(uint32_t)(e & 0xFFFFFFFFull);
          pb = s_pb[lo];
          slot = (sr * 0x9E3779B1u) >> (32 - hcap_log2);
        }
        if (pass == 0) {
          // order-free: distinct super-reads and per-strand list lengths
          if (valid) {
            bool ok = true;
            for (;;) {
              const uint32_t old = atomicCAS(&tkey[slot], 0u, sr + 1);
              if (old == 0) { if (atomicAdd(&s_used, 1u) >= used_limit) { s_flag = 1; ok = false; } break; }
              if (old == sr + 1) break;
              slot = (slot + 1) & (hcap - 1);
            }
            if (ok) atomicAdd(fwd ? &tcf[slot] : &tcb[slot], 1u);
          }
        } else {
          if (valid) while (tkey[slot] != sr + 1) slot = (slot + 1) & (hcap - 1);
          // Order-preserving multisplit over (slot, strand) keys.  The four waves hold
          // consecutive 64-hit runs; they take the list cursors in wave order (LDS only,
          // after all loads are in flight).  Within a wave, hits of one k-mer record hit
          // distinct super-reads (except SRs holding the k-mer twice), so the run is
          // processed record segment by record segment (usually 1-2), each segment in
          // one conflict-free step; a tag check catches in-record repeats.
          const uint32_t key = (slot << 1) | (fwd ? 0u : 1u);
          uint32_t pos = 0;
          for (uint32_t w = 0; w < B / 64; ++w) {
            if (wave == w) {
              uint64_t active = __ballot(valid);
              while (active) {
                const int leader = __ffsll((unsigned long long)active) - 1;
                const uint32_t lrec = __builtin_amdgcn_readlane(rec, leader);
                const bool in_seg = rec == lrec;
                const uint64_t seg = __ballot(in_seg);
                if (in_seg) tag[key] = (uint8_t)lane;
                if (GLOBAL_TABLE) __threadfence_block();
                __builtin_amdgcn_s_waitcnt(0);
                __builtin_amdgcn_wave_barrier();
                const bool dup = in_seg && tag[key] != (uint8_t)lane;
                if (!__ballot(dup)) {
                  if (in_seg) { uint32_t* cur = fwd ? &tcf[slot] : &tcb[slot]; pos = *cur; *cur = pos + 1; }
                } else {
                  const uint32_t k2 = in_seg ? key : 0xFFFFFFFFu;
                  uint64_t act2 = seg;
                  while (act2) {
                    const int l2 = __ffsll((unsigned long long)act2) - 1;
                    const uint32_t lk = __builtin_amdgcn_readlane(k2, l2);
                    const uint64_t peers = __ballot(k2 == lk);
                    uint32_t* cur = (lk & 1) ? &tcb[lk >> 1] : &tcf[lk >> 1];
                    if (k2 == lk) {
                      const uint32_t b = *cur;
                      pos = b + (uint32_t)__popcll(peers & lt_mask);
                      if (lane == l2) *cur = b + (uint32_t)__popcll(peers);
                    }
                    act2 &= ~peers;
                  }
                }
                if (GLOBAL_TABLE) __threadfence_block();
                __builtin_amdgcn_s_waitcnt(0);
                __builtin_amdgcn_wave_barrier();
                active &= ~seg;
              }
            }
            __syncthreads();
          }
          if (valid) *(int2*)&O.nodes[hbase + pos] = make_int2(pb, fwd ? so : -so);
        }
      }
      __syncthreads();
    }
    if (pass == 0) {
      if (s_flag) {  // table too full: this read is redone with a larger table
        if (tid == 0) { const uint32_t o = atomicAdd(O.n_overflow, 1u); O.overflow_reads[o] = r; }
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
      const uint32_t enn = block_excl_scan<B>(nn, s_scan, tn);
      if (tid == 0) {
        s_cbase = atomicAdd(O.chain_count, tn);
        atomicAdd(&stats[ST_CHAINS], (unsigned long long)tn);
      }
      __syncthreads();
      uint32_t b0 = esum, ci = s_cbase + enn;
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
    }
  }
}

// chains by descending length class (ceil log2 of nf + nb): long chains start
// first and lanes of a wave get chains of similar length
DEV uint32_t chain_bucket(const ChainDesc& d) {
  const uint32_t t = d.nf + d.nb;
  return t ? 31u - (uint32_t)__clz(t) : 0u;  // floor(log2)
}
__global__ void k_chain_hist(const ChainDesc* __restrict__ chains, uint32_t n, uint32_t* hist) {
  __shared__ uint32_t h[32];
  if (threadIdx.x < 32) h[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x)
    atomicAdd(&h[chain_bucket(chains[c])], 1u);
  __syncthreads();
  if (threadIdx.x < 32 && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}
__global__ void k_chain_perm(const ChainDesc* __restrict__ chains, uint32_t n, uint32_t* cursor, uint32_t* perm) {
  // block-aggregated: one global atomic per (block, bucket)
  __shared__ uint32_t cnt[32], base[32];
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (threadIdx.x < 32) cnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t b = 0, loc = 0;
  if (c < n) { b = chain_bucket(chains[c]); loc = atomicAdd(&cnt[b], 1u); }
  __syncthreads();
  if (threadIdx.x < 32 && cnt[threadIdx.x]) base[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], cnt[threadIdx.x]);
  __syncthreads();
  if (c < n) perm[base[b] + loc] = c;
}

// ================================================================= chain
// One LANE per chain (read, super-read): both strands' LIS, the fit, the
// filters and --max-match, i.e. coarse_aligner::align_sequence_max's loop body
// (coarse_aligner.cc:42-60) for one frags_pos entry.  A wave runs 64 chains;
// the typical LIS scan stops at the list head, which stays in registers.
DEV bool affine_ok(double a, double b, double C, double df, double ds) {
  // (s.first <= b + a*s.second) && (s.second <= b + a*s.first) && s.first <= C && s.second <= C
  return (df <= __dadd_rn(b, __dmul_rn(a, ds))) && (ds <= __dadd_rn(b, __dmul_rn(a, df))) && df <= C && ds <= C;
}
DEV bool linear_ok(double a, double df, double ds) {
  return (df <= __dmul_rn(a, ds)) && (ds <= __dmul_rn(a, df));
}

// lis_align::compute_L_P (lis_align.hpp:139-182) + indices (:190-204),
// restated literally: singly linked list L, first acceptable predecessor in
// list order, insertion after the first node of minimal length seen before
// it.  The window test uses X[i] - X[anc_{W-1}(j)], which equals
// sum_buffer::test_sum exactly (all values are small integers).
// Returns the LIS length; the ascending lis is left in A[0..len).aux.
DEV uint32_t lane_lis(Node* __restrict__ A, uint32_t n, const LisParams& lp, uint64_t& tests) {
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  uint32_t head = NONE, longest = 0, longest_ind = 0;
  int32_t hpb = 0, hsr = 0, hrpb = 0, hrsr = 0;  // head node cached in registers
  uint32_t hnxt = NONE, hlen = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const int2 xi = *(const int2*)&A[i];
    uint32_t prev = NONE, prev_len = 0, prev_nxt = NONE, found = NONE;
    uint32_t f_len = 0;
    int32_t f_rpb = 0, f_rsr = 0;
    if (head != NONE) {
      uint32_t it = head, lj = hlen, nx = hnxt;
      int32_t jpb = hpb, jsr = hsr, jrpb = hrpb, jrsr = hrsr;
      for (;;) {
        ++tests;
        if (xi.y > jsr) {
          bool ok;
          if (lp.mer_all) ok = true;
          else if (lp.W == 1) ok = affine_ok(lp.a, lp.b, lp.C, (double)(xi.x - jpb), (double)(xi.y - jsr));
          else if (lp.W == 0 || lj < lp.W) ok = true;  // !will_be_filled()
          else {
            uint32_t anc = it;
            for (uint32_t w = 1; w < lp.W; ++w) anc = A[anc].P;
            const int2 xa = *(const int2*)&A[anc];
            ok = affine_ok(lp.a, lp.b, lp.C, (double)(xi.x - xa.x), (double)(xi.y - xa.y));
          }
          if (ok) { found = it; f_len = lj; f_rpb = jrpb; f_rsr = jrsr; break; }
        }
        if (prev == NONE || lj < prev_len) { prev = it; prev_len = lj; prev_nxt = nx; }
        it = nx;
        if (it == NONE) break;
        const Node nd = A[it];
        jpb = nd.pb; jsr = nd.sr; jrpb = nd.rpb; jrsr = nd.rsr; lj = nd.len; nx = nd.nxt;
      }
    }
    Node e;
    e.pb = xi.x; e.sr = xi.y; e.aux = 0;
    if (found != NONE) { e.len = f_len + 1; e.rpb = f_rpb; e.rsr = f_rsr; e.P = found; }
    else { e.len = 1; e.rpb = xi.x; e.rsr = xi.y; e.P = NONE; }
    if (prev == NONE) {  // insert at the head
      e.nxt = head;
      head = i; hpb = e.pb; hsr = e.sr; hrpb = e.rpb; hrsr = e.rsr; hnxt = e.nxt; hlen = e.len;
    } else {
      e.nxt = prev_nxt;
      A[prev].nxt = i;
      if (prev == head) hnxt = i;
    }
    A[i] = e;
    if (longest < e.len &&
        (lp.seq_all || linear_ok(lp.a, (double)(xi.x - e.rpb), (double)(xi.y - e.rsr)))) {
      longest = e.len; longest_ind = i;
    }
  }
  uint32_t s = longest_ind;
  for (uint32_t t = 0; t < longest; ++t) { A[longest - 1 - t].aux = s; s = A[s].P; }
  return longest;
}

// compute_kmers_info (pb_aligner.cc:84-143) along one lis.
// ids: unitig ids of the fwd name; rev => bwd name (reversed list).
DEV uint32_t kmers_info_run(const uint32_t* ids, uint32_t nsz, bool rev, const AlignParamsDev& P, const Node* A,
                            uint32_t nlis, bool fwd_align, uint32_t ql, int32_t* mers, int32_t* bases) {
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
    const int32_t so = A[A[t].aux].sr;
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

// compute_coords_info (pb_aligner.cc:11-82) + the filters of
// align_sequence_max (coarse_aligner.cc:46-54). Returns true if kept.
DEV bool coords_record(const IndexView& ix, const AlignParamsDev& P, const ChainDesc& d, uint32_t rl,
                       const Node* A, uint32_t nlis, bool fwd_align, Rec& R) {
  const uint32_t k = P.k;
  const uint32_t ql = (uint32_t)(ix.sr_start[d.sr + 1] - ix.sr_start[d.sr]);
  R.nb_mers = (int32_t)nlis; R.pb_cons = 0; R.sr_cons = 0; R.pb_cover = k; R.sr_cover = k;
  R.ql = ql; R.sr = d.sr; R.read = d.read; R.flags = (P.forward && !fwd_align) ? 2u : 0u;
  R.n_info = 0; R.reserved = 0; R.info_off = 0; R.emit = 0;
  R.stretch = 0; R.offset = 0; R.avg_err = 0;
  if (nlis == 0) return false;
  // least_square_2d::add (least_square_2d.hpp:47-67), x = sr offset, y = pb offset
  double EX = 0, EY = 0, EXX = 0, EXY = 0, VX = 0, CXY = 0, NB = 0;
  long n = 0;
  int2 prev = *(const int2*)&A[A[0].aux];
  const int2 first = prev;
  for (uint32_t t = 0; t < nlis; ++t) {
    const int2 c = *(const int2*)&A[A[t].aux];
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
  const int2 last = prev;
  if (n == 1) {
    R.stretch = 1.0; R.offset = __dadd_rn(EY, -EX); R.avg_err = 0;
  } else {
    const double a = __ddiv_rn(CXY, VX), b = __ddiv_rn(NB, VX);
    R.stretch = a; R.offset = b;
    double e = 0;
    for (uint32_t t = 0; t < nlis; ++t) {
      const int2 c = *(const int2*)&A[A[t].aux];
      e = __dadd_rn(e, fabs(__dadd_rn(__dadd_rn(__dmul_rn(a, (double)c.y), b), -(double)c.x)));
    }
    R.avg_err = __ddiv_rn(e, (double)n);
  }
  R.rs = first.x;
  R.re = (int32_t)((uint32_t)last.x + k - 1u);
  R.qs = first.y; R.qe = last.y;
  // coords_info::canonicalize (pb_aligner.hpp:151-167)
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
  // filters: fabs(stretch)==0, min_mers (-M), min_bases (-B)  (pb_aligner.hpp:169-174)
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

__global__ __launch_bounds__(256) void k_chain(IndexView ix, AlignParamsDev P, LisParams lp,
                                               const ChainDesc* __restrict__ chains, const uint32_t* __restrict__ perm,
                                               uint32_t n_chains, Node* __restrict__ nodes,
                                               const uint64_t* __restrict__ roff, ChainOut O) {
  uint64_t tests = 0;
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < n_chains; w += gridDim.x * blockDim.x) {
    const ChainDesc d = chains[perm ? perm[w] : w];
    Node* F = nodes + d.hit_base;
    Node* B = F + d.nf;
    uint32_t nf = d.nf, nb = d.nb;
    uint32_t lf = lane_lis(F, nf, lp, tests);
    uint32_t lb = lane_lis(B, nb, lp, tests);
    const uint32_t rl = (uint32_t)(roff[d.read + 1] - roff[d.read]);
    for (uint32_t emit = 0;; ++emit) {
      const bool fwd_align = lf >= lb;
      const uint32_t nl = fwd_align ? lf : lb;
      if (nl == 0) break;
      const Node* A = fwd_align ? F : B;
      Rec R;
      if (!coords_record(ix, P, d, rl, A, nl, fwd_align, R)) break;
      R.emit = emit;
      bool ok = true;
      if (P.unitigs_k) {
        const uint32_t u0 = ix.sr_uoff[d.sr], nsz = ix.sr_uoff[d.sr + 1] - u0;
        const uint32_t need = nsz ? 2 * nsz - 1 : 0;
        if (need) {
          const unsigned long long io = atomicAdd(O.info_count, (unsigned long long)need);
          if (io + need <= O.info_cap) {
            R.n_info = kmers_info_run(ix.sr_uids + u0, nsz, (R.flags & 2u) != 0, P, A, nl, fwd_align, R.ql,
                                      O.info_m + io, O.info_b + io);
            R.info_off = io;
          } else {
            ok = false;
          }
        }
      }
      const uint32_t ri = atomicAdd(O.rec_count, 1u);
      if (ri < O.rec_cap && ok) O.recs[ri] = R;
      else atomicAdd(&O.stats[ST_REC_OVERFLOW], 1ull);
      if (!P.max_match) break;
      // mer_lists::discard_update_LIS (pb_aligner.hpp:86-92): the longer lis, bwd on ties;
      // off_lis::discard_LIS (pb_aligner.hpp:47-61) keeps the remaining offsets in order
      Node* D = lf > lb ? F : B;
      uint32_t& nD = lf > lb ? nf : nb;
      uint32_t& lD = lf > lb ? lf : lb;
      uint32_t wpos = 0, li = 0;
      for (uint32_t rpos = 0; rpos < nD; ++rpos) {
        if (li < lD && rpos == D[li].aux) { ++li; continue; }
        *(int2*)&D[wpos++] = *(const int2*)&D[rpos];
      }
      nD -= lD;
      lD = lane_lis(D, nD, lp, tests);
    }
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

void launch_group(IndexView ix, const KRec* krec, const uint64_t* roff, const uint32_t* n_kept, const uint32_t* thr,
                  const uint64_t* hit_off, uint64_t node_base, uint32_t r0, const uint32_t* read_list, uint32_t n_list,
                  uint32_t hcap_log2, uint32_t* gtable, GroupOut O, unsigned long long* stats, hipStream_t st) {
  if (!n_list) return;
  if (!gtable) {  // LDS table: hcap_log2 <= 13
    const size_t lds = ((size_t)7 << hcap_log2) / 2 * sizeof(uint32_t);
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)k_group<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 16 * 1024);
      attr = true;
    }
    hipLaunchKernelGGL((k_group<false>), dim3(n_list), dim3(GROUP_BLOCK), lds, st, ix, krec, roff, n_kept, thr, hit_off,
                       node_base, r0, read_list, n_list, hcap_log2, gtable, O, stats);
  } else {
    hipLaunchKernelGGL((k_group<true>), dim3(n_list), dim3(GROUP_BLOCK), 0, st, ix, krec, roff, n_kept, thr, hit_off,
                       node_base, r0, read_list, n_list, hcap_log2, gtable, O, stats);
  }
}
uint64_t group_table_words(uint32_t hcap_log2) { return ((uint64_t)7 << hcap_log2) / 2; }

static uint32_t grid_for(uint32_t n, uint32_t block, uint32_t cap = 65536) {
  uint64_t g = ((uint64_t)n + block - 1) / block;
  return (uint32_t)(g < 1 ? 1 : (g > cap ? cap : g));
}
void launch_chain_hist(const ChainDesc* chains, uint32_t n, uint32_t* hist, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_chain_hist, dim3(grid_for(n, 256, 2048)), dim3(256), 0, st, chains, n, hist);
}
void launch_chain_perm(const ChainDesc* chains, uint32_t n, uint32_t* cursor, uint32_t* perm, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_chain_perm, dim3((n + 255) / 256), dim3(256), 0, st, chains, n, cursor, perm);
}
void launch_chain(IndexView ix, AlignParamsDev P, LisParams lp, const ChainDesc* chains, const uint32_t* perm,
                  uint32_t n, Node* nodes, const uint64_t* roff, ChainOut O, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_chain, dim3(grid_for(n, 256)), dim3(256), 0, st, ix, P, lp, chains, perm, n, nodes, roff, O);
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
