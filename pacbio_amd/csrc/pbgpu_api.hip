// pbgpu_api.hip -- host side of the C ABI (include/pbgpu.h): FASTA loading
// with the reference's compact_dna rules, device index build, the per-batch
// pipeline on one HIP stream, result download and coords formatting.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pbgpu.h"
#include "pbgpu_internal.h"
#include "count_pack.h"
#include "pbgpu_host.h"

namespace pbgpu {
// kernels (pbgpu_kernels.hip)
void launch_build_keys(IndexView ix, uint32_t km, uint32_t K, uint32_t ebits, uint64_t N, const uint64_t* sel,
                       uint64_t Nsel, uint64_t* keys, uint64_t* vals, hipStream_t st);
void launch_part_ids(IndexView ix, uint32_t km, uint64_t N, uint32_t P, uint8_t* pid, unsigned long long* hist,
                     hipStream_t st);
void launch_table_insert(const ulonglong2* kh, uint64_t U, uint64_t base, ulonglong2* table, uint64_t bucket_mask,
                         uint64_t* filt, uint32_t filt_shift, hipStream_t st);
void launch_runs(const uint64_t* keys, const uint64_t* uidx, uint64_t N, uint32_t sh, uint64_t* run_start, hipStream_t st);
void launch_occ_fill(const uint64_t* vals, const uint64_t* uidx, const uint64_t* kpos, uint64_t N, uint64_t* occ,
                     hipStream_t st);
void launch_headers(const uint64_t* keys, const uint64_t* kpos, const uint64_t* run_start, uint64_t U, uint64_t* occ,
                    ulonglong2* table, uint64_t bucket_mask, uint32_t k, uint32_t ebits, uint64_t* filt,
                    uint32_t filt_shift, ulonglong2* kh, hipStream_t st);
enum { SEED_WHOLE = 0, SEED_COUNTS = 1, SEED_FINISH = 2 };  // k_seed modes (pbgpu_kernels.hip)
void launch_seed(int mode, IndexView ix, const uint8_t* seq, const uint64_t* roff, uint32_t n_reads, AlignParamsDev P,
                 KRec* krec, uint32_t* n_kept, uint32_t* thr, uint64_t* nhits, unsigned long long* stats,
                 uint32_t* gcount, uint64_t null_ptr, hipStream_t st);
void launch_group(IndexView ix, const KRec* krec, const uint64_t* roff, const uint32_t* n_kept, const uint32_t* thr,
                  const uint64_t* hit_off, uint64_t node_base, uint32_t r0, const uint2* read_list, uint32_t n_list,
                  uint32_t hcap_log2, uint32_t* gtable, GroupOut O, unsigned long long* stats, hipStream_t st,
                  int mode = 0);
uint64_t group_table_words(uint32_t hcap_log2);
void launch_sr_ul(const uint32_t* ids, uint64_t n, const int32_t* ul, uint64_t n_ul, int32_t* out, hipStream_t st);
void launch_counts_pack16(bool unpack, const uint32_t* src, uint64_t n, uint32_t* dst, hipStream_t st);
void launch_occ_sr(const uint64_t* occ, uint64_t n, uint32_t* out, hipStream_t st);
#ifndef PBGPU_GROUP_BIG_LOG2
#define PBGPU_GROUP_BIG_LOG2 13
#endif
constexpr uint32_t kGroupLdsMaxLog2 = PBGPU_GROUP_BIG_LOG2;  // 8192-slot table, 96 KiB of LDS
void launch_init_slen(const ChainDesc* chains, uint32_t n_chains, uint32_t* slen, hipStream_t st);
void launch_sr_meta(const uint64_t* sr_start, const uint32_t* sr_uoff, uint64_t n_sr, const int32_t* sr_ul, SrMeta* out,
                    hipStream_t st);
void launch_strand_order(const uint32_t* slen, uint32_t n_items, uint32_t* hist, uint32_t* cursor, uint32_t* perm,
                         int phase, hipStream_t st, const ChainDesc* chains = nullptr, uint2* pinfo = nullptr);
void launch_chain_order(const uint32_t* lisl, uint32_t n, uint32_t* hist, uint32_t* cursor, uint32_t* perm, int phase,
                        unsigned long long* sums, hipStream_t st);
void launch_lis(bool big_nodes, const ChainDesc* chains, const uint32_t* items, uint32_t n_items, const uint32_t* slen,
                const int2* X, void* N, int2* pts, uint32_t* lisl, LisParams lp, int keep_idx,
                unsigned long long* stats, hipStream_t st, const uint32_t* nshift = nullptr);
void launch_node32_place(const ChainDesc* chains, const uint32_t* items, uint32_t n, const uint32_t* slen,
                         uint32_t* nshift, unsigned long long* total, hipStream_t st);
uint32_t node32_chunk();
void launch_coords(IndexView ix, AlignParamsDev P, const ChainDesc* chains, const uint32_t* list, uint32_t n,
                   const uint64_t* roff, uint32_t emit, ChainOut O, hipStream_t st);
void launch_discard(const ChainDesc* chains, const uint32_t* list, uint32_t n, const uint32_t* lisl, uint32_t* slen,
                    int2* X, const void* N16, const void* N32, const uint32_t* nshift, uint32_t* items_small,
                    uint32_t* n_small, uint32_t* items_big, uint32_t* n_big, hipStream_t st);
void launch_lis_wave(int tier, const ChainDesc* chains, const uint32_t* items, uint32_t n_items, const uint32_t* slen,
                     int2* X, void* N16, int2* pts, uint32_t* lisl, LisParams lp, int keep_idx,
                     unsigned long long* stats, hipStream_t st);
uint32_t lis_class_bounds(int which);
uint32_t lis_lane_max();
void launch_lis_lane(const ChainDesc* chains, const uint32_t* items, uint32_t n_items, const uint32_t* slen, int2* X,
                     void* N16, int2* pts, uint32_t* lisl, LisParams lp, int keep_idx, unsigned long long* stats,
                     hipStream_t st, const uint2* pinfo = nullptr);
uint32_t len_buckets();
void launch_strand_order(const ChainDesc* chains, const uint32_t* items, uint32_t n_items, const uint32_t* slen, int2* X,
                         hipStream_t st);
uint32_t big_bucket();
void launch_fine_win_sort(const Rec* recs, const uint64_t* rec_off, uint32_t n_reads, uint64_t* gscratch, uint32_t* idx,
                          hipStream_t st);
void launch_fine_sort(const uint32_t* keys, const int2* vals, const uint64_t* woff, const uint64_t* hit_off, uint32_t r0,
                      uint32_t nr, uint64_t w_sub0, uint32_t* gcount, uint32_t* okeys, int2* ovals, hipStream_t st);
void launch_fine_windows(const Rec* recs, uint32_t n, uint64_t* keys, uint32_t* idx, int phase, const uint64_t* roff,
                         uint32_t fk, FineWin* out, hipStream_t st);
void launch_fine_hits(bool emit, IndexView fx, const uint8_t* seq, const uint64_t* roff, uint32_t r0, uint32_t nr,
                      const FineWin* win, const uint64_t* woff, uint64_t* read_hits, const uint64_t* hit_off,
                      uint64_t w_sub0, uint32_t* keys, int2* vals, unsigned long long* stats, hipStream_t st);
void launch_list_bounds(const uint32_t* keys, uint64_t G, uint32_t* lstart, uint32_t* lend, hipStream_t st);
void launch_fine_desc(IndexView ix, const Rec* recs, uint64_t w_sub0, uint32_t nwin, const uint32_t* lstart,
                      const uint32_t* lend, int with_info, ChainDesc* chains, uint32_t* emit_of,
                      unsigned long long* info_need, hipStream_t st);
void launch_fine_empty(IndexView ix, uint32_t k, const ChainDesc* chains, uint32_t n, const uint32_t* lisl,
                       const uint32_t* emit_of, ChainOut O, hipStream_t st);
void launch_rec_hist(const uint32_t* rec_read, uint32_t n, uint32_t* per_read, hipStream_t st);
void launch_rec_scatter(const uint32_t* rec_read, uint32_t n, const uint64_t* rec_off, uint32_t* cursor, uint32_t* order,
                        hipStream_t st);
// order[rec_off[rec_read[i]] + rec_slot[i]] = i (the slots counted at emission)
void launch_rec_place(const uint32_t* rec_read, const uint32_t* rec_slot, uint32_t n, const uint64_t* rec_off,
                      uint32_t* order, hipStream_t st);
#ifdef PBGPU_GRAPH_CHECK
void graph_check_report();
#endif
int rec_sort_lcap();
uint64_t rec_sort_max_tiles(uint64_t nrec);
void launch_rec_sort(const Rec* recs, const uint64_t* rec_off, const uint32_t* order, uint64_t* gscratch,
                     uint32_t n_reads, uint64_t nrec, uint2* tiles, uint32_t* ctr, Rec* out, hipStream_t st);
}  // namespace pbgpu

using namespace pbgpu;

// error state, dbuf, temp_storage: pbgpu_host.h
thread_local std::string g_err;
bool stall_debug() {
  static const bool on = getenv("PBGPU_DEBUG_STALL") != nullptr;
  return on;
}
bool stall_debug_allocs() {
  static const bool on = getenv("PBGPU_DEBUG_STALL") && atoi(getenv("PBGPU_DEBUG_STALL")) >= 2;
  return on;
}
double stall_threshold_s() {
  static const double t = getenv("PBGPU_DEBUG_STALL_MS") ? atof(getenv("PBGPU_DEBUG_STALL_MS")) * 1e-3 : 0.5;
  return t;
}
void stall_report(double seconds, const char* call, const char* file, int line) {
  fprintf(stderr, "pbgpu stall: %.3f s in %s (%s:%d)\n", seconds, call, file, line);
}
void alloc_note(size_t bytes, const void* caller) {
  Dl_info di{};
  const uintptr_t base = dladdr(caller, &di) ? (uintptr_t)di.dli_fbase : 0;
  fprintf(stderr, "pbgpu alloc: %zu bytes, scale %.2f, allocs on this thread %llu, caller +0x%zx\n", bytes,
          tl_grow_scale, (unsigned long long)tl_dev_allocs, (size_t)((uintptr_t)caller - base));
}
// ------------------------------------------------------------------ names
// super_read_name::parse (super_read_name.cc:74-90) -> unitig ids + oris
static void parse_unitigs(std::string_view name, std::vector<uint32_t>& id, std::vector<uint8_t>& ori) {
  id.clear(); ori.clear();
  if (name.empty()) return;
  size_t pn = 0;
  for (;;) {
    size_t us = name.find('_', pn);
    const char* s = name.data() + pn;  // NUL-terminated (NameTable)
    char* end;
    errno = 0;
    unsigned long v = strtoul(s, &end, 10);
    if (end == s || errno == ERANGE) { id.clear(); ori.clear(); return; }
    const char oc = us != std::string_view::npos ? name[us - 1] : name[name.size() - 1];
    id.push_back((uint32_t)v & 0x7fffffffu);
    ori.push_back(oc == 'R');
    if (us == std::string::npos) break;
    pn = us + 1;
  }
}


// code of a base in the last (len % 8) bases of a line: non-ACGT keeps the
// previous code (compact_dna.hpp:108-136)
static inline uint64_t tail_code(char ch, uint64_t c) {
  switch (ch) {
  case 'a': case 'A': return 0;
  case 'c': case 'C': return 1;
  case 'g': case 'G': return 2;
  case 't': case 'T': return 3;
  default: return c;
  }
}

// host threads: the caller's count, else OMP_NUM_THREADS (the job's CPU share
// on a shared box), else every core
static int host_threads(int req) {
  if (req > 0) return req;
  if (const char* e = getenv("OMP_NUM_THREADS")) {
    const int v = atoi(e);
    if (v > 0) return v;
  }
  return (int)std::max(1u, std::thread::hardware_concurrency());
}

// host-side text accumulation with compact_dna line encoding
struct text_builder {
  std::vector<uint64_t> words;  // MSB-first
  uint64_t n = 0;
  std::vector<uint64_t> starts{0};
  NameTable names;
  int threads = 1;              // host threads for the names and the slice packer
  // Set (instead of filling `words`) by the pointer path: packs bases [b0, b0 + L)
  // of the text into `out` (L / 32 + 2 zeroed words), so that a shard packs its own
  // slice only.
  std::function<void(uint64_t b0, uint64_t L, std::vector<uint64_t>& out)> pack_slice;
  void reserve(uint64_t bases) { words.reserve(bases / 32 + 2); }
  inline void put(uint64_t code) {
    const uint64_t w = n >> 5;
    if (w >= words.size()) words.resize(std::max<size_t>(w + 1, words.size() * 2), 0);
    words[w] |= code << (62 - 2 * (n & 31));
    ++n;
  }
  // compact_dna::copy_from_str (compact_dna.hpp:89-136) on an 8-aligned line
  void add_line(const char* s, size_t len) {
    const size_t fast = len & ~(size_t)7;
    for (size_t i = 0; i < fast; ++i) {
      const unsigned b = (unsigned char)s[i];
      put(((b >> 1) ^ (b >> 2)) & 3);
    }
    uint64_t c = 0;
    for (size_t i = fast; i < len; ++i) put(c = tail_code(s[i], c));
  }
  void end_record(std::string_view header, uint64_t start) {
    if (n > start) { names.push_back(header); starts.push_back(n); }
  }
};

static void load_fasta(const char* path, text_builder& tb) {
  std::ifstream is(path);
  if (!is.good()) throw bad_input(std::string("Can't open file ") + path);
  int c = is.peek();
  if (c != '>') throw bad_input(std::string("Not in fasta format: ") + path);
  std::string line, header;
  for (; c != EOF; c = is.peek()) {
    std::getline(is, header);
    const uint64_t start = tb.n;
    for (c = is.peek(); c != '>' && c != EOF; c = is.peek()) {
      std::getline(is, line);
      tb.add_line(line.data(), line.size());
    }
    tb.end_record(std::string_view(header).substr(1), start);
  }
}

// Buckets (of 4 slots) of the k-mer table for U keys, a power of two.  Load
// <= 0.5 (slots >= 2U), so a probe sequence is short and a missed k-mer stops at
// its first bucket; but a table that would take more than 1/8 of the device
// (the 50M-super-read C5 shards: 2G k-mers, 137 GB at load <= 0.5) is sized to
// load <= 0.85 instead -- linear probing over 64-B buckets stays at ~1.1
// probes a hit there, and the presence filter keeps misses off the table.
static uint64_t table_buckets(uint64_t U) {
  uint64_t b = 1;
  while (b * 2 < U) b <<= 1;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && b * 64 > total_b / 8) {
    b = 1;
    while ((double)b * 4 * 0.85 < (double)U) b <<= 1;
  }
  return b;
}

// One sorted run of (key, value) pairs -> occurrence lists.  keys/vals hold
// M sorted pairs (spare_k / spare_v: scratch of M entries each); writes the
// lists and headers into `occ` (block-local header indices) and either inserts
// the k-mers into `table` or, with kh, returns {canon, payload} per k-mer.
struct RunsOut { uint64_t U = 0, kept = 0; };
static RunsOut lists_from_sorted(uint64_t* keys, uint64_t* vals, uint64_t* spare_k, uint64_t* spare_v, uint64_t M,
                                 uint32_t km, uint32_t ebits, hipStream_t st, dbuf<uint8_t>& tmp, dbuf<uint64_t>& occ,
                                 dbuf<ulonglong2>* table, uint64_t* n_buckets, dbuf<uint64_t>* filt, uint32_t* filt_log2,
                                 dbuf<ulonglong2>* kh) {
  const uint32_t sh = ebits + 1;  // keys >> sh = canonical km-mer
  // uidx = inclusive scan of run heads (into spare_k), kpos = exclusive scan of keep (M+1, into a new buffer)
  struct HeadOp {
    const uint64_t* keys; uint32_t sh;
    __host__ __device__ uint64_t operator()(const uint64_t& i) const {
      return (i == 0 || (keys[i] >> sh) != (keys[i - 1] >> sh)) ? 1ull : 0ull;
    }
  };
  struct KeepOp {
    const uint64_t* vals; uint64_t N;
    __host__ __device__ uint64_t operator()(const uint64_t& i) const { return (i < N && vals[i] != ~0ull) ? 1ull : 0ull; }
  };
  hipcub::CountingInputIterator<uint64_t> cnt(0);
  hipcub::TransformInputIterator<uint64_t, HeadOp, hipcub::CountingInputIterator<uint64_t>> heads(cnt, HeadOp{keys, sh});
  uint64_t* uidx = spare_k;
  size_t tbytes = 0;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tbytes, heads, uidx, M, st));
  HIPCHK(hipcub::DeviceScan::InclusiveSum(temp_storage(tmp, tbytes), tbytes, heads, uidx, M, st));
  dbuf<uint64_t> kpos;
  kpos.alloc(M + 1);
  hipcub::TransformInputIterator<uint64_t, KeepOp, hipcub::CountingInputIterator<uint64_t>> keeps(cnt, KeepOp{vals, M});
  tbytes = 0;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tbytes, keeps, kpos.p, M + 1, st));
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(temp_storage(tmp, tbytes), tbytes, keeps, kpos.p, M + 1, st));
  RunsOut o;
  HIPCHK(hipMemcpyAsync(&o.U, uidx + M - 1, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&o.kept, kpos.p + M, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const uint64_t U = o.U, kept = o.kept;
  uint64_t* run_start = spare_v;  // U + 1 <= M + 1 ... spare_v has M entries; U < M unless all distinct
  dbuf<uint64_t> rs_extra;
  if (U + 1 > M) { rs_extra.alloc(U + 1); run_start = rs_extra.p; }
  launch_runs(keys, uidx, M, sh, run_start, st);
  HIPCHK(hipMemcpyAsync(run_start + U, &M, 8, hipMemcpyHostToDevice, st));
  occ.alloc(2 * U + kept + 2);  // + an empty header {0, 0} at 2U + kept (the whole index's null_ptr)
  HIPCHK(hipMemsetAsync(occ.p + 2 * U + kept, 0, 16, st));
  launch_occ_fill(vals, uidx, kpos.p, M, occ.p, st);
  ulonglong2* tp = nullptr;
  uint64_t buckets = 1;
  uint64_t* fp = nullptr;
  uint32_t flog = 0;
  if (table) {
    buckets = table_buckets(U);
    *n_buckets = buckets;
    table->alloc(4 * buckets);
    HIPCHK(hipMemsetAsync(table->p, 0xFF, table->bytes(), st));
    tp = table->p;
    // presence filter: PBGPU_FILTER_BITS bits per k-mer (default 16, 0 = none), a power of two of words
    if (filt) {
      const char* e = getenv("PBGPU_FILTER_BITS");
      const uint64_t bits = e ? strtoull(e, nullptr, 10) : 16;
      if (bits) {
        flog = 6;  // >= 64 words
        while ((1ull << flog) < U * bits / 64) ++flog;
        filt->alloc(1ull << flog);
        HIPCHK(hipMemsetAsync(filt->p, 0, filt->bytes(), st));
        fp = filt->p;
        *filt_log2 = flog;
      }
    }
  } else {
    kh->alloc(U + 1);
  }
  launch_headers(keys, kpos.p, run_start, U, occ.p, tp, buckets - 1, km, ebits, fp, 64 - flog, kh ? kh->p : nullptr, st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));  // the temporaries above are freed on return
  return o;
}

// Hash table + occurrence lists of the km-mers of the text (layout in
// pbgpu_internal.h): sort keys (k_build_keys) -> radix sort -> runs of equal
// canonical km-mer -> occurrence lists and headers -> table.  ebits > 0
// orders each list by the K - km bases that follow (the fine sub-index).
// A text whose sort buffers (~48 B a position) do not fit beside the index is
// built in P partitions by hash of the canonical km-mer (all occurrences of a
// km-mer in one partition): each partition is selected in enumeration order
// (stable), sorted and turned into its own occurrence block and k-mer list;
// the blocks are then laid end to end and the k-mers inserted into one table.
// PBGPU_BUILD_PARTS forces P (tests).
static void build_kmer_table(pbgpu_index* ix, uint32_t km, uint32_t K, uint32_t ebits, hipStream_t st,
                             dbuf<ulonglong2>& table, dbuf<uint64_t>& occ, uint64_t& n_buckets, uint64_t& n_kmers,
                             uint64_t& n_occ, dbuf<uint64_t>* filt = nullptr, uint32_t* filt_log2 = nullptr) {
  const uint64_t N = ix->n >= km ? ix->n - km + 1 : 0;
  IndexView v = ix->view();
  if (N == 0) {
    n_buckets = 1;
    table.alloc(4);
    HIPCHK(hipMemset(table.p, 0xFF, table.bytes()));
    occ.alloc(2);
    HIPCHK(hipMemset(occ.p, 0, occ.bytes()));  // the empty header (ix->null_ptr = 0)
    n_kmers = n_occ = 0;
    return;
  }
  const int key_bits = (int)(2 * km + 1 + ebits);
  uint32_t P = 1;
  if (const char* e = getenv("PBGPU_BUILD_PARTS")) {
    P = (uint32_t)std::max(1l, std::min(255l, strtol(e, nullptr, 10)));
  } else {
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    // one pass: 4 sort arrays + scan + lists ~56 B a position; partitioned: ~48 B a
    // partition position + the finished blocks (~9 B a position) + their k-mer
    // lists (16 B a k-mer, ~8 B a position at C4/C5 coverage) + 1 B of partition ids
    if (56.0 * N > 0.8 * (double)free_b || N >= (1ull << 31)) {
      P = 2;
      while (P < 255 && (48.0 * N / P + 18.0 * N > 0.8 * (double)free_b || N / P >= (1ull << 31))) P *= 2;
      if (P > 255) P = 255;
    }
  }
  if (P == 1) {
    dbuf<uint64_t> k0, k1, v0, v1;
    k0.alloc(N); k1.alloc(N); v0.alloc(N); v1.alloc(N);
    launch_build_keys(v, km, K, ebits, N, nullptr, N, k0.p, v0.p, st);
    HIPCHK(hipGetLastError());
    dbuf<uint8_t> tmp;
    size_t tbytes = 0;
    hipcub::DoubleBuffer<uint64_t> dk(k0.p, k1.p), dv(v0.p, v1.p);
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tbytes, dk, dv, N, 0, key_bits, st));
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(temp_storage(tmp, tbytes), tbytes, dk, dv, N, 0, key_bits, st));
    const RunsOut o = lists_from_sorted(dk.Current(), dv.Current(), dk.Alternate(), dv.Alternate(), N, km, ebits, st,
                                        tmp, occ, &table, &n_buckets, filt, filt_log2, nullptr);
    n_kmers = o.U;
    n_occ = o.kept;
    return;
  }
  // ---- partitioned build
  std::vector<uint64_t> Np(P);
  dbuf<uint8_t> pid, tmp;
  pid.alloc(N);
  {
    dbuf<unsigned long long> hist;
    hist.alloc(P);
    HIPCHK(hipMemsetAsync(hist.p, 0, P * 8, st));
    launch_part_ids(v, km, N, P, pid.p, hist.p, st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(Np.data(), hist.p, P * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  const uint64_t maxNp = std::max<uint64_t>(1, *std::max_element(Np.begin(), Np.end()));
  std::vector<dbuf<uint64_t>> blocks(P);
  std::vector<dbuf<ulonglong2>> khs(P);
  std::vector<RunsOut> ro(P);
  {
    dbuf<uint64_t> sel, k0, k1, v0, v1, nsel;
    sel.alloc(maxNp); k0.alloc(maxNp); k1.alloc(maxNp); v0.alloc(maxNp); v1.alloc(maxNp); nsel.alloc(1);
    struct PidSel {
      const uint8_t* pid; uint8_t p;
      __host__ __device__ bool operator()(const uint64_t& i) const { return pid[i] == p; }
    };
    for (uint32_t p = 0; p < P; ++p) {
      // stable selection of the partition's enumeration indices, in chunks of < 2^31 items
      uint64_t got = 0;
      for (uint64_t c0 = 0; c0 < N; c0 += (1ull << 30)) {
        const int cn = (int)std::min<uint64_t>(N - c0, 1ull << 30);
        hipcub::CountingInputIterator<uint64_t> it(c0);
        size_t tb = 0;
        HIPCHK(hipcub::DeviceSelect::If(nullptr, tb, it, sel.p + got, nsel.p, cn, PidSel{pid.p, (uint8_t)p}, st));
        HIPCHK(hipcub::DeviceSelect::If(temp_storage(tmp, tb), tb, it, sel.p + got, nsel.p, cn,
                                        PidSel{pid.p, (uint8_t)p}, st));
        uint64_t ns = 0;
        HIPCHK(hipMemcpyAsync(&ns, nsel.p, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        got += ns & 0xFFFFFFFFull;  // DeviceSelect writes the count as its offset type (int / uint32)
      }
      if (got != Np[p]) throw std::runtime_error("partitioned index build: selection count mismatch");
      const uint64_t M = Np[p];
      if (M == 0) {
        blocks[p].alloc(1);
        ro[p] = RunsOut{};
        continue;
      }
      launch_build_keys(v, km, K, ebits, N, sel.p, M, k0.p, v0.p, st);
      HIPCHK(hipGetLastError());
      size_t tbytes = 0;
      hipcub::DoubleBuffer<uint64_t> dk(k0.p, k1.p), dv(v0.p, v1.p);
      HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tbytes, dk, dv, M, 0, key_bits, st));
      HIPCHK(hipcub::DeviceRadixSort::SortPairs(temp_storage(tmp, tbytes), tbytes, dk, dv, M, 0, key_bits, st));
      ro[p] = lists_from_sorted(dk.Current(), dv.Current(), dk.Alternate(), dv.Alternate(), M, km, ebits, st, tmp,
                                blocks[p], nullptr, nullptr, nullptr, nullptr, &khs[p]);
    }
  }
  pid.release();
  tmp.release();
  uint64_t U = 0, kept = 0;
  for (uint32_t p = 0; p < P; ++p) { U += ro[p].U; kept += ro[p].kept; }
  // The blocks are laid end to end into one array.  When the array does not fit
  // beside them, they wait in host memory instead (one copy out and back).
  std::vector<std::vector<uint64_t>> staged;
  {
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    if ((2 * U + kept + 2) * 8.0 > 0.9 * (double)free_b) {
      staged.resize(P);
      for (uint32_t p = 0; p < P; ++p) {
        const uint64_t len = 2 * ro[p].U + ro[p].kept;
        staged[p].resize(len);
        if (len) HIPCHK(hipMemcpy(staged[p].data(), blocks[p].p, len * 8, hipMemcpyDeviceToHost));
        blocks[p].release();
      }
    }
  }
  occ.alloc(2 * U + kept + 2);
  HIPCHK(hipMemsetAsync(occ.p + 2 * U + kept, 0, 16, st));  // the null header
  std::vector<uint64_t> base(P);
  uint64_t b = 0;
  for (uint32_t p = 0; p < P; ++p) {
    base[p] = b;
    const uint64_t len = 2 * ro[p].U + ro[p].kept;
    if (len && staged.empty()) HIPCHK(hipMemcpyAsync(occ.p + b, blocks[p].p, len * 8, hipMemcpyDeviceToDevice, st));
    if (len && !staged.empty()) {
      HIPCHK(hipMemcpy(occ.p + b, staged[p].data(), len * 8, hipMemcpyHostToDevice));
      std::vector<uint64_t>().swap(staged[p]);
    }
    HIPCHK(hipStreamSynchronize(st));
    blocks[p].release();
    b += len;
  }
  const uint64_t buckets = table_buckets(U);
  n_buckets = buckets;
  table.alloc(4 * buckets);
  HIPCHK(hipMemsetAsync(table.p, 0xFF, table.bytes(), st));
  uint64_t* fp = nullptr;
  uint32_t flog = 0;
  if (filt) {
    const char* e = getenv("PBGPU_FILTER_BITS");
    const uint64_t bits = e ? strtoull(e, nullptr, 10) : 16;
    if (bits) {
      flog = 6;
      while ((1ull << flog) < U * bits / 64) ++flog;
      filt->alloc(1ull << flog);
      HIPCHK(hipMemsetAsync(filt->p, 0, filt->bytes(), st));
      fp = filt->p;
      *filt_log2 = flog;
    }
  }
  for (uint32_t p = 0; p < P; ++p) {
    if (ro[p].U) launch_table_insert(khs[p].p, ro[p].U, base[p], table.p, buckets - 1, fp, 64 - flog, st);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipStreamSynchronize(st));
  n_kmers = U;
  n_occ = kept;
}

// IndexView::occ_sr, when PBGPU_OCC_SR=1 (4 B per occ word): derived, never cached
static void make_occ_sr(pbgpu_index* ix, hipStream_t st) {
  const char* e = getenv("PBGPU_OCC_SR");
  if (!e || atoi(e) == 0 || !ix->occ.n) return;
  ix->occ_sr.alloc(ix->occ.n);
  launch_occ_sr(ix->occ.p, ix->occ.n, ix->occ_sr.p, st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
}

static void build_device_index(pbgpu_index* ix, text_builder& tb) {
  auto t0 = std::chrono::steady_clock::now();
  HIPCHK(hipSetDevice(ix->device));
  hipStream_t st;
  HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct stream_guard { hipStream_t s; ~stream_guard() { (void)hipStreamDestroy(s); } } sg{st};
  const uint32_t k = ix->k;
  ix->n_total = tb.n;
  ix->n_sr = tb.names.size();
  ix->gstart = tb.starts;
  // names, bwd names (frag_info.hpp:22-35), unitig ids -- of every super-read (host)
  ix->name_fwd = std::move(tb.names);
  // unitig ids and reversed names (frag_info.hpp:22-35), in parallel over ranges of
  // super-reads (50M names at C5): each range builds its own id list and name blob,
  // then the ranges are laid end to end
  std::vector<uint32_t> uoff(ix->n_sr + 1, 0), uids;
  {
    const uint64_t nsr = ix->n_sr, nparts = std::max<uint64_t>(1, std::min<uint64_t>(nsr, (uint64_t)tb.threads * 8));
    std::vector<std::vector<uint32_t>> pids(nparts);
    std::vector<std::vector<char>> pblob(nparts);
    std::vector<uint64_t>& boff = ix->name_bwd.off;
    boff.assign(nsr + 1, 0);
    std::atomic<uint64_t> next(0);
    run_parallel(tb.threads, [&]() {
      std::vector<uint32_t> id;
      std::vector<uint8_t> ori;
      char num[16];
      for (uint64_t q; (q = next.fetch_add(1)) < nparts;) {
        std::vector<char>& b = pblob[q];
        for (uint64_t i = nsr * q / nparts; i < nsr * (q + 1) / nparts; ++i) {
          const std::string_view fw = ix->name_fwd[i];
          parse_unitigs(fw, id, ori);
          uoff[i] = (uint32_t)id.size();  // count; offsets below
          pids[q].insert(pids[q].end(), id.begin(), id.end());
          const size_t b0 = b.size();
          if (!id.empty()) {
            for (size_t t = 0; t < id.size(); ++t) {
              const size_t s = id.size() - 1 - t;
              if (t) b.push_back('_');
              const int w = snprintf(num, sizeof num, "%u", id[s]);
              b.insert(b.end(), num, num + w);
              b.push_back(ori[s] ? 'F' : 'R');
            }
          } else {
            b.insert(b.end(), fw.begin(), fw.end());
          }
          b.push_back(0);
          boff[i + 1] = b.size() - b0;  // length + NUL; offsets below
        }
      }
    });
    uint64_t tot = 0;
    for (uint64_t i = 0; i < nsr; ++i) { const uint32_t c = uoff[i]; uoff[i] = (uint32_t)tot; tot += c; }
    if (tot >= (1ull << 32)) throw bad_input("more than 2^32 unitig ids in the super-read names");
    uoff[nsr] = (uint32_t)tot;
    uids.reserve(tot);
    for (auto& v : pids) { uids.insert(uids.end(), v.begin(), v.end()); std::vector<uint32_t>().swap(v); }
    for (uint64_t i = 0; i < nsr; ++i) boff[i + 1] += boff[i];
    ix->name_bwd.blob.resize(boff[nsr]);
    std::vector<uint64_t> pstart(nparts + 1, 0);
    for (uint64_t q = 0; q < nparts; ++q) pstart[q + 1] = pstart[q] + pblob[q].size();
    next = 0;
    run_parallel(tb.threads, [&]() {
      for (uint64_t q; (q = next.fetch_add(1)) < nparts;) {
        if (!pblob[q].empty()) memcpy(ix->name_bwd.blob.data() + pstart[q], pblob[q].data(), pblob[q].size());
        std::vector<char>().swap(pblob[q]);
      }
    });
  }
  if (!tb.pack_slice) tb.words.resize(tb.n / 32 + 2, 0);
  // This device's super-reads: all of them, or shard `shard` of n_shards -- the
  // super-reads starting in [total * s / S, total * (s + 1) / S) of the text --
  // plus the next k - 1 bases (the seam), so that an occurrence crossing into the
  // next shard is counted here, once.
  const uint64_t total = tb.n;
  auto first_sr_at = [&](uint64_t b) -> uint64_t {  // first super-read starting at or after base b
    return (uint64_t)(std::lower_bound(ix->gstart.begin(), ix->gstart.end() - 1, b) - ix->gstart.begin());
  };
  ix->sr_begin = ix->n_shards > 1 ? first_sr_at(total * ix->shard / ix->n_shards) : 0;
  ix->sr_end = ix->n_shards > 1 && ix->shard + 1 < ix->n_shards ? first_sr_at(total * (ix->shard + 1) / ix->n_shards)
                                                                  : ix->n_sr;
  const uint64_t b0 = ix->gstart[ix->sr_begin], b1 = ix->gstart[ix->sr_end];
  const uint64_t seam = std::min<uint64_t>(k - 1, total - b1);
  const uint64_t L = b1 - b0 + seam;
  ix->n = L;
  std::vector<uint64_t> words;
  if (tb.pack_slice) {
    words.assign(L / 32 + 2, 0);
    tb.pack_slice(b0, L, words);
  } else if (b0 == 0 && b1 + seam == total) {
    words.swap(tb.words);
  } else {  // re-align the slice [b0, b0 + L) of the packed text to base 0
    const uint64_t W = tb.words.size(), j0 = b0 >> 5;
    const uint32_t sh = (uint32_t)(b0 & 31) * 2;
    words.assign(L / 32 + 2, 0);
    for (uint64_t i = 0; i < words.size(); ++i) {
      const uint64_t a = j0 + i < W ? tb.words[j0 + i] : 0, c = j0 + i + 1 < W ? tb.words[j0 + i + 1] : 0;
      words[i] = sh ? (a << sh) | (c >> (64 - sh)) : a;
    }
    if (L & 31) words[L >> 5] &= ~0ull << (64 - 2 * (L & 31));
    for (uint64_t i = (L >> 5) + 1; i < words.size(); ++i) words[i] = 0;
    std::vector<uint64_t>().swap(tb.words);
  }
  ix->text.alloc(words.size());
  HIPCHK(hipMemcpy(ix->text.p, words.data(), words.size() * 8, hipMemcpyHostToDevice));
  std::vector<uint64_t>().swap(words);
  const uint64_t nloc = ix->sr_end - ix->sr_begin;
  ix->sr_start.resize(nloc + 1);
  for (uint64_t i = 0; i <= nloc; ++i) ix->sr_start[i] = ix->gstart[ix->sr_begin + i] - b0;
  ix->d_sr_start.alloc(ix->sr_start.size());
  HIPCHK(hipMemcpy(ix->d_sr_start.p, ix->sr_start.data(), ix->sr_start.size() * 8, hipMemcpyHostToDevice));
  std::vector<uint32_t> luoff(nloc + 1);
  for (uint64_t i = 0; i <= nloc; ++i) luoff[i] = uoff[ix->sr_begin + i] - uoff[ix->sr_begin];
  ix->sr_uoff.alloc(luoff.size());
  HIPCHK(hipMemcpy(ix->sr_uoff.p, luoff.data(), luoff.size() * 4, hipMemcpyHostToDevice));
  ix->sr_uids.alloc(std::max<size_t>(luoff[nloc], 1));
  if (luoff[nloc])
    HIPCHK(hipMemcpy(ix->sr_uids.p, uids.data() + uoff[ix->sr_begin], (size_t)luoff[nloc] * 4, hipMemcpyHostToDevice));

  build_kmer_table(ix, k, k, 0, st, ix->table, ix->occ, ix->buckets, ix->n_kmers, ix->n_occ, &ix->filt,
                   &ix->filt_log2);
  ix->null_ptr = 2 * ix->n_kmers + ix->n_occ;
  make_occ_sr(ix, st);
  if (ix->fk)
    build_kmer_table(ix, ix->fk, k, 2 * (k - ix->fk) + 1, st, ix->f_table, ix->f_occv, ix->f_buckets, ix->f_kmers,
                     ix->f_occ);
  HIPCHK(hipStreamSynchronize(st));
  ix->build_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

static pbgpu_status index_common(const pbgpu_index_params* p) {
  if (!p) return fail(PBGPU_ERR_INVALID, "null params");
  if (p->k < 2 || p->k > 31) return fail(PBGPU_ERR_UNSUPPORTED, "k=%u outside [2,31]", p->k);
  if (p->fine_k > p->k)
    return fail(PBGPU_ERR_UNSUPPORTED, "fine_k (%u) > k (%u): PSA::search assumes the pattern is at most max_size "
                "(mer_sa_imp.hpp:366)", p->fine_k, p->k);
  if (p->psa_min >= p->k)
    return fail(PBGPU_ERR_UNSUPPORTED,
                "psa_min (%u) >= k (%u): the reference's hit order then depends on thread timing (mer_sa_imp.hpp:247)",
                p->psa_min, p->k);
  if (p->n_shards > 1 && p->shard >= p->n_shards)
    return fail(PBGPU_ERR_INVALID, "shard %u out of range (n_shards %u)", p->shard, p->n_shards);
  if (p->n_shards > 1 && p->fine_k)
    return fail(PBGPU_ERR_UNSUPPORTED, "the fine aligner (-F) runs on a whole index only (n_shards = 1)");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PBGPU_ERR_DEVICE, "no HIP device available");
  if (p->device < 0 || p->device >= ndev) return fail(PBGPU_ERR_INVALID, "device %d out of range", p->device);
  return PBGPU_OK;
}

extern "C" {

int pbgpu_abi_version(void) { return PBGPU_ABI_VERSION; }
const char* pbgpu_last_error(void) { return g_err.c_str(); }
int pbgpu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

pbgpu_status pbgpu_device_synchronize(int device) {
  API_TRY
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipDeviceSynchronize());
  return PBGPU_OK;
  API_CATCH
}

// Random 64-B sector gather over a large buffer: SURVEY 8(d)'s B_rand, the
// roofline of the index probes and occurrence-list reads.  Four lanes load one
// sector (16 B each); every lane keeps UNR sectors in flight.
namespace {
constexpr int GATHER_UNR = 8;
__global__ __launch_bounds__(256) void k_gather_sectors(const uint4* __restrict__ buf, uint64_t n_sectors,
                                                        uint32_t iters, uint32_t seed, uint4* __restrict__ sink) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t grp = gid >> 2;
  const uint32_t part = threadIdx.x & 3;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint32_t it = 0; it < iters; ++it) {
    uint4 v[GATHER_UNR];
#pragma unroll
    for (int u = 0; u < GATHER_UNR; ++u) {
      uint64_t h = (grp * GATHER_UNR + u) * 0x9E3779B97F4A7C15ull + ((uint64_t)(it + 1) * seed);
      h ^= h >> 31; h *= 0xD6E8FEB86659FD93ull; h ^= h >> 32;
      v[u] = buf[(h % n_sectors) * 4 + part];
    }
#pragma unroll
    for (int u = 0; u < GATHER_UNR; ++u) { acc.x ^= v[u].x; acc.y ^= v[u].y; acc.z ^= v[u].z; acc.w ^= v[u].w; }
  }
  if ((acc.x & 0xFFFFF) == 0x12345) sink[gid & 1023] = acc;  // keeps the loads live, practically never stores
}
// Runs of 64 x 8 B (one 512-B contiguous run per wave-instruction, 8-B-aligned
// words, 64-B-aligned runs): the access shape of k_group's occurrence-list reads
// (a k-mer's occurrences are consecutive 8-B entries).  Calibrates FETCH_SIZE
// for that shape and gives its achievable rate.
__global__ __launch_bounds__(256) void k_gather_runs(const uint2* __restrict__ buf, uint64_t n_runs, uint32_t iters,
                                                     uint32_t seed, uint2* __restrict__ sink) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t wv = gid >> 6;
  const uint32_t lane = threadIdx.x & 63;
  uint2 acc = make_uint2(0, 0);
  for (uint32_t it = 0; it < iters; ++it) {
    uint2 v[GATHER_UNR];
#pragma unroll
    for (int u = 0; u < GATHER_UNR; ++u) {
      uint64_t h = (wv * GATHER_UNR + u) * 0x9E3779B97F4A7C15ull + ((uint64_t)(it + 1) * seed);
      h ^= h >> 31; h *= 0xD6E8FEB86659FD93ull; h ^= h >> 32;
      v[u] = buf[(h % n_runs) * 64 + lane];
    }
#pragma unroll
    for (int u = 0; u < GATHER_UNR; ++u) { acc.x ^= v[u].x; acc.y ^= v[u].y; }
  }
  if ((acc.x & 0xFFFFF) == 0x12345) sink[gid & 1023] = acc;
}
// The exact access shape of k_group's occurrence reads (round 6, to calibrate FETCH_SIZE
// for it): a wave takes RUNS runs of GG_RUN consecutive 8-B words at random 8-B-aligned
// starts (a k-mer's occurrence list; C2's mean is ~52), lanes 0..GG_RUN-1 one word each.
// MODE 0: k_group's pass 0 alone -- the 4-B super-read id, the high half of each word
// (stride 8 B); MODE 1: pass 1 alone -- the whole 8-B word; MODE 2: both, as k_group
// runs them, all of a wave's runs in pass 0 and then all of them again in pass 1 (a
// wave's RUNS runs, ~416 KB, stand for one read's lists: with every wave of the chip in
// flight the second reads find nothing of the first in L2 or the Infinity Cache).
// The wave counts the 64-B sectors and 128-B lines its runs span (sec[0], sec[1], each
// pass counted) so FETCH_SIZE can be read against a known byte count.
constexpr uint32_t GG_RUN = 52, GG_RUNS = 1024, GG_UNR = 8;
extern "C++" {
template <int MODE>
__global__ __launch_bounds__(256) void k_gather_group(const uint2* __restrict__ buf, uint64_t n_words, uint32_t seed,
                                                      unsigned long long* __restrict__ sec, uint2* __restrict__ sink) {
  const uint64_t wv = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  const bool on = lane < GG_RUN;
  const uint64_t span = n_words - GG_RUN;
  auto start = [&](uint32_t r) -> uint64_t {
    uint64_t h = (wv * GG_RUNS + r) * 0x9E3779B97F4A7C15ull + (uint64_t)seed * 0xBF58476D1CE4E5B9ull;
    h ^= h >> 31; h *= 0xD6E8FEB86659FD93ull; h ^= h >> 32;
    return h % span;
  };
  const uint32_t* w32 = reinterpret_cast<const uint32_t*>(buf);
  uint32_t acc = 0;
  unsigned long long s64 = 0, l128 = 0;
  for (int pass = (MODE == 1 ? 1 : 0); pass <= (MODE == 0 ? 0 : 1); ++pass) {
    for (uint32_t r0 = 0; r0 < GG_RUNS; r0 += GG_UNR) {
      uint32_t v[GG_UNR];
#pragma unroll
      for (uint32_t u = 0; u < GG_UNR; ++u) {
        const uint64_t w = start(r0 + u) + (on ? lane : 0);
        if (pass == 0) {
          v[u] = w32[2 * w + 1];
        } else {
          const uint2 x = buf[w];
          v[u] = x.x ^ x.y;
        }
      }
#pragma unroll
      for (uint32_t u = 0; u < GG_UNR; ++u) acc ^= on ? v[u] : 0u;
      if (lane == 0) {
#pragma unroll
        for (uint32_t u = 0; u < GG_UNR; ++u) {
          const uint64_t b0 = start(r0 + u) * 8, b1 = b0 + GG_RUN * 8 - 1;
          s64 += (b1 >> 6) - (b0 >> 6) + 1;
          l128 += (b1 >> 7) - (b0 >> 7) + 1;
        }
      }
    }
  }
  if (lane == 0) { atomicAdd(&sec[0], s64); atomicAdd(&sec[1], l128); }
  if ((acc & 0xFFFFF) == 0x12345) sink[(wv * 64 + lane) & 1023] = make_uint2(acc, 0);
}
}  // extern "C++"
}  // namespace

pbgpu_status pbgpu_measure_group_shape(int device, uint64_t buffer_bytes, int mode, double* gbps, uint64_t* sectors64,
                                       uint64_t* lines128, uint64_t* alg_bytes) {
  if (!gbps || buffer_bytes < (64u << 20) || mode < 0 || mode > 2) return fail(PBGPU_ERR_INVALID, "bad argument");
  API_TRY
  HIPCHK(hipSetDevice(device));
  dbuf<uint2> buf, sink;
  dbuf<unsigned long long> sec;
  const uint64_t n_words = buffer_bytes / 8;
  buf.ensure_fixed(n_words);
  HIPCHK(hipMemset(buf.p, 0x5A, n_words * 8));
  sink.ensure_fixed(1024);
  sec.ensure_fixed(2);
  hipDeviceProp_t pr;
  HIPCHK(hipGetDeviceProperties(&pr, device));
  const uint32_t blocks = (uint32_t)pr.multiProcessorCount * 8;
  hipStream_t st;
  HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0)); HIPCHK(hipEventCreate(&e1));
  auto launch = [&](uint32_t seed) {
    if (mode == 0)
      hipLaunchKernelGGL(k_gather_group<0>, dim3(blocks), dim3(256), 0, st, buf.p, n_words, seed, sec.p, sink.p);
    else if (mode == 1)
      hipLaunchKernelGGL(k_gather_group<1>, dim3(blocks), dim3(256), 0, st, buf.p, n_words, seed, sec.p, sink.p);
    else
      hipLaunchKernelGGL(k_gather_group<2>, dim3(blocks), dim3(256), 0, st, buf.p, n_words, seed, sec.p, sink.p);
  };
  launch(3u);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemsetAsync(sec.p, 0, 16, st));
  HIPCHK(hipEventRecord(e0, st));
  const int reps = 3;
  for (int r = 0; r < reps; ++r) launch(5u + 2u * r);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(e1, st));
  HIPCHK(hipEventSynchronize(e1));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[2];
  HIPCHK(hipMemcpy(h, sec.p, 16, hipMemcpyDeviceToHost));
  const double runs = (double)blocks * 4 * GG_RUNS * (mode == 2 ? 2 : 1);  // run reads per launch
  const double alg = (double)blocks * 4 * GG_RUNS * GG_RUN * (mode == 0 ? 4.0 : mode == 1 ? 8.0 : 12.0);
  (void)runs;
  // per launch: the sectors / lines the runs span, and the algorithmic bytes (4 B a word in
  // pass 0, 8 B in pass 1); the rate is the 64-B-sector bytes moved per second
  if (sectors64) *sectors64 = h[0] / reps;
  if (lines128) *lines128 = h[1] / reps;
  if (alg_bytes) *alg_bytes = (uint64_t)alg;
  *gbps = (double)h[0] * 64.0 / (ms * 1e-3) / 1e9;
  (void)hipEventDestroy(e0); (void)hipEventDestroy(e1); (void)hipStreamDestroy(st);
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_measure_gather(int device, uint64_t buffer_bytes, double* gbps) {
  return pbgpu_measure_gather_shape(device, buffer_bytes, 64, gbps);
}

pbgpu_status pbgpu_check_reciprocal(int device, uint32_t n_max, uint64_t* mismatches) {
  if (!mismatches || n_max == 0) return fail(PBGPU_ERR_INVALID, "bad argument");
  API_TRY
  HIPCHK(hipSetDevice(device));
  dbuf<unsigned long long> bad;
  bad.ensure_fixed(1);
  HIPCHK(hipMemset(bad.p, 0, 8));
  launch_check_recip(n_max, bad.p, nullptr);
  HIPCHK(hipGetLastError());
  unsigned long long nb = 0;
  HIPCHK(hipMemcpy(&nb, bad.p, 8, hipMemcpyDeviceToHost));
  *mismatches = nb;
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_measure_gather_shape(int device, uint64_t buffer_bytes, uint32_t unit_bytes, double* gbps) {
  if (!gbps || buffer_bytes < (1u << 20) || (unit_bytes != 64 && unit_bytes != 512))
    return fail(PBGPU_ERR_INVALID, "bad argument");
  API_TRY
  HIPCHK(hipSetDevice(device));
  dbuf<uint4> buf, sink;
  const uint64_t n_units = buffer_bytes / unit_bytes;
  buf.ensure(n_units * unit_bytes / 16);
  sink.ensure(1024);
  hipDeviceProp_t pr;
  HIPCHK(hipGetDeviceProperties(&pr, device));
  const uint32_t blocks = (uint32_t)pr.multiProcessorCount * 8, iters = 64;
  hipStream_t st;
  HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0)); HIPCHK(hipEventCreate(&e1));
  auto launch = [&](uint32_t seed) {
    if (unit_bytes == 64)
      hipLaunchKernelGGL(k_gather_sectors, dim3(blocks), dim3(256), 0, st, buf.p, n_units, iters, seed, sink.p);
    else
      hipLaunchKernelGGL(k_gather_runs, dim3(blocks), dim3(256), 0, st, (const uint2*)buf.p, n_units, iters, seed,
                         (uint2*)sink.p);
  };
  launch(7u);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(e0, st));
  const int reps = 3;
  for (int r = 0; r < reps; ++r) launch(11u + 2u * r);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(e1, st));
  HIPCHK(hipEventSynchronize(e1));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  // bytes moved: sectors: 4 lanes x 16 B per 64-B sector; runs: 64 lanes x 8 B per 512-B run
  const double units_per_launch = unit_bytes == 64 ? (double)blocks * 256 / 4 * GATHER_UNR * iters
                                                   : (double)blocks * 256 / 64 * GATHER_UNR * iters;
  const double bytes = (double)reps * units_per_launch * unit_bytes;
  *gbps = bytes / (ms * 1e-3) / 1e9;
  (void)hipEventDestroy(e0); (void)hipEventDestroy(e1); (void)hipStreamDestroy(st);
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_index_build_fasta(const char* const* paths, size_t n_paths, const pbgpu_index_params* params,
                                     pbgpu_index** out) {
  if (!out || (!paths && n_paths)) return fail(PBGPU_ERR_INVALID, "null argument");
  pbgpu_status s = index_common(params);
  if (s != PBGPU_OK) return s;
  API_TRY
  text_builder tb;
  tb.threads = host_threads(params->threads);
  for (size_t i = 0; i < n_paths; ++i) load_fasta(paths[i], tb);
  std::unique_ptr<pbgpu_index> ix(new pbgpu_index);
  ix->device = params->device; ix->k = params->k; ix->psa_min = params->psa_min; ix->fk = params->fine_k;
  if (params->n_shards > 1) { ix->shard = params->shard; ix->n_shards = params->n_shards; }
  build_device_index(ix.get(), tb);
  *out = ix.release();
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_index_build(const char* const* names, const char* const* seqs, const uint64_t* lens, size_t n,
                               const pbgpu_index_params* params, pbgpu_index** out) {
  if (!out || (n && (!names || !seqs || !lens))) return fail(PBGPU_ERR_INVALID, "null argument");
  pbgpu_status s = index_common(params);
  if (s != PBGPU_OK) return s;
  API_TRY
  text_builder tb;
  tb.threads = host_threads(params->threads);
  // every non-empty record is a super-read (end_record); the text is packed per
  // slice by build_device_index, in parallel, each super-read one compact_dna line
  std::vector<uint64_t> rec;  // record of each super-read
  for (size_t i = 0; i < n; ++i)
    if (lens[i]) { rec.push_back(i); tb.starts.push_back(tb.starts.back() + lens[i]); }
  tb.n = tb.starts.back();
  {  // the names into one blob: lengths, offsets, then parallel copies
    const uint64_t nr = rec.size(), chunk = 1 << 16;
    std::vector<uint64_t>& no = tb.names.off;
    no.assign(nr + 1, 0);
    std::atomic<uint64_t> next(0);
    run_parallel(tb.threads, [&]() {
      for (uint64_t c; (c = next.fetch_add(chunk)) < nr;)
        for (uint64_t i = c; i < std::min(nr, c + chunk); ++i) no[i + 1] = strlen(names[rec[i]]) + 1;
    });
    for (uint64_t i = 0; i < nr; ++i) no[i + 1] += no[i];
    tb.names.blob.resize(no[nr]);
    next = 0;
    run_parallel(tb.threads, [&]() {
      for (uint64_t c; (c = next.fetch_add(chunk)) < nr;)
        for (uint64_t i = c; i < std::min(nr, c + chunk); ++i)
          memcpy(tb.names.blob.data() + no[i], names[rec[i]], no[i + 1] - no[i]);
    });
  }
  const std::vector<uint64_t>& gs = tb.starts;
  const int T = tb.threads;
  tb.pack_slice = [&, T](uint64_t b0, uint64_t L, std::vector<uint64_t>& out) {
    const uint64_t nw = (L + 31) / 32, chunk = 1 << 16;  // words per task (2 Mbases)
    std::atomic<uint64_t> next(0);
    run_parallel(T, [&]() {
      for (uint64_t w0; (w0 = next.fetch_add(chunk)) < nw;) {
        const uint64_t lo = w0 * 32, hi = std::min(L, (w0 + chunk) * 32);  // slice-local bases
        uint64_t i = (uint64_t)(std::upper_bound(gs.begin(), gs.end(), b0 + lo) - gs.begin()) - 1;
        for (uint64_t pos = lo; pos < hi; ++i) {
          const char* sq = seqs[rec[i]];
          const uint64_t len = lens[rec[i]], j0 = b0 + pos - gs[i];
          const uint64_t j1 = std::min(len, j0 + (hi - pos));
          const uint64_t fast = len & ~(uint64_t)7;
          // compact_dna::copy_from_str (compact_dna.hpp:89-136), the line being the record:
          // 8-aligned part by the bit trick, the tail keeping the last code over non-ACGT
          uint64_t c = 0;
          for (uint64_t j = fast; j < std::min(j0, len); ++j) c = tail_code(sq[j], c);
          for (uint64_t j = j0; j < j1; ++j, ++pos) {
            uint64_t code;
            if (j < fast) {
              const unsigned b = (unsigned char)sq[j];
              code = ((b >> 1) ^ (b >> 2)) & 3;
            } else {
              code = c = tail_code(sq[j], c);
            }
            out[pos >> 5] |= code << (62 - 2 * (pos & 31));
          }
        }
      }
    });
  };
  std::unique_ptr<pbgpu_index> ix(new pbgpu_index);
  ix->device = params->device; ix->k = params->k; ix->psa_min = params->psa_min; ix->fk = params->fine_k;
  if (params->n_shards > 1) { ix->shard = params->shard; ix->n_shards = params->n_shards; }
  build_device_index(ix.get(), tb);
  *out = ix.release();
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_index_free(pbgpu_index* ix) {
  if (!ix) return PBGPU_OK;
  (void)hipSetDevice(ix->device);
  delete ix;
  return PBGPU_OK;
}

pbgpu_status pbgpu_index_replicate(const pbgpu_index* src, int device, pbgpu_index** out) {
  if (!src || !out) return fail(PBGPU_ERR_INVALID, "null argument");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return fail(PBGPU_ERR_INVALID, "device %d out of range", device);
  API_TRY
  HIPCHK(hipSetDevice(device));
  std::unique_ptr<pbgpu_index> ix(new pbgpu_index);
  ix->device = device;
  ix->k = src->k; ix->psa_min = src->psa_min;
  ix->n = src->n; ix->n_sr = src->n_sr; ix->n_kmers = src->n_kmers; ix->n_occ = src->n_occ; ix->buckets = src->buckets;
  ix->build_seconds = src->build_seconds;
  ix->name_fwd = src->name_fwd; ix->name_bwd = src->name_bwd; ix->sr_start = src->sr_start;
  ix->filt_log2 = src->filt_log2;
  ix->shard = src->shard; ix->n_shards = src->n_shards;
  ix->sr_begin = src->sr_begin; ix->sr_end = src->sr_end; ix->n_total = src->n_total;
  ix->gstart = src->gstart; ix->null_ptr = src->null_ptr;
  ix->fk = src->fk; ix->f_buckets = src->f_buckets; ix->f_kmers = src->f_kmers; ix->f_occ = src->f_occ;
  auto cp = [&](auto& dst, const auto& s) {  // device-to-device (peer when the devices differ)
    dst.alloc(s.n);
    if (!s.n) return;
    if (device == src->device) HIPCHK(hipMemcpy(dst.p, s.p, s.bytes(), hipMemcpyDeviceToDevice));
    else HIPCHK(hipMemcpyPeer(dst.p, device, s.p, src->device, s.bytes()));
  };
  cp(ix->text, src->text); cp(ix->d_sr_start, src->d_sr_start); cp(ix->occ, src->occ); cp(ix->table, src->table);
  cp(ix->sr_uoff, src->sr_uoff); cp(ix->sr_uids, src->sr_uids); cp(ix->filt, src->filt);
  cp(ix->f_occv, src->f_occv); cp(ix->f_table, src->f_table); cp(ix->occ_sr, src->occ_sr);
  HIPCHK(hipDeviceSynchronize());
  *out = ix.release();
  return PBGPU_OK;
  API_CATCH
}

// ---------------------------------------------------------------- index cache
// File: magic, version, tag, the scalars, the host vectors, then each device
// array as (element count, element size, bytes), streamed through one pinned
// 64 MiB buffer.
}  // extern "C"
namespace {
constexpr char kCacheMagic[8] = {'P', 'B', 'G', 'P', 'U', 'I', 'X', '\0'};
// The file holds raw device layouts (bucket hash, filter hash, header packing,
// element sizes): kIndexLayout is bumped with any change to them (pbgpu_internal.h),
// and the version also carries the ABI version.
constexpr uint64_t kCacheVersion = ((uint64_t)PBGPU_ABI_VERSION << 32) | kIndexLayout;
struct cache_file {
  FILE* f = nullptr;
  const char* path;
  ~cache_file() { if (f) fclose(f); }
  void put(const void* p, size_t n) {
    if (n && fwrite(p, 1, n, f) != n) throw bad_input(std::string("index cache: write failed: ") + path);
  }
  void get(void* p, size_t n) {
    if (n && fread(p, 1, n, f) != n) throw bad_input(std::string("index cache: truncated or unreadable: ") + path);
  }
  void put_u64(uint64_t v) { put(&v, 8); }
  uint64_t get_u64() { uint64_t v; get(&v, 8); return v; }
  void put_str(const std::string& v) { put_u64(v.size()); put(v.data(), v.size()); }
  std::string get_str(uint64_t max_len) {
    const uint64_t n = get_u64();
    if (n > max_len) throw bad_input(std::string("index cache: corrupt string length: ") + path);
    std::string v(n, '\0');
    get(&v[0], n);
    return v;
  }
};
struct pinned_chunk {
  static constexpr size_t kBytes = 64ull << 20;
  char* p = nullptr;
  pinned_chunk() { HIPCHK(hipHostMalloc((void**)&p, kBytes)); }
  ~pinned_chunk() { if (p) (void)hipHostFree(p); }
};
template <typename T>
void cache_put_dbuf(cache_file& cf, pinned_chunk& pc, const dbuf<T>& b) {
  cf.put_u64(b.n);
  cf.put_u64(sizeof(T));
  const size_t bytes = b.bytes();
  for (size_t o = 0; o < bytes; o += pinned_chunk::kBytes) {
    const size_t m = std::min(pinned_chunk::kBytes, bytes - o);
    HIPCHK(hipMemcpy(pc.p, (const char*)b.p + o, m, hipMemcpyDeviceToHost));
    cf.put(pc.p, m);
  }
}
template <typename T>
void cache_get_dbuf(cache_file& cf, pinned_chunk& pc, dbuf<T>& b) {
  const uint64_t n = cf.get_u64(), es = cf.get_u64();
  if (es != sizeof(T) || n > (1ull << 44)) throw bad_input(std::string("index cache: corrupt array header: ") + cf.path);
  b.alloc(n);
  const size_t bytes = b.bytes();
  for (size_t o = 0; o < bytes; o += pinned_chunk::kBytes) {
    const size_t m = std::min(pinned_chunk::kBytes, bytes - o);
    cf.get(pc.p, m);
    HIPCHK(hipMemcpy((char*)b.p + o, pc.p, m, hipMemcpyHostToDevice));
  }
}
}  // namespace
extern "C" {

pbgpu_status pbgpu_index_save(const pbgpu_index* ix, const char* path, const char* tag) {
  if (!ix || !path) return fail(PBGPU_ERR_INVALID, "null argument");
  API_TRY
  HIPCHK(hipSetDevice(ix->device));
  const std::string tmp = std::string(path) + ".tmp";
  {
    cache_file cf;
    cf.path = path;
    cf.f = fopen(tmp.c_str(), "wb");
    if (!cf.f) return fail(PBGPU_ERR_IO, "cannot write index cache '%s'", tmp.c_str());
    cf.put(kCacheMagic, 8);
    cf.put_u64(kCacheVersion);
    cf.put_str(tag ? tag : "");
    const uint64_t sc[] = {ix->k, ix->psa_min, ix->n, ix->n_sr, ix->n_kmers, ix->n_occ, ix->buckets, ix->filt_log2,
                           ix->shard, ix->n_shards, ix->sr_begin, ix->sr_end, ix->n_total, ix->null_ptr, ix->fk,
                           ix->f_buckets, ix->f_kmers, ix->f_occ};
    cf.put_u64(sizeof(sc) / 8);
    cf.put(sc, sizeof(sc));
    for (const NameTable* t : {&ix->name_fwd, &ix->name_bwd}) {
      cf.put_u64(t->off.size()); cf.put(t->off.data(), t->off.size() * 8);
      cf.put_u64(t->blob.size()); cf.put(t->blob.data(), t->blob.size());
    }
    cf.put_u64(ix->sr_start.size()); cf.put(ix->sr_start.data(), ix->sr_start.size() * 8);
    cf.put_u64(ix->gstart.size()); cf.put(ix->gstart.data(), ix->gstart.size() * 8);
    pinned_chunk pc;
    cache_put_dbuf(cf, pc, ix->text); cache_put_dbuf(cf, pc, ix->d_sr_start); cache_put_dbuf(cf, pc, ix->occ);
    cache_put_dbuf(cf, pc, ix->table); cache_put_dbuf(cf, pc, ix->sr_uoff); cache_put_dbuf(cf, pc, ix->sr_uids);
    cache_put_dbuf(cf, pc, ix->filt); cache_put_dbuf(cf, pc, ix->f_occv); cache_put_dbuf(cf, pc, ix->f_table);
    cf.put(kCacheMagic, 8);  // trailer: a file cut short anywhere fails to load
    if (fflush(cf.f) != 0) return fail(PBGPU_ERR_IO, "cannot write index cache '%s'", tmp.c_str());
  }
  if (rename(tmp.c_str(), path) != 0) return fail(PBGPU_ERR_IO, "cannot rename '%s' to '%s'", tmp.c_str(), path);
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_index_load(const char* path, int device, const char* tag, pbgpu_index** out) {
  if (!path || !out) return fail(PBGPU_ERR_INVALID, "null argument");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return fail(PBGPU_ERR_INVALID, "device %d out of range", device);
  API_TRY
  const auto t0 = std::chrono::steady_clock::now();
  cache_file cf;
  cf.path = path;
  cf.f = fopen(path, "rb");
  if (!cf.f) return fail(PBGPU_ERR_IO, "cannot open index cache '%s'", path);
  char magic[8];
  cf.get(magic, 8);
  if (memcmp(magic, kCacheMagic, 8) != 0) return fail(PBGPU_ERR_IO, "'%s' is not an index cache", path);
  if (cf.get_u64() != kCacheVersion) return fail(PBGPU_ERR_IO, "'%s': index cache of another version", path);
  if (cf.get_str(1 << 20) != std::string(tag ? tag : ""))
    return fail(PBGPU_ERR_IO, "'%s': index cache saved for other inputs or parameters (tag differs)", path);
  uint64_t sc[18];
  if (cf.get_u64() != 18) return fail(PBGPU_ERR_IO, "'%s': corrupt index cache header", path);
  cf.get(sc, sizeof(sc));
  HIPCHK(hipSetDevice(device));
  std::unique_ptr<pbgpu_index> ix(new pbgpu_index);
  ix->device = device;
  ix->k = (uint32_t)sc[0]; ix->psa_min = (uint32_t)sc[1]; ix->n = sc[2]; ix->n_sr = sc[3]; ix->n_kmers = sc[4];
  ix->n_occ = sc[5]; ix->buckets = sc[6]; ix->filt_log2 = (uint32_t)sc[7]; ix->shard = (uint32_t)sc[8];
  ix->n_shards = (uint32_t)sc[9]; ix->sr_begin = sc[10]; ix->sr_end = sc[11]; ix->n_total = sc[12];
  ix->null_ptr = sc[13]; ix->fk = (uint32_t)sc[14]; ix->f_buckets = sc[15]; ix->f_kmers = sc[16]; ix->f_occ = sc[17];
  for (NameTable* t : {&ix->name_fwd, &ix->name_bwd}) {
    const uint64_t no = cf.get_u64();
    if (no == 0 || no > (1ull << 32)) return fail(PBGPU_ERR_IO, "'%s': corrupt index cache (names)", path);
    t->off.resize(no); cf.get(t->off.data(), no * 8);
    const uint64_t nb = cf.get_u64();
    if (nb > (1ull << 40) || t->off[0] != 0 || t->off[no - 1] != nb)
      return fail(PBGPU_ERR_IO, "'%s': corrupt index cache (names)", path);
    t->blob.resize(nb); cf.get(t->blob.data(), nb);
    for (uint64_t i = 0; i + 1 < no; ++i)  // increasing, each name NUL-terminated
      if (t->off[i + 1] <= t->off[i] || t->blob[t->off[i + 1] - 1] != 0)
        return fail(PBGPU_ERR_IO, "'%s': corrupt index cache (names)", path);
  }
  uint64_t m = cf.get_u64();
  if (m > (1ull << 34)) return fail(PBGPU_ERR_IO, "'%s': corrupt index cache (starts)", path);
  ix->sr_start.resize(m); cf.get(ix->sr_start.data(), m * 8);
  m = cf.get_u64();
  if (m > (1ull << 34)) return fail(PBGPU_ERR_IO, "'%s': corrupt index cache (starts)", path);
  ix->gstart.resize(m); cf.get(ix->gstart.data(), m * 8);
  pinned_chunk pc;
  cache_get_dbuf(cf, pc, ix->text); cache_get_dbuf(cf, pc, ix->d_sr_start); cache_get_dbuf(cf, pc, ix->occ);
  cache_get_dbuf(cf, pc, ix->table); cache_get_dbuf(cf, pc, ix->sr_uoff); cache_get_dbuf(cf, pc, ix->sr_uids);
  cache_get_dbuf(cf, pc, ix->filt); cache_get_dbuf(cf, pc, ix->f_occv); cache_get_dbuf(cf, pc, ix->f_table);
  cf.get(magic, 8);
  if (memcmp(magic, kCacheMagic, 8) != 0) return fail(PBGPU_ERR_IO, "'%s': index cache trailer missing", path);
  // the scalars the kernels index with must agree with the array sizes (a corrupt but
  // untruncated file must not lead to out-of-bounds device reads)
  const bool fine = ix->fk != 0;
  if (ix->name_fwd.size() != ix->n_sr || ix->name_bwd.size() != ix->n_sr || ix->gstart.size() != ix->n_sr + 1 || ix->sr_begin > ix->sr_end ||
      ix->sr_end > ix->n_sr || ix->sr_start.size() != ix->sr_end - ix->sr_begin + 1 ||
      ix->d_sr_start.n != ix->sr_start.size() || ix->table.n != 4 * ix->buckets || ix->buckets == 0 ||
      (ix->buckets & (ix->buckets - 1)) != 0 || ix->filt.n != (ix->filt_log2 ? 1ull << ix->filt_log2 : 0) ||
      ix->filt_log2 >= 48 || ix->occ.n < ix->null_ptr + 2 || ix->text.n * 32 < ix->n ||
      (fine && (ix->f_table.n != 4 * ix->f_buckets || ix->f_buckets == 0 ||
                (ix->f_buckets & (ix->f_buckets - 1)) != 0)) ||
      (!fine && ix->f_table.n != 0))
    return fail(PBGPU_ERR_IO, "'%s': inconsistent index cache", path);
  HIPCHK(hipDeviceSynchronize());
  ix->build_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *out = ix.release();
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_index_get_info(const pbgpu_index* ix, pbgpu_index_info* info) {
  if (!ix || !info) return fail(PBGPU_ERR_INVALID, "null argument");
  info->n_sr = ix->n_sr; info->text_len = ix->n; info->n_kmers = ix->n_kmers; info->n_occurrences = ix->n_occ;
  info->sr_begin = ix->sr_begin; info->sr_end = ix->sr_end;
  info->table_buckets = ix->buckets; info->device_bytes = ix->device_bytes(); info->build_seconds = ix->build_seconds;
  info->filter_bytes = ix->filt.bytes();
  return PBGPU_OK;
}
const char* pbgpu_index_sr_name(const pbgpu_index* ix, uint32_t sr, int bwd) {
  if (!ix || sr >= ix->n_sr) return nullptr;
  return bwd ? ix->name_bwd.c_str(sr) : ix->name_fwd.c_str(sr);
}
uint32_t pbgpu_index_sr_len(const pbgpu_index* ix, uint32_t sr) {
  if (!ix || sr >= ix->n_sr) return 0;
  return (uint32_t)(ix->gstart[sr + 1] - ix->gstart[sr]);
}

void pbgpu_align_params_default(pbgpu_align_params* p) {
  memset(p, 0, sizeof(*p));
  p->k = 17; p->stretch_factor = 1.3; p->stretch_constant = 10; p->stretch_cap = 10000; p->window_size = 1;
  p->max_count = 5000; p->mers_matching = 0; p->bases_matching = 17;
}

}  // extern "C"


// print_details input (jf_aligner.cc:72-108) of one sub-batch: every (read,
// super-read) chain's final fwd / bwd lists and the printed lis, marked by
// walking the lis points (pairs are unique within a list) along the list.
static void capture_details(pbgpu_aligner* al, uint32_t nch, uint64_t Hs) {
  hipStream_t st = al->st;
  std::vector<ChainDesc> ch(nch);
  std::vector<uint32_t> sl(2ull * nch), ll(2ull * nch);
  std::vector<int2> X(Hs), pts(Hs);
  if (nch) {
    HIPCHK(hipMemcpyAsync(ch.data(), al->chains.p, nch * sizeof(ChainDesc), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(sl.data(), al->slen.p, 2ull * nch * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(ll.data(), al->lisl.p, 2ull * nch * 4, hipMemcpyDeviceToHost, st));
  }
  if (Hs) {
    HIPCHK(hipMemcpyAsync(X.data(), al->X.p, Hs * sizeof(int2), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(pts.data(), al->pts.p, Hs * sizeof(int2), hipMemcpyDeviceToHost, st));
  }
  HIPCHK(hipStreamSynchronize(st));
  auto& D = al->det;
  for (uint32_t c = 0; c < nch; ++c) {
    const ChainDesc& d = ch[c];
    const uint32_t nF = sl[2 * c], nB = sl[2 * c + 1], lf = ll[2 * c], lb = ll[2 * c + 1];
    const bool fa = lf > lb;  // print_details: fwd only if strictly longer (jf_aligner.cc:77)
    D.read.push_back(d.read); D.sr.push_back(d.sr); D.nf.push_back(nF);
    const int2* P = pts.data() + d.hit_base + (fa ? 0 : d.nf);
    const uint32_t nl = fa ? lf : lb;
    for (int strand = 0; strand < 2; ++strand) {
      const int2* L = X.data() + d.hit_base + (strand ? d.nf : 0);
      const uint32_t n = strand ? nB : nF;
      uint32_t li = 0;
      const bool mine = (strand == 0) == fa;
      for (uint32_t i = 0; i < n; ++i) {
        D.hits.push_back(L[i].x); D.hits.push_back(L[i].y);
        const int2 q = mine && li < nl ? pt_get(P, li) : make_int2(0, 0);
        const bool in = mine && li < nl && q.x == L[i].x && q.y == L[i].y;
        D.lis.push_back(in ? 1 : 0);
        li += in;
      }
      if (mine && li != nl) throw std::runtime_error("details: lis points not found in their list");
    }
    D.hoff.push_back(D.lis.size());
  }
}

// Fills r from a host batch on the aligner's stream.  Device buffers only grow
// (a reused pbgpu_reads allocates nothing once it is large enough: hipFree
// would synchronize the device and stall the other aligners' streams).
void upload_reads_into(pbgpu_aligner* al, const pbgpu_read_batch* b, pbgpu_reads* r) {
  hipStream_t st = al->st;
  r->owner = al;
  r->device = al->device;
  r->n_reads = b->n_reads;
  r->h_off.resize(b->n_reads + 1);
  const uint64_t o0 = b->n_reads ? b->offsets[0] : 0;
  for (uint64_t i = 0; i <= b->n_reads; ++i) {
    r->h_off[i] = b->n_reads ? b->offsets[i] - o0 : 0;
    if (i && r->h_off[i] < r->h_off[i - 1]) throw std::invalid_argument("offsets must be non-decreasing");
  }
  r->n_bases = r->h_off[b->n_reads];
  if (r->n_bases > 0xFFFFFFFFull * 8) throw unsupported("batch too large");
  r->seq.ensure(r->n_bases + 1);
  if (r->n_bases) HIPCHK(hipMemcpyAsync(r->seq.p, b->seq + o0, r->n_bases, hipMemcpyHostToDevice, st));
  r->off.ensure(b->n_reads + 1);
  HIPCHK(hipMemcpyAsync(r->off.p, r->h_off.data(), (b->n_reads + 1) * 8, hipMemcpyHostToDevice, st));
  r->has_names = b->names != nullptr && b->name_offsets != nullptr;
  if (r->has_names) {
    std::vector<uint64_t>& no = r->h_name_off;
    no.resize(b->n_reads + 1);
    const uint64_t n0 = b->n_reads ? b->name_offsets[0] : 0;
    for (uint64_t i = 0; i <= b->n_reads; ++i) {
      no[i] = b->n_reads ? b->name_offsets[i] - n0 : 0;
      if (i && no[i] < no[i - 1]) throw std::invalid_argument("name offsets must be non-decreasing");
    }
    // (name lengths grow with the read ids of a file: 32 bytes a read at least)
    r->names.ensure(std::max<uint64_t>(no[b->n_reads] + 1, 32 * (b->n_reads + 1)));
    if (no[b->n_reads]) HIPCHK(hipMemcpyAsync(r->names.p, b->names + n0, no[b->n_reads], hipMemcpyHostToDevice, st));
    r->name_off.ensure(b->n_reads + 1);
    HIPCHK(hipMemcpyAsync(r->name_off.p, no.data(), (b->n_reads + 1) * 8, hipMemcpyHostToDevice, st));
  }
  HIPCHK(hipStreamSynchronize(st));  // the host vectors above are the copies' sources
}


extern "C" {

pbgpu_status pbgpu_aligner_create(const pbgpu_index* ix, const pbgpu_align_params* params, pbgpu_aligner** out) {
  if (!ix || !params || !out) return fail(PBGPU_ERR_INVALID, "null argument");
  if (params->k != ix->k) return fail(PBGPU_ERR_INVALID, "aligner k (%u) != index k (%u)", params->k, ix->k);
  if (params->max_count <= 0)
    return fail(PBGPU_ERR_INVALID, "max_count must be > 0 (0 means INT_MAX upstream, which is undefined behaviour)");
  if (params->n_unitigs && !params->forward)
    return fail(PBGPU_ERR_INVALID, "Forward flag must be used if passing unitigs lengths");
  if (params->fine_k && params->fine_k != ix->fk)
    return fail(PBGPU_ERR_INVALID, "aligner fine_k (%u) != the index's fine sub-index k (%u): build the index with fine_k",
                params->fine_k, ix->fk);
  if (params->unitigs_k && !params->unitig_lengths)
    return fail(PBGPU_ERR_INVALID, "unitigs_k given without unitig lengths");
  API_TRY
  HIPCHK(hipSetDevice(ix->device));
  std::unique_ptr<pbgpu_aligner> al(new pbgpu_aligner);
  al->ix = ix;
  al->device = ix->device;
  // kmers_info holds 2 u - 1 ints a record (u: the unitigs of its super-read's name,
  // pb_aligner.cc:84-143): the first estimate is twice the index's mean, grown on overflow
  {
    const double mean_u = (double)ix->sr_uids.n / (double)std::max<uint64_t>(1, ix->sr_end - ix->sr_begin);
    al->info_per_chain = (uint64_t)std::min(32.0, std::max(8.0, std::ceil(2.0 * (2.0 * mean_u - 1.0)) + 4.0));
  }
  al->prm = *params;
  al->prm.unitig_lengths = nullptr;
  if (params->unitigs_k && params->n_unitigs) {
    al->ul.alloc(params->n_unitigs);
    HIPCHK(hipMemcpy(al->ul.p, params->unitig_lengths, params->n_unitigs * 4, hipMemcpyHostToDevice));
  }
  AlignParamsDev& P = al->P;
  P.k = params->k; P.window = params->window_size;
  P.a = params->stretch_factor; P.b = params->stretch_constant; P.C = params->stretch_cap;
  P.forward = params->forward; P.max_match = params->max_match; P.max_count = params->max_count;
  P.mers_factor = params->mers_matching / 100.0; P.bases_factor = params->bases_matching / 100.0;
  P.unitigs_k = params->unitigs_k && params->n_unitigs ? params->unitigs_k : 0;
  P.ul = al->ul.p; P.n_ul = params->unitigs_k ? params->n_unitigs : 0;
  P.sr_ul = nullptr; P.sr_meta = nullptr;
  if (P.unitigs_k) {  // lengths along every super-read name, resolved once (k_coords' kmers_info)
    const uint64_t nu = ix->sr_uids.n;
    al->sr_ul.alloc(std::max<uint64_t>(nu, 1));
    launch_sr_ul(ix->sr_uids.p, nu, al->ul.p, P.n_ul, al->sr_ul.p, nullptr);
    HIPCHK(hipGetLastError());
    // and per super-read its length, name range and first lengths in one line (PBGPU_SR_META=0: off)
    static const bool meta_on = !(getenv("PBGPU_SR_META") && !atoi(getenv("PBGPU_SR_META")));
    const uint64_t nloc = ix->sr_end - ix->sr_begin;
    if (meta_on && nloc) {
      al->sr_meta.alloc(nloc);
      launch_sr_meta(ix->d_sr_start.p, ix->sr_uoff.p, nloc, al->sr_ul.p, al->sr_meta.p, nullptr);
      HIPCHK(hipGetLastError());
      P.sr_meta = al->sr_meta.p;
    }
    HIPCHK(hipDeviceSynchronize());
    P.sr_ul = al->sr_ul.p;
  }
  al->lp.W = params->window_size; al->lp.a = params->stretch_factor; al->lp.b = params->stretch_constant;
  al->lp.C = params->stretch_cap; al->lp.mer_all = 0; al->lp.seq_all = 0; al->lp.ordered = 0;
  if (params->fine_k) {  // fine_aligner (fine_aligner.hpp:31-37): align_k = fine_k, compute_coords_info(forward = true)
    al->fine = true;
    al->PF = P;
    al->PF.k = params->fine_k; al->PF.forward = 1; al->PF.max_match = 0; al->PF.fine = 1;
    al->lpf = al->lp;
    al->lpf.W = 1; al->lpf.mer_all = 1; al->lpf.seq_all = 1;  // lis_align::accept_all, window 1 (fine_aligner.cc:43-46)
  }
  HIPCHK(hipStreamCreateWithFlags(&al->st, hipStreamNonBlocking));
  for (auto& e : al->ev) HIPCHK(hipEventCreate(&e));
  al->stats.alloc(ST_N + 1);  // + the fine stage's kmers_info capacity counter
  al->info_count.alloc(1);
  al->counters.alloc(128);
  al->n32total.alloc(1);
  al->rec_tile_ctr.alloc(2);
  *out = al.release();
  return PBGPU_OK;
  API_CATCH
}

// PBGPU_DEBUG_BUFFERS=1: each aligner's device buffers at its free, largest first (the
// working set by buffer; pbgpu_run_stats.device_peak_bytes is the device-wide figure)
static void buffer_report(const pbgpu_aligner* al) {
  std::vector<std::pair<const char*, size_t>> v = {
      {"ul", al->ul.bytes()},
      {"sr_ul", al->sr_ul.bytes()},
      {"krec", al->krec.bytes()},
      {"n_kept", al->n_kept.bytes()},
      {"thr", al->thr.bytes()},
      {"rec_per_read", al->rec_per_read.bytes()},
      {"rec_cursor", al->rec_cursor.bytes()},
      {"order", al->order.bytes()},
      {"ovf_items", al->ovf_items.bytes()},
      {"rcur", al->rcur.bytes()},
      {"counters", al->counters.bytes()},
      {"sort_scratch", al->sort_scratch.bytes()},
      {"nhits", al->nhits.bytes()},
      {"hit_off", al->hit_off.bytes()},
      {"rec_off", al->rec_off.bytes()},
      {"huge_elems", al->huge_elems.bytes()},
      {"hits", al->hits.bytes()},
      {"chains", al->chains.bytes()},
      {"perm", al->perm.bytes()},
      {"X", al->X.bytes()},
      {"pts", al->pts.bytes()},
      {"nodes", al->nodes.bytes()},
      {"nodes32", al->nodes32.bytes()},
      {"n32shift", al->n32shift.bytes()},
      {"lisl", al->lisl.bytes()},
      {"hist", al->hist.bytes()},
      {"slen", al->slen.bytes()},
      {"recs", al->recs.bytes()},
      {"recs_sorted", al->recs_sorted.bytes()},
      {"rec_read", al->rec_read.bytes()},
      {"rec_slot", al->rec_slot.bytes()},
      {"info_m", al->info_m.bytes()},
      {"info_b", al->info_b.bytes()},
      {"tmp", al->tmp.bytes()},
      {"gtable", al->gtable.bytes()},
      {"stats", al->stats.bytes()},
      {"info_count", al->info_count.bytes()},
      {"ovf_list", al->ovf_list.bytes()},
      {"read_list", al->read_list.bytes()},
      {"gcount", al->gcount.bytes()},
      {"gcount16", al->gcount16.bytes()},
      {"fwin", al->fwin.bytes()},
      {"fread_hits", al->fread_hits.bytes()},
      {"lstart", al->lstart.bytes()},
      {"lend", al->lend.bytes()},
      {"emit_of", al->emit_of.bytes()},
      {"X2", al->X2.bytes()},
      {"g_poff", al->g_poff.bytes()},
      {"g_pre", al->g_pre.bytes()},
      {"g_sizes", al->g_sizes.bytes()},
      {"g_desc", al->g_desc.bytes()}, {"g_spo", al->g_spo.bytes()}, {"g_fd", al->g_fd.bytes()}, {"g_fu0", al->g_fu0.bytes()},
      {"g_imp", al->g_imp.bytes()},
      {"g_out", al->g_out.bytes()},
      {"g_ecnt", al->g_ecnt.bytes()},
      {"g_eoff", al->g_eoff.bytes()},
      {"g_edges", al->g_edges.bytes()},
      {"g_eovf", al->g_eovf.bytes()},
      {"g_maxn", al->g_maxn.bytes()},
      {"g_ovf", al->g_ovf.bytes()},
      {"g_ovf_list", al->g_ovf_list.bytes()},
      {"g_cand", al->g_cand.bytes()},
      {"g_ord", al->g_ord.bytes()},
      {"g_ivs", al->g_ivs.bytes()},
      {"g_mo", al->g_mo.bytes()},
      {"g_mc", al->g_mc.bytes()},
      {"g_mcount", al->g_mcount.bytes()},
      {"g_munits", al->g_munits.bytes()},
      {"g_nhost", al->g_nhost.bytes()},
      {"g_mhost", al->g_mhost.bytes()},
      {"g_moff", al->g_moff.bytes()},
      {"g_uused", al->g_uused.bytes()},
      {"g_rsize", al->g_rsize.bytes()},
      {"g_isize", al->g_isize.bytes()},
      {"g_hroff", al->g_hroff.bytes()},
      {"g_hioff", al->g_hioff.bytes()},
      {"g_hrec", al->g_hrec.bytes()},
      {"g_hgraph", al->g_hgraph.bytes()},
      {"g_hinfo", al->g_hinfo.bytes()},
      {"fmt_len", al->fmt_len.bytes()},
      {"fmt_pos", al->fmt_pos.bytes()},
      {"text", al->text.bytes()},
      {"redo[0]", al->redo[0].bytes()},
      {"redo[1]", al->redo[1].bytes()},
      {"redo[2]", al->redo[2].bytes()},
      {"fwk[0]", al->fwk[0].bytes()},
      {"fwk[1]", al->fwk[1].bytes()},
      {"fwi[0]", al->fwi[0].bytes()},
      {"fwi[1]", al->fwi[1].bytes()},
      {"fkeys[0]", al->fkeys[0].bytes()},
      {"fkeys[1]", al->fkeys[1].bytes()}};
  std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
  size_t tot = 0;
  for (const auto& e : v) tot += e.second;
  fprintf(stderr, "pbgpu buffers: aligner %p device %d: %.3f GB in all;", (const void*)al, al->device, tot * 1e-9);
  for (const auto& e : v)
    if (e.second >= (16u << 20)) fprintf(stderr, " %s %.3f", e.first, e.second * 1e-9);
  fprintf(stderr, "\n");
}

pbgpu_status pbgpu_aligner_free(pbgpu_aligner* al) {
  if (!al) return PBGPU_OK;
  if (getenv("PBGPU_DEBUG_BUFFERS")) buffer_report(al);
  (void)hipSetDevice(al->device);  // not al->ix: the index may be freed first
#ifdef PBGPU_GRAPH_CHECK
  if (al->graph) { (void)hipDeviceSynchronize(); graph_check_report(); }
#endif
  for (auto& e : al->ev) if (e) (void)hipEventDestroy(e);
  if (al->g_fork) (void)hipEventDestroy(al->g_fork);
  if (al->g_join) (void)hipEventDestroy(al->g_join);
  if (al->g_side) (void)hipStreamDestroy(al->g_side);
  if (al->g_join2) (void)hipEventDestroy(al->g_join2);
  if (al->g_side2) (void)hipStreamDestroy(al->g_side2);
  if (al->grp_fork) (void)hipEventDestroy(al->grp_fork);
  if (al->grp_join) (void)hipEventDestroy(al->grp_join);
  if (al->grp_side) (void)hipStreamDestroy(al->grp_side);
  if (al->st) (void)hipStreamDestroy(al->st);
  delete al;
  return PBGPU_OK;
}

pbgpu_status pbgpu_reads_upload(pbgpu_aligner* al, const pbgpu_read_batch* b, pbgpu_reads** out) {
  if (!al || !b || !out || (b->n_reads && (!b->offsets || !b->seq))) return fail(PBGPU_ERR_INVALID, "null argument");
  API_TRY
  HIPCHK(hipSetDevice(al->ix->device));
  std::unique_ptr<pbgpu_reads> r(new pbgpu_reads);
  upload_reads_into(al, b, r.get());
  *out = r.release();
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_reads_free(pbgpu_reads* r) {
  if (!r) return PBGPU_OK;
  (void)hipSetDevice(r->device);
  delete r;
  return PBGPU_OK;
}

pbgpu_status pbgpu_shard_counts(pbgpu_aligner* al, const pbgpu_reads* rd) {
  if (!al || !rd) return fail(PBGPU_ERR_INVALID, "null argument");
  if (rd->owner != al) return fail(PBGPU_ERR_INVALID, "reads were uploaded for another aligner");
  API_TRY
  HIPCHK(hipSetDevice(al->ix->device));
  const uint32_t n = (uint32_t)rd->n_reads;
  al->gcount.ensure(rd->n_bases + 1);
  al->gcount_n = rd->n_bases;
  HIPCHK(hipMemsetAsync(al->gcount.p, 0, (rd->n_bases + 1) * 4, al->st));
  if (n) {
    HIPCHK(hipMemsetAsync(al->stats.p, 0, ST_N * 8, al->st));
    launch_seed(SEED_COUNTS, al->ix->view(), rd->seq.p, rd->off.p, n, al->P, nullptr, nullptr, nullptr, nullptr,
                al->stats.p, al->gcount.p, al->ix->null_ptr, al->st);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipStreamSynchronize(al->st));
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_shard_counts_download(pbgpu_aligner* al, uint32_t* host, uint64_t n) {
  if (!al || (!host && n)) return fail(PBGPU_ERR_INVALID, "null argument");
  if (n != al->gcount_n) return fail(PBGPU_ERR_INVALID, "count buffer holds %llu entries", (unsigned long long)al->gcount_n);
  API_TRY
  HIPCHK(hipSetDevice(al->ix->device));
  if (n) HIPCHK(hipMemcpy(host, al->gcount.p, n * 4, hipMemcpyDeviceToHost));
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_shard_counts_upload(pbgpu_aligner* al, const uint32_t* host, uint64_t n) {
  if (!al || (!host && n)) return fail(PBGPU_ERR_INVALID, "null argument");
  API_TRY
  HIPCHK(hipSetDevice(al->ix->device));
  // a fresh aligner (the shard rebuilt for the alignment pass) takes the summed counts
  // without computing its own first; pbgpu_align_resident_shard checks n against the batch
  al->gcount.ensure(n + 1);
  al->gcount_n = n;
  if (n) HIPCHK(hipMemcpy(al->gcount.p, host, n * 4, hipMemcpyHostToDevice));
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_rccl_unique_id(uint8_t id[128]) {
  if (!id) return fail(PBGPU_ERR_INVALID, "null argument");
  static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return fail(PBGPU_ERR_DEVICE, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  memcpy(id, &u, 128);
  return PBGPU_OK;
}

pbgpu_status pbgpu_rccl_comm_create(int device, int n_ranks, int rank, const uint8_t id[128], pbgpu_comm** out) {
  if (!id || !out || n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(PBGPU_ERR_INVALID, "bad argument");
  API_TRY
  HIPCHK(hipSetDevice(device));
  ncclUniqueId u;
  memcpy(&u, id, 128);
  std::unique_ptr<pbgpu_comm> c(new pbgpu_comm);
  c->device = device;
  c->n_ranks = n_ranks;
  const ncclResult_t r = ncclCommInitRank(&c->comm, n_ranks, u, rank);
  if (r != ncclSuccess) return fail(PBGPU_ERR_DEVICE, "ncclCommInitRank: %s", ncclGetErrorString(r));
  *out = c.release();
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_rccl_comm_free(pbgpu_comm* c) {
  if (!c) return PBGPU_OK;
  (void)hipSetDevice(c->device);
  (void)ncclCommDestroy(c->comm);
  delete c;
  return PBGPU_OK;
}

uint64_t pbgpu_rccl_comm_last_bytes(const pbgpu_comm* c) { return c ? c->last_bytes : 0; }

pbgpu_status pbgpu_shard_counts_allreduce(pbgpu_aligner* al, pbgpu_comm* c) {
  if (!al || !c) return fail(PBGPU_ERR_INVALID, "null argument");
  if (c->device != al->ix->device) return fail(PBGPU_ERR_INVALID, "communicator and aligner are on different devices");
  API_TRY
  HIPCHK(hipSetDevice(al->ix->device));
  if (al->gcount_n) {
    // two saturated counts per ncclUint32 when no half can carry (count_pack.h), else u32
    const uint64_t n = al->gcount_n;
    ncclResult_t r;
    if (counts_pack16_ok((uint32_t)c->n_ranks, (uint32_t)al->P.max_count)) {
      const uint64_t nw = counts_packed_words(n);
      al->gcount16.ensure(nw);
      launch_counts_pack16(false, al->gcount.p, n, al->gcount16.p, al->st);
      HIPCHK(hipGetLastError());
      r = ncclAllReduce(al->gcount16.p, al->gcount16.p, nw, ncclUint32, ncclSum, c->comm, al->st);
      if (r == ncclSuccess) {
        launch_counts_pack16(true, al->gcount16.p, n, al->gcount.p, al->st);
        HIPCHK(hipGetLastError());
      }
      c->last_bytes = nw * 4;
    } else {
      r = ncclAllReduce(al->gcount.p, al->gcount.p, n, ncclUint32, ncclSum, c->comm, al->st);
      c->last_bytes = n * 4;
    }
    if (r != ncclSuccess) return fail(PBGPU_ERR_DEVICE, "ncclAllReduce: %s", ncclGetErrorString(r));
  }
  HIPCHK(hipStreamSynchronize(al->st));
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_align_resident_shard(pbgpu_aligner* al, const pbgpu_reads* rd) {
  if (!al || !rd) return fail(PBGPU_ERR_INVALID, "null argument");
  if (rd->owner != al) return fail(PBGPU_ERR_INVALID, "reads were uploaded for another aligner");
  if (al->fine || al->details) return fail(PBGPU_ERR_UNSUPPORTED, "-F and --details run on a whole index only");
  if (al->gcount_n != rd->n_bases) return fail(PBGPU_ERR_INVALID, "no summed counts for this batch (pbgpu_shard_counts)");
  API_TRY
  HIPCHK(hipSetDevice(al->ix->device));
  aligner_pipeline(al, rd, SEED_FINISH, al->gcount.p);
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_align_resident(pbgpu_aligner* al, const pbgpu_reads* rd) {
  if (!al || !rd) return fail(PBGPU_ERR_INVALID, "null argument");
  if (rd->owner != al) return fail(PBGPU_ERR_INVALID, "reads were uploaded for another aligner");
  if (al->ix->n_shards > 1)
    return fail(PBGPU_ERR_INVALID, "sharded index: use pbgpu_shard_counts + pbgpu_align_resident_shard");
  API_TRY
  HIPCHK(hipSetDevice(al->ix->device));
  aligner_pipeline(al, rd);
  return PBGPU_OK;
  API_CATCH
}

}  // extern "C"

static float ev_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

// Strands (chain, fwd|bwd) in length order -> the LIS tiers (k_lis with
// 32-bit nodes above LIS_U16_MAX hits, k_lis with 16-bit nodes above
// LISW_LARGE, k_lis_w below), then the chains in lis-length order in al->perm
// for k_coords.  restore: k_group's lists need their order restored
// (k_strand_order / in k_lis_w); lists built in order (the fine aligner's) do
// not.  timed: record the k_lis slot events.  Returns the chains placed.
static uint32_t lis_stage(pbgpu_aligner* al, uint32_t nch, uint64_t Hs, const LisParams& lp0, int keep_idx,
                          bool restore, bool timed) {
  hipStream_t st = al->st;
  LisParams lp = lp0;
  lp.ordered = restore ? 0 : 1;
  // strands (chain, fwd|bwd) in length order -> k_lis (16-bit nodes; 32-bit for the longest strands)
  const uint32_t NB = len_buckets();
  al->hist.ensure(2 * NB);
  al->perm.ensure(2ull * nch + 1);
  al->lisl.ensure(2ull * nch + 1);
  al->slen.ensure(2ull * nch + 1);
  al->pinfo.ensure(2ull * nch + 1);
  uint32_t n_big = 0, n_mid = 0, n_w2 = 0, n_w1 = 0, n_w0 = 0;  // items in classes above LIS_U16_MAX / LISW_LARGE / LISW_SMALL / LISW_TINY
  auto order = [&](int which, uint32_t n_in) -> uint32_t {  // returns the number of items placed
    HIPCHK(hipMemsetAsync(al->hist.p, 0, NB * 4, st));
    if (which == 0) launch_strand_order(al->slen.p, n_in, al->hist.p, nullptr, nullptr, 0, st);
    else launch_chain_order(al->lisl.p, n_in, al->hist.p, nullptr, nullptr, 0,
                            timed ? al->stats.p + ST_FIT_CHAINS : nullptr, st);  // k_coords' work counters
    std::vector<uint32_t> h(NB), cur(NB);
    HIPCHK(hipMemcpyAsync(h.data(), al->hist.p, NB * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (getenv("PBGPU_DUMP_LEN_HIST")) {  // diagnostics: length-class histogram of this ordering pass
      fprintf(stderr, "len_hist %s:", which == 0 ? "strands" : "chains");
      for (uint32_t b = 0; b < NB; ++b) if (h[b]) fprintf(stderr, " %u:%u", b, h[b]);
      fprintf(stderr, "\n");
    }
    uint32_t acc = 0;
    for (int b = (int)NB - 1; b >= 1; --b) {  // longest first; bucket 0 = empty
      cur[b] = acc; acc += h[b];
      if ((uint32_t)b == big_bucket()) n_big = acc;  // items in buckets >= big_bucket(): > LIS_U16_MAX hits
      if ((uint32_t)b == lis_class_bounds(1)) n_mid = acc;
      if ((uint32_t)b == lis_class_bounds(0)) n_w2 = acc;
      if ((uint32_t)b == lis_class_bounds(3)) n_w1 = acc;
      if ((uint32_t)b == lis_lane_max() + 1) n_w0 = acc;  // len_bucket(n) = n below 128
    }
    cur[0] = acc;
    HIPCHK(hipMemcpyAsync(al->hist.p + NB, cur.data(), NB * 4, hipMemcpyHostToDevice, st));
    if (which == 0) launch_strand_order(al->slen.p, n_in, nullptr, al->hist.p + NB, al->perm.p, 1, st, al->chains.p,
                                        al->pinfo.p);
    else launch_chain_order(al->lisl.p, n_in, nullptr, al->hist.p + NB, al->perm.p, 1, nullptr, st);
    HIPCHK(hipGetLastError());
    return acc;
  };
  launch_init_slen(al->chains.p, nch, al->slen.p, st);
  HIPCHK(hipMemsetAsync(al->lisl.p, 0, 2ull * nch * 4, st));
  const uint32_t n_strands = order(0, 2 * nch);
  const uint32_t nbig = n_big;
  // 32-bit nodes: the strands above LIS_U16_MAX hits only, packed (k_node32_place);
  // a first reservation at the aligner's first call, so a later batch's long
  // strand rarely allocates
  (void)Hs;
  if (!al->nodes32.n) al->nodes32.ensure_fixed(32ull << 20);
  al->n32shift.ensure(2ull * nch + 1);
  if (nbig) {
    HIPCHK(hipMemsetAsync(al->n32total.p, 0, 8, st));
    launch_node32_place(al->chains.p, al->perm.p, nbig, al->slen.p, al->n32shift.p, al->n32total.p, st);
    unsigned long long chunks = 0;
    HIPCHK(hipMemcpyAsync(&chunks, al->n32total.p, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    al->nodes32.ensure((chunks + 1) * node32_chunk() * 16);
  }
  // strands longer than k_lis_w's LDS capacity: restore list order in place first.
  // (Running the tiers on separate streams was measured slower: they contend.)
  if (restore) launch_strand_order(al->chains.p, al->perm.p, n_mid, al->slen.p, al->X.p, st);
  if (timed) HIPCHK(hipEventRecord(al->ev[11], st));
  launch_lis(true, al->chains.p, al->perm.p, nbig, al->slen.p, al->X.p, al->nodes32.p, al->pts.p, al->lisl.p, lp,
             keep_idx, al->stats.p, st, al->n32shift.p);
  // 4095 < n <= 65535: lane-per-strand chunked kernel; n <= 4095: wave-per-strand kernels
  const uint32_t nmid = n_mid, nw2 = n_w2, nw1 = n_w1;
  launch_lis(false, al->chains.p, al->perm.p + nbig, nmid - nbig, al->slen.p, al->X.p, al->nodes.p, al->pts.p,
             al->lisl.p, lp, keep_idx, al->stats.p, st);
  launch_lis_wave(2, al->chains.p, al->perm.p + nmid, nw2 - nmid, al->slen.p, al->X.p, al->nodes.p, al->pts.p,
                  al->lisl.p, lp, keep_idx, al->stats.p, st);
  launch_lis_wave(1, al->chains.p, al->perm.p + nw2, nw1 - nw2, al->slen.p, al->X.p, al->nodes.p,
                  al->pts.p, al->lisl.p, lp, keep_idx, al->stats.p, st);
  // the shortest strands: lane per strand
  const uint32_t nw0 = std::max(n_w0, nw1);
  launch_lis_lane(al->chains.p, al->perm.p + nw0, n_strands - nw0, al->slen.p, al->X.p, al->nodes.p, al->pts.p,
                  al->lisl.p, lp, keep_idx, al->stats.p, st, Hs < (1ull << 32) ? al->pinfo.p + nw0 : nullptr);
  if (timed) HIPCHK(hipEventRecord(al->ev[10], st));  // the timed k_lis slot: tier-0 k_lis_w alone
  // tier 0 (9..255 hits).  (A 16-wave tier of its strands of <= 64 hits was measured
  // no faster: C2 LIS 20.7 vs 20.8 ms, C4r 47.0 vs 48.7, profiles/r05p_lisw.txt.)
  launch_lis_wave(0, al->chains.p, al->perm.p + nw1, nw0 - nw1, al->slen.p, al->X.p, al->nodes.p,
                  al->pts.p, al->lisl.p, lp, keep_idx, al->stats.p, st);
  HIPCHK(hipGetLastError());
  if (timed) HIPCHK(hipEventRecord(al->ev[12], st));
  // chains in lis-length order -> k_coords; record/info capacity
  const uint32_t n_fit = order(1, nch);
  return n_fit;
}

// Bump allocation over the batch's per-hit buffers (X, pts, nodes), which are dead once the
// records are out: the graph stage's temporaries (and the records sort's keys) are carved
// from them instead of holding buffers of their own (round 5: the two working sets are
// disjoint in time, so an aligner holds their maximum, not their sum).  A request that
// does not fit falls back to the buffer given.
struct DeadHits {
  struct Region { uint8_t* p; size_t n, used; };
  Region r[3];
  explicit DeadHits(pbgpu_aligner* al)
      : r{{(uint8_t*)al->X.p, al->X.bytes(), 0}, {(uint8_t*)al->pts.p, al->pts.bytes(), 0},
          {(uint8_t*)al->nodes.p, al->nodes.bytes(), 0}} {}
  // In a ramped batch (pbgpu_run's first batches, tl_grow_scale > 1) a temporary whose
  // full-batch size would not fit even an empty dead buffer gets its own buffer now,
  // sized for a full batch (round 5: C4r's edge blocks, 512 B a record, fit the first
  // batch's dead buffers and were allocated in batch 2, 4-5 GB each)
  template <typename T>
  T* take(dbuf<T>& own, size_t cnt) {
    const size_t bytes = cnt * sizeof(T);
    size_t largest = 0;
    for (auto& x : r) largest = std::max(largest, x.p ? x.n : 0);
    const bool never = tl_grow_scale > 1.0 && (double)bytes * tl_grow_scale > (double)largest;
    if (!never && !getenv("PBGPU_NO_CARVE"))
      for (auto& x : r) {
        const size_t a = (x.used + 255) & ~(size_t)255;
        if (x.p && a + bytes <= x.n) { x.used = a + bytes; return reinterpret_cast<T*>(x.p + a); }
      }
    own.ensure(cnt);
    return own.p;
  }
};

// Records grouped per read and sorted by (rs, re, ql, sr, emit): al->recs[0..nrec)
// -> al->recs_sorted, al->rec_off.  timed: event around the sort kernel.
// counted: every record's read count and slot were taken at emission (ChainOut.per_read)
static void records_stage(pbgpu_aligner* al, uint32_t n, uint32_t nrec, bool timed, bool counted = false) {
  hipStream_t st = al->st;
  al->rec_per_read.ensure(n); al->rec_cursor.ensure(n);
  if (!counted) {
    HIPCHK(hipMemsetAsync(al->rec_per_read.p, 0, n * 4, st));
    HIPCHK(hipMemsetAsync(al->rec_cursor.p, 0, n * 4, st));
    launch_rec_hist(al->rec_read.p, nrec, al->rec_per_read.p, st);
  }
  launch_excl_scan(al->rec_per_read.p, nullptr, n, al->rec_off.p,
                   (uint64_t*)temp_storage(al->tmp, excl_scan_scratch_words(n) * 8), st);
  al->order.ensure(nrec + 1);
  DeadHits dead(al);  // (every sub-batch's hits are done with)
  uint64_t* sort_keys = dead.take(al->sort_scratch, 6ull * nrec + 6);
  al->recs_sorted.ensure(nrec + 1);
  if (counted) launch_rec_place(al->rec_read.p, al->rec_slot.p, nrec, al->rec_off.p, al->order.p, st);
  else launch_rec_scatter(al->rec_read.p, nrec, al->rec_off.p, al->rec_cursor.p, al->order.p, st);
  uint2* tiles = dead.take(al->rec_tiles, rec_sort_max_tiles(nrec));
  HIPCHK(hipMemsetAsync(al->rec_tile_ctr.p, 0, 8, st));
  if (timed) HIPCHK(hipEventRecord(al->ev[15], st));
  launch_rec_sort(al->recs.p, al->rec_off.p, al->order.p, sort_keys, n, nrec, tiles, al->rec_tile_ctr.p,
                  al->recs_sorted.p, st);
  HIPCHK(hipGetLastError());
}

// fine_aligner::thread::align_sequence (fine_aligner.cc:38-51) for the whole
// batch, on the coarse records sorted per read (al->recs_sorted / rec_off):
// windows -> per-read windowed hit counts -> sub-batches of <= hit_budget hits:
// hits in list order -> stable sort by (window, strand) -> chains -> LIS
// (accept_all) -> k_coords (align_k = fine_k, forward, unfiltered) + the
// hit-less windows -> records.  The fine records replace the coarse ones.
static void fine_stage(pbgpu_aligner* al, const pbgpu_reads* rd) {
  const pbgpu_index* ix = al->ix;
  const IndexView v = ix->view(), fv = ix->fine_view();
  hipStream_t st = al->st;
  const uint32_t n = (uint32_t)rd->n_reads;
  const uint32_t nwin = (uint32_t)al->last_records;
  std::vector<uint64_t> woff(n + 1);
  HIPCHK(hipMemcpyAsync(woff.data(), al->rec_off.p, (n + 1) * 8, hipMemcpyDeviceToHost, st));
  // windows sorted by (read, super-read) (the lookup side of prime_frags_pos's std::map)
  al->fwin.ensure(nwin + 1); al->fwi[0].ensure(nwin + 1);
  DeadHits dead(al);  // (the coarse hits are done with; the fine ones come after the windows)
  launch_fine_win_sort(al->recs_sorted.p, al->rec_off.p, n, dead.take(al->sort_scratch, 6ull * nwin + 6), al->fwi[0].p,
                       st);
  launch_fine_windows(al->recs_sorted.p, nwin, nullptr, al->fwi[0].p, 1, rd->off.p, al->PF.k, al->fwin.p, st);
  HIPCHK(hipGetLastError());
  // windowed hits per read
  al->fread_hits.ensure(n + 1);
  launch_fine_hits(false, fv, rd->seq.p, rd->off.p, 0, n, al->fwin.p, al->rec_off.p, al->fread_hits.p, nullptr, 0,
                   nullptr, nullptr, al->stats.p, st);
  HIPCHK(hipGetLastError());
  std::vector<uint64_t> rh(n), hoff(n + 1, 0);
  HIPCHK(hipMemcpyAsync(rh.data(), al->fread_hits.p, (size_t)n * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  for (uint32_t r = 0; r < n; ++r) hoff[r + 1] = hoff[r] + rh[r];
  const uint64_t budget = std::min<uint64_t>(al->hit_budget, 0xFFFFFFF0ull);
  uint64_t rec_done = 0, info_done = 0;
  unsigned long long* info_need = al->stats.p + ST_N;  // scratch slot past the stat slots
  // sub-batches of about equal hits (ceil(total / budget) of them), each <= budget
  const uint64_t n_sub = (hoff[n] + budget - 1) / budget;
  const uint64_t target = n_sub ? (hoff[n] + n_sub - 1) / n_sub : 0;
  for (uint32_t r0 = 0; r0 < n;) {
    uint32_t r1 = r0 + 1;
    while (r1 < n && hoff[r1] - hoff[r0] < target && hoff[r1 + 1] - hoff[r0] <= budget) ++r1;
    const uint64_t Hs = hoff[r1] - hoff[r0];
    if (Hs > 0xFFFFFFF0ull) throw unsupported("a single read has more than 2^32 fine hits");
    const uint64_t ws0 = woff[r0];
    const uint32_t nws = (uint32_t)(woff[r1] - ws0);
    if (nws == 0) { r0 = r1; continue; }
    // sub-batch-relative hit offsets of its reads
    std::vector<uint64_t> rel(r1 - r0 + 1);  // (+ the end of the last read: k_fine_sort)
    for (uint32_t r = r0; r <= r1; ++r) rel[r - r0] = hoff[r] - hoff[r0];
    al->hit_off.ensure(n + 1);
    HIPCHK(hipMemcpyAsync(al->hit_off.p + r0, rel.data(), rel.size() * 8, hipMemcpyHostToDevice, st));
    al->fkeys[0].ensure(Hs + 1); al->fkeys[1].ensure(Hs + 1);
    al->X.ensure(Hs + 1); al->X2.ensure(Hs + 1);
    launch_fine_hits(true, fv, rd->seq.p, rd->off.p, r0, r1 - r0, al->fwin.p, al->rec_off.p, nullptr, al->hit_off.p,
                     ws0, al->fkeys[0].p, al->X.p, al->stats.p, st);
    HIPCHK(hipGetLastError());
    al->lstart.ensure(2ull * nws);  // (also the sort's key counts of reads with many windows)
    launch_fine_sort(al->fkeys[0].p, al->X.p, al->rec_off.p, al->hit_off.p, r0, r1 - r0, ws0, al->lstart.p,
                     al->fkeys[1].p, al->X2.p, st);
    HIPCHK(hipGetLastError());
    al->fkeys[0].swap(al->fkeys[1]);
    al->X.swap(al->X2);
    al->lstart.ensure(2ull * nws); al->lend.ensure(2ull * nws);
    HIPCHK(hipMemsetAsync(al->lstart.p, 0, 2ull * nws * 4, st));
    HIPCHK(hipMemsetAsync(al->lend.p, 0, 2ull * nws * 4, st));
    launch_list_bounds(al->fkeys[0].p, Hs, al->lstart.p, al->lend.p, st);
    al->chains.ensure(nws + 1); al->emit_of.ensure(nws + 1);
    HIPCHK(hipMemsetAsync(info_need, 0, 8, st));
    launch_fine_desc(v, al->recs_sorted.p, ws0, nws, al->lstart.p, al->lend.p, al->PF.unitigs_k != 0, al->chains.p,
                     al->emit_of.p, info_need, st);
    HIPCHK(hipGetLastError());
    al->pts.ensure(Hs + 9); al->nodes.ensure((Hs + 1) * 8);  // pts: + one 64-byte row (k_coords row loads)
    const uint32_t n_fit = lis_stage(al, nws, Hs, al->lpf, 0, false, false);
    unsigned long long need = 0;
    HIPCHK(hipMemcpyAsync(&need, info_need, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    al->recs.grow_keep(rec_done + nws + 1, rec_done, st);
    al->rec_read.grow_keep(al->recs.n, rec_done, st);
    if (al->PF.unitigs_k) {
      al->info_m.grow_keep(info_done + need + 1, info_done, st);
      al->info_b.grow_keep(info_done + need + 1, info_done, st);
    } else {
      al->info_m.ensure(1); al->info_b.ensure(1);
    }
    uint32_t rc32 = (uint32_t)rec_done;
    HIPCHK(hipMemcpyAsync(al->counters.p + 4, &rc32, 4, hipMemcpyHostToDevice, st));
    unsigned long long ic = info_done;
    HIPCHK(hipMemcpyAsync(al->info_count.p, &ic, 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(al->stats.p + ST_REC_OVERFLOW, 0, 8, st));
    ChainOut CO{};
    CO.pts = al->pts.p; CO.lisl = al->lisl.p;
    CO.redo = nullptr; CO.n_redo = al->counters.p + 8;
    CO.recs = al->recs.p; CO.rec_read = al->rec_read.p; CO.rec_count = al->counters.p + 4;
    CO.rec_cap = (uint32_t)std::min<uint64_t>(al->recs.n, 0xFFFFFFFFu);
    CO.info_m = al->info_m.p; CO.info_b = al->info_b.p; CO.info_count = al->info_count.p; CO.info_cap = al->info_m.n;
    CO.stats = al->stats.p;
    CO.emit_of = al->emit_of.p;
    launch_coords(v, al->PF, al->chains.p, al->perm.p, n_fit, rd->off.p, 0, CO, st);
    launch_fine_empty(v, al->PF.k, al->chains.p, nws, al->lisl.p, al->emit_of.p, CO, st);
    HIPCHK(hipGetLastError());
    uint32_t nrec = 0;
    unsigned long long ninfo = 0, ovf = 0;
    HIPCHK(hipMemcpyAsync(&nrec, al->counters.p + 4, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&ninfo, al->info_count.p, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&ovf, al->stats.p + ST_REC_OVERFLOW, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (ovf || nrec != rec_done + nws)
      throw std::runtime_error("fine aligner: record / kmers_info capacity mismatch");
    rec_done = nrec; info_done = ninfo;
    r0 = r1;
  }
  al->last_records = rec_done;
  al->last_info = info_done;
  records_stage(al, n, (uint32_t)rec_done, false);
}

// create_mega_reads' overlap graph of the final records (pbgpu_aligner_set_graph):
// implied positions and name prefix sums per record, the per-read sort, the traversal.
static void graph_stage(pbgpu_aligner* al, const pbgpu_reads* rd) {
  hipStream_t st = al->st;
  DeadHits dead(al);
  const uint32_t n = (uint32_t)rd->n_reads;
  const uint64_t nrec = al->last_records;
  GraphDev G{};
  G.recs = al->recs_sorted.p; G.rec_off = al->rec_off.p; G.roff = rd->off.p;
  G.noff = al->g_names->noff.p; G.units = al->g_names->units.p; G.ul = al->g_names->ul.p; G.n_ul = al->g_names->n_ul;
  G.info_m = al->info_m.p; G.info_b = al->info_b.p;
  G.play = al->g_play; G.nb_errors = al->g_errors; G.k = al->g_k; G.bases = al->g_bases;
  // PBGPU_GRAPH_NMAX (tests): a lower cap on the records of a read traversed on the device
  G.nmax = GRAPH_NMAX_BIG;
  if (const char* e = getenv("PBGPU_GRAPH_NMAX")) G.nmax = (uint32_t)std::min<long>(GRAPH_NMAX_BIG, std::max(0l, atol(e)));
  // reads of more records relax with their state in HBM (k_graph_relax_big): an LDS
  // tier's block of 4096-8192 records holds a CU alone, the HBM blocks share CUs (C4r graph
  // stage 200 -> 160 ms at 2048; at 1024 with the path records, C2 32.4 -> 30.2 ms, C4r
  // +1 ms, profiles/r05zf_graph_ab.txt; PBGPU_RELAX_BIG_MIN sets it)
  G.relax_big_min = 1024;
  if (const char* e = getenv("PBGPU_RELAX_BIG_MIN"))
    G.relax_big_min = (uint32_t)std::min<long>(GRAPH_NMAX, std::max(0l, atol(e)));
  // reads past GRAPH_NMAX records keep their sort keys and node state here (6 words a record)
  G.scratch = dead.take(al->sort_scratch, 6ull * nrec + 6);
  al->g_maxn.ensure(1);
  G.poff = dead.take(al->g_poff, nrec + 1); G.max_n = al->g_maxn.p;
  uint32_t* g_sizes = dead.take(al->g_sizes, nrec + 1);
  HIPCHK(hipMemsetAsync(al->g_maxn.p, 0, 4, st));
  launch_graph_sizes(G, n, nrec, g_sizes, (uint64_t*)temp_storage(al->tmp, excl_scan_scratch_words(nrec) * 8), st);
  HIPCHK(hipGetLastError());
  uint64_t tot = 0;
  uint32_t max_n = 0;
  HIPCHK(hipMemcpyAsync(&tot, G.poff + nrec, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&max_n, al->g_maxn.p, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  // k_graph keeps name offsets as 32 bits (a batch of 2^32 unitigs would be 48 GB of names)
  if (tot >= (1ull << 32)) throw bad_input("more than 2^32 name unitigs in one batch's records");
  // (with device mega-reads the nodes are temporaries too: only the host reads' come down)
  uint32_t* g_pre = dead.take(al->g_pre, 3 * tot + 3);
  G.pp = (uint2*)g_pre; G.ounits = g_pre + 2 * (tot + 1);
#ifdef PBGPU_GRAPH_CHECK
  G.units_total = tot;
#endif
  G.imp = dead.take(al->g_imp, nrec + 1); G.desc = dead.take(al->g_desc, nrec + 1);
  G.spo = dead.take(al->g_spo, nrec + 1);
  G.fis = dead.take(al->g_fd, 3 * (nrec + 1)); G.fie = G.fis + (nrec + 1); G.fer = G.fie + (nrec + 1);
  G.fu0 = dead.take(al->g_fu0, nrec + 1);
  if (al->g_mega) G.out = dead.take(al->g_out, nrec + 1);
  else { al->g_out.ensure(nrec + 1); G.out = al->g_out.p; }
  al->g_ovf.ensure(2);
  G.ecnt = dead.take(al->g_ecnt, nrec + 1); G.eoff = dead.take(al->g_eoff, nrec + 1);
  G.ovf_list = dead.take(al->g_ovf_list, nrec + 1);
  G.edges = dead.take(al->g_edges, nrec * GRAPH_EBLK);
  G.bmax = dead.take(al->g_bmax, nrec / 64 + 2);
  G.ovf = al->g_ovf.p;
  uint64_t ovf[2];
  HIPCHK(launch_graph(G, n, nrec, max_n, st, al->g_side, al->g_fork, al->g_join, ovf));
  HIPCHK(hipGetLastError());
  G.eovf = dead.take(al->g_eovf, std::max<uint64_t>(ovf[1], nrec) + 1);  // (a floor: the next batches rarely grow it)
  HIPCHK(launch_graph_relax(G, n, nrec, max_n, ovf[0], st, al->g_side, al->g_side2, al->g_fork, al->g_join,
                            al->g_join2));
  HIPCHK(hipGetLastError());
  al->acc.graph_ovf_nodes += ovf[0];
  al->g_mtotal = al->g_munits_used = 0;
  al->g_hosts = 0;
  if (!al->g_mega) return;
  // components, tiling and the printed mega-reads' paths on the device
  G.mega = 1; G.tiling = al->g_tiling; G.trim = al->g_trim;
  G.min_density = al->g_min_density; G.min_len = al->g_min_len;
  G.cand = dead.take(al->g_cand, nrec + 1); G.ord = dead.take(al->g_ord, 3 * nrec + 3);
  G.ivs = dead.take(al->g_ivs, 2 * nrec + 2); G.mo = dead.take(al->g_mo, nrec + 1);
  al->g_mcount.ensure(n + 1); al->g_mhost.ensure(n + 1); al->g_moff.ensure(n + 1);
  al->g_munits.ensure(tot + 1); al->g_uused.ensure(1); al->g_nhost.ensure(1);
  G.mcount = al->g_mcount.p; G.mhost = al->g_mhost.p; G.munits = al->g_munits.p; G.units_used = al->g_uused.p;
  G.units_cap = tot; G.n_recs = nrec; G.n_host = al->g_nhost.p;
  HIPCHK(hipMemsetAsync(al->g_uused.p, 0, 8, st));
  HIPCHK(hipMemsetAsync(al->g_nhost.p, 0, 4, st));
  launch_mega(G, n, st);
  HIPCHK(hipGetLastError());
  launch_excl_scan(al->g_mcount.p, nullptr, n, al->g_moff.p,
                   (uint64_t*)temp_storage(al->tmp, excl_scan_scratch_words(n) * 8), st);
  uint64_t cnt[3] = {0, 0, 0};
  HIPCHK(hipMemcpyAsync(&cnt[0], al->g_moff.p + n, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&cnt[1], al->g_uused.p, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&cnt[2], al->g_nhost.p, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  al->g_mtotal = cnt[0];
  al->g_munits_used = std::min<uint64_t>(cnt[1], tot);
  al->g_hosts = cnt[2];
  al->acc.graph_host_reads += cnt[2];
  al->g_mc.ensure(cnt[0] + 1);
  launch_mega_pack(G, n, al->g_moff.p, al->g_mc.p, st);
  HIPCHK(hipGetLastError());
  al->g_hrecs = al->g_hinfos = 0;
  // the reads left to the host (since round 5 only reads past GRAPH_NMAX_BIG records, or
  // past PBGPU_GRAPH_NMAX in tests): their packing buffers hold four reads of
  // GRAPH_NMAX records from the first batch on (no allocation after it unless a batch
  // has more), the per-record sizes and offsets are temporaries
  constexpr uint64_t host_room = 4 * (uint64_t)(GRAPH_NMAX + 1);
  al->g_rsize.ensure(n + 1); al->g_hroff.ensure(n + 1);
  al->g_hrec.ensure(host_room); al->g_hgraph.ensure(host_room);
  al->g_hinfo.ensure(2 * host_room * (al->last_info / std::max<uint64_t>(1, nrec) + 2));
  if (!al->g_hosts) return;
  // the reads left to the host: their records, nodes and info packed (a small download)
  uint32_t* g_isize = dead.take(al->g_isize, nrec + 1);
  uint64_t* g_hioff = dead.take(al->g_hioff, nrec + 1);
  launch_host_sizes(G, n, al->g_rsize.p, g_isize, st);
  launch_excl_scan(al->g_rsize.p, nullptr, n, al->g_hroff.p,
                   (uint64_t*)temp_storage(al->tmp, excl_scan_scratch_words(n) * 8), st);
  launch_excl_scan(g_isize, nullptr, nrec, g_hioff, (uint64_t*)temp_storage(al->tmp, excl_scan_scratch_words(nrec) * 8),
                   st);
  uint64_t hc[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(&hc[0], al->g_hroff.p + n, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&hc[1], g_hioff + nrec, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  al->g_hrecs = hc[0]; al->g_hinfos = hc[1];
  al->g_hrec.ensure(hc[0] + 1); al->g_hgraph.ensure(hc[0] + 1); al->g_hinfo.ensure(2 * hc[1] + 2);
  launch_host_pack(G, n, al->g_hroff.p, g_hioff, al->g_hrec.p, al->g_hgraph.p, al->g_hinfo.p,
                   al->g_hinfo.p + hc[1] + 1, st);
  HIPCHK(hipGetLastError());
}

void aligner_pipeline(pbgpu_aligner* al, const pbgpu_reads* rd, int seed_mode, uint32_t* gcount) {
  const pbgpu_index* ix = al->ix;
  const IndexView v = ix->view();
  hipStream_t st = al->st;
  const uint32_t n = (uint32_t)rd->n_reads;
  al->have_result = false;
  al->last_reads = n;
  al->det.clear();
  al->acc.n_batches++;
  al->acc.n_reads += n;
  al->acc.n_bases += rd->n_bases;
  al->rec_off.ensure(n + 1);
  if (n == 0) {
    HIPCHK(hipMemsetAsync(al->rec_off.p, 0, 8, st));
    HIPCHK(hipStreamSynchronize(st));
    al->last_records = 0; al->last_info = 0; al->have_result = true;
    return;
  }
  HIPCHK(hipMemsetAsync(al->stats.p, 0, ST_N * 8, st));
  // The batch in chunks of reads of at most chunk_bases bases: per chunk its seeding
  // (KRec, 16 B a base) and its sub-batches, the records appended.  One chunk unless the
  // batch is larger than the device holds (round 4: one 3.6-Gbase C3 call ran out of HBM;
  // the caller had to cut it).  The hit budget is likewise held to the free memory.
  size_t mem_free = 0, mem_tot = 0;
  HIPCHK(hipMemGetInfo(&mem_free, &mem_tot));
  const uint64_t mem_avail = (uint64_t)mem_free + al->krec.bytes() + al->X.bytes() + al->pts.bytes() + al->nodes.bytes();
  uint64_t chunk_bases = std::max<uint64_t>(1ull << 26, mem_avail / 16 / 8);
  if (const char* e = getenv("PBGPU_CHUNK_BASES")) chunk_bases = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
  // a hit costs 24 B of per-hit buffers (X, pts, nodes) plus, through the chains it makes
  // (chains_per_hit), a chain's descriptor and LIS state (~40 B), records (96 + 8 B each,
  // rec_per_chain of them) and kmers_info (2 x 4 B x info_per_chain): sub-batches of at
  // most the free memory / 1.25 by that sum once chains_per_hit is learnt from a sub-batch,
  // a third of it before (the first estimate is C2's 1/80; C4's reads make 1 chain per 9 hits)
  const double per_hit = 24.0 + al->chains_per_hit * (40.0 + 104.0 * al->rec_per_chain * (al->P.max_match ? 2.0 : 1.0) +
                                                      8.0 * (double)al->info_per_chain);
  const uint64_t budget = std::max<uint64_t>(
      1ull << 20, std::min<uint64_t>(al->hit_budget, (uint64_t)((double)mem_avail / per_hit / (al->cph_learned ? 1.25 : 3.0))));
  const uint32_t hcap_log2 = 11;
  std::vector<uint64_t> h_roff;  // host copy of the read offsets (the chunk cuts)
  if (rd->h_off.size() == (size_t)n + 1) {
    h_roff = rd->h_off;
  } else {
    h_roff.resize(n + 1);
    HIPCHK(hipMemcpyAsync(h_roff.data(), rd->off.p, (n + 1) * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  al->n_kept.ensure(n); al->thr.ensure(n); al->nhits.ensure(n); al->hit_off.ensure(n + 1);
  std::vector<uint64_t>& hoff = al->h_hoff;
  hoff.resize(n + 1);
  al->ovf_items.ensure(n); al->ovf_grow.ensure(n);
  al->ovf_list.ensure(n);  // (used only by batches with reads past the first group tier)
  al->rcur.ensure(n);
  uint64_t rec_done = 0, info_done = 0;
  // records counted per read as they are emitted (ChainOut.per_read), unless --max-match
  // re-emits or a sub-batch is redone after a record overflow: then records_stage counts
  static const bool rec_hist = getenv("PBGPU_REC_HIST") != nullptr;  // (A/B: always count afterwards)
  bool counted = !al->P.max_match && !rec_hist;
  al->rec_per_read.ensure(n);
  if (counted) HIPCHK(hipMemsetAsync(al->rec_per_read.p, 0, (size_t)n * 4, st));
  double ms_group = 0, ms_lis = 0, ms_fit = 0, ms_seed = 0;
  double k_ms[PBGPU_KERNEL_N] = {};
  uint64_t k_n[PBGPU_KERNEL_N] = {};
  uint64_t n_chains = 0, n_tests = 0;
  for (uint32_t c0 = 0; c0 < n;) {
  uint32_t c1 = c0 + 1;
  while (c1 < n && h_roff[c1 + 1] - h_roff[c0] <= chunk_bases) ++c1;
  const uint32_t ncr = c1 - c0;
  const uint64_t cb0 = h_roff[c0];
  // ---------------------------------------------------------------- seed
  // KRec of the chunk's bases: the kernels index it by absolute base offset (roff), so the
  // pointer handed to them is shifted back by the chunk's first base
  al->krec.ensure_capped(h_roff[c1] - cb0 + 1, al->base_cap ? al->base_cap + 1 : ~(size_t)0);
  // (as an address computation: the shifted pointer lies below the allocation when cb0 > 0,
  // and the kernels only index it at offsets >= cb0)
  KRec* const krec = reinterpret_cast<KRec*>(reinterpret_cast<uintptr_t>(al->krec.p) - (uintptr_t)cb0 * sizeof(KRec));
  HIPCHK(hipEventRecord(al->ev[0], st));
  launch_seed(seed_mode, v, rd->seq.p, rd->off.p + c0, ncr, al->P, krec, al->n_kept.p + c0, al->thr.p + c0,
              al->nhits.p + c0, al->stats.p, gcount, ix->null_ptr, st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(al->ev[1], st));
  // hit offsets relative to the chunk's first read
  launch_excl_scan(nullptr, al->nhits.p + c0, ncr, al->hit_off.p + c0,
                   (uint64_t*)temp_storage(al->tmp, excl_scan_scratch_words(ncr) * 8), st);
  HIPCHK(hipMemcpyAsync(hoff.data() + c0, al->hit_off.p + c0, (size_t)(ncr + 1) * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  ms_seed += ev_ms(al->ev[0], al->ev[1]);
  k_ms[PBGPU_KERNEL_SEED] += ev_ms(al->ev[0], al->ev[1]); k_n[PBGPU_KERNEL_SEED]++;
  // ------------------------------------- sub-batches: group -> chains (retry)
  // sub-batches of about equal hits (ceil(total / budget) of them), each <= budget
  const uint64_t n_sub = (hoff[c1] + budget - 1) / budget;
  const uint64_t target = n_sub ? (hoff[c1] + n_sub - 1) / n_sub : 0;
  for (uint32_t r0 = c0; r0 < c1;) {
    uint32_t r1 = r0 + 1;
    while (r1 < c1 && hoff[r1] - hoff[r0] < target && hoff[r1 + 1] - hoff[r0] <= budget) ++r1;
    const uint64_t Hs = hoff[r1] - hoff[r0];
    const uint32_t nr = r1 - r0;
    // per-hit buffers: at most the hit budget's (a read past it forms a sub-batch of its own)
    const uint64_t hcap = std::max<uint64_t>(Hs, std::min<uint64_t>(budget, 1ull << 40)) + 64;
    al->X.ensure_capped(Hs + 1 + GROUP_SINKS, hcap + GROUP_SINKS);
    al->pts.ensure_capped(Hs + 9, hcap);  // pts: + one 64-byte row (k_coords row loads)
    al->nodes.ensure_capped((Hs + 1) * 8, hcap * 8);
    al->chains.ensure(std::min<uint64_t>(Hs, (uint64_t)nr << 10) + 1);  // grown below if a batch needs more
    GroupOut O;
    O.X = al->X.p; O.chains = al->chains.p;
    O.sink = al->X.p + Hs + 1;  // k_group's lanes without a hit store here
    O.chain_count = al->counters.p;
    O.chain_cap = (uint32_t)std::min<uint64_t>(al->chains.n, 0xFFFFFFFFu);
    O.n_overflow = al->counters.p + 3;
    O.overflow_items = al->ovf_items.p; O.overflow_grow = al->ovf_grow.p;
    O.rcur = al->rcur.p;
    // Reads longest first (hits), so the long-read tail starts early.  The predicted
    // super-read count of a read (hits x chains-per-hit of earlier batches) picks its
    // table: 2048 LDS slots (4 waves), 8192 LDS slots (16 waves), and beyond that the
    // 8192-slot table over several hash partitions of its super-reads, a work item (and
    // block) each.  A misprediction only costs time: an overflowing item goes again in
    // the next tier or split in two.
    uint32_t n_small = 0, n_bigr = 0, n_bkt = 0, n_split = 0, split_pmax = 0;
    {
      const auto th0 = std::chrono::steady_clock::now();
      // Longest first by a counting sort over hit-count classes (exact below 128 hits, 16
      // classes per octave above; stable within a class): the order only schedules the
      // reads, so classes are as good as an exact sort, and O(n) where std::stable_sort
      // took milliseconds of host time while the GPU waited
      constexpr uint32_t NCL = 128 + 16 * 58;
      auto cls = [](uint64_t h) -> uint32_t {
        if (h < 128) return (uint32_t)h;
        const uint32_t l = 63u - (uint32_t)__builtin_clzll(h);
        return 128u + 16u * (l - 7u) + (uint32_t)((h >> (l - 4u)) & 15u);
      };
      std::vector<uint32_t>& rl = al->h_order;
      std::vector<uint32_t>& cnt = al->h_class;
      rl.resize(nr); cnt.assign(NCL + 1, 0);
      for (uint32_t r = r0; r < r1; ++r) ++cnt[NCL - 1 - cls(hoff[r + 1] - hoff[r])];
      for (uint32_t c = 0, acc = 0; c <= NCL; ++c) { const uint32_t v = cnt[c]; cnt[c] = acc; acc += v; }
      for (uint32_t r = r0; r < r1; ++r) rl[cnt[NCL - 1 - cls(hoff[r + 1] - hoff[r])]++] = r;
      const double fill_small = 0.95 * (double)((1u << hcap_log2) - (1u << hcap_log2) / 4);
      // tests: PBGPU_GROUP_PRED_SCALE=0 routes every read to the smallest table (all overflow paths)
      const double pred_scale = getenv("PBGPU_GROUP_PRED_SCALE") ? atof(getenv("PBGPU_GROUP_PRED_SCALE")) : 1.0;
#ifndef PBGPU_GROUP_BIG_FILL8
#define PBGPU_GROUP_BIG_FILL8 6
#endif
      const double fill_big = 0.95 * (double)((1u << kGroupLdsMaxLog2) / 8 * PBGPU_GROUP_BIG_FILL8);
      std::vector<uint2>& rs = al->h_small;
      std::vector<uint2>& rb = al->h_big;
      std::vector<uint2>& rbb = al->h_bkt;   // partition items of bucketed reads (MODE 2)
      std::vector<uint2>& rsp = al->h_split;  // one split item per bucketed read (MODE 1)
      rs.clear(); rb.clear(); rbb.clear(); rsp.clear();
      // PBGPU_GROUP_BUCKETS=0 (A/B): every partition item enumerates its read's hits (round 5)
      const bool buckets_on = !(getenv("PBGPU_GROUP_BUCKETS") && !atoi(getenv("PBGPU_GROUP_BUCKETS")));
      // (1.5 with the 16-wave split; with the 8-wave one 2.0: C4 overflowing items 1514 -> 76 per
      // 50k reads, group 91.8 -> 89.7 ms, profiles/r06bk_bucket_margin.txt)
      const double bucket_margin = getenv("PBGPU_GROUP_BUCKET_MARGIN") ? atof(getenv("PBGPU_GROUP_BUCKET_MARGIN")) : 2.0;
      // every read past the 4-wave tier is bucketed (P >= 1).  (From P >= 2 with the 2048-slot
      // bucket items: C4 group 127 -> 103 ms and C4r 43.2 -> 40.0 against P >= 3, C2 31.6 -> 32.2,
      // profiles/r06m_bucket_minp_lg11.txt; then P >= 1 with the 8-wave split: C4 94.1 -> 90.5,
      // C4r and C2 within 0.4 ms, profiles/r06sp_split_block.txt)
      const uint32_t bucket_minp = getenv("PBGPU_GROUP_BUCKET_MINP") ? (uint32_t)atoi(getenv("PBGPU_GROUP_BUCKET_MINP")) : 1;
      // the bucket items' table: 2^bkt_log2 slots (11: the 2048-slot, 4-wave blocks of the first
      // tier, five a CU; 13: the 8192-slot 16-wave blocks, one a CU), P sized for its fill limit
      // (PBGPU_GROUP_BUCKET_LOG2, A/B: 10 .. 13, below the first tier's table too)
      const uint32_t bkt_log2 = getenv("PBGPU_GROUP_BUCKET_LOG2")
          ? std::min<uint32_t>(kGroupLdsMaxLog2, std::max<uint32_t>(10, (uint32_t)atoi(getenv("PBGPU_GROUP_BUCKET_LOG2"))))
          : std::min<uint32_t>(kGroupLdsMaxLog2, std::max<uint32_t>(hcap_log2, 11));
      al->bkt_log2 = bkt_log2;
      const double fill_bkt = bkt_log2 >= kGroupLdsMaxLog2 ? fill_big
                                                           : 0.95 * (double)((1u << bkt_log2) - (1u << bkt_log2) / 4);
      uint32_t boff_words = 0;
      split_pmax = 0;
      al->h_bmeta.assign(nr, make_uint2(0u, 0u));
      // tests: PBGPU_GROUP_FIRST_P=P puts every read in the smallest table as P hash-partition
      // items, so a one-read call can overflow P items at once
      const uint32_t first_p = getenv("PBGPU_GROUP_FIRST_P") ? (uint32_t)atoi(getenv("PBGPU_GROUP_FIRST_P")) : 0;
      for (uint32_t r : rl) {
        if (first_p) {
          for (uint32_t q = 0; q < std::min<uint32_t>(first_p, 4096); ++q) rs.push_back(group_item(r, q, std::min<uint32_t>(first_p, 4096)));
          continue;
        }
        const double pred = (double)(hoff[r + 1] - hoff[r]) * al->chains_per_hit * pred_scale;
        if (pred <= fill_small) { rs.push_back(group_item(r, 0, 1)); continue; }
        const uint32_t P = (uint32_t)std::min(4096.0, std::max(1.0, std::ceil(pred / fill_big)));
        if (P >= bucket_minp && buckets_on) {
          // bucketed: its hits are enumerated once (the split item) into Pb buckets, which
          // its Pb partition items stream.  An item costs its bucket's entries plus a table
          // clear and compaction, so more, smaller partitions cost little, while an item
          // that overflows redoes its bucket in a later round: Pb takes a margin over the
          // prediction (C4: an overflow round of ~8 ms in a 92-ms sub-batch at 1.0)
          const uint32_t Pb = (uint32_t)std::min(4096.0, std::ceil(pred * bucket_margin / fill_bkt));
          split_pmax = std::max(split_pmax, Pb);
          al->h_bmeta[r - r0] = make_uint2(boff_words, Pb);
          boff_words += Pb + 1;
          rsp.push_back(group_item(r, 0, Pb));
          for (uint32_t q = 0; q < Pb; ++q) rbb.push_back(group_item(r, q, Pb));
          continue;
        }
        for (uint32_t q = 0; q < P; ++q) rb.push_back(group_item(r, q, P));
      }
      n_small = (uint32_t)rs.size(); n_bigr = (uint32_t)rb.size();
      n_bkt = (uint32_t)rbb.size(); n_split = (uint32_t)rsp.size();
      al->acc.group_bucketed_reads += n_split;
      rs.insert(rs.end(), rb.begin(), rb.end());
      rs.insert(rs.end(), rbb.begin(), rbb.end());
      rs.insert(rs.end(), rsp.begin(), rsp.end());
      // sized in every batch, bucketed reads or not: a run's first batches may have none and a
      // later one some (C2 create_mega_reads: two allocations after the first batch)
      al->bmeta.ensure(n);
      al->boff.ensure(std::max<uint32_t>(boff_words + 1, 4096));
      if (n_split) {
        HIPCHK(hipMemcpyAsync(al->bmeta.p + r0, al->h_bmeta.data(), (size_t)nr * sizeof(uint2), hipMemcpyHostToDevice, st));
      }
      al->acc.ms_host_order += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count();
      // the work items of a batch vary with its reads' partitions far more than the reads do
      // (a bucketed read is 1 + P items): lists of 12 B an item, sized for 16 items a read at
      // least, so a later batch's count does not allocate (test_no_device_allocation_after_first_batch)
      const size_t item_room = std::max<size_t>(rs.size(), 16ull * nr + 4096);
      al->read_list.ensure(item_room);
      HIPCHK(hipMemcpyAsync(al->read_list.p, rs.data(), rs.size() * sizeof(uint2), hipMemcpyHostToDevice, st));
      // every work item of the first round may overflow (a read split in P items holds P of
      // them): the overflow list holds one entry per item, not one per read
      al->ovf_items.ensure(item_room); al->ovf_grow.ensure(item_room);
      O.overflow_items = al->ovf_items.p; O.overflow_grow = al->ovf_grow.p;
      O.overflow_cap = (uint32_t)std::min<size_t>(al->ovf_items.n, 0xFFFFFFFFu);
      // the bucketed reads' staging: the sub-batch's LIS buffers, unused until the LIS stage
      O.stage_x = al->pts.p; O.stage_sr = reinterpret_cast<uint32_t*>(al->nodes.p);
      O.boff = al->boff.p; O.bmeta = al->bmeta.p;
    }
    for (int attempt = 0;; ++attempt) {
      HIPCHK(hipEventRecord(al->ev[5], st));
      HIPCHK(hipMemsetAsync(al->counters.p, 0, 16 * 4, st));
      HIPCHK(hipMemsetAsync(al->rcur.p + r0, 0, (size_t)nr * 4, st));
      static_assert(ST_LIS_TESTS == ST_CHAINS + 1, "per-attempt stat slots are adjacent");
      HIPCHK(hipMemsetAsync(al->stats.p + ST_CHAINS, 0, 16, st));  // redone on a retry: counted per attempt
      // PBGPU_GROUP_OVERLAP=1 (experiment): the 16-wave tier's reads -- the longest -- on a side
      // stream, started first, beside the 4-wave tier
      static const bool overlap = getenv("PBGPU_GROUP_OVERLAP") && atoi(getenv("PBGPU_GROUP_OVERLAP"));
      // The split of the bucketed reads (every attempt: a retry after the LIS stage finds the
      // staging overwritten) on a side stream beside the other tiers, their partition items
      // after both: alone, a launch of a few long reads' splits held the GPU for its longest
      // (C2: +1.7 ms of group stage)
      // the split beside the 16-wave tier (both long) on a side stream; beside the 4-wave
      // tier alone it would stretch that launch (C2 tier 0 21.2 -> 26.2 ms) for little: serial
      const bool split_side = n_split && n_bigr;
      if (n_split) {
        hipStream_t sst = st;
        if (split_side) {
          if (!al->grp_side) {
            HIPCHK(hipStreamCreateWithFlags(&al->grp_side, hipStreamNonBlocking));
            HIPCHK(hipEventCreateWithFlags(&al->grp_fork, hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&al->grp_join, hipEventDisableTiming));
          }
          HIPCHK(hipEventRecord(al->grp_fork, st));
          HIPCHK(hipStreamWaitEvent(al->grp_side, al->grp_fork, 0));
          sst = al->grp_side;
        }
        // the split's LDS holds a count and a cursor per partition: sized for the launch's
        // largest P (its scan and cursors), not the 4096 a read may reach
        uint32_t split_log2 = 6;
        while ((1u << split_log2) < split_pmax + 1 && split_log2 < 12) ++split_log2;
        launch_group(v, krec, rd->off.p, al->n_kept.p, al->thr.p, al->hit_off.p, hoff[r0], 0,
                     al->read_list.p + n_small + n_bigr + n_bkt, n_split, split_log2, nullptr, O, al->stats.p, sst, 1);
        HIPCHK(hipGetLastError());
        if (split_side) HIPCHK(hipEventRecord(al->grp_join, al->grp_side));
      }
      if (overlap && n_bigr && !n_split) {
        if (!al->grp_side) {
          HIPCHK(hipStreamCreateWithFlags(&al->grp_side, hipStreamNonBlocking));
          HIPCHK(hipEventCreateWithFlags(&al->grp_fork, hipEventDisableTiming));
          HIPCHK(hipEventCreateWithFlags(&al->grp_join, hipEventDisableTiming));
        }
        HIPCHK(hipEventRecord(al->grp_fork, st));
        HIPCHK(hipStreamWaitEvent(al->grp_side, al->grp_fork, 0));
        launch_group(v, krec, rd->off.p, al->n_kept.p, al->thr.p, al->hit_off.p, hoff[r0], 0,
                     al->read_list.p + n_small, n_bigr, kGroupLdsMaxLog2, nullptr, O, al->stats.p, al->grp_side);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(al->grp_join, al->grp_side));
      }
      HIPCHK(hipEventRecord(al->ev[8], st));
      launch_group(v, krec, rd->off.p, al->n_kept.p, al->thr.p, al->hit_off.p, hoff[r0], 0, al->read_list.p, n_small,
                   hcap_log2, nullptr, O, al->stats.p, st);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(al->ev[9], st));
      if (overlap && n_bigr && !n_split) {
        HIPCHK(hipStreamWaitEvent(st, al->grp_join, 0));
      } else {
        launch_group(v, krec, rd->off.p, al->n_kept.p, al->thr.p, al->hit_off.p, hoff[r0], 0,
                     al->read_list.p + n_small, n_bigr, kGroupLdsMaxLog2, nullptr, O, al->stats.p, st);
        HIPCHK(hipGetLastError());
      }
      if (split_side) HIPCHK(hipStreamWaitEvent(st, al->grp_join, 0));
      launch_group(v, krec, rd->off.p, al->n_kept.p, al->thr.p, al->hit_off.p, hoff[r0], 0,
                   al->read_list.p + n_small + n_bigr, n_bkt, al->bkt_log2, nullptr, O, al->stats.p, st, 2);
      HIPCHK(hipGetLastError());
      uint32_t cnt[4];
      HIPCHK(hipMemcpyAsync(cnt, al->counters.p, 16, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      // reads touching more super-reads than their table holds: the 8192-slot LDS
      // table, then HBM tables growing until they fit
      uint32_t n_ovf = cnt[3];
      if (n_ovf > O.overflow_cap) throw std::runtime_error("group overflow list past its capacity");
      al->acc.group_overflow_items += n_ovf;
      uint32_t lg = hcap_log2;
      while (n_ovf) {
        std::vector<uint2>& ovf = al->h_items;
        ovf.resize(n_ovf);
        std::vector<uint32_t> grow(n_ovf);
        HIPCHK(hipMemcpyAsync(ovf.data(), al->ovf_items.p, n_ovf * sizeof(uint2), hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(grow.data(), al->ovf_grow.p, n_ovf * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        uint64_t mx = 0;
        for (const uint2& it : ovf) mx = std::max(mx, hoff[it.x + 1] - hoff[it.x]);
        // Next: the 8192-slot LDS table, an overflowing item split into f items (partition p
        // of P is exactly partitions p f .. p f + f - 1 of P f; the read's other partitions
        // keep their lists), f the power of two >= its growth estimate (nk / k-mers taken when
        // the table filled; x 1/4 from the 2048-slot table's fill limit to the 8192-slot
        // one's), while every item's P stays <= 4096; past that, HBM tables x4 each round
        // (results do not depend on the tier).  On C4r reads the HBM tier took 75 ms a launch
        // (r04h) for what split LDS items do in a fraction, and splitting by the estimate
        // rather than in two saves rounds, each a launch of a few long items.
        const bool refine_off = getenv("PBGPU_GROUP_REFINE") && !atoi(getenv("PBGPU_GROUP_REFINE"));  // (tests)
        // (each item carries the table it filled: the first round holds both tiers' items)
        auto split_of = [&](uint32_t i) -> uint32_t {
          const uint32_t g = grow[i] & 0xFFFFFFu;
          const uint32_t tl = grow[i] >> 24;  // the table it filled: 2^tl slots; the next one is 2^13
          const uint32_t sh = tl < kGroupLdsMaxLog2 ? kGroupLdsMaxLog2 - tl : 0;
          const uint32_t need = sh ? (g + (1u << sh) - 1) >> sh : std::max<uint32_t>(2, g);
          uint32_t f = 1;
          while (f < need && f < 64) f <<= 1;
          return f;
        };
        bool refine = !refine_off;
        if (refine)
          for (uint32_t i = 0; i < n_ovf; ++i) refine &= (uint64_t)(ovf[i].y >> 16) * split_of(i) <= 4096;
        if (refine) {
          std::vector<uint2> next;
          next.reserve(2 * (size_t)n_ovf);
          bool split = false;
          for (uint32_t i = 0; i < n_ovf; ++i) {
            const uint32_t p = ovf[i].y & 0xFFFFu, P = ovf[i].y >> 16, f = split_of(i);
            split |= f > 1;
            for (uint32_t t = 0; t < f; ++t) next.push_back(group_item(ovf[i].x, p * f + t, P * f));
          }
          ovf.swap(next);
          n_ovf = (uint32_t)ovf.size();
          if (split) ++al->acc.group_refines;
          lg = kGroupLdsMaxLog2;
        } else {
          lg = lg < kGroupLdsMaxLog2 ? kGroupLdsMaxLog2 : lg + 2;
        }
        if (lg > kGroupLdsMaxLog2 && (1ull << (lg - 2)) > 2 * mx + 256)
          throw std::runtime_error("group table growth did not converge");
        // the items of bucketed reads (they stream their bucket: MODE 2) after the others
        const uint32_t n_plain = (uint32_t)(std::stable_partition(ovf.begin(), ovf.end(), [&](const uint2& it) {
                                              return al->h_bmeta[it.x - r0].y == 0;
                                            }) - ovf.begin());
        al->ovf_list.ensure(n_ovf);
        al->ovf_items.ensure(n_ovf); al->ovf_grow.ensure(n_ovf);  // (this round's overflow: at most its items)
        O.overflow_items = al->ovf_items.p; O.overflow_grow = al->ovf_grow.p;
        O.overflow_cap = (uint32_t)std::min<size_t>(al->ovf_items.n, 0xFFFFFFFFu);
        HIPCHK(hipMemcpyAsync(al->ovf_list.p, ovf.data(), n_ovf * sizeof(uint2), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemsetAsync(al->counters.p + 3, 0, 4, st));
        for (int mode = 0; mode <= 2; mode += 2) {
          const uint32_t i0 = mode ? n_plain : 0, ni = mode ? n_ovf - n_plain : n_plain;
          if (!ni) continue;
          if (lg <= kGroupLdsMaxLog2) {
            launch_group(v, krec, rd->off.p, al->n_kept.p, al->thr.p, al->hit_off.p, hoff[r0], 0,
                         al->ovf_list.p + i0, ni, lg, nullptr, O, al->stats.p, st, mode);
            HIPCHK(hipGetLastError());
          } else {
            al->acc.group_hbm_reads += ni;
            const uint64_t words = group_table_words(lg);
            const uint32_t grp = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ni, (1ull << 28) / words));
            al->gtable.ensure_fixed((uint64_t)grp * words);
            for (uint32_t s0 = 0; s0 < ni; s0 += grp) {
              const uint32_t m = std::min(grp, ni - s0);
              HIPCHK(hipMemsetAsync(al->gtable.p, 0, (size_t)m * words * 4, st));
              launch_group(v, krec, rd->off.p, al->n_kept.p, al->thr.p, al->hit_off.p, hoff[r0], 0,
                           al->ovf_list.p + i0 + s0, m, lg, al->gtable.p, O, al->stats.p, st, mode);
              HIPCHK(hipGetLastError());
            }
          }
        }
        HIPCHK(hipMemcpyAsync(cnt, al->counters.p, 16, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        n_ovf = cnt[3];
        if (n_ovf > O.overflow_cap) throw std::runtime_error("group overflow list past its capacity");
        al->acc.group_overflow_items += n_ovf;
      }
#ifndef PBGPU_EXP_GROUP_ONLY
      const uint32_t nch = cnt[0];
#else  // experiment: time the group stage alone (no chains go further; tier routing as usual)
      const uint32_t nch = 0;
      if (Hs) al->chains_per_hit = std::max(1e-4, 1.1 * (double)cnt[0] / (double)Hs);
#endif
      if (nch > O.chain_cap) {  // descriptor buffer too small: grow, redo this sub-batch's grouping
        if (attempt > 8) throw std::runtime_error("chain descriptor capacity did not converge");
        al->chains.ensure((uint64_t)nch + nch / 8 + 1);
        O.chains = al->chains.p;
        O.chain_cap = (uint32_t)std::min<uint64_t>(al->chains.n, 0xFFFFFFFFu);
        continue;
      }
      HIPCHK(hipEventRecord(al->ev[6], st));
      const uint32_t n_fit = lis_stage(al, nch, Hs, al->lp, al->P.max_match, true, true);
      const uint64_t rec_est = (uint64_t)std::ceil((double)nch * std::min(1.0, al->rec_per_chain)) * (al->P.max_match ? 2 : 1);
      const uint64_t rec_need = rec_done + rec_est + 1024 * (attempt + 1);
      al->recs.grow_keep(std::max<uint64_t>(rec_need, al->rec_hint), rec_done, st);
      al->rec_read.grow_keep(al->recs.n, rec_done, st);
      al->rec_slot.grow_keep(al->recs.n, rec_done, st);
      if (al->P.unitigs_k) {
        const uint64_t info_need = info_done + rec_est * al->info_per_chain + 4096;
        al->info_m.grow_keep(info_need, info_done, st);
        al->info_b.grow_keep(info_need, info_done, st);
      } else {
        al->info_m.ensure(1); al->info_b.ensure(1);
      }
      uint32_t rc32 = (uint32_t)rec_done;
      HIPCHK(hipMemcpyAsync(al->counters.p + 4, &rc32, 4, hipMemcpyHostToDevice, st));
      unsigned long long ic = info_done;
      HIPCHK(hipMemcpyAsync(al->info_count.p, &ic, 8, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemsetAsync(al->stats.p + ST_REC_OVERFLOW, 0, 8, st));
      if (al->P.max_match) { al->redo[0].ensure(nch + 1); al->redo[1].ensure(nch + 1); al->redo[2].ensure(nch + 1); }
      uint32_t* n_redo = al->counters.p + 8;  // [8] redo count, [9] small items, [10] big items
      HIPCHK(hipMemsetAsync(n_redo, 0, 12, st));
      ChainOut CO{};
      CO.pts = al->pts.p; CO.lisl = al->lisl.p;
      CO.redo = al->P.max_match ? al->redo[0].p : nullptr; CO.n_redo = n_redo;
      CO.recs = al->recs.p; CO.rec_read = al->rec_read.p; CO.rec_count = al->counters.p + 4;
      CO.rec_cap = (uint32_t)std::min<uint64_t>(al->recs.n, 0xFFFFFFFFu);
      CO.info_m = al->info_m.p; CO.info_b = al->info_b.p; CO.info_count = al->info_count.p; CO.info_cap = al->info_m.n;
      CO.stats = al->stats.p;
      CO.emit_of = nullptr;  // coarse: the round index is the emission index
      CO.per_read = counted ? al->rec_per_read.p : nullptr;
      CO.rec_slot = al->rec_slot.p;
      HIPCHK(hipEventRecord(al->ev[13], st));
      launch_coords(v, al->P, al->chains.p, al->perm.p, n_fit, rd->off.p, 0, CO, st);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(al->ev[14], st));  // the timed k_coords slot: the first launch alone
      // --max-match rounds: discard the emitted lis, redo the strand's LIS, emit again
      for (uint32_t round = 1, cur = 0; al->P.max_match; ++round) {
        uint32_t nr3[3];
        HIPCHK(hipMemcpyAsync(nr3, n_redo, 12, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        const uint32_t nre = nr3[0];
        if (!nre) break;
        uint32_t* list = al->redo[cur].p;
        uint32_t* small = al->perm.p;            // free after the coords order pass consumed it
        uint32_t* big = al->perm.p + nch;
        HIPCHK(hipMemsetAsync(n_redo, 0, 12, st));
        launch_discard(al->chains.p, list, nre, al->lisl.p, al->slen.p, al->X.p, al->nodes.p, al->nodes32.p,
                       al->n32shift.p, small, n_redo + 1, big, n_redo + 2, st);
        HIPCHK(hipMemcpyAsync(nr3, n_redo, 12, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        launch_lis(false, al->chains.p, small, nr3[1], al->slen.p, al->X.p, al->nodes.p, al->pts.p, al->lisl.p, al->lp,
                   1, al->stats.p, st);
        launch_lis(true, al->chains.p, big, nr3[2], al->slen.p, al->X.p, al->nodes32.p, al->pts.p, al->lisl.p, al->lp,
                   1, al->stats.p, st, al->n32shift.p);  // strands only shrink: placed by the first pass
        cur ^= 1;
        CO.redo = al->redo[cur].p;
        HIPCHK(hipMemsetAsync(n_redo, 0, 4, st));
        // the chain list of this round is the previous round's redo list
        HIPCHK(hipMemcpyAsync(al->redo[2].p, list, (size_t)nre * 4, hipMemcpyDeviceToDevice, st));
        launch_coords(v, al->P, al->chains.p, al->redo[2].p, nre, rd->off.p, round, CO, st);
        HIPCHK(hipGetLastError());
      }
      HIPCHK(hipEventRecord(al->ev[7], st));
      uint32_t nrec = 0;
      unsigned long long ninfo = 0, ovf = 0;
      HIPCHK(hipMemcpyAsync(&nrec, al->counters.p + 4, 4, hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(&ninfo, al->info_count.p, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(&ovf, al->stats.p + ST_REC_OVERFLOW, 8, hipMemcpyDeviceToHost, st));
      unsigned long long sub[2];
      HIPCHK(hipMemcpyAsync(sub, al->stats.p + ST_CHAINS, 16, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      ms_group += ev_ms(al->ev[5], al->ev[6]);
      ms_lis += ev_ms(al->ev[6], al->ev[12]);
      ms_fit += ev_ms(al->ev[12], al->ev[7]);
      k_ms[PBGPU_KERNEL_GROUP] += ev_ms(al->ev[8], al->ev[9]);
      k_ms[PBGPU_KERNEL_LIS] += ev_ms(al->ev[10], al->ev[12]);
      k_ms[PBGPU_KERNEL_COORDS] += ev_ms(al->ev[13], al->ev[14]);
      k_n[PBGPU_KERNEL_GROUP]++; k_n[PBGPU_KERNEL_LIS]++; k_n[PBGPU_KERNEL_COORDS]++;
      if (ovf == 0 && nrec <= al->recs.n) {
        if (al->details) capture_details(al, nch, Hs);
        const uint64_t sub_recs = nrec - rec_done;
        rec_done = nrec; info_done = ninfo;
        n_chains += sub[0]; n_tests += sub[1];
#ifndef PBGPU_EXP_GROUP_ONLY
        if (Hs) al->chains_per_hit = std::max(1e-4, 1.1 * (double)nch / (double)Hs);
        if (Hs) al->cph_learned = true;
#endif
        // (records a chain yields, with a margin; max-match rounds are counted by rec_est's x2)
        if (nch && !al->P.max_match)
          al->rec_per_chain = std::min(1.0, std::max(0.02, 1.25 * (double)sub_recs / (double)nch + 0.01));
        break;
      }
      if (attempt > 8) throw std::runtime_error("record buffer growth did not converge");
      counted = false;  // this attempt's emitted records were counted: records_stage recounts
      // grow (keeping the records of earlier sub-batches) and redo this sub-batch from the group pass
      al->rec_hint = std::max<uint64_t>(al->rec_hint, (uint64_t)nrec + 4096);
      if (ninfo > info_done + rec_est * al->info_per_chain) al->info_per_chain = al->info_per_chain * 2 + 16;
      al->rec_per_chain = 1.0;
    }
    r0 = r1;
  }
  c0 = c1;
  }  // chunks
  al->last_records = rec_done;
  al->last_info = info_done;
  HIPCHK(hipEventRecord(al->ev[3], st));
  const uint32_t nrec = (uint32_t)al->last_records;
  records_stage(al, n, nrec, true, counted);
  HIPCHK(hipEventRecord(al->ev[4], st));
  if (al->fine) {
    HIPCHK(hipEventRecord(al->ev[16], st));
    fine_stage(al, rd);
    HIPCHK(hipEventRecord(al->ev[17], st));
  }
  if (al->graph) {
    HIPCHK(hipEventRecord(al->ev[18], st));
    graph_stage(al, rd);
    HIPCHK(hipEventRecord(al->ev[19], st));
  }
  unsigned long long sv[ST_N];
  HIPCHK(hipMemcpyAsync(sv, al->stats.p, sizeof sv, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  al->acc.n_kmers += sv[ST_KMERS]; al->acc.n_probes += sv[ST_PROBES]; al->acc.n_kept += sv[ST_KEPT];
  al->acc.n_hits += sv[ST_HITS]; al->acc.n_chains += n_chains; al->acc.n_lis_tests += n_tests;
  al->acc.n_records += nrec;
  al->acc.g0_kept += sv[ST_G0_KEPT]; al->acc.g0_hits += sv[ST_G0_HITS]; al->acc.g0_chains += sv[ST_G0_CHAINS];
  al->acc.l0_hits += sv[ST_L0_HITS]; al->acc.l0_strands += sv[ST_L0_STRANDS];
  al->acc.fit_chains += sv[ST_FIT_CHAINS]; al->acc.fit_points += sv[ST_FIT_POINTS];
  al->acc.n_filter += sv[ST_FILTER];
  al->acc.l0_points += sv[ST_L0_POINTS];
  if (al->fine) {
    al->acc.n_fine_hits += sv[ST_FINE_HITS];
    al->acc.n_fine_windows += nrec;
    al->acc.ms_fine += ev_ms(al->ev[16], al->ev[17]);
  }
  if (al->graph) {
    al->acc.ms_graph += ev_ms(al->ev[18], al->ev[19]);
    al->acc.graph_records += al->last_records;
  }
  al->acc.ms_seed += ms_seed;
  al->acc.ms_group += ms_group;
  al->acc.ms_lis += ms_lis;
  al->acc.ms_fit += ms_fit;
  al->acc.ms_records += ev_ms(al->ev[3], al->ev[4]);
  k_ms[PBGPU_KERNEL_REC_SORT] += ev_ms(al->ev[15], al->ev[4]); k_n[PBGPU_KERNEL_REC_SORT]++;
  for (int i = 0; i < PBGPU_KERNEL_N; ++i) { al->acc.kernel_ms[i] += k_ms[i]; al->acc.kernel_launches[i] += k_n[i]; }
  al->have_result = true;
}

// ---------------------------------------------------------------- download
struct coords_holder {
  pbgpu_coords_batch c{};
  std::vector<uint64_t> off;
  std::vector<pbgpu_record> recs;
  std::vector<int32_t> km, kb;
  std::vector<pbgpu_graph_node> graph;
  std::vector<uint64_t> moff;
  std::vector<pbgpu_mega_read> mega;
  std::vector<uint32_t> munits;
  std::vector<uint8_t> mhost;
};
// the device mega-reads of the aligner's last alignment into host vectors
static void download_mega(pbgpu_aligner* al, std::vector<uint64_t>& moff, std::vector<pbgpu_mega_read>& mega,
                          std::vector<uint32_t>& munits, std::vector<uint8_t>& mhost) {
  static_assert(sizeof(pbgpu_mega_read) == sizeof(MegaOut), "mega-read layout");
  const uint64_t n = al->last_reads;
  moff.resize(n + 1); mhost.resize(n + 1); mega.resize(al->g_mtotal); munits.resize(al->g_munits_used);
  if (n && al->last_records) {
    HIPCHK(hipMemcpy(moff.data(), al->g_moff.p, (n + 1) * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(mhost.data(), al->g_mhost.p, n, hipMemcpyDeviceToHost));
  } else {
    std::fill(moff.begin(), moff.end(), 0ull);
    std::fill(mhost.begin(), mhost.end(), (uint8_t)0);
  }
  if (!mega.empty()) HIPCHK(hipMemcpy(mega.data(), al->g_mc.p, mega.size() * sizeof(MegaOut), hipMemcpyDeviceToHost));
  if (!munits.empty()) HIPCHK(hipMemcpy(munits.data(), al->g_munits.p, munits.size() * 4, hipMemcpyDeviceToHost));
}

extern "C" {

pbgpu_status pbgpu_download(pbgpu_aligner* al, pbgpu_coords_batch** out) {
  if (!al || !out) return fail(PBGPU_ERR_INVALID, "null argument");
  if (!al->have_result) return fail(PBGPU_ERR_INVALID, "no result to download");
  API_TRY
  HIPCHK(hipSetDevice(al->ix->device));
  std::unique_ptr<coords_holder> h(new coords_holder);
  const uint64_t n = al->last_reads;
  // device mega-reads: the records of the reads left to the host only, packed
  const bool dev_mega = al->graph && al->g_mega;
  const uint64_t nr = dev_mega ? al->g_hrecs : al->last_records, ni = dev_mega ? al->g_hinfos : al->last_info;
  h->off.assign(n + 1, 0);
  if (!dev_mega || al->g_hosts)
    HIPCHK(hipMemcpy(h->off.data(), dev_mega ? al->g_hroff.p : al->rec_off.p, (n + 1) * 8, hipMemcpyDeviceToHost));
  h->recs.resize(nr);
  static_assert(sizeof(pbgpu_record) == sizeof(Rec), "record layout");
  if (nr)
    HIPCHK(hipMemcpy(h->recs.data(), dev_mega ? al->g_hrec.p : al->recs_sorted.p, nr * sizeof(Rec), hipMemcpyDeviceToHost));
  if (al->ix->sr_begin)  // a shard's device super-read ids are local
    for (auto& r : h->recs) r.sr_index += (uint32_t)al->ix->sr_begin;
  if (ni) {
    h->km.resize(ni); h->kb.resize(ni);
    HIPCHK(hipMemcpy(h->km.data(), dev_mega ? al->g_hinfo.p : al->info_m.p, ni * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(h->kb.data(), dev_mega ? al->g_hinfo.p + ni + 1 : al->info_b.p, ni * 4, hipMemcpyDeviceToHost));
  }
  h->c.n_reads = n; h->c.n_records = nr; h->c.read_offsets = h->off.data(); h->c.records = h->recs.data();
  h->c.n_info = ni; h->c.kmers_info = h->km.data(); h->c.bases_info = h->kb.data();
  if (al->graph) {
    static_assert(sizeof(pbgpu_graph_node) == sizeof(GraphNode), "graph node layout");
    h->graph.resize(nr);
    if (nr)
      HIPCHK(hipMemcpy(h->graph.data(), dev_mega ? al->g_hgraph.p : al->g_out.p, nr * sizeof(GraphNode),
                       hipMemcpyDeviceToHost));
    h->c.graph = h->graph.data();
  }
  if (dev_mega) {
    download_mega(al, h->moff, h->mega, h->munits, h->mhost);
    h->c.mega_offsets = h->moff.data(); h->c.mega = h->mega.data(); h->c.mega_units = h->munits.data();
    h->c.mega_host = h->mhost.data();
  }
  *out = &h.release()->c;
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_coords_free(pbgpu_coords_batch* c) {
  if (!c) return PBGPU_OK;
  delete reinterpret_cast<coords_holder*>(c);  // c is the first member
  return PBGPU_OK;
}

// Per read, the shards' record runs (each sorted) merged by the per-read sort
// key of the whole index: (rs, re, ql) (jf_aligner.cc:148-154, coords_info::
// operator<) with the (sr_index, emit) tie-break; kmers_info copied along.
pbgpu_status pbgpu_coords_merge(const pbgpu_coords_batch* const* parts, uint64_t n_parts, pbgpu_coords_batch** out) {
  if (!parts || !out || !n_parts) return fail(PBGPU_ERR_INVALID, "null argument");
  for (uint64_t p = 0; p < n_parts; ++p) {
    if (!parts[p]) return fail(PBGPU_ERR_INVALID, "null part");
    if (parts[p]->n_reads != parts[0]->n_reads) return fail(PBGPU_ERR_INVALID, "parts cover different read batches");
  }
  API_TRY
  std::unique_ptr<coords_holder> h(new coords_holder);
  const uint64_t n = parts[0]->n_reads;
  uint64_t nr = 0, ni = 0;
  for (uint64_t p = 0; p < n_parts; ++p) { nr += parts[p]->n_records; ni += parts[p]->n_info; }
  h->off.assign(n + 1, 0);
  h->recs.reserve(nr);
  h->km.reserve(ni); h->kb.reserve(ni);
  auto before = [](const pbgpu_record& a, const pbgpu_record& b) {
    if (a.rs != b.rs) return a.rs < b.rs;
    if (a.re != b.re) return a.re < b.re;
    if (a.ql != b.ql) return a.ql < b.ql;
    if (a.sr_index != b.sr_index) return a.sr_index < b.sr_index;
    return a.emit < b.emit;
  };
  std::vector<std::pair<uint64_t, uint64_t>> run;  // (part, record)
  for (uint64_t r = 0; r < n; ++r) {
    run.clear();
    for (uint64_t p = 0; p < n_parts; ++p)
      for (uint64_t i = parts[p]->read_offsets[r]; i < parts[p]->read_offsets[r + 1]; ++i) run.emplace_back(p, i);
    std::sort(run.begin(), run.end(), [&](const std::pair<uint64_t, uint64_t>& a, const std::pair<uint64_t, uint64_t>& b) {
      return before(parts[a.first]->records[a.second], parts[b.first]->records[b.second]);
    });
    for (const auto& q : run) {
      const pbgpu_coords_batch* c = parts[q.first];
      pbgpu_record R = c->records[q.second];
      const uint64_t io = h->km.size();
      h->km.insert(h->km.end(), c->kmers_info + R.info_offset, c->kmers_info + R.info_offset + R.n_info);
      h->kb.insert(h->kb.end(), c->bases_info + R.info_offset, c->bases_info + R.info_offset + R.n_info);
      R.info_offset = io;
      h->recs.push_back(R);
    }
    h->off[r + 1] = h->recs.size();
  }
  h->c.n_reads = n; h->c.n_records = h->recs.size(); h->c.read_offsets = h->off.data(); h->c.records = h->recs.data();
  h->c.n_info = h->km.size(); h->c.kmers_info = h->km.data(); h->c.bases_info = h->kb.data();
  *out = &h.release()->c;
  return PBGPU_OK;
  API_CATCH
}

// 64-bit hash of a byte range, a word at a time (the graph arrays' identity)
static uint64_t hash_words(const void* data, uint64_t bytes, uint64_t h) {
  const uint8_t* b = (const uint8_t*)data;
  uint64_t i = 0;
  for (; i + 8 <= bytes; i += 8) {
    uint64_t w;
    memcpy(&w, b + i, 8);
    h = (h ^ w) * 0x100000001B3ull;
    h ^= h >> 29;
  }
  for (; i < bytes; ++i) h = (h ^ b[i]) * 0x100000001B3ull;
  return h ^ bytes;
}

pbgpu_status pbgpu_aligner_set_graph(pbgpu_aligner* al, const pbgpu_graph_params* p) {
  if (!al) return fail(PBGPU_ERR_INVALID, "null argument");
  if (!p) { al->graph = false; return PBGPU_OK; }
  if (al->ix->n_shards > 1) return fail(PBGPU_ERR_UNSUPPORTED, "the device overlap graph runs on a whole index only");
  if (p->n_sr != al->ix->n_sr) return fail(PBGPU_ERR_INVALID, "graph names: one unitig list per super-read of the index");
  if (!p->name_offsets || (p->name_offsets[p->n_sr] && !p->name_units) || (p->n_unitigs && !p->unitig_lengths))
    return fail(PBGPU_ERR_INVALID, "null graph array");
  if (p->k_len == 0) return fail(PBGPU_ERR_INVALID, "graph k-mer length 0");
  if (p->mega_reads && (p->tiling < PBGPU_TILING_NONE || p->tiling > PBGPU_TILING_WEIGHTED))
    return fail(PBGPU_ERR_INVALID, "graph tiling %d", p->tiling);
  for (uint64_t i = 0; i < p->n_sr; ++i)
    if (p->name_offsets[i + 1] < p->name_offsets[i] || p->name_offsets[i + 1] - p->name_offsets[i] > 0xFFFFu)
      return fail(PBGPU_ERR_INVALID, "graph names: offsets not ascending, or a name of more than 65535 unitigs");
  API_TRY
  HIPCHK(hipSetDevice(al->ix->device));
  const uint64_t nu = p->name_offsets[p->n_sr];
  {
    // one device copy per index: an aligner given the same arrays reuses it
    const uint64_t h = hash_words(p->name_units, nu * 4, hash_words(p->unitig_lengths, p->n_unitigs * 4,
                                  hash_words(p->name_offsets, (p->n_sr + 1) * 8, 0x9E3779B97F4A7C15ull)));
    pbgpu_index* ix = const_cast<pbgpu_index*>(al->ix);  // the shared copy is guarded by names_mu
    std::lock_guard<std::mutex> lk(ix->names_mu);
    std::shared_ptr<GraphNames> g = ix->graph_names;
    if (!g || g->hash != h || g->n_sr != p->n_sr || g->n_units != nu || g->n_ul != p->n_unitigs) {
      g = std::make_shared<GraphNames>();
      g->hash = h; g->n_sr = p->n_sr; g->n_units = nu; g->n_ul = p->n_unitigs;
      g->noff.ensure_fixed(p->n_sr + 1); g->units.ensure_fixed(nu + 1); g->ul.ensure_fixed(p->n_unitigs + 1);
      HIPCHK(hipMemcpy(g->noff.p, p->name_offsets, (p->n_sr + 1) * 8, hipMemcpyHostToDevice));
      if (nu) HIPCHK(hipMemcpy(g->units.p, p->name_units, nu * 4, hipMemcpyHostToDevice));
      if (p->n_unitigs) HIPCHK(hipMemcpy(g->ul.p, p->unitig_lengths, p->n_unitigs * 4, hipMemcpyHostToDevice));
      ix->graph_names = g;
    }
    al->g_names = g;
  }
  al->g_play = p->overlap_play; al->g_errors = p->nb_errors; al->g_k = p->k_len; al->g_bases = p->maximize_bases != 0;
  al->g_mega = p->mega_reads != 0;
  al->g_tiling = p->tiling; al->g_trim = p->trim != 0;
  al->g_min_density = p->min_density; al->g_min_len = p->min_len;
  if (!al->g_side) {
    HIPCHK(hipStreamCreateWithFlags(&al->g_side, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&al->g_side2, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&al->g_fork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&al->g_join, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&al->g_join2, hipEventDisableTiming));
  }
  al->graph = true;
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_aligner_set_details(pbgpu_aligner* al, int enable) {
  if (!al) return fail(PBGPU_ERR_INVALID, "null argument");
  if (enable && al->ix->n_shards > 1) return fail(PBGPU_ERR_UNSUPPORTED, "--details runs on a whole index only");
  al->details = enable != 0;
  return PBGPU_OK;
}

}  // extern "C"

struct details_holder {
  pbgpu_details_batch d{};
  std::vector<uint64_t> roff, hoff;
  std::vector<uint32_t> sr, nf;
  std::vector<int32_t> hits;
  std::vector<uint8_t> lis;
};

extern "C" {

pbgpu_status pbgpu_download_details(pbgpu_aligner* al, pbgpu_details_batch** out) {
  if (!al || !out) return fail(PBGPU_ERR_INVALID, "null argument");
  if (!al->have_result || !al->details) return fail(PBGPU_ERR_INVALID, "no details (enable them before aligning)");
  API_TRY
  std::unique_ptr<details_holder> h(new details_holder);
  const auto& D = al->det;
  const uint64_t n = al->last_reads, nl = D.read.size();
  // lists grouped by read, first-hit (chain) order within a read
  h->roff.assign(n + 1, 0);
  for (uint64_t i = 0; i < nl; ++i) h->roff[D.read[i] + 1]++;
  for (uint64_t r = 0; r < n; ++r) h->roff[r + 1] += h->roff[r];
  std::vector<uint64_t> cur(h->roff.begin(), h->roff.end() - 1), order(nl);
  for (uint64_t i = 0; i < nl; ++i) order[cur[D.read[i]]++] = i;
  h->sr.resize(nl); h->nf.resize(nl); h->hoff.resize(nl + 1); h->hoff[0] = 0;
  h->hits.resize(D.hits.size()); h->lis.resize(D.lis.size());
  for (uint64_t j = 0; j < nl; ++j) {
    const uint64_t i = order[j], a = D.hoff[i], b = D.hoff[i + 1], o = h->hoff[j];
    h->sr[j] = D.sr[i]; h->nf[j] = D.nf[i];
    std::copy(D.hits.begin() + 2 * a, D.hits.begin() + 2 * b, h->hits.begin() + 2 * o);
    std::copy(D.lis.begin() + a, D.lis.begin() + b, h->lis.begin() + o);
    h->hoff[j + 1] = o + (b - a);
  }
  auto& d = h->d;
  d.n_reads = n; d.n_lists = nl; d.n_hits = h->lis.size();
  d.read_offsets = h->roff.data(); d.list_sr = h->sr.data(); d.hit_offsets = h->hoff.data();
  d.n_fwd = h->nf.data(); d.hits = h->hits.data(); d.in_lis = h->lis.data();
  *out = &h.release()->d;
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_details_free(pbgpu_details_batch* d) {
  delete reinterpret_cast<details_holder*>(d);  // d is the first member
  return PBGPU_OK;
}

// print_details (jf_aligner.cc:72-108)
pbgpu_status pbgpu_format_details(const pbgpu_index* ix, const pbgpu_details_batch* d, const char* const* hdrs,
                                  int threads, char** text, uint64_t* len) {
  if (!ix || !d || !text || !len || (d->n_reads && !hdrs)) return fail(PBGPU_ERR_INVALID, "null argument");
  API_TRY
  const uint64_t n = d->n_reads;
  if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
  std::vector<std::string> parts(std::max<uint64_t>(1, (uint64_t)threads * 4));
  const uint64_t np = parts.size();
  std::atomic<uint64_t> next(0);
  auto work = [&]() {
    char buf[64];
    for (;;) {
      const uint64_t pi = next.fetch_add(1);
      if (pi >= np) break;
      std::string& o = parts[pi];
      for (uint64_t r = n * pi / np; r < n * (pi + 1) / np; ++r) {
        const char* h = hdrs[r];
        const size_t nl = strcspn(h, " \t\n\v\f\r");
        for (uint64_t l = d->read_offsets[r]; l < d->read_offsets[r + 1]; ++l) {
          o.append(h, nl); o += ' '; o += ix->name_fwd[d->list_sr[l]];
          const uint64_t a = d->hit_offsets[l], e = d->hit_offsets[l + 1], m = a + d->n_fwd[l];
          uint64_t fi = a, bi = m;
          while (fi < m || bi < e) {
            const uint64_t i = (fi < m && (bi == e || d->hits[2 * fi] <= d->hits[2 * bi])) ? fi++ : bi++;
            const int w = snprintf(buf, sizeof buf, d->in_lis[i] ? " [%d:%d]" : " %d:%d", d->hits[2 * i], d->hits[2 * i + 1]);
            o.append(buf, (size_t)w);
          }
          o += '\n';
        }
      }
    }
  };
  run_parallel(threads, work);
  uint64_t total = 0;
  for (auto& p : parts) total += p.size();
  char* t = (char*)malloc(total + 1);
  if (!t) return fail(PBGPU_ERR_NOMEM, "host allocation failed");
  uint64_t o = 0;
  for (auto& p : parts) { memcpy(t + o, p.data(), p.size()); o += p.size(); }
  t[o] = 0;
  *text = t; *len = o;
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_align_batch(pbgpu_aligner* al, const pbgpu_read_batch* b, pbgpu_coords_batch** out) {
  pbgpu_reads* r = nullptr;
  pbgpu_status s = pbgpu_reads_upload(al, b, &r);
  if (s != PBGPU_OK) return s;
  s = pbgpu_align_resident(al, r);
  if (s == PBGPU_OK) s = pbgpu_download(al, out);
  pbgpu_reads_free(r);
  return s;
}

pbgpu_status pbgpu_aligner_get_stats(const pbgpu_aligner* al, pbgpu_stats* s) {
  if (!al || !s) return fail(PBGPU_ERR_INVALID, "null argument");
  *s = al->acc;
  return PBGPU_OK;
}
pbgpu_status pbgpu_aligner_reset_stats(pbgpu_aligner* al) {
  if (!al) return fail(PBGPU_ERR_INVALID, "null argument");
  memset(&al->acc, 0, sizeof al->acc);
  return PBGPU_OK;
}

pbgpu_status pbgpu_aligner_set_hit_budget(pbgpu_aligner* al, uint64_t hits) {
  if (!al) return fail(PBGPU_ERR_INVALID, "null argument");
  if (hits == 0) return fail(PBGPU_ERR_INVALID, "hit budget must be > 0");
  al->hit_budget = hits;
  return PBGPU_OK;
}

// print_coords (jf_aligner.cc:41-70).  std::ostream << double with default
// flags is libstdc++'s "%.*g" at precision 6.
pbgpu_status pbgpu_format_coords(const pbgpu_index* ix, const pbgpu_coords_batch* c, const char* const* hdrs,
                                 const uint64_t* lens, int compact, int header, int zero_match, int threads,
                                 char** text, uint64_t* len) {
  if (!ix || !c || !text || !len || (c->n_reads && (!hdrs || !lens))) return fail(PBGPU_ERR_INVALID, "null argument");
  API_TRY
  const uint64_t n = c->n_reads;
  if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
  std::vector<std::string> parts(std::max<uint64_t>(1, (uint64_t)threads * 4));
  const uint64_t np = parts.size();
  std::atomic<uint64_t> next(0);
  auto work = [&]() {
    char buf[512];
    for (;;) {
      const uint64_t pi = next.fetch_add(1);
      if (pi >= np) break;
      const uint64_t r0 = n * pi / np, r1 = n * (pi + 1) / np;
      std::string& o = parts[pi];
      for (uint64_t r = r0; r < r1; ++r) {
        const uint64_t a = c->read_offsets[r], b = c->read_offsets[r + 1];
        if (a == b && !zero_match) continue;
        const char* h = hdrs[r];
        const size_t nl = strcspn(h, " \t\n\v\f\r");
        if (compact) {
          o += '>'; o += std::to_string(b - a); o += ' '; o.append(h, nl); o += '\n';
        }
        for (uint64_t i = a; i < b; ++i) {
          const pbgpu_record& R = c->records[i];
          if (!compact) { o.append(h, nl); o += ' '; }
          int w = snprintf(buf, sizeof buf, "%d %d %d %d %d %u %u %u %u %llu %u %.6g %.6g %.6g ", R.rs, R.re, R.qs, R.qe,
                           R.nb_mers, R.pb_cons, R.sr_cons, R.pb_cover, R.sr_cover, (unsigned long long)lens[r], R.ql,
                           R.stretch, R.offset, R.avg_err);
          o.append(buf, (size_t)w);
          o += (R.flags & 2u) ? ix->name_bwd[R.sr_index] : ix->name_fwd[R.sr_index];
          for (uint32_t t = 0; t < R.n_info; ++t) {
            w = snprintf(buf, sizeof buf, " %d:%d", c->kmers_info[R.info_offset + t], c->bases_info[R.info_offset + t]);
            o.append(buf, (size_t)w);
          }
          o += '\n';
        }
      }
    }
  };
  run_parallel(threads, work);
  std::string hdr;
  if (header)
    hdr = std::string("Rstart Rend Qstart Qend Nmers Rcons Qcons Rcover Qcover Rlen Qlen Stretch Offset Err") +
          (compact ? "" : " Rname") + " Qname\n";
  uint64_t total = hdr.size();
  for (auto& p : parts) total += p.size();
  char* t = (char*)malloc(total + 1);
  if (!t) return fail(PBGPU_ERR_NOMEM, "host allocation failed");
  uint64_t o = 0;
  memcpy(t, hdr.data(), hdr.size()); o += hdr.size();
  for (auto& p : parts) { memcpy(t + o, p.data(), p.size()); o += p.size(); }
  t[o] = 0;
  *text = t; *len = o;
  return PBGPU_OK;
  API_CATCH
}

void pbgpu_free_text(char* text) { free(text); }

}  // extern "C"
