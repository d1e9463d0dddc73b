// pbgpu_host.h -- host-side objects behind the C ABI (include/pbgpu.h),
// shared by pbgpu_api.hip (index, aligner, batch pipeline), pbgpu_format.hip
// (device coords text) and pbgpu_run.hip (the file-to-file driver).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "../../include/pbgpu.h"
#include "pbgpu_internal.h"

using namespace pbgpu;

// ------------------------------------------------------------ error state
extern thread_local std::string g_err;  // pbgpu_api.hip
inline pbgpu_status fail(pbgpu_status s, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return s;
}
struct hip_error : std::runtime_error {
  hipError_t e;
  hip_error(hipError_t e_, const char* what) : std::runtime_error(what), e(e_) {}
};
// PBGPU_DEBUG_STALL=1: report any HIP call that blocks the host for more than half a second
// (file:line and the call), to find where a slow run waits
bool stall_debug();
bool stall_debug_allocs();  // PBGPU_DEBUG_STALL=2: also every device allocation
double stall_threshold_s();  // PBGPU_DEBUG_STALL_MS: the report threshold (default 500 ms)
void stall_report(double seconds, const char* call, const char* file, int line);
// PBGPU_DEBUG_STALL=2: one line per device allocation with its size and the caller's
// offset in libpbgpu.so (nm -C maps it to the function that grew the buffer)
void alloc_note(size_t bytes, const void* caller);
#define HIPCHK(x)                                                                                      \
  do {                                                                                                 \
    const bool _dbg = stall_debug();                                                                   \
    const auto _t0 = _dbg ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{}; \
    hipError_t _e = (x);                                                                               \
    if (_dbg) {                                                                                        \
      const double _dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - _t0).count(); \
      if (_dt > stall_threshold_s()) stall_report(_dt, #x, __FILE__, __LINE__);                                        \
    }                                                                                                  \
    if (_e != hipSuccess) {                                                                            \
      char _b[512];                                                                                    \
      snprintf(_b, sizeof _b, "%s failed at %s:%d: %s", #x, __FILE__, __LINE__, hipGetErrorString(_e)); \
      throw hip_error(_e, _b);                                                                         \
    }                                                                                                  \
  } while (0)
// a call whose status is ignored (frees), timed like HIPCHK under PBGPU_DEBUG_STALL
#define HIPFREE(x)                                                                                     \
  do {                                                                                                 \
    const bool _dbg = stall_debug();                                                                   \
    const auto _t0 = _dbg ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{}; \
    (void)(x);                                                                                         \
    if (_dbg) {                                                                                        \
      const double _dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - _t0).count(); \
      if (_dt > stall_threshold_s()) stall_report(_dt, #x, __FILE__, __LINE__);                                        \
    }                                                                                                  \
  } while (0)
struct bad_input : std::runtime_error { using std::runtime_error::runtime_error; };

// n strings in one allocation: string i is blob[off[i], off[i + 1] - 1), NUL-terminated
// (50M super-read names at C5: one blob frees at once, 100M std::strings did not)
struct NameTable {
  std::vector<char> blob;
  std::vector<uint64_t> off{0};
  size_t size() const { return off.size() - 1; }
  std::string_view operator[](size_t i) const { return std::string_view(blob.data() + off[i], off[i + 1] - off[i] - 1); }
  const char* c_str(size_t i) const { return blob.data() + off[i]; }
  void push_back(const char* s, size_t n) {
    blob.insert(blob.end(), s, s + n);
    blob.push_back(0);
    off.push_back(blob.size());
  }
  void push_back(std::string_view s) { push_back(s.data(), s.size()); }
};
struct pbgpu_comm {  // an RCCL communicator of the sharded-index count exchange
  ncclComm_t comm = nullptr;
  int device = 0;
  int n_ranks = 1;
  uint64_t last_bytes = 0;  // payload of the last count all-reduce (count_pack.h)
};
struct unsupported : std::runtime_error { using std::runtime_error::runtime_error; };

#define API_TRY try { (void)hipGetLastError();  /* launch checks below see only this call's errors */
#define API_CATCH                                                                 \
  }                                                                               \
  catch (const hip_error& e) {                                                    \
    return fail(e.e == hipErrorOutOfMemory ? PBGPU_ERR_NOMEM : PBGPU_ERR_DEVICE, "%s", e.what()); \
  }                                                                               \
  catch (const bad_input& e) { return fail(PBGPU_ERR_IO, "%s", e.what()); }       \
  catch (const unsupported& e) { return fail(PBGPU_ERR_UNSUPPORTED, "%s", e.what()); } \
  catch (const std::bad_alloc&) { return fail(PBGPU_ERR_NOMEM, "host allocation failed"); } \
  catch (const std::exception& e) { return fail(PBGPU_ERR_INTERNAL, "%s", e.what()); }

// work() on `threads` host threads (this one included); an exception in any of
// them is rethrown here after all have joined (none may leave a std::thread)
template <typename F>
void run_parallel(int threads, F&& work) {
  std::mutex mu;
  std::exception_ptr first;
  auto guarded = [&]() {
    try {
      work();
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu);
      if (!first) first = std::current_exception();
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(guarded);
  guarded();
  for (auto& t : th) t.join();
  if (first) std::rethrow_exception(first);
}

// --------------------------------------------------------- device buffer
// Allocation accounting and sizing of the per-batch buffers.  Every device
// allocation (hipMalloc of a dbuf) and pinned host allocation is counted on the
// thread that makes it: in pbgpu_run each aligner runs on its own worker
// thread, so the counts after a worker's first batch are what the run path
// still allocates (pbgpu_run_stats.n_device_allocs_late; round-3 review: a
// growing buffer's hipFree + hipMalloc now and then blocked a cold run for
// seconds).  tl_grow_scale is set by the worker to batch_bases / the batch's
// target when the batch is a ramped one filled to its target (the first
// batches of a run are 1/8 .. 1/2 of a full batch; a batch cut short by the
// end of the input has no full batches after it and keeps 1):
// a per-batch buffer that must grow is then sized for a full batch with 1.5x
// headroom (a ramped first batch holds few reads, so its hit and record
// densities vary), and the full batches that follow allocate nothing.  Round 5:
// 1.5x, not 2x (a cold C2 create_mega_reads run held 63 GB of buffers); the
// per-hit buffers are also capped by the aligner's hit budget (ensure_capped),
// which pbgpu_run sets per aligner, so they never follow the ramp's estimate
// past it.
inline thread_local uint64_t tl_dev_allocs = 0, tl_pinned_allocs = 0, tl_dev_bytes = 0;
// device bytes held by this thread's allocations and their high-water mark (a worker's
// aligner: its working set; pbgpu_run_stats.device_peak_bytes sums the workers' peaks)
inline thread_local int64_t tl_dev_live = 0, tl_dev_peak = 0;
inline thread_local double tl_alloc_s = 0;   // seconds in hipMalloc / hipFree of dbufs
inline thread_local double tl_pinned_s = 0;  // seconds in the run path's hipHostMalloc / hipHostFree
inline double mono_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
inline thread_local double tl_grow_scale = 1.0;
inline size_t grow_target(size_t cnt) {
  const double s = tl_grow_scale;
  return s > 1.0 ? (size_t)((double)cnt * s * 1.5) + 1 : cnt + cnt / 4;
}
template <typename T>
struct dbuf {
  T* p = nullptr;
  size_t n = 0;
  dbuf() = default;
  dbuf(const dbuf&) = delete;
  dbuf& operator=(const dbuf&) = delete;
  ~dbuf() { release(); }
  void release() {
    if (p) {
      const double t = mono_s();
      HIPFREE(hipFree(p));
      tl_alloc_s += mono_s() - t;
      tl_dev_live -= (int64_t)(n * sizeof(T));
    }
    p = nullptr; n = 0;
  }
  __attribute__((noinline)) void alloc(size_t cnt) {
    release();
    if (cnt) {
      if (stall_debug_allocs()) alloc_note(cnt * sizeof(T), __builtin_return_address(0));
      const double t = mono_s();
      HIPCHK(hipMalloc((void**)&p, cnt * sizeof(T)));
      tl_alloc_s += mono_s() - t;
      ++tl_dev_allocs; tl_dev_bytes += cnt * sizeof(T);
      tl_dev_live += (int64_t)(cnt * sizeof(T)); tl_dev_peak = std::max(tl_dev_peak, tl_dev_live);
      n = cnt;
    }
  }
  // A per-batch buffer grows to at least twice its size (first: grow_target of the
  // request): a run's batches vary, and every reallocation is a device-wide hipFree
  // plus a hipMalloc, which now and then blocks for seconds (PBGPU_DEBUG_STALL)
  void ensure(size_t cnt) { if (cnt > n) alloc(std::max(grow_target(cnt), n + n / 2)); }
  // the same, never sized past cap (a buffer whose need is bounded: the per-hit buffers
  // by the hit budget of a sub-batch) unless cnt itself is
  void ensure_capped(size_t cnt, size_t cap) {
    if (cnt > n) alloc(std::max(cnt, std::min(std::max(grow_target(cnt), n + n / 2), cap)));
  }
  // a buffer whose size does not follow the batch's (never scaled by tl_grow_scale)
  void ensure_fixed(size_t cnt) { if (cnt > n) alloc(std::max(cnt + cnt / 4, 2 * n)); }
  // grow keeping the first `keep` elements (stream-ordered copy)
  __attribute__((noinline)) void grow_keep(size_t cnt, size_t keep, hipStream_t st) {
    if (cnt <= n) return;
    T* q = nullptr;
    const size_t nn = std::max(tl_grow_scale > 1.0 ? grow_target(cnt) : cnt, n + n / 2);
    if (stall_debug_allocs()) alloc_note(nn * sizeof(T), __builtin_return_address(0));
    const double t = mono_s();
    HIPCHK(hipMalloc((void**)&q, nn * sizeof(T)));
    tl_alloc_s += mono_s() - t;
    ++tl_dev_allocs; tl_dev_bytes += nn * sizeof(T);
    tl_dev_live += (int64_t)(nn * sizeof(T)); tl_dev_peak = std::max(tl_dev_peak, tl_dev_live);
    if (p && keep) HIPCHK(hipMemcpyAsync(q, p, keep * sizeof(T), hipMemcpyDeviceToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    release();
    p = q; n = nn;
  }
  size_t bytes() const { return n * sizeof(T); }
  void swap(dbuf& o) { std::swap(p, o.p); std::swap(n, o.n); }
};

// scan scratch (a few words per tile of the scanned array): 1 MB at least, so
// that a batch's later and larger scans do not grow it one by one
inline void* temp_storage(dbuf<uint8_t>& t, size_t bytes) {
  t.ensure_fixed(std::max<size_t>(bytes, 1 << 20));
  return t.p;
}


// create_mega_reads' super-read names as unitig lists and the unitig lengths on one
// device (pbgpu_aligner_set_graph), shared by every aligner of the index that is
// given the same arrays (content hash): one copy per device, not one per stream
struct GraphNames {
  uint64_t hash = 0, n_sr = 0, n_units = 0, n_ul = 0;
  dbuf<uint64_t> noff;
  dbuf<uint32_t> units;
  dbuf<int32_t> ul;
};

// ------------------------------------------------------------------ index
struct pbgpu_index {
  int device = 0;
  uint32_t k = 0, psa_min = 0;
  uint64_t n = 0, n_sr = 0, n_kmers = 0, n_occ = 0, buckets = 0;
  double build_seconds = 0;
  NameTable name_fwd, name_bwd;
  std::vector<uint64_t> sr_start;            // host copy
  dbuf<uint64_t> text, d_sr_start, occ;
  dbuf<uint32_t> occ_sr;  // IndexView::occ_sr (PBGPU_OCC_SR=1), derived from occ
  dbuf<ulonglong2> table;
  dbuf<uint32_t> sr_uoff, sr_uids;
  // presence filter of the coarse table's k-mers (k_seed), 2^filt_log2 words; none if empty
  dbuf<uint64_t> filt;
  uint32_t filt_log2 = 0;
  // index sharded by super-read range: this shard holds super-reads
  // [sr_begin, sr_end) (device arrays use local ids) plus a k-1-base seam
  uint32_t shard = 0, n_shards = 1;
  uint64_t sr_begin = 0, sr_end = 0, n_total = 0;
  std::vector<uint64_t> gstart;   // global text offsets of all super-reads (host)
  uint64_t null_ptr = 0;          // empty occurrence header: k-mers absent from this shard
  // fine (-F) sub-index: same table / occurrence layout over fine_k-mers
  uint32_t fk = 0;
  uint64_t f_buckets = 0, f_kmers = 0, f_occ = 0;
  dbuf<uint64_t> f_occv;
  dbuf<ulonglong2> f_table;
  // super-read names on the device (device coords text, pbgpu_format.hip), built on first use
  std::mutex names_mu;
  bool names_ready = false;
  dbuf<char> d_name_fwd, d_name_bwd;
  dbuf<uint64_t> d_name_fwd_off, d_name_bwd_off;
  // the graph names of this index's aligners (GraphNames), guarded by names_mu
  std::shared_ptr<GraphNames> graph_names;
  IndexView view() const {
    IndexView v;
    v.text = text.p; v.n = n; v.sr_start = d_sr_start.p; v.n_sr = (uint32_t)(sr_end - sr_begin); v.k = k;
    v.table = table.p; v.bucket_mask = buckets - 1; v.occ = occ.p; v.sr_uoff = sr_uoff.p; v.sr_uids = sr_uids.p;
    v.occ_sr = occ_sr.n ? occ_sr.p : nullptr;
    v.filt = filt.n ? filt.p : nullptr; v.filt_shift = 64 - filt_log2;
    return v;
  }
  IndexView fine_view() const {
    IndexView v = view();
    v.k = fk; v.table = f_table.p; v.bucket_mask = f_buckets - 1; v.occ = f_occv.p; v.occ_sr = nullptr;
    v.filt = nullptr;
    return v;
  }
  uint64_t device_bytes() const {
    return text.bytes() + d_sr_start.bytes() + occ.bytes() + table.bytes() + sr_uoff.bytes() + sr_uids.bytes() +
           f_occv.bytes() + f_table.bytes() + filt.bytes() + occ_sr.bytes();
  }
};

// ---------------------------------------------------------------- aligner
struct pbgpu_reads {
  pbgpu_aligner* owner = nullptr;
  int device = 0;  // kept here: the owner may be freed first
  uint64_t n_reads = 0, n_bases = 0;
  std::vector<uint64_t> h_off;
  dbuf<uint8_t> seq;
  dbuf<uint64_t> off;
  // read names (up to the first whitespace) for the device coords text
  bool has_names = false;
  dbuf<char> names;
  dbuf<uint64_t> name_off;
  std::vector<uint64_t> h_name_off;
};

struct pbgpu_aligner {
  const pbgpu_index* ix = nullptr;
  int device = 0;
  pbgpu_align_params prm{};
  AlignParamsDev P{};
  LisParams lp{};
  hipStream_t st = nullptr;
  dbuf<int32_t> ul, sr_ul;  // unitig lengths; the same resolved along every super-read name (k_sr_ul)
  dbuf<SrMeta> sr_meta;     // per super-read of the index: AlignParamsDev::sr_meta (k_sr_meta)
  // per-batch buffers
  dbuf<KRec> krec;
  dbuf<uint32_t> n_kept, thr, rec_per_read, rec_cursor, order, counters;
  dbuf<uint2> ovf_items;
  dbuf<uint32_t> ovf_grow;
  dbuf<uint32_t> rcur;
  dbuf<uint64_t> sort_scratch;  // k_rec_sort keys of reads above its LDS capacity: 6 words per record
  dbuf<uint2> rec_tiles;        // (read, tile) work items of those reads (carved from the dead hit buffers)
  dbuf<uint2> pinfo;            // per permuted strand: {first hit, hits} (lis_stage's strand order)
  dbuf<uint2> bmeta;            // per read of the call: {bucket offsets base, P0} of bucketed reads (GroupOut)
  dbuf<uint32_t> boff;          // the bucketed reads' bucket offsets (P0 + 1 each)
  dbuf<uint32_t> rec_tile_ctr;  // their count and the longest such read
  dbuf<uint64_t> nhits, hit_off, rec_off, huge_elems;
  dbuf<int2> hits;
  dbuf<ChainDesc> chains;
  dbuf<uint32_t> perm;
  dbuf<int2> X, pts;
  dbuf<uint8_t> nodes, nodes32;  // LNode<uint16_t> per hit / LNode<uint32_t> per hit of the long strands
  dbuf<uint32_t> n32shift;       // per strand item: its first node chunk in nodes32 (k_node32_place)
  dbuf<unsigned long long> n32total;
  dbuf<uint32_t> lisl, hist, slen;
  dbuf<uint32_t> redo[3];
  dbuf<Rec> recs, recs_sorted;
  dbuf<uint32_t> rec_read;  // the read of every record of recs (written with it)
  dbuf<uint32_t> rec_slot;  // its rank among its read's records (ChainOut.rec_slot)
  dbuf<int32_t> info_m, info_b;
  dbuf<uint8_t> tmp;
  dbuf<uint32_t> gtable;
  dbuf<unsigned long long> stats, info_count;
  // last result
  uint64_t last_reads = 0, last_records = 0, last_info = 0;
  bool have_result = false;
  // stats
  pbgpu_stats acc{};
  hipEvent_t ev[20]{};
  hipStream_t g_side = nullptr;  // the overlap graph's long-read tier (set_graph)
  hipEvent_t g_fork = nullptr, g_join = nullptr, g_join2 = nullptr;
  hipStream_t g_side2 = nullptr;  // the overlap graph's 1025-2048-record tier
  hipStream_t grp_side = nullptr;  // the group stage's 16-wave tier (PBGPU_GROUP_OVERLAP)
  hipEvent_t grp_fork = nullptr, grp_join = nullptr;
  uint64_t hit_budget = 4000000000ull, rec_hint = 0, info_per_chain = 32;
  // records a chain yields (kept by the filters), learnt from the sub-batches so far: the
  // record buffers of a sub-batch are sized by it instead of one record per chain (C4: 278 M
  // chains in a sub-batch, 27 GB of records and 71 GB of kmers_info sized by the chains ran
  // the device out of memory beside its 126-GB index); an overflow redoes the sub-batch and
  // resets it to 1
  double rec_per_chain = 1.0;
  uint32_t bkt_log2 = 13;    // the bucket items' table size of the current sub-batch (group stage)
  bool cph_learned = false;  // chains_per_hit measured on a sub-batch (the hit budget's margin)
  // pbgpu_run: the most bases a batch holds (0 = unknown): the per-base buffers never grow past it
  uint64_t base_cap = 0;
  double chains_per_hit = 1.0 / 80;  // k_group tier estimate (C2: 1.1 x 1/90), refined after every batch
  dbuf<uint2> ovf_list, read_list;  // k_group work items (group_item): the overflow round's, the launch's
  std::vector<uint32_t> h_order, h_class;  // host scratch of the group stage's read order
  std::vector<uint2> h_small, h_big, h_items, h_bkt, h_split, h_bmeta;
  std::vector<uint64_t> h_hoff;
  // sharded index: per-base k-mer counts of the current batch (SEED_COUNTS, then summed)
  dbuf<uint32_t> gcount;
  dbuf<uint32_t> gcount16;  // the counts packed two per u32 for the all-reduce (count_pack.h)
  uint64_t gcount_n = ~0ull;
  // -F: fine aligner pass (params of k_coords with align_k = fine_k, forward, unfiltered)
  bool fine = false;
  AlignParamsDev PF{};
  LisParams lpf{};
  dbuf<FineWin> fwin;
  dbuf<uint64_t> fwk[2], fread_hits;
  dbuf<uint32_t> fwi[2], fkeys[2], lstart, lend, emit_of;
  dbuf<int2> X2;
  // --details: final coarse lists of the last alignment, in sub-batch chain order
  bool details = false;
  struct {
    std::vector<uint32_t> read, sr, nf;
    std::vector<uint64_t> hoff{0};
    std::vector<int32_t> hits;
    std::vector<uint8_t> lis;
    void clear() { read.clear(); sr.clear(); nf.clear(); hoff.assign(1, 0); hits.clear(); lis.clear(); }
  } det;
  // create_mega_reads' overlap graph (pbgpu_aligner_set_graph): names and unitig lengths
  // on the device, per-batch scratch, the last alignment's nodes
  bool graph = false;
  double g_play = 0, g_errors = 0;
  uint32_t g_k = 0;
  int g_bases = 0;
  std::shared_ptr<GraphNames> g_names;  // shared with the index's other aligners
  dbuf<uint64_t> g_poff;
  dbuf<uint32_t> g_pre, g_sizes;
  dbuf<GDesc> g_desc;
  dbuf<uint32_t> g_spo;
  dbuf<double> g_fd;
  dbuf<uint32_t> g_fu0;
  dbuf<double> g_bmax;
  dbuf<double2> g_imp;
  dbuf<GraphNode> g_out;
  dbuf<uint32_t> g_ecnt;
  dbuf<uint64_t> g_eoff;
  dbuf<uint2> g_edges, g_eovf;
  dbuf<uint32_t> g_maxn;
  dbuf<uint64_t> g_ovf, g_ovf_list;
  // mega-reads on the device (pbgpu_graph_params.mega_reads)
  bool g_mega = false;
  int g_tiling = 0, g_trim = 0;
  double g_min_density = 0, g_min_len = 0;
  dbuf<MegaTmp> g_cand;
  dbuf<int32_t> g_ord;
  dbuf<double2> g_ivs;
  dbuf<MegaOut> g_mo, g_mc;
  dbuf<uint32_t> g_mcount, g_munits, g_nhost;
  dbuf<uint8_t> g_mhost;
  dbuf<uint64_t> g_moff;
  dbuf<unsigned long long> g_uused;
  uint64_t g_mtotal = 0, g_munits_used = 0, g_hosts = 0;  // the last alignment's
  // the reads left to the host, packed: read offsets, records, nodes, info
  dbuf<uint32_t> g_rsize, g_isize;
  dbuf<uint64_t> g_hroff, g_hioff;
  dbuf<Rec> g_hrec;
  dbuf<GraphNode> g_hgraph;
  dbuf<int32_t> g_hinfo;
  uint64_t g_hrecs = 0, g_hinfos = 0;
  // device coords text of the last alignment (pbgpu_format.hip)
  dbuf<uint32_t> fmt_len;
  dbuf<uint64_t> fmt_pos;
  dbuf<char> text;
  uint64_t text_len = 0;
};

// the whole device path on a resident batch (seed_mode: SEED_WHOLE = 0; the
// sharded-index modes pass SEED_FINISH and the summed counts)
void aligner_pipeline(pbgpu_aligner* al, const pbgpu_reads* rd, int seed_mode = 0, uint32_t* gcount = nullptr);
void upload_reads_into(pbgpu_aligner* al, const pbgpu_read_batch* b, pbgpu_reads* r);
uint64_t format_device_text(pbgpu_aligner* al, const pbgpu_reads* rd, int compact, int zero_match);
