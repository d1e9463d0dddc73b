// pbgpu_run.hip -- the file-to-file driver behind pbgpu_run (include/pbgpu.h):
// the reference's jf_aligner main loop (jf_aligner.cc:205-230) and worker
// (print_alignments, :110-159) re-laid out for GPUs.
//
//   reader thread   PacBio FASTA/FASTQ (plain or gzip, zlib) -> batches of
//                   ~batch_bases bases: bases, offsets, read names
//   worker threads  one per aligner (aligners_per_device per listed index):
//                   take the next batch (dynamic assignment), upload into
//                   grow-only device buffers, run the device path, format the
//                   coords text on the device (pbgpu_format.hip), copy it into
//                   a pinned host buffer
//   writer thread   writes the texts in batch order (one write() stream: on
//                   the GPU box one stream writes the page cache at ~10 GB/s
//                   and parallel pwrite()s do not go faster, the inode lock
//                   serializes them -- profiles/r02_probe_io.txt)
// Backpressure: the pinned pool holds workers + 2 buffers, so a slow writer
// stalls the workers instead of growing memory.  The first error of any
// thread stops all of them and is returned (no exit() from a worker).
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <atomic>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <thread>

#include "pbgpu_host.h"

namespace {

// PBGPU_TIMELINE=1: one stderr line per batch and stage (seconds since the run began), to
// see where a run's wall goes (fill, first-batch allocations, tail)
static bool timeline() {
  static const bool on = getenv("PBGPU_TIMELINE") && atoi(getenv("PBGPU_TIMELINE"));
  return on;
}
static double g_tl0 = 0;
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ------------------------------------------------------------ run state
struct RunState {
  std::mutex mu;
  bool stop = false;
  pbgpu_status status = PBGPU_OK;
  std::string msg;
  std::condition_variable* cvs[4] = {};
  std::atomic<bool>* any_stop = nullptr;  // shared by the parts of a run: one failure stops them all
  void fail(pbgpu_status s, const std::string& m) {
    {
      std::lock_guard<std::mutex> lk(mu);
      if (status == PBGPU_OK) { status = s; msg = m; }
      stop = true;
    }
    if (any_stop) any_stop->store(true);
    for (auto* cv : cvs) if (cv) cv->notify_all();
  }
  bool stopped() {
    if (any_stop && any_stop->load()) return true;
    std::lock_guard<std::mutex> lk(mu);
    return stop;
  }
};

// condition waits re-check every 50 ms: RunState::fail notifies without the
// waiters' mutexes, so a notification can slip between a check and the wait
template <class L, class P>
void wait_until(std::condition_variable& cv, L& lk, P pred) {
  while (!cv.wait_for(lk, std::chrono::milliseconds(50), pred)) {
  }
}

// the API_CATCH classification, for a thread's exception
void record_exception(RunState& rs) {
  try {
    throw;
  } catch (const hip_error& e) {
    rs.fail(e.e == hipErrorOutOfMemory ? PBGPU_ERR_NOMEM : PBGPU_ERR_DEVICE, e.what());
  } catch (const bad_input& e) {
    rs.fail(PBGPU_ERR_IO, e.what());
  } catch (const unsupported& e) {
    rs.fail(PBGPU_ERR_UNSUPPORTED, e.what());
  } catch (const std::bad_alloc&) {
    rs.fail(PBGPU_ERR_NOMEM, "host allocation failed");
  } catch (const std::exception& e) {
    rs.fail(PBGPU_ERR_INTERNAL, e.what());
  }
}

// ------------------------------------------------------------ pinned memory
struct PinnedVec {  // growable pinned byte buffer (H2D at full PCIe rate, no staging)
  char* p = nullptr;
  size_t cap = 0, n = 0;
  PinnedVec() = default;
  PinnedVec(const PinnedVec&) = delete;
  PinnedVec& operator=(const PinnedVec&) = delete;
  ~PinnedVec() { if (p) (void)hipHostFree(p); }
  void reserve(size_t c) {
    if (c <= cap) return;
    const size_t nc = std::max(c, cap + cap / 2);
    char* q = nullptr;
    const double t0 = mono_s();
    HIPCHK(hipHostMalloc((void**)&q, nc, hipHostMallocDefault));
    ++tl_pinned_allocs;
    if (n) memcpy(q, p, n);
    if (p) HIPFREE(hipHostFree(p));
    tl_pinned_s += mono_s() - t0;
    p = q;
    cap = nc;
  }
  void append(const char* s, size_t len) {
    if (n + len > cap) reserve(n + len);
    memcpy(p + n, s, len);
    n += len;
  }
};

// ------------------------------------------------------------ input
// Lines of a sequence of files: plain files by read(), gzip (magic 1f 8b) by zlib.
// With a byte range [begin, ...) over the concatenation of plain files, the
// source starts at the first line that begins at or after `begin`; line_off()
// is the global offset of the last line returned (part files, pbgpu_run_params.n_parts).
class LineSource {
 public:
  explicit LineSource(const std::vector<std::string>& paths, uint64_t begin = 0, bool ranged = false)
      : paths_(paths), begin_(begin) {
    buf_.resize(1 << 24);
    if (ranged) {
      uint64_t b = 0;
      for (const auto& p : paths_) { base_of_.push_back(b); b += file_size(p); }
      // whole files before `begin` are skipped
      while (fi_ < paths_.size() && (fi_ + 1 >= paths_.size() ? b : base_of_[fi_ + 1]) <= begin_) ++fi_;
    }
  }
  ~LineSource() { close_cur(); }
  static uint64_t file_size(const std::string& path) {
    struct stat st {};
    if (stat(path.c_str(), &st) != 0) throw bad_input("Can't open PacBio file '" + path + "'");
    return (uint64_t)st.st_size;
  }
  // next line without its '\n' (pointer valid until the next call); false at
  // the end of the current file -- next_file() then opens the next one
  bool line(const char*& p, size_t& len) {
    for (;;) {
      if (pos_ < end_) {
        const char* s = buf_.data() + pos_;
        const char* nl = (const char*)memchr(s, '\n', end_ - pos_);
        line_off_ = file_base_ + buf_off_ + pos_;
        if (nl) {
          p = s; len = (size_t)(nl - s);
          pos_ += len + 1;
          return true;
        }
        if (eof_) {  // last line without a newline
          p = s; len = end_ - pos_;
          pos_ = end_;
          return true;
        }
      } else if (eof_) {
        return false;
      }
      fill();
    }
  }
  uint64_t line_off() const { return line_off_; }
  bool next_file() {
    close_cur();
    if (fi_ >= paths_.size()) return false;
    const std::string& path = paths_[fi_];
    file_base_ = base_of_.empty() ? 0 : base_of_[fi_];
    ++fi_;
    fd_ = open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw bad_input("Can't open PacBio file '" + path + "'");
    unsigned char mg[2] = {0, 0};
    const ssize_t m = pread(fd_, mg, 2, 0);
    pos_ = end_ = 0;
    buf_off_ = 0;
    eof_ = false;
    if (m == 2 && mg[0] == 0x1f && mg[1] == 0x8b) {
      if (begin_ || !base_of_.empty()) throw unsupported("part files need plain (not gzip) PacBio input");
      gz_ = gzdopen(fd_, "rb");
      if (!gz_) throw bad_input("Can't open gzip PacBio file '" + path + "'");
      fd_ = -1;  // owned by gz_
      gzbuffer(gz_, 1 << 20);
    }
    if (begin_ > file_base_) {  // the range starts inside this file: from the line after offset begin - 1
      const uint64_t at = begin_ - file_base_ - 1;
      if (lseek(fd_, (off_t)at, SEEK_SET) < 0) throw bad_input("seek failed in PacBio file '" + path + "'");
      buf_off_ = at;
      const char* p;
      size_t len;
      line(p, len);  // the rest of the line holding byte begin - 1 (empty if it is a '\n')
    }
    begin_ = 0;  // later files are read whole
    return true;
  }

 private:
  void close_cur() {
    if (gz_) { gzclose(gz_); gz_ = nullptr; }
    if (fd_ >= 0) { close(fd_); fd_ = -1; }
  }
  void fill() {
    if (pos_ > 0) {  // keep the partial line at the front
      memmove(buf_.data(), buf_.data() + pos_, end_ - pos_);
      buf_off_ += pos_;
      end_ -= pos_;
      pos_ = 0;
    }
    if (end_ == buf_.size()) buf_.resize(buf_.size() * 2);  // a line longer than the buffer
    const size_t want = std::min<size_t>(buf_.size() - end_, 1u << 30);
    ssize_t got;
    if (gz_) {
      got = gzread(gz_, buf_.data() + end_, (unsigned)want);
      if (got < 0) {
        int e;
        throw bad_input(std::string("read error in PacBio file: ") + gzerror(gz_, &e));
      }
    } else {
      do { got = read(fd_, buf_.data() + end_, want); } while (got < 0 && errno == EINTR);
      if (got < 0) throw bad_input(std::string("read error in PacBio file: ") + strerror(errno));
    }
    if (got == 0) eof_ = true;
    end_ += (size_t)got;
  }
  std::vector<std::string> paths_;
  uint64_t begin_ = 0;
  std::vector<uint64_t> base_of_;  // global offset of each file (range mode)
  uint64_t file_base_ = 0, buf_off_ = 0, line_off_ = 0;  // current file's offset, file offset of buf_[0]
  size_t fi_ = 0;
  int fd_ = -1;
  gzFile gz_ = nullptr;
  std::vector<char> buf_;
  size_t pos_ = 0, end_ = 0;
  bool eof_ = true;
};

struct Batch {
  uint64_t id = 0;
  // a ramped batch filled to its target: the full batches after it are this much larger
  // (tl_grow_scale while it is aligned); 1 for full batches and for the input's last one
  double grow_scale = 1.0;
  PinnedVec seq;
  std::string names;
  std::vector<uint64_t> off{0}, name_off{0};
  std::vector<std::string> headers;  // full header lines (--details only)
  uint64_t n() const { return off.size() - 1; }
  void clear() {
    seq.n = 0;
    names.clear();
    off.assign(1, 0);
    name_off.assign(1, 0);
    headers.clear();
  }
};

// whole_sequence_parser semantics (jellyfish 2.x, as used at jf_aligner.cc:206-207):
// FASTA header = line after '>', sequence = the following lines concatenated;
// FASTQ '@' header, one sequence line, '+' line, quality line.
// With a range [begin, end) (part files): the reads whose FASTA header line
// starts in it.
class ReadParser {
 public:
  ReadParser(const std::vector<std::string>& paths, bool keep_headers, uint64_t begin = 0, uint64_t end = ~0ull)
      : src_(paths, begin, begin != 0 || end != ~0ull), keep_(keep_headers), end_(end), ranged_(begin != 0 || end != ~0ull) {
    open_ = src_.next_file();
    if (ranged_) {  // skip to the first header of the range (FASTA only)
      const char* p;
      size_t len;
      for (;;) {
        while (open_ && !src_.line(p, len)) open_ = src_.next_file();
        if (!open_) break;
        if (len && p[0] == '@') throw unsupported("part files need FASTA PacBio input (a FASTQ record start is ambiguous)");
        if (len && p[0] == '>') { pending_.assign(p, len); pending_off_ = src_.line_off(); have_pending_ = true; break; }
      }
    }
  }
  // appends up to ~batch_bases bases worth of reads; false when nothing was added
  bool fill(Batch& b, uint64_t batch_bases) {
    while (open_ && b.seq.n < batch_bases) {
      if (!one(b)) open_ = src_.next_file();
    }
    return b.n() > 0;
  }

 private:
  bool one(Batch& b) {
    const char* p;
    size_t len;
    uint64_t hoff;
    if (have_pending_) {
      have_pending_ = false;
      hdr_.swap(pending_);
      hoff = pending_off_;
    } else {
      do {
        if (!src_.line(p, len)) return false;
      } while (len == 0);
      hdr_.assign(p, len);
      hoff = src_.line_off();
    }
    if (ranged_ && hoff >= end_) { open_ = false; return false; }  // the next part's read
    const char c0 = hdr_[0];
    if (c0 != '>' && c0 != '@') throw bad_input("PacBio input is neither FASTA nor FASTQ");
    if (ranged_ && c0 == '@') throw unsupported("part files need FASTA PacBio input (a FASTQ record start is ambiguous)");
    if (c0 == '@') {
      if (src_.line(p, len)) b.seq.append(p, len);
      src_.line(p, len);  // '+'
      src_.line(p, len);  // quality
    } else {
      while (src_.line(p, len)) {
        if (len && p[0] == '>') { pending_.assign(p, len); pending_off_ = src_.line_off(); have_pending_ = true; break; }
        b.seq.append(p, len);
      }
    }
    // name = header up to the first whitespace (jf_aligner.cc:133-134)
    const size_t nl = strcspn(hdr_.c_str() + 1, " \t\n\v\f\r");
    b.names.append(hdr_, 1, nl);
    b.name_off.push_back(b.names.size());
    b.off.push_back(b.seq.n);
    if (keep_) b.headers.emplace_back(hdr_, 1);
    return true;
  }
  LineSource src_;
  bool keep_;
  uint64_t end_;
  bool ranged_;
  bool open_ = false;
  bool have_pending_ = false;
  uint64_t pending_off_ = 0;
  std::string hdr_, pending_;
};

// ------------------------------------------------------------ plumbing
template <class T>
class Queue {  // bounded, closable, stops with the run
 public:
  Queue(size_t cap, RunState& rs, int slot) : cap_(cap), rs_(rs) { rs.cvs[slot] = &cv_; }
  bool push(T v) {
    std::unique_lock<std::mutex> lk(mu_);
    wait_until(cv_, lk, [&] { return q_.size() < cap_ || rs_.stopped(); });
    if (rs_.stopped()) return false;
    q_.push_back(std::move(v));
    cv_.notify_all();
    return true;
  }
  bool pop(T& v) {
    std::unique_lock<std::mutex> lk(mu_);
    wait_until(cv_, lk, [&] { return !q_.empty() || closed_ || rs_.stopped(); });
    if (rs_.stopped() || q_.empty()) return false;
    v = std::move(q_.front());
    q_.pop_front();
    cv_.notify_all();
    return true;
  }
  void close() {
    std::lock_guard<std::mutex> lk(mu_);
    closed_ = true;
    cv_.notify_all();
  }

 private:
  size_t cap_;
  RunState& rs_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<T> q_;
  bool closed_ = false;
};

struct Pinned {
  char* p = nullptr;
  size_t cap = 0;
};

// Text buffers: they grow to the largest text seen and live as long as the
// runner.  Batch id may take one only while id < written + n (written =
// batches the writer has finished): the batch the writer waits for can then
// always get a buffer, however far the other workers run ahead.
class TextPool {
 public:
  explicit TextPool(size_t n) : n_(n) { free_.resize(n); }
  ~TextPool() { for (auto& b : free_) if (b.p) (void)hipHostFree(b.p); }
  void start(RunState* rs) {  // a new run: batch ids restart at 0
    std::lock_guard<std::mutex> lk(mu_);
    rs_ = rs;
    written_ = 0;
    rs->cvs[1] = &cv_;
  }
  bool get(uint64_t id, size_t need, Pinned& out) {
    std::unique_lock<std::mutex> lk(mu_);
    wait_until(cv_, lk, [&] { return (!free_.empty() && id < written_ + n_) || rs_->stopped(); });
    if (rs_->stopped()) return false;
    out = free_.back();
    free_.pop_back();
    lk.unlock();
    if (out.cap < need) {
      if (out.p) HIPFREE(hipHostFree(out.p));
      out.p = nullptr;
      out.cap = 0;
      const size_t cap = grow_target(need);
      hipError_t e = hipSuccess;
      const double t0 = mono_s();
      HIPFREE(e = hipHostMalloc((void**)&out.p, cap, hipHostMallocDefault));
      tl_pinned_s += mono_s() - t0;
      if (e != hipSuccess) { put(Pinned{}, false); HIPCHK(e); }
      ++tl_pinned_allocs;
      out.cap = cap;
    }
    return true;
  }
  void advance() {  // a batch written without a pinned buffer (records consumer)
    std::lock_guard<std::mutex> lk(mu_);
    ++written_;
    cv_.notify_all();
  }
  void put(Pinned b, bool written) {
    std::lock_guard<std::mutex> lk(mu_);
    free_.push_back(b);
    if (written) ++written_;
    cv_.notify_all();
  }

 private:
  size_t n_;
  uint64_t written_ = 0;
  RunState* rs_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Pinned> free_;
};

struct Done {  // a batch's formatted output, waiting for its turn
  Pinned text;       // device-formatted coords (pinned)
  uint64_t len = 0;
  char* mtext = nullptr;  // or: host text from the records consumer (malloc'd)
  std::string details;
};

void write_all(int fd, const char* p, uint64_t n, const char* what) {
  while (n) {
    const ssize_t w = write(fd, p, (size_t)std::min<uint64_t>(n, 1ull << 30));
    if (w < 0) {
      if (errno == EINTR) continue;
      throw bad_input(std::string("write to ") + what + " failed: " + strerror(errno));
    }
    p += w;
    n -= (uint64_t)w;
  }
}

// CPUs of the NUMA node the GPU hangs off (sysfs), within this process's
// allowed set; empty when unknown.  The writer copies every coords byte from
// pinned memory into the page cache: on the GPU's node both are local.
std::vector<int> gpu_node_cpus(int device) {
  std::vector<int> out;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return out;
  for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
  int node = -1;
  {
    FILE* f = fopen((std::string("/sys/bus/pci/devices/") + bus + "/numa_node").c_str(), "r");
    if (!f) return out;
    if (fscanf(f, "%d", &node) != 1) node = -1;
    fclose(f);
  }
  if (node < 0) return out;
  FILE* f = fopen(("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str(), "r");
  if (!f) return out;
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) CPU_ZERO(&allowed);
  int a = 0, b = 0;
  char sep = 0;
  while (fscanf(f, "%d", &a) == 1) {
    b = a;
    if (fscanf(f, "%c", &sep) == 1 && sep == '-') {
      if (fscanf(f, "%d", &b) != 1) break;
      if (fscanf(f, "%c", &sep) != 1) sep = 0;
    }
    for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &allowed)) out.push_back(c);
    if (sep != ',') break;
  }
  fclose(f);
  return out;
}
void pin_to(const std::vector<int>& cpus) {
  if (cpus.empty()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus) CPU_SET(c, &set);
  (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}
}  // namespace

// Long-lived resources of the driver: aligners, their resident read buffers,
// the pinned batch and text buffers.  A server-style caller (bench.py) runs
// many files through one runner; the CLI runs one.
// The records of an aligner's last batch in pinned host memory, as a
// pbgpu_coords_batch view (the records consumer's input): no zero-filled
// vectors, no pageable staging copies; valid until the next download.
struct RecordsView {
  PinnedVec off, recs, km, kb, graph, moff, mega, munits, mhost;
  pbgpu_coords_batch c{};
  // on growth, room for the next batches of a ramp (PinnedVec grows by 1.5x)
  static void room(PinnedVec& v, uint64_t bytes) {
    if (v.cap < bytes) v.reserve(std::max<uint64_t>(grow_target(std::max<uint64_t>(bytes, 1)), 2 * bytes));
  }
  static void room_fixed(PinnedVec& v, uint64_t bytes) {  // (not scaled with the batch)
    if (v.cap < bytes) v.reserve(std::max<uint64_t>(bytes + bytes / 4, 2 * v.cap));
  }
  // With device mega-reads, everything a batch downloads is small and nearly fixed in
  // size: reserved when the runner is made, so that the first batches' pinned
  // allocations (a few ms each, serialized across the workers) do not stall the
  // pipeline.  Reads a batch: at most batch_bases / 1000 + 4096 (reads of 1 kb on
  // average), 4 mega-reads a read of 16 unitigs each; records and info of four reads
  // left to the host, 32 info entries a record.  A batch that needs more grows them.
  void reserve_mega(uint64_t batch_bases) {
    const uint64_t reads = batch_bases / 1000 + 4096, host_room = 4 * (uint64_t)(GRAPH_NMAX + 1);
    off.reserve((reads + 1) * 8); moff.reserve((reads + 1) * 8); mhost.reserve(reads + 1);
    mega.reserve(4 * reads * sizeof(MegaOut)); munits.reserve(64 * reads * 4);
    recs.reserve(host_room * sizeof(Rec)); graph.reserve(host_room * sizeof(GraphNode));
    km.reserve(host_room * 32 * 4); kb.reserve(host_room * 32 * 4);
  }
  void download(pbgpu_aligner* al) {
    const uint64_t n = al->last_reads;
    static_assert(sizeof(pbgpu_record) == sizeof(Rec), "record layout");
    c = pbgpu_coords_batch{};
    // device mega-reads: the records of the reads left to the host only, packed
    const bool dev_mega = al->graph && al->g_mega;
    const uint64_t nr = dev_mega ? al->g_hrecs : al->last_records, ni = dev_mega ? al->g_hinfos : al->last_info;
    const uint64_t* d_off = dev_mega ? al->g_hroff.p : al->rec_off.p;
    const Rec* d_rec = dev_mega ? al->g_hrec.p : al->recs_sorted.p;
    const GraphNode* d_graph = dev_mega ? al->g_hgraph.p : al->g_out.p;
    const int32_t* d_km = dev_mega ? al->g_hinfo.p : al->info_m.p;
    const int32_t* d_kb = dev_mega ? al->g_hinfo.p + al->g_hinfos + 1 : al->info_b.p;
    room(off, (n + 1) * 8);
    if (!dev_mega || al->g_hosts) HIPCHK(hipMemcpyAsync(off.p, d_off, (n + 1) * 8, hipMemcpyDeviceToHost, al->st));
    else memset(off.p, 0, (n + 1) * 8);
    // (with device mega-reads only the reads left to the host come down -- since round 5
    // only reads of more than GRAPH_NMAX_BIG records, or past PBGPU_GRAPH_NMAX in tests --:
    // room for four reads of GRAPH_NMAX records from the start, not scaled with the
    // batch -- sized by the batch it was a few hundred MB of pinned memory, ~50 ms of the
    // first batch's critical path -- and grown if a batch has more)
    const uint64_t host_room = 4 * (uint64_t)(GRAPH_NMAX + 1);
    const uint64_t nr_room = dev_mega ? std::max<uint64_t>(nr, host_room) : nr;
    const uint64_t ni_room =
        dev_mega ? std::max<uint64_t>(ni, host_room * (al->last_info / std::max<uint64_t>(1, al->last_records) + 2)) : ni;
    if (dev_mega) {
      room_fixed(recs, nr_room * sizeof(Rec)); room_fixed(km, ni_room * 4); room_fixed(kb, ni_room * 4);
    } else {
      room(recs, nr_room * sizeof(Rec)); room(km, ni_room * 4); room(kb, ni_room * 4);
    }
    if (nr) HIPCHK(hipMemcpyAsync(recs.p, d_rec, nr * sizeof(Rec), hipMemcpyDeviceToHost, al->st));
    if (ni) {
      HIPCHK(hipMemcpyAsync(km.p, d_km, ni * 4, hipMemcpyDeviceToHost, al->st));
      HIPCHK(hipMemcpyAsync(kb.p, d_kb, ni * 4, hipMemcpyDeviceToHost, al->st));
    }
    if (al->graph) {
      if (dev_mega) room_fixed(graph, nr_room * sizeof(GraphNode));
      else room(graph, nr_room * sizeof(GraphNode));
      if (nr) HIPCHK(hipMemcpyAsync(graph.p, d_graph, nr * sizeof(GraphNode), hipMemcpyDeviceToHost, al->st));
    }
    if (dev_mega) {
      const uint64_t nm = al->g_mtotal, nu = al->g_munits_used;
      room(moff, (n + 1) * 8); room(mhost, n + 1); room(mega, nm * sizeof(MegaOut)); room(munits, nu * 4);
      if (al->last_records) {
        HIPCHK(hipMemcpyAsync(moff.p, al->g_moff.p, (n + 1) * 8, hipMemcpyDeviceToHost, al->st));
        HIPCHK(hipMemcpyAsync(mhost.p, al->g_mhost.p, n, hipMemcpyDeviceToHost, al->st));
      } else {
        memset(moff.p, 0, (n + 1) * 8);
        memset(mhost.p, 0, n + 1);
      }
      if (nm) HIPCHK(hipMemcpyAsync(mega.p, al->g_mc.p, nm * sizeof(MegaOut), hipMemcpyDeviceToHost, al->st));
      if (nu) HIPCHK(hipMemcpyAsync(munits.p, al->g_munits.p, nu * 4, hipMemcpyDeviceToHost, al->st));
      c.mega_offsets = (const uint64_t*)moff.p; c.mega = (const pbgpu_mega_read*)mega.p;
      c.mega_units = (const uint32_t*)munits.p; c.mega_host = (const uint8_t*)mhost.p;
    }
    HIPCHK(hipStreamSynchronize(al->st));
    pbgpu_record* r = (pbgpu_record*)recs.p;
    if (al->ix->sr_begin)  // a shard's device super-read ids are local
      for (uint64_t i = 0; i < nr; ++i) r[i].sr_index += (uint32_t)al->ix->sr_begin;
    c.n_reads = n; c.n_records = nr; c.read_offsets = (const uint64_t*)off.p; c.records = r;
    c.n_info = ni; c.kmers_info = (const int32_t*)km.p; c.bases_info = (const int32_t*)kb.p;
    c.graph = al->graph ? (const pbgpu_graph_node*)graph.p : nullptr;
  }
};

// One output file's pipeline: its aligners (indices into the runner's), its
// batch buffers and pinned text pool (aligners + 2 each, recycled).
struct RunPart {
  std::vector<size_t> al;
  std::vector<std::unique_ptr<Batch>> batches;
  std::unique_ptr<TextPool> texts;
};

struct pbgpu_runner {
  std::vector<pbgpu_aligner*> al;
  std::vector<std::unique_ptr<RecordsView>> views;  // per aligner (records consumer runs)
  std::vector<std::unique_ptr<pbgpu_reads>> rd;
  bool details = false;
  bool side = false;  // a second output file (details, or the records consumer's side text)
  uint64_t batch_bases = 0;
  std::vector<RunPart> parts;  // one, or n_parts (part files)
  std::mutex run_mu;           // one run at a time
  // device working set (pbgpu_run_stats.device_peak_bytes): per device its used bytes
  // (hipMemGetInfo) before the aligners were made, and the most seen after any batch
  static constexpr int kMaxDev = 64;
  uint64_t dev_base[kMaxDev] = {};
  std::atomic<uint64_t> dev_peak[kMaxDev] = {};
  void note_device_use(int d) {
    size_t fr = 0, tot = 0;
    if (d < 0 || d >= kMaxDev || hipMemGetInfo(&fr, &tot) != hipSuccess) return;
    const uint64_t used = (uint64_t)(tot - fr);
    uint64_t cur = dev_peak[d].load();
    while (used > cur && !dev_peak[d].compare_exchange_weak(cur, used)) {}
  }
  ~pbgpu_runner() {
    rd.clear();
    for (auto* a : al) pbgpu_aligner_free(a);
  }
};

// One part's pipeline (all of the run unless part files): reader over the
// part's input range, its aligners' workers, the writer of its file(s).
static void run_part(pbgpu_runner* R, RunPart& part, const pbgpu_run_params* run, const std::vector<std::string>& paths,
                     uint64_t range_begin, uint64_t range_end, int cfd, int dfd, bool write_header, RunState& rs,
                     pbgpu_run_stats& S) {
  const bool details = R->details;
  const uint64_t batch_bases = R->batch_bases;
  const int hthreads = run->host_threads > 0 ? run->host_threads
                                             : (int)std::max(1u, std::thread::hardware_concurrency());
  const size_t W = part.al.size();
  Queue<Batch*> inq(W + 1, rs, 0);
  Queue<Batch*> freeq(part.batches.size() + 1, rs, 3);
  for (auto& b : part.batches) freeq.push(b.get());
  part.texts->start(&rs);
  std::mutex dmu;
  std::condition_variable dcv;
  rs.cvs[2] = &dcv;
  std::map<uint64_t, Done> done;
  uint64_t n_batches_total = ~0ull;  // set by the reader when it finishes
  std::mutex smu;                    // stats

  // PBGPU_RAMP: the first batch holds batch_bases >> ramp bases, doubling up to batch_bases
  const uint32_t ramp = getenv("PBGPU_RAMP") ? (uint32_t)atoi(getenv("PBGPU_RAMP")) : 3u;
  // PBGPU_WRITE_CHUNK: bytes per write() call
  const uint64_t wchunk = getenv("PBGPU_WRITE_CHUNK") ? strtoull(getenv("PBGPU_WRITE_CHUNK"), nullptr, 10)
                                                      : (64ull << 20);
  auto reader = [&]() {
    try {
      ReadParser rp(paths, details, range_begin, range_end);
      for (uint64_t id = 0;; ++id) {
        Batch* b = nullptr;
        if (!freeq.pop(b)) break;
        const double t0 = now_s();
        b->clear();
        b->id = id;
        // ramp: the first batches are small so the writer (the slowest stage) starts
        // after a short pipeline fill; then full batches (GPU efficiency)
        // (no shift once the ramp is done: a left shift by the batch id wraps past 2^64)
        const uint64_t sh = id >= ramp ? 0 : ramp - id;
        const uint64_t want = sh == 0 ? batch_bases : std::max<uint64_t>(1, sh >= 64 ? 0 : batch_bases >> sh);
        const bool any = rp.fill(*b, want);
        b->grow_scale = sh && b->seq.n >= want ? (double)batch_bases / (double)want : 1.0;
        {
          std::lock_guard<std::mutex> lk(smu);
          S.read_seconds += now_s() - t0;
        }
        if (!any) {
          std::lock_guard<std::mutex> lk(dmu);
          n_batches_total = id;
          dcv.notify_all();
          break;
        }
        if (timeline())
          fprintf(stderr, "pbgpu tl read %llu bases %llu %.4f %.4f\n", (unsigned long long)id,
                  (unsigned long long)b->seq.n, t0 - g_tl0, now_s() - g_tl0);
        if (!inq.push(b)) break;
      }
    } catch (...) {
      record_exception(rs);
    }
    inq.close();
  };

  auto worker = [&](size_t pwi) {
    const size_t wi = part.al[pwi];
    pbgpu_aligner* al = R->al[wi];
    pbgpu_reads* rd = R->rd[wi].get();
    try {
      HIPCHK(hipSetDevice(al->device));
      Batch* b = nullptr;
      bool first = true;
      while (inq.pop(b)) {
        pbgpu_read_batch rb{b->n(), b->seq.p, b->off.data(), b->names.data(), b->name_off.data()};
        // buffers that grow in this batch are sized for a full batch (pbgpu_host.h)
        tl_grow_scale = std::min(64.0, std::max(1.0, b->grow_scale));
        const uint64_t a0 = tl_dev_allocs, p0 = tl_pinned_allocs, by0 = tl_dev_bytes;
        const double as0 = tl_alloc_s, ps0 = tl_pinned_s;
        const double t0 = now_s();
        upload_reads_into(al, &rb, rd);
        const double t1 = now_s();
        aligner_pipeline(al, rd);
        const double t2 = now_s();
        Done d;
        double t3, t4, t5;
        if (run->records_fn) {  // records to the host consumer (create_mega_reads)
          RecordsView& V = *R->views[wi];
          V.download(al);
          const pbgpu_coords_batch* cb = &V.c;
          t3 = t4 = now_s();
          std::vector<std::string> nm(b->n());
          std::vector<const char*> np(b->n());
          std::vector<uint64_t> lens(b->n());
          for (uint64_t i = 0; i < b->n(); ++i) {
            nm[i].assign(b->names.data() + b->name_off[i], b->name_off[i + 1] - b->name_off[i]);
            np[i] = nm[i].c_str();
            lens[i] = b->off[i + 1] - b->off[i];
          }
          uint64_t tl = 0, sl = 0;
          char* side = nullptr;
          int fst = 0;
          d.mtext = run->records_fn(run->records_user, al->ix, cb, np.data(), lens.data(), &tl, &side, &sl, &fst);
          if (side) { d.details.assign(side, sl); free(side); }
          if (fst) { free(d.mtext); throw std::runtime_error("the records consumer failed"); }
          d.len = d.mtext ? tl : 0;
          t5 = now_s();
        } else {
          const uint64_t len = format_device_text(al, rd, run->compact, run->zero_match);
          HIPCHK(hipStreamSynchronize(al->st));
          t3 = now_s();
          if (!part.texts->get(b->id, len + 1, d.text)) break;
          t4 = now_s();
          if (len) HIPCHK(hipMemcpyAsync(d.text.p, al->text.p, len, hipMemcpyDeviceToHost, al->st));
          HIPCHK(hipStreamSynchronize(al->st));
          t5 = now_s();
          d.len = len;
        }
        if (details) {
          pbgpu_details_batch* db = nullptr;
          if (pbgpu_download_details(al, &db) != PBGPU_OK) throw std::runtime_error(pbgpu_last_error());
          std::vector<const char*> hp(b->n());
          for (size_t i = 0; i < hp.size(); ++i) hp[i] = b->headers[i].c_str();
          char* txt = nullptr;
          uint64_t tl = 0;
          const pbgpu_status s = pbgpu_format_details(al->ix, db, hp.data(), hthreads, &txt, &tl);
          pbgpu_details_free(db);
          if (s != PBGPU_OK) throw std::runtime_error(pbgpu_last_error());
          d.details.assign(txt, tl);
          pbgpu_free_text(txt);
        }
        const uint64_t id = b->id, nreads = b->n(), nbases = b->seq.n;
        if (timeline())
          fprintf(stderr, "pbgpu tl work %llu aligner %zu allocs %llu (%.4f s) pinned %llu (%.4f s) %.4f %.4f %.4f %.4f %.4f\n",
                  (unsigned long long)id, wi, (unsigned long long)(tl_dev_allocs - a0), tl_alloc_s - as0,
                  (unsigned long long)(tl_pinned_allocs - p0), tl_pinned_s - ps0, t0 - g_tl0, t1 - g_tl0, t2 - g_tl0,
                  t3 - g_tl0, t5 - g_tl0);
        freeq.push(b);  // the batch's host buffers are free again
        {
          std::lock_guard<std::mutex> lk(smu);
          S.upload_seconds += t1 - t0;
          S.align_seconds += t2 - t1;
          S.format_seconds += t3 - t2;
          S.d2h_seconds += t5 - t4;
          S.n_batches++;
          S.n_reads += nreads;
          S.n_bases += nbases;
          S.n_records += al->last_records;
          if (al->graph && al->g_mega) S.graph_host_reads += al->g_hosts;
          S.n_device_allocs += tl_dev_allocs - a0;
          S.n_pinned_allocs += tl_pinned_allocs - p0;
          S.device_alloc_bytes += tl_dev_bytes - by0;
          S.alloc_seconds += tl_alloc_s - as0;
          if (!first) {
            S.n_device_allocs_late += tl_dev_allocs - a0;
            S.n_pinned_allocs_late += tl_pinned_allocs - p0;
          }
        }
        first = false;
        R->note_device_use(al->device);
        {
          std::lock_guard<std::mutex> lk(dmu);
          done.emplace(id, std::move(d));
          dcv.notify_all();
        }
      }
    } catch (...) {
      record_exception(rs);
    }
  };

  // the writer thread runs on the first GPU's NUMA node (PBGPU_WRITER_NUMA=0: anywhere).
  // C2 coords out, interleaved A/B runs on two boxes: 1.32 Gbases/s mean over five
  // runs pinned, 1.25 unpinned (run-to-run spread ±10%).
  const char* wn = getenv("PBGPU_WRITER_NUMA");
  const std::vector<int> writer_cpus = (!wn || atoi(wn)) ? gpu_node_cpus(R->al[part.al[0]]->device) : std::vector<int>();
  auto writer = [&]() {
    pin_to(writer_cpus);
    try {
      if (write_header && !run->records_fn) {
        std::string h = std::string("Rstart Rend Qstart Qend Nmers Rcons Qcons Rcover Qcover Rlen Qlen Stretch Offset Err") +
                        (run->compact ? "" : " Rname") + " Qname\n";
        write_all(cfd, h.data(), h.size(), "coords");
        S.coords_bytes += h.size();
      }
      for (uint64_t next = 0;; ++next) {
        Done d;
        {
          const double t0 = now_s();
          std::unique_lock<std::mutex> lk(dmu);
          wait_until(dcv, lk, [&] { return done.count(next) || next >= n_batches_total || rs.stopped(); });
          if (rs.stopped() || !done.count(next)) break;
          d = std::move(done[next]);
          done.erase(next);
          lk.unlock();
          std::lock_guard<std::mutex> sl(smu);
          S.writer_idle_seconds += now_s() - t0;
        }
        const double t1 = now_s();
        const char* src = d.mtext ? d.mtext : d.text.p;
        for (uint64_t o = 0; o < d.len; o += wchunk)
          write_all(cfd, src + o, std::min<uint64_t>(wchunk, d.len - o), "coords");
        if (dfd >= 0) write_all(dfd, d.details.data(), d.details.size(), "details");
        {
          std::lock_guard<std::mutex> sl(smu);
          S.write_seconds += now_s() - t1;
          S.coords_bytes += d.len;
          S.details_bytes += d.details.size();
        }
        if (timeline()) fprintf(stderr, "pbgpu tl write %llu %.4f %.4f\n", (unsigned long long)next, t1 - g_tl0, now_s() - g_tl0);
        if (d.mtext) {
          free(d.mtext);
          part.texts->advance();
        } else {
          part.texts->put(d.text, true);
        }
      }
    } catch (...) {
      record_exception(rs);
    }
  };

  std::thread rt(reader), wt(writer);
  std::vector<std::thread> ws;
  for (size_t i = 0; i < W; ++i) ws.emplace_back(worker, i);
  for (auto& t : ws) t.join();
  {  // workers are gone: nothing more can arrive (stops the writer if the run failed mid-way)
    std::unique_lock<std::mutex> lk(dmu);
    const bool early = n_batches_total == ~0ull;
    lk.unlock();
    if (early && !rs.stopped()) rs.fail(PBGPU_ERR_INTERNAL, "the workers ended before the input did");
    dcv.notify_all();
  }
  rt.join();
  wt.join();
  {
    std::lock_guard<std::mutex> lk(dmu);
    for (auto& kv : done) {
      if (kv.second.mtext) free(kv.second.mtext);
      else part.texts->put(kv.second.text, false);
    }
    done.clear();
  }
}

static void runner_run(pbgpu_runner* R, const pbgpu_run_params* run, pbgpu_run_stats* stats) {
  std::lock_guard<std::mutex> run_lock(R->run_mu);
  const double t_start = now_s();
  g_tl0 = t_start;
  const size_t P = R->parts.size();
  // outputs first (early error reporting, jf_aligner.cc:170-178); part p writes
  // <path>.p when there are several parts
  std::vector<int> cfd(P, 1), dfd(P, -1);
  struct fds_guard {
    std::vector<int>& a; std::vector<int>& b;
    ~fds_guard() { for (int f : a) if (f > 2) close(f); for (int f : b) if (f > 2) close(f); }
  } fg{cfd, dfd};
  auto part_path = [&](const char* p, size_t i) { return P > 1 ? std::string(p) + "." + std::to_string(i) : std::string(p); };
  if (P > 1 && !run->coords_path) throw bad_input("part files need a coords path");
  for (size_t i = 0; i < P; ++i) {
    if (run->coords_path) {
      const std::string cp = part_path(run->coords_path, i);
      cfd[i] = open(cp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
      if (cfd[i] < 0) throw bad_input("Failed to open coords file '" + cp + "': " + strerror(errno));
    }
    if (R->side) {
      const std::string dp = part_path(run->details_path, i);
      dfd[i] = open(dp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
      if (dfd[i] < 0) throw bad_input("Failed to open details file '" + dp + "': " + strerror(errno));
    }
  }
  const double t_open = now_s() - t_start;
  std::vector<std::string> paths;
  for (size_t i = 0; i < run->n_pb_paths; ++i) paths.emplace_back(run->pb_paths[i]);
  // part p: the reads whose header starts in [T p / P, T (p + 1) / P) of the inputs
  // (byte ranges need sizes: a FIFO, a process substitution or a device reports 0
  // and would give every part an empty range, so only regular files are split)
  uint64_t T = 0;
  if (P > 1)
    for (const auto& p : paths) {
      struct stat st {};
      if (stat(p.c_str(), &st) != 0) throw bad_input("Can't open PacBio file '" + p + "'");
      if (!S_ISREG(st.st_mode))
        throw unsupported("part files need regular PacBio files to split by byte range; '" + p +
                          "' is a pipe or device");
      T += (uint64_t)st.st_size;
    }
  std::atomic<bool> any_stop(false);
  std::vector<std::unique_ptr<RunState>> rss;
  std::vector<pbgpu_run_stats> SP(P);
  for (size_t i = 0; i < P; ++i) {
    rss.emplace_back(new RunState);
    rss.back()->any_stop = &any_stop;
    SP[i] = pbgpu_run_stats{};
  }
  auto part_fn = [&](size_t i) {
    const uint64_t b = P > 1 ? T * i / P : 0, e = P > 1 ? T * (i + 1) / P : ~0ull;
    try {
      run_part(R, R->parts[i], run, paths, b, e, cfd[i], dfd[i], run->header && i == 0, *rss[i], SP[i]);
    } catch (...) {
      record_exception(*rss[i]);
    }
  };
  if (P == 1) {
    part_fn(0);
  } else {
    std::vector<std::thread> pt;
    for (size_t i = 0; i < P; ++i) pt.emplace_back(part_fn, i);
    for (auto& t : pt) t.join();
  }
  for (auto& r : rss) {
    if (r->status == PBGPU_OK) continue;
    switch (r->status) {
      case PBGPU_ERR_IO: throw bad_input(r->msg);
      case PBGPU_ERR_UNSUPPORTED: throw unsupported(r->msg);
      case PBGPU_ERR_NOMEM: throw std::bad_alloc();
      default: throw std::runtime_error(r->msg);
    }
  }
  pbgpu_run_stats S{};
  for (const auto& x : SP) {  // counts and busy seconds summed over the parts
    S.n_batches += x.n_batches; S.n_reads += x.n_reads; S.n_bases += x.n_bases; S.n_records += x.n_records;
    S.coords_bytes += x.coords_bytes; S.details_bytes += x.details_bytes;
    S.read_seconds += x.read_seconds; S.upload_seconds += x.upload_seconds; S.align_seconds += x.align_seconds;
    S.format_seconds += x.format_seconds; S.d2h_seconds += x.d2h_seconds; S.write_seconds += x.write_seconds;
    S.writer_idle_seconds += x.writer_idle_seconds;
    S.n_device_allocs += x.n_device_allocs; S.n_device_allocs_late += x.n_device_allocs_late;
    S.n_pinned_allocs += x.n_pinned_allocs; S.n_pinned_allocs_late += x.n_pinned_allocs_late;
    S.device_alloc_bytes += x.device_alloc_bytes; S.alloc_seconds += x.alloc_seconds;
    S.graph_host_reads += x.graph_host_reads;
  }
  for (int d = 0; d < pbgpu_runner::kMaxDev; ++d)
    if (R->dev_base[d]) S.device_peak_bytes += R->dev_peak[d].load() - R->dev_base[d];
  S.open_seconds = t_open;
  const double tc = now_s();
  for (size_t i = 0; i < P; ++i) {
    if (cfd[i] > 2) {
      const int fd = cfd[i];
      cfd[i] = -1;
      if (close(fd)) throw bad_input(std::string("closing the coords file failed: ") + strerror(errno));
    }
  }
  S.close_seconds = now_s() - tc;
  S.wall_seconds = now_s() - t_start;
  if (stats) *stats = S;
}

extern "C" {

pbgpu_status pbgpu_host_alloc(uint64_t bytes, void** out) {
  if (!out) return fail(PBGPU_ERR_INVALID, "null argument");
  API_TRY
  *out = nullptr;
  HIPCHK(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_host_free(void* p) {
  if (p) (void)hipHostFree(p);
  return PBGPU_OK;
}

static uint64_t run_hit_budget() {
  const char* e = getenv("PBGPU_RUN_HIT_BUDGET");
  const uint64_t v = e ? strtoull(e, nullptr, 10) : 0;
  return v ? v : 192ull << 20;
}

pbgpu_status pbgpu_runner_create(pbgpu_index* const* indexes, size_t n_indexes, const pbgpu_align_params* params,
                                 const pbgpu_run_params* run, pbgpu_runner** out) {
  if (!indexes || !n_indexes || !params || !run || !out) return fail(PBGPU_ERR_INVALID, "null argument");
  for (size_t i = 0; i < n_indexes; ++i) {
    if (!indexes[i]) return fail(PBGPU_ERR_INVALID, "null index");
    if (indexes[i]->n_shards > 1) return fail(PBGPU_ERR_UNSUPPORTED, "the driver needs whole (unsharded) indexes");
  }
  API_TRY
  // the loops below switch devices: the caller's current device is restored on the way out
  int caller_dev = 0;
  HIPCHK(hipGetDevice(&caller_dev));
  struct RestoreDevice {
    int d;
    ~RestoreDevice() { (void)hipSetDevice(d); }
  } restore_device{caller_dev};
  std::unique_ptr<pbgpu_runner> R(new pbgpu_runner);
  for (size_t i = 0; i < n_indexes; ++i) {  // the devices' use before the aligners (the indexes, other work)
    const int d = indexes[i]->device;
    if (d < 0 || d >= pbgpu_runner::kMaxDev || R->dev_base[d]) continue;
    size_t fr = 0, tot = 0;
    HIPCHK(hipSetDevice(d));
    HIPCHK(hipMemGetInfo(&fr, &tot));
    R->dev_base[d] = (uint64_t)(tot - fr);
    R->dev_peak[d] = R->dev_base[d];
  }
  const uint32_t per_dev = run->aligners_per_device ? run->aligners_per_device : 2;
  R->batch_bases = run->batch_bases ? run->batch_bases : (64ull << 20);
  R->details = run->details_path != nullptr && run->records_fn == nullptr;  // --details coords output
  R->side = run->details_path != nullptr;
  for (size_t i = 0; i < n_indexes; ++i)
    for (uint32_t j = 0; j < per_dev; ++j) {
      pbgpu_aligner* a = nullptr;
      const pbgpu_status s = pbgpu_aligner_create(indexes[i], params, &a);
      if (s != PBGPU_OK) return s;
      // the run path's hit budget: a batch's sub-batches hold at most this many hits, so
      // the per-hit buffers (24 B a hit) stay at ~6 GB an aligner whatever the batch
      // (a 64-Mbase batch: ~370 M hits on C2, ~750 M on C4r-shaped reads; round 4 sized
      // them for the whole batch with 2x headroom, 63 GB for a cold C2 run).
      // PBGPU_RUN_HIT_BUDGET overrides it.
      a->hit_budget = run_hit_budget();
      // a batch ends with the read that reaches batch_bases (reads are < 1/8 of a batch here
      // in practice; a larger one still fits, as an allocation of its own)
      a->base_cap = R->batch_bases + (R->batch_bases >> 3);
      R->al.push_back(a);
      R->rd.emplace_back(new pbgpu_reads);
      R->views.emplace_back(new RecordsView);
      if (run->records_fn && run->graph && run->graph->mega_reads) {
        RecordsView& V = *R->views.back();
        V.reserve_mega(R->batch_bases);
        // the first device -> pinned copy on a stream blocked for 7-8 ms inside
        // hipMemcpyAsync (the copy path's first use) in each worker's first batch:
        // taken here, once, with a small and a large copy each way
        HIPCHK(hipSetDevice(a->device));
        dbuf<char> w;
        w.alloc(1 << 20);
        HIPCHK(hipMemcpyAsync(V.mega.p, w.p, 8, hipMemcpyDeviceToHost, a->st));
        HIPCHK(hipMemcpyAsync(V.mega.p, w.p, 1 << 20, hipMemcpyDeviceToHost, a->st));
        HIPCHK(hipMemcpyAsync(w.p, V.mega.p, 8, hipMemcpyHostToDevice, a->st));
        HIPCHK(hipMemcpyAsync(w.p, V.mega.p, 1 << 20, hipMemcpyHostToDevice, a->st));
        HIPCHK(hipStreamSynchronize(a->st));
      }
      if (R->details) pbgpu_aligner_set_details(a, 1);
      if (run->records_fn && run->graph) {
        const pbgpu_status g = pbgpu_aligner_set_graph(a, run->graph);
        if (g != PBGPU_OK) return g;
      }
    }
  const size_t W = R->al.size();
  const size_t P = run->n_parts > 1 ? run->n_parts : 1;
  if (P > W) return fail(PBGPU_ERR_INVALID, "%zu part files need at least as many aligners (%zu)", P, W);
  if (P > 1 && run->records_fn) return fail(PBGPU_ERR_UNSUPPORTED, "part files with a records consumer");
  R->parts.resize(P);
  for (size_t p = 0; p < P; ++p) {
    RunPart& part = R->parts[p];
    for (size_t i = W * p / P; i < W * (p + 1) / P; ++i) part.al.push_back(i);
    for (size_t i = 0; i < part.al.size() + 2; ++i) {
      part.batches.emplace_back(new Batch);
      part.batches.back()->seq.reserve(R->batch_bases + (R->batch_bases >> 2));
    }
    part.texts.reset(new TextPool(part.al.size() + 2));
  }
  *out = R.release();
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_runner_run(pbgpu_runner* R, const pbgpu_run_params* run, pbgpu_run_stats* stats) {
  if (!R || !run || (!run->pb_paths && run->n_pb_paths)) return fail(PBGPU_ERR_INVALID, "null argument");
  if ((run->details_path != nullptr) != R->side)
    return fail(PBGPU_ERR_INVALID, "--details must be given to pbgpu_runner_create and every run alike");
  API_TRY
  runner_run(R, run, stats);
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_runner_free(pbgpu_runner* R) {
  delete R;
  return PBGPU_OK;
}

pbgpu_status pbgpu_run(pbgpu_index* const* indexes, size_t n_indexes, const pbgpu_align_params* params,
                       const pbgpu_run_params* run, pbgpu_run_stats* stats) {
  pbgpu_runner* R = nullptr;
  pbgpu_status s = pbgpu_runner_create(indexes, n_indexes, params, run, &R);
  if (s != PBGPU_OK) return s;
  s = pbgpu_runner_run(R, run, stats);
  pbgpu_runner_free(R);
  return s;
}

}  // extern "C"
