// jf_aligner -- drop-in CLI for the reference's jf_aligner
// (src_jf_aligner/jf_aligner.cc:161-233, options jf_aligner_cmdline.yaggo:1-77)
// running the coarse aligner on an MI355X through the pbgpu C ABI.
//
// Same flags, same coords (and --details) text.  Reads are processed in
// batches; output is written in input order (what the reference prints with
// -t 1).  -F runs the fine aligner on the device after the coarse one.
#include <getopt.h>

#include <algorithm>
#include <cerrno>
#include <limits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/pbgpu.h"

static void die(const std::string& m) {
  fprintf(stderr, "jf_aligner: %s\n", m.c_str());
  exit(1);
}
static void check(pbgpu_status s, const char* what) {
  if (s != PBGPU_OK) die(std::string(what) + ": " + pbgpu_last_error());
}

// yaggo uint64 with suffix (k, M, G, ...)
static uint64_t parse_suffix(const char* s) {
  char* e;
  errno = 0;
  double v = strtod(s, &e);
  if (e == s || errno) die(std::string("invalid size '") + s + "'");
  switch (*e) {
  case 'k': v *= 1e3; break;
  case 'M': v *= 1e6; break;
  case 'G': v *= 1e9; break;
  case 'T': v *= 1e12; break;
  case 0: break;
  default: die(std::string("invalid suffix in '") + s + "'");
  }
  return (uint64_t)v;
}
static uint32_t parse_u32(const char* s, const char* opt) {
  char* e;
  errno = 0;
  unsigned long v = strtoul(s, &e, 10);
  if (e == s || *e || errno || v > 0xFFFFFFFFul) die(std::string("invalid value for ") + opt + ": '" + s + "'");
  return (uint32_t)v;
}
static double parse_f64(const char* s, const char* opt) {
  char* e;
  errno = 0;
  double v = strtod(s, &e);
  if (e == s || *e || errno) die(std::string("invalid value for ") + opt + ": '" + s + "'");
  return v;
}

// read_unitigs_lengths (misc.cc:11-19): pairs "name len", vector index = line order
static std::vector<int32_t> read_unitigs_lengths(const char* path) {
  std::ifstream is(path);
  if (!is.good()) die(std::string("Failed to open unitig lengths map file '") + path + "'");
  std::vector<int32_t> v;
  std::string name;
  unsigned int len;
  is >> name >> len;
  while (is.good()) { v.push_back((int32_t)len); is >> name >> len; }
  return v;
}
// read_unitigs_sequences (misc.cc:21-28)
static std::vector<int32_t> read_unitigs_sequences(const char* path) {
  std::ifstream is(path);
  if (!is.good()) die(std::string("Failed to open unitig sequence file '") + path + "'");
  std::vector<int32_t> v;
  std::string seq;
  while (is.ignore(std::numeric_limits<std::streamsize>::max(), '\n')) {
    std::getline(is, seq);
    v.push_back((int32_t)seq.size());
  }
  return v;
}

// FASTA/FASTQ streaming reader: header = line after '>'/'@', sequence =
// concatenated lines (whole_sequence_parser semantics).
struct read_stream {
  std::vector<const char*> files;
  size_t fi = 0;
  FILE* f = nullptr;
  char* line = nullptr;
  size_t cap = 0;
  bool have_pending = false;
  std::string pending;
  ~read_stream() { if (f) fclose(f); free(line); }
  bool getl(std::string& out) {
    for (;;) {
      if (!f) {
        if (fi >= files.size()) return false;
        f = fopen(files[fi++], "r");
        if (!f) die(std::string("Can't open PacBio file '") + files[fi - 1] + "'");
      }
      ssize_t l = getline(&line, &cap, f);
      if (l < 0) { fclose(f); f = nullptr; continue; }
      if (l > 0 && line[l - 1] == '\n') --l;
      out.assign(line, (size_t)l);
      return true;
    }
  }
  // next record; false at end
  bool next(std::string& header, std::string& seq) {
    std::string l;
    if (have_pending) { l.swap(pending); have_pending = false; }
    else {
      do { if (!getl(l)) return false; } while (l.empty());
    }
    if (l[0] == '@') {
      header = l.substr(1);
      seq.clear();
      getl(seq);
      std::string plus, qual;
      getl(plus); getl(qual);
      return true;
    }
    if (l[0] != '>') die("PacBio input is neither FASTA nor FASTQ");
    header = l.substr(1);
    seq.clear();
    while (getl(l)) {
      if (!l.empty() && l[0] == '>') { pending.swap(l); have_pending = true; break; }
      seq += l;
    }
    return true;
  }
};

int main(int argc, char** argv) {
  pbgpu_align_params ap;
  pbgpu_align_params_default(&ap);
  uint32_t psa_min = 13, threads = 1;
  bool s_given = false, m_given = false, k_given = false, no_header = false, zero = false, compact = true;
  const char* coords_path = nullptr;
  const char* details_path = nullptr;
  const char* ul_path = nullptr;
  const char* us_path = nullptr;
  std::vector<const char*> srs, pbs;
  int device = 0;
  uint64_t batch_bases = 256ull << 20;
  uint32_t streams = 2;
  enum { O_PSA = 256, O_SC, O_SF, O_CAP, O_WIN, O_DETAILS, O_COORDS, O_MAXM, O_MAXC, O_COMPACT, O_NOCOMPACT, O_DEV, O_BATCH, O_STREAMS };
  static struct option lo[] = {
      {"size", 1, 0, 's'}, {"mer", 1, 0, 'm'}, {"fine-mer", 1, 0, 'F'}, {"psa-min", 1, 0, O_PSA},
      {"threads", 1, 0, 't'}, {"stretch-constant", 1, 0, O_SC}, {"stretch-factor", 1, 0, O_SF},
      {"stretch-cap", 1, 0, O_CAP}, {"window-size", 1, 0, O_WIN}, {"forward", 0, 0, 'f'},
      {"bases-matching", 1, 0, 'B'}, {"mers-matching", 1, 0, 'M'}, {"details", 1, 0, O_DETAILS},
      {"coords", 1, 0, O_COORDS}, {"max-match", 0, 0, O_MAXM}, {"no-header", 0, 0, 'H'},
      {"zero-match", 0, 0, '0'}, {"max-count", 1, 0, O_MAXC}, {"unitigs-lengths", 1, 0, 'l'},
      {"unitigs-sequences", 1, 0, 'u'}, {"compact", 0, 0, O_COMPACT}, {"no-compact", 0, 0, O_NOCOMPACT},
      {"k-mer", 1, 0, 'k'}, {"superreads", 1, 0, 'r'}, {"pacbio", 1, 0, 'p'},
      {"device", 1, 0, O_DEV}, {"batch-bases", 1, 0, O_BATCH},
      {"streams", 1, 0, O_STREAMS}, {0, 0, 0, 0}};
  int c;
  while ((c = getopt_long(argc, argv, "s:m:F:t:fB:M:H0l:u:k:r:p:", lo, nullptr)) != -1) {
    switch (c) {
    case 's': parse_suffix(optarg); s_given = true; break;  // required, unused (legacy)
    case 'm': ap.k = parse_u32(optarg, "-m"); m_given = true; break;
    case 'F': ap.fine_k = parse_u32(optarg, "-F"); break;
    case O_PSA: psa_min = parse_u32(optarg, "--psa-min"); break;
    case 't': threads = parse_u32(optarg, "-t"); break;
    case O_SC: ap.stretch_constant = (double)(int)strtol(optarg, nullptr, 10); break;
    case O_SF: ap.stretch_factor = parse_f64(optarg, "--stretch-factor"); break;
    case O_CAP: ap.stretch_cap = parse_f64(optarg, "--stretch-cap"); break;
    case O_WIN: ap.window_size = parse_u32(optarg, "--window-size"); break;
    case 'f': ap.forward = 1; break;
    case 'B': ap.bases_matching = parse_f64(optarg, "-B"); break;
    case 'M': ap.mers_matching = parse_f64(optarg, "-M"); break;
    case O_DETAILS: details_path = optarg; break;
    case O_COORDS: coords_path = optarg; break;
    case O_MAXM: ap.max_match = 1; break;
    case 'H': no_header = true; break;
    case '0': zero = true; break;
    case O_MAXC: ap.max_count = (int32_t)parse_u32(optarg, "--max-count"); break;
    case 'l': ul_path = optarg; ap.forward = 1; break;
    case 'u': us_path = optarg; ap.forward = 1; break;
    case O_COMPACT: compact = true; break;
    case O_NOCOMPACT: compact = false; break;
    case 'k': ap.unitigs_k = parse_u32(optarg, "-k"); k_given = true; break;
    case 'r': srs.push_back(optarg); break;
    case 'p': pbs.push_back(optarg); break;
    case O_DEV: device = (int)parse_u32(optarg, "--device"); break;
    case O_BATCH: batch_bases = parse_suffix(optarg); break;
    case O_STREAMS: streams = std::max(1u, parse_u32(optarg, "--streams")); break;
    default: die("bad option (see jf_aligner_cmdline.yaggo)");
    }
  }
  if (!s_given) die("-s, --size is required");
  if (!m_given) die("-m, --mer is required");
  if (ul_path && us_path) die("-u conflicts with -l");
  if (!details_path && !coords_path) die("No output file given. Doing nothing ungracefully.");  // jf_aligner.cc:166-167
  if (ap.max_count == 0) die("--max-count 0 is undefined behaviour in the reference (coarse_aligner.cc:86)");
  std::vector<int32_t> ul;
  if (ul_path || us_path) {
    if (!k_given)
      die("The mer length used for generating the k-unitigs (-k, --k-mer) is required if the unitig lengths "
          "(-l, --unitig-lengths or -u, --unitigs-sequences) is passed.");
    ul = ul_path ? read_unitigs_lengths(ul_path) : read_unitigs_sequences(us_path);
    ap.unitig_lengths = ul.data();
    ap.n_unitigs = ul.size();
  } else {
    ap.unitigs_k = 0;
  }
  FILE* out = coords_path ? fopen(coords_path, "w") : stdout;
  if (!out) die(std::string("Failed to open coords file '") + coords_path + "'");
  FILE* dout = details_path ? fopen(details_path, "w") : nullptr;
  if (details_path && !dout) die(std::string("Failed to open details file '") + details_path + "'");

  pbgpu_index_params ip{ap.k, psa_min, device, (int)threads, ap.fine_k};
  pbgpu_index* ix = nullptr;
  check(pbgpu_index_build_fasta(srs.data(), srs.size(), &ip, &ix), "index");
  if (!no_header) {
    fputs("Rstart Rend Qstart Qend Nmers Rcons Qcons Rcover Qcover Rlen Qlen Stretch Offset Err", out);
    if (!compact) fputs(" Rname", out);
    fputs(" Qname\n", out);
  }
  // Batches are pipelined over `streams` aligners (own HIP stream and buffers
  // each, one shared index), one host thread per aligner: while one batch is
  // on the GPU the next is read and the previous formatted.  A worker takes
  // the next batch under the reader lock, aligns and formats it, then waits
  // for its turn so the files come out in input order.
  read_stream rs;
  rs.files = pbs;
  std::mutex rd_mu, wr_mu;
  std::condition_variable wr_cv;
  bool more = true;
  uint64_t next_batch = 0, next_write = 0;
  auto worker = [&]() {
    pbgpu_aligner* al = nullptr;
    check(pbgpu_aligner_create(ix, &ap, &al), "aligner");
    if (dout) check(pbgpu_aligner_set_details(al, 1), "details");
    std::string h, s;
    for (;;) {
      std::vector<std::string> headers;
      std::string seq;
      std::vector<uint64_t> offs{0};
      uint64_t me;
      {
        std::lock_guard<std::mutex> lk(rd_mu);
        while (seq.size() < batch_bases && more && (more = rs.next(h, s))) {
          headers.push_back(h);
          seq += s;
          offs.push_back(seq.size());
        }
        if (headers.empty()) break;
        me = next_batch++;
      }
      pbgpu_read_batch b{headers.size(), seq.data(), offs.data()};
      pbgpu_coords_batch* cb = nullptr;
      check(pbgpu_align_batch(al, &b, &cb), "align");
      std::vector<const char*> hp(headers.size());
      std::vector<uint64_t> lens(headers.size());
      for (size_t i = 0; i < headers.size(); ++i) { hp[i] = headers[i].c_str(); lens[i] = offs[i + 1] - offs[i]; }
      char* text = nullptr;
      uint64_t tl = 0;
      check(pbgpu_format_coords(ix, cb, hp.data(), lens.data(), compact ? 1 : 0, 0, zero ? 1 : 0,
                                (int)std::max(1u, threads), &text, &tl), "format");
      pbgpu_coords_free(cb);
      char* dtext = nullptr;
      uint64_t dtl = 0;
      if (dout) {
        pbgpu_details_batch* db = nullptr;
        check(pbgpu_download_details(al, &db), "details");
        check(pbgpu_format_details(ix, db, hp.data(), (int)std::max(1u, threads), &dtext, &dtl), "format details");
        pbgpu_details_free(db);
      }
      std::unique_lock<std::mutex> lk(wr_mu);
      wr_cv.wait(lk, [&] { return next_write == me; });
      fwrite(text, 1, tl, out);
      if (dout) fwrite(dtext, 1, dtl, dout);
      ++next_write;
      lk.unlock();
      wr_cv.notify_all();
      pbgpu_free_text(text);
      if (dtext) pbgpu_free_text(dtext);
    }
    pbgpu_aligner_free(al);
  };
  std::vector<std::thread> pool;
  for (uint32_t i = 0; i < streams; ++i) pool.emplace_back(worker);
  for (auto& t : pool) t.join();
  if (coords_path) fclose(out);
  if (dout) fclose(dout);
  pbgpu_index_free(ix);
  return 0;
}
