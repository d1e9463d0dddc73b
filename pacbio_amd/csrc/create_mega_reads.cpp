// create_mega_reads -- drop-in CLI for the reference's create_mega_reads
// (src_jf_aligner/create_mega_reads.cc:95-167, options
// create_mega_reads_cmdline.yaggo:1-84), the production caller of the aligner
// (mega_reads_assemble_cluster2.sh:485).
//
// The coarse (and, with -F, fine) alignment runs on MI355X GPUs through
// pbgpu_run, exactly as jf_aligner's: forward = true and unitig lengths
// required (create_mega_reads.cc:140-148).  By default the per-read overlap
// graph, longest path, components, tiling and printed unitig paths run on the
// GPU after each batch's records are sorted (k_graph*, k_mega; ABI 5,
// pbgpu_aligner_set_graph); the host only writes the text, on -t threads.  The
// host restatement (overlap_graph.cpp) runs --dot, --host-graph and the reads
// the device leaves to it (more than GRAPH_NMAX_BIG = 65,535 records; round 5).  The mega-reads of each
// batch are written in input order (the reference's output with -t 1).
// GPU options as in jf_aligner: --devices, --streams, --batch-bases, --timing
// (stage times as JSON on stderr).
#include <getopt.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <mutex>
#include <stdexcept>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pbgpu.h"
#include "index_cache.h"
#include "overlap_graph.hpp"

using namespace megareads;

static void die(const std::string& m) {
  fprintf(stderr, "create_mega_reads: %s\n", m.c_str());
  exit(1);
}
static void check(pbgpu_status s, const char* what) {
  if (s != PBGPU_OK) die(std::string(what) + ": " + pbgpu_last_error());
}
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

// misc.cc:11-19
static std::vector<int> read_unitigs_lengths(const char* path) {
  std::ifstream is(path);
  if (!is.good()) die(std::string("Failed to open unitig lengths map file '") + path + "'");
  std::vector<int> v;
  std::string name;
  unsigned int len;
  is >> name >> len;
  while (is.good()) { v.push_back((int)len); is >> name >> len; }
  return v;
}
// misc.cc:30-37: header line, then one sequence line, per unitig (a trailing
// newline yields one more, empty, unitig -- as upstream)
static void read_unitigs_sequences(const char* path, std::vector<int>& lens, std::vector<std::string>& seqs) {
  std::ifstream is(path);
  if (!is.good()) die(std::string("Failed to open unitigs sequence file '") + path + "'");
  while (is.ignore(std::numeric_limits<std::streamsize>::max(), '\n')) {
    seqs.push_back("");
    std::getline(is, seqs.back());
    lens.push_back((int)seqs.back().size());
  }
}

struct Ctx {
  Params gp;
  int threads = 1;
  bool dot = false;
  // unitig lists of every super-read name, fwd and reversed (frag_info.hpp:18-35)
  std::vector<unitig_list> fwd, bwd;
};

// pbgpu_run records consumer: the create_mega_reads worker (create_mega_reads.cc:55-90)
// for every read of the batch, in parallel over reads, output in read order.
static char* mega_reads_batch(void* user, const pbgpu_index* ix, const pbgpu_coords_batch* cb,
                              const char* const* names, const uint64_t* lens, uint64_t* text_len, char** side,
                              uint64_t* side_len, int* status) {
  (void)ix;
  Ctx& C = *(Ctx*)user;
  try {
    const uint64_t n = cb->n_reads;
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)C.threads, n));
    const uint64_t parts = std::min<uint64_t>(n, (uint64_t)T * 8);
    std::vector<std::string> out(parts), dout(parts);
    std::atomic<uint64_t> next(0);
    std::mutex err_mu;
    std::string err;  // the first error of any thread (no exception may leave a std::thread)
    auto work = [&]() {
      try {
      ReadGraph g(C.gp);
      std::vector<Coord> coords;
      for (;;) {
        const uint64_t pi = next.fetch_add(1);
        if (pi >= parts) break;
        std::ostringstream os, ds;
        for (uint64_t r = n * pi / parts; r < n * (pi + 1) / parts; ++r) {
          if (cb->mega && !cb->mega_host[r]) {  // finished on the device: print only
            g.print_device(os, names[r], cb->mega + cb->mega_offsets[r], cb->mega_offsets[r + 1] - cb->mega_offsets[r],
                           cb->mega_units);
            continue;
          }
          coords.clear();
          for (uint64_t i = cb->read_offsets[r]; i < cb->read_offsets[r + 1]; ++i) {
            const pbgpu_record& R = cb->records[i];
            Coord c;
            c.rs = R.rs; c.re = R.re; c.qs = R.qs; c.qe = R.qe; c.nb_mers = R.nb_mers;
            c.sr_cover = R.sr_cover;
            c.rl = lens[r]; c.ql = R.ql;
            c.stretch = R.stretch; c.offset = R.offset; c.avg_err = R.avg_err;
            c.name = (R.flags & 2u) ? &C.bwd[R.sr_index] : &C.fwd[R.sr_index];
            c.kmers_info = cb->kmers_info + R.info_offset;
            c.bases_info = cb->bases_info + R.info_offset;
            c.n_info = R.n_info;
            coords.push_back(c);
          }
          g.process(coords, names[r], os, C.dot ? &ds : nullptr,
                    cb->graph ? cb->graph + cb->read_offsets[r] : nullptr);
        }
        out[pi] = os.str();
        if (C.dot) dout[pi] = ds.str();
      }
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(err_mu);
        if (err.empty()) err = e.what();
        next.store(parts);  // the other threads stop at their next part
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    if (!err.empty()) throw std::runtime_error(err);
    auto join = [](const std::vector<std::string>& v, uint64_t* len) -> char* {
      uint64_t tot = 0;
      for (auto& s : v) tot += s.size();
      char* p = (char*)malloc(tot + 1);
      if (!p) throw std::bad_alloc();
      uint64_t o = 0;
      for (auto& s : v) { memcpy(p + o, s.data(), s.size()); o += s.size(); }
      p[o] = 0;
      *len = o;
      return p;
    };
    if (C.dot) *side = join(dout, side_len);
    *status = 0;
    return join(out, text_len);
  } catch (const std::exception& e) {
    fprintf(stderr, "create_mega_reads: %s\n", e.what());
    *status = 1;
    return nullptr;
  }
}

int main(int argc, char** argv) {
  pbgpu_align_params ap;
  pbgpu_align_params_default(&ap);
  ap.forward = 1;  // create_mega_reads.cc:142
  Ctx C;
  uint32_t psa_min = 13, threads = 1, streams = 2;
  bool timing = false;
  const char* index_cache = nullptr;  // --index-cache PATH (index_cache.h)
  bool s_given = false, m_given = false, k_given = false;
  const char *out_path = nullptr, *dot_path = nullptr, *ul_path = nullptr, *us_path = nullptr;
  std::vector<const char*> srs, pbs;
  std::vector<int> devices;
  uint64_t batch_bases = 64ull << 20;
  bool host_graph = false;  // --host-graph: traverse the overlap graph on the host (else on the GPU)
  enum { O_PSA = 256, O_DOT, O_SC, O_SF, O_CAP, O_WIN, O_MAXM, O_MAXC, O_TRIM, O_DEVS, O_BATCH, O_STREAMS, O_TIMING, O_CACHE,
         O_HOSTG };
  static struct option lo[] = {
      {"size", 1, 0, 's'}, {"mer", 1, 0, 'm'}, {"fine-mer", 1, 0, 'F'}, {"psa-min", 1, 0, O_PSA},
      {"unitigs-lengths", 1, 0, 'l'}, {"unitigs-sequences", 1, 0, 'u'}, {"k-mer", 1, 0, 'k'},
      {"threads", 1, 0, 't'}, {"output", 1, 0, 'o'}, {"dot", 1, 0, O_DOT}, {"stretch-constant", 1, 0, O_SC},
      {"stretch-factor", 1, 0, O_SF}, {"stretch-cap", 1, 0, O_CAP}, {"window-size", 1, 0, O_WIN},
      {"overlap-play", 1, 0, 'O'}, {"errors", 1, 0, 'e'}, {"bases-matching", 1, 0, 'B'},
      {"mers-matching", 1, 0, 'M'}, {"max-match", 0, 0, O_MAXM}, {"max-count", 1, 0, O_MAXC}, {"bases", 0, 0, 'b'},
      {"density", 1, 0, 'd'}, {"min-length", 1, 0, 'L'}, {"tiling", 1, 0, 'T'}, {"trim", 1, 0, O_TRIM},
      {"superreads", 1, 0, 'r'}, {"pacbio", 1, 0, 'p'}, {"devices", 1, 0, O_DEVS}, {"batch-bases", 1, 0, O_BATCH},
      {"streams", 1, 0, O_STREAMS}, {"timing", 0, 0, O_TIMING}, {"index-cache", 1, 0, O_CACHE},
      {"host-graph", 0, 0, O_HOSTG}, {0, 0, 0, 0}};
  int c;
  while ((c = getopt_long(argc, argv, "s:m:F:l:u:k:t:o:O:e:B:M:bd:L:T:r:p:", lo, nullptr)) != -1) {
    switch (c) {
    case 's': parse_suffix(optarg); s_given = true; break;  // required, unused (legacy)
    case 'm': ap.k = parse_u32(optarg, "-m"); m_given = true; break;
    case 'F': ap.fine_k = parse_u32(optarg, "-F"); break;
    case O_PSA: psa_min = parse_u32(optarg, "--psa-min"); break;
    case 'l': ul_path = optarg; break;
    case 'u': us_path = optarg; break;
    case 'k': ap.unitigs_k = parse_u32(optarg, "-k"); k_given = true; break;
    case 't': threads = std::max(1u, parse_u32(optarg, "-t")); break;
    case 'o': out_path = optarg; break;
    case O_DOT: dot_path = optarg; break;
    case O_SC: ap.stretch_constant = (double)(int)strtol(optarg, nullptr, 10); break;
    case O_SF: ap.stretch_factor = parse_f64(optarg, "--stretch-factor"); break;
    case O_CAP: ap.stretch_cap = parse_f64(optarg, "--stretch-cap"); break;
    case O_WIN: ap.window_size = parse_u32(optarg, "--window-size"); break;
    case 'O': C.gp.overlap_play = parse_f64(optarg, "-O"); break;
    case 'e': C.gp.nb_errors = parse_f64(optarg, "-e"); break;
    case 'B': ap.bases_matching = parse_f64(optarg, "-B"); break;
    case 'M': ap.mers_matching = parse_f64(optarg, "-M"); break;
    case O_MAXM: ap.max_match = 1; break;
    case O_MAXC: ap.max_count = (int32_t)parse_u32(optarg, "--max-count"); break;
    case 'b': C.gp.maximize_bases = true; break;
    case 'd': C.gp.min_density = parse_f64(optarg, "-d"); break;
    case 'L': C.gp.min_len = parse_f64(optarg, "-L"); break;
    case 'T': {
      const std::string t = optarg;
      if (t == "none") C.gp.tiling = Tiling::NONE;
      else if (t == "greedy") C.gp.tiling = Tiling::GREEDY;
      else if (t == "maximal") C.gp.tiling = Tiling::MAXIMAL;
      else if (t == "weighted") C.gp.tiling = Tiling::WEIGHTED;
      else die("invalid --tiling '" + t + "' (none, greedy, maximal, weighted)");
      break;
    }
    case O_TRIM: {
      const std::string t = optarg;
      if (t == "none") C.gp.trim = Trim::NONE;
      else if (t == "match") C.gp.trim = Trim::MATCH;
      // create_mega_reads.cc:47-49 turns the graph thread's trimming on for "match" only:
      // "branch" leaves it at NONE (the graph itself would treat BRANCH as MATCH,
      // overlap_graph.cc:126-127, but the CLI never passes it)
      else if (t == "branch") C.gp.trim = Trim::NONE;
      else die("invalid --trim '" + t + "' (none, match, branch)");
      break;
    }
    case 'r': srs.push_back(optarg); break;
    case 'p': pbs.push_back(optarg); break;
    case O_DEVS: {
      std::string l = optarg;
      for (size_t a = 0; a <= l.size();) {
        size_t e = l.find(',', a);
        if (e == std::string::npos) e = l.size();
        devices.push_back((int)parse_u32(l.substr(a, e - a).c_str(), "--devices"));
        a = e + 1;
      }
      break;
    }
    case O_BATCH: batch_bases = parse_suffix(optarg); break;
    case O_STREAMS: streams = std::max(1u, parse_u32(optarg, "--streams")); break;
    case O_TIMING: timing = true; break;
    case O_CACHE: index_cache = optarg; break;
    case O_HOSTG: host_graph = true; break;
    default: die("bad option (see create_mega_reads_cmdline.yaggo)");
    }
  }
  if (!s_given) die("-s, --size is required");
  if (!m_given) die("-m, --mer is required");
  if (!k_given) die("-k, --k-mer is required");
  if (ul_path && us_path) die("-u conflicts with -l");
  if (!ul_path && !us_path) die("the unitig lengths (-l) or sequences (-u) are required");
  if (ap.max_count == 0) die("--max-count 0 is undefined behaviour in the reference (coarse_aligner.cc:86)");
  std::vector<int> ul;
  std::vector<std::string> useqs;
  if (ul_path) ul = read_unitigs_lengths(ul_path);
  else read_unitigs_sequences(us_path, ul, useqs);
  std::vector<int32_t> ul32(ul.begin(), ul.end());
  ap.unitig_lengths = ul32.data();
  ap.n_unitigs = ul32.size();
  C.gp.k_len = ap.unitigs_k;
  C.gp.unitig_lengths = &ul;
  C.gp.unitig_sequences = us_path ? &useqs : nullptr;
  C.threads = (int)threads;
  C.dot = dot_path != nullptr;
  if (devices.empty()) devices.push_back(0);

  // index: built once, replicated per distinct device (create_mega_reads.cc:131-132)
  pbgpu_index_params ip{ap.k, psa_min, devices[0], (int)threads, ap.fine_k, 0, 1};
  std::vector<std::pair<int, pbgpu_index*>> built;
  auto index_on = [&](int dev) -> pbgpu_index* {
    for (auto& b : built) if (b.first == dev) return b.second;
    pbgpu_index* ix = nullptr;
    if (built.empty()) check(index_from_cache(index_cache, srs, ip, &ix, timing), "index");
    else check(pbgpu_index_replicate(built[0].second, dev, &ix), "index replica");
    built.emplace_back(dev, ix);
    return ix;
  };
  std::vector<pbgpu_index*> per_entry;
  for (int d : devices) per_entry.push_back(index_on(d));
  {  // unitig lists of every super-read name (fwd; bwd = reversed), in parallel
    pbgpu_index_info info;
    check(pbgpu_index_get_info(per_entry[0], &info), "index info");
    const uint64_t nsr = info.n_sr;
    C.fwd.resize(nsr);
    C.bwd.resize(nsr);
    std::vector<std::thread> th;
    const unsigned T = std::max(1u, threads);
    for (unsigned t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        for (uint64_t i = nsr * t / T; i < nsr * (t + 1) / T; ++i) {
          const char* nm = pbgpu_index_sr_name(per_entry[0], (uint32_t)i, 0);
          C.fwd[i] = parse_name(nm ? nm : "");
          C.bwd[i] = C.fwd[i].empty() ? C.fwd[i] : reverse_name(C.fwd[i]);
        }
      });
    for (auto& t : th) t.join();
  }
  pbgpu_run_params rp{};
  rp.pb_paths = pbs.data();
  rp.n_pb_paths = pbs.size();
  rp.coords_path = out_path;
  rp.details_path = dot_path;
  rp.compact = 1;
  rp.header = 0;
  rp.aligners_per_device = streams;
  rp.batch_bases = batch_bases;
  rp.host_threads = (int)threads;
  rp.records_fn = mega_reads_batch;
  rp.records_user = &C;
  // the overlap graph's traversal on the GPU (the host keeps --dot runs, whose edge
  // lines come out in traversal order, and --host-graph)
  std::vector<uint64_t> name_off(C.fwd.size() + 1, 0);
  std::vector<uint32_t> name_units;
  pbgpu_graph_params gp{};
  if (!host_graph && !C.dot) {
    for (size_t i = 0; i < C.fwd.size(); ++i) {
      name_units.insert(name_units.end(), C.fwd[i].begin(), C.fwd[i].end());
      name_off[i + 1] = name_units.size();
    }
    gp.overlap_play = C.gp.overlap_play;
    gp.nb_errors = C.gp.nb_errors;
    gp.k_len = C.gp.k_len;
    gp.maximize_bases = C.gp.maximize_bases;
    gp.n_sr = C.fwd.size();
    gp.name_offsets = name_off.data();
    gp.name_units = name_units.data();
    gp.unitig_lengths = ul32.data();
    gp.n_unitigs = ul32.size();
    // components, tiling and the printed paths on the device too (the host prints)
    gp.mega_reads = 1;
    gp.tiling = C.gp.tiling == Tiling::NONE ? PBGPU_TILING_NONE
              : C.gp.tiling == Tiling::GREEDY ? PBGPU_TILING_GREEDY
              : C.gp.tiling == Tiling::MAXIMAL ? PBGPU_TILING_MAXIMAL : PBGPU_TILING_WEIGHTED;
    gp.trim = C.gp.trim != Trim::NONE;
    gp.min_density = C.gp.min_density;
    gp.min_len = C.gp.min_len;
    rp.graph = &gp;
  }
  pbgpu_run_stats st{};
  const pbgpu_status rs = pbgpu_run(per_entry.data(), per_entry.size(), &ap, &rp, &st);
  const std::string err = rs == PBGPU_OK ? "" : pbgpu_last_error();
  for (auto& b : built) pbgpu_index_free(b.second);
  if (rs != PBGPU_OK) die("align: " + err);
  if (timing)
    fprintf(stderr,
            "{\"wall_s\": %.6f, \"batches\": %llu, \"reads\": %llu, \"bases\": %llu, \"records\": %llu, "
            "\"output_bytes\": %llu, \"read_s\": %.6f, \"upload_s\": %.6f, \"align_s\": %.6f, "
            "\"download_s\": %.6f, \"graph_s\": %.6f, \"write_s\": %.6f, \"writer_idle_s\": %.6f, "
            "\"device_allocs\": %llu, \"device_allocs_late\": %llu, \"pinned_allocs\": %llu, "
            "\"pinned_allocs_late\": %llu, \"device_alloc_bytes\": %llu, \"alloc_s\": %.6f, "
            "\"device_peak_bytes\": %llu, \"graph_host_reads\": %llu}\n",
            st.wall_seconds, (unsigned long long)st.n_batches, (unsigned long long)st.n_reads,
            (unsigned long long)st.n_bases, (unsigned long long)st.n_records, (unsigned long long)st.coords_bytes,
            st.read_seconds, st.upload_seconds, st.align_seconds, st.format_seconds, st.d2h_seconds, st.write_seconds,
            st.writer_idle_seconds, (unsigned long long)st.n_device_allocs,
            (unsigned long long)st.n_device_allocs_late, (unsigned long long)st.n_pinned_allocs,
            (unsigned long long)st.n_pinned_allocs_late, (unsigned long long)st.device_alloc_bytes,
            st.alloc_seconds, (unsigned long long)st.device_peak_bytes, (unsigned long long)st.graph_host_reads);
  return 0;
}
