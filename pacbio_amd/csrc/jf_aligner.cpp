// jf_aligner -- drop-in CLI for the reference's jf_aligner
// (src_jf_aligner/jf_aligner.cc:161-233, options jf_aligner_cmdline.yaggo:1-77)
// running the coarse aligner on MI355X GPUs through the pbgpu C ABI.
//
// Same flags, same coords (and --details) text.  The super-read index is
// built once on the first device and replicated to the others; pbgpu_run
// then streams the PacBio files (plain or gzip) in batches over
// --streams aligners per device, formats the coords on the devices and
// writes them in input order (what the reference prints with -t 1).
// -F runs the fine aligner on the device after the coarse one.
// GPU-only options: --devices 0,1,.. (default 0; a device may repeat),
// --streams (aligners per device), --batch-bases, --timing (stage times on
// stderr as one JSON line), --parts P (coords in P part files <coords>.0 ..
// .P-1 written in parallel, whose concatenation is the one-file output; the
// reference's split-and-cat, mega_reads_assemble_cluster2.sh:325-354,447).
#include <getopt.h>

#include <algorithm>
#include <cerrno>
#include <limits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "../../include/pbgpu.h"
#include "index_cache.h"

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
  std::vector<int> devices;
  uint64_t batch_bases = 64ull << 20;
  uint32_t streams = 2, parts = 0;
  bool timing = false;
  const char* index_cache = nullptr;  // --index-cache PATH (index_cache.h)
  enum { O_PSA = 256, O_SC, O_SF, O_CAP, O_WIN, O_DETAILS, O_COORDS, O_MAXM, O_MAXC, O_COMPACT, O_NOCOMPACT, O_DEV, O_BATCH,
         O_STREAMS, O_DEVS, O_TIMING, O_CACHE, O_PARTS };
  static struct option lo[] = {
      {"size", 1, 0, 's'}, {"mer", 1, 0, 'm'}, {"fine-mer", 1, 0, 'F'}, {"psa-min", 1, 0, O_PSA},
      {"threads", 1, 0, 't'}, {"stretch-constant", 1, 0, O_SC}, {"stretch-factor", 1, 0, O_SF},
      {"stretch-cap", 1, 0, O_CAP}, {"window-size", 1, 0, O_WIN}, {"forward", 0, 0, 'f'},
      {"bases-matching", 1, 0, 'B'}, {"mers-matching", 1, 0, 'M'}, {"details", 1, 0, O_DETAILS},
      {"coords", 1, 0, O_COORDS}, {"max-match", 0, 0, O_MAXM}, {"no-header", 0, 0, 'H'},
      {"zero-match", 0, 0, '0'}, {"max-count", 1, 0, O_MAXC}, {"unitigs-lengths", 1, 0, 'l'},
      {"unitigs-sequences", 1, 0, 'u'}, {"compact", 0, 0, O_COMPACT}, {"no-compact", 0, 0, O_NOCOMPACT},
      {"k-mer", 1, 0, 'k'}, {"superreads", 1, 0, 'r'}, {"pacbio", 1, 0, 'p'},
      {"device", 1, 0, O_DEV}, {"devices", 1, 0, O_DEVS}, {"batch-bases", 1, 0, O_BATCH},
      {"streams", 1, 0, O_STREAMS}, {"timing", 0, 0, O_TIMING}, {"index-cache", 1, 0, O_CACHE},
      {"parts", 1, 0, O_PARTS}, {0, 0, 0, 0}};
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
    case O_DEV: devices.assign(1, (int)parse_u32(optarg, "--device")); break;
    case O_DEVS: {
      devices.clear();
      std::string l = optarg;
      for (size_t a = 0; a <= l.size();) {
        size_t e = l.find(',', a);
        if (e == std::string::npos) e = l.size();
        devices.push_back((int)parse_u32(l.substr(a, e - a).c_str(), "--devices"));
        a = e + 1;
      }
      break;
    }
    case O_TIMING: timing = true; break;
    case O_CACHE: index_cache = optarg; break;
    case O_PARTS: parts = parse_u32(optarg, "--parts"); break;
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
  if (devices.empty()) devices.push_back(0);

  // one index per distinct device: built on the first, replicated to the rest
  // (jf_aligner.cc:202-203 builds it once and shares it between threads)
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

  pbgpu_run_params rp{};
  rp.pb_paths = pbs.data();
  rp.n_pb_paths = pbs.size();
  rp.coords_path = coords_path;
  rp.details_path = details_path;
  rp.compact = compact ? 1 : 0;
  rp.header = no_header ? 0 : 1;
  rp.zero_match = zero ? 1 : 0;
  rp.aligners_per_device = streams;
  rp.batch_bases = batch_bases;
  rp.host_threads = (int)threads;
  rp.n_parts = parts;
  if (parts > 1 && !coords_path) die("--parts needs --coords");
  pbgpu_run_stats st{};
  const pbgpu_status rs = pbgpu_run(per_entry.data(), per_entry.size(), &ap, &rp, &st);
  const std::string err = rs == PBGPU_OK ? "" : pbgpu_last_error();
  for (auto& b : built) pbgpu_index_free(b.second);
  if (rs != PBGPU_OK) die("align: " + err);
  if (timing)
    fprintf(stderr,
            "{\"wall_s\": %.6f, \"batches\": %llu, \"reads\": %llu, \"bases\": %llu, \"records\": %llu, "
            "\"coords_bytes\": %llu, \"read_s\": %.6f, \"upload_s\": %.6f, \"align_s\": %.6f, \"format_s\": %.6f, "
            "\"d2h_s\": %.6f, \"write_s\": %.6f, \"writer_idle_s\": %.6f, "
            "\"device_allocs\": %llu, \"device_allocs_late\": %llu, \"pinned_allocs\": %llu, "
            "\"pinned_allocs_late\": %llu, \"device_alloc_bytes\": %llu, \"alloc_s\": %.6f, "
            "\"device_peak_bytes\": %llu}\n",
            st.wall_seconds, (unsigned long long)st.n_batches, (unsigned long long)st.n_reads,
            (unsigned long long)st.n_bases, (unsigned long long)st.n_records, (unsigned long long)st.coords_bytes,
            st.read_seconds, st.upload_seconds, st.align_seconds, st.format_seconds, st.d2h_seconds, st.write_seconds,
            st.writer_idle_seconds, (unsigned long long)st.n_device_allocs,
            (unsigned long long)st.n_device_allocs_late, (unsigned long long)st.n_pinned_allocs,
            (unsigned long long)st.n_pinned_allocs_late, (unsigned long long)st.device_alloc_bytes,
            st.alloc_seconds, (unsigned long long)st.device_peak_bytes);
  return 0;
}
