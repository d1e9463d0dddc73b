// TEST INFRASTRUCTURE (our code). Times two components of the reference on
// inputs written by tools/calib_ref.py, for the CPU baseline's speed ratio to
// the reference (calibrate the restatement against the reference
// on identical inputs).  Single thread for the timed loops.
//
//   ref_bench psa FASTA MIN MAX THREADS QUERIES
//     the reference's PSA (src_psa/psa.hpp:130-153, mer_sa_imp.hpp) over the text
//     sequence_psa::append_fasta makes (superread_parser.cc:12-46), then
//     PSA::search of every query (the find_pos_size of superread_parser.hpp:183-192)
//     and a walk over every hit's text position (pos_iterator, :110-140).
//     QUERIES: u32 n, u32 k, then n * k bytes.
//   ref_bench lis STRANDS A B CAP WINDOW
//     lis_align::indices (lis_align.hpp:207-214) with affine_capped(A, B, CAP) and
//     linear(A), as coarse_aligner builds them (coarse_aligner.hpp:55-72), on every
//     strand.  STRANDS: u32 n, then per strand u32 N and N pairs of i32.
// Prints one JSON line.
#include <unistd.h>
#include <cassert>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <src_psa/global_timer.hpp>
#include <src_psa/compact_dna.hpp>
#include <src_psa/psa.hpp>
#include <src_lis/lis_align.hpp>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static std::vector<char> slurp(const char* path) {
  std::ifstream is(path, std::ios::binary);
  return std::vector<char>((std::istreambuf_iterator<char>(is)), std::istreambuf_iterator<char>());
}

static int bench_psa(const char* fasta, unsigned min_size, unsigned max_size, unsigned threads, const char* qpath) {
  const double t0 = now();
  std::ifstream is(fasta);
  std::vector<uint64_t> seq;
  size_t off = 0;
  std::string line;
  while (std::getline(is, line)) {
    if (!line.empty() && line[0] == '>') continue;
    if (seq.size() * sizeof(uint64_t) * 4 < line.size() + off)
      seq.resize(std::max(1 + (size_t)(line.size() + off) / (sizeof(uint64_t) * 4), seq.size() * 2));
    compact_dna::copy_from_str(compact_dna::iterator(seq.data(), 2, 0) + off, line);
    off += line.size();
  }
  PSA<compact_dna::const_iterator> psa(compact_dna::const_iterator_at(seq.data()), off, min_size, max_size, threads);
  const double t1 = now();
  const std::vector<char> q = slurp(qpath);
  uint32_t n = 0, k = 0;
  memcpy(&n, q.data(), 4);
  memcpy(&k, q.data() + 4, 4);
  const char* pat = q.data() + 8;
  uint64_t hits = 0, sum = 0;
  const double t2 = now();
  for (uint32_t i = 0; i < n; ++i) {
    const auto r = psa.search(pat + (size_t)i * k, k);
    hits += r.first;
    for (uint64_t j = 0; j < r.first; ++j) sum += psa[r.second + j];
  }
  const double t3 = now();
  printf("{\"text_len\": %zu, \"build_s\": %.3f, \"queries\": %u, \"k\": %u, \"search_s\": %.6f, \"hits\": %llu, "
         "\"checksum\": %llu}\n",
         off, t1 - t0, n, k, t3 - t2, (unsigned long long)hits, (unsigned long long)sum);
  return 0;
}

static int bench_lis(const char* spath, double a, double b, double cap, size_t window) {
  const std::vector<char> f = slurp(spath);
  const char* p = f.data();
  uint32_t n = 0;
  memcpy(&n, p, 4);
  p += 4;
  std::vector<std::vector<std::pair<int, int>>> S(n);
  uint64_t elems = 0;
  for (auto& s : S) {
    uint32_t N = 0;
    memcpy(&N, p, 4);
    p += 4;
    s.resize(N);
    for (auto& x : s) {
      memcpy(&x.first, p, 4);
      memcpy(&x.second, p + 4, 4);
      p += 8;
    }
    elems += N;
  }
  lis_align::affine_capped am(a, b, cap);
  lis_align::linear ls(a);
  std::forward_list<lis_align::element<double>> L;
  std::vector<unsigned int> P, res;
  uint64_t total = 0;
  const double t0 = now();
  for (const auto& s : S) {  // the do_LIS overload with a reused P (pb_aligner.hpp:34-38)
    L.clear();
    res.clear();
    total += lis_align::indices(s.cbegin(), s.cend(), L, P, res, window, am, ls);
  }
  const double t1 = now();
  printf("{\"strands\": %u, \"elements\": %llu, \"lis_s\": %.6f, \"lis_total\": %llu}\n", n,
         (unsigned long long)elems, t1 - t0, (unsigned long long)total);
  return 0;
}

int main(int argc, char* argv[]) {
  if (argc == 7 && !strcmp(argv[1], "psa"))
    return bench_psa(argv[2], atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), argv[6]);
  if (argc == 7 && !strcmp(argv[1], "lis"))
    return bench_lis(argv[2], atof(argv[3]), atof(argv[4]), atof(argv[5]), atoi(argv[6]));
  fprintf(stderr, "usage: ref_bench psa FASTA MIN MAX THREADS QUERIES | lis STRANDS A B CAP WINDOW\n");
  return 1;
}
