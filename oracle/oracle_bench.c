/* TEST INFRASTRUCTURE ONLY: the oracle's side of tools/calib_ref.py's speed
 * calibration against the reference (oracle/ref_harness/ref_bench.cc times the
 * reference on the same inputs).  Single thread for the timed loops.
 *
 *   oracle_bench lookup FASTA K QUERIES
 *     index build (oracle_index_build_fasta), then the exact-match lookup of every
 *     query with its positions written out and summed (the oracle's restatement of
 *     find_pos_size + pos_iterator, superread_parser.hpp:110-192).
 *   oracle_bench lis STRANDS A B CAP WINDOW
 *     oracle_lis (the restatement of lis_align::indices) on every strand.
 * Input formats: see ref_bench.cc.  Prints one JSON line. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pb_oracle.h"

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static char* slurp(const char* path, size_t* len) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  *len = (size_t)ftell(f);
  fseek(f, 0, SEEK_SET);
  char* b = malloc(*len + 1);
  if (fread(b, 1, *len, f) != *len) { fclose(f); free(b); return NULL; }
  fclose(f);
  return b;
}

static int code_of(char c) {
  switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return -1;
  }
}

static int bench_lookup(const char* fasta, uint32_t k, const char* qpath) {
  const double t0 = now();
  const char* paths[1] = {fasta};
  oracle_index* ix = oracle_index_build_fasta(paths, 1, k, 8);
  if (!ix) { fprintf(stderr, "index build failed\n"); return 1; }
  const double t1 = now();
  size_t len = 0;
  char* q = slurp(qpath, &len);
  if (!q) return 1;
  uint32_t n = 0, qk = 0;
  memcpy(&n, q, 4);
  memcpy(&qk, q + 4, 4);
  if (qk != k) { fprintf(stderr, "query k %u != index k %u\n", qk, k); return 1; }
  const size_t cap = 1 << 20;
  uint64_t* pos = malloc(cap * sizeof(uint64_t));
  uint64_t hits = 0, sum = 0;
  const double t2 = now();
  for (uint32_t i = 0; i < n; ++i) {
    const char* p = q + 8 + (size_t)i * k;
    uint64_t code = 0;
    for (uint32_t j = 0; j < k; ++j) code = (code << 2) | (uint64_t)code_of(p[j]);
    const uint64_t c = oracle_index_lookup(ix, code, pos, cap);
    const uint64_t m = c < cap ? c : cap;
    for (uint64_t j = 0; j < m; ++j) sum += pos[j];
    hits += c;
  }
  const double t3 = now();
  printf("{\"text_len\": %llu, \"build_s\": %.3f, \"queries\": %u, \"k\": %u, \"search_s\": %.6f, \"hits\": %llu, "
         "\"checksum\": %llu}\n",
         (unsigned long long)oracle_index_text_len(ix), t1 - t0, n, k, t3 - t2, (unsigned long long)hits,
         (unsigned long long)sum);
  free(pos);
  free(q);
  oracle_index_free(ix);
  return 0;
}

static int bench_lis(const char* spath, double a, double b, double cap, uint32_t window) {
  size_t len = 0;
  char* f = slurp(spath, &len);
  if (!f) return 1;
  const char* p = f;
  uint32_t n = 0;
  memcpy(&n, p, 4);
  p += 4;
  /* index the strands first, so the timed loop is the LIS alone */
  const int32_t** X = malloc((size_t)n * sizeof(*X));
  uint32_t* N = malloc((size_t)n * sizeof(*N));
  uint64_t elems = 0;
  uint32_t maxn = 1;
  for (uint32_t s = 0; s < n; ++s) {
    memcpy(&N[s], p, 4);
    p += 4;
    X[s] = (const int32_t*)p;
    p += (size_t)N[s] * 8;
    elems += N[s];
    if (N[s] > maxn) maxn = N[s];
  }
  uint32_t* out = malloc((size_t)maxn * sizeof(uint32_t));
  uint64_t total = 0;
  const double t0 = now();
  for (uint32_t s = 0; s < n; ++s) total += oracle_lis(X[s], N[s], window, 0, a, b, cap, 0, a, out);
  const double t1 = now();
  printf("{\"strands\": %u, \"elements\": %llu, \"lis_s\": %.6f, \"lis_total\": %llu}\n", n, (unsigned long long)elems,
         t1 - t0, (unsigned long long)total);
  free(out);
  free(N);
  free(X);
  free(f);
  return 0;
}

int main(int argc, char** argv) {
  if (argc == 5 && !strcmp(argv[1], "lookup")) return bench_lookup(argv[2], (uint32_t)atoi(argv[3]), argv[4]);
  if (argc == 7 && !strcmp(argv[1], "lis"))
    return bench_lis(argv[2], atof(argv[3]), atof(argv[4]), atof(argv[5]), (uint32_t)atoi(argv[6]));
  fprintf(stderr, "usage: oracle_bench lookup FASTA K QUERIES | lis STRANDS A B CAP WINDOW\n");
  return 1;
}
