/*
 * pb_oracle_cli.c -- TEST INFRASTRUCTURE ONLY. jf_aligner-compatible
 * command line (jf_aligner_cmdline.yaggo:1-77, jf_aligner.cc:161-233) over
 * the CPU restatement, used to produce golden coords files.
 * Reads are written in input order (what the reference prints at -t 1).
 */
#define _GNU_SOURCE
#include "pb_oracle.h"

#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void usage_die(const char* msg) { fprintf(stderr, "pb_oracle: %s\n", msg); exit(1); }

/* read_unitigs_lengths (misc.cc:11-19): "name len" pairs, index = line */
static int32_t* read_ul(const char* path, size_t* n) {
  FILE* f = fopen(path, "r");
  if (!f) usage_die("Failed to open unitig lengths map file");
  size_t cap = 1024, c = 0;
  int32_t* v = malloc(cap * sizeof(int32_t));
  char name[4096]; unsigned int len;
  while (fscanf(f, "%4095s %u", name, &len) == 2) {
    if (c == cap) { cap *= 2; v = realloc(v, cap * sizeof(int32_t)); }
    v[c++] = (int32_t)len;
  }
  fclose(f);
  *n = c;
  return v;
}

/* read_unitigs_sequences (misc.cc:21-28): length of the line after each header line */
static int32_t* read_us(const char* path, size_t* n) {
  FILE* f = fopen(path, "r");
  if (!f) usage_die("Failed to open unitig sequence file");
  size_t cap = 1024, c = 0;
  int32_t* v = malloc(cap * sizeof(int32_t));
  char* line = NULL; size_t lc = 0; ssize_t l;
  while ((l = getline(&line, &lc, f)) >= 0) {            /* skip header */
    ssize_t s = getline(&line, &lc, f);
    if (s < 0) s = 0;
    else if (s > 0 && line[s - 1] == '\n') --s;
    if (c == cap) { cap *= 2; v = realloc(v, cap * sizeof(int32_t)); }
    v[c++] = (int32_t)s;
  }
  free(line); fclose(f);
  *n = c;
  return v;
}

typedef struct { char** names; char** seqs; uint64_t* lens; size_t n, cap; } readset;

static void rs_push(readset* r, char* name, char* seq, uint64_t len) {
  if (r->n == r->cap) {
    r->cap = r->cap ? 2 * r->cap : 256;
    r->names = realloc(r->names, r->cap * sizeof(char*));
    r->seqs = realloc(r->seqs, r->cap * sizeof(char*));
    r->lens = realloc(r->lens, r->cap * sizeof(uint64_t));
  }
  r->names[r->n] = name; r->seqs[r->n] = seq; r->lens[r->n] = len; ++r->n;
}

/* FASTA / FASTQ reader: header = line after '>'/'@', sequence = concatenated lines */
static void read_reads(const char* path, readset* rs) {
  FILE* f = fopen(path, "r");
  if (!f) usage_die("Can't open PacBio file");
  char* line = NULL; size_t lc = 0; ssize_t l;
  char* name = NULL; char* seq = NULL; size_t sl = 0, sc = 0;
  int fastq = 0;
  while ((l = getline(&line, &lc, f)) >= 0) {
    if (l > 0 && line[l - 1] == '\n') line[--l] = 0;
    if (!name && l == 0) continue;
    if (line[0] == '>' || (line[0] == '@' && (!name || fastq))) {
      if (name) rs_push(rs, name, seq, sl);
      fastq = line[0] == '@';
      name = strdup(line + 1); seq = malloc(1); seq[0] = 0; sl = 0; sc = 1;
      if (fastq) {
        ssize_t s = getline(&line, &lc, f);
        if (s > 0 && line[s - 1] == '\n') line[--s] = 0;
        if (s > 0) { free(seq); seq = strdup(line); sl = (size_t)s; }
        s = getline(&line, &lc, f); /* '+' */
        s = getline(&line, &lc, f); /* qual */
        (void)s;
        rs_push(rs, name, seq, sl); name = NULL; seq = NULL;
      }
      continue;
    }
    if (!name) continue;
    if (sl + (size_t)l + 1 > sc) { while (sl + (size_t)l + 1 > sc) sc *= 2; seq = realloc(seq, sc); }
    memcpy(seq + sl, line, (size_t)l); sl += (size_t)l; seq[sl] = 0;
  }
  if (name) rs_push(rs, name, seq, sl);
  free(line); fclose(f);
}

int main(int argc, char** argv) {
  oracle_params p; oracle_params_default(&p);
  int threads = 1, header = 1, zero = 0, compact = 1, s_given = 0, m_given = 0, k_given = 0;
  const char* coords = NULL; const char* details = NULL; const char* ul_path = NULL; const char* us_path = NULL;
  const char** srs = NULL; size_t n_srs = 0;
  const char** pbs = NULL; size_t n_pbs = 0;
  enum { O_PSA = 256, O_SC, O_SF, O_CAP, O_WIN, O_DETAILS, O_COORDS, O_MAXM, O_MAXC, O_COMPACT, O_NOCOMPACT };
  static struct option lo[] = {
    {"size", 1, 0, 's'}, {"mer", 1, 0, 'm'}, {"fine-mer", 1, 0, 'F'}, {"psa-min", 1, 0, O_PSA},
    {"threads", 1, 0, 't'}, {"stretch-constant", 1, 0, O_SC}, {"stretch-factor", 1, 0, O_SF},
    {"stretch-cap", 1, 0, O_CAP}, {"window-size", 1, 0, O_WIN}, {"forward", 0, 0, 'f'},
    {"bases-matching", 1, 0, 'B'}, {"mers-matching", 1, 0, 'M'}, {"details", 1, 0, O_DETAILS},
    {"coords", 1, 0, O_COORDS}, {"max-match", 0, 0, O_MAXM}, {"no-header", 0, 0, 'H'},
    {"zero-match", 0, 0, '0'}, {"max-count", 1, 0, O_MAXC}, {"unitigs-lengths", 1, 0, 'l'},
    {"unitigs-sequences", 1, 0, 'u'}, {"compact", 0, 0, O_COMPACT}, {"no-compact", 0, 0, O_NOCOMPACT},
    {"k-mer", 1, 0, 'k'}, {"superreads", 1, 0, 'r'}, {"pacbio", 1, 0, 'p'}, {0, 0, 0, 0}};
  int c;
  while ((c = getopt_long(argc, argv, "s:m:F:t:fB:M:H0l:u:k:r:p:", lo, NULL)) != -1) {
    switch (c) {
    case 's': s_given = 1; break; /* required, unused (legacy) */
    case 'm': p.k = (uint32_t)strtoul(optarg, NULL, 10); m_given = 1; break;
    case 'F': p.fine_k = (uint32_t)strtoul(optarg, NULL, 10); break;
    case O_PSA: p.psa_min = (uint32_t)strtoul(optarg, NULL, 10); break;
    case 't': threads = atoi(optarg); break;
    case O_SC: p.stretch_constant = (double)atoi(optarg); break;
    case O_SF: p.stretch_factor = strtod(optarg, NULL); break;
    case O_CAP: p.stretch_cap = strtod(optarg, NULL); break;
    case O_WIN: p.window_size = (uint32_t)strtoul(optarg, NULL, 10); break;
    case 'f': p.forward = 1; break;
    case 'B': p.bases_matching = strtod(optarg, NULL); break;
    case 'M': p.mers_matching = strtod(optarg, NULL); break;
    case O_DETAILS: details = optarg; break;
    case O_COORDS: coords = optarg; break;
    case O_MAXM: p.max_match = 1; break;
    case 'H': header = 0; break;
    case '0': zero = 1; break;
    case O_MAXC: p.max_count = (int32_t)strtoul(optarg, NULL, 10); break;
    case 'l': ul_path = optarg; p.forward = 1; break;
    case 'u': us_path = optarg; p.forward = 1; break;
    case O_COMPACT: compact = 1; break;
    case O_NOCOMPACT: compact = 0; break;
    case 'k': p.unitigs_k = (uint32_t)strtoul(optarg, NULL, 10); k_given = 1; break;
    case 'r': srs = realloc(srs, (n_srs + 1) * sizeof(char*)); srs[n_srs++] = optarg; break;
    case 'p': pbs = realloc(pbs, (n_pbs + 1) * sizeof(char*)); pbs[n_pbs++] = optarg; break;
    default: usage_die("bad option");
    }
  }
  if (!s_given || !m_given) usage_die("-s and -m are required");
  if (!details && !coords) usage_die("No output file given. Doing nothing ungracefully."); /* jf_aligner.cc:166-167 */
  if (ul_path && us_path) usage_die("-u conflicts with -l");
  if (p.max_count == 0) usage_die("--max-count 0 is undefined behaviour in the reference (coarse_aligner.cc:86)");
  int32_t* ul = NULL; size_t n_ul = 0;
  if (ul_path || us_path) {
    if (!k_given) usage_die("-k is required with -l/-u");
    ul = ul_path ? read_ul(ul_path, &n_ul) : read_us(us_path, &n_ul);
    p.unitig_lengths = ul; p.n_unitigs = n_ul;
  } else {
    p.unitigs_k = 0; /* unitigs_lengths() only called with -l/-u (jf_aligner.cc:215) */
  }
  oracle_index* ix = oracle_index_build_fasta(srs, n_srs, p.k, threads);
  if (p.fine_k && oracle_index_build_fine(ix, p.fine_k, threads) != 0)
    usage_die("-F must be in [1, -m] with -m <= 31 (PSA::search assumes the pattern is at most max_size, mer_sa_imp.hpp:366)");
  readset rs; memset(&rs, 0, sizeof(rs));
  for (size_t i = 0; i < n_pbs; ++i) read_reads(pbs[i], &rs);
  size_t olen, dlen = 0;
  char* dtext = NULL;
  char* out = oracle_align_format_ex(ix, &p, (const char* const*)rs.names, (const char* const*)rs.seqs, rs.lens, rs.n,
                                     threads, compact, header, zero, &olen, details ? &dtext : NULL, &dlen);
  FILE* o = coords ? fopen(coords, "w") : stdout;
  if (!o) usage_die("can't open coords output");
  fwrite(out, 1, olen, o);
  if (coords) fclose(o);
  free(out);
  if (details) {
    FILE* d = fopen(details, "w");
    if (!d) usage_die("can't open details output");
    fwrite(dtext, 1, dlen, d);
    fclose(d);
    free(dtext);
  }
  for (size_t i = 0; i < rs.n; ++i) { free(rs.names[i]); free(rs.seqs[i]); }
  free(rs.names); free(rs.seqs); free(rs.lens); free(ul); free(srs); free(pbs);
  oracle_index_free(ix);
  return 0;
}
