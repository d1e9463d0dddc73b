/*
 * pb_oracle.c -- TEST INFRASTRUCTURE ONLY (parity oracle + "port" CPU
 * baseline). Never linked into the product path. See pb_oracle.h for the
 * pinning status of each piece.
 *
 * Build: -O2 -ffp-contract=off (the reference is built for plain x86-64:
 * SSE2 doubles, no FMA; every double expression below keeps the reference's
 * operation order).
 */
#define _GNU_SOURCE
#include "pb_oracle.h"

#include <errno.h>
#include <stdarg.h>
#include <limits.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define DIE(...) do { fprintf(stderr, "pb_oracle: " __VA_ARGS__); fputc('\n', stderr); abort(); } while (0)

static void* xmalloc(size_t n) { void* p = malloc(n ? n : 1); if (!p) DIE("out of memory (%zu)", n); return p; }
static void* xcalloc(size_t n, size_t s) { void* p = calloc(n ? n : 1, s ? s : 1); if (!p) DIE("out of memory"); return p; }
static void* xrealloc(void* q, size_t n) { void* p = realloc(q, n ? n : 1); if (!p) DIE("out of memory (%zu)", n); return p; }
static char* xstrdup(const char* s) { size_t l = strlen(s); char* r = xmalloc(l + 1); memcpy(r, s, l + 1); return r; }

/* ======================================================================
 * Jellyfish mer_dna restatement (k <= 32, one word, first base MSB).
 * ==================================================================== */
static inline int jf_code(unsigned char c) {
  switch (c) {
  case 'A': case 'a': return 0;
  case 'C': case 'c': return 1;
  case 'G': case 'g': return 2;
  case 'T': case 't': return 3;
  default: return -1;
  }
}
static inline uint64_t mer_mask(uint32_t k) { return k >= 32 ? ~(uint64_t)0 : (((uint64_t)1 << (2 * k)) - 1); }

/* is_ssr (coarse_aligner.cc:8-15): nm.shift_right(nm.base(0)) twice,
 * i.e. cyclic right rotations by one base. */
int oracle_is_ssr(uint64_t m, uint32_t k) {
  uint64_t nm = m;
  for (int i = 0; i < 2; ++i) {
    uint64_t b = nm & 3;
    nm = (nm >> 2) | (b << (2 * (k - 1)));
    if (nm == m) return 1;
  }
  return 0;
}

/* ======================================================================
 * compact_dna line encoding (compact_dna.hpp:89-136), 8-aligned buffer.
 * ==================================================================== */
void oracle_encode_line(const char* line, size_t len, uint8_t* codes) {
  size_t fast = len & ~(size_t)7;
  for (size_t i = 0; i < fast; ++i) {
    unsigned b = (unsigned char)line[i];
    codes[i] = (uint8_t)(((b >> 1) ^ (b >> 2)) & 3); /* char_to_code8 */
  }
  uint8_t c = 0; /* copy_from_str_slow: unknown chars repeat the last code */
  for (size_t i = fast; i < len; ++i) {
    int x = jf_code((unsigned char)line[i]);
    if (x >= 0) c = (uint8_t)x;
    codes[i] = c;
  }
}

/* ======================================================================
 * super_read_name (super_read_name.cc:74-90, 11-20, 38-47).
 * ==================================================================== */
typedef struct { uint32_t n; uint32_t* id; uint8_t* ori; } unitig_list;

static void unitigs_parse(const char* name, unitig_list* out) {
  out->n = 0; out->id = NULL; out->ori = NULL;
  size_t len = strlen(name);
  if (len == 0) return;
  uint32_t cap = 4, n = 0;
  uint32_t* id = xmalloc(cap * sizeof(uint32_t));
  uint8_t* ori = xmalloc(cap);
  size_t pn = 0;
  for (;;) {
    const char* us = strchr(name + pn, '_');
    const char* s = name + pn;
    char* end;
    errno = 0;
    unsigned long v = strtoul(s, &end, 10);
    if (end == s || errno == ERANGE) { free(id); free(ori); return; } /* invalid_argument -> clear */
    char oc = us ? us[-1] : name[len - 1];
    if (n == cap) { cap *= 2; id = xrealloc(id, cap * sizeof(uint32_t)); ori = xrealloc(ori, cap); }
    id[n] = ((uint32_t)v) & 0x7fffffffu; /* u_id_ori: id_:31 */
    ori[n] = (oc == 'R');
    ++n;
    if (!us) break;
    pn = (size_t)(us - name) + 1;
  }
  out->n = n; out->id = id; out->ori = ori;
}

static char* unitigs_name(const unitig_list* u) {
  size_t cap = 16 + (size_t)u->n * 13, o = 0;
  char* r = xmalloc(cap);
  r[0] = 0;
  for (uint32_t i = 0; i < u->n; ++i)
    o += (size_t)snprintf(r + o, cap - o, "%s%u%c", i ? "_" : "", u->id[i], u->ori[i] ? 'R' : 'F');
  return r;
}

int oracle_sr_name_reverse(const char* name, char* out, size_t cap) {
  unitig_list u;
  unitigs_parse(name, &u);
  if (u.n == 0) { snprintf(out, cap, "%s", name); return 0; }
  unitig_list r = { u.n, xmalloc(u.n * sizeof(uint32_t)), xmalloc(u.n) };
  for (uint32_t i = 0; i < u.n; ++i) { r.id[i] = u.id[u.n - 1 - i]; r.ori[i] = !u.ori[u.n - 1 - i]; }
  char* s = unitigs_name(&r);
  snprintf(out, cap, "%s", s);
  free(s); free(u.id); free(u.ori); free(r.id); free(r.ori);
  return (int)u.n;
}

/* ======================================================================
 * Index: every text position x in [0, n-k] sorted by (k-mer, x desc).
 * Restates the observable behaviour of PSA::search (mer_sa_imp.hpp:369-479)
 * for k > psa_min: the exact occurrence set in descending position order
 * (sort tie-break si > sj, mer_sa_imp.hpp:363).
 * ==================================================================== */
typedef struct {
  uint64_t     start;   /* global text offset */
  uint32_t     len;
  char*        name_fwd;
  char*        name_bwd;
  unitig_list  fwd;     /* unitigs of the fwd name (bwd = reversed) */
} sr_rec;

struct oracle_index {
  uint32_t k;
  uint64_t n;           /* text length */
  uint8_t* text;        /* one 2-bit code per byte */
  size_t   n_sr, cap_sr;
  sr_rec*  sr;
  uint64_t n_pos;       /* n - k + 1 (0 if n < k) */
  uint64_t* keys;       /* sorted k-mer codes */
  uint64_t* pos;        /* positions, same order */
  uint32_t dir_bits;
  uint64_t* dir;        /* bucket directory over the top dir_bits of the code */
  /* fine (-F) sub-index (oracle_index_build_fine) */
  uint32_t fk, fshift, fdir_bits;
  uint64_t fn_pos;
  uint64_t* fkeys;      /* (T[x, x+k) zero-padded past n) << 1 | (x + k <= n), sorted */
  uint64_t* fpos;
  uint64_t* fdir;       /* directory over the top fdir_bits of the fine_k-mer */
};

typedef struct {
  uint64_t* src_k; uint64_t* src_v; uint64_t* dst_k; uint64_t* dst_v;
  uint64_t lo, hi; uint32_t shift; uint64_t* hist; /* 256 per thread */
  pthread_barrier_t* bar; int tid, nt; uint64_t** all_hist;
} radix_job;

static void* radix_hist(void* arg) {
  radix_job* j = arg;
  memset(j->hist, 0, 256 * sizeof(uint64_t));
  for (uint64_t i = j->lo; i < j->hi; ++i) j->hist[(j->src_k[i] >> j->shift) & 255]++;
  return NULL;
}
static void* radix_scatter(void* arg) {
  radix_job* j = arg;
  for (uint64_t i = j->lo; i < j->hi; ++i) {
    uint64_t d = (j->src_k[i] >> j->shift) & 255;
    uint64_t o = j->hist[d]++;
    j->dst_k[o] = j->src_k[i];
    j->dst_v[o] = j->src_v[i];
  }
  return NULL;
}

/* Stable LSD radix sort of (keys, vals) on the low `bits` bits. */
static void radix_sort(uint64_t** pk, uint64_t** pv, uint64_t n, uint32_t bits, int nt) {
  if (nt < 1) nt = 1;
  if (n < (uint64_t)nt * 4096) nt = 1;
  uint64_t* k2 = xmalloc(n * sizeof(uint64_t));
  uint64_t* v2 = xmalloc(n * sizeof(uint64_t));
  uint64_t* k = *pk; uint64_t* v = *pv;
  radix_job* jobs = xcalloc((size_t)nt, sizeof(radix_job));
  uint64_t* hists = xcalloc((size_t)nt * 256, sizeof(uint64_t));
  pthread_t* th = xcalloc((size_t)nt, sizeof(pthread_t));
  for (uint32_t shift = 0; shift < bits; shift += 8) {
    for (int t = 0; t < nt; ++t) {
      jobs[t].src_k = k; jobs[t].src_v = v; jobs[t].dst_k = k2; jobs[t].dst_v = v2;
      jobs[t].lo = n * (uint64_t)t / (uint64_t)nt; jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)nt;
      jobs[t].shift = shift; jobs[t].hist = hists + 256 * (size_t)t;
    }
    if (nt == 1) radix_hist(&jobs[0]);
    else { for (int t = 0; t < nt; ++t) pthread_create(&th[t], NULL, radix_hist, &jobs[t]);
           for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL); }
    uint64_t sum = 0;
    for (int d = 0; d < 256; ++d)
      for (int t = 0; t < nt; ++t) { uint64_t c = hists[256 * (size_t)t + d]; hists[256 * (size_t)t + d] = sum; sum += c; }
    if (nt == 1) radix_scatter(&jobs[0]);
    else { for (int t = 0; t < nt; ++t) pthread_create(&th[t], NULL, radix_scatter, &jobs[t]);
           for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL); }
    uint64_t* tk = k; k = k2; k2 = tk;
    uint64_t* tv = v; v = v2; v2 = tv;
  }
  free(k2); free(v2); free(jobs); free(hists); free(th);
  *pk = k; *pv = v;
}


static void index_add_sr(oracle_index* ix, const char* header, uint64_t start, uint64_t len) {
  if (ix->n_sr == ix->cap_sr) { ix->cap_sr = ix->cap_sr ? 2 * ix->cap_sr : 64; ix->sr = xrealloc(ix->sr, ix->cap_sr * sizeof(sr_rec)); }
  sr_rec* r = &ix->sr[ix->n_sr++];
  r->start = start; r->len = (uint32_t)len;
  r->name_fwd = xstrdup(header);
  unitigs_parse(header, &r->fwd);
  if (r->fwd.n > 0) { /* frag_info.hpp:22-35 */
    unitig_list b = { r->fwd.n, xmalloc(r->fwd.n * sizeof(uint32_t)), xmalloc(r->fwd.n) };
    for (uint32_t i = 0; i < b.n; ++i) { b.id[i] = r->fwd.id[b.n - 1 - i]; b.ori[i] = !r->fwd.ori[b.n - 1 - i]; }
    r->name_bwd = unitigs_name(&b);
    free(b.id); free(b.ori);
  } else {
    r->name_bwd = xstrdup(header);
  }
}

static void text_reserve(oracle_index* ix, uint64_t* cap, uint64_t need) {
  if (need <= *cap) return;
  uint64_t nc = *cap ? *cap : 1 << 16;
  while (nc < need) nc *= 2;
  ix->text = xrealloc(ix->text, nc);
  *cap = nc;
}

static void index_finish(oracle_index* ix, int threads) {
  uint32_t k = ix->k;
  ix->n_pos = ix->n >= k ? ix->n - k + 1 : 0;
  uint64_t np = ix->n_pos;
  uint64_t* keys = xmalloc((np ? np : 1) * sizeof(uint64_t));
  uint64_t* pos = xmalloc((np ? np : 1) * sizeof(uint64_t));
  /* positions in DESCENDING order so that the stable sort keeps x desc */
  if (np) {
    uint64_t m = 0, mask = mer_mask(k);
    for (uint32_t i = 0; i + 1 < k; ++i) m = (m << 2) | ix->text[i];
    for (uint64_t x = 0; x < np; ++x) {
      m = ((m << 2) | ix->text[x + k - 1]) & mask;
      keys[np - 1 - x] = m;
      pos[np - 1 - x] = x;
    }
  }
  radix_sort(&keys, &pos, np, 2 * k, threads);
  ix->keys = keys; ix->pos = pos;
  ix->dir_bits = 2 * k < 20 ? 2 * k : 20;
  size_t nd = ((size_t)1 << ix->dir_bits) + 1;
  ix->dir = xcalloc(nd, sizeof(uint64_t));
  uint32_t sh = 2 * k - ix->dir_bits;
  for (uint64_t i = 0; i < np; ++i) ix->dir[(keys[i] >> sh) + 1]++;
  for (size_t i = 1; i < nd; ++i) ix->dir[i] += ix->dir[i - 1];
}

static oracle_index* index_new(uint32_t k) {
  if (k < 1 || k > 32) DIE("k must be in [1,32]");
  oracle_index* ix = xcalloc(1, sizeof(oracle_index));
  ix->k = k;
  return ix;
}

oracle_index* oracle_index_build_fasta(const char* const* paths, size_t n_paths, uint32_t k, int threads) {
  oracle_index* ix = index_new(k);
  uint64_t cap = 0;
  char* line = NULL; size_t lcap = 0;
  char* header = xstrdup("");
  for (size_t f = 0; f < n_paths; ++f) {
    FILE* fp = fopen(paths[f], "r");
    if (!fp) DIE("Can't open file %s", paths[f]);
    int c = fgetc(fp);
    if (c != '>') DIE("Not in fasta format");
    ungetc(c, fp);
    ssize_t l;
    int have = 0; uint64_t start = ix->n;
    while ((l = getline(&line, &lcap, fp)) >= 0) {
      if (l > 0 && line[l - 1] == '\n') line[--l] = 0; /* std::getline */
      if (line[0] == '>') {
        if (have && ix->n > start) index_add_sr(ix, header, start, ix->n - start);
        free(header); header = xstrdup(line + 1); have = 1; start = ix->n;
        continue;
      }
      text_reserve(ix, &cap, ix->n + (uint64_t)l);
      oracle_encode_line(line, (size_t)l, ix->text + ix->n);
      ix->n += (uint64_t)l;
    }
    if (have && ix->n > start) index_add_sr(ix, header, start, ix->n - start);
    fclose(fp);
  }
  free(line); free(header);
  index_finish(ix, threads);
  return ix;
}

oracle_index* oracle_index_build_mem(const char* const* names, const char* const* seqs,
                                     const uint64_t* lens, size_t n, uint32_t k, int threads) {
  oracle_index* ix = index_new(k);
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += lens[i];
  ix->text = xmalloc(total ? total : 1);
  for (size_t i = 0; i < n; ++i) {
    if (lens[i] == 0) continue;
    oracle_encode_line(seqs[i], lens[i], ix->text + ix->n);
    index_add_sr(ix, names[i], ix->n, lens[i]);
    ix->n += lens[i];
  }
  index_finish(ix, threads);
  return ix;
}

void oracle_index_free(oracle_index* ix) {
  if (!ix) return;
  for (size_t i = 0; i < ix->n_sr; ++i) {
    free(ix->sr[i].name_fwd); free(ix->sr[i].name_bwd);
    free(ix->sr[i].fwd.id); free(ix->sr[i].fwd.ori);
  }
  free(ix->sr); free(ix->text); free(ix->keys); free(ix->pos); free(ix->dir);
  free(ix->fkeys); free(ix->fpos); free(ix->fdir); free(ix);
}
size_t oracle_index_nb_sr(const oracle_index* ix) { return ix->n_sr; }
uint64_t oracle_index_text_len(const oracle_index* ix) { return ix->n; }
uint32_t oracle_index_sr_len(const oracle_index* ix, size_t i) { return ix->sr[i].len; }
const char* oracle_index_sr_name(const oracle_index* ix, size_t i, int bwd) { return bwd ? ix->sr[i].name_bwd : ix->sr[i].name_fwd; }
int oracle_index_base(const oracle_index* ix, uint64_t pos) { return ix->text[pos]; }

/* [lo, hi) range of code in the sorted arrays */
static void index_range(const oracle_index* ix, uint64_t code, uint64_t* plo, uint64_t* phi) {
  uint32_t sh = 2 * ix->k - ix->dir_bits;
  uint64_t b = code >> sh;
  uint64_t lo = ix->dir[b], hi = ix->dir[b + 1];
  uint64_t l = lo, h = hi;
  while (l < h) { uint64_t m = l + (h - l) / 2; if (ix->keys[m] < code) l = m + 1; else h = m; }
  uint64_t first = l;
  h = hi;
  while (l < h) { uint64_t m = l + (h - l) / 2; if (ix->keys[m] <= code) l = m + 1; else h = m; }
  *plo = first; *phi = l;
}

uint64_t oracle_index_lookup(const oracle_index* ix, uint64_t code, uint64_t* pos_out, uint64_t cap) {
  uint64_t lo, hi;
  index_range(ix, code, &lo, &hi);
  for (uint64_t i = lo; i < hi && i - lo < cap; ++i) pos_out[i - lo] = ix->pos[i];
  return hi - lo;
}

/* ----------------------------------------------------------------------
 * Fine sub-index.  For a pattern P of fine_k bases the reference searches the
 * PSA built with mer_size = min(fine_k, psa_min) and max_size = k
 * (jf_aligner.cc:202-203).  Its matches are the x with T[x, x+fine_k) == P,
 * x <= n - fine_k, in SA order: sort_one_mer (mer_sa_imp.hpp:351-364)
 * compares T[x+mer_size, min(n, x+k)) lexicographically (a proper prefix
 * first) and breaks ties by x descending; the bases mer_size..fine_k are P's
 * own, so the order is that of the extension T[x+fine_k, min(n, x+k)).
 * Key = the k bases at x, zero-padded past n, << 1 | (x + k <= n): a
 * truncated extension sorts before any full one it prefixes, and two
 * truncated ones with equal padded keys keep x descending (the shorter one,
 * at the larger x, first), as the reference's comparator does.
 * ------------------------------------------------------------------------ */
int oracle_index_build_fine(oracle_index* ix, uint32_t fk, int threads) {
  const uint32_t k = ix->k;
  if (fk < 1 || fk > k || k > 31) return -1;
  free(ix->fkeys); free(ix->fpos); free(ix->fdir);
  ix->fk = fk;
  ix->fshift = 2 * (k - fk) + 1;
  const uint64_t n = ix->n;
  const uint64_t np = n >= fk ? n - fk + 1 : 0;
  ix->fn_pos = np;
  uint64_t* keys = xmalloc((np ? np : 1) * sizeof(uint64_t));
  uint64_t* pos = xmalloc((np ? np : 1) * sizeof(uint64_t));
  const uint64_t mask = mer_mask(k);
  uint64_t m = 0;
  for (uint32_t i = 0; i + 1 < k; ++i) m = (m << 2) | (i < n ? ix->text[i] : 0);
  for (uint64_t x = 0; x < np; ++x) {
    const uint64_t q = x + k - 1;
    m = ((m << 2) | (q < n ? ix->text[q] : 0)) & mask;
    keys[np - 1 - x] = (m << 1) | (x + k <= n ? 1u : 0u);
    pos[np - 1 - x] = x;
  }
  radix_sort(&keys, &pos, np, 2 * k + 1, threads);
  ix->fkeys = keys; ix->fpos = pos;
  ix->fdir_bits = 2 * fk < 20 ? 2 * fk : 20;
  const size_t nd = ((size_t)1 << ix->fdir_bits) + 1;
  ix->fdir = xcalloc(nd, sizeof(uint64_t));
  const uint32_t sh = ix->fshift + 2 * fk - ix->fdir_bits;
  for (uint64_t i = 0; i < np; ++i) ix->fdir[(keys[i] >> sh) + 1]++;
  for (size_t i = 1; i < nd; ++i) ix->fdir[i] += ix->fdir[i - 1];
  return 0;
}

static void fine_range(const oracle_index* ix, uint64_t code, uint64_t* plo, uint64_t* phi) {
  const uint32_t sh = 2 * ix->fk - ix->fdir_bits;
  const uint64_t b = code >> sh;
  uint64_t l = ix->fdir[b], h = ix->fdir[b + 1];
  const uint64_t hi0 = h;
  while (l < h) { uint64_t md = l + (h - l) / 2; if ((ix->fkeys[md] >> ix->fshift) < code) l = md + 1; else h = md; }
  const uint64_t first = l;
  h = hi0;
  while (l < h) { uint64_t md = l + (h - l) / 2; if ((ix->fkeys[md] >> ix->fshift) <= code) l = md + 1; else h = md; }
  *plo = first; *phi = l;
}

uint64_t oracle_index_lookup_fine(const oracle_index* ix, uint64_t code, uint64_t* pos_out, uint64_t cap) {
  if (!ix->fkeys) DIE("fine sub-index not built");
  uint64_t lo, hi;
  fine_range(ix, code, &lo, &hi);
  for (uint64_t i = lo; i < hi && i - lo < cap; ++i) pos_out[i - lo] = ix->fpos[i];
  return hi - lo;
}

/* pos_iterator::operator++ (superread_parser.hpp:110-140): SR holding x */
static size_t sr_of(const oracle_index* ix, uint64_t x) {
  size_t l = 0, h = ix->n_sr;
  while (l < h) { size_t m = l + (h - l) / 2; if (ix->sr[m].start <= x) l = m + 1; else h = m; }
  return l - 1;
}

/* ======================================================================
 * lis_align (lis_align.hpp:17-214) -- literal restatement with a singly
 * linked list and sum_buffer windows.
 * ==================================================================== */
typedef struct { double f, s; } sp_t;
typedef struct {
  sp_t*  v;        /* window storage (W entries) */
  size_t next;
  int    filled;
  sp_t   sum;
} sumbuf;

static inline int sb_will_be_filled(const sumbuf* b, size_t W) { return b->filled || b->next == W - 1; }
static inline sp_t sb_test_sum(const sumbuf* b, sp_t x) {
  sp_t r = { b->sum.f + x.f, b->sum.s + x.s };
  if (b->filled || b->next > 0) { r.f -= b->v[b->next].f; r.s -= b->v[b->next].s; }
  return r;
}
static inline void sb_push(sumbuf* b, size_t W, sp_t x) {
  if (W) {
    b->sum = sb_test_sum(b, x);
    b->v[b->next] = x;
    b->next = (b->next + 1) % W;
    b->filled = b->filled || (b->next == 0);
  }
}

typedef struct lnode {
  int32_t  next;   /* index of next node, -1 = end */
  uint32_t elt, len;
  sumbuf   win;
  sp_t     full;
} lnode;

typedef struct {
  int mer_kind; double a, b, C;
  int seq_kind; double sa;
} accept_t;

static inline int accept_mer(const accept_t* ac, sp_t s) {
  if (ac->mer_kind) return 1;
  return (s.f <= ac->b + ac->a * s.s) && (s.s <= ac->b + ac->a * s.f) && s.f <= ac->C && s.s <= ac->C;
}
static inline int accept_seq(const accept_t* ac, sp_t s) {
  if (ac->seq_kind) return 1;
  return (s.f <= ac->sa * s.s) && (s.s <= ac->sa * s.f);
}

typedef struct {
  lnode* nodes; size_t cap_nodes;
  sp_t*  wins;  size_t cap_wins;
  uint32_t* P;  size_t cap_P;
} lis_scratch;

static void lis_scratch_free(lis_scratch* s) { free(s->nodes); free(s->wins); free(s->P); memset(s, 0, sizeof(*s)); }

/* compute_L_P + indices_reversed. X is N (first, second) pairs. */
static uint32_t lis_run(const int32_t* X, uint32_t N, size_t W, const accept_t* ac,
                        lis_scratch* sc, uint32_t* out) {
  if (N == 0) return 0;
  if (sc->cap_nodes < N) { sc->cap_nodes = N; sc->nodes = xrealloc(sc->nodes, N * sizeof(lnode)); }
  if (sc->cap_wins < (size_t)N * W) { sc->cap_wins = (size_t)N * W; sc->wins = xrealloc(sc->wins, sc->cap_wins * sizeof(sp_t)); }
  if (sc->cap_P < N) { sc->cap_P = N; sc->P = xrealloc(sc->P, N * sizeof(uint32_t)); }
  lnode* nd = sc->nodes; uint32_t* P = sc->P;
  int32_t head = -1;
  uint32_t longest = 0, longest_ind = 0;
  for (uint32_t i = 0; i < N; ++i) {
    lnode* e = &nd[i];
    e->elt = i; e->len = 1; e->next = -1;
    e->win.v = sc->wins + (size_t)i * W; e->win.next = 0; e->win.filled = 0; e->win.sum.f = 0; e->win.sum.s = 0;
    for (size_t w = 0; w < W; ++w) { e->win.v[w].f = 0; e->win.v[w].s = 0; }
    e->full.f = 0; e->full.s = 0;
    P[i] = N;
    int32_t prev = -1; /* -1 = before_begin */
    for (int32_t it = head; it >= 0 && nd[it].len >= e->len; it = nd[it].next) {
      const uint32_t j = nd[it].elt;
      if (X[2 * i + 1] > X[2 * j + 1] && e->len < nd[it].len + 1) {
        sp_t add = { (double)(X[2 * i] - X[2 * j]), (double)(X[2 * i + 1] - X[2 * j + 1]) };
        sp_t ns = sb_test_sum(&nd[it].win, add);
        if (!sb_will_be_filled(&nd[it].win, W) || accept_mer(ac, ns)) {
          e->len = nd[it].len + 1;
          P[i] = j;
          /* e_longest.span_window = it->span_window (vector copy) */
          for (size_t w = 0; w < W; ++w) e->win.v[w] = nd[it].win.v[w];
          e->win.next = nd[it].win.next; e->win.filled = nd[it].win.filled; e->win.sum = nd[it].win.sum;
          sb_push(&e->win, W, add);
          e->full.f = nd[it].full.f + add.f; e->full.s = nd[it].full.s + add.s;
          break;
        }
      }
      if (prev < 0 || nd[it].len < nd[prev].len) prev = it;
    }
    if (prev < 0) { e->next = head; head = (int32_t)i; }
    else { e->next = nd[prev].next; nd[prev].next = (int32_t)i; }
    if (longest < e->len && accept_seq(ac, e->full)) { longest = e->len; longest_ind = i; }
  }
  uint32_t s = longest_ind;
  for (uint32_t t = 0; t < longest; ++t, s = P[s]) out[longest - 1 - t] = s;
  return longest;
}

uint32_t oracle_lis(const int32_t* X, uint32_t N, uint32_t window, int mer_kind, double a, double b, double C,
                    int seq_kind, double seq_a, uint32_t* out) {
  accept_t ac = { mer_kind, a, b, C, seq_kind, seq_a };
  lis_scratch sc; memset(&sc, 0, sizeof(sc));
  uint32_t r = lis_run(X, N, window, &ac, &sc, out);
  lis_scratch_free(&sc);
  return r;
}

/* ======================================================================
 * least_square_2d (least_square_2d.hpp:37-80)
 * ==================================================================== */
typedef struct { double EX, EY, EXX, EXY, VX, CXY, NB; long n; } lsq_t;
static inline void lsq_add(lsq_t* l, double x, double y) {
  ++l->n;
  const double deltaX = x - l->EX;
  l->EX += deltaX / (double)l->n;
  const double ndeltaX = x - l->EX;
  l->VX += deltaX * ndeltaX;
  const double deltaY = y - l->EY;
  l->EY += deltaY / (double)l->n;
  const double ndeltaY = y - l->EY;
  const double deltaXX = x * x - l->EXX;
  l->EXX += deltaXX / (double)l->n;
  const double deltaXY = x * y - l->EXY;
  l->EXY += deltaXY / (double)l->n;
  l->CXY += deltaX * ndeltaY;
  l->NB += deltaXY * ndeltaX - deltaXX * ndeltaY;
}

void oracle_lsq(const double* x, const double* y, size_t n, double out[9]) {
  lsq_t l; memset(&l, 0, sizeof(l));
  for (size_t i = 0; i < n; ++i) lsq_add(&l, x[i], y[i]);
  out[0] = l.EX; out[1] = l.EY; out[2] = l.EXX; out[3] = l.EXY; out[4] = l.VX; out[5] = l.CXY; out[6] = l.NB;
  out[7] = l.CXY / l.VX; out[8] = l.NB / l.VX;
}

/* ======================================================================
 * compute_kmers_info (pb_aligner.cc:84-143)
 * ==================================================================== */
#define INVALID_ID 0x7fffffffu
typedef struct {
  int32_t* mers; int32_t* bases; uint32_t size; /* size 0 => empty (error/clear) */
  const uint32_t* ids; uint32_t n_ids; int rev;  /* unitig ids, rev => read backwards */
  uint32_t cunitig; int32_t cend; int32_t prev_pos;
  uint32_t align_k, unitigs_k;
  const int32_t* ul; size_t n_ul;
  int error;
} kinfo_t;

static inline uint32_t ki_id(const kinfo_t* s, size_t i) {
  if (i >= s->n_ids) return INVALID_ID;
  return s->rev ? s->ids[s->n_ids - 1 - i] : s->ids[i];
}

static void kinfo_init(kinfo_t* s, const uint32_t* ids, uint32_t n_ids, int rev,
                       uint32_t unitigs_k, uint32_t align_k, const int32_t* ul, size_t n_ul,
                       int32_t* mers, int32_t* bases) {
  s->mers = mers; s->bases = bases; s->size = 0;
  s->ids = ids; s->n_ids = n_ids; s->rev = rev;
  s->cunitig = 0; s->cend = 0; s->prev_pos = (int32_t)(0u - align_k);
  s->align_k = align_k; s->unitigs_k = unitigs_k; s->ul = ul; s->n_ul = n_ul;
  s->error = 0;
  if (unitigs_k) {
    uint32_t id = ki_id(s, 0);
    if (id != INVALID_ID && id < n_ul) {
      s->size = 2 * n_ids - 1;
      memset(mers, 0, s->size * sizeof(int32_t));
      memset(bases, 0, s->size * sizeof(int32_t));
      s->cend = ul[id];
    } else {
      s->error = 1; /* vectors cleared; later add_mer writes are unobservable */
    }
  }
}

static void kinfo_add(kinfo_t* s, int32_t pos) {
  if (!s->unitigs_k || s->error) return;
  const int32_t k = (int32_t)s->align_k, uk = (int32_t)s->unitigs_k;
  const uint32_t nsz = s->n_ids;
  int32_t cendi;
  const int32_t sr_pos = abs(pos);
  const int32_t new_bases = k < sr_pos - s->prev_pos ? k : sr_pos - s->prev_pos;
  while (sr_pos + k > s->cend + 1) {
    if (s->cend >= sr_pos) {
      if ((size_t)s->cunitig >= (size_t)nsz - 1) goto error;
      int32_t mx = sr_pos > s->prev_pos + k ? sr_pos : s->prev_pos + k;
      const int32_t nb_bases = s->cend - mx + 1;
      s->bases[2 * s->cunitig] += nb_bases;
      s->bases[2 * s->cunitig + 1] += nb_bases;
    }
    uint32_t id = ki_id(s, ++s->cunitig);
    if (id == INVALID_ID || id >= s->n_ul) goto error;
    s->cend = (int32_t)((uint32_t)s->cend + (uint32_t)s->ul[id] - (uint32_t)uk + 1u);
  }
  ++s->mers[2 * s->cunitig];
  s->bases[2 * s->cunitig] += new_bases;
  cendi = s->cend;
  for (uint32_t i = s->cunitig;
       ((size_t)i < (size_t)nsz - 1) && ((uint32_t)sr_pos + (uint32_t)k > (uint32_t)cendi - (uint32_t)uk + 1u); ++i) {
    const int32_t full_mer = sr_pos + uk > cendi + 1;
    s->mers[2 * i + 1] += full_mer;
    s->mers[2 * i + 2] += full_mer;
    int32_t t = sr_pos + k - cendi + uk - 2;
    const int32_t nb_bases = new_bases < t ? new_bases : t;
    s->bases[2 * i + 1] += nb_bases;
    s->bases[2 * i + 2] += nb_bases;
    uint32_t id = ki_id(s, i + 1);
    if (id != INVALID_ID && id < s->n_ul)
      cendi = (int32_t)((uint32_t)cendi + (uint32_t)s->ul[id] - (uint32_t)uk + 1u);
    else
      goto error;
  }
  s->prev_pos = sr_pos;
  return;
error:
  s->error = 1;
  s->size = 0;
}

uint32_t oracle_kmers_info(const char* sr_name, const int32_t* ul, size_t n_ul, uint32_t unitigs_k, uint32_t align_k,
                           const int32_t* pos, size_t n_pos, int32_t* mers_out, int32_t* bases_out, uint32_t cap) {
  unitig_list u; unitigs_parse(sr_name, &u);
  uint32_t need = u.n ? 2 * u.n - 1 : 0;
  int32_t* m = xcalloc(need + 1, sizeof(int32_t));
  int32_t* b = xcalloc(need + 1, sizeof(int32_t));
  kinfo_t s; kinfo_init(&s, u.id, u.n, 0, unitigs_k, align_k, ul, n_ul, m, b);
  for (size_t i = 0; i < n_pos; ++i) kinfo_add(&s, pos[i]);
  uint32_t r = s.size;
  for (uint32_t i = 0; i < r && i < cap; ++i) { mers_out[i] = m[i]; bases_out[i] = b[i]; }
  free(m); free(b); free(u.id); free(u.ori);
  return r;
}

/* ======================================================================
 * compute_coords_info (pb_aligner.cc:11-82) + coords_info (hpp:103-175)
 * ==================================================================== */
typedef struct { int32_t* off; uint32_t n, cap; uint32_t* lis; uint32_t nlis, caplis; } offlist;

static void offlist_push(offlist* l, int32_t pb, int32_t sr) {
  if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 16; l->off = xrealloc(l->off, 2 * (size_t)l->cap * sizeof(int32_t)); }
  l->off[2 * l->n] = pb; l->off[2 * l->n + 1] = sr; ++l->n;
}

typedef struct {
  uint32_t k, unitigs_k; const int32_t* ul; size_t n_ul; int forward;
  int int_abs;  /* oracle_params.legacy_int_abs */
} cinfo_ctx;

static void rec_canonicalize(oracle_record* r, int forward, uint32_t k) {
  if (r->qs < 0) {
    if (forward) {
      r->qs = (int32_t)(uint32_t)(r->ql + (uint64_t)(int64_t)r->qs - (uint64_t)k + 2);
      r->qe = (int32_t)(uint32_t)(r->ql + (uint64_t)(int64_t)r->qe + 1);
      r->rn = 1;
      r->offset -= r->stretch * (double)(r->ql + 1) - (double)k;
    } else {
      r->qs = (int32_t)((uint32_t)(-r->qs) + k - 1u);
      r->qe = -r->qe;
      r->stretch = -r->stretch;
      r->offset += (double)(k - 1u);
    }
  } else {
    r->qe = (int32_t)((uint32_t)r->qe + k - 1u);
  }
}
static inline double imp_s(const oracle_record* r) {
  double v = r->stretch + r->offset; double m = (double)r->rl < v ? (double)r->rl : v; return 1.0 > m ? 1.0 : m;
}
static inline double imp_e(const oracle_record* r) {
  double v = r->stretch * (double)r->ql + r->offset; double m = (double)r->rl < v ? (double)r->rl : v; return 1.0 > m ? 1.0 : m;
}
static inline int32_t imp_len(const oracle_record* r) { long v = lrint(imp_e(r) - imp_s(r)); return (int32_t)(labs(v) + 1); }
static inline int min_bases(const oracle_record* r, double factor, uint32_t k) {
  return factor * (double)(imp_len(r) - 2 * (int32_t)k) <= (double)r->pb_cover;
}
static inline int min_mers(const oracle_record* r, double factor, uint32_t k) {
  return factor * (double)((uint32_t)imp_len(r) - k + 1u) <= (double)r->nb_mers;
}

/* The record's kmers_info vectors are malloc'd (n_info entries). */
static void compute_coords_info(const sr_rec* sr, uint32_t sr_index, const offlist* fwd, const offlist* bwd,
                                uint64_t pb_size, const cinfo_ctx* cx, oracle_record* r) {
  const uint32_t k = cx->k;
  const int fwd_align = fwd->nlis >= bwd->nlis;
  const uint32_t nb = fwd_align ? fwd->nlis : bwd->nlis;
  memset(r, 0, sizeof(*r));
  r->nb_mers = (int32_t)nb; r->pb_cover = k; r->sr_cover = k;
  r->rl = pb_size; r->ql = sr->len; r->sr_index = sr_index;
  r->use_bwd_name = (cx->forward && !fwd_align);
  if (nb == 0) return;
  const offlist* L = fwd_align ? fwd : bwd;
  const unitig_list* u = &sr->fwd;
  uint32_t nsz = u->n;
  int32_t* m = NULL; int32_t* b = NULL;
  kinfo_t ki;
  if (cx->unitigs_k) { m = xcalloc(2 * (size_t)nsz + 1, sizeof(int32_t)); b = xcalloc(2 * (size_t)nsz + 1, sizeof(int32_t)); }
  kinfo_init(&ki, u->id, nsz, r->use_bwd_name, cx->unitigs_k, k, cx->ul, cx->n_ul, m, b);
  lsq_t ls; memset(&ls, 0, sizeof(ls));
  const int32_t* pf = &L->off[2 * L->lis[0]];
  int32_t prev_pb = pf[0], prev_sr = pf[1];
  int32_t pos = fwd_align ? prev_sr : (int32_t)(uint32_t)(r->ql + (uint64_t)(int64_t)prev_sr - k + 2);
  kinfo_add(&ki, pos);
  lsq_add(&ls, (double)prev_sr, (double)prev_pb);
  for (uint32_t t = 1; t < L->nlis; ++t) {
    const int32_t* c = &L->off[2 * L->lis[t]];
    const uint32_t pb_diff = (uint32_t)(c[0] - prev_pb);
    r->pb_cons += pb_diff == 1;
    r->pb_cover += k < pb_diff ? k : pb_diff;
    const uint32_t sr_diff = (uint32_t)(c[1] - prev_sr);
    r->sr_cons += sr_diff == 1;
    r->sr_cover += k < sr_diff ? k : sr_diff;
    pos = fwd_align ? c[1] : (int32_t)(uint32_t)(r->ql + (uint64_t)(int64_t)c[1] - k + 2);
    kinfo_add(&ki, pos);
    lsq_add(&ls, (double)c[1], (double)c[0]);
    prev_pb = c[0]; prev_sr = c[1];
  }
  double e = 0;
  if (ls.n == 1) {
    r->stretch = 1.0;
    r->offset = ls.EY - ls.EX;
    r->avg_err = 0;
  } else if (ls.n > 1) {
    const double a = r->stretch = ls.CXY / ls.VX;
    const double bb = r->offset = ls.NB / ls.VX;
    for (uint32_t t = 0; t < L->nlis; ++t) {
      const int32_t* c = &L->off[2 * L->lis[t]];
      const double d = a * (double)c[1] + bb - (double)c[0];
      e += cx->int_abs ? (double)abs((int)d) : fabs(d);
    }
    r->avg_err = e / (double)ls.n;
  }
  const int32_t* first = &L->off[2 * L->lis[0]];
  const int32_t* last = &L->off[2 * L->lis[L->nlis - 1]];
  r->rs = first[0];
  r->re = (int32_t)((uint32_t)last[0] + k - 1u);
  r->qs = first[1];
  r->qe = last[1];
  rec_canonicalize(r, cx->forward, k);
  if (cx->unitigs_k && ki.size) { r->n_info = ki.size; r->kmers_info = m; r->bases_info = b; }
  else { free(m); free(b); r->n_info = 0; }
}

int oracle_coords_info(const char* sr_name, uint32_t sr_len,
                       const int32_t* fwd, uint32_t n_fwd, const uint32_t* fwd_lis, uint32_t n_fwd_lis,
                       const int32_t* bwd, uint32_t n_bwd, const uint32_t* bwd_lis, uint32_t n_bwd_lis,
                       uint64_t pb_size, uint32_t align_k, uint32_t unitigs_k,
                       const int32_t* ul, size_t n_ul, int forward, oracle_record* out) {
  oracle_index tmp; memset(&tmp, 0, sizeof(tmp));
  tmp.k = align_k;
  index_add_sr(&tmp, sr_name, 0, sr_len);
  offlist f = { (int32_t*)fwd, n_fwd, n_fwd, (uint32_t*)fwd_lis, n_fwd_lis, n_fwd_lis };
  offlist b = { (int32_t*)bwd, n_bwd, n_bwd, (uint32_t*)bwd_lis, n_bwd_lis, n_bwd_lis };
  cinfo_ctx cx = { align_k, unitigs_k, ul, n_ul, forward, 0 };
  compute_coords_info(&tmp.sr[0], 0, &f, &b, pb_size, &cx, out);
  free(tmp.sr[0].name_fwd); free(tmp.sr[0].name_bwd); free(tmp.sr[0].fwd.id); free(tmp.sr[0].fwd.ori); free(tmp.sr);
  return 0;
}

/* off_lis::discard_LIS (pb_aligner.hpp:47-61) */
static void discard_lis(offlist* l) {
  if (l->nlis == 0) return;
  uint32_t li = 0;
  uint32_t w = l->lis[li++];
  for (uint32_t r = w + 1; r < l->n; ++r) {
    if (li < l->nlis && r == l->lis[li]) ++li;
    else { l->off[2 * w] = l->off[2 * r]; l->off[2 * w + 1] = l->off[2 * r + 1]; ++w; }
  }
  l->n -= l->nlis;
}

static void do_lis(offlist* l, size_t W, const accept_t* ac, lis_scratch* sc) {
  if (l->caplis < l->n) { l->caplis = l->n; l->lis = xrealloc(l->lis, (size_t)l->caplis * sizeof(uint32_t)); }
  l->nlis = lis_run(l->off, l->n, W, ac, sc, l->lis);
}

/* growable text buffer (formatting of coords and details) */
typedef struct { char* s; size_t n, cap; } sbuf;
static void sb_reserve(sbuf* b, size_t extra) {
  if (b->n + extra + 1 > b->cap) { size_t nc = b->cap ? b->cap : 4096; while (nc < b->n + extra + 1) nc *= 2; b->s = xrealloc(b->s, nc); b->cap = nc; }
}
static void sb_printf(sbuf* b, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static void sb_printf(sbuf* b, const char* fmt, ...) {
  va_list ap;
  for (;;) {
    sb_reserve(b, 256);
    va_start(ap, fmt);
    int r = vsnprintf(b->s + b->n, b->cap - b->n, fmt, ap);
    va_end(ap);
    if (r < 0) DIE("vsnprintf");
    if ((size_t)r < b->cap - b->n) { b->n += (size_t)r; return; }
    sb_reserve(b, (size_t)r + 1);
  }
}

/* ======================================================================
 * Per-read aligner: fetch_super_reads (coarse_aligner.cc:81-141) +
 * align_sequence_max (coarse_aligner.cc:42-60).
 * ==================================================================== */
void oracle_params_default(oracle_params* p) {
  memset(p, 0, sizeof(*p));
  p->k = 17; p->psa_min = 13; p->stretch_constant = 10; p->stretch_factor = 1.3; p->stretch_cap = 10000;
  p->window_size = 1; p->max_count = 5000; p->bases_matching = 17.0; p->mers_matching = 0.0;
}

typedef struct { uint64_t lo_a, hi_a, lo_b, hi_b; uint64_t count; int canon; int32_t pb_off; } kinfo_entry;

typedef struct {
  int32_t* slot_of_sr;   /* n_sr, -1 = none */
  uint32_t* touched; uint32_t n_touched, cap_touched;
  offlist* fwd; offlist* bwd; uint32_t cap_lists;
  kinfo_entry* ent; size_t cap_ent;
  uint64_t* cnts; size_t cap_cnts;
  lis_scratch sc;
  size_t n_sr;
  /* fine (-F) windows: one per coarse record (fine_aligner.hpp:50-58) */
  struct fine_win* fw; uint32_t cap_fw;
  int32_t* fhead;        /* n_sr: first window of the super-read, -1 = none */
} worker_t;

typedef struct fine_win {
  uint32_t sr; int32_t next;  /* next window of the same super-read */
  double begin, end;          /* sr_local_ml (fine_aligner.hpp:12-17) */
  offlist fwd, bwd;
} fine_win;

static void worker_init(worker_t* w, size_t n_sr) {
  memset(w, 0, sizeof(*w));
  w->n_sr = n_sr;
  w->slot_of_sr = xmalloc((n_sr ? n_sr : 1) * sizeof(int32_t));
  w->fhead = xmalloc((n_sr ? n_sr : 1) * sizeof(int32_t));
  for (size_t i = 0; i < n_sr; ++i) { w->slot_of_sr[i] = -1; w->fhead[i] = -1; }
}
static void worker_free(worker_t* w) {
  for (uint32_t i = 0; i < w->cap_lists; ++i) { free(w->fwd[i].off); free(w->fwd[i].lis); free(w->bwd[i].off); free(w->bwd[i].lis); }
  free(w->fwd); free(w->bwd); free(w->touched); free(w->slot_of_sr); free(w->ent); free(w->cnts);
  for (uint32_t i = 0; i < w->cap_fw; ++i) { free(w->fw[i].fwd.off); free(w->fw[i].fwd.lis); free(w->fw[i].bwd.off); free(w->fw[i].bwd.lis); }
  free(w->fw); free(w->fhead);
  lis_scratch_free(&w->sc);
}

static uint32_t worker_slot(worker_t* w, uint32_t sr) {
  int32_t s = w->slot_of_sr[sr];
  if (s >= 0) return (uint32_t)s;
  if (w->n_touched == w->cap_lists) {
    uint32_t nc = w->cap_lists ? 2 * w->cap_lists : 64;
    w->fwd = xrealloc(w->fwd, nc * sizeof(offlist)); w->bwd = xrealloc(w->bwd, nc * sizeof(offlist));
    w->touched = xrealloc(w->touched, nc * sizeof(uint32_t));
    for (uint32_t i = w->cap_lists; i < nc; ++i) { memset(&w->fwd[i], 0, sizeof(offlist)); memset(&w->bwd[i], 0, sizeof(offlist)); }
    w->cap_lists = nc;
  }
  uint32_t slot = w->n_touched++;
  w->touched[slot] = sr;
  w->fwd[slot].n = 0; w->bwd[slot].n = 0; w->fwd[slot].nlis = 0; w->bwd[slot].nlis = 0;
  w->slot_of_sr[sr] = (int32_t)slot;
  return slot;
}

static int cmp_u64(const void* a, const void* b) {
  uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b; return x < y ? -1 : x > y;
}
static int cmp_rec(const void* a, const void* b) {
  const oracle_record* x = a; const oracle_record* y = b;
  if (x->rs != y->rs) return x->rs < y->rs ? -1 : 1;
  if (x->re != y->re) return x->re < y->re ? -1 : 1;
  if (x->ql != y->ql) return x->ql < y->ql ? -1 : 1;
  if (x->sr_index != y->sr_index) return x->sr_index < y->sr_index ? -1 : 1;
  return x->emit < y->emit ? -1 : x->emit > y->emit;
}

/* print_details (jf_aligner.cc:72-108) for one super-read of frags_pos, in
 * its final state: fwd and bwd lists merged by pb offset (fwd first on
 * ties), the elements of the longer lis (fwd only if strictly longer) in
 * brackets. */
static void details_line(sbuf* det, const char* pbname, size_t pbname_len, const char* srname,
                         const offlist* F, const offlist* B) {
  sb_printf(det, "%.*s %s", (int)pbname_len, pbname, srname);
  const int fa = F->nlis > B->nlis;
  const offlist* L = fa ? F : B;
  uint32_t li = 0, fi = 0, bi = 0;
  while (fi < F->n || bi < B->n) {
    int32_t pb, so; int in_lis;
    if (fi < F->n && (bi == B->n || F->off[2 * fi] <= B->off[2 * bi])) {
      pb = F->off[2 * fi]; so = F->off[2 * fi + 1];
      in_lis = fa && li < L->nlis && L->lis[li] == fi;
      ++fi;
    } else {
      pb = B->off[2 * bi]; so = B->off[2 * bi + 1];
      in_lis = !fa && li < L->nlis && L->lis[li] == bi;
      ++bi;
    }
    if (in_lis) { sb_printf(det, " [%d:%d]", pb, so); ++li; }
    else sb_printf(det, " %d:%d", pb, so);
  }
  sb_printf(det, "\n");
}

/* fine_aligner::thread::align_sequence (fine_aligner.cc:38-51): one window
 * per coarse record (prime_frags_pos, fine_aligner.hpp:50-58), every
 * fine_k-mer of the read looked up (no SSR / toggle / count filters) and its
 * hits kept in each window of the super-read whose [begin, end] holds the pb
 * offset (fetch_local_super_reads, fine_aligner.cc:7-36), LIS with
 * accept_all and window 1, compute_coords_info(forward = true) with
 * align_k = fine_k and no filters.  Replaces coarse[0..nc) by the fine
 * records (malloc'd, *nf).  A window without hits gives nb_mers = 0, whose
 * rs/re/qs/qe the reference leaves uninitialized (pb_aligner.cc:27 returns
 * before setting them): they are 0 here. */
static oracle_record* fine_align_read(const oracle_index* ix, const oracle_params* p, worker_t* w,
                                      const char* seq, size_t len, const oracle_record* coarse, size_t nc,
                                      size_t* nf) {
  const uint32_t fk = ix->fk;
  if (w->cap_fw < nc) {
    w->fw = xrealloc(w->fw, nc * sizeof(fine_win));
    for (uint32_t i = w->cap_fw; i < nc; ++i) memset(&w->fw[i], 0, sizeof(fine_win));
    w->cap_fw = (uint32_t)nc;
  }
  for (size_t i = nc; i-- > 0;) {  /* window lists per super-read, in coarse order */
    const oracle_record* c = &coarse[i];
    fine_win* fw = &w->fw[i];
    fw->sr = c->sr_index;
    const double b = c->stretch + c->offset - c->avg_err;
    const double e = c->stretch * (double)c->ql + c->offset + c->avg_err - (double)fk;
    fw->begin = 0.0 < b ? b : 0.0;                       /* std::max((double)0, b) */
    fw->end = e < (double)c->rl ? e : (double)c->rl;     /* std::min((double)rl, e) */
    fw->fwd.n = fw->bwd.n = 0; fw->fwd.nlis = fw->bwd.nlis = 0;
    fw->next = w->fhead[fw->sr];
    w->fhead[fw->sr] = (int32_t)i;
  }
  const uint64_t mask = mer_mask(fk);
  uint64_t m = 0, rm = 0; uint32_t rlen = 0;
  for (size_t i = 0; i < len; ++i) {
    const int c = jf_code((unsigned char)seq[i]);
    if (c < 0) { rlen = 0; continue; }
    ++rlen;
    m = ((m << 2) | (uint64_t)c) & mask;
    rm = (rm >> 2) | ((uint64_t)(3 - c) << (2 * (fk - 1)));
    if (rlen < fk) continue;
    const int canon = m < rm;
    const int32_t pb_off = (int32_t)(i + 1) - (int32_t)fk + 1;
    for (int half = 0; half < 2; ++half) {
      uint64_t lo, hi;
      fine_range(ix, half ? (canon ? rm : m) : (canon ? m : rm), &lo, &hi);
      for (uint64_t q = lo; q < hi; ++q) {
        const uint64_t x = ix->fpos[q];
        const size_t s = sr_of(ix, x);
        if (w->fhead[s] < 0) continue;
        if (x + fk > ix->sr[s].start + ix->sr[s].len) continue;
        const int32_t off = (int32_t)(x - ix->sr[s].start + 1);
        const int32_t it_off = half ? -off : off;
        const int32_t fin = canon ? it_off : -it_off;
        for (int32_t wi = w->fhead[s]; wi >= 0; wi = w->fw[wi].next) {
          fine_win* fw = &w->fw[wi];
          if ((double)pb_off >= fw->begin && (double)pb_off <= fw->end)
            offlist_push(fin > 0 ? &fw->fwd : &fw->bwd, pb_off, fin);
        }
      }
    }
  }
  accept_t all = { 1, 0, 0, 0, 1, 0 };
  cinfo_ctx cx = { fk, p->unitigs_k, p->unitig_lengths, p->n_unitigs, 1, p->legacy_int_abs };
  oracle_record* recs = xmalloc((nc ? nc : 1) * sizeof(oracle_record));
  for (size_t i = 0; i < nc; ++i) {
    fine_win* fw = &w->fw[i];
    do_lis(&fw->fwd, 1, &all, &w->sc);
    do_lis(&fw->bwd, 1, &all, &w->sc);
    compute_coords_info(&ix->sr[fw->sr], fw->sr, &fw->fwd, &fw->bwd, (uint64_t)len, &cx, &recs[i]);
    recs[i].emit = (uint32_t)i;
    w->fhead[fw->sr] = -1;
  }
  *nf = nc;
  return recs;
}

static int align_read_w(const oracle_index* ix, const oracle_params* p, worker_t* w,
                        const char* seq, size_t len, oracle_read_result* out,
                        sbuf* det, const char* pbname, size_t pbname_len) {
  const uint32_t k = ix->k;
  const uint64_t mask = mer_mask(k);
  const int32_t max_count = p->max_count ? p->max_count : INT_MAX;
  size_t n_ent = 0;
  /* --- fetch_super_reads: k-mer loop --- */
  uint64_t m = 0, rm = 0; uint32_t rlen = 0; uint32_t flag = 1;
  for (size_t i = 0; i < len; ++i) {
    int c = jf_code((unsigned char)seq[i]);
    if (c < 0) { rlen = 0; continue; }
    ++rlen;
    m = ((m << 2) | (uint64_t)c) & mask;
    rm = (rm >> 2) | ((uint64_t)(3 - c) << (2 * (k - 1)));
    if (rlen < k) continue;
    if (!p->legacy_no_filter) {
      if (oracle_is_ssr(m, k)) continue;
      if (rlen <= 17) { flag = 1 - flag; if (flag == 1) continue; }
    }
    const int canon = m < rm;
    const uint64_t a = canon ? m : rm, b = canon ? rm : m;
    kinfo_entry e;
    index_range(ix, a, &e.lo_a, &e.hi_a);
    index_range(ix, b, &e.lo_b, &e.hi_b);
    e.count = (e.hi_a - e.lo_a) + (e.hi_b - e.lo_b);
    if (e.count == 0) continue;
    if (!p->legacy_no_filter && max_count && e.count >= (uint64_t)max_count) continue;
    e.canon = canon;
    e.pb_off = (int32_t)(i + 1) - (int32_t)k + 1; /* parser.offset<0>() */
    if (n_ent == w->cap_ent) { w->cap_ent = w->cap_ent ? 2 * w->cap_ent : 1024; w->ent = xrealloc(w->ent, w->cap_ent * sizeof(kinfo_entry)); }
    w->ent[n_ent++] = e;
  }
  /* --- 99% count threshold (coarse_aligner.cc:117-125) --- */
  uint64_t threshold;
  if (p->legacy_no_filter) threshold = UINT64_MAX;
  else {
    const uint32_t sum_thresh = (uint32_t)round((double)n_ent * 0.99);
    if (n_ent > sum_thresh) {
      if (w->cap_cnts < n_ent) { w->cap_cnts = n_ent; w->cnts = xrealloc(w->cnts, n_ent * sizeof(uint64_t)); }
      for (size_t i = 0; i < n_ent; ++i) w->cnts[i] = w->ent[i].count;
      qsort(w->cnts, n_ent, sizeof(uint64_t), cmp_u64);
      threshold = w->cnts[sum_thresh];
    } else {
      threshold = (uint32_t)((uint32_t)max_count + 1u);
    }
  }
  /* --- expansion into per-SR fwd/bwd lists --- */
  w->n_touched = 0;
  for (size_t t = 0; t < n_ent; ++t) {
    const kinfo_entry* e = &w->ent[t];
    if (e->count > threshold) continue;
    for (int half = 0; half < 2; ++half) {
      uint64_t lo = half ? e->lo_b : e->lo_a, hi = half ? e->hi_b : e->hi_a;
      for (uint64_t q = lo; q < hi; ++q) {
        const uint64_t x = ix->pos[q];
        const size_t s = sr_of(ix, x);
        if (x + k > ix->sr[s].start + ix->sr[s].len) continue; /* crosses the SR end */
        const int32_t off = (int32_t)(x - ix->sr[s].start + 1);
        const int32_t it_off = half ? -off : off;
        const int32_t fin = e->canon ? it_off : -it_off;
        const uint32_t slot = worker_slot(w, (uint32_t)s);
        if (fin > 0) offlist_push(&w->fwd[slot], e->pb_off, fin);
        else offlist_push(&w->bwd[slot], e->pb_off, fin);
      }
    }
  }
  /* --- chaining + coords (align_sequence_max) --- */
  accept_t ac = { 0, p->stretch_factor, p->stretch_constant, p->stretch_cap, 0, p->stretch_factor };
  cinfo_ctx cx = { k, p->unitigs_k, p->unitig_lengths, p->n_unitigs, p->forward, p->legacy_int_abs };
  const double Mf = p->mers_matching / 100.0, Bf = p->bases_matching / 100.0;
  size_t nrec = 0, caprec = 0; oracle_record* recs = NULL;
  for (uint32_t slot = 0; slot < w->n_touched; ++slot) {
    const uint32_t sr = w->touched[slot];
    offlist* F = &w->fwd[slot]; offlist* B = &w->bwd[slot];
    do_lis(F, p->window_size, &ac, &w->sc);
    do_lis(B, p->window_size, &ac, &w->sc);
    uint32_t emit = 0;
    for (;;) {
      oracle_record r;
      compute_coords_info(&ix->sr[sr], sr, F, B, (uint64_t)len, &cx, &r);
      int keep = 1;
      if (r.nb_mers == 0) keep = 0;
      else if (fabs(r.stretch) == 0.0) keep = 0;
      else if (Mf != 0.0 && !min_mers(&r, Mf, k)) keep = 0;
      else if (Bf > 0.0 && !min_bases(&r, Bf, k)) keep = 0;
      if (!keep) { free(r.kmers_info); free(r.bases_info); break; }
      r.emit = emit++;
      if (nrec == caprec) { caprec = caprec ? 2 * caprec : 16; recs = xrealloc(recs, caprec * sizeof(oracle_record)); }
      recs[nrec++] = r;
      if (!p->max_match) break;
      offlist* D = F->nlis > B->nlis ? F : B; /* mer_lists::discard_update_LIS */
      discard_lis(D);
      do_lis(D, p->window_size, &ac, &w->sc);
    }
    if (det) details_line(det, pbname, pbname_len, ix->sr[sr].name_fwd, F, B);
    w->slot_of_sr[sr] = -1;
  }
  if (p->fine_k) {
    size_t nf = 0;
    oracle_record* fr = fine_align_read(ix, p, w, seq, len, recs, nrec, &nf);
    for (size_t i = 0; i < nrec; ++i) { free(recs[i].kmers_info); free(recs[i].bases_info); }
    free(recs);
    recs = fr; nrec = nf;
  }
  qsort(recs, nrec, sizeof(oracle_record), cmp_rec);
  out->n = nrec; out->recs = recs;
  return 0;
}

int oracle_align_read(const oracle_index* ix, const oracle_params* p, const char* seq, size_t len, oracle_read_result* out) {
  if (p->k != ix->k) DIE("params.k != index k");
  if (p->fine_k && p->fine_k != ix->fk) DIE("params.fine_k != the index's fine sub-index");
  worker_t w; worker_init(&w, ix->n_sr);
  int r = align_read_w(ix, p, &w, seq, len, out, NULL, NULL, 0);
  worker_free(&w);
  return r;
}

void oracle_read_result_free(oracle_read_result* r) {
  for (size_t i = 0; i < r->n; ++i) { free(r->recs[i].kmers_info); free(r->recs[i].bases_info); }
  free(r->recs); r->recs = NULL; r->n = 0;
}

/* ======================================================================
 * Formatting (jf_aligner.cc:32-70) and the threaded driver.
 * ==================================================================== */
static void format_read(sbuf* b, const oracle_index* ix, const char* header, uint64_t pb_size,
                        const oracle_read_result* r, int compact, int zero_match) {
  if (r->n == 0 && !zero_match) return;
  /* name = header up to the first whitespace (jf_aligner.cc:133-134) */
  size_t nl = strcspn(header, " \t\n\v\f\r");
  if (compact) sb_printf(b, ">%zu %.*s\n", r->n, (int)nl, header);
  for (size_t i = 0; i < r->n; ++i) {
    const oracle_record* c = &r->recs[i];
    if (!compact) sb_printf(b, "%.*s ", (int)nl, header);
    /* std::ostream << double == printf("%.6g") (libstdc++ num_put) */
    sb_printf(b, "%d %d %d %d %d %u %u %u %u %llu %llu %.6g %.6g %.6g %s",
              c->rs, c->re, c->qs, c->qe, c->nb_mers, c->pb_cons, c->sr_cons, c->pb_cover, c->sr_cover,
              (unsigned long long)pb_size, (unsigned long long)c->ql, c->stretch, c->offset, c->avg_err,
              c->use_bwd_name ? ix->sr[c->sr_index].name_bwd : ix->sr[c->sr_index].name_fwd);
    for (uint32_t t = 0; t < c->n_info; ++t) sb_printf(b, " %d:%d", c->kmers_info[t], c->bases_info[t]);
    sb_printf(b, "\n");
  }
}

typedef struct {
  const oracle_index* ix; const oracle_params* p;
  const char* const* names; const char* const* seqs; const uint64_t* lens; size_t n;
  int compact, zero_match, do_format;
  sbuf* outs; sbuf* dets; atomic_size_t next; atomic_ullong nrec;
} drv_t;

static void* drv_worker(void* arg) {
  drv_t* d = arg;
  worker_t w; worker_init(&w, d->ix->n_sr);
  for (;;) {
    size_t i = atomic_fetch_add(&d->next, 1);
    if (i >= d->n) break;
    oracle_read_result r;
    sbuf* det = d->dets ? &d->dets[i] : NULL;
    const char* nm = d->names ? d->names[i] : "";
    align_read_w(d->ix, d->p, &w, d->seqs[i], d->lens[i], &r, det, nm, strcspn(nm, " \t\n\v\f\r"));
    atomic_fetch_add(&d->nrec, r.n);
    if (d->do_format) format_read(&d->outs[i], d->ix, d->names[i], d->lens[i], &r, d->compact, d->zero_match);
    oracle_read_result_free(&r);
  }
  worker_free(&w);
  return NULL;
}

static void run_driver(drv_t* d, int threads) {
  if (threads < 1) threads = 1;
  pthread_t* th = xcalloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, drv_worker, d);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
}

static char* join_parts(sbuf* parts, size_t n, const char* head, size_t* out_len) {
  sbuf all = { 0, 0, 0 };
  if (head) sb_printf(&all, "%s", head);
  for (size_t i = 0; i < n; ++i) {
    if (parts[i].n) { sb_reserve(&all, parts[i].n); memcpy(all.s + all.n, parts[i].s, parts[i].n); all.n += parts[i].n; }
    free(parts[i].s);
  }
  free(parts);
  sb_reserve(&all, 0);
  all.s[all.n] = 0;
  *out_len = all.n;
  return all.s;
}

char* oracle_align_format(const oracle_index* ix, const oracle_params* p, const char* const* names,
                          const char* const* seqs, const uint64_t* lens, size_t n, int threads,
                          int compact, int header, int zero_match, size_t* out_len) {
  return oracle_align_format_ex(ix, p, names, seqs, lens, n, threads, compact, header, zero_match, out_len, NULL, NULL);
}

char* oracle_align_format_ex(const oracle_index* ix, const oracle_params* p, const char* const* names,
                             const char* const* seqs, const uint64_t* lens, size_t n, int threads,
                             int compact, int header, int zero_match, size_t* out_len,
                             char** details, size_t* details_len) {
  if (p->k != ix->k) DIE("params.k != index k");
  if (p->fine_k && p->fine_k != ix->fk) DIE("params.fine_k != the index's fine sub-index");
  drv_t d; memset(&d, 0, sizeof(d));
  d.ix = ix; d.p = p; d.names = names; d.seqs = seqs; d.lens = lens; d.n = n;
  d.compact = compact; d.zero_match = zero_match; d.do_format = 1;
  d.outs = xcalloc(n ? n : 1, sizeof(sbuf));
  if (details) d.dets = xcalloc(n ? n : 1, sizeof(sbuf));
  atomic_init(&d.next, 0); atomic_init(&d.nrec, 0);
  run_driver(&d, threads);
  char head[160];
  snprintf(head, sizeof head, "Rstart Rend Qstart Qend Nmers Rcons Qcons Rcover Qcover Rlen Qlen Stretch Offset Err%s Qname\n",
           compact ? "" : " Rname");
  if (details) *details = join_parts(d.dets, n, NULL, details_len);
  return join_parts(d.outs, n, header ? head : NULL, out_len);
}

double oracle_align_timed(const oracle_index* ix, const oracle_params* p, const char* const* seqs,
                          const uint64_t* lens, size_t n, int threads, uint64_t* n_records) {
  if (p->fine_k && p->fine_k != ix->fk) DIE("params.fine_k != the index's fine sub-index");
  drv_t d; memset(&d, 0, sizeof(d));
  d.ix = ix; d.p = p; d.seqs = seqs; d.lens = lens; d.n = n;
  atomic_init(&d.next, 0); atomic_init(&d.nrec, 0);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  run_driver(&d, threads);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (n_records) *n_records = atomic_load(&d.nrec);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
