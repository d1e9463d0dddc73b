/*
 * pb_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C11) of the reference jf_aligner coarse path
 * (alekseyzimin/PacBio, src_jf_aligner + src_lis + src_psa), used as the
 * parity oracle for the MI355X path and as the "port" CPU baseline in
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library.  The product path
 * (pacbio_amd/, libpbgpu.so) never links, loads or calls it.
 *
 * Parity pins (see DESIGN.md "Oracle"):
 *   - LIS (lis_align::compute_L_P), least_square_2d, PSA search order and
 *     compact_dna encoding, super_read_name parse/reverse are pinned by
 *     executing the reference's own sources (oracle/_ref, built by
 *     oracle/Makefile from /root/reference) on seeded inputs; the vectors
 *     are committed under tests/golden/.
 *   - compute_kmers_info, compute_coords_info are pinned by the known-answer
 *     vectors of tests/test_kmers_info.cc and tests/test_compute_coords_info.cc.
 *   - fetch_super_reads / coarse_aligner / print_coords cannot be executed
 *     (they need the un-vendored Jellyfish 2.x and yaggo); they are restated
 *     from source and pinned semantically by tests/test_pb_aligner.cc and
 *     tests/aligner_output (see DESIGN.md for what that leaves unpinned).
 *
 * Third-party semantics restated here (absent from /root/reference):
 *   Jellyfish 2.x `mer_dna` (configure.ac:17, `jellyfish-2.0`, version not
 *   pinned beyond the 2.0 API): 2-bit code A0 C1 G2 T3 (case-insensitive),
 *   every other byte is "not DNA"; k <= 32 mers live in one uint64 with the
 *   FIRST base in the most significant bits; shift_left(c) appends at the low
 *   end; shift_right(c) inserts at the high end; base(0) is the LAST base;
 *   operator< is the integer compare of that code.
 */
#ifndef PB_ORACLE_H
#define PB_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- params */
typedef struct {
  uint32_t k;                 /* -m, mer size (<= 32) */
  uint32_t psa_min;           /* --psa-min (only affects k <= psa_min order) */
  double   stretch_constant;  /* --stretch-constant (b of affine_capped) */
  double   stretch_factor;    /* --stretch-factor (a) */
  double   stretch_cap;       /* --stretch-cap (C) */
  uint32_t window_size;       /* --window-size */
  int      forward;           /* -f (also implied by -l/-u) */
  int      max_match;         /* --max-match */
  int32_t  max_count;         /* --max-count (0 => INT_MAX, jf_aligner.cc:213) */
  double   mers_matching;     /* -M (percent) */
  double   bases_matching;    /* -B (percent) */
  uint32_t unitigs_k;         /* -k (0 = no k-unitig accounting) */
  const int32_t* unitig_lengths; /* -l table (index = line number) */
  size_t   n_unitigs;
  /* test-only knob: 1 => skip SSR / toggle / count threshold (the
   * semantics tests/test_pb_aligner.cc:68 was written against) */
  int      legacy_no_filter;
  /* test-only knob: 1 => the average error sums int abs() of each point's
   * residual (truncated to int, as `abs` on a double resolved to the C int
   * abs in the older aligner that wrote tests/mega_reads_output/expect_coords;
   * least_square_2d.hpp:82-90 keeps that loop, commented out) */
  int      legacy_int_abs;
  /* -F: fine_aligner k (0 = off).  The index must carry the fine sub-index
   * (oracle_index_build_fine) for this k. */
  uint32_t fine_k;
} oracle_params;

void oracle_params_default(oracle_params* p);

/* ---------------------------------------------------------------- index */
typedef struct oracle_index oracle_index;

/* Build from FASTA files (superread_parser.cc:12-46 semantics: multi-line,
 * full header line kept, empty records dropped, per-line compact_dna
 * encoding). */
oracle_index* oracle_index_build_fasta(const char* const* paths, size_t n_paths,
                                       uint32_t k, int threads);
/* Build from in-memory records: each sequence is ONE line. */
oracle_index* oracle_index_build_mem(const char* const* names,
                                     const char* const* seqs,
                                     const uint64_t* lens, size_t n,
                                     uint32_t k, int threads);
void     oracle_index_free(oracle_index* ix);
size_t   oracle_index_nb_sr(const oracle_index* ix);
uint64_t oracle_index_text_len(const oracle_index* ix);
uint32_t oracle_index_sr_len(const oracle_index* ix, size_t i);
const char* oracle_index_sr_name(const oracle_index* ix, size_t i, int bwd);
/* Text base code at global position (0..3). */
int      oracle_index_base(const oracle_index* ix, uint64_t pos);

/* Exact-match lookup of an MSB-first k-mer code: returns the total count
 * (including SR-boundary-crossing occurrences) and writes up to `cap`
 * positions in reference order (descending text position). */
uint64_t oracle_index_lookup(const oracle_index* ix, uint64_t code,
                             uint64_t* pos_out, uint64_t cap);

/* Fine (-F) sub-index over the short mer size fine_k <= k: every position in
 * SA order for a fine_k-mer pattern (sort_one_mer, mer_sa_imp.hpp:351-364).
 * Returns 0, or -1 if fine_k is outside [1, k] or k > 31. */
int      oracle_index_build_fine(oracle_index* ix, uint32_t fine_k, int threads);
/* Exact-match lookup of a fine_k-mer code in the fine sub-index: total count
 * and up to `cap` positions in the reference's SA order. */
uint64_t oracle_index_lookup_fine(const oracle_index* ix, uint64_t code,
                                  uint64_t* pos_out, uint64_t cap);

/* ---------------------------------------------------------------- records */
typedef struct {
  int32_t  rs, re, qs, qe, nb_mers;
  uint32_t pb_cons, sr_cons, pb_cover, sr_cover;
  uint64_t rl, ql;
  int32_t  rn;
  uint32_t sr_index;
  int32_t  use_bwd_name;
  double   stretch, offset, avg_err;
  uint32_t n_info;            /* length of kmers_info / bases_info */
  int32_t* kmers_info;
  int32_t* bases_info;
  uint32_t emit;              /* emission index within (read, SR) */
} oracle_record;

typedef struct {
  size_t         n;
  oracle_record* recs;        /* sorted by (rs, re, ql, sr_index, emit) */
} oracle_read_result;

/* Align one read (coarse_aligner::align_sequence_max). */
int  oracle_align_read(const oracle_index* ix, const oracle_params* p,
                       const char* seq, size_t len, oracle_read_result* out);
void oracle_read_result_free(oracle_read_result* r);

/* Align n reads with `threads` workers and format the coords text exactly
 * as jf_aligner print_coords does (jf_aligner.cc:32-70), reads in input
 * order. Returns malloc'd text (caller frees) and its size. */
char* oracle_align_format(const oracle_index* ix, const oracle_params* p,
                          const char* const* names, const char* const* seqs,
                          const uint64_t* lens, size_t n, int threads,
                          int compact, int header, int zero_match,
                          size_t* out_len);

/* oracle_align_format, and with details != NULL also the --details text
 * (print_details, jf_aligner.cc:72-108): per read, one line per super-read
 * of the coarse frags_pos in first-hit order (the reference iterates an
 * unordered_map).  Caller frees both texts. */
char* oracle_align_format_ex(const oracle_index* ix, const oracle_params* p,
                             const char* const* names, const char* const* seqs,
                             const uint64_t* lens, size_t n, int threads,
                             int compact, int header, int zero_match,
                             size_t* out_len, char** details, size_t* details_len);

/* Timing helper for the CPU baseline: aligns n reads with `threads`
 * workers, returns wall seconds (records discarded). */
double oracle_align_timed(const oracle_index* ix, const oracle_params* p,
                          const char* const* seqs, const uint64_t* lens,
                          size_t n, int threads, uint64_t* n_records);

/* ---------------------------------------------------------------- pieces */
/* lis_align::indices (lis_align.hpp:139-214). X is N (first, second) int
 * pairs. mer_kind/seq_kind: 0 = affine_capped(a,b,C) / linear(a),
 * 1 = accept_all. Returns the LIS length, writes indices to out. */
uint32_t oracle_lis(const int32_t* X, uint32_t N, uint32_t window,
                    int mer_kind, double a, double b, double C,
                    int seq_kind, double seq_a, uint32_t* out);

/* least_square_2d (least_square_2d.hpp:37-80): out = EX,EY,EXX,EXY,VX,CXY,NB,a,b */
void oracle_lsq(const double* x, const double* y, size_t n, double out[9]);

/* compute_kmers_info (pb_aligner.cc:84-143): feed positions, returns the
 * final vectors (n_out = 0 when the error path cleared them). */
uint32_t oracle_kmers_info(const char* sr_name, const int32_t* ul, size_t n_ul,
                           uint32_t unitigs_k, uint32_t align_k,
                           const int32_t* pos, size_t n_pos,
                           int32_t* mers_out, int32_t* bases_out, uint32_t cap);

/* compute_coords_info (pb_aligner.cc:11-82) on explicit lists. */
int oracle_coords_info(const char* sr_name, uint32_t sr_len,
                       const int32_t* fwd, uint32_t n_fwd, const uint32_t* fwd_lis, uint32_t n_fwd_lis,
                       const int32_t* bwd, uint32_t n_bwd, const uint32_t* bwd_lis, uint32_t n_bwd_lis,
                       uint64_t pb_size, uint32_t align_k, uint32_t unitigs_k,
                       const int32_t* ul, size_t n_ul, int forward,
                       oracle_record* out);

/* super_read_name parse (super_read_name.cc:74-90) + reverse name. */
int oracle_sr_name_reverse(const char* name, char* out, size_t cap);

/* compact_dna encoding of one line (compact_dna.hpp:89-136) assuming a
 * 16-byte aligned line buffer: returns 2-bit codes per base. */
void oracle_encode_line(const char* line, size_t len, uint8_t* codes);

/* is_ssr (coarse_aligner.cc:8-15) */
int oracle_is_ssr(uint64_t m, uint32_t k);

#ifdef __cplusplus
}
#endif
#endif
