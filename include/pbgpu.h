/*
 * pbgpu.h -- C ABI of the MI355X-native jf_aligner hot path.
 *
 * This is the drop-in boundary for the reference's C++ class API on the
 * L4 -> L3 line: the CLIs (jf_aligner, create_mega_reads)
 * call it instead of
 *   superread_parse(first, last, min, max)        superread_parser.hpp:219-224
 *   coarse_aligner(psa, k, factor, constant, cap,  coarse_aligner.hpp:55-72
 *                  window, forward, max_match, max_count, M, B)
 *   coarse_aligner::unitigs_lengths(ul, k)         coarse_aligner.hpp:76-81
 *   coarse_aligner::thread::align_sequence_max()   coarse_aligner.cc:68-72
 *   coarse_aligner::thread::coords()               coarse_aligner.hpp:146
 *   print_coords_header / print_coords             jf_aligner.cc:32-70
 * Differences by design: reads are aligned in batches (one call per batch,
 * not per read); records carry an SR index instead of frag_info pointers;
 * records of a read come back already sorted by (rs, re, ql) with the
 * deterministic tie-break (sr_index, emission order).
 *
 * Plain pointers and sizes only; no exceptions cross this boundary.  Every
 * function returns a pbgpu_status; pbgpu_last_error() returns a thread-local
 * message for the last failure on the calling thread.
 * Thread-safety: distinct aligners may be used concurrently; one aligner is
 * single-threaded (like coarse_aligner::thread).  The index is read-only
 * after build and may be shared by aligners on the same device.
 */
#ifndef PBGPU_H
#define PBGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBGPU_ABI_VERSION 8

typedef enum pbgpu_status {
  PBGPU_OK = 0,
  PBGPU_ERR_INVALID = 1,      /* bad argument (std::logic_error / yaggo error() upstream) */
  PBGPU_ERR_IO = 2,           /* cannot open / parse input (std::runtime_error upstream) */
  PBGPU_ERR_NOMEM = 3,        /* device or host allocation failed */
  PBGPU_ERR_DEVICE = 4,       /* HIP runtime error, or no usable GPU */
  PBGPU_ERR_UNSUPPORTED = 5,  /* configuration outside the implemented envelope */
  PBGPU_ERR_INTERNAL = 6
} pbgpu_status;

typedef struct pbgpu_index pbgpu_index;
typedef struct pbgpu_aligner pbgpu_aligner;
typedef struct pbgpu_reads pbgpu_reads;

int         pbgpu_abi_version(void);
const char* pbgpu_last_error(void);
/* number of visible GPUs (0 if none); never fails */
int         pbgpu_device_count(void);
/* hipDeviceSynchronize on `device` (bench brackets its timed region with it) */
pbgpu_status pbgpu_device_synchronize(int device);
/* Measurement aid (no reference counterpart): bandwidth of uniformly random
 * 64-byte sector loads over a fresh device buffer of buffer_bytes, all CUs
 * (SURVEY 8(d) B_rand, the random-access roofline).  Frees the buffer. */
pbgpu_status pbgpu_measure_gather(int device, uint64_t buffer_bytes, double* gbps);
/* The same for another access shape: unit_bytes 64 (random 64-B sectors, as
 * pbgpu_measure_gather) or 512 (random 512-B runs read as 64 consecutive 8-B
 * words, the shape of k_group's occurrence-list reads). */
pbgpu_status pbgpu_measure_gather_shape(int device, uint64_t buffer_bytes, uint32_t unit_bytes, double* gbps);
/* Measurement aid: k_group's occurrence-read shape (runs of 52 consecutive 8-B words at
 * random 8-B-aligned starts): mode 0 reads the 4-B id half of each word (pass 0), mode 1
 * the 8-B words (pass 1), mode 2 both passes over the same runs, as k_group does.  Per
 * launch: the 64-B sectors and 128-B lines the runs span and the algorithmic bytes, the
 * known counts to read FETCH_SIZE against; *gbps = sector bytes per second. */
pbgpu_status pbgpu_measure_group_shape(int device, uint64_t buffer_bytes, int mode, double* gbps, uint64_t* sectors64,
                                       uint64_t* lines128, uint64_t* alg_bytes);
/* Self-check of the fit's reciprocal (least_square_2d.hpp:47-67 divides by the
 * point count n): the device's shortened RN(1/n) against a correctly rounded
 * division for every n in [1, n_max]; *mismatches = the count that differ
 * (0 expected). */
pbgpu_status pbgpu_check_reciprocal(int device, uint32_t n_max, uint64_t* mismatches);

/* ------------------------------------------------------------------ index
 * Replaces superread_parse() + sequence_psa (superread_parser.hpp:53-224):
 * the super-read text is 2-bit packed with the reference's compact_dna line
 * rules, and a canonical k-mer hash index (counts incl. SR-boundary-crossing
 * occurrences, non-crossing occurrence lists in descending text position) is
 * built on and kept resident in device memory. */
typedef struct {
  uint32_t k;        /* -m, mer size: 2 <= k <= 31 */
  uint32_t psa_min;  /* --psa-min; must be < k (k <= psa_min gives a
                        thread-order-dependent hit order upstream) */
  int32_t  device;   /* HIP device ordinal */
  int32_t  threads;  /* host threads for FASTA parsing (0 = all cores) */
  uint32_t fine_k;   /* -F: also build the short-mer sub-index for the fine
                        aligner (jf_aligner.cc:200-203), 1 <= fine_k <= k;
                        0 = none.  Its occurrence lists follow the PSA order
                        of a pattern shorter than max_size = k: the k - fine_k
                        bases after each occurrence, then position descending
                        (mer_sa_imp.hpp:351-364). */
  uint32_t shard;    /* n_shards > 1: build shard `shard` of an index sharded by */
  uint32_t n_shards; /* super-read range; 0 or 1 = the whole set.  See
                        "Sharded index" below. */
} pbgpu_index_params;

/* superread_parser.cc:12-46: multi-line FASTA, full header line kept as the
 * name, empty records dropped.  PBGPU_ERR_IO for a missing file or a file
 * that does not start with '>' ("Not in fasta format"). */
pbgpu_status pbgpu_index_build_fasta(const char* const* paths, size_t n_paths,
                                     const pbgpu_index_params* params, pbgpu_index** out);
/* In-memory super-reads, each sequence treated as one FASTA line. */
pbgpu_status pbgpu_index_build(const char* const* names, const char* const* seqs,
                               const uint64_t* lens, size_t n,
                               const pbgpu_index_params* params, pbgpu_index** out);
pbgpu_status pbgpu_index_free(pbgpu_index* ix);

typedef struct {
  uint64_t n_sr;            /* super-reads kept */
  uint64_t text_len;        /* concatenated bases */
  uint64_t n_kmers;         /* canonical k-mers (distinct) */
  uint64_t n_occurrences;   /* non-crossing occurrences stored */
  uint64_t table_buckets;   /* 64-byte hash buckets */
  uint64_t device_bytes;    /* resident index footprint */
  double   build_seconds;
  uint64_t sr_begin, sr_end; /* super-reads held on the device (all of them unless sharded) */
  uint64_t filter_bytes;    /* k_seed's presence filter (0 = none) */
} pbgpu_index_info;
pbgpu_status pbgpu_index_get_info(const pbgpu_index* ix, pbgpu_index_info* info);
/* frag_info.hpp:18-35: fwd name = header line, bwd name = reversed unitigs */
const char*  pbgpu_index_sr_name(const pbgpu_index* ix, uint32_t sr, int bwd);
uint32_t     pbgpu_index_sr_len(const pbgpu_index* ix, uint32_t sr);

/* ---------------------------------------------------------------- aligner
 * coarse_aligner ctor (coarse_aligner.hpp:55-72) + unitigs_lengths(). */
typedef struct {
  uint32_t k;                 /* must equal the index k */
  double   stretch_factor;    /* --stretch-factor (1.3) */
  double   stretch_constant;  /* --stretch-constant (10) */
  double   stretch_cap;       /* --stretch-cap (10000) */
  uint32_t window_size;       /* --window-size (1) */
  int32_t  forward;           /* -f */
  int32_t  max_match;         /* --max-match */
  int32_t  max_count;         /* --max-count (5000); 0 is rejected: INT_MAX semantics are UB upstream */
  double   mers_matching;     /* -M percent (0) */
  double   bases_matching;    /* -B percent (17) */
  uint32_t unitigs_k;         /* -k; 0 = no k-unitig accounting */
  const int32_t* unitig_lengths; /* -l table, index = line number (misc.cc:11-19); copied */
  uint64_t n_unitigs;
  uint32_t fine_k;            /* -F; 0 = off.  Must equal the index's fine_k.  The
                                 coarse records then only define the windows of
                                 fine_aligner (fine_aligner.hpp:24-63) and the
                                 batch's records are the fine ones. */
} pbgpu_align_params;

void         pbgpu_align_params_default(pbgpu_align_params* p);
/* unitig lengths with forward == 0 -> PBGPU_ERR_INVALID (coarse_aligner.hpp:77) */
pbgpu_status pbgpu_aligner_create(const pbgpu_index* ix, const pbgpu_align_params* params,
                                  pbgpu_aligner** out);
pbgpu_status pbgpu_aligner_free(pbgpu_aligner* al);

/* ------------------------------------------------------------------ reads */
typedef struct {
  uint64_t    n_reads;
  const char* seq;            /* concatenated ASCII bases (any bytes; non-ACGT reset k-mers) */
  const uint64_t* offsets;    /* n_reads + 1 offsets into seq */
  /* optional (NULL = none): read names -- the header up to its first
     whitespace (jf_aligner.cc:133-134) -- concatenated, for the device coords
     text (pbgpu_format_device) */
  const char* names;
  const uint64_t* name_offsets; /* n_reads + 1 offsets into names */
} pbgpu_read_batch;

/* ---------------------------------------------------------------- records
 * coords_info (pb_aligner.hpp:103-175) without pointers. */
typedef struct {
  int32_t  rs, re, qs, qe;
  int32_t  nb_mers;
  uint32_t pb_cons, sr_cons, pb_cover, sr_cover;
  uint32_t ql;                /* super-read length */
  uint32_t sr_index;          /* index into the index's super-reads */
  uint32_t read;              /* read index within the batch */
  uint32_t emit;              /* emission order within (read, super-read) (--max-match) */
  uint32_t flags;             /* bit0 rn, bit1 use the bwd (reversed) name */
  uint32_t n_info;            /* kmers_info / bases_info length */
  uint32_t reserved;
  uint64_t info_offset;       /* into kmers_info / bases_info */
  double   stretch, offset, avg_err;
} pbgpu_record;

typedef struct {
  uint64_t n_reads;
  uint64_t n_records;
  const uint64_t* read_offsets;  /* n_reads + 1 into records */
  const pbgpu_record* records;    /* per read sorted by (rs, re, ql, sr_index, emit) */
  uint64_t n_info;
  const int32_t* kmers_info;
  const int32_t* bases_info;
  /* create_mega_reads' overlap graph of every record, in record order, when the
   * aligner has pbgpu_aligner_set_graph on (else NULL); see pbgpu_graph_node */
  const struct pbgpu_graph_node* graph;
  /* pbgpu_graph_params.mega_reads: per read, its printed mega-reads in print order
   * (n_reads + 1 offsets into mega; a read with none prints nothing), or, where
   * mega_host[r] is set, nothing from the device: the read is finished on the
   * host from its records, graph nodes and info, which are then the only ones in
   * records / graph / kmers_info (read_offsets index them; the other reads'
   * ranges are empty). */
  const uint64_t* mega_offsets;
  const struct pbgpu_mega_read* mega;
  const uint32_t* mega_units;
  const uint8_t* mega_host;
} pbgpu_coords_batch;

/* Host batch in, host records out (synchronous). */
pbgpu_status pbgpu_align_batch(pbgpu_aligner* al, const pbgpu_read_batch* batch,
                               pbgpu_coords_batch** out);
pbgpu_status pbgpu_coords_free(pbgpu_coords_batch* c);

/* Device-resident path (used by bench.py: inputs resident in HBM). */
pbgpu_status pbgpu_reads_upload(pbgpu_aligner* al, const pbgpu_read_batch* batch, pbgpu_reads** out);
pbgpu_status pbgpu_reads_free(pbgpu_reads* r);
/* Runs the whole GPU path on a resident batch; records stay on the device
 * until pbgpu_download().  Synchronous. */
pbgpu_status pbgpu_align_resident(pbgpu_aligner* al, const pbgpu_reads* reads);
pbgpu_status pbgpu_download(pbgpu_aligner* al, pbgpu_coords_batch** out);

/* Per-stage device time (HIP events on the aligner's stream, summed over
 * calls since the last reset), per-kernel time (events immediately around a
 * single launch of the named kernel: the first-tier k_group launch, the
 * tier-0 k_lis_w launch, k_coords, k_seed, k_rec_sort) and algorithmic
 * counters. */
enum {
  PBGPU_KERNEL_SEED = 0,
  PBGPU_KERNEL_GROUP = 1,
  PBGPU_KERNEL_LIS = 2,
  PBGPU_KERNEL_COORDS = 3,
  PBGPU_KERNEL_REC_SORT = 4,
  PBGPU_KERNEL_N = 8
};
typedef struct {
  uint64_t n_batches;
  uint64_t n_reads, n_bases;
  uint64_t n_kmers;        /* valid PB k-mers */
  uint64_t n_probes;       /* hash-bucket probes (64 B each) */
  uint64_t n_kept;         /* k-mers kept after SSR/toggle/max-count */
  uint64_t n_hits;         /* (pb_off, sr_off) hits grouped */
  uint64_t n_chains;       /* (read, super-read) chains */
  uint64_t n_lis_tests;    /* LIS predecessor tests */
  uint64_t n_records;
  double   ms_seed, ms_group, ms_lis, ms_fit, ms_records;
  double   kernel_ms[PBGPU_KERNEL_N];
  uint64_t kernel_launches[PBGPU_KERNEL_N];
  /* work completed inside the timed first-tier k_group launches (kept k-mers
   * of the reads they finished, hits scattered, chains emitted) */
  uint64_t g0_kept, g0_hits, g0_chains;
  /* work of the timed k_lis slot (the tier-0 wave-per-strand launches, strands
   * of <= 255 hits): hits and strands */
  uint64_t l0_hits, l0_strands;
  /* fine aligner (-F): windowed hits, windows (= fine records), device time */
  uint64_t n_fine_hits, n_fine_windows;
  double   ms_fine;
  /* work of the timed k_coords slot (coarse): chains fitted, lis points streamed */
  uint64_t fit_chains, fit_points;
  /* presence-filter words read by k_seed (8 B each) before the bucket probes */
  uint64_t n_filter;
  /* lis points written by the timed k_lis slot (tier-0 strands) */
  uint64_t l0_points;
  /* overlap graph (pbgpu_aligner_set_graph): device time, records traversed on the device */
  double   ms_graph;
  uint64_t graph_records;
  /* overlap graph nodes of more than 64 edges (the rest past their block, written
   * by a second pass over those nodes) */
  uint64_t graph_ovf_nodes;
  /* host time ordering a batch's reads for the group stage (the GPU waits for it) */
  double   ms_host_order;
  /* overlap graph: reads left to the host graph (more than 65535 records; 8192 before ABI 7) */
  uint64_t graph_host_reads;
  /* ABI 7: group-stage rounds that doubled the hash partitions of the reads
   * overflowing the 8192-slot table (instead of an HBM table), and reads grouped
   * in HBM tables */
  uint64_t group_refines, group_hbm_reads;
  /* ABI 8: group-stage work items (a read, or one hash partition of a long read's
   * super-reads) whose table overflowed, summed over the rounds */
  uint64_t group_overflow_items;
  /* ABI 8: reads grouped from buckets (their hits enumerated once into P >= 2 hash
   * partitions, each partition's item streaming its bucket) */
  uint64_t group_bucketed_reads;
} pbgpu_stats;
pbgpu_status pbgpu_aligner_get_stats(const pbgpu_aligner* al, pbgpu_stats* s);
pbgpu_status pbgpu_aligner_reset_stats(pbgpu_aligner* al);
/* Tuning: the maximum number of seed hits grouped and chained per device
 * sub-batch (default 4e9, about 128 GB of working buffers at most; a batch is
 * split into equal sub-batches of at most this many hits).  A read whose
 * hits exceed it forms a sub-batch of its own.  Results do not depend on it. */
pbgpu_status pbgpu_aligner_set_hit_budget(pbgpu_aligner* al, uint64_t hits);

/* ---------------------------------------------------------- sharded index
 * For super-read sets whose index does not fit one GPU (the C5
 * configuration).  Shard s of S (pbgpu_index_params.shard / n_shards) holds the
 * super-reads whose text starts in [T*s/S, T*(s+1)/S) (T = total bases) plus
 * the next k-1 bases, so every occurrence -- super-read-end crossing ones
 * included -- is counted by exactly one shard; names of all super-reads stay
 * on the host.  Every shard aligns every read of the batch:
 *   1. pbgpu_shard_counts: this shard's count of each looked-up k-mer of the
 *      batch, saturated at max_count + 1, into the aligner's count buffer (one
 *      uint32 per base of the batch);
 *   2. the counts are summed over the shards, in place: over RCCL/xGMI with
 *      pbgpu_shard_counts_allreduce (ncclAllReduce, sum), or through host
 *      memory (pbgpu_shard_counts_download / _upload).  The saturated sum
 *      decides the max-count filter and the 99% threshold exactly as the
 *      whole count does;
 *   3. pbgpu_align_resident_shard: the rest of the path on this shard's
 *      super-reads (chains never span super-reads); records carry the global
 *      sr_index;
 *   4. pbgpu_coords_merge of the shards' batches: each read's records merged in
 *      (rs, re, ql, sr_index, emit) order.
 * pbgpu_align_batch / pbgpu_align_resident reject a sharded index; -F and
 * --details run on a whole index only. */
typedef struct pbgpu_comm pbgpu_comm;
pbgpu_status pbgpu_shard_counts(pbgpu_aligner* al, const pbgpu_reads* reads);
pbgpu_status pbgpu_shard_counts_download(pbgpu_aligner* al, uint32_t* host, uint64_t n);
/* upload: n = the batch's bases; also on an aligner that has not run
 * pbgpu_shard_counts (a shard rebuilt for the alignment pass, SURVEY 8(e) on fewer GPUs than shards) */
pbgpu_status pbgpu_shard_counts_upload(pbgpu_aligner* al, const uint32_t* host, uint64_t n);
/* RCCL: rank 0 makes the 128-byte id, the caller hands it to every rank (any
 * host channel), each rank creates its communicator on its aligner's device. */
pbgpu_status pbgpu_rccl_unique_id(uint8_t id[128]);
pbgpu_status pbgpu_rccl_comm_create(int device, int n_ranks, int rank, const uint8_t id[128], pbgpu_comm** out);
pbgpu_status pbgpu_rccl_comm_free(pbgpu_comm* comm);
pbgpu_status pbgpu_shard_counts_allreduce(pbgpu_aligner* al, pbgpu_comm* comm);
/* Bytes each rank contributed to its last count all-reduce: 2 per read base
 * when n_ranks * (max_count + 1) < 65536 (two saturated 16-bit counts per
 * ncclUint32), else 4. */
uint64_t pbgpu_rccl_comm_last_bytes(const pbgpu_comm* comm);
pbgpu_status pbgpu_align_resident_shard(pbgpu_aligner* al, const pbgpu_reads* reads);
/* Host-side merge (no device work); the result is freed with pbgpu_coords_free. */
pbgpu_status pbgpu_coords_merge(const pbgpu_coords_batch* const* parts, uint64_t n_parts, pbgpu_coords_batch** out);

/* ---------------------------------------------------------- overlap graph
 * create_mega_reads' per-read overlap graph traversal on the device
 * (overlap_graph::traverse, overlap_graph.cc:7-59, with node_info::reset,
 * overlap_graph.hpp:24-34, and union_find.cc): with it on, every alignment
 * also leaves, per record, the node state the reference's traverse() ends with
 * -- longest path, its start and previous node, its unitig count, the
 * start / end node flags and the union-find root -- so the host only collects
 * the components, tiles and prints (create_mega_reads.cc:79-89).  Node indices
 * are read-local record indices (the records of a read in pbgpu_coords_batch
 * order).  A read with more records than the device traversal holds is marked
 * PBGPU_GRAPH_HOST and left to the host. */
typedef struct {
  double overlap_play;            /* -O, --overlap-play */
  double nb_errors;               /* -e, --errors */
  uint32_t k_len;                 /* -k, --k-mer (k-unitigs) */
  int32_t maximize_bases;         /* -b, --bases: path length in bases (sr_cover), else k-mers */
  /* every super-read name as its unitig list (super_read_name::parse,
   * super_read_name.cc:74-90): unitig u = id << 1 | (orientation 'R');
   * n_sr + 1 offsets into units; a name that does not parse is empty */
  uint64_t n_sr;
  const uint64_t* name_offsets;
  const uint32_t* name_units;
  /* unitig lengths (-l / -u), indexed by unitig id; ids past the end count 0 */
  const int32_t* unitig_lengths;
  uint64_t n_unitigs;
  /* mega_reads != 0: the rest of the per-read work on the device too -- the
   * components' terminal nodes (mega_reads_per_comp, overlap_graph.cc:116-161,
   * with trim_match), the tiling (tile_greedy / tile_maximal,
   * overlap_graph.cc:163-252) and the unitig paths and numbers each printed
   * mega-read needs (print_mega_reads, overlap_graph.cc:254-299): the batch
   * then carries pbgpu_coords_batch.mega* instead of records for every read
   * traversed on the device. */
  int32_t mega_reads;
  int32_t tiling;                 /* PBGPU_TILING_*  (-T) */
  int32_t trim;                   /* 0 none, 1 match (--trim; "branch" is none, create_mega_reads.cc:47-49) */
  double min_density;             /* -d */
  double min_len;                 /* -L */
} pbgpu_graph_params;
#define PBGPU_TILING_NONE     0
#define PBGPU_TILING_GREEDY   1
#define PBGPU_TILING_MAXIMAL  2
#define PBGPU_TILING_WEIGHTED 3
/* One printed mega-read of print_mega_reads (overlap_graph.cc:254-299):
 * "imp_s imp_e rs re qs qend lpath density name sr_len" with the unitig path
 * (n_units unitigs at unit_offset of pbgpu_coords_batch.mega_units) as name;
 * start_unitig / nb_unitigs select the path's unitigs whose sequence -u prints. */
typedef struct pbgpu_mega_read {
  double   imp_s, imp_e, density;
  int32_t  rs, re, qs, lpath;     /* start node's rs, end node's re, start node's qs - start offset */
  int32_t  sr_len, start_unitig, nb_unitigs;
  uint32_t n_units;
  uint64_t qend;
  uint64_t unit_offset;
} pbgpu_mega_read;
/* p = NULL turns it off.  Whole (unsharded) index only. */
pbgpu_status pbgpu_aligner_set_graph(pbgpu_aligner* al, const pbgpu_graph_params* p);
typedef struct pbgpu_graph_node {
  int32_t  lpath;                 /* node_info::lpath */
  int32_t  lstart, lprev;         /* -1 = none */
  int32_t  lunitigs;
  uint32_t root;                  /* union-find root of the node's component */
  uint32_t flags;                 /* PBGPU_GRAPH_* */
} pbgpu_graph_node;
#define PBGPU_GRAPH_START 1u          /* node_info::start_node */
#define PBGPU_GRAPH_END   2u          /* node_info::end_node */
#define PBGPU_GRAPH_HOST  0x80000000u /* not traversed on the device: the host traverses the read */

/* ---------------------------------------------------------------- details
 * --details (print_details, jf_aligner.cc:72-108): with details enabled, each
 * alignment also keeps, per read, every super-read of the coarse frags_pos
 * with its final fwd and bwd hit lists (after any --max-match discards) and
 * the elements of the printed lis (the fwd lis if strictly longer, else the
 * bwd one).  Lists of a read come in first-hit order; the reference iterates
 * an unordered_map there. */
pbgpu_status pbgpu_aligner_set_details(pbgpu_aligner* al, int enable);
typedef struct {
  uint64_t n_reads, n_lists, n_hits;
  const uint64_t* read_offsets;  /* n_reads + 1 into the lists */
  const uint32_t* list_sr;       /* super-read of each list */
  const uint64_t* hit_offsets;   /* n_lists + 1 into hits: the fwd hits, then the bwd hits */
  const uint32_t* n_fwd;         /* fwd hits of each list */
  const int32_t*  hits;          /* (pb offset, signed sr offset) pairs */
  const uint8_t*  in_lis;        /* per hit: 1 if part of the printed lis */
} pbgpu_details_batch;
/* details of the last alignment (PBGPU_ERR_INVALID if details were off) */
pbgpu_status pbgpu_download_details(pbgpu_aligner* al, pbgpu_details_batch** out);
pbgpu_status pbgpu_details_free(pbgpu_details_batch* d);

/* --------------------------------------------------------------- output
 * print_coords_header + print_coords (jf_aligner.cc:32-70): headers are the
 * full FASTA header lines of the reads (name = up to the first whitespace),
 * read_lens the read lengths (Rlen).  Text is malloc'd; free with
 * pbgpu_free_text. */
pbgpu_status pbgpu_format_coords(const pbgpu_index* ix, const pbgpu_coords_batch* c,
                                 const char* const* read_headers, const uint64_t* read_lens,
                                 int compact, int header, int zero_match, int threads,
                                 char** text, uint64_t* len);
/* print_details (jf_aligner.cc:72-108): "name sr_name pb:sr ... [pb:sr] ...",
 * fwd and bwd hits merged by pb offset (fwd first on ties), lis hits in
 * brackets. */
pbgpu_status pbgpu_format_details(const pbgpu_index* ix, const pbgpu_details_batch* d,
                                  const char* const* read_headers, int threads,
                                  char** text, uint64_t* len);
void         pbgpu_free_text(char* text);

/* print_coords on the device: the last alignment's records (reads uploaded
 * with names) as the coords text -- byte-identical to pbgpu_format_coords
 * with header = 0 -- into a device buffer owned by the aligner; *text_len =
 * its length.  pbgpu_text_download copies its first len bytes to dst (pinned
 * host memory from pbgpu_host_alloc is copied at full PCIe rate). */
pbgpu_status pbgpu_format_device(pbgpu_aligner* al, const pbgpu_reads* reads, int compact, int zero_match,
                                 uint64_t* text_len);
pbgpu_status pbgpu_text_download(pbgpu_aligner* al, void* dst, uint64_t len);
pbgpu_status pbgpu_host_alloc(uint64_t bytes, void** out);   /* pinned host memory */
pbgpu_status pbgpu_host_free(void* p);
/* Test aid (no reference counterpart): the device formatter's rendering of
 * one double, run on the host -- std::ostream << v at precision 6, i.e.
 * printf("%.6g", v).  out needs 32 bytes; returns the length. */
int          pbgpu_format_double(double v, char* out);

/* A replica of an index on another device (device-to-device copies of the
 * resident arrays; no rebuild).  SURVEY 8(e): read-sharded multi-GPU runs
 * keep one replica per GPU. */
pbgpu_status pbgpu_index_replicate(const pbgpu_index* src, int device, pbgpu_index** out);

/* On-disk index cache ("optionally add an on-disk index
 * cache"; the reference rebuilds its PSA on every run, superread_parser.hpp:
 * 219-224).  pbgpu_index_save writes every host and device array of a built
 * index to `path` with a caller-chosen `tag` (e.g. k, psa_min, fine_k and the
 * super-read files' sizes and times); pbgpu_index_load rebuilds it on `device`
 * from the file alone, and fails with PBGPU_ERR_IO when the file is missing,
 * truncated, of another format version, or saved with another tag. */
pbgpu_status pbgpu_index_save(const pbgpu_index* ix, const char* path, const char* tag);
pbgpu_status pbgpu_index_load(const char* path, int device, const char* tag, pbgpu_index** out);

/* ---------------------------------------------------------------- driver
 * The jf_aligner main loop (jf_aligner.cc:205-230, print_alignments :110-159)
 * as one call: PacBio FASTA / FASTQ files (plain or gzip) are parsed in
 * batches; every entry of `indexes` gets `aligners_per_device` aligners (own
 * HIP stream and host thread each; the same index may be listed twice);
 * batches go to whichever aligner is free (dynamic assignment absorbs read
 * length skew); each is aligned and formatted on its device, copied to pinned
 * host memory and written in input order -- the output is the reference's
 * with -t 1 (per-read records sorted, reads in input order). */
typedef struct {
  const char* const* pb_paths;    /* -p, --pacbio (FASTA/FASTQ, plain or gzip) */
  size_t n_pb_paths;
  const char* coords_path;        /* --coords; NULL = stdout */
  const char* details_path;       /* --details; NULL = none */
  int32_t compact;                /* --compact (default on) */
  int32_t header;                 /* print_coords_header unless -H */
  int32_t zero_match;             /* -0 */
  uint32_t aligners_per_device;   /* 0 = 2 */
  uint64_t batch_bases;           /* bases per batch; 0 = 64 M */
  int32_t host_threads;           /* --details formatting threads; 0 = all */
  /* Optional consumer of the records (create_mega_reads, create_mega_reads.cc:
   * 25-93): when set, each batch's records are downloaded and handed to it on
   * the worker thread instead of being formatted as coords; the text it returns
   * (malloc'd, freed by the driver; NULL = none) is written to coords_path and
   * its side text (*side_text, e.g. the --dot graph) to details_path, both in
   * batch order.  Nonzero *status from it stops the run (PBGPU_ERR_INTERNAL). */
  char* (*records_fn)(void* user, const pbgpu_index* ix, const pbgpu_coords_batch* coords,
                      const char* const* read_names, const uint64_t* read_lens, uint64_t* text_len,
                      char** side_text, uint64_t* side_len, int* status);
  void* records_user;
  /* Part files (0 or 1 = one file).  With P > 1 the output goes to P files
   * <coords_path>.0 .. .<P-1> (and <details_path>.p), each with its own reader,
   * aligners and writer thread: part p holds the reads whose FASTA header
   * starts in [p T / P, (p + 1) T / P) of the concatenated input files (T
   * bytes), so the parts concatenated are the one-file output -- the
   * reference's split-and-cat (mega_reads_assemble_cluster2.sh:325-354,447) in
   * one process, without the single writer's page-cache ceiling.  The aligners
   * are split between the parts in order (part p: aligners [p W / P, (p + 1)
   * W / P) of the W, so with one index per part each part runs on its own
   * device).  Plain FASTA input only; fixed at pbgpu_runner_create. */
  uint32_t n_parts;
  /* With records_fn: create_mega_reads' overlap graph on the device for every
   * batch (pbgpu_aligner_set_graph on each aligner; the records consumer gets
   * pbgpu_coords_batch.graph).  NULL = off.  Fixed at pbgpu_runner_create. */
  const pbgpu_graph_params* graph;
} pbgpu_run_params;

typedef struct {
  double   wall_seconds;          /* first batch read -> coords file closed */
  uint64_t n_batches, n_reads, n_bases, n_records, coords_bytes, details_bytes;
  /* busy seconds per stage, summed over the threads doing it */
  double   read_seconds;          /* reader: parse input into batches */
  double   upload_seconds;        /* workers: host -> device read copies */
  double   align_seconds;         /* workers: the device pipeline (host wall) */
  double   format_seconds;        /* workers: device text formatting (records_fn: record download) */
  double   d2h_seconds;           /* workers: text -> pinned host memory (records_fn: the consumer) */
  double   write_seconds;         /* writer: write() calls */
  double   writer_idle_seconds;   /* writer: waiting for the next batch in order */
  double   open_seconds;          /* opening (creating / truncating) the output files */
  double   close_seconds;         /* closing the coords file after the last write */
  /* allocations made by the workers during the run: device (hipMalloc) and
   * pinned host; _late = in any worker's batches after its first (the run
   * path sizes its per-batch buffers for a full batch when they first grow,
   * so these are 0 unless a batch needs more than 2x the first's density) */
  uint64_t n_device_allocs, n_device_allocs_late;
  uint64_t n_pinned_allocs, n_pinned_allocs_late;
  /* bytes of those device allocations, and the seconds the workers spent in
   * hipMalloc / hipFree (a call that blocks shows here) */
  uint64_t device_alloc_bytes;
  double   alloc_seconds;
  /* ABI 7: the device working set -- the workers' largest live device bytes (each
   * worker's aligner buffers at their high-water mark), summed over the workers --
   * and, with records_fn and a device graph, the reads whose graph the host finished */
  uint64_t device_peak_bytes;
  uint64_t graph_host_reads;
} pbgpu_run_stats;

pbgpu_status pbgpu_run(pbgpu_index* const* indexes, size_t n_indexes, const pbgpu_align_params* params,
                       const pbgpu_run_params* run, pbgpu_run_stats* stats);
/* The same as a long-lived object (pbgpu_run = create + run + free): the
 * aligners, their device buffers and the pinned batch / text buffers are kept
 * between runs, so a service aligning many files pays their setup once.
 * create uses run->aligners_per_device, batch_bases and whether
 * details_path is set; every run must agree on details. */
typedef struct pbgpu_runner pbgpu_runner;
pbgpu_status pbgpu_runner_create(pbgpu_index* const* indexes, size_t n_indexes, const pbgpu_align_params* params,
                                 const pbgpu_run_params* run, pbgpu_runner** out);
pbgpu_status pbgpu_runner_run(pbgpu_runner* runner, const pbgpu_run_params* run, pbgpu_run_stats* stats);
pbgpu_status pbgpu_runner_free(pbgpu_runner* runner);

#ifdef __cplusplus
}
#endif
#endif /* PBGPU_H */
