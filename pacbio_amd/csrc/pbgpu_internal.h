// pbgpu_internal.h -- shared device/host layouts of the MI355X jf_aligner path.
//
// HBM layout (resident index, built once per device):
//   text     : uint64[ceil(n/32)+2]  2-bit bases, MSB-first within a word
//              (word w holds bases 32w..32w+31, base 32w in bits 63..62)
//   sr_start : uint64[n_sr+1]        global text offset of every super-read
//   table    : ulonglong2[4*buckets] 64-byte buckets of 4 {key, payload} slots,
//              key = canonical k-mer code (EMPTY = ~0), payload =
//              occ_ptr << 24 | min(count_total, 2^24-1)
//   occ      : uint64[]              per canonical k-mer: 2 header words
//              {count_total | pal<<32, nA | nB<<32} then nA occurrences of the
//              canonical k-mer and nB of its reverse complement, each
//              (sr_id << 32 | 1-based offset), descending text position
//              (the SA tie-break of mer_sa_imp.hpp:363).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace pbgpu {

// Version of the device index layout above (bucket hash, presence-filter hash,
// header packing, element sizes).  Bump it with any change to them: the on-disk
// index cache (pbgpu_index_save / load) refuses files of another layout.
constexpr uint32_t kIndexLayout = 3;

constexpr uint64_t EMPTY_KEY = ~0ull;
constexpr uint32_t SAT_COUNT = 0xFFFFFFu;
constexpr uint32_t INVALID_UNITIG = 0x7fffffffu;

struct IndexView {
  const uint64_t* text;
  uint64_t n;
  const uint64_t* sr_start;   // n_sr + 1
  uint32_t n_sr;
  uint32_t k;
  const ulonglong2* table;    // 4 slots per bucket
  uint64_t bucket_mask;
  const uint64_t* occ;
  // optional: the super-read id (high word) of every occ word, packed (k_group's
  // counting pass reads 4 B a hit from it instead of an 8-B entry's line); null: none
  const uint32_t* occ_sr;
  const uint32_t* sr_uoff;    // n_sr + 1 offsets into sr_uids
  const uint32_t* sr_uids;    // unitig ids of the fwd name (super_read_name::unitig_id)
  const uint64_t* filt;       // presence filter of the table's canonical k-mers (null: none)
  uint32_t filt_shift;        // word index = filter hash >> filt_shift
};

// per super-read, what k_coords' prologue reads (one 32-byte line): its length, its name's
// range in sr_uids / sr_ul, and the name's first SR_META_UL resolved unitig lengths
constexpr uint32_t SR_META_UL = 5;
struct SrMeta {
  uint32_t ql, u0, nsz;
  int32_t ul[SR_META_UL];
};
static_assert(sizeof(SrMeta) == 32, "one 32-byte line");
struct AlignParamsDev {
  uint32_t k;
  uint32_t window;
  double a, b, C;          // affine_capped(stretch_factor, stretch_constant, stretch_cap)
  int32_t forward, max_match;
  int32_t max_count;       // never 0 here
  double mers_factor;      // M / 100
  double bases_factor;     // B / 100
  uint32_t unitigs_k;
  const int32_t* ul;
  uint64_t n_ul;
  const int32_t* sr_ul;    // unitig length of every name entry (index sr_uids order), INT32_MIN if unusable
  const SrMeta* sr_meta;   // (with sr_ul) per super-read: SrMeta
  int32_t fine;            // fine_aligner pass: every chain emits a record, no filters (fine_aligner.cc:43-48)
};

// fine_aligner window (sr_local_ml, fine_aligner.hpp:12-17) of one coarse
// record: implied first / last start base of a k-mer in the read.  Sorted by
// (read, super-read); w = the coarse record (list id) it belongs to.
struct FineWin {
  uint32_t sr, w;
  double begin, end;
};

// kept k-mer record, one per kept PB k-mer, in read order
struct KRec {
  int32_t pb_off;       // 1-based start of the k-mer in the read
  uint32_t count;       // total occurrences of m and rm (incl. crossing)
  uint64_t occ_ptr;     // header index in occ; bit 63 = is_canonical (m < rm)
};

struct ChainDesc {
  uint32_t read, sr;
  uint32_t nf, nb;
  uint64_t hit_base;     // first fwd node; bwd nodes follow at hit_base + nf
};

// Per-hit buffers of a sub-batch (hit index = read-local list position +
// the read's hit offset):
//   X    int2  (pb offset, signed sr offset), written by k_group in list order
//   N16  8 B   LIS node per hit, LNode<uint16_t> (strands of <= 65535 hits)
//   N32  16 B  LIS node per hit of the longer strands, LNode<uint32_t>, packed
//              (hit index + a per-strand shift, k_node32_place; round 5: it was
//              per hit of the whole sub-batch)
//   pts  int2  the strand's LIS points X[lis[0..len)) after k_lis
// LNode: singly linked list of lis_align::compute_L_P (lis_align.hpp:139-182);
// nxt doubles as the lis index array after the forward pass (--max-match).
template <typename I>
struct LNode {
  I nxt, len, P, root;
};
static_assert(sizeof(LNode<uint16_t>) == 8 && sizeof(LNode<uint32_t>) == 16, "node sizes");
constexpr uint32_t LIS_U16_MAX = 0xFFFFu;   // strands up to this many hits use 16-bit nodes

struct Rec {
  int32_t rs, re, qs, qe, nb_mers;
  uint32_t pb_cons, sr_cons, pb_cover, sr_cover;
  uint32_t ql, sr, read, emit, flags, n_info, reserved;
  uint64_t info_off;
  double stretch, offset, avg_err;
};
static_assert(sizeof(Rec) == 96, "Rec layout must match pbgpu_record");

enum StatSlot {
  ST_KMERS = 0, ST_PROBES, ST_KEPT, ST_HITS, ST_CHAINS, ST_LIS_TESTS, ST_RECORDS,
  ST_REC_OVERFLOW, ST_INFO_USED, ST_GROUP_OVERFLOW,
  ST_G0_KEPT, ST_G0_HITS, ST_G0_CHAINS,  // work completed by first-tier (4-wave LDS) k_group launches
  ST_L0_HITS, ST_L0_STRANDS,             // work of the tier-0 (n <= 255) k_lis_w launches
  ST_FINE_HITS,                          // fine aligner: windowed hits
  ST_FIT_CHAINS, ST_FIT_POINTS,          // coarse k_coords work: chains, lis points (counted by the chain order pass)
  ST_FILTER,                             // presence-filter words read by k_seed (8 B each)
  ST_L0_POINTS,                          // lis points written by the tier-0 k_lis_w launches
  ST_N
};

constexpr uint32_t GROUP_SINKS = 256;  // spread over lines and channels, not one hot address
struct GroupOut {
  int2* X;
  int2* sink;              // GROUP_SINKS entries past the sub-batch's lists: the stores of lanes without a hit
  ChainDesc* chains;
  uint32_t* chain_count;
  uint32_t chain_cap;
  uint2* overflow_items;   // the work items whose table overflowed (group_item)
  uint32_t* overflow_grow;  // per overflowing item: ceil(its k-mers / those its pass 0 had taken) | table log2 << 24
  uint32_t* n_overflow;
  uint32_t overflow_cap;    // entries of overflow_items / overflow_grow (>= the launch's work items)
  uint32_t* rcur;          // per read: hits placed so far by its partitions (P > 1 items)
  // Bucketed reads (round 6): a read predicted to need P >= 2 hash partitions has its hits
  // enumerated once by a split launch (k_group MODE 1), which writes them, stably by
  // partition, to a staging copy in the sub-batch's LIS buffers (free until the LIS stage):
  // stage_sr = super-read | bwd << 31, stage_x = {pb offset, 1-based sr offset}, at
  // the read's hit range; bucket p of the read is [boff[bmeta.x + p], boff[bmeta.x + p + 1]),
  // read-local, bmeta[r] = {boff base, P0}.  Its partition items (MODE 2) then stream their
  // bucket instead of re-enumerating every hit of the read (C4: ~4 items a read each did).
  int2* stage_x;
  uint32_t* stage_sr;
  uint32_t* boff;
  const uint2* bmeta;
};
// k_group work item {read, partition | partitions << 16}: the read's hits whose super-read
// falls in hash partition `partition` of `partitions` (floor(h * P / 2^32) of the id's hash,
// so partition p of P is exactly partitions 2p and 2p + 1 of 2P)
inline __host__ __device__ uint2 group_item(uint32_t r, uint32_t part, uint32_t nparts) { return make_uint2(r, part | nparts << 16); }

struct LisParams {
  uint32_t W;
  double a, b, C;   // affine_capped; seq uses linear(a)
  int mer_all, seq_all;  // accept_all (lis_align.hpp) for the step / whole-chain test (fine aligner)
  int ordered;           // lists are already in list order (no k_group order restoration)
};

// Lis points of one strand, written by the LIS kernels into the strand's own
// region of the per-hit array pts (room for n >= len int2) and read by
// k_coords and the details capture.  Two layouts:
//  * compact (len >= 2, every point within 65535 of the last one in x and y):
//    word 0 = last.x | PT_COMPACT, word 1 = last.y, word 2 + i =
//    (last.x - x_i) << 16 | (last.y - y_i) -- 4 bytes a point;
//  * wide: pts[i] = (x_i, y_i), x_i > 0 (a pb offset) so word 0 has no flag.
constexpr uint32_t PT_COMPACT = 0x80000000u;
__host__ __device__ inline bool pt_fits(int2 last, int2 p) {
  return (uint32_t)(last.x - p.x) < 65536u && (uint32_t)(last.y - p.y) < 65536u;
}
__host__ __device__ inline uint32_t pt_word(int2 last, int2 p) {
  return (uint32_t)(last.x - p.x) << 16 | (uint32_t)(last.y - p.y);
}
__host__ __device__ inline int2 pt_decode(int2 last, uint32_t w) {
  return make_int2(last.x - (int32_t)(w >> 16), last.y - (int32_t)(w & 0xFFFFu));
}
// point i of the lis stored at region (host side: details)
__host__ __device__ inline int2 pt_get(const int2* region, uint32_t i) {
  const uint32_t* w = (const uint32_t*)region;
  if (w[0] & PT_COMPACT) return pt_decode(make_int2((int32_t)(w[0] & ~PT_COMPACT), (int32_t)w[1]), w[2 + i]);
  return region[i];
}

struct ChainOut {
  const int2* pts;
  const uint32_t* lisl;
  uint32_t* redo;          // --max-match: chains to discard + redo
  uint32_t* n_redo;
  Rec* recs;
  uint32_t* rec_read;       // per record its read (records_stage's histogram / scatter read 4 B, not a 96-B record)
  uint32_t* rec_count;
  uint32_t rec_cap;
  int32_t* info_m;
  int32_t* info_b;
  unsigned long long* info_count;
  uint64_t info_cap;
  unsigned long long* stats;
  const uint32_t* emit_of;  // fine pass: per chain, the emission index of its coarse record (else null)
  // (coarse pass without --max-match) per read its record count, and per record its
  // rank among its read's (the counter's old value): records_stage then places the
  // records with neither a histogram nor a scatter of atomics.  Null: not counted.
  uint32_t* per_read;
  uint32_t* rec_slot;
};

// Exclusive scan of n counts (u32 or u64, exactly one of in32 / in64 non-null) into
// n + 1 offsets, out[n] = the total (pbgpu_kernels.hip; replaces a library scan on the
// per-batch path).  scratch: excl_scan_scratch_words(n) words.
// every d in [1, n_max]: the fit's reciprocal (recip_int) against __ddiv_rn(1.0, d); mismatches added to *bad
void launch_check_recip(uint32_t n_max, unsigned long long* bad, hipStream_t st);
uint64_t excl_scan_scratch_words(uint64_t n);
void launch_excl_scan(const uint32_t* in32, const uint64_t* in64, uint64_t n, uint64_t* out, uint64_t* scratch,
                      hipStream_t st);

// create_mega_reads' overlap graph on the device (pbgpu_kernels.hip, k_graph_*):
// node_info after overlap_graph::traverse for every record, in the record order
// of recs_sorted (the layout of pbgpu_graph_node, include/pbgpu.h).
struct GraphNode {
  int32_t lpath, lstart, lprev, lunitigs;
  uint32_t root, flags;
};
static_assert(sizeof(GraphNode) == 24, "GraphNode layout must match pbgpu_graph_node");
constexpr uint32_t GRAPH_START = 1u, GRAPH_END = 2u, GRAPH_HOST = 1u << 31;  // flags
constexpr uint32_t GRAPH_NMAX = 8192;  // records of a read traversed with its node state in LDS
// records of a read traversed on the device at all (more: GRAPH_HOST): past GRAPH_NMAX the
// sort keys and the node state live in the read's region of GraphDev::scratch; an edge
// names its node j in 16 bits
constexpr uint32_t GRAPH_NMAX_BIG = 65535;
// a record in the per-read sorted order (k_graph's ring of sorted positions)
// A node's descriptor in sorted order, one 64-byte line: what k_graph_edges tests for
// a pair, the name's first GRAPH_U units included, so a scan past the staged window
// reads one line a node (round 4: the descriptor plus a scattered load per unit).  The
// name's offset (G.poff[read base + idx]) is read only for a pair that overlaps.
constexpr uint32_t GRAPH_U = 8;  // names of at most this many unitigs are matched in registers
struct alignas(64) GDesc {
  double imp_s, imp_e, err;
  uint16_t idx, nsz;           // its record index in the read (< GRAPH_NMAX_BIG), name unitigs
  uint32_t lp_add;             // nb_mers or sr_cover
  uint32_t u[GRAPH_U];         // the name's first units in the record's orientation (0 past nsz)
};
static_assert(sizeof(GDesc) == 64, "a descriptor is one 64-byte line");
struct GraphDev {
  const Rec* recs;            // recs_sorted
  const uint64_t* rec_off;    // per read, into recs
  const uint64_t* roff;       // read offsets (read lengths)
  const uint64_t* noff;       // super-read names: n_sr + 1 offsets into units
  const uint32_t* units;      // unitig id << 1 | R (super_read_name::parse)
  const int32_t* ul;          // unitig lengths
  uint64_t n_ul;
  const int32_t* info_m;      // kmers_info / bases_info
  const int32_t* info_b;
  double play, nb_errors;     // -O, -e
  uint32_t k;                 // -k
  int bases;                  // -b
  uint32_t nmax;              // reads with more records go to the host (<= GRAPH_NMAX_BIG; tests lower it)
  uint32_t relax_big_min;     // reads with more records relax with their state in HBM (k_graph_relax_big)
  double2* imp;               // per record: implied start, end
  uint64_t* poff;             // per record: its prefix sums' offset (nsz + 1 each)
  uint2* pp;                  // prefix sums along the name: {unitig lengths, info[2u] - info[2u - 1]}
  uint32_t* ounits;           // the name's unitigs in the record's orientation (at poff)
  GDesc* desc;                // per read, in sorted order
  uint32_t* spo;              // per sorted position: its record's poff (loaded beside desc)
  // per sorted position, the fields k_graph_edges' prefilter reads, one array each (a scan
  // reads them coalesced): implied start, end, error, first unitig of the name
  double *fis, *fie, *fer;
  uint32_t* fu0;
  // per 64 sorted positions of the batch (q >> 6): the largest imp_e of its nodes with
  // imp_s > 1 (NaN as +inf; -inf if none): k_graph_edges skips a whole block when node i
  // is past it by more than 31 (every node of it is "not advancing", overlap_graph.cc:20)
  double* bmax;
  GraphNode* out;
  // the traversal's edges (k_graph_edges): per node in sorted order its count, its
  // first GRAPH_EBLK edges in a block of its own (edges + q * GRAPH_EBLK) and, past
  // them, the rest at eovf + eoff[q]; an edge is {j's record index | unitigs added
  // << 16, path increment}.  ovf: {nodes listed in ovf_list, overflow edges}
  uint32_t* max_n;  // the most records of a read in the batch (k_graph_sizes; gates the tiers)
  uint32_t* ecnt;
  uint64_t* eoff;
  uint2* edges;
  uint2* eovf;
  uint64_t* ovf;
  uint64_t* ovf_list;
  // mega-reads on the device (pbgpu_graph_params.mega_reads)
  int mega, tiling, trim;
  double min_density, min_len;
  struct MegaTmp* cand;       // per read region [rec_off[r], rec_off[r + 1]): scratch
  int32_t* ord;               // 3 int scratch regions of n_recs each
  double2* ivs;               // 2 double2 scratch regions of n_recs each
  struct MegaOut* mo;         // per read region: its printed mega-reads in print order
  uint32_t* mcount;           // per read: printed mega-reads
  uint8_t* mhost;             // per read: 1 = left to the host
  uint32_t* munits;           // the printed paths' unitigs (units_cap), allocated by units_used
  unsigned long long* units_used;
  uint64_t units_cap;
  uint64_t n_recs;
#ifdef PBGPU_GRAPH_CHECK
  uint64_t units_total;       // poff[n_recs]: the batch's name units / prefix sums (bounds-check build)
#endif
  uint32_t* n_host;           // reads left to the host
  // 6 words per record (the records stage's sort scratch, free by then): reads of more
  // than GRAPH_NMAX records keep their sort keys, then their node state, then k_mega's
  // root bitmap in their region [6 rec_off[r], 6 rec_off[r + 1])
  uint64_t* scratch;
};
// mega_read_info (overlap_graph.hpp:48-58) of a candidate, with its node's lpath and root
struct MegaTmp {
  double imp_s, imp_e, tiling_start, tiling_end, density;
  int32_t start_node, end_node, start_unitig, end_unitig, start_offset, end_offset, nb_unitigs, lpath;
  uint32_t root, pad;
};
// the layout of pbgpu_mega_read (include/pbgpu.h)
struct MegaOut {
  double imp_s, imp_e, density;
  int32_t rs, re, qs, lpath;
  int32_t sr_len, start_unitig, nb_unitigs;
  uint32_t n_units;
  uint64_t qend;
  uint64_t unit_offset;
};
static_assert(sizeof(MegaOut) == 72, "MegaOut layout must match pbgpu_mega_read");
// after launch_graph: components, tiling and print paths per read (mega != 0)
void launch_mega(const GraphDev& G, uint32_t n_reads, hipStream_t st);
// the printed mega-reads of every read packed in read order: mc[moff[r] ..]
void launch_mega_pack(const GraphDev& G, uint32_t n_reads, const uint64_t* moff, MegaOut* mc, hipStream_t st);
// the reads left to the host (mhost): per record its info size if its read is one (else 0)
void launch_host_sizes(const GraphDev& G, uint32_t n_reads, uint32_t* rsize, uint32_t* isize, hipStream_t st);
// their records (info offsets rebased), graph nodes and kmers / bases info, packed in read order
void launch_host_pack(const GraphDev& G, uint32_t n_reads, const uint64_t* hroff, const uint64_t* hioff, Rec* hrec,
                      GraphNode* hgraph, int32_t* hinfo_m, int32_t* hinfo_b, hipStream_t st);
// G.poff from the records' name sizes (then the caller sizes pul / pco by poff[n_recs])
// (and *G.max_n: the most records of a read, for the tiers' launches)
void launch_graph_sizes(const GraphDev& G, uint32_t n_reads, uint64_t n_recs, uint32_t* sizes, uint64_t* scan_scratch,
                        hipStream_t st);
// implied positions and prefix sums, the per-read sort, every node's edges (G.ecnt,
// the first GRAPH_EBLK of each in G.edges, sized n_recs * GRAPH_EBLK; the nodes with
// more listed: ovf[2] = {nodes, edges past their blocks}, the stream synchronized);
// then, with G.eovf sized for them, launch_graph_relax writes those and traverses
// -> G.out.  side / side2: streams for the reads of more than GRAPH_NM_SMALL records
// (their sort and relaxation run beside the others'); fork / join / join2: events
// ordering them with st
#ifndef PBGPU_GRAPH_EBLK
#define PBGPU_GRAPH_EBLK 64
#endif
constexpr uint32_t GRAPH_EBLK = PBGPU_GRAPH_EBLK;
// (max_n: *G.max_n as k_graph_sizes left it; tiers above it are not launched)
hipError_t launch_graph(const GraphDev& G, uint32_t n_reads, uint64_t n_recs, uint32_t max_n, hipStream_t st,
                        hipStream_t side, hipEvent_t fork, hipEvent_t join, uint64_t* ovf);
hipError_t launch_graph_relax(const GraphDev& G, uint32_t n_reads, uint64_t n_recs, uint32_t max_n, uint64_t n_ovf,
                              hipStream_t st, hipStream_t side, hipStream_t side2, hipEvent_t fork, hipEvent_t join,
                              hipEvent_t join2);

}  // namespace pbgpu
