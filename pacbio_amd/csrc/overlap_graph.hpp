// overlap_graph.hpp -- create_mega_reads' per-read graph work, host C++ fed by
// the GPU coords records (pbgpu_run's records consumer).
//
// Restates /root/reference/src_jf_aligner/overlap_graph.{hpp,cc} and the
// create_mega_reads worker (create_mega_reads.cc:55-90): the records of one
// PacBio read, sorted by (rs, re, ql), are nodes; two nodes overlap when their
// implied positions on the read and their super-read names (a dovetail of
// k-unitigs) agree; a longest path is kept per node and connected components
// are tracked with union-find; each component's best terminal node is a
// mega-read candidate; the candidates are tiled (greedy / maximal / weighted)
// and printed.  The reference's boost::icl interval set (tile_greedy) is
// replaced by a small ordered set of joined right-open intervals.
#pragma once
#include <stdint.h>

#include <ostream>
#include <string>
#include <vector>

#include "../../include/pbgpu.h"  // pbgpu_graph_node: the traversal done on the device

namespace megareads {

// super_read_name::u_id_ori (super_read_name.hpp:16-37): bit 0 = orientation (R),
// bits 1.. = unitig id (31 bits); equality on the raw word
typedef uint32_t unitig_t;
inline unitig_t make_unitig(uint32_t id, bool rev) { return (id & 0x7fffffffu) << 1 | (rev ? 1u : 0u); }
inline uint32_t unitig_id(unitig_t u) { return u >> 1; }
inline bool unitig_rev(unitig_t u) { return u & 1u; }
typedef std::vector<unitig_t> unitig_list;

constexpr uint32_t INVALID_ID = 0x7fffffffu;  // super_read_name::invalid_id

// super_read_name::parse (super_read_name.cc:74-90); empty on a malformed name
unitig_list parse_name(const std::string& name);
// super_read_name::get_reverse (super_read_name.cc:38-47)
unitig_list reverse_name(const unitig_list& u);
// super_read_name::overlap (super_read_name.cc:49-72): the largest m such that the
// last m unitigs of a are the first m of b (0 if either has < 2 unitigs)
int name_overlap(const unitig_list& a, const unitig_list& b);
// operator<< (super_read_name.cc:92-100)
void print_name(std::ostream& os, const unitig_list& u);

// union_find.{hpp,cc}: union by rank with path compression, over node indices
struct UnionFind {
  std::vector<int> parent, rank;
  void reset(int n);
  int root(int s);
  void unite(int a, int b);  // union_sets(a, b): ties attach b's root under a's
};

// The coords_info fields the graph reads (pb_aligner.hpp:103-175)
struct Coord {
  int rs, re, qs, qe, nb_mers;
  uint32_t sr_cover;
  uint64_t rl, ql;  // PacBio read length, super-read length
  double stretch, offset, avg_err;
  const unitig_list* name;  // name_u->unitigs
  const int32_t* kmers_info;
  const int32_t* bases_info;
  uint32_t n_info;
};

struct Node {  // node_info (overlap_graph.hpp:11-42)
  bool start_node, end_node;
  double imp_s, imp_e;
  int lstart, lprev, lpath, lunitigs;
};

struct MegaRead {  // mega_read_info (overlap_graph.hpp:48-58)
  int start_node, end_node;
  int start_unitig, end_unitig;
  int start_offset, end_offset;
  int nb_unitigs;
  double imp_s, imp_e;
  double tiling_start, tiling_end;
  double density;
};

enum class Tiling { NONE, GREEDY, MAXIMAL, WEIGHTED };
enum class Trim { NONE, MATCH, BRANCH };

struct Params {
  double overlap_play = 1.3;   // -O
  unsigned k_len = 0;          // -k
  double nb_errors = 3.0;      // -e
  bool maximize_bases = false; // -b
  double min_density = 0.029;  // -d
  double min_len = 100.0;      // -L
  Tiling tiling = Tiling::GREEDY;
  Trim trim = Trim::NONE;
  const std::vector<int>* unitig_lengths = nullptr;
  const std::vector<std::string>* unitig_sequences = nullptr;  // -u: print the mega-read sequence
};

// One worker's scratch (overlap_graph::thread): process() takes one read's
// records in (rs, re, ql) order and appends its mega-reads (and, with dot, its
// graph) to the streams.
class ReadGraph {
 public:
  explicit ReadGraph(const Params& p) : p_(p) {}
  // dev: the read's nodes as the device traversal left them (pbgpu_aligner_set_graph),
  // one per record; NULL, or a read marked PBGPU_GRAPH_HOST, is traversed here
  void process(const std::vector<Coord>& coords, const std::string& pb_name, std::ostream& out, std::ostream* dot,
               const pbgpu_graph_node* dev = nullptr);
  // the read's mega-reads computed on the device (pbgpu_graph_params.mega_reads), printed
  // as print_mega_reads prints them (overlap_graph.hpp:253-262, overlap_graph.cc:254-299)
  void print_device(std::ostream& out, const std::string& pb_name, const pbgpu_mega_read* m, uint64_t n,
                    const uint32_t* units) const;

 private:
  friend struct ReadGraphTest;  // tests/cpp/og_driver.cpp (tiling properties)
  int ulen(uint32_t id) const;
  void traverse(std::ostream* dot);
  void components(std::ostream* dot);
  MegaRead make(int i) const;
  void trim_match(MegaRead& mr) const;
  int tile_greedy(const std::vector<int>& order, std::vector<int>& res) const;
  int tile_maximal(const std::vector<int>& order, std::vector<int>& res) const;
  void print(std::ostream& out, const std::vector<int>& order, std::ostream* dot) const;
  void print_sequence(std::ostream& os, const unitig_list& u, int start, int nb) const;

  const Params& p_;
  const std::vector<Coord>* coords_ = nullptr;
  std::vector<Node> nodes_;
  UnionFind uf_;
  std::vector<int> sort_nodes_, sort_tiling_, tiled_mr_;
  std::vector<double> weights_;
  std::vector<std::pair<int, MegaRead>> comp_;  // per component root (ascending), its mega-read
  std::vector<const MegaRead*> mega_reads_;
  // traverse()'s per-read scratch: prefix sums over each node's name, the sorted
  // nodes (read-only part, and the path state the traversal updates, in sorted order)
  struct SortedNode {
    double imp_s, imp_e, avg_err;
    const unitig_t* name;
    const uint32_t *pul, *pco;  // its prefix sums
    int idx, nsz;        // node index, unitigs in its name
    unitig_t u0;         // first unitig of its name
    unsigned lp_add;     // its path length contribution (sr_cover with -b, else nb_mers)
  };
  struct PathState {
    double ls_imp_s;     // imp_s of the node's path start (lstart, or itself)
    int lpath, lstart, lprev, lunitigs;
    bool start_node, end_node;
  };
  std::vector<PathState> state_;
  const pbgpu_graph_node* dev_ = nullptr;  // the current read's device traversal (roots), or NULL
  std::vector<size_t> pre_off_;
  std::vector<uint32_t> pul_, pco_;
  std::vector<SortedNode> sorted_;
};

}  // namespace megareads
