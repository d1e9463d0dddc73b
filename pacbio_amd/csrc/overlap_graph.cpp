// overlap_graph.cpp -- see overlap_graph.hpp.  Each function cites the
// reference code it restates (paths under /root/reference/src_jf_aligner/).
#include "overlap_graph.hpp"

#include <algorithm>
#include <cstdlib>
#include <iomanip>
#include <limits>
#include <stdexcept>

namespace megareads {

// super_read_name::parse (super_read_name.cc:74-90): tokens split on '_', each an
// unsigned number (std::stoul prefix) whose orientation is the character before
// the '_' (or the last character); any token without a leading number empties
// the list.
unitig_list parse_name(const std::string& name) {
  unitig_list res;
  if (name.empty()) return res;
  size_t pn = 0;
  for (;;) {
    const size_t n = name.find('_', pn);
    const char* s = name.c_str() + pn;
    while (*s == ' ' || (*s >= '\t' && *s <= '\r')) ++s;  // std::stoul skips leading space
    const char* p = s;
    if (*p == '+' || *p == '-') ++p;
    if (*p < '0' || *p > '9') return unitig_list();
    const unsigned long v = strtoul(s, nullptr, 10);
    const char ori = n != std::string::npos ? name[n - 1] : name[name.size() - 1];
    res.push_back(make_unitig((uint32_t)v, ori == 'R'));
    if (n == std::string::npos) break;
    pn = n + 1;
  }
  return res;
}

// super_read_name::reverse (super_read_name.cc:38-47)
unitig_list reverse_name(const unitig_list& u) {
  unitig_list r(u.rbegin(), u.rend());
  for (auto& x : r) x ^= 1u;
  return r;
}

// super_read_name::overlap (super_read_name.cc:49-72)
int name_overlap(const unitig_list& a, const unitig_list& b) {
  if (b.empty()) return 0;
  const int sa = (int)a.size(), sb = (int)b.size();
  if (sa < 2 || sb < 2) return 0;
  const int start = std::max(sa - sb + 1, 1);
  for (int i = start; i < sa; ++i) {
    if (b[0] != a[i]) continue;
    int j = i + 1;
    while (j < sa && a[j] == b[j - i]) ++j;
    if (j == sa) return sa - i;
  }
  return 0;
}

void print_name(std::ostream& os, const unitig_list& u) {
  for (size_t i = 0; i < u.size(); ++i) {
    if (i) os << '_';
    os << unitig_id(u[i]) << (unitig_rev(u[i]) ? 'R' : 'F');
  }
}

// union_find.cc:6-23
void UnionFind::reset(int n) {
  parent.resize(n);
  rank.assign(n, 0);
  for (int i = 0; i < n; ++i) parent[i] = i;
}
int UnionFind::root(int s) {
  int r = s;
  while (parent[r] != r) r = parent[r];
  while (parent[s] != r) { const int n = parent[s]; parent[s] = r; s = n; }
  return r;
}
void UnionFind::unite(int a, int b) {
  const int r1 = root(a), r2 = root(b);
  if (rank[r1] > rank[r2]) parent[r2] = r1;
  else if (rank[r1] < rank[r2]) parent[r1] = r2;
  else if (r1 != r2) { parent[r2] = r1; ++rank[r1]; }
}

int ReadGraph::ulen(uint32_t id) const {  // unitigs_lengths[id] (out of range: 0, the reference reads past the end)
  const auto& L = *p_.unitig_lengths;
  return id < L.size() ? L[id] : 0;
}

static int32_t info_at(const Coord& c, bool bases, int i) {  // kmers_info / bases_info [i] (missing: 0)
  if (i < 0 || (uint32_t)i >= c.n_info) return 0;
  return bases ? c.bases_info[i] : c.kmers_info[i];
}

// overlap_graph::traverse (overlap_graph.cc:7-59).  Same visit order, tests and
// early break as the reference; the per-pair sums over the overlapping unitigs
// (u_overlap_len, common_overlap) come from per-node prefix sums computed once
// per read, and the sorted nodes' implied positions sit in one array.  (C2
// reads carry ~560 records and ~12k overlapping pairs each.)
void ReadGraph::traverse(std::ostream* dot) {
  const auto& coords = *coords_;
  const double play = p_.overlap_play;
  const unsigned k = p_.k_len;
  const size_t n = sort_nodes_.size();
  // prefix sums per node j over its name's unitigs u < m:
  //   pul[m] = sum ulen(unitig u), pco[m] = sum info[2u] - sum_{u >= 1} info[2u - 1]
  // (int arithmetic as in the reference's loop, wrapping instead of overflowing)
  pre_off_.resize(coords.size() + 1);
  pre_off_[0] = 0;
  for (size_t j = 0; j < coords.size(); ++j) pre_off_[j + 1] = pre_off_[j] + coords[j].name->size() + 1;
  pul_.resize(pre_off_.back());
  pco_.resize(pre_off_.back());
  for (size_t j = 0; j < coords.size(); ++j) {
    const Coord& cj = coords[j];
    const unitig_list& nm = *cj.name;
    uint32_t* ul = &pul_[pre_off_[j]];
    uint32_t* co = &pco_[pre_off_[j]];
    ul[0] = co[0] = 0;
    for (size_t u = 0; u < nm.size(); ++u) {
      ul[u + 1] = ul[u] + (uint32_t)ulen(unitig_id(nm[u]));
      co[u + 1] = co[u] + (uint32_t)info_at(cj, p_.maximize_bases, 2 * (int)u) -
                  (u > 0 ? (uint32_t)info_at(cj, p_.maximize_bases, 2 * (int)u - 1) : 0u);
    }
  }
  sorted_.resize(n);
  state_.resize(n);
  for (size_t i = 0; i < n; ++i) {
    const int it = sort_nodes_[i];
    const unitig_list& nm = *coords[it].name;
    sorted_[i] = SortedNode{nodes_[it].imp_s, nodes_[it].imp_e, coords[it].avg_err, nm.data(),
                            &pul_[pre_off_[it]], &pco_[pre_off_[it]], it, (int)nm.size(),
                            nm.empty() ? 0u : nm[0],
                            p_.maximize_bases ? coords[it].sr_cover : (unsigned)coords[it].nb_mers};
    const Node& d = nodes_[it];
    state_[i] = PathState{d.imp_s, d.lpath, d.lstart, d.lprev, d.lunitigs, d.start_node, d.end_node};
  }
  for (size_t i = 0; i != n; ++i) {
    const SortedNode& si_ = sorted_[i];
    const int it_i = si_.idx;
    PathState& ni = state_[i];
    const double imp_e_i = si_.imp_e;
    if (imp_e_i >= (double)coords[it_i].rl) continue;  // hanging off the 3' end
    const int sa = si_.nsz;
    const unitig_t* a = si_.name;
    const double err_i = si_.avg_err;
    for (size_t j = i + 1; j != n; ++j) {
      const SortedNode& sj = sorted_[j];
      if (sj.imp_s <= 1) continue;               // hanging off the 5' end
      if (imp_e_i > sj.imp_e + 31) continue;     // not advancing
      const double position_len = imp_e_i - sj.imp_s;
      const double error1 = err_i + sj.avg_err;
      const double error = p_.nb_errors * error1;
      if (position_len * play + error < k) break;  // implied overlap shorter than a k-mer
      // name_overlap(name_i, name_j) on the cached first unitig and size of name j
      const int sb = sj.nsz;
      if (sa < 2 || sb < 2) continue;
      int nb_u_overlap = 0;
      for (int t = std::max(sa - sb + 1, 1); t < sa; ++t) {
        if (a[t] != sj.u0) continue;
        int q = t + 1;
        while (q < sa && a[q] == sj.name[q - t]) ++q;
        if (q == sa) { nb_u_overlap = sa - t; break; }
      }
      if (!nb_u_overlap) continue;
      // the same super-read (name_i == name_j; equal names have equal sizes)
      if (sb == sa && (sj.name == a || std::equal(a, a + sa, sj.name))) continue;
      const int it_j = sj.idx;
      // nb_u_overlap <= |name_j|, so every unitig of the sums is in name j
      int u_overlap_len = (int)sj.pul[nb_u_overlap];
      const int common_overlap = (int)sj.pco[nb_u_overlap];
      u_overlap_len = (int)((unsigned)u_overlap_len - (unsigned)(nb_u_overlap - 1) * (k - 1));
      if (u_overlap_len > play * position_len + error || position_len > play * (u_overlap_len + error)) continue;
      // an overlap between nodes i and j
      PathState& nj = state_[j];
      ni.end_node = false;
      nj.start_node = false;
      // (nodes already under one parent are already one set: unite would change no root)
      if (uf_.parent[it_i] != uf_.parent[it_j]) uf_.unite(it_i, it_j);
      const int nlpath = (int)((unsigned)ni.lpath + sj.lp_add - (unsigned)common_overlap);
      // ls_imp_s: the implied start of the node's path start (nodes_[lstart].imp_s, or its own)
      if (nlpath > nj.lpath || (nlpath == nj.lpath && (nj.lstart == -1 || ni.ls_imp_s > nj.ls_imp_s))) {
        nj.lpath = nlpath;
        nj.lstart = ni.lstart == -1 ? it_i : ni.lstart;
        nj.ls_imp_s = ni.ls_imp_s;
        nj.lprev = it_i;
        nj.lunitigs = ni.lunitigs + sb - nb_u_overlap;
      }
      if (dot) *dot << "n" << it_i << " -> n" << it_j << " [tooltip=\"...\", label=\"" << common_overlap << "\"];\n";
    }
  }
  for (size_t i = 0; i < n; ++i) {
    Node& d = nodes_[sorted_[i].idx];
    const PathState& ps = state_[i];
    d.lpath = ps.lpath; d.lstart = ps.lstart; d.lprev = ps.lprev; d.lunitigs = ps.lunitigs;
    d.start_node = ps.start_node; d.end_node = ps.end_node;
  }
}

// mega_read_info::make (overlap_graph.cc:61-76)
MegaRead ReadGraph::make(int i) const {
  const auto& coords = *coords_;
  MegaRead r;
  r.start_node = nodes_[i].lstart == -1 ? i : nodes_[i].lstart;
  r.end_node = i;
  r.start_unitig = 0;
  r.nb_unitigs = nodes_[r.end_node].lunitigs;
  r.end_unitig = (int)(coords[r.end_node].n_info / 2);
  r.imp_s = coords[r.start_node].stretch + coords[r.start_node].offset;
  r.imp_e = coords[r.end_node].stretch * (double)coords[r.end_node].ql + coords[r.end_node].offset;
  r.tiling_start = coords[r.start_node].rs;
  r.tiling_end = coords[i].re;
  r.start_offset = 0;
  r.end_offset = 0;
  r.density = 0;
  return r;
}

// overlap_graph::trim_match (overlap_graph.cc:78-114)
void ReadGraph::trim_match(MegaRead& mr) const {
  const auto& coords = *coords_;
  const unsigned k = p_.k_len;
  if (nodes_[mr.start_node].imp_s < 1) {
    const Coord& c = coords[mr.start_node];
    int offset = 0;
    for (mr.start_unitig = 0; mr.start_unitig < (int)c.n_info; mr.start_unitig += 2) {
      if (c.kmers_info[mr.start_unitig]) break;
      const int u = mr.start_unitig / 2;
      offset += ulen(u < (int)c.name->size() ? unitig_id((*c.name)[u]) : INVALID_ID);
    }
    mr.start_unitig /= 2;
    mr.nb_unitigs -= mr.start_unitig;
    offset = (int)((unsigned)offset - (k - 1) * (unsigned)mr.start_unitig);
    mr.start_offset = offset;
    mr.imp_s = c.stretch * (offset + 1) + c.offset;
  }
  {
    const Coord& c = coords[mr.end_node];
    if (nodes_[mr.end_node].imp_e > (double)c.ql) {
      int offset = 0;
      for (mr.end_unitig = (int)c.n_info - 1; mr.end_unitig >= 0; mr.end_unitig -= 2) {
        if (c.kmers_info[mr.end_unitig]) break;
        const int u = mr.end_unitig / 2;
        offset += ulen(u < (int)c.name->size() ? unitig_id((*c.name)[u]) : INVALID_ID);
      }
      mr.end_unitig /= 2;
      const int removed = (int)(c.n_info / 2) - mr.end_unitig;
      mr.nb_unitigs -= removed;
      offset = (int)((unsigned)offset - (k - 1) * (unsigned)removed);
      mr.end_offset = offset;
      mr.imp_e = c.stretch * (double)(c.ql - (uint64_t)(int64_t)offset) + c.offset;  // size_t arithmetic upstream
    }
  }
}

// overlap_graph::mega_reads_per_comp (overlap_graph.cc:116-161).  The reference
// keys components by the union-find root's address inside the node vector, so
// a std::map iterates them in root-index order: comp_ is kept sorted by root.
void ReadGraph::components(std::ostream* dot) {
  const auto& coords = *coords_;
  const int n = (int)coords.size();
  comp_.clear();
  for (int i = 0; i < n; ++i) {
    const Node& node = nodes_[i];
    MegaRead mr = make(i);
    if (p_.trim != Trim::NONE) trim_match(mr);
    const double imp_len = std::min((double)coords[0].rl + 0.5, mr.tiling_end) - std::max(0.5, mr.tiling_start);
    mr.density = (double)node.lpath / imp_len;
    if (dot) {
      const char* color = node.start_node ? ", color=\"blue\"" : node.end_node ? ", color=\"green\"" : "";
      const Coord& ci = coords[i];
      *dot << std::fixed << "n" << i << " [label=\"" << i << " L" << ci.ql << " #" << ci.nb_mers << "\\nP(" << ci.rs
           << ',' << ci.re << ") S(" << ci.qs << ',' << ci.qe << ")" << "\\nI(" << std::setprecision(2) << node.imp_s
           << ',' << node.imp_e << ")" << "\\nLP #" << node.lpath << " L" << std::setprecision(1) << imp_len << " d"
           << std::setprecision(2) << mr.density << "\"" << color << "];\n";
    }
    if (!node.end_node || mr.density < p_.min_density || (mr.tiling_end - mr.tiling_start) < p_.min_len) continue;
    const int root = dev_ ? (int)dev_[i].root : uf_.root(i);
    auto it = std::lower_bound(comp_.begin(), comp_.end(), root,
                               [](const std::pair<int, MegaRead>& a, int r) { return a.first < r; });
    if (it == comp_.end() || it->first != root) {
      comp_.insert(it, std::make_pair(root, mr));
    } else {
      const Node& on = nodes_[it->second.end_node];  // current terminal node of the longest path
      if (node.lpath > on.lpath || (node.lpath == on.lpath && mr.density > it->second.density)) it->second = mr;
    }
  }
  mega_reads_.clear();
  sort_tiling_.clear();
  for (const auto& c : comp_) {
    sort_tiling_.push_back((int)mega_reads_.size());
    mega_reads_.push_back(&c.second);
  }
}

namespace {
// boost::icl::interval_set<double> of right-open intervals: disjoint, sorted,
// touching intervals joined (what tile_greedy's `covered` relies on)
struct IntervalSet {
  std::vector<std::pair<double, double>> v;
  void add(double lo, double hi) {
    if (!(lo < hi)) return;  // empty
    auto it = std::lower_bound(v.begin(), v.end(), lo, [](const std::pair<double, double>& x, double l) {
      return x.second < l;  // intervals ending before lo (not touching) stay
    });
    auto e = it;
    while (e != v.end() && e->first <= hi) {
      lo = std::min(lo, e->first);
      hi = std::max(hi, e->second);
      ++e;
    }
    it = v.erase(it, e);
    v.insert(it, std::make_pair(lo, hi));
  }
  // does any piece of (this & [lo, hi)) have length >= m?
  bool large_overlap(double lo, double hi, double m) const {
    for (const auto& x : v) {
      const double a = std::max(lo, x.first), b = std::min(hi, x.second);
      if (a < b && b - a >= m) return true;
    }
    return false;
  }
};
inline double ilen(double lo, double hi) { return hi > lo ? hi - lo : 0.0; }
}  // namespace

// overlap_graph::tile_greedy (overlap_graph.cc:163-197)
int ReadGraph::tile_greedy(const std::vector<int>& order, std::vector<int>& res) const {
  IntervalSet covered;
  std::vector<std::pair<double, double>> placed;
  int score = 0;
  const double play = p_.overlap_play;
  for (const int it_i : order) {
    const MegaRead& mr = *mega_reads_[it_i];
    const double lo = mr.tiling_start, hi = mr.tiling_end;
    const double max_overlap = std::max(p_.k_len * play, ilen(lo, hi) * (play - 0.9));
    if (covered.large_overlap(lo, hi, max_overlap)) continue;
    bool contains = false;
    for (const auto& x : placed)  // boost::icl::contains(x, pos): an empty pos is contained
      if (!(lo < hi) || (x.first < x.second && x.first <= lo && hi <= x.second)) { contains = true; break; }
    if (contains) continue;
    covered.add(lo, hi);
    placed.emplace_back(lo, hi);
    score += nodes_[it_i].lpath;  // (sic: indexed by mega-read, overlap_graph.cc:191)
    res.push_back(it_i);
  }
  return score;
}

// overlap_graph::tile_maximal (overlap_graph.cc:199-252)
int ReadGraph::tile_maximal(const std::vector<int>& order, std::vector<int>& res) const {
  struct Info { int score; double pos; int node, previous, length; };
  std::vector<Info> info;
  info.reserve(order.size());
  auto it = order.cbegin();
  if (it == order.cend()) return 0;
  info.push_back({nodes_[mega_reads_[*it]->end_node].lpath, mega_reads_[*it]->tiling_end, *it, -1, 1});
  for (++it; it != order.cend(); ++it) {
    const double lpath_start = mega_reads_[*it]->tiling_start;
    const double key = std::min(lpath_start + p_.k_len * p_.overlap_play, mega_reads_[*it]->tiling_end);
    const auto lb = std::upper_bound(info.cbegin(), info.cend(), key, [](double x, const Info& y) { return x < y.pos; });
    int i = (int)(lb - info.cbegin()) - 1;
    while (i >= 0 && mega_reads_[info[i].node]->tiling_start >= lpath_start) i = info[i].previous;
    const int nscore = (i >= 0 ? info[i].score : 0) + nodes_[mega_reads_[*it]->end_node].lpath;
    if (nscore > info.back().score)
      info.push_back({nscore, mega_reads_[*it]->tiling_end, *it, i, (i >= 0 ? info[i].length : 0) + 1});
  }
  res.resize(info.back().length);
  int ptr = (int)info.size() - 1;
  for (auto r = res.rbegin(); r != res.rend(); ++r) {
    *r = info[ptr].node;
    ptr = info[ptr].previous;
  }
  return info.back().score;
}

// super_read_name::print_sequence (super_read_name.cc:114-137)
void ReadGraph::print_sequence(std::ostream& os, const unitig_list& u, int start, int nb) const {
  const auto& seqs = *p_.unitig_sequences;
  const size_t b = std::min<size_t>((size_t)start, u.size());
  const size_t e = nb == -1 ? u.size() : std::min<size_t>((size_t)start + (size_t)nb, u.size());
  for (size_t i = b; i < e; ++i) {
    const uint32_t id = unitig_id(u[i]);
    if (id >= seqs.size()) throw std::out_of_range("unitig id beyond the unitig sequences");
    const std::string& s = seqs[id];
    const size_t off = i == b ? 0 : (size_t)p_.k_len - 1;
    if (off >= s.size()) continue;
    if (unitig_rev(u[i])) {
      for (auto c = s.crbegin() + off; c != s.crend(); ++c) {
        switch (*c) {
          case 'a': case 'A': os << 'T'; break;
          case 'c': case 'C': os << 'G'; break;
          case 'g': case 'G': os << 'C'; break;
          case 't': case 'T': os << 'A'; break;
          default: os << 'N';
        }
      }
    } else {
      os << (s.c_str() + off);
    }
  }
}

// overlap_graph::print_mega_reads (overlap_graph.cc:254-299)
void ReadGraph::print(std::ostream& out, const std::vector<int>& order, std::ostream* dot) const {
  const auto& coords = *coords_;
  const unsigned k = p_.k_len;
  for (const int cmr : order) {
    const MegaRead& mr = *mega_reads_[cmr];
    const Node& end_n = nodes_[mr.end_node];
    const Coord& end_c = coords[mr.end_node];
    const Coord& start_c = coords[mr.start_node];
    // the path's unitigs, prepended from the end node back along lprev
    // (super_read_name::prepend, super_read_name.cc:29-36)
    unitig_list sr((size_t)std::max(0, end_n.lunitigs), 0u);
    auto prepend = [&](size_t offset, const unitig_list& rhs, size_t first, size_t last) -> size_t {
      if (first > last || first >= rhs.size()) return offset;
      const size_t to_copy = std::min(last, rhs.size() - 1) - first + 1;
      if (to_copy > offset) return offset;
      const size_t no = offset - to_copy;
      std::copy_n(rhs.begin() + first, to_copy, sr.begin() + no);
      return no;
    };
    size_t offset = prepend(sr.size(), *end_c.name, 0, end_c.name->size() - 1);
    int node_j = mr.end_node, node_i = end_n.lprev;
    while (node_i >= 0) {
      const size_t overlap = (size_t)nodes_[node_i].lunitigs + coords[node_j].name->size() - (size_t)nodes_[node_j].lunitigs;
      const size_t last = coords[node_i].name->size() - 1 - overlap;
      offset = prepend(offset, *coords[node_i].name, 0, last);
      if (dot) *dot << "n" << node_i << " -> n" << node_j << " [color=\"red\"];\n";
      node_j = node_i;
      node_i = nodes_[node_i].lprev;
    }
    int sr_len = 0;
    for (int i = mr.start_unitig; i < mr.start_unitig + mr.nb_unitigs; ++i)
      sr_len += ulen(i >= 0 && (size_t)i < sr.size() ? unitig_id(sr[i]) : INVALID_ID);
    sr_len = (int)((unsigned)sr_len - (unsigned)(mr.nb_unitigs - 1) * (k - 1));
    // (sr_len + end_offset - (ql - qe)) is size_t arithmetic upstream
    const uint64_t qend = (uint64_t)(int64_t)(sr_len + mr.end_offset) - (end_c.ql - (uint64_t)(int64_t)end_c.qe);
    out << std::fixed << std::setprecision(2) << mr.imp_s << ' ' << mr.imp_e << ' ' << start_c.rs << ' ' << end_c.re
        << ' ' << (start_c.qs - mr.start_offset) << ' ' << qend << ' ' << end_n.lpath << ' ' << std::setprecision(4)
        << mr.density << ' ';
    print_name(out, sr);
    out << ' ' << sr_len;
    if (p_.unitig_sequences) {
      out << ' ';
      print_sequence(out, sr, mr.start_unitig, mr.nb_unitigs);
    }
    out << '\n';
  }
}

void ReadGraph::print_device(std::ostream& out, const std::string& pb_name, const pbgpu_mega_read* m, uint64_t n,
                             const uint32_t* units) const {
  if (!n) return;
  out << '>' << pb_name << '\n';
  for (uint64_t t = 0; t < n; ++t) {
    const pbgpu_mega_read& mr = m[t];
    const unitig_list sr(units + mr.unit_offset, units + mr.unit_offset + mr.n_units);
    out << std::fixed << std::setprecision(2) << mr.imp_s << ' ' << mr.imp_e << ' ' << mr.rs << ' ' << mr.re << ' '
        << mr.qs << ' ' << mr.qend << ' ' << mr.lpath << ' ' << std::setprecision(4) << mr.density << ' ';
    print_name(out, sr);
    out << ' ' << mr.sr_len;
    if (p_.unitig_sequences) {
      out << ' ';
      print_sequence(out, sr, mr.start_unitig, mr.nb_unitigs);
    }
    out << '\n';
  }
}

// create_mega_reads.cc:79-89 for one read.  The reference's std::sort calls
// leave ties in an unspecified order; here every sort is stable (ties keep the
// input order: records in (rs, re, ql, sr_index, emit) order).
void ReadGraph::process(const std::vector<Coord>& coords, const std::string& pb_name, std::ostream& out,
                        std::ostream* dot, const pbgpu_graph_node* dev) {
  coords_ = &coords;
  const int n = (int)coords.size();
  dev_ = dev && n && !dot && !(dev[0].flags & PBGPU_GRAPH_HOST) ? dev : nullptr;
  if (dev_) {  // traversed on the device: its node state, the host's implied positions
    nodes_.resize(n);
    for (int i = 0; i < n; ++i) {
      const Coord& c = coords[i];
      const pbgpu_graph_node& g = dev_[i];
      Node& d = nodes_[i];
      d.start_node = (g.flags & PBGPU_GRAPH_START) != 0;
      d.end_node = (g.flags & PBGPU_GRAPH_END) != 0;
      d.imp_s = c.stretch + c.offset;
      d.imp_e = c.stretch * (double)c.ql + c.offset;
      d.lstart = g.lstart; d.lprev = g.lprev; d.lpath = g.lpath; d.lunitigs = g.lunitigs;
    }
  } else {
  // overlap_graph::thread::reset (overlap_graph.hpp:177-196) + node_info::reset (:24-34)
  nodes_.resize(n);
  sort_nodes_.resize(n);
  uf_.reset(n);
  for (int i = 0; i < n; ++i) {
    const Coord& c = coords[i];
    Node& d = nodes_[i];
    d.start_node = d.end_node = true;
    d.imp_s = c.stretch + c.offset;
    d.imp_e = c.stretch * (double)c.ql + c.offset;
    d.lstart = d.lprev = -1;
    d.lpath = p_.maximize_bases ? (int)c.sr_cover : c.nb_mers;
    d.lunitigs = (int)c.name->size();
    sort_nodes_[i] = i;
  }
  std::stable_sort(sort_nodes_.begin(), sort_nodes_.end(), [&](int i, int j) {
    return nodes_[i].imp_s < nodes_[j].imp_s || (nodes_[i].imp_s == nodes_[j].imp_s && nodes_[i].imp_e < nodes_[j].imp_e);
  });
  if (dot) {
    *dot << "digraph \"" << pb_name << "\" {\nnode [fontsize=\"10\"];\n";
    for (const int it : sort_nodes_) {
      *dot << "n" << it << "[tooltip=\"";
      print_name(*dot, *coords[it].name);
      *dot << "\"];\n";
    }
  }
  traverse(dot);
  }
  components(dot);  // term_node_per_comp
  switch (p_.tiling) {
    case Tiling::GREEDY:
    case Tiling::WEIGHTED: {
      if (p_.tiling == Tiling::GREEDY) {
        std::stable_sort(sort_tiling_.begin(), sort_tiling_.end(), [&](int i, int j) {
          return nodes_[mega_reads_[j]->end_node].lpath < nodes_[mega_reads_[i]->end_node].lpath;
        });
      } else {
        if (mega_reads_.size() > weights_.size()) weights_.resize(mega_reads_.size());
        for (const int i : sort_tiling_)
          weights_[i] = mega_reads_[i]->density * mega_reads_[i]->density *
                        (coords[mega_reads_[i]->end_node].re - coords[mega_reads_[i]->start_node].rs + 1);
        std::stable_sort(sort_tiling_.begin(), sort_tiling_.end(), [&](int i, int j) { return weights_[j] < weights_[i]; });
      }
      tiled_mr_.clear();
      tile_greedy(sort_tiling_, tiled_mr_);
      break;
    }
    case Tiling::MAXIMAL:
      // (with no candidate the reference leaves the previous read's tiling in place;
      // nothing is printed then, so it is cleared here)
      if (sort_tiling_.empty()) tiled_mr_.clear();
      std::stable_sort(sort_tiling_.begin(), sort_tiling_.end(),
                [&](int i, int j) { return mega_reads_[i]->tiling_end < mega_reads_[j]->tiling_end; });
      tile_maximal(sort_tiling_, tiled_mr_);
      break;
    case Tiling::NONE:
      break;
  }
  if (p_.tiling != Tiling::NONE)
    std::stable_sort(tiled_mr_.begin(), tiled_mr_.end(), [&](int i, int j) {
      const double si = mega_reads_[i]->imp_s, sj = mega_reads_[j]->imp_s;
      return si < sj || (si == sj && mega_reads_[i]->imp_e < mega_reads_[j]->imp_e);
    });
  // overlap_graph::thread::print_mega_reads (overlap_graph.hpp:253-262)
  if (!comp_.empty()) {
    out << '>' << pb_name << '\n';
    print(out, tiled_mr_.empty() ? sort_tiling_ : tiled_mr_, dot);
    if (dot) *dot << "}\n";
  }
}

}  // namespace megareads
