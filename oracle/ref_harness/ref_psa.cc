// TEST INFRASTRUCTURE (our code). Builds the reference's PSA
// (src_psa/psa.hpp:130-153, mer_sa_imp.hpp) over a concatenated text made
// exactly as sequence_psa::append_fasta does (superread_parser.cc:12-46:
// per-line compact_dna::copy_from_str, no separators) and answers exact
// searches the way sequence_psa::find_pos_size does (superread_parser.hpp:183-192).
// argv: fasta min_size max_size threads ; stdin: one query pattern per line.
// Output per query: "count pos1 pos2 ..." in SA order (the reference's hit order).
// unistd.h first: psa.hpp pulls in boost yield.hpp, which #defines `fork`
// (the reference TUs include it earlier through Jellyfish headers).
#include <unistd.h>
#include <thread>
#include <cassert>
#include <cstring>
#include <fstream>
#include <iostream>
#include <mutex>
#include <string>
#include <vector>
#include <src_psa/global_timer.hpp>
#include <src_psa/compact_dna.hpp>
#include <src_psa/psa.hpp>

int main(int argc, char* argv[]) {
  if(argc != 5) { std::cerr << "usage: fasta min max threads\n"; return 1; }
  std::ifstream is(argv[1]);
  std::vector<uint64_t> seq;
  size_t off = 0;
  std::string line;
  while(std::getline(is, line)) {
    if(!line.empty() && line[0] == '>') continue;
    if(seq.size() * sizeof(uint64_t) * 4 < line.size() + off)
      seq.resize(std::max(1 + (size_t)(line.size() + off) / (sizeof(uint64_t) * 4), seq.size() * 2));
    compact_dna::copy_from_str(compact_dna::iterator(seq.data(), 2, 0) + off, line);
    off += line.size();
  }
  const unsigned min_size = std::atoi(argv[2]), max_size = std::atoi(argv[3]), threads = std::atoi(argv[4]);
  PSA<compact_dna::const_iterator> psa(compact_dna::const_iterator_at(seq.data()), off, min_size, max_size, threads);
  std::cerr << "check " << psa.check() << '\n';
  while(std::getline(std::cin, line)) {
    auto r = psa.search(line.c_str(), line.size());
    std::cout << r.first;
    for(uint64_t i = 0; i < r.first; ++i) std::cout << ' ' << psa[r.second + i];
    std::cout << '\n';
  }
  return 0;
}
