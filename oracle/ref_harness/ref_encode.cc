// TEST INFRASTRUCTURE (our code). Encodes lines from stdin with the
// reference's own compact_dna::copy_from_str (src_psa/compact_dna.hpp:109-136),
// each line read with std::getline into a std::string exactly as
// sequence_psa::append_fasta does (superread_parser.cc:24-30), and prints the
// 2-bit codes (0-3) read back through compact_dna::const_iterator.
#include <iostream>
#include <string>
#include <vector>
#include <src_psa/compact_dna.hpp>

int main() {
  std::string line;
  while(std::getline(std::cin, line)) {
    std::vector<uint64_t> mem(line.size() / 32 + 2, 0);
    compact_dna::copy_from_str(compact_dna::iterator(mem.data(), 2, 0), line);
    auto it = compact_dna::const_iterator_at(mem.data());
    for(size_t i = 0; i < line.size(); ++i, ++it) std::cout << (int)*it;
    std::cout << '\n';
  }
  return 0;
}
