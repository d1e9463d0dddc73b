// TEST INFRASTRUCTURE (our code). For each stdin line (a super-read name),
// builds the reference's super_read_name (src_jf_aligner/super_read_name.cc),
// and prints: nb_unitigs <TAB> reversed name() <TAB> fwd ids (space separated),
// i.e. what frag_info (frag_info.hpp:22-35) stores as bwd.name / unitigs.
#include <iostream>
#include <string>
#include <src_jf_aligner/super_read_name.hpp>

int main() {
  std::string line;
  while(std::getline(std::cin, line)) {
    super_read_name n(line);
    std::cout << n.size() << '\t' << (n.size() ? n.get_reverse().name() : line) << '\t';
    for(size_t i = 0; i < n.size(); ++i) std::cout << (i ? " " : "") << n.unitig_id(i);
    std::cout << '\n';
  }
  return 0;
}
