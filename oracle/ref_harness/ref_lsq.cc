// TEST INFRASTRUCTURE (our code). Drives the reference's own
// src_jf_aligner/least_square_2d.hpp on cases from stdin: "n" then n "x y"
// integer pairs. Prints EX EY EXX EXY VX CXY NB a b as C99 hex floats.
#include <cstdio>
#include <iostream>
#include <vector>
#include <src_jf_aligner/least_square_2d.hpp>

int main() {
  size_t n;
  while(std::cin >> n) {
    least_square_2d ls;
    for(size_t i = 0; i < n; ++i) { long x, y; std::cin >> x >> y; ls.add(x, y); }
    std::printf("%a %a %a %a %a %a %a %a %a\n", ls.EX, ls.EY, ls.EXX, ls.EXY, ls.VX, ls.CXY, ls.NB, ls.a(), ls.b());
  }
  return 0;
}
