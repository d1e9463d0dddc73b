// TEST INFRASTRUCTURE (our code). Drives the reference's own
// src_lis/lis_align.hpp (lis_align::indices, lis_align.hpp:207-214, the
// overload off_lis::do_LIS uses, pb_aligner.hpp:42-46) on cases read from
// stdin:  "N W mer_kind a b C seq_kind seq_a" then N "first second" pairs.
// mer_kind/seq_kind 0 = affine_capped / linear, 1 = accept_all.
// Prints the LIS indices, one case per line.
#include <iostream>
#include <cassert>
#include <cstring>
#include <mutex>
#include <src_lis/lis_align.hpp>

int main() {
  size_t N, W; int mk, sk; double a, b, C, sa;
  while(std::cin >> N >> W >> mk >> a >> b >> C >> sk >> sa) {
    std::vector<std::pair<int, int>> X(N);
    for(auto& x : X) std::cin >> x.first >> x.second;
    std::forward_list<lis_align::element<double>> L;
    std::vector<unsigned int> res;
    lis_align::affine_capped am(a, b, C);
    lis_align::linear ls(sa);
    lis_align::accept_all all;
    unsigned int n;
    if(mk == 0 && sk == 0) n = lis_align::indices(X.cbegin(), X.cend(), L, res, W, am, ls);
    else if(mk == 0)       n = lis_align::indices(X.cbegin(), X.cend(), L, res, W, am, all);
    else if(sk == 0)       n = lis_align::indices(X.cbegin(), X.cend(), L, res, W, all, ls);
    else                   n = lis_align::indices(X.cbegin(), X.cend(), L, res, W, all, all);
    std::cout << n;
    for(unsigned int i = 0; i < n; ++i) std::cout << ' ' << res[i];
    std::cout << '\n';
  }
  return 0;
}
