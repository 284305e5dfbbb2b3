// Drop-in for the reference's test/mm_reader.cpp: defines
//   std::tuple<std::vector<double>, std::vector<int>, std::vector<int>>
//   read_file(std::string)
// (declared in test/utils.hpp:60) on libcgx's parallel Matrix-Market loader
// (cgx_mm_read, include/cgx.h), with the same semantics (quirks Q1-Q3).
// Link it in place of mm_reader.cpp:
//   g++ -std=c++17 -I<cgx>/include -I<reference>/test <reference>/test/Tester.cpp
//       examples/cgx_read_file.cpp -L<cgx>/conjugategradient_amd -lcgx
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "cgx.h"

std::tuple<std::vector<double>, std::vector<int>, std::vector<int>> read_file(
    std::string filename) {
  int64_t n = 0, nnz = 0;
  int *rp = nullptr, *cl = nullptr;
  double *vl = nullptr;
  if (cgx_mm_read(filename.c_str(), 0, &n, &nnz, &rp, &cl, &vl) != CGX_OK)
    throw std::runtime_error(cgx_last_error());
  std::vector<double> data(vl, vl + nnz);
  std::vector<int> cols(cl, cl + nnz);
  std::vector<int> rows(rp, rp + n + 1);
  cgx_free_host(rp);
  cgx_free_host(cl);
  cgx_free_host(vl);
  return std::make_tuple(std::move(data), std::move(cols), std::move(rows));
}
