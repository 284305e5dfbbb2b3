// mm_ref_wrap.cpp — C entry point around the REFERENCE's own Matrix-Market
// loader (test/mm_reader.cpp:154-171, declared at test/utils.hpp:60), which
// oracle/Makefile compiles unmodified from /root/reference into
// oracle/_ref/libmmref.so. Test infrastructure only: tests/ use it to pin the
// oracle's loader restatement (cg_oracle.c orc_read_mtx) and the product's
// loader bit-exact against the reference.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <tuple>
#include <vector>

std::tuple<std::vector<double>, std::vector<int>, std::vector<int>>
read_file(std::string filename);

extern "C" int mmref_read(const char *path, int64_t *n, int64_t *nnz,
                          int **rowptr, int **col, double **val) {
  auto [data, cols, rows] = read_file(path);
  *n = (int64_t)rows.size() - 1;  // Tester.cpp:27
  *nnz = (int64_t)data.size();
  *rowptr = (int *)std::malloc(rows.size() * sizeof(int));
  *col = (int *)std::malloc((cols.size() ? cols.size() : 1) * sizeof(int));
  *val = (double *)std::malloc((data.size() ? data.size() : 1) * sizeof(double));
  std::memcpy(*rowptr, rows.data(), rows.size() * sizeof(int));
  std::memcpy(*col, cols.data(), cols.size() * sizeof(int));
  std::memcpy(*val, data.data(), data.size() * sizeof(double));
  return 0;
}

extern "C" void mmref_free(void *p) { std::free(p); }
