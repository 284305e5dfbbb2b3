// solve_poisson.cpp — the drop-in C++ API end to end, written like the
// reference's test/Tester.cpp (same calls, same output line "N NNZ ms
// accuracy") but on a synthetic Dirichlet Poisson matrix built in memory, so
// it needs no input file.
//
//   solve_poisson [dim=3] [n=64] [tol=1e-8]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <vector>

#include "CG.hpp"

using namespace CGSolver;

static void poisson(int dim, int n, std::vector<double> &val, std::vector<int> &col,
                    std::vector<int> &rowptr) {
  const long nz = dim == 3 ? n : 1, nxy = (long)n * n;
  rowptr.assign(1, 0);
  for (long z = 0; z < nz; ++z)
    for (long y = 0; y < n; ++y)
      for (long x = 0; x < n; ++x) {
        const long row = x + n * y + nxy * z;
        auto add = [&](long c, double v) {
          col.push_back((int)c);
          val.push_back(v);
        };
        if (dim == 3 && z > 0) add(row - nxy, -1.0);
        if (y > 0) add(row - n, -1.0);
        if (x > 0) add(row - 1, -1.0);
        add(row, 2.0 * dim);
        if (x < n - 1) add(row + 1, -1.0);
        if (y < n - 1) add(row + n, -1.0);
        if (dim == 3 && z < nz - 1) add(row + nxy, -1.0);
        rowptr.push_back((int)col.size());
      }
}

int main(int argc, char **argv) {
  const int dim = argc > 1 ? std::atoi(argv[1]) : 3;
  const int n = argc > 2 ? std::atoi(argv[2]) : 64;
  const double tol = argc > 3 ? std::atof(argv[3]) : 1e-8;
  std::vector<double> data;
  std::vector<int> cols, rows;
  poisson(dim, n, data, cols, rows);
  std::vector<double> target(rows.size() - 1);
  for (size_t i = 0; i < target.size(); i++) target[i] = i + 1;  // Tester.cpp:29-30

  auto cgp = CG<double, CGSolver::Debuglevel::None>::createCG();
  auto cg = *cgp;  // copyable, as Tester.cpp:38 requires
  cg.setMatrix(data, cols, rows);
  cg.setTarget(target);
  auto t0 = std::chrono::steady_clock::now();
  cg.solve(tol);
  auto t1 = std::chrono::steady_clock::now();
  auto result = cg.extract();
  const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  std::cout << cg.getDimension() << " " << data.size() << " " << ms << " " << cg.accuracy()
            << " iterations=" << cg.iterations() << std::endl;
  return result.size() == target.size() ? 0 : 1;
}
