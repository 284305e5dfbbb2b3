// vecops_check.cpp — every VectorOperations<double> method of the drop-in
// header (include/VectorOperations.hpp; reference src/VectorOperations.hpp:
// 110-466) called the way the reference's callers do, with DEVICE scalars.
// Inputs come from a raw file the test writes; outputs go to a raw file the
// test compares with the oracle (tests/test_cpp_vecops.py).
//
//   vecops_check in.bin out.bin
// in.bin : int64 n, int64 nnz, int32 rowptr[n+1], int32 col[nnz],
//          f64 val[nnz], f64 x[n], f64 y[n], f64 a, f64 b, f64 r0
// out.bin: f64 dot_optimised, dot, dot_trivial, norm (each accumulated onto
//          r0, Q4), then f64 saxpby[n], sambx[n], sapbx[n], spmv[n],
//          sapbx_inplace[n] (Result aliases X)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "VectorOperations.hpp"

using namespace CGSolver;

template <class T> static void rd(FILE *f, T *p, size_t n) {
  if (std::fread(p, sizeof(T), n, f) != n) {
    std::fprintf(stderr, "short read\n");
    std::exit(2);
  }
}

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  FILE *f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  int64_t n = 0, nnz = 0;
  rd(f, &n, 1);
  rd(f, &nnz, 1);
  std::vector<int> rowptr(n + 1), col(nnz);
  std::vector<double> val(nnz), hx(n), hy(n);
  double a = 0, b = 0, r0 = 0;
  rd(f, rowptr.data(), rowptr.size());
  rd(f, col.data(), col.size());
  rd(f, val.data(), val.size());
  rd(f, hx.data(), hx.size());
  rd(f, hy.data(), hy.size());
  rd(f, &a, 1);
  rd(f, &b, 1);
  rd(f, &r0, 1);
  std::fclose(f);

  acpp::sycl::queue q;
  Matrix<double> A(q, val, col, rowptr);
  Vector<double> X(q, hx), Y(q, hy), R(q, (size_t)n), Xc(q, hx);
  Scalar<double> sa(q, a), sb(q, b);
  Scalar<double> d_opt(q, r0), d_raw(q, r0), d_triv(q, r0), d_norm(q, r0);
  VectorOperations<double> ops(q);
  ops.setVectorSize((size_t)n);
  std::vector<double> out;
  auto scalar = [&](Scalar<double> &s) {
    double v = 0;
    acpp::sycl::detail::check(cgx_d2h(q.native(), &v, s.ptr(), sizeof(double)), "d2h");
    out.push_back(v);
  };
  auto vec = [&](Vector<double> &v) {
    std::vector<double> h(n);
    acpp::sycl::detail::check(cgx_d2h(q.native(), h.data(), v.ptr(), n * sizeof(double)), "d2h");
    out.insert(out.end(), h.begin(), h.end());
  };
  ops.dot_product_optimised(X, Y, d_opt.ptr(), {}, (size_t)n);
  ops.dot_product(X.ptr(), Y.ptr(), d_raw.ptr(), {}, (size_t)n);
  ops.dot_product_trivial(X, Y, d_triv, {}, 12345 /* ignored, Q7 */);
  ops.norm(X, d_norm);
  q.wait();
  scalar(d_opt);
  scalar(d_raw);
  scalar(d_triv);
  scalar(d_norm);
  ops.saxpby(X, Y, sa, sb, R, {}, (size_t)n);
  q.wait();
  vec(R);
  ops.sambx(X, Y, sb, R, {}, 7 /* ignored, Q7 */);
  q.wait();
  vec(R);
  ops.sapbx(X, Y, sb, R);
  q.wait();
  vec(R);
  ops.spmv(A, X, R, (size_t)nnz, {}, (size_t)n);
  q.wait();
  vec(R);
  ops.sapbx(Xc, Y, sb, Xc);  // in place (CG.hpp:390 updates x this way)
  q.wait();
  vec(Xc);
  FILE *o = std::fopen(argv[2], "wb");
  if (!o) return 3;
  std::fwrite(out.data(), sizeof(double), out.size(), o);
  std::fclose(o);
  std::printf("vecops ok n=%lld\n", (long long)n);
  return 0;
}
