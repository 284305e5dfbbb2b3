#ifndef CG_HPP
#define CG_HPP
/**
 * @file CG.hpp
 * Drop-in for the reference's src/CG.hpp: class CGSolver::CG<DT, Debuglevel>
 * with the same members (cited per member), running on libcgx's gfx950
 * kernels (include/cgx.h). test/Tester.cpp compiles against it unmodified.
 *
 * solve() keeps the reference's iteration semantics: the body
 * runs, then stops if r.r at the START of the body is NaN or its square root
 * is <= improvement; at most N + 1 bodies; improvement 0 runs until r.r
 * underflows (then x is NaN, as in the reference). Instead of 12 submissions
 * and a host drain per iteration (CG.hpp:359-436) it runs three fused kernels
 * per iteration with device-resident scalars and polls the stop flag every
 * few iterations.
 */
#include <AdaptiveCpp/sycl/sycl.hpp>
#include <algorithm>
#include <cassert>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <exception>
#include <iostream>
#include <memory>
#include <ostream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "LinearAlgebraTypes.hpp"
#include "VectorOperations.hpp"

namespace CGSolver {

namespace asycl = acpp::sycl;

namespace detail {
struct CgDeleter {
  void operator()(cgx_cg *c) const {
    if (c) cgx_cg_destroy(c);
  }
};
}  // namespace detail

/**
 * @class CG (CG.hpp:53-601)
 * Set matrix, right-hand side and optional initial guess, solve, extract.
 */
template <typename DT, Debuglevel debug = Debuglevel::None> class CG {
 public:
  using Scalar = ::CGSolver::Scalar<DT>;
  using Matrix = ::CGSolver::Matrix<DT>;
  using Vector = ::CGSolver::Vector<DT>;

  /** :61 — no device memory is allocated yet */
  CG(asycl::queue &queue) : _queue(queue), A(queue), x(_queue), b(_queue) {
    if constexpr (debug == Debuglevel::Verbose) std::clog << "Constructing CG Object\n";
  }

  /** :70-77 — a CG on a default queue */
  static std::unique_ptr<CG> createCG() {
    asycl::queue q;
    std::unique_ptr<CG> cg(new CG(q));
    return cg;
  }

  /** :87-93 — CSR triple from the host */
  void setMatrix(std::vector<DT> &data, std::vector<int> &columns, std::vector<int> &rows) {
    if constexpr (debug == Debuglevel::Verbose) std::clog << "Setting Matrix\n";
    A.init(data, columns, rows);
    _solver.reset();
  }

  /** :102 — a device matrix, moved */
  void setMatrix(Matrix &&M) {
    A = std::forward<Matrix>(M);
    _solver.reset();
  }

  /** :156 */
  int getDimension() const { return this->A.N(); }

  /** :164-170 */
  void setTarget(std::vector<DT> &_data) {
    b.init(_data);
    executeQueue();
  }

  /** :206 */
  void setTarget(Vector &&V) { b = std::forward<Vector>(V); }

  /** :215-219 (sic) — initial guess from the host */
  void setInital(std::vector<DT> &_data) {
    x.init(_data);
    executeQueue();
  }

  /** :235 (empty in the reference) */
  void calculateExpectedStepCount(DT accuracy) {}

  /** :244 — initial guess on the device, moved */
  void setInitial(Vector &&V) { x = std::forward<Vector>(V); }

  /**
   * :255-454 — Solve A x = b.
   * @throw std::runtime_error if b or A is missing (:266-272)
   */
  void solve(DT improvement = static_cast<DT>(0)) {
    if constexpr (debug == Debuglevel::Verbose) std::clog << "Solving System\n";
    // :260-261 (its constructor prints the work-group line under Verbose)
    VectorOperations<DT, debug> vecops(this->_queue);
    vecops.setVectorSize(A.N());
    if (this->b.data() == nullptr) throw std::runtime_error("No right hand side to solve for");
    if (this->A.columns().get() == nullptr) throw std::runtime_error("No Matrix given");
    const auto N = A.N();
    if (x.ptr() == nullptr) {
      if constexpr (debug == Debuglevel::Verbose) std::clog << "x init empty" << std::endl;
      x.init_empty(N);
    }
    cgx_cg *s = solver();  // the solver's vectors and scalars (:276-302)
    if constexpr (debug == Debuglevel::Verbose) std::clog << "Prepared Memory" << std::endl;
    // :314-341: r = b - A x, p = r, rxr = r.r
    check(cgx_cg_begin(s, b.ptr(), x.ptr(), (double)improvement, _max_iterations), "solve");
    if constexpr (debug == Debuglevel::Verbose) {
      check(cgx_sync(_queue.native()), "solve");
      std::clog << "Init done" << std::endl;
      std::clog << "Entering Loop" << std::endl;
    }
    // :359-436: at most N + 1 bodies (or the extension's cap)
    int64_t cap = static_cast<int64_t>(N) + 1;
    if (_max_iterations >= 0) cap = std::min<int64_t>(cap, std::max<int64_t>(_max_iterations, 1));
    int64_t bodies = 0;
    int stopped = 0;
    check(cgx_cg_run(s, cap, &bodies, &stopped), "solve");
    double rxr = 0;
    check(cgx_cg_rxr(s, &rxr), "solve");  // :437-440
    _iterations = bodies;
    _final_rxr = rxr;
    this->is_solved = true;
    if constexpr (debug == Debuglevel::Verbose) {
      // :428-434: the progress line the reference writes after every body
      // whose counter is a multiple of 100, in the same order and format
      // (written here once the device loop has finished: the loop does not
      // return to the host per body)
      for (int64_t counter = 0; counter < bodies; counter += 100) {
        std::clog << "\r\033[2K";
        std::clog << ((static_cast<double>(counter) / N) * 100) << "%";
        std::flush(std::clog);
      }
      std::clog << std::endl;  // :450-453
      std::clog << "Finished solving" << std::endl;
    }
  }

  /** :463-515 — |sum (b - A x)^2 / sum x^2| (squared norms) */
  DT accuracy() {
    if constexpr (debug == Debuglevel::Verbose) std::clog << "Calculating accuracy" << std::endl;
    double out = 0;
    check(cgx_accuracy(_queue.native(), A.schedule(), b.ptr(), x.ptr(), &out), "accuracy");
    return static_cast<DT>(out);
  }

  /** :517-523 */
  std::vector<DT> extract() {
    std::vector<DT> ret(A.N());
    check(cgx_d2h(_queue.native(), ret.data(), x.ptr(), A.N() * sizeof(DT)), "extract");
    return ret;
  }

  /** :529-532 — resizes `result` to N */
  void extractTo(std::vector<DT> &result) {
    result.resize(A.N());
    check(cgx_d2h(_queue.native(), result.data(), x.ptr(), A.N() * sizeof(DT)), "extractTo");
  }

  /** :555-558 */
  std::size_t memoryFootprint() const {
    return (2 * this->A.NNZ() + (4 * this->A.N())) * sizeof(DT) +
           (2 * this->A.N() * sizeof(int));
  }

  // ---- extensions (not in the reference) -------------------------------
  /** loop bodies executed by the last solve() */
  long long iterations() const { return _iterations; }
  /** r.r after the last body (the value the reference reads back, :437-438) */
  double finalResidualSquared() const { return _final_rxr; }
  /** cap the loop bodies (< 0: the reference cap N + 1) */
  void setMaxIterations(long long m) { _max_iterations = m; }

 private:
  void executeQueue() {
    try {
      this->_queue.wait_and_throw();
    } catch (asycl::exception &e) {
      std::cerr << "Caught Sycl Exception " << e.what() << std::endl;
      throw e;
    } catch (std::exception &e) {
      std::cerr << "Caught Exception " << e.what() << std::endl;
      throw e;
    }
  }

  static void check(int rc, const char *what) { asycl::detail::check(rc, what); }

  cgx_cg *solver() {
    cgx_csr *sched = A.schedule();
    if (!_solver || _solver_for != sched) {
      cgx_cg *c = nullptr;
      check(cgx_cg_create(_queue.native(), sched, &c), "cgx_cg_create");
      _solver = std::shared_ptr<cgx_cg>(c, detail::CgDeleter());
      _solver_for = sched;
    }
    return _solver.get();
  }

  asycl::queue _queue;
  bool is_solved = false;
  Matrix A;
  Vector x;
  Vector b;
  std::shared_ptr<cgx_cg> _solver;
  cgx_csr *_solver_for = nullptr;
  long long _iterations = 0;
  double _final_rxr = 0;
  long long _max_iterations = -1;
};

};  // namespace CGSolver

#endif /*CG_HPP */
