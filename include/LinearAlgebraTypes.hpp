/**
 * @file LinearAlgebraTypes.hpp
 * Device storage of the drop-in CG API: Matrix (CSR), Vector, Scalar.
 *
 * Interface of the reference's src/LinearAlgebraTypes.hpp (cited per member);
 * storage is HBM owned through shared_ptrs whose deleter returns it to libcgx
 * (the Asycl_deleter of :43-49), so copies share buffers as in the reference.
 * Differences, on purpose:
 *  - Matrix::init re-reads the size on every call (the reference keeps the
 *    first one, :104 — SURVEY §8 quirk Q8);
 *  - Matrix also owns the SpMV row-block schedule libcgx needs (built from the
 *    host row pointer at init).
 */
#ifndef MATRIX_HPP
#define MATRIX_HPP

#include <AdaptiveCpp/sycl/sycl.hpp>
#include <cassert>
#include <cstddef>
#include <memory>
#include <type_traits>
#include <vector>

#include "cgx.h"

namespace CGSolver {

namespace asycl = acpp::sycl;

/** @enum Debuglevel (LinearAlgebraTypes.hpp:26-30) */
enum Debuglevel {
  None,     ///< No output
  Verbose,  ///< All possible outputs
};

namespace detail {
template <class DT> constexpr int dtype() {
  static_assert(std::is_same<DT, double>::value || std::is_same<DT, float>::value,
                "DT must be double or float");
  return std::is_same<DT, float>::value ? CGX_F32 : CGX_F64;
}
template <class T> T *device_alloc(asycl::queue &q, std::size_t n) {
  void *p = nullptr;
  asycl::detail::check(cgx_alloc(q.native(), (n ? n : 1) * sizeof(T), &p), "cgx_alloc");
  return static_cast<T *>(p);
}
struct CsrDeleter {
  void operator()(cgx_csr *c) const {
    if (c) cgx_csr_destroy(c);
  }
};
}  // namespace detail

/** @brief Deallocator functor bound to a queue (LinearAlgebraTypes.hpp:43-49) */
template <class DT> struct Asycl_deleter {
  asycl::queue _q;
  Asycl_deleter(asycl::queue &q) : _q(q) {}
  void operator()(DT *_ptr) { cgx_free(_q.native(), _ptr); }
};

/** @brief CSR matrix on the device (LinearAlgebraTypes.hpp:57-132) */
template <class DT> class Matrix {
 public:
  explicit Matrix(asycl::queue q) : _queue(q), _size(0), _NNZ(0), _N(0) {}
  explicit Matrix(asycl::queue q, const std::size_t size)
      : _queue(q), _size(size), _NNZ(0), _N(size ? size - 1 : 0) {}
  explicit Matrix(asycl::queue q, std::vector<DT> &data, std::vector<int> &cols,
                  std::vector<int> &rows)
      : _queue(q), _size(rows.size()), _NNZ(data.size()), _N(rows.size() - 1) {
    init(data, cols, rows);
    _queue.wait();
  }

  auto data() { return _data; }
  auto data_ptr() { return _data.get(); }
  auto columns() { return _columns; }
  auto columns_ptr() { return _columns.get(); }
  auto rows() { return _rows; }
  auto rows_ptr() { return _rows.get(); }
  auto N() const { return _N; }
  auto NNZ() const { return _NNZ; }

  /** @brief Upload a CSR triple (LinearAlgebraTypes.hpp:101-121) */
  auto init(std::vector<DT> &data, std::vector<int> &cols, std::vector<int> &rows) {
    _size = rows.size();
    _N = _size - 1;
    _NNZ = data.size();
    _data = std::shared_ptr<DT[]>(detail::device_alloc<DT>(_queue, _NNZ),
                                  Asycl_deleter<DT>(_queue));
    _columns = std::shared_ptr<int[]>(detail::device_alloc<int>(_queue, _NNZ),
                                      Asycl_deleter<int>(_queue));
    _rows = std::shared_ptr<int[]>(detail::device_alloc<int>(_queue, _size),
                                   Asycl_deleter<int>(_queue));
    asycl::detail::check(cgx_h2d(_queue.native(), _data.get(), data.data(), _NNZ * sizeof(DT)),
                         "Matrix::init");
    asycl::detail::check(cgx_h2d(_queue.native(), _columns.get(), cols.data(),
                                 _NNZ * sizeof(int)), "Matrix::init");
    asycl::detail::check(cgx_h2d(_queue.native(), _rows.get(), rows.data(),
                                 _size * sizeof(int)), "Matrix::init");
    cgx_csr *c = nullptr;
    asycl::detail::check(cgx_csr_create(_queue.native(), (int64_t)_N, (int64_t)_NNZ,
                                        _rows.get(), _columns.get(), _data.get(),
                                        detail::dtype<DT>(), rows.data(), &c),
                         "cgx_csr_create");
    _csr = std::shared_ptr<cgx_csr>(c, detail::CsrDeleter());
  }

  /** libcgx schedule handle (built by init; lazily for moved-in matrices). */
  cgx_csr *schedule() {
    if (!_csr && _rows) {
      cgx_csr *c = nullptr;
      asycl::detail::check(cgx_csr_create(_queue.native(), (int64_t)_N, (int64_t)_NNZ,
                                          _rows.get(), _columns.get(), _data.get(),
                                          detail::dtype<DT>(), nullptr, &c),
                           "cgx_csr_create");
      _csr = std::shared_ptr<cgx_csr>(c, detail::CsrDeleter());
    }
    return _csr.get();
  }

 private:
  asycl::queue _queue;
  std::size_t _size;
  std::size_t _NNZ;
  std::size_t _N;
  std::shared_ptr<DT[]> _data;
  std::shared_ptr<int[]> _columns;
  std::shared_ptr<int[]> _rows;
  std::shared_ptr<cgx_csr> _csr;
};

/** @brief Vector on the device (LinearAlgebraTypes.hpp:143-203) */
template <class DT> class Vector {
 public:
  explicit Vector(asycl::queue q) : _q(q), _N(0) {}
  explicit Vector(asycl::queue q, const std::size_t N) : _q(q), _N(N) { init_empty(_N); }
  explicit Vector(asycl::queue q, std::vector<DT> &data) : _q(q), _N(0) {
    init(data);
    _q.wait();
  }

  /** @brief allocate and zero (:160-171) */
  asycl::event init_empty(std::size_t size = 0) {
    if (size != 0 && _N == 0) _N = size;
    assert(_N != 0);
    _ptr = std::shared_ptr<DT[]>(detail::device_alloc<DT>(_q, _N), Asycl_deleter<DT>(_q));
    asycl::detail::check(cgx_fill(_q.native(), detail::dtype<DT>(), _ptr.get(), 0.0, _N),
                         "Vector::init_empty");
    return asycl::event(_q);
  }

  /** @brief copy a host vector (:177-183) */
  asycl::event init(std::vector<DT> &data) {
    _ptr = std::shared_ptr<DT[]>(detail::device_alloc<DT>(_q, data.size()),
                                 Asycl_deleter<DT>(_q));
    asycl::detail::check(
        cgx_h2d_async(_q.native(), _ptr.get(), data.data(), data.size() * sizeof(DT)),
        "Vector::init");
    if (_N == 0) _N = data.size();
    return asycl::event(_q);
  }

  auto data() { return _ptr; }
  auto ptr() { return _ptr.get(); }
  auto N() { return _N; }

 private:
  asycl::queue _q;
  std::size_t _N;
  std::shared_ptr<DT[]> _ptr;
};

/** @brief Device-resident scalar (LinearAlgebraTypes.hpp:210-250) */
template <class DT> class Scalar {
 public:
  explicit Scalar(asycl::queue q, DT value_ = static_cast<DT>(0)) : _q(q) { init(value_); }

  auto init(DT value_) {
    value = std::shared_ptr<DT>(detail::device_alloc<DT>(_q, 1), Asycl_deleter<DT>(_q));
    asycl::detail::check(cgx_h2d(_q.native(), value.get(), &value_, sizeof(DT)),
                         "Scalar::init");
  }
  auto ptr() { return value.get(); }
  constexpr operator DT *() const { return value.get(); }
  DT *operator*() { return value.get(); }

 private:
  asycl::queue _q;
  std::shared_ptr<DT> value;
};

}  // namespace CGSolver

#endif /*MATRIX_HPP*/
