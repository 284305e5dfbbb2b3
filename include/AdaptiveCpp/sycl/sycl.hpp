// AdaptiveCpp/sycl/sycl.hpp — the include name the reference's driver uses
// (test/Tester.cpp:3,7: `#include <AdaptiveCpp/sycl/sycl.hpp>` and
// `using namespace acpp::sycl;`). This is NOT a SYCL implementation: it only
// provides the queue / event / exception handles the drop-in CG API passes
// around (src/CG.hpp:61,590). A queue is a shared handle to one libcgx
// context: one gfx950 device and one in-order HIP stream (include/cgx.h).
// Nothing here declares CG, Timer or read_file, so Tester.cpp's two using-
// directives stay unambiguous.
#ifndef CGX_ACPP_SYCL_HPP
#define CGX_ACPP_SYCL_HPP

#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>

#include "../../cgx.h"

namespace acpp {
namespace sycl {

class exception : public std::runtime_error {
 public:
  explicit exception(const std::string &what) : std::runtime_error(what) {}
};

namespace detail {
inline void check(int rc, const char *what) {
  if (rc != CGX_OK) throw exception(std::string(what) + ": " + cgx_last_error());
}
struct CtxDeleter {
  void operator()(cgx_ctx *c) const {
    if (c) cgx_destroy(c);
  }
};
}  // namespace detail

// The default-constructed queue selects device $CGX_DEVICE (default 0), as
// the reference's default queue selects the default device (CG.hpp:72).
class queue {
 public:
  queue() : queue(default_device()) {}
  explicit queue(int device) {
    cgx_ctx *c = nullptr;
    detail::check(cgx_create(device, &c), "cgx_create");
    ctx_ = std::shared_ptr<cgx_ctx>(c, detail::CtxDeleter());
  }
  void wait() { detail::check(cgx_sync(ctx_.get()), "queue::wait"); }
  void wait_and_throw() { wait(); }
  cgx_ctx *native() const { return ctx_.get(); }
  bool operator==(const queue &o) const { return ctx_ == o.ctx_; }

 private:
  static int default_device() {
    const char *e = std::getenv("CGX_DEVICE");
    return e ? std::atoi(e) : 0;
  }
  std::shared_ptr<cgx_ctx> ctx_;
};

// The stream is in order, so an event only marks a point in it.
class event {
 public:
  event() = default;
  explicit event(const queue &q) : q_(std::make_shared<queue>(q)) {}
  void wait() {
    if (q_) q_->wait();
  }

 private:
  std::shared_ptr<queue> q_;
};

}  // namespace sycl
}  // namespace acpp

#endif
