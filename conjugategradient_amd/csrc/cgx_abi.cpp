// cgx_abi.cpp — the C ABI of libcgx.so (include/cgx.h): contexts, memory,
// CSR schedules, VectorOperations kernels and the fused CG driver.
//
// The reference drives one SYCL queue and drains it after every iteration
// (src/CG.hpp:425, executeQueue :561-578). Here the iteration scalars live on
// the device (CgScalars ring, cgx_internal.h), iterations are enqueued in
// chunks (optionally replayed from a hipGraph), and the host polls the device
// stop flag once per chunk while the next chunk is already queued.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <tuple>
#include <type_traits>
#include <thread>
#include <unordered_map>
#include <vector>

#include "cgx_objects.h"

namespace cgx {

static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

int hip_fail(hipError_t e, const char *what) {
  set_error("%s failed: %s (%d)", what, hipGetErrorString(e), (int)e);
  return CGX_EHIP;
}

std::vector<int> build_row_blocks(const int *rowptr, int64_t n, int *max_row_nnz, int tile,
                                  const std::vector<int64_t> *cuts) {
  const int cap = tile - 6;                            // quad loads (kTileCap)
  const int rows_max = tile / 8;  // 2048 -> 256, 1024 -> 128, 512 -> 64 rows
  std::vector<int> rb;
  rb.reserve((size_t)(n / 128 + 2));
  rb.push_back(0);
  int64_t row = 0;
  int mx = 0;
  size_t ci = 0;
  while (row < n) {
    const int64_t start = row;
    // the next cut after this block's first row: the block ends before it
    while (cuts && ci < cuts->size() && (*cuts)[ci] <= start) ++ci;
    const int64_t lim = (cuts && ci < cuts->size()) ? (*cuts)[ci] : n;
    int len = rowptr[row + 1] - rowptr[row];
    if (len > cap) {  // a long row gets a workgroup of its own
      mx = std::max(mx, len);
      ++row;
    } else {
      int64_t acc = 0;
      while (row < lim && row - start < rows_max) {
        len = rowptr[row + 1] - rowptr[row];
        if (acc + len > cap) break;
        acc += len;
        mx = std::max(mx, len);
        ++row;
      }
    }
    rb.push_back((int)row);
  }
  if (max_row_nnz) *max_row_nnz = mx;
  return rb;
}

namespace {

struct DeviceGuard {
  explicit DeviceGuard(int dev) { (void)hipSetDevice(dev); }
};

template <typename T> int enqueue_iter(cgx_cg *cg, int slot);

int poll_state(cgx_cg *cg, void *h_dst, hipStream_t s) {
  const size_t bytes = cg->dtype == CGX_F32 ? sizeof(CgScalars<float>) : sizeof(CgScalars<double>);
  CGX_HIP(hipMemcpyAsync(h_dst, cg->st, bytes, hipMemcpyDeviceToHost, s));
  return CGX_OK;
}

// read {active[slot], bodies, stopped, rxr[slot]} from a host copy of CgScalars
struct StateView {
  int active;
  long long bodies;
  int stopped;
  double rxr;
};
// (tail_fault: partitioned mode 4's last-workgroup r.r all-reduce timed out —
// the run stops as on stopped == 3)
StateView view_state(const cgx_cg *cg, const void *h, int slot) {
  StateView v{};
  if (cg->dtype == CGX_F32) {
    const auto *s = (const CgScalars<float> *)h;
    v = StateView{s->tail_fault ? 0 : s->active[slot], s->bodies,
                  s->tail_fault ? 3 : s->stopped, (double)s->rxr[slot]};
  } else {
    const auto *s = (const CgScalars<double> *)h;
    v = StateView{s->tail_fault ? 0 : s->active[slot], s->bodies,
                  s->tail_fault ? 3 : s->stopped, s->rxr[slot]};
  }
  return v;
}

hipEvent_t next_event(cgx_cg *cg) {
  if (cg->ev_used == cg->ev_pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    cg->ev_pool.push_back(e);
  }
  return cg->ev_pool[cg->ev_used++];
}

// Time one launch when timing is on: an event pair around `launch` (the
// launch as the stream sees it, dispatch latency included) and a pair its
// first kernel's dispatch records itself (g_exec: the kernel's execution, as
// rocprofv3 reports it; absent for launches that do not take them).
template <class F> int timed(cgx_cg *cg, int kid, hipStream_t s, F &&launch) {
  if (!cg->timing) {
    CGX_HIP(launch());
    return CGX_OK;
  }
  const size_t i0 = cg->ev_used;
  hipEvent_t e0 = next_event(cg), e1 = next_event(cg), x0 = next_event(cg), x1 = next_event(cg);
  CGX_REQUIRE(e0 && e1 && x0 && x1, CGX_EHIP, "hipEventCreate failed");
  CGX_HIP(hipEventRecord(e0, s));
  g_exec = ExecTiming{x0, x1, false};
  const hipError_t le = launch();
  const bool used = g_exec.used;
  g_exec = ExecTiming{};
  CGX_HIP(le);
  CGX_HIP(hipEventRecord(e1, s));
  cg->ev_pending.emplace_back(used ? kid + 16 : kid, i0);
  return CGX_OK;
}

// Accumulate pending event pairs; only the first `active_iters` iterations'
// kernels (3 per iteration, plus an init kernel if pending) count: kernels of
// iterations after the stop return at entry and would skew the averages.
int harvest_events(cgx_cg *cg, int64_t active_iters) {
  int64_t iter_seen = 0;
  const int last_kid = cg->coop ? 1 : (cg->fused || cg->fdefer) ? 2 : 3;
  for (auto &pr : cg->ev_pending) {
    const bool exec = pr.first >= 16;  // the dispatch recorded its own pair too
    const int kid = pr.first & 15;
    float ms = 0, xs = 0;
    CGX_HIP(hipEventElapsedTime(&ms, cg->ev_pool[pr.second], cg->ev_pool[pr.second + 1]));
    if (exec)
      CGX_HIP(hipEventElapsedTime(&xs, cg->ev_pool[pr.second + 2], cg->ev_pool[pr.second + 3]));
    const bool count = kid == 0 || iter_seen < active_iters;
    if (count) {
      cg->t_ms[kid] += ms;
      cg->t_calls[kid] += 1;
      if (exec) {
        cg->t_exec_ms[kid] += xs;
        cg->t_exec_calls[kid] += 1;
      }
    }
    if (kid == last_kid) ++iter_seen;
  }
  cg->ev_pending.clear();
  cg->ev_used = 0;
  return CGX_OK;
}

// SpMV + p.Ap of body `slot` on p, with the halo exchange of a partitioned
// matrix: a SELL matrix split into interior and boundary slices runs the
// interior ones while the exchange is in flight (RCCL on the comm stream),
// then the boundary ones; otherwise exchange, then one SpMV. *np: partials.
template <typename T>
int enqueue_spmv_dot(cgx_cg *cg, T *p, int slot, int rev, int *np) {
  cgx_csr *A = cg->A;
  hipStream_t s = cg->ctx->stream;
  auto *st = (CgScalars<T> *)cg->st;
  auto *ws = (RedWs<T> *)cg->ws;
  T *Ap = (T *)cg->Ap;
  int rc;
  const bool halo = A->dist && A->halo.n_ghost + A->halo.send_total > 0;
  if (halo && A->peer.on) {
    // device peer transport: push p's boundary entries into the neighbours,
    // run the interior slices, wait for the neighbours' entries, then the
    // boundary slices (or wait, then one launch when the matrix is not split).
    // A split SELL matrix carries the push in the interior launch's first
    // workgroups (k_spmv_dot_push: the xGMI stores overlap the interior
    // slices, one launch less)
    const bool split = A->split_ni > 0 && (launch_variant(A->dev, A->dtype) & (2048 | 8192));
    const int wg0 = A->peer.dev.nsend * kPushWG;
    // the interior slices by the lean walk (its layout skips the boundary ones)
    const bool lean_in = split && vl_active(A->dev) && A->dev.vl_split;
    const bool merged = split && wg0 > 0 && (lean_in || Launch<T>::push_supported(A->dev));
    // (the wait stays a launch of its own: round 2's folded form had the
    // boundary workgroups spin on flags raised by the same launch's first
    // workgroups, which relies on their being resident; removed in round 3,
    // DESIGN.md §9)
    if (!merged && (rc = peer_push<T>(A, p, st, slot, s))) return rc;
    const int gi = !split  ? 0
                   : lean_in ? A->dev.vl_grid
                   : merged  ? Launch<T>::slice_grid_push(A->dev, A->split_ni, wg0)
                             : Launch<T>::slice_grid(A->dev, A->split_ni);
    // the boundary slices wait for the neighbours' pushes themselves and read
    // the ghosts from the landing buffer (k_spmv_dot_bnd): no k_peer_wait
    // launch, no copy into p's ghost tail (matrices without the split keep
    // k_peer_wait before their one launch)
    // the boundary rows run as CSR-stream blocks (their own entry order; the
    // SELL copy holds them only as placeholders) with the wait folded in
    const bool rows = split && A->bnd_nblk > 0;
    const bool fold = split && A->split_nb > 0 && (rows || Launch<T>::bnd_supported(A->dev));
    if ((rc = timed(cg, 1, s, [&] {
           hipError_t e = hipSuccess;
           if (lean_in)
             e = Launch<T>::spmv_lean_interior(A->dev, p, Ap, st, slot, ws, s, rev,
                                               merged ? &A->peer.dev : nullptr, wg0);
           else if (merged)
             e = Launch<T>::spmv_dot_slices_push(A->dev, A->d_split, A->split_ni, 0, p, Ap, st,
                                                 slot, ws, s, rev, A->peer.dev, wg0);
           else if (split)
             e = Launch<T>::spmv_dot_slices(A->dev, A->d_split, A->split_ni, 0, p, Ap, st, slot,
                                            ws, s, rev);
           // the one-waiter form: one workgroup waits, the boundary grid does not
           if (e == hipSuccess && fold && A->peer.one_waiter &&
               peer_wait_one<T>(A, st, slot, s))
             e = hipErrorLaunchFailure;
           if (e == hipSuccess && fold)
             return rows ? Launch<T>::spmv_dot_rows(A->dev, A->d_bnd_blk, A->bnd_nblk, gi, p, Ap,
                                                    st, slot, ws, s, &A->peer.dev)
                         : Launch<T>::spmv_dot_slices_bnd(A->dev, A->d_split + A->split_ni,
                                                          A->split_nb, gi, p, Ap, st, slot, ws, s,
                                                          rev, A->peer.dev);
           if (e == hipSuccess && peer_wait<T>(A, p, st, slot, s)) e = hipErrorLaunchFailure;
           if (e == hipSuccess)
             e = split ? Launch<T>::spmv_dot_slices(A->dev, A->d_split + A->split_ni, A->split_nb,
                                                    gi, p, Ap, st, slot, ws, s, rev)
                       : Launch<T>::spmv_dot(A->dev, p, Ap, st, slot, ws, s, rev);
           return e;
         })))
      return rc;
    *np = !split ? Launch<T>::spmv_parts(A->dev)
                 : gi + (rows ? Launch<T>::rows_grid(A->dev, A->bnd_nblk)
                              : Launch<T>::slice_grid(A->dev, A->split_nb));
    return CGX_OK;
  }
  if (halo && A->split_ni > 0 && (launch_variant(A->dev, A->dtype) & (2048 | 8192))) {
    bool async = false;
    if ((rc = dist_halo_post(A, p, s, &async))) return rc;
    const bool lean_in = vl_active(A->dev) && A->dev.vl_split;
    const bool rows = A->bnd_nblk > 0;
    const int gi = lean_in ? A->dev.vl_grid : Launch<T>::slice_grid(A->dev, A->split_ni);
    // one timed region: interior slices, the wait for the halo, boundary slices
    if ((rc = timed(cg, 1, s, [&] {
           hipError_t e =
               lean_in ? Launch<T>::spmv_lean_interior(A->dev, p, Ap, st, slot, ws, s, rev,
                                                       nullptr, 0)
                       : Launch<T>::spmv_dot_slices(A->dev, A->d_split, A->split_ni, 0, p, Ap,
                                                    st, slot, ws, s, rev);
           if (e == hipSuccess && async) e = hipStreamWaitEvent(s, A->ev_halo, 0);
           if (e == hipSuccess)
             e = rows ? Launch<T>::spmv_dot_rows(A->dev, A->d_bnd_blk, A->bnd_nblk, gi, p, Ap, st,
                                                 slot, ws, s, nullptr)
                      : Launch<T>::spmv_dot_slices(A->dev, A->d_split + A->split_ni, A->split_nb,
                                                   gi, p, Ap, st, slot, ws, s, rev);
           return e;
         })))
      return rc;
    *np = gi + (rows ? Launch<T>::rows_grid(A->dev, A->bnd_nblk)
                     : Launch<T>::slice_grid(A->dev, A->split_nb));
    return CGX_OK;
  }
  if (halo && (rc = dist_halo_exchange(A, p, s))) return rc;
  if ((rc = timed(cg, 1, s,
                  [&] { return Launch<T>::spmv_dot(A->dev, p, Ap, st, slot, ws, s, rev); })))
    return rc;
  *np = Launch<T>::spmv_parts(A->dev);
  return CGX_OK;
}

// A partitioned run's dot: the local partials summed, then all-reduced into
// *dst — by the device peer transport in one kernel, or finalized into the
// scalar ring and all-reduced by the setup transport (RCCL / host).
template <typename T>
int dist_dot(cgx_cg *cg, const T *part, int np, T *dst, int slot, int which) {
  hipStream_t s = cg->ctx->stream;
  if (cg->A->peer.on)
    return peer_allreduce<T>(cg->A, part, np, dst, (CgScalars<T> *)cg->st, slot, s, which);
  CGX_HIP(Launch<T>::finalize(part, np, dst, s));
  return dist_allreduce_scalar(cg->ctx, dst, cg->dtype, 1, s);
}

// The device peer transport's two all-reduces of a body run inside the
// kernels that consume them (update_r: p.Ap, the x/p update: r.r; every
// workgroup polls the mailboxes, peerdev::world_sum) instead of as two
// one-workgroup launches (k_peer_allreduce, round 2's form).
// (the one-waiter form, ranks sharing a GPU: k_peer_allreduce's one
// workgroup per dot instead, through dist_dot; the same sums)
static const PeerDev *fused_ar(const cgx_cg *cg) {
  return (cg->A->dist && cg->A->peer.on && !cg->A->peer.one_waiter) ? &cg->A->peer.dev : nullptr;
}

template <typename T> int enqueue_iter(cgx_cg *cg, int slot) {
  cgx_csr *A = cg->A;
  hipStream_t s = cg->ctx->stream;
  auto *st = (CgScalars<T> *)cg->st;
  auto *ws = (RedWs<T> *)cg->ws;
  T *p = (T *)cg->p, *Ap = (T *)cg->Ap, *r = (T *)cg->r, *x = (T *)cg->x;
  int rc;
  // The dots travel as per-workgroup partials summed by the next kernel
  // (single device). A partitioned run finalizes each local dot into the
  // scalar ring, all-reduces it, and the next kernel reads the ring.
  const int npr = Launch<T>::update_parts(cg->n);
  // sweep directions: each kernel starts where the previous one ended
  const int par = cg->altdir ? (slot & 1) : 0, rpar = cg->altdir ? 1 - par : 0;
  int npp = 0;
  const PeerDev *far = fused_ar(cg);
  const bool sep = A->dist && !far;  // a separate all-reduce step per dot
  if ((rc = enqueue_spmv_dot<T>(cg, p, slot, par, &npp))) return rc;
  if (sep && (rc = dist_dot<T>(cg, ws->pap_part, npp, &st->pAp[slot], slot, 1))) return rc;
  if ((rc = timed(cg, 2, s, [&] {
         return Launch<T>::update_r(cg->n, r, Ap, st, slot, ws, s, false, sep ? 0 : npp, rpar,
                                    nullptr, 0, far);
       })))
    return rc;
  if (sep && (rc = dist_dot<T>(cg, ws->rr_part, npr, &st->rr[slot], slot, 2))) return rc;
  if ((rc = timed(cg, 3, s, [&] {
         return Launch<T>::update_xp(cg->n, x, p, r, st, slot, ws, sep ? 0 : npr, s, par, far);
       })))
    return rc;
  return CGX_OK;
}

// Deferred-x iteration (mode 3): body k uses p buffer k mod 4 and writes
// p_{k+1} into the next one; x is brought up to date in every slot-3 body
// and at the end of each run (flush_pending_x). Same values as mode 1.
template <typename T> int enqueue_iter_defer(cgx_cg *cg, int slot) {
  cgx_csr *A = cg->A;
  hipStream_t s = cg->ctx->stream;
  auto *st = (CgScalars<T> *)cg->st;
  auto *ws = (RedWs<T> *)cg->ws;
  T *P[4] = {(T *)cg->p, (T *)cg->pk[0], (T *)cg->pk[1], (T *)cg->pk[2]};
  T *p = P[slot], *pn = P[(slot + 1) & 3];
  T *Ap = (T *)cg->Ap, *r = (T *)cg->r, *x = (T *)cg->x;
  // r is updated in place (a ping-pong between two buffers measured 5-9%
  // slower in update_r)
  int rc;
  const int npr = Launch<T>::update_parts(cg->n);
  // sweep directions: each kernel starts where the previous one ended
  const int par = cg->altdir ? (slot & 1) : 0, rpar = cg->altdir ? 1 - par : 0;
  int npp = 0;
  const PeerDev *far = fused_ar(cg);
  const bool sep = A->dist && !far;  // a separate all-reduce step per dot
  if (cg->recompute) {
    // mode 6: kernel 1 keeps only p.Ap, kernel 2 forms A p again and updates
    // r in the walk's epilogue (no Ap vector: 8 N bytes written and read
    // less per body), kernel 3 as mode 3's (np_rr: kernel 2's grid)
    if ((rc = timed(cg, 1, s, [&] { return Launch<T>::lean_dot(A->dev, p, st, slot, ws, s, par); })))
      return rc;
    if ((rc = timed(cg, 2, s, [&] {
           return Launch<T>::lean_updr(A->dev, p, r, st, slot, ws, s, rpar);
         })))
      return rc;
    return timed(cg, 3, s, [&] {
      return Launch<T>::update_p_defer(cg->n, x, p, pn, P, r, st, slot, ws,
                                       lean_updr_parts(A->dev), s, par, nullptr);
    });
  }
  if ((rc = enqueue_spmv_dot<T>(cg, p, slot, par, &npp))) return rc;
  if (sep && (rc = dist_dot<T>(cg, ws->pap_part, npp, &st->pAp[slot], slot, 1))) return rc;
  if ((rc = timed(cg, 2, s, [&] {
         return Launch<T>::update_r(cg->n, r, Ap, st, slot, ws, s, false, sep ? 0 : npp, rpar,
                                    nullptr, 0, far);
       })))
    return rc;
  if (sep && (rc = dist_dot<T>(cg, ws->rr_part, npr, &st->rr[slot], slot, 2))) return rc;
  if ((rc = timed(cg, 3, s, [&] {
         return Launch<T>::update_p_defer(cg->n, x, p, pn, P, r, st, slot, ws, sep ? 0 : npr, s,
                                          par, far);
       })))
    return rc;
  return CGX_OK;
}

// Mode 4 on a partitioned matrix (enqueue_iter_fdefer's partitioned body):
// f64 over the device peer transport, the interior by the lean walk (its
// layout skips the boundary slices) and the boundary rows as CSR-stream
// blocks, i.e. the stencil slabs of SURVEY §8(e)
bool dist_fd_ok(const cgx_csr *A, int dtype) {
  return A->dist && A->peer.on && dtype == CGX_F64 &&
         A->halo.n_ghost + A->halo.send_total > 0 && A->split_ni > 0 &&
         (launch_variant(A->dev, A->dtype) & (2048 | 8192)) && vl_active(A->dev) &&
         A->dev.vl_split && A->bnd_nblk > 0;
}

// Fused deferred-x iteration (mode 4): two kernels per body on one device.
// Kernel 1 computes p_k = r + beta p_{k-1} where the SpMV reads it and
// stores it into P[k mod 4] (no separate p update: one read of p less per
// body), kernel 2 is update_r with the stop rule; in slot 3 it also applies
// the group's x updates from the four p buffers (k_update_r_flush). Same
// values as modes 1 and 3, bit for bit.
template <typename T> int enqueue_iter_fdefer(cgx_cg *cg, int slot) {
  cgx_csr *A = cg->A;
  hipStream_t s = cg->ctx->stream;
  auto *st = (CgScalars<T> *)cg->st;
  auto *ws = (RedWs<T> *)cg->ws;
  T *P[4] = {(T *)cg->p, (T *)cg->pk[0], (T *)cg->pk[1], (T *)cg->pk[2]};
  T *Ap = (T *)cg->Ap, *r = (T *)cg->r, *x = (T *)cg->x;
  int rc;
  const int npr = Launch<T>::update_parts(cg->n);
  const int par = cg->altdir ? (slot & 1) : 0, rpar = cg->altdir ? 1 - par : 0;
  if (A->dist) {
    // partitioned (dist_fd_ok: device peer transport, lean interior, boundary
    // row blocks): kernel 1 the interior walk with the push of the formed p_k
    // in front, then the boundary rows after the neighbours' pushes, then
    // update_r with the p.Ap all-reduce, the stop rule and (slot 3) the flush
    CGX_REQUIRE(dist_fd_ok(A, cg->dtype), CGX_ESTATE,
                "mode 4 on a partitioned matrix: the device peer transport or the lean "
                "interior is no longer set up");
    const PeerDev &PD = A->peer.dev;
    const int wg0 = PD.nsend * kPushWG;
    const int gi = A->dev.vl_grid;
    if ((rc = timed(cg, 1, s, [&] {
           hipError_t e = Launch<T>::spmv_fd_lean_push(A->dev, r, P[(slot + 3) & 3], P[slot], Ap,
                                                       st, slot, ws, s, par, PD, wg0);
           if (e == hipSuccess && A->peer.one_waiter && peer_wait_one<T>(A, st, slot, s))
             e = hipErrorLaunchFailure;
           if (e == hipSuccess)
             e = Launch<T>::spmv_fd_rows_bnd(A->dev, A->d_bnd_blk, A->bnd_nblk, gi, r,
                                             P[(slot + 3) & 3], P[slot], Ap, st, slot, ws, s, PD);
           return e;
         })))
      return rc;
    const int npp = gi + Launch<T>::rows_grid(A->dev, A->bnd_nblk);
    // the one-waiter form: p.Ap all-reduced by one workgroup into st first
    // (the partials in sum_parts order, as kernel 3 would); kernel 3 then
    // reads it from st and only its last workgroup waits (on r.r)
    const bool one = A->peer.one_waiter;
    if (one && (rc = peer_allreduce<T>(A, ws->pap_part, npp, &st->pAp[slot], st, slot, s, 1)))
      return rc;
    return timed(cg, 2, s, [&] {
      return Launch<T>::update_r_peer_rule(cg->n, r, Ap, st, slot, ws, one ? 0 : npp, rpar, x,
                                           slot == 3 ? P : nullptr, s, PD);
    });
  }
  if (cg->recompute) {
    // mode 7: kernel 1 forms p_k into P[slot] with p.Ap only (the tile walk,
    // no Ap vector), kernel 2 forms A p_k again from it and updates r with
    // the stop rule; slot 3 applies the group's x updates after it
    // (k_flush_group). 60 N bytes per body against mode 6's 66 N.
    if ((rc = timed(cg, 1, s, [&] {
           return Launch<T>::fd_dot_tile(A->dev, r, P[(slot + 3) & 3], P[slot], st, slot, ws,
                                         A->dev.vl_grid, s, par);
         })))
      return rc;
    if ((rc = timed(cg, 2, s, [&] {
           return Launch<T>::lean_updr_rule(A->dev, P[slot], r, st, slot, ws, s, rpar);
         })))
      return rc;
    if (slot == 3)
      return timed(cg, 3, s, [&] { return Launch<T>::flush_group(cg->n, x, P, st, s, par); });
    return CGX_OK;
  }
  const int npp = Launch<T>::fd_parts(A->dev);
  if ((rc = timed(cg, 1, s, [&] {
         return Launch<T>::spmv_fd(A->dev, r, P[(slot + 3) & 3], P[slot], Ap, st, slot, ws, npr,
                                   s, par);
       })))
    return rc;
  // kernel 2: update_r with the stop rule; in slot 3 it also applies the
  // group's deferred x updates (one launch instead of a separate flush)
  if ((rc = timed(cg, 2, s, [&] {
         return slot == 3 ? Launch<T>::update_r_flush(cg->n, r, Ap, st, slot, ws, npp, rpar, x, P,
                                                      s)
                          : Launch<T>::update_r(cg->n, r, Ap, st, slot, ws, s, false, npp, rpar,
                                                nullptr, 1);
       })))
    return rc;
  return CGX_OK;
}

// Fused iteration (single device): x/p update folded into the next SpMV.
template <typename T> int enqueue_iter_fused(cgx_cg *cg, int slot) {
  cgx_csr *A = cg->A;
  hipStream_t s = cg->ctx->stream;
  auto *st = (CgScalars<T> *)cg->st;
  auto *ws = (RedWs<T> *)cg->ws;
  T *P[2] = {(T *)cg->p, (T *)cg->p2};
  T *pp = P[(slot + 3) & 1], *pc = P[slot & 1];
  T *Ap = (T *)cg->Ap, *r = (T *)cg->r, *x = (T *)cg->x;
  int rc;
  if ((rc = timed(cg, 1, s, [&] {
         return Launch<T>::spmv_fused(A->dev, r, pp, pc, x, Ap, st, slot, ws, s);
       })))
    return rc;
  if ((rc = timed(cg, 2, s,
                  [&] { return Launch<T>::update_r(cg->n, r, Ap, st, slot, ws, s, true); })))
    return rc;
  return CGX_OK;
}

// bodies per mode-5 launch: 8 poll intervals (a launch ends early at the stop,
// so a larger chunk costs nothing but the host's view of progress)
int64_t coop_chunk(const cgx_cg *cg) { return (int64_t)cg->poll_every * 8; }

// Mode 5: `bodies` bodies from `slot` in one persistent launch
int enqueue_coop(cgx_cg *cg, int slot, int64_t bodies) {
  const CsrDev &A = cg->A->dev;
  const int m = (int)std::min<int64_t>(bodies, 1 << 30);
  return timed(cg, 1, cg->ctx->stream, [&] {
    return cg_coop(cg->n, cg->coop_r, cg->coop_stream, A.rowptr, A.col, (const double *)A.val,
                   (double *)cg->x, (double *)cg->r, (double *)cg->p, (double *)cg->p2,
                   (CgScalars<double> *)cg->st, slot, m, (CoopWs *)cg->coop_ws, cg->coop_ticks,
                   (unsigned long long *)cg->coop_trace, cg->coop_stall, cg->ctx->stream);
  });
}

// $CGX_COOP_R: the streamed form's rows per thread (unset: the fewest that fit)
int coop_want_r() {
  const char *e = std::getenv("CGX_COOP_R");
  return e ? std::atoi(e) : 0;
}

int enqueue_iter_any(cgx_cg *cg, int slot) {
  if (cg->fdefer)
    return cg->dtype == CGX_F32 ? enqueue_iter_fdefer<float>(cg, slot)
                                : enqueue_iter_fdefer<double>(cg, slot);
  if (cg->defer)
    return cg->dtype == CGX_F32 ? enqueue_iter_defer<float>(cg, slot)
                                : enqueue_iter_defer<double>(cg, slot);
  if (cg->fused)
    return cg->dtype == CGX_F32 ? enqueue_iter_fused<float>(cg, slot)
                                : enqueue_iter_fused<double>(cg, slot);
  return cg->dtype == CGX_F32 ? enqueue_iter<float>(cg, slot) : enqueue_iter<double>(cg, slot);
}

// Fused mode leaves the last body's x update pending, mode 3 up to three:
// apply them (idempotent).
int flush_pending_x(cgx_cg *cg) {
  if (cg->fdefer) {
    // bodies of an unfinished group (a finished one was applied by its slot-3
    // flush), then the final r.r record when the run ended on an active body
    hipStream_t s = cg->ctx->stream;
    // (mode 7: kernel 2 is the lean walk, one r.r partial per workgroup)
    const int npr = cg->recompute ? cg->A->dev.vl_grid
                    : cg->dtype == CGX_F32 ? Launch<float>::update_parts(cg->n)
                                           : Launch<double>::update_parts(cg->n);
    if (cg->dtype == CGX_F32) {
      float *P[4] = {(float *)cg->p, (float *)cg->pk[0], (float *)cg->pk[1], (float *)cg->pk[2]};
      if (cg->slot != 0)
        CGX_HIP(Launch<float>::flush_defer(cg->n, (float *)cg->x, P, (CgScalars<float> *)cg->st, s));
      CGX_HIP(Launch<float>::rr_settle((CgScalars<float> *)cg->st, (RedWs<float> *)cg->ws, npr, s));
    } else {
      double *P[4] = {(double *)cg->p, (double *)cg->pk[0], (double *)cg->pk[1],
                      (double *)cg->pk[2]};
      if (cg->slot != 0)
        CGX_HIP(Launch<double>::flush_defer(cg->n, (double *)cg->x, P,
                                            (CgScalars<double> *)cg->st, s));
      // (partitioned: kernel 3 recorded the world r.r itself)
      if (!cg->A->dist)
        CGX_HIP(Launch<double>::rr_settle((CgScalars<double> *)cg->st, (RedWs<double> *)cg->ws,
                                          npr, s));
    }
    return CGX_OK;
  }
  if (cg->defer) {
    hipStream_t s = cg->ctx->stream;
    if (cg->dtype == CGX_F32) {
      float *P[4] = {(float *)cg->p, (float *)cg->pk[0], (float *)cg->pk[1], (float *)cg->pk[2]};
      CGX_HIP(Launch<float>::flush_defer(cg->n, (float *)cg->x, P, (CgScalars<float> *)cg->st, s));
    } else {
      double *P[4] = {(double *)cg->p, (double *)cg->pk[0], (double *)cg->pk[1],
                      (double *)cg->pk[2]};
      CGX_HIP(Launch<double>::flush_defer(cg->n, (double *)cg->x, P,
                                          (CgScalars<double> *)cg->st, s));
    }
    return CGX_OK;
  }
  if (!cg->fused) return CGX_OK;
  const int last = (cg->slot + 3) & 3;
  hipStream_t s = cg->ctx->stream;
  void *P[2] = {cg->p, cg->p2};
  if (cg->dtype == CGX_F32)
    CGX_HIP(Launch<float>::flush_x(cg->n, (float *)cg->x, (const float *)P[last & 1],
                                   (CgScalars<float> *)cg->st, last, (RedWs<float> *)cg->ws, s));
  else
    CGX_HIP(Launch<double>::flush_x(cg->n, (double *)cg->x, (const double *)P[last & 1],
                                    (CgScalars<double> *)cg->st, last, (RedWs<double> *)cg->ws,
                                    s));
  return CGX_OK;
}

// A cached exec may still be in flight (cgx_cg_run keeps two chunks queued):
// the stream drains before any is destroyed.
void drop_graph(cgx_cg *cg) {
  if (cg->graphs.empty()) return;
  (void)hipStreamSynchronize(cg->ctx->stream);
  for (auto &kv : cg->graphs) (void)hipGraphExecDestroy(kv.second);
  cg->graphs.clear();
}

// Capture `iters` iterations starting at slot `slot0` (slots slot0 ..
// slot0 + iters - 1 mod 4) as one graph, cached under (slot0, iters).
int build_graph(cgx_cg *cg, int slot0, int64_t iters, hipGraphExec_t *out) {
  if (cg->graph_x != cg->x) drop_graph(cg);
  hipStream_t s = cg->ctx->stream;
  CGX_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  int rc = CGX_OK;
  for (int64_t i = 0; i < iters && rc == CGX_OK; ++i)
    rc = enqueue_iter_any(cg, (int)((slot0 + i) & 3));
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(s, &g);
  if (rc) {
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  CGX_HIP(e);
  hipGraphExec_t ge = nullptr;
  e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  CGX_HIP(e);
  // the executable graph's packets onto the device now, not at its first
  // launch (cgx_cg_prepare: out of a timed region)
  if ((e = hipGraphUpload(ge, s)) != hipSuccess) {
    (void)hipGraphExecDestroy(ge);
    CGX_HIP(e);
  }
  cg->graph_x = cg->x;
  cg->graphs[{slot0, iters}] = ge;
  *out = ge;
  return CGX_OK;
}

bool graph_ok(const cgx_cg *cg) {
  // RCCL / host-transport calls are kept out of captured graphs (the peer
  // transport's iteration is all kernels); timing needs eager launches
  return cg->use_graph && !cg->timing && !cg->coop && (!cg->A->dist || cg->A->peer.on);
}

// The graph for a chunk of `iters` bodies from `slot0`: a cached one, else a
// new capture when `build` (full poll_every chunks, and cgx_cg_prepare),
// else null (the chunk is launched eagerly).
int chunk_graph(cgx_cg *cg, int slot0, int64_t iters, bool build, hipGraphExec_t *out) {
  *out = nullptr;
  if (cg->graph_x == cg->x) {
    auto it = cg->graphs.find({slot0, iters});
    if (it != cg->graphs.end()) {
      *out = it->second;
      return CGX_OK;
    }
  }
  if (!build) return CGX_OK;
  if (cg->graphs.size() >= 16) drop_graph(cg);  // bound the cache
  return build_graph(cg, slot0, iters, out);
}

}  // namespace
}  // namespace cgx

using namespace cgx;

// ===========================================================================
// errors / version / devices
// ===========================================================================
extern "C" const char *cgx_last_error(void) { return g_err.c_str(); }
extern "C" const char *cgx_version(void) { return "cgx 0.1.0 gfx950"; }

extern "C" int cgx_device_count(int *count) {
  CGX_REQUIRE(count, CGX_EINVAL, "count is NULL");
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *count = c;
  return CGX_OK;
}

// ===========================================================================
// context
// ===========================================================================
extern "C" int cgx_create(int device, cgx_ctx **out) {
  CGX_REQUIRE(out, CGX_EINVAL, "out is NULL");
  *out = nullptr;
  int cnt = 0;
  CGX_HIP(hipGetDeviceCount(&cnt));
  CGX_REQUIRE(device >= 0 && device < cnt, CGX_EINVAL, "device %d out of range (%d visible)",
              device, cnt);
  CGX_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  CGX_HIP(hipGetDeviceProperties(&prop, device));
  CGX_REQUIRE(std::strncmp(prop.gcnArchName, "gfx950", 6) == 0, CGX_EUNSUPPORTED,
              "device %d is %s; libcgx is built for gfx950 (MI355X) only", device,
              prop.gcnArchName);
  auto *ctx = new cgx_ctx();
  ctx->device = device;
  hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&ctx->ws, sizeof(RedWs<double>));
  if (e == hipSuccess) e = hipMemset(ctx->ws, 0, sizeof(RedWs<double>));
  if (e == hipSuccess) e = hipMalloc(&ctx->scratch, 64);
  if (e == hipSuccess) e = hipHostMalloc(&ctx->h_pinned, 1024, hipHostMallocDefault);
  // the scalar state a standalone SpMV (cgx_spmv) runs k_spmv_dot with:
  // slot 0 active, its p.Ap partials into ctx->ws (not read)
  if (e == hipSuccess) e = hipMalloc(&ctx->spmv_st, sizeof(CgScalars<double>) + sizeof(CgScalars<float>));
  if (e == hipSuccess) {
    CgScalars<double> sd{};
    CgScalars<float> sf{};
    sd.active[0] = sf.active[0] = 1;
    e = hipMemcpy(ctx->spmv_st, &sd, sizeof(sd), hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy((char *)ctx->spmv_st + sizeof(sd), &sf, sizeof(sf), hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    cgx_destroy(ctx);
    return hip_fail(e, "cgx_create");
  }
  *out = ctx;
  return CGX_OK;
}

void cgx::ctx_retain(cgx_ctx *ctx) { ctx->refs.fetch_add(1, std::memory_order_relaxed); }

static void ctx_free(cgx_ctx *ctx);

void cgx::ctx_release(cgx_ctx *ctx) {
  if (ctx->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) ctx_free(ctx);
}

void cgx::csr_retain(cgx_csr *A) { A->refs.fetch_add(1, std::memory_order_relaxed); }

static void csr_free(cgx_csr *A);

void cgx::csr_release(cgx_csr *A) {
  if (A->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) csr_free(A);
}

// The owner's release: the context lives on while matrices or solvers made
// on it do (the last of them frees it).
extern "C" int cgx_destroy(cgx_ctx *ctx) {
  if (!ctx) return CGX_OK;
  ctx_release(ctx);
  return CGX_OK;
}

static void ctx_free(cgx_ctx *ctx) {
  DeviceGuard g(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  dist_comm_destroy(ctx);
  if (ctx->ws) (void)hipFree(ctx->ws);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->spmv_st) (void)hipFree(ctx->spmv_st);
  if (ctx->h_pinned) (void)hipHostFree(ctx->h_pinned);
  for (int b = 0; b < 2; ++b) {
    if (ctx->stage[b]) (void)hipHostFree(ctx->stage[b]);
    if (ctx->stage_ev[b]) (void)hipEventDestroy(ctx->stage_ev[b]);
  }
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

extern "C" int cgx_sync(cgx_ctx *ctx) {
  CGX_REQUIRE(ctx, CGX_EINVAL, "ctx is NULL");
  DeviceGuard g(ctx->device);
  CGX_HIP(hipStreamSynchronize(ctx->stream));
  return CGX_OK;
}

extern "C" int cgx_get_stream(cgx_ctx *ctx, void **s) {
  CGX_REQUIRE(ctx && s, CGX_EINVAL, "NULL argument");
  *s = (void *)ctx->stream;
  return CGX_OK;
}

extern "C" int cgx_get_device(cgx_ctx *ctx, int *d) {
  CGX_REQUIRE(ctx && d, CGX_EINVAL, "NULL argument");
  *d = ctx->device;
  return CGX_OK;
}

extern "C" int cgx_max_work_group_size(cgx_ctx *ctx, int *size) {
  CGX_REQUIRE(ctx && size, CGX_EINVAL, "NULL argument");
  CGX_HIP(hipDeviceGetAttribute(size, hipDeviceAttributeMaxThreadsPerBlock, ctx->device));
  return CGX_OK;
}

// ===========================================================================
// memory
// ===========================================================================
extern "C" int cgx_alloc(cgx_ctx *ctx, size_t bytes, void **d_out) {
  CGX_REQUIRE(ctx && d_out, CGX_EINVAL, "NULL argument");
  DeviceGuard g(ctx->device);
  *d_out = nullptr;
  hipError_t e = hipMalloc(d_out, bytes ? bytes : 1);
  if (e == hipErrorOutOfMemory) {
    set_error("hipMalloc(%zu) out of device memory", bytes);
    return CGX_ENOMEM;
  }
  CGX_HIP(e);
  return CGX_OK;
}

extern "C" int cgx_free(cgx_ctx *ctx, void *d) {
  CGX_REQUIRE(ctx, CGX_EINVAL, "ctx is NULL");
  if (!d) return CGX_OK;
  DeviceGuard g(ctx->device);
  CGX_HIP(hipStreamSynchronize(ctx->stream));
  CGX_HIP(hipFree(d));
  return CGX_OK;
}

// Large device -> host copies into pageable memory (extract() of a 256^3
// solution, a CSR download) go through a ring of two pinned 64 MiB chunks:
// the DMA engine fills chunk k+1 while several host threads copy chunk k out
// (15-17 GB/s against 10 for one hipMemcpy, profiles/r01_setup.json). Small
// copies use one hipMemcpyAsync.
constexpr size_t kStageChunk = size_t(64) << 20;
constexpr size_t kStageMin = size_t(16) << 20;

static bool staged(size_t bytes) { return bytes >= kStageMin; }

static int ensure_stage(cgx_ctx *ctx) {
  for (int b = 0; b < 2; ++b) {
    if (!ctx->stage[b]) CGX_HIP(hipHostMalloc(&ctx->stage[b], kStageChunk, hipHostMallocDefault));
    if (!ctx->stage_ev[b]) CGX_HIP(hipEventCreateWithFlags(&ctx->stage_ev[b], hipEventDisableTiming));
  }
  return CGX_OK;
}

static void par_memcpy(void *dst, const void *src, size_t len) {
  const unsigned hw = std::thread::hardware_concurrency();
  const int nt = (int)std::max<size_t>(1, std::min<size_t>(std::min(hw ? hw : 1u, 8u), len >> 22));
  if (nt <= 1) {
    std::memcpy(dst, src, len);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) {
    const size_t a = len * t / nt, b = len * (t + 1) / nt;
    th.emplace_back([=] { std::memcpy((char *)dst + a, (const char *)src + a, b - a); });
  }
  for (auto &x : th) x.join();
}

// Host -> device: ROCm's pageable path already runs at 50-55 GB/s for a
// 1.5 GB CSR on MI355X (a pinned ring measured no faster:
// profiles/r01_setup.json), so one hipMemcpyAsync.
extern "C" int cgx_h2d(cgx_ctx *ctx, void *dst, const void *src, size_t bytes) {
  CGX_REQUIRE(ctx && (bytes == 0 || (dst && src)), CGX_EINVAL, "NULL argument");
  DeviceGuard g(ctx->device);
  CGX_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  CGX_HIP(hipStreamSynchronize(ctx->stream));
  return CGX_OK;
}

extern "C" int cgx_h2d_async(cgx_ctx *ctx, void *dst, const void *src, size_t bytes) {
  CGX_REQUIRE(ctx && (bytes == 0 || (dst && src)), CGX_EINVAL, "NULL argument");
  DeviceGuard g(ctx->device);
  CGX_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  return CGX_OK;
}

extern "C" int cgx_d2h(cgx_ctx *ctx, void *dst, const void *src, size_t bytes) {
  CGX_REQUIRE(ctx && (bytes == 0 || (dst && src)), CGX_EINVAL, "NULL argument");
  DeviceGuard g(ctx->device);
  if (!staged(bytes)) {
    CGX_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    CGX_HIP(hipStreamSynchronize(ctx->stream));
    return CGX_OK;
  }
  if (int rc = ensure_stage(ctx)) return rc;
  // DMA chunk k+1 while the host copies chunk k out of the ring
  const size_t nchunks = (bytes + kStageChunk - 1) / kStageChunk;
  auto issue = [&](size_t k) -> int {
    const int b = (int)(k & 1);
    const size_t off = k * kStageChunk, len = std::min(kStageChunk, bytes - off);
    CGX_HIP(hipMemcpyAsync(ctx->stage[b], (const char *)src + off, len, hipMemcpyDeviceToHost,
                           ctx->stream));
    CGX_HIP(hipEventRecord(ctx->stage_ev[b], ctx->stream));
    return CGX_OK;
  };
  if (int rc = issue(0)) return rc;
  for (size_t k = 0; k < nchunks; ++k) {
    if (k + 1 < nchunks)
      if (int rc = issue(k + 1)) return rc;
    const int b = (int)(k & 1);
    const size_t off = k * kStageChunk, len = std::min(kStageChunk, bytes - off);
    CGX_HIP(hipEventSynchronize(ctx->stage_ev[b]));
    par_memcpy((char *)dst + off, ctx->stage[b], len);
  }
  return CGX_OK;
}

extern "C" int cgx_d2d(cgx_ctx *ctx, void *dst, const void *src, size_t bytes) {
  CGX_REQUIRE(ctx && (bytes == 0 || (dst && src)), CGX_EINVAL, "NULL argument");
  DeviceGuard g(ctx->device);
  CGX_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  return CGX_OK;
}

extern "C" int cgx_fill(cgx_ctx *ctx, int dtype, void *d, double v, size_t n) {
  CGX_REQUIRE(ctx && (n == 0 || d), CGX_EINVAL, "NULL argument");
  if (n == 0) return CGX_OK;
  DeviceGuard g(ctx->device);
  if (dtype == CGX_F32) CGX_HIP(Launch<float>::fill((float *)d, (float)v, (int64_t)n, ctx->stream));
  else CGX_HIP(Launch<double>::fill((double *)d, v, (int64_t)n, ctx->stream));
  return CGX_OK;
}

int autotune_spmv(cgx_csr *A);
int build_sell(cgx_csr *A, const int *h_rowptr, const int *h_col, int R = 0,
               const std::vector<char> *skip = nullptr);
int build_value_codes(cgx_csr *A);
void free_sell(cgx_csr *A);

// CSR-stream's 16-bit column deltas (variant bit kC16): built on demand;
// false when some entry's delta from its row block's first row does not fit
static void free_col16(cgx_csr *A) {
  if (A->d_col16) (void)hipFree(A->d_col16);
  A->d_col16 = nullptr;
  A->dev.col16 = nullptr;
}
// The interleaved val / col copy of the CSR-stream forms (kIL; round 6,
// verdict r5 item 3): the values and columns of each chunk of kIlCh pairs
// side by side in one allocation (cgx_internal.h), so the loop reads one
// stream instead of two arrays whose relative placement moved the kernel by
// +-15% (DESIGN.md §8 "Round 5"). Built on demand; the matrix's own arrays
// stay the caller's.
static void free_il(cgx_csr *A) {
  if (A->d_il) (void)hipFree(A->d_il);
  A->d_il = nullptr;
  A->dev.il = nullptr;
}
static bool build_il(cgx_csr *A) {
  if (A->dev.il) return true;
  if (A->dev.nnz < 2) return false;
  hipStream_t s = A->ctx->stream;
  const int es = (int)dtype_size(A->dtype);
  void *d = nullptr;
  hipError_t e = hipMalloc(&d, (size_t)il_bytes(A->dev.nnz, es));
  if (e == hipSuccess) e = il_build(A->dev, es, (char *)d, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    if (d) (void)hipFree(d);
    (void)hipGetLastError();
    return false;
  }
  A->d_il = d;
  A->dev.il = (const char *)d;
  return true;
}

static bool build_col16(cgx_csr *A) {
  if (A->dev.col16) return true;
  if (A->dev.nnz < 2 || A->dev.nrb < 1 || !A->dev.rb || !A->dev.rbk) return false;
  hipStream_t s = A->ctx->stream;
  void *d = nullptr;
  unsigned *bad = nullptr;
  hipError_t e = hipMalloc(&d, (size_t)(A->dev.nnz + 2) * sizeof(short));
  if (e == hipSuccess) e = hipMalloc((void **)&bad, sizeof(unsigned));
  if (e == hipSuccess) e = hipMemsetAsync(bad, 0, sizeof(unsigned), s);
  if (e == hipSuccess) e = col16_build(A->dev, (short *)d, bad, s);
  unsigned h = 1;
  if (e == hipSuccess) e = hipMemcpyAsync(&h, bad, sizeof(unsigned), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (bad) (void)hipFree(bad);
  if (e != hipSuccess || h != 0) {
    if (d) (void)hipFree(d);
    (void)hipGetLastError();
    return false;
  }
  A->d_col16 = d;
  A->dev.col16 = (const short *)d;
  return true;
}

// CSR-stream's row-block visit order (CsrDev::rbo). A matrix from a 3-D
// grid gathers p at +-D (one plane) from every row; in the natural order the
// XCD's workgroups reach a plane's rows again only after ~2 D rows of val/col
// have streamed through its 4 MB L2, so the p lines at +-D are fetched again
// (round 3's PMC: 1.19x the CSR bytes at 256^3). Walking chunks of W rows of
// a plane through all planes of the XCD's eighth puts them W rows apart.
static void free_block_order(cgx_csr *A) {
  if (A->d_rbo) (void)hipFree(A->d_rbo);
  A->d_rbo = nullptr;
  A->dev.rbo = nullptr;
  A->dev.ob_D = A->dev.ob_W = 0;
}

// The largest positive column offset (col - row) that at least a quarter of
// a sample of rows has (64 runs of 64 rows, evenly spaced); 0 when none.
static int dominant_offset(cgx_csr *A, const int *hrp) {
  const int64_t n = A->dev.n;
  if (n < 4096 || A->dev.nnz < 1) return 0;
  hipStream_t s = A->ctx->stream;
  std::unordered_map<int, int> cnt;
  int rows = 0;
  std::vector<int> c;
  for (int i = 0; i < 64; ++i) {
    const int64_t r0 = (int64_t)i * (n - 64) / 63;
    const int k0 = hrp[r0], k1 = hrp[r0 + 64];
    if (k1 <= k0) continue;
    c.resize((size_t)(k1 - k0));
    if (hipMemcpyAsync(c.data(), A->dev.col + k0, c.size() * sizeof(int), hipMemcpyDeviceToHost,
                       s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    for (int64_t r = r0; r < r0 + 64; ++r) {
      ++rows;
      for (int k = hrp[r]; k < hrp[r + 1]; ++k) {
        const int64_t o = (int64_t)c[(size_t)(k - k0)] - r;
        if (o > 0 && o < (int64_t(1) << 30)) ++cnt[(int)o];
      }
    }
  }
  int D = 0;
  for (const auto &kv : cnt)
    if (4 * kv.second >= rows && kv.first > D) D = kv.first;
  return D;
}

// Build the order: W > 0 chunk rows, W < 0 automatic. Returns CGX_OK with no
// order when the matrix has no plane offset worth it (automatic) or refuses
// an explicit W then.
static int build_block_order(cgx_csr *A, int W) {
  free_block_order(A);
  if (W == 0) return CGX_OK;
  const int64_t n = A->dev.n;
  const int nrb = A->dev.nrb;
  DeviceGuard g(A->ctx->device);
  hipStream_t s = A->ctx->stream;
  std::vector<int> hrp((size_t)n + 1), rb((size_t)nrb + 1);
  CGX_HIP(hipMemcpyAsync(hrp.data(), A->dev.rowptr, hrp.size() * sizeof(int),
                         hipMemcpyDeviceToHost, s));
  CGX_HIP(hipMemcpyAsync(rb.data(), A->dev.rb, rb.size() * sizeof(int), hipMemcpyDeviceToHost, s));
  CGX_HIP(hipStreamSynchronize(s));
  const int D = dominant_offset(A, hrp.data());
  // planes of the XCD's eighth, and the rows its 256 workgroups hold at once
  const int64_t Z = D > 0 ? (n / 8) / D : 0;
  const double bpr = 12.0 * (double)A->dev.nnz / (double)n + 16.0;
  const int64_t R = 256 * ((n + nrb - 1) / nrb);
  if (W < 0) {
    // worth it when two planes of stream overflow half an L2 and the eighth
    // holds several planes
    if (D <= 0 || Z < 4 || 2.0 * D * bpr < 2.0 * (1 << 20)) return CGX_OK;
    W = (int)std::max<int64_t>(R / Z, (n + nrb - 1) / nrb);
  } else if (D <= 0 || Z < 2) {
    set_error("block order: the matrix has no dominant plane offset (D = %d, %lld planes per "
              "XCD eighth)", D, (long long)Z);
    return CGX_EINVAL;
  }
  std::vector<int> ord((size_t)nrb);
  for (int gi = 0; gi < 8; ++gi) {
    const int lo = (int)(((int64_t)nrb * gi) >> 3), hi = (int)(((int64_t)nrb * (gi + 1)) >> 3);
    if (hi <= lo) continue;
    const int64_t base = rb[(size_t)lo];
    for (int b = lo; b < hi; ++b) ord[(size_t)b] = b;
    std::stable_sort(ord.begin() + lo, ord.begin() + hi, [&](int x, int y) {
      const int64_t ux = rb[(size_t)x] - base, uy = rb[(size_t)y] - base;
      const int64_t cx = (ux % D) / W, cy = (uy % D) / W;
      if (cx != cy) return cx < cy;
      return ux / D < uy / D;
    });
  }
  void *d = nullptr;
  CGX_HIP(hipMalloc(&d, ord.size() * sizeof(int)));
  hipError_t e = hipMemcpyAsync(d, ord.data(), ord.size() * sizeof(int), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    (void)hipFree(d);
    return hip_fail(e, "build_block_order");
  }
  A->d_rbo = d;
  A->dev.rbo = (const int *)d;
  A->dev.ob_D = D;
  A->dev.ob_W = W;
  return CGX_OK;
}

extern "C" int cgx_csr_set_block_order(cgx_csr *A, int chunk_rows) {
  CGX_REQUIRE(A, CGX_EINVAL, "A is NULL");
  CGX_REQUIRE(chunk_rows >= -1, CGX_EINVAL, "chunk_rows must be >= -1");
  return build_block_order(A, chunk_rows);
}

extern "C" int cgx_csr_block_order_info(cgx_csr *A, int *D, int *chunk_rows) {
  CGX_REQUIRE(A && D && chunk_rows, CGX_EINVAL, "NULL argument");
  *D = A->dev.rbo ? A->dev.ob_D : 0;
  *chunk_rows = A->dev.rbo ? A->dev.ob_W : 0;
  return CGX_OK;
}

// ===========================================================================
// CSR
// ===========================================================================
extern "C" int cgx_csr_create(cgx_ctx *ctx, int64_t n, int64_t nnz, const int *d_rowptr,
                              const int *d_col, const void *d_val, int dtype,
                              const int *h_rowptr, cgx_csr **out) {
  CGX_REQUIRE(ctx && out && d_rowptr, CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(n >= 1 && n < (int64_t(1) << 31) - 1, CGX_EINVAL, "n=%lld out of range",
              (long long)n);
  CGX_REQUIRE(nnz >= 0 && nnz < (int64_t(1) << 31), CGX_EINVAL, "nnz=%lld out of range",
              (long long)nnz);
  CGX_REQUIRE(nnz == 0 || (d_col && d_val), CGX_EINVAL, "NULL column/value arrays");
  CGX_REQUIRE(dtype == CGX_F64 || dtype == CGX_F32, CGX_EINVAL, "bad dtype %d", dtype);
  DeviceGuard g(ctx->device);
  *out = nullptr;
  const auto t_start = std::chrono::steady_clock::now();
  std::vector<int> hrp;
  if (!h_rowptr) {
    hrp.resize((size_t)n + 1);
    CGX_HIP(hipMemcpyAsync(hrp.data(), d_rowptr, ((size_t)n + 1) * sizeof(int),
                           hipMemcpyDeviceToHost, ctx->stream));
    CGX_HIP(hipStreamSynchronize(ctx->stream));
    h_rowptr = hrp.data();
  }
  for (int64_t i = 0; i < n; ++i) {
    if (h_rowptr[i + 1] < h_rowptr[i]) {
      set_error("rowptr is not monotone at row %lld", (long long)i);
      return CGX_EINVAL;
    }
  }
  CGX_REQUIRE(h_rowptr[0] >= 0 && h_rowptr[n] <= nnz, CGX_EINVAL,
              "rowptr range [%d, %d] outside [0, nnz=%lld]", h_rowptr[0], h_rowptr[n],
              (long long)nnz);
  int mx = 0;
  std::vector<int> rb = build_row_blocks(h_rowptr, n, &mx);
  const size_t nrb1 = rb.size();
  rb.resize(2 * nrb1);  // second half: entry offset of each row block
  for (size_t i = 0; i < nrb1; ++i) rb[nrb1 + i] = h_rowptr[rb[i]];
  auto *A = new cgx_csr();
  A->ctx = ctx;
  ctx_retain(ctx);
  setup_begin(A);
  A->setup_last = t_start;  // the rowptr checks and row blocks above count too
  A->dtype = dtype;
  A->max_row_nnz = mx;
  A->dev = CsrDev{n, nnz, d_rowptr, d_col, d_val, nullptr, nullptr, (int)nrb1 - 1, kTile};
  hipError_t e = hipMalloc(&A->d_rb, rb.size() * sizeof(int));
  if (e == hipSuccess)
    e = hipMemcpyAsync(A->d_rb, rb.data(), rb.size() * sizeof(int), hipMemcpyHostToDevice,
                       ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    cgx_csr_destroy(A);
    return hip_fail(e, "cgx_csr_create");
  }
  A->dev.rb = A->d_rb;
  A->dev.rbk = A->d_rb + nrb1;
  A->n_global = n;
  setup_mark(A, 0);
  int rc = build_sell(A, h_rowptr, nullptr, 0);
  setup_mark(A, 2);  // (build_sell marks its own part as phase 1)
  if (!rc) rc = autotune_spmv(A);
  setup_mark(A, 4);
  A->setup_open = false;
  if (rc) {
    cgx_csr_destroy(A);
    return rc;
  }
  *out = A;
  return CGX_OK;
}

// The owner's release: a solver made on the matrix keeps it alive.
extern "C" int cgx_csr_destroy(cgx_csr *A) {
  if (!A) return CGX_OK;
  csr_release(A);
  return CGX_OK;
}

static void csr_free(cgx_csr *A) {
  cgx_ctx *ctx = A->ctx;
  {
    DeviceGuard g(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (A->d_rb) (void)hipFree(A->d_rb);
    if (A->d_ext) (void)hipFree(A->d_ext);
    free_sell(A);
    free_col16(A);
    free_il(A);
    free_block_order(A);
    peer_destroy(A);
    dist_destroy_halo(A);
  }
  delete A;
  ctx_release(ctx);
}

// Rebuild the row-block schedule for another tile size (2048 or 1024).
extern "C" int cgx_csr_set_tile(cgx_csr *A, int tile) {
  CGX_REQUIRE(A, CGX_EINVAL, "A is NULL");
  CGX_REQUIRE(tile == 2048 || tile == 1024 || tile == 512, CGX_EINVAL,
              "tile must be 2048, 1024 or 512 (wave tiles)");
  if (tile == A->dev.tile) return CGX_OK;
  DeviceGuard g(A->ctx->device);
  hipStream_t s = A->ctx->stream;
  const int64_t n = A->dev.n;
  std::vector<int> hrp((size_t)n + 1);
  CGX_HIP(hipMemcpyAsync(hrp.data(), A->dev.rowptr, hrp.size() * sizeof(int),
                         hipMemcpyDeviceToHost, s));
  CGX_HIP(hipStreamSynchronize(s));
  int mx = 0;
  std::vector<int> rb = build_row_blocks(hrp.data(), n, &mx, tile);
  const size_t nrb1 = rb.size();
  rb.resize(2 * nrb1);
  for (size_t i = 0; i < nrb1; ++i) rb[nrb1 + i] = hrp[rb[i]];
  int *d = nullptr;
  CGX_HIP(hipMalloc(&d, rb.size() * sizeof(int)));
  CGX_HIP(hipMemcpyAsync(d, rb.data(), rb.size() * sizeof(int), hipMemcpyHostToDevice, s));
  CGX_HIP(hipStreamSynchronize(s));
  free_block_order(A);  // an order of the old blocks
  if (A->d_rb) CGX_HIP(hipFree(A->d_rb));
  A->d_rb = d;
  A->dev.rb = d;
  A->dev.rbk = d + nrb1;
  A->dev.nrb = (int)nrb1 - 1;
  A->dev.tile = tile;
  return CGX_OK;
}

extern "C" int cgx_csr_variant(cgx_csr *A, int *variant) {
  CGX_REQUIRE(A && variant, CGX_EINVAL, "NULL argument");
  *variant = launch_variant(A->dev, A->dtype);
  return CGX_OK;
}

extern "C" int cgx_csr_info(cgx_csr *A, int64_t *n, int64_t *nnz, int64_t *rbs, int *mx) {
  CGX_REQUIRE(A, CGX_EINVAL, "A is NULL");
  if (n) *n = A->dev.n;
  if (nnz) *nnz = A->dev.nnz;
  if (rbs) *rbs = A->dev.nrb;
  if (mx) *mx = A->max_row_nnz;
  return CGX_OK;
}

void free_lean(cgx_csr *A) {
  for (void **p : {&A->d_vl_cls, &A->d_vl_tab}) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
  }
  A->dev.vl_cls = nullptr;
  A->dev.vl_tab = nullptr;
  A->dev.vl_grid = A->dev.vl_nst = A->dev.vl_D = A->dev.vl_a = 0;
  A->dev.vl_P = A->dev.vl_K = A->dev.vl_lds = A->dev.vl_split = A->dev.vl_team = 0;
  A->vl_tab_h.clear();
  A->dev.lean = false;
  A->vl_slice_cls.clear();
  A->vl_ncls = 0;
}

void free_sell(cgx_csr *A) {
  free_lean(A);
  A->sell_pool.clear();
  for (void **p : {&A->d_sell_sl, &A->d_sell_dict, &A->d_sell_idx, &A->d_sell_val,
                   &A->d_sell_order, (void **)&A->d_split, &A->d_sell_mask, &A->d_sell_vc,
                   &A->d_sell_vdict, &A->d_sell_vc4, &A->d_sell_sl_t, &A->d_vct}) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
  }
  A->dev.sl = nullptr;
  A->dev.sdict = nullptr;
  A->dev.sidx = nullptr;
  A->dev.sval = nullptr;
  A->dev.nsl = 0;
  A->dev.sorder = nullptr;
  A->dev.sell_kind = 0;
  A->dev.smask = nullptr;
  A->dev.svc = nullptr;
  A->dev.svdict = nullptr;
  A->dev.nvdict = 0;
  A->dev.svc4 = nullptr;
  A->dev.sl_t = nullptr;
  A->dev.vct = nullptr;
  A->dev.nvt = 0;
  A->vt_slices = 0;
  A->split_ni = A->split_nb = 0;
  A->split_bd_h.clear();
  A->split_ordered = false;
  if (A->d_bnd_blk) (void)hipFree(A->d_bnd_blk);
  A->d_bnd_blk = nullptr;
  A->bnd_nblk = 0;
  A->dev.sell_partial = 0;
  A->dev.sell_r = 1;
  A->dev.sell_maxw = 0;
  A->dev.march_k = A->dev.march_a = A->dev.march_len = 0;
  A->dev.march_pat = -1;
  A->sell_padded = 0;
  A->sell_idx_words = 0;
  A->vc_chunks = 0;
}

// SELL layout of a host CSR (cgx_internal.h SellSlice; DESIGN.md §SpMV
// formats) with R rows per lane (slices of 64 R rows). Qualifies when every
// slice has rows of at most kSellMaxWidth entries and at most kSellMaxDict
// distinct (col - row) offsets, and the padding adds at most a quarter of the
// entries (+4096) — stencil and other banded matrices. Returns false
// (outputs unspecified) otherwise. voff_total: value slots of the layout
// (the kernel reads one chunk beyond).
static bool sell_plan_host(int64_t n, const int *rowptr, const int *col, int R,
                           std::vector<SellSlice> &sl, std::vector<int> &pool,
                           std::vector<unsigned long long> &idx, int64_t &voff_total) {
  const int64_t nnz = (int64_t)rowptr[n] - rowptr[0];
  const int64_t H = (int64_t)kSellRows * R;  // rows per slice
  if (nnz < 1 || (R != 1 && R != 2) || n + H >= (int64_t(1) << 31)) return false;
  const int64_t nsl = (n + H - 1) / H;
  sl.assign((size_t)nsl, SellSlice{});
  int64_t voff = 0, ioff = 0, padded = 0;
  for (int64_t q = 0; q < nsl; ++q) {
    const int64_t r0 = q * H, r1 = std::min(n, r0 + H);
    int w = 0;
    for (int64_t i = r0; i < r1; ++i) w = std::max(w, rowptr[i + 1] - rowptr[i]);
    if (w > kSellMaxWidth) return false;
    sl[(size_t)q] = SellSlice{voff, ioff, 0, w};
    voff += H * w;
    ioff += H * ((w + 7) / 8);
    padded += (r1 - r0) * w;
  }
  if (padded > nnz + nnz / 4 + 4096) return false;  // small matrices: padding is noise
  // per-slice dictionaries (first-seen order), shared between equal slices
  pool.clear();
  std::vector<std::pair<std::vector<int>, int>> seen;  // recent distinct dictionaries
  idx.assign((size_t)ioff, ~0ull);
  std::vector<int> d;
  d.reserve(kSellMaxDict);
  for (int64_t q = 0; q < nsl; ++q) {
    SellSlice &m = sl[(size_t)q];
    const int64_t r0 = q * H, r1 = std::min(n, r0 + H);
    d.clear();
    for (int64_t i = r0; i < r1; ++i) {
      const int64_t l = (i - r0) / R, r = (i - r0) % R;  // lane, row of the lane
      for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) {
        const int off = col[k] - (int)i;
        size_t t = 0;
        while (t < d.size() && d[t] != off) ++t;
        if (t == d.size()) {
          if (d.size() == (size_t)kSellMaxDict) return false;
          d.push_back(off);
        }
        const int j = k - rowptr[i];
        unsigned long long &wd =
            idx[(size_t)(m.ioff + ((int64_t)(j >> 3) * kSellRows + l) * R + r)];
        const int sh = 8 * (j & 7);
        wd = (wd & ~(0xffull << sh)) | ((unsigned long long)t << sh);
      }
    }
    int base = -1;
    for (auto &e : seen)
      if (e.first == d) {
        base = e.second;
        break;
      }
    if (base < 0) {
      base = (int)pool.size();
      pool.insert(pool.end(), d.begin(), d.end());
      if (seen.size() >= 16) seen.erase(seen.begin());
      seen.emplace_back(d, base);
    }
    m.dict = base;
  }
  pool.resize(pool.size() + kSellMaxDict, 0);  // every lane of the last dictionary reads in bounds
  voff_total = voff;
  return true;
}

// SELL-P plan (2 rows per lane, slices of 128 rows): per slice the sorted
// union of its (col - row) offsets, at most kSellPatMax; rows must have
// strictly ascending columns (then a row's set slots are its CSR order).
// Padding bound as in sell_plan_host. maxw: the widest pattern.
// skip: slices that hold placeholders (a partitioned matrix's boundary
// slices, never run in this layout), exempt from the sorted-rows rule.
static bool sellp_plan_host(int64_t n, const int *rowptr, const int *col,
                            std::vector<SellSlice> &sl, std::vector<int> &pool,
                            int64_t &voff_total, int &maxw,
                            const std::vector<char> *skip = nullptr) {
  const int64_t nnz = (int64_t)rowptr[n] - rowptr[0];
  const int64_t H = 2 * kSellRows;
  if (nnz < 1 || n + H >= (int64_t(1) << 31)) return false;
  const int64_t nsl = (n + H - 1) / H;
  sl.assign((size_t)nsl, SellSlice{});
  pool.clear();
  std::vector<std::pair<std::vector<int>, int>> seen;
  std::vector<int> P;
  int64_t voff = 0, coff = 0, padded = 0;
  maxw = 0;
  for (int64_t q = 0; q < nsl; ++q) {
    const int64_t r0 = q * H, r1 = std::min(n, r0 + H);
    P.clear();
    for (int64_t i = r0; i < r1; ++i) {
      for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) {
        if (k > rowptr[i] && col[k] <= col[k - 1] &&
            !(skip && (size_t)q < skip->size() && (*skip)[(size_t)q]))
          return false;  // unsorted or duplicate
        const int off = col[k] - (int)i;
        auto it = std::lower_bound(P.begin(), P.end(), off);
        if (it == P.end() || *it != off) {
          if ((int)P.size() == kSellPatMax) return false;
          P.insert(it, off);
        }
      }
    }
    const int W = std::max<int>(1, (int)P.size());
    if (P.empty()) P.push_back(0);
    int base = -1;
    for (auto &e : seen)
      if (e.first == P) {
        base = e.second;
        break;
      }
    if (base < 0) {
      base = (int)pool.size();
      pool.insert(pool.end(), P.begin(), P.end());
      if (seen.size() >= 16) seen.erase(seen.begin());
      seen.emplace_back(P, base);
    }
    sl[(size_t)q] = SellSlice{voff, coff, base, W};  // coff: value-code chunks (16 B)
    voff += H * W;
    coff += kSellRows * ((W + 7) / 8);
    padded += (r1 - r0) * W;
    maxw = std::max(maxw, W);
  }
  if (padded > nnz + nnz / 4 + 4096) return false;
  pool.resize(pool.size() + kSellPatMax, 0);  // the kernel reads up to 7 slots past a pattern
  voff_total = voff;
  return true;
}

// sellp_plan_host's plan with the per-slice patterns formed on the device
// (k_sellp_plan: no column download, one wave per slice); the pattern pool
// (recent-16 sharing), offsets and the padding bound on the host, in slice
// order as sellp_plan_host. *ok = false when the matrix does not qualify.
static int sellp_plan_device(cgx_ctx *ctx, int64_t n, int64_t nnz, const int *d_rowptr,
                             const int *d_col, const std::vector<char> *skip,
                             std::vector<SellSlice> &sl, std::vector<int> &pool,
                             int64_t &voff_total, int &maxw, bool *ok) {
  *ok = false;
  const int64_t H = 2 * kSellRows;
  if (nnz < 1 || n + H >= (int64_t(1) << 31)) return CGX_OK;
  const int64_t nsl = (n + H - 1) / H;
  hipStream_t s = ctx->stream;
  int *d_pat = nullptr, *d_w = nullptr;
  char *d_skip = nullptr;
  std::vector<int> hpat((size_t)(nsl * kSellPatMax)), hw((size_t)nsl);
  hipError_t e = hipMalloc(&d_pat, hpat.size() * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&d_w, hw.size() * sizeof(int));
  if (e == hipSuccess && skip && !skip->empty()) {
    std::vector<char> sk((size_t)nsl, 0);
    std::copy(skip->begin(), skip->begin() + std::min<size_t>(skip->size(), sk.size()), sk.begin());
    e = hipMalloc(&d_skip, sk.size());
    if (e == hipSuccess) e = hipMemcpyAsync(d_skip, sk.data(), sk.size(), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
  }
  if (e == hipSuccess)
    e = sellp_plan_dev(n, nsl, d_rowptr, d_col, d_skip, d_pat, d_w, s);
  if (e == hipSuccess)
    e = hipMemcpyAsync(hw.data(), d_w, hw.size() * sizeof(int), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess)
    e = hipMemcpyAsync(hpat.data(), d_pat, hpat.size() * sizeof(int), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  for (void *p : {(void *)d_pat, (void *)d_w, (void *)d_skip})
    if (p) (void)hipFree(p);
  if (e != hipSuccess) return hip_fail(e, "cgx_csr_create(SELL-P plan)");
  sl.assign((size_t)nsl, SellSlice{});
  pool.clear();
  std::vector<std::pair<std::vector<int>, int>> seen;
  std::vector<int> P;
  int64_t voff = 0, coff = 0, padded = 0;
  maxw = 0;
  for (int64_t q = 0; q < nsl; ++q) {
    const int wq = hw[(size_t)q];
    if (wq < 0 || wq > kSellPatMax) return CGX_OK;  // unsorted row, or too many offsets
    const int64_t r0 = q * H, r1 = std::min(n, r0 + H);
    P.assign(hpat.begin() + q * kSellPatMax, hpat.begin() + q * kSellPatMax + wq);
    const int W = std::max<int>(1, (int)P.size());
    if (P.empty()) P.push_back(0);
    int base = -1;
    for (auto &pe : seen)
      if (pe.first == P) {
        base = pe.second;
        break;
      }
    if (base < 0) {
      base = (int)pool.size();
      pool.insert(pool.end(), P.begin(), P.end());
      if (seen.size() >= 16) seen.erase(seen.begin());
      seen.emplace_back(P, base);
    }
    sl[(size_t)q] = SellSlice{voff, coff, base, W};
    voff += H * W;
    coff += kSellRows * ((W + 7) / 8);
    padded += (r1 - r0) * W;
    maxw = std::max(maxw, W);
  }
  if (padded > nnz + nnz / 4 + 4096) return CGX_OK;
  pool.resize(pool.size() + kSellPatMax, 0);
  voff_total = voff;
  *ok = true;
  return CGX_OK;
}

// Plane-march plan (variant bit 2097152, cgx_kernels.hip spmv_sellpv_march):
// the most common slice pattern must be {-D, -a, -1, 0, 1, a, D} (3-D
// 7-point) or {-D, -1, 0, 1, D} (2-D 5-point) with D a positive multiple of
// the 128-row slice and 1 < a < D. Slices with another pattern (or the same
// pattern at another pool base) still run, through the per-slice form.
static void plan_march(const std::vector<SellSlice> &sl, const std::vector<int> &pool,
                       int64_t nx, size_t es, CsrDev &dev) {
  dev.march_k = dev.march_a = dev.march_len = 0;
  dev.march_pat = -1;
  if (sl.empty() || (uint64_t)nx * es >= (uint64_t(1) << 32)) return;
  std::map<std::pair<int, int>, int64_t> freq;  // (pool base, width) -> slices
  for (const SellSlice &m : sl) ++freq[{m.dict, m.width}];
  auto best = freq.begin();
  for (auto i = freq.begin(); i != freq.end(); ++i)
    if (i->second > best->second) best = i;
  const int base = best->first.first, W = best->first.second;
  if (best->second * 2 < (int64_t)sl.size() || (W != 5 && W != 7)) return;
  const int *o = pool.data() + base;
  const int D = o[W - 1], H = 2 * kSellRows;
  if (D <= 0 || D % H != 0 || o[0] != -D) return;
  int a = 0;
  if (W == 7) {
    a = o[5];
    if (!(a > 1 && a < D && o[1] == -a && o[2] == -1 && o[3] == 0 && o[4] == 1)) return;
  } else if (!(o[1] == -1 && o[2] == 0 && o[3] == 1)) {
    return;
  }
  dev.march_k = D / H;
  dev.march_a = a;
  dev.march_pat = base;
}

extern "C" int cgx_sellp_plan(const int *h_rowptr, const int *h_col, int64_t n, int64_t *nsl,
                              int64_t **slices, int64_t *npat, int **pat, int64_t *value_slots,
                              int *max_width) {
  CGX_REQUIRE(h_rowptr && h_col && nsl && slices && npat && pat && value_slots && max_width,
              CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(n >= 1, CGX_EINVAL, "n=%lld", (long long)n);
  std::vector<SellSlice> sl;
  std::vector<int> pool;
  int64_t voff = 0;
  int mw = 0;
  *nsl = *npat = *value_slots = 0;
  *max_width = 0;
  *slices = nullptr;
  *pat = nullptr;
  if (n < 2 || !sellp_plan_host(n, h_rowptr, h_col, sl, pool, voff, mw)) return CGX_OK;
  *slices = (int64_t *)std::malloc(sl.size() * 4 * sizeof(int64_t));
  *pat = (int *)std::malloc(pool.size() * sizeof(int));
  CGX_REQUIRE(*slices && *pat, CGX_ENOMEM, "host allocation failed");
  for (size_t q = 0; q < sl.size(); ++q) {
    (*slices)[4 * q] = sl[q].voff;
    (*slices)[4 * q + 1] = sl[q].ioff;
    (*slices)[4 * q + 2] = sl[q].dict;
    (*slices)[4 * q + 3] = sl[q].width;
  }
  std::memcpy(*pat, pool.data(), pool.size() * sizeof(int));
  *nsl = (int64_t)sl.size();
  *npat = (int64_t)pool.size();
  *value_slots = voff;
  *max_width = mw;
  return CGX_OK;
}

// cgx_sellp_plan's outputs from the device plan (k_sellp_plan) of a CSR in
// device memory: the same slices, pattern pool and widths (tests compare)
extern "C" int cgx_sellp_plan_device(cgx_ctx *ctx, const int *d_rowptr, const int *d_col,
                                     int64_t n, int64_t nnz, int64_t *nsl, int64_t **slices,
                                     int64_t *npat, int **pat, int64_t *value_slots,
                                     int *max_width) {
  CGX_REQUIRE(ctx && d_rowptr && d_col && nsl && slices && npat && pat && value_slots &&
                  max_width,
              CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(n >= 1, CGX_EINVAL, "n=%lld", (long long)n);
  DeviceGuard g(ctx->device);
  std::vector<SellSlice> sl;
  std::vector<int> pool;
  int64_t voff = 0;
  int mw = 0;
  *nsl = *npat = *value_slots = 0;
  *max_width = 0;
  *slices = nullptr;
  *pat = nullptr;
  bool ok = false;
  if (n >= 2)
    if (int rc = sellp_plan_device(ctx, n, nnz, d_rowptr, d_col, nullptr, sl, pool, voff, mw, &ok))
      return rc;
  if (!ok) return CGX_OK;
  *slices = (int64_t *)std::malloc(sl.size() * 4 * sizeof(int64_t));
  *pat = (int *)std::malloc(pool.size() * sizeof(int));
  CGX_REQUIRE(*slices && *pat, CGX_ENOMEM, "host allocation failed");
  for (size_t q = 0; q < sl.size(); ++q) {
    (*slices)[4 * q] = sl[q].voff;
    (*slices)[4 * q + 1] = sl[q].ioff;
    (*slices)[4 * q + 2] = sl[q].dict;
    (*slices)[4 * q + 3] = sl[q].width;
  }
  std::memcpy(*pat, pool.data(), pool.size() * sizeof(int));
  *nsl = (int64_t)sl.size();
  *npat = (int64_t)pool.size();
  *value_slots = voff;
  *max_width = mw;
  return CGX_OK;
}

extern "C" int cgx_sell_plan(const int *h_rowptr, const int *h_col, int64_t n, int rows_per_lane,
                             int64_t *nsl,
                             int64_t **slices, int64_t *ndict, int **dict, int64_t *nidx,
                             unsigned long long **idx, int64_t *value_slots) {
  CGX_REQUIRE(h_rowptr && h_col && nsl && slices && ndict && dict && nidx && idx && value_slots,
              CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(n >= 1, CGX_EINVAL, "n=%lld", (long long)n);
  std::vector<SellSlice> sl;
  std::vector<int> pool;
  std::vector<unsigned long long> ix;
  int64_t voff = 0;
  *nsl = *ndict = *nidx = *value_slots = 0;
  *slices = nullptr;
  *dict = nullptr;
  *idx = nullptr;
  CGX_REQUIRE(rows_per_lane == 1 || rows_per_lane == 2, CGX_EINVAL, "rows_per_lane must be 1 or 2");
  if (!sell_plan_host(n, h_rowptr, h_col, rows_per_lane, sl, pool, ix, voff)) return CGX_OK;
  *slices = (int64_t *)std::malloc(std::max<size_t>(sl.size(), 1) * 4 * sizeof(int64_t));
  *dict = (int *)std::malloc(pool.size() * sizeof(int));
  *idx = (unsigned long long *)std::malloc(std::max<size_t>(ix.size(), 1) * 8);
  CGX_REQUIRE(*slices && *dict && *idx, CGX_ENOMEM, "host allocation failed");
  for (size_t q = 0; q < sl.size(); ++q) {
    (*slices)[4 * q] = sl[q].voff;
    (*slices)[4 * q + 1] = sl[q].ioff;
    (*slices)[4 * q + 2] = sl[q].dict;
    (*slices)[4 * q + 3] = sl[q].width;
  }
  std::memcpy(*dict, pool.data(), pool.size() * sizeof(int));
  if (!ix.empty()) std::memcpy(*idx, ix.data(), ix.size() * 8);
  *nsl = (int64_t)sl.size();
  *ndict = (int64_t)pool.size();
  *nidx = (int64_t)ix.size();
  *value_slots = voff;
  return CGX_OK;
}

// Visit order of the slices. P is the stride of the farthest
// band (the largest |col - row|: a z-plane of a 3-D stencil). Within each
// XCD's eighth of the slices (the kernel's sell_range split), chunks of 128
// slices of a plane are walked through all the planes before the next
// chunk. The slices in flight on an XCD (1024 waves) then span ~8 planes of
// one chunk, and the p rows they gather (~1.3 MB at 256^3) stay in the
// XCD's 4 MB L2, where plane-by-plane order spans two whole planes and
// re-fetches p. Empty when planes are small (< 256 slices).
// The same order over a list of slice ids (ascending; a partitioned matrix's
// interior slices, cgx_dist.cpp): positions are split into eighths as the
// kernel's sell_range splits a list. Empty when no reordering applies.
std::vector<int> chunked_slice_order(const std::vector<int> &ids, int64_t H, int64_t P,
                                     int64_t kChunk) {
  std::vector<int> order;
  if (P / H < 2 * kChunk) return order;
  const int64_t m = (int64_t)ids.size();
  order.resize((size_t)m);
  std::vector<std::tuple<int64_t, int64_t, int64_t, int>> key;
  for (int g = 0; g < 8; ++g) {
    const int64_t lo = (m * g) >> 3, hi = (m * (g + 1)) >> 3;
    key.clear();
    for (int64_t i = lo; i < hi; ++i) {
      const int q = ids[(size_t)i];
      const int64_t r0 = (int64_t)q * H, z = r0 / P, u = (r0 % P) / H;
      key.emplace_back(u / kChunk, z, u, q);
    }
    std::sort(key.begin(), key.end());
    for (size_t k = 0; k < key.size(); ++k) order[(size_t)lo + k] = std::get<3>(key[k]);
  }
  return order;
}
static std::vector<int> sell_visit_order(int64_t nsl, int64_t H, int64_t P, int64_t kChunk) {
  std::vector<int> ids((size_t)nsl);
  for (int64_t q = 0; q < nsl; ++q) ids[(size_t)q] = (int)q;
  return chunked_slice_order(ids, H, P, kChunk);
}

// Value codes of A's SELL-P copy (cgx_internal.h kVcMax): the
// dictionary starts from the distinct values of an evenly spread sample of
// the value array; the pack kernel reports values it lacks, which join the
// dictionary for another pass, until every value is found or there are more
// than kVcMax of them (then the matrix keeps plain SELL-P values; not an
// error). Errors are device failures only.
template <typename T> static int build_value_codes_t(cgx_csr *A) {
  using B = typename std::conditional<sizeof(T) == 8, uint64_t, uint32_t>::type;
  cgx_ctx *ctx = A->ctx;
  hipStream_t s = ctx->stream;
  const int64_t nnz = A->dev.nnz;
  const T *val = (const T *)A->dev.val;
  std::vector<B> dict;
  auto add = [&](const T *v, size_t cnt) {
    for (size_t i = 0; i < cnt; ++i) {
      B b;
      std::memcpy(&b, v + i, sizeof(B));
      auto it = std::lower_bound(dict.begin(), dict.end(), b);
      if (it == dict.end() || *it != b) {
        if ((int)dict.size() == kVcMax) return false;
        dict.insert(it, b);
      }
    }
    return true;
  };
  {  // sample: 64 pieces of up to 1024 values
    constexpr int64_t kPieces = 64, kPiece = 1024;
    std::vector<T> h((size_t)std::min<int64_t>(nnz, kPieces * kPiece));
    if ((int64_t)h.size() == nnz) {
      CGX_HIP(hipMemcpyAsync(h.data(), val, h.size() * sizeof(T), hipMemcpyDeviceToHost, s));
    } else {
      for (int64_t q = 0; q < kPieces; ++q) {
        const int64_t at = (nnz - kPiece) * q / (kPieces - 1);
        CGX_HIP(hipMemcpyAsync(h.data() + q * kPiece, val + at, kPiece * sizeof(T),
                               hipMemcpyDeviceToHost, s));
      }
    }
    CGX_HIP(hipStreamSynchronize(s));
    if (!add(h.data(), h.size())) return CGX_OK;
  }
  int64_t chunks = 0;
  {
    std::vector<SellSlice> last(1);
    CGX_HIP(hipMemcpyAsync(last.data(), A->dev.sl + (A->dev.nsl - 1), sizeof(SellSlice),
                           hipMemcpyDeviceToHost, s));
    CGX_HIP(hipStreamSynchronize(s));
    chunks = last[0].ioff + kSellRows * ((last[0].width + 7) / 8);
  }
  void *codes = nullptr, *ddict = nullptr, *dmiss = nullptr;
  hipError_t e = hipMalloc(&codes, (size_t)chunks * 16);
  if (e == hipSuccess) e = hipMalloc(&ddict, kVcDict * sizeof(T));
  if (e == hipSuccess) e = hipMalloc(&dmiss, sizeof(int) + kVcDict * sizeof(T) + 16);
  bool ok = false;
  for (int pass = 0; pass < 16 && e == hipSuccess; ++pass) {
    std::vector<T> hd(kVcDict, T(0));
    std::memcpy(hd.data(), dict.data(), dict.size() * sizeof(T));
    e = hipMemcpyAsync(ddict, hd.data(), kVcDict * sizeof(T), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemsetAsync(dmiss, 0, sizeof(int), s);
    if (e == hipSuccess)
      e = Launch<T>::sellpv_pack(A->dev, val, (const T *)ddict, (int)dict.size(),
                                 (unsigned char *)codes, (int *)dmiss,
                                 (T *)((char *)dmiss + 16), s);
    int nmiss = 0;
    std::vector<T> mv(kVcDict);
    if (e == hipSuccess)
      e = hipMemcpyAsync(&nmiss, dmiss, sizeof(int), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess)
      e = hipMemcpyAsync(mv.data(), (char *)dmiss + 16, kVcDict * sizeof(T),
                         hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) break;
    if (nmiss == 0) {
      ok = true;
      break;
    }
    if (!add(mv.data(), (size_t)std::min(nmiss, kVcDict))) break;
  }
  if (dmiss) (void)hipFree(dmiss);
  if (e != hipSuccess || !ok) {
    if (codes) (void)hipFree(codes);
    if (ddict) (void)hipFree(ddict);
    if (e != hipSuccess) return hip_fail(e, "cgx_csr_create(value codes)");
    return CGX_OK;
  }
  A->d_sell_vc = codes;
  A->d_sell_vdict = ddict;
  A->dev.svc = codes;
  A->dev.svdict = ddict;
  A->dev.nvdict = (int)dict.size();
  A->vc_chunks = chunks;
  if ((int)dict.size() <= kVc4Max) {  // 4-bit codes: half the code stream
    void *c4 = nullptr;
    e = hipMalloc(&c4, (size_t)chunks * 8);
    if (e == hipSuccess) e = Launch<T>::vc_narrow(codes, c4, chunks, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
      if (c4) (void)hipFree(c4);
      return hip_fail(e, "cgx_csr_create(4-bit value codes)");
    }
    A->d_sell_vc4 = c4;
    A->dev.svc4 = c4;
  }
  return CGX_OK;
}

// Value-code templates (cgx_internal.h kVT): the kVtMax most
// frequent 4-bit code chunks that at least kVtMin slices share (hashes on
// the device, counted here), and the template slice table in which every
// slice whose chunk equals one of them byte for byte (checked on the
// device) points at it. The matrix then also has the kVT forms; the
// autotune decides. $CGX_VT=0 skips it. Errors are device failures only.
static int build_value_templates(cgx_csr *A) {
  constexpr int64_t kVtMin = 64;
  if (!A->dev.svc4 || A->dev.sell_maxw > 8 || A->dev.nsl < kVtMin) return CGX_OK;
  if (const char *env = std::getenv("CGX_VT"))
    if (std::atoi(env) == 0) return CGX_OK;
  hipStream_t s = A->ctx->stream;
  const int64_t nsl = A->dev.nsl;
  unsigned long long *dh = nullptr;
  CGX_HIP(hipMalloc(&dh, (size_t)nsl * 8));
  std::vector<unsigned long long> h((size_t)nsl);
  hipError_t e = vc_hash(A->dev, dh, s);
  if (e == hipSuccess)
    e = hipMemcpyAsync(h.data(), dh, (size_t)nsl * 8, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(dh);
  if (e != hipSuccess) return hip_fail(e, "cgx_csr_create(template hashes)");
  std::unordered_map<unsigned long long, std::pair<int64_t, int64_t>> cnt;  // count, first slice
  for (int64_t q = 0; q < nsl; ++q)
    if (h[q]) {
      auto it = cnt.try_emplace(h[q], 0, q).first;
      it->second.first += 1;
    }
  std::vector<std::pair<int64_t, int64_t>> top;  // (count, slice)
  for (const auto &kv : cnt)
    if (kv.second.first >= kVtMin) top.push_back(kv.second);
  std::sort(top.begin(), top.end(), [](const auto &a, const auto &b) {
    return a.first != b.first ? a.first > b.first : a.second < b.second;
  });
  if (top.size() > (size_t)kVtMax) top.resize(kVtMax);
  if (top.empty()) return CGX_OK;
  const int nt = (int)top.size();
  void *vct = nullptr, *slt = nullptr, *dcnt = nullptr;
  e = hipMalloc(&vct, (size_t)nt * 64 * 8);
  if (e == hipSuccess) e = hipMalloc(&slt, (size_t)nsl * sizeof(SellSlice));
  if (e == hipSuccess) e = hipMalloc(&dcnt, sizeof(unsigned));
  if (e == hipSuccess) e = hipMemsetAsync(dcnt, 0, sizeof(unsigned), s);
  for (int t = 0; t < nt && e == hipSuccess; ++t) {  // template t: slice top[t]'s chunk
    SellSlice m;
    e = hipMemcpyAsync(&m, A->dev.sl + top[t].second, sizeof(m), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess)
      e = hipMemcpyAsync((char *)vct + (size_t)t * 512,
                         (const unsigned long long *)A->dev.svc4 + m.ioff, 512,
                         hipMemcpyDeviceToDevice, s);
  }
  unsigned matched = 0;
  if (e == hipSuccess)
    e = vc_match(A->dev, (const unsigned long long *)vct, nt, (SellSlice *)slt, (unsigned *)dcnt, s);
  if (e == hipSuccess) e = hipMemcpyAsync(&matched, dcnt, sizeof(unsigned), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (dcnt) (void)hipFree(dcnt);
  if (e != hipSuccess) {
    if (vct) (void)hipFree(vct);
    if (slt) (void)hipFree(slt);
    return hip_fail(e, "cgx_csr_create(value-code templates)");
  }
  A->d_vct = vct;
  A->d_sell_sl_t = slt;
  A->dev.vct = vct;
  A->dev.sl_t = (const SellSlice *)slt;
  A->dev.nvt = nt;
  A->vt_slices = matched;
  return CGX_OK;
}

// Lean stencil walk (cgx_internal.h kVL): the class of every
// template slice whose pattern is a subset of the stencil's {-D, -a, -1, 0,
// +1, +a, +D} and whose template chunk holds one value per slot for every row
// (absent only at the x-line ends' -1 of lane 0 row 0 and +1 of lane 63 row
// 1, with that slot's value finite), in slice order; the class table; D and
// a, taken from the most frequent 7-wide (or, 2-D, 5-wide) stencil pattern
// of the template slices. Host work over the slice table; returns CGX_OK
// with no classes when the matrix has none. Single-device matrices only.
static int build_lean_classes(cgx_csr *A, std::vector<VlClass> &tab) {
  tab.clear();
  A->vl_slice_cls.clear();
  const CsrDev &d = A->dev;
  if (!d.sl_t || !d.vct || d.nvt < 1 || !d.svc4 || !d.svdict || d.sell_maxw > 8 ||
      A->sell_pool.empty() || (uint64_t)(d.n + 2) * dtype_size(A->dtype) >= (uint64_t(1) << 32))
    return CGX_OK;
  hipStream_t s = A->ctx->stream;
  const int64_t nsl = d.nsl;
  std::vector<SellSlice> sl((size_t)nsl);
  std::vector<unsigned long long> chunks((size_t)d.nvt * 64);
  std::vector<double> vd(kVcDict);
  std::vector<float> vdf;
  CGX_HIP(hipMemcpyAsync(sl.data(), d.sl_t, (size_t)nsl * sizeof(SellSlice),
                         hipMemcpyDeviceToHost, s));
  CGX_HIP(hipMemcpyAsync(chunks.data(), d.vct, chunks.size() * 8, hipMemcpyDeviceToHost, s));
  if (A->dtype == CGX_F32) {
    vdf.resize(kVcDict);
    CGX_HIP(hipMemcpyAsync(vdf.data(), d.svdict, kVcDict * sizeof(float), hipMemcpyDeviceToHost,
                           s));
  } else {
    CGX_HIP(hipMemcpyAsync(vd.data(), d.svdict, kVcDict * sizeof(double), hipMemcpyDeviceToHost,
                           s));
  }
  CGX_HIP(hipStreamSynchronize(s));
  if (!vdf.empty())
    for (int k = 0; k < kVcDict; ++k) vd[k] = (double)vdf[k];
  const std::vector<int> &pool = A->sell_pool;
  auto offs = [&](const SellSlice &m, int j) { return pool[(size_t)m.dict + j]; };
  // the stencil: (D, a) of the most frequent full pattern among template slices
  std::map<std::pair<int, int>, int64_t> freq;
  for (const SellSlice &m : sl) {
    const int W = m.width & kVtWidthMask;
    if ((m.width >> 16) == 0) continue;
    if (W == 7 && offs(m, 2) == -1 && offs(m, 3) == 0 && offs(m, 4) == 1 &&
        offs(m, 1) == -offs(m, 5) && offs(m, 0) == -offs(m, 6) && offs(m, 5) > 1 &&
        offs(m, 6) > offs(m, 5))
      ++freq[{offs(m, 6), offs(m, 5)}];
    else if (W == 5 && offs(m, 1) == -1 && offs(m, 2) == 0 && offs(m, 3) == 1 &&
             offs(m, 0) == -offs(m, 4) && offs(m, 4) > 1)
      ++freq[{offs(m, 4), 0}];
  }
  if (freq.empty()) return CGX_OK;
  auto best = freq.begin();
  for (auto it = freq.begin(); it != freq.end(); ++it)
    if (it->second > best->second) best = it;
  const int D = best->first.first, a = best->first.second;
  // canonical slot of offset o (-1: none)
  auto canon = [&](int o) {
    if (o == -D) return 0;
    if (a > 0 && o == -a) return 1;
    if (o == -1) return 2;
    if (o == 0) return 3;
    if (o == 1) return 4;
    if (a > 0 && o == a) return 5;
    if (o == D) return 6;
    return -1;
  };
  // the class of (template t, pattern at pool base pb of width W), or -1
  auto make = [&](int t, int pb, int W, VlClass &c) -> bool {
    std::memset(&c, 0, sizeof(c));
    int slot_of[8];
    bool seen[7] = {};
    for (int j = 0; j < W; ++j) {
      const int q = canon(pool[(size_t)pb + j]);
      if (q < 0 || seen[q]) return false;
      seen[q] = true;
      slot_of[j] = q;
    }
    if (!seen[2] || !seen[3] || !seen[4]) return false;
    const unsigned long long *w = chunks.data() + (size_t)t * 64;
    auto code = [&](int l, int j, int r) { return (unsigned)(w[l] >> (8 * j + 4 * r)) & 0xfu; };
    for (int j = W; j < 8; ++j)  // slots past the pattern: empty in every row
      for (int l = 0; l < 64; ++l)
        if (code(l, j, 0) != 0xfu || code(l, j, 1) != 0xfu) return false;
    c.plo = c.phi = 1;
    for (int j = 0; j < W; ++j) {
      const int q = slot_of[j];
      int k = -1;
      for (int r = 0; r < 2; ++r)
        for (int l = 0; l < 64; ++l) {
          const unsigned cd = code(l, j, r);
          if (cd == 0xfu) {
            if (q == 2 && r == 0 && l == 0) {
              c.plo = 0;
              continue;
            }
            if (q == 4 && r == 1 && l == 63) {
              c.phi = 0;
              continue;
            }
            return false;
          }
          if (k < 0) k = (int)cd;
          else if ((int)cd != k) return false;  // codes are distinct bit patterns
        }
      if (k < 0) return false;
      c.v[q] = vd[k];
      if (q == 0) c.pres |= 1;
      if (q == 1) c.pres |= 2;
      if (q == 5) c.pres |= 4;
      if (q == 6) c.pres |= 8;
    }
    if ((!c.plo && !std::isfinite(c.v[2])) || (!c.phi && !std::isfinite(c.v[4]))) return false;
    c.zlo = -std::copysign(0.0, c.v[2]);
    c.zhi = -std::copysign(0.0, c.v[4]);
    return true;
  };
  std::map<std::pair<int, int>, int> ids;  // (template, pool base) -> class (-1: none)
  A->vl_slice_cls.assign((size_t)nsl, 0xff);
  int64_t lean = 0;
  for (int64_t q = 0; q < nsl; ++q) {
    const SellSlice &m = sl[(size_t)q];
    const int t = (m.width >> 16) - 1, W = m.width & kVtWidthMask;
    if (t < 0 || (q + 1) * 2 * kSellRows > d.n) continue;  // a template chunk, a full slice
    auto it = ids.find({t, m.dict});
    if (it == ids.end()) {
      VlClass c;
      int id = -1;
      if ((int)tab.size() < kVlMaxCls && make(t, m.dict, W, c)) {
        id = (int)tab.size();
        tab.push_back(c);
      }
      it = ids.emplace(std::make_pair(t, m.dict), id).first;
    }
    if (it->second >= 0) {
      A->vl_slice_cls[(size_t)q] = (unsigned char)it->second;
      ++lean;
    }
  }
  if (lean == 0) {
    tab.clear();
    A->vl_slice_cls.clear();
    return CGX_OK;
  }
  A->dev.vl_D = D;
  A->dev.vl_a = a;
  return CGX_OK;
}

// The classes in the wave-major layout of a G-workgroup launch (G a multiple
// of 8: waves of XCD group g walk its eighth of the slices with step G / 2)
// and the table, on the device; the lean walk is then available at grid G.
static int build_lean_layout(cgx_csr *A, const std::vector<VlClass> &tab, int G) {
  // (G <= kMaxGrid: the walk's p.Ap partials land in RedWs::pap_part, and a
  // split matrix's boundary launch writes its own after them)
  if (A->vl_slice_cls.empty() || tab.empty() || G < 8 || G % 8 || G > kMaxGrid)
    return CGX_EINVAL;
  const int64_t nsl = A->dev.nsl;
  const int step = G / 2;
  // the chunked walk (spmv_lean) where a plane holds several chunks of step
  // slices and every XCD group's eighth is whole planes
  const int D = A->dev.vl_D;
  const int64_t K = D % (2 * kSellRows) == 0 ? D / (2 * kSellRows) : 0;
  const bool chunked = K > step && K % step == 0 && nsl % (8 * K) == 0;
  const int64_t P = chunked ? nsl / 8 / K : 0;
  int64_t nst = 0;
  for (int g = 0; g < 8; ++g) {
    const int64_t lo = (nsl * g) >> 3, end = (nsl * (g + 1)) >> 3;
    nst = std::max<int64_t>(nst, (end - lo + step - 1) / step);
  }
  nst = (nst + 3) & ~int64_t(3);
  // the forward sweep's rows, then the reversed sweep's (slice lo + end - 1 - q)
  std::vector<unsigned char> h((size_t)(2 * 8 * step * nst), 0xff);
  for (int rev = 0; rev < 2; ++rev)
    for (int g = 0; g < 8; ++g) {
      const int64_t lo = (nsl * g) >> 3, end = (nsl * (g + 1)) >> 3;
      for (int w = 0; w < step; ++w) {
        unsigned char *row = h.data() + (size_t)((int64_t)(rev * 8 * step + g * step + w) * nst);
        int64_t j = 0;
        for (int64_t q = lo + w, zp = 0, cb = 0; q < end; ++j) {
          row[j] = A->vl_slice_cls[(size_t)(rev ? lo + end - 1 - q : q)];
          if (!chunked) {
            q += step;
            continue;
          }
          if (++zp == P) {
            zp = 0;
            cb += step;
          }
          q = cb >= K ? end : lo + zp * K + cb + w;
        }
      }
    }
  void *dc = nullptr, *dt = nullptr;
  hipStream_t s = A->ctx->stream;
  hipError_t e = hipMalloc(&dc, h.size());
  if (e == hipSuccess) e = hipMalloc(&dt, tab.size() * sizeof(VlClass));
  if (e == hipSuccess) e = hipMemcpyAsync(dc, h.data(), h.size(), hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = hipMemcpyAsync(dt, tab.data(), tab.size() * sizeof(VlClass), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    if (dc) (void)hipFree(dc);
    if (dt) (void)hipFree(dt);
    return hip_fail(e, "cgx_csr_create(lean stencil classes)");
  }
  for (void *p : {A->d_vl_cls, A->d_vl_tab})
    if (p) (void)hipFree(p);
  A->d_vl_cls = dc;
  A->d_vl_tab = dt;
  A->dev.vl_cls = (const unsigned char *)dc;
  A->dev.vl_tab = (const VlClass *)dt;
  A->dev.vl_grid = G;
  A->dev.vl_nst = (int)nst;
  A->dev.vl_P = (int)P;
  A->dev.vl_K = chunked ? (int)K : 0;
  // the per-slice form's slices: a few (256^3: 8) read the dictionary where
  // it lies; many (512^3: 1,036) are cheaper from an LDS copy
  int64_t generic = 0;
  for (unsigned char c : A->vl_slice_cls) generic += c == 0xff;
  A->dev.vl_lds = generic >= 64 ? 1 : 0;
  A->vl_ncls = (int)tab.size();
  A->vl_tab_h = tab;
  return CGX_OK;
}

// The lean walk's grid: G / 2 waves per XCD step; with the step a plane's
// slices K = D / 128 (or K / 2, K / 4 ...) the +-D gathers are the wave's
// own centers one (two, four) steps away, hits in its XCD's L2. That grid
// when it keeps at least half the resident workgroups, else the resident
// cap (a 2-D stencil's +-D, a few slices away, sit inside any step).
// Measured in the loop (profiles/r04_lean_pipe512.log): 512^3 631 us at the
// plane-matched 1,024 against 665 at 1,280; at 256^3 the two tie (55.8 /
// 56.4 us).
static int lean_grid(const cgx_csr *A) {
  const int res = A->dtype == CGX_F32 ? Launch<float>::lean_resident()
                                      : Launch<double>::lean_resident();
  const int cap = std::max(8, std::min(res, kMaxGrid) / 8 * 8);
  const int D = A->dev.vl_D;
  if (D > 0 && D % (2 * kSellRows) == 0) {
    int G = 2 * (D / (2 * kSellRows));
    while (G > cap && G % 16 == 0) G /= 2;
    if (G <= cap && 2 * G >= cap && G % 8 == 0) return G;
  }
  return cap;
}

// build the lean walk's classes and, at grid G (0: the first candidate), its
// device layout; false when the matrix has no lean slices
static bool build_lean(cgx_csr *A, int G = 0) {
  std::vector<VlClass> tab;
  if (build_lean_classes(A, tab) != CGX_OK || tab.empty()) return false;
  if (G == 0) G = lean_grid(A);
  return build_lean_layout(A, tab, G) == CGX_OK;
}
// A partitioned matrix whose loop SpMV is the lean walk: its boundary slices
// (the split's, run by the boundary launch with the ghosts) become class
// 0xfe, skipped by the walk, and the layout is rebuilt at the same grid; the
// walk then runs the interior slices (spmv_lean_interior). Boundary slices
// never take the whole-matrix walk (vl_whole).
int lean_mark_split(cgx_csr *A, const std::vector<int> &boundary) {
  if (!A->dev.lean || A->vl_slice_cls.empty() || A->vl_tab_h.empty() || boundary.empty())
    return CGX_OK;
  for (int q : boundary)
    if (q >= 0 && (size_t)q < A->vl_slice_cls.size()) A->vl_slice_cls[(size_t)q] = 0xfe;
  const std::vector<VlClass> tab = A->vl_tab_h;
  if (int rc = build_lean_layout(A, tab, A->dev.vl_grid)) return rc;
  A->dev.vl_split = 1;
  return CGX_OK;
}

// the variant under the lean walk: its generic slices' form (4-bit value
// codes on templates, the pipelined stencil walk's requirements)
constexpr int kVlBase = 2050 | 32768 | 262144 | 524288 | 1048576 | kVT;

int build_value_codes(cgx_csr *A) {
  if (!A->dev.sl || !A->dev.sell_kind || A->dev.nsl < 1 || A->dev.nnz < 1) return CGX_OK;
  const int rc =
      A->dtype == CGX_F32 ? build_value_codes_t<float>(A) : build_value_codes_t<double>(A);
  return rc ? rc : build_value_templates(A);
}

// SELL copy of A on the device with R rows per lane (0: the default layout),
// when the matrix qualifies (sell_plan_host); otherwise A keeps only the
// CSR-stream schedule and this returns CGX_OK. Errors are device failures
// only. cgx_csr_set_sell selects R (0 drops the copy).
int build_sell(cgx_csr *A, const int *h_rowptr, const int *h_col, int R,
               const std::vector<char> *skip) {
  // R: 1 / 2 dictionary SELL with R rows per lane, 3 SELL-P (2 rows per
  // lane), 0 the default: SELL-P where the matrix qualifies, else R = 2
  bool fallback = false;
  if (R == 0) {
    R = 3;
    fallback = true;
  }
  free_sell(A);
  const int64_t n = A->dev.n, nnz = A->dev.nnz;
  if (nnz < 1 || A->max_row_nnz > kSellMaxWidth) return CGX_OK;
  cgx_ctx *ctx = A->ctx;
  hipStream_t s = ctx->stream;
  std::vector<SellSlice> sl;
  std::vector<int> pool;
  std::vector<unsigned long long> idx;
  int64_t voff = 0;
  int kind = 0, maxw = 0;
  const int64_t nx = A->dev.n + A->halo.n_ghost;
  if (R == 3) {
    // (the patterns on the device: the host plan's download of the column
    // array and its loop over every entry were most of the setup, round 6)
    bool ok = false;
    if (nx >= 2)
      if (int rc = sellp_plan_device(ctx, n, nnz, A->dev.rowptr, A->dev.col, skip, sl, pool, voff,
                                     maxw, &ok))
        return rc;
    if (ok) {
      kind = maxw <= 8 ? 1 : 2;
      R = 2;
    } else if (fallback) {
      R = 2;
    } else {
      return CGX_OK;
    }
  }
  std::vector<int> hc, hr;
  if (!kind && !h_rowptr) {
    hr.resize((size_t)n + 1);
    CGX_HIP(hipMemcpyAsync(hr.data(), A->dev.rowptr, hr.size() * sizeof(int),
                           hipMemcpyDeviceToHost, s));
    CGX_HIP(hipStreamSynchronize(s));
    h_rowptr = hr.data();
  }
  if (!kind && !h_col) {
    hc.resize((size_t)nnz);
    CGX_HIP(hipMemcpyAsync(hc.data(), A->dev.col, (size_t)nnz * sizeof(int),
                           hipMemcpyDeviceToHost, s));
    CGX_HIP(hipStreamSynchronize(s));
    h_col = hc.data();
  }
  if (!kind && !sell_plan_host(n, h_rowptr, h_col, R, sl, pool, idx, voff)) return CGX_OK;
  const int64_t nsl = (int64_t)sl.size();
  const size_t es = dtype_size(A->dtype);
  hipError_t e = hipMalloc(&A->d_sell_sl, sl.size() * sizeof(SellSlice));
  if (e == hipSuccess) e = hipMalloc(&A->d_sell_dict, pool.size() * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&A->d_sell_idx, std::max<size_t>(idx.size(), 1) * 8);
  if (e == hipSuccess)  // + one chunk of slack: the kernel reads 8 slots per chunk
    e = hipMalloc(&A->d_sell_val, (size_t)(voff + 8 * kSellRows * R) * es);
  if (e == hipSuccess)
    e = hipMemcpyAsync(A->d_sell_sl, sl.data(), sl.size() * sizeof(SellSlice),
                       hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = hipMemcpyAsync(A->d_sell_dict, pool.data(), pool.size() * sizeof(int),
                       hipMemcpyHostToDevice, s);
  if (e == hipSuccess && !idx.empty())
    e = hipMemcpyAsync(A->d_sell_idx, idx.data(), idx.size() * 8, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && kind)  // one mask per row, rows padded to whole slices
    e = hipMalloc(&A->d_sell_mask, (size_t)(nsl * 2 * kSellRows) * (kind == 2 ? 4 : 1));
  if (e != hipSuccess) {
    free_sell(A);
    return hip_fail(e, "cgx_csr_create(SELL copy)");
  }
  // visit order: automatic for single-device matrices whose planes span at
  // least two chunks of 512 slices (the XCD's ~1,024 slices in flight then
  // hold every +-plane gather in its L2: 512^3 SpMV 793 -> 710 us, the
  // iteration 463 -> 483 it/s; profiles/r03m_order_chunk.log). 256^3
  // planes (512 slices) keep the natural order, which is the same walk
  // (chunks of 128 slices, round 2's form, were no faster at 256^3: DESIGN.md
  // §8).
  {
    int64_t P = 0;
    for (int v : pool) P = std::max<int64_t>(P, v < 0 ? -(int64_t)v : v);
    std::vector<int> order;
    if (!A->dist) order = sell_visit_order(nsl, (int64_t)kSellRows * R, P, 512);
    if (!order.empty()) {
      e = hipMalloc(&A->d_sell_order, order.size() * sizeof(int));
      if (e == hipSuccess)
        e = hipMemcpyAsync(A->d_sell_order, order.data(), order.size() * sizeof(int),
                           hipMemcpyHostToDevice, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e != hipSuccess) {
        free_sell(A);
        return hip_fail(e, "cgx_csr_create(SELL order)");
      }
      A->dev.sorder = (const int *)A->d_sell_order;
    }
  }
  A->dev.sl = (const SellSlice *)A->d_sell_sl;
  A->dev.sdict = (const int *)A->d_sell_dict;
  A->dev.sell_partial = (kind && skip) ? 1 : 0;
  A->sell_pool = pool;
  A->dev.sidx = (const unsigned long long *)A->d_sell_idx;
  A->dev.sval = A->d_sell_val;
  A->dev.nsl = nsl;
  A->dev.sell_r = R;
  A->dev.sell_kind = kind;
  A->dev.smask = A->d_sell_mask;
  A->dev.nx = nx;
  A->dev.sell_maxw = 0;
  for (const SellSlice &m : sl) A->dev.sell_maxw = std::max(A->dev.sell_maxw, m.width);
  if (kind == 1) plan_march(sl, pool, nx, dtype_size(A->dtype), A->dev);
  A->sell_padded = voff;
  A->sell_idx_words = (int64_t)idx.size();
  if (kind && A->dtype == CGX_F32)
    e = Launch<float>::sellp_pack(A->dev, (const float *)A->dev.val, (float *)A->d_sell_val,
                                  A->d_sell_mask, s);
  else if (kind)
    e = Launch<double>::sellp_pack(A->dev, (const double *)A->dev.val, (double *)A->d_sell_val,
                                   A->d_sell_mask, s);
  else if (A->dtype == CGX_F32)
    e = Launch<float>::sell_pack(A->dev, (const float *)A->dev.val, (float *)A->d_sell_val, s);
  else
    e = Launch<double>::sell_pack(A->dev, (const double *)A->dev.val, (double *)A->d_sell_val, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);  // host vectors die here
  if (e != hipSuccess) {
    free_sell(A);
    return hip_fail(e, "cgx_csr_create(SELL pack)");
  }
  setup_mark(A, 1);
  if (kind) {
    const char *env = std::getenv("CGX_VALUE_CODES");
    if (!env || std::atoi(env) != 0) return build_value_codes(A);
  }
  return CGX_OK;
}

// The setup cost of cgx_csr_create(_dist) by phase (cgx.h)
extern "C" int cgx_csr_setup_times(cgx_csr *A, double *ms, int cap, int *count) {
  CGX_REQUIRE(A && count, CGX_EINVAL, "NULL argument");
  *count = 6;
  for (int k = 0; k < 6 && k < cap && ms; ++k) ms[k] = A->setup_ms[k];
  return CGX_OK;
}

extern "C" int cgx_csr_set_sell(cgx_csr *A, int rows_per_lane) {
  CGX_REQUIRE(A, CGX_EINVAL, "A is NULL");
  CGX_REQUIRE(rows_per_lane >= 0 && rows_per_lane <= 3, CGX_EINVAL,
              "layout must be 0 (drop the SELL copy), 1 or 2 (dictionary SELL, rows per "
              "lane) or 3 (SELL-P)");
  DeviceGuard g(A->ctx->device);
  if (rows_per_lane == 0) {
    free_sell(A);
    if (A->dev.variant & (2048 | 8192)) A->dev.variant = 0;
    return CGX_OK;
  }
  int rc = build_sell(A, nullptr, nullptr, rows_per_lane);
  if (rc) return rc;
  if (!A->dev.sl && (A->dev.variant & (2048 | 8192))) A->dev.variant = 0;
  return CGX_OK;
}

extern "C" int cgx_csr_stream_bytes(cgx_csr *A, int64_t *bytes) {
  CGX_REQUIRE(A && bytes, CGX_EINVAL, "NULL argument");
  const int v = launch_variant(A->dev, A->dtype);
  const int64_t es = (int64_t)dtype_size(A->dtype), nsl = A->dev.nsl;
  const int64_t desc = nsl * (int64_t)sizeof(SellSlice);
  if (v & kVL) {  // one class byte per slice; the per-slice form's slices: descriptor and
                  // (not templated) chunk
    int64_t gen = 0;
    for (unsigned char c : A->vl_slice_cls) gen += c == 0xff;
    *bytes = 4 * (int64_t)A->dev.vl_grid * A->dev.vl_nst + gen * (int64_t)sizeof(SellSlice) +
             8 * (A->vc_chunks - 64 * A->vt_slices) + 512 * (int64_t)A->dev.nvt +
             (int64_t)A->vl_ncls * (int64_t)sizeof(VlClass);
  } else if ((v & 32768) && (v & kVT))  // template slices read their chunk from LDS
    *bytes = 8 * (A->vc_chunks - 64 * A->vt_slices) + desc + 512 * (int64_t)A->dev.nvt;
  else if (v & 32768)
    *bytes = ((v & 262144) ? 8 : 16) * A->vc_chunks + desc;
  else if (v & 8192)
    *bytes = es * A->sell_padded + nsl * 2 * kSellRows * ((v & 16384) ? 4 : 1) + desc;
  else if (v & 2048)
    *bytes = es * A->sell_padded + 8 * A->sell_idx_words + desc;
  else if (v & kIL)  // the interleaved copy's pairs (a block's first pair may be shared)
    *bytes = (2 * es + 8) * ((A->dev.nnz + 1) / 2) + 4 * (A->dev.n + 1);
  else
    *bytes = (es + ((v & kC16) ? 2 : 4)) * A->dev.nnz + 4 * (A->dev.n + 1);
  return CGX_OK;
}

extern "C" int cgx_csr_value_codes(cgx_csr *A, int *n_values) {
  CGX_REQUIRE(A && n_values, CGX_EINVAL, "NULL argument");
  *n_values = A->dev.svc ? A->dev.nvdict : 0;
  return CGX_OK;
}

extern "C" int cgx_csr_templates(cgx_csr *A, int *n_templates, int64_t *slices) {
  CGX_REQUIRE(A && n_templates && slices, CGX_EINVAL, "NULL argument");
  *n_templates = A->dev.sl_t ? A->dev.nvt : 0;
  *slices = A->dev.sl_t ? A->vt_slices : 0;
  return CGX_OK;
}

extern "C" int cgx_csr_lean_info(cgx_csr *A, int *classes, int64_t *slices, int *grid, int *D,
                                 int *a, int *chunked) {
  CGX_REQUIRE(A && classes && slices && grid && D && a && chunked, CGX_EINVAL,
              "NULL argument");
  *chunked = A->dev.vl_cls && A->dev.vl_P > 0 ? 1 : 0;
  const bool on = A->dev.vl_cls != nullptr;
  int64_t cnt = 0;
  if (on)
    for (unsigned char c : A->vl_slice_cls) cnt += c < 0xfe;  // 0xff / 0xfe: not lean
  *classes = on ? A->vl_ncls : 0;
  *slices = cnt;
  *grid = on ? A->dev.vl_grid : 0;
  *D = on ? A->dev.vl_D : 0;
  *a = on ? A->dev.vl_a : 0;
  return CGX_OK;
}

extern "C" int cgx_csr_autotune_record(cgx_csr *A, int *variants, int *kinds, float *us,
                                       int cap, int *count) {
  CGX_REQUIRE(A && count && cap >= 0, CGX_EINVAL, "bad argument");
  CGX_REQUIRE(cap == 0 || (variants && kinds && us), CGX_EINVAL, "NULL output array");
  *count = (int)A->tune.size();
  for (int i = 0; i < cap && i < *count; ++i) {
    variants[i] = A->tune[(size_t)i].variant;
    kinds[i] = A->tune[(size_t)i].kind;
    us[i] = A->tune[(size_t)i].us;
  }
  return CGX_OK;
}

extern "C" int cgx_csr_set_lean_team(cgx_csr *A, int on) {
  CGX_REQUIRE(A, CGX_EINVAL, "A is NULL");
  CGX_REQUIRE(!on || (A->dev.vl_cls && !A->dev.vl_split && !A->dev.sell_partial &&
                      A->dev.vl_grid % 32 == 0 && A->dtype == CGX_F64),
              CGX_EUNSUPPORTED,
              "the team walk needs an f64 whole-matrix lean layout whose grid is a multiple "
              "of 32");
  A->dev.vl_team = on ? 1 : 0;
  return CGX_OK;
}

extern "C" int cgx_csr_lean_team(cgx_csr *A, int *on) {
  CGX_REQUIRE(A && on, CGX_EINVAL, "NULL argument");
  *on = A->dev.vl_cls && A->dev.vl_team ? 1 : 0;
  return CGX_OK;
}

extern "C" int cgx_csr_march_info(cgx_csr *A, int *stride, int *offset_a, int *run_planes) {
  CGX_REQUIRE(A && stride && offset_a && run_planes, CGX_EINVAL, "NULL argument");
  const bool on = A->dev.svc && A->dev.sell_maxw <= 8 && A->dev.march_k > 0;
  *stride = on ? A->dev.march_k : 0;
  *offset_a = on ? A->dev.march_a : 0;
  *run_planes = on ? A->dev.march_len : 0;
  return CGX_OK;
}

extern "C" int cgx_csr_visit_order(cgx_csr *A, int *ordered) {
  CGX_REQUIRE(A && ordered, CGX_EINVAL, "NULL argument");
  *ordered = A->dev.sorder ? 1 : (A->split_ni > 0 && A->split_ordered) ? 2 : 0;
  return CGX_OK;
}

extern "C" int cgx_csr_sell_info(cgx_csr *A, int *has_sell, int64_t *padded) {
  CGX_REQUIRE(A, CGX_EINVAL, "A is NULL");
  if (has_sell) *has_sell = !A->dev.sl ? 0 : (A->dev.sell_kind ? 3 : A->dev.sell_r);
  if (padded) *padded = A->sell_padded;
  return CGX_OK;
}

// A request names a form k_spmv_dot is instantiated for (CGX_SPMV_LIST,
// the forms cgx_csr_variant reports) or one of the request forms below,
// which resolve to such a form on a matrix with the right copies (the
// checks in cgx_csr_set_variant); the lean walk is handled before this.
static bool known_variant(int v) {
  static const int ok[] = {0,  1,  2,  3,  4,  5,  6,  7,  12, 13, 14, 15, 133, 135, 264, 265, 266,
                           267, 2048, 2050, 2056, 2058, 6144, 6146, 8192, 8194, 24576, 24578,
                           34816, 34818, 40960, 40962, 296960, 296962, 559104, 559106,
                           821248, 821250, 1607680, 1607682, 1869824, 1869826,
                           9209856, 9209858, 10258434, 12355584, 12355586, 10258432};
  for (int k : ok)
    if (k == v) return true;
  return spmv_listed(v);
}

extern "C" int cgx_csr_set_variant(cgx_csr *A, int variant) {
  CGX_REQUIRE(A, CGX_EINVAL, "A is NULL");
  if (variant & kVL) {  // the lean stencil walk (at its first grid candidate unless built)
    CGX_REQUIRE((variant & ~kVL) == 0 || (variant & ~kVL) == kVlBase ||
                    (variant & ~kVL) == ((kVlBase & ~2048) | 8192),
                CGX_EINVAL, "unknown SpMV variant %d (the lean walk is %d)", variant,
                kVL | kVlBase);
    CGX_REQUIRE(A->dev.sl_t, CGX_EUNSUPPORTED,
                "variant %d needs value-code templates, which this matrix does not have",
                variant);
    DeviceGuard g(A->ctx->device);
    if (!A->dev.vl_cls) {
      CGX_REQUIRE(build_lean(A), CGX_EUNSUPPORTED,
                  "variant %d: no slice of this matrix qualifies for the lean stencil walk",
                  variant);
    }
    A->dev.variant = kVlBase;
    A->dev.lean = true;
    // a split partitioned matrix: the walk runs its interior only (the
    // boundary slices class 0xfe), as cgx_csr_create_dist leaves it
    if (A->split_ni > 0 && !A->dev.vl_split) {
      if (int rc = lean_mark_split(A, A->split_bd_h)) return rc;
    }
    return CGX_OK;
  }
  A->dev.lean = false;
  // (a SELL-family request resolves against the matrix's layout, as the
  // autotune's own candidates do; the check below refuses one with no kernel)
  constexpr int kSellBits = 2 | 16 | 2048 | 4096 | 8192 | 16384 | 32768 | 262144 | 524288 |
                            1048576 | 2097152 | kVT;
  CGX_REQUIRE(known_variant(variant) ||
                  ((variant & (2048 | 8192)) && (variant & ~kSellBits) == 0),
              CGX_EINVAL, "unknown SpMV variant %d", variant);
  CGX_REQUIRE(!(variant & (2048 | 8192)) || A->dev.sl, CGX_EUNSUPPORTED,
              "variant %d needs the SELL-64 copy, which this matrix does not have", variant);
  CGX_REQUIRE(!(variant & 32768) || A->dev.svc, CGX_EUNSUPPORTED,
              "variant %d needs SELL-P value codes, which this matrix does not have", variant);
  CGX_REQUIRE(!(variant & 262144) || A->dev.svc4, CGX_EUNSUPPORTED,
              "variant %d needs 4-bit value codes (at most 15 distinct values)", variant);
  CGX_REQUIRE(!(variant & kVT) || A->dev.sl_t, CGX_EUNSUPPORTED,
              "variant %d needs value-code templates, which this matrix does not have", variant);
  if (variant & kIL) {
    DeviceGuard g(A->ctx->device);
    CGX_REQUIRE(build_il(A), CGX_EUNSUPPORTED,
                "variant %d: the interleaved val / col copy could not be built", variant);
  }
  if ((variant & kC16) && !(variant & 8192)) {
    DeviceGuard g(A->ctx->device);
    CGX_REQUIRE(build_col16(A), CGX_EUNSUPPORTED,
                "variant %d needs 16-bit column deltas: a column of this matrix lies more than "
                "32767 rows from its row block's first row", variant);
  }
  // the bit mask is not enough: check the form the request resolves to on
  // this matrix has a kernel (e.g. 2138112, plane march without the pipe
  // bits, has none)
  const int old = A->dev.variant;
  A->dev.variant = variant;
  if (!launch_variant_ok(A->dev, A->dtype)) {
    const int resolved = launch_variant(A->dev, A->dtype);
    A->dev.variant = old;
    set_error("SpMV variant %d resolves to %d on this matrix, which has no kernel", variant,
              resolved);
    return CGX_EINVAL;
  }
  return CGX_OK;
}

// Pick the SpMV variant for this matrix on this device: the measured best
// differs by matrix (non-temporal val/col loads help the 2-D 5-point matrix,
// cost the 3-D 7-point one; the SELL-64 copy, where the matrix has one,
// streams 9 B per entry instead of 12) and is cheap to measure — a
// few launches on scratch vectors. $CGX_SPMV_VARIANT forces a variant. The
// SELL copy is freed when a CSR-stream variant wins.
//
// Every candidate is timed in kTuneRounds interleaved rounds (3 launches
// each after one warm-up launch) and scored by its median round. The
// candidates are ranked by preference (the most specialised form first: the
// lean walk, then the value-code forms with templates ... down to plain
// CSR-stream), and a candidate displaces the preferred one only when its
// median is at least kTuneMargin faster: two forms within a few percent of
// each other no longer flip with a box's momentary state (VERDICT r4:
// 565250 in one rep, 10264578 in the next of the same command). The record
// (every candidate's median µs per launch) is kept on the matrix
// (cgx_csr_autotune_record).
//
// A partitioned matrix whose SELL copy is split (interior slices without
// ghost columns, boundary slices with: cgx_dist.cpp) is timed on what its
// loop runs there: the SELL forms over the interior slice list, the lean
// walk over the interior slices (boundary slices class 0xfe).
constexpr int kTuneRounds = 5;
constexpr float kTuneMargin = 0.03f;

static int tune_pick(const std::vector<float> &med) {  // med in preference order
  int inc = 0;
  for (int i = 1; i < (int)med.size(); ++i)
    if (med[(size_t)i] < med[(size_t)inc] * (1.0f - kTuneMargin)) inc = i;
  return inc;
}

static float median_of(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 1e30f : v[v.size() / 2];
}

// the boundary slices of a split matrix marked 0xfe in its lean class list
// and the layout rebuilt at grid G (lean_mark_split without the lean flag)
static int lean_split_layout(cgx_csr *A, int G) {
  for (int q : A->split_bd_h)
    if (q >= 0 && (size_t)q < A->vl_slice_cls.size()) A->vl_slice_cls[(size_t)q] = 0xfe;
  const std::vector<VlClass> tab = A->vl_tab_h;
  if (int rc = build_lean_layout(A, tab, G)) return rc;
  A->dev.vl_split = 1;
  return CGX_OK;
}

int autotune_spmv(cgx_csr *A) {
  A->tune.clear();
  if (const char *env = std::getenv("CGX_SPMV_VARIANT")) {
    // the same checks as cgx_csr_set_variant: a mistyped value fails here,
    // not later as a kernel launch error; "V:G" forces the lean walk's grid
    const int v = std::atoi(env);
    const char *colon = std::strchr(env, ':');
    const int G = colon ? std::atoi(colon + 1) : 0;
    if (cgx_csr_set_variant(A, v) != CGX_OK) {
      const std::string why = g_err;
      set_error("$CGX_SPMV_VARIANT=%s: %s", env, why.c_str());
      return CGX_EINVAL;
    }
    if ((v & kVL) && colon) {  // "V:G" (G 0: the first grid candidate)
      std::vector<VlClass> tab;
      if (build_lean_classes(A, tab) != CGX_OK || tab.empty() ||
          build_lean_layout(A, tab, G > 0 ? G : lean_grid(A)) != CGX_OK) {
        set_error("$CGX_SPMV_VARIANT=%s: no lean walk at grid %d", env, G);
        return CGX_EINVAL;
      }
    }
    if (!(v & (2048 | 8192 | kVL))) free_sell(A);
    return CGX_OK;
  }
  const int64_t bytes = A->dev.nnz * (int64_t)(dtype_size(A->dtype) + sizeof(int));
  if (bytes < (int64_t(64) << 20)) {  // small: the size heuristic, SELL where built
    if (A->dev.sl)
      A->dev.variant = (A->dev.svc4 ? (2048 | 32768 | 262144) : A->dev.svc ? (2048 | 32768) : 2048) |
                       (A->dev.svc && A->dev.sell_maxw <= 8 ? 524288 | 1048576 : 0);
    return CGX_OK;
  }
  // (the software-pipelined SELL forms, 2056/2058, measured slower than the
  // plain ones on MI355X: profiles/r01_tune_sell.log; reachable by request)
  // A matrix stream far beyond the 256 MB Infinity Cache is never re-read
  // from it, and inside the CG loop its non-temporal form keeps p and the
  // vectors the other kernels hand over cached: 512^3 ran 305 it/s with nt
  // against 281 with default-policy loads, a choice the isolated timing below
  // cannot see (it ran both within 1%). Such matrices tune the format only.
  const bool big = bytes > (int64_t(512) << 20);
  // cache-resident CSR also tries the unpipelined paired loop (5) and the
  // quad loads (265): the G3 stand-in's SpMV runs 23.6 / 23.8 us in them
  // against 25.3 in the pipelined 13 (profiles/r02_irr_variants.log)
  std::vector<int> cands = big ? std::vector<int>{15} : std::vector<int>{13, 15, 5, 265};
  // and the paired loop on 16-bit column deltas (10 B per entry) where they fit
  if (!big && build_col16(A)) cands.push_back(133);
  // (the pipelined paired loop on the interleaved val / col copy, kIL, is
  // not a candidate: 376 against 373 us at 256^3, 25.3 against 24.9 on the
  // G3 stand-in, 306 against 297 at 4096^2, its stream-only ablation 336
  // against 324 — profiles/r6f_tune_il_*.log; reachable by request)
  if (A->dev.sl) {
    if (!big) cands.push_back(2048);
    cands.push_back(2050);
  }
  // SELL-P value codes: 1 B per slot instead of 8 (4-bit codes: 0.5 B), and
  // their software-pipelined loop (bit 524288) where no slice is over 8 wide,
  // that loop with the +-1 neighbours taken from the adjacent lanes (bit
  // 1048576: one gather pair fewer per offset -1 / +1)
  for (int c4 : {0, 262144}) {
    if (!A->dev.svc || (c4 && !A->dev.svc4)) continue;
    // (a y-march form measured 93-124 us against 72 for the templated
    // consecutive walk at 256^3, profiles/r03_ymarch_tune.log: removed)
    for (int pipe : {0, 524288, 524288 | 1048576, 524288 | 1048576 | 2097152,
                     524288 | kVT, 524288 | 1048576 | kVT, 524288 | 1048576 | 2097152 | kVT}) {
      if (pipe && A->dev.sell_maxw > 8) continue;
      if ((pipe & 2097152) && A->dev.march_k < 1) continue;
      if ((pipe & kVT) && (!c4 || !A->dev.sl_t)) continue;
      if (!big) cands.push_back(2048 | 32768 | c4 | pipe);
      cands.push_back(2050 | 32768 | c4 | pipe);
    }
  }
  // preference order: the most specialised form first (the list above grows
  // in that direction)
  std::reverse(cands.begin(), cands.end());
  // a split partitioned matrix: the SELL forms time its interior slice list
  const bool split = A->dist && A->d_split && A->split_ni > 0 && A->dev.sl;
  cgx_ctx *ctx = A->ctx;
  hipStream_t s = ctx->stream;
  const size_t es = dtype_size(A->dtype);
  const size_t nx = (size_t)(A->dev.n + A->halo.n_ghost);
  void *x = nullptr, *y = nullptr, *st = nullptr;
  hipError_t e = hipMalloc(&x, nx * es);
  if (e == hipSuccess) e = hipMalloc(&y, nx * es);
  if (e == hipSuccess) e = hipMalloc(&st, sizeof(CgScalars<double>));
  if (e == hipSuccess) e = hipMemsetAsync(x, 0, nx * es, s);
  if (e == hipSuccess) e = hipMemsetAsync(st, 0, sizeof(CgScalars<double>), s);
  const int one = 1;
  const size_t off = A->dtype == CGX_F32 ? offsetof(CgScalars<float>, active)
                                         : offsetof(CgScalars<double>, active);
  if (e == hipSuccess) e = hipMemcpyAsync((char *)st + off, &one, sizeof(int), hipMemcpyHostToDevice, s);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  // one launch of candidate form `how` (0: k_spmv_dot of dv's variant over
  // the matrix or, split, its interior slices; 1: the lean walk (interior
  // when split); 2: k_spmv_fd)
  void *ap = nullptr;
  bool err_set = false;
  auto launch = [&](const CsrDev &dv, int how) -> hipError_t {
    if (A->dtype == CGX_F32) {
      CgScalars<float> *sf = (CgScalars<float> *)st;
      RedWs<float> *wf = (RedWs<float> *)ctx->ws;
      if (how == 3)
        return Launch<float>::spmv_dot_rows(A->dev, A->d_bnd_blk, A->bnd_nblk, 0, (const float *)x,
                                            (float *)y, sf, 0, wf, s, nullptr);
      if (how == 1)
        return split ? Launch<float>::spmv_lean_interior(dv, (const float *)x, (float *)y, sf, 0,
                                                         wf, s, 0, nullptr, 0)
                     : Launch<float>::spmv_dot(dv, (const float *)x, (float *)y, sf, 0, wf, s);
      if (split && (dv.variant & (2048 | 8192)))
        return Launch<float>::spmv_dot_slices(dv, A->d_split, A->split_ni, 0, (const float *)x,
                                              (float *)y, sf, 0, wf, s);
      return Launch<float>::spmv_dot_variant(dv.variant, dv, (const float *)x, (float *)y, sf,
                                             wf, s);
    }
    CgScalars<double> *sd = (CgScalars<double> *)st;
    RedWs<double> *wd = (RedWs<double> *)ctx->ws;
    if (how == 3)
      return Launch<double>::spmv_dot_rows(A->dev, A->d_bnd_blk, A->bnd_nblk, 0,
                                           (const double *)x, (double *)y, sd, 0, wd, s, nullptr);
    if (how == 2)
      return Launch<double>::spmv_fd(dv, (const double *)x, (const double *)x, (double *)y,
                                     (double *)ap, sd, 0, wd, Launch<double>::update_parts(A->dev.n),
                                     s);
    if (how == 1)
      return split ? Launch<double>::spmv_lean_interior(dv, (const double *)x, (double *)y, sd, 0,
                                                        wd, s, 0, nullptr, 0)
                   : Launch<double>::spmv_dot(dv, (const double *)x, (double *)y, sd, 0, wd, s);
    if (split && (dv.variant & (2048 | 8192)))
      return Launch<double>::spmv_dot_slices(dv, A->d_split, A->split_ni, 0, (const double *)x,
                                             (double *)y, sd, 0, wd, s);
    return Launch<double>::spmv_dot_variant(dv.variant, dv, (const double *)x, (double *)y, sd, wd,
                                            s);
  };
  // interleaved rounds over the forms; per form the median round's µs per
  // launch (3 launches after a warm-up one)
  auto time_forms = [&](const std::vector<CsrDev> &forms, const std::vector<int> &how,
                        std::vector<float> &med) {
    std::vector<std::vector<float>> t(forms.size());
    for (int round = 0; round < kTuneRounds && e == hipSuccess; ++round)
      for (size_t ci = 0; ci < forms.size() && e == hipSuccess; ++ci) {
        float tot = 0;
        for (int rep = 0; rep < 4 && e == hipSuccess; ++rep) {
          if (rep == 1) e = hipEventRecord(e0, s);
          if (e == hipSuccess) e = launch(forms[ci], how[ci]);
        }
        if (e == hipSuccess) e = hipEventRecord(e1, s);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        if (e == hipSuccess) e = hipEventElapsedTime(&tot, e0, e1);
        if (e == hipSuccess) t[ci].push_back(tot * 1e3f / 3);
        if (e != hipSuccess && !err_set) {
          set_error("cgx_csr_create: SpMV autotune candidate %d (resolved %d) failed: %s",
                    forms[ci].variant, launch_variant(forms[ci], A->dtype), hipGetErrorString(e));
          err_set = true;
        }
      }
    med.resize(forms.size());
    for (size_t ci = 0; ci < forms.size(); ++ci) med[ci] = median_of(t[ci]);
  };
  std::vector<CsrDev> forms;
  std::vector<int> how;
  for (int v : cands) {
    CsrDev dv = A->dev;  // the candidate as the matrix's variant (kVT: template slice table)
    dv.variant = v;
    dv.lean = false;
    forms.push_back(dv);
    how.push_back(0);
  }
  // A split matrix's boundary rows run as their own CSR-stream launch beside
  // a SELL or lean interior, while a CSR-stream pick runs the whole matrix in
  // one launch: the boundary launch is timed in the same rounds and added to
  // the interior forms before the pick
  const bool bnd_rows = split && A->d_bnd_blk && A->bnd_nblk > 0;
  if (bnd_rows) {
    forms.push_back(A->dev);
    how.push_back(3);
  }
  std::vector<float> med;
  time_forms(forms, how, med);
  const float bnd_us = bnd_rows && e == hipSuccess ? med.back() : 0.0f;
  if (bnd_rows && e == hipSuccess) med.pop_back();
  auto interior = [&](int v) { return split && (v & (2048 | 8192)); };
  int best_v = 0;
  float best_us = 1e30f;
  if (e == hipSuccess) {
    std::vector<float> pick = med;
    for (size_t ci = 0; ci < cands.size(); ++ci)
      if (interior(cands[ci])) pick[ci] += bnd_us;
    const int k = tune_pick(pick);
    best_v = cands[(size_t)k];
    best_us = pick[(size_t)k];
    for (size_t ci = 0; ci < cands.size(); ++ci)
      A->tune.push_back({cands[ci], interior(cands[ci]) ? CGX_TUNE_DOT_INTERIOR : CGX_TUNE_DOT,
                         med[ci]});
    if (bnd_rows) A->tune.push_back({13, CGX_TUNE_BOUNDARY, bnd_us});
  }
  // A 2-D plane-march winner runs the loop as mode 4 (fd_auto), i.e. as
  // k_spmv_fd, whose register budget differs from k_spmv_dot's: with value-
  // code templates it holds 3 waves per SIMD against 2 (152 against 169
  // VGPRs) while k_spmv_dot loses one (profiles/r03_vt3.log: 4096^2 loop
  // 95-99 against 103-104 us, isolated k_spmv_dot 58.6 against 54.2). The
  // march and its template form are therefore decided on their fd kernels
  // (the template form preferred).
  if (e == hipSuccess && !split && A->dtype == CGX_F64 && (best_v & 2097152) &&
      !(best_v & kVT) && A->dev.march_k > 0 && A->dev.march_a == 0 && A->dev.sl_t) {
    e = hipMalloc(&ap, nx * es);
    std::vector<CsrDev> fdf(2, A->dev);
    fdf[0].variant = best_v | kVT;
    fdf[1].variant = best_v;
    std::vector<float> fm;
    if (e == hipSuccess) time_forms(fdf, {2, 2}, fm);
    if (e == hipSuccess) {
      for (int k = 0; k < 2; ++k) A->tune.push_back({fdf[(size_t)k].variant, 2, fm[(size_t)k]});
      if (tune_pick(fm) == 0) best_v |= kVT;
    }
  }
  // The lean stencil walk (kVL) at its grid against the winner so far, the
  // walk preferred (its generic slices run the template value-code form, its
  // base variant). (A software-pipelined form, two slices' gathers in flight
  // per wave, measured slower in the loop: 747 against 631 us at 512^3,
  // profiles/r04_lean_pipe512.log; not built.)
  std::vector<VlClass> vtab;
  int lean_G = 0;
  bool lean_team = false;
  // A 2-D plane-march winner runs the loop in mode 4 (fd_auto: two kernels
  // per body, the p update inside the march's SpMV), which the lean walk's
  // mode 3 does not beat (4096^2: 4,983 against 5,187-5,372 it/s,
  // profiles/r04a_configs.log against r03p): it is not offered there.
  const bool march2d = (best_v & 2097152) && A->dev.march_k > 0 && A->dev.march_a == 0;
  if (e == hipSuccess && A->dev.sl_t && !march2d && build_lean_classes(A, vtab) == CGX_OK &&
      !vtab.empty()) {
    const int G = lean_grid(A);
    if (build_lean_layout(A, vtab, G) != CGX_OK) e = hipErrorOutOfMemory;
    if (e == hipSuccess && split && lean_split_layout(A, G) != CGX_OK) e = hipErrorOutOfMemory;
    std::vector<CsrDev> lf(2, A->dev);
    lf[0].variant = kVlBase;
    lf[0].lean = true;
    lf[1].variant = best_v;
    lf[1].lean = false;
    std::vector<float> lm;
    if (e == hipSuccess) time_forms(lf, {1, 0}, lm);
    if (e == hipSuccess) {
      // both timings of this comparison go into the record: the walk and the
      // pick so far, re-timed in the same rounds (verdict r5: a record that
      // showed only the walk hid a re-timed incumbent that won)
      A->tune.push_back({kVL | kVlBase, split ? CGX_TUNE_LEAN_INTERIOR : CGX_TUNE_LEAN, lm[0]});
      A->tune.push_back({best_v, CGX_TUNE_INCUMBENT, lm[1]});
      std::vector<float> pick = lm;
      if (split) pick[0] += bnd_us;
      if (interior(best_v)) pick[1] += bnd_us;
      if (tune_pick(pick) == 0) lean_G = G;
      else best_us = pick[1];
    }
    // mode 4's fused walk in its team form (a whole-matrix walk whose grid
    // splits into 1,024-thread workgroups by XCD: G / 4 a multiple of 8),
    // by rule: where p alone exceeds the Infinity Cache (>= 32 M rows, where
    // fd_auto runs mode 4). In the loop 512^3 took 1,000 against 1,065 us
    // (548 against 520 it/s) and 256^3 113 against 127; the 256 x 256 x 32
    // slab (4 steps per wave) 18.5 against 15.8 (profiles/r05l_team_ab.log).
    // Timed alone on a warm cache the team form loses (256^3 111 against 97
    // us, 512^3 1,004 against 821): the isolated timing does not see what it
    // saves in the loop, so it is not timed here.
    if (e == hipSuccess && lean_G > 0 && !split && G % 32 == 0 && A->dtype == CGX_F64 &&
        A->dev.n >= (int64_t(32) << 20))
      lean_team = true;
  }
  (void)best_us;
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  for (void *p : {x, y, st, ap})
    if (p) (void)hipFree(p);
  if (e != hipSuccess) {
    free_lean(A);
    A->tune.clear();
    if (!err_set) set_error("cgx_csr_create: SpMV autotune: %s", hipGetErrorString(e));
    return CGX_EHIP;
  }
  if (lean_G > 0) {
    free_il(A);
    // (a split matrix keeps its boundary marks and vl_split)
    if (int rc = build_lean_layout(A, vtab, lean_G)) return rc;
    A->dev.variant = kVlBase;
    A->dev.lean = true;
    A->dev.vl_team = lean_team ? 1 : 0;
    return CGX_OK;
  }
  free_lean(A);
  A->dev.variant = best_v;
  if (!(best_v & (2048 | 8192))) free_sell(A);
  if (!(best_v & kC16) || (best_v & 8192)) free_col16(A);
  if (!(best_v & kIL)) free_il(A);
  return CGX_OK;
}

// x with ghost values for a distributed matrix: copy into A->d_ext + exchange
static int dist_extend(cgx_csr *A, const void *d_x, const void **x_ext) {
  *x_ext = d_x;
  if (!A->dist) return CGX_OK;
  const size_t es = dtype_size(A->dtype);
  if (!A->d_ext) CGX_HIP(hipMalloc(&A->d_ext, (size_t)(A->dev.n + A->halo.n_ghost + 1) * es));
  CGX_HIP(hipMemcpyAsync(A->d_ext, d_x, (size_t)A->dev.n * es, hipMemcpyDeviceToDevice,
                         A->ctx->stream));
  int rc = dist_halo_exchange(A, A->d_ext, A->ctx->stream);
  if (rc) return rc;
  *x_ext = A->d_ext;
  return CGX_OK;
}

// ===========================================================================
// VectorOperations
// ===========================================================================
extern "C" int cgx_spmv(cgx_ctx *ctx, cgx_csr *A, const void *x, void *y, int64_t count) {
  CGX_REQUIRE(ctx && A && x && y, CGX_EINVAL, "NULL argument");
  // VectorOperations.hpp:444: assert(vector_size != 0 && A.N() == vector_size)
  CGX_REQUIRE(count == A->dev.n, CGX_EINVAL, "spmv count %lld != A.N() %lld",
              (long long)count, (long long)A->dev.n);
  DeviceGuard g(ctx->device);
  const void *xe = x;
  int rc = dist_extend(A, x, &xe);
  if (rc) return rc;
  if (A->dtype == CGX_F32)
    CGX_HIP(Launch<float>::spmv(A->dev, (const float *)xe, (float *)y,
                                (CgScalars<float> *)((char *)ctx->spmv_st +
                                                     sizeof(CgScalars<double>)),
                                (RedWs<float> *)ctx->ws, ctx->stream));
  else
    CGX_HIP(Launch<double>::spmv(A->dev, (const double *)xe, (double *)y,
                                 (CgScalars<double> *)ctx->spmv_st, (RedWs<double> *)ctx->ws,
                                 ctx->stream));
  return CGX_OK;
}

extern "C" int cgx_dot_acc(cgx_ctx *ctx, int dtype, int64_t n, const void *x, const void *y,
                           void *res) {
  CGX_REQUIRE(ctx && x && y && res && n >= 0, CGX_EINVAL, "bad argument");
  DeviceGuard g(ctx->device);
  if (dtype == CGX_F32)
    CGX_HIP(Launch<float>::dot_acc(n, (const float *)x, (const float *)y, (float *)res,
                                   (RedWs<float> *)ctx->ws, ctx->stream));
  else
    CGX_HIP(Launch<double>::dot_acc(n, (const double *)x, (const double *)y, (double *)res,
                                    (RedWs<double> *)ctx->ws, ctx->stream));
  return CGX_OK;
}

extern "C" int cgx_norm_acc(cgx_ctx *ctx, int dtype, int64_t n, const void *x, void *res) {
  return cgx_dot_acc(ctx, dtype, n, x, x, res);
}

static int axpby_any(cgx_ctx *ctx, int mode, int dtype, int64_t n, const void *x,
                     const void *y, const void *a, const void *b, void *res) {
  CGX_REQUIRE(ctx && x && y && b && res && n >= 0, CGX_EINVAL, "bad argument");
  CGX_REQUIRE(mode != AX_SAXPBY || a, CGX_EINVAL, "saxpby needs a");
  if (n == 0) return CGX_OK;
  DeviceGuard g(ctx->device);
  if (dtype == CGX_F32)
    CGX_HIP(Launch<float>::axpby(mode, n, (const float *)x, (const float *)y,
                                 (const float *)a, (const float *)b, (float *)res,
                                 ctx->stream));
  else
    CGX_HIP(Launch<double>::axpby(mode, n, (const double *)x, (const double *)y,
                                  (const double *)a, (const double *)b, (double *)res,
                                  ctx->stream));
  return CGX_OK;
}

extern "C" int cgx_sapbx(cgx_ctx *ctx, int dtype, int64_t n, const void *x, const void *y,
                         const void *b, void *res) {
  return axpby_any(ctx, AX_SAPBX, dtype, n, x, y, nullptr, b, res);
}
extern "C" int cgx_sambx(cgx_ctx *ctx, int dtype, int64_t n, const void *x, const void *y,
                         const void *b, void *res) {
  return axpby_any(ctx, AX_SAMBX, dtype, n, x, y, nullptr, b, res);
}
extern "C" int cgx_saxpby(cgx_ctx *ctx, int dtype, int64_t n, const void *x, const void *y,
                          const void *a, const void *b, void *res) {
  return axpby_any(ctx, AX_SAXPBY, dtype, n, x, y, a, b, res);
}

extern "C" int cgx_scalar_div(cgx_ctx *ctx, int dtype, const void *num, const void *den,
                              void *out) {
  CGX_REQUIRE(ctx && num && den && out, CGX_EINVAL, "NULL argument");
  DeviceGuard g(ctx->device);
  if (dtype == CGX_F32)
    CGX_HIP(Launch<float>::scalar_div((const float *)num, (const float *)den, (float *)out,
                                      ctx->stream));
  else
    CGX_HIP(Launch<double>::scalar_div((const double *)num, (const double *)den,
                                       (double *)out, ctx->stream));
  return CGX_OK;
}

// ===========================================================================
// fused CG
// ===========================================================================
extern "C" int cgx_cg_create(cgx_ctx *ctx, cgx_csr *A, cgx_cg **out) {
  CGX_REQUIRE(ctx && A && out, CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(A->ctx == ctx, CGX_EINVAL, "matrix belongs to another context");
  DeviceGuard g(ctx->device);
  *out = nullptr;
  auto *cg = new cgx_cg();
  cg->ctx = ctx;
  cg->A = A;
  ctx_retain(ctx);
  csr_retain(A);
  cg->dtype = A->dtype;
  cg->n = A->dev.n;
  const size_t es = dtype_size(cg->dtype);
  const size_t next = (size_t)(cg->n + A->halo.n_ghost);
  const size_t stb = cg->dtype == CGX_F32 ? sizeof(CgScalars<float>) : sizeof(CgScalars<double>);
  const size_t wsb = cg->dtype == CGX_F32 ? sizeof(RedWs<float>) : sizeof(RedWs<double>);
  // r and Ap carry one slack element: k_update_r's first loads are clamped
  // 16-byte pairs, which for n = 1 would reach one element past the end
  hipError_t e = hipMalloc(&cg->r, ((size_t)cg->n + 1) * es);
  if (e == hipSuccess) e = hipMalloc(&cg->p, next * es);
  if (e == hipSuccess) e = hipMalloc(&cg->Ap, (next + 1) * es);
  if (e == hipSuccess && !A->dist) e = hipMalloc(&cg->p2, (size_t)cg->n * es);
  if (e == hipSuccess) e = hipMalloc(&cg->st, stb);
  if (e == hipSuccess) e = hipMalloc(&cg->ws, wsb);
  if (e == hipSuccess) e = hipMemsetAsync(cg->st, 0, stb, ctx->stream);
  if (e == hipSuccess) e = hipMemsetAsync(cg->ws, 0, wsb, ctx->stream);
  if (e == hipSuccess) e = hipMemsetAsync(cg->p, 0, next * es, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    cgx_cg_destroy(cg);
    if (e == hipErrorOutOfMemory) {
      set_error("cgx_cg_create: out of device memory (n=%lld)", (long long)cg->n);
      return CGX_ENOMEM;
    }
    return hip_fail(e, "cgx_cg_create");
  }
  cg->fused = false;
  // alternating sweep directions: +0.5-2% at 256^3
  cg->altdir = true;
  *out = cg;
  // auto mode: the x update deferred over four p buffers, in three kernels
  // (mode 3: +4-8% over mode 1 at 256^3) or, where it pays,
  // two (mode 4, fd_auto); plain three kernels when the three extra p buffers
  // do not fit
  if (cgx_cg_set_mode(cg, 0) != CGX_OK) cg->defer = cg->fdefer = cg->recompute = false;
  return CGX_OK;
}

// Auto mode picks 4 (fused deferred-x) where its kernel 1 adds no gathers
// or the iteration is launch-bound, 3 elsewhere (profiles/r02_fd_*.log):
//   * the 2-D plane march (gathers none: +-D from registers, +-1 from lanes):
//     4096^2 4,927 against 4,632 it/s;
//   * cache-resident stencil matrices (under 64 MB of CSR, the small-matrix
//     rule's stencil form): two launches per body instead of three, 128^2
//     96.7k against 80.0k it/s;
// and not where kernel 1 doubles real gathers: 256^3 3,700 against 4,210,
// 512^3 405 against 467, the G3 stand-in (CSR-stream) 19.96k against 22.5k.
static bool fd_auto(const cgx_cg *cg) {
  const cgx_csr *A = cg->A;
  // partitioned: the lean interior with this rank's vectors inside the
  // Infinity Cache (<= 4 M rows, lean_cached's bound below): on the 2-rank
  // rehearsal of 256^3 / 8's 256 x 256 x 32 slab 95.3-96.3 us per body
  // against 101.5-102.8 in mode 3 (profiles/r05u_dist_rehearsal.log). A
  // partitioned body uses the same push, wait and all-reduce tags in modes 3
  // and 4, so a rank whose autotune gave it another interior form can run
  // mode 3 beside them (bench.py still makes the ranks agree)
  if (A->dist) return dist_fd_ok(A, cg->dtype) && A->dev.n <= (int64_t(4) << 20);
  if (cg->dtype != CGX_F64 || !Launch<double>::fd_supported(A->dev)) return false;
  const int v = launch_variant(A->dev, cg->dtype);
  const bool march2d = (v & 2097152) && A->dev.march_a == 0;
  const bool small = A->dev.nnz * (int64_t)(sizeof(double) + sizeof(int)) < (int64_t(64) << 20);
  // the lean walk with cache-resident vectors (<= 32 MB, stream_nt's bound):
  // the 256 x 256 x 32 slab 29.5-29.8 us per body in mode 4 against
  // 31.9-32.1 in mode 3; at 256^3 mode 3 wins (5,182-5,208 against
  // 4,750-4,807 it/s; profiles/r04_dist_ab.log, r04b_slab.log)
  const bool lean_cached = vl_whole(A->dev) && A->dev.n <= (int64_t(4) << 20);
  // ... and with p alone past the Infinity Cache (>= 32 M rows: no p line the
  // p update writes survives to the SpMV, which mode 3's gain at 256^3 is):
  // 512^3 520 against 508 it/s, 548 with the fused walk's team form
  // (profiles/r05l_team_ab.log)
  const bool lean_big = vl_whole(A->dev) && A->dev.n >= (int64_t(32) << 20);
  return march2d || (small && (v & 1048576)) || lean_cached || lean_big;
}

// Auto mode picks 5 (the persistent body) for small single-device f64
// problems whose rows hold at most kCoopK entries: one workgroup of 1024
// threads per 1024 rows, at most kCoopMaxG of them (profiles/r03_coop_*.log:
// 128^2 5.97 against 9.61 us per body in mode 4, 256^2 6.9 against 10.0,
// 40^3 8.0 against 10.6; an irregular 100k-row matrix with longer rows
// ties, 14.8 against 14.9 in mode 3).
// Every workgroup of a mode-5 launch must be resident at once: one per CU at
// most (1,024 threads hold a CU's waves; the 256-thread forms are given the
// same bound), so the grid may not exceed the device's CUs (a partitioned
// device mode exposes fewer than kCoopMaxG)
static int device_cus(const cgx_cg *cg) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cg->ctx->device) !=
      hipSuccess)
    return 0;
  return cus;
}
static bool coop_fits(const cgx_cg *cg, int R) {
  if (R <= 0) return false;
  const int64_t per = (int64_t)1024 * R;
  return (cg->n + per - 1) / per <= device_cus(cg);
}
// The streamed form (2): rows of any length, R <= 8 rows per thread of
// 1,024-thread workgroups, one per CU at most
static int coop_stream_r(const cgx_cg *cg) {
  return coop_stream_rows(cg->n, coop_want_r(), device_cus(cg));
}
// auto: where neither register form applies (rows past 7 entries, or past
// kCoopMaxG workgroups), the matrix is on the CSR-stream path (it has no
// SELL copy: the stencils' SELL-P / value-code bodies win there) and the
// streamed form fits with at most kCoopStreamAutoR rows per thread — where
// it was measured to win (profiles/r03_coop_stream.log: irregular 100k /
// 200k / 400k rows 11.2 / 12.5 / 18.9 us per body against 14.3 / 16.6 /
// 19.6 in mode 3; at 4 and more rows per thread, and on the stencils, the
// three-kernel bodies are faster). $CGX_COOP_STREAM=0: never; 1: whenever
// it fits.
constexpr int kCoopStreamAutoR = 2;
static bool coop_stream_auto(const cgx_cg *cg) {
  const cgx_csr *A = cg->A;
  if (A->dist || cg->dtype != CGX_F64 || cg->coop_stream_want == 0) return false;
  const int R = coop_stream_r(cg);
  if (R <= 0) return false;
  if (cg->coop_stream_want == 1) return true;
  const bool csr_path = !A->dev.sl;  // no SELL copy: the SpMV is CSR-stream
  return csr_path && R <= kCoopStreamAutoR;
}
static bool coop_auto(const cgx_cg *cg) {
  const cgx_csr *A = cg->A;
  if (A->dist || cg->dtype != CGX_F64) return false;
  // rows whose entries all sit in registers (7 in the 1,024-thread form)
  return A->max_row_nnz <= 7 && coop_rows_per_thread(cg->n, kCoopMaxG) == 1 && coop_fits(cg, 1);
}

extern "C" int cgx_cg_set_mode(cgx_cg *cg, int mode) {
  CGX_REQUIRE(cg, CGX_EINVAL, "cg is NULL");
  CGX_REQUIRE(mode >= 0 && mode <= 7, CGX_EINVAL,
              "mode %d: 0 auto, 1 three kernels, 2 fused, 3 three kernels with deferred x, "
              "4 fused with deferred x, 5 persistent body, 6 recomputed Ap, 7 fused with "
              "recomputed Ap", mode);
  CGX_REQUIRE(mode != 6 || (!cg->A->dist && vl_whole(cg->A->dev)), CGX_EUNSUPPORTED,
              "mode 6 (recomputed Ap) needs the lean stencil walk on a single device");
  CGX_REQUIRE(mode != 7 || (!cg->A->dist && cg->dtype == CGX_F64 && lean_tile_ok(cg->A->dev)),
              CGX_EUNSUPPORTED,
              "mode 7 (fused, recomputed Ap) needs f64 and the tile form of the lean stencil walk "
              "(a 3-D stencil layout, one plane per step) on a single device");
  int coop_r = 0;
  if (!cg->begun) {  // mode 5's form and test hook
    cg->coop_stall = -1;
    if (const char *e = std::getenv("CGX_COOP_INJECT_STALL")) cg->coop_stall = std::atoi(e);
    cg->coop_stream_want = -1;
    if (const char *e = std::getenv("CGX_COOP_STREAM")) cg->coop_stream_want = std::atoi(e);
  }
  bool stream = false;
  if (mode == 5) {
    CGX_REQUIRE(!cg->A->dist && cg->dtype == CGX_F64, CGX_EUNSUPPORTED,
                "mode 5 (persistent body) runs f64 on a single device");
    // rows past the register entries (7 in the 1,024-thread form) read their
    // tails per thread from the CSR arrays in the register forms: the
    // streamed form is faster there (irregular 100k rows: 11.2 against 15.0
    // us per body, profiles/r03_coop_stream*.log) and is taken when it fits
    const bool prefer_stream =
        cg->coop_stream_want == 1 ||
        (cg->coop_stream_want != 0 && cg->A->max_row_nnz > 7 && coop_stream_r(cg) > 0);
    if (!prefer_stream) {
      coop_r = coop_rows_per_thread(cg->n, kCoopMaxG);
      if (coop_r > 0 && !coop_fits(cg, coop_r)) coop_r = 0;
    }
    if (coop_r == 0 && cg->coop_stream_want != 0) {
      coop_r = coop_stream_r(cg);
      stream = coop_r > 0;
    }
    CGX_REQUIRE(coop_r > 0, CGX_EUNSUPPORTED,
                "mode 5 (persistent body) takes at most %lld rows (%d workgroups of 1024 "
                "threads, %d rows per thread; n = %lld)",
                (long long)std::min(device_cus(cg), kCoopMaxG) * 1024 * kCoopStreamMaxR,
                std::min(device_cus(cg), kCoopMaxG), kCoopStreamMaxR, (long long)cg->n);
  }
  CGX_REQUIRE(!(mode == 2 && cg->A->dist), CGX_EUNSUPPORTED,
              "the fused iteration (mode 2) runs on a single device");
  CGX_REQUIRE(!(mode == 4 && cg->A->dist) || dist_fd_ok(cg->A, cg->dtype), CGX_EUNSUPPORTED,
              "mode 4 on a partitioned matrix needs f64, the device peer transport and the lean "
              "interior walk with boundary row blocks (partitioned matrices otherwise use mode 1 "
              "or 3)");
  CGX_REQUIRE(mode != 2 || (cg->dtype == CGX_F32 ? Launch<float>::fused_supported(cg->A->dev)
                                                 : Launch<double>::fused_supported(cg->A->dev)),
              CGX_EUNSUPPORTED, "mode 2 needs a production SpMV format (variant %d has no fused "
              "kernel)", launch_variant(cg->A->dev, cg->dtype));
  CGX_REQUIRE(mode != 4 || cg->A->dist ||
                  (cg->dtype == CGX_F64 && Launch<double>::fd_supported(cg->A->dev)),
              CGX_EUNSUPPORTED, "mode 4 needs an f64 matrix in a production SpMV format "
              "(variant %d has no fused kernel)", launch_variant(cg->A->dev, cg->dtype));
  if (mode == 0) {
    mode = coop_auto(cg) ? 5 : fd_auto(cg) ? 4 : 3;
    if (mode == 5) coop_r = coop_rows_per_thread(cg->n, kCoopMaxG);
    if (mode != 5 || coop_r == 0) {
      mode = coop_stream_auto(cg) ? 5 : fd_auto(cg) ? 4 : 3;
      if (mode == 5) {
        coop_r = coop_stream_r(cg);
        stream = true;
      }
    }
    // the whole-matrix lean walk between fd_auto's two bounds (256^3):
    // mode 6, Ap recomputed by a second walk instead of stored — 5,207-5,214
    // against 4,920-4,944 it/s in mode 3 (profiles/r6h_mode6_ab.log)
    if (mode == 3 && !cg->A->dist && vl_whole(cg->A->dev)) mode = 6;
  }
  const bool f = mode == 2, d = mode == 3 || mode == 6, fd = mode == 4 || mode == 7, c = mode == 5;
  const bool rc6 = mode == 6 || mode == 7;
  if (f != cg->fused || d != cg->defer || fd != cg->fdefer || c != cg->coop ||
      rc6 != cg->recompute) {
    CGX_REQUIRE(!cg->begun, CGX_ESTATE, "set the mode before cgx_cg_begin");
    drop_graph(cg);
  }
  if (c && !cg->coop_ws) {
    DeviceGuard g(cg->ctx->device);
    CGX_HIP(hipMalloc(&cg->coop_ws, sizeof(CoopWs)));
    if (const char *e = std::getenv("CGX_COOP_TRACE"); e && std::atoi(e)) {
      CGX_HIP(hipMalloc(&cg->coop_trace, kCoopTraceWords * sizeof(unsigned long long)));
      CGX_HIP(hipMemset(cg->coop_trace, 0, kCoopTraceWords * sizeof(unsigned long long)));
    }
    int clk_khz = 0;
    if (hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, cg->ctx->device) !=
            hipSuccess ||
        clk_khz <= 0)
      clk_khz = 100000;  // 100 MHz on gfx9
    cg->coop_ticks = (long long)clk_khz * 1000 * 2;  // 2 s: a resident grid never waits so long
    if (const char *e = std::getenv("CGX_COOP_TIMEOUT_MS"))
      cg->coop_ticks = (long long)clk_khz * std::max(1, std::atoi(e));
  }
  cg->coop = c;
  if (c) {
    cg->coop_r = coop_r;
    cg->coop_stream = stream;
  }
  if ((d || fd) && !cg->pk[0]) {  // three more p buffers (with the ghost tail when partitioned)
    DeviceGuard g(cg->ctx->device);
    const size_t bytes = (size_t)(cg->n + cg->A->halo.n_ghost) * dtype_size(cg->dtype);
    for (int k = 0; k < 3; ++k) {
      hipError_t e = hipMalloc(&cg->pk[k], bytes);
      if (e == hipSuccess) e = hipMemsetAsync(cg->pk[k], 0, bytes, cg->ctx->stream);
      if (e != hipSuccess) {
        for (int j = 0; j <= k; ++j) {
          if (cg->pk[j]) (void)hipFree(cg->pk[j]);
          cg->pk[j] = nullptr;
        }
        return hip_fail(e, "cgx_cg_set_mode(3)");
      }
    }
    CGX_HIP(hipStreamSynchronize(cg->ctx->stream));
  }
  cg->fused = f;
  cg->defer = d;
  cg->fdefer = fd;
  cg->recompute = rc6;
  return CGX_OK;
}

// mode 4's kernel 1 grid against the SpMV's (equal: mode 4 == mode 1 bit
// for bit; else the p.Ap partials split differently)
extern "C" int cgx_csr_fd_grid(cgx_csr *A, int *fd_grid, int *spmv_grid) {
  CGX_REQUIRE(A && fd_grid && spmv_grid, CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(A->dtype == CGX_F64 && Launch<double>::fd_supported(A->dev), CGX_EUNSUPPORTED,
              "no mode-4 kernel for this matrix");
  DeviceGuard g(A->ctx->device);
  *fd_grid = Launch<double>::fd_parts(A->dev);
  *spmv_grid = Launch<double>::spmv_parts(A->dev);
  return CGX_OK;
}

extern "C" int cgx_cg_get_mode(cgx_cg *cg, int *mode) {
  CGX_REQUIRE(cg && mode, CGX_EINVAL, "NULL argument");
  *mode = cg->coop       ? 5
          : cg->fdefer   ? (cg->recompute ? 7 : 4)
          : cg->recompute ? 6
          : cg->defer     ? 3
          : cg->fused     ? 2
                          : 1;
  return CGX_OK;
}

extern "C" int cgx_cg_destroy(cgx_cg *cg) {
  if (!cg) return CGX_OK;
  DeviceGuard g(cg->ctx->device);
  (void)hipStreamSynchronize(cg->ctx->stream);
  drop_graph(cg);
  for (auto e : cg->ev_pool) (void)hipEventDestroy(e);
  for (hipEvent_t e : cg->run_ev)
    if (e) (void)hipEventDestroy(e);
  for (void *p : {cg->r, cg->p, cg->p2, cg->Ap, cg->st, cg->ws, cg->pk[0], cg->pk[1], cg->pk[2],
                  cg->coop_ws, cg->coop_trace})
    if (p) (void)hipFree(p);
  cgx_csr *A = cg->A;
  cgx_ctx *ctx = cg->ctx;
  delete cg;
  csr_release(A);
  ctx_release(ctx);
  return CGX_OK;
}

extern "C" int cgx_cg_config(cgx_cg *cg, int poll_every, int use_graph) {
  CGX_REQUIRE(cg, CGX_EINVAL, "cg is NULL");
  if (poll_every > 0) {
    if (poll_every != cg->poll_every) drop_graph(cg);
    cg->poll_every = poll_every;
  }
  if (use_graph >= 0) cg->use_graph = use_graph != 0;
  return CGX_OK;
}

extern "C" int cgx_cg_begin(cgx_cg *cg, const void *b, void *x, double tol,
                            int64_t max_bodies) {
  CGX_REQUIRE(cg, CGX_EINVAL, "cg is NULL");
  // CG.hpp:266-272
  CGX_REQUIRE(b, CGX_ESTATE, "No right hand side to solve for");
  CGX_REQUIRE(x, CGX_EINVAL, "x is NULL");
  DeviceGuard g(cg->ctx->device);
  cgx_csr *A = cg->A;
  hipStream_t s = cg->ctx->stream;
  const int64_t n_ref = (A->dist ? A->n_global : A->dev.n);
  long long cap = (long long)n_ref + 1;  // counter++ < N  (CG.hpp:436)
  if (max_bodies >= 0) cap = std::min<long long>(cap, std::max<long long>(max_bodies, 1));
  cg->b = b;
  cg->x = x;
  if (cg->fused)  // p_{-1} = 0 for body 0 of the fused iteration
    CGX_HIP(hipMemsetAsync(cg->p2, 0, (size_t)cg->n * dtype_size(cg->dtype), s));
  if (cg->fdefer)  // mode 4: body 0 reads p_{-1} = P[3] (times beta = 0)
    CGX_HIP(hipMemsetAsync(cg->pk[2], 0, (size_t)cg->n * dtype_size(cg->dtype), s));
  const void *xe = x;
  int rc;
  if (A->dist && A->peer.on) {
    // PeerState::fault is sticky (every later peer kernel returns at entry):
    // a matrix whose transport timed out once fails every later solve until
    // cgx_dist_peer_enable rebuilds it, instead of skipping its all-reduces
    int fault = 0;
    CGX_HIP(hipMemcpyAsync(&fault, (const char *)A->peer.state + offsetof(PeerState, fault),
                           sizeof(int), hipMemcpyDeviceToHost, s));
    CGX_HIP(hipStreamSynchronize(s));
    CGX_REQUIRE(!fault, CGX_ENCCL,
                "peer transport: an earlier device-side wait on this matrix timed out; call "
                "cgx_dist_peer_enable again (collectively) before the next solve");
  }
  if (A->dist) {
    // initial guess with ghost values, staged in the Ap buffer (free at init)
    const size_t es = dtype_size(cg->dtype);
    CGX_HIP(hipMemcpyAsync(cg->Ap, x, (size_t)cg->n * es, hipMemcpyDeviceToDevice, s));
    if (A->peer.on) {
      rc = cg->dtype == CGX_F32
               ? peer_push<float>(A, (const float *)cg->Ap, nullptr, 0, s)
               : peer_push<double>(A, (const double *)cg->Ap, nullptr, 0, s);
      if (!rc)
        rc = cg->dtype == CGX_F32 ? peer_wait<float>(A, (float *)cg->Ap, nullptr, 0, s)
                                  : peer_wait<double>(A, (double *)cg->Ap, nullptr, 0, s);
    } else {
      rc = dist_halo_exchange(A, cg->Ap, s);
    }
    if (rc) return rc;
    xe = cg->Ap;
  }
  rc = timed(cg, 0, s, [&] {
    if (cg->dtype == CGX_F32)
      return Launch<float>::cg_init(A->dev, (const float *)xe, (const float *)b, (float *)cg->r,
                                    (float *)cg->p, (CgScalars<float> *)cg->st,
                                    (RedWs<float> *)cg->ws, (float)tol, cap, s);
    return Launch<double>::cg_init(A->dev, (const double *)xe, (const double *)b,
                                   (double *)cg->r, (double *)cg->p,
                                   (CgScalars<double> *)cg->st, (RedWs<double> *)cg->ws, tol,
                                   cap, s);
  });
  if (rc) return rc;
  if (A->dist && A->peer.on) {
    // the init kernel left the local r.r's double-length pair in rr_part[0..1]
    // (and its value in rxr[0]); all-reduce the pair into rxr[0]
    if (cg->dtype == CGX_F32) {
      auto *st = (CgScalars<float> *)cg->st;
      rc = peer_allreduce<float>(A, ((RedWs<float> *)cg->ws)->rr_part, 1, &st->rxr[0], nullptr,
                                 0, s, 0);
    } else {
      auto *st = (CgScalars<double> *)cg->st;
      rc = peer_allreduce<double>(A, ((RedWs<double> *)cg->ws)->rr_part, 1, &st->rxr[0],
                                  nullptr, 0, s, 0);
    }
    if (rc) return rc;
  } else if (A->dist) {
    const size_t off = cg->dtype == CGX_F32 ? offsetof(CgScalars<float>, rxr)
                                            : offsetof(CgScalars<double>, rxr);
    if ((rc = dist_allreduce_scalar(cg->ctx, (char *)cg->st + off, cg->dtype, 1, s))) return rc;
  }
  cg->slot = 0;
  cg->begun = true;
  return CGX_OK;
}

extern "C" int cgx_cg_run(cgx_cg *cg, int64_t bodies, int64_t *bodies_total, int *stopped) {
  CGX_REQUIRE(cg, CGX_EINVAL, "cg is NULL");
  CGX_REQUIRE(cg->begun, CGX_ESTATE, "cgx_cg_run before cgx_cg_begin");
  DeviceGuard g(cg->ctx->device);
  hipStream_t s = cg->ctx->stream;
  const bool use_graph = graph_ok(cg);
  if (cg->graph_x != cg->x) drop_graph(cg);
  // Two host staging buffers: chunk c's state is read while chunk c+1 runs.
  auto *hbuf = (char *)cg->ctx->h_pinned;
  for (int k = 0; k < 2; ++k)
    if (!cg->run_ev[k]) CGX_HIP(hipEventCreateWithFlags(&cg->run_ev[k], hipEventDisableTiming));
  hipEvent_t *ev = cg->run_ev;
  struct Pending { int buf; int slot_after; int64_t iters; };
  std::vector<Pending> q;
  int64_t remaining = bodies;
  int chunk_id = 0, rc = CGX_OK;
  bool done = false;
  long long last_bodies = -1;
  int last_stopped = 0;
  long long bodies_before = -1;
  bool flushed = false;
  auto wait_one = [&]() -> int {
    Pending pd = q.front();
    q.erase(q.begin());
    CGX_HIP(hipEventSynchronize(ev[pd.buf]));
    StateView v = view_state(cg, hbuf + 256 * pd.buf, pd.slot_after);
    if (cg->timing) {
      const long long before = bodies_before < 0 ? 0 : bodies_before;
      (void)before;
    }
    last_bodies = v.bodies;
    last_stopped = v.stopped;
    if (!v.active) done = true;
    return CGX_OK;
  };
  // bodies executed before this call (for the timing harvest)
  if (cg->timing) {
    CGX_HIP(hipStreamSynchronize(s));
    if ((rc = poll_state(cg, hbuf, s))) return rc;
    CGX_HIP(hipStreamSynchronize(s));
    bodies_before = view_state(cg, hbuf, cg->slot).bodies;
    // an init kernel may still be pending in the event list
  }
  while (!done && (remaining > 0 || !q.empty())) {
    if (remaining > 0 && q.size() < 2) {
      // mode 5: one launch per chunk of coop_chunk bodies (it leaves at the stop)
      const int64_t chunk = std::min<int64_t>(remaining, cg->coop ? coop_chunk(cg) : cg->poll_every);
      hipGraphExec_t ge = nullptr;
      if (use_graph && (rc = chunk_graph(cg, cg->slot, chunk, chunk == cg->poll_every, &ge))) break;
      if (cg->coop) {
        if ((rc = enqueue_coop(cg, cg->slot, chunk))) break;
      } else if (ge) {
        CGX_HIP(hipGraphLaunch(ge, s));
      } else {
        for (int64_t i = 0; i < chunk && rc == CGX_OK; ++i) rc = enqueue_iter_any(cg, (cg->slot + (int)i) & 3);
        if (rc) break;
      }
      cg->slot = (int)((cg->slot + chunk) & 3);
      remaining -= chunk;
      const int buf = chunk_id++ & 1;
      if ((rc = poll_state(cg, hbuf + 256 * buf, s))) break;
      CGX_HIP(hipEventRecord(ev[buf], s));
      q.push_back(Pending{buf, cg->slot, chunk});
      if (remaining == 0 && !cg->A->dist && !cg->coop && !(cg->defer && cg->slot == 0)) {
        // the end-of-run x flush reads only device state and the slot, so a
        // single-device run queues it behind its last chunk instead of after
        // the host has seen that chunk finish (one host round trip less).
        // (Modes 3 / 6 ending at slot 0: the slot-3 body applied the group, so
        // the flush is needed only if the run stopped inside the group; the
        // host decides once it has read the state below)
        if ((rc = flush_pending_x(cg))) break;
        flushed = true;
      }
      continue;
    }
    if ((rc = wait_one())) break;
  }
  // drain whatever is still queued
  while (rc == CGX_OK && !q.empty()) rc = wait_one();
  if (rc) return rc;
  if (last_stopped == 3) {
    set_error("peer transport: a device-side wait timed out (a rank stopped responding, or "
              "$CGX_PEER_TIMEOUT_S is too short); the solve was stopped");
    return CGX_ENCCL;
  }
  if (last_stopped == 4) {
    set_error("mode 5: a grid-wide exchange of the persistent body timed out (a workgroup of "
              "the launch was not resident); the solve was stopped, x is not updated");
    return CGX_EHIP;
  }
  // (modes 3 / 6 at slot 0 with every body active: the group is applied)
  const bool applied = cg->defer && cg->slot == 0 && last_stopped == 0 && !cg->A->dist;
  if (!flushed && !applied && (rc = flush_pending_x(cg))) return rc;
  CGX_HIP(hipStreamSynchronize(s));
  if (cg->timing) {
    CGX_HIP(hipStreamSynchronize(s));
    const int64_t active_iters = last_bodies - (bodies_before < 0 ? 0 : bodies_before);
    if ((rc = harvest_events(cg, active_iters))) return rc;
  }
  if (bodies_total) *bodies_total = last_bodies;
  if (stopped) *stopped = last_stopped;
  return CGX_OK;
}

extern "C" int cgx_cg_prepare(cgx_cg *cg, int64_t bodies) {
  CGX_REQUIRE(cg, CGX_EINVAL, "cg is NULL");
  CGX_REQUIRE(cg->begun, CGX_ESTATE, "cgx_cg_prepare before cgx_cg_begin");
  if (!graph_ok(cg) || bodies < 1) return CGX_OK;
  DeviceGuard g(cg->ctx->device);
  if (cg->graph_x != cg->x) drop_graph(cg);
  // the chunk sequence cgx_cg_run(bodies) walks from the current slot
  int slot = cg->slot;
  for (int64_t remaining = bodies; remaining > 0;) {
    const int64_t chunk = std::min<int64_t>(remaining, cg->poll_every);
    hipGraphExec_t ge = nullptr;
    if (int rc = chunk_graph(cg, slot, chunk, true, &ge)) return rc;
    slot = (int)((slot + chunk) & 3);
    remaining -= chunk;
  }
  return CGX_OK;
}

extern "C" int cgx_cg_coop_shape(cgx_cg *cg, int *rows_per_thread, int *threads,
                                 int *workgroups, int *form) {
  CGX_REQUIRE(cg && rows_per_thread && threads && workgroups && form, CGX_EINVAL,
              "NULL argument");
  CGX_REQUIRE(cg->coop, CGX_ESTATE, "the solver is not in mode 5");
  *rows_per_thread = cg->coop_r;
  *threads = 1024;
  const int64_t per = (int64_t)*threads * cg->coop_r;
  *workgroups = (int)((cg->n + per - 1) / per);
  *form = cg->coop_stream ? 2 : 0;
  return CGX_OK;
}

extern "C" int cgx_cg_coop_trace(cgx_cg *cg, uint64_t *host, int64_t words) {
  CGX_REQUIRE(cg && host, CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(cg->coop_trace, CGX_ESTATE, "no trace: set CGX_COOP_TRACE=1 before mode 5");
  DeviceGuard g(cg->ctx->device);
  CGX_HIP(hipStreamSynchronize(cg->ctx->stream));
  const int64_t w = std::min<int64_t>(words, kCoopTraceWords);
  CGX_HIP(hipMemcpy(host, cg->coop_trace, (size_t)w * 8, hipMemcpyDeviceToHost));
  return CGX_OK;
}

extern "C" int cgx_cg_rxr(cgx_cg *cg, double *rxr) {
  CGX_REQUIRE(cg && rxr, CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(cg->begun, CGX_ESTATE, "cgx_cg_rxr before cgx_cg_begin");
  DeviceGuard g(cg->ctx->device);
  auto *h = (char *)cg->ctx->h_pinned;
  int rc;
  if ((rc = poll_state(cg, h, cg->ctx->stream))) return rc;
  CGX_HIP(hipStreamSynchronize(cg->ctx->stream));
  // the rxr after the last body sits in the slot of the first skipped body
  const long long bodies = view_state(cg, h, 0).bodies;
  *rxr = view_state(cg, h, (int)(bodies & 3)).rxr;
  return CGX_OK;
}

extern "C" int cgx_cg_solve(cgx_cg *cg, const void *b, void *x, double tol, int64_t max_bodies,
                            int64_t *bodies_out, double *rxr_out) {
  int rc = cgx_cg_begin(cg, b, x, tol, max_bodies);
  if (rc) return rc;
  const int64_t n_ref = cg->A->dist ? cg->A->n_global : cg->n;
  int64_t cap = n_ref + 1;
  if (max_bodies >= 0) cap = std::min<int64_t>(cap, std::max<int64_t>(max_bodies, 1));
  int64_t total = 0;
  int stopped = 0;
  if ((rc = cgx_cg_run(cg, cap, &total, &stopped))) return rc;
  DeviceGuard g(cg->ctx->device);
  if (rxr_out) {
    // the rxr after the last body sits in the slot of the first skipped body
    auto *h = (char *)cg->ctx->h_pinned;
    if ((rc = poll_state(cg, h, cg->ctx->stream))) return rc;
    CGX_HIP(hipStreamSynchronize(cg->ctx->stream));
    *rxr_out = view_state(cg, h, (int)(total & 3)).rxr;
  }
  if (bodies_out) *bodies_out = total;
  return CGX_OK;
}

extern "C" int cgx_cg_set_kernel_timing(cgx_cg *cg, int enable) {
  CGX_REQUIRE(cg, CGX_EINVAL, "cg is NULL");
  cg->timing = enable != 0;
  for (int i = 0; i < 4; ++i) {
    cg->t_ms[i] = 0;
    cg->t_calls[i] = 0;
    cg->t_exec_ms[i] = 0;
    cg->t_exec_calls[i] = 0;
  }
  cg->ev_pending.clear();
  cg->ev_used = 0;
  return CGX_OK;
}

extern "C" int cgx_cg_kernel_exec_times(cgx_cg *cg, double *avg_ms, int64_t *calls) {
  CGX_REQUIRE(cg, CGX_EINVAL, "cg is NULL");
  DeviceGuard g(cg->ctx->device);
  if (!cg->ev_pending.empty()) {
    CGX_HIP(hipStreamSynchronize(cg->ctx->stream));
    int rc = harvest_events(cg, 0);
    if (rc) return rc;
  }
  for (int i = 0; i < 4; ++i) {
    if (avg_ms)
      avg_ms[i] = cg->t_exec_calls[i] ? cg->t_exec_ms[i] / (double)cg->t_exec_calls[i] : 0.0;
    if (calls) calls[i] = cg->t_exec_calls[i];
  }
  return CGX_OK;
}

extern "C" int cgx_cg_kernel_times(cgx_cg *cg, double *avg_ms, int64_t *calls) {
  CGX_REQUIRE(cg, CGX_EINVAL, "cg is NULL");
  DeviceGuard g(cg->ctx->device);
  if (!cg->ev_pending.empty()) {  // an init kernel timed outside cgx_cg_run
    CGX_HIP(hipStreamSynchronize(cg->ctx->stream));
    int rc = harvest_events(cg, 0);
    if (rc) return rc;
  }
  for (int i = 0; i < 4; ++i) {
    if (avg_ms) avg_ms[i] = cg->t_calls[i] ? cg->t_ms[i] / (double)cg->t_calls[i] : 0.0;
    if (calls) calls[i] = cg->t_calls[i];
  }
  return CGX_OK;
}

// ===========================================================================
// accuracy (CG.hpp:463-515)
// ===========================================================================
extern "C" int cgx_accuracy(cgx_ctx *ctx, cgx_csr *A, const void *b, const void *x,
                            double *out) {
  CGX_REQUIRE(ctx && A && b && x && out, CGX_EINVAL, "NULL argument");
  DeviceGuard g(ctx->device);
  const void *xe = x;
  int rc = dist_extend(A, x, &xe);
  if (rc) return rc;
  double h[2];
  if (A->dtype == CGX_F32) {
    CGX_HIP(Launch<float>::accuracy(A->dev, (const float *)b, (const float *)xe,
                                    (float *)ctx->scratch, (RedWs<float> *)ctx->ws,
                                    ctx->stream));
    if (A->dist && (rc = dist_allreduce_scalar(ctx, ctx->scratch, CGX_F32, 2, ctx->stream)))
      return rc;
    float hf[2];
    CGX_HIP(hipMemcpyAsync(hf, ctx->scratch, sizeof(hf), hipMemcpyDeviceToHost, ctx->stream));
    CGX_HIP(hipStreamSynchronize(ctx->stream));
    h[0] = hf[0];
    h[1] = hf[1];
    *out = (double)std::fabs(hf[0] / hf[1]);
    return CGX_OK;
  }
  CGX_HIP(Launch<double>::accuracy(A->dev, (const double *)b, (const double *)xe,
                                   (double *)ctx->scratch, (RedWs<double> *)ctx->ws,
                                   ctx->stream));
  if (A->dist && (rc = dist_allreduce_scalar(ctx, ctx->scratch, CGX_F64, 2, ctx->stream)))
    return rc;
  CGX_HIP(hipMemcpyAsync(h, ctx->scratch, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  CGX_HIP(hipStreamSynchronize(ctx->stream));
  *out = std::fabs(h[0] / h[1]);
  return CGX_OK;
}

// ===========================================================================
// synthetic inputs
// ===========================================================================
extern "C" int64_t cgx_poisson_nnz(int dim, int nx, int ny, int nz, int64_t row_begin,
                                   int64_t row_end) {
  if (dim != 2 && dim != 3) return -1;
  return poisson_row_offset(dim, nx, ny, dim == 3 ? nz : 1, row_end) -
         poisson_row_offset(dim, nx, ny, dim == 3 ? nz : 1, row_begin);
}

extern "C" int cgx_poisson_fill(cgx_ctx *ctx, int dtype, int dim, int nx, int ny, int nz,
                                int64_t row_begin, int64_t row_end, int *d_rowptr, int *d_col,
                                void *d_val) {
  CGX_REQUIRE(ctx && d_rowptr && d_col && d_val, CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(dim == 2 || dim == 3, CGX_EINVAL, "dim must be 2 or 3");
  CGX_REQUIRE(nx > 0 && ny > 0 && (dim == 2 || nz > 0), CGX_EINVAL, "bad grid");
  const int zz = dim == 3 ? nz : 1;
  const int64_t n = (int64_t)nx * ny * zz;
  CGX_REQUIRE(row_begin >= 0 && row_begin <= row_end && row_end <= n, CGX_EINVAL,
              "bad row range");
  DeviceGuard g(ctx->device);
  if (dtype == CGX_F32)
    CGX_HIP(Launch<float>::poisson(dim, nx, ny, zz, row_begin, row_end, d_rowptr, d_col,
                                   (float *)d_val, ctx->stream));
  else
    CGX_HIP(Launch<double>::poisson(dim, nx, ny, zz, row_begin, row_end, d_rowptr, d_col,
                                    (double *)d_val, ctx->stream));
  return CGX_OK;
}

extern "C" int cgx_iota(cgx_ctx *ctx, int dtype, void *d_b, int64_t n, double offset) {
  CGX_REQUIRE(ctx && d_b && n >= 0, CGX_EINVAL, "bad argument");
  if (n == 0) return CGX_OK;
  DeviceGuard g(ctx->device);
  if (dtype == CGX_F32) CGX_HIP(Launch<float>::iota((float *)d_b, n, offset, ctx->stream));
  else CGX_HIP(Launch<double>::iota((double *)d_b, n, offset, ctx->stream));
  return CGX_OK;
}

// ===========================================================================
// diagnostics: time one SpMV(+p.Ap) variant (bits: cgx_kernels.hip spmv_rows)
// ===========================================================================
extern "C" int cgx_tune_spmv(cgx_ctx *ctx, cgx_csr *A, int variant, const void *x, void *y,
                             int iters, double *avg_ms) {
  CGX_REQUIRE(ctx && A && x && y && avg_ms && iters > 0, CGX_EINVAL, "bad argument");
  CGX_REQUIRE(!A->dist, CGX_EUNSUPPORTED, "tuning runs on a single-device matrix");
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  void *st = nullptr;
  CGX_HIP(hipMalloc(&st, sizeof(CgScalars<double>)));
  CGX_HIP(hipMemsetAsync(st, 0, sizeof(CgScalars<double>), s));
  const int one = 1;
  const size_t off = A->dtype == CGX_F32 ? offsetof(CgScalars<float>, active)
                                         : offsetof(CgScalars<double>, active);
  CGX_HIP(hipMemcpyAsync((char *)st + off, &one, sizeof(int), hipMemcpyHostToDevice, s));
  hipEvent_t e0, e1;
  CGX_HIP(hipEventCreate(&e0));
  CGX_HIP(hipEventCreate(&e1));
  hipError_t e = hipSuccess;
  CsrDev dv = A->dev;  // the requested form as the matrix's (kVT: template slice table)
  dv.variant = variant;
  for (int i = 0; i <= iters && e == hipSuccess; ++i) {  // first launch = warm-up
    if (i == 1) e = hipEventRecord(e0, s);
    if (e != hipSuccess) break;
    if (A->dtype == CGX_F32)
      e = Launch<float>::spmv_dot_variant(variant, dv, (const float *)x, (float *)y,
                                          (CgScalars<float> *)st, (RedWs<float> *)ctx->ws, s);
    else
      e = Launch<double>::spmv_dot_variant(variant, dv, (const double *)x, (double *)y,
                                           (CgScalars<double> *)st, (RedWs<double> *)ctx->ws, s);
  }
  if (e == hipSuccess) e = hipEventRecord(e1, s);
  if (e == hipSuccess) e = hipEventSynchronize(e1);
  float ms = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(st);
  CGX_HIP(e);
  *avg_ms = ms / iters;
  return CGX_OK;
}
