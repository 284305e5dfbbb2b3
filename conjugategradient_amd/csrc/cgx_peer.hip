// cgx_peer.hip — device peer transport of the row-partitioned CG over xGMI
// (DESIGN.md §9).
//
// The reference is single-device (src/CG.hpp:61,70-77); the partitioned
// iteration needs, per body, one halo exchange of p and two scalar
// all-reduces (p.Ap, r.r). RCCL does them as host-enqueued collectives, which
// keeps the iteration out of a hipGraph and costs ~10-20 us each on 8 GPUs.
// Here they are three small kernels that read and write the other ranks'
// memory directly (one process per GPU; buffers exported with hipIpc and
// mapped into every peer):
//
//   k_peer_push       gathers the p entries each neighbour needs and stores
//                     them into that neighbour's landing buffer, then raises
//                     one flag per workgroup there (system-scope release);
//   k_peer_wait       polls this rank's flags, then copies the landing buffer
//                     into p's ghost area (the boundary SpMV reads it next);
//   k_peer_allreduce  one workgroup: sums the local partials, stores the value
//                     and a tag into every rank's mailbox, polls its own
//                     mailbox until every rank's tag arrived, and sums the
//                     world values IN RANK ORDER — bit-identical on all ranks,
//                     so alpha, beta and the stop rule agree everywhere.
//
// Landing buffers, mailboxes and flags are uncached device memory
// (hipDeviceMallocUncached): remote stores and local loads meet in HBM with
// no stale L2 line on either side. Tags are the count of all-reduces done
// (PeerState::ar, identical on every rank because every rank runs the same
// sequence); two parity slots per mailbox suffice because a rank can only
// start all-reduce m+2 after every rank contributed to m+1, i.e. finished
// reading m. A landing buffer is rewritten only by the next body's push,
// which starts after the r.r all-reduce of this body, i.e. after every rank
// finished this body's SpMV. Every spin is bounded (PeerDev::spin_ticks of
// the 100 MHz wall clock); a timeout sets PeerState::fault and the body's
// stopped = 3, and every later peer kernel returns at entry.
//
// cgx_dist_peer_enable builds the transport collectively over the setup
// transport (RCCL or the host one) and checks it against that transport:
// a halo exchange of a known vector must match bit for bit, and three
// all-reduces of known values must be exact. All ranks agree on the outcome;
// on any failure the partitioned solver keeps the setup transport.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cgx_objects.h"
#include "cgx_peer_dev.h"

namespace cgx {
namespace {

using peerdev::ld_sys;
using peerdev::ld_sysd;
using peerdev::st_sys;
using peerdev::st_sysd;
using peerdev::skip_body;

using peerdev::spin_ge;

using peerdev::raise_fault;

// k_peer_push: grid = nsend x kPushWG (peerdev::push_wg); the split SpMV
// of a SELL matrix carries the same workgroups at the front of its interior
// launch instead (k_spmv_dot_push)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_peer_push(const T *__restrict__ v, PeerDev P,
                                                       CgScalars<T> *st, int slot) {
  peerdev::push_wg<T>(v, P, st, slot, blockIdx.x);
}

// k_peer_wait: every workgroup's first wave polls the flags of every rank
// that sends here (all kPushWG of each) for this body's tag, then the
// workgroup copies its share of the landing buffer into v's ghost area.
// v == nullptr (peer_wait_one, one workgroup): the wait alone; the boundary
// launch behind it reads the landing buffer itself
template <typename T>
__global__ __launch_bounds__(kBlock) void k_peer_wait(T *__restrict__ v, PeerDev P,
                                                       CgScalars<T> *st, int slot) {
  __shared__ int ok_s;
  if (skip_body(st, slot, P.state)) return;
  if (!peerdev::wait_pushes(P, peerdev::body_tag(st, slot, P.state), &ok_s)) {
    if (threadIdx.x == 0) raise_fault(st, slot, P.state);
    return;
  }
  if (!v) return;
  const T *land = reinterpret_cast<const T *>(P.land_local);
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < P.n_ghost; k += stride)
    v[P.n_local + k] = land[k];
}

// k_peer_allreduce: one workgroup. *dst = sum over ranks in rank order of
// each rank's sum of its part[0..np) (fixed order within the rank). which:
// 0 a setup / init all-reduce (tag ar + 1; both body bases follow it), 1 / 2
// the body's first / second (tag arb[slot & 1] + which; the second sets the
// next body's base)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_peer_allreduce(const T *__restrict__ part, int np,
                                                            T *dst, CgScalars<T> *st, int slot,
                                                            PeerDev P, int which) {
  __shared__ double red[2 * (kBlock / 64)];
  __shared__ int ok_s;
  if (skip_body(st, slot, P.state)) return;
  // this rank's double-length sum of its np partial pairs in sum_parts_dd's
  // order (the fused form's value, bit for bit)
  Dd<double> v(0.0);
  for (int k = threadIdx.x; k < np; k += kBlock)
    v += Dd<double>((double)part[2 * k], (double)part[2 * k + 1]);
  v = wave_sum_dd(v);
  if ((threadIdx.x & 63) == 0) {
    red[2 * (threadIdx.x >> 6)] = v.hi;
    red[2 * (threadIdx.x >> 6) + 1] = v.lo;
  }
  __syncthreads();
  Dd<double> mine(red[0], red[1]);
  for (int w = 1; w < kBlock / 64; ++w) mine += Dd<double>(red[2 * w], red[2 * w + 1]);
  const unsigned long long tag = which ? P.state->arb[slot & 1] + which : P.state->ar + 1;
  const int par = (int)(tag & 1);
  if (threadIdx.x < 64) {
    bool ok = true;
    if ((int)threadIdx.x < P.world) {
      char *box = P.ctl[threadIdx.x];
      double *val = reinterpret_cast<double *>(box) + 2 * (par * kPeerMax + P.rank);
      st_sysd(val, mine.hi);
      st_sysd(val + 1, mine.lo);
      __threadfence_system();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st_sys(reinterpret_cast<unsigned long long *>(box + kPeerTagOff) + par * kPeerMax + P.rank,
             tag);
      const auto *tags = reinterpret_cast<const unsigned long long *>(P.ctl[P.rank] + kPeerTagOff);
      ok = spin_ge(tags + par * kPeerMax + threadIdx.x, tag, P.spin_ticks);
    }
    ok = __all(ok);
    if (threadIdx.x == 0) ok_s = ok;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  if (!ok_s) {
    raise_fault(st, slot, P.state);
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const double *vals = reinterpret_cast<const double *>(P.ctl[P.rank]) + 2 * par * kPeerMax;
  Dd<double> s(0.0);
  for (int q = 0; q < P.world; ++q) s += Dd<double>(ld_sysd(vals + 2 * q), ld_sysd(vals + 2 * q + 1));
  *dst = (T)s.value();
  P.state->ar = tag;
  if (which == 0) P.state->arb[0] = P.state->arb[1] = tag;
  if (which == 2) P.state->arb[(slot + 1) & 1] = tag;
}

constexpr int kWaitGridMax = 256;

int wait_grid(int64_t n_ghost) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(kWaitGridMax, (n_ghost + 2047) / 2048));
}

}  // namespace

// ---- enqueue helpers (cgx_objects.h) ---------------------------------------
template <typename T>
int peer_push(cgx_csr *A, const T *v_ext, CgScalars<T> *st, int slot, hipStream_t s) {
  const PeerDev &P = A->peer.dev;
  if (P.nsend == 0) return CGX_OK;
  hipLaunchKernelGGL(k_peer_push<T>, dim3(P.nsend * kPushWG), dim3(kBlock), 0, s, v_ext, P, st,
                     slot);
  CGX_HIP(hipGetLastError());
  return CGX_OK;
}

template <typename T> int peer_wait(cgx_csr *A, T *v_ext, CgScalars<T> *st, int slot, hipStream_t s) {
  PeerDev P = A->peer.dev;
  P.nopoll = 0;  // this launch is the one that polls
  if (P.nrecv == 0) return CGX_OK;
  // (the one-waiter form: one workgroup polls and copies)
  hipLaunchKernelGGL(k_peer_wait<T>, dim3(A->peer.one_waiter ? 1 : wait_grid(P.n_ghost)),
                     dim3(kBlock), 0, s, v_ext, P, st, slot);
  CGX_HIP(hipGetLastError());
  return CGX_OK;
}

template <typename T> int peer_wait_one(cgx_csr *A, CgScalars<T> *st, int slot, hipStream_t s) {
  PeerDev P = A->peer.dev;
  P.nopoll = 0;
  if (P.nrecv == 0) return CGX_OK;
  hipLaunchKernelGGL(k_peer_wait<T>, dim3(1), dim3(kBlock), 0, s, (T *)nullptr, P, st, slot);
  CGX_HIP(hipGetLastError());
  return CGX_OK;
}

template <typename T>
int peer_allreduce(cgx_csr *A, const T *part, int np, T *dst, CgScalars<T> *st, int slot,
                   hipStream_t s, int which) {
  hipLaunchKernelGGL(k_peer_allreduce<T>, dim3(1), dim3(kBlock), 0, s, part, np, dst, st, slot,
                     A->peer.dev, which);
  CGX_HIP(hipGetLastError());
  return CGX_OK;
}

template int peer_push<double>(cgx_csr *, const double *, CgScalars<double> *, int, hipStream_t);
template int peer_push<float>(cgx_csr *, const float *, CgScalars<float> *, int, hipStream_t);
template int peer_wait<double>(cgx_csr *, double *, CgScalars<double> *, int, hipStream_t);
template int peer_wait<float>(cgx_csr *, float *, CgScalars<float> *, int, hipStream_t);
template int peer_wait_one<double>(cgx_csr *, CgScalars<double> *, int, hipStream_t);
template int peer_wait_one<float>(cgx_csr *, CgScalars<float> *, int, hipStream_t);
template int peer_allreduce<double>(cgx_csr *, const double *, int, double *, CgScalars<double> *,
                                    int, hipStream_t, int);
template int peer_allreduce<float>(cgx_csr *, const float *, int, float *, CgScalars<float> *,
                                   int, hipStream_t, int);

int peer_destroy(cgx_csr *A) {
  Peer &pr = A->peer;
  for (void *m : pr.mapped)
    if (m) (void)hipIpcCloseMemHandle(m);
  pr.mapped.clear();
  for (void **p : {&pr.ctl, &pr.land, &pr.state})
    if (*p) {
      (void)hipFree(*p);
      *p = nullptr;
    }
  pr.on = false;
  pr.dev = PeerDev{};
  pr.colocated = 1;
  pr.one_waiter = false;
  return CGX_OK;
}

}  // namespace cgx

using namespace cgx;

namespace {

// what every rank publishes at setup
struct PeerCard {
  hipIpcMemHandle_t ctl, land;
  int64_t recv_off[kPeerMax];  // where rank q's values start in my landing buffer (-1: none)
  int64_t recv_cnt[kPeerMax];
  int ok;                      // this rank got this far
  int pad;
  char bus[32];                // PCI bus id of the rank's device (ranks sharing a GPU)
  int one_req;                 // $CGX_PEER_ONE_WAITER: -1 unset, 0 fused form, 1 one-waiter
  int pad2;
};

int all_ok(cgx_ctx *ctx, int mine, int *all) {
  std::vector<int> v((size_t)ctx->world, 0);
  int rc = comm_allgather(ctx, &mine, sizeof(int), v.data());
  if (rc) return rc;
  *all = 1;
  for (int x : v) *all = *all && x;
  return CGX_OK;
}

// the transport against the setup transport: halo of a known vector
// bit-identical, three all-reduces of known values exact
template <typename T> int self_test(cgx_csr *A, bool *ok) {
  *ok = false;
  cgx_ctx *ctx = A->ctx;
  hipStream_t s = ctx->stream;
  const int64_t n = A->dev.n, ng = A->halo.n_ghost, next = n + ng;
  std::vector<T> h((size_t)next, T(0));
  for (int64_t k = 0; k < n; ++k) h[k] = (T)(0.25 + (double)(A->row_begin + k));
  T *v1 = nullptr, *v2 = nullptr, *part = nullptr, *res = nullptr;
  int rc = CGX_OK;
  hipError_t e = hipMalloc(&v1, next * sizeof(T));
  if (e == hipSuccess) e = hipMalloc(&v2, next * sizeof(T));
  if (e == hipSuccess) e = hipMalloc(&part, 4 * sizeof(T));
  if (e == hipSuccess) e = hipMalloc(&res, 4 * sizeof(T));
  if (e == hipSuccess) e = hipMemcpyAsync(v1, h.data(), next * sizeof(T), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(v2, h.data(), next * sizeof(T), hipMemcpyHostToDevice, s);
  if (e != hipSuccess) rc = hip_fail(e, "peer self-test (alloc)");
  if (!rc) rc = dist_halo_exchange(A, v1, s);  // the setup transport's answer
  if (!rc) rc = peer_push<T>(A, v2, nullptr, 0, s);
  if (!rc) rc = peer_wait<T>(A, v2, nullptr, 0, s);
  T want[3] = {T(0), T(0), T(0)};
  for (int r = 0; r < 3 && !rc; ++r) {
    // two partial pairs (hi, lo): (rank + 1) (r + 1) and 0.5
    const T mine[4] = {(T)(ctx->rank + 1) * (T)(r + 1), T(0), (T)0.5, T(0)};
    for (int q = 0; q < ctx->world; ++q) want[r] += (T)(q + 1) * (T)(r + 1) + (T)0.5;
    e = hipMemcpyAsync(part, mine, 4 * sizeof(T), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) rc = hip_fail(e, "peer self-test (copy)");
    if (!rc) rc = peer_allreduce<T>(A, part, 2, res + r, nullptr, 0, s, 0);
    if (!rc) {
      e = hipStreamSynchronize(s);  // `part` is reused
      if (e != hipSuccess) rc = hip_fail(e, "peer self-test (all-reduce)");
    }
  }
  std::vector<T> g1((size_t)ng + 1), g2((size_t)ng + 1);
  T got[3];
  PeerState ps{};
  if (!rc && ng) {
    e = hipMemcpyAsync(g1.data(), v1 + n, ng * sizeof(T), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(g2.data(), v2 + n, ng * sizeof(T), hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) rc = hip_fail(e, "peer self-test (download)");
  }
  if (!rc) {
    e = hipMemcpyAsync(got, res, 3 * sizeof(T), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess)
      e = hipMemcpyAsync(&ps, A->peer.state, sizeof(ps), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) rc = hip_fail(e, "peer self-test (results)");
  }
  if (!rc) {
    bool good = ps.fault == 0 && std::memcmp(g1.data(), g2.data(), ng * sizeof(T)) == 0;
    for (int r = 0; r < 3; ++r) good = good && got[r] == want[r];
    if (!good)
      set_error("peer transport self-test failed on rank %d (fault %d, halo %s, sums %g/%g)",
                ctx->rank, ps.fault,
                std::memcmp(g1.data(), g2.data(), ng * sizeof(T)) ? "differs" : "ok",
                (double)got[0], (double)want[0]);
    *ok = good;
  }
  for (T *p : {v1, v2, part, res})
    if (p) (void)hipFree(p);
  return rc;
}

}  // namespace

// Collective over the matrix's communicator. Builds the device peer transport
// for A (partitioned) and checks it; *enabled = 1 when every rank passed,
// else the solver keeps the setup transport (*enabled = 0, not an error;
// cgx_last_error() says why). $CGX_PEER=0 skips it.
extern "C" int cgx_dist_peer_enable(cgx_csr *A, int *enabled) {
  CGX_REQUIRE(A && enabled, CGX_EINVAL, "NULL argument");
  *enabled = 0;
  CGX_REQUIRE(A->dist, CGX_EINVAL, "cgx_dist_peer_enable needs a partitioned matrix");
  cgx_ctx *ctx = A->ctx;
  CGX_HIP(hipSetDevice(ctx->device));
  if (A->peer.on) {
    // already on: keep it unless a spin timed out on any rank (the fault is
    // sticky, cgx_cg_begin refuses such a matrix); then every rank rebuilds
    // it together
    int fault = 0;
    CGX_HIP(hipMemcpy(&fault, (const char *)A->peer.state + offsetof(PeerState, fault),
                      sizeof(int), hipMemcpyDeviceToHost));
    int all_clean = 0;
    if (int rc0 = all_ok(ctx, fault ? 0 : 1, &all_clean)) return rc0;
    if (all_clean) {
      *enabled = 1;
      return CGX_OK;
    }
    CGX_HIP(hipStreamSynchronize(ctx->stream));
    peer_destroy(A);
  }
  const int world = ctx->world, me = ctx->rank;
  int mine_ok = 1;
  std::string why;
  if (const char *env = std::getenv("CGX_PEER"))
    if (std::atoi(env) == 0) {
      mine_ok = 0;
      why = "$CGX_PEER=0";
    }
  if (world < 2 || world > kPeerMax) {
    mine_ok = 0;
    why = "world size outside 2.." + std::to_string(kPeerMax);
  }
  // every rank decides together whether to try at all ($CGX_PEER may differ)
  int go = 0, rc = all_ok(ctx, mine_ok, &go);
  if (rc) return rc;
  if (!go) {
    set_error("peer transport not tried: %s", why.empty() ? "another rank declined" : why.c_str());
    return CGX_OK;
  }
  Peer &pr = A->peer;
  const Halo &h = A->halo;
  const size_t es = dtype_size(A->dtype);
  hipStream_t s = ctx->stream;
  PeerCard card{};
  std::memset(&card, 0, sizeof(card));
  for (int q = 0; q < kPeerMax; ++q) card.recv_off[q] = -1;
  for (size_t i = 0; i < h.nbr.size(); ++i) {
    card.recv_off[h.nbr[i]] = h.recv_off[i];
    card.recv_cnt[h.nbr[i]] = h.recv_cnt[i];
  }
  hipError_t e = hipExtMallocWithFlags(&pr.ctl, kPeerCtlBytes, hipDeviceMallocUncached);
  if (e == hipSuccess)
    e = hipExtMallocWithFlags(&pr.land, std::max<size_t>(1, (size_t)h.n_ghost) * es,
                              hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMalloc(&pr.state, sizeof(PeerState));
  if (e == hipSuccess) e = hipMemsetAsync(pr.ctl, 0, kPeerCtlBytes, s);
  if (e == hipSuccess) e = hipMemsetAsync(pr.land, 0, std::max<size_t>(1, (size_t)h.n_ghost) * es, s);
  PeerState st0{1, 0, 0, {1, 1}, {}};  // tags start at 1: a zeroed flag never matches
  if (e == hipSuccess) e = hipMemcpyAsync(pr.state, &st0, sizeof(st0), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess) e = hipIpcGetMemHandle(&card.ctl, pr.ctl);
  if (e == hipSuccess) e = hipIpcGetMemHandle(&card.land, pr.land);
  card.ok = e == hipSuccess;
  if (!card.ok) why = std::string("allocation / IPC export: ") + hipGetErrorString(e);
  if (hipDeviceGetPCIBusId(card.bus, (int)sizeof(card.bus) - 1, ctx->device) != hipSuccess)
    card.bus[0] = 0;
  card.one_req = -1;
  if (const char *env = std::getenv("CGX_PEER_ONE_WAITER")) card.one_req = std::atoi(env) ? 1 : 0;
  std::vector<PeerCard> cards((size_t)world);
  if ((rc = comm_allgather(ctx, &card, sizeof(card), cards.data()))) {
    peer_destroy(A);
    return rc;
  }
  bool ok = true;
  for (const PeerCard &c : cards) ok = ok && c.ok;
  // ranks sharing this rank's GPU, and the form every rank takes: the
  // one-waiter form when any two ranks share a device (or any rank asks for
  // it), the fused form otherwise (or when a rank asks for it and none for
  // the one-waiter form); every rank sees the same cards, so all agree
  int colocated = 0, one = -1;
  bool shared = false;
  for (int q = 0; q < world; ++q) {
    const PeerCard &c = cards[q];
    if (c.bus[0] && std::strncmp(c.bus, card.bus, sizeof(c.bus)) == 0) ++colocated;
    for (int u = 0; u < q; ++u)
      shared = shared || (c.bus[0] && std::strncmp(c.bus, cards[u].bus, sizeof(c.bus)) == 0);
    if (c.one_req == 1) one = 1;
    if (c.one_req == 0 && one < 0) one = 0;
  }
  pr.colocated = std::max(1, colocated);
  pr.one_waiter = one < 0 ? shared : one == 1;
  PeerDev &P = pr.dev;
  P = PeerDev{};
  P.rank = me;
  P.world = world;
  P.state = (PeerState *)pr.state;
  P.send_idx = h.d_send_idx;
  P.land_local = pr.land;
  P.n_local = A->dev.n;
  P.n_ghost = h.n_ghost;
  int clk_khz = 0;
  if (hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, ctx->device) != hipSuccess ||
      clk_khz <= 0)
    clk_khz = 100000;  // 100 MHz on gfx9
  double secs = 10.0;
  if (const char *env = std::getenv("CGX_PEER_TIMEOUT_S")) secs = std::max(0.01, std::atof(env));
  // the self-test gives up sooner: a transport that cannot deliver there
  // falls back instead of stalling the setup
  P.spin_ticks = (long long)(2.0 * clk_khz * 1000.0);
  // map every rank's ctl (all-reduce) and the send neighbours' landing buffers
  for (int q = 0; q < world && ok; ++q) {
    if (q == me) {
      P.ctl[q] = (char *)pr.ctl;
      continue;
    }
    void *m = nullptr;
    e = hipIpcOpenMemHandle(&m, cards[q].ctl, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      ok = false;
      why = std::string("hipIpcOpenMemHandle(ctl of rank ") + std::to_string(q) +
            "): " + hipGetErrorString(e);
      break;
    }
    pr.mapped.push_back(m);
    P.ctl[q] = (char *)m;
  }
  for (size_t i = 0; i < h.nbr.size() && ok; ++i) {
    const int q = h.nbr[i];
    if (h.send_cnt[i] > 0) {
      if (cards[q].recv_off[me] < 0 || cards[q].recv_cnt[me] != h.send_cnt[i]) {
        ok = false;
        why = "halo plans disagree between ranks " + std::to_string(me) + " and " +
              std::to_string(q);
        break;
      }
      void *m = nullptr;
      e = hipIpcOpenMemHandle(&m, cards[q].land, hipIpcMemLazyEnablePeerAccess);
      if (e != hipSuccess) {
        ok = false;
        why = std::string("hipIpcOpenMemHandle(landing buffer of rank ") + std::to_string(q) +
              "): " + hipGetErrorString(e);
        break;
      }
      pr.mapped.push_back(m);
      const int k = P.nsend++;
      P.send_rank[k] = q;
      P.land_remote[k] = (char *)m + (size_t)cards[q].recv_off[me] * es;
      P.send_off[k] = h.send_off[i];
      P.send_cnt[k] = h.send_cnt[i];
    }
    if (h.recv_cnt[i] > 0) P.recv_rank[P.nrecv++] = q;
  }
  // every rank mapped its peers (or nobody runs the test kernels)
  int all = 0;
  if ((rc = all_ok(ctx, ok ? 1 : 0, &all))) {
    peer_destroy(A);
    return rc;
  }
  bool passed = false;
  if (all) {
    // a failure here is this rank's "no": every rank must still reach the
    // collective below (an RCCL collective would wait for a missing rank)
    rc = A->dtype == CGX_F32 ? self_test<float>(A, &passed) : self_test<double>(A, &passed);
    if (rc) passed = false;
    if (!passed) why = cgx_last_error();
    rc = CGX_OK;
  } else if (why.empty()) {
    why = "another rank could not map its peers";
  }
  if ((rc = all_ok(ctx, passed ? 1 : 0, &all))) {
    peer_destroy(A);
    return rc;
  }
  if (!all) {
    peer_destroy(A);
    set_error("peer transport disabled: %s", why.empty() ? "another rank failed its self-test"
                                                         : why.c_str());
    return CGX_OK;
  }
  P.spin_ticks = (long long)(secs * clk_khz * 1000.0);
  P.nopoll = pr.one_waiter ? 1 : 0;
  pr.on = true;
  *enabled = 1;
  return CGX_OK;
}

extern "C" int cgx_dist_peer_info(cgx_csr *A, int *enabled) {
  CGX_REQUIRE(A && enabled, CGX_EINVAL, "NULL argument");
  *enabled = A->peer.on ? 1 : 0;
  return CGX_OK;
}

// The peer transport's iteration form (cgx.h): ranks sharing this rank's GPU
// and whether the one-waiter form runs (see Peer::one_waiter)
extern "C" int cgx_dist_peer_form(cgx_csr *A, int *colocated, int *one_waiter) {
  CGX_REQUIRE(A && colocated && one_waiter, CGX_EINVAL, "NULL argument");
  *colocated = A->peer.on ? A->peer.colocated : 0;
  *one_waiter = A->peer.on && A->peer.one_waiter ? 1 : 0;
  return CGX_OK;
}
