// cgx_dist.cpp — row-partitioned CG across the GPUs of one node (SURVEY.md
// §8(e)): one process per GPU, contiguous row blocks.
//
// The reference is single-device; this file adds the
// partition. Per iteration:
//   * halo exchange of p: every rank packs the p entries its neighbours need
//     (k_gather) and sends them; received values land in p's ghost area
//     [n_local, n_local + n_ghost), grouped by owner, so the SpMV reads local
//     and ghost entries from one array;
//   * all-reduce of p.Ap and of r.r (one scalar each, in place on the device
//     scalar ring; every rank then derives identical alpha / beta / stop).
// Transport: RCCL over xGMI (cgx_dist_init: ncclSend/ncclRecv inside one
// group, ncclAllReduce), or a host-staged transport whose collectives are
// caller callbacks (cgx_dist_init_host) — the latter lets several ranks share
// one GPU (RCCL refuses that) so the whole device path is testable on a
// single-GPU box. Setup (cgx_csr_create_dist) builds the plan from the local
// rows' global column indices with the host-only helpers cgx_plan_ghosts /
// cgx_plan_remap, which the CPU test-suite also drives over a gloo world.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cgx_objects.h"

int autotune_spmv(cgx_csr *A);  // cgx_abi.cpp
int build_sell(cgx_csr *A, const int *h_rowptr, const int *h_col, int R,
               const std::vector<char> *skip);
int lean_mark_split(cgx_csr *A, const std::vector<int> &boundary);  // cgx_abi.cpp
std::vector<int> chunked_slice_order(const std::vector<int> &ids, int64_t H, int64_t P,
                                     int64_t kChunk);  // cgx_abi.cpp

namespace cgx {

static int nccl_fail(ncclResult_t r, const char *what) {
  set_error("%s failed: %s", what, ncclGetErrorString(r));
  return CGX_ENCCL;
}

#define CGX_NCCL(expr)                                          \
  do {                                                          \
    ncclResult_t r_ = (expr);                                   \
    if (r_ != ncclSuccess) return ::cgx::nccl_fail(r_, #expr);  \
  } while (0)

#define CGX_CB(expr)                                                   \
  do {                                                                 \
    int r_ = (expr);                                                   \
    if (r_ != 0) {                                                     \
      ::cgx::set_error("host transport callback %s failed (%d)", #expr, r_); \
      return CGX_ENCCL;                                                \
    }                                                                  \
  } while (0)

static ncclDataType_t nccl_type(int dtype) { return dtype == CGX_F32 ? ncclFloat : ncclDouble; }

static bool multi(const cgx_ctx *ctx) { return ctx->world > 1 && (ctx->comm || ctx->host); }

// ---- setup collectives on HOST buffers ----------------------------------
int comm_allgather(cgx_ctx *ctx, const void *mine, size_t bytes, void *all) {
  std::memcpy((char *)all + bytes * ctx->rank, mine, bytes);
  if (!multi(ctx)) return CGX_OK;
  if (ctx->host) {
    CGX_CB(ctx->host->allgather(ctx->host->user, mine, bytes, all));
    return CGX_OK;
  }
  hipStream_t s = ctx->stream;
  void *d = nullptr;
  CGX_HIP(hipMalloc(&d, bytes * ctx->world));
  CGX_HIP(hipMemcpyAsync((char *)d + bytes * ctx->rank, mine, bytes, hipMemcpyHostToDevice, s));
  CGX_NCCL(ncclAllGather((char *)d + bytes * ctx->rank, d, bytes, ncclChar, ctx->comm, s));
  CGX_HIP(hipMemcpyAsync(all, d, bytes * ctx->world, hipMemcpyDeviceToHost, s));
  CGX_HIP(hipStreamSynchronize(s));
  CGX_HIP(hipFree(d));
  return CGX_OK;
}

// pairwise exchange of host byte buffers with the listed peers
static int comm_exchange(cgx_ctx *ctx, const std::vector<int> &peers,
                         const std::vector<const void *> &send, const std::vector<size_t> &sbytes,
                         const std::vector<void *> &recv, const std::vector<size_t> &rbytes) {
  if (peers.empty()) return CGX_OK;
  if (ctx->host) {
    CGX_CB(ctx->host->exchange(ctx->host->user, (int)peers.size(), peers.data(), send.data(),
                               sbytes.data(), recv.data(), rbytes.data()));
    return CGX_OK;
  }
  hipStream_t s = ctx->stream;
  size_t st = 0, rt = 0;
  for (size_t i = 0; i < peers.size(); ++i) {
    st += sbytes[i];
    rt += rbytes[i];
  }
  char *ds = nullptr, *dr = nullptr;
  CGX_HIP(hipMalloc(&ds, st + 1));
  CGX_HIP(hipMalloc(&dr, rt + 1));
  size_t so = 0, ro = 0;
  for (size_t i = 0; i < peers.size(); ++i) {
    if (sbytes[i]) CGX_HIP(hipMemcpyAsync(ds + so, send[i], sbytes[i], hipMemcpyHostToDevice, s));
    so += sbytes[i];
  }
  CGX_NCCL(ncclGroupStart());
  so = ro = 0;
  for (size_t i = 0; i < peers.size(); ++i) {
    if (sbytes[i]) CGX_NCCL(ncclSend(ds + so, sbytes[i], ncclChar, peers[i], ctx->comm, s));
    if (rbytes[i]) CGX_NCCL(ncclRecv(dr + ro, rbytes[i], ncclChar, peers[i], ctx->comm, s));
    so += sbytes[i];
    ro += rbytes[i];
  }
  CGX_NCCL(ncclGroupEnd());
  ro = 0;
  for (size_t i = 0; i < peers.size(); ++i) {
    if (rbytes[i]) CGX_HIP(hipMemcpyAsync(recv[i], dr + ro, rbytes[i], hipMemcpyDeviceToHost, s));
    ro += rbytes[i];
  }
  CGX_HIP(hipStreamSynchronize(s));
  CGX_HIP(hipFree(ds));
  CGX_HIP(hipFree(dr));
  return CGX_OK;
}

// ---- per-iteration collectives on DEVICE buffers ------------------------
int dist_halo_exchange(cgx_csr *A, void *vec_ext, hipStream_t s) {
  if (!A->dist) return CGX_OK;
  cgx_ctx *ctx = A->ctx;
  Halo &h = A->halo;
  if (!multi(ctx) || (h.n_ghost == 0 && h.send_total == 0)) return CGX_OK;
  const size_t es = dtype_size(A->dtype);
  if (h.send_total > 0) {
    if (A->dtype == CGX_F32)
      CGX_HIP(Launch<float>::gather((const float *)vec_ext, h.d_send_idx, h.send_total,
                                    (float *)h.d_send_buf, s));
    else
      CGX_HIP(Launch<double>::gather((const double *)vec_ext, h.d_send_idx, h.send_total,
                                     (double *)h.d_send_buf, s));
  }
  if (ctx->host) {
    // stage through pinned host memory, exchange by callback, copy back
    char *hs = (char *)h.h_send, *hr = (char *)h.h_recv;
    if (h.send_total)
      CGX_HIP(hipMemcpyAsync(hs, h.d_send_buf, (size_t)h.send_total * es, hipMemcpyDeviceToHost, s));
    CGX_HIP(hipStreamSynchronize(s));
    std::vector<const void *> sp;
    std::vector<void *> rp;
    std::vector<size_t> sb, rb;
    for (size_t i = 0; i < h.nbr.size(); ++i) {
      sp.push_back(hs + (size_t)h.send_off[i] * es);
      sb.push_back((size_t)h.send_cnt[i] * es);
      rp.push_back(hr + (size_t)h.recv_off[i] * es);
      rb.push_back((size_t)h.recv_cnt[i] * es);
    }
    CGX_CB(ctx->host->exchange(ctx->host->user, (int)h.nbr.size(), h.nbr.data(), sp.data(),
                               sb.data(), rp.data(), rb.data()));
    if (h.n_ghost)
      CGX_HIP(hipMemcpyAsync((char *)vec_ext + (size_t)A->dev.n * es, hr, (size_t)h.n_ghost * es,
                             hipMemcpyHostToDevice, s));
    CGX_HIP(hipStreamSynchronize(s));
    return CGX_OK;
  }
  const ncclDataType_t t = nccl_type(A->dtype);
  CGX_NCCL(ncclGroupStart());
  for (size_t i = 0; i < h.nbr.size(); ++i) {
    if (h.send_cnt[i] > 0)
      CGX_NCCL(ncclSend((char *)h.d_send_buf + (size_t)h.send_off[i] * es,
                        (size_t)h.send_cnt[i], t, h.nbr[i], ctx->comm, s));
    if (h.recv_cnt[i] > 0)
      CGX_NCCL(ncclRecv((char *)vec_ext + (size_t)(A->dev.n + h.recv_off[i]) * es,
                        (size_t)h.recv_cnt[i], t, h.nbr[i], ctx->comm, s));
  }
  CGX_NCCL(ncclGroupEnd());
  return CGX_OK;
}

// The asynchronous host transport's exchange: a host function on the comm
// stream, between the D2H of the packed entries and the H2D of the ghosts. It
// runs on the runtime's callback thread and makes no HIP calls; a failure is
// kept in async_rc and reported by the next host collective (which
// synchronises the solver stream, itself behind ev_halo).
static void host_exchange_cb(void *arg) {
  auto *A = (cgx_csr *)arg;
  Halo &h = A->halo;
  const size_t es = dtype_size(A->dtype);
  char *hs = (char *)h.h_send, *hr = (char *)h.h_recv;
  std::vector<const void *> sp;
  std::vector<void *> rp;
  std::vector<size_t> sb, rb;
  for (size_t i = 0; i < h.nbr.size(); ++i) {
    sp.push_back(hs + (size_t)h.send_off[i] * es);
    sb.push_back((size_t)h.send_cnt[i] * es);
    rp.push_back(hr + (size_t)h.recv_off[i] * es);
    rb.push_back((size_t)h.recv_cnt[i] * es);
  }
  const int r = A->ctx->host->exchange(A->ctx->host->user, (int)h.nbr.size(), h.nbr.data(),
                                       sp.data(), sb.data(), rp.data(), rb.data());
  if (r != 0) A->ctx->host_async_rc.store(r);
}

static int dist_async_status(cgx_ctx *ctx) {
  const int r = ctx->host_async_rc.exchange(0);
  if (r) {
    set_error("asynchronous host halo exchange callback failed (%d)", r);
    return CGX_ENCCL;
  }
  return CGX_OK;
}

int dist_halo_post(cgx_csr *A, void *vec_ext, hipStream_t s, bool *async) {
  *async = false;
  cgx_ctx *ctx = A->ctx;
  Halo &h = A->halo;
  if (!A->dist || !multi(ctx) || (h.n_ghost == 0 && h.send_total == 0)) return CGX_OK;
  const bool host_async = ctx->host && ctx->host_async;
  if ((ctx->host && !host_async) || !ctx->cstream || !A->ev_pack || !A->ev_halo)
    return dist_halo_exchange(A, vec_ext, s);  // synchronous
  int rc;
  if ((rc = dist_async_status(ctx))) return rc;
  const size_t es = dtype_size(A->dtype);
  if (h.send_total > 0) {
    if (A->dtype == CGX_F32)
      CGX_HIP(Launch<float>::gather((const float *)vec_ext, h.d_send_idx, h.send_total,
                                    (float *)h.d_send_buf, s));
    else
      CGX_HIP(Launch<double>::gather((const double *)vec_ext, h.d_send_idx, h.send_total,
                                     (double *)h.d_send_buf, s));
  }
  // the exchange runs on the comm stream once the pack (and everything before
  // it on s) is done; the interior rows proceed on s meanwhile
  CGX_HIP(hipEventRecord(A->ev_pack, s));
  CGX_HIP(hipStreamWaitEvent(ctx->cstream, A->ev_pack, 0));
  if (host_async) {
    // D2H, the exchange as a host function, H2D — all ordered on cstream
    if (h.send_total)
      CGX_HIP(hipMemcpyAsync(h.h_send, h.d_send_buf, (size_t)h.send_total * es,
                             hipMemcpyDeviceToHost, ctx->cstream));
    CGX_HIP(hipLaunchHostFunc(ctx->cstream, host_exchange_cb, A));
    if (h.n_ghost)
      CGX_HIP(hipMemcpyAsync((char *)vec_ext + (size_t)A->dev.n * es, h.h_recv,
                             (size_t)h.n_ghost * es, hipMemcpyHostToDevice, ctx->cstream));
    CGX_HIP(hipEventRecord(A->ev_halo, ctx->cstream));
    h.async_calls += 1;
    *async = true;
    return CGX_OK;
  }
  const ncclDataType_t t = nccl_type(A->dtype);
  CGX_NCCL(ncclGroupStart());
  for (size_t i = 0; i < h.nbr.size(); ++i) {
    if (h.send_cnt[i] > 0)
      CGX_NCCL(ncclSend((char *)h.d_send_buf + (size_t)h.send_off[i] * es,
                        (size_t)h.send_cnt[i], t, h.nbr[i], ctx->comm, ctx->cstream));
    if (h.recv_cnt[i] > 0)
      CGX_NCCL(ncclRecv((char *)vec_ext + (size_t)(A->dev.n + h.recv_off[i]) * es,
                        (size_t)h.recv_cnt[i], t, h.nbr[i], ctx->comm, ctx->cstream));
  }
  CGX_NCCL(ncclGroupEnd());
  CGX_HIP(hipEventRecord(A->ev_halo, ctx->cstream));
  *async = true;
  return CGX_OK;
}

int dist_allreduce_scalar(cgx_ctx *ctx, void *d_val, int dtype, int count, hipStream_t s) {
  if (!multi(ctx)) return CGX_OK;
  if (ctx->host) {
    CGX_REQUIRE(count <= 8, CGX_EINVAL, "host all-reduce of %d values", count);
    const size_t es = dtype_size(dtype);
    auto *h = (char *)ctx->h_pinned + 512;  // [0, 512) is cgx_cg_run's poll staging
    CGX_HIP(hipMemcpyAsync(h, d_val, es * count, hipMemcpyDeviceToHost, s));
    CGX_HIP(hipStreamSynchronize(s));
    // a failed asynchronous exchange on this rank still enters the
    // collective (its peers would otherwise wait in it forever) and carries
    // the failure in a status word beside the values: all ranks fail together
    const int mine = dist_async_status(ctx);
    const std::string why = mine ? cgx_last_error() : "";
    double v[9];
    for (int i = 0; i < count; ++i)
      v[i] = dtype == CGX_F32 ? (double)((float *)h)[i] : ((double *)h)[i];
    v[count] = mine ? 1.0 : 0.0;
    CGX_CB(ctx->host->allreduce(ctx->host->user, v, count + 1));
    if (mine) {
      set_error("%s", why.c_str());
      return mine;
    }
    CGX_REQUIRE(v[count] == 0.0, CGX_ENCCL,
                "host transport: the halo exchange failed on %g other rank(s)", v[count]);
    for (int i = 0; i < count; ++i) {
      if (dtype == CGX_F32) ((float *)h)[i] = (float)v[i];
      else ((double *)h)[i] = v[i];
    }
    CGX_HIP(hipMemcpyAsync(d_val, h, es * count, hipMemcpyHostToDevice, s));
    CGX_HIP(hipStreamSynchronize(s));
    return dist_async_status(ctx);  // s waited on every halo posted before
  }
  CGX_NCCL(ncclAllReduce(d_val, d_val, (size_t)count, nccl_type(dtype), ncclSum, ctx->comm, s));
  return CGX_OK;
}

int dist_destroy_halo(cgx_csr *A) {
  // an exchange still queued on the comm stream reads this matrix's halo
  // (the asynchronous host transport's host function): drain it first
  if (A->ctx && A->ctx->cstream) (void)hipStreamSynchronize(A->ctx->cstream);
  if (A->ev_pack) (void)hipEventDestroy(A->ev_pack);
  if (A->ev_halo) (void)hipEventDestroy(A->ev_halo);
  A->ev_pack = A->ev_halo = nullptr;
  if (A->halo.d_send_idx) (void)hipFree(A->halo.d_send_idx);
  if (A->halo.d_send_buf) (void)hipFree(A->halo.d_send_buf);
  if (A->halo.h_send) (void)hipHostFree(A->halo.h_send);
  if (A->halo.h_recv) (void)hipHostFree(A->halo.h_recv);
  A->halo.d_send_idx = nullptr;
  A->halo.d_send_buf = nullptr;
  A->halo.h_send = A->halo.h_recv = nullptr;
  return CGX_OK;
}

int dist_comm_destroy(cgx_ctx *ctx) {
  if (ctx->cstream) {
    (void)hipStreamSynchronize(ctx->cstream);
    (void)hipStreamDestroy(ctx->cstream);
    ctx->cstream = nullptr;
  }
  if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
  ctx->comm = nullptr;
  delete ctx->host;
  ctx->host = nullptr;
  return CGX_OK;
}

}  // namespace cgx

using namespace cgx;

// ===========================================================================
// host-only plan helpers (no device access; usable without a GPU)
// ===========================================================================

// Ghost columns of a local row block: the sorted distinct global columns
// outside [row_begin, row_begin + n_local), and how many of them each rank
// owns (begins/counts: every rank's row range, indexed by rank).
extern "C" int cgx_plan_ghosts(int64_t n_local, int64_t row_begin, int64_t nnz, const int *col,
                               int world, const int64_t *begins, const int64_t *counts,
                               int64_t *n_ghost, int64_t **ghosts, int64_t *recv_cnt) {
  CGX_REQUIRE(col || nnz == 0, CGX_EINVAL, "col is NULL");
  CGX_REQUIRE(n_ghost && ghosts && recv_cnt && begins && counts && world >= 1, CGX_EINVAL,
              "NULL argument");
  // ghosts sorted by global index are grouped by owner only when the row
  // ranges are ordered by rank
  for (int r = 1; r < world; ++r)
    CGX_REQUIRE(begins[r] >= begins[r - 1] + counts[r - 1], CGX_EINVAL,
                "row ranges must be contiguous and ordered by rank");
  const int64_t lo = row_begin, hi = row_begin + n_local;
  std::vector<int64_t> g;
  for (int64_t k = 0; k < nnz; ++k) {
    const int64_t c = col[k];
    if (c < lo || c >= hi) g.push_back(c);
  }
  std::sort(g.begin(), g.end());
  g.erase(std::unique(g.begin(), g.end()), g.end());
  std::fill(recv_cnt, recv_cnt + world, 0);
  int owner = 0;
  for (int64_t c : g) {  // g ascending and ranges ordered: owner only grows
    while (owner < world && c >= begins[owner] + counts[owner]) ++owner;
    CGX_REQUIRE(owner < world && c >= begins[owner], CGX_EINVAL,
                "column %lld is owned by no rank", (long long)c);
    recv_cnt[owner] += 1;
  }
  *n_ghost = (int64_t)g.size();
  *ghosts = (int64_t *)std::malloc(std::max<size_t>(g.size(), 1) * sizeof(int64_t));
  std::copy(g.begin(), g.end(), *ghosts);
  return CGX_OK;
}

// Rewrite global columns to local numbering: own rows -> c - row_begin,
// ghosts -> n_local + position in the sorted ghost list.
extern "C" int cgx_plan_remap(int64_t n_local, int64_t row_begin, int64_t nnz, int *col,
                              int64_t n_ghost, const int64_t *ghosts) {
  CGX_REQUIRE(col || nnz == 0, CGX_EINVAL, "col is NULL");
  const int64_t lo = row_begin, hi = row_begin + n_local;
  for (int64_t k = 0; k < nnz; ++k) {
    const int64_t c = col[k];
    if (c >= lo && c < hi) {
      col[k] = (int)(c - lo);
    } else {
      const int64_t *it = std::lower_bound(ghosts, ghosts + n_ghost, c);
      CGX_REQUIRE(it != ghosts + n_ghost && *it == c, CGX_EINVAL,
                  "column %lld missing from ghost list", (long long)c);
      col[k] = (int)(n_local + (it - ghosts));
    }
  }
  return CGX_OK;
}

extern "C" void cgx_free_host(void *p) { std::free(p); }

extern "C" int cgx_row_blocks(const int *rowptr, int64_t n, int64_t *nrb, int **rb,
                              int *max_row_nnz) {
  CGX_REQUIRE(rowptr && nrb && rb, CGX_EINVAL, "NULL argument");
  std::vector<int> v = build_row_blocks(rowptr, n, max_row_nnz);
  *nrb = (int64_t)v.size() - 1;
  *rb = (int *)std::malloc(v.size() * sizeof(int));
  std::copy(v.begin(), v.end(), *rb);
  return CGX_OK;
}

// ===========================================================================
// communicators
// ===========================================================================
extern "C" int cgx_nccl_unique_id(char *id_out, size_t len) {
  CGX_REQUIRE(id_out && len >= sizeof(ncclUniqueId), CGX_EINVAL, "buffer too small (%zu < %zu)",
              len, sizeof(ncclUniqueId));
  ncclUniqueId id;
  CGX_NCCL(ncclGetUniqueId(&id));
  std::memcpy(id_out, &id, sizeof(id));
  return CGX_OK;
}

extern "C" int cgx_dist_init(cgx_ctx *ctx, int rank, int world, const char *id, size_t len) {
  CGX_REQUIRE(ctx && id && len >= sizeof(ncclUniqueId), CGX_EINVAL, "bad argument");
  CGX_REQUIRE(world >= 1 && rank >= 0 && rank < world, CGX_EINVAL, "bad rank/world");
  CGX_REQUIRE(!ctx->comm && !ctx->host, CGX_ESTATE, "communicator already initialised");
  CGX_HIP(hipSetDevice(ctx->device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t comm = nullptr;
  CGX_NCCL(ncclCommInitRank(&comm, world, uid, rank));
  ctx->comm = comm;
  if (world > 1) CGX_HIP(hipStreamCreateWithFlags(&ctx->cstream, hipStreamNonBlocking));
  ctx->rank = rank;
  ctx->world = world;
  return CGX_OK;
}

extern "C" int cgx_dist_init_host(cgx_ctx *ctx, int rank, int world, cgx_allgather_fn ag,
                                  cgx_allreduce_fn ar, cgx_exchange_fn ex, void *user) {
  CGX_REQUIRE(ctx && ag && ar && ex, CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(world >= 1 && rank >= 0 && rank < world, CGX_EINVAL, "bad rank/world");
  CGX_REQUIRE(!ctx->comm && !ctx->host, CGX_ESTATE, "communicator already initialised");
  ctx->host = new HostComm{ag, ar, ex, user};
  ctx->rank = rank;
  ctx->world = world;
  return CGX_OK;
}

// Host transport only: run the per-iteration halo exchange on a comm stream
// (D2H, the exchange callback as a host function, H2D, then an event the
// solver stream waits on) so that a split SpMV's interior slices overlap it —
// the same stream/event ordering as the RCCL exchange. Call before creating
// the partitioned matrices (their events are made at creation).
extern "C" int cgx_dist_host_async(cgx_ctx *ctx, int on) {
  CGX_REQUIRE(ctx, CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(ctx->host, CGX_ESTATE, "no host transport (cgx_dist_init_host first)");
  CGX_HIP(hipSetDevice(ctx->device));
  if (on && !ctx->cstream && ctx->world > 1)
    CGX_HIP(hipStreamCreateWithFlags(&ctx->cstream, hipStreamNonBlocking));
  ctx->host_async = on != 0;
  return CGX_OK;
}

extern "C" int cgx_csr_halo_async_calls(cgx_csr *A, int64_t *calls) {
  CGX_REQUIRE(A && calls, CGX_EINVAL, "NULL argument");
  *calls = A->halo.async_calls;
  return CGX_OK;
}

extern "C" int cgx_dist_rank(cgx_ctx *ctx, int *rank, int *world) {
  CGX_REQUIRE(ctx && rank && world, CGX_EINVAL, "NULL argument");
  *rank = ctx->rank;
  *world = ctx->world;
  return CGX_OK;
}

extern "C" int cgx_dist_allreduce_sum(cgx_ctx *ctx, double *value) {
  CGX_REQUIRE(ctx && value, CGX_EINVAL, "NULL argument");
  if (!multi(ctx)) return CGX_OK;
  CGX_HIP(hipSetDevice(ctx->device));
  CGX_HIP(hipMemcpyAsync(ctx->scratch, value, sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  int rc = dist_allreduce_scalar(ctx, ctx->scratch, CGX_F64, 1, ctx->stream);
  if (rc) return rc;
  CGX_HIP(hipMemcpyAsync(value, ctx->scratch, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  CGX_HIP(hipStreamSynchronize(ctx->stream));
  return CGX_OK;
}

// ===========================================================================
// distributed CSR
// ===========================================================================
extern "C" int cgx_csr_create_dist(cgx_ctx *ctx, int64_t n_global, int64_t row_begin,
                                   int64_t n_local, int64_t nnz_local, const int *d_rowptr,
                                   int *d_col, const void *d_val, int dtype, cgx_csr **out) {
  CGX_REQUIRE(ctx && out && d_rowptr && d_col && d_val, CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(ctx->world == 1 || multi(ctx), CGX_ESTATE, "cgx_dist_init first");
  CGX_REQUIRE(n_local >= 1 && row_begin >= 0 && row_begin + n_local <= n_global, CGX_EINVAL,
              "bad local row range");
  CGX_REQUIRE(dtype == CGX_F64 || dtype == CGX_F32, CGX_EINVAL, "bad dtype %d", dtype);
  CGX_HIP(hipSetDevice(ctx->device));
  *out = nullptr;
  hipStream_t s = ctx->stream;
  const int world = ctx->world, me = ctx->rank;
  int rc;
  const auto t_start = std::chrono::steady_clock::now();
  // 1. every rank's row range
  std::vector<int64_t> part(2 * (size_t)world, 0);
  const int64_t mine[2] = {row_begin, n_local};
  if ((rc = comm_allgather(ctx, mine, sizeof(mine), part.data()))) return rc;
  std::vector<int64_t> begins(world), counts(world);
  for (int r = 0; r < world; ++r) {
    begins[r] = part[2 * r];
    counts[r] = part[2 * r + 1];
  }
  // 2. local structure to the host, ghost list
  std::vector<int> hrp((size_t)n_local + 1), hcol((size_t)nnz_local);
  CGX_HIP(hipMemcpyAsync(hrp.data(), d_rowptr, hrp.size() * sizeof(int), hipMemcpyDeviceToHost, s));
  CGX_HIP(hipMemcpyAsync(hcol.data(), d_col, hcol.size() * sizeof(int), hipMemcpyDeviceToHost, s));
  CGX_HIP(hipStreamSynchronize(s));
  CGX_REQUIRE(hrp[0] == 0 && hrp[n_local] == nnz_local, CGX_EINVAL,
              "local rowptr must run from 0 to nnz_local");
  int64_t n_ghost = 0;
  int64_t *gp = nullptr;
  std::vector<int64_t> recv_cnt(world, 0);
  if ((rc = cgx_plan_ghosts(n_local, row_begin, nnz_local, hcol.data(), world, begins.data(),
                            counts.data(), &n_ghost, &gp, recv_cnt.data())))
    return rc;
  std::vector<int64_t> ghosts(gp, gp + n_ghost);
  cgx_free_host(gp);
  // 3. every rank's receive counts -> my send counts
  std::vector<int64_t> cmat((size_t)world * world, 0);
  if ((rc = comm_allgather(ctx, recv_cnt.data(), world * sizeof(int64_t), cmat.data()))) return rc;
  auto *A = new cgx_csr();
  A->ctx = ctx;
  ctx_retain(ctx);
  A->dtype = dtype;
  A->dist = true;
  A->n_global = n_global;
  A->row_begin = row_begin;
  Halo &h = A->halo;
  h.n_ghost = n_ghost;
  int64_t roff = 0, soff = 0;
  for (int r = 0; r < world; ++r) {
    const int64_t rc_ = recv_cnt[r], sc_ = cmat[(size_t)r * world + me];
    if (r == me || (rc_ == 0 && sc_ == 0)) continue;
    h.nbr.push_back(r);
    h.recv_cnt.push_back(rc_);
    h.recv_off.push_back(roff);
    h.send_cnt.push_back(sc_);
    h.send_off.push_back(soff);
    roff += rc_;
    soff += sc_;
  }
  h.send_total = soff;
  // 4. request lists: the global ids I need go to their owners
  std::vector<int> req(ghosts.begin(), ghosts.end()), inc((size_t)std::max<int64_t>(soff, 1));
  {
    std::vector<const void *> sp;
    std::vector<void *> rp;
    std::vector<size_t> sb, rb;
    for (size_t i = 0; i < h.nbr.size(); ++i) {
      sp.push_back(req.data() + h.recv_off[i]);
      sb.push_back((size_t)h.recv_cnt[i] * sizeof(int));
      rp.push_back(inc.data() + h.send_off[i]);
      rb.push_back((size_t)h.send_cnt[i] * sizeof(int));
    }
    if ((rc = comm_exchange(ctx, h.nbr, sp, sb, rp, rb))) {
      cgx_csr_destroy(A);
      return rc;
    }
  }
  for (int64_t i = 0; i < soff; ++i) {
    const int64_t g = inc[i];
    if (g < row_begin || g >= row_begin + n_local) {
      cgx_csr_destroy(A);
      set_error("rank %d was asked for row %lld it does not own", me, (long long)g);
      return CGX_EINVAL;
    }
    inc[i] = (int)(g - row_begin);
  }
  const size_t es = dtype_size(dtype);
  hipError_t e = hipMalloc(&h.d_send_idx, (size_t)std::max<int64_t>(soff, 1) * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&h.d_send_buf, (size_t)std::max<int64_t>(soff, 1) * es);
  if (e == hipSuccess && soff)
    e = hipMemcpyAsync(h.d_send_idx, inc.data(), (size_t)soff * sizeof(int),
                       hipMemcpyHostToDevice, s);
  if (e == hipSuccess && ctx->host) {
    e = hipHostMalloc(&h.h_send, (size_t)std::max<int64_t>(soff, 1) * es, hipHostMallocDefault);
    if (e == hipSuccess)
      e = hipHostMalloc(&h.h_recv, (size_t)std::max<int64_t>(n_ghost, 1) * es,
                        hipHostMallocDefault);
  }
  if (e != hipSuccess) {
    cgx_csr_destroy(A);
    return hip_fail(e, "cgx_csr_create_dist(send plan)");
  }
  // 5. columns to local numbering, back to the device
  if ((rc = cgx_plan_remap(n_local, row_begin, nnz_local, hcol.data(), n_ghost, ghosts.data()))) {
    cgx_csr_destroy(A);
    return rc;
  }
  e = hipMemcpyAsync(d_col, hcol.data(), hcol.size() * sizeof(int), hipMemcpyHostToDevice, s);
  // 6. boundary rows (any ghost column) in 128-row slices (the SELL-P
  // slice), and the SpMV schedule over the local rows (+ entry offsets), cut
  // at the ends of the boundary runs so its blocks lie inside or outside them
  const int64_t HS = 2 * kSellRows;
  const int64_t nsl_b = (n_local + HS - 1) / HS;
  std::vector<char> bslice((size_t)nsl_b, 0);
  for (int64_t r = 0; r < n_local; ++r)
    for (int64_t k = hrp[(size_t)r]; k < hrp[(size_t)r + 1]; ++k)
      if (hcol[(size_t)k] >= n_local) {
        bslice[(size_t)(r / HS)] = 1;
        break;
      }
  std::vector<int64_t> cuts;
  for (int64_t q = 0; q < nsl_b; ++q)
    if (bslice[(size_t)q] != (q > 0 ? bslice[(size_t)q - 1] : 0)) cuts.push_back(q * HS);
  int mx = 0;
  std::vector<int> rb = build_row_blocks(hrp.data(), n_local, &mx, kTile, &cuts);
  const size_t nrb1 = rb.size();
  rb.resize(2 * nrb1);
  for (size_t i = 0; i < nrb1; ++i) rb[nrb1 + i] = hrp[rb[i]];
  if (e == hipSuccess) e = hipMalloc(&A->d_rb, rb.size() * sizeof(int));
  if (e == hipSuccess)
    e = hipMemcpyAsync(A->d_rb, rb.data(), rb.size() * sizeof(int), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    cgx_csr_destroy(A);
    return hip_fail(e, "cgx_csr_create_dist(schedule)");
  }
  A->max_row_nnz = mx;
  A->dev = CsrDev{n_local, nnz_local, d_rowptr, d_col, d_val, A->d_rb, A->d_rb + nrb1,
                  (int)nrb1 - 1, kTile};
  // the boundary slices are placeholders in the SELL copy (their rows may be
  // unsorted locally: ghosts from lower ranks are numbered after the own
  // rows); the boundary launch runs their rows as CSR-stream blocks
  setup_begin(A);
  A->setup_last = t_start;
  setup_mark(A, 0);
  if ((rc = build_sell(A, hrp.data(), hcol.data(), 0, h.n_ghost > 0 ? &bslice : nullptr))) {
    cgx_csr_destroy(A);
    return rc;
  }
  setup_mark(A, 2);
  // interior / boundary slices of the SELL copy: the halo exchange overlaps
  // the interior ones (enqueue_iter); a slab of a stencil has one boundary
  // plane per neighbour. Built before the autotune, which times the SELL
  // forms and the lean walk over the interior list (freed with the SELL copy
  // when a CSR-stream form wins).
  if (A->dev.sl && h.n_ghost > 0) {
    const int64_t H = (int64_t)kSellRows * A->dev.sell_r, nsl = A->dev.nsl;
    std::vector<int> in, bd;
    for (int64_t q = 0; q < nsl; ++q) {
      // boundary: inside a 128-row run that holds a ghost column (the rows
      // the boundary launch's CSR blocks cover, so no row runs twice)
      const bool ghost = bslice[(size_t)(q * H / HS)] != 0;
      (ghost ? bd : in).push_back((int)q);
    }
    // the interior slices in the chunked visit order of a single-device
    // matrix (cgx_abi.cpp build_sell), planed by the farthest local band
    // (ghost columns excluded): the 512x512x64 slab's planes span 2,048
    // slices, as 512^3's do
    if (!in.empty() && !bd.empty()) {
      int64_t P = 0;
      for (int64_t r = 0; r < n_local; ++r)
        for (int64_t k = hrp[(size_t)r]; k < hrp[(size_t)r + 1]; ++k) {
          const int64_t c = hcol[(size_t)k];
          if (c < n_local) P = std::max<int64_t>(P, c > r ? c - r : r - c);
        }
      std::vector<int> o = chunked_slice_order(in, H, P, 512);
      if (!o.empty()) {
        in.swap(o);
        A->split_ordered = true;
      }
    }
    if (!in.empty() && !bd.empty()) {
      A->split_bd_h = bd;
      in.insert(in.end(), bd.begin(), bd.end());
      e = hipMalloc(&A->d_split, in.size() * sizeof(int));
      if (e == hipSuccess)
        e = hipMemcpyAsync(A->d_split, in.data(), in.size() * sizeof(int), hipMemcpyHostToDevice,
                           s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e == hipSuccess && ctx->cstream && !A->ev_pack)
        e = hipEventCreateWithFlags(&A->ev_pack, hipEventDisableTiming);
      if (e == hipSuccess && ctx->cstream && !A->ev_halo)
        e = hipEventCreateWithFlags(&A->ev_halo, hipEventDisableTiming);
      if (e != hipSuccess) {
        cgx_csr_destroy(A);
        return hip_fail(e, "cgx_csr_create_dist(slice split)");
      }
      A->split_ni = (int)(in.size() - bd.size());
      A->split_nb = (int)bd.size();
      // the boundary rows' CSR-stream blocks (whole blocks: the schedule is
      // cut at the runs' ends)
      std::vector<int> blk;
      for (int b = 0; b + 1 < (int)nrb1; ++b)
        if (bslice[(size_t)(rb[(size_t)b] / HS)]) blk.push_back(b);
      if (!blk.empty()) {
        e = hipMalloc(&A->d_bnd_blk, blk.size() * sizeof(int));
        if (e == hipSuccess)
          e = hipMemcpyAsync(A->d_bnd_blk, blk.data(), blk.size() * sizeof(int),
                             hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
          cgx_csr_destroy(A);
          return hip_fail(e, "cgx_csr_create_dist(boundary blocks)");
        }
        A->bnd_nblk = (int)blk.size();
      }
    }
  }
  setup_mark(A, 3);
  if ((rc = autotune_spmv(A))) {
    cgx_csr_destroy(A);
    return rc;
  }
  setup_mark(A, 4);
  if (!A->dev.sl) A->split_bd_h.clear();  // a CSR-stream form won: no split
  // a lean loop SpMV walks the interior only (the boundary slices are the
  // boundary launch's)
  if (A->split_ni > 0 && (rc = lean_mark_split(A, A->split_bd_h))) {
    cgx_csr_destroy(A);
    return rc;
  }
  setup_mark(A, 5);
  A->setup_open = false;
  *out = A;
  return CGX_OK;
}

extern "C" int cgx_csr_split_info(cgx_csr *A, int *ni, int *nb) {
  CGX_REQUIRE(A, CGX_EINVAL, "A is NULL");
  if (ni) *ni = A->split_ni;
  if (nb) *nb = A->split_nb;
  return CGX_OK;
}

extern "C" int cgx_csr_halo_info(cgx_csr *A, int64_t *ghosts, int *neighbours) {
  CGX_REQUIRE(A, CGX_EINVAL, "A is NULL");
  if (ghosts) *ghosts = A->halo.n_ghost;
  if (neighbours) *neighbours = (int)A->halo.nbr.size();
  return CGX_OK;
}
