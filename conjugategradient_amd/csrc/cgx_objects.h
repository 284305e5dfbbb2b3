// cgx_objects.h — definitions of the opaque C-ABI handles (cgx.h), shared by
// cgx_abi.cpp (single-device engine) and cgx_dist.cpp (RCCL row partition).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/cgx.h"
#include "cgx_internal.h"

struct ncclComm;

namespace cgx {

void set_error(const char *fmt, ...);
int hip_fail(hipError_t e, const char *what);

#define CGX_HIP(expr)                                   \
  do {                                                  \
    hipError_t e_ = (expr);                             \
    if (e_ != hipSuccess) return ::cgx::hip_fail(e_, #expr); \
  } while (0)

#define CGX_REQUIRE(cond, code, ...)   \
  do {                                 \
    if (!(cond)) {                     \
      ::cgx::set_error(__VA_ARGS__);   \
      return (code);                   \
    }                                  \
  } while (0)

inline size_t dtype_size(int dtype) { return dtype == CGX_F32 ? 4 : 8; }

// Halo plan of a row-partitioned matrix (cgx_dist.cpp).
struct Halo {
  int64_t n_ghost = 0;
  std::vector<int> nbr;            // neighbour ranks
  std::vector<int64_t> recv_cnt;   // ghosts received from nbr[i] (contiguous)
  std::vector<int64_t> recv_off;   // offset of that run inside the ghost area
  std::vector<int64_t> send_cnt;   // entries sent to nbr[i]
  std::vector<int64_t> send_off;   // offset inside send_idx / send_buf
  int *d_send_idx = nullptr;       // local row indices to pack, all nbrs
  void *d_send_buf = nullptr;      // packed values
  void *h_send = nullptr;          // pinned staging (host transport only)
  void *h_recv = nullptr;
  int64_t send_total = 0;
  int64_t async_calls = 0;         // exchanges posted on the comm stream (host transport)
};

// Device peer transport over xGMI (cgx_peer.hip): the
// iteration's halo exchange and both dot all-reduces as plain kernels that
// store straight into the other ranks' memory (hipIpc-mapped, uncached), so
// a partitioned iteration is all kernels and graph-capturable.
constexpr int kPeerMax = 16;  // ranks of one node
constexpr int kPushWG = 16;   // push workgroups (and flags) per neighbour
struct PeerState {            // device, per matrix
  unsigned long long ar;      // all-reduces completed (the tag of the last)
  int fault;                  // a spin timed out: every later peer kernel returns
  int pad;
  // the tag base of the body in slot s is arb[s & 1]: its push and wait use
  // it, its two all-reduces base + 1 and base + 2; the second writes
  // arb[(s + 1) & 1] (read by no kernel of this body, so the all-reduce can
  // run inside a many-workgroup consumer kernel)
  unsigned long long arb[2];
  // the highest all-reduce tag a workgroup of a consumer kernel has claimed
  // to publish (peerdev::world_sum): the first workgroup to arrive for a tag
  // publishes it, whichever it is, so no workgroup waits on one that may not
  // be resident
  unsigned long long pub;
};
struct PeerDev {  // kernel argument (by value)
  char *ctl[kPeerMax];            // rank q's mailbox + flags, as mapped here
  void *land_remote[kPeerMax];    // send neighbour i: where my values land on it
  int send_rank[kPeerMax];        // send neighbour i's rank
  int64_t send_off[kPeerMax];     // send neighbour i: first entry in send_idx
  int64_t send_cnt[kPeerMax];
  int recv_rank[kPeerMax];        // ranks whose values land here
  const int *send_idx;
  const void *land_local;         // my landing buffer (n_ghost values)
  PeerState *state;
  int64_t n_local, n_ghost;
  long long spin_ticks;           // wall-clock ticks before a spin gives up
  int rank, world, nsend, nrecv;
  // one-waiter form (Peer::one_waiter): a one-workgroup k_peer_wait launch
  // precedes the boundary launch, whose workgroups then skip the flag poll
  int nopoll;
  int pad_;
};
// mailbox layout inside a rank's ctl allocation: val[2][kPeerMax] double-
// length pairs (hi, lo), tag[2][kPeerMax] u64 (parity = tag & 1), then
// flag[kPeerMax][kPushWG] u64
constexpr int kPeerTagOff = 4 * kPeerMax * 8;
constexpr int kPeerFlagOff = 6 * kPeerMax * 8;
constexpr size_t kPeerCtlBytes = kPeerFlagOff + (size_t)kPeerMax * kPushWG * 8;
struct Peer {
  bool on = false;
  void *ctl = nullptr;    // this rank's ctl (uncached, IPC-exported)
  void *land = nullptr;   // this rank's landing buffer (uncached, IPC-exported)
  void *state = nullptr;  // PeerState
  std::vector<void *> mapped;  // IPC mappings of other ranks' buffers
  PeerDev dev{};
  // ranks whose device is this rank's (PCI bus id; 1 on a one-GPU-per-rank
  // node) and the iteration form taken on every rank (cgx_dist_peer_enable):
  // in the one-waiter form at most one workgroup per rank waits on another
  // rank at any time (k_peer_wait with one workgroup before the boundary
  // launch, k_peer_allreduce before the kernels that consume a dot), so
  // ranks that share a GPU cannot starve each other of CUs; the fused form
  // lets whole grids wait, which is safe only when no waiting grid holds the
  // CUs a peer needs to make progress (DESIGN.md §9 "Ranks sharing a GPU")
  int colocated = 1;
  bool one_waiter = false;
};

// Host-staged transport (cgx_dist_init_host): collectives are callbacks.
struct HostComm {
  cgx_allgather_fn allgather;
  cgx_allreduce_fn allreduce;
  cgx_exchange_fn exchange;
  void *user;
};

}  // namespace cgx

// Lifetime: a context is referenced by its owner (cgx_create .. cgx_destroy)
// and by every cgx_csr / cgx_cg made on it; a matrix by its owner and by every
// solver made on it. The last release frees the object, so handles may be
// destroyed in any order (cgx_destroy before cgx_csr_destroy is valid).
struct cgx_ctx {
  std::atomic<int> refs{1};
  int device = 0;
  hipStream_t stream = nullptr;
  void *ws = nullptr;           // cgx::RedWs<double> (large enough for float)
  void *scratch = nullptr;      // 2 doubles for accuracy() results
  void *spmv_st = nullptr;      // CgScalars<double>, then <float>: slot 0 active (cgx_spmv)
  void *h_pinned = nullptr;     // pinned host staging (1 KiB: polls | host all-reduce)
  // pinned ring for large host<->device copies (cgx_h2d / cgx_d2h), lazily
  void *stage[2] = {nullptr, nullptr};
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  // multi-GPU
  ncclComm *comm = nullptr;
  cgx::HostComm *host = nullptr;
  int rank = 0, world = 1;
  hipStream_t cstream = nullptr;  // halo exchange, overlapped with interior rows
  bool host_async = false;        // host transport: exchange on cstream (cgx_dist_host_async)
  // the asynchronous exchange callback's status (a host function on cstream;
  // read once the solver stream, which waited on it, has synchronised)
  std::atomic<int> host_async_rc{0};
};

struct cgx_csr {
  std::atomic<int> refs{1};
  cgx_ctx *ctx = nullptr;
  cgx::CsrDev dev{};
  int dtype = CGX_F64;
  int *d_rb = nullptr;
  int max_row_nnz = 0;
  // distributed view
  bool dist = false;
  int64_t n_global = 0, row_begin = 0;
  cgx::Halo halo;
  void *d_ext = nullptr;  // scratch vector with ghost area (n + n_ghost)
  // SELL-64 copy (cgx::CsrDev::sl ...), null when absent
  void *d_sell_sl = nullptr, *d_sell_dict = nullptr, *d_sell_idx = nullptr;
  void *d_sell_val = nullptr;
  void *d_sell_order = nullptr;
  void *d_sell_mask = nullptr;  // SELL-P slot masks
  void *d_sell_vc = nullptr, *d_sell_vdict = nullptr;  // SELL-P value codes, dictionary
  void *d_sell_vc4 = nullptr;                          // 4-bit value codes
  void *d_sell_sl_t = nullptr, *d_vct = nullptr;       // value-code templates (kVT)
  int64_t vt_slices = 0;                               // slices that read a template
  void *d_col16 = nullptr;  // CSR-stream 16-bit column deltas (cgx::CsrDev::col16)
  void *d_il = nullptr;     // CSR-stream interleaved val / col copy (cgx::CsrDev::il)
  void *d_rbo = nullptr;    // CSR-stream block visit order (cgx::CsrDev::rbo)
  // lean stencil walk (kVL, cgx_abi.cpp build_lean): per-slice classes in
  // slice order (host), their device layout for grid dev.vl_grid, the table
  std::vector<int> sell_pool;               // the SELL-P pattern pool (host copy)
  std::vector<unsigned char> vl_slice_cls;  // class per slice (0xff: per-slice form)
  int vl_ncls = 0;
  std::vector<cgx::VlClass> vl_tab_h;  // the class table (host copy, for a re-layout)
  void *d_vl_cls = nullptr, *d_vl_tab = nullptr;
  // partitioned SELL matrix: slices without ghost columns, then those with
  // (d_split[0, split_ni) interior, [split_ni, split_ni + split_nb) boundary)
  int *d_split = nullptr;
  int split_ni = 0, split_nb = 0;
  // the boundary rows as CSR-stream row blocks (block ids into dev.rb; the
  // schedule is cut at the boundary runs' ends): the boundary launch runs
  // CSR-stream, in the rows' own entry order
  int *d_bnd_blk = nullptr;
  int bnd_nblk = 0;
  bool split_ordered = false;  // interior list in the chunked visit order
  std::vector<int> split_bd_h;  // the boundary slices (host copy: the lean walk's 0xfe marks)
  // the SpMV autotune's record (cgx_abi.cpp autotune_spmv): every form timed,
  // how (CGX_TUNE_* of cgx.h) and its median µs per launch
  struct TuneRec {
    int variant, kind;
    float us;
  };
  std::vector<TuneRec> tune;
  hipEvent_t ev_pack = nullptr, ev_halo = nullptr;
  cgx::Peer peer;  // device peer transport (cgx_dist_peer_enable)
  int64_t sell_padded = 0;
  int64_t sell_idx_words = 0;  // dictionary SELL index words
  int64_t vc_chunks = 0;       // value-code chunk-lanes (16 B each, 8 B in 4-bit form)
  // setup cost by phase (cgx_csr_setup_times): 0 schedule / halo plan,
  // 1 SELL plan + pack, 2 value codes + templates, 3 interior / boundary
  // split, 4 SpMV autotune (lean layouts included), 5 the rest; wall ms
  double setup_ms[6] = {0, 0, 0, 0, 0, 0};
  bool setup_open = false;
  std::chrono::steady_clock::time_point setup_last{};
};

struct cgx_cg {
  cgx_ctx *ctx = nullptr;
  cgx_csr *A = nullptr;
  int dtype = CGX_F64;
  int64_t n = 0;
  void *r = nullptr, *p = nullptr, *Ap = nullptr;  // p, Ap: n + n_ghost
  void *p2 = nullptr;   // second p buffer of the fused iteration (single device)
  bool fused = false;   // two kernels per iteration (x/p update folded into SpMV)
  bool defer = false;   // mode 3: x updated once per 4 bodies from 4 p buffers
  bool fdefer = false;  // mode 4: p update folded into the SpMV, x deferred as mode 3
  bool recompute = false;  // mode 6 (with defer): Ap formed again in update_r's walk, not stored
  bool coop = false;    // mode 5: persistent body, one launch per chunk (cgx_coop.hip)
  int coop_r = 0;       // its rows per thread
  int coop_stall = -1;  // tests: a launch's body whose p.Ap partial workgroup 0
                        // withholds ($CGX_COOP_INJECT_STALL; -1 none)
  void *coop_ws = nullptr;  // cgx::CoopWs
  bool coop_stream = false;  // form 2: the matrix read every body (k_cg_coop_st)
  int coop_stream_want = -1; // $CGX_COOP_STREAM: -1 auto, 0 never, 1 always
  void *coop_trace = nullptr;  // $CGX_COOP_TRACE: phase stamps (cgx_cg_coop_trace)
  long long coop_ticks = 0; // wall-clock ticks before an exchange spin gives up
  bool altdir = false;  // alternate the kernels' sweep directions (Infinity-Cache reuse)
  void *pk[3] = {nullptr, nullptr, nullptr};  // p buffers 1..3 of mode 3 (n + n_ghost)
  void *st = nullptr;   // cgx::CgScalars<T>
  void *ws = nullptr;   // cgx::RedWs<T>
  const void *b = nullptr;
  void *x = nullptr;
  int slot = 0;
  bool begun = false;
  int poll_every = 32;
  bool use_graph = true;
  // captured iterations, keyed by (first slot, bodies): full chunks of
  // `poll_every` from any slot (built on first use) and the chunks
  // cgx_cg_prepare built ahead of a run; all captured for x = graph_x
  std::map<std::pair<int, int64_t>, hipGraphExec_t> graphs;
  void *graph_x = nullptr;
  // cgx_cg_run's two poll events, created once (an event create and destroy
  // per run sat inside every caller's timed region)
  hipEvent_t run_ev[2] = {nullptr, nullptr};
  // kernel timing
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<std::pair<int, size_t>> ev_pending;  // (kernel id, event index)
  double t_ms[4] = {0, 0, 0, 0};
  int64_t t_calls[4] = {0, 0, 0, 0};
  double t_exec_ms[4] = {0, 0, 0, 0};      // the dispatch's own event pairs (g_exec)
  int64_t t_exec_calls[4] = {0, 0, 0, 0};
};

namespace cgx {
// setup phase timing (cgx_csr::setup_ms): the wall time since the last mark
// is charged to `phase` while cgx_csr_create(_dist) runs
inline void setup_begin(cgx_csr *A) {
  A->setup_open = true;
  A->setup_last = std::chrono::steady_clock::now();
}
inline void setup_mark(cgx_csr *A, int phase) {
  if (!A->setup_open) return;
  const auto now = std::chrono::steady_clock::now();
  A->setup_ms[phase] += std::chrono::duration<double, std::milli>(now - A->setup_last).count();
  A->setup_last = now;
}
// reference counts (cgx_abi.cpp): retain on a handle made from the object,
// release when that handle (or the owner) lets go; the last release frees
void ctx_retain(cgx_ctx *ctx);
void ctx_release(cgx_ctx *ctx);
void csr_retain(cgx_csr *A);
void csr_release(cgx_csr *A);
// cgx_dist.cpp
int dist_halo_exchange(cgx_csr *A, void *d_vec_ext, hipStream_t s);
// Overlapped form: pack on s, exchange on the context's comm stream (RCCL,
// *async = true: s must wait on A->ev_halo before reading the ghosts) or
// synchronously (host transport).
int dist_halo_post(cgx_csr *A, void *d_vec_ext, hipStream_t s, bool *async);
int dist_allreduce_scalar(cgx_ctx *ctx, void *d_val, int dtype, int count, hipStream_t s);
int dist_destroy_halo(cgx_csr *A);
int dist_comm_destroy(cgx_ctx *ctx);
// setup collective on host buffers over the setup transport (RCCL / host)
int comm_allgather(cgx_ctx *ctx, const void *mine, size_t bytes, void *all);
// cgx_peer.hip: the peer transport's per-iteration steps (enqueue on s)
template <typename T> int peer_push(cgx_csr *A, const T *v_ext, CgScalars<T> *st, int slot,
                                    hipStream_t s);
template <typename T> int peer_wait(cgx_csr *A, T *v_ext, CgScalars<T> *st, int slot,
                                    hipStream_t s);
// the one-waiter form's wait: one workgroup polls the push flags (no copy;
// the boundary launch behind it reads the landing buffer with P.nopoll)
template <typename T> int peer_wait_one(cgx_csr *A, CgScalars<T> *st, int slot, hipStream_t s);
// *dst = sum over ranks of (sum of part[0..np)), identical bits on every rank
// which: 0 setup / init, 1 and 2 the body's p.Ap and r.r (k_peer_allreduce)
template <typename T> int peer_allreduce(cgx_csr *A, const T *part, int np, T *dst,
                                         CgScalars<T> *st, int slot, hipStream_t s, int which);
int peer_destroy(cgx_csr *A);
}  // namespace cgx
