// cgx_coop.hip — persistent CG body for cache-resident problems (mode 5).
//
// One launch runs up to m loop bodies of CG::solve (src/CG.hpp:359-436): the
// SpMV (VectorOperations.hpp:438-466), both dots (:287-309) and the three
// updates (CG.hpp:380-418) of every body, with the stop rule (CG.hpp:396-404,
// 436) applied after each. Where a three-launch body of a small problem is
// mostly kernel boundaries (128^2: ~9.6 us per body, of which the work is a
// fraction), this body pays two grid-wide exchanges instead.
//
// Layout (the register form): workgroup g of 1,024 threads owns rows
// [1024 g, 1024 (g + 1)), one per thread. Each thread keeps its row's x, r,
// p and its first 7 entries (columns and values) in registers for the whole
// launch; the rest of a longer row is read from the CSR arrays. (Round 3's
// 256- and 512-thread shapes and its tagged p / r hand-off measured no faster
// and were removed in round 4.)
//
// Per body k (two exchanges, DESIGN.md §5 "persistent body"):
//   1. SpMV on p_k. p_k[j] of a gathered column is formed where it is read,
//      p_k[j] = r_k[j] + beta_{k-1} p_{k-1}[j], from r_k and p_{k-1} as their
//      owners stored them (the same rounded operations the owner applies to
//      its own p: every workgroup gets the identical p_k[j]); the launch's
//      first body reads p_k itself. Row sums in ascending entry order from 0,
//      products rounded before the add: Ap is bit-identical to the
//      reference's per-row loop.
//   2. p.Ap: workgroup partials exchanged (A), summed in workgroup order by
//      every workgroup (identical everywhere); alpha.
//   3. x += alpha p, r -= alpha Ap in registers; r stored for the gatherers.
//   4. r.r: exchange B; beta; stop rule.
// p_k (own rows) is stored into buffer k mod 2 (cgx_cg::p / p2) for the next
// body's gathers; at the end of the launch p_{k+1}, x and r are left in the
// standard buffers (cgx_cg::p, x, r) and the scalar ring as the three-kernel
// body leaves them, so any mode can continue the solve.
//
// Exchanges follow the MI355X guide's placement-independent hand-off (§6
// Guideline 16, R1/R2): the handed-off vector entries are stored write-through
// (agent-scope relaxed atomic stores = sc1) and every storing wave drains
// them (s_waitcnt vmcnt(0)) before its workgroup publishes; a partial is two
// 8-byte {tag, half} granules written by one atomic store each (the data is
// the flag); one wave per workgroup sweeps all granules until every tag is
// this body's; every load of handed-off data is an agent-scope atomic load.
// No workgroup index, dispatch order or XCD placement enters the protocol.
// The grid is one workgroup per CU at most (G <= min(kCoopMaxG, CUs)), and
// cg_coop refuses a launch the occupancy API does not place whole (every
// workgroup must be resident at once); every spin is bounded by the wall
// clock, and a
// workgroup that gives up raises CoopWs::tmo so the others leave too
// (CgScalars::stopped = 4).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "cgx_internal.h"

namespace cgx {
namespace {

__device__ __forceinline__ double ld_ag(const double *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ag(double *p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_ag(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ag(unsigned long long *p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave sum in a fixed order on DPP lane moves (no LDS round trips): quad
// butterflies, the 8- and 16-lane mirrors, then rows 0+1 and 2+3 and their
// sum into lane 63 (row_bcast15 / row_bcast31). Lanes the moves do not
// reach add 0.0. The result is read from lane 63.
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ double dpp(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, RM, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, RM, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp<0xB1>(v);         // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);         // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);        // row_half_mirror: the other quad of 8
  v += dpp<0x140>(v);        // row_mirror: the other 8 of 16
  v += dpp<0x142, 0xa>(v);   // row_bcast15: rows 1, 3 add rows 0, 2
  v += dpp<0x143, 0xc>(v);   // row_bcast31: rows 2, 3 add lane 31
  return __shfl(v, 63, 64);  // every lane
}

// fixed-order workgroup sum of NT threads (every thread gets it); lds: NT / 64
// slots used by no other block_sum until the next __syncthreads after this one
template <int NT>
__device__ __forceinline__ double block_sum(double v, double *lds) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = lds[0];
#pragma unroll
  for (int w = 1; w < NT / 64; ++w) s += lds[w];
  return s;
}

// Publish this workgroup's partial for exchange `tag` (thread 0), after every
// wave drained its handed-off stores.
__device__ __forceinline__ void publish(unsigned long long *gran, double part, unsigned tag) {
  if (threadIdx.x == 0) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(part);
    const unsigned long long hi = (unsigned long long)tag << 32;
    st_ag(gran + 2 * blockIdx.x, hi | (u & 0xffffffffull));
    st_ag(gran + 2 * blockIdx.x + 1, hi | (u >> 32));
  }
}

// Every workgroup: wave 0 sweeps all G partials until every tag is `tag`,
// sums them in workgroup order (lane l: partials l, l + 64, l + 128, l + 192;
// then the wave's shuffle tree), broadcasts through LDS. false: a spin gave up.
__device__ __forceinline__ bool collect(const unsigned long long *gran, unsigned tag,
                                        long long ticks, unsigned *tmo, double *res_lds,
                                        int *ok_lds, int nap) {
  const int G = gridDim.x;
  static_assert(kCoopMaxG <= 256, "collect reads four partials per lane");
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    double v = 0.0;
    bool ok = true;
    const long long t0 = wall_clock64();
    // lane l holds partials l + 64 q (q < 4), read in one pass
    unsigned long long a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
    for (;;) {
      bool got = true;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (l + 64 * q < G) {
          a[q] = ld_ag(gran + 2 * (l + 64 * q));
          b[q] = ld_ag(gran + 2 * (l + 64 * q) + 1);
          got = got && (unsigned)(a[q] >> 32) == tag && (unsigned)(b[q] >> 32) == tag;
        }
      }
      if (__all(got)) break;
      const bool late = wall_clock64() - t0 > ticks ||
                        __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__any(late)) {
        ok = false;
        break;
      }
      for (int z = 0; z < nap; ++z) __builtin_amdgcn_s_sleep(1);
    }
    if (ok) {
      if (l < G) v = __longlong_as_double((long long)((a[0] & 0xffffffffull) | ((b[0] & 0xffffffffull) << 32)));
#pragma unroll
      for (int q = 1; q < 4; ++q)
        if (l + 64 * q < G)
          v += __longlong_as_double((long long)((a[q] & 0xffffffffull) | ((b[q] & 0xffffffffull) << 32)));
    }
    v = wave_sum(v);
    if (l == 0) {
      *res_lds = v;
      *ok_lds = ok;
      if (!ok) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return *ok_lds != 0;
}

__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Diagnostics ($CGX_COOP_TRACE, cgx_cg_coop_trace): thread 0 of every
// workgroup stamps the wall clock at the phases of bodies 8-15 of a launch
#define CGX_COOP_TR(ph)                                                                  \
  if (trace && i >= 8 && i < 16 && t == 0)                                               \
    trace[((size_t)blockIdx.x * 8 + (i - 8)) * 8 + (ph)] = wall_clock64();

// Entries per row held in registers: kCoopK, 7 in the 1,024-thread form
// (its 128-VGPR budget: 8 spilled 44 bytes per lane; a 7-point row fits)
template <int NT> constexpr int coop_kc() { return NT == 1024 ? 7 : kCoopK; }

// Shared prologue: this thread's rows, their first KC entries, x, r, p.
#define CGX_COOP_PROLOGUE                                                        \
  constexpr int KC = coop_kc<NT>();                                              \
  __shared__ double red[2][NT / 64]; /* [exchange A / B] */                      \
  __shared__ double res;                                                         \
  __shared__ int okf;                                                            \
  if (!st->active[slot0]) return; /* the same word for every workgroup */        \
  const int t = threadIdx.x;                                                     \
  double rxr = st->rxr[slot0];                                                   \
  const double tol = st->tol;                                                    \
  const long long cap = st->cap;                                                 \
  long long bodies = st->bodies;                                                 \
  int64_t row[R], rb[R];                                                         \
  int cnt[R];                                                                    \
  int cc[R][KC];                                                             \
  double cv[R][KC];                                                          \
  double xr[R], rv[R], pv[R];                                                    \
  _Pragma("unroll") for (int u = 0; u < R; ++u) {                                \
    row[u] = ((int64_t)blockIdx.x * R + u) * NT + t;                             \
    const bool ok = row[u] < n;                                                  \
    rb[u] = ok ? rowptr[row[u]] : 0;                                             \
    cnt[u] = ok ? rowptr[row[u] + 1] - (int)rb[u] : 0;                           \
    _Pragma("unroll") for (int k = 0; k < KC; ++k) {                         \
      cc[u][k] = k < cnt[u] ? col[rb[u] + k] : 0;                                \
      cv[u][k] = k < cnt[u] ? val[rb[u] + k] : 0.0;                              \
    }                                                                            \
    xr[u] = ok ? x[row[u]] : 0.0;                                                \
    rv[u] = ok ? r[row[u]] : 0.0;                                                \
    pv[u] = ok ? p0[row[u]] : 0.0;                                               \
  }

// The body's record and stop rule, as k_update_xp (CG.hpp:396-404, 436);
// returns cont
__device__ __forceinline__ bool coop_record(CgScalars<double> *st, int s, double pAp, double rr,
                                            double alpha, double rxr, double tol,
                                            long long bodies, long long cap) {
  const bool cond = isnan(rxr) || sqrt(rxr) <= tol;
  const bool cont = !cond && bodies < cap;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // read by the host after the launch
    st->pAp[s] = pAp;
    st->rr[s] = rr;
    st->alpha[s] = alpha;
    st->rxr[(s + 1) & 3] = rr;
    st->bodies = bodies;
    st->stopped = cond ? 1 : (cont ? 0 : 2);
    st->active[(s + 1) & 3] = cont ? 1 : 0;
    if (!cont)
      for (int q = 0; q < 4; ++q) st->active[q] = 0;
  }
  return cont;
}

__device__ __forceinline__ void coop_gave_up(CgScalars<double> *st) {
  if (threadIdx.x == 0) {  // a spin gave up (okf == 0 in every workgroup that gets here)
    st->stopped = 4;
    for (int q = 0; q < 4; ++q) st->active[q] = 0;
  }
}

// The register form: r and p_k stored with agent-scope
// stores (sc1) into r and p0 / p1, every storing wave drained before its
// workgroup publishes; the gathers of a body run after both exchanges.
template <int R, int NT>
__global__ __launch_bounds__(NT, 1) void k_cg_coop_wt(
    int64_t n, const int *__restrict__ rowptr, const int *__restrict__ col,
    const double *__restrict__ val, double *__restrict__ x, double *r, double *p0, double *p1,
    CgScalars<double> *st, int slot0, int m, CoopWs *cw, long long ticks,
    unsigned long long *trace, int nap, int stall) {
  CGX_COOP_PROLOGUE
  double beta = 0.0;
  for (int i = 0; i < m; ++i) {
    const int s = (slot0 + i) & 3;
    const unsigned tag = (unsigned)i + 1u;
    CGX_COOP_TR(0)
    double *pcur = (i & 1) ? p1 : p0;         // p_k of this body (own rows stored here)
    const double *pprev = (i & 1) ? p0 : p1;  // p_{k-1}: the previous body's buffer
    double q[R];
    if (i == 0) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < KC; ++k)
          if (k < cnt[u]) acc += cv[u][k] * ld_ag(p0 + cc[u][k]);
        for (int k = KC; k < cnt[u]; ++k) acc += val[rb[u] + k] * ld_ag(p0 + col[rb[u] + k]);
        q[u] = acc;
      }
    } else {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        pv[u] = rv[u] + beta * pv[u];  // p = r + beta p (CG.hpp:418), own rows
        if (row[u] < n) st_ag(pcur + row[u], pv[u]);
      }
#pragma unroll
      for (int u = 0; u < R; ++u) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < KC; ++k)
          if (k < cnt[u]) {
            const int j = cc[u][k];
            acc += cv[u][k] * (ld_ag(r + j) + beta * ld_ag(pprev + j));
          }
        for (int k = KC; k < cnt[u]; ++k) {
          const int j = col[rb[u] + k];
          acc += val[rb[u] + k] * (ld_ag(r + j) + beta * ld_ag(pprev + j));
        }
        q[u] = acc;
      }
    }
    CGX_COOP_TR(1)
    // p.Ap (CG.hpp:374-379)
    double part = 0.0;
#pragma unroll
    for (int u = 0; u < R; ++u) part += pv[u] * q[u];
    drain();  // this wave's p stores are out before the workgroup publishes
    part = block_sum<NT>(part, red[0]);
    CGX_COOP_TR(2)
    // fault injection (tests): workgroup 0 withholds body `stall`'s p.Ap
    // partial, so every other workgroup's bounded spin gives up
    if (!(i == stall && blockIdx.x == 0)) publish(cw->ga, part, tag);
    if (!collect(cw->ga, tag, ticks, &cw->tmo, &res, &okf, nap)) break;
    CGX_COOP_TR(3)
    const double pAp = res;
    const double alpha = rxr / pAp;
    // x += alpha p; r -= alpha Ap; r.r   (CG.hpp:381-393, 406-407)
    part = 0.0;
#pragma unroll
    for (int u = 0; u < R; ++u) {
      xr[u] = xr[u] + alpha * pv[u];
      rv[u] = rv[u] - alpha * q[u];
      if (row[u] < n) st_ag(r + row[u], rv[u]);
      part += rv[u] * rv[u];
    }
    drain();
    part = block_sum<NT>(part, red[1]);
    CGX_COOP_TR(4)
    publish(cw->gb, part, tag);
    CGX_COOP_TR(5)
    if (!collect(cw->gb, tag, ticks, &cw->tmo, &res, &okf, nap)) break;
    CGX_COOP_TR(6)
    const double rr = res;
    ++bodies;
    const bool cont = coop_record(st, s, pAp, rr, alpha, rxr, tol, bodies, cap);
    beta = rr / rxr;
    rxr = rr;
    if (!cont || i == m - 1) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        if (row[u] < n) {
          p0[row[u]] = rv[u] + beta * pv[u];  // p_{k+1}, and x, in the standard buffers
          x[row[u]] = xr[u];
        }
      }
      return;
    }
  }
  coop_gave_up(st);
}

// Form 2 (streamed, problems past the register forms: more rows than
// kCoopMaxG x 1,024, or rows longer than 7 entries): 1,024 threads, R rows
// per thread, r of the rows in registers, x and p in LDS (the 128-VGPR
// budget of 16 waves per CU), the matrix read every body. Chunk u of
// workgroup g is rows [(g R + u) 1024, + 1024), whose entries are
// contiguous: the workgroup's threads load them coalesced (entry e by thread
// e mod 1024, four per pass in flight), form each product
// val[e] * p_k[col[e]] (p_k[j] = r_k[j] + beta p_{k-1}[j], as the register form) and
// stage it in LDS; thread t then sums its row's products in ascending entry
// order from 0 — the reference's row loop, bit for bit. A chunk of more than
// coop_stage<R>() entries (long rows) is summed by its row threads from the
// CSR arrays instead. Exchanges, updates and the record as the register form.
constexpr int kCoopStP = 5;  // streamed form: entries per thread of a one-pass chunk
template <int R> constexpr int coop_stage() { return (160 * 1024 - R * 1024 * 16 - 1024) / 8; }
template <int R>
__global__ __launch_bounds__(1024, 1) void k_cg_coop_st(
    int64_t n, const int *__restrict__ rowptr, const int *__restrict__ col,
    const double *__restrict__ val, double *__restrict__ x, double *r, double *p0, double *p1,
    CgScalars<double> *st, int slot0, int m, CoopWs *cw, long long ticks,
    unsigned long long *trace, int nap, int stall) {
  constexpr int NT = 1024, C = coop_stage<R>();
  __shared__ double stage[C];
  __shared__ double xs[R][NT];  // this workgroup's x
  __shared__ double ps[R][NT];  // and p (p_k of its rows)
  __shared__ double red[2][NT / 64];
  __shared__ double res;
  __shared__ int okf;
  if (!st->active[slot0]) return;
  const int t = threadIdx.x;
  double rxr = st->rxr[slot0];
  const double tol = st->tol;
  const long long cap = st->cap;
  long long bodies = st->bodies;
  // row u of this thread: (g R + u) 1024 + tq; tq is re-made opaque every
  // body so the compiler re-forms the row addresses instead of holding R of
  // them (64-bit) across the body loop
  int tq = t, gq = blockIdx.x;
  auto rowid = [&](int u) { return ((int64_t)gq * R + u) * NT + tq; };
  // per row: its first entry's offset in its chunk << 16 | its entry count
  // (chunks of at most C entries; others take the CSR path)
  unsigned oc[R];
  double rv[R];
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const int64_t f = ((int64_t)blockIdx.x * R + u) * NT, w = rowid(u);
    const bool ok = w < n;
    const int b0 = f < n ? rowptr[f] : 0;
    const int rb = ok ? rowptr[w] : 0;
    oc[u] = ok ? ((unsigned)(rb - b0) << 16) | (unsigned)(rowptr[w + 1] - rb) : 0u;
    xs[u][t] = ok ? x[w] : 0.0;
    rv[u] = ok ? r[w] : 0.0;
    ps[u][t] = ok ? p0[w] : 0.0;
  }
  double beta = 0.0;
  for (int i = 0; i < m; ++i) {
    const int s = (slot0 + i) & 3;
    const unsigned tag = (unsigned)i + 1u;
    asm volatile("" : "+v"(tq), "+s"(gq));
    CGX_COOP_TR(0)
    double *pcur = (i & 1) ? p1 : p0;
    const double *pprev = (i & 1) ? p0 : p1;
    if (i > 0) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const double pu = rv[u] + beta * ps[u][t];  // p = r + beta p (CG.hpp:418), own rows
        ps[u][t] = pu;
        if (rowid(u) < n) st_ag(pcur + rowid(u), pu);
      }
    }
    // p_k[j] as every reader forms it, r_k[j] + beta p_{k-1}[j]; the launch's
    // first body reads p_k itself (p_k[j] + 0 p_k[j]: the same value for
    // finite p) — no branch between the gathers of a pass
    const double *ga = i == 0 ? p0 : r, *gb = i == 0 ? p0 : pprev;
    const double bk = i == 0 ? 0.0 : beta;
    auto pk = [&](int j) { return ld_ag(ga + j) + bk * ld_ag(gb + j); };
    double q[R];
    // chunk u's entries [base, base + E)
    auto span = [&](int u, int &base, int &E) {
      const int64_t f = ((int64_t)gq * R + u) * NT;
      base = f < n ? rowptr[f] : 0;
      E = f < n ? rowptr[f + NT < n ? f + NT : n] - base : 0;
    };
    // a chunk of at most PW entries is one pass of P per thread, its col/val
    // loaded while the previous chunk's gathers are in flight
    constexpr int P = kCoopStP, PW = P * NT < C ? P * NT : C;
    int jj[P];
    double vv[P];
    auto load = [&](int base, int E) {
#pragma unroll
      for (int z = 0; z < P; ++z) {  // clamped: no branch before the loads
        const int e = min(z * NT + t, E - 1);
        jj[z] = col[base + e];
        vv[z] = val[base + e];
      }
    };
    int bn, en;
    span(0, bn, en);
    if (en > 0 && en <= PW) load(bn, en);
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int base = bn, E = en;
      double acc = 0.0;
      double pr[P];
      // jj / vv hold this chunk only when load() ran for it (0 < E <= PW); an
      // empty chunk (past n) must not gather through stale indices
      if (E > 0 && E <= PW) {
#pragma unroll
        for (int z = 0; z < P; ++z) pr[z] = vv[z] * pk(jj[z]);
      }
      if (u + 1 < R) {
        span(u + 1, bn, en);
        if (en > 0 && en <= PW) load(bn, en);
      }
      if (E <= C) {
        if (E <= PW) {
#pragma unroll
          for (int z = 0; z < P; ++z)
            if (z * NT + t < E) stage[z * NT + t] = pr[z];
        } else {
#pragma unroll 1
          for (int s0 = 0; s0 < E; s0 += 4 * NT) {
            int j4[4];
            double v4[4], p4[4];
#pragma unroll
            for (int z = 0; z < 4; ++z) {
              const int e = min(s0 + z * NT + t, E - 1);
              j4[z] = col[base + e];
              v4[z] = val[base + e];
            }
#pragma unroll
            for (int z = 0; z < 4; ++z) p4[z] = v4[z] * pk(j4[z]);
#pragma unroll
            for (int z = 0; z < 4; ++z) {
              const int e = s0 + z * NT + t;
              if (e < E) stage[e] = p4[z];
            }
          }
        }
        __syncthreads();
        const int o = (int)(oc[u] >> 16), c = (int)(oc[u] & 0xffffu);
        for (int k = 0; k < c; ++k) acc += stage[o + k];
        __syncthreads();  // the next chunk overwrites the stage
      } else if (rowid(u) < n) {  // long rows in the chunk: every row from the CSR arrays
        const int rb = rowptr[rowid(u)], re = rowptr[rowid(u) + 1];
#pragma unroll 1
        for (int k = rb; k < re; ++k) acc += val[k] * pk(col[k]);
      }
      q[u] = acc;
    }
    CGX_COOP_TR(1)
    // p.Ap (CG.hpp:374-379)
    double part = 0.0;
#pragma unroll
    for (int u = 0; u < R; ++u) part += ps[u][t] * q[u];
    drain();  // this wave's p stores are out before the workgroup publishes
    part = block_sum<NT>(part, red[0]);
    CGX_COOP_TR(2)
    if (!(i == stall && blockIdx.x == 0)) publish(cw->ga, part, tag);
    if (!collect(cw->ga, tag, ticks, &cw->tmo, &res, &okf, nap)) break;
    CGX_COOP_TR(3)
    const double pAp = res;
    const double alpha = rxr / pAp;
    // x += alpha p; r -= alpha Ap; r.r   (CG.hpp:381-393, 406-407)
    part = 0.0;
#pragma unroll
    for (int u = 0; u < R; ++u) {
      xs[u][t] = xs[u][t] + alpha * ps[u][t];
      rv[u] = rv[u] - alpha * q[u];
      if (rowid(u) < n) st_ag(r + rowid(u), rv[u]);
      part += rv[u] * rv[u];
    }
    drain();
    part = block_sum<NT>(part, red[1]);
    CGX_COOP_TR(4)
    publish(cw->gb, part, tag);
    CGX_COOP_TR(5)
    if (!collect(cw->gb, tag, ticks, &cw->tmo, &res, &okf, nap)) break;
    CGX_COOP_TR(6)
    const double rr = res;
    ++bodies;
    const bool cont = coop_record(st, s, pAp, rr, alpha, rxr, tol, bodies, cap);
    beta = rr / rxr;
    rxr = rr;
    if (!cont || i == m - 1) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        if (rowid(u) < n) {
          p0[rowid(u)] = rv[u] + beta * ps[u][t];  // p_{k+1}, and x, in the standard buffers
          x[rowid(u)] = xs[u][t];
        }
      }
      return;
    }
  }
  coop_gave_up(st);
}

}  // namespace

int coop_rows_per_thread(int64_t n, int max_g) {
  // one row per thread of 1,024 (128 VGPRs at 16 waves per CU)
  return (n + 1023) / 1024 <= std::min(max_g, kCoopMaxG) ? 1 : 0;
}

int coop_stream_rows(int64_t n, int want, int max_g) {
  for (int R = 1; R <= kCoopStreamMaxR; ++R) {
    if (want > 0 && R != want) continue;
    if ((n + 1024LL * R - 1) / (1024LL * R) <= std::min(max_g, kCoopMaxG)) return R;
  }
  return 0;
}

// every workgroup of a G-workgroup launch of fn resident at once: the
// occupancy API's workgroups per CU x the device's CUs (cached per kernel)
static bool coop_resident(const void *fn, int NT, int G) {
  static std::mutex mu;
  static std::map<std::pair<const void *, int>, int> cap;
  std::lock_guard<std::mutex> lk(mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  const auto key = std::make_pair(fn, dev);
  auto it = cap.find(key);
  if (it == cap.end()) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NT, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return false;
    it = cap.emplace(key, per_cu * cus).first;
  }
  return G <= it->second;
}

hipError_t cg_coop(int64_t n, int R, bool streamed, const int *rowptr, const int *col,
                   const double *val, double *x, double *r, double *p0, double *p1,
                   CgScalars<double> *st, int slot0, int m, CoopWs *cw, long long ticks,
                   unsigned long long *trace, int stall, hipStream_t s) {
  constexpr int NT = 1024, nap = 1;  // one s_sleep(1) per exchange poll
  const int G = (int)((n + (int64_t)NT * R - 1) / ((int64_t)NT * R));
  if (G < 1 || G > kCoopMaxG || m < 1) return hipErrorInvalidValue;
  if (streamed ? (R < 1 || R > kCoopStreamMaxR) : R != 1) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(cw, 0, sizeof(CoopWs), s);
  if (e != hipSuccess) return e;
  const void *fn = nullptr;
  if (!streamed) {
    fn = (const void *)k_cg_coop_wt<1, NT>;
  } else {
    switch (R) {
      case 1: fn = (const void *)k_cg_coop_st<1>; break;
      case 2: fn = (const void *)k_cg_coop_st<2>; break;
      case 3: fn = (const void *)k_cg_coop_st<3>; break;
      case 4: fn = (const void *)k_cg_coop_st<4>; break;
      case 5: fn = (const void *)k_cg_coop_st<5>; break;
      case 6: fn = (const void *)k_cg_coop_st<6>; break;
      case 7: fn = (const void *)k_cg_coop_st<7>; break;
      case 8: fn = (const void *)k_cg_coop_st<8>; break;
      default: return hipErrorInvalidValue;
    }
  }
  // (the occupancy check first: a refusal then names the cause before the
  // runtime's own)
  if (!coop_resident(fn, NT, G)) return hipErrorCooperativeLaunchTooLarge;
  // A cooperative launch (verdict r5): the runtime guarantees that all G
  // workgroups are resident together, which the two grid-wide exchanges per
  // body need; a plain launch only had the occupancy estimate above, and any
  // other work on the device could hold a CU a late workgroup needed. Mode 5
  // runs outside the iteration graphs (graph_ok), so capture is not needed.
  void *args[] = {(void *)&n,  (void *)&rowptr, (void *)&col,   (void *)&val,
                  (void *)&x,  (void *)&r,      (void *)&p0,    (void *)&p1,
                  (void *)&st, (void *)&slot0,  (void *)&m,     (void *)&cw,
                  (void *)&ticks, (void *)&trace, (void *)&nap, (void *)&stall};
  return hipLaunchCooperativeKernel(fn, dim3(G), dim3(NT), args, 0, s);
}

}  // namespace cgx
