// cgx_coop.hip — persistent CG body for cache-resident problems (mode 5).
//
// One launch runs up to m loop bodies of CG::solve (src/CG.hpp:359-436): the
// SpMV (VectorOperations.hpp:438-466), both dots (:287-309) and the three
// updates (CG.hpp:380-418) of every body, with the stop rule (CG.hpp:396-404,
// 436) applied after each. Where a three-launch body of a small problem is
// mostly kernel boundaries (128^2: ~9.6 us per body, of which the work is a
// fraction), this body pays two grid-wide exchanges instead.
//
// Layout: workgroup g owns rows [g 256 R, (g + 1) 256 R), thread t rows
// g 256 R + 256 u + t (u < R). Each thread keeps its rows' x, r, p and the
// first kCoopK entries of each row (columns and values) in registers for the
// whole launch; the rest of a longer row is read from the CSR arrays.
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
// The grid is one workgroup per CU at most (kCoopMaxG <= CUs / 2, so every
// workgroup is resident), every spin is bounded by the wall clock, and a
// workgroup that gives up raises CoopWs::tmo so the others leave too
// (CgScalars::stopped = 4).
#include <hip/hip_runtime.h>

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

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;  // lane 0
}

// fixed-order workgroup sum, valid in thread 0
__device__ __forceinline__ double block_sum(double v, double *lds) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  const double s = ((lds[0] + lds[1]) + lds[2]) + lds[3];
  __syncthreads();
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
// sums them in workgroup order (lane l: partials l, l + 64; then the wave's
// shuffle tree), broadcasts through LDS. false: a spin gave up.
__device__ __forceinline__ bool collect(const unsigned long long *gran, unsigned tag,
                                        long long ticks, unsigned *tmo, double *res_lds,
                                        int *ok_lds) {
  const int G = gridDim.x;
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    double v = 0.0;
    bool ok = true;
    const long long t0 = wall_clock64();
    for (int c = 0; c * 64 < G && ok; ++c) {
      const int w = l + 64 * c;
      const bool mine = w < G;
      unsigned long long a = 0, b = 0;
      for (;;) {
        bool got = true;
        if (mine) {
          a = ld_ag(gran + 2 * w);
          b = ld_ag(gran + 2 * w + 1);
          got = (unsigned)(a >> 32) == tag && (unsigned)(b >> 32) == tag;
        }
        if (__all(got)) break;
        const bool late = wall_clock64() - t0 > ticks ||
                          __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__any(late)) {
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (ok && mine)
        v += __longlong_as_double((long long)((a & 0xffffffffull) | ((b & 0xffffffffull) << 32)));
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

template <int R>
__global__ __launch_bounds__(kBlock, 1) void k_cg_coop(
    int64_t n, const int *__restrict__ rowptr, const int *__restrict__ col,
    const double *__restrict__ val, double *__restrict__ x, double *r, double *p0, double *p1,
    CgScalars<double> *st, int slot0, int m, CoopWs *cw, long long ticks) {
  __shared__ double red[4];
  __shared__ double res;
  __shared__ int okf;
  if (!st->active[slot0]) return;  // the same word for every workgroup
  const int t = threadIdx.x;
  double rxr = st->rxr[slot0];
  const double tol = st->tol;
  const long long cap = st->cap;
  long long bodies = st->bodies;

  int64_t row[R], rb[R];
  int cnt[R];
  int cc[R][kCoopK];
  double cv[R][kCoopK];
  double xr[R], rv[R], pv[R];
#pragma unroll
  for (int u = 0; u < R; ++u) {
    row[u] = ((int64_t)blockIdx.x * R + u) * kBlock + t;
    const bool ok = row[u] < n;
    rb[u] = ok ? rowptr[row[u]] : 0;
    cnt[u] = ok ? rowptr[row[u] + 1] - (int)rb[u] : 0;
#pragma unroll
    for (int k = 0; k < kCoopK; ++k) {
      cc[u][k] = k < cnt[u] ? col[rb[u] + k] : 0;
      cv[u][k] = k < cnt[u] ? val[rb[u] + k] : 0.0;
    }
    xr[u] = ok ? x[row[u]] : 0.0;
    rv[u] = ok ? r[row[u]] : 0.0;
    pv[u] = ok ? p0[row[u]] : 0.0;
  }

  double beta = 0.0;
  for (int i = 0; i < m; ++i) {
    const int s = (slot0 + i) & 3;
    const unsigned tag = (unsigned)i + 1u;
    double *pcur = (i & 1) ? p1 : p0;         // p_k of this body (own rows stored here)
    const double *pprev = (i & 1) ? p0 : p1;  // p_{k-1}: the previous body's buffer
    double q[R];
    if (i == 0) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < kCoopK; ++k)
          if (k < cnt[u]) acc += cv[u][k] * ld_ag(p0 + cc[u][k]);
        for (int k = kCoopK; k < cnt[u]; ++k) acc += val[rb[u] + k] * ld_ag(p0 + col[rb[u] + k]);
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
        for (int k = 0; k < kCoopK; ++k)
          if (k < cnt[u]) {
            const int j = cc[u][k];
            acc += cv[u][k] * (ld_ag(r + j) + beta * ld_ag(pprev + j));
          }
        for (int k = kCoopK; k < cnt[u]; ++k) {
          const int j = col[rb[u] + k];
          acc += val[rb[u] + k] * (ld_ag(r + j) + beta * ld_ag(pprev + j));
        }
        q[u] = acc;
      }
    }
    // p.Ap (CG.hpp:374-379)
    double part = 0.0;
#pragma unroll
    for (int u = 0; u < R; ++u) part += pv[u] * q[u];
    drain();  // this wave's p stores are out before the workgroup publishes
    part = block_sum(part, red);
    publish(cw->ga, part, tag);
    if (!collect(cw->ga, tag, ticks, &cw->tmo, &res, &okf)) break;
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
    part = block_sum(part, red);
    publish(cw->gb, part, tag);
    if (!collect(cw->gb, tag, ticks, &cw->tmo, &res, &okf)) break;
    const double rr = res;
    // stop rule, as k_update_xp (CG.hpp:396-404, 436)
    ++bodies;
    const bool cond = isnan(rxr) || sqrt(rxr) <= tol;
    const bool cont = !cond && bodies < cap;
    beta = rr / rxr;
    if (blockIdx.x == 0 && t == 0) {  // the record (read by the host after the launch)
      st->pAp[s] = pAp;
      st->rr[s] = rr;
      st->alpha[s] = alpha;
      st->rxr[(s + 1) & 3] = rr;
      st->bodies = bodies;
      st->stopped = cond ? 1 : (cont ? 0 : 2);
      st->active[(s + 1) & 3] = cont ? 1 : 0;
      if (!cont)
        for (int q2 = 0; q2 < 4; ++q2) st->active[q2] = 0;
    }
    rxr = rr;
    if (!cont || i == m - 1) {
      // p_{k+1} = r + beta p, and x, into the standard buffers
#pragma unroll
      for (int u = 0; u < R; ++u) {
        if (row[u] < n) {
          p0[row[u]] = rv[u] + beta * pv[u];
          x[row[u]] = xr[u];
        }
      }
      return;
    }
  }
  // a spin gave up (okf == 0 in every workgroup that reaches here)
  if (t == 0) {
    st->stopped = 4;
    for (int q2 = 0; q2 < 4; ++q2) st->active[q2] = 0;
  }
}

}  // namespace

int coop_rows_per_thread(int64_t n, int want) {
  static const int opts[] = {1, 2, 4};
  for (int R : opts) {
    if (want > 0 && R != want) continue;
    if ((n + (int64_t)kBlock * R - 1) / ((int64_t)kBlock * R) <= kCoopMaxG) return R;
  }
  return 0;
}

hipError_t cg_coop(int64_t n, int R, const int *rowptr, const int *col, const double *val,
                   double *x, double *r, double *p0, double *p1, CgScalars<double> *st, int slot0,
                   int m, CoopWs *cw, long long ticks, hipStream_t s) {
  const int G = (int)((n + (int64_t)kBlock * R - 1) / ((int64_t)kBlock * R));
  if (G < 1 || G > kCoopMaxG || m < 1) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(cw, 0, sizeof(CoopWs), s);
  if (e != hipSuccess) return e;
  switch (R) {
    case 1:
      k_cg_coop<1><<<G, kBlock, 0, s>>>(n, rowptr, col, val, x, r, p0, p1, st, slot0, m, cw, ticks);
      break;
    case 2:
      k_cg_coop<2><<<G, kBlock, 0, s>>>(n, rowptr, col, val, x, r, p0, p1, st, slot0, m, cw, ticks);
      break;
    case 4:
      k_cg_coop<4><<<G, kBlock, 0, s>>>(n, rowptr, col, val, x, r, p0, p1, st, slot0, m, cw, ticks);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace cgx
