// cgx_kernels.hip — gfx950 kernels of the CG hot path.
//
// Reference path (XeniaHerr/ConjugateGradient): the loop body of CG::solve
// (src/CG.hpp:359-436) issues 12 commands per iteration — fill, scalar reset,
// CSR-scalar SpMV (VectorOperations.hpp:438-466), two dot products
// (:287-309), three AXPY-type updates (:380-428), three single_task scalar
// kernels and a dead copy. Here one iteration is three bandwidth kernels:
//
//   k_spmv_dot   Ap = A p, and p.Ap                  (CG.hpp:374-379)
//   k_update_r   alpha; r -= alpha Ap, and r.r        (CG.hpp:381-393,406-407)
//   k_update_xp  alpha, beta; x += alpha p; p = r + beta p; stop rule
//                                                     (CG.hpp:390,396-418,436)
//
// Design notes (DESIGN.md has the long form):
//  * SpMV is CSR-stream: a workgroup owns a row block (<= 256 rows, <= 2048
//    entries); its entries are read with coalesced loads, multiplied by the
//    gathered p values and staged in LDS, then each thread sums one row in
//    ascending column order starting from 0 — the reference's per-row order
//    (VectorOperations.hpp:456-459), so Ap is bit-identical to it.
//  * Rows longer than a tile get a whole workgroup (tree-summed).
//  * Dots are reduced deterministically: fixed-order wave shuffles, LDS,
//    per-workgroup partials stored write-through (sc1), a ticket, and the
//    last workgroup sums the partials in index order (MI355X guide §6 G16,
//    hand-off table row 1). No float atomics.
//  * Grids are persistent (<= 2048 WGs = 8 per CU); row blocks are dealt so
//    that consecutive row blocks run on one XCD (blockIdx % 8 groups), which
//    keeps the p gather window in that XCD's L2.
//  * Build with -ffp-contract=off: every product is rounded before the add,
//    as in the reference's expressions.
#include <hip/hip_runtime.h>

#include "cgx_internal.h"

namespace cgx {
namespace {

// ---------------------------------------------------------------------------
// write-through (sc1) scalar hand-off helpers
// ---------------------------------------------------------------------------
template <typename T> struct Bits;
template <> struct Bits<double> {
  using U = unsigned long long;
  static __device__ __forceinline__ U to(double v) { return (U)__double_as_longlong(v); }
  static __device__ __forceinline__ double from(U u) { return __longlong_as_double((long long)u); }
};
template <> struct Bits<float> {
  using U = unsigned int;
  static __device__ __forceinline__ U to(float v) { return __float_as_uint(v); }
  static __device__ __forceinline__ float from(U u) { return __uint_as_float(u); }
};

template <typename T> __device__ __forceinline__ void store_sc1(T *p, T v) {
  using U = typename Bits<T>::U;
  __hip_atomic_store(reinterpret_cast<U *>(p), Bits<T>::to(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T> __device__ __forceinline__ T load_sc1(const T *p) {
  using U = typename Bits<T>::U;
  return Bits<T>::from(__hip_atomic_load(reinterpret_cast<U *>(const_cast<T *>(p)),
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

template <typename T> __device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;  // lane 0 holds the sum
}

// Fixed-order block sum of K values; result valid in thread 0.
template <typename T, int K>
__device__ __forceinline__ void block_sum(T (&v)[K], T *lds) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = wave_sum(v[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) lds[k * 4 + w] = v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k)
      v[k] = ((lds[k * 4 + 0] + lds[k * 4 + 1]) + lds[k * 4 + 2]) + lds[k * 4 + 3];
  }
  __syncthreads();
}

// Grid-wide deterministic reduction. Every workgroup publishes its block sum
// write-through and takes a ticket; the workgroup that takes the last ticket
// sums all partials in workgroup order. Returns true in that workgroup, whose
// thread 0 then holds the totals in v[].
template <typename T, int K>
__device__ __forceinline__ bool grid_reduce(T (&v)[K], RedWs<T> *ws, T *lds, int *flag) {
  block_sum<T, K>(v, lds);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) store_sc1(&ws->partials[k * kMaxGrid + blockIdx.x], v[k]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(&ws->ticket, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    *flag = (prev == gridDim.x - 1);
  }
  __syncthreads();
  if (!*flag) return false;
  T acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    acc[k] = T(0);
    for (unsigned i = threadIdx.x; i < gridDim.x; i += kBlock)
      acc[k] += load_sc1(&ws->partials[k * kMaxGrid + i]);
  }
  block_sum<T, K>(acc, lds);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = acc[k];
    __hip_atomic_store(&ws->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return true;
}

// XCD-grouped logical workgroup id: blocks b and b+8 share an XCD (observed
// dispatch, speed only — MI355X guide §Workgroup dispatch), so give each
// blockIdx%8 group a contiguous range of logical ids.
__device__ __forceinline__ int logical_block() {
  const int G = gridDim.x, b = blockIdx.x;
  return (G & 7) ? b : (b & 7) * (G >> 3) + (b >> 3);
}

// ---------------------------------------------------------------------------
// CSR-stream SpMV over row blocks with a row epilogue
// ---------------------------------------------------------------------------
struct CsrArgs {
  const int *__restrict__ rowptr;
  const int *__restrict__ col;
  const int *__restrict__ rb;   // first row of each row block (nrb + 1)
  const int *__restrict__ rbk;  // rowptr[rb[i]]: first entry of each row block
  int nrb;
};

template <typename T> struct SpmvLds {
  T prod[kTile + 2];  // + 2 scratch slots for branch-free out-of-range stores
  int rp[kRowsPerBlock + 1];
  T red[4 * kMaxRed];
  int flag;
};

// Variant bits of the SpMV row loop (A/B-tested with cgx_tune_spmv):
//   1  XCD-contiguous work split: the blockIdx%8 group g walks row blocks
//      [g*nrb/8, (g+1)*nrb/8), so the p rows a block gathers were mostly just
//      fetched into the same XCD's L2 by its neighbours;
//   2  non-temporal loads for the once-read val/col streams (keep L2 for p);
//   4  paired loads: val as 16-B (f64) pairs and col as 8-B pairs from an
//      aligned base (the schedule caps a tile at kTile-2 entries so 4 passes
//      of 256 pairs always cover it).
template <typename T> struct PairOf;
template <> struct PairOf<double> { typedef double V __attribute__((ext_vector_type(2))); };
template <> struct PairOf<float> { typedef float V __attribute__((ext_vector_type(2))); };
typedef int Int2 __attribute__((ext_vector_type(2)));

template <bool NT, typename P> __device__ __forceinline__ P ldg(const P *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <int V>
__device__ __forceinline__ void work_range(int nrb, int &first, int &step, int &end) {
  const int G = gridDim.x;
  if ((V & 1) && (G & 7) == 0) {
    const int g = blockIdx.x & 7, per = G >> 3;
    first = (int)(((int64_t)nrb * g) >> 3) + (blockIdx.x >> 3);
    end = (int)(((int64_t)nrb * (g + 1)) >> 3);
    step = per;
  } else {
    first = logical_block();
    step = G;
    end = nrb;
  }
}

template <typename T, int V, class Epi>
__device__ __forceinline__ void spmv_rows(const CsrArgs &A, const T *__restrict__ val,
                                          const T *__restrict__ x, Epi &epi,
                                          SpmvLds<T> &sm) {
  constexpr bool NT = (V & 2) != 0;
  constexpr bool PAIRS = (V & 4) != 0;
  const int t = threadIdx.x;
  int first, step, end;
  work_range<V>(A.nrb, first, step, end);
  for (int b = first; b < end; b += step) {
    const int r0 = A.rb[b], r1 = A.rb[b + 1];
    const int nrows = r1 - r0;
    for (int i = t; i <= nrows; i += kBlock) sm.rp[i] = A.rowptr[r0 + i];
    __syncthreads();
    const int k0 = sm.rp[0];
    const int cnt = sm.rp[nrows] - k0;
    if (cnt <= kTileCap) {
      if (cnt > 0) {
        if constexpr (PAIRS) {
          using PV = typename PairOf<T>::V;
          constexpr int U = kTile / (2 * kBlock);
          const int ka = k0 & ~1;
          const int npairs = (k0 + cnt - ka + 1) >> 1;
          const PV *v2 = reinterpret_cast<const PV *>(val + ka);
          const Int2 *c2 = reinterpret_cast<const Int2 *>(A.col + ka);
          PV v[U];
          Int2 c[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int j = min(t + u * kBlock, npairs - 1);
            v[u] = ldg<NT>(v2 + j);
            c[u] = ldg<NT>(c2 + j);
          }
          T g0[U], g1[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            g0[u] = x[c[u].x];
            g1[u] = x[c[u].y];
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int pos = 2 * (t + u * kBlock) + ka - k0;
            if (pos >= 0 && pos < cnt) sm.prod[pos] = v[u].x * g0[u];
            if (pos + 1 >= 0 && pos + 1 < cnt) sm.prod[pos + 1] = v[u].y * g1[u];
          }
        } else {
          constexpr int U = kTile / kBlock;
          T v[U];
          int c[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int k = min(t + u * kBlock, cnt - 1);
            v[u] = ldg<NT>(val + k0 + k);
            c[u] = ldg<NT>(A.col + k0 + k);
          }
          T g[U];
#pragma unroll
          for (int u = 0; u < U; ++u) g[u] = x[c[u]];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int k = t + u * kBlock;
            if (k < cnt) sm.prod[k] = v[u] * g[u];
          }
        }
      }
      __syncthreads();
      if (t < nrows) {
        const int a = sm.rp[t] - k0, e = sm.rp[t + 1] - k0;
        epi.pre(r0 + t);
        T s = T(0);
        for (int j = a; j < e; ++j) s += sm.prod[j];
        epi.row(r0 + t, s);
      }
      __syncthreads();
    } else {
      // One row longer than a tile (the schedule isolates such rows).
      T s[1] = {T(0)};
      for (int k = t; k < cnt; k += kBlock) s[0] += val[k0 + k] * x[A.col[k0 + k]];
      block_sum<T, 1>(s, sm.red);
      if (t == 0) {
        epi.pre(r0);
        epi.row(r0, s[0]);
      }
      __syncthreads();
    }
  }
}

// Software-pipelined form (variant bit 8, paired loads only): while a block
// gathers p and sums its rows, the val/col pairs of the block it processes
// next are already in flight. Every load is issued unconditionally (clamped
// to valid addresses) so the compiler's in-order vmcnt bookkeeping can wait
// for the current block's gathers without draining the prefetch.
template <typename T, int V, class Epi>
__device__ __forceinline__ void spmv_rows_pipe(const CsrArgs &A, const T *__restrict__ val,
                                               const T *__restrict__ x, Epi &epi,
                                               SpmvLds<T> &sm) {
  constexpr bool NT = (V & 2) != 0;
  using PV = typename PairOf<T>::V;
  constexpr int U = kTile / (2 * kBlock);
  const int t = threadIdx.x;
  int b, step, end;
  work_range<V>(A.nrb, b, step, end);
  if (b >= end) return;
  int r0 = A.rb[b], r1 = A.rb[b + 1], k0 = A.rbk[b], k1 = A.rbk[b + 1];
  PV v[U];
  Int2 c[U];
  auto issue = [&](int kk0, int kk1, PV(&vv)[U], Int2(&cc)[U]) {
    const bool ok = kk1 > kk0;  // empty blocks read pairs [0, 1] (nnz >= 2)
    const int ka = ok ? (kk0 & ~1) : 0;
    const int np = ok ? ((kk1 - ka + 1) >> 1) : 1;
    const PV *v2 = reinterpret_cast<const PV *>(val + ka);
    const Int2 *c2 = reinterpret_cast<const Int2 *>(A.col + ka);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = min(t + u * kBlock, np - 1);
      vv[u] = ldg<NT>(v2 + j);
      cc[u] = ldg<NT>(c2 + j);
    }
  };
  issue(k0, k1, v, c);
  for (;;) {
    const int nb = b + step;
    const bool has_next = nb < end;
    const int nbb = has_next ? nb : b;
    const int nr0 = A.rb[nbb], nr1 = A.rb[nbb + 1], nk0 = A.rbk[nbb], nk1 = A.rbk[nbb + 1];
    const int nrows = r1 - r0, cnt = k1 - k0;
    const int tr = min(t, max(nrows - 1, 0));
    const int a = A.rowptr[r0 + tr] - k0, e = A.rowptr[r0 + tr + 1] - k0;
    epi.pre(r0 + tr);
    T g0[U], g1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      g0[u] = x[c[u].x];
      g1[u] = x[c[u].y];
    }
    __builtin_amdgcn_sched_barrier(0);
    PV vn[U];
    Int2 cn[U];
    issue(nk0, nk1, vn, cn);
    __builtin_amdgcn_sched_barrier(0);
    {
      // branch-free: lanes outside [0, cnt) store into the scratch slots
      const int ka = k0 & ~1;
      const int lim = min(cnt, kTileCap);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int pos = 2 * (t + u * kBlock) + ka - k0;
        const int q0 = (pos >= 0 && pos < lim) ? pos : kTile;
        const int q1 = (pos + 1 >= 0 && pos + 1 < lim) ? pos + 1 : kTile + 1;
        sm.prod[q0] = v[u].x * g0[u];
        sm.prod[q1] = v[u].y * g1[u];
      }
    }
    if (cnt <= kTileCap) {
      __syncthreads();
      if (t < nrows) {
        T s = T(0);
        for (int j = a; j < e; ++j) s += sm.prod[j];
        epi.row(r0 + t, s);
      }
      __syncthreads();
    } else {
      // one row longer than a tile
      __syncthreads();
      T s[1] = {T(0)};
      for (int k = t; k < cnt; k += kBlock) s[0] += val[k0 + k] * x[A.col[k0 + k]];
      block_sum<T, 1>(s, sm.red);
      if (t == 0) epi.row(r0, s[0]);
      __syncthreads();
    }
    if (!has_next) break;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = vn[u];
      c[u] = cn[u];
    }
    b = nb;
    r0 = nr0;
    r1 = nr1;
    k0 = nk0;
    k1 = nk1;
  }
}

template <typename T, int V, class Epi>
__device__ __forceinline__ void spmv_any(const CsrArgs &A, const T *__restrict__ val,
                                         const T *__restrict__ x, Epi &epi, SpmvLds<T> &sm) {
  if constexpr ((V & 8) != 0) spmv_rows_pipe<T, V, Epi>(A, val, x, epi, sm);
  else spmv_rows<T, V, Epi>(A, val, x, epi, sm);
}

// Row epilogues: pre(i) loads the row's own operands early (the pipelined
// loop issues it before the next block's prefetch, so waiting on it never
// waits on the prefetch); row(i, s) consumes the row sum.
template <typename T> struct EpiStore {
  T *__restrict__ y;
  __device__ __forceinline__ void pre(int) {}
  __device__ __forceinline__ void row(int i, T s) { y[i] = s; }
};
template <typename T> struct EpiDot {  // helper = A p; value2 += helper.p
  T *__restrict__ Ap;
  const T *__restrict__ p;
  T acc, pv;
  __device__ __forceinline__ void pre(int i) { pv = p[i]; }
  __device__ __forceinline__ void row(int i, T s) {
    Ap[i] = s;
    acc += s * pv;
  }
};
template <typename T> struct EpiInit {  // CG.hpp:325-331 (+ :341)
  const T *__restrict__ b;
  T *__restrict__ r;
  T *__restrict__ p;
  T acc, bv;
  __device__ __forceinline__ void pre(int i) { bv = b[i]; }
  __device__ __forceinline__ void row(int i, T s) {
    const T ri = bv - s;
    r[i] = ri;
    p[i] = ri;
    acc += ri * ri;
  }
};
template <typename T> struct EpiAccuracy {  // CG.hpp:489-497
  const T *__restrict__ b;
  const T *__restrict__ x;
  T acc0, acc1, bv, xv;
  __device__ __forceinline__ void pre(int i) {
    bv = b[i];
    xv = x[i];
  }
  __device__ __forceinline__ void row(int i, T s) {
    const T a = bv - s;
    acc0 += a * a;
    acc1 += xv * xv;
  }
};

template <typename T, int V>
__global__ __launch_bounds__(kBlock) void k_spmv(CsrArgs A, const T *__restrict__ val,
                                                 const T *__restrict__ x, T *__restrict__ y) {
  __shared__ SpmvLds<T> sm;
  EpiStore<T> e{y};
  spmv_any<T, V>(A, val, x, e, sm);
}

template <typename T, int V>
__global__ __launch_bounds__(kBlock) void k_cg_init(CsrArgs A, const T *__restrict__ val,
                                                    const T *__restrict__ x,
                                                    const T *__restrict__ b, T *__restrict__ r,
                                                    T *__restrict__ p, CgScalars<T> *st,
                                                    RedWs<T> *ws, T tol, long long cap) {
  __shared__ SpmvLds<T> sm;
  EpiInit<T> e{b, r, p, T(0), T(0)};
  spmv_any<T, V>(A, val, x, e, sm);
  T v[1] = {e.acc};
  if (grid_reduce<T, 1>(v, ws, sm.red, &sm.flag) && threadIdx.x == 0) {
    st->rxr[0] = v[0];
    st->pAp[0] = st->rr[0] = T(0);
    st->tol = tol;
    st->active[0] = 1;
    st->active[1] = st->active[2] = st->active[3] = 0;
    st->bodies = 0;
    st->cap = cap;
    st->stopped = 0;
  }
}

template <typename T, int V>
__global__ __launch_bounds__(kBlock) void k_spmv_dot(CsrArgs A, const T *__restrict__ val,
                                                     const T *__restrict__ p,
                                                     T *__restrict__ Ap, CgScalars<T> *st,
                                                     int slot, RedWs<T> *ws) {
  if (!st->active[slot]) return;
  __shared__ SpmvLds<T> sm;
  EpiDot<T> e{Ap, p, T(0), T(0)};
  spmv_any<T, V>(A, val, p, e, sm);
  T v[1] = {e.acc};
  if (grid_reduce<T, 1>(v, ws, sm.red, &sm.flag) && threadIdx.x == 0) st->pAp[slot] = v[0];
}

template <typename T, int V>
__global__ __launch_bounds__(kBlock) void k_accuracy(CsrArgs A, const T *__restrict__ val,
                                                     const T *__restrict__ b,
                                                     const T *__restrict__ x, T *out2,
                                                     RedWs<T> *ws) {
  __shared__ SpmvLds<T> sm;
  EpiAccuracy<T> e{b, x, T(0), T(0), T(0), T(0)};
  spmv_any<T, V>(A, val, x, e, sm);
  T v[2] = {e.acc0, e.acc1};
  if (grid_reduce<T, 2>(v, ws, sm.red, &sm.flag) && threadIdx.x == 0) {
    out2[0] = v[0];
    out2[1] = v[1];
  }
}

// ---------------------------------------------------------------------------
// streaming vector kernels (16 B per lane where the pointers allow it)
// ---------------------------------------------------------------------------
template <typename T> struct Vec2;
template <> struct Vec2<double> { using V = double2; };
template <> struct Vec2<float> { using V = float2; };

// r = r - alpha * Ap ; rr = r.r          (CG.hpp:381-393, 406-407)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_update_r(int64_t n, T *__restrict__ r,
                                                     const T *__restrict__ Ap,
                                                     CgScalars<T> *st, int slot,
                                                     RedWs<T> *ws) {
  if (!st->active[slot]) return;
  __shared__ T red[4];
  __shared__ int flag;
  const T alpha = st->rxr[slot] / st->pAp[slot];
  using V = typename Vec2<T>::V;
  const int64_t n2 = n >> 1;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  V *r2 = reinterpret_cast<V *>(r);
  const V *a2 = reinterpret_cast<const V *>(Ap);
  T acc = T(0);
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  for (; i + 3 * stride < n2; i += 4 * stride) {
    V rv[4], av[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { rv[u] = r2[i + u * stride]; av[u] = a2[i + u * stride]; }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      rv[u].x = rv[u].x - alpha * av[u].x;
      rv[u].y = rv[u].y - alpha * av[u].y;
      r2[i + u * stride] = rv[u];
      acc += rv[u].x * rv[u].x;
      acc += rv[u].y * rv[u].y;
    }
  }
  for (; i < n2; i += stride) {
    V rv = r2[i];
    const V av = a2[i];
    rv.x = rv.x - alpha * av.x;
    rv.y = rv.y - alpha * av.y;
    r2[i] = rv;
    acc += rv.x * rv.x;
    acc += rv.y * rv.y;
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const T v = r[n - 1] - alpha * Ap[n - 1];
    r[n - 1] = v;
    acc += v * v;
  }
  T v[1] = {acc};
  if (grid_reduce<T, 1>(v, ws, red, &flag) && threadIdx.x == 0) st->rr[slot] = v[0];
}

// x = x + alpha p ; p = r + beta p ; stop rule   (CG.hpp:390, 396-418, 436)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_update_xp(int64_t n, T *__restrict__ x,
                                                      T *__restrict__ p,
                                                      const T *__restrict__ r,
                                                      CgScalars<T> *st, int slot) {
  const int nxt = (slot + 1) & 3;
  if (!st->active[slot]) {
    if (blockIdx.x == 0 && threadIdx.x == 0) st->active[nxt] = 0;
    return;
  }
  const T rxr = st->rxr[slot];
  const T alpha = rxr / st->pAp[slot];
  const T rr = st->rr[slot];
  const T beta = rr / rxr;
  using V = typename Vec2<T>::V;
  const int64_t n2 = n >> 1;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  V *x2 = reinterpret_cast<V *>(x);
  V *p2 = reinterpret_cast<V *>(p);
  const V *rv2 = reinterpret_cast<const V *>(r);
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  for (; i + 3 * stride < n2; i += 4 * stride) {
    V xv[4], pv[4], rv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      xv[u] = x2[i + u * stride];
      pv[u] = p2[i + u * stride];
      rv[u] = rv2[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      xv[u].x = xv[u].x + alpha * pv[u].x;
      xv[u].y = xv[u].y + alpha * pv[u].y;
      pv[u].x = rv[u].x + beta * pv[u].x;
      pv[u].y = rv[u].y + beta * pv[u].y;
      x2[i + u * stride] = xv[u];
      p2[i + u * stride] = pv[u];
    }
  }
  for (; i < n2; i += stride) {
    V xv = x2[i], pv = p2[i];
    const V rv = rv2[i];
    xv.x = xv.x + alpha * pv.x;
    xv.y = xv.y + alpha * pv.y;
    pv.x = rv.x + beta * pv.x;
    pv.y = rv.y + beta * pv.y;
    x2[i] = xv;
    p2[i] = pv;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (n & 1) {
      const T pv = p[n - 1];
      x[n - 1] = x[n - 1] + alpha * pv;
      p[n - 1] = r[n - 1] + beta * pv;
    }
    const long long m = st->bodies + 1;
    st->bodies = m;
    const bool cond = isnan(rxr) || sqrt(rxr) <= st->tol;
    const bool cont = !cond && m < st->cap;
    st->active[nxt] = cont ? 1 : 0;
    st->rxr[nxt] = rr;
    st->stopped = cond ? 1 : (cont ? 0 : 2);
  }
}

// *res += x.y (dot_product_trivial / norm: accumulate, Q4)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_dot_acc(int64_t n, const T *__restrict__ x,
                                                    const T *__restrict__ y, T *res,
                                                    RedWs<T> *ws) {
  __shared__ T red[4];
  __shared__ int flag;
  T acc = T(0);
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    acc += x[i] * y[i];
  T v[1] = {acc};
  if (grid_reduce<T, 1>(v, ws, red, &flag) && threadIdx.x == 0) *res = *res + v[0];
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_axpby(int mode, int64_t n, const T *x,
                                                  const T *y, const T *a, const T *b,
                                                  T *res) {
  const T bv = *b;
  const T av = (mode == AX_SAXPBY) ? *a : T(0);
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const T xv = x[i], yv = y[i];
    T o;
    if (mode == AX_SAPBX) o = xv + bv * yv;        // VectorOperations.hpp:423
    else if (mode == AX_SAMBX) o = xv - bv * yv;   // :392
    else o = av * xv + bv * yv;                    // :362
    res[i] = o;
  }
}

template <typename T>
__global__ void k_scalar_div(const T *num, const T *den, T *out) { *out = *num / *den; }

template <typename T>
__global__ __launch_bounds__(kBlock) void k_fill(T *d, T v, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) d[i] = v;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_iota(T *d, int64_t n, double offset) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    d[i] = T(double(i) + 1.0 + offset);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_gather(const T *__restrict__ src,
                                                   const int *__restrict__ idx, int64_t n,
                                                   T *__restrict__ dst) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    dst[i] = src[idx[i]];
}

// Poisson rows [row_begin, row_end): columns ascending (-z,-y,-x,d,+x,+y,+z).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_poisson(int dim, int nx, int ny, int nz,
                                                    int64_t row_begin, int64_t row_end,
                                                    int *__restrict__ rowptr,
                                                    int *__restrict__ col,
                                                    T *__restrict__ val) {
  const int64_t nrows = row_end - row_begin;
  const int64_t base = poisson_row_offset(dim, nx, ny, nz, row_begin);
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t nxy = (int64_t)nx * ny;
  const T diag = T(2 * dim), off = T(-1);
  for (int64_t li = (int64_t)blockIdx.x * kBlock + threadIdx.x; li <= nrows; li += stride) {
    const int64_t row = row_begin + li;
    const int64_t k0 = poisson_row_offset(dim, nx, ny, nz, row) - base;
    rowptr[li] = (int)k0;
    if (li == nrows) continue;
    const int64_t z = (dim == 3) ? row / nxy : 0;
    const int64_t rem = row - z * nxy;
    const int64_t y = rem / nx, xx = rem - y * nx;
    int64_t k = k0;
    if (dim == 3 && z > 0) { col[k] = (int)(row - nxy); val[k++] = off; }
    if (y > 0) { col[k] = (int)(row - nx); val[k++] = off; }
    if (xx > 0) { col[k] = (int)(row - 1); val[k++] = off; }
    col[k] = (int)row; val[k++] = diag;
    if (xx < nx - 1) { col[k] = (int)(row + 1); val[k++] = off; }
    if (y < ny - 1) { col[k] = (int)(row + nx); val[k++] = off; }
    if (dim == 3 && z < nz - 1) { col[k] = (int)(row + nxy); val[k++] = off; }
  }
}

inline int elem_grid(int64_t n, int per_thread) {
  int64_t g = (n + (int64_t)kBlock * per_thread - 1) / ((int64_t)kBlock * per_thread);
  if (g < 1) g = 1;
  if (g > kMaxGrid) g = kMaxGrid;
  return (int)g;
}

inline CsrArgs args(const CsrDev &A) { return CsrArgs{A.rowptr, A.col, A.rb, A.rbk, A.nrb}; }

}  // namespace

// number of stored entries in rows [0, row) of the Poisson matrix
__host__ __device__ int64_t poisson_row_offset(int dim, int nx, int ny, int nz, int64_t row) {
  const int64_t nxy = (int64_t)nx * ny;
  int64_t cnt = row;  // diagonals
  const int64_t lines = row / nx, xx = row - lines * nx;
  cnt += lines * 2 * (int64_t)(nx - 1) + (xx > 0 ? xx - 1 : 0) + (xx < nx - 1 ? xx : nx - 1);
  const int64_t planes = row / nxy, rem = row - planes * nxy;
  const int64_t ycount = (int64_t)nx * (ny - 1);
  cnt += planes * 2 * ycount + (rem > nx ? rem - nx : 0) + (rem < ycount ? rem : ycount);
  if (dim == 3) {
    const int64_t zcount = nxy * (nz - 1);
    cnt += (row > nxy ? row - nxy : 0) + (row < zcount ? row : zcount);
  }
  return cnt;
}

template <typename T> int Launch<T>::grid_rows(int nrb) {
  return nrb < kMaxGrid ? (nrb < 1 ? 1 : nrb) : kMaxGrid;
}
template <typename T> int Launch<T>::grid_elems(int64_t n) { return elem_grid(n, 8); }

#define CGX_LAUNCH(kernel, grid, ...)                                              \
  do {                                                                             \
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), 0, s, __VA_ARGS__);       \
    return hipGetLastError();                                                      \
  } while (0)

// SpMV variant used in production (bits: see spmv_rows / spmv_rows_pipe),
// chosen with cgx_tune_spmv on MI355X (profiles/r01_tune_spmv.log):
// pipelined + paired + XCD split, with non-temporal val/col loads only when
// the matrix outgrows the 256 MiB Infinity Cache (a cache-resident matrix is
// re-read every iteration, nt loads would throw that reuse away). Without
// 16-B aligned val / 8-B aligned col the paired and pipelined bits drop.
constexpr int kSpmvV = -1;
constexpr int64_t kNtMinBytes = int64_t(256) << 20;

template <typename T> inline int spmv_variant(const CsrDev &A, int v = kSpmvV) {
  if (v < 0) v = (A.nnz * int64_t(sizeof(T) + sizeof(int)) >= kNtMinBytes) ? 15 : 13;
  v &= 15;
  if (((uintptr_t)A.val % (2 * sizeof(T))) || ((uintptr_t)A.col % 8) || A.nnz < 2) v &= ~12;
  if ((v & 8) && !(v & 4)) v &= ~8;  // the pipelined loop uses paired loads
  return v;
}

#define CGX_LAUNCH_V(KERNEL, VV, ...)                                          \
  do {                                                                         \
    hipLaunchKernelGGL((KERNEL<T, VV>), dim3(grid_rows(A.nrb)), dim3(kBlock), 0, s, \
                       __VA_ARGS__);                                           \
    return hipGetLastError();                                                  \
  } while (0)

#define CGX_SPMV_SWITCH(v, KERNEL, ...)                                        \
  switch (v) {                                                                 \
    case 0: CGX_LAUNCH_V(KERNEL, 0, __VA_ARGS__);                              \
    case 1: CGX_LAUNCH_V(KERNEL, 1, __VA_ARGS__);                              \
    case 2: CGX_LAUNCH_V(KERNEL, 2, __VA_ARGS__);                              \
    case 3: CGX_LAUNCH_V(KERNEL, 3, __VA_ARGS__);                              \
    case 4: CGX_LAUNCH_V(KERNEL, 4, __VA_ARGS__);                              \
    case 5: CGX_LAUNCH_V(KERNEL, 5, __VA_ARGS__);                              \
    case 6: CGX_LAUNCH_V(KERNEL, 6, __VA_ARGS__);                              \
    case 7: CGX_LAUNCH_V(KERNEL, 7, __VA_ARGS__);                              \
    case 12: CGX_LAUNCH_V(KERNEL, 12, __VA_ARGS__);                            \
    case 13: CGX_LAUNCH_V(KERNEL, 13, __VA_ARGS__);                            \
    case 14: CGX_LAUNCH_V(KERNEL, 14, __VA_ARGS__);                            \
    default: CGX_LAUNCH_V(KERNEL, 15, __VA_ARGS__);                            \
  }

template <typename T>
hipError_t Launch<T>::spmv(const CsrDev &A, const T *x, T *y, hipStream_t s) {
  CGX_SPMV_SWITCH(spmv_variant<T>(A), k_spmv, args(A), (const T *)A.val, x, y);
}
template <typename T>
hipError_t Launch<T>::cg_init(const CsrDev &A, const T *x, const T *b, T *r, T *p,
                              CgScalars<T> *st, RedWs<T> *ws, T tol, long long cap,
                              hipStream_t s) {
  CGX_SPMV_SWITCH(spmv_variant<T>(A), k_cg_init, args(A), (const T *)A.val, x, b, r, p, st, ws,
                  tol, cap);
}
template <typename T>
hipError_t Launch<T>::spmv_dot(const CsrDev &A, const T *p, T *Ap, CgScalars<T> *st,
                               int slot, RedWs<T> *ws, hipStream_t s) {
  CGX_SPMV_SWITCH(spmv_variant<T>(A), k_spmv_dot, args(A), (const T *)A.val, p, Ap, st, slot,
                  ws);
}
template <typename T>
hipError_t Launch<T>::spmv_dot_variant(int v, const CsrDev &A, const T *p, T *Ap,
                                       CgScalars<T> *st, RedWs<T> *ws, hipStream_t s) {
  CGX_SPMV_SWITCH(spmv_variant<T>(A, v), k_spmv_dot, args(A), (const T *)A.val, p, Ap, st, 0,
                  ws);
}
template <typename T>
hipError_t Launch<T>::update_r(int64_t n, T *r, const T *Ap, CgScalars<T> *st, int slot,
                               RedWs<T> *ws, hipStream_t s) {
  CGX_LAUNCH(k_update_r<T>, grid_elems(n), n, r, Ap, st, slot, ws);
}
template <typename T>
hipError_t Launch<T>::update_xp(int64_t n, T *x, T *p, const T *r, CgScalars<T> *st,
                                int slot, hipStream_t s) {
  CGX_LAUNCH(k_update_xp<T>, grid_elems(n), n, x, p, r, st, slot);
}
template <typename T>
hipError_t Launch<T>::dot_acc(int64_t n, const T *x, const T *y, T *res, RedWs<T> *ws,
                              hipStream_t s) {
  CGX_LAUNCH(k_dot_acc<T>, elem_grid(n, 8), n, x, y, res, ws);
}
template <typename T>
hipError_t Launch<T>::axpby(int mode, int64_t n, const T *x, const T *y, const T *a,
                            const T *b, T *res, hipStream_t s) {
  CGX_LAUNCH(k_axpby<T>, elem_grid(n, 4), mode, n, x, y, a, b, res);
}
template <typename T>
hipError_t Launch<T>::scalar_div(const T *num, const T *den, T *out, hipStream_t s) {
  hipLaunchKernelGGL(k_scalar_div<T>, dim3(1), dim3(1), 0, s, num, den, out);
  return hipGetLastError();
}
template <typename T> hipError_t Launch<T>::fill(T *d, T v, int64_t n, hipStream_t s) {
  CGX_LAUNCH(k_fill<T>, elem_grid(n, 4), d, v, n);
}
template <typename T>
hipError_t Launch<T>::iota(T *d, int64_t n, double offset, hipStream_t s) {
  CGX_LAUNCH(k_iota<T>, elem_grid(n, 4), d, n, offset);
}
template <typename T>
hipError_t Launch<T>::accuracy(const CsrDev &A, const T *b, const T *x, T *out2,
                               RedWs<T> *ws, hipStream_t s) {
  CGX_SPMV_SWITCH(spmv_variant<T>(A), k_accuracy, args(A), (const T *)A.val, b, x, out2, ws);
}
template <typename T>
hipError_t Launch<T>::poisson(int dim, int nx, int ny, int nz, int64_t row_begin,
                              int64_t row_end, int *rowptr, int *col, T *val,
                              hipStream_t s) {
  CGX_LAUNCH(k_poisson<T>, elem_grid(row_end - row_begin + 1, 4), dim, nx, ny, nz, row_begin,
             row_end, rowptr, col, val);
}
template <typename T>
hipError_t Launch<T>::gather(const T *src, const int *idx, int64_t n, T *dst,
                             hipStream_t s) {
  CGX_LAUNCH(k_gather<T>, elem_grid(n, 4), src, idx, n, dst);
}

template struct Launch<double>;
template struct Launch<float>;

}  // namespace cgx
