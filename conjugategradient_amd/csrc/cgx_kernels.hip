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
#include <hip/hip_ext.h>

#include <algorithm>
#include <map>
#include <mutex>

#include <cstdlib>
#include <type_traits>

#include "cgx_dd.h"
#include "cgx_internal.h"
#include "cgx_objects.h"
#include "cgx_peer_dev.h"

namespace cgx {
thread_local ExecTiming g_exec;
namespace {

// a launch that takes the pending execution-timing events (g_exec) when set
#define CGX_GGL(K, G, B, SH, S, ...)                                       \
  do {                                                                    \
    if (g_exec.start) {                                                   \
      hipEvent_t e0_ = g_exec.start, e1_ = g_exec.stop;                   \
      g_exec.start = g_exec.stop = nullptr;                               \
      g_exec.used = true;                                                 \
      hipExtLaunchKernelGGL(K, G, B, SH, S, e0_, e1_, 0, __VA_ARGS__);    \
    } else {                                                              \
      hipLaunchKernelGGL(K, G, B, SH, S, __VA_ARGS__);                    \
    }                                                                     \
  } while (0)
inline hipError_t cgx_lk(const void *k, dim3 g, dim3 b, void **args, size_t sh, hipStream_t s) {
  if (g_exec.start) {
    hipEvent_t e0 = g_exec.start, e1 = g_exec.stop;
    g_exec.start = g_exec.stop = nullptr;
    g_exec.used = true;
    return hipExtLaunchKernel(k, g, b, args, sh, s, e0, e1, 0);
  }
  return hipLaunchKernel(k, g, b, args, sh, s);
}


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

// Fixed-order workgroup sum of one pair per thread; valid in thread 0.
// lds: 2 T per wave (8 for a 256-thread workgroup).
template <typename T> __device__ __forceinline__ Dd<T> block_sum_dd(Dd<T> v, T *lds) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int W = kBlock / 64;
  v = wave_sum_dd(v);
  if (lane == 0) {
    lds[2 * w] = v.hi;
    lds[2 * w + 1] = v.lo;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    v = Dd<T>(lds[0], lds[1]);
#pragma unroll
    for (int k = 1; k < W; ++k) v += Dd<T>(lds[2 * k], lds[2 * k + 1]);
  }
  __syncthreads();
  return v;
}

// A workgroup's partial of a dot: slot i of part holds the pair (hi at 2 i,
// lo at 2 i + 1). Uniform control flow; thread 0 stores.
template <typename T>
__device__ __forceinline__ void store_part(T *part, int i, Dd<T> v, T *lds) {
  v = block_sum_dd(v, lds);
  if (threadIdx.x == 0) {
    part[2 * i] = v.hi;
    part[2 * i + 1] = v.lo;
  }
}
template <typename T> __device__ __forceinline__ Dd<T> load_part(const T *part, int i) {
  using V = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
  const V v = *reinterpret_cast<const V *>(part + 2 * i);
  return Dd<T>(v.x, v.y);
}

// Sum of the previous kernel's per-workgroup partials, in the same fixed
// order in every workgroup (thread t: t, t + 256, ...; then block_sum_dd),
// so all workgroups get the identical value. Stream order makes the
// producer's plain stores visible; no atomics, no write-through. Uniform
// control flow. lds: 8 T.
template <typename T>
__device__ __forceinline__ Dd<T> sum_parts_dd(const T *__restrict__ part, int np, T *lds) {
  __shared__ T bc[2];
  Dd<T> v(T(0));
  for (int i = threadIdx.x; i < np; i += kBlock) v += load_part(part, i);
  v = block_sum_dd(v, lds);
  if (threadIdx.x == 0) {
    bc[0] = v.hi;
    bc[1] = v.lo;
  }
  __syncthreads();
  return Dd<T>(bc[0], bc[1]);
}
template <typename T>
__device__ __forceinline__ T sum_parts(const T *__restrict__ part, int np, T *lds) {
  return sum_parts_dd(part, np, lds).value();
}

// LDS-only workgroup barrier: waits for this wave's LDS operations, not for
// its outstanding global loads (__syncthreads would drain those too).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// sum_parts in two steps, same order and value, for a kernel that issues
// its first stream loads in between: parts_load puts this thread's partials
// in registers (all loads issued, none waited for); parts_sum adds them and
// reduces over the workgroup through LDS with LDS-only barriers, so loads
// issued after parts_load stay in flight (vmcnt waits in issue order).
constexpr int kPartsPerThread = 2 * kMaxGrid / kBlock;  // split SpMV: 2 launches
// (KP: the loads per thread, a launch's bound on ceil(np / kBlock); the
// vector kernels are instantiated for 4, 8 and 16 so a launch after a
// 1,024-workgroup SpMV does not issue 16)
template <typename T, int KP>
__device__ __forceinline__ void parts_load(const T *__restrict__ part, int np, Dd<T> (&pl)[KP]) {
#pragma unroll
  for (int k = 0; k < KP; ++k)  // unconditional (np >= 1): exact vmcnt waits
    pl[k] = load_part(part, min((int)threadIdx.x + k * kBlock, np - 1));
}
// parts_load for a kernel with no stream loads behind it: only the np
// partials are loaded (a few at small grids; parts_load issues
// kPartsPerThread per thread whatever np is)
template <typename T>
__device__ __forceinline__ void parts_load_np(const T *__restrict__ part, int np,
                                              Dd<T> (&pl)[kPartsPerThread]) {
#pragma unroll
  for (int k = 0; k < kPartsPerThread; ++k) {
    const int i = (int)threadIdx.x + k * kBlock;
    pl[k] = i < np ? load_part(part, i) : Dd<T>(T(0));
  }
}
template <typename T, int KP>
__device__ __forceinline__ Dd<T> parts_sum_dd(const Dd<T> (&pl)[KP], int np, T *lds) {
  __shared__ T bc[2];
  Dd<T> v(T(0));
#pragma unroll
  for (int k = 0; k < KP; ++k)
    if ((int)threadIdx.x + k * kBlock < np) v += pl[k];  // sum_parts order
  v = wave_sum_dd(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    lds[2 * w] = v.hi;
    lds[2 * w + 1] = v.lo;
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    v = Dd<T>(lds[0], lds[1]);
#pragma unroll
    for (int k = 1; k < kBlock / 64; ++k) v += Dd<T>(lds[2 * k], lds[2 * k + 1]);
    bc[0] = v.hi;
    bc[1] = v.lo;
  }
  lds_barrier();
  return Dd<T>(bc[0], bc[1]);
}
template <typename T, int KP>
__device__ __forceinline__ T parts_sum(const Dd<T> (&pl)[KP], int np, T *lds) {
  return parts_sum_dd(pl, np, lds).value();
}

// Late active check (measured in round 2):
// a body kernel issues its first loads (scalars, partials, first stream
// block; valid memory whether or not the body runs) together with the
// active flag and branches on the flag afterwards, so a cache-resident
// body pays one load round trip before its first store instead of two.
// LLVM sinks a load whose only uses lie in one successor of the branch;
// keep() in the inactive successor uses them there too (an empty asm: it
// waits for them on that path only), so they stay where they were issued.
template <typename T> __device__ __forceinline__ void keep(const T &a) {
  if constexpr (sizeof(T) == 16) {
    asm volatile("" ::"v"(a.x), "v"(a.y));
  } else {
    asm volatile("" ::"v"(a));
  }
}
template <typename T> __device__ __forceinline__ void keep(const Dd<T> &a) {
  asm volatile("" ::"v"(a.hi), "v"(a.lo));
}
template <typename T, int K> __device__ __forceinline__ void keep(const T (&a)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) keep(a[k]);
}

// Grid-wide deterministic reduction. Every workgroup publishes its block sum
// write-through and takes the ticket of its group (blockIdx % kRedGroups). The
// last arrival of a group sums the group's partials in workgroup order and
// takes the top ticket; the last group sums the group sums in group order.
// The result is independent of arrival order. Returns true in that final
// workgroup, whose thread 0 then holds the totals in v[].
template <typename T, int K>
__device__ __forceinline__ bool grid_reduce(T (&v)[K], RedWs<T> *ws, T *lds, int *flag) {
  block_sum<T, K>(v, lds);
  const unsigned G = gridDim.x;
  const unsigned g = blockIdx.x % kRedGroups;
  const unsigned ngroups = G < (unsigned)kRedGroups ? G : (unsigned)kRedGroups;
  const unsigned members = (G - g + kRedGroups - 1) / kRedGroups;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) store_sc1(&ws->partials[k * kMaxGrid + blockIdx.x], v[k]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(&ws->ticket[g], 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    *flag = (prev == members - 1);
  }
  __syncthreads();
  if (!*flag) return false;
  // last of group g: sum the group's partials in workgroup order
  T acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    acc[k] = T(0);
    for (unsigned i = g + kRedGroups * threadIdx.x; i < G; i += kRedGroups * kBlock)
      acc[k] += load_sc1(&ws->partials[k * kMaxGrid + i]);
  }
  block_sum<T, K>(acc, lds);
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(&ws->ticket[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int k = 0; k < K; ++k) store_sc1(&ws->gsum[k * kRedGroups + g], acc[k]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(&ws->top, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    *flag = (prev == ngroups - 1);
  }
  __syncthreads();
  if (!*flag) return false;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      T t = T(0);
      for (unsigned q = 0; q < ngroups; ++q) t += load_sc1(&ws->gsum[k * kRedGroups + q]);
      v[k] = t;
    }
    __hip_atomic_store(&ws->top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return true;
}

// grid_reduce of one double-length pair (the loop's dots: k_cg_init's r.r,
// the fused mode's p.Ap and r.r): the same tickets and order, pairs in
// partials[i] / partials[kMaxGrid + i] and gsum[g] / gsum[kRedGroups + g].
// True in the final workgroup, whose thread 0 then holds the total in v.
template <typename T>
__device__ __forceinline__ bool grid_reduce_dd(Dd<T> &v, RedWs<T> *ws, T *lds, int *flag) {
  v = block_sum_dd(v, lds);
  const unsigned G = gridDim.x;
  const unsigned g = blockIdx.x % kRedGroups;
  const unsigned ngroups = G < (unsigned)kRedGroups ? G : (unsigned)kRedGroups;
  const unsigned members = (G - g + kRedGroups - 1) / kRedGroups;
  if (threadIdx.x == 0) {
    store_sc1(&ws->partials[blockIdx.x], v.hi);
    store_sc1(&ws->partials[kMaxGrid + blockIdx.x], v.lo);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(&ws->ticket[g], 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    *flag = (prev == members - 1);
  }
  __syncthreads();
  if (!*flag) return false;
  Dd<T> acc(T(0));
  for (unsigned i = g + kRedGroups * threadIdx.x; i < G; i += kRedGroups * kBlock)
    acc += Dd<T>(load_sc1(&ws->partials[i]), load_sc1(&ws->partials[kMaxGrid + i]));
  acc = block_sum_dd(acc, lds);
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(&ws->ticket[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    store_sc1(&ws->gsum[g], acc.hi);
    store_sc1(&ws->gsum[kRedGroups + g], acc.lo);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(&ws->top, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    *flag = (prev == ngroups - 1);
  }
  __syncthreads();
  if (!*flag) return false;
  if (threadIdx.x == 0) {
    Dd<T> t(T(0));
    for (unsigned q = 0; q < ngroups; ++q)
      t += Dd<T>(load_sc1(&ws->gsum[q]), load_sc1(&ws->gsum[kRedGroups + q]));
    v = t;
    __hip_atomic_store(&ws->top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
  int64_t n;
  // SELL-64 copy (variant bit 2048)
  const SellSlice *__restrict__ sl;
  const int *__restrict__ sdict;
  const unsigned long long *__restrict__ sidx;
  const void *sval;
  int64_t nsl;
  const int *__restrict__ sorder;
  int rev;       // per launch: walk the rows high to low (alternating sweeps)
  int part_off;  // per launch: first partial slot of k_spmv_dot (split launches)
  const void *smask;  // SELL-P slot masks
  int64_t nx;         // gathered vector length
  const void *svc;    // SELL-P value codes (variant bit 32768)
  const void *svdict; // their dictionary (kVcDict entries)
  const void *svc4;   // 4-bit value codes (variant bit 262144)
  // plane march (variant bit 2097152): slices a plane apart (0: no march
  // pattern), the pattern's +-a offset (0: 2-D form), its pool base, and
  // the run length in planes (0: fill the grid)
  int mk, mo, mpat, ml;
  // leading workgroups of the launch that do something else (the halo push
  // of k_spmv_dot_push): the SpMV's work split and partials use blockIdx -
  // wg0 of gridDim - wg0 workgroups (a multiple of 8 keeps the XCD groups)
  int wg0;
  // value-code templates (kVT; sl is then the template slice table)
  const unsigned long long *vct;
  const short *__restrict__ col16;  // 16-bit column deltas (kC16)
  int nvt;
  // lean stencil walk (kVL): wave-major class bytes, class table, bytes per
  // wave row, the stencil's D and a
  const unsigned char *__restrict__ vl_cls;
  const VlClass *vl_tab;
  int vl_nst, vl_D, vl_a;
  int vl_P, vl_K;  // the chunked walk: planes per XCD group, slices per plane (0: natural)
  // the walk's per-slice-form slices are many enough (cgx_abi.cpp
  // build_lean_layout) to copy the value dictionary and the templates to LDS
  // before it; else they read them where they lie (no barrier at the start)
  int vl_lds;
  // CSR-stream block visit order (cgx_abi.cpp build_block_order): walk
  // position -> row block, a permutation within each XCD eighth (null: natural)
  const int *__restrict__ rbo;
  // the interleaved val / col copy (kIL)
  const char *__restrict__ il;
};

// the row block at walk position `pos` of the CSR-stream forms
__device__ __forceinline__ int block_at(const CsrArgs &A, int pos) {
  return A.rbo ? A.rbo[pos] : pos;
}

// Tile geometry of a variant: bit 64 selects half tiles (1024 entries /
// 128 rows per row block) — fewer registers per thread, more workgroups per
// CU to hide the gather latency. The matrix's row-block schedule must have
// been built for the same tile (cgx_csr_set_tile).
template <int V> struct TileOf {
  static constexpr int tile = (V & 64) ? 1024 : 2048;
  static constexpr int cap = tile - 2;  // paired loads read up to 2 extra entries
  static constexpr int rows = (V & 64) ? 128 : 256;
};

template <typename T, int TILE = kTile> struct SpmvLds {
  T prod[TILE + 4];  // + 4 scratch slots for branch-free out-of-range stores
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

// A paired (or quad) column load may run past the block's last entry kk1 - 1
// and, in the matrix's last block, past the end of the column array: the
// index it reads there is not a column. Elements at or past kk1 take the
// first element's column (always in range); their products land in scratch
// slots and are never summed. The over-read itself cannot fault: a pair
// (quad) load is naturally aligned, so it never crosses a page the array's
// last element does not also occupy.
__device__ __forceinline__ Int2 tail_cols(Int2 c, int e0, int kk1) {
  if (e0 + 1 >= kk1) c.y = c.x;
  return c;
}

// Non-temporal loads and stores for the vector streams whose data is not
// read again before far more than the 256 MB Infinity Cache has streamed
// past (Ap after k_update_r, x and the old p buffers in the flushing body):
// they then leave the cache to the vectors that the next kernel re-reads
// ("cache policy").
constexpr bool kStreamNt = true;
// ... but only for vectors too large for the working set to stay in the
// Infinity Cache: with vectors of <= 32 MB (the 256^3/8 slab's 16.8 MB, the
// G3 stand-in's 12.7 MB) every vector of the iteration is re-read from it,
// and plain loads and stores ran the slab bodies 2-3% faster
// (profiles/r03_slab_nt.log)
constexpr int64_t kNtVecBytes = int64_t(32) << 20;
// loads in flight per thread and trip in k_update_r (8 measured slower,
// DESIGN.md §7)
constexpr int kUR = 4;
template <typename T> __device__ __forceinline__ bool stream_nt(int64_t n) {
  return kStreamNt && n * (int64_t)sizeof(T) > kNtVecBytes;
}
// HIP vector types (double2, float2 of element T): non-temporal through the
// native vector of two T
template <bool NT, typename T, typename P> __device__ __forceinline__ P ldv(const P *p) {
  if constexpr (NT) {
    typedef T N __attribute__((ext_vector_type(2)));
    const N v = __builtin_nontemporal_load(reinterpret_cast<const N *>(p));
    P r;
    r.x = v.x;
    r.y = v.y;
    return r;
  } else {
    return *p;
  }
}
template <bool NT, typename T, typename P> __device__ __forceinline__ void stv(P *p, P v) {
  if constexpr (NT) {
    typedef T N __attribute__((ext_vector_type(2)));
    N n;
    n.x = v.x;
    n.y = v.y;
    __builtin_nontemporal_store(n, reinterpret_cast<N *>(p));
  } else {
    *p = v;
  }
}
template <bool NT, typename P> __device__ __forceinline__ P ldg(const P *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// Where the SpMV takes its x_j from: a stored vector, or p_j computed on the
// fly as r_j + beta * p_old_j (the fused iteration; the same expression the
// reference evaluates for p, CG.hpp:418, so the value is bit-identical).
// pair(c): elements c and c + 1 in one load of 2 T at T's alignment (SELL-P)
template <typename T> struct PairU;
template <> struct PairU<double> {
  typedef double V __attribute__((ext_vector_type(2), aligned(8)));
};
template <> struct PairU<float> { typedef float V __attribute__((ext_vector_type(2), aligned(4))); };
template <typename T> struct GatherX {
  const T *__restrict__ x;
  __device__ __forceinline__ T operator()(int c) const { return x[c]; }
  __device__ __forceinline__ typename PairU<T>::V pair(int c) const {
    return *reinterpret_cast<const typename PairU<T>::V *>(x + c);
  }
  // the pair at byte offset b (< 4 GiB): a scalar base plus a 32-bit vector
  // offset, one VALU add per gather instead of a 64-bit address
  __device__ __forceinline__ typename PairU<T>::V pair_b(unsigned b) const {
    return *reinterpret_cast<const typename PairU<T>::V *>(reinterpret_cast<const char *>(x) +
                                                           b);
  }
  // element i by a scalar load (uniform i)
  __device__ __forceinline__ T at_s(int i) const {
    return ((const __attribute__((address_space(4))) T *)x)[i];
  }
  // the tile walk's loads and their values (GatherP forms p_k from its pair)
  using Raw = typename PairU<T>::V;
  using Raw1 = T;
  __device__ __forceinline__ Raw raw_b(unsigned b) const { return pair_b(b); }
  __device__ __forceinline__ Raw form(const Raw &w) const { return w; }
  __device__ __forceinline__ Raw1 raw1(int i) const { return x[i]; }
  __device__ __forceinline__ T form1(const Raw1 &w) const { return w; }
};
// The boundary slices of a partitioned matrix with the peer transport's wait
// folded in (k_spmv_dot_bnd): x below n is this rank's p, from n on the
// ghost values are read where the neighbours pushed them, the landing buffer
// (uncached memory, its entry k is ghost n + k), instead of from p's ghost
// tail after a copy. Scalar reads of the landing buffer go through vector
// loads (no scalar-cache copy of memory other GPUs rewrite every body).
template <typename T> struct GatherXL {
  const T *__restrict__ x;
  const T *__restrict__ land;
  int n;
  __device__ __forceinline__ T operator()(int c) const { return c < n ? x[c] : land[c - n]; }
  __device__ __forceinline__ typename PairU<T>::V pair(int c) const {
    using U = typename PairU<T>::V;
    if (c + 1 < n) return *reinterpret_cast<const U *>(x + c);
    if (c >= n) return *reinterpret_cast<const U *>(land + (c - n));
    U r;  // the pair across the boundary: p[n - 1], ghost n
    r.x = x[c];
    r.y = land[0];
    return r;
  }
  __device__ __forceinline__ typename PairU<T>::V pair_b(unsigned b) const {
    return pair((int)(b / (unsigned)sizeof(T)));
  }
  __device__ __forceinline__ T at_s(int i) const {
    if (i < n) return ((const __attribute__((address_space(4))) T *)x)[i];
    return __hip_atomic_load(const_cast<T *>(land + (i - n)), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
  }
};

// NTP: p_{k-1} read non-temporally (the plane march reads each of its lines
// once as a center; mode 4 reads it again only in the slot-3 x flush)
template <typename T, bool NTP = false> struct GatherP {
  const T *__restrict__ r;
  const T *__restrict__ pp;
  T beta;
  __device__ __forceinline__ T operator()(int c) const { return r[c] + beta * pp[c]; }
  __device__ __forceinline__ typename PairU<T>::V pair(int c) const {
    using U = typename PairU<T>::V;
    const U a = *reinterpret_cast<const U *>(r + c);
    const U *pb = reinterpret_cast<const U *>(pp + c);
    U b;
    if constexpr (NTP) b = __builtin_nontemporal_load(pb);
    else b = *pb;
    U o;
    o.x = a.x + beta * b.x;
    o.y = a.y + beta * b.y;
    return o;
  }
  __device__ __forceinline__ typename PairU<T>::V pair_b(unsigned b) const {
    using U = typename PairU<T>::V;
    const U a = *reinterpret_cast<const U *>(reinterpret_cast<const char *>(r) + b);
    const U q = *reinterpret_cast<const U *>(reinterpret_cast<const char *>(pp) + b);
    U o;
    o.x = a.x + beta * q.x;
    o.y = a.y + beta * q.y;
    return o;
  }
  __device__ __forceinline__ T at_s(int i) const {
    return ((const __attribute__((address_space(4))) T *)r)[i] +
           beta * ((const __attribute__((address_space(4))) T *)pp)[i];
  }
  // pair_b in two halves: the loads (issued a step early by the team walk's
  // prefetch) and the forming (pair_b's expression, so the same value)
  struct Raw {
    typename PairU<T>::V a, q;
  };
  __device__ __forceinline__ Raw raw_b(unsigned b) const {
    using U = typename PairU<T>::V;
    return Raw{*reinterpret_cast<const U *>(reinterpret_cast<const char *>(r) + b),
               *reinterpret_cast<const U *>(reinterpret_cast<const char *>(pp) + b)};
  }
  __device__ __forceinline__ typename PairU<T>::V form(const Raw &w) const {
    typename PairU<T>::V o;
    o.x = w.a.x + beta * w.q.x;
    o.y = w.a.y + beta * w.q.y;
    return o;
  }
  struct Raw1 {
    T a, q;
  };
  __device__ __forceinline__ Raw1 raw1(int i) const { return Raw1{r[i], pp[i]}; }
  __device__ __forceinline__ T form1(const Raw1 &w) const { return w.a + beta * w.q; }
};
// Mode 4's boundary rows of a partitioned matrix (k_spmv_fd_bnd): own
// columns form p_k as GatherP, ghosts (from n on) are the neighbours' formed
// p_k where their pushes landed (GatherXL's landing buffer)
template <typename T> struct GatherPL {
  GatherP<T> g;
  const T *__restrict__ land;
  int n;
  __device__ __forceinline__ T operator()(int c) const { return c < n ? g(c) : land[c - n]; }
  __device__ __forceinline__ typename PairU<T>::V pair(int c) const {
    using U = typename PairU<T>::V;
    if (c + 1 < n) return g.pair(c);
    if (c >= n) return *reinterpret_cast<const U *>(land + (c - n));
    U r;
    r.x = g(c);
    r.y = land[0];
    return r;
  }
  __device__ __forceinline__ typename PairU<T>::V pair_b(unsigned b) const {
    return pair((int)(b / (unsigned)sizeof(T)));
  }
  __device__ __forceinline__ T at_s(int i) const {
    if (i < n) return g.at_s(i);
    return __hip_atomic_load(const_cast<T *>(land + (i - n)), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
  }
};

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

template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void spmv_rows(const CsrArgs &A, const T *__restrict__ val,
                                          const Gather &x, Epi &epi,
                                          SpmvLds<T, TileOf<V>::tile> &sm) {
  using TL = TileOf<V>;
  constexpr bool NT = (V & 2) != 0;
  constexpr bool PAIRS = (V & 4) != 0;
  const int t = threadIdx.x;
  int first, step, end;
  work_range<V>(A.nrb, first, step, end);
  for (int bp = first; bp < end; bp += step) {
    const int b = block_at(A, bp);
    const int r0 = A.rb[b], r1 = A.rb[b + 1];
    const int nrows = r1 - r0;
    const int k0 = A.rbk[b];
    const int cnt = A.rbk[b + 1] - k0;
    if (cnt <= TL::cap) {
      // this thread's row bounds and own operands go out with the block's
      // entries (none waits on another): two memory round trips per block,
      // the entries and then the gathers
      const int tr = min(t, max(nrows - 1, 0));
      const int ra = A.rowptr[r0 + tr] - k0, re = A.rowptr[r0 + tr + 1] - k0;
      epi.pre(r0 + tr);
      if (cnt > 0) {
        if constexpr (PAIRS) {
          using PV = typename PairOf<T>::V;
          constexpr int U = TL::tile / (2 * kBlock);
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
            if constexpr ((V & kC16) != 0) {
              // 16-bit deltas from the block's first row; a pair's element
              // outside the block (the one before k0 when k0 is odd, those
              // past its end) is relative to another block: it takes r0
              typedef short S2 __attribute__((ext_vector_type(2)));
              const S2 h = ldg<NT>(reinterpret_cast<const S2 *>(A.col16 + ka) + j);
              const int e0 = ka + 2 * j;
              c[u].x = (e0 >= k0 && e0 < k0 + cnt) ? r0 + (int)h.x : r0;
              c[u].y = (e0 + 1 >= k0 && e0 + 1 < k0 + cnt) ? r0 + (int)h.y : r0;
            } else {
              c[u] = tail_cols(ldg<NT>(c2 + j), ka + 2 * j, k0 + cnt);
            }
          }
          T g0[U], g1[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            g0[u] = x(c[u].x);
            g1[u] = x(c[u].y);
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int pos = 2 * (t + u * kBlock) + ka - k0;
            if (pos >= 0 && pos < cnt) sm.prod[pos] = v[u].x * g0[u];
            if (pos + 1 >= 0 && pos + 1 < cnt) sm.prod[pos + 1] = v[u].y * g1[u];
          }
        } else {
          constexpr int U = TL::tile / kBlock;
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
          for (int u = 0; u < U; ++u) g[u] = x(c[u]);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int k = t + u * kBlock;
            if (k < cnt) sm.prod[k] = v[u] * g[u];
          }
        }
      }
      __syncthreads();
      if (t < nrows) {
        T s = T(0);
        for (int j = ra; j < re; ++j) s += sm.prod[j];
        epi.row(r0 + t, s);
      }
      __syncthreads();
    } else {
      // One row longer than a tile (the schedule isolates such rows).
      T s[1] = {T(0)};
      for (int k = t; k < cnt; k += kBlock) s[0] += val[k0 + k] * x(A.col[k0 + k]);
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
template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void spmv_rows_pipe(const CsrArgs &A, const T *__restrict__ val,
                                               const Gather &x, Epi &epi,
                                               SpmvLds<T, TileOf<V>::tile> &sm) {
  using TL = TileOf<V>;
  constexpr bool NT = (V & 2) != 0;
  using PV = typename PairOf<T>::V;
  constexpr int U = TL::tile / (2 * kBlock);
  const int t = threadIdx.x;
  int b, step, end;
  work_range<V>(A.nrb, b, step, end);
  if (b >= end) return;
  const int b0 = block_at(A, b);
  int r0 = A.rb[b0], r1 = A.rb[b0 + 1], k0 = A.rbk[b0], k1 = A.rbk[b0 + 1];
  PV v[U];
  Int2 c[U];
  auto issue = [&](int kk0, int kk1, PV(&vv)[U], Int2(&cc)[U]) {
    const bool ok = kk1 > kk0;  // empty blocks read pairs [0, 1] (nnz >= 2)
    const int ka = ok ? (kk0 & ~1) : 0;
    const int np = ok ? ((kk1 - ka + 1) >> 1) : 1;
    if constexpr ((V & kIL) != 0) {
      // pair P of the matrix (entries 2P, 2P + 1): chunk P / kIlCh holds
      // kIlCh value pairs, then kIlCh column pairs (the same pairs, loads and
      // values as below, from one array)
      constexpr int64_t CB = (int64_t)kIlCh * (sizeof(PV) + sizeof(Int2));
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = min(t + u * kBlock, np - 1);
        const unsigned P = (unsigned)(ka >> 1) + (unsigned)j;
        const char *cb = A.il + (int64_t)(P >> kIlLog) * CB;
        const unsigned w = P & (kIlCh - 1);
        vv[u] = ldg<NT>(reinterpret_cast<const PV *>(cb) + w);
        cc[u] = tail_cols(ldg<NT>(reinterpret_cast<const Int2 *>(cb + kIlCh * sizeof(PV)) + w),
                          ka + 2 * j, kk1);
      }
      return;
    }
    const PV *v2 = reinterpret_cast<const PV *>(val + ka);
    const Int2 *c2 = reinterpret_cast<const Int2 *>(A.col + ka);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = min(t + u * kBlock, np - 1);
      vv[u] = ldg<NT>(v2 + j);
      cc[u] = tail_cols(ldg<NT>(c2 + j), ka + 2 * j, kk1);
    }
  };
  issue(k0, k1, v, c);
  for (;;) {
    const int nb = b + step;
    const bool has_next = nb < end;
    const int nbb = block_at(A, has_next ? nb : b);
    const int nr0 = A.rb[nbb], nr1 = A.rb[nbb + 1], nk0 = A.rbk[nbb], nk1 = A.rbk[nbb + 1];
    const int nrows = r1 - r0, cnt = k1 - k0;
    const int tr = min(t, max(nrows - 1, 0));
    const int a = A.rowptr[r0 + tr] - k0, e = A.rowptr[r0 + tr + 1] - k0;
    epi.pre(r0 + tr);
    T g0[U], g1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr ((V & 16) != 0) {  // ablation (timing only): no gathers
        g0[u] = T(c[u].x & 1);
        g1[u] = T(c[u].y & 1);
      } else {
        g0[u] = x(c[u].x);
        g1[u] = x(c[u].y);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    PV vn[U];
    Int2 cn[U];
    issue(nk0, nk1, vn, cn);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((V & 32) != 0) {  // ablation (timing only): no LDS / row phase
      T s = T(0);
#pragma unroll
      for (int u = 0; u < U; ++u) s += v[u].x * g0[u] + v[u].y * g1[u];
      if (t < nrows) epi.row(r0 + t, s);
    } else {
    {
      // branch-free: lanes outside [0, cnt) store into the scratch slots
      const int ka = k0 & ~1;
      const int lim = min(cnt, TL::cap);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int pos = 2 * (t + u * kBlock) + ka - k0;
        const int q0 = (pos >= 0 && pos < lim) ? pos : TL::tile;
        const int q1 = (pos + 1 >= 0 && pos + 1 < lim) ? pos + 1 : TL::tile + 1;
        sm.prod[q0] = v[u].x * g0[u];
        sm.prod[q1] = v[u].y * g1[u];
      }
    }
    if (cnt <= TL::cap) {
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
      for (int k = t; k < cnt; k += kBlock) s[0] += val[k0 + k] * x(A.col[k0 + k]);
      block_sum<T, 1>(s, sm.red);
      if (t == 0) epi.row(r0, s[0]);
      __syncthreads();
    }
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

template <typename T> struct QuadOf;
template <> struct QuadOf<double> { typedef double V __attribute__((ext_vector_type(4))); };
template <> struct QuadOf<float> { typedef float V __attribute__((ext_vector_type(4))); };
typedef int Int4 __attribute__((ext_vector_type(4)));

template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void spmv_rows_quad(const CsrArgs &A, const T *__restrict__ val,
                                               const Gather &x, Epi &epi,
                                               SpmvLds<T, TileOf<V>::tile> &sm) {
  using TL = TileOf<V>;
  constexpr bool NT = (V & 2) != 0;
  using QV = typename QuadOf<T>::V;
  constexpr int U = TL::tile / (4 * kBlock);
  constexpr int CAP = TL::tile - 6;  // quads read up to 6 extra entries
  const int t = threadIdx.x;
  int b, step, end;
  work_range<V>(A.nrb, b, step, end);
  if (b >= end) return;
  const int b0 = block_at(A, b);
  int r0 = A.rb[b0], r1 = A.rb[b0 + 1], k0 = A.rbk[b0], k1 = A.rbk[b0 + 1];
  QV v[U];
  Int4 c[U];
  auto issue = [&](int kk0, int kk1, QV(&vv)[U], Int4(&cc)[U]) {
    const bool ok = kk1 > kk0;  // empty blocks read quad [0, 4) (nnz >= 4)
    const int ka = ok ? (kk0 & ~3) : 0;
    const int nq = ok ? ((kk1 - ka + 3) >> 2) : 1;
    const QV *v4 = reinterpret_cast<const QV *>(val + ka);
    const Int4 *c4 = reinterpret_cast<const Int4 *>(A.col + ka);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = min(t + u * kBlock, nq - 1);
      vv[u] = ldg<NT>(v4 + j);
      Int4 q = ldg<NT>(c4 + j);
      const int e0 = ka + 4 * j;  // see tail_cols
      if (e0 + 1 >= kk1) q.y = q.x;
      if (e0 + 2 >= kk1) q.z = q.x;
      if (e0 + 3 >= kk1) q.w = q.x;
      cc[u] = q;
    }
  };
  issue(k0, k1, v, c);
  for (;;) {
    const int nb = b + step;
    const bool has_next = nb < end;
    const int nbb = block_at(A, has_next ? nb : b);
    const int nr0 = A.rb[nbb], nr1 = A.rb[nbb + 1], nk0 = A.rbk[nbb], nk1 = A.rbk[nbb + 1];
    const int nrows = r1 - r0, cnt = k1 - k0;
    const int tr = min(t, max(nrows - 1, 0));
    const int rpt = A.rowptr[r0 + tr];
    epi.pre(r0 + tr);
    T g[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      g[u][0] = x(c[u].x);
      g[u][1] = x(c[u].y);
      g[u][2] = x(c[u].z);
      g[u][3] = x(c[u].w);
    }
    __builtin_amdgcn_sched_barrier(0);
    QV vn[U];
    Int4 cn[U];
    issue(nk0, nk1, vn, cn);
    __builtin_amdgcn_sched_barrier(0);
    {
      const int ka = k0 & ~3;
      const int lim = min(cnt, CAP);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int pos = 4 * (t + u * kBlock) + ka - k0;
        const T vq[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int pq = pos + q;
          const int dst = (pq >= 0 && pq < lim) ? pq : TL::tile + q;
          sm.prod[dst] = vq[q] * g[u][q];
        }
      }
      if (t < nrows) sm.rp[t] = rpt;
      if (t == 0) sm.rp[nrows] = k1;
    }
    if (cnt <= CAP) {
      __syncthreads();
      if (t < nrows) {
        const int a = sm.rp[t] - k0, e = sm.rp[t + 1] - k0;
        T s = T(0);
        for (int j = a; j < e; ++j) s += sm.prod[j];
        epi.row(r0 + t, s);
      }
      __syncthreads();
    } else {
      // one row longer than a tile
      __syncthreads();
      T s[1] = {T(0)};
      for (int k = t; k < cnt; k += kBlock) s[0] += val[k0 + k] * x(A.col[k0 + k]);
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

// ---------------------------------------------------------------------------
// SELL-64 SpMV (variant bit 2048; layout: cgx_internal.h SellSlice). One
// wave per 64-row slice, lane l owns row 64 s + l and sums its entries in
// ascending order in a register, so the row sums are bit-identical to the
// CSR-stream forms (and to CG.hpp's SpMV) with no LDS staging and no rowptr
// reads. A column is row + dict[k]: the slice's offset dictionary sits in
// one VGPR (lane i holds entry i) and ds_bpermute fetches entry k, so the
// index stream is 1 B per entry instead of 4 (9 B/entry in f64 instead of
// 12). XCD split as variant bit 1: the waves of one XCD walk a contiguous
// slice range, consecutive slices on the waves of one workgroup.
// Bit 2: non-temporal value/index loads. Bit 16 (timing ablation, spmv_dot
// only): no gathers.
// ---------------------------------------------------------------------------
template <typename T> struct SellLds {
  T vdict[kVcDict];  // value-code dictionary (variant bit 32768)
  unsigned long long vt[kVtMax * 64];  // value-code templates (variant bit kVT)
  T red[4 * kMaxRed];
  int flag;
  int rp[1];  // unused (keeps the SpmvLds member set)
};

// The waves of one XCD walk a contiguous slice range (as variant bit 1);
// consecutive slices on the waves of one workgroup. Slice indices fit int
// (n < 2^31), which keeps the loop control on the scalar unit.
__device__ __forceinline__ void sell_range(int nsl, int wg0, int &first, int &step, int &end,
                                           int &lo) {
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = (int)gridDim.x - wg0, b = (int)blockIdx.x - wg0;
  if ((G & 7) == 0) {
    const int g = b & 7;
    lo = (int)(((int64_t)nsl * g) >> 3);
    first = lo + (b >> 3) * 4 + wid;
    end = (int)(((int64_t)nsl * (g + 1)) >> 3);
    step = (G >> 3) * 4;
  } else {
    lo = 0;
    first = b * 4 + wid;
    end = nsl;
    step = G * 4;
  }
}

// One slice, any width. Every load is unconditional (no branches around
// them, so the in-order vmcnt wait before the gathers covers the index word
// only): slots past the slice width re-read the last slot (same lines: no
// new L2 requests) and padding entries gather the row's own x (clamped to
// the last row) and are dropped at the add.
template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void sell_slice(const CsrArgs &A, const Gather &x, Epi &epi, int s) {
  constexpr bool NT = (V & 2) != 0;
  const T *__restrict__ sval = static_cast<const T *>(A.sval);
  const int lane = threadIdx.x & 63;
  const SellSlice m = A.sl[s];
  const int row = s * kSellRows + lane;
  const bool live = row < A.n;
  const int rowc = live ? row : (int)A.n - 1;
  epi.pre(rowc);
  const int dv = A.sdict[m.dict + lane];
  T acc = T(0);
  for (int c = 0; c < m.width; c += 8) {
    const unsigned long long iw =
        ldg<NT>(A.sidx + m.ioff + (int64_t)(c >> 3) * kSellRows + lane);
    const T *vp = sval + m.voff + (int64_t)c * kSellRows + lane;
    T v[8], g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ldg<NT>(vp + min(j, m.width - 1 - c) * kSellRows);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned k = (unsigned)(iw >> (8 * j)) & 0xffu;
      const int off = __builtin_amdgcn_ds_bpermute((int)(k << 2), dv);
      if constexpr ((V & 16) != 0) g[j] = T(k & 1);
      else g[j] = x(k != kSellPad ? row + off : rowc);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned k = (unsigned)(iw >> (8 * j)) & 0xffu;
      const T t = acc + v[j] * g[j];
      acc = (k != kSellPad) ? t : acc;
    }
  }
  if (live) epi.row(row, acc);
}

// The k-th slice to visit: A.sorder[k] where the host built a visit order
// (cgx_abi.cpp sell_visit_order), else k. Wave-uniform scalar load.
__device__ __forceinline__ int slice_at(const CsrArgs &A, int k) {
  if (!A.sorder) return k;
  return ((const __attribute__((address_space(4))) int *)A.sorder)
      [__builtin_amdgcn_readfirstlane(k)];
}

template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void spmv_sell(const CsrArgs &A, const Gather &x, Epi &epi) {
  int s, step, end, lo;
  sell_range((int)A.nsl, A.wg0, s, step, end, lo);
  for (; s < end; s += step)
    sell_slice<T, V, Epi, Gather>(A, x, epi, slice_at(A, A.rev ? lo + end - 1 - s : s));
}

// Software-pipelined SELL (variant bits 2048 | 8; matrices whose slices are
// at most 8 wide, one index word per row): while slice s gathers x and sums
// its rows, the values, index word and dictionary of the wave's next slice
// are in flight, so the HBM latency of the stream is off the slice's
// critical path. Same sums, same order as spmv_sell. The loop runs over full
// slices only (every lane a live row, so nothing is predicated and nothing
// can be sunk past the prefetch); a partial last slice takes sell_slice.
template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void spmv_sell_pipe(const CsrArgs &A, const Gather &x, Epi &epi) {
  constexpr bool NT = (V & 2) != 0;
  const T *__restrict__ sval = static_cast<const T *>(A.sval);
  const int lane = threadIdx.x & 63;
  int first, step, end, lo;
  sell_range((int)A.nsl, A.wg0, first, step, end, lo);
  const int full = (int)(A.n / kSellRows);  // slices whose 64 rows all exist
  const int pend = min(end, full);
  auto issue = [&](int q, unsigned long long &iw, T(&v)[8], int &dv) {
    // wave-uniform, read-only: a scalar load through the constant address
    // space (a vector load would need a vmcnt(0) wait, draining the gathers
    // in flight before the prefetch is issued)
    const auto *cs = (const __attribute__((address_space(4))) SellSlice *)A.sl;
    const int qi = __builtin_amdgcn_readfirstlane(q);
    const int64_t voff = cs[qi].voff, ioff = cs[qi].ioff;
    const int dict = cs[qi].dict, width = cs[qi].width;
    const T *vp = sval + voff + lane;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ldg<NT>(vp + min(j, width - 1) * kSellRows);
    iw = ldg<NT>(A.sidx + ioff + lane);
    dv = A.sdict[dict + lane];
  };
  int s = first;
  if (s < pend) {
    unsigned long long iw;
    T v[8];
    int dv;
    issue(s, iw, v, dv);
    for (;;) {
      const int ns = s + step;
      const bool has_next = ns < pend;
      const int row = s * kSellRows + lane;
      epi.pre(row);
      T g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned k = (unsigned)(iw >> (8 * j)) & 0xffu;
        const int off = __builtin_amdgcn_ds_bpermute((int)(k << 2), dv);
        if constexpr ((V & 16) != 0) g[j] = T(k & 1);
        else g[j] = x(k != kSellPad ? row + off : row);
      }
      __builtin_amdgcn_sched_barrier(0);
      unsigned long long iwn;
      T vn[8];
      int dvn;
      issue(has_next ? ns : s, iwn, vn, dvn);
      __builtin_amdgcn_sched_barrier(0);
      T acc = T(0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned k = (unsigned)(iw >> (8 * j)) & 0xffu;
        const T t = acc + v[j] * g[j];
        acc = (k != kSellPad) ? t : acc;
      }
      epi.row(row, acc);
      if (!has_next) break;
      iw = iwn;
      dv = dvn;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = vn[j];
      s = ns;
    }
    s += step;
  }
  // the partial last slice, if this wave owns it
  for (; s < end; s += step)
    if (s >= full) sell_slice<T, V, Epi, Gather>(A, x, epi, s);
}

// SELL with 2 rows per lane (variant bit 4096; slices of 128 rows): lane l
// owns rows 128 s + 2 l and + 1, so each value and index access is one
// 16-byte load (two rows' slot j, two rows' index word) — half the load
// instructions per row of the 1-row form, which streams at 8 bytes per lane.
// Same per-row sums in the same order. Gathers stay one 8-byte load per
// entry.
typedef unsigned long long Ull2 __attribute__((ext_vector_type(2)));
template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void sell_slice2(const CsrArgs &A, const Gather &x, Epi &epi, int s) {
  constexpr bool NT = (V & 2) != 0;
  using PV = typename PairOf<T>::V;
  const PV *__restrict__ sval = static_cast<const PV *>(A.sval);
  const Ull2 *__restrict__ sidx = reinterpret_cast<const Ull2 *>(A.sidx);
  const int lane = threadIdx.x & 63;
  const SellSlice m = A.sl[s];
  const int r0 = s * (2 * kSellRows) + 2 * lane;
  const bool l0 = r0 < A.n, l1 = r0 + 1 < A.n;
  const int rc0 = l0 ? r0 : (int)A.n - 1, rc1 = l1 ? r0 + 1 : (int)A.n - 1;
  epi.pre2(rc0, rc1);
  const int dv = A.sdict[m.dict + lane];
  T acc0 = T(0), acc1 = T(0);
  for (int c = 0; c < m.width; c += 8) {
    // voff and ioff are multiples of 128 entries / words: 16-byte aligned
    const Ull2 iw = ldg<NT>(sidx + (m.ioff >> 1) + (int64_t)(c >> 3) * kSellRows + lane);
    const PV *vp = sval + (m.voff >> 1) + (int64_t)c * kSellRows + lane;
    PV v[8];
    T g0[8], g1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ldg<NT>(vp + min(j, m.width - 1 - c) * kSellRows);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned k0 = (unsigned)(iw.x >> (8 * j)) & 0xffu;
      const unsigned k1 = (unsigned)(iw.y >> (8 * j)) & 0xffu;
      const int o0 = __builtin_amdgcn_ds_bpermute((int)(k0 << 2), dv);
      const int o1 = __builtin_amdgcn_ds_bpermute((int)(k1 << 2), dv);
      if constexpr ((V & 16) != 0) {
        g0[j] = T(k0 & 1);
        g1[j] = T(k1 & 1);
      } else {
        g0[j] = x(k0 != kSellPad ? r0 + o0 : rc0);
        g1[j] = x(k1 != kSellPad ? r0 + 1 + o1 : rc1);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned k0 = (unsigned)(iw.x >> (8 * j)) & 0xffu;
      const unsigned k1 = (unsigned)(iw.y >> (8 * j)) & 0xffu;
      const T t0 = acc0 + v[j].x * g0[j];
      const T t1 = acc1 + v[j].y * g1[j];
      acc0 = (k0 != kSellPad) ? t0 : acc0;
      acc1 = (k1 != kSellPad) ? t1 : acc1;
    }
  }
  epi.row2(r0, acc0, acc1, l0, l1);
}

template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void spmv_sell2(const CsrArgs &A, const Gather &x, Epi &epi) {
  int s, step, end, lo;
  sell_range((int)A.nsl, A.wg0, s, step, end, lo);
  for (; s < end; s += step)
    sell_slice2<T, V, Epi, Gather>(A, x, epi, slice_at(A, A.rev ? lo + end - 1 - s : s));
}

// SELL-P (variant bit 8192; 16384: u32 masks): the dictionary SELL layout
// with 2 rows per lane, but each slice stores its sorted offset pattern
// o_0 < ... < o_{W-1} once (read as scalars) and every row a mask of the
// slots it uses; values sit in pattern slots (zero where a row has no
// entry). Slot j of both rows of a lane gathers x[r0 + o_j] and
// x[r0 + 1 + o_j] as one unaligned pair load (clamped to the vector; a
// clamped end selects the other half). Rows sum their set slots in
// ascending offset order = their CSR order (columns strictly ascending,
// checked at build), so the sums are bit-identical. Index stream: one mask
// per row (1 or 4 bytes) instead of 8 bytes.
template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void sellp_slice2(const CsrArgs &A, const Gather &x, Epi &epi, int s) {
  constexpr bool NT = (V & 2) != 0;
  using PV = typename PairOf<T>::V;
  using MT = typename std::conditional<(V & 16384) != 0, unsigned, unsigned char>::type;
  const PV *__restrict__ sval = static_cast<const PV *>(A.sval);
  const MT *__restrict__ smask = static_cast<const MT *>(A.smask);
  const auto *cs = (const __attribute__((address_space(4))) SellSlice *)A.sl;
  const auto *pat = (const __attribute__((address_space(4))) int *)A.sdict;
  const int lane = threadIdx.x & 63;
  const int si = __builtin_amdgcn_readfirstlane(s);
  const int64_t voff = cs[si].voff;
  const int pbase = cs[si].dict, W = cs[si].width;
  const int r0 = si * (2 * kSellRows) + 2 * lane;
  const bool l0 = r0 < A.n, l1 = r0 + 1 < A.n;
  const int rc0 = l0 ? r0 : (int)A.n - 1, rc1 = l1 ? r0 + 1 : (int)A.n - 1;
  epi.pre2(rc0, rc1);
  // both rows' masks in one load (r0 even; rows past n: mask 0, array padded)
  using MT2 = typename std::conditional<(V & 16384) != 0, unsigned long long,
                                        unsigned short>::type;
  const MT2 mm = *reinterpret_cast<const MT2 *>(smask + r0);
  constexpr int MB = 8 * (int)sizeof(MT);
  const unsigned m0 = (unsigned)(mm & ((MT2(1) << (MB - 1) << 1) - 1)), m1 = (unsigned)(mm >> MB);
  const int nxm2 = (int)A.nx - 2;
  T acc0 = T(0), acc1 = T(0);
  for (int c = 0; c < W; c += 8) {
    const PV *vp = sval + (voff >> 1) + (int64_t)c * kSellRows + lane;
    PV v[8];
    T g0[8], g1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ldg<NT>(vp + min(j, W - 1 - c) * kSellRows);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = pat[pbase + min(c + j, W - 1)];
      const int base = r0 + o;
      const int cb = min(max(base, 0), nxm2);
      if constexpr ((V & 16) != 0) {
        g0[j] = T(cb & 1);
        g1[j] = T(cb & 2);
      } else {
        const auto g = x.pair(cb);
        g0[j] = base <= nxm2 ? g.x : g.y;
        g1[j] = base >= 0 ? g.y : g.x;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int b = c + j;
      const bool in = b < W;
      const T t0 = acc0 + v[j].x * g0[j];
      const T t1 = acc1 + v[j].y * g1[j];
      acc0 = (in && ((m0 >> (b & 31)) & 1u)) ? t0 : acc0;
      acc1 = (in && ((m1 >> (b & 31)) & 1u)) ? t1 : acc1;
    }
  }
  epi.row2(r0, acc0, acc1, l0, l1);
}

template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void spmv_sellp(const CsrArgs &A, const Gather &x, Epi &epi) {
  int s, step, end, lo;
  sell_range((int)A.nsl, A.wg0, s, step, end, lo);
  for (; s < end; s += step)
    sellp_slice2<T, V, Epi, Gather>(A, x, epi, slice_at(A, A.rev ? lo + end - 1 - s : s));
}

// SELL-P with value codes (variant bit 32768 | 8192): the SELL-P slice walk
// and pair gathers, but each slot's value comes from a 1-byte code into the
// matrix's value dictionary (in LDS) instead of an 8-byte value, and the
// code also says whether the row has an entry there (kVcAbsent), so no mask
// is read: the matrix stream is 8 B per row pair and chunk of 8 slots
// instead of 128 + 2. Decoding returns the stored value's exact bits, so the
// sums are the SELL-P sums, bit for bit.
template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void sellpv_slice2(const CsrArgs &A, const Gather &x, Epi &epi,
                                              const T *__restrict__ vd, int s,
                                              const unsigned long long *vt = nullptr) {
  constexpr bool NT = (V & 2) != 0;
  const Ull2 *__restrict__ codes = static_cast<const Ull2 *>(A.svc);
  const auto *cs = (const __attribute__((address_space(4))) SellSlice *)A.sl;
  const auto *pat = (const __attribute__((address_space(4))) int *)A.sdict;
  const int lane = threadIdx.x & 63;
  const int si = __builtin_amdgcn_readfirstlane(s);
  const int64_t coff = cs[si].ioff;
  // kVT: the template slice table's width carries the template id + 1 in
  // its high half (0: the slice streams its own chunk)
  const int wraw = cs[si].width, pbase = cs[si].dict, W = wraw & kVtWidthMask;
  const int tid = (wraw >> 16) - 1;
  const int r0 = si * (2 * kSellRows) + 2 * lane;
  const bool l0 = r0 < A.n, l1 = r0 + 1 < A.n;
  const int rc0 = l0 ? r0 : (int)A.n - 1, rc1 = l1 ? r0 + 1 : (int)A.n - 1;
  epi.pre2(rc0, rc1);
  const int nxm2 = (int)A.nx - 2;
  T acc0 = T(0), acc1 = T(0);
  // bit 131072: gather and sum the chunk in two halves of 4 slots (half the
  // registers in flight)
  constexpr int HS = (V & 131072) ? 4 : 8;
  constexpr bool C4 = (V & 262144) != 0;  // 4-bit codes: one 8-byte word per lane
  const unsigned long long *__restrict__ codes4 =
      static_cast<const unsigned long long *>(A.svc4);
  for (int c = 0; c < W; c += 8) {
    Ull2 cw;
    if constexpr (C4) {
      if constexpr ((V & kVT) != 0) {  // template slice (one chunk): from LDS
        cw.x = tid >= 0 ? vt[tid * 64 + lane]
                        : ldg<NT>(codes4 + coff + (int64_t)(c >> 3) * kSellRows + lane);
      } else {
        cw.x = ldg<NT>(codes4 + coff + (int64_t)(c >> 3) * kSellRows + lane);
      }
      cw.y = 0;
    } else {
      cw = ldg<NT>(codes + coff + (int64_t)(c >> 3) * kSellRows + lane);
    }
#pragma unroll
    for (int h = 0; h < 8; h += HS) {
    T g0[HS], g1[HS];
#pragma unroll
    for (int jj = 0; jj < HS; ++jj) {
      const int j = h + jj;
      const int o = pat[pbase + min(c + j, W - 1)];
      const int base = r0 + o;
      const int cb = min(max(base, 0), nxm2);
      if constexpr ((V & 16) != 0) {
        g0[jj] = T(cb & 1);
        g1[jj] = T(cb & 2);
      } else {
        const auto g = x.pair(cb);
        g0[jj] = base <= nxm2 ? g.x : g.y;
        g1[jj] = base >= 0 ? g.y : g.x;
      }
    }
#pragma unroll
    for (int jj = 0; jj < HS; ++jj) {
      const int j = h + jj;
      unsigned k0, k1;
      bool on0, on1;
      if constexpr (C4) {
        k0 = (unsigned)(cw.x >> (8 * j)) & 0xfu;
        k1 = (unsigned)(cw.x >> (8 * j + 4)) & 0xfu;
        on0 = k0 != 0xfu;
        on1 = k1 != 0xfu;
      } else {
        const unsigned long long w = j < 4 ? cw.x : cw.y;
        k0 = (unsigned)(w >> (16 * (j & 3))) & 0xffu;
        k1 = (unsigned)(w >> (16 * (j & 3) + 8)) & 0xffu;
        on0 = k0 != kVcAbsent;
        on1 = k1 != kVcAbsent;
      }
      const T t0 = acc0 + vd[k0] * g0[jj];
      const T t1 = acc1 + vd[k1] * g1[jj];
      acc0 = on0 ? t0 : acc0;
      acc1 = on1 ? t1 : acc1;
    }
    if constexpr (HS < 8) __builtin_amdgcn_sched_barrier(0);
    }
  }
  epi.row2(r0, acc0, acc1, l0, l1);
}

// Whole-wave lane shifts by one (DPP wave_shr:1 / wave_shl:1): lane l gets
// lane l - 1's (l + 1's) value; lane 0 (63), which has no source, keeps
// `edge`.
template <typename T> __device__ __forceinline__ T wave_shr1(T v, T edge);
template <typename T> __device__ __forceinline__ T wave_shl1(T v, T edge);
template <> __device__ __forceinline__ double wave_shr1(double v, double edge) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(edge), __double2loint(v), 0x138, 0xf,
                                             0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(edge), __double2hiint(v), 0x138, 0xf,
                                             0xf, false);
  return __hiloint2double(hi, lo);
}
template <> __device__ __forceinline__ double wave_shl1(double v, double edge) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(edge), __double2loint(v), 0x130, 0xf,
                                             0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(edge), __double2hiint(v), 0x130, 0xf,
                                             0xf, false);
  return __hiloint2double(hi, lo);
}
template <> __device__ __forceinline__ float wave_shr1(float v, float edge) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v),
                                                    0x138, 0xf, 0xf, false));
}
template <> __device__ __forceinline__ float wave_shl1(float v, float edge) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v),
                                                    0x130, 0xf, 0xf, false));
}

// Software-pipelined value-code SELL-P (variant bit 524288; every slice at
// most 8 wide, i.e. one code chunk): while slice s gathers and sums, the
// next slice's descriptor and offset pattern (a dependent pair of scalar
// loads) and its code word are in flight, so a slice's critical path is its
// own gathers. Same sums in the same order as sellpv_slice2.
template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void spmv_sellpv_pipe(const CsrArgs &A, const Gather &x, Epi &epi,
                                                 const T *__restrict__ vd,
                                                 const unsigned long long *vt) {
  constexpr bool NT = (V & 2) != 0;
  constexpr bool C4 = (V & 262144) != 0;
  constexpr bool CR = (V & 1048576) != 0;  // stencil slices: +-1 by lane shifts
  const auto *cs = (const __attribute__((address_space(4))) SellSlice *)A.sl;
  const auto *pat = (const __attribute__((address_space(4))) int *)A.sdict;
  const Ull2 *__restrict__ codes = static_cast<const Ull2 *>(A.svc);
  const unsigned long long *__restrict__ codes4 =
      static_cast<const unsigned long long *>(A.svc4);
  const int lane = threadIdx.x & 63;
  const int nxm2 = (int)A.nx - 2;
  int s, step, end, lo;
  sell_range((int)A.nsl, A.wg0, s, step, end, lo);
  if (s >= end) return;
  // tid: the slice's template (kVT; -1: it streams its own chunk)
  auto code_at = [&](int64_t coff, int tid) {
    Ull2 cw;
    if constexpr ((V & kVT) != 0) {
      // template slice (uniform): the chunk comes from LDS, no HBM read
      if (tid >= 0) {
        cw.x = vt[tid * 64 + lane];
        cw.y = 0;
        return cw;
      }
    }
    if constexpr (C4) {
      cw.x = ldg<NT>(codes4 + coff + lane);
      cw.y = 0;
    } else {
      cw = ldg<NT>(codes + coff + lane);
    }
    return cw;
  };
  int si = __builtin_amdgcn_readfirstlane(slice_at(A, A.rev ? lo + end - 1 - s : s));
  int W = cs[si].width & kVtWidthMask;
  int o[8];
  {
    const int pb = cs[si].dict;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = pat[pb + min(j, W - 1)];
  }
  Ull2 cwA = code_at(cs[si].ioff, (cs[si].width >> 16) - 1), cwB;
  // slice si is interior when the pairs of its lowest and highest offset
  // (o[0], o[7] = o[W-1]: the pattern is sorted) lie inside x for every
  // lane, dead lanes of a last partial slice included, and byte offsets
  // into x fit 32 bits
  const bool off32 = (uint64_t)A.nx * sizeof(T) < (uint64_t(1) << 32);
  auto inner_slice = [&](int sl, int omin, int omax) {
    const int fr = sl * (2 * kSellRows);
    return off32 && fr + omin >= 0 && fr + 2 * kSellRows - 2 + omax <= nxm2;
  };
  // one slice; the code word rotates by argument, never by copy (a copy of
  // a register whose load is in flight waits for it, and at the loop's
  // back edge that wait also drained the Ap store: the prefetch never
  // overlapped anything). The loop below runs it twice per trip.
  auto body = [&](const Ull2 &cw, Ull2 &cwn) -> bool {
    const int ns = s + step;
    const bool has_next = ns < end;
    const int nk = has_next ? ns : s;
    const int sn = __builtin_amdgcn_readfirstlane(slice_at(A, A.rev ? lo + end - 1 - nk : nk));
    const int wrn = cs[sn].width, pbn = cs[sn].dict;
    const int Wn = wrn & kVtWidthMask;
    const int64_t coffn = cs[sn].ioff;
    const int r0 = si * (2 * kSellRows) + 2 * lane;
    const bool l0 = r0 < A.n, l1 = r0 + 1 < A.n;
    const int rc0 = l0 ? r0 : (int)A.n - 1, rc1 = l1 ? r0 + 1 : (int)A.n - 1;
    T g0[8], g1[8];
    const bool inner = inner_slice(si, o[0], o[7]);
    // stencil slices (bit 1048576): offsets -1, 0, +1 in slots K..K+2 of a
    // WW-wide pattern (K = 2, WW = 7: the 3-D 7-point interior; K = 1,
    // WW = 5: 2-D 5-point). The center pair x[r0], x[r0 + 1] is one aligned
    // load (and the dot's p); x[r0 - 1] and x[r0 + 2] come from the
    // neighbour lanes (DPP wave shifts), the slice's outer two, x[first - 1]
    // and x[first + 128], from scalar loads: three vector loads fewer per
    // slice. Every vector load is issued before the shifts wait.
    auto near = [&](auto kc, auto wc) {
      constexpr int K = decltype(kc)::value, WW = decltype(wc)::value;
      const unsigned rb = (unsigned)r0 * (unsigned)sizeof(T);
      const auto c = x.pair_b(rb);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j < K || (j > K + 2 && j < WW)) {
          const auto g = x.pair_b(rb + (unsigned)o[j] * (unsigned)sizeof(T));
          g0[j] = g.x;
          g1[j] = g.y;
        } else if (j >= WW) {
          g0[j] = g1[j] = T(0);
        }
      }
      const int fr = si * (2 * kSellRows);
      const T elo = x.at_s(fr - 1), ehi = x.at_s(fr + 2 * kSellRows);
      __builtin_amdgcn_sched_barrier(0);
      const T left = wave_shr1(c.y, elo), right = wave_shl1(c.x, ehi);
      g0[K] = left;
      g1[K] = c.x;
      g0[K + 1] = c.x;
      g1[K + 1] = c.y;
      g0[K + 2] = c.y;
      g1[K + 2] = right;
      epi.pre2c(rc0, rc1, c.x, c.y);
    };
    if (CR && inner && W == 7 && o[2] == -1 && o[3] == 0 && o[4] == 1) {
      near(std::integral_constant<int, 2>{}, std::integral_constant<int, 7>{});
    } else if (CR && inner && W == 5 && o[1] == -1 && o[2] == 0 && o[3] == 1) {
      near(std::integral_constant<int, 1>{}, std::integral_constant<int, 5>{});
    } else if (inner) {
      // interior slice (uniform): every pair lies inside x, so no clamps and
      // no end selects; the address is one 32-bit add to a scalar base
      epi.pre2(rc0, rc1);
      const unsigned rb = (unsigned)r0 * (unsigned)sizeof(T);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr ((V & 16) != 0) {
          g0[j] = T(rb & 1);
          g1[j] = T(rb & 2);
        } else {
          const auto g = x.pair_b(rb + (unsigned)o[j] * (unsigned)sizeof(T));
          g0[j] = g.x;
          g1[j] = g.y;
        }
      }
    } else {
      epi.pre2(rc0, rc1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int base = r0 + o[j];
        const int cb = min(max(base, 0), nxm2);
        if constexpr ((V & 16) != 0) {
          g0[j] = T(cb & 1);
          g1[j] = T(cb & 2);
        } else {
          const auto g = x.pair(cb);
          g0[j] = base <= nxm2 ? g.x : g.y;
          g1[j] = base >= 0 ? g.y : g.x;
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    int on[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) on[j] = pat[pbn + min(j, Wn - 1)];
    cwn = code_at(coffn, (wrn >> 16) - 1);
    __builtin_amdgcn_sched_barrier(0);
    T acc0 = T(0), acc1 = T(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      unsigned k0, k1;
      bool on0, on1;
      if constexpr (C4) {
        k0 = (unsigned)(cw.x >> (8 * j)) & 0xfu;
        k1 = (unsigned)(cw.x >> (8 * j + 4)) & 0xfu;
        on0 = k0 != 0xfu;
        on1 = k1 != 0xfu;
      } else {
        const unsigned long long w = j < 4 ? cw.x : cw.y;
        k0 = (unsigned)(w >> (16 * (j & 3))) & 0xffu;
        k1 = (unsigned)(w >> (16 * (j & 3) + 8)) & 0xffu;
        on0 = k0 != kVcAbsent;
        on1 = k1 != kVcAbsent;
      }
      const T t0 = acc0 + vd[k0] * g0[j];
      const T t1 = acc1 + vd[k1] * g1[j];
      acc0 = on0 ? t0 : acc0;
      acc1 = on1 ? t1 : acc1;
    }
    epi.row2(r0, acc0, acc1, l0, l1);
    if (!has_next) return false;
    si = sn;
    W = Wn;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = on[j];
    s = ns;
    return true;
  };
  while (body(cwA, cwB) && body(cwB, cwA)) {
  }
}

// Plane march (variant bit 2097152, on the pipelined stencil form 1875968):
// for a matrix whose dominant slice pattern is {-D, -a, -1, 0, +1, +a, +D}
// (3-D 7-point: a = nx, D = nx ny) or {-D, -1, 0, +1, +D} (2-D 5-point:
// D = nx) with D a multiple of the 128-row slice (D = 128 K), a wave walks
// the slices c, c + K, c + 2K, ... of one column through a run of L planes
// instead of consecutive slices. The x pairs at -D and +D of slice s are the
// center pairs of the slices before and after it in the walk, already in
// registers: no gathers. In the consecutive walk each x line is fetched as
// the center, and again as the +D and -D gathers of slices a plane away,
// after 1-3 MB of other traffic passed the XCD's L2. Here it is fetched
// once as a center (plus one extra center per end of a run), so only the
// +-a gathers (the same plane, neighbouring columns walked in step by the
// neighbouring waves) go to L2. Per slice: code word, center pair of
// s + 2K, +-a gathers, one edge load (lane 0: x[first - 1], lane 63:
// x[first + 128], the DPP shifts' fill values), the Ap store; the loads of
// slice s + K are issued before slice s sums. The per-row sums run in the
// same slot order as every SELL-P form, so Ap is bit-identical.
// Slices that are not of the march pattern (boundary planes and lines, the
// ragged end) run sellpv_slice2. Work items are (run z, column c), z-major,
// split over the XCDs like slices (sell_range); L from A.ml or, when 0, so
// that the items about fill the grid's waves. Needs every slice <= 8 wide
// (one code chunk per slice: slice s's codes at chunk s).
template <typename T, int V, bool S3, class Epi, class Gather>
__device__ __forceinline__ void spmv_sellpv_march(const CsrArgs &A, const Gather &x, Epi &epi,
                                                  const T *__restrict__ vd,
                                                  const unsigned long long *vt) {
  constexpr bool NT = (V & 2) != 0;
  constexpr bool C4 = (V & 262144) != 0;
  constexpr int H = 2 * kSellRows;
  using PV = typename PairU<T>::V;
  const Ull2 *__restrict__ codes = static_cast<const Ull2 *>(A.svc);
  const unsigned long long *__restrict__ codes4 =
      static_cast<const unsigned long long *>(A.svc4);
  const int lane = threadIdx.x & 63;
  const int K = A.mk, nsl = (int)A.nsl;
  const int nfull = (int)(A.n / H);  // slices whose 128 rows all exist
  const int a = A.mo;  // the +-a slots of the 3-D form
  constexpr int W7 = S3 ? 7 : 5;
  const int nxm2 = (int)A.nx - 2;
  const int planes = (nsl + K - 1) / K;
  int L = A.ml;
  if (L <= 0) {
    const int zc = max(1, (int)gridDim.x * (kBlock / 64) / K);
    L = (planes + zc - 1) / zc;
  }
  const int Z = (planes + L - 1) / L;
  // byte offsets into x fit 32 bits (else every slice takes sellpv_slice2)
  const bool off32 = (uint64_t)A.nx * sizeof(T) < (uint64_t(1) << 32);
  int it, step, end, lo;
  sell_range(K * Z, A.wg0, it, step, end, lo);
  // tid: the slice's template (kVT; -1: it streams its own chunk)
  auto code_at = [&](int sl, int tid) {
    Ull2 cw;
    if constexpr ((V & kVT) != 0) {
      if (tid >= 0) {
        cw.x = vt[tid * 64 + lane];
        cw.y = 0;
        return cw;
      }
    }
    if constexpr (C4) {
      cw.x = ldg<NT>(codes4 + (int64_t)sl * kSellRows + lane);
      cw.y = 0;
    } else {
      cw = ldg<NT>(codes + (int64_t)sl * kSellRows + lane);
    }
    return cw;
  };
  auto center = [&](int sl) { return x.pair(min(sl * H + 2 * lane, nxm2)); };
  // slice descriptors (dict, width) by VECTOR loads: a scalar load in the
  // loop would make every LDS dictionary read wait for it (SMEM returns out
  // of order, so any LDS use waits lgkmcnt(0)); `zv` is an opaque zero that
  // keeps the address divergent to the compiler
  int zv;
  asm volatile("v_mov_b32 %0, 0" : "=v"(zv));
  const Int2 *__restrict__ cdw = reinterpret_cast<const Int2 *>(
      reinterpret_cast<const char *>(A.sl) + offsetof(SellSlice, dict));
  using Desc = Int2;
  auto desc = [&](int sl) { return cdw[(int64_t)sl * (sizeof(SellSlice) / sizeof(Int2)) + zv]; };
  // the slice's template (kVT: the width's high half; -1: none)
  auto dio = [&](const Desc &d) {
    if constexpr ((V & kVT) != 0) return (__builtin_amdgcn_readfirstlane(d.y) >> 16) - 1;
    else return -1;
  };
  auto uni = [](int v) { return __builtin_amdgcn_readfirstlane(v); };
  // slice sl walks the march pattern: its descriptor names the pattern, its
  // +-D neighbours exist (whole slices of rows), every pair lies inside x
  auto fast = [&](int sl, int dict, int w) {
    return off32 && dict == A.mpat && (w & kVtWidthMask) == W7 && sl >= K && sl + K < nfull;
  };
  for (; it < end; it += step) {
    const int z = it / K, c = it - z * K;
    int s = c + z * L * K;
    if (s >= nsl) continue;
    const int last = min(c + ((z + 1) * L - 1) * K, c + (nsl - 1 - c) / K * K);
    // every load is issued, at safe addresses for a slice that is not fast
    // (a fixed load count keeps the compiler's in-order vmcnt waits exact)
    struct Batch {
      Ull2 cw;
      PV gm, gp;
      T edge;
    };
    auto issue = [&](int sl, bool fs, int io, Batch &b) {
      b.cw = code_at(sl, io);
      const int fr = sl * H;
      const unsigned rb = (unsigned)min(fr + 2 * lane, nxm2) * (unsigned)sizeof(T);
      if constexpr (S3 && (V & 16) != 0) {
        // bit 16 (timing ablation, spmv_dot only): no +-a gathers at all
        b.gm.x = b.gm.y = b.gp.x = b.gp.y = T(rb & 1);
      } else if constexpr (S3) {
        const unsigned ab = fs ? (unsigned)a * (unsigned)sizeof(T) : 0u;
        b.gm = x.pair_b(rb - ab);
        b.gp = x.pair_b(rb + ab);
      }
      b.edge = x(fs ? (lane == 63 ? fr + H : fr - 1) : fr);
    };
    // slice s from its batch and the center pairs of s - K, s, s + K
    auto sum = [&](int s, bool f, const Batch &b, const PV &cprev, const PV &ccur,
                   const PV &cnext) {
      if (f) {
        const int r0 = s * H + 2 * lane;
        T g0[8], g1[8];
        const T left = wave_shr1(ccur.y, b.edge), right = wave_shl1(ccur.x, b.edge);
        constexpr int K1 = S3 ? 2 : 1;  // slot of offset -1
        // slots 0 / 6 (-D, +D) from the walk, 1 / 5 (-a, +a) gathered (a
        // y-march, +-nx from the walk and +-nx ny gathered, measured
        // 93-124 against 72 us at 256^3 in round 3: removed)
        constexpr int JM = 0, JG = 1;
        g0[JM] = cprev.x;
        g1[JM] = cprev.y;
        if constexpr (S3) {
          g0[JG] = b.gm.x;
          g1[JG] = b.gm.y;
          g0[6 - JG] = b.gp.x;
          g1[6 - JG] = b.gp.y;
        }
        g0[K1] = left;
        g1[K1] = ccur.x;
        g0[K1 + 1] = ccur.x;
        g1[K1 + 1] = ccur.y;
        g0[K1 + 2] = ccur.y;
        g1[K1 + 2] = right;
        g0[W7 - 1 - JM] = cnext.x;
        g1[W7 - 1 - JM] = cnext.y;
        epi.pre2c(r0, r0 + 1, ccur.x, ccur.y);
        T acc0 = T(0), acc1 = T(0);
#pragma unroll
        for (int j = 0; j < W7; ++j) {
          unsigned k0, k1;
          bool on0, on1;
          if constexpr (C4) {
            k0 = (unsigned)(b.cw.x >> (8 * j)) & 0xfu;
            k1 = (unsigned)(b.cw.x >> (8 * j + 4)) & 0xfu;
            on0 = k0 != 0xfu;
            on1 = k1 != 0xfu;
          } else {
            const unsigned long long w = j < 4 ? b.cw.x : b.cw.y;
            k0 = (unsigned)(w >> (16 * (j & 3))) & 0xffu;
            k1 = (unsigned)(w >> (16 * (j & 3) + 8)) & 0xffu;
            on0 = k0 != kVcAbsent;
            on1 = k1 != kVcAbsent;
          }
          const T t0 = acc0 + vd[k0] * g0[j];
          const T t1 = acc1 + vd[k1] * g1[j];
          acc0 = on0 ? t0 : acc0;
          acc1 = on1 ? t1 : acc1;
        }
        epi.row2(r0, acc0, acc1, true, true);
      } else {
        sellpv_slice2<T, V, Epi, Gather>(A, x, epi, vd, s, vt);
        // drain: this path's load count is not fixed (a loop over code
        // chunks); a merge with an unknown count would make the compiler
        // wait vmcnt(0) before the next descriptor on every step
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt/lgkmcnt untouched
      }
    };
    // one step: the next slice's descriptor decides its batch; issue that
    // batch, the descriptor after it and the center two planes on; then sum
    // slice s (whose loads were issued one step earlier). Buffers rotate by
    // argument, never by copy: a copy of a register whose load is in flight
    // waits for it (the loop below is unrolled four times so every role
    // returns to its register).
    auto stepf = [&](int &s, bool &f, const Desc &dcur, Desc &dnew, const Batch &bc, Batch &bn,
                     const PV &cm, const PV &c0, const PV &cp, PV &cnn) {
      const int sn = s + K;
      const bool has_next = sn <= last;
      const bool fn = has_next && fast(sn, uni(dcur.x), uni(dcur.y));
      __builtin_amdgcn_sched_barrier(0);
      const int snk = has_next ? sn : s;
      const int snn = min(snk + K, nsl - 1);
      dnew = desc(snn);
      issue(snk, fn, dio(dcur), bn);
      cnn = center(snn);
      __builtin_amdgcn_sched_barrier(0);
      sum(s, f, bc, cm, c0, cp);
      s = sn;
      f = fn;
      return has_next;
    };
    // prologue: slice s's batch, the centers of s - K, s, s + K, the
    // descriptor of s + K
    // descriptor of s + K (the first step's) early: the first step waits
    // for it, and so for every load issued before it
    const Desc d0 = desc(s);
    Desc dA = desc(min(s + K, nsl - 1)), dB;
    PV c0 = center(max(s - K, 0)), c1 = center(s), c2, c3;
    bool f = fast(s, uni(d0.x), uni(d0.y));
    Batch bA, bB;
    issue(s, f, dio(d0), bA);
    c2 = center(min(s + K, nsl - 1));
    for (;;) {
      if (!stepf(s, f, dA, dB, bA, bB, c0, c1, c2, c3)) break;
      if (!stepf(s, f, dB, dA, bB, bA, c1, c2, c3, c0)) break;
      if (!stepf(s, f, dA, dB, bA, bB, c2, c3, c0, c1)) break;
      if (!stepf(s, f, dB, dA, bB, bA, c3, c0, c1, c2)) break;
    }
  }
}

template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void spmv_sellpv(const CsrArgs &A, const Gather &x, Epi &epi,
                                            T *vd, unsigned long long *vt) {
  const T *__restrict__ src = static_cast<const T *>(A.svdict);
  for (int i = threadIdx.x; i < kVcDict; i += kBlock) vd[i] = src[i];
  if constexpr ((V & kVT) != 0)  // the value-code templates next to the dictionary
    for (int i = threadIdx.x; i < A.nvt * 64; i += kBlock) vt[i] = A.vct[i];
  __syncthreads();
  if constexpr ((V & 2097152) != 0) {
    if (A.mk > 0) {
      if (A.mo > 0) spmv_sellpv_march<T, V, true, Epi, Gather>(A, x, epi, vd, vt);
      else spmv_sellpv_march<T, V, false, Epi, Gather>(A, x, epi, vd, vt);
      return;
    }
  }
  if constexpr ((V & 524288) != 0) {
    spmv_sellpv_pipe<T, V, Epi, Gather>(A, x, epi, vd, vt);
    return;
  }
  int s, step, end, lo;
  sell_range((int)A.nsl, A.wg0, s, step, end, lo);
  for (; s < end; s += step)
    sellpv_slice2<T, V, Epi, Gather>(A, x, epi, vd,
                                     slice_at(A, A.rev ? lo + end - 1 - s : s), vt);
}


// Lean stencil walk (kVL; cgx_internal.h, DESIGN.md §4 "lean stencil walk").
// The launch's grid G (a multiple of 8) is the one the class bytes were laid
// out for; the waves of XCD group g walk its eighth of the slices with
// step G / 2, like sell_range, so with G / 2 equal to the slices of a plane
// (D = 128 G / 2 rows) a wave's +-D gathers are the lines it loads as its
// own centers one step before and after, still in its XCD's L2
// (tools/probes/stencil_floor.hip: 42 us at 256^3 with G = 1024 against 61
// with G = 2048). A lean slice (class byte c < 0xff) issues its center pair,
// its present +-D / +-a pairs (an absent slot re-reads the center, an L1
// hit, and is not added) and the scalar edges x[first - 1], x[first + 128]
// at once, waits once, takes +-1 from the neighbour lanes (DPP) and sums
// both rows in the canonical slot order, which is their CSR order: Ap is the
// per-row loop's, bit for bit. Its values come from the class table (scalar
// loads that hit the constant cache): no code word, no dictionary read, no
// per-slot select. Other slices (boundary lines and planes of another
// pattern, chunks no template matched) run sellpv_slice2 on the template
// value codes. The class bytes of 256 steps come in one dword per lane and
// are read with v_readlane: no scalar load per slice waits on the memory
// behind the constant cache.
// the select-free interior path of the lean walk (37.3 against 38.5 us for
// mode 6's p.Ap walk at 256^3 without it, profiles/r6t_*)
constexpr bool LEAN_FULL = true;
template <typename T, class Epi, class Gather>
__device__ __forceinline__ void spmv_lean(const CsrArgs &A, const Gather &x, Epi &epi,
                                          const T *__restrict__ vd,
                                          const unsigned long long *vt) {
  constexpr int VG = 8192 | 32768 | 262144 | 524288 | kVT | 2;  // the generic slices' form
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // (the first A.wg0 workgroups of a launch with the halo push do that
  // instead; a multiple of 8, so the XCD groups stay)
  const int G = (int)gridDim.x - A.wg0, b = (int)blockIdx.x - A.wg0, g = b & 7;
  const int step = (G >> 3) * 4, w = (b >> 3) * 4 + wid;
  const int nsl = (int)A.nsl;
  const int lo = (int)(((int64_t)nsl * g) >> 3), end = (int)(((int64_t)nsl * (g + 1)) >> 3);
  // rows of the reversed sweep (A.rev: slice lo + end - 1 - s at walk
  // position s, as sell_range's walkers) follow the forward ones
  const unsigned *__restrict__ row = reinterpret_cast<const unsigned *>(
      A.vl_cls + (int64_t)((A.rev ? 8 * step : 0) + g * step + w) * A.vl_nst);
  const int nw = A.vl_nst >> 2;  // class words of this wave's row
  const auto *tab = (const __attribute__((address_space(4))) VlClass *)A.vl_tab;
  const unsigned oD = (unsigned)A.vl_D * (unsigned)sizeof(T);
  const unsigned oa = (unsigned)A.vl_a * (unsigned)sizeof(T);
  unsigned cw = 0;
  // the chunked walk (A.vl_P > 0; cgx_abi.cpp build_lean_layout): the
  // group's eighth is P whole planes of K slices and step divides K; wave w
  // walks chunk position w of chunk c through the P planes, chunk after
  // chunk, so its +-D neighbours are its own centers one step away also
  // when a plane is wider than the group's waves (512^3)
  const int P = A.vl_P, K = A.vl_K;
  int zp = 0, cb = 0;  // plane and chunk base of the chunked walk's step
  auto next = [&](int s) {
    if (P == 0) return s + step;
    if (++zp == P) {
      zp = 0;
      cb += step;
    }
    return cb >= K ? end : lo + zp * K + cb + w;
  };
  const int D = A.vl_D, a = A.vl_a;
  const int nxi = (int)A.nx;
  // the +-D carry: when the wave's next slice is the one a plane on (walk
  // position s + Kp: the plane-matched step, or the chunked walk inside a
  // chunk), the pair this slice gathers a plane ahead is that slice's center
  // and this slice's center is its pair a plane behind, so neither is loaded
  // again (in the reversed sweep "ahead" is -D)
  const int Kp = D / (2 * kSellRows);
  const bool carry_walk = D % (2 * kSellRows) == 0 && (P > 0 ? K == Kp : step == Kp);
  using PV = decltype(x.pair_b(0u));
  PV c_ahead, c_ct;
  int carry_s = -1;  // the walk position the carried pairs belong to
  for (int s = lo + w, j = 0; s < end; s = next(s), ++j) {
    if ((j & 255) == 0) {  // the classes of the next 256 steps, lane l: steps 4l .. 4l + 3
      const int k = (j >> 2) + lane;
      cw = k < nw ? row[k] : ~0u;
      // waited for here (an asm use), and from here on a plain register: the
      // loop's other iterations do not wait on the memory counter for it
      // (which would also drain the previous slice's Ap store)
      asm volatile("" : "+v"(cw));
    }
    const unsigned word = (unsigned)__builtin_amdgcn_readlane((int)cw, (j & 255) >> 2);
    const int c = (int)((word >> (8 * (j & 3))) & 0xffu);
    const int si = A.rev ? lo + end - 1 - s : s;
    if (c == 0xfe) continue;  // a partitioned matrix's boundary slice: the boundary launch's
    if (c == 0xff) {
      sellpv_slice2<T, VG, Epi, Gather>(A, x, epi, vd, si, vt);
      continue;
    }
    // every load of the slice at once, none of them waiting on another: the
    // gathers' addresses follow the slice's position (in bounds, else the
    // center), not its class, whose presence bits only select the adds
    const int fr = si * (2 * kSellRows);
    const T elo = x.at_s(fr > 0 ? fr - 1 : 0);
    const T ehi = x.at_s(fr + 2 * kSellRows < nxi ? fr + 2 * kSellRows : nxi - 1);
    const int r0 = fr + 2 * lane;
    const unsigned rb = (unsigned)r0 * (unsigned)sizeof(T);
    const unsigned omD = rb - (fr >= D ? oD : 0u);
    const unsigned opD = rb + (fr + 2 * kSellRows + D <= nxi ? oD : 0u);
    PV ct, behind;
    if (s == carry_s) {
      ct = c_ahead;
      behind = c_ct;
    } else {
      ct = x.pair_b(rb);
      behind = x.pair_b(A.rev ? opD : omD);
    }
    const PV ahead = x.pair_b(A.rev ? omD : opD);
    const auto gma = x.pair_b(rb - (a > 0 && fr >= a ? oa : 0u));
    const auto gpa = x.pair_b(rb + (a > 0 && fr + 2 * kSellRows + a <= nxi ? oa : 0u));
    const PV gmD = A.rev ? ahead : behind;
    const PV gpD = A.rev ? behind : ahead;
    c_ahead = ahead;
    c_ct = ct;
    carry_s = carry_walk ? s + Kp : -1;
    const int pres = tab[c].pres;
    T v[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) v[q] = T(tab[c].v[q]);
    // an absent x-line end: v * (-copysign(0, v)) = -0.0, the identity of +
    const T lo_e = tab[c].plo ? elo : -__builtin_copysign(T(0), v[2]);
    const T hi_e = tab[c].phi ? ehi : -__builtin_copysign(T(0), v[4]);
    const T left = wave_shr1(ct.y, lo_e), right = wave_shl1(ct.x, hi_e);
    epi.pre2c(r0, r0 + 1, ct.x, ct.y);
    T a0 = T(0), a1 = T(0);
    if (LEAN_FULL && pres == 15) {  // every slot present (the interior): no select
      a0 = a0 + v[0] * gmD.x;
      a1 = a1 + v[0] * gmD.y;
      a0 = a0 + v[1] * gma.x;
      a1 = a1 + v[1] * gma.y;
      a0 = a0 + v[2] * left;
      a1 = a1 + v[2] * ct.x;
      a0 = a0 + v[3] * ct.x;
      a1 = a1 + v[3] * ct.y;
      a0 = a0 + v[4] * ct.y;
      a1 = a1 + v[4] * right;
      a0 = a0 + v[5] * gpa.x;
      a1 = a1 + v[5] * gpa.y;
      a0 = a0 + v[6] * gpD.x;
      a1 = a1 + v[6] * gpD.y;
    } else {
      if (pres & 1) {
        a0 = a0 + v[0] * gmD.x;
        a1 = a1 + v[0] * gmD.y;
      }
      if (pres & 2) {
        a0 = a0 + v[1] * gma.x;
        a1 = a1 + v[1] * gma.y;
      }
      a0 = a0 + v[2] * left;
      a1 = a1 + v[2] * ct.x;
      a0 = a0 + v[3] * ct.x;
      a1 = a1 + v[3] * ct.y;
      a0 = a0 + v[4] * ct.y;
      a1 = a1 + v[4] * right;
      if (pres & 4) {
        a0 = a0 + v[5] * gpa.x;
        a1 = a1 + v[5] * gpa.y;
      }
      if (pres & 8) {
        a0 = a0 + v[6] * gpD.x;
        a1 = a1 + v[6] * gpD.y;
      }
    }
    epi.row2(r0, a0, a1, true, true);
  }
}

// Team form of the lean walk, mode 4's fused kernel only (CsrDev::vl_team;
// DESIGN.md §4 "team walk"; as the plain SpMV it ran 64-66 against 48 us at
// 256^3, the per-step barrier costing more than the gathers it saves):
// one 1,024-thread workgroup per CU, its 16 waves at 16 consecutive walk
// positions of the class layout a 4-wave grid of 4x the workgroups was built
// for (the same rows of class bytes, the same step). At every step the 16
// waves hold 16 consecutive slices of one plane (or plane chunk), so a
// slice's +-a neighbours (a / 128 slices away) and its x-line's outer
// neighbours (one slice away) are, but for the team's edge waves, another
// wave's center pair of the same step: each wave publishes its center pair to
// LDS, one LDS barrier, and reads those pairs from there instead of
// gathering them (their L1 -> L2 requests are what the walk's requests beyond
// the compulsory center lines are: PMC). With GatherP (mode 4)
// the published pairs are the formed p_k, so a neighbour's pair costs no r /
// p_{k-1} loads either. Per row the same products in the same order as the
// 4-wave walk: Ap bit for bit.
constexpr int kTeamWaves = 16;
constexpr int kTeamBlock = 64 * kTeamWaves;
// the team walk's prefetch register (Gather::Raw where it prefetches)
template <class G, bool PF> struct PfRaw {
  using type = int;
};
template <class G> struct PfRaw<G, true> {
  using type = typename G::Raw;
};
template <typename T> struct TeamLds {
  typename PairU<T>::V pub[2][kTeamWaves][64];  // published centers, double-buffered by step
  SellLds<T> sell;                              // the per-slice form's dictionary, reductions
  T red[2 * kTeamWaves];
};

// PF: the +-D pair a step ahead of the one the sums use is loaded (raw, in
// Gather's halves) before the step's barrier and formed the step after, so
// each wave keeps a load in flight across its barrier, LDS reads, sums and
// stores instead of waiting a full memory round trip per step
template <typename T, class Epi, class Gather, bool PF = false>
__device__ __forceinline__ void spmv_lean_team(const CsrArgs &A, const Gather &x, Epi &epi,
                                               const T *__restrict__ vd,
                                               const unsigned long long *vt, TeamLds<T> &tl) {
  constexpr int VG = 8192 | 32768 | 262144 | 524288 | kVT | 2;  // the generic slices' form
  using PV = decltype(x.pair_b(0u));
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int Gt = (int)gridDim.x, b = (int)blockIdx.x, g = b & 7;
  const int step = (Gt >> 3) * kTeamWaves;  // the layout grid's G / 2
  const int w0 = (b >> 3) * kTeamWaves, w = w0 + wid;
  const int nsl = (int)A.nsl;
  const int lo = (int)(((int64_t)nsl * g) >> 3), end = (int)(((int64_t)nsl * (g + 1)) >> 3);
  const unsigned *__restrict__ row = reinterpret_cast<const unsigned *>(
      A.vl_cls + (int64_t)((A.rev ? 8 * step : 0) + g * step + w) * A.vl_nst);
  const int nw = A.vl_nst >> 2;
  const auto *tab = (const __attribute__((address_space(4))) VlClass *)A.vl_tab;
  const unsigned oD = (unsigned)A.vl_D * (unsigned)sizeof(T);
  const unsigned oa = (unsigned)A.vl_a * (unsigned)sizeof(T);
  const int P = A.vl_P, K = A.vl_K;
  const int D = A.vl_D, a = A.vl_a;
  const int nxi = (int)A.nx;
  const int Kp = D / (2 * kSellRows);
  const bool carry_walk = D % (2 * kSellRows) == 0 && (P > 0 ? K == Kp : step == Kp);
  // the +-a neighbours' walk offset (0: not whole slices, always gathered)
  const int asl = (a > 0 && a % (2 * kSellRows) == 0) ? a / (2 * kSellRows) : 0;
  // trips: every wave of the team takes the same number (one barrier each);
  // the plane-matched walk's last trip may leave the higher waves idle
  const int trips = P > 0 ? (K / step) * P : (end - lo - w0 + step - 1) / step;
  int zp = 0, cb = 0;
  int s = lo + w;
  unsigned cw = 0;
  PV c_ahead, c_ct;
  int carry_s = -1;
  typename PfRaw<Gather, PF>::type nraw{};
  int npos = -1;  // PF: the walk position whose ahead pair nraw holds
  // the ahead pair's byte offset of the slice at walk position s0
  [[maybe_unused]] auto ahead_b = [&](int s0) {
    const int f = (A.rev ? lo + end - 1 - s0 : s0) * (2 * kSellRows);
    const unsigned r = (unsigned)(f + 2 * lane) * (unsigned)sizeof(T);
    return A.rev ? r - (f >= D ? oD : 0u) : r + (f + 2 * kSellRows + D <= nxi ? oD : 0u);
  };
  for (int j = 0; j < trips; ++j) {
    if ((j & 255) == 0) {
      const int k = (j >> 2) + lane;
      cw = k < nw ? row[k] : ~0u;
      asm volatile("" : "+v"(cw));
    }
    const bool act = s < end;
    const unsigned word = (unsigned)__builtin_amdgcn_readlane((int)cw, (j & 255) >> 2);
    const int c = act ? (int)((word >> (8 * (j & 3))) & 0xffu) : 0xfe;
    const int si = A.rev ? lo + end - 1 - s : s;
    const int fr = si * (2 * kSellRows);
    const int r0 = fr + 2 * lane;
    const unsigned rb = (unsigned)r0 * (unsigned)sizeof(T);
    const unsigned omD = rb - (fr >= D ? oD : 0u);
    const unsigned opD = rb + (fr + 2 * kSellRows + D <= nxi ? oD : 0u);
    const int buf = j & 1;
    PV ct, behind, ahead;
    if (c < 0xfe) {
      if (s == carry_s) {
        ct = c_ahead;
        behind = c_ct;
      } else {
        ct = x.pair_b(rb);
        behind = x.pair_b(A.rev ? opD : omD);
      }
      if constexpr (PF) {
        ahead = s == npos ? x.form(nraw) : x.pair_b(A.rev ? omD : opD);
      } else {
        ahead = x.pair_b(A.rev ? omD : opD);
      }
      tl.pub[buf][wid][lane] = ct;
    } else if (c == 0xff) {
      tl.pub[buf][wid][lane] = x.pair_b(rb);  // the neighbours' pairs
    }
    if constexpr (PF) {  // the next position's ahead pair, in flight across this step
      int sn;
      if (P == 0) {
        sn = s + step;
      } else {
        const int zn = zp + 1 == P ? 0 : zp + 1, cn = zp + 1 == P ? cb + step : cb;
        sn = cn >= K ? end : lo + zn * K + cn + w;
      }
      npos = -1;
      if (sn < end) {
        nraw = x.raw_b(ahead_b(sn));
        npos = sn;
      }
    }
    lds_barrier();
    if (c == 0xff) {
      sellpv_slice2<T, VG, Epi, Gather>(A, x, epi, vd, si, vt);
    } else if (c < 0xfe) {
      // the neighbour waves at this step (the same trip: positions +-1, +-asl
      // away) where they are in the team and active, else a gather
      const int dm = A.rev ? 1 : -1;  // the walk offset of the slice before this one
      auto in_team = [&](int off) {
        const int x2 = wid + off;
        return x2 >= 0 && x2 < kTeamWaves && s + off >= lo && s + off < end;
      };
      T elo, ehi;
      if (fr > 0 && in_team(dm))
        elo = tl.pub[buf][wid + dm][63].y;
      else
        elo = x.at_s(fr > 0 ? fr - 1 : 0);
      if (fr + 2 * kSellRows < nxi && in_team(-dm))
        ehi = tl.pub[buf][wid - dm][0].x;
      else
        ehi = x.at_s(fr + 2 * kSellRows < nxi ? fr + 2 * kSellRows : nxi - 1);
      PV gma, gpa;
      const bool ma = a > 0 && fr >= a, pa = a > 0 && fr + 2 * kSellRows + a <= nxi;
      if (ma && asl > 0 && in_team(dm * asl)) gma = tl.pub[buf][wid + dm * asl][lane];
      else gma = x.pair_b(rb - (ma ? oa : 0u));
      if (pa && asl > 0 && in_team(-dm * asl)) gpa = tl.pub[buf][wid - dm * asl][lane];
      else gpa = x.pair_b(rb + (pa ? oa : 0u));
      const PV gmD = A.rev ? ahead : behind;
      const PV gpD = A.rev ? behind : ahead;
      c_ahead = ahead;
      c_ct = ct;
      carry_s = carry_walk ? s + Kp : -1;
      const int pres = tab[c].pres;
      T v[7];
#pragma unroll
      for (int q = 0; q < 7; ++q) v[q] = T(tab[c].v[q]);
      const T lo_e = tab[c].plo ? elo : -__builtin_copysign(T(0), v[2]);
      const T hi_e = tab[c].phi ? ehi : -__builtin_copysign(T(0), v[4]);
      const T left = wave_shr1(ct.y, lo_e), right = wave_shl1(ct.x, hi_e);
      epi.pre2c(r0, r0 + 1, ct.x, ct.y);
      T a0 = T(0), a1 = T(0);
      if (pres & 1) {
        a0 = a0 + v[0] * gmD.x;
        a1 = a1 + v[0] * gmD.y;
      }
      if (pres & 2) {
        a0 = a0 + v[1] * gma.x;
        a1 = a1 + v[1] * gma.y;
      }
      a0 = a0 + v[2] * left;
      a1 = a1 + v[2] * ct.x;
      a0 = a0 + v[3] * ct.x;
      a1 = a1 + v[3] * ct.y;
      a0 = a0 + v[4] * ct.y;
      a1 = a1 + v[4] * right;
      if (pres & 4) {
        a0 = a0 + v[5] * gpa.x;
        a1 = a1 + v[5] * gpa.y;
      }
      if (pres & 8) {
        a0 = a0 + v[6] * gpD.x;
        a1 = a1 + v[6] * gpD.y;
      }
      epi.row2(r0, a0, a1, true, true);
    }
    // the next position (the plane-matched walk: one step; the chunked walk:
    // the next plane of the chunk, then the next chunk)
    if (P == 0) {
      s += step;
    } else {
      if (++zp == P) {
        zp = 0;
        cb += step;
      }
      s = cb >= K ? end : lo + zp * K + cb + w;
    }
  }
}

// the team's fixed-order sum of one pair per thread (valid in thread 0;
// red: 2 T per wave)
template <typename T> __device__ __forceinline__ Dd<T> team_sum(Dd<T> v, T *red) {
  v = wave_sum_dd(v);
  if ((threadIdx.x & 63) == 0) {
    red[2 * (threadIdx.x >> 6)] = v.hi;
    red[2 * (threadIdx.x >> 6) + 1] = v.lo;
  }
  __syncthreads();
  Dd<T> s(T(0));
  if (threadIdx.x == 0)
#pragma unroll
    for (int i = 0; i < kTeamWaves; ++i) s += Dd<T>(red[2 * i], red[2 * i + 1]);
  return s;
}
// sum_parts's value (its order: threads 0..255 as a 256-thread workgroup)
// in a team workgroup
template <typename T> __device__ __forceinline__ T team_sum_parts(const T *part, int np, T *red) {
  __shared__ T bc;
  Dd<T> v(T(0));
  if (threadIdx.x < kBlock)
    for (int i = threadIdx.x; i < np; i += kBlock) v += load_part(part, i);
  v = wave_sum_dd(v);
  if ((threadIdx.x & 63) == 0 && threadIdx.x < kBlock) {
    red[2 * (threadIdx.x >> 6)] = v.hi;
    red[2 * (threadIdx.x >> 6) + 1] = v.lo;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    v = Dd<T>(red[0], red[1]);
#pragma unroll
    for (int k = 1; k < kBlock / 64; ++k) v += Dd<T>(red[2 * k], red[2 * k + 1]);
    bc = v.value();
  }
  __syncthreads();
  return bc;
}

// LDS layout of a variant's kernel
template <typename T, int V> struct LdsSel { using type = SpmvLds<T, TileOf<V>::tile>; };
template <typename T, int V>
using LdsOf = typename std::conditional<
    (V & (2048 | 8192)) != 0, SellLds<T>,
    SpmvLds<T, TileOf<V>::tile>>::type;

template <typename T, int V, class Epi, class Gather>
__device__ __forceinline__ void spmv_any(const CsrArgs &A, const T *__restrict__ val,
                                         const Gather &x, Epi &epi, LdsOf<T, V> &sm) {
  if constexpr ((V & 32768) != 0) spmv_sellpv<T, V, Epi, Gather>(A, x, epi, sm.vdict, sm.vt);
  else if constexpr ((V & 8192) != 0) spmv_sellp<T, V, Epi, Gather>(A, x, epi);
  else if constexpr ((V & 4096) != 0) spmv_sell2<T, V, Epi, Gather>(A, x, epi);
  else if constexpr ((V & 2048) != 0 && (V & 8) != 0) spmv_sell_pipe<T, V, Epi, Gather>(A, x, epi);
  else if constexpr ((V & 2048) != 0) spmv_sell<T, V, Epi, Gather>(A, x, epi);
  else if constexpr ((V & 256) != 0) spmv_rows_quad<T, V, Epi, Gather>(A, val, x, epi, sm);
  else if constexpr ((V & 8) != 0) spmv_rows_pipe<T, V, Epi, Gather>(A, val, x, epi, sm);
  else spmv_rows<T, V, Epi, Gather>(A, val, x, epi, sm);
}

// Row epilogues: pre(i) loads the row's own operands early (the pipelined
// loop issues it before the next block's prefetch, so waiting on it never
// waits on the prefetch); row(i, s) consumes the row sum.
// pre2 / row2: the same for two rows (SELL with 2 rows per lane); a row
// past the matrix end is given clamped (pre2) and flagged dead (row2).
// pre2c(i0, i1, c0, c1): pre2 when the gathered vector's elements at the
// two rows, c0 = x[i0], c1 = x[i1], are already in registers (the
// value-code kernel's center pair); only EpiDot, whose p IS the gathered
// vector (k_spmv_dot), uses them.
template <typename T> struct EpiDot {  // helper = A p; value2 += helper.p
  T *__restrict__ Ap;
  const T *__restrict__ p;
  Dd<T> acc;  // p.Ap (double-length)
  T pv, pv1;
  __device__ __forceinline__ void pre(int i) { pv = p[i]; }
  __device__ __forceinline__ void pre2c(int, int, T c0, T c1) {
    pv = c0;
    pv1 = c1;
  }
  __device__ __forceinline__ void row(int i, T s) {
    Ap[i] = s;
    acc += s * pv;
  }
  __device__ __forceinline__ void pre2(int i0, int i1) {
    using PV = typename PairOf<T>::V;
    if (i1 == i0 + 1 && (((uintptr_t)(p + i0)) & (sizeof(PV) - 1)) == 0) {  // one pair load
      const PV v = *reinterpret_cast<const PV *>(p + i0);
      pv = v.x;
      pv1 = v.y;
    } else {
      pv = p[i0];
      pv1 = p[i1];
    }
  }
  __device__ __forceinline__ void row2(int i, T s0, T s1, bool l0, bool l1) {
    using PV = typename PairOf<T>::V;
    if (l0 && l1 && (((uintptr_t)(Ap + i)) & (sizeof(PV) - 1)) == 0) {  // one pair store
      PV v;
      v.x = s0;
      v.y = s1;
      *reinterpret_cast<PV *>(Ap + i) = v;
    } else {
      if (l0) Ap[i] = s0;
      if (l1) Ap[i + 1] = s1;
    }
    if (l0) acc += s0 * pv;
    if (l1) acc += s1 * pv1;
  }
};
template <typename T> struct EpiInit {  // CG.hpp:325-331 (+ :341)
  const T *__restrict__ b;
  T *__restrict__ r;
  T *__restrict__ p;
  Dd<T> acc;  // r.r (double-length)
  T bv, bv1;
  __device__ __forceinline__ void pre(int i) { bv = b[i]; }
  __device__ __forceinline__ void pre2c(int i0, int i1, T, T) { pre2(i0, i1); }
  __device__ __forceinline__ void row(int i, T s) {
    const T ri = bv - s;
    r[i] = ri;
    p[i] = ri;
    acc += ri * ri;
  }
  __device__ __forceinline__ void pre2(int i0, int i1) {
    bv = b[i0];
    bv1 = b[i1];
  }
  __device__ __forceinline__ void row2(int i, T s0, T s1, bool l0, bool l1) {
    if (l0) row(i, s0);
    if (l1) {
      const T ri = bv1 - s1;
      r[i + 1] = ri;
      p[i + 1] = ri;
      acc += ri * ri;
    }
  }
};
// Fused iteration k: p_k = r_k + beta_{k-1} p_{k-1} (CG.hpp:418 of body
// k-1), x += alpha_{k-1} p_{k-1} (CG.hpp:390 of body k-1, deferred), then
// helper = A p_k and value2 += helper.p_k (CG.hpp:374-379 of body k).
template <typename T> struct EpiFused {
  const T *__restrict__ r;
  const T *__restrict__ pp;  // p_{k-1}
  T *__restrict__ pc;        // p_k
  T *__restrict__ x;
  T *__restrict__ Ap;
  T alpha, beta;
  bool do_x;
  Dd<T> acc;  // p.Ap (double-length)
  T rv, pv, xv, rv1, pv1, xv1;
  __device__ __forceinline__ void pre2c(int i0, int i1, T, T) { pre2(i0, i1); }
  __device__ __forceinline__ void pre(int i) {
    rv = r[i];
    pv = pp[i];
    xv = x[i];
  }
  __device__ __forceinline__ void row(int i, T s) {
    const T pi = rv + beta * pv;
    pc[i] = pi;
    Ap[i] = s;
    acc += s * pi;
    if (do_x) x[i] = xv + alpha * pv;
  }
  __device__ __forceinline__ void pre2(int i0, int i1) {
    pre(i0);
    rv1 = r[i1];
    pv1 = pp[i1];
    xv1 = x[i1];
  }
  __device__ __forceinline__ void row2(int i, T s0, T s1, bool l0, bool l1) {
    if (l0) row(i, s0);
    if (l1) {
      const T pi = rv1 + beta * pv1;
      pc[i + 1] = pi;
      Ap[i + 1] = s1;
      acc += s1 * pi;
      if (do_x) x[i + 1] = xv1 + alpha * pv1;
    }
  }
};
// Fused deferred-x iteration (mode 4), the SpMV's epilogue: p_k = r_k +
// beta_{k-1} p_{k-1} (CG.hpp:418 of body k-1) is computed where the SpMV
// reads it (GatherP, also for the center pair the value-code forms hand to
// pre2c) and stored once into this body's p buffer; then helper = A p_k and
// value2 += helper.p_k (CG.hpp:374-379) exactly as EpiDot.
template <typename T, bool NTP = false, bool NTS = false> struct EpiFD {
  T *__restrict__ Ap;
  T *__restrict__ pc;
  GatherP<T, NTP> g;
  Dd<T> acc;  // p.Ap (double-length)
  T pv, pv1;
  __device__ __forceinline__ void pre(int i) { pv = g(i); }
  __device__ __forceinline__ void pre2c(int, int, T c0, T c1) {
    pv = c0;
    pv1 = c1;
  }
  __device__ __forceinline__ void row(int i, T s) {
    pc[i] = pv;
    Ap[i] = s;
    acc += s * pv;
  }
  __device__ __forceinline__ void pre2(int i0, int i1) {
    if (i1 == i0 + 1) {
      const auto v = g.pair(i0);
      pv = v.x;
      pv1 = v.y;
    } else {
      pv = g(i0);
      pv1 = g(i1);
    }
  }
  __device__ __forceinline__ void row2(int i, T s0, T s1, bool l0, bool l1) {
    using PV = typename PairOf<T>::V;
    if (l0 && l1 && (((uintptr_t)(Ap + i)) & (sizeof(PV) - 1)) == 0) {  // pair stores
      PV a, q;
      a.x = s0;
      a.y = s1;
      q.x = pv;
      q.y = pv1;
      if constexpr (NTS) {  // streams past the Infinity Cache
        __builtin_nontemporal_store(a, reinterpret_cast<PV *>(Ap + i));
        __builtin_nontemporal_store(q, reinterpret_cast<PV *>(pc + i));
      } else {
        *reinterpret_cast<PV *>(Ap + i) = a;
        *reinterpret_cast<PV *>(pc + i) = q;
      }
    } else {
      if (l0) {
        Ap[i] = s0;
        pc[i] = pv;
      }
      if (l1) {
        Ap[i + 1] = s1;
        pc[i + 1] = pv1;
      }
    }
    if (l0) acc += s0 * pv;
    if (l1) acc += s1 * pv1;
  }
};
// Recomputed-Ap body (mode 6), kernel 1: value2 += helper.p (CG.hpp:378-
// 379) with helper = A p not stored — kernel 2 forms it again.
template <typename T> struct EpiDotOnly {
  const T *__restrict__ p;
  Dd<T> acc;  // p.Ap (double-length)
  T pv, pv1;
  __device__ __forceinline__ void pre(int i) { pv = p[i]; }
  __device__ __forceinline__ void pre2c(int, int, T c0, T c1) {
    pv = c0;
    pv1 = c1;
  }
  __device__ __forceinline__ void row(int, T s) { acc += s * pv; }
  __device__ __forceinline__ void pre2(int i0, int i1) {
    pv = p[i0];
    pv1 = p[i1];
  }
  __device__ __forceinline__ void row2(int, T s0, T s1, bool l0, bool l1) {
    if (l0) acc += s0 * pv;
    if (l1) acc += s1 * pv1;
  }
};
// Recomputed-Ap fused body (mode 7), kernel 1: p_k = r + beta p_{k-1}
// (CG.hpp:418) stored into P[k mod 4] and value2 += helper.p_k with helper =
// A p_k not stored — kernel 2 forms it again from the stored p_k
template <typename T> struct EpiFDDot {
  T *__restrict__ pc;
  GatherP<T> g;
  Dd<T> acc;  // p.Ap (double-length)
  T pv, pv1;
  __device__ __forceinline__ void pre(int i) { pv = g(i); }
  __device__ __forceinline__ void pre2c(int, int, T c0, T c1) {
    pv = c0;
    pv1 = c1;
  }
  __device__ __forceinline__ void row(int i, T s) {
    pc[i] = pv;
    acc += s * pv;
  }
  __device__ __forceinline__ void pre2(int i0, int i1) {
    if (i1 == i0 + 1) {
      const auto v = g.pair(i0);
      pv = v.x;
      pv1 = v.y;
    } else {
      pv = g(i0);
      pv1 = g(i1);
    }
  }
  __device__ __forceinline__ void row2(int i, T s0, T s1, bool l0, bool l1) {
    using PV = typename PairOf<T>::V;
    if (l0 && l1 && (((uintptr_t)(pc + i)) & (sizeof(PV) - 1)) == 0) {
      PV q;
      q.x = pv;
      q.y = pv1;
      *reinterpret_cast<PV *>(pc + i) = q;
    } else {
      if (l0) pc[i] = pv;
      if (l1) pc[i + 1] = pv1;
    }
    if (l0) acc += s0 * pv;
    if (l1) acc += s1 * pv1;
  }
};
// Mode 6, kernel 2: r = r - alpha helper (CG.hpp:392-393) with helper = A p
// formed again here (the same per-row sum as kernel 1's, bit for bit, so
// the same r as update_r's from a stored Ap), and value3 += r.r
// (CG.hpp:406-407)
template <typename T> struct EpiUpdR {
  T *__restrict__ r;
  T alpha;
  Dd<T> acc;  // r.r (double-length)
  T rv, rv1;
  __device__ __forceinline__ void pre(int i) { rv = r[i]; }
  __device__ __forceinline__ void pre2c(int i0, int i1, T, T) { pre2(i0, i1); }
  __device__ __forceinline__ void row(int i, T s) {
    const T v = rv - alpha * s;
    r[i] = v;
    acc += v * v;
  }
  __device__ __forceinline__ void pre2(int i0, int i1) {
    using PV = typename PairOf<T>::V;
    if (i1 == i0 + 1 && (((uintptr_t)(r + i0)) & (sizeof(PV) - 1)) == 0) {
      const PV v = *reinterpret_cast<const PV *>(r + i0);
      rv = v.x;
      rv1 = v.y;
    } else {
      rv = r[i0];
      rv1 = r[i1];
    }
  }
  __device__ __forceinline__ void row2(int i, T s0, T s1, bool l0, bool l1) {
    using PV = typename PairOf<T>::V;
    const T v0 = rv - alpha * s0, v1 = rv1 - alpha * s1;
    if (l0 && l1 && (((uintptr_t)(r + i)) & (sizeof(PV) - 1)) == 0) {
      PV v;
      v.x = v0;
      v.y = v1;
      *reinterpret_cast<PV *>(r + i) = v;
    } else {
      if (l0) r[i] = v0;
      if (l1) r[i + 1] = v1;
    }
    if (l0) acc += v0 * v0;
    if (l1) acc += v1 * v1;
  }
};
template <typename T> struct EpiAccuracy {  // CG.hpp:489-497
  const T *__restrict__ b;
  const T *__restrict__ x;
  T acc0, acc1, bv, xv, bv1, xv1;
  __device__ __forceinline__ void pre2c(int i0, int i1, T, T) { pre2(i0, i1); }
  __device__ __forceinline__ void pre(int i) {
    bv = b[i];
    xv = x[i];
  }
  __device__ __forceinline__ void row(int i, T s) {
    const T a = bv - s;
    acc0 += a * a;
    acc1 += xv * xv;
  }
  __device__ __forceinline__ void pre2(int i0, int i1) {
    pre(i0);
    bv1 = b[i1];
    xv1 = x[i1];
  }
  __device__ __forceinline__ void row2(int i, T s0, T s1, bool l0, bool l1) {
    if (l0) row(i, s0);
    if (l1) {
      const T a = bv1 - s1;
      acc0 += a * a;
      acc1 += xv1 * xv1;
    }
  }
};

template <typename T, int V>
__global__ __launch_bounds__(kBlock) void k_cg_init(CsrArgs A, const T *__restrict__ val,
                                                    const T *__restrict__ x,
                                                    const T *__restrict__ b, T *__restrict__ r,
                                                    T *__restrict__ p, CgScalars<T> *st,
                                                    RedWs<T> *ws, T tol, long long cap) {
  __shared__ LdsOf<T, V> sm;
  EpiInit<T> e{b, r, p, T(0), T(0), T(0)};
  spmv_any<T, V>(A, val, GatherX<T>{x}, e, sm);
  Dd<T> v = e.acc;
  if (grid_reduce_dd(v, ws, sm.red, &sm.flag) && threadIdx.x == 0) {
    st->rxr[0] = v.value();
    ws->rr_part[0] = v.hi;  // the pair, for a partitioned run's all-reduce
    ws->rr_part[1] = v.lo;
    st->pAp[0] = st->rr[0] = T(0);
    st->tol = tol;
    st->active[0] = 1;
    st->active[1] = st->active[2] = st->active[3] = 0;
    st->xpend[0] = st->xpend[1] = st->xpend[2] = st->xpend[3] = 0;
    for (int t = 0; t < 4; ++t) st->ran[t] = st->skip[t] = 0;
    st->bodies = 0;
    st->cap = cap;
    st->stopped = 0;
    st->tail_fault = 0;
  }
}

// Waves per SIMD a SpMV kernel asks the register allocator for: the
// value-code SELL-P form needs 8 (its persistent grid of kMaxGrid workgroups
// is then resident at once); the rest take what they get.
template <int V> struct SpmvWaves {
  // the plane march with templates: held to the 4 waves per SIMD (128
  // VGPRs, a 12-byte spill) the streamed-code march gets (it took 130 and 3)
  static constexpr int w = (V & 32768) && (V & (65536 | 131072)) ? 8
                           : ((V & kVT) && (V & 2097152)) ? 4
                                                          : 1;
};
// k_spmv_fd: the same except the template march (held to 4 waves it
// spilled 140 bytes; it takes 152 VGPRs, 3 waves, against 169 and 2 for the
// streamed-code march)
template <int V> struct FdWaves {
  static constexpr int w = ((V & kVT) && (V & 2097152)) ? 1 : SpmvWaves<V>::w;
};

template <typename T, int V>
__global__ __launch_bounds__(kBlock, SpmvWaves<V>::w) void k_spmv_dot(CsrArgs A,
                                                                      const T *__restrict__ val,
                                                     const T *__restrict__ p,
                                                     T *__restrict__ Ap, CgScalars<T> *st,
                                                     int slot, RedWs<T> *ws) {
  if (!st->active[slot]) return;  // (A.rev: the launcher's sweep direction)
  __shared__ LdsOf<T, V> sm;
  EpiDot<T> e{Ap, p, T(0), T(0), T(0)};
  spmv_any<T, V>(A, val, GatherX<T>{p}, e, sm);
  // this workgroup's share of p.Ap; k_update_r sums the partials
  store_part(ws->pap_part, A.part_off + blockIdx.x, e.acc, sm.red);
}

// k_spmv_dot in the lean stencil walk (kVL): the same epilogue and partials
// the lean walk's LDS copy of the value dictionary and the templates (a
// uniform branch: every thread of the workgroup takes it or none)
template <typename T>
__device__ __forceinline__ void lean_lds(const CsrArgs &A, SellLds<T> &sm) {
  const T *__restrict__ src = static_cast<const T *>(A.svdict);
  for (int i = threadIdx.x; i < kVcDict; i += kBlock) sm.vdict[i] = src[i];
  for (int i = threadIdx.x; i < A.nvt * 64; i += kBlock) sm.vt[i] = A.vct[i];
  __syncthreads();
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_spmv_lean(CsrArgs A, const T *__restrict__ p,
                                                      T *__restrict__ Ap, CgScalars<T> *st,
                                                      int slot, RedWs<T> *ws) {
  if (!st->active[slot]) return;
  __shared__ SellLds<T> sm;
  const T *vd = static_cast<const T *>(A.svdict);
  const unsigned long long *vt = A.vct;
  if (A.vl_lds) {
    lean_lds(A, sm);
    vd = sm.vdict;
    vt = sm.vt;
  }
  EpiDot<T> e{Ap, p, T(0), T(0), T(0)};
  spmv_lean<T>(A, GatherX<T>{p}, e, vd, vt);
  store_part(ws->pap_part, A.part_off + blockIdx.x - A.wg0, e.acc, sm.red);
}

// Recomputed-Ap body (mode 6; cgx_abi.cpp enqueue_iter_defer), kernel 1 of
// 3: the lean walk's A p with only p.Ap kept (no Ap stored: 8 N bytes less
// written, and kernel 2 reads p instead of Ap, which the walk just pulled
// through the Infinity Cache)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_spmv_lean_dot(CsrArgs A, const T *__restrict__ p,
                                                          CgScalars<T> *st, int slot,
                                                          RedWs<T> *ws) {
  if (!st->active[slot]) return;
  __shared__ SellLds<T> sm;
  const T *vd = static_cast<const T *>(A.svdict);
  const unsigned long long *vt = A.vct;
  if (A.vl_lds) {
    lean_lds(A, sm);
    vd = sm.vdict;
    vt = sm.vt;
  }
  EpiDotOnly<T> e{p, T(0), T(0), T(0)};
  // (the walk with the next slice's gathers issued before the current
  // slice's sums ran 54.4 against 39-40 us here: profiles/r6m_lean_dot_prefetch_ab.log)
  spmv_lean<T>(A, GatherX<T>{p}, e, vd, vt);
  store_part(ws->pap_part, blockIdx.x, e.acc, sm.red);
}

// Mode 6, kernel 2 of 3: alpha from kernel 1's p.Ap partials (sum_parts, as
// update_r), the records update_r makes (pAp, alpha, the group's skip
// mark), then the lean walk forms A p again and updates r in its epilogue;
// r.r partials for the p update. Every value is mode 3's.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_spmv_lean_updr(CsrArgs A, const T *__restrict__ p,
                                                           T *__restrict__ r, CgScalars<T> *st,
                                                           int slot, RedWs<T> *ws, int np_pap) {
  if (!st->active[slot]) return;
  __shared__ SellLds<T> sm;
  const T pAp = sum_parts(ws->pap_part, np_pap, sm.red);
  const T alpha = st->rxr[slot] / pAp;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->pAp[slot] = pAp;
    st->alpha[slot] = alpha;
    st->skip[slot] = 0;
  }
  const T *vd = static_cast<const T *>(A.svdict);
  const unsigned long long *vt = A.vct;
  if (A.vl_lds) {
    lean_lds(A, sm);
    vd = sm.vdict;
    vt = sm.vt;
  }
  EpiUpdR<T> e{r, alpha, T(0), T(0), T(0)};
  spmv_lean<T>(A, GatherX<T>{p}, e, vd, vt);
  store_part(ws->rr_part, blockIdx.x, e.acc, sm.red);
}

// The tile walk's prefetch of an epilogue's own rows: none by default;
// EpiUpdRT's r pairs come with the plane's outside pairs, two steps early
struct NoPre {};
template <class Epi> struct EpiPre {
  using type = NoPre;
  __device__ __forceinline__ static NoPre fetch(const Epi &, int) { return NoPre{}; }
  __device__ __forceinline__ static void take(Epi &, const NoPre &) {}
};
// Mode 6's kernel 2 in the tile walk: EpiUpdR with r's pair prefetched
// (pre2c loads nothing; the generic slices' pre / pre2 load as EpiUpdR)
template <typename T> struct EpiUpdRT : EpiUpdR<T> {
  __device__ __forceinline__ void pre2c(int, int, T, T) {}
};
template <typename T> struct EpiPre<EpiUpdRT<T>> {
  using type = typename PairOf<T>::V;
  __device__ __forceinline__ static type fetch(const EpiUpdRT<T> &e, int r0) {
    return *reinterpret_cast<const type *>(e.r + r0);
  }
  __device__ __forceinline__ static void take(EpiUpdRT<T> &e, const type &v) {
    e.rv = v.x;
    e.rv1 = v.y;
  }
};

// Lane l's value of v for every lane (l uniform)
template <typename T> __device__ __forceinline__ T lane_bcast(T v, int l);
template <> __device__ __forceinline__ double lane_bcast(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
template <> __device__ __forceinline__ float lane_bcast(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Tile form of the lean walk (lean_tile_ok; DESIGN.md §4 "tile walk"): one
// wave walks Y consecutive walk positions of the class layout (Y slices of
// a plane: Y / M x-lines when a = 128 M rows) through its XCD group's planes,
// with the planes it needs DIST steps ahead already in flight. The 4-wave
// walk has one slice's loads in flight per wave (1 KB of HBM lines at 4
// waves per SIMD, 112 VGPRs: no room for a second set) and waits a memory
// round trip every step; here a slot of the ring holds a plane's Y center
// pairs, the +-a pairs from outside the tile and the x-line edge values, and
// a step sums plane i from slots i - 1, i, i + 1 while planes i + 2 ..
// i + 1 + DIST are on their way (one wave per SIMD, its VGPRs to spare).
// Inside the tile the +-a neighbours (k +- M) and the x-line neighbours of
// the slices' end rows are other slices' centers, read from registers. Per
// row the same products in the same order as spmv_lean: Ap bit for bit.
template <typename T, int Y, int M, int DIST, bool REV, class Epi, class Gather>
__device__ __forceinline__ void spmv_lean_tile(const CsrArgs &A, const Gather &x, Epi &epi,
                                               const T *__restrict__ vd,
                                               const unsigned long long *vt, int zs) {
  constexpr int VG = 8192 | 32768 | 262144 | 524288 | kVT | 2;  // the generic slices' form
  constexpr int NRC = DIST + 3;                 // center ring: planes i - 1 .. i + 1 + DIST
  constexpr int U = NRC % 2 ? 2 * NRC : NRC;    // unroll: both rings return to slot 0
  constexpr int NE = M < Y ? M : Y;             // outside +-a pairs per side
  using PV = decltype(x.pair_b(0u));
  using Raw = typename Gather::Raw;    // a pair's loads (GatherP: r's and p_{k-1}'s)
  using Raw1 = typename Gather::Raw1;
  // a formed pair kept in a Raw slot (GatherP: in its a half) and read back
  auto to_raw = [](const PV &v) {
    Raw w;
    if constexpr (std::is_same<Raw, PV>::value) w = v;
    else w.a = v;
    return w;
  };
  auto formed = [](const Raw &w) -> PV {
    if constexpr (std::is_same<Raw, PV>::value) return w;
    else return w.a;
  };
  struct CSlot {
    Raw c[Y];  // the plane's center pairs (formed in place the step before their first use)
  };
  using Pre = typename EpiPre<Epi>::type;  // the epilogue's own rows (EpiUpdRT: r's pairs)
  struct ESlot {  // (two slots: plane i's, plane i + 1's)
    Raw em[NE];   // -a pairs of slices 0 .. NE - 1 (outside the tile)
    Raw ep[NE];   // +a pairs of slices Y - NE .. Y - 1
    Raw1 e;       // lane 0: row fr0 - 1; lane 63: row fr0 + 128 Y (the tile's x-line edges)
    Pre pre[Y];
  };
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // workgroup b: XCD group g = b mod 8, tile t of the plane, part zp of the
  // group's planes (zs parts: more waves per SIMD)
  const int b = (int)blockIdx.x, g = b & 7;
  const int tpg = (int)gridDim.x / (8 * zs);  // tiles of workgroups per plane
  const int step = tpg * 4 * Y;               // walk positions per plane (the layout's)
  const int t = (b >> 3) % tpg, zp = (b >> 3) / tpg;
  const int q0 = (t * 4 + wid) * Y;
  const int nsl = (int)A.nsl;
  const int lo = (int)(((int64_t)nsl * g) >> 3), end = (int)(((int64_t)nsl * (g + 1)) >> 3);
  const int J = (end - lo) / step;  // planes of the group (<= 256: one class word per lane)
  const int ib = zp * J / zs, ie = (zp + 1) * J / zs;  // this wave's walk indices
  const int nw = A.vl_nst >> 2;
  const auto *tab = (const __attribute__((address_space(4))) VlClass *)A.vl_tab;
  const int a = A.vl_a, nxi = (int)A.nx;
  const unsigned oa = (unsigned)a * (unsigned)sizeof(T);
  unsigned cw[Y];
#pragma unroll
  for (int k = 0; k < Y; ++k) {
    const unsigned *__restrict__ row = reinterpret_cast<const unsigned *>(
        A.vl_cls + (int64_t)(g * step + q0 + k) * A.vl_nst);
    const unsigned w = row[lane < nw ? lane : 0];  // (every lane loads: a fixed load count)
    cw[k] = lane < nw ? w : ~0u;
  }
  // walk index i: plane lo / step + (rev ? J - 1 - i : i); indices -1 and J
  // are the neighbouring groups' planes (or, at the matrix's ends, clamped to
  // an in-bounds slice whose pairs the class marks absent)
  auto first_row = [&](int i) {
    const int j = REV ? J - 1 - i : i;
    const int s0 = lo + q0 + j * step;
    return ((s0 < 0 || s0 + Y > nsl) ? lo + q0 : s0) * (2 * kSellRows);
  };
  auto load_c = [&](int i, CSlot &sl) {
    const int fr0 = first_row(i);
#pragma unroll
    for (int k = 0; k < Y; ++k)
      sl.c[k] = x.raw_b((unsigned)(fr0 + k * 2 * kSellRows + 2 * lane) * (unsigned)sizeof(T));
  };
  auto load_e = [&](int i, ESlot &sl) {
    const int fr0 = first_row(i);
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const int fr = fr0 + k * 2 * kSellRows;
      const unsigned rb = (unsigned)(fr + 2 * lane) * (unsigned)sizeof(T);
      sl.em[k] = x.raw_b(rb - (a > 0 && fr >= a ? oa : 0u));
    }
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const int fr = fr0 + (Y - NE + k) * 2 * kSellRows;
      const unsigned rb = (unsigned)(fr + 2 * lane) * (unsigned)sizeof(T);
      sl.ep[k] = x.raw_b(rb + (a > 0 && fr + 2 * kSellRows + a <= nxi ? oa : 0u));
    }
    const int elo = fr0 > 0 ? fr0 - 1 : 0;
    const int ehi = fr0 + Y * 2 * kSellRows < nxi ? fr0 + Y * 2 * kSellRows : nxi - 1;
    sl.e = x.raw1(lane == 0 ? elo : lane == 63 ? ehi : fr0 + 2 * lane);
#pragma unroll
    for (int k = 0; k < Y; ++k) sl.pre[k] = EpiPre<Epi>::fetch(epi, fr0 + k * 2 * kSellRows + 2 * lane);
  };
  // plane i's sums: behind / center / ahead in walk order (-D / +D swap in
  // the reversed sweep)
  // the centers of the plane a step ahead of the sums, formed (GatherP: p_k
  // = r + beta p_{k-1}, once per pair; GatherX: the loaded pair)
  auto form_c = [&](CSlot &sl) {
#pragma unroll
    for (int k = 0; k < Y; ++k) sl.c[k] = to_raw(x.form(sl.c[k]));
  };
  auto sum = [&](int i, const CSlot &sb, const CSlot &sc, const CSlot &sa, const ESlot &se) {
    const int j = REV ? J - 1 - i : i;
    const int s0 = lo + q0 + j * step;
    const int jb = j >> 2, jsh = 8 * (j & 3);  // plane j's class byte (the forward rows)
#pragma unroll
    for (int k = 0; k < Y; ++k) {
      const unsigned word = (unsigned)__builtin_amdgcn_readlane((int)cw[k], jb);
      const int c = (int)((word >> jsh) & 0xffu);
      const int si = s0 + k;
      if (c >= 0xfe) continue;  // the generic slices run after the walk
      const int fr = si * (2 * kSellRows);
      const int r0 = fr + 2 * lane;
      const PV ct = formed(sc.c[k]);
      const PV gmD = formed(REV ? sa.c[k] : sb.c[k]);
      const PV gpD = formed(REV ? sb.c[k] : sa.c[k]);
      PV gma, gpa;
      if (k >= M) gma = formed(sc.c[k >= M ? k - M : 0]);
      else gma = x.form(se.em[k < NE ? k : 0]);
      if (k + M < Y) gpa = formed(sc.c[k + M < Y ? k + M : 0]);
      else gpa = x.form(se.ep[k - (Y - NE) >= 0 ? k - (Y - NE) : 0]);
      const int pres = tab[c].pres;
      T v[7];
#pragma unroll
      for (int q = 0; q < 7; ++q) v[q] = T(tab[c].v[q]);
      const T e_f = (k == 0 || k == Y - 1) ? x.form1(se.e) : T(0);
      const T elo = k == 0 ? e_f : lane_bcast(formed(sc.c[k > 0 ? k - 1 : 0]).y, 63);
      const T ehi = k == Y - 1 ? e_f : lane_bcast(formed(sc.c[k + 1 < Y ? k + 1 : 0]).x, 0);
      const T lo_e = tab[c].plo ? elo : -__builtin_copysign(T(0), v[2]);
      const T hi_e = tab[c].phi ? ehi : -__builtin_copysign(T(0), v[4]);
      const T left = wave_shr1(ct.y, lo_e), right = wave_shl1(ct.x, hi_e);
      epi.pre2c(r0, r0 + 1, ct.x, ct.y);
      EpiPre<Epi>::take(epi, se.pre[k]);
      T a0 = T(0), a1 = T(0);
      if (pres == 15) {  // every slot present (the interior): no select
        a0 = a0 + v[0] * gmD.x;
        a1 = a1 + v[0] * gmD.y;
        a0 = a0 + v[1] * gma.x;
        a1 = a1 + v[1] * gma.y;
        a0 = a0 + v[2] * left;
        a1 = a1 + v[2] * ct.x;
        a0 = a0 + v[3] * ct.x;
        a1 = a1 + v[3] * ct.y;
        a0 = a0 + v[4] * ct.y;
        a1 = a1 + v[4] * right;
        a0 = a0 + v[5] * gpa.x;
        a1 = a1 + v[5] * gpa.y;
        a0 = a0 + v[6] * gpD.x;
        a1 = a1 + v[6] * gpD.y;
      } else {
        if (pres & 1) {
          a0 = a0 + v[0] * gmD.x;
          a1 = a1 + v[0] * gmD.y;
        }
        if (pres & 2) {
          a0 = a0 + v[1] * gma.x;
          a1 = a1 + v[1] * gma.y;
        }
        a0 = a0 + v[2] * left;
        a1 = a1 + v[2] * ct.x;
        a0 = a0 + v[3] * ct.x;
        a1 = a1 + v[3] * ct.y;
        a0 = a0 + v[4] * ct.y;
        a1 = a1 + v[4] * right;
        if (pres & 4) {
          a0 = a0 + v[5] * gpa.x;
          a1 = a1 + v[5] * gpa.y;
        }
        if (pres & 8) {
          a0 = a0 + v[6] * gpD.x;
          a1 = a1 + v[6] * gpD.y;
        }
      }
      epi.row2(r0, a0, a1, true, true);
    }
  };
  CSlot cr[NRC];
  ESlot er[2];
  // prologue: walk indices ib - 1 .. ib + DIST + 1 in center slots 0 .. NRC - 1
  // (index ib + i in slot (i + 1) mod NRC), ib and ib + 1's outside pairs
#pragma unroll
  for (int u = 0; u < NRC; ++u) load_c(ib + u - 1, cr[u]);
  load_e(ib, er[0]);
  load_e(ib + 1, er[1]);
  form_c(cr[0]);  // planes ib - 1 and ib; plane i + 1 at step i
  form_c(cr[1]);
  // step i (u = i - ib): sums from center slots u, u + 1, u + 2 (mod NRC) and
  // outside slot u mod 2, then plane i + 2 + DIST into center slot u (the one
  // plane i - 1 held) and plane i + 2's outside pairs into slot u mod 2.
  // Unrolled so every slot keeps its registers (no copy of a register with a
  // load in flight); the loads are never skipped (past the walk's end they
  // re-read an in-bounds plane), so every path issues the same loads and the
  // waits count only what a step needs
  for (int i0 = ib; i0 < ie; i0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u;
      form_c(cr[(u + 2) % NRC]);
      if (i < ie) sum(i, cr[u % NRC], cr[(u + 1) % NRC], cr[(u + 2) % NRC], er[u % 2]);
      load_c(i + 2 + DIST, cr[u % NRC]);
      load_e(i + 2, er[u % 2]);
    }
  }
  // the slices of other patterns (class 0xff: boundary lines and planes of
  // another pattern, chunks no template matched), one inlined copy of the
  // per-slice form for them all
  for (int i = ib; i < ie; ++i) {
    const int j = REV ? J - 1 - i : i;
#pragma unroll
    for (int k = 0; k < Y; ++k) {
      const unsigned word = (unsigned)__builtin_amdgcn_readlane((int)cw[k], j >> 2);
      if (((word >> (8 * (j & 3))) & 0xffu) == 0xff)
        sellpv_slice2<T, VG, Epi, Gather>(A, x, epi, vd, lo + q0 + j * step + k, vt);
    }
  }
}

// Mode 6's kernel 1 in the tile walk (lean_tile_ok): k_spmv_lean_dot's
// values; kTileZ parts of each group's planes, kTileW waves per SIMD
// (measured, profiles/r6t_*: Y 2 / Z 2 / DIST 1 35.8 us; DIST 2 42.1; Y 4 Z 4
// 40.8; Y 4 Z 2 DIST 3, two waves per SIMD, 40.1)
constexpr int kTileY = 2, kTileM = 2, kTileDist = 1, kTileZ = 2;
constexpr int kTileW = 4 * kTileZ / kTileY;  // waves per SIMD at the 1,024-workgroup layout
template <typename T>
__global__ __launch_bounds__(kBlock, kTileW) void k_spmv_lean_dot_tile(CsrArgs A,
                                                                       const T *__restrict__ p,
                                                                       CgScalars<T> *st, int slot,
                                                                       RedWs<T> *ws) {
  if (!st->active[slot]) return;
  __shared__ SellLds<T> sm;
  const T *vd = static_cast<const T *>(A.svdict);
  const unsigned long long *vt = A.vct;
  if (A.vl_lds) {
    lean_lds(A, sm);
    vd = sm.vdict;
    vt = sm.vt;
  }
  EpiDotOnly<T> e{p, T(0), T(0), T(0)};
  if (A.rev)  // (a template: the +-D roles swap without a select per pair)
    spmv_lean_tile<T, kTileY, kTileM, kTileDist, true>(A, GatherX<T>{p}, e, vd, vt, kTileZ);
  else
    spmv_lean_tile<T, kTileY, kTileM, kTileDist, false>(A, GatherX<T>{p}, e, vd, vt, kTileZ);
  store_part(ws->pap_part, blockIdx.x, e.acc, sm.red);
}

// Mode 6's kernel 2 in the tile walk (lean_tile_ok): k_spmv_lean_updr's
// values, r's pairs prefetched with the planes
template <typename T>
__global__ __launch_bounds__(kBlock, kTileW) void k_spmv_lean_updr_tile(CsrArgs A,
                                                                        const T *__restrict__ p,
                                                                        T *__restrict__ r,
                                                                        CgScalars<T> *st, int slot,
                                                                        RedWs<T> *ws, int np_pap) {
  if (!st->active[slot]) return;
  __shared__ SellLds<T> sm;
  const T pAp = sum_parts(ws->pap_part, np_pap, sm.red);
  const T alpha = st->rxr[slot] / pAp;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->pAp[slot] = pAp;
    st->alpha[slot] = alpha;
    st->skip[slot] = 0;
  }
  const T *vd = static_cast<const T *>(A.svdict);
  const unsigned long long *vt = A.vct;
  if (A.vl_lds) {
    lean_lds(A, sm);
    vd = sm.vdict;
    vt = sm.vt;
  }
  EpiUpdRT<T> e;
  e.r = r;
  e.alpha = alpha;
  e.acc = Dd<T>(T(0));
  if (A.rev)
    spmv_lean_tile<T, kTileY, kTileM, kTileDist, true>(A, GatherX<T>{p}, e, vd, vt, kTileZ);
  else
    spmv_lean_tile<T, kTileY, kTileM, kTileDist, false>(A, GatherX<T>{p}, e, vd, vt, kTileZ);
  store_part(ws->rr_part, blockIdx.x, e.acc, sm.red);
}

// Mode 7 (cgx_abi.cpp enqueue_iter_fdefer), kernel 1 of 2 (3 in slot 3):
// k_spmv_fd_lean's preamble (beta from body k-1's r.r partials, the records,
// slot 0 opening a group) and its p_k = r + beta p_{k-1} into P[s], in the
// tile walk: the ring's center pairs are formed once, a step before their
// first use, and serve as the -D / center / +D and in-tile +-a pairs; only
// the tile's outside +-a pairs and x-line edges are formed where used. No Ap
// vector: p.Ap partials only (kernel 2 forms A p_k again).
// (its ring holds two pairs per position, r's and p_{k-1}'s: kFdZ parts,
// kFdW waves per SIMD; at four waves it spilled)
// (Z 1 DIST 1: 101 us at 256^3; Z 1 DIST 0 105, Z 1 DIST 2 123, Z 2 DIST 0
// 111 with a spill; profiles/r6t_*)
constexpr int kFdZ = 1, kFdDist = 1, kFdW = 4 * kFdZ / kTileY;
template <typename T>
__global__ __launch_bounds__(kBlock, kFdW) void k_spmv_fd_dot_tile(
    CsrArgs A, const T *__restrict__ r, const T *__restrict__ pold, T *__restrict__ pc,
    CgScalars<T> *st, int slot, RedWs<T> *ws, int np_rr) {
  __shared__ SellLds<T> sm;
  const int prev = (slot + 3) & 3;
  const long long bodies = st->bodies;
  const bool act = st->active[slot] != 0;
  if (slot == 0 && blockIdx.x == 0 && threadIdx.x == 0)
    for (int t = 0; t < 4; ++t) st->ran[t] = 0;
  if (!act) {
    if (blockIdx.x == 0 && bodies > 0 && (int)(bodies & 3) == slot) {
      const T rr = sum_parts(ws->rr_part, np_rr, sm.red);
      if (threadIdx.x == 0) {
        st->rr[prev] = rr;
        st->rxr[slot] = rr;
      }
    }
    return;
  }
  T beta = T(0);
  if (bodies > 0) {
    const T rr = sum_parts(ws->rr_part, np_rr, sm.red);
    beta = rr / st->rxr[prev];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->rr[prev] = rr;  // the record
      st->rxr[slot] = rr;
    }
  }
  const T *vd = static_cast<const T *>(A.svdict);
  const unsigned long long *vt = A.vct;
  if (A.vl_lds) {
    lean_lds(A, sm);
    vd = sm.vdict;
    vt = sm.vt;
  }
  const GatherP<T> g{r, pold, beta};
  EpiFDDot<T> e{pc, g, T(0), T(0), T(0)};
  if (A.rev)
    spmv_lean_tile<T, kTileY, kTileM, kFdDist, true>(A, g, e, vd, vt, kFdZ);
  else
    spmv_lean_tile<T, kTileY, kTileM, kFdDist, false>(A, g, e, vd, vt, kFdZ);
  store_part(ws->pap_part, blockIdx.x, e.acc, sm.red);
}

// Mode 7, kernel 2: k_spmv_lean_updr on the stored p_k with update_r's stop
// rule (the r.r the body started with, which kernel 1 recorded; bodies, the
// next slot's active flag, ran[slot]) — mode 4's kernel 2 with A p_k formed
// again instead of read
template <typename T>
__global__ __launch_bounds__(kBlock) void k_spmv_lean_updr_rule(CsrArgs A,
                                                                const T *__restrict__ p,
                                                                T *__restrict__ r,
                                                                CgScalars<T> *st, int slot,
                                                                RedWs<T> *ws, int np_pap) {
  if (!st->active[slot]) {
    if (blockIdx.x == 0 && threadIdx.x == 0) st->active[(slot + 1) & 3] = 0;
    return;
  }
  __shared__ SellLds<T> sm;
  const T pAp = sum_parts(ws->pap_part, np_pap, sm.red);
  const T rxr = st->rxr[slot];
  const T alpha = rxr / pAp;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->pAp[slot] = pAp;
    st->alpha[slot] = alpha;
    st->skip[slot] = 0;
    const long long m = st->bodies + 1;  // stop rule, as k_update_xp
    st->bodies = m;
    const bool cond = isnan(rxr) || sqrt(rxr) <= st->tol;
    const bool cont = !cond && m < st->cap;
    st->active[(slot + 1) & 3] = cont ? 1 : 0;
    st->stopped = cond ? 1 : (cont ? 0 : 2);
    st->ran[slot] = 1;
  }
  const T *vd = static_cast<const T *>(A.svdict);
  const unsigned long long *vt = A.vct;
  if (A.vl_lds) {
    lean_lds(A, sm);
    vd = sm.vdict;
    vt = sm.vt;
  }
  EpiUpdR<T> e{r, alpha, T(0), T(0), T(0)};
  spmv_lean<T>(A, GatherX<T>{p}, e, vd, vt);
  store_part(ws->rr_part, blockIdx.x, e.acc, sm.red);
}

// The interior SpMV of a partitioned SELL matrix with the device peer
// transport's halo push in its first A.wg0 workgroups (peerdev::push_wg, as
// k_peer_push): the push's xGMI stores overlap the interior slices instead
// of running as a launch of their own before them. The SpMV workgroups are
// k_spmv_dot's, renumbered from wg0 (sell_range), partials at
// part_off + blockIdx - wg0.
template <typename T, int V>
__global__ __launch_bounds__(kBlock, SpmvWaves<V>::w) void k_spmv_dot_push(
    CsrArgs A, const T *__restrict__ val, const T *__restrict__ p, T *__restrict__ Ap,
    CgScalars<T> *st, int slot, RedWs<T> *ws, PeerDev P) {
  if ((int)blockIdx.x < A.wg0) {
    peerdev::push_wg<T>(p, P, st, slot, blockIdx.x);
    return;
  }
  if (!st->active[slot]) return;
  __shared__ LdsOf<T, V> sm;
  EpiDot<T> e{Ap, p, T(0), T(0), T(0)};
  spmv_any<T, V>(A, val, GatherX<T>{p}, e, sm);
  store_part(ws->pap_part, A.part_off + blockIdx.x - A.wg0, e.acc, sm.red);
}

// A partitioned matrix's interior slices by the lean walk (its layout skips
// the boundary slices) with the halo push in the first A.wg0 workgroups, as
// k_spmv_dot_push does for the slice-list form
template <typename T>
__global__ __launch_bounds__(kBlock) void k_spmv_lean_push(CsrArgs A, const T *__restrict__ p,
                                                           T *__restrict__ Ap, CgScalars<T> *st,
                                                           int slot, RedWs<T> *ws, PeerDev P) {
  if ((int)blockIdx.x < A.wg0) {
    peerdev::push_wg<T>(p, P, st, slot, blockIdx.x);
    return;
  }
  if (!st->active[slot]) return;
  __shared__ SellLds<T> sm;
  const T *vd = static_cast<const T *>(A.svdict);
  const unsigned long long *vt = A.vct;
  if (A.vl_lds) {
    lean_lds(A, sm);
    vd = sm.vdict;
    vt = sm.vt;
  }
  EpiDot<T> e{Ap, p, T(0), T(0), T(0)};
  spmv_lean<T>(A, GatherX<T>{p}, e, vd, vt);
  store_part(ws->pap_part, A.part_off + blockIdx.x - A.wg0, e.acc, sm.red);
}

// The boundary slices with the peer transport's wait folded in (round 3;
// DESIGN.md §9): every workgroup's first wave polls the push flags of every
// rank that sends here for this body's tag (k_peer_wait's poll, bounded),
// then the workgroup runs its slices gathering ghosts from the landing
// buffer (GatherXL). It waits only on other GPUs' pushes, which were raised
// by their interior launches and depend on nothing in this launch, so the
// protocol needs no workgroup of this launch to be resident or dispatched
// before another. One launch per body less than push / wait / boundary.
template <typename T, int V>
__global__ __launch_bounds__(kBlock, SpmvWaves<V>::w) void k_spmv_dot_bnd(
    CsrArgs A, const T *__restrict__ val, const T *__restrict__ p, T *__restrict__ Ap,
    CgScalars<T> *st, int slot, RedWs<T> *ws, PeerDev P) {
  if (peerdev::skip_body(st, slot, P.state)) return;
  __shared__ int ok_s;
  if (!peerdev::wait_pushes(P, peerdev::body_tag(st, slot, P.state), &ok_s)) {
    if (threadIdx.x == 0) peerdev::raise_fault(st, slot, P.state);
    return;
  }
  __shared__ LdsOf<T, V> sm;
  EpiDot<T> e{Ap, p, T(0), T(0), T(0)};
  spmv_any<T, V>(A, val, GatherXL<T>{p, reinterpret_cast<const T *>(P.land_local), (int)A.n}, e,
                 sm);
  store_part(ws->pap_part, A.part_off + blockIdx.x, e.acc, sm.red);
}

// Fused deferred-x iteration (mode 4), kernel 1 of 2 for body k in slot s
// (cgx_abi.cpp enqueue_iter_fdefer): p_k into P[s] from r and P[s-1] (EpiFD),
// helper = A p_k, this workgroup's p.Ap partial. beta_{k-1} = r.r / rxr from
// body k-1's update_r partials, summed in sum_parts order as
// k_update_p_defer does, so every value is the one of modes 1 and 3; body 0
// (bodies == 0) takes beta = 0 against a zeroed P[3]. Workgroup 0 records
// rxr[s] (the r.r body k starts with) — also in the first skipped body,
// where the host reads the final r.r — and, in slot 0, opens a new group of
// deferred x updates (ran[] cleared; the slot-3 flush has applied the last).
template <typename T, int V>
__global__ __launch_bounds__(kBlock, FdWaves<V>::w) void k_spmv_fd(
    CsrArgs A, const T *__restrict__ val, const T *__restrict__ r, const T *__restrict__ pold,
    T *__restrict__ pc, T *__restrict__ Ap, CgScalars<T> *st, int slot, RedWs<T> *ws,
    int np_rr) {
  __shared__ LdsOf<T, V> sm;
  const int prev = (slot + 3) & 3;
  // (the flag checked before the partials' loads: the late-active form was
  // 0.16 us slower here at 128^2, profiles/r02_late_active.log)
  const long long bodies = st->bodies;
  const bool act = st->active[slot] != 0;
  if (slot == 0 && blockIdx.x == 0 && threadIdx.x == 0)
    for (int t = 0; t < 4; ++t) st->ran[t] = 0;
  if (!act) {
    if (blockIdx.x == 0 && bodies > 0 && (int)(bodies & 3) == slot) {
      const T rr = sum_parts(ws->rr_part, np_rr, sm.red);
      if (threadIdx.x == 0) {
        st->rr[prev] = rr;
        st->rxr[slot] = rr;
      }
    }
    return;
  }
  T beta = T(0);
  if (bodies > 0) {
    const T rr = sum_parts(ws->rr_part, np_rr, sm.red);
    beta = rr / st->rxr[prev];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->rr[prev] = rr;  // the record
      st->rxr[slot] = rr;
    }
  }
  constexpr bool NTP = (V & 2097152) != 0;  // plane march: p_{k-1} lines read once
  const GatherP<T, NTP> g{r, pold, beta};
  EpiFD<T, NTP> e{Ap, pc, g, T(0), T(0), T(0)};
  spmv_any<T, V>(A, val, g, e, sm);
  store_part(ws->pap_part, A.part_off + blockIdx.x, e.acc, sm.red);
}

// k_spmv_fd in the lean stencil walk (kVL): the gathers form p_k = r +
// beta p_{k-1} from both vectors (GatherP), the epilogue stores p_k and Ap
// (EpiFD); the same preamble (beta from the r.r partials, the record of the
// previous body's r.r)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_spmv_fd_lean(
    CsrArgs A, const T *__restrict__ r, const T *__restrict__ pold, T *__restrict__ pc,
    T *__restrict__ Ap, CgScalars<T> *st, int slot, RedWs<T> *ws, int np_rr) {
  __shared__ SellLds<T> sm;
  const int prev = (slot + 3) & 3;
  const long long bodies = st->bodies;
  const bool act = st->active[slot] != 0;
  if (slot == 0 && blockIdx.x == 0 && threadIdx.x == 0)
    for (int t = 0; t < 4; ++t) st->ran[t] = 0;
  if (!act) {
    if (blockIdx.x == 0 && bodies > 0 && (int)(bodies & 3) == slot) {
      const T rr = sum_parts(ws->rr_part, np_rr, sm.red);
      if (threadIdx.x == 0) {
        st->rr[prev] = rr;
        st->rxr[slot] = rr;
      }
    }
    return;
  }
  T beta = T(0);
  if (bodies > 0) {
    const T rr = sum_parts(ws->rr_part, np_rr, sm.red);
    beta = rr / st->rxr[prev];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->rr[prev] = rr;  // the record
      st->rxr[slot] = rr;
    }
  }
  const T *vd = static_cast<const T *>(A.svdict);
  const unsigned long long *vt = A.vct;
  if (A.vl_lds) {
    lean_lds(A, sm);
    vd = sm.vdict;
    vt = sm.vt;
  }
  const GatherP<T> g{r, pold, beta};
  EpiFD<T> e{Ap, pc, g, T(0), T(0), T(0)};
  spmv_lean<T>(A, g, e, vd, vt);
  store_part(ws->pap_part, A.part_off + blockIdx.x, e.acc, sm.red);
}

// k_spmv_fd_lean in the team form (CsrDev::vl_team): the published centers
// are the formed p_k, so an in-team neighbour costs no r / p_{k-1} loads
template <typename T, bool PF, bool NTS>
__global__ __launch_bounds__(kTeamBlock) void k_spmv_fd_lean_t(
    CsrArgs A, const T *__restrict__ r, const T *__restrict__ pold, T *__restrict__ pc,
    T *__restrict__ Ap, CgScalars<T> *st, int slot, RedWs<T> *ws, int np_rr) {
  __shared__ TeamLds<T> tl;
  const int prev = (slot + 3) & 3;
  const long long bodies = st->bodies;
  const bool act = st->active[slot] != 0;
  if (slot == 0 && blockIdx.x == 0 && threadIdx.x == 0)
    for (int t = 0; t < 4; ++t) st->ran[t] = 0;
  if (!act) {
    if (blockIdx.x == 0 && bodies > 0 && (int)(bodies & 3) == slot) {
      const T rr = team_sum_parts(ws->rr_part, np_rr, tl.red);
      if (threadIdx.x == 0) {
        st->rr[prev] = rr;
        st->rxr[slot] = rr;
      }
    }
    return;
  }
  T beta = T(0);
  if (bodies > 0) {
    const T rr = team_sum_parts(ws->rr_part, np_rr, tl.red);
    beta = rr / st->rxr[prev];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->rr[prev] = rr;  // the record
      st->rxr[slot] = rr;
    }
  }
  const T *vd = static_cast<const T *>(A.svdict);
  const unsigned long long *vt = A.vct;
  if (A.vl_lds) {
    for (int i = threadIdx.x; i < kVcDict; i += kTeamBlock) tl.sell.vdict[i] = vd[i];
    for (int i = threadIdx.x; i < A.nvt * 64; i += kTeamBlock) tl.sell.vt[i] = vt[i];
    __syncthreads();
    vd = tl.sell.vdict;
    vt = tl.sell.vt;
  }
  const GatherP<T> g{r, pold, beta};
  EpiFD<T, false, NTS> e{Ap, pc, g, T(0), T(0), T(0)};
  spmv_lean_team<T, EpiFD<T, false, NTS>, GatherP<T>, PF>(A, g, e, vd, vt, tl);
  const Dd<T> v = team_sum(e.acc, tl.red);
  if (threadIdx.x == 0) {
    ws->pap_part[2 * (A.part_off + blockIdx.x)] = v.hi;
    ws->pap_part[2 * (A.part_off + blockIdx.x) + 1] = v.lo;
  }
}

// Mode 4 on a partitioned matrix (device peer transport), kernel 1 of 3:
// k_spmv_fd_lean over the interior slices, with the halo push of the formed
// p_k (the value this rank's own SpMV forms for those rows) in the first
// A.wg0 workgroups. beta = rxr[s] / rxr[s-1]: the world r.r of body k-1 was
// all-reduced by the last workgroup of its kernel 3 (k_update_r_peer_rule),
// so no workgroup here waits on another rank (on a GPU shared by ranks, a
// whole grid spinning would hold the CUs the other ranks need to publish).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_spmv_fd_lean_push(
    CsrArgs A, const T *__restrict__ r, const T *__restrict__ pold, T *__restrict__ pc,
    T *__restrict__ Ap, CgScalars<T> *st, int slot, RedWs<T> *ws, PeerDev P) {
  __shared__ SellLds<T> sm;
  const int prev = (slot + 3) & 3;
  const long long bodies = st->bodies;
  const bool act = st->active[slot] != 0 && !P.state->fault;
  if (slot == 0 && blockIdx.x == 0 && threadIdx.x == 0)
    for (int t = 0; t < 4; ++t) st->ran[t] = 0;
  if (!act) return;
  const T beta = bodies > 0 ? st->rxr[slot] / st->rxr[prev] : T(0);
  const GatherP<T> g{r, pold, beta};
  if ((int)blockIdx.x < A.wg0) {
    peerdev::push_wg_from<T>(g, P, st, slot, blockIdx.x);
    return;
  }
  const T *vd = static_cast<const T *>(A.svdict);
  const unsigned long long *vt = A.vct;
  if (A.vl_lds) {
    lean_lds(A, sm);
    vd = sm.vdict;
    vt = sm.vt;
  }
  EpiFD<T> e{Ap, pc, g, T(0), T(0), T(0)};
  spmv_lean<T>(A, g, e, vd, vt);
  store_part(ws->pap_part, A.part_off + blockIdx.x - A.wg0, e.acc, sm.red);
}

// Mode 4 on a partitioned matrix, kernel 2 of 3: the boundary rows as
// CSR-stream blocks after k_spmv_dot_bnd's wait for the neighbours' pushes;
// own columns form p_k from r and p_{k-1} with kernel 1's beta (the same
// division), ghosts are the pushed p_k in the landing buffer. The rows' p_k
// and Ap are stored, their p.Ap partials at part_off.
template <typename T, int V>
__global__ __launch_bounds__(kBlock, SpmvWaves<V>::w) void k_spmv_fd_bnd(
    CsrArgs A, const T *__restrict__ val, const T *__restrict__ r, const T *__restrict__ pold,
    T *__restrict__ pc, T *__restrict__ Ap, CgScalars<T> *st, int slot, RedWs<T> *ws,
    PeerDev P) {
  if (peerdev::skip_body(st, slot, P.state)) return;
  __shared__ int ok_s;
  if (!peerdev::wait_pushes(P, peerdev::body_tag(st, slot, P.state), &ok_s)) {
    if (threadIdx.x == 0) peerdev::raise_fault(st, slot, P.state);
    return;
  }
  const int prev = (slot + 3) & 3;
  const T beta = st->bodies > 0 ? st->rxr[slot] / st->rxr[prev] : T(0);
  __shared__ LdsOf<T, V> sm;
  const GatherP<T> g{r, pold, beta};
  EpiFD<T> e{Ap, pc, g, T(0), T(0), T(0)};
  spmv_any<T, V>(A, val, GatherPL<T>{g, reinterpret_cast<const T *>(P.land_local), (int)A.n}, e,
                 sm);
  store_part(ws->pap_part, A.part_off + blockIdx.x, e.acc, sm.red);
}

// The final r.r of a mode-4 run that ended on an active body (no kernel 1
// followed to record it): rxr[s] of the next slot, as k_spmv_fd records it.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_rr_settle(CgScalars<T> *st, RedWs<T> *ws, int np_rr) {
  __shared__ T red[4 * kMaxRed];
  const long long bodies = st->bodies;
  if (bodies <= 0) return;
  const int slot = (int)(bodies & 3);
  const T rr = sum_parts(ws->rr_part, np_rr, red);
  if (threadIdx.x == 0) {
    st->rr[(slot + 3) & 3] = rr;
    st->rxr[slot] = rr;
  }
}

// Fused iteration, kernel 1 of 2 (slot s of body k). Reads active[s] (run
// body k), xpend[s-1] (the x update of body k-1 is still pending) and
// bodies == 0 (body 0: p_{-1} = 0, beta = 0). With body k inactive it only
// applies the pending x update. The last workgroup publishes p.Ap and clears
// xpend[s-1].
template <typename T, int V>
__global__ __launch_bounds__(kBlock) void k_spmv_fused(CsrArgs A, const T *__restrict__ val,
                                                       const T *__restrict__ r,
                                                       const T *__restrict__ pp,
                                                       T *__restrict__ pc, T *__restrict__ x,
                                                       T *__restrict__ Ap, CgScalars<T> *st,
                                                       int slot, RedWs<T> *ws) {
  const int prev = (slot + 3) & 3;
  const bool act = st->active[slot] != 0;
  const bool xp = st->xpend[prev] != 0;
  if (!act && !xp) return;
  __shared__ LdsOf<T, V> sm;
  const T alpha = xp ? st->rxr[prev] / st->pAp[prev] : T(0);
  Dd<T> v(T(0));
  if (act) {
    const T beta = st->bodies == 0 ? T(0) : st->rr[prev] / st->rxr[prev];
    EpiFused<T> e{r, pp, pc, x, Ap, alpha, beta, xp, T(0), T(0), T(0), T(0), T(0), T(0), T(0)};
    spmv_any<T, V>(A, val, GatherP<T>{r, pp, beta}, e, sm);
    v = e.acc;
  } else {
    // stopped after body k-1: only its deferred x update remains
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < A.n; i += stride)
      x[i] = x[i] + alpha * pp[i];
  }
  if (grid_reduce_dd(v, ws, sm.red, &sm.flag) && threadIdx.x == 0) {
    if (act) st->pAp[slot] = v.value();
    if (xp) st->xpend[prev] = 0;
  }
}

// Apply a pending x update (end of a run of fused iterations): x += alpha p.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_flush_x(int64_t n, T *__restrict__ x,
                                                    const T *__restrict__ p, CgScalars<T> *st,
                                                    int slot, RedWs<T> *ws) {
  if (!st->xpend[slot]) return;
  __shared__ T red[8];
  __shared__ int flag;
  const T alpha = st->rxr[slot] / st->pAp[slot];
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    x[i] = x[i] + alpha * p[i];
  T v[1] = {T(0)};
  if (grid_reduce<T, 1>(v, ws, red, &flag) && threadIdx.x == 0) st->xpend[slot] = 0;
}

template <typename T, int V>
__global__ __launch_bounds__(kBlock) void k_accuracy(CsrArgs A, const T *__restrict__ val,
                                                     const T *__restrict__ b,
                                                     const T *__restrict__ x, T *out2,
                                                     RedWs<T> *ws) {
  __shared__ LdsOf<T, V> sm;
  EpiAccuracy<T> e{b, x, T(0), T(0), T(0), T(0), T(0), T(0)};
  spmv_any<T, V>(A, val, GatherX<T>{x}, e, sm);
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
// FUSED: kernel 2 of 2 of the fused iteration, which also runs the stop rule
// (CG.hpp:396-404, 410-417, 436) and marks body k's x update as pending.
// PEER (partitioned run, device peer transport): p.Ap from this rank's
// partials, then all-reduced here (peerdev::world_sum, tag base + 1) instead
// of by a k_peer_allreduce launch before this kernel.
template <typename T> __device__ __forceinline__ void peer_fault(CgScalars<T> *st, int slot,
                                                                 const PeerDev *P) {
  if (threadIdx.x == 0) {
    P->state->fault = 1;
    st->active[slot] = 0;
    st->stopped = 3;
  }
}

// mode 4's group flush folded into slot 3's update_r: x and the group's p buffers
template <typename T> struct XFlush {
  T *x;
  const T *P[4];
};
// Mode 4, slot 3: the group's deferred x updates, x = (((x + a0 p0) + a1
// p1) + a2 p2) + a3 p3 over the slots whose use[] is set (the slots that ran
// in this group and no end-of-run flush applied: k_flush_defer's rule;
// k_spmv_fd of the next slot 0 clears ran[]). 16-byte lanes over this
// launch's grid; x and the p buffers are not re-read before the next group
// overwrites them.
template <typename T>
__device__ __forceinline__ void flush_group_range(int64_t n, T *__restrict__ x,
                                                  const T *__restrict__ P0,
                                                  const T *__restrict__ P1,
                                                  const T *__restrict__ P2,
                                                  const T *__restrict__ P3, const T (&a)[4],
                                                  const bool (&use)[4], int rev) {
  using V = typename Vec2<T>::V;
  const int64_t n2 = n >> 1;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  V *x2 = reinterpret_cast<V *>(x);
  const V *Q[4] = {reinterpret_cast<const V *>(P0), reinterpret_cast<const V *>(P1),
                   reinterpret_cast<const V *>(P2), reinterpret_cast<const V *>(P3)};
  auto body = [&](int64_t i, auto sntc) {
    constexpr bool S = decltype(sntc)::value;
    V xv = ldv<S, T>(x2 + i);
    V q[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) q[t] = ldv<S, T>(Q[t] + i);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (use[t]) {
        xv.x = xv.x + a[t] * q[t].x;
        xv.y = xv.y + a[t] * q[t].y;
      }
    }
    stv<S, T>(x2 + i, xv);
  };
  auto E = [&](int64_t j) { return rev ? n2 - 1 - j : j; };
  auto loop = [&](auto sntc) {
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + stride < n2; i += 2 * stride) {
      body(E(i), sntc);
      body(E(i + stride), sntc);
    }
    for (; i < n2; i += stride) body(E(i), sntc);
  };
  if (stream_nt<T>(n))
    loop(std::true_type{});
  else
    loop(std::false_type{});
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    T xv = x[n - 1];
    const T *Ps[4] = {P0, P1, P2, P3};
    for (int t = 0; t < 4; ++t)
      if (use[t]) xv = xv + a[t] * Ps[t][n - 1];
    x[n - 1] = xv;
  }
}


template <typename T, bool FUSED, bool PEER, bool SNT, bool GF = false, int KP = kPartsPerThread>
// rin == r: in place (modes 1, 2); else r ping-pongs between two buffers.
// GF (mode 4, slot 3): after r, the group's deferred x updates (xf), also
// when the body itself is inactive (the group's earlier bodies that ran).
__device__ __forceinline__ void update_r_body(int64_t n, const T *rin, T *r,
                                              const T *__restrict__ Ap, CgScalars<T> *st,
                                              int slot, RedWs<T> *ws, int np_pap, int rev,
                                              int rule, const PeerDev *P,
                                              const XFlush<T> *xf = nullptr) {
  // rule (mode 4, kernel 2 of 2): this kernel also runs the stop rule
  // (CG.hpp:396-404, 436: on the r.r the body started with, which k_spmv_fd
  // recorded) and marks the body's x update pending (ran[slot])
  const auto *cst = (const __attribute__((address_space(4))) CgScalars<T> *)st;
  const bool act = cst->active[slot] != 0;  // branched on after the first loads
  __shared__ T red[8];
  __shared__ int flag;
  using V = typename Vec2<T>::V;
  const int64_t n2 = n >> 1;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  V *r2 = reinterpret_cast<V *>(r);
  const V *ri2 = reinterpret_cast<const V *>(rin);
  const V *a2 = reinterpret_cast<const V *>(Ap);
  auto E = [&](int64_t j) { return rev ? n2 - 1 - j : j; };  // sweep direction
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  // p.Ap: the spmv_dot partials (single device) or st (fused mode, or
  // partitioned runs after the all-reduce). The partials' loads go out
  // first, then this thread's first block of r and Ap (which do not need
  // alpha), then the partials are summed while that block is in flight.
  // scalar loads (lgkmcnt): a vector load issued after the prefetch would
  // make its wait drain the prefetch too
  const T rxr = cst->rxr[slot];
  const T pAp_st = cst->pAp[slot];
  Dd<T> pl[KP];
  const bool from_parts = !FUSED && np_pap > 0;
  if (from_parts) parts_load(ws->pap_part, np_pap, pl);
  V rv[kUR], av[kUR];
#pragma unroll
  for (int u = 0; u < kUR; ++u) {  // clamped (r and Ap have a slack element): no branch
    const int64_t j = E(min(i + u * stride, n2 > 0 ? n2 - 1 : 0));
    rv[u] = ri2[j];
    av[u] = ldv<SNT, T>(a2 + j);  // Ap is dead after this kernel
  }
  // the group flush's alphas and flags of the earlier slots (written by
  // earlier launches; this one writes only slot 3's)
  T ga[4] = {T(0), T(0), T(0), T(0)};
  bool guse[4] = {false, false, false, false};
  if constexpr (GF) {
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      ga[t] = cst->alpha[t];
      guse[t] = cst->ran[t] != 0 && cst->skip[t] == 0;
    }
  }
  if (!act) {
    keep(rxr);
    keep(pAp_st);
    if (from_parts) keep(pl);
    keep(rv);
    keep(av);
    if ((FUSED || rule) && blockIdx.x == 0 && threadIdx.x == 0) st->active[(slot + 1) & 3] = 0;
    if constexpr (GF) {
      if (guse[0] || guse[1] || guse[2])
        flush_group_range<T>(n, xf->x, xf->P[0], xf->P[1], xf->P[2], xf->P[3], ga, guse, rev);
    }
    return;
  }
  const Dd<T> pd = from_parts ? parts_sum_dd(pl, np_pap, red) : Dd<T>(pAp_st);
  T pAp = pd.value();
  // (PEER without partials: the one-waiter form's k_peer_allreduce has put
  // the world p.Ap into st already)
  if (PEER && from_parts) {
    __shared__ double wres;
    __shared__ int wok;
    if (P->state->fault) {  // an earlier spin timed out: stop this body too
      peer_fault(st, slot, P);
      return;
    }
    if (!peerdev::world_sum(Dd<double>((double)pd.hi, (double)pd.lo),
                            P->state->arb[slot & 1] + 1, *P, &wres, &wok)) {
      peer_fault(st, slot, P);
      return;
    }
    pAp = (T)wres;
  }
  const T alpha = rxr / pAp;
  if (!FUSED && blockIdx.x == 0 && threadIdx.x == 0) {  // the record; the deferred x update
    st->pAp[slot] = pAp;
    st->alpha[slot] = alpha;
    st->skip[slot] = 0;
    if (rule) {  // stop rule, as k_update_xp
      const long long m = st->bodies + 1;
      st->bodies = m;
      const bool cond = isnan(rxr) || sqrt(rxr) <= st->tol;
      const bool cont = !cond && m < st->cap;
      st->active[(slot + 1) & 3] = cont ? 1 : 0;
      st->stopped = cond ? 1 : (cont ? 0 : 2);
      st->ran[slot] = 1;
    }
  }
  Dd<T> acc(T(0));  // r.r (double-length)
  for (bool first = true; i + (kUR - 1) * stride < n2; i += kUR * stride, first = false) {
    if (!first) {
#pragma unroll
      for (int u = 0; u < kUR; ++u) {
        rv[u] = ri2[E(i + u * stride)];
        av[u] = ldv<SNT, T>(a2 + E(i + u * stride));
      }
    }
#pragma unroll
    for (int u = 0; u < kUR; ++u) {
      rv[u].x = rv[u].x - alpha * av[u].x;
      rv[u].y = rv[u].y - alpha * av[u].y;
      r2[E(i + u * stride)] = rv[u];
      acc += rv[u].x * rv[u].x;
      acc += rv[u].y * rv[u].y;
    }
  }
  for (; i < n2; i += stride) {
    V rv = ri2[E(i)];
    const V av = a2[E(i)];
    rv.x = rv.x - alpha * av.x;
    rv.y = rv.y - alpha * av.y;
    r2[E(i)] = rv;
    acc += rv.x * rv.x;
    acc += rv.y * rv.y;
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const T v = rin[n - 1] - alpha * Ap[n - 1];
    r[n - 1] = v;
    acc += v * v;
  }
  if constexpr (GF) {
    ga[3] = alpha;
    guse[3] = true;
    flush_group_range<T>(n, xf->x, xf->P[0], xf->P[1], xf->P[2], xf->P[3], ga, guse, rev);
  }
  Dd<T> v = acc;
  if constexpr (!FUSED) {  // this workgroup's share of r.r; the next kernel sums them
    v = block_sum_dd(v, red);
    if (threadIdx.x == 0) {
      if (PEER && rule) {  // ... or this kernel's last workgroup (k_update_r_peer_rule)
        store_sc1(&ws->rr_part[2 * blockIdx.x], v.hi);
        store_sc1(&ws->rr_part[2 * blockIdx.x + 1], v.lo);
      } else {
        ws->rr_part[2 * blockIdx.x] = v.hi;
        ws->rr_part[2 * blockIdx.x + 1] = v.lo;
      }
    }
    return;
  }
  if (grid_reduce_dd(v, ws, red, &flag) && threadIdx.x == 0) {
    st->rr[slot] = v.value();
    if (FUSED) {
      const int nxt = (slot + 1) & 3;
      const T rxr = st->rxr[slot];
      const long long m = st->bodies + 1;
      st->bodies = m;
      const bool cond = isnan(rxr) || sqrt(rxr) <= st->tol;
      const bool cont = !cond && m < st->cap;
      st->active[nxt] = cont ? 1 : 0;
      st->rxr[nxt] = st->rr[slot];
      st->xpend[slot] = 1;
      st->stopped = cond ? 1 : (cont ? 0 : 2);
    }
  }
}

template <typename T, bool FUSED, int KP = kPartsPerThread>
__global__ __launch_bounds__(kBlock) void k_update_r(int64_t n, const T *rin, T *r,
                                                     const T *__restrict__ Ap,
                                                     CgScalars<T> *st, int slot,
                                                     RedWs<T> *ws, int np_pap, int rev,
                                                     int rule) {
  if (stream_nt<T>(n))
    update_r_body<T, FUSED, false, true, false, KP>(n, rin, r, Ap, st, slot, ws, np_pap, rev,
                                                    rule, nullptr);
  else
    update_r_body<T, FUSED, false, false, false, KP>(n, rin, r, Ap, st, slot, ws, np_pap, rev,
                                                     rule, nullptr);
}
// Mode 4, slot 3: update_r with the stop rule and the group's x flush in one
// launch (k_flush_group's values, bit for bit)
template <typename T, int KP = kPartsPerThread>
__global__ __launch_bounds__(kBlock) void k_update_r_flush(int64_t n, T *r,
                                                           const T *__restrict__ Ap,
                                                           CgScalars<T> *st, int slot,
                                                           RedWs<T> *ws, int np_pap, int rev,
                                                           XFlush<T> xf) {
  if (stream_nt<T>(n))
    update_r_body<T, false, false, true, true, KP>(n, r, r, Ap, st, slot, ws, np_pap, rev, 1,
                                                   nullptr, &xf);
  else
    update_r_body<T, false, false, false, true, KP>(n, r, r, Ap, st, slot, ws, np_pap, rev, 1,
                                                    nullptr, &xf);
}
template <typename T>
__global__ __launch_bounds__(kBlock) void k_update_r_peer(int64_t n, T *r,
                                                          const T *__restrict__ Ap,
                                                          CgScalars<T> *st, int slot,
                                                          RedWs<T> *ws, int np_pap, int rev,
                                                          PeerDev P) {
  if (stream_nt<T>(n))
    update_r_body<T, false, true, true>(n, r, r, Ap, st, slot, ws, np_pap, rev, 0, &P);
  else
    update_r_body<T, false, true, false>(n, r, r, Ap, st, slot, ws, np_pap, rev, 0, &P);
}
// true in the workgroup of the grid that arrives last (two-level tickets as
// grid_reduce: ticket[b % kRedGroups], then top; each reset by its last
// arrival). Thread 0 of every workgroup has issued its sc1 stores before.
template <typename T> __device__ __forceinline__ bool last_arrival(RedWs<T> *ws, int *flag) {
  const unsigned G = gridDim.x, g = blockIdx.x % kRedGroups;
  const unsigned ngroups = G < (unsigned)kRedGroups ? G : (unsigned)kRedGroups;
  const unsigned members = (G - g + kRedGroups - 1) / kRedGroups;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bool last = __hip_atomic_fetch_add(&ws->ticket[g], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT) == members - 1;
    if (last) {
      __hip_atomic_store(&ws->ticket[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = __hip_atomic_fetch_add(&ws->top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             ngroups - 1;
      if (last) __hip_atomic_store(&ws->top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// Mode 4 on a partitioned matrix, kernel 3 of 3: update_r with the p.Ap
// all-reduce (tag base + 1) and the stop rule; in slot 3 (GF) the group's x
// flush as k_update_r_flush. The workgroup that finishes last sums the r.r
// partials (sum_parts order over sc1 loads: mode 3's value) and all-reduces
// them (tag base + 2, as mode 3's p update), records the world r.r where the
// next body's kernels 1 and 2 read it (rxr[s+1]) and sets the next body's
// tag base: one workgroup waits on the other ranks, not a whole grid.
template <typename T, bool GF>
__global__ __launch_bounds__(kBlock) void k_update_r_peer_rule(int64_t n, T *r,
                                                               const T *__restrict__ Ap,
                                                               CgScalars<T> *st, int slot,
                                                               RedWs<T> *ws, int np_pap, int rev,
                                                               PeerDev P, XFlush<T> xf) {
  if (stream_nt<T>(n))
    update_r_body<T, false, true, true, GF>(n, r, r, Ap, st, slot, ws, np_pap, rev, 1, &P, &xf);
  else
    update_r_body<T, false, true, false, GF>(n, r, r, Ap, st, slot, ws, np_pap, rev, 1, &P, &xf);
  // every workgroup arrives, whichever way it left the body (a ticket left
  // short would break the next grid reduction on this workspace)
  __shared__ int lastf;
  if (!last_arrival(ws, &lastf)) return;
  // another workgroup of this launch may have faulted on the p.Ap wait after
  // this one read the flag: read it again past the cache
  if (!st->active[slot] ||
      __hip_atomic_load(&P.state->fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    return;
  __shared__ T red[8];
  __shared__ T bc[2];
  Dd<T> v(T(0));
  for (int i = threadIdx.x; i < (int)gridDim.x; i += kBlock)
    v += Dd<T>(load_sc1(&ws->rr_part[2 * i]), load_sc1(&ws->rr_part[2 * i + 1]));
  v = block_sum_dd(v, red);
  if (threadIdx.x == 0) {
    bc[0] = v.hi;
    bc[1] = v.lo;
  }
  __syncthreads();
  const unsigned long long t = P.state->arb[slot & 1] + 2;
  __shared__ double wres;
  __shared__ int wok;
  const bool ok = peerdev::world_sum(Dd<double>((double)bc[0], (double)bc[1]), t, P, &wres, &wok);
  if (threadIdx.x == 0) {
    if (!ok) {
      P.state->fault = 1;
      st->tail_fault = 1;
      return;
    }
    const T w = (T)wres;
    st->rr[slot] = w;  // the record
    st->rxr[(slot + 1) & 3] = w;
    P.state->ar = t;
    P.state->arb[(slot + 1) & 1] = t;
  }
}

// x = x + alpha p ; p = r + beta p ; stop rule   (CG.hpp:390, 396-418, 436)
template <typename T, bool PEER>
__device__ __forceinline__ void update_xp_body(int64_t n, T *__restrict__ x, T *__restrict__ p,
                                               const T *__restrict__ r, CgScalars<T> *st,
                                               int slot, RedWs<T> *ws, int np_rr, int rev,
                                               const PeerDev *P) {
  const int nxt = (slot + 1) & 3;
  if (!st->active[slot]) {
    if (blockIdx.x == 0 && threadIdx.x == 0) st->active[nxt] = 0;
    return;
  }
  __shared__ T red[8];
  const T rxr = st->rxr[slot];
  const T alpha = rxr / st->pAp[slot];
  const Dd<T> rd = np_rr > 0 ? sum_parts_dd(ws->rr_part, np_rr, red) : Dd<T>(st->rr[slot]);
  T rr = rd.value();
  if constexpr (PEER) {  // r.r all-reduced here (tag base + 2)
    __shared__ double wres;
    __shared__ int wok;
    if (P->state->fault) {  // an earlier spin timed out: stop this body too
      peer_fault(st, slot, P);
      return;
    }
    if (!peerdev::world_sum(Dd<double>((double)rd.hi, (double)rd.lo), P->state->arb[slot & 1] + 2, *P, &wres,
                            &wok)) {
      peer_fault(st, slot, P);
      return;
    }
    rr = (T)wres;
  }
  const T beta = rr / rxr;
  using V = typename Vec2<T>::V;
  const int64_t n2 = n >> 1;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  V *x2 = reinterpret_cast<V *>(x);
  V *p2 = reinterpret_cast<V *>(p);
  const V *rv2 = reinterpret_cast<const V *>(r);
  auto E = [&](int64_t j) { return rev ? n2 - 1 - j : j; };  // sweep direction
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  for (; i + 3 * stride < n2; i += 4 * stride) {
    V xv[4], pv[4], rv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      xv[u] = x2[E(i + u * stride)];
      pv[u] = p2[E(i + u * stride)];
      rv[u] = rv2[E(i + u * stride)];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      xv[u].x = xv[u].x + alpha * pv[u].x;
      xv[u].y = xv[u].y + alpha * pv[u].y;
      pv[u].x = rv[u].x + beta * pv[u].x;
      pv[u].y = rv[u].y + beta * pv[u].y;
      x2[E(i + u * stride)] = xv[u];
      p2[E(i + u * stride)] = pv[u];
    }
  }
  for (; i < n2; i += stride) {
    V xv = x2[E(i)], pv = p2[E(i)];
    const V rv = rv2[E(i)];
    xv.x = xv.x + alpha * pv.x;
    xv.y = xv.y + alpha * pv.y;
    pv.x = rv.x + beta * pv.x;
    pv.y = rv.y + beta * pv.y;
    x2[E(i)] = xv;
    p2[E(i)] = pv;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (n & 1) {
      const T pv = p[n - 1];
      x[n - 1] = x[n - 1] + alpha * pv;
      p[n - 1] = r[n - 1] + beta * pv;
    }
    if (np_rr > 0) st->rr[slot] = rr;  // the record
    const long long m = st->bodies + 1;
    st->bodies = m;
    const bool cond = isnan(rxr) || sqrt(rxr) <= st->tol;
    const bool cont = !cond && m < st->cap;
    st->active[nxt] = cont ? 1 : 0;
    st->rxr[nxt] = rr;
    st->stopped = cond ? 1 : (cont ? 0 : 2);
    if constexpr (PEER) {  // the next body's tag base
      const unsigned long long t = P->state->arb[slot & 1] + 2;
      P->state->ar = t;
      P->state->arb[(slot + 1) & 1] = t;
    }
  }
}
template <typename T>
__global__ __launch_bounds__(kBlock) void k_update_xp(int64_t n, T *__restrict__ x,
                                                      T *__restrict__ p,
                                                      const T *__restrict__ r,
                                                      CgScalars<T> *st, int slot,
                                                      RedWs<T> *ws, int np_rr, int rev) {
  update_xp_body<T, false>(n, x, p, r, st, slot, ws, np_rr, rev, nullptr);
}
template <typename T>
__global__ __launch_bounds__(kBlock) void k_update_xp_peer(int64_t n, T *__restrict__ x,
                                                           T *__restrict__ p,
                                                           const T *__restrict__ r,
                                                           CgScalars<T> *st, int slot,
                                                           RedWs<T> *ws, int np_rr, int rev,
                                                           PeerDev P) {
  update_xp_body<T, true>(n, x, p, r, st, slot, ws, np_rr, rev, &P);
}

// *res += x.y (dot_product_trivial / norm: accumulate, Q4)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_dot_acc(int64_t n, const T *__restrict__ x,
                                                    const T *__restrict__ y, T *res,
                                                    RedWs<T> *ws) {
  __shared__ T red[8];
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

// SELL values: slot j of row i = val[rowptr[i] + j], 0 past the row's end
// (those slots carry the padding index, the SpMV never multiplies them).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_sell_pack(int64_t n, int64_t nsl, int R,
                                                      const int *__restrict__ rowptr,
                                                      const T *__restrict__ val,
                                                      const SellSlice *__restrict__ sl,
                                                      T *__restrict__ sval) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t H = (int64_t)kSellRows * R;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nsl * H; i += stride) {
    const SellSlice m = sl[i / H];
    const int li = (int)(i % H), l = li / R, r = li % R;
    const int a = i < n ? rowptr[i] : 0;
    const int len = i < n ? rowptr[i + 1] - a : 0;
    for (int j = 0; j < m.width; ++j)
      sval[m.voff + ((int64_t)j * kSellRows + l) * R + r] = j < len ? val[a + j] : T(0);
  }
}

// SELL-P values and masks: row i of slice q puts entry (col c) in the slot of
// offset c - i in the slice's pattern (both ascending), zero elsewhere, and
// sets that slot's mask bit. Rows past n: zeros, mask 0.
template <typename T, typename MT>
__global__ __launch_bounds__(kBlock) void k_sellp_pack(int64_t n, int64_t nsl,
                                                       const int *__restrict__ rowptr,
                                                       const int *__restrict__ col,
                                                       const T *__restrict__ val,
                                                       const SellSlice *__restrict__ sl,
                                                       const int *__restrict__ pat,
                                                       T *__restrict__ sval, MT *__restrict__ mask) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t H = 2 * kSellRows;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nsl * H; i += stride) {
    const SellSlice m = sl[i / H];
    const int li = (int)(i % H), l = li >> 1, r = li & 1;
    const int *P = pat + m.dict;
    int a = 0, e = 0;
    if (i < n) {
      a = rowptr[i];
      e = rowptr[i + 1];
    }
    unsigned bits = 0;
    int k = a;
    for (int j = 0; j < m.width; ++j) {
      T v = T(0);
      if (k < e && col[k] - (int)i == P[j]) {
        v = val[k++];
        bits |= 1u << j;
      }
      sval[m.voff + ((int64_t)j * kSellRows + l) * 2 + r] = v;
    }
    mask[i] = (MT)bits;
  }
}

// SELL-P plan on the device (cgx_abi.cpp sellp_plan_device; the host
// restatement is sellp_plan_host, which the CPU tests and cgx_sellp_plan
// keep): one wave per 128-row slice (2 rows per lane, as the SELL-P layout)
// forms the ascending union of its rows' (col - row) offsets by repeated
// wave minima above the last offset taken (at most kSellPatMax + 1 rounds),
// and checks that every row has strictly ascending columns (slices marked in
// skip are exempt). w[q]: the pattern's width (0: no entries), kSellPatMax +
// 1 when it has more offsets, -1 for an unsorted row; pat[q * kSellPatMax +
// j]: the offsets. No column array crosses to the host (256^3: 468 MB).
__global__ __launch_bounds__(kBlock) void k_sellp_plan(int64_t n, int64_t nsl,
                                                       const int *__restrict__ rowptr,
                                                       const int *__restrict__ col,
                                                       const char *__restrict__ skip,
                                                       int *__restrict__ pat,
                                                       int *__restrict__ w) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (q >= nsl) return;  // wave-uniform
  const int64_t i0 = q * 2 * kSellRows + 2 * lane;
  int a[2], e[2];
  bool bad = false;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    a[r] = e[r] = 0;
    if (i0 + r < n) {
      a[r] = rowptr[i0 + r];
      e[r] = rowptr[i0 + r + 1];
    }
    for (int k = a[r] + 1; k < e[r]; ++k) bad = bad || col[k] <= col[k - 1];
  }
  if (__any(bad) && !(skip && skip[q])) {
    if (lane == 0) w[q] = -1;
    return;
  }
  long long last = LLONG_MIN;
  int cnt = 0;
  for (;;) {
    long long m = LLONG_MAX;
#pragma unroll
    for (int r = 0; r < 2; ++r)
      for (int k = a[r]; k < e[r]; ++k) {
        const long long off = (long long)col[k] - (i0 + r);
        if (off > last && off < m) m = off;
      }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const long long t = __shfl_xor(m, o, 64);
      m = t < m ? t : m;
    }
    if (m == LLONG_MAX) break;
    if (cnt == kSellPatMax) {
      cnt = kSellPatMax + 1;
      break;
    }
    if (lane == 0) pat[q * kSellPatMax + cnt] = (int)m;
    ++cnt;
    last = m;
  }
  if (lane == 0) w[q] = cnt;
}

// SELL-P value codes: the slot layout of k_sellp_pack, each stored value
// replaced by its index in the sorted dictionary `dict` of nd bit patterns
// (binary search on the bits: -0.0 / 0.0 and NaN payloads stay distinct);
// empty slots and rows past n: kVcAbsent. A value not in the dictionary
// counts in *miss and the first kVcDict of them land in missv (the host adds
// them to the dictionary and packs again, or drops the codes).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_sellpv_pack(int64_t n, int64_t nsl,
                                                        const int *__restrict__ rowptr,
                                                        const int *__restrict__ col,
                                                        const T *__restrict__ val,
                                                        const SellSlice *__restrict__ sl,
                                                        const int *__restrict__ pat,
                                                        const T *__restrict__ dict, int nd,
                                                        unsigned char *__restrict__ codes,
                                                        int *miss, T *missv) {
  using B = typename Bits<T>::U;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t H = 2 * kSellRows;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nsl * H; i += stride) {
    const SellSlice m = sl[i / H];
    const int li = (int)(i % H), l = li >> 1, r = li & 1;
    const int *P = pat + m.dict;
    int a = 0, e = 0;
    if (i < n) {
      a = rowptr[i];
      e = rowptr[i + 1];
    }
    int k = a;
    const int W8 = (m.width + 7) & ~7;
    for (int j = 0; j < W8; ++j) {
      unsigned code = kVcAbsent;
      if (j < m.width && k < e && col[k] - (int)i == P[j]) {
        const B vb = __builtin_bit_cast(B, val[k++]);
        int lo = 0, hi = nd;  // first dictionary entry >= vb
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (__builtin_bit_cast(B, dict[mid]) < vb) lo = mid + 1;
          else hi = mid;
        }
        if (lo < nd && __builtin_bit_cast(B, dict[lo]) == vb) code = (unsigned)lo;
        else {
          const int q = atomicAdd(miss, 1);
          if (q < kVcDict) missv[q] = val[k - 1];
        }
      }
      codes[(m.ioff + (int64_t)(j >> 3) * kSellRows + l) * 16 + 2 * (j & 7) + r] =
          (unsigned char)code;
    }
  }
}

// 4-bit value codes from the 8-bit ones (dictionary of at most kVc4Max
// values): chunk-lane t's 16 bytes (slot j: bytes 2 j, 2 j + 1 for rows 0, 1)
// become 8 bytes, byte j = row 0's code | row 1's code << 4, kVcAbsent -> 0xf.
__global__ __launch_bounds__(kBlock) void k_vc_narrow(const unsigned char *__restrict__ c8,
                                                      unsigned char *__restrict__ c4,
                                                      int64_t chunks) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < chunks; t += stride) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned a = c8[t * 16 + 2 * j], b = c8[t * 16 + 2 * j + 1];
      c4[t * 8 + j] = (unsigned char)((a == kVcAbsent ? 0xfu : a) |
                                      ((b == kVcAbsent ? 0xfu : b) << 4));
    }
  }
}

// ---- value-code templates (kVT, cgx_abi.cpp build_value_templates) --------
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ unsigned long long wave_xor64(unsigned long long h) {
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)h, o, 64);
    const unsigned hi = (unsigned)__shfl_xor((int)(unsigned)(h >> 32), o, 64);
    h ^= ((unsigned long long)hi << 32) | lo;
  }
  return h;
}
// one wave per slice: a hash of its 64-word 4-bit code chunk (0: the slice
// is wider than one chunk, no template)
__global__ __launch_bounds__(kBlock) void k_vc_hash(const SellSlice *__restrict__ sl, int64_t nsl,
                                                    const unsigned long long *__restrict__ c4,
                                                    unsigned long long *__restrict__ hash) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (s >= nsl) return;  // wave-uniform
  const SellSlice m = sl[s];
  unsigned long long h = 0;
  if (m.width <= 8) h = mix64(c4[m.ioff + lane] ^ (0x9E3779B97F4A7C15ull * (unsigned)(lane + 1)));
  h = wave_xor64(h);
  if (lane == 0) hash[s] = m.width <= 8 ? (h ? h : 1) : 0;
}
// one wave per slice: the template slice table — slice s's descriptor with
// (t + 1) << 16 added to its width when its chunk equals template t in
// every byte (checked here, whatever the hashes said), else unchanged;
// *count: matched slices
__global__ __launch_bounds__(kBlock) void k_vc_match(const SellSlice *__restrict__ sl, int64_t nsl,
                                                     const unsigned long long *__restrict__ c4,
                                                     const unsigned long long *__restrict__ tmpl,
                                                     int nt, SellSlice *__restrict__ sl_t,
                                                     unsigned *count) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (s >= nsl) return;  // wave-uniform
  SellSlice m = sl[s];
  int hit = -1;
  if (m.width <= 8) {
    const unsigned long long w = c4[m.ioff + lane];
    for (int t = 0; t < nt && hit < 0; ++t)
      if (__all(w == tmpl[t * 64 + lane])) hit = t;
  }
  if (lane == 0) {
    if (hit >= 0) {
      m.width |= (hit + 1) << 16;
      atomicAdd(count, 1u);
    }
    sl_t[s] = m;
  }
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

inline CsrArgs args(const CsrDev &A) {
  CsrArgs a{A.rowptr, A.col,   A.rb,   A.rbk,  A.nrb,  A.n,
            A.sl,     A.sdict, A.sidx, A.sval, A.nsl, A.sorder, 0, 0,
            A.smask,  A.nx > 0 ? A.nx : A.n, A.svc, A.svdict, A.svc4,
            A.march_k, A.march_a, A.march_pat, A.march_len};
  if (vt_active(A)) {  // the same condition spmv_variant keeps kVT under
    a.sl = A.sl_t;
    a.vct = static_cast<const unsigned long long *>(A.vct);
    a.nvt = A.nvt;
  }
  a.col16 = A.col16;
  a.rbo = A.rbo;
  a.il = A.il;
  if (vl_active(A)) {
    a.vl_cls = A.vl_cls;
    a.vl_tab = A.vl_tab;
    a.vl_nst = A.vl_nst;
    a.vl_D = A.vl_D;
    a.vl_a = A.vl_a;
    a.vl_P = A.vl_P;
    a.vl_K = A.vl_K;
    a.vl_lds = A.vl_lds;
  }
  return a;
}

}  // namespace

hipError_t sellp_plan_dev(int64_t n, int64_t nsl, const int *rowptr, const int *col,
                          const char *skip, int *pat, int *w, hipStream_t s) {
  const int64_t per = kBlock / 64;
  CGX_GGL(k_sellp_plan, dim3((unsigned)((nsl + per - 1) / per)), dim3(kBlock), 0, s, n, nsl,
          rowptr, col, skip, pat, w);
  return hipGetLastError();
}

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
// Streaming kernels: at most `cap` workgroups, each walking its share in a
// grid-stride loop. Fewer, longer-lived workgroups stream better than the
// 8-per-CU persistent grid the SpMV uses: k_update_r 256 (1 per CU), the
// x/p updates 512 (2 per CU; the flushing body keeps 8 streams in flight);
// A/B in DESIGN.md §4 (gpurun_out r44/r45).
constexpr int kGridUpdateR = 256;
constexpr int kGridUpdateP = 512;
template <typename T> int Launch<T>::grid_elems(int64_t n, int cap) {
  int64_t g = (n + (int64_t)kBlock * 8 - 1) / ((int64_t)kBlock * 8);
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}


// Deferred-x iteration (mode 3), kernel 3 of 3 for body k in slot s:
// p_{k+1} = r + beta p_k into the next of four p buffers (CG.hpp:418) and
// the stop rule (CG.hpp:396-404, 410-417, 436) as in k_update_xp, but the x
// update (CG.hpp:390) is applied once per four bodies: in slot 3 (FLUSH),
// x = (((x + a0 p0) + a1 p1) + a2 p2) + a3 p3 over the slots an end-of-run
// flush has not applied yet — per element the same rounded operations in
// the same order as four in-place updates, so x is bit-identical, for
// 8 N + 8 N (x) + 24 N (p0..p2) bytes once instead of 16 N four times.
// In slot 3, pn is P0 (p_{k+1} replaces p_{k-3}): every element's flush
// operands are loaded before its stores, and pn / P0 carry no __restrict__.
template <typename T, bool FLUSH, bool PEER, bool SNT>
__device__ __forceinline__ void update_p_defer_body(int64_t n, T *__restrict__ x, const T *p,
                                                    T *pn, const T *P0, const T *P1,
                                                    const T *P2, const T *__restrict__ r,
                                                    CgScalars<T> *st, int slot, RedWs<T> *ws,
                                                    int np_rr, int rev, const PeerDev *PD) {
  const int nxt = (slot + 1) & 3;
  // the flag, rxr and the r.r partials in one round trip
  const auto *cst = (const __attribute__((address_space(4))) CgScalars<T> *)st;
  const bool act = cst->active[slot] != 0;
  const T rxr = cst->rxr[slot];
  const T rr_st = cst->rr[slot];
  Dd<T> pl[kPartsPerThread];
  if (np_rr > 0) parts_load_np(ws->rr_part, np_rr, pl);
  using V = typename Vec2<T>::V;
  const int64_t n2 = n >> 1;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  auto E = [&](int64_t j) { return rev ? n2 - 1 - j : j; };  // sweep direction
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  // the non-flushing body: this thread's first four elements of p_k and r
  // go out with the partials, before beta (as update_r's first block), so
  // their round trip overlaps the partial sum
  V pv0[4], rv0[4];
  if constexpr (!FLUSH) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // clamped (p and r have a slack element): no branch
      const int64_t j = E(min(i + u * stride, n2 > 0 ? n2 - 1 : 0));
      pv0[u] = ldv<SNT, T>(reinterpret_cast<const V *>(p) + j);
      rv0[u] = ldv<SNT, T>(reinterpret_cast<const V *>(r) + j);
    }
  }
  if (!act) {
    keep(rxr);
    keep(rr_st);
    if (np_rr > 0) keep(pl);
    if constexpr (!FLUSH) {
      keep(pv0);
      keep(rv0);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) st->active[nxt] = 0;
    return;
  }
  __shared__ T red[8];
  const Dd<T> rd = np_rr > 0 ? parts_sum_dd(pl, np_rr, red) : Dd<T>(rr_st);
  T rr = rd.value();
  if constexpr (PEER) {  // r.r all-reduced here (tag base + 2)
    __shared__ double wres;
    __shared__ int wok;
    if (PD->state->fault) {  // an earlier spin timed out: stop this body too
      peer_fault(st, slot, PD);
      return;
    }
    if (!peerdev::world_sum(Dd<double>((double)rd.hi, (double)rd.lo), PD->state->arb[slot & 1] + 2, *PD,
                            &wres, &wok)) {
      peer_fault(st, slot, PD);
      return;
    }
    rr = (T)wres;
  }
  const T beta = rr / rxr;
  // slot-3 flush: alphas and skips of the group, written by earlier launches
  T a[4] = {T(0), T(0), T(0), T(0)};
  bool use[4] = {false, false, false, false};
  if constexpr (FLUSH) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      a[t] = st->alpha[t];
      use[t] = st->skip[t] == 0;
    }
  }
  const V *p2 = reinterpret_cast<const V *>(p);
  V *pn2 = reinterpret_cast<V *>(pn);
  const V *rv2 = reinterpret_cast<const V *>(r);
  V *x2 = reinterpret_cast<V *>(x);
  const V *Q[3] = {reinterpret_cast<const V *>(P0), reinterpret_cast<const V *>(P1),
                   reinterpret_cast<const V *>(P2)};
  auto body = [&](int64_t i) {
    // r and p_k are not re-read before the next SpMV and update_r have
    // streamed them out of the Infinity Cache: non-temporal loads leave it
    // to p_{k+1}, which the next SpMV reads first (+2.9% per iteration at
    // 256^3: SpMV 90.3 against 93.2 us, this kernel 88.4 against 91.3;
    // profiles/r02_pupd_nt.log)
    const V pv = ldv<SNT, T>(p2 + i);
    const V rv = ldv<SNT, T>(rv2 + i);
    V q[3], xv;
    if constexpr (FLUSH) {  // x and the old p buffers: not read again soon
      xv = ldv<SNT, T>(x2 + i);
#pragma unroll
      for (int t = 0; t < 3; ++t) q[t] = ldv<SNT, T>(Q[t] + i);  // before pn (= P0) is written
    }
    V o;
    o.x = rv.x + beta * pv.x;
    o.y = rv.y + beta * pv.y;
    if constexpr (FLUSH) {
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        if (use[t]) {
          xv.x = xv.x + a[t] * q[t].x;
          xv.y = xv.y + a[t] * q[t].y;
        }
      }
      if (use[3]) {
        xv.x = xv.x + a[3] * pv.x;
        xv.y = xv.y + a[3] * pv.y;
      }
      stv<SNT, T>(x2 + i, xv);
    }
    pn2[i] = o;
  };
  if constexpr (!FLUSH) {
    // the first block from the early loads (a block past the end: its
    // clamped loads are not stored)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i + u * stride < n2) {
        V o;
        o.x = rv0[u].x + beta * pv0[u].x;
        o.y = rv0[u].y + beta * pv0[u].y;
        pn2[E(i + u * stride)] = o;
      }
    }
    i += 4 * stride;
  }
  for (; i + 3 * stride < n2; i += 4 * stride) {
#pragma unroll
    for (int u = 0; u < 4; ++u) body(E(i + u * stride));
  }
  for (; i < n2; i += stride) body(E(i));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (n & 1) {
      const T pv = p[n - 1];
      if constexpr (FLUSH) {
        T xv = x[n - 1];
        const T *Ps[4] = {P0, P1, P2, p};
        for (int t = 0; t < 4; ++t)
          if (use[t]) xv = xv + a[t] * Ps[t][n - 1];
        x[n - 1] = xv;
      }
      pn[n - 1] = r[n - 1] + beta * pv;
    }
    // stop rule, as k_update_xp
    if (np_rr > 0) st->rr[slot] = rr;  // the record
    const long long m = st->bodies + 1;
    st->bodies = m;
    const bool cond = isnan(rxr) || sqrt(rxr) <= st->tol;
    const bool cont = !cond && m < st->cap;
    st->active[nxt] = cont ? 1 : 0;
    st->rxr[nxt] = rr;
    st->stopped = cond ? 1 : (cont ? 0 : 2);
    if constexpr (FLUSH) {
      for (int t = 0; t < 4; ++t) st->ran[t] = 0;
    } else {
      st->ran[slot] = 1;
    }
    if constexpr (PEER) {  // the next body's tag base
      const unsigned long long t = PD->state->arb[slot & 1] + 2;
      PD->state->ar = t;
      PD->state->arb[(slot + 1) & 1] = t;
    }
  }
}
template <typename T, bool FLUSH>
__global__ __launch_bounds__(kBlock) void k_update_p_defer(int64_t n, T *__restrict__ x,
                                                           const T *p, T *pn, const T *P0,
                                                           const T *P1, const T *P2,
                                                           const T *__restrict__ r,
                                                           CgScalars<T> *st, int slot,
                                                           RedWs<T> *ws, int np_rr, int rev) {
  if (stream_nt<T>(n))
    update_p_defer_body<T, FLUSH, false, true>(n, x, p, pn, P0, P1, P2, r, st, slot, ws, np_rr,
                                               rev, nullptr);
  else
    update_p_defer_body<T, FLUSH, false, false>(n, x, p, pn, P0, P1, P2, r, st, slot, ws, np_rr,
                                                rev, nullptr);
}
template <typename T, bool FLUSH>
__global__ __launch_bounds__(kBlock) void k_update_p_defer_peer(
    int64_t n, T *__restrict__ x, const T *p, T *pn, const T *P0, const T *P1, const T *P2,
    const T *__restrict__ r, CgScalars<T> *st, int slot, RedWs<T> *ws, int np_rr, int rev,
    PeerDev PD) {
  if (stream_nt<T>(n))
    update_p_defer_body<T, FLUSH, true, true>(n, x, p, pn, P0, P1, P2, r, st, slot, ws, np_rr,
                                              rev, &PD);
  else
    update_p_defer_body<T, FLUSH, true, false>(n, x, p, pn, P0, P1, P2, r, st, slot, ws, np_rr,
                                               rev, &PD);
}

// End of a run in mode 3: apply the bodies of the current group that ran and
// were not applied yet, in slot order. k_mark_defer then marks them applied
// (a separate launch: the workgroups here read the marks).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_flush_defer(int64_t n, T *__restrict__ x,
                                                        const T *__restrict__ P0,
                                                        const T *__restrict__ P1,
                                                        const T *__restrict__ P2,
                                                        const T *__restrict__ P3,
                                                        const CgScalars<T> *st) {
  T a[4];
  bool use[4];
  bool any = false;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    a[t] = st->alpha[t];
    use[t] = st->ran[t] != 0 && st->skip[t] == 0;
    any = any || use[t];
  }
  if (!any) return;
  // 16-byte lanes, the group flush's loop (the end of the driver's 20-body
  // bench window pays this launch: 8-byte lanes took 75.6 us at 256^3, r04d)
  flush_group_range<T>(n, x, P0, P1, P2, P3, a, use, 0);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_flush_group(int64_t n, T *__restrict__ x,
                                                        const T *__restrict__ P0,
                                                        const T *__restrict__ P1,
                                                        const T *__restrict__ P2,
                                                        const T *__restrict__ P3,
                                                        const CgScalars<T> *st, int rev) {
  T a[4];
  bool use[4];
  bool any = false;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    a[t] = st->alpha[t];
    use[t] = st->ran[t] != 0 && st->skip[t] == 0;
    any = any || use[t];
  }
  if (!any) return;
  flush_group_range<T>(n, x, P0, P1, P2, P3, a, use, rev);
}

// *dst = sum of part[0..np) in sum_parts order (partitioned runs: the local
// dot before its RCCL all-reduce)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_finalize(const T *__restrict__ part, int np, T *dst) {
  __shared__ T red[8];
  const T v = sum_parts(part, np, red);
  if (threadIdx.x == 0) *dst = v;
}

template <typename T> __global__ void k_mark_defer(CgScalars<T> *st) {
  for (int t = 0; t < 4; ++t)
    if (st->ran[t]) st->skip[t] = 1;
}

#define CGX_LAUNCH(kernel, grid, ...)                                              \
  do {                                                                             \
    CGX_GGL(kernel, dim3(grid), dim3(kBlock), 0, s, __VA_ARGS__);       \
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
  if (v < 0 && A.variant > 0) v = A.variant;  // chosen by cgx_csr_create's autotune
  if (v >= 0 && (v & (2048 | 8192))) {
    // the variant follows the SELL copy's layout: bit 4096 for 2 rows per
    // lane; pipelined (bit 8) for 1 row per lane and slices <= 8 wide
    if (A.sl && A.sell_kind && (v & 32768) && A.svc)
      return 32768 | 8192 |
             (v & (16 | 2 | 65536 | 131072 | (A.svc4 ? 262144 : 0) |
                   (A.sell_maxw <= 8 ? 524288 | 1048576 : 0) |
                   (A.sell_maxw <= 8 && A.march_k > 0 ? 2097152 : 0))) |
             (vt_active(A) ? kVT : 0);
    if (A.sl && A.sell_kind) return 8192 | (A.sell_kind == 2 ? 16384 : 0) | (v & (16 | 2));
    if (A.sl && A.sell_r == 2) return 2048 | 4096 | (v & (16 | 2));
    if (A.sl) return v & (2048 | 16 | 2 | (A.sell_maxw <= 8 ? 8 : 0));
    v = -1;  // no SELL copy: CSR-stream
  }
  if (v < 0) v = (A.nnz * int64_t(sizeof(T) + sizeof(int)) >= kNtMinBytes) ? 15 : 13;
  // bits 16/32: timing ablations, only reachable through cgx_tune_spmv; the
  // retired half-tile (64), three-stage (128) and wave-tile (512) bits drop
  // (a schedule built for smaller tiles fits the full-tile kernels)
  const bool c16 = (v & kC16) && A.col16 && (v & 4) && !(v & (8 | 256));
  // the interleaved copy: the pipelined paired loop only (13 | kIL, 15 | kIL)
  const bool il = (v & kIL) && A.il && (v & 12) == 12 && !(v & (256 | kC16)) && A.nnz >= 2;
  v &= 1023 & ~(64 | 128 | 512);
  if (il) return v | kIL;
  if (((uintptr_t)A.val % (2 * sizeof(T))) || ((uintptr_t)A.col % 8) || A.nnz < 2)
    return 0;  // plain loads, no pipelining (any schedule with <= 2042-entry blocks)
  if (c16) return v | kC16;  // 132..135: paired loop, 16-bit column deltas
  if ((v & 256) && (((uintptr_t)A.val % (4 * sizeof(T))) || ((uintptr_t)A.col % 16) ||
                    A.nnz < 4))
    v &= ~256;  // quads need 4-entry alignment
  if (v & 256) return 256 | 8 | (v & 3);  // 264..267
  if ((v & 8) && !(v & 4)) v &= ~8;  // the pipelined loop uses paired loads
  return v;
}

#define CGX_LAUNCH_V(KERNEL, VV, ...)                                          \
  do {                                                                         \
    CGX_GGL((KERNEL<T, VV>), dim3(spmv_grid_), dim3(kBlock), 0, s,   \
                       __VA_ARGS__);                                           \
    return hipGetLastError();                                                  \
  } while (0)

// The SpMV forms k_spmv_dot is instantiated for (and cgx_csr_set_variant
// accepts, cgx_abi.cpp known_variant): CSR-stream 0-7 (bits 1 XCD split, 2
// non-temporal, 4 paired loads), 12-15 (+8 pipelined), 264-267 (quads);
// dictionary SELL 2048/2050/2056/2058/6144/6146; SELL-P 8192/8194 (+16384:
// 24576/24578); value-code SELL-P and its pipelined / stencil / plane-march
// loops. (Round 1's half-tile, three-stage and wave-tile CSR forms and
// round 3's row-gather form, negative results recorded in DESIGN.md §8, are
// not built.) One-off
// kernels (cg init, accuracy) run CSR-stream: every form gives the same
// per-row sums.
#define CGX_SPMV_SWITCH(v, KERNEL, ...)                        \
  switch (v) {                                                 \
    case 0: CGX_LAUNCH_V(KERNEL, 0, __VA_ARGS__);              \
    case 1: CGX_LAUNCH_V(KERNEL, 1, __VA_ARGS__);              \
    case 2: CGX_LAUNCH_V(KERNEL, 2, __VA_ARGS__);              \
    case 3: CGX_LAUNCH_V(KERNEL, 3, __VA_ARGS__);              \
    case 4: CGX_LAUNCH_V(KERNEL, 4, __VA_ARGS__);              \
    case 5: CGX_LAUNCH_V(KERNEL, 5, __VA_ARGS__);              \
    case 6: CGX_LAUNCH_V(KERNEL, 6, __VA_ARGS__);              \
    case 7: CGX_LAUNCH_V(KERNEL, 7, __VA_ARGS__);              \
    case 12: CGX_LAUNCH_V(KERNEL, 12, __VA_ARGS__);            \
    case 13: CGX_LAUNCH_V(KERNEL, 13, __VA_ARGS__);            \
    case 14: CGX_LAUNCH_V(KERNEL, 14, __VA_ARGS__);            \
    case 15: CGX_LAUNCH_V(KERNEL, 15, __VA_ARGS__);            \
    case 264: CGX_LAUNCH_V(KERNEL, 264, __VA_ARGS__);          \
    case 265: CGX_LAUNCH_V(KERNEL, 265, __VA_ARGS__);          \
    case 266: CGX_LAUNCH_V(KERNEL, 266, __VA_ARGS__);          \
    case 267: CGX_LAUNCH_V(KERNEL, 267, __VA_ARGS__);          \
    case 133: CGX_LAUNCH_V(KERNEL, 133, __VA_ARGS__);          \
    case 67108877: CGX_LAUNCH_V(KERNEL, 67108877, __VA_ARGS__);\
    case 67108879: CGX_LAUNCH_V(KERNEL, 67108879, __VA_ARGS__);\
    case 135: CGX_LAUNCH_V(KERNEL, 135, __VA_ARGS__);          \
    case 2048: CGX_LAUNCH_V(KERNEL, 2048, __VA_ARGS__);        \
    case 2050: CGX_LAUNCH_V(KERNEL, 2050, __VA_ARGS__);        \
    case 2056: CGX_LAUNCH_V(KERNEL, 2056, __VA_ARGS__);        \
    case 2058: CGX_LAUNCH_V(KERNEL, 2058, __VA_ARGS__);        \
    case 6144: CGX_LAUNCH_V(KERNEL, 6144, __VA_ARGS__);        \
    case 6146: CGX_LAUNCH_V(KERNEL, 6146, __VA_ARGS__);        \
    case 8192: CGX_LAUNCH_V(KERNEL, 8192, __VA_ARGS__);        \
    case 8194: CGX_LAUNCH_V(KERNEL, 8194, __VA_ARGS__);        \
    case 24576: CGX_LAUNCH_V(KERNEL, 24576, __VA_ARGS__);      \
    case 24578: CGX_LAUNCH_V(KERNEL, 24578, __VA_ARGS__);      \
    case 40960: CGX_LAUNCH_V(KERNEL, 40960, __VA_ARGS__);      \
    case 40962: CGX_LAUNCH_V(KERNEL, 40962, __VA_ARGS__);      \
    case 303104: CGX_LAUNCH_V(KERNEL, 303104, __VA_ARGS__);    \
    case 303106: CGX_LAUNCH_V(KERNEL, 303106, __VA_ARGS__);    \
    case 565248: CGX_LAUNCH_V(KERNEL, 565248, __VA_ARGS__);    \
    case 565250: CGX_LAUNCH_V(KERNEL, 565250, __VA_ARGS__);    \
    case 827392: CGX_LAUNCH_V(KERNEL, 827392, __VA_ARGS__);    \
    case 827394: CGX_LAUNCH_V(KERNEL, 827394, __VA_ARGS__);    \
    case 1613824: CGX_LAUNCH_V(KERNEL, 1613824, __VA_ARGS__);  \
    case 1613826: CGX_LAUNCH_V(KERNEL, 1613826, __VA_ARGS__);  \
    case 1875968: CGX_LAUNCH_V(KERNEL, 1875968, __VA_ARGS__);  \
    case 1875970: CGX_LAUNCH_V(KERNEL, 1875970, __VA_ARGS__);  \
    case 3710976: CGX_LAUNCH_V(KERNEL, 3710976, __VA_ARGS__);  \
    case 3710978: CGX_LAUNCH_V(KERNEL, 3710978, __VA_ARGS__);  \
    case 3973120: CGX_LAUNCH_V(KERNEL, 3973120, __VA_ARGS__);  \
    case 3973122: CGX_LAUNCH_V(KERNEL, 3973122, __VA_ARGS__);  \
    case 9216000: CGX_LAUNCH_V(KERNEL, 9216000, __VA_ARGS__);  \
    case 9216002: CGX_LAUNCH_V(KERNEL, 9216002, __VA_ARGS__);  \
    case 10264576: CGX_LAUNCH_V(KERNEL, 10264576, __VA_ARGS__);\
    case 10264578: CGX_LAUNCH_V(KERNEL, 10264578, __VA_ARGS__);\
    case 12361728: CGX_LAUNCH_V(KERNEL, 12361728, __VA_ARGS__);\
    case 12361730: CGX_LAUNCH_V(KERNEL, 12361730, __VA_ARGS__);\
    case 20750336: CGX_LAUNCH_V(KERNEL, 20750336, __VA_ARGS__);\
    case 20750338: CGX_LAUNCH_V(KERNEL, 20750338, __VA_ARGS__);\
    case 29138944: CGX_LAUNCH_V(KERNEL, 29138944, __VA_ARGS__);\
    case 29138946: CGX_LAUNCH_V(KERNEL, 29138946, __VA_ARGS__);\
    default: return hipErrorInvalidValue;                      \
  }

// Workgroups of k_spmv_dot<T, v> resident on the device at once (occupancy
// x CUs; 0: unknown variant). The SpMV grid is capped to it: a persistent
// grid larger than what fits runs its last workgroups as a second wave,
// after the first ones finish their fixed shares, and that tail measured
// 8% of the value-code kernel at 256^3 (tools/gpu_vc_ab.sh).
#define CGX_SPMV_LIST(X)                                                                    \
  X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(12) X(13) X(14) X(15) X(264) X(265) X(266)      \
  X(133) X(135) X(67108877) X(67108879)                                                     \
  X(267) X(2048) X(2050) X(2056) X(2058) X(6144) X(6146) X(8192) X(8194) X(24576) X(24578)  \
  X(40960) X(40962) X(303104) X(303106) X(565248) X(565250) X(827392) X(827394) X(1613824)  \
  X(1613826) X(1875968) X(1875970) X(3710976) X(3710978) X(3973120) X(3973122)              \
  X(9216000) X(9216002) X(10264576) X(10264578)                                             \
  X(12361728) X(12361730) X(20750336) X(20750338) X(29138944) X(29138946)
template <typename T> const void *spmv_dot_kernel(int v) {
  switch (v) {
#define CGX_KP(VV) \
  case VV: return reinterpret_cast<const void *>(&k_spmv_dot<T, VV>);
    CGX_SPMV_LIST(CGX_KP)
#undef CGX_KP
    default: return nullptr;
  }
}

template <typename T> int spmv_dot_resident(int v) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, int> cache;  // (device, variant) -> workgroups
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({dev, v});
  if (it != cache.end()) return it->second;
  int res = 0;
  if (const void *k = spmv_dot_kernel<T>(v)) {
    int nb = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kBlock, 0) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      res = nb * cus;
  }
  cache[{dev, v}] = res;
  return res;
}

template <typename T> static int cap_resident(int grid, int v) {
  const int r = spmv_dot_resident<T>(v);
  return (r > 0 && r < grid) ? r : grid;
}

// The standalone SpMV (VectorOperations::spmv, cgx_spmv) is the loop's
// k_spmv_dot in the matrix's variant, slot 0 of a context state that is
// always active; its p.Ap partials land in ws and are not read.
template <typename T>
hipError_t Launch<T>::spmv(const CsrDev &A, const T *x, T *y, CgScalars<T> *st, RedWs<T> *ws,
                           hipStream_t s) {
  return spmv_dot(A, x, y, st, 0, ws, s, 0);
}
// One-off SpMV kernels (the init r = b - A x, accuracy()) run CSR-stream on
// the caller's CSR arrays, whatever the loop's form: every form computes the
// same per-row sums, and one launch per solve does not pay for an
// instantiation per form. 13: pipelined paired loads (0 when val / col are
// not aligned for them).
#define CGX_CSR_ONEOFF(KERNEL, ...)                                             \
  do {                                                                          \
    const int spmv_grid_ = grid_rows(A.nrb);                                    \
    if (spmv_variant<T>(A, 13) == 13) CGX_LAUNCH_V(KERNEL, 13, __VA_ARGS__);    \
    CGX_LAUNCH_V(KERNEL, 0, __VA_ARGS__);                                       \
  } while (0)
template <typename T>
hipError_t Launch<T>::cg_init(const CsrDev &A, const T *x, const T *b, T *r, T *p,
                              CgScalars<T> *st, RedWs<T> *ws, T tol, long long cap,
                              hipStream_t s) {
  CGX_CSR_ONEOFF(k_cg_init, args(A), (const T *)A.val, x, b, r, p, st, ws, tol, cap);
}
// The tile walk (spmv_lean_tile) takes the lean layout when it is the
// plane-per-step carry walk of a 3-D stencil with a = 2 slices, every XCD
// group whole planes (<= 256 of them) and a plane's positions whole tiles;
// $CGX_LEAN_TILE=0 keeps the 4-wave walk
bool lean_tile_ok(const CsrDev &A) {
  static const int env = [] {
    const char *e = getenv("CGX_LEAN_TILE");
    return e ? atoi(e) : 1;
  }();
  if (!env || !vl_whole(A) || A.vl_P != 0 || A.vl_a != kTileM * 2 * kSellRows) return false;
  const int64_t step = A.vl_grid / 2;
  if (step <= 0 || A.vl_D != step * 2 * kSellRows || step % (4 * kTileY)) return false;
  if (A.nsl % 8 || (A.nsl / 8) % step || (A.nsl / 8) / step > 256) return false;
  // at least 8 planes per wave: a part's two halo planes are loaded again (the
  // 256 x 256 x 32 slab, 4 planes per XCD group, ran its p.Ap walk in 11.6
  // against 8.2 us in the 4-wave form, profiles/r6final_slab_*)
  return (A.nsl / 8) / step >= 8 * kTileZ;
}
// p.Ap partials of mode 6's kernel 1: one per workgroup of its launch
int lean_dot_parts(const CsrDev &A) {
  return lean_tile_ok(A) ? A.vl_grid / kTileY * kTileZ : A.vl_grid;  // 8 step kTileZ / (4 Y)
}
int fd_dot_parts(const CsrDev &A) { return A.vl_grid / kTileY * kFdZ; }
// mode 6's kernel 2 in the tile form ($CGX_LEAN_TILE_UPDR=1; with r's pairs
// prefetched it ran 74.4 against 68.6 us at 256^3, profiles/r6t_*: off by
// default), and its r.r partials
bool lean_updr_tile(const CsrDev &A) {
  static const int env = [] {
    const char *e = getenv("CGX_LEAN_TILE_UPDR");
    return e ? atoi(e) : 0;
  }();
  return env && lean_tile_ok(A);
}
int lean_updr_parts(const CsrDev &A) {
  return lean_updr_tile(A) ? A.vl_grid / kTileY * kTileZ : A.vl_grid;
}
template <typename T> int Launch<T>::lean_resident() {
  static std::mutex mu;
  static std::map<int, int> cache;  // device -> workgroups
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int nb = 0, cus = 0, res = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void *)&k_spmv_lean<T>, kBlock,
                                                   0) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
    res = nb * cus;
  cache[dev] = res;
  return res;
}
template <typename T>
hipError_t Launch<T>::spmv_dot(const CsrDev &A, const T *p, T *Ap, CgScalars<T> *st,
                               int slot, RedWs<T> *ws, hipStream_t s, int rev) {
  CsrArgs a = args(A);
  a.rev = rev;
  if (vl_whole(A)) {  // the lean stencil walk: its own grid (the class layout's)
    CGX_GGL(k_spmv_lean<T>, dim3(A.vl_grid), dim3(kBlock), 0, s, a, p, Ap, st, slot, ws);
    return hipGetLastError();
  }
  if (A.sell_partial && (spmv_variant<T>(A) & (2048 | 8192))) {
    // the SELL copy lacks the boundary rows: the whole matrix as CSR-stream
    CsrDev d = A;
    d.variant = 13;
    d.lean = false;
    d.rbo = nullptr;
    return spmv_dot(d, p, Ap, st, slot, ws, s, rev);
  }
  const int v = spmv_variant<T>(A);
  const int spmv_grid_ = cap_resident<T>(grid_rows(A.nrb), v);
  CGX_SPMV_SWITCH(v, k_spmv_dot, a, (const T *)A.val, p, Ap, st, slot, ws);
}
template <typename T>
hipError_t Launch<T>::lean_dot(const CsrDev &A, const T *p, CgScalars<T> *st, int slot,
                               RedWs<T> *ws, hipStream_t s, int rev) {
  if (!vl_whole(A)) return hipErrorInvalidValue;
  CsrArgs a = args(A);
  a.rev = rev;
  if (lean_tile_ok(A)) {
    CGX_GGL(k_spmv_lean_dot_tile<T>, dim3(lean_dot_parts(A)), dim3(kBlock), 0, s, a, p, st,
            slot, ws);
    return hipGetLastError();
  }
  CGX_GGL(k_spmv_lean_dot<T>, dim3(A.vl_grid), dim3(kBlock), 0, s, a, p, st, slot, ws);
  return hipGetLastError();
}
template <typename T>
hipError_t Launch<T>::fd_dot_tile(const CsrDev &A, const T *r, const T *pold, T *pc,
                                  CgScalars<T> *st, int slot, RedWs<T> *ws, int np_rr,
                                  hipStream_t s, int rev) {
  if (!lean_tile_ok(A)) return hipErrorInvalidValue;
  CsrArgs a = args(A);
  a.rev = rev;
  CGX_GGL(k_spmv_fd_dot_tile<T>, dim3(fd_dot_parts(A)), dim3(kBlock), 0, s, a, r, pold, pc, st,
          slot, ws, np_rr);
  return hipGetLastError();
}
template <typename T>
hipError_t Launch<T>::lean_updr_rule(const CsrDev &A, const T *p, T *r, CgScalars<T> *st,
                                     int slot, RedWs<T> *ws, hipStream_t s, int rev) {
  if (!lean_tile_ok(A)) return hipErrorInvalidValue;
  CsrArgs a = args(A);
  a.rev = rev;
  CGX_GGL(k_spmv_lean_updr_rule<T>, dim3(A.vl_grid), dim3(kBlock), 0, s, a, p, r, st, slot, ws,
          fd_dot_parts(A));
  return hipGetLastError();
}
template <typename T>
hipError_t Launch<T>::lean_updr(const CsrDev &A, const T *p, T *r, CgScalars<T> *st, int slot,
                                RedWs<T> *ws, hipStream_t s, int rev) {
  if (!vl_whole(A)) return hipErrorInvalidValue;
  CsrArgs a = args(A);
  a.rev = rev;
  if (lean_updr_tile(A)) {
    CGX_GGL(k_spmv_lean_updr_tile<T>, dim3(lean_updr_parts(A)), dim3(kBlock), 0, s, a, p, r, st,
            slot, ws, lean_dot_parts(A));
    return hipGetLastError();
  }
  CGX_GGL(k_spmv_lean_updr<T>, dim3(A.vl_grid), dim3(kBlock), 0, s, a, p, r, st, slot, ws,
          lean_dot_parts(A));
  return hipGetLastError();
}
template <typename T>
hipError_t Launch<T>::spmv_lean_interior(const CsrDev &A, const T *p, T *Ap, CgScalars<T> *st,
                                         int slot, RedWs<T> *ws, hipStream_t s, int rev,
                                         const PeerDev *P, int wg0) {
  if (!vl_active(A) || !A.vl_split || (P && (wg0 < 0 || wg0 % 8))) return hipErrorInvalidValue;
  CsrArgs a = args(A);
  a.rev = rev;
  a.part_off = 0;
  a.wg0 = P ? wg0 : 0;
  if (P) {
    CGX_GGL(k_spmv_lean_push<T>, dim3(a.wg0 + A.vl_grid), dim3(kBlock), 0, s, a, p, Ap,
                       st, slot, ws, *P);
  } else {
    CGX_GGL(k_spmv_lean<T>, dim3(A.vl_grid), dim3(kBlock), 0, s, a, p, Ap, st, slot,
                       ws);
  }
  return hipGetLastError();
}
// SpMV + p.Ap over a list of SELL slices (a partitioned matrix's interior or
// boundary slices), its partials at [part_off, part_off + grid)
template <typename T>
hipError_t Launch<T>::spmv_dot_slices(const CsrDev &A, const int *list, int count, int part_off,
                                      const T *p, T *Ap, CgScalars<T> *st, int slot,
                                      RedWs<T> *ws, hipStream_t s, int rev) {
  const int v = spmv_variant<T>(A) & ~2097152;  // a slice list is walked in list order
  if (!(v & (2048 | 8192)) || count < 1) return hipErrorInvalidValue;
  CsrArgs a = args(A);
  a.sorder = list;
  a.nsl = count;
  a.part_off = part_off;
  a.rev = rev;
  const int spmv_grid_ = slice_grid(A, count);
  CGX_SPMV_SWITCH(v, k_spmv_dot, a, (const T *)A.val, p, Ap, st, slot, ws);
}
template <typename T> int Launch<T>::slice_grid(const CsrDev &A, int count) {
  const int g = (count + 3) / 4;  // one wave per slice, 4 waves per workgroup
  return cap_resident<T>(g < 1 ? 1 : (g > kMaxGrid ? kMaxGrid : g),
                         spmv_variant<T>(A) & ~2097152);
}
template <typename T>
hipError_t Launch<T>::spmv_dot_variant(int v, const CsrDev &A, const T *p, T *Ap,
                                       CgScalars<T> *st, RedWs<T> *ws, hipStream_t s) {
  if (v & kVL) {  // the lean walk (A's class layout)
    CsrDev d = A;
    d.variant = v & ~kVL;
    d.lean = true;
    if (!vl_active(d)) return hipErrorInvalidValue;
    return spmv_dot(d, p, Ap, st, 0, ws, s, 0);
  }
  const int vv = spmv_variant<T>(A, v);
  const int spmv_grid_ = cap_resident<T>(grid_rows(A.nrb), vv);
  switch (vv) {  // CSR-stream timing ablations (bits 16 / 32), tuning only
    case 31: CGX_LAUNCH_V(k_spmv_dot, 31, args(A), (const T *)A.val, p, Ap, st, 0, ws);
    case 47: CGX_LAUNCH_V(k_spmv_dot, 47, args(A), (const T *)A.val, p, Ap, st, 0, ws);
    case 63: CGX_LAUNCH_V(k_spmv_dot, 63, args(A), (const T *)A.val, p, Ap, st, 0, ws);
    case 67108927: CGX_LAUNCH_V(k_spmv_dot, 67108927, args(A), (const T *)A.val, p, Ap, st, 0, ws);
    case 67108911: CGX_LAUNCH_V(k_spmv_dot, 67108911, args(A), (const T *)A.val, p, Ap, st, 0, ws);
    default: break;
  }
  CGX_SPMV_SWITCH(vv, k_spmv_dot, args(A), (const T *)A.val, p, Ap, st, 0, ws);
}
template <typename T>
hipError_t Launch<T>::update_r(int64_t n, T *r, const T *Ap, CgScalars<T> *st, int slot,
                               RedWs<T> *ws, hipStream_t s, bool fused, int np_pap, int rev,
                               const T *rin, int rule, const PeerDev *peer) {
  if (!rin) rin = r;
  if (peer) {
    if (fused || rule || rin != r) return hipErrorInvalidValue;
    CGX_GGL((k_update_r_peer<T>), dim3(grid_elems(n, kGridUpdateR)), dim3(kBlock), 0,
                       s, n, r, Ap, st, slot, ws, np_pap, rev, *peer);
    return hipGetLastError();
  }
  if (fused) {
    CGX_GGL((k_update_r<T, true>), dim3(grid_elems(n, kMaxGrid)), dim3(kBlock), 0, s,
                       n, rin, r,
                       Ap, st, slot, ws, 0, 0, 0);
  } else {
    const int g = grid_elems(n, kGridUpdateR);
    if (np_pap <= 4 * kBlock)
      CGX_GGL((k_update_r<T, false, 4>), dim3(g), dim3(kBlock), 0, s, n, rin, r, Ap, st, slot,
              ws, np_pap, rev, rule);
    else if (np_pap <= 8 * kBlock)
      CGX_GGL((k_update_r<T, false, 8>), dim3(g), dim3(kBlock), 0, s, n, rin, r, Ap, st, slot,
              ws, np_pap, rev, rule);
    else
      CGX_GGL((k_update_r<T, false>), dim3(g), dim3(kBlock), 0, s, n, rin, r, Ap, st, slot, ws,
              np_pap, rev, rule);
  }
  return hipGetLastError();
}

// ---- mode 4 (fused deferred-x iteration): k_spmv_fd is instantiated for
// the production SpMV forms only (CSR-stream, SELL-P, value-code SELL-P and
// its pipelined / stencil / plane-march loops), f64 only; other variants
// keep mode 3 (fd_supported).
#define CGX_FD_LIST(X)                                                                 \
  X(13) X(15) X(8192) X(8194) X(40960) X(40962) X(303104) X(303106) X(565248) X(565250) \
  X(827392) X(827394) X(1613824) X(1613826) X(1875968) X(1875970) X(3710976) X(3710978) \
  X(3973120) X(3973122) X(9216000) X(9216002) X(10264576) X(10264578) X(12361728)      \
  X(12361730)

// mode 2 (k_spmv_fused): mode 4's forms, plain CSR-stream and the
// dictionary SELL forms small matrices take
#define CGX_FUSED_LIST(X)                                                                \
  CGX_FD_LIST(X) X(0) X(5) X(133) X(265) X(2048) X(2050) X(2056) X(2058) X(6144) X(6146) X(24576) \
  X(24578)

template <typename T> static const void *spmv_fd_kernel(int v) {
  if constexpr (!std::is_same<T, double>::value) {
    (void)v;
    return nullptr;
  } else {
    switch (v) {
#define CGX_KF(VV) \
  case VV: return reinterpret_cast<const void *>(&k_spmv_fd<T, VV>);
      CGX_FD_LIST(CGX_KF)
#undef CGX_KF
      default: return nullptr;
    }
  }
}

// resident workgroups of k_spmv_fd<v> (0: unknown), as spmv_dot_resident
template <typename T> static int spmv_fd_resident(int v) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({dev, v});
  if (it != cache.end()) return it->second;
  int res = 0;
  if (const void *k = spmv_fd_kernel<T>(v)) {
    int nb = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kBlock, 0) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      res = nb * cus;
  }
  cache[{dev, v}] = res;
  return res;
}

template <typename T> bool Launch<T>::fd_supported(const CsrDev &A) {
  return spmv_fd_kernel<T>(spmv_variant<T>(A)) != nullptr;
}
// k_spmv_fd's grid: the SpMV's (grid_rows) capped at its own resident
// workgroups. It carries more VGPRs than k_spmv_dot (e.g. 107 against 96,
// 147 against 124), so on a matrix big enough to fill the chip the cap is
// lower and the p.Ap partials split differently: mode 4 then equals mode 1
// to rounding (the sum order of one dot), not bit for bit. Holding k_spmv_fd
// to k_spmv_dot's waves per SIMD instead spilled 20-56 VGPRs to scratch.
template <typename T> int Launch<T>::fd_parts(const CsrDev &A) {
  if (vl_whole(A)) return A.vl_team ? A.vl_grid / 4 : A.vl_grid;
  const int grid = grid_rows(A.nrb);
  const int r = spmv_fd_resident<T>(spmv_variant<T>(A));
  return (r > 0 && r < grid) ? r : grid;
}
template <typename T>
hipError_t Launch<T>::spmv_fd(const CsrDev &A, const T *r, const T *pold, T *pc, T *Ap,
                              CgScalars<T> *st, int slot, RedWs<T> *ws, int np_rr,
                              hipStream_t s, int rev) {
  const void *k = spmv_fd_kernel<T>(spmv_variant<T>(A));
  if (!k) return hipErrorInvalidValue;
  CsrArgs a = args(A);
  a.rev = rev;
  if constexpr (std::is_same<T, double>::value) {
    if (vl_whole(A)) {  // the lean walk at its class layout's grid
      // (the team form with its +-D prefetch: 1,025-1,042 against 1,067-1,079
      // us per launch at 512^3, profiles/r06b_team_prefetch_ab.log)
      // (and its p_k / Ap stores non-temporal: the team form runs walks of >= 32
      // M rows, whose vectors are past the Infinity Cache; 544-545 against
      // 532-537 it/s at 512^3, profiles/r06k_team_nt_stores_ab.log)
      if (A.vl_team)
        CGX_GGL((k_spmv_fd_lean_t<T, true, true>), dim3(A.vl_grid / 4), dim3(kTeamBlock), 0, s, a,
                r, pold, pc, Ap, st, slot, ws, np_rr);
      else
        CGX_GGL(k_spmv_fd_lean<T>, dim3(A.vl_grid), dim3(kBlock), 0, s, a, r, pold, pc, Ap, st,
                slot, ws, np_rr);
      return hipGetLastError();
    }
  }
  const T *val = (const T *)A.val;
  void *kargs[] = {&a, (void *)&val, (void *)&r, (void *)&pold, (void *)&pc, (void *)&Ap,
                   (void *)&st, (void *)&slot, (void *)&ws, (void *)&np_rr};
  return cgx_lk(k, dim3(fd_parts(A)), dim3(kBlock), kargs, 0, s);
}
// ---- the interior SpMV with the halo push in front (k_spmv_dot_push): the
// SELL forms a partitioned matrix takes (no plane march: slice lists)
#define CGX_PUSH_LIST(X)                                                                \
  X(2048) X(2050) X(6144) X(6146) X(8192) X(8194) X(24576) X(24578) X(40960) X(40962)  \
  X(303104) X(303106) X(565248) X(565250) X(827392) X(827394) X(1613824) X(1613826)     \
  X(1875968) X(1875970) X(9216000) X(9216002) X(10264576) X(10264578)

template <typename T> static const void *spmv_push_kernel(int v) {
  switch (v) {
#define CGX_KPU(VV) \
  case VV: return reinterpret_cast<const void *>(&k_spmv_dot_push<T, VV>);
    CGX_PUSH_LIST(CGX_KPU)
#undef CGX_KPU
    default: return nullptr;
  }
}

template <typename T> static const void *spmv_bnd_kernel(int v) {
  switch (v) {
#define CGX_KBN(VV) \
  case VV: return reinterpret_cast<const void *>(&k_spmv_dot_bnd<T, VV>);
    CGX_PUSH_LIST(CGX_KBN)
    CGX_KBN(13) CGX_KBN(0)  // the boundary rows as CSR-stream blocks (spmv_dot_rows)
#undef CGX_KBN
    default: return nullptr;
  }
}
template <typename T> bool Launch<T>::bnd_supported(const CsrDev &A) {
  return spmv_bnd_kernel<T>(spmv_variant<T>(A) & ~2097152) != nullptr;
}
template <typename T>
hipError_t Launch<T>::spmv_dot_slices_bnd(const CsrDev &A, const int *list, int count,
                                          int part_off, const T *p, T *Ap, CgScalars<T> *st,
                                          int slot, RedWs<T> *ws, hipStream_t s, int rev,
                                          const PeerDev &P) {
  const int v = spmv_variant<T>(A) & ~2097152;
  const void *k = spmv_bnd_kernel<T>(v);
  if (!k || count < 1) return hipErrorInvalidValue;
  CsrArgs a = args(A);
  a.sorder = list;
  a.nsl = count;
  a.part_off = part_off;
  a.rev = rev;
  const T *val = (const T *)A.val;
  PeerDev pd = P;
  void *kargs[] = {&a, (void *)&val, (void *)&p, (void *)&Ap, (void *)&st, (void *)&slot,
                   (void *)&ws, (void *)&pd};
  return cgx_lk(k, dim3(slice_grid(A, count)), dim3(kBlock), kargs, 0, s);
}

template <typename T> int Launch<T>::rows_grid(const CsrDev &A, int count) {
  return cap_resident<T>(grid_rows(count), spmv_variant<T>(A, 13));
}
template <typename T>
hipError_t Launch<T>::spmv_dot_rows(const CsrDev &A, const int *blocks, int count, int part_off,
                                    const T *p, T *Ap, CgScalars<T> *st, int slot, RedWs<T> *ws,
                                    hipStream_t s, const PeerDev *P) {
  const int v = spmv_variant<T>(A, 13);  // 13, or 0 for unaligned val / col
  if (count < 1 || (v != 13 && v != 0)) return hipErrorInvalidValue;
  CsrArgs a = args(A);
  a.rbo = blocks;
  a.nrb = count;
  a.part_off = part_off;
  const T *val = (const T *)A.val;
  const int grid = rows_grid(A, count);
  if (P) {
    const void *k = spmv_bnd_kernel<T>(v);
    PeerDev pd = *P;
    void *kargs[] = {&a, (void *)&val, (void *)&p, (void *)&Ap, (void *)&st, (void *)&slot,
                     (void *)&ws, (void *)&pd};
    return cgx_lk(k, dim3(grid), dim3(kBlock), kargs, 0, s);
  }
  const int spmv_grid_ = grid;
  if (v == 13) CGX_LAUNCH_V(k_spmv_dot, 13, a, val, p, Ap, st, slot, ws);
  CGX_LAUNCH_V(k_spmv_dot, 0, a, val, p, Ap, st, slot, ws);
}
template <typename T> bool Launch<T>::push_supported(const CsrDev &A) {
  return spmv_push_kernel<T>(spmv_variant<T>(A) & ~2097152) != nullptr;
}
// SpMV workgroups of the pushing interior launch over `count` slices: the
// interior launch's resident grid less the push workgroups (all resident)
template <typename T> int Launch<T>::slice_grid_push(const CsrDev &A, int count, int wg0) {
  const int g = slice_grid(A, count);
  const int r = spmv_dot_resident<T>(spmv_variant<T>(A) & ~2097152);
  const int cap = r > 0 ? r - wg0 : g;
  return std::max(1, std::min(g, cap));
}
template <typename T>
hipError_t Launch<T>::spmv_dot_slices_push(const CsrDev &A, const int *list, int count,
                                           int part_off, const T *p, T *Ap, CgScalars<T> *st,
                                           int slot, RedWs<T> *ws, hipStream_t s, int rev,
                                           const PeerDev &P, int wg0) {
  const int v = spmv_variant<T>(A) & ~2097152;
  const void *k = spmv_push_kernel<T>(v);
  if (!k || count < 1 || wg0 % 8) return hipErrorInvalidValue;
  CsrArgs a = args(A);
  a.sorder = list;
  a.nsl = count;
  a.part_off = part_off;
  a.rev = rev;
  a.wg0 = wg0;
  const T *val = (const T *)A.val;
  PeerDev pd = P;
  void *kargs[] = {&a, (void *)&val, (void *)&p, (void *)&Ap, (void *)&st, (void *)&slot,
                   (void *)&ws, (void *)&pd};
  return cgx_lk(k, dim3(wg0 + slice_grid_push(A, count, wg0)), dim3(kBlock), kargs, 0,
                         s);
}

template <typename T>
hipError_t Launch<T>::flush_group(int64_t n, T *x, T *const P[4], CgScalars<T> *st,
                                  hipStream_t s, int rev) {
  CGX_LAUNCH(k_flush_group<T>, grid_elems(n, kGridUpdateP), n, x, (const T *)P[0],
             (const T *)P[1], (const T *)P[2], (const T *)P[3], (const CgScalars<T> *)st, rev);
}
template <typename T>
hipError_t Launch<T>::update_r_flush(int64_t n, T *r, const T *Ap, CgScalars<T> *st, int slot,
                                     RedWs<T> *ws, int np_pap, int rev, T *x, T *const P[4],
                                     hipStream_t s) {
  const XFlush<T> xf{x, {P[0], P[1], P[2], P[3]}};
  if (np_pap <= 4 * kBlock)
    CGX_LAUNCH((k_update_r_flush<T, 4>), grid_elems(n, kGridUpdateR), n, r, Ap, st, slot, ws,
               np_pap, rev, xf);
  if (np_pap <= 8 * kBlock)
    CGX_LAUNCH((k_update_r_flush<T, 8>), grid_elems(n, kGridUpdateR), n, r, Ap, st, slot, ws,
               np_pap, rev, xf);
  CGX_LAUNCH(k_update_r_flush<T>, grid_elems(n, kGridUpdateR), n, r, Ap, st, slot, ws, np_pap,
             rev, xf);
}
template <typename T>
hipError_t Launch<T>::rr_settle(CgScalars<T> *st, RedWs<T> *ws, int np_rr, hipStream_t s) {
  CGX_LAUNCH(k_rr_settle<T>, 1, st, ws, np_rr);
}
template <typename T>
hipError_t Launch<T>::spmv_fd_lean_push(const CsrDev &A, const T *r, const T *pold, T *pc, T *Ap,
                                        CgScalars<T> *st, int slot, RedWs<T> *ws, hipStream_t s,
                                        int rev, const PeerDev &P, int wg0) {
  if constexpr (!std::is_same<T, double>::value) {
    return hipErrorInvalidValue;
  } else {
    if (!vl_active(A) || !A.vl_split || wg0 < 0 || wg0 % 8) return hipErrorInvalidValue;
    CsrArgs a = args(A);
    a.rev = rev;
    a.part_off = 0;
    a.wg0 = wg0;
    CGX_GGL(k_spmv_fd_lean_push<T>, dim3(wg0 + A.vl_grid), dim3(kBlock), 0, s, a, r, pold, pc,
            Ap, st, slot, ws, P);
    return hipGetLastError();
  }
}
template <typename T>
hipError_t Launch<T>::spmv_fd_rows_bnd(const CsrDev &A, const int *blocks, int count,
                                       int part_off, const T *r, const T *pold, T *pc, T *Ap,
                                       CgScalars<T> *st, int slot, RedWs<T> *ws, hipStream_t s,
                                       const PeerDev &P) {
  if constexpr (!std::is_same<T, double>::value) {
    return hipErrorInvalidValue;
  } else {
    const int v = spmv_variant<T>(A, 13);  // 13, or 0 for unaligned val / col
    if (count < 1 || (v != 13 && v != 0)) return hipErrorInvalidValue;
    CsrArgs a = args(A);
    a.rbo = blocks;
    a.nrb = count;
    a.part_off = part_off;
    const T *val = (const T *)A.val;
    const int grid = rows_grid(A, count);
    if (v == 13)
      CGX_GGL((k_spmv_fd_bnd<T, 13>), dim3(grid), dim3(kBlock), 0, s, a, val, r, pold, pc, Ap, st,
              slot, ws, P);
    else
      CGX_GGL((k_spmv_fd_bnd<T, 0>), dim3(grid), dim3(kBlock), 0, s, a, val, r, pold, pc, Ap, st,
              slot, ws, P);
    return hipGetLastError();
  }
}
template <typename T>
hipError_t Launch<T>::update_r_peer_rule(int64_t n, T *r, const T *Ap, CgScalars<T> *st, int slot,
                                         RedWs<T> *ws, int np_pap, int rev, T *x, T *const *P4,
                                         hipStream_t s, const PeerDev &P) {
  if constexpr (!std::is_same<T, double>::value) {
    return hipErrorInvalidValue;
  } else {
    const int grid = grid_elems(n, kGridUpdateR);
    if (P4) {
      const XFlush<T> xf{x, {P4[0], P4[1], P4[2], P4[3]}};
      CGX_GGL((k_update_r_peer_rule<T, true>), dim3(grid), dim3(kBlock), 0, s, n, r, Ap, st, slot,
              ws, np_pap, rev, P, xf);
    } else {
      const XFlush<T> xf{nullptr, {nullptr, nullptr, nullptr, nullptr}};
      CGX_GGL((k_update_r_peer_rule<T, false>), dim3(grid), dim3(kBlock), 0, s, n, r, Ap, st,
              slot, ws, np_pap, rev, P, xf);
    }
    return hipGetLastError();
  }
}
template <typename T> int Launch<T>::spmv_parts(const CsrDev &A) {
  if (vl_whole(A)) return A.vl_grid;
  if (A.sell_partial && (spmv_variant<T>(A) & (2048 | 8192)))  // spmv_dot's CSR-stream
    return cap_resident<T>(grid_rows(A.nrb), spmv_variant<T>(A, 13));
  return cap_resident<T>(grid_rows(A.nrb), spmv_variant<T>(A));  // = spmv_dot's grid
}
template <typename T> int Launch<T>::update_parts(int64_t n) {
  return grid_elems(n, kGridUpdateR);  // k_update_r's grid: one r.r partial per workgroup
}
template <typename T>
hipError_t Launch<T>::finalize(const T *part, int np, T *dst, hipStream_t s) {
  CGX_LAUNCH(k_finalize<T>, 1, part, np, dst);
}
template <typename T>
hipError_t Launch<T>::spmv_fused(const CsrDev &A, const T *r, const T *pp, T *pc, T *x, T *Ap,
                                 CgScalars<T> *st, int slot, RedWs<T> *ws, hipStream_t s) {
  const int spmv_grid_ = grid_rows(A.nrb);
  switch (spmv_variant<T>(A)) {  // mode 4's forms and the small-matrix ones
#define CGX_KFU(VV)                                                                   \
  case VV:                                                                            \
    CGX_LAUNCH_V(k_spmv_fused, VV, args(A), (const T *)A.val, r, pp, pc, x, Ap, st, slot, ws);
    CGX_FUSED_LIST(CGX_KFU)
#undef CGX_KFU
    default: return hipErrorInvalidValue;
  }
}
template <typename T> bool Launch<T>::fused_supported(const CsrDev &A) {
  switch (spmv_variant<T>(A)) {
#define CGX_KFS(VV) case VV:
    CGX_FUSED_LIST(CGX_KFS)
#undef CGX_KFS
    return true;
    default: return false;
  }
}
template <typename T>
hipError_t Launch<T>::flush_x(int64_t n, T *x, const T *p, CgScalars<T> *st, int slot,
                              RedWs<T> *ws, hipStream_t s) {
  CGX_LAUNCH(k_flush_x<T>, elem_grid(n, 4), n, x, p, st, slot, ws);
}
template <typename T>
hipError_t Launch<T>::update_xp(int64_t n, T *x, T *p, const T *r, CgScalars<T> *st,
                                int slot, RedWs<T> *ws, int np_rr, hipStream_t s, int rev,
                                const PeerDev *peer) {
  if (peer)
    CGX_LAUNCH(k_update_xp_peer<T>, grid_elems(n, kGridUpdateP), n, x, p, r, st, slot, ws, np_rr,
               rev, *peer);
  CGX_LAUNCH(k_update_xp<T>, grid_elems(n, kGridUpdateP), n, x, p, r, st, slot, ws, np_rr, rev);
}
template <typename T>
hipError_t Launch<T>::update_p_defer(int64_t n, T *x, const T *p, T *pn, T *const P[4],
                                     const T *r, CgScalars<T> *st, int slot, RedWs<T> *ws,
                                     int np_rr, hipStream_t s, int rev, const PeerDev *peer) {
  if (peer && slot == 3)
    CGX_LAUNCH((k_update_p_defer_peer<T, true>), grid_elems(n, kGridUpdateP), n, x, p, pn,
               (const T *)P[0], (const T *)P[1], (const T *)P[2], r, st, slot, ws, np_rr, rev,
               *peer);
  if (peer)
    CGX_LAUNCH((k_update_p_defer_peer<T, false>), grid_elems(n, kGridUpdateP), n, x, p, pn,
               (const T *)P[0], (const T *)P[1], (const T *)P[2], r, st, slot, ws, np_rr, rev,
               *peer);
  if (slot == 3) {
    CGX_LAUNCH((k_update_p_defer<T, true>), grid_elems(n, kGridUpdateP), n, x, p, pn,
               (const T *)P[0],
               (const T *)P[1], (const T *)P[2], r, st, slot, ws, np_rr, rev);
  }
  CGX_LAUNCH((k_update_p_defer<T, false>), grid_elems(n, kGridUpdateP), n, x, p, pn,
             (const T *)P[0],
             (const T *)P[1], (const T *)P[2], r, st, slot, ws, np_rr, rev);
}
template <typename T>
hipError_t Launch<T>::flush_defer(int64_t n, T *x, T *const P[4], CgScalars<T> *st,
                                  hipStream_t s) {
  CGX_GGL(k_flush_defer<T>, dim3(grid_elems(n, kGridUpdateP)), dim3(kBlock), 0, s, n, x,
                     (const T *)P[0], (const T *)P[1], (const T *)P[2], (const T *)P[3],
                     (const CgScalars<T> *)st);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  CGX_GGL(k_mark_defer<T>, dim3(1), dim3(1), 0, s, st);
  return hipGetLastError();
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
  CGX_GGL(k_scalar_div<T>, dim3(1), dim3(1), 0, s, num, den, out);
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
  CGX_CSR_ONEOFF(k_accuracy, args(A), (const T *)A.val, b, x, out2, ws);
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

template <typename T>
hipError_t Launch<T>::sell_pack(const CsrDev &A, const T *val, T *sval, hipStream_t s) {
  CGX_LAUNCH(k_sell_pack<T>, elem_grid(A.nsl * kSellRows * A.sell_r, 4), A.n, A.nsl, A.sell_r,
             A.rowptr, val, A.sl, sval);
}

// (kVL added when the loop's SpMV is the lean walk)
int launch_variant(const CsrDev &A, int dtype) {
  return (dtype == 1 /* CGX_F32 */ ? spmv_variant<float>(A) : spmv_variant<double>(A)) |
         (vl_active(A) ? kVL : 0);
}

bool spmv_listed(int v) { return spmv_dot_kernel<double>(v) != nullptr; }

bool launch_variant_ok(const CsrDev &A, int dtype) {
  return dtype == 1 /* CGX_F32 */ ? spmv_dot_kernel<float>(spmv_variant<float>(A)) != nullptr
                                  : spmv_dot_kernel<double>(spmv_variant<double>(A)) != nullptr;
}

template <typename T>
hipError_t Launch<T>::sellp_pack(const CsrDev &A, const T *val, T *sval, void *mask,
                                 hipStream_t s) {
  const int g = elem_grid(A.nsl * kSellRows * 2, 4);
  if (A.sell_kind == 2)
    CGX_GGL((k_sellp_pack<T, unsigned>), dim3(g), dim3(kBlock), 0, s, A.n, A.nsl,
                       A.rowptr, A.col, val, A.sl, A.sdict, sval, (unsigned *)mask);
  else
    CGX_GGL((k_sellp_pack<T, unsigned char>), dim3(g), dim3(kBlock), 0, s, A.n, A.nsl,
                       A.rowptr, A.col, val, A.sl, A.sdict, sval, (unsigned char *)mask);
  return hipGetLastError();
}

template <typename T>
hipError_t Launch<T>::sellpv_pack(const CsrDev &A, const T *val, const T *dict, int nd,
                                  unsigned char *codes, int *miss, T *missv, hipStream_t s) {
  const int g = elem_grid(A.nsl * kSellRows * 2, 4);
  CGX_GGL(k_sellpv_pack<T>, dim3(g), dim3(kBlock), 0, s, A.n, A.nsl, A.rowptr, A.col,
                     val, A.sl, A.sdict, dict, nd, codes, miss, missv);
  return hipGetLastError();
}

template <typename T>
hipError_t Launch<T>::vc_narrow(const void *codes8, void *codes4, int64_t chunks,
                                hipStream_t s) {
  CGX_GGL(k_vc_narrow, dim3(elem_grid(chunks, 4)), dim3(kBlock), 0, s,
                     (const unsigned char *)codes8, (unsigned char *)codes4, chunks);
  return hipGetLastError();
}

hipError_t vc_hash(const CsrDev &A, unsigned long long *hash, hipStream_t s) {
  const int g = (int)((A.nsl + 3) / 4);
  CGX_GGL(k_vc_hash, dim3(g), dim3(kBlock), 0, s, A.sl, A.nsl,
                     (const unsigned long long *)A.svc4, hash);
  return hipGetLastError();
}
hipError_t vc_match(const CsrDev &A, const unsigned long long *tmpl, int nt, SellSlice *sl_t,
                    unsigned *count, hipStream_t s) {
  const int g = (int)((A.nsl + 3) / 4);
  CGX_GGL(k_vc_match, dim3(g), dim3(kBlock), 0, s, A.sl, A.nsl,
                     (const unsigned long long *)A.svc4, tmpl, nt, sl_t, count);
  return hipGetLastError();
}

// 16-bit column deltas (kC16): one workgroup per row block (grid-stride)
__global__ __launch_bounds__(kBlock) void k_col16(const int *__restrict__ rb,
                                                   const int *__restrict__ rbk,
                                                   const int *__restrict__ col, int nrb,
                                                   short *__restrict__ col16, unsigned *bad) {
  unsigned nbad = 0;
  for (int b = blockIdx.x; b < nrb; b += gridDim.x) {
    const int r0 = rb[b];
    for (int k = rbk[b] + threadIdx.x; k < rbk[b + 1]; k += kBlock) {
      const int d = col[k] - r0;
      const bool fits = d >= -32768 && d <= 32767;
      col16[k] = fits ? (short)d : (short)0;
      nbad += fits ? 0u : 1u;
    }
  }
  if (nbad) atomicAdd(bad, nbad);
}

hipError_t col16_build(const CsrDev &A, short *col16, unsigned *bad, hipStream_t s) {
  if (A.nrb < 1) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(col16, 0, (size_t)(A.nnz + 2) * sizeof(short), s);
  if (e != hipSuccess) return e;
  const int grid = A.nrb < kMaxGrid ? A.nrb : kMaxGrid;
  CGX_GGL(k_col16, dim3(grid), dim3(kBlock), 0, s, A.rb, A.rbk, A.col, A.nrb, col16,
                     bad);
  return hipGetLastError();
}

// The interleaved val / col copy (kIL): pair P (entries 2P, 2P + 1; past
// nnz: 0) into chunk P / kIlCh, values first, then columns
template <typename T>
__global__ __launch_bounds__(kBlock) void k_il_pack(int64_t nnz, int64_t pairs,
                                                    const T *__restrict__ val,
                                                    const int *__restrict__ col, char *il) {
  using PV = typename PairOf<T>::V;
  constexpr int64_t CB = (int64_t)kIlCh * (sizeof(PV) + sizeof(Int2));
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t P = (int64_t)blockIdx.x * kBlock + threadIdx.x; P < pairs; P += stride) {
    const int64_t e = 2 * P;
    PV v;
    Int2 c;
    v.x = val[e];
    c.x = col[e];
    v.y = e + 1 < nnz ? val[e + 1] : T(0);
    c.y = e + 1 < nnz ? col[e + 1] : 0;
    char *cb = il + (P >> kIlLog) * CB;
    reinterpret_cast<PV *>(cb)[P & (kIlCh - 1)] = v;
    reinterpret_cast<Int2 *>(cb + kIlCh * sizeof(PV))[P & (kIlCh - 1)] = c;
  }
}

hipError_t il_build(const CsrDev &A, int es, char *il, hipStream_t s) {
  if (A.nnz < 2) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(il, 0, (size_t)il_bytes(A.nnz, es), s);
  if (e != hipSuccess) return e;
  const int64_t pairs = (A.nnz + 1) / 2;
  const int grid = elem_grid(pairs, 4);
  if (es == 8)
    CGX_GGL(k_il_pack<double>, dim3(grid), dim3(kBlock), 0, s, A.nnz, pairs,
            (const double *)A.val, A.col, il);
  else
    CGX_GGL(k_il_pack<float>, dim3(grid), dim3(kBlock), 0, s, A.nnz, pairs,
            (const float *)A.val, A.col, il);
  return hipGetLastError();
}

template struct Launch<double>;
template struct Launch<float>;

}  // namespace cgx
