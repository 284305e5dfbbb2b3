// cgx_dd.h — double-length (hi + lo) sums of the CG loop's two dots, shared
// by the kernels (cgx_kernels.hip) and the peer transport's all-reduce
// (cgx_peer.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace cgx {

// ---- the loop's two dots as double-length sums (round 6) -------------------
// p.Ap and r.r (and the initial r.r) are accumulated as unevaluated pairs
// hi + lo: every addition is TwoSum (Knuth), whose rounding error joins lo,
// from the per-thread sums through the workgroup partials and the partial
// sums to the world sum of the ranks, and only the final value is rounded
// to T. That value is the exact sum of the per-row products (each product
// is rounded as in the reference's expression) to within ~n u^2 of the sum
// of their magnitudes (u = 2^-53), so it no longer depends on how the rows
// were dealt to threads, workgroups, launches, SpMV forms, sweep directions
// or ranks: two such splits can round apart only when the exact sum lies
// that close to a rounding boundary of T (relative width ~2 n u, about 1e-8
// at 256^3). Built with -ffp-contract=off, so no FMA contracts the TwoSum.
// (f32 solves keep f32 pairs: twice the accuracy, not this independence.)
template <typename T> struct Dd {
  T hi, lo;
  Dd() = default;
  __host__ __device__ constexpr Dd(T h, T l = T(0)) : hi(h), lo(l) {}
  __device__ __forceinline__ Dd &operator+=(T x) {
    const T t = hi + x;
    const T z = t - hi;
    lo += (hi - (t - z)) + (x - z);
    hi = t;
    return *this;
  }
  __device__ __forceinline__ Dd &operator+=(const Dd &o) {
    *this += o.hi;
    lo += o.lo;
    return *this;
  }
  __device__ __forceinline__ T value() const { return hi + lo; }
};

template <typename T> __device__ __forceinline__ Dd<T> wave_sum_dd(Dd<T> v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const Dd<T> o(__shfl_down(v.hi, off, 64), __shfl_down(v.lo, off, 64));
    v += o;
  }
  return v;  // lane 0 holds the sum
}

}  // namespace cgx
