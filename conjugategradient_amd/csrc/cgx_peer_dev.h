// cgx_peer_dev.h — device side of the peer transport shared by the
// transport's own kernels (cgx_peer.hip) and the SpMV launch that carries the
// halo push in its leading workgroups (cgx_kernels.hip k_spmv_dot_push).
#pragma once

#include <hip/hip_runtime.h>

#include "cgx_dd.h"
#include "cgx_objects.h"

namespace cgx {
namespace peerdev {

__device__ __forceinline__ unsigned long long ld_sys(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(unsigned long long *p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double ld_sysd(const double *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sysd(double *p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T>
__device__ __forceinline__ bool skip_body(const CgScalars<T> *st, int slot, const PeerState *ps) {
  return (st && !st->active[slot]) || ps->fault;
}

// the tag a body's push / wait use (setup and init steps, st == nullptr:
// the running all-reduce count)
template <typename T>
__device__ __forceinline__ unsigned long long body_tag(const CgScalars<T> *st, int slot,
                                                       const PeerState *ps) {
  return st ? ps->arb[slot & 1] : ps->ar;
}

// poll *p >= want; false after `ticks` of the constant wall clock
__device__ __forceinline__ bool spin_ge(const unsigned long long *p, unsigned long long want,
                                        long long ticks) {
  const long long t0 = wall_clock64();
  while (ld_sys(p) < want) {
    if (wall_clock64() - t0 > ticks) return false;
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

// The workgroup's wait for every sending rank's kPushWG push flags of tag
// `tag` (the first wave polls, bounded); uniform control flow, false on a
// timeout. With P.nopoll a one-workgroup k_peer_wait launch has already
// waited (the one-waiter form): nothing to poll, the kernel boundary orders
// the landing buffer's reads after it.
__device__ __forceinline__ bool wait_pushes(const PeerDev &P, unsigned long long tag,
                                            int *ok_lds) {
  if (P.nopoll) return true;
  if (threadIdx.x < 64) {
    const auto *flags = reinterpret_cast<const unsigned long long *>(P.ctl[P.rank] + kPeerFlagOff);
    bool ok = true;
    for (int j = threadIdx.x; j < P.nrecv * kPushWG; j += 64)
      ok = ok && spin_ge(flags + P.recv_rank[j / kPushWG] * kPushWG + (j % kPushWG), tag,
                         P.spin_ticks);
    ok = __all(ok);
    if (threadIdx.x == 0) *ok_lds = ok;
  }
  __syncthreads();
  if (!*ok_lds) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
  return true;
}

// The world sum of `mine` (this rank's local sum, the same in every
// workgroup of the calling kernel) for all-reduce tag t: the first workgroup
// of the kernel to arrive here stores value and tag into every rank's
// mailbox, every workgroup polls its own mailbox until all ranks' tags
// arrived and sums the values in rank order (bit-identical everywhere).
// The publisher is chosen by an agent-scope claim on PeerState::pub (a
// plain load first, so only the early arrivals contend), never by a
// workgroup index: the workgroup that publishes is one that is running, so
// the spins never wait on a workgroup that is not yet resident (dispatch
// order is undefined). Uniform control flow; thread 0's lds slots carry the
// result. false: a spin timed out.
__device__ __forceinline__ bool world_sum(Dd<double> mine, unsigned long long t,
                                          const PeerDev &P, double *res_lds, int *ok_lds) {
  const int par = (int)(t & 1);
  if (threadIdx.x < 64) {
    int claim = 0;
    if (threadIdx.x == 0)
      claim = __hip_atomic_load(&P.state->pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < t &&
              __hip_atomic_fetch_max(&P.state->pub, t, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT) < t;
    const bool publisher = __shfl(claim, 0, 64) != 0;
    bool ok = true;
    if ((int)threadIdx.x < P.world) {
      if (publisher) {
        char *box = P.ctl[threadIdx.x];
        double *val = reinterpret_cast<double *>(box) + 2 * (par * kPeerMax + P.rank);
        st_sysd(val, mine.hi);
        st_sysd(val + 1, mine.lo);
        __threadfence_system();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_sys(reinterpret_cast<unsigned long long *>(box + kPeerTagOff) + par * kPeerMax +
                   P.rank,
               t);
      }
      const auto *tags = reinterpret_cast<const unsigned long long *>(P.ctl[P.rank] + kPeerTagOff);
      ok = spin_ge(tags + par * kPeerMax + threadIdx.x, t, P.spin_ticks);
    }
    ok = __all(ok);
    if (threadIdx.x == 0) {
      *ok_lds = ok;
      if (ok) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
        // the ranks' pairs in rank order, rounded once: the world value no
        // longer depends on how the rows were split between the ranks
        const double *vals =
            reinterpret_cast<const double *>(P.ctl[P.rank]) + 2 * par * kPeerMax;
        Dd<double> s(0.0);
        for (int q = 0; q < P.world; ++q) s += Dd<double>(ld_sysd(vals + 2 * q), ld_sysd(vals + 2 * q + 1));
        *res_lds = s.value();
      }
    }
  }
  __syncthreads();
  return *ok_lds != 0;
}

// Push workgroup wg of nsend x kPushWG: chunk g of send neighbour i's list
// into its landing buffer, then flag [my rank][g] there with this body's tag
// (body_tag). Every storing wave drains its stores, then one lane
// releases them at system scope and raises the flag (MI355X guide, "Valid
// forms"; the asm wait after the fence guards the compiler hazard noted
// there).
// get(j): the value pushed for own row j (v[j], or mode 4's p_k formed as
// r_j + beta p_{k-1,j}: the value the owner's SpMV forms for its own rows)
template <typename T, class Get>
__device__ __forceinline__ void push_wg_from(const Get &get, const PeerDev &P, CgScalars<T> *st,
                                             int slot, int wg) {
  if (skip_body(st, slot, P.state)) return;
  const unsigned long long tag = body_tag(st, slot, P.state);
  const int i = wg / kPushWG, g = wg % kPushWG;
  const int64_t cnt = P.send_cnt[i], off = P.send_off[i];
  const int64_t c0 = cnt * g / kPushWG, c1 = cnt * (g + 1) / kPushWG;
  T *dst = reinterpret_cast<T *>(P.land_remote[i]);
  const int *idx = P.send_idx + off;
  for (int64_t k = c0 + threadIdx.x; k < c1; k += kBlock) dst[k] = get(idx[k]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    auto *flag = reinterpret_cast<unsigned long long *>(P.ctl[P.send_rank[i]] + kPeerFlagOff);
    st_sys(flag + P.rank * kPushWG + g, tag);
  }
}
template <typename T>
__device__ __forceinline__ void push_wg(const T *__restrict__ v, const PeerDev &P,
                                        CgScalars<T> *st, int slot, int wg) {
  push_wg_from<T>([v](int j) { return v[j]; }, P, st, slot, wg);
}

template <typename T>
__device__ __forceinline__ void raise_fault(CgScalars<T> *st, int slot, PeerState *ps) {
  ps->fault = 1;
  if (st) {
    st->active[slot] = 0;
    st->stopped = 3;
  }
}

}  // namespace peerdev
}  // namespace cgx
