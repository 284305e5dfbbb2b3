// What does the 256^3 7-point SpMV (+ p.Ap partials) cost on MI355X when a
// slice's values come from a per-template scalar table (no code words, no
// LDS dictionary, no per-slot masks)? Kernels over the SELL-P walk of the
// library (128-row slices, 2 rows per lane, XCD-contiguous slice ranges),
// each checked bit for bit against a 1-row-per-thread reference, timed with
// HIP events right after a kernel that rewrites p (p is then the freshest
// 134 MB in the Infinity Cache, as after the CG loop's p update).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o /tmp/sf stencil_floor.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));         \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int NX = 256, NY = 256, NZ = 256;
constexpr int AO = NX, DO = NX * NY;
constexpr long long N = (long long)NX * NY * NZ;
constexpr int NSL = (int)(N / 128);

struct Tpl {  // one template: per-slot values (row-symmetric), absent-edge zeros
  double v[8];
  double zlo, zhi;  // -copysign(0, v): v * z == -0.0, the identity of +
  int plo, phi;     // lane 0 row 0 has the -1 entry / lane 63 row 1 the +1 entry
  int pad[2];
};

__device__ __forceinline__ double shr1(double v, double edge) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(edge), __double2loint(v), 0x138, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(edge), __double2hiint(v), 0x138, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double shl1(double v, double edge) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(edge), __double2loint(v), 0x130, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(edge), __double2hiint(v), 0x130, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ void slice_range(int &first, int &step, int &end) {
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = gridDim.x, b = blockIdx.x, g = b & 7;
  const int lo = (int)(((long long)NSL * g) >> 3);
  first = lo + (b >> 3) * 4 + wid;
  end = (int)(((long long)NSL * (g + 1)) >> 3);
  step = (G >> 3) * 4;
}

__device__ __forceinline__ bool lean_slice(int s) {
  const int y = (s >> 1) & (NY - 1), z = s >> 9;
  return z > 0 && z < NZ - 1 && y > 0 && y < NY - 1;
}

__device__ __forceinline__ double sload(const double *p, int i) {
  return ((const __attribute__((address_space(4))) double *)p)[i];
}

// one row, the reference's order (-D, -a, -1, 0, +1, +a, +D), absent skipped
__device__ __forceinline__ double row_ref(const double *__restrict__ p, long long i) {
  const int x = (int)(i & (NX - 1)), y = (int)((i >> 8) & (NY - 1)), z = (int)(i >> 16);
  double s = 0.0;
  if (z > 0) s = s + (-1.0) * p[i - DO];
  if (y > 0) s = s + (-1.0) * p[i - AO];
  if (x > 0) s = s + (-1.0) * p[i - 1];
  s = s + 6.0 * p[i];
  if (x < NX - 1) s = s + (-1.0) * p[i + 1];
  if (y < NY - 1) s = s + (-1.0) * p[i + AO];
  if (z < NZ - 1) s = s + (-1.0) * p[i + DO];
  return s;
}

__device__ __forceinline__ double block_sum(double v, double *lds) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) lds[w] = v;
  __syncthreads();
  double r = 0;
  if (threadIdx.x == 0) r = ((lds[0] + lds[1]) + lds[2]) + lds[3];
  return r;
}

__global__ __launch_bounds__(256) void k_ref(const double *__restrict__ p, double *__restrict__ Ap) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < N) Ap[i] = row_ref(p, i);
}

// p = q (the "p update" stand-in before each timed SpMV)
typedef double D2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_write_p(const D2 *__restrict__ q, D2 *__restrict__ p, long long n2) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long long)gridDim.x * 256)
    p[i] = __builtin_nontemporal_load(q + i);
}

// the generic slice (boundary lines and planes): two rows per lane
__device__ __forceinline__ void slice_generic(const double *__restrict__ p, double *__restrict__ Ap,
                                              int s, double &dot) {
  const int lane = threadIdx.x & 63;
  const long long r0 = (long long)s * 128 + 2 * lane;
  const double a0 = row_ref(p, r0), a1 = row_ref(p, r0 + 1);
  Ap[r0] = a0;
  Ap[r0 + 1] = a1;
  dot += a0 * p[r0];
  dot += a1 * p[r0 + 1];
}

struct Buf {
  double2 mD, ma, c, pa, pD;
  double elo, ehi;
};

template <bool VEDGE>
__device__ __forceinline__ void issue(const double *__restrict__ p, int s, Buf &b) {
  const int lane = threadIdx.x & 63;
  const unsigned rb = (unsigned)(s * 128 + 2 * lane) * 8u;
  const char *pc = reinterpret_cast<const char *>(p);
  b.c = *reinterpret_cast<const double2 *>(pc + rb);
  b.mD = *reinterpret_cast<const double2 *>(pc + rb - DO * 8u);
  b.ma = *reinterpret_cast<const double2 *>(pc + rb - AO * 8u);
  b.pa = *reinterpret_cast<const double2 *>(pc + rb + AO * 8u);
  b.pD = *reinterpret_cast<const double2 *>(pc + rb + DO * 8u);
  if constexpr (VEDGE) {
    // lane 0: x[first - 1], lane 63: x[first + 128]; the others re-read their
    // own center (same lines)
    const int e = lane == 0 ? s * 128 - 1 : lane == 63 ? s * 128 + 128 : s * 128 + 2 * lane;
    b.elo = p[e];
    b.ehi = b.elo;
  } else {
    b.elo = sload(p, s * 128 - 1);
    b.ehi = sload(p, s * 128 + 128);
  }
}

__device__ __forceinline__ void compute(double *__restrict__ Ap, int s, const Buf &b,
                                        const Tpl &t, double &dot) {
  const int lane = threadIdx.x & 63;
  const double elo = t.plo ? b.elo : t.zlo;
  const double ehi = t.phi ? b.ehi : t.zhi;
  const double left = shr1(b.c.y, elo), right = shl1(b.c.x, ehi);
  double a0 = 0.0, a1 = 0.0;
  a0 = a0 + t.v[0] * b.mD.x;
  a1 = a1 + t.v[0] * b.mD.y;
  a0 = a0 + t.v[1] * b.ma.x;
  a1 = a1 + t.v[1] * b.ma.y;
  a0 = a0 + t.v[2] * left;
  a1 = a1 + t.v[2] * b.c.x;
  a0 = a0 + t.v[3] * b.c.x;
  a1 = a1 + t.v[3] * b.c.y;
  a0 = a0 + t.v[4] * b.c.y;
  a1 = a1 + t.v[4] * right;
  a0 = a0 + t.v[5] * b.pa.x;
  a1 = a1 + t.v[5] * b.pa.y;
  a0 = a0 + t.v[6] * b.pD.x;
  a1 = a1 + t.v[6] * b.pD.y;
  double2 o;
  o.x = a0;
  o.y = a1;
  *reinterpret_cast<double2 *>(Ap + (long long)s * 128 + 2 * lane) = o;
  dot += a0 * b.c.x;
  dot += a1 * b.c.y;
}

__device__ __forceinline__ Tpl tpl_at(const Tpl *__restrict__ tab, int t) {
  const auto *tp = (const __attribute__((address_space(4))) Tpl *)tab + t;
  Tpl r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r.v[j] = tp->v[j];
  r.zlo = tp->zlo;
  r.zhi = tp->zhi;
  r.plo = tp->plo;
  r.phi = tp->phi;
  return r;
}

// variant 0: one slice at a time (loads, wait, compute)
// variant 1: next slice's loads issued before this slice's compute
// TID: how a slice finds its template: 0 a scalar load of stid[s] per slice,
// 1 arithmetic (s & 1, no load), 2 one vector load of stid for the wave's
// next 64 slices, then v_readlane per slice
// GEN: 0 boundary slices by the generic path, 1 skipped (timing only)
template <int VAR, bool VEDGE, int WAVES, int TID, int GEN>
__global__ __launch_bounds__(256, WAVES) void k_lean(const double *__restrict__ p, double *__restrict__ Ap,
                                                     const Tpl *__restrict__ tab, const int *__restrict__ stid,
                                                     double *__restrict__ part) {
  __shared__ double lds[4];
  int s, step, end;
  slice_range(s, step, end);
  const int lane = threadIdx.x & 63;
  double dot = 0.0;
  int bv = 0, kb = 64;
  auto tid_of = [&](int sl) -> int {
    if constexpr (TID == 0) {
      return ((const __attribute__((address_space(4))) int *)stid)[sl];
    } else if constexpr (TID == 1) {
      return sl & 1;
    } else {
      if (kb == 64) {
        bv = stid[min(sl + lane * step, end - 1)];
        kb = 0;
      }
      return __builtin_amdgcn_readlane(bv, kb++);
    }
  };
  auto generic = [&](int sl) {
    (void)tid_of(sl);
    if constexpr (GEN == 0) slice_generic(p, Ap, sl, dot);
  };
  if constexpr (VAR == 0) {
    for (; s < end; s += step) {
      if (!lean_slice(s)) {
        generic(s);
        continue;
      }
      Buf b;
      issue<VEDGE>(p, s, b);
      const Tpl t = tpl_at(tab, tid_of(s));
      compute(Ap, s, b, t, dot);
    }
  } else {
    while (s < end) {
      if (!lean_slice(s)) {
        generic(s);
        s += step;
        continue;
      }
      Buf A, B;
      issue<VEDGE>(p, s, A);
      // body(cur in X, prefetch into Y): returns whether the walk goes on in the
      // lean loop with Y holding the next slice
      auto body = [&](Buf &X, Buf &Y) -> bool {
        const int ns = s + step;
        const bool hn = ns < end && lean_slice(ns);
        issue<VEDGE>(p, hn ? ns : s, Y);
        const Tpl t = tpl_at(tab, tid_of(s));
        compute(Ap, s, X, t, dot);
        s = ns;
        return hn;
      };
      while (body(A, B) && body(B, A)) {
      }
    }
  }
  const double v = block_sum(dot, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = v;
}

// ceiling: the same walk, center pair loaded, Ap = 6 p stored, the dot
template <int WAVES>
__global__ __launch_bounds__(256, WAVES) void k_copy(const double *__restrict__ p, double *__restrict__ Ap,
                                                     double *__restrict__ part) {
  __shared__ double lds[4];
  int s, step, end;
  slice_range(s, step, end);
  const int lane = threadIdx.x & 63;
  double dot = 0.0;
  for (; s < end; s += step) {
    const long long r0 = (long long)s * 128 + 2 * lane;
    const double2 c = *reinterpret_cast<const double2 *>(p + r0);
    double2 o;
    o.x = 6.0 * c.x;
    o.y = 6.0 * c.y;
    *reinterpret_cast<double2 *>(Ap + r0) = o;
    dot += o.x * c.x;
    dot += o.y * c.y;
  }
  const double v = block_sum(dot, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = v;
}

// the same walk with all five loads per slice (no template, values -1/6
// constant, no masks: the wrong answer on edges; a timing ablation)
template <int WAVES>
__global__ __launch_bounds__(256, WAVES) void k_five(const double *__restrict__ p, double *__restrict__ Ap,
                                                     double *__restrict__ part) {
  __shared__ double lds[4];
  int s, step, end;
  slice_range(s, step, end);
  const int lane = threadIdx.x & 63;
  double dot = 0.0;
  for (; s < end; s += step) {
    const int y = (s >> 1) & (NY - 1), z = s >> 9;
    if (!(z > 0 && z < NZ - 1)) continue;
    const long long r0 = (long long)s * 128 + 2 * lane;
    const double2 c = *reinterpret_cast<const double2 *>(p + r0);
    const double2 a = *reinterpret_cast<const double2 *>(p + r0 - DO);
    const double2 b = *reinterpret_cast<const double2 *>(p + r0 + DO);
    const double2 d = *reinterpret_cast<const double2 *>(p + r0 - (y > 0 ? AO : 0));
    const double2 e = *reinterpret_cast<const double2 *>(p + r0 + (y < NY - 1 ? AO : 0));
    double2 o;
    o.x = (((6.0 * c.x - a.x) - b.x) - d.x) - e.x;
    o.y = (((6.0 * c.y - a.y) - b.y) - d.y) - e.y;
    *reinterpret_cast<double2 *>(Ap + r0) = o;
    dot += o.x * c.x;
    dot += o.y * c.y;
  }
  const double v = block_sum(dot, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = v;
}


// timing ablation: five loads per slice; bit 1: -D real, 2: +D real, 4: -a
// real, 8: +a real (a load that is not real re-reads the center address: same
// lines, an L1 hit); WGW waves per workgroup take consecutive slices
template <int MASK, int WGW>
__global__ __launch_bounds__(64 * WGW) void k_abl(const double *__restrict__ p, double *__restrict__ Ap,
                                                  double *__restrict__ part) {
  __shared__ double lds[16];
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = gridDim.x, b = blockIdx.x, g = b & 7;
  const int lo = (int)(((long long)NSL * g) >> 3);
  int s = lo + (b >> 3) * WGW + wid;
  const int end = (int)(((long long)NSL * (g + 1)) >> 3);
  const int step = (G >> 3) * WGW;
  const int lane = threadIdx.x & 63;
  double dot = 0.0;
  for (; s < end; s += step) {
    const int z = s >> 9;
    if (!(z > 0 && z < NZ - 1)) continue;
    const long long r0 = (long long)s * 128 + 2 * lane;
    const double2 c = *reinterpret_cast<const double2 *>(p + r0);
    const double2 a = *reinterpret_cast<const double2 *>(p + r0 - ((MASK & 1) ? DO : 0));
    const double2 bb = *reinterpret_cast<const double2 *>(p + r0 + ((MASK & 2) ? DO : 0));
    const double2 d = *reinterpret_cast<const double2 *>(p + r0 - ((MASK & 4) ? AO : 0));
    const double2 e = *reinterpret_cast<const double2 *>(p + r0 + ((MASK & 8) ? AO : 0));
    double2 o;
    o.x = (((6.0 * c.x - a.x) - bb.x) - d.x) - e.x;
    o.y = (((6.0 * c.y - a.y) - bb.y) - d.y) - e.y;
    *reinterpret_cast<double2 *>(Ap + r0) = o;
    dot += o.x * c.x;
    dot += o.y * c.y;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) dot += __shfl_down(dot, off, 64);
  if (lane == 0) lds[wid] = dot;
  __syncthreads();
  if (threadIdx.x == 0) {
    double v = 0;
    for (int w = 0; w < WGW; ++w) v += lds[w];
    part[blockIdx.x] = v;
  }
}

template <class K>
int resident(K kern) {
  int nb = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 256, 0));
  return nb;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  double *p, *q, *Ap, *Ar, *part;
  Tpl *tab;
  int *stid;
  CK(hipMalloc(&p, N * 8));
  CK(hipMalloc(&q, N * 8));
  CK(hipMalloc(&Ap, N * 8));
  CK(hipMalloc(&Ar, N * 8));
  CK(hipMalloc(&part, 65536 * 8));
  CK(hipMalloc(&tab, 2 * sizeof(Tpl)));
  CK(hipMalloc(&stid, NSL * 4));
  {
    std::vector<double> h(N);
    unsigned long long z = 88172645463325252ull;
    for (long long i = 0; i < N; ++i) {
      z ^= z << 13;
      z ^= z >> 7;
      z ^= z << 17;
      h[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5;
    }
    CK(hipMemcpy(q, h.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(p, h.data(), N * 8, hipMemcpyHostToDevice));
    Tpl t[2];
    memset(t, 0, sizeof(t));
    for (int k = 0; k < 2; ++k) {
      for (int j = 0; j < 7; ++j) t[k].v[j] = j == 3 ? 6.0 : -1.0;
      t[k].zlo = -copysign(0.0, t[k].v[2]);
      t[k].zhi = -copysign(0.0, t[k].v[4]);
      t[k].plo = k == 1;  // second half: x = 128 has its -1 entry
      t[k].phi = k == 0;  // first half: x = 127 has its +1 entry
    }
    CK(hipMemcpy(tab, t, sizeof(t), hipMemcpyHostToDevice));
    std::vector<int> st(NSL);
    for (int s = 0; s < NSL; ++s) st[s] = s & 1;
    CK(hipMemcpy(stid, st.data(), NSL * 4, hipMemcpyHostToDevice));
  }
  hipLaunchKernelGGL(k_ref, dim3((unsigned)(N / 256)), dim3(256), 0, 0, p, Ar);
  CK(hipDeviceSynchronize());
  std::vector<double> ref(N), got(N);
  CK(hipMemcpy(ref.data(), Ar, N * 8, hipMemcpyDeviceToHost));

  struct V {
    const char *name;
    const void *fn;
    int kind;  // 0 lean, 1 copy, 2 five
    int grid;
    bool check;
    int block = 256;
  };
  std::vector<V> vs;
  auto add = [&](const char *nm, const void *fn, int kind, int occ, bool check) {
    for (int mult : {0, 1, 2}) {
      int g = mult == 0 ? 512 : mult == 1 ? 1024 : 2048;
      if (g > occ * cus) continue;
      g = std::max(8, g / 8 * 8);
      char *buf = (char *)malloc(96);
      snprintf(buf, 96, "%s g%d", nm, g);
      vs.push_back({buf, fn, kind, g, check, 256});
    }
  };
#define ADDL(VAR, VE, W, TID, GEN)                                                          \
  add("lean v" #VAR " ve" #VE " w" #W " tid" #TID " gen" #GEN,                               \
      (const void *)k_lean<VAR, VE, W, TID, GEN>, 0, resident(k_lean<VAR, VE, W, TID, GEN>), GEN == 0)
  ADDL(0, false, 8, 0, 0);
  ADDL(0, false, 8, 1, 0);
  ADDL(0, false, 8, 2, 0);
  ADDL(0, false, 8, 0, 1);
  ADDL(0, false, 8, 1, 1);
  ADDL(0, true, 8, 1, 1);
  ADDL(1, false, 8, 1, 1);
  ADDL(1, true, 8, 1, 1);
  ADDL(1, true, 8, 2, 0);
  ADDL(1, true, 8, 2, 1);
  add("copy w8", (const void *)k_copy<8>, 1, resident(k_copy<8>), false);
  add("five w8", (const void *)k_five<8>, 2, resident(k_five<8>), false);
#define ADDA(M, W)                                                                            \
  for (int gg : {1024, 2048, 4096}) {                                                         \
    char *buf = (char *)malloc(96);                                                           \
    snprintf(buf, 96, "abl mask%d wgw%d g%d", M, W, gg * 4 / W);                              \
    vs.push_back({buf, (const void *)k_abl<M, W>, 3, gg * 4 / W, false, 64 * W});             \
  }
  ADDA(15, 4);

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> t(vs.size());
  for (int r = 0; r < reps; ++r) {
    for (size_t k = 0; k < vs.size(); ++k) {
      hipLaunchKernelGGL(k_write_p, dim3(1024), dim3(256), 0, 0, (const D2 *)q, (D2 *)p, N / 2);
      CK(hipEventRecord(e0, 0));
      if (vs[k].kind == 0) {
        void *args[] = {&p, &Ap, &tab, &stid, &part};
        CK(hipLaunchKernel(vs[k].fn, dim3(vs[k].grid), dim3(256), args, 0, 0));
      } else {
        void *args[] = {&p, &Ap, &part};
        CK(hipLaunchKernel(vs[k].fn, dim3(vs[k].grid), dim3(vs[k].block), args, 0, 0));
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[k].push_back(ms * 1000.f);
      if (r == 0 && vs[k].check) {
        CK(hipMemcpy(got.data(), Ap, N * 8, hipMemcpyDeviceToHost));
        long long bad = 0;
        for (long long i = 0; i < N; ++i)
          if (memcmp(&got[i], &ref[i], 8) != 0 && ++bad < 4)
            printf("  %s: row %lld got %.17g want %.17g\n", vs[k].name, i, got[i], ref[i]);
        printf("check %-28s %s (%lld rows differ)\n", vs[k].name, bad ? "FAIL" : "bit-exact", bad);
      }
    }
  }
  const double bytes = 2.0 * N * 8;
  for (size_t k = 0; k < vs.size(); ++k) {
    std::vector<float> x = t[k];
    std::sort(x.begin(), x.end());
    const double med = x[x.size() / 2];
    printf("%-30s median %7.2f us  min %7.2f us  %6.3f TB/s (p+Ap)  frac %.3f\n", vs[k].name, med,
           x[0], bytes / med * 1e-6, bytes / med * 1e-6 / 8.0);
  }
  return 0;
}
