// ipc_probe.hip — feasibility probe for a device-side peer transport
// (DESIGN.md §9): W processes share GPU 0 (or use GPU r when several are
// visible), exchange hipIpc handles of their mailbox buffers, and run
//   1. an in-kernel all-reduce ping (1 workgroup, value + tag per rank),
//   2. the same, one kernel launch per all-reduce,
//   3. a halo push: 64 workgroups write 512 KB into the next rank's landing
//      buffer, flag per workgroup; the receiver waits, copies, checks.
// Every spin is bounded (2 s of wall clock); a timeout sets an error word.
//   hipcc --offload-arch=gfx950 -O3 tools/ipc_probe.hip -o build/ipc_probe
//   build/ipc_probe [world=2] [uncached=1]
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "rank %d: %s failed: %s\n", g_rank, #x, hipGetErrorString(e_)); \
      _exit(3);                                                                \
    }                                                                          \
  } while (0)

static int g_rank = 0;
constexpr int kMaxW = 8;
constexpr long long kSpin = 200000000LL;  // 2 s at the 100 MHz wall clock

struct Peers {
  double *box[kMaxW];          // mailbox of rank q (values: [2][kMaxW], tags after)
  double *land[kMaxW];         // halo landing buffer of rank q
  unsigned long long *flag[kMaxW];
};

__device__ inline void st_sys(unsigned long long *p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline unsigned long long ld_sys(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void st_sysd(double *p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline double ld_sysd(const double *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one all-reduce: lane q < W stores my value into rank q's mailbox, fences,
// stores the tag; then lane s < W polls my mailbox's tag from rank s
__device__ bool allreduce_once(const Peers &P, int rank, int W, long long it, double v,
                               double *out) {
  const int l = threadIdx.x;
  const int par = (int)(it & 1);
  if (l < W) {
    double *b = P.box[l];
    st_sysd(b + par * kMaxW + rank, v);
    __threadfence_system();
    st_sys((unsigned long long *)(b + 2 * kMaxW) + par * kMaxW + rank, (unsigned long long)it);
  }
  double *mine = P.box[rank];
  const long long t0 = wall_clock64();
  bool ok = true;
  if (l < W) {
    const unsigned long long *tg = (const unsigned long long *)(mine + 2 * kMaxW) + par * kMaxW + l;
    while (ld_sys(tg) < (unsigned long long)it) {
      if (wall_clock64() - t0 > kSpin) { ok = false; break; }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  ok = __all(ok || l >= W);
  __threadfence_system();
  double s = 0;
  if (ok)
    for (int q = 0; q < W; ++q) s += ld_sysd(mine + par * kMaxW + q);  // rank order
  *out = s;
  return ok;
}

__global__ void k_ar_loop(Peers P, int rank, int W, long long it0, int iters, int *err,
                          long long *ticks) {
  const long long t0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
    const long long it = it0 + i;
    double s;
    if (!allreduce_once(P, rank, W, it, (double)(rank * 1000 + it), &s)) {
      if (threadIdx.x == 0) atomicAdd(err, 1);
      return;
    }
    double want = 0;
    for (int q = 0; q < W; ++q) want += (double)(q * 1000 + it);
    if (s != want && threadIdx.x == 0) atomicAdd(err + 1, 1);
  }
  if (threadIdx.x == 0) *ticks = wall_clock64() - t0;
}

// halo push: block b of 64 writes its 8 KB slice of the payload into the
// next rank's landing buffer, then (after a system fence) its flag
__global__ void k_push(Peers P, int rank, int W, long long it, int n) {
  const int to = (rank + 1) % W;
  double *dst = P.land[to];
  const int per = n / gridDim.x;
  for (int i = threadIdx.x; i < per; i += blockDim.x) {
    const int k = blockIdx.x * per + i;
    dst[k] = (double)(rank * 7 + k) + 0.5 * (double)it;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    st_sys(P.flag[to] + rank * 64 + blockIdx.x, (unsigned long long)it);
  }
}

__global__ void k_recv(Peers P, int rank, int W, long long it, int n, double *local, int *err) {
  const int from = (rank + W - 1) % W;
  __shared__ int ok;
  if (threadIdx.x < 64) {
    const unsigned long long *f = P.flag[rank] + from * 64 + threadIdx.x;
    const long long t0 = wall_clock64();
    bool good = true;
    while (ld_sys(f) < (unsigned long long)it) {
      if (wall_clock64() - t0 > kSpin) { good = false; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    good = __all(good);
    if (threadIdx.x == 0) ok = good;
  }
  __syncthreads();
  if (!ok) {
    if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(err, 1);
    return;
  }
  __threadfence_system();
  const double *src = P.land[rank];
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    const double v = ld_sysd(src + k);
    local[k] = v;
    if (v != (double)(from * 7 + k) + 0.5 * (double)it) atomicAdd(err + 1, 1);
  }
}

static std::string path_of(const char *dir, const char *what, int r) {
  return std::string(dir) + "/" + what + std::to_string(r);
}

static void put_handle(const char *dir, const char *what, int r, void *ptr) {
  hipIpcMemHandle_t h;
  CK(hipIpcGetMemHandle(&h, ptr));
  std::string p = path_of(dir, what, r), t = p + ".tmp";
  FILE *f = fopen(t.c_str(), "wb");
  fwrite(&h, sizeof(h), 1, f);
  fclose(f);
  rename(t.c_str(), p.c_str());
}

static void *get_handle(const char *dir, const char *what, int r) {
  std::string p = path_of(dir, what, r);
  hipIpcMemHandle_t h;
  for (int i = 0; i < 3000; ++i) {
    FILE *f = fopen(p.c_str(), "rb");
    if (f) {
      size_t k = fread(&h, sizeof(h), 1, f);
      fclose(f);
      if (k == 1) {
        void *ptr = nullptr;
        CK(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
        return ptr;
      }
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  fprintf(stderr, "rank %d: no handle %s\n", g_rank, p.c_str());
  _exit(4);
}

static void barrier(const char *dir, const char *name, int W) {
  std::string p = path_of(dir, name, g_rank);
  FILE *f = fopen(p.c_str(), "w");
  fclose(f);
  for (int q = 0; q < W; ++q) {
    std::string pq = path_of(dir, name, q);
    for (int i = 0; i < 3000 && access(pq.c_str(), F_OK) != 0; ++i)
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
}

static int run(int rank, int W, bool uncached, const char *dir) {
  g_rank = rank;
  int ndev = 0;
  CK(hipGetDeviceCount(&ndev));
  CK(hipSetDevice(rank % ndev));
  const int nhalo = 64 * 1024;  // 512 KB of doubles
  auto xalloc = [&](void **p, size_t b) {
    if (uncached) CK(hipExtMallocWithFlags(p, b, hipDeviceMallocUncached));
    else CK(hipMalloc(p, b));
    CK(hipMemset(*p, 0, b));
  };
  void *box, *land, *flag;
  xalloc(&box, 4096);
  xalloc(&land, nhalo * sizeof(double));
  xalloc(&flag, kMaxW * 64 * 8);
  CK(hipDeviceSynchronize());
  put_handle(dir, "box", rank, box);
  put_handle(dir, "land", rank, land);
  put_handle(dir, "flag", rank, flag);
  Peers P{};
  for (int q = 0; q < W; ++q) {
    if (q == rank) {
      P.box[q] = (double *)box;
      P.land[q] = (double *)land;
      P.flag[q] = (unsigned long long *)flag;
    } else {
      P.box[q] = (double *)get_handle(dir, "box", q);
      P.land[q] = (double *)get_handle(dir, "land", q);
      P.flag[q] = (unsigned long long *)get_handle(dir, "flag", q);
    }
  }
  barrier(dir, "opened", W);
  int *err;
  long long *ticks;
  double *local;
  CK(hipMalloc(&err, 64));
  CK(hipMemset(err, 0, 64));
  CK(hipMalloc(&ticks, 64));
  CK(hipMalloc(&local, nhalo * sizeof(double)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // 1. in-kernel loop
  const int iters = 2000;
  hipLaunchKernelGGL(k_ar_loop, dim3(1), dim3(64), 0, s, P, rank, W, 1LL, iters, err, ticks);
  CK(hipStreamSynchronize(s));
  int herr[4];
  long long ht;
  CK(hipMemcpy(herr, err, 16, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&ht, ticks, 8, hipMemcpyDeviceToHost));
  printf("{\"rank\": %d, \"test\": \"ar_loop\", \"uncached\": %d, \"timeouts\": %d, \"wrong\": %d, "
         "\"us_per_allreduce\": %.3f}\n", rank, (int)uncached, herr[0], herr[1],
         herr[0] ? -1.0 : ht / 100.0 / iters);
  fflush(stdout);
  if (herr[0]) return 5;
  // 2. one launch per all-reduce
  barrier(dir, "t2", W);
  const int iters2 = 500;
  auto c0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters2; ++i)
    hipLaunchKernelGGL(k_ar_loop, dim3(1), dim3(64), 0, s, P, rank, W, (long long)(iters + 1 + i),
                       1, err, ticks);
  CK(hipStreamSynchronize(s));
  double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c0).count();
  CK(hipMemcpy(herr, err, 16, hipMemcpyDeviceToHost));
  printf("{\"rank\": %d, \"test\": \"ar_launch\", \"uncached\": %d, \"timeouts\": %d, \"wrong\": %d, "
         "\"us_per_allreduce\": %.3f}\n", rank, (int)uncached, herr[0], herr[1], us / iters2);
  fflush(stdout);
  if (herr[0]) return 6;
  // 3. halo push + receive
  barrier(dir, "t3", W);
  const int iters3 = 200;
  c0 = std::chrono::steady_clock::now();
  for (int i = 1; i <= iters3; ++i) {
    hipLaunchKernelGGL(k_push, dim3(64), dim3(256), 0, s, P, rank, W, (long long)i, nhalo);
    hipLaunchKernelGGL(k_recv, dim3(64), dim3(256), 0, s, P, rank, W, (long long)i, nhalo, local,
                       err + 2);
    // the landing buffer is reused next iteration: a sender may overwrite
    // it only after this rank consumed it — an all-reduce orders that
    hipLaunchKernelGGL(k_ar_loop, dim3(1), dim3(64), 0, s, P, rank, W,
                       (long long)(iters + iters2 + 1 + i), 1, err, ticks);
  }
  CK(hipStreamSynchronize(s));
  us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c0).count();
  CK(hipMemcpy(herr, err, 16, hipMemcpyDeviceToHost));
  printf("{\"rank\": %d, \"test\": \"halo\", \"uncached\": %d, \"timeouts\": %d, \"wrong\": %d, "
         "\"us_per_iter\": %.3f}\n", rank, (int)uncached, herr[2] + herr[0], herr[3] + herr[1],
         us / iters3);
  fflush(stdout);
  barrier(dir, "done", W);
  for (int q = 0; q < W; ++q)
    if (q != rank) {
      CK(hipIpcCloseMemHandle(P.box[q]));
      CK(hipIpcCloseMemHandle(P.land[q]));
      CK(hipIpcCloseMemHandle(P.flag[q]));
    }
  return (herr[2] || herr[3] || herr[1]) ? 7 : 0;
}

int main(int argc, char **argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 2;
  const bool uncached = argc > 2 ? atoi(argv[2]) != 0 : true;
  char dir[] = "/tmp/ipcprobeXXXXXX";
  if (!mkdtemp(dir)) return 2;
  // fork BEFORE any HIP call: every rank initialises its own runtime
  pid_t kids[kMaxW];
  for (int r = 1; r < W; ++r) {
    pid_t p = fork();
    if (p == 0) _exit(run(r, W, uncached, dir));
    kids[r] = p;
  }
  int rc = run(0, W, uncached, dir);
  for (int r = 1; r < W; ++r) {
    int st = 0;
    waitpid(kids[r], &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st)) rc = rc ? rc : 10 + r;
  }
  printf("{\"probe\": \"done\", \"world\": %d, \"uncached\": %d, \"rc\": %d}\n", W, (int)uncached, rc);
  return rc;
}
