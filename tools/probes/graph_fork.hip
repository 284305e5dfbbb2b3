// Does a captured hipGraph run two independent branches concurrently on
// MI355X? Two spin kernels (~100 us each, few workgroups) captured (a) on one
// stream, (b) forked onto a second stream with events. Prints ms per replay.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(long long ticks, int *out) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  int *d;
  CK(hipMalloc(&d, 4096));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t f, j, t0, t1;
  CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const long long ticks = 10000;  // 100 us at the 100 MHz wall clock
  for (int fork = 0; fork < 2; ++fork) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal));
    if (fork) {
      CK(hipEventRecord(f, a));
      CK(hipStreamWaitEvent(b, f, 0));
      hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, b, ticks, d);
      hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, a, ticks, d + 64);
      CK(hipEventRecord(j, b));
      CK(hipStreamWaitEvent(a, j, 0));
    } else {
      hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, a, ticks, d);
      hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, a, ticks, d + 64);
    }
    CK(hipStreamEndCapture(a, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, a));
    CK(hipStreamSynchronize(a));
    CK(hipEventRecord(t0, a));
    for (int r = 0; r < 20; ++r) CK(hipGraphLaunch(ge, a));
    CK(hipEventRecord(t1, a));
    CK(hipEventSynchronize(t1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("%s: %.1f us per replay (2 x 100 us kernels)\n", fork ? "forked" : "serial", ms * 1000 / 20);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
