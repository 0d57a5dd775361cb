// HIP-event timing vs the device's own clock, for the bench's k_cadmm launch timing.
// The step shape of the C-ADMM bench on one stream: a short kernel ("bucket"), event A, the timed
// kernel, event B, a short kernel ("rollout"), host wait on B.  The timed kernel busy-waits a fixed
// span of the shader's real-time clock in every workgroup (1,024 workgroups of 64 lanes), and
// records its first start / last end through global atomics, so each launch's device span is known
// exactly.  Variants: the timed kernel with ~2 KB/lane of scratch (as k_cadmm), and the events
// created with hipEventDisableSystemFence.
//
//   hipcc --offload-arch=gfx950 -O2 tools/event_probe.hip -o tools/event_probe && tools/event_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

__device__ __forceinline__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

__global__ void spin(unsigned long long ticks, unsigned long long* ts) {
  const unsigned long long t0 = rt();
  while (rt() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
  if (ts && threadIdx.x == 0) {
    atomicMin(ts, t0);
    atomicMax(ts + 1, rt());
  }
}

// the same span with a private array that lives in scratch (~2 KB per lane)
__global__ void spin_scratch(unsigned long long ticks, unsigned long long* ts, int k) {
  volatile double a[256];
  const unsigned long long t0 = rt();
  for (int i = 0; i < 256; ++i) a[i] = i * (double)k;
  double s = 0;
  while (rt() - t0 < ticks) {
    s += a[(threadIdx.x + (int)s) & 255];
    __builtin_amdgcn_s_sleep(2);
  }
  if (ts && threadIdx.x == 0) {
    atomicMin(ts, t0);
    atomicMax(ts + 1, rt() + (s < -1.0 ? 1 : 0));
  }
}

int main() {
  int khz = 0;
  CHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const double tick_us = 1e3 / khz;
  printf("wall clock %d kHz\n", khz);
  hipStream_t st;
  CHK(hipStreamCreate(&st));
  unsigned long long* ts;
  CHK(hipMalloc(&ts, 2 * sizeof(unsigned long long)));
  const unsigned long long init[2] = {~0ull, 0ull};
  const int reps = 20;
  const unsigned long long us = (unsigned long long)(1.0 / tick_us + 0.5);  // ticks per microsecond
  for (int variant = 0; variant < 4; ++variant) {
    const bool scratch = variant & 1, nofence = variant & 2;
    hipEvent_t a, b;
    if (nofence) {
      CHK(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
      CHK(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
    } else {
      CHK(hipEventCreate(&a));
      CHK(hipEventCreate(&b));
    }
    double ev_sum = 0, dev_sum = 0;
    for (int r = 0; r < reps + 2; ++r) {
      CHK(hipMemcpyAsync(ts, init, sizeof(init), hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(spin, dim3(1), dim3(512), 0, st, 50 * us, nullptr);  // the "bucket"
      CHK(hipEventRecord(a, st));
      if (scratch)
        hipLaunchKernelGGL(spin_scratch, dim3(1024), dim3(64), 0, st, 1000 * us, ts, r);
      else
        hipLaunchKernelGGL(spin, dim3(1024), dim3(64), 0, st, 1000 * us, ts);
      CHK(hipEventRecord(b, st));
      hipLaunchKernelGGL(spin, dim3(8192), dim3(64), 0, st, 150 * us, nullptr);  // the "rollout"
      CHK(hipGetLastError());
      CHK(hipEventSynchronize(b));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, a, b));
      unsigned long long h[2];
      CHK(hipMemcpyAsync(h, ts, sizeof(h), hipMemcpyDeviceToHost, st));
      CHK(hipStreamSynchronize(st));
      if (r >= 2) {
        ev_sum += ms * 1e3;
        dev_sum += (h[1] - h[0]) * tick_us;
      }
    }
    printf("{\"variant\": \"%s%s\", \"event_us\": %.1f, \"device_span_us\": %.1f}\n", scratch ? "scratch" : "plain",
           nofence ? "+nofence" : "", ev_sum / reps, dev_sum / reps);
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
  }
  CHK(hipFree(ts));
  CHK(hipStreamDestroy(st));
  return 0;
}
