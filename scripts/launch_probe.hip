// Per-launch cost on one stream, back to back: a small kernel alone, with a
// hipEventRecord after each launch, and with the event attached to the
// launch itself (hipExtLaunchKernelGGL's stop event). Prints one JSON line.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <chrono>

__global__ void small_kernel(int *out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = i;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  int *d;
  CK(hipMalloc(&d, 1 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const int N = 4000;
  double us[3];
  for (int mode = 0; mode < 3; mode++) {
    for (int rep = 0; rep < 2; rep++) {
      CK(hipStreamSynchronize(s));
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < N; i++) {
        if (mode == 2) {
          hipExtLaunchKernelGGL(small_kernel, dim3(8), dim3(256), 0, s, nullptr, ev, 0, d, 2048);
        } else {
          hipLaunchKernelGGL(small_kernel, dim3(8), dim3(256), 0, s, d, 2048);
          if (mode == 1) CK(hipEventRecord(ev, s));
        }
      }
      CK(hipStreamSynchronize(s));
      auto t1 = std::chrono::steady_clock::now();
      us[mode] = std::chrono::duration<double, std::micro>(t1 - t0).count() / N;
    }
  }
  CK(hipEventSynchronize(ev));
  printf("{\"launch_us\": %.2f, \"launch_plus_record_us\": %.2f, \"ext_launch_stop_event_us\": %.2f}\n",
         us[0], us[1], us[2]);
  return 0;
}
