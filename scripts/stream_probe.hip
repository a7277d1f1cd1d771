// What HIP does with a stream handle after hipStreamDestroy while the
// stream still has a kernel running: does destroy wait for the kernel, and
// what do hipStreamQuery / hipEventRecord return on the stale handle (and on
// a new stream that may reuse the address)? JSON lines; on this image the
// stale-handle calls take the process down (the first line survives).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <chrono>

__global__ void spin_kernel(unsigned long long cycles, int *flag) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < cycles) __builtin_amdgcn_s_sleep(100);
  if (threadIdx.x == 0) *flag = 1;
}

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
  int *d_flag, h_flag = 0;
  if (hipMalloc(&d_flag, 4) != hipSuccess) return 1;
  (void)hipMemset(d_flag, 0, 4);
  (void)hipDeviceSynchronize();
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  // ~300 ms at 100 MHz
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, 30000000ull, d_flag);
  auto t0 = std::chrono::steady_clock::now();
  const hipError_t ed = hipStreamDestroy(s);
  const double destroy_ms = ms_since(t0);
  (void)hipMemcpy(&h_flag, d_flag, 4, hipMemcpyDeviceToHost);  // (null stream)
  const int kernel_done_after_destroy = h_flag;
  printf("{\"destroy_ms\": %.1f, \"destroy_rc\": %d, \"kernel_done_when_checked\": %d}\n",
         destroy_ms, (int)ed, kernel_done_after_destroy);
  fflush(stdout);  // (the calls on the stale handle below may not return)
  const hipError_t eq = hipStreamQuery(s);
  const hipError_t er = hipEventRecord(ev, s);
  (void)hipGetLastError();
  hipStream_t s2;
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  const int same_address = s2 == s;
  printf("{\"destroy_ms\": %.1f, \"destroy_rc\": %d, \"kernel_done_when_checked\": %d, "
         "\"query_stale_rc\": %d, \"record_stale_rc\": %d, \"new_stream_same_address\": %d}\n",
         destroy_ms, (int)ed, kernel_done_after_destroy, (int)eq, (int)er, same_address);
  (void)hipStreamDestroy(s2);
  return 0;
}
