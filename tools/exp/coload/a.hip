// Probe (tools/exp/coload): when does HIP load a translation unit's code
// object?  TU a: one small kernel and the timed driver; TU b: many template
// instantiations (stand-in for the engine's xor_stream width set).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
__global__ void small_kernel(int *p) { if (threadIdx.x == 0) p[blockIdx.x] += 1; }
void launch_b(int which, int *p, hipStream_t s);
static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int main() {
  double t = now_ms();
  hipSetDevice(0);
  hipFree(nullptr);
  printf("{\"step\": \"init\", \"ms\": %.2f}\n", now_ms() - t);
  t = now_ms();
  hipStream_t s; int *p;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipMalloc(&p, 4096);
  hipMemsetAsync(p, 0, 4096, s);
  hipStreamSynchronize(s);
  printf("{\"step\": \"stream_malloc_memset\", \"ms\": %.2f}\n", now_ms() - t);
  t = now_ms();
  hipLaunchKernelGGL(small_kernel, dim3(1), dim3(64), 0, s, p);
  hipStreamSynchronize(s);
  printf("{\"step\": \"first_launch_tu_a\", \"ms\": %.2f}\n", now_ms() - t);
  t = now_ms();
  launch_b(0, p, s);
  hipStreamSynchronize(s);
  printf("{\"step\": \"first_launch_tu_b\", \"ms\": %.2f}\n", now_ms() - t);
  t = now_ms();
  launch_b(7, p, s);
  hipStreamSynchronize(s);
  printf("{\"step\": \"second_kernel_tu_b\", \"ms\": %.2f}\n", now_ms() - t);
  int h = 0;
  hipMemcpy(&h, p, 4, hipMemcpyDeviceToHost);
  printf("{\"step\": \"check\", \"value\": %d}\n", h);
  return h == 3 ? 0 : 1;
}
