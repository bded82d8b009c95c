// TU b of the coload probe: 256 instantiations of a kernel with a few KiB of code each.
#include <hip/hip_runtime.h>
template <int K>
__global__ void many_kernel(int *p) {
  unsigned x = threadIdx.x * 2654435761u + K;
#pragma unroll
  for (int i = 0; i < 64; i++) x = (x ^ (x >> 7)) * 0x9E3779B1u + i * K;
  if (threadIdx.x == 0 && x != 1u) p[0] += 1;
  else if (x == 1u) p[1] = (int)x;
}
template <int K>
static void launch_one(int which, int *p, hipStream_t s) {
  if (which == K) hipLaunchKernelGGL(many_kernel<K>, dim3(1), dim3(64), 0, s, p);
  if constexpr (K + 1 < 256) launch_one<K + 1>(which, p, s);
}
void launch_b(int which, int *p, hipStream_t s) { launch_one<0>(which, p, s); }
