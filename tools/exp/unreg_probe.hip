// unreg_probe -- does hipHostRegister / hipHostUnregister wait for device
// work that does not touch the registered memory?  (tools only; the MAP read
// path of the pipeline unregisters each batch's mapping at slot reuse.)
// A 4 GiB H2D from a pinned buffer is put on a stream (~70 ms), then a
// registration / unregistration of an unrelated 64 MiB range is timed while
// it runs.  One JSON line per case.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

static double now() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}
#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                           \
    }                                                                                    \
  } while (0)

int main() {
  const size_t big = 4ull << 30, small = 64u << 20;
  CK(hipSetDevice(0));
  void *hbig, *dbig;
  CK(hipHostMalloc(&hbig, big, hipHostMallocDefault));
  CK(hipMalloc(&dbig, big));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  char *a = (char *)mmap(nullptr, small, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
  memset(a, 1, small);
  for (unsigned fl : {0u, (unsigned)hipHostRegisterReadOnly}) {
    for (int rep = 0; rep < 3; rep++) {
      // idle device
      double t0 = now();
      CK(hipHostRegister(a, small, fl));
      double t1 = now();
      CK(hipHostUnregister(a));
      double t2 = now();
      // busy device: a long copy in flight
      CK(hipMemcpyAsync(dbig, hbig, big, hipMemcpyHostToDevice, s));
      double t3 = now();
      CK(hipHostRegister(a, small, fl));
      double t4 = now();
      hipError_t q1 = hipStreamQuery(s);
      double t5 = now();
      CK(hipHostUnregister(a));
      double t6 = now();
      hipError_t q2 = hipStreamQuery(s);
      CK(hipStreamSynchronize(s));
      double t7 = now();
      printf("{\"flags\":%u,\"rep\":%d,\"idle_reg_ms\":%.3f,\"idle_unreg_ms\":%.3f,\"busy_reg_ms\":%.3f,"
             "\"copy_pending_after_reg\":%d,\"busy_unreg_ms\":%.3f,\"copy_pending_after_unreg\":%d,"
             "\"copy_ms\":%.3f}\n",
             fl, rep, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t4 - t3) * 1e3, q1 == hipErrorNotReady, (t6 - t5) * 1e3,
             q2 == hipErrorNotReady, (t7 - t3) * 1e3);
      fflush(stdout);
    }
  }
  return 0;
}
