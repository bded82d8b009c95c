// unreg_thread_probe -- while one thread sits in hipHostUnregister (which
// waits for the device's outstanding work), can another thread keep
// submitting?  (tools only; decides whether the pipeline's MAP ranges can be
// released by a helper thread during a run.)
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

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

static char *g_a;
static const size_t kSmall = 64u << 20;
static double g_unreg_ms;
static void *unreg(void *) {
  double t0 = now();
  CK(hipHostUnregister(g_a));
  g_unreg_ms = (now() - t0) * 1e3;
  return nullptr;
}

int main() {
  const size_t big = 4ull << 30;
  CK(hipSetDevice(0));
  void *hbig, *dbig, *hs, *ds;
  CK(hipHostMalloc(&hbig, big, hipHostMallocDefault));
  CK(hipMalloc(&dbig, big));
  CK(hipHostMalloc(&hs, 1 << 20, hipHostMallocDefault));
  CK(hipMalloc(&ds, 1 << 20));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  g_a = (char *)mmap(nullptr, kSmall, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
  memset(g_a, 1, kSmall);
  char *b = (char *)mmap(nullptr, kSmall, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
  memset(b, 2, kSmall);
  for (int rep = 0; rep < 3; rep++) {
    CK(hipHostRegister(g_a, kSmall, hipHostRegisterReadOnly));
    CK(hipMemcpyAsync(dbig, hbig, big, hipMemcpyHostToDevice, s1));  // ~75 ms
    const double t0 = now();
    pthread_t th;
    pthread_create(&th, nullptr, unreg, nullptr);
    usleep(5000);  // the helper is inside hipHostUnregister now
    // the main thread keeps working: a small copy on another stream, a register, a sync of that stream
    const double t1 = now();
    CK(hipMemcpyAsync(ds, hs, 1 << 20, hipMemcpyHostToDevice, s2));
    const double t2 = now();
    CK(hipHostRegister(b, kSmall, hipHostRegisterReadOnly));
    const double t3 = now();
    CK(hipStreamSynchronize(s2));
    const double t4 = now();
    pthread_join(th, nullptr);
    const double t5 = now();
    CK(hipStreamSynchronize(s1));
    CK(hipHostUnregister(b));
    printf("{\"rep\":%d,\"main_copy_submit_ms\":%.3f,\"main_register_ms\":%.3f,\"main_sync_small_ms\":%.3f,"
           "\"helper_unreg_ms\":%.3f,\"join_at_ms\":%.3f}\n",
           rep, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3, g_unreg_ms, (t5 - t0) * 1e3);
    fflush(stdout);
  }
  // and munmap cost of populated file-like mappings, for scale: 2 GiB anonymous
  const size_t big2 = 2ull << 30;
  char *c = (char *)mmap(nullptr, big2, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
  double t0 = now();
  CK(hipHostRegister(c, big2, hipHostRegisterReadOnly));
  double t1 = now();
  CK(hipHostUnregister(c));
  double t2 = now();
  munmap(c, big2);
  double t3 = now();
  printf("{\"bytes\":%zu,\"register_ms\":%.3f,\"unregister_idle_ms\":%.3f,\"munmap_ms\":%.3f}\n", big2,
         (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3);
  return 0;
}
