// reg_probe -- what it costs to let the DMA engine read chunk files straight
// out of the page cache (tools only; DESIGN.md 6.7 / VERDICT r03 next #3).
//
// F files of S bytes in a tmpfs directory, three ways to move them to HBM:
//   read    : 8 threads pread() into a pinned slab, then one H2D
//   perfile : mmap each file, hipHostRegister it, one H2D per file, unregister
//   region  : mmap every file MAP_FIXED into one reserved range, register the
//             range once, one H2D, unregister
// Prints one JSON line per variant (wall seconds of register / copy / total).
// argv[4] = N: N host threads memcpy 64 MiB buffers in a loop meanwhile
// (contention for host memory bandwidth, as 8 GPUs' pipelines on one host).
#include <hip/hip_runtime.h>

#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <vector>

static double now() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                   \
    }                                                                            \
  } while (0)

static const char *g_dir;
static size_t g_S;
static int g_F;
static unsigned char *g_slab;

static volatile int g_stop;
static void *contender(void *) {
  const size_t n = 64u << 20;
  char *a = (char *)malloc(n), *b = (char *)malloc(n);
  memset(a, 1, n);
  memset(b, 2, n);
  while (!g_stop) memcpy(a, b, n);
  free(a);
  free(b);
  return nullptr;
}

static void fname(char *b, size_t cap, int i) { snprintf(b, cap, "%s/c%05d", g_dir, i); }

struct RA {
  int t, nt;
};
static void *reader(void *p) {
  RA *a = (RA *)p;
  char fn[512];
  for (int i = a->t; i < g_F; i += a->nt) {
    fname(fn, sizeof fn, i);
    int fd = open(fn, O_RDONLY);
    size_t got = 0;
    while (got < g_S) {
      ssize_t r = pread(fd, g_slab + (size_t)i * g_S + got, g_S - got, got);
      if (r <= 0) break;
      got += r;
    }
    close(fd);
  }
  return nullptr;
}

struct PF {
  int t, nt;
  unsigned flags;
  void *dev;
  double reg, unreg;
  int fails;
};
static void *perfile(void *p) {
  PF *a = (PF *)p;
  char fn[512];
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int i = a->t; i < g_F; i += a->nt) {
    fname(fn, sizeof fn, i);
    int fd = open(fn, O_RDONLY);
    void *m = mmap(nullptr, g_S, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
    close(fd);
    double t0 = now();
    hipError_t e = hipHostRegister(m, g_S, a->flags);
    a->reg += now() - t0;
    if (e != hipSuccess) {
      (void)hipGetLastError();
      a->fails++;
      munmap(m, g_S);
      continue;
    }
    CK(hipMemcpyAsync((char *)a->dev + (size_t)i * g_S, m, g_S, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    t0 = now();
    CK(hipHostUnregister(m));
    a->unreg += now() - t0;
    munmap(m, g_S);
  }
  CK(hipStreamDestroy(s));
  return nullptr;
}

static int check(void *dev, const unsigned char *want, int i) {
  std::vector<unsigned char> got(g_S);
  CK(hipMemcpy(got.data(), (char *)dev + (size_t)i * g_S, g_S, hipMemcpyDeviceToHost));
  return memcmp(got.data(), want, g_S) == 0;
}

int main(int argc, char **argv) {
  g_dir = argc > 1 ? argv[1] : "/dev/shm/bcp_reg_probe";
  g_F = argc > 2 ? atoi(argv[2]) : 512;
  g_S = argc > 3 ? strtoull(argv[3], nullptr, 0) : (512u << 10);
  const int reps = 3;
  const int ncont = argc > 4 ? atoi(argv[4]) : 0;
  std::vector<pthread_t> cth(ncont);
  const size_t total = (size_t)g_F * g_S;
  mkdir(g_dir, 0700);
  std::vector<unsigned char> buf(g_S);
  char fn[512];
  std::vector<unsigned char> first(g_S);
  for (int i = 0; i < g_F; i++) {
    for (size_t j = 0; j < g_S; j += 8) {
      unsigned long long x = (unsigned long long)i * 0x9E3779B97F4A7C15ull + j * 0xBF58476D1CE4E5B9ull;
      x ^= x >> 31;
      memcpy(&buf[j], &x, 8);
    }
    if (i == g_F / 2) first = buf;
    fname(fn, sizeof fn, i);
    int fd = open(fn, O_CREAT | O_TRUNC | O_WRONLY, 0600);
    if (write(fd, buf.data(), g_S) != (ssize_t)g_S) return 3;
    close(fd);
  }
  CK(hipSetDevice(0));
  for (int i = 0; i < ncont; i++) pthread_create(&cth[i], nullptr, contender, nullptr);
  printf("{\"contending_threads\":%d}\n", ncont);
  void *dev;
  CK(hipMalloc(&dev, total));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

  // ---- read() into a pinned slab
  CK(hipHostMalloc((void **)&g_slab, total, hipHostMallocDefault));
  for (int r = 0; r < reps; r++) {
    double t0 = now();
    pthread_t th[8];
    RA ra[8];
    for (int t = 0; t < 8; t++) {
      ra[t] = {t, 8};
      pthread_create(&th[t], nullptr, reader, &ra[t]);
    }
    for (int t = 0; t < 8; t++) pthread_join(th[t], nullptr);
    double t1 = now();
    CK(hipMemcpyAsync(dev, g_slab, total, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    double t2 = now();
    printf("{\"variant\":\"read8+h2d\",\"files\":%d,\"file_bytes\":%zu,\"read_s\":%.5f,\"h2d_s\":%.5f,"
           "\"h2d_GBps\":%.2f,\"total_GBps\":%.2f,\"ok\":%d}\n",
           g_F, g_S, t1 - t0, t2 - t1, total / (t2 - t1) / 1e9, total / (t2 - t0) / 1e9,
           check(dev, first.data(), g_F / 2));
    fflush(stdout);
  }
  CK(hipHostFree(g_slab));

  // ---- per-file register
  const unsigned flagsets[2] = {hipHostRegisterReadOnly, hipHostRegisterDefault};
  for (unsigned fl : flagsets) {
    for (int nt : {1, 8}) {
      CK(hipMemset(dev, 0, total));
      double t0 = now();
      pthread_t th[8];
      PF pf[8];
      for (int t = 0; t < nt; t++) {
        pf[t] = {t, nt, fl, dev, 0, 0, 0};
        pthread_create(&th[t], nullptr, perfile, &pf[t]);
      }
      double reg = 0, unreg = 0;
      int fails = 0;
      for (int t = 0; t < nt; t++) {
        pthread_join(th[t], nullptr);
        reg += pf[t].reg;
        unreg += pf[t].unreg;
        fails += pf[t].fails;
      }
      double t1 = now();
      printf("{\"variant\":\"perfile_register\",\"flags\":%u,\"threads\":%d,\"files\":%d,\"reg_s_sum\":%.5f,"
             "\"reg_us_per_file\":%.1f,\"unreg_us_per_file\":%.1f,\"wall_s\":%.5f,\"total_GBps\":%.2f,"
             "\"fails\":%d,\"ok\":%d}\n",
             fl, nt, g_F, reg, reg / g_F * 1e6, unreg / g_F * 1e6, t1 - t0, total / (t1 - t0) / 1e9, fails,
             fails ? -1 : check(dev, first.data(), g_F / 2));
      fflush(stdout);
    }
  }

  // ---- one region of MAP_FIXED file mappings, registered once (populated
  // by mmap, or -- pop 0 -- faulted in by the registration itself)
  for (int pop : {1, 0})
  for (unsigned fl : flagsets) {
    for (int r = 0; r < reps; r++) {
      CK(hipMemset(dev, 0, total));
      double t0 = now();
      char *base = (char *)mmap(nullptr, total, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
      int mfail = 0;
      for (int i = 0; i < g_F; i++) {
        fname(fn, sizeof fn, i);
        int fd = open(fn, O_RDONLY);
        void *m = mmap(base + (size_t)i * g_S, g_S, PROT_READ, MAP_SHARED | MAP_FIXED | (pop ? MAP_POPULATE : 0), fd, 0);
        close(fd);
        if (m == MAP_FAILED) mfail++;
      }
      double t1 = now();
      hipError_t e = hipHostRegister(base, total, fl);
      double t2 = now();
      double t3 = t2, t4 = t2;
      int ok = -1;
      if (e == hipSuccess) {
        CK(hipMemcpyAsync(dev, base, total, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        t3 = now();
        CK(hipHostUnregister(base));
        t4 = now();
        ok = check(dev, first.data(), g_F / 2);
      } else {
        fprintf(stderr, "region register flags %u: %s\n", fl, hipGetErrorString(e));
        (void)hipGetLastError();
      }
      munmap(base, total);
      double t5 = now();
      printf("{\"variant\":\"region_register\",\"populate\":%d,\"flags\":%u,\"files\":%d,\"mmap_s\":%.5f,\"reg_s\":%.5f,"
             "\"h2d_s\":%.5f,\"h2d_GBps\":%.2f,\"unreg_s\":%.5f,\"munmap_s\":%.5f,\"total_GBps\":%.2f,"
             "\"map_fail\":%d,\"reg_rc\":%d,\"ok\":%d}\n",
             pop, fl, g_F, t1 - t0, t2 - t1, t3 - t2, e == hipSuccess ? total / (t3 - t2) / 1e9 : 0.0, t4 - t3, t5 - t4,
             e == hipSuccess ? total / (t5 - t0) / 1e9 : 0.0, mfail, (int)e, ok);
      fflush(stdout);
    }
  }
  g_stop = 1;
  for (int i = 0; i < ncont; i++) pthread_join(cth[i], nullptr);
  CK(hipFree(dev));
  for (int i = 0; i < g_F; i++) {
    fname(fn, sizeof fn, i);
    unlink(fn);
  }
  rmdir(g_dir);
  return 0;
}
