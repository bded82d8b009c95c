// Reads of pinned HOST memory by a kernel, by how the memory was pinned
// (r05, tools/exp/zero_copy_probe.py: the protocol's in-place fold reads host
// rows at 45-48 GB/s, a large hipMemcpyAsync moves 57 GB/s).  One launch
// XORs 3 host arrays of `mb` MiB into a 4th (the fold's access pattern:
// 16-byte vectors, a 256-thread workgroup per CU striding over the arrays),
// timed with events, for each allocation kind and load kind:
//   coherent     hipHostMalloc(default)             (fine-grained)
//   noncoherent  hipHostMalloc(hipHostMallocNonCoherent)
//   registered   malloc'd pages + hipHostRegister   (what bcp_host_alloc uses)
//   device       hipMalloc (HBM: the kernel's own ceiling)
// Output: one JSON line per (kind, load, grid).
//   hipcc --offload-arch=gfx950 -O3 -o tools/exp/zc_mtype tools/exp/zc_mtype.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int NT>
__global__ __launch_bounds__(256) void xor3(v4u *__restrict__ out, const v4u *__restrict__ a,
                                            const v4u *__restrict__ b, const v4u *__restrict__ c,
                                            size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    v4u x, y, z;
    if (NT) {
      x = __builtin_nontemporal_load(a + i);
      y = __builtin_nontemporal_load(b + i);
      z = __builtin_nontemporal_load(c + i);
      __builtin_nontemporal_store(x ^ y ^ z, out + i);
    } else {
      x = a[i];
      y = b[i];
      z = c[i];
      out[i] = x ^ y ^ z;
    }
  }
}

static void *alloc(const char *kind, size_t n) {
  void *p = nullptr;
  if (!strcmp(kind, "coherent")) CK(hipHostMalloc(&p, n, hipHostMallocDefault));
  else if (!strcmp(kind, "noncoherent")) CK(hipHostMalloc(&p, n, hipHostMallocNonCoherent));
  else if (!strcmp(kind, "registered")) {
    p = aligned_alloc(2 << 20, n);
    memset(p, 1, n);
    CK(hipHostRegister(p, n, hipHostRegisterDefault));
  } else CK(hipMalloc(&p, n));
  return p;
}

static void release(const char *kind, void *p) {
  if (!strcmp(kind, "coherent") || !strcmp(kind, "noncoherent")) CK(hipHostFree(p));
  else if (!strcmp(kind, "registered")) {
    CK(hipHostUnregister(p));
    free(p);
  } else CK(hipFree(p));
}

int main(int argc, char **argv) {
  const size_t mb = argc > 1 ? strtoull(argv[1], nullptr, 10) : 256;
  const size_t bytes = mb << 20, n = bytes / 16;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const char *kinds[] = {"coherent", "noncoherent", "registered", "device"};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const char *kind : kinds) {
    v4u *src[3], *out;
    for (auto &s : src) {
      s = (v4u *)alloc(kind, bytes);
      CK(hipMemset(s, 0x5a, bytes));
    }
    out = (v4u *)alloc(kind, bytes);
    CK(hipDeviceSynchronize());
    for (int nt = 0; nt < 2; nt++)
      for (int gmul : {1, 4, 16}) {
        const int grid = cus * gmul;
        float best = 1e30f;
        for (int rep = 0; rep < 4; rep++) {
          CK(hipEventRecord(e0));
          if (nt) xor3<1><<<grid, 256>>>(out, src[0], src[1], src[2], n);
          else xor3<0><<<grid, 256>>>(out, src[0], src[1], src[2], n);
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (rep && ms < best) best = ms;
        }
        printf("{\"kind\": \"%s\", \"nt\": %d, \"grid\": %d, \"MiB_per_array\": %zu, \"ms\": %.3f, "
               "\"read_GBps\": %.2f, \"write_GBps\": %.2f}\n",
               kind, nt, grid, mb, best, 3.0 * bytes / best / 1e6, 1.0 * bytes / best / 1e6);
        fflush(stdout);
      }
    for (auto &s : src) release(kind, s);
    release(kind, out);
  }
  return 0;
}
