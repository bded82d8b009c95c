// xor_exp6.hip -- narrow stripes (3-4 sources): why do they stream below
// both the copy (N = 1: 85.6 %) and the 8-wide fold (88.4 %)?  (NOT product
// code; tools only.)  profiles/r02/desc/mix_ceiling_r2c1.jsonl: N = 3 84.4 %,
// N = 4 83.8 %; the descriptor kernel on config-5 shapes (~3.3 bytes read
// per byte written) sits at the same rate.  The shipped narrow schedule takes
// two consecutive tiles per queue grab and folds them one after the other:
// the compiler cannot move tile x+1's loads above tile x's stores (it cannot
// rule out aliasing), so every grab drains the lane's loads twice.  Variants:
//
//   shipped   xor_stream<N,8,0,full>, grab 2 (the product kernel)
//   grab1     the same kernel, one tile per grab
//   fused     grab 2, both tiles' loads first, then the XORs and both stores
//             (one drain per grab), compiler's register target / budgets
//   restrict  grab 2, tile after tile, but sources and output __restrict__
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ibeegfs-chunk-parity_amd/csrc -Iinclude \
//         tools/exp/xor_exp6.hip -o tools/exp/xor_exp6
//   ./tools/exp/xor_exp6 [input GiB] [reps] > sweep.jsonl
#include "bcp_kernels.hip"

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__);      \
      exit(2);                                                                                 \
    }                                                                                          \
  } while (0)

namespace bcp {

// G consecutive tiles of one grab, every load first (tiles never straddle a
// stripe: tps is a multiple of G here).
template <int N, int U, int G>
__device__ __forceinline__ void fused_tiles(const StreamArgs &a, uint32_t t0) {
  const uint32_t s = t0 / a.tps;
  const uint32_t tin = t0 - s * a.tps;
  const uint64_t sb = (uint64_t)(uintptr_t)a.src + (uint64_t)s * a.stripe_stride;
  glob<v4u> *db = gp<v4u>((uint64_t)(uintptr_t)a.dst + (uint64_t)s * a.dst_stride);
  v4u x[G][N][U];
#pragma unroll
  for (int g = 0; g < G; g++)
#pragma unroll
    for (int k = 0; k < N; k++) {
      const glob<v4u> *pk = gp<v4u>(sb + (uint64_t)k * a.src_stride) + tile_vec<U>(tin + g, 0);
#pragma unroll
      for (int u = 0; u < U; u++) x[g][k][u] = ld_nt(pk + u * 64);
    }
#pragma unroll
  for (int g = 0; g < G; g++)
#pragma unroll
    for (int u = 0; u < U; u++) {
      v4u acc = x[g][0][u];
#pragma unroll
      for (int k = 1; k < N; k++) acc ^= x[g][k][u];
      __builtin_nontemporal_store(acc, db + tile_vec<U>(tin + g, u));
    }
}

template <int N, int U>
__device__ __forceinline__ void restrict_tile(const v4u *__restrict__ s0, const v4u *__restrict__ s1,
                                              const v4u *__restrict__ s2, const v4u *__restrict__ s3,
                                              v4u *__restrict__ d, uint32_t vb) {
  v4u x[N][U];
  const v4u *__restrict__ sp[4] = {s0, s1, s2, s3};
#pragma unroll
  for (int k = 0; k < N; k++)
#pragma unroll
    for (int u = 0; u < U; u++) x[k][u] = __builtin_nontemporal_load(sp[k] + vb + u * 64);
#pragma unroll
  for (int u = 0; u < U; u++) {
    v4u acc = x[0][u];
#pragma unroll
    for (int k = 1; k < N; k++) acc ^= x[k][u];
    __builtin_nontemporal_store(acc, d + vb + u * 64);
  }
}

template <int N, int U, int G, int MODE>
__device__ __forceinline__ void narrow_loop(const StreamArgs &a) {
  __shared__ uint32_t next[2];
  if (threadIdx.x == 0) next[0] = queue_grab(a.ctr, a.base);
  __syncthreads();
  uint32_t c = __builtin_amdgcn_readfirstlane(next[0]);
  int slot = 0;
  const uint32_t nunits = a.ntiles / G;
  while (c < nunits) {
    if constexpr (MODE == 0) {
      fused_tiles<N, U, G>(a, c * G);
    } else {
      const uint32_t t0 = c * G;
      const uint32_t s = t0 / a.tps;
      const char *sb = a.src + (uint64_t)s * a.stripe_stride;
      const v4u *s0 = (const v4u *)sb;
      const v4u *s1 = (const v4u *)(sb + a.src_stride);
      const v4u *s2 = (const v4u *)(sb + 2 * a.src_stride);
      const v4u *s3 = (const v4u *)(sb + 3 * a.src_stride);
      v4u *d = (v4u *)(a.dst + (uint64_t)s * a.dst_stride);
#pragma unroll
      for (int g = 0; g < G; g++) restrict_tile<N, U>(s0, s1, s2, s3, d, tile_vec<U>(t0 - s * a.tps + g, 0));
    }
    slot ^= 1;
    if (threadIdx.x == 0) next[slot] = queue_grab(a.ctr, a.base);
    __syncthreads();
    c = __builtin_amdgcn_readfirstlane(next[slot]);
  }
}

template <int N, int U, int G, int MODE>
__global__ __launch_bounds__(kBlock) void xn(StreamArgs a) {
  narrow_loop<N, U, G, MODE>(a);
}
template <int N, int U, int G, int MODE, int W>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W, W))) void xn_w(StreamArgs a) {
  narrow_loop<N, U, G, MODE>(a);
}

}  // namespace bcp

typedef void (*KFn)(bcp::StreamArgs);
struct Entry {
  const char *name;
  int n;
  KFn fn;
  int grab;  // StreamArgs.grab for the product kernel; units of the fused forms
};

static const Entry kV[] = {
    {"shipped grab2", 3, bcp::xor_stream<3, 8, 0, bcp::kQueueFull>, 2},
    {"grab1", 3, bcp::xor_stream<3, 8, 0, bcp::kQueueFull>, 1},
    {"fused2", 3, bcp::xn<3, 8, 2, 0>, 2},
    {"fused2 wpe4", 3, bcp::xn_w<3, 8, 2, 0, 4>, 2},
    {"fused2 wpe2", 3, bcp::xn_w<3, 8, 2, 0, 2>, 2},
    {"restrict2", 3, bcp::xn<3, 8, 2, 1>, 2},
    {"restrict2 wpe4", 3, bcp::xn_w<3, 8, 2, 1, 4>, 2},
    {"shipped grab2", 4, bcp::xor_stream<4, 8, 0, bcp::kQueueFull>, 2},
    {"grab1", 4, bcp::xor_stream<4, 8, 0, bcp::kQueueFull>, 1},
    {"fused2", 4, bcp::xn<4, 8, 2, 0>, 2},
    {"fused2 wpe4", 4, bcp::xn_w<4, 8, 2, 0, 4>, 2},
    {"fused2 wpe2", 4, bcp::xn_w<4, 8, 2, 0, 2>, 2},
    {"restrict2", 4, bcp::xn<4, 8, 2, 1>, 2},
    {"restrict2 wpe4", 4, bcp::xn_w<4, 8, 2, 1, 4>, 2},
};

int main(int argc, char **argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 24.0;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const uint64_t S = 512 * 1024;
  const uint64_t in_max = (uint64_t)(gib * (1ull << 30)) / (12 * S) * (12 * S);  // divisible by 3 and 4 rows
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount * 29 / 32;  // the product's streaming grid
  char *src, *dst, *ref3, *ref4;
  unsigned long long *ctr, *dcount;
  CK(hipMalloc(&src, in_max));
  CK(hipMalloc(&dst, in_max / 3));
  CK(hipMalloc(&ref3, in_max / 3));
  CK(hipMalloc(&ref4, in_max / 4));
  CK(hipMalloc(&ctr, 256));
  CK(hipMalloc(&dcount, 8));
  CK(hipMemset(ctr, 0, 256));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(bcp::launch_fill_synthetic(st, prop.multiProcessorCount * 8, src, in_max, 1ull, 0));
  unsigned long long base = 0;
  const int nv = sizeof(kV) / sizeof(kV[0]);
  auto launch = [&](int v, char *out) {
    const uint64_t N = (uint64_t)kV[v].n, stripes = in_max / (N * S);
    bcp::StreamArgs a{};
    a.dst = out;
    a.dst_stride = S;
    a.src = src;
    a.stripe_stride = N * S;
    a.src_stride = S;
    a.vps = (uint32_t)(S / 16);
    a.tps = (uint32_t)(S / 16 / (256 * 8));
    a.ntiles = (uint32_t)(stripes * a.tps);
    a.nsrc = (uint32_t)N;
    a.grab = (uint32_t)kV[v].grab;
    a.ctr = ctr;
    a.base = base;
    hipLaunchKernelGGL(kV[v].fn, dim3(grid), dim3(256), 0, st, a);
    CK(hipGetLastError());
    base += (a.ntiles + a.grab - 1) / a.grab + grid;  // successful grabs + one failing grab per workgroup
  };
  // references: the shipped kernel of each width
  launch(0, ref3);
  launch(7, ref4);
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> times(nv);
  std::vector<long long> bad(nv, -1);
  for (int r = 0; r < reps; r++) {
    for (int v = 0; v < nv; v++) {
      const uint64_t out_bytes = in_max / kV[v].n;
      if (r == 0) {
        CK(hipMemsetAsync(dst, 0, out_bytes, st));
        launch(v, dst);
        CK(hipMemsetAsync(dcount, 0, 8, st));
        CK(bcp::launch_compare(st, grid, dst, kV[v].n == 3 ? ref3 : ref4, out_bytes, dcount));
        unsigned long long h;
        CK(hipMemcpyAsync(&h, dcount, 8, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        bad[v] = (long long)h;
      }
      launch(v, dst);  // one launch queued ahead of the first event
      CK(hipEventRecord(e0, st));
      launch(v, dst);
      launch(v, dst);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      times[v].push_back(ms / 2);
    }
    fprintf(stderr, "rep %d/%d done\n", r + 1, reps);
  }
  for (int v = 0; v < nv; v++) {
    auto ts = times[v];
    std::sort(ts.begin(), ts.end());
    const float med = ts[ts.size() / 2];
    const double bytes = (double)in_max + (double)(in_max / kV[v].n);
    printf("{\"nsrc\": %d, \"variant\": \"%s\", \"median_ms\": %.4f, \"min_ms\": %.4f, \"GBps\": %.1f, "
           "\"frac_8TBs\": %.4f, \"mismatch_bytes\": %lld}\n",
           kV[v].n, kV[v].name, med, ts[0], bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12, bad[v]);
  }
  return 0;
}
