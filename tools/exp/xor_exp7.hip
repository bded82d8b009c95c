// xor_exp7.hip -- cache policy of the stream kernel's loads and stores under
// the SHIPPED schedule (work queue, U = 8, waves_per_eu 6).  (NOT product code;
// tools only.)  r01 compared store hints only under the static schedule it
// later dropped (exp 1, 67-71 % for every hint); the queue kernel always used
// nt loads + nt stores.  The guide (MI355X_MICROARCH.md, stores of each
// flavour): plain / nt stores keep the line in the XCD's L2, sc1 / sc0 sc1
// drop it; nt / sc1 loads bypass L1.  Variants, same tile body otherwise:
//   LD 0 nt, 1 plain;  ST 0 nt, 1 plain, 2 sc1, 3 sc0 sc1, 4 nt sc1
// (ST >= 2 through inline `global_store_dwordx4 ... off <bits>`, vector stores.
// Measured r4af: those three wrote WRONG bytes -- the compiler does not track
// the store-data hazard of an inline-asm store, so a following VALU may
// overwrite the data VGPRs before the store reads them; their times are not
// evidence.  The compiler-generated variants (nt / plain) are exact.)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ibeegfs-chunk-parity_amd/csrc -Iinclude \
//         tools/exp/xor_exp7.hip -o tools/exp/xor_exp7
//   ./tools/exp/xor_exp7 [stripes] [rounds] > policy.jsonl
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

template <int LD>
__device__ __forceinline__ v4u ld_p(const glob<v4u> *p) {
  if constexpr (LD == 0) return __builtin_nontemporal_load(p);
  else return *p;
}

template <int ST>
__device__ __forceinline__ void st_p(v4u v, glob<v4u> *p) {
  if constexpr (ST == 0) {
    __builtin_nontemporal_store(v, p);
  } else if constexpr (ST == 1) {
    *p = v;
  } else if constexpr (ST == 2) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  } else if constexpr (ST == 3) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  } else {
    asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
  }
}

// stream_tile<8, 8, 0, false>'s full-tile path with the policies as parameters
template <int LD, int ST>
__device__ __forceinline__ void tile(const StreamArgs &a, uint32_t t) {
  constexpr int U = 8, NSRC = 8;
  const uint32_t s = t / a.tps;
  const uint32_t tin = t - s * a.tps;
  const uint64_t sb = (uint64_t)(uintptr_t)a.src + (uint64_t)s * a.stripe_stride;
  glob<v4u> *db = gp<v4u>((uint64_t)(uintptr_t)a.dst + (uint64_t)s * a.dst_stride);
  const uint32_t vb = tile_vec<U>(tin, 0);
  v4u x[NSRC][U];
#pragma unroll
  for (int k = 0; k < NSRC; k++) {
    const glob<v4u> *pk = gp<v4u>(sb + (uint64_t)k * a.src_stride) + vb;
#pragma unroll
    for (int u = 0; u < U; u++) x[k][u] = ld_p<LD>(pk + u * 64);
  }
  v4u acc[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    acc[u] = x[0][u];
#pragma unroll
    for (int k = 1; k < NSRC; k++) acc[u] ^= x[k][u];
  }
#pragma unroll
  for (int u = 0; u < U; u++) st_p<ST>(acc[u], db + vb + u * 64);
}

template <int LD, int ST>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6, 6))) void xs_pol(StreamArgs a) {
  __shared__ uint32_t next[2];
  if (threadIdx.x == 0) next[0] = queue_grab(a.ctr, a.base);
  __syncthreads();
  uint32_t t = __builtin_amdgcn_readfirstlane(next[0]);
  int slot = 0;
  while (t < a.ntiles) {
    tile<LD, ST>(a, t);
    slot ^= 1;
    if (threadIdx.x == 0) next[slot] = queue_grab(a.ctr, a.base);
    __syncthreads();
    t = __builtin_amdgcn_readfirstlane(next[slot]);
  }
}

}  // namespace bcp

typedef void (*KFn)(bcp::StreamArgs);
struct Entry {
  const char *name;
  KFn fn;
};

static const Entry kV[] = {
    {"shipped xor_stream_w<8,8,0,full,6> (ld nt, st nt)", bcp::xor_stream_w<8, 8, 0, bcp::kQueueFull, 6>},
    {"replica ld nt, st nt", bcp::xs_pol<0, 0>},
    {"ld nt, st plain", bcp::xs_pol<0, 1>},
    {"ld nt, st sc1", bcp::xs_pol<0, 2>},
    {"ld nt, st sc0 sc1", bcp::xs_pol<0, 3>},
    {"ld nt, st nt sc1", bcp::xs_pol<0, 4>},
    {"ld plain, st nt", bcp::xs_pol<1, 0>},
    {"ld plain, st plain", bcp::xs_pol<1, 1>},
};

int main(int argc, char **argv) {
  const uint64_t stripes = argc > 1 ? strtoull(argv[1], 0, 10) : 12500;
  const int rounds = argc > 2 ? atoi(argv[2]) : 6;
  const uint64_t S = 512 * 1024, N = 8;
  const uint64_t in_bytes = stripes * N * S, out_bytes = stripes * S;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount * 29 / 32;
  char *src, *dst, *ref;
  unsigned long long *ctr, *dcount;
  CK(hipMalloc(&src, in_bytes));
  CK(hipMalloc(&dst, out_bytes));
  CK(hipMalloc(&ref, out_bytes));
  CK(hipMalloc(&ctr, 256));
  CK(hipMalloc(&dcount, 8));
  CK(hipMemset(ctr, 0, 256));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(bcp::launch_fill_synthetic(st, prop.multiProcessorCount * 8, src, in_bytes, 1ull, 0));
  unsigned long long base = 0;
  const int nv = sizeof(kV) / sizeof(kV[0]);
  auto launch = [&](int v, char *out) {
    bcp::StreamArgs a{};
    a.dst = out;
    a.dst_stride = S;
    a.src = src;
    a.stripe_stride = N * S;
    a.src_stride = S;
    a.vps = (uint32_t)(S / 16);
    a.tps = (uint32_t)(S / 16 / (256 * 8));
    a.ntiles = (uint32_t)(stripes * a.tps);
    a.nsrc = N;
    a.ctr = ctr;
    a.base = base;
    hipLaunchKernelGGL(kV[v].fn, dim3(grid), dim3(256), 0, st, a);
    CK(hipGetLastError());
    base += a.ntiles + grid;
  };
  launch(0, ref);
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> times(nv);
  std::vector<long long> bad(nv, -1);
  for (int r = 0; r < rounds; r++) {
    for (int i = 0; i < nv; i++) {
      const int v = r % 2 ? nv - 1 - i : i;  // alternate the order round by round
      if (r == 0) {
        CK(hipMemsetAsync(dst, 0, out_bytes, st));
        CK(hipMemsetAsync(dcount, 0, 8, st));  // (launch_compare accumulates)
        launch(v, dst);
        CK(bcp::launch_compare(st, grid, dst, ref, out_bytes, dcount));
        unsigned long long h;
        CK(hipMemcpyAsync(&h, dcount, 8, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        bad[v] = (long long)h;
      }
      launch(v, dst);  // one launch queued ahead of the first event
      CK(hipEventRecord(e0, st));
      for (int k = 0; k < 4; k++) launch(v, dst);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      times[v].push_back(ms / 4);
    }
    fprintf(stderr, "round %d/%d done\n", r + 1, rounds);
  }
  for (int v = 0; v < nv; v++) {
    auto ts = times[v];
    std::sort(ts.begin(), ts.end());
    const float med = ts[ts.size() / 2];
    const double bytes = (double)(in_bytes + out_bytes);
    printf("{\"variant\": \"%s\", \"median_ms\": %.4f, \"min_ms\": %.4f, \"max_ms\": %.4f, \"frac_8TBs\": %.4f, "
           "\"mismatch_bytes\": %lld}\n",
           kV[v].name, med, ts[0], ts.back(), bytes / (med * 1e-3) / 8e12, bad[v]);
  }
  return 0;
}
