// xor_exp9.hip -- r05: the stream kernel's ADDRESS registers.  (NOT product
// code; tools only.)  The shipped xor_stream_w<8,8,0,full,6> addresses every
// load and store with a 64-bit VGPR pair (`global_load_dwordx4 v, v[a:a+1],
// off`): a pair per source plus pairs for the u >= 4 offsets the 13-bit
// immediate cannot reach, and under the waves_per_eu(6) budget of 80 VGPRs it
// spills 24 bytes per lane per tile (2 scratch stores + 3 reloads inside the
// tile loop).  Here each source's base is the stripe's uniform address
// (SGPRs) and the lane's offset inside the tile one 32-bit VGPR, written so
// the compiler can select the saddr form (`global_load_dwordx4 v, v_off,
// s[b:b+1] offset:imm`): sgpr base + zext(u32 offset).  Same schedule and
// tile body otherwise; waves-per-EU budgets W = 5..8 (the address registers
// it saves can hold more loads in flight, or more waves).  Every variant's
// output is compared with the shipped kernel's byte for byte.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ibeegfs-chunk-parity_amd/csrc -Iinclude \
//         tools/exp/xor_exp9.hip -o tools/exp/xor_exp9
//   ./tools/exp/xor_exp9 [stripes] [rounds] > addr.jsonl
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

// uniform byte base + zero-extended 32-bit lane offset
__device__ __forceinline__ const glob<v4u> *at(uint64_t base, uint32_t off) {
  return (const glob<v4u> *)((const glob<unsigned char> *)(uintptr_t)base + off);
}
__device__ __forceinline__ glob<v4u> *at_w(uint64_t base, uint32_t off) {
  return (glob<v4u> *)((glob<unsigned char> *)(uintptr_t)base + off);
}

template <int U>
__device__ __forceinline__ void tile_s(const StreamArgs &a, uint32_t t) {
  constexpr int NSRC = 8;
  const uint32_t s = t / a.tps;
  const uint32_t tin = t - s * a.tps;
  const uint64_t sb = (uint64_t)(uintptr_t)a.src + (uint64_t)s * a.stripe_stride;
  const uint64_t db = (uint64_t)(uintptr_t)a.dst + (uint64_t)s * a.dst_stride;
  const uint32_t off = tile_vec<U>(tin, 0) * 16u;  // this lane's first vector of the tile, bytes
  v4u x[NSRC][U];
#pragma unroll
  for (int k = 0; k < NSRC; k++) {
    const uint64_t bk = sb + (uint64_t)k * a.src_stride;
#pragma unroll
    for (int u = 0; u < U; u++) x[k][u] = __builtin_nontemporal_load(at(bk, off + u * 1024u));
  }
  v4u acc[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    acc[u] = x[0][u];
#pragma unroll
    for (int k = 1; k < NSRC; k++) acc[u] ^= x[k][u];
  }
#pragma unroll
  for (int u = 0; u < U; u++) __builtin_nontemporal_store(acc[u], at_w(db, off + u * 1024u));
}

template <int U, int W>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W, W))) void xs_saddr(StreamArgs a) {
  __shared__ uint32_t next[2];
  if (threadIdx.x == 0) next[0] = queue_grab(a.ctr, a.base);
  __syncthreads();
  uint32_t t = __builtin_amdgcn_readfirstlane(next[0]);
  int slot = 0;
  while (t < a.ntiles) {
    tile_s<U>(a, t);
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
  int U;
  int blocks_per_cu;
};

static const Entry kV[] = {
    {"shipped xor_stream_w<8,8,0,full,6> (64-bit VGPR addresses)", bcp::xor_stream_w<8, 8, 0, bcp::kQueueFull, 6>, 8, 1},
    {"saddr U8 W6", bcp::xs_saddr<8, 6>, 8, 1},
    {"saddr U8 W5", bcp::xs_saddr<8, 5>, 8, 1},
    {"saddr U8 W7", bcp::xs_saddr<8, 7>, 8, 1},
    {"saddr U8 W8", bcp::xs_saddr<8, 8>, 8, 1},
    {"saddr U8 W4", bcp::xs_saddr<8, 4>, 8, 1},
    {"saddr U8 W6, 2 WG/CU", bcp::xs_saddr<8, 6>, 8, 2},
};

int main(int argc, char **argv) {
  const uint64_t stripes = argc > 1 ? strtoull(argv[1], 0, 10) : 12500;
  const int rounds = argc > 2 ? atoi(argv[2]) : 6;
  const uint64_t S = 512 * 1024, N = 8;
  const uint64_t in_bytes = stripes * N * S, out_bytes = stripes * S;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
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
    const int grid = prop.multiProcessorCount * 29 / 32 * kV[v].blocks_per_cu;
    bcp::StreamArgs a{};
    a.dst = out;
    a.dst_stride = S;
    a.src = src;
    a.stripe_stride = N * S;
    a.src_stride = S;
    a.vps = (uint32_t)(S / 16);
    a.tps = (uint32_t)(S / 16 / (256 * kV[v].U));
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
        CK(hipMemsetAsync(dcount, 0, 8, st));
        launch(v, dst);
        CK(bcp::launch_compare(st, prop.multiProcessorCount, dst, ref, out_bytes, dcount));
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
