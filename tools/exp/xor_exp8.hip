// xor_exp8.hip -- r05: the stream kernel's STORE (and load) cache policy
// through the compiler's buffer intrinsics, which carry the cache bits in
// their aux operand and whose data hazards the compiler tracks.  (NOT product
// code; tools only.)  r04's exp7 could write sc1 / sc0 sc1 / nt sc1 stores
// only as inline assembly, and those variants wrote wrong bytes (the store
// read its data registers after hipcc had reused them), so their times were
// no evidence.  Same schedule and tile body as the
// shipped xor_stream_w<8,8,0,full,6>; each wave stores its 8 KiB run of the
// tile through a buffer descriptor built from wave-uniform values
// (cdna_hip_programming.md T8), aux = the gfx950 cache-policy bits
// (sc0 = 1, nt = 2, sc1 = 16).  Every variant's output is compared with the
// shipped kernel's byte for byte.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ibeegfs-chunk-parity_amd/csrc -Iinclude \
//         tools/exp/xor_exp8.hip -o tools/exp/xor_exp8
//   ./tools/exp/xor_exp8 [stripes] [rounds] > policy.jsonl
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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(uint64_t base, uint32_t bytes) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  void *p = (void *)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// LDA: 0 = global nt loads (shipped), else buffer loads with aux = LDA - 1
// STA: buffer stores with aux = STA (0 plain, 2 nt, 16 sc1, 17 sc0 sc1, 18 nt sc1, 3 sc0 nt)
template <int LDA, int STA>
__device__ __forceinline__ void tile(const StreamArgs &a, uint32_t t) {
  constexpr int U = 8, NSRC = 8;
  const uint32_t s = t / a.tps;
  const uint32_t tin = t - s * a.tps;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  const uint64_t sb = (uint64_t)(uintptr_t)a.src + (uint64_t)s * a.stripe_stride;
  const uint64_t run = ((uint64_t)tin * (256u * U) + (uint64_t)wave * (64u * U)) * 16u;  // this wave's run
  v4u x[NSRC][U];
#pragma unroll
  for (int k = 0; k < NSRC; k++) {
    if constexpr (LDA == 0) {
      const glob<v4u> *pk = gp<v4u>(sb + (uint64_t)k * a.src_stride + run) + lane;
#pragma unroll
      for (int u = 0; u < U; u++) x[k][u] = __builtin_nontemporal_load(pk + u * 64);
    } else {
      const __amdgpu_buffer_rsrc_t r = wave_rsrc(sb + (uint64_t)k * a.src_stride + run, 64u * U * 16u);
#pragma unroll
      for (int u = 0; u < U; u++) {
        auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (u * 64 + lane) * 16, 0, LDA - 1);
        x[k][u] = v4u{v[0], v[1], v[2], v[3]};
      }
    }
  }
  v4u acc[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    acc[u] = x[0][u];
#pragma unroll
    for (int k = 1; k < NSRC; k++) acc[u] ^= x[k][u];
  }
  const __amdgpu_buffer_rsrc_t w = wave_rsrc((uint64_t)(uintptr_t)a.dst + (uint64_t)s * a.dst_stride + run,
                                             64u * U * 16u);
#pragma unroll
  for (int u = 0; u < U; u++) {
    __attribute__((ext_vector_type(4))) unsigned int v = {acc[u][0], acc[u][1], acc[u][2], acc[u][3]};
    __builtin_amdgcn_raw_buffer_store_b128(v, w, (u * 64 + lane) * 16, 0, STA);
  }
}

template <int LDA, int STA>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6, 6))) void xs_buf(StreamArgs a) {
  __shared__ uint32_t next[2];
  if (threadIdx.x == 0) next[0] = queue_grab(a.ctr, a.base);
  __syncthreads();
  uint32_t t = __builtin_amdgcn_readfirstlane(next[0]);
  int slot = 0;
  while (t < a.ntiles) {
    tile<LDA, STA>(a, t);
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
    {"shipped xor_stream_w<8,8,0,full,6> (global ld nt, st nt)", bcp::xor_stream_w<8, 8, 0, bcp::kQueueFull, 6>},
    {"ld global nt, st buffer nt", bcp::xs_buf<0, 2>},
    {"ld global nt, st buffer plain", bcp::xs_buf<0, 0>},
    {"ld global nt, st buffer sc1", bcp::xs_buf<0, 16>},
    {"ld global nt, st buffer sc0 sc1", bcp::xs_buf<0, 17>},
    {"ld global nt, st buffer nt sc1", bcp::xs_buf<0, 18>},
    {"ld global nt, st buffer sc0 nt", bcp::xs_buf<0, 3>},
    {"ld buffer nt, st buffer nt", bcp::xs_buf<3, 2>},
    {"ld buffer sc1, st buffer nt", bcp::xs_buf<17, 2>},
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
        CK(hipMemsetAsync(dcount, 0, 8, st));
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
