// xor_exp5.hip -- how many loads per wave should be in flight?  (NOT product
// code; tools only.)  The shipped xor_stream<8,8,0,kQueueFull> body is written
// "every load of the tile first", but the compiler's scheduler, aiming at
// occupancy it never gets (one workgroup per CU), software-pipelines it into
// 74 VGPRs with ~8-10 16-byte loads per lane outstanding (s_waitcnt vmcnt(8..9)
// in the ISA).  waves_per_eu(1) lets it keep all 64 in flight (276 VGPRs;
// exp 8: 82-84 %).  This sweeps the register budget between the two with the
// product's own tile body (stream_tile from bcp_kernels.hip), so the depth the
// scheduler picks moves with it:
//   amdgpu_waves_per_eu(W, W)  W = 8 (<= 64 VGPRs) ... 2 (<= 256)
//   amdgpu_num_vgpr(R)
// Second use: tile size U = 4 / 8 / 16 under the budget.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ibeegfs-chunk-parity_amd/csrc -Iinclude \
//         tools/exp/xor_exp5.hip -o tools/exp/xor_exp5
//   ./tools/exp/xor_exp5 [stripes] [reps] > sweep.jsonl
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

template <int U>
__device__ __forceinline__ void queue_loop(const StreamArgs &a) {
  __shared__ uint32_t next[2];
  if (threadIdx.x == 0) next[0] = queue_grab(a.ctr, a.base);
  __syncthreads();
  uint32_t t = __builtin_amdgcn_readfirstlane(next[0]);
  int slot = 0;
  while (t < a.ntiles) {
    stream_tile<8, U, 0, false>(a, t);
    slot ^= 1;
    if (threadIdx.x == 0) next[slot] = queue_grab(a.ctr, a.base);
    __syncthreads();
    t = __builtin_amdgcn_readfirstlane(next[slot]);
  }
}

template <int U, int W>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W, W))) void xs_uw(StreamArgs a) {
  queue_loop<U>(a);
}
template <int U>
__global__ __launch_bounds__(kBlock) void xs_u(StreamArgs a) {
  queue_loop<U>(a);
}

}  // namespace bcp

typedef void (*KFn)(bcp::StreamArgs);
struct Entry {
  const char *name;
  KFn fn;
  int u;
};

// (The r01 sweep of waves_per_eu 1..8 and amdgpu_num_vgpr at U = 8 is
// profiles/r01/depth/exp5_wpe_sweep.jsonl; this is the tile-size sweep under
// the shipped budget.)
static const Entry kV[] = {
    {"shipped xor_stream_w<8,8,0,full,6>", bcp::xor_stream_w<8, 8, 0, bcp::kQueueFull, 6>, 8},
    {"U=8 no budget", bcp::xs_u<8>, 8},
    {"U=16 wpe 6", bcp::xs_uw<16, 6>, 16},
    {"U=16 wpe 5", bcp::xs_uw<16, 5>, 16},
    {"U=16 wpe 7", bcp::xs_uw<16, 7>, 16},
    {"U=16 no budget", bcp::xs_u<16>, 16},
    {"U=4 wpe 6", bcp::xs_uw<4, 6>, 4},
    {"U=4 wpe 7", bcp::xs_uw<4, 7>, 4},
    {"U=4 wpe 5", bcp::xs_uw<4, 5>, 4},
    {"U=4 no budget", bcp::xs_u<4>, 4},
};

int main(int argc, char **argv) {
  const uint64_t stripes = argc > 1 ? strtoull(argv[1], 0, 10) : 12500;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
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
    a.tps = (uint32_t)(S / 16 / (256 * kV[v].u));
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
  for (int r = 0; r < reps; r++) {
    for (int v = 0; v < nv; v++) {
      if (r == 0) {
        CK(hipMemsetAsync(dst, 0, out_bytes, st));
        launch(v, dst);
        CK(bcp::launch_compare(st, grid, dst, ref, out_bytes, dcount));
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
    const double bytes = (double)(in_bytes + out_bytes);
    printf("{\"variant\": \"%s\", \"median_ms\": %.4f, \"min_ms\": %.4f, \"GBps\": %.1f, \"frac_8TBs\": %.4f, "
           "\"mismatch_bytes\": %lld}\n",
           kV[v].name, med, ts[0], bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12, bad[v]);
  }
  return 0;
}
