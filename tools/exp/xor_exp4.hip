// xor_exp4.hip -- LDS staging of the stripe tile, done the way the CDNA4
// guide prescribes for a pipelined stream (NOT product code; tools only):
// global_load_lds_dwordx4 (glds) into NBUF LDS buffers, counted vmcnt so the
// next tiles' DMA stays in flight while the current tile is XORed from LDS,
// raw s_barrier only.  A device-wide atomic queue cannot be used here (hipcc
// waits vmcnt(0) at the first use of any ordinary load result while a glds is
// in flight, which would drain the pipeline), so tiles are handed out
// grid-stride: workgroup b takes tiles b, b + G, b + 2G, ... (G = grid), which
// keeps the chip's tiles in one ascending window like the queue does.  The
// register-staged kernel is timed beside it with the queue (shipped) and with
// the same grid-stride schedule.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/exp/xor_exp4.hip -o tools/exp/xor_exp4
//   ./tools/exp/xor_exp4 [stripes] [reps] > sweep.jsonl
//
// Result (profiles/r01/kernel_exp_9_lds_pipeline.jsonl, 7 reps, one box):
// shipped register staging + queue 8.77 ms (84.1 %); on the grid-stride
// schedule register staging 73.8 % (U = 8) and pipelined LDS staging 71.0 %
// (U = 2, 2 buffers; U = 1 with 2/3/4 buffers 69-70 %, 2 WG/CU 63 %).  On equal
// schedules LDS staging trails register staging by ~3 points (the data is read
// once: the LDS round trip adds work and caps the tile at the LDS size), and
// the schedule it cannot use -- the atomic queue -- is worth 10 points.
#include <hip/hip_runtime.h>
#include <stdint.h>
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

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int NSRC = 8;
constexpr int KB = 256;

struct Args {
  char *dst;
  const char *src;
  uint64_t S;
  uint32_t tps, ntiles;
  unsigned long long *ctr;
  unsigned long long base;
};

__device__ __forceinline__ uint32_t grab(unsigned long long *ctr, unsigned long long base) {
  const unsigned long long v = atomicAdd(ctr, 1ull) - base;
  return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)v;
}

// Register staging (the shipped xor_stream<8,U,0> body); QUEUE = 1: atomic
// work queue (shipped), 0: grid-stride.
template <int U, int QUEUE>
__global__ __launch_bounds__(KB) void xr(Args a) {
  constexpr uint32_t tile_v = KB * U;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ uint32_t nx[2];
  uint32_t t;
  int slot = 0;
  if (QUEUE) {
    if (threadIdx.x == 0) nx[0] = grab(a.ctr, a.base);
    __syncthreads();
    t = __builtin_amdgcn_readfirstlane(nx[0]);
  } else {
    t = blockIdx.x;
  }
  while (t < a.ntiles) {
    const uint32_t s = t / a.tps, tin = t - s * a.tps;
    const uint32_t vb = tin * tile_v + wave * 64 * U + lane;
    const v4u *sb = reinterpret_cast<const v4u *>(a.src + (uint64_t)s * NSRC * a.S);
    v4u *db = reinterpret_cast<v4u *>(a.dst + (uint64_t)s * a.S);
    v4u x[NSRC][U];
#pragma unroll
    for (int k = 0; k < NSRC; k++)
#pragma unroll
      for (int u = 0; u < U; u++) x[k][u] = __builtin_nontemporal_load(sb + k * (a.S / 16) + vb + u * 64);
#pragma unroll
    for (int u = 0; u < U; u++) {
      v4u acc = x[0][u];
#pragma unroll
      for (int k = 1; k < NSRC; k++) acc ^= x[k][u];
      __builtin_nontemporal_store(acc, db + vb + u * 64);
    }
    if (QUEUE) {
      slot ^= 1;
      if (threadIdx.x == 0) nx[slot] = grab(a.ctr, a.base);
      __syncthreads();
      t = __builtin_amdgcn_readfirstlane(nx[slot]);
    } else {
      t += gridDim.x;
    }
  }
}

// LDS staging: NBUF buffers of one tile each (8 sources x 4 waves x U KiB);
// each wave DMAs and reads only its own part, so waves never wait for each
// other (no barrier in the loop at all).
template <int U, int NBUF>
__global__ __launch_bounds__(KB) void xl(Args a) {
  constexpr uint32_t tile_v = KB * U;
  constexpr int PER_TILE = NSRC * U;  // glds per lane per tile
  __shared__ v4u stage[NBUF][4][NSRC][U][64];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  auto dma = [&](uint32_t t, int b) {
    const uint32_t s = t / a.tps, tin = t - s * a.tps;
    const uint32_t vb = tin * tile_v + wave * 64 * U + lane;
    const v4u *sb = reinterpret_cast<const v4u *>(a.src + (uint64_t)s * NSRC * a.S);
#pragma unroll
    for (int k = 0; k < NSRC; k++)
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds((const void *)(sb + k * (a.S / 16) + vb + u * 64),
                                         (__attribute__((address_space(3))) void *)&stage[b][wave][k][u][0], 16, 0,
                                         2 /* nt */);
  };
  const uint32_t G = gridDim.x;
  uint32_t t = blockIdx.x;
  // prologue: NBUF - 1 tiles in flight
#pragma unroll
  for (int p = 0; p < NBUF - 1; p++)
    if (t + p * G < a.ntiles) dma(t + p * G, p);
  int b = 0;
  while (t < a.ntiles) {
    const uint32_t tn = t + (NBUF - 1) * G;
    const bool more = tn < a.ntiles;
    if (more) dma(tn, (b + NBUF - 1) % NBUF);
    // tile t retired once at most (tiles issued after it) * PER_TILE DMAs
    // remain (the previous tile's stores are older still).
    // Count the DMAs issued after tile t that may stay in flight.
    uint32_t ahead = 0;
#pragma unroll
    for (int p = 1; p < NBUF; p++) ahead += (t + p * G < a.ntiles) ? 1u : 0u;
    switch (ahead * PER_TILE) {
#define W_(n) case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
      W_(0) W_(8) W_(16) W_(24) W_(32) W_(48) W_(64)
#undef W_
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
    const uint32_t s = t / a.tps, tin = t - s * a.tps;
    const uint32_t vb = tin * tile_v + wave * 64 * U + lane;
    v4u *db = reinterpret_cast<v4u *>(a.dst + (uint64_t)s * a.S);
#pragma unroll
    for (int u = 0; u < U; u++) {
      v4u acc = stage[b][wave][0][u][lane];
#pragma unroll
      for (int k = 1; k < NSRC; k++) acc ^= stage[b][wave][k][u][lane];
      __builtin_nontemporal_store(acc, db + vb + u * 64);
    }
    // the next DMA into buffer b is issued only after these LDS reads
    // completed (their values were consumed by the stores above)
    b = (b + 1) % NBUF;
    t += G;
  }
}

__global__ void fill(uint64_t *p, uint64_t n, uint64_t seed) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t x = seed + i + 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    p[i] = x ^ (x >> 31);
  }
}

__global__ void diff(const uint64_t *a, const uint64_t *b, uint64_t n, unsigned long long *out) {
  unsigned long long c = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c += a[i] != b[i];
  if (c) atomicAdd(out, c);
}

typedef void (*KFn)(Args);
struct Entry {
  const char *name;
  KFn fn;
  int u, queue, bpc;
};

static const Entry kV[] = {
    {"reg_queue_u8 (shipped)", xr<8, 1>, 8, 1, 1},
    {"reg_gridstride_u8", xr<8, 0>, 8, 0, 1},
    {"reg_gridstride_u4", xr<4, 0>, 4, 0, 1},
    {"reg_gridstride_u4_bpc2", xr<4, 0>, 4, 0, 2},
    {"lds_u2_2buf", xl<2, 2>, 2, 0, 1},
    {"lds_u1_2buf", xl<1, 2>, 1, 0, 1},
    {"lds_u1_4buf", xl<1, 4>, 1, 0, 1},
    {"lds_u1_3buf", xl<1, 3>, 1, 0, 1},
    {"lds_u1_2buf_bpc2", xl<1, 2>, 1, 0, 2},
};

int main(int argc, char **argv) {
  const uint64_t stripes = argc > 1 ? strtoull(argv[1], 0, 10) : 12500;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const uint64_t S = 512 * 1024;
  const uint64_t in_bytes = stripes * NSRC * S, out_bytes = stripes * S;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
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
  hipLaunchKernelGGL(fill, dim3(cus * 8), dim3(256), 0, st, (uint64_t *)src, in_bytes / 8, 1ull);
  unsigned long long base = 0;
  const int nv = sizeof(kV) / sizeof(kV[0]);
  auto launch = [&](int v, char *out) {
    Args a;
    a.dst = out;
    a.src = src;
    a.S = S;
    a.tps = (uint32_t)(S / 16 / (KB * kV[v].u));
    a.ntiles = (uint32_t)(stripes * a.tps);
    a.ctr = ctr;
    a.base = base;
    const int grid = std::min<int>(cus * kV[v].bpc, a.ntiles);
    hipLaunchKernelGGL(kV[v].fn, dim3(grid), dim3(KB), 0, st, a);
    CK(hipGetLastError());
    if (kV[v].queue) base += a.ntiles + grid;
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
        CK(hipMemsetAsync(dcount, 0, 8, st));
        hipLaunchKernelGGL(diff, dim3(cus * 4), dim3(256), 0, st, (const uint64_t *)dst, (const uint64_t *)ref,
                           out_bytes / 8, dcount);
        unsigned long long h;
        CK(hipMemcpyAsync(&h, dcount, 8, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        bad[v] = (long long)h;
      }
      CK(hipEventRecord(e0, st));
      launch(v, dst);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      times[v].push_back(ms);
    }
    fprintf(stderr, "rep %d/%d done\n", r + 1, reps);
  }
  for (int v = 0; v < nv; v++) {
    auto ts = times[v];
    std::sort(ts.begin(), ts.end());
    const float med = ts[ts.size() / 2];
    const double bytes = (double)(in_bytes + out_bytes);
    printf("{\"variant\": \"%s\", \"vecs\": %d, \"queue\": %d, \"blocks_per_cu\": %d, \"median_ms\": %.4f, "
           "\"min_ms\": %.4f, \"GBps\": %.1f, \"frac_8TBs\": %.4f, \"mismatch_words\": %lld}\n",
           kV[v].name, kV[v].u, kV[v].queue, kV[v].bpc, med, ts[0], bytes / (med * 1e-3) / 1e9,
           bytes / (med * 1e-3) / 8e12, bad[v]);
  }
  return 0;
}
