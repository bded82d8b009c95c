// xor_exp3.hip -- third round of kernel-design experiments (NOT product code;
// tools only): hiding the work-queue grab and, for the pointer-table
// (rebuild) form, the descriptor loads behind the data stream.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-atomic-optimizer-strategy=None \
//         tools/exp/xor_exp3.hip -o tools/exp/xor_exp3
//   ./tools/exp/xor_exp3 [stripes] [reps] > sweep.jsonl
// (the atomic optimizer turns the grab into a wave-combined atomic whose
// result is waited for at once, which would defeat AHEAD 3)
//
// Result (profiles/r01/kernel_exp_8_grab_ahead.jsonl, 7 reps): the shipped
// schedule stays best -- gen 8.544 ms (86.3 %), rebuild 8.593 ms (85.8 %).
// Hiding the grab costs 1-3 % (pre 84.8 %, ahead 83.3 %; rebuild ahead2
// 82.7 %), one wave per SIMD with every load of the tile in flight
// (waves_per_eu(1)) 82-84 %, 2 WG/CU 80-83 %.  The read-only ceiling of the
// same schedule is 91.9-92.0 % for both layouts.  The atomic round trip is not
// the limiter; more data in flight per CU only widens the address window.
// -DXE3_PRESTORE (profiles/r01/kernel_exp_8b_grab_before_stores.jsonl): the
// grab between the XORs and the stores (AHEAD 4) 81.7 % vs 84.9 % shipped.
//
// Shipped schedule (bcp_kernels.hip xor_stream): thread 0 grabs tile t+1 with
// one atomicAdd AFTER the stores of tile t, then one barrier; the atomic's
// round trip is a bubble in which the CU (1 workgroup per CU) has no loads in
// flight.  Variants:
//   AHEAD 0  shipped (grab after the stores)
//   AHEAD 1  grab issued right behind tile t's loads; its result is published
//            through LDS after the stores (same single barrier)
//   AHEAD 2  two tiles known in advance: the grab for t+2 goes out behind t's
//            loads and the pointer-table loads of t+1 are issued during t
//            (pointer-table form only)
//   AHEAD 3  grab issued right before tile t's loads
//   AHEAD 4  grab issued after the XORs, before the stores
// Workloads: GATHER 0 = config 2 gen (strided [stripes][8][S] -> [stripes][S]);
// GATHER 1 = config 3 rebuild (dense pointer table: 7 survivors of the source
// array + the parity array -> a third array).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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

template <typename T>
using const_as = const __attribute__((address_space(4))) T;
template <typename T>
__device__ __forceinline__ const_as<T> *cst(const T *p) { return (const_as<T> *)(uintptr_t)p; }
template <typename T>
using glob = __attribute__((address_space(1))) T;
template <typename T>
__device__ __forceinline__ glob<T> *gp(uint64_t p) { return (glob<T> *)(uintptr_t)p; }

struct Src {
  uint64_t ptr, len;
};

struct Args {
  char *dst;
  const char *src;
  const Src *table;  // GATHER: nsrc entries per stripe
  const uint64_t *dsts;  // GATHER: output pointer per stripe
  uint64_t S;
  uint32_t vps, tps, ntiles;
  unsigned long long *ctr;
  unsigned long long base;
};

__device__ __forceinline__ uint32_t grab(unsigned long long *ctr, unsigned long long base) {
  const unsigned long long v = atomicAdd(ctr, 1ull) - base;
  return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)v;
}
__device__ __forceinline__ uint32_t rel(unsigned long long v, unsigned long long base) {
  v -= base;
  return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)v;
}

enum { MODE_XOR = 0, MODE_READ = 1 };

template <int U, int GATHER, int AHEAD, int MODE>
__device__ __forceinline__ void xe3_body(const Args &a) {
  constexpr uint32_t tile_v = KB * U;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ uint32_t nx[2];
  v4u sink = {0u, 0u, 0u, 0u};
  uint32_t t, tn = 0xFFFFFFFFu;
  int slot = 0;
  if (threadIdx.x == 0) {
    nx[0] = grab(a.ctr, a.base);
    if (AHEAD == 2) nx[1] = grab(a.ctr, a.base);
  }
  __syncthreads();
  t = __builtin_amdgcn_readfirstlane(nx[0]);
  if (AHEAD == 2) {
    tn = __builtin_amdgcn_readfirstlane(nx[1]);
    slot = 1;
  }
  uint64_t ptr[NSRC];
  uint64_t dptr = 0;
  auto load_ptrs = [&](uint32_t tt, uint64_t *p, uint64_t &d) {
    const uint32_t s = tt / a.tps;
    const_as<Src> *sl = cst(a.table) + (uint64_t)s * NSRC;
#pragma unroll
    for (int k = 0; k < NSRC; k++) p[k] = sl[k].ptr;
    d = cst(a.dsts)[s];
  };
  if (GATHER && AHEAD == 2 && t < a.ntiles) load_ptrs(t, ptr, dptr);
  while (t < a.ntiles) {
    const uint32_t s = t / a.tps;
    const uint32_t tin = t - s * a.tps;
    const uint32_t vb = tin * tile_v + wave * 64 * U + lane;
    if (GATHER && AHEAD != 2) load_ptrs(t, ptr, dptr);
    if (!GATHER) {
      const uint64_t sb = (uint64_t)(uintptr_t)a.src + (uint64_t)s * NSRC * a.S;
#pragma unroll
      for (int k = 0; k < NSRC; k++) ptr[k] = sb + (uint64_t)k * a.S;
      dptr = (uint64_t)(uintptr_t)a.dst + (uint64_t)s * a.S;
    }
    unsigned long long g = 0;
    if (AHEAD == 3 && threadIdx.x == 0) g = atomicAdd(a.ctr, 1ull);
    v4u x[NSRC][U];
#pragma unroll
    for (int k = 0; k < NSRC; k++)
#pragma unroll
      for (int u = 0; u < U; u++) x[k][u] = __builtin_nontemporal_load(gp<v4u>(ptr[k]) + vb + u * 64);
    if ((AHEAD == 1 || AHEAD == 2) && threadIdx.x == 0) g = atomicAdd(a.ctr, 1ull);
    uint64_t pn[NSRC];
    uint64_t dn = 0;
    if (GATHER && AHEAD == 2 && tn < a.ntiles) load_ptrs(tn, pn, dn);
    v4u acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      acc[u] = x[0][u];
#pragma unroll
      for (int k = 1; k < NSRC; k++) acc[u] ^= x[k][u];
    }
    if (AHEAD == 4 && threadIdx.x == 0) g = atomicAdd(a.ctr, 1ull);
    if constexpr (MODE == MODE_READ) {
#pragma unroll
      for (int u = 0; u < U; u++) sink ^= acc[u];
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) __builtin_nontemporal_store(acc[u], gp<v4u>(dptr) + vb + u * 64);
    }
    slot ^= 1;
    if (threadIdx.x == 0) nx[slot] = AHEAD >= 1 ? rel(g, a.base) : grab(a.ctr, a.base);
    __syncthreads();
    if (AHEAD == 2) {
      t = tn;
      tn = __builtin_amdgcn_readfirstlane(nx[slot]);
      if (GATHER) {
#pragma unroll
        for (int k = 0; k < NSRC; k++) ptr[k] = pn[k];
        dptr = dn;
      }
    } else {
      t = __builtin_amdgcn_readfirstlane(nx[slot]);
    }
  }
  if constexpr (MODE == MODE_READ) {
    if (sink.x == 0x12345678u && sink.y == 0x9abcdef0u) a.dst[threadIdx.x] = 1;  // keep the loads
  }
}

template <int U, int GATHER, int AHEAD, int MODE>
__global__ __launch_bounds__(KB) void xe3(Args a) { xe3_body<U, GATHER, AHEAD, MODE>(a); }
// one wave per SIMD: the compiler may hold every load of a tile in flight
template <int U, int GATHER, int AHEAD, int MODE>
__global__ __launch_bounds__(KB) __attribute__((amdgpu_waves_per_eu(1, 1))) void xe3w(Args a) {
  xe3_body<U, GATHER, AHEAD, MODE>(a);
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
  int u, gather, ahead, mode, bpc;
};

#define X(name, U, G, A, M, BPC) {name, xe3<U, G, A, M>, U, G, A, M, BPC}
#define W(name, U, G, A, M, BPC) {name, xe3w<U, G, A, M>, U, G, A, M, BPC}
static const Entry kV[] = {
#ifdef XE3_PRESTORE
    X("gen_base_u8", 8, 0, 0, MODE_XOR, 1),
    X("gen_prestore_u8", 8, 0, 4, MODE_XOR, 1),
    X("gen_base_u4", 4, 0, 0, MODE_XOR, 1),
    X("gen_prestore_u4", 4, 0, 4, MODE_XOR, 1),
    X("gen_prestore_u4_bpc2", 4, 0, 4, MODE_XOR, 2),
    X("reb_base_u8", 8, 1, 0, MODE_XOR, 1),
    X("reb_prestore_u8", 8, 1, 4, MODE_XOR, 1),
#else
    X("gen_base_u8", 8, 0, 0, MODE_XOR, 1),
    X("gen_ahead_u8", 8, 0, 1, MODE_XOR, 1),
    X("gen_base_u4", 4, 0, 0, MODE_XOR, 1),
    X("gen_ahead_u4", 4, 0, 1, MODE_XOR, 1),
    X("gen_pre_u8", 8, 0, 3, MODE_XOR, 1),
    X("gen_pre_u4", 4, 0, 3, MODE_XOR, 1),
    X("gen_pre_u4_bpc2", 4, 0, 3, MODE_XOR, 2),
    X("gen_ahead_u4_bpc2", 4, 0, 1, MODE_XOR, 2),
    X("gen_ahead_u8_bpc2", 8, 0, 1, MODE_XOR, 2),
    W("gen_w1_base_u8", 8, 0, 0, MODE_XOR, 1),
    W("gen_w1_pre_u8", 8, 0, 3, MODE_XOR, 1),
    W("gen_w1_ahead_u8", 8, 0, 1, MODE_XOR, 1),
    W("gen_w1_pre_u4", 4, 0, 3, MODE_XOR, 1),
    W("gen_w1_pre_u16", 16, 0, 3, MODE_XOR, 1),
    X("gen_read_base_u8", 8, 0, 0, MODE_READ, 1),
    X("gen_read_ahead_u8", 8, 0, 1, MODE_READ, 1),
    X("reb_base_u8", 8, 1, 0, MODE_XOR, 1),
    X("reb_ahead_u8", 8, 1, 1, MODE_XOR, 1),
    X("reb_pre_u8", 8, 1, 3, MODE_XOR, 1),
    X("reb_ahead2_u8", 8, 1, 2, MODE_XOR, 1),
    X("reb_ahead2_u4", 4, 1, 2, MODE_XOR, 1),
    X("reb_ahead2_u4_bpc2", 4, 1, 2, MODE_XOR, 2),
    W("reb_w1_pre_u8", 8, 1, 3, MODE_XOR, 1),
    W("reb_w1_ahead2_u8", 8, 1, 2, MODE_XOR, 1),
    X("reb_read_base_u8", 8, 1, 0, MODE_READ, 1),
#endif
};
#undef X
#undef W

int main(int argc, char **argv) {
  const uint64_t stripes = argc > 1 ? strtoull(argv[1], 0, 10) : 12500;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const uint64_t S = 512 * 1024;
  const uint64_t in_bytes = stripes * NSRC * S, out_bytes = stripes * S;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  char *src, *par, *dst, *ref_gen, *ref_reb;
  Src *table;
  uint64_t *dsts;
  unsigned long long *ctr, *dcount;
  // XE3_CONTIG=1: physically contiguous allocations (hipDeviceMallocContiguous)
  const bool contig = getenv("XE3_CONTIG") && atoi(getenv("XE3_CONTIG"));
  auto dalloc = [&](char **p, size_t n) {
    if (contig) CK(hipExtMallocWithFlags((void **)p, n, hipDeviceMallocContiguous));
    else CK(hipMalloc(p, n));
  };
  dalloc(&src, in_bytes);
  dalloc(&par, out_bytes);
  dalloc(&dst, out_bytes);
  dalloc(&ref_gen, out_bytes);
  dalloc(&ref_reb, out_bytes);
  CK(hipMalloc(&table, stripes * NSRC * sizeof(Src)));
  CK(hipMalloc(&dsts, stripes * sizeof(uint64_t)));
  CK(hipMalloc(&ctr, 256));
  CK(hipMalloc(&dcount, 8));
  CK(hipMemset(ctr, 0, 256));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipLaunchKernelGGL(fill, dim3(cus * 8), dim3(256), 0, st, (uint64_t *)src, in_bytes / 8, 1ull);
  const uint32_t vps = S / 16;
  unsigned long long base = 0;
  const int nv = sizeof(kV) / sizeof(kV[0]);
  // rebuild tables: victim 3; survivors then the parity body; output to dst (set per launch)
  std::vector<Src> h_table(stripes * NSRC);
  for (uint64_t s = 0; s < stripes; s++) {
    int i = 0;
    for (int k = 0; k < NSRC; k++)
      if (k != 3) h_table[s * NSRC + i++] = Src{(uint64_t)(uintptr_t)(src + (s * NSRC + k) * S), S};
    h_table[s * NSRC + i] = Src{(uint64_t)(uintptr_t)(par + s * S), S};
  }
  CK(hipMemcpy(table, h_table.data(), h_table.size() * sizeof(Src), hipMemcpyHostToDevice));
  std::vector<uint64_t> h_dsts(stripes);
  char *cur_dsts_for = nullptr;
  auto set_dsts = [&](char *out) {
    if (cur_dsts_for == out) return;
    for (uint64_t s = 0; s < stripes; s++) h_dsts[s] = (uint64_t)(uintptr_t)(out + s * S);
    CK(hipMemcpyAsync(dsts, h_dsts.data(), stripes * 8, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    cur_dsts_for = out;
  };
  auto launch = [&](int v, char *out) {
    Args a;
    a.dst = out;
    a.src = src;
    a.table = table;
    a.dsts = dsts;
    a.S = S;
    a.vps = vps;
    a.tps = vps / (KB * kV[v].u);
    a.ntiles = (uint32_t)(stripes * a.tps);
    a.ctr = ctr;
    a.base = base;
    int grid = std::min<int>(cus * kV[v].bpc, a.ntiles);
    if (getenv("XE3_GRID")) grid = std::min<int>(atoi(getenv("XE3_GRID")), a.ntiles);  // A/B of the grid size
    hipLaunchKernelGGL(kV[v].fn, dim3(grid), dim3(KB), 0, st, a);
    CK(hipGetLastError());
    // every workgroup makes one failing grab (AHEAD 2: two)
    base += a.ntiles + (uint64_t)grid * (kV[v].ahead == 2 ? 2 : 1);
  };
  // references: gen -> par (the parity used by rebuild), and ref_gen; rebuild of victim 3 -> ref_reb
  launch(0, par);
  launch(0, ref_gen);
  set_dsts(ref_reb);
  int reb_base = -1;
  for (int v = 0; v < nv; v++)
    if (!strcmp(kV[v].name, "reb_base_u8")) reb_base = v;
  launch(reb_base, ref_reb);
  CK(hipStreamSynchronize(st));
  {
    // rebuilt chunk must equal source 3
    CK(hipMemsetAsync(dcount, 0, 8, st));
    unsigned long long tot = 0;
    for (uint64_t s = 0; s < stripes; s += 97) {
      CK(hipMemsetAsync(dcount, 0, 8, st));
      hipLaunchKernelGGL(diff, dim3(64), dim3(256), 0, st, (const uint64_t *)(ref_reb + s * S),
                         (const uint64_t *)(src + (s * NSRC + 3) * S), S / 8, dcount);
      unsigned long long h;
      CK(hipMemcpyAsync(&h, dcount, 8, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
      tot += h;
    }
    fprintf(stderr, "rebuild reference vs source 3 (sampled): %llu mismatching words\n", tot);
    if (tot) return 3;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  set_dsts(dst);
  std::vector<std::vector<float>> times(nv);
  std::vector<long long> bad(nv, -1);
  for (int r = 0; r < reps; r++) {
    for (int v = 0; v < nv; v++) {
      if (r == 0 && kV[v].mode == MODE_XOR) {
        CK(hipMemsetAsync(dst, 0, out_bytes, st));
        launch(v, dst);
        CK(hipMemsetAsync(dcount, 0, 8, st));
        hipLaunchKernelGGL(diff, dim3(cus * 4), dim3(256), 0, st, (const uint64_t *)dst,
                           (const uint64_t *)(kV[v].gather ? ref_reb : ref_gen), out_bytes / 8, dcount);
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
    const double bytes = kV[v].mode == MODE_XOR ? (double)(in_bytes + out_bytes) : (double)in_bytes;
    printf("{\"variant\": \"%s\", \"vecs\": %d, \"gather\": %d, \"ahead\": %d, \"blocks_per_cu\": %d, "
           "\"median_ms\": %.4f, \"min_ms\": %.4f, \"GBps\": %.1f, \"frac_8TBs\": %.4f, \"mismatch_words\": %lld}\n",
           kV[v].name, kV[v].u, kV[v].gather, kV[v].ahead, kV[v].bpc, med, ts[0], bytes / (med * 1e-3) / 1e9,
           bytes / (med * 1e-3) / 8e12, bad[v]);
  }
  return 0;
}
