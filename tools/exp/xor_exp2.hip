// xor_exp2.hip -- second round of kernel-design experiments on the shipped
// work-queue schedule (NOT product code; tools only).  Interleaved A/B in one
// process over the config-2 fold (12,500 stripes x 8 x 512 KiB), every
// variant's output checked against variant 0 (= the shipped xor_stream<8,4,0>
// design).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/exp/xor_exp2.hip -o tools/exp/xor_exp2
//   ./tools/exp/xor_exp2 [stripes] [reps] > sweep.jsonl
//
// Result (profiles/r01/kernel_exp_4.jsonl): nothing beats the shipped design
// by more than the 0.4 % noise; the same schedule reading only (no stores)
// runs at 82 % of 8 TB/s, so the XOR at 79.3 % is within 3 % of its own
// read ceiling; LDS-DMA staging 64 % (U = 2) / 36 % (U = 1); default-policy
// or sc1 loads -6 %; plain stores -8 %, sc1 stores -4 %.  ("write_only"
// measures the queue counter, ~83 grabs/us, not HBM.)
//
// Axes: load flavour (global nt / buffer aux bits), store flavour (nt /
// plain / buffer sc1 / sc0 sc1), deferred stores (tile i's stores issued after
// tile i+1's loads), workgroup size (256 / 512 threads), LDS-DMA staging
// (global_load_lds_dwordx4 of the 8 source rows of a tile, XOR from LDS), and
// the read-only / write-only ceilings of the same schedule.
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

enum { LD_GNT = 0, LD_BNT = 1, LD_BSC1 = 2, LD_BPLAIN = 3 };
enum { ST_NT = 0, ST_PLAIN = 1, ST_BSC1 = 2, ST_BSC01 = 3, ST_NONE = 4 };
enum { MODE_XOR = 0, MODE_READ = 1, MODE_WRITE = 2 };

struct Args {
  char *dst;
  const char *src;
  uint64_t pitch;  // source row pitch (bytes); stripe pitch = NSRC * pitch
  uint32_t vps, tps, ntiles;
  unsigned long long *ctr;
  unsigned long long base;
};

__device__ __forceinline__ uint32_t grab(unsigned long long *ctr, unsigned long long base) {
  const unsigned long long v = atomicAdd(ctr, 1ull) - base;
  return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)v;
}

template <int KB, int U, int LD, int ST, int DEFER, int MODE>
__global__ __launch_bounds__(KB) void xe2(Args a) {
  constexpr uint32_t tile_v = KB * U;
  const uint64_t S = a.pitch;
  const uint64_t SO = (uint64_t)a.vps * 16;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ uint32_t next[2];
  if (threadIdx.x == 0) next[0] = grab(a.ctr, a.base);
  __syncthreads();
  uint32_t t = __builtin_amdgcn_readfirstlane(next[0]);
  int slot = 0;
  v4u prev[U];
  v4u *prev_db = nullptr;
  uint32_t prev_vb = 0;
  bool have_prev = false;
  v4u sink = {0u, 0u, 0u, 0u};
  while (t < a.ntiles) {
    const uint32_t s = t / a.tps;
    const uint32_t tin = t - s * a.tps;
    const char *sb = a.src + (uint64_t)s * NSRC * S;
    v4u *db = reinterpret_cast<v4u *>(a.dst + (uint64_t)s * SO);
    const uint32_t vb = tin * tile_v + wave * 64 * U + lane;
    v4u acc[U];
    if constexpr (MODE == MODE_WRITE) {
#pragma unroll
      for (int u = 0; u < U; u++) acc[u] = v4u{t, vb, (uint32_t)u, 7u};
    } else {
      v4u x[NSRC][U];
      if constexpr (LD == LD_GNT) {
#pragma unroll
        for (int k = 0; k < NSRC; k++)
#pragma unroll
          for (int u = 0; u < U; u++)
            x[k][u] = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(sb + k * S) + vb + u * 64);
      } else {
        constexpr int aux = LD == LD_BNT ? 2 : LD == LD_BSC1 ? 16 : 0;
        __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc((void *)sb, (short)0, (int)(NSRC * S), 0x00020000);
#pragma unroll
        for (int k = 0; k < NSRC; k++)
#pragma unroll
          for (int u = 0; u < U; u++)
            x[k][u] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)((vb + u * 64) * 16), (int)(k * S), aux);
      }
      if constexpr (DEFER) {
        // stores of the previous tile go out behind this tile's loads
        __builtin_amdgcn_sched_barrier(0);
        if (have_prev) {
#pragma unroll
          for (int u = 0; u < U; u++) __builtin_nontemporal_store(prev[u], prev_db + prev_vb + u * 64);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        acc[u] = x[0][u];
#pragma unroll
        for (int k = 1; k < NSRC; k++) acc[u] ^= x[k][u];
      }
    }
    if constexpr (MODE == MODE_READ) {
#pragma unroll
      for (int u = 0; u < U; u++) sink ^= acc[u];
    } else if constexpr (DEFER) {
#pragma unroll
      for (int u = 0; u < U; u++) prev[u] = acc[u];
      prev_db = db;
      prev_vb = vb;
      have_prev = true;
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) {
        v4u *p = db + vb + u * 64;
        if constexpr (ST == ST_NT) __builtin_nontemporal_store(acc[u], p);
        else if constexpr (ST == ST_PLAIN) *p = acc[u];
        else {
          __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void *)db, (short)0, (int)SO, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(acc[u], w, (int)((vb + u * 64) * 16), 0, ST == ST_BSC1 ? 16 : 17);
        }
      }
    }
    slot ^= 1;
    if (threadIdx.x == 0) next[slot] = grab(a.ctr, a.base);
    __syncthreads();
    t = __builtin_amdgcn_readfirstlane(next[slot]);
  }
  if constexpr (DEFER && MODE == MODE_XOR) {
    if (have_prev) {
#pragma unroll
      for (int u = 0; u < U; u++) __builtin_nontemporal_store(prev[u], prev_db + prev_vb + u * 64);
    }
  }
  if constexpr (MODE == MODE_READ) {
    if (sink.x == 0x12345678u && sink.y == 0x9abcdef0u) a.dst[threadIdx.x] = 1;  // keep the loads
  }
}

// LDS-DMA staging: each wave DMAs its 8 x 64 x U x 16 B share of the tile
// straight into LDS (global_load_lds_dwordx4), waits, XORs from LDS.
template <int U>
__global__ __launch_bounds__(256) void xe2_lds(Args a) {
  constexpr int KB = 256;
  constexpr uint32_t tile_v = KB * U;
  const uint64_t S = (uint64_t)a.vps * 16;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ v4u stage[4][NSRC][U][64];  // 4 waves x 8 x U x 1 KiB
  __shared__ uint32_t next[2];
  if (threadIdx.x == 0) next[0] = grab(a.ctr, a.base);
  __syncthreads();
  uint32_t t = __builtin_amdgcn_readfirstlane(next[0]);
  int slot = 0;
  while (t < a.ntiles) {
    const uint32_t s = t / a.tps;
    const uint32_t tin = t - s * a.tps;
    const char *sb = a.src + (uint64_t)s * NSRC * S;
    v4u *db = reinterpret_cast<v4u *>(a.dst + (uint64_t)s * S);
    const uint32_t vb = tin * tile_v + wave * 64 * U + lane;
#pragma unroll
    for (int k = 0; k < NSRC; k++)
#pragma unroll
      for (int u = 0; u < U; u++) {
        const v4u *g = reinterpret_cast<const v4u *>(sb + k * S) + vb + u * 64;
        __builtin_amdgcn_global_load_lds((const void *)g, (__attribute__((address_space(3))) void *)&stage[wave][k][u][0],
                                         16, 0, 2);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    v4u acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      acc[u] = stage[wave][0][u][lane];
#pragma unroll
      for (int k = 1; k < NSRC; k++) acc[u] ^= stage[wave][k][u][lane];
    }
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_nontemporal_store(acc[u], db + vb + u * 64);
    slot ^= 1;
    if (threadIdx.x == 0) next[slot] = grab(a.ctr, a.base);
    __syncthreads();
    t = __builtin_amdgcn_readfirstlane(next[slot]);
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
  int kb, u, mode, bpc;  // bpc: workgroups per CU launched
  int pad;               // source row pitch = 512 KiB + pad (output unchanged)
};

#define X(name, KB, U, LD, ST, DEF, MODE, BPC) {name, xe2<KB, U, LD, ST, DEF, MODE>, KB, U, MODE, BPC, 0}
#define P(name, PAD) {name, xe2<256, 4, LD_GNT, ST_NT, 0, MODE_XOR>, 256, 4, MODE_XOR, 8, PAD}
static const Entry kV[] = {
#if defined(XE2_OCC2)
    X("base", 256, 4, LD_GNT, ST_NT, 0, MODE_XOR, 8),
    X("u4_bpc1", 256, 4, LD_GNT, ST_NT, 0, MODE_XOR, 1),
    X("u8_bpc1", 256, 8, LD_GNT, ST_NT, 0, MODE_XOR, 1),
    X("u16_bpc1", 256, 16, LD_GNT, ST_NT, 0, MODE_XOR, 1),
    X("u8_bpc1_defer", 256, 8, LD_GNT, ST_NT, 1, MODE_XOR, 1),
    X("u4_bpc1_defer", 256, 4, LD_GNT, ST_NT, 1, MODE_XOR, 1),
    X("wg512_u8_bpc1", 512, 8, LD_GNT, ST_NT, 0, MODE_XOR, 1),
    X("wg128_u8_bpc2", 128, 8, LD_GNT, ST_NT, 0, MODE_XOR, 2),
    X("wg128_u16_bpc1", 128, 16, LD_GNT, ST_NT, 0, MODE_XOR, 1),
    X("wg128_u8_bpc1", 128, 8, LD_GNT, ST_NT, 0, MODE_XOR, 1),
    X("wg64_u16_bpc2", 64, 16, LD_GNT, ST_NT, 0, MODE_XOR, 2),
    X("u8_bpc1_bnt", 256, 8, LD_BNT, ST_NT, 0, MODE_XOR, 1),
    X("read_u8_bpc1", 256, 8, LD_GNT, ST_NONE, 0, MODE_READ, 1),
#elif defined(XE2_OCC)
    X("base", 256, 4, LD_GNT, ST_NT, 0, MODE_XOR, 8),
    X("bpc1", 256, 4, LD_GNT, ST_NT, 0, MODE_XOR, 1),
    X("bpc2", 256, 4, LD_GNT, ST_NT, 0, MODE_XOR, 2),
    X("bpc3", 256, 4, LD_GNT, ST_NT, 0, MODE_XOR, 3),
    X("bpc4", 256, 4, LD_GNT, ST_NT, 0, MODE_XOR, 4),
    X("u8_bpc1", 256, 8, LD_GNT, ST_NT, 0, MODE_XOR, 1),
    X("u8_bpc2", 256, 8, LD_GNT, ST_NT, 0, MODE_XOR, 2),
    X("u8_bpc4", 256, 8, LD_GNT, ST_NT, 0, MODE_XOR, 4),
    X("wg512_u4_bpc1", 512, 4, LD_GNT, ST_NT, 0, MODE_XOR, 1),
    X("wg512_u4_bpc2", 512, 4, LD_GNT, ST_NT, 0, MODE_XOR, 2),
    X("wg1024_u4_bpc1", 1024, 4, LD_GNT, ST_NT, 0, MODE_XOR, 1),
    X("wg1024_u2_bpc1", 1024, 2, LD_GNT, ST_NT, 0, MODE_XOR, 1),
    X("defer_bpc2", 256, 4, LD_GNT, ST_NT, 1, MODE_XOR, 2),
    X("defer_bpc4", 256, 4, LD_GNT, ST_NT, 1, MODE_XOR, 4),
#elif defined(XE2_PITCH)
    X("base", 256, 4, LD_GNT, ST_NT, 0, MODE_XOR, 8),
    P("pad256", 256),
    P("pad1k", 1024),
    P("pad4k", 4096),
    P("pad8k", 8192),
    P("pad16k", 16384),
    P("pad64k", 65536),
    P("pad3968", 3968),
    P("pad12k", 12288),
    {"read_only", xe2<256, 4, LD_GNT, ST_NONE, 0, MODE_READ>, 256, 4, MODE_READ, 8, 0},
    {"read_only_pad4k", xe2<256, 4, LD_GNT, ST_NONE, 0, MODE_READ>, 256, 4, MODE_READ, 8, 4096},
#else
    X("base", 256, 4, LD_GNT, ST_NT, 0, MODE_XOR, 8),
    X("read_only", 256, 4, LD_GNT, ST_NONE, 0, MODE_READ, 8),
    X("write_only", 256, 4, LD_GNT, ST_NT, 0, MODE_WRITE, 8),
    X("st_plain", 256, 4, LD_GNT, ST_PLAIN, 0, MODE_XOR, 8),
    X("st_bsc1", 256, 4, LD_GNT, ST_BSC1, 0, MODE_XOR, 8),
    X("st_bsc01", 256, 4, LD_GNT, ST_BSC01, 0, MODE_XOR, 8),
    X("ld_bnt", 256, 4, LD_BNT, ST_NT, 0, MODE_XOR, 8),
    X("ld_bsc1", 256, 4, LD_BSC1, ST_NT, 0, MODE_XOR, 8),
    X("ld_bplain", 256, 4, LD_BPLAIN, ST_NT, 0, MODE_XOR, 8),
    X("defer", 256, 4, LD_GNT, ST_NT, 1, MODE_XOR, 8),
    X("wg512_u2", 512, 2, LD_GNT, ST_NT, 0, MODE_XOR, 4),
    X("wg512_u4", 512, 4, LD_GNT, ST_NT, 0, MODE_XOR, 4),
    X("wg1024_u2", 1024, 2, LD_GNT, ST_NT, 0, MODE_XOR, 2),
    X("base_bpc4", 256, 4, LD_GNT, ST_NT, 0, MODE_XOR, 4),
    X("base_bpc6", 256, 4, LD_GNT, ST_NT, 0, MODE_XOR, 6),
    {"lds_dma_u1", xe2_lds<1>, 256, 1, MODE_XOR, 8, 0},
    {"lds_dma_u2", xe2_lds<2>, 256, 2, MODE_XOR, 8, 0},
#endif
};
#undef X

int main(int argc, char **argv) {
  const uint64_t stripes = argc > 1 ? strtoull(argv[1], 0, 10) : 12500;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const uint64_t S = 512 * 1024;
  const uint64_t in_bytes = stripes * NSRC * S, out_bytes = stripes * S;
  const uint64_t max_pad = 65536;
  const uint64_t alloc_in = stripes * NSRC * (S + max_pad);
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  char *src, *dst, *ref;
  unsigned long long *ctr, *dcount;
  CK(hipMalloc(&src, alloc_in));
  CK(hipMalloc(&dst, out_bytes));
  CK(hipMalloc(&ref, out_bytes));
  CK(hipMalloc(&ctr, 256));
  CK(hipMalloc(&dcount, 8));
  CK(hipMemset(ctr, 0, 256));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipLaunchKernelGGL(fill, dim3(cus * 8), dim3(256), 0, st, (uint64_t *)src, alloc_in / 8, 1ull);
  const uint32_t vps = S / 16;
  unsigned long long base = 0;
  const int nv = sizeof(kV) / sizeof(kV[0]);
  auto launch = [&](int v, char *out) {
    Args a;
    a.dst = out;
    a.src = src;
    a.pitch = S + kV[v].pad;
    a.vps = vps;
    a.tps = vps / (kV[v].kb * kV[v].u);
    a.ntiles = (uint32_t)(stripes * a.tps);
    a.ctr = ctr;
    a.base = base;
    int grid = std::min<int>(cus * kV[v].bpc, a.ntiles);
    hipLaunchKernelGGL(kV[v].fn, dim3(grid), dim3(kV[v].kb), 0, st, a);
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
      if (r == 0) CK(hipMemsetAsync(dst, 0, out_bytes, st));
      launch(v, dst);
      if (r == 0 && kV[v].mode == MODE_XOR && kV[v].pad == 0) {
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
    const double bytes = kV[v].mode == MODE_XOR ? (double)(in_bytes + out_bytes)
                         : kV[v].mode == MODE_READ ? (double)in_bytes : (double)out_bytes;
    printf("{\"variant\": \"%s\", \"wg\": %d, \"vecs\": %d, \"blocks_per_cu\": %d, \"median_ms\": %.4f, "
           "\"min_ms\": %.4f, \"GBps\": %.1f, \"frac_8TBs\": %.4f, \"mismatch_words\": %lld, \"pad\": %d}\n",
           kV[v].name, kV[v].kb, kV[v].u, kV[v].bpc, med, ts[0], bytes / (med * 1e-3) / 1e9,
           bytes / (med * 1e-3) / 8e12, bad[v], kV[v].pad);
  }
  return 0;
}
