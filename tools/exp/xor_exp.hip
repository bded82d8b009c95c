// xor_exp.hip -- kernel-design experiments for the 8-wide fast path (NOT
// product code; tools only).  One binary times a table of variants of the
// config-2 fold (12,500 stripes x 8 x 512 KiB) interleaved in one process and
// checks each variant's output against variant 0 (the shipped design).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DXE_SWEEP2|-DXE_SWEEP3] \
//         tools/exp/xor_exp.hip -o tools/exp/xor_exp
//   ./tools/exp/xor_exp [stripes] [reps] [blocks_per_cu list] > sweep.jsonl
//
// profiles/r01/kernel_exp_1.jsonl = default table, _2 = XE_SWEEP2 (queue
// chunk size x U x layout), _3 = XE_SWEEP3 (wave-level queues, prefetch,
// per-XCD counters).  Result: one-tile-per-grab workgroup queue with
// wave-contiguous lanes, U = 4, global nt loads (shipped as xor_stream).
//
// Axes: lane layout (lane-interleaved / wave-contiguous), load flavour
// (global nt / buffer loads with cache-policy aux bits), store flavour,
// tile schedule (static contiguous / dynamic atomic chunks / grid-stride),
// load ordering (compiler-interleaved / all loads first), grid size.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                     \
    }                                                                              \
  } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;
constexpr int NSRC = 8;

// gfx94x/gfx950 cache-policy aux bits of buffer instructions: sc0 = 1, nt = 2, sc1 = 16.
enum Ld { LD_GNT = 0, LD_GPLAIN = 1, LD_B = 2 };
enum St { ST_GNT = 0, ST_GPLAIN = 1, ST_B = 2 };

struct Var {
  int layout;   // 0 lane-interleaved, 1 wave-contiguous
  int ld;       // Ld
  int ld_aux;   // for LD_B
  int st;       // St
  int st_aux;   // for ST_B
  int sched;    // 0 static contiguous, 1 dynamic chunks, 2 grid-stride
  int allfirst; // 1: all NSRC*U loads issued before any XOR
};

template <int LAYOUT, int LD, int LDAUX, int ST, int STAUX, int SCHED, int ALLF, int U, int CH>
__global__ __launch_bounds__(kBlock) void xe_kernel(char *__restrict__ dst, const char *__restrict__ src,
                                                    uint32_t vps, uint32_t tps, uint32_t ntiles,
                                                    unsigned *ctr) {
  constexpr uint32_t tile_v = kBlock * U;
  const uint64_t S = (uint64_t)vps * 16;
  __shared__ uint32_t sh_t;
  uint32_t t0, t1;
  if constexpr (SCHED == 0) {
    t0 = (uint32_t)(((uint64_t)blockIdx.x * ntiles) / gridDim.x);
    t1 = (uint32_t)(((uint64_t)(blockIdx.x + 1) * ntiles) / gridDim.x);
  } else {
    t0 = blockIdx.x;
    t1 = ntiles;
  }
  uint32_t t = t0;
  if constexpr (SCHED == 1) {
    if (threadIdx.x == 0) sh_t = atomicAdd(ctr, CH);
    __syncthreads();
    t = sh_t;
    t1 = min(t + CH, ntiles);
  }
  while (t < t1) {
    const uint32_t s = t / tps;
    const uint32_t tin = t - s * tps;
    const char *sb = src + (uint64_t)s * NSRC * S;
    char *db = dst + (uint64_t)s * S;
    uint32_t vin[U];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int u = 0; u < U; u++)
      vin[u] = LAYOUT == 0 ? tin * tile_v + u * kBlock + threadIdx.x : tin * tile_v + wave * 64 * U + u * 64 + lane;
    v4u x[NSRC][U];
    if constexpr (LD == LD_B) {
      __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)sb, (short)0, (int)(NSRC * S), 0x00020000);
#pragma unroll
      for (int k = 0; k < NSRC; k++)
#pragma unroll
        for (int u = 0; u < U; u++) {
          x[k][u] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(vin[u] * 16), (int)(k * S), LDAUX);
        }
    } else {
#pragma unroll
      for (int k = 0; k < NSRC; k++)
#pragma unroll
        for (int u = 0; u < U; u++) {
          const v4u *p = reinterpret_cast<const v4u *>(sb + k * S) + vin[u];
          x[k][u] = LD == LD_GNT ? __builtin_nontemporal_load(p) : *p;
        }
    }
    if constexpr (ALLF) __builtin_amdgcn_sched_barrier(0);
    v4u acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      acc[u] = x[0][u];
#pragma unroll
      for (int k = 1; k < NSRC; k++) acc[u] ^= x[k][u];
    }
    if constexpr (ST == ST_B) {
      __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void *)db, (short)0, (int)S, 0x00020000);
#pragma unroll
      for (int u = 0; u < U; u++) __builtin_amdgcn_raw_buffer_store_b128(acc[u], w, (int)(vin[u] * 16), 0, STAUX);
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) {
        v4u *p = reinterpret_cast<v4u *>(db) + vin[u];
        if constexpr (ST == ST_GNT) __builtin_nontemporal_store(acc[u], p);
        else *p = acc[u];
      }
    }
    if constexpr (SCHED == 0) {
      t++;
    } else if constexpr (SCHED == 2) {
      t += gridDim.x;
    } else {
      t++;
      if (t >= t1) {
        __syncthreads();
        if (threadIdx.x == 0) sh_t = atomicAdd(ctr, CH);
        __syncthreads();
        t = sh_t;
        t1 = min(t + CH, ntiles);
      }
    }
  }
}


// Dynamic tile queue, second generation.  WAVE: each wave pulls its own tile
// (64 lanes x U vectors per source) with no workgroup barrier; otherwise the
// workgroup pulls 256 x U vectors (wave-contiguous).  PF: fetch the next tile
// index while the current one streams.  NCTR: counters (1, or 8 = per XCD
// round-robin, tile = c * NCTR + x).
template <int WAVE, int U, int PF, int NCTR>
__global__ __launch_bounds__(kBlock) void xe_dyn2(char *__restrict__ dst, const char *__restrict__ src,
                                                  uint32_t vps, uint32_t tps, uint32_t ntiles, unsigned *ctr) {
  const uint64_t S = (uint64_t)vps * 16;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr uint32_t tile_v = (WAVE ? 64 : kBlock) * U;
  const uint32_t x = NCTR > 1 ? blockIdx.x % NCTR : 0;
  unsigned *my = ctr + x * 32;  // 128 B apart
  __shared__ uint32_t sh[2];
  auto grab = [&]() -> uint32_t {
    uint32_t c;
    if constexpr (WAVE) {
      uint32_t v = 0;
      if (lane == 0) v = atomicAdd(my, 1u);
      c = __builtin_amdgcn_readfirstlane(v);
    } else {
      c = 0;  // filled by caller via LDS
    }
    return c * NCTR + x;
  };
  uint32_t t, tn = 0;
  int slot = 0;
  if constexpr (WAVE) {
    t = grab();
    if (PF) tn = grab();
  } else {
    if (threadIdx.x == 0) sh[0] = atomicAdd(my, 1u) * NCTR + x;
    __syncthreads();
    t = sh[0];
  }
  while (t < ntiles) {
    uint32_t pending = 0;
    if (!WAVE && PF && threadIdx.x == 0) pending = atomicAdd(my, 1u) * NCTR + x;  // next tile, in flight
    const uint32_t s = t / tps;
    const uint32_t tin = t - s * tps;
    const char *sb = src + (uint64_t)s * NSRC * S;
    char *db = dst + (uint64_t)s * S;
    const uint32_t vb = WAVE ? tin * tile_v + lane : tin * tile_v + wave * 64 * U + lane;
    v4u x_[NSRC][U];
#pragma unroll
    for (int k = 0; k < NSRC; k++)
#pragma unroll
      for (int u = 0; u < U; u++)
        x_[k][u] = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(sb + k * S) + vb + u * 64);
    v4u acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      acc[u] = x_[0][u];
#pragma unroll
      for (int k = 1; k < NSRC; k++) acc[u] ^= x_[k][u];
    }
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_nontemporal_store(acc[u], reinterpret_cast<v4u *>(db) + vb + u * 64);
    if constexpr (WAVE) {
      if (PF) { t = tn; tn = grab(); }
      else t = grab();
    } else {
      if (PF) {
        // two slots: the write of iteration i+1 never races the reads of iteration i.
        slot ^= 1;
        if (threadIdx.x == 0) sh[slot] = pending;
        __syncthreads();
        t = sh[slot];
      } else {
        __syncthreads();
        if (threadIdx.x == 0) sh[0] = atomicAdd(my, 1u) * NCTR + x;
        __syncthreads();
        t = sh[0];
      }
    }
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

typedef void (*KFn)(char *, const char *, uint32_t, uint32_t, uint32_t, unsigned *);

struct Entry {
  const char *name;
  KFn fn;
  int sched;
  int u;
  int wave;  // 1: tiles are per wave (64 x U vectors)
};

#define E(name, L, LD, LA, ST, SA, SC, AF) {name, xe_kernel<L, LD, LA, ST, SA, SC, AF, 4, 4>, SC, 4, 0}
#define D(name, L, LD, LA, U, CH) {name, xe_kernel<L, LD, LA, ST_GNT, 0, 1, 0, U, CH>, 1, U, 0}
#define D2(name, W, U, PF, NC) {name, xe_dyn2<W, U, PF, NC>, 1, U, W}
static const Entry kVariants[] = {
#if defined(XE_SWEEP3)
    E("base", 0, LD_GNT, 0, ST_GNT, 0, 0, 0),
    D("dyn_w_g_u4_c1", 1, LD_GNT, 0, 4, 1),
    D2("d2_wg_u4", 0, 4, 0, 1),
    D2("d2_wg_u4_pf", 0, 4, 1, 1),
    D2("d2_wg_u4_x8", 0, 4, 0, 8),
    D2("d2_wg_u4_pf_x8", 0, 4, 1, 8),
    D2("d2_wg_u2_pf", 0, 2, 1, 1),
    D2("d2_wv_u4", 1, 4, 0, 1),
    D2("d2_wv_u4_pf", 1, 4, 1, 1),
    D2("d2_wv_u8", 1, 8, 0, 1),
    D2("d2_wv_u8_pf", 1, 8, 1, 1),
    D2("d2_wv_u16_pf", 1, 16, 1, 1),
    D2("d2_wv_u8_pf_x8", 1, 8, 1, 8),
    D2("d2_wv_u4_pf_x8", 1, 4, 1, 8),
    D2("d2_wv_u16_pf_x8", 1, 16, 1, 8),
#elif defined(XE_SWEEP2)
    E("base", 0, LD_GNT, 0, ST_GNT, 0, 0, 0),
    D("dyn_l_g_u4_c1", 0, LD_GNT, 0, 4, 1),
    D("dyn_l_g_u4_c2", 0, LD_GNT, 0, 4, 2),
    D("dyn_l_g_u4_c4", 0, LD_GNT, 0, 4, 4),
    D("dyn_l_g_u4_c8", 0, LD_GNT, 0, 4, 8),
    D("dyn_l_g_u4_c16", 0, LD_GNT, 0, 4, 16),
    D("dyn_w_g_u4_c1", 1, LD_GNT, 0, 4, 1),
    D("dyn_w_g_u4_c2", 1, LD_GNT, 0, 4, 2),
    D("dyn_w_g_u4_c4", 1, LD_GNT, 0, 4, 4),
    D("dyn_w_g_u4_c8", 1, LD_GNT, 0, 4, 8),
    D("dyn_w_g_u4_c16", 1, LD_GNT, 0, 4, 16),
    D("dyn_w_b_u4_c1", 1, LD_B, 2, 4, 1),
    D("dyn_w_b_u4_c2", 1, LD_B, 2, 4, 2),
    D("dyn_w_b_u4_c4", 1, LD_B, 2, 4, 4),
    D("dyn_w_b_u4_c8", 1, LD_B, 2, 4, 8),
    D("dyn_w_b_u4_c16", 1, LD_B, 2, 4, 16),
    D("dyn_l_b_u4_c4", 0, LD_B, 2, 4, 4),
    D("dyn_w_b_u2_c2", 1, LD_B, 2, 2, 2),
    D("dyn_w_b_u2_c4", 1, LD_B, 2, 2, 4),
    D("dyn_w_b_u2_c8", 1, LD_B, 2, 2, 8),
    D("dyn_w_b_u8_c1", 1, LD_B, 2, 8, 1),
    D("dyn_w_b_u8_c2", 1, LD_B, 2, 8, 2),
    D("dyn_w_b_u8_c4", 1, LD_B, 2, 8, 4),
    D("dyn_w_g_u8_c2", 1, LD_GNT, 0, 8, 2),
    D("dyn_w_b_u1_c8", 1, LD_B, 2, 1, 8),
    D("dyn_w_b_u1_c16", 1, LD_B, 2, 1, 16),
#else
    E("base", 0, LD_GNT, 0, ST_GNT, 0, 0, 0),
    E("wavecontig", 1, LD_GNT, 0, ST_GNT, 0, 0, 0),
    E("allfirst", 0, LD_GNT, 0, ST_GNT, 0, 0, 1),
    E("dyn", 0, LD_GNT, 0, ST_GNT, 0, 1, 0),
    E("gridstride", 0, LD_GNT, 0, ST_GNT, 0, 2, 0),
    E("bld_nt", 0, LD_B, 2, ST_GNT, 0, 0, 0),
    E("bld_plain", 0, LD_B, 0, ST_GNT, 0, 0, 0),
    E("bld_sc1", 0, LD_B, 16, ST_GNT, 0, 0, 0),
    E("bld_sc0sc1", 0, LD_B, 17, ST_GNT, 0, 0, 0),
    E("bld_sc1nt", 0, LD_B, 18, ST_GNT, 0, 0, 0),
    E("bst_nt", 0, LD_GNT, 0, ST_B, 2, 0, 0),
    E("bst_sc1", 0, LD_GNT, 0, ST_B, 16, 0, 0),
    E("bst_sc0sc1", 0, LD_GNT, 0, ST_B, 17, 0, 0),
    E("bst_sc0sc1nt", 0, LD_GNT, 0, ST_B, 19, 0, 0),
    E("gst_plain", 0, LD_GNT, 0, ST_GPLAIN, 0, 0, 0),
    E("bld_nt_allfirst", 0, LD_B, 2, ST_GNT, 0, 0, 1),
    E("wave_bld_nt_dyn", 1, LD_B, 2, ST_GNT, 0, 1, 0),
    E("wave_dyn", 1, LD_GNT, 0, ST_GNT, 0, 1, 0),
#endif
};
#undef E

int main(int argc, char **argv) {
  const uint64_t stripes = argc > 1 ? strtoull(argv[1], 0, 10) : 12500;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const char *bpc_list = argc > 3 ? argv[3] : "7,8,14,16";
  const uint64_t S = 512 * 1024;
  const uint64_t in_bytes = stripes * NSRC * S, out_bytes = stripes * S;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  char *src, *dst, *ref;
  unsigned *ctr;
  unsigned long long *dcount;
  CK(hipMalloc(&src, in_bytes));
  CK(hipMalloc(&dst, out_bytes));
  CK(hipMalloc(&ref, out_bytes));
  CK(hipMalloc(&ctr, 8 * 128));
  CK(hipMalloc(&dcount, 8));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipLaunchKernelGGL(fill, dim3(cus * 8), dim3(256), 0, st, (uint64_t *)src, in_bytes / 8, 1ull);
  const uint32_t vps = S / 16;
  std::vector<int> bpcs;
  for (const char *p = bpc_list; *p;) {
    bpcs.push_back(atoi(p));
    while (*p && *p != ',') p++;
    if (*p) p++;
  }
  const int nv = sizeof(kVariants) / sizeof(kVariants[0]);
  auto launch = [&](int v, int grid, char *out) {
    const uint32_t tps = vps / ((kVariants[v].wave ? 64 : kBlock) * kVariants[v].u);
    const uint32_t ntiles = (uint32_t)(stripes * tps);
    if (kVariants[v].sched == 1) CK(hipMemsetAsync(ctr, 0, 8 * 128, st));
    if (kVariants[v].sched == 1) grid = std::min<int>(grid, ntiles);
    hipLaunchKernelGGL(kVariants[v].fn, dim3(grid), dim3(kBlock), 0, st, out, src, vps, tps, ntiles, ctr);
    CK(hipGetLastError());
  };
  launch(0, cus * 16, ref);
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = (double)stripes * (NSRC + 1) * S;
  std::vector<std::vector<float>> times((size_t)nv * bpcs.size());
  std::vector<long long> bad((size_t)nv * bpcs.size(), -1);
  for (int r = 0; r < reps; r++) {
    for (int v = 0; v < nv; v++)
      for (size_t b = 0; b < bpcs.size(); b++) {
        const int grid = cus * bpcs[b];
        launch(v, grid, dst);  // warm
        CK(hipEventRecord(e0, st));
        launch(v, grid, dst);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        times[v * bpcs.size() + b].push_back(ms);
        if (r == 0) {
          CK(hipMemsetAsync(dcount, 0, 8, st));
          hipLaunchKernelGGL(diff, dim3(cus * 4), dim3(256), 0, st, (const uint64_t *)dst, (const uint64_t *)ref,
                             out_bytes / 8, dcount);
          unsigned long long h;
          CK(hipMemcpyAsync(&h, dcount, 8, hipMemcpyDeviceToHost, st));
          CK(hipStreamSynchronize(st));
          bad[v * bpcs.size() + b] = (long long)h;
          CK(hipMemsetAsync(dst, 0, out_bytes, st));
        }
      }
    fprintf(stderr, "rep %d/%d done\n", r + 1, reps);
  }
  for (int v = 0; v < nv; v++)
    for (size_t b = 0; b < bpcs.size(); b++) {
      auto ts = times[v * bpcs.size() + b];
      std::sort(ts.begin(), ts.end());
      const float med = ts[ts.size() / 2];
      printf("{\"variant\": \"%s\", \"blocks_per_cu\": %d, \"median_ms\": %.4f, \"min_ms\": %.4f, "
             "\"GBps\": %.1f, \"frac_8TBs\": %.4f, \"mismatch_words\": %lld}\n",
             kVariants[v].name, bpcs[b], med, ts[0], bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12,
             bad[v * bpcs.size() + b]);
    }
  return 0;
}
