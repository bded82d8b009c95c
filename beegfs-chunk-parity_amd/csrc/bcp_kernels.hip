// bcp_kernels.hip -- CDNA4 (gfx950) kernels of the chunk-XOR parity engine.
//
// The arithmetic is the reference's xor_parity
// (src/beegfs-raid5/common/task_processing.c:96-109): out = XOR of N source
// chunks, zero-padded to the output length.  It is a read-once integer stream
// (N loads + 1 store per output byte, no reuse), so the design rules are the
// HBM ones: 16-byte lanes (global_load_dwordx4), every source load of a lane
// issued before the XORs, non-temporal hints so the 8:1 read stream does not
// churn L2/MALL, and a device-wide tile queue that keeps the chip's loads in
// one narrow ascending address window.
//
// Kernels:
//   xor_stream<NSRC,U,GATHER>  uniform stripes, 16-B aligned geometry (hot path;
//                              strided or pointer-table addressing)
//   xor_desc<U>               descriptor batches: variable lengths, zero pad,
//                             rebuild truncation, window replay, any alignment
//   fill_synthetic / xor_fold / compare   synthetic inputs and verification
#include "bcp_internal.h"

namespace bcp {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef v4u v4u_u __attribute__((aligned(1)));  // unaligned 16-byte view

template <typename T>
__device__ __forceinline__ v4u ld_nt(const T *p) { return __builtin_nontemporal_load(p); }

// Descriptor tables (stripes, sources, tile prefixes) are never written while
// a kernel runs.  Reading them through the constant address space lets the
// compiler use scalar loads (s_load, own lgkm counter) for the uniform
// indices; through a generic pointer they become vector loads whose
// s_waitcnt vmcnt(0) drains the data loads in flight on every tile.
template <typename T>
using const_as = const __attribute__((address_space(4))) T;
template <typename T>
__device__ __forceinline__ const_as<T> *cst(const T *p) {
  return (const_as<T> *)(uintptr_t)p;
}

// Data pointers taken from descriptor tables are plain integers; without an
// address space the compiler emits flat loads, which also count on lgkmcnt,
// so every scalar-load wait would drain the whole data stream.  Cast them to
// the global address space.
template <typename T>
using glob = __attribute__((address_space(1))) T;
template <typename T>
__device__ __forceinline__ glob<T> *gp(uint64_t p) {
  return (glob<T> *)(uintptr_t)p;
}
__device__ __forceinline__ v4u zero4() { return v4u{0u, 0u, 0u, 0u}; }

// 16 bytes of source `p` (readable length len) at offset off, zero past len.
typedef glob<const unsigned char> gbyte;
__device__ __forceinline__ v4u ld16(gbyte *p) { return __builtin_nontemporal_load((const glob<v4u_u> *)p); }

// The one vector of a source that straddles its end: n (1..15) readable bytes
// at p, zeros after.  Static byte indices keep w[] in registers.
__device__ __forceinline__ v4u load_straddle(gbyte *p, uint32_t n) {
  unsigned int w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (uint32_t i = 0; i < 16; i++)
    if (i < n) w[i >> 2] |= (unsigned int)p[i] << (8 * (i & 3));
  return v4u{w[0], w[1], w[2], w[3]};
}


// ---------------------------------------------------------------------------
// Streaming fold (hot path).  A tile is kBlock*U 16-byte vectors of one
// stripe's output (32 KiB at the default U = 8, one 256-thread workgroup per
// CU); wave w of the workgroup owns the contiguous run [w*64*U, (w+1)*64*U)
// of the tile, lane l vectors l, l+64, ... so each wave streams 8 KiB
// contiguous per source and every NSRC*U load of a lane is independent of the
// others.
//
// Tile schedule (r01 sweeps, profiles/r01/kernel_exp_*.jsonl): a device-wide
// work queue.  Thread 0 of a workgroup takes the next tile index with one
// atomic per tile, so the tiles in flight on the whole chip are always a
// narrow, ascending address window (~16 stripes at config 2).  It beat
// per-workgroup contiguous tile runs by 12-14 % and a grid-stride schedule by
// 10 points on the same box (exp 1-3, 9).
// The counter is monotone: launch k starts at `base`, every tile index
// handed out is atomicAdd(ctr, 1) - base, and each workgroup makes exactly one
// failing grab, so a launch consumes ntiles + grid counts and the host
// advances base by that (no reset between launches).
//
// Addressing: GATHER = 0 -> source k of stripe s at src + s*stripe_stride +
// k*src_stride, output at dst + s*dst_stride.  GATHER = 1 -> pointers from a
// descriptor batch whose stripes are uniform (same nsrc, out_len, every
// source at least out_len long, all 16-byte aligned) -- the rebuild shape.
// NSRC == 0 means "runtime nsrc".
// ---------------------------------------------------------------------------
template <int U>
__device__ __forceinline__ uint32_t tile_vec(uint32_t tin, int u) {
  return tin * (uint32_t)(kBlock * U) + (threadIdx.x >> 6) * (64u * U) + (uint32_t)u * 64u + (threadIdx.x & 63u);
}

// Rolling load window of the descriptor kernel's covering-source fold
// (PIPE > 0: xor_desc_p<U, 5>, the shipped form at U = 8 and 16).  Folds G
// sources x U vectors per lane into acc, issuing the loads as units of H =
// U/4 vectors with D = 5 units in flight: unit j + D - 1 goes out before unit
// j is XORed, and sched_barrier keeps the compiler from hoisting every load
// of the tile above the XORs (which it does when the kernel runs at one wave
// per SIMD anyway), so (D - 1) * H .. D * H loads per lane are outstanding.
// Every load of a tile in flight at once widens the chip's address window and
// costs HBM rate: the window is +1.3 points on config-5 shapes, +1.8 on
// config-2 shapes through xor_desc, and on tiles with more than 8 sources
// (desc_tile_wide) 16-wide stripes 69 -> 81 % (profiles/r01/depth/; the other
// unit shapes measured there -- H = U, U/2, U/8 with D = 2..5 -- lost and are
// gone).  Grouped tiles keep all their <= 32 loads in flight: a window there
// cost 1.4 points (depth/ab3_group_window_probe.jsonl); the same window in
// xor_stream measured 2 points below the compiler's own schedule.
template <int U, int PIPE>
struct PipeShape {
  static_assert(PIPE == 5, "one rolling-window shape");
  static constexpr int H = U >= 4 ? U / 4 : 1;
  static constexpr int D = 5;
};

template <int G, int U, int PIPE, typename V, typename F>
__device__ __forceinline__ void rolling_fold(v4u (&acc)[U], F base) {
  constexpr int H = PipeShape<U, PIPE>::H, D = PipeShape<U, PIPE>::D;
  constexpr int UPS = U / H;  // units per source
  constexpr int NU = G * UPS;
  v4u x[D][H];
#pragma unroll
  for (int j = 0; j < D - 1 && j < NU; j++) {
    const glob<V> *p = base(j / UPS);
#pragma unroll
    for (int h = 0; h < H; h++) x[j % D][h] = __builtin_nontemporal_load(p + ((j % UPS) * H + h) * 64);
  }
#pragma unroll
  for (int j = 0; j < NU; j++) {
    if (j + D - 1 < NU) {
      const int jn = j + D - 1;
      const glob<V> *p = base(jn / UPS);
#pragma unroll
      for (int h = 0; h < H; h++) x[jn % D][h] = __builtin_nontemporal_load(p + ((jn % UPS) * H + h) * 64);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < H; h++) acc[(j % UPS) * H + h] ^= x[j % D][h];
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int NSRC, int U, int GATHER, bool PARTIAL>
__device__ __forceinline__ void stream_tile(const StreamArgs &a, uint32_t t) {
  const uint32_t nsrc = NSRC > 0 ? (uint32_t)NSRC : a.nsrc;
  const uint32_t s = t / a.tps;
  const uint32_t tin = t - s * a.tps;
  uint64_t sb = 0;
  const_as<bcp_source> *sl = nullptr;
  glob<v4u> *db;
  if constexpr (GATHER) {
    // Dense batches (first_src == s * nsrc, the usual layout) need no
    // dependent load of first_src: both table reads go out together.
    const_as<bcp_stripe> *ds = cst(a.stripes) + s;
    sl = cst(a.sources) + (a.dense ? s * nsrc : ds->first_src);
    db = gp<v4u>(ds->dst);
  } else {
    sb = (uint64_t)(uintptr_t)a.src + (uint64_t)s * a.stripe_stride;
    db = gp<v4u>((uint64_t)(uintptr_t)a.dst + (uint64_t)s * a.dst_stride);
  }
  auto src_k = [&](uint32_t k) -> const glob<v4u> * {
    if constexpr (GATHER) return gp<v4u>(sl[k].ptr);
    else return gp<v4u>(sb + (uint64_t)k * a.src_stride);
  };
  v4u acc[U];
  if (!PARTIAL || (tin + 1) * (uint32_t)(kBlock * U) <= a.vps) {
    const uint32_t vb = tile_vec<U>(tin, 0);
    if constexpr (NSRC > 0) {
      // Every load of the tile first, then the XOR tree: the compiler keeps
      // the scheduling freedom (fewer VGPRs than an interleaved chain).
      v4u x[NSRC][U];
#pragma unroll
      for (int k = 0; k < NSRC; k++) {
        const glob<v4u> *pk = src_k(k) + vb;
#pragma unroll
        for (int u = 0; u < U; u++) x[k][u] = ld_nt(pk + u * 64);
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        acc[u] = x[0][u];
#pragma unroll
        for (int k = 1; k < NSRC; k++) acc[u] ^= x[k][u];
      }
    } else {
      const glob<v4u> *p0 = src_k(0) + vb;
#pragma unroll
      for (int u = 0; u < U; u++) acc[u] = ld_nt(p0 + u * 64);
#pragma unroll 4
      for (uint32_t k = 1; k < nsrc; k++) {
        const glob<v4u> *pk = src_k(k) + vb;
#pragma unroll
        for (int u = 0; u < U; u++) acc[u] ^= ld_nt(pk + u * 64);
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_nontemporal_store(acc[u], db + vb + u * 64);
  } else if constexpr (PARTIAL) {
    // Last, partial tile of a stripe: per-vector bounds (masked loads, all
    // issued before the XORs when the width is known); the byte tail (a
    // chunk length that is not a multiple of 16) in the lane that owns it.
    if constexpr (NSRC > 0) {
      v4u x[NSRC][U];
#pragma unroll
      for (int k = 0; k < NSRC; k++)
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t v = tile_vec<U>(tin, u);
          x[k][u] = v < a.vps ? ld_nt(src_k(k) + v) : zero4();
        }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t v = tile_vec<U>(tin, u);
        v4u acc = x[0][u];
#pragma unroll
        for (int k = 1; k < NSRC; k++) acc ^= x[k][u];
        if (v < a.vps) __builtin_nontemporal_store(acc, db + v);
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t v = tile_vec<U>(tin, u);
      if (NSRC == 0 && v < a.vps) {
        v4u x = ld_nt(src_k(0) + v);
        for (uint32_t k = 1; k < nsrc; k++) x ^= ld_nt(src_k(k) + v);
        __builtin_nontemporal_store(x, db + v);
      } else if (v == a.vps && a.tail) {
        v4u x = zero4();
        for (uint32_t k = 0; k < nsrc; k++)
          x ^= load_straddle((gbyte *)(src_k(k) + v), a.tail);
        glob<unsigned char> *d = (glob<unsigned char> *)(db + v);
        for (uint32_t i = 0; i < a.tail; i++) d[i] = (unsigned char)(x[i >> 2] >> (8 * (i & 3)));
      }
    }
  }
}

__device__ __forceinline__ uint32_t queue_grab(unsigned long long *ctr, unsigned long long base) {
  const unsigned long long v = atomicAdd(ctr, 1ull) - base;
  return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)v;
}

// KIND: kQueueFull (every tile full: the config-2 shapes), kQueuePartial
// (stripes end in a partial tile).  Separate instantiations because the
// partial-tile code path costs ~15-25 VGPRs at U = 8 even when never taken.
// (r01's static schedule -- a contiguous tile range per workgroup -- lost to
// the work queue by 12-14 % and is gone.)
constexpr int kQueueFull = 0, kQueuePartial = 1;

template <int NSRC, int U, int GATHER, int KIND>
__device__ __forceinline__ void stream_body(const StreamArgs &a) {
  constexpr bool PARTIAL = KIND != kQueueFull;
  // Two LDS slots: thread 0 writes slot i+1 only after the barrier that
  // every wave reaches after reading slot i, so one barrier per tile is enough.
  __shared__ uint32_t next[2];
  if (threadIdx.x == 0) next[0] = queue_grab(a.ctr, a.base);
  __syncthreads();
  uint32_t t = __builtin_amdgcn_readfirstlane(next[0]);
  int slot = 0;
  if constexpr (NSRC >= 1 && NSRC <= 4) {
    // Narrow stripes: a.grab consecutive tiles per queue grab (a tile moves
    // only (NSRC + 1) x 32 KiB at U = 8, and one counter serves ~60-80
    // grabs per microsecond: at one tile per grab, N = 1..2 are
    // counter-bound).
    const uint32_t g = a.grab ? a.grab : 1u;  // the host always sets >= 1; never divide by 0
    const uint32_t nunits = (a.ntiles + g - 1) / g;
    while (t < nunits) {
      const uint32_t t0 = t * g, t1 = min(t0 + g, a.ntiles);
      for (uint32_t x = t0; x < t1; x++) stream_tile<NSRC, U, GATHER, PARTIAL>(a, x);
      slot ^= 1;
      if (threadIdx.x == 0) next[slot] = queue_grab(a.ctr, a.base);
      __syncthreads();
      t = __builtin_amdgcn_readfirstlane(next[slot]);
    }
  } else {
    while (t < a.ntiles) {
      stream_tile<NSRC, U, GATHER, PARTIAL>(a, t);
      slot ^= 1;
      if (threadIdx.x == 0) next[slot] = queue_grab(a.ctr, a.base);
      __syncthreads();
      t = __builtin_amdgcn_readfirstlane(next[slot]);
    }
  }
}

template <int NSRC, int U, int GATHER, int KIND>
__global__ __launch_bounds__(kBlock) void xor_stream(StreamArgs a) {
  stream_body<NSRC, U, GATHER, KIND>(a);
}

// The same kernel with a register budget of W waves per SIMD
// (amdgpu_waves_per_eu; W = 6 where it won, launch_xor_stream).  The body says "every
// load of the tile first"; the compiler software-pipelines it into the
// budget it aims for, so W sets how many loads per lane stay in flight: no
// budget (its own occupancy target) ~5-9, W = 6 ~14, W = 7 8, W = 1-2 ~43.
// On config 2, W = 6 is +0.8..1.0 point over no budget in three separate
// interleaved A/Bs, W = 7 -2.6, W = 5 -1.3, W <= 4 -1.5..-2.5
// (tools/exp/xor_exp5.hip, profiles/r01/depth/); the pointer-table form
// (rebuild) measured neutral, so only the strided form takes it.
template <int NSRC, int U, int GATHER, int KIND, int W>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W, W))) void xor_stream_w(StreamArgs a) {
  stream_body<NSRC, U, GATHER, KIND>(a);
}

// ---------------------------------------------------------------------------
// Descriptor path helpers.
// ---------------------------------------------------------------------------

__device__ __forceinline__ v4u load_src_tail(gbyte *p, uint64_t len, uint64_t off) {
  if (off + 16 <= len) return ld16(p + off);
  if (off >= len) return zero4();
  return load_straddle(p + off, (uint32_t)(len - off));
}

// Offset inside a source after the reference's window replay (quirk A3-q1):
// a source whose last readable window is lw re-sends window lw for every later
// window w (chunk_sender does not refill its buffer once data_sent >= fd_size,
// task_processing.c:291-308).
__device__ __forceinline__ uint64_t replay_offset(uint64_t j, uint64_t len, uint64_t window) {
  if (len == 0) return j;  // reads as zeros anyway
  const uint64_t w = j / window;
  const uint64_t lw = (len - 1) / window;
  return w > lw ? j - (w - lw) * window : j;
}

__device__ __forceinline__ void store_tail(glob<unsigned char> *d, uint64_t out_len, uint64_t off, v4u v) {
  if (off + 16 <= out_len) {
    __builtin_nontemporal_store(v, (glob<v4u_u> *)(d + off));
    return;
  }
  if (off >= out_len) return;
  const uint32_t n = (uint32_t)(out_len - off);
#pragma unroll
  for (uint32_t i = 0; i < 16; i++)
    if (i < n) d[off + i] = (unsigned char)(v[i >> 2] >> (8 * (i & 3)));
}

// ---------------------------------------------------------------------------
// Descriptor kernel.  Tiles of tile_bytes output bytes are numbered across the
// batch (tile_start prefix) and handed out by the same work queue as
// xor_stream, one tile per grab.  A small setup kernel (desc_tiles) first writes one 16-byte
// record per tile (stripe, tile index, coverage counts, source run), so a
// tile costs one scalar load before its stripe and source loads, instead of a
// search over tile_start.  Lanes are wave-contiguous as in xor_stream.  Per
// tile and per source the coverage test is uniform: a source either covers
// the whole tile, misses it (skipped: zero padding), or ends inside it
// (per-lane tail path).  The staged source runs are sorted longest first, so
// the covering sources are a prefix of the run and are folded by one fully
// unrolled fold_cover<G> (G = how many cover, up to 8 at a time).
// Window-replay stripes take the per-lane path for every source.
// ---------------------------------------------------------------------------
// G sources that all cover the tile: every load first, then the XOR tree
// (the xor_stream pattern).  One base address per source and immediate
// offsets per vector: a 64-bit address per load would cost 2 VGPRs each.
template <int G, int U, int PIPE = 0, typename P>
__device__ __forceinline__ void fold_cover(v4u (&acc)[U], P src, uint32_t lane_off) {
  if constexpr (PIPE > 0 && G > 1) {
    rolling_fold<G, U, PIPE, v4u_u>(acc, [&](int i) { return gp<const v4u_u>(src[i] + lane_off); });
    return;
  }
  v4u x[G][U];
#pragma unroll
  for (int i = 0; i < G; i++) {
    const glob<v4u_u> *p = gp<const v4u_u>(src[i] + lane_off);
#pragma unroll
    for (int u = 0; u < U; u++) x[i][u] = __builtin_nontemporal_load(p + u * 64);
  }
#pragma unroll
  for (int u = 0; u < U; u++)
#pragma unroll
    for (int i = 0; i < G; i++) acc[u] ^= x[i][u];
}

// Grouped tile: M consecutive full subtiles, each the XOR of the same C
// covering sources.  Every load of the tile first (C*M*U per lane, at most
// 32: group_rows), then the XORs and the M subtiles' stores.  (Written per
// subtile instead, the loads of subtile j+1 cannot move above the stores of
// subtile j -- the compiler cannot rule out aliasing -- and each subtile
// drains the pipe: config-5 shapes 78 -> 70 %.)
template <int C, int M, int U, typename RT>
__device__ __forceinline__ void fold_group(const RT &r, uint32_t lane_off) {
  constexpr uint32_t T = (uint32_t)kBlock * U * 16u;  // == b.tile_bytes
  v4u x[C][M][U];
#pragma unroll
  for (int i = 0; i < C; i++) {
    const glob<v4u_u> *p = gp<const v4u_u>(r.src[i] + lane_off);
#pragma unroll
    for (int j = 0; j < M; j++)
#pragma unroll
      for (int u = 0; u < U; u++) x[i][j][u] = __builtin_nontemporal_load(p + j * (T / 16) + u * 64);
  }
  glob<v4u_u> *q = gp<v4u_u>(r.dst + lane_off);
#pragma unroll
  for (int j = 0; j < M; j++)
#pragma unroll
    for (int u = 0; u < U; u++) {
      v4u a = x[0][j][u];
#pragma unroll
      for (int i = 1; i < C; i++) a ^= x[i][j][u];
      __builtin_nontemporal_store(a, q + j * (T / 16) + u * 64);
    }
}

// General tile: window replay (quirk A3-q1; only when max_cs exceeds the
// transfer window) or more than kTileSrcs sources reaching in.  Each output
// vector on its own through the stripe/source tables; rare, so compact.
template <int U>
__device__ __noinline__ void desc_tile_general(const DescBatch &b, uint32_t stripe, uint32_t tile,
                                               uint32_t first_src) {
  const_as<bcp_stripe> *dp_ = cst(b.stripes) + stripe;
  const_as<bcp_source> *srcs = cst(b.sources) + first_src;
  const uint32_t nsrc = dp_->nsrc;
  const uint64_t out_len = dp_->out_len, window = dp_->window;
  glob<unsigned char> *dp = gp<unsigned char>(dp_->dst);
  const uint64_t lane_off = (uint64_t)tile * b.tile_bytes +
                            (uint64_t)((threadIdx.x >> 6) * (64u * U) + (threadIdx.x & 63u)) * 16u;
#pragma unroll 1
  for (int u = 0; u < U; u++) {
    const uint64_t off = lane_off + (uint64_t)u * 1024u;
    if (off >= out_len) break;
    v4u x = zero4();
    for (uint32_t k = 0; k < nsrc; k++) {
      const uint64_t len = srcs[k].len;
      const uint64_t o = window ? replay_offset(off, len, window) : off;
      x ^= load_src_tail(gp<const unsigned char>(srcs[k].ptr), len, o);
    }
    store_tail(dp, out_len, off, x);
  }
}

// Source addresses of a staged run, offset to a tile (fold_cover's src[i]).
struct RunAt {
  const_as<bcp_source> *s;
  uint64_t off;
  __device__ __forceinline__ uint64_t operator[](int i) const { return s[i].ptr + off; }
};

// Wide tile: more than kTileSrcs sources reach into it (stripes wider than 8,
// up to BCP_MAX_SOURCES).  The record cannot list them, so they come from the
// staged run (sorted longest first: [0, nfull) cover, [nfull, nany) end
// inside): covering sources eight at a time through fold_cover, then the
// partial ones, as in the plain path.
template <int U, int PIPE>
__device__ __noinline__ void desc_tile_wide(const DescBatch &b, uint32_t stripe, uint32_t sub, uint32_t first_src,
                                            uint32_t nfull, uint32_t nany) {
  constexpr int WP = PIPE;  // the window also over the eight-at-a-time covering folds
  const_as<bcp_stripe> *dp_ = cst(b.stripes) + stripe;
  const_as<bcp_source> *srcs = cst(b.sources) + first_src;
  const uint64_t tile_off = (uint64_t)sub * b.tile_bytes;
  const uint32_t lane_off = ((threadIdx.x >> 6) * (64u * U) + (threadIdx.x & 63u)) * 16u;
  v4u acc[U];
#pragma unroll
  for (int u = 0; u < U; u++) acc[u] = zero4();
  uint32_t k = 0;
  for (; k + 8 <= nfull; k += 8) fold_cover<8, U, WP>(acc, RunAt{srcs + k, tile_off}, lane_off);
  const RunAt rest{srcs + k, tile_off};
  switch (nfull - k) {
    case 7: fold_cover<7, U, WP>(acc, rest, lane_off); break;
    case 6: fold_cover<6, U, WP>(acc, rest, lane_off); break;
    case 5: fold_cover<5, U, WP>(acc, rest, lane_off); break;
    case 4: fold_cover<4, U, WP>(acc, rest, lane_off); break;
    case 3: fold_cover<3, U, WP>(acc, rest, lane_off); break;
    case 2: fold_cover<2, U, WP>(acc, rest, lane_off); break;
    case 1: fold_cover<1, U, WP>(acc, rest, lane_off); break;
    default: break;
  }
  for (k = nfull; k < nany; k++) {
    gbyte *p = gp<const unsigned char>(srcs[k].ptr + tile_off);
    const uint64_t len = srcs[k].len - tile_off;  // < tile_bytes: ends inside the tile
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] ^= load_src_tail(p, len, lane_off + u * 1024u);
  }
  const uint64_t out_len = dp_->out_len;
  glob<unsigned char> *dp = gp<unsigned char>(dp_->dst + tile_off);
  if (tile_off + b.tile_bytes <= out_len) {
    glob<v4u_u> *q = (glob<v4u_u> *)(dp + lane_off);
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_nontemporal_store(acc[u], q + u * 64);
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) store_tail(dp, out_len - tile_off, lane_off + u * 1024u, acc[u]);
  }
}

// One plain or grouped tile from its record r: any type with the DescTile
// members (the device-written record read through the constant address
// space, or the register view of xor_desc_args).  tile_bytes = kBlock*U*16.
template <int U, int PIPE, typename RT>
__device__ __forceinline__ void desc_plain(const RT &r, uint32_t tile_bytes) {
  const uint32_t meta = r.meta;
  // this lane's vector u = 0 inside the tile; vector u is at + u * 1024
  const uint32_t lane_off = ((threadIdx.x >> 6) * (64u * U) + (threadIdx.x & 63u)) * 16u;
  const uint32_t nfull = meta & 0xFFu, nany = (meta >> 8) & 0xFFu;
  const uint32_t m = ((meta >> 16) & 0xFFu) + 1u;
  if (m > 1) {
    switch (nfull << 4 | m) {
#define BCP_GROUP(c, mm) \
  case (c << 4 | mm):                                                 \
    if constexpr (c * mm <= group_rows(U)) {                           \
      fold_group<c, mm, U>(r, lane_off);                               \
      return;                                                          \
    }                                                                  \
    break;
      BCP_GROUP(1, 2) BCP_GROUP(1, 3) BCP_GROUP(1, 4) BCP_GROUP(1, 5) BCP_GROUP(1, 6) BCP_GROUP(1, 7)
      BCP_GROUP(1, 8) BCP_GROUP(2, 2) BCP_GROUP(2, 3) BCP_GROUP(2, 4) BCP_GROUP(3, 2) BCP_GROUP(4, 2)
#undef BCP_GROUP
      default: break;
    }
    // Shapes desc_tiles does not write for this U (C*M > group_rows(U));
    // correct anyway: one subtile at a time.
    for (uint32_t j = 0; j < m; j++) {
      v4u acc[U];
#pragma unroll
      for (int u = 0; u < U; u++) acc[u] = zero4();
      const uint32_t off = lane_off + j * tile_bytes;
      constexpr int FP = U >= 16 ? PIPE : 0;  // at U = 16 all loads at once would spill
      switch (nfull) {
        case 4: fold_cover<4, U, FP>(acc, r.src, off); break;
        case 3: fold_cover<3, U, FP>(acc, r.src, off); break;
        case 2: fold_cover<2, U, FP>(acc, r.src, off); break;
        default: fold_cover<1, U, FP>(acc, r.src, off); break;
      }
      glob<v4u_u> *q = gp<v4u_u>(r.dst + off);
#pragma unroll
      for (int u = 0; u < U; u++) __builtin_nontemporal_store(acc[u], q + u * 64);
    }
    return;
  }
  v4u acc[U];
#pragma unroll
  for (int u = 0; u < U; u++) acc[u] = zero4();
  switch (nfull) {
    case 8: fold_cover<8, U, PIPE>(acc, r.src, lane_off); break;
    case 7: fold_cover<7, U, PIPE>(acc, r.src, lane_off); break;
    case 6: fold_cover<6, U, PIPE>(acc, r.src, lane_off); break;
    case 5: fold_cover<5, U, PIPE>(acc, r.src, lane_off); break;
    case 4: fold_cover<4, U, PIPE>(acc, r.src, lane_off); break;
    case 3: fold_cover<3, U, PIPE>(acc, r.src, lane_off); break;
    case 2: fold_cover<2, U, PIPE>(acc, r.src, lane_off); break;
    case 1: fold_cover<1, U, PIPE>(acc, r.src, lane_off); break;
    default: break;
  }
  // Sources ending inside the tile: whole vectors below the end as masked
  // loads (no per-lane byte path in the way of the loads), then the one vector
  // that straddles the end, in the lane that owns it.
  for (uint32_t k = nfull; k < nany; k++) {
    gbyte *p = gp<const unsigned char>(r.src[k]);
    const uint32_t len = r.src_bytes[k];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (lane_off + u * 1024u + 16u <= len) acc[u] ^= ld16(p + lane_off + u * 1024u);
  }
  for (uint32_t k = nfull; k < nany; k++) {
    const uint32_t len = r.src_bytes[k];
    if (len & 15u) {
      const uint32_t soff = len & ~15u;  // offset of the straddling vector inside the tile
#pragma unroll
      for (int u = 0; u < U; u++)
        if (lane_off + u * 1024u == soff) acc[u] ^= load_straddle(gp<const unsigned char>(r.src[k]) + soff, len & 15u);
    }
  }
  glob<unsigned char> *dp = gp<unsigned char>(r.dst);
  const uint32_t out_bytes = r.out_bytes;
  if (out_bytes == tile_bytes) {
    glob<v4u_u> *q = (glob<v4u_u> *)(dp + lane_off);
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_nontemporal_store(acc[u], q + u * 64);
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) store_tail(dp, out_bytes, lane_off + u * 1024u, acc[u]);
  }
}

template <int U, int PIPE>
__device__ __forceinline__ void desc_tile(const DescBatch &b, uint32_t t) {
  const_as<DescTile> &r = cst(b.tiles)[t];
  const uint32_t meta = r.meta;
  if (meta & kTileGeneral) {
    if (meta & kTileWide)
      desc_tile_wide<U, PIPE>(b, r.src_bytes[0], r.src_bytes[1], r.src_bytes[2], meta & 0xFFu, (meta >> 8) & 0xFFu);
    else
      desc_tile_general<U>(b, r.src_bytes[0], r.src_bytes[1], r.src_bytes[2]);
    return;
  }
  desc_plain<U, PIPE>(r, b.tile_bytes);
}

template <int U, int PIPE>
__device__ __forceinline__ void desc_body(const DescBatch &b) {
  // Work queue, one tile per grab (two LDS slots as in stream_body).  A
  // grab-ahead form (the next tile taken and its record touched before the
  // current one is folded) measured no gain and is gone.
  __shared__ uint32_t next[2];
  if (threadIdx.x == 0) next[0] = queue_grab(b.ctr, b.base);
  __syncthreads();
  uint32_t t = __builtin_amdgcn_readfirstlane(next[0]);
  int slot = 0;
  while (t < b.ntiles) {
    desc_tile<U, PIPE>(b, t);
    slot ^= 1;
    if (threadIdx.x == 0) next[slot] = queue_grab(b.ctr, b.base);
    __syncthreads();
    t = __builtin_amdgcn_readfirstlane(next[slot]);
  }
}

template <int U>
__global__ __launch_bounds__(kBlock) void xor_desc(DescBatch b) {
  desc_body<U, 0>(b);
}

// The rolling-window form (PipeShape): U = 8 and 16.
template <int U, int PIPE>
__global__ __launch_bounds__(kBlock) void xor_desc_p(DescBatch b) {
  desc_body<U, PIPE>(b);
}

// ---------------------------------------------------------------------------
// Small descriptor batches (a few stripes, <= 8 sources each, no window):
// the whole descriptor travels in the kernel arguments (DescArgs, runs
// sorted longest first) and every tile derives its record in scalar
// registers -- no desc_tiles launch, no staged tables, one launch.  Tiles are
// single subtiles (no grouping: the batch is latency-bound, not byte-bound).
// ---------------------------------------------------------------------------
struct ArgSrc {  // r.src[i]: source i of the stripe's run, offset to the tile
  const_as<uint64_t> *p;
  uint64_t off;
  __device__ __forceinline__ uint64_t operator[](uint32_t i) const { return p[i] + off; }
};
struct ArgLen {  // r.src_bytes[i]: readable bytes of source i inside the tile
  const_as<uint64_t> *len;
  uint64_t off, T;
  __device__ __forceinline__ uint32_t operator[](uint32_t i) const {
    const uint64_t l = len[i] - off;
    return (uint32_t)(l < T ? l : T);
  }
};
struct ArgRec {
  uint64_t dst;
  uint32_t out_bytes, meta;
  ArgSrc src;
  ArgLen src_bytes;
};

template <int U>
__global__ __launch_bounds__(kBlock) void xor_desc_args(DescArgs a) {
  // read in place from the kernarg segment (the only explicit argument, at
  // offset 0): dynamic indices become scalar loads, nothing is copied
  const_as<DescArgs> *A = (const_as<DescArgs> *)__builtin_amdgcn_kernarg_segment_ptr();
  constexpr uint32_t T = (uint32_t)kBlock * U * 16u;
  __shared__ uint32_t next[2];
  if (threadIdx.x == 0) next[0] = queue_grab(a.ctr, a.base);
  __syncthreads();
  uint32_t t = __builtin_amdgcn_readfirstlane(next[0]);
  int slot = 0;
  while (t < a.ntiles) {
    uint32_t s = 0;
    while (s + 1 < a.nstripes && t >= A->tile_start[s + 1]) s++;
    const uint64_t off = (uint64_t)(t - A->tile_start[s]) * T;
    const uint32_t first = A->first[s], n = A->nsrc[s];
    uint32_t nf = 0, na = 0;
    for (uint32_t k = 0; k < n; k++) {
      const uint64_t len = A->src_len[first + k];
      nf += len >= off + T;
      na += len > off;
    }
    const uint64_t out_left = A->out_len[s] - off;
    ArgRec r;
    r.dst = A->dst[s] + off;
    r.out_bytes = (uint32_t)(out_left < T ? out_left : T);
    r.meta = nf | na << 8;
    r.src = ArgSrc{A->src_ptr + first, off};
    r.src_bytes = ArgLen{A->src_len + first, off, T};
    desc_plain<U, 0>(r, T);
    slot ^= 1;
    if (threadIdx.x == 0) next[slot] = queue_grab(a.ctr, a.base);
    __syncthreads();
    t = __builtin_amdgcn_readfirstlane(next[slot]);
  }
}

// Tile records of a descriptor batch: one wave per stripe, one lane per
// subtile.  A lane whose subtile starts a tile (tile_starts, the host's rule)
// writes the record at tile_start[s] + (tile starts before it).
__device__ __forceinline__ void write_tile(const DescBatch &b, uint32_t s, const bcp_stripe &d,
                                           const bcp_source *run, DescTile *out, uint64_t sub0, uint32_t m,
                                           uint32_t nfull, uint32_t nany) {
  const uint64_t T = b.tile_bytes;
  const uint64_t off = sub0 * T, want = (uint64_t)m * T;
  DescTile rec;
  rec.dst = d.dst + off;
  rec.out_bytes = (uint32_t)(d.out_len - off < want ? d.out_len - off : want);
  if (d.window != 0 && d.window % T == 0 && m == 1) {
    // Window replay (A3-q1) on a tile that lies inside one transfer window:
    // the replay is uniform over the tile, so source k is read from
    // ptr + mapped offset (its last readable window re-sent for every later
    // window) -- a plain tile with per-source addresses.  Covering sources
    // first, then the ones ending inside the tile; more than kTileSrcs
    // reaching in falls back to the general path.
    const uint64_t w = off / d.window;
    uint32_t nf = 0, na = 0;
    for (int pass = 0; pass < 2; pass++)
      for (uint32_t k = 0; k < d.nsrc; k++) {
        const uint64_t len = run[k].len;
        if (len == 0) continue;
        const uint64_t lw = (len - 1) / d.window;
        const uint64_t mo = w > lw ? off - (w - lw) * d.window : off;
        if (len <= mo) continue;
        const uint64_t eff = len - mo;
        if ((pass == 0) != (eff >= T)) continue;
        if (na < (uint32_t)kTileSrcs) {
          rec.src[na] = run[k].ptr + mo;
          rec.src_bytes[na] = (uint32_t)(eff < T ? eff : T);
        }
        na++;
        nf += pass == 0;
      }
    if (na <= (uint32_t)kTileSrcs) {
      for (uint32_t k = na; k < (uint32_t)kTileSrcs; k++) {
        rec.src[k] = 0;
        rec.src_bytes[k] = 0;
      }
      rec.meta = nf | na << 8;
      *out = rec;
      return;
    }
  }
  if (d.window != 0 || nany > (uint32_t)kTileSrcs) {
    rec.meta = d.window != 0 ? kTileGeneral : (kTileGeneral | kTileWide | nfull | nany << 8);
    rec.src_bytes[0] = s;
    rec.src_bytes[1] = (uint32_t)sub0;
    rec.src_bytes[2] = d.first_src;
#pragma unroll
    for (int k = 3; k < kTileSrcs; k++) rec.src_bytes[k] = 0;
#pragma unroll
    for (int k = 0; k < kTileSrcs; k++) rec.src[k] = 0;
  } else {
    rec.meta = nfull | nany << 8 | (m - 1) << 16;
#pragma unroll
    for (int k = 0; k < kTileSrcs; k++) {
      const bool in = (uint32_t)k < nany;
      const uint64_t len = in ? run[k].len : 0;
      rec.src[k] = in ? run[k].ptr + off : 0;
      rec.src_bytes[k] = in ? (uint32_t)(len - off < want ? len - off : want) : 0;
    }
  }
  *out = rec;
}

__global__ __launch_bounds__(kBlock) void desc_tiles(DescBatch b) {
  const uint32_t s = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (s >= b.nstripes) return;
  const uint32_t lane = threadIdx.x & 63u;
  const bcp_stripe d = b.stripes[s];
  const bcp_source *run = b.sources + d.first_src;
  auto len_at = [run](uint32_t k) { return run[k].len; };
  const uint64_t T = b.tile_bytes;
  const uint64_t nsub = (d.out_len + T - 1) / T;
  DescTile *out = b.tiles + b.tile_start[s];
  uint32_t carry = 0;
  for (uint64_t base = 0; base < nsub; base += 64) {
    const uint64_t i = base + lane;
    const bool valid = i < nsub;
    SubClass cur{0, 0, false};
    bool st = false;
    if (valid) {
      if (d.window) {
        st = true;
      } else {
        cur = sub_class(len_at, d.nsrc, d.out_len, T, i);
        const SubClass prev = i ? sub_class(len_at, d.nsrc, d.out_len, T, i - 1) : SubClass{0, 0, false};
        st = tile_starts(prev, cur, i, T);
      }
    }
    const uint64_t mask = __ballot(st);
    const uint32_t nt = b.tile_start[s + 1] - b.tile_start[s];
    if (st && carry + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull)) < nt) {
      const uint32_t idx = carry + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
      uint32_t m = 1;
      if (!d.window && cur.g) {
        const uint32_t mmax = (uint32_t)group_rows((int)(T / 4096u)) / cur.nf;
        while (m < mmax && i + m < nsub) {
          const SubClass nx = sub_class(len_at, d.nsrc, d.out_len, T, i + m);
          if (tile_starts(cur, nx, i + m, T)) break;
          m++;
        }
      }
      write_tile(b, s, d, run, out + idx, i, m, cur.nf, d.window ? d.nsrc : cur.na);
    }
    carry += (uint32_t)__popcll(mask);
  }
  // The host counted the same cut (count_tiles); should the two ever differ,
  // leftover slots become empty tiles (no loads, no stores), never stale
  // records from an earlier batch.
  const uint32_t nt = b.tile_start[s + 1] - b.tile_start[s];
  for (uint32_t k = carry + lane; k < nt; k += 64) {
    DescTile e = {};
    out[k] = e;
  }
}

// ---------------------------------------------------------------------------
// Resident fold ring (RingArgs, bcp_internal.h).  Workgroup 0's first wave is
// the watcher, every other workgroup a worker.
// Tickets and parts: the host cuts each piece into `parts` tiles (a field of
// its entry; ~32 KiB of output each, 1..16).  Announcing ticket t at
// entry e, the watcher sets claim[e] = t << 16 | parts << 8 (claimed 0) and
// done_cnt[e] = t << 16 before it advances `pub`.  A worker reads `cur` (the
// ticket being claimed, relative to base), and while t = base + cur < pub it
// claims part n of t by a CAS on claim[e] -- the word carries the ticket, so
// a stale claimer can never take a part of the entry's next ticket -- or,
// when every part is claimed, moves `cur` on by a CAS.  The tile's last
// finisher (done_cnt[e]'s low byte reaching parts - 1) writes done[e].
// Exit conditions every wave reaches: the watcher closes after idle_ticks
// without a new ticket or once the host sets stop while nothing is pending;
// a worker leaves when the watcher has closed and `cur` has reached the last
// announced ticket (every part of every announced ticket claimed, and the
// claimed ones are folded before their claimers look again), or after
// hard_ticks of waiting (no watcher: never in a healthy launch).
// Memory ordering: host rows and the entry are read after a system-scope
// acquire; a tile's stores go out behind every wave's vmcnt(0) wait, a
// barrier and a system-scope release by lane 0 before it counts the tile;
// the last tile of a ticket acquires and releases again before its done
// word (system scope: the reader is the host).  The explicit vmcnt(0) after
// each release fence keeps the flag behind the write-back whatever the
// compiler proves about the scoreboard (MI355X_MICROARCH.md, compiler hazard).
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

template <typename T>
__device__ __forceinline__ T ld_agent(const T *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void ring_watch(const RingArgs &a) {
  const uint32_t lane = threadIdx.x;  // one wave
  unsigned long long pub = a.base;
  unsigned long long last = now_ticks();
  for (;;) {
    const uint32_t e = (uint32_t)(pub & a.kmask);
    const unsigned long long s = __hip_atomic_load(&a.host[e].seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (s == pub + 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the entry's body, written before seq
      const glob<v4u> *src = gp<v4u>((uint64_t)(uintptr_t)(a.host + e));
      glob<v4u> *dst = gp<v4u>((uint64_t)(uintptr_t)(a.copy + e));
      const v4u body = src[lane];
      dst[lane] = body;
      if (lane == 1) {  // bytes 16..31: out_len, nsrc, parts
        const unsigned long long parts = body[3] & 0xFFu;
        __hip_atomic_store(&a.claim[e], pub << 16 | parts << 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.cnt[e], pub << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(&a.state->pub, pub + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pub++;
      last = now_ticks();
      continue;
    }
    if (__hip_atomic_load(a.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
    if (now_ticks() - last > a.idle_ticks) break;
    __builtin_amdgcn_s_sleep(4);
  }
  if (lane == 0) {
    __hip_atomic_store(a.closed, pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // pub before quit
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&a.state->quit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One tile: bytes [lo, lo + tb) of the ticket's piece, lane l owning vectors
// l + 256 u (u < tb / 4 KiB <= 8).  Sources that cover the tile are folded
// four at a time with every load first; a source ending inside it takes the
// masked path (load_src_tail); zero padding is never read.
__device__ __forceinline__ void ring_tile(const RingEntry &E, uint32_t parts, uint32_t part) {
  const uint64_t out_len = E.out_len;
  uint64_t tb = (out_len + parts - 1) / parts;
  tb = (tb + 4095u) & ~(uint64_t)4095u;
  const uint64_t lo = (uint64_t)part * tb;
  if (lo >= out_len) return;
  const uint32_t nv = (uint32_t)(tb >> 12);  // 1..8 (the host keeps tb <= 32 KiB)
  const uint64_t hi = lo + tb;
  const uint32_t nsrc = E.nsrc;
  const uint32_t lane_off = threadIdx.x * 16u;
  v4u acc[8];
#pragma unroll
  for (int u = 0; u < 8; u++) acc[u] = zero4();
  for (uint32_t k0 = 0; k0 < nsrc; k0 += 4) {
    v4u x[4][8];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t k = k0 + i;
      const bool full = k < nsrc && E.src[k].len >= hi;
      gbyte *p = gp<const unsigned char>(full ? E.src[k].ptr + lo + lane_off : 0);
#pragma unroll
      for (int u = 0; u < 8; u++) x[i][u] = full && (uint32_t)u < nv ? ld16(p + u * 4096) : zero4();
    }
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int u = 0; u < 8; u++) acc[u] ^= x[i][u];
  }
  for (uint32_t k = 0; k < nsrc; k++) {
    const uint64_t len = E.src[k].len;
    if (len <= lo || len >= hi) continue;
    gbyte *p = gp<const unsigned char>(E.src[k].ptr);
#pragma unroll
    for (int u = 0; u < 8; u++)
      if ((uint32_t)u < nv) acc[u] ^= load_src_tail(p, len, lo + lane_off + u * 4096u);
  }
  glob<unsigned char> *d = gp<unsigned char>(E.dst);
#pragma unroll
  for (int u = 0; u < 8; u++)
    if ((uint32_t)u < nv) store_tail(d, out_len, lo + lane_off + u * 4096u, acc[u]);
}

// Thread 0: the next (ticket, part) to fold, packed t << 16 | parts << 8 |
// part, or ~0 when the launch is over for this workgroup.
__device__ __forceinline__ unsigned long long ring_claim(const RingArgs &a) {
  const unsigned long long t0 = now_ticks();
  for (;;) {
    const unsigned long long c = ld_agent(&a.state->cur);
    const unsigned long long t = a.base + c;
    if (t >= ld_agent(&a.state->pub)) {
      if (ld_agent(&a.state->quit)) {
        // quit is stored after the last pub: one more look decides
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (a.base + ld_agent(&a.state->cur) >= ld_agent(&a.state->pub)) return ~0ull;
        continue;
      }
      if (now_ticks() - t0 > a.hard_ticks) return ~0ull;
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the watcher's claim word for t
    const uint32_t e = (uint32_t)(t & a.kmask);
    unsigned long long v = ld_agent(&a.claim[e]);
    if ((v >> 16) != t) continue;  // cur moved on meanwhile: look again
    const uint32_t parts = (uint32_t)(v >> 8) & 0xFFu, n = (uint32_t)v & 0xFFu;
    if (n >= parts) {  // every part of t is taken: on to t + 1
      unsigned long long cc = c;
      __hip_atomic_compare_exchange_strong(&a.state->cur, &cc, c + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    if (__hip_atomic_compare_exchange_strong(&a.claim[e], &v, v + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return t << 16 | (unsigned long long)parts << 8 | n;
  }
}

__device__ __forceinline__ void ring_work(const RingArgs &a) {
  __shared__ unsigned long long s_g[2];
  __shared__ RingEntry s_e;
  int slot = 0;
  for (;;) {
    if (threadIdx.x == 0) s_g[slot] = ring_claim(a);
    __syncthreads();
    const unsigned long long g = s_g[slot];
    slot ^= 1;
    if (g == ~0ull) return;
    const unsigned long long t = g >> 16;
    const uint32_t parts = (uint32_t)(g >> 8) & 0xFFu, part = (uint32_t)g & 0xFFu;
    const uint32_t e = (uint32_t)(t & a.kmask);
    // the entry's copy (HBM, written by the watcher) and the host rows: fresh
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (threadIdx.x < 64) {
      const unsigned long long *q = (const unsigned long long *)(a.copy + e) + 2 * threadIdx.x;
      unsigned long long *w = (unsigned long long *)&s_e + 2 * threadIdx.x;
      w[0] = ld_agent(q);
      w[1] = ld_agent(q + 1);
    }
    __syncthreads();
    ring_tile(s_e, parts, part);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's stores done; s_e free for the next tile
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned long long old =
          __hip_atomic_fetch_add(&a.cnt[e], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (old == (t << 16 | (unsigned long long)(parts - 1))) {
        // the ticket's last tile: the other tiles' stores were released
        // before their counts; order them before the done word
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&a.done[(size_t)e * kRingDoneStride], t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void fold_ring(RingArgs a) {
  if (blockIdx.x == 0) {
    if (threadIdx.x < 64) ring_watch(a);
    return;
  }
  ring_work(a);
}

// ---------------------------------------------------------------------------
// Synthetic data: byte b of the stream = byte (b & 7) of splitmix64(seed + b/8)
// (same stream as oracle_fill_synthetic).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(kBlock) void fill_synthetic(unsigned char *dst, uint64_t bytes, uint64_t seed,
                                                        uint64_t byte_offset) {
  const uint64_t nvec = bytes / 16;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const bool fast = (byte_offset & 7) == 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nvec; i += stride) {
    if (fast) {
      const uint64_t w = (byte_offset >> 3) + 2 * i;
      const uint64_t a = splitmix64(seed + w), c = splitmix64(seed + w + 1);
      v4u v{(unsigned int)a, (unsigned int)(a >> 32), (unsigned int)c, (unsigned int)(c >> 32)};
      *reinterpret_cast<v4u_u *>(dst + 16 * i) = v;
    } else {
      for (int q = 0; q < 16; q++) {
        const uint64_t bb = byte_offset + 16 * i + q;
        dst[16 * i + q] = (unsigned char)(splitmix64(seed + (bb >> 3)) >> (8 * (bb & 7)));
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < (bytes & 15)) {
    const uint64_t i = nvec * 16 + threadIdx.x;
    const uint64_t bb = byte_offset + i;
    dst[i] = (unsigned char)(splitmix64(seed + (bb >> 3)) >> (8 * (bb & 7)));
  }
}

// XOR-fold: out4 (16 bytes) ^= XOR of all 16-byte lanes; tail byte i of the
// buffer lands in fold byte (i % 16).
__global__ __launch_bounds__(kBlock) void xor_fold(const unsigned char *src, uint64_t bytes, uint32_t *out4) {
  const uint64_t nvec = bytes / 16;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  v4u acc = zero4();
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nvec; i += stride)
    acc ^= ld_nt(reinterpret_cast<const v4u *>(src) + i);  // fold requires 16-B aligned src
  if (blockIdx.x == 0 && threadIdx.x < (bytes & 15)) {
    const uint64_t i = nvec * 16 + threadIdx.x;
    const uint32_t q = (uint32_t)(i & 15);
    acc[q >> 2] ^= (unsigned int)src[i] << (8 * (q & 3));
  }
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int c = 0; c < 4; c++) acc[c] ^= __shfl_xor(acc[c], off, 64);
  }
  __shared__ v4u part[kBlock / 64];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    v4u r = part[0];
    for (int w = 1; w < kBlock / 64; w++) r ^= part[w];
    for (int c = 0; c < 4; c++)
      if (r[c]) atomicXor(out4 + c, r[c]);
  }
}

// Number of differing bytes between a and b (both 16-B aligned).
__global__ __launch_bounds__(kBlock) void compare_bytes(const unsigned char *a, const unsigned char *b,
                                                       uint64_t bytes, unsigned long long *out) {
  const uint64_t nvec = bytes / 16;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  unsigned long long cnt = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nvec; i += stride) {
    const v4u x = ld_nt(reinterpret_cast<const v4u *>(a) + i) ^ ld_nt(reinterpret_cast<const v4u *>(b) + i);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const unsigned int w = x[c];
      cnt += ((w & 0xFFu) != 0) + ((w & 0xFF00u) != 0) + ((w & 0xFF0000u) != 0) + ((w & 0xFF000000u) != 0);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < (bytes & 15)) {
    const uint64_t i = nvec * 16 + threadIdx.x;
    cnt += a[i] != b[i];
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
  __shared__ unsigned long long part[kBlock / 64];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long r = 0;
    for (int w = 0; w < kBlock / 64; w++) r += part[w];
    if (r) atomicAdd(out, r);
  }
}

// ---------------------------------------------------------------------------
// Launchers.
// ---------------------------------------------------------------------------
template <int NSRC, int U, int GATHER, int W>
static hipError_t launch_stream_w(hipStream_t st, int grid, const StreamArgs &a) {
  if (a.vps % (uint32_t)(kBlock * U) != 0 || a.tail != 0)
    hipLaunchKernelGGL((xor_stream_w<NSRC, U, GATHER, kQueuePartial, W>), dim3(grid), dim3(kBlock), 0, st, a);
  else
    hipLaunchKernelGGL((xor_stream_w<NSRC, U, GATHER, kQueueFull, W>), dim3(grid), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}


template <int NSRC, int U, int GATHER>
static hipError_t launch_stream_nu(hipStream_t st, int grid, const StreamArgs &a) {
  if (a.vps % (uint32_t)(kBlock * U) != 0 || a.tail != 0)
    hipLaunchKernelGGL((xor_stream<NSRC, U, GATHER, kQueuePartial>), dim3(grid), dim3(kBlock), 0, st, a);
  else
    hipLaunchKernelGGL((xor_stream<NSRC, U, GATHER, kQueueFull>), dim3(grid), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}

template <int U, int GATHER>
static hipError_t launch_stream_u(hipStream_t st, int grid, const StreamArgs &a) {
#define BCP_NSRC_CASE(n) \
  case n: return launch_stream_nu<n, U, GATHER>(st, grid, a);
  switch (a.nsrc) {
    BCP_NSRC_CASE(1) BCP_NSRC_CASE(2) BCP_NSRC_CASE(3) BCP_NSRC_CASE(4) BCP_NSRC_CASE(5)
    BCP_NSRC_CASE(6) BCP_NSRC_CASE(7) BCP_NSRC_CASE(8) BCP_NSRC_CASE(9) BCP_NSRC_CASE(10)
    BCP_NSRC_CASE(11) BCP_NSRC_CASE(12) BCP_NSRC_CASE(16)
    default:
      return launch_stream_nu<0, U, GATHER>(st, grid, a);
  }
#undef BCP_NSRC_CASE
}

uint32_t stream_tiles_per_stripe(uint64_t chunk_bytes, int vecs) {
  const uint64_t vps = (chunk_bytes + 15) / 16;  // the byte tail is a (partial) vector too
  const uint64_t tile_v = (uint64_t)kBlock * vecs;
  return (uint32_t)((vps + tile_v - 1) / tile_v);
}

hipError_t launch_xor_stream(hipStream_t st, int grid, int vecs, bool gather, const StreamArgs &a) {
  if (a.ntiles == 0) return hipSuccess;
  // Register budget W = 6 (profiles/r01/depth/ab18_wpe_widths.jsonl): +0.8
  // (N = 8), +0.9..+6.6 (N = 5..7 at U = 8) and +0.3..+3.8 (N = 9..12, 16 at
  // U = 4; ab19) on the strided form, but -1.4 / -4.5 at N = 3 / 4 (W = 5 /
  // 7 there: -1.1 / -1.6 at N = 3, -1.7 / +0.45 at N = 4; ab20), which keep
  // the compiler's schedule; the pointer-table form takes it for N = 8 (+0.1).
  if (vecs == 8 && a.nsrc == 8)
    return gather ? launch_stream_w<8, 8, 1, 6>(st, grid, a) : launch_stream_w<8, 8, 0, 6>(st, grid, a);
  if (!gather && vecs == 8) {
    switch (a.nsrc) {
      case 5: return launch_stream_w<5, 8, 0, 6>(st, grid, a);
      case 6: return launch_stream_w<6, 8, 0, 6>(st, grid, a);
      case 7: return launch_stream_w<7, 8, 0, 6>(st, grid, a);
      default: break;
    }
  }
  if (!gather && vecs == 4) {
    switch (a.nsrc) {
      case 9: return launch_stream_w<9, 4, 0, 6>(st, grid, a);
      case 10: return launch_stream_w<10, 4, 0, 6>(st, grid, a);
      case 11: return launch_stream_w<11, 4, 0, 6>(st, grid, a);
      case 12: return launch_stream_w<12, 4, 0, 6>(st, grid, a);
      case 16: return launch_stream_w<16, 4, 0, 6>(st, grid, a);
      default: break;
    }
  }
  if (gather) {
    switch (vecs) {
      case 1: return launch_stream_u<1, 1>(st, grid, a);
      case 4: return launch_stream_u<4, 1>(st, grid, a);
      case 8: return launch_stream_u<8, 1>(st, grid, a);
      default: return launch_stream_u<2, 1>(st, grid, a);
    }
  }
  switch (vecs) {
    case 1: return launch_stream_u<1, 0>(st, grid, a);
    case 4: return launch_stream_u<4, 0>(st, grid, a);
    case 8: return launch_stream_u<8, 0>(st, grid, a);
    default: return launch_stream_u<2, 0>(st, grid, a);
  }
}

hipError_t launch_desc_tiles(hipStream_t st, const DescBatch &b) {
  if (b.nstripes == 0) return hipSuccess;
  const uint32_t waves = kBlock / 64;  // one wave per stripe
  hipLaunchKernelGGL(desc_tiles, dim3((b.nstripes + waves - 1) / waves), dim3(kBlock), 0, st, b);
  return hipGetLastError();
}

hipError_t launch_xor_desc(hipStream_t st, int grid, int vecs, const DescBatch &b) {
  if (b.ntiles == 0) return hipSuccess;
  if ((uint32_t)grid > b.ntiles) grid = (int)b.ntiles;
  if (vecs == 16) {
    // 64 KiB subtiles (engine option desc_vecs_per_thread 16): half the queue
    // grabs and record loads of U = 8
    hipLaunchKernelGGL((xor_desc_p<16, 5>), dim3(grid), dim3(kBlock), 0, st, b);
    return hipGetLastError();
  }
  if (vecs == 8) {
    hipLaunchKernelGGL((xor_desc_p<8, 5>), dim3(grid), dim3(kBlock), 0, st, b);
    return hipGetLastError();
  }
  switch (vecs) {
    case 1: hipLaunchKernelGGL((xor_desc<1>), dim3(grid), dim3(kBlock), 0, st, b); break;
    case 4: hipLaunchKernelGGL((xor_desc<4>), dim3(grid), dim3(kBlock), 0, st, b); break;
    default: hipLaunchKernelGGL((xor_desc<2>), dim3(grid), dim3(kBlock), 0, st, b); break;
  }
  return hipGetLastError();
}

hipError_t launch_xor_desc_args(hipStream_t st, int grid, int vecs, const DescArgs &a) {
  if (a.ntiles == 0) return hipSuccess;
  if ((uint32_t)grid > a.ntiles) grid = (int)a.ntiles;
  switch (vecs) {
    case 1: hipLaunchKernelGGL((xor_desc_args<1>), dim3(grid), dim3(kBlock), 0, st, a); break;
    case 4: hipLaunchKernelGGL((xor_desc_args<4>), dim3(grid), dim3(kBlock), 0, st, a); break;
    case 8: hipLaunchKernelGGL((xor_desc_args<8>), dim3(grid), dim3(kBlock), 0, st, a); break;
    default: hipLaunchKernelGGL((xor_desc_args<2>), dim3(grid), dim3(kBlock), 0, st, a); break;
  }
  return hipGetLastError();
}

hipError_t launch_fold_ring(hipStream_t st, int workers, const RingArgs &a) {
  if (workers < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fold_ring, dim3(1 + workers), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_fill_synthetic(hipStream_t st, int grid, char *dst, uint64_t bytes, uint64_t seed,
                                 uint64_t byte_offset) {
  if (bytes == 0) return hipSuccess;
  hipLaunchKernelGGL(fill_synthetic, dim3(grid), dim3(kBlock), 0, st, (unsigned char *)dst, bytes, seed,
                     byte_offset);
  return hipGetLastError();
}

hipError_t launch_xor_fold(hipStream_t st, int grid, const char *src, uint64_t bytes, uint32_t *out4) {
  if (bytes == 0) return hipSuccess;
  hipLaunchKernelGGL(xor_fold, dim3(grid), dim3(kBlock), 0, st, (const unsigned char *)src, bytes, out4);
  return hipGetLastError();
}

hipError_t launch_compare(hipStream_t st, int grid, const char *a, const char *b, uint64_t bytes,
                          unsigned long long *out) {
  if (bytes == 0) return hipSuccess;
  hipLaunchKernelGGL(compare_bytes, dim3(grid), dim3(kBlock), 0, st, (const unsigned char *)a,
                     (const unsigned char *)b, bytes, out);
  return hipGetLastError();
}

}  // namespace bcp
