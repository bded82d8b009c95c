// bcp_kernels.hip -- CDNA4 (gfx950) kernels of the chunk-XOR parity engine.
//
// The arithmetic is the reference's xor_parity
// (src/beegfs-raid5/common/task_processing.c:96-109): out = XOR of N source
// chunks, zero-padded to the output length.  It is a read-once integer stream
// (N loads + 1 store per output byte, no reuse), so the design rules are the
// HBM ones: 16-byte lanes (global_load_dwordx4), every source load of a lane
// issued before the XORs, non-temporal hints so the 8:1 read stream does not
// churn L2/MALL, and a persistent grid sized to the CU count.
//
// Kernels:
//   xor_strided_fast<NSRC,U>  uniform stripes, 16-B aligned geometry (hot path)
//   xor_desc<U>               descriptor batches: variable lengths, zero pad,
//                             rebuild truncation, window replay, any alignment
//   fill_synthetic / xor_fold / compare   synthetic inputs and verification
#include "bcp_internal.h"

namespace bcp {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef v4u v4u_u __attribute__((aligned(1)));  // unaligned 16-byte view

__device__ __forceinline__ v4u ld_nt(const v4u *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ v4u zero4() { return v4u{0u, 0u, 0u, 0u}; }

// ---------------------------------------------------------------------------
// Fast path.  Stripe s, source k starts at src + s*stripe_stride + k*src_stride
// and holds vps 16-byte vectors; output s at dst + s*dst_stride.  A tile is
// kBlock*U vectors of one stripe.  Lane l of a tile owns vectors l, l+256, ...
// so each wave-instruction moves 1 KiB contiguous per source, and all
// NSRC*U loads of a lane are issued before its XORs.  NSRC == 0 means
// "runtime nsrc".  POL selects the cache policy and the tile schedule
// (kPolPlainLoad / kPolPlainStore / kPolContig bits, see bcp_internal.h).
// ---------------------------------------------------------------------------
template <int POL>
__device__ __forceinline__ v4u ld_pol(const v4u *p) {
  if constexpr (POL & kPolPlainLoad) return *p;
  else return __builtin_nontemporal_load(p);
}
template <int POL>
__device__ __forceinline__ void st_pol(v4u *p, v4u v) {
  if constexpr (POL & kPolPlainStore) *p = v;
  else __builtin_nontemporal_store(v, p);
}

template <int NSRC, int U, int POL>
__device__ __forceinline__ void fast_tile(char *__restrict__ dst, uint64_t dst_stride, const char *__restrict__ src,
                                          uint64_t stripe_stride, uint64_t src_stride, uint32_t vps, uint32_t tps,
                                          uint32_t nsrc, uint32_t t) {
  constexpr uint32_t tile_v = kBlock * U;
  const uint32_t s = t / tps;
  const uint32_t tin = t - s * tps;
  const char *sb = src + (uint64_t)s * stripe_stride;
  v4u *db = reinterpret_cast<v4u *>(dst + (uint64_t)s * dst_stride);
  const uint32_t v0 = tin * tile_v + threadIdx.x;
  v4u acc[U];
  if (tin * tile_v + tile_v <= vps) {
    const v4u *p0 = reinterpret_cast<const v4u *>(sb) + v0;
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = ld_pol<POL>(p0 + u * kBlock);
    if constexpr (NSRC > 0) {
#pragma unroll
      for (int k = 1; k < NSRC; k++) {
        const v4u *pk = reinterpret_cast<const v4u *>(sb + k * src_stride) + v0;
#pragma unroll
        for (int u = 0; u < U; u++) acc[u] ^= ld_pol<POL>(pk + u * kBlock);
      }
    } else {
#pragma unroll 4
      for (uint32_t k = 1; k < nsrc; k++) {
        const v4u *pk = reinterpret_cast<const v4u *>(sb + k * src_stride) + v0;
#pragma unroll
        for (int u = 0; u < U; u++) acc[u] ^= ld_pol<POL>(pk + u * kBlock);
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) st_pol<POL>(db + v0 + u * kBlock, acc[u]);
  } else {
    // Last, partial tile of a stripe: per-vector bounds.
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t v = v0 + u * kBlock;
      if (v < vps) {
        v4u a = ld_pol<POL>(reinterpret_cast<const v4u *>(sb) + v);
        for (uint32_t k = 1; k < nsrc; k++) a ^= ld_pol<POL>(reinterpret_cast<const v4u *>(sb + k * src_stride) + v);
        st_pol<POL>(db + v, a);
      }
    }
  }
}

template <int NSRC, int U, int POL>
__global__ __launch_bounds__(kBlock) void xor_strided_fast(
    char *__restrict__ dst, uint64_t dst_stride, const char *__restrict__ src,
    uint64_t stripe_stride, uint64_t src_stride, uint32_t vps, uint32_t tps,
    uint32_t ntiles, uint32_t nsrc_rt) {
  const uint32_t nsrc = NSRC > 0 ? (uint32_t)NSRC : nsrc_rt;
  if constexpr (POL & kPolContig) {
    // Workgroup b owns tiles [b*T/G, (b+1)*T/G): one contiguous run each.
    const uint32_t t0 = (uint32_t)(((uint64_t)blockIdx.x * ntiles) / gridDim.x);
    const uint32_t t1 = (uint32_t)(((uint64_t)(blockIdx.x + 1) * ntiles) / gridDim.x);
    for (uint32_t t = t0; t < t1; t++)
      fast_tile<NSRC, U, POL>(dst, dst_stride, src, stripe_stride, src_stride, vps, tps, nsrc, t);
  } else {
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
      fast_tile<NSRC, U, POL>(dst, dst_stride, src, stripe_stride, src_stride, vps, tps, nsrc, t);
  }
}

// ---------------------------------------------------------------------------
// Descriptor path helpers.
// ---------------------------------------------------------------------------

// 16 bytes of source `p` (readable length len) at offset off, zero past len.
__device__ __forceinline__ v4u load_src_tail(const unsigned char *p, uint64_t len, uint64_t off) {
  if (off + 16 <= len) return *reinterpret_cast<const v4u_u *>(p + off);
  if (off >= len) return zero4();
  unsigned int w[4] = {0u, 0u, 0u, 0u};
  const uint32_t n = (uint32_t)(len - off);
  for (uint32_t i = 0; i < n; i++) w[i >> 2] |= (unsigned int)p[off + i] << (8 * (i & 3));
  return v4u{w[0], w[1], w[2], w[3]};
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

__device__ __forceinline__ void store_tail(unsigned char *d, uint64_t out_len, uint64_t off, v4u v) {
  if (off + 16 <= out_len) {
    *reinterpret_cast<v4u_u *>(d + off) = v;
    return;
  }
  if (off >= out_len) return;
  const uint32_t n = (uint32_t)(out_len - off);
  for (uint32_t i = 0; i < n; i++) d[off + i] = (unsigned char)(v[i >> 2] >> (8 * (i & 3)));
}

// ---------------------------------------------------------------------------
// Descriptor kernel.  Tiles of tile_bytes output bytes are numbered across the
// batch (tile_start prefix); workgroup b owns the contiguous tile range
// [b*T/G, (b+1)*T/G), so it finds its first stripe by one binary search and
// then walks forward.  Per tile and per source the coverage test is uniform:
// a source either covers the whole tile (unconditional 16-B loads, four
// sources in flight together), misses it (skipped: zero padding), or ends
// inside it (per-lane tail path).  Window-replay stripes take the per-lane
// path for every source.
// ---------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(kBlock) void xor_desc(DescBatch b) {
  const uint32_t g = gridDim.x;
  const uint32_t t_begin = (uint32_t)(((uint64_t)blockIdx.x * b.ntiles) / g);
  const uint32_t t_end = (uint32_t)(((uint64_t)(blockIdx.x + 1) * b.ntiles) / g);
  if (t_begin >= t_end) return;
  uint32_t lo = 0, hi = b.nstripes;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (b.tile_start[mid] <= t_begin) lo = mid; else hi = mid;
  }
  uint32_t s = lo;
  const uint64_t tile_bytes = b.tile_bytes;
  for (uint32_t t = t_begin; t < t_end; t++) {
    while (b.tile_start[s + 1] <= t) s++;
    const bcp_stripe d = b.stripes[s];
    const uint64_t tile_off = (uint64_t)(t - b.tile_start[s]) * tile_bytes;
    const uint64_t tile_end = tile_off + tile_bytes;
    uint64_t j[U];
#pragma unroll
    for (int u = 0; u < U; u++) j[u] = tile_off + ((uint64_t)u * kBlock + threadIdx.x) * 16u;
    v4u acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = zero4();
    const bcp_source *srcs = b.sources + d.first_src;
    uint32_t k = 0;
    if (d.window == 0) {
      // Groups of four sources that all cover the tile: 4*U loads in flight.
      for (; k + 4 <= d.nsrc; k += 4) {
        const bcp_source s0 = srcs[k], s1 = srcs[k + 1], s2 = srcs[k + 2], s3 = srcs[k + 3];
        if (s0.len >= tile_end && s1.len >= tile_end && s2.len >= tile_end && s3.len >= tile_end) {
          const unsigned char *p0 = (const unsigned char *)s0.ptr, *p1 = (const unsigned char *)s1.ptr;
          const unsigned char *p2 = (const unsigned char *)s2.ptr, *p3 = (const unsigned char *)s3.ptr;
          v4u x0[U], x1[U], x2[U], x3[U];
#pragma unroll
          for (int u = 0; u < U; u++) {
            x0[u] = *reinterpret_cast<const v4u_u *>(p0 + j[u]);
            x1[u] = *reinterpret_cast<const v4u_u *>(p1 + j[u]);
            x2[u] = *reinterpret_cast<const v4u_u *>(p2 + j[u]);
            x3[u] = *reinterpret_cast<const v4u_u *>(p3 + j[u]);
          }
#pragma unroll
          for (int u = 0; u < U; u++) acc[u] ^= (x0[u] ^ x1[u]) ^ (x2[u] ^ x3[u]);
        } else {
          const bcp_source ss[4] = {s0, s1, s2, s3};
#pragma unroll
          for (int i = 0; i < 4; i++) {
            if (ss[i].len <= tile_off) continue;  // zero padding
            const unsigned char *p = (const unsigned char *)ss[i].ptr;
#pragma unroll
            for (int u = 0; u < U; u++) acc[u] ^= load_src_tail(p, ss[i].len, j[u]);
          }
        }
      }
      for (; k < d.nsrc; k++) {
        const bcp_source sk = srcs[k];
        if (sk.len <= tile_off) continue;
        const unsigned char *p = (const unsigned char *)sk.ptr;
        if (sk.len >= tile_end) {
#pragma unroll
          for (int u = 0; u < U; u++) acc[u] ^= *reinterpret_cast<const v4u_u *>(p + j[u]);
        } else {
#pragma unroll
          for (int u = 0; u < U; u++) acc[u] ^= load_src_tail(p, sk.len, j[u]);
        }
      }
    } else {
      for (; k < d.nsrc; k++) {
        const bcp_source sk = srcs[k];
        const unsigned char *p = (const unsigned char *)sk.ptr;
#pragma unroll
        for (int u = 0; u < U; u++) {
          if (j[u] < d.out_len)
            acc[u] ^= load_src_tail(p, sk.len, replay_offset(j[u], sk.len, d.window));
        }
      }
    }
    unsigned char *dp = (unsigned char *)d.dst;
    if (tile_end <= d.out_len) {
#pragma unroll
      for (int u = 0; u < U; u++) *reinterpret_cast<v4u_u *>(dp + j[u]) = acc[u];
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) store_tail(dp, d.out_len, j[u], acc[u]);
    }
  }
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
template <int NSRC, int U, int POL>
static hipError_t launch_fast_nu(hipStream_t st, int grid, char *dst, uint64_t dst_stride, const char *src,
                                 uint64_t stripe_stride, uint64_t src_stride, uint32_t vps, uint32_t tps,
                                 uint32_t ntiles, uint32_t nsrc) {
  hipLaunchKernelGGL((xor_strided_fast<NSRC, U, POL>), dim3(grid), dim3(kBlock), 0, st, dst, dst_stride, src,
                     stripe_stride, src_stride, vps, tps, ntiles, nsrc);
  return hipGetLastError();
}

// The hot 8-wide stripe gets every policy variant; other widths use the
// default policy (non-temporal loads and stores, grid-stride tiles).
template <int U>
static hipError_t launch_fast_u(hipStream_t st, int grid, int pol, char *dst, uint64_t dst_stride, const char *src,
                                uint64_t stripe_stride, uint64_t src_stride, uint32_t vps, uint32_t tps,
                                uint32_t ntiles, uint32_t nsrc) {
#define BCP_ARGS st, grid, dst, dst_stride, src, stripe_stride, src_stride, vps, tps, ntiles, nsrc
#define BCP_NSRC_CASE(n) \
  case n: return launch_fast_nu<n, U, 0>(BCP_ARGS);
  if (nsrc == 8) {
    switch (pol & 7) {
      case 1: return launch_fast_nu<8, U, 1>(BCP_ARGS);
      case 2: return launch_fast_nu<8, U, 2>(BCP_ARGS);
      case 3: return launch_fast_nu<8, U, 3>(BCP_ARGS);
      case 4: return launch_fast_nu<8, U, 4>(BCP_ARGS);
      case 5: return launch_fast_nu<8, U, 5>(BCP_ARGS);
      case 6: return launch_fast_nu<8, U, 6>(BCP_ARGS);
      case 7: return launch_fast_nu<8, U, 7>(BCP_ARGS);
      default: return launch_fast_nu<8, U, 0>(BCP_ARGS);
    }
  }
  switch (nsrc) {
    BCP_NSRC_CASE(1) BCP_NSRC_CASE(2) BCP_NSRC_CASE(3) BCP_NSRC_CASE(4) BCP_NSRC_CASE(5)
    BCP_NSRC_CASE(6) BCP_NSRC_CASE(7) BCP_NSRC_CASE(9) BCP_NSRC_CASE(10)
    BCP_NSRC_CASE(11) BCP_NSRC_CASE(12) BCP_NSRC_CASE(16)
    default:
      return launch_fast_nu<0, U, 0>(BCP_ARGS);
  }
#undef BCP_NSRC_CASE
#undef BCP_ARGS
}

hipError_t launch_xor_strided_fast(hipStream_t st, int grid, int vecs, int pol, char *dst, uint64_t dst_stride,
                                   const char *src, uint64_t stripe_stride, uint64_t src_stride,
                                   uint64_t nstripes, uint32_t nsrc, uint64_t chunk_bytes) {
  const uint32_t vps = (uint32_t)(chunk_bytes / 16);
  const uint32_t tile_v = (uint32_t)kBlock * vecs;
  const uint32_t tps = (vps + tile_v - 1) / tile_v;
  const uint64_t ntiles = nstripes * tps;
  if (ntiles == 0) return hipSuccess;
  if (ntiles > 0x7FFFFFFFull) return hipErrorInvalidValue;
  if ((uint64_t)grid > ntiles) grid = (int)ntiles;
  switch (vecs) {
    case 1: return launch_fast_u<1>(st, grid, pol, dst, dst_stride, src, stripe_stride, src_stride, vps, tps, (uint32_t)ntiles, nsrc);
    case 4: return launch_fast_u<4>(st, grid, pol, dst, dst_stride, src, stripe_stride, src_stride, vps, tps, (uint32_t)ntiles, nsrc);
    default: return launch_fast_u<2>(st, grid, pol, dst, dst_stride, src, stripe_stride, src_stride, vps, tps, (uint32_t)ntiles, nsrc);
  }
}

hipError_t launch_xor_desc(hipStream_t st, int grid, int vecs, const DescBatch &b) {
  if (b.ntiles == 0) return hipSuccess;
  if ((uint32_t)grid > b.ntiles) grid = (int)b.ntiles;
  switch (vecs) {
    case 1: hipLaunchKernelGGL((xor_desc<1>), dim3(grid), dim3(kBlock), 0, st, b); break;
    case 4: hipLaunchKernelGGL((xor_desc<4>), dim3(grid), dim3(kBlock), 0, st, b); break;
    default: hipLaunchKernelGGL((xor_desc<2>), dim3(grid), dim3(kBlock), 0, st, b); break;
  }
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
