// bcp_internal.h -- shared between the engine (bcp_engine.hip) and the kernels
// (bcp_kernels.hip).  Not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdint.h>

#include "bcp.h"

namespace bcp {

constexpr int kBlock = 256;        // threads per workgroup (4 waves of 64)
constexpr int kMaxVecsPerThread = 4;

// Fast-path policy bits (8-wide stripes only; other widths use 0).
constexpr int kPolPlainLoad = 1;   // default-policy loads instead of non-temporal
constexpr int kPolPlainStore = 2;  // default-policy stores instead of non-temporal
constexpr int kPolContig = 4;      // contiguous tile range per workgroup instead of grid-stride

// Defaults from the r01 interleaved sweep on MI355X (profiles/r01/sweep_fast.jsonl):
// 16 x 256-thread workgroups per CU (8 resident, the rest queue behind them),
// 4 vectors per lane, contiguous tile runs, non-temporal loads and stores.
struct Tuning {
    int blocks_per_cu = 16;     // 256-thread workgroups launched per CU
    int vecs_per_thread = 4;    // 16-byte vectors per lane per tile
    int policy = kPolContig;    // kPol* bits for the 8-wide fast path
};

// Device-side form of one stripe descriptor batch.
struct DescBatch {
    const bcp_stripe *stripes;  // [nstripes]
    const bcp_source *sources;  // [nsources]
    const uint32_t *tile_start; // [nstripes + 1] prefix of tiles per stripe
    uint32_t nstripes;
    uint32_t ntiles;
    uint32_t tile_bytes;        // bytes of output per tile
};

// Kernel launchers (bcp_kernels.hip).  All return hipError_t.
hipError_t launch_xor_strided_fast(hipStream_t st, int grid, int vecs, int pol,
                                   char *dst, uint64_t dst_stride,
                                   const char *src, uint64_t stripe_stride,
                                   uint64_t src_stride, uint64_t nstripes,
                                   uint32_t nsrc, uint64_t chunk_bytes);
hipError_t launch_xor_desc(hipStream_t st, int grid, int vecs,
                           const DescBatch &b);
hipError_t launch_fill_synthetic(hipStream_t st, int grid, char *dst,
                                 uint64_t bytes, uint64_t seed,
                                 uint64_t byte_offset);
hipError_t launch_xor_fold(hipStream_t st, int grid, const char *src,
                           uint64_t bytes, uint32_t *out4);
hipError_t launch_compare(hipStream_t st, int grid, const char *a,
                          const char *b, uint64_t bytes,
                          unsigned long long *out);

// Tile size used by the descriptor kernel for a given vecs_per_thread.
inline uint32_t desc_tile_bytes(int vecs) { return (uint32_t)kBlock * vecs * 16u; }

}  // namespace bcp
