// bcp_internal.h -- shared between the engine (bcp_engine.hip) and the kernels
// (bcp_kernels.hip).  Not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdint.h>

#include "bcp.h"

namespace bcp {

constexpr int kBlock = 256;        // threads per workgroup (4 waves of 64)
constexpr int kMaxVecsPerThread = 8;     // xor_stream and xor_desc

// Tile schedules of the streaming kernel.
constexpr int kSchedQueue = 0;   // device-wide work queue (default)
constexpr int kSchedStatic = 1;  // contiguous tile range per workgroup (r01 design; A/B only)

// Defaults from the r01 interleaved sweeps on MI355X (profiles/r01/):
// xor_stream: one 256-thread workgroup per CU with 8 vectors per lane (the
// fewer tiles in flight, the narrower the queue's address window:
// kernel_exp_6/7), work-queue schedule, non-temporal loads and stores.
struct Tuning {
    int blocks_per_cu = 1;      // xor_stream: 256-thread workgroups launched per CU
    int vecs_per_thread = 8;    // xor_stream: 16-byte vectors per lane per tile (1, 2, 4, 8)
    int schedule = kSchedQueue; // xor_stream: kSched*
    // xor_desc, config-5 shapes (profiles/r01/mixed/): 2 workgroups per CU,
    // 8 vectors per lane, one 32 KiB tile per queue grab = 77.3 % (U = 4 needed
    // 2-tile grabs: 72.9 %; 1 WG/CU 71.9-75.4 %).  Mixed-size tiles read ~2.4x
    // fewer bytes than config-2 tiles, so the grab size is per kernel.
    int desc_blocks_per_cu = 2;
    int desc_vecs = 8;          // 1, 2, 4, 8
    int desc_grab = 1;          // tiles per work-queue grab
    int desc_schedule = kSchedQueue;
};

// Arguments of the streaming kernel (xor_stream).
struct StreamArgs {
    char *dst;                  // GATHER = 0: output of stripe s at dst + s*dst_stride
    uint64_t dst_stride;
    const char *src;            // GATHER = 0: source k of stripe s at src + s*stripe_stride + k*src_stride
    uint64_t stripe_stride;
    uint64_t src_stride;
    const bcp_stripe *stripes;  // GATHER = 1: uniform descriptor batch (device copy)
    const bcp_source *sources;
    uint32_t vps;               // 16-byte vectors per stripe output
    uint32_t tps;               // tiles per stripe
    uint32_t ntiles;
    uint32_t nsrc;
    uint32_t dense;             // GATHER = 1: stripes[s].first_src == s * nsrc for every s
    unsigned long long *ctr;    // work-queue counter (per queue)
    unsigned long long base;    // counter value at the start of this launch
    int sched;                  // kSched*
};

// Device-side form of one stripe descriptor batch.
struct DescBatch {
    const bcp_stripe *stripes;  // [nstripes]
    const bcp_source *sources;  // [nsources]
    const uint32_t *tile_start; // [nstripes + 1] prefix of tiles per stripe
    uint32_t nstripes;
    uint32_t ntiles;
    uint32_t tile_bytes;        // bytes of output per tile
    unsigned long long *ctr;    // work-queue counter (per queue), as StreamArgs
    unsigned long long base;
    int sched;                  // kSched*
    uint32_t grab;              // kSchedQueue: tiles per grab
};

// Kernel launchers (bcp_kernels.hip).  All return hipError_t.
// Streaming fold.  Consumes ntiles + grid counts of a.ctr when a.sched is
// kSchedQueue; the caller clamps grid to [1, ntiles].
hipError_t launch_xor_stream(hipStream_t st, int grid, int vecs, bool gather,
                             const StreamArgs &a);
uint32_t stream_tiles_per_stripe(uint64_t chunk_bytes, int vecs);
// Descriptor kernel; same work-queue accounting as launch_xor_stream.
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
