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

// Defaults from the r01-r03 interleaved sweeps on MI355X (profiles/r01/,
// DESIGN.md section 4): xor_stream runs one 256-thread workgroup per CU with 8
// vectors per lane (the fewer tiles in flight, the narrower the work queue's
// address window: kernel_exp_6/7), non-temporal loads and stores.  The
// schedules and load shapes that lost those sweeps (static tile ranges,
// grab-ahead, other rolling windows and register budgets, blocking-sync
// waits) are gone from the engine; their numbers stay in profiles/ and
// DESIGN.md.
struct Tuning {
    int blocks_per_cu = 1;      // xor_stream: 256-thread workgroups launched per CU
    int vecs_per_thread = 0;    // xor_stream: 16-byte vectors per lane per tile (1, 2, 4, 8; 0 = by batch size)
    // xor_desc (tools/exp/desc_probe.py, profiles/r01/mixed/, depth/): 8
    // vectors per lane, one 32 KiB tile per queue grab; workgroups per CU
    // 0 = auto (desc_grid_for: one per CU).
    int desc_blocks_per_cu = 0;
    int desc_vecs = 0;          // 1, 2, 4, 8, 16; 0 = by batch size (desc_vecs_for)
    int desc_args_max = 16;     // batches of at most this many stripes go in the kernel arguments (0 = never)
    int stream_grid = 0;        // xor_stream: explicit workgroup count (0: 29/32 of CUs x blocks_per_cu)
    int desc_grid = 0;          // xor_desc: explicit workgroup count (0: desc_grid_for)
    int contiguous_alloc = 0;   // 1: bcp_dev_alloc asks for physically contiguous buffers >= 64 MiB
    // Descriptor tables up to this many bytes are read by the kernels from
    // pinned host memory instead of being copied (tools/batch_curve.py):
    // the pointer-table xor_stream reads its table once per tile (a win up
    // to ~16 stripes of 8), desc_tiles once per batch (a win up to >= 512).
    int table_host_max = 4096;
    int desc_table_host_max = 128 * 1024;
    // bcp_host_alloc / bcp_host_alloc_mapped: 1 = ordinary huge-page memory
    // registered with HIP (CPU copies into and out of it run at malloc speed),
    // 0 = hipHostMalloc.
    int host_registered = 1;
    // xor_desc: a batch resubmitted on a ring slot with byte-identical staged
    // tables reuses that slot's tile records (no table upload, no desc_tiles):
    // the A/B of desc_tiles' concurrent HBM traffic (tools/exp/desc_records_ab.py).
    int desc_reuse_records = 0;
    // Resident fold ring waits (bcp_ring_wait): spin this long, then sleep
    // this long between looks (0: sched_yield instead).
    int ring_spin_us = 4;
    int ring_sleep_us = 10;
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
    uint32_t vps;               // whole 16-byte vectors per stripe output
    uint32_t tail;              // bytes after them (0..15): the last, partial vector
    uint32_t tps;               // tiles per stripe
    uint32_t ntiles;
    uint32_t nsrc;
    uint32_t dense;             // GATHER = 1: stripes[s].first_src == s * nsrc for every s
    unsigned long long *ctr;    // work-queue counter (per queue)
    unsigned long long base;    // counter value at the start of this launch
    uint32_t grab;              // tiles per queue grab (NSRC 1..4 instantiations; others take 1)
};

// One tile of a descriptor batch, written on the device by desc_tiles.  The
// record is self-contained so that the fold needs ONE dependent scalar load
// per tile before its data loads (in r01 every extra dependent round trip
// in the per-tile chain cost 5-15 % of HBM rate at 1-2 workgroups per CU).
// Plain tiles are one subtile of tile_bytes and list the sources reaching
// into it, sorted longest first: [0, nfull) cover it, [nfull, nany) end
// inside it (src_bytes readable bytes); zero padding is not listed.  Grouped
// tiles are m > 1 consecutive full subtiles covered by the same nfull <= 4
// sources and no others (nfull * m <= 8 rows, so a grouped tile moves about
// as many bytes as an 8-source one -- group_rows: on config-5 shapes a
// third of the subtiles are covered by a single source).  General tiles take
// the table path, stripe / subtile / first_src in src_bytes[0..2]: window
// replay (per-lane path), or more than kTileSrcs sources reaching in
// (kTileWide, counts in meta: eight-at-a-time folds from the staged run).
constexpr int kTileSrcs = 8;
struct alignas(64) DescTile {
    uint64_t dst;                   // output address of this tile's first subtile
    uint32_t out_bytes;             // output bytes of the tile
    uint32_t meta;                  // nfull | nany << 8 | (m - 1) << 16 | kTileGeneral
    uint64_t src[kTileSrcs];        // source address + offset of the tile's first subtile
    uint32_t src_bytes[kTileSrcs];  // readable bytes from src[k] (plain tiles)
};
constexpr uint32_t kTileGeneral = 0x80000000u;
constexpr uint32_t kTileWide = 0x40000000u;  // with kTileGeneral: > kTileSrcs sources, no window
static_assert(sizeof(DescTile) == 128, "tile record is two s_load_dwordx16");
static_assert(kTileSrcs == 8, "xor_desc_args counts covering sources in scalar registers");

// Rows (source x subtile pairs) of a grouped tile for U vectors per lane:
// every load of the tile is in flight at once, so C*M*U <= 32 keeps the
// fold within the register budget of the 8-source plain fold.
__host__ __device__ constexpr int group_rows(int U) { return U >= 16 ? 2 : U >= 8 ? 4 : 8; }

// How one stripe is cut into tiles.  Shared by the host (tile counts per
// stripe) and desc_tiles (records, one lane per subtile), so both cut
// identically.  A subtile i is groupable when the same nf sources cover it
// completely, nobody else reaches into it, its output is full and 2*nf <=
// group_rows.  A tile starts at every non-groupable subtile and, inside a run
// of groupable subtiles with the same nf, at the run start and at every
// subtile index that is a multiple of group_rows / nf (local rule: a lane
// decides from subtiles i-1 and i alone).
struct SubClass {
    uint32_t nf, na;  // sources covering the subtile / reaching into it
    bool g;           // groupable
};

// len_at(k): length of source k of the stripe's run, sorted longest first.
template <typename LenAt>
__host__ __device__ inline SubClass sub_class(LenAt len_at, uint32_t nsrc, uint64_t out_len, uint64_t sub_bytes,
                                              uint64_t i) {
    const uint64_t off = i * sub_bytes, end = off + sub_bytes;
    uint32_t nf = 0, na = 0;
    for (uint32_t k = 0; k < nsrc; k++) {
        const uint64_t len = len_at(k);
        nf += len >= end;
        na += len > off;
    }
    const uint32_t rows = (uint32_t)group_rows((int)(sub_bytes / 4096u));
    return SubClass{nf, na, nf == na && nf >= 1 && 2 * nf <= rows && end <= out_len};
}

__host__ __device__ inline bool tile_starts(const SubClass &prev, const SubClass &cur, uint64_t i, uint64_t sub_bytes) {
    if (!cur.g || i == 0 || !prev.g || prev.nf != cur.nf) return true;
    const uint32_t mmax = (uint32_t)group_rows((int)(sub_bytes / 4096u)) / cur.nf;
    return i % mmax == 0;
}

// Tiles of one stripe, by the rule above, in O(nsrc): between breakpoints
// (a source stops covering, a source stops reaching in, the output turns
// partial) every subtile has the same class.  Equal to counting tile_starts
// over every subtile (tests/native/tile_cut_test.cpp checks both).
template <typename LenAt>
__host__ __device__ inline uint64_t count_tiles(LenAt len_at, uint32_t nsrc, uint64_t out_len, uint64_t sub_bytes,
                                                bool window) {
    const uint64_t nsub = (out_len + sub_bytes - 1) / sub_bytes;
    if (window) return nsub;
    const uint32_t rows = (uint32_t)group_rows((int)(sub_bytes / 4096u));
    uint32_t nf = nsrc, na = nsrc;
    SubClass prev{0, 0, false};
    uint64_t count = 0, j = 0;
    while (j < nsub) {
        const uint64_t off = j * sub_bytes, end = off + sub_bytes;
        while (na > 0 && len_at(na - 1) <= off) na--;
        while (nf > 0 && len_at(nf - 1) < end) nf--;
        const SubClass cur{nf, na, nf == na && nf >= 1 && 2 * nf <= rows && end <= out_len};
        uint64_t jn = nsub;
        if (nf > 0 && len_at(nf - 1) / sub_bytes < jn) jn = len_at(nf - 1) / sub_bytes;
        if (na > 0 && (len_at(na - 1) + sub_bytes - 1) / sub_bytes < jn) jn = (len_at(na - 1) + sub_bytes - 1) / sub_bytes;
        if (end <= out_len && out_len / sub_bytes < jn) jn = out_len / sub_bytes;
        if (jn <= j) jn = j + 1;  // cannot happen (see the breakpoints); keeps progress
        if (!cur.g) {
            count += jn - j;
        } else {
            const uint64_t mmax = rows / cur.nf;
            count += tile_starts(prev, cur, j, sub_bytes);
            if (jn - 1 >= j + 1) count += (jn - 1) / mmax - j / mmax;  // multiples of mmax in [j+1, jn-1]
        }
        prev = cur;
        j = jn;
    }
    return count;
}

// Device-side form of one stripe descriptor batch.
struct DescBatch {
    const bcp_stripe *stripes;  // [nstripes]
    const bcp_source *sources;  // staged runs, each sorted by len, longest first
    const uint32_t *tile_start; // [nstripes + 1] prefix of tiles per stripe
    DescTile *tiles;            // [ntiles] (device; written by desc_tiles)
    uint32_t nstripes;
    uint32_t ntiles;
    uint32_t tile_bytes;        // bytes of output per tile
    unsigned long long *ctr;    // work-queue counter (per queue), as StreamArgs
    unsigned long long base;
};

// A small descriptor batch passed whole in the kernel arguments
// (xor_desc_args): <= kArgStripes stripes, <= kArgSources sources in all, each
// stripe's run sorted longest first, <= kTileSrcs per stripe, no window.
constexpr int kArgStripes = 16;
constexpr int kArgSources = 128;  // DescArgs stays < 3 KiB of the 4 KiB kernarg space
struct DescArgs {
    uint64_t dst[kArgStripes];
    uint64_t out_len[kArgStripes];
    uint32_t first[kArgStripes];
    uint32_t nsrc[kArgStripes];
    uint32_t tile_start[kArgStripes + 1];  // prefix of tiles (one per subtile)
    uint32_t nstripes, ntiles;
    uint64_t src_ptr[kArgSources];
    uint64_t src_len[kArgSources];
    unsigned long long *ctr;  // work-queue counter (per queue), as StreamArgs
    unsigned long long base;
};

// ---------------------------------------------------------------------------
// Resident fold ring (bcp_ring_*, include/bcp.h).  One launch stays on the
// device and folds stripes that callers publish into a ring of descriptors
// in pinned host memory: no launch and no stream sync per stripe (the P
// role's protocol folds one window at a time, task_processing.c:203-226).
//   ticket  one piece of a stripe (<= kRingPieceMax output bytes), numbered
//           from 0 in publication order; entry = ticket % K
//   tile    one of a ticket's `parts` (its output / parts, rounded up to
//           4 KiB, <= 32 KiB), the unit a worker workgroup claims
// Host: writes the entry, then seq = ticket + 1 (release).  Device: one
// watcher wave polls seq in ticket order, copies the entry to HBM and
// advances `pub`; workers claim the parts of the tickets below `pub` in
// ticket order (fold_ring, bcp_kernels.hip), and the last tile of a ticket
// writes done[entry] = ticket + 1 to host memory.  After idle_ticks without a new ticket (or on stop) the watcher
// writes the first ticket it did not take to *closed and the launch drains:
// every ticket below it was folded, none at or above it was touched, and the
// host relaunches from there (bcp_engine.hip, ring_live_locked).
// ---------------------------------------------------------------------------
constexpr int kRingMaxParts = 16;                       // tiles per ticket, at most
constexpr uint64_t kRingTileBytes = (uint64_t)32 << 10;  // a tile's output, at most
constexpr uint64_t kRingPieceMax = kRingMaxParts * kRingTileBytes;
struct RingEntry {
    unsigned long long seq;  // ticket + 1 once published (written last)
    uint64_t dst;            // output of this piece
    uint64_t out_len;        // <= kRingPieceMax
    uint32_t nsrc, parts;    // parts: tiles of this piece, ceil(out_len / 32 KiB) (1..16)
    uint64_t rsv[4];
    bcp_source src[BCP_MAX_SOURCES];  // offset to the piece, len clamped to it
    uint64_t pad[8];
};
static_assert(sizeof(RingEntry) == 1024, "one 16-byte load per lane of one wave copies an entry");
static_assert(offsetof(RingEntry, parts) == 28, "the watcher reads parts from lane 1's word, dword 3");
// Host-side control words the device writes or reads (pinned, coherent).
struct RingCtl {
    unsigned long long closed;  // first ticket the last launch did not take; ~0 while a launch is live
    unsigned long long pad0[15];
    unsigned int stop;          // host: drain and exit once idle
    unsigned int pad1[31];
    // then done[K * kRingDoneStride]
};
constexpr int kRingDoneStride = 8;  // one 64-byte line per entry's done word
// Device-side state (HBM): the ticket being claimed, announced tickets, quit flag, each
// on its own 128-byte line; then claim[K] and cnt[K] (per entry: ticket <<
// 16 | parts << 8 | parts claimed, and ticket << 16 | tiles folded; set by
// the watcher when it announces the entry's ticket) and the entries' copies.
struct RingState {
    unsigned long long cur;     // the ticket being claimed, relative to the launch's base
    unsigned long long pad0[15];
    unsigned long long pub;     // tickets announced (absolute; 0 at launch)
    unsigned long long pad1[15];
    unsigned int quit;          // the watcher closed this launch
    unsigned int pad2[31];
};
struct RingArgs {
    const RingEntry *host;           // [K] pinned host memory
    unsigned long long *done;        // host, [K * kRingDoneStride]
    unsigned long long *closed;      // host (RingCtl::closed)
    const unsigned int *stop;        // host (RingCtl::stop)
    RingState *state;                // HBM
    unsigned long long *claim;       // HBM [K]
    unsigned long long *cnt;         // HBM [K]
    RingEntry *copy;                 // HBM [K]
    unsigned long long base;         // first ticket of this launch
    unsigned long long idle_ticks;   // watcher: close after this long without a ticket (s_memrealtime ticks)
    unsigned long long hard_ticks;   // worker: give up waiting after this long (no watcher)
    uint32_t kmask, kshift;          // K - 1, log2 K
};

// Kernel launchers (bcp_kernels.hip).  All return hipError_t.
// Streaming fold.  Consumes ceil(ntiles / grab) + grid counts of a.ctr; the
// caller clamps grid to [1, ntiles].
hipError_t launch_xor_stream(hipStream_t st, int grid, int vecs, bool gather, const StreamArgs &a);
uint32_t stream_tiles_per_stripe(uint64_t chunk_bytes, int vecs);
// Descriptor batch: desc_tiles (one wave per stripe writes its tile records
// into b.tiles), then the fold; same work-queue accounting as
// launch_xor_stream.
hipError_t launch_desc_tiles(hipStream_t st, const DescBatch &b);
hipError_t launch_xor_desc(hipStream_t st, int grid, int vecs, const DescBatch &b);
// Small batch in the arguments; same work-queue accounting (ntiles + grid).
hipError_t launch_xor_desc_args(hipStream_t st, int grid, int vecs, const DescArgs &a);
// Resident fold ring: 1 watcher workgroup + `workers`.
hipError_t launch_fold_ring(hipStream_t st, int workers, const RingArgs &a);
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
