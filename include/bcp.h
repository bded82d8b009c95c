/*
 * bcp.h -- C ABI of the MI355X chunk-XOR parity engine (libbcp.so).
 *
 * Drop-in boundary for the arithmetic seam of runefriborg/beegfs-chunk-parity:
 *
 *   static void xor_parity(uint8_t *restrict dst, size_t nbytes,
 *                          const uint8_t *data, int nsources);
 *       -- src/beegfs-raid5/common/task_processing.c:96-109
 *
 * which the P role (parity_generator, task_processing.c:117-245) calls once
 * per 10 MiB window.  This ABI replaces it with
 *   (1) bcp_xor_parity(): the same signature and semantics, on the GPU;
 *   (2) an engine/queue lifecycle (one queue = one HIP stream pair, one per
 *       lane thread, gen/main.c:821-845 runs 12 lanes per rank);
 *   (3) batched asynchronous submission of stripe descriptors, because one
 *       512 KiB x 8 stripe is ~1 us of HBM time -- far below a launch;
 *   (4) query / wait on completion, and HIP-event timing for the bench.
 *
 * Conventions: plain C types only; every function returns 0 or a negative
 * errno value (-EINVAL, -ENOMEM, -ENODEV, -EIO, -EAGAIN); nothing throws
 * across the ABI.  An engine is thread-safe; a queue belongs to one thread
 * at a time.  There is no CPU fallback: without a usable gfx950 device every
 * compute entry point returns -ENODEV.
 *
 * Semantics of every XOR entry point (bit-exact with the reference,
 * SURVEY.md §8(a)):
 *   out[j] = XOR_k  src_k'[j]         for 0 <= j < out_len
 * where src_k'[j] = src_k[j] if j < len_k else 0 (zero padding), except when
 * a stripe carries window W != 0: then byte j of window w = j / W of a source
 * with last readable window lw_k = (len_k - 1) / W and w > lw_k replays
 * window lw_k (chunk_sender never refills its buffer after EOF,
 * task_processing.c:291-308, quirk A3-q1).  len_k = 0 always reads zeros.
 */
#ifndef BCP_H
#define BCP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 4 (r06): the resident fold ring (bcp_ring_*) and the P role's fold
 * through it (bcp_task.h, bcp_task_set_fold_ring) added.
 * 3 (r05): the pipeline's MAP read mode (BCP_READ_MAP), its
 * bcp_pipeline_timing fields and bcp_host_register_dma_src removed.
 * 2 (r04): bcp_task.h's bcp_run_stats gained `refused`, bcp_pipeline_opts
 * `read_mode`, bcp_pipeline_timing the MAP fields; bcp_host_register_dma_src
 * added.  Since 1 (r03): fold modes ZERO_COPY, STAGED, STREAMED and
 * DEVICE_ROWS, bcp_dev_alloc_hostwrite and the engine keys they used were
 * removed, and the default window padding became BCP_PAD_AUTO
 * ("ABI history"). */
#define BCP_ABI_VERSION 4
#define BCP_MAX_SOURCES 56                  /* MAX_STORAGE_TARGETS, common.h:18 */
#define BCP_WINDOW_BYTES (10u * 1024u * 1024u) /* FILE_TRANSFER_BUFFER_SIZE, task_processing.c:20 */

typedef struct bcp_engine bcp_engine;
typedef struct bcp_queue bcp_queue;

/* One source of a stripe: device address and readable length in bytes. */
typedef struct bcp_source {
    uint64_t ptr;
    uint64_t len;
} bcp_source;

/* One stripe: out[0..out_len) = XOR of sources[first_src .. first_src+nsrc).
 * window = 0 for plain zero padding, or the transfer window (normally
 * BCP_WINDOW_BYTES, must be a multiple of 16) when the stream exceeded one
 * window and the reference's replay semantics apply. */
typedef struct bcp_stripe {
    uint64_t dst;
    uint64_t out_len;
    uint32_t first_src;
    uint32_t nsrc;
    uint64_t window;
} bcp_stripe;

/* ---- library / device ------------------------------------------------- */
int bcp_abi_version(void);
/* Number of visible HIP devices (0 without a GPU; never fails for that). */
int bcp_device_count(int *count);
/* Human-readable message for a return code. */
const char *bcp_strerror(int rc);

/* ---- engine lifecycle ------------------------------------------------- */
/* Create an engine bound to `device` (HIP ordinal). */
int bcp_engine_create(int device, bcp_engine **out);
int bcp_engine_destroy(bcp_engine *eng);
/* Device properties the bench reports: CU count and the name string. */
int bcp_engine_info(bcp_engine *eng, int *num_cus, char *name, size_t name_cap);
/* PCI bus id of the engine's device ("dddd:bb:dd.f"): identifies the physical
 * GPU across processes whatever HIP_VISIBLE_DEVICES renumbers (bench.py counts
 * distinct devices with it, so ranks sharing a GPU are not reported as more
 * GPUs).  -EINVAL if bus_id_cap is too small. */
int bcp_engine_pci_bus_id(bcp_engine *eng, char *bus_id, size_t bus_id_cap);

/* ---- queues (one in-order HIP stream each) ----------------------------- */
/* Work on one queue runs in submission order.  Overlap (copy beside compute)
 * comes from using two queues ordered by events, as the pipeline does. */
int bcp_queue_create(bcp_engine *eng, bcp_queue **out);
int bcp_queue_destroy(bcp_queue *q);
/* Block until everything submitted to q has finished. */
int bcp_queue_sync(bcp_queue *q);
/* 0 if idle, -EAGAIN if work is pending. */
int bcp_queue_query(bcp_queue *q);

/* ---- completion handles (HIP events) ---------------------------------- */
typedef struct bcp_event bcp_event;
int bcp_event_create(bcp_engine *eng, bcp_event **out);
int bcp_event_destroy(bcp_event *ev);
/* Mark the current tail of q; later bcp_queue_wait_event() / bcp_event_sync()
 * see everything submitted to q before this call. */
int bcp_event_record(bcp_event *ev, bcp_queue *q);
/* Make later work on q wait (on the device) for ev. */
int bcp_queue_wait_event(bcp_queue *q, bcp_event *ev);
/* Host wait; bcp_event_query: 0 done, -EAGAIN pending. */
int bcp_event_sync(bcp_event *ev);
int bcp_event_query(bcp_event *ev);

/* ---- memory ----------------------------------------------------------- */
int bcp_dev_alloc(bcp_engine *eng, size_t bytes, void **dptr);
int bcp_dev_free(bcp_engine *eng, void *dptr);
/* Pinned (page-locked) host memory for staging (registered huge-page memory
 * by default, option host_registered). */
int bcp_host_alloc(bcp_engine *eng, size_t bytes, void **hptr);
/* Pinned host memory that kernels read and write in place over PCIe
 * (coherent, mapped at the same address on the device): the P role's window
 * rows and parity blocks (bcp_task.c, the fold server's shared arena), which
 * the fold reads and writes in place.  Free with bcp_host_free. */
int bcp_host_alloc_mapped(bcp_engine *eng, size_t bytes, void **hptr);
int bcp_host_free(bcp_engine *eng, void *hptr);
/* Register caller-owned host memory (e.g. a shared mapping other processes
 * write) so kernels read and write it in place at the same address, like
 * bcp_host_alloc_mapped memory; -EIO if the device cannot address it at its
 * host address.  Unregister before the memory is unmapped or reused. */
int bcp_host_register(bcp_engine *eng, void *hptr, size_t bytes);
int bcp_host_unregister(bcp_engine *eng, void *hptr);
/* Async copies, in order on q. */
int bcp_h2d_async(bcp_queue *q, void *dst, const void *src, size_t bytes);
int bcp_d2h_async(bcp_queue *q, void *dst, const void *src, size_t bytes);
int bcp_d2d_async(bcp_queue *q, void *dst, const void *src, size_t bytes);
/* Pitched H2D: `rows` rows of `row_bytes`, host pitch hpitch, device pitch dpitch. */
int bcp_h2d_2d_async(bcp_queue *q, void *dst, size_t dpitch, const void *src,
                     size_t hpitch, size_t row_bytes, size_t rows);
int bcp_memset_async(bcp_queue *q, void *dst, int value, size_t bytes);

/* ---- XOR kernels (device pointers, asynchronous on q) ------------------ */
/* Uniform stripes: src is [nstripes][nsrc][chunk_bytes] contiguous, dst is
 * [nstripes][chunk_bytes].  Any alignment / length is accepted; 16-byte
 * aligned pointers with chunk_bytes % 16 == 0 take the streaming fast path. */
int bcp_xor_uniform_async(bcp_queue *q, void *dst, const void *src,
                          uint64_t nstripes, uint32_t nsrc,
                          uint64_t chunk_bytes);
/* Same, but sources given by a stride: source k of stripe s starts at
 * src + s*stripe_stride + k*src_stride; output s at dst + s*dst_stride. */
int bcp_xor_strided_async(bcp_queue *q, void *dst, uint64_t dst_stride,
                          const void *src, uint64_t stripe_stride,
                          uint64_t src_stride, uint64_t nstripes,
                          uint32_t nsrc, uint64_t chunk_bytes);
/* Descriptor batch (variable lengths, zero padding, rebuild truncation,
 * window replay).  Host arrays are copied before return. */
int bcp_xor_stripes_async(bcp_queue *q, const bcp_stripe *stripes,
                          uint32_t nstripes, const bcp_source *sources,
                          uint32_t nsources);

/* ---- resident fold ring ------------------------------------------------ */
/* One kernel launch that stays on the device and folds stripes published
 * into a ring of descriptors in pinned host memory: no launch and no stream
 * sync per stripe.  For callers that fold one small stripe at a time from
 * many threads -- the P role's windows, task_processing.c:203-226, 12 lanes
 * per rank (gen/main.c:821-889) -- where a launch + sync per window is the
 * bound.  Same semantics as bcp_xor_stripes_async for one stripe with
 * window 0 (sources and output anywhere the device can address: pinned
 * mapped host memory or device memory; any alignment and length).
 *
 * The launch starts on the first submission and ends by itself after
 * idle_us without one (it is relaunched on the next); bcp_ring_destroy ends
 * it at once.  While it is live it holds 1 + `workers` workgroups of the
 * device, and HIP calls that wait for the whole device (hipFree,
 * hipHostUnregister, device synchronisation) wait until it idles out.
 * A ring is thread-safe: any thread may submit and wait. */
typedef struct bcp_ring bcp_ring;
/* workers: worker workgroups (0 = default 64, at most 4096); idle_us: idle
 * time before the launch ends (0 = default 5000, at most 10 s). */
int bcp_ring_create(bcp_engine *eng, int workers, int idle_us, bcp_ring **out);
/* Publish stripe (window must be 0; nsrc <= BCP_MAX_SOURCES; out_len <=
 * 255 x 512 KiB) with its sources[0 .. nsrc) (stripe->first_src is ignored).
 * Returns at once with a handle for bcp_ring_wait / _query; blocks only while
 * the ring is full.  The caller keeps sources and output untouched until the
 * handle completes. */
int bcp_ring_submit(bcp_ring *r, const bcp_stripe *stripe, const bcp_source *sources, uint64_t *handle);
/* Block until the stripe behind handle is folded and visible to the host;
 * -EIO if the ring's launch failed. */
int bcp_ring_wait(bcp_ring *r, uint64_t handle);
/* 0 done, -EAGAIN pending, -EIO failed. */
int bcp_ring_query(bcp_ring *r, uint64_t handle);
/* Stops the launch (pending stripes are folded first) and frees the ring;
 * every handle must have been waited for. */
int bcp_ring_destroy(bcp_ring *r);
/* How waiters wait: spin spin_us, then sleep sleep_us between looks (0:
 * sched_yield); defaults from the engine options ring_spin_us /
 * ring_sleep_us (4 / 10). */
int bcp_ring_set_wait(bcp_ring *r, int spin_us, int sleep_us);
/* Pieces published (a stripe is cut into 512 KiB pieces) and launches made
 * since the ring was created. */
int bcp_ring_stats(bcp_ring *r, uint64_t *pieces, uint64_t *launches);

/* ---- drop-in for xor_parity (task_processing.c:96-109) ----------------- */
/* Host pointers, synchronous, same contract as the reference: dst gets
 * XOR of the nsources rows of `data` ([nsources][nbytes]).  nsources is
 * 1..BCP_MAX_SOURCES (-EINVAL otherwise: the P role never folds zero rows,
 * it unlinks the parity chunk instead, task_processing.c:141-144).  Runs on a
 * process-wide engine (device from $BCP_DEVICE, default 0) and a per-thread
 * queue with pinned staging; returns -ENODEV without a GPU. */
int bcp_xor_parity(uint8_t *dst, size_t nbytes, const uint8_t *data,
                   int nsources);

/* ---- verification / synthetic data (device) --------------------------- */
/* Fill with the splitmix64 byte stream: byte b = byte (b&7) of
 * splitmix64(seed + (byte_offset + b)/8).  Same stream as the oracle's
 * oracle_fill_synthetic, so checks need no bulk host copy. */
int bcp_dev_fill_synthetic_async(bcp_queue *q, void *dst, uint64_t bytes,
                                 uint64_t seed, uint64_t byte_offset);
/* XOR-fold of a buffer into 16 bytes (out16_dev is device memory). */
int bcp_dev_xor_fold_async(bcp_queue *q, const void *src, uint64_t bytes,
                           void *out16_dev);
/* Count of differing bytes between two device buffers into *out_dev (u64). */
int bcp_dev_compare_async(bcp_queue *q, const void *a, const void *b,
                          uint64_t bytes, void *out_dev);

/* ---- timing (HIP events on the queue's stream) ------------------------- */
int bcp_queue_mark(bcp_queue *q, int slot);           /* slot 0..63 */
int bcp_queue_elapsed_ms(bcp_queue *q, int slot_from, int slot_to,
                         float *ms);

/* Tuning knobs for the fast path (bench / autotune only; 0 = default). */
int bcp_set_tuning(bcp_engine *eng, int blocks_per_cu, int vecs_per_thread);
/* Named knob (unknown keys and out-of-range values: -EINVAL):
 *  uniform streaming kernel: "blocks_per_cu" (1..32, default 1),
 *   "vecs_per_thread" (1, 2, 4, 8; 0 = the default: 8, or 4 / 2 for batches
 *   of few tiles), "stream_grid" (explicit workgroup count; 0 = the default,
 *   blocks_per_cu on 29 of every 32 CUs), "table_host_max" (bytes: a
 *   pointer table up to this size is read from pinned host memory instead of
 *   being copied first; default 4096);
 *  descriptor kernel (mixed sizes, windows, unaligned): "desc_blocks_per_cu"
 *   (0 = the default, one per CU; 1..32), "desc_vecs_per_thread" (1, 2, 4,
 *   8, 16; 0 = by batch size; 16 = 64 KiB subtiles, batches through
 *   desc_tiles only -- small batches in the kernel arguments use 8),
 *   "desc_grid" (explicit workgroup count; 0 = default), "desc_args_max"
 *   (batches of at most this many stripes, 0..16, travel in the kernel
 *   arguments; default 16), "desc_table_host_max" (as table_host_max;
 *   default 131072), "desc_reuse_records" (1: a batch resubmitted on a ring
 *   slot with byte-identical staged tables reuses that slot's tile records;
 *   default 0, an A/B knob);
 *  resident fold ring: "ring_spin_us" (a waiter spins this long, default 4)
 *   and "ring_sleep_us" (then sleeps this long between looks, default 10;
 *   0 = sched_yield instead);
 *  memory: "contiguous_alloc" (1: bcp_dev_alloc requests physically
 *   contiguous memory for buffers of 64 MiB and more; default 0),
 *   "host_registered" (bcp_host_alloc / bcp_host_alloc_mapped: 1 = ordinary
 *   huge-page memory registered with HIP, the default -- CPU copies into and
 *   out of it run at malloc speed; 0 = hipHostMalloc; env
 *   BCP_HOST_REGISTERED).
 * The kernels' schedule (device-wide tile work queue), register budgets and
 * load windows are fixed: the alternatives lost the r01-r03 sweeps
 * (DESIGN.md section 4). */
int bcp_set_option(bcp_engine *eng, const char *key, int value);
/* Current value of a named knob (same keys), or of the engine's latest
 * launch: "last_stream_vecs" (vecs_per_thread of the streaming kernel),
 * "last_desc_vecs" and "last_desc_form" (descriptor kernel: 1 = desc_tiles +
 * xor_desc, 2 = xor_desc_args). */
int bcp_get_option(bcp_engine *eng, const char *key, int *value);
/* Timer slots for bcp_queue_mark / bcp_queue_elapsed_ms. */
#define BCP_TIMER_SLOTS 64

#ifdef __cplusplus
}
#endif

#endif /* BCP_H */
