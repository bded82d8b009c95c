// bcp_engine.hip -- C ABI of libbcp.so (include/bcp.h): engine, queues,
// events, memory, XOR submission and the xor_parity drop-in.
//
// The engine replaces the CPU fold at task_processing.c:211 (xor_parity,
// :96-109).  Design points (MI355X):
//  * one in-order HIP stream per queue; lanes (gen/main.c:821-845) each own a
//    queue, so twelve lanes overlap their copies and kernels on the device;
//  * descriptor batches are staged through a per-queue ring of pinned slots
//    and uploaded on the queue's copy stream (the kernel's stream waits by
//    event), so submission never synchronises with earlier work of the same
//    queue and the upload for launch k+1 overlaps kernel k;
//  * grids are persistent: CUs x blocks_per_cu workgroups of 256 threads;
//    both kernels take tiles from a per-queue device work queue (monotone
//    counter, base advanced on the host per launch).
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <new>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "bcp_internal.h"

using namespace bcp;

struct bcp_engine {
  int device = 0;
  int num_cus = 0;
  char name[256] = {0};
  Tuning tuning;
  pthread_mutex_t lock = PTHREAD_MUTEX_INITIALIZER;
  std::atomic<int> last_stream_vecs{0};  // U of the latest xor_stream launch (tools)
  std::atomic<int> last_desc_vecs{0};    // U of the latest descriptor-kernel launch (tools)
  std::atomic<int> last_desc_form{0};    // 1 xor_desc (desc_tiles), 2 xor_desc_args
};

namespace {

constexpr int kRingSlots = 4;
constexpr int kTimerSlots = 64;

struct DescSlot {
  void *host = nullptr;   // pinned staging
  void *dev = nullptr;    // device copy
  size_t cap = 0;
  hipEvent_t done = nullptr;    // recorded after the kernel that read `dev`
  hipEvent_t copied = nullptr;  // recorded on the copy stream after host -> dev (or after desc_tiles there)
  bool used = false;
  DescTile *tiles = nullptr;    // this slot's tile records (desc_tiles -> xor_desc)
  size_t tiles_cap = 0;         // in records
  // desc_reuse_records: the launch parameters and a copy of the staged
  // tables the records were made from; rec_ok only while `dev` and `tiles`
  // still hold them (any other use of the slot clears it)
  uint64_t rec_key = 0;
  void *rec_copy = nullptr;
  size_t rec_len = 0;
  bool rec_ok = false;
};

}  // namespace

struct bcp_queue {
  bcp_engine *eng = nullptr;
  hipStream_t stream = nullptr;
  DescSlot ring[kRingSlots];
  int next_slot = 0;
  unsigned long long *qctr = nullptr;  // work-queue counter of xor_stream (device)
  unsigned long long qbase = 0;        // its value when the next launch starts
  hipEvent_t timer[kTimerSlots] = {};
  hipStream_t copy_stream = nullptr;   // descriptor-table uploads (created on first use)
  bool broken = false;                 // work-queue counter could not be restarted after a failed launch
};

struct bcp_event {
  bcp_engine *eng = nullptr;
  hipEvent_t ev = nullptr;
};

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
#define HIP_RC(expr)                                                            \
  do {                                                                          \
    hipError_t e_ = (expr);                                                     \
    if (e_ != hipSuccess) {                                                     \
      if (getenv("BCP_VERBOSE"))                                                \
        fprintf(stderr, "bcp: %s failed: %s (%s:%d)\n", #expr,                 \
                hipGetErrorString(e_), __FILE__, __LINE__);                     \
      return hip_to_errno(e_);                                                  \
    }                                                                           \
  } while (0)

static int hip_to_errno(hipError_t e) {
  switch (e) {
    case hipSuccess: return 0;
    case hipErrorOutOfMemory: return -ENOMEM;
    case hipErrorNoDevice:
    case hipErrorInvalidDevice: return -ENODEV;
    case hipErrorInvalidValue: return -EINVAL;
    case hipErrorNotReady: return -EAGAIN;
    default: return -EIO;
  }
}

static int set_device(bcp_engine *e) {
  HIP_RC(hipSetDevice(e->device));
  return 0;
}

// Work-queue accounting after a launch that takes tiles from q->qctr.  On
// success the next launch starts `consumed` counts later.  On any error the
// kernel may or may not have taken counts, so the counter is restarted
// (memset on the stream, ordered after anything that did run) and the base
// reset; if even that fails the queue refuses further XOR work (-EIO)
// instead of starting a later launch partway through its tile range.
static int queue_launched(bcp_queue *q, hipError_t e, uint64_t consumed) {
  if (e == hipSuccess) {
    q->qbase += consumed;
    return 0;
  }
  if (hipMemsetAsync(q->qctr, 0, sizeof(unsigned long long), q->stream) == hipSuccess) q->qbase = 0;
  else q->broken = true;
  return hip_to_errno(e);
}

// Workgroups of the streaming kernel: stream_grid if set, else blocks_per_cu
// per CU on 29 of every 32 CUs (232 on MI355X): in interleaved A/B runs the
// slightly narrower grid beat a full one by 0.6-0.9 points of HBM peak on
// config-2 gen and tied on rebuild (profiles/r01/grid_*.jsonl: 240 against
// 256); with the waves_per_eu(6) budget, same-allocation sweeps put the
// optimum at 228-236 (232: +0.3 / +0.4 over 240 on gen, +0.1 on rebuild;
// profiles/r01/depth/ab9_grid_wpe6.jsonl, ab12_stream_grid_fine.jsonl).
static int grid_for(const bcp_engine *e) {
  if (e->tuning.stream_grid > 0) return e->tuning.stream_grid;
  int g = e->num_cus * e->tuning.blocks_per_cu * 29 / 32;
  return g > 0 ? g : 232;
}

// Workgroups of the descriptor kernel.  Auto (desc_blocks_per_cu 0): one
// per CU on every CU.  With the rolling load window (PIPE 5) that is the
// best grid for every non-uniform shape measured -- config-5 shapes +1.3
// points over the earlier 2 per CU, 1-4 MiB mixed +0.4, equal-length mixed
// +0.5 over 15/16 of the CUs, 16-wide +0.8 (tools/exp/desc_probe.py,
// profiles/r01/depth/ab10_desc_grid.jsonl, ab11_desc_grid_fine.jsonl).
// Uniform stripes would prefer 29/32 of the CUs, but they take xor_stream.
static int desc_grid_for(const bcp_engine *e) {
  if (e->tuning.desc_grid > 0) return e->tuning.desc_grid;
  const int bpc = e->tuning.desc_blocks_per_cu > 0 ? e->tuning.desc_blocks_per_cu : 1;
  const int g = e->num_cus * bpc;
  return g > 0 ? g : 256;
}

static bool stream_vecs_ok(int v) { return v == 1 || v == 2 || v == 4 || v == 8; }

// Tiles per work-queue grab for stripes of 1-4 sources (auto): two.  One
// tile per grab leaves N = 1 (a copy) at 62 % of HBM peak and N = 2 at 77 %,
// bound by the single counter; two per grab 84 / 83 %, N = 3..4 level or
// +0.5; three or more widen the address window and lose 2-6 points
// (profiles/r01/depth/ab15_narrow_stripes.jsonl, ab16_narrow_grab.jsonl).
static uint32_t stream_grab_auto(uint32_t nsrc) { return nsrc >= 1 && nsrc <= 4 ? 2u : 1u; }

// Vectors per lane (tile size) of one xor_stream launch.  Explicit tuning
// wins; auto (0) keeps U = 8 (32 KiB per source per tile, the large-batch
// optimum) unless the batch is small: with fewer than ~16 tiles per
// workgroup the last tiles of the queue leave most CUs idle, and halving the
// tile halves that tail.  Thresholds from tools/batch_curve.py
// (profiles/r01/batch_tune.jsonl, 8 x 512 KiB stripes): U = 2 for 1-2
// stripes (-38 %), U = 4 up to 128 stripes (-3..-25 %), U = 8 from 256.
// Stripes wider than 8 sources take U = 4 (the same ~256 KiB of loads per
// tile): 16-wide 74-75 -> 87 % of HBM peak, 12-wide level
// (profiles/r01/depth/ab5_wide_stream_tile_size.jsonl).
static int stream_vecs(const bcp_engine *e, uint64_t chunk_bytes, uint64_t nstripes, uint32_t nsrc) {
  if (e->tuning.vecs_per_thread) return e->tuning.vecs_per_thread;
  const uint64_t t8 = nstripes * stream_tiles_per_stripe(chunk_bytes, 8);
  const uint64_t g = (uint64_t)grid_for(e);
  if (t8 * 5 < g) return 2;
  if (t8 < 16 * g || nsrc > 8) return 4;
  return 8;
}
static bool desc_vecs_ok(int v) { return v == 1 || v == 2 || v == 4 || v == 8 || v == 16; }

// Vectors per lane of the descriptor kernel.  Explicit tuning wins; auto (0,
// the default): 32 KiB tiles (U = 8) once the batch has twice as many of them
// as the grid has workgroups, 16 KiB from half the grid, 8 KiB below -- a
// one-stripe batch of 512 KiB is 16 tiles at U = 8, i.e. 16 CUs busy; 64 at
// U = 2 (the streaming kernel's small-batch rule, stream_vecs).
static int desc_vecs_for(const bcp_engine *e, uint64_t tiles8);

static bool aligned16(uint64_t x) { return (x & 15u) == 0; }

// A slot none of whose kernels is still running.
static bool slot_idle(DescSlot *s) { return !s->used || hipEventQuery(s->done) == hipSuccess; }

// Grow an idle slot's tables to at least `bytes`.
static int slot_grow(DescSlot *s, size_t bytes) {
  s->rec_ok = false;
  if (s->host) HIP_RC(hipHostFree(s->host));
  if (s->dev) HIP_RC(hipFree(s->dev));
  s->host = s->dev = nullptr;
  s->cap = 0;
  size_t cap = 64 * 1024;
  while (cap < bytes) cap *= 2;
  HIP_RC(hipHostMalloc(&s->host, cap, hipHostMallocDefault));
  HIP_RC(hipMalloc(&s->dev, cap));
  s->cap = cap;
  return 0;
}

// Reserve a ring slot of at least `bytes`; waits only if that slot's
// previous kernel has not finished (kRingSlots submissions ago).  A slot
// that must grow grows the queue's other idle slots with it: a queue's
// batches are alike, and a slot first reached later (the fourth submission:
// a block's first timed launch after three warm-up ones) would otherwise
// allocate on the path to its kernel.
static int ring_acquire(bcp_queue *q, size_t bytes, DescSlot **out) {
  DescSlot *s = &q->ring[q->next_slot];
  q->next_slot = (q->next_slot + 1) % kRingSlots;
  if (s->used) HIP_RC(hipEventSynchronize(s->done));
  if (s->cap < bytes) {
    int rc = slot_grow(s, bytes);
    if (rc) return rc;
    for (int j = 0; j < kRingSlots; j++) {
      DescSlot *o = &q->ring[j];
      if (o != s && o->cap < bytes && slot_idle(o) && (rc = slot_grow(o, bytes))) return rc;
    }
  }
  if (!s->done) HIP_RC(hipEventCreateWithFlags(&s->done, hipEventDisableTiming));
  if (!s->copied) HIP_RC(hipEventCreateWithFlags(&s->copied, hipEventDisableTiming));
  *out = s;
  return 0;
}

// Upload a slot's tables on the queue's copy stream and make the compute
// stream wait for them: the upload for launch k+1 overlaps kernel k instead
// of sitting between them in stream order.  (The slot's previous kernel has
// finished: ring_acquire waited for it.)  Tables of at most host_max bytes
// are not copied: the kernels read them from the pinned slot over PCIe,
// which for small batches costs less than the copy and the cross-stream wait
// (tools/batch_curve.py, profiles/r01/batch/).  Returns the tables' address
// as the kernels see it.
// compute_waits = false: the caller enqueues more on the copy stream (the
// descriptor batch's desc_tiles) and makes the compute stream wait after it.
static int stage_tables(bcp_queue *q, DescSlot *slot, size_t bytes, size_t host_max, char **tables,
                        bool compute_waits = true) {
  if (bytes <= host_max) {
    *tables = (char *)slot->host;
    return 0;
  }
  if (!q->copy_stream) HIP_RC(hipStreamCreateWithFlags(&q->copy_stream, hipStreamNonBlocking));
  HIP_RC(hipMemcpyAsync(slot->dev, slot->host, bytes, hipMemcpyHostToDevice, q->copy_stream));
  if (compute_waits) {
    HIP_RC(hipEventRecord(slot->copied, q->copy_stream));
    HIP_RC(hipStreamWaitEvent(q->stream, slot->copied, 0));
  }
  *tables = (char *)slot->dev;
  return 0;
}

// ---------------------------------------------------------------------------
// library / device
// ---------------------------------------------------------------------------
extern "C" int bcp_abi_version(void) { return BCP_ABI_VERSION; }

// Set once a HIP runtime with a device was initialised by this library: a
// forked child cannot use it (bcp_gen_run_procs refuses to fork then).
static std::atomic<int> g_hip_touched{0};
extern "C" int bcpi_hip_touched(void) { return g_hip_touched.load(std::memory_order_relaxed); }

extern "C" int bcp_device_count(int *count) {
  if (!count) return -EINVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  if (n > 0) g_hip_touched.store(1, std::memory_order_relaxed);
  *count = n;
  return 0;
}

extern "C" const char *bcp_strerror(int rc) {
  switch (rc) {
    case 0: return "ok";
    case -EINVAL: return "invalid argument";
    case -ENOMEM: return "out of memory";
    case -ENODEV: return "no usable HIP device";
    case -EAGAIN: return "work pending";
    case -EIO: return "HIP runtime error";
    default: return "unknown error";
  }
}

// ---------------------------------------------------------------------------
// engine
// ---------------------------------------------------------------------------
extern "C" int bcp_engine_create(int device, bcp_engine **out) {
  if (!out) return -EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -ENODEV;
  g_hip_touched.store(1, std::memory_order_relaxed);
  if (device < 0 || device >= n) return -ENODEV;
  hipDeviceProp_t prop;
  HIP_RC(hipGetDeviceProperties(&prop, device));
  bcp_engine *e = new (std::nothrow) bcp_engine();
  if (!e) return -ENOMEM;
  e->device = device;
  e->num_cus = prop.multiProcessorCount;
  snprintf(e->name, sizeof(e->name), "%s (%s)", prop.name, prop.gcnArchName);
  // (engine options are set with bcp_set_option; the one environment default
  // left is the host memory kind, for processes a caller cannot reach: ranks)
  if (const char *v = getenv("BCP_HOST_REGISTERED")) e->tuning.host_registered = atoi(v) ? 1 : 0;
  *out = e;
  return 0;
}

extern "C" int bcp_engine_destroy(bcp_engine *eng) {
  if (!eng) return -EINVAL;
  delete eng;
  return 0;
}

extern "C" int bcp_engine_info(bcp_engine *eng, int *num_cus, char *name, size_t name_cap) {
  if (!eng) return -EINVAL;
  if (num_cus) *num_cus = eng->num_cus;
  if (name && name_cap) snprintf(name, name_cap, "%s", eng->name);
  return 0;
}

extern "C" int bcp_engine_pci_bus_id(bcp_engine *eng, char *bus_id, size_t bus_id_cap) {
  if (!eng || !bus_id || bus_id_cap < 13 || bus_id_cap > (1u << 20)) return -EINVAL;
  HIP_RC(hipDeviceGetPCIBusId(bus_id, (int)bus_id_cap, eng->device));
  return 0;
}

extern "C" int bcp_set_option(bcp_engine *eng, const char *key, int value) {
  if (!eng || !key) return -EINVAL;
  int rc = 0;
  pthread_mutex_lock(&eng->lock);
  if (!strcmp(key, "blocks_per_cu") && value >= 1 && value <= 32) eng->tuning.blocks_per_cu = value;
  else if (!strcmp(key, "vecs_per_thread") && (value == 0 || stream_vecs_ok(value))) eng->tuning.vecs_per_thread = value;
  else if (!strcmp(key, "desc_blocks_per_cu") && value >= 0 && value <= 32) eng->tuning.desc_blocks_per_cu = value;
  else if (!strcmp(key, "desc_vecs_per_thread") && (value == 0 || desc_vecs_ok(value))) eng->tuning.desc_vecs = value;
  else if (!strcmp(key, "desc_args_max") && value >= 0 && value <= kArgStripes) eng->tuning.desc_args_max = value;
  else if (!strcmp(key, "stream_grid") && value >= 0 && value <= 65536) eng->tuning.stream_grid = value;
  else if (!strcmp(key, "desc_grid") && value >= 0 && value <= 65536) eng->tuning.desc_grid = value;
  else if (!strcmp(key, "contiguous_alloc") && (value == 0 || value == 1)) eng->tuning.contiguous_alloc = value;
  else if (!strcmp(key, "table_host_max") && value >= 0 && value <= (1 << 24)) eng->tuning.table_host_max = value;
  else if (!strcmp(key, "host_registered") && (value == 0 || value == 1)) eng->tuning.host_registered = value;
  else if (!strcmp(key, "desc_reuse_records") && (value == 0 || value == 1)) eng->tuning.desc_reuse_records = value;
  else if (!strcmp(key, "desc_table_host_max") && value >= 0 && value <= (1 << 24))
    eng->tuning.desc_table_host_max = value;
  else if (!strcmp(key, "ring_spin_us") && value >= 0 && value <= 1000000) eng->tuning.ring_spin_us = value;
  else if (!strcmp(key, "ring_sleep_us") && value >= 0 && value <= 100000) eng->tuning.ring_sleep_us = value;
  else rc = -EINVAL;
  pthread_mutex_unlock(&eng->lock);
  return rc;
}

extern "C" int bcp_get_option(bcp_engine *eng, const char *key, int *value) {
  if (!eng || !key || !value) return -EINVAL;
  int rc = 0;
  pthread_mutex_lock(&eng->lock);
  const Tuning &t = eng->tuning;
  if (!strcmp(key, "blocks_per_cu")) *value = t.blocks_per_cu;
  else if (!strcmp(key, "vecs_per_thread")) *value = t.vecs_per_thread;
  else if (!strcmp(key, "desc_blocks_per_cu")) *value = t.desc_blocks_per_cu;
  else if (!strcmp(key, "desc_vecs_per_thread")) *value = t.desc_vecs;
  else if (!strcmp(key, "desc_args_max")) *value = t.desc_args_max;
  else if (!strcmp(key, "stream_grid")) *value = t.stream_grid;
  else if (!strcmp(key, "desc_grid")) *value = t.desc_grid;
  else if (!strcmp(key, "contiguous_alloc")) *value = t.contiguous_alloc;
  else if (!strcmp(key, "table_host_max")) *value = t.table_host_max;
  else if (!strcmp(key, "host_registered")) *value = t.host_registered;
  else if (!strcmp(key, "desc_reuse_records")) *value = t.desc_reuse_records;
  else if (!strcmp(key, "desc_table_host_max")) *value = t.desc_table_host_max;
  else if (!strcmp(key, "ring_spin_us")) *value = t.ring_spin_us;
  else if (!strcmp(key, "ring_sleep_us")) *value = t.ring_sleep_us;
  else if (!strcmp(key, "last_stream_vecs")) *value = eng->last_stream_vecs.load(std::memory_order_relaxed);
  else if (!strcmp(key, "last_desc_vecs")) *value = eng->last_desc_vecs.load(std::memory_order_relaxed);
  else if (!strcmp(key, "last_desc_form")) *value = eng->last_desc_form.load(std::memory_order_relaxed);
  else rc = -EINVAL;
  pthread_mutex_unlock(&eng->lock);
  return rc;
}

extern "C" int bcp_set_tuning(bcp_engine *eng, int blocks_per_cu, int vecs_per_thread) {
  if (!eng) return -EINVAL;
  if (blocks_per_cu < 0 || blocks_per_cu > 32) return -EINVAL;
  if (vecs_per_thread != 0 && !stream_vecs_ok(vecs_per_thread)) return -EINVAL;
  const Tuning defaults;
  pthread_mutex_lock(&eng->lock);
  eng->tuning.blocks_per_cu = blocks_per_cu ? blocks_per_cu : defaults.blocks_per_cu;
  eng->tuning.vecs_per_thread = vecs_per_thread ? vecs_per_thread : defaults.vecs_per_thread;
  pthread_mutex_unlock(&eng->lock);
  return 0;
}

// ---------------------------------------------------------------------------
// queues / events
// ---------------------------------------------------------------------------
extern "C" int bcp_queue_create(bcp_engine *eng, bcp_queue **out) {
  if (!eng || !out) return -EINVAL;
  *out = nullptr;
  int rc = set_device(eng);
  if (rc) return rc;
  bcp_queue *q = new (std::nothrow) bcp_queue();
  if (!q) return -ENOMEM;
  q->eng = eng;
  hipError_t e = hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&q->qctr, 256);
  if (e == hipSuccess) e = hipMemsetAsync(q->qctr, 0, 256, q->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(q->stream);
  if (e != hipSuccess) {
    if (q->qctr) (void)hipFree(q->qctr);
    if (q->stream) (void)hipStreamDestroy(q->stream);
    delete q;
    return hip_to_errno(e);
  }
  *out = q;
  return 0;
}

extern "C" int bcp_queue_destroy(bcp_queue *q) {
  if (!q) return -EINVAL;
  set_device(q->eng);
  (void)hipStreamSynchronize(q->stream);
  if (q->copy_stream) (void)hipStreamSynchronize(q->copy_stream);
  for (auto &s : q->ring) {
    if (s.host) (void)hipHostFree(s.host);
    if (s.dev) (void)hipFree(s.dev);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.copied) (void)hipEventDestroy(s.copied);
    if (s.tiles) (void)hipFree(s.tiles);
    free(s.rec_copy);
  }
  if (q->copy_stream) (void)hipStreamDestroy(q->copy_stream);
  for (auto &t : q->timer)
    if (t) (void)hipEventDestroy(t);
  if (q->qctr) (void)hipFree(q->qctr);
  (void)hipStreamDestroy(q->stream);
  delete q;
  return 0;
}

// hipStreamSynchronize (the runtime's spin-then-yield wait; a blocking-sync
// event measured no better for the per-task protocol's 12 lanes on a 16-core
// share, r02).
extern "C" int bcp_queue_sync(bcp_queue *q) {
  if (!q) return -EINVAL;
  HIP_RC(hipStreamSynchronize(q->stream));
  return 0;
}

extern "C" int bcp_queue_query(bcp_queue *q) {
  if (!q) return -EINVAL;
  hipError_t e = hipStreamQuery(q->stream);
  if (e == hipErrorNotReady) return -EAGAIN;
  return hip_to_errno(e);
}

extern "C" int bcp_event_create(bcp_engine *eng, bcp_event **out) {
  if (!eng || !out) return -EINVAL;
  int rc = set_device(eng);
  if (rc) return rc;
  bcp_event *ev = new (std::nothrow) bcp_event();
  if (!ev) return -ENOMEM;
  ev->eng = eng;
  hipError_t e = hipEventCreateWithFlags(&ev->ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    delete ev;
    return hip_to_errno(e);
  }
  *out = ev;
  return 0;
}

extern "C" int bcp_event_destroy(bcp_event *ev) {
  if (!ev) return -EINVAL;
  (void)hipEventDestroy(ev->ev);
  delete ev;
  return 0;
}

extern "C" int bcp_event_record(bcp_event *ev, bcp_queue *q) {
  if (!ev || !q) return -EINVAL;
  HIP_RC(hipEventRecord(ev->ev, q->stream));
  return 0;
}

extern "C" int bcp_queue_wait_event(bcp_queue *q, bcp_event *ev) {
  if (!ev || !q) return -EINVAL;
  HIP_RC(hipStreamWaitEvent(q->stream, ev->ev, 0));
  return 0;
}

extern "C" int bcp_event_sync(bcp_event *ev) {
  if (!ev) return -EINVAL;
  HIP_RC(hipEventSynchronize(ev->ev));
  return 0;
}

extern "C" int bcp_event_query(bcp_event *ev) {
  if (!ev) return -EINVAL;
  hipError_t e = hipEventQuery(ev->ev);
  if (e == hipErrorNotReady) return -EAGAIN;
  return hip_to_errno(e);
}

extern "C" int bcp_queue_mark(bcp_queue *q, int slot) {
  if (!q || slot < 0 || slot >= kTimerSlots) return -EINVAL;
  if (!q->timer[slot]) HIP_RC(hipEventCreate(&q->timer[slot]));
  HIP_RC(hipEventRecord(q->timer[slot], q->stream));
  return 0;
}

extern "C" int bcp_queue_elapsed_ms(bcp_queue *q, int a, int b, float *ms) {
  if (!q || !ms || a < 0 || b < 0 || a >= kTimerSlots || b >= kTimerSlots) return -EINVAL;
  if (!q->timer[a] || !q->timer[b]) return -EINVAL;
  HIP_RC(hipEventSynchronize(q->timer[b]));
  HIP_RC(hipEventElapsedTime(ms, q->timer[a], q->timer[b]));
  return 0;
}

// ---------------------------------------------------------------------------
// memory
// ---------------------------------------------------------------------------
// Option "contiguous_alloc" (off by default): large buffers requested
// physically contiguous.  In interleaved A/B runs that helped the regular
// 512 KiB-stride streams (gen +0.5-1.0, rebuild +0.8-1.3 points) but cost
// the config-5 mixed shapes 2 points (profiles/r01/contig_alloc_ab*.jsonl),
// so it stays a knob.  Falls back to a default allocation.
constexpr size_t kContigMin = (size_t)64 << 20;

extern "C" int bcp_dev_alloc(bcp_engine *eng, size_t bytes, void **dptr) {
  if (!eng || !dptr) return -EINVAL;
  *dptr = nullptr;
  int rc = set_device(eng);
  if (rc) return rc;
  if (eng->tuning.contiguous_alloc && bytes >= kContigMin) {
    if (hipExtMallocWithFlags(dptr, bytes, hipDeviceMallocContiguous) == hipSuccess) return 0;
    (void)hipGetLastError();  // clear the sticky error of the failed attempt
    *dptr = nullptr;
  }
  HIP_RC(hipMalloc(dptr, bytes ? bytes : 16));
  return 0;
}

extern "C" int bcp_dev_free(bcp_engine *eng, void *dptr) {
  if (!eng) return -EINVAL;
  if (!dptr) return 0;
  set_device(eng);
  HIP_RC(hipFree(dptr));
  return 0;
}

namespace {
int alloc_registered(size_t bytes, void **out);
}

extern "C" int bcp_host_alloc(bcp_engine *eng, size_t bytes, void **hptr) {
  if (!eng || !hptr) return -EINVAL;
  *hptr = nullptr;
  int rc = set_device(eng);
  if (rc) return rc;
  if (eng->tuning.host_registered && alloc_registered(bytes ? bytes : 16, hptr) == 0) return 0;
  HIP_RC(hipHostMalloc(hptr, bytes ? bytes : 16, hipHostMallocDefault));
  return 0;
}

// Ordinary (THP-backed) host memory registered with HIP: allocations made
// by bcp_host_alloc_mapped in "registered" form, freed by bcp_host_free.
namespace {
struct RegAlloc {
  RegAlloc *next;
  void *p;
};
pthread_mutex_t g_reg_lock = PTHREAD_MUTEX_INITIALIZER;
RegAlloc *g_reg = nullptr;

// First touch of a fresh allocation, split over up to 8 threads for big ones:
// zeroing the pages is the cost of a pinned slab (a pipeline's 8 x 256 MiB
// took 0.25-0.38 s of a config-1 CLI run on one thread,
// profiles/r05/pipeline/c1_cli_r5e.jsonl); faults of one process scale
// across threads.
struct TouchArg {
  char *p;
  size_t n;
};
void *touch_range(void *a) {
  TouchArg *t = (TouchArg *)a;
  memset(t->p, 0, t->n);
  return nullptr;
}
void first_touch(void *p, size_t n) {
  const size_t piece = (size_t)32 << 20;
  int nt = (int)std::min<size_t>(8, n / piece);
  if (nt < 2) {
    memset(p, 0, n);
    return;
  }
  pthread_t th[8];
  TouchArg args[8];
  const size_t huge = (size_t)2 << 20;
  const size_t per = (n / nt + huge - 1) / huge * huge;
  int started = 0;
  for (int i = 0; i < nt; i++) {
    const size_t off = (size_t)i * per;
    args[i] = {(char *)p + off, off >= n ? 0 : std::min(per, n - off)};
    if (i == 0 || pthread_create(&th[i], nullptr, touch_range, &args[i]) != 0) {
      touch_range(&args[i]);  // this thread's share, or one a thread could not take
      th[i] = pthread_t();
      continue;
    }
    started |= 1 << i;
  }
  for (int i = 1; i < nt; i++)
    if (started >> i & 1) pthread_join(th[i], nullptr);
}

// posix_memalign (2 MiB, MADV_HUGEPAGE) + first touch + hipHostRegister
// (mapped): the CPU side stays normal write-back, huge-page-backed memory;
// the device reads and writes it at the same address.
int alloc_registered(size_t bytes, void **out) {
  const size_t huge = (size_t)2 << 20;
  const size_t n = (bytes + huge - 1) / huge * huge;
  RegAlloc *r = (RegAlloc *)malloc(sizeof(RegAlloc));
  void *p = nullptr;
  if (!r || posix_memalign(&p, huge, n) != 0) {
    free(r);
    return -ENOMEM;
  }
  (void)madvise(p, n, MADV_HUGEPAGE);
  first_touch(p, n);  // fault the pages in here, not under the first copy
  void *dev = nullptr;
  if (hipHostRegister(p, n, hipHostRegisterMapped) != hipSuccess ||
      hipHostGetDevicePointer(&dev, p, 0) != hipSuccess || dev != p) {
    (void)hipGetLastError();
    if (dev) (void)hipHostUnregister(p);
    free(p);
    free(r);
    return -EIO;  // the kernels address host rows by their host address
  }
  r->p = p;
  pthread_mutex_lock(&g_reg_lock);
  r->next = g_reg;
  g_reg = r;
  pthread_mutex_unlock(&g_reg_lock);
  *out = p;
  return 0;
}

// 1 if p came from alloc_registered (then unregistered and freed here).
int free_registered(void *p) {
  pthread_mutex_lock(&g_reg_lock);
  RegAlloc **pp = &g_reg;
  while (*pp && (*pp)->p != p) pp = &(*pp)->next;
  RegAlloc *r = *pp;
  if (r) *pp = r->next;
  pthread_mutex_unlock(&g_reg_lock);
  if (!r) return 0;
  (void)hipHostUnregister(p);
  free(p);
  free(r);
  return 1;
}
}  // namespace

// Mapped host memory for the P role's rows and output.  Default (option
// host_registered = 1): ordinary huge-page memory registered with HIP -- the
// chunk reads into the rows and the parity write out of the output are plain
// CPU copies, and over hipHostMalloc'd memory they ran so much slower that
// the per-task protocol lost ~40 % with the CPU fold itself unchanged
// (config 5, same box, same run: 14.8-18.2 against 24.8-29.7 GiB/s over
// ordinary memory; profiles/r02/protocol/host_kind_ab*.jsonl).  Falls back to
// hipHostMalloc (coherent, mapped).
extern "C" int bcp_host_alloc_mapped(bcp_engine *eng, size_t bytes, void **hptr) {
  if (!eng || !hptr) return -EINVAL;
  *hptr = nullptr;
  int rc = set_device(eng);
  if (rc) return rc;
  const unsigned flags = hipHostMallocMapped | hipHostMallocCoherent;
  if (eng->tuning.host_registered && alloc_registered(bytes ? bytes : 16, hptr) == 0) return 0;
  HIP_RC(hipHostMalloc(hptr, bytes ? bytes : 16, flags));
  return 0;
}

extern "C" int bcp_host_free(bcp_engine *eng, void *hptr) {
  if (!eng) return -EINVAL;
  if (!hptr) return 0;
  if (free_registered(hptr)) return 0;
  HIP_RC(hipHostFree(hptr));
  return 0;
}

extern "C" int bcp_host_register(bcp_engine *eng, void *hptr, size_t bytes) {
  if (!eng || !hptr || !bytes) return -EINVAL;
  int rc = set_device(eng);
  if (rc) return rc;
  void *dev = nullptr;
  if (hipHostRegister(hptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable) != hipSuccess) {
    (void)hipGetLastError();
    return -EIO;
  }
  if (hipHostGetDevicePointer(&dev, hptr, 0) != hipSuccess || dev != hptr) {
    (void)hipGetLastError();
    (void)hipHostUnregister(hptr);
    return -EIO;  // the kernels address host rows by their host address
  }
  return 0;
}

extern "C" int bcp_host_unregister(bcp_engine *eng, void *hptr) {
  if (!eng || !hptr) return -EINVAL;
  int rc = set_device(eng);
  if (rc) return rc;
  HIP_RC(hipHostUnregister(hptr));
  return 0;
}

extern "C" int bcp_h2d_async(bcp_queue *q, void *dst, const void *src, size_t bytes) {
  if (!q || (bytes && (!dst || !src))) return -EINVAL;
  if (!bytes) return 0;
  HIP_RC(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, q->stream));
  return 0;
}

extern "C" int bcp_d2h_async(bcp_queue *q, void *dst, const void *src, size_t bytes) {
  if (!q || (bytes && (!dst || !src))) return -EINVAL;
  if (!bytes) return 0;
  HIP_RC(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, q->stream));
  return 0;
}

extern "C" int bcp_d2d_async(bcp_queue *q, void *dst, const void *src, size_t bytes) {
  if (!q || (bytes && (!dst || !src))) return -EINVAL;
  if (!bytes) return 0;
  HIP_RC(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, q->stream));
  return 0;
}

extern "C" int bcp_h2d_2d_async(bcp_queue *q, void *dst, size_t dpitch, const void *src, size_t hpitch,
                                size_t row_bytes, size_t rows) {
  if (!q || row_bytes > dpitch || row_bytes > hpitch) return -EINVAL;
  if (!rows || !row_bytes) return 0;
  if (!dst || !src) return -EINVAL;
  HIP_RC(hipMemcpy2DAsync(dst, dpitch, src, hpitch, row_bytes, rows, hipMemcpyHostToDevice, q->stream));
  return 0;
}

extern "C" int bcp_memset_async(bcp_queue *q, void *dst, int value, size_t bytes) {
  if (!q || (bytes && !dst)) return -EINVAL;
  if (!bytes) return 0;
  HIP_RC(hipMemsetAsync(dst, value, bytes, q->stream));
  return 0;
}

// ---------------------------------------------------------------------------
// XOR submission
// ---------------------------------------------------------------------------

// Launch the streaming kernel on q (device-wide work queue).
static int launch_stream(bcp_queue *q, bool gather, int vecs, StreamArgs a, uint64_t ntiles) {
  bcp_engine *e = q->eng;
  if (ntiles == 0) return 0;
  if (ntiles > 0xFFFFFFF0ull) return -EINVAL;
  a.ntiles = (uint32_t)ntiles;
  a.ctr = q->qctr;
  a.base = q->qbase;
  // Tiles per grab: the kernels for 1-4 sources take several (stream_body).
  a.grab = stream_grab_auto(a.nsrc);
  const uint64_t nunits = (ntiles + a.grab - 1) / a.grab;
  int grid = grid_for(e);
  if ((uint64_t)grid > nunits) grid = (int)nunits;
  if (q->broken) return -EIO;
  (void)hipGetLastError();  // an error left by an earlier call must not read as this launch's
  const hipError_t le = launch_xor_stream(q->stream, grid, vecs, gather, a);
  if (le == hipSuccess) e->last_stream_vecs.store(vecs, std::memory_order_relaxed);
  return queue_launched(q, le, nunits + (uint64_t)grid);
}

// A batch is uniform when every stripe has the same nsrc and out_len, every
// source is at least out_len long (so neither zero padding nor window replay
// can apply) and all addresses are 16-byte multiples: then the streaming
// kernel's pointer-table form computes it (rebuild's shape; a length that is
// not a multiple of 16 ends in a byte tail).
static bool uniform_batch(const bcp_stripe *st, uint32_t nstripes, const bcp_source *so) {
  const uint32_t n = st[0].nsrc;
  const uint64_t len = st[0].out_len;
  if (n == 0 || len == 0 || len / 16 >= 0xFFFFFFFFull) return false;
  for (uint32_t i = 0; i < nstripes; i++) {
    if (st[i].nsrc != n || st[i].out_len != len || !aligned16(st[i].dst)) return false;
    for (uint32_t k = 0; k < n; k++) {
      const bcp_source &x = so[st[i].first_src + k];
      if (x.len < len || !aligned16(x.ptr)) return false;
    }
  }
  return true;
}

// Submit a descriptor batch (host arrays) on q.
static int desc_vecs_for(const bcp_engine *e, uint64_t tiles8) {
  if (e->tuning.desc_vecs) return e->tuning.desc_vecs;
  const uint64_t g = (uint64_t)desc_grid_for(e);
  if (tiles8 * 2 < g) return 2;
  if (tiles8 < 2 * g) return 4;
  return 8;
}

// Host staging threads: a small pool made on first use (7 threads that sleep
// between jobs), so a large batch's staging does not pay thread start-ups
// (~15 us each) on the path to its kernel.  One job at a time; a caller that
// finds the pool busy stages on its own thread.
namespace {
struct StagePool {
  std::mutex run;  // one job at a time (try_lock)
  std::mutex mu;
  std::condition_variable go, fin;
  const std::function<void(uint32_t)> *job = nullptr;
  uint32_t nparts = 0, claimed = 0, done = 0;
  uint64_t gen = 0;
  int nthreads = 0;

  void work_on(std::unique_lock<std::mutex> &lk) {  // with mu held: take parts until none is left
    while (claimed < nparts) {
      const uint32_t i = claimed++;
      const std::function<void(uint32_t)> *j = job;
      lk.unlock();
      (*j)(i);
      lk.lock();
      if (++done == nparts) fin.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      go.wait(lk, [&] { return gen != seen; });
      seen = gen;
      work_on(lk);
    }
  }
};

StagePool *stage_pool() {
  static StagePool *P = [] {
    StagePool *p = new StagePool();  // never freed: its threads live as long as the process
    for (int t = 0; t < 7; t++) {
      try {
        std::thread(&StagePool::loop, p).detach();
        p->nthreads++;
      } catch (...) {
        break;
      }
    }
    return p;
  }();
  return P;
}
}  // namespace

// fn(lo, hi) over [0, n): on this thread, or split over the staging pool and
// this thread when there are at least 2 * per items.
template <typename F>
static void par_for(uint32_t n, uint32_t per, F fn) {
  uint32_t nt = std::min<uint32_t>(8, n / (per ? per : 1));
  StagePool *P = nt >= 2 ? stage_pool() : nullptr;
  if (P) nt = std::min<uint32_t>(nt, (uint32_t)P->nthreads + 1);
  if (nt < 2 || !P->run.try_lock()) {
    fn(0, n);
    return;
  }
  const uint32_t chunk = (n + nt - 1) / nt;
  const std::function<void(uint32_t)> job = [&](uint32_t i) {
    const uint32_t lo = std::min(n, i * chunk), hi = std::min(n, lo + chunk);
    if (lo < hi) fn(lo, hi);
  };
  {
    std::unique_lock<std::mutex> lk(P->mu);
    P->job = &job;
    P->nparts = nt;
    P->claimed = P->done = 0;
    P->gen++;
    P->go.notify_all();
    P->work_on(lk);  // this thread takes parts too
    P->fin.wait(lk, [&] { return P->done == P->nparts; });
    P->job = nullptr;
  }
  P->run.unlock();
}

// Small batches (engine option desc_args_max, default kArgStripes stripes):
// the whole descriptor in the kernel arguments, one launch (xor_desc_args).
// Returns 1 if the batch does not qualify (caller takes the general path).
static int submit_desc_args(bcp_queue *q, const bcp_stripe *stripes, uint32_t nstripes, const bcp_source *sources,
                            int vecs) {
  bcp_engine *e = q->eng;
  if (nstripes > (uint32_t)e->tuning.desc_args_max || nstripes > (uint32_t)kArgStripes) return 1;
  uint32_t nsrc_all = 0;
  for (uint32_t i = 0; i < nstripes; i++) {
    if (stripes[i].window || stripes[i].nsrc > (uint32_t)kTileSrcs) return 1;
    nsrc_all += stripes[i].nsrc;
  }
  if (nsrc_all > (uint32_t)kArgSources) return 1;
  const uint64_t T = desc_tile_bytes(vecs);
  DescArgs a;
  memset(&a, 0, sizeof(a));
  uint64_t acc = 0;
  uint32_t k = 0;
  for (uint32_t i = 0; i < nstripes; i++) {
    const bcp_stripe &st = stripes[i];
    a.dst[i] = st.dst;
    a.out_len[i] = st.out_len;
    a.first[i] = k;
    a.nsrc[i] = st.nsrc;
    a.tile_start[i] = (uint32_t)acc;
    acc += (st.out_len + T - 1) / T;
    if (acc > 0xFFFFFFF0ull) return 1;
    for (uint32_t j = 0; j < st.nsrc; j++) {  // insertion sort, longest first (submit_desc)
      const bcp_source x = sources[st.first_src + j];
      uint32_t m = k + j;
      while (m > k && a.src_len[m - 1] < x.len) {
        a.src_ptr[m] = a.src_ptr[m - 1];
        a.src_len[m] = a.src_len[m - 1];
        m--;
      }
      a.src_ptr[m] = x.ptr;
      a.src_len[m] = x.len;
    }
    k += st.nsrc;
  }
  a.tile_start[nstripes] = (uint32_t)acc;
  a.nstripes = nstripes;
  a.ntiles = (uint32_t)acc;
  if (!acc) return 0;
  if (q->broken) return -EIO;
  a.ctr = q->qctr;
  a.base = q->qbase;
  int grid = desc_grid_for(e);
  if ((uint64_t)grid > acc) grid = (int)acc;
  (void)hipGetLastError();  // see launch_stream
  const hipError_t le = launch_xor_desc_args(q->stream, grid, vecs, a);
  if (le == hipSuccess) {
    e->last_desc_vecs.store(vecs, std::memory_order_relaxed);
    e->last_desc_form.store(2, std::memory_order_relaxed);
  }
  return queue_launched(q, le, acc + (uint64_t)grid);
}

// Submit a descriptor batch (host arrays) on q.
static int submit_desc(bcp_queue *q, const bcp_stripe *stripes, uint32_t nstripes, const bcp_source *sources,
                       uint32_t nsources) {
  bcp_engine *e = q->eng;
  // Validate, count 32 KiB tiles (the tile size is chosen from them).
  uint64_t tiles8 = 0;
  bool plain = true;  // no tile takes the general / wide path (those read the tables per tile)
  for (uint32_t i = 0; i < nstripes; i++) {
    const bcp_stripe &s = stripes[i];
    plain = plain && s.window == 0 && s.nsrc <= (uint32_t)kTileSrcs;
    if ((uint64_t)s.first_src + s.nsrc > nsources) return -EINVAL;
    if (s.nsrc > BCP_MAX_SOURCES) return -EINVAL;
    if (s.out_len && !s.dst) return -EINVAL;
    if (s.window && (s.window & 15u)) return -EINVAL;
    for (uint32_t k = 0; k < s.nsrc; k++) {
      const bcp_source &x = sources[s.first_src + k];
      if (x.len && !x.ptr) return -EINVAL;
    }
    tiles8 += (s.out_len + desc_tile_bytes(8) - 1) / desc_tile_bytes(8);
  }
  if (tiles8 == 0) return 0;
  if (tiles8 > 0xFFFFFFF0ull / 4) return -EINVAL;
  const int vecs = desc_vecs_for(e, tiles8);
  const uint32_t tile_bytes = desc_tile_bytes(vecs);
  if (uniform_batch(stripes, nstripes, sources)) {
    const uint64_t len = stripes[0].out_len;
    const int sv = stream_vecs(e, len, nstripes, stripes[0].nsrc);
    const uint32_t tps = stream_tiles_per_stripe(len, sv);
    const size_t off_src = ((size_t)nstripes * sizeof(bcp_stripe) + 15) & ~(size_t)15;
    const size_t bytes = off_src + (size_t)nsources * sizeof(bcp_source);
    DescSlot *slot = nullptr;
    int rc = ring_acquire(q, bytes, &slot);
    if (rc) return rc;
    slot->rec_ok = false;  // its tables and records are about to be overwritten
    // (large tables -- config 3's 100,000 sources, 2 MB -- copied by the
    // staging pool: this runs before the kernel whenever the queue is idle)
    char *const hs = (char *)slot->host;
    const size_t sb = (size_t)nstripes * sizeof(bcp_stripe), ob = (size_t)nsources * sizeof(bcp_source);
    const uint32_t pieces = (uint32_t)((sb + ob) >> 16) + 1;  // 64 KiB pieces
    par_for(pieces, 8, [&](uint32_t lo, uint32_t hi) {
      for (uint32_t i = lo; i < hi; i++) {
        const size_t a = (size_t)i << 16, b = std::min(sb + ob, a + ((size_t)1 << 16));
        if (a < sb) memcpy(hs + a, (const char *)stripes + a, std::min(b, sb) - a);
        if (b > sb) {
          const size_t a2 = std::max(a, sb);
          memcpy(hs + off_src + (a2 - sb), (const char *)sources + (a2 - sb), b - a2);
        }
      }
    });
    char *d = nullptr;
    if ((rc = stage_tables(q, slot, bytes, (size_t)e->tuning.table_host_max, &d))) return rc;
    StreamArgs a{};
    a.stripes = (const bcp_stripe *)d;
    a.sources = (const bcp_source *)(d + off_src);
    a.vps = (uint32_t)(len / 16);
    a.tail = (uint32_t)(len % 16);
    a.tps = tps;
    a.nsrc = stripes[0].nsrc;
    a.dense = 1;
    for (uint32_t i = 0; i < nstripes && a.dense; i++) a.dense = stripes[i].first_src == i * a.nsrc;
    rc = launch_stream(q, true, sv, a, (uint64_t)nstripes * tps);
    if (rc) return rc;
    HIP_RC(hipEventRecord(slot->done, q->stream));
    slot->used = true;
    return 0;
  }
  {
    // the argument form is instantiated up to U = 8 (its batches are small)
    const int rc = submit_desc_args(q, stripes, nstripes, sources, vecs > 8 ? 8 : vecs);
    if (rc <= 0) return rc;
  }
  // Staged copy: every stripe gets its own run of sources sorted by length,
  // longest first (XOR is commutative), so the sources that cover a tile are
  // always a prefix of the run (desc_tile).  Runs are laid out afresh, so
  // stripes whose caller ranges overlap stay independent.
  uint64_t nstaged = 0;
  for (uint32_t i = 0; i < nstripes; i++) nstaged += stripes[i].nsrc;
  if (nstaged > 0xFFFFFFFFull) return -EINVAL;
  const size_t off_src = (size_t)nstripes * sizeof(bcp_stripe);
  const size_t off_tiles = (off_src + (size_t)nstaged * sizeof(bcp_source) + 15) & ~(size_t)15;
  const size_t bytes = off_tiles + ((size_t)nstripes + 1) * sizeof(uint32_t);
  DescSlot *slot = nullptr;
  int rc = ring_acquire(q, bytes, &slot);
  if (rc) return rc;
  char *h = (char *)slot->host;
  bcp_stripe *hs = (bcp_stripe *)h;
  bcp_source *hso = (bcp_source *)(h + off_src);
  uint32_t *ts = (uint32_t *)(h + off_tiles);
  {
    uint32_t next_src = 0;
    for (uint32_t i = 0; i < nstripes; i++) {
      hs[i].first_src = next_src;  // (the rest of hs[i] is staged below)
      next_src += stripes[i].nsrc;
    }
  }
  // Per stripe: its run sorted by length and its tile count (sub_class /
  // tile_starts; desc_tiles repeats the cut).  Large batches are staged by
  // several threads: this host work runs before the kernel can start
  // whenever the queue is idle (a block's first launch: config-5 shapes,
  // 6,600 stripes, tools/exp/submit_cost.py).
  par_for(nstripes, 1024, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; i++) {
      const uint32_t first = hs[i].first_src;
      hs[i] = stripes[i];
      hs[i].first_src = first;
      bcp_source *run = hso + first;
      for (uint32_t k = 0; k < stripes[i].nsrc; k++) {
        // insertion sort, descending len (runs are short: <= BCP_MAX_SOURCES)
        const bcp_source x = sources[stripes[i].first_src + k];
        uint32_t m = k;
        while (m > 0 && run[m - 1].len < x.len) {
          run[m] = run[m - 1];
          m--;
        }
        run[m] = x;
      }
      const uint64_t c = count_tiles([run](uint32_t k) { return run[k].len; }, hs[i].nsrc, hs[i].out_len,
                                     tile_bytes, hs[i].window != 0);
      ts[i] = c > 0xFFFFFFF0ull ? 0xFFFFFFF1u : (uint32_t)c;
    }
  });
  uint64_t acc64 = 0;
  for (uint32_t i = 0; i < nstripes; i++) {
    const uint64_t c = ts[i];
    ts[i] = (uint32_t)acc64;
    acc64 += c;
    if (acc64 > 0xFFFFFFF0ull) return -EINVAL;
  }
  const uint32_t acc = (uint32_t)acc64;
  ts[nstripes] = acc;
  // Host-resident tables only when desc_tiles alone reads them: the general
  // and wide tile paths read them again per tile.
  const size_t host_max = plain ? (size_t)e->tuning.desc_table_host_max : 0;
  // desc_reuse_records: byte-identical tables and launch parameters on this
  // slot as the last descriptor batch it ran -> its records stand (where the
  // tables are read from is part of the key: the device copy exists only if
  // they were uploaded)
  const uint64_t key = ((uint64_t)acc << 32) ^ ((uint64_t)tile_bytes << 5) ^ ((uint64_t)vecs << 1) ^
                       (uint64_t)(bytes <= host_max);
  const bool reuse = e->tuning.desc_reuse_records && slot->rec_ok && slot->rec_key == key &&
                     slot->rec_len == bytes && slot->tiles_cap >= acc && memcmp(slot->rec_copy, h, bytes) == 0;
  slot->rec_ok = false;
  if (slot->tiles_cap < acc) {
    // the slot's previous kernels have finished (ring_acquire waited); the
    // queue's other idle slots grow with it (as ring_acquire grows tables)
    const size_t cap = std::max<size_t>(acc + acc / 4, 1u << 12);
    for (int j = 0; j < kRingSlots; j++) {
      DescSlot *o = &q->ring[j];
      if (o != slot && (o->tiles_cap >= acc || !slot_idle(o))) continue;
      o->rec_ok = false;
      if (o->tiles) HIP_RC(hipFree(o->tiles));
      o->tiles = nullptr;
      o->tiles_cap = 0;
      HIP_RC(hipMalloc((void **)&o->tiles, cap * sizeof(DescTile)));
      o->tiles_cap = cap;
    }
  }
  int grid = desc_grid_for(e);
  if ((uint32_t)grid > acc) grid = (int)acc;
  // Large batches: desc_tiles on the copy stream (after the table upload),
  // so it overlaps the previous batch's fold on the compute stream instead of
  // sitting between two folds; the fold waits for it by event.  Small batches
  // keep it in line (a cross-stream wait costs more than it hides).
  const bool side = acc >= 2u * (uint32_t)grid;
  char *d = nullptr;
  if (reuse) d = bytes <= host_max ? (char *)slot->host : (char *)slot->dev;  // uploaded last time, unchanged
  else if ((rc = stage_tables(q, slot, bytes, host_max, &d, !side))) return rc;
  DescBatch b;
  b.stripes = (const bcp_stripe *)d;
  b.sources = (const bcp_source *)(d + off_src);
  b.tile_start = (const uint32_t *)(d + off_tiles);
  b.tiles = slot->tiles;
  b.nstripes = nstripes;
  b.ntiles = acc;
  b.tile_bytes = tile_bytes;
  b.ctr = q->qctr;
  b.base = q->qbase;
  if (q->broken) return -EIO;
  (void)hipGetLastError();  // see launch_stream
  if (reuse) {
  } else if (side) {
    if (!q->copy_stream) HIP_RC(hipStreamCreateWithFlags(&q->copy_stream, hipStreamNonBlocking));
    HIP_RC(launch_desc_tiles(q->copy_stream, b));
    HIP_RC(hipEventRecord(slot->copied, q->copy_stream));
    HIP_RC(hipStreamWaitEvent(q->stream, slot->copied, 0));
  } else {
    HIP_RC(launch_desc_tiles(q->stream, b));
  }
  const hipError_t le = launch_xor_desc(q->stream, grid, vecs, b);
  if (le == hipSuccess) {
    e->last_desc_vecs.store(vecs, std::memory_order_relaxed);
    e->last_desc_form.store(1, std::memory_order_relaxed);
  }
  if ((rc = queue_launched(q, le, (uint64_t)acc + (uint64_t)grid))) return rc;
  HIP_RC(hipEventRecord(slot->done, q->stream));
  slot->used = true;
  if (e->tuning.desc_reuse_records && !reuse) {
    if (slot->rec_len < bytes || !slot->rec_copy) {
      free(slot->rec_copy);
      slot->rec_copy = malloc(bytes);
      slot->rec_len = 0;
    }
    if (slot->rec_copy) {
      memcpy(slot->rec_copy, h, bytes);
      slot->rec_len = bytes;
      slot->rec_key = key;
      slot->rec_ok = true;
    }
  } else if (reuse) {
    slot->rec_ok = true;
  }
  return 0;
}

extern "C" int bcp_xor_stripes_async(bcp_queue *q, const bcp_stripe *stripes, uint32_t nstripes,
                                     const bcp_source *sources, uint32_t nsources) {
  if (!q || (nstripes && !stripes) || (nsources && !sources)) return -EINVAL;
  if (!nstripes) return 0;
  int rc = set_device(q->eng);
  if (rc) return rc;
  return submit_desc(q, stripes, nstripes, sources, nsources);
}

extern "C" int bcp_xor_strided_async(bcp_queue *q, void *dst, uint64_t dst_stride, const void *src,
                                     uint64_t stripe_stride, uint64_t src_stride, uint64_t nstripes,
                                     uint32_t nsrc, uint64_t chunk_bytes) {
  if (!q || nsrc == 0 || nsrc > BCP_MAX_SOURCES) return -EINVAL;
  if (!nstripes || !chunk_bytes) return 0;
  if (!dst || !src) return -EINVAL;
  bcp_engine *e = q->eng;
  int rc = set_device(e);
  if (rc) return rc;
  const bool fast = aligned16((uint64_t)dst) && aligned16((uint64_t)src) && aligned16(dst_stride) &&
                    aligned16(stripe_stride) && aligned16(src_stride) && chunk_bytes / 16 < 0xFFFFFFFFull;
  if (fast) {
    StreamArgs a{};
    a.dst = (char *)dst;
    a.dst_stride = dst_stride;
    a.src = (const char *)src;
    a.stripe_stride = stripe_stride;
    a.src_stride = src_stride;
    a.vps = (uint32_t)(chunk_bytes / 16);
    a.tail = (uint32_t)(chunk_bytes % 16);
    const int sv = stream_vecs(e, chunk_bytes, nstripes, nsrc);
    a.tps = stream_tiles_per_stripe(chunk_bytes, sv);
    a.nsrc = nsrc;
    return launch_stream(q, false, sv, a, nstripes * a.tps);
  }
  // General geometry: express as descriptors (any alignment / tail).
  if (nstripes * nsrc > 0xFFFFFFFFull || nstripes > 0xFFFFFFFFull) return -EINVAL;
  std::vector<bcp_stripe> st;
  std::vector<bcp_source> so;
  try {  // nothing may throw across the C ABI
    st.resize(nstripes);
    so.resize(nstripes * nsrc);
  } catch (const std::bad_alloc &) {
    return -ENOMEM;
  }
  for (uint64_t s = 0; s < nstripes; s++) {
    st[s].dst = (uint64_t)dst + s * dst_stride;
    st[s].out_len = chunk_bytes;
    st[s].first_src = (uint32_t)(s * nsrc);
    st[s].nsrc = nsrc;
    st[s].window = 0;
    for (uint32_t k = 0; k < nsrc; k++) {
      so[s * nsrc + k].ptr = (uint64_t)src + s * stripe_stride + k * src_stride;
      so[s * nsrc + k].len = chunk_bytes;
    }
  }
  return submit_desc(q, st.data(), (uint32_t)nstripes, so.data(), (uint32_t)so.size());
}

extern "C" int bcp_xor_uniform_async(bcp_queue *q, void *dst, const void *src, uint64_t nstripes, uint32_t nsrc,
                                     uint64_t chunk_bytes) {
  return bcp_xor_strided_async(q, dst, chunk_bytes, src, chunk_bytes * nsrc, chunk_bytes, nstripes, nsrc,
                               chunk_bytes);
}

// ---------------------------------------------------------------------------
// resident fold ring (RingArgs in bcp_internal.h, kernel fold_ring)
// ---------------------------------------------------------------------------
namespace {
constexpr uint32_t kRingEntries = 512;        // tickets in flight (12 lanes x 4 ranks x <= 5 ranges fit)
constexpr unsigned long long kRingLive = ~0ull;  // RingCtl::closed while a launch is live
constexpr uint64_t kRingMaxPieces = 255;      // a handle carries the piece count in 8 bits
}  // namespace

struct bcp_ring {
  bcp_engine *eng = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ended = nullptr;     // recorded after each launch
  bool launched = false;
  RingEntry *host = nullptr;      // [K] pinned, coherent
  RingCtl *ctl = nullptr;         // pinned, coherent: closed, stop, done[]
  unsigned long long *done = nullptr;
  char *dev = nullptr;            // RingState | cnt[K] | copy[K]
  int workers = 64;
  unsigned long long idle_ticks = 0, hard_ticks = 0;
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;  // publication and launches
  uint64_t next = 0;              // next ticket
  std::atomic<int> broken{0};
  std::atomic<uint64_t> launches{0};
  std::atomic<int> spin_us{4}, sleep_us{10};  // waits (bcp_ring_set_wait; from the engine's options)
};

static size_t ring_dev_bytes() {
  return sizeof(RingState) + 2 * kRingEntries * sizeof(unsigned long long) + kRingEntries * sizeof(RingEntry);
}

static unsigned long long ring_load(const unsigned long long *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

static void ring_free(bcp_ring *r) {
  if (r->ended) (void)hipEventDestroy(r->ended);
  if (r->stream) (void)hipStreamDestroy(r->stream);
  if (r->dev) (void)hipFree(r->dev);
  if (r->host) (void)hipHostFree(r->host);
  if (r->ctl) (void)hipHostFree(r->ctl);
  pthread_mutex_destroy(&r->mu);
  delete r;
}

extern "C" int bcp_ring_create(bcp_engine *eng, int workers, int idle_us, bcp_ring **out) {
  if (!eng || !out || workers < 0 || workers > 4096 || idle_us < 0 || idle_us > 10000000) return -EINVAL;
  *out = nullptr;
  int rc = set_device(eng);
  if (rc) return rc;
  bcp_ring *r = new (std::nothrow) bcp_ring();
  if (!r) return -ENOMEM;
  r->eng = eng;
  r->workers = workers ? workers : 64;
  r->spin_us.store(eng->tuning.ring_spin_us, std::memory_order_relaxed);
  r->sleep_us.store(eng->tuning.ring_sleep_us, std::memory_order_relaxed);
  int khz = 0;  // s_memrealtime rate
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, eng->device) != hipSuccess || khz <= 0)
    khz = 100000;
  const unsigned long long idle = idle_us ? (unsigned long long)idle_us : 5000ull;
  r->idle_ticks = idle * (unsigned long long)khz / 1000ull;
  r->hard_ticks = 4 * r->idle_ticks + 100ull * (unsigned long long)khz;  // + 100 ms
  const size_t ctl_bytes = sizeof(RingCtl) + (size_t)kRingEntries * kRingDoneStride * sizeof(unsigned long long);
  hipError_t e = hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&r->ended, hipEventDisableTiming);
  if (e == hipSuccess)
    e = hipHostMalloc((void **)&r->host, kRingEntries * sizeof(RingEntry), hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostMalloc((void **)&r->ctl, ctl_bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipMalloc((void **)&r->dev, ring_dev_bytes());
  if (e == hipSuccess) e = hipMemsetAsync(r->dev, 0, ring_dev_bytes(), r->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    ring_free(r);
    return hip_to_errno(e);
  }
  memset(r->host, 0, kRingEntries * sizeof(RingEntry));
  memset(r->ctl, 0, ctl_bytes);
  r->done = (unsigned long long *)(r->ctl + 1);
  __atomic_store_n(&r->ctl->closed, 0ull, __ATOMIC_RELEASE);  // no launch yet; the first starts at ticket 0
  *out = r;
  return 0;
}

// Under r->mu: make sure a launch will take the tickets published so far.  A
// closed launch (the watcher wrote the first ticket it did not take) is
// drained, then a new one starts from that ticket.  Tickets below it were
// all folded; none at or above it was touched (fold_ring), so nothing is
// folded twice.
static int ring_live_locked(bcp_ring *r) {
  const unsigned long long c = ring_load(&r->ctl->closed);
  if (c == kRingLive) return 0;
  if (r->broken.load(std::memory_order_relaxed)) return -EIO;
  int rc = set_device(r->eng);
  if (rc) return rc;
  hipError_t e = hipSuccess;
  if (r->launched) e = hipEventSynchronize(r->ended);  // the closed launch drains within microseconds
  __atomic_store_n(&r->ctl->closed, kRingLive, __ATOMIC_RELEASE);
  if (e == hipSuccess) e = hipMemsetAsync(r->dev, 0, sizeof(RingState), r->stream);
  if (e == hipSuccess) {
    RingArgs a;
    a.host = r->host;
    a.done = r->done;
    a.closed = &r->ctl->closed;
    a.stop = &r->ctl->stop;
    a.state = (RingState *)r->dev;
    a.claim = (unsigned long long *)(r->dev + sizeof(RingState));
    a.cnt = a.claim + kRingEntries;
    a.copy = (RingEntry *)(r->dev + sizeof(RingState) + 2 * kRingEntries * sizeof(unsigned long long));
    a.base = c;
    a.idle_ticks = r->idle_ticks;
    a.hard_ticks = r->hard_ticks;
    a.kmask = kRingEntries - 1;
    a.kshift = (uint32_t)__builtin_ctz(kRingEntries);
    (void)hipGetLastError();
    e = launch_fold_ring(r->stream, r->workers, a);
  }
  if (e == hipSuccess) e = hipEventRecord(r->ended, r->stream);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    r->broken.store(1, std::memory_order_relaxed);
    __atomic_store_n(&r->ctl->closed, c, __ATOMIC_RELEASE);  // no launch: waiters see it and fail
    return hip_to_errno(e);
  }
  r->launched = true;
  r->launches.fetch_add(1, std::memory_order_relaxed);
  return 0;
}

static inline void cpu_relax() { __builtin_ia32_pause(); }

// Ticket t is folded (its done word reached t + 1: done words only grow).
static bool ring_ticket_done(const bcp_ring *r, uint64_t t) {
  return ring_load(&r->done[(size_t)(t & (kRingEntries - 1)) * kRingDoneStride]) >= t + 1;
}

static uint64_t mono_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// Wait for ticket t; relaunch when the live launch closed before taking it.
// Spins with pause for ring_spin_us, then sleeps ring_sleep_us between looks
// (engine options): the waiters are the protocol's P lanes, dozens per
// process, and a spinning one takes the CPU the source lanes copy chunks
// with (config 1 is CPU-bound on a 16-CPU share).  The thread's timer slack
// is set to 1 us once, so the sleeps are as short as asked.
static int ring_wait_ticket(bcp_ring *r, uint64_t t) {
  static thread_local bool slack_set = false;
  const uint64_t spin_ns = (uint64_t)r->spin_us.load(std::memory_order_relaxed) * 1000u;
  const long sleep_ns = (long)r->sleep_us.load(std::memory_order_relaxed) * 1000L;
  uint64_t t0 = 0, last_query = 0;
  for (;;) {
    if (ring_ticket_done(r, t)) return 0;
    if (r->broken.load(std::memory_order_relaxed)) return -EIO;
    if (ring_load(&r->ctl->closed) != kRingLive) {
      pthread_mutex_lock(&r->mu);
      const int rc = ring_live_locked(r);
      pthread_mutex_unlock(&r->mu);
      if (rc) return rc;
      continue;
    }
    const uint64_t now = mono_ns();
    if (!t0) t0 = last_query = now;
    if (now - last_query > 1000000u) {
      // a launch that ended without closing (a fault) never completes t
      last_query = now;
      pthread_mutex_lock(&r->mu);
      const hipError_t q = r->launched ? hipEventQuery(r->ended) : hipErrorNotReady;
      const bool dead = q != hipErrorNotReady && ring_load(&r->ctl->closed) == kRingLive && !ring_ticket_done(r, t);
      if (q != hipSuccess && q != hipErrorNotReady) (void)hipGetLastError();
      if (dead) r->broken.store(1, std::memory_order_relaxed);
      pthread_mutex_unlock(&r->mu);
      if (dead) return -EIO;
    }
    if (now - t0 < spin_ns) {
      for (int i = 0; i < 16; i++) cpu_relax();
    } else if (sleep_ns > 0) {
      if (!slack_set) {
        (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
        slack_set = true;
      }
      const struct timespec ts = {0, sleep_ns};
      nanosleep(&ts, nullptr);
    } else {
      sched_yield();
    }
  }
}

extern "C" int bcp_ring_submit(bcp_ring *r, const bcp_stripe *stripe, const bcp_source *sources, uint64_t *handle) {
  if (!r || !stripe || !handle || (stripe->nsrc && !sources)) return -EINVAL;
  const bcp_stripe s = *stripe;
  if (s.window != 0 || s.nsrc > BCP_MAX_SOURCES || (s.out_len && !s.dst)) return -EINVAL;
  for (uint32_t k = 0; k < s.nsrc; k++)
    if (sources[k].len && !sources[k].ptr) return -EINVAL;
  const uint64_t pieces = (s.out_len + kRingPieceMax - 1) / kRingPieceMax;
  if (pieces > kRingMaxPieces) return -EINVAL;
  *handle = 0;
  if (!pieces) return 0;
  // Reserve the tickets; each is then this caller's alone.  The watcher takes
  // tickets in order, so a later caller's published tickets wait for ours.
  pthread_mutex_lock(&r->mu);
  if (r->broken.load(std::memory_order_relaxed)) {
    pthread_mutex_unlock(&r->mu);
    return -EIO;
  }
  const uint64_t first = r->next;
  r->next += pieces;
  pthread_mutex_unlock(&r->mu);
  int rc = 0;
  for (uint64_t i = 0; i < pieces && !rc; i++) {
    const uint64_t t = first + i;
    RingEntry *E = r->host + (t & (kRingEntries - 1));
    // the entry's previous ticket must be folded before it is reused (it
    // is earlier in ticket order, so it never waits for ours)
    if (t >= kRingEntries && (rc = ring_wait_ticket(r, t - kRingEntries))) break;
    const uint64_t p0 = i * kRingPieceMax;
    const uint64_t plen = std::min<uint64_t>(kRingPieceMax, s.out_len - p0);
    E->dst = s.dst + p0;
    E->out_len = plen;
    E->nsrc = s.nsrc;
    E->parts = (uint32_t)((plen + kRingTileBytes - 1) / kRingTileBytes);  // 1..16 (plen <= kRingPieceMax)
    for (uint32_t k = 0; k < s.nsrc; k++) {
      const uint64_t len = sources[k].len > p0 ? std::min<uint64_t>(sources[k].len - p0, plen) : 0;
      E->src[k].ptr = len ? sources[k].ptr + p0 : 0;
      E->src[k].len = len;
    }
    __atomic_store_n(&E->seq, (unsigned long long)(t + 1), __ATOMIC_RELEASE);
  }
  if (rc) {
    // reserved tickets that were never published would stall every later
    // one: the ring is unusable from here on
    r->broken.store(1, std::memory_order_relaxed);
    return rc;
  }
  if (ring_load(&r->ctl->closed) != kRingLive) {
    // no live launch (or it just closed): start one.  A launch that closes
    // after this look is caught by the waiters (ring_wait_ticket).
    pthread_mutex_lock(&r->mu);
    rc = ring_live_locked(r);
    pthread_mutex_unlock(&r->mu);
    if (rc) return rc;
  }
  *handle = (first << 8) | pieces;
  return 0;
}

extern "C" int bcp_ring_wait(bcp_ring *r, uint64_t handle) {
  if (!r) return -EINVAL;
  const uint64_t first = handle >> 8, n = handle & 0xFF;
  for (uint64_t t = first; t < first + n; t++) {
    const int rc = ring_wait_ticket(r, t);
    if (rc) return rc;
  }
  return 0;
}

extern "C" int bcp_ring_query(bcp_ring *r, uint64_t handle) {
  if (!r) return -EINVAL;
  const uint64_t first = handle >> 8, n = handle & 0xFF;
  for (uint64_t t = first; t < first + n; t++)
    if (!ring_ticket_done(r, t)) {
      if (r->broken.load(std::memory_order_relaxed)) return -EIO;
      if (ring_load(&r->ctl->closed) != kRingLive) {
        pthread_mutex_lock(&r->mu);
        const int rc = ring_live_locked(r);
        pthread_mutex_unlock(&r->mu);
        if (rc) return rc;
      }
      return -EAGAIN;
    }
  return 0;
}

extern "C" int bcp_ring_set_wait(bcp_ring *r, int spin_us, int sleep_us) {
  if (!r || spin_us < 0 || spin_us > 1000000 || sleep_us < 0 || sleep_us > 100000) return -EINVAL;
  r->spin_us.store(spin_us, std::memory_order_relaxed);
  r->sleep_us.store(sleep_us, std::memory_order_relaxed);
  return 0;
}

extern "C" int bcp_ring_stats(bcp_ring *r, uint64_t *pieces, uint64_t *launches) {
  if (!r) return -EINVAL;
  pthread_mutex_lock(&r->mu);
  if (pieces) *pieces = r->next;
  pthread_mutex_unlock(&r->mu);
  if (launches) *launches = r->launches.load(std::memory_order_relaxed);
  return 0;
}

extern "C" int bcp_ring_destroy(bcp_ring *r) {
  if (!r) return -EINVAL;
  set_device(r->eng);
  pthread_mutex_lock(&r->mu);
  __atomic_store_n(&r->ctl->stop, 1u, __ATOMIC_RELEASE);
  int rc = 0;
  if (r->launched && hipEventSynchronize(r->ended) != hipSuccess) {
    (void)hipGetLastError();
    rc = -EIO;
  }
  pthread_mutex_unlock(&r->mu);
  (void)hipStreamSynchronize(r->stream);
  ring_free(r);
  return rc;
}

// ---------------------------------------------------------------------------
// verification / synthetic data
// ---------------------------------------------------------------------------
extern "C" int bcp_dev_fill_synthetic_async(bcp_queue *q, void *dst, uint64_t bytes, uint64_t seed,
                                            uint64_t byte_offset) {
  if (!q || (bytes && !dst)) return -EINVAL;
  int rc = set_device(q->eng);
  if (rc) return rc;
  HIP_RC(launch_fill_synthetic(q->stream, grid_for(q->eng), (char *)dst, bytes, seed, byte_offset));
  return 0;
}

extern "C" int bcp_dev_xor_fold_async(bcp_queue *q, const void *src, uint64_t bytes, void *out16_dev) {
  if (!q || !out16_dev || (bytes && !src)) return -EINVAL;
  if (!aligned16((uint64_t)src)) return -EINVAL;
  int rc = set_device(q->eng);
  if (rc) return rc;
  HIP_RC(hipMemsetAsync(out16_dev, 0, 16, q->stream));
  HIP_RC(launch_xor_fold(q->stream, grid_for(q->eng), (const char *)src, bytes, (uint32_t *)out16_dev));
  return 0;
}

extern "C" int bcp_dev_compare_async(bcp_queue *q, const void *a, const void *b, uint64_t bytes, void *out_dev) {
  if (!q || !out_dev || (bytes && (!a || !b))) return -EINVAL;
  if (!aligned16((uint64_t)a) || !aligned16((uint64_t)b)) return -EINVAL;
  int rc = set_device(q->eng);
  if (rc) return rc;
  HIP_RC(hipMemsetAsync(out_dev, 0, 8, q->stream));
  HIP_RC(launch_compare(q->stream, grid_for(q->eng), (const char *)a, (const char *)b, bytes,
                        (unsigned long long *)out_dev));
  return 0;
}

// ---------------------------------------------------------------------------
// xor_parity drop-in (task_processing.c:96-109)
// ---------------------------------------------------------------------------
namespace {

pthread_once_t g_once = PTHREAD_ONCE_INIT;
bcp_engine *g_engine = nullptr;
int g_engine_rc = 0;

void init_global_engine() {
  int dev = 0;
  if (const char *v = getenv("BCP_DEVICE")) dev = atoi(v);
  g_engine_rc = bcp_engine_create(dev, &g_engine);
}

struct DropinState {
  bcp_queue *q = nullptr;
  void *dev = nullptr;
  size_t cap = 0;
  ~DropinState() {
    if (q) {
      bcp_queue_destroy(q);  // synchronises first: nothing uses dev below
      if (dev) bcp_dev_free(g_engine, dev);
    }
  }
};
thread_local DropinState t_dropin;

}  // namespace

extern "C" int bcp_xor_parity(uint8_t *dst, size_t nbytes, const uint8_t *data, int nsources) {
  if (nsources < 1 || nsources > BCP_MAX_SOURCES) return -EINVAL;
  if (!nbytes) return 0;
  if (!dst || !data) return -EINVAL;
  pthread_once(&g_once, init_global_engine);
  if (g_engine_rc) return g_engine_rc;
  DropinState &st = t_dropin;
  int rc = 0;
  if (!st.q && (rc = bcp_queue_create(g_engine, &st.q))) return rc;
  // Device layout: sources at a 256-byte pitch so every row is aligned, then
  // the output row.
  const size_t pitch = (nbytes + 255) & ~(size_t)255;
  const size_t need = pitch * ((size_t)nsources + 1);
  if (st.cap < need) {
    if (st.dev) bcp_dev_free(g_engine, st.dev);
    st.dev = nullptr;
    st.cap = 0;
    if ((rc = bcp_dev_alloc(g_engine, need, &st.dev))) return rc;
    st.cap = need;
  }
  char *dv = (char *)st.dev;
  char *dout = dv + pitch * (size_t)nsources;
  if (!(rc = bcp_h2d_2d_async(st.q, dv, pitch, data, nbytes, nbytes, (size_t)nsources)) &&
      !(rc = bcp_xor_strided_async(st.q, dout, pitch, dv, pitch * nsources, pitch, 1, (uint32_t)nsources, nbytes)))
    rc = bcp_d2h_async(st.q, dst, dout, nbytes);
  // also after a failed submission: nothing of this call stays in flight on
  // the caller's buffers or the thread's device rows
  const int src = bcp_queue_sync(st.q);
  return rc ? rc : src;
}
