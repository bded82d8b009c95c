/*
 * bcp_task.h -- per-rank chunk-streaming interface of the parity engine
 * (host C layer of libbcp.so).
 *
 * Drop-in for the reference's task layer:
 *   int process_task(HostState *hs, const char *path, const FileInfo *fi,
 *                    TaskInfo ti);
 *       -- src/beegfs-raid5/common/task_processing.h:20-24
 * with the reference's types (common.h:15-48, task_processing.h:7-18,
 * progress_reporting.h:10-20) kept field for field, so the callers
 * process_list (gen/main.c:116-164) and do_file (rebuild/main.c:40-89) bind
 * unchanged.  What differs is underneath:
 *   - the P role folds the received windows on the GPU through the engine
 *     (include/bcp.h) instead of the CPU xor_parity;
 *   - ranks are loopback ranks (threads of one process) talking through an
 *     MPI-like point-to-point transport (bcp_lb_*) matched by
 *     (source, tag) in FIFO order, in place of MPI_COMM_WORLD.
 * Behaviour kept from the reference: message flow and sizes, 10 MiB windows
 * with the replay-after-EOF quirk, parity chunk file format (u64 chunk_size[n]
 * header in ascending storage-target order + max_cs XOR bytes), rebuild
 * truncation, the corrupt list, sticky per-rank errors (/dev/zero, /dev/null).
 */
#ifndef BCP_TASK_H
#define BCP_TASK_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#include "bcp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- shared types and bit layout (common.h:15-48) ---------------------- */
#define MODIFY_EVENT 'm'
#define UNLINK_EVENT 'd'
#define MAX_STORAGE_TARGETS 56
#define TEST_BIT(x, i) ((x) & (1ULL << (i)))
#define GET_P(loc) ((int)((loc) >> 56))
#define P_MASK UINT64_C(0xFF00000000000000)
#define L_MASK UINT64_C(0x00FFFFFFFFFFFFFF)
#define WITH_P(loc, P) (((loc) & L_MASK) | (((uint64_t)(P) << 56) & P_MASK))
#define NO_P UINT64_C(0xFF)
#define P_IS_INVALID(loc) (GET_P(loc) == NO_P || TEST_BIT((loc), GET_P(loc)))
#define DB_VERSION 1

typedef struct {
    int64_t timestamp;
    uint64_t locations; /* bits 0..55 chunk holders, bits 56..63 parity target P */
} FileInfo;

/* progress_reporting.h:10-20 */
typedef struct {
    double dt;
    size_t nfiles;
    size_t bytes_read;
    size_t bytes_written;
    double total_time;
    size_t total_nfiles;
    size_t total_bytes_read;
    size_t total_bytes_written;
} ProgressSample;
#define PROGRESS_SAMPLE_INIT {0.0, 0, 0, 0, 0.0, 0, 0, 0}

typedef struct {
    int read_dir;
    int is_rebuilding;
    int actual_P_st; /* only valid when rebuilding */
    int tag;
    ProgressSample *sample;
} TaskInfo;

/* task_processing.h:7-18 */
typedef struct {
    int storage_target;
    int corrupt_files_fd;
    int error;
    const char *error_path;
    int fd_null;
    int fd_zero;
    int write_dir;
    int read_chunk_dir;
    int read_parity_dir;
    FILE *log;
} HostState;

/* storage target -> rank map, defined by the caller (gen/main.c:48,
 * rebuild/main.c:34 define it the same way). */
extern int st2rank[MAX_STORAGE_TARGETS];

/* Returns non-zero if this rank took part in the task and it is not a delete
 * task.  Errors are logged to hs->log and made sticky in hs->error. */
int process_task(HostState *hs, const char *path, const FileInfo *fi, TaskInfo ti);

/* ---- GPU binding of the P role ----------------------------------------- */
/* Device used by the P role of storage target st: devices[st] if a map was
 * given, else st % device_count.  Engines are created lazily, one per device. */
int bcp_task_set_device_map(const int *devices, int ntargets);
/* How the P role folds a window on the GPU (both read the pinned window rows
 * in place over PCIe, data bytes only, and write the parity block in place).
 * BATCHED: the window is handed to the device's fold service (flat
 * combining, no thread of its own): a waiting lane leads a launch that folds
 * EVERY window the P roles of this process (or, through the node fold
 * server, of every rank process) have pending as ONE descriptor batch and
 * wakes each lane when its own window is done (process_task stays
 * synchronous per task, as the reference's window loop is,
 * task_processing.c:203-226).
 * PIPELINED (default): the fold follows the senders' reads.  The P role
 * registers its window rows; a source filling one directly (the loopback
 * transport's send_fill) reads its chunk in 256 KiB pieces and publishes
 * each final prefix; the source whose piece completes a byte range of every
 * row (at least 128 KiB and a quarter window) launches its fold on the lane's
 * queue (no sync) -- or publishes it to the device's fold ring
 * (bcp_task_set_fold_ring) -- so the rows' PCIe reads overlap the file
 * reads; after the receives, the rest and one wait.  Windows it cannot follow (multi-window
 * tasks, other transports, folds by a node fold server) go to the fold
 * service as in BATCHED.
 * Returns the previous mode, or -EINVAL. */
#define BCP_FOLD_BATCHED 2
#define BCP_FOLD_PIPELINED 5
int bcp_task_set_fold_mode(int mode);
/* PIPELINED counters since the process started: windows folded by following
 * their rows, and range folds launched for them (ranges / windows > 1: the
 * fold overlapped the reads). */
int bcp_task_pipe_stats(uint64_t *windows, uint64_t *ranges);
/* Row watches registered right now (PIPELINED windows between their first
 * receive and their fold): 0 whenever no task runs -- a watch that outlived
 * its window would let a later fill into memory at the same address publish
 * to a dead P role (tests check it after every pipelined run, failures and
 * drains included). */
size_t bcp_task_watch_live(void);
/* The wire of a gen task's single window (max_cs <= 10 MiB):
 *   BCP_PAD_AUTO (default): implicit padding -- a source sends its chunk's
 *     bytes only and the P role supplies the zeros past them -- when the
 *     transport is one of this library's own (loopback ranks, socketpair rank
 *     processes: every P role is this library's); the reference's wire
 *     (every window zero-padded to buffer_size, task_processing.c:302-303)
 *     through any table a caller installs with bcp_task_set_transport (an MPI
 *     binding may reach the reference's parity_generator, which folds whole
 *     rows);
 *   0: implicit padding through every transport (a caller whose P roles are
 *     all this library's);
 *   1: the reference's wire through every transport.
 * The P role of this library takes either.  Returns the previous value or
 * -EINVAL. */
#define BCP_PAD_AUTO (-1)
int bcp_task_set_explicit_padding(int on);
/* The fold service: how many batches may be on a device at once (1..16, each
 * led by one waiting lane on its own queue; default 1: pure flat
 * combining).  Returns the
 * previous value or -EINVAL. */
int bcp_task_set_fold_inflight(int k);
/* Fold-service counters since the last shutdown: windows
 * folded and launches issued (windows / launches = the batching achieved). */
int bcp_task_fold_stats(uint64_t *windows, uint64_t *launches);
/* PIPELINED folds through the device's resident fold ring (bcp_ring_*,
 * include/bcp.h): 1 (default) -- every range fold and every whole-window fold
 * of a PIPELINED P role (and of a node fold server) is one publication into a
 * launch that stays on the device, and the lane waits for its own pieces:
 * no launch and no stream sync per window; 0 -- range folds launch on the
 * lane's queue and whole windows go to the fold service.  BATCHED mode
 * always uses the fold service.  The ring of a device lives until
 * bcp_task_shutdown; its launch ends by itself 5 ms after the last fold.
 * Returns the previous value or -EINVAL. */
int bcp_task_set_fold_ring(int on);
/* How the P lanes wait for their folds in the ring (bcp_ring_set_wait) --
 * for the rings now and those made later; tools and A/B runs. */
int bcp_task_set_ring_wait(int spin_us, int sleep_us);
/* Pieces (<= 512 KiB of parity each) published to the fold rings and
 * launches of them since the process started. */
int bcp_task_ring_stats(uint64_t *pieces, uint64_t *launches);
/* Lane deferral, for the CALLING THREAD (a lane): d = 1..4 -- a single-window P task
 * whose fold goes to the fold ring returns once the fold is published; the
 * wait for it, the parity write (the rebuild's truncation) and the close
 * happen on the process's completion threads (bcp_task_set_fold_tuning
 * "completion_threads"; with 0, on this thread when its next task has
 * published its own fold or sent its windows, the oldest beyond d - 1 of
 * them).  The thread holds at most d such tasks (its next publication waits
 * for the oldest); bcp_task_flush / bcp_task_thread_release (or the thread's
 * end) wait for all of them.  The lane's next tasks then overlap the previous
 * ones' folds and writes.  Files, bytes
 * and sticky errors are the same; an error of the deferred part becomes
 * sticky when it completes.  0 (default): process_task returns with the
 * parity written, as the reference's does.  libbcp's runners turn it on for
 * lanes that write no DB entries (a DB entry must not precede its file).
 * Returns the previous value or -EINVAL. */
int bcp_task_set_lane_deferral(int on);
/* Complete the calling thread's deferred P tasks, if any (a lane calls it
 * before its list's end is reported: MPI barrier, DB sync, exit). */
void bcp_task_flush(void);
/* Tools and A/B runs: the P role's fold shape.  "ring_workers" (16: worker
 * workgroups of the rings; a new value ends the current rings -- call it
 * between runs -- and the next fold makes new ones), "pipe_piece_kib" (256: bytes a
 * source reads between two publishes of its row), "pipe_step_kib" (128: the
 * smallest range folded before the window is complete, at least a quarter
 * window), "defer_depth" (2: lane deferral depth of libbcp's runners,
 * 0..4), "completion_threads" (4: threads completing deferred P tasks,
 * 0..16; 0 = each lane completes its own), "lb_spin_us" (0: how long a
 * blocked loopback receive or fill send polls before it sleeps, 0..1000).  Returns the previous value or -EINVAL. */
int bcp_task_set_fold_tuning(const char *key, int value);
/* Wall time spent per protocol phase, summed over every task of every lane
 * since the last reset (seconds[i] for i < nphases; the last two entries are
 * task COUNTS, not seconds).  Returns BCP_PHASES.  P role: size exchange,
 * fold resources, waiting for the window rows (the parity open + header run
 * after the first window's receives are posted, inside this phase), the fold,
 * the parity write, close; source role: open + size exchange, the window
 * sends (from the P role's receive, i.e. the chunk reads). */
#define BCP_PHASE_P_SIZES 0
#define BCP_PHASE_P_OPEN 1
#define BCP_PHASE_P_ROWS 2
#define BCP_PHASE_P_FOLD 3
#define BCP_PHASE_P_WRITE 4
#define BCP_PHASE_P_CLOSE 5
#define BCP_PHASE_S_SIZES 6
#define BCP_PHASE_S_SEND 7
#define BCP_PHASE_P_TASKS 8
#define BCP_PHASE_S_TASKS 9
#define BCP_PHASES 10
int bcp_task_phase_stats(double *seconds, int nphases, int reset);
/* Release the engines and every lane's queues / staging (call after all
 * lanes have joined). */
int bcp_task_shutdown(void);
/* Release the calling thread's queue and staging buffers. */
void bcp_task_thread_release(void);

/* Test injection point: when set, the P role calls fn instead of the GPU
 * (host logic tests on machines without a GPU).  The product never sets it;
 * every use is logged to hs->log. fn gets n rows of `pitch` bytes. */
typedef int (*bcp_xor_hook_fn)(uint8_t *dst, size_t nbytes, const uint8_t *data, size_t pitch, int nsrc,
                               void *ctx);
void bcp_task_set_xor_hook(bcp_xor_hook_fn fn, void *ctx);

/* Failure injection for tests (the product never sets it): the next `count`
 * passes through `site` fail as if the allocation / thread creation had,
 * after `after` passes succeed.  Sites: the P role's fold resources (as
 * -ENOMEM), its single drain row (then a bounded 64 KiB per-thread drain
 * with truncated receives is used), the source role's window buffer, the
 * runners' lane-thread creation, and a source's chunk read into a row it
 * fills directly (as EIO; a source reading in pieces for a PIPELINED P role
 * fails a piece after the first), and the node fold server dropping a rank's
 * connection instead of answering a fold (the server process takes the
 * setting when a rank pool forks it), and the pipeline's O_DIRECT read of a
 * piece ending short before the end of its file (DIRECT read mode: the rest
 * of the piece is then read through the page cache), and the P role's write
 * of a parity window or rebuilt chunk (as ENOSPC; on the lane or on a
 * completion thread).  count 0 clears the site. */
#define BCP_INJECT_FOLD_RES 1
#define BCP_INJECT_DRAIN_ROW 2
#define BCP_INJECT_SEND_BUF 4
#define BCP_INJECT_THREAD 8
#define BCP_INJECT_READ 16
#define BCP_INJECT_FOLD_SERVER 32
#define BCP_INJECT_DIRECT_READ 64
#define BCP_INJECT_PARITY_WRITE 128
int bcp_task_inject_failure(int site, int after, int count);

/* ---- transport seam (the MPI subset process_task speaks) ---------------- */
/* process_task talks to its peers through exactly the point-to-point subset
 * the reference uses (task_processing.c:43-52,120-130,151-166,203-209,
 * 274-307): blocking send / recv, non-blocking isend / irecv, wait, waitall,
 * matched by (source rank, tag), non-overtaking per (source, destination,
 * tag), ranks numbered as st2rank numbers them.  A transport is this table;
 * every entry returns 0 or a negative errno (a receive shorter than the
 * message may return -EMSGSIZE and must still consume it).  send_fill is
 * optional (NULL: the source role reads each window into its own buffer and
 * sends that, as the reference does); when present it is the zero-copy send
 * of bcp_lb_send_fill.  An MPI binding maps each entry onto
 * MPI_Send / MPI_Recv / MPI_Isend / MPI_Irecv / MPI_Wait / MPI_Waitall on
 * MPI_COMM_WORLD with MPI_BYTE. */
typedef int (*bcp_lb_fill_fn)(void *ctx, void *dst, size_t n);
typedef struct bcp_transport_ops {
    void *ctx;
    int (*send)(void *ctx, const void *buf, size_t n, int dst, int tag);
    int (*recv)(void *ctx, void *buf, size_t n, int src, int tag);
    int (*isend)(void *ctx, const void *buf, size_t n, int dst, int tag, void **req);
    int (*irecv)(void *ctx, void *buf, size_t n, int src, int tag, void **req);
    int (*wait)(void *ctx, void *req);
    int (*waitall)(void *ctx, int n, void **reqs);
    int (*send_fill)(void *ctx, bcp_lb_fill_fn fill, void *fill_ctx, size_t n, int dst, int tag);
} bcp_transport_ops;
/* Install the transport process_task uses from now on (copied); NULL
 * restores the default, the in-process loopback below.  -EINVAL if a
 * mandatory entry is missing.  Not to be changed while tasks run. */
int bcp_task_set_transport(const bcp_transport_ops *ops);
/* The loopback transport as an ops table (the default). */
const bcp_transport_ops *bcp_lb_transport(void);

/* Ranks as PROCESSES: a world of world_size ranks connected pairwise by
 * Unix socketpairs (created before fork; each rank process attaches as its
 * rank and gets a transport whose receives are progressed by the waiting
 * threads themselves, unexpected messages buffered).  Any number of threads
 * of a rank process may use it (the 12 lanes). */
typedef struct bcp_sock_world bcp_sock_world;
int bcp_sock_world_create(int world_size, bcp_sock_world **out);
/* In the rank's process: keep rank's sockets, close the others, fill *ops
 * (pass it to bcp_task_set_transport).  Once per process. */
int bcp_sock_world_attach(bcp_sock_world *w, int rank, bcp_transport_ops *ops);
/* Close whatever sockets this process still holds and free the world. */
int bcp_sock_world_destroy(bcp_sock_world *w);

/* ---- loopback rank transport (replaces the MPI subset of §2) ----------- */
/* A world of `world_size` ranks inside this process.  Every thread acting
 * for rank r calls bcp_lb_set_rank(r) first.  Semantics follow MPI
 * point-to-point: blocking send (up to 4 KiB buffered and returning at once,
 * as an MPI eager send; larger ones rendezvous: return once a receiver has the
 * data), non-blocking send (eager copy), posted receives matched in order by
 * (source, tag), non-overtaking per (source, destination, tag).  A program
 * correct under MPI_Send's rules does not depend on which one happens. */
typedef struct bcp_lb_req bcp_lb_req;
int bcp_lb_init(int world_size);
int bcp_lb_finalize(void);
int bcp_lb_world_size(void);
void bcp_lb_set_rank(int rank);
int bcp_lb_rank(void);
int bcp_lb_send(const void *buf, size_t n, int dst, int tag);
int bcp_lb_recv(void *buf, size_t n, int src, int tag, size_t *received);
int bcp_lb_isend(const void *buf, size_t n, int dst, int tag, bcp_lb_req **req);
int bcp_lb_irecv(void *buf, size_t n, int src, int tag, bcp_lb_req **req);
int bcp_lb_wait(bcp_lb_req *req, size_t *received);
int bcp_lb_waitall(int n, bcp_lb_req **reqs);
/* Zero-copy blocking send: instead of copying a buffer, the sender's
 * fill(ctx, dst, n) writes the n-byte payload straight into the matched
 * receive buffer (e.g. read() from the chunk file), on the sending thread,
 * once a receiver is matched.  Same matching and ordering as bcp_lb_send;
 * fill returns 0 or a negative errno, which bcp_lb_send_fill returns. */
int bcp_lb_send_fill(bcp_lb_fill_fn fill, void *ctx, size_t n, int dst, int tag);

/* Lanes of the rebuild runners (bcp_rebuild_run[_db|_procs], rank pools):
 * 1 = the reference's single lane (default); with L, item i goes to lane
 * i % L with MPI tag i % L on every rank -- the same files (the corrupt
 * lists' lines may come in another order).  Returns the previous value or
 * -EINVAL (1..64). */
int bcp_task_set_rebuild_lanes(int nlanes);

/* ---- node fold server for independent rank processes (an MPI job) ------
 * One process per node serves folds for every rank on a Unix socket
 * (bcp_fold_server_serve; it is the only process with a HIP runtime; serves
 * max_conns connections then returns, 0 = forever).  A rank calls
 * bcp_fold_server_connect once, before its tasks: its P-role window rows
 * and outputs then come from an arena of arena_bytes in a memfd it shares
 * with the server (SCM_RIGHTS), and its folds go to the server over nconn
 * connections (lane tag modulo nconn), batched with every other rank's.
 * Receives into the rows are the caller's (MPI_Irecv, the loopback or socket
 * transports).  The rank pool does the same by itself (bcp_rank_pool_*). */
int bcp_fold_server_serve(const char *socket_path, int max_conns);
int bcp_fold_server_connect(const char *socket_path, size_t arena_bytes, int nconn);
/* Windows the node fold server folded for this process so far. */
int bcp_fold_server_stats(uint64_t *windows);

/* ---- callers: generation lanes and rebuild (loopback drivers) ---------- */
typedef struct {
    const char *path;   /* chunk path relative to <store>/chunks and /parity */
    FileInfo fi;
} bcp_work_item;

typedef struct {
    double seconds;
    uint64_t tasks;            /* process_task calls that returned non-zero */
    uint64_t bytes_read;       /* ProgressSample totals over every rank/lane */
    uint64_t bytes_written;
    int errors;                /* ranks that ended with a sticky error */
    uint64_t refused;          /* items skipped because their path would leave the
                                  store (absolute, ".."): no parity was written and
                                  no DB entry made for them (ABI version 2) */
} bcp_run_stats;

/* ---- persistent chunk state (persistent_db.{c,h}) ---------------------- */
/* path -> FileInfo, iterated in bytewise key order -- the reference's
 * LevelDB store (persistent_db.c:23-145) as a self-contained append-log +
 * hash table (LevelDB is absent here).  Every call returns 0 / -errno;
 * bcp_pdb_get returns 1 found, 0 absent.  Thread-safe.  The key
 * "?db_version" is reserved (persistent_db.c:13): the version lives in the
 * log header and a mismatch makes bcp_pdb_open return -EPROTO
 * (the reference's errx "Incompatible DB", :72-75). */
#define BCP_PDB_MAX_KEY 255  /* mkdir_for_file's char[256], task_processing.c:31-32 */
typedef struct bcp_pdb bcp_pdb;
int bcp_pdb_open(const char *folder, uint64_t expected_version, bcp_pdb **out);  /* pdb_init */
int bcp_pdb_close(bcp_pdb *db);                                                  /* pdb_term */
int bcp_pdb_set(bcp_pdb *db, const char *key, size_t keylen, const FileInfo *val);
int bcp_pdb_del(bcp_pdb *db, const char *key, size_t keylen);
int bcp_pdb_get(bcp_pdb *db, const char *key, size_t keylen, FileInfo *val);
size_t bcp_pdb_count(bcp_pdb *db);
int bcp_pdb_sync(bcp_pdb *db);  /* fsync the log (LevelDB sync = 1 equivalent) */
/* pdb_iterate: fn(key, keylen, value, ctx) over a snapshot in key order until
 * it returns non-zero. */
typedef int (*bcp_pdb_visit_fn)(const char *key, size_t keylen, const FileInfo *val, void *ctx);
int bcp_pdb_iterate(bcp_pdb *db, bcp_pdb_visit_fn fn, void *ctx);
/* Snapshot as work items sorted by path (one allocation; paths inside). */
int bcp_pdb_items(bcp_pdb *db, bcp_work_item **items, size_t *nitems);
void bcp_pdb_items_free(bcp_work_item *items);

/* Greedy lane assignment of gen/assign_lanes.c:12-46 (16-deep history per
 * lane, tasks sharing targets kept apart).  Identical output to the
 * reference on x86-64, including its int-shift of P. */
void bcp_assign_lanes(int nlanes, uint64_t njobs, const FileInfo *jobs, int *lane);

/* Parity generation over loopback ranks: storage target k (0..ntargets-1) is
 * rank k+1 with store <root>/st<k>/{chunks,parity}; every rank runs nlanes
 * lane threads that walk the same worklist (process_list, gen/main.c:116-164:
 * own lane only, NO_P skipped, MPI tag = lane).  Lanes come from
 * bcp_assign_lanes when lanes == NULL. */
int bcp_gen_run(const char *store_root, int ntargets, const bcp_work_item *items, size_t nitems, int nlanes,
                const int *lanes, FILE *log, bcp_run_stats *stats);

/* Rebuild of one lost target over loopback ranks (do_file, rebuild/main.c:
 * 40-89): items in DB key order, skip rules, re-roled locations, the
 * P-holder reads <store>/parity, single lane with tag 0.  Survivors whose
 * chunk mtime is newer than FileInfo.timestamp are appended (one path per
 * line) to corrupt_list_path. */
int bcp_rebuild_run(const char *store_root, int ntargets, int rebuild_target, const bcp_work_item *items,
                    size_t nitems, const char *corrupt_list_path, FILE *log, bcp_run_stats *stats);

/* The same two drivers with every storage target's rank as its own PROCESS
 * (fork; socketpair transport, bcp_sock_world_*), the way the reference's
 * ranks run under mpirun: rank k+1 = target k runs its lanes as threads and
 * reports its counters to the caller through a pipe.  The calling process
 * must not have used the GPU yet (a forked child cannot use a HIP runtime
 * its parent initialised): -EBUSY if this library already did.  -ECHILD if a
 * rank process died.  Fork safety: the caller may be multithreaded; between
 * fork and their work the children use only what survives fork in one
 * thread (glibc's malloc, fresh mutexes, threads they create; environment
 * defaults are set without setenv's lock) -- but a caller's OWN locks held
 * by another thread at the fork (stdio on the log FILE, say) stay held in
 * the children, so do not write to `log` from another thread while a pool
 * is being created. */
int bcp_gen_run_procs(const char *store_root, int ntargets, const bcp_work_item *items, size_t nitems,
                      int nlanes, const int *lanes, FILE *log, bcp_run_stats *stats);
int bcp_rebuild_run_procs(const char *store_root, int ntargets, int rebuild_target, const bcp_work_item *items,
                          size_t nitems, const char *corrupt_list_path, FILE *log, bcp_run_stats *stats);
/* The same ranks kept alive across runs (a long-lived job's ranks, as under
 * mpirun): bcp_rank_pool_create forks one process per storage target (the
 * caller must not have used the GPU yet: -EBUSY), and every gen / rebuild run
 * is a command to all of them; each rank keeps its HIP engine, fold service
 * and registered window rows from run to run.  A run takes the caller's
 * P-role settings at the time of the call (fold mode, fold service width,
 * window padding, test hook -- a hook's code must have been loaded before
 * the pool was created: -EFAULT otherwise).  A rank whose run cannot start,
 * or that dies, fails the run (-ECHILD or its -errno) and breaks the pool:
 * later runs return -EPIPE; destroy it and create another.  The gen/rebuild
 * _procs drivers above are one-run pools. */
typedef struct bcp_rank_pool bcp_rank_pool;
int bcp_rank_pool_create(int ntargets, FILE *log, bcp_rank_pool **out);
int bcp_rank_pool_gen(bcp_rank_pool *pool, const char *store_root, const bcp_work_item *items, size_t nitems,
                      int nlanes, const int *lanes, bcp_run_stats *stats);
int bcp_rank_pool_rebuild(bcp_rank_pool *pool, const char *store_root, int rebuild_target,
                          const bcp_work_item *items, size_t nitems, const char *corrupt_list_path,
                          bcp_run_stats *stats);
int bcp_rank_pool_destroy(bcp_rank_pool *pool);

/* With the persistent state: bcp_gen_run plus, after every task of a lane
 * of rank k, the process_list DB update (gen/main.c:146-149: set when the
 * item still has holders, else delete) on target k's replica
 * <root>/st<k>/db. */
int bcp_gen_run_db(const char *store_root, int ntargets, const bcp_work_item *items, size_t nitems, int nlanes,
                   const int *lanes, FILE *log, bcp_run_stats *stats);
/* Rebuild walking the DB at db_folder in key order (rebuild/main.c:223-225);
 * NULL = the replica of the first surviving target.  -ENOENT if absent. */
int bcp_rebuild_run_db(const char *store_root, int ntargets, int rebuild_target, const char *db_folder,
                       const char *corrupt_list_path, FILE *log, bcp_run_stats *stats);

/* ---- chunk-event records and worklist planning ------------------------- */
/* Record stream per storage target (bp-find-all-chunks/main.c:25-33,
 * gen-chunkmod-filelist.py:35-41): {i64 ts, u64 size, u64 event 'm'|'d',
 * u64 len, char path[len]}, native-endian.  Events aggregate per path as
 * fih_add_info does (gen/file_info_hash.c:24-31). */
typedef struct bcp_eventset bcp_eventset;
int bcp_eventset_create(bcp_eventset **out);
void bcp_eventset_destroy(bcp_eventset *s);
/* Feed bytes of target st's stream; a partial trailing record is carried. */
int bcp_eventset_feed(bcp_eventset *s, int st, const void *buf, size_t len);
int bcp_eventset_feed_file(bcp_eventset *s, int st, const char *path);
size_t bcp_eventset_count(const bcp_eventset *s);
int bcp_eventset_get(const bcp_eventset *s, size_t i, const char **path, int64_t *timestamp, uint64_t *modified,
                     uint64_t *deleted, uint64_t *size);
/* simple_hash of gen/main.c:67-74 (djb2 over signed chars). */
uint32_t bcp_path_hash(const char *p, size_t len);
/* get_store_weight of gen/main.c:403-427 for a store directory fd. */
int bcp_store_weight(int dirfd);
/* The worklist of one gen run, in the reference's per-coordinator rounds:
 * path -> eater simple_hash(path) % ntargets (gen/main.c:310); per eater,
 * arrival (= the event set's first-seen) order shuffled with the fixed-seed
 * PCG32 then sorted by total size (:710-711); the eaters' lists one round
 * after another in target order (:758-797).  Each item merged with the
 * previous state `prev` (sorted by path), deleted holders dropped, P chosen
 * by select_P with the cumulative weights cum_weight[0..ntargets-1], NO_P
 * when unchanged (:772-788).  out[i].path points into the event set.
 * *nout = number of events; round_start (NULL or ntargets + 1 entries):
 * round k is out[round_start[k] .. round_start[k+1]) -- lanes are assigned
 * per round (:823). */
int bcp_plan_rounds(const bcp_eventset *s, int ntargets, const int *cum_weight, const bcp_work_item *prev,
                    size_t nprev, bcp_work_item *out, size_t out_cap, size_t *nout, size_t *round_start);
/* The same with the rounds in MPI rank order: round r is broadcast by the
 * eater of storage target round_st[r] (a permutation of 0..ntargets-1, as
 * bcp_map_targets derives it; NULL = target order).  bcp_plan_rounds is this
 * with NULL. */
int bcp_plan_rounds_ordered(const bcp_eventset *s, int ntargets, const int *cum_weight, const int *round_st,
                            const bcp_work_item *prev, size_t nprev, bcp_work_item *out, size_t out_cap,
                            size_t *nout, size_t *round_start);
/* Storage-target index and round order of gen/main.c:498-499, 506-541:
 * prev_ids[nprev] = the previous run's targetNumIDs in index order (RunData),
 * rank_ids[ntargets] = the targetNumID of each eater rank in MPI rank order.
 * Targets found in prev keep their index, new ones are appended in rank
 * order; out st_ids[ntargets] (the new index order) and round_st[ntargets]
 * (the target whose eater broadcasts round r).  -EEXIST a rank repeats an id
 * already placed ("Duplicate targetNumID"), -ENODEV fewer targets than prev
 * or a previous target without a rank ("Storage target missing!"). */
int bcp_map_targets(const int32_t *prev_ids, int nprev, const int32_t *rank_ids, int ntargets, int32_t *st_ids,
                    int *round_st);
/* The round order of a store: <root>/rank_order (the targetNumID of every
 * target's eater in MPI rank order, whitespace separated -- the hostfile's
 * order, src/beegfs-parity-gen:114-117) mapped onto the st<k> directories
 * (their ids: st<k>/targetNumID, k+1 when absent); identity when the file is
 * absent.  Used by bcp_gen_round*. */
int bcp_store_round_order(const char *store_root, int ntargets, int *round_st);
/* The same without the round boundaries. */
int bcp_plan_worklist(const bcp_eventset *s, int ntargets, const int *cum_weight, const bcp_work_item *prev,
                      size_t nprev, bcp_work_item *out, size_t out_cap, size_t *nout);
/* bcp_assign_lanes over each round separately (gen/main.c:823): lane[i] for
 * the whole list; round_start as bcp_plan_rounds fills it. */
void bcp_assign_lanes_rounds(int nlanes, int nrounds, const size_t *round_start, const FileInfo *jobs, int *lane);

/* bp-find-all-chunks (src/bp-find-all-chunks/main.c:17-45): one 'm' record
 * per regular file under chunks_dir, path relative to it, written to out_fd
 * in the record format above -- or fed straight into an event set as target
 * st's stream (the --complete input of phase 1, gen/main.c:622-624). */
int bcp_scan_chunks(const char *chunks_dir, int out_fd, uint64_t *nrecords);
int bcp_eventset_scan(bcp_eventset *s, int st, const char *chunks_dir, uint64_t *nrecords);
/* Storage-target bookkeeping of gen/main.c:472-551 over <root>/st<k>: ids
 * from st<k>/targetNumID (k+1 when absent), checked against and saved to
 * run_data_path.  -EEXIST duplicate id, -ENODEV fewer targets or a target
 * whose id changed ("Storage target missing!"), -EPROTO version stamp (the
 * file's own format stamp, 1; not the struct ABI: BCP_ABI_VERSION).  With a
 * <root>/rank_order (bcp_store_round_order) also its mapping as the reference
 * derives it from the previous run's list (bcp_map_targets): -EPROTO when
 * targets added since are not numbered in the order the reference appends
 * them (rank order).
 * First run (no previous list), a DELIBERATE DEVIATION: the reference numbers
 * the targets in rank order there (gen/main.c:508-527: every rank's id
 * appended in rank order, so index i is the i-th rank); here the st<k>
 * directories exist before any run and keep their index k, and rank_order
 * only orders the rounds.  With a rank_order that differs from the
 * directories' order, a first run's target indices -- and so select_P's
 * placements -- differ from the reference's; stores whose directories are
 * created in rank order (bcp_store.make_store, the CLI) are unaffected. */
#define BCP_TASK_ABI_VERSION 4 /* = BCP_ABI_VERSION (include/bcp.h) */
int bcp_check_targets(const char *store_root, int ntargets, const char *run_data_path, FILE *log);

/* Cumulative store weights st_weight (gen/main.c:485, 528-536) of
 * <root>/st<k>, k < ntargets. */
int bcp_store_cum_weights(const char *store_root, int ntargets, int *cum_weight);
/* One phase-2 gen round (gen/main.c:716-797): previous state from target
 * 0's replica, worklist planned from `events` (cum_weight NULL = the stores'
 * own weights), then bcp_gen_run_db.  *nplanned = worklist length. */
int bcp_gen_round(const char *store_root, int ntargets, const bcp_eventset *events, const int *cum_weight,
                  int nlanes, FILE *log, bcp_run_stats *stats, size_t *nplanned);
/* The same round with rank processes (bcp_gen_run_procs); every replica is
 * updated after the run, only when it finished without errors. */
int bcp_gen_round_procs(const char *store_root, int ntargets, const bcp_eventset *events, const int *cum_weight,
                        int nlanes, FILE *log, bcp_run_stats *stats, size_t *nplanned);

/* ---- batched end-to-end pipeline (loopback stores) ---------------------- */
typedef struct {
    int device;          /* HIP device */
    size_t slab_bytes;   /* pinned / device slab per slot (grown to the largest stripe) */
    int io_threads;      /* io threads = 2 x this (reads and writes share them); 0 = 8 per GPU, at
                            most half the CPUs the process may use (affinity, cgroup quota), at least 2
                            (capped at 64) */
    int nslots;          /* slabs in flight per device (2..8) */
    int ndevices;        /* GPUs device .. device+ndevices-1 (mod the visible count),
                            batches round-robin (0 = 1) */
    int read_mode;       /* how chunk bytes reach the device (BCP_READ_*; ABI version 2) */
} bcp_pipeline_opts;
/* Read paths of the pipeline's input:
 *   COPY: io threads read() each chunk into the slot's pinned slab, one H2D
 *     per batch (page cache -> slab -> device: the CPU copies every byte);
 *   DIRECT: the io threads read each chunk file with O_DIRECT straight into
 *     the pinned slab (page layout: every file from offset 0 at a page-aligned
 *     slab offset): on a disk-backed store the
 *     storage device's DMA fills the slab and no CPU copies the bytes.  A
 *     file the filesystem will not read that way (open or read refused) is
 *     read through the page cache instead, piece by piece.  O_DIRECT reads
 *     bypass the page cache: for a store whose chunks are cached (just
 *     written, or on tmpfs) COPY is the faster choice.
 *   AUTO (0): chosen per run between COPY and DIRECT -- COPY when every
 *     source directory of the run (<root>/st<k>/chunks, parity) is tmpfs / ramfs,
 *     or when a sample of the run's chunks (mincore over the first 16 MiB of
 *     one source in each of up to 64 tasks) is mostly in the page cache,
 *     DIRECT otherwise (a cold store on a disk); bcp_pipeline_timing.read_mode
 *     says which.  Env BCP_PIPELINE_READ=copy|direct names a mode instead.
 * (2 was MAP -- mmap + read-only registration of the chunk files -- removed
 * in ABI 3: AUTO never chose it; bcp_pipeline_create returns -EINVAL for it.) */
#define BCP_READ_AUTO 0
#define BCP_READ_COPY 1
#define BCP_READ_DIRECT 3

/* Parity generation for local stores without per-task messaging: chunk
 * files are read by io threads into pinned slabs, copied H2D on a side
 * queue, folded by one descriptor-kernel launch per batch, copied D2H on
 * another side queue and written as parity chunk files -- byte-identical
 * to bcp_gen_run's (same header, padding and window replay).  NO_P items are
 * skipped; items without holders unlink their parity chunk.  opts may be
 * NULL ({0, 256 MiB, 0, 4, 1, AUTO}: 4 slots beat 3 by 8-15 % on every
 * workload in two interleaved A/Bs).
 * Footprint per device: nslots x (input + output slab) of pinned host memory
 * and the same of HBM -- 4 x 2 x 256 MiB = 2 GiB pinned + 2 GiB HBM by
 * default, 16 GiB pinned over 8 GPUs (slabs grow to the largest stripe's
 * inputs) -- plus 2 x io_threads io threads (16 per GPU by default, within
 * the CPUs the process may use): one pool that reads chunks and writes
 * parity files, taking reads first.  posix_fallocate of each output (as
 * task_processing.c:186) is skipped where that output's directory is tmpfs /
 * ramfs (it would zero every page the write fills again). */
int bcp_pipeline_gen(const char *store_root, int ntargets, const bcp_work_item *items, size_t nitems,
                     const bcp_pipeline_opts *opts, FILE *log, bcp_run_stats *stats);
/* The same as a long-lived object: engine, queues, io threads and pinned /
 * device slabs are set up once and reused by every run (a resident service
 * pays page pinning and stream creation once). */
typedef struct bcp_pipeline bcp_pipeline;
int bcp_pipeline_create(const bcp_pipeline_opts *opts, bcp_pipeline **out);
int bcp_pipeline_run(bcp_pipeline *pl, const char *store_root, int ntargets, const bcp_work_item *items,
                     size_t nitems, FILE *log, bcp_run_stats *stats);
int bcp_pipeline_destroy(bcp_pipeline *pl);
/* Where the host thread of the pipeline's last run spent its wall time
 * (seconds; for tools): stat phase, blocked on a batch's reads (the next
 * batch's reads are already queued then), waiting for a slot's previous
 * batch to be written before queueing reads into it, building and submitting
 * batches, and the drain after the last submission; DIRECT mode: the data
 * bytes read with O_DIRECT and the pieces read through the page cache
 * instead.  (ABI 3 removed the MAP fields map / mapped_bytes / map_fallbacks.) */
typedef struct {
    double stat, read_wait, slot_wait, submit, drain;
    uint32_t batches;    /* device batches */
    uint32_t read_jobs;  /* io read jobs (one per 1 MiB piece of a chunk read into a slab) */
    int read_mode;       /* the mode the run used (BCP_READ_COPY / DIRECT) */
    uint64_t direct_bytes;
    uint32_t direct_fallbacks;
} bcp_pipeline_timing;
int bcp_pipeline_last_timing(const bcp_pipeline *pl, bcp_pipeline_timing *out);
/* Rebuild of one lost target with the batched pipeline (do_file's selection
 * and roles, rebuild/main.c:40-89): per item the surviving chunks and the
 * parity body are folded on the device and the lost chunk is written to
 * <root>/st<target>/chunks truncated to its size in the parity header;
 * survivors newer than FileInfo.timestamp are appended to the corrupt list.
 * Byte-identical to bcp_rebuild_run. */
int bcp_pipeline_rebuild(bcp_pipeline *pl, const char *store_root, int ntargets, int rebuild_target,
                         const bcp_work_item *items, size_t nitems, const char *corrupt_list_path, FILE *log,
                         bcp_run_stats *stats);
/* bcp_gen_round with the batched pipeline as the engine; the replicas are
 * updated after the run, only when it finished without errors. */
int bcp_gen_round_pipeline(bcp_pipeline *pl, const char *store_root, int ntargets, const bcp_eventset *events,
                           const int *cum_weight, FILE *log, bcp_run_stats *stats, size_t *nplanned);
/* Stage times (seconds) of this process's latest round (bcp_gen_round*):
 * reading the previous state from replica 0, planning (event set -> rounds
 * -> worklist against that state), the run over the planned items, and the
 * replicas' update (pipeline and rank-process rounds; the DB runner updates
 * its replicas inside the run).  Returns BCP_ROUND_STAGES. */
#define BCP_ROUND_DB_READ 0
#define BCP_ROUND_PLAN 1
#define BCP_ROUND_RUN 2
#define BCP_ROUND_REPLICAS 3
#define BCP_ROUND_STAGES 4
int bcp_gen_round_timing(double *seconds, int nstages);

#ifdef __cplusplus
}
#endif

#endif /* BCP_TASK_H */
