/* bcp_fold.h -- internal to libbcp's host layer (bcpf_ / bcpi_ names stay out
 * of the export map): the P role's window fold as the roles in bcp_task.c use
 * it.
 *
 *   bcp_fold.c     engines per device, the per-device fold service (flat
 *                  combining: every pending window of every lane and rank in
 *                  ONE descriptor launch), the pool of pinned window rows,
 *                  and the pipelined fold that follows the sources' reads
 *                  (row watches, range folds on the lane's queue);
 *   bcp_foldsrv.c  the node fold server: rank processes without a HIP
 *                  runtime send their windows (rows in a shared arena) to
 *                  ONE process that folds them through the same service.
 */
#pragma once

#include <pthread.h>

#include "bcp_host.h"

#define BCPF_MAX_DEVICES 64
#define BCPF_ROW_ALIGN 256u

/* ---- settings snapshot (bcp_task.c) ---------------------------------------- */
void bcpf_hook_get(bcp_xor_hook_fn *fn, void **ctx);

/* ---- engines (bcp_fold.c) -------------------------------------------------- */
/* The engine of storage target st's P role (device map, else st % ndev). */
int bcpf_engine_for_target(int st, bcp_engine **out, int *device);
/* Any live engine (for unregistering host memory), or NULL. */
bcp_engine *bcpf_any_engine(void);

/* ---- resident fold rings (bcp_ring_*, one per device) ----------------------- */
/* The device's ring (made on first use), or NULL if it cannot be made. */
bcp_ring *bcpf_ring_for(int dev, bcp_engine *e);
/* One window's fold on device dev: through its ring when use_ring (and the
 * ring exists), else the fold service; returns once it is on the host. */
int bcpf_fold_device(int dev, bcp_engine *e, int use_ring, const uint8_t *rows, size_t pitch, const size_t *valid,
                     size_t nbytes, int n, uint8_t *out);

/* ---- fold service ----------------------------------------------------------- */
typedef struct fold_svc fold_svc;
int bcpf_svc_get(int dev, bcp_engine *e, fold_svc **out);
/* out = XOR of n rows of `pitch` bytes, row j's first valid[j] bytes (zeros
 * past them), nbytes long; returns once it is on the host. */
int bcpf_fold_batched(fold_svc *S, const uint8_t *rows, size_t pitch, const size_t *valid, size_t nbytes, int n,
                      uint8_t *out);

/* ---- fold resources: pinned rows + output, pooled across tasks and lanes --- */
typedef struct fold_res {
    struct fold_res *next;
    int device;        /* -1: no GPU in this process (test hook, or folds by the node fold server) */
    bcp_engine *eng;
    bcp_queue *q;      /* the pipelined fold's range launches (made on first use) */
    uint8_t *h_win[2]; /* window rows [n][pitch] (pinned + device-mapped when device >= 0) */
    uint8_t *h_par;    /* fold output */
    size_t h_cap, h_cap1, hp_cap;
} fold_res;

/* Rows for rows_bytes (a second set when windows > 1) and an nbytes output
 * for storage target st; use_gpu = 0: plain or arena memory, no engine. */
int bcpf_res_acquire(int st, int use_gpu, size_t rows_bytes, size_t nbytes, uint64_t windows, fold_res **out);
void bcpf_res_release(fold_res *R);

/* One window's fold (replaces xor_parity at task_processing.c:211): by the
 * node fold server when the rows are in its arena, by the test hook when one
 * is set, else through the device's fold service.  tag: the lane's MPI tag. */
int bcpf_fold_window(fold_res *R, HostState *hs, int tag, bcp_xor_hook_fn hook, void *ctx, int use_ring,
                     const uint8_t *rows, size_t pitch, const size_t *valid, size_t nbytes, int n, uint8_t *out);

/* ---- pipelined fold: row watches ------------------------------------------ */
typedef struct row_watch {
    pthread_mutex_t mu;
    size_t prog[MAX_STORAGE_TARGETS];
    int redo; /* a published prefix was replaced (read error: zeros): fold it all again */
    int err;  /* first range-fold launch error */
    fold_res *R;
    bcp_xor_hook_fn hook;
    void *hook_ctx;
    const uint8_t *rows;
    size_t pitch, nbytes, lo; /* lo: bytes folded or claimed */
    const size_t *valid;
    uint8_t *out;
    size_t step; /* smallest range folded before the window is complete */
    int n;
    bcp_ring *ring; /* ranges go to the resident fold ring (else R->q) */
    uint64_t hnd[8];
    int nh;
} row_watch;
#define BCPF_WATCH_HANDLES 8

/* Bytes a source reads between two publishes of its row's final prefix
 * (256 KiB; bcp_task_set_fold_tuning "pipe_piece_kib"). */
size_t bcpf_watch_piece(void);


/* Register the window's n rows (1), or 0 when the table is full (fold it
 * whole).  The ranges go to `ring` when it is given, else R->q must exist
 * (unless hook is set). */
int bcpf_watch_rows(row_watch *W, fold_res *R, bcp_ring *ring, bcp_xor_hook_fn hook, void *hook_ctx,
                    const uint8_t *rows, size_t pitch, const size_t *valid, int n, size_t nbytes, uint8_t *out);
/* After the receives: unregister, fold the rest (fold = 0: only wait for the
 * ranges in flight), sync once.  0 or the first error. */
int bcpf_finish_rows(row_watch *W, int fold);
/* The same for a ring watch, without waiting: the rest is published and the
 * ring handles of every range in flight are handed to the caller (hnd has
 * room for BCPF_WATCH_HANDLES + 1), who waits for them before the rows or
 * the output are touched.  On an error every range has landed and nothing
 * is handed over. */
int bcpf_finish_rows_submit(row_watch *W, uint64_t *hnd, int *nh);
/* One whole window into the ring without waiting (*hnd for bcp_ring_wait). */
int bcpf_ring_submit_window(bcp_ring *r, const uint8_t *rows, size_t pitch, const size_t *valid, size_t nbytes,
                            int n, uint8_t *out, uint64_t *hnd);
/* The watch of the row being filled at `row` (row j of it), or NULL. */
row_watch *bcpf_watch_find(const void *row, int *j);
/* A source's new final prefix of row j; folds every range it completes. */
void bcpf_watch_publish(row_watch *w, int j, size_t bytes, int redo);

/* ---- node fold server, rank side (bcp_foldsrv.c) ------------------------- */
/* 1 once this process sends its folds to a node fold server. */
int bcpf_srv_attached(void);
/* The test double the server process inherited (fold requests ask for it). */
bcp_xor_hook_fn bcpf_srv_hook(void);
/* The fold of one window by the server (rows and out in the arena);
 * -ENXIO if they are not there, so the caller folds elsewhere. */
int bcpf_fold_remote(int st, int tag, const uint8_t *rows, size_t pitch, const size_t *valid, size_t nbytes, int n,
                     uint8_t *out, int with_hook);
