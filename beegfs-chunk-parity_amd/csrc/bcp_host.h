/* bcp_host.h -- internal to the C host layer of libbcp.so (not the ABI; the
 * bcpi_ prefix keeps these out of the export map). */
#pragma once

#include "bcp_task.h"

/* Failure injection (bcp_task_inject_failure): 1 if this pass through
 * `site` must fail. */
int bcpi_inject_hit(int site);
/* Non-zero once this library initialised a HIP runtime that found a device
 * (bcp_engine.hip): a forked child could not use it. */
int bcpi_hip_touched(void);

/* The P-role settings of this process (fold mode, fold service width, test
 * hook, window padding): a rank pool (bcp_pool.c) hands the caller's
 * settings to its rank processes with every run. */
typedef struct {
    int fold_mode, fold_inflight, explicit_pad, fold_ring;
    bcp_xor_hook_fn hook;
    void *hook_ctx;
} bcpi_settings;
void bcpi_settings_get(bcpi_settings *s);
int bcpi_settings_apply(const bcpi_settings *s);

/* Shared row arena of a socket world (bcp_sock.c): memory mapped shared
 * before the rank processes fork, so every rank sees it at the same address.
 * A rank's P role takes its window rows from its own slice; a source of
 * another process then reads its chunk straight into them (the socket
 * transport's fill send) instead of sending the bytes through the socket.
 * bcpi_arena_alloc returns NULL when this process has no slice or the slice
 * is full (the caller allocates elsewhere); bcpi_arena_free returns 1 if p
 * came from bcpi_arena_alloc. */
void *bcpi_arena_alloc(size_t bytes, size_t *got);
int bcpi_arena_free(void *p);
/* Fill sends of this process so far: into an arena row / as a message
 * (the receive lay outside the arena). */
void bcpi_sock_fill_counts(uint64_t *arena, uint64_t *msg);
/* The used arena block holding p (base, size); 0 if p is not in one. */
int bcpi_arena_block(const void *p, void **base, size_t *size);
/* Close every socket of w this process holds (the arena stays mapped). */
void bcpi_sock_world_close_fds(bcp_sock_world *w);
/* The whole arena of a world (every rank's slice); 0 if it has none. */
int bcpi_sock_world_arena(const bcp_sock_world *w, void **lo, void **hi);

/* Node fold server (bcp_foldsrv.c): ONE process holds the GPU and folds the
 * window rows of every rank process's P role, which live in the shared
 * arena, in batches across ranks (the fold service of bcp_fold.c, fed over
 * sockets); the ranks never start a HIP runtime.  The server runs
 * bcpi_foldsrv_main over its ends of nconn connections (one thread each)
 * until every one is closed; a rank attaches its own connections. */
int bcpi_foldsrv_main(int nconn, const int *fds, void *arena_lo, void *arena_hi);
void bcpi_foldsrv_attach(int nconn, const int *fds);
/* Windows the server folded for this process so far. */
uint64_t bcpi_foldsrv_folds(void);
/* 1 if ops is this library's socket transport (bcp_sock_world_attach). */
int bcpi_sock_transport_is(const bcp_transport_ops *ops);
/* The fold service's width (bcp_task_set_fold_inflight). */
int bcpi_fold_inflight(void);
/* PIPELINED folds through the resident fold ring (bcp_task_set_fold_ring). */
int bcpi_fold_ring(void);
/* Lane deferral depth of libbcp's runners (2; bcp_task_set_fold_tuning
 * "defer_depth"). */
int bcpi_defer_depth(void);
#define BCP_DEFER_MAX 4
/* Completion threads for deferred P tasks (4; bcp_task_set_fold_tuning
 * "completion_threads", 0 = each lane completes its own). */
#define BCP_COMPLETION_MAX 16
int bcpi_completion_threads(void);
/* The loopback transport's spin before a blocked wait sleeps, in us (0;
 * bcp_task_set_fold_tuning "lb_spin_us"); us < 0 only reads.  Returns the
 * previous value. */
int bcpi_lb_spin_us(int us);
/* Drain the deferred-completion queue and join its threads (bcp_task_shutdown). */
void bcpt_completion_stop(void);
/* Make [base, base + bytes) this process's arena slice (a memfd shared with
 * a node fold server, bcp_fold_server_connect). */
void bcpi_arena_set(void *base, size_t bytes);

/* 1 if path (n bytes, or up to its NUL when n is (size_t)-1) names a file
 * inside a target's chunks / parity directory: relative, no ".." component,
 * no embedded NUL (bcp_changelog.c). */
int bcpi_path_ok(const char *path, size_t n);
