/*
 * bcp_fold.c -- the P role's window fold on the GPU (what replaces
 * xor_parity at task_processing.c:211 inside parity_generator).
 *
 * Two ways to fold a window (bcp_task_set_fold_mode):
 *   BATCHED    the window goes to its device's fold service: flat combining,
 *              no thread of its own -- a waiting lane leads a launch that
 *              folds EVERY window pending on the device (all lanes, all
 *              ranks of this process, or of every rank process through the
 *              node fold server) as ONE descriptor batch, syncs once and
 *              wakes exactly the lanes it completed;
 *   PIPELINED  (default) the fold follows the sources' reads: the P role
 *              registers its window rows (row watches); a source filling one
 *              directly (loopback send_fill) reads its chunk in 256 KiB
 *              pieces and publishes each final prefix, and whoever completes
 *              a byte range of every row launches that range's fold on the P
 *              lane's queue without a sync; after the receives the P role
 *              folds the rest and syncs once.  Windows it cannot follow go to
 *              the fold service.
 * Both read the rows in place over PCIe (pinned, device-mapped host memory;
 * data bytes only -- the zero padding of a gen window is the kernel's).
 * Under PIPELINED the folds go to the device's resident fold ring
 * (bcp_ring_*, default; bcp_task_set_fold_ring): every range and window is
 * one publication into a launch that stays on the device, and the P lane
 * waits for its own pieces -- no launch and no stream sync per window.  With
 * the ring off, ranges launch on the P lane's queue and windows go to the
 * fold service as before.
 *
 * Resources are pooled: rows and output blocks stay pinned from task to
 * task (and run to run in a rank pool); engines are per device.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "bcp_fold.h"

#define MIN_(a, b) ((a) < (b) ? (a) : (b))
#define MAX_(a, b) ((a) > (b) ? (a) : (b))

static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER; /* engines, services, pool */

/* ---- engines ------------------------------------------------------------- */
static bcp_engine *g_engines[BCPF_MAX_DEVICES];
static int g_engine_rc[BCPF_MAX_DEVICES];
static int g_devmap[MAX_STORAGE_TARGETS];
static int g_devmap_n = 0;

int bcp_task_set_device_map(const int *devices, int ntargets)
{
    if (ntargets < 0 || ntargets > MAX_STORAGE_TARGETS || (ntargets && !devices))
        return -EINVAL;
    pthread_mutex_lock(&g_mu);
    for (int i = 0; i < ntargets; i++)
        g_devmap[i] = devices[i];
    g_devmap_n = ntargets;
    pthread_mutex_unlock(&g_mu);
    return 0;
}

int bcpf_engine_for_target(int st, bcp_engine **out, int *device)
{
    int ndev = 0;
    bcp_device_count(&ndev);
    if (ndev <= 0)
        return -ENODEV;
    int dev = st % ndev;
    pthread_mutex_lock(&g_mu);
    if (st < g_devmap_n)
        dev = g_devmap[st];
    if (dev < 0 || dev >= ndev || dev >= BCPF_MAX_DEVICES) {
        pthread_mutex_unlock(&g_mu);
        return -ENODEV;
    }
    if (!g_engines[dev] && !g_engine_rc[dev])
        g_engine_rc[dev] = bcp_engine_create(dev, &g_engines[dev]);
    int rc = g_engine_rc[dev];
    *out = g_engines[dev];
    pthread_mutex_unlock(&g_mu);
    *device = dev;
    return rc;
}

bcp_engine *bcpf_any_engine(void)
{
    bcp_engine *e = NULL;
    pthread_mutex_lock(&g_mu);
    for (int d = 0; d < BCPF_MAX_DEVICES && !e; d++)
        e = g_engines[d];
    pthread_mutex_unlock(&g_mu);
    return e;
}

/* ---- resident fold rings (one per device) ---------------------------------
 * Made on first use, destroyed by bcp_task_shutdown.  Workers: 16 worker
 * workgroups read host rows at the link's rate in the protocol's shape (3 x
 * 512 KiB stripes, 4-12 lanes: 56.6-57.0 GB/s, against 46.1 for one launch
 * per stripe and 47-48 with 64-128 workers; tools/exp/zero_copy_probe.py,
 * profiles/r06/protocol/zc_ring_r6a.jsonl). */
static bcp_ring *g_ring[BCPF_MAX_DEVICES];
static int g_ring_rc[BCPF_MAX_DEVICES];
static int g_fold_ring = 1;
static uint64_t g_ring_pieces, g_ring_launches; /* of rings already destroyed */
static int g_ring_spin_us = -1, g_ring_sleep_us = -1; /* bcp_task_set_ring_wait; -1: the engine's */
static int g_ring_workers = 16;
/* The pipelined fold's shape (bcp_task_set_fold_tuning): a source publishes
 * its row after every g_pipe_piece bytes read; a range is folded once every
 * row has at least max(g_pipe_step, window / 4) more bytes. */
static size_t g_pipe_piece = (size_t)256 << 10;
static size_t g_pipe_step = (size_t)128 << 10;
static int g_defer_depth = 2;
static int g_completion_threads = 4;

size_t bcpf_watch_piece(void) { return __atomic_load_n(&g_pipe_piece, __ATOMIC_RELAXED); }
int bcpi_defer_depth(void) { return __atomic_load_n(&g_defer_depth, __ATOMIC_RELAXED); }
int bcpi_completion_threads(void) { return __atomic_load_n(&g_completion_threads, __ATOMIC_RELAXED); }

int bcp_task_set_fold_tuning(const char *key, int value)
{
    if (!key)
        return -EINVAL;
    int prev;
    pthread_mutex_lock(&g_mu);
    if (!strcmp(key, "ring_workers") && value >= 1 && value <= 1024) {
        prev = g_ring_workers;
        g_ring_workers = value; /* rings made from now on: the current ones end below */
    } else if (!strcmp(key, "pipe_piece_kib") && value >= 4 && value <= 10240) {
        prev = (int)(g_pipe_piece >> 10);
        __atomic_store_n(&g_pipe_piece, (size_t)value << 10, __ATOMIC_RELAXED);
    } else if (!strcmp(key, "pipe_step_kib") && value >= 4 && value <= 10240) {
        prev = (int)(g_pipe_step >> 10);
        g_pipe_step = (size_t)value << 10;
    } else if (!strcmp(key, "defer_depth") && value >= 0 && value <= BCP_DEFER_MAX) {
        prev = g_defer_depth;
        __atomic_store_n(&g_defer_depth, value, __ATOMIC_RELAXED);
    } else if (!strcmp(key, "lb_spin_us") && value >= 0 && value <= 1000) {
        prev = bcpi_lb_spin_us(value);
    } else if (!strcmp(key, "completion_threads") && value >= 0 && value <= BCP_COMPLETION_MAX) {
        prev = g_completion_threads; /* more start on next use; fewer after bcp_task_shutdown */
        __atomic_store_n(&g_completion_threads, value, __ATOMIC_RELAXED);
    } else {
        prev = -EINVAL;
    }
    /* a new worker count: the devices' rings end now (no fold may be in
     * flight: between runs), the next fold makes them anew */
    bcp_ring *old_ring[BCPF_MAX_DEVICES] = {0};
    if (!strcmp(key, "ring_workers") && prev >= 0 && prev != value)
        for (int d = 0; d < BCPF_MAX_DEVICES; d++) {
            old_ring[d] = g_ring[d];
            g_ring[d] = NULL;
            g_ring_rc[d] = 0;
            if (old_ring[d]) {
                uint64_t a = 0, b = 0;
                (void)bcp_ring_stats(old_ring[d], &a, &b);
                g_ring_pieces += a;
                g_ring_launches += b;
            }
        }
    pthread_mutex_unlock(&g_mu);
    for (int d = 0; d < BCPF_MAX_DEVICES; d++)
        if (old_ring[d])
            (void)bcp_ring_destroy(old_ring[d]);
    return prev;
}

int bcp_task_set_fold_ring(int on)
{
    if (on != 0 && on != 1)
        return -EINVAL;
    pthread_mutex_lock(&g_mu);
    const int prev = g_fold_ring;
    g_fold_ring = on;
    pthread_mutex_unlock(&g_mu);
    return prev;
}

int bcpi_fold_ring(void)
{
    pthread_mutex_lock(&g_mu);
    const int on = g_fold_ring;
    pthread_mutex_unlock(&g_mu);
    return on;
}

bcp_ring *bcpf_ring_for(int dev, bcp_engine *e)
{
    if (dev < 0 || dev >= BCPF_MAX_DEVICES || !e)
        return NULL;
    pthread_mutex_lock(&g_mu);
    if (!g_ring[dev] && !g_ring_rc[dev]) {
        g_ring_rc[dev] = bcp_ring_create(e, g_ring_workers, 0, &g_ring[dev]);
        if (!g_ring_rc[dev] && g_ring_spin_us >= 0)
            (void)bcp_ring_set_wait(g_ring[dev], g_ring_spin_us, g_ring_sleep_us);
    }
    bcp_ring *r = g_ring[dev];
    pthread_mutex_unlock(&g_mu);
    return r;
}

int bcp_task_set_ring_wait(int spin_us, int sleep_us)
{
    if (spin_us < 0 || spin_us > 1000000 || sleep_us < 0 || sleep_us > 100000)
        return -EINVAL;
    pthread_mutex_lock(&g_mu);
    g_ring_spin_us = spin_us;
    g_ring_sleep_us = sleep_us;
    for (int d = 0; d < BCPF_MAX_DEVICES; d++)
        if (g_ring[d])
            (void)bcp_ring_set_wait(g_ring[d], spin_us, sleep_us);
    pthread_mutex_unlock(&g_mu);
    return 0;
}

int bcp_task_ring_stats(uint64_t *pieces, uint64_t *launches)
{
    uint64_t p = 0, l = 0;
    pthread_mutex_lock(&g_mu);
    p = g_ring_pieces;
    l = g_ring_launches;
    for (int d = 0; d < BCPF_MAX_DEVICES; d++)
        if (g_ring[d]) {
            uint64_t a = 0, b = 0;
            (void)bcp_ring_stats(g_ring[d], &a, &b);
            p += a;
            l += b;
        }
    pthread_mutex_unlock(&g_mu);
    if (pieces)
        *pieces = p;
    if (launches)
        *launches = l;
    return 0;
}

/* One stripe through the ring: n rows at `pitch`, row j's first valid[j]
 * bytes, into out[0, nbytes); returns once it is on the host. */
static int ring_fold(bcp_ring *r, const uint8_t *rows, size_t pitch, const size_t *valid, size_t nbytes, int n,
                     uint8_t *out)
{
    uint64_t h = 0;
    int rc = bcpf_ring_submit_window(r, rows, pitch, valid, nbytes, n, out, &h);
    return rc ? rc : bcp_ring_wait(r, h);
}

int bcpf_fold_device(int dev, bcp_engine *e, int use_ring, const uint8_t *rows, size_t pitch, const size_t *valid,
                     size_t nbytes, int n, uint8_t *out)
{
    bcp_ring *r = use_ring ? bcpf_ring_for(dev, e) : NULL;
    if (r)
        return ring_fold(r, rows, pitch, valid, nbytes, n, out);
    fold_svc *S = NULL;
    int rc = bcpf_svc_get(dev, e, &S);
    return rc ? rc : bcpf_fold_batched(S, rows, pitch, valid, nbytes, n, out);
}

/* ---- fold service ----------------------------------------------------------
 * One per device.  A P role appends its window and, if fewer than
 * max_inflight batches are on the device, becomes a leader: it takes EVERY
 * pending window (its own included), folds them with one descriptor batch on
 * a free slot's queue, syncs once and completes them all; otherwise it
 * sleeps until a leader has completed its window, or is woken to lead a
 * later batch.  A lone lane (the single rebuild lane) folds its own window
 * directly; when every slot is busy, the windows that arrive meanwhile share
 * the next launch. */
typedef struct fold_job {
    struct fold_job *next;
    const uint8_t *rows;
    size_t pitch, nbytes;
    const size_t *valid;
    int n;
    uint8_t *out;
    int done, rc;
    pthread_cond_t cv; /* its lane sleeps here: woken when done, or to lead */
} fold_job;

#define MAX_INFLIGHT 16

typedef struct {
    bcp_queue *q;
    bcp_stripe *st;
    bcp_source *so;
    size_t st_cap, so_cap;
    int busy;
} fold_slot;

struct fold_svc {
    bcp_engine *eng;
    int inflight;     /* batches on the device (leaders folding) */
    int max_inflight; /* concurrent batches, each on its own slot's queue */
    fold_slot slot[MAX_INFLIGHT];
    pthread_mutex_t mu;
    fold_job *head, *tail;
    uint64_t windows, launches;
};

static fold_svc *g_svc[BCPF_MAX_DEVICES];
static uint64_t g_svc_windows, g_svc_launches; /* of services already shut down */
static int g_fold_inflight = 1;

int bcp_task_set_fold_inflight(int k)
{
    if (k < 1 || k > MAX_INFLIGHT)
        return -EINVAL;
    pthread_mutex_lock(&g_mu);
    const int prev = g_fold_inflight;
    g_fold_inflight = k;
    for (int d = 0; d < BCPF_MAX_DEVICES; d++)
        if (g_svc[d]) {
            pthread_mutex_lock(&g_svc[d]->mu);
            g_svc[d]->max_inflight = k;
            pthread_mutex_unlock(&g_svc[d]->mu);
        }
    pthread_mutex_unlock(&g_mu);
    return prev;
}

int bcpi_fold_inflight(void)
{
    pthread_mutex_lock(&g_mu);
    const int k = g_fold_inflight;
    pthread_mutex_unlock(&g_mu);
    return k;
}

static int slot_tables(fold_slot *F, size_t nst, size_t nso)
{
    if (nst > F->st_cap) {
        bcp_stripe *p = realloc(F->st, nst * 2 * sizeof(*p));
        if (!p)
            return -ENOMEM;
        F->st = p;
        F->st_cap = nst * 2;
    }
    if (nso > F->so_cap) {
        bcp_source *p = realloc(F->so, nso * 2 * sizeof(*p));
        if (!p)
            return -ENOMEM;
        F->so = p;
        F->so_cap = nso * 2;
    }
    return 0;
}

/* A leader's batch on its slot (called without S->mu; the slot is its own). */
static int slot_fold(fold_svc *S, fold_slot *F, fold_job *batch)
{
    int rc = F->q ? 0 : bcp_queue_create(S->eng, &F->q);
    if (rc)
        return rc;
    size_t nst = 0, nso = 0;
    for (fold_job *j = batch; j; j = j->next) {
        nst++;
        nso += (size_t)j->n;
    }
    rc = nst > 0xFFFFFFFFu || nso > 0xFFFFFFFFu ? -EINVAL : slot_tables(F, nst, nso);
    if (rc)
        return rc;
    size_t i = 0, k = 0;
    for (fold_job *j = batch; j; j = j->next, i++) {
        F->st[i] = (bcp_stripe){(uint64_t)(uintptr_t)j->out, j->nbytes, (uint32_t)k, (uint32_t)j->n, 0};
        for (int r = 0; r < j->n; r++, k++)
            F->so[k] = (bcp_source){(uint64_t)(uintptr_t)(j->rows + (size_t)r * j->pitch), j->valid[r]};
    }
    rc = bcp_xor_stripes_async(F->q, F->st, (uint32_t)nst, F->so, (uint32_t)nso);
    return rc ? rc : bcp_queue_sync(F->q);
}

static void svc_destroy(fold_svc *S)
{
    if (!S)
        return;
    for (int i = 0; i < MAX_INFLIGHT; i++) {
        if (S->slot[i].q)
            bcp_queue_destroy(S->slot[i].q); /* synchronises first */
        free(S->slot[i].st);
        free(S->slot[i].so);
    }
    pthread_mutex_destroy(&S->mu);
    free(S);
}

int bcpf_svc_get(int dev, bcp_engine *e, fold_svc **out)
{
    pthread_mutex_lock(&g_mu);
    fold_svc *S = g_svc[dev];
    int rc = 0;
    if (!S) {
        S = calloc(1, sizeof(*S));
        if (!S)
            rc = -ENOMEM;
        else {
            S->eng = e;
            S->max_inflight = g_fold_inflight;
            pthread_mutex_init(&S->mu, NULL);
            g_svc[dev] = S;
        }
    }
    pthread_mutex_unlock(&g_mu);
    *out = S;
    return rc;
}

int bcpf_fold_batched(fold_svc *S, const uint8_t *rows, size_t pitch, const size_t *valid, size_t nbytes, int n,
                      uint8_t *out)
{
    fold_job j = {.rows = rows, .pitch = pitch, .nbytes = nbytes, .valid = valid, .n = n, .out = out};
    pthread_cond_init(&j.cv, NULL);
    pthread_mutex_lock(&S->mu);
    if (S->tail)
        S->tail->next = &j;
    else
        S->head = &j;
    S->tail = &j;
    while (!j.done) {
        if (S->inflight >= S->max_inflight || !S->head) {
            pthread_cond_wait(&j.cv, &S->mu);
            continue;
        }
        /* lead a batch: everything pending (this window, unless another
         * leader took it already) on a free slot */
        fold_slot *F = NULL;
        for (int i = 0; i < MAX_INFLIGHT && !F; i++)
            if (!S->slot[i].busy)
                F = &S->slot[i];
        F->busy = 1;
        S->inflight++;
        fold_job *batch = S->head;
        S->head = S->tail = NULL;
        pthread_mutex_unlock(&S->mu);
        const int rc = slot_fold(S, F, batch);
        pthread_mutex_lock(&S->mu);
        size_t nb = 0;
        for (fold_job *x = batch, *nx; x; x = nx, nb++) {
            nx = x->next; /* x lives on its lane's stack: read next before done */
            x->rc = rc;
            x->done = 1;
            if (x != &j)
                pthread_cond_signal(&x->cv); /* its lane runs once we unlock */
        }
        S->windows += nb;
        S->launches += 1;
        S->inflight--;
        F->busy = 0;
        if (S->head)
            pthread_cond_signal(&S->head->cv); /* windows that came meanwhile: a leader */
    }
    pthread_mutex_unlock(&S->mu);
    pthread_cond_destroy(&j.cv);
    return j.rc;
}

int bcp_task_fold_stats(uint64_t *windows, uint64_t *launches)
{
    uint64_t w = 0, l = 0;
    pthread_mutex_lock(&g_mu);
    w = g_svc_windows;
    l = g_svc_launches;
    for (int d = 0; d < BCPF_MAX_DEVICES; d++)
        if (g_svc[d]) {
            pthread_mutex_lock(&g_svc[d]->mu);
            w += g_svc[d]->windows;
            l += g_svc[d]->launches;
            pthread_mutex_unlock(&g_svc[d]->mu);
        }
    pthread_mutex_unlock(&g_mu);
    if (windows)
        *windows = w;
    if (launches)
        *launches = l;
    return 0;
}

/* ---- fold resources -------------------------------------------------------
 * One resource = window rows (two sets for a multi-window task: the next
 * window is received while one is folded) + an output block, pinned and
 * device-mapped (registered huge-page memory, bcp_host_alloc_mapped); from
 * this rank's slice of a shared row arena when the process has one (rank
 * processes: other ranks' sources read their chunks straight into them, and
 * a node fold server reads them), registered with the GPU when this process
 * folds.  Host-only resources (test hook, node fold server) use plain or
 * arena memory.  Every free happens with no work in flight on it: a task's
 * folds are synchronised before its resource returns to the pool, and the
 * pool is emptied by bcp_task_shutdown after every lane has returned. */
static fold_res *g_pool = NULL; /* free list, under g_mu */

static void host_free(fold_res *R, void *p)
{
    if (!p)
        return;
    void *ab;
    size_t az;
    if (bcpi_arena_block(p, &ab, &az) && ab == p) {
        /* a block of the shared arena: the mapping stays.  Unregistered before
         * it goes back to the arena, so another lane that takes the block next
         * registers it for itself and no unregister of ours can follow that. */
        if (R->device >= 0)
            (void)bcp_host_unregister(R->eng, p);
        bcpi_arena_free(p);
        return;
    }
    if (R->device >= 0)
        bcp_host_free(R->eng, p);
    else
        free(p);
}

static void res_destroy(fold_res *R)
{
    if (R->q)
        bcp_queue_destroy(R->q); /* synchronises first: no range fold reads the rows below */
    host_free(R, R->h_win[0]);
    host_free(R, R->h_win[1]);
    host_free(R, R->h_par);
    free(R);
}

void bcpf_res_release(fold_res *R)
{
    if (!R)
        return;
    pthread_mutex_lock(&g_mu);
    R->next = g_pool;
    g_pool = R;
    pthread_mutex_unlock(&g_mu);
}

/* arena: take the block from the shared arena when there is one */
static int grow(fold_res *R, uint8_t **p, size_t *cap, size_t need, int arena)
{
    if (*cap >= need && *p)
        return 0;
    host_free(R, *p);
    *p = NULL;
    *cap = 0;
    /* next power of two (>= 1 MiB): a worklist sorted by size (gen/main.c:
     * 703-715) would otherwise re-pin rows at nearly every task */
    size_t c = (size_t)1 << 20;
    while (c < need)
        c <<= 1;
    if (arena && (*p = bcpi_arena_alloc(c, &c))) {
        if (R->device < 0 || !bcp_host_register(R->eng, *p, c)) {
            *cap = c;
            return 0;
        }
        bcpi_arena_free(*p); /* not addressable by the device: ordinary memory */
        *p = NULL;
        c = (size_t)1 << 20;
        while (c < need)
            c <<= 1;
    }
    int rc = 0;
    if (R->device >= 0)
        rc = bcp_host_alloc_mapped(R->eng, c, (void **)p);
    else if (!(*p = malloc(c)))
        rc = -ENOMEM;
    if (!rc)
        *cap = c;
    return rc;
}

int bcpf_res_acquire(int st, int use_gpu, size_t rows_bytes, size_t nbytes, uint64_t windows, fold_res **out)
{
    int rc = 0, dev = -1;
    bcp_engine *e = NULL;
    *out = NULL;
    if (bcpi_inject_hit(BCP_INJECT_FOLD_RES))
        return -ENOMEM;
    if (use_gpu && (rc = bcpf_engine_for_target(st, &e, &dev)))
        return rc;
    /* prefer a free resource of the same device that is already big enough */
    pthread_mutex_lock(&g_mu);
    fold_res **best = NULL;
    for (fold_res **pp = &g_pool; *pp; pp = &(*pp)->next) {
        if ((*pp)->device != dev)
            continue;
        if (!best)
            best = pp;
        if ((*pp)->h_cap >= rows_bytes && ((*pp)->h_cap1 >= rows_bytes || windows < 2) && (*pp)->hp_cap >= nbytes) {
            best = pp;
            break;
        }
    }
    fold_res *R = NULL;
    if (best) {
        R = *best;
        *best = R->next;
        R->next = NULL;
    }
    pthread_mutex_unlock(&g_mu);
    if (!R) {
        R = calloc(1, sizeof(*R));
        if (!R)
            return -ENOMEM;
        R->device = dev;
        R->eng = e;
    }
    if ((rc = grow(R, &R->h_win[0], &R->h_cap, rows_bytes, 1)) ||
        (windows > 1 && (rc = grow(R, &R->h_win[1], &R->h_cap1, rows_bytes, 1))) ||
        (rc = grow(R, &R->h_par, &R->hp_cap, nbytes, dev < 0 && bcpf_srv_attached()))) {
        res_destroy(R); /* (with a node fold server the output is an arena block too) */
        return rc;
    }
    *out = R;
    return 0;
}

int bcpf_fold_window(fold_res *R, HostState *hs, int tag, bcp_xor_hook_fn hook, void *ctx, int use_ring,
                     const uint8_t *rows, size_t pitch, const size_t *valid, size_t nbytes, int n, uint8_t *out)
{
    void *ab;
    size_t az;
    /* the node fold server folds (with a test double only if it has the
     * same one: it was forked when the pool was made) */
    if (R->device < 0 && bcpf_srv_attached() && (!hook || hook == bcpf_srv_hook()) && bcpi_arena_block(rows, &ab, &az))
        return bcpf_fold_remote(hs->storage_target, tag, rows, pitch, valid, nbytes, n, out, hook != NULL);
    if (hook) {
        static int warned = 0; /* lanes race here: atomic exchange */
        if (!__atomic_exchange_n(&warned, 1, __ATOMIC_RELAXED) && hs->log) {
            fprintf(hs->log, "bcp_fold.c: XOR test hook active on st %d (no GPU fold)\n", hs->storage_target);
            fflush(hs->log);
        }
        return hook(out, nbytes, rows, pitch, n, ctx);
    }
    return bcpf_fold_device(R->device, R->eng, use_ring, rows, pitch, valid, nbytes, n, out);
}

/* ---- pipelined fold: row watches -------------------------------------------
 * A P role that folds its window range by range registers the window's rows
 * here, keyed by row address; a source that fills one of them directly reads
 * its chunk in pieces and publishes, after each, how many leading bytes of
 * the row are final.  Open addressing with backward-shift deletion; the live
 * count lets every other fill skip the lock.  An entry lives exactly from
 * bcpf_watch_rows to bcpf_finish_rows of its window: both run on the P lane,
 * around the receives, and every fill into the rows has returned before the
 * receives complete, so no publish can reach a watch after its window. */
#define WATCH_SLOTS 4096u
#define PIPE_ALIGN ((size_t)4096)     /* range boundaries */

typedef struct {
    const void *row;
    row_watch *w;
    int j;
} watch_slot;
static watch_slot g_watch[WATCH_SLOTS];
static pthread_mutex_t g_watch_lock = PTHREAD_MUTEX_INITIALIZER;
static size_t g_watch_live;
static uint64_t g_pipe_windows, g_pipe_ranges; /* bcp_task_pipe_stats */

int bcp_task_pipe_stats(uint64_t *windows, uint64_t *ranges)
{
    if (windows)
        *windows = __atomic_load_n(&g_pipe_windows, __ATOMIC_RELAXED);
    if (ranges)
        *ranges = __atomic_load_n(&g_pipe_ranges, __ATOMIC_RELAXED);
    return 0;
}

size_t bcp_task_watch_live(void)
{
    return __atomic_load_n(&g_watch_live, __ATOMIC_ACQUIRE);
}

static size_t watch_hash(const void *p)
{
    uint64_t x = (uint64_t)(uintptr_t)p;
    x ^= x >> 29;
    x *= UINT64_C(0xbf58476d1ce4e5b9);
    x ^= x >> 32;
    return (size_t)x & (WATCH_SLOTS - 1);
}

/* 0, or -ENOSPC when the table is half full (the caller folds unwatched). */
static int watch_add(const void *row, row_watch *w, int j)
{
    pthread_mutex_lock(&g_watch_lock);
    if (g_watch_live * 2 >= WATCH_SLOTS) {
        pthread_mutex_unlock(&g_watch_lock);
        return -ENOSPC;
    }
    size_t i = watch_hash(row);
    while (g_watch[i].row)
        i = (i + 1) & (WATCH_SLOTS - 1);
    g_watch[i] = (watch_slot){row, w, j};
    __atomic_store_n(&g_watch_live, g_watch_live + 1, __ATOMIC_RELEASE);
    pthread_mutex_unlock(&g_watch_lock);
    return 0;
}

static void watch_del(const void *row)
{
    pthread_mutex_lock(&g_watch_lock);
    size_t i = watch_hash(row);
    while (g_watch[i].row && g_watch[i].row != row)
        i = (i + 1) & (WATCH_SLOTS - 1);
    if (g_watch[i].row) {
        /* backward shift: pull later entries of the probe run into the hole */
        size_t hole = i;
        for (size_t k = (i + 1) & (WATCH_SLOTS - 1); g_watch[k].row; k = (k + 1) & (WATCH_SLOTS - 1)) {
            const size_t home = watch_hash(g_watch[k].row);
            if (((k - home) & (WATCH_SLOTS - 1)) >= ((k - hole) & (WATCH_SLOTS - 1))) {
                g_watch[hole] = g_watch[k];
                hole = k;
            }
        }
        g_watch[hole].row = NULL;
        __atomic_store_n(&g_watch_live, g_watch_live - 1, __ATOMIC_RELEASE);
    }
    pthread_mutex_unlock(&g_watch_lock);
}

row_watch *bcpf_watch_find(const void *row, int *j)
{
    if (!__atomic_load_n(&g_watch_live, __ATOMIC_ACQUIRE))
        return NULL;
    row_watch *w = NULL;
    pthread_mutex_lock(&g_watch_lock);
    for (size_t i = watch_hash(row); g_watch[i].row; i = (i + 1) & (WATCH_SLOTS - 1))
        if (g_watch[i].row == row) {
            w = g_watch[i].w;
            *j = g_watch[i].j;
            break;
        }
    pthread_mutex_unlock(&g_watch_lock);
    return w;
}

/* Fold out[lo, hi) = XOR of the rows' [lo, hi) on the lane's queue, no sync
 * (under the test hook: the hook, at once, over whole rows whose padding the
 * P role zeroed before the receives).  Callers hold w->mu: the queue is one
 * lane's, and launches on it must not interleave. */
static int launch_range(row_watch *w, size_t lo, size_t hi)
{
    __atomic_fetch_add(&g_pipe_ranges, 1, __ATOMIC_RELAXED);
    if (w->hook)
        return w->hook(w->out + lo, hi - lo, w->rows + lo, w->pitch, w->n, w->hook_ctx);
    bcp_stripe st = {(uint64_t)(uintptr_t)(w->out + lo), hi - lo, 0, (uint32_t)w->n, 0};
    bcp_source so[MAX_STORAGE_TARGETS];
    for (int j = 0; j < w->n; j++) {
        const size_t len = w->valid[j] > lo ? MIN_(w->valid[j], hi) - lo : 0;
        so[j] = (bcp_source){(uint64_t)(uintptr_t)(w->rows + (size_t)j * w->pitch + lo), len};
    }
    if (!w->ring)
        return bcp_xor_stripes_async(w->R->q, &st, 1, so, (uint32_t)w->n);
    if (w->nh == BCPF_WATCH_HANDLES) {
        /* (ranges are at least a quarter window: never more than ~5) */
        for (int i = 0; i < w->nh; i++) {
            const int rc = bcp_ring_wait(w->ring, w->hnd[i]);
            if (rc)
                return rc;
        }
        w->nh = 0;
    }
    uint64_t h = 0;
    const int rc = bcp_ring_submit(w->ring, &st, so, &h);
    if (!rc)
        w->hnd[w->nh++] = h;
    return rc;
}

/* Under w->mu: launch every range all rows have delivered past w->lo. */
static void range_claim(row_watch *w)
{
    while (!w->redo && !w->err && w->lo < w->nbytes) {
        size_t avail = w->nbytes;
        for (int j = 0; j < w->n; j++)
            avail = MIN_(avail, w->prog[j] >= w->valid[j] ? w->nbytes : w->prog[j]);
        if (avail < w->nbytes && avail < w->lo + w->step)
            return;
        const size_t hi = avail >= w->nbytes ? w->nbytes : avail / PIPE_ALIGN * PIPE_ALIGN;
        const int rc = launch_range(w, w->lo, hi);
        if (rc)
            w->err = rc;
        else
            w->lo = hi;
    }
}

/* A source's new final prefix of row j; the range it completes is folded by
 * this thread (the P lane may not get a CPU before the reads end: a woken
 * source runs on the CPU of the lane that posted its receive). */
void bcpf_watch_publish(row_watch *w, int j, size_t bytes, int redo)
{
    pthread_mutex_lock(&w->mu);
    if (bytes > w->prog[j])
        w->prog[j] = bytes;
    w->redo |= redo;
    range_claim(w);
    pthread_mutex_unlock(&w->mu);
}

int bcpf_watch_rows(row_watch *W, fold_res *R, bcp_ring *ring, bcp_xor_hook_fn hook, void *hook_ctx,
                    const uint8_t *rows, size_t pitch, const size_t *valid, int n, size_t nbytes, uint8_t *out)
{
    pthread_mutex_init(&W->mu, NULL);
    W->ring = hook ? NULL : ring;
    W->nh = 0;
    memset(W->prog, 0, sizeof(W->prog));
    W->redo = W->err = 0;
    W->R = R;
    W->hook = hook;
    W->hook_ctx = hook_ctx;
    W->rows = rows;
    W->pitch = pitch;
    W->nbytes = nbytes;
    W->lo = 0;
    W->valid = valid;
    W->out = out;
    pthread_mutex_lock(&g_mu);
    const size_t step = g_pipe_step;
    pthread_mutex_unlock(&g_mu);
    W->step = MAX_(step, nbytes / 4); /* at most ~5 ranges per window */
    W->n = n;
    for (int j = 0; j < n; j++)
        if (watch_add(rows + (size_t)j * pitch, W, j)) {
            while (j-- > 0)
                watch_del(rows + (size_t)j * pitch);
            pthread_mutex_destroy(&W->mu);
            return 0;
        }
    return 1;
}

/* (Writing the ranges folded so far while the last one folds, behind an
 * event the launching source records, measured slower on every workload --
 * config 5 by a quarter, r2bh / r2bi -- and is gone.) */
/* Wait for every range of W in the ring (0 or the first error). */
static int ring_wait_all(row_watch *W)
{
    int rc = 0;
    for (int i = 0; i < W->nh; i++) {
        const int e = bcp_ring_wait(W->ring, W->hnd[i]);
        rc = rc ? rc : e;
    }
    W->nh = 0;
    return rc;
}

/* Unregister the rows and launch what is left to fold (fold = 0: nothing).
 * A redo (a source replaced published bytes with zeros) refolds the whole
 * window -- in the ring only after the ranges in flight have landed: ring
 * pieces run side by side, so an earlier range could otherwise overwrite
 * the refold's output with what it read before the zeros. */
static int finish_launch(row_watch *W, int fold, int *wait_rc)
{
    for (int j = 0; j < W->n; j++)
        watch_del(W->rows + (size_t)j * W->pitch);
    int rc = W->err;
    const size_t lo = W->redo ? 0 : W->lo;
    __atomic_fetch_add(&g_pipe_windows, 1, __ATOMIC_RELAXED);
    *wait_rc = 0;
    if (W->ring && W->redo)
        *wait_rc = ring_wait_all(W);
    if (fold && !rc && lo < W->nbytes)
        rc = launch_range(W, lo, W->nbytes);
    return rc;
}

int bcpf_finish_rows(row_watch *W, int fold)
{
    int wrc = 0;
    const int rc = finish_launch(W, fold, &wrc);
    /* the one wait -- also after an error: ranges may be in flight */
    int src = wrc;
    if (W->ring) {
        const int e = ring_wait_all(W);
        src = src ? src : e;
    } else if (!W->hook) {
        src = bcp_queue_sync(W->R->q);
    }
    pthread_mutex_destroy(&W->mu);
    return rc ? rc : src;
}

int bcpf_finish_rows_submit(row_watch *W, uint64_t *hnd, int *nh)
{
    int wrc = 0;
    int rc = finish_launch(W, 1, &wrc);
    rc = rc ? rc : wrc;
    if (rc) /* nothing is handed over: every range in flight lands first */
        (void)ring_wait_all(W);
    for (int i = 0; i < W->nh; i++)
        hnd[i] = W->hnd[i];
    *nh = W->nh;
    W->nh = 0;
    pthread_mutex_destroy(&W->mu);
    return rc;
}

int bcpf_ring_submit_window(bcp_ring *r, const uint8_t *rows, size_t pitch, const size_t *valid, size_t nbytes,
                            int n, uint8_t *out, uint64_t *hnd)
{
    bcp_stripe st = {(uint64_t)(uintptr_t)out, nbytes, 0, (uint32_t)n, 0};
    bcp_source so[MAX_STORAGE_TARGETS];
    for (int j = 0; j < n; j++)
        so[j] = (bcp_source){(uint64_t)(uintptr_t)(rows + (size_t)j * pitch), MIN_(valid[j], nbytes)};
    return bcp_ring_submit(r, &st, so, hnd);
}

/* ---- shutdown -------------------------------------------------------------- */
int bcp_task_shutdown(void)
{
    bcp_task_thread_release();
    bcpt_completion_stop(); /* every lane has returned: the queue drains */
    /* fold services first: they hold queues on the engines (all lanes have
     * returned, so no batch is in flight) */
    pthread_mutex_lock(&g_mu);
    fold_svc *svc[BCPF_MAX_DEVICES];
    for (int d = 0; d < BCPF_MAX_DEVICES; d++) {
        svc[d] = g_svc[d];
        g_svc[d] = NULL;
        if (svc[d]) {
            g_svc_windows += svc[d]->windows;
            g_svc_launches += svc[d]->launches;
        }
    }
    fold_res *R = g_pool;
    g_pool = NULL;
    bcp_ring *ring[BCPF_MAX_DEVICES];
    for (int d = 0; d < BCPF_MAX_DEVICES; d++) {
        ring[d] = g_ring[d];
        g_ring[d] = NULL;
        g_ring_rc[d] = 0;
        if (ring[d]) {
            uint64_t a = 0, b = 0;
            (void)bcp_ring_stats(ring[d], &a, &b);
            g_ring_pieces += a;
            g_ring_launches += b;
        }
    }
    pthread_mutex_unlock(&g_mu);
    for (int d = 0; d < BCPF_MAX_DEVICES; d++)
        svc_destroy(svc[d]);
    for (int d = 0; d < BCPF_MAX_DEVICES; d++)
        if (ring[d])
            (void)bcp_ring_destroy(ring[d]); /* every lane has returned: nothing pending */
    while (R) {
        fold_res *nx = R->next;
        res_destroy(R);
        R = nx;
    }
    pthread_mutex_lock(&g_mu);
    for (int d = 0; d < BCPF_MAX_DEVICES; d++) {
        if (g_engines[d])
            bcp_engine_destroy(g_engines[d]);
        g_engines[d] = NULL;
        g_engine_rc[d] = 0;
    }
    pthread_mutex_unlock(&g_mu);
    return 0;
}
