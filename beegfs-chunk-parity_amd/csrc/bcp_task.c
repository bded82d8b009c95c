/*
 * bcp_task.c -- the per-rank chunk-streaming protocol (process_task) with the
 * P role's fold on the GPU.
 *
 * Behaviour follows the reference's roles and message flow
 * (src/beegfs-raid5/common/task_processing.c):
 *   process_task      :325-340  dispatch by role
 *   parity_generator  :117-245  P role: sizes -> max_cs -> windows -> parity
 *   chunk_sender      :247-322  source role: size -> windows (zero padded)
 * What is underneath is this library's:
 *   - the peers are reached through a transport table (bcp_task_set_transport:
 *     in-process loopback ranks by default, socketpair-connected rank
 *     processes, or an MPI binding), exactly the point-to-point subset the
 *     reference uses;
 *   - the window fold (xor_parity at :211) runs on the GPU over pinned,
 *     device-mapped window rows (256-byte pitch, so every row is 16-byte
 *     aligned for the streaming kernel): per lane on its own HIP queue --
 *     rows DMA'd to HBM one by one as they arrive, data bytes only (STREAMED),
 *     read in place over PCIe (ZERO_COPY), or copied after the last one
 *     (STAGED) -- or through a per-device fold service that batches the
 *     pending windows of every lane and rank into one launch (BATCHED);
 *   - nothing aborts: when the P role cannot get fold resources it still
 *     drains its senders through one bounded row and raises the sticky error;
 *     a source without a window buffer sends zeros and raises it.
 */
#define _GNU_SOURCE
#include <assert.h>
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <time.h>
#include <unistd.h>

#include "bcp_host.h"

#define WINDOW ((uint64_t)BCP_WINDOW_BYTES)
#define ROW_ALIGN 256u
#define MAX_DEVICES 64
#define DRAIN_SMALL 16384u

__attribute__((weak)) int st2rank[MAX_STORAGE_TARGETS];

#define LOGERR(format, ...)                                                                      \
    do {                                                                                        \
        if (hs->log) {                                                                          \
            fprintf(hs->log, "%s:%d (%s): " format, __FILE__, __LINE__, __func__, __VA_ARGS__); \
            fflush(hs->log);                                                                    \
        }                                                                                       \
    } while (0)

#define MIN_(a, b) ((a) < (b) ? (a) : (b))
#define MAX_(a, b) ((a) > (b) ? (a) : (b))

/* ---- global state: engines, device map, test hook, transport ------------ */
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static bcp_engine *g_engines[MAX_DEVICES];
static int g_engine_rc[MAX_DEVICES];
static int g_devmap[MAX_STORAGE_TARGETS];
static int g_devmap_n = 0;
static bcp_xor_hook_fn g_hook = NULL;
static void *g_hook_ctx = NULL;
static int g_fold_mode = BCP_FOLD_PIPELINED;
static int g_explicit_pad = 0; /* 1: sources pad every window, as the reference does */
static bcp_transport_ops g_tp;
static int g_tp_set = 0;

/* Never written: the source role's windows when it has no buffer of its own
 * (zero pages until read; .bss costs no file or resident memory). */
static uint8_t g_zero_window[BCP_WINDOW_BYTES];

/* ---- row watches (BCP_FOLD_PIPELINED) ------------------------------------
 * A P role that folds its window range by range registers the window's rows
 * here, keyed by row address; a source that fills one of them directly
 * (send_fill) reads its chunk in pieces and publishes, after each, how many
 * leading bytes of the row are final.  Open addressing with backward-shift
 * deletion; the live count lets every other fill skip the lock. */
struct fold_res;
typedef struct {
    pthread_mutex_t mu;
    size_t prog[MAX_STORAGE_TARGETS];
    int redo; /* a published prefix was replaced (read error: zeros): fold it all again */
    int err;  /* first range-fold launch error */
    /* the window's fold: whoever completes a range launches it (range_claim) */
    struct fold_res *R;
    bcp_xor_hook_fn hook;
    void *hook_ctx;
    const uint8_t *rows;
    size_t pitch, nbytes, lo; /* lo: bytes folded or claimed */
    const size_t *valid;
    uint8_t *out;
    size_t step; /* smallest range folded before the window is complete */
    int n;
    int remote, st, tag; /* ranges go to the node fold server (connection of lane `tag`) */
} row_watch;

#define WATCH_SLOTS 4096u
#define WATCH_PIECE ((size_t)256 << 10) /* bytes a source reads between publishes */

/* experiment knob BCP_PIPE_PIECE (bytes, >= 64 KiB): the piece size */
static size_t watch_piece(void)
{
    static size_t piece;
    size_t p = __atomic_load_n(&piece, __ATOMIC_RELAXED);
    if (!p) {
        const char *v = getenv("BCP_PIPE_PIECE");
        p = v ? (size_t)strtoull(v, NULL, 0) : WATCH_PIECE;
        p = p < ((size_t)64 << 10) ? WATCH_PIECE : p;
        __atomic_store_n(&piece, p, __ATOMIC_RELAXED);
    }
    return p;
}
typedef struct {
    const void *row;
    row_watch *w;
    int j;
} watch_slot;
static watch_slot g_watch[WATCH_SLOTS];
static pthread_mutex_t g_watch_lock = PTHREAD_MUTEX_INITIALIZER;
static size_t g_watch_live;

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

static row_watch *watch_find(const void *row, int *j)
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

static void range_claim(row_watch *w);

/* A source's new final prefix of row j; the range it completes is folded
 * by this thread (the lane of the P role may not get a CPU before the reads
 * end: a woken source runs on the CPU of the lane that posted its receive). */
static void watch_publish(row_watch *w, int j, size_t bytes, int redo)
{
    pthread_mutex_lock(&w->mu);
    if (bytes > w->prog[j])
        w->prog[j] = bytes;
    w->redo |= redo;
    range_claim(w);
    pthread_mutex_unlock(&w->mu);
}

int bcpi_row_watched(const void *row)
{
    int j = 0;
    return watch_find(row, &j) != NULL;
}

void bcpi_row_progress(const void *row, size_t bytes, int redo)
{
    int j = 0;
    row_watch *W = watch_find(row, &j);
    if (W)
        watch_publish(W, j, bytes, redo);
}

int bcp_task_set_device_map(const int *devices, int ntargets)
{
    if (ntargets < 0 || ntargets > MAX_STORAGE_TARGETS || (ntargets && !devices))
        return -EINVAL;
    pthread_mutex_lock(&g_lock);
    for (int i = 0; i < ntargets; i++)
        g_devmap[i] = devices[i];
    g_devmap_n = ntargets;
    pthread_mutex_unlock(&g_lock);
    return 0;
}

int bcp_task_set_fold_mode(int mode)
{
    if (mode != BCP_FOLD_ZERO_COPY && mode != BCP_FOLD_STAGED && mode != BCP_FOLD_BATCHED &&
        mode != BCP_FOLD_STREAMED && mode != BCP_FOLD_DEVICE_ROWS && mode != BCP_FOLD_PIPELINED)
        return -EINVAL;
    pthread_mutex_lock(&g_lock);
    int prev = g_fold_mode;
    g_fold_mode = mode;
    pthread_mutex_unlock(&g_lock);
    return prev;
}

int bcp_task_set_explicit_padding(int on)
{
    if (on != 0 && on != 1)
        return -EINVAL;
    return __atomic_exchange_n(&g_explicit_pad, on, __ATOMIC_ACQ_REL);
}

void bcp_task_set_xor_hook(bcp_xor_hook_fn fn, void *ctx)
{
    pthread_mutex_lock(&g_lock);
    g_hook = fn;
    g_hook_ctx = ctx;
    pthread_mutex_unlock(&g_lock);
}

int bcp_task_set_transport(const bcp_transport_ops *ops)
{
    if (ops && (!ops->send || !ops->recv || !ops->isend || !ops->irecv || !ops->wait || !ops->waitall))
        return -EINVAL;
    pthread_mutex_lock(&g_lock);
    if (ops)
        g_tp = *ops;
    g_tp_set = ops != NULL;
    pthread_mutex_unlock(&g_lock);
    return 0;
}

/* The transport of one task (a snapshot: stable for the task's duration). */
static bcp_transport_ops transport_now(void)
{
    pthread_mutex_lock(&g_lock);
    bcp_transport_ops t = g_tp_set ? g_tp : *bcp_lb_transport();
    pthread_mutex_unlock(&g_lock);
    return t;
}

/* ---- failure injection (tests) ------------------------------------------ */
#define NSITES 6
static int g_inj_after[NSITES], g_inj_count[NSITES];

static int site_index(int site)
{
    switch (site) {
    case BCP_INJECT_FOLD_RES: return 0;
    case BCP_INJECT_DRAIN_ROW: return 1;
    case BCP_INJECT_SEND_BUF: return 2;
    case BCP_INJECT_THREAD: return 3;
    case BCP_INJECT_READ: return 4;
    case BCP_INJECT_FOLD_SERVER: return 5;
    default: return -1;
    }
}

int bcp_task_inject_failure(int site, int after, int count)
{
    const int i = site_index(site);
    if (i < 0 || after < 0 || count < 0)
        return -EINVAL;
    pthread_mutex_lock(&g_lock);
    g_inj_after[i] = after;
    g_inj_count[i] = count;
    pthread_mutex_unlock(&g_lock);
    return 0;
}

int bcpi_inject_hit(int site)
{
    const int i = site_index(site);
    if (i < 0)
        return 0;
    int hit = 0;
    pthread_mutex_lock(&g_lock);
    if (g_inj_count[i] > 0) {
        if (g_inj_after[i] > 0)
            g_inj_after[i]--;
        else {
            g_inj_count[i]--;
            hit = 1;
        }
    }
    pthread_mutex_unlock(&g_lock);
    return hit;
}

static int engine_for_target(int st, bcp_engine **out, int *device)
{
    int ndev = 0;
    bcp_device_count(&ndev);
    if (ndev <= 0)
        return -ENODEV;
    int dev = st % ndev;
    pthread_mutex_lock(&g_lock);
    if (st < g_devmap_n)
        dev = g_devmap[st];
    if (dev < 0 || dev >= ndev || dev >= MAX_DEVICES) {
        pthread_mutex_unlock(&g_lock);
        return -ENODEV;
    }
    if (!g_engines[dev] && !g_engine_rc[dev])
        g_engine_rc[dev] = bcp_engine_create(dev, &g_engines[dev]);
    int rc = g_engine_rc[dev];
    *out = g_engines[dev];
    pthread_mutex_unlock(&g_lock);
    *device = dev;
    return rc;
}

/* ---- fold service (BCP_FOLD_BATCHED) --------------------------------------
 * One per device, flat combining: a P role appends its window (rows +
 * output, mapped host memory; row j's data bytes) and, if fewer than
 * max_inflight batches are on the device, becomes a leader -- it takes EVERY
 * pending window (its own included), folds them with one descriptor batch on
 * a free slot's queue, syncs once and completes them all; otherwise it
 * sleeps until a leader has completed its window, or leads a later batch
 * itself.  The batch size follows the load with no thread of its own: a lone
 * lane (the single rebuild lane) folds its window directly, and when every
 * slot is busy the windows that arrive meanwhile share the next launch.  Rows are read over PCIe for their data bytes only: a gen-mode
 * window is padded to the stripe's largest chunk, and the padding is zeros
 * the kernel supplies itself. */
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

typedef struct {
    bcp_engine *eng;
    int inflight;     /* batches on the device (leaders folding) */
    int max_inflight; /* concurrent batches, each on its own slot's queue */
    fold_slot slot[MAX_INFLIGHT];
    pthread_mutex_t mu;
    fold_job *head, *tail;
    uint64_t windows, launches;
} fold_svc;

static fold_svc *g_svc[MAX_DEVICES];
static uint64_t g_svc_windows, g_svc_launches; /* of services already shut down */
static int g_fold_inflight = 1;

int bcp_task_set_fold_inflight(int k)
{
    if (k < 1 || k > MAX_INFLIGHT)
        return -EINVAL;
    pthread_mutex_lock(&g_lock);
    const int prev = g_fold_inflight;
    g_fold_inflight = k;
    for (int d = 0; d < MAX_DEVICES; d++)
        if (g_svc[d]) {
            pthread_mutex_lock(&g_svc[d]->mu);
            g_svc[d]->max_inflight = k;
            pthread_mutex_unlock(&g_svc[d]->mu);
        }
    pthread_mutex_unlock(&g_lock);
    return prev;
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
            bcp_queue_destroy(S->slot[i].q);
        free(S->slot[i].st);
        free(S->slot[i].so);
    }
    pthread_mutex_destroy(&S->mu);
    free(S);
}

/* The service of device dev (made on first use; slot queues on first use). */
static int svc_get(int dev, bcp_engine *e, fold_svc **out)
{
    pthread_mutex_lock(&g_lock);
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
    pthread_mutex_unlock(&g_lock);
    *out = S;
    return rc;
}

/* Wakeups are targeted: a leader wakes exactly the lanes whose windows it
 * folded, and the lane at the head of the pending list to lead the next
 * batch -- not every waiting lane (up to 12 lanes x every rank) on every
 * completion. */
static int fold_batched(fold_svc *S, const uint8_t *rows, size_t pitch, const size_t *valid, size_t nbytes, int n,
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
        /* lead a batch: everything pending (this window, if no other leader
         * took it yet) on a free slot */
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
    pthread_mutex_lock(&g_lock);
    w = g_svc_windows;
    l = g_svc_launches;
    for (int d = 0; d < MAX_DEVICES; d++)
        if (g_svc[d]) {
            pthread_mutex_lock(&g_svc[d]->mu);
            w += g_svc[d]->windows;
            l += g_svc[d]->launches;
            pthread_mutex_unlock(&g_svc[d]->mu);
        }
    pthread_mutex_unlock(&g_lock);
    if (windows)
        *windows = w;
    if (launches)
        *launches = l;
    return 0;
}

/* ---- node fold server (rank processes; bcp_host.h) -------------------------
 * Rank processes that each start a HIP runtime put one context per rank on
 * the GPU (nine on one MI355X for config 5); the device's queues, not the
 * fold, then set the rate.  With the server, the P roles'
 * window rows and outputs live in the socket world's shared arena and every
 * fold goes to ONE process that holds the GPU: one thread per connection
 * reads a request (rows, pitch, data bytes per row, output), registers the
 * arena blocks it has not seen, and folds through the fold service above
 * (flat combining: windows of every rank share a launch); the reply carries
 * the fold's status.  A rank has several connections (lane tag modulo their
 * number), each used by one lane at a time, request then reply. */
#define FS_MAGIC 0x62636673u /* "bcfs" */
#define FS_MAX_CONN 64

typedef struct {
    uint32_t magic;
    int32_t n, st, pad;
    uint64_t rows, pitch, nbytes, out;
    uint64_t rows_base, rows_size, out_base, out_size;
} fs_req;

typedef struct {
    uint32_t magic;
    int32_t rc;
} fs_rep;

static int fs_io(int fd, void *buf, size_t n, int wr)
{
    uint8_t *p = buf;
    while (n) {
        ssize_t r = wr ? send(fd, p, n, MSG_NOSIGNAL) : read(fd, p, n); /* a closed peer: EPIPE, no SIGPIPE */
        if (r < 0 && errno == EINTR)
            continue;
        if (r <= 0)
            return r < 0 ? -errno : -EPIPE;
        p += r;
        n -= (size_t)r;
    }
    return 0;
}

/* rank side */
static struct {
    int fd;
    pthread_mutex_t mu;
} g_srv[FS_MAX_CONN];
static int g_srv_n;
static __thread int t_lane_tag;
static uint64_t g_remote_folds; /* windows folded by the server for this process */

uint64_t bcpi_foldsrv_folds(void)
{
    return __atomic_load_n(&g_remote_folds, __ATOMIC_RELAXED);
}

int bcp_fold_server_stats(uint64_t *windows)
{
    if (!windows)
        return -EINVAL;
    *windows = bcpi_foldsrv_folds();
    return 0;
}

static bcp_xor_hook_fn g_srv_hook; /* the test double the server inherited */

void bcpi_foldsrv_attach(int nconn, const int *fds)
{
    pthread_mutex_lock(&g_lock);
    g_srv_hook = g_hook; /* the server was forked from the same state */
    pthread_mutex_unlock(&g_lock);
    g_srv_n = 0;
    for (int i = 0; i < nconn && i < FS_MAX_CONN; i++) {
        g_srv[i].fd = fds[i];
        pthread_mutex_init(&g_srv[i].mu, NULL);
        g_srv_n++;
    }
}

/* The fold of one window by the node fold server (rows and out in the
 * arena); -ENXIO if they are not, so the caller folds elsewhere. */
#define FS_HOOK 1  /* the server folds with the test double it inherited (CPU tests; whole rows) */
#define FS_RANGE 2 /* a range of a pipelined window: no reply; a failure is kept for FS_FINAL */
#define FS_FINAL 4 /* the window's last request: its reply carries the ranges' first failure */

static int fold_remote(int st, int tag, const uint8_t *rows, size_t pitch, const size_t *valid, size_t nbytes, int n,
                       uint8_t *out, int flags)
{
    fs_req q = {FS_MAGIC, n, st, flags, (uint64_t)(uintptr_t)rows, pitch, nbytes, (uint64_t)(uintptr_t)out,
                0, 0, 0, 0};
    void *rb, *ob;
    size_t rs, os;
    if (n < 1 || n > MAX_STORAGE_TARGETS || !bcpi_arena_block(rows, &rb, &rs) || !bcpi_arena_block(out, &ob, &os))
        return -ENXIO;
    q.rows_base = (uint64_t)(uintptr_t)rb;
    q.rows_size = rs;
    q.out_base = (uint64_t)(uintptr_t)ob;
    q.out_size = os;
    uint64_t v[MAX_STORAGE_TARGETS];
    for (int j = 0; j < n; j++)
        v[j] = valid[j];
    /* the lane's own connection: a pipelined window's ranges (sent by
     * whichever thread reads a source's progress) and its final request go
     * down the same one, and the server handles a connection in order */
    const int c = (tag < 0 ? -tag : tag) % g_srv_n;
    fs_rep r = {FS_MAGIC, 0};
    pthread_mutex_lock(&g_srv[c].mu);
    int rc = fs_io(g_srv[c].fd, &q, sizeof(q), 1);
    if (!rc)
        rc = fs_io(g_srv[c].fd, v, (size_t)n * sizeof(uint64_t), 1);
    if (!rc && !(flags & FS_RANGE))
        rc = fs_io(g_srv[c].fd, &r, sizeof(r), 0);
    pthread_mutex_unlock(&g_srv[c].mu);
    if (!rc && r.magic != FS_MAGIC)
        rc = -EPROTO;
    if (!rc && !r.rc)
        __atomic_fetch_add(&g_remote_folds, 1, __ATOMIC_RELAXED);
    return rc ? rc : r.rc;
}

/* server side */
static struct {
    pthread_mutex_t mu;
    struct {
        uint8_t *p;
        size_t n;
    } reg[4096];
    int nreg;
} g_fs = {.mu = PTHREAD_MUTEX_INITIALIZER};

/* A client's arena as this server sees it: the rank pool's is mapped at
 * the same address in every process (delta 0); a connected client's memfd
 * (bcp_fold_server_connect) is mapped here at base, its own at client_base. */
typedef struct fs_map {
    struct fs_map *next;
    uint64_t token, client_base;
    uint8_t *base;
    size_t size;
    int refs;
} fs_map;
static fs_map *g_fs_maps; /* under g_fs.mu */

typedef struct {
    int fd;
    uint64_t lo, hi; /* client addresses a request may name */
    int64_t delta;   /* server address = client address + delta */
    fs_map *map;     /* NULL: the rank pool's inherited arena */
} fs_conn;

static int fs_block_ok(const fs_conn *c, uint64_t base, uint64_t size, uint64_t p, uint64_t len)
{
    return size > 0 && base >= c->lo && base <= c->hi && size <= c->hi - base && p >= base && p <= base + size &&
           len <= base + size - p;
}

/* Register an arena block with the device once (blocks are reused at the
 * same place and size, so a registration stays valid while its mapping
 * lives). */
static int fs_register(bcp_engine *e, uint64_t base, uint64_t size)
{
    int rc = 0;
    pthread_mutex_lock(&g_fs.mu);
    int i = 0;
    for (; i < g_fs.nreg; i++)
        if ((uint64_t)(uintptr_t)g_fs.reg[i].p == base && g_fs.reg[i].n == size)
            break;
    if (i == g_fs.nreg) {
        if (g_fs.nreg == (int)(sizeof(g_fs.reg) / sizeof(g_fs.reg[0])))
            rc = -ENOSPC;
        else if (!(rc = bcp_host_register(e, (void *)(uintptr_t)base, (size_t)size))) {
            g_fs.reg[g_fs.nreg].p = (uint8_t *)(uintptr_t)base;
            g_fs.reg[g_fs.nreg].n = (size_t)size;
            g_fs.nreg++;
        }
    }
    pthread_mutex_unlock(&g_fs.mu);
    return rc;
}

/* The last connection of a client is gone: unregister its blocks, unmap. */
static void fs_map_put(fs_map *m)
{
    if (!m)
        return;
    pthread_mutex_lock(&g_fs.mu);
    if (--m->refs > 0) {
        pthread_mutex_unlock(&g_fs.mu);
        return;
    }
    for (fs_map **pp = &g_fs_maps; *pp; pp = &(*pp)->next)
        if (*pp == m) {
            *pp = m->next;
            break;
        }
    for (int i = 0; i < g_fs.nreg;)
        if (g_fs.reg[i].p >= m->base && g_fs.reg[i].p < m->base + m->size) {
            bcp_engine *e = NULL;
            pthread_mutex_lock(&g_lock);
            for (int d = 0; d < MAX_DEVICES && !e; d++)
                e = g_engines[d];
            pthread_mutex_unlock(&g_lock);
            if (e)
                (void)bcp_host_unregister(e, g_fs.reg[i].p);
            g_fs.reg[i] = g_fs.reg[--g_fs.nreg];
        } else {
            i++;
        }
    pthread_mutex_unlock(&g_fs.mu);
    munmap(m->base, m->size);
    free(m);
}

static void fs_serve_conn(fs_conn *c)
{
    const int fd = c->fd;
    int range_err = 0; /* first failed FS_RANGE fold since the last FS_FINAL */
    for (;;) {
        fs_req q;
        if (fs_io(fd, &q, sizeof(q), 0))
            break; /* the rank closed its end */
        uint64_t v[MAX_STORAGE_TARGETS];
        size_t valid[MAX_STORAGE_TARGETS];
        fs_rep r = {FS_MAGIC, 0};
        if (q.magic != FS_MAGIC || q.n < 1 || q.n > MAX_STORAGE_TARGETS)
            break; /* out of step: drop the connection (the rank sees EPIPE) */
        if (fs_io(fd, v, (size_t)q.n * sizeof(uint64_t), 0))
            break;
        if (bcpi_inject_hit(BCP_INJECT_FOLD_SERVER))
            break; /* (failure injection) the rank's fold sees EPIPE */
        int ok = fs_block_ok(c, q.out_base, q.out_size, q.out, q.nbytes) && q.pitch > 0 && q.nbytes <= q.pitch;
        for (int j = 0; j < q.n && ok; j++) {
            valid[j] = (size_t)v[j];
            ok = v[j] <= q.pitch && fs_block_ok(c, q.rows_base, q.rows_size, q.rows + (uint64_t)j * q.pitch,
                                                (q.pad & FS_HOOK) ? q.nbytes : v[j]);
        }
        /* client addresses -> this process's */
        q.rows += (uint64_t)c->delta;
        q.out += (uint64_t)c->delta;
        q.rows_base += (uint64_t)c->delta;
        q.out_base += (uint64_t)c->delta;
        bcp_engine *e = NULL;
        fold_svc *S = NULL;
        int dev = -1;
        bcp_xor_hook_fn hook = NULL;
        void *hctx = NULL;
        if (q.pad & FS_HOOK) {
            pthread_mutex_lock(&g_lock);
            hook = g_hook;
            hctx = g_hook_ctx;
            pthread_mutex_unlock(&g_lock);
        }
        if (!ok)
            r.rc = -EFAULT;
        else if (q.nbytes == 0)
            r.rc = 0; /* a final request with nothing left to fold */
        else if (q.pad & FS_HOOK)
            r.rc = hook ? hook((uint8_t *)(uintptr_t)q.out, (size_t)q.nbytes, (const uint8_t *)(uintptr_t)q.rows,
                               (size_t)q.pitch, q.n, hctx)
                        : -ENOSYS;
        else if (!(r.rc = engine_for_target(q.st, &e, &dev)) && !(r.rc = fs_register(e, q.rows_base, q.rows_size)) &&
                 !(r.rc = fs_register(e, q.out_base, q.out_size)) && !(r.rc = svc_get(dev, e, &S)))
            r.rc = fold_batched(S, (const uint8_t *)(uintptr_t)q.rows, (size_t)q.pitch, valid, (size_t)q.nbytes,
                                q.n, (uint8_t *)(uintptr_t)q.out);
        if (q.pad & FS_RANGE) {
            if (r.rc && !range_err)
                range_err = r.rc;
            continue; /* folded (synchronously, in order) -- no reply */
        }
        if (q.pad & FS_FINAL) {
            if (!r.rc)
                r.rc = range_err;
            range_err = 0;
        }
        if (fs_io(fd, &r, sizeof(r), 1))
            break;
    }
    close(fd);
}

static void *fs_conn_main(void *arg)
{
    fs_conn *c = arg;
    fs_serve_conn(c);
    free(c);
    return NULL;
}

int bcpi_foldsrv_main(int nconn, const int *fds, void *arena_lo, void *arena_hi)
{
    /* batches in flight at once (the fold service's width; every rank's
     * windows share it): environment BCP_FOLD_SERVER_INFLIGHT */
    if (getenv("BCP_FOLD_SERVER_INFLIGHT"))
        (void)bcp_task_set_fold_inflight(atoi(getenv("BCP_FOLD_SERVER_INFLIGHT")));
    pthread_t th[FS_MAX_CONN * MAX_STORAGE_TARGETS];
    int started = 0;
    for (int i = 0; i < nconn && i < (int)(sizeof(th) / sizeof(th[0])); i++) {
        fs_conn *c = calloc(1, sizeof(*c));
        if (c) {
            c->fd = fds[i];
            c->lo = (uint64_t)(uintptr_t)arena_lo;
            c->hi = (uint64_t)(uintptr_t)arena_hi;
        }
        if (c && pthread_create(&th[started], NULL, fs_conn_main, c) == 0) {
            started++;
        } else {
            free(c);
            close(fds[i]); /* the rank's lanes on it see EPIPE */
        }
    }
    for (int i = 0; i < started; i++)
        pthread_join(th[i], NULL);
    /* registrations end with the process; the fold service and engines go */
    return bcp_task_shutdown();
}

/* ---- the node fold server for independent processes (an MPI job) -------
 * bcp_fold_server_serve: a node's fold server on a Unix socket; a rank
 * (bcp_fold_server_connect) sends, on each of its connections, a hello
 * {magic, token, arena address, size} with its arena's memfd (SCM_RIGHTS);
 * the server maps each client's arena once and translates its addresses. */
#define FS_HELLO 0x62636668u /* "bcfh" */
typedef struct {
    uint32_t magic, pad;
    uint64_t token, base, size;
} fs_hello;

static int fs_recv_hello(int fd, fs_hello *h, int *memfd)
{
    char cbuf[CMSG_SPACE(sizeof(int))];
    struct iovec iov = {h, sizeof(*h)};
    struct msghdr mh = {0};
    mh.msg_iov = &iov;
    mh.msg_iovlen = 1;
    mh.msg_control = cbuf;
    mh.msg_controllen = sizeof(cbuf);
    *memfd = -1;
    ssize_t r;
    while ((r = recvmsg(fd, &mh, MSG_CMSG_CLOEXEC)) < 0 && errno == EINTR)
        ;
    if (r != (ssize_t)sizeof(*h) || h->magic != FS_HELLO)
        return -EPROTO;
    for (struct cmsghdr *cm = CMSG_FIRSTHDR(&mh); cm; cm = CMSG_NXTHDR(&mh, cm))
        if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_RIGHTS)
            memcpy(memfd, CMSG_DATA(cm), sizeof(int));
    return *memfd >= 0 ? 0 : -EPROTO;
}

static void *fs_accepted_main(void *arg)
{
    fs_conn *c = arg;
    fs_hello h;
    int memfd = -1;
    fs_map *m = NULL;
    if (!fs_recv_hello(c->fd, &h, &memfd) && h.size > 0) {
        pthread_mutex_lock(&g_fs.mu);
        for (m = g_fs_maps; m && m->token != h.token; m = m->next)
            ;
        if (!m && (m = calloc(1, sizeof(*m)))) {
            void *b = mmap(NULL, (size_t)h.size, PROT_READ | PROT_WRITE, MAP_SHARED, memfd, 0);
            if (b == MAP_FAILED) {
                free(m);
                m = NULL;
            } else {
                m->token = h.token;
                m->client_base = h.base;
                m->base = b;
                m->size = (size_t)h.size;
                m->next = g_fs_maps;
                g_fs_maps = m;
            }
        }
        if (m)
            m->refs++;
        pthread_mutex_unlock(&g_fs.mu);
    }
    if (memfd >= 0)
        close(memfd);
    if (m) {
        c->map = m;
        c->lo = m->client_base;
        c->hi = m->client_base + m->size;
        c->delta = (int64_t)((uint64_t)(uintptr_t)m->base - m->client_base);
        fs_serve_conn(c);
        fs_map_put(m);
    } else {
        close(c->fd);
    }
    free(c);
    return NULL;
}

int bcp_fold_server_serve(const char *socket_path, int max_conns)
{
    if (!socket_path || strlen(socket_path) >= sizeof(((struct sockaddr_un *)0)->sun_path) || max_conns < 0)
        return -EINVAL;
    if (getenv("BCP_FOLD_SERVER_INFLIGHT"))
        (void)bcp_task_set_fold_inflight(atoi(getenv("BCP_FOLD_SERVER_INFLIGHT")));
    const int ls = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (ls < 0)
        return -errno;
    struct sockaddr_un a = {0};
    a.sun_family = AF_UNIX;
    strcpy(a.sun_path, socket_path);
    unlink(socket_path);
    if (bind(ls, (struct sockaddr *)&a, sizeof(a)) != 0 || listen(ls, 256) != 0) {
        const int e = -errno;
        close(ls);
        return e;
    }
    pthread_t *th = calloc(max_conns ? (size_t)max_conns : 1, sizeof(pthread_t));
    int n = 0, rc = th ? 0 : -ENOMEM;
    while (!rc && (max_conns == 0 || n < max_conns)) {
        const int fd = accept4(ls, NULL, NULL, SOCK_CLOEXEC);
        if (fd < 0) {
            if (errno == EINTR)
                continue;
            rc = -errno;
            break;
        }
        fs_conn *c = calloc(1, sizeof(*c));
        pthread_t t;
        if (!c || pthread_create(max_conns ? &th[n] : &t, NULL, fs_accepted_main, c ? (c->fd = fd, c) : NULL) != 0) {
            free(c);
            close(fd);
            continue;
        }
        if (!max_conns)
            pthread_detach(t);
        n++;
    }
    close(ls);
    unlink(socket_path);
    for (int i = 0; max_conns && i < n; i++) /* (serving forever: never here) */
        pthread_join(th[i], NULL);
    free(th);
    const int src = bcp_task_shutdown();
    return rc ? rc : src;
}

int bcp_fold_server_connect(const char *socket_path, size_t arena_bytes, int nconn)
{
    if (!socket_path || strlen(socket_path) >= sizeof(((struct sockaddr_un *)0)->sun_path) || nconn < 1 ||
        nconn > FS_MAX_CONN || arena_bytes < ((size_t)2 << 20) || g_srv_n > 0)
        return -EINVAL;
    arena_bytes = arena_bytes / ((size_t)2 << 20) * ((size_t)2 << 20);
    const int mfd = memfd_create("bcp-fold-rows", MFD_CLOEXEC);
    if (mfd < 0)
        return -errno;
    int rc = ftruncate(mfd, (off_t)arena_bytes) ? -errno : 0;
    void *base = rc ? MAP_FAILED : mmap(NULL, arena_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, mfd, 0);
    if (!rc && base == MAP_FAILED)
        rc = -errno;
    int fds[FS_MAX_CONN];
    int made = 0;
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    const fs_hello h = {FS_HELLO, 0, ((uint64_t)getpid() << 32) ^ (uint64_t)ts.tv_nsec,
                        (uint64_t)(uintptr_t)base, arena_bytes};
    for (; !rc && made < nconn; made++) {
        const int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
        struct sockaddr_un a = {0};
        a.sun_family = AF_UNIX;
        strcpy(a.sun_path, socket_path);
        int crc = fd < 0 ? -errno : 0;
        /* a server still starting (socket file missing, or bound but not
         * yet listening): retry for up to ~2 s */
        for (int t = 0; !crc && connect(fd, (struct sockaddr *)&a, sizeof(a)) != 0; t++) {
            if ((errno != ECONNREFUSED && errno != ENOENT && errno != EAGAIN) || t >= 200) {
                crc = -errno;
                break;
            }
            usleep(10000);
        }
        if (crc) {
            rc = crc;
            if (fd >= 0)
                close(fd);
            break;
        }
        char cbuf[CMSG_SPACE(sizeof(int))];
        memset(cbuf, 0, sizeof(cbuf));
        struct iovec iov = {(void *)&h, sizeof(h)};
        struct msghdr mh = {0};
        mh.msg_iov = &iov;
        mh.msg_iovlen = 1;
        mh.msg_control = cbuf;
        mh.msg_controllen = sizeof(cbuf);
        struct cmsghdr *cm = CMSG_FIRSTHDR(&mh);
        cm->cmsg_level = SOL_SOCKET;
        cm->cmsg_type = SCM_RIGHTS;
        cm->cmsg_len = CMSG_LEN(sizeof(int));
        memcpy(CMSG_DATA(cm), &mfd, sizeof(int));
        if (sendmsg(fd, &mh, MSG_NOSIGNAL) != (ssize_t)sizeof(h)) {
            rc = -errno;
            close(fd);
            break;
        }
        fds[made] = fd;
    }
    close(mfd); /* the mapping and the server's copies keep the memory */
    if (rc) {
        for (int i = 0; i < made; i++)
            close(fds[i]);
        if (base != MAP_FAILED)
            munmap(base, arena_bytes);
        return rc;
    }
    bcpi_arena_set(base, arena_bytes); /* this process's P-role rows and outputs come from it */
    bcpi_foldsrv_attach(made, fds); /* (a test double set now is asked of the server too: FS_HOOK) */
    return 0;
}

/* ---- fold resources: a shared pool, reused across tasks, lanes and runs --
 * One resource = pinned, device-mapped window rows + output block (+ a HIP
 * queue and device buffers for the per-lane fold modes, made on first use).
 * The P role takes one for the duration of a task and gives it back, so a
 * long-running rank pays page pinning once, not per task or per lane thread.
 * Host-only resources (test hook) use plain memory. */
typedef struct fold_res {
    struct fold_res *next;
    int device;         /* -1: host-only (hook) */
    bcp_engine *eng;
    bcp_queue *q;       /* per-lane fold modes only */
    uint8_t *h_win[2];  /* window rows [n][pitch] (pinned + mapped when device >= 0) */
    int rows_dev;       /* h_win are device memory the host writes (DEVICE_ROWS) */
    uint8_t *h_par;     /* fold output */
    size_t h_cap, h_cap1, hp_cap;
    void *d_src, *d_out;
    size_t d_cap, dout_cap;
} fold_res;

static fold_res *g_pool = NULL; /* free list, under g_lock */

typedef struct {
    uint8_t *send_buf;  /* chunk_sender window buffer */
    size_t send_cap;
} lane_res;

static __thread lane_res t_res;

static void host_free(fold_res *R, void *p)
{
    if (!p)
        return;
    if (bcpi_arena_free(p)) { /* a row block of the socket world's shared arena */
        if (R->device >= 0)
            (void)bcp_host_unregister(R->eng, p);
        return;
    }
    if (R->device >= 0)
        bcp_host_free(R->eng, p);
    else
        free(p);
}

static void rows_free(fold_res *R, void *p)
{
    if (p && R->rows_dev)
        bcp_dev_free(R->eng, p);
    else
        host_free(R, p);
}

static void res_destroy(fold_res *R)
{
    rows_free(R, R->h_win[0]);
    rows_free(R, R->h_win[1]);
    host_free(R, R->h_par);
    if (R->device >= 0) {
        if (R->d_src)
            bcp_dev_free(R->eng, R->d_src);
        if (R->d_out)
            bcp_dev_free(R->eng, R->d_out);
        if (R->q)
            bcp_queue_destroy(R->q);
    }
    free(R);
}

void bcp_task_thread_release(void)
{
    free(t_res.send_buf);
    t_res.send_buf = NULL;
    t_res.send_cap = 0;
}

int bcp_task_shutdown(void)
{
    bcp_task_thread_release();
    /* fold services first: they hold queues on the engines (all lanes have
     * returned, so no batch is in flight) */
    pthread_mutex_lock(&g_lock);
    for (int d = 0; d < MAX_DEVICES; d++) {
        fold_svc *S = g_svc[d];
        g_svc[d] = NULL;
        if (!S)
            continue;
        g_svc_windows += S->windows;
        g_svc_launches += S->launches;
        svc_destroy(S);
    }
    pthread_mutex_unlock(&g_lock);
    pthread_mutex_lock(&g_lock);
    fold_res *R = g_pool;
    g_pool = NULL;
    pthread_mutex_unlock(&g_lock);
    while (R) {
        fold_res *nx = R->next;
        res_destroy(R);
        R = nx;
    }
    pthread_mutex_lock(&g_lock);
    for (int d = 0; d < MAX_DEVICES; d++) {
        if (g_engines[d])
            bcp_engine_destroy(g_engines[d]);
        g_engines[d] = NULL;
        g_engine_rc[d] = 0;
    }
    pthread_mutex_unlock(&g_lock);
    return 0;
}

static void res_release(fold_res *R)
{
    if (!R)
        return;
    pthread_mutex_lock(&g_lock);
    R->next = g_pool;
    g_pool = R;
    pthread_mutex_unlock(&g_lock);
}

/* kind: 0 host (pinned + mapped on a GPU resource), 1 device memory the
 * host writes (window rows under DEVICE_ROWS), 2 host window rows: from
 * this rank's slice of the socket world's shared arena when there is one
 * (other rank processes' sources then read their chunks straight into them,
 * bcp_sock.c), registered with the GPU; else as 0 */
static int grow(fold_res *R, uint8_t **p, size_t *cap, size_t need, int kind)
{
    if (*cap >= need && *p)
        return 0;
    if (kind == 1)
        bcp_dev_free(R->eng, *p);
    else
        host_free(R, *p);
    *p = NULL;
    *cap = 0;
    /* next power of two (>= 1 MiB): a worklist sorted by size (gen/main.c:
     * 703-715) would otherwise re-pin rows at nearly every task */
    size_t c = (size_t)1 << 20;
    while (c < need)
        c <<= 1;
    int rc = 0;
    if (kind == 2 && (*p = bcpi_arena_alloc(c, &c))) {
        if (R->device < 0 || !bcp_host_register(R->eng, *p, c)) {
            *cap = c;
            return 0;
        }
        bcpi_arena_free(*p); /* not addressable by the device: ordinary rows */
        *p = NULL;
        c = (size_t)1 << 20;
        while (c < need)
            c <<= 1;
    }
    if (kind == 1)
        rc = bcp_dev_alloc_hostwrite(R->eng, c, (void **)p);
    else if (R->device >= 0)
        rc = bcp_host_alloc_mapped(R->eng, c, (void **)p);
    else if (!(*p = malloc(c)))
        rc = -ENOMEM;
    if (!rc)
        *cap = c;
    return rc;
}

static int grow_dev(fold_res *R, void **p, size_t *cap, size_t need)
{
    if (*cap >= need && *p)
        return 0;
    if (*p)
        bcp_dev_free(R->eng, *p);
    *p = NULL;
    *cap = 0;
    size_t c = MAX_(need, (size_t)1 << 20);
    int rc = bcp_dev_alloc(R->eng, c, p);
    if (!rc)
        *cap = c;
    return rc;
}

/* Take a resource for storage target st with room for rows_bytes of window
 * rows (twice when `windows` > 1: the next window is received while one is
 * folded; a single-window task needs one set) and an nbytes fold output.
 * use_gpu = 0 under the test hook; dev_rows: rows in device memory the host
 * writes (DEVICE_ROWS). */
static int res_acquire(HostState *hs, int use_gpu, int dev_rows, size_t rows_bytes, size_t nbytes, uint64_t windows,
                       fold_res **out)
{
    int rc = 0, dev = -1;
    bcp_engine *e = NULL;
    *out = NULL;
    if (bcpi_inject_hit(BCP_INJECT_FOLD_RES))
        return -ENOMEM;
    if (use_gpu && (rc = engine_for_target(hs->storage_target, &e, &dev)))
        return rc;
    /* prefer a free resource of the same device that is already big enough */
    pthread_mutex_lock(&g_lock);
    fold_res **best = NULL;
    for (fold_res **pp = &g_pool; *pp; pp = &(*pp)->next) {
        if ((*pp)->device != dev)
            continue;
        if (!best || ((*best)->rows_dev != dev_rows && (*pp)->rows_dev == dev_rows))
            best = pp;
        if ((*pp)->rows_dev == dev_rows && (*pp)->h_cap >= rows_bytes && ((*pp)->h_cap1 >= rows_bytes || windows < 2) && (*pp)->hp_cap >= nbytes) {
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
    pthread_mutex_unlock(&g_lock);
    if (!R) {
        R = calloc(1, sizeof(*R));
        if (!R)
            return -ENOMEM;
        R->device = dev;
        R->eng = e;
    }
    if (R->rows_dev != dev_rows) { /* rows of the other kind: drop them */
        rows_free(R, R->h_win[0]);
        rows_free(R, R->h_win[1]);
        R->h_win[0] = R->h_win[1] = NULL;
        R->h_cap = R->h_cap1 = 0;
        R->rows_dev = dev_rows;
    }
    const int row_kind = dev_rows ? 1 : 2;
    if ((rc = grow(R, &R->h_win[0], &R->h_cap, rows_bytes, row_kind)) ||
        (windows > 1 && (rc = grow(R, &R->h_win[1], &R->h_cap1, rows_bytes, row_kind))) ||
        (rc = grow(R, &R->h_par, &R->hp_cap, nbytes, dev < 0 && g_srv_n > 0 ? 2 : 0)))
        goto fail; /* (with a node fold server the output is an arena block too) */
    *out = R;
    return 0;
fail:
    res_destroy(R);
    return rc;
}

/* The fold of one window (replaces xor_parity at task_processing.c:211):
 * out = XOR of n rows of `pitch` bytes, nbytes each. */
static int fold_window(fold_res *R, HostState *hs, int mode, bcp_xor_hook_fn hook, void *ctx, const uint8_t *rows,
                       size_t pitch, const size_t *valid, size_t nbytes, int n, uint8_t *out)
{
    void *ab;
    size_t az;
    /* the node fold server folds (with a test double only if it has the
     * same one: it was forked when the pool was made) */
    if (R->device < 0 && g_srv_n > 0 && (!hook || hook == g_srv_hook) && bcpi_arena_block(rows, &ab, &az))
        return fold_remote(hs->storage_target, t_lane_tag, rows, pitch, valid, nbytes, n, out, hook ? FS_HOOK : 0);
    if (hook) {
        static int warned = 0; /* lanes race here: atomic exchange */
        if (!__atomic_exchange_n(&warned, 1, __ATOMIC_RELAXED))
            LOGERR("XOR test hook active on st %d (no GPU fold)\n", hs->storage_target);
        return hook(out, nbytes, rows, pitch, n, ctx);
    }
    int rc;
    if (mode == BCP_FOLD_BATCHED || mode == BCP_FOLD_DEVICE_ROWS || mode == BCP_FOLD_PIPELINED) {
        /* DEVICE_ROWS: the rows were stored through the BAR by other threads
         * (write-combined); their hand-over to this one passed locked
         * instructions, and this fence drains this thread's own (a socket
         * receive copies into the rows on this thread) before the launch */
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        fold_svc *S = NULL;
        if ((rc = svc_get(R->device, R->eng, &S)))
            return rc;
        return fold_batched(S, rows, pitch, valid, nbytes, n, out);
    }
    if (!R->q && (rc = bcp_queue_create(R->eng, &R->q)))
        return rc;
    if (mode == BCP_FOLD_ZERO_COPY) {
        /* rows and out are mapped pinned memory (grow): the kernel streams
         * row j's data bytes (valid[j]) over PCIe, no copy commands; the
         * zeros past them are the kernel's */
        bcp_stripe st = {(uint64_t)(uintptr_t)out, nbytes, 0, (uint32_t)n, 0};
        bcp_source so[MAX_STORAGE_TARGETS];
        for (int j = 0; j < n; j++)
            so[j] = (bcp_source){(uint64_t)(uintptr_t)(rows + (size_t)j * pitch), valid[j]};
        if ((rc = bcp_xor_stripes_async(R->q, &st, 1, so, (uint32_t)n)))
            return rc;
        return bcp_queue_sync(R->q);
    }
    if ((rc = grow_dev(R, &R->d_src, &R->d_cap, pitch * (size_t)n)) || (rc = grow_dev(R, &R->d_out, &R->dout_cap, nbytes)))
        return rc;
    if ((rc = bcp_h2d_async(R->q, R->d_src, rows, pitch * (size_t)n)))
        return rc;
    if ((rc = bcp_xor_strided_async(R->q, R->d_out, pitch, R->d_src, pitch * (size_t)n, pitch, 1, (uint32_t)n,
                                    nbytes)))
        return rc;
    if ((rc = bcp_d2h_async(R->q, out, R->d_out, nbytes)))
        return rc;
    return bcp_queue_sync(R->q);
}

/* STREAMED mode, per window: wait for the rows in source order and, as each
 * arrives, copy its data bytes (valid[j]) to device row j on the lane's
 * queue -- the DMA of row j overlaps the senders still filling rows j+1...
 * Every posted request is waited for, whatever fails.  Returns the first
 * transport error in *trc and the first copy error as the result. */
static int stream_rows_in(const bcp_transport_ops *T, fold_res *R, void **req, int n, const uint8_t *rows,
                          size_t pitch, const size_t *valid, int *trc)
{
    int crc = 0;
    *trc = 0;
    for (int j = 0; j < n; j++) {
        int e = req[j] ? T->wait(T->ctx, req[j]) : 0;
        req[j] = NULL;
        if (e && !*trc)
            *trc = e;
        if (!e && !crc && valid[j])
            crc = bcp_h2d_async(R->q, (uint8_t *)R->d_src + (size_t)j * pitch, rows + (size_t)j * pitch, valid[j]);
    }
    return crc;
}

/* STREAMED mode: fold the device rows (row j = valid[j] data bytes, zero
 * padded to nbytes) into the pinned output block, then sync. */
static int stream_fold(fold_res *R, int n, size_t pitch, const size_t *valid, size_t nbytes, uint8_t *out)
{
    bcp_stripe st = {(uint64_t)(uintptr_t)out, nbytes, 0, (uint32_t)n, 0};
    bcp_source so[MAX_STORAGE_TARGETS];
    for (int j = 0; j < n; j++)
        so[j] = (bcp_source){(uint64_t)(uintptr_t)((uint8_t *)R->d_src + (size_t)j * pitch), valid[j]};
    int rc = bcp_xor_stripes_async(R->q, &st, 1, so, (uint32_t)n);
    return rc ? rc : bcp_queue_sync(R->q);
}

/* ---- PIPELINED mode --------------------------------------------------------
 * The window's rows are watched while the sources fill them: the fold of
 * every byte range that all rows have delivered (data bytes only, valid[j])
 * is launched on the lane's queue, without a sync, by the source whose
 * piece completed it, so most of the rows' PCIe reads overlap the sources'
 * file reads; after the receives the P role folds the rest (at least the
 * last piece) and syncs once.  Short kernels only: nothing on the device
 * waits for the host. */
#define PIPE_STEP ((size_t)128 << 10)   /* smallest range worth a launch (also >= a quarter window) */
#define PIPE_ALIGN ((size_t)4096)       /* range boundaries */

static uint64_t g_pipe_windows, g_pipe_ranges; /* bcp_task_pipe_stats */

int bcp_task_pipe_stats(uint64_t *windows, uint64_t *ranges)
{
    if (windows)
        *windows = __atomic_load_n(&g_pipe_windows, __ATOMIC_RELAXED);
    if (ranges)
        *ranges = __atomic_load_n(&g_pipe_ranges, __ATOMIC_RELAXED);
    return 0;
}

/* Fold out[lo, hi) = XOR of the rows' [lo, hi) on the lane's queue, no sync
 * (under the test hook: the hook, at once, over whole rows whose padding the
 * P role zeroed before the receives).  Callers hold w->mu: the queue is one
 * lane's, and launches on it must not interleave. */
static int launch_range(const row_watch *w, size_t lo, size_t hi)
{
    __atomic_fetch_add(&g_pipe_ranges, 1, __ATOMIC_RELAXED);
    if (w->hook)
        return w->hook(w->out + lo, hi - lo, w->rows + lo, w->pitch, w->n, w->hook_ctx);
    if (w->remote) { /* the node fold server folds the range; no reply (FS_RANGE) */
        size_t v[MAX_STORAGE_TARGETS];
        for (int j = 0; j < w->n; j++)
            v[j] = w->valid[j] > lo ? MIN_(w->valid[j], hi) - lo : 0;
        return fold_remote(w->st, w->tag, w->rows + lo, w->pitch, v, hi - lo, w->n, w->out + lo, FS_RANGE);
    }
    bcp_stripe st = {(uint64_t)(uintptr_t)(w->out + lo), hi - lo, 0, (uint32_t)w->n, 0};
    bcp_source so[MAX_STORAGE_TARGETS];
    for (int j = 0; j < w->n; j++) {
        const size_t len = w->valid[j] > lo ? MIN_(w->valid[j], hi) - lo : 0;
        so[j] = (bcp_source){(uint64_t)(uintptr_t)(w->rows + (size_t)j * w->pitch + lo), len};
    }
    return bcp_xor_stripes_async(w->R->q, &st, 1, so, (uint32_t)w->n);
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

static int watch_rows(row_watch *W, fold_res *R, bcp_xor_hook_fn hook, void *hook_ctx, const uint8_t *rows,
                      size_t pitch, const size_t *valid, int n, size_t nbytes, uint8_t *out, int remote, int st,
                      int tag)
{
    pthread_mutex_init(&W->mu, NULL);
    W->remote = remote;
    W->st = st;
    W->tag = tag;
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
    W->step = MAX_(PIPE_STEP, nbytes / 4); /* at most ~5 launches per window */
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

/* After the receives (every fill has returned, so no source launches any
 * more): unregister, fold the rest (all of it after a redo), the one sync
 * -- also after an error, since ranges may be in flight.  fold = 0: sync
 * only (the task failed).  (Writing the ranges folded so far while the last
 * one folds, behind an event the launching source records, measured slower
 * on every workload -- config 5 by a quarter, r2bh / r2bi -- and is gone.) */
static int finish_rows(row_watch *W, int fold)
{
    for (int j = 0; j < W->n; j++)
        watch_del(W->rows + (size_t)j * W->pitch);
    int rc = W->err;
    const size_t lo = W->redo ? 0 : W->lo;
    __atomic_fetch_add(&g_pipe_windows, 1, __ATOMIC_RELAXED);
    int src = 0;
    if (W->remote && !W->hook) {
        /* the tail (or nothing) as the final request: answered once the
         * server has folded every range sent before it on the connection */
        size_t v[MAX_STORAGE_TARGETS];
        const size_t a = fold && !rc ? lo : W->nbytes;
        for (int j = 0; j < W->n; j++)
            v[j] = W->valid[j] > a ? MIN_(W->valid[j], W->nbytes) - a : 0;
        if (a < W->nbytes)
            __atomic_fetch_add(&g_pipe_ranges, 1, __ATOMIC_RELAXED);
        src = fold_remote(W->st, W->tag, W->rows + (a < W->nbytes ? a : 0), W->pitch, v, W->nbytes - a, W->n,
                          W->out + (a < W->nbytes ? a : 0), FS_FINAL);
    } else {
        if (fold && !rc && lo < W->nbytes)
            rc = launch_range(W, lo, W->nbytes);
        src = W->hook ? 0 : bcp_queue_sync(W->R->q);
    }
    pthread_mutex_destroy(&W->mu);
    return rc ? rc : src;
}

/* ---- file helpers (task_processing.c:29-79) ----------------------------- */

/* mkdir -p for the directories of `filename` under wdir. */
static void mkdir_for_file(int wdir, const char *filename)
{
    size_t len = strlen(filename);
    char *tmp = malloc(len + 1);
    if (!tmp)
        return;
    memcpy(tmp, filename, len + 1);
    for (char *p = tmp + 1; *p; p++) {
        if (*p == '/') {
            *p = 0;
            mkdirat(wdir, tmp, S_IRWXU);
            *p = '/';
        }
    }
    free(tmp);
}

static int open_chunk_readonly(int rdir, const char *path)
{
    int fd = openat(rdir, path, O_RDONLY);
    if (fd > 0)
        posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
    return fd;
}

static int open_new_parity(int wdir, const char *path, off_t expected_size)
{
    mkdir_for_file(wdir, path);
    int fd = openat(wdir, path, O_CREAT | O_WRONLY | O_TRUNC, S_IRUSR | S_IWUSR);
    if (fd > 0 && expected_size > 0)
        posix_fallocate(fd, 0, expected_size);
    return fd;
}

/* Corrupt list entry (task_processing.c:54-60); written whole, one line. */
static void push_corrupt_path(HostState *hs, const char *path)
{
    size_t len = strlen(path);
    char *line = malloc(len + 2);
    if (!line)
        return;
    memcpy(line, path, len);
    line[len] = '\n';
    ssize_t w = write(hs->corrupt_files_fd, line, len + 1);
    (void)w;
    free(line);
}

static int active_ranks(uint64_t locations) { return __builtin_popcountll(locations & L_MASK); }

/* The sticky per-rank error (task_processing.c:232-236,313-317).  The lanes
 * of a rank share hs; the reference writes hs->error / error_path from them
 * without a lock (a data race).  Here the first error wins by
 * compare-and-swap and only the winner sets error_path.  Returns 1 if this
 * call raised it. */
static int raise_sticky_error(HostState *hs, int err, const char *path)
{
    int expected = 0;
    if (!__atomic_compare_exchange_n(&hs->error, &expected, err, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE))
        return 0;
    hs->error_path = strdup(path);
    return 1;
}

/* errno value for the sticky error from a negative library / transport code */
static int as_errno(int rc) { return rc < 0 ? -rc : (rc ? rc : EIO); }

/* ---- phase accounting (bcp_task_phase_stats) -----------------------------
 * Wall time per P-role phase summed over tasks (relaxed atomics: a few ns
 * per task), to see where a task's latency goes on a given box. */
static uint64_t g_phase_ns[BCP_PHASES];

static uint64_t mono_ns(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000u + (uint64_t)t.tv_nsec;
}

static void phase_add(int ph, uint64_t *t)
{
    const uint64_t now = mono_ns();
    __atomic_fetch_add(&g_phase_ns[ph], now - *t, __ATOMIC_RELAXED);
    *t = now;
}

int bcp_task_phase_stats(double *seconds, int nphases, int reset)
{
    if (nphases < 0 || (nphases && !seconds))
        return -EINVAL;
    for (int i = 0; i < BCP_PHASES; i++) {
        const uint64_t v = reset ? __atomic_exchange_n(&g_phase_ns[i], 0, __ATOMIC_RELAXED)
                                 : __atomic_load_n(&g_phase_ns[i], __ATOMIC_RELAXED);
        if (i < nphases)
            seconds[i] = i >= BCP_PHASE_P_TASKS ? (double)v : (double)v * 1e-9; /* counts, else ns -> s */
    }
    return BCP_PHASES;
}

/* ---- roles ------------------------------------------------------------- */

/* Post one receive per source (window row j at base + j * pitch).  Every
 * source gets its receive even if an earlier post failed (a live sender must
 * never be left blocked); a failed post leaves its slot NULL.  Returns the
 * first error. */
static int post_recvs(const bcp_transport_ops *T, void **req, int n, uint8_t *base, size_t pitch, size_t len,
                      const int *ranks, int tag)
{
    int first = 0;
    for (int j = 0; j < n; j++) {
        req[j] = NULL;
        int rc = T->irecv(T->ctx, base + (size_t)j * pitch, len, ranks[j], tag, &req[j]);
        if (rc) {
            req[j] = NULL;
            if (!first)
                first = rc;
        }
    }
    return first;
}

/* Wait for every request actually posted (never leave a receive pending on
 * a buffer that goes away); returns the first error. */
static int wait_posted(const bcp_transport_ops *T, void **req, int n)
{
    void *live[MAX_STORAGE_TARGETS];
    int m = 0;
    for (int j = 0; j < n; j++)
        if (req[j])
            live[m++] = req[j];
    for (int j = 0; j < n; j++)
        req[j] = NULL;
    return m ? T->waitall(T->ctx, m, live) : 0;
}

/* The P role without fold resources: every window of every source is still
 * received (the senders block until it is), source by source into ONE row
 * reused for all of them; without even that row, into a 16 KiB stack row
 * with truncating receives.  Nothing is folded or written. */
static int drain_windows(const bcp_transport_ops *T, const int *ranks, int n, size_t buffer_size,
                         uint64_t expected_messages, int tag)
{
    uint8_t small[DRAIN_SMALL];
    uint8_t *row = bcpi_inject_hit(BCP_INJECT_DRAIN_ROW) ? NULL : malloc(buffer_size ? buffer_size : 1);
    uint8_t *dst = row ? row : small;
    const size_t cap = row ? buffer_size : MIN_(buffer_size, (size_t)DRAIN_SMALL);
    int rc = 0;
    for (uint64_t w = 0; w < expected_messages; w++)
        for (int j = 0; j < n; j++) {
            int e = T->recv(T->ctx, dst, cap, ranks[j], tag);
            if (e && e != -EMSGSIZE && !rc)
                rc = e;
        }
    free(row);
    return rc;
}

/* Once per task: open the parity chunk (open: no sticky error) and write the
 * gen header, the chunk sizes (:199-201; hdr NULL when rebuilding), to it or
 * to the null device. */
static void open_parity_chunk(HostState *hs, const char *path, uint64_t final_size, int open, int *fd,
                              int *opened, int *have_had_error, const uint64_t *hdr, int n)
{
    if (*opened)
        return;
    *opened = 1;
    if (open) {
        const int f = open_new_parity(hs->write_dir, path, (off_t)final_size);
        if (f <= 0) {
            *have_had_error = errno;
            LOGERR("cannot open parity chunk '%s': %s\n", path, strerror(errno));
        } else {
            *fd = f;
        }
    }
    if (hdr && write(*fd, hdr, sizeof(uint64_t) * (size_t)n) <= 0)
        *have_had_error = errno;
}

static void parity_generator(const bcp_transport_ops *T, const char *path, const FileInfo *task, TaskInfo ti,
                             HostState *hs)
{
    const int n = active_ranks(task->locations);
    int ranks[MAX_STORAGE_TARGETS];
    for (int i = 0, j = 0; i < MAX_STORAGE_TARGETS; i++)
        if (TEST_BIT(task->locations, i))
            ranks[j++] = st2rank[i];

    /* nobody holds a chunk any more: the parity chunk goes too (:141-144) */
    if (n == 0) {
        unlinkat(hs->write_dir, path, 0);
        return;
    }

    void *req[MAX_STORAGE_TARGETS];
    uint64_t chunk_sizes[MAX_STORAGE_TARGETS] = {0};
    int have_had_error = 0, trc = 0;
    uint64_t tph = mono_ns();
    if (ti.is_rebuilding) {
        /* the parity holder forwards the stored header (:149-156) */
        trc = T->recv(T->ctx, chunk_sizes, (size_t)n * sizeof(uint64_t), st2rank[ti.actual_P_st], ti.tag);
    } else {
        trc = post_recvs(T, req, n, (uint8_t *)chunk_sizes, sizeof(uint64_t), sizeof(uint64_t), ranks, ti.tag);
        int w = wait_posted(T, req, n);
        trc = trc ? trc : w;
    }
    if (trc) {
        have_had_error = as_errno(trc);
        LOGERR("chunk sizes for '%s' not received: %s\n", path, strerror(have_had_error));
    }

    uint64_t max_cs = 0;
    for (int j = 0; j < n; j++)
        max_cs = MAX_(max_cs, chunk_sizes[j]);
    for (int j = 0; j < n; j++)
        req[j] = NULL;
    for (int j = 0; j < n; j++)
        if ((trc = T->isend(T->ctx, &max_cs, sizeof(max_cs), ranks[j], ti.tag, &req[j]))) {
            req[j] = NULL;
            break;
        }
    {
        int w = wait_posted(T, req, n);
        trc = trc ? trc : w;
    }
    if (trc && !have_had_error) {
        have_had_error = as_errno(trc);
        LOGERR("window size for '%s' not sent: %s\n", path, strerror(have_had_error));
    }

    phase_add(BCP_PHASE_P_SIZES, &tph);
    uint64_t final_parity_chunk_size = max_cs + (uint64_t)n * sizeof(uint64_t);
    if (ti.is_rebuilding) {
        /* index of this (rebuilt) target in the stored header (:169-174) */
        uint64_t loc = task->locations & ~(UINT64_C(1) << ti.actual_P_st) & L_MASK;
        uint64_t my_mask = (UINT64_C(1) << hs->storage_target) - 1;
        final_parity_chunk_size = chunk_sizes[active_ranks(loc & my_mask)];
    }

    const size_t buffer_size = (size_t)MIN_(WINDOW, max_cs);
    const size_t pitch = (buffer_size + ROW_ALIGN - 1) / ROW_ALIGN * ROW_ALIGN;
    const uint64_t final_size = max_cs + (uint64_t)n * 8u;
    const uint64_t expected_messages = (max_cs + WINDOW - 1) / WINDOW;
    uint64_t data_left = max_cs;

    pthread_mutex_lock(&g_lock);
    bcp_xor_hook_fn hook = g_hook;
    void *hook_ctx = g_hook_ctx;
    const int mode = g_fold_mode; /* one mode for the whole task */
    pthread_mutex_unlock(&g_lock);

    if (!have_had_error)
        have_had_error = __atomic_load_n(&hs->error, __ATOMIC_ACQUIRE);
    fold_res *L = NULL;
    /* (experiment knob BCP_HOOK_PINNED_ROWS: the test-hook fold over the same
     * pinned device-mapped rows the GPU folds use, to separate the memory
     * kind from the fold in tools/exp measurements) */
    const int pinned_rows = hook == NULL || getenv("BCP_HOOK_PINNED_ROWS") != NULL;
    const int dev_rows = hook == NULL && mode == BCP_FOLD_DEVICE_ROWS;
    /* a node fold server (rank processes) folds for the fold-service modes:
     * rows and output from the arena, no HIP runtime in this process */
    const int remote = g_srv_n > 0 && (hook != NULL || mode == BCP_FOLD_BATCHED || mode == BCP_FOLD_PIPELINED);
    t_lane_tag = ti.tag;
    int res_rc = expected_messages ? res_acquire(hs, remote ? 0 : pinned_rows, dev_rows, pitch * (size_t)n,
                                                 buffer_size, expected_messages, &L)
                                   : 0;
    if (remote && !res_rc && L) {
        void *b;
        size_t z;
        if (!bcpi_arena_block(L->h_win[0], &b, &z) || !bcpi_arena_block(L->h_par, &b, &z) ||
            (expected_messages > 1 && !bcpi_arena_block(L->h_win[1], &b, &z))) {
            /* the arena slice is full: fold in this process as without a server */
            res_release(L);
            L = NULL;
            res_rc = res_acquire(hs, pinned_rows, dev_rows, pitch * (size_t)n, buffer_size, expected_messages, &L);
        }
    }
    if (res_rc) {
        LOGERR("no fold resources for '%s' on st %d: %s\n", path, hs->storage_target, bcp_strerror(res_rc));
        if (!have_had_error)
            have_had_error = as_errno(res_rc);
    }

    /* The parity chunk is opened (and its gen header written) once the first
     * window's receives are posted, so the sources read their chunks while
     * this thread creates, truncates and allocates the file; the reference
     * opens it before its first receive (:183-206).  Same bytes, same errors. */
    int P_fd = hs->fd_null, opened = 0;
    const int open_parity = have_had_error == 0;
    /* (experiment knob BCP_TASK_SERIAL_IO: the reference's order, the open
     * before the first receive) */
    const int serial_io = getenv("BCP_TASK_SERIAL_IO") != NULL;
    if (!open_parity)
        LOGERR("'%s' goes to the null device: error %d is sticky on this rank\n", path, have_had_error);

    /* STREAMED: the lane's queue and device rows; row j's data bytes.  A
     * gen-mode single-window row holds chunk_sizes[j] bytes then the
     * sender's zero padding (chunk_sender reads a chunk up to the size it
     * reported); anything else (rebuild: the survivors' current sizes are
     * not sent; windows past the first: replay) is taken whole. */
    int streamed = mode == BCP_FOLD_STREAMED && !hook && !res_rc && expected_messages > 0;
    size_t valid[MAX_STORAGE_TARGETS];
    const int implicit_pad = !ti.is_rebuilding && expected_messages == 1; /* as chunk_sender decides */
    for (int j = 0; j < n; j++)
        valid[j] = implicit_pad ? (size_t)MIN_(chunk_sizes[j], (uint64_t)buffer_size) : buffer_size;
    if (streamed) {
        int src = L->q ? 0 : bcp_queue_create(L->eng, &L->q);
        if (!src)
            src = grow_dev(L, &L->d_src, &L->d_cap, pitch * (size_t)n);
        if (src) {
            LOGERR("no device rows for '%s' on st %d: %s\n", path, hs->storage_target, bcp_strerror(src));
            if (!have_had_error)
                have_had_error = as_errno(src);
            streamed = 0;
        }
    }

    /* folds that read whole rows (the test hook, STAGED) */
    const int pad_rows = implicit_pad && !res_rc && (hook != NULL || mode == BCP_FOLD_STAGED);
    /* PIPELINED: one window whose rows the sources fill directly (send_fill
     * transports); otherwise it folds like ZERO_COPY */
    /* (the sources publish their progress through this process's watch
     * table and launch range folds on this lane's queue: in-process ranks,
     * i.e. the loopback transport, only) */
    void *rb_;
    size_t rz_;
    /* rank processes: rows in the arena, folds by the node fold server; the
     * sources report their progress over the sockets (PROG frames).  Opt-in
     * (environment BCP_XPROC_PIPELINE=1): measured no faster than whole
     * windows through the server on config 1 / 5 and slower on the one-lane
     * rebuild (r2d0), so PIPELINED ranks fold their windows BATCHED */
    const char *xpe = getenv("BCP_XPROC_PIPELINE"); /* read per task: ranks fork from callers that read it */
    const int xproc = xpe && atoi(xpe) > 0 && !res_rc && L && L->device < 0 && g_srv_n > 0 && T->send_fill &&
                      T->send_fill != bcp_lb_transport()->send_fill && bcpi_arena_block(L->h_win[0], &rb_, &rz_);
    /* folds go to a node fold server (rows in its arena): ranges too */
    const int remote_fold = !res_rc && L && L->device < 0 && g_srv_n > 0 && bcpi_arena_block(L->h_win[0], &rb_, &rz_);
    /* (through a server, whole windows batched across ranks beat range by
     * range: r2d0 for rank processes, r2d3 for loopback ranks of a
     * connected process -- config 5 41-54 vs 36-46 GiB/s; so ranges go to
     * a server only with BCP_XPROC_PIPELINE=1) */
    int pipelined = mode == BCP_FOLD_PIPELINED && !res_rc && expected_messages == 1 && T->send_fill &&
                    ((T->send_fill == bcp_lb_transport()->send_fill && (!remote_fold || (xpe && atoi(xpe) > 0))) ||
                     xproc);
    if (pipelined && !hook && !remote_fold && !L->q && bcp_queue_create(L->eng, &L->q))
        pipelined = 0;
    if (serial_io && !res_rc)
        open_parity_chunk(hs, path, final_size, open_parity, &P_fd, &opened, &have_had_error,
                          ti.is_rebuilding ? NULL : chunk_sizes, n);
    phase_add(BCP_PHASE_P_OPEN, &tph);
    if (res_rc) {
        int drc = drain_windows(T, ranks, n, buffer_size, expected_messages, ti.tag);
        if (drc)
            LOGERR("draining the senders of '%s' failed: %s\n", path, strerror(as_errno(drc)));
        if (ti.sample)
            ti.sample->bytes_written += buffer_size * expected_messages;
        goto done;
    }

    if (expected_messages == 0)
        open_parity_chunk(hs, path, final_size, open_parity, &P_fd, &opened, &have_had_error,
                          ti.is_rebuilding ? NULL : chunk_sizes, n);

    uint8_t *win_a = L ? L->h_win[0] : NULL, *win_b = L ? L->h_win[1] : NULL, *pblk = L ? L->h_par : NULL;
    for (int j = 0; j < n; j++)
        req[j] = NULL;
    for (uint64_t msg_i = 0; msg_i < expected_messages; msg_i++) {
        /* After a transport error the loop keeps receiving every window from
         * every source (failed peers fail fast): live senders finish their
         * task instead of blocking; nothing more is folded or written. */
        row_watch W;
        int watched = 0;
        if (msg_i == 0) {
            /* implicit padding (chunk_sender): a fold that reads whole rows
             * gets the zeros past each chunk, written before the sources
             * fill the data bytes; the other folds read valid[j] bytes */
            if (pad_rows)
                for (int j = 0; j < n; j++)
                    if (valid[j] < buffer_size)
                        memset(win_a + (size_t)j * pitch + valid[j], 0, buffer_size - valid[j]);
            watched = pipelined && !have_had_error &&
                      watch_rows(&W, L, hook, hook_ctx, win_a, pitch, valid, n, buffer_size, pblk,
                                 remote_fold && !hook, hs->storage_target, ti.tag);
            trc = post_recvs(T, req, n, win_a, pitch, buffer_size, ranks, ti.tag);
            open_parity_chunk(hs, path, final_size, open_parity, &P_fd, &opened, &have_had_error,
                              ti.is_rebuilding ? NULL : chunk_sizes, n);
        }
        int w = 0, crc = 0;
        if (streamed && !have_had_error && !trc)
            crc = stream_rows_in(T, L, req, n, win_a, pitch, valid, &w);
        else
            w = wait_posted(T, req, n);
        trc = trc ? trc : w;
        if (crc && !have_had_error) {
            have_had_error = EIO;
            LOGERR("row copy of '%s' failed: %s\n", path, bcp_strerror(crc));
        }
        if (msg_i + 1 != expected_messages) {
            int p2 = post_recvs(T, req, n, win_b, pitch, buffer_size, ranks, ti.tag);
            trc = trc ? trc : p2;
        }
        phase_add(BCP_PHASE_P_ROWS, &tph);
        if (trc && !have_had_error) {
            have_had_error = as_errno(trc);
            LOGERR("windows of '%s' not received: %s\n", path, strerror(have_had_error));
        }
        /* fold window msg_i on the GPU while the senders fill win_b */
        if (!have_had_error) {
            int frc = watched    ? finish_rows(&W, 1)
                      : streamed ? stream_fold(L, n, pitch, valid, buffer_size, pblk)
                                 : fold_window(L, hs, mode, hook, hook_ctx, win_a, pitch, valid, buffer_size, n, pblk);
            if (frc) {
                have_had_error = EIO;
                LOGERR("GPU fold of '%s' failed: %s\n", path, bcp_strerror(frc));
            }
        } else if (watched) {
            (void)finish_rows(&W, 0); /* ranges in flight read these rows */
        }
        phase_add(BCP_PHASE_P_FOLD, &tph);
        if (!have_had_error) {
            size_t wsize = (size_t)MIN_((uint64_t)buffer_size, data_left);
            ssize_t wr = write(P_fd, pblk, wsize);
            if (wr <= 0) {
                have_had_error = errno;
                LOGERR("write of '%s' failed with %d (%s) after %llu bytes\n", path, errno, strerror(errno),
                       (unsigned long long)(final_size - data_left));
            }
            data_left -= wsize;
        }
        if (ti.sample)
            ti.sample->bytes_written += buffer_size;
        phase_add(BCP_PHASE_P_WRITE, &tph);
        uint8_t *t = win_a;
        win_a = win_b;
        win_b = t;
    }

    if (ti.is_rebuilding && P_fd != hs->fd_null)
        if (ftruncate(P_fd, (off_t)final_parity_chunk_size) != 0 && !have_had_error)
            have_had_error = errno;

done:
    if (have_had_error != 0 && raise_sticky_error(hs, have_had_error, path))
        LOGERR("error on '%s' is now sticky for st %d\n", path, hs->storage_target);
    res_release(L);
    if (P_fd != hs->fd_null)
        close(P_fd);
    phase_add(BCP_PHASE_P_CLOSE, &tph);
    __atomic_fetch_add(&g_phase_ns[BCP_PHASE_P_TASKS], 1, __ATOMIC_RELAXED);
}

static uint8_t *sender_buffer(size_t need)
{
    lane_res *L = &t_res;
    if (L->send_cap < need || !L->send_buf) {
        free(L->send_buf);
        L->send_buf = NULL;
        L->send_cap = 0;
        if (bcpi_inject_hit(BCP_INJECT_SEND_BUF))
            return NULL;
        size_t cap = MAX_(need, (size_t)1 << 20);
        if ((L->send_buf = malloc(cap)))
            L->send_cap = cap;
    }
    return L->send_buf;
}

/* One window of the source role, produced straight into the receiver's
 * buffer (send_fill): the file's next bytes, zero padded after a short read;
 * zeros after an open or read error or for an empty chunk (A3-q2). */
typedef struct {
    int fd;
    uint64_t fd_size, data_to_send, data_sent;
    int err;
    HostState *hs;
    const char *path;
    int implicit_pad; /* produce the chunk's bytes only (chunk_sender) */
} window_fill;

/* Bytes of the window starting at data_sent that carry the chunk (up to the
 * size it reported, and never past data_to_send). */
static size_t window_data_bytes(uint64_t data_to_send, uint64_t fd_size, uint64_t data_sent, size_t n)
{
    const uint64_t lim = MIN_(data_to_send, fd_size);
    return data_sent < lim ? (size_t)MIN_((uint64_t)n, lim - data_sent) : 0;
}

static void fill_bytes(window_fill *w, uint8_t *data, size_t n);

static int fill_window(void *ctx, void *dst, size_t n)
{
    fill_bytes(ctx, dst, n);
    /* dst may be device memory stored through the BAR (DEVICE_ROWS): drain
     * this thread's write-combining buffers before the window is handed on */
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    return 0;
}

/* Publish a final prefix of the row being filled: to a P role of this
 * process (its row watch), or, through the socket transport, to a P role in
 * another process (PROG frames, bcpi_fill_progress). */
static void fill_publish(row_watch *W, int wj, int xp, size_t bytes, int redo)
{
    if (W)
        watch_publish(W, wj, bytes, redo);
    else if (xp)
        (void)bcpi_fill_progress(bytes, redo); /* a lost report only delays the fold to the tail */
}

static void fill_bytes(window_fill *w, uint8_t *data, size_t n)
{
    HostState *hs = w->hs;
    /* the bytes this window must define: all n, or with implicit padding
     * the chunk's own (the P role supplies the zeros past them) */
    const size_t need = w->implicit_pad ? window_data_bytes(w->data_to_send, w->fd_size, w->data_sent, n) : n;
    int wj = 0;
    row_watch *W = watch_find(data, &wj); /* a P role folding this row as it fills */
    const int xp = !W && bcpi_fill_progress_on(); /* ... in another rank process */
    if (w->err != 0 || w->data_sent >= w->fd_size) {
        memset(data, 0, need);
        fill_publish(W, wj, xp, need, 0);
        return;
    }
    /* up to the size the chunk reported (not past it should the file have
     * grown since fstat: the parity body then agrees with its header) */
    const uint64_t left = MIN_(w->data_to_send, w->fd_size) - w->data_sent;
    const size_t want = (size_t)MIN_((uint64_t)n, left);
    ssize_t r;
    if (!W && !xp) {
        r = bcpi_inject_hit(BCP_INJECT_READ) ? (errno = EIO, -1) : read(w->fd, data, want);
    } else {
        /* in pieces, publishing the final prefix after each (EOF ends it) */
        size_t got = 0;
        r = 0;
        while (got < want) {
            ssize_t k = got && bcpi_inject_hit(BCP_INJECT_READ) ? (errno = EIO, -1)
                                                                : read(w->fd, data + got, MIN_(watch_piece(), want - got));
            if (k <= 0) {
                r = k < 0 ? k : (ssize_t)got;
                break;
            }
            got += (size_t)k;
            r = (ssize_t)got;
            if (got < want)
                fill_publish(W, wj, xp, got, 0);
        }
    }
    if (r < 0) {
        w->err = errno;
        memset(data, 0, need);
        LOGERR("read of '%s' failed with %d (%s) after %llu bytes\n", w->path, errno, strerror(errno),
               (unsigned long long)w->data_sent);
        fill_publish(W, wj, xp, need, 1); /* the zeros replace bytes already published */
        return;
    }
    if ((size_t)r < need)
        memset(data + r, 0, need - (size_t)r);
    fill_publish(W, wj, xp, MAX_(need, (size_t)r), 0);
}

static void chunk_sender(const bcp_transport_ops *T, const char *path, const FileInfo *task, TaskInfo ti,
                         HostState *hs)
{
    const int my_st = hs->storage_target;
    const int coordinator = st2rank[GET_P(task->locations)];
    const int ntargets = active_ranks(task->locations);
    uint64_t fd_size = 0;
    int have_had_error = 0, trc = 0;
    uint64_t tph = mono_ns();
    int fd = open_chunk_readonly(ti.read_dir, path);
    if (fd <= 0) {
        have_had_error = errno;
        fd = hs->fd_zero;
        LOGERR("cannot open '%s': %d (%s)\n", path, errno, strerror(errno));
    } else {
        struct stat st;
        fstat(fd, &st);
        fd_size = (uint64_t)st.st_size;
        if (ti.is_rebuilding && ti.actual_P_st == my_st)
            fd_size -= (uint64_t)ntargets * sizeof(uint64_t);
        if (ti.is_rebuilding && ti.actual_P_st != my_st && st.st_mtime > task->timestamp)
            push_corrupt_path(hs, path);
    }

    if (ti.is_rebuilding && ti.actual_P_st == my_st) {
        /* the parity holder forwards the stored header instead of a size */
        uint64_t chunk_sizes[MAX_STORAGE_TARGETS] = {0};
        ssize_t r = read(fd, chunk_sizes, (size_t)ntargets * sizeof(uint64_t));
        (void)r;
        trc = T->send(T->ctx, chunk_sizes, (size_t)ntargets * sizeof(uint64_t), coordinator, ti.tag);
    } else if (!ti.is_rebuilding) {
        trc = T->send(T->ctx, &fd_size, sizeof(fd_size), coordinator, ti.tag);
    }

    uint64_t data_to_send = 0;
    if (!trc)
        trc = T->recv(T->ctx, &data_to_send, sizeof(data_to_send), coordinator, ti.tag);
    if (trc) {
        /* no window size: nothing more can be exchanged for this task */
        if (!have_had_error)
            have_had_error = as_errno(trc);
        LOGERR("size exchange for '%s' failed: %s\n", path, strerror(as_errno(trc)));
        goto done;
    }

    phase_add(BCP_PHASE_S_SIZES, &tph);
    const size_t buffer_size = (size_t)MIN_(WINDOW, data_to_send);
    /* Implicit padding: in gen with ONE window (max_cs <= WINDOW) the P role
     * takes row j's first chunk_sizes[j] bytes and supplies the zeros past
     * them itself (parity_generator), so the window carries the chunk's
     * bytes only -- a fill of that many bytes, or a shorter message (an MPI
     * receive takes a message shorter than its buffer).  The reference pads
     * every window to buffer_size with zeros (task_processing.c:302-303);
     * the parity is the same, and the padding (up to 60x the data for a
     * small chunk in a stripe of large ones) neither crosses PCIe into
     * device rows nor a socket. */
    const int implicit_pad =
        !ti.is_rebuilding && data_to_send <= WINDOW && !__atomic_load_n(&g_explicit_pad, __ATOMIC_ACQUIRE);
    /* Zero copy (a transport with send_fill): every window is read straight
     * into P's window row, unless a later window could replay this one
     * (A3-q1: the file ends before max_cs and more than one window is sent),
     * which needs the sender's own buffer. */
    const int replay = fd_size < data_to_send && data_to_send > buffer_size;
    uint8_t *data = NULL;
    if (!(T->send_fill && !replay)) {
        data = sender_buffer(buffer_size);
        if (!data) {
            if (!have_had_error)
                have_had_error = ENOMEM;
            LOGERR("no window buffer for '%s': sending zeros\n", path);
        }
    }
    if (T->send_fill && (!replay || !data)) {
        window_fill wf = {fd, fd_size, data_to_send, 0, have_had_error, hs, path, implicit_pad};
        while (wf.data_sent < data_to_send) {
            if (ti.sample)
                ti.sample->bytes_read += buffer_size;
            int e = T->send_fill(T->ctx, fill_window, &wf, buffer_size, coordinator, ti.tag);
            if (e && e != -EMSGSIZE && !trc)
                trc = e;
            wf.data_sent += buffer_size;
        }
        have_had_error = wf.err;
        goto sent;
    }
    if (!data) {
        /* no buffer and no fill send: the windows go out as zeros */
        for (uint64_t sent = 0; sent < data_to_send; sent += buffer_size) {
            if (ti.sample)
                ti.sample->bytes_read += buffer_size;
            int e = T->send(T->ctx, g_zero_window, buffer_size, coordinator, ti.tag);
            if (e && !trc)
                trc = e;
        }
        goto sent;
    }
    /* A buffer that is never filled is sent as zeros: the reference sends
     * uninitialised memory for a zero-length chunk (quirk A3-q2). */
    if (have_had_error != 0 || fd_size == 0)
        memset(data, 0, buffer_size);

    uint64_t data_sent = 0;
    while (data_sent < data_to_send) {
        uint64_t left = MIN_(data_to_send, fd_size) - data_sent; /* up to the reported size (fill_window) */
        const size_t msg = implicit_pad ? window_data_bytes(data_to_send, fd_size, data_sent, buffer_size)
                                        : buffer_size;
        /* once the file is exhausted the previous window is re-sent (A3-q1) */
        if (have_had_error == 0 && data_sent < fd_size) {
            ssize_t r = read(fd, data, (size_t)MIN_((uint64_t)buffer_size, left));
            if (r < 0) {
                have_had_error = errno;
                memset(data, 0, msg);
                LOGERR("read of '%s' failed with %d (%s) after %llu bytes\n", path, errno, strerror(errno),
                       (unsigned long long)data_sent);
            }
            if (r >= 0 && (size_t)r < msg)
                memset(data + r, 0, msg - (size_t)r);
        }
        if (ti.sample)
            ti.sample->bytes_read += buffer_size;
        data_sent += buffer_size;
        int e = T->send(T->ctx, data, msg, coordinator, ti.tag);
        if (e && !trc)
            trc = e;
    }

sent:
    if (trc && !have_had_error) {
        have_had_error = as_errno(trc);
        LOGERR("windows of '%s' not sent: %s\n", path, strerror(have_had_error));
    }
done:
    /* ENOENT: the chunk vanished after planning; an unlink event follows. */
    if (have_had_error != 0 && have_had_error != ENOENT && raise_sticky_error(hs, have_had_error, path))
        LOGERR("error on '%s' is now sticky for st %d\n", path, hs->storage_target);
    if (fd != hs->fd_zero)
        close(fd);
    phase_add(BCP_PHASE_S_SEND, &tph);
    __atomic_fetch_add(&g_phase_ns[BCP_PHASE_S_TASKS], 1, __ATOMIC_RELAXED);
}

int process_task(HostState *hs, const char *path, const FileInfo *fi, TaskInfo ti)
{
    assert(GET_P(fi->locations) != (int)NO_P);
    assert(P_IS_INVALID(fi->locations) == 0);
    assert(hs->storage_target >= 0);

    const bcp_transport_ops T = transport_now();
    if (GET_P(fi->locations) == hs->storage_target)
        parity_generator(&T, path, fi, ti, hs);
    else if (TEST_BIT(fi->locations, hs->storage_target))
        chunk_sender(&T, path, fi, ti, hs);
    else
        return 0;
    return active_ranks(fi->locations) != 0;
}

void bcpi_settings_get(bcpi_settings *s)
{
    pthread_mutex_lock(&g_lock);
    s->fold_mode = g_fold_mode;
    s->fold_inflight = g_fold_inflight;
    s->hook = g_hook;
    s->hook_ctx = g_hook_ctx;
    pthread_mutex_unlock(&g_lock);
    s->explicit_pad = __atomic_load_n(&g_explicit_pad, __ATOMIC_ACQUIRE);
}

int bcpi_settings_apply(const bcpi_settings *s)
{
    int rc = bcp_task_set_fold_mode(s->fold_mode);
    if (rc >= 0)
        rc = bcp_task_set_fold_inflight(s->fold_inflight);
    if (rc >= 0)
        rc = bcp_task_set_explicit_padding(s->explicit_pad);
    if (rc < 0)
        return rc;
    bcp_task_set_xor_hook(s->hook, s->hook_ctx);
    return 0;
}
