/*
 * bcp_task.c -- the per-rank chunk-streaming protocol (process_task): the
 * roles, their settings and their transport.
 *
 * Behaviour follows the reference's roles and message flow
 * (src/beegfs-raid5/common/task_processing.c):
 *   process_task      :325-340  dispatch by role
 *   parity_generator  :117-245  P role: sizes -> max_cs -> windows -> parity
 *   chunk_sender      :247-322  source role: size -> windows (zero padded)
 * What is underneath is this library's:
 *   - the peers are reached through a transport table (bcp_task_set_transport:
 *     in-process loopback ranks by default, socketpair-connected rank
 *     processes, or a caller's binding such as MPI), exactly the
 *     point-to-point subset the reference uses;
 *   - the window fold (xor_parity at :211) runs on the GPU over pinned,
 *     device-mapped window rows (256-byte pitch, so every row is 16-byte
 *     aligned for the streaming kernel): bcp_fold.c (fold service, pipelined
 *     fold) and bcp_foldsrv.c (the node fold server of rank processes);
 *   - nothing aborts: when the P role cannot get fold resources it still
 *     drains its senders through one bounded row and raises the sticky error;
 *     a source without a window buffer sends zeros and raises it.
 * Every setting is read once per task under the settings lock; nothing on
 * the per-task path reads the environment.
 */
#define _GNU_SOURCE
#include <assert.h>
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <time.h>
#include <unistd.h>

#include "bcp_fold.h"

#define WINDOW ((uint64_t)BCP_WINDOW_BYTES)
#define ROW_ALIGN BCPF_ROW_ALIGN
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

/* ---- settings: fold mode, window padding, test hook, transport ------------ */
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static bcp_xor_hook_fn g_hook = NULL;
static void *g_hook_ctx = NULL;
static int g_fold_mode = BCP_FOLD_PIPELINED;
static int g_pad = BCP_PAD_AUTO;
static bcp_transport_ops g_tp;
static int g_tp_set = 0;

/* Never written: the source role's windows when it has no buffer of its own
 * (zero pages until read; .bss costs no file or resident memory). */
static uint8_t g_zero_window[BCP_WINDOW_BYTES];

int bcp_task_set_fold_mode(int mode)
{
    if (mode != BCP_FOLD_BATCHED && mode != BCP_FOLD_PIPELINED)
        return -EINVAL;
    pthread_mutex_lock(&g_lock);
    int prev = g_fold_mode;
    g_fold_mode = mode;
    pthread_mutex_unlock(&g_lock);
    return prev;
}

int bcp_task_set_explicit_padding(int on)
{
    if (on != BCP_PAD_AUTO && on != 0 && on != 1)
        return -EINVAL;
    pthread_mutex_lock(&g_lock);
    const int prev = g_pad;
    g_pad = on;
    pthread_mutex_unlock(&g_lock);
    return prev;
}

void bcp_task_set_xor_hook(bcp_xor_hook_fn fn, void *ctx)
{
    pthread_mutex_lock(&g_lock);
    g_hook = fn;
    g_hook_ctx = ctx;
    pthread_mutex_unlock(&g_lock);
}

void bcpf_hook_get(bcp_xor_hook_fn *fn, void **ctx)
{
    pthread_mutex_lock(&g_lock);
    *fn = g_hook;
    *ctx = g_hook_ctx;
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

/* Everything one task reads of the settings, in one snapshot: stable for the
 * task's duration whatever another thread sets meanwhile. */
typedef struct {
    bcp_transport_ops T;
    bcp_xor_hook_fn hook;
    void *hook_ctx;
    int fold_mode;
    int fold_ring;    /* PIPELINED folds through the device's resident ring */
    int implicit_pad; /* sources may send a one-window gen chunk's bytes only */
} task_settings;

/* Implicit padding is this library's wire: only towards peers that are this
 * library's P roles for certain -- its own transports (loopback ranks, its
 * socketpair rank processes) -- unless the caller chose.  A caller's table
 * (an MPI binding) may connect to the reference's parity_generator, which
 * folds whole buffer_size rows (task_processing.c:206-211), so it gets the
 * reference's zero-padded windows (:302-303) by default. */
static int own_transport(const bcp_transport_ops *T)
{
    return T->send == bcp_lb_transport()->send || bcpi_sock_transport_is(T);
}

static void settings_now(task_settings *s)
{
    pthread_mutex_lock(&g_lock);
    s->T = g_tp_set ? g_tp : *bcp_lb_transport();
    s->hook = g_hook;
    s->hook_ctx = g_hook_ctx;
    s->fold_mode = g_fold_mode;
    const int pad = g_pad;
    pthread_mutex_unlock(&g_lock);
    s->implicit_pad = pad == BCP_PAD_AUTO ? own_transport(&s->T) : pad == 0;
    s->fold_ring = s->fold_mode == BCP_FOLD_PIPELINED && bcpi_fold_ring();
}

/* ---- failure injection (tests) ------------------------------------------ */
#define NSITES 8
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
    case BCP_INJECT_DIRECT_READ: return 6;
    case BCP_INJECT_PARITY_WRITE: return 7;
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

/* ---- the source role's window buffer (per lane thread) -------------------- */
typedef struct {
    uint8_t *send_buf; /* chunk_sender window buffer */
    size_t send_cap;
} lane_res;

static __thread lane_res t_res;

/* ---- deferred P-role completion (lane deferral) ---------------------------
 * A lane that opted in (bcp_task_set_lane_deferral: libbcp's own runners,
 * for lanes that keep no DB) lets a single-window P task return once its
 * fold is published to the device's resident ring: the wait for the fold,
 * the parity write, the rebuild's truncation and the file's close happen
 * when this lane's next task has published its own fold or finished
 * sending (or at bcp_task_flush / bcp_task_thread_release).  So a lane's
 * next task overlaps the previous one's fold and write, as two buffers of
 * parity_generator's own window loop overlap receive and fold
 * (task_processing.c:203-226).  Same bytes, same files; an error of the
 * deferred part becomes sticky when it completes. */
typedef struct {
    int active;
    HostState *hs;
    char *path;
    fold_res *L;
    bcp_ring *ring;
    uint64_t hnd[BCPF_WATCH_HANDLES + 1];
    int nh;
    int fd;
    uint8_t *pblk;
    size_t wsize;
    int rebuilding;
    uint64_t final_size; /* rebuild: the rebuilt chunk's size */
    uint64_t final_total;
} deferred_p;

/* This lane's deferred P tasks, oldest first (at most t_defer_on). */
static __thread deferred_p t_def[BCP_DEFER_MAX];
static __thread int t_ndef;
static __thread int t_defer_on;

int bcp_task_set_lane_deferral(int on)
{
    if (on < 0 || on > BCP_DEFER_MAX)
        return -EINVAL;
    const int prev = t_defer_on;
    t_defer_on = on;
    return prev;
}

static int raise_sticky_error(HostState *hs, int err, const char *path);
static uint64_t mono_ns(void);
static void phase_add(int ph, uint64_t *t);

static void deferred_complete(deferred_p *d)
{
    if (!d->active)
        return;
    d->active = 0;
    HostState *hs = d->hs;
    uint64_t tph = mono_ns();
    int err = 0;
    for (int i = 0; i < d->nh; i++) {
        const int rc = bcp_ring_wait(d->ring, d->hnd[i]);
        if (rc && !err) {
            err = EIO;
            LOGERR("GPU fold of '%s' failed: %s\n", d->path, bcp_strerror(rc));
        }
    }
    if (!err) {
        ssize_t wr = bcpi_inject_hit(BCP_INJECT_PARITY_WRITE) ? (errno = ENOSPC, -1) : write(d->fd, d->pblk, d->wsize);
        if (wr <= 0) {
            err = errno;
            LOGERR("write of '%s' failed with %d (%s) after %llu bytes\n", d->path, errno, strerror(errno),
                   (unsigned long long)(d->final_total - d->wsize));
        }
    }
    if (d->rebuilding && d->fd != hs->fd_null)
        if (ftruncate(d->fd, (off_t)d->final_size) != 0 && !err)
            err = errno;
    if (err && raise_sticky_error(hs, err, d->path))
        LOGERR("error on '%s' is now sticky for st %d\n", d->path, hs->storage_target);
    bcpf_res_release(d->L);
    if (d->fd != hs->fd_null)
        close(d->fd);
    free(d->path);
    phase_add(BCP_PHASE_P_WRITE, &tph);
}

/* Complete this lane's oldest deferred tasks until at most `keep` remain. */
static void deferred_trim(int keep)
{
    while (t_ndef > keep) {
        deferred_complete(&t_def[0]);
        for (int i = 1; i < t_ndef; i++)
            t_def[i - 1] = t_def[i];
        t_ndef--;
    }
}

/* ---- completion threads ---------------------------------------------------
 * The deferred part of a lane's tasks (fold wait, write, truncation, close)
 * runs on a few threads of this process (bcp_task_set_fold_tuning
 * "completion_threads", default 4), so the lane goes straight on to its next
 * task; with 0 the lane completes its own, oldest first, when it next
 * publishes (deferred_trim).  Either way a lane holds at most `depth`
 * deferred tasks -- their rows stay reserved until they complete -- and
 * bcp_task_flush waits for its own.  A lane thread that ends without a flush
 * is flushed by its key's destructor.  bcp_task_shutdown drains the queue
 * and joins the threads (bcpt_completion_stop). */
typedef struct {
    int pending; /* this lane's items in the queue or being completed */
    int init;
    pthread_cond_t done; /* signalled (under cq_mu) when one of them completes */
} cq_lane;

typedef struct cq_item {
    struct cq_item *next;
    deferred_p d;
    cq_lane *lane; /* the submitting lane's */
} cq_item;

static pthread_mutex_t cq_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t cq_work = PTHREAD_COND_INITIALIZER;
static cq_item *cq_head, *cq_tail;
static int cq_nthreads, cq_quit;
static pthread_t cq_tid[BCP_COMPLETION_MAX];
/* each lane waits on its own condition: a completion wakes its lane only,
 * not every lane at its depth limit */
static __thread cq_lane t_cq;
static pthread_key_t cq_key;
static pthread_once_t cq_key_once = PTHREAD_ONCE_INIT;

static void *cq_main(void *arg)
{
    (void)arg;
    pthread_mutex_lock(&cq_mu);
    for (;;) {
        while (!cq_head && !cq_quit)
            pthread_cond_wait(&cq_work, &cq_mu);
        cq_item *it = cq_head;
        if (!it)
            break; /* stopping, and nothing is left */
        cq_head = it->next;
        if (!cq_head)
            cq_tail = NULL;
        pthread_mutex_unlock(&cq_mu);
        deferred_complete(&it->d);
        pthread_mutex_lock(&cq_mu);
        it->lane->pending--;
        pthread_cond_signal(&it->lane->done);
        free(it);
    }
    pthread_mutex_unlock(&cq_mu);
    return NULL;
}

static void cq_wait_own(int below)
{
    if (!t_cq.init)
        return; /* this thread never handed a task over */
    pthread_mutex_lock(&cq_mu);
    while (t_cq.pending > below)
        pthread_cond_wait(&t_cq.done, &cq_mu);
    pthread_mutex_unlock(&cq_mu);
}

static void cq_thread_end(void *v)
{
    (void)v;
    deferred_trim(0);
    cq_wait_own(0);
    if (t_cq.init) {
        pthread_cond_destroy(&t_cq.done);
        t_cq.init = 0;
    }
}

static void cq_make_key(void) { (void)pthread_key_create(&cq_key, cq_thread_end); }

/* The completion threads wanted now, started on first use; 0 = none. */
static int cq_threads(void)
{
    const int want = bcpi_completion_threads();
    if (want <= 0)
        return 0;
    pthread_mutex_lock(&cq_mu);
    while (cq_nthreads < want && !cq_quit && pthread_create(&cq_tid[cq_nthreads], NULL, cq_main, NULL) == 0)
        cq_nthreads++;
    const int n = cq_quit ? 0 : cq_nthreads;
    pthread_mutex_unlock(&cq_mu);
    return n;
}

/* Hand a published task's deferred part over: to the completion threads, or
 * keep it on this lane (completing the oldest beyond depth - 1 first). */
static void deferred_add(const deferred_p *d)
{
    cq_item *it = cq_threads() > 0 ? malloc(sizeof *it) : NULL;
    if (!it) {
        deferred_trim(t_defer_on - 1);
        t_def[t_ndef++] = *d;
        return;
    }
    if (!t_cq.init) {
        (void)pthread_once(&cq_key_once, cq_make_key);
        (void)pthread_setspecific(cq_key, (void *)1); /* flushed at thread end */
        pthread_cond_init(&t_cq.done, NULL);
        t_cq.init = 1;
    }
    it->next = NULL;
    it->d = *d;
    it->lane = &t_cq;
    pthread_mutex_lock(&cq_mu);
    while (t_cq.pending >= t_defer_on)
        pthread_cond_wait(&t_cq.done, &cq_mu);
    t_cq.pending++;
    if (cq_tail)
        cq_tail->next = it;
    else
        cq_head = it;
    cq_tail = it;
    pthread_cond_signal(&cq_work);
    pthread_mutex_unlock(&cq_mu);
}

void bcpt_completion_stop(void)
{
    pthread_mutex_lock(&cq_mu);
    cq_quit = 1;
    pthread_cond_broadcast(&cq_work);
    const int n = cq_nthreads;
    pthread_mutex_unlock(&cq_mu);
    for (int i = 0; i < n; i++)
        pthread_join(cq_tid[i], NULL);
    pthread_mutex_lock(&cq_mu);
    cq_nthreads = 0;
    cq_quit = 0;
    pthread_mutex_unlock(&cq_mu);
}

void bcp_task_flush(void)
{
    deferred_trim(0);
    cq_wait_own(0);
}

void bcp_task_thread_release(void)
{
    bcp_task_flush();
    free(t_res.send_buf);
    t_res.send_buf = NULL;
    t_res.send_cap = 0;
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
static void parity_generator(const task_settings *ts, const char *path, const FileInfo *task, TaskInfo ti,
                             HostState *hs)
{
    const bcp_transport_ops *T = &ts->T;
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

    const bcp_xor_hook_fn hook = ts->hook;
    void *const hook_ctx = ts->hook_ctx;
    const size_t buffer_size = (size_t)MIN_(WINDOW, max_cs);
    /* rows 256-byte aligned for the GPU's 16-byte vector loads; under the
     * test hook (a CPU fold) contiguous, as the reference's receive buffer
     * is (data_a + src * buffer_size, :206) */
    const size_t pitch = hook ? buffer_size : (buffer_size + ROW_ALIGN - 1) / ROW_ALIGN * ROW_ALIGN;
    const uint64_t final_size = max_cs + (uint64_t)n * 8u;
    const uint64_t expected_messages = (max_cs + WINDOW - 1) / WINDOW;
    uint64_t data_left = max_cs;

    if (!have_had_error)
        have_had_error = __atomic_load_n(&hs->error, __ATOMIC_ACQUIRE);
    fold_res *L = NULL;
    /* a node fold server (rank processes) folds: rows and output from the
     * arena, no HIP runtime in this process */
    const int remote = bcpf_srv_attached();
    int res_rc = expected_messages ? bcpf_res_acquire(hs->storage_target, !remote && hook == NULL, pitch * (size_t)n,
                                                      buffer_size, expected_messages, &L)
                                   : 0;
    if (remote && !res_rc && L) {
        void *b;
        size_t z;
        if (!bcpi_arena_block(L->h_win[0], &b, &z) || !bcpi_arena_block(L->h_par, &b, &z) ||
            (expected_messages > 1 && !bcpi_arena_block(L->h_win[1], &b, &z))) {
            /* the arena slice is full: fold in this process as without a server */
            bcpf_res_release(L);
            L = NULL;
            res_rc = bcpf_res_acquire(hs->storage_target, hook == NULL, pitch * (size_t)n, buffer_size,
                                      expected_messages, &L);
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
    if (!open_parity)
        LOGERR("'%s' goes to the null device: error %d is sticky on this rank\n", path, have_had_error);

    /* Row j's data bytes.  A gen-mode single-window row holds chunk_sizes[j]
     * bytes then zeros (sent by the source, or -- implicit padding -- not
     * sent at all); the GPU folds read the data bytes only and supply the
     * zeros.  Anything else (rebuild: the survivors' current sizes are not
     * sent; windows past the first: replay) is taken whole. */
    size_t valid[MAX_STORAGE_TARGETS];
    const int data_only = !ti.is_rebuilding && expected_messages == 1;
    for (int j = 0; j < n; j++)
        valid[j] = data_only ? (size_t)MIN_(chunk_sizes[j], (uint64_t)buffer_size) : buffer_size;
    /* a fold that reads whole rows (the test hook) gets the zeros written into
     * the rows before the receives, whichever padding the sources use */
    const int pad_rows = data_only && !res_rc && hook != NULL;
    /* PIPELINED: one window whose rows in-process sources fill directly (the
     * loopback transport's send_fill: the sources publish their progress to
     * this process's row watches and launch range folds on this lane's
     * queue); everything else folds the whole window through the fold
     * service or the node fold server */
    void *rb_;
    size_t rz_;
    const int remote_fold = !res_rc && L && L->device < 0 && remote && bcpi_arena_block(L->h_win[0], &rb_, &rz_);
    int pipelined = ts->fold_mode == BCP_FOLD_PIPELINED && !res_rc && expected_messages == 1 && T->send_fill &&
                    T->send_fill == bcp_lb_transport()->send_fill && !remote_fold;
    /* the resident fold ring of the P role's device (PIPELINED; the fold
     * service and lane queues otherwise) */
    bcp_ring *const ring = ts->fold_ring && !res_rc && L && L->device >= 0 && !hook ? bcpf_ring_for(L->device, L->eng)
                                                                                     : NULL;
    if (pipelined && !hook && !ring && !L->q && bcp_queue_create(L->eng, &L->q))
        pipelined = 0;
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

    /* lane deferral: a single-window task whose fold goes to the ring returns
     * once the fold is published (deferred_p) */
    const int defer = t_defer_on && ring && expected_messages == 1;
    int deferred = 0;
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
            if (pad_rows)
                for (int j = 0; j < n; j++)
                    if (valid[j] < buffer_size)
                        memset(win_a + (size_t)j * pitch + valid[j], 0, buffer_size - valid[j]);
            watched = pipelined && !have_had_error &&
                      bcpf_watch_rows(&W, L, ring, hook, hook_ctx, win_a, pitch, valid, n, buffer_size, pblk);
            trc = post_recvs(T, req, n, win_a, pitch, buffer_size, ranks, ti.tag);
            open_parity_chunk(hs, path, final_size, open_parity, &P_fd, &opened, &have_had_error,
                              ti.is_rebuilding ? NULL : chunk_sizes, n);
        }
        int w = wait_posted(T, req, n);
        trc = trc ? trc : w;
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
        if (!have_had_error && defer) {
            deferred_p d = {0};
            int frc = watched ? bcpf_finish_rows_submit(&W, d.hnd, &d.nh)
                              : bcpf_ring_submit_window(ring, win_a, pitch, valid, buffer_size, n, pblk, &d.hnd[d.nh++]);
            if (frc) {
                if (!watched)
                    d.nh = 0; /* (a failed submission hands nothing over) */
                have_had_error = EIO;
                LOGERR("GPU fold of '%s' failed: %s\n", path, bcp_strerror(frc));
            } else {
                d.active = 1;
                d.hs = hs;
                d.path = strdup(path);
                d.L = L;
                d.ring = ring;
                d.fd = P_fd;
                d.pblk = pblk;
                d.wsize = (size_t)MIN_((uint64_t)buffer_size, data_left);
                d.rebuilding = ti.is_rebuilding;
                d.final_size = final_parity_chunk_size;
                d.final_total = final_size;
                if (!d.path) { /* no memory for the record: complete it here */
                    d.path = (char *)path;
                    deferred_complete(&d);
                    d.path = NULL;
                } else {
                    /* this fold is on the device: its completion goes to the
                     * completion threads, or waits on this lane */
                    deferred_add(&d);
                }
                deferred = 1;
                if (ti.sample)
                    ti.sample->bytes_written += buffer_size;
                phase_add(BCP_PHASE_P_FOLD, &tph);
                break;
            }
        } else if (!have_had_error) {
            int frc = watched ? bcpf_finish_rows(&W, 1)
                              : bcpf_fold_window(L, hs, ti.tag, hook, hook_ctx, ring != NULL, win_a, pitch, valid,
                                                 buffer_size, n, pblk);
            if (frc) {
                have_had_error = EIO;
                LOGERR("GPU fold of '%s' failed: %s\n", path, bcp_strerror(frc));
            }
        } else if (watched) {
            (void)bcpf_finish_rows(&W, 0); /* ranges in flight read these rows */
        }
        phase_add(BCP_PHASE_P_FOLD, &tph);
        if (!have_had_error) {
            size_t wsize = (size_t)MIN_((uint64_t)buffer_size, data_left);
            ssize_t wr = bcpi_inject_hit(BCP_INJECT_PARITY_WRITE) ? (errno = ENOSPC, -1) : write(P_fd, pblk, wsize);
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

    if (deferred) {
        /* the record owns the resources, the file and its error */
        __atomic_fetch_add(&g_phase_ns[BCP_PHASE_P_TASKS], 1, __ATOMIC_RELAXED);
        return;
    }
    if (ti.is_rebuilding && P_fd != hs->fd_null)
        if (ftruncate(P_fd, (off_t)final_parity_chunk_size) != 0 && !have_had_error)
            have_had_error = errno;

done:
    if (have_had_error != 0 && raise_sticky_error(hs, have_had_error, path))
        LOGERR("error on '%s' is now sticky for st %d\n", path, hs->storage_target);
    bcpf_res_release(L);
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
static void fill_bytes(window_fill *w, uint8_t *data, size_t n)
{
    HostState *hs = w->hs;
    /* the bytes this window must define: all n, or with implicit padding
     * the chunk's own (the P role supplies the zeros past them) */
    const size_t need = w->implicit_pad ? window_data_bytes(w->data_to_send, w->fd_size, w->data_sent, n) : n;
    int wj = 0;
    row_watch *W = bcpf_watch_find(data, &wj); /* a P role folding this row as it fills */
    if (w->err != 0 || w->data_sent >= w->fd_size) {
        memset(data, 0, need);
        if (W)
            bcpf_watch_publish(W, wj, need, 0);
        return;
    }
    /* up to the size the chunk reported (not past it should the file have
     * grown since fstat: the parity body then agrees with its header) */
    const uint64_t left = MIN_(w->data_to_send, w->fd_size) - w->data_sent;
    const size_t want = (size_t)MIN_((uint64_t)n, left);
    ssize_t r;
    if (!W) {
        r = bcpi_inject_hit(BCP_INJECT_READ) ? (errno = EIO, -1) : read(w->fd, data, want);
    } else {
        /* in pieces, publishing the final prefix after each (EOF ends it) */
        size_t got = 0;
        r = 0;
        while (got < want) {
            ssize_t k = got && bcpi_inject_hit(BCP_INJECT_READ)
                            ? (errno = EIO, -1)
                            : read(w->fd, data + got, MIN_(bcpf_watch_piece(), want - got));
            if (k <= 0) {
                r = k < 0 ? k : (ssize_t)got;
                break;
            }
            got += (size_t)k;
            r = (ssize_t)got;
            if (got < want)
                bcpf_watch_publish(W, wj, got, 0);
        }
    }
    if (r < 0) {
        w->err = errno;
        memset(data, 0, need);
        LOGERR("read of '%s' failed with %d (%s) after %llu bytes\n", w->path, errno, strerror(errno),
               (unsigned long long)w->data_sent);
        if (W)
            bcpf_watch_publish(W, wj, need, 1); /* the zeros replace bytes already published */
        return;
    }
    if ((size_t)r < need)
        memset(data + r, 0, need - (size_t)r);
    if (W)
        bcpf_watch_publish(W, wj, MAX_(need, (size_t)r), 0);
}

static int fill_window(void *ctx, void *dst, size_t n)
{
    fill_bytes(ctx, dst, n);
    return 0;
}

static void chunk_sender(const task_settings *ts, const char *path, const FileInfo *task, TaskInfo ti,
                         HostState *hs)
{
    const bcp_transport_ops *T = &ts->T;
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
    /* Implicit padding: in gen with ONE window (max_cs <= WINDOW) this
     * library's P role takes row j's first chunk_sizes[j] bytes and supplies
     * the zeros past them itself (parity_generator), so the window carries
     * the chunk's bytes only -- a fill of that many bytes, or a shorter
     * message (an MPI receive takes a message shorter than its buffer).  The
     * reference pads every window to buffer_size with zeros
     * (task_processing.c:302-303); the parity is the same, and the padding
     * (up to 60x the data for a small chunk in a stripe of large ones)
     * neither crosses PCIe nor a socket.  Only where the P roles are this
     * library's (task_settings.implicit_pad). */
    const int implicit_pad = !ti.is_rebuilding && data_to_send <= WINDOW && ts->implicit_pad;
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
        uint64_t left = MIN_(data_to_send, fd_size) - data_sent; /* up to the reported size (fill_bytes) */
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
    /* this lane's deferred P tasks but the newest depth - 1 (their folds had
     * the sends' time to land) */
    deferred_trim(t_defer_on > 0 ? t_defer_on - 1 : 0);
}

int process_task(HostState *hs, const char *path, const FileInfo *fi, TaskInfo ti)
{
    assert(GET_P(fi->locations) != (int)NO_P);
    assert(P_IS_INVALID(fi->locations) == 0);
    assert(hs->storage_target >= 0);

    /* A path that would name a file outside the rank's chunk / parity
     * directories (absolute, "..") is refused -- by every rank alike, so the
     * task is skipped everywhere and no message goes unanswered.  (The
     * reference trusts its worklist here.) */
    if (!bcpi_path_ok(path, (size_t)-1)) {
        LOGERR("refusing '%s': not a path inside the store\n", path);
        return 0;
    }
    task_settings ts;
    settings_now(&ts);
    if (GET_P(fi->locations) == hs->storage_target)
        parity_generator(&ts, path, fi, ti, hs);
    else if (TEST_BIT(fi->locations, hs->storage_target))
        chunk_sender(&ts, path, fi, ti, hs);
    else
        return 0;
    return active_ranks(fi->locations) != 0;
}

void bcpi_settings_get(bcpi_settings *s)
{
    pthread_mutex_lock(&g_lock);
    s->fold_mode = g_fold_mode;
    s->hook = g_hook;
    s->hook_ctx = g_hook_ctx;
    s->explicit_pad = g_pad;
    pthread_mutex_unlock(&g_lock);
    s->fold_inflight = bcpi_fold_inflight();
    s->fold_ring = bcpi_fold_ring();
}

int bcpi_settings_apply(const bcpi_settings *s)
{
    int rc = bcp_task_set_fold_mode(s->fold_mode);
    if (rc >= 0)
        rc = bcp_task_set_fold_inflight(s->fold_inflight);
    if (rc >= 0)
        rc = bcp_task_set_fold_ring(s->fold_ring);
    if (rc >= 0 && bcp_task_set_explicit_padding(s->explicit_pad) == -EINVAL) /* (returns BCP_PAD_AUTO = -1 too) */
        rc = -EINVAL;
    if (rc < 0)
        return rc;
    bcp_task_set_xor_hook(s->hook, s->hook_ctx);
    return 0;
}
