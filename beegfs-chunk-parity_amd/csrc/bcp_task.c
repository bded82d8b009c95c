/*
 * bcp_task.c -- the per-rank chunk-streaming protocol (process_task) with the
 * P role's fold on the GPU.
 *
 * Follows the reference's roles and message flow
 * (src/beegfs-raid5/common/task_processing.c):
 *   process_task      :325-340  dispatch by role
 *   parity_generator  :117-245  P role: sizes -> max_cs -> windows -> parity
 *   chunk_sender      :247-322  source role: size -> windows (zero padded)
 * over the loopback transport (bcp_loopback.c) instead of MPI.  The window
 * fold (xor_parity at :211) becomes one XOR kernel on the lane's own HIP
 * queue that reads the pinned window rows (256-byte pitch, so every row is
 * 16-byte aligned for the fast kernel) and writes the pinned parity block in
 * place over PCIe (zero copy; the staged H2D -> kernel -> D2H form is kept as
 * bcp_task_set_fold_mode(BCP_FOLD_STAGED)).  Twelve lanes per rank keep
 * twelve queues of folds in flight on the device.
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
#include <unistd.h>

#include "bcp_task.h"

#define WINDOW ((uint64_t)BCP_WINDOW_BYTES)
#define ROW_ALIGN 256u
#define MAX_DEVICES 64

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

/* ---- engines / device map / test hook ---------------------------------- */
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static bcp_engine *g_engines[MAX_DEVICES];
static int g_engine_rc[MAX_DEVICES];
static int g_devmap[MAX_STORAGE_TARGETS];
static int g_devmap_n = 0;
static bcp_xor_hook_fn g_hook = NULL;
static void *g_hook_ctx = NULL;
static int g_fold_mode = BCP_FOLD_ZERO_COPY;

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
    if (mode != BCP_FOLD_ZERO_COPY && mode != BCP_FOLD_STAGED)
        return -EINVAL;
    pthread_mutex_lock(&g_lock);
    int prev = g_fold_mode;
    g_fold_mode = mode;
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

/* ---- fold resources: a shared pool, reused across tasks, lanes and runs --
 * One resource = one HIP queue + pinned window rows + device buffers.  The P
 * role takes one for the duration of a task and gives it back, so a
 * long-running rank pays queue creation and page pinning once, not per task
 * or per lane thread.  Host-only resources (test hook) use plain memory. */
typedef struct fold_res {
    struct fold_res *next;
    int device;         /* -1: host-only (hook) */
    bcp_engine *eng;
    bcp_queue *q;
    uint8_t *h_win[2];  /* window rows [n][pitch] (pinned when device >= 0) */
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
    if (R->device >= 0)
        bcp_host_free(R->eng, p);
    else
        free(p);
}

static void res_destroy(fold_res *R)
{
    host_free(R, R->h_win[0]);
    host_free(R, R->h_win[1]);
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

static int grow(fold_res *R, uint8_t **p, size_t *cap, size_t need)
{
    if (*cap >= need && *p)
        return 0;
    host_free(R, *p);
    *p = NULL;
    *cap = 0;
    size_t c = MAX_(need, (size_t)1 << 20);
    int rc = 0;
    if (R->device >= 0)
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
 * rows and an nbytes fold output.  use_gpu = 0 under the test hook. */
static int res_acquire(HostState *hs, int use_gpu, size_t rows_bytes, size_t nbytes, fold_res **out)
{
    int rc = 0, dev = -1;
    bcp_engine *e = NULL;
    *out = NULL;
    if (use_gpu && (rc = engine_for_target(hs->storage_target, &e, &dev)))
        return rc;
    /* prefer a free resource of the same device that is already big enough */
    pthread_mutex_lock(&g_lock);
    fold_res **best = NULL;
    for (fold_res **pp = &g_pool; *pp; pp = &(*pp)->next) {
        if ((*pp)->device != dev)
            continue;
        if (!best)
            best = pp;
        if ((*pp)->h_cap >= rows_bytes && (*pp)->h_cap1 >= rows_bytes && (*pp)->hp_cap >= nbytes) {
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
        if (use_gpu && (rc = bcp_queue_create(e, &R->q))) {
            free(R);
            return rc;
        }
    }
    if ((rc = grow(R, &R->h_win[0], &R->h_cap, rows_bytes)) || (rc = grow(R, &R->h_win[1], &R->h_cap1, rows_bytes)) ||
        (rc = grow(R, &R->h_par, &R->hp_cap, nbytes)))
        goto fail;
    *out = R;
    return 0;
fail:
    res_destroy(R);
    return rc;
}

/* The fold of one window (replaces xor_parity at task_processing.c:211):
 * out = XOR of n rows of `pitch` bytes, nbytes each. */
static int fold_window(fold_res *R, HostState *hs, bcp_xor_hook_fn hook, void *ctx, const uint8_t *rows,
                       size_t pitch, size_t nbytes, int n, uint8_t *out)
{
    if (hook) {
        static int warned = 0; /* lanes race here: atomic exchange */
        if (!__atomic_exchange_n(&warned, 1, __ATOMIC_RELAXED))
            LOGERR("XOR test hook active on st %d (no GPU fold)\n", hs->storage_target);
        return hook(out, nbytes, rows, pitch, n, ctx);
    }
    int rc;
    pthread_mutex_lock(&g_lock);
    const int mode = g_fold_mode;
    pthread_mutex_unlock(&g_lock);
    if (mode == BCP_FOLD_ZERO_COPY) {
        /* rows and out are mapped pinned memory (grow): the kernel streams
         * them over PCIe, no copy commands */
        if ((rc = bcp_xor_strided_async(R->q, out, pitch, rows, pitch * (size_t)n, pitch, 1, (uint32_t)n, nbytes)))
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

/* ---- roles ------------------------------------------------------------- */

static void parity_generator(const char *path, const FileInfo *task, TaskInfo ti, HostState *hs)
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

    bcp_lb_req *req[MAX_STORAGE_TARGETS];
    uint64_t chunk_sizes[MAX_STORAGE_TARGETS] = {0};
    if (ti.is_rebuilding) {
        bcp_lb_recv(chunk_sizes, (size_t)n * sizeof(uint64_t), st2rank[ti.actual_P_st], ti.tag, NULL);
    } else {
        for (int j = 0; j < n; j++)
            bcp_lb_irecv(&chunk_sizes[j], sizeof(uint64_t), ranks[j], ti.tag, &req[j]);
        bcp_lb_waitall(n, req);
    }

    uint64_t max_cs = 0;
    for (int j = 0; j < n; j++)
        max_cs = MAX_(max_cs, chunk_sizes[j]);
    for (int j = 0; j < n; j++)
        bcp_lb_isend(&max_cs, sizeof(max_cs), ranks[j], ti.tag, &req[j]);
    bcp_lb_waitall(n, req);

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
    pthread_mutex_unlock(&g_lock);

    fold_res *L = NULL;
    int have_had_error = __atomic_load_n(&hs->error, __ATOMIC_ACQUIRE);
    int res_rc = expected_messages ? res_acquire(hs, hook == NULL, pitch * (size_t)n, buffer_size, &L) : 0;
    uint8_t *scratch = NULL; /* receive space if staging could not be set up */
    uint8_t *win_a, *win_b, *pblk;
    if (res_rc) {
        LOGERR("no parity engine for '%s' on st %d: %s\n", path, hs->storage_target, bcp_strerror(res_rc));
        if (!have_had_error)
            have_had_error = res_rc == -ENODEV ? ENODEV : (res_rc == -ENOMEM ? ENOMEM : EIO);
        scratch = malloc(2 * pitch * (size_t)n + buffer_size + 1);
        if (!scratch)
            abort(); /* cannot even drain the senders */
        win_a = scratch;
        win_b = scratch + pitch * (size_t)n;
        pblk = scratch + 2 * pitch * (size_t)n;
    } else if (expected_messages) {
        win_a = L->h_win[0];
        win_b = L->h_win[1];
        pblk = L->h_par;
    } else {
        win_a = win_b = pblk = NULL; /* header-only parity chunk */
    }

    int P_fd = hs->fd_null;
    if (have_had_error == 0) {
        P_fd = open_new_parity(hs->write_dir, path, (off_t)final_size);
        if (P_fd <= 0) {
            have_had_error = errno;
            LOGERR("opened parity chunk '%s' with error = '%s'\n", path, strerror(errno));
            P_fd = hs->fd_null;
        }
    } else {
        LOGERR("using null for '%s', we already have global errno %d\n", path, have_had_error);
    }

    /* gen: the chunk sizes head the parity chunk (:199-201) */
    if (!ti.is_rebuilding)
        if (write(P_fd, chunk_sizes, sizeof(uint64_t) * (size_t)n) <= 0)
            have_had_error = errno;

    for (uint64_t msg_i = 0; msg_i < expected_messages; msg_i++) {
        if (msg_i == 0)
            for (int j = 0; j < n; j++)
                bcp_lb_irecv(win_a + (size_t)j * pitch, buffer_size, ranks[j], ti.tag, &req[j]);
        bcp_lb_waitall(n, req);
        if (msg_i + 1 != expected_messages)
            for (int j = 0; j < n; j++)
                bcp_lb_irecv(win_b + (size_t)j * pitch, buffer_size, ranks[j], ti.tag, &req[j]);
        /* fold window msg_i on the GPU while the senders fill win_b */
        if (!have_had_error) {
            int frc = fold_window(L, hs, hook, hook_ctx, win_a, pitch, buffer_size, n, pblk);
            if (frc) {
                have_had_error = EIO;
                LOGERR("GPU fold of '%s' failed: %s\n", path, bcp_strerror(frc));
            }
        }
        if (!have_had_error) {
            size_t wsize = (size_t)MIN_((uint64_t)buffer_size, data_left);
            ssize_t w = write(P_fd, pblk, wsize);
            if (w <= 0) {
                have_had_error = errno;
                LOGERR("writing '%s' caused new error %d (%s) after %llu bytes\n", path, errno, strerror(errno),
                       (unsigned long long)(final_size - data_left));
            }
            data_left -= wsize;
        }
        if (ti.sample)
            ti.sample->bytes_written += buffer_size;
        uint8_t *t = win_a;
        win_a = win_b;
        win_b = t;
    }

    if (ti.is_rebuilding && P_fd != hs->fd_null)
        if (ftruncate(P_fd, (off_t)final_parity_chunk_size) != 0 && !have_had_error)
            have_had_error = errno;

    if (have_had_error != 0 && raise_sticky_error(hs, have_had_error, path))
        LOGERR("local error on '%s' elevated to global error\n", path);
    free(scratch);
    res_release(L);
    if (P_fd != hs->fd_null)
        close(P_fd);
}

static uint8_t *sender_buffer(size_t need)
{
    lane_res *L = &t_res;
    if (L->send_cap < need || !L->send_buf) {
        free(L->send_buf);
        L->send_cap = MAX_(need, (size_t)1 << 20);
        L->send_buf = malloc(L->send_cap);
        if (!L->send_buf)
            L->send_cap = 0;
    }
    return L->send_buf;
}

/* One window of the source role, produced straight into the receiver's
 * buffer (bcp_lb_send_fill): the file's next bytes, zero padded after a short
 * read; zeros after an open or read error or for an empty chunk (A3-q2). */
typedef struct {
    int fd;
    uint64_t fd_size, data_to_send, data_sent;
    int err;
    HostState *hs;
    const char *path;
} window_fill;

static int fill_window(void *ctx, void *dst, size_t n)
{
    window_fill *w = ctx;
    HostState *hs = w->hs;
    uint8_t *data = dst;
    if (w->err != 0 || w->data_sent >= w->fd_size) {
        memset(data, 0, n);
        return 0;
    }
    const uint64_t left = w->data_to_send - w->data_sent;
    ssize_t r = read(w->fd, data, (size_t)MIN_((uint64_t)n, left));
    if (r < 0) {
        w->err = errno;
        memset(data, 0, n);
        LOGERR("reading '%s' caused new error %d (%s) after %llu bytes\n", w->path, errno, strerror(errno),
               (unsigned long long)w->data_sent);
        return 0;
    }
    if ((size_t)r < n)
        memset(data + r, 0, n - (size_t)r);
    return 0;
}

static void chunk_sender(const char *path, const FileInfo *task, TaskInfo ti, HostState *hs)
{
    const int my_st = hs->storage_target;
    const int coordinator = st2rank[GET_P(task->locations)];
    const int ntargets = active_ranks(task->locations);
    uint64_t fd_size = 0;
    int have_had_error = 0;
    int fd = open_chunk_readonly(ti.read_dir, path);
    if (fd <= 0) {
        have_had_error = errno;
        fd = hs->fd_zero;
        LOGERR("opening '%s' caused new error %d (%s)\n", path, errno, strerror(errno));
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
        bcp_lb_send(chunk_sizes, (size_t)ntargets * sizeof(uint64_t), coordinator, ti.tag);
    } else if (!ti.is_rebuilding) {
        bcp_lb_send(&fd_size, sizeof(fd_size), coordinator, ti.tag);
    }

    uint64_t data_to_send = 0;
    bcp_lb_recv(&data_to_send, sizeof(data_to_send), coordinator, ti.tag, NULL);

    const size_t buffer_size = (size_t)MIN_(WINDOW, data_to_send);
    /* Zero copy: every window is read straight into P's window row, unless a
     * later window could replay this one (A3-q1: the file ends before max_cs
     * and more than one window is sent), which needs the sender's own buffer. */
    if (!(fd_size < data_to_send && data_to_send > buffer_size)) {
        window_fill wf = {fd, fd_size, data_to_send, 0, have_had_error, hs, path};
        while (wf.data_sent < data_to_send) {
            if (ti.sample)
                ti.sample->bytes_read += buffer_size;
            bcp_lb_send_fill(fill_window, &wf, buffer_size, coordinator, ti.tag);
            wf.data_sent += buffer_size;
        }
        have_had_error = wf.err;
        goto done;
    }
    uint8_t *data = sender_buffer(buffer_size);
    if (!data)
        abort();
    /* A buffer that is never filled is sent as zeros: the reference sends
     * uninitialised memory for a zero-length chunk (quirk A3-q2). */
    if (have_had_error != 0 || fd_size == 0)
        memset(data, 0, buffer_size);

    uint64_t data_sent = 0;
    while (data_sent < data_to_send) {
        uint64_t left = data_to_send - data_sent;
        /* once the file is exhausted the previous window is re-sent (A3-q1) */
        if (have_had_error == 0 && data_sent < fd_size) {
            ssize_t r = read(fd, data, (size_t)MIN_((uint64_t)buffer_size, left));
            if (r < 0) {
                have_had_error = errno;
                memset(data, 0, buffer_size);
                LOGERR("reading '%s' caused new error %d (%s) after %llu bytes\n", path, errno, strerror(errno),
                       (unsigned long long)data_sent);
            }
            if (r >= 0 && (size_t)r < buffer_size)
                memset(data + r, 0, buffer_size - (size_t)r);
        }
        if (ti.sample)
            ti.sample->bytes_read += buffer_size;
        data_sent += buffer_size;
        bcp_lb_send(data, buffer_size, coordinator, ti.tag);
    }

done:
    /* ENOENT: the chunk vanished after planning; an unlink event follows. */
    if (have_had_error != 0 && have_had_error != ENOENT && raise_sticky_error(hs, have_had_error, path))
        LOGERR("local error on '%s' elevated to global error\n", path);
    if (fd != hs->fd_zero)
        close(fd);
}

int process_task(HostState *hs, const char *path, const FileInfo *fi, TaskInfo ti)
{
    assert(GET_P(fi->locations) != (int)NO_P);
    assert(P_IS_INVALID(fi->locations) == 0);
    assert(hs->storage_target >= 0);

    if (GET_P(fi->locations) == hs->storage_target)
        parity_generator(path, fi, ti, hs);
    else if (TEST_BIT(fi->locations, hs->storage_target))
        chunk_sender(path, fi, ti, hs);
    else
        return 0;
    return active_ranks(fi->locations) != 0;
}
