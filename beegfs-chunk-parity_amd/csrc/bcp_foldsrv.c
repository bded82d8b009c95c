/*
 * bcp_foldsrv.c -- the node fold server.
 *
 * Rank processes that each start a HIP runtime put one context per rank on
 * the GPU (nine on one MI355X for config 5), and the device's queues, not the
 * fold, then set the rate.  With the server, the P roles'
 * window rows and outputs live in a shared arena and every fold goes to ONE
 * process that holds the GPU: one thread per connection reads a request
 * (rows, pitch, data bytes per row, output), registers the arena blocks it
 * has not seen, and folds through the fold service (bcp_fold.c: flat
 * combining, so windows of every rank share a launch); the reply carries the
 * fold's status.  Every request is answered before the next is read, so a
 * connection carries one window at a time: a rank's lanes share its
 * connections (lane tag modulo their number) under a per-connection mutex
 * held from request to reply.
 *
 * Two ways to reach it: a rank pool (bcp_pool.c) forks the server with the
 * socket world's arena mapped at the same address in every process; an
 * independent process (an MPI rank) connects to a server on a Unix socket
 * (bcp_fold_server_connect) and passes its arena as a memfd, which the
 * server maps once per client and translates addresses into.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include "bcp_fold.h"

#define FS_MAGIC 0x62636673u /* "bcfs" */
#define FS_MAX_CONN 64
#define FS_HOOK 1 /* the server folds with the test double it inherited (CPU tests; whole rows) */

typedef struct {
    uint32_t magic;
    int32_t n, st, flags;
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

/* ---- rank side -------------------------------------------------------------- */
static struct {
    int fd;
    pthread_mutex_t mu;
} g_srv[FS_MAX_CONN];
static int g_srv_n;
static uint64_t g_remote_folds;     /* windows folded by the server for this process */
static bcp_xor_hook_fn g_srv_hook; /* the test double the server inherited */

int bcpf_srv_attached(void)
{
    return g_srv_n > 0;
}

bcp_xor_hook_fn bcpf_srv_hook(void)
{
    return g_srv_hook;
}

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

void bcpi_foldsrv_attach(int nconn, const int *fds)
{
    void *ctx;
    bcpf_hook_get(&g_srv_hook, &ctx); /* the server was forked from the same state */
    g_srv_n = 0;
    for (int i = 0; i < nconn && i < FS_MAX_CONN; i++) {
        g_srv[i].fd = fds[i];
        pthread_mutex_init(&g_srv[i].mu, NULL);
        g_srv_n++;
    }
}

int bcpf_fold_remote(int st, int tag, const uint8_t *rows, size_t pitch, const size_t *valid, size_t nbytes, int n,
                     uint8_t *out, int with_hook)
{
    fs_req q = {FS_MAGIC, n, st, with_hook ? FS_HOOK : 0, (uint64_t)(uintptr_t)rows, pitch, nbytes,
                (uint64_t)(uintptr_t)out, 0, 0, 0, 0};
    void *rb, *ob;
    size_t rs, os;
    if (g_srv_n < 1 || n < 1 || n > MAX_STORAGE_TARGETS || !bcpi_arena_block(rows, &rb, &rs) ||
        !bcpi_arena_block(out, &ob, &os))
        return -ENXIO;
    q.rows_base = (uint64_t)(uintptr_t)rb;
    q.rows_size = rs;
    q.out_base = (uint64_t)(uintptr_t)ob;
    q.out_size = os;
    uint64_t v[MAX_STORAGE_TARGETS];
    for (int j = 0; j < n; j++)
        v[j] = valid[j];
    const int c = (tag < 0 ? -(tag + 1) : tag) % g_srv_n;
    fs_rep r = {FS_MAGIC, 0};
    pthread_mutex_lock(&g_srv[c].mu); /* request and reply: one window on the connection at a time */
    int rc = fs_io(g_srv[c].fd, &q, sizeof(q), 1);
    if (!rc)
        rc = fs_io(g_srv[c].fd, v, (size_t)n * sizeof(uint64_t), 1);
    if (!rc)
        rc = fs_io(g_srv[c].fd, &r, sizeof(r), 0);
    pthread_mutex_unlock(&g_srv[c].mu);
    if (!rc && r.magic != FS_MAGIC)
        rc = -EPROTO;
    if (!rc && !r.rc)
        __atomic_fetch_add(&g_remote_folds, 1, __ATOMIC_RELAXED);
    return rc ? rc : r.rc;
}

/* ---- server side ---------------------------------------------------------------- */
static struct {
    pthread_mutex_t mu;
    struct {
        uint8_t *p;
        size_t n;
    } reg[4096];
    int nreg;
} g_fs = {.mu = PTHREAD_MUTEX_INITIALIZER};

/* A client's arena as this server sees it: the rank pool's is mapped at the
 * same address in every process (delta 0); a connected client's memfd is
 * mapped here at base, its own at client_base. */
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

/* Register an arena block with the device once.  Arena blocks never move or
 * change size (bcpi_arena_alloc: a block keeps its place and size class for
 * the arena's lifetime), so a registration keyed by (base, size) stays valid
 * while its mapping lives: the rank pool's arena outlives the server, a
 * connected client's is unregistered before it is unmapped (fs_map_put). */
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

/* The last connection of a client is gone -- every fold it asked for was
 * answered, so none is in flight: unregister its blocks, unmap. */
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
    bcp_engine *e = bcpf_any_engine();
    for (int i = 0; i < g_fs.nreg;)
        if (g_fs.reg[i].p >= m->base && g_fs.reg[i].p < m->base + m->size) {
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

/* The server folds through its device's resident ring when its own
 * settings say so (PIPELINED with the ring on), else through the fold
 * service. */
static int srv_use_ring(void)
{
    bcpi_settings s;
    bcpi_settings_get(&s);
    return s.fold_mode == BCP_FOLD_PIPELINED && s.fold_ring;
}

static void fs_serve_conn(fs_conn *c)
{
    const int fd = c->fd;
    for (;;) {
        fs_req q;
        if (fs_io(fd, &q, sizeof(q), 0))
            break; /* the rank closed its end */
        uint64_t v[MAX_STORAGE_TARGETS];
        size_t valid[MAX_STORAGE_TARGETS];
        fs_rep r = {FS_MAGIC, 0};
        if (q.magic != FS_MAGIC || q.n < 1 || q.n > MAX_STORAGE_TARGETS || (q.flags & ~FS_HOOK))
            break; /* out of step: drop the connection (the rank sees EPIPE) */
        if (fs_io(fd, v, (size_t)q.n * sizeof(uint64_t), 0))
            break;
        if (bcpi_inject_hit(BCP_INJECT_FOLD_SERVER))
            break; /* (failure injection) the rank's fold sees EPIPE */
        const int hooked = (q.flags & FS_HOOK) != 0;
        int ok = fs_block_ok(c, q.out_base, q.out_size, q.out, q.nbytes) && q.pitch > 0 && q.nbytes <= q.pitch;
        for (int j = 0; j < q.n && ok; j++) {
            valid[j] = (size_t)v[j];
            ok = v[j] <= q.pitch &&
                 fs_block_ok(c, q.rows_base, q.rows_size, q.rows + (uint64_t)j * q.pitch, hooked ? q.nbytes : v[j]);
        }
        /* client addresses -> this process's */
        q.rows += (uint64_t)c->delta;
        q.out += (uint64_t)c->delta;
        q.rows_base += (uint64_t)c->delta;
        q.out_base += (uint64_t)c->delta;
        bcp_engine *e = NULL;
        int dev = -1;
        bcp_xor_hook_fn hook = NULL;
        void *hctx = NULL;
        if (hooked)
            bcpf_hook_get(&hook, &hctx);
        if (!ok)
            r.rc = -EFAULT;
        else if (q.nbytes == 0)
            r.rc = 0;
        else if (hooked)
            r.rc = hook ? hook((uint8_t *)(uintptr_t)q.out, (size_t)q.nbytes, (const uint8_t *)(uintptr_t)q.rows,
                               (size_t)q.pitch, q.n, hctx)
                        : -ENOSYS;
        else if (!(r.rc = bcpf_engine_for_target(q.st, &e, &dev)) && !(r.rc = fs_register(e, q.rows_base, q.rows_size)) &&
                 !(r.rc = fs_register(e, q.out_base, q.out_size)))
            /* the server's own settings: the ring when PIPELINED with the
             * ring on, else the fold service */
            r.rc = bcpf_fold_device(dev, e, srv_use_ring(), (const uint8_t *)(uintptr_t)q.rows, (size_t)q.pitch, valid,
                                    (size_t)q.nbytes, q.n, (uint8_t *)(uintptr_t)q.out);
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

/* batches in flight at once (the fold service's width; every rank's windows
 * share it): environment BCP_FOLD_SERVER_INFLIGHT, read once at start-up */
static void server_inflight_from_env(void)
{
    const char *v = getenv("BCP_FOLD_SERVER_INFLIGHT");
    if (v)
        (void)bcp_task_set_fold_inflight(atoi(v));
}

int bcpi_foldsrv_main(int nconn, const int *fds, void *arena_lo, void *arena_hi)
{
    server_inflight_from_env();
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

/* ---- independent processes (an MPI job) over a Unix socket -------------------
 * A rank (bcp_fold_server_connect) sends, on each of its connections, a hello
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
    server_inflight_from_env();
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
    const fs_hello h = {FS_HELLO, 0, ((uint64_t)getpid() << 32) ^ (uint64_t)ts.tv_nsec, (uint64_t)(uintptr_t)base,
                        arena_bytes};
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
    bcpi_foldsrv_attach(made, fds);     /* (a test double set now is asked of the server too: FS_HOOK) */
    return 0;
}
