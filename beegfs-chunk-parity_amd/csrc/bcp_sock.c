/*
 * bcp_sock.c -- the transport for ranks that are PROCESSES (bcp_sock_world).
 *
 * The reference's ranks are MPI processes (one per storage target,
 * src/beegfs-parity-gen:114-127) and process_task speaks the point-to-point
 * subset of task_processing.c:43-52,120-130,151-166,203-209,274-307.  Here a
 * world of N ranks is N*(N-1)/2 Unix socketpairs created before fork; each
 * rank process keeps its N-1 ends.  Messages are framed {magic, tag, len} +
 * payload, so per (source, destination) the byte stream is the message order
 * and MPI's non-overtaking rule per (source, destination, tag) holds.
 *
 * Progress without a progress thread: a thread waiting for a receive from
 * source s becomes the reader of s's socket if nobody else is.  It reads one
 * frame header, and the payload goes straight into the oldest posted receive
 * with that (source, tag) if there is one, else into an unexpected-message
 * buffer that a later receive takes (the match is re-checked under the lock
 * after the payload is in, so a receive posted meanwhile is never missed).
 * The other waiters on that socket sleep on their own request's condition
 * variable in a per-(source, socket) queue: a completed request wakes only
 * its owner, and a reader whose own request completes hands the reading to
 * the oldest waiter left (no broadcast to every lane of the rank per frame).
 * Sends write the frame under a per-destination lock (the lanes of a rank
 * share its sockets).  Writes block only on a full socket buffer, which the
 * destination drains as soon as any of its threads waits on us -- the MPI
 * rendezvous contract the protocol is written for.
 *
 * Fill sends (send_fill, the source role's windows): the world maps a
 * shared row arena before fork, one slice per rank, and a rank's P role
 * takes its window rows from its slice (bcpi_arena_alloc).  A fill send is
 * a rendezvous: RTS {tag, n} to the receiver; whoever matches it with a
 * posted receive answers CTS {address, capacity} when the receive buffer
 * lies in the arena (else address 0: the sender falls back to an ordinary
 * message); the sender runs fill() straight into that address -- read() of
 * the chunk file into the P role's row, one copy instead of three (file ->
 * buffer -> socket -> row) -- and sends DONE {n}, which completes the
 * receive.  CTS travels on a second, control socketpair: the thread that
 * answers may be the reader of the data socket, which must never block on
 * a write (two readers blocked writing into full data sockets would wait
 * for each other); at most one CTS per blocked fill sender is ever in
 * flight, so a control socket never fills.  Environment BCP_SOCK_ARENA_MB (per rank; default 2048, 0 = no
 * arena and no fill sends).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <unistd.h>

#include "bcp_host.h"
#include "bcp_task.h"

#define FRAME_MAGIC 0x62637066u /* "bcpf": a message */
#define FRAME_RTS 0x62637072u   /* "bcpr": fill send of len bytes wants a receive */
#define FRAME_CTS 0x62637063u   /* "bcpc": {address, capacity} of the matched receive */
#define FRAME_DONE 0x62637064u  /* "bcpd": {bytes} filled; completes the receive */

typedef struct {
    uint32_t magic;
    int32_t tag;
    uint64_t len;
} frame_hdr;

typedef struct sk_msg {
    struct sk_msg *next;
    int src, tag;
    size_t n;
    uint8_t *data;
    int rts; /* an unmatched fill send of n bytes (no data) */
} sk_msg;

typedef struct sk_req {
    struct sk_req *next;
    int src, tag;
    void *buf;
    size_t cap, received;
    int status;
    int done;
    uint64_t cts_addr, cts_cap; /* fill-send side: the receiver's answer */
    int ctl;                    /* waits on the control socket (a fill send's CTS) */
    int busy;                   /* its payload is being read into buf by the socket's reader */
    pthread_cond_t cv;          /* its owner sleeps here (progress_until) */
    int queued;                 /* in the wait queue of (src, ctl) */
    struct sk_req *wnext;
} sk_req;

struct bcp_sock_world {
    int world, rank;      /* rank < 0 until attached */
    int *fds;             /* [world][world]: fds[a*world+b] = a's end towards b (-1 closed) */
    int *cfds;            /* the same for the control sockets (CTS) */
    pthread_mutex_t mu;
    sk_req **wq;              /* per (peer, socket): [2 * peer + ctl], waiters of that socket, oldest first */
    pthread_mutex_t *send_mu; /* per peer */
    pthread_mutex_t *ctl_mu;  /* per peer: control-socket writes */
    int *reading;             /* per peer: a thread is reading that socket */
    int *reading_ctl;         /* per peer: ... that control socket */
    int *dead;                /* per peer: socket failed / closed (errno) */
    sk_req *posted_head, *posted_tail;
    sk_msg *unexp_head, *unexp_tail;
    sk_req *filling; /* receives matched to a fill send, waiting for DONE */
    sk_req *cts_wait; /* fill sends waiting for CTS (src = destination) */
    uint8_t *arena;   /* shared row arena: world slices of `slice` bytes */
    size_t slice;
};

/* This process's arena slice (set by bcp_sock_world_attach). */
#define ARENA_MAX_BLOCKS 4096
static pthread_mutex_t g_arena_mu = PTHREAD_MUTEX_INITIALIZER;
static uint8_t *g_arena_lo, *g_arena_hi; /* the whole arena: CTS addresses are checked against it */
static uint8_t *g_slice;
static size_t g_slice_bytes, g_slice_used;
static struct {
    uint8_t *p;
    size_t n;
    int used;
} g_blocks[ARENA_MAX_BLOCKS];
static int g_nblocks;

void *bcpi_arena_alloc(size_t bytes, size_t *got)
{
    size_t c = (size_t)2 << 20; /* 2 MiB classes: blocks stay 2 MiB aligned in the slice */
    while (c < bytes)
        c <<= 1;
    void *p = NULL;
    pthread_mutex_lock(&g_arena_mu);
    if (g_slice) {
        for (int i = 0; i < g_nblocks && !p; i++)
            if (!g_blocks[i].used && g_blocks[i].n == c) {
                g_blocks[i].used = 1;
                p = g_blocks[i].p;
            }
        if (!p && g_nblocks < ARENA_MAX_BLOCKS && g_slice_used + c <= g_slice_bytes) {
            p = g_slice + g_slice_used;
            g_slice_used += c;
            g_blocks[g_nblocks].p = p;
            g_blocks[g_nblocks].n = c;
            g_blocks[g_nblocks].used = 1;
            g_nblocks++;
        }
    }
    pthread_mutex_unlock(&g_arena_mu);
    if (p && got)
        *got = c;
    return p;
}

int bcpi_arena_free(void *p)
{
    int found = 0;
    pthread_mutex_lock(&g_arena_mu);
    for (int i = 0; i < g_nblocks && !found; i++)
        if (g_blocks[i].p == p && g_blocks[i].used) {
            g_blocks[i].used = 0;
            found = 1;
        }
    pthread_mutex_unlock(&g_arena_mu);
    return found;
}

void bcpi_arena_set(void *base, size_t bytes)
{
    pthread_mutex_lock(&g_arena_mu);
    g_arena_lo = base;
    g_arena_hi = (uint8_t *)base + bytes;
    g_slice = base;
    g_slice_bytes = bytes;
    g_slice_used = 0;
    g_nblocks = 0;
    pthread_mutex_unlock(&g_arena_mu);
}

int bcpi_arena_block(const void *p, void **base, size_t *size)
{
    const uint8_t *b = p;
    int found = 0;
    pthread_mutex_lock(&g_arena_mu);
    for (int i = 0; i < g_nblocks && !found; i++)
        if (g_blocks[i].used && b >= g_blocks[i].p && b < g_blocks[i].p + g_blocks[i].n) {
            *base = g_blocks[i].p;
            *size = g_blocks[i].n;
            found = 1;
        }
    pthread_mutex_unlock(&g_arena_mu);
    return found;
}

void bcpi_sock_world_close_fds(bcp_sock_world *w)
{
    for (int i = 0; w && i < w->world * w->world; i++) {
        if (w->fds[i] >= 0)
            close(w->fds[i]);
        if (w->cfds[i] >= 0)
            close(w->cfds[i]);
        w->fds[i] = w->cfds[i] = -1;
    }
}

int bcpi_sock_world_arena(const bcp_sock_world *w, void **lo, void **hi)
{
    if (!w || !w->arena)
        return 0;
    *lo = w->arena;
    *hi = w->arena + w->slice * (size_t)w->world;
    return 1;
}

static uint64_t g_fill_arena, g_fill_msg; /* fill sends into an arena row / as a message */

void bcpi_sock_fill_counts(uint64_t *arena, uint64_t *msg)
{
    *arena = __atomic_load_n(&g_fill_arena, __ATOMIC_RELAXED);
    *msg = __atomic_load_n(&g_fill_msg, __ATOMIC_RELAXED);
}

static int in_arena(const void *p, size_t n)
{
    const uint8_t *b = p;
    return g_arena_lo && b >= g_arena_lo && b <= g_arena_hi && n <= (size_t)(g_arena_hi - b);
}

static sk_req g_sent; /* the completed request every isend returns (eager) */

/* 2 * world * (world - 1) socket ends exist before fork (data + control): 57
 * ranks need ~6,400 descriptors, beyond the usual soft limit of 1,024.  The
 * soft limit is raised (no privilege needed) only as far as the worlds alive
 * need -- their ends plus headroom for the caller's own -- and the caller's
 * limit is restored when the last world is destroyed. */
static pthread_mutex_t g_nofile_mu = PTHREAD_MUTEX_INITIALIZER;
static int g_nofile_worlds;
static size_t g_nofile_need;
static struct rlimit g_nofile_saved;
static int g_nofile_raised;

static void nofile_raise(size_t ends)
{
    pthread_mutex_lock(&g_nofile_mu);
    struct rlimit rl;
    if (g_nofile_worlds++ == 0) {
        g_nofile_need = 0;
        g_nofile_raised = getrlimit(RLIMIT_NOFILE, &g_nofile_saved) == 0;
    }
    g_nofile_need += ends;
    if (g_nofile_raised && getrlimit(RLIMIT_NOFILE, &rl) == 0) {
        const rlim_t want = (rlim_t)(g_nofile_saved.rlim_cur + g_nofile_need + 256);
        if (rl.rlim_cur < want) {
            rl.rlim_cur = want < rl.rlim_max ? want : rl.rlim_max;
            (void)setrlimit(RLIMIT_NOFILE, &rl);
        }
    }
    pthread_mutex_unlock(&g_nofile_mu);
}

static void nofile_release(size_t ends)
{
    pthread_mutex_lock(&g_nofile_mu);
    g_nofile_need -= ends < g_nofile_need ? ends : g_nofile_need;
    if (--g_nofile_worlds == 0 && g_nofile_raised) {
        struct rlimit rl;
        if (getrlimit(RLIMIT_NOFILE, &rl) == 0) {
            rl.rlim_cur = g_nofile_saved.rlim_cur;
            (void)setrlimit(RLIMIT_NOFILE, &rl);
        }
        g_nofile_raised = 0;
    }
    pthread_mutex_unlock(&g_nofile_mu);
}

int bcp_sock_world_create(int world_size, bcp_sock_world **out)
{
    if (!out || world_size < 1 || world_size > 4096)
        return -EINVAL;
    *out = NULL;
    bcp_sock_world *w = calloc(1, sizeof(*w));
    if (!w)
        return -ENOMEM;
    /* from here every failure goes through bcp_sock_world_destroy, which releases it */
    nofile_raise((size_t)2 * (size_t)world_size * (size_t)(world_size - 1));
    w->world = world_size;
    w->rank = -1;
    w->fds = malloc((size_t)world_size * (size_t)world_size * sizeof(int));
    w->cfds = malloc((size_t)world_size * (size_t)world_size * sizeof(int));
    w->send_mu = calloc((size_t)world_size, sizeof(pthread_mutex_t));
    w->ctl_mu = calloc((size_t)world_size, sizeof(pthread_mutex_t));
    w->reading = calloc((size_t)world_size, sizeof(int));
    w->reading_ctl = calloc((size_t)world_size, sizeof(int));
    w->dead = calloc((size_t)world_size, sizeof(int));
    w->wq = calloc((size_t)world_size * 2, sizeof(sk_req *));
    if (!w->fds || !w->cfds || !w->send_mu || !w->ctl_mu || !w->reading || !w->reading_ctl || !w->dead || !w->wq) {
        if (w->fds)
            for (int i = 0; i < world_size * world_size; i++)
                w->fds[i] = -1;
        if (w->cfds)
            for (int i = 0; i < world_size * world_size; i++)
                w->cfds[i] = -1;
        bcp_sock_world_destroy(w);
        return -ENOMEM;
    }
    for (int i = 0; i < world_size * world_size; i++)
        w->fds[i] = w->cfds[i] = -1;
    size_t mb = 2048;
    if (getenv("BCP_SOCK_ARENA_MB"))
        mb = (size_t)strtoull(getenv("BCP_SOCK_ARENA_MB"), NULL, 10);
    if (mb) {
        /* address space only: pages exist once a P role touches its rows */
        const size_t slice = mb << 20;
        void *a = mmap(NULL, slice * (size_t)world_size, PROT_READ | PROT_WRITE,
                       MAP_SHARED | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
        if (a != MAP_FAILED) {
            w->arena = a;
            w->slice = slice;
        }
    }
    pthread_mutex_init(&w->mu, NULL);
    for (int i = 0; i < world_size; i++) {
        pthread_mutex_init(&w->send_mu[i], NULL);
        pthread_mutex_init(&w->ctl_mu[i], NULL);
    }
    for (int a = 0; a < world_size; a++)
        for (int b = a + 1; b < world_size; b++) {
            int sv[2], cv[2];
            if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, sv) != 0) {
                int e = -errno;
                bcp_sock_world_destroy(w);
                return e;
            }
            int sz = 4 << 20; /* room for a few 512 KiB windows in flight per pair */
            setsockopt(sv[0], SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
            setsockopt(sv[1], SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
            w->fds[a * world_size + b] = sv[0];
            w->fds[b * world_size + a] = sv[1];
            if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, cv) != 0) {
                int e = -errno;
                bcp_sock_world_destroy(w);
                return e;
            }
            w->cfds[a * world_size + b] = cv[0];
            w->cfds[b * world_size + a] = cv[1];
        }
    *out = w;
    return 0;
}

int bcp_sock_world_destroy(bcp_sock_world *w)
{
    if (!w)
        return -EINVAL;
    for (int i = 0; i < w->world * w->world; i++) {
        if (w->fds && w->fds[i] >= 0)
            close(w->fds[i]);
        if (w->cfds && w->cfds[i] >= 0)
            close(w->cfds[i]);
    }
    for (sk_msg *m = w->unexp_head; m;) {
        sk_msg *nx = m->next;
        free(m->data);
        free(m);
        m = nx;
    }
    free(w->fds);
    free(w->cfds);
    nofile_release((size_t)2 * (size_t)w->world * (size_t)(w->world - 1));
    free(w->send_mu);
    free(w->ctl_mu);
    free(w->reading);
    free(w->reading_ctl);
    free(w->dead);
    free(w->wq);
    if (w->arena) {
        pthread_mutex_lock(&g_arena_mu);
        if (g_arena_lo == w->arena) {
            g_arena_lo = g_arena_hi = g_slice = NULL;
            g_slice_bytes = g_slice_used = 0;
            g_nblocks = 0;
        }
        pthread_mutex_unlock(&g_arena_mu);
        munmap(w->arena, w->slice * (size_t)w->world);
    }
    free(w);
    return 0;
}

/* ---- raw I/O ------------------------------------------------------------ */

static int write_all(int fd, const void *buf, size_t n)
{
    const uint8_t *p = buf;
    while (n) {
        ssize_t r = send(fd, p, n, MSG_NOSIGNAL);
        if (r < 0) {
            if (errno == EINTR)
                continue;
            return -errno;
        }
        p += r;
        n -= (size_t)r;
    }
    return 0;
}

static int read_all(int fd, void *buf, size_t n)
{
    uint8_t *p = buf;
    while (n) {
        ssize_t r = read(fd, p, n);
        if (r < 0) {
            if (errno == EINTR)
                continue;
            return -errno;
        }
        if (r == 0)
            return -EPIPE; /* peer process gone */
        p += r;
        n -= (size_t)r;
    }
    return 0;
}

/* Read and drop n bytes (the part of a message beyond a short receive). */
static int discard(int fd, size_t n)
{
    uint8_t tmp[4096];
    while (n) {
        size_t c = n < sizeof(tmp) ? n : sizeof(tmp);
        int rc = read_all(fd, tmp, c);
        if (rc)
            return rc;
        n -= c;
    }
    return 0;
}

static int peer_fd(bcp_sock_world *w, int peer)
{
    if (w->rank < 0 || peer < 0 || peer >= w->world || peer == w->rank)
        return -1;
    return w->fds[w->rank * w->world + peer];
}

/* ---- matching (under w->mu) ---------------------------------------------- */

static sk_req *take_posted(bcp_sock_world *w, int src, int tag)
{
    sk_req *prev = NULL;
    for (sk_req *r = w->posted_head; r; prev = r, r = r->next)
        if (r->src == src && r->tag == tag) {
            if (prev)
                prev->next = r->next;
            else
                w->posted_head = r->next;
            if (w->posted_tail == r)
                w->posted_tail = prev;
            r->next = NULL;
            return r;
        }
    return NULL;
}

/* Unlink r itself if it is still posted. */
static void remove_posted(bcp_sock_world *w, sk_req *r)
{
    sk_req *prev = NULL;
    for (sk_req *x = w->posted_head; x; prev = x, x = x->next)
        if (x == r) {
            if (prev)
                prev->next = x->next;
            else
                w->posted_head = x->next;
            if (w->posted_tail == x)
                w->posted_tail = prev;
            x->next = NULL;
            return;
        }
}

/* First request of an unordered list (filling / cts_wait) for (src, tag). */
static sk_req *take_list(sk_req **head, int src, int tag)
{
    for (sk_req **pp = head; *pp; pp = &(*pp)->next)
        if ((*pp)->src == src && (*pp)->tag == tag) {
            sk_req *r = *pp;
            *pp = r->next;
            r->next = NULL;
            return r;
        }
    return NULL;
}

static void push_list(sk_req **head, sk_req *r)
{
    sk_req **pp = head;
    while (*pp)
        pp = &(*pp)->next;
    r->next = NULL;
    *pp = r;
}

static void drop_list(sk_req **head, sk_req *r)
{
    for (sk_req **pp = head; *pp; pp = &(*pp)->next)
        if (*pp == r) {
            *pp = r->next;
            r->next = NULL;
            return;
        }
}

/* Unlink r from whichever list holds it (a failed peer's requests). */
static void unlink_req(bcp_sock_world *w, sk_req *r)
{
    remove_posted(w, r);
    drop_list(&w->filling, r);
    drop_list(&w->cts_wait, r);
}

static sk_msg *take_unexp(bcp_sock_world *w, int src, int tag)
{
    sk_msg *prev = NULL;
    for (sk_msg *m = w->unexp_head; m; prev = m, m = m->next)
        if (m->src == src && m->tag == tag) {
            if (prev)
                prev->next = m->next;
            else
                w->unexp_head = m->next;
            if (w->unexp_tail == m)
                w->unexp_tail = prev;
            m->next = NULL;
            return m;
        }
    return NULL;
}

static void deliver_msg(sk_req *r, sk_msg *m)
{
    size_t c = m->n <= r->cap ? m->n : r->cap;
    if (c)
        memcpy(r->buf, m->data, c);
    r->received = c;
    r->status = m->n <= r->cap ? 0 : -EMSGSIZE;
    r->done = 1;
    free(m->data);
    free(m);
}

/* ---- waiters (under w->mu) ------------------------------------------------ */

static void wq_push(bcp_sock_world *w, sk_req *r)
{
    if (r->queued)
        return;
    sk_req **pp = &w->wq[2 * r->src + r->ctl];
    while (*pp)
        pp = &(*pp)->wnext;
    r->wnext = NULL;
    *pp = r;
    r->queued = 1;
}

static void wq_remove(bcp_sock_world *w, sk_req *r)
{
    if (!r->queued)
        return;
    for (sk_req **pp = &w->wq[2 * r->src + r->ctl]; *pp; pp = &(*pp)->wnext)
        if (*pp == r) {
            *pp = r->wnext;
            break;
        }
    r->wnext = NULL;
    r->queued = 0;
}

/* r changed (completed, or its peer failed): its owner looks again. */
static void wake_req(bcp_sock_world *w, sk_req *r)
{
    wq_remove(w, r);
    pthread_cond_signal(&r->cv);
}

/* Every waiter of peer s (its sockets failed). */
static void wake_peer(bcp_sock_world *w, int s)
{
    for (int c = 0; c < 2; c++)
        while (w->wq[2 * s + c])
            wake_req(w, w->wq[2 * s + c]);
}

/* One frame {magic, tag, len} + payload to peer, under its send lock. */
static int send_frame(bcp_sock_world *w, int peer, uint32_t magic, int tag, uint64_t len, const void *pl,
                      size_t pn)
{
    const int fd = peer_fd(w, peer);
    if (fd < 0)
        return -EINVAL;
    frame_hdr h = {magic, tag, len};
    pthread_mutex_lock(&w->send_mu[peer]);
    int rc = write_all(fd, &h, sizeof(h));
    if (!rc && pn)
        rc = write_all(fd, pl, pn);
    pthread_mutex_unlock(&w->send_mu[peer]);
    return rc;
}

/* Answer a fill send from src: the receive's arena address, or 0 (send an
 * ordinary message instead). */
static int send_cts(bcp_sock_world *w, int src, int tag, const void *addr, size_t cap)
{
    if (w->rank < 0 || src < 0 || src >= w->world || src == w->rank)
        return -EINVAL;
    const int fd = w->cfds[w->rank * w->world + src];
    struct {
        frame_hdr h;
        uint64_t pl[2];
    } f = {{FRAME_CTS, tag, 2 * sizeof(uint64_t)},
           {(uint64_t)(uintptr_t)addr, (uint64_t)cap}};
    pthread_mutex_lock(&w->ctl_mu[src]);
    int rc = write_all(fd, &f, sizeof(f));
    pthread_mutex_unlock(&w->ctl_mu[src]);
    return rc;
}

/* One CTS from src's control socket (called by the thread holding
 * reading_ctl[src]). */
static int read_ctl_one(bcp_sock_world *w, int src)
{
    struct {
        frame_hdr h;
        uint64_t pl[2];
    } f;
    int rc = read_all(w->cfds[w->rank * w->world + src], &f, sizeof(f));
    if (rc)
        return rc;
    if (f.h.magic != FRAME_CTS || f.h.len != sizeof(f.pl))
        return -EPROTO;
    pthread_mutex_lock(&w->mu);
    sk_req *r = take_list(&w->cts_wait, src, f.h.tag);
    if (r) {
        r->cts_addr = f.pl[0];
        r->cts_cap = f.pl[1];
        r->status = 0;
        r->done = 1;
        wake_req(w, r);
    }
    pthread_mutex_unlock(&w->mu);
    return r ? 0 : -EPROTO;
}

/* The oldest posted receive for (src, tag), left posted. */
static sk_req *peek_posted(bcp_sock_world *w, int src, int tag)
{
    for (sk_req *r = w->posted_head; r; r = r->next)
        if (r->src == src && r->tag == tag)
            return r;
    return NULL;
}

/* Control frames of the fill-send rendezvous (RTS / CTS / DONE). */
static int read_control(bcp_sock_world *w, int src, const frame_hdr *h)
{
    const int fd = peer_fd(w, src);
    int rc = 0;
    if (h->magic == FRAME_RTS) {
        pthread_mutex_lock(&w->mu);
        sk_req *r = peek_posted(w, src, h->tag);
        const void *addr = NULL;
        size_t cap = 0;
        if (r && in_arena(r->buf, r->cap)) {
            remove_posted(w, r);
            push_list(&w->filling, r);
            addr = r->buf;
            cap = r->cap;
        } else if (!r) {
            /* no receive yet: the irecv that takes it answers */
            sk_msg *m = calloc(1, sizeof(*m));
            if (!m) {
                pthread_mutex_unlock(&w->mu);
                return -ENOMEM;
            }
            m->src = src;
            m->tag = h->tag;
            m->n = (size_t)h->len;
            m->rts = 1;
            if (w->unexp_tail)
                w->unexp_tail->next = m;
            else
                w->unexp_head = m;
            w->unexp_tail = m;
            pthread_mutex_unlock(&w->mu);
            return 0;
        }
        pthread_mutex_unlock(&w->mu);
        return send_cts(w, src, h->tag, addr, cap); /* addr 0: the data comes as a message */
    }
    if (h->magic == FRAME_DONE) {
        uint64_t n = 0;
        if (h->len != sizeof(n))
            return -EPROTO;
        if ((rc = read_all(fd, &n, sizeof(n))))
            return rc;
        pthread_mutex_lock(&w->mu);
        sk_req *r = take_list(&w->filling, src, h->tag);
        if (r) {
            r->received = n <= r->cap ? (size_t)n : r->cap;
            r->status = n <= r->cap ? 0 : -EMSGSIZE;
            r->done = 1;
            wake_req(w, r);
        }
        pthread_mutex_unlock(&w->mu);
        return r ? 0 : -EPROTO;
    }
    return -EPROTO;
}

/* One frame from src: straight into a posted receive, or buffered.  Called
 * by the thread holding reading[src], without the lock. */
static int read_one(bcp_sock_world *w, int src)
{
    const int fd = peer_fd(w, src);
    frame_hdr h;
    int rc = read_all(fd, &h, sizeof(h));
    if (rc)
        return rc;
    if (h.magic != FRAME_MAGIC)
        return read_control(w, src, &h);
    pthread_mutex_lock(&w->mu);
    sk_req *r = take_posted(w, src, h.tag);
    if (r)
        r->busy = 1; /* its waiter leaves it to us, even if the peer is failed meanwhile */
    pthread_mutex_unlock(&w->mu);
    if (r) {
        size_t c = h.len <= r->cap ? (size_t)h.len : r->cap;
        rc = c ? read_all(fd, r->buf, c) : 0;
        if (!rc && h.len > c)
            rc = discard(fd, (size_t)(h.len - c));
        pthread_mutex_lock(&w->mu);
        r->received = c;
        r->status = rc ? rc : (h.len <= r->cap ? 0 : -EMSGSIZE);
        r->busy = 0;
        r->done = 1;
        wake_req(w, r);
        pthread_mutex_unlock(&w->mu);
        return rc;
    }
    sk_msg *m = calloc(1, sizeof(*m));
    uint8_t *data = malloc(h.len ? (size_t)h.len : 1);
    if (!m || !data) {
        free(m);
        free(data);
        discard(fd, (size_t)h.len);
        return -ENOMEM;
    }
    if ((rc = h.len ? read_all(fd, data, (size_t)h.len) : 0)) {
        free(m);
        free(data);
        return rc;
    }
    m->src = src;
    m->tag = h.tag;
    m->n = (size_t)h.len;
    m->data = data;
    pthread_mutex_lock(&w->mu);
    /* a receive may have been posted while the payload came in */
    if ((r = take_posted(w, src, h.tag))) {
        deliver_msg(r, m);
        wake_req(w, r);
    } else {
        if (w->unexp_tail)
            w->unexp_tail->next = m;
        else
            w->unexp_head = m;
        w->unexp_tail = m;
    }
    pthread_mutex_unlock(&w->mu);
    return 0;
}

/* Block until r completes, reading r's source socket when nobody else is. */
static int progress_until(bcp_sock_world *w, sk_req *r)
{
    pthread_mutex_lock(&w->mu);
    while (!r->done) {
        const int s = r->src;
        if (w->dead[s] && !r->busy) {
            /* (a request whose payload the reader is still copying is left
             * to it: the peer can be failed by another thread -- a CTS that
             * could not be sent, sk_irecv -- while that copy runs) */
            unlink_req(w, r); /* so nobody completes it after it is freed */
            r->status = -w->dead[s];
            r->done = 1;
            break;
        }
        int *rd = r->ctl ? &w->reading_ctl[s] : &w->reading[s];
        if (*rd || r->busy) {
            /* another thread reads the socket (or r's payload): sleep until
             * r completes or the reading is handed over */
            wq_push(w, r);
            pthread_cond_wait(&r->cv, &w->mu);
            continue;
        }
        *rd = 1;
        pthread_mutex_unlock(&w->mu);
        int rc = r->ctl ? read_ctl_one(w, s) : read_one(w, s);
        pthread_mutex_lock(&w->mu);
        *rd = 0;
        if (rc && rc != -EMSGSIZE && rc != -ENOMEM) {
            w->dead[s] = -rc;
            wake_peer(w, s);
        } else if (r->done && w->wq[2 * s + r->ctl]) {
            /* leaving: the oldest waiter left becomes the reader */
            wake_req(w, w->wq[2 * s + r->ctl]);
        }
    }
    wq_remove(w, r);
    pthread_mutex_unlock(&w->mu);
    return r->status;
}

/* ---- transport entries ---------------------------------------------------- */

static int sk_send(void *ctx, const void *buf, size_t n, int dst, int tag)
{
    bcp_sock_world *w = ctx;
    if (peer_fd(w, dst) < 0 || (n && !buf))
        return -EINVAL;
    return send_frame(w, dst, FRAME_MAGIC, tag, (uint64_t)n, buf, n);
}

static int sk_isend(void *ctx, const void *buf, size_t n, int dst, int tag, void **req)
{
    /* eager: the frame is in the socket (or written through) on return */
    int rc = sk_send(ctx, buf, n, dst, tag);
    if (req)
        *req = rc ? NULL : &g_sent;
    return rc;
}

static int sk_irecv(void *ctx, void *buf, size_t n, int src, int tag, void **req)
{
    bcp_sock_world *w = ctx;
    if (!req || peer_fd(w, src) < 0 || (n && !buf))
        return -EINVAL;
    sk_req *r = calloc(1, sizeof(*r));
    if (!r)
        return -ENOMEM;
    pthread_cond_init(&r->cv, NULL);
    r->src = src;
    r->tag = tag;
    r->buf = buf;
    r->cap = n;
    pthread_mutex_lock(&w->mu);
    sk_msg *m = take_unexp(w, src, tag);
    int rts = m && m->rts, fill = 0;
    if (m && !rts) {
        deliver_msg(r, m);
    } else if (rts && in_arena(buf, n)) {
        push_list(&w->filling, r); /* the sender fills buf, then DONE */
        fill = 1;
    } else {
        if (w->posted_tail)
            w->posted_tail->next = r;
        else
            w->posted_head = r;
        w->posted_tail = r;
    }
    pthread_mutex_unlock(&w->mu);
    *req = r;
    if (rts) {
        free(m);
        /* a sender waits for this answer; if it cannot be sent, the peer is
         * failed here as the read path fails it (its sockets are unusable
         * for this rendezvous): r completes with the error when waited for */
        const int crc = send_cts(w, src, tag, fill ? buf : NULL, fill ? n : 0);
        if (crc) {
            pthread_mutex_lock(&w->mu);
            if (!w->dead[src])
                w->dead[src] = crc < 0 ? -crc : EIO;
            wake_peer(w, src);
            pthread_mutex_unlock(&w->mu);
        }
    }
    return 0;
}

/* Stream n zero bytes as one message (a fill send without memory). */
static int send_zeros(bcp_sock_world *w, size_t n, int dst, int tag)
{
    static const uint8_t z[65536];
    const int fd = peer_fd(w, dst);
    frame_hdr h = {FRAME_MAGIC, tag, (uint64_t)n};
    pthread_mutex_lock(&w->send_mu[dst]);
    int rc = write_all(fd, &h, sizeof(h));
    for (size_t k = 0; !rc && k < n; k += sizeof(z))
        rc = write_all(fd, z, n - k < sizeof(z) ? n - k : sizeof(z));
    pthread_mutex_unlock(&w->send_mu[dst]);
    return rc;
}

/* Fill send (rendezvous, see the top of the file): fill() writes the n-byte
 * payload straight into the receiver's arena row; a receive outside the
 * arena gets an ordinary message produced by fill() into a scratch buffer.
 * Returns fill's error, else the transport's. */
static int sk_send_fill(void *ctx, bcp_lb_fill_fn fill, void *fctx, size_t n, int dst, int tag)
{
    bcp_sock_world *w = ctx;
    if (peer_fd(w, dst) < 0 || !fill)
        return -EINVAL;
    sk_req *r = calloc(1, sizeof(*r));
    if (!r)
        return -ENOMEM;
    pthread_cond_init(&r->cv, NULL);
    r->src = dst;
    r->tag = tag;
    r->ctl = 1;
    pthread_mutex_lock(&w->mu);
    push_list(&w->cts_wait, r);
    pthread_mutex_unlock(&w->mu);
    int rc = send_frame(w, dst, FRAME_RTS, tag, (uint64_t)n, NULL, 0);
    if (rc) {
        pthread_mutex_lock(&w->mu);
        drop_list(&w->cts_wait, r);
        pthread_mutex_unlock(&w->mu);
        pthread_cond_destroy(&r->cv);
        free(r);
        return rc;
    }
    rc = progress_until(w, r);
    uint8_t *addr = (uint8_t *)(uintptr_t)r->cts_addr;
    const size_t cap = (size_t)r->cts_cap;
    pthread_cond_destroy(&r->cv);
    free(r);
    if (rc)
        return rc;
    int frc;
    __atomic_fetch_add(addr ? &g_fill_arena : &g_fill_msg, 1, __ATOMIC_RELAXED);
    if (!addr) {
        /* zeroed: a fill may define only its chunk's bytes (implicit padding) */
        uint8_t *tmp = calloc(1, n ? n : 1);
        if (!tmp) {
            rc = send_zeros(w, n, dst, tag);
            return rc ? rc : -ENOMEM;
        }
        frc = fill(fctx, tmp, n);
        rc = sk_send(w, tmp, n, dst, tag);
        free(tmp);
        return frc ? frc : rc;
    }
    if (!in_arena(addr, cap)) {
        const uint64_t zero = 0;
        (void)send_frame(w, dst, FRAME_DONE, tag, sizeof(zero), &zero, sizeof(zero));
        return -EPROTO;
    }
    if (n <= cap) {
        frc = fill(fctx, addr, n);
    } else {
        /* truncated receive (MPI_ERR_TRUNCATE): produce all, keep cap */
        uint8_t *tmp = calloc(1, n);
        frc = tmp ? fill(fctx, tmp, n) : -ENOMEM;
        if (tmp && cap)
            memcpy(addr, tmp, cap);
        free(tmp);
    }
    const uint64_t got = (uint64_t)n;
    rc = send_frame(w, dst, FRAME_DONE, tag, sizeof(got), &got, sizeof(got));
    return frc ? frc : rc;
}

static int sk_wait(void *ctx, void *req)
{
    bcp_sock_world *w = ctx;
    if (!req)
        return -EINVAL;
    if (req == &g_sent)
        return 0;
    sk_req *r = req;
    int st = progress_until(w, r);
    pthread_cond_destroy(&r->cv);
    free(r);
    return st;
}

static int sk_waitall(void *ctx, int n, void **reqs)
{
    int rc = 0;
    for (int i = 0; i < n; i++) {
        int e = sk_wait(ctx, reqs[i]);
        if (e && !rc)
            rc = e;
        reqs[i] = NULL;
    }
    return rc;
}

static int sk_recv(void *ctx, void *buf, size_t n, int src, int tag)
{
    void *r = NULL;
    int rc = sk_irecv(ctx, buf, n, src, tag, &r);
    return rc ? rc : sk_wait(ctx, r);
}

int bcpi_sock_transport_is(const bcp_transport_ops *ops)
{
    return ops && ops->send == sk_send;
}

int bcp_sock_world_attach(bcp_sock_world *w, int rank, bcp_transport_ops *ops)
{
    if (!w || !ops || rank < 0 || rank >= w->world || w->rank >= 0)
        return -EINVAL;
    /* keep only this rank's ends: the other ranks' processes hold theirs */
    for (int a = 0; a < w->world; a++)
        for (int b = 0; b < w->world; b++)
            if (a != rank) {
                if (w->fds[a * w->world + b] >= 0)
                    close(w->fds[a * w->world + b]);
                if (w->cfds[a * w->world + b] >= 0)
                    close(w->cfds[a * w->world + b]);
                w->fds[a * w->world + b] = w->cfds[a * w->world + b] = -1;
            }
    w->rank = rank;
    if (w->arena) {
        pthread_mutex_lock(&g_arena_mu);
        g_arena_lo = w->arena;
        g_arena_hi = w->arena + w->slice * (size_t)w->world;
        g_slice = w->arena + w->slice * (size_t)rank;
        g_slice_bytes = w->slice;
        g_slice_used = 0;
        g_nblocks = 0;
        pthread_mutex_unlock(&g_arena_mu);
    }
    memset(ops, 0, sizeof(*ops));
    ops->ctx = w;
    ops->send = sk_send;
    ops->recv = sk_recv;
    ops->isend = sk_isend;
    ops->irecv = sk_irecv;
    ops->wait = sk_wait;
    ops->waitall = sk_waitall;
    /* without an arena the sources send from their own window buffer, as
     * the reference does */
    ops->send_fill = w->arena ? sk_send_fill : NULL;
    return 0;
}
