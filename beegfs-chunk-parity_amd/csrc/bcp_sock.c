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
 * Sends write the frame under a per-destination lock (the lanes of a rank
 * share its sockets).  Writes block only on a full socket buffer, which the
 * destination drains as soon as any of its threads waits on us -- the MPI
 * rendezvous contract the protocol is written for.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include "bcp_task.h"

#define FRAME_MAGIC 0x62637066u /* "bcpf" */

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
} sk_msg;

typedef struct sk_req {
    struct sk_req *next;
    int src, tag;
    void *buf;
    size_t cap, received;
    int status;
    int done;
} sk_req;

struct bcp_sock_world {
    int world, rank;      /* rank < 0 until attached */
    int *fds;             /* [world][world]: fds[a*world+b] = a's end towards b (-1 closed) */
    pthread_mutex_t mu;
    pthread_cond_t cv;
    pthread_mutex_t *send_mu; /* per peer */
    int *reading;             /* per peer: a thread is reading that socket */
    int *dead;                /* per peer: socket failed / closed (errno) */
    sk_req *posted_head, *posted_tail;
    sk_msg *unexp_head, *unexp_tail;
};

static sk_req g_sent; /* the completed request every isend returns (eager) */

int bcp_sock_world_create(int world_size, bcp_sock_world **out)
{
    if (!out || world_size < 1 || world_size > 4096)
        return -EINVAL;
    *out = NULL;
    bcp_sock_world *w = calloc(1, sizeof(*w));
    if (!w)
        return -ENOMEM;
    w->world = world_size;
    w->rank = -1;
    w->fds = malloc((size_t)world_size * (size_t)world_size * sizeof(int));
    w->send_mu = calloc((size_t)world_size, sizeof(pthread_mutex_t));
    w->reading = calloc((size_t)world_size, sizeof(int));
    w->dead = calloc((size_t)world_size, sizeof(int));
    if (!w->fds || !w->send_mu || !w->reading || !w->dead) {
        bcp_sock_world_destroy(w);
        return -ENOMEM;
    }
    for (int i = 0; i < world_size * world_size; i++)
        w->fds[i] = -1;
    pthread_mutex_init(&w->mu, NULL);
    pthread_cond_init(&w->cv, NULL);
    for (int i = 0; i < world_size; i++)
        pthread_mutex_init(&w->send_mu[i], NULL);
    for (int a = 0; a < world_size; a++)
        for (int b = a + 1; b < world_size; b++) {
            int sv[2];
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
        }
    *out = w;
    return 0;
}

int bcp_sock_world_destroy(bcp_sock_world *w)
{
    if (!w)
        return -EINVAL;
    if (w->fds)
        for (int i = 0; i < w->world * w->world; i++)
            if (w->fds[i] >= 0)
                close(w->fds[i]);
    for (sk_msg *m = w->unexp_head; m;) {
        sk_msg *nx = m->next;
        free(m->data);
        free(m);
        m = nx;
    }
    free(w->fds);
    free(w->send_mu);
    free(w->reading);
    free(w->dead);
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

/* One frame from src: straight into a posted receive, or buffered.  Called
 * by the thread holding reading[src], without the lock. */
static int read_one(bcp_sock_world *w, int src)
{
    const int fd = peer_fd(w, src);
    frame_hdr h;
    int rc = read_all(fd, &h, sizeof(h));
    if (!rc && h.magic != FRAME_MAGIC)
        rc = -EPROTO;
    if (rc)
        return rc;
    pthread_mutex_lock(&w->mu);
    sk_req *r = take_posted(w, src, h.tag);
    pthread_mutex_unlock(&w->mu);
    if (r) {
        size_t c = h.len <= r->cap ? (size_t)h.len : r->cap;
        rc = c ? read_all(fd, r->buf, c) : 0;
        if (!rc && h.len > c)
            rc = discard(fd, (size_t)(h.len - c));
        pthread_mutex_lock(&w->mu);
        r->received = c;
        r->status = rc ? rc : (h.len <= r->cap ? 0 : -EMSGSIZE);
        r->done = 1;
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
    if ((r = take_posted(w, src, h.tag)))
        deliver_msg(r, m);
    else {
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
        if (w->dead[s]) {
            remove_posted(w, r); /* so nobody completes it after it is freed */
            r->status = -w->dead[s];
            r->done = 1;
            break;
        }
        if (w->reading[s]) {
            pthread_cond_wait(&w->cv, &w->mu);
            continue;
        }
        w->reading[s] = 1;
        pthread_mutex_unlock(&w->mu);
        int rc = read_one(w, s);
        pthread_mutex_lock(&w->mu);
        w->reading[s] = 0;
        if (rc && rc != -EMSGSIZE && rc != -ENOMEM)
            w->dead[s] = -rc;
        pthread_cond_broadcast(&w->cv);
    }
    pthread_mutex_unlock(&w->mu);
    return r->status;
}

/* ---- transport entries ---------------------------------------------------- */

static int sk_send(void *ctx, const void *buf, size_t n, int dst, int tag)
{
    bcp_sock_world *w = ctx;
    const int fd = peer_fd(w, dst);
    if (fd < 0 || (n && !buf))
        return -EINVAL;
    frame_hdr h = {FRAME_MAGIC, tag, (uint64_t)n};
    pthread_mutex_lock(&w->send_mu[dst]);
    int rc = write_all(fd, &h, sizeof(h));
    if (!rc && n)
        rc = write_all(fd, buf, n);
    pthread_mutex_unlock(&w->send_mu[dst]);
    return rc;
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
    r->src = src;
    r->tag = tag;
    r->buf = buf;
    r->cap = n;
    pthread_mutex_lock(&w->mu);
    sk_msg *m = take_unexp(w, src, tag);
    if (m)
        deliver_msg(r, m);
    else {
        if (w->posted_tail)
            w->posted_tail->next = r;
        else
            w->posted_head = r;
        w->posted_tail = r;
    }
    pthread_mutex_unlock(&w->mu);
    *req = r;
    return 0;
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

int bcp_sock_world_attach(bcp_sock_world *w, int rank, bcp_transport_ops *ops)
{
    if (!w || !ops || rank < 0 || rank >= w->world || w->rank >= 0)
        return -EINVAL;
    /* keep only this rank's ends: the other ranks' processes hold theirs */
    for (int a = 0; a < w->world; a++)
        for (int b = 0; b < w->world; b++)
            if (a != rank && w->fds[a * w->world + b] >= 0) {
                close(w->fds[a * w->world + b]);
                w->fds[a * w->world + b] = -1;
            }
    w->rank = rank;
    memset(ops, 0, sizeof(*ops));
    ops->ctx = w;
    ops->send = sk_send;
    ops->recv = sk_recv;
    ops->isend = sk_isend;
    ops->irecv = sk_irecv;
    ops->wait = sk_wait;
    ops->waitall = sk_waitall;
    ops->send_fill = NULL; /* sources send from their own window buffer, as the reference does */
    return 0;
}
