/*
 * bcp_loopback.c -- point-to-point transport between loopback ranks.
 *
 * Replaces the MPI subset the chunk-streaming protocol uses
 * (task_processing.c:43-52,120-130,159-166,206-209,274-307: MPI_Send,
 * MPI_Recv, MPI_Isend, MPI_Irecv, MPI_Wait(all) on MPI_COMM_WORLD, matched by
 * source and tag) for ranks that are threads of one process.
 *
 * Matching: every destination rank has an inbox of unmatched sends (FIFO by
 * arrival) and a list of posted receives (FIFO by posting).  An arriving send
 * takes the oldest posted receive with its (source, tag); a new receive takes
 * the oldest inbox entry with its (source, tag).  That gives MPI's
 * non-overtaking order per (source, destination, tag).
 *
 * Copies: blocking sends are rendezvous -- the receiver copies straight from
 * the sender's buffer (one memcpy, outside the lock) and then releases the
 * sender; non-blocking sends are eager (copied at post time; the protocol only
 * uses them for the 8-byte max_cs broadcast).  Fill sends (bcp_lb_send_fill)
 * copy nothing: once matched, the receiver's buffer is handed to the sending
 * thread, whose callback writes the payload into it (the chunk sender reads
 * its file straight into the P role's window row).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "bcp_task.h"

struct bcp_lb_req;

typedef struct lb_msg {
    struct lb_msg *next;
    int src, tag;
    const void *buf;     /* payload (sender's or eager copy) */
    size_t n;
    int eager;           /* payload is owned by this record */
    int done;            /* rendezvous: receiver finished copying */
    int fill;            /* fill send: payload produced by the sender into `target` */
    struct bcp_lb_req *target; /* fill send: the matched receive */
    pthread_cond_t cv;   /* rendezvous sender waits here */
} lb_msg;

struct bcp_lb_req {
    struct bcp_lb_req *next;
    int is_recv;
    int src, tag;        /* recv: match key */
    void *buf;
    size_t cap;
    size_t received;
    int status;          /* 0 or -EMSGSIZE */
    int done;
    pthread_cond_t cv;
};

typedef struct {
    lb_msg *inbox_head, *inbox_tail;
    bcp_lb_req *posted_head, *posted_tail;
} lb_rank;

static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static lb_rank *g_ranks = NULL;
static int g_world = 0;
static __thread int t_rank = -1;

int bcp_lb_init(int world_size)
{
    if (world_size <= 0)
        return -EINVAL;
    pthread_mutex_lock(&g_lock);
    if (g_ranks) {
        pthread_mutex_unlock(&g_lock);
        return -EBUSY;
    }
    g_ranks = calloc((size_t)world_size, sizeof(lb_rank));
    if (!g_ranks) {
        pthread_mutex_unlock(&g_lock);
        return -ENOMEM;
    }
    g_world = world_size;
    pthread_mutex_unlock(&g_lock);
    return 0;
}

int bcp_lb_finalize(void)
{
    pthread_mutex_lock(&g_lock);
    int leftover = 0;
    for (int r = 0; r < g_world; r++) {
        for (lb_msg *m = g_ranks[r].inbox_head; m;) {
            lb_msg *nx = m->next;
            leftover++;
            if (m->eager) {
                free((void *)m->buf);
                pthread_cond_destroy(&m->cv);
                free(m);
            }
            m = nx;
        }
        if (g_ranks[r].posted_head)
            leftover++;
    }
    free(g_ranks);
    g_ranks = NULL;
    g_world = 0;
    pthread_mutex_unlock(&g_lock);
    return leftover ? -EPIPE : 0;
}

int bcp_lb_world_size(void) { return g_world; }
void bcp_lb_set_rank(int rank) { t_rank = rank; }
int bcp_lb_rank(void) { return t_rank; }

static int check_peer(int peer)
{
    if (!g_ranks || peer < 0 || peer >= g_world || t_rank < 0 || t_rank >= g_world)
        return -EINVAL;
    return 0;
}

/* Copy a matched payload into a receive request (called without the lock). */
static void deliver(bcp_lb_req *r, const void *buf, size_t n)
{
    size_t c = n <= r->cap ? n : r->cap;
    if (c)
        memcpy(r->buf, buf, c);
    r->received = c;
    r->status = n <= r->cap ? 0 : -EMSGSIZE;
}

/* Remove and return the oldest posted receive at `dst` matching (src, tag). */
static bcp_lb_req *take_posted(lb_rank *d, int src, int tag)
{
    bcp_lb_req *prev = NULL;
    for (bcp_lb_req *r = d->posted_head; r; prev = r, r = r->next) {
        if (r->src == src && r->tag == tag) {
            if (prev)
                prev->next = r->next;
            else
                d->posted_head = r->next;
            if (d->posted_tail == r)
                d->posted_tail = prev;
            r->next = NULL;
            return r;
        }
    }
    return NULL;
}

static lb_msg *take_inbox(lb_rank *d, int src, int tag)
{
    lb_msg *prev = NULL;
    for (lb_msg *m = d->inbox_head; m; prev = m, m = m->next) {
        if (m->src == src && m->tag == tag) {
            if (prev)
                prev->next = m->next;
            else
                d->inbox_head = m->next;
            if (d->inbox_tail == m)
                d->inbox_tail = prev;
            m->next = NULL;
            return m;
        }
    }
    return NULL;
}

static void push_inbox(lb_rank *d, lb_msg *m)
{
    m->next = NULL;
    if (d->inbox_tail)
        d->inbox_tail->next = m;
    else
        d->inbox_head = m;
    d->inbox_tail = m;
}

static void complete_req(bcp_lb_req *r)
{
    pthread_mutex_lock(&g_lock);
    r->done = 1;
    pthread_cond_signal(&r->cv);
    pthread_mutex_unlock(&g_lock);
}

int bcp_lb_send(const void *buf, size_t n, int dst, int tag)
{
    int rc = check_peer(dst);
    if (rc)
        return rc;
    pthread_mutex_lock(&g_lock);
    lb_rank *d = &g_ranks[dst];
    bcp_lb_req *r = take_posted(d, t_rank, tag);
    if (r) {
        pthread_mutex_unlock(&g_lock);
        deliver(r, buf, n);
        int st = r->status; /* r belongs to the receiver once completed */
        complete_req(r);
        return st;
    }
    lb_msg m = {0};
    m.src = t_rank;
    m.tag = tag;
    m.buf = buf;
    m.n = n;
    pthread_cond_init(&m.cv, NULL);
    push_inbox(d, &m);
    while (!m.done)
        pthread_cond_wait(&m.cv, &g_lock);
    pthread_mutex_unlock(&g_lock);
    pthread_cond_destroy(&m.cv);
    return 0;
}

/* Run the sender's fill into a matched receive and complete it. */
static int fill_into(bcp_lb_req *r, bcp_lb_fill_fn fill, void *ctx, size_t n)
{
    int frc;
    if (n <= r->cap) {
        frc = fill(ctx, r->buf, n);
        r->received = n;
        r->status = 0;
    } else {
        /* truncated receive (MPI_ERR_TRUNCATE): produce all, keep cap */
        void *tmp = malloc(n ? n : 1);
        if (!tmp) {
            frc = -ENOMEM;
            r->received = 0;
        } else {
            frc = fill(ctx, tmp, n);
            if (r->cap)
                memcpy(r->buf, tmp, r->cap);
            free(tmp);
            r->received = r->cap;
        }
        r->status = -EMSGSIZE;
    }
    const int st = frc ? frc : r->status;
    complete_req(r);
    return st;
}

int bcp_lb_send_fill(bcp_lb_fill_fn fill, void *ctx, size_t n, int dst, int tag)
{
    int rc = check_peer(dst);
    if (rc)
        return rc;
    if (!fill)
        return -EINVAL;
    pthread_mutex_lock(&g_lock);
    lb_rank *d = &g_ranks[dst];
    bcp_lb_req *r = take_posted(d, t_rank, tag);
    if (!r) {
        lb_msg m = {0};
        m.src = t_rank;
        m.tag = tag;
        m.n = n;
        m.fill = 1;
        pthread_cond_init(&m.cv, NULL);
        push_inbox(d, &m);
        while (!m.target)
            pthread_cond_wait(&m.cv, &g_lock);
        r = m.target;
        pthread_mutex_unlock(&g_lock);
        pthread_cond_destroy(&m.cv);
    } else {
        pthread_mutex_unlock(&g_lock);
    }
    return fill_into(r, fill, ctx, n);
}

int bcp_lb_isend(const void *buf, size_t n, int dst, int tag, bcp_lb_req **req)
{
    int rc = check_peer(dst);
    if (rc)
        return rc;
    bcp_lb_req *s = calloc(1, sizeof(*s));
    if (!s)
        return -ENOMEM;
    pthread_cond_init(&s->cv, NULL);
    s->done = 1; /* eager: complete at post */
    pthread_mutex_lock(&g_lock);
    lb_rank *d = &g_ranks[dst];
    bcp_lb_req *r = take_posted(d, t_rank, tag);
    if (r) {
        pthread_mutex_unlock(&g_lock);
        deliver(r, buf, n);
        complete_req(r);
    } else {
        lb_msg *m = calloc(1, sizeof(*m));
        void *copy = malloc(n ? n : 1);
        if (!m || !copy) {
            pthread_mutex_unlock(&g_lock);
            free(m);
            free(copy);
            pthread_cond_destroy(&s->cv);
            free(s);
            return -ENOMEM;
        }
        if (n)
            memcpy(copy, buf, n);
        m->src = t_rank;
        m->tag = tag;
        m->buf = copy;
        m->n = n;
        m->eager = 1;
        pthread_cond_init(&m->cv, NULL);
        push_inbox(d, m);
        pthread_mutex_unlock(&g_lock);
    }
    if (req)
        *req = s;
    else {
        pthread_cond_destroy(&s->cv);
        free(s);
    }
    return 0;
}

int bcp_lb_irecv(void *buf, size_t n, int src, int tag, bcp_lb_req **req)
{
    int rc = check_peer(src);
    if (rc)
        return rc;
    if (!req)
        return -EINVAL;
    bcp_lb_req *r = calloc(1, sizeof(*r));
    if (!r)
        return -ENOMEM;
    pthread_cond_init(&r->cv, NULL);
    r->is_recv = 1;
    r->src = src;
    r->tag = tag;
    r->buf = buf;
    r->cap = n;
    pthread_mutex_lock(&g_lock);
    lb_rank *me = &g_ranks[t_rank];
    lb_msg *m = take_inbox(me, src, tag);
    if (m && m->fill) {
        /* hand the buffer to the sending thread; it completes r */
        r->next = NULL;
        m->target = r;
        pthread_cond_signal(&m->cv);
        pthread_mutex_unlock(&g_lock);
    } else if (m) {
        pthread_mutex_unlock(&g_lock);
        deliver(r, m->buf, m->n);
        r->done = 1;
        if (m->eager) {
            free((void *)m->buf);
            pthread_cond_destroy(&m->cv);
            free(m);
        } else {
            pthread_mutex_lock(&g_lock);
            m->done = 1; /* m lives on the sender's stack: signal under the lock */
            pthread_cond_signal(&m->cv);
            pthread_mutex_unlock(&g_lock);
        }
    } else {
        r->next = NULL;
        if (me->posted_tail)
            me->posted_tail->next = r;
        else
            me->posted_head = r;
        me->posted_tail = r;
        pthread_mutex_unlock(&g_lock);
    }
    *req = r;
    return 0;
}

int bcp_lb_wait(bcp_lb_req *r, size_t *received)
{
    if (!r)
        return -EINVAL;
    pthread_mutex_lock(&g_lock);
    while (!r->done)
        pthread_cond_wait(&r->cv, &g_lock);
    pthread_mutex_unlock(&g_lock);
    int st = r->status;
    if (received)
        *received = r->received;
    pthread_cond_destroy(&r->cv);
    free(r);
    return st;
}

int bcp_lb_waitall(int n, bcp_lb_req **reqs)
{
    int rc = 0;
    for (int i = 0; i < n; i++) {
        int e = bcp_lb_wait(reqs[i], NULL);
        if (e && !rc)
            rc = e;
        reqs[i] = NULL;
    }
    return rc;
}

int bcp_lb_recv(void *buf, size_t n, int src, int tag, size_t *received)
{
    bcp_lb_req *r = NULL;
    int rc = bcp_lb_irecv(buf, n, src, tag, &r);
    if (rc)
        return rc;
    return bcp_lb_wait(r, received);
}

/* ---- the loopback world as a transport table (process_task's default) ---- */
static int lbt_send(void *ctx, const void *buf, size_t n, int dst, int tag)
{
    (void)ctx;
    return bcp_lb_send(buf, n, dst, tag);
}
static int lbt_recv(void *ctx, void *buf, size_t n, int src, int tag)
{
    (void)ctx;
    return bcp_lb_recv(buf, n, src, tag, NULL);
}
static int lbt_isend(void *ctx, const void *buf, size_t n, int dst, int tag, void **req)
{
    (void)ctx;
    return bcp_lb_isend(buf, n, dst, tag, (bcp_lb_req **)req);
}
static int lbt_irecv(void *ctx, void *buf, size_t n, int src, int tag, void **req)
{
    (void)ctx;
    return bcp_lb_irecv(buf, n, src, tag, (bcp_lb_req **)req);
}
static int lbt_wait(void *ctx, void *req)
{
    (void)ctx;
    return bcp_lb_wait((bcp_lb_req *)req, NULL);
}
static int lbt_waitall(void *ctx, int n, void **reqs)
{
    (void)ctx;
    return bcp_lb_waitall(n, (bcp_lb_req **)reqs);
}
static int lbt_send_fill(void *ctx, bcp_lb_fill_fn fill, void *fctx, size_t n, int dst, int tag)
{
    (void)ctx;
    return bcp_lb_send_fill(fill, fctx, n, dst, tag);
}

static const bcp_transport_ops g_lb_ops = {NULL,     lbt_send, lbt_recv,    lbt_isend,    lbt_irecv,
                                           lbt_wait, lbt_waitall, lbt_send_fill};

const bcp_transport_ops *bcp_lb_transport(void) { return &g_lb_ops; }
