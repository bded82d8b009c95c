/*
 * bcp_loopback.c -- point-to-point transport between loopback ranks.
 *
 * Replaces the MPI subset the chunk-streaming protocol uses
 * (task_processing.c:43-52,120-130,159-166,206-209,274-307: MPI_Send,
 * MPI_Recv, MPI_Isend, MPI_Irecv, MPI_Wait(all) on MPI_COMM_WORLD, matched by
 * source and tag) for ranks that are threads of one process.
 *
 * Matching: every destination rank has an inbox of unmatched sends (FIFO by
 * arrival) and a list of posted receives (FIFO by posting), split into
 * LB_SHARDS channels by tag, each with its own lock (the protocol's tag is the
 * lane: the lanes of one rank do not contend for one lock).  An arriving send
 * takes the oldest posted receive with its (source, tag) in its channel; a new
 * receive takes the oldest inbox entry with its (source, tag).  That gives
 * MPI's non-overtaking order per (source, destination, tag).
 *
 * Copies: blocking sends above LB_EAGER_MAX are rendezvous -- the receiver
 * copies straight from the sender's buffer (one memcpy, outside the lock) and
 * then releases the sender; smaller blocking sends and all non-blocking sends
 * are eager (copied at post time, the sender goes on: the protocol's 8-byte
 * chunk sizes and max_cs broadcast, the rebuild's size table).  Fill sends (bcp_lb_send_fill)
 * copy nothing: once matched, the receiver's buffer is handed to the sending
 * thread, whose callback writes the payload into it (the chunk sender reads
 * its file straight into the P role's window row).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "bcp_host.h"
#include "bcp_task.h"

/* Waiting: a blocked receive (and a fill send whose receive is not posted
 * yet) first watches its flag for up to lb_spin_us (bcp_task_set_fold_tuning
 * "lb_spin_us"), as MPI's shared-memory transports poll, then sleeps on its
 * condition.  Completers set the flag with a release store under the channel
 * lock; a waiter that saw it while spinning takes that lock once before it
 * frees the request, so the completer's signal has returned. */
static int g_lb_spin_ns;

int bcpi_lb_spin_us(int us)
{
    const int prev = __atomic_load_n(&g_lb_spin_ns, __ATOMIC_RELAXED) / 1000;
    if (us >= 0)
        __atomic_store_n(&g_lb_spin_ns, us * 1000, __ATOMIC_RELAXED);
    return prev;
}

static uint64_t lb_now_ns(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000u + (uint64_t)t.tv_nsec;
}

/* spin until *flag is non-zero or the budget is spent; 1 if it was seen */
static int lb_spin_int(const int *flag)
{
    const int budget = __atomic_load_n(&g_lb_spin_ns, __ATOMIC_RELAXED);
    if (budget <= 0)
        return 0;
    const uint64_t t0 = lb_now_ns();
    for (;;) {
        for (int i = 0; i < 64; i++) {
            if (__atomic_load_n(flag, __ATOMIC_ACQUIRE))
                return 1;
            __builtin_ia32_pause();
        }
        if (lb_now_ns() - t0 >= (uint64_t)budget)
            return 0;
    }
}

struct bcp_lb_req;

typedef struct lb_msg {
    struct lb_msg *next;
    int src, tag;
    const void *buf;     /* payload (sender's or eager copy) */
    size_t n;
    int eager;           /* payload is owned by this record (free_eager) */
    int done;            /* rendezvous: receiver finished copying */
    int fill;            /* fill send: payload produced by the sender into `target` */
    struct bcp_lb_req *target; /* fill send: the matched receive */
    int target_set;      /* fill send: target is set (release store; spinning senders) */
    pthread_cond_t cv;   /* rendezvous sender waits here */
} lb_msg;

struct bcp_lb_req {
    struct bcp_lb_req *next;
    pthread_mutex_t *mu; /* the channel lock done / cv are guarded by */
    int is_recv;
    int src, tag;        /* recv: match key */
    void *buf;
    size_t cap;
    size_t received;
    int status;          /* 0 or -EMSGSIZE */
    int done;
    pthread_cond_t cv;
};

/* Channels per destination rank (a power of two; tags map by their low bits). */
#define LB_SHARDS 64

typedef struct {
    pthread_mutex_t mu;
    lb_msg *inbox_head, *inbox_tail;
    bcp_lb_req *posted_head, *posted_tail;
} __attribute__((aligned(64))) lb_chan;

static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER; /* init / finalize */
static lb_chan *g_chans = NULL;                            /* g_world x LB_SHARDS */
static int g_world = 0;
static __thread int t_rank = -1;

static lb_chan *chan_of(int rank, int tag)
{
    return &g_chans[(size_t)rank * LB_SHARDS + ((unsigned)tag & (LB_SHARDS - 1))];
}

/* Blocking sends up to this size are buffered (eager): the protocol's 8-byte
 * chunk sizes and the rebuild's size table need no rendezvous. */
#define LB_EAGER_MAX 4096

/* An eager inbox record: 1 = payload malloc'd apart (isend), 2 = inline (send). */
static void free_eager(lb_msg *m)
{
    if (m->eager == 1) {
        free((void *)m->buf);
        pthread_cond_destroy(&m->cv);
    }
    free(m);
}

int bcp_lb_init(int world_size)
{
    if (world_size <= 0)
        return -EINVAL;
    pthread_mutex_lock(&g_lock);
    if (g_chans) {
        pthread_mutex_unlock(&g_lock);
        return -EBUSY;
    }
    lb_chan *c = aligned_alloc(64, (size_t)world_size * LB_SHARDS * sizeof(lb_chan));
    if (!c) {
        pthread_mutex_unlock(&g_lock);
        return -ENOMEM;
    }
    memset(c, 0, (size_t)world_size * LB_SHARDS * sizeof(lb_chan));
    for (size_t i = 0; i < (size_t)world_size * LB_SHARDS; i++)
        pthread_mutex_init(&c[i].mu, NULL);
    g_chans = c;
    g_world = world_size;
    pthread_mutex_unlock(&g_lock);
    return 0;
}

int bcp_lb_finalize(void)
{
    pthread_mutex_lock(&g_lock);
    int leftover = 0;
    for (size_t i = 0; g_chans && i < (size_t)g_world * LB_SHARDS; i++) {
        lb_chan *c = &g_chans[i];
        for (lb_msg *m = c->inbox_head; m;) {
            lb_msg *nx = m->next;
            leftover++;
            if (m->eager)
                free_eager(m);
            m = nx;
        }
        if (c->posted_head)
            leftover++;
        pthread_mutex_destroy(&c->mu);
    }
    free(g_chans);
    g_chans = NULL;
    g_world = 0;
    pthread_mutex_unlock(&g_lock);
    return leftover ? -EPIPE : 0;
}

int bcp_lb_world_size(void) { return g_world; }
void bcp_lb_set_rank(int rank) { t_rank = rank; }
int bcp_lb_rank(void) { return t_rank; }

static int check_peer(int peer)
{
    if (!g_chans || peer < 0 || peer >= g_world || t_rank < 0 || t_rank >= g_world)
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

/* Remove and return the oldest posted receive in channel d matching (src, tag). */
static bcp_lb_req *take_posted(lb_chan *d, int src, int tag)
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

static lb_msg *take_inbox(lb_chan *d, int src, int tag)
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

static void push_inbox(lb_chan *d, lb_msg *m)
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
    pthread_mutex_t *mu = r->mu;
    pthread_mutex_lock(mu);
    __atomic_store_n(&r->done, 1, __ATOMIC_RELEASE);
    pthread_cond_signal(&r->cv);
    pthread_mutex_unlock(mu);
}

int bcp_lb_send(const void *buf, size_t n, int dst, int tag)
{
    int rc = check_peer(dst);
    if (rc)
        return rc;
    lb_chan *d = chan_of(dst, tag);
    pthread_mutex_lock(&d->mu);
    bcp_lb_req *r = take_posted(d, t_rank, tag);
    if (r) {
        pthread_mutex_unlock(&d->mu);
        deliver(r, buf, n);
        int st = r->status; /* r belongs to the receiver once completed */
        complete_req(r);
        return st;
    }
    if (n <= LB_EAGER_MAX) {
        /* small: buffered, the sender goes on (MPI_Send may buffer; shared-
         * memory MPIs do below their eager limit) */
        lb_msg *m = calloc(1, sizeof(*m) + (n ? n : 1));
        if (!m) {
            pthread_mutex_unlock(&d->mu);
            return -ENOMEM;
        }
        if (n)
            memcpy(m + 1, buf, n);
        m->src = t_rank;
        m->tag = tag;
        m->buf = m + 1;
        m->n = n;
        m->eager = 2;
        push_inbox(d, m);
        pthread_mutex_unlock(&d->mu);
        return 0;
    }
    lb_msg m = {0};
    m.src = t_rank;
    m.tag = tag;
    m.buf = buf;
    m.n = n;
    pthread_cond_init(&m.cv, NULL);
    push_inbox(d, &m);
    while (!m.done)
        pthread_cond_wait(&m.cv, &d->mu);
    pthread_mutex_unlock(&d->mu);
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
    lb_chan *d = chan_of(dst, tag);
    pthread_mutex_lock(&d->mu);
    bcp_lb_req *r = take_posted(d, t_rank, tag);
    if (!r) {
        lb_msg m = {0};
        m.src = t_rank;
        m.tag = tag;
        m.n = n;
        m.fill = 1;
        pthread_cond_init(&m.cv, NULL);
        push_inbox(d, &m);
        if (__atomic_load_n(&g_lb_spin_ns, __ATOMIC_RELAXED) > 0) {
            pthread_mutex_unlock(&d->mu);
            (void)lb_spin_int((const int *)&m.target_set);
            pthread_mutex_lock(&d->mu);
        }
        while (!m.target)
            pthread_cond_wait(&m.cv, &d->mu);
        r = m.target;
        pthread_mutex_unlock(&d->mu);
        pthread_cond_destroy(&m.cv);
    } else {
        pthread_mutex_unlock(&d->mu);
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
    s->mu = &chan_of(dst, tag)->mu;
    lb_chan *d = chan_of(dst, tag);
    pthread_mutex_lock(&d->mu);
    bcp_lb_req *r = take_posted(d, t_rank, tag);
    if (r) {
        pthread_mutex_unlock(&d->mu);
        deliver(r, buf, n);
        complete_req(r);
    } else {
        lb_msg *m = calloc(1, sizeof(*m));
        void *copy = malloc(n ? n : 1);
        if (!m || !copy) {
            pthread_mutex_unlock(&d->mu);
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
        pthread_mutex_unlock(&d->mu);
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
    lb_chan *me = chan_of(t_rank, tag);
    r->mu = &me->mu;
    pthread_mutex_lock(&me->mu);
    lb_msg *m = take_inbox(me, src, tag);
    if (m && m->fill) {
        /* hand the buffer to the sending thread; it completes r */
        r->next = NULL;
        m->target = r;
        __atomic_store_n(&m->target_set, 1, __ATOMIC_RELEASE);
        pthread_cond_signal(&m->cv);
        pthread_mutex_unlock(&me->mu);
    } else if (m) {
        pthread_mutex_unlock(&me->mu);
        deliver(r, m->buf, m->n);
        r->done = 1;
        if (m->eager) {
            free_eager(m);
        } else {
            pthread_mutex_lock(&me->mu);
            m->done = 1; /* m lives on the sender's stack: signal under the lock */
            pthread_cond_signal(&m->cv);
            pthread_mutex_unlock(&me->mu);
        }
    } else {
        r->next = NULL;
        if (me->posted_tail)
            me->posted_tail->next = r;
        else
            me->posted_head = r;
        me->posted_tail = r;
        pthread_mutex_unlock(&me->mu);
    }
    *req = r;
    return 0;
}

int bcp_lb_wait(bcp_lb_req *r, size_t *received)
{
    if (!r)
        return -EINVAL;
    pthread_mutex_t *mu = r->mu;
    (void)lb_spin_int(&r->done);
    pthread_mutex_lock(mu); /* also: the completer's signal has returned */
    while (!r->done)
        pthread_cond_wait(&r->cv, mu);
    pthread_mutex_unlock(mu);
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
