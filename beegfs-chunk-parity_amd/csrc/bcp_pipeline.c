/*
 * bcp_pipeline.c -- batched end-to-end parity generation on one node.
 *
 * The per-task protocol (bcp_task.c) moves one stripe per round trip; this
 * is the throughput form of the same computation for loopback stores, where
 * every chunk file is local: stripes are batched into pinned slabs and the
 * device does one descriptor-kernel launch per batch (SURVEY.md §7 "hard
 * parts": batching vs the per-task interface).
 *
 *   io pool (reads first)     chunk files -> pinned input slab   [slot s]
 *   h2d queue                 pinned -> device slab, event H
 *   compute queue             wait H, xor_desc over the batch, event K
 *   d2h queue                 wait K, parity bodies -> pinned output slab, event D
 *   io pool (the same)        wait D, parity files = u64 sizes[n] + body
 *
 * Slots are recycled round-robin, so batch b+1 is read while batch b is on
 * the device and batch b-1 is being written; H2D and D2H run on their own
 * queues beside the kernel (PCIe is full duplex).  With ndevices > 1 the
 * batches go round-robin to the node's GPUs (each with its own engine, queues
 * and slots; stripes are independent, so nothing crosses GPUs): PCIe, not the
 * kernel, bounds this path, and every GPU brings its own link.
 *
 * Output files are byte-identical to parity_generator's
 * (task_processing.c:146-226): header in ascending storage-target order, then
 * the windowed XOR (replay semantics past one 10 MiB window); a missing chunk
 * counts as size 0 / zeros; an item with no holders unlinks its parity chunk.
 *
 * Rebuild mode (bcp_pipeline_rebuild) is the same machinery with do_file's
 * roles (rebuild/main.c:40-89, task_processing.c:146-174,228-230,263-280):
 * the sources are the surviving chunks plus the parity body (read after the
 * u64 header), max_cs = max(header), and the lost chunk is written to the
 * victim's chunks directory truncated to header[index of the victim];
 * survivors newer than FileInfo.timestamp go to the corrupt list.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <linux/magic.h>
#include <sys/mman.h>
#include <sys/vfs.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <time.h>
#include <unistd.h>

#include "bcp_host.h"
#include "bcp_runner.h"

#define ROW 256u
#define PAGE 4096u
#define WINDOW ((uint64_t)BCP_WINDOW_BYTES)
#define RUP(x) (((x) + ROW - 1) / ROW * ROW)
#define RUP_PAGE(x) (((x) + PAGE - 1) / PAGE * PAGE)

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + (double)t.tv_nsec * 1e-9;
}

/* ---- a small job pool ---------------------------------------------------
 * Jobs are intrusive: every argument struct starts with a `job`, and the
 * caller owns its storage (arrays sized before a run starts), so pushing a
 * job cannot fail half way through a batch and leave a latch that never
 * reaches zero. */
typedef struct job {
    struct job *next;
    void (*fn)(struct job *);
} job;

typedef struct {
    pthread_mutex_t lock;
    pthread_cond_t cv;
    job *head, *tail;
    job *hhead, *htail;   /* taken first (pool_push_hi) */
    int stop;
    int nthreads;
    pthread_t *th;
} pool;

static void *pool_main(void *p)
{
    pool *P = p;
    for (;;) {
        pthread_mutex_lock(&P->lock);
        while (!P->head && !P->hhead && !P->stop)
            pthread_cond_wait(&P->cv, &P->lock);
        job *j = P->hhead ? P->hhead : P->head;
        if (!j) {
            pthread_mutex_unlock(&P->lock);
            return NULL;
        }
        if (j == P->hhead) {
            P->hhead = j->next;
            if (!P->hhead)
                P->htail = NULL;
        } else {
            P->head = j->next;
            if (!P->head)
                P->tail = NULL;
        }
        pthread_mutex_unlock(&P->lock);
        j->fn(j);
    }
}

static void pool_stop(pool *P);

/* All n threads or none: a partial start joins what it started. */
static int pool_start(pool *P, int n)
{
    memset(P, 0, sizeof(*P));
    pthread_mutex_init(&P->lock, NULL);
    pthread_cond_init(&P->cv, NULL);
    P->th = calloc((size_t)n, sizeof(pthread_t));
    if (!P->th) {
        pthread_mutex_destroy(&P->lock);
        pthread_cond_destroy(&P->cv);
        return -ENOMEM;
    }
    for (int i = 0; i < n; i++) {
        if (pthread_create(&P->th[i], NULL, pool_main, P) != 0) {
            pool_stop(P);
            return -EAGAIN;
        }
        P->nthreads++;
    }
    return 0;
}

static void pool_push(pool *P, job *j, void (*fn)(job *))
{
    j->fn = fn;
    j->next = NULL;
    pthread_mutex_lock(&P->lock);
    if (P->tail)
        P->tail->next = j;
    else
        P->head = j;
    P->tail = j;
    pthread_cond_signal(&P->cv);
    pthread_mutex_unlock(&P->lock);
}

/* The same, ahead of every job pushed with pool_push. */
static void pool_push_hi(pool *P, job *j, void (*fn)(job *))
{
    j->fn = fn;
    j->next = NULL;
    pthread_mutex_lock(&P->lock);
    if (P->htail)
        P->htail->next = j;
    else
        P->hhead = j;
    P->htail = j;
    pthread_cond_signal(&P->cv);
    pthread_mutex_unlock(&P->lock);
}

static void pool_stop(pool *P)
{
    pthread_mutex_lock(&P->lock);
    P->stop = 1;
    pthread_cond_broadcast(&P->cv);
    pthread_mutex_unlock(&P->lock);
    for (int i = 0; i < P->nthreads; i++)
        pthread_join(P->th[i], NULL);
    free(P->th);
    pthread_mutex_destroy(&P->lock);
    pthread_cond_destroy(&P->cv);
}

/* countdown latch */
typedef struct {
    pthread_mutex_t lock;
    pthread_cond_t cv;
    long left;
    double t_zero;        /* when the count reached zero */
} latch;

static void latch_init(latch *l, long n)
{
    pthread_mutex_init(&l->lock, NULL);
    pthread_cond_init(&l->cv, NULL);
    l->left = n;
    l->t_zero = n ? 0.0 : now_s();
}
static void latch_down(latch *l)
{
    pthread_mutex_lock(&l->lock);
    if (--l->left == 0) {
        l->t_zero = now_s();
        pthread_cond_broadcast(&l->cv);
    }
    pthread_mutex_unlock(&l->lock);
}
static void latch_wait(latch *l)
{
    pthread_mutex_lock(&l->lock);
    while (l->left > 0)
        pthread_cond_wait(&l->cv, &l->lock);
    pthread_mutex_unlock(&l->lock);
}
static void latch_destroy(latch *l)
{
    pthread_mutex_destroy(&l->lock);
    pthread_cond_destroy(&l->cv);
}

/* ---- plan --------------------------------------------------------------- */
typedef struct {
    const char *path;
    int p;                               /* output target: P (gen) or the victim (rebuild) */
    int n;                               /* sources */
    int holders[MAX_STORAGE_TARGETS];    /* source targets, ascending */
    int rebuild;                         /* 1: rebuild task */
    int parity_src;                      /* rebuild: index of the parity body among the sources */
    int64_t timestamp;                   /* rebuild: FileInfo.timestamp (corrupt check) */
    uint64_t size[MAX_STORAGE_TARGETS];  /* source lengths at stat time (0 = missing);
                                            gen: also the parity header */
    uint64_t src_off[MAX_STORAGE_TARGETS];/* file offset of the source data (parity body: 8n) */
    uint64_t max_cs;
    uint64_t out_len;                    /* gen: max_cs; rebuild: header[victim index] */
    uint64_t in_off[MAX_STORAGE_TARGETS];/* offsets in the input slab (page layout, DIRECT:
                                            of the file's first byte, page-aligned; the data
                                            then starts src_off further) */
    uint64_t out_off;                    /* offset in the output slab */
    int batch;
    int prealloc;                        /* posix_fallocate the output first (not where the
                                            output target's directory is tmpfs: do_write) */
} task;

typedef struct {
    job j;                               /* first: the pool's link */
    const char *root;
    task *t;
    latch *done;
    int corrupt_fd;                      /* rebuild: corrupt list (or -1) */
} stat_arg;

typedef struct {
    uint8_t *h_in, *h_out;
    void *d_in, *d_out;
    size_t in_cap, out_cap;
    bcp_event *ev_h, *ev_k, *ev_d;
    latch reads, writes;
    int busy;             /* writes of the previous batch pending */
} slot;



/* One read job: bytes [off, off + len) of source k's data, into dst (its
 * place in the slab + off).  Sources are read in pieces of at most PIECE
 * bytes, so a batch's big chunks spread over the io threads instead of one
 * thread finishing a 4 MiB chunk while the others idle.  DIRECT mode: off and
 * len are of the file itself (page-aligned, the page layout puts the file's
 * first byte at a page of the slab), read with O_DIRECT. */
#define PIECE ((uint64_t)1 << 20)
typedef struct {
    job j;
    const char *root;
    task *t;
    int k;                /* source */
    uint64_t off, len;
    uint8_t *dst;
    uint64_t *bytes;      /* accumulated under lock: {data bytes, of them read with O_DIRECT,
                             DIRECT pieces read through the page cache instead} */
    latch *done;
    int direct;
} read_arg;

static uint64_t pieces_of(uint64_t size)
{
    return (size + PIECE - 1) / PIECE;
}

/* Read jobs of source k: PIECE-sized pieces of its data, or (DIRECT) of the
 * file prefix up to the data's end, page-rounded. */
static uint64_t read_extent(const task *t, int k, int direct)
{
    if (!t->size[k])
        return 0;
    return direct ? RUP_PAGE(t->src_off[k] + t->size[k]) : t->size[k];
}

typedef struct {
    job j;
    const char *root;
    task *t;
    const uint8_t *body;
    latch *done;
    FILE *log;
    int *errors;
    int prealloc;         /* posix_fallocate first (not on tmpfs: see do_write) */
} write_arg;

typedef struct {
    job j;
    slot *S;
    const char *root;
    task *tasks;
    write_arg *wa;        /* one per task of the run */
    size_t first, last;
    pool *io;
    FILE *log;
    int *errors;
    int *dev_rc;
} complete_arg;

static pthread_mutex_t g_stat_lock = PTHREAD_MUTEX_INITIALIZER;

static void chunk_file(char *buf, size_t cap, const char *root, int st, const char *dir, const char *path)
{
    snprintf(buf, cap, "%s/st%d/%s/%s", root, st, dir, path);
}

/* Corrupt list line (task_processing.c:54-60, 268-271), written whole. */
static void push_corrupt(int fd, const char *path)
{
    if (fd < 0)
        return;
    size_t len = strlen(path);
    char *line = malloc(len + 2);
    if (!line)
        return;
    memcpy(line, path, len);
    line[len] = '\n';
    ssize_t w = write(fd, line, len + 1);
    (void)w;
    free(line);
}

static void do_stat(job *p)
{
    stat_arg *a = (stat_arg *)p;
    task *t = a->t;
    char fn[4352];
    t->max_cs = 0;
    if (!t->rebuild) {
        for (int k = 0; k < t->n; k++) {
            chunk_file(fn, sizeof(fn), a->root, t->holders[k], "chunks", t->path);
            struct stat st;
            t->size[k] = stat(fn, &st) == 0 ? (uint64_t)st.st_size : 0;
            t->src_off[k] = 0;
            if (t->size[k] > t->max_cs)
                t->max_cs = t->size[k];
        }
        t->out_len = t->max_cs;
        latch_down(a->done);
        return;
    }
    /* rebuild: survivors as they are now; the parity holder contributes its
     * stored header (sizes at generation) and the body after it */
    uint64_t header[MAX_STORAGE_TARGETS] = {0};
    const int n = t->n;
    for (int k = 0; k < n; k++) {
        struct stat st;
        if (k == t->parity_src) {
            chunk_file(fn, sizeof(fn), a->root, t->holders[k], "parity", t->path);
            int fd = open(fn, O_RDONLY);
            uint64_t fsize = 0;
            if (fd >= 0) {
                if (fstat(fd, &st) == 0)
                    fsize = (uint64_t)st.st_size;
                ssize_t r = pread(fd, header, (size_t)n * 8u, 0); /* a short header reads as zeros */
                (void)r;
                close(fd);
            }
            t->src_off[k] = (uint64_t)n * 8u;
            t->size[k] = fsize > t->src_off[k] ? fsize - t->src_off[k] : 0;
        } else {
            chunk_file(fn, sizeof(fn), a->root, t->holders[k], "chunks", t->path);
            t->src_off[k] = 0;
            if (stat(fn, &st) == 0) {
                t->size[k] = (uint64_t)st.st_size;
                if (st.st_mtime > t->timestamp)
                    push_corrupt(a->corrupt_fd, t->path);
            } else {
                t->size[k] = 0;
            }
        }
    }
    for (int k = 0; k < n; k++)
        if (header[k] > t->max_cs)
            t->max_cs = header[k];
    /* the victim's index in the header: survivors (and the victim) below it */
    int idx = 0;
    for (int k = 0; k < n; k++)
        if (k != t->parity_src && t->holders[k] < t->p)
            idx++;
    t->out_len = header[idx];
    /* sources longer than max_cs are only read up to it (data_to_send) */
    for (int k = 0; k < n; k++)
        if (t->size[k] > t->max_cs)
            t->size[k] = t->max_cs;
    latch_down(a->done);
}

static void do_read(job *p)
{
    read_arg *a = (read_arg *)p;
    task *t = a->t;
    const uint64_t want = a->len;
    const uint64_t foff = a->direct ? a->off : t->src_off[a->k] + a->off; /* file offset of dst[0] */
    uint64_t got = 0;
    int direct = 0, fell_back = 0;
    if (want) {
        char fn[4352];
        const int is_parity = t->rebuild && a->k == t->parity_src;
        chunk_file(fn, sizeof(fn), a->root, t->holders[a->k], is_parity ? "parity" : "chunks", t->path);
        int fd = -1;
        if (a->direct) {
            fd = open(fn, O_RDONLY | O_DIRECT);
            direct = fd >= 0;
            fell_back = !direct;
        }
        if (fd < 0)
            fd = open(fn, O_RDONLY);
        if (fd >= 0) {
            if (!direct)
                posix_fadvise(fd, (off_t)foff, (off_t)want, POSIX_FADV_SEQUENTIAL);
            while (got < want) {
                ssize_t r = pread(fd, a->dst + got, (size_t)(want - got), (off_t)(foff + got));
                if (direct && r > 3000 && bcpi_inject_hit(BCP_INJECT_DIRECT_READ)) {
                    /* (failure injection) short before the end: what the read
                     * did deliver past the cut is spoilt, the fallback must
                     * read it again */
                    memset(a->dst + got + 3000, 0xA5, (size_t)r - 3000);
                    r = 3000;
                }
                if (r > 0)
                    got += (uint64_t)r;
                struct stat sb;
                if (direct && (r < 0 || (got % PAGE && got < want && fstat(fd, &sb) == 0 &&
                                         (uint64_t)sb.st_size > foff + got))) {
                    /* refused (EINVAL: alignment the filesystem wants bigger,
                     * EFAULT: memory it cannot pin) or short before the end
                     * of the file: the rest of the piece through the page cache */
                    close(fd);
                    fd = open(fn, O_RDONLY);
                    direct = 0;
                    fell_back = 1;
                    if (fd < 0)
                        break;
                    continue;
                }
                if (r <= 0 || (direct && got % PAGE))
                    break; /* end of file (an O_DIRECT read ends short there) */
            }
            if (fd >= 0)
                close(fd);
        }
    }
    /* the source's data inside this piece; what the file no longer holds is
     * zero padded, as chunk_sender does (:302-303) */
    const uint64_t d_lo = a->direct ? t->src_off[a->k] : foff;
    const uint64_t d_hi = a->direct ? d_lo + t->size[a->k] : foff + want;
    const uint64_t lo = d_lo > foff ? d_lo : foff;
    const uint64_t hi = d_hi < foff + want ? d_hi : foff + want;
    const uint64_t have = foff + got;
    uint64_t data = 0;
    if (hi > lo) {
        const uint64_t z = have > lo ? have : lo;
        if (z < hi)
            memset(a->dst + (z - foff), 0, (size_t)(hi - z));
        data = (have < hi ? have : hi) > lo ? (have < hi ? have : hi) - lo : 0;
    }
    pthread_mutex_lock(&g_stat_lock);
    a->bytes[0] += data;
    if (a->direct) {
        if (fell_back)
            a->bytes[2]++;
        else
            a->bytes[1] += data;
    }
    pthread_mutex_unlock(&g_stat_lock);
    latch_down(a->done);
}

static void mkdir_parents(char *fn)
{
    for (char *q = fn + 1; *q; q++)
        if (*q == '/') {
            *q = 0;
            mkdir(fn, S_IRWXU);
            *q = '/';
        }
}

static void do_write(job *p)
{
    write_arg *a = (write_arg *)p;
    task *t = a->t;
    char fn[4352];
    chunk_file(fn, sizeof(fn), a->root, t->p, t->rebuild ? "chunks" : "parity", t->path);
    /* directories only when the file cannot be created (mkdir_for_file,
     * task_processing.c:30-40, does every level first: a lookup per level
     * per file).  (Overwriting an existing file in place instead of
     * O_TRUNC, to reuse its page-cache pages, measured no different:
     * profiles/r04/pipeline/lib_ab_overwrite_in_place_r4r.jsonl.) */
    int fd = open(fn, O_CREAT | O_WRONLY | O_TRUNC, S_IRUSR | S_IWUSR);
    if (fd < 0 && errno == ENOENT) {
        mkdir_parents(fn);
        fd = open(fn, O_CREAT | O_WRONLY | O_TRUNC, S_IRUSR | S_IWUSR);
    }
    int bad = fd < 0;
    if (!bad) {
        /* gen: u64 sizes header + body; rebuild: the chunk itself */
        const size_t hdr = t->rebuild ? 0 : 8u * (size_t)t->n;
        uint64_t total = hdr + t->out_len;
        /* The reference reserves the file's space first (task_processing.c:186):
         * on a disk that keeps it in one extent and fails early when full.  On
         * tmpfs it makes the kernel allocate and ZERO every page before the
         * write fills it again -- one more pass over the parity bytes for
         * nothing -- so it is skipped there (the file is the same). */
        if (total && a->prealloc)
            posix_fallocate(fd, 0, (off_t)total);
        struct iovec iov[2] = {{t->size, hdr}, {(void *)a->body, (size_t)t->out_len}};
        uint64_t done = 0;
        int idx = total ? 0 : 2; /* an empty rebuilt chunk: nothing to write */
        while (idx < 2 && !bad) {
            ssize_t w = writev(fd, iov + idx, 2 - idx);
            if (w <= 0) {
                bad = 1;
                break;
            }
            done += (uint64_t)w;
            size_t left = (size_t)w;
            while (idx < 2 && left >= iov[idx].iov_len) {
                left -= iov[idx].iov_len;
                idx++;
            }
            if (idx < 2) {
                iov[idx].iov_base = (uint8_t *)iov[idx].iov_base + left;
                iov[idx].iov_len -= left;
            }
        }
        (void)done;
        close(fd);
    }
    if (bad) {
        pthread_mutex_lock(&g_stat_lock);
        (*a->errors)++;
        if (a->log)
            fprintf(a->log, "bcp_pipeline: writing parity '%s' failed: %s\n", fn, strerror(errno));
        pthread_mutex_unlock(&g_stat_lock);
    }
    latch_down(a->done);
}

/* Completion stage (one thread, batches in order): wait for the batch's D2H,
 * then hand its parity files to the io pool (behind every queued read). */
static void do_complete(job *p)
{
    /* The run frees its job arrays once every write of the batch has counted
     * down, which may be before this function returns: copy what it needs
     * and touch neither `a` nor a pushed write job after handing it over. */
    const complete_arg a = *(complete_arg *)p;
    int rc = bcp_event_sync(a.S->ev_d);
    if (rc) {
        pthread_mutex_lock(&g_stat_lock);
        *a.dev_rc = rc;
        pthread_mutex_unlock(&g_stat_lock);
        for (size_t i = a.first; i < a.last; i++)
            latch_down(&a.S->writes);
    } else {
        for (size_t i = a.first; i < a.last; i++) {
            write_arg *w = &a.wa[i];
            *w = (write_arg){{0}, a.root, &a.tasks[i], a.S->h_out + a.tasks[i].out_off, &a.S->writes, a.log, a.errors,
                             a.tasks[i].prealloc};
            pool_push(a.io, &w->j, do_write);
        }
    }
}

static int slot_alloc(bcp_engine *e, slot *s, size_t in_cap, size_t out_cap)
{
    int rc;
    memset(s, 0, sizeof(*s));
    if ((rc = bcp_host_alloc(e, in_cap, (void **)&s->h_in)) || (rc = bcp_host_alloc(e, out_cap, (void **)&s->h_out)) ||
        (rc = bcp_dev_alloc(e, in_cap, &s->d_in)) || (rc = bcp_dev_alloc(e, out_cap, &s->d_out)) ||
        (rc = bcp_event_create(e, &s->ev_h)) || (rc = bcp_event_create(e, &s->ev_k)) ||
        (rc = bcp_event_create(e, &s->ev_d)))
        return rc;
    s->in_cap = in_cap;
    s->out_cap = out_cap;
    return 0;
}

static void slot_free(bcp_engine *e, slot *s)
{
    bcp_host_free(e, s->h_in);
    bcp_host_free(e, s->h_out);
    bcp_dev_free(e, s->d_in);
    bcp_dev_free(e, s->d_out);
    if (s->ev_h)
        bcp_event_destroy(s->ev_h);
    if (s->ev_k)
        bcp_event_destroy(s->ev_k);
    if (s->ev_d)
        bcp_event_destroy(s->ev_d);
}

/* One GPU of the pipeline: engine, h2d / compute / d2h queues, slots. */
typedef struct {
    bcp_engine *eng;
    bcp_queue *qh, *qk, *qd;
    slot *slots;
} dev_lane;

struct bcp_pipeline {
    bcp_pipeline_opts o;
    int read_mode;      /* BCP_READ_AUTO (decided per run), COPY or DIRECT */
    int ndev;
    dev_lane *dev;
    pool io, completer; /* io: 2 x io_threads threads, chunk reads ahead of parity writes */
    int pools;
    size_t in_cap, out_cap;
    bcp_stripe *st;
    bcp_source *so;
    size_t desc_cap;    /* stripes the descriptor arrays hold */
    bcp_pipeline_timing last; /* of the last run */
};

int bcp_pipeline_last_timing(const bcp_pipeline *pl, bcp_pipeline_timing *out)
{
    if (!pl || !out)
        return -EINVAL;
    *out = pl->last;
    return 0;
}

static void free_slots(bcp_pipeline *pl)
{
    for (int d = 0; d < pl->ndev; d++) {
        dev_lane *L = &pl->dev[d];
        if (!L->slots)
            continue;
        for (int s = 0; s < pl->o.nslots; s++)
            slot_free(L->eng, &L->slots[s]);
        free(L->slots);
        L->slots = NULL;
    }
}

int bcp_pipeline_destroy(bcp_pipeline *pl)
{
    if (!pl)
        return -EINVAL;
    /* only the pools that started (pool_start is all or nothing) */
    if (pl->pools & 2)
        pool_stop(&pl->completer);
    if (pl->pools & 1)
        pool_stop(&pl->io);
    if (pl->dev) {
        /* queues first (each synchronises its streams): no copy or kernel may
         * still use a slot when its memory goes */
        for (int d = 0; d < pl->ndev; d++) {
            dev_lane *L = &pl->dev[d];
            if (L->qh)
                bcp_queue_destroy(L->qh);
            if (L->qk)
                bcp_queue_destroy(L->qk);
            if (L->qd)
                bcp_queue_destroy(L->qd);
            L->qh = L->qk = L->qd = NULL;
        }
        free_slots(pl);
        for (int d = 0; d < pl->ndev; d++)
            if (pl->dev[d].eng)
                bcp_engine_destroy(pl->dev[d].eng);
        free(pl->dev);
    }
    free(pl->st);
    free(pl->so);
    free(pl);
    return 0;
}

static int ensure_slots(bcp_pipeline *pl, size_t in_cap, size_t out_cap)
{
    if (pl->dev[0].slots && in_cap <= pl->in_cap && out_cap <= pl->out_cap)
        return 0;
    free_slots(pl);
    in_cap = in_cap > pl->in_cap ? in_cap : pl->in_cap;
    out_cap = out_cap > pl->out_cap ? out_cap : pl->out_cap;
    for (int d = 0; d < pl->ndev; d++) {
        dev_lane *L = &pl->dev[d];
        L->slots = calloc((size_t)pl->o.nslots, sizeof(slot));
        if (!L->slots)
            return -ENOMEM;
        for (int s = 0; s < pl->o.nslots; s++) {
            int rc = slot_alloc(L->eng, &L->slots[s], in_cap, out_cap);
            if (rc)
                return rc;
        }
    }
    pl->in_cap = in_cap;
    pl->out_cap = out_cap;
    return 0;
}

/* CPUs this process may use: its affinity mask, capped by the cgroup's CPU
 * quota (v2 cpu.max, else v1 cfs). */
static int usable_cpus(void)
{
    cpu_set_t set;
    int n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 0;
    if (n <= 0)
        n = (int)sysconf(_SC_NPROCESSORS_ONLN);
    long long q = -1, per = 0;
    FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r");
    if (f) {
        char qs[32];
        if (fscanf(f, "%31s %lld", qs, &per) == 2 && strcmp(qs, "max"))
            q = atoll(qs);
        fclose(f);
    } else if ((f = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r"))) {
        if (fscanf(f, "%lld", &q) != 1)
            q = -1;
        fclose(f);
        if ((f = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r"))) {
            if (fscanf(f, "%lld", &per) != 1)
                per = 0;
            fclose(f);
        }
    }
    if (q > 0 && per > 0) {
        const long long c = (q + per / 2) / per;
        if (c >= 1 && c < n)
            n = (int)c;
    }
    return n > 0 ? n : 1;
}

int bcp_pipeline_create(const bcp_pipeline_opts *opts_in, bcp_pipeline **out)
{
    if (!out)
        return -EINVAL;
    *out = NULL;
    bcp_pipeline_opts o = {0, 256u << 20, 0, 4, 1, BCP_READ_AUTO};
    if (opts_in)
        o = *opts_in;
    /* 2 was the MAP read mode (ABI 2), removed in ABI 3: never chosen by
     * AUTO and level with or behind COPY */
    if (o.read_mode != BCP_READ_AUTO && o.read_mode != BCP_READ_COPY && o.read_mode != BCP_READ_DIRECT)
        return -EINVAL;
    if (o.read_mode == BCP_READ_AUTO) { /* stays AUTO (decided per run) unless the env names a mode */
        const char *env = getenv("BCP_PIPELINE_READ");
        o.read_mode = !env                     ? BCP_READ_AUTO
                      : !strcmp(env, "copy")   ? BCP_READ_COPY
                      : !strcmp(env, "direct") ? BCP_READ_DIRECT
                                               : BCP_READ_AUTO;
    }
    if (o.ndevices < 1)
        o.ndevices = 1;
    /* io threads 0 = auto: 8 per GPU, and the io pool twice that (reads and
     * writes share it, below).  One GPU's PCIe link takes what ~8 threads
     * copy out of the page cache (8 + 8 beat 16 + 16 on a 16-CPU share,
     * profiles/r02/protocol/pipeline_io_threads_ab_r2e4.jsonl), and every
     * further GPU brings its own link and its own CPU share -- but never more
     * than half the CPUs this process may run on, so the pool has no more
     * threads than CPUs: beyond that they only measure oversubscription. */
    if (o.io_threads == 0) {
        const int half = usable_cpus() / 2;
        o.io_threads = 8 * o.ndevices;
        if (o.io_threads > half)
            o.io_threads = half > 2 ? half : 2;
    }
    int ndev_vis = 0;
    bcp_device_count(&ndev_vis);
    if (o.device < 0 || o.ndevices > 64)
        return -EINVAL;
    if (o.slab_bytes < (1u << 20))
        o.slab_bytes = 1u << 20;
    if (o.io_threads < 1)
        o.io_threads = 1;
    if (o.io_threads > 64)
        o.io_threads = 64;
    if (o.nslots < 2)
        o.nslots = 2;
    if (o.nslots > 8)
        o.nslots = 8;
    bcp_pipeline *pl = calloc(1, sizeof(*pl));
    if (!pl)
        return -ENOMEM;
    pl->o = o;
    pl->read_mode = o.read_mode; /* AUTO: COPY or DIRECT, chosen per run (auto_read_mode) */
    int rc = 0;
    pl->dev = calloc((size_t)o.ndevices, sizeof(dev_lane));
    if (!pl->dev) {
        free(pl);
        return -ENOMEM;
    }
    pl->ndev = o.ndevices;
    for (int d = 0; d < pl->ndev; d++) {
        dev_lane *L = &pl->dev[d];
        /* devices wrap modulo the visible count: more lanes than GPUs runs
         * several lanes per GPU (how the multi-device path is tested on one) */
        const int dev = ndev_vis > 0 ? (o.device + d) % ndev_vis : o.device + d;
        if ((rc = bcp_engine_create(dev, &L->eng)) || (rc = bcp_queue_create(L->eng, &L->qh)) ||
            (rc = bcp_queue_create(L->eng, &L->qk)) || (rc = bcp_queue_create(L->eng, &L->qd)))
            goto fail;
    }
    /* One io pool of 2 x io_threads threads reads chunks and writes parity
     * files, reads first: the reads feed the link, a batch's writes only gate
     * its slot's reuse four batches later, and where the host's CPU time
     * bounds the run a thread never idles in one pool while the other has
     * work.  (Separate pools, writes first and push order measured within the
     * box-to-box spread of this order on six boxes and were removed in r05:
     * profiles/r04/pipeline/shared_io_ab*.jsonl) */
    if ((rc = pool_start(&pl->io, 2 * o.io_threads)))
        goto fail;
    pl->pools |= 1;
    if ((rc = pool_start(&pl->completer, 1)))
        goto fail;
    pl->pools |= 2;
    if ((rc = ensure_slots(pl, o.slab_bytes, o.slab_bytes)))
        goto fail;
    *out = pl;
    return 0;
fail:
    bcp_pipeline_destroy(pl);
    return rc;
}

static int pipeline_exec(bcp_pipeline *pl, const char *store_root, task *tasks, size_t nt, int corrupt_fd,
                         FILE *log, bcp_run_stats *stats, double t0);

/* Bytes source k of t takes in the input slab: its data at 256-byte pitch
 * (COPY), or the whole file prefix up to the data's end at page pitch (DIRECT:
 * files are read from offset 0 into page-aligned slab offsets, the rebuild
 * parity body sits 8n in). */
static uint64_t span_of(const task *t, int k, int page_layout)
{
    if (!page_layout)
        return RUP(t->size[k]);
    return t->size[k] ? RUP_PAGE(t->src_off[k] + t->size[k]) : 0;
}

/* Where source k's data starts, relative to the slab. */
static uint64_t data_off(const task *t, int k, int page_layout)
{
    return t->in_off[k] + (page_layout ? t->src_off[k] : 0);
}

int bcp_pipeline_run(bcp_pipeline *pl, const char *store_root, int ntargets, const bcp_work_item *items,
                     size_t nitems, FILE *log, bcp_run_stats *stats)
{
    if (!pl || !store_root || ntargets < 1 || ntargets > MAX_STORAGE_TARGETS || (nitems && !items))
        return -EINVAL;
    double t0 = now_s();
    int rc = 0;

    /* validate everything before touching any file */
    for (size_t i = 0; i < nitems; i++) {
        uint64_t loc = items[i].fi.locations;
        int P = GET_P(loc);
        if ((uint64_t)P == NO_P)
            continue;
        if (!items[i].path || P >= ntargets || TEST_BIT(loc, P) || ((loc & L_MASK) >> ntargets))
            return -EINVAL;
    }
    /* tasks: skip NO_P, unlink deletes now (no data moves for them) */
    task *tasks = calloc(nitems ? nitems : 1, sizeof(task));
    if (!tasks)
        return -ENOMEM;
    size_t nt = 0;
    for (size_t i = 0; i < nitems; i++) {
        uint64_t loc = items[i].fi.locations;
        int P = GET_P(loc);
        if ((uint64_t)P == NO_P)
            continue;
        if (!bcpi_path_ok(items[i].path, (size_t)-1)) { /* as process_task: refused, skipped */
            if (log)
                fprintf(log, "bcp_pipeline: refusing '%s': not a path inside the store\n", items[i].path);
            continue;
        }
        if ((loc & L_MASK) == 0) {
            char fn[4352];
            chunk_file(fn, sizeof(fn), store_root, P, "parity", items[i].path);
            unlink(fn);
            continue;
        }
        task *t = &tasks[nt++];
        t->path = items[i].path;
        t->p = P;
        for (int k = 0; k < MAX_STORAGE_TARGETS; k++)
            if (TEST_BIT(loc, k))
                t->holders[t->n++] = k;
    }
    rc = pipeline_exec(pl, store_root, tasks, nt, -1, log, stats, t0);
    free(tasks);
    if (stats)
        stats->refused = bcpr_count_refused(items, nitems, -1);
    return rc;
}

/* One batch between queueing its reads and submitting it. */
typedef struct {
    size_t first, last;        /* tasks */
    uint64_t in_used;          /* input bytes */
    int reads_live;            /* S->reads initialised and not yet waited for */
    dev_lane *L;
    slot *S;
} bstate;

/* AUTO's read path for one run: COPY where the chunks are in memory anyway
 * (tmpfs / ramfs, or a sample of the run's sources mostly resident in the
 * page cache -- just written, or read before), DIRECT for a cold store on a
 * disk, where O_DIRECT lets the storage device fill the slabs without a CPU
 * copy (1.1-1.4x).  The sample: the first 16 MiB of one
 * source in each of up to 64 tasks spread over the run, mincore() on a
 * mapping of it. */
/* Filesystem of every storage target's directory a run touches, looked up
 * once per run: <root>/st<k>/{chunks,parity} are often separate mounts, so
 * the choices below are made per target, never from the store root. */
typedef struct {
    signed char mem[MAX_STORAGE_TARGETS][2]; /* [k][0 chunks, 1 parity]: 1 tmpfs / ramfs, 0 not, -1 unknown yet */
} fs_kinds;

static int dir_in_memory(fs_kinds *fk, const char *root, int k, int parity)
{
    signed char *m = &fk->mem[k][parity];
    if (*m < 0) {
        char dn[4352];
        snprintf(dn, sizeof(dn), "%s/st%d/%s", root, k, parity ? "parity" : "chunks");
        struct statfs sf;
        *m = statfs(dn, &sf) == 0 && (sf.f_type == TMPFS_MAGIC || sf.f_type == RAMFS_MAGIC);
    }
    return *m;
}

/* AUTO's read path for one run: COPY where the chunks are in memory anyway
 * (every source directory of the run on tmpfs / ramfs, or a sample of the
 * run's sources mostly resident in the page cache -- just written, or read
 * before), DIRECT for a cold store on a disk, where O_DIRECT lets the storage
 * device fill the slabs without a CPU copy (1.1-1.4x).
 * The sample: the first 16 MiB of one source in each of up to 64 tasks spread
 * over the run, mincore() on a mapping of it. */
static int auto_read_mode(const char *root, const task *tasks, size_t nt, fs_kinds *fk)
{
    int all_mem = 1;
    for (size_t i = 0; i < nt && all_mem; i++)
        for (int k = 0; k < tasks[i].n && all_mem; k++)
            all_mem = dir_in_memory(fk, root, tasks[i].holders[k], tasks[i].rebuild && k == tasks[i].parity_src);
    if (all_mem)
        return BCP_READ_COPY;
    const uint64_t cap = (uint64_t)16 << 20;
    unsigned char *vec = malloc(cap / PAGE);
    if (!vec)
        return BCP_READ_COPY;
    uint64_t pages = 0, resident = 0;
    char fn[4352];
    for (size_t i = 0; i < nt; i += nt / 64 + 1) {
        const task *t = &tasks[i];
        for (int k = 0; k < t->n; k++) {
            if (!t->size[k])
                continue;
            const int is_parity = t->rebuild && k == t->parity_src;
            chunk_file(fn, sizeof(fn), root, t->holders[k], is_parity ? "parity" : "chunks", t->path);
            const uint64_t len = t->src_off[k] + t->size[k] < cap ? t->src_off[k] + t->size[k] : cap;
            int fd = open(fn, O_RDONLY);
            if (fd < 0)
                continue;
            void *m = mmap(NULL, (size_t)len, PROT_READ, MAP_SHARED, fd, 0);
            close(fd);
            if (m == MAP_FAILED)
                continue;
            const uint64_t np = (len + PAGE - 1) / PAGE;
            if (mincore(m, (size_t)len, vec) == 0) {
                pages += np;
                for (uint64_t q = 0; q < np; q++)
                    resident += vec[q] & 1;
            }
            munmap(m, (size_t)len);
            break; /* one source per sampled task */
        }
    }
    free(vec);
    return pages && resident * 2 < pages ? BCP_READ_DIRECT : BCP_READ_COPY;
}

/* Stat, batch and stream the tasks through the slots (both read paths).
 * Takes no ownership of tasks. */
static int pipeline_exec(bcp_pipeline *pl, const char *store_root, task *tasks, size_t nt, int corrupt_fd,
                         FILE *log, bcp_run_stats *stats, double t0)
{
    fs_kinds fk;
    memset(&fk, -1, sizeof(fk));
    const int nslots = pl->o.nslots;
    int rc = 0, errors = 0, dev_rc = 0;
    uint64_t rd[3] = {0, 0, 0}, bytes_written = 0, ntasks = 0; /* rd: see read_arg.bytes */
    const double t_stat = now_s();
    memset(&pl->last, 0, sizeof(pl->last)); /* a run that fails early reports zeros, not the previous run */

    /* 1. stat every chunk (parallel) */
    {
        latch l;
        latch_init(&l, (long)nt);
        stat_arg *args = calloc(nt ? nt : 1, sizeof(stat_arg));
        if (!args) {
            latch_destroy(&l);
            return -ENOMEM;
        }
        for (size_t i = 0; i < nt; i++) {
            args[i] = (stat_arg){{0}, store_root, &tasks[i], &l, corrupt_fd};
            pool_push(&pl->io, &args[i].j, do_stat);
        }
        latch_wait(&l);
        latch_destroy(&l);
        free(args);
    }
    /* the reference reserves every output's space first (task_processing.c:186),
     * except where that output's directory is tmpfs / ramfs (do_write) */
    for (size_t i = 0; i < nt; i++)
        tasks[i].prealloc = !dir_in_memory(&fk, store_root, tasks[i].p, !tasks[i].rebuild);

    /* 2. plan batches: inputs at 256-byte pitch (DIRECT: page pitch), outputs
     * at 256 */
    const int mode = pl->read_mode == BCP_READ_AUTO ? auto_read_mode(store_root, tasks, nt, &fk) : pl->read_mode;
    const int dir = mode == BCP_READ_DIRECT; /* page layout */
    size_t in_cap = pl->in_cap, out_cap = pl->out_cap;
    for (size_t i = 0; i < nt; i++) {
        uint64_t in = 0;
        for (int k = 0; k < tasks[i].n; k++)
            in += span_of(&tasks[i], k, dir);
        if (in > in_cap)
            in_cap = (size_t)in;
        if (RUP(tasks[i].out_len) > out_cap)
            out_cap = (size_t)RUP(tasks[i].out_len);
    }
    if ((rc = ensure_slots(pl, in_cap, out_cap))) {
        return rc;
    }
    in_cap = pl->in_cap;
    out_cap = pl->out_cap;
    /* A small job (a changelog round's subset) cut at slab capacity makes a
     * few big batches: on ndev GPUs (batches go round-robin) most devices
     * would idle -- a 1 GiB round is 4 batches of 256 MiB for 8 GPUs.  Aim
     * for >= 4 batches per slot and device, >= 16 MiB each, never above the
     * slab (the largest task still fits, ensure_slots above).  On one GPU
     * this changed nothing measurable (r2av: the round's pipeline 48 ms vs
     * 46 before). */
    uint64_t plan_in = in_cap;
    {
        uint64_t total_in = 0, max_in = 0;
        for (size_t i = 0; i < nt; i++) {
            uint64_t in = 0;
            for (int k = 0; k < tasks[i].n; k++)
                in += span_of(&tasks[i], k, dir);
            total_in += in;
            max_in = in > max_in ? in : max_in;
        }
        const uint64_t want = (uint64_t)4 * (uint64_t)nslots * (uint64_t)pl->ndev;
        uint64_t per = total_in / want + 1;
        per = per < ((uint64_t)16 << 20) ? ((uint64_t)16 << 20) : per;
        plan_in = per < plan_in ? per : plan_in;
        plan_in = plan_in < max_in ? max_in : plan_in;
    }
    /* Ramps.  Once the reads outrun the link, the run is the host-to-device
     * copies back to back plus what cannot overlap them: the first batch's
     * reads before the first copy, and after the last copy the last batch's
     * kernel, D2H and parity writes.  Both scale with the batch, so batches
     * start at RAMP_MIN and double (a batch holds at most what the run has
     * consumed so far, per device) and end halving (at most half of what
     * remains, per device): r03 timing showed 6-10 ms of a 51 ms config-1
     * run spent in the drain behind 160 MiB batches. */
    const uint64_t RAMP_MIN = (uint64_t)16 << 20;
    uint64_t total_in_all = 0;
    for (size_t i = 0; i < nt; i++)
        for (int k = 0; k < tasks[i].n; k++)
            total_in_all += span_of(&tasks[i], k, dir);
    int nbatches = 0;
    {
        uint64_t in_used = 0, out_used = 0, consumed = 0, limit = plan_in;
        for (size_t i = 0; i < nt; i++) {
            task *t = &tasks[i];
            uint64_t in = 0;
            for (int k = 0; k < t->n; k++)
                in += span_of(t, k, dir);
            if (i == 0 || in_used + in > limit || out_used + RUP(t->out_len) > out_cap) {
                nbatches++;
                consumed += in_used;
                in_used = out_used = 0;
                const uint64_t up = consumed / (uint64_t)pl->ndev;
                const uint64_t down = (total_in_all - consumed) / (2u * (uint64_t)pl->ndev);
                limit = up < down ? up : down;
                limit = limit < RAMP_MIN ? RAMP_MIN : limit;
                limit = limit > plan_in ? plan_in : limit;
            }
            t->batch = nbatches - 1;
            for (int k = 0; k < t->n; k++) {
                t->in_off[k] = in_used;
                in_used += span_of(t, k, dir);
            }
            t->out_off = out_used;
            out_used += RUP(t->out_len);
        }
    }
    if (pl->desc_cap < nt) {
        free(pl->st);
        free(pl->so);
        pl->st = malloc((nt ? nt : 1) * sizeof(bcp_stripe));
        pl->so = malloc((nt ? nt : 1) * MAX_STORAGE_TARGETS * sizeof(bcp_source));
        pl->desc_cap = (pl->st && pl->so) ? nt : 0;
        if (!pl->desc_cap) {
            return -ENOMEM;
        }
    }
    bcp_stripe *st = pl->st;
    bcp_source *so = pl->so;
    /* every job of the run, before the first one is queued: a read job per
     * piece of every source, a write job per task, a completion per batch */
    size_t nreads_all = 0;
    for (size_t i = 0; i < nt; i++)
        for (int k = 0; k < tasks[i].n; k++)
            nreads_all += (size_t)pieces_of(read_extent(&tasks[i], k, dir));
    read_arg *ra = calloc(nreads_all ? nreads_all : 1, sizeof(read_arg));
    write_arg *wa = calloc(nt ? nt : 1, sizeof(write_arg));
    complete_arg *cargs = calloc(nbatches ? (size_t)nbatches : 1, sizeof(complete_arg));
    bstate *bs = calloc(nbatches ? (size_t)nbatches : 1, sizeof(bstate));
    if (!ra || !wa || !cargs || !bs) {
        free(ra);
        free(wa);
        free(cargs);
        free(bs);
        return -ENOMEM;
    }
    size_t rnext = 0;
    bcp_pipeline_timing tm = {0};
    tm.stat = now_s() - t_stat;
    tm.batches = (uint32_t)nbatches;

    /* 3. stream the batches through the slots.  Batch b+1's reads are
     * queued before the host waits for batch b's, so the io threads go from
     * one batch to the next without idling at a batch's last chunks; b is on
     * the device meanwhile and earlier batches are being written (4 slots by
     * default: a slot's parity writes gate its reuse). */
    {
        size_t first = 0;
        for (int b = 0; b < nbatches; b++) {
            bs[b].first = first;
            while (first < nt && tasks[first].batch == b)
                first++;
            bs[b].last = first;
        }
    }
    int started = 0; /* batches whose reads are queued */
    for (int b = 0; b < nbatches && !rc; b++) {
        /* queue batch b+1's reads into its slot (after the slot's previous
         * batch has been written), ahead of every queued parity write */
        for (; started < nbatches && started <= b + 1; started++) {
            bstate *B = &bs[started];
            B->L = &pl->dev[started % pl->ndev];
            B->S = &B->L->slots[(started / pl->ndev) % nslots];
            double tw = now_s();
            if (B->S->busy) { /* writes of batch started - nslots still running */
                latch_wait(&B->S->writes);
                latch_destroy(&B->S->writes);
                B->S->busy = 0;
            }
            tm.slot_wait += now_s() - tw;
            uint64_t in_used = 0;
            long nreads = 0;
            for (size_t i = B->first; i < B->last; i++)
                for (int k = 0; k < tasks[i].n; k++) {
                    const uint64_t end = tasks[i].in_off[k] + span_of(&tasks[i], k, dir);
                    if (end > in_used)
                        in_used = end;
                    nreads += (long)pieces_of(read_extent(&tasks[i], k, dir));
                }
            B->in_used = in_used;
            latch_init(&B->S->reads, nreads);
            B->reads_live = 1;
            for (size_t i = B->first; i < B->last; i++)
                for (int k = 0; k < tasks[i].n; k++) {
                    const uint64_t e = read_extent(&tasks[i], k, dir);
                    uint8_t *d = B->S->h_in + (dir ? tasks[i].in_off[k] : data_off(&tasks[i], k, dir));
                    for (uint64_t o = 0; o < e; o += PIECE) {
                        read_arg *a = &ra[rnext++];
                        *a = (read_arg){{0}, store_root, &tasks[i], k, o, e - o < PIECE ? e - o : PIECE, d + o, rd,
                                        &B->S->reads, dir};
                        pool_push_hi(&pl->io, &a->j, do_read);
                    }
                }
            tm.read_jobs += (uint32_t)nreads;
        }
        bstate *B = &bs[b];
        dev_lane *L = B->L;
        slot *S = B->S;
        const uint64_t in_used = B->in_used;
        const size_t first = B->first, last = B->last;
        const double t_wait0 = now_s();
        latch_wait(&S->reads);
        latch_destroy(&S->reads);
        B->reads_live = 0;
        const double ts = now_s();
        tm.read_wait += ts - t_wait0; /* blocked on this batch's reads */
        uint32_t ns = 0, nsrc = 0;
        uint64_t out_used = 0;
        for (size_t i = first; i < last; i++) {
            task *t = &tasks[i];
            st[ns] = (bcp_stripe){(uint64_t)S->d_out + t->out_off, t->out_len, nsrc, (uint32_t)t->n,
                                  t->max_cs > WINDOW ? WINDOW : 0};
            for (int k = 0; k < t->n; k++)
                so[nsrc++] = (bcp_source){(uint64_t)S->d_in + data_off(t, k, dir), t->size[k]};
            ns++;
            if (t->out_off + RUP(t->out_len) > out_used)
                out_used = t->out_off + RUP(t->out_len);
        }
        /* device: H2D (side queue) -> kernel -> D2H (side queue) */
        if ((in_used && (rc = bcp_h2d_async(L->qh, S->d_in, S->h_in, (size_t)in_used))) ||
            (rc = bcp_event_record(S->ev_h, L->qh)) || (rc = bcp_queue_wait_event(L->qk, S->ev_h)) ||
            (rc = bcp_xor_stripes_async(L->qk, st, ns, so, nsrc)) || (rc = bcp_event_record(S->ev_k, L->qk)) ||
            (rc = bcp_queue_wait_event(L->qd, S->ev_k)) ||
            (rc = bcp_d2h_async(L->qd, S->h_out, S->d_out, (size_t)out_used)) ||
            (rc = bcp_event_record(S->ev_d, L->qd)))
            break;
        /* writes start once the batch's D2H is done (completion thread); the
         * host moves on to batch b+1 meanwhile */
        latch_init(&S->writes, (long)(last - first));
        S->busy = 1;
        complete_arg *ca = &cargs[b];
        *ca = (complete_arg){{0}, S, store_root, tasks, wa, first, last, &pl->io, log, &errors, &dev_rc};
        pool_push(&pl->completer, &ca->j, do_complete);
        for (size_t i = first; i < last; i++)
            bytes_written += (tasks[i].rebuild ? 0 : 8u * (uint64_t)tasks[i].n) + tasks[i].out_len;
        ntasks += last - first;
        tm.submit += now_s() - ts;
    }
    /* a failed submission leaves batch b+1's reads queued: let them finish
     * before the slab and the jobs go away */
    for (int b = 0; b < started; b++)
        if (bs[b].reads_live) {
            latch_wait(&bs[b].S->reads);
            latch_destroy(&bs[b].S->reads);
            bs[b].reads_live = 0;
        }
    free(bs);
    const double td = now_s();
    for (int d = 0; d < pl->ndev; d++)
        for (int s = 0; s < nslots; s++) {
            slot *S = &pl->dev[d].slots[s];
            if (S->busy) {
                latch_wait(&S->writes);
                latch_destroy(&S->writes);
                S->busy = 0;
            }
        }
    /* after a failed submission part of a batch may still be on the device:
     * nothing of this run stays in flight on the slots past its return */
    for (int d = 0; d < pl->ndev; d++) {
        dev_lane *L = &pl->dev[d];
        const int s1 = bcp_queue_sync(L->qh), s2 = bcp_queue_sync(L->qk), s3 = bcp_queue_sync(L->qd);
        if (!rc && !dev_rc)
            dev_rc = s1 ? s1 : s2 ? s2 : s3;
    }
    /* every job has run: the writes latched above, the completions before them */
    free(ra);
    free(wa);
    free(cargs);
    tm.drain = now_s() - td;
    tm.read_mode = mode;
    tm.direct_bytes = rd[1];
    tm.direct_fallbacks = (uint32_t)rd[2];
    pl->last = tm;
    if (!rc && dev_rc)
        rc = dev_rc;
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        stats->seconds = now_s() - t0;
        stats->tasks = ntasks;
        stats->bytes_read = rd[0];
        stats->bytes_written = bytes_written;
        stats->errors = errors;
    }
    return rc;
}

int bcp_pipeline_rebuild(bcp_pipeline *pl, const char *store_root, int ntargets, int rebuild_target,
                         const bcp_work_item *items, size_t nitems, const char *corrupt_list_path, FILE *log,
                         bcp_run_stats *stats)
{
    if (!pl || !store_root || ntargets < 2 || ntargets > MAX_STORAGE_TARGETS || rebuild_target < 0 ||
        rebuild_target >= ntargets || (nitems && !items))
        return -EINVAL;
    double t0 = now_s();
    for (size_t i = 0; i < nitems; i++) {
        uint64_t loc = items[i].fi.locations;
        int P = GET_P(loc);
        if ((uint64_t)P == NO_P)
            continue;
        if (!items[i].path || P >= ntargets || TEST_BIT(loc, P) || ((loc & L_MASK) >> ntargets))
            return -EINVAL;
    }
    int corrupt_fd = -1;
    if (corrupt_list_path) {
        corrupt_fd = open(corrupt_list_path, O_WRONLY | O_CREAT | O_TRUNC | O_APPEND, S_IRUSR | S_IWUSR);
        if (corrupt_fd < 0)
            return -errno;
    }
    task *tasks = calloc(nitems ? nitems : 1, sizeof(task));
    if (!tasks) {
        if (corrupt_fd >= 0)
            close(corrupt_fd);
        return -ENOMEM;
    }
    size_t nt = 0;
    for (size_t i = 0; i < nitems; i++) {
        const FileInfo *fi = &items[i].fi;
        const int P = GET_P(fi->locations);
        /* do_file's skip rules (rebuild/main.c:48-51) */
        if ((uint64_t)P == NO_P || P == rebuild_target || !TEST_BIT(fi->locations, rebuild_target))
            continue;
        if (!bcpi_path_ok(items[i].path, (size_t)-1)) { /* as process_task: refused, skipped */
            if (log)
                fprintf(log, "bcp_pipeline: refusing '%s': not a path inside the store\n", items[i].path);
            continue;
        }
        task *t = &tasks[nt++];
        t->path = items[i].path;
        t->p = rebuild_target;
        t->rebuild = 1;
        t->timestamp = fi->timestamp;
        /* sources: the surviving holders and the parity holder, ascending
         * (the re-roled locations of rebuild/main.c:55-60) */
        const uint64_t src = ((fi->locations & L_MASK) | (UINT64_C(1) << P)) & ~(UINT64_C(1) << rebuild_target);
        t->parity_src = -1;
        for (int k = 0; k < MAX_STORAGE_TARGETS; k++)
            if (TEST_BIT(src, k)) {
                if (k == P)
                    t->parity_src = t->n;
                t->holders[t->n++] = k;
            }
    }
    int rc = pipeline_exec(pl, store_root, tasks, nt, corrupt_fd, log, stats, t0);
    free(tasks);
    if (stats)
        stats->refused = bcpr_count_refused(items, nitems, rebuild_target);
    if (corrupt_fd >= 0)
        close(corrupt_fd);
    return rc;
}

int bcp_pipeline_gen(const char *store_root, int ntargets, const bcp_work_item *items, size_t nitems,
                     const bcp_pipeline_opts *opts, FILE *log, bcp_run_stats *stats)
{
    bcp_pipeline *pl = NULL;
    int rc = bcp_pipeline_create(opts, &pl);
    if (rc)
        return rc;
    rc = bcp_pipeline_run(pl, store_root, ntargets, items, nitems, log, stats);
    bcp_pipeline_destroy(pl);
    return rc;
}
