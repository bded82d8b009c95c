/*
 * bcp_changelog.c -- chunk-event records and worklist planning (the data
 * formats on either side of the hot path).
 *
 * Record stream (one per storage target), native-endian, no padding:
 *     i64 timestamp, u64 chunk_size, u64 event ('m' | 'd'), u64 path_len,
 *     char path[path_len]
 * as written by bp-find-all-chunks (main.c:25-33) and the changelog filter
 * (gen-chunkmod-filelist.py:35-41) and parsed by feed_targets_with
 * (gen/main.c:286-336).
 *
 * Aggregation per path (fih_add_info, gen/file_info_hash.c:24-31): the
 * newest timestamp, a 'modified' and a 'deleted' target bitmask, and the
 * summed chunk size (gen/main.c:688, used to order the worklist).
 *
 * Worklist (gen/main.c:703-715, 768-791): PCG32 shuffle with the reference's
 * fixed seed then the libc qsort by size; per path, merge with the previous
 * state (fill_in_missing_fields, :92-100), drop deleted holders, choose P by
 * select_P (:388-401: PCG32 seeded with simple_hash(path), weighted by the
 * cumulative free-space weights, never a holder), and mark NO_P when the
 * item is unchanged against the previous state.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <sys/statvfs.h>
#include <unistd.h>

#include "bcp_host.h"

/* ---- PCG32 (pcg-random.org minimal C, as used at gen/main.c:338-372) ---- */
typedef struct {
    uint64_t state, inc;
} pcg32;

static uint32_t pcg32_next(pcg32 *r)
{
    uint64_t old = r->state;
    r->state = old * 6364136223846793005ULL + (r->inc | 1);
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((-rot) & 31));
}

static void pcg32_seed(pcg32 *r, uint64_t initstate, uint64_t initseq)
{
    r->state = 0u;
    r->inc = (initseq << 1u) | 1u;
    pcg32_next(r);
    r->state += initstate;
    pcg32_next(r);
}

static uint32_t pcg32_bounded(pcg32 *r, uint32_t bound)
{
    uint32_t threshold = -bound % bound;
    for (;;) {
        uint32_t x = pcg32_next(r);
        if (x >= threshold)
            return x % bound;
    }
}

/* simple_hash (gen/main.c:67-74): djb2 over the path's (signed) chars. */
uint32_t bcp_path_hash(const char *p, size_t len)
{
    uint32_t h = 5381;
    for (size_t i = 0; i < len; i++)
        h = h + (h << 5) + (uint32_t)(int32_t)(signed char)p[i];
    return h;
}

/* ---- event set ---------------------------------------------------------- */
typedef struct {
    char *path;
    size_t len;
    int64_t timestamp;
    uint64_t modified, deleted;
    uint64_t size;   /* summed chunk sizes */
} ev_entry;

struct bcp_eventset {
    ev_entry *e;
    size_t n, cap;
    uint32_t *slots;  /* open addressing: index+1, 0 = empty */
    size_t nslots;
    size_t pending_len[MAX_STORAGE_TARGETS]; /* partial record carried between feeds */
    uint8_t *pend[MAX_STORAGE_TARGETS];
};

int bcp_eventset_create(bcp_eventset **out)
{
    if (!out)
        return -EINVAL;
    bcp_eventset *s = calloc(1, sizeof(*s));
    if (!s)
        return -ENOMEM;
    s->nslots = 1024;
    s->slots = calloc(s->nslots, sizeof(uint32_t));
    if (!s->slots) {
        free(s);
        return -ENOMEM;
    }
    *out = s;
    return 0;
}

void bcp_eventset_destroy(bcp_eventset *s)
{
    if (!s)
        return;
    for (size_t i = 0; i < s->n; i++)
        free(s->e[i].path);
    for (int k = 0; k < MAX_STORAGE_TARGETS; k++)
        free(s->pend[k]);
    free(s->e);
    free(s->slots);
    free(s);
}

static uint64_t fnv64(const char *p, size_t n)
{
    uint64_t h = 1469598103934665603ULL;
    for (size_t i = 0; i < n; i++)
        h = (h ^ (uint8_t)p[i]) * 1099511628211ULL;
    return h;
}

static int rehash(bcp_eventset *s)
{
    size_t ns = s->nslots * 2;
    uint32_t *sl = calloc(ns, sizeof(uint32_t));
    if (!sl)
        return -ENOMEM;
    for (size_t i = 0; i < s->n; i++) {
        size_t h = (size_t)fnv64(s->e[i].path, s->e[i].len) & (ns - 1);
        while (sl[h])
            h = (h + 1) & (ns - 1);
        sl[h] = (uint32_t)(i + 1);
    }
    free(s->slots);
    s->slots = sl;
    s->nslots = ns;
    return 0;
}

static int add_event(bcp_eventset *s, int st, const char *path, size_t len, int64_t ts, uint64_t size, uint64_t ev)
{
    if ((s->n + 1) * 2 > s->nslots && rehash(s))
        return -ENOMEM;
    size_t h = (size_t)fnv64(path, len) & (s->nslots - 1);
    ev_entry *e = NULL;
    while (s->slots[h]) {
        ev_entry *c = &s->e[s->slots[h] - 1];
        if (c->len == len && memcmp(c->path, path, len) == 0) {
            e = c;
            break;
        }
        h = (h + 1) & (s->nslots - 1);
    }
    if (!e) {
        if (s->n == s->cap) {
            size_t nc = s->cap ? 2 * s->cap : 256;
            ev_entry *ne = realloc(s->e, nc * sizeof(ev_entry));
            if (!ne)
                return -ENOMEM;
            s->e = ne;
            s->cap = nc;
        }
        e = &s->e[s->n];
        memset(e, 0, sizeof(*e));
        e->path = malloc(len + 1);
        if (!e->path)
            return -ENOMEM;
        memcpy(e->path, path, len);
        e->path[len] = 0;
        e->len = len;
        s->n++;
        s->slots[h] = (uint32_t)s->n;
    }
    /* fih_add_info (file_info_hash.c:24-31) */
    if (ts > e->timestamp)
        e->timestamp = ts;
    if (ev == UNLINK_EVENT)
        e->deleted |= UINT64_C(1) << st;
    else
        e->modified |= UINT64_C(1) << st;
    e->size += size;
    return 0;
}

/* A record's path becomes <store>/st<k>/{chunks,parity}/<path> on every
 * target: beyond the reference's check (relative, gen/main.c:306) it must
 * not carry a NUL (the C string would name another file) or a ".."
 * component (it would name a file outside the store).  process_task
 * applies the same rule. */
int bcpi_path_ok(const char *p, size_t n)
{
    if (n == (size_t)-1)
        n = strlen(p);
    else if (memchr(p, 0, n))
        return 0;
    if (n == 0 || p[0] == '/')
        return 0;
    for (size_t i = 0; i < n;) {
        size_t j = i;
        while (j < n && p[j] != '/')
            j++;
        if (j - i == 2 && p[i] == '.' && p[i + 1] == '.')
            return 0;
        i = j + 1;
    }
    return 1;
}

/* Parse whole records from buf; a trailing partial record is kept for the
 * next call on the same target (feed_targets_with keeps it in its buffer). */
static int parse(bcp_eventset *s, int st, const uint8_t *buf, size_t len, size_t *used)
{
    size_t off = 0;
    while (len - off >= 32) {
        int64_t ts;
        uint64_t size, ev, plen;
        memcpy(&ts, buf + off, 8);
        memcpy(&size, buf + off + 8, 8);
        memcpy(&ev, buf + off + 16, 8);
        memcpy(&plen, buf + off + 24, 8);
        if (plen == 0 || plen > 4096)
            return -EINVAL;
        if (len - off - 32 < plen)
            break;
        const char *path = (const char *)buf + off + 32;
        if (!bcpi_path_ok(path, (size_t)plen))
            return -EINVAL; /* relative to the chunk dir (gen/main.c:306), and inside it */
        int rc = add_event(s, st, path, (size_t)plen, ts, size, ev);
        if (rc)
            return rc;
        off += 32 + (size_t)plen;
    }
    *used = off;
    return 0;
}

int bcp_eventset_feed(bcp_eventset *s, int st, const void *buf, size_t len)
{
    if (!s || st < 0 || st >= MAX_STORAGE_TARGETS || (len && !buf))
        return -EINVAL;
    const uint8_t *b = buf;
    size_t used = 0;
    int rc;
    if (s->pending_len[st]) {
        /* complete the carried partial record first */
        size_t pl = s->pending_len[st];
        uint8_t *tmp = malloc(pl + len);
        if (!tmp)
            return -ENOMEM;
        memcpy(tmp, s->pend[st], pl);
        memcpy(tmp + pl, b, len);
        rc = parse(s, st, tmp, pl + len, &used);
        if (rc) {
            free(tmp);
            return rc;
        }
        size_t rest = pl + len - used;
        uint8_t *np = rest ? malloc(rest) : NULL;
        if (rest && !np) {
            free(tmp);
            return -ENOMEM;
        }
        if (rest)
            memcpy(np, tmp + used, rest);
        free(tmp);
        free(s->pend[st]);
        s->pend[st] = np;
        s->pending_len[st] = rest;
        return 0;
    }
    rc = parse(s, st, b, len, &used);
    if (rc)
        return rc;
    if (used < len) {
        s->pend[st] = malloc(len - used);
        if (!s->pend[st])
            return -ENOMEM;
        memcpy(s->pend[st], b + used, len - used);
        s->pending_len[st] = len - used;
    }
    return 0;
}

int bcp_eventset_feed_file(bcp_eventset *s, int st, const char *path)
{
    if (!s || !path)
        return -EINVAL;
    int fd = open(path, O_RDONLY);
    if (fd < 0)
        return -errno;
    uint8_t buf[64 * 1024];
    int rc = 0;
    for (;;) {
        ssize_t r = read(fd, buf, sizeof(buf));
        if (r < 0) {
            rc = -errno;
            break;
        }
        if (r == 0)
            break;
        if ((rc = bcp_eventset_feed(s, st, buf, (size_t)r)))
            break;
    }
    close(fd);
    if (!rc && s->pending_len[st])
        rc = -EPROTO; /* stream ended inside a record */
    return rc;
}

size_t bcp_eventset_count(const bcp_eventset *s) { return s ? s->n : 0; }

int bcp_eventset_get(const bcp_eventset *s, size_t i, const char **path, int64_t *timestamp, uint64_t *modified,
                     uint64_t *deleted, uint64_t *size)
{
    if (!s || i >= s->n)
        return -EINVAL;
    const ev_entry *e = &s->e[i];
    if (path)
        *path = e->path;
    if (timestamp)
        *timestamp = e->timestamp;
    if (modified)
        *modified = e->modified;
    if (deleted)
        *deleted = e->deleted;
    if (size)
        *size = e->size;
    return 0;
}

/* ---- planning ----------------------------------------------------------- */

/* get_store_weight (gen/main.c:403-427): 1000*log2(%free + 1.1), with an
 * optional free_space.override file (bytes available) in the store dir. */
int bcp_store_weight(int dirfd)
{
    struct statvfs info;
    if (fstatvfs(dirfd, &info) == -1 || info.f_blocks == 0)
        return 0;
    int64_t block_count = (int64_t)info.f_blocks;
    int64_t blocks_free = (int64_t)info.f_bfree;
    int fd = openat(dirfd, "free_space.override", O_RDONLY);
    if (fd != -1) {
        char avail[64] = {0};
        ssize_t r = read(fd, avail, sizeof(avail) - 1);
        close(fd);
        if (r < 0)
            return -EIO;
        long long v = atoll(avail);
        blocks_free = v > 0 ? v : 0;
        blocks_free /= (int64_t)info.f_bsize;
    }
    double pct_free = (double)(100LL * blocks_free / block_count);
    return (int)(1000 * log2(pct_free + 1.1));
}

/* select_P (gen/main.c:388-401) */
static void select_p(const char *path, FileInfo *fi, int ntargets, const int *cum_weight)
{
    if (__builtin_popcountll(fi->locations & L_MASK) == ntargets)
        return;
    /* guard the reference's retry loop: some non-holder must carry weight */
    int any = 0;
    for (int t = 0; t < ntargets && !any; t++)
        any = !TEST_BIT(fi->locations, t) && cum_weight[t] - (t ? cum_weight[t - 1] : 0) > 0;
    if (!any)
        return;
    pcg32 rng;
    pcg32_seed(&rng, bcp_path_hash(path, strlen(path)), 0);
    uint64_t P;
    do {
        int r = (int)pcg32_bounded(&rng, (uint32_t)cum_weight[ntargets - 1]);
        for (P = 0; r >= cum_weight[P]; P++) {
        }
    } while (TEST_BIT(fi->locations, P));
    fi->locations = WITH_P(fi->locations, P);
}

/* fill_in_missing_fields (gen/main.c:92-100) */
static void fill_in_missing(FileInfo *dst, const FileInfo *src)
{
    uint64_t old_P = (uint64_t)GET_P(src->locations);
    dst->locations = (dst->locations | src->locations) & L_MASK;
    /* the reference tests bit old_P with a 64-bit shift; for NO_P (255) x86
     * masks the count to 63, a bit L_MASK has just cleared -> "not set" */
    if (TEST_BIT(dst->locations, old_P & 63) == 0)
        dst->locations = WITH_P(dst->locations, old_P);
    else
        dst->locations = WITH_P(dst->locations, NO_P);
}

static const bcp_work_item *find_prev(const bcp_work_item *prev, size_t nprev, const char *path)
{
    size_t lo = 0, hi = nprev;
    while (lo < hi) {
        size_t mid = (lo + hi) / 2;
        int c = strcmp(prev[mid].path, path);
        if (c == 0)
            return &prev[mid];
        if (c < 0)
            lo = mid + 1;
        else
            hi = mid;
    }
    return NULL;
}

typedef struct {
    uint64_t size;
    uint64_t idx;
} size_index;

/* cmp_entries (gen/main.c:179-189) */
static int cmp_size(const void *a, const void *b)
{
    uint64_t x = ((const size_index *)a)->size, y = ((const size_index *)b)->size;
    if (x < y)
        return -1;
    if (x == y)
        return 0;
    return 1;
}

/*
 * Phase 2's worklist as the reference's coordinators produce it.  Phase 1
 * sends every path to the eater of storage target simple_hash(path) %
 * ntargets (gen/main.c:310, eater_rank_from_st :77-80); each eater keeps its
 * paths in arrival order, shuffles them with the fixed-seed PCG32 and sorts
 * them by total size (:710-711); then the eaters broadcast their lists one
 * round at a time, in MPI rank order (:758-797: communicator rank i is world
 * rank 2i-1, the eater of storage target rank2st[2i-1]), and every round is
 * planned item by item against the DB (:772-788) and given its own lanes
 * (:823).  round_st[r] = the storage target whose eater broadcasts round r
 * (bcp_map_targets derives it as :506-541 does; NULL = target order, the
 * order of every first run).  Arrival order = the event set's first-seen
 * order (targets fed 0, 1, ...: the reference's interleaving of several
 * feeders is not deterministic).  round_start[r] is where round r begins in
 * out; round_start[ntargets] = *nout.
 */
int bcp_plan_rounds_ordered(const bcp_eventset *s, int ntargets, const int *cum_weight, const int *round_st,
                            const bcp_work_item *prev, size_t nprev, bcp_work_item *out, size_t out_cap,
                            size_t *nout, size_t *round_start)
{
    if (!s || ntargets < 1 || ntargets > MAX_STORAGE_TARGETS || !cum_weight || (nprev && !prev) || !nout)
        return -EINVAL;
    if (round_st) { /* a permutation of the targets */
        uint64_t seen = 0;
        for (int r = 0; r < ntargets; r++) {
            if (round_st[r] < 0 || round_st[r] >= ntargets || (seen >> round_st[r] & 1))
                return -EINVAL;
            seen |= UINT64_C(1) << round_st[r];
        }
    }
    if (cum_weight[ntargets - 1] <= 0)
        return -EINVAL;
    for (size_t i = 1; i < nprev; i++)
        if (strcmp(prev[i - 1].path, prev[i].path) >= 0)
            return -EINVAL; /* prev must be sorted by path, unique */
    *nout = s->n;
    if (out_cap < s->n)
        return out ? -ENOSPC : 0;
    size_index *order = malloc((s->n ? s->n : 1) * sizeof(size_index));
    uint32_t *eater = malloc((s->n ? s->n : 1) * sizeof(uint32_t));
    if (!order || !eater) {
        free(order);
        free(eater);
        return -ENOMEM;
    }
    /* bucket by eater in one pass (arrival order kept inside each bucket) */
    size_t start[MAX_STORAGE_TARGETS + 1] = {0};
    for (size_t i = 0; i < s->n; i++) {
        eater[i] = bcp_path_hash(s->e[i].path, strlen(s->e[i].path)) % (uint32_t)ntargets;
        start[eater[i] + 1]++;
    }
    for (int k = 0; k < ntargets; k++)
        start[k + 1] += start[k];
    {
        size_t fill[MAX_STORAGE_TARGETS];
        memcpy(fill, start, sizeof(fill));
        for (size_t i = 0; i < s->n; i++)
            order[fill[eater[i]]++] = (size_index){s->e[i].size, i};
    }
    /* the eaters' buckets in place (target order), then copied round by round */
    size_index *rounds = round_st ? malloc((s->n ? s->n : 1) * sizeof(size_index)) : order;
    if (!rounds) {
        free(order);
        free(eater);
        return -ENOMEM;
    }
    size_t j = 0;
    for (int r = 0; r < ntargets; r++) {
        const int k = round_st ? round_st[r] : r;
        if (round_start)
            round_start[r] = j;
        const size_t m = start[k + 1] - start[k];
        size_index *mine = rounds + j;
        if (round_st)
            memcpy(mine, order + start[k], m * sizeof(size_index));
        /* shuffle (gen/main.c:373-386, a fresh fixed-seed generator per
         * eater) then sort by total size */
        if (m > 1) {
            pcg32 rng = {0x853c49e6748fea9bULL, 0xda3e39cb94b95bdbULL};
            for (size_t i = m - 1; i > 0; i--) {
                size_t r = pcg32_next(&rng) % (i + 1);
                size_index t = mine[r];
                mine[r] = mine[i];
                mine[i] = t;
            }
        }
        /* The reference sorts with the C library's qsort (gen/main.c:711),
         * whose order of equal sizes is the library's: glibc <= 2.36
         * merge-sorts (stable), later versions do not.  Calling the same qsort
         * with the same comparator on the same shuffled array gives the
         * reference's order on any libc. */
        qsort(mine, m, sizeof(size_index), cmp_size);
        for (size_t t = 0; t < m; t++, j++) {
            const ev_entry *e = &s->e[mine[t].idx];
            FileInfo fi = {e->timestamp, WITH_P(e->modified, NO_P)};
            const bcp_work_item *old = find_prev(prev, nprev, e->path);
            if (old)
                fill_in_missing(&fi, &old->fi);
            fi.locations &= ~e->deleted;
            if (P_IS_INVALID(fi.locations))
                select_p(e->path, &fi, ntargets, cum_weight);
            if (old && old->fi.timestamp == fi.timestamp && old->fi.locations == fi.locations)
                fi.locations = WITH_P(fi.locations, NO_P);
            out[j].path = e->path; /* owned by the event set */
            out[j].fi = fi;
        }
    }
    if (round_start)
        round_start[ntargets] = j;
    if (rounds != order)
        free(rounds);
    free(order);
    free(eater);
    return 0;
}

int bcp_plan_rounds(const bcp_eventset *s, int ntargets, const int *cum_weight, const bcp_work_item *prev,
                    size_t nprev, bcp_work_item *out, size_t out_cap, size_t *nout, size_t *round_start)
{
    return bcp_plan_rounds_ordered(s, ntargets, cum_weight, NULL, prev, nprev, out, out_cap, nout, round_start);
}

int bcp_plan_worklist(const bcp_eventset *s, int ntargets, const int *cum_weight, const bcp_work_item *prev,
                      size_t nprev, bcp_work_item *out, size_t out_cap, size_t *nout)
{
    return bcp_plan_rounds(s, ntargets, cum_weight, prev, nprev, out, out_cap, nout, NULL);
}
