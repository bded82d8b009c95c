/*
 * bcp_scan.c -- the producers around a generation round on one node:
 *
 *   bcp_scan_chunks / bcp_eventset_scan
 *       bp-find-all-chunks (src/bp-find-all-chunks/main.c:17-45): walk a
 *       store's chunks directory and emit one 'm' record per regular file,
 *       {i64 mtime, u64 size, u64 'm', u64 len, path relative to the chunks
 *       dir}; the --complete input of phase 1 (gen/main.c:622-624).
 *   bcp_check_targets
 *       the storage-target bookkeeping of gen/main.c:472-551 (RunData
 *       "last run" file, targetNumID per store, GIT_VERSION stamp): targets
 *       may be added, never lost, duplicated or moved.
 *
 * The reference's phase-1 scatter (feeders -> eaters by simple_hash(path) %
 * ntargets, gen/main.c:238-336, 576-699) spreads aggregation over MPI ranks;
 * here every target's stream is fed into one event set, target 0 first.  The
 * aggregation is identical (fih_add_info is per path), and so is the order:
 * bcp_plan_rounds re-partitions the event set by the same hash, keeps each
 * eater's paths in first-seen order (= arrival order if feeder k's records
 * reach the eaters before feeder k+1's -- the reference's own interleaving of
 * concurrent feeders is not deterministic) and emits the eaters' rounds in
 * target order (gen/main.c:710-711, 758).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <ftw.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "bcp_task.h"

#define SCAN_BUF (64 * 1024) /* bp-find-all-chunks/main.c:14 */

typedef struct {
    unsigned char buf[SCAN_BUF];
    size_t used;
    int fd;              /* >= 0: write the stream here */
    bcp_eventset *set;   /* else: feed it here */
    int st;
    size_t prefix;       /* strlen(chunks_dir) + 1 */
    int rc;
    uint64_t nrec;
} scan_ctx;

/* nftw has no user pointer; scans are serialised by this lock. */
static pthread_mutex_t g_scan_lock = PTHREAD_MUTEX_INITIALIZER;
static scan_ctx *g_scan;

static int flush_scan(scan_ctx *c)
{
    if (!c->used)
        return 0;
    if (c->fd >= 0) {
        size_t off = 0;
        while (off < c->used) {
            ssize_t w = write(c->fd, c->buf + off, c->used - off);
            if (w < 0 && errno == EINTR)
                continue;
            if (w < 0)
                return -errno;
            off += (size_t)w;
        }
    } else {
        int rc = bcp_eventset_feed(c->set, c->st, c->buf, c->used);
        if (rc)
            return rc;
    }
    c->used = 0;
    return 0;
}

static int visit(const char *fpath, const struct stat *sb, int typeflag, struct FTW *ftw)
{
    (void)ftw;
    scan_ctx *c = g_scan;
    if (typeflag != FTW_F)
        return 0;
    const char *rel = fpath + c->prefix;
    const size_t len = strlen(rel);
    if (len == 0 || len > BCP_PDB_MAX_KEY)
        return 0;
    const uint64_t f[4] = {(uint64_t)(int64_t)sb->st_mtime, (uint64_t)sb->st_size, 'm', len};
    if (sizeof(f) + len + c->used >= sizeof(c->buf) && (c->rc = flush_scan(c)))
        return 1;
    memcpy(c->buf + c->used, f, sizeof(f));
    memcpy(c->buf + c->used + sizeof(f), rel, len);
    c->used += sizeof(f) + len;
    c->nrec++;
    return 0;
}

static int scan(const char *chunks_dir, int fd, bcp_eventset *set, int st, uint64_t *nrec)
{
    if (!chunks_dir || (fd < 0 && !set))
        return -EINVAL;
    struct stat sb;
    if (stat(chunks_dir, &sb) != 0)
        return -errno;
    if (!S_ISDIR(sb.st_mode))
        return -ENOTDIR;
    scan_ctx *c = calloc(1, sizeof(*c));
    if (!c)
        return -ENOMEM;
    c->fd = fd;
    c->set = set;
    c->st = st;
    size_t dl = strlen(chunks_dir);
    while (dl > 1 && chunks_dir[dl - 1] == '/')
        dl--;
    c->prefix = dl + 1;
    char *root = strndup(chunks_dir, dl);
    if (!root) {
        free(c);
        return -ENOMEM;
    }
    pthread_mutex_lock(&g_scan_lock);
    g_scan = c;
    int r = nftw(root, visit, 100, FTW_PHYS); /* ftw(".", visitor, 100) in the reference */
    g_scan = NULL;
    pthread_mutex_unlock(&g_scan_lock);
    int rc = c->rc;
    if (!rc && r < 0)
        rc = -errno;
    if (!rc)
        rc = flush_scan(c);
    if (nrec)
        *nrec = c->nrec;
    free(root);
    free(c);
    return rc;
}

int bcp_scan_chunks(const char *chunks_dir, int out_fd, uint64_t *nrecords)
{
    if (out_fd < 0)
        return -EINVAL;
    return scan(chunks_dir, out_fd, NULL, 0, nrecords);
}

int bcp_eventset_scan(bcp_eventset *s, int st, const char *chunks_dir, uint64_t *nrecords)
{
    if (!s || st < 0 || st >= MAX_STORAGE_TARGETS)
        return -EINVAL;
    return scan(chunks_dir, -1, s, st, nrecords);
}

/* ---- storage-target bookkeeping (gen/main.c:472-551) ------------------- */

#define RUN_MAGIC "BCPRUN01"

/* Stamp of the run_data file's format (the reference's Target.version =
 * GIT_VERSION, checked at gen/main.c:500-502).  The format has not changed
 * since it was introduced (1); the r04 build stamped its struct ABI version 2
 * instead, so 2 reads as the same format and is rewritten as 1. */
#define RUN_DATA_VERSION 1u
#define RUN_DATA_VERSION_R04 2u

typedef struct {
    char magic[8];
    uint32_t version;    /* RUN_DATA_VERSION */
    uint32_t ntargets;
    int32_t ids[MAX_STORAGE_TARGETS];
} run_data;

static int read_target_id(const char *root, int k, int32_t *id)
{
    char p[4096];
    int n = snprintf(p, sizeof(p), "%s/st%d/targetNumID", root, k);
    if (n < 0 || (size_t)n >= sizeof(p))
        return -ENAMETOOLONG;
    FILE *f = fopen(p, "r");
    if (!f) {
        if (errno != ENOENT)
            return -errno;
        *id = k + 1; /* a store without the file: its position is its identity */
        return 0;
    }
    char s[20] = {0};
    size_t got = fread(s, 1, sizeof(s) - 1, f); /* read(target_ID_fd, targetID_s, 20) */
    fclose(f);
    if (!got)
        return -EPROTO;
    *id = atoi(s);
    return 0;
}

/* gen/main.c:498-499, 506-541 on the coordinator after the Gathers: every
 * target found in the previous run's list keeps its storage-target index
 * (a second rank with an id already placed: "Duplicate targetNumID"),
 * targets not in it are appended in rank order, and an index left without a
 * rank is "Storage target missing!"; st2rank[i] = the rank of target i, and
 * round r (communicator rank r+1 = world rank 2r+1, :570-574, :758) is
 * broadcast by the eater of target rank2st[2r+1]. */
int bcp_map_targets(const int32_t *prev_ids, int nprev, const int32_t *rank_ids, int ntargets, int32_t *st_ids,
                    int *round_st)
{
    if (ntargets < 1 || ntargets > MAX_STORAGE_TARGETS || nprev < 0 || nprev > MAX_STORAGE_TARGETS ||
        (nprev && !prev_ids) || !rank_ids || !st_ids || !round_st)
        return -EINVAL;
    if (ntargets < nprev)
        return -ENODEV; /* "Fewer targets than last run, something is wrong!" */
    int32_t ids[2 * MAX_STORAGE_TARGETS];
    int rank_of[2 * MAX_STORAGE_TARGETS];
    for (int j = 0; j < nprev; j++) {
        ids[j] = prev_ids[j];
        rank_of[j] = -1;
    }
    int k = nprev;
    for (int r = 0; r < ntargets; r++) {
        int found = 0;
        for (int j = 0; j < nprev; j++)
            if (ids[j] == rank_ids[r]) {
                if (rank_of[j] != -1)
                    return -EEXIST; /* "Duplicate targetNumID = %d" */
                rank_of[j] = r;
                found = 1;
                break;
            }
        if (!found) {
            ids[k] = rank_ids[r];
            rank_of[k++] = r;
        }
    }
    for (int i = 0; i < ntargets; i++)
        if (rank_of[i] == -1)
            return -ENODEV; /* "Storage target missing! targetNumID = %d" */
    for (int i = 0; i < ntargets; i++) {
        st_ids[i] = ids[i];
        round_st[rank_of[i]] = i;
    }
    return 0;
}

/* <root>/rank_order: the targetNumID of every storage target's eater rank in
 * MPI rank order -- the order of the hosts in the hostfile the parity-gen
 * script builds from etc/hosts (src/beegfs-parity-gen:114-117), whitespace
 * separated.  Absent: target order.  -ENOENT absent, -EPROTO malformed. */
static int read_rank_order(const char *root, int ntargets, int32_t *rank_ids)
{
    char p[4096];
    int n = snprintf(p, sizeof(p), "%s/rank_order", root);
    if (n < 0 || (size_t)n >= sizeof(p))
        return -ENAMETOOLONG;
    FILE *f = fopen(p, "r");
    if (!f)
        return errno == ENOENT ? -ENOENT : -errno;
    int got = 0, rc = 0;
    long v;
    while (fscanf(f, "%ld", &v) == 1) {
        if (got >= ntargets || v < INT32_MIN || v > INT32_MAX) {
            rc = -EPROTO;
            break;
        }
        rank_ids[got++] = (int32_t)v;
    }
    if (!rc && (!feof(f) || got != ntargets))
        rc = -EPROTO;
    fclose(f);
    return rc;
}

int bcp_store_round_order(const char *store_root, int ntargets, int *round_st)
{
    if (!store_root || !round_st || ntargets < 1 || ntargets > MAX_STORAGE_TARGETS)
        return -EINVAL;
    int32_t cur[MAX_STORAGE_TARGETS], rank_ids[MAX_STORAGE_TARGETS], st_ids[MAX_STORAGE_TARGETS];
    int rc = read_rank_order(store_root, ntargets, rank_ids);
    if (rc == -ENOENT) {
        for (int r = 0; r < ntargets; r++)
            round_st[r] = r;
        return 0;
    }
    if (rc)
        return rc;
    for (int k = 0; k < ntargets; k++)
        if ((rc = read_target_id(store_root, k, &cur[k])))
            return rc;
    /* the directories are the persisted index order (bcp_check_targets) */
    return bcp_map_targets(cur, ntargets, rank_ids, ntargets, st_ids, round_st);
}

int bcp_check_targets(const char *store_root, int ntargets, const char *run_data_path, FILE *log)
{
    if (!store_root || !run_data_path || ntargets < 1 || ntargets > MAX_STORAGE_TARGETS)
        return -EINVAL;
    run_data cur;
    memset(&cur, 0, sizeof(cur));
    memcpy(cur.magic, RUN_MAGIC, 8);
    cur.version = RUN_DATA_VERSION;
    cur.ntargets = (uint32_t)ntargets;
    for (int k = 0; k < ntargets; k++) {
        int rc = read_target_id(store_root, k, &cur.ids[k]);
        if (rc)
            return rc;
        for (int j = 0; j < k; j++)
            if (cur.ids[j] == cur.ids[k]) {
                if (log)
                    fprintf(log, "Duplicate targetNumID = %d\n", cur.ids[k]);
                return -EEXIST;
            }
    }
    run_data last;
    memset(&last, 0, sizeof(last));
    int fd = open(run_data_path, O_RDWR | O_CREAT | O_CLOEXEC, 0600);
    if (fd < 0)
        return -errno;
    ssize_t got = read(fd, &last, sizeof(last));
    if (got == (ssize_t)sizeof(last) && !memcmp(last.magic, RUN_MAGIC, 8)) {
        if (last.version != RUN_DATA_VERSION && last.version != RUN_DATA_VERSION_R04) {
            if (log)
                fprintf(log, "Version mismatch\n");
            close(fd);
            return -EPROTO;
        }
        if (cur.ntargets < last.ntargets) {
            if (log)
                fprintf(log, "Fewer targets than last run, something is wrong!\n");
            close(fd);
            return -ENODEV;
        }
        /* targets keep their storage-target index across runs; new ones are
         * appended (gen/main.c:508-526) -- with fixed <root>/st<k> stores an
         * index whose id changed is a lost target */
        for (uint32_t k = 0; k < last.ntargets; k++)
            if (last.ids[k] != cur.ids[k]) {
                if (log)
                    fprintf(log, "Storage target missing! targetNumID = %d\n", last.ids[k]);
                close(fd);
                return -ENODEV;
            }
    } else if (got != 0) {
        close(fd);
        return -EPROTO;
    }
    /* the rank order (<root>/rank_order) against the index order the
     * reference would derive from the previous run's list (gen/main.c:506-541;
     * a first run: the directories' order): targets added since must be
     * numbered st<k> in the order the reference appends them, rank order */
    {
        int32_t rank_ids[MAX_STORAGE_TARGETS], st_ids[MAX_STORAGE_TARGETS];
        int round_st[MAX_STORAGE_TARGETS];
        int rc = read_rank_order(store_root, ntargets, rank_ids);
        if (rc != -ENOENT) {
            const int first = !(got == (ssize_t)sizeof(last));
            if (!rc)
                rc = bcp_map_targets(first ? cur.ids : last.ids, first ? ntargets : (int)last.ntargets, rank_ids,
                                     ntargets, st_ids, round_st);
            for (int k = 0; k < ntargets && !rc; k++)
                if (st_ids[k] != cur.ids[k]) {
                    if (log)
                        fprintf(log, "st%d holds targetNumID %d, but the rank order appends %d there\n", k,
                                cur.ids[k], st_ids[k]);
                    rc = -EPROTO;
                }
            if (rc) {
                if (log && rc != -EPROTO)
                    fprintf(log, "rank_order: %s\n", strerror(-rc));
                close(fd);
                return rc;
            }
        }
    }
    int rc = 0;
    if (pwrite(fd, &cur, sizeof(cur), 0) != (ssize_t)sizeof(cur))
        rc = -EIO;
    close(fd);
    return rc;
}
