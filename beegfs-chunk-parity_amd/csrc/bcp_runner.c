/*
 * bcp_runner.c -- the callers of process_task, as loopback ranks.
 *
 *   bcp_assign_lanes  gen/assign_lanes.c:12-46
 *   bcp_gen_run       gen/main.c:116-164 (process_list) + the lane launch at
 *                     :821-889 and the per-rank HostState setup at :723-743
 *   bcp_rebuild_run   rebuild/main.c:40-89 (do_file) + setup at :200-225
 *   bcp_gen_run_db / bcp_rebuild_run_db / bcp_gen_round
 *                     the same with the persistent state: per-target DB
 *                     replicas updated after every task (gen/main.c:146-149),
 *                     rebuild walking a DB in key order (rebuild/main.c:
 *                     223-225), and a whole phase-2 round from chunk events
 *                     (gen/main.c:716-797: load DB, plan, run)
 *
 * Every storage target k is rank k+1 (rank 0 is the coordinator, idle here
 * as in the reference's phase 2), with its store at <root>/st<k>/{chunks,
 * parity}: a set of threads of this process on the loopback transport, or
 * (bcp_*_run_procs, the rank pool in bcp_pool.c) a process of its own on the
 * socketpair transport, as the reference's ranks are under mpirun.  Lane threads start behind a gate: if
 * one cannot be created, none has begun a task, so the others are released
 * without work and joined, and the run returns -EAGAIN (no partner lane is
 * ever left waiting for a rank that does not exist).  The worklist is shared memory instead of an
 * MPI_Bcast (gen/main.c:794-797); every rank still walks it in the same order,
 * which is what keeps the per-(pair, tag) message order consistent.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <dlfcn.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "bcp_runner.h"

#define PER_LANE 16
#define LANE_MASK 15

void bcp_assign_lanes(int nlanes, uint64_t njobs, const FileInfo *jobs, int *lane)
{
    if (nlanes <= 0 || !lane)
        return;
    uint64_t *prev = calloc((size_t)nlanes * PER_LANE, sizeof(uint64_t));
    int *offsets = calloc((size_t)nlanes, sizeof(int));
    if (!prev || !offsets) {
        for (uint64_t i = 0; i < njobs; i++)
            lane[i] = (int)(i % (uint64_t)nlanes);
        free(prev);
        free(offsets);
        return;
    }
    for (uint64_t i = 0; i < njobs; i++) {
        /* The reference forms the P bit as (1 << GET_P(x)) with an int: on
         * x86-64 the shift count is taken mod 32 and the int sign-extends
         * into the u64 mask.  Reproduced so lanes match for every P,
         * including NO_P items (assigned, then skipped by process_list). */
        const uint32_t p = (uint32_t)GET_P(jobs[i].locations);
        const uint64_t pbit = (uint64_t)(int64_t)(int32_t)(UINT32_C(1) << (p & 31u));
        const uint64_t target = (jobs[i].locations & L_MASK) | pbit;
        const int lane_offset = (int)(i % (uint64_t)nlanes);
        int best_idx = lane_offset;
        int best_so_far = 0;
        for (int j0 = 0; j0 < nlanes; j0++) {
            const int j = (lane_offset + j0) % nlanes;
            int dist = PER_LANE;
            const int off = offsets[j];
            /* distance to the most recent task in lane j that shares a target */
            for (int k = 0; k < PER_LANE; k++)
                if (target & prev[j * PER_LANE + ((off + k) & LANE_MASK)])
                    dist = PER_LANE - k;
            if (dist > best_so_far) {
                best_so_far = dist;
                best_idx = j;
            }
        }
        lane[i] = best_idx;
        prev[best_idx * PER_LANE + offsets[best_idx]] = target;
        offsets[best_idx] = (offsets[best_idx] + 1) & LANE_MASK;
    }
    free(offsets);
    free(prev);
}

void bcp_assign_lanes_rounds(int nlanes, int nrounds, const size_t *round_start, const FileInfo *jobs, int *lane)
{
    for (int r = 0; r < nrounds; r++)
        bcp_assign_lanes(nlanes, (uint64_t)(round_start[r + 1] - round_start[r]), jobs + round_start[r],
                         lane + round_start[r]);
}

double bcpr_now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + (double)t.tv_nsec * 1e-9;
}

/* ---- per-target host state -------------------------------------------- */

int bcpr_open_store(const char *root, int st, int rebuilding, int corrupt_fd, FILE *log, HostState *hs)
{
    char path[4096];
    memset(hs, 0, sizeof(*hs));
    hs->storage_target = st;
    hs->log = log;
    hs->corrupt_files_fd = corrupt_fd;
    snprintf(path, sizeof(path), "%s/st%d", root, st);
    int store_fd = open(path, O_DIRECTORY | O_RDONLY);
    if (store_fd < 0)
        return -errno;
    if (mkdirat(store_fd, "parity", 0700) == -1 && errno != EEXIST) {
        close(store_fd);
        return -errno;
    }
    hs->fd_null = open("/dev/null", O_WRONLY);
    hs->fd_zero = open("/dev/zero", O_RDONLY);
    int chunks = openat(store_fd, "chunks", O_DIRECTORY | O_RDONLY);
    int parity = openat(store_fd, "parity", O_DIRECTORY | O_RDONLY);
    close(store_fd);
    if (chunks < 0 || parity < 0 || hs->fd_null < 0 || hs->fd_zero < 0)
        return -ENOENT;
    if (rebuilding) {
        /* rebuild/main.c:210-212: rebuilt chunks are written into chunks/ */
        hs->write_dir = chunks;
        hs->read_chunk_dir = chunks;
        hs->read_parity_dir = parity;
    } else {
        /* gen/main.c:740-742 */
        hs->write_dir = parity;
        hs->read_chunk_dir = chunks;
        hs->read_parity_dir = -1;
        /* keep the parity fd open through write_dir only */
    }
    return 0;
}

void bcpr_close_store(HostState *hs, int rebuilding)
{
    if (hs->fd_null > 0)
        close(hs->fd_null);
    if (hs->fd_zero > 0)
        close(hs->fd_zero);
    if (hs->read_chunk_dir > 0)
        close(hs->read_chunk_dir);
    if (rebuilding) {
        if (hs->read_parity_dir > 0)
            close(hs->read_parity_dir);
    } else if (hs->write_dir > 0) {
        close(hs->write_dir);
    }
    if (hs->error && hs->log)
        fprintf(hs->log, "started using zero/null after '%s' gave error %d (%s) on st %d\n",
                hs->error_path ? hs->error_path : "?", hs->error, strerror(hs->error), hs->storage_target);
}

/* ---- start gate ----------------------------------------------------------- */
/* Lane side: wait until the runner opens the gate; 1 = run, 0 = cancelled. */
int bcpr_gate_pass(start_gate *g)
{
    pthread_mutex_lock(&g->mu);
    while (!g->open)
        pthread_cond_wait(&g->cv, &g->mu);
    const int run = !g->cancel;
    pthread_mutex_unlock(&g->mu);
    return run;
}

void bcpr_gate_open(start_gate *g, int cancel)
{
    pthread_mutex_lock(&g->mu);
    g->cancel = cancel;
    g->open = 1;
    pthread_cond_broadcast(&g->cv);
    pthread_mutex_unlock(&g->mu);
}

int bcpr_spawn(pthread_t *th, void *(*fn)(void *), void *arg)
{
    if (bcpi_inject_hit(BCP_INJECT_THREAD))
        return EAGAIN;
    return pthread_create(th, NULL, fn, arg);
}

/* ---- generation lanes --------------------------------------------------- */

/* Items a run skips for their path (process_task refuses a path that would
 * leave the store on every rank): gen counts every item with a P, rebuild
 * the items do_file's skip rules keep (rebuild_target >= 0). */
uint64_t bcpr_count_refused(const bcp_work_item *items, size_t nitems, int rebuild_target)
{
    uint64_t n = 0;
    for (size_t i = 0; i < nitems; i++) {
        const uint64_t loc = items[i].fi.locations;
        const int P = GET_P(loc);
        if ((uint64_t)P == NO_P)
            continue;
        if (rebuild_target >= 0 && (P == rebuild_target || !TEST_BIT(loc, rebuild_target)))
            continue;
        n += !bcpi_path_ok(items[i].path, (size_t)-1);
    }
    return n;
}

/* process_list (gen/main.c:116-164) for one lane of one rank. */
void *bcpr_gen_lane(void *p)
{
    lane_arg *a = p;
    if (!bcpr_gate_pass(a->gate))
        return NULL;
    bcp_lb_set_rank(a->rank);
    /* a lane without a DB lets its P tasks' writes trail by one task (a DB
     * entry must not precede its parity file) */
    (void)bcp_task_set_lane_deferral(a->db == NULL ? bcpi_defer_depth() : 0);
    TaskInfo ti = {a->hs->read_chunk_dir, 0, -1, a->lane, &a->sample};
    for (size_t i = 0; i < a->nitems; i++) {
        if (a->lanes[i] != a->lane)
            continue;
        if ((uint64_t)GET_P(a->items[i].fi.locations) == NO_P)
            continue;
        double t0 = bcpr_now_s();
        int report = process_task(a->hs, a->items[i].path, &a->items[i].fi, ti);
        if (a->db && bcpi_path_ok(a->items[i].path, (size_t)-1)) {
            /* gen/main.c:146-149: keep the entry while it has holders (a
             * refused path got no parity: the DB must not claim it has) */
            const char *key = a->items[i].path;
            int rc = (a->items[i].fi.locations & L_MASK) ? bcp_pdb_set(a->db, key, strlen(key), &a->items[i].fi)
                                                          : bcp_pdb_del(a->db, key, strlen(key));
            if (rc && !a->db_rc)
                a->db_rc = rc;
        }
        if (report) {
            a->sample.dt += bcpr_now_s() - t0;
            a->sample.nfiles += 1;
            a->tasks++;
        }
    }
    bcp_task_thread_release(); /* (completes a deferred P task first) */
    (void)bcp_task_set_lane_deferral(0);
    return NULL;
}

/* <root>/st<k>/db, the replica of storage target k. */
static int db_path(const char *root, int k, char *out, size_t cap)
{
    int n = snprintf(out, cap, "%s/st%d/db", root, k);
    return (n < 0 || (size_t)n >= cap) ? -ENAMETOOLONG : 0;
}

int bcpr_check_items(int ntargets, const bcp_work_item *items, size_t nitems)
{
    for (size_t i = 0; i < nitems; i++) {
        uint64_t loc = items[i].fi.locations;
        if (!items[i].path || strlen(items[i].path) == 0)
            return -EINVAL;
        if ((loc & L_MASK) >> ntargets)
            return -EINVAL; /* chunk on a target outside the world */
        int P = GET_P(loc);
        if ((uint64_t)P != NO_P && (P >= ntargets || TEST_BIT(loc, P)))
            return -EINVAL; /* process_task asserts P_IS_INVALID == 0 */
    }
    return 0;
}

static int gen_run_impl(const char *store_root, int ntargets, const bcp_work_item *items, size_t nitems,
                        int nlanes, const int *lanes_in, int use_db, FILE *log, bcp_run_stats *stats);

int bcp_gen_run(const char *store_root, int ntargets, const bcp_work_item *items, size_t nitems, int nlanes,
                const int *lanes_in, FILE *log, bcp_run_stats *stats)
{
    return gen_run_impl(store_root, ntargets, items, nitems, nlanes, lanes_in, 0, log, stats);
}

int bcp_gen_run_db(const char *store_root, int ntargets, const bcp_work_item *items, size_t nitems, int nlanes,
                   const int *lanes_in, FILE *log, bcp_run_stats *stats)
{
    return gen_run_impl(store_root, ntargets, items, nitems, nlanes, lanes_in, 1, log, stats);
}

static int gen_run_impl(const char *store_root, int ntargets, const bcp_work_item *items, size_t nitems,
                        int nlanes, const int *lanes_in, int use_db, FILE *log, bcp_run_stats *stats)
{
    if (!store_root || ntargets < 1 || ntargets > MAX_STORAGE_TARGETS || nlanes < 1 || nlanes > 64 ||
        (nitems && !items))
        return -EINVAL;
    int rc = bcpr_check_items(ntargets, items, nitems);
    if (rc)
        return rc;
    int *lanes = NULL;
    if (!lanes_in) {
        FileInfo *fis = malloc((nitems ? nitems : 1) * sizeof(FileInfo));
        lanes = malloc((nitems ? nitems : 1) * sizeof(int));
        if (!fis || !lanes) {
            free(fis);
            free(lanes);
            return -ENOMEM;
        }
        for (size_t i = 0; i < nitems; i++)
            fis[i] = items[i].fi;
        bcp_assign_lanes(nlanes, nitems, fis, lanes);
        free(fis);
    }
    const int *use_lanes = lanes_in ? lanes_in : lanes;
    for (int k = 0; k < MAX_STORAGE_TARGETS; k++)
        st2rank[k] = k < ntargets ? k + 1 : -1;
    if ((rc = bcp_lb_init(ntargets + 1))) {
        free(lanes);
        return rc;
    }
    HostState *hs = calloc((size_t)ntargets, sizeof(HostState));
    lane_arg *args = calloc((size_t)ntargets * nlanes, sizeof(lane_arg));
    pthread_t *th = calloc((size_t)ntargets * nlanes, sizeof(pthread_t));
    bcp_pdb **dbs = calloc((size_t)ntargets, sizeof(bcp_pdb *));
    if (!hs || !args || !th || !dbs) {
        rc = -ENOMEM;
        goto out;
    }
    for (int k = 0; k < ntargets; k++)
        if ((rc = bcpr_open_store(store_root, k, 0, -1, log, &hs[k])))
            goto out;
    for (int k = 0; use_db && k < ntargets; k++) {
        char dp[4096];
        if ((rc = db_path(store_root, k, dp, sizeof(dp))) || (rc = bcp_pdb_open(dp, DB_VERSION, &dbs[k])))
            goto out;
    }
    double t0 = bcpr_now_s();
    int started = 0, spawn_rc = 0;
    start_gate gate = START_GATE_INIT;
    for (int k = 0; k < ntargets && !spawn_rc; k++)
        for (int l = 0; l < nlanes && !spawn_rc; l++) {
            lane_arg *a = &args[k * nlanes + l];
            a->hs = &hs[k];
            a->items = items;
            a->nitems = nitems;
            a->lanes = use_lanes;
            a->lane = l;
            a->rank = k + 1;
            a->db = dbs[k];
            a->gate = &gate;
            if ((spawn_rc = bcpr_spawn(&th[started], bcpr_gen_lane, a)) == 0)
                started++;
        }
    bcpr_gate_open(&gate, spawn_rc != 0);
    for (int i = 0; i < started; i++)
        pthread_join(th[i], NULL);
    if (spawn_rc) {
        if (log)
            fprintf(log, "bcp_gen_run: lane thread %d of %d not created (%s); no task was started\n", started,
                    ntargets * nlanes, strerror(spawn_rc));
        rc = -EAGAIN;
        goto out;
    }
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        stats->seconds = bcpr_now_s() - t0;
        for (int i = 0; i < started; i++) {
            stats->tasks += args[i].tasks;
            stats->bytes_read += args[i].sample.bytes_read;
            stats->bytes_written += args[i].sample.bytes_written;
        }
        for (int k = 0; k < ntargets; k++)
            stats->errors += hs[k].error != 0;
        stats->refused = bcpr_count_refused(items, nitems, -1);
    }
    for (int i = 0; i < started && !rc; i++)
        rc = args[i].db_rc;
out:
    if (hs)
        for (int k = 0; k < ntargets; k++)
            bcpr_close_store(&hs[k], 0);
    if (dbs)
        for (int k = 0; k < ntargets; k++)
            if (dbs[k]) {
                int crc = bcp_pdb_close(dbs[k]);
                if (!rc && crc)
                    rc = crc;
            }
    free(dbs);
    {
        int frc = bcp_lb_finalize();
        if (!rc && frc)
            rc = frc; /* unmatched messages: a protocol bug */
    }
    free(th);
    free(args);
    free(hs);
    free(lanes);
    return rc;
}

/* ---- rebuild ------------------------------------------------------------ */

/* Rebuild lanes (bcp_task_set_rebuild_lanes): the reference rebuilds with
 * one lane (rebuild/main.c walks its DB in one thread, tag 0); tasks are
 * independent, so L lanes per rank -- item i on lane i % L with tag i % L,
 * the same on every rank since every rank walks the same list -- give the
 * same files, the corrupt lists' lines possibly in another order. */
static int g_rebuild_lanes = 1;

int bcp_task_set_rebuild_lanes(int nlanes)
{
    if (nlanes < 1 || nlanes > 64)
        return -EINVAL;
    return __atomic_exchange_n(&g_rebuild_lanes, nlanes, __ATOMIC_ACQ_REL);
}

int bcpr_rebuild_lanes(void)
{
    return __atomic_load_n(&g_rebuild_lanes, __ATOMIC_ACQUIRE);
}

/* do_file (rebuild/main.c:40-89) over the whole item list, one lane. */
void *bcpr_rebuild_rank(void *p)
{
    rebuild_arg *a = p;
    if (a->gate && !bcpr_gate_pass(a->gate))
        return NULL;
    bcp_lb_set_rank(a->rank);
    (void)bcp_task_set_lane_deferral(bcpi_defer_depth());
    const int my_st = a->hs->storage_target;
    const int victim = a->rebuild_target;
    const int nl = a->nlanes > 1 ? a->nlanes : 1;
    for (size_t i = 0; i < a->nitems; i++) {
        if (nl > 1 && (int)(i % (size_t)nl) != a->lane)
            continue;
        const FileInfo *fi = &a->items[i].fi;
        const int P = GET_P(fi->locations);
        if ((uint64_t)P == NO_P || P == victim || TEST_BIT(fi->locations, victim) == 0)
            continue;
        FileInfo mod = *fi;
        /* the parity holder becomes a source, the victim the new "P" */
        mod.locations |= UINT64_C(1) << P;
        mod.locations &= ~(UINT64_C(1) << victim);
        mod.locations = WITH_P(mod.locations, (uint64_t)victim);
        const int rdir = (P == my_st) ? a->hs->read_parity_dir : a->hs->read_chunk_dir;
        TaskInfo ti = {rdir, 1, P, nl > 1 ? a->lane : 0, &a->sample};
        double t0 = bcpr_now_s();
        if (process_task(a->hs, a->items[i].path, &mod, ti)) {
            a->sample.dt += bcpr_now_s() - t0;
            a->sample.nfiles += 1;
            a->tasks++;
        }
    }
    bcp_task_thread_release(); /* (completes a deferred P task first) */
    (void)bcp_task_set_lane_deferral(0);
    return NULL;
}

int bcp_rebuild_run(const char *store_root, int ntargets, int rebuild_target, const bcp_work_item *items,
                    size_t nitems, const char *corrupt_list_path, FILE *log, bcp_run_stats *stats)
{
    if (!store_root || ntargets < 2 || ntargets > MAX_STORAGE_TARGETS || rebuild_target < 0 ||
        rebuild_target >= ntargets || (nitems && !items))
        return -EINVAL;
    int rc = bcpr_check_items(ntargets, items, nitems);
    if (rc)
        return rc;
    for (int k = 0; k < MAX_STORAGE_TARGETS; k++)
        st2rank[k] = k < ntargets ? k + 1 : -1;
    int corrupt_fd = -1;
    if (corrupt_list_path) {
        corrupt_fd = open(corrupt_list_path, O_WRONLY | O_CREAT | O_TRUNC | O_APPEND, S_IRUSR | S_IWUSR);
        if (corrupt_fd < 0)
            return -errno;
    } else {
        corrupt_fd = open("/dev/null", O_WRONLY);
    }
    if ((rc = bcp_lb_init(ntargets + 1))) {
        close(corrupt_fd);
        return rc;
    }
    const int nl = bcpr_rebuild_lanes();
    HostState *hs = calloc((size_t)ntargets, sizeof(HostState));
    rebuild_arg *args = calloc((size_t)ntargets * (size_t)nl, sizeof(rebuild_arg));
    pthread_t *th = calloc((size_t)ntargets * (size_t)nl, sizeof(pthread_t));
    if (!hs || !args || !th) {
        rc = -ENOMEM;
        goto out;
    }
    for (int k = 0; k < ntargets; k++)
        if ((rc = bcpr_open_store(store_root, k, 1, corrupt_fd, log, &hs[k])))
            goto out;
    double t0 = bcpr_now_s();
    int started = 0, spawn_rc = 0;
    start_gate gate = START_GATE_INIT;
    for (int t = 0; t < ntargets * nl && !spawn_rc; t++) {
        const int k = t / nl;
        args[t] = (rebuild_arg){&hs[k], items, nitems, rebuild_target, k + 1, &gate, PROGRESS_SAMPLE_INIT, 0,
                                t % nl, nl};
        if ((spawn_rc = bcpr_spawn(&th[t], bcpr_rebuild_rank, &args[t])) == 0)
            started++;
    }
    bcpr_gate_open(&gate, spawn_rc != 0);
    for (int k = 0; k < started; k++)
        pthread_join(th[k], NULL);
    if (spawn_rc) {
        if (log)
            fprintf(log, "bcp_rebuild_run: lane thread %d of %d not created (%s); no task was started\n", started,
                    ntargets * nl, strerror(spawn_rc));
        rc = -EAGAIN;
        goto out;
    }
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        stats->seconds = bcpr_now_s() - t0;
        for (int t = 0; t < ntargets * nl; t++) {
            stats->tasks += args[t].tasks;
            stats->bytes_read += args[t].sample.bytes_read;
            stats->bytes_written += args[t].sample.bytes_written;
        }
        for (int k = 0; k < ntargets; k++)
            stats->errors += hs[k].error != 0;
        stats->refused = bcpr_count_refused(items, nitems, rebuild_target);
    }
out:
    if (hs)
        for (int k = 0; k < ntargets; k++)
            bcpr_close_store(&hs[k], 1);
    {
        int frc = bcp_lb_finalize();
        if (!rc && frc)
            rc = frc;
    }
    close(corrupt_fd);
    free(th);
    free(args);
    free(hs);
    return rc;
}

/* ---- with the persistent state ------------------------------------------ */

int bcp_rebuild_run_db(const char *store_root, int ntargets, int rebuild_target, const char *db_folder,
                       const char *corrupt_list_path, FILE *log, bcp_run_stats *stats)
{
    if (!store_root || ntargets < 2 || rebuild_target < 0 || rebuild_target >= ntargets)
        return -EINVAL;
    char dp[4096];
    if (!db_folder) {
        /* the replica of the first surviving target (the reference's
         * orchestration copies a surviving DB before a rebuild) */
        int rc = db_path(store_root, rebuild_target == 0 ? 1 : 0, dp, sizeof(dp));
        if (rc)
            return rc;
        db_folder = dp;
    }
    struct stat sb;
    if (stat(db_folder, &sb) != 0)
        return -errno; /* never create an empty DB for a rebuild */
    bcp_pdb *db = NULL;
    int rc = bcp_pdb_open(db_folder, DB_VERSION, &db);
    if (rc)
        return rc;
    bcp_work_item *items = NULL;
    size_t n = 0;
    rc = bcp_pdb_items(db, &items, &n); /* key order, as pdb_iterate */
    bcp_pdb_close(db);
    if (rc)
        return rc;
    rc = bcp_rebuild_run(store_root, ntargets, rebuild_target, items, n, corrupt_list_path, log, stats);
    bcp_pdb_items_free(items);
    return rc;
}

int bcp_store_cum_weights(const char *store_root, int ntargets, int *cum_weight)
{
    if (!store_root || !cum_weight || ntargets < 1 || ntargets > MAX_STORAGE_TARGETS)
        return -EINVAL;
    int total = 0;
    for (int k = 0; k < ntargets; k++) {
        char p[4096];
        int n = snprintf(p, sizeof(p), "%s/st%d", store_root, k);
        if (n < 0 || (size_t)n >= sizeof(p))
            return -ENAMETOOLONG;
        int fd = open(p, O_DIRECTORY | O_RDONLY | O_CLOEXEC);
        if (fd < 0)
            return -errno;
        total += bcp_store_weight(fd); /* get_store_weight, gen/main.c:403-427, 485 */
        close(fd);
        cum_weight[k] = total; /* st_weight (gen/main.c:528-536) */
    }
    return total > 0 ? 0 : -ENOSPC;
}

/* Apply the process_list DB update (gen/main.c:146-149) for every processed
 * item to every replica (the batched pipeline has no per-rank lanes).  The
 * replicas are independent files: one thread each (a changelog round's
 * updates otherwise cost a serial open + replay + append per target). */
typedef struct {
    const char *root;
    int k;
    const bcp_work_item *items;
    size_t n;
    int rc;
} replica_job;

static void *update_replica(void *p)
{
    replica_job *J = p;
    char dp[4096];
    bcp_pdb *db = NULL;
    int rc = db_path(J->root, J->k, dp, sizeof(dp));
    if (!rc)
        rc = bcp_pdb_open(dp, DB_VERSION, &db);
    for (size_t i = 0; i < J->n && !rc; i++) {
        if ((uint64_t)GET_P(J->items[i].fi.locations) == NO_P || !bcpi_path_ok(J->items[i].path, (size_t)-1))
            continue;
        const char *key = J->items[i].path;
        rc = (J->items[i].fi.locations & L_MASK) ? bcp_pdb_set(db, key, strlen(key), &J->items[i].fi)
                                                 : bcp_pdb_del(db, key, strlen(key));
    }
    if (db) {
        int crc = bcp_pdb_close(db);
        if (!rc)
            rc = crc;
    }
    J->rc = rc;
    return NULL;
}

static int update_replicas(const char *root, int ntargets, const bcp_work_item *items, size_t n)
{
    replica_job jobs[MAX_STORAGE_TARGETS];
    pthread_t th[MAX_STORAGE_TARGETS];
    int started[MAX_STORAGE_TARGETS] = {0};
    for (int k = 0; k < ntargets; k++) {
        jobs[k] = (replica_job){root, k, items, n, 0};
        started[k] = pthread_create(&th[k], NULL, update_replica, &jobs[k]) == 0;
        if (!started[k])
            update_replica(&jobs[k]); /* no thread: on this one */
    }
    int rc = 0;
    for (int k = 0; k < ntargets; k++) {
        if (started[k])
            pthread_join(th[k], NULL);
        if (jobs[k].rc && !rc)
            rc = jobs[k].rc;
    }
    return rc;
}

/* Stage times of the latest round in this process (bcp_gen_round_timing). */
static double g_round_t[BCP_ROUND_STAGES];
static pthread_mutex_t g_round_mu = PTHREAD_MUTEX_INITIALIZER;

int bcp_gen_round_timing(double *seconds, int nstages)
{
    if (nstages < 0 || (nstages && !seconds))
        return -EINVAL;
    pthread_mutex_lock(&g_round_mu);
    for (int i = 0; i < nstages && i < BCP_ROUND_STAGES; i++)
        seconds[i] = g_round_t[i];
    pthread_mutex_unlock(&g_round_mu);
    return BCP_ROUND_STAGES;
}

static int round_impl(bcp_pipeline *pl, int procs, const char *store_root, int ntargets, const bcp_eventset *events,
                      const int *cum_weight_in, int nlanes, FILE *log, bcp_run_stats *stats, size_t *nplanned)
{
    double tt[BCP_ROUND_STAGES] = {0};
    double tmark = bcpr_now_s();
    if (!store_root || !events || ntargets < 1 || ntargets > MAX_STORAGE_TARGETS)
        return -EINVAL;
    int cw[MAX_STORAGE_TARGETS];
    int rc = 0;
    if (cum_weight_in)
        memcpy(cw, cum_weight_in, (size_t)ntargets * sizeof(int));
    else if ((rc = bcp_store_cum_weights(store_root, ntargets, cw)))
        return rc;
    /* previous state: the replica of target 0 (all replicas receive the same
     * updates; the reference's eaters read their own, gen/main.c:777) */
    char dp[4096];
    if ((rc = db_path(store_root, 0, dp, sizeof(dp))))
        return rc;
    bcp_pdb *db = NULL;
    if ((rc = bcp_pdb_open(dp, DB_VERSION, &db)))
        return rc;
    bcp_work_item *prev = NULL;
    size_t nprev = 0;
    rc = bcp_pdb_items(db, &prev, &nprev);
    bcp_pdb_close(db);
    if (rc)
        return rc;
    tt[BCP_ROUND_DB_READ] = bcpr_now_s() - tmark;
    tmark = bcpr_now_s();
    size_t n = 0, round_start[MAX_STORAGE_TARGETS + 1];
    bcp_work_item *work = NULL;
    int *lanes = NULL;
    int round_st[MAX_STORAGE_TARGETS];
    rc = bcp_store_round_order(store_root, ntargets, round_st); /* the eaters' rounds in MPI rank order */
    if (!rc)
        rc = bcp_plan_worklist(events, ntargets, cw, prev, nprev, NULL, 0, &n);
    if (!rc) {
        work = malloc((n ? n : 1) * sizeof(bcp_work_item));
        rc = work ? bcp_plan_rounds_ordered(events, ntargets, cw, round_st, prev, nprev, work, n, &n, round_start)
                  : -ENOMEM;
    }
    if (!rc && !pl) {
        /* lanes per coordinator round (gen/main.c:823); the lanes walk the
         * rounds back to back (the reference barriers between rounds, :789;
         * every rank walks the same list, so the messages match either way) */
        FileInfo *fis = malloc((n ? n : 1) * sizeof(FileInfo));
        lanes = malloc((n ? n : 1) * sizeof(int));
        if (!fis || !lanes) {
            rc = -ENOMEM;
        } else {
            for (size_t i = 0; i < n; i++)
                fis[i] = work[i].fi;
            bcp_assign_lanes_rounds(nlanes, ntargets, round_start, fis, lanes);
        }
        free(fis);
    }
    tt[BCP_ROUND_PLAN] = bcpr_now_s() - tmark;
    tmark = bcpr_now_s();
    if (!rc && !pl && !procs)
        rc = bcp_gen_run_db(store_root, ntargets, work, n, nlanes, lanes, log, stats);
    if (!rc && (pl || procs)) {
        bcp_run_stats st;
        memset(&st, 0, sizeof(st));
        rc = pl ? bcp_pipeline_run(pl, store_root, ntargets, work, n, log, &st)
                : bcp_gen_run_procs(store_root, ntargets, work, n, nlanes, lanes, log, &st);
        tt[BCP_ROUND_RUN] = bcpr_now_s() - tmark;
        tmark = bcpr_now_s();
        if (!rc && st.errors == 0)
            rc = update_replicas(store_root, ntargets, work, n); /* only after the parity is on disk */
        tt[BCP_ROUND_REPLICAS] = bcpr_now_s() - tmark;
        if (stats)
            *stats = st;
    } else {
        tt[BCP_ROUND_RUN] = bcpr_now_s() - tmark; /* (the DB runner updates its replicas as it goes) */
    }
    pthread_mutex_lock(&g_round_mu);
    memcpy(g_round_t, tt, sizeof(tt));
    pthread_mutex_unlock(&g_round_mu);
    if (nplanned)
        *nplanned = n;
    free(lanes);
    free(work);
    bcp_pdb_items_free(prev);
    return rc;
}

int bcp_gen_round(const char *store_root, int ntargets, const bcp_eventset *events, const int *cum_weight,
                  int nlanes, FILE *log, bcp_run_stats *stats, size_t *nplanned)
{
    return round_impl(NULL, 0, store_root, ntargets, events, cum_weight, nlanes, log, stats, nplanned);
}

int bcp_gen_round_procs(const char *store_root, int ntargets, const bcp_eventset *events, const int *cum_weight,
                        int nlanes, FILE *log, bcp_run_stats *stats, size_t *nplanned)
{
    return round_impl(NULL, 1, store_root, ntargets, events, cum_weight, nlanes, log, stats, nplanned);
}

int bcp_gen_round_pipeline(bcp_pipeline *pl, const char *store_root, int ntargets, const bcp_eventset *events,
                           const int *cum_weight, FILE *log, bcp_run_stats *stats, size_t *nplanned)
{
    if (!pl)
        return -EINVAL;
    return round_impl(pl, 0, store_root, ntargets, events, cum_weight, 0, log, stats, nplanned);
}
