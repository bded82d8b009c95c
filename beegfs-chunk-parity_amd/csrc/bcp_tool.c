/*
 * bcp_tool.c -- command-line front end (bin/bcp) over libbcp.so for
 * loopback stores <root>/st<k>/{chunks,parity,db}: the single-node
 * counterpart of the reference's programs.
 *
 *   bcp find-all-chunks <chunks_dir>
 *       bp-find-all-chunks: the record stream on stdout.
 *   bcp parity-gen --complete|--partial [--pipeline|--protocol|--procs] [--fold MODE]
 *                  [--read PATH] [--lanes N] [--force] [--changelog DIR] <store_root> <ntargets>
 *       beegfs-parity-gen + bp-parity-gen (src/beegfs-parity-gen:1-135,
 *       gen/main.c): target bookkeeping, phase 1 from a scan of every
 *       target (--complete) or from record files DIR/st<k> (--partial,
 *       default DIR = <root>/changelog), then one round against the
 *       persistent state.  Engines (byte-identical output):
 *         --pipeline (default): the batched pipeline on every visible GPU --
 *           the faster engine for local stores;
 *         --protocol: the per-rank protocol (process_task, 12 lanes per rank,
 *           ranks as threads) -- the reference's interface;
 *         --procs: the same with one process per target, as under mpirun.
 *       --fold picks the protocol P role's GPU fold: pipelined (default) or
 *       batched; --read the pipeline's read path (bcp_pipeline_opts.read_mode):
 *       auto (default: copy for stores in memory, direct for a cold store on a
 *       disk), copy, or direct (O_DIRECT into the pinned slabs); --read with
 *       --protocol / --procs and --fold with the pipeline are refused (usage):
 *       each names a path the other engines do not have.  A --complete over
 *       an existing state needs --force and first
 *       deletes the old parity data and DBs (the script's clean_old,
 *       :94-108, :120-126).  On success <root>/last-gen-timestamp.
 *   bcp parity-rebuild [--pipeline|--protocol|--procs] [--fold MODE] [--read PATH] [--lanes N]
 *                      [--db DIR] [--corrupt FILE] <store_root> <ntargets> <target>
 *       beegfs-parity-rebuild + bp-parity-rebuild (rebuild/main.c), through
 *       the batched pipeline (default), the per-rank protocol (--protocol)
 *       or rank processes (--procs).
 *
 * Items whose path would leave the store (absolute, "..") are skipped and
 * counted as refused; a run with refused items exits 1.
 *
 * Exit status 0 on success, 1 on any error (message on stderr).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <ftw.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "bcp_task.h"

static int usage(void)
{
    fputs("usage: bcp find-all-chunks <chunks_dir>\n"
          "       bcp parity-gen --complete|--partial [--pipeline|--protocol|--procs] [--fold MODE] [--read PATH]\n"
          "                      [--lanes N] [--force] [--changelog DIR] <store_root> <ntargets>\n"
          "       bcp parity-rebuild [--pipeline|--protocol|--procs] [--fold MODE] [--read PATH] [--lanes N]\n"
          "                          [--db DIR] [--corrupt FILE] <store_root> <ntargets> <target>\n"
          "       engine: --pipeline (default: batched pipeline on every GPU) | --protocol (per-rank\n"
          "               process_task, ranks as threads) | --procs (ranks as processes)\n"
          "       MODE (protocol P-role fold): pipelined (default) | batched\n"
          "       PATH (pipeline read path): auto (default: copy in memory, direct for cold disk stores) | copy |\n"
          "            direct (O_DIRECT)\n"
          "       --read applies to the pipeline only, --fold to --protocol / --procs only\n",
          stderr);
    return 1;
}

static int g_read_mode = BCP_READ_AUTO;

static int read_mode_arg(const char *s)
{
    if (!strcmp(s, "auto"))
        return BCP_READ_AUTO;
    if (!strcmp(s, "copy"))
        return BCP_READ_COPY;
    if (!strcmp(s, "direct"))
        return BCP_READ_DIRECT;
    return -1;
}

static int fold_mode_arg(const char *s)
{
    if (!strcmp(s, "batched"))
        return BCP_FOLD_BATCHED;
    if (!strcmp(s, "pipelined"))
        return BCP_FOLD_PIPELINED;
    return -1;
}

/* The batched pipeline on every visible GPU (each brings its own PCIe link;
 * io threads scale with them).  job_bytes (0: unknown) sizes the slabs: the
 * pipeline cuts a run into batches of at most job / (4 x slots x GPUs)
 * anyway, so bigger slabs would only be pinned and zeroed for nothing -- the
 * setup of a one-shot run (a config-1 --complete: 2 GiB of slabs, 0.25-0.38 s
 * of a 0.6 s process, profiles/r05/pipeline/c1_cli_r5e.jsonl).  Slabs still
 * grow to a stripe that does not fit. */
static int pipeline_on_all_gpus(bcp_pipeline **pl, uint64_t job_bytes)
{
    int ndev = 0;
    bcp_device_count(&ndev);
    const uint64_t devs = ndev > 0 ? (uint64_t)ndev : 1, full = (uint64_t)256 << 20, least = (uint64_t)16 << 20;
    uint64_t slab = full;
    if (job_bytes) {
        slab = job_bytes / (4 * 4 * devs) + 1;
        slab = (slab + least - 1) / least * least;
        slab = slab < least ? least : slab > full ? full : slab;
    }
    const bcp_pipeline_opts o = {0, (size_t)slab, 0, 4, (int)devs, g_read_mode};
    return bcp_pipeline_create(&o, pl);
}

/* Bytes a --complete run stages: the chunk bytes the scan's records announce
 * plus a page per chunk (DIRECT reads place every source at page pitch).
 * Only a --complete run's records are its whole input: a --partial run reads
 * every holder's chunk of each changed stripe, which the changelog's records
 * do not list, so it keeps the library's default slabs (0). */
static uint64_t job_bytes_of(const bcp_eventset *es, int complete)
{
    if (!complete)
        return 0;
    uint64_t total = 0;
    const size_t n = bcp_eventset_count(es);
    for (size_t i = 0; i < n; i++) {
        const char *p;
        int64_t ts;
        uint64_t m, d, sz = 0;
        if (bcp_eventset_get(es, i, &p, &ts, &m, &d, &sz) == 0)
            total += sz + 4096;
    }
    return total;
}

static int fail(const char *what, int rc)
{
    fprintf(stderr, "bcp: %s: %s\n", what, strerror(rc < 0 ? -rc : rc));
    return 1;
}

static int rm_visit(const char *p, const struct stat *sb, int flag, struct FTW *ftw)
{
    (void)sb;
    (void)flag;
    if (ftw->level == 0)
        return 0; /* keep the directory itself */
    return remove(p) != 0 && errno != ENOENT;
}

static int clear_dir(const char *dir)
{
    struct stat sb;
    if (stat(dir, &sb) != 0)
        return errno == ENOENT ? 0 : -errno;
    return nftw(dir, rm_visit, 64, FTW_DEPTH | FTW_PHYS) == 0 ? 0 : -EIO;
}

static int cmd_find(int argc, char **argv)
{
    if (argc != 1)
        return usage();
    int rc = bcp_scan_chunks(argv[0], STDOUT_FILENO, NULL);
    return rc ? fail("find-all-chunks", rc) : 0;
}

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + (double)t.tv_nsec * 1e-9;
}

static int cmd_gen(int argc, char **argv)
{
    const double t_start = now_s();
    int complete = -1, engines = 0, use_pipeline = 1, use_procs = 0, lanes = 12, force = 0, read_arg = 0, fold_arg = 0;
    const char *changelog = NULL;
    int i = 0;
    for (; i < argc && argv[i][0] == '-'; i++) {
        if (!strcmp(argv[i], "--complete"))
            complete = 1;
        else if (!strcmp(argv[i], "--partial"))
            complete = 0;
        else if (!strcmp(argv[i], "--pipeline"))
            engines++, use_pipeline = 1;
        else if (!strcmp(argv[i], "--protocol"))
            engines++, use_pipeline = 0;
        else if (!strcmp(argv[i], "--procs"))
            engines++, use_pipeline = 0, use_procs = 1;
        else if (!strcmp(argv[i], "--fold") && i + 1 < argc) {
            fold_arg = 1;
            if (fold_mode_arg(argv[++i]) < 0 || bcp_task_set_fold_mode(fold_mode_arg(argv[i])) < 0)
                return usage();
        }
        else if (!strcmp(argv[i], "--read") && i + 1 < argc) {
            read_arg = 1;
            if ((g_read_mode = read_mode_arg(argv[++i])) < 0)
                return usage();
        }
        else if (!strcmp(argv[i], "--force"))
            force = 1;
        else if (!strcmp(argv[i], "--lanes") && i + 1 < argc)
            lanes = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--changelog") && i + 1 < argc)
            changelog = argv[++i];
        else
            return usage();
    }
    if (complete < 0 || argc - i != 2 || engines > 1 || (read_arg && !use_pipeline) || (fold_arg && use_pipeline))
        return usage();
    const char *root = argv[i];
    const int ntargets = atoi(argv[i + 1]);
    if (ntargets < 1 || ntargets > MAX_STORAGE_TARGETS || lanes < 1 || lanes > 64)
        return usage();
    char p[4096];
    snprintf(p, sizeof(p), "%s/run_data", root);
    int rc = bcp_check_targets(root, ntargets, p, stderr);
    if (rc)
        return fail("storage targets", rc);
    char ts_path[4096];
    snprintf(ts_path, sizeof(ts_path), "%s/last-gen-timestamp", root);
    struct stat sb;
    if (complete && stat(ts_path, &sb) == 0) {
        if (!force) {
            fputs("bcp: a complete run has already been done; --force deletes all existing parity data\n", stderr);
            return 1;
        }
        for (int k = 0; k < ntargets; k++) {
            snprintf(p, sizeof(p), "%s/st%d/parity", root, k);
            if ((rc = clear_dir(p)))
                return fail("removing old parity data", rc);
            snprintf(p, sizeof(p), "%s/st%d/db", root, k);
            if ((rc = clear_dir(p)))
                return fail("removing old parity databases", rc);
        }
    }
    const time_t started = time(NULL);
    const double t_phase1 = now_s();
    bcp_eventset *es = NULL;
    if ((rc = bcp_eventset_create(&es)))
        return fail("event set", rc);
    uint64_t nrec = 0;
    for (int k = 0; k < ntargets && !rc; k++) {
        if (complete) {
            uint64_t n = 0;
            snprintf(p, sizeof(p), "%s/st%d/chunks", root, k);
            rc = bcp_eventset_scan(es, k, p, &n);
            nrec += n;
        } else {
            if (changelog)
                snprintf(p, sizeof(p), "%s/st%d", changelog, k);
            else
                snprintf(p, sizeof(p), "%s/changelog/st%d", root, k);
            if (stat(p, &sb) == 0)
                rc = bcp_eventset_feed_file(es, k, p);
        }
    }
    if (rc) {
        bcp_eventset_destroy(es);
        return fail(complete ? "scanning chunks" : "reading changelog", rc);
    }
    printf("Total number of events found: %8zu\n", bcp_eventset_count(es));
    const double t_round = now_s();
    double t_setup = t_round;
    bcp_run_stats st;
    memset(&st, 0, sizeof(st));
    size_t planned = 0;
    if (use_pipeline) {
        bcp_pipeline *pl = NULL;
        rc = pipeline_on_all_gpus(&pl, job_bytes_of(es, complete == 1));
        t_setup = now_s();
        if (!rc)
            rc = bcp_gen_round_pipeline(pl, root, ntargets, es, NULL, stderr, &st, &planned);
        if (pl)
            bcp_pipeline_destroy(pl);
    } else if (use_procs) {
        rc = bcp_gen_round_procs(root, ntargets, es, NULL, lanes, stderr, &st, &planned);
    } else {
        rc = bcp_gen_round(root, ntargets, es, NULL, lanes, stderr, &st, &planned);
        bcp_task_shutdown();
    }
    bcp_eventset_destroy(es);
    if (rc)
        return fail("parity generation", rc);
    const double t_end = now_s();
    printf("worklist %zu items, %llu tasks, %.3f s, %.1f MiB read, %.1f MiB written, %d rank errors, "
           "%llu refused (%s)\n",
           planned, (unsigned long long)st.tasks, st.seconds, st.bytes_read / 1048576.0,
           st.bytes_written / 1048576.0, st.errors, (unsigned long long)st.refused,
           use_pipeline ? "pipeline" : use_procs ? "rank processes" : "protocol");
    /* stage timings, as the reference's rank 0 prints them (gen/main.c:920-928) */
    printf("timings: init %.3f s, phase1 %.3f s, engine setup %.3f s, round %.3f s (run %.3f s), total %.3f s\n",
           t_phase1 - t_start, t_round - t_phase1, t_setup - t_round, t_end - t_setup, st.seconds, t_end - t_start);
    if (st.refused)
        fprintf(stderr, "bcp: %llu item(s) refused: paths outside the store have no parity\n",
                (unsigned long long)st.refused);
    if (st.errors || st.refused)
        return 1;
    FILE *f = fopen(ts_path, "w");
    if (!f)
        return fail("last-gen-timestamp", errno);
    fprintf(f, "%lld\n", (long long)started);
    fclose(f);
    (void)nrec;
    return 0;
}

static int cmd_rebuild(int argc, char **argv)
{
    const char *db = NULL, *corrupt = NULL;
    int engines = 0, use_pipeline = 1, use_procs = 0, read_arg = 0, fold_arg = 0;
    int i = 0;
    for (; i < argc && argv[i][0] == '-'; i++) {
        if (!strcmp(argv[i], "--db") && i + 1 < argc)
            db = argv[++i];
        else if (!strcmp(argv[i], "--corrupt") && i + 1 < argc)
            corrupt = argv[++i];
        else if (!strcmp(argv[i], "--pipeline"))
            engines++, use_pipeline = 1;
        else if (!strcmp(argv[i], "--protocol"))
            engines++, use_pipeline = 0;
        else if (!strcmp(argv[i], "--procs"))
            engines++, use_pipeline = 0, use_procs = 1;
        else if (!strcmp(argv[i], "--fold") && i + 1 < argc) {
            fold_arg = 1;
            if (fold_mode_arg(argv[++i]) < 0 || bcp_task_set_fold_mode(fold_mode_arg(argv[i])) < 0)
                return usage();
        } else if (!strcmp(argv[i], "--read") && i + 1 < argc) {
            read_arg = 1;
            if ((g_read_mode = read_mode_arg(argv[++i])) < 0)
                return usage();
        } else if (!strcmp(argv[i], "--lanes") && i + 1 < argc) {
            if (bcp_task_set_rebuild_lanes(atoi(argv[++i])) < 0) /* (the reference rebuilds with one) */
                return usage();
        } else
            return usage();
    }
    if (argc - i != 3 || engines > 1 || (read_arg && !use_pipeline) || (fold_arg && use_pipeline))
        return usage();
    const char *root = argv[i];
    const int ntargets = atoi(argv[i + 1]), target = atoi(argv[i + 2]);
    bcp_run_stats st;
    memset(&st, 0, sizeof(st));
    int rc;
    if (use_pipeline || use_procs) {
        char dp[4096];
        if (!db) {
            snprintf(dp, sizeof(dp), "%s/st%d/db", root, target == 0 ? 1 : 0);
            db = dp;
        }
        struct stat sb;
        bcp_pdb *pdb = NULL;
        bcp_work_item *items = NULL;
        size_t n = 0;
        rc = stat(db, &sb) == 0 ? 0 : -errno;
        if (!rc)
            rc = bcp_pdb_open(db, DB_VERSION, &pdb);
        if (!rc) {
            rc = bcp_pdb_items(pdb, &items, &n);
            bcp_pdb_close(pdb);
        }
        if (!rc && use_procs) {
            rc = bcp_rebuild_run_procs(root, ntargets, target, items, n, corrupt, stderr, &st);
        } else if (!rc) {
            bcp_pipeline *pl = NULL;
            rc = pipeline_on_all_gpus(&pl, 0);
            if (!rc)
                rc = bcp_pipeline_rebuild(pl, root, ntargets, target, items, n, corrupt, stderr, &st);
            if (pl)
                bcp_pipeline_destroy(pl);
        }
        bcp_pdb_items_free(items);
    } else {
        rc = bcp_rebuild_run_db(root, ntargets, target, db, corrupt, stderr, &st);
        bcp_task_shutdown();
    }
    if (rc)
        return fail("rebuild", rc);
    printf("rebuilt target %d: %llu tasks, %.3f s, %.1f MiB read, %.1f MiB written, %d rank errors, "
           "%llu refused (%s)\n",
           target, (unsigned long long)st.tasks, st.seconds, st.bytes_read / 1048576.0,
           st.bytes_written / 1048576.0, st.errors, (unsigned long long)st.refused,
           use_pipeline ? "pipeline" : use_procs ? "rank processes" : "protocol");
    return (st.errors || st.refused) ? 1 : 0;
}

int main(int argc, char **argv)
{
    if (argc < 2)
        return usage();
    if (!strcmp(argv[1], "find-all-chunks"))
        return cmd_find(argc - 2, argv + 2);
    if (!strcmp(argv[1], "parity-gen"))
        return cmd_gen(argc - 2, argv + 2);
    if (!strcmp(argv[1], "parity-rebuild"))
        return cmd_rebuild(argc - 2, argv + 2);
    return usage();
}
