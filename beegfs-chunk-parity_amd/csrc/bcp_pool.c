/*
 * bcp_pool.c -- ranks as processes: the rank pool (bcp_rank_pool_*) and the
 * one-run forms bcp_gen_run_procs / bcp_rebuild_run_procs.  Each rank runs
 * the same lanes as the thread runner (bcp_runner.c) inside a process of its
 * own, on the socketpair transport (bcp_sock.c), with its P-role folds sent
 * to the node fold server (bcp_foldsrv.c) by default.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include "bcp_runner.h"

/* ---- ranks as processes: the rank pool -----------------------------------
 * One forked process per storage target, connected by a bcp_sock_world --
 * the shape of the reference's deployment (one MPI process per target,
 * src/beegfs-parity-gen:114-127).  A pool forks its ranks ONCE; every run is
 * a command sent to each rank over its own socketpair (the work items, the
 * lanes and the caller's P-role settings), and each rank answers with one
 * record on a shared result pipe (< PIPE_BUF: atomic).  A rank keeps its HIP
 * engine, fold service and registered window rows from run to run, as a
 * long-lived MPI rank does.  A rank whose run cannot start (store missing,
 * a lane thread not created) reports and exits: its partners see its
 * sockets close and fail the tasks they share with it, and the pool is
 * broken (-EPIPE for later runs).  bcp_gen_run_procs / bcp_rebuild_run_procs
 * are one-run pools. */
typedef struct {
    int rank;
    int error;        /* the rank's sticky error at the end */
    int rc;           /* 0 = ran; < 0: the run could not start (the rank exits) */
    uint64_t seq;     /* the command answered */
    uint64_t tasks, bytes_read, bytes_written;
} rank_report;

#define POOL_MAGIC 0x62637072u /* "bcpr" */
enum { POOL_GEN = 1, POOL_REBUILD = 2, POOL_QUIT = 3 };

typedef struct {
    uint32_t magic, op;
    int32_t nlanes, rebuild_target, has_lanes;
    bcpi_settings settings;
    uint64_t seq, nitems, root_len, corrupt_len, paths_len;
} pool_cmd;

struct bcp_rank_pool {
    int ntargets;
    pid_t pids[MAX_STORAGE_TARGETS]; /* -1 once reaped */
    int cmd_fd[MAX_STORAGE_TARGETS];
    int res_fd;
    int broken;
    uint64_t seq;
    FILE *log;
    pid_t srv_pid; /* node fold server (BCP_FOLD_SERVER), -1 if none */
};

typedef struct {
    const char *root;
    int nlanes, rebuilding, rebuild_target, corrupt_fd;
    const bcp_work_item *items;
    size_t nitems;
    const int *lanes;
    FILE *log;
} procs_job;

static int io_full(int fd, void *buf, size_t n, int writing)
{
    uint8_t *p = buf;
    while (n) {
        ssize_t r = writing ? send(fd, p, n, MSG_NOSIGNAL) : read(fd, p, n);
        if (r < 0 && errno == EINTR)
            continue;
        if (r <= 0)
            return r == 0 ? -EPIPE : -errno;
        p += r;
        n -= (size_t)r;
    }
    return 0;
}

/* One run of rank k+1 inside its process (the lanes of gen, or the single
 * rebuild lane).  rep->rc < 0 if the run could not start. */
static void rank_run(const procs_job *J, int k, rank_report *rep)
{
    HostState hs;
    int rc = bcpr_open_store(J->root, k, J->rebuilding, J->corrupt_fd, J->log, &hs);
    if (!rc && !J->rebuilding) {
        lane_arg *args = calloc((size_t)J->nlanes, sizeof(lane_arg));
        pthread_t *th = calloc((size_t)J->nlanes, sizeof(pthread_t));
        start_gate gate = START_GATE_INIT;
        int started = 0, src = 0;
        if (!args || !th)
            src = ENOMEM;
        for (int l = 0; l < J->nlanes && !src; l++) {
            args[l] = (lane_arg){&hs, J->items, J->nitems, J->lanes, l, k + 1, NULL, &gate, PROGRESS_SAMPLE_INIT, 0, 0};
            if ((src = bcpr_spawn(&th[l], bcpr_gen_lane, &args[l])) == 0)
                started++;
        }
        bcpr_gate_open(&gate, src != 0); /* all lanes or none */
        for (int l = 0; l < started; l++)
            pthread_join(th[l], NULL);
        for (int l = 0; l < started && !src; l++) {
            rep->tasks += args[l].tasks;
            rep->bytes_read += args[l].sample.bytes_read;
            rep->bytes_written += args[l].sample.bytes_written;
        }
        rc = src ? -src : 0;
        free(args);
        free(th);
    } else if (!rc) {
        const int nl = J->nlanes > 1 ? J->nlanes : 1; /* the caller's rebuild lanes */
        rebuild_arg *ra = calloc((size_t)nl, sizeof(rebuild_arg));
        pthread_t *rt = calloc((size_t)nl, sizeof(pthread_t));
        start_gate gate = START_GATE_INIT;
        int started = 0, src = (!ra || !rt) ? ENOMEM : 0;
        for (int l = 0; l < nl && !src; l++) {
            ra[l] = (rebuild_arg){&hs, J->items, J->nitems, J->rebuild_target, k + 1, &gate, PROGRESS_SAMPLE_INIT,
                                  0, l, nl};
            if ((src = bcpr_spawn(&rt[l], bcpr_rebuild_rank, &ra[l])) == 0)
                started++;
        }
        bcpr_gate_open(&gate, src != 0);
        for (int l = 0; l < started; l++) {
            pthread_join(rt[l], NULL);
            rep->tasks += ra[l].tasks;
            rep->bytes_read += ra[l].sample.bytes_read;
            rep->bytes_written += ra[l].sample.bytes_written;
        }
        rc = src ? -src : 0;
        free(ra);
        free(rt);
    }
    if (!rc) {
        rep->error = hs.error;
        bcpr_close_store(&hs, J->rebuilding);
    }
    rep->rc = rc;
}

/* Read one command's payload and run it; returns the report. */
static void rank_command(const pool_cmd *c, int cmd_fd, int k, FILE *log, rank_report *rep)
{
    char *root = NULL, *corrupt = NULL, *paths = NULL;
    FileInfo *fis = NULL;
    uint32_t *plen = NULL;
    int32_t *lanes = NULL;
    bcp_work_item *items = NULL;
    const size_t n = (size_t)c->nitems;
    int rc = 0;
    if (c->root_len == 0 || c->root_len > 4096 || c->corrupt_len > 4096 || c->nitems > ((uint64_t)1 << 32) ||
        c->paths_len > ((uint64_t)1 << 40) || (c->op == POOL_GEN && !c->has_lanes)) {
        rep->rc = -EPROTO;
        return;
    }
    root = calloc(c->root_len + 1, 1);
    corrupt = calloc(c->corrupt_len + 1, 1);
    paths = malloc(c->paths_len + n + 1);
    fis = malloc((n ? n : 1) * sizeof(FileInfo));
    plen = malloc((n ? n : 1) * sizeof(uint32_t));
    lanes = c->has_lanes ? malloc((n ? n : 1) * sizeof(int32_t)) : NULL;
    items = malloc((n ? n : 1) * sizeof(bcp_work_item));
    if (!root || !corrupt || !paths || !fis || !plen || !items || (c->has_lanes && !lanes))
        rc = -ENOMEM;
    /* a rank that cannot take its command whole (the channel would be out
     * of step) reports and exits like any rank whose run cannot start */
    if (!rc)
        rc = io_full(cmd_fd, root, c->root_len, 0);
    if (!rc && c->corrupt_len)
        rc = io_full(cmd_fd, corrupt, c->corrupt_len, 0);
    if (!rc)
        rc = io_full(cmd_fd, fis, n * sizeof(FileInfo), 0);
    if (!rc)
        rc = io_full(cmd_fd, plen, n * sizeof(uint32_t), 0);
    /* paths packed back to back; each gets its NUL here */
    uint64_t total = 0;
    for (size_t i = 0; !rc && i < n; i++)
        total += plen[i];
    if (!rc && total != c->paths_len)
        rc = -EPROTO;
    for (size_t i = 0, off = 0; !rc && i < n; i++) {
        rc = io_full(cmd_fd, paths + off, plen[i], 0);
        paths[off + plen[i]] = 0;
        items[i] = (bcp_work_item){paths + off, fis[i]};
        off += plen[i] + 1;
    }
    if (!rc && c->has_lanes)
        rc = io_full(cmd_fd, lanes, n * sizeof(int32_t), 0);
    int corrupt_fd = -1;
    if (!rc && c->op == POOL_REBUILD) {
        corrupt_fd = c->corrupt_len ? open(corrupt, O_WRONLY | O_CREAT | O_APPEND, S_IRUSR | S_IWUSR)
                                    : open("/dev/null", O_WRONLY);
        if (corrupt_fd < 0)
            rc = -errno;
    }
    /* a hook is a function of the caller's process: usable here only if it
     * was mapped when the pool forked */
    Dl_info dl;
    if (!rc && c->settings.hook && !dladdr((void *)c->settings.hook, &dl))
        rc = -EFAULT;
    if (!rc)
        rc = bcpi_settings_apply(&c->settings);
    if (!rc) {
        procs_job J = {root, c->nlanes, c->op == POOL_REBUILD, c->rebuild_target, corrupt_fd, items, n,
                       (const int *)lanes, log};
        rank_run(&J, k, rep);
    } else {
        rep->rc = rc;
    }
    if (corrupt_fd >= 0)
        close(corrupt_fd);
    free(root);
    free(corrupt);
    free(paths);
    free(fis);
    free(plen);
    free(lanes);
    free(items);
}

/* In a child just forked from a possibly multithreaded caller: set an
 * environment default without setenv, whose lock another thread of the
 * parent may have held at the fork (only this thread exists in the child,
 * and glibc's malloc is made usable again across fork).  The new environ
 * array is the child's for the rest of its life. */
static void child_env_default(const char *name, const char *value)
{
    extern char **environ;
    if (getenv(name))
        return;
    size_t n = 0;
    while (environ && environ[n])
        n++;
    char **env = malloc((n + 2) * sizeof(char *));
    const size_t len = strlen(name) + strlen(value) + 2;
    char *kv = malloc(len);
    if (!env || !kv) {
        free(env);
        free(kv);
        return;
    }
    snprintf(kv, len, "%s=%s", name, value);
    for (size_t i = 0; i < n; i++)
        env[i] = environ[i];
    env[n] = kv;
    env[n + 1] = NULL;
    environ = env;
}

/* The body of rank process k+1 (never returns): serve commands until QUIT
 * or the caller's end closes. */
static void rank_main(bcp_sock_world *w, int k, int cmd_fd, int res_fd, FILE *log, int nconn, const int *srv_fds)
{
    /* Every rank process holds its own HIP context on a GPU that several
     * ranks share.  With HIP's default of 4 hardware queues each, 9 ranks on
     * one MI355X oversubscribed its queues and the GPU fold fell to 11.9 GiB/s
     * (config-5 shapes, below the CPU fold's 16.4); with 2 queues each it ran
     * at 19.9 (1: 20.2) -- profiles/r02/protocol/pool_hwq_r2ab_*.  A rank
     * needs two (a queue's compute and copy streams), so that is the default
     * unless the caller set GPU_MAX_HW_QUEUES; HIP reads it at its first call,
     * which comes after this in the rank. */
    child_env_default("GPU_MAX_HW_QUEUES", "2");
    /* P-role rows inherited from the caller (host memory: the caller has no
     * HIP runtime here) go; this rank takes its rows from its arena slice */
    bcp_task_shutdown();
    if (nconn)
        bcpi_foldsrv_attach(nconn, srv_fds); /* folds go to the node fold server */
    bcp_transport_ops ops;
    int arc = bcp_sock_world_attach(w, k + 1, &ops);
    if (!arc)
        arc = bcp_task_set_transport(&ops);
    for (;;) {
        pool_cmd c;
        if (io_full(cmd_fd, &c, sizeof(c), 0) || c.magic != POOL_MAGIC || c.op == POOL_QUIT)
            break;
        rank_report rep = {k + 1, 0, 0, c.seq, 0, 0, 0};
        if (arc)
            rep.rc = arc;
        else
            rank_command(&c, cmd_fd, k, log, &rep);
        if (log && getenv("BCP_SOCK_STATS")) {
            uint64_t fa = 0, fm = 0;
            bcpi_sock_fill_counts(&fa, &fm);
            uint64_t pw = 0, pr = 0;
            bcp_task_pipe_stats(&pw, &pr);
            fprintf(log,
                    "rank %d: fill sends %llu into arena rows, %llu as messages; %llu windows folded by the server;"
                    " pipelined windows %llu ranges %llu\n",
                    k + 1, (unsigned long long)fa, (unsigned long long)fm, (unsigned long long)bcpi_foldsrv_folds(),
                    (unsigned long long)pw, (unsigned long long)pr);
            fflush(log);
        }
        ssize_t wr = write(res_fd, &rep, sizeof(rep));
        (void)wr;
        if (rep.rc)
            break; /* the run could not start: leave, so partners fail fast */
    }
    bcp_task_shutdown();
    close(res_fd);
    close(cmd_fd);
    bcp_sock_world_destroy(w);
    _exit(0);
}

int bcp_rank_pool_create(int ntargets, FILE *log, bcp_rank_pool **out)
{
    if (!out || ntargets < 1 || ntargets > MAX_STORAGE_TARGETS)
        return -EINVAL;
    *out = NULL;
    if (bcpi_hip_touched())
        return -EBUSY; /* children could not use the HIP runtime of this process */
    bcp_rank_pool *P = calloc(1, sizeof(*P));
    if (!P)
        return -ENOMEM;
    P->ntargets = ntargets;
    P->log = log;
    P->res_fd = -1;
    for (int k = 0; k < MAX_STORAGE_TARGETS; k++) {
        P->pids[k] = -1;
        P->cmd_fd[k] = -1;
        st2rank[k] = k < ntargets ? k + 1 : -1; /* inherited by the ranks */
    }
    P->srv_pid = -1;
    bcp_sock_world *w = NULL;
    int rc = bcp_sock_world_create(ntargets + 1, &w);
    int res[2] = {-1, -1};
    if (!rc && pipe(res) != 0)
        rc = -errno;
    if (rc) {
        if (w)
            bcp_sock_world_destroy(w);
        free(P);
        return rc;
    }
    if (log)
        fflush(log);
    fflush(stdout);
    fflush(stderr);
    /* Node fold server (default; environment BCP_FOLD_SERVER=0 turns it
     * off; needs the shared arena): one process holds the GPU for every
     * rank's folds, over BCP_FOLD_SERVER_CONNS (default 12) connections per
     * rank.  Config 5 over nine rank processes on one MI355X (r02): 35-37 GiB/s,
     * against 13-14 with a HIP context per rank. */
    int nconn = 0, *sfd = NULL, *rfd = NULL;
    void *alo = NULL, *ahi = NULL;
    const char *fs = getenv("BCP_FOLD_SERVER");
    if ((!fs || atoi(fs) > 0) && bcpi_sock_world_arena(w, &alo, &ahi)) {
        nconn = getenv("BCP_FOLD_SERVER_CONNS") ? atoi(getenv("BCP_FOLD_SERVER_CONNS")) : 12;
        nconn = nconn < 1 ? 1 : nconn > 64 ? 64 : nconn;
        sfd = malloc(sizeof(int) * (size_t)(ntargets * nconn));
        rfd = malloc(sizeof(int) * (size_t)(ntargets * nconn));
        if (!sfd || !rfd)
            rc = -ENOMEM;
        int made = 0;
        for (; !rc && made < ntargets * nconn; made++) {
            int sv[2];
            if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, sv) != 0) {
                rc = -errno;
                break;
            }
            sfd[made] = sv[0];
            rfd[made] = sv[1];
        }
        pid_t sp = rc ? -1 : fork();
        if (sp == 0) {
            close(res[0]);
            close(res[1]);
            for (int i = 0; i < made; i++)
                close(rfd[i]);
            bcpi_sock_world_close_fds(w); /* the ranks' sockets: EOF must reach partners */
            child_env_default("GPU_MAX_HW_QUEUES", "4");
            bcpi_foldsrv_main(made, sfd, alo, ahi);
            _exit(0);
        }
        for (int i = 0; i < made; i++)
            close(sfd[i]);
        if (sp < 0 && !rc)
            rc = -errno;
        P->srv_pid = sp;
        if (rc) {
            for (int i = 0; i < made; i++)
                close(rfd[i]);
            free(sfd);
            free(rfd);
            close(res[0]);
            close(res[1]);
            bcp_sock_world_destroy(w);
            if (sp > 0)
                waitpid(sp, NULL, 0);
            free(P);
            return rc;
        }
    }
    for (int k = 0; k < ntargets && !rc; k++) {
        int sv[2];
        if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, sv) != 0) {
            rc = -errno;
            break;
        }
        pid_t pid = fork();
        if (pid == 0) {
            close(sv[0]);
            close(res[0]);
            for (int j = 0; j < k; j++)
                close(P->cmd_fd[j]); /* the other ranks' command channels */
            for (int i = 0; i < ntargets * nconn; i++)
                if (i / nconn != k)
                    close(rfd[i]); /* the other ranks' fold-server connections */
            rank_main(w, k, sv[1], res[1], log, nconn, nconn ? rfd + k * nconn : NULL);
        }
        close(sv[1]);
        if (pid < 0) {
            rc = -errno;
            close(sv[0]);
            break;
        }
        P->pids[k] = pid;
        P->cmd_fd[k] = sv[0];
    }
    close(res[1]);
    P->res_fd = res[0];
    for (int i = 0; i < ntargets * nconn; i++)
        close(rfd[i]);
    free(sfd);
    free(rfd);
    bcp_sock_world_destroy(w); /* the ranks hold their own ends now */
    if (rc) {
        bcp_rank_pool_destroy(P);
        return rc;
    }
    *out = P;
    return 0;
}

static int pool_run(bcp_rank_pool *P, int op, const char *root, const bcp_work_item *items, size_t nitems,
                    int nlanes, const int *lanes, int rebuild_target, const char *corrupt, bcp_run_stats *stats)
{
    if (P->broken)
        return -EPIPE;
    pool_cmd c;
    memset(&c, 0, sizeof(c));
    c.magic = POOL_MAGIC;
    c.op = (uint32_t)op;
    c.nlanes = nlanes;
    c.rebuild_target = rebuild_target;
    c.has_lanes = lanes != NULL;
    bcpi_settings_get(&c.settings);
    c.seq = ++P->seq;
    c.nitems = nitems;
    c.root_len = strlen(root);
    c.corrupt_len = corrupt ? strlen(corrupt) : 0;
    FileInfo *fis = malloc((nitems ? nitems : 1) * sizeof(FileInfo));
    uint32_t *plen = malloc((nitems ? nitems : 1) * sizeof(uint32_t));
    int32_t *ln = lanes ? malloc((nitems ? nitems : 1) * sizeof(int32_t)) : NULL;
    if (!fis || !plen || (lanes && !ln)) {
        free(fis);
        free(plen);
        free(ln);
        return -ENOMEM;
    }
    for (size_t i = 0; i < nitems; i++) {
        fis[i] = items[i].fi;
        plen[i] = (uint32_t)strlen(items[i].path);
        c.paths_len += plen[i];
        if (ln)
            ln[i] = lanes[i];
    }
    double t0 = bcpr_now_s();
    int rc = 0, sent[MAX_STORAGE_TARGETS] = {0};
    for (int k = 0; k < P->ntargets; k++) {
        const int fd = P->cmd_fd[k];
        int e = fd < 0 ? -EPIPE : io_full(fd, &c, sizeof(c), 1);
        if (!e)
            e = io_full(fd, (void *)root, c.root_len, 1);
        if (!e && c.corrupt_len)
            e = io_full(fd, (void *)corrupt, c.corrupt_len, 1);
        if (!e)
            e = io_full(fd, fis, nitems * sizeof(FileInfo), 1);
        if (!e)
            e = io_full(fd, plen, nitems * sizeof(uint32_t), 1);
        for (size_t i = 0; !e && i < nitems; i++)
            e = io_full(fd, (void *)items[i].path, plen[i], 1);
        if (!e && ln)
            e = io_full(fd, ln, nitems * sizeof(int32_t), 1);
        if (e && !rc)
            rc = -ECHILD; /* a rank is gone */
        sent[k] = !e;
    }
    free(fis);
    free(plen);
    free(ln);
    /* one report per rank that got the command, or its death */
    bcp_run_stats st;
    memset(&st, 0, sizeof(st));
    int done[MAX_STORAGE_TARGETS] = {0}, pending = 0;
    for (int k = 0; k < P->ntargets; k++)
        pending += sent[k];
    while (pending > 0) {
        struct pollfd pfd = {P->res_fd, POLLIN, 0};
        int pr = poll(&pfd, 1, 200);
        if (pr > 0) {
            rank_report rep;
            ssize_t r = read(P->res_fd, &rep, sizeof(rep));
            if (r == (ssize_t)sizeof(rep) && rep.seq == c.seq && rep.rank >= 1 && rep.rank <= P->ntargets &&
                sent[rep.rank - 1] && !done[rep.rank - 1]) {
                done[rep.rank - 1] = 1;
                pending--;
                st.tasks += rep.tasks;
                st.bytes_read += rep.bytes_read;
                st.bytes_written += rep.bytes_written;
                st.errors += rep.error != 0;
                if (rep.rc && !rc)
                    rc = rep.rc;
                continue;
            }
            if (r == 0)
                break; /* every rank is gone */
            continue;
        }
        /* no report: has a rank that owes one died?  (its own pids only:
         * the caller's other children are not ours to reap) */
        for (int k = 0; k < P->ntargets; k++) {
            int status;
            if (P->pids[k] <= 0 || waitpid(P->pids[k], &status, WNOHANG) != P->pids[k])
                continue;
            P->pids[k] = -1;
            if (sent[k] && !done[k]) {
                done[k] = 1;
                pending--;
                if (!rc)
                    rc = -ECHILD;
            }
        }
    }
    if (pending > 0 && !rc)
        rc = -ECHILD; /* reports missing: every rank is gone */
    st.seconds = bcpr_now_s() - t0;
    st.refused = bcpr_count_refused(items, nitems, op == POOL_REBUILD ? rebuild_target : -1);
    if (stats)
        *stats = st;
    if (rc)
        P->broken = 1;
    return rc;
}

int bcp_rank_pool_gen(bcp_rank_pool *P, const char *store_root, const bcp_work_item *items, size_t nitems,
                      int nlanes, const int *lanes_in, bcp_run_stats *stats)
{
    if (!P || !store_root || !*store_root || nlanes < 1 || nlanes > 64 || (nitems && !items))
        return -EINVAL;
    int rc = bcpr_check_items(P->ntargets, items, nitems);
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
    rc = pool_run(P, POOL_GEN, store_root, items, nitems, nlanes, lanes_in ? lanes_in : lanes, -1, NULL, stats);
    free(lanes);
    return rc;
}

int bcp_rank_pool_rebuild(bcp_rank_pool *P, const char *store_root, int rebuild_target, const bcp_work_item *items,
                          size_t nitems, const char *corrupt_list_path, bcp_run_stats *stats)
{
    if (!P || !store_root || !*store_root || P->ntargets < 2 || rebuild_target < 0 ||
        rebuild_target >= P->ntargets || (nitems && !items))
        return -EINVAL;
    int rc = bcpr_check_items(P->ntargets, items, nitems);
    if (rc)
        return rc;
    if (corrupt_list_path) { /* truncated once here; the ranks append */
        int fd = open(corrupt_list_path, O_WRONLY | O_CREAT | O_TRUNC, S_IRUSR | S_IWUSR);
        if (fd < 0)
            return -errno;
        close(fd);
    }
    return pool_run(P, POOL_REBUILD, store_root, items, nitems, bcpr_rebuild_lanes(), NULL, rebuild_target,
                    corrupt_list_path, stats);
}

int bcp_rank_pool_destroy(bcp_rank_pool *P)
{
    if (!P)
        return 0;
    pool_cmd q;
    memset(&q, 0, sizeof(q));
    q.magic = POOL_MAGIC;
    q.op = POOL_QUIT;
    for (int k = 0; k < P->ntargets; k++)
        if (P->cmd_fd[k] >= 0) {
            (void)io_full(P->cmd_fd[k], &q, sizeof(q), 1);
            close(P->cmd_fd[k]); /* EOF: a rank that missed QUIT leaves too */
            P->cmd_fd[k] = -1;
        }
    int rc = 0;
    for (int k = 0; k < P->ntargets; k++)
        if (P->pids[k] > 0) {
            int status = 0;
            while (waitpid(P->pids[k], &status, 0) < 0 && errno == EINTR)
                ;
            if (!WIFEXITED(status) || WEXITSTATUS(status) != 0)
                rc = -ECHILD;
            P->pids[k] = -1;
        }
    if (P->srv_pid > 0) { /* leaves once every rank closed its connections */
        int status = 0;
        while (waitpid(P->srv_pid, &status, 0) < 0 && errno == EINTR)
            ;
        if (!WIFEXITED(status) || WEXITSTATUS(status) != 0)
            rc = -ECHILD;
        P->srv_pid = -1;
    }
    if (P->res_fd >= 0)
        close(P->res_fd);
    free(P);
    return rc;
}

int bcp_gen_run_procs(const char *store_root, int ntargets, const bcp_work_item *items, size_t nitems, int nlanes,
                      const int *lanes, FILE *log, bcp_run_stats *stats)
{
    if (!store_root || ntargets < 1 || ntargets > MAX_STORAGE_TARGETS || nlanes < 1 || nlanes > 64 ||
        (nitems && !items))
        return -EINVAL;
    int rc = bcpr_check_items(ntargets, items, nitems);
    if (rc)
        return rc;
    bcp_rank_pool *P = NULL;
    if ((rc = bcp_rank_pool_create(ntargets, log, &P)))
        return rc;
    rc = bcp_rank_pool_gen(P, store_root, items, nitems, nlanes, lanes, stats);
    int drc = bcp_rank_pool_destroy(P);
    return rc ? rc : drc;
}

int bcp_rebuild_run_procs(const char *store_root, int ntargets, int rebuild_target, const bcp_work_item *items,
                          size_t nitems, const char *corrupt_list_path, FILE *log, bcp_run_stats *stats)
{
    if (!store_root || ntargets < 2 || ntargets > MAX_STORAGE_TARGETS || rebuild_target < 0 ||
        rebuild_target >= ntargets || (nitems && !items))
        return -EINVAL;
    int rc = bcpr_check_items(ntargets, items, nitems);
    if (rc)
        return rc;
    bcp_rank_pool *P = NULL;
    if ((rc = bcp_rank_pool_create(ntargets, log, &P)))
        return rc;
    rc = bcp_rank_pool_rebuild(P, store_root, rebuild_target, items, nitems, corrupt_list_path, stats);
    int drc = bcp_rank_pool_destroy(P);
    return rc ? rc : drc;
}
