/* TEST: a caller shaped like the reference's bp-parity-gen (gen/main.c):
 * it defines its own `int st2rank[MAX_STORAGE_TARGETS]` and HostState per
 * rank (gen/main.c:48,723-743), runs one PROCESS per storage target (as
 * mpirun does) and calls process_task from lane threads with tag = lane
 * (process_list, gen/main.c:116-164) -- linked against libbcp.so with the
 * socketpair transport in place of MPI.  Checks:
 *   - the boundary types have the reference's layout on x86-64 (sizeof /
 *     offsetof of FileInfo, TaskInfo, HostState, ProgressSample);
 *   - the caller's st2rank is the one libbcp uses (interposition: the
 *     library's is weak) -- ranks are numbered 10 + st here, not k + 1;
 *   - every parity chunk equals the zero-padded XOR of its chunks, header
 *     first.
 * The P role's fold is a CPU test double (no GPU in this test).
 *   usage: caller_test <scratch dir>            prints "caller_test ok" */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include "bcp_task.h"

int st2rank[MAX_STORAGE_TARGETS]; /* the caller's own, as gen/main.c:48 */

#define NT 5      /* storage targets */
#define NRANKS 16 /* world: ranks 10..14 are the targets, the rest idle */
#define MAX_LANES 12
static int NLANES = 3; /* lanes per rank; BCP_CALLER_LANES=1..12 (tools/tsan_host.sh runs 3 and 12) */
#define NFILES 24

#define CHECK(c)                                                           \
    do {                                                                   \
        if (!(c)) {                                                        \
            fprintf(stderr, "caller_test: %s:%d: %s\n", __FILE__, __LINE__, #c); \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

static int cpu_fold(uint8_t *dst, size_t nbytes, const uint8_t *data, size_t pitch, int nsrc, void *ctx)
{
    (void)ctx;
    memcpy(dst, data, nbytes);
    for (int k = 1; k < nsrc; k++)
        for (size_t i = 0; i < nbytes; i++)
            dst[i] ^= data[(size_t)k * pitch + i];
    return 0;
}

static uint8_t byte_of(int file, int st, size_t j) { return (uint8_t)((j * 131u + (unsigned)file * 7u + (unsigned)st * 31u) >> 3); }

static size_t len_of(int file, int st) { return (size_t)((file * 7919 + st * 104729) % 300000); }

typedef struct {
    FileInfo fi[NFILES];
    char path[NFILES][64];
    int lane[NFILES];
} worklist;

typedef struct {
    HostState *hs;
    const worklist *wl;
    int lane;
    ProgressSample sample;
} lane_params;

/* process_list (gen/main.c:116-164), without the DB */
static void *process_list(void *p)
{
    lane_params *lp = p;
    TaskInfo ti = {lp->hs->read_chunk_dir, 0, -1, lp->lane, &lp->sample};
    for (int i = 0; i < NFILES; i++) {
        if (lp->wl->lane[i] != lp->lane || (uint64_t)GET_P(lp->wl->fi[i].locations) == NO_P)
            continue;
        process_task(lp->hs, lp->wl->path[i], &lp->wl->fi[i], ti);
    }
    return NULL;
}

static void rank_main(bcp_sock_world *w, const char *root, int st, const worklist *wl)
{
    bcp_transport_ops ops;
    CHECK(bcp_sock_world_attach(w, st2rank[st], &ops) == 0);
    CHECK(bcp_task_set_transport(&ops) == 0);
    bcp_task_set_xor_hook(cpu_fold, NULL);
    char d[4096];
    HostState hs;
    memset(&hs, 0, sizeof(hs));
    hs.storage_target = st;
    hs.log = stderr;
    hs.fd_null = open("/dev/null", O_WRONLY);
    hs.fd_zero = open("/dev/zero", O_RDONLY);
    hs.corrupt_files_fd = -1;
    snprintf(d, sizeof(d), "%s/st%d/chunks", root, st);
    hs.read_chunk_dir = open(d, O_DIRECTORY | O_RDONLY);
    snprintf(d, sizeof(d), "%s/st%d/parity", root, st);
    hs.write_dir = open(d, O_DIRECTORY | O_RDONLY);
    hs.read_parity_dir = -1;
    CHECK(hs.read_chunk_dir > 0 && hs.write_dir > 0);
    pthread_t th[MAX_LANES];
    lane_params lp[MAX_LANES];
    for (int l = 0; l < NLANES; l++) {
        lp[l] = (lane_params){&hs, wl, l, PROGRESS_SAMPLE_INIT};
        CHECK(pthread_create(&th[l], NULL, process_list, &lp[l]) == 0);
    }
    for (int l = 0; l < NLANES; l++)
        pthread_join(th[l], NULL);
    bcp_task_shutdown();
    _exit(hs.error ? 3 : 0);
}

int main(int argc, char **argv)
{
    CHECK(argc == 2);
    /* ---- layout of the boundary types (common.h:15-42, task_processing.h:7-18,
     * progress_reporting.h:10-20) on LP64 */
    CHECK(sizeof(FileInfo) == 16 && offsetof(FileInfo, timestamp) == 0 && offsetof(FileInfo, locations) == 8);
    CHECK(sizeof(ProgressSample) == 64 && offsetof(ProgressSample, bytes_written) == 24 &&
          offsetof(ProgressSample, total_bytes_written) == 56);
    CHECK(sizeof(TaskInfo) == 24 && offsetof(TaskInfo, read_dir) == 0 && offsetof(TaskInfo, is_rebuilding) == 4 &&
          offsetof(TaskInfo, actual_P_st) == 8 && offsetof(TaskInfo, tag) == 12 && offsetof(TaskInfo, sample) == 16);
    CHECK(sizeof(HostState) == 56 && offsetof(HostState, storage_target) == 0 &&
          offsetof(HostState, corrupt_files_fd) == 4 && offsetof(HostState, error) == 8 &&
          offsetof(HostState, error_path) == 16 && offsetof(HostState, fd_null) == 24 &&
          offsetof(HostState, fd_zero) == 28 && offsetof(HostState, write_dir) == 32 &&
          offsetof(HostState, read_chunk_dir) == 36 && offsetof(HostState, read_parity_dir) == 40 &&
          offsetof(HostState, log) == 48);

    const char *root = argv[1];
    if (getenv("BCP_CALLER_LANES"))
        NLANES = atoi(getenv("BCP_CALLER_LANES"));
    CHECK(NLANES >= 1 && NLANES <= MAX_LANES);
    char d[4096];
    mkdir(root, 0700);
    for (int st = 0; st < NT; st++) {
        snprintf(d, sizeof(d), "%s/st%d", root, st);
        mkdir(d, 0700);
        snprintf(d, sizeof(d), "%s/st%d/chunks", root, st);
        mkdir(d, 0700);
        snprintf(d, sizeof(d), "%s/st%d/parity", root, st);
        mkdir(d, 0700);
    }
    /* the worklist: file i on 1..4 targets, P = a target outside them */
    static worklist wl;
    FileInfo fis[NFILES];
    for (int i = 0; i < NFILES; i++) {
        const int P = i % NT;
        const int width = 1 + i % (NT - 1);
        uint64_t loc = 0;
        for (int k = 1; k <= width; k++) {
            const int st = (P + k) % NT;
            loc |= UINT64_C(1) << st;
            snprintf(wl.path[i], sizeof(wl.path[i]), "d%d/f%d", i % 3, i);
            snprintf(d, sizeof(d), "%s/st%d/chunks/d%d", root, st, i % 3);
            mkdir(d, 0700);
            snprintf(d, sizeof(d), "%s/st%d/chunks/%s", root, st, wl.path[i]);
            FILE *f = fopen(d, "wb");
            CHECK(f);
            for (size_t j = 0; j < len_of(i, st); j++)
                fputc(byte_of(i, st, j), f);
            fclose(f);
        }
        wl.fi[i].timestamp = 0;
        wl.fi[i].locations = WITH_P(loc, (uint64_t)P);
        fis[i] = wl.fi[i];
    }
    bcp_assign_lanes(NLANES, NFILES, fis, wl.lane);
    for (int k = 0; k < MAX_STORAGE_TARGETS; k++)
        st2rank[k] = k < NT ? 10 + k : -1;

    bcp_sock_world *w = NULL;
    CHECK(bcp_sock_world_create(NRANKS, &w) == 0);
    pid_t pids[NT];
    for (int st = 0; st < NT; st++) {
        pids[st] = fork();
        CHECK(pids[st] >= 0);
        if (pids[st] == 0)
            rank_main(w, root, st, &wl);
    }
    bcp_sock_world_destroy(w);
    for (int st = 0; st < NT; st++) {
        int status = 0;
        CHECK(waitpid(pids[st], &status, 0) == pids[st]);
        CHECK(WIFEXITED(status) && WEXITSTATUS(status) == 0);
    }
    /* ---- every parity chunk: header u64 sizes (ascending target) + XOR */
    for (int i = 0; i < NFILES; i++) {
        const int P = GET_P(wl.fi[i].locations);
        size_t max_cs = 0, n = 0;
        uint64_t hdr[NT];
        for (int st = 0; st < NT; st++)
            if (TEST_BIT(wl.fi[i].locations, st)) {
                hdr[n++] = len_of(i, st);
                if (len_of(i, st) > max_cs)
                    max_cs = len_of(i, st);
            }
        snprintf(d, sizeof(d), "%s/st%d/parity/%s", root, P, wl.path[i]);
        FILE *f = fopen(d, "rb");
        CHECK(f);
        uint64_t got[NT];
        CHECK(fread(got, 8, n, f) == n && memcmp(got, hdr, 8 * n) == 0);
        for (size_t j = 0; j < max_cs; j++) {
            uint8_t x = 0;
            for (int st = 0; st < NT; st++)
                if (TEST_BIT(wl.fi[i].locations, st) && j < len_of(i, st))
                    x ^= byte_of(i, st, j);
            CHECK(fgetc(f) == x);
        }
        CHECK(fgetc(f) == EOF);
        fclose(f);
    }
    printf("caller_test ok: %d files over %d rank processes, caller-defined st2rank (10 + st)\n", NFILES, NT);
    return 0;
}
