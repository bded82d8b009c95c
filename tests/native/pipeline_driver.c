/* Host-code sanitizer driver on a GPU box (tools/tsan_pipeline.sh): a
 * loopback store of mixed chunk sizes.
 *  1. The batched pipeline: parity gen through bcp_pipeline_run with both
 *     read paths (COPY, DIRECT) and two device lanes wrapping onto the
 *     visible GPUs (small slabs, few io threads, so batches, slot reuse and
 *     the io pool's two job kinds all interleave); then one target lost and
 *     rebuilt by bcp_pipeline_rebuild.
 *  2. The per-task protocol over loopback ranks (bcp_gen_run, 3 lanes per
 *     rank; bcp_rebuild_run), once through the resident fold ring with lane
 *     deferral (the default; the loopback transport polling 20 us before it
 *     sleeps) and once through the lane queues: ring submission and waits
 *     from every P lane at once, deferred completions on the completion
 *     threads, relaunches after the ring idles out between runs.
 * Every parity file is checked against a CPU XOR written here and every
 * rebuilt chunk against the lost one.  The C host layer and the engine's
 * host code are built with -fsanitize=thread (clang); device code is not. */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "bcp_task.h"

#define NT 9
#define NFILES 90
#define VICTIM 4

static void mkdirs(const char *p)
{
    char tmp[512];
    snprintf(tmp, sizeof tmp, "%s", p);
    for (char *s = tmp + 1; *s; s++)
        if (*s == '/') {
            *s = 0;
            mkdir(tmp, 0755);
            *s = '/';
        }
    mkdir(tmp, 0755);
}

static void write_file(const char *path, const uint8_t *d, size_t n)
{
    char dir[512];
    snprintf(dir, sizeof dir, "%s", path);
    *strrchr(dir, '/') = 0;
    mkdirs(dir);
    int fd = open(path, O_CREAT | O_WRONLY | O_TRUNC, 0644);
    if (fd < 0 || (n && write(fd, d, n) != (ssize_t)n)) {
        perror(path);
        exit(2);
    }
    close(fd);
}

static uint8_t *read_file(const char *path, size_t *n)
{
    int fd = open(path, O_RDONLY);
    if (fd < 0)
        return NULL;
    struct stat sb;
    fstat(fd, &sb);
    uint8_t *b = malloc((size_t)sb.st_size + 1);
    ssize_t r = read(fd, b, (size_t)sb.st_size);
    close(fd);
    *n = r > 0 ? (size_t)r : 0;
    return b;
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void)
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

static const char *root;
static bcp_work_item *items;
static char (*names)[64];
static uint8_t *chunk[NFILES][NT];
static size_t len[NFILES][NT];

/* every parity file = u64 sizes (ascending holders) + zero-padded XOR */
static int check_parity(const char *what)
{
    char path[512];
    int bad = 0;
    for (int i = 0; i < NFILES; i++) {
        const uint64_t loc = items[i].fi.locations;
        const int p = (int)(loc >> 56);
        size_t maxn = 0;
        int n = 0;
        for (int t = 0; t < NT; t++)
            if (loc >> t & 1) {
                n++;
                maxn = len[i][t] > maxn ? len[i][t] : maxn;
            }
        uint8_t *want = calloc(8 * (size_t)n + maxn + 1, 1);
        int k = 0;
        for (int t = 0; t < NT; t++)
            if (loc >> t & 1) {
                memcpy(want + 8 * k++, &len[i][t], 8);
                for (size_t j = 0; j < len[i][t]; j++)
                    want[8 * (size_t)n + j] ^= chunk[i][t][j];
            }
        snprintf(path, sizeof path, "%s/st%d/parity/%s", root, p, names[i]);
        size_t got_n = 0;
        uint8_t *got = read_file(path, &got_n);
        if (!got || got_n != 8 * (size_t)n + maxn || memcmp(got, want, got_n)) {
            fprintf(stderr, "parity mismatch: %s file %s\n", what, names[i]);
            bad++;
        }
        free(got);
        free(want);
    }
    return bad;
}

static void remove_parity(void)
{
    char path[512];
    for (int i = 0; i < NFILES; i++) {
        snprintf(path, sizeof path, "%s/st%d/parity/%s", root, (int)(items[i].fi.locations >> 56), names[i]);
        unlink(path);
    }
}

static void lose_victim(void)
{
    char path[512];
    for (int i = 0; i < NFILES; i++)
        if (items[i].fi.locations >> VICTIM & 1) {
            snprintf(path, sizeof path, "%s/st%d/chunks/%s", root, VICTIM, names[i]);
            unlink(path);
        }
}

static int check_victim(const char *what)
{
    char path[512];
    int bad = 0;
    for (int i = 0; i < NFILES; i++)
        if (items[i].fi.locations >> VICTIM & 1) {
            snprintf(path, sizeof path, "%s/st%d/chunks/%s", root, VICTIM, names[i]);
            size_t got_n = 0;
            uint8_t *got = read_file(path, &got_n);
            if (!got || got_n != len[i][VICTIM] || memcmp(got, chunk[i][VICTIM], got_n)) {
                fprintf(stderr, "rebuilt chunk mismatch: %s file %s\n", what, names[i]);
                bad++;
            }
            free(got);
        }
    return bad;
}

int main(int argc, char **argv)
{
    root = argc > 1 ? argv[1] : "/tmp/bcp_tsan_pipeline";
    char path[512];
    items = calloc(NFILES, sizeof *items);
    names = calloc(NFILES, 64);
    for (int i = 0; i < NFILES; i++) {
        const int p = i % NT;
        uint64_t loc = 0;
        snprintf(names[i], 64, "m%d/chunk%d", i % 5, i);
        for (int t = 0; t < NT; t++) {
            if (t == p || rnd() % 3 == 0)
                continue;
            loc |= 1ull << t;
            /* mostly up to 3 MiB, some empty, some of a few bytes, not multiples of 16 */
            const uint64_t r = rnd() % 16;
            size_t n = r == 0 ? 0 : r == 1 ? (size_t)(rnd() % 40) : (size_t)(rnd() % (3u << 20));
            uint8_t *d = malloc(n + 1);
            for (size_t j = 0; j < n; j++)
                d[j] = (uint8_t)rnd();
            snprintf(path, sizeof path, "%s/st%d/chunks/%s", root, t, names[i]);
            write_file(path, d, n);
            chunk[i][t] = d;
            len[i][t] = n;
        }
        if (!loc) { /* at least one holder */
            const int t = (p + 1) % NT;
            loc = 1ull << t;
            chunk[i][t] = malloc(1);
            snprintf(path, sizeof path, "%s/st%d/chunks/%s", root, t, names[i]);
            write_file(path, chunk[i][t], 0);
        }
        items[i].path = names[i];
        items[i].fi.timestamp = 1LL << 40;
        items[i].fi.locations = loc | ((uint64_t)p << 56);
    }
    for (int t = 0; t < NT; t++) {
        snprintf(path, sizeof path, "%s/st%d/parity", root, t);
        mkdirs(path);
    }
    int bad = 0;
    const int modes[2] = {BCP_READ_COPY, BCP_READ_DIRECT};
    for (int m = 0; m < 2; m++) {
        bcp_pipeline_opts o = {0, (size_t)8 << 20, 2, 3, 2, modes[m]};
        bcp_pipeline *pl = NULL;
        int rc = bcp_pipeline_create(&o, &pl);
        if (rc) {
            fprintf(stderr, "pipeline_create: %d\n", rc);
            return 1;
        }
        bcp_run_stats st;
        for (int rep = 0; rep < 2 && !rc; rep++)
            rc = bcp_pipeline_run(pl, root, NT, items, NFILES, NULL, &st);
        if (rc || st.errors) {
            fprintf(stderr, "pipeline_run mode %d: rc=%d errors=%d\n", modes[m], rc, st.errors);
            return 1;
        }
        char what[32];
        snprintf(what, sizeof what, "pipeline mode %d", modes[m]);
        bad += check_parity(what);
        /* lose VICTIM, rebuild it (DB key order does not matter for the bytes) */
        lose_victim();
        rc = bcp_pipeline_rebuild(pl, root, NT, VICTIM, items, NFILES, NULL, NULL, &st);
        if (rc || st.errors) {
            fprintf(stderr, "pipeline_rebuild mode %d: rc=%d errors=%d\n", modes[m], rc, st.errors);
            return 1;
        }
        bad += check_victim(what);
        bcp_pipeline_destroy(pl);
    }
    for (int ring = 1; ring >= 0; ring--) {
        const char *what = ring ? "protocol, fold ring" : "protocol, lane queues";
        bcp_task_set_fold_ring(ring);
        /* the ring pass with the transport's spin-before-sleep waits */
        bcp_task_set_fold_tuning("lb_spin_us", ring ? 20 : 0);
        remove_parity();
        bcp_run_stats st;
        int rc = bcp_gen_run(root, NT, items, NFILES, 3, NULL, NULL, &st);
        if (rc || st.errors) {
            fprintf(stderr, "gen_run %s: rc=%d errors=%d\n", what, rc, st.errors);
            return 1;
        }
        bad += check_parity(what);
        lose_victim();
        rc = bcp_rebuild_run(root, NT, VICTIM, items, NFILES, NULL, NULL, &st);
        if (rc || st.errors) {
            fprintf(stderr, "rebuild_run %s: rc=%d errors=%d\n", what, rc, st.errors);
            return 1;
        }
        bad += check_victim(what);
    }
    bcp_task_shutdown();
    printf("%s: %d problems\n", bad ? "FAILED" : "OK", bad);
    return bad ? 1 : 0;
}
