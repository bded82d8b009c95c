/* Protocol driver for host-code sanitizer runs (tools/tsan_host.sh): a small
 * loopback store, parity gen over 12 lanes (P role folded by the CPU test
 * double), then a rebuild of one target, compared with the lost chunks.
 * No GPU call is made. */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "bcp_task.h"

int test_cpu_xor(uint8_t *dst, size_t nbytes, const uint8_t *data, size_t pitch, int nsrc, void *ctx);

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
    if (fd < 0 || write(fd, d, n) != (ssize_t)n) {
        perror(path);
        exit(2);
    }
    close(fd);
}

int main(int argc, char **argv)
{
    const char *root = argc > 1 ? argv[1] : "/tmp/bcp_sanitize_store";
    /* "pipelined": the P roles fold range by range as the sources publish
     * pieces (BCP_FOLD_PIPELINED; sources fill from many lanes at once) */
    const int pipelined = argc > 2 && !strcmp(argv[2], "pipelined");
    const int nt = 6, nfiles = 60, maxlen = pipelined ? 1200000 : 300000;
    char path[512];
    srand(7);
    bcp_work_item *items = calloc(nfiles, sizeof *items);
    char (*names)[64] = calloc(nfiles, 64);
    uint8_t **lost = calloc(nfiles, sizeof *lost);
    size_t *lost_n = calloc(nfiles, sizeof *lost_n);
    for (int i = 0; i < nfiles; i++) {
        const int p = i % nt;
        uint64_t loc = 0;
        snprintf(names[i], 64, "d%02d/chunk%d", i % 7, i);
        for (int t = 0; t < nt; t++) {
            if (t == p || (rand() % 4) == 0)
                continue;
            loc |= 1ull << t;
            size_t n = (size_t)(rand() % maxlen);
            uint8_t *d = malloc(n + 1);
            for (size_t j = 0; j < n; j++)
                d[j] = (uint8_t)rand();
            snprintf(path, sizeof path, "%s/st%d/chunks/%s", root, t, names[i]);
            write_file(path, d, n);
            if (t == 2) {
                lost[i] = d;
                lost_n[i] = n;
            } else {
                free(d);
            }
        }
        items[i].path = names[i];
        items[i].fi.timestamp = 1LL << 40;
        items[i].fi.locations = loc | ((uint64_t)p << 56);
    }
    for (int t = 0; t < nt; t++) {
        snprintf(path, sizeof path, "%s/st%d/parity", root, t);
        mkdirs(path);
    }
    bcp_task_set_xor_hook(test_cpu_xor, NULL);
    if (bcp_task_set_fold_mode(pipelined ? BCP_FOLD_PIPELINED : BCP_FOLD_BATCHED) < 0)
        return 3;
    bcp_run_stats st;
    int rc = bcp_gen_run(root, nt, items, nfiles, 12, NULL, NULL, &st);
    if (rc || st.errors) {
        fprintf(stderr, "gen_run rc=%d errors=%d\n", rc, st.errors);
        return 1;
    }
    for (int i = 0; i < nfiles; i++)
        if (lost[i]) {
            snprintf(path, sizeof path, "%s/st2/chunks/%s", root, names[i]);
            unlink(path);
        }
    rc = bcp_rebuild_run(root, nt, 2, items, nfiles, NULL, NULL, &st);
    if (rc || st.errors) {
        fprintf(stderr, "rebuild_run rc=%d errors=%d\n", rc, st.errors);
        return 1;
    }
    int bad = 0;
    for (int i = 0; i < nfiles; i++) {
        if (!lost[i])
            continue;
        snprintf(path, sizeof path, "%s/st2/chunks/%s", root, names[i]);
        int fd = open(path, O_RDONLY);
        uint8_t *got = malloc(lost_n[i] + 1);
        ssize_t r = fd >= 0 ? read(fd, got, lost_n[i] + 1) : -1;
        if (r != (ssize_t)lost_n[i] || memcmp(got, lost[i], lost_n[i]))
            bad++;
        if (fd >= 0)
            close(fd);
        free(got);
        free(lost[i]);
    }
    /* error path: target 0's parity directories d00..d06 become files, so
     * every parity write on target 0 fails (ENOTDIR) from many lanes at once;
     * the rank's sticky error is raised exactly once */
    for (int d = 0; d < 7; d++) {
        char dir[512];
        snprintf(dir, sizeof dir, "%s/st0/parity/d%02d", root, d);
        char cmd[600];
        snprintf(cmd, sizeof cmd, "rm -rf '%s'", dir);
        if (system(cmd) != 0)
            return 2;
        write_file(dir, (const uint8_t *)"x", 1);
    }
    rc = bcp_gen_run(root, nt, items, nfiles, 12, NULL, NULL, &st);
    if (rc || st.errors != 1) {
        fprintf(stderr, "sabotaged gen_run rc=%d errors=%d (want 1)\n", rc, st.errors);
        bad++;
    }
    bcp_task_shutdown();
    printf("%s: %d problems\n", bad ? "FAILED" : "OK", bad);
    return bad ? 1 : 0;
}
