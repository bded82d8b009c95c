/*
 * tmpfs_io_probe.c -- what the host itself allows the pipeline's io threads
 * (tools only): T threads writing / reading 1 GiB of 2 MiB files in a tmpfs
 * directory, and copying memory, for T = 1, 2, 4, 8, 16.  Writes three ways:
 * into fresh files (unlinked first), O_TRUNC over the previous files (the
 * pipeline's writers), and over them in place (no truncation).  One JSON line
 * per measurement, GB/s.
 *
 *   gcc -O2 -pthread tools/exp/tmpfs_io_probe.c -o tools/exp/tmpfs_io_probe
 *   tools/exp/tmpfs_io_probe /dev/shm/bcp_io_probe
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#define FILE_BYTES ((size_t)2 << 20)
#define NFILES 512 /* 1 GiB */

static const char *g_dir;
static int g_op, g_threads;
static uint8_t *g_src;
static uint8_t **g_dst;

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + (double)t.tv_nsec * 1e-9;
}

enum { W_FRESH, W_TRUNC, W_INPLACE, READ, COPY };
static const char *NAMES[] = {"write_fresh", "write_trunc", "write_inplace", "read", "memcpy"};

static void *worker(void *p)
{
    const int id = (int)(intptr_t)p;
    char fn[4096];
    for (int f = id; f < NFILES; f += g_threads) {
        snprintf(fn, sizeof(fn), "%s/f%04d", g_dir, f);
        if (g_op == COPY) {
            memcpy(g_dst[id], g_src + (size_t)(f % 8) * FILE_BYTES, FILE_BYTES);
            continue;
        }
        if (g_op == W_FRESH)
            unlink(fn);
        int flags = g_op == READ ? O_RDONLY : O_WRONLY | O_CREAT | (g_op == W_INPLACE ? 0 : O_TRUNC);
        int fd = open(fn, flags, 0600);
        if (fd < 0) {
            perror(fn);
            exit(1);
        }
        size_t done = 0;
        while (done < FILE_BYTES) {
            ssize_t r = g_op == READ ? pread(fd, g_dst[id] + done, FILE_BYTES - done, (off_t)done)
                                     : pwrite(fd, g_src + (size_t)(f % 8) * FILE_BYTES + done, FILE_BYTES - done,
                                              (off_t)done);
            if (r <= 0) {
                perror("io");
                exit(1);
            }
            done += (size_t)r;
        }
        close(fd);
    }
    return NULL;
}

static double run(int op, int threads)
{
    g_op = op;
    g_threads = threads;
    pthread_t th[64];
    const double t0 = now_s();
    for (int i = 0; i < threads; i++)
        pthread_create(&th[i], NULL, worker, (void *)(intptr_t)i);
    for (int i = 0; i < threads; i++)
        pthread_join(th[i], NULL);
    return now_s() - t0;
}

int main(int argc, char **argv)
{
    if (argc != 2) {
        fprintf(stderr, "usage: %s <dir on tmpfs>\n", argv[0]);
        return 2;
    }
    g_dir = argv[1];
    mkdir(g_dir, 0700);
    g_src = malloc(8 * FILE_BYTES);
    g_dst = calloc(64, sizeof(uint8_t *));
    for (size_t i = 0; i < 8 * FILE_BYTES; i++)
        g_src[i] = (uint8_t)(i * 2654435761u >> 13);
    for (int i = 0; i < 64; i++) {
        g_dst[i] = malloc(FILE_BYTES);
        memset(g_dst[i], 1, FILE_BYTES);
    }
    run(W_FRESH, 8); /* the files exist from here on */
    const int ts[] = {1, 2, 4, 8, 16};
    for (int rep = 0; rep < 3; rep++)
        for (size_t k = 0; k < sizeof(ts) / sizeof(ts[0]); k++)
            for (int op = W_FRESH; op <= COPY; op++) {
                const double s = run(op, ts[k]);
                printf("{\"rep\": %d, \"op\": \"%s\", \"threads\": %d, \"GBps\": %.2f}\n", rep, NAMES[op], ts[k],
                       (double)NFILES * FILE_BYTES / s / 1e9);
                fflush(stdout);
            }
    for (int f = 0; f < NFILES; f++) {
        char fn[4096];
        snprintf(fn, sizeof(fn), "%s/f%04d", g_dir, f);
        unlink(fn);
    }
    rmdir(g_dir);
    return 0;
}
