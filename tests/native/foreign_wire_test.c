/* TEST: libbcp's source role (process_task -> chunk_sender) sending to a P
 * role shaped like the REFERENCE's parity_generator through a transport
 * table the caller installs (a stand-in for an MPI binding: bcp_lb_* behind
 * wrapper functions, no send_fill, so libbcp cannot tell it from MPI).
 *
 * The reference's P role receives every window into buffer_size rows it
 * malloc'd and never cleared (task_processing.c:176-178, 203-209) and folds
 * WHOLE rows (xor_parity over buffer_size bytes, :206-211); it relies on its
 * senders zero-padding each window (:302-303).  Here its rows are pre-filled
 * with garbage (0xA5) before every receive.
 *
 *   foreign_wire_test <scratch dir> <pad>
 *     pad "auto": bcp_task_set_explicit_padding(BCP_PAD_AUTO) (the default):
 *                 through a caller's table the senders must use the
 *                 reference's wire -> every parity equals the zero-padded
 *                 XOR; prints "foreign_wire ok"
 *     pad "implicit": forced implicit padding (0): short windows, the
 *                 garbage past each chunk is folded -> prints
 *                 "foreign_wire mismatch" (the hazard the default avoids)
 * The reference's parity_generator itself needs <mpi.h> (absent; stand-in
 * headers are not allowed), so its receive-and-fold loop is restated here. */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "bcp_task.h"

int st2rank[MAX_STORAGE_TARGETS];

#define NSRC 3
#define P_ST NSRC /* the P role's storage target */
#define NFILES 4

#define CHECK(c)                                                                       \
    do {                                                                               \
        if (!(c)) {                                                                    \
            fprintf(stderr, "foreign_wire_test: %s:%d: %s\n", __FILE__, __LINE__, #c); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

/* chunk lengths per file (one 10 MiB window each: max_cs <= 10 MiB) */
static const size_t LENS[NFILES][NSRC] = {
    {1000, 70000, 3}, {5, 200000, 131072}, {524288, 524288, 524288}, {0, 17, 4096}};

static uint8_t byte_of(int file, int st, size_t j) { return (uint8_t)((j * 2654435761u + file * 97u + st * 13u) >> 7); }

/* ---- the caller's transport: the loopback ranks behind other functions --- */
static int f_send(void *c, const void *b, size_t n, int d, int t) { (void)c; return bcp_lb_send(b, n, d, t); }
static int f_recv(void *c, void *b, size_t n, int s, int t) { (void)c; return bcp_lb_recv(b, n, s, t, NULL); }
static int f_isend(void *c, const void *b, size_t n, int d, int t, void **r)
{
    (void)c;
    return bcp_lb_isend(b, n, d, t, (bcp_lb_req **)r);
}
static int f_irecv(void *c, void *b, size_t n, int s, int t, void **r)
{
    (void)c;
    return bcp_lb_irecv(b, n, s, t, (bcp_lb_req **)r);
}
static int f_wait(void *c, void *r) { (void)c; return bcp_lb_wait(r, NULL); }
static int f_waitall(void *c, int n, void **r) { (void)c; return bcp_lb_waitall(n, (bcp_lb_req **)r); }

static const char *g_root;

static void *source_main(void *arg)
{
    const int st = (int)(intptr_t)arg;
    bcp_lb_set_rank(st2rank[st]);
    char d[4096];
    HostState hs;
    memset(&hs, 0, sizeof(hs));
    hs.storage_target = st;
    hs.log = stderr;
    hs.fd_null = open("/dev/null", O_WRONLY);
    hs.fd_zero = open("/dev/zero", O_RDONLY);
    hs.corrupt_files_fd = -1;
    snprintf(d, sizeof(d), "%s/st%d/chunks", g_root, st);
    hs.read_chunk_dir = open(d, O_DIRECTORY | O_RDONLY);
    hs.write_dir = -1;
    hs.read_parity_dir = -1;
    CHECK(hs.read_chunk_dir > 0);
    const uint64_t loc = WITH_P((UINT64_C(1) << NSRC) - 1, (uint64_t)P_ST);
    for (int i = 0; i < NFILES; i++) {
        char path[32];
        snprintf(path, sizeof(path), "f%d", i);
        FileInfo fi = {0, loc};
        TaskInfo ti = {hs.read_chunk_dir, 0, -1, 0, NULL};
        process_task(&hs, path, &fi, ti);
    }
    CHECK(hs.error == 0);
    bcp_task_thread_release();
    return NULL;
}

/* parity_generator (task_processing.c:117-245), gen, one window per source,
 * restated: sizes in, max_cs out, windows of buffer_size into stale rows,
 * whole-row fold.  Returns 1 if every parity equals the zero-padded XOR. */
static int reference_p_role(void)
{
    bcp_lb_set_rank(st2rank[P_ST]);
    int ok = 1;
    for (int i = 0; i < NFILES; i++) {
        uint64_t sizes[NSRC], max_cs = 0;
        for (int k = 0; k < NSRC; k++)
            CHECK(bcp_lb_recv(&sizes[k], sizeof(uint64_t), st2rank[k], 0, NULL) == 0);
        for (int k = 0; k < NSRC; k++)
            max_cs = sizes[k] > max_cs ? sizes[k] : max_cs;
        for (int k = 0; k < NSRC; k++)
            CHECK(bcp_lb_send(&max_cs, sizeof(max_cs), st2rank[k], 0) == 0);
        const size_t buffer_size = max_cs;
        uint8_t *data = malloc(NSRC * buffer_size + 1);
        memset(data, 0xA5, NSRC * buffer_size + 1); /* what a reused malloc row holds */
        for (int k = 0; k < NSRC; k++)
            CHECK(bcp_lb_recv(data + k * buffer_size, buffer_size, st2rank[k], 0, NULL) == 0);
        uint8_t *par = calloc(1, buffer_size + 1);
        for (int k = 0; k < NSRC; k++) /* xor_parity over whole rows */
            for (size_t j = 0; j < buffer_size; j++)
                par[j] ^= data[k * buffer_size + j];
        for (size_t j = 0; j < buffer_size && ok; j++) {
            uint8_t want = 0;
            for (int k = 0; k < NSRC; k++)
                want ^= j < LENS[i][k] ? byte_of(i, k, j) : 0;
            ok = par[j] == want;
        }
        free(data);
        free(par);
    }
    return ok;
}

int main(int argc, char **argv)
{
    CHECK(argc == 3);
    g_root = argv[1];
    const int pad = !strcmp(argv[2], "auto") ? BCP_PAD_AUTO : 0;
    char d[4096];
    mkdir(g_root, 0700);
    for (int st = 0; st < NSRC; st++) {
        snprintf(d, sizeof(d), "%s/st%d", g_root, st);
        mkdir(d, 0700);
        snprintf(d, sizeof(d), "%s/st%d/chunks", g_root, st);
        mkdir(d, 0700);
        for (int i = 0; i < NFILES; i++) {
            snprintf(d, sizeof(d), "%s/st%d/chunks/f%d", g_root, st, i);
            FILE *f = fopen(d, "wb");
            CHECK(f);
            for (size_t j = 0; j < LENS[i][st]; j++)
                fputc(byte_of(i, st, j), f);
            fclose(f);
        }
    }
    for (int k = 0; k < MAX_STORAGE_TARGETS; k++)
        st2rank[k] = k <= P_ST ? k + 1 : -1;
    CHECK(bcp_lb_init(P_ST + 2) == 0);
    const bcp_transport_ops ops = {NULL, f_send, f_recv, f_isend, f_irecv, f_wait, f_waitall, NULL};
    CHECK(bcp_task_set_transport(&ops) == 0);
    CHECK(bcp_task_set_explicit_padding(pad) >= BCP_PAD_AUTO);
    pthread_t th[NSRC];
    for (int st = 0; st < NSRC; st++)
        CHECK(pthread_create(&th[st], NULL, source_main, (void *)(intptr_t)st) == 0);
    const int ok = reference_p_role();
    for (int st = 0; st < NSRC; st++)
        pthread_join(th[st], NULL);
    bcp_task_set_transport(NULL);
    bcp_lb_finalize();
    puts(ok ? "foreign_wire ok" : "foreign_wire mismatch");
    return 0;
}
