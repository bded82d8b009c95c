/*
 * bcp_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference chunk-XOR parity path of
 * runefriborg/beegfs-chunk-parity, written from the reference's documented
 * behaviour (not copied).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed
 * CPU baseline.  The product library (beegfs-chunk-parity_amd/lib/libbcp.so)
 * never links or calls it.
 *
 * Parity pinning: the reference's own xor_parity (task_processing.c:96-109,
 * which needs only libc headers) is compiled unchanged into
 * oracle/_ref/libref_xor.so (oracle/Makefile `ref`); its outputs are the 77
 * xor_parity fixtures and the folds of the 4 parity-file fixtures in
 * tests/golden/ref_xor.json, which this restatement must reproduce
 * (tests/test_oracle_ref.py), and where _ref is built it is also compared with
 * the reference function directly on random misaligned shapes.  The MPI roles
 * around the fold (window assembly, padding, replay: task_processing.c:117-322)
 * include <mpi.h>, which is absent (stand-in headers are not allowed), so
 * that assembly is pinned by the survey's known-answer SHA-256 values
 * (tests/test_oracle_kat.py, tests/golden/kats.json).
 *
 * Compiled with the reference's own flags (-std=gnu99 -Os, build.sh:8) so
 * that oracle_xor_parity doubles as the CPU baseline.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

#define ORACLE_WINDOW (10u * 1024u * 1024u) /* task_processing.c:20 */
#define ORACLE_MAX_SOURCES 56               /* common.h:18 */

/*
 * xor_parity -- task_processing.c:96-109.
 * dst = data[0] ^ data[1] ^ ... ^ data[n-1], data laid out [n][nbytes].
 * Same statement order as the reference: copy source 0, then fold each later
 * source with 8-byte words while i + 8 < nbytes, finishing with single bytes.
 */
void oracle_xor_parity(uint8_t *restrict dst, size_t nbytes,
                       const uint8_t *data, int nsources)
{
    memcpy(dst, data, nbytes);
    for (int s = 1; s < nsources; s++) {
        const uint8_t *src = data + (size_t)s * nbytes;
        size_t i = 0;
        for (; i + 8 < nbytes; i += 8) {
            uint64_t a, b;
            memcpy(&a, dst + i, 8);
            memcpy(&b, src + i, 8);
            a ^= b;
            memcpy(dst + i, &a, 8);
        }
        for (; i < nbytes; i++)
            dst[i] ^= src[i];
    }
}

/*
 * xor_parity over rows `pitch` bytes apart, with the signature of libbcp's
 * bcp_xor_hook_fn: lets tools time the protocol with the reference's CPU
 * fold in place of the GPU (the "reference CPU path" of config 1).
 */
int oracle_xor_rows(uint8_t *dst, size_t nbytes, const uint8_t *data, size_t pitch, int nsrc, void *ctx)
{
    (void)ctx;
    memcpy(dst, data, nbytes);
    for (int s = 1; s < nsrc; s++) {
        const uint8_t *src = data + (size_t)s * pitch;
        size_t i = 0;
        for (; i + 8 < nbytes; i += 8) {
            uint64_t a, b;
            memcpy(&a, dst + i, 8);
            memcpy(&b, src + i, 8);
            a ^= b;
            memcpy(dst + i, &a, 8);
        }
        for (; i < nbytes; i++)
            dst[i] ^= src[i];
    }
    return 0;
}

/*
 * One source's sender state: mirrors chunk_sender's loop
 * (task_processing.c:282-308).  `data` persists across windows; a window is
 * refilled only while data_sent < fd_size, so once the file is exhausted the
 * previous window is re-sent unchanged (quirk A3-q1).  A file
 * that never refills its buffer (size 0, or an open error) sends zeros here
 * (the reference sends uninitialised malloc memory for size 0 -- quirk A3-q2,
 * defined as zeros).
 */
typedef struct {
    const uint8_t *file;  /* file contents after any skipped header */
    uint64_t fd_size;     /* bytes available to read */
    uint64_t pos;         /* file offset */
    uint64_t data_sent;
} oracle_sender;

static void sender_next_window(oracle_sender *s, uint8_t *data,
                               size_t buffer_size, uint64_t data_to_send)
{
    uint64_t data_left = data_to_send - s->data_sent;
    if (s->data_sent < s->fd_size) {
        uint64_t want = buffer_size < data_left ? buffer_size : data_left;
        uint64_t avail = s->fd_size - s->pos;
        uint64_t r = want < avail ? want : avail;
        memcpy(data, s->file + s->pos, r);
        s->pos += r;
        if (r < buffer_size)
            memset(data + r, 0, buffer_size - r);
    }
    s->data_sent += buffer_size;
}

/*
 * Runs the P-role window loop of parity_generator (task_processing.c:176-226)
 * over n senders and writes the XORed stream (max_cs bytes, no header) to out.
 */
static int run_windows(uint8_t *out, oracle_sender *snd, int n,
                       uint64_t max_cs, uint64_t window)
{
    size_t buffer_size = max_cs < window ? (size_t)max_cs : (size_t)window;
    uint64_t expected = (max_cs + window - 1) / window;
    if (expected == 0)
        return 0;
    uint8_t *data = calloc((size_t)n, buffer_size ? buffer_size : 1);
    uint8_t *pblk = malloc(buffer_size ? buffer_size : 1);
    if (!data || !pblk) {
        free(data);
        free(pblk);
        return -1;
    }
    uint64_t left = max_cs, off = 0;
    for (uint64_t w = 0; w < expected; w++) {
        for (int k = 0; k < n; k++)
            sender_next_window(&snd[k], data + (size_t)k * buffer_size,
                               buffer_size, max_cs);
        oracle_xor_parity(pblk, buffer_size, data, n);
        uint64_t wsize = buffer_size < left ? buffer_size : left;
        memcpy(out + off, pblk, wsize);
        off += wsize;
        left -= wsize;
    }
    free(data);
    free(pblk);
    return 0;
}

/*
 * Gen-mode parity chunk file (task_processing.c:146-226 with the senders of
 * :247-322): header u64 chunk_size[n] in ascending storage-target order
 * (:199-201), then max_cs bytes of windowed XOR (:203-226).
 * chunks[k] may be NULL (open error -> zero data, size 0).
 * Returns the file length (8n + max_cs) or -1 if out_cap is too small.
 */
int64_t oracle_gen_parity_file(uint8_t *out, uint64_t out_cap,
                               const uint8_t *const *chunks,
                               const uint64_t *lens, int n, uint64_t window)
{
    if (n <= 0 || n > ORACLE_MAX_SOURCES)
        return -1;
    if (window == 0)
        window = ORACLE_WINDOW;
    uint64_t max_cs = 0;
    for (int k = 0; k < n; k++) {
        uint64_t c = chunks[k] ? lens[k] : 0;
        if (c > max_cs)
            max_cs = c;
    }
    uint64_t total = 8ull * (uint64_t)n + max_cs;
    if (out_cap < total)
        return -1;
    oracle_sender snd[ORACLE_MAX_SOURCES];
    for (int k = 0; k < n; k++) {
        uint64_t c = chunks[k] ? lens[k] : 0;
        memcpy(out + 8 * k, &c, 8); /* host-endian header */
        snd[k] = (oracle_sender){chunks[k], c, 0, 0};
    }
    if (run_windows(out + 8ull * n, snd, n, max_cs, window) != 0)
        return -1;
    return (int64_t)total;
}

/*
 * Rebuild-mode output (task_processing.c:146-174, 228-230, with the parity
 * holder's chunk_sender skipping the header, :263-278).  Sources are the
 * surviving chunks (their *current* contents; NULL = unreadable) plus the
 * parity body.  max_cs comes from the stored header, not the survivors.
 * The rebuilt chunk is truncated to header[victim_index].
 * Returns the rebuilt length, or -1 on a malformed call.
 */
int64_t oracle_rebuild_chunk(uint8_t *out, uint64_t out_cap,
                             const uint8_t *parity_file, uint64_t parity_len,
                             const uint8_t *const *survivors,
                             const uint64_t *surv_lens, int nsurv,
                             int victim_index, uint64_t window)
{
    int n = nsurv + 1; /* header entries: survivors + victim */
    if (nsurv < 0 || n > ORACLE_MAX_SOURCES || victim_index < 0 ||
        victim_index >= n)
        return -1;
    if (window == 0)
        window = ORACLE_WINDOW;
    uint64_t hdr = 8ull * (uint64_t)n;
    if (parity_len < hdr)
        return -1;
    uint64_t sizes[ORACLE_MAX_SOURCES];
    memcpy(sizes, parity_file, hdr);
    uint64_t max_cs = 0;
    for (int k = 0; k < n; k++)
        if (sizes[k] > max_cs)
            max_cs = sizes[k];
    uint64_t cv = sizes[victim_index];
    uint8_t *body = malloc(max_cs ? max_cs : 1);
    if (!body)
        return -1;
    oracle_sender snd[ORACLE_MAX_SOURCES];
    for (int k = 0; k < nsurv; k++)
        snd[k] = (oracle_sender){survivors[k],
                                 survivors[k] ? surv_lens[k] : 0, 0, 0};
    snd[nsurv] = (oracle_sender){parity_file + hdr, parity_len - hdr, 0, 0};
    if (run_windows(body, snd, n, max_cs, window) != 0 || out_cap < cv) {
        free(body);
        return -1;
    }
    memcpy(out, body, cv);
    free(body);
    return (int64_t)cv;
}

/*
 * Index of the rebuilt target inside the stored header
 * (task_processing.c:169-174): survivors below the victim, with the parity
 * holder excluded.  `locations` is the re-roled FileInfo of do_file
 * (rebuild/main.c:55-60).  Uses 64-bit shifts where the reference shifts an
 * int (identical for storage targets < 31).
 */
int oracle_rebuild_index(uint64_t locations, int actual_P_st, int victim_st)
{
    const uint64_t L = UINT64_C(0x00FFFFFFFFFFFFFF);
    uint64_t loc = locations & ~(UINT64_C(1) << actual_P_st) & L;
    uint64_t below = (UINT64_C(1) << victim_st) - 1;
    return __builtin_popcountll(loc & below);
}

/* --- KAT generators ---------------------------------- */

/* KAT-1: data[i] = (uint8_t)(((uint64_t)i * 2654435761u) >> 13) */
void oracle_fill_kat1(uint8_t *buf, uint64_t len)
{
    for (uint64_t i = 0; i < len; i++)
        buf[i] = (uint8_t)((i * 2654435761u) >> 13);
}

/* KAT-2..4: byte j of chunk k = (uint8_t)((((uint64_t)k << 32) + j) * 2654435761u >> 13) */
void oracle_fill_kat_chunk(uint8_t *buf, uint64_t len, uint64_t k)
{
    for (uint64_t j = 0; j < len; j++)
        buf[j] = (uint8_t)((((k << 32) + j) * 2654435761u) >> 13);
}

/* splitmix64 stream used for synthetic stripes: word w = splitmix64(seed + w). */
static inline uint64_t splitmix64(uint64_t x)
{
    x += UINT64_C(0x9E3779B97F4A7C15);
    x = (x ^ (x >> 30)) * UINT64_C(0xBF58476D1CE4E5B9);
    x = (x ^ (x >> 27)) * UINT64_C(0x94D049BB133111EB);
    return x ^ (x >> 31);
}

void oracle_fill_synthetic(uint8_t *buf, uint64_t len, uint64_t seed,
                           uint64_t byte_offset)
{
    /* byte b of the virtual stream = byte (b & 7) of splitmix64(seed + b/8) */
    for (uint64_t i = 0; i < len; i++) {
        uint64_t b = byte_offset + i;
        uint64_t w = splitmix64(seed + (b >> 3));
        buf[i] = (uint8_t)(w >> (8 * (b & 7)));
    }
}

/* --- CPU baseline timing (bench.py cpu_baseline leg) -------------------- */

typedef void (*xor_fn)(uint8_t *, size_t, const uint8_t *, int);

typedef struct {
    xor_fn fn;         /* the fold timed: oracle_xor_parity or the reference's own */
    uint8_t *pool;     /* [nstripes][nsrc][chunk] */
    uint8_t *out;      /* [nstripes][chunk] */
    uint64_t nstripes, chunk;
    int nsrc;
    double seconds;    /* minimum wall time */
    uint64_t stripes_done;
    double elapsed;
} bench_arg;

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void *bench_thread(void *p)
{
    bench_arg *a = p;
    double t0 = now_s(), t;
    uint64_t done = 0;
    do {
        for (uint64_t s = 0; s < a->nstripes; s++) {
            a->fn(a->out + s * a->chunk, a->chunk,
                  a->pool + s * a->chunk * a->nsrc, a->nsrc);
            done++;
        }
        t = now_s();
    } while (t - t0 < a->seconds);
    a->stripes_done = done;
    a->elapsed = t - t0;
    return NULL;
}

/*
 * Times fn (xor_parity's signature; NULL = oracle_xor_parity) over `nthreads`
 * private pools of nstripes stripes (nsrc x chunk bytes each, synthetic
 * data), for at least `seconds`.  Returns aggregate algorithmic bytes/s
 * ((nsrc+1)*chunk per stripe) or <0.
 */
double oracle_bench_xor_fn(void *fn, int nthreads, uint64_t nstripes, int nsrc,
                           uint64_t chunk, double seconds)
{
    if (nthreads < 1 || nthreads > 256 || nsrc < 1)
        return -1.0;
    bench_arg args[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; t++) {
        args[t] = (bench_arg){0};
        args[t].fn = fn ? (xor_fn)fn : oracle_xor_parity;
        args[t].pool = malloc(nstripes * nsrc * chunk);
        args[t].out = malloc(nstripes * chunk);
        if (!args[t].pool || !args[t].out) {
            for (int u = 0; u <= t; u++) {
                free(args[u].pool);
                free(args[u].out);
            }
            return -2.0;
        }
        /* cheap non-constant fill; content does not affect integer XOR speed */
        uint64_t *w = (uint64_t *)args[t].pool;
        for (uint64_t i = 0; i < nstripes * nsrc * chunk / 8; i++)
            w[i] = splitmix64(i + 1000003ull * t);
        memset(args[t].out, 0, nstripes * chunk);
        args[t].nstripes = nstripes;
        args[t].chunk = chunk;
        args[t].nsrc = nsrc;
        args[t].seconds = seconds;
    }
    for (int t = 0; t < nthreads; t++)
        pthread_create(&th[t], NULL, bench_thread, &args[t]);
    double bytes = 0, worst = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        bytes += (double)args[t].stripes_done * (nsrc + 1) * (double)chunk;
        if (args[t].elapsed > worst)
            worst = args[t].elapsed;
        free(args[t].pool);
        free(args[t].out);
    }
    return bytes / worst;
}

double oracle_bench_xor(int nthreads, uint64_t nstripes, int nsrc,
                        uint64_t chunk, double seconds)
{
    return oracle_bench_xor_fn(NULL, nthreads, nstripes, nsrc, chunk, seconds);
}

/*
 * Mixed chunk sizes (config 5), as the reference's P role folds them: per
 * stripe one window of max_cs = max(len_k) bytes per source, each source's
 * bytes followed by zeros (chunk_sender zero-pads a short read,
 * task_processing.c:302-303), folded by fn = xor_parity(dst, max_cs, rows, n)
 * (task_processing.c:209).  lens is [nshapes][nsrc]; thread t folds the
 * shapes t, t+nthreads, ... (at least one each, cycled) from private buffers
 * for at least `seconds`.  Returns aggregate algorithmic bytes/s (sum of the
 * lengths + max_cs per stripe: the padding is not data) or < 0.  Every shape
 * must be <= one 10 MiB window (config 5's are <= 4 MiB).
 */
typedef struct {
    xor_fn fn;
    int nsrc;
    uint64_t nshapes;       /* this thread's shapes */
    uint8_t **rows;         /* [nshapes] -> nsrc * max_cs bytes */
    uint8_t *out;           /* largest max_cs */
    uint64_t *max_cs, *alg; /* [nshapes] */
    double seconds, elapsed, bytes;
} shape_arg;

static void *shape_thread(void *p)
{
    shape_arg *a = p;
    double t0 = now_s(), t, bytes = 0;
    do {
        for (uint64_t s = 0; s < a->nshapes; s++) {
            a->fn(a->out, a->max_cs[s], a->rows[s], a->nsrc);
            bytes += (double)a->alg[s];
        }
        t = now_s();
    } while (t - t0 < a->seconds);
    a->bytes = bytes;
    a->elapsed = t - t0;
    return NULL;
}

double oracle_bench_xor_shapes_fn(void *fn, int nthreads, const uint64_t *lens, uint64_t nshapes, int nsrc,
                                  double seconds)
{
    if (nthreads < 1 || nthreads > 256 || nsrc < 1 || nshapes < 1 || !lens)
        return -1.0;
    static shape_arg args[256];
    pthread_t th[256];
    double rc = 0;
    memset(args, 0, sizeof(args));
    for (int t = 0; t < nthreads; t++) {
        shape_arg *a = &args[t];
        a->fn = fn ? (xor_fn)fn : oracle_xor_parity;
        a->nsrc = nsrc;
        a->seconds = seconds;
        a->nshapes = nshapes > (uint64_t)nthreads ? (nshapes - (uint64_t)t + (uint64_t)nthreads - 1) / (uint64_t)nthreads : 1;
        a->rows = calloc(a->nshapes, sizeof(uint8_t *));
        a->max_cs = calloc(a->nshapes, sizeof(uint64_t));
        a->alg = calloc(a->nshapes, sizeof(uint64_t));
        if (!a->rows || !a->max_cs || !a->alg) {
            rc = -2.0;
            goto out;
        }
        uint64_t biggest = 1;
        for (uint64_t s = 0; s < a->nshapes; s++) {
            const uint64_t *l = lens + ((t + s * (uint64_t)nthreads) % nshapes) * (uint64_t)nsrc;
            uint64_t m = 0, sum = 0;
            for (int k = 0; k < nsrc; k++) {
                m = l[k] > m ? l[k] : m;
                sum += l[k];
            }
            if (m > 10u * 1024u * 1024u) {
                rc = -1.0;
                goto out;
            }
            a->max_cs[s] = m;
            a->alg[s] = sum + m;
            biggest = m > biggest ? m : biggest;
            a->rows[s] = malloc((size_t)(m ? m : 1) * (size_t)nsrc);
            if (!a->rows[s]) {
                rc = -2.0;
                goto out;
            }
            for (int k = 0; k < nsrc; k++) {
                uint8_t *row = a->rows[s] + (size_t)k * m;
                for (uint64_t i = 0; i < l[k]; i += 8) {
                    const uint64_t w = splitmix64(i / 8 + 7919ull * (uint64_t)k + 104729ull * s);
                    memcpy(row + i, &w, l[k] - i < 8 ? (size_t)(l[k] - i) : 8u);
                }
                memset(row + l[k], 0, (size_t)(m - l[k]));
            }
        }
        a->out = malloc((size_t)biggest);
        if (!a->out) {
            rc = -2.0;
            goto out;
        }
    }
    for (int t = 0; t < nthreads; t++)
        pthread_create(&th[t], NULL, shape_thread, &args[t]);
    double bytes = 0, worst = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        bytes += args[t].bytes;
        worst = args[t].elapsed > worst ? args[t].elapsed : worst;
    }
    rc = bytes / worst;
out:
    for (int t = 0; t < nthreads; t++) {
        shape_arg *a = &args[t];
        if (a->rows)
            for (uint64_t s = 0; s < a->nshapes; s++)
                free(a->rows[s]);
        free(a->rows);
        free(a->max_cs);
        free(a->alg);
        free(a->out);
    }
    return rc;
}
