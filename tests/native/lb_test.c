/* Loopback transport checks (CPU): bcp_lb_send_fill against posted and
 * unposted receives, ordering with plain sends on the same (source, tag),
 * truncation, fill errors, small blocking sends that do not wait for their
 * receive (eager), and tags that share a matching channel (tag and tag + 64)
 * kept apart and in order.  Two ranks as two threads. */
#include <errno.h>
#include <stdint.h>
#include <pthread.h>
#include <stdio.h>
#include <string.h>

#include "bcp_task.h"

static int fill_pattern(void *ctx, void *dst, size_t n)
{
    unsigned char base = *(unsigned char *)ctx;
    for (size_t i = 0; i < n; i++)
        ((unsigned char *)dst)[i] = (unsigned char)(base + i);
    return 0;
}

static int fill_fail(void *ctx, void *dst, size_t n)
{
    (void)ctx;
    memset(dst, 0, n);
    return -EIO;
}

static int failures = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            failures++;                                                   \
        }                                                                 \
    } while (0)

static void *sender(void *arg)
{
    (void)arg;
    bcp_lb_set_rank(0);
    unsigned char b1 = 1, b2 = 50, b3 = 100;
    /* 1: receiver posts late (fill waits for the match) */
    CHECK(bcp_lb_send_fill(fill_pattern, &b1, 4096, 1, 7) == 0);
    /* 2: plain send then fill send then plain send on the same tag: order kept */
    char msg[16] = "plain-one";
    CHECK(bcp_lb_send(msg, 10, 1, 8) == 0);
    CHECK(bcp_lb_send_fill(fill_pattern, &b2, 100, 1, 8) == 0);
    CHECK(bcp_lb_send("plain-two", 10, 1, 8) == 0);
    /* 3: truncated receive */
    CHECK(bcp_lb_send_fill(fill_pattern, &b3, 64, 1, 9) == -EMSGSIZE);
    /* 4: fill error reaches the sender, the receiver still completes */
    CHECK(bcp_lb_send_fill(fill_fail, NULL, 32, 1, 10) == -EIO);
    /* 5: receiver already posted (handshake first) */
    int go = 0;
    CHECK(bcp_lb_recv(&go, sizeof go, 1, 11, NULL) == 0);
    CHECK(bcp_lb_send_fill(fill_pattern, &b1, 256, 1, 12) == 0);
    /* 6: small blocking sends return before any receive is posted (the
     * receiver waits on tag 21 first: a rendezvous here would deadlock) */
    for (uint64_t v = 1; v <= 3; v++)
        CHECK(bcp_lb_send(&v, sizeof v, 1, 20) == 0);
    CHECK(bcp_lb_send(&go, sizeof go, 1, 21) == 0);
    /* 7: tags 30 and 94 share a channel; interleaved, received out of order */
    for (uint64_t v = 0; v < 4; v++)
        CHECK(bcp_lb_send(&v, sizeof v, 1, v % 2 ? 94 : 30) == 0);
    for (int t = 0; t < 200; t += 7) /* many tags, many channels */
        CHECK(bcp_lb_send(&t, sizeof t, 1, 1000 + t) == 0);
    return NULL;
}

int main(void)
{
    CHECK(bcp_lb_init(2) == 0);
    bcp_lb_set_rank(1);
    pthread_t th;
    pthread_create(&th, NULL, sender, NULL);
    unsigned char buf[8192];
    size_t got = 0;
    /* 1 */
    struct timespec ts = {0, 20 * 1000 * 1000};
    nanosleep(&ts, NULL);
    CHECK(bcp_lb_recv(buf, sizeof buf, 0, 7, &got) == 0 && got == 4096);
    int ok = 1;
    for (int i = 0; i < 4096; i++)
        ok &= buf[i] == (unsigned char)(1 + i);
    CHECK(ok);
    /* 2 */
    CHECK(bcp_lb_recv(buf, sizeof buf, 0, 8, &got) == 0 && got == 10 && !strcmp((char *)buf, "plain-one"));
    CHECK(bcp_lb_recv(buf, sizeof buf, 0, 8, &got) == 0 && got == 100 && buf[0] == 50 && buf[99] == (unsigned char)149);
    CHECK(bcp_lb_recv(buf, sizeof buf, 0, 8, &got) == 0 && got == 10 && !strcmp((char *)buf, "plain-two"));
    /* 3 */
    memset(buf, 0xEE, 64);
    CHECK(bcp_lb_recv(buf, 16, 0, 9, &got) == -EMSGSIZE && got == 16 && buf[0] == 100 && buf[15] == 115 &&
          buf[16] == 0xEE);
    /* 4 */
    CHECK(bcp_lb_recv(buf, sizeof buf, 0, 10, &got) == 0 && got == 32);
    /* 5: post first, then release the sender */
    bcp_lb_req *r = NULL;
    CHECK(bcp_lb_irecv(buf, sizeof buf, 0, 12, &r) == 0);
    int go = 1;
    CHECK(bcp_lb_send(&go, sizeof go, 0, 11) == 0);
    CHECK(bcp_lb_wait(r, &got) == 0 && got == 256 && buf[255] == (unsigned char)(1 + 255));
    /* 6 */
    CHECK(bcp_lb_recv(&go, sizeof go, 0, 21, NULL) == 0);
    for (uint64_t v = 1; v <= 3; v++) {
        uint64_t x = 0;
        CHECK(bcp_lb_recv(&x, sizeof x, 0, 20, &got) == 0 && got == 8 && x == v);
    }
    /* 7: tag 94 first (values 1, 3), then tag 30 (0, 2); then the 29 tags backwards */
    pthread_join(th, NULL);
    for (uint64_t want = 1; want < 4; want += 2) {
        uint64_t x = 99;
        CHECK(bcp_lb_recv(&x, sizeof x, 0, 94, NULL) == 0 && x == want);
    }
    for (uint64_t want = 0; want < 4; want += 2) {
        uint64_t x = 99;
        CHECK(bcp_lb_recv(&x, sizeof x, 0, 30, NULL) == 0 && x == want);
    }
    for (int t = 196; t >= 0; t -= 7) {
        int x = -1;
        CHECK(bcp_lb_recv(&x, sizeof x, 0, 1000 + t, NULL) == 0 && x == t);
    }
    CHECK(bcp_lb_finalize() == 0);
    printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
    return failures ? 1 : 0;
}
