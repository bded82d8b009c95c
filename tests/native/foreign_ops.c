/* TEST: a caller's transport table -- the shape of the MPI binding in
 * INTEGRATION.md (blocking and non-blocking point-to-point, no send_fill) --
 * built on the loopback ranks behind wrapper functions, so libbcp cannot tell
 * it from a foreign transport: it gets the reference's zero-padded wire and
 * folds every window through the fold service.  foreign_ops() returns the
 * table for bcp_task_set_transport. */
#include "bcp_task.h"

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

static const bcp_transport_ops g_ops = {NULL, f_send, f_recv, f_isend, f_irecv, f_wait, f_waitall, NULL};

const bcp_transport_ops *foreign_ops(void) { return &g_ops; }
