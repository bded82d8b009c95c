/* bcp_runner.h -- internal: what the thread runner (bcp_runner.c) and the
 * rank pool (bcp_pool.c) share -- a rank's host state, the lane start gate
 * and the lane bodies (process_list / do_file).  Not part of the C ABI. */
#pragma once

#include <pthread.h>

#include "bcp_host.h"

typedef struct {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int open, cancel;
} start_gate;

#define START_GATE_INIT {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, 0, 0}

typedef struct {
    HostState *hs;
    const bcp_work_item *items;
    size_t nitems;
    const int *lanes;
    int lane;
    int rank;
    bcp_pdb *db;         /* this rank's replica, or NULL */
    start_gate *gate;
    ProgressSample sample;
    uint64_t tasks;
    int db_rc;
} lane_arg;

typedef struct {
    HostState *hs;
    const bcp_work_item *items;
    size_t nitems;
    int rebuild_target;
    int rank;
    start_gate *gate;
    ProgressSample sample;
    uint64_t tasks;
    int lane, nlanes; /* items i with i % nlanes == lane, MPI tag = lane */
} rebuild_arg;

double bcpr_now_s(void);
/* <root>/st<st>/{chunks,parity} as the rank's HostState (gen/main.c:723-743,
 * rebuild/main.c:200-225); bcpr_close_store closes what it opened. */
int bcpr_open_store(const char *root, int st, int rebuilding, int corrupt_fd, FILE *log, HostState *hs);
void bcpr_close_store(HostState *hs, int rebuilding);
/* Lane side: wait until the runner opens the gate; 1 = run, 0 = cancelled. */
int bcpr_gate_pass(start_gate *g);
void bcpr_gate_open(start_gate *g, int cancel);
/* pthread_create, or EAGAIN under failure injection (BCP_INJECT_THREAD) */
int bcpr_spawn(pthread_t *th, void *(*fn)(void *), void *arg);
/* process_list (gen/main.c:116-164) for one lane of one rank; arg lane_arg */
void *bcpr_gen_lane(void *p);
/* do_file (rebuild/main.c:40-89) over the item list, one lane; arg rebuild_arg */
void *bcpr_rebuild_rank(void *p);
int bcpr_rebuild_lanes(void);
/* -EINVAL for an item process_task would assert on or that names a target
 * outside the world */
int bcpr_check_items(int ntargets, const bcp_work_item *items, size_t nitems);
uint64_t bcpr_count_refused(const bcp_work_item *items, size_t nitems, int rebuild_target);
