/* Lock-contention counters for a diagnostic build of the C host layer
 * (tools/exp/lockstat/build.sh; never in the product): every
 * pthread_mutex_lock / pthread_cond_wait in csrc/*.c is counted per call site,
 * contended = the lock was held when asked for.  Dumped at exit to stderr. */
#pragma once
#include <pthread.h>
int lockstat_lock(pthread_mutex_t *m, const char *f, int l);
int lockstat_wait(pthread_cond_t *c, pthread_mutex_t *m, const char *f, int l);
#define pthread_mutex_lock(m) lockstat_lock((m), __FILE__, __LINE__)
#define pthread_cond_wait(c, m) lockstat_wait((c), (m), __FILE__, __LINE__)
