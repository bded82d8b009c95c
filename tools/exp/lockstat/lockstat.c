#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define NSITES 512
typedef struct { const char *f; int l; int kind; uint64_t calls, contended; } site;
static site g_sites[NSITES];

static site *get(const char *f, int l, int kind)
{
    size_t h = ((uintptr_t)f * 31u + (unsigned)l * 7u + (unsigned)kind) % NSITES;
    for (int k = 0; k < NSITES; k++, h = (h + 1) % NSITES) {
        site *s = &g_sites[h];
        const char *cur = __atomic_load_n(&s->f, __ATOMIC_ACQUIRE);
        if (cur == f && s->l == l && s->kind == kind)
            return s;
        if (!cur) {
            const char *z = NULL;
            if (__atomic_compare_exchange_n(&s->f, &z, (const char *)"?", 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
                s->l = l;
                s->kind = kind;
                __atomic_store_n(&s->f, f, __ATOMIC_RELEASE);
                return s;
            }
            while (__atomic_load_n(&s->f, __ATOMIC_ACQUIRE) == (const char *)"?")
                ;
            if (s->f == f && s->l == l && s->kind == kind)
                return s;
        }
    }
    return &g_sites[0];
}

int lockstat_lock(pthread_mutex_t *m, const char *f, int l)
{
    site *s = get(f, l, 0);
    __atomic_fetch_add(&s->calls, 1, __ATOMIC_RELAXED);
    if (pthread_mutex_trylock(m) == 0)
        return 0;
    __atomic_fetch_add(&s->contended, 1, __ATOMIC_RELAXED);
    return pthread_mutex_lock(m);
}

int lockstat_wait(pthread_cond_t *c, pthread_mutex_t *m, const char *f, int l)
{
    site *s = get(f, l, 1);
    __atomic_fetch_add(&s->calls, 1, __ATOMIC_RELAXED);
    return pthread_cond_wait(c, m);
}

__attribute__((destructor)) static void dump(void)
{
    for (int i = 0; i < NSITES; i++)
        if (g_sites[i].f && g_sites[i].calls)
            fprintf(stderr, "lockstat %s %s:%d calls %llu contended %llu\n", g_sites[i].kind ? "wait" : "lock",
                    g_sites[i].f, g_sites[i].l, (unsigned long long)g_sites[i].calls,
                    (unsigned long long)g_sites[i].contended);
}
