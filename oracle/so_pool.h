/*
 * so_pool.h -- a persistent worker pool for the CPU batch drivers of
 * suruga_oracle.c and ossl_aead.c.  TEST / BENCHMARK INFRASTRUCTURE ONLY.
 *
 * sp_run(fn, ctx, nt) calls fn(ctx, t, nt) for t = 0 .. nt-1, t = 0 on the
 * calling thread and the others on pool threads that are created on first use
 * and then parked on a condition variable, so a timed batch pays no thread
 * creation (round 2 spawned and joined one pthread per batch call per thread,
 * which dominated the 16-record slices of bench.py's CPU sample).  Callers are
 * serialised: one batch runs on the pool at a time.  Header-only (static), so
 * each library that includes it owns its own pool.
 */
#ifndef SO_POOL_H
#define SO_POOL_H

#include <pthread.h>
#include <stdint.h>

#define SP_MAX_THREADS 1024

typedef void (*sp_fn)(void* ctx, int t, int nt);

typedef struct {
    pthread_mutex_t run_mu; /* one batch at a time */
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    int nth;       /* worker threads created (indices 1 .. nth) */
    uint64_t gen;  /* batch generation */
    int busy;      /* workers still inside the current generation */
    sp_fn fn;
    void* ctx;
    int nt;
} sp_pool_t;

static sp_pool_t sp_pool = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER,
                            PTHREAD_COND_INITIALIZER, 0, 0, 0, 0, 0, 0};
static uint64_t sp_born[SP_MAX_THREADS + 1]; /* the generation current when worker i was created */

static void* sp_worker(void* arg) {
    const int me = (int)(intptr_t)arg;
    uint64_t seen;
    pthread_mutex_lock(&sp_pool.mu);
    seen = sp_born[me]; /* a worker created for the current batch still runs it */
    pthread_mutex_unlock(&sp_pool.mu);
    for (;;) {
        sp_fn fn;
        void* ctx;
        int nt;
        pthread_mutex_lock(&sp_pool.mu);
        while (sp_pool.gen == seen) pthread_cond_wait(&sp_pool.go, &sp_pool.mu);
        seen = sp_pool.gen;
        fn = sp_pool.fn;
        ctx = sp_pool.ctx;
        nt = sp_pool.nt;
        pthread_mutex_unlock(&sp_pool.mu);
        if (me < nt) fn(ctx, me, nt);
        pthread_mutex_lock(&sp_pool.mu);
        if (--sp_pool.busy == 0) pthread_cond_signal(&sp_pool.done);
        pthread_mutex_unlock(&sp_pool.mu);
    }
    return 0;
}

/* Runs fn on nt threads (the caller is thread 0) and returns when all are done. */
static void sp_run(sp_fn fn, void* ctx, int nt) {
    if (nt < 1) nt = 1;
    if (nt > SP_MAX_THREADS) nt = SP_MAX_THREADS;
    if (nt == 1) {
        fn(ctx, 0, 1);
        return;
    }
    pthread_mutex_lock(&sp_pool.run_mu);
    pthread_mutex_lock(&sp_pool.mu);
    while (sp_pool.nth < nt - 1) { /* workers never exit: the pool only grows */
        pthread_t th;
        pthread_attr_t at;
        pthread_attr_init(&at);
        pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
        sp_born[sp_pool.nth + 1] = sp_pool.gen;
        const int ok = pthread_create(&th, &at, sp_worker, (void*)(intptr_t)(sp_pool.nth + 1)) == 0;
        pthread_attr_destroy(&at);
        if (!ok) break;
        ++sp_pool.nth;
    }
    if (nt > sp_pool.nth + 1) nt = sp_pool.nth + 1; /* thread creation refused: run on what exists */
    sp_pool.fn = fn;
    sp_pool.ctx = ctx;
    sp_pool.nt = nt;
    sp_pool.busy = sp_pool.nth;
    ++sp_pool.gen;
    pthread_cond_broadcast(&sp_pool.go);
    pthread_mutex_unlock(&sp_pool.mu);
    fn(ctx, 0, nt);
    pthread_mutex_lock(&sp_pool.mu);
    while (sp_pool.busy > 0) pthread_cond_wait(&sp_pool.done, &sp_pool.mu);
    pthread_mutex_unlock(&sp_pool.mu);
    pthread_mutex_unlock(&sp_pool.run_mu);
}

/* [begin, end) of `count` items for thread t of nt (contiguous, sizes differ by <= 1) */
static void sp_range(size_t count, int t, int nt, size_t* begin, size_t* end) {
    const size_t base = count / (size_t)nt, extra = count % (size_t)nt;
    *begin = (size_t)t * base + ((size_t)t < extra ? (size_t)t : extra);
    *end = *begin + base + ((size_t)t < extra ? 1u : 0u);
}

#endif
