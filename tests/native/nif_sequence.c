/* nif_sequence.c — the C-ABI call sequence of the Erlang NIF in INTEGRATION.md §2, without
 * Erlang: engine -> batcher (tm_batcher_create) -> match_async-style submits from several
 * "scheduler" threads, each publish answered through a callback that posts a message to the
 * publishing "process" (a mailbox standing in for enif_send; the process waits for it as
 * `receive` would) -> writes through the batcher between windows (batch_apply/2) -> destroy,
 * which must drain every queued publish.
 *
 *   nif_sequence cpu   over a custom backend (tm_batcher_create_fn): no GPU needed
 *   nif_sequence gpu   over a real engine on device 0; every publish's ids are checked
 *                      against a brute-force restatement of emqx_topic:match/2
 *                      (apps/emqx/src/emqx_topic.erl:78-102)
 * Test infrastructure (tests/test_nif_sequence.py runs it); exit status 0 = pass. */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/emqx_tm.h"
#include "../../include/emqx_tm_batcher.h"

#define SCHEDULERS 8
#define PUBS_PER_SCHEDULER 3000
#define MAXIDS 64

static int failures = 0;
static pthread_mutex_t fail_mu = PTHREAD_MUTEX_INITIALIZER;
static void fail(const char *what, const char *topic) {
    pthread_mutex_lock(&fail_mu);
    if (failures++ < 10) fprintf(stderr, "FAIL %s: %s\n", what, topic);
    pthread_mutex_unlock(&fail_mu);
}

/* ---- emqx_topic:match/2, restated (test oracle) */
static int level(const char *s, size_t n, size_t *pos, const char **w, size_t *wl) {
    if (*pos > n) return 0;
    size_t st = *pos, e = st;
    while (e < n && s[e] != '/') e++;
    *w = s + st;
    *wl = e - st;
    *pos = e + 1;
    return 1;
}
static int topic_match(const char *t, const char *f) {
    size_t tn = strlen(t), fn = strlen(f), tp = 0, fp = 0;
    if (tn && t[0] == '$' && fn && (f[0] == '+' || f[0] == '#') && (fn == 1 || f[1] == '/')) return 0;
    for (;;) {
        const char *tw, *fw;
        size_t tl, fl;
        int ht = level(t, tn, &tp, &tw, &tl), hf = level(f, fn, &fp, &fw, &fl);
        if (!hf) return !ht;
        if (fl == 1 && fw[0] == '#' && fp > fn) return 1; /* '#' last: zero or more levels */
        if (!ht) return 0;
        if (fl == 1 && fw[0] == '+') continue;
        if (fl != tl || memcmp(fw, tw, tl) != 0) return 0;
    }
}

/* ---- routes */
typedef struct { const char *filter; uint64_t id; int live; } route;
static route routes[] = {
    {"a/+/c", 1, 1}, {"a/#", 2, 1}, {"#", 3, 1}, {"+/b/+", 4, 1}, {"$SYS/#", 5, 1}, {"a/b/c", 6, 1},
    {"x//y", 7, 1}, {"+", 8, 1}, {"+/+", 9, 1}, {"sport/tennis/#", 10, 1}, {"a/b/c", 11, 1}, {"$SYS/+/x", 12, 1},
};
#define NROUTES (sizeof routes / sizeof routes[0])
static const char *topics[] = {"a/b/c", "a", "a/b", "x//y", "$SYS/n/x", "$SYS", "sport/tennis", "sport/tennis/p1/r",
                               "q", "", "/", "a/+/c", "a/#", "b/b/b", "zz/b/q", "$x/b/y"};
#define NTOPICS (sizeof topics / sizeof topics[0])

static int expected(const char *t, uint64_t *out) {
    int n = 0;
    for (size_t r = 0; r < NROUTES; r++)
        if (routes[r].live && topic_match(t, routes[r].filter)) out[n++] = routes[r].id;
    return n;
}
static int is_badarg(const char *t) {
    size_t n = strlen(t), p = 0;
    const char *w;
    size_t wl;
    while (level(t, n, &p, &w, &wl))
        if (wl == 1 && (w[0] == '+' || w[0] == '#')) return 1;
    return 0;
}
static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* ---- a "process": one mailbox; the callback is the NIF's on_match (enif_send) */
typedef struct {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int n_msgs;
    int32_t status;
    uint32_t n;
    uint64_t ids[MAXIDS];
} mailbox;

typedef struct { mailbox *mb; } pub_ctx; /* the NIF's {pid, env, ref} */

static void on_match(void *ctx, int32_t status, const uint64_t *ids, uint32_t n) {
    pub_ctx *c = ctx;
    mailbox *mb = c->mb;
    pthread_mutex_lock(&mb->mu);
    mb->status = status;
    mb->n = n < MAXIDS ? n : MAXIDS;
    if (ids) memcpy(mb->ids, ids, mb->n * 8);
    mb->n_msgs++;
    pthread_cond_signal(&mb->cv);
    pthread_mutex_unlock(&mb->mu);
    free(c);
}

static tm_batcher *g_b;
static int g_gpu;
static int fake_answer(const char *t, uint64_t *ids); /* cpu backend's answers */

static void *scheduler(void *arg) {
    const int me = (int)(intptr_t)arg;
    mailbox mb;
    pthread_mutex_init(&mb.mu, NULL);
    pthread_cond_init(&mb.cv, NULL);
    mb.n_msgs = 0;
    for (int k = 0; k < PUBS_PER_SCHEDULER; k++) {
        const char *t = topics[(me * 7 + k) % NTOPICS];
        pub_ctx *c = malloc(sizeof *c);
        c->mb = &mb;
        const int before = mb.n_msgs;
        if (tm_batcher_submit(g_b, (const uint8_t *)t, (uint32_t)strlen(t), on_match, c) != TM_OK) {
            free(c);
            fail("submit", t);
            continue;
        }
        pthread_mutex_lock(&mb.mu); /* receive {tm_match, Ref, Result} */
        while (mb.n_msgs == before) pthread_cond_wait(&mb.cv, &mb.mu);
        pthread_mutex_unlock(&mb.mu);
        uint64_t exp[MAXIDS];
        int ne = g_gpu ? expected(t, exp) : fake_answer(t, exp);
        if (is_badarg(t)) {
            if (mb.status != TM_BADARG) fail("badarg", t);
            continue;
        }
        if (mb.status != TM_TOPIC_OK || (int)mb.n != ne) {
            fail("count", t);
            continue;
        }
        qsort(mb.ids, mb.n, 8, cmp_u64);
        qsort(exp, ne, 8, cmp_u64);
        if (memcmp(mb.ids, exp, ne * 8)) fail("ids", t);
    }
    pthread_mutex_destroy(&mb.mu);
    pthread_cond_destroy(&mb.cv);
    return NULL;
}

static int run_schedulers(void) {
    pthread_t th[SCHEDULERS];
    for (int i = 0; i < SCHEDULERS; i++) pthread_create(&th[i], NULL, scheduler, (void *)(intptr_t)i);
    for (int i = 0; i < SCHEDULERS; i++) pthread_join(th[i], NULL);
    return failures;
}

/* ---- cpu backend: answers from the restated match over the route table */
static int fake_answer(const char *t, uint64_t *ids) { return expected(t, ids); }
static int fake_batch(void *be, const uint8_t *bytes, const uint32_t *off, uint32_t n, uint32_t mode,
                      tm_batch_view *v) {
    (void)be;
    (void)mode;
    static uint32_t *o, *cnt;
    static int32_t *st;
    static uint64_t *ids;
    static uint32_t cap;
    if (n > cap) {
        cap = n;
        o = realloc(o, n * 4);
        cnt = realloc(cnt, n * 4);
        st = realloc(st, n * 4);
        ids = realloc(ids, (size_t)n * MAXIDS * 8);
    }
    char t[256];
    for (uint32_t i = 0; i < n; i++) {
        uint32_t len = off[i + 1] - off[i];
        memcpy(t, bytes + off[i], len);
        t[len] = 0;
        o[i] = i * MAXIDS;
        st[i] = is_badarg(t) ? TM_BADARG : TM_TOPIC_OK;
        cnt[i] = st[i] ? 0 : (uint32_t)expected(t, ids + (size_t)i * MAXIDS);
    }
    v->off = o;
    v->cnt = cnt;
    v->ids = ids;
    v->status = st;
    return TM_OK;
}

/* publishes left in flight when destroy begins must all be answered */
static int drained;
static void on_drain(void *ctx, int32_t status, const uint64_t *ids, uint32_t n) {
    (void)ctx;
    (void)ids;
    (void)n;
    if (status >= 0) __atomic_add_fetch(&drained, 1, __ATOMIC_RELAXED);
}

int main(int argc, char **argv) {
    g_gpu = argc > 1 && !strcmp(argv[1], "gpu");
    tm_engine *eng = NULL;
    tm_batcher_config cfg = {.max_batch = 1024, .max_wait_us = 100, .mode = TM_MATCH_ALL, .delivery_threads = 4};
    int rc;
    if (g_gpu) {
        tm_config ec;
        memset(&ec, 0, sizeof ec);
        if ((rc = tm_create(&ec, &eng)) != TM_OK) return fprintf(stderr, "tm_create %d\n", rc), 2;
        if ((rc = tm_batcher_create(eng, &cfg, &g_b)) != TM_OK) return fprintf(stderr, "batcher %d\n", rc), 2;
        /* batch_apply/2: the route table through the batcher */
        tm_op ops[NROUTES];
        for (size_t r = 0; r < NROUTES; r++)
            ops[r] = (tm_op){.op = TM_OP_ADD, .flags = 0, .filter = (const uint8_t *)routes[r].filter,
                             .filter_len = (uint32_t)strlen(routes[r].filter), .id = routes[r].id};
        uint64_t ep = 0;
        if ((rc = tm_batcher_apply(g_b, ops, NROUTES)) || (rc = tm_batcher_commit(g_b, &ep)))
            return fprintf(stderr, "apply %d\n", rc), 2;
    } else {
        if ((rc = tm_batcher_create_fn(fake_batch, NULL, &cfg, &g_b)) != TM_OK) return fprintf(stderr, "fn %d\n", rc), 2;
        /* writes need an engine batcher */
        if (tm_batcher_apply(g_b, NULL, 0) != TM_ESTATE) fail("apply on a custom backend", "");
    }
    run_schedulers();
    if (g_gpu) { /* a second epoch while the batcher runs: delete two routes, add one */
        tm_op ops[3] = {{.op = TM_OP_DEL, .filter = (const uint8_t *)"#", .filter_len = 1, .id = 3},
                        {.op = TM_OP_DEL, .filter = (const uint8_t *)"a/b/c", .filter_len = 5, .id = 11},
                        {.op = TM_OP_ADD, .filter = (const uint8_t *)"b/+", .filter_len = 3, .id = 13}};
        routes[2].live = 0;
        routes[10].live = 0;
        uint64_t ep = 0;
        if ((rc = tm_batcher_apply(g_b, ops, 3)) || (rc = tm_batcher_commit(g_b, &ep)))
            return fprintf(stderr, "apply %d\n", rc), 2;
        run_schedulers(); /* "b/+" (13) is not in routes[]: no topic of the set matches it */
    }
    /* batcher_destroy/1 with publishes still queued: every one is answered first */
    const int inflight = 5000;
    for (int i = 0; i < inflight; i++)
        if (tm_batcher_submit(g_b, (const uint8_t *)"a/b/c", 5, on_drain, NULL) != TM_OK) fail("submit", "drain");
    tm_batcher_destroy(g_b);
    if (drained != inflight) fail("drain", "destroy");
    if (eng) tm_destroy(eng);
    printf("nif_sequence %s: %d failures, %d publishes\n", g_gpu ? "gpu" : "cpu", failures,
           SCHEDULERS * PUBS_PER_SCHEDULER * (g_gpu ? 2 : 1) + inflight);
    return failures ? 1 : 0;
}
