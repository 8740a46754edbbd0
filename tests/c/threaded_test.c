/*
 * threaded_test.c -- concurrency of the drop-in liberasurecode.so.1 (include/erasurecode.h).
 *
 * Restates the scenarios of the reference's test/liberasurecode_threaded_test.c (which cannot be
 * compiled here: it includes the autoconf-generated config_liberasurecode.h): for each backend,
 * two threads racing instance_destroy on one descriptor, two racing instance_create, and
 * encode / decode / reconstruct_fragment / fragments_needed / get_fragment_size each racing a
 * destroy of their descriptor (the op returns 0 or -EBACKENDNOTAVAIL, the destroy always
 * succeeds).  Then a stress phase the reference does not have: NTHREADS threads sharing one
 * descriptor, each running encode -> decode (with erasures) -> reconstruct round trips on its own
 * random objects and checking every byte (the per-call GPU staging pool under contention).
 *
 * usage: threaded_test <backend_id> <k> <m> <hd> [nthreads] [iterations]
 */
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "erasurecode.h"

#define CHECK(cond)                                                                     \
    do {                                                                                \
        if (!(cond)) {                                                                  \
            fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #cond);    \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

static ec_backend_id_t g_be;
static struct ec_args g_args;

static char *random_buffer(int n, unsigned *seed)
{
    char *b = malloc(n);
    CHECK(b);
    for (int i = 0; i < n; i++) b[i] = (char)(rand_r(seed) & 0xff);
    return b;
}

/* ---- races against instance_destroy ---- */

static void *destroy_thread(void *arg)
{
    int *rc = malloc(sizeof(int));
    *rc = liberasurecode_instance_destroy(*(int *)arg);
    CHECK(*rc == 0 || *rc == -EBACKENDNOTAVAIL);
    return rc;
}

static void race_destroy(void)
{
    int desc = liberasurecode_instance_create(g_be, &g_args);
    CHECK(desc > 0);
    pthread_t a, b;
    int *ra, *rb;
    pthread_create(&a, NULL, destroy_thread, &desc);
    pthread_create(&b, NULL, destroy_thread, &desc);
    pthread_join(a, (void **)&ra);
    pthread_join(b, (void **)&rb);
    CHECK((*ra == 0) != (*rb == 0));  /* exactly one wins */
    CHECK(*ra == -EBACKENDNOTAVAIL || *rb == -EBACKENDNOTAVAIL);
    free(ra);
    free(rb);
}

static void *create_thread(void *arg)
{
    (void)arg;
    int *d = malloc(sizeof(int));
    *d = liberasurecode_instance_create(g_be, &g_args);
    return d;
}

static void race_create(void)
{
    pthread_t a, b;
    int *da, *db;
    pthread_create(&a, NULL, create_thread, NULL);
    pthread_create(&b, NULL, create_thread, NULL);
    pthread_join(a, (void **)&da);
    pthread_join(b, (void **)&db);
    CHECK(*da > 0 && *db > 0 && *da != *db);
    CHECK(liberasurecode_instance_destroy(*da) == 0);
    CHECK(liberasurecode_instance_destroy(*db) == 0);
    free(da);
    free(db);
}

struct op_state {
    int op;          /* 0 encode, 1 decode, 2 reconstruct, 3 fragments_needed, 4 fragment_size */
    int desc, desc2; /* desc2 stays alive for the cleanups */
    char *obj;
    int obj_len;
    char **frags;
    int nfrags;
    uint64_t frag_len;
};

static void *op_thread(void *arg)
{
    struct op_state *s = arg;
    int *rc = malloc(sizeof(int));
    if (s->op == 0) {
        char **d = NULL, **p = NULL;
        uint64_t fl = 0;
        *rc = liberasurecode_encode(s->desc, s->obj, s->obj_len, &d, &p, &fl);
        if (*rc == 0) CHECK(liberasurecode_encode_cleanup(s->desc2, d, p) == 0);
    } else if (s->op == 1) {
        char *out = NULL;
        uint64_t out_len = 0;
        *rc = liberasurecode_decode(s->desc, s->frags, s->nfrags, s->frag_len, 0, &out, &out_len);
        if (*rc == 0) CHECK(liberasurecode_decode_cleanup(s->desc2, out) == 0);
    } else if (s->op == 2) {
        char *out = malloc(s->frag_len);
        *rc = liberasurecode_reconstruct_fragment(s->desc, s->frags, s->nfrags, s->frag_len, 0, out);
        free(out);
    } else if (s->op == 3) {
        int recon[2] = {0, -1}, excl[1] = {-1};
        int *needed = malloc(sizeof(int) * (g_args.k + g_args.m + 1));
        *rc = liberasurecode_fragments_needed(s->desc, recon, excl, needed);
        free(needed);
    } else {
        *rc = liberasurecode_get_fragment_size(s->desc, 1 << 20);
        if (*rc > 0) *rc = 0;
    }
    CHECK(*rc == 0 || *rc == -EBACKENDNOTAVAIL);
    return rc;
}

static void race_op(int op)
{
    unsigned seed = 7 + op;
    struct op_state s;
    memset(&s, 0, sizeof(s));
    s.op = op;
    s.desc = liberasurecode_instance_create(g_be, &g_args);
    s.desc2 = liberasurecode_instance_create(g_be, &g_args);
    CHECK(s.desc > 0 && s.desc2 > 0);
    s.obj_len = 1 << 20;
    s.obj = random_buffer(s.obj_len, &seed);
    char **d = NULL, **p = NULL;
    if (op == 1 || op == 2) {
        CHECK(liberasurecode_encode(s.desc2, s.obj, s.obj_len, &d, &p, &s.frag_len) == 0);
        s.frags = malloc(sizeof(char *) * (g_args.k + g_args.m));
        for (int i = 0; i < g_args.k; i++) s.frags[s.nfrags++] = d[i];
        for (int i = 0; i < g_args.m; i++) s.frags[s.nfrags++] = p[i];
        if (op == 2) s.frags++, s.nfrags--; /* fragment 0 is the one to rebuild */
    }
    pthread_t a, b;
    int *ra, *rb;
    pthread_create(&b, NULL, op_thread, &s);
    pthread_create(&a, NULL, destroy_thread, &s.desc);
    pthread_join(a, (void **)&ra);
    pthread_join(b, (void **)&rb);
    CHECK(*ra == 0); /* destroy always succeeds */
    if (d) {
        if (op == 2) s.frags--;
        CHECK(liberasurecode_encode_cleanup(s.desc2, d, p) == 0);
        free(s.frags);
    }
    CHECK(liberasurecode_instance_destroy(s.desc2) == 0);
    free(ra);
    free(rb);
    free(s.obj);
}

/* ---- shared-descriptor stress ---- */

struct stress_state {
    int desc;
    int id;
    int iters;
};

static void *stress_thread(void *arg)
{
    struct stress_state *s = arg;
    unsigned seed = 1000u + (unsigned)s->id;
    const int n = g_args.k + g_args.m;
    const int max_lost = g_args.m < (g_args.hd > 0 ? g_args.hd - 1 : g_args.m)
                             ? g_args.m : (g_args.hd > 0 ? g_args.hd - 1 : g_args.m);
    for (int it = 0; it < s->iters; it++) {
        int len = 1 + (int)(rand_r(&seed) % (3 << 20));
        char *obj = random_buffer(len, &seed);
        char **d = NULL, **p = NULL;
        uint64_t fl = 0;
        CHECK(liberasurecode_encode(s->desc, obj, len, &d, &p, &fl) == 0);
        char **all = malloc(sizeof(char *) * n);
        for (int i = 0; i < g_args.k; i++) all[i] = d[i];
        for (int i = 0; i < g_args.m; i++) all[g_args.k + i] = p[i];
        /* lose `lost` random distinct fragments */
        int lost = 1 + (int)(rand_r(&seed) % max_lost);
        int *gone = calloc(n, sizeof(int));
        for (int c = 0; c < lost;) {
            int i = (int)(rand_r(&seed) % n);
            if (!gone[i]) gone[i] = 1, c++;
        }
        char **avail = malloc(sizeof(char *) * n);
        int na = 0, first_lost = -1;
        for (int i = 0; i < n; i++) {
            if (gone[i]) {
                if (first_lost < 0) first_lost = i;
            } else {
                avail[na++] = all[i];
            }
        }
        char *out = NULL;
        uint64_t out_len = 0;
        CHECK(liberasurecode_decode(s->desc, avail, na, fl, 0, &out, &out_len) == 0);
        CHECK(out_len == (uint64_t)len && memcmp(out, obj, len) == 0);
        CHECK(liberasurecode_decode_cleanup(s->desc, out) == 0);
        char *rebuilt = malloc(fl);
        CHECK(liberasurecode_reconstruct_fragment(s->desc, avail, na, fl, first_lost, rebuilt) == 0);
        CHECK(memcmp(rebuilt, all[first_lost], fl) == 0);
        free(rebuilt);
        free(avail);
        free(gone);
        free(all);
        CHECK(liberasurecode_encode_cleanup(s->desc, d, p) == 0);
        free(obj);
    }
    return NULL;
}

int main(int argc, char **argv)
{
    if (argc < 5) {
        fprintf(stderr, "usage: %s backend k m hd [nthreads] [iterations]\n", argv[0]);
        return 2;
    }
    g_be = (ec_backend_id_t)atoi(argv[1]);
    memset(&g_args, 0, sizeof(g_args));
    g_args.k = atoi(argv[2]);
    g_args.m = atoi(argv[3]);
    g_args.hd = atoi(argv[4]);
    g_args.w = 16;
    g_args.ct = CHKSUM_CRC32;
    int nthreads = argc > 5 ? atoi(argv[5]) : 8;
    int iters = argc > 6 ? atoi(argv[6]) : 4;
    if (!liberasurecode_backend_available(g_be)) {
        printf("skip: backend %d not available\n", g_be);
        return 3;
    }
    race_destroy();
    printf("race_destroy ok\n");
    race_create();
    printf("race_create ok\n");
    for (int op = 0; op < 5; op++) {
        race_op(op);
        printf("race_op %d ok\n", op);
    }
    int desc = liberasurecode_instance_create(g_be, &g_args);
    CHECK(desc > 0);
    pthread_t *t = malloc(sizeof(pthread_t) * nthreads);
    struct stress_state *st = malloc(sizeof(struct stress_state) * nthreads);
    for (int i = 0; i < nthreads; i++) {
        st[i].desc = desc;
        st[i].id = i;
        st[i].iters = iters;
        pthread_create(&t[i], NULL, stress_thread, &st[i]);
    }
    for (int i = 0; i < nthreads; i++) pthread_join(t[i], NULL);
    CHECK(liberasurecode_instance_destroy(desc) == 0);
    printf("stress %d threads x %d ok\n", nthreads, iters);
    free(t);
    free(st);
    return 0;
}
