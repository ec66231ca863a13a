/*
 * Host-side sanitizer driver (SURVEY.md §5 "sanitizers / race detection"):
 * the C++ host code of libmpix_redop.so and libmpix_coll.so, built with
 * -fsanitize=address,undefined or -fsanitize=thread (mpich_amd/csrc/Makefile
 * targets `asan` / `tsan`), driven from plain C the way an MPICH integrator
 * would: ranks are pthreads on the in-process host-memory transport, the
 * test oracle's C combine installed (the product has no CPU compute path).
 *
 * Every collective's result is checked against the closed forms of MPICH's
 * own tests (redscatblk3.c:48-78 for reduce-scatter, allred.c's SUM rule for
 * allreduce, reduce.c for reduce, scantst.c for scan), with ragged counts,
 * MPI_IN_PLACE and every algorithm; then the argument and legality paths of
 * both libraries (no GPU is touched).  Exit status = number of errors.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mpix_coll.h"
#include "mpix_redop.h"

int oracle_combine(const void *in, void *inout, long count, int dt, int op, void *stream);

#define PMAX 8
static int g_errs;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

static void err(const char *what, int rank, long i, long got, long want)
{
    pthread_mutex_lock(&g_mu);
    if (g_errs < 20)
        fprintf(stderr, "%s: rank %d [%ld] = %ld, expected %ld\n", what, rank, i, got, want);
    ++g_errs;
    pthread_mutex_unlock(&g_mu);
}

typedef struct {
    int rank, size, algo;
    MPIX_Comm comm;
    long n;             /* per-rank block (RSB) or vector length */
    int in_place;
} Arg;

static void *rsb_rank(void *p)
{
    Arg *a = p;
    const int P = a->size, r = a->rank;
    int *send = malloc(sizeof(int) * (size_t) (P * a->n + 1));
    int *recv = malloc(sizeof(int) * (size_t) (P * a->n + 1));
    for (int b = 0; b < P; ++b)         /* redscatblk3.c:43-48: block b of rank r holds r + b */
        for (long i = 0; i < a->n; ++i)
            (a->in_place ? recv : send)[b * a->n + i] = r + b;
    int rc = MPIX_Reduce_scatter_block(a->in_place ? NULL : send, recv, a->n, MPIX_MPI_INT,
                                       MPIX_SUM, a->comm, a->algo, NULL, 0);
    if (rc)
        err("MPIX_Reduce_scatter_block rc", r, -1, rc, 0);
    for (long i = 0; i < a->n && !rc; ++i)
        if (recv[i] != P * r + P * (P - 1) / 2)
            err("reduce_scatter_block", r, i, recv[i], P * r + P * (P - 1) / 2);
    free(send);
    free(recv);
    return NULL;
}

static void *rs_ragged_rank(void *p)
{
    Arg *a = p;
    const int P = a->size, r = a->rank;
    MPIX_Aint cnts[PMAX];
    long total = 0, disp = 0;
    for (int q = 0; q < P; ++q) {
        cnts[q] = (q * 7 + 3) % 5;      /* zeros included */
        total += cnts[q];
    }
    for (int q = 0; q < r; ++q)
        disp += cnts[q];
    double *send = malloc(sizeof(double) * (size_t) (total + 1));
    double *recv = malloc(sizeof(double) * (size_t) (total + 1));
    for (long i = 0; i < total; ++i)
        send[i] = (double) (i + 100 * r);
    int rc = MPIX_Reduce_scatter(send, recv, cnts, MPIX_MPI_DOUBLE, MPIX_SUM, a->comm, a->algo,
                                 NULL, 0);
    if (rc)
        err("MPIX_Reduce_scatter rc", r, -1, rc, 0);
    for (long i = 0; i < cnts[r] && !rc; ++i) {
        double want = (double) P * (double) (disp + i) + 100.0 * P * (P - 1) / 2;
        if (recv[i] != want)
            err("reduce_scatter ragged", r, i, (long) recv[i], (long) want);
    }
    free(send);
    free(recv);
    return NULL;
}

static void *allreduce_rank(void *p)
{
    Arg *a = p;
    const int P = a->size, r = a->rank;
    int *send = malloc(sizeof(int) * (size_t) a->n);
    int *recv = malloc(sizeof(int) * (size_t) a->n);
    for (long i = 0; i < a->n; ++i)
        (a->in_place ? recv : send)[i] = (int) i + r;
    int rc = MPIX_Allreduce(a->in_place ? NULL : send, recv, a->n, MPIX_MPI_INT, MPIX_SUM,
                            a->comm, a->algo, NULL, 0);
    if (rc)
        err("MPIX_Allreduce rc", r, -1, rc, 0);
    for (long i = 0; i < a->n && !rc; ++i)
        if (recv[i] != P * (int) i + P * (P - 1) / 2)
            err("allreduce", r, i, recv[i], P * (int) i + P * (P - 1) / 2);
    free(send);
    free(recv);
    return NULL;
}

static void *reduce_rank(void *p)
{
    Arg *a = p;
    const int P = a->size, r = a->rank, root = P - 1;
    int *send = malloc(sizeof(int) * (size_t) a->n);
    int *recv = malloc(sizeof(int) * (size_t) a->n);
    for (long i = 0; i < a->n; ++i)
        send[i] = (int) i;              /* reduce.c: in[i] = i, root gets i * P */
    int rc = MPIX_Reduce(send, r == root ? recv : NULL, a->n, MPIX_MPI_INT, MPIX_SUM, root,
                         a->comm, a->algo, NULL, 0);
    if (rc)
        err("MPIX_Reduce rc", r, -1, rc, 0);
    for (long i = 0; r == root && i < a->n && !rc; ++i)
        if (recv[i] != (int) i * P)
            err("reduce", r, i, recv[i], (int) i * P);
    free(send);
    free(recv);
    return NULL;
}

static void *scan_rank(void *p)
{
    Arg *a = p;
    const int r = a->rank;
    int *send = malloc(sizeof(int) * (size_t) a->n);
    int *recv = malloc(sizeof(int) * (size_t) a->n);
    for (long i = 0; i < a->n; ++i)
        send[i] = (int) i + r;          /* scantst.c-like: prefix sums */
    int rc = MPIX_Scan(send, recv, a->n, MPIX_MPI_INT, MPIX_SUM, a->comm, NULL, 0);
    if (rc)
        err("MPIX_Scan rc", r, -1, rc, 0);
    for (long i = 0; i < a->n && !rc; ++i) {
        int want = (r + 1) * (int) i + r * (r + 1) / 2;
        if (recv[i] != want)
            err("scan", r, i, recv[i], want);
    }
    free(send);
    free(recv);
    return NULL;
}

/* P threads, one per rank, on a fresh host communicator */
static void run(int P, void *(*fn)(void *), int algo, long n, int in_place)
{
    MPIX_Comm comms[PMAX];
    if (MPIX_Comm_create_local(P, NULL, comms)) {
        err("MPIX_Comm_create_local", -1, P, 1, 0);
        return;
    }
    pthread_t th[PMAX];
    Arg args[PMAX];
    for (int r = 0; r < P; ++r) {
        MPIX_Comm_set_combine(comms[r], (MPIX_Combine_fn) oracle_combine);
        args[r] = (Arg){r, P, algo, comms[r], n, in_place};
        pthread_create(&th[r], NULL, fn, &args[r]);
    }
    for (int r = 0; r < P; ++r)
        pthread_join(th[r], NULL);
    for (int r = 0; r < P; ++r)
        if (MPIX_Comm_free(comms[r]))
            err("MPIX_Comm_free", r, -1, 1, 0);
}

/* legality, handles and argument errors of both libraries (host only) */
static void boundary(void)
{
    int n_legal = 0;
    for (uint32_t opi = 1; opi <= 15; ++opi)
        for (uint32_t idx = 1; idx < 0x4d; ++idx) {
            MPIX_Op op = (MPIX_Op) (0x58000000u | opi);
            MPIX_Datatype dt = (MPIX_Datatype) (0x4c000000u | idx);
            n_legal += MPIX_Redop_op_dt_check(op, dt);
            (void) MPIX_Redop_is_supported(op, 17, dt);
            (void) MPIX_Datatype_internal(dt);
            (void) MPIX_Datatype_extent(dt);
            (void) MPIX_Datatype_size(dt);
        }
    if (n_legal < 100)
        err("legal pairs", -1, 0, n_legal, 100);
    int x[8] = {0}, y[8] = {0};
    if (MPIX_Reduce_local(x, y, -1, MPIX_MPI_INT, MPIX_SUM) != MPIX_REDOP_ERR_COUNT)
        err("negative count", -1, 0, 1, 0);
    if (MPIX_Reduce_local(NULL, y, 4, MPIX_MPI_INT, MPIX_SUM) != MPIX_REDOP_ERR_BUFFER)
        err("NULL inbuf", -1, 0, 1, 0);
    if (MPIX_Reduce_local(x, x + 1, 4, MPIX_MPI_INT, MPIX_SUM) != MPIX_REDOP_ERR_BUFFER)
        err("aliased", -1, 0, 1, 0);
    if (MPIX_Reduce_local(x, y, 4, MPIX_MPI_FLOAT, MPIX_BAND) != MPIX_REDOP_ERR_OP)
        err("BAND on float", -1, 0, 1, 0);
    if (MPIX_Reduce_local(x, y, 0, MPIX_MPI_INT, MPIX_SUM) != MPIX_REDOP_SUCCESS)
        err("count 0", -1, 0, 1, 0);
    MPIX_Redop_set_support(1, 64, 1 << 20, 1 << 20);
    if (MPIX_Redop_is_supported(MPIX_SUM, 17, MPIX_MPI_FLOAT))
        err("threshold", -1, 0, 1, 0);
    if (MPIX_Redop_is_supported_buffers(MPIX_SUM, 4, MPIX_MPI_FLOAT, x, y))
        err("host floor", -1, 0, 1, 0);
    MPIX_Redop_set_support(1, -1, 16 << 20, 4 << 20);
    /* collectives: bad arguments and declined pairs on every rank, no hang */
    MPIX_Comm c[3];
    if (MPIX_Comm_create_local(3, NULL, c) == MPIX_REDOP_SUCCESS) {
        if (MPIX_Reduce_scatter_block(x, y, 1, MPIX_MPI_INT, MPIX_SUM, c[0], 99, NULL, 0) !=
            MPIX_REDOP_ERR_ARG)
            err("bad algorithm", 0, 0, 1, 0);
        if (MPIX_Reduce_scatter_block(x, y, -1, MPIX_MPI_INT, MPIX_SUM, c[0], 0, NULL, 0) !=
            MPIX_REDOP_ERR_COUNT)
            err("negative recvcount", 0, 0, 1, 0);
        /* MAX on bf16: the one legal family without a kernel (op_fns.c asserts too) */
        if (MPIX_Reduce_scatter_block(x, y, 1, (MPIX_Datatype) 0x4c00024c, MPIX_MAX, c[0], 1, NULL,
                                      0) != MPIX_REDOP_ERR_TYPE)
            err("bf16 MAX declined", 0, 0, 1, 0);
        if (MPIX_Reduce_scatter_block(x, y, 1, MPIX_MPI_BYTE, MPIX_EQUAL, c[0], 1, NULL, 0) !=
            MPIX_REDOP_ERR_OP)
            err("EQUAL refused", 0, 0, 1, 0);
        for (int r = 0; r < 3; ++r)
            MPIX_Comm_free(c[r]);
    }
    if (MPIX_Comm_free(NULL) != MPIX_REDOP_ERR_ARG)
        err("free NULL", -1, 0, 1, 0);
}

int main(void)
{
    static const int Ps[] = {1, 2, 3, 4, 5, 7, 8};
    for (size_t k = 0; k < sizeof Ps / sizeof Ps[0]; ++k) {
        const int P = Ps[k];
        for (int algo = MPIX_RSB_AUTO; algo <= MPIX_RSB_LAST; ++algo) {
            run(P, rsb_rank, algo, 1000 + P, 0);
            run(P, rsb_rank, algo, 37, 1);
            run(P, rs_ragged_rank, algo, 0, 0);
        }
        for (int algo = MPIX_ALLREDUCE_AUTO; algo <= MPIX_ALLREDUCE_LAST; ++algo) {
            run(P, allreduce_rank, algo, 1031, 0);
            run(P, allreduce_rank, algo, 64, 1);
        }
        for (int algo = MPIX_REDUCE_AUTO; algo <= MPIX_REDUCE_SCATTER_GATHER; ++algo)
            run(P, reduce_rank, algo, 1031, 0);
        run(P, scan_rank, 0, 513, 0);
    }
    boundary();
    MPIX_Redop_finalize();
    printf("coll_host_sanitize: %d errors\n", g_errs);
    return g_errs;
}
