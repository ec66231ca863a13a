/* host_bench.c -- CPU-baseline harness for bench.py (TEST/MEASUREMENT
 * INFRASTRUCTURE, never linked into the product; built into
 * oracle/build/liboracle_redop.so next to the oracle it times).
 *
 * The reference path (MPICH's op_fns.c loop, restated by redop_oracle.c) is
 * one thread per rank; its "all cores" aggregate runs one
 * thread per physical core on disjoint slices.  To be a fair host figure the
 * threads are pinned (one CPU each) and every thread allocates and first-
 * touches its own slice on its own CPU, so each slice lives in the NUMA node
 * of the core that streams it.  A host STREAM-style triad (fp32, the
 * same pinned, first-touched layout; in place, see triad_inplace) gives the
 * host-memory roofline the CPU figure is read against.
 *
 * Both runners start the threads once, then time whole passes (all threads
 * between two barriers) until `seconds` have passed (at least 3 passes), and
 * return the best and median pass time. */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

int oracle_reduce_local(const void *in, void *inout, long count, int dt, int op);
long oracle_extent(int dt);

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

enum { K_REDUCE = 0, K_TRIAD = 1, K_PAIR = 2 };

/* the host roofline kernel: a += 0.5 b, vectorised -- the combine's own
 * traffic (2 reads + 1 write per element into lines it has just read, so no
 * write-allocate), i.e. STREAM's triad in the in-place form */
__attribute__((optimize("O3", "tree-vectorize"), noinline))
static void triad_inplace(float *restrict a, const float *restrict b, long n)
{
    for (long i = 0; i < n; ++i)
        a[i] = a[i] + 0.5f * b[i];
}

struct hb_shared {
    int kind, nthreads, dt, op;
    long count;                 /* elements over all threads */
    double seconds;
    pthread_barrier_t bar;
    volatile int stop;
    int rc;
    int passes;
    double *times;              /* per pass, filled by thread 0 */
    double *times2;             /* K_PAIR: the triad half of each pass */
    int max_passes;
    double t_first, t_last;     /* start of the first pass, end of the last */
};

struct hb_thread {
    struct hb_shared *sh;
    int tid, cpu;
};

static void *hb_run(void *p)
{
    struct hb_thread *t = p;
    struct hb_shared *sh = t->sh;
    if (t->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(t->cpu, &set);
        (void) pthread_setaffinity_np(pthread_self(), sizeof set, &set);
    }
    const long per = (sh->count + sh->nthreads - 1) / sh->nthreads;
    const long lo = (long) t->tid * per;
    const long n = lo >= sh->count ? 0 : (lo + per > sh->count ? sh->count - lo : per);
    const long ext = sh->kind == K_REDUCE ? oracle_extent(sh->dt) : 4;
    const size_t bytes = (size_t) (n > 0 ? n : 1) * (size_t) ext;
    /* first touch on the pinned CPU: the pages land in its NUMA node; 2 MiB
     * pages where the kernel gives them (numpy asks for them too, and a
     * 4 KiB-page TLB walk per 64 B line halves one core's stream rate) */
    char *a = NULL, *b = NULL;
    if (posix_memalign((void **) &a, 1 << 21, bytes) || posix_memalign((void **) &b, 1 << 21, bytes))
        sh->rc = 1;
    else {
        (void) madvise(a, bytes, MADV_HUGEPAGE);
        (void) madvise(b, bytes, MADV_HUGEPAGE);
    }
    if (sh->rc != 1) {
        float *fa = (float *) a, *fb = (float *) b;
        unsigned x = 0x5EED0001u + (unsigned) t->tid;
        for (long i = 0; i < (long) (bytes / 4); ++i) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            fa[i] = (float) (x & 0xffff) * (1.0f / 65536.0f) - 0.5f;
            fb[i] = (float) ((x >> 16) & 0xffff) * (1.0f / 65536.0f) - 0.5f;
        }
    }
    pthread_barrier_wait(&sh->bar);
    const double t_end = now_s() + sh->seconds;
    for (int pass = 0;; ++pass) {
        pthread_barrier_wait(&sh->bar);
        if (sh->stop || sh->rc)
            break;
        double t0 = now_s();
        if (n > 0 && a && b) {
            if (sh->kind != K_TRIAD) {
                if (oracle_reduce_local(b, a, n, sh->dt, sh->op))
                    sh->rc = 2;
            } else {
                triad_inplace((float *) a, (const float *) b, n);
            }
        }
        pthread_barrier_wait(&sh->bar);
        /* K_PAIR: the triad right after the reduce, on the same threads, pages
         * and quota window, so the two rates are read off the same pass */
        double t1 = now_s(), t2 = t1;
        if (sh->kind == K_PAIR) {
            if (n > 0 && a && b)
                triad_inplace((float *) a, (const float *) b, n);
            pthread_barrier_wait(&sh->bar);
            t2 = now_s();
        }
        if (t->tid == 0) {
            if (pass == 0)
                sh->t_first = t0;
            sh->t_last = t2;
            if (pass < sh->max_passes) {
                sh->times[pass] = t1 - t0;
                if (sh->times2)
                    sh->times2[pass] = t2 - t1;
            }
            sh->passes = pass + 1;
            if ((now_s() >= t_end && pass >= 2) || pass + 1 >= sh->max_passes)
                sh->stop = 1;
        }
    }
    free(a);
    free(b);
    return NULL;
}

static int cmp_d(const void *x, const void *y)
{
    double a = *(const double *) x, b = *(const double *) y;
    return a < b ? -1 : a > b;
}

static double median_of(double *v, int n)
{
    qsort(v, (size_t) n, sizeof(double), cmp_d);
    return v[n / 2];
}

/* pair_out (K_PAIR only, may be NULL otherwise): [0] triad best, [1] triad
 * median, [2] median over passes of reduce time / triad time */
static int hb(int kind, long count, int dt, int op, int nthreads, const int *cpus, double seconds,
              double *best_s, double *median_s, int *passes, double *span_s, double *pair_out)
{
    if (nthreads < 1 || nthreads > 1024 || count < 1)
        return 1;
    struct hb_shared sh;
    memset(&sh, 0, sizeof sh);
    sh.kind = kind;
    sh.nthreads = nthreads;
    sh.dt = dt;
    sh.op = op;
    sh.count = count;
    sh.seconds = seconds;
    sh.max_passes = 100000;
    sh.times = calloc((size_t) sh.max_passes, sizeof(double));
    sh.times2 = kind == K_PAIR ? calloc((size_t) sh.max_passes, sizeof(double)) : NULL;
    pthread_barrier_init(&sh.bar, NULL, (unsigned) nthreads);
    pthread_t *th = calloc((size_t) nthreads, sizeof(pthread_t));
    struct hb_thread *ts = calloc((size_t) nthreads, sizeof(struct hb_thread));
    for (int i = 0; i < nthreads; ++i) {
        ts[i] = (struct hb_thread) {&sh, i, cpus ? cpus[i] : -1};
        pthread_create(&th[i], NULL, hb_run, &ts[i]);
    }
    for (int i = 0; i < nthreads; ++i)
        pthread_join(th[i], NULL);
    pthread_barrier_destroy(&sh.bar);
    int np = sh.passes < sh.max_passes ? sh.passes : sh.max_passes;
    if (np > 0 && sh.times2 && pair_out) {
        double *ratio = calloc((size_t) np, sizeof(double));
        for (int i = 0; i < np; ++i)
            ratio[i] = sh.times2[i] > 0 ? sh.times[i] / sh.times2[i] : 0;
        pair_out[2] = median_of(ratio, np);
        free(ratio);
        pair_out[1] = median_of(sh.times2, np);
        pair_out[0] = sh.times2[0];
    }
    if (np > 0) {
        qsort(sh.times, (size_t) np, sizeof(double), cmp_d);
        *best_s = sh.times[0];
        *median_s = sh.times[np / 2];
    }
    free(sh.times2);
    *passes = np;
    *span_s = sh.t_last - sh.t_first;
    free(sh.times);
    free(th);
    free(ts);
    return sh.rc;
}

/* MPI_Reduce_local(dt, op) over `count` elements split across pinned threads;
 * *span_s = wall time from the first pass's start to the last pass's end
 * (passes / span is the sustained rate, including any cgroup throttling) */
int oracle_bench_reduce(long count, int dt, int op, int nthreads, const int *cpus, double seconds,
                        double *best_s, double *median_s, int *passes, double *span_s)
{
    return hb(K_REDUCE, count, dt, op, nthreads, cpus, seconds, best_s, median_s, passes, span_s,
              NULL);
}

/* in-place triad a += 0.5 b on `count` fp32 elements (12 bytes each moved) */
int oracle_bench_triad(long count, int nthreads, const int *cpus, double seconds, double *best_s,
                       double *median_s, int *passes, double *span_s)
{
    return hb(K_TRIAD, count, 0, 0, nthreads, cpus, seconds, best_s, median_s, passes, span_s,
              NULL);
}

/* MPI_Reduce_local(dt, op) and the host triad in the same passes: each pass
 * runs the reduce on every thread, a barrier, then the triad on the same
 * slices (a triad timed in its own leg ran in other
 * cgroup quota windows and on other pages than the reduce it was read
 * against).  *best_s / *median_s are the reduce's; pair_out[0..2] = triad
 * best, triad median, median over passes of reduce / triad time */
int oracle_bench_pair(long count, int dt, int op, int nthreads, const int *cpus, double seconds,
                      double *best_s, double *median_s, int *passes, double *span_s,
                      double *pair_out)
{
    return hb(K_PAIR, count, dt, op, nthreads, cpus, seconds, best_s, median_s, passes, span_s,
              pair_out);
}

/* ---------------------------------------------------------------------------
 * One rank's host work in MPICH's recursive-halving reduce-scatter-block
 * (src/mpi/coll/reduce_scatter_block/reduce_scatter_block_intra_recursive_
 * halving.c), the CPU baseline of bench.py's N > 1 line.
 * The reference keeps the whole vector in host temporaries
 * (MPIR_CHKLMEM_MALLOC tmp_recvbuf / tmp_results, :80-88), copies the send
 * buffer into tmp_results (:91-96), then per step combines what arrived in
 * tmp_recvbuf into tmp_results with MPIR_Reduce_local (:219-221) -- the
 * odd ranks of a non-power-of-two world first fold their even neighbour's
 * whole vector (:118-131) -- and finally copies its block to recvbuf
 * (:232-235).  This times exactly that local work on one pinned core (the
 * reference runs one thread per rank), with the received bytes already in
 * tmp_recvbuf: the exchange itself is not the CPU's work to time.  The index
 * arithmetic (newcnts / newdisps / send_idx / recv_idx / last_idx) is the
 * reference's, so the step sizes and offsets are the ones its combines use.
 * --------------------------------------------------------------------------- */
struct rsb_job {
    long recvcount;
    int P, rank, cpu, reps, dt, op;
    double copy_in, combine, copy_out, total;   /* medians, s */
    long combined;                              /* elements combined per call */
    int rc;
};

static void *rsb_run(void *p)
{
    struct rsb_job *j = p;
    if (j->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(j->cpu, &set);
        (void) pthread_setaffinity_np(pthread_self(), sizeof set, &set);
    }
    const long ext = oracle_extent(j->dt);
    const int P = j->P, rank = j->rank;
    const long rc = j->recvcount, total = (long) P * rc;
    const size_t bytes = (size_t) total * (size_t) ext;
    char *send = NULL, *trecv = NULL, *tres = NULL, *recv = NULL;
    if (posix_memalign((void **) &send, 1 << 21, bytes) ||
        posix_memalign((void **) &trecv, 1 << 21, bytes) ||
        posix_memalign((void **) &tres, 1 << 21, bytes) ||
        posix_memalign((void **) &recv, 1 << 21, (size_t) rc * (size_t) ext)) {
        j->rc = 1;
        free(send); free(trecv); free(tres); free(recv);
        return NULL;
    }
    (void) madvise(send, bytes, MADV_HUGEPAGE);
    (void) madvise(trecv, bytes, MADV_HUGEPAGE);
    (void) madvise(tres, bytes, MADV_HUGEPAGE);
    /* first touch on the pinned core: values in [-0.5, 0.5) for fp32 (the
     * bench's fp32 SUM), bytes for anything else */
    unsigned x = 0x5EED0C00u + (unsigned) rank;
    for (size_t i = 0; i + 4 <= bytes; i += 4) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        const float f = (float) (x & 0xffff) * (1.0f / 65536.0f) - 0.5f;
        const float g = (float) ((x >> 16) & 0xffff) * (1.0f / 65536.0f) - 0.5f;
        memcpy(send + i, &f, 4);
        memcpy(trecv + i, &g, 4);
        memcpy(tres + i, &f, 4);
    }
    memset(recv, 0, (size_t) rc * (size_t) ext);

    int pof2 = 1;
    while (pof2 * 2 <= P)
        pof2 *= 2;
    const int rem = P - pof2;
    int newrank;
    if (rank < 2 * rem)
        newrank = rank % 2 == 0 ? -1 : rank / 2;
    else
        newrank = rank - rem;
    long newcnts[64], newdisps[64];
    for (int i = 0; i < pof2; ++i) {
        const int old_i = i < rem ? i * 2 + 1 : i + rem;
        newcnts[i] = old_i < 2 * rem ? 2 * rc : rc;
    }
    newdisps[0] = 0;
    for (int i = 1; i < pof2; ++i)
        newdisps[i] = newdisps[i - 1] + newcnts[i - 1];

    const int reps = j->reps < 1 ? 1 : (j->reps > 64 ? 64 : j->reps);
    double tc_in[64], tc[64], tc_out[64], tt[64];
    long combined = 0;
    for (int r = 0; r < reps && !j->rc; ++r) {
        combined = 0;
        const double t0 = now_s();
        memcpy(tres, send, bytes);                              /* :91-96 */
        const double t1 = now_s();
        if (rank < 2 * rem && rank % 2 == 1) {                  /* :118-131 */
            if (oracle_reduce_local(trecv, tres, total, j->dt, j->op))
                j->rc = 2;
            combined += total;
        }
        if (newrank != -1) {
            int mask = pof2 >> 1, send_idx = 0, recv_idx = 0, last_idx = pof2;
            while (mask > 0) {                                  /* :164-229 */
                const int newdst = newrank ^ mask;
                long recv_cnt = 0;
                if (newrank < newdst) {
                    send_idx = recv_idx + mask;
                    for (int i = recv_idx; i < send_idx; ++i)
                        recv_cnt += newcnts[i];
                } else {
                    recv_idx = send_idx + mask;
                    for (int i = recv_idx; i < last_idx; ++i)
                        recv_cnt += newcnts[i];
                }
                if (recv_cnt) {
                    const size_t off = (size_t) newdisps[recv_idx] * (size_t) ext;
                    if (oracle_reduce_local(trecv + off, tres + off, recv_cnt, j->dt, j->op))
                        j->rc = 2;
                    combined += recv_cnt;
                }
                send_idx = recv_idx;
                last_idx = recv_idx + mask;
                mask >>= 1;
            }
        }
        const double t2 = now_s();
        memcpy(recv, tres + (size_t) rank * (size_t) rc * (size_t) ext,
               (size_t) rc * (size_t) ext);                     /* :232-235 */
        const double t3 = now_s();
        tc_in[r] = t1 - t0;
        tc[r] = t2 - t1;
        tc_out[r] = t3 - t2;
        tt[r] = t3 - t0;
    }
    if (!j->rc) {
        j->copy_in = median_of(tc_in, reps);
        j->combine = median_of(tc, reps);
        j->copy_out = median_of(tc_out, reps);
        j->total = median_of(tt, reps);
        j->combined = combined;
    }
    free(send);
    free(trecv);
    free(tres);
    free(recv);
    return NULL;
}

/* out[0..3] = median seconds of the local copy in, the combines, the copy
 * out and the whole call; out[4] = elements combined per call */
int oracle_bench_rsb_rank(long recvcount, int P, int rank, int cpu, int reps, int dt, int op,
                          double *out)
{
    if (P < 1 || P > 64 || rank < 0 || rank >= P || recvcount < 1)
        return 1;
    struct rsb_job j;
    memset(&j, 0, sizeof j);
    j.recvcount = recvcount;
    j.P = P;
    j.rank = rank;
    j.cpu = cpu;
    j.reps = reps;
    j.dt = dt;
    j.op = op;
    pthread_t th;
    if (pthread_create(&th, NULL, rsb_run, &j))
        return 3;
    pthread_join(th, NULL);
    if (j.rc)
        return j.rc;
    out[0] = j.copy_in;
    out[1] = j.combine;
    out[2] = j.copy_out;
    out[3] = j.total;
    out[4] = (double) j.combined;
    return 0;
}
