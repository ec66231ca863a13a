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

enum { K_REDUCE = 0, K_TRIAD = 1 };

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
            if (sh->kind == K_REDUCE) {
                if (oracle_reduce_local(b, a, n, sh->dt, sh->op))
                    sh->rc = 2;
            } else {
                triad_inplace((float *) a, (const float *) b, n);
            }
        }
        pthread_barrier_wait(&sh->bar);
        if (t->tid == 0) {
            const double t1 = now_s();
            if (pass == 0)
                sh->t_first = t0;
            sh->t_last = t1;
            if (pass < sh->max_passes)
                sh->times[pass] = t1 - t0;
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

static int hb(int kind, long count, int dt, int op, int nthreads, const int *cpus, double seconds,
              double *best_s, double *median_s, int *passes, double *span_s)
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
    if (np > 0) {
        qsort(sh.times, (size_t) np, sizeof(double), cmp_d);
        *best_s = sh.times[0];
        *median_s = sh.times[np / 2];
    }
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
    return hb(K_REDUCE, count, dt, op, nthreads, cpus, seconds, best_s, median_s, passes, span_s);
}

/* in-place triad a += 0.5 b on `count` fp32 elements (12 bytes each moved) */
int oracle_bench_triad(long count, int nthreads, const int *cpus, double seconds, double *best_s,
                       double *median_s, int *passes, double *span_s)
{
    return hb(K_TRIAD, count, 0, 0, nthreads, cpus, seconds, best_s, median_s, passes, span_s);
}
