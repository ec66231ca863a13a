// persist_zc_probe.hip -- pageable operands through ONE persistent zero-copy
// kernel instead of one zero-copy kernel per chunk.
//
// The library's wave form (redop_capi.cpp `waved`) pays ~0.12-0.16 ms per
// chunk kernel (its ramp and, above all, the drain of its posted PCIe writes at
// the kernel's end: profiles/r03_zero_copy_split.json), so it needs 64 MiB
// chunks, whose pipeline fill and drain cost again.  Here one kernel runs for
// the whole call: host threads copy chunk k into a page-locked ring slot and
// raise ready[k % 3]; workgroups take tiles by ticket (so no workgroup ever
// waits on one that is not resident), wait for their chunk's flag, combine over
// PCIe, fence at system scope and count the chunk's tiles; the last tile of a
// chunk raises done[k % 3], and the host threads copy the result out.
// Only one workgroup per chunk (the holder of its first tile) polls the host
// flag; the others poll a device-memory copy of it.  Every wait has a
// wall-clock limit (s_memrealtime, 100 MHz): an error flag ends all workgroups.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/persist_zc_probe.hip \
//        -o tools/bin/persist_zc_probe -Impich_amd/../include -Lmpich_amd -lmpix_redop \
//        -Wl,-rpath,$PWD/mpich_amd -lpthread
// Run:   tools/bin/persist_zc_probe [MiB per operand] [grid] (one JSON line on stdout)
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "mpix_redop.h"

#define CK(x)                                                                        \
    do {                                                                             \
        auto _e = (x);                                                               \
        if ((int) _e != 0) {                                                         \
            fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int) _e);    \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int NT = 256, U = 4;
constexpr uint64_t kTilePk = (uint64_t) NT * U;        // 16-byte packets per tile (16 KiB)
constexpr uint64_t kTimeout = 10ull * 100000000ull;    // 10 s of the 100 MHz wall clock

struct ZcArgs {
    char *ring;                 // device mapping of the page-locked ring: 3 x (in | inout)
    uint64_t half;              // bytes of each half
    const uint64_t *cnt;        // device: float count of chunk k
    const uint64_t *tstart;     // device: first ticket of chunk k (nchunks + 1 entries)
    uint64_t total;             // tickets
    unsigned *ticket;           // device counters, zero at launch
    unsigned *done_cnt;         // [3]
    uint64_t *dev_ready;        // [3]
    unsigned *error;
    uint64_t *host_ready;       // page-locked [3]: k + 1 once chunk k is in slot k % 3
    uint64_t *host_done;        // page-locked [3]: k + 1 once chunk k's result is there
};

// FENCE: system-scope release per tile before it is counted (what the host's
// copy-out needs); WAIT: honour the ready flags (false: raw rate over the ring)
template <bool FENCE, bool WAIT>
__global__ void __launch_bounds__(256) k_zc_persist(ZcArgs a)
{
    __shared__ uint64_t s_t;
    __shared__ int s_abort;
    uint32_t k = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            s_t = atomicAdd(a.ticket, 1u);
            s_abort = 0;
        }
        __syncthreads();
        const uint64_t t = s_t;
        if (t >= a.total)
            break;
        while (t >= a.tstart[k + 1])
            ++k;
        const uint64_t j = t - a.tstart[k];
        const int slot = (int) (k % 3);
        if (WAIT && threadIdx.x == 0) {
            const uint64_t want = (uint64_t) k + 1;
            const uint64_t t0 = wall_clock64();
            if (j == 0) {       // the chunk's sentinel polls the host flag
                while (__hip_atomic_load(&a.host_ready[slot], __ATOMIC_ACQUIRE,
                                         __HIP_MEMORY_SCOPE_SYSTEM) != want) {
                    if (__hip_atomic_load(a.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                        wall_clock64() - t0 > kTimeout) {
                        atomicOr(a.error, 1u);
                        s_abort = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(8);
                }
                if (!s_abort)
                    __hip_atomic_store(&a.dev_ready[slot], want, __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_AGENT);
            } else {
                while (__hip_atomic_load(&a.dev_ready[slot], __ATOMIC_ACQUIRE,
                                         __HIP_MEMORY_SCOPE_AGENT) != want) {
                    if (__hip_atomic_load(a.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                        wall_clock64() - t0 > kTimeout) {
                        atomicOr(a.error, 1u);
                        s_abort = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(8);
                }
            }
        }
        __syncthreads();
        if (s_abort)
            break;
        const uint64_t npk = a.cnt[k] / 4;
        const v4u *vin = reinterpret_cast<const v4u *>(a.ring + (size_t) slot * 2 * a.half);
        v4u *vio = reinterpret_cast<v4u *>(a.ring + (size_t) slot * 2 * a.half + a.half);
        const uint64_t base = j * kTilePk + threadIdx.x;
        v4u x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (base + u * NT < npk)
                x[u] = vio[base + u * NT];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (base + u * NT < npk)
                y[u] = vin[base + u * NT];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (base + u * NT < npk) {
                float4 p = __builtin_bit_cast(float4, x[u]), q = __builtin_bit_cast(float4, y[u]);
                p.x += q.x; p.y += q.y; p.z += q.z; p.w += q.w;
                vio[base + u * NT] = __builtin_bit_cast(v4u, p);
            }
        if (FENCE)
            __threadfence_system();     // this lane's stores visible to the host
        else
            __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned tiles = (unsigned) (a.tstart[k + 1] - a.tstart[k]);
            if (atomicAdd(&a.done_cnt[slot], 1u) + 1 == tiles) {
                a.done_cnt[slot] = 0;
                __hip_atomic_store(&a.host_done[slot], (uint64_t) k + 1, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        __syncthreads();                // s_t is rewritten next round
    }
}

__attribute__((target("avx2"))) static void copy_nt(char *dst, const char *src, size_t n)
{
    size_t head = (32 - ((uintptr_t) dst & 31)) & 31;
    head = std::min(head, n);
    memcpy(dst, src, head);
    dst += head, src += head, n -= head;
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        __m256i a = _mm256_loadu_si256((const __m256i *) (src + i));
        __m256i b = _mm256_loadu_si256((const __m256i *) (src + i + 32));
        __m256i c = _mm256_loadu_si256((const __m256i *) (src + i + 64));
        __m256i d = _mm256_loadu_si256((const __m256i *) (src + i + 96));
        _mm256_stream_si256((__m256i *) (dst + i), a);
        _mm256_stream_si256((__m256i *) (dst + i + 32), b);
        _mm256_stream_si256((__m256i *) (dst + i + 64), c);
        _mm256_stream_si256((__m256i *) (dst + i + 96), d);
    }
    _mm_sfence();
    memcpy(dst + i, src + i, n - i);
}

struct Barrier {
    std::atomic<int> left, gen{0};
    int n;
    explicit Barrier(int n_) : left(n_), n(n_) {}
    void wait()
    {
        int g = gen.load(std::memory_order_acquire);
        if (left.fetch_sub(1, std::memory_order_acq_rel) == 1) {
            left.store(n, std::memory_order_relaxed);
            gen.fetch_add(1, std::memory_order_release);
            return;
        }
        while (gen.load(std::memory_order_acquire) == g)
            std::this_thread::yield();
    }
};

struct Persist {
    size_t half = 0;
    char *ring = nullptr, *ring_dev = nullptr;
    uint64_t *hflags = nullptr;     // host_ready[3], host_done[3]
    char *dmem = nullptr;           // counters + tables
    hipStream_t s{};
    int grid = 512;
};

static double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// inout[0:count] += in[0:count] (fp32), both pageable; returns 0 or an error
static bool g_fence = true;

static int persist_call(Persist &P, const float *in, float *io, uint64_t count, size_t chunk_bytes,
                        int W)
{
    const uint64_t C = chunk_bytes / 4;
    std::vector<uint64_t> cnt, ts{0};
    for (uint64_t off = 0; off < count; off += C) {
        cnt.push_back(std::min(C, count - off));
        ts.push_back(ts.back() + (cnt.back() / 4 + kTilePk - 1) / kTilePk);
    }
    const int64_t n = (int64_t) cnt.size();
    if (count % 4 || chunk_bytes > P.half || n > 4096)
        return 9;
    uint64_t *dcnt = (uint64_t *) (P.dmem + 4096), *dts = dcnt + 4096;
    unsigned *ctr = (unsigned *) P.dmem;        // ticket, done_cnt[3], error
    uint64_t *dready = (uint64_t *) (P.dmem + 64);
    CK(hipMemcpyAsync(dcnt, cnt.data(), n * 8, hipMemcpyHostToDevice, P.s));
    CK(hipMemcpyAsync(dts, ts.data(), (n + 1) * 8, hipMemcpyHostToDevice, P.s));
    CK(hipMemsetAsync(P.dmem, 0, 256, P.s));
    for (int i = 0; i < 6; ++i)
        __atomic_store_n(&P.hflags[i], 0, __ATOMIC_RELEASE);
    ZcArgs a{P.ring_dev, P.half, dcnt, dts, ts.back(), ctr, ctr + 1, dready, ctr + 4,
             P.hflags, P.hflags + 3};
    if (g_fence)
        hipLaunchKernelGGL((k_zc_persist<true, true>), dim3(P.grid), dim3(NT), 0, P.s, a);
    else
        hipLaunchKernelGGL((k_zc_persist<false, true>), dim3(P.grid), dim3(NT), 0, P.s, a);
    CK(hipGetLastError());
    Barrier bar(W);
    std::atomic<int> err{0};
    auto slice = [&](int w, size_t bytes, size_t *lo, size_t *len) {
        size_t per = ((bytes + W - 1) / W + 4095) & ~(size_t) 4095;
        *lo = std::min(bytes, per * w);
        *len = std::min(bytes - *lo, per);
    };
    auto work = [&](int w) {
        for (int64_t st = 0; st <= n + 1; ++st) {
            if (st < n) {
                const uint64_t off = (uint64_t) st * C;
                char *h = P.ring + (size_t) (st % 3) * 2 * P.half;
                size_t lo, len;
                slice(w, cnt[st] * 4, &lo, &len);
                if (len) {
                    copy_nt(h + lo, (const char *) (in + off) + lo, len);
                    copy_nt(h + P.half + lo, (const char *) (io + off) + lo, len);
                }
            }
            bar.wait();
            if (w == 0 && st < n)
                __atomic_store_n(&P.hflags[st % 3], (uint64_t) st + 1, __ATOMIC_RELEASE);
            if (st >= 2 && !err.load()) {
                const int64_t k = st - 2;
                const double t0 = now_ms();
                while (__atomic_load_n(&P.hflags[3 + k % 3], __ATOMIC_ACQUIRE) != (uint64_t) k + 1)
                    if (now_ms() - t0 > 5000) {
                        err = 1;
                        break;
                    }
                if (!err.load()) {
                    size_t lo, len;
                    slice(w, cnt[k] * 4, &lo, &len);
                    if (len)
                        memcpy((char *) (io + (uint64_t) k * C) + lo,
                               P.ring + (size_t) (k % 3) * 2 * P.half + P.half + lo, len);
                }
            }
            bar.wait();
        }
    };
    std::vector<std::thread> pool;
    for (int w = 1; w < W; ++w)
        pool.emplace_back(work, w);
    work(0);
    for (auto &t : pool)
        t.join();
    if (err.load()) {       // the kernel ends by its own clock; release it early
        unsigned one = 1;
        (void) hipMemcpy(ctr + 4, &one, 4, hipMemcpyHostToDevice);
    }
    CK(hipStreamSynchronize(P.s));
    unsigned kerr = 0;
    CK(hipMemcpy(&kerr, ctr + 4, 4, hipMemcpyDeviceToHost));
    return err.load() ? 3 : (kerr ? 4 : 0);
}

int main(int argc, char **argv)
{
    const size_t mib = argc > 1 ? (size_t) atoll(argv[1]) : 1024;
    const uint64_t count = mib * (1 << 20) / 4;
    CK(hipSetDevice(0));
    CK(MPIX_Redop_init());
    Persist P;
    P.half = (size_t) 64 << 20;
    if (argc > 2)
        P.grid = atoi(argv[2]);
    void *h = nullptr, *hd = nullptr;
    CK(hipHostMalloc(&h, 3 * 2 * P.half, hipHostMallocDefault));
    CK(hipHostGetDevicePointer(&hd, h, 0));
    P.ring = (char *) h;
    P.ring_dev = (char *) hd;
    CK(hipHostMalloc((void **) &P.hflags, 64, hipHostMallocDefault));
    CK(hipMalloc((void **) &P.dmem, 4096 + 2 * 4096 * 8 + 64));
    CK(hipStreamCreateWithFlags(&P.s, hipStreamNonBlocking));

    float *in = (float *) aligned_alloc(4096, count * 4);
    float *io = (float *) aligned_alloc(4096, count * 4);
    float *ref = (float *) aligned_alloc(4096, count * 4);
    uint64_t x = 0x5EED0007ull;
    for (uint64_t i = 0; i < count; ++i) {
        x ^= x >> 12, x ^= x << 25, x ^= x >> 27;
        const uint32_t r = (uint32_t) ((x * 2685821657736338717ull) >> 40);
        in[i] = (float) r / (1u << 24) - 0.5f;
        io[i] = (float) (r & 0xffff) / 65536.0f;
    }
    memcpy(ref, io, count * 4);
    const int W = 8;
    // parity: the library's call (its default pageable form) against the
    // persistent form, same operands, bit for bit
    CK(MPIX_Reduce_local(in, ref, (MPIX_Aint) count, (MPIX_Datatype) 0x4c00040a, MPIX_SUM));
    int rc = persist_call(P, in, io, count, (size_t) 16 << 20, W);
    if (rc) {
        fprintf(stderr, "persistent call failed: %d\n", rc);
        return rc;
    }
    const bool same = memcmp(ref, io, count * 4) == 0;
    if (!same) {
        uint64_t i = 0;
        while (i < count && ((uint32_t *) ref)[i] == ((uint32_t *) io)[i])
            ++i;
        fprintf(stderr, "mismatch at %llu: %g vs %g\n", (unsigned long long) i, ref[i], io[i]);
        return 5;
    }
    const size_t chunks[] = {(size_t) 4 << 20, (size_t) 8 << 20, (size_t) 16 << 20, (size_t) 32 << 20,
                             (size_t) 64 << 20};
    std::vector<double> lib_ms;
    std::vector<std::vector<double>> per(5);
    const int reps = 3;
    for (int round = 0; round < 3; ++round) {
        for (int r = 0; r < reps; ++r) {
            const double t0 = now_ms();
            CK(MPIX_Reduce_local(in, ref, (MPIX_Aint) count, (MPIX_Datatype) 0x4c00040a, MPIX_SUM));
            lib_ms.push_back(now_ms() - t0);
        }
        for (int c = 0; c < 5; ++c)
            for (int r = 0; r < reps; ++r) {
                const double t0 = now_ms();
                rc = persist_call(P, in, io, count, chunks[c], W);
                per[c].push_back(now_ms() - t0);
                if (rc) {
                    fprintf(stderr, "persistent call failed: %d\n", rc);
                    return rc;
                }
            }
    }
    auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    // raw rates: the persistent kernel over the ring with no flags (every
    // chunk k in slot k % 3, 64 MiB chunks), with and without the per-tile
    // fence, against one zero-copy library call on page-locked 1 GiB operands
    auto raw = [&](bool fence) {
        const uint64_t C = P.half / 4;
        std::vector<uint64_t> cnt, ts{0};
        for (uint64_t off = 0; off < count; off += C) {
            cnt.push_back(std::min(C, count - off));
            ts.push_back(ts.back() + (cnt.back() / 4 + kTilePk - 1) / kTilePk);
        }
        uint64_t *dcnt = (uint64_t *) (P.dmem + 4096), *dts = dcnt + 4096;
        unsigned *ctr = (unsigned *) P.dmem;
        CK(hipMemcpy(dcnt, cnt.data(), cnt.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(dts, ts.data(), ts.size() * 8, hipMemcpyHostToDevice));
        ZcArgs a{P.ring_dev, P.half, dcnt, dts, ts.back(), ctr, ctr + 1, (uint64_t *) (P.dmem + 64),
                 ctr + 4, P.hflags, P.hflags + 3};
        std::vector<double> v;
        for (int r = 0; r < 4; ++r) {
            CK(hipMemsetAsync(P.dmem, 0, 256, P.s));
            CK(hipStreamSynchronize(P.s));
            const double t0 = now_ms();
            if (fence)
                hipLaunchKernelGGL((k_zc_persist<true, false>), dim3(P.grid), dim3(NT), 0, P.s, a);
            else
                hipLaunchKernelGGL((k_zc_persist<false, false>), dim3(P.grid), dim3(NT), 0, P.s, a);
            CK(hipStreamSynchronize(P.s));
            if (r)
                v.push_back(now_ms() - t0);
        }
        return med(v);
    };
    const double raw_fence = raw(true), raw_nofence = raw(false);
    float *pin = nullptr, *pio = nullptr;
    CK(hipHostMalloc((void **) &pin, count * 4, hipHostMallocDefault));
    CK(hipHostMalloc((void **) &pio, count * 4, hipHostMallocDefault));
    memcpy(pin, in, count * 4);
    memcpy(pio, io, count * 4);
    std::vector<double> pinned;
    for (int r = 0; r < 4; ++r) {
        const double t0 = now_ms();
        CK(MPIX_Reduce_local(pin, pio, (MPIX_Aint) count, (MPIX_Datatype) 0x4c00040a, MPIX_SUM));
        if (r)
            pinned.push_back(now_ms() - t0);
    }
    // the pipeline without the per-tile fence (parity checked on one call)
    g_fence = false;
    memcpy(ref, io, count * 4);
    CK(MPIX_Reduce_local(in, ref, (MPIX_Aint) count, (MPIX_Datatype) 0x4c00040a, MPIX_SUM));
    rc = persist_call(P, in, io, count, (size_t) 16 << 20, W);
    const bool same_nf = rc == 0 && memcmp(ref, io, count * 4) == 0;
    std::vector<double> nf16, nf64;
    for (int r = 0; r < 3 && rc == 0; ++r) {
        double t0 = now_ms();
        rc = persist_call(P, in, io, count, (size_t) 16 << 20, W);
        nf16.push_back(now_ms() - t0);
        t0 = now_ms();
        rc = rc ? rc : persist_call(P, in, io, count, (size_t) 64 << 20, W);
        nf64.push_back(now_ms() - t0);
    }
    if (rc) {
        fprintf(stderr, "no-fence persistent call failed: %d\n", rc);
        return rc;
    }
    printf("{\"raw_persistent_fence_ms\": %.2f, \"raw_persistent_nofence_ms\": %.2f, "
           "\"pinned_one_call_ms\": %.2f, \"nofence_parity\": %s, \"nofence_16MiB_ms\": %.2f, "
           "\"nofence_64MiB_ms\": %.2f}\n",
           raw_fence, raw_nofence, med(pinned), same_nf ? "true" : "false", med(nf16), med(nf64));
    printf("{\"probe\": \"persist_zc_probe\", \"bytes\": %zu, \"W\": %d, \"grid\": %d, \"parity_vs_library\": %s, "
           "\"library_wave_ms\": %.2f",
           (size_t) count * 4, W, P.grid, same ? "true" : "false", med(lib_ms));
    for (int c = 0; c < 5; ++c)
        printf(", \"persistent_%zuMiB_ms\": %.2f", chunks[c] >> 20, med(per[c]));
    printf("}\n");
    return 0;
}
