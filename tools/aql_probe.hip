// aql_probe.hip -- can a synchronous combine skip the HIP stream machinery?
//
// The sync call today: hipLaunchKernel on a library stream, then
// hipStreamWriteValue32 (a blit kernel) stores a word into pinned host memory
// that the caller spins on (profiles/r03_sync_gap.json: 8.7 us of runtime
// completion after the kernel, 6.9 us return + relaunch).  This probe writes
// the kernel's AQL dispatch packet straight into a private HSA queue of the
// same GPU and spins on the packet's own completion signal (decremented by the
// CP after the kernel's end-of-kernel release), i.e. no second packet.
// The kernel object is the very one HIP loaded: found by its mangled name
// among the process's loaded HSA executables (hsa_ven_amd_loader).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/aql_probe.hip \
//        -o tools/bin/aql_probe -lhsa-runtime64
// Run:   tools/bin/aql_probe [reps]   (one JSON object on stdout)
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                        \
    do {                                                                             \
        auto _e = (x);                                                               \
        if ((int) _e != 0) {                                                         \
            fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int) _e);    \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

// fp32 SUM over 16-byte packets, 256 threads x 4 packets per lane per tile,
// one tile per workgroup; reads no hidden kernel argument (block size is a
// constant, the grid's stride comes in as an argument), so a hand-built AQL
// packet needs only the explicit arguments.
constexpr int NT = 256, U = 4;
__global__ void __launch_bounds__(256) k_sum_q(const v4u *__restrict__ in, v4u *__restrict__ io,
                                                uint64_t npk, uint64_t stride)
{
    if (stride == 0)
        return;
    for (uint64_t i = (uint64_t) blockIdx.x * NT * U + threadIdx.x; i < npk; i += stride) {
        v4u a[U], b[U];
        if (i + (U - 1) * NT < npk) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                a[u] = __builtin_nontemporal_load(io + i + u * NT);
#pragma unroll
            for (int u = 0; u < U; ++u)
                b[u] = __builtin_nontemporal_load(in + i + u * NT);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float4 x = __builtin_bit_cast(float4, a[u]), y = __builtin_bit_cast(float4, b[u]);
                x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
                __builtin_nontemporal_store(__builtin_bit_cast(v4u, x), io + i + u * NT);
            }
        } else {
            for (int u = 0; u < U; ++u) {
                uint64_t k = i + u * NT;
                if (k < npk) {
                    float4 x = __builtin_bit_cast(float4, io[k]), y = __builtin_bit_cast(float4, in[k]);
                    x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
                    io[k] = __builtin_bit_cast(v4u, x);
                }
            }
        }
    }
}

struct Args {
    const v4u *in;
    v4u *io;
    uint64_t npk;
    uint64_t stride;
};

static hsa_agent_t g_gpu, g_cpu;
static hsa_amd_hdp_flush_t g_hdp{};
static int g_bdf = -1;
static hsa_amd_memory_pool_t g_karg_pool;
static bool g_have_pool = false;

static hsa_status_t find_agents(hsa_agent_t a, void *)
{
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU) {
        uint32_t bdf = 0;
        hsa_agent_get_info(a, (hsa_agent_info_t) HSA_AMD_AGENT_INFO_BDFID, &bdf);
        if ((int) bdf == g_bdf)
            g_gpu = a;
    } else if (t == HSA_DEVICE_TYPE_CPU && g_cpu.handle == 0) {
        g_cpu = a;
    }
    return HSA_STATUS_SUCCESS;
}

static hsa_status_t find_pool(hsa_amd_memory_pool_t p, void *)
{
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL)
        return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !g_have_pool) {
        g_karg_pool = p;
        g_have_pool = true;
    }
    return HSA_STATUS_SUCCESS;
}

struct Sym {
    std::string want;
    uint64_t kobj = 0;
    uint32_t karg = 0, grp = 0, priv = 0;
    int seen = 0;
};

static hsa_status_t sym_cb(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t s, void *d)
{
    Sym *S = (Sym *) d;
    hsa_symbol_kind_t k;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &k);
    if (k != HSA_SYMBOL_KIND_KERNEL)
        return HSA_STATUS_SUCCESS;
    uint32_t len = 0;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
    std::string name(len, '\0');
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME, &name[0]);
    ++S->seen;
    if (name == S->want || name == S->want + ".kd") {
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &S->kobj);
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &S->karg);
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &S->grp);
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &S->priv);
    } else if (getenv("AQL_PROBE_NAMES")) {
        fprintf(stderr, "symbol %s\n", name.c_str());
    }
    return HSA_STATUS_SUCCESS;
}

static hsa_ven_amd_loader_1_03_pfn_t g_ldr;
static hsa_status_t exe_cb(hsa_executable_t e, void *d)
{
    hsa_executable_iterate_agent_symbols(e, g_gpu, sym_cb, d);
    return HSA_STATUS_SUCCESS;
}

struct Aql {
    hsa_queue_t *q = nullptr;
    hsa_signal_t sig{};
    Sym sym;
};

struct Variant {
    const char *name;
    Args *karg;         // host kernarg pool or fine-grained VRAM
    bool dev_karg;
    int acq, rel;       // fence scopes
    std::vector<double> big, one;
};

static void dispatch(Aql &A, Variant &v, const Args &a, uint32_t grid)
{
    *v.karg = a;
    if (v.dev_karg) {   // BAR writes into VRAM: flush the host data path, then read back
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        if (g_hdp.HDP_MEM_FLUSH_CNTL) {
            *(volatile uint32_t *) g_hdp.HDP_MEM_FLUSH_CNTL = 1u;
            (void) *(volatile uint32_t *) g_hdp.HDP_MEM_FLUSH_CNTL;
        }
        (void) *(volatile uint64_t *) &v.karg->stride;
    }
    hsa_signal_store_relaxed(A.sig, 1);
    uint64_t idx = hsa_queue_add_write_index_relaxed(A.q, 1);
    while (idx - hsa_queue_load_read_index_scacquire(A.q) >= A.q->size) {
    }
    hsa_kernel_dispatch_packet_t *pk =
        (hsa_kernel_dispatch_packet_t *) A.q->base_address + (idx & (A.q->size - 1));
    pk->workgroup_size_x = NT;
    pk->workgroup_size_y = 1;
    pk->workgroup_size_z = 1;
    pk->reserved0 = 0;
    pk->grid_size_x = grid * NT;
    pk->grid_size_y = 1;
    pk->grid_size_z = 1;
    pk->private_segment_size = A.sym.priv;
    pk->group_segment_size = A.sym.grp;
    pk->kernel_object = A.sym.kobj;
    pk->kernarg_address = v.karg;
    pk->reserved2 = 0;
    pk->completion_signal = A.sig;
    uint16_t hdr = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                   (1 << HSA_PACKET_HEADER_BARRIER) |
                   (v.acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                   (v.rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    __atomic_store_n((uint32_t *) pk, (uint32_t) hdr | ((uint32_t) setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(A.q->doorbell_signal, idx);
}

static hsa_amd_memory_pool_t g_vram_fg;
static bool g_have_vram_fg = false;
static hsa_status_t find_vram_pool(hsa_amd_memory_pool_t p, void *)
{
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL)
        return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    {
        hsa_amd_memory_pool_access_t acc = HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED;
        hsa_amd_agent_memory_pool_get_info(g_cpu, p, HSA_AMD_AGENT_MEMORY_POOL_INFO_ACCESS, &acc);
        fprintf(stderr, "VRAM pool flags %#x: CPU access %d\n", flags, (int) acc);
        if (acc != HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED && !g_have_vram_fg) {
            g_vram_fg = p;
            g_have_vram_fg = true;
        }
    }
    return HSA_STATUS_SUCCESS;
}

static bool wait_sig(Aql &A)
{
    auto t0 = std::chrono::steady_clock::now();
    while (hsa_signal_load_scacquire(A.sig) != 0) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5))
            return false;
    }
    return true;
}

static double now_us()
{
    return std::chrono::duration<double, std::micro>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv)
{
    int reps = argc > 1 ? atoi(argv[1]) : 50;
    CK(hipSetDevice(0));
    int bus = 0, devn = 0, dom = 0;
    CK(hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, 0));
    CK(hipDeviceGetAttribute(&devn, hipDeviceAttributePciDeviceId, 0));
    CK(hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, 0));
    g_bdf = (bus << 8) | (devn << 3);   // function 0

    const size_t bytes = (size_t) 1 << 30;
    const uint64_t npk = bytes / 16;
    v4u *in = nullptr, *io = nullptr;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&io, bytes));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // in = 1.0f, io = 0.0f
    {
        std::vector<float> one(1 << 20, 1.0f);
        for (size_t off = 0; off < bytes; off += one.size() * 4)
            CK(hipMemcpy((char *) in + off, one.data(), one.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemset(io, 0, bytes));
        CK(hipDeviceSynchronize());
    }
    const uint32_t tile = NT * U;
    const uint32_t grid_big = (uint32_t) ((npk + tile - 1) / tile);
    // one HIP launch loads the code object
    hipLaunchKernelGGL(k_sum_q, dim3(1), dim3(NT), 0, s, in, io, (uint64_t) 0, (uint64_t) tile);
    CK(hipStreamSynchronize(s));
    const char *kname = hipKernelNameRefByPtr((const void *) k_sum_q, s);
    if (!kname) {
        fprintf(stderr, "no kernel name\n");
        return 2;
    }

    CK(hsa_init());
    CK(hsa_iterate_agents(find_agents, nullptr));
    if (g_gpu.handle == 0) {
        fprintf(stderr, "no HSA agent with BDF %x\n", g_bdf);
        return 2;
    }
    CK(hsa_amd_agent_iterate_memory_pools(g_cpu, find_pool, nullptr));
    if (!g_have_pool) {
        fprintf(stderr, "no kernarg pool\n");
        return 2;
    }
    CK(hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(g_ldr), &g_ldr));
    Aql A;
    A.sym.want = kname;
    CK(g_ldr.hsa_ven_amd_loader_iterate_executables(exe_cb, &A.sym));
    if (!A.sym.kobj) {
        fprintf(stderr, "kernel %s not found among %d kernel symbols\n", kname, A.sym.seen);
        return 2;
    }
    fprintf(stderr, "kernel %s: kobj %#lx karg %u grp %u priv %u\n", kname,
            (unsigned long) A.sym.kobj, A.sym.karg, A.sym.grp, A.sym.priv);
    if (A.sym.karg < sizeof(Args)) {
        fprintf(stderr, "kernarg segment %u smaller than the explicit arguments\n", A.sym.karg);
        return 2;
    }
    CK(hsa_queue_create(g_gpu, 256, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX,
                        UINT32_MAX, &A.q));
    CK(hsa_amd_signal_create(1, 0, nullptr, 0, &A.sig));
    const size_t kbytes = std::max<uint32_t>(A.sym.karg, 256);
    void *kp = nullptr;
    CK(hsa_amd_memory_pool_allocate(g_karg_pool, kbytes, 0, &kp));
    CK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, kp));
    memset(kp, 0, kbytes);
    void *kd = nullptr;
    CK(hsa_amd_agent_iterate_memory_pools(g_gpu, find_vram_pool, nullptr));
    if (hsa_agent_get_info(g_gpu, (hsa_agent_info_t) HSA_AMD_AGENT_INFO_HDP_FLUSH, &g_hdp) != HSA_STATUS_SUCCESS)
        memset(&g_hdp, 0, sizeof g_hdp);
    fprintf(stderr, "HDP flush register %p\n", (void *) g_hdp.HDP_MEM_FLUSH_CNTL);
    if (g_have_vram_fg && hsa_amd_memory_pool_allocate(g_vram_fg, kbytes, 0, &kd) == HSA_STATUS_SUCCESS) {
        if (hsa_amd_agents_allow_access(1, &g_cpu, nullptr, kd) != HSA_STATUS_SUCCESS)
            kd = nullptr;
        else
            memset(kd, 0, kbytes);
    }
    const int SYS = HSA_FENCE_SCOPE_SYSTEM, AG = HSA_FENCE_SCOPE_AGENT;
    std::vector<Variant> V;
    V.push_back({"aql_hostkarg_sys_sys", (Args *) kp, false, SYS, SYS, {}, {}});
    if (kd) {
        V.push_back({"aql_devkarg_sys_sys", (Args *) kd, true, SYS, SYS, {}, {}});
        V.push_back({"aql_devkarg_agent_sys", (Args *) kd, true, AG, SYS, {}, {}});
        V.push_back({"aql_devkarg_agent_agent", (Args *) kd, true, AG, AG, {}, {}});
    }

    // pinned host word for the HIP path (as libmpix_redop does)
    uint32_t *flag = nullptr;
    CK(hipHostMalloc((void **) &flag, 64, hipHostMallocCoherent));
    *flag = 0;
    uint32_t seq = 0;

    // --- correctness of each AQL variant on a small call first
    double p0 = 0, p1 = 0, full = 0;    // expected: packet 0, packet 1, the tail
    for (Variant &v : V) {
        dispatch(A, v, Args{in, io, 1024, (uint64_t) tile}, 1);
        if (!wait_sig(A)) {
            fprintf(stderr, "AQL dispatch (%s) did not complete in 5 s\n", v.name);
            return 3;
        }
        p0 += 1;
        p1 += 1;
        float h[8];
        CK(hipMemcpy(h, io, 32, hipMemcpyDeviceToHost));
        if (h[0] != (float) p0 || h[4] != (float) p1) {
            fprintf(stderr, "AQL small call (%s) wrong: %g want %g\n", v.name, h[0], p0);
            return 4;
        }
    }

    auto hip_call = [&](uint64_t n, uint32_t grid) {
        hipLaunchKernelGGL(k_sum_q, dim3(grid), dim3(NT), 0, s, in, io, n, (uint64_t) grid * tile);
        ++seq;
        CK(hipStreamWriteValue32(s, flag, seq, 0));
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
        }
    };
    auto aql_call = [&](Variant &v, uint64_t n, uint32_t grid) {
        dispatch(A, v, Args{in, io, n, (uint64_t) grid * tile}, grid);
        if (!wait_sig(A)) {
            fprintf(stderr, "AQL dispatch (%s) did not complete in 5 s\n", v.name);
            exit(3);
        }
    };

    std::vector<double> hip_big, hip_one;
    for (int round = 0; round < 3; ++round) {
        for (int r = 0; r < reps; ++r) {
            double t0 = now_us();
            hip_call(npk, grid_big);
            hip_big.push_back(now_us() - t0);
        }
        full += reps; p0 += reps; p1 += reps;
        for (Variant &v : V) {
            for (int r = 0; r < reps; ++r) {
                double t0 = now_us();
                aql_call(v, npk, grid_big);
                v.big.push_back(now_us() - t0);
            }
            full += reps; p0 += reps; p1 += reps;
        }
        for (int r = 0; r < 20 * reps; ++r) {
            double t0 = now_us();
            hip_call(1, 1);
            hip_one.push_back(now_us() - t0);
        }
        p0 += 20 * reps;
        for (Variant &v : V) {
            for (int r = 0; r < 20 * reps; ++r) {
                double t0 = now_us();
                aql_call(v, 1, 1);
                v.one.push_back(now_us() - t0);
            }
            p0 += 20 * reps;
        }
    }
    std::vector<float> chk(1 << 20);
    CK(hipMemcpy(chk.data(), (char *) io + bytes - chk.size() * 4, chk.size() * 4,
                 hipMemcpyDeviceToHost));
    bool ok = true;
    for (float v : chk)
        ok = ok && v == (float) full;
    float h8[8];
    CK(hipMemcpy(h8, io, 32, hipMemcpyDeviceToHost));
    for (int k = 0; k < 4; ++k)
        ok = ok && h8[k] == (float) p0 && h8[4 + k] == (float) p1;
    if (!ok)
        fprintf(stderr, "check: tail %g (want %g), p0 %g (want %g), p1 %g (want %g)\n", chk[0], full,
                h8[0], p0, h8[4], p1);

    auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    auto mn = [](std::vector<double> v) { return *std::min_element(v.begin(), v.end()); };
    printf("{\"probe\": \"aql_probe\", \"reps\": %d, \"bytes\": %zu, \"grid\": %u, \"kernarg\": %u, "
           "\"hip_1GiB_us\": {\"median\": %.1f, \"min\": %.1f}, "
           "\"hip_1elem_us\": {\"median\": %.2f, \"min\": %.2f}",
           reps, bytes, grid_big, A.sym.karg, med(hip_big), mn(hip_big), med(hip_one), mn(hip_one));
    for (Variant &v : V)
        printf(", \"%s\": {\"1GiB_us_median\": %.1f, \"1GiB_us_min\": %.1f, \"1elem_us_median\": %.2f, "
               "\"1elem_us_min\": %.2f}",
               v.name, med(v.big), mn(v.big), med(v.one), mn(v.one));
    printf(", \"checked\": %s}\n", ok ? "true" : "false");
    hsa_signal_destroy(A.sig);
    hsa_queue_destroy(A.q);
    hsa_amd_memory_pool_free(kp);
    if (kd)
        hsa_amd_memory_pool_free(kd);
    return ok ? 0 : 5;
}
