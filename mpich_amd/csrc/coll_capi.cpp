// coll_capi.cpp -- libmpix_coll.so: MPICH's reduce-scatter / allreduce
// schedules in C++ host code (include/mpix_coll.h), every combine step a call
// into libmpix_redop.so's HIP kernels, every exchange step one group of
// point-to-point operations on a transport:
//
//   RCCL        ncclGroupStart / ncclSend + ncclRecv / ncclGroupEnd on the
//               collective's stream (one process per MI355X, xGMI between them)
//   local       ranks are threads of one process; a receive is a stream-ordered
//               hipMemcpyAsync from the sender's buffer after the sender's
//               "ready" event, and the sender's stream then waits for the
//               receiver's "done" event before it may touch that buffer again
//   host-local  the same over host memory with memcpy (schedule tests without
//               a GPU; a combine must be installed, there is no CPU compute path)
//   custom      a caller-supplied exchange function
//
// The schedules restate, index for index, the reference algorithms cited in
// include/mpix_coll.h; mpich_amd/coll.py holds the same schedules over
// torch.distributed and the oracle (oracle/redop_oracle.c) simulates them in
// one process -- the tests hold all three to the same bits.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "mpix_coll.h"

namespace {

enum Kind { K_CCL, K_LOCAL_DEV, K_LOCAL_HOST, K_CUSTOM };

// a rank's receive group completion event, shared by the senders that must
// wait for it; the last sender to enqueue its wait destroys it
struct DoneEv {
    hipEvent_t ev = nullptr;
    int refs = 0;
};

struct Slot {
    const void *buf = nullptr;
    size_t bytes = 0;
    hipEvent_t ready = nullptr;     // sender's stream state when the send was posted
    std::shared_ptr<DoneEv> done;   // receiver's copy completion
    bool consumed = false;
};

// shared mailbox of a local communicator: slots keyed (src, dst, seq), seq
// counting the messages of that ordered pair (MPI's non-overtaking order)
struct Local {
    int size = 0;
    bool host = false;
    std::vector<int> devices;
    bool peer_ok = true;    // every rank's device can read every other's (pulls allowed)
    std::mutex m;
    std::condition_variable cv;
    std::map<std::tuple<int, int, uint64_t>, Slot> slots;
};

// a peer that never reaches the matching step is an application bug; fail the
// call instead of hanging the process.  The deadline is on the system clock:
// libstdc++ waits on it with pthread_cond_timedwait, which ThreadSanitizer
// intercepts (a steady-clock wait_for goes through pthread_cond_clockwait,
// which GCC 11's TSan does not, and reads as a double lock)
const auto kPeerTimeout = std::chrono::seconds(300);
std::chrono::system_clock::time_point peer_deadline()
{
    return std::chrono::system_clock::now() + kPeerTimeout;
}

}  // namespace

struct MPIX_Comm_s {
    int rank = 0, size = 1;
    Kind kind = K_CUSTOM;
    ncclComm_t nccl = nullptr;
    std::shared_ptr<Local> local;
    MPIX_Exchange_fn xfn = nullptr;
    void *xctx = nullptr;
    MPIX_Combine_fn combine = nullptr;
    int device = -1;
    hipStream_t own_stream = nullptr;
    void *stream = nullptr;         // stream of the blocking forms (NULL: own_stream)
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
    hipEvent_t scratch_ev = nullptr;   // recorded after the last collective that used scratch
    hipStream_t aux = nullptr;         // combine stream of the pipelined pairwise schedule
    std::vector<hipEvent_t> pipe_ev;   // its hand-off events (chunk k arrived, combines done)
    std::vector<uint64_t> send_seq, recv_seq;
    int xkind = MPIX_XPORT_DEVICE;     // custom communicators: memory kind of the transport
    char *stage = nullptr;             // MPIX_XPORT_STAGED: pinned staging of one exchange
    size_t stage_bytes = 0;
    hipEvent_t stage_ev = nullptr;     // recorded after the copies out of the staging memory
    char *tok = nullptr;               // barrier tokens / published records, (1 + size) slots
    char *win = nullptr;               // pull window (header + data), see ensure_windows
    hipEvent_t win_ev = nullptr;       // recorded after the last pull that used the window
    size_t win_bytes = 0;
    std::vector<char *> win_old;       // outgrown / rejected windows, freed with the comm
    std::vector<void *> peer_map;      // peers' pull windows, mapped and verified
    bool win_broken = false;           // pulls given up on this communicator
    // what actually ran (MPIX_Comm_get_state): the schedule of the last
    // reduce-scatter / allreduce after AUTO and any fallback, the calls whose
    // requested schedule did not run, window verification attempts that failed
    int last_rs = -1, last_ar = -1;
    int fallbacks = 0, win_retries = 0;
    int same_node = -1;                // every rank on this host (IPC possible): -1 not yet asked
    size_t max_msg = 0;                // MPIX_Comm_set_max_message: split above this (0: never)
    size_t rh_min = 0;                 // MPIX_Comm_set_rh_overlap (rh_overlap_default at creation)
    size_t rh_created = 0;             // that creation-time value: what -1 restores
    struct Nonce { int rank, attempt; uint64_t n0, n1; };
    std::vector<Nonce> nonce_hist;     // every window nonce published (MPIX_COLL_TRACE)
    struct Shared {                    // MPIX_Comm_alloc_shared windows
        char *base;                    // header + bytes
        size_t bytes;
        std::vector<void *> maps;      // peers' copies, mapped and verified
    };
    std::vector<Shared> shared;
    bool timing = false;               // MPIX_Comm_set_step_timing
    std::vector<std::pair<std::string, hipEvent_t>> marks;
    bool host() const { return kind == K_LOCAL_HOST || (kind == K_CUSTOM && device < 0); }
    // threads driving several devices pull from each other's buffers only with
    // peer access between every pair of them (else the pull schedules run
    // their transport form, same bits); processes decide by their windows
    bool pulls_possible() const { return !(kind == K_LOCAL_DEV && local && !local->peer_ok); }
};

namespace {

int hip_fail(hipError_t e) { return e == hipSuccess ? MPIX_REDOP_SUCCESS : MPIX_REDOP_ERR_OTHER; }

// A requested schedule that could not run: record what runs instead, so the
// caller can tell (MPIX_Comm_get_state) -- never one schedule's time under
// another's name.  Printed under MPIX_COLL_TRACE.
void ran_instead(MPIX_Comm c, int *last, int alg)
{
    ++c->fallbacks;
    *last = alg;
    if (getenv("MPIX_COLL_TRACE"))
        fprintf(stderr, "[mpix_coll rank %d] requested schedule did not run: schedule %d instead\n",
                c->rank, alg);
}

#define TRY(x) do { int rc_ = (x); if (rc_ != MPIX_REDOP_SUCCESS) return rc_; } while (0)
#define HTRY(x) do { if ((x) != hipSuccess) return MPIX_REDOP_ERR_OTHER; } while (0)

size_t round256(size_t b) { return (b + 255) & ~(size_t) 255; }

int pof2_of(int n)
{
    int p = 1;
    while (p * 2 <= n)
        p *= 2;
    return p;
}

int set_device(MPIX_Comm c)
{
    if (c->device >= 0)
        HTRY(hipSetDevice(c->device));
    return MPIX_REDOP_SUCCESS;
}

hipStream_t stream_of(void *s) { return static_cast<hipStream_t>(s); }

// ------------------------------------------------------------ transports
// RCCL communicators split at 1 GiB: no count reaches 2^31 in RCCL
constexpr size_t kMaxMsg = size_t(1) << 30;

// Messages above `max` bytes go as several consecutive messages to the same
// peer within the one exchange group; both sides split the same lengths the
// same way, so the k-th send of a pair matches its k-th receive in posting
// order with equal sizes (what ncclSend/ncclRecv pairing requires).
void split_messages(std::vector<MPIX_P2p_op> *ops, size_t max)
{
    if (!max)
        return;
    bool any = false;
    for (const MPIX_P2p_op &o : *ops)
        any |= o.bytes > max;
    if (!any)
        return;
    std::vector<MPIX_P2p_op> out;
    for (const MPIX_P2p_op &o : *ops) {
        char *p = static_cast<char *>(o.buf);
        for (size_t off = 0; off < o.bytes; off += max)
            out.push_back(MPIX_P2p_op{o.peer, o.is_recv, p + off,
                                      o.bytes - off < max ? o.bytes - off : max});
    }
    ops->swap(out);
}

int exchange_ccl(MPIX_Comm c, const MPIX_P2p_op *ops, int nops, hipStream_t s)
{
    if (ncclGroupStart() != ncclSuccess)
        return MPIX_REDOP_ERR_OTHER;
    ncclResult_t r = ncclSuccess;
    for (int i = 0; i < nops && r == ncclSuccess; ++i)
        r = ops[i].is_recv ? ncclRecv(ops[i].buf, ops[i].bytes, ncclUint8, ops[i].peer, c->nccl, s)
                           : ncclSend(ops[i].buf, ops[i].bytes, ncclUint8, ops[i].peer, c->nccl, s);
    ncclResult_t r2 = ncclGroupEnd();
    return (r == ncclSuccess && r2 == ncclSuccess) ? MPIX_REDOP_SUCCESS : MPIX_REDOP_ERR_OTHER;
}

int exchange_local(MPIX_Comm c, const MPIX_P2p_op *ops, int nops, hipStream_t s)
{
    Local &L = *c->local;
    const bool host = L.host;
    typedef std::tuple<int, int, uint64_t> Key;
    std::vector<Key> sends, recvs;
    bool any_send = false;
    for (int i = 0; i < nops; ++i)
        any_send |= !ops[i].is_recv && ops[i].bytes;
    // phase 1: post the sends, with the stream position they must follow
    hipEvent_t ready = nullptr;
    if (!host && any_send) {
        HTRY(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        HTRY(hipEventRecord(ready, s));
    }
    {
        std::lock_guard<std::mutex> g(L.m);
        for (int i = 0; i < nops; ++i) {
            if (ops[i].is_recv || !ops[i].bytes)
                continue;
            Key k(c->rank, ops[i].peer, c->send_seq[ops[i].peer]++);
            Slot &sl = L.slots[k];
            sl.buf = ops[i].buf;
            sl.bytes = ops[i].bytes;
            sl.ready = ready;
            sends.push_back(k);
        }
    }
    L.cv.notify_all();
    // phase 2: each receive copies from the matching posted send
    int rc = MPIX_REDOP_SUCCESS;
    for (int i = 0; i < nops && rc == MPIX_REDOP_SUCCESS; ++i) {
        if (!ops[i].is_recv || !ops[i].bytes)
            continue;
        Key k(ops[i].peer, c->rank, c->recv_seq[ops[i].peer]++);
        Slot sl;
        {
            std::unique_lock<std::mutex> g(L.m);
            if (!L.cv.wait_until(g, peer_deadline(), [&] { return L.slots.count(k) != 0; })) {
                rc = MPIX_REDOP_ERR_OTHER;
                break;
            }
            sl = L.slots[k];
        }
        if (sl.bytes > ops[i].bytes) {          // MPI_ERR_TRUNCATE
            rc = MPIX_REDOP_ERR_COUNT;
            break;
        }
        if (host) {
            memcpy(ops[i].buf, sl.buf, sl.bytes);
        } else if (hipStreamWaitEvent(s, sl.ready, 0) != hipSuccess ||
                   hipMemcpyAsync(ops[i].buf, sl.buf, sl.bytes, hipMemcpyDefault, s) != hipSuccess) {
            rc = MPIX_REDOP_ERR_OTHER;
        }
        recvs.push_back(k);
    }
    std::shared_ptr<DoneEv> done;
    if (!recvs.empty()) {
        done = std::make_shared<DoneEv>();
        done->refs = (int) recvs.size();
        if (!host && (hipEventCreateWithFlags(&done->ev, hipEventDisableTiming) != hipSuccess ||
                      hipEventRecord(done->ev, s) != hipSuccess))
            rc = MPIX_REDOP_ERR_OTHER;
    }
    {   // mark consumed even on failure so the senders do not wait forever
        std::lock_guard<std::mutex> g(L.m);
        for (auto &k : recvs) {
            Slot &sl = L.slots[k];
            sl.done = done;
            sl.consumed = true;
        }
    }
    L.cv.notify_all();
    // phase 3: this stream may reuse its send buffers only after the copies
    for (auto &k : sends) {
        std::shared_ptr<DoneEv> d;
        {
            std::unique_lock<std::mutex> g(L.m);
            if (!L.cv.wait_until(g, peer_deadline(), [&] { return L.slots[k].consumed; })) {
                rc = MPIX_REDOP_ERR_OTHER;
                continue;
            }
            d = L.slots[k].done;
            L.slots.erase(k);
        }
        if (!host && d && d->ev && hipStreamWaitEvent(s, d->ev, 0) != hipSuccess)
            rc = MPIX_REDOP_ERR_OTHER;
        std::lock_guard<std::mutex> g(L.m);
        if (d && --d->refs == 0 && d->ev)
            (void) hipEventDestroy(d->ev);      // waits already enqueued; HIP frees it later
    }
    if (ready)
        (void) hipEventDestroy(ready);
    return rc;
}

// MPIX_XPORT_STAGED: the transport only sees host memory, so the device
// buffers are staged through one pinned area per exchange -- the pattern of
// MPIR_Coll_host_buffer_alloc / swap_back (coll_impl.c:305-381).  The stream is
// synchronised first (send data complete, and the previous exchange's copies
// out of the staging area done), the transport runs on the host, and what
// arrived goes back to the device buffers stream-ordered, ahead of the combine.
int exchange_staged(MPIX_Comm c, const MPIX_P2p_op *ops, int nops, hipStream_t s)
{
    size_t total = 0;
    for (int i = 0; i < nops; ++i)
        total += round256(ops[i].bytes);
    if (c->stage_ev)
        HTRY(hipEventSynchronize(c->stage_ev));
    else
        HTRY(hipEventCreateWithFlags(&c->stage_ev, hipEventDisableTiming));
    if (c->stage_bytes < total) {
        if (c->stage)
            HTRY(hipHostFree(c->stage));
        c->stage = nullptr;
        c->stage_bytes = 0;
        void *h = nullptr;
        HTRY(hipHostMalloc(&h, total, hipHostMallocDefault));
        c->stage = static_cast<char *>(h);
        c->stage_bytes = total;
    }
    std::vector<MPIX_P2p_op> h(ops, ops + nops);
    size_t off = 0;
    for (int i = 0; i < nops; ++i) {
        h[i].buf = c->stage + off;
        if (!ops[i].is_recv)
            HTRY(hipMemcpyAsync(h[i].buf, ops[i].buf, ops[i].bytes, hipMemcpyDefault, s));
        off += round256(ops[i].bytes);
    }
    HTRY(hipStreamSynchronize(s));
    if (c->xfn(c->xctx, c->rank, h.data(), nops, nullptr))
        return MPIX_REDOP_ERR_OTHER;
    for (int i = 0; i < nops; ++i)
        if (ops[i].is_recv)
            HTRY(hipMemcpyAsync(ops[i].buf, h[i].buf, ops[i].bytes, hipMemcpyDefault, s));
    HTRY(hipEventRecord(c->stage_ev, s));
    return MPIX_REDOP_SUCCESS;
}

// env MPIX_COLL_TRACE: every exchange step (and the pull's published
// records) as one stderr line per rank -- how a mismatched schedule is found
bool coll_trace()
{
    static const bool t = getenv("MPIX_COLL_TRACE") != nullptr;
    return t;
}

int exchange(MPIX_Comm c, const std::vector<MPIX_P2p_op> &ops, hipStream_t s)
{
    // zero-length messages are not sent (both sides know the lengths, so
    // both skip them; the reference does the same, e.g.
    // reduce_scatter_intra_recursive_halving.c:188-208)
    std::vector<MPIX_P2p_op> nz;
    nz.reserve(ops.size());
    for (const MPIX_P2p_op &o : ops)
        if (o.bytes)
            nz.push_back(o);
    if (nz.empty())
        return MPIX_REDOP_SUCCESS;
    split_messages(&nz, c->max_msg);
    if (coll_trace()) {     // one line per exchange step: what this rank posts
        std::string line = "[mpix_coll rank " + std::to_string(c->rank) + "/" +
                           std::to_string(c->size) + "]";
        for (const MPIX_P2p_op &o : nz)
            line += std::string(" ") + (o.is_recv ? "<" : ">") + std::to_string(o.peer) + ":" +
                    std::to_string(o.bytes);
        fprintf(stderr, "%s\n", line.c_str());
    }
    switch (c->kind) {
        case K_CCL:
            return exchange_ccl(c, nz.data(), (int) nz.size(), s);
        case K_LOCAL_DEV:
        case K_LOCAL_HOST:
            return exchange_local(c, nz.data(), (int) nz.size(), s);
        default:
            if (c->xkind == MPIX_XPORT_STAGED)
                return exchange_staged(c, nz.data(), (int) nz.size(), s);
            return c->xfn(c->xctx, c->rank, nz.data(), (int) nz.size(), s) ? MPIX_REDOP_ERR_OTHER
                                                                           : MPIX_REDOP_SUCCESS;
    }
}

MPIX_P2p_op snd(int peer, const void *buf, size_t bytes)
{
    return MPIX_P2p_op{peer, 0, const_cast<void *>(buf), bytes};
}
MPIX_P2p_op rcv(int peer, void *buf, size_t bytes) { return MPIX_P2p_op{peer, 1, buf, bytes}; }

// per-step breakdown (MPIX_Comm_set_step_timing): an event on the stream
// after each phase of a schedule
int mark(MPIX_Comm c, const char *label, hipStream_t s)
{
    if (!c->timing || c->host())
        return MPIX_REDOP_SUCCESS;
    hipEvent_t e;
    HTRY(hipEventCreate(&e));
    HTRY(hipEventRecord(e, s));
    c->marks.emplace_back(label, e);
    return MPIX_REDOP_SUCCESS;
}

// one published record per rank (barrier tokens are 1-byte records)
constexpr size_t kRec = 256;

// token buffer: (1 + size) record slots, then the barrier's own bytes (one to
// send, one per peer to receive), so a barrier still in flight on one stream
// never lands in a record slot another stream's allgather is reading
size_t tok_bytes(MPIX_Comm c) { return kRec * (size_t) (c->size + 1) + round256(1 + (size_t) c->size); }
char *barrier_tok(MPIX_Comm c) { return c->tok + kRec * (size_t) (c->size + 1); }

int token_buffer(MPIX_Comm c, hipStream_t s)
{
    if (c->tok)
        return MPIX_REDOP_SUCCESS;
    const size_t bytes = tok_bytes(c);
    if (c->host()) {
        c->tok = static_cast<char *>(calloc(1, bytes));
        return c->tok ? MPIX_REDOP_SUCCESS : MPIX_REDOP_ERR_OTHER;
    }
    void *p = nullptr;
    HTRY(hipMalloc(&p, bytes));
    // zeroed ON the collective's stream: a plain hipMemset runs on the null
    // stream, which a non-blocking stream does not wait for, and could land
    // after the record this rank is about to copy in (peers then saw zeros)
    HTRY(hipMemsetAsync(p, 0, bytes, s));
    c->tok = static_cast<char *>(p);
    return MPIX_REDOP_SUCCESS;
}

// every rank's `bytes` (<= kRec) of host data to every rank: one group of
// P-1 sends and P-1 receives; out[q * kRec ...] holds rank q's (own included).
// Synchronous: returns once the records are in host memory.
int allgather_records(MPIX_Comm c, const void *mine, size_t bytes, std::vector<char> *out,
                      hipStream_t s)
{
    TRY(token_buffer(c, s));
    const int P = c->size;
    out->assign(kRec * (size_t) P, 0);
    std::vector<MPIX_P2p_op> ops;
    for (int q = 0; q < P; ++q)
        if (q != c->rank) {
            ops.push_back(snd(q, c->tok, bytes));
            ops.push_back(rcv(q, c->tok + kRec * (size_t) (1 + q), bytes));
        }
    if (c->host()) {
        memcpy(c->tok, mine, bytes);
        TRY(exchange(c, ops, s));
        memcpy(out->data(), c->tok + kRec, kRec * (size_t) P);
    } else {
        HTRY(hipMemcpyAsync(c->tok, mine, bytes, hipMemcpyHostToDevice, s));
        TRY(exchange(c, ops, s));
        HTRY(hipMemcpyAsync(out->data(), c->tok + kRec, kRec * (size_t) P, hipMemcpyDeviceToHost,
                            s));
        HTRY(hipStreamSynchronize(s));
    }
    memcpy(out->data() + kRec * (size_t) c->rank, mine, bytes);
    return MPIX_REDOP_SUCCESS;
}

// a 1-byte message to and from every peer, on the collective's stream
int barrier(MPIX_Comm c, hipStream_t s)
{
    if (c->size == 1)
        return MPIX_REDOP_SUCCESS;
    TRY(token_buffer(c, s));
    std::vector<MPIX_P2p_op> ops;
    char *t = barrier_tok(c);
    for (int q = 0; q < c->size; ++q)
        if (q != c->rank) {
            ops.push_back(snd(q, t, 1));
            ops.push_back(rcv(q, t + 1 + q, 1));
        }
    return exchange(c, ops, s);
}

// ------------------------------------------------------------ data movement
int copy(MPIX_Comm c, void *dst, const void *src, size_t bytes, hipStream_t s)
{
    if (!bytes || dst == src)
        return MPIX_REDOP_SUCCESS;
    if (c->host()) {
        memmove(dst, src, bytes);
        return MPIX_REDOP_SUCCESS;
    }
    return hip_fail(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s));
}

// MPIR_Reduce_local(in, inout, count, datatype, op) of the schedule
int combine(MPIX_Comm c, const void *in, void *inout, MPIX_Aint count, MPIX_Datatype dt, MPIX_Op op,
            hipStream_t s)
{
    if (!count)
        return MPIX_REDOP_SUCCESS;
    if (c->combine)
        return c->combine(in, inout, count, dt, op, s);
    if (c->host())
        return MPIX_Reduce_local(in, inout, count, dt, op);
    return MPIX_Reduce_local_async(in, inout, count, dt, op, s);
}

// k received blocks folded in order: one multi-input kernel pass (16 at most
// per launch), the same association as k combine() calls
int combine_multi(MPIX_Comm c, const std::vector<const void *> &ins, void *inout, MPIX_Aint count,
                  MPIX_Datatype dt, MPIX_Op op, hipStream_t s)
{
    if (c->combine || c->host()) {
        for (const void *p : ins)
            TRY(combine(c, p, inout, count, dt, op, s));
        return MPIX_REDOP_SUCCESS;
    }
    for (size_t lo = 0; lo < ins.size(); lo += 16) {
        int k = (int) std::min<size_t>(16, ins.size() - lo);
        TRY(MPIX_Reduce_local_multi_async(ins.data() + lo, k, inout, count, dt, op, s));
    }
    return MPIX_REDOP_SUCCESS;
}

int combine_to(MPIX_Comm c, const void *a, const void *b, void *out, MPIX_Aint count,
               MPIX_Datatype dt, MPIX_Op op, hipStream_t s, size_t ext)
{
    if (out == a || count == 0)
        return count ? combine(c, b, out, count, dt, op, s) : MPIX_REDOP_SUCCESS;
    if (!c->combine && !c->host()) {
        const void *ins[2] = {a, b};
        return MPIX_Reduce_local_tree_async(ins, 2, out, count, dt, op, s);
    }
    TRY(copy(c, out, a, (size_t) count * ext, s));
    return combine(c, b, out, count, dt, op, s);
}

// out = a OP b (a in the inout role, b in the in role) without first copying
// a into out: one 2-slot tree kernel (MPIX_Reduce_local_tree_async); host /
// custom-combine communicators copy, then combine -- the same operands either way
int combine_to(MPIX_Comm c, const void *a, const void *b, void *out, MPIX_Aint count,
               MPIX_Datatype dt, MPIX_Op op, hipStream_t s, size_t ext);

// The communicator's scratch is shared by every collective issued on it, on
// any stream: a new user is ordered behind the previous one on the device
// (stream wait on scratch_ev, no host sync), and the buffer is only freed
// for growth once that work has drained.
int scratch(MPIX_Comm c, size_t bytes, hipStream_t s, char **out)
{
    if (!c->host()) {
        if (!c->scratch_ev)
            HTRY(hipEventCreateWithFlags(&c->scratch_ev, hipEventDisableTiming));
        HTRY(hipStreamWaitEvent(s, c->scratch_ev, 0));
    }
    if (c->scratch_bytes < bytes) {
        if (c->scratch) {
            if (c->host()) {
                free(c->scratch);
            } else {
                HTRY(hipEventSynchronize(c->scratch_ev));
                HTRY(hipFree(c->scratch));
            }
            c->scratch = nullptr;
            c->scratch_bytes = 0;
        }
        if (c->host()) {
            c->scratch = malloc(bytes);
            if (!c->scratch)
                return MPIX_REDOP_ERR_OTHER;
        } else {
            HTRY(hipMalloc(&c->scratch, bytes));
        }
        c->scratch_bytes = bytes;
    }
    *out = static_cast<char *>(c->scratch);
    return MPIX_REDOP_SUCCESS;
}

int workspace(MPIX_Comm c, void *ws, size_t ws_bytes, size_t need, hipStream_t s, char **out)
{
    if (!need) {
        *out = nullptr;
        return MPIX_REDOP_SUCCESS;
    }
    if (ws) {
        if (ws_bytes < need)
            return MPIX_REDOP_ERR_ARG;
        *out = static_cast<char *>(ws);
        return MPIX_REDOP_SUCCESS;
    }
    return scratch(c, need, s, out);
}

// after a collective enqueued its work on s: mark where the scratch is free
int release_scratch(MPIX_Comm c, const char *used, int rc, hipStream_t s)
{
    if (used && used == c->scratch && c->scratch_ev) {
        int rc2 = hip_fail(hipEventRecord(c->scratch_ev, s));
        return rc ? rc : rc2;
    }
    return rc;
}

int finish(MPIX_Comm c, int rc, hipStream_t s, bool blocking)
{
    if (rc == MPIX_REDOP_SUCCESS && blocking && !c->host())
        rc = hip_fail(hipStreamSynchronize(s));
    return rc;
}

// MPIX_EQUAL compares whole packed buffers behind one 8-byte header
// (opequal.c:20-35); MPIR_Reduce_equal / MPIR_Allreduce_equal run it only
// through schedules that never split the message (binomial reduce, recursive
// doubling allreduce), so the block-splitting schedules refuse it
bool splits_message_forbidden(MPIX_Op op) { return ((uint32_t) op & 0xffu) == 0x0fu &&
                                                   ((uint32_t) op >> 24) == 0x58u; }

int check_args(MPIX_Comm c, const void *recvbuf, MPIX_Aint count, MPIX_Datatype dt, MPIX_Op op,
               size_t *ext)
{
    if (!c)
        return MPIX_REDOP_ERR_ARG;
    if (count < 0)
        return MPIX_REDOP_ERR_COUNT;
    if (!MPIX_Redop_op_dt_check(op, dt))
        return MPIX_REDOP_ERR_OP;
    *ext = (size_t) MPIX_Datatype_extent(dt);
    if (!*ext)
        return MPIX_REDOP_ERR_TYPE;
    // a pair no kernel covers (MPI_LONG_DOUBLE, REAL16, ...) would only fail
    // at its first combine, mid-schedule, with peers still posted to this
    // rank: decline it here, before any exchange, so every rank returns the
    // same error (the reference computes these on the CPU, which the caller
    // keeps for them).  A custom combine takes whatever it is given.  The
    // test is the knob-independent one: MPIX_REDOP_ENABLE / _THRESHOLD steer
    // MPIX_Redop_is_supported's callers (reduce_local.c's branch), not the
    // collectives, as MPIR_CVAR_ENABLE_YAKSA_REDUCTION only moves reductions
    // back to the CPU
    if (!c->combine && !MPIX_Redop_has_gpu_path(op, dt))
        return MPIX_REDOP_ERR_TYPE;
    if (!recvbuf && count)
        return MPIX_REDOP_ERR_BUFFER;
    return MPIX_REDOP_SUCCESS;
}

// ------------------------------------------------------------ schedules
// The communicator's second stream and its hand-off events (pipelined
// schedules): at least `nev` events.
int ensure_aux(MPIX_Comm c, size_t nev)
{
    if (!c->aux)
        HTRY(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    while (c->pipe_ev.size() < nev) {
        hipEvent_t e;
        HTRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->pipe_ev.push_back(e);
    }
    return MPIX_REDOP_SUCCESS;
}

// Smallest half-step (bytes) whose combine recursive halving moves onto the
// second stream (rs_recursive_halving_overlap); 0 = never.  By default 1 MiB
// on RCCL communicators, where the exchange crosses xGMI links and the
// combine has the HBM to itself, and off on the others: where the exchange is
// a device copy on the same GPU (local communicators) the two compete for HBM
// and the split only adds its launches and events -- 1.8 % (4 ranks) and
// 5.8 % (8 ranks) slower on one GPU (tools/rh_overlap_probe.py,
// profiles/r04_rh_overlap_probe.json).  MPIX_COLL_RH_OVERLAP (0 off, N > 0
// the bytes) overrides the default for every communicator created after it is
// set -- read once, at creation; MPIX_Comm_set_rh_overlap per communicator.
size_t rh_overlap_default(Kind kind)
{
    const size_t dflt = kind == K_CCL ? size_t(1) << 20 : 0;
    const char *e = getenv("MPIX_COLL_RH_OVERLAP");
    if (!e || !*e)
        return dflt;
    char *end = nullptr;
    unsigned long long v = strtoull(e, &end, 10);
    return (end && *end == '\0') ? (size_t) v : dflt;
}

size_t rh_overlap_min(MPIX_Comm c) { return c->rh_min; }

// The overlapped form applies to P a power of two >= 4 with equal blocks on a
// device communicator combining with the library's kernels (a custom combine
// is called on the collective's stream only).
bool rh_overlap_applies(MPIX_Comm c, const std::vector<size_t> &cnts, size_t ext)
{
    const int P = c->size;
    if (c->host() || c->combine || P < 4 || (P & (P - 1)))
        return false;
    for (size_t n : cnts)
        if (n != cnts[0])
            return false;
    const size_t min = rh_overlap_min(c);
    // the first step's kept quarter is the largest half-step that can split
    return min && (size_t) (P / 4) * cnts[0] * ext >= min;
}

// rs_recursive_halving with communication and computation overlapped
// (SURVEY.md §7 step 5), P = 2^k >= 4, equal blocks of rc elements.  A step's
// combine is cut in two along the next step's split: the half the next step
// sends is combined first on the collective's stream s -- the next exchange
// waits for it -- and the half it keeps on the communicator's second stream,
// where it runs under the next exchange.  The next step receives into the
// part of this step's receive buffer the sent half was just read from (dead
// by then; the same size with equal blocks), so the kept half's combine and
// the next receive touch disjoint bytes; s waits for the second stream before
// the next combine reads the kept half.  Every element is still combined
// once per step with the same two operands in the same roles: same bits.
// Half-steps under rh_overlap_min() are combined whole on s.
int rs_recursive_halving_overlap(const char *sb, char *rb, size_t rc, MPIX_Datatype dt,
                                 MPIX_Op op, MPIX_Comm c, char *ws, hipStream_t s, size_t ext)
{
    const int rank = c->rank, size = c->size;
    const size_t total = rc * (size_t) size, blk = rc * ext, min = rh_overlap_min(c);
    char *tmp_results = ws;
    char *tmp_recvbuf = ws + round256(total * ext);
    TRY(ensure_aux(c, 2));
    hipEvent_t ev_in = c->pipe_ev[0], ev_kept = c->pipe_ev[1];
    TRY(mark(c, "start", s));
    int mask = size >> 1, send_idx = 0, recv_idx = 0;
    bool in_rb = false, kept_pending = false;
    char *rbuf = nullptr;       // where this step's partner half lands
    while (mask > 0) {
        const int dst = rank ^ mask;
        if (rank < dst)
            send_idx = recv_idx + mask;
        else
            recv_idx = send_idx + mask;
        const bool first = mask == size >> 1;
        const char *cur = first ? sb : tmp_results;
        if (first)
            rbuf = tmp_recvbuf + (size_t) recv_idx * blk;
        const size_t n = (size_t) mask * rc;
        TRY(exchange(c, {snd(dst, cur + (size_t) send_idx * blk, n * ext), rcv(dst, rbuf, n * ext)},
                     s));
        TRY(mark(c, "exchange", s));
        const char *own = cur + (size_t) recv_idx * blk;
        char *out = tmp_results + (size_t) recv_idx * blk;
        if (mask == 1 && recv_idx == rank && (own == rb || own + blk <= rb || rb + blk <= own)) {
            out = rb;
            in_rb = true;
        }
        if (kept_pending) {     // `own` is the half the second stream combined last step
            HTRY(hipStreamWaitEvent(s, ev_kept, 0));
            kept_pending = false;
        }
        const int half = mask >> 1;
        if (half && (size_t) half * blk >= min) {
            // the next step keeps the lower half iff this rank is the lower of
            // its next pair; the other half is what it sends
            const bool keep_low = rank < (rank ^ half);
            const size_t k_off = keep_low ? 0 : (size_t) half * blk;
            const size_t s_off = keep_low ? (size_t) half * blk : 0;
            HTRY(hipEventRecord(ev_in, s));
            HTRY(hipStreamWaitEvent(c->aux, ev_in, 0));
            TRY(combine_to(c, own + k_off, rbuf + k_off, out + k_off, (MPIX_Aint) half * rc, dt,
                           op, c->aux, ext));
            HTRY(hipEventRecord(ev_kept, c->aux));
            kept_pending = true;
            TRY(combine_to(c, own + s_off, rbuf + s_off, out + s_off, (MPIX_Aint) half * rc, dt,
                           op, s, ext));
            TRY(mark(c, "combine (sent half)", s));
            rbuf += s_off;      // the next partner half lands where the sent half was
        } else {
            TRY(combine_to(c, own, rbuf, out, (MPIX_Aint) n, dt, op, s, ext));
            TRY(mark(c, "combine", s));
        }
        send_idx = recv_idx;
        mask >>= 1;
    }
    if (kept_pending)
        HTRY(hipStreamWaitEvent(s, ev_kept, 0));
    if (!in_rb)
        TRY(copy(c, rb, tmp_results + (size_t) rank * blk, blk, s));         // :232-240
    TRY(mark(c, "epilogue", s));
    return MPIX_REDOP_SUCCESS;
}

// MPIR_Reduce_scatter_intra_recursive_halving
// (reduce_scatter_intra_recursive_halving.c:38-260; the _block variant,
// reduce_scatter_block_intra_recursive_halving.c:38-260, is the case of
// equal counts).  cnts[i] = elements of rank i's result block.
int rs_recursive_halving(const char *sb, char *rb, const std::vector<size_t> &cnts,
                         MPIX_Datatype dt, MPIX_Op op, MPIX_Comm c, char *ws, hipStream_t s,
                         size_t ext)
{
    const int rank = c->rank, size = c->size;
    std::vector<size_t> disps(size, 0);
    for (int i = 1; i < size; ++i)
        disps[i] = disps[i - 1] + cnts[i - 1];
    const size_t total = disps[size - 1] + cnts[size - 1];
    if (!total)
        return MPIX_REDOP_SUCCESS;
    if (rh_overlap_applies(c, cnts, ext))
        return rs_recursive_halving_overlap(sb, rb, cnts[0], dt, op, c, ws, s, ext);
    char *tmp_results = ws;
    char *tmp_recvbuf = ws + round256(total * ext);
    const int pof2 = pof2_of(size), rem = size - pof2;
    // P a power of two: no up-front copy of sendbuf into tmp_results (:91-96);
    // the first step reads its halves from sendbuf and writes the combined
    // half into tmp_results, the last writes this rank's block into recvbuf
    // -- the same operands in the same roles, one HBM pass of the whole
    // vector less
    const bool direct = rem == 0;
    TRY(mark(c, "start", s));
    if (!direct) {
        TRY(copy(c, tmp_results, sb, total * ext, s));                     // :91-96
        TRY(mark(c, "local copy", s));
    }
    int newrank;
    if (rank < 2 * rem) {                                                   // :110-137
        if (rank % 2 == 0) {
            TRY(exchange(c, {snd(rank + 1, tmp_results, total * ext)}, s));
            newrank = -1;
        } else {
            TRY(exchange(c, {rcv(rank - 1, tmp_recvbuf, total * ext)}, s));
            TRY(combine(c, tmp_recvbuf, tmp_results, (MPIX_Aint) total, dt, op, s));
            newrank = rank / 2;
        }
        TRY(mark(c, "prologue", s));
    } else {
        newrank = rank - rem;
    }
    if (newrank != -1) {                                                    // :139-229
        std::vector<size_t> newcnts(pof2), newdisps(pof2, 0);
        for (int i = 0; i < pof2; ++i) {
            int old_i = i < rem ? i * 2 + 1 : i + rem;
            newcnts[i] = old_i < 2 * rem ? cnts[old_i] + cnts[old_i - 1] : cnts[old_i];
        }
        for (int i = 1; i < pof2; ++i)
            newdisps[i] = newdisps[i - 1] + newcnts[i - 1];
        auto sum = [&](int lo, int hi) {
            size_t t = 0;
            for (int i = lo; i < hi; ++i)
                t += newcnts[i];
            return t;
        };
        int mask = pof2 >> 1, send_idx = 0, recv_idx = 0, last_idx = pof2;
        bool in_rb = false;         // this rank's block already written to recvbuf
        while (mask > 0) {
            int newdst = newrank ^ mask;
            int dst = newdst < rem ? newdst * 2 + 1 : newdst + rem;
            size_t send_cnt, recv_cnt;
            if (newrank < newdst) {
                send_idx = recv_idx + mask;
                send_cnt = sum(send_idx, last_idx);
                recv_cnt = sum(recv_idx, send_idx);
            } else {
                recv_idx = send_idx + mask;
                send_cnt = sum(send_idx, recv_idx);
                recv_cnt = sum(recv_idx, last_idx);
            }
            const char *cur = direct && mask == pof2 >> 1 ? sb : tmp_results;
            // zero-length legs are skipped on both sides (:188-208)
            TRY(exchange(c, {snd(dst, cur + newdisps[send_idx] * ext, send_cnt * ext),
                             rcv(dst, tmp_recvbuf + newdisps[recv_idx] * ext, recv_cnt * ext)}, s));
            TRY(mark(c, "exchange", s));
            char *out = tmp_results + newdisps[recv_idx] * ext;
            const char *own = cur + newdisps[recv_idx] * ext;
            const size_t nbytes = recv_cnt * ext;
            // the last step's half is this rank's block: written straight into
            // recvbuf, unless that would overwrite the half being read -- with
            // MPI_IN_PLACE at P = 2 the first step is the last and reads
            // recvbuf itself ([disps[1], +c1) against [0, c1) at rank 1)
            if (direct && mask == 1 && recv_idx == newrank &&
                (own == rb || own + nbytes <= rb || rb + nbytes <= own)) {
                out = rb;
                in_rb = true;
            }
            TRY(combine_to(c, own, tmp_recvbuf + newdisps[recv_idx] * ext, out,
                           (MPIX_Aint) recv_cnt, dt, op, s, ext));
            TRY(mark(c, "combine", s));
            send_idx = recv_idx;
            last_idx = recv_idx + mask;
            mask >>= 1;
        }
        if (!in_rb)
            TRY(copy(c, rb, tmp_results + disps[rank] * ext, cnts[rank] * ext, s));   // :232-240
    }
    if (rank < 2 * rem) {                                                   // :245-262
        if (rank % 2)
            TRY(exchange(c, {snd(rank - 1, tmp_results + disps[rank - 1] * ext,
                                 cnts[rank - 1] * ext)}, s));
        else
            TRY(exchange(c, {rcv(rank + 1, rb, cnts[rank] * ext)}, s));
    }
    TRY(mark(c, "epilogue", s));
    return MPIX_REDOP_SUCCESS;
}

// True when the multipath recursive halving applies: P a power of two >= 4
// and equal blocks (every rank's half has the same size at every step, so a
// relay knows what it forwards without a size exchange).
bool multipath_shape(const std::vector<size_t> &cnts, int size)
{
    if (size < 4 || (size & (size - 1)))
        return false;
    for (size_t n : cnts)
        if (n != cnts[0])
            return false;
    return true;
}

// relay masks of a step with mask m: one of every pair {a, a ^ m}, a != m
// (the smaller), so first hops (r ^ a) and second hops (r ^ a ^ m) together
// use each of the other P - 2 links once
std::vector<int> relay_masks(int m, int size)
{
    std::vector<int> A;
    for (int a = 1; a < size; ++a)
        if (a != m && a < (a ^ m))
            A.push_back(a);
    return A;
}

size_t multipath_relay_bytes(size_t recvcount, size_t ext, int size)
{
    return (size_t) (size / 2 - 1) * round256(recvcount * ext);
}

// One exchange step of a recursive-halving schedule routed over every link
// (P a power of two >= 4, the same D elements moving each way between every
// rank r and its partner r ^ mask).  Rank r's D elements at sbase are cut into
// n = P/2 parts: part 0 goes to the partner directly, part j to the relay
// r ^ a_j, which forwards it to its own r ^ a_j ^ mask = the partner.  Every
// rank is at once source, relay for the ranks r ^ a_j and destination of its
// partner's relayed parts, so all P - 1 directed links of every rank carry
// D / n.  The relay hops are pipelined in C chunks per part: group g moves
// direct and first-hop chunk g and forwards chunk g - 1.  The partner's D
// elements land at rbase exactly as one direct receive would leave them.
// relay: (P/2 - 1) slots of `slot` bytes (>= one part).
int multipath_exchange(MPIX_Comm c, const char *sbase, char *rbase, size_t D, int mask, char *relay,
                       size_t slot, hipStream_t s, size_t ext)
{
    const int rank = c->rank;
    const std::vector<int> A = relay_masks(mask, c->size);
    const size_t n = A.size() + 1;
    auto lo = [&](size_t j) { return D * j / n; };   // part j: [lo(j), lo(j+1))
    // chunks per part: >= 4 MiB each, at most 8 (one group when small)
    size_t C = ((lo(1) - lo(0)) * ext) >> 22;
    C = C < 1 ? 1 : (C > 8 ? 8 : C);
    auto piece = [&](size_t j, size_t k, size_t *off, size_t *len) {
        const size_t pl = lo(j + 1) - lo(j);
        const size_t a = pl * k / C, b = pl * (k + 1) / C;
        *off = lo(j) + a;
        *len = b - a;
    };
    for (size_t g = 0; g <= C; ++g) {
        std::vector<MPIX_P2p_op> ops;
        size_t off, len;
        if (g < C) {
            piece(0, g, &off, &len);
            ops.push_back(snd(rank ^ mask, sbase + off * ext, len * ext));
            ops.push_back(rcv(rank ^ mask, rbase + off * ext, len * ext));
            for (size_t j = 1; j < n; ++j) {
                piece(j, g, &off, &len);
                ops.push_back(snd(rank ^ A[j - 1], sbase + off * ext, len * ext));
                ops.push_back(rcv(rank ^ A[j - 1], relay + (j - 1) * slot + (off - lo(j)) * ext,
                                  len * ext));
            }
        }
        if (g > 0) {
            for (size_t j = 1; j < n; ++j) {
                piece(j, g - 1, &off, &len);
                ops.push_back(snd(rank ^ A[j - 1] ^ mask,
                                  relay + (j - 1) * slot + (off - lo(j)) * ext, len * ext));
                ops.push_back(rcv(rank ^ A[j - 1] ^ mask, rbase + off * ext, len * ext));
            }
        }
        TRY(exchange(c, ops, s));
    }
    return MPIX_REDOP_SUCCESS;
}

// MPIX_RSB_RECURSIVE_HALVING_MULTIPATH: rs_recursive_halving's schedule with
// every exchange step spread over all links (multipath_exchange), then one
// combine per step into tmp_results: same operands, same order, same bits.
int rs_recursive_halving_multipath(const char *sb, char *rb, const std::vector<size_t> &cnts,
                                   MPIX_Datatype dt, MPIX_Op op, MPIX_Comm c, char *ws,
                                   hipStream_t s, size_t ext)
{
    const int rank = c->rank, size = c->size;
    const size_t rc = cnts[0], total = rc * size;
    char *tmp_results = ws;
    char *tmp_recvbuf = ws + round256(total * ext);
    char *relay = tmp_recvbuf + round256(total * ext);     // (P/2 - 1) part slots
    const size_t slot = round256(rc * ext);                 // a part is at most one block
    // as rs_recursive_halving with P a power of two: the first step reads
    // sendbuf, the last writes this rank's block into recvbuf (no copies)
    TRY(mark(c, "start", s));
    int mask = size >> 1, send_idx = 0, recv_idx = 0;
    bool in_rb = false;
    while (mask > 0) {
        if (rank < (rank ^ mask))
            send_idx = recv_idx + mask;
        else
            recv_idx = send_idx + mask;
        const size_t D = (size_t) mask * rc;             // both halves, every rank
        const char *cur = mask == size >> 1 ? sb : tmp_results;
        char *rbase = tmp_recvbuf + (size_t) recv_idx * rc * ext;
        TRY(multipath_exchange(c, cur + (size_t) send_idx * rc * ext, rbase, D, mask, relay, slot,
                               s, ext));
        TRY(mark(c, "exchange", s));
        char *out = tmp_results + (size_t) recv_idx * rc * ext;
        if (mask == 1 && recv_idx == rank) {
            out = rb;
            in_rb = true;
        }
        TRY(combine_to(c, cur + (size_t) recv_idx * rc * ext, rbase, out, (MPIX_Aint) D, dt, op, s,
                       ext));
        TRY(mark(c, "combine", s));
        send_idx = recv_idx;
        mask >>= 1;
    }
    if (!in_rb)
        TRY(copy(c, rb, tmp_results + (size_t) rank * rc * ext, rc * ext, s));   // :232-240
    TRY(mark(c, "epilogue", s));
    return MPIX_REDOP_SUCCESS;
}

// MPIR_Reduce_scatter_intra_pairwise (reduce_scatter_intra_pairwise.c:42-115;
// the _block variant …_block_intra_pairwise.c:42-104 with equal counts):
// step i = 1..P-1 sends block (rank+i) to rank+i and folds the block
// received from rank-i into the result, in that order.  `concurrent` posts
// all P-1 exchanges as one group (every xGMI link busy at once) and folds
// the P-1 blocks in one multi-input pass; same order, same bits.
// MPI_IN_PLACE (sb == rb): blocks go out of recvbuf, the own block is
// reduced where it lies and moved to the front at the end (:58-64, :71-115).
int rs_pairwise(const char *sb, char *rb, const std::vector<size_t> &cnts, MPIX_Datatype dt,
                MPIX_Op op, MPIX_Comm c, char *ws, hipStream_t s, size_t ext, bool concurrent)
{
    const int rank = c->rank, size = c->size;
    std::vector<size_t> disps(size, 0);
    for (int i = 1; i < size; ++i)
        disps[i] = disps[i - 1] + cnts[i - 1];
    const size_t blk = cnts[rank] * ext, sstride = round256(blk);
    const bool in_place = sb == rb;
    char *acc = in_place ? rb + disps[rank] * ext : rb;
    TRY(mark(c, "start", s));
    if (!in_place)
        TRY(copy(c, rb, sb + disps[rank] * ext, blk, s));                   // :58-64
    if (!concurrent) {
        for (int i = 1; i < size; ++i) {
            int dst = (rank + i) % size, src = (rank - i + size) % size;
            TRY(exchange(c, {snd(dst, sb + disps[dst] * ext, cnts[dst] * ext),
                             rcv(src, ws, blk)}, s));
            TRY(combine(c, ws, acc, (MPIX_Aint) cnts[rank], dt, op, s));
        }
    } else {
        std::vector<MPIX_P2p_op> ops;
        std::vector<const void *> ins;
        for (int i = 1; i < size; ++i) {
            int dst = (rank + i) % size, src = (rank - i + size) % size;
            ops.push_back(snd(dst, sb + disps[dst] * ext, cnts[dst] * ext));
            ops.push_back(rcv(src, ws + (i - 1) * sstride, blk));
            ins.push_back(ws + (i - 1) * sstride);
        }
        TRY(exchange(c, ops, s));
        TRY(mark(c, "exchange", s));
        if (cnts[rank])
            TRY(combine_multi(c, ins, acc, (MPIX_Aint) cnts[rank], dt, op, s));
        TRY(mark(c, "combine", s));
    }
    if (in_place && rank != 0) {
        // with uneven counts the own block can overlap the front of recvbuf;
        // device copies must not overlap, so go through the (free) workspace
        if (disps[rank] * ext < blk && !c->host()) {
            TRY(copy(c, ws, acc, blk, s));
            TRY(copy(c, rb, ws, blk, s));
        } else {
            TRY(copy(c, rb, acc, blk, s));
        }
    }
    return MPIX_REDOP_SUCCESS;
}

// rs_pairwise with `concurrent`, cut into chunks: chunk k of every one of the
// P-1 messages moves in one exchange group on the collective's stream while
// the combine of chunk k-1 runs on the communicator's second stream, so the
// multi-input combine hides behind the transfer.  A chunk is the same element
// range [k*q, ...) of a message on both sides (q from the receiver's count),
// every element still folds its P-1 inputs in the same order: same bits.
int rs_pairwise_pipelined(const char *sb, char *rb, const std::vector<size_t> &cnts,
                          MPIX_Datatype dt, MPIX_Op op, MPIX_Comm c, char *ws, hipStream_t s,
                          size_t ext)
{
    const int rank = c->rank, size = c->size;
    const size_t blk = cnts[rank] * ext;
    // the chunk count must be the same on every rank (both ends of a message
    // cut it alike), so it follows the largest block: chunks of >= 4 MiB of
    // it, at most kPipeChunks
    size_t maxblk = 0;
    for (size_t n : cnts)
        maxblk = n * ext > maxblk ? n * ext : maxblk;
    if (c->host() || c->combine || size == 1 || maxblk < (size_t(8) << 20))
        return rs_pairwise(sb, rb, cnts, dt, op, c, ws, s, ext, true);
    constexpr size_t kPipeChunks = 8;
    size_t nch = maxblk >> 22;
    if (nch > kPipeChunks)
        nch = kPipeChunks;
    TRY(ensure_aux(c, nch + 1));
    std::vector<size_t> disps(size, 0);
    for (int i = 1; i < size; ++i)
        disps[i] = disps[i - 1] + cnts[i - 1];
    const size_t sstride = round256(blk);
    const bool in_place = sb == rb;
    char *acc = in_place ? rb + disps[rank] * ext : rb;
    if (!in_place)
        TRY(copy(c, rb, sb + disps[rank] * ext, blk, s));
    auto lo = [nch](size_t n, size_t k) { return n * k / nch; };    // chunk k: [lo(k), lo(k+1))
    for (size_t k = 0; k < nch; ++k) {
        std::vector<MPIX_P2p_op> ops;
        std::vector<const void *> ins;
        const size_t r0 = lo(cnts[rank], k), r1 = lo(cnts[rank], k + 1);
        for (int i = 1; i < size; ++i) {
            const int dst = (rank + i) % size, src = (rank - i + size) % size;
            const size_t s0 = lo(cnts[dst], k), s1 = lo(cnts[dst], k + 1);
            ops.push_back(snd(dst, sb + (disps[dst] + s0) * ext, (s1 - s0) * ext));
            ops.push_back(rcv(src, ws + (i - 1) * sstride + r0 * ext, (r1 - r0) * ext));
            ins.push_back(ws + (i - 1) * sstride + r0 * ext);
        }
        TRY(exchange(c, ops, s));
        // chunk k (and, for k = 0, the own-block copy) is in: hand it over
        HTRY(hipEventRecord(c->pipe_ev[k], s));
        HTRY(hipStreamWaitEvent(c->aux, c->pipe_ev[k], 0));
        if (r1 > r0)
            TRY(combine_multi(c, ins, acc + r0 * ext, (MPIX_Aint) (r1 - r0), dt, op, c->aux));
    }
    HTRY(hipEventRecord(c->pipe_ev[nch], c->aux));
    HTRY(hipStreamWaitEvent(s, c->pipe_ev[nch], 0));
    if (in_place && rank != 0) {
        if (disps[rank] * ext < blk) {
            TRY(copy(c, ws, acc, blk, s));
            TRY(copy(c, rb, ws, blk, s));
        } else {
            TRY(copy(c, rb, acc, blk, s));
        }
    }
    return MPIX_REDOP_SUCCESS;
}

size_t rs_workspace(size_t total, size_t mine, size_t ext, int size, int algo);
int bitrev(int r, int pof2);

// ---- pull windows --------------------------------------------------------
// The pulls read peers' memory directly.  Ranks that are threads of one
// process (K_LOCAL_DEV) share the address space and read each other's user
// buffers.  Across processes the memory must be mapped through hipIpc, and
// mapping the USER buffers per call is not safe on this platform: once
// allocations have been freed and re-made, a freshly opened handle can map
// another allocation -- an earlier one, another rank's, even the opener's own
// (tools/ipc_multi_probe.py: 19 of 58 reads wrong at 4 ranks on one GPU,
// profiles/r02_ipc_multi_probe.json).  So every rank keeps a WINDOW: device
// memory the library owns, exported once, mapped once by every peer, and
// verified at mapping time -- its 256-byte header carries a random 128-bit
// nonce that each peer reads back through its mapping and compares with the
// published one; the ranks then agree that all mappings are right, or retry
// with a new window (up to 3 times; the rejected ones stay allocated so their
// identity is never reused), or give the pulls up for this communicator
// (they run the RCCL-transport schedules instead, with the same bits).  A
// call copies its input into the window (one local HBM pass), and peers read
// it from there.  Windows grow (never shrink) to the largest message; an
// outgrown one stays allocated until MPIX_Comm_free for the same reason.
constexpr size_t kWinHdr = 256;

struct WinRec {
    int32_t valid;
    int32_t pad;
    uint64_t bytes;
    uint64_t nonce[2];
    char handle[sizeof(hipIpcMemHandle_t)];
};
static_assert(sizeof(WinRec) <= kRec, "window record size");

struct LocalRec {   // K_LOCAL_DEV: the raw address
    int32_t valid;
    int32_t pad;
    uint64_t raw;
};

// MPIX_COLL_TRACE: what a mapping that failed verification shows instead --
// the nonce of an earlier window (whose, from which attempt), of this round's
// window of another rank, or nothing published
void trace_wrong_window(MPIX_Comm c, int q, const uint64_t seen[2], const std::vector<char> &all)
{
    const char *what = "no published nonce";
    int who = -1, when = -1;
    for (int p = 0; p < c->size; ++p) {
        WinRec r;
        memcpy(&r, all.data() + kRec * (size_t) p, sizeof r);
        if (r.nonce[0] == seen[0] && r.nonce[1] == seen[1]) {
            what = "this round's window of rank";
            who = p;
        }
    }
    for (const auto &h : c->nonce_hist)
        if (who < 0 && h.n0 == seen[0] && h.n1 == seen[1]) {
            what = "an earlier window of rank";
            who = h.rank;
            when = h.attempt;
        }
    fprintf(stderr, "[mpix_coll rank %d] window of rank %d reads %016llx%016llx: %s %d (attempt %d)\n",
            c->rank, q, (unsigned long long) seen[0], (unsigned long long) seen[1], what, who, when);
    for (int p = 0; p < c->size; ++p) {   // the published handles, to compare
        WinRec r;
        memcpy(&r, all.data() + kRec * (size_t) p, sizeof r);
        fprintf(stderr, "[mpix_coll rank %d]   handle of rank %d:", c->rank, p);
        for (size_t b = 0; b < sizeof r.handle; ++b)
            fprintf(stderr, "%02x", (unsigned char) r.handle[b]);
        fprintf(stderr, "\n");
    }
}

void close_maps(std::vector<void *> *maps)
{
    for (void *m : *maps)
        if (m)
            (void) hipIpcCloseMemHandle(m);
    maps->clear();
}

// Collective: a new device allocation of kWinHdr + `bytes` on every rank,
// exported (one rank at a time), mapped by every peer (maps[q]) and verified
// through the mapping by the nonce in its header, with every rank agreeing on
// the outcome.  On a
// failed verification all ranks retry (3 attempts; the rejected allocations
// stay allocated, in win_old, so their identity is never reused).  *w = NULL
// on every rank when no attempt succeeded.
int verified_window(MPIX_Comm c, size_t bytes, hipStream_t s, char **w_out,
                    std::vector<void *> *maps)
{
    *w_out = nullptr;
    // IPC handles open only on the exporter's node: a communicator spanning
    // nodes would allocate three message-size windows per attempt before
    // giving up.  One record exchange, once per communicator, settles it
    // first: the kernel's boot id and the host name must match on every rank.
    if (c->same_node < 0) {
        char me[kRec];
        memset(me, 0, sizeof me);
        if (FILE *f = fopen("/proc/sys/kernel/random/boot_id", "r")) {
            if (!fgets(me, 64, f))
                me[0] = 0;
            fclose(f);
        }
        (void) gethostname(me + 64, 128);
        if (const char *id = getenv("MPIX_COLL_NODE_ID"))    // test hook: pretend another node
            snprintf(me + 192, 64, "%s", id);
        std::vector<char> all;
        TRY(allgather_records(c, me, sizeof me, &all, s));
        c->same_node = 1;
        for (int q = 0; q < c->size; ++q)
            if (memcmp(all.data() + kRec * (size_t) q, me, sizeof me) != 0)
                c->same_node = 0;
        if (!c->same_node && coll_trace())
            fprintf(stderr, "[mpix_coll rank %d] peers on other nodes: no pull windows\n", c->rank);
    }
    if (!c->same_node)
        return MPIX_REDOP_SUCCESS;
    std::random_device rd;
    for (int attempt = 0; attempt < 3; ++attempt) {
        void *w = nullptr;
        WinRec me;
        memset(&me, 0, sizeof me);
        auto make = [&]() {
            if (hipMalloc(&w, kWinHdr + bytes) == hipSuccess) {
                me.nonce[0] = ((uint64_t) rd() << 32) ^ rd() ^ ((uint64_t) c->rank << 48);
                me.nonce[1] = ((uint64_t) rd() << 32) ^ rd() ^ (uint64_t) attempt;
                hipIpcMemHandle_t h;
                hipError_t e = hipMemcpy(w, me.nonce, sizeof me.nonce, hipMemcpyHostToDevice);
                if (e == hipSuccess)
                    e = hipIpcGetMemHandle(&h, w);
                if (e == hipSuccess) {
                    memcpy(me.handle, &h, sizeof h);
                    me.valid = 1;
                    me.bytes = bytes;
                } else if (coll_trace()) {
                    fprintf(stderr, "[mpix_coll rank %d] window export failed: %s\n", c->rank,
                            hipGetErrorString(e));
                }
                // test hook: this rank publishes a nonce its window does not hold, as
                // a mapping of the wrong memory would show it to the peers
                const char *fault = getenv("MPIX_COLL_WINDOW_FAULT");
                if (fault && atoi(fault) == c->rank)
                    me.nonce[1] ^= 1;
            }
            (void) hipGetLastError();
        };
        maps->assign(c->size, nullptr);
        int good = 1;
        // open and verify peer q's window from its published record
        auto check = [&](int q, const std::vector<char> &recs) {
            WinRec r;
            memcpy(&r, recs.data() + kRec * (size_t) q, sizeof r);
            if (!r.valid || r.bytes < bytes) {
                good = 0;
                return;
            }
            hipIpcMemHandle_t h;
            memcpy(&h, r.handle, sizeof h);
            void *m = nullptr;
            uint64_t seen[2] = {0, 0};
            const hipError_t e = hipIpcOpenMemHandle(&m, h, hipIpcMemLazyEnablePeerAccess);
            if (e != hipSuccess) {
                (void) hipGetLastError();
                good = 0;
                if (coll_trace())
                    fprintf(stderr, "[mpix_coll rank %d] window of rank %d: open failed: %s\n",
                            c->rank, q, hipGetErrorString(e));
                return;
            }
            (*maps)[q] = m;
            if (hipMemcpy(seen, m, sizeof seen, hipMemcpyDeviceToHost) != hipSuccess ||
                seen[0] != r.nonce[0] || seen[1] != r.nonce[1]) {
                (void) hipGetLastError();
                good = 0;
                if (coll_trace())
                    trace_wrong_window(c, q, seen, recs);
            }
        };
        std::vector<char> all;
        // One exporter at a time: rank e makes its window and publishes it,
        // every other rank maps and checks it, then rank e + 1.  With every
        // rank exporting at once, a peer's freshly opened handle mapped
        // ANOTHER rank's new window in 6 of 12 four-rank runs on one GPU (all
        // 3 attempts failing in 4); one at a time, no mapping was wrong in 12
        // runs and the rare failed export passed on the retry
        // (tools/win_grow_probe.py, profiles/r02_window_growth.json).
        // MPIX_COLL_WINDOW_SERIAL=0 restores the concurrent exports.
        const char *eser = getenv("MPIX_COLL_WINDOW_SERIAL");
        if (!eser || atoi(eser)) {
            all.assign(kRec * (size_t) c->size, 0);
            for (int e = 0; e < c->size; ++e) {
                WinRec none;
                memset(&none, 0, sizeof none);
                if (e == c->rank)
                    make();
                std::vector<char> one;
                TRY(allgather_records(c, e == c->rank ? &me : &none, sizeof me, &one, s));
                memcpy(all.data() + kRec * (size_t) e, one.data() + kRec * (size_t) e, kRec);
                if (e != c->rank && good)
                    check(e, one);
            }
            good = good && me.valid;
        } else {
            make();
            TRY(allgather_records(c, &me, sizeof me, &all, s));
            good = me.valid;
            for (int q = 0; q < c->size && good; ++q)
                if (q != c->rank)
                    check(q, all);
        }
        for (int q = 0; q < c->size && coll_trace(); ++q) {   // every nonce published, for the trace
            WinRec r;
            memcpy(&r, all.data() + kRec * (size_t) q, sizeof r);
            c->nonce_hist.push_back({q, attempt, r.nonce[0], r.nonce[1]});
        }
        // agreement: every rank's mappings verified, or nobody uses them
        std::vector<char> votes;
        TRY(allgather_records(c, &good, sizeof good, &votes, s));
        bool all_good = true;
        for (int q = 0; q < c->size; ++q) {
            int v;
            memcpy(&v, votes.data() + kRec * (size_t) q, sizeof v);
            all_good = all_good && v == 1;
        }
        if (coll_trace())
            fprintf(stderr, "[mpix_coll rank %d] pull window %zu B attempt %d: mine %d, all %d\n",
                    c->rank, bytes, attempt, good, (int) all_good);
        if (all_good) {
            *w_out = static_cast<char *>(w);
            return MPIX_REDOP_SUCCESS;
        }
        close_maps(maps);
        ++c->win_retries;
        if (w)
            c->win_old.push_back(static_cast<char *>(w));     // never reused, see above
    }
    return MPIX_REDOP_SUCCESS;
}

// Every rank's pull window holds at least `need` data bytes and every peer's
// is mapped and verified (*ok), or the pulls are off for this communicator
// (*ok = false on every rank).  Collective: every rank calls it with the same
// `need` (the message size), so all ranks grow at the same calls.
int ensure_windows(MPIX_Comm c, size_t need, hipStream_t s, bool *ok)
{
    *ok = false;
    if (c->win_broken)
        return MPIX_REDOP_SUCCESS;
    // the window is shared by pulls issued on any stream: a new user is
    // ordered behind the previous one (its closing barrier) on the device
    if (!c->win_ev)
        HTRY(hipEventCreateWithFlags(&c->win_ev, hipEventDisableTiming));
    if (c->win && c->win_bytes >= need) {
        HTRY(hipStreamWaitEvent(s, c->win_ev, 0));
        *ok = true;
        return MPIX_REDOP_SUCCESS;
    }
    HTRY(hipEventSynchronize(c->win_ev));   // nothing in flight reads the old mappings
    HTRY(hipStreamSynchronize(s));
    close_maps(&c->peer_map);
    if (c->win) {                       // outgrown: kept allocated, see above
        c->win_old.push_back(c->win);
        c->win = nullptr;
        c->win_bytes = 0;
    }
    const size_t bytes = std::max(need, 2 * c->win_bytes);
    char *w;
    TRY(verified_window(c, bytes, s, &w, &c->peer_map));
    if (!w) {
        c->win_broken = true;
        if (coll_trace())
            fprintf(stderr, "[mpix_coll rank %d] pull windows given up: the RCCL-transport "
                            "schedules run instead\n", c->rank);
        return MPIX_REDOP_SUCCESS;
    }
    c->win = w;
    c->win_bytes = bytes;
    *ok = true;
    return MPIX_REDOP_SUCCESS;
}

// The shared window (MPIX_Comm_alloc_shared) holding [p, p + bytes), and p's
// offset in it; -1 if none.
int64_t shared_of(MPIX_Comm c, const void *p, size_t bytes, int64_t *off)
{
    const char *x = static_cast<const char *>(p);
    for (size_t i = 0; i < c->shared.size(); ++i) {
        const char *b = c->shared[i].base + kWinHdr;
        if (x >= b && x + bytes <= b + c->shared[i].bytes) {
            *off = x - b;
            return (int64_t) i;
        }
    }
    *off = 0;
    return -1;
}

// Do all ranks hold `n` buffers (ps[i], bytes[i]) in the same shared windows
// at the same offsets?  Then a pull reads the peers' copies in place (no copy
// into the pull window).  Collective once the communicator has shared windows:
// the ranks compare (window, offset) records, after their streams have
// finished writing the buffers -- the "inputs ready" point of the pull.
int shared_direct(MPIX_Comm c, int n, const void *const *ps, const size_t *bytes, hipStream_t s,
                  bool *direct, std::vector<int64_t> *where)
{
    *direct = false;
    if (c->shared.empty() || c->kind == K_LOCAL_DEV)
        return MPIX_REDOP_SUCCESS;
    int64_t me[4] = {-1, 0, -1, 0};
    for (int i = 0; i < n && i < 2; ++i)
        me[2 * i] = shared_of(c, ps[i], bytes[i], &me[2 * i + 1]);
    HTRY(hipStreamSynchronize(s));
    std::vector<char> all;
    TRY(allgather_records(c, me, sizeof me, &all, s));
    bool same = true;
    for (int q = 0; q < c->size && same; ++q) {
        int64_t r[4];
        memcpy(r, all.data() + kRec * (size_t) q, sizeof r);
        for (int i = 0; i < 2 * n; ++i)
            same = same && r[i] == me[i];
    }
    for (int i = 0; i < n; ++i)
        same = same && me[2 * i] >= 0;
    *direct = same;
    where->assign(me, me + 2 * n);
    if (coll_trace())
        fprintf(stderr, "[mpix_coll rank %d] shared-window pull: %s\n", c->rank,
                same ? "direct" : "copy");
    return MPIX_REDOP_SUCCESS;
}

// MPIX_RSB_PULL: the pairwise schedule with the transport and the receive
// buffers folded into the combine.  Every rank's inputs become readable by
// its peers -- in its pull window (another process: copied in, then a
// stream-ordered barrier) or in place (threads of one process: the address
// is all-gathered after the stream has finished writing the inputs) -- and
// ONE multi-input kernel reads block `rank` of every peer in the order of
// …_intra_pairwise.c:86-100 (i = 1..P-1, source rank - i), i.e. the bits of
// PAIRWISE; a closing barrier on the stream keeps every rank from reusing its
// window / buffer before all peers have pulled from it.
//
// tree (MPIX_RSB_RECURSIVE_HALVING_PULL, P a power of two): the same pull,
// but the kernel folds the P blocks as recursive halving's steps would
// (MPIX_Reduce_local_tree_async with slot s = rank ^ bitrev(s): the first
// step's partner rank ^ P/2 in slot 1, …recursive_halving.c:164-229), writing
// the result straight into recvbuf: the bits of RECURSIVE_HALVING, with every
// link busy at once and one read of each block instead of log2(P) exchange +
// combine rounds.
int rs_pull(const char *sb, char *rb, const std::vector<size_t> &cnts, MPIX_Datatype dt, MPIX_Op op,
            MPIX_Comm c, hipStream_t s, size_t ext, bool tree = false)
{
    const int rank = c->rank, size = c->size;
    std::vector<size_t> disps(size, 0);
    for (int i = 1; i < size; ++i)
        disps[i] = disps[i - 1] + cnts[i - 1];
    size_t total = 0;
    for (size_t n : cnts)
        total += n;
    auto fallback = [&]() -> int {     // same bits: one-group pairwise / recursive halving
        const int alg = tree ? MPIX_RSB_RECURSIVE_HALVING : MPIX_RSB_PAIRWISE;
        ran_instead(c, &c->last_rs, alg);
        char *w;
        TRY(workspace(c, nullptr, 0, rs_workspace(total, cnts[rank], ext, size, alg), s, &w));
        return release_scratch(c, w,
                               tree ? rs_recursive_halving(sb, rb, cnts, dt, op, c, w, s, ext)
                                    : rs_pairwise(sb, rb, cnts, dt, op, c, w, s, ext, true),
                               s);
    };
    if (c->host() || c->combine || size > 16 || !c->pulls_possible())
        return fallback();
    const size_t blk = cnts[rank] * ext;
    const bool in_place = sb == rb;
    char *acc = in_place ? rb + disps[rank] * ext : rb;
    TRY(mark(c, "start", s));
    std::vector<const char *> bases(size, sb);  // where each rank's inputs are read
    bool used_win = false;
    if (c->kind == K_LOCAL_DEV) {
        // threads of one process: the user buffers themselves
        LocalRec me{1, 0, reinterpret_cast<uint64_t>(sb)};
        HTRY(hipStreamSynchronize(s));  // this rank's inputs complete before anyone reads them
        std::vector<char> all;
        TRY(allgather_records(c, &me, sizeof me, &all, s));
        for (int q = 0; q < size; ++q) {
            LocalRec r;
            memcpy(&r, all.data() + kRec * (size_t) q, sizeof r);
            bases[q] = reinterpret_cast<const char *>(r.raw);
        }
    } else {
        bool direct;
        std::vector<int64_t> where;
        const void *ps[1] = {sb};
        const size_t nbs[1] = {total * ext};
        TRY(shared_direct(c, 1, ps, nbs, s, &direct, &where));
        if (direct) {                   // every rank's input in a shared window: read in place
            for (int q = 0; q < size; ++q)
                if (q != rank)
                    bases[q] = static_cast<const char *>(c->shared[where[0]].maps[q]) + kWinHdr +
                               where[1];
        } else {
            bool ok;
            TRY(ensure_windows(c, total * ext, s, &ok));
            if (!ok)
                return fallback();
            used_win = true;
            // the blocks the peers read (this rank's own block is read from sb)
            char *wd = c->win + kWinHdr;
            TRY(copy(c, wd, sb, disps[rank] * ext, s));
            TRY(copy(c, wd + (disps[rank] + cnts[rank]) * ext, sb + (disps[rank] + cnts[rank]) * ext,
                     (total - disps[rank] - cnts[rank]) * ext, s));
            TRY(barrier(c, s));         // every window filled
            for (int q = 0; q < size; ++q)
                if (q != rank)
                    bases[q] = static_cast<const char *>(c->peer_map[q]) + kWinHdr;
        }
    }
    if (!in_place && !tree)
        TRY(copy(c, rb, sb + disps[rank] * ext, blk, s));                   // :58-64
    std::vector<const void *> ins;
    if (tree) {
        // slot s: rank ^ bitrev(s) (P a power of two); otherwise the
        // reference's fold (:110-137) is the first level -- slot pair (2t, 2t+1)
        // is new rank v = nr ^ bitrev(t): inout the odd rank 2v + 1, in the even
        // 2v, or new rank v's own input alone -- and its block holds this rank's
        const int pof2 = pof2_of(size), rem = size - pof2;
        const int nr = rank < 2 * rem ? rank / 2 : rank - rem;
        const int k = rem ? 2 * pof2 : pof2;
        for (int sl = 0; sl < k; ++sl) {
            int src;
            if (!rem) {
                src = rank ^ bitrev(sl, size);
            } else {
                const int v = nr ^ bitrev(sl / 2, pof2), j = sl % 2;
                src = v < rem ? (j ? 2 * v : 2 * v + 1) : (j ? -1 : v + rem);
            }
            ins.push_back(src < 0 ? nullptr : bases[src] + disps[rank] * ext);
        }
    } else {
        for (int i = 1; i < size; ++i)
            ins.push_back(bases[(rank - i + size) % size] + disps[rank] * ext);
    }
    TRY(mark(c, "publish", s));
    if (cnts[rank] && tree)
        TRY(MPIX_Reduce_local_tree_async(ins.data(), (int) ins.size(), acc, (MPIX_Aint) cnts[rank],
                                         dt, op, s));
    else if (cnts[rank])
        TRY(combine_multi(c, ins, acc, (MPIX_Aint) cnts[rank], dt, op, s));
    TRY(mark(c, "pull+combine", s));
    TRY(barrier(c, s));                 // peers done reading this rank's buffer / window
    if (used_win)
        HTRY(hipEventRecord(c->win_ev, s));
    if (in_place && rank != 0) {
        if (disps[rank] * ext < blk) {
            char *w;
            TRY(scratch(c, round256(blk), s, &w));
            TRY(copy(c, w, acc, blk, s));
            TRY(copy(c, rb, w, blk, s));
            TRY(release_scratch(c, w, MPIX_REDOP_SUCCESS, s));
        } else {
            TRY(copy(c, rb, acc, blk, s));
        }
    }
    return MPIX_REDOP_SUCCESS;
}

// generic.json:277-291 / :316-341: recursive halving below 512 KiB of total
// message, pairwise above (commutative ops)
int rs_choose(int algorithm, size_t total_bytes)
{
    if (algorithm != MPIX_RSB_AUTO)
        return algorithm;
    return total_bytes < (512u << 10) ? MPIX_RSB_RECURSIVE_HALVING : MPIX_RSB_PAIRWISE;
}

int rsb_choose(int algorithm, size_t recvcount, size_t ext, int size)
{
    return rs_choose(algorithm, recvcount * ext * size);
}

// scratch bytes of a schedule: total = all ranks' elements, mine = this
// rank's result elements
size_t rs_workspace(size_t total, size_t mine, size_t ext, int size, int algo)
{
    if (size == 1)
        return 0;
    switch (algo) {
        case MPIX_RSB_RECURSIVE_HALVING:
            return 2 * round256(total * ext);
        case MPIX_RSB_RECURSIVE_HALVING_MULTIPATH:   // + the relay slots (total = size * mine)
            return 2 * round256(total * ext) +
                   (total == mine * (size_t) size ? multipath_relay_bytes(mine, ext, size) : 0);
        case MPIX_RSB_PAIRWISE:
        case MPIX_RSB_PAIRWISE_PIPELINED:
            return (size - 1) * round256(mine * ext);
        case MPIX_RSB_PAIRWISE_SEQUENTIAL:
            return round256(mine * ext);
        case MPIX_RSB_RECURSIVE_HALVING_PULL:       // P > 16 runs RECURSIVE_HALVING
            return size > 16 ? 2 * round256(total * ext) : 0;
        default:
            return 0;
    }
}

// MPI_Reduce: tmp_buf, plus the accumulator a non-root rank has no recvbuf for
size_t reduce_workspace(size_t nb, bool is_root)
{
    return round256(nb) + (is_root ? 0 : round256(nb));
}

size_t rsb_workspace(size_t recvcount, size_t ext, int size, int algo)
{
    return rs_workspace(recvcount * size, recvcount, ext, size, algo);
}

int bitrev(int r, int pof2)
{
    int out = 0;
    for (int b = pof2 >> 1; b; b >>= 1) {
        out = (out << 1) | (r & 1);
        r >>= 1;
    }
    return out;
}

// MPIR_Allreduce_intra_reduce_scatter_allgather
// (allreduce_intra_reduce_scatter_allgather.c:41-277); `direct` replaces the
// log2(P) allgather exchanges (:191-226) by one group of P-1 direct ones --
// the allgather only moves finished blocks, so the bits do not change.
// `multipath` (MPIX_ALLREDUCE_RSAG_MULTIPATH) routes each reduce-scatter step
// over every link (multipath_exchange) when P is a power of two >= 4 and the
// blocks are equal; the relay slots live in tmp's half that the step does not
// receive into (never read again), so the workspace stays count elements.
int allreduce_rsag(char *rb, size_t count, MPIX_Datatype dt, MPIX_Op op, MPIX_Comm c, char *tmp,
                   hipStream_t s, size_t ext, bool direct, bool multipath = false)
{
    const int rank = c->rank, size = c->size;
    const int pof2 = pof2_of(size), rem = size - pof2;
    const size_t nb = count * ext;
    int newrank;
    if (rank < 2 * rem) {                                                   // :85-112
        if (rank % 2 == 0) {
            TRY(exchange(c, {snd(rank + 1, rb, nb)}, s));
            newrank = -1;
        } else {
            TRY(exchange(c, {rcv(rank - 1, tmp, nb)}, s));
            TRY(combine(c, tmp, rb, (MPIX_Aint) count, dt, op, s));
            newrank = rank / 2;
        }
    } else {
        newrank = rank - rem;
    }
    if (newrank != -1) {
        std::vector<size_t> cnts(pof2), disps(pof2, 0);
        for (int i = 0; i < pof2; ++i)
            cnts[i] = count / pof2 + ((size_t) i < count % pof2 ? 1 : 0);
        for (int i = 1; i < pof2; ++i)
            disps[i] = disps[i - 1] + cnts[i - 1];
        auto sum = [&](int lo, int hi) {
            size_t t = 0;
            for (int i = lo; i < hi; ++i)
                t += cnts[i];
            return t;
        };
        auto real = [&](int nr) { return nr < rem ? nr * 2 + 1 : nr + rem; };
        int mask = 1, send_idx = 0, recv_idx = 0, last_idx = pof2;
        int mp_steps = 0;           // reduce-scatter steps that ran over the relays
        while (mask < pof2) {                                               // :138-189
            int newdst = newrank ^ mask;
            size_t send_cnt, recv_cnt;
            if (newrank < newdst) {
                send_idx = recv_idx + pof2 / (mask * 2);
                send_cnt = sum(send_idx, last_idx);
                recv_cnt = sum(recv_idx, send_idx);
            } else {
                recv_idx = send_idx + pof2 / (mask * 2);
                send_cnt = sum(send_idx, recv_idx);
                recv_cnt = sum(recv_idx, last_idx);
            }
            const size_t parts = (size_t) pof2 / 2;
            const bool mp_step = multipath && rem == 0 && pof2 >= 4 && count % pof2 == 0 &&
                                 send_cnt >= parts * (parts - 1);
            if (mp_step) {
                ++mp_steps;
                // send_cnt == recv_cnt here; relay slots fit in send_cnt elements
                const size_t slot = (send_cnt + parts - 1) / parts * ext;
                TRY(multipath_exchange(c, rb + disps[send_idx] * ext, tmp + disps[recv_idx] * ext,
                                       send_cnt, mask, tmp + disps[send_idx] * ext, slot, s, ext));
            } else {
                TRY(exchange(c, {snd(real(newdst), rb + disps[send_idx] * ext, send_cnt * ext),
                                 rcv(real(newdst), tmp + disps[recv_idx] * ext, recv_cnt * ext)},
                             s));
            }
            TRY(combine(c, tmp + disps[recv_idx] * ext, rb + disps[recv_idx] * ext,
                        (MPIX_Aint) recv_cnt, dt, op, s));
            send_idx = recv_idx;
            mask <<= 1;
            if (mask < pof2)
                last_idx = recv_idx + pof2 / mask;
        }
        // a step too small for the relay slots runs the plain exchange (the
        // last, smallest steps first); the call counts as MULTIPATH while its
        // first step -- the one that moves the most -- went over the relays,
        // and as the plain schedule only when no step did
        if (multipath && !mp_steps)
            ran_instead(c, &c->last_ar, MPIX_ALLREDUCE_REDUCE_SCATTER_ALLGATHER);
        mask >>= 1;
        if (direct) {
            const int mine = bitrev(newrank, pof2);
            std::vector<MPIX_P2p_op> ops;
            for (int q = 0; q < pof2; ++q) {
                if (q == newrank)
                    continue;
                const int b = bitrev(q, pof2);
                ops.push_back(snd(real(q), rb + disps[mine] * ext, cnts[mine] * ext));
                ops.push_back(rcv(real(q), rb + disps[b] * ext, cnts[b] * ext));
            }
            TRY(exchange(c, ops, s));
            mask = 0;
        }
        while (mask > 0) {                                                  // :191-226
            int newdst = newrank ^ mask;
            size_t send_cnt, recv_cnt;
            if (newrank < newdst) {
                if (mask != pof2 / 2)
                    last_idx = last_idx + pof2 / (mask * 2);
                recv_idx = send_idx + pof2 / (mask * 2);
                send_cnt = sum(send_idx, recv_idx);
                recv_cnt = sum(recv_idx, last_idx);
            } else {
                recv_idx = send_idx - pof2 / (mask * 2);
                send_cnt = sum(send_idx, last_idx);
                recv_cnt = sum(recv_idx, send_idx);
            }
            TRY(exchange(c, {snd(real(newdst), rb + disps[send_idx] * ext, send_cnt * ext),
                             rcv(real(newdst), rb + disps[recv_idx] * ext, recv_cnt * ext)}, s));
            if (newrank > newdst)
                send_idx = recv_idx;
            mask >>= 1;
        }
    }
    if (rank < 2 * rem) {                                                   // :229-238
        if (rank % 2)
            TRY(exchange(c, {snd(rank - 1, rb, nb)}, s));
        else
            TRY(exchange(c, {rcv(rank + 1, rb, nb)}, s));
    }
    return MPIX_REDOP_SUCCESS;
}

// MPIX_ALLREDUCE_PULL: the Rabenseifner allreduce's association (same bits as
// REDUCE_SCATTER_ALLGATHER) as two pulls over the IPC mappings, P a power of
// two <= 16 on a device communicator.  Reduce-scatter: rank r owns block
// bitrev(r) (the halving steps of :138-189 keep the half selected by bit 0,
// then bit 1, ...), which recursive halving with masks 1, 2, 4, ... folds as
// MPIX_Reduce_local_tree_async does with slot s = r ^ s; ONE tree kernel reads
// that block of every rank's input (peers' from their pull windows, or from
// their buffers for threads of one process) and writes it out.  Allgather:
// after a barrier, ONE copy kernel reads every peer's finished block
// (MPIX_Copy_multi_async).  A closing barrier keeps every rank's window /
// buffers in place until its peers are done.  No workspace.  Other shapes:
// the sendbuf copy + REDUCE_SCATTER_ALLGATHER.
int allreduce_rsag(char *rb, size_t count, MPIX_Datatype dt, MPIX_Op op, MPIX_Comm c, char *tmp,
                   hipStream_t s, size_t ext, bool direct, bool multipath);

int allreduce_pull(const char *sendbuf, char *rb, size_t count, MPIX_Datatype dt, MPIX_Op op,
                   MPIX_Comm c, void *ws, size_t ws_bytes, hipStream_t s, size_t ext)
{
    const int rank = c->rank, size = c->size;
    const size_t nb = count * ext;
    auto fallback = [&]() -> int {
        ran_instead(c, &c->last_ar, MPIX_ALLREDUCE_REDUCE_SCATTER_ALLGATHER);
        if (sendbuf)
            TRY(copy(c, rb, sendbuf, nb, s));
        char *tmp;
        TRY(workspace(c, ws, ws_bytes, round256(nb), s, &tmp));
        return release_scratch(c, tmp, allreduce_rsag(rb, count, dt, op, c, tmp, s, ext, true,
                                                      false), s);
    };
    if (c->host() || c->combine || size > 16 || !c->pulls_possible())
        return fallback();
    const char *in = sendbuf ? sendbuf : rb;
    // the reference's layout (:85-127): P - pof2 even/odd pairs fold first (the
    // odd rank keeps going as new rank i), then pof2 new ranks share pof2
    // blocks; new rank v owns block bitrev(v)
    const int pof2 = pof2_of(size), rem = size - pof2;
    std::vector<size_t> cnts(pof2), disps(pof2, 0);
    for (int i = 0; i < pof2; ++i)
        cnts[i] = count / pof2 + ((size_t) i < count % pof2 ? 1 : 0);
    for (int i = 1; i < pof2; ++i)
        disps[i] = disps[i - 1] + cnts[i - 1];
    auto real = [rem](int v) { return v < rem ? 2 * v + 1 : v + rem; };
    const int nr = rank < 2 * rem ? (rank % 2 ? rank / 2 : -1) : rank - rem;
    const int mine = nr >= 0 ? bitrev(nr, pof2) : -1;     // -1: a folded-away even rank
    // in_base[q]: where rank q's input is read; out_base[q]: where its
    // reduced block is read in the allgather; out: where this rank's goes
    std::vector<const char *> in_base(size, in), out_base(size, rb);
    bool used_win = false;
    char *out = mine >= 0 ? rb + disps[mine] * ext : nullptr;
    TRY(mark(c, "start", s));
    if (c->kind == K_LOCAL_DEV) {     // threads of one process: the user buffers
        struct Recs {
            LocalRec in, out;
        } me{{1, 0, reinterpret_cast<uint64_t>(in)}, {1, 0, reinterpret_cast<uint64_t>(rb)}};
        static_assert(sizeof(Recs) <= kRec, "allreduce pull records");
        HTRY(hipStreamSynchronize(s));  // inputs complete before anyone reads them
        std::vector<char> all;
        TRY(allgather_records(c, &me, sizeof me, &all, s));
        for (int q = 0; q < size; ++q) {
            Recs r;
            memcpy(&r, all.data() + kRec * (size_t) q, sizeof r);
            in_base[q] = reinterpret_cast<const char *>(r.in.raw);
            out_base[q] = reinterpret_cast<const char *>(r.out.raw);
        }
    } else {                            // processes
        bool direct;
        std::vector<int64_t> where;
        const void *ps[2] = {in, rb};
        const size_t nbs[2] = {nb, nb};
        TRY(shared_direct(c, 2, ps, nbs, s, &direct, &where));
        if (direct) {                   // input and result in shared windows: in place
            for (int q = 0; q < size; ++q) {
                if (q == rank)
                    continue;
                in_base[q] = static_cast<const char *>(c->shared[where[0]].maps[q]) + kWinHdr +
                             where[1];
                out_base[q] = static_cast<const char *>(c->shared[where[2]].maps[q]) + kWinHdr +
                              where[3];
            }
        } else {                        // the pull windows
            bool ok;
            TRY(ensure_windows(c, nb, s, &ok));
            if (!ok)
                return fallback();
            used_win = true;
            char *wd = c->win + kWinHdr;
            if (mine >= 0) {            // every block but this rank's own (only it reads that)
                TRY(copy(c, wd, in, disps[mine] * ext, s));
                TRY(copy(c, wd + (disps[mine] + cnts[mine]) * ext,
                         in + (disps[mine] + cnts[mine]) * ext,
                         nb - (disps[mine] + cnts[mine]) * ext, s));
                out = wd + disps[mine] * ext;   // peers read it from the window
            } else {
                TRY(copy(c, wd, in, nb, s));
            }
            TRY(barrier(c, s));         // every window filled
            for (int q = 0; q < size; ++q)
                if (q != rank)
                    in_base[q] = out_base[q] = static_cast<const char *>(c->peer_map[q]) + kWinHdr;
        }
    }
    TRY(mark(c, "publish", s));
    if (mine >= 0 && cnts[mine]) {
        // slot s of the tree: without a fold, rank nr ^ s (masks 1, 2, ...:
        // :138-189); with one, slot pair (2t, 2t + 1) is new rank v = nr ^ t's
        // fold -- inout the odd rank 2v + 1, in the even 2v (:94-108) -- or
        // new rank v's own input alone
        const int k = rem ? 2 * pof2 : pof2;
        std::vector<const void *> ins(k, nullptr);
        for (int sl = 0; sl < k; ++sl) {
            int src;
            if (!rem) {
                src = nr ^ sl;
            } else {
                const int v = nr ^ (sl / 2), j = sl % 2;
                src = v < rem ? (j ? 2 * v : 2 * v + 1) : (j ? -1 : v + rem);
            }
            if (src >= 0)
                ins[sl] = in_base[src] + disps[mine] * ext;
        }
        TRY(MPIX_Reduce_local_tree_async(ins.data(), k, out, (MPIX_Aint) cnts[mine], dt, op, s));
    }
    TRY(mark(c, "reduce-scatter pull", s));
    TRY(barrier(c, s));                 // every block final (and every input read)
    std::vector<const void *> srcs;
    std::vector<void *> dsts;
    std::vector<MPIX_Aint> bytes;
    for (int v = 0; v < pof2; ++v) {
        const int q = real(v), b = bitrev(v, pof2);
        const char *src = q == rank ? out : out_base[q] + disps[b] * ext;
        if (src == rb + disps[b] * ext)
            continue;                   // this rank's block already in place
        srcs.push_back(src);
        dsts.push_back(rb + disps[b] * ext);
        bytes.push_back((MPIX_Aint) (cnts[b] * ext));
    }
    for (size_t lo = 0; lo < srcs.size(); lo += 16) {
        const int n = (int) std::min<size_t>(16, srcs.size() - lo);
        TRY(MPIX_Copy_multi_async(srcs.data() + lo, dsts.data() + lo, bytes.data() + lo, n, s));
    }
    TRY(mark(c, "allgather pull", s));
    TRY(barrier(c, s));                 // peers done reading this rank's window / buffers
    if (used_win)
        HTRY(hipEventRecord(c->win_ev, s));
    return MPIX_REDOP_SUCCESS;
}

// MPIR_Allreduce_intra_recursive_doubling (allreduce_intra_recursive_doubling.c:24-150)
int allreduce_rd(char *rb, size_t count, MPIX_Datatype dt, MPIX_Op op, MPIX_Comm c, char *tmp,
                 hipStream_t s, size_t ext)
{
    const int rank = c->rank, size = c->size;
    const int pof2 = pof2_of(size), rem = size - pof2;
    const size_t nb = count * ext;
    int newrank;
    if (rank < 2 * rem) {                                                   // :59-86
        if (rank % 2 == 0) {
            TRY(exchange(c, {snd(rank + 1, rb, nb)}, s));
            newrank = -1;
        } else {
            TRY(exchange(c, {rcv(rank - 1, tmp, nb)}, s));
            TRY(combine(c, tmp, rb, (MPIX_Aint) count, dt, op, s));
            newrank = rank / 2;
        }
    } else {
        newrank = rank - rem;
    }
    if (newrank != -1) {
        for (int mask = 1; mask < pof2; mask <<= 1) {                       // :97-129
            int newdst = newrank ^ mask;
            int dst = newdst < rem ? newdst * 2 + 1 : newdst + rem;
            TRY(exchange(c, {snd(dst, rb, nb), rcv(dst, tmp, nb)}, s));
            TRY(combine(c, tmp, rb, (MPIX_Aint) count, dt, op, s));
        }
    }
    if (rank < 2 * rem) {                                                   // :131-141
        if (rank % 2)
            TRY(exchange(c, {snd(rank - 1, rb, nb)}, s));
        else
            TRY(exchange(c, {rcv(rank + 1, rb, nb)}, s));
    }
    return MPIX_REDOP_SUCCESS;
}

// MPIR_Reduce_intra_binomial (reduce_intra_binomial.c:12-131) for the
// predefined (commutative) ops: relative to the root, a rank receives from
// relrank|mask for every mask below its lowest set bit, in increasing mask
// order, folding each child in with MPIR_Reduce_local(tmp_buf, recvbuf), then
// sends its result to relrank & ~mask.  acc: the root's recvbuf, or a
// temporary on the other ranks; tmp: count elements.
int reduce_binomial(char *acc, size_t count, MPIX_Datatype dt, MPIX_Op op, int root, MPIX_Comm c,
                    char *tmp, hipStream_t s, size_t ext)
{
    const int rank = c->rank, size = c->size;
    const size_t nb = count * ext;
    const int relrank = (rank - root + size) % size;
    for (int mask = 1; mask < size; mask <<= 1) {                           // :84-121
        if ((mask & relrank) == 0) {
            int source = relrank | mask;
            if (source < size) {
                TRY(exchange(c, {rcv((source + root) % size, tmp, nb)}, s));
                TRY(combine(c, tmp, acc, (MPIX_Aint) count, dt, op, s));
            }
        } else {
            TRY(exchange(c, {snd(((relrank & ~mask) + root) % size, acc, nb)}, s));
            break;
        }
    }
    return MPIX_REDOP_SUCCESS;
}

// MPIR_Reduce_intra_reduce_scatter_gather (reduce_intra_reduce_scatter_gather.c
// :40-330): odd ranks below 2*rem fold into their EVEN left neighbour (the
// opposite of the allreduce's pairing), a reduce-scatter by recursive halving
// with increasing distance over blocks cnts[i] = count/pof2 (+1 for the first
// count%pof2), then a binomial gather of the finished blocks to the root
// (an excluded odd root takes block 0 from rank 0 and newrank 0's place).
int reduce_rsg(char *acc, size_t count, MPIX_Datatype dt, MPIX_Op op, int root, MPIX_Comm c,
               char *tmp, hipStream_t s, size_t ext)
{
    const int rank = c->rank, size = c->size;
    const int pof2 = pof2_of(size), rem = size - pof2;
    const size_t nb = count * ext;
    int newrank;
    if (rank < 2 * rem) {                                                   // :110-134
        if (rank % 2) {
            TRY(exchange(c, {snd(rank - 1, acc, nb)}, s));
            newrank = -1;
        } else {
            TRY(exchange(c, {rcv(rank + 1, tmp, nb)}, s));
            TRY(combine(c, tmp, acc, (MPIX_Aint) count, dt, op, s));
            newrank = rank / 2;
        }
    } else {
        newrank = rank - rem;
    }
    std::vector<size_t> cnts(pof2, count / pof2), disps(pof2, 0);
    for (size_t i = 0; i < count % (size_t) pof2; ++i)
        cnts[i] += 1;
    for (int i = 1; i < pof2; ++i)
        disps[i] = disps[i - 1] + cnts[i - 1];
    auto sum = [&](int lo, int hi) {
        size_t t = 0;
        for (int i = lo; i < hi; ++i)
            t += cnts[i];
        return t;
    };
    int send_idx = 0, recv_idx = 0, last_idx = 0;
    if (newrank != -1) {                                                    // :150-210
        last_idx = pof2;
        for (int mask = 1; mask < pof2;) {
            int newdst = newrank ^ mask;
            int dst = newdst < rem ? newdst * 2 : newdst + rem;
            size_t send_cnt, recv_cnt;
            if (newrank < newdst) {
                send_idx = recv_idx + pof2 / (mask * 2);
                send_cnt = sum(send_idx, last_idx);
                recv_cnt = sum(recv_idx, send_idx);
            } else {
                recv_idx = send_idx + pof2 / (mask * 2);
                send_cnt = sum(send_idx, recv_idx);
                recv_cnt = sum(recv_idx, last_idx);
            }
            TRY(exchange(c, {snd(dst, acc + disps[send_idx] * ext, send_cnt * ext),
                             rcv(dst, tmp + disps[recv_idx] * ext, recv_cnt * ext)}, s));
            TRY(combine(c, tmp + disps[recv_idx] * ext, acc + disps[recv_idx] * ext,
                        (MPIX_Aint) recv_cnt, dt, op, s));
            send_idx = recv_idx;
            mask <<= 1;
            if (mask < pof2)
                last_idx = recv_idx + pof2 / mask;
        }
    }
    int newroot;                                                            // :215-250
    if (root < 2 * rem) {
        if (root % 2) {
            if (rank == root) {
                TRY(exchange(c, {rcv(0, acc, cnts[0] * ext)}, s));
                newrank = 0;
                send_idx = 0;
                last_idx = 2;
            } else if (newrank == 0) {
                TRY(exchange(c, {snd(root, acc, cnts[0] * ext)}, s));
                newrank = -1;
            }
            newroot = 0;
        } else {
            newroot = root / 2;
        }
    } else {
        newroot = root - rem;
    }
    if (newrank != -1) {                                                    // :252-318
        int j = 0, mask = 1;
        while (mask < pof2) {
            mask <<= 1;
            ++j;
        }
        mask >>= 1;
        --j;
        while (mask > 0) {
            int newdst = newrank ^ mask;
            int dst = newdst < rem ? newdst * 2 : newdst + rem;
            if (newdst == 0 && root < 2 * rem && root % 2)
                dst = root;
            const int newdst_tree_root = (newdst >> j) << j;
            const int newroot_tree_root = (newroot >> j) << j;
            size_t send_cnt, recv_cnt;
            if (newrank < newdst) {
                if (mask != pof2 / 2)
                    last_idx = last_idx + pof2 / (mask * 2);
                recv_idx = send_idx + pof2 / (mask * 2);
                send_cnt = sum(send_idx, recv_idx);
                recv_cnt = sum(recv_idx, last_idx);
            } else {
                recv_idx = send_idx - pof2 / (mask * 2);
                send_cnt = sum(send_idx, last_idx);
                recv_cnt = sum(recv_idx, send_idx);
            }
            if (newdst_tree_root == newroot_tree_root) {
                TRY(exchange(c, {snd(dst, acc + disps[send_idx] * ext, send_cnt * ext)}, s));
                break;
            }
            TRY(exchange(c, {rcv(dst, acc + disps[recv_idx] * ext, recv_cnt * ext)}, s));
            if (newrank > newdst)
                send_idx = recv_idx;
            mask >>= 1;
            --j;
        }
    }
    return MPIX_REDOP_SUCCESS;
}

// MPIR_Scan_intra_recursive_doubling (scan_intra_recursive_doubling.c:60-150)
// and MPIR_Exscan_intra_recursive_doubling (exscan_intra_recursive_doubling.c
// :60-160), commutative ops: partial_scan travels to rank ^ mask each step; a
// rank above its partner folds the incoming partial into partial_scan and
// into its result (Exscan: the first one is copied, not folded; rank 0's
// result is left untouched), a rank below folds it into partial_scan only.
// rb already holds the own contribution for Scan; ps = partial_scan.
int scan_rd(char *rb, char *ps, size_t count, MPIX_Datatype dt, MPIX_Op op, MPIX_Comm c,
            char *tmp, hipStream_t s, size_t ext, bool exclusive)
{
    const int rank = c->rank, size = c->size;
    const size_t nb = count * ext;
    bool flag = false;
    for (int mask = 1; mask < size; mask <<= 1) {
        const int dst = rank ^ mask;
        if (dst >= size)
            continue;
        TRY(exchange(c, {snd(dst, ps, nb), rcv(dst, tmp, nb)}, s));
        if (rank > dst) {
            TRY(combine(c, tmp, ps, (MPIX_Aint) count, dt, op, s));
            if (!exclusive) {
                TRY(combine(c, tmp, rb, (MPIX_Aint) count, dt, op, s));
            } else if (rank != 0) {
                if (!flag)
                    TRY(copy(c, rb, tmp, nb, s));
                else
                    TRY(combine(c, tmp, rb, (MPIX_Aint) count, dt, op, s));
                flag = true;
            }
        } else {
            TRY(combine(c, tmp, ps, (MPIX_Aint) count, dt, op, s));
        }
    }
    return MPIX_REDOP_SUCCESS;
}

int scan_entry(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype dt, MPIX_Op op,
               MPIX_Comm c, void *ws, size_t ws_bytes, void *stream, bool blocking,
               bool exclusive)
{
    size_t ext;
    TRY(check_args(c, recvbuf, count, dt, op, &ext));
    if (!count)
        return MPIX_REDOP_SUCCESS;
    TRY(set_device(c));
    hipStream_t s = stream_of(stream);
    char *rb = static_cast<char *>(recvbuf);
    const size_t nb = (size_t) count * ext;
    char *w;
    TRY(workspace(c, ws, ws_bytes, 2 * round256(nb), s, &w));
    char *ps = w, *tmp = w + round256(nb);
    const void *own = sendbuf ? sendbuf : recvbuf;      // NULL = MPI_IN_PLACE
    TRY(copy(c, ps, own, nb, s));
    if (!exclusive && sendbuf)
        TRY(copy(c, rb, sendbuf, nb, s));
    int rc = scan_rd(rb, ps, (size_t) count, dt, op, c, tmp, s, ext, exclusive);
    return finish(c, release_scratch(c, w, rc, s), s, blocking);
}

// MPI_Reduce(sendbuf, recvbuf, count, datatype, op, root).  The root's
// sendbuf NULL = MPI_IN_PLACE; other ranks accumulate in the workspace.
int reduce_entry(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype dt, MPIX_Op op,
                 int root, MPIX_Comm c, int algorithm, void *ws, size_t ws_bytes, void *stream,
                 bool blocking)
{
    size_t ext;
    if (!c)
        return MPIX_REDOP_ERR_ARG;
    if (root < 0 || root >= c->size)
        return MPIX_REDOP_ERR_ARG;      // MPI_ERR_ROOT has no class in mpix_redop.h
    const bool is_root = c->rank == root;
    TRY(check_args(c, is_root ? recvbuf : sendbuf, count, dt, op, &ext));
    if (algorithm < MPIX_REDUCE_AUTO || algorithm > MPIX_REDUCE_SCATTER_GATHER)
        return MPIX_REDOP_ERR_ARG;
    if (!count)
        return MPIX_REDOP_SUCCESS;
    if (!is_root && !sendbuf)
        return MPIX_REDOP_ERR_BUFFER;
    const int pof2 = pof2_of(c->size);
    const size_t nb = (size_t) count * ext;
    if (algorithm == MPIX_REDUCE_AUTO && splits_message_forbidden(op))
        algorithm = MPIX_REDUCE_BINOMIAL;       // MPIR_Reduce_equal: binomial only
    if (algorithm == MPIX_REDUCE_AUTO)  // generic.json:206-250 (intra, builtin op)
        algorithm = (nb <= 2048 || (size_t) count < (size_t) pof2) ? MPIX_REDUCE_BINOMIAL
                                                                   : MPIX_REDUCE_SCATTER_GATHER;
    if (algorithm == MPIX_REDUCE_SCATTER_GATHER && splits_message_forbidden(op))
        return MPIX_REDOP_ERR_OP;
    if (algorithm == MPIX_REDUCE_SCATTER_GATHER && (size_t) count < (size_t) pof2)
        return MPIX_REDOP_ERR_COUNT;    // the reference asserts count >= pof2 (:86)
    TRY(set_device(c));
    hipStream_t s = stream_of(stream);
    char *w;
    TRY(workspace(c, ws, ws_bytes, reduce_workspace(nb, is_root), s, &w));
    char *acc = is_root ? static_cast<char *>(recvbuf) : w + round256(nb);
    if (!is_root || sendbuf)                                                // :43-47
        TRY(copy(c, acc, sendbuf, nb, s));
    int rc = MPIX_REDOP_SUCCESS;
    if (c->size > 1)
        rc = algorithm == MPIX_REDUCE_BINOMIAL
                 ? reduce_binomial(acc, (size_t) count, dt, op, root, c, w, s, ext)
                 : reduce_rsg(acc, (size_t) count, dt, op, root, c, w, s, ext);
    return finish(c, release_scratch(c, w, rc, s), s, blocking);
}

// MPIR_Allreduce_intra_ring (allreduce_intra_ring.c:10-105): blocks of
// ceil(count/P) (the last ones short or empty); in step i = 0..P-2 a rank
// sends block (rank-1-i) to rank+1 and folds block (rank-2-i) received from
// rank-1 into recvbuf.  The allgather only moves finished blocks, so it is
// ONE group of direct exchanges here (every xGMI link at once) -- same bits
// as the reference's ring allgatherv.
int allreduce_ring(char *rb, size_t count, MPIX_Datatype dt, MPIX_Op op, MPIX_Comm c, char *tmp,
                   hipStream_t s, size_t ext)
{
    const int rank = c->rank, size = c->size;
    std::vector<size_t> cnts(size, 0), displs(size, 0);
    size_t total = 0;
    for (int i = 0; i < size; ++i) {                                        // :34-42
        cnts[i] = (count + size - 1) / size;
        if (total + cnts[i] > count) {
            cnts[i] = count - total;
            break;
        }
        total += cnts[i];
    }
    for (int i = 1; i < size; ++i)
        displs[i] = displs[i - 1] + cnts[i - 1];
    const int src = (size + rank - 1) % size, dst = (rank + 1) % size;
    for (int i = 0; i < size - 1; ++i) {                                    // :57-76
        const int recv_rank = (size + rank - 2 - i) % size;
        const int send_rank = (size + rank - 1 - i) % size;
        TRY(exchange(c, {rcv(src, tmp, cnts[recv_rank] * ext),
                         snd(dst, rb + displs[send_rank] * ext, cnts[send_rank] * ext)}, s));
        TRY(combine(c, tmp, rb + displs[recv_rank] * ext, (MPIX_Aint) cnts[recv_rank], dt, op,
                    s));
    }
    // after step P-2 rank r has folded block r - P = r: that is its finished
    // block, the one MPIR_Allgatherv_intra_ring then circulates (:79-81)
    const int mine = rank;
    std::vector<MPIX_P2p_op> ops;
    for (int q = 0; q < size; ++q) {
        if (q == rank)
            continue;
        const int theirs = q;
        ops.push_back(snd(q, rb + displs[mine] * ext, cnts[mine] * ext));
        ops.push_back(rcv(q, rb + displs[theirs] * ext, cnts[theirs] * ext));
    }
    return exchange(c, ops, s);
}

// MPI_Reduce_scatter (cnts = recvcounts) and MPI_Reduce_scatter_block
// (equal cnts).  sendbuf NULL = MPI_IN_PLACE: recvbuf holds all ranks' inputs.
int rs_entry(const void *sendbuf, void *recvbuf, const std::vector<size_t> &cnts, MPIX_Datatype dt,
             MPIX_Op op, MPIX_Comm c, int algorithm, void *ws, size_t ws_bytes, void *stream,
             bool blocking)
{
    size_t ext, total = 0;
    for (size_t n : cnts)
        total += n;
    TRY(check_args(c, recvbuf, (MPIX_Aint) cnts[c->rank], dt, op, &ext));
    if (algorithm < MPIX_RSB_AUTO || algorithm > MPIX_RSB_LAST)
        return MPIX_REDOP_ERR_ARG;
    if (splits_message_forbidden(op))
        return MPIX_REDOP_ERR_OP;
    if (!total)
        return MPIX_REDOP_SUCCESS;
    if (!recvbuf && !sendbuf)
        return MPIX_REDOP_ERR_BUFFER;
    TRY(set_device(c));
    hipStream_t s = stream_of(stream);
    char *rb = static_cast<char *>(recvbuf);
    const char *sb = sendbuf ? static_cast<const char *>(sendbuf) : rb;
    int algo = rs_choose(algorithm, total * ext);
    c->last_rs = algo;
    if (algo == MPIX_RSB_RECURSIVE_HALVING_MULTIPATH && !multipath_shape(cnts, c->size))
        ran_instead(c, &c->last_rs, algo = MPIX_RSB_RECURSIVE_HALVING);
    if (algo == MPIX_RSB_RECURSIVE_HALVING_PULL && c->size > 16)
        ran_instead(c, &c->last_rs, algo = MPIX_RSB_RECURSIVE_HALVING);
    if (c->size == 1)
        return finish(c, sendbuf ? copy(c, rb, sb, cnts[0] * ext, s) : MPIX_REDOP_SUCCESS, s,
                      blocking);
    char *w;
    TRY(workspace(c, ws, ws_bytes, rs_workspace(total, cnts[c->rank], ext, c->size, algo), s, &w));
    if (algo == MPIX_RSB_PULL || algo == MPIX_RSB_RECURSIVE_HALVING_PULL)
        return finish(c, rs_pull(sb, rb, cnts, dt, op, c, s, ext,
                                 algo == MPIX_RSB_RECURSIVE_HALVING_PULL),
                      s, blocking);
    int rc = algo == MPIX_RSB_RECURSIVE_HALVING
                 ? rs_recursive_halving(sb, rb, cnts, dt, op, c, w, s, ext)
             : algo == MPIX_RSB_RECURSIVE_HALVING_MULTIPATH
                 ? rs_recursive_halving_multipath(sb, rb, cnts, dt, op, c, w, s, ext)
                 : algo == MPIX_RSB_PAIRWISE_PIPELINED
                       ? rs_pairwise_pipelined(sb, rb, cnts, dt, op, c, w, s, ext)
                       : rs_pairwise(sb, rb, cnts, dt, op, c, w, s, ext, algo == MPIX_RSB_PAIRWISE);
    return finish(c, release_scratch(c, w, rc, s), s, blocking);
}

int rsb_entry(const void *sendbuf, void *recvbuf, MPIX_Aint recvcount, MPIX_Datatype dt, MPIX_Op op,
              MPIX_Comm c, int algorithm, void *ws, size_t ws_bytes, void *stream, bool blocking)
{
    if (!c)
        return MPIX_REDOP_ERR_ARG;
    if (recvcount < 0)
        return MPIX_REDOP_ERR_COUNT;
    return rs_entry(sendbuf, recvbuf, std::vector<size_t>(c->size, (size_t) recvcount), dt, op, c,
                    algorithm, ws, ws_bytes, stream, blocking);
}

int rs_counts(MPIX_Comm c, const MPIX_Aint *recvcounts, std::vector<size_t> *cnts)
{
    if (!c)
        return MPIX_REDOP_ERR_ARG;
    if (!recvcounts)
        return MPIX_REDOP_ERR_COUNT;
    cnts->resize(c->size);
    for (int i = 0; i < c->size; ++i) {
        if (recvcounts[i] < 0)
            return MPIX_REDOP_ERR_COUNT;
        (*cnts)[i] = (size_t) recvcounts[i];
    }
    return MPIX_REDOP_SUCCESS;
}

int allreduce_entry(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype dt,
                    MPIX_Op op, MPIX_Comm c, int algorithm, void *ws, size_t ws_bytes, void *stream,
                    bool blocking)
{
    size_t ext;
    TRY(check_args(c, recvbuf, count, dt, op, &ext));
    if (algorithm < MPIX_ALLREDUCE_AUTO || algorithm > MPIX_ALLREDUCE_LAST)
        return MPIX_REDOP_ERR_ARG;
    if (!count)
        return MPIX_REDOP_SUCCESS;
    TRY(set_device(c));
    hipStream_t s = stream_of(stream);
    char *rb = static_cast<char *>(recvbuf);
    const size_t nb = (size_t) count * ext;
    const int pof2 = pof2_of(c->size);
    if (algorithm == MPIX_ALLREDUCE_AUTO)       // generic.json:99-135 (builtin ops)
        algorithm = (nb > 8 && (size_t) count >= (size_t) pof2 && !splits_message_forbidden(op))
                        ? MPIX_ALLREDUCE_REDUCE_SCATTER_ALLGATHER
                        : MPIX_ALLREDUCE_RECURSIVE_DOUBLING;
    if ((algorithm == MPIX_ALLREDUCE_REDUCE_SCATTER_ALLGATHER ||
         algorithm == MPIX_ALLREDUCE_RSAG_RD_ALLGATHER ||
         algorithm == MPIX_ALLREDUCE_RSAG_MULTIPATH || algorithm == MPIX_ALLREDUCE_PULL) &&
        (size_t) count < (size_t) pof2)
        return MPIX_REDOP_ERR_COUNT;    // :127
    if (algorithm != MPIX_ALLREDUCE_RECURSIVE_DOUBLING && splits_message_forbidden(op))
        return MPIX_REDOP_ERR_OP;       // MPIR_Allreduce_equal uses recursive doubling only
    c->last_ar = algorithm;
    if (algorithm == MPIX_ALLREDUCE_RSAG_MULTIPATH && c->size > 1 &&
        !(c->size >= 4 && !(c->size & (c->size - 1)) && (size_t) count % (size_t) pof2 == 0))
        ran_instead(c, &c->last_ar, MPIX_ALLREDUCE_REDUCE_SCATTER_ALLGATHER);
    if (algorithm == MPIX_ALLREDUCE_PULL && c->size > 1)
        return finish(c, allreduce_pull(static_cast<const char *>(sendbuf), rb, (size_t) count, dt,
                                        op, c, ws, ws_bytes, s, ext),
                      s, blocking);
    if (sendbuf)
        TRY(copy(c, rb, sendbuf, nb, s));
    if (c->size == 1)
        return finish(c, MPIX_REDOP_SUCCESS, s, blocking);
    char *tmp;
    TRY(workspace(c, ws, ws_bytes, round256(nb), s, &tmp));
    int rc = algorithm == MPIX_ALLREDUCE_RECURSIVE_DOUBLING
                 ? allreduce_rd(rb, (size_t) count, dt, op, c, tmp, s, ext)
             : algorithm == MPIX_ALLREDUCE_RING
                 ? allreduce_ring(rb, (size_t) count, dt, op, c, tmp, s, ext)
                 : allreduce_rsag(rb, (size_t) count, dt, op, c, tmp, s, ext,
                                  algorithm != MPIX_ALLREDUCE_RSAG_RD_ALLGATHER,
                                  c->last_ar == MPIX_ALLREDUCE_RSAG_MULTIPATH);
    return finish(c, release_scratch(c, tmp, rc, s), s, blocking);
}

MPIX_Comm new_comm(int rank, int size, Kind kind)
{
    MPIX_Comm c = new MPIX_Comm_s;
    c->rank = rank;
    c->size = size;
    c->kind = kind;
    c->send_seq.assign(size, 0);
    c->recv_seq.assign(size, 0);
    c->rh_min = c->rh_created = rh_overlap_default(kind);
    return c;
}

int make_own_stream(MPIX_Comm c)
{
    if (c->host())
        return MPIX_REDOP_SUCCESS;
    TRY(set_device(c));
    HTRY(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
    return MPIX_REDOP_SUCCESS;
}

}  // namespace

extern "C" {

int MPIX_Ccl_get_unique_id(void *id_out)
{
    static_assert(sizeof(ncclUniqueId) <= MPIX_CCL_UNIQUE_ID_BYTES, "unique id size");
    if (!id_out)
        return MPIX_REDOP_ERR_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess)
        return MPIX_REDOP_ERR_OTHER;
    memset(id_out, 0, MPIX_CCL_UNIQUE_ID_BYTES);
    memcpy(id_out, &id, sizeof id);
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_create_ccl(int rank, int size, const void *id, MPIX_Comm *comm)
{
    if (!comm || !id || size < 1 || rank < 0 || rank >= size)
        return MPIX_REDOP_ERR_ARG;
    *comm = nullptr;
    int dev;
    HTRY(hipGetDevice(&dev));
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    MPIX_Comm c = new_comm(rank, size, K_CCL);
    c->device = dev;
    c->max_msg = kMaxMsg;
    if (ncclCommInitRank(&c->nccl, size, uid, rank) != ncclSuccess) {     // rccl.c:43
        delete c;
        return MPIX_REDOP_ERR_OTHER;
    }
    int rc = make_own_stream(c);
    if (rc) {
        ncclCommDestroy(c->nccl);
        delete c;
        return rc;
    }
    *comm = c;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_create_local(int size, const int *devices, MPIX_Comm *comms)
{
    if (!comms || size < 1)
        return MPIX_REDOP_ERR_ARG;
    auto L = std::make_shared<Local>();
    L->size = size;
    L->host = devices == nullptr;
    if (devices) {
        L->devices.assign(devices, devices + size);
        // ranks on distinct devices read each other's buffers in the pull
        // schedules: peer access for every ordered pair, as the reference's
        // HIP init hook enables it (yaksuri_hip_init_hooks.c:164-181).
        // Without it the pulls run their transport form (same bits) and the
        // exchanges are runtime-staged device-to-device copies.
        for (int a = 0; a < size; ++a)
            for (int b = 0; b < size; ++b)
                if (devices[a] != devices[b] && !MPIX_Redop_peer_access(devices[a], devices[b]))
                    L->peer_ok = false;
    }
    for (int r = 0; r < size; ++r) {
        MPIX_Comm c = new_comm(r, size, L->host ? K_LOCAL_HOST : K_LOCAL_DEV);
        c->local = L;
        c->device = devices ? devices[r] : -1;
        int rc = make_own_stream(c);
        if (rc) {
            for (int q = 0; q < r; ++q)
                MPIX_Comm_free(comms[q]);
            delete c;
            return rc;
        }
        comms[r] = c;
    }
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_create_custom(int rank, int size, MPIX_Exchange_fn fn, void *ctx, int memory_kind,
                            MPIX_Comm *comm)
{
    if (!comm || !fn || size < 1 || rank < 0 || rank >= size || memory_kind < MPIX_XPORT_DEVICE ||
        memory_kind > MPIX_XPORT_STAGED)
        return MPIX_REDOP_ERR_ARG;
    MPIX_Comm c = new_comm(rank, size, K_CUSTOM);
    c->xfn = fn;
    c->xctx = ctx;
    c->xkind = memory_kind;
    if (memory_kind != MPIX_XPORT_HOST) {
        int dev;
        if (hipGetDevice(&dev) != hipSuccess) {
            delete c;
            return MPIX_REDOP_ERR_OTHER;
        }
        c->device = dev;
    }
    int rc = make_own_stream(c);
    if (rc) {
        delete c;
        return rc;
    }
    *comm = c;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_set_combine(MPIX_Comm comm, MPIX_Combine_fn fn)
{
    if (!comm)
        return MPIX_REDOP_ERR_ARG;
    comm->combine = fn;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_set_max_message(MPIX_Comm comm, MPIX_Aint bytes)
{
    if (!comm || bytes < 0 || (comm->kind == K_CCL && (bytes == 0 || (size_t) bytes > kMaxMsg)))
        return MPIX_REDOP_ERR_ARG;
    comm->max_msg = (size_t) bytes;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_set_rh_overlap(MPIX_Comm comm, MPIX_Aint min_bytes)
{
    if (!comm || min_bytes < -1)
        return MPIX_REDOP_ERR_ARG;
    // -1: the value the communicator was created with (the kind's default,
    // or MPIX_COLL_RH_OVERLAP as it read then)
    comm->rh_min = min_bytes == -1 ? comm->rh_created : (size_t) min_bytes;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_get_rh_overlap(MPIX_Comm comm, MPIX_Aint *min_bytes)
{
    if (!comm || !min_bytes)
        return MPIX_REDOP_ERR_ARG;
    *min_bytes = (MPIX_Aint) comm->rh_min;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_set_stream(MPIX_Comm comm, void *stream)
{
    if (!comm)
        return MPIX_REDOP_ERR_ARG;
    comm->stream = stream;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_barrier(MPIX_Comm comm)
{
    if (!comm)
        return MPIX_REDOP_ERR_ARG;
    TRY(set_device(comm));
    hipStream_t s = stream_of(comm->stream ? comm->stream : comm->own_stream);
    return finish(comm, barrier(comm, s), s, true);
}

int MPIX_Comm_alloc_shared(MPIX_Comm comm, size_t bytes, void **ptr)
{
    if (!comm || !ptr)
        return MPIX_REDOP_ERR_ARG;
    *ptr = nullptr;
    if (comm->host())
        return MPIX_REDOP_ERR_ARG;
    TRY(set_device(comm));
    hipStream_t s = stream_of(comm->stream ? comm->stream : comm->own_stream);
    MPIX_Comm_s::Shared sh{nullptr, bytes, {}};
    if (comm->kind == K_LOCAL_DEV || comm->size == 1) {
        // one address space: plain device memory (the pulls read peers directly)
        void *p = nullptr;
        HTRY(hipMalloc(&p, kWinHdr + bytes));
        sh.base = static_cast<char *>(p);
    } else {
        TRY(verified_window(comm, bytes, s, &sh.base, &sh.maps));
        if (!sh.base)
            return MPIX_REDOP_ERR_OTHER;    // every rank: no verified mapping
    }
    comm->shared.push_back(std::move(sh));
    *ptr = comm->shared.back().base + kWinHdr;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_free_shared(MPIX_Comm comm, void *ptr)
{
    if (!comm)
        return MPIX_REDOP_ERR_ARG;
    for (size_t i = 0; i < comm->shared.size(); ++i) {
        if (comm->shared[i].base + kWinHdr != ptr)
            continue;
        TRY(MPIX_Comm_barrier(comm));   // every peer done with every copy
        close_maps(&comm->shared[i].maps);
        // kept allocated until MPIX_Comm_free: a freed allocation's identity
        // must not come back (see verified_window)
        comm->win_old.push_back(comm->shared[i].base);
        comm->shared.erase(comm->shared.begin() + (long) i);
        return MPIX_REDOP_SUCCESS;
    }
    return MPIX_REDOP_ERR_BUFFER;
}

int MPIX_Comm_get_state(MPIX_Comm comm, int *pulls_enabled, int *last_rs_algorithm,
                        int *last_allreduce_algorithm, int *window_retries, int *fallbacks)
{
    if (!comm)
        return MPIX_REDOP_ERR_ARG;
    // same_node -1 (not asked yet: settled by the first pull's record
    // exchange) counts as enabled; a communicator found to span nodes is not
    if (pulls_enabled)
        *pulls_enabled = !comm->host() && !comm->combine && comm->size <= 16 &&
                         !comm->win_broken && comm->same_node != 0 && comm->pulls_possible();
    if (last_rs_algorithm)
        *last_rs_algorithm = comm->last_rs;
    if (last_allreduce_algorithm)
        *last_allreduce_algorithm = comm->last_ar;
    if (window_retries)
        *window_retries = comm->win_retries;
    if (fallbacks)
        *fallbacks = comm->fallbacks;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_set_step_timing(MPIX_Comm comm, int enable)
{
    if (!comm)
        return MPIX_REDOP_ERR_ARG;
    comm->timing = enable != 0;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_step_times(MPIX_Comm comm, double *ms, char (*labels)[32], int max, int *n)
{
    if (!comm || !n || max < 0 || (max && !ms))
        return MPIX_REDOP_ERR_ARG;
    *n = 0;
    int rc = MPIX_REDOP_SUCCESS;
    if (!comm->marks.empty() && hipEventSynchronize(comm->marks.back().second) != hipSuccess)
        rc = MPIX_REDOP_ERR_OTHER;
    for (size_t k = 1; k < comm->marks.size() && rc == MPIX_REDOP_SUCCESS && *n < max; ++k) {
        float t = 0.f;
        if (hipEventElapsedTime(&t, comm->marks[k - 1].second, comm->marks[k].second) != hipSuccess) {
            rc = MPIX_REDOP_ERR_OTHER;
            break;
        }
        ms[*n] = t;
        if (labels) {
            strncpy(labels[*n], comm->marks[k].first.c_str(), 31);
            labels[*n][31] = 0;
        }
        ++*n;
    }
    for (auto &m : comm->marks)
        (void) hipEventDestroy(m.second);
    comm->marks.clear();
    return rc;
}

int MPIX_Comm_rank(MPIX_Comm comm, int *rank)
{
    if (!comm || !rank)
        return MPIX_REDOP_ERR_ARG;
    *rank = comm->rank;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_size(MPIX_Comm comm, int *size)
{
    if (!comm || !size)
        return MPIX_REDOP_ERR_ARG;
    *size = comm->size;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Comm_free(MPIX_Comm comm)
{
    if (!comm)
        return MPIX_REDOP_ERR_ARG;
    int rc = MPIX_REDOP_SUCCESS;
    if (!comm->host()) {
        if (set_device(comm) != MPIX_REDOP_SUCCESS)
            rc = MPIX_REDOP_ERR_OTHER;
        if (comm->own_stream && hipStreamSynchronize(comm->own_stream) != hipSuccess)
            rc = MPIX_REDOP_ERR_OTHER;
        if (comm->scratch_ev)   // the scratch may still be in use on a caller stream
            (void) hipEventSynchronize(comm->scratch_ev);
        if (comm->scratch)
            (void) hipFree(comm->scratch);
        if (comm->scratch_ev)
            (void) hipEventDestroy(comm->scratch_ev);
        if (comm->own_stream)
            (void) hipStreamDestroy(comm->own_stream);
        if (comm->aux) {
            if (hipStreamSynchronize(comm->aux) != hipSuccess)
                rc = MPIX_REDOP_ERR_OTHER;
            (void) hipStreamDestroy(comm->aux);
        }
        for (hipEvent_t e : comm->pipe_ev)
            (void) hipEventDestroy(e);
        if (comm->stage_ev) {
            (void) hipEventSynchronize(comm->stage_ev);
            (void) hipEventDestroy(comm->stage_ev);
        }
        if (comm->stage)
            (void) hipHostFree(comm->stage);
        if (comm->tok)
            (void) hipFree(comm->tok);
        if (comm->win_ev) {
            (void) hipEventSynchronize(comm->win_ev);
            (void) hipEventDestroy(comm->win_ev);
        }
        close_maps(&comm->peer_map);
        if (comm->win)
            (void) hipFree(comm->win);
        for (char *w : comm->win_old)
            (void) hipFree(w);
        for (auto &sh : comm->shared) {
            close_maps(&sh.maps);
            (void) hipFree(sh.base);
        }
        for (auto &m : comm->marks)
            (void) hipEventDestroy(m.second);
    } else {
        free(comm->scratch);
        free(comm->tok);
    }
    if (comm->nccl && ncclCommDestroy(comm->nccl) != ncclSuccess)         // rccl.c:237-250
        rc = MPIX_REDOP_ERR_OTHER;
    delete comm;        // the last local handle takes the shared mailbox with it
    return rc;
}

size_t MPIX_Reduce_scatter_block_workspace(MPIX_Aint recvcount, MPIX_Datatype datatype,
                                           MPIX_Comm comm, int algorithm)
{
    size_t ext = (size_t) MPIX_Datatype_extent(datatype);
    if (!comm || !ext || recvcount <= 0)
        return 0;
    return rsb_workspace((size_t) recvcount, ext, comm->size,
                         rsb_choose(algorithm, (size_t) recvcount, ext, comm->size));
}

int MPIX_Reduce_scatter_block(const void *sendbuf, void *recvbuf, MPIX_Aint recvcount,
                              MPIX_Datatype datatype, MPIX_Op op, MPIX_Comm comm, int algorithm,
                              void *workspace, size_t workspace_bytes)
{
    return rsb_entry(sendbuf, recvbuf, recvcount, datatype, op, comm, algorithm, workspace,
                     workspace_bytes, comm ? (comm->stream ? comm->stream : comm->own_stream) : 0,
                     true);
}

int MPIX_Reduce_scatter_block_async(const void *sendbuf, void *recvbuf, MPIX_Aint recvcount,
                                    MPIX_Datatype datatype, MPIX_Op op, MPIX_Comm comm,
                                    int algorithm, void *workspace, size_t workspace_bytes,
                                    void *stream)
{
    return rsb_entry(sendbuf, recvbuf, recvcount, datatype, op, comm, algorithm, workspace,
                     workspace_bytes, stream, false);
}

size_t MPIX_Reduce_scatter_workspace(const MPIX_Aint *recvcounts, MPIX_Datatype datatype,
                                     MPIX_Comm comm, int algorithm)
{
    size_t ext = (size_t) MPIX_Datatype_extent(datatype), total = 0;
    std::vector<size_t> cnts;
    if (!ext || rs_counts(comm, recvcounts, &cnts) != MPIX_REDOP_SUCCESS)
        return 0;
    for (size_t n : cnts)
        total += n;
    return rs_workspace(total, cnts[comm->rank], ext, comm->size,
                        rs_choose(algorithm, total * ext));
}

int MPIX_Reduce_scatter(const void *sendbuf, void *recvbuf, const MPIX_Aint *recvcounts,
                        MPIX_Datatype datatype, MPIX_Op op, MPIX_Comm comm, int algorithm,
                        void *workspace, size_t workspace_bytes)
{
    std::vector<size_t> cnts;
    TRY(rs_counts(comm, recvcounts, &cnts));
    return rs_entry(sendbuf, recvbuf, cnts, datatype, op, comm, algorithm, workspace,
                    workspace_bytes, comm->stream ? comm->stream : comm->own_stream, true);
}

int MPIX_Reduce_scatter_async(const void *sendbuf, void *recvbuf, const MPIX_Aint *recvcounts,
                              MPIX_Datatype datatype, MPIX_Op op, MPIX_Comm comm, int algorithm,
                              void *workspace, size_t workspace_bytes, void *stream)
{
    std::vector<size_t> cnts;
    TRY(rs_counts(comm, recvcounts, &cnts));
    return rs_entry(sendbuf, recvbuf, cnts, datatype, op, comm, algorithm, workspace,
                    workspace_bytes, stream, false);
}

size_t MPIX_Reduce_workspace(MPIX_Aint count, MPIX_Datatype datatype, int root, MPIX_Comm comm)
{
    size_t ext = (size_t) MPIX_Datatype_extent(datatype);
    if (!comm || !ext || count <= 0)
        return 0;
    return reduce_workspace((size_t) count * ext, comm->rank == root);
}

int MPIX_Reduce(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
                MPIX_Op op, int root, MPIX_Comm comm, int algorithm, void *workspace,
                size_t workspace_bytes)
{
    return reduce_entry(sendbuf, recvbuf, count, datatype, op, root, comm, algorithm, workspace,
                        workspace_bytes,
                        comm ? (comm->stream ? comm->stream : comm->own_stream) : 0, true);
}

int MPIX_Reduce_async(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
                      MPIX_Op op, int root, MPIX_Comm comm, int algorithm, void *workspace,
                      size_t workspace_bytes, void *stream)
{
    return reduce_entry(sendbuf, recvbuf, count, datatype, op, root, comm, algorithm, workspace,
                        workspace_bytes, stream, false);
}

size_t MPIX_Scan_workspace(MPIX_Aint count, MPIX_Datatype datatype, MPIX_Comm comm)
{
    size_t ext = (size_t) MPIX_Datatype_extent(datatype);
    if (!comm || !ext || count <= 0)
        return 0;
    return 2 * round256((size_t) count * ext);
}

int MPIX_Scan(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
              MPIX_Op op, MPIX_Comm comm, void *workspace, size_t workspace_bytes)
{
    return scan_entry(sendbuf, recvbuf, count, datatype, op, comm, workspace, workspace_bytes,
                      comm ? (comm->stream ? comm->stream : comm->own_stream) : 0, true, false);
}

int MPIX_Scan_async(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
                    MPIX_Op op, MPIX_Comm comm, void *workspace, size_t workspace_bytes,
                    void *stream)
{
    return scan_entry(sendbuf, recvbuf, count, datatype, op, comm, workspace, workspace_bytes,
                      stream, false, false);
}

int MPIX_Exscan(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
                MPIX_Op op, MPIX_Comm comm, void *workspace, size_t workspace_bytes)
{
    return scan_entry(sendbuf, recvbuf, count, datatype, op, comm, workspace, workspace_bytes,
                      comm ? (comm->stream ? comm->stream : comm->own_stream) : 0, true, true);
}

int MPIX_Exscan_async(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
                      MPIX_Op op, MPIX_Comm comm, void *workspace, size_t workspace_bytes,
                      void *stream)
{
    return scan_entry(sendbuf, recvbuf, count, datatype, op, comm, workspace, workspace_bytes,
                      stream, false, true);
}

size_t MPIX_Allreduce_workspace(MPIX_Aint count, MPIX_Datatype datatype, MPIX_Comm comm)
{
    size_t ext = (size_t) MPIX_Datatype_extent(datatype);
    if (!comm || !ext || count <= 0 || comm->size == 1)
        return 0;
    return round256((size_t) count * ext);
}

int MPIX_Allreduce(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
                   MPIX_Op op, MPIX_Comm comm, int algorithm, void *workspace,
                   size_t workspace_bytes)
{
    return allreduce_entry(sendbuf, recvbuf, count, datatype, op, comm, algorithm, workspace,
                           workspace_bytes,
                           comm ? (comm->stream ? comm->stream : comm->own_stream) : 0, true);
}

int MPIX_Allreduce_async(const void *sendbuf, void *recvbuf, MPIX_Aint count,
                         MPIX_Datatype datatype, MPIX_Op op, MPIX_Comm comm, int algorithm,
                         void *workspace, size_t workspace_bytes, void *stream)
{
    return allreduce_entry(sendbuf, recvbuf, count, datatype, op, comm, algorithm, workspace,
                           workspace_bytes, stream, false);
}

}  // extern "C"
