// vmm_ipc_probe.cpp -- P processes on one GPU share device memory each round,
// two ways, and check what every peer's mapping really shows:
//   ipc  hipMalloc + hipIpcGetMemHandle, handle bytes sent to the peers,
//        hipIpcOpenMemHandle (the pull windows' mechanism)
//   vmm  hipMemCreate (POSIX-fd shareable) + hipMemExportToShareableHandle,
//        the descriptor itself passed to the peers over a unix socket
//        (SCM_RIGHTS), hipMemImportFromShareableHandle + hipMemMap
// Each allocation's first 16 bytes hold a random nonce that travels with the
// handle; a peer reading another nonce has mapped the wrong memory.  Every
// round makes new allocations of the same size in every process (the
// lock-step pattern of a growing pull window); the old ones stay allocated
// (mode keep) or are freed (mode free); peers' mappings are closed after the
// check.  The parent never touches HIP; children initialise it after fork.
// Build: hipcc -O2 -std=c++17 -o tools/bin/vmm_ipc_probe tools/vmm_ipc_probe.cpp
// Usage: vmm_ipc_probe [P=4] [rounds=8] [MiB=512] [keep|free]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "rank %d %s:%d %s\n", rank, __FILE__, __LINE__, hipGetErrorString(e_)); \
    _exit(2); } } while (0)

struct Msg {
    int from;
    int kind;               // 0 ipc, 1 vmm
    uint64_t nonce[2];
    hipIpcMemHandle_t h;
};

static int send_msg(int sock, const Msg &m, int fd)
{
    struct iovec io = {(void *) &m, sizeof m};
    char ctrl[CMSG_SPACE(sizeof(int))];
    struct msghdr mh;
    memset(&mh, 0, sizeof mh);
    mh.msg_iov = &io;
    mh.msg_iovlen = 1;
    if (fd >= 0) {
        memset(ctrl, 0, sizeof ctrl);
        mh.msg_control = ctrl;
        mh.msg_controllen = sizeof ctrl;
        struct cmsghdr *c = CMSG_FIRSTHDR(&mh);
        c->cmsg_level = SOL_SOCKET;
        c->cmsg_type = SCM_RIGHTS;
        c->cmsg_len = CMSG_LEN(sizeof(int));
        memcpy(CMSG_DATA(c), &fd, sizeof fd);
    }
    return sendmsg(sock, &mh, 0) == (ssize_t) sizeof m ? 0 : -1;
}

static int recv_msg(int sock, Msg *m, int *fd)
{
    struct iovec io = {(void *) m, sizeof *m};
    char ctrl[CMSG_SPACE(sizeof(int))];
    struct msghdr mh;
    memset(&mh, 0, sizeof mh);
    mh.msg_iov = &io;
    mh.msg_iovlen = 1;
    mh.msg_control = ctrl;
    mh.msg_controllen = sizeof ctrl;
    *fd = -1;
    if (recvmsg(sock, &mh, MSG_WAITALL) != (ssize_t) sizeof *m)
        return -1;
    for (struct cmsghdr *c = CMSG_FIRSTHDR(&mh); c; c = CMSG_NXTHDR(&mh, c))
        if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_RIGHTS)
            memcpy(fd, CMSG_DATA(c), sizeof *fd);
    return 0;
}

static int child(int rank, int P, int rounds, size_t bytes, bool keep, const std::vector<int> &socks)
{
    CK(hipSetDevice(0));
    std::random_device rd;
    hipMemAllocationProp prop;
    memset(&prop, 0, sizeof prop);
    prop.type = hipMemAllocationTypePinned;
    prop.requestedHandleTypes = hipMemHandleTypePosixFileDescriptor;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    const size_t sz = (bytes + gran - 1) / gran * gran;
    hipMemAccessDesc acc;
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    int ipc_bad = 0, vmm_bad = 0, ipc_err = 0, vmm_err = 0;
    std::vector<void *> old_ipc;
    std::vector<std::pair<void *, hipMemGenericAllocationHandle_t>> old_vmm;
    for (int r = 0; r < rounds; ++r) {
        // ipc
        void *p = nullptr;
        CK(hipMalloc(&p, bytes));
        Msg mi;
        memset(&mi, 0, sizeof mi);
        mi.from = rank;
        mi.kind = 0;
        mi.nonce[0] = ((uint64_t) rd() << 32) ^ rd();
        mi.nonce[1] = ((uint64_t) rd() << 32) ^ rd() ^ (uint64_t) r;
        CK(hipMemcpy(p, mi.nonce, 16, hipMemcpyHostToDevice));
        CK(hipIpcGetMemHandle(&mi.h, p));
        // vmm
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, sz, &prop, 0));
        void *va = nullptr;
        CK(hipMemAddressReserve(&va, sz, gran, nullptr, 0));
        CK(hipMemMap(va, sz, 0, h, 0));
        CK(hipMemSetAccess(va, sz, &acc, 1));
        Msg mv;
        memset(&mv, 0, sizeof mv);
        mv.from = rank;
        mv.kind = 1;
        mv.nonce[0] = ((uint64_t) rd() << 32) ^ rd();
        mv.nonce[1] = ((uint64_t) rd() << 32) ^ rd() ^ (uint64_t) r;
        CK(hipMemcpy(va, mv.nonce, 16, hipMemcpyHostToDevice));
        int fd = -1;
        CK(hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0));
        for (int q = 0; q < P; ++q)
            if (q != rank && (send_msg(socks[q], mi, -1) || send_msg(socks[q], mv, fd))) {
                fprintf(stderr, "rank %d: send to %d failed\n", rank, q);
                _exit(3);
            }
        close(fd);
        std::vector<void *> maps;
        std::vector<std::pair<void *, hipMemGenericAllocationHandle_t>> vmaps;
        for (int q = 0; q < P; ++q) {
            if (q == rank)
                continue;
            for (int k = 0; k < 2; ++k) {
                Msg m;
                int rfd;
                if (recv_msg(socks[q], &m, &rfd) || m.from != q) {
                    fprintf(stderr, "rank %d: recv from %d failed\n", rank, q);
                    _exit(3);
                }
                uint64_t seen[2] = {0, 0};
                if (m.kind == 0) {
                    void *mp = nullptr;
                    if (hipIpcOpenMemHandle(&mp, m.h, hipIpcMemLazyEnablePeerAccess) != hipSuccess ||
                        hipMemcpy(seen, mp, 16, hipMemcpyDeviceToHost) != hipSuccess) {
                        ++ipc_err;
                        (void) hipGetLastError();
                    } else if (seen[0] != m.nonce[0] || seen[1] != m.nonce[1]) {
                        ++ipc_bad;
                    }
                    if (mp)
                        maps.push_back(mp);
                } else {
                    hipMemGenericAllocationHandle_t ih;
                    void *iva = nullptr;
                    if (hipMemImportFromShareableHandle(&ih, (void *) (intptr_t) rfd,
                                                        hipMemHandleTypePosixFileDescriptor) != hipSuccess ||
                        hipMemAddressReserve(&iva, sz, gran, nullptr, 0) != hipSuccess ||
                        hipMemMap(iva, sz, 0, ih, 0) != hipSuccess ||
                        hipMemSetAccess(iva, sz, &acc, 1) != hipSuccess ||
                        hipMemcpy(seen, iva, 16, hipMemcpyDeviceToHost) != hipSuccess) {
                        ++vmm_err;
                        (void) hipGetLastError();
                    } else {
                        if (seen[0] != m.nonce[0] || seen[1] != m.nonce[1])
                            ++vmm_bad;
                        vmaps.push_back({iva, ih});
                    }
                    if (rfd >= 0)
                        close(rfd);
                }
            }
        }
        // peers done reading: a byte each way
        for (int q = 0; q < P; ++q)
            if (q != rank) {
                char b = 1;
                if (write(socks[q], &b, 1) != 1)
                    _exit(3);
            }
        for (int q = 0; q < P; ++q)
            if (q != rank) {
                char b;
                if (read(socks[q], &b, 1) != 1)
                    _exit(3);
            }
        for (void *mp : maps)
            (void) hipIpcCloseMemHandle(mp);
        for (auto &v : vmaps) {
            (void) hipMemUnmap(v.first, sz);
            (void) hipMemAddressFree(v.first, sz);
            (void) hipMemRelease(v.second);
        }
        if (keep) {
            old_ipc.push_back(p);
            old_vmm.push_back({va, h});
        } else {
            CK(hipFree(p));
            CK(hipMemUnmap(va, sz));
            CK(hipMemAddressFree(va, sz));
            CK(hipMemRelease(h));
        }
    }
    printf("{\"rank\": %d, \"rounds\": %d, \"reads\": %d, \"ipc_wrong\": %d, \"ipc_errors\": %d, "
           "\"vmm_wrong\": %d, \"vmm_errors\": %d}\n", rank, rounds, rounds * (P - 1), ipc_bad,
           ipc_err, vmm_bad, vmm_err);
    fflush(stdout);
    return 0;
}

int main(int argc, char **argv)
{
    const int P = argc > 1 ? atoi(argv[1]) : 4;
    const int rounds = argc > 2 ? atoi(argv[2]) : 8;
    const size_t bytes = (size_t) (argc > 3 ? atoi(argv[3]) : 512) << 20;
    const bool keep = !(argc > 4 && strcmp(argv[4], "free") == 0);
    if (P < 2 || P > 16)
        return 1;
    // socks[i][j]: rank i's end of the pair (i, j)
    std::vector<std::vector<int>> socks(P, std::vector<int>(P, -1));
    for (int i = 0; i < P; ++i)
        for (int j = i + 1; j < P; ++j) {
            int sv[2];
            if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv))
                return 1;
            socks[i][j] = sv[0];
            socks[j][i] = sv[1];
        }
    std::vector<pid_t> kids;
    for (int r = 0; r < P; ++r) {
        pid_t pid = fork();
        if (pid == 0) {
            const int rank = r;
            (void) rank;
            _exit(child(r, P, rounds, bytes, keep, socks[r]));
        }
        kids.push_back(pid);
    }
    int rc = 0;
    for (pid_t k : kids) {
        int st = 0;
        waitpid(k, &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st))
            rc = 1;
    }
    return rc;
}
