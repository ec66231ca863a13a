"""MPI_Reduce_scatter_block schedules over torch.distributed.

Restates MPIR_Reduce_scatter_block_intra_recursive_halving
(src/mpi/coll/reduce_scatter_block/reduce_scatter_block_intra_recursive_halving.c:38-260)
for one process per GPU:

  * the temporaries live in device memory (the reference mallocs them on the
    host, :80-88, and so reduces on the CPU even for device buffers);
  * the partial chunks move with torch.distributed point-to-point ops -- the
    "nccl" backend is RCCL on ROCm, so each step is one grouped
    ncclSend/ncclRecv pair over the xGMI link to the partner;
  * every received chunk is combined by the HIP kernel through the C-ABI
    (MPIX_Reduce_local_async on torch's current stream, which already waits
    for the receive), in the reference's operand order
    MPIR_Reduce_local(tmp_recvbuf, tmp_results) -- so the fp association, and
    therefore every bit, matches the CPU schedule.

`reduce_scatter_block_pairwise` restates
MPIR_Reduce_scatter_block_intra_pairwise (…_intra_pairwise.c:42-104),
MPICH's large-message choice (maint/tuning/coll/mpir/generic.json:324-328),
MI355X-first: the P-1 exchanges are posted as ONE group, so every xGMI link
of the node carries one block at the same time (the reference runs them as
P-1 sequential sendrecvs), and the P-1 received blocks are folded into the
result by one multi-input kernel pass in the reference's order i = 1..P-1
(same association as its P-1 MPIR_Reduce_local calls, so the same bits).

The combine can be injected (`combine=`) so the schedules themselves can be
exercised on CPU with the gloo backend; the default is the HIP path and
there is no CPU fallback.
"""
import os
import torch
import torch.distributed as dist

TAG = 0


def _pof2(n):
    p = 1
    while p * 2 <= n:
        p *= 2
    return p


def _default_combine(datatype, op):
    from . import redop

    def combine(inbuf, inoutbuf, count):
        redop.check(redop.reduce_local_async(inbuf, inoutbuf, count, datatype, op),
                    'MPIX_Reduce_local_async')
    return combine


# largest single message handed to the p2p layer: bigger ones go as several
# messages to the same peer in the same group (matched in posting order), so
# no count ever reaches 2^31 bytes inside the transport
MAX_MSG_BYTES = 1 << 30


def _p2p(fn, t, peer, group):
    """P2POps moving tensor `t` to/from `peer`, split at MAX_MSG_BYTES"""
    step = max(1, MAX_MSG_BYTES // t.element_size())
    flat = t.reshape(-1)
    return [dist.P2POp(fn, flat[k:k + step], peer, group=group, tag=TAG)
            for k in range(0, flat.numel(), step)]


def _exchange(send_t, dst_send, recv_t, src_recv, group):
    ops = []
    if send_t is not None:
        ops += _p2p(dist.isend, send_t, dst_send, group)
    if recv_t is not None:
        ops += _p2p(dist.irecv, recv_t, src_recv, group)
    if not ops:
        return
    for w in dist.batch_isend_irecv(ops):
        w.wait()


def plan(rank, comm_size, recvcount):
    """The per-step schedule of the reference for `rank`: a list of
    (peer, send_off, send_cnt, recv_off, recv_cnt) in elements, plus the
    non-power-of-two prologue/epilogue roles.  Pure index arithmetic
    (…recursive_halving.c:98-229)."""
    pof2 = _pof2(comm_size)
    rem = comm_size - pof2
    if rank < 2 * rem:
        newrank = -1 if rank % 2 == 0 else rank // 2
    else:
        newrank = rank - rem
    steps = []
    if newrank != -1:
        newcnts = []
        for i in range(pof2):
            old_i = i * 2 + 1 if i < rem else i + rem
            newcnts.append(2 * recvcount if old_i < 2 * rem else recvcount)
        newdisps = [0] * pof2
        for i in range(1, pof2):
            newdisps[i] = newdisps[i - 1] + newcnts[i - 1]
        mask = pof2 >> 1
        send_idx = recv_idx = 0
        last_idx = pof2
        while mask > 0:
            newdst = newrank ^ mask
            dst = newdst * 2 + 1 if newdst < rem else newdst + rem
            if newrank < newdst:
                send_idx = recv_idx + mask
                send_cnt = sum(newcnts[send_idx:last_idx])
                recv_cnt = sum(newcnts[recv_idx:send_idx])
            else:
                recv_idx = send_idx + mask
                send_cnt = sum(newcnts[send_idx:recv_idx])
                recv_cnt = sum(newcnts[recv_idx:last_idx])
            steps.append((dst, newdisps[send_idx], send_cnt, newdisps[recv_idx], recv_cnt))
            send_idx = recv_idx
            last_idx = recv_idx + mask
            mask >>= 1
    return dict(pof2=pof2, rem=rem, newrank=newrank, steps=steps)


class _StepTimer:
    """Per-step breakdown of a schedule: device events on
    the current stream around each exchange (the stream waits for the
    receive) and each combine; read with `.result()` after a synchronize."""

    def __init__(self, on_device):
        self.on = on_device
        self.marks = []

    def mark(self, tag):
        if self.on:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.marks.append((tag, e))

    def result(self):
        out = []
        for (t0, e0), (t1, e1) in zip(self.marks, self.marks[1:]):
            out.append(dict(phase=t1, ms=round(e0.elapsed_time(e1), 4)))
        return out


def reduce_scatter_block(sendbuf, recvbuf, recvcount, datatype, op, group=None, combine=None,
                         extent=None, workspace=None, timer=None):
    """MPI_Reduce_scatter_block(sendbuf, recvbuf, recvcount, datatype, op, comm).

    sendbuf: tensor holding comm_size*recvcount elements (any torch dtype;
    it is addressed as bytes); recvbuf: tensor of recvcount elements.
    sendbuf=None is MPI_IN_PLACE: recvbuf then holds the comm_size*recvcount
    input elements and receives the result in its first block (:91-96).  The
    op must be commutative (all predefined ops are; :62-67).
    workspace: optional (tmp_results, tmp_recvbuf) byte tensors to reuse.
    timer: optional list; a step timer is appended whose .result() is the
    per-step breakdown [{'phase': 'exchange k' | 'combine k' | ..., 'ms': t}]
    (device tensors only; read it after a torch.cuda.synchronize()).
    """
    rank = dist.get_rank(group)
    size = dist.get_world_size(group)
    if extent is None:
        from . import redop
        extent = redop.datatype_extent(datatype)
    if combine is None:
        combine = _default_combine(datatype, op)
    g2l = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    total = size * recvcount
    rb = recvbuf.reshape(-1).view(torch.uint8)
    sb = rb if sendbuf is None else sendbuf.reshape(-1).view(torch.uint8)
    if size == 1:
        if sendbuf is not None:
            rb[:recvcount * extent].copy_(sb[:recvcount * extent])
        return recvbuf
    if workspace is not None:
        tmp_results, tmp_recvbuf = workspace
        tmp_results = tmp_results[:total * extent]
        tmp_recvbuf = tmp_recvbuf[:total * extent]
    else:
        tmp_results = torch.empty(total * extent, dtype=torch.uint8, device=sb.device)
        tmp_recvbuf = torch.empty_like(tmp_results)
    tm = _StepTimer(timer is not None and sb.is_cuda)
    tm.mark('start')
    tmp_results.copy_(sb[:total * extent])                          # :91-96
    tm.mark('local copy')

    def el(off, cnt):
        return slice(off * extent, (off + cnt) * extent)

    p = plan(rank, size, recvcount)
    rem = p['rem']
    if rank < 2 * rem:                                              # :110-137
        if rank % 2 == 0:
            _exchange(tmp_results, g2l(rank + 1), None, None, group)
        else:
            _exchange(None, None, tmp_recvbuf, g2l(rank - 1), group)
            combine(tmp_recvbuf, tmp_results, total)
        tm.mark('prologue')
    for k, (dst, soff, scnt, roff, rcnt) in enumerate(p['steps']):  # :164-229
        _exchange(tmp_results[el(soff, scnt)] if scnt else None, g2l(dst),
                  tmp_recvbuf[el(roff, rcnt)] if rcnt else None, g2l(dst), group)
        tm.mark('exchange %d' % k)
        if rcnt:
            combine(tmp_recvbuf[el(roff, rcnt)], tmp_results[el(roff, rcnt)], rcnt)
        tm.mark('combine %d' % k)
    if p['newrank'] != -1:                                          # :232-234
        rb[:recvcount * extent].copy_(tmp_results[el(rank * recvcount, recvcount)])
    if rank < 2 * rem:                                              # :241-253
        if rank % 2:
            _exchange(tmp_results[el((rank - 1) * recvcount, recvcount)], g2l(rank - 1),
                      None, None, group)
        else:
            _exchange(None, None, rb[:recvcount * extent], g2l(rank + 1), group)
    tm.mark('epilogue')
    if timer is not None:
        timer.append(tm)
    return recvbuf


def reduce_scatter_block_pairwise(sendbuf, recvbuf, recvcount, datatype, op, group=None,
                                  combine=None, extent=None, workspace=None, concurrent=True):
    """MPI_Reduce_scatter_block, pairwise exchange (reference algorithm
    `pairwise`).  workspace: optional byte tensor of >= (P-1) * (block bytes
    rounded up to 256) for the received blocks.  sendbuf=None is
    MPI_IN_PLACE: blocks are sent from recvbuf, the own block is reduced in
    place and moved to the front at the end (:58-64, :71-110)."""
    rank = dist.get_rank(group)
    size = dist.get_world_size(group)
    if extent is None:
        from . import redop
        extent = redop.datatype_extent(datatype)
    g2l = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    rb = recvbuf.reshape(-1).view(torch.uint8)
    in_place = sendbuf is None
    sb = rb if in_place else sendbuf.reshape(-1).view(torch.uint8)
    blk = recvcount * extent

    def block(i):
        return slice(i * blk, (i + 1) * blk)

    acc = rb[block(rank)] if in_place else rb[:blk]         # where the result accumulates
    if not in_place:
        rb[:blk].copy_(sb[block(rank)])                             # :60-64
    if size == 1:
        return recvbuf
    nslot = size - 1 if concurrent else 1
    # slots start on 256-byte boundaries so every received block has the same
    # 16-byte phase as the result and takes the packet kernel
    sstride = (blk + 255) // 256 * 256
    if workspace is not None:
        slots = workspace[:nslot * sstride]
    else:
        slots = torch.empty(nslot * sstride, dtype=torch.uint8, device=sb.device)

    def slot(i):
        return slots[i * sstride:i * sstride + blk]
    peers = [((rank + i) % size, (rank - i + size) % size) for i in range(1, size)]
    def finish():
        if in_place and rank != 0:      # :102-110: the result moves to the front
            rb[:blk].copy_(acc)
        return recvbuf
    if not concurrent:                                              # the reference's loop
        for dst, src in peers:
            _exchange(sb[block(dst)], g2l(dst), slot(0), g2l(src), group)
            if combine is not None:
                combine(slot(0), acc, recvcount)
            else:
                _default_combine(datatype, op)(slot(0), acc, recvcount)
        return finish()
    ops = []
    for i, (dst, src) in enumerate(peers):
        ops += _p2p(dist.isend, sb[block(dst)], g2l(dst), group)
        ops += _p2p(dist.irecv, slot(i), g2l(src), group)
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    ins = [slot(i) for i in range(size - 1)]
    if combine is not None:
        for x in ins:                                               # :86-100, i = 1..P-1
            combine(x, acc, recvcount)
    else:
        from . import redop
        for lo in range(0, len(ins), 16):
            redop.check(redop.reduce_local_multi_async(ins[lo:lo + 16], acc, recvcount,
                                                       datatype, op),
                        'MPIX_Reduce_local_multi_async')
    return finish()


ALGORITHMS = {'recursive_halving': reduce_scatter_block, 'pairwise': reduce_scatter_block_pairwise}


def reduce_scatter_block_auto(sendbuf, recvbuf, recvcount, datatype, op, group=None, **kw):
    """Algorithm selection mirroring MPIR_CVAR_REDUCE_SCATTER_BLOCK_INTRA_ALGORITHM
    (cvars.txt:1712-1726): env value `recursive_halving` or `pairwise`;
    `auto` follows generic.json:316-341 (recursive halving below 512 KiB per
    rank, pairwise above)."""
    algo = os.environ.get('MPIR_CVAR_REDUCE_SCATTER_BLOCK_INTRA_ALGORITHM', 'auto')
    if algo not in ALGORITHMS:
        ext = kw.get('extent')
        if ext is None:
            from . import redop
            ext = redop.datatype_extent(datatype)
        total = recvcount * ext * dist.get_world_size(group)
        algo = 'recursive_halving' if total < (512 << 10) else 'pairwise'
    return ALGORITHMS[algo](sendbuf, recvbuf, recvcount, datatype, op, group=group, **kw)


def _bitrev(r, pof2):
    """Block a rank owns after the distance-doubling reduce-scatter of
    MPIR_Allreduce_intra_reduce_scatter_allgather (:138-189): recv_idx ends at
    the bit reversal of newrank over log2(pof2) bits."""
    out, b = 0, pof2 >> 1
    while b:
        out = (out << 1) | (r & 1)
        r >>= 1
        b >>= 1
    return out


def allreduce(sendbuf, recvbuf, count, datatype, op, group=None, combine=None, extent=None,
              workspace=None, allgather='direct'):
    """MPI_Allreduce by reduce-scatter + allgather (Rabenseifner):
    MPIR_Allreduce_intra_reduce_scatter_allgather
    (src/mpi/coll/allreduce/allreduce_intra_reduce_scatter_allgather.c:41-277),
    MPICH's choice for builtin ops with count >= pof2 (generic.json:99-135).
    Device buffers; RCCL point-to-point transport; every partial is combined
    by the HIP kernel in the reference's order, so results are bit-identical
    to the reference schedule -- unlike ncclAllReduce (rccl.c:223), whose
    association is RCCL's own and whose op set stops at SUM/PROD/MIN/MAX.
    sendbuf=None means MPI_IN_PLACE (recvbuf holds the input).

    allgather: 'recursive_doubling' is the reference's second phase
    (:191-226, log2(P) sequential exchanges, one link busy per step);
    'direct' (default) posts the same final blocks as ONE group of P-1 sends
    and P-1 receives, so every xGMI link carries one block at once.  The
    allgather only moves finished bytes, so both give the same bits."""
    if allgather not in ('direct', 'recursive_doubling'):
        raise ValueError('allgather must be direct or recursive_doubling')
    rank = dist.get_rank(group)
    size = dist.get_world_size(group)
    if extent is None:
        from . import redop
        extent = redop.datatype_extent(datatype)
    if combine is None:
        combine = _default_combine(datatype, op)
    g2l = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    rb = recvbuf.reshape(-1).view(torch.uint8)
    if sendbuf is not None:
        rb[:count * extent].copy_(sendbuf.reshape(-1).view(torch.uint8)[:count * extent])
    if size == 1 or count == 0:
        return recvbuf
    pof2 = _pof2(size)
    rem = size - pof2
    if count < pof2:
        raise ValueError('reduce_scatter_allgather allreduce needs count >= pof2 (:127); '
                         'the reference uses recursive doubling below that')
    tmp = workspace[:count * extent] if workspace is not None else \
        torch.empty(count * extent, dtype=torch.uint8, device=rb.device)

    def el(off, cnt):
        return slice(off * extent, (off + cnt) * extent)

    if rank < 2 * rem:                                              # :85-112
        if rank % 2 == 0:
            _exchange(rb[:count * extent], g2l(rank + 1), None, None, group)
            newrank = -1
        else:
            _exchange(None, None, tmp, g2l(rank - 1), group)
            combine(tmp, rb[:count * extent], count)
            newrank = rank // 2
    else:
        newrank = rank - rem
    if newrank != -1:
        cnts = [count // pof2 + (1 if i < count % pof2 else 0) for i in range(pof2)]
        disps = [0] * pof2
        for i in range(1, pof2):
            disps[i] = disps[i - 1] + cnts[i - 1]

        def real(nr):
            return nr * 2 + 1 if nr < rem else nr + rem
        mask, send_idx, recv_idx, last_idx = 1, 0, 0, pof2
        while mask < pof2:                                          # :138-189
            newdst = newrank ^ mask
            if newrank < newdst:
                send_idx = recv_idx + pof2 // (mask * 2)
                send_cnt, recv_cnt = sum(cnts[send_idx:last_idx]), sum(cnts[recv_idx:send_idx])
            else:
                recv_idx = send_idx + pof2 // (mask * 2)
                send_cnt, recv_cnt = sum(cnts[send_idx:recv_idx]), sum(cnts[recv_idx:last_idx])
            _exchange(rb[el(disps[send_idx], send_cnt)], g2l(real(newdst)),
                      tmp[el(disps[recv_idx], recv_cnt)], g2l(real(newdst)), group)
            combine(tmp[el(disps[recv_idx], recv_cnt)], rb[el(disps[recv_idx], recv_cnt)],
                    recv_cnt)
            send_idx = recv_idx
            mask <<= 1
            if mask < pof2:
                last_idx = recv_idx + pof2 // mask
        mask >>= 1
        if allgather == 'direct':
            mine = _bitrev(newrank, pof2)
            ops = []
            for q in range(pof2):
                if q == newrank:
                    continue
                b = _bitrev(q, pof2)
                ops += _p2p(dist.isend, rb[el(disps[mine], cnts[mine])], g2l(real(q)), group)
                ops += _p2p(dist.irecv, rb[el(disps[b], cnts[b])], g2l(real(q)), group)
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            mask = 0
        while mask > 0:                                             # :191-226
            newdst = newrank ^ mask
            if newrank < newdst:
                if mask != pof2 // 2:
                    last_idx = last_idx + pof2 // (mask * 2)
                recv_idx = send_idx + pof2 // (mask * 2)
                send_cnt, recv_cnt = sum(cnts[send_idx:recv_idx]), sum(cnts[recv_idx:last_idx])
            else:
                recv_idx = send_idx - pof2 // (mask * 2)
                send_cnt, recv_cnt = sum(cnts[send_idx:last_idx]), sum(cnts[recv_idx:send_idx])
            _exchange(rb[el(disps[send_idx], send_cnt)], g2l(real(newdst)),
                      rb[el(disps[recv_idx], recv_cnt)], g2l(real(newdst)), group)
            if newrank > newdst:
                send_idx = recv_idx
            mask >>= 1
    if rank < 2 * rem:                                              # :229-238
        if rank % 2:
            _exchange(rb[:count * extent], g2l(rank - 1), None, None, group)
        else:
            _exchange(None, None, rb[:count * extent], g2l(rank + 1), group)
    return recvbuf


_ipc_cache = {}


def ipc_cache_clear():
    """Unmap every cached peer allocation (call before peers free buffers
    that were used with reduce_scatter_block_pull)."""
    from . import redop
    for base in _ipc_cache.values():
        redop.ipc_close(base)
    _ipc_cache.clear()


def _sync_barrier(group):
    torch.cuda.synchronize()
    dist.barrier(group=group)


def reduce_scatter_block_pull(sendbuf, recvbuf, recvcount, datatype, op, group=None,
                              extent=None):
    """MPI_Reduce_scatter_block as ONE fused pull + combine kernel
    (SURVEY.md §8(f)2): every rank maps its peers' send buffers
    (hipIpc*, as MPICH's ipc/gpu shm path does, mpl_gpu_hip.c:174-204) and a
    single multi-input kernel reads block `rank` of all P-1 peers directly
    over xGMI -- all links at once, no receive buffer, no copy -- folding them
    into the result in the pairwise order i = 1..P-1
    (…_intra_pairwise.c:86-100), i.e. bit-identical to the reference pairwise
    schedule.  Peer mappings are cached (ipc_cache_clear() drops them).
    Costs two barriers per call: peers' inputs must be complete before the
    pull and must stay untouched until every rank has pulled."""
    from . import redop
    rank = dist.get_rank(group)
    size = dist.get_world_size(group)
    if extent is None:
        extent = redop.datatype_extent(datatype)
    rb = recvbuf.reshape(-1).view(torch.uint8)
    in_place = sendbuf is None      # MPI_IN_PLACE: peers pull from recvbuf, own block reduced there
    sb = rb if in_place else sendbuf.reshape(-1).view(torch.uint8)
    blk = recvcount * extent
    acc = rb[rank * blk:(rank + 1) * blk] if in_place else rb[:blk]
    if not in_place:
        rb[:blk].copy_(sb[rank * blk:(rank + 1) * blk])
    if size == 1:
        return recvbuf
    handle, off = redop.ipc_export(sb)
    infos = [None] * size
    dist.all_gather_object(infos, (handle, off), group=group)
    bases = []
    for r, (h, o) in enumerate(infos):
        if r == rank:
            bases.append(sb.data_ptr())
            continue
        key = (r, h)
        if key not in _ipc_cache:
            _ipc_cache[key] = redop.ipc_open(h)
        bases.append(_ipc_cache[key] + o)
    _sync_barrier(group)                        # every peer's sendbuf is complete
    ins = [bases[(rank - i + size) % size] + rank * blk for i in range(1, size)]
    for lo in range(0, len(ins), 16):
        redop.check(redop.reduce_local_multi_async(ins[lo:lo + 16], acc, recvcount,
                                                   datatype, op), 'MPIX_Reduce_local_multi_async')
    _sync_barrier(group)                        # nobody reuses sendbuf while peers read it
    if in_place and rank != 0:
        rb[:blk].copy_(acc)
    return recvbuf


ALGORITHMS['pull'] = reduce_scatter_block_pull


def allreduce_recursive_doubling(sendbuf, recvbuf, count, datatype, op, group=None, combine=None,
                                 extent=None, workspace=None):
    """MPIR_Allreduce_intra_recursive_doubling
    (src/mpi/coll/allreduce/allreduce_intra_recursive_doubling.c:24-150) for
    the predefined (commutative) ops: log2(P) full-vector exchanges, each
    folded in with MPIR_Reduce_local(tmp_buf, recvbuf).  Used below pof2
    elements, where the reduce-scatter schedule cannot split the vector."""
    rank = dist.get_rank(group)
    size = dist.get_world_size(group)
    if extent is None:
        from . import redop
        extent = redop.datatype_extent(datatype)
    if combine is None:
        combine = _default_combine(datatype, op)
    g2l = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    rb = recvbuf.reshape(-1).view(torch.uint8)
    nb = count * extent
    if sendbuf is not None:
        rb[:nb].copy_(sendbuf.reshape(-1).view(torch.uint8)[:nb])
    if size == 1 or count == 0:
        return recvbuf
    pof2 = _pof2(size)
    rem = size - pof2
    tmp = workspace[:nb] if workspace is not None else \
        torch.empty(nb, dtype=torch.uint8, device=rb.device)
    if rank < 2 * rem:                                              # :59-86
        if rank % 2 == 0:
            _exchange(rb[:nb], g2l(rank + 1), None, None, group)
            newrank = -1
        else:
            _exchange(None, None, tmp, g2l(rank - 1), group)
            combine(tmp, rb[:nb], count)
            newrank = rank // 2
    else:
        newrank = rank - rem
    if newrank != -1:
        mask = 1
        while mask < pof2:                                          # :97-129
            newdst = newrank ^ mask
            dst = newdst * 2 + 1 if newdst < rem else newdst + rem
            _exchange(rb[:nb], g2l(dst), tmp, g2l(dst), group)
            combine(tmp, rb[:nb], count)
            mask <<= 1
    if rank < 2 * rem:                                              # :131-141
        if rank % 2:
            _exchange(rb[:nb], g2l(rank - 1), None, None, group)
        else:
            _exchange(None, None, rb[:nb], g2l(rank + 1), group)
    return recvbuf


def allreduce_auto(sendbuf, recvbuf, count, datatype, op, group=None, **kw):
    """MPI_Allreduce algorithm choice: MPIR_CVAR_ALLREDUCE_INTRA_ALGORITHM
    (`recursive_doubling` | `reduce_scatter_allgather`) or, by default,
    generic.json:99-135 for builtin ops: recursive doubling up to 8 bytes of
    message or below pof2 elements (the reduce-scatter needs count >= pof2,
    :127), the reduce-scatter + allgather schedule otherwise."""
    algo = os.environ.get('MPIR_CVAR_ALLREDUCE_INTRA_ALGORITHM', 'auto')
    if algo not in ('recursive_doubling', 'reduce_scatter_allgather'):
        ext = kw.get('extent')
        if ext is None:
            from . import redop
            ext = redop.datatype_extent(datatype)
        algo = 'reduce_scatter_allgather' \
            if count * ext > 8 and count >= _pof2(dist.get_world_size(group)) \
            else 'recursive_doubling'
    fn = allreduce if algo == 'reduce_scatter_allgather' else allreduce_recursive_doubling
    return fn(sendbuf, recvbuf, count, datatype, op, group=group, **kw)
