"""Island model across GPUs: one process per GPU (``torch.distributed`` for
rendezvous), demes resident on their rank's GPU, and ``migRing``
(``deap/tools/migration.py:4-51``) with the emigrant blocks exchanged
point-to-point over xGMI by RCCL from inside ``libdeapmi.so``.

The reference runs islands as processes exchanging pickled emigrants through
pipes (examples/ga/onemax_island.py:45-75) or as SCOOP tasks
(examples/ga/onemax_island_scoop.py:61-67).  Here a migration is:

1. every deme selects its k emigrants (a device selection operator, e.g.
   ``selBest``) and its immigrants (the emigrants themselves by default, or
   ``random.sample`` drawn on the device);
2. ``dm_mig_ring_rccl`` packs them into contiguous blocks (genomes, wvalues,
   valid), moves the blocks along ``migarray`` (default ring d -> d+1):
   same-rank hops are plain device references, cross-rank hops one grouped
   ``ncclSend``/``ncclRecv`` pair each (RCCL point-to-point), and
3. applies the reference's sequential value-equality placement on the
   receiver (``dm_mig_place``) — no second round trip.

The data path shards naturally (islands are independent between migrations),
so the only exchange is k*(G+F) bytes per deme per migration.  With a
non-RCCL backend (``gloo``, CPU tests) the same routing runs through
``torch.distributed`` batched P2P on host-staged blocks (:func:`route_blocks`).
"""
import ctypes

import torch
import torch.distributed as dist

from . import _lib
from .ops import resolve
from .tools.migration import pack, place, replacement_indices
from .device import zeros as _zeros


def migRingDistributed(demes, deme_ids, n_demes, k, selection, replacement=None,
                       migarray=None, *, stream=None, group=None, record=None,
                       force_p2p=False):
    """migRing over demes spread across ranks.

    ``demes``: the DevicePopulations held by this rank; ``deme_ids``: their
    global indices (0..n_demes-1), any split (every rank passes its own).
    ``record``: optional list; one dict per call is appended with this rank's
    host copies of the emigrant / immigrant row indices per local deme (what
    a replay in the oracle needs).  ``force_p2p`` routes hops between two
    local demes through RCCL as well (test hook: exercises the RCCL data path
    on one GPU)."""
    from .ops import default_stream
    stream = stream or default_stream()
    if migarray is None:
        migarray = list(range(1, n_demes)) + [0]
    if len(migarray) != n_demes:
        raise ValueError("migarray must have one entry per deme")
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    me = dist.get_rank(group) if dist.is_initialized() else 0
    owner = owner_map(deme_ids, n_demes, world, group)
    e_idx, i_idx = [], []
    for pop in demes:                                              # migration.py:39-46
        e_idx.append(_select(selection, pop, k, stream))
        i_idx.append(None if replacement is None
                     else replacement_indices(replacement, pop, k, stream))
    if record is not None:
        record.append({"ids": list(deme_ids),
                       "emigrants": [e.cpu().numpy().copy() for e in e_idx],
                       "immigrants": [None if i is None else i.cpu().numpy().copy()
                                      for i in i_idx]})
    if _uses_rccl(group) or (world == 1 and force_p2p):
        # every rank takes this route (the choice depends on the backend only)
        # and joins the communicator, a rank without demes included
        ctx = demes[0].ctx if demes else _current_ctx()
        comm = rccl_comm(ctx, group)
        _mig_ring_rccl(ctx, comm, demes, deme_ids, n_demes, migarray, owner, k, e_idx, i_idx,
                       force_p2p)
        return
    # host-staged route (gloo / CPU backends)
    emig, immig = {}, {}
    for d, pop, e, i in zip(deme_ids, demes, e_idx, i_idx):
        emig[d] = pack(pop, e)
        immig[d] = emig[d] if i is None else pack(pop, i)
    received = route_blocks(emig, lambda d: torch.empty_like(immig[d]), owner, migarray,
                            me, group)
    local = dict(zip(deme_ids, demes))
    for frm, to in enumerate(migarray):                            # migration.py:48-51
        if to in local and (frm, to) in received:
            place(local[to], immig[to], received[(frm, to)], k)


def _uses_rccl(group):
    """RCCL route iff the process group's backend is nccl (= RCCL on ROCm).
    Decided from the backend alone so that every rank — one that holds no
    deme included — takes the same route (the communicator set-up and the
    exchange are collective)."""
    return dist.is_initialized() and dist.get_backend(group) == "nccl"


def _current_ctx():
    from .device import Context
    return Context.get()


def route_blocks(emig, make_recv, owner, migarray, me, group=None):
    """Move emigrant blocks ``from_deme -> migarray[from_deme]`` with
    ``torch.distributed`` P2P (non-RCCL backends).

    ``emig``: this rank's {deme: block}; ``make_recv(d)`` allocates the receive
    buffer for local deme ``d``; ``owner``: global deme -> rank.  Same-rank
    hops are references; cross-rank hops are one isend/irecv pair each,
    issued as a single batched P2P group.  Device blocks are staged through
    host memory for backends without device P2P.  Returns {(from, to): block}
    for every hop into a local deme."""
    received, ops, staged = {}, [], []
    for frm, to in enumerate(migarray):
        src_rank, dst_rank = owner[frm], owner[to]
        if src_rank == me and dst_rank == me:
            received[(frm, to)] = emig[frm]
        elif src_rank == me:
            ops.append(dist.P2POp(dist.isend, _host(emig[frm]), dst_rank, group))
        elif dst_rank == me:
            buf = make_recv(to)
            hbuf = _host(buf)
            staged.append((buf, hbuf))
            received[(frm, to)] = buf
            ops.append(dist.P2POp(dist.irecv, hbuf, src_rank, group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    for buf, hbuf in staged:
        if hbuf is not buf:
            buf.copy_(hbuf)
    return received


def _host(t):
    return t if not t.is_cuda else t.cpu()


def _select(selection, pop, k, stream):
    op, a, kw = resolve(selection)
    return op(pop, k, *a, stream=stream, **kw)


_OWNERS = {}


def owner_map(deme_ids, n_demes, world, group):
    """Global deme -> rank, agreed by all ranks (one all_gather of the deme
    ids the first time a (group, split) is seen; any split is accepted as
    long as every deme has exactly one owner)."""
    if world == 1:
        if sorted(deme_ids) != list(range(n_demes)):
            raise ValueError("a single rank must hold every deme")
        return {d: 0 for d in range(n_demes)}
    key = (id(group), n_demes, tuple(deme_ids))
    if key in _OWNERS:
        return _OWNERS[key]
    parts = [None] * world
    dist.all_gather_object(parts, list(deme_ids), group=group)
    owner = {}
    for r, ids in enumerate(parts):
        for d in ids:
            if d in owner or not 0 <= d < n_demes:
                raise ValueError("deme %d owned twice or out of range" % d)
            owner[d] = r
    if len(owner) != n_demes:
        raise ValueError("demes %s have no owner" % sorted(set(range(n_demes)) - set(owner)))
    _OWNERS[key] = owner
    return owner


# ---------------------------------------------------------------------------
# RCCL communicator held by libdeapmi (dm_comm), one per (process group, device)
# ---------------------------------------------------------------------------
class RcclComm:
    """``dm_comm``: rank 0 draws the RCCL unique id, every rank receives it
    through a ``torch.distributed`` broadcast and joins with dm_comm_init."""

    def __init__(self, ctx, group=None):
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        lib = _lib.load()
        uid = (ctypes.c_uint8 * _lib.DM_COMM_ID_BYTES)()
        if rank == 0:
            _lib.check(lib.dm_comm_get_unique_id(uid), "dm_comm_get_unique_id")
        if world > 1:
            t = torch.tensor(list(uid), dtype=torch.uint8, device=ctx.device)
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast(t, src=src, group=group)
            for i, v in enumerate(t.cpu().tolist()):
                uid[i] = v
        self.handle = ctypes.c_void_p()
        _lib.check(lib.dm_comm_init(ctx.bind(), world, rank, uid, ctypes.byref(self.handle)),
                   "dm_comm_init")
        self.world, self.rank = world, rank

    def close(self):
        if self.handle:
            _lib.check(_lib.load().dm_comm_destroy(self.handle), "dm_comm_destroy")
            self.handle = ctypes.c_void_p()


_COMMS = {}


def rccl_comm(ctx, group=None):
    """The communicator of (process group, device), created on first use
    (collective: every rank of the group calls this in the same migration)."""
    key = (id(group), ctx.device.index, dist.is_initialized())
    c = _COMMS.get(key)
    if c is None:
        c = _COMMS[key] = RcclComm(ctx, group)
    return c


def close_comms():
    """Destroy every communicator this process created (before
    ``dist.destroy_process_group``)."""
    while _COMMS:
        _, c = _COMMS.popitem()
        c.close()


def _ptr_array(tensors):
    arr = (ctypes.c_void_p * max(len(tensors), 1))()
    for i, t in enumerate(tensors):
        arr[i] = None if t is None else t.data_ptr()
    return arr


def _mig_ring_rccl(ctx, comm, demes, deme_ids, n_demes, migarray, owner, k, e_idx, i_idx,
                   force_p2p):
    n_local = len(demes)
    pops = (_lib.DevicePop * max(n_local, 1))(*[p.c_pop() for p in demes])
    ids = (ctypes.c_int32 * max(n_local, 1))(*deme_ids)
    mig = (ctypes.c_int32 * n_demes)(*migarray)
    own = (ctypes.c_int32 * n_demes)(*[owner[d] for d in range(n_demes)])
    e_idx = [e.to(torch.int32).contiguous() for e in e_idx]
    i_idx = [None if i is None else i.to(torch.int32).contiguous() for i in i_idx]
    _lib.call("dm_mig_ring_rccl", ctx.bind(), comm.handle, n_local, pops, ids, n_demes, mig, own, int(k),
              _ptr_array(e_idx), _ptr_array(i_idx), None,
              _lib.DM_MIG_FORCE_P2P if force_p2p else 0)


def eaSimpleDemes(demes, toolbox, cxpb, mutpb, ngen, mig_every=5, *, deme_ids=None,
                  n_demes=None, streams=None, stats=None, halloffame=None, verbose=False,
                  mode=None, decisions=None, record=None, group=None, force_p2p=False,
                  callback=None):
    """The multi-demic GA loop of ``examples/ga/onemax_multidemic.py:79-93``
    on device demes, each deme's generation one fused launch
    (select -> clone -> varAnd -> evaluate, ``dm_generation``)::

        for gen in 1..ngen:
            for deme in demes:
                deme[:] = toolbox.select(deme, len(deme))
                deme[:] = varAnd(deme, toolbox, cxpb, mutpb)
                evaluate the invalid individuals
                logbook.record(gen=gen, deme=idx, evals=nevals, **stats.compile(deme))
                halloffame.update(deme)
            if gen % mig_every == 0:
                toolbox.migrate(demes)

    ``toolbox.migrate`` is a registration of ``tools.migRing`` (its ``k``,
    ``selection``, ``replacement``, ``migarray`` keywords are used); with
    ``deme_ids`` / ``n_demes`` the demes are this rank's share of a global
    ring and the migration runs through :func:`migRingDistributed` (RCCL).
    ``streams``: one RandomStream per deme (default: seeded from the deme id).
    ``decisions``: dict deme_id -> list (dump: filled per generation; inject:
    read).  ``record``: list receiving each migration's selected indices.
    ``callback(gen, stage, demes)`` (test hook) runs after every generation
    (stage "generation") and after every migration (stage "migration").
    Returns ``(demes, logbook)``; generation 0 evaluates invalid individuals."""
    from .algorithms import GenerationStep, _check_pop, _eval
    from .ops import RandomStream
    from .tools.support import Logbook
    for d in demes:
        _check_pop(d)
    deme_ids = list(range(len(demes))) if deme_ids is None else list(deme_ids)
    n_demes = len(demes) if n_demes is None else n_demes
    if streams is None:
        streams = [RandomStream(0, island=d) for d in deme_ids]
    mig_op, mig_a, mig_kw = resolve(toolbox.migrate)
    mig_kw = dict(mig_kw)
    for name, v in zip(("k", "selection", "replacement", "migarray"), mig_a):
        mig_kw[name] = v
    steps = [GenerationStep(d, toolbox, cxpb, mutpb) for d in demes]
    # a rank may hold no deme (any split, owner_map): it still joins every
    # migration, which is collective
    dev = demes[0].device if demes else torch.device("cuda", torch.cuda.current_device())
    nev = _zeros((len(demes), ngen + 1), torch.int64, dev)
    logbook = Logbook()
    logbook.header = ["gen", "deme", "evals"] + (stats.fields if stats else [])
    recs = []

    def book(gen, i, d):
        if halloffame is not None:
            halloffame.update(d)
        recs.append((gen, i, stats.compile(d) if stats else {}))

    for i, d in enumerate(demes):                         # onemax_multidemic.py:71-76
        ev = steps[i].ev
        _lib.call("dm_evaluate", d.ctx.bind(), ctypes.byref(d.c_pop()), ctypes.byref(ev), 1,
                  ctypes.c_void_p(nev[i].data_ptr()))
        book(0, deme_ids[i], d)
    offspring = [d.like(len(d), capacity=d.capacity) for d in demes]
    for gen in range(1, ngen + 1):
        for i, d in enumerate(demes):
            dec = None if decisions is None else decisions.setdefault(deme_ids[i], [])
            steps[i].step(d, offspring[i], streams[i],
                          ctypes.c_void_p(nev[i].data_ptr() + 8 * gen), mode, dec, gen - 1)
            d.swap_storage(offspring[i])
            book(gen, deme_ids[i], d)
        if callback is not None:
            callback(gen, "generation", demes)
        if mig_every and gen % mig_every == 0:
            if n_demes == len(demes) and group is None and not dist.is_initialized() \
                    and not force_p2p:
                mig_op(demes, stream=streams[0], record=record, **mig_kw)
            else:
                migRingDistributed(demes, deme_ids, n_demes,
                                   stream=streams[0] if streams else None, group=group,
                                   record=record, force_p2p=force_p2p, **mig_kw)
            if callback is not None:
                callback(gen, "migration", demes)
    counts = nev.cpu().tolist()
    pos = {d: i for i, d in enumerate(deme_ids)}
    from .algorithms import _materialise
    for gen, d, rec in recs:
        logbook.record(gen=gen, deme=d, evals=counts[pos[d]][gen], **_materialise(rec))
    if verbose:
        print(logbook.stream)
    return demes, logbook


def mig_plan(n_demes, migarray, owner, me, force_p2p=False):
    """The hops ``dm_mig_plan`` computes for rank ``me`` (host-only): a list of
    (kind, from, to, peer) with kind "local" / "send" / "recv"."""
    lib = _lib.load()
    mig = (ctypes.c_int32 * n_demes)(*(migarray if migarray is not None
                                       else list(range(1, n_demes)) + [0]))
    own = (ctypes.c_int32 * n_demes)(*[owner[d] for d in range(n_demes)])
    cap = 2 * n_demes
    hops = (_lib.MigHop * cap)()
    nh = ctypes.c_int32(0)
    _lib.check(lib.dm_mig_plan(n_demes, mig, own, me, _lib.DM_MIG_FORCE_P2P if force_p2p else 0,
                               hops, cap, ctypes.byref(nh)), "dm_mig_plan")
    names = {_lib.DM_HOP_LOCAL: "local", _lib.DM_HOP_SEND: "send", _lib.DM_HOP_RECV: "recv"}
    return [(names[h.kind], h.from_, h.to, h.peer) for h in hops[:nh.value]]


__all__ = ["migRingDistributed", "eaSimpleDemes", "route_blocks", "owner_map", "mig_plan",
           "RcclComm", "close_comms"]
