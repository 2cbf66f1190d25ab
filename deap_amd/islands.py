"""Island model across GPUs: one process per GPU (``torch.distributed``,
backend "nccl" = RCCL on ROCm), demes resident on their rank's GPU, and
``migRing`` (``deap/tools/migration.py:4-51``) with the emigrant blocks
exchanged point-to-point over xGMI.

The reference runs islands as processes exchanging pickled emigrants through
pipes (examples/ga/onemax_island.py:45-75) or as SCOOP tasks
(examples/ga/onemax_island_scoop.py:61-67).  Here a migration is:

1. every deme selects its k emigrants (device ``selBest``) and its immigrants
   (the emigrants themselves by default) and packs them into one contiguous
   block (``dm_pack_rows``: genomes, wvalues, valid);
2. blocks move along ``migarray`` (default ring d -> d+1): same-rank hops are
   plain device references, cross-rank hops are one ``isend``/``irecv`` pair
   per hop in a single batched P2P group (RCCL point-to-point);
3. each receiving deme applies the reference's sequential value-equality
   placement locally (``dm_mig_place``) — no second round trip.

The data path shards naturally (islands are independent between migrations),
so the only collective traffic is k*(G+F) bytes per deme per migration.
"""
import torch
import torch.distributed as dist

from .ops import resolve
from .tools.migration import pack, place, replacement_indices


def migRingDistributed(demes, deme_ids, n_demes, k, selection, replacement=None,
                       migarray=None, *, stream=None, group=None):
    """migRing over demes spread across ranks.

    ``demes``: the DevicePopulations owned by this rank; ``deme_ids``: their
    global indices (0..n_demes-1); every rank must own the demes
    ``rank * per_rank ... (rank+1) * per_rank - 1`` of an even split (or pass
    explicit ids consistently on all ranks).  Works with any backend whose
    P2P supports the tensors' device (nccl for GPU tensors, gloo for CPU)."""
    from .ops import default_stream
    stream = stream or default_stream()
    if migarray is None:
        migarray = list(range(1, n_demes)) + [0]
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    owner = owner_map(deme_ids, n_demes, world, group)
    local = dict(zip(deme_ids, demes))
    emig, immig = {}, {}
    for d, pop in local.items():
        e_idx = _select(selection, pop, k, stream)
        emig[d] = pack(pop, e_idx)
        if replacement is None:
            immig[d] = emig[d]
        else:
            immig[d] = pack(pop, replacement_indices(replacement, pop, k, stream))
    me = dist.get_rank(group) if dist.is_initialized() else 0
    received = route_blocks(emig, lambda d: torch.empty_like(immig[d]), owner, migarray,
                            me, group)
    for d, pop in local.items():
        place(pop, immig[d], received[d], k)


def route_blocks(emig, make_recv, owner, migarray, me, group=None):
    """Move emigrant blocks ``from_deme -> migarray[from_deme]``.

    ``emig``: this rank's {deme: block}; ``make_recv(d)`` allocates the receive
    buffer for local deme ``d``; ``owner``: global deme -> rank.  Same-rank
    hops are device references; cross-rank hops are one isend/irecv pair each,
    issued as a single batched P2P group (RCCL groupStart/groupEnd).  Returns
    {local deme: received block}."""
    received, ops = {}, []
    for frm, to in enumerate(migarray):
        src_rank, dst_rank = owner[frm], owner[to]
        if src_rank == me and dst_rank == me:
            received[to] = emig[frm]
        elif src_rank == me:
            ops.append(dist.P2POp(dist.isend, emig[frm], dst_rank, group))
        elif dst_rank == me:
            buf = make_recv(to)
            received[to] = buf
            ops.append(dist.P2POp(dist.irecv, buf, src_rank, group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return received


def _select(selection, pop, k, stream):
    op, a, kw = resolve(selection)
    return op(pop, k, *a, stream=stream, **kw)


def owner_map(deme_ids, n_demes, world, group):
    """Global deme -> rank, agreed by all ranks."""
    if world == 1:
        return {d: 0 for d in range(n_demes)}
    me = dist.get_rank(group)
    # ownership follows from the even contiguous split every rank agrees on
    per = n_demes // world
    if per * world == n_demes and list(deme_ids) == list(range(me * per, (me + 1) * per)):
        return {d: d // per for d in range(n_demes)}
    raise ValueError("demes must be split evenly and contiguously across ranks")


__all__ = ["migRingDistributed", "route_blocks", "owner_map"]
