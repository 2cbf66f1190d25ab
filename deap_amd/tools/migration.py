"""Ring migration between demes (``deap/tools/migration.py:4-51``).

``migRing(populations, k, selection, replacement=None, migarray=None)`` works
in place on a list of :class:`DevicePopulation` demes on one GPU; the
multi-GPU form (one or more demes per rank, emigrants exchanged with RCCL
point-to-point over xGMI) is :func:`deap_amd.islands.migRingDistributed`.

Semantics kept from the reference: all emigrants are selected before any
placement; immigrants default to the emigrants themselves; for each
``from_deme`` in order, every immigrant ``j`` is located in the *current*
destination deme by value equality (``list.index``) and that slot receives
emigrant ``j`` — so a second equal-valued immigrant can re-hit the slot just
filled by an equal emigrant, exactly like the reference.
"""
import ctypes

from .. import _lib
from ..ops import DeviceOperator, default_stream


def _torch():
    import torch
    return torch


def pack(pop, idx):
    """Pack rows ``idx`` of ``pop`` into one contiguous block (genomes,
    wvalues, valid) — the unit sent between ranks."""
    torch = _torch()
    k = int(idx.numel())
    nbytes = _lib.load().dm_pack_bytes(ctypes.byref(pop.c_pop()), k)
    block = torch.empty((max(int(nbytes), 16),), dtype=torch.uint8, device=pop.device)
    if k:
        ctx = pop.ctx.bind()
        _lib.call("dm_pack_rows", ctx, ctypes.byref(pop.c_pop()),
                  ctypes.c_void_p(idx.data_ptr()), k, ctypes.c_void_p(block.data_ptr()))
    return block


def place(pop, immigrant_block, emigrant_block, k):
    """Sequential first-match placement into one receiving deme
    (``migration.py:48-51``).  Returns the slots written (device int32)."""
    torch = _torch()
    slots = torch.empty((max(k, 1),), dtype=torch.int32, device=pop.device)
    if k:
        ctx = pop.ctx.bind()
        _lib.call("dm_mig_place", ctx, ctypes.byref(pop.c_pop()),
                  ctypes.c_void_p(immigrant_block.data_ptr()),
                  ctypes.c_void_p(emigrant_block.data_ptr()), int(k),
                  ctypes.c_void_p(slots.data_ptr()))
    return slots[:k]


def select_indices(selection, pop, k, stream):
    from ..ops import resolve
    op, a, kw = resolve(selection)
    return op(pop, k, *a, stream=stream, **kw)


class _MigRing(DeviceOperator):
    kind = "migrate"

    def __call__(self, populations, k, selection, replacement=None, migarray=None, *,
                 stream=None):
        stream = stream or default_stream()
        nbr_demes = len(populations)
        if migarray is None:
            migarray = list(range(1, nbr_demes)) + [0]
        emigrants, immigrants = [], []
        for deme in populations:                                   # migration.py:39-46
            e_idx = select_indices(selection, deme, k, stream)
            emigrants.append(pack(deme, e_idx))
            if replacement is None:
                immigrants.append(emigrants[-1])
            else:
                r_idx = replacement_indices(replacement, deme, k, stream)
                immigrants.append(pack(deme, r_idx))
        for from_deme, to_deme in enumerate(migarray):             # migration.py:48-51
            place(populations[to_deme], immigrants[to_deme], emigrants[from_deme], k)


def replacement_indices(replacement, pop, k, stream):
    """``replacement(pop, k)``: a device selection operator, or ``random.sample``
    (k distinct indices drawn on the device stream)."""
    import random as _random
    from ..ops import DeviceOperator as _Op, resolve
    if replacement is _random.sample:
        return sample_indices(pop, k, stream)
    op, a, kw = resolve(replacement)
    return op(pop, k, *a, stream=stream, **kw)


def sample_indices(pop, k, stream):
    """k distinct indices of ``pop`` (random.sample semantics) from the device stream."""
    torch = _torch()
    n = len(pop)
    if k > n:
        raise ValueError("Sample larger than population or is negative")
    r = stream.next()
    g = torch.Generator(device="cpu")
    g.manual_seed((r.seed ^ (r.island << 40) ^ (r.gen << 20)) & 0x7FFFFFFFFFFFFFFF)
    idx = torch.randperm(n, generator=g)[:k].to(torch.int32)
    return idx.to(pop.device)


migRing = _MigRing("migRing", "deap/tools/migration.py:4-51")

__all__ = ["migRing"]
