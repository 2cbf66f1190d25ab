"""Ring migration between demes (``deap/tools/migration.py:4-51``).

``migRing(populations, k, selection, replacement=None, migarray=None)`` works
in place on a list of :class:`DevicePopulation` demes on one GPU (one
``dm_mig_ring`` call for the whole migration); the multi-GPU form (demes on
several ranks, emigrants exchanged with RCCL point-to-point over xGMI) is
:func:`deap_amd.islands.migRingDistributed`.

Semantics kept from the reference: all emigrants are selected before any
placement; immigrants default to the emigrants themselves; for each
``from_deme`` in order, every immigrant ``j`` is located in the *current*
destination deme by ``list.index`` (identity, then value equality) and that
slot receives emigrant ``j`` — so a second equal-valued immigrant can re-hit
the slot just filled by an equal emigrant, exactly like the reference.
``replacement=random.sample`` draws k distinct rows on the device
(``dm_sel_sample``, counter-based RNG).
"""
import ctypes

from .. import _lib
from ..ops import DeviceOperator, default_stream


def _torch():
    import torch
    return torch


def pack(pop, idx):
    """Pack rows ``idx`` of ``pop`` into one contiguous block (genomes,
    wvalues, valid, source rows) — the unit sent between ranks."""
    torch = _torch()
    k = int(idx.numel())
    nbytes = _lib.load().dm_pack_bytes(ctypes.byref(pop.c_pop()), k)
    block = torch.empty((max(int(nbytes), 16),), dtype=torch.uint8, device=pop.device)
    if k:
        idx = idx.to(device=pop.device, dtype=torch.int32).contiguous()
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
                 stream=None, record=None):
        """``record``: optional list; one dict per call is appended with host
        copies of every deme's emigrant and immigrant row indices."""
        torch = _torch()
        stream = stream or default_stream()
        nbr_demes = len(populations)
        if nbr_demes == 0:
            return
        if migarray is None:
            migarray = list(range(1, nbr_demes)) + [0]               # migration.py:34
        if len(migarray) != nbr_demes:
            raise ValueError("migarray must have one entry per deme")
        emig, immig = [], []
        for deme in populations:                                   # migration.py:39-46
            emig.append(select_indices(selection, deme, k, stream).to(torch.int32).contiguous())
            immig.append(None if replacement is None else
                         replacement_indices(replacement, deme, k, stream)
                         .to(torch.int32).contiguous())
        if record is not None:
            record.append({"emigrants": [e.cpu().numpy().copy() for e in emig],
                           "immigrants": [None if i is None else i.cpu().numpy().copy()
                                          for i in immig]})
        pops = (_lib.DevicePop * nbr_demes)(*[p.c_pop() for p in populations])
        mig = (ctypes.c_int32 * nbr_demes)(*migarray)
        e_arr = (ctypes.c_void_p * nbr_demes)(*[e.data_ptr() for e in emig])
        i_arr = (ctypes.c_void_p * nbr_demes)(*[None if i is None else i.data_ptr()
                                                for i in immig])
        ctx = populations[0].ctx.bind()
        _lib.call("dm_mig_ring", ctx, nbr_demes, pops, mig, int(k), e_arr, i_arr, None)


def replacement_indices(replacement, pop, k, stream):
    """``replacement(pop, k)``: a device selection operator, or ``random.sample``
    (k distinct indices drawn on the device stream)."""
    import random as _random
    from ..ops import resolve
    if replacement is _random.sample:
        return sample_indices(pop, k, stream)
    op, a, kw = resolve(replacement)
    return op(pop, k, *a, stream=stream, **kw)


def sample_indices(pop, k, stream):
    """k distinct row indices of ``pop`` in draw order — ``random.sample``
    semantics — drawn on the device (``dm_sel_sample``)."""
    torch = _torch()
    n = len(pop)
    if k > n or k < 0:
        raise ValueError("Sample larger than population or is negative")
    out = torch.empty((max(k, 1),), dtype=torch.int32, device=pop.device)
    _lib.call("dm_sel_sample", pop.ctx.bind(), n, int(k), stream.next(),
              ctypes.c_void_p(out.data_ptr()))
    return out[:k]


migRing = _MigRing("migRing", "deap/tools/migration.py:4-51")

__all__ = ["migRing"]
