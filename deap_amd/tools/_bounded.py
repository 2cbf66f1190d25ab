"""Launcher of ``dm_vary_bounded``: the bounded real-valued operators of DEAP's
NSGA-II example (``cxSimulatedBinaryBounded``, crossover.py:291-360;
``mutPolynomialBounded``, mutation.py:51-95) and the loop body that chains
them (examples/ga/nsga2.py:96-105).

Decisions (modes "inject" / "dump") are a dict of float64 device tensors:
``cx_u`` [k//2] (pair ``random() <= cxpb``), ``sbx_u`` [k//2, dim, 3] (per gene
gate / rand / swap of SBX), ``mut_u`` [2*(k//2), dim, 2] (per gene gate / rand
of the polynomial mutation).  Each value is consumed only where the reference
would call ``random.random()``.
"""
import ctypes
from collections.abc import Sequence

import numpy as np

from .. import _lib
from ..device import zeros as _zeros


def _arg(args, kwargs, pos, name, op):
    if len(args) > pos:
        return args[pos]
    if name in kwargs:
        return kwargs[name]
    raise TypeError("%s() missing required argument: '%s'" % (op, name))


def _bound(val, name, size, what):
    """Scalar or sequence bound -> float or tuple of ``size`` floats; a short
    sequence is the reference's IndexError (crossover.py:317-322,
    mutation.py:67-73)."""
    if isinstance(val, Sequence) or hasattr(val, "__len__"):
        if len(val) < size:
            raise IndexError("%s must be at least the size of %s: %d < %d"
                             % (name, what, len(val), size))
        return tuple(float(x) for x in list(val)[:size])
    return float(val)


def sbx_params(args, kwargs):
    """(eta, low, up) of cxSimulatedBinaryBounded(ind1, ind2, eta, low, up)."""
    op = "cxSimulatedBinaryBounded"
    return {"eta": float(_arg(args, kwargs, 0, "eta", op)), "low": _arg(args, kwargs, 1, "low", op),
            "up": _arg(args, kwargs, 2, "up", op)}


def poly_params(args, kwargs):
    """(eta, low, up, indpb) of mutPolynomialBounded(individual, eta, low, up, indpb)."""
    op = "mutPolynomialBounded"
    return {"eta": float(_arg(args, kwargs, 0, "eta", op)), "low": _arg(args, kwargs, 1, "low", op),
            "up": _arg(args, kwargs, 2, "up", op),
            "indpb": float(_arg(args, kwargs, 3, "indpb", op))}


def vary_bounded(population, index, sbx, poly, cxpb, decisions=None, mode=None, stream=None):
    """Run dm_vary_bounded; returns the offspring population (k = len(index)
    or len(population)).  ``sbx`` / ``poly``: parameter dicts or None."""
    import torch
    from ..device import DevicePopulation
    from ..ops import default_stream, mode_code
    if not isinstance(population, DevicePopulation):
        raise TypeError("bounded variation works on a DevicePopulation, got %r" % type(population))
    stream = stream or default_stream()
    dev = population.device
    dim = population.dim
    keep = []
    v = _lib.BoundedVar()
    v.cxpb = float(cxpb)
    bounds = None
    if sbx is not None:
        v.cx = 1
        v.eta_cx = sbx["eta"]
        bounds = (_bound(sbx["low"], "low", dim, "the shorter individual"),
                  _bound(sbx["up"], "up", dim, "the shorter individual"))
    if poly is not None:
        v.mut = 1
        v.eta_mut = poly["eta"]
        v.indpb = poly["indpb"]
        pb = (_bound(poly["low"], "low", dim, "individual"),
              _bound(poly["up"], "up", dim, "individual"))
        if bounds is not None and pb != bounds:
            raise ValueError("fused SBX + polynomial mutation needs the same low/up bounds")
        bounds = pb
    for name, b in zip(("low", "up"), bounds):
        if isinstance(b, tuple):
            t = torch.tensor(b, dtype=torch.float64, device=dev)
            keep.append(t)
            setattr(v, name + "_vec", t.data_ptr())
        else:
            setattr(v, name, b)

    if index is not None:
        on_device = isinstance(index, torch.Tensor) and index.device.type != "cpu"
        if not on_device:
            # host indices are checked here (the reference's IndexError); device
            # indices (e.g. from selTournamentDCD) are not synced back — the
            # kernel turns an out-of-range row into a NaN, invalid child
            h = np.asarray(index.cpu() if isinstance(index, torch.Tensor) else index)
            if h.size and (int(h.min()) < 0 or int(h.max()) >= len(population)):
                raise IndexError("list index out of range")
            index = torch.from_numpy(np.ascontiguousarray(h, dtype=np.int32))
        idx = index.to(device=dev, dtype=torch.int32).contiguous()
        k = len(idx)
    else:
        idx = None
        k = len(population)
    offspring = population.like(k)
    code = mode_code(mode or "native")
    pairs = k // 2
    nmut = 2 * pairs if sbx is not None else k  # rows of mut_u
    cx_u = sbx_u = mut_u = None
    if code != _lib.DM_RNG_NATIVE:
        if decisions is None:
            raise ValueError("mode %r needs a decisions dict" % mode)
        if code == _lib.DM_RNG_DUMP:
            if sbx is not None:
                decisions["cx_u"] = _zeros((max(pairs, 1),), torch.float64, dev)
                decisions["sbx_u"] = _zeros((max(pairs, 1), dim, 3), torch.float64, dev)
            if poly is not None:
                decisions["mut_u"] = _zeros((max(nmut, 1), dim, 2), torch.float64, dev)
        if sbx is not None:
            cx_u = decisions["cx_u"].to(device=dev, dtype=torch.float64).contiguous()
            sbx_u = decisions["sbx_u"].to(device=dev, dtype=torch.float64).contiguous()
            if cx_u.numel() < pairs or sbx_u.numel() < pairs * dim * 3:
                raise ValueError("decisions cx_u / sbx_u too short")
            keep += [cx_u, sbx_u]
        if poly is not None:
            mut_u = decisions["mut_u"].to(device=dev, dtype=torch.float64).contiguous()
            if mut_u.numel() < nmut * dim * 2:
                raise ValueError("decisions mut_u too short")
            keep.append(mut_u)
    ptr = (lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None)
    ctx = population.ctx.bind()
    _lib.call("dm_vary_bounded", ctx, ctypes.byref(population.c_pop()), ptr(idx),
              ctypes.byref(offspring.c_pop()), ctypes.byref(v), stream.next(), code,
              ptr(cx_u), ptr(sbx_u), ptr(mut_u))
    offspring._keepalive = keep  # tensors read by the queued kernel
    return offspring
