"""Single-objective selection (``deap/tools/selection.py``) on device.

Each operator takes a :class:`~deap_amd.device.DevicePopulation` and returns a
device ``int32`` tensor of the selected row indices — the device form of
DEAP's "list of references"; ``population.take(idx)`` materialises the clone
(``toolbox.clone``) of the selection.
"""
import ctypes

from .. import _lib
from ..ops import DeviceOperator, default_stream, mode_code


def _torch():
    import torch
    return torch


def _check(individuals):
    from ..device import DevicePopulation
    if not isinstance(individuals, DevicePopulation):
        raise TypeError("deap_amd selection operators work on a DevicePopulation, got %r"
                        % type(individuals))


def _fit_attr(kw):
    fa = kw.pop("fit_attr", "fitness")
    if fa != "fitness":
        raise ValueError("only fit_attr='fitness' is stored on the device")


class _Tournament(DeviceOperator):
    kind = "select"

    def __call__(self, individuals, k, tournsize=None, fit_attr="fitness", *, stream=None,
                 mode=None, decisions=None):
        _check(individuals)
        if tournsize is None:
            raise TypeError("selTournament() missing required argument: 'tournsize'")
        _fit_attr({"fit_attr": fit_attr})
        torch = _torch()
        k = int(k)
        out = torch.empty((max(k, 1),), dtype=torch.int32, device=individuals.device)[:k]
        stream = stream or default_stream()
        code = mode_code(mode or "native")
        dec = None
        if code != _lib.DM_RNG_NATIVE:
            if decisions is None:
                from ..decisions import Decisions
                decisions = Decisions.allocate(k, individuals.dim, individuals.device,
                                               tournsize=int(tournsize), cx=False, mut=False)
            dec = decisions.c_struct()
        ctx = individuals.ctx.bind()
        _lib.call("dm_sel_tournament", ctx, ctypes.byref(individuals.c_pop()), k, int(tournsize),
                  stream.next(), code, ctypes.byref(dec) if dec is not None else None,
                  ctypes.c_void_p(out.data_ptr()) if k else None)
        if decisions is not None:
            out.decisions = decisions
        return out


class _Random(DeviceOperator):
    kind = "select"

    def __call__(self, individuals, k, *, stream=None, mode=None, decisions=None):
        _check(individuals)
        torch = _torch()
        k = int(k)
        out = torch.empty((max(k, 1),), dtype=torch.int32, device=individuals.device)[:k]
        stream = stream or default_stream()
        code = mode_code(mode or "native")
        dec = None
        if code != _lib.DM_RNG_NATIVE:
            if decisions is None:
                from ..decisions import Decisions
                decisions = Decisions.allocate(k, individuals.dim, individuals.device,
                                               tournsize=1, cx=False, mut=False)
            dec = decisions.c_struct()
        ctx = individuals.ctx.bind()
        _lib.call("dm_sel_random", ctx, len(individuals), k, stream.next(), code,
                  ctypes.byref(dec) if dec is not None else None,
                  ctypes.c_void_p(out.data_ptr()) if k else None)
        if decisions is not None:
            out.decisions = decisions
        return out


class _Sorted(DeviceOperator):
    kind = "select"

    def __init__(self, name, ref, entry):
        super().__init__(name, ref)
        self.entry = entry

    def __call__(self, individuals, k, fit_attr="fitness", *, stream=None, **_):
        _check(individuals)
        _fit_attr({"fit_attr": fit_attr})
        torch = _torch()
        k = int(min(int(k), len(individuals)))
        out = torch.empty((max(k, 1),), dtype=torch.int32, device=individuals.device)[:k]
        if k:
            ctx = individuals.ctx.bind()
            _lib.call(self.entry, ctx, ctypes.byref(individuals.c_pop()), k,
                      ctypes.c_void_p(out.data_ptr()))
        return out


selTournament = _Tournament("selTournament", "deap/tools/selection.py:51-69")
selRandom = _Random("selRandom", "deap/tools/selection.py:12-24")
selBest = _Sorted("selBest", "deap/tools/selection.py:27-36", "dm_sel_best")
selWorst = _Sorted("selWorst", "deap/tools/selection.py:39-48", "dm_sel_worst")

__all__ = ["selTournament", "selRandom", "selBest", "selWorst"]
