"""NSGA-II selection core (``deap/tools/emo.py:15-143``) on device.

Results are device ``int32`` index tensors in the reference's order:

* :func:`sortNondominated` returns the list of fronts, each a tensor of row
  indices in DEAP's front order (grouping of equal fitnesses by first
  appearance, dominance peel order), truncated once ``min(n, k)`` individuals
  are sorted;
* :func:`assignCrowdingDist` writes ``population.crowding_dist`` (float64
  tensor, ``fitness.crowding_dist`` of the reference);
* :func:`selNSGA2` returns the chosen indices (fronts but the last, then the
  last front by decreasing crowding distance, stable).
"""
import ctypes

import numpy as np

from .. import _lib
from ..ops import DeviceOperator
from ..device import zeros as _zeros


def _torch():
    import torch
    return torch


def _host_array(x):
    """A host numpy view of an index / decision array (device tensors are
    copied, never computed on)."""
    if hasattr(x, "detach"):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def _host_index(front):
    return np.ascontiguousarray(_host_array(front), dtype=np.int32).ravel()


def _check(individuals):
    from ..device import DevicePopulation
    if not isinstance(individuals, DevicePopulation):
        raise TypeError("deap_amd NSGA-II operators work on a DevicePopulation, got %r"
                        % type(individuals))


def _weights(pop):
    return (ctypes.c_double * pop.nobj)(*pop.weights)


def _sort(individuals, k, first_front_only):
    torch = _torch()
    n = len(individuals)
    order = torch.empty((max(n, 1),), dtype=torch.int32, device=individuals.device)
    fstart = torch.empty((max(n, 1) + 1,), dtype=torch.int32, device=individuals.device)
    rank = torch.empty((max(n, 1),), dtype=torch.int32, device=individuals.device)
    nsorted = ctypes.c_int64(0)
    nfronts = ctypes.c_int32(0)
    ctx = individuals.ctx.bind()
    _lib.call("dm_sort_nondominated", ctx, ctypes.byref(individuals.c_pop()), int(k),
              int(bool(first_front_only)), ctypes.c_void_p(order.data_ptr()),
              ctypes.c_void_p(fstart.data_ptr()), ctypes.c_void_p(rank.data_ptr()),
              ctypes.byref(nsorted), ctypes.byref(nfronts))
    return order, fstart, rank, nsorted.value, nfronts.value


class _SortNondominated(DeviceOperator):
    kind = "sort"

    def __call__(self, individuals, k, first_front_only=False):
        _check(individuals)
        if k == 0:
            return []
        if len(individuals) == 0:
            # the reference builds `fronts = [[]]` before any peel (emo.py:96-117)
            torch = _torch()
            return [torch.empty((0,), dtype=torch.int32, device=individuals.device)]
        order, fstart, _rank, _ns, nf = _sort(individuals, k, first_front_only)
        bounds = fstart[: nf + 1].cpu().tolist()
        return [order[bounds[f]:bounds[f + 1]] for f in range(nf)]


class _CrowdingDist(DeviceOperator):
    kind = "crowding"

    def __call__(self, individuals, fronts=None):
        """Crowding distance of ``individuals`` taken as one front (reference
        semantics), or of every front in ``fronts`` (index tensors)."""
        _check(individuals)
        torch = _torch()
        n = len(individuals)
        if n == 0:
            return
        dev = individuals.device
        if fronts is None:
            order = torch.from_numpy(np.arange(n, dtype=np.int32)).to(dev)
            fstart = torch.from_numpy(np.array([0, n], dtype=np.int32)).to(dev)
            nf = 1
        else:
            # user-supplied fronts: concatenated on the host (one copy each
            # way, no device kernel); the library's own selNSGA2 never takes
            # this path
            parts = [_host_index(f) for f in fronts]
            order = torch.from_numpy(np.concatenate(parts) if parts else
                                     np.zeros(0, np.int32)).to(dev)
            sizes = np.cumsum([0] + [len(f) for f in parts]).astype(np.int32)
            fstart = torch.from_numpy(sizes).to(dev)
            nf = len(fronts)
        if individuals.crowding_dist is None or len(individuals.crowding_dist) < n:
            individuals.crowding_dist = _zeros((individuals.capacity,), torch.float64, dev)
        ctx = individuals.ctx.bind()
        _lib.call("dm_crowding_dist", ctx, ctypes.byref(individuals.c_pop()), _weights(individuals),
                  ctypes.c_void_p(order.data_ptr()), ctypes.c_void_p(fstart.data_ptr()), nf,
                  ctypes.c_void_p(individuals.crowding_dist.data_ptr()))
        return individuals.crowding_dist[:n]


class _SelNSGA2(DeviceOperator):
    kind = "select"

    def __call__(self, individuals, k, nd="standard", *, stream=None, **_):
        _check(individuals)
        if nd == "log":
            return _sel_nsga2_log(individuals, int(k))
        if nd != "standard":
            raise Exception('selNSGA2: The choice of non-dominated sorting '
                            'method "{0}" is invalid.'.format(nd))
        torch = _torch()
        n = len(individuals)
        k = int(k)
        out = torch.empty((max(k, 1),), dtype=torch.int32, device=individuals.device)
        if individuals.crowding_dist is None or len(individuals.crowding_dist) < n:
            individuals.crowding_dist = _zeros((individuals.capacity,), torch.float64,
                                                individuals.device)
        if k == 0 or n == 0:
            return out[:0]
        ctx = individuals.ctx.bind()
        _lib.call("dm_sel_nsga2", ctx, ctypes.byref(individuals.c_pop()), _weights(individuals), k,
                  ctypes.c_void_p(out.data_ptr()),
                  ctypes.c_void_p(individuals.crowding_dist.data_ptr()))
        return out[: min(k, n)]


def _log_fronts(individuals, k, first_front_only):
    """Fronts in sortLogNondominated's order (emo.py:246-276), ordered in the
    library (dm_sort_log_nondominated): the Pareto ranks of the device sort
    (Fortin et al.'s divide and conquer computes the same ranks); inside a
    front the unique fitnesses follow ``fitnesses.sort(reverse=True)``
    (lexicographic wvalues, descending) and equal fitnesses keep population
    order (``unique_fits[...].append``)."""
    torch = _torch()
    n = len(individuals)
    dev = individuals.device
    order = torch.empty((max(n, 1),), dtype=torch.int32, device=dev)
    fstart = torch.empty((max(n, 1) + 1,), dtype=torch.int32, device=dev)
    nsorted = ctypes.c_int64(0)
    nfronts = ctypes.c_int32(0)
    ctx = individuals.ctx.bind()
    _lib.call("dm_sort_log_nondominated", ctx, ctypes.byref(individuals.c_pop()), int(k),
              int(bool(first_front_only)), ctypes.c_void_p(order.data_ptr()),
              ctypes.c_void_p(fstart.data_ptr()), ctypes.byref(nsorted), ctypes.byref(nfronts))
    nf = nfronts.value
    bounds = fstart[: nf + 1].cpu().tolist()
    return [order[bounds[f]:bounds[f + 1]] for f in range(nf)]


class _SortLogNondominated(DeviceOperator):
    kind = "sort"

    def __call__(self, individuals, k, first_front_only=False):
        _check(individuals)
        if k == 0:
            return []
        if len(individuals) == 0:
            raise IndexError("list index out of range")  # individuals[0] (emo.py:252)
        fronts = _log_fronts(individuals, k, first_front_only)
        return fronts[0] if first_front_only else fronts


def _sel_nsga2_log(individuals, k):
    """selNSGA2(nd='log') (emo.py:15-50 over sortLogNondominated), in the
    library (dm_sel_nsga2_log): crowding on every front in its log order, all
    fronts but the last, then the last one by decreasing crowding distance
    (stable, as ``sorted(..., reverse=True)``)."""
    torch = _torch()
    n = len(individuals)
    out = torch.empty((max(k, 1),), dtype=torch.int32, device=individuals.device)
    if individuals.crowding_dist is None or len(individuals.crowding_dist) < n:
        individuals.crowding_dist = _zeros((individuals.capacity,), torch.float64,
                                           individuals.device)
    if k == 0 or n == 0:
        return out[:0]
    ctx = individuals.ctx.bind()
    _lib.call("dm_sel_nsga2_log", ctx, ctypes.byref(individuals.c_pop()), _weights(individuals),
              k, ctypes.c_void_p(out.data_ptr()),
              ctypes.c_void_p(individuals.crowding_dist.data_ptr()))
    return out[: min(k, n)]


class _SelTournamentDCD(DeviceOperator):
    kind = "select"

    def __call__(self, individuals, k, *, stream=None, mode=None, decisions=None, **_):
        """Returns 4*ceil(k/4) indices (the reference appends four per step of
        ``range(0, k, 4)``).  Needs ``individuals.crowding_dist`` (set by
        selNSGA2 / assignCrowdingDist) as the reference needs
        ``fitness.crowding_dist``.  ``decisions``: dict with int32 device
        tensors ``perm1``, ``perm2`` [n] and uint8 ``coin`` [4*ceil(k/4)],
        read in mode "inject", filled in mode "dump"."""
        from ..ops import default_stream, mode_code
        _check(individuals)
        torch = _torch()
        if individuals.crowding_dist is None:
            raise AttributeError("'Fitness' object has no attribute 'crowding_dist'")
        stream = stream or default_stream()
        n, k = len(individuals), int(k)
        if len(individuals.crowding_dist) < n:
            raise ValueError("crowding_dist holds %d values for %d individuals"
                             % (len(individuals.crowding_dist), n))
        k4 = (k + 3) // 4 * 4
        dev = individuals.device
        out = torch.empty((max(k4, 1),), dtype=torch.int32, device=dev)
        code = mode_code(mode or "native")
        p1 = p2 = coin = None
        if code != _lib.DM_RNG_NATIVE:
            if code == _lib.DM_RNG_DUMP:
                decisions["perm1"] = torch.empty((max(n, 1),), dtype=torch.int32, device=dev)
                decisions["perm2"] = torch.empty((max(n, 1),), dtype=torch.int32, device=dev)
                decisions["coin"] = _zeros((max(k4, 1),), torch.uint8, dev)
            else:
                # injected decisions: device tensors of the kernel's dtypes, long
                # enough, and permutations of range(n) (the kernel dereferences
                # fitness rows through them)
                # (checked on the host: no device kernel)
                decisions = dict(decisions)
                for name, dt, need in (("perm1", np.int32, n), ("perm2", np.int32, n),
                                       ("coin", np.uint8, k4)):
                    h = np.ascontiguousarray(_host_array(decisions[name]), dtype=dt).ravel()
                    if h.size < need:
                        raise ValueError("decisions[%r] holds %d values, %d needed"
                                         % (name, h.size, need))
                    if name != "coin" and n and not np.array_equal(np.sort(h[:n]),
                                                                   np.arange(n, dtype=np.int32)):
                        raise ValueError("decisions[%r] is not a permutation of range(%d)"
                                         % (name, n))
                    decisions[name] = torch.from_numpy(h).to(dev)
            p1, p2, coin = decisions["perm1"], decisions["perm2"], decisions["coin"]
        ptr = (lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None)
        ctx = individuals.ctx.bind()
        _lib.call("dm_sel_tournament_dcd", ctx, ctypes.byref(individuals.c_pop()),
                  ctypes.c_void_p(individuals.crowding_dist.data_ptr()), k, stream.next(), code,
                  ptr(p1), ptr(p2), ptr(coin), ctypes.c_void_p(out.data_ptr()))
        return out[:k4]


sortNondominated = _SortNondominated("sortNondominated", "deap/tools/emo.py:53-117")
sortLogNondominated = _SortLogNondominated("sortLogNondominated", "deap/tools/emo.py:234-441")
assignCrowdingDist = _CrowdingDist("assignCrowdingDist", "deap/tools/emo.py:119-143")
selNSGA2 = _SelNSGA2("selNSGA2", "deap/tools/emo.py:15-50")
selTournamentDCD = _SelTournamentDCD("selTournamentDCD", "deap/tools/emo.py:145-195")

__all__ = ["selNSGA2", "sortNondominated", "sortLogNondominated", "selTournamentDCD"]  # assignCrowdingDist is not exported (emo.py:842-843)
