"""Per-generation bookkeeping (``deap/tools/support.py``): Statistics, Logbook,
HallOfFame, with device-side reductions for :class:`DevicePopulation` inputs.

* ``Statistics.compile`` on a device population evaluates the common numpy
  reducers (mean / std / min / max / sum, with or without ``axis``) as device
  reductions over ``fitness.values`` and defers the host copy to the logbook
  flush; any other registered function receives the host values exactly as in
  the reference (``support.py:199-210``).
* ``HallOfFame.update`` keeps the reference's insertion semantics
  (``support.py:517-560``); with ``maxsize == 1`` the device computes the
  first lexicographic argmax, otherwise the candidates are materialised.
"""
import bisect
import copy
import ctypes
import functools
import operator
from collections import defaultdict

import numpy as np


# ---------------------------------------------------------------------------
# Statistics
# ---------------------------------------------------------------------------
class _ValuesProbe:
    """Detects keys of the form ``lambda ind: ind.fitness.values``."""
    SENTINEL = object()

    class _F:
        values = None

    def __init__(self):
        self.fitness = self._F()
        self.fitness.values = self.SENTINEL


def _is_values_key(key):
    try:
        return key(_ValuesProbe()) is _ValuesProbe.SENTINEL
    except Exception:  # noqa: BLE001 - arbitrary user key
        return False


_DEVICE_REDUCERS = {}


def _device_reducer(func):
    try:
        _DEVICE_REDUCERS[np.mean] = lambda t, axis: t.mean() if axis is None else t.mean(dim=axis)
        _DEVICE_REDUCERS[np.std] = (lambda t, axis: t.std(unbiased=False) if axis is None
                                    else t.std(dim=axis, unbiased=False))
        _DEVICE_REDUCERS[np.min] = lambda t, axis: t.min() if axis is None else t.min(dim=axis).values
        _DEVICE_REDUCERS[np.max] = lambda t, axis: t.max() if axis is None else t.max(dim=axis).values
        _DEVICE_REDUCERS[np.sum] = lambda t, axis: t.sum() if axis is None else t.sum(dim=axis)
        _DEVICE_REDUCERS[np.amin] = _DEVICE_REDUCERS[np.min]
        _DEVICE_REDUCERS[np.amax] = _DEVICE_REDUCERS[np.max]
    except AttributeError:
        pass
    return _DEVICE_REDUCERS.get(func)


def _identity(obj):
    return obj


class Statistics:
    """``deap/tools/support.py:154-210``"""

    def __init__(self, key=_identity):
        self.key = key
        self.functions = dict()
        self.fields = []

    def register(self, name, function, *args, **kargs):
        self.functions[name] = functools.partial(function, *args, **kargs)
        self.fields.append(name)

    def compile(self, data):
        from ..device import DevicePopulation
        if isinstance(data, DevicePopulation):
            return self._compile_device(data)
        values = tuple(self.key(elem) for elem in data)
        return {name: fn(values) for name, fn in self.functions.items()}

    def _compile_device(self, pop):
        if not _is_values_key(self.key):
            # arbitrary key: materialise individuals (reference semantics)
            inds = pop.to_individuals()
            values = tuple(self.key(ind) for ind in inds)
            return {name: fn(values) for name, fn in self.functions.items()}
        vals = pop.fitness_values()
        out = {}
        host = None
        for name, fn in self.functions.items():
            red = _device_reducer(fn.func)
            kw = dict(fn.keywords or {})
            axis = kw.pop("axis", None)
            if red is not None and not fn.args and not kw:
                t = red(vals, axis)
                out[name] = functools.partial(_to_numpy, t)
            else:
                if host is None:
                    host = tuple(tuple(r) for r in vals.cpu().numpy().tolist())
                out[name] = fn(host)
        return out


def _to_numpy(t):
    a = t.detach().cpu().numpy()
    return a[()] if a.ndim == 0 else a


class MultiStatistics(dict):
    """``deap/tools/support.py:212-259``"""

    def compile(self, data):
        record = {}
        for name, stats in self.items():
            record[name] = stats.compile(data)
        return record

    @property
    def fields(self):
        return sorted(self.keys())

    def register(self, name, function, *args, **kargs):
        for stats in self.values():
            stats.register(name, function, *args, **kargs)


# ---------------------------------------------------------------------------
# Logbook (deap/tools/support.py:261-487): chronological list of dict records
# with chapters (dict-valued fields) and an incremental text stream.
# ---------------------------------------------------------------------------
class Logbook(list):
    def __init__(self):
        super().__init__()
        self.buffindex = 0
        self.chapters = defaultdict(Logbook)
        self.header = None
        self.log_header = True
        self._widths = {}

    def record(self, **infos):
        shared = {k: v for k, v in infos.items() if not isinstance(v, dict)}
        flat = {}
        for key, value in infos.items():
            if isinstance(value, dict):
                sub = dict(value)
                sub.update(shared)
                self.chapters[key].record(**sub)
            else:
                flat[key] = value
        self.append(flat)

    def select(self, *names):
        cols = tuple([entry.get(name) for entry in self] for name in names)
        return cols[0] if len(names) == 1 else cols

    @property
    def stream(self):
        start, self.buffindex = self.buffindex, len(self)
        return self.__str__(start)

    def pop(self, index=0):
        if index < self.buffindex:
            self.buffindex -= 1
        return super().pop(index)

    def _columns(self):
        if self.header:
            return list(self.header)
        keys = sorted(self[0].keys()) if self else []
        return keys + sorted(self.chapters.keys())

    @staticmethod
    def _fmt(value):
        return "{0:n}".format(value) if isinstance(value, float) else str(value)

    def _cells(self, row, cols):
        out = []
        for name in cols:
            if name in self.chapters:
                chap = self.chapters[name]
                ccols = chap._columns()
                crow = chap[row] if row < len(chap) else {}
                out.append(" ".join(self._fmt(crow.get(c, "")) for c in ccols))
            else:
                out.append(self._fmt(self[row].get(name, "")))
        return out

    def __str__(self, startindex=0):
        cols = self._columns()
        rows = [self._cells(i, cols) for i in range(startindex, len(self))]
        for j, name in enumerate(cols):
            w = max([len(name)] + [len(r[j]) for r in rows])
            self._widths[name] = max(self._widths.get(name, 0), w)
        lines = []
        if startindex == 0 and self.log_header:
            lines.append("\t".join(n.ljust(self._widths[n]) for n in cols))
        for r in rows:
            lines.append("\t".join(c.ljust(self._widths[n]) for c, n in zip(r, cols)))
        return "\n".join(lines)


# ---------------------------------------------------------------------------
# HallOfFame (deap/tools/support.py:490-588)
# ---------------------------------------------------------------------------
class HallOfFame:
    def __init__(self, maxsize, similar=operator.eq):
        self.maxsize = maxsize
        self.keys = list()
        self.items = list()
        self.similar = similar

    def update(self, population):
        from ..device import DevicePopulation
        if isinstance(population, DevicePopulation):
            self._update_device(population)
            return
        for ind in population:
            if len(self) == 0 and self.maxsize != 0:
                self.insert(population[0])
                continue
            if ind.fitness > self[-1].fitness or len(self) < self.maxsize:
                if any(self.similar(ind, hofer) for hofer in self):
                    continue
                if len(self) >= self.maxsize:
                    self.remove(-1)
                self.insert(ind)

    def _update_device(self, pop):
        n = len(pop)
        if n == 0 or self.maxsize == 0:
            return
        # maxsize 1 too: a first-argmax shortcut is wrong when the argmax is
        # similar to the hofer but a lesser non-similar row beats the hofer
        self._update_candidates(pop)

    def _update_candidates(self, pop):
        """HallOfFame.update for any maxsize / similar without copying the
        population: the reference loop (support.py:528-548) runs on host over a
        candidate set C = the K best rows (device selBest: wvalues desc, index
        asc) in population order.  With t the fitness of the K-th row, the loop
        is accepted once it leaves a full hall whose every entry is strictly
        better than t (else K grows): a row outside C (fitness <= t) is then
        never in the final hall — it would be the worst entry when a better
        row of C arrives and be evicted, or be skipped as not better than the
        worst — and while present it only holds a slot a row of C later takes
        (equal genomes have equal fitness within one evaluated population)."""
        from .selection import selBest
        n = len(pop)
        K = min(n, max(4 * self.maxsize, 64))
        while True:
            order = selBest(pop, K).cpu().tolist()
            trial = copy.copy(self)
            trial.keys, trial.items = list(self.keys), list(self.items)
            rows = sorted(set(order) | ({0} if len(self) == 0 else set()))
            inds = dict(zip(rows, pop.to_individuals(indices=rows)))
            trial._loop(rows, inds)
            if K >= n:
                break
            t = inds[order[-1]].fitness
            if len(trial) == self.maxsize and trial[-1].fitness > t:
                break
            K = min(n, 4 * K)
        self.keys, self.items = trial.keys, trial.items

    def _loop(self, rows, inds):
        """support.py:528-548 over the rows of a candidate set, in order."""
        for i in rows:
            ind = inds[i]
            if len(self) == 0 and self.maxsize != 0:
                # first iteration with an empty hall: population[0] goes in
                self.insert(inds[0])
                continue
            if ind.fitness > self[-1].fitness or len(self) < self.maxsize:
                if any(self.similar(ind, hofer) for hofer in self):
                    continue
                if len(self) >= self.maxsize:
                    self.remove(-1)
                self.insert(ind)

    def insert(self, item):
        item = copy.deepcopy(item)
        i = bisect.bisect_right(self.keys, item.fitness)
        self.items.insert(len(self) - i, item)
        self.keys.insert(i, item.fitness)

    def remove(self, index):
        del self.keys[len(self) - (index % len(self) + 1)]
        del self.items[index]

    def clear(self):
        del self.items[:]
        del self.keys[:]

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]

    def __iter__(self):
        return iter(self.items)

    def __reversed__(self):
        return reversed(self.items)

    def __str__(self):
        return str(self.items)


__all__ = ["Statistics", "MultiStatistics", "Logbook", "HallOfFame"]
