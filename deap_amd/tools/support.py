"""Per-generation bookkeeping (``deap/tools/support.py``): Statistics, Logbook,
HallOfFame, with device-side reductions for :class:`DevicePopulation` inputs.

* ``Statistics.compile`` on a device population evaluates the common numpy
  reducers (mean / std / min / max / sum, with or without ``axis``) as device
  reductions over ``fitness.values`` and defers the host copy to the logbook
  flush; any other registered function receives the host values exactly as in
  the reference (``support.py:199-210``).
* ``HallOfFame.update`` keeps the reference's insertion semantics
  (``support.py:517-560``).  With value-equality ``similar`` (the default
  ``operator.eq`` or ``numpy.array_equal``) only a candidate set of the best
  rows (device ``selBest``) is materialised; any other ``similar`` walks the
  whole population on the host, as the reference does.
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
        out = {}
        host = None
        kstats = None
        for name, fn in self.functions.items():
            kw = dict(fn.keywords or {})
            axis = kw.pop("axis", None)
            pick = _KERNEL_STATS.get(fn.func)
            if pick is not None and not fn.args and not kw and axis in (None, 0):
                # one dm_fitness_stats pass serves every such reducer: per
                # objective (axis=0), or over all values (axis=None: the
                # objectives' rows combined on the host)
                if kstats is None:
                    kstats = _KernelStats(pop)
                out[name] = functools.partial(kstats.value, fn.func, axis)
                continue
            # any other reducer: the reference's call on host values (one copy
            # of the weighted fitness, divided by the weights on the host) of the
            # VALID rows, as dm_fitness_stats reduces them (an invalid
            # individual's fitness.values is (), which the reference's numpy
            # reducers cannot combine with the others at all)
            if host is None:
                vals = pop.fitness_values().numpy()
                ok = pop.valid[:len(pop)].cpu().numpy().astype(bool)
                host = tuple(tuple(r) for r in vals[ok].tolist())
            out[name] = fn(host)
        return out


# numpy reducer -> value from a dm_fitness_stats row
# {min, max, mean, m2, sum, argmin, argmax, count} (include/deapmi.h)
_KERNEL_STATS = {
    np.min: lambda r: r[0], np.amin: lambda r: r[0], np.max: lambda r: r[1],
    np.amax: lambda r: r[1], np.mean: lambda r: r[2], np.sum: lambda r: r[4],
    np.var: lambda r: r[3] / r[7] if r[7] else np.float64("nan"),
    np.std: lambda r: np.sqrt(r[3] / r[7]) if r[7] else np.float64("nan"),
    np.argmin: lambda r: np.int64(r[5]), np.argmax: lambda r: np.int64(r[6]),
}


class _KernelStats:
    """One asynchronous ``dm_fitness_stats`` launch; the host copy happens on
    the first value read (the logbook flush), not in the generation loop."""

    def __init__(self, pop):
        import torch
        from .. import _lib
        self.nobj = pop.nobj
        self.out = torch.empty((pop.nobj * 8,), dtype=torch.float64, device=pop.device)
        w = (ctypes.c_double * pop.nobj)(*pop.weights)
        _lib.call("dm_fitness_stats", pop.ctx.bind(), ctypes.byref(pop.c_pop()), w,
                  ctypes.c_void_p(self.out.data_ptr()))
        self._host = None

    def rows(self):
        if self._host is None:
            self._host = self.out.cpu().numpy().reshape(self.nobj, 8)
        return self._host

    def value(self, func, axis):
        rows = self.rows()
        pick = _KERNEL_STATS[func]
        if axis == 0:
            return np.array([pick(r) for r in rows])
        if self.nobj == 1:
            return np.float64(pick(rows[0])) if pick not in _INT_PICKS else pick(rows[0])
        return _combined(func, rows, self.nobj)


def _combined(func, rows, nobj):
    """``func(values)`` over every objective value of the population (axis
    None on ``nobj`` > 1 objectives: numpy flattens the [n][nobj] tuple)
    from the per-objective rows {min, max, mean, m2, sum, argmin, argmax,
    count}: extrema of the extrema, sums of the sums, the Welford parts
    combined (Chan et al.) for mean / var / std, and for argmin / argmax the
    first flattened position (row * nobj + objective) holding the extremum."""
    mn, mx, mean, m2, sm, amn, amx, cnt = (np.array([r[i] for r in rows]) for i in range(8))
    if func in (np.min, np.amin):
        return np.float64(np.min(mn))
    if func in (np.max, np.amax):
        return np.float64(np.max(mx))
    if func is np.sum:
        return np.float64(np.sum(sm))
    total = np.sum(cnt)
    if func in (np.argmin, np.argmax):
        ext, arg = (mn, amn) if func is np.argmin else (mx, amx)
        if np.isnan(ext).any():  # numpy: the first NaN in flattened order
            flat = [int(arg[o]) * nobj + o for o in range(nobj) if np.isnan(ext[o])]
        else:
            best = np.min(ext) if func is np.argmin else np.max(ext)
            flat = [int(arg[o]) * nobj + o for o in range(nobj) if ext[o] == best]
        return np.int64(min(flat)) if flat else np.int64(0)
    if not total:
        return np.float64("nan")
    mu = np.sum(cnt * mean) / total
    if func is np.mean:
        return np.float64(mu)
    var = (np.sum(m2) + np.sum(cnt * (mean - mu) ** 2)) / total
    return np.float64(var if func is np.var else np.sqrt(var))


_INT_PICKS = (_KERNEL_STATS[np.argmin], _KERNEL_STATS[np.argmax])


def _typed_rows(pop, raw):
    """Host rows of raw genome bytes ([rows][stride] uint8) as the typed
    genome words genes_view() gives: int64 words for packed bits, else the
    float genes."""
    from .. import _lib
    if pop.gtype == _lib.DM_BITS:
        return raw.view(np.int64)[:, : (pop.dim + 63) // 64]
    if pop.gtype == _lib.DM_F32:
        return raw.view(np.float32)[:, : pop.dim]
    return raw.view(np.float64)[:, : pop.dim]


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
# with chapters (dict-valued fields) and an incremental text stream whose
# layout is the reference's character for character (pinned by
# tests/golden/support.npz, generated by the reference itself).
# ---------------------------------------------------------------------------
class Logbook(list):
    def __init__(self):
        super().__init__()
        self.buffindex = 0
        self.chapters = defaultdict(Logbook)
        self.columns_len = None
        self.header = None
        self.log_header = True

    def record(self, **infos):
        """Append one record; dict-valued fields go to the chapter of that
        name together with every non-dict field (support.py:335-349)."""
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

    def __delitem__(self, key):
        idx = range(*key.indices(len(self))) if isinstance(key, slice) else [key]
        for i in sorted(idx, reverse=True):
            self.pop(i)
            for chapter in self.chapters.values():
                chapter.pop(i)

    def pop(self, index=0):
        if index < self.buffindex:
            self.buffindex -= 1
        return super().pop(index)

    @staticmethod
    def _cell(value):
        # floats (numpy float64 included) use the locale-aware general format
        return "{0:n}".format(value) if isinstance(value, float) else "{0}".format(value)

    def _lines(self, start):
        """Text lines from record ``start`` on (with the header block when
        ``start == 0``); column widths only ever grow (columns_len)."""
        cols = list(self.header) if self.header else \
            sorted(self[0].keys()) + sorted(self.chapters.keys())
        if not self.columns_len or len(self.columns_len) != len(cols):
            self.columns_len = [len(c) for c in cols]
        chap = {name: ch._lines(start) for name, ch in self.chapters.items()}
        # a chapter's lines start with its own header block at start == 0
        skip = {name: (len(t) - len(self) if start == 0 else 0) for name, t in chap.items()}
        rows = []
        for i, entry in enumerate(self[start:]):
            row = []
            for j, name in enumerate(cols):
                cell = chap[name][i + skip[name]] if name in chap else \
                    self._cell(entry.get(name, ""))
                self.columns_len[j] = max(self.columns_len[j], len(cell))
                row.append(cell)
            rows.append(row)
        if start == 0 and self.log_header:
            depth = 1
            if self.chapters:
                depth += max(len(t) for t in chap.values()) - len(self) + 1
            head = [[] for _ in range(depth)]
            for j, name in enumerate(cols):
                if name in chap:
                    width = max(len(line.expandtabs()) for line in chap[name])
                    pad = depth - 2 - skip[name]
                    for i in range(pad):
                        head[i].append(" " * width)
                    head[pad].append(name.center(width))
                    head[pad + 1].append("-" * width)
                    for i in range(skip[name]):
                        head[pad + 2 + i].append(chap[name][i])
                else:
                    width = max(len(r[j].expandtabs()) for r in rows)
                    for line in head[:-1]:
                        line.append(" " * width)
                    head[-1].append(name)
            rows = head + rows
        fmt = "\t".join("{%d:<%d}" % (i, w) for i, w in enumerate(self.columns_len))
        return [fmt.format(*r) for r in rows]

    def __str__(self, startindex=0):
        return "\n".join(self._lines(startindex))


# ---------------------------------------------------------------------------
# HallOfFame (deap/tools/support.py:490-588)
# ---------------------------------------------------------------------------
_VALUE_SIMILAR = (operator.eq, np.array_equal)


def _host_fitness(weights):
    from ..device import HostFitness
    return HostFitness(weights)


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
        if self.similar in _VALUE_SIMILAR:
            # maxsize 1 too: a first-argmax shortcut is wrong when the argmax is
            # similar to the hofer but a lesser non-similar row beats the hofer
            self._update_candidates(pop)
            return
        # a user `similar` may match rows of different fitness; the candidate
        # argument below does not hold then, so walk the whole population
        rows = list(range(n))
        self._loop(rows, dict(zip(rows, pop.to_individuals())))

    def _update_candidates(self, pop):
        """HallOfFame.update for any maxsize / similar without copying the
        population: the reference loop (support.py:528-548) runs on host over a
        candidate set C = the K best rows (device selBest: wvalues desc, index
        asc) in population order.  Used only when ``similar`` is value equality
        (``operator.eq`` / ``numpy.array_equal``), which matches rows of equal
        genome and therefore equal fitness.  With t the fitness of the K-th row, the loop
        is accepted once it leaves a full hall whose every entry is strictly
        better than t (else K grows): a row outside C (fitness <= t) is then
        never in the final hall — it would be the worst entry when a better
        row of C arrives and be evicted, or be skipped as not better than the
        worst — and while present it only holds a slot a row of C later takes
        (equal genomes have equal fitness within one evaluated population).

        Only C's rows leave the GPU (one gather), as numpy rows: ``similar``
        is evaluated as row equality in numpy (element-wise ``==``: NaN genes
        are never similar and -0.0 == 0.0, as list / array equality of
        separate objects behaves), and host individuals are built only for
        the rows that enter the hall."""
        K = min(len(pop), max(4 * self.maxsize, 64))
        while True:
            if self._try_candidates(pop, K, *self._fetch_candidates(pop, K)()):
                return
            K = min(len(pop), 4 * K)

    def _fetch_candidates(self, pop, K):
        """Device part of one candidate round: selBest(K) and the gather of
        those rows (and row 0), copied to pinned host memory asynchronously.
        Returns a callable that waits for the copies (only them: work queued
        on the stream after this call is not waited for) and yields
        (order, rows, genes, wvalues, valid) for _try_candidates."""
        import torch
        from .. import _lib
        from .selection import selBest
        order = selBest(pop, K)  # int32 rows, fitness descending (device)
        # the K rows and row 0 gathered by the library (dm_gather) into a
        # candidate population of the same layout: no PyTorch index kernels
        cand = self._candidates_buffer(pop, K + 1)
        ctx = pop.ctx.bind()
        _lib.call("dm_gather", ctx, ctypes.byref(pop.c_pop()), ctypes.c_void_p(order.data_ptr()),
                  ctypes.byref(cand.c_pop(0, K)))
        _lib.call("dm_gather", ctx, ctypes.byref(pop.c_pop(0, 1)), None,
                  ctypes.byref(cand.c_pop(K, 1)))
        dev = (order, cand.genes[: K + 1], cand.wvalues[: K + 1], cand.valid[: K + 1])
        host = self._staging(dev)
        for h, t in zip(host, dev):
            h.copy_(t, non_blocking=True)
        done = torch.cuda.Event()
        done.record()

        def wait():
            done.synchronize()
            o, g, w, v = (h.numpy() for h in host)
            idx = np.append(o.astype(np.int64), 0)
            return idx, _typed_rows(pop, g), w, v
        return wait

    def _candidates_buffer(self, pop, rows):
        """A DevicePopulation of ``pop``'s layout with room for ``rows`` rows,
        kept between updates (grown when a larger K is asked for)."""
        buf = self.__dict__.get("_cand")
        if (buf is None or buf.capacity < rows or buf.stride != pop.stride or
                buf.gtype != pop.gtype or buf.nobj != pop.nobj or buf.device != pop.device):
            buf = self.__dict__["_cand"] = pop.like(rows, capacity=max(rows, 256))
        buf.resize(rows)
        return buf

    def _staging(self, dev):
        """Pinned host buffers for one candidate gather, two sets used in
        turn: eaSimple has at most one gather in flight while the next is
        queued, and reusing our own buffers keeps pinned allocations (which
        can synchronise the device) out of the generation loop."""
        import torch
        sets = self.__dict__.setdefault("_pinned", [None, None])
        i = self.__dict__["_pinned_turn"] = 1 - self.__dict__.get("_pinned_turn", 1)
        cur = sets[i]
        if cur is None or any(h.shape[0] < t.shape[0] or h.shape[1:] != t.shape[1:] or
                              h.dtype != t.dtype for h, t in zip(cur, dev)):
            cur = sets[i] = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in dev]
        return [h[: t.shape[0]] for h, t in zip(cur, dev)]

    def _try_candidates(self, pop, K, idx, graw, wv, valid):
        """One round of the candidate loop over the gathered rows; commits and
        returns True when accepted (see _update_candidates)."""
        from ..device import unpack_bits
        from .. import _lib
        n = len(pop)
        order = idx[:-1].tolist()
        pos = {int(r): i for i, r in enumerate(idx.tolist())}  # row -> gathered position
        rows = sorted(set(order) | ({0} if len(self) == 0 else set()))
        sel = np.array([pos[r] for r in rows], dtype=np.int64)
        genes = graw[sel]
        if pop.gtype == _lib.DM_BITS:
            genes = unpack_bits(genes.view(np.uint64), pop.dim)
        genes = np.ascontiguousarray(genes)
        wv, ok = wv[sel].copy(), valid[sel].astype(bool)
        trial = copy.copy(self)
        trial.keys, trial.items = list(self.keys), list(self.items)
        trial._garr = dict(self._garr_cache())
        fits = []
        for r in range(len(rows)):
            f = _host_fitness(pop.weights)
            if ok[r]:
                f.wvalues = tuple(float(x) for x in wv[r])
            fits.append(f)
        trial._loop_rows(pop, rows, genes, wv, ok, fits)
        if K < n:
            t = fits[rows.index(order[-1])]
            if not (len(trial) == self.maxsize and trial[-1].fitness > t):
                return False
        self.keys, self.items = trial.keys, trial.items
        self._garr = {id(it): trial._garr[id(it)] for it in self.items
                      if trial._garr.get(id(it), (None,))[0] is it}
        return True

    def update_begin(self, population):
        """``update(population)`` split in two for a generation loop: the
        device work is queued now and the host part runs in the returned
        callable, which a driver calls after queueing the next generation so
        the host loop overlaps that generation's kernel.  ``population``'s
        rows must stay unchanged until the callable returns (eaSimple's
        parent buffer is rewritten two generations later)."""
        from ..device import DevicePopulation
        if not (isinstance(population, DevicePopulation) and self.similar in _VALUE_SIMILAR
                and len(population) and self.maxsize):
            self.update(population)
            return lambda: None
        view = population.view()
        K = min(len(view), max(4 * self.maxsize, 64))
        fetched = self._fetch_candidates(view, K)

        def complete():
            if not self._try_candidates(view, K, *fetched()):
                self._update_candidates_from(view, min(len(view), 4 * K))
        return complete

    def _update_candidates_from(self, pop, K):
        while True:
            if self._try_candidates(pop, K, *self._fetch_candidates(pop, K)()):
                return
            K = min(len(pop), 4 * K)

    def _garr_cache(self):
        cache = getattr(self, "_garr", None)
        if cache is None:
            cache = self._garr = {}
        return cache

    def _genome(self, item):
        """numpy view of a hofer's genome, cached by identity (the entry keeps
        its object, so a recycled id never aliases another individual)."""
        cache = self._garr_cache()
        ent = cache.get(id(item))
        if ent is None or ent[0] is not item:
            ent = cache[id(item)] = (item, np.asarray(item))
        return ent[1]

    def __getstate__(self):
        state = dict(self.__dict__)
        for k in ("_garr", "_pinned", "_pinned_turn", "_cand"):  # transient device buffers
            state.pop(k, None)
        return state

    def _loop_rows(self, pop, rows, genes, wv, ok, fits):
        """support.py:528-548 over candidate rows held as numpy rows."""
        def make(r):
            ind = pop.make_individual(genes[r], wv[r], ok[r])
            self._garr_cache()[id(ind)] = (ind, genes[r])
            return ind
        for r in range(len(rows)):
            if len(self) == 0 and self.maxsize != 0:
                # first iteration with an empty hall: population[0] goes in
                self._insert_owned(make(rows.index(0)))
                continue
            if fits[r] > self[-1].fitness or len(self) < self.maxsize:
                g = genes[r]
                if any(np.array_equal(g, self._genome(h)) for h in self):
                    continue
                if len(self) >= self.maxsize:
                    self.remove(-1)
                self._insert_owned(make(r))

    def _insert_owned(self, item):
        """insert() without the deepcopy: ``item`` is a fresh host individual."""
        i = bisect.bisect_right(self.keys, item.fitness)
        self.items.insert(len(self) - i, item)
        self.keys.insert(i, item.fitness)

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
