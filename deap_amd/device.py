"""Device context and the structure-of-arrays population.

A :class:`DevicePopulation` is DEAP's ``list`` of individuals turned into
device buffers that stay resident in HBM across generations:

* ``genes``   — ``[capacity, stride]`` bytes, one genome row per individual
  (packed bits: ``ceil(dim/64)`` little-endian uint64 words, gene ``i`` at word
  ``i >> 6`` bit ``i & 63``; ``array('f')`` -> fp32 rows; ``array('d')`` or
  lists of floats -> fp64 rows);
* ``wvalues`` — ``[capacity, nobj]`` float64, the *weighted* fitness
  (``deap/base.py:187-198``);
* ``valid``   — ``[capacity]`` uint8, ``Fitness.valid`` (``deap/base.py:226-229``).

The buffers are PyTorch tensors (buffer ownership only); every computation on
them goes through ``libdeapmi.so``.
"""
import array as _array
import contextlib
import ctypes

import numpy as np

from . import _lib
from ._lib import DevicePop

GTYPE_NAMES = {"bits": _lib.DM_BITS, "f32": _lib.DM_F32, "f64": _lib.DM_F64}


def _torch():
    import torch
    return torch


def row_stride(gtype, dim):
    """Bytes per genome row: padded to 4-gene vectors, then to whole 128-B
    lines (rows of >= 128 B) or to a power of two (shorter rows), so no row
    shares an HBM line with its neighbour.  Rastrigin-1000D fp64 rows are
    8064 B: with 8000-B rows every odd row straddles lines and the row copy
    tops out at 5.15 TB/s instead of 5.6 (tools_gpu/bwtest2.hip).
    The pad bytes are never read or written by the kernels."""
    if gtype == _lib.DM_BITS:
        b = ((dim + 63) // 64) * 8
    elif gtype == _lib.DM_F32:
        b = ((dim + 3) // 4) * 16
    else:
        b = ((dim + 3) // 4) * 32
    b = (b + 15) // 16 * 16
    if b >= 128:
        return (b + 127) // 128 * 128
    p = 16
    while p < b:
        p *= 2
    return p


class Context:
    """One ``dm_ctx`` per device; the stream is re-bound to torch's current
    stream before every call so launches order with the caller's work."""

    _by_device = {}

    def __init__(self, device_index):
        lib = _lib.load()
        torch = _torch()
        if not torch.cuda.is_available():
            raise _lib.DeviceUnavailable("no ROCm GPU visible to PyTorch")
        self.device = torch.device("cuda", device_index)
        self.handle = ctypes.c_void_p()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(lib.dm_ctx_create(device_index, ctypes.c_void_p(stream),
                                     ctypes.byref(self.handle)), "dm_ctx_create")
        self._stream = stream

    @classmethod
    def get(cls, device=None):
        torch = _torch()
        if device is None:
            if not torch.cuda.is_available():
                raise _lib.DeviceUnavailable("no ROCm GPU visible to PyTorch")
            idx = torch.cuda.current_device()
        else:
            idx = torch.device(device).index or 0
        ctx = cls._by_device.get(idx)
        if ctx is None:
            ctx = cls(idx)
            cls._by_device[idx] = ctx
        ctx.bind()
        return ctx

    def bind(self):
        stream = _torch().cuda.current_stream(self.device).cuda_stream
        if stream != self._stream:
            _lib.check(_lib.load().dm_ctx_set_stream(self.handle, ctypes.c_void_p(stream)))
            self._stream = stream
        return self.handle

    def sync(self):
        _lib.check(_lib.load().dm_ctx_sync(self.handle), "dm_ctx_sync")


def zeros(shape, dtype, device):
    """A zero-filled device tensor: ``torch.empty`` (buffer ownership) zeroed
    by the library on the current stream (``dm_zero``: hipMemsetAsync), so
    buffer set-up launches no PyTorch fill kernel."""
    torch = _torch()
    t = torch.empty(shape, dtype=dtype, device=device)
    if t.numel():
        ctx = Context.get(t.device)
        _lib.call("dm_zero", ctx.handle, ctypes.c_void_p(t.data_ptr()),
                  t.numel() * t.element_size())
    return t


@contextlib.contextmanager
def dominance_path(name, device=None):
    """Run sortNondominated / selNSGA2 on one of the library's cross-check
    dominance paths (``"compare"``, ``"peel_d"``, ``"ballot"``, ``"lds"``;
    ``"default"`` is the product path) inside the block -- test and
    measurement use: every path gives the same fronts."""
    ctx = Context.get(device)
    _lib.call("dm_ctx_set_dom_path", ctx.handle, _lib.DM_DOM_PATHS[name])
    try:
        yield
    finally:
        _lib.call("dm_ctx_set_dom_path", ctx.handle, 0)


def gtype_of(individual_class=None, typecode=None, gtype=None):
    """Map a DEAP Individual type (``creator.create(..., array.array, typecode=...)``)
    to a device genome type."""
    if gtype is not None:
        return GTYPE_NAMES[gtype] if isinstance(gtype, str) else int(gtype)
    if typecode is None and individual_class is not None:
        typecode = getattr(individual_class, "typecode", None)
    if typecode in ("b", "B", "h", "H", "i", "I", "l", "L", "q", "Q", "?"):
        return _lib.DM_BITS
    if typecode == "f":
        return _lib.DM_F32
    return _lib.DM_F64


class FitnessValues:
    """The unweighted fitness values of a device population (``Fitness.values
    = wvalues / weights``, deap/base.py:184-185) as returned by a device
    objective: held as the device's weighted values and turned into numpy on
    the host when read (``numpy()``, ``np.asarray``, or ``cpu()`` for a
    torch CPU tensor), so an evaluation call launches no division kernel and
    copies nothing until the values are used."""

    def __init__(self, wvalues, weights):
        self._wv = wvalues
        self._w = np.asarray(weights, dtype=np.float64)

    def numpy(self):
        return self._wv.cpu().numpy() / self._w

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a if dtype is None else a.astype(dtype)

    def cpu(self):
        return _torch().from_numpy(self.numpy())

    @property
    def shape(self):
        return tuple(self._wv.shape)

    def __len__(self):
        return int(self._wv.shape[0])


class DevicePopulation:
    """A population resident on one GPU (SoA).  ``len(pop)`` is the number of
    individuals; rows ``[0, len)`` are live.  Drivers swap storage in place so
    ``population[:] = offspring`` (``deap/algorithms.py:181``) costs nothing."""

    def __init__(self, n, dim, gtype="f64", weights=(1.0,), device=None, capacity=None,
                 individual_class=None):
        torch = _torch()
        self.ctx = Context.get(device)
        self.device = self.ctx.device
        self.gtype = gtype_of(gtype=gtype) if not isinstance(gtype, int) else gtype
        self.dim = int(dim)
        self.weights = tuple(float(w) for w in weights)
        if not 1 <= len(self.weights) <= _lib.DM_MAX_OBJ:
            raise ValueError("between 1 and %d fitness weights supported" % _lib.DM_MAX_OBJ)
        self.nobj = len(self.weights)
        self.stride = row_stride(self.gtype, self.dim)
        self.capacity = int(capacity if capacity is not None else n)
        if n > self.capacity:
            raise ValueError("n > capacity")
        self.n = int(n)
        self.individual_class = individual_class
        self.genes = zeros((self.capacity, self.stride), torch.uint8, self.device)
        self.wvalues = zeros((self.capacity, self.nobj), torch.float64, self.device)
        self.valid = zeros((self.capacity,), torch.uint8, self.device)
        self.crowding_dist = None  # set by selNSGA2 / assignCrowdingDist

    # -- C view -------------------------------------------------------------
    def c_pop(self, start=0, count=None):
        count = self.n - start if count is None else count
        p = DevicePop()
        p.genes = self.genes.data_ptr() + start * self.stride
        p.wvalues = self.wvalues.data_ptr() + start * self.nobj * 8
        p.valid = self.valid.data_ptr() + start
        p.n = count
        p.stride = self.stride
        p.dim = self.dim
        p.gtype = self.gtype
        p.nobj = self.nobj
        return p

    # -- container protocol --------------------------------------------------
    def __len__(self):
        return self.n

    def resize(self, n):
        if n > self.capacity:
            raise ValueError("resize beyond capacity %d" % self.capacity)
        self.n = int(n)

    def view(self):
        """A second handle on the current buffers: later ``swap_storage`` calls
        on this population do not move the view."""
        import copy
        return copy.copy(self)

    def like(self, n=None, capacity=None):
        """Empty population with the same layout."""
        n = self.n if n is None else n
        return DevicePopulation(n, self.dim, self.gtype, self.weights, self.device,
                                capacity if capacity is not None else max(n, 1) if n else 1,
                                self.individual_class)

    def swap_storage(self, other):
        """``population[:] = other`` without copying (buffers exchanged)."""
        for attr in ("genes", "wvalues", "valid", "n", "capacity", "crowding_dist"):
            a, b = getattr(self, attr), getattr(other, attr)
            setattr(self, attr, b)
            setattr(other, attr, a)

    # -- typed views -----------------------------------------------------------
    def genes_view(self):
        """Typed tensor view ``[n, dim]`` (floats) or ``[n, words]`` (bits)."""
        torch = _torch()
        rows = self.genes[: self.n]
        if self.gtype == _lib.DM_BITS:
            return rows.view(torch.int64)[:, : (self.dim + 63) // 64]
        if self.gtype == _lib.DM_F32:
            return rows.view(torch.float32)[:, : self.dim]
        return rows.view(torch.float64)[:, : self.dim]

    def fitness_values(self):
        """Unweighted values ``wvalues / weights`` (``deap/base.py:184-185``),
        read lazily: :class:`FitnessValues` copies the weighted values to the
        host and divides there when asked (no device kernel)."""
        return FitnessValues(self.wvalues[: self.n], self.weights)

    # -- host transfer ---------------------------------------------------------
    def genes_numpy(self):
        """Host copy of the genomes: uint8 ``[n, dim]`` 0/1 for bits, else float."""
        g = self.genes_view().cpu().numpy()
        if self.gtype == _lib.DM_BITS:
            return unpack_bits(g.view(np.uint64), self.dim)
        return np.ascontiguousarray(g)

    def to_numpy(self):
        """(genes, wvalues, valid) on the host."""
        return (self.genes_numpy(), self.wvalues[: self.n].cpu().numpy().copy(),
                self.valid[: self.n].cpu().numpy().astype(bool))

    def rows_numpy(self, indices):
        """(genes, wvalues, valid) of the rows ``indices`` only: gathered on the
        device, then copied (a HallOfFame candidate set, not the population)."""
        torch = _torch()
        idx = torch.as_tensor(list(indices), dtype=torch.int64).to(self.device)
        g = self.genes_view()[idx].cpu().numpy()
        if self.gtype == _lib.DM_BITS:
            g = unpack_bits(g.view(np.uint64), self.dim)
        return (np.ascontiguousarray(g), self.wvalues[: self.n][idx].cpu().numpy().copy(),
                self.valid[: self.n][idx].cpu().numpy().astype(bool))

    @classmethod
    def from_numpy(cls, genes, weights=(1.0,), gtype=None, wvalues=None, valid=None,
                   device=None, capacity=None, individual_class=None):
        """Upload host genomes (``[n, dim]``: 0/1 ints for bits, floats otherwise)."""
        torch = _torch()
        genes = np.asarray(genes)
        if genes.ndim != 2:
            raise ValueError("genes must be [n, dim]")
        n, dim = genes.shape
        if gtype is None:
            gtype = "bits" if genes.dtype.kind in "biu" else ("f32" if genes.dtype == np.float32
                                                               else "f64")
        pop = cls(n, dim, gtype, weights, device, capacity, individual_class)
        buf = np.zeros((n, pop.stride), dtype=np.uint8)
        if pop.gtype == _lib.DM_BITS:
            packed = pack_bits(genes)
            buf[:, : packed.shape[1] * 8] = packed.view(np.uint8).reshape(n, -1)
        elif pop.gtype == _lib.DM_F32:
            buf[:, : dim * 4] = np.ascontiguousarray(genes, dtype=np.float32).view(np.uint8)
        else:
            buf[:, : dim * 8] = np.ascontiguousarray(genes, dtype=np.float64).view(np.uint8)
        if n:
            pop.genes[:n].copy_(torch.from_numpy(buf))
            if wvalues is not None:
                pop.wvalues[:n].copy_(torch.from_numpy(np.asarray(wvalues, np.float64)
                                                       .reshape(n, pop.nobj)))
            if valid is not None:
                pop.valid[:n].copy_(torch.from_numpy(np.asarray(valid, np.uint8)))
        return pop

    @classmethod
    def from_individuals(cls, individuals, weights=None, gtype=None, device=None, capacity=None):
        """Upload a list of DEAP-style individuals (sequences with ``.fitness``)."""
        if not individuals:
            raise ValueError("empty population")
        first = individuals[0]
        if weights is None:
            weights = first.fitness.weights
        if gtype is None:
            tc = getattr(first, "typecode", None)
            if tc is not None:
                gtype = {_lib.DM_BITS: "bits", _lib.DM_F32: "f32", _lib.DM_F64: "f64"}[
                    gtype_of(typecode=tc)]
            else:
                gtype = "bits" if all(isinstance(x, (int, bool)) for x in first) else "f64"
        dt = np.uint8 if gtype == "bits" else (np.float32 if gtype == "f32" else np.float64)
        genes = np.array([list(ind) for ind in individuals], dtype=dt)
        wv = np.array([ind.fitness.wvalues if ind.fitness.valid else (0.0,) * len(weights)
                       for ind in individuals], dtype=np.float64)
        valid = np.array([ind.fitness.valid for ind in individuals], dtype=np.uint8)
        return cls.from_numpy(genes, weights, gtype, wv, valid, device, capacity,
                              type(first))

    def to_individuals(self, individual_class=None, indices=None):
        """Materialise host individuals (DEAP semantics: ``fitness.wvalues`` set
        when valid).  ``individual_class`` defaults to the creator type the
        population was built from; plain lists otherwise."""
        from .base import Fitness
        cls_ = individual_class or self.individual_class
        if indices is None:
            genes, wv, valid = self.to_numpy()
            rows = range(self.n)
        else:
            genes, wv, valid = self.rows_numpy(indices)
            rows = range(len(genes))
        return [self.make_individual(genes[i], wv[i], valid[i], cls_) for i in rows]

    def make_individual(self, gene_row, wv_row, valid, individual_class=None):
        """One host individual from a host copy of its row (unpacked genes)."""
        cls_ = individual_class or self.individual_class
        vals = gene_row.tolist()
        if cls_ is None:
            ind = _HostIndividual(vals)
            ind.fitness = _make_fitness(self.weights)
        else:
            ind = cls_(vals)
        if not hasattr(ind, "fitness"):
            ind.fitness = _make_fitness(self.weights)
        if valid:
            ind.fitness.wvalues = tuple(float(x) for x in wv_row)
        return ind

    def __repr__(self):
        names = {v: k for k, v in GTYPE_NAMES.items()}
        return "DevicePopulation(n=%d, dim=%d, gtype=%s, weights=%r, device=%s)" % (
            self.n, self.dim, names[self.gtype], self.weights, self.device)


class _HostIndividual(list):
    pass


def _make_fitness(weights):
    return HostFitness(weights)


def _host_fitness_class():
    from .base import Fitness

    class HostFitness(Fitness):
        """Fitness of materialised host individuals: the weights live on the
        instance, so the individuals pickle (the reference's checkpoint
        pattern, doc/tutorials/advanced/checkpoint.rst:21-65)."""

        def __init__(self, weights=(1.0,), values=()):
            self.weights = tuple(weights)
            super().__init__(values)

        def __deepcopy__(self, memo):
            c = HostFitness(self.weights)
            c.wvalues = self.wvalues
            return c

    HostFitness.__module__ = __name__
    HostFitness.__qualname__ = "HostFitness"
    return HostFitness


HostFitness = _host_fitness_class()


def pack_bits(bits):
    """[n, dim] 0/1 -> [n, ceil(dim/64)] uint64, gene i at word i>>6 bit i&63."""
    bits = np.asarray(bits).astype(bool)
    n, dim = bits.shape
    words = (dim + 63) // 64
    padded = np.zeros((n, words * 64), dtype=bool)
    padded[:, :dim] = bits
    by = np.packbits(padded.reshape(n, words * 8, 8), axis=2, bitorder="little").reshape(n, words * 8)
    return by.view(np.uint64).reshape(n, words)


def unpack_bits(words, dim):
    words = np.ascontiguousarray(np.asarray(words, dtype=np.uint64))
    n = words.shape[0]
    by = words.view(np.uint8).reshape(n, -1)
    bits = np.unpackbits(by, axis=1, bitorder="little")
    return bits[:, :dim].astype(np.uint8)
