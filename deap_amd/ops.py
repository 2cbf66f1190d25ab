"""Device operator descriptors and the random stream.

Every operator exported by :mod:`deap_amd.tools` / :mod:`deap_amd.benchmarks`
is a :class:`DeviceOperator`: a callable that works on whole
:class:`~deap_amd.device.DevicePopulation` objects and that the drivers in
:mod:`deap_amd.algorithms` recognise inside a ``toolbox.register`` partial, so
the fused kernels can be parameterised from the registered keywords.
"""
import functools

from . import _lib


class DeviceOperator:
    kind = "op"

    def __init__(self, name, ref):
        self.__name__ = name
        self.__qualname__ = name
        self.ref = ref  # reference file:line this operator reproduces
        self.__doc__ = "%s — device restatement of DEAP's %s (%s)." % (name, name, ref)

    def __repr__(self):
        return "<deap_amd %s %s>" % (self.kind, self.__name__)

    def bind_params(self, args, kwargs):
        """Registered partial arguments -> dict of parameters."""
        return dict(kwargs)


def resolve(registered):
    """``toolbox.<alias>`` -> (operator, args, keywords).  Accepts a bare
    operator or a (possibly nested) functools.partial of one."""
    args, kw = (), {}
    f = registered
    while isinstance(f, functools.partial):
        args = tuple(f.args) + args
        merged = dict(f.keywords or {})
        merged.update(kw)
        kw = merged
        f = f.func
    if not isinstance(f, DeviceOperator):
        raise TypeError("%r is not a deap_amd device operator; register one of deap_amd.tools / "
                        "deap_amd.benchmarks (there is no CPU fallback)" % (registered,))
    return f, args, kw


class RandomStream:
    """Counter-based random stream of the engine (the device analogue of the
    ``random`` module state DEAP draws from).  Each kernel launch consumes one
    counter value, so a run is reproducible from (seed, island) and the call
    sequence, independent of launch geometry and GPU count."""

    def __init__(self, seed=0, island=0):
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.island = int(island)
        self.counter = 0

    def next(self):
        r = _lib.Rng()
        r.seed = self.seed
        r.island = self.island & 0xFFFF
        r.gen = self.counter & 0xFFFFFFFF
        self.counter += 1
        return r

    def getstate(self):
        return (self.seed, self.island, self.counter)

    def setstate(self, state):
        self.seed, self.island, self.counter = state


_default_stream = RandomStream(0)


def seed(value=0, island=0):
    """Reset the default device random stream (``random.seed`` analogue)."""
    global _default_stream
    _default_stream = RandomStream(value, island)
    return _default_stream


def default_stream():
    return _default_stream


def mode_code(mode):
    return {"native": _lib.DM_RNG_NATIVE, "inject": _lib.DM_RNG_INJECT,
            "dump": _lib.DM_RNG_DUMP}[mode]
