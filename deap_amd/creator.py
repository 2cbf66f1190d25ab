"""Run-time class factory with DEAP's behaviour (``deap/creator.py:96-171``).

``create("FitnessMax", base.Fitness, weights=(1.0,))`` and
``create("Individual", array.array, typecode="b", fitness=FitnessMax)`` build
the same classes as the reference; the device layer reads ``typecode`` and
``fitness.weights`` from them to pick the device genome type
(packed bits / fp32 / fp64, :func:`deap_amd.device.gtype_of`).
"""
import array
import copy
import warnings

_module_globals = globals()


class _ArrayIndividual(array.array):
    """array.array base whose instances may carry attributes; deepcopy and
    pickling keep them (``deap/creator.py:76-93``)."""

    @staticmethod
    def __new__(cls, seq=()):
        return super().__new__(cls, cls.typecode, seq)

    def __deepcopy__(self, memo):
        twin = self.__class__(self)
        memo[id(self)] = twin
        twin.__dict__.update(copy.deepcopy(self.__dict__, memo))
        return twin

    def __reduce__(self):
        return (self.__class__, (list(self),), self.__dict__)


_REPLACE = {array.array: _ArrayIndividual}


def create(name, base, **kargs):
    """Create class ``name`` deriving from ``base`` in this module's namespace.

    Keyword values that are classes become per-instance attributes built at
    construction time (e.g. ``fitness=FitnessMax``); other values become class
    attributes (e.g. ``weights=(1.0,)``, ``typecode='d'``)."""
    if name in _module_globals:
        warnings.warn("A class named '%s' has already been created and it will be overwritten. "
                      "Consider deleting previous creation of that class or rename it." % name,
                      RuntimeWarning)
    per_instance = {k: v for k, v in kargs.items() if isinstance(v, type)}
    class_attrs = {k: v for k, v in kargs.items() if not isinstance(v, type)}
    base = _REPLACE.get(base, base)

    def __init__(self, *args, **kw):
        for attr, factory in per_instance.items():
            setattr(self, attr, factory())
        if base.__init__ is not object.__init__:
            base.__init__(self, *args, **kw)

    cls = type(str(name), (base,), class_attrs)
    cls.__init__ = __init__
    cls.__module__ = __name__
    _module_globals[name] = cls
    return cls
