"""Toolbox and Fitness with DEAP's semantics (``deap/base.py``).

``Toolbox`` is the plugin boundary of the hot path (``deap/base.py:33-122``):
operators are bound with :func:`functools.partial` exactly as in DEAP, so
``toolbox.register("mate", tools.cxBlend, alpha=0.5)`` reads the same.  The
device drivers in :mod:`deap_amd.algorithms` read ``pfunc.func`` /
``pfunc.args`` / ``pfunc.keywords`` to pick the kernel and its parameters.

``Fitness`` is the host-side object used when individuals are materialised
(hall of fame, ``DevicePopulation.to_individuals``); on the device the same
data lives in the ``wvalues``/``valid`` arrays of the population and the
kernels implement the same comparisons (``csrc/common.hpp`` ``fit_gt``).
"""
import copy
import functools
import operator
from collections.abc import Sequence


class Toolbox:
    """Operator registry (``deap/base.py:33-122``).

    ``clone`` defaults to :func:`copy.deepcopy` and ``map`` to :func:`map` as
    in the reference; with a device population both are subsumed by the fused
    generation kernel (the clone is the selection gather, the map is the
    evaluation launch)."""

    def __init__(self):
        self.register("clone", copy.deepcopy)
        self.register("map", map)

    def register(self, alias, function, *args, **kargs):
        """Bind ``function`` with default arguments under ``alias``
        (``deap/base.py:52-91``)."""
        bound = functools.partial(function, *args, **kargs)
        bound.__name__ = alias
        bound.__doc__ = function.__doc__
        # copy the instance dict of plain functions / operator objects, never of classes
        if not isinstance(function, type) and hasattr(function, "__dict__"):
            bound.__dict__.update(dict(function.__dict__))
        setattr(self, alias, bound)

    def unregister(self, alias):
        """``deap/base.py:93-98``"""
        delattr(self, alias)

    def decorate(self, alias, *decorators):
        """Re-register ``alias`` with its function wrapped by ``decorators``,
        applied in order (``deap/base.py:100-122``)."""
        old = getattr(self, alias)
        fn = old.func
        for deco in decorators:
            fn = deco(fn)
        self.register(alias, fn, *old.args, **old.keywords)


class Fitness:
    """Weighted fitness (``deap/base.py:125-270``).

    ``wvalues`` holds ``values * weights`` (set once on assignment), so every
    comparison is a maximisation on ``wvalues``; ``valid`` means non-empty.
    """

    weights = None
    wvalues = ()

    def __init__(self, values=()):
        if self.weights is None:
            raise TypeError("Can't instantiate abstract %r with abstract attribute weights."
                            % (self.__class__,))
        if not isinstance(self.weights, Sequence):
            raise TypeError("Attribute weights of %r must be a sequence." % (self.__class__,))
        if values:
            self.values = values

    # values <-> wvalues ---------------------------------------------------
    @property
    def values(self):
        return tuple(wv / w for wv, w in zip(self.wvalues, self.weights))

    @values.setter
    def values(self, values):
        assert len(values) == len(self.weights), \
            "Assigned values have not the same length than fitness weights"
        try:
            self.wvalues = tuple(operator.mul(v, w) for v, w in zip(values, self.weights))
        except TypeError as exc:
            raise TypeError("Both weights and assigned values must be a sequence of numbers "
                            "when assigning to values of %r. Currently assigning value(s) %r "
                            "of %r to a fitness with weights %s."
                            % (self.__class__, values, type(values), self.weights)) from exc

    @values.deleter
    def values(self):
        self.wvalues = ()

    def getValues(self):
        return self.values

    def setValues(self, values):
        self.values = values

    def delValues(self):
        del self.values

    @property
    def valid(self):
        return len(self.wvalues) != 0

    # Pareto dominance (deap/base.py:209-224): no objective worse, one better.
    def dominates(self, other, obj=slice(None)):
        better = False
        for mine, theirs in zip(self.wvalues[obj], other.wvalues[obj]):
            if mine < theirs:
                return False
            better = better or mine > theirs
        return better

    # Lexicographic comparisons on wvalues; __gt__/__ge__ are the negations of
    # __le__/__lt__ exactly as in the reference (NaN-sensitive).
    def __le__(self, other):
        return self.wvalues <= other.wvalues

    def __lt__(self, other):
        return self.wvalues < other.wvalues

    def __gt__(self, other):
        return not self <= other

    def __ge__(self, other):
        return not self < other

    def __eq__(self, other):
        return self.wvalues == other.wvalues

    def __ne__(self, other):
        return not self == other

    def __hash__(self):
        return hash(self.wvalues)

    def __deepcopy__(self, memo):
        twin = type(self)()
        twin.wvalues = self.wvalues
        return twin

    def __str__(self):
        return str(self.values if self.valid else ())

    def __repr__(self):
        return "%s.%s(%r)" % (type(self).__module__, type(self).__name__,
                              self.values if self.valid else ())
