"""Population initialisation on the device (stand-in for
``tools.initRepeat``/``initIterate``, ``deap/tools/init.py:3-51``: the
reference draws genes one by one from ``random``; here rows are drawn from the
counter-based stream so a 2^20-row population never touches the host)."""
import ctypes

from .. import _lib
from ..device import DevicePopulation, gtype_of
from ..ops import default_stream


def initPopulation(individual_class=None, n=0, dim=0, low=0.0, high=1.0, *, gtype=None,
                   weights=None, device=None, capacity=None, stream=None):
    """``n`` individuals of ``dim`` genes: bits i.i.d. Bernoulli(1/2)
    (``random.randint(0, 1)``), floats ``random.uniform(low, high)``.
    ``individual_class`` is a ``creator`` type whose ``typecode`` and
    ``fitness.weights`` pick the genome type and fitness weights."""
    if weights is None:
        fit_cls = None
        if individual_class is not None:
            fit_cls = _fitness_class(individual_class)
        weights = fit_cls.weights if fit_cls is not None else (1.0,)
    gt = gtype_of(individual_class, gtype=gtype)
    pop = DevicePopulation(n, dim, gt, weights, device, capacity, individual_class)
    stream = stream or default_stream()
    ctx = pop.ctx.bind()
    _lib.call("dm_init_uniform", ctx, ctypes.byref(pop.c_pop()), float(low), float(high),
              stream.next())
    return pop


def _fitness_class(individual_class):
    try:
        probe = individual_class()
    except TypeError:
        probe = None
    fit = getattr(probe, "fitness", None)
    return type(fit) if fit is not None else None


__all__ = ["initPopulation"]
