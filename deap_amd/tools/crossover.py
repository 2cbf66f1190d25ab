"""Crossover operators (``deap/tools/crossover.py``) as device operators.

Called on a :class:`~deap_amd.device.DevicePopulation` they mate every
consecutive pair ``(2i, 2i+1)`` — the batch form of ``mate(ind1, ind2)`` — and
return the offspring population (parents untouched, as after
``toolbox.clone``).  Inside ``varAnd``/``eaSimple``/``varOr`` they only
parameterise the fused kernel.
"""
from .. import _lib
from ..ops import DeviceOperator


class _Crossover(DeviceOperator):
    kind = "mate"
    code = _lib.DM_CX_NONE

    def params(self, args, kwargs):
        return {}

    def fill(self, var, args, kwargs):
        var.cx = self.code
        for k, v in self.params(args, kwargs).items():
            setattr(var, k, v)

    def __call__(self, population, *args, decisions=None, mode=None, stream=None, **kwargs):
        from ..algorithms import _apply_variation
        return _apply_variation(population, self, args, kwargs, None, (), {}, 1.0, 0.0,
                                decisions, mode, stream)


class _TwoPoint(_Crossover):
    code = _lib.DM_CX_TWOPOINT


class _Blend(_Crossover):
    code = _lib.DM_CX_BLEND

    def params(self, args, kwargs):
        if args:
            alpha = args[0]
        elif "alpha" in kwargs:
            alpha = kwargs["alpha"]
        else:
            raise TypeError("cxBlend() missing required argument: 'alpha'")
        return {"alpha": float(alpha)}


class _SimulatedBinaryBounded(DeviceOperator):
    """Batch form mates every pair (2i, 2i+1); inside ``varBounded`` it
    parameterises the fused NSGA-II variation kernel (``dm_vary_bounded``)."""
    kind = "mate"

    def params(self, args, kwargs):
        from ._bounded import sbx_params
        return sbx_params(args, kwargs)

    def __call__(self, population, *args, decisions=None, mode=None, stream=None, **kwargs):
        from ._bounded import vary_bounded
        # every pair is mated: the pair gate random() <= 1.0 always holds
        return vary_bounded(population, None, self.params(args, kwargs), None, 1.0,
                            decisions, mode, stream)


cxTwoPoint = _TwoPoint("cxTwoPoint", "deap/tools/crossover.py:37-60")
cxBlend = _Blend("cxBlend", "deap/tools/crossover.py:241-260")

cxSimulatedBinaryBounded = _SimulatedBinaryBounded("cxSimulatedBinaryBounded",
                                                   "deap/tools/crossover.py:291-360")

__all__ = ["cxTwoPoint", "cxBlend", "cxSimulatedBinaryBounded"]
