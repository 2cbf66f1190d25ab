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


cxTwoPoint = _TwoPoint("cxTwoPoint", "deap/tools/crossover.py:37-60")
cxBlend = _Blend("cxBlend", "deap/tools/crossover.py:241-260")

__all__ = ["cxTwoPoint", "cxBlend"]
