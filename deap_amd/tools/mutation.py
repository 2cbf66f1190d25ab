"""Mutation operators (``deap/tools/mutation.py``) as device operators.

Called on a population they mutate every individual (the batch form of
``mutate(ind)``) and return the mutants; inside the drivers they parameterise
the fused kernel.
"""
from collections.abc import Sequence

from .. import _lib
from ..ops import DeviceOperator


class _Mutation(DeviceOperator):
    kind = "mutate"
    code = _lib.DM_MUT_NONE

    def fill(self, var, args, kwargs, population=None):
        var.mut = self.code
        for k, v in self.params(args, kwargs, population).items():
            setattr(var, k, v)

    def __call__(self, population, *args, decisions=None, mode=None, stream=None, **kwargs):
        from ..algorithms import _apply_variation
        return _apply_variation(population, None, (), {}, self, args, kwargs, 0.0, 1.0,
                                decisions, mode, stream)


def _arg(args, kwargs, pos, name):
    if len(args) > pos:
        return args[pos]
    if name in kwargs:
        return kwargs[name]
    raise TypeError("missing required argument: '%s'" % name)


class _FlipBit(_Mutation):
    code = _lib.DM_MUT_FLIPBIT

    def params(self, args, kwargs, population=None):
        return {"indpb": float(_arg(args, kwargs, 0, "indpb"))}


class _Gaussian(_Mutation):
    code = _lib.DM_MUT_GAUSSIAN

    def params(self, args, kwargs, population=None):
        mu = _arg(args, kwargs, 0, "mu")
        sigma = _arg(args, kwargs, 1, "sigma")
        indpb = float(_arg(args, kwargs, 2, "indpb"))
        out = {"indpb": indpb, "mu": 0.0, "sigma": 1.0, "mu_vec": None, "sigma_vec": None}
        size = population.dim if population is not None else None
        keep = []
        for name, val in (("mu", mu), ("sigma", sigma)):
            if isinstance(val, Sequence):
                # deap/tools/mutation.py:37-42
                if size is not None and len(val) < size:
                    raise IndexError("%s must be at least the size of individual: %d < %d"
                                     % (name, len(val), size))
                import torch
                t = torch.tensor([float(x) for x in val], dtype=torch.float64,
                                 device=population.device)
                keep.append(t)
                out[name + "_vec"] = t.data_ptr()
            else:
                out[name] = float(val)
        out["_keepalive"] = keep
        return out

    def fill(self, var, args, kwargs, population=None):
        var.mut = self.code
        p = self.params(args, kwargs, population)
        var._keepalive = p.pop("_keepalive")
        for k, v in p.items():
            setattr(var, k, v)


class _PolynomialBounded(DeviceOperator):
    """Batch form mutates every individual; inside ``varBounded`` it
    parameterises the fused NSGA-II variation kernel (``dm_vary_bounded``)."""
    kind = "mutate"

    def params(self, args, kwargs, population=None):
        from ._bounded import poly_params
        return poly_params(args, kwargs)

    def __call__(self, population, *args, decisions=None, mode=None, stream=None, **kwargs):
        from ._bounded import vary_bounded
        return vary_bounded(population, None, None, self.params(args, kwargs), 0.0,
                            decisions, mode, stream)


mutFlipBit = _FlipBit("mutFlipBit", "deap/tools/mutation.py:124-142")
mutGaussian = _Gaussian("mutGaussian", "deap/tools/mutation.py:17-48")

mutPolynomialBounded = _PolynomialBounded("mutPolynomialBounded", "deap/tools/mutation.py:51-95")

__all__ = ["mutFlipBit", "mutGaussian", "mutPolynomialBounded"]
