"""Objective functions of ``deap/benchmarks/__init__.py`` (plus OneMax from
``README.md:85-86``) as device objectives.

``benchmarks.rastrigin(pop)`` evaluates every row of a
:class:`~deap_amd.device.DevicePopulation` on the GPU, stores the weighted
fitness (``fitness.values = fit``) and returns the unweighted values as a
``[n, nobj]`` tensor.  Registered as ``toolbox.evaluate`` the objective is fused
into the generation kernel.  DTLZ functions take ``obj`` (and ``alpha`` for
DTLZ4) exactly like the reference, usually bound with
``toolbox.register("evaluate", benchmarks.dtlz2, obj=3)``.
"""
import ctypes

from .. import _lib
from ..ops import DeviceOperator


class DeviceObjective(DeviceOperator):
    kind = "evaluate"

    def __init__(self, name, ref, code, nobj=1, needs_obj=False, needs_alpha=False):
        super().__init__(name, ref)
        self.code = code
        self.fixed_nobj = nobj
        self.needs_obj = needs_obj
        self.needs_alpha = needs_alpha

    def eval_struct(self, weights, args=(), kwargs=None):
        kwargs = kwargs or {}
        ev = _lib.Eval()
        ev.fn = self.code
        obj = 0
        if self.needs_obj:
            if args:
                obj = args[0]
            elif "obj" in kwargs:
                obj = kwargs["obj"]
            else:
                raise TypeError("%s() missing required argument: 'obj'" % self.__name__)
        if self.needs_alpha:
            if len(args) > 1:
                alpha = args[1]
            elif "alpha" in kwargs:
                alpha = kwargs["alpha"]
            else:
                raise TypeError("%s() missing required argument: 'alpha'" % self.__name__)
            ev.alpha = float(alpha)
        ev.obj = int(obj)
        for i, w in enumerate(weights):
            ev.weights[i] = float(w)
        return ev

    def __call__(self, population, *args, only_invalid=False, nevals=None, **kwargs):
        from ..device import DevicePopulation
        if not isinstance(population, DevicePopulation):
            raise TypeError("deap_amd objectives evaluate DevicePopulation batches; got %r"
                            % type(population))
        ev = self.eval_struct(population.weights, args, kwargs)
        ctx = population.ctx.bind()
        c = population.c_pop()
        ptr = ctypes.c_void_p(nevals.data_ptr()) if nevals is not None else None
        _lib.call("dm_evaluate", ctx, ctypes.byref(c), ctypes.byref(ev), int(bool(only_invalid)),
                  ptr)
        return population.fitness_values()


onemax = DeviceObjective("onemax", "README.md:85-86", _lib.DM_EVAL_ONEMAX)
rastrigin = DeviceObjective("rastrigin", "deap/benchmarks/__init__.py:220-240",
                            _lib.DM_EVAL_RASTRIGIN)
rosenbrock = DeviceObjective("rosenbrock", "deap/benchmarks/__init__.py:98-118",
                             _lib.DM_EVAL_ROSENBROCK)
sphere = DeviceObjective("sphere", "deap/benchmarks/__init__.py:62-78", _lib.DM_EVAL_SPHERE)
zdt1 = DeviceObjective("zdt1", "deap/benchmarks/__init__.py:391-403", _lib.DM_EVAL_ZDT1, 2)
zdt2 = DeviceObjective("zdt2", "deap/benchmarks/__init__.py:405-419", _lib.DM_EVAL_ZDT2, 2)
zdt3 = DeviceObjective("zdt3", "deap/benchmarks/__init__.py:421-435", _lib.DM_EVAL_ZDT3, 2)
zdt4 = DeviceObjective("zdt4", "deap/benchmarks/__init__.py:437-450", _lib.DM_EVAL_ZDT4, 2)
zdt6 = DeviceObjective("zdt6", "deap/benchmarks/__init__.py:452-465", _lib.DM_EVAL_ZDT6, 2)
dtlz1 = DeviceObjective("dtlz1", "deap/benchmarks/__init__.py:467-493", _lib.DM_EVAL_DTLZ1, None,
                        needs_obj=True)
dtlz2 = DeviceObjective("dtlz2", "deap/benchmarks/__init__.py:495-521", _lib.DM_EVAL_DTLZ2, None,
                        needs_obj=True)
dtlz3 = DeviceObjective("dtlz3", "deap/benchmarks/__init__.py:523-548", _lib.DM_EVAL_DTLZ3, None,
                        needs_obj=True)
dtlz4 = DeviceObjective("dtlz4", "deap/benchmarks/__init__.py:550-577", _lib.DM_EVAL_DTLZ4, None,
                        needs_obj=True, needs_alpha=True)

__all__ = ["onemax", "rastrigin", "rosenbrock", "sphere", "zdt1", "zdt2", "zdt3", "zdt4", "zdt6",
           "dtlz1", "dtlz2", "dtlz3", "dtlz4", "DeviceObjective"]
