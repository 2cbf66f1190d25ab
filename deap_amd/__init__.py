"""deap_amd — MI355X (gfx950) engine for DEAP's per-generation population hot
path behind DEAP's own API (``creator``, ``base.Toolbox``, ``tools``,
``algorithms``, ``benchmarks``).

Populations live on the GPU as structure-of-arrays buffers
(:class:`deap_amd.device.DevicePopulation`); every stage runs as a
hand-written HIP kernel in ``libdeapmi.so`` (C ABI: ``include/deapmi.h``).
There is no CPU fallback: without the library or a GPU, device operations
raise :class:`deap_amd._lib.DeviceUnavailable`.
"""
__version__ = "0.1.0"
__revision__ = "0.1.0"  # tracks DEAP 1.3.1 semantics

from . import base, creator  # noqa: F401
from .ops import seed  # noqa: F401


def __getattr__(name):
    # lazy: tools/algorithms/benchmarks import torch
    import importlib
    if name in ("tools", "algorithms", "benchmarks", "device", "islands", "decisions",
                "checkpoint"):
        return importlib.import_module("." + name, __name__)
    raise AttributeError(name)
