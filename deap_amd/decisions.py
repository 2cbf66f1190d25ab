"""Pre-drawn random decisions in DEAP's vocabulary (``struct dm_decisions``).

Parity with the reference is defined on decisions: the
tournament aspirants drawn by ``selRandom`` (``deap/tools/selection.py:24``),
the crossover flag and raw ``randint`` cut draws of ``varAnd``/``cxTwoPoint``
(``deap/algorithms.py:72``, ``deap/tools/crossover.py:50-51``), the per-gene
``random()`` of ``cxBlend`` (``crossover.py:256``), the mutation flag and
per-gene mask of ``mutFlipBit``/``mutGaussian`` and the ``random.gauss``
value added (``deap/tools/mutation.py:44-46, 139-141``), and the varOr op
choice plus sampled indices (``deap/algorithms.py:231-243``).

``mode="inject"`` feeds them to the kernels; ``mode="dump"`` lets the kernels
draw natively and write every decision here, so the same decisions can be
replayed into DEAP (``tests/golden``) or into the CPU oracle.
"""
import ctypes

import numpy as np

from . import _lib
from .device import zeros as _zeros

FIELDS = ("aspirants", "cx_flag", "cx_raw", "blend_u", "mut_flag", "mut_mask", "gauss",
          "varor_op", "varor_idx")


class Decisions:
    def __init__(self, **tensors):
        for f in FIELDS:
            setattr(self, f, tensors.get(f))

    @classmethod
    def allocate(cls, k, dim, device, tournsize=0, cx=True, blend=False, mut=True, gauss=False,
                 varor=False):
        """Zeroed buffers sized for ``k`` children (dump mode)."""
        import torch
        kw = {}
        words = (dim + 63) // 64
        npairs = k if varor else k // 2
        if tournsize:
            kw["aspirants"] = _zeros((k, tournsize), torch.int32, device)
        if cx:
            kw["cx_flag"] = _zeros((max(npairs, 1),), torch.uint8, device)
            kw["cx_raw"] = _zeros((max(npairs, 1), 2), torch.int32, device)
        if blend:
            kw["blend_u"] = _zeros((max(npairs, 1), dim), torch.float64, device)
        if mut:
            kw["mut_flag"] = _zeros((k,), torch.uint8, device)
            kw["mut_mask"] = _zeros((k, words), torch.int64, device)
        if gauss:
            kw["gauss"] = _zeros((k, dim), torch.float64, device)
        if varor:
            kw["varor_op"] = _zeros((k,), torch.int32, device)
            kw["varor_idx"] = _zeros((k, 2), torch.int32, device)
        return cls(**kw)

    @classmethod
    def from_numpy(cls, device, **arrays):
        """Upload host arrays (inject mode).  ``mut_mask`` may be given as a
        ``[k, dim]`` 0/1 matrix; it is packed to uint64 words."""
        import torch
        from .device import pack_bits
        kw = {}
        dtypes = {"aspirants": np.int32, "cx_flag": np.uint8, "cx_raw": np.int32,
                  "blend_u": np.float64, "mut_flag": np.uint8, "gauss": np.float64,
                  "varor_op": np.int32, "varor_idx": np.int32}
        for name, arr in arrays.items():
            if arr is None:
                continue
            if name not in FIELDS:
                raise KeyError(name)
            a = np.asarray(arr)
            if name == "mut_mask":
                if a.dtype != np.uint64 and a.dtype != np.int64:
                    a = pack_bits(a)
                a = np.ascontiguousarray(a).view(np.int64)
            else:
                a = np.ascontiguousarray(a, dtype=dtypes[name])
            if a.size == 0:
                a = np.zeros((1,) + a.shape[1:], a.dtype)
            kw[name] = torch.from_numpy(a).to(device)
        return cls(**kw)

    def numpy(self):
        out = {}
        for f in FIELDS:
            t = getattr(self, f)
            if t is not None:
                a = t.cpu().numpy()
                out[f] = a.view(np.uint64) if f == "mut_mask" else a
        return out

    def c_struct(self):
        d = _lib.Decisions()
        for f in FIELDS:
            t = getattr(self, f)
            setattr(d, f, ctypes.c_void_p(t.data_ptr()) if t is not None else None)
        return d
