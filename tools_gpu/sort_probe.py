"""Per-kernel cost of the pair sort's paths (sort.hip): run under
``rocprofv3 --kernel-trace`` and read the kernel durations in call order.

usage: python tools_gpu/sort_probe.py   (prints the config order it ran)"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from deap_amd import _lib  # noqa: E402
from deap_amd.device import Context  # noqa: E402

CONFIGS = [  # (nseg, seglen, end_bit)
    (1, 64, 64), (1, 1024, 64), (1, 4096, 8), (1, 4096, 16), (1, 4096, 32), (1, 4096, 64),
    (1, 1 << 18, 64), (2, 212_480, 64), (1, 1 << 18, 32),
]
REPS = 10


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    fn = lib.dm_test_sort_pairs
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                   ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    ctx = Context.get(dev)
    rng = np.random.default_rng(0)
    for nseg, seglen, end in CONFIGS:
        n = nseg * seglen
        base = torch.from_numpy(rng.integers(0, 2**63, n, dtype=np.int64)).to(dev)
        vals = torch.arange(n, dtype=torch.int32, device=dev)
        for _ in range(REPS):
            k = base.clone()
            _lib.check(fn(ctx.handle, ctypes.c_void_p(k.data_ptr()), ctypes.c_void_p(vals.data_ptr()),
                          nseg, seglen, 0, end), "sort")
        print("config", nseg, seglen, end, flush=True)


if __name__ == "__main__":
    main()
