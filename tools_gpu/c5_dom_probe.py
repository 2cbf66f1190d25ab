"""Fixed-input selNSGA2 for kernel A/B under rocprofv3: 2N = 2^18 DTLZ2-shaped
fitnesses (directions on the unit sphere scaled by 1 + g), selNSGA2 to N,
`reps` times (argv[1], default 5).  Library variants come via DEAPMI_LIB."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from deap_amd import tools
from deap_amd.device import DevicePopulation
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
m = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = 1 << 18
rng = np.random.default_rng(103)
d = np.abs(rng.normal(size=(n, m)))
d /= np.linalg.norm(d, axis=1, keepdims=True)
wv = -(d * (1.0 + rng.exponential(0.3, size=(n, 1))))
pop = DevicePopulation.from_numpy(np.zeros((n, 1)), weights=(-1.0,) * m, gtype="f64", wvalues=wv,
                                  valid=np.ones(n))
tools.selNSGA2(pop, n // 2)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    ch = tools.selNSGA2(pop, n // 2)
torch.cuda.synchronize()
print("selNSGA2 2^18 -> 2^17: %.3f ms per call" % ((time.perf_counter() - t0) / reps * 1e3))
