#!/usr/bin/env python3
"""Case files for the bdemu harness (format in harness.cpp).

golden<j>.bin: the six sortNondominated golden vectors of tests/golden/nsga2.npz
(weighted fitness, k, the reference's order and front starts; case 4 is the
n = 64, M = 4 input whose first m = 4 bitset call faulted on the GPU in round 4).
rand_m<M>_n<N>_<kind>.bin: seeded synthetic inputs without a reference order
(checked against the harness's brute-force sort): small integer objectives
(many ties and duplicated fitnesses) and continuous points near a sphere shell.
"""
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def write(path, wv, k, order=None, fstart=None):
    wv = np.ascontiguousarray(wv, dtype=np.float64)
    n, m = wv.shape
    with open(path, "wb") as f:
        f.write(b"BDE1")
        f.write(struct.pack("<qiq", n, m, int(k)))
        f.write(wv.tobytes())
        order = np.zeros(0, np.int32) if order is None else np.asarray(order, np.int32)
        f.write(struct.pack("<q", len(order)))
        f.write(order.tobytes())
        fs = np.zeros(1, np.int32) if fstart is None else np.asarray(fstart, np.int32)
        f.write(struct.pack("<i", len(fs) - 1))
        f.write(fs.tobytes())


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "build", "cases")
    os.makedirs(out, exist_ok=True)
    d = np.load(os.path.join(REPO, "tests", "golden", "nsga2.npz"))
    j = 0
    while "nd%d_wv" % j in d.files:
        p = "nd%d_" % j
        write(os.path.join(out, "golden%d.bin" % j), d[p + "wv"], int(d[p + "k"]), d[p + "order"],
              d[p + "fstart"])
        j += 1
    rng = np.random.default_rng(20261018)
    for m in (2, 3, 4):
        for n in (64, 777, 4096):
            wv = rng.integers(0, 12 if n < 1000 else 40, size=(n, m)).astype(np.float64)
            write(os.path.join(out, "rand_m%d_n%d_int.bin" % (m, n)), wv, n)
            x = rng.standard_normal((n, m))
            x = np.abs(x) / np.linalg.norm(x, axis=1, keepdims=True) * (1 + 0.3 * rng.random((n, 1)))
            write(os.path.join(out, "rand_m%d_n%d_shell.bin" % (m, n)), -x, n // 2)


if __name__ == "__main__":
    main()
