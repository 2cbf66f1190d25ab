"""LDS bank cycles of the count pass's prefix-set reads (bitdom.hip
bd_count_kernel): each lane reads the four 16-B pieces of ONE random 64-B set
per objective (k = its local rank bound, uniform over the chunk's 513 sets),
piece j = (step + lane) & 3, by ds_read_b128.  gfx950 services a b128 read in
4 groups of 16 lanes, one LDS cycle per group when the 16 pieces fall in 16
distinct 16-B bank quads (bank of byte a = (a / 4) mod 64); identical addresses
broadcast (MI355X_MICROARCH.md, LDS).  Prints the expected cycles per group per
read (1.0 = conflict-free) for the layout in use and for swizzled ones.

    python tools_gpu/lds_conflict_sim.py
"""
import numpy as np

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[lane + 32 for lane in g] for g in GROUPS]


def cycles(quad, trials=4000, seed=1):
    rng = np.random.default_rng(seed)
    tot = 0
    for _ in range(trials):
        k = rng.integers(0, 513, 64)
        for step in range(4):
            for g in GROUPS:
                load = {}
                for lane in g:
                    j = (step + (lane & 3)) & 3
                    load.setdefault(quad(int(k[lane]), j) % 16, set()).add((int(k[lane]), j))
                tot += max(len(v) for v in load.values())
    return tot / (trials * 4 * len(GROUPS))


LAYOUTS = {
    "in use: set k at 64 k, lane-rotated pieces": lambda k, j: 4 * (k & 3) + j,
    "sets padded to 80 B": lambda k, j: 5 * k + j,
    "piece index XOR (k >> 2) & 3": lambda k, j: 4 * (k & 3) + (j ^ ((k >> 2) & 3)),
    "piece index XOR k & 3 (rotate by k mod 4)": lambda k, j: 4 * (k & 3) + ((j + k) & 3),
}

if __name__ == "__main__":
    for name, fn in LAYOUTS.items():
        print("%-45s %.3f cycles per lane group per read" % (name, cycles(fn)))
