"""Distribution of round 5's selTournamentDCD permutations (a keyed 4-round
balanced Feistel network on 2 hb bits, cycle-walked into [0, n)), simulated
with ideal (uniformly random) round functions: chi-square of the
position-of-i histogram against random.sample's uniform permutations.  The
round-6 library sorts Philox keys instead (nsga2.hip dcd_keys_kernel).

    python tools_gpu/dcd_perm_sim.py [ROUNDS] [SAMPLES]"""
import sys

import numpy as np
from scipy.stats import chi2


def feistel_perm(n, rng, rounds):
    hb = 1
    while (1 << (2 * hb)) < n:
        hb += 1
    mask = (1 << hb) - 1
    f = rng.integers(0, 1 << hb, size=(rounds, 1 << hb))
    out = np.empty(n, int)
    for i in range(n):
        x = i
        while True:
            left, right = x >> hb, x & mask
            for r in range(rounds):
                left, right = right, left ^ f[r][right]
            x = (left << hb) | right
            if x < n:
                break
        out[i] = x
    return out


if __name__ == "__main__":
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    samples = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    rng = np.random.default_rng(0)
    for n in (5, 8, 12, 16, 33):
        h = np.zeros((n, n))
        for _ in range(samples):
            h[np.arange(n), feistel_perm(n, rng, rounds)] += 1
        e = samples / n
        stat = ((h - e) ** 2 / e).sum()
        print("n=%2d rounds=%d chi-square p=%.3g  largest cell off uniform %.1f %%"
              % (n, rounds, chi2.sf(stat, (n - 1) ** 2), 100 * np.abs(h / e - 1).max()))
