#!/usr/bin/env python3
"""Generate the golden vectors that pin the oracle — run in the BUILD
container only (needs /root/reference; the fixtures it writes travel, the
reference does not).

The reference (DEAP 1.3.1, Python-2 source) is made importable exactly as its
own setup.py prescribes (``use_2to3=True``, setup.py:90): a scratch copy under
/tmp is converted with lib2to3.  Nothing from it is copied into the repo.

Parity is defined on random *decisions*: DEAP draws through the module-level
functions ``random.random / randint / choice / gauss / sample``; they are
replaced by iterators over pre-drawn decision arrays in DEAP's consumption
order, so DEAP consumes exactly the decisions the GPU and the oracle get.
The C1 trajectory (README OneMax, examples/ga/onemax_short.py, seed 64) is
recorded the other way round: DEAP runs with the real Mersenne Twister and a
recording wrapper captures every decision it draws.

Usage:  python tests/golden/make_golden.py            # writes tests/golden/*.npz
"""
import array
import importlib
import os
import random
import shutil
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/deap"
SCRATCH = "/tmp/deap_oracle"
NOT_TAKEN = 1.0 - 2.0 ** -53  # random() value that fails every `< p` test with p < 1
TAKEN = 0.0


def load_reference():
    if not os.path.isdir(os.path.join(SCRATCH, "deap")):
        shutil.rmtree(SCRATCH, ignore_errors=True)
        os.makedirs(SCRATCH)
        shutil.copytree(REF, os.path.join(SCRATCH, "deap"))
        for root, dirs, files in os.walk(SCRATCH):
            for f in files + dirs:
                os.chmod(os.path.join(root, f), 0o755)
        subprocess.check_call([sys.executable, "-W", "ignore", "-m", "lib2to3", "-w", "-n",
                               "deap"], cwd=SCRATCH, stdout=subprocess.DEVNULL,
                              stderr=subprocess.DEVNULL)
    sys.path.insert(0, SCRATCH)
    mods = {}
    for name in ("deap", "deap.base", "deap.creator", "deap.tools", "deap.algorithms",
                 "deap.benchmarks", "deap.tools.emo"):
        mods[name] = importlib.import_module(name)
    return mods


class Replay:
    """Module-level random stubs served from per-function queues."""

    def __init__(self, floats=(), ints=(), choices=(), gausses=(), samples=()):
        self.q = {"random": list(floats), "randint": list(ints), "choice": list(choices),
                  "gauss": list(gausses), "sample": list(samples)}
        self.saved = {}

    def __enter__(self):
        for name in ("random", "randint", "choice", "gauss", "sample"):
            self.saved[name] = getattr(random, name)
        q = self.q
        random.random = lambda: q["random"].pop(0)
        random.randint = lambda a, b: q["randint"].pop(0)
        random.choice = lambda seq: seq[q["choice"].pop(0)]
        random.gauss = lambda mu, sigma: q["gauss"].pop(0)
        random.sample = lambda seq, k: [seq[i] for i in q["sample"].pop(0)]
        return self

    def __exit__(self, *exc):
        for name, fn in self.saved.items():
            setattr(random, name, fn)
        for name, left in self.q.items():
            assert not left, "unconsumed %s decisions: %d" % (name, len(left))


def flag(b):
    return TAKEN if b else NOT_TAKEN


def make_types(D, typecode, weights):
    creator = D["deap.creator"]
    base = D["deap.base"]
    for name in ("FitG", "IndG"):
        if hasattr(creator, name):
            delattr(creator, name)
    creator.create("FitG", base.Fitness, weights=weights)
    if typecode == "list":
        creator.create("IndG", list, fitness=creator.FitG)
    else:
        creator.create("IndG", array.array, typecode=typecode, fitness=creator.FitG)
    return creator.IndG


def to_inds(Ind, genes, wvalues=None, valid=None):
    out = []
    for i, row in enumerate(genes):
        ind = Ind([int(x) for x in row] if genes.dtype == np.uint8 else [float(x) for x in row])
        if wvalues is not None and (valid is None or valid[i]):
            ind.fitness.values = tuple(float(w) / float(ww) for w, ww in
                                       zip(wvalues[i], ind.fitness.weights))
        out.append(ind)
    return out


def from_inds(inds, dtype, m):
    genes = np.array([list(ind) for ind in inds], dtype=dtype)
    wv = np.array([ind.fitness.wvalues if ind.fitness.valid else (0.0,) * m for ind in inds],
                  np.float64)
    valid = np.array([ind.fitness.valid for ind in inds], bool)
    return genes, wv, valid


# ---------------------------------------------------------------------------
def gen_eval(D, rng):
    bm = D["deap.benchmarks"]
    out = {}
    cases = [("rastrigin", 1000, (-5.12, 5.12), {}), ("rastrigin", 37, (-50, 50), {}),
             ("rosenbrock", 1000, (-2.048, 2.048), {}), ("rosenbrock", 13, (-3, 3), {}),
             ("sphere", 64, (-1, 1), {}),
             ("zdt1", 30, (0, 1), {}), ("zdt2", 30, (0, 1), {}), ("zdt3", 30, (0, 1), {}),
             ("zdt4", 10, (0, 1), {}), ("zdt6", 10, (0, 1), {}),
             ("dtlz1", 7, (0, 1), {"obj": 3}), ("dtlz2", 12, (0, 1), {"obj": 3}),
             ("dtlz3", 12, (0, 1), {"obj": 3}), ("dtlz4", 12, (0, 1), {"obj": 3, "alpha": 100}),
             ("dtlz2", 14, (0, 1), {"obj": 5})]
    for j, (name, dim, (lo, hi), kw) in enumerate(cases):
        n = 24
        x = rng.uniform(lo, hi, size=(n, dim))
        if name.startswith("zdt4"):
            x[:, 1:] = rng.uniform(-5, 5, size=(n, dim - 1))
        fn = getattr(bm, name)
        vals = np.array([fn(list(map(float, row)), **kw) for row in x], np.float64)
        out["eval%d_x" % j] = x
        out["eval%d_f" % j] = vals
        out["eval%d_meta" % j] = np.array([name, str(kw)])
    # OneMax (README) on 0/1 genomes
    bits = rng.integers(0, 2, size=(32, 100)).astype(np.uint8)
    out["onemax_x"] = bits
    out["onemax_f"] = bits.sum(axis=1).astype(np.float64)
    # float32 genomes: DEAP evaluates the stored fp32 values widened to fp64
    x32 = rng.uniform(-5.12, 5.12, size=(16, 100)).astype(np.float32)
    Ind = make_types(D, "f", (-1.0,))
    out["rastrigin_f32_x"] = x32
    out["rastrigin_f32_f"] = np.array([bm.rastrigin(Ind(list(map(float, r))))[0] for r in x32])
    return out


def gen_varand(D, rng):
    algorithms = D["deap.algorithms"]
    tools = D["deap.tools"]
    base = D["deap.base"]
    out = {}
    cases = [("bits", "list", 100, 40, "twopoint", "flipbit"),
             ("bits", "b", 4096, 10, "twopoint", "flipbit"),
             ("f64", "d", 1000, 12, "blend", "gaussian"),
             ("f64", "d", 30, 33, "twopoint", "gaussian"),
             ("f32", "f", 50, 20, "blend", "gaussian")]
    for j, (gt, tc, dim, n, cx, mut) in enumerate(cases):
        Ind = make_types(D, tc, (1.0,))
        if gt == "bits":
            genes = rng.integers(0, 2, size=(n, dim)).astype(np.uint8)
        else:
            genes = rng.uniform(-5, 5, size=(n, dim)).astype(np.float32 if gt == "f32"
                                                              else np.float64)
        wv = rng.integers(0, 50, size=(n, 1)).astype(np.float64)
        valid = np.ones(n, bool)
        cxpb, mutpb, indpb, alpha = 0.5, 0.3, 0.05, 0.5
        npairs = n // 2
        cx_flag = rng.random(npairs) < cxpb
        cx_raw = np.stack([rng.integers(1, dim + 1, npairs), rng.integers(1, dim, npairs)], 1)
        blend_u = rng.random((npairs, dim))
        mut_flag = rng.random(n) < mutpb
        mask = rng.random((n, dim)) < indpb
        gauss = rng.normal(0.0, 1.0, size=(n, dim))
        floats, ints, gausses = [], [], []
        for p in range(npairs):
            floats.append(flag(cx_flag[p]))
            if cx_flag[p]:
                if cx == "twopoint":
                    ints.extend(int(v) for v in cx_raw[p])
                else:
                    floats.extend(float(v) for v in blend_u[p])
        for i in range(n):
            floats.append(flag(mut_flag[i]))
            if mut_flag[i]:
                for g in range(dim):
                    floats.append(flag(mask[i, g]))
                    if mut == "gaussian" and mask[i, g]:
                        gausses.append(float(gauss[i, g]))
        tb = base.Toolbox()
        if cx == "twopoint":
            tb.register("mate", tools.cxTwoPoint)
        else:
            tb.register("mate", tools.cxBlend, alpha=alpha)
        if mut == "flipbit":
            tb.register("mutate", tools.mutFlipBit, indpb=indpb)
        else:
            tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=indpb)
        pop = to_inds(Ind, genes, wv, valid)
        with Replay(floats=floats, ints=ints, gausses=gausses):
            off = algorithms.varAnd(pop, tb, cxpb, mutpb)
        og, owv, ovalid = from_inds(off, genes.dtype, 1)
        key = "va%d_" % j
        out.update({key + "genes": genes, key + "wv": wv, key + "valid": valid,
                    key + "cx_flag": cx_flag, key + "cx_raw": cx_raw, key + "blend_u": blend_u,
                    key + "mut_flag": mut_flag, key + "mask": mask, key + "gauss": gauss,
                    key + "out_genes": og, key + "out_wv": owv, key + "out_valid": ovalid,
                    key + "meta": np.array([gt, tc, cx, mut, str(cxpb), str(mutpb),
                                            str(indpb), str(alpha)])})
    return out


def gen_selection(D, rng):
    tools = D["deap.tools"]
    out = {}
    for j, (n, m, t) in enumerate([(64, 1, 3), (40, 2, 4), (33, 3, 2)]):
        weights = tuple([1.0, -1.0, 1.0][:m])
        Ind = make_types(D, "d", weights)
        wv = rng.integers(0, 6, size=(n, m)).astype(np.float64)  # heavy ties
        genes = rng.uniform(0, 1, size=(n, 3))
        pop = to_inds(Ind, genes, wv)
        k = n
        asp = rng.integers(0, n, size=(k, t))
        with Replay(choices=[int(a) for a in asp.ravel()]):
            chosen = tools.selTournament(pop, k, tournsize=t)
        idx = [next(i for i, p in enumerate(pop) if p is c) for c in chosen]
        best = tools.selBest(pop, 10)
        worst = tools.selWorst(pop, 10)
        key = "sel%d_" % j
        out.update({key + "wv": wv, key + "asp": asp, key + "out": np.array(idx),
                    key + "best": np.array([next(i for i, p in enumerate(pop) if p is c)
                                            for c in best]),
                    key + "worst": np.array([next(i for i, p in enumerate(pop) if p is c)
                                             for c in worst]),
                    key + "weights": np.array(weights)})
    return out


def gen_ea_generation(D, rng):
    """One eaSimple generation body (select -> varAnd -> evaluate invalid)
    with replayed decisions, for the fused kernel."""
    algorithms = D["deap.algorithms"]
    tools = D["deap.tools"]
    base = D["deap.base"]
    bm = D["deap.benchmarks"]
    out = {}
    cases = [("f64", "d", 1000, 16, "blend", "gaussian", "rastrigin", (-1.0,)),
             ("f64", "d", 100, 21, "blend", "gaussian", "rosenbrock", (-1.0,)),
             ("bits", "b", 4096, 16, "twopoint", "flipbit", "onemax", (1.0,)),
             ("bits", "list", 100, 30, "twopoint", "flipbit", "onemax", (1.0,))]
    for j, (gt, tc, dim, n, cx, mut, objective, weights) in enumerate(cases):
        Ind = make_types(D, tc, weights)
        if gt == "bits":
            genes = rng.integers(0, 2, size=(n, dim)).astype(np.uint8)
        else:
            genes = rng.uniform(-5.12, 5.12, size=(n, dim))
        if objective == "onemax":
            evalf = lambda ind: (sum(ind),)  # noqa: E731 - README.md:85-86
        else:
            evalf = getattr(bm, objective)
        pop = to_inds(Ind, genes)
        for ind in pop:
            ind.fitness.values = evalf(ind)
        genes0, wv0, valid0 = from_inds(pop, genes.dtype, 1)
        t, cxpb, mutpb, indpb, alpha = 3, 0.5, 0.2, 0.05, 0.5
        asp = rng.integers(0, n, size=(n, t))
        npairs = n // 2
        cx_flag = rng.random(npairs) < cxpb
        cx_raw = np.stack([rng.integers(1, dim + 1, npairs), rng.integers(1, dim, npairs)], 1)
        blend_u = rng.random((npairs, dim))
        mut_flag = rng.random(n) < mutpb
        mask = rng.random((n, dim)) < indpb
        gauss = rng.normal(0.0, 1.0, size=(n, dim))
        floats, ints, gausses = [], [], []
        for p in range(npairs):
            floats.append(flag(cx_flag[p]))
            if cx_flag[p]:
                if cx == "twopoint":
                    ints.extend(int(v) for v in cx_raw[p])
                else:
                    floats.extend(float(v) for v in blend_u[p])
        for i in range(n):
            floats.append(flag(mut_flag[i]))
            if mut_flag[i]:
                for g in range(dim):
                    floats.append(flag(mask[i, g]))
                    if mut == "gaussian" and mask[i, g]:
                        gausses.append(float(gauss[i, g]))
        tb = base.Toolbox()
        tb.register("evaluate", evalf)
        tb.register("select", tools.selTournament, tournsize=t)
        if cx == "twopoint":
            tb.register("mate", tools.cxTwoPoint)
        else:
            tb.register("mate", tools.cxBlend, alpha=alpha)
        if mut == "flipbit":
            tb.register("mutate", tools.mutFlipBit, indpb=indpb)
        else:
            tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=indpb)
        with Replay(floats=floats, ints=ints, gausses=gausses,
                    choices=[int(a) for a in asp.ravel()]):
            pop2, log = algorithms.eaSimple(pop, tb, cxpb, mutpb, 1, verbose=False)
        og, owv, ovalid = from_inds(pop2, genes.dtype, 1)
        key = "ea%d_" % j
        out.update({key + "genes": genes0, key + "wv": wv0, key + "valid": valid0,
                    key + "asp": asp, key + "cx_flag": cx_flag, key + "cx_raw": cx_raw,
                    key + "blend_u": blend_u, key + "mut_flag": mut_flag, key + "mask": mask,
                    key + "gauss": gauss, key + "out_genes": og, key + "out_wv": owv,
                    key + "out_valid": ovalid,
                    key + "nevals": np.array(log.select("nevals")),
                    key + "meta": np.array([gt, tc, cx, mut, objective, str(t), str(cxpb),
                                            str(mutpb), str(indpb), str(alpha), str(weights[0])])})
    return out


def gen_varor(D, rng):
    algorithms = D["deap.algorithms"]
    tools = D["deap.tools"]
    base = D["deap.base"]
    out = {}
    cases = [("f64", "d", 12, 20, 30, "blend", "gaussian"),
             ("bits", "list", 70, 16, 25, "twopoint", "flipbit")]
    for j, (gt, tc, dim, n, lam, cx, mut) in enumerate(cases):
        Ind = make_types(D, tc, (-1.0, -1.0))
        genes = (rng.integers(0, 2, size=(n, dim)).astype(np.uint8) if gt == "bits"
                 else rng.uniform(0, 1, size=(n, dim)))
        wv = rng.uniform(-5, 0, size=(n, 2))
        valid = np.ones(n, bool)
        pop = to_inds(Ind, genes, wv, valid)
        cxpb, mutpb, indpb, alpha = 0.5, 0.3, 0.1, 0.5
        op_u = rng.random(lam)
        op = np.where(op_u < cxpb, 0, np.where(op_u < cxpb + mutpb, 1, 2))
        idx = np.zeros((lam, 2), np.int64)
        cx_raw = np.stack([rng.integers(1, dim + 1, lam), rng.integers(1, dim, lam)], 1)
        blend_u = rng.random((lam, dim))
        mask = rng.random((lam, dim)) < indpb
        gauss = rng.normal(0, 1, size=(lam, dim))
        floats, ints, choices, gausses, samples = [], [], [], [], []
        for c in range(lam):
            floats.append(float(op_u[c]))
            if op[c] == 0:
                a, b = rng.choice(n, 2, replace=False)
                idx[c] = (a, b)
                samples.append([int(a), int(b)])
                if cx == "twopoint":
                    ints.extend(int(v) for v in cx_raw[c])
                else:
                    floats.extend(float(v) for v in blend_u[c])
            else:
                a = int(rng.integers(0, n))
                idx[c] = (a, 0)
                choices.append(a)
                if op[c] == 1:
                    for g in range(dim):
                        floats.append(flag(mask[c, g]))
                        if mut == "gaussian" and mask[c, g]:
                            gausses.append(float(gauss[c, g]))
        tb = base.Toolbox()
        if cx == "twopoint":
            tb.register("mate", tools.cxTwoPoint)
        else:
            tb.register("mate", tools.cxBlend, alpha=alpha)
        if mut == "flipbit":
            tb.register("mutate", tools.mutFlipBit, indpb=indpb)
        else:
            tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=indpb)
        with Replay(floats=floats, ints=ints, choices=choices, gausses=gausses, samples=samples):
            off = algorithms.varOr(pop, tb, lam, cxpb, mutpb)
        og, owv, ovalid = from_inds(off, genes.dtype, 2)
        key = "vo%d_" % j
        out.update({key + "genes": genes, key + "wv": wv, key + "valid": valid,
                    key + "op": op, key + "op_u": op_u, key + "idx": idx, key + "cx_raw": cx_raw,
                    key + "blend_u": blend_u, key + "mask": mask, key + "gauss": gauss,
                    key + "out_genes": og, key + "out_wv": owv, key + "out_valid": ovalid,
                    key + "meta": np.array([gt, tc, cx, mut, str(lam), str(cxpb), str(mutpb),
                                            str(indpb), str(alpha)])})
    return out


def gen_nsga2(D, rng):
    tools = D["deap.tools"]
    emo = D["deap.tools.emo"]
    out = {}
    cases = [(200, 2, "ties", 100), (300, 3, "ties", 150), (257, 3, "cont", 128),
             (120, 2, "dups", 60), (64, 4, "ties", 64), (150, 3, "cont", 500)]
    for j, (n, m, kind, k) in enumerate(cases):
        weights = tuple([-1.0, -1.0, 1.0, -1.0][:m])
        Ind = make_types(D, "d", weights)
        if kind == "ties":
            vals = rng.integers(0, 7, size=(n, m)).astype(np.float64)
        elif kind == "dups":
            base_pts = rng.uniform(0, 1, size=(n // 4, m))
            vals = base_pts[rng.integers(0, n // 4, n)]
        else:
            vals = rng.uniform(0, 1, size=(n, m))
        wv = vals * np.array(weights)
        genes = rng.uniform(0, 1, size=(n, 2))
        pop = to_inds(Ind, genes, wv)
        ident = {id(p): i for i, p in enumerate(pop)}
        fronts = tools.sortNondominated(pop, k)
        flat = [ident[id(p)] for f in fronts for p in f]
        fstart = np.cumsum([0] + [len(f) for f in fronts])
        # crowding on each front (emo.assignCrowdingDist is not exported)
        for f in fronts:
            emo.assignCrowdingDist(f)
        crowd = np.array([pop[i].fitness.crowding_dist for i in flat])
        pop2 = to_inds(Ind, genes, wv)
        ident2 = {id(p): i for i, p in enumerate(pop2)}
        chosen = tools.selNSGA2(pop2, k)
        key = "nd%d_" % j
        out.update({key + "wv": wv, key + "weights": np.array(weights), key + "k": np.array(k),
                    key + "order": np.array(flat), key + "fstart": fstart,
                    key + "crowd": crowd,
                    key + "chosen": np.array([ident2[id(p)] for p in chosen])})
        ff = tools.sortNondominated(to_inds(Ind, genes, wv), k, first_front_only=True)
        out[key + "first"] = np.array([len(ff[0])])
    return out


def gen_dcd(D, rng):
    """selTournamentDCD (emo.py:145-195): two random.sample permutations and a
    random() coin for each tied tournament, fed in DEAP's call order."""
    tools = D["deap.tools"]
    out = {}
    cases = [(64, 2, 64), (100, 3, 37), (40, 2, 40), (200, 3, 120), (33, 2, 30)]
    for j, (n, m, k) in enumerate(cases):
        weights = tuple([-1.0, 1.0, -1.0][:m])
        Ind = make_types(D, "d", weights)
        vals = rng.integers(0, 4, size=(n, m)).astype(np.float64)  # many mutual non-dominance
        wv = vals * np.array(weights)
        crowd = rng.choice([0.0, 0.25, 0.5, np.inf], size=n)      # many crowding ties
        pop = to_inds(Ind, rng.uniform(0, 1, size=(n, 2)), wv)
        for ind, c in zip(pop, crowd):
            ind.fitness.crowding_dist = float(c)
        ident = {id(p): i for i, p in enumerate(pop)}
        p1, p2 = rng.permutation(n), rng.permutation(n)
        k4 = (k + 3) // 4 * 4
        coin = rng.integers(0, 2, size=k4).astype(np.uint8)
        floats = []
        for i in range(0, k, 4):
            for slot, (a, b) in enumerate([(p1[i], p1[i + 1]), (p1[i + 2], p1[i + 3]),
                                           (p2[i], p2[i + 1]), (p2[i + 2], p2[i + 3])]):
                fa, fb = pop[a].fitness, pop[b].fitness
                if not fa.dominates(fb) and not fb.dominates(fa) and \
                        fa.crowding_dist == fb.crowding_dist:
                    floats.append(0.25 if coin[i + slot] else 0.75)
        with Replay(floats=floats, samples=[list(p1), list(p2)]):
            chosen = tools.selTournamentDCD(pop, k)
        key = "dcd%d_" % j
        out.update({key + "wv": wv, key + "crowd": crowd, key + "k": np.array(k),
                    key + "perm1": p1.astype(np.int32), key + "perm2": p2.astype(np.int32),
                    key + "coin": coin,
                    key + "chosen": np.array([ident[id(c)] for c in chosen], np.int32)})
    return out


def gen_sbx(D, rng):
    """The NSGA-II variation loop (examples/ga/nsga2.py:96-105) with
    cxSimulatedBinaryBounded (crossover.py:291-360) and mutPolynomialBounded
    (mutation.py:51-95): position-indexed random() decisions cx_u / sbx_u /
    mut_u are fed to DEAP in its consumption order."""
    tools = D["deap.tools"]
    base = D["deap.base"]
    out = {}
    cases = [  # n, dim, k, cxpb, eta_cx, eta_mut, indpb, vector bounds
        (40, 30, 40, 0.9, 20.0, 20.0, 1.0 / 30, False),
        (33, 12, 31, 0.9, 20.0, 20.0, 0.25, True),
        (24, 7, 24, 0.6, 0.5, 2.0, 0.5, False),
        (50, 5, 18, 1.0, 100.0, 100.0, 1.0, True),
    ]
    for j, (n, dim, k, cxpb, eta_c, eta_m, indpb, vec) in enumerate(cases):
        if vec:
            low = [float(v) for v in rng.uniform(-3, 0, size=dim)]
            up = [float(v) for v in rng.uniform(0.5, 3, size=dim)]
        else:
            low, up = 0.0, 1.0
        lo = np.broadcast_to(np.asarray(low, np.float64), (dim,))
        hi = np.broadcast_to(np.asarray(up, np.float64), (dim,))
        genes = lo + (hi - lo) * rng.uniform(0, 1, size=(n, dim))
        # duplicated genes (|x1 - x2| <= 1e-14 branch) and genes on the bounds
        genes[1::5, :] = genes[0::5, :][: len(genes[1::5])]
        edge = rng.uniform(size=(n, dim))
        genes = np.where(edge < 0.05, lo, np.where(edge > 0.95, hi, genes))
        idx = rng.integers(0, n, size=k).astype(np.int32)
        if j == 0:
            idx = np.arange(k, dtype=np.int32)
        pairs = k // 2
        cx_u = rng.uniform(0, 1, size=pairs)
        sbx_u = rng.uniform(0, 1, size=(pairs, dim, 3))
        mut_u = rng.uniform(0, 1, size=(2 * pairs, dim, 2))
        Ind = make_types(D, "d", (-1.0, -1.0))
        pop = to_inds(Ind, genes, np.zeros((n, 2)))
        tb = base.Toolbox()
        tb.register("mate", tools.cxSimulatedBinaryBounded, low=low, up=up, eta=eta_c)
        tb.register("mutate", tools.mutPolynomialBounded, low=low, up=up, eta=eta_m, indpb=indpb)
        floats = []
        for p in range(pairs):
            a, b = genes[idx[2 * p]], genes[idx[2 * p + 1]]
            floats.append(float(cx_u[p]))
            if cx_u[p] <= cxpb:
                for i in range(dim):
                    floats.append(float(sbx_u[p, i, 0]))
                    if sbx_u[p, i, 0] <= 0.5 and abs(a[i] - b[i]) > 1e-14:
                        floats += [float(sbx_u[p, i, 1]), float(sbx_u[p, i, 2])]
            for c in (2 * p, 2 * p + 1):
                for i in range(dim):
                    floats.append(float(mut_u[c, i, 0]))
                    if mut_u[c, i, 0] <= indpb:
                        floats.append(float(mut_u[c, i, 1]))
        with Replay(floats=floats):
            offspring = [tb.clone(pop[i]) for i in idx]
            for ind1, ind2 in zip(offspring[::2], offspring[1::2]):
                if random.random() <= cxpb:
                    tb.mate(ind1, ind2)
                tb.mutate(ind1)
                tb.mutate(ind2)
                del ind1.fitness.values, ind2.fitness.values
        key = "sbx%d_" % j
        out.update({key + "genes": genes, key + "idx": idx, key + "low": lo.copy(),
                    key + "up": hi.copy(), key + "vec": np.array(int(vec)),
                    key + "meta": np.array([cxpb, eta_c, eta_m, indpb]),
                    key + "cx_u": cx_u, key + "sbx_u": sbx_u, key + "mut_u": mut_u,
                    key + "out": np.array([list(o) for o in offspring], np.float64),
                    key + "valid": np.array([o.fitness.valid for o in offspring])})
    return out


def gen_nsga2log(D, rng):
    """sortLogNondominated (emo.py:234-441) and selNSGA2(nd='log') (emo.py:15-50)
    on tie-heavy integer fitnesses (deterministic: no random draws)."""
    tools = D["deap.tools"]
    out = {}
    cases = [(40, 2, 30), (120, 3, 60), (200, 3, 199), (64, 2, 64), (90, 4, 45), (50, 3, 500)]
    for j, (n, m, k) in enumerate(cases):
        weights = tuple([-1.0, 1.0, -1.0, 1.0][:m])
        Ind = make_types(D, "d", weights)
        vals = rng.integers(0, 6 if m < 4 else 4, size=(n, m)).astype(np.float64)
        wv = vals * np.array(weights)
        pop = to_inds(Ind, rng.uniform(0, 1, size=(n, 2)), wv)
        ident = {id(p): i for i, p in enumerate(pop)}
        fronts = tools.emo.sortLogNondominated(pop, k)
        chosen = tools.selNSGA2(pop, k, nd="log")
        key = "log%d_" % j
        out.update({key + "wv": wv, key + "k": np.array(k),
                    key + "order": np.array([ident[id(x)] for f in fronts for x in f], np.int32),
                    key + "sizes": np.array([len(f) for f in fronts], np.int32),
                    key + "chosen": np.array([ident[id(c)] for c in chosen], np.int32)})
    return out


def gen_migration(D, rng):
    tools = D["deap.tools"]
    out = {}
    for j, (ndemes, n, dim, k, repl) in enumerate([(3, 40, 6, 5, None), (4, 30, 5, 6, "sample"),
                                                   (2, 25, 4, 8, None)]):
        Ind = make_types(D, "d", (1.0,))
        # few distinct genomes -> duplicates inside and across demes
        palette = rng.integers(0, 3, size=(6, dim)).astype(np.float64)
        demes, raw = [], []
        for d in range(ndemes):
            g = palette[rng.integers(0, len(palette), n)]
            wv = g.sum(axis=1, keepdims=True)
            raw.append((g.copy(), wv.copy()))
            demes.append(to_inds(Ind, g, wv))
        sel_idx = []
        samples = []
        for d in range(ndemes):
            best = tools.selBest(demes[d], k)
            sel_idx.append([next(i for i, p in enumerate(demes[d]) if p is b) for b in best])
            if repl == "sample":
                samples.append([int(x) for x in rng.choice(n, k, replace=False)])
        with Replay(samples=samples):
            tools.migRing(demes, k, tools.selBest,
                          replacement=(random.sample if repl == "sample" else None))
        key = "mig%d_" % j
        for d in range(ndemes):
            out[key + "in_genes%d" % d] = raw[d][0]
            out[key + "in_wv%d" % d] = raw[d][1]
            out[key + "sel%d" % d] = np.array(sel_idx[d])
            out[key + "out_genes%d" % d] = np.array([list(p) for p in demes[d]])
            out[key + "out_wv%d" % d] = np.array([p.fitness.wvalues for p in demes[d]])
            if repl == "sample":
                out[key + "repl%d" % d] = np.array(samples[d])
        out[key + "meta"] = np.array([str(ndemes), str(k), str(repl)])
    return out


def gen_c1_trajectory(D):
    """examples/ga/onemax_short.py (seed 64, pop 300, 100 bits, eaSimple
    cxpb 0.5 mutpb 0.2, 40 gens) with every decision recorded."""
    creator = D["deap.creator"]
    base = D["deap.base"]
    tools = D["deap.tools"]
    algorithms = D["deap.algorithms"]
    Ind = make_types(D, "b", (1.0,))
    tb = base.Toolbox()
    tb.register("attr_bool", random.randint, 0, 1)
    tb.register("individual", tools.initRepeat, Ind, tb.attr_bool, 100)
    tb.register("population", tools.initRepeat, list, tb.individual)
    tb.register("evaluate", lambda ind: (sum(ind),))
    tb.register("mate", tools.cxTwoPoint)
    tb.register("mutate", tools.mutFlipBit, indpb=0.05)
    tb.register("select", tools.selTournament, tournsize=3)
    random.seed(64)
    pop = tb.population(n=300)
    init = np.array([list(p) for p in pop], np.uint8)
    log_calls = []
    real = {name: getattr(random, name) for name in ("random", "randint", "choice")}

    def rec_random():
        v = real["random"]()
        log_calls.append(("random", v))
        return v

    def rec_randint(a, b):
        v = real["randint"](a, b)
        log_calls.append(("randint", v))
        return v

    def rec_choice(seq):
        i = random._inst._randbelow(len(seq))  # CPython 3.10 choice()
        log_calls.append(("choice", i))
        return seq[i]

    random.random, random.randint, random.choice = rec_random, rec_randint, rec_choice
    try:
        pop, log = algorithms.eaSimple(pop, tb, cxpb=0.5, mutpb=0.2, ngen=40, verbose=False)
    finally:
        for name, fn in real.items():
            setattr(random, name, fn)
    # split the recorded stream into per-generation decision arrays
    n, dim, t, ngen = 300, 100, 3, 40
    it = iter(log_calls)
    out = {"c1_init": init, "c1_final": np.array([list(p) for p in pop], np.uint8),
           "c1_final_wv": np.array([p.fitness.wvalues for p in pop]),
           "c1_nevals": np.array(log.select("nevals"))}
    asp_all, cxf_all, raw_all, mutf_all, mask_all = [], [], [], [], []
    for g in range(ngen):
        asp = np.array([next(it)[1] for _ in range(n * t)]).reshape(n, t)
        cxf = np.zeros(n // 2, bool)
        raw = np.zeros((n // 2, 2), np.int64)
        for p in range(n // 2):
            kind, v = next(it)
            assert kind == "random"
            cxf[p] = v < 0.5
            if cxf[p]:
                raw[p] = (next(it)[1], next(it)[1])
        mutf = np.zeros(n, bool)
        mask = np.zeros((n, dim), bool)
        for i in range(n):
            kind, v = next(it)
            mutf[i] = v < 0.2
            if mutf[i]:
                mask[i] = [next(it)[1] < 0.05 for _ in range(dim)]
        asp_all.append(asp)
        cxf_all.append(cxf)
        raw_all.append(raw)
        mutf_all.append(mutf)
        mask_all.append(mask)
    assert next(it, None) is None
    out.update({"c1_asp": np.array(asp_all), "c1_cx_flag": np.array(cxf_all),
                "c1_cx_raw": np.array(raw_all), "c1_mut_flag": np.array(mutf_all),
                "c1_mask": np.packbits(np.array(mask_all), axis=-1)})
    return out


def gen_selrandom(D, rng):
    """selRandom (selection.py:12-24) with replayed random.choice draws, and one
    eaSimple generation with toolbox.select = selRandom (the fused
    DM_SEL_RANDOM path of dm_generation)."""
    tools = D["deap.tools"]
    algorithms = D["deap.algorithms"]
    base = D["deap.base"]
    bm = D["deap.benchmarks"]
    out = {}
    for j, (n, k) in enumerate([(50, 50), (17, 40), (1000, 7)]):
        Ind = make_types(D, "d", (1.0,))
        pop = to_inds(Ind, rng.uniform(0, 1, size=(n, 3)), rng.uniform(0, 1, size=(n, 1)))
        idx = rng.integers(0, n, size=k)
        with Replay(choices=[int(a) for a in idx]):
            chosen = tools.selRandom(pop, k)
        out["sr%d_n" % j] = np.array(n)
        out["sr%d_choice" % j] = idx
        out["sr%d_out" % j] = np.array([next(i for i, p in enumerate(pop) if p is c)
                                        for c in chosen])
    cases = [("f64", "d", 200, 24, "blend", "gaussian", "rastrigin", (-1.0,)),
             ("bits", "b", 300, 31, "twopoint", "flipbit", "onemax", (1.0,))]
    for j, (gt, tc, dim, n, cx, mut, objective, weights) in enumerate(cases):
        Ind = make_types(D, tc, weights)
        genes = (rng.integers(0, 2, size=(n, dim)).astype(np.uint8) if gt == "bits"
                 else rng.uniform(-5.12, 5.12, size=(n, dim)))
        evalf = (lambda ind: (sum(ind),)) if objective == "onemax" else getattr(bm, objective)
        pop = to_inds(Ind, genes)
        for ind in pop:
            ind.fitness.values = evalf(ind)
        genes0, wv0, valid0 = from_inds(pop, genes.dtype, 1)
        cxpb, mutpb, indpb, alpha = 0.5, 0.2, 0.05, 0.5
        asp = rng.integers(0, n, size=(n, 1))
        npairs = n // 2
        cx_flag = rng.random(npairs) < cxpb
        cx_raw = np.stack([rng.integers(1, dim + 1, npairs), rng.integers(1, dim, npairs)], 1)
        blend_u = rng.random((npairs, dim))
        mut_flag = rng.random(n) < mutpb
        mask = rng.random((n, dim)) < indpb
        gauss = rng.normal(0.0, 1.0, size=(n, dim))
        floats, ints, gausses = [], [], []
        for p in range(npairs):
            floats.append(flag(cx_flag[p]))
            if cx_flag[p]:
                if cx == "twopoint":
                    ints.extend(int(v) for v in cx_raw[p])
                else:
                    floats.extend(float(v) for v in blend_u[p])
        for i in range(n):
            floats.append(flag(mut_flag[i]))
            if mut_flag[i]:
                for g in range(dim):
                    floats.append(flag(mask[i, g]))
                    if mut == "gaussian" and mask[i, g]:
                        gausses.append(float(gauss[i, g]))
        tb = base.Toolbox()
        tb.register("evaluate", evalf)
        tb.register("select", tools.selRandom)
        if cx == "twopoint":
            tb.register("mate", tools.cxTwoPoint)
        else:
            tb.register("mate", tools.cxBlend, alpha=alpha)
        if mut == "flipbit":
            tb.register("mutate", tools.mutFlipBit, indpb=indpb)
        else:
            tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=indpb)
        with Replay(floats=floats, ints=ints, gausses=gausses,
                    choices=[int(a) for a in asp.ravel()]):
            pop2, log = algorithms.eaSimple(pop, tb, cxpb, mutpb, 1, verbose=False)
        og, owv, ovalid = from_inds(pop2, genes.dtype, 1)
        key = "srea%d_" % j
        out.update({key + "genes": genes0, key + "wv": wv0, key + "valid": valid0,
                    key + "asp": asp, key + "cx_flag": cx_flag, key + "cx_raw": cx_raw,
                    key + "blend_u": blend_u, key + "mut_flag": mut_flag, key + "mask": mask,
                    key + "gauss": gauss, key + "out_genes": og, key + "out_wv": owv,
                    key + "nevals": np.array(log.select("nevals")),
                    key + "meta": np.array([gt, tc, cx, mut, objective, str(weights[0])])})
    return out


PORT_CASES = [("rastrigin", "d", 1000, 256), ("onemax", "b", 4096, 128),
              ("rosenbrock", "d", 300, 200)]


def _reference_ea(D, problem, tc, dim, n, ngen, seed, mapper=None):
    """The reference's own eaSimple run a user writes (README.md:72-103 /
    examples/ga/onemax_mp.py) with the real Mersenne Twister; returns
    (population, logbook, seconds of eaSimple)."""
    import time
    tools = D["deap.tools"]
    algorithms = D["deap.algorithms"]
    base = D["deap.base"]
    bm = D["deap.benchmarks"]
    weights = (1.0,) if problem == "onemax" else (-1.0,)
    Ind = make_types(D, tc, weights)
    random.seed(seed)
    if problem == "onemax":
        pop = [Ind(random.randint(0, 1) for _ in range(dim)) for _ in range(n)]
    else:
        lo, hi = (-5.12, 5.12) if problem == "rastrigin" else (-2.048, 2.048)
        pop = [Ind(random.uniform(lo, hi) for _ in range(dim)) for _ in range(n)]
    tb = base.Toolbox()
    if mapper is not None:
        tb.register("map", mapper)
    if problem == "onemax":
        tb.register("evaluate", _onemax_eval)
        tb.register("mate", tools.cxTwoPoint)
        tb.register("mutate", tools.mutFlipBit, indpb=0.05)
    else:
        tb.register("evaluate", getattr(bm, problem))
        tb.register("mate", tools.cxBlend, alpha=0.5)
        tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
    tb.register("select", tools.selTournament, tournsize=3)
    t0 = time.perf_counter()
    pop, log = algorithms.eaSimple(pop, tb, 0.5, 0.2, ngen, verbose=False)
    return pop, log, time.perf_counter() - t0


def _onemax_eval(ind):
    return (sum(ind),)  # README.md:85-86


def gen_port(D):
    """Calibration of oracle/deap_port.py (the CPU baseline bench.py times):
    the reference's seeded eaSimple outputs (bit-exact target) and, in
    port_calibration.json, the reference-vs-port wall time on the same
    configuration in this container (within +-20 %)."""
    import json
    import multiprocessing
    import time
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import deap_port
    out = {}
    for j, (problem, tc, dim, n) in enumerate(PORT_CASES):
        pop, log, _ = _reference_ea(D, problem, tc, dim, n, 2, 1)
        m = 1
        g, wv, ok = from_inds(pop, np.uint8 if tc == "b" else np.float64, m)
        key = "port%d_" % j
        out.update({key + "genes": g, key + "wv": wv, key + "nevals": np.array(log.select("nevals")),
                    key + "meta": np.array([problem, tc, str(dim), str(n)])})
    cal = {"note": "seconds of eaSimple(ngen=2) including its generation-0 evaluation, same "
                   "seed, this build container; median of 3 (reference = 2to3 copy of "
                   "/root/reference/deap, oracle/deap_port.evolve(time_gen0=True))",
           "cpu_count": os.cpu_count(), "cases": []}
    for problem, tc, dim, n, workers in [("rastrigin", "d", 1000, 2048, 1),
                                         ("onemax", "b", 4096, 2048, 1),
                                         ("rastrigin", "d", 1000, 4096, 8)]:
        ref_t, port_t = [], []
        for _ in range(3):
            if workers > 1:
                pool = multiprocessing.Pool(workers)
                try:
                    ref_t.append(_reference_ea(D, problem, tc, dim, n, 2, 1, pool.map)[2])
                finally:
                    pool.close()
                    pool.join()
            else:
                ref_t.append(_reference_ea(D, problem, tc, dim, n, 2, 1)[2])
            port_t.append(deap_port.evolve(problem, n, dim, 2, workers if workers > 1 else None,
                                           1, time_gen0=True)[1])
        r, p = sorted(ref_t)[1], sorted(port_t)[1]
        cal["cases"].append({"problem": problem, "genome": "array('%s')" % tc, "dim": dim,
                             "pop": n, "workers": workers, "reference_s": round(r, 4),
                             "port_s": round(p, 4), "port_over_reference": round(p / r, 4)})
        print(cal["cases"][-1])
    with open(os.path.join(HERE, "port_calibration.json"), "w") as f:
        json.dump(cal, f, indent=1)
    return out


def gen_support(D, rng):
    """HallOfFame.update (support.py:490-588) over a sequence of populations
    with duplicates and fitness ties, and the text of Logbook streams
    (support.py:261-487) fed by Statistics / MultiStatistics compiles."""
    import operator
    tools = D["deap.tools"]
    out = {}
    hof_cases = [(1, (1.0,), "eq"), (5, (1.0,), "eq"), (12, (1.0, -1.0), "eq"),
                 (40, (-1.0,), "eq"), (3, (1.0,), "array_equal"), (7, (1.0,), "first_gene")]
    for j, (maxsize, weights, sim) in enumerate(hof_cases):
        similar = {"eq": operator.eq, "array_equal": np.array_equal,
                   "first_gene": lambda a, b: a[0] == b[0]}[sim]
        Ind = make_types(D, "d", weights)
        hof = tools.HallOfFame(maxsize, similar=similar)
        key = "hof%d_" % j
        for gen in range(4):
            n = 300
            genes = rng.integers(0, 4, size=(n, 6)).astype(np.float64)
            genes[rng.integers(0, n, 30)] = genes[rng.integers(0, n, 30)]  # duplicates
            wv = np.stack([genes.sum(1) // 2 + gen * 0.5] +
                          ([-genes[:, 0]] if len(weights) > 1 else []), 1) * np.array(weights)
            pop = to_inds(Ind, genes, wv)
            hof.update(pop)
            out[key + "genes%d" % gen] = genes
            out[key + "wv%d" % gen] = wv
            out[key + "hof_genes%d" % gen] = np.array([list(h) for h in hof])
            out[key + "hof_wv%d" % gen] = np.array([h.fitness.wvalues for h in hof])
        out[key + "meta"] = np.array([str(maxsize), sim] + [str(w) for w in weights])
    # Logbook text: Statistics on fitness values, a header, one stream per gen
    Ind = make_types(D, "d", (-1.0,))
    stats = tools.Statistics(key=lambda ind: ind.fitness.values)
    stats.register("avg", np.mean)
    stats.register("std", np.std)
    stats.register("min", np.min)
    stats.register("max", np.max)
    log = tools.Logbook()
    log.header = ["gen", "nevals"] + stats.fields
    streams = []
    for gen in range(5):
        n = 64 + 7 * gen
        wv = -np.round(rng.uniform(0, 10 ** gen, size=(n, 1)), 3)
        pop = to_inds(Ind, np.zeros((n, 2)), wv)
        out["log_wv%d" % gen] = wv
        log.record(gen=gen, nevals=n - gen, **stats.compile(pop))
        streams.append(log.stream)
    out["log_streams"] = np.array(streams)
    out["log_str"] = np.array(str(log))
    # MultiStatistics -> chapters (examples/gp/symbreg.py:76-84 layout)
    stats_fit = tools.Statistics(lambda ind: ind.fitness.values)
    stats_size = tools.Statistics(len)
    mstats = tools.MultiStatistics(fitness=stats_fit, size=stats_size)
    mstats.register("avg", np.mean)
    mstats.register("max", np.max)
    log2 = tools.Logbook()
    log2.header = "gen", "evals", "fitness", "size"
    log2.chapters["fitness"].header = "min", "avg", "max"
    log2.chapters["size"].header = "avg", "max"
    mstats.register("min", np.min)
    streams = []
    for gen in range(4):
        n = 40 + gen
        wv = -np.round(rng.uniform(0, 5, size=(n, 1)), 2)
        pop = to_inds(Ind, np.zeros((n, 3 + gen)), wv)
        out["mlog_wv%d" % gen] = wv
        log2.record(gen=gen, evals=n, **mstats.compile(pop))
        streams.append(log2.stream)
    out["mlog_streams"] = np.array(streams)
    out["mlog_str"] = np.array(str(log2))
    return out


def sphere_fitness(n, m, seed):
    """DTLZ2-shaped objective vectors (directions on the positive unit sphere
    scaled by 1 + g): the shape of the C5 population's fitnesses."""
    rng = np.random.default_rng(seed)
    d = np.abs(rng.normal(size=(n, m)))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return d * (1.0 + rng.exponential(0.3, size=(n, 1)))


def gen_port_nsga2(D):
    """Calibration of the C5 CPU baseline (oracle/deap_port.py sel_nsga2 with
    nd='standard' / 'log'): reference selNSGA2 vs port wall time on the same
    DTLZ2-shaped minimisation fitnesses in this container (+-20 %), and the
    chosen individuals (identical)."""
    import json
    import time
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import deap_port
    tools = D["deap.tools"]
    weights = (-1.0, -1.0, -1.0)
    Ind = make_types(D, "d", weights)
    cal = {"note": "seconds of one selNSGA2(2N -> N) on DTLZ2-shaped fitnesses, this build "
                   "container, median of 3 (reference = 2to3 copy of /root/reference/deap; "
                   "port = oracle/deap_port.time_sel_nsga2)", "cpu_count": os.cpu_count(),
           "cases": []}
    for nd, n in (("standard", 1024), ("standard", 2048), ("log", 16384), ("log", 65536)):
        wv = -sphere_fitness(n, 3, 5)
        ref_t, port_t = [], []
        for _ in range(3):
            pop = to_inds(Ind, np.zeros((n, 1)), wv)
            t0 = time.perf_counter()
            chosen = tools.selNSGA2(pop, n // 2, nd=nd)
            ref_t.append(time.perf_counter() - t0)
            port_t.append(deap_port.time_sel_nsga2(wv, weights, n // 2, nd))
        ident = {id(ind): i for i, ind in enumerate(pop)}
        ref_idx = [ident[id(c)] for c in chosen]
        ppop = deap_port.nsga2_population(wv, weights)
        pident = {id(ind): i for i, ind in enumerate(ppop)}
        port_idx = [pident[id(c)] for c in deap_port.sel_nsga2(ppop, n // 2, nd)]
        r, p = sorted(ref_t)[1], sorted(port_t)[1]
        cal["cases"].append({"nd": nd, "n": n, "objectives": 3, "reference_s": round(r, 4),
                             "port_s": round(p, 4), "port_over_reference": round(p / r, 4),
                             "same_choice": ref_idx == port_idx})
        print(cal["cases"][-1])
    with open(os.path.join(HERE, "port_nsga2_calibration.json"), "w") as f:
        json.dump(cal, f, indent=1)


def main():
    D = load_reference()
    if sys.argv[1:] == ["log"]:
        np.savez_compressed(os.path.join(HERE, "nsga2log.npz"),
                            **gen_nsga2log(D, np.random.default_rng(13)))
        return
    if sys.argv[1:] == ["sbx"]:
        np.savez_compressed(os.path.join(HERE, "sbx.npz"),
                            **gen_sbx(D, np.random.default_rng(91)))
        return
    if sys.argv[1:] == ["round2"]:  # fixtures added in round 2 (existing ones untouched)
        np.savez_compressed(os.path.join(HERE, "selrandom.npz"),
                            **gen_selrandom(D, np.random.default_rng(5)))
        np.savez_compressed(os.path.join(HERE, "support.npz"),
                            **gen_support(D, np.random.default_rng(17)))
        np.savez_compressed(os.path.join(HERE, "port.npz"), **gen_port(D))
        return
    if sys.argv[1:] == ["port_nsga2"]:
        gen_port_nsga2(D)
        return
    if sys.argv[1:] == ["dcd"]:  # regenerate one fixture without touching the rest
        np.savez_compressed(os.path.join(HERE, "dcd.npz"),
                            **gen_dcd(D, np.random.default_rng(77)))
        return
    rng = np.random.default_rng(20260415)
    os.makedirs(HERE, exist_ok=True)
    np.savez_compressed(os.path.join(HERE, "eval.npz"), **gen_eval(D, rng))
    np.savez_compressed(os.path.join(HERE, "varand.npz"), **gen_varand(D, rng))
    np.savez_compressed(os.path.join(HERE, "selection.npz"), **gen_selection(D, rng))
    np.savez_compressed(os.path.join(HERE, "generation.npz"), **gen_ea_generation(D, rng))
    np.savez_compressed(os.path.join(HERE, "varor.npz"), **gen_varor(D, rng))
    np.savez_compressed(os.path.join(HERE, "nsga2.npz"), **gen_nsga2(D, rng))
    np.savez_compressed(os.path.join(HERE, "migration.npz"), **gen_migration(D, rng))
    np.savez_compressed(os.path.join(HERE, "c1_trajectory.npz"), **gen_c1_trajectory(D))
    np.savez_compressed(os.path.join(HERE, "dcd.npz"), **gen_dcd(D, np.random.default_rng(77)))
    np.savez_compressed(os.path.join(HERE, "sbx.npz"), **gen_sbx(D, np.random.default_rng(91)))
    np.savez_compressed(os.path.join(HERE, "nsga2log.npz"),
                        **gen_nsga2log(D, np.random.default_rng(13)))
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
