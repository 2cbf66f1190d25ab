"""DEAP-faithful pure-Python generation loop — TEST INFRASTRUCTURE / CPU
baseline only (see oracle/__init__.py).

Restates, with the reference's data types and call order, the CPU path a DEAP
user runs:

* individuals are ``array.array`` subclasses carrying a ``fitness`` object
  (``deap/creator.py:76-93``; ``array('b')`` as in examples/ga/onemax_mp.py:35,
  ``array('d')`` as in examples/ga/nsga2.py:32);
* ``toolbox.clone`` is ``copy.deepcopy`` (``deap/base.py:49``) — the dominant
  CPU cost of a generation;
* ``toolbox.map`` is ``multiprocessing.Pool.map`` (examples/ga/onemax_mp.py:58-59);
* operators draw from the stdlib ``random`` module in DEAP's order
  (``algorithms.py:33-82``, ``crossover.py:37-60,241-260``,
  ``mutation.py:17-48,124-142``, ``selection.py:12-69``).

``run(...)`` times ``ngen`` generations of ``eaSimple`` and returns
individual-generations per second.
"""
import array
import copy
import math
import multiprocessing
import operator
import random
import time


class Fitness:
    weights = (-1.0,)

    def __init__(self):
        self.wvalues = ()

    @property
    def valid(self):
        return len(self.wvalues) != 0

    @property
    def values(self):
        return tuple(map(operator.truediv, self.wvalues, self.weights))

    @values.setter
    def values(self, vals):
        self.wvalues = tuple(map(operator.mul, vals, self.weights))

    @values.deleter
    def values(self):
        self.wvalues = ()

    def __le__(self, other):
        return self.wvalues <= other.wvalues

    def __gt__(self, other):
        return not self.__le__(other)

    def __deepcopy__(self, memo):
        c = self.__class__()
        c.wvalues = self.wvalues
        return c


class FitnessMax(Fitness):
    weights = (1.0,)


class FitnessMin(Fitness):
    weights = (-1.0,)


class _Ind(array.array):
    typecode = "d"
    fitness_cls = FitnessMin

    def __new__(cls, seq=()):
        return super().__new__(cls, cls.typecode, seq)

    def __init__(self, seq=()):
        self.fitness = self.fitness_cls()

    def __deepcopy__(self, memo):
        c = self.__class__(self)
        memo[id(self)] = c
        c.__dict__.update(copy.deepcopy(self.__dict__, memo))
        return c

    def __reduce__(self):
        return (self.__class__, (list(self),), self.__dict__)


class IndDouble(_Ind):
    typecode = "d"
    fitness_cls = FitnessMin


class IndBits(_Ind):
    typecode = "b"
    fitness_cls = FitnessMax


# --- objectives (module level: picklable for Pool.map) ----------------------
def rastrigin(ind):
    return (10 * len(ind) + sum(g * g - 10 * math.cos(2 * math.pi * g) for g in ind),)


def rosenbrock(ind):
    return (sum(100 * (x * x - y) ** 2 + (1. - x) ** 2 for x, y in zip(ind[:-1], ind[1:])),)


def onemax(ind):
    return (sum(ind),)


# --- operators ----------------------------------------------------------------
def cx_two_point(a, b):
    size = min(len(a), len(b))
    c1 = random.randint(1, size)
    c2 = random.randint(1, size - 1)
    if c2 >= c1:
        c2 += 1
    else:
        c1, c2 = c2, c1
    a[c1:c2], b[c1:c2] = b[c1:c2], a[c1:c2]
    return a, b


def cx_blend(a, b, alpha):
    for i, (x1, x2) in enumerate(zip(a, b)):
        gamma = (1. + 2. * alpha) * random.random() - alpha
        a[i] = (1. - gamma) * x1 + gamma * x2
        b[i] = gamma * x1 + (1. - gamma) * x2
    return a, b


def mut_gaussian(ind, mu, sigma, indpb):
    for i in range(len(ind)):
        if random.random() < indpb:
            ind[i] += random.gauss(mu, sigma)
    return ind,


def mut_flip_bit(ind, indpb):
    for i in range(len(ind)):
        if random.random() < indpb:
            ind[i] = type(ind[i])(not ind[i])
    return ind,


def sel_tournament(inds, k, tournsize):
    chosen = []
    for _ in range(k):
        aspirants = [random.choice(inds) for _ in range(tournsize)]
        chosen.append(max(aspirants, key=operator.attrgetter("fitness")))
    return chosen


def var_and(population, clone, mate, mutate, cxpb, mutpb):
    offspring = [clone(ind) for ind in population]
    for i in range(1, len(offspring), 2):
        if random.random() < cxpb:
            offspring[i - 1], offspring[i] = mate(offspring[i - 1], offspring[i])
            del offspring[i - 1].fitness.values, offspring[i].fitness.values
    for i in range(len(offspring)):
        if random.random() < mutpb:
            offspring[i], = mutate(offspring[i])
            del offspring[i].fitness.values
    return offspring


def ea_simple_generations(pop, evaluate, mate, mutate, select, cxpb, mutpb, ngen, mapper):
    for _ in range(ngen):
        offspring = select(pop, len(pop))
        offspring = var_and(offspring, copy.deepcopy, mate, mutate, cxpb, mutpb)
        invalid = [ind for ind in offspring if not ind.fitness.valid]
        for ind, fit in zip(invalid, mapper(evaluate, invalid)):
            ind.fitness.values = fit
        pop[:] = offspring
    return pop


def evolve(problem="rastrigin", n=4096, dim=1000, ngen=2, workers=None, seed=1,
           time_gen0=False):
    """Seed the stdlib ``random``, build the population as the reference's
    ``toolbox.population`` would (initRepeat of ``random.uniform`` /
    ``random.randint`` per gene), evaluate it and run ``ngen`` eaSimple
    generations (cxpb 0.5, mutpb 0.2, tournsize 3; algorithms.py:149-181).
    Returns (population, seconds of the timed generations, workers); with
    ``time_gen0`` the timed region also covers the generation-0 evaluation,
    as timing a whole ``eaSimple`` call does (calibration against the
    reference)."""
    random.seed(seed)
    if problem == "onemax":
        pop = [IndBits(random.randint(0, 1) for _ in range(dim)) for _ in range(n)]
        evaluate = onemax
        mate = cx_two_point
        mutate = lambda ind: mut_flip_bit(ind, 0.05)  # noqa: E731
    else:
        lo, hi = (-5.12, 5.12) if problem == "rastrigin" else (-2.048, 2.048)
        pop = [IndDouble(random.uniform(lo, hi) for _ in range(dim)) for _ in range(n)]
        evaluate = rastrigin if problem == "rastrigin" else rosenbrock
        mate = lambda a, b: cx_blend(a, b, 0.5)  # noqa: E731
        mutate = lambda ind: mut_gaussian(ind, 0.0, 1.0, 0.05)  # noqa: E731
    select = lambda inds, k: sel_tournament(inds, k, 3)  # noqa: E731
    pool = None
    mapper = map
    if workers and workers > 1:
        pool = multiprocessing.Pool(workers)
        mapper = pool.map
    try:
        t0 = time.perf_counter()
        for ind, fit in zip(pop, mapper(evaluate, pop)):
            ind.fitness.values = fit
        if not time_gen0:
            t0 = time.perf_counter()
        ea_simple_generations(pop, evaluate, mate, mutate, select, 0.5, 0.2, ngen, mapper)
        dt = time.perf_counter() - t0
    finally:
        if pool is not None:
            pool.close()
            pool.join()
    return pop, dt, (workers or 1)


def run(problem="rastrigin", n=4096, dim=1000, ngen=2, workers=None, seed=1):
    """Time ``ngen`` eaSimple generations of the reference's CPU path.
    Returns (ind-gen/s, seconds, workers)."""
    _pop, dt, used = evolve(problem, n, dim, ngen, workers, seed)
    return n * ngen / dt, dt, used


# ---------------------------------------------------------------------------
# NSGA-II selection — the C5 CPU baseline (deap/tools/emo.py).  Same data
# types as the reference (Fitness objects hashed on wvalues, lists of
# individuals, dict-grouped unique fitnesses) and the same algorithms, so the
# timing is DEAP's; outputs are pinned by tests/golden/nsga2*.npz.
# ---------------------------------------------------------------------------
import bisect  # noqa: E402
from collections import defaultdict  # noqa: E402


class MOFitness(Fitness):
    """base.Fitness with several objectives: hashed / compared on wvalues
    (base.py:231,246), ``dominates`` as base.py:209-224."""
    weights = (-1.0, -1.0, -1.0)

    def __hash__(self):
        return hash(self.wvalues)

    def __eq__(self, other):
        return self.wvalues == other.wvalues

    def dominates(self, other, obj=slice(None)):
        better = False
        for mine, theirs in zip(self.wvalues[obj], other.wvalues[obj]):
            if mine > theirs:
                better = True
            elif mine < theirs:
                return False
        return better


class MOInd(list):
    """An individual of examples/ga/nsga2.py (a sequence with a fitness)."""

    def __init__(self, seq=(), weights=(-1.0, -1.0, -1.0)):
        super().__init__(seq)
        self.fitness = MOFitness()
        self.fitness.weights = weights


def sort_nondominated(individuals, k, first_front_only=False):
    """emo.py:53-117: all-pairs dominance over the unique fitnesses, then the
    peel of fronts until k individuals are sorted."""
    if k == 0:
        return []
    groups = defaultdict(list)
    for ind in individuals:
        groups[ind.fitness].append(ind)
    fits = list(groups.keys())
    n_above = defaultdict(int)
    below = defaultdict(list)
    front = []
    for i, a in enumerate(fits):
        for b in fits[i + 1:]:
            if a.dominates(b):
                n_above[b] += 1
                below[a].append(b)
            elif b.dominates(a):
                n_above[a] += 1
                below[b].append(a)
        if n_above[a] == 0:
            front.append(a)
    fronts = [[]]
    for f in front:
        fronts[-1].extend(groups[f])
    done = len(fronts[-1])
    if not first_front_only:
        target = min(len(individuals), k)
        while done < target:
            fronts.append([])
            released = []
            for p in front:
                for d in below[p]:
                    n_above[d] -= 1
                    if n_above[d] == 0:
                        released.append(d)
                        done += len(groups[d])
                        fronts[-1].extend(groups[d])
            front = released
    return fronts


def assign_crowding_dist(individuals):
    """emo.py:119-143."""
    if len(individuals) == 0:
        return
    dist = [0.0] * len(individuals)
    crowd = [(ind.fitness.values, i) for i, ind in enumerate(individuals)]
    nobj = len(individuals[0].fitness.values)
    for o in range(nobj):
        crowd.sort(key=lambda e: e[0][o])
        dist[crowd[0][1]] = float("inf")
        dist[crowd[-1][1]] = float("inf")
        if crowd[-1][0][o] == crowd[0][0][o]:
            continue
        norm = nobj * float(crowd[-1][0][o] - crowd[0][0][o])
        for lo, mid, hi in zip(crowd[:-2], crowd[1:-1], crowd[2:]):
            dist[mid[1]] += (hi[0][o] - lo[0][o]) / norm
    for i, d in enumerate(dist):
        individuals[i].fitness.crowding_dist = d


def sel_nsga2(individuals, k, nd="standard", return_fronts=False):
    """emo.py:15-50.  ``return_fronts``: also return the sorted fronts (test
    use: one sort serves both checks)."""
    if nd == "standard":
        fronts = sort_nondominated(individuals, k)
    elif nd == "log":
        fronts = sort_log_nondominated(individuals, k)
    else:
        raise Exception("selNSGA2: The choice of non-dominated sorting method %r is invalid." % nd)
    for f in fronts:
        assign_crowding_dist(f)
    chosen = [ind for f in fronts[:-1] for ind in f]
    rest = k - len(chosen)
    if rest > 0:
        last = sorted(fronts[-1], key=lambda ind: ind.fitness.crowding_dist, reverse=True)
        chosen.extend(last[:rest])
    return (chosen, fronts) if return_fronts else chosen


# Fortin et al. (2013), generalised reduced run-time non-dominated sort, as
# emo.py:201-455 implements it: fitnesses in descending lexicographic order,
# recursive median splits on the last objective, sweeps on the first two.
def _dominated_by(w1, w2):
    """emo.py:206-220: w2 dominates w1."""
    strict = False
    for a, b in zip(w1, w2):
        if a > b:
            return False
        if a < b:
            strict = True
    return strict


def _median(seq, obj):
    """emo.py:222-232 (mean of the two middle values for even lengths)."""
    vals = sorted(s[obj] for s in seq)
    n = len(vals)
    return vals[(n - 1) // 2] if n % 2 else (vals[(n - 1) // 2] + vals[n // 2]) / 2.0


def _halves(items, obj, med):
    """Two ways of splitting at the median (ties with the upper or the lower
    part), emo.py:299-325 / 375-412."""
    up_a, low_a, up_b, low_b = [], [], [], []
    for f in items:
        v = f[obj]
        if v > med:
            up_a.append(f)
            up_b.append(f)
        elif v < med:
            low_a.append(f)
            low_b.append(f)
        else:
            up_a.append(f)
            low_b.append(f)
    return up_a, low_a, up_b, low_b


def _stair_max(fstairs, idx, rank):
    return max(fstairs[:idx], key=rank.__getitem__)


def _nd_a(fits, obj, rank):
    """sortNDHelperA (emo.py:278-297)."""
    if len(fits) < 2:
        return
    if len(fits) == 2:
        if _dominated_by(fits[1][:obj + 1], fits[0][:obj + 1]):
            rank[fits[1]] = max(rank[fits[1]], rank[fits[0]] + 1)
    elif obj == 1:
        _sweep_a(fits, rank)
    elif len(frozenset(f[obj] for f in fits)) == 1:
        _nd_a(fits, obj - 1, rank)
    else:
        up_a, low_a, up_b, low_b = _halves(fits, obj, _median(fits, obj))
        if abs(len(up_a) - len(low_a)) <= abs(len(up_b) - len(low_b)):
            best, worst = up_a, low_a
        else:
            best, worst = up_b, low_b
        _nd_a(best, obj, rank)
        _nd_b(best, worst, obj - 1, rank)
        _nd_a(worst, obj, rank)


def _sweep_a(fits, rank):
    """sweepA (emo.py:327-344)."""
    stairs = [-fits[0][1]]
    fstairs = [fits[0]]
    for f in fits[1:]:
        idx = bisect.bisect_right(stairs, -f[1])
        if 0 < idx <= len(stairs):
            rank[f] = max(rank[f], rank[_stair_max(fstairs, idx, rank)] + 1)
        for i in range(idx, len(fstairs)):
            if rank[fstairs[i]] == rank[f]:
                del stairs[i]
                del fstairs[i]
                break
        stairs.insert(idx, -f[1])
        fstairs.insert(idx, f)


def _nd_b(best, worst, obj, rank):
    """sortNDHelperB (emo.py:346-373)."""
    if not best or not worst:
        return
    if len(best) == 1 or len(worst) == 1:
        for h in worst:
            hs = h[:obj + 1]
            for b in best:
                bs = b[:obj + 1]
                if _dominated_by(hs, bs) or hs == bs:
                    rank[h] = max(rank[h], rank[b] + 1)
    elif obj == 1:
        _sweep_b(best, worst, rank)
    elif min(b[obj] for b in best) >= max(h[obj] for h in worst):
        _nd_b(best, worst, obj - 1, rank)
    elif max(b[obj] for b in best) >= min(h[obj] for h in worst):
        med = _median(best if len(best) > len(worst) else worst, obj)
        b1a, b2a, b1b, b2b = _halves(best, obj, med)
        w1a, w2a, w1b, w2b = _halves(worst, obj, med)
        if (abs(len(b1a) - len(b2a) + len(w1a) - len(w2a))
                <= abs(len(b1b) - len(b2b) + len(w1b) - len(w2b))):
            b1, b2, w1, w2 = b1a, b2a, w1a, w2a
        else:
            b1, b2, w1, w2 = b1b, b2b, w1b, w2b
        _nd_b(b1, w1, obj, rank)
        _nd_b(b1, w2, obj - 1, rank)
        _nd_b(b2, w2, obj, rank)


def _sweep_b(best, worst, rank):
    """sweepB (emo.py:414-443)."""
    stairs, fstairs = [], []
    it = iter(best)
    nb = next(it, False)
    for h in worst:
        while nb and h[:2] <= nb[:2]:
            keep = True
            for i, fs in enumerate(fstairs):
                if rank[fs] == rank[nb]:
                    if fs[1] > nb[1]:
                        keep = False
                    else:
                        del stairs[i], fstairs[i]
                    break
            if keep:
                idx = bisect.bisect_right(stairs, -nb[1])
                stairs.insert(idx, -nb[1])
                fstairs.insert(idx, nb)
            nb = next(it, False)
        idx = bisect.bisect_right(stairs, -h[1])
        if 0 < idx <= len(stairs):
            rank[h] = max(rank[h], rank[_stair_max(fstairs, idx, rank)] + 1)


def sort_log_nondominated(individuals, k, first_front_only=False):
    """emo.py:234-276."""
    if k == 0:
        return []
    groups = defaultdict(list)
    for ind in individuals:
        groups[ind.fitness.wvalues].append(ind)
    fits = list(groups.keys())
    rank = dict.fromkeys(fits, 0)
    fits.sort(reverse=True)
    _nd_a(fits, len(individuals[0].fitness.wvalues) - 1, rank)
    fronts = [[] for _ in range(max(rank.values()) + 1)]
    for f in fits:
        fronts[rank[f]].extend(groups[f])
    if first_front_only:
        return fronts[0]
    total = 0
    for i, f in enumerate(fronts):
        total += len(f)
        if total >= k:
            return fronts[:i + 1]
    return fronts


def nsga2_population(wvalues, weights):
    """Individuals of examples/ga/nsga2.py carrying the given wvalues."""
    pop = []
    for row in wvalues:
        ind = MOInd([0.0], weights)
        ind.fitness.wvalues = tuple(float(x) for x in row)
        pop.append(ind)
    return pop


def time_sel_nsga2(wvalues, weights, k, nd="standard"):
    """Seconds of one sel_nsga2 call on host individuals."""
    pop = nsga2_population(wvalues, weights)
    t0 = time.perf_counter()
    sel_nsga2(pop, k, nd)
    return time.perf_counter() - t0
