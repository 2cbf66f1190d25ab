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
