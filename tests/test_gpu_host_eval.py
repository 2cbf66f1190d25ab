"""The host-evaluate bridge: ``toolbox.evaluate`` may be
any Python callable on one individual -- the reference README's own

    def evalOneMax(individual):
        return sum(individual),

(README.md:85-86).  The drivers gather the invalid rows, run
``toolbox.map(toolbox.evaluate, invalid_ind)`` on host individuals and write
the fitness back with ``dm_set_fitness`` (deap/algorithms.py:149-152,
171-174)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def evalOneMax(individual):
    return sum(individual),


def _toolbox(evaluate, select="tournament"):
    from deap_amd import base, tools
    tb = base.Toolbox()
    tb.register("evaluate", evaluate)
    tb.register("mate", tools.cxTwoPoint)
    tb.register("mutate", tools.mutFlipBit, indpb=0.05)
    tb.register("select", tools.selTournament, tournsize=3)
    return tb


def test_readme_loop_with_its_own_evaluate_reproduces_the_reference(gpu):
    """README OneMax (examples/ga/onemax_short.py, seed 64) with the README's
    evalOneMax registered as is: the reference's 40 generations of decisions
    replayed give its final population, fitness and nevals per generation."""
    from deap_amd import algorithms
    from deap_amd.decisions import Decisions
    from deap_amd.device import DevicePopulation
    d = golden("c1_trajectory.npz")
    pop = DevicePopulation.from_numpy(d["c1_init"], weights=(1.0,), gtype="bits")
    decs = [Decisions.from_numpy(gpu, aspirants=d["c1_asp"][g], cx_flag=d["c1_cx_flag"][g],
                                 cx_raw=d["c1_cx_raw"][g], mut_flag=d["c1_mut_flag"][g],
                                 mut_mask=np.unpackbits(d["c1_mask"][g], axis=-1)[:, :100])
            for g in range(40)]
    calls = []

    def counting_map(fn, inds):
        inds = list(inds)
        calls.append(len(inds))
        return map(fn, inds)

    tb = _toolbox(evalOneMax)
    tb.register("map", counting_map)
    pop, log = algorithms.eaSimple(pop, tb, 0.5, 0.2, 40, verbose=False, decisions=decs,
                                   mode="inject")
    g, wv, ok = pop.to_numpy()
    assert np.array_equal(g, d["c1_final"])
    assert np.array_equal(wv, d["c1_final_wv"]) and ok.all()
    assert log.select("nevals") == d["c1_nevals"].tolist()
    assert calls == d["c1_nevals"].tolist()  # one toolbox.map per generation, invalid only


def test_host_and_device_evaluate_give_the_same_run(gpu):
    """Native (counter-based) decisions: the host evalOneMax and the device
    onemax objective give bit-identical eaSimple runs (genomes, fitness,
    nevals, statistics), and the same for eaMuPlusLambda."""
    from deap_amd import algorithms, benchmarks, tools
    from deap_amd.ops import RandomStream

    def run(evaluate, driver):
        stream = RandomStream(31)
        pop = tools.initPopulation(n=2000, dim=256, gtype="bits", weights=(1.0,), stream=stream)
        stats = tools.Statistics(key=lambda ind: ind.fitness.values)
        stats.register("max", np.max)
        stats.register("avg", np.mean)
        tb = _toolbox(evaluate)
        if driver == "simple":
            pop, log = algorithms.eaSimple(pop, tb, 0.5, 0.2, 6, stats=stats, verbose=False,
                                           stream=stream)
        else:
            pop, log = algorithms.eaMuPlusLambda(pop, tb, 2000, 1000, 0.5, 0.3, 4, stats=stats,
                                                 verbose=False, stream=stream)
        return pop.to_numpy(), log
    for driver in ("simple", "mupluslambda"):
        (g1, w1, o1), l1 = run(benchmarks.onemax, driver)
        (g2, w2, o2), l2 = run(evalOneMax, driver)
        assert np.array_equal(g1, g2) and np.array_equal(w1, w2) and np.array_equal(o1, o2)
        assert l1.select("nevals") == l2.select("nevals")
        assert l1.select("max") == l2.select("max") and l1.select("avg") == l2.select("avg")


def test_host_evaluate_errors_follow_the_reference(gpu):
    """A fitness of the wrong length raises (base.py:181-185 assigns
    ``values * weights`` element-wise; DEAP fails on the mismatch)."""
    from deap_amd import algorithms, tools
    from deap_amd.ops import RandomStream
    pop = tools.initPopulation(n=64, dim=32, gtype="bits", weights=(1.0,),
                               stream=RandomStream(1))
    tb = _toolbox(lambda ind: (1.0, 2.0))
    with pytest.raises(ValueError):
        algorithms.eaSimple(pop, tb, 0.5, 0.2, 1, verbose=False)
