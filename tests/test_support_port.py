"""CPU checks pinned by fixtures the reference itself produced
(tests/golden/make_golden.py round2):

* oracle/deap_port.py — the CPU baseline bench.py times — reproduces the
  reference's seeded eaSimple runs bit for bit, and its speed was within
  +-20 % of the reference's on the same configurations;
* the Logbook text layout (deap/tools/support.py:261-487) character for
  character, Statistics / MultiStatistics chapters included;
* HallOfFame.update (support.py:490-588) on host individuals: duplicates,
  ties, maxsize 1-40, value and custom `similar`."""
import json
import operator
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden


def test_deap_port_reproduces_reference_ea_simple():
    from oracle import deap_port
    d = golden("port.npz")
    j = 0
    while "port%d_genes" % j in d:
        problem, tc, dim, n = d["port%d_meta" % j]
        pop, _, _ = deap_port.evolve(str(problem), int(n), int(dim), 2, None, 1)
        g = np.array([list(ind) for ind in pop], dtype=np.uint8 if tc == "b" else np.float64)
        wv = np.array([ind.fitness.wvalues for ind in pop])
        assert np.array_equal(g, d["port%d_genes" % j]), problem
        assert np.array_equal(wv, d["port%d_wv" % j]), problem
        j += 1
    assert j == 3


def test_deap_port_speed_calibrated_against_reference():
    with open(os.path.join(GOLDEN, "port_calibration.json")) as f:
        cal = json.load(f)
    assert len(cal["cases"]) >= 3
    for c in cal["cases"]:
        assert 0.8 <= c["port_over_reference"] <= 1.2, c


def _stats_pop(wv, dim=2):
    from deap_amd import base, creator
    creator.create("FitMinS", base.Fitness, weights=(-1.0,))
    creator.create("IndS", list, fitness=creator.FitMinS)
    out = []
    for w in wv:
        ind = creator.IndS([0.0] * dim)
        ind.fitness.values = (float(w[0]) / -1.0,)
        out.append(ind)
    return out


def test_logbook_stream_matches_reference_text():
    from deap_amd import tools
    d = golden("support.npz")
    stats = tools.Statistics(key=lambda ind: ind.fitness.values)
    stats.register("avg", np.mean)
    stats.register("std", np.std)
    stats.register("min", np.min)
    stats.register("max", np.max)
    log = tools.Logbook()
    log.header = ["gen", "nevals"] + stats.fields
    for gen in range(5):
        wv = d["log_wv%d" % gen]
        log.record(gen=gen, nevals=len(wv) - gen, **stats.compile(_stats_pop(wv)))
        assert log.stream == str(d["log_streams"][gen]), gen
    assert str(log) == str(d["log_str"])


def test_logbook_chapters_match_reference_text():
    from deap_amd import tools
    d = golden("support.npz")
    stats_fit = tools.Statistics(lambda ind: ind.fitness.values)
    stats_size = tools.Statistics(len)
    mstats = tools.MultiStatistics(fitness=stats_fit, size=stats_size)
    mstats.register("avg", np.mean)
    mstats.register("max", np.max)
    log = tools.Logbook()
    log.header = "gen", "evals", "fitness", "size"
    log.chapters["fitness"].header = "min", "avg", "max"
    log.chapters["size"].header = "avg", "max"
    mstats.register("min", np.min)
    for gen in range(4):
        wv = d["mlog_wv%d" % gen]
        log.record(gen=gen, evals=len(wv), **mstats.compile(_stats_pop(wv, 3 + gen)))
        assert log.stream == str(d["mlog_streams"][gen]), gen
    assert str(log) == str(d["mlog_str"])
    assert log.chapters["fitness"].select("gen") == [0, 1, 2, 3]
    del log[0]
    assert log.select("gen") == [1, 2, 3] and log.chapters["size"].select("gen") == [1, 2, 3]


HOF_SIMILAR = {"eq": operator.eq, "array_equal": np.array_equal,
               "first_gene": lambda a, b: a[0] == b[0]}


def hof_cases():
    d = golden("support.npz")
    j = 0
    while "hof%d_meta" % j in d:
        meta = d["hof%d_meta" % j]
        yield j, int(meta[0]), str(meta[1]), tuple(float(w) for w in meta[2:])
        j += 1


@pytest.mark.parametrize("case", list(hof_cases()), ids=lambda c: "hof%d" % c[0])
def test_hall_of_fame_host_matches_reference(case):
    from deap_amd import base, creator, tools
    j, maxsize, sim, weights = case
    d = golden("support.npz")
    creator.create("FitH", base.Fitness, weights=weights)
    creator.create("IndH", list, fitness=creator.FitH)
    hof = tools.HallOfFame(maxsize, similar=HOF_SIMILAR[sim])
    for gen in range(4):
        pop = []
        for g, w in zip(d["hof%d_genes%d" % (j, gen)], d["hof%d_wv%d" % (j, gen)]):
            ind = creator.IndH(g.tolist())
            ind.fitness.values = tuple(float(x) / ww for x, ww in zip(w, weights))
            pop.append(ind)
        hof.update(pop)
        assert [list(h) for h in hof] == d["hof%d_hof_genes%d" % (j, gen)].tolist()
        assert [list(h.fitness.wvalues) for h in hof] == d["hof%d_hof_wv%d" % (j, gen)].tolist()


def _port_fronts(wv, weights, k, nd):
    from oracle import deap_port
    pop = deap_port.nsga2_population(wv, weights)
    ident = {id(ind): i for i, ind in enumerate(pop)}
    fronts = (deap_port.sort_log_nondominated(pop, k) if nd == "log"
              else deap_port.sort_nondominated(pop, k))
    pop2 = deap_port.nsga2_population(wv, weights)
    ident2 = {id(ind): i for i, ind in enumerate(pop2)}
    chosen = [ident2[id(c)] for c in deap_port.sel_nsga2(pop2, k, nd)]
    return [[ident[id(x)] for x in f] for f in fronts], chosen


def test_deap_port_nsga2_reproduces_reference():
    """The C5 CPU baseline (oracle/deap_port.py sel_nsga2 with nd='standard'
    and 'log', emo.py:15-143,234-455 on reference-typed individuals) gives the
    reference's fronts and chosen individuals on the golden cases."""
    d = golden("nsga2.npz")
    for j in range(6):
        key = "nd%d_" % j
        wv, k = d[key + "wv"], int(d[key + "k"])
        fronts, chosen = _port_fronts(wv, tuple(d[key + "weights"]), k, "standard")
        assert [i for f in fronts for i in f] == d[key + "order"].tolist(), j
        assert chosen == d[key + "chosen"].tolist(), j
    d = golden("nsga2log.npz")
    for j in range(6):
        key = "log%d_" % j
        wv, k = d[key + "wv"], int(d[key + "k"])
        fronts, chosen = _port_fronts(wv, tuple([-1.0, 1.0, -1.0, 1.0][:wv.shape[1]]), k, "log")
        assert [len(f) for f in fronts] == d[key + "sizes"].tolist(), j
        assert [i for f in fronts for i in f] == d[key + "order"].tolist(), j
        assert chosen == d[key + "chosen"].tolist(), j


def test_deap_port_nsga2_speed_calibrated_against_reference():
    """Port vs reference selNSGA2 wall time, measured in the build container
    by tests/golden/make_golden.py port_nsga2: within +-20 %, same choice."""
    with open(os.path.join(GOLDEN, "port_nsga2_calibration.json")) as f:
        cal = json.load(f)
    assert {c["nd"] for c in cal["cases"]} == {"standard", "log"}
    for c in cal["cases"]:
        assert 0.8 <= c["port_over_reference"] <= 1.2, c
        assert c["same_choice"], c
