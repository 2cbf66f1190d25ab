"""Host-side API mirror (Toolbox / Fitness / creator / Logbook / Statistics /
HallOfFame on host lists) and operator resolution, on CPU."""
import array
import functools
import operator
import random

import numpy as np
import pytest

from deap_amd import base, creator


def test_toolbox_register_partial_and_decorate():
    tb = base.Toolbox()
    assert tb.clone([1, [2]]) == [1, [2]]
    tb.register("f", lambda a, b, c=3: (a, b, c), 2, c=4)
    assert tb.f(3) == (2, 3, 4)
    assert tb.f.__name__ == "f"
    tb.decorate("f", lambda fn: (lambda *a, **k: ("deco",) + fn(*a, **k)))
    assert tb.f(3) == ("deco", 2, 3, 4)
    tb.unregister("f")
    assert not hasattr(tb, "f")


def test_fitness_semantics():
    creator.create("FMaxMin", base.Fitness, weights=(1.0, -1.0))
    f1, f2 = creator.FMaxMin(), creator.FMaxMin()
    assert not f1.valid
    f1.values = (2.0, 3.0)
    assert f1.wvalues == (2.0, -3.0) and f1.values == (2.0, 3.0)
    f2.values = (2.0, 4.0)
    assert f1 > f2 and f1.dominates(f2) and not f2.dominates(f1)
    f2.values = (2.0, 3.0)
    assert f1 == f2 and not f1.dominates(f2) and not (f1 > f2)
    del f1.values
    assert not f1.valid
    with pytest.raises(TypeError):
        base.Fitness()
    with pytest.raises(AssertionError):
        f2.values = (1.0,)


def test_creator_array_individual():
    creator.create("FMax1", base.Fitness, weights=(1.0,))
    creator.create("IndB", array.array, typecode="b", fitness=creator.FMax1)
    ind = creator.IndB([1, 0, 1])
    ind.fitness.values = (2,)
    import copy
    c = copy.deepcopy(ind)
    assert list(c) == [1, 0, 1] and c.fitness.values == (2.0,) and c.fitness is not ind.fitness
    from deap_amd.device import gtype_of
    from deap_amd import _lib
    assert gtype_of(creator.IndB) == _lib.DM_BITS
    creator.create("IndF", array.array, typecode="f", fitness=creator.FMax1)
    assert gtype_of(creator.IndF) == _lib.DM_F32
    creator.create("IndL", list, fitness=creator.FMax1)
    assert gtype_of(creator.IndL) == _lib.DM_F64


def test_operator_resolution():
    from deap_amd import tools, benchmarks
    from deap_amd.ops import resolve
    tb = base.Toolbox()
    tb.register("mate", tools.cxBlend, alpha=0.5)
    tb.register("evaluate", benchmarks.dtlz2, obj=3)
    op, a, kw = resolve(tb.mate)
    assert op is tools.cxBlend and kw == {"alpha": 0.5}
    op, a, kw = resolve(tb.evaluate)
    ev = op.eval_struct((-1.0, -1.0, -1.0), a, kw)
    assert ev.obj == 3 and ev.weights[2] == -1.0
    tb.register("bad", lambda x: x)
    with pytest.raises(TypeError):
        resolve(tb.bad)


def test_drivers_reject_host_lists():
    from deap_amd import algorithms, tools
    tb = base.Toolbox()
    with pytest.raises(TypeError):
        algorithms.eaSimple([[0, 1]], tb, 0.5, 0.2, 1)
    with pytest.raises(TypeError):
        tools.selTournament([[0, 1]], 1, 3)


def test_logbook_and_statistics_on_host_lists():
    from deap_amd import tools
    creator.create("FMaxS", base.Fitness, weights=(1.0,))
    pop = []
    for v in (1.0, 3.0, 2.0):
        f = creator.FMaxS()
        f.values = (v,)
        pop.append(type("I", (), {"fitness": f})())
    stats = tools.Statistics(lambda ind: ind.fitness.values)
    stats.register("avg", np.mean)
    stats.register("max", np.max)
    rec = stats.compile(pop)
    assert rec == {"avg": 2.0, "max": 3.0}
    log = tools.Logbook()
    log.header = ["gen", "nevals", "avg", "max"]
    log.record(gen=0, nevals=3, **rec)
    log.record(gen=1, nevals=2, **rec)
    assert log.select("gen") == [0, 1]
    assert log.select("gen", "nevals") == ([0, 1], [3, 2])
    text = log.stream
    assert "gen" in text.splitlines()[0] and len(text.splitlines()) == 3
    assert log.stream == ""


def test_hall_of_fame_on_host_lists():
    from deap_amd import tools
    creator.create("FMaxH", base.Fitness, weights=(1.0,))
    creator.create("IndH", list, fitness=creator.FMaxH)
    pop = []
    for genes, v in (([1], 1.0), ([2], 5.0), ([2], 5.0), ([3], 4.0), ([4], 5.0)):
        ind = creator.IndH(genes)
        ind.fitness.values = (v,)
        pop.append(ind)
    hof = tools.HallOfFame(2)
    hof.update(pop)
    # value pinned against the reference HallOfFame (bisect_right insertion)
    assert [list(i) for i in hof] == [[4], [2]]


def test_checkpoint_reference_types_keep_order_and_chapters():
    """export_reference_dict hands DEAP a tools.HallOfFame / tools.Logbook
    (checkpoint.rst:21-65): to_reference_types rebuilds them through the
    given module's classes — here deap_amd.tools, which mirrors DEAP's API —
    with equal-fitness entries in the same order, the same similar() and the
    logbook's records, header, chapters and stream position."""
    import operator
    from deap_amd import checkpoint, tools
    creator.create("FMaxC", base.Fitness, weights=(1.0,))
    creator.create("IndC", list, fitness=creator.FMaxC)
    pop = []
    for genes, v in (([1], 1.0), ([2], 5.0), ([3], 5.0), ([4], 4.0), ([5], 5.0)):
        ind = creator.IndC(genes)
        ind.fitness.values = (v,)
        pop.append(ind)
    hof = tools.HallOfFame(4)
    hof.update(pop)
    log = tools.Logbook()
    log.header = ["gen", "fit"]
    log.record(gen=0, fit={"max": 1.0})
    log.record(gen=1, fit={"max": 2.0})
    _ = log.stream
    h2, l2 = checkpoint.to_reference_types(hof, log, tools)
    assert type(h2) is tools.HallOfFame and type(l2) is tools.Logbook
    assert [list(i) for i in h2] == [list(i) for i in hof]
    assert h2.maxsize == 4 and h2.similar is operator.eq
    assert list(l2) == list(log) and l2.header == log.header and l2.buffindex == log.buffindex
    assert l2.chapters["fit"].select("max") == [1.0, 2.0]
    h3, l3 = checkpoint.to_reference_types(None, None, tools)
    assert h3 is None and l3 is None
    # entries of another class (deap_amd host individuals of a DevicePopulation
    # without a creator class) come back as the given individual_class
    creator.create("IndC2", list, fitness=creator.FMaxC)
    h4, _ = checkpoint.to_reference_types(hof, None, tools, creator.IndC2)
    assert all(type(i) is creator.IndC2 for i in h4)
    assert [list(i) for i in h4] == [list(i) for i in hof]
    assert [i.fitness.values for i in h4] == [i.fitness.values for i in hof]
