"""Generational drivers on device-resident populations (``deap/algorithms.py``).

Signatures and return values follow the reference; the population argument is
a :class:`~deap_amd.device.DevicePopulation` and every variation / selection
operator must be a ``deap_amd`` device operator (a plain Python function
there raises ``TypeError``).  ``evaluate`` may be a device objective
(``deap_amd.benchmarks``, fused into the generation kernel) or any Python
callable on one individual, such as the reference README's ``evalOneMax``:
the :class:`HostEvaluator` bridge gathers the invalid rows, runs
``toolbox.map(toolbox.evaluate, invalid_ind)`` on host individuals and
writes the fitness back (``dm_set_fitness``), exactly the reference's
``algorithms.py:171-174``.  Each generation is one fused
kernel launch (select -> clone -> varAnd -> evaluate, ``dm_generation``) for
``eaSimple``; ``eaMuPlusLambda`` runs ``varOr`` (``dm_var_or``) then the
selection over ``population + offspring``.  Per-generation bookkeeping
(``nevals``, statistics) is accumulated on the device and read back once at
the end unless ``verbose`` asks for a line per generation.

Extra keyword-only arguments (not in DEAP) control the random decisions:
``stream`` (a :class:`~deap_amd.ops.RandomStream`, default the global one),
``mode`` ("native" | "inject" | "dump") and ``decisions`` (a list with one
:class:`~deap_amd.decisions.Decisions` per generation: read in inject mode,
appended to in dump mode).
"""
import ctypes
import functools

from . import _lib
from .decisions import Decisions
from .device import DevicePopulation
from .ops import default_stream, mode_code, resolve
from .tools.support import Logbook
from .device import zeros as _zeros


def _torch():
    import torch
    return torch


def _check_pop(population):
    if not isinstance(population, DevicePopulation):
        raise TypeError("deap_amd drivers operate on a DevicePopulation (got %r); build one with "
                        "deap_amd.tools.initPopulation or DevicePopulation.from_individuals"
                        % type(population))


def _variation(population, mate, mutate, cxpb, mutpb):
    var = _lib.Variation()
    var.cxpb = float(cxpb)
    var.mutpb = float(mutpb)
    var.sigma = 1.0
    if mate is not None:
        op, a, kw = mate
        op.fill(var, a, kw)
    if mutate is not None:
        op, a, kw = mutate
        op.fill(var, a, kw, population)
    return var


class HostEvaluator:
    """``toolbox.evaluate`` that is a plain Python callable (not a device
    objective): evaluates the invalid individuals of a device population on
    the host, as the reference's loop does (``deap/algorithms.py:149-152,
    171-174``)::

        invalid_ind = [ind for ind in offspring if not ind.fitness.valid]
        fitnesses = toolbox.map(toolbox.evaluate, invalid_ind)
        for ind, fit in zip(invalid_ind, fitnesses):
            ind.fitness.values = fit

    The invalid rows (read from the device ``valid`` array, in population
    order) are gathered on the device (``dm_gather``), copied once to the
    host and materialised as individuals of the population's creator class;
    ``values * weights`` (``Fitness.wvalues``, base.py:184-198) goes back in
    one copy and one scatter (``dm_set_fitness``).  Returns the number of
    evaluations (``nevals``)."""

    def __init__(self, toolbox):
        self.evaluate = toolbox.evaluate
        self.map = getattr(toolbox, "map", map)

    def __call__(self, population):
        import numpy as np
        torch = _torch()
        n = len(population)
        if n == 0:
            return 0
        ok = population.valid[:n].cpu().numpy()
        inv = np.flatnonzero(ok == 0).astype(np.int32)
        k = int(inv.size)
        if k == 0:
            return 0
        ctx = population.ctx.bind()
        idx = torch.from_numpy(inv).to(population.device)
        batch = population.like(k, capacity=k)
        _lib.call("dm_gather", ctx, ctypes.byref(population.c_pop()),
                  ctypes.c_void_p(idx.data_ptr()), ctypes.byref(batch.c_pop()))
        inds = batch.to_individuals()
        fits = list(self.map(self.evaluate, inds))
        if len(fits) != k:
            raise ValueError("evaluate returned %d fitnesses for %d individuals" % (len(fits), k))
        w = np.asarray(population.weights, dtype=np.float64)
        vals = np.empty((k, population.nobj), dtype=np.float64)
        for i, fit in enumerate(fits):
            if len(fit) != population.nobj:
                raise ValueError("evaluate returned %d values, the fitness has %d weights"
                                 % (len(fit), population.nobj))
            vals[i] = [float(x) for x in fit]
        wv = torch.from_numpy(vals * w).to(population.device)  # Fitness.values setter
        _lib.call("dm_set_fitness", ctx, ctypes.byref(population.c_pop()),
                  ctypes.c_void_p(idx.data_ptr()), k, ctypes.c_void_p(wv.data_ptr()))
        return k


def _evaluator(toolbox):
    """(device objective spec, None) or (None, HostEvaluator) for
    ``toolbox.evaluate``."""
    from .ops import DeviceOperator
    f = toolbox.evaluate
    while isinstance(f, functools.partial):
        f = f.func
    if isinstance(f, DeviceOperator):
        return resolve(toolbox.evaluate), None
    if callable(f):
        return None, HostEvaluator(toolbox)
    raise TypeError("toolbox.evaluate is not callable: %r" % (toolbox.evaluate,))


def _eval(population, evaluate):
    if evaluate is None:
        e = _lib.Eval()
        e.fn = _lib.DM_EVAL_NONE
        return e
    op, a, kw = evaluate
    return op.eval_struct(population.weights, a, kw)


def _mode_and_decisions(mode, decisions, gen_index, k, population, tournsize, var, varor=False):
    """Decide the RNG mode of one launch and its decisions buffer."""
    if mode is None:
        mode = "native"
    code = mode_code(mode)
    if code == _lib.DM_RNG_NATIVE:
        return code, None
    if code == _lib.DM_RNG_INJECT:
        d = decisions[gen_index] if isinstance(decisions, (list, tuple)) else decisions
        if d is None:
            raise ValueError("inject mode needs decisions")
        return code, d
    d = Decisions.allocate(k, population.dim, population.device, tournsize=tournsize,
                           cx=var.cx != _lib.DM_CX_NONE, blend=var.cx == _lib.DM_CX_BLEND,
                           mut=var.mut != _lib.DM_MUT_NONE,
                           gauss=var.mut == _lib.DM_MUT_GAUSSIAN, varor=varor)
    if isinstance(decisions, list):
        decisions.append(d)
    return code, d


def _apply_variation(population, mate_op, mate_args, mate_kw, mut_op, mut_args, mut_kw, cxpb,
                     mutpb, decisions=None, mode=None, stream=None):
    """Direct call of a crossover / mutation operator on a population."""
    _check_pop(population)
    mate = (mate_op, mate_args, mate_kw) if mate_op is not None else None
    mutate = (mut_op, mut_args, mut_kw) if mut_op is not None else None
    return _var_and(population, mate, mutate, cxpb, mutpb, decisions, mode, stream)


def _var_and(population, mate, mutate, cxpb, mutpb, decisions, mode, stream):
    stream = stream or default_stream()
    var = _variation(population, mate, mutate, cxpb, mutpb)
    offspring = population.like()
    code, d = _mode_and_decisions(mode, decisions, 0, len(population), population, 0, var)
    ev = _eval(population, None)
    ctx = population.ctx.bind()
    dec = d.c_struct() if d is not None else None
    _lib.call("dm_generation", ctx, ctypes.byref(population.c_pop()),
              ctypes.byref(offspring.c_pop()), _lib.DM_SEL_IDENTITY, 0, None, ctypes.byref(var),
              ctypes.byref(ev), stream.next(), code,
              ctypes.byref(dec) if dec is not None else None, None)
    return offspring


def varAnd(population, toolbox, cxpb, mutpb, *, decisions=None, mode=None, stream=None):
    """Crossover AND mutation on a cloned population (``deap/algorithms.py:33-82``).

    Pairs ``(2i-1... )``: for i = 1, 3, 5, ... ``random() < cxpb`` mates
    offspring[i-1] and offspring[i]; then every offspring is mutated when
    ``random() < mutpb``.  Modified individuals have their fitness invalidated.
    Returns a new population; the input is untouched."""
    _check_pop(population)
    mate = resolve(toolbox.mate)
    mutate = resolve(toolbox.mutate)
    return _var_and(population, mate, mutate, cxpb, mutpb, decisions, mode, stream)


def varBounded(population, toolbox, cxpb, index=None, *, decisions=None, mode=None,
               stream=None):
    """The variation body of DEAP's NSGA-II loop (``examples/ga/nsga2.py:96-105``;
    also ``tests/test_algorithms.py:96-104``), one fused launch
    (``dm_vary_bounded``)::

        offspring = [toolbox.clone(ind) for ind in population[index]]
        for ind1, ind2 in zip(offspring[::2], offspring[1::2]):
            if random.random() <= cxpb:
                toolbox.mate(ind1, ind2)
            toolbox.mutate(ind1); toolbox.mutate(ind2)
            del ind1.fitness.values, ind2.fitness.values

    ``toolbox.mate`` must be ``cxSimulatedBinaryBounded`` and ``toolbox.mutate``
    ``mutPolynomialBounded`` (same low/up).  ``index``: device int tensor of
    selected rows (e.g. from ``selTournamentDCD``), default all rows.  Returns
    the offspring population (fitness invalid except an odd last clone)."""
    from .tools._bounded import vary_bounded
    from .tools.crossover import cxSimulatedBinaryBounded
    from .tools.mutation import mutPolynomialBounded
    _check_pop(population)
    mop, ma, mkw = resolve(toolbox.mate)
    uop, ua, ukw = resolve(toolbox.mutate)
    if mop is not cxSimulatedBinaryBounded or uop is not mutPolynomialBounded:
        raise TypeError("varBounded needs mate=cxSimulatedBinaryBounded and "
                        "mutate=mutPolynomialBounded, got %r / %r" % (mop, uop))
    return vary_bounded(population, index, mop.params(ma, mkw), uop.params(ua, ukw), cxpb,
                        decisions, mode, stream)


def _selection_spec(toolbox):
    op, a, kw = resolve(toolbox.select)
    return op, a, kw


class _Bookkeeping:
    """nevals + statistics recorded per generation, on device when possible."""

    def __init__(self, population, ngen, stats, halloffame, verbose):
        torch = _torch()
        self.nevals = _zeros((ngen + 1,), torch.int64, population.device)
        self.stats = stats
        self.hof = halloffame
        self.verbose = verbose
        self.records = []
        self.host_nevals = {}  # generations evaluated by a HostEvaluator
        self.logbook = Logbook()
        self.logbook.header = ["gen", "nevals"] + (stats.fields if stats else [])

    pending_hof = None

    def complete_hof(self):
        if self.pending_hof is not None:
            done, self.pending_hof = self.pending_hof, None
            done()

    def nevals_ptr(self, gen):
        return ctypes.c_void_p(self.nevals.data_ptr() + 8 * gen)

    def record(self, gen, population, defer_hof=False):
        """``defer_hof``: queue the HallOfFame's device work now and run its
        host part at ``complete_hof()`` (after the next generation is queued)."""
        if self.hof is not None:
            begin = getattr(self.hof, "update_begin", None)
            if defer_hof and begin is not None:
                self.pending_hof = begin(population)
            else:
                self.hof.update(population)
        rec = self.stats.compile(population) if self.stats else {}
        self.records.append((gen, rec))
        if self.verbose:
            self._flush_one(gen, rec)

    def _flush_one(self, gen, rec):
        nev = self.host_nevals[gen] if gen in self.host_nevals else int(self.nevals[gen].item())
        self.logbook.record(gen=gen, nevals=nev, **_materialise(rec))
        print(self.logbook.stream)

    def finish(self):
        if not self.verbose:
            nev = self.nevals.cpu().tolist()
            for gen, v in self.host_nevals.items():
                nev[gen] = v
            for gen, rec in self.records:
                self.logbook.record(gen=gen, nevals=nev[gen], **_materialise(rec))
        return self.logbook


def _materialise(rec):
    out = {}
    for k, v in rec.items():
        out[k] = v() if callable(v) else v
    return out


class GenerationStep:
    """One eaSimple generation body bound to a toolbox: ``step(parents,
    children)`` launches the fused select -> clone -> varAnd -> evaluate
    kernel (``dm_generation``) on the current stream.  eaSimple is a loop of
    these; ``bench.py`` times them."""

    def __init__(self, population, toolbox, cxpb, mutpb, evaluate=True):
        from .tools.selection import selRandom, selTournament
        self._selTournament, self._selRandom = selTournament, selRandom
        self.mate = resolve(toolbox.mate)
        self.mutate = resolve(toolbox.mutate)
        # a host `evaluate` (HostEvaluator): the kernel varies only, the
        # driver evaluates the invalid children afterwards
        self.evaluate, self.host_eval = _evaluator(toolbox) if evaluate else (None, None)
        self.sel = _selection_spec(toolbox)
        self.var = _variation(population, self.mate, self.mutate, cxpb, mutpb)
        self.ev = _eval(population, self.evaluate)

    def step(self, parents, children, stream, nevals_ptr=None, mode=None, decisions=None,
             gen_index=0):
        sel_op, sel_args, sel_kw = self.sel
        n = len(parents)
        sel_kind, tournsize, sel_index = _fused_selection(sel_op, sel_args, sel_kw, parents,
                                                          self._selTournament, self._selRandom,
                                                          stream)
        code, d = _mode_and_decisions(mode, decisions, gen_index, n, parents,
                                      tournsize if sel_kind in (_lib.DM_SEL_TOURNAMENT,
                                                                _lib.DM_SEL_RANDOM) else 0,
                                      self.var)
        dec = d.c_struct() if d is not None else None
        children.resize(n)
        _lib.call("dm_generation", parents.ctx.bind(), ctypes.byref(parents.c_pop()),
                  ctypes.byref(children.c_pop()), sel_kind, tournsize,
                  ctypes.c_void_p(sel_index.data_ptr()) if sel_index is not None else None,
                  ctypes.byref(self.var), ctypes.byref(self.ev), stream.next(), code,
                  ctypes.byref(dec) if dec is not None else None, nevals_ptr)


def eaSimple(population, toolbox, cxpb, mutpb, ngen, stats=None, halloffame=None,
             verbose=__debug__, *, decisions=None, mode=None, stream=None):
    """The simple generational GA (``deap/algorithms.py:85-189``).

    gen 0 evaluates invalid individuals; each later generation is
    ``select(population, len(population))`` -> ``varAnd`` -> evaluate invalid
    -> ``population[:] = offspring``, fused into one kernel when the selection
    is ``selTournament``/``selRandom``.  Returns ``(population, logbook)``."""
    _check_pop(population)
    stream = stream or default_stream()
    step = GenerationStep(population, toolbox, cxpb, mutpb)
    book = _Bookkeeping(population, ngen, stats, halloffame, verbose)
    ctx = population.ctx.bind()
    host = step.host_eval

    # generation 0: evaluate the invalid individuals                      :149-160
    if host is None:
        _lib.call("dm_evaluate", ctx, ctypes.byref(population.c_pop()), ctypes.byref(step.ev), 1,
                  book.nevals_ptr(0))
    else:
        book.host_nevals[0] = host(population)
    book.record(0, population)

    offspring = population.like(len(population), capacity=population.capacity)
    # the HallOfFame's host loop for generation g runs while generation g + 1
    # is on the GPU (g's rows are rewritten only by generation g + 2)
    defer = not verbose and host is None
    for gen in range(1, ngen + 1):
        step.step(population, offspring, stream, book.nevals_ptr(gen), mode, decisions, gen - 1)
        if host is not None:
            book.host_nevals[gen] = host(offspring)                        # :171-174
        book.complete_hof()
        population.swap_storage(offspring)                                 # :181
        book.record(gen, population, defer_hof=defer)
    book.complete_hof()
    return population, book.finish()


def _fused_selection(sel_op, sel_args, sel_kw, population, selTournament, selRandom, stream):
    n = len(population)
    if sel_op is selTournament:
        k, tournsize = _tournament_args(sel_args, sel_kw, n)
        if k == n and sel_kw.get("fit_attr", "fitness") == "fitness":
            return _lib.DM_SEL_TOURNAMENT, tournsize, None
    if sel_op is selRandom and not sel_args and "k" not in sel_kw:
        return _lib.DM_SEL_RANDOM, 1, None
    idx = sel_op(population, n, *sel_args, stream=stream, **sel_kw)
    return _lib.DM_SEL_INDEX, 0, idx


def _tournament_args(args, kw, n):
    # select(population, len(population)) with tournsize bound in the toolbox
    if "tournsize" in kw:
        return n, int(kw["tournsize"])
    if args:
        return n, int(args[0])
    raise TypeError("selTournament() missing required argument: 'tournsize'")


def varOr(population, toolbox, lambda_, cxpb, mutpb, *, decisions=None, mode=None, stream=None,
          evaluate=False, out=None):
    """Crossover OR mutation OR reproduction (``deap/algorithms.py:192-245``).
    Returns a population of ``lambda_`` offspring."""
    _check_pop(population)
    assert (cxpb + mutpb) <= 1.0, (
        "The sum of the crossover and mutation probabilities must be smaller or equal to 1.0.")
    stream = stream or default_stream()
    mate = resolve(toolbox.mate)
    mutate = resolve(toolbox.mutate)
    var = _variation(population, mate, mutate, cxpb, mutpb)
    spec, host = _evaluator(toolbox) if evaluate else (None, None)
    ev = _eval(population, spec)
    offspring = out if out is not None else population.like(lambda_, capacity=lambda_)
    code, d = _mode_and_decisions(mode, decisions, 0, lambda_, population, 0, var, varor=True)
    dec = d.c_struct() if d is not None else None
    ctx = population.ctx.bind()
    _lib.call("dm_var_or", ctx, ctypes.byref(population.c_pop()),
              ctypes.byref(offspring.c_pop(0, lambda_)), ctypes.byref(var), ctypes.byref(ev),
              stream.next(), code, ctypes.byref(dec) if dec is not None else None, None)
    if host is not None:
        host(offspring)
    return offspring


class MuPlusLambdaStep:
    """One (mu + lambda) generation body (``deap/algorithms.py:316-329``) bound
    to a toolbox: varOr of ``lambda_`` offspring appended after the parents
    (with evaluation of the invalid ones fused in), HallOfFame update on the
    offspring, ``select(population + offspring, mu)`` and the gather of the
    chosen rows.  ``eaMuPlusLambda`` is a loop of these; ``bench.py`` times
    them (config C5: selNSGA2 on DTLZ2)."""

    def __init__(self, population, toolbox, mu, lambda_, cxpb, mutpb, comma=False):
        if comma:
            assert lambda_ >= mu, "lambda must be greater or equal to mu."
        self.comma = comma
        assert (cxpb + mutpb) <= 1.0, (
            "The sum of the crossover and mutation probabilities must be smaller or equal to 1.0.")
        self.mu, self.lambda_ = mu, lambda_
        self.sel = _selection_spec(toolbox)
        self.var = _variation(population, resolve(toolbox.mate), resolve(toolbox.mutate), cxpb,
                              mutpb)
        spec, self.host_eval = _evaluator(toolbox)
        self.ev = _eval(population, spec)
        self.last_nevals = None  # set by a host evaluation
        n0 = len(population)
        cap = max(n0, mu) + lambda_
        self.combined = population.like(n0 + lambda_, capacity=cap)
        self.nxt = population.like(mu, capacity=cap)
        self.n = n0
        # combined rows [0, n) = population
        _lib.call("dm_gather", population.ctx.bind(), ctypes.byref(population.c_pop()), None,
                  ctypes.byref(self.combined.c_pop(0, n0)))

    def step(self, stream, nevals_ptr=None, mode=None, decisions=None, gen_index=0,
             halloffame=None):
        comb, n, lam = self.combined, self.n, self.lambda_
        ctx = comb.ctx.bind()
        code, d = _mode_and_decisions(mode, decisions, gen_index, lam, comb, 0, self.var,
                                      varor=True)
        dec = d.c_struct() if d is not None else None
        _lib.call("dm_var_or", ctx, ctypes.byref(comb.c_pop(0, n)),
                  ctypes.byref(comb.c_pop(n, lam)), ctypes.byref(self.var), ctypes.byref(self.ev),
                  stream.next(), code, ctypes.byref(dec) if dec is not None else None, nevals_ptr)
        comb.resize(n + lam)
        if self.host_eval is not None:
            self.last_nevals = self.host_eval(_View(comb, n, lam))       # :319-322
        if halloffame is not None:
            halloffame.update(_View(comb, n, lam))
        sel_op, sel_args, sel_kw = self.sel
        # (mu + lambda): select(population + offspring, mu); (mu, lambda):
        # select(offspring, mu) (algorithms.py:428-429)
        pool = _View(comb, n, lam) if self.comma else comb
        idx = sel_op(pool, self.mu, *sel_args, stream=stream, **sel_kw)
        self.nxt.resize(self.mu)
        _lib.call("dm_gather", ctx, ctypes.byref(pool.c_pop()), ctypes.c_void_p(idx.data_ptr()),
                  ctypes.byref(self.nxt.c_pop(0, self.mu)))
        if getattr(pool, "crowding_dist", None) is not None:
            # fitness.crowding_dist travels with the clones (base.py:252-261
            # copies the fitness object): one library gather, buffers of the
            # same capacity swap with the storage below
            if self.nxt.crowding_dist is None or \
                    len(self.nxt.crowding_dist) < len(pool.crowding_dist):
                self.nxt.crowding_dist = pool.crowding_dist.new_empty(len(pool.crowding_dist))
            _lib.call("dm_gather_f64", ctx, ctypes.c_void_p(pool.crowding_dist.data_ptr()),
                      ctypes.c_void_p(idx.data_ptr()), len(idx),
                      ctypes.c_void_p(self.nxt.crowding_dist.data_ptr()))
        comb.swap_storage(self.nxt)
        self.n = self.mu
        comb.resize(self.mu)
        return comb


def eaMuPlusLambda(population, toolbox, mu, lambda_, cxpb, mutpb, ngen, stats=None,
                   halloffame=None, verbose=__debug__, *, decisions=None, mode=None,
                   stream=None):
    """(mu + lambda) evolution (``deap/algorithms.py:248-337``): varOr ->
    evaluate invalid -> ``population[:] = select(population + offspring, mu)``.
    The concatenation keeps parents first, then offspring, as in the reference
    (the order matters to NSGA-II's front order)."""
    _check_pop(population)
    return _mu_lambda(population, toolbox, mu, lambda_, cxpb, mutpb, ngen, stats, halloffame,
                      verbose, decisions, mode, stream, comma=False)


def _mu_lambda(population, toolbox, mu, lambda_, cxpb, mutpb, ngen, stats, halloffame, verbose,
               decisions, mode, stream, comma):
    stream = stream or default_stream()
    assert (cxpb + mutpb) <= 1.0, (
        "The sum of the crossover and mutation probabilities must be smaller or equal to 1.0.")
    spec, host = _evaluator(toolbox)
    ev = _eval(population, spec)
    book = _Bookkeeping(population, ngen, stats, halloffame, verbose)
    ctx = population.ctx.bind()

    if host is None:
        _lib.call("dm_evaluate", ctx, ctypes.byref(population.c_pop()), ctypes.byref(ev), 1,
                  book.nevals_ptr(0))
    else:
        book.host_nevals[0] = host(population)
    book.record(0, population)

    step = MuPlusLambdaStep(population, toolbox, mu, lambda_, cxpb, mutpb, comma=comma)
    for gen in range(1, ngen + 1):
        combined = step.step(stream, book.nevals_ptr(gen), mode, decisions, gen - 1, halloffame)
        if step.host_eval is not None:
            book.host_nevals[gen] = step.last_nevals
        rec = stats.compile(combined) if stats else {}
        book.records.append((gen, rec))
        if verbose:
            book._flush_one(gen, rec)
    combined = step.combined
    # hand the final population back in place
    final = population.like(mu, capacity=max(mu, 1))
    _lib.call("dm_gather", ctx, ctypes.byref(combined.c_pop(0, mu)), None,
              ctypes.byref(final.c_pop()))
    final.crowding_dist = combined.crowding_dist
    population.swap_storage(final)
    return population, book.finish()


def eaMuCommaLambda(population, toolbox, mu, lambda_, cxpb, mutpb, ngen, stats=None,
                    halloffame=None, verbose=__debug__, *, decisions=None, mode=None,
                    stream=None):
    """(mu, lambda) evolution (``deap/algorithms.py:340-437``): varOr ->
    evaluate invalid -> HallOfFame.update(offspring) ->
    ``population[:] = select(offspring, mu)``."""
    _check_pop(population)
    assert lambda_ >= mu, "lambda must be greater or equal to mu."
    return _mu_lambda(population, toolbox, mu, lambda_, cxpb, mutpb, ngen, stats, halloffame,
                      verbose, decisions, mode, stream, comma=True)


class _View(DevicePopulation):
    """Row range of a population, sharing its buffers (no copy)."""

    def __init__(self, base, start, count):  # pylint: disable=super-init-not-called
        self.__dict__.update(base.__dict__)
        self.genes = base.genes[start:start + count]
        self.wvalues = base.wvalues[start:start + count]
        self.valid = base.valid[start:start + count]
        self.n = count
        self.capacity = count


__all__ = ["varAnd", "eaSimple", "varOr", "eaMuPlusLambda", "eaMuCommaLambda", "varBounded"]  # + GenerationStep, MuPlusLambdaStep
