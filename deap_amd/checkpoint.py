"""Checkpoint / resume of a device-resident evolution.

The reference documents checkpointing as a user pattern: pickle a dict of
``population``, ``generation``, ``halloffame``, ``logbook`` and
``random.getstate()`` every few generations and reload it to continue
(doc/tutorials/advanced/checkpoint.rst:21-65; individuals pickle through
creator.py:70-71,91-92).  Here the same dict is written without pickle: one
``.npz`` (loadable with ``allow_pickle=False``) holding the population's raw
device rows (genomes exactly as laid out in HBM, ``wvalues``, ``valid``,
``crowding_dist``) and a JSON header with the layout, the counter-based
:class:`~deap_amd.ops.RandomStream` state ``(seed, island, counter)``, the
generation, the logbook records and the hall-of-fame entries.  Because every
kernel draws from Philox keyed by that state, a resumed run reproduces the
uninterrupted run bit for bit (tests/test_gpu_parity.py::
test_checkpoint_resume_is_bit_exact).
"""
import json

import numpy as np

FORMAT = "deap_amd.checkpoint/1"


def _pop_arrays(population):
    n = len(population)
    out = {"genes": population.genes[:n].cpu().numpy(),
           "wvalues": population.wvalues[:n].cpu().numpy(),
           "valid": population.valid[:n].cpu().numpy()}
    if getattr(population, "crowding_dist", None) is not None:
        out["crowding_dist"] = population.crowding_dist[:n].cpu().numpy()
    return out


def _pop_meta(population):
    return {"n": len(population), "dim": population.dim, "gtype": int(population.gtype),
            "weights": list(population.weights), "stride": population.stride}


def _jsonable(v):
    if isinstance(v, (np.floating, np.integer)):
        return v.item()
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, dict):
        return {k: _jsonable(x) for k, x in v.items()}
    return v


def _logbook_json(logbook):
    """A Logbook with its chapters (MultiStatistics records are split into
    chapters by ``Logbook.record``, support.py:342-349), recursively."""
    return {"header": _jsonable(logbook.header), "records": _jsonable(list(logbook)),
            "buffindex": logbook.buffindex,
            "chapters": {name: _logbook_json(ch) for name, ch in logbook.chapters.items()}}


def _logbook_from_json(h):
    from .tools.support import Logbook
    lb = Logbook()
    lb.header = h["header"]
    lb.extend(dict(r) for r in h["records"])
    lb.buffindex = h.get("buffindex", 0)
    for name, ch in h.get("chapters", {}).items():
        lb.chapters[name] = _logbook_from_json(ch)
    return lb


def header(population, stream=None, generation=None, halloffame=None, logbook=None,
           extra=None):
    """The JSON-serialisable part of a checkpoint."""
    h = {"format": FORMAT, "population": _pop_meta(population),
         "stream": list(stream.getstate()) if stream is not None else None,
         "generation": generation, "extra": _jsonable(extra)}
    if logbook is not None:
        h["logbook"] = _logbook_json(logbook)
    if halloffame is not None:
        h["halloffame"] = {"maxsize": halloffame.maxsize,
                           "items": [[_jsonable(list(ind)), list(ind.fitness.wvalues)]
                                     for ind in halloffame]}
    return h


def save(path, population, stream=None, generation=None, halloffame=None, logbook=None,
         extra=None):
    """Write ``population`` (+ RNG state, generation, hall of fame, logbook)."""
    arrays = _pop_arrays(population)
    h = header(population, stream, generation, halloffame, logbook, extra)
    arrays["header"] = np.frombuffer(json.dumps(h).encode(), dtype=np.uint8)
    with open(path, "wb") as f:
        np.savez(f, **arrays)


def read_header(path):
    with np.load(path, allow_pickle=False) as z:
        return json.loads(bytes(z["header"]).decode())


def load(path, device=None, individual_class=None, capacity=None):
    """Read a checkpoint written by :func:`save`.  Returns a dict with
    ``population`` (a DevicePopulation on ``device``), ``stream``
    (RandomStream), ``generation``, ``halloffame``, ``logbook``, ``extra``."""
    import torch
    from .device import DevicePopulation
    from .ops import RandomStream
    from .tools.support import HallOfFame, Logbook
    with np.load(path, allow_pickle=False) as z:
        h = json.loads(bytes(z["header"]).decode())
        if h.get("format") != FORMAT:
            raise ValueError("not a deap_amd checkpoint: %r" % h.get("format"))
        meta = h["population"]
        n = meta["n"]
        pop = DevicePopulation(n, meta["dim"], meta["gtype"], tuple(meta["weights"]), device,
                               capacity if capacity is not None else max(n, 1),
                               individual_class)
        if pop.stride != meta["stride"]:
            raise ValueError("row layout changed (stride %d, checkpoint %d)"
                             % (pop.stride, meta["stride"]))
        if n:
            pop.genes[:n].copy_(torch.from_numpy(z["genes"]))
            pop.wvalues[:n].copy_(torch.from_numpy(z["wvalues"]))
            pop.valid[:n].copy_(torch.from_numpy(z["valid"]))
        if "crowding_dist" in z.files:
            pop.crowding_dist = torch.zeros((pop.capacity,), dtype=torch.float64,
                                            device=pop.device)
            pop.crowding_dist[:n].copy_(torch.from_numpy(z["crowding_dist"]))
    out = {"population": pop, "generation": h.get("generation"), "extra": h.get("extra"),
           "stream": None, "halloffame": None, "logbook": None}
    if h.get("stream") is not None:
        st = RandomStream()
        st.setstate(tuple(h["stream"]))
        out["stream"] = st
    if h.get("logbook") is not None:
        out["logbook"] = _logbook_from_json(h["logbook"])
    if h.get("halloffame") is not None:
        hof = HallOfFame(h["halloffame"]["maxsize"])
        items = h["halloffame"]["items"]
        if items:
            genes = np.array([g for g, _ in items])
            wv = np.array([w for _, w in items], dtype=np.float64)
            tmp = DevicePopulation.from_numpy(genes, pop.weights, meta["gtype"], wv,
                                              np.ones(len(items)), pop.device,
                                              individual_class=individual_class)
            # worst first: equal-fitness entries then come back in their order
            # (insert places a newcomer before the equal keys, support.py:550-560)
            for ind in reversed(tmp.to_individuals()):
                hof.insert(ind)
        out["halloffame"] = hof
    return out


def export_reference_dict(population, generation=None, halloffame=None, logbook=None,
                          stream=None, individual_class=None):
    """The checkpoint dict of the reference's tutorial
    (doc/tutorials/advanced/checkpoint.rst:21-65):
    ``dict(population=..., generation=..., halloffame=..., logbook=...,
    rndstate=...)`` with the population materialised as host individuals
    (``individual_class`` — e.g. a DEAP ``creator.Individual`` — or plain
    lists carrying a ``fitness``; ``fitness.wvalues`` set for valid rows), the
    hall of fame and logbook as given, and ``rndstate`` = the counter-based
    stream state ``(seed, island, counter)`` (the device does not draw from
    Python's ``random``; the tuple resumes the same stream through
    :func:`import_reference_dict`).  A user who pickles it, as the tutorial
    does, gets a file that their DEAP code can read."""
    return {"population": population.to_individuals(individual_class),
            "generation": generation, "halloffame": halloffame, "logbook": logbook,
            "rndstate": tuple(stream.getstate()) if stream is not None else None}


def import_reference_dict(cp, weights=None, gtype=None, device=None, capacity=None):
    """Rebuild a device population from a reference-shaped checkpoint dict
    (``population``: individuals with ``fitness.wvalues`` — valid iff non-empty
    — as DEAP pickles them, or as :func:`export_reference_dict` produced them).
    ``weights`` default to the first individual's ``fitness.weights``; genome
    type by ``gtype`` or inferred (DevicePopulation.from_individuals).
    Returns a dict with ``population`` (DevicePopulation), ``generation``,
    ``halloffame``, ``logbook`` and ``stream`` (a RandomStream when ``rndstate``
    is a ``(seed, island, counter)`` tuple, else None)."""
    from .device import DevicePopulation
    from .ops import RandomStream
    pop = DevicePopulation.from_individuals(list(cp["population"]), weights, gtype, device,
                                            capacity)
    stream = None
    rs = cp.get("rndstate")
    if isinstance(rs, (tuple, list)) and len(rs) == 3 and all(isinstance(x, int) for x in rs):
        stream = RandomStream()
        stream.setstate(tuple(rs))
    return {"population": pop, "generation": cp.get("generation"),
            "halloffame": cp.get("halloffame"), "logbook": cp.get("logbook"), "stream": stream}


__all__ = ["save", "load", "read_header", "header", "export_reference_dict",
           "import_reference_dict"]
