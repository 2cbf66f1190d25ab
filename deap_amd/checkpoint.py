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
from .device import zeros as _zeros

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
            pop.crowding_dist = _zeros((pop.capacity,), torch.float64, pop.device)
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


def _reference_tools():
    """DEAP's own ``deap.tools`` when it is importable (a user switching from
    the reference has it), else None."""
    try:
        from deap import tools as ref_tools  # noqa: F401  (the user's DEAP)
    except ImportError:
        return None
    return ref_tools


def _as_class(ind, individual_class):
    """A hall entry as ``individual_class`` (e.g. DEAP's creator.Individual):
    the same genes, the same weighted fitness when it is valid."""
    out = individual_class(ind)
    if ind.fitness.valid:
        out.fitness.wvalues = tuple(ind.fitness.wvalues)
    return out


def to_reference_types(halloffame, logbook, tools_module, individual_class=None):
    """Rebuild a hall of fame and a logbook as ``tools_module.HallOfFame`` /
    ``tools_module.Logbook`` objects (DEAP's classes when exporting for DEAP).
    With ``individual_class`` (a DEAP creator class) the hall's entries are
    rebuilt as that class too, so unpickling needs DEAP only; without it they
    stay the hall's own individuals (deap_amd host individuals when the hall
    was filled from a DevicePopulation without a creator class).  The hall
    keeps its order (insertion worst first re-creates equal-fitness order
    exactly, support.py:550-560); the logbook keeps header, records, chapters
    and the stream position."""
    hof = lb = None
    if halloffame is not None:
        hof = tools_module.HallOfFame(halloffame.maxsize, halloffame.similar)
        for ind in reversed(list(halloffame)):
            hof.insert(ind if individual_class is None else _as_class(ind, individual_class))
    if logbook is not None:
        lb = _copy_logbook(logbook, tools_module.Logbook)
    return hof, lb


def _copy_logbook(src, cls):
    lb = cls()
    lb.header = list(src.header) if src.header is not None else None
    lb.extend(dict(r) for r in src)
    lb.buffindex = src.buffindex
    for name, ch in src.chapters.items():
        lb.chapters[name] = _copy_logbook(ch, cls)
    return lb


def export_reference_dict(population, generation=None, halloffame=None, logbook=None,
                          stream=None, individual_class=None, tools_module=None):
    """The checkpoint dict of the reference's tutorial
    (doc/tutorials/advanced/checkpoint.rst:21-65):
    ``dict(population=..., generation=..., halloffame=..., logbook=...,
    rndstate=random.getstate())``.

    * ``population``: host individuals (``individual_class`` — e.g. DEAP's
      ``creator.Individual`` — or plain lists carrying a ``fitness``;
      ``fitness.wvalues`` set for valid rows);
    * ``halloffame`` / ``logbook``: DEAP's ``tools.HallOfFame`` /
      ``tools.Logbook`` holding the same entries when DEAP is importable (or
      ``tools_module``'s classes), otherwise the deap_amd objects (same API);
    * ``rndstate``: ``random.getstate()`` — what the tutorial passes to
      ``random.setstate`` (checkpoint.rst:32);
    * ``device_stream``: the counter-based device stream ``(seed, island,
      counter)`` that :func:`import_reference_dict` resumes bit-exactly (the
      device never draws from Python's ``random``)."""
    import random
    tm = tools_module if tools_module is not None else _reference_tools()
    if tm is not None:
        halloffame, logbook = to_reference_types(halloffame, logbook, tm, individual_class)
    return {"population": population.to_individuals(individual_class),
            "generation": generation, "halloffame": halloffame, "logbook": logbook,
            "rndstate": random.getstate(),
            "device_stream": tuple(stream.getstate()) if stream is not None else None}


def _stream_triple(v):
    return (isinstance(v, (tuple, list)) and len(v) == 3
            and all(isinstance(x, int) for x in v))


def import_reference_dict(cp, weights=None, gtype=None, device=None, capacity=None):
    """Rebuild a device population from a reference-shaped checkpoint dict
    (``population``: individuals with ``fitness.wvalues`` — valid iff non-empty
    — as DEAP pickles them, or as :func:`export_reference_dict` produced them).
    ``weights`` default to the first individual's ``fitness.weights``; genome
    type by ``gtype`` or inferred (DevicePopulation.from_individuals).
    Returns a dict with ``population`` (DevicePopulation), ``generation``,
    ``halloffame``, ``logbook`` and ``stream`` (a RandomStream from
    ``device_stream``; a checkpoint written by DEAP itself has none — the run
    then continues on a fresh stream).  ``rndstate`` is left to the caller's
    ``random.setstate`` exactly as in the tutorial."""
    from .device import DevicePopulation
    from .ops import RandomStream
    pop = DevicePopulation.from_individuals(list(cp["population"]), weights, gtype, device,
                                            capacity)
    stream = None
    ds = cp.get("device_stream")
    if ds is None and _stream_triple(cp.get("rndstate")):
        ds = cp["rndstate"]  # round-2 exports kept the stream under rndstate
    if _stream_triple(ds):
        stream = RandomStream()
        stream.setstate(tuple(ds))
    return {"population": pop, "generation": cp.get("generation"),
            "halloffame": cp.get("halloffame"), "logbook": cp.get("logbook"), "stream": stream}


__all__ = ["save", "load", "read_header", "header", "export_reference_dict",
           "import_reference_dict", "to_reference_types"]
