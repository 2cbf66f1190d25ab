"""CPU oracle for the deap_amd hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker /
reported baseline: the product (``deap_amd``) never imports, calls or falls
back to it.

* :mod:`oracle.ops` restates each hot-path function of DEAP 1.3.1 in plain
  Python/numpy, consuming explicit random *decisions* (so the same decisions
  replayed into DEAP, into this oracle and into the GPU must give the same
  offspring).  Every function cites the reference file:line it follows.
* :mod:`oracle.philox` is the counter-based RNG of the device, in numpy
  (integer-exact), pinned by the Random123 known-answer vectors.
* :mod:`oracle.deap_port` is a DEAP-API-faithful pure-Python generation loop
  (``array('b')``/``array('d')`` genomes, ``toolbox.clone = deepcopy``,
  ``multiprocessing.Pool.map``) used as the CPU baseline of ``bench.py``.

Pinning: the oracle is checked against golden vectors produced by the
reference itself (``tests/golden/make_golden.py`` imports a 2to3 copy of
``/root/reference/deap`` in the build container and replays the same
decisions through it); the fixtures travel, the reference does not.
"""
