"""Islands across processes with the real device kernels (the
device pack / placement under a multi-rank ``migRingDistributed`` had only
run with host stand-ins).

Two processes share the one GPU of the test box (RCCL refuses two ranks on
one device, so the process group is ``gloo`` and the emigrant blocks are
host-staged by ``route_blocks``; every pack, selection and placement is the
device kernel of ``libdeapmi.so``).  Each rank runs ``eaSimpleDemes`` on its
share of 4 OneMax demes with migRing every 5 generations
(``examples/ga/onemax_multidemic.py:79-93``, ``deap/tools/migration.py:4-51``).
Philox streams are keyed by the deme id, so the split over ranks cannot
change a single bit: the result must equal the one-process run, which
``test_gpu_islands.py`` replays in the oracle.  Splits include a rank that
holds no deme (it must still join every migration)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_DEMES, N, DIM, NGEN, K = 4, 96, 100, 12, 5


def _toolbox():
    from deap_amd import base, benchmarks, tools
    tb = base.Toolbox()
    tb.register("evaluate", benchmarks.onemax)
    tb.register("mate", tools.cxTwoPoint)
    tb.register("mutate", tools.mutFlipBit, indpb=0.05)
    tb.register("select", tools.selTournament, tournsize=3)
    tb.register("migrate", tools.migRing, k=K, selection=tools.selBest)
    return tb


def _evolve(ids, n_demes=N_DEMES, migarray=None):
    from deap_amd import islands, tools
    from deap_amd.ops import RandomStream
    streams = [RandomStream(64, island=d) for d in ids]
    demes = [tools.initPopulation(n=N, dim=DIM, low=0, high=1, gtype="bits", weights=(1.0,),
                                  stream=s) for s in streams]
    tb = _toolbox()
    if migarray is not None:
        tb.register("migrate", tools.migRing, k=K, selection=tools.selBest, migarray=migarray)
    demes, log = islands.eaSimpleDemes(demes, tb, 0.5, 0.2, NGEN, mig_every=5, deme_ids=ids,
                                       n_demes=n_demes, streams=streams)
    return {d: p.to_numpy() for d, p in zip(ids, demes)}, log


def _worker(rank, world, port, ids_by_rank, migarray, q, backend="gloo"):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # gloo: both ranks on the one GPU of the box; nccl (RCCL): one GPU per rank
    torch.cuda.set_device(rank if backend == "nccl" else 0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", rank))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        got, log = _evolve(ids_by_rank[rank], migarray=migarray)
        q.put((rank, {d: (g, wv) for d, (g, wv, _) in got.items()},
               [(r["gen"], r["deme"], r["evals"]) for r in log]))
    except BaseException as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e), None))
        raise
    finally:
        from deap_amd import islands
        islands.close_comms()
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("ids_by_rank,migarray", [
    ([[0, 1], [2, 3]], None),          # even split, ring crosses ranks twice
    ([[0, 2], [1, 3]], None),          # interleaved: every hop is cross-rank
    ([[0, 1, 2, 3], []], None),        # rank 1 holds no deme
    ([[3], [0, 1, 2]], [2, 3, 1, 0]),  # uneven split, another permutation
])
def test_two_ranks_equal_one_process(gpu, ids_by_rank, migarray):
    _run_two_ranks(ids_by_rank, migarray, "gloo")


def _run_two_ranks(ids_by_rank, migarray, backend):
    import torch.multiprocessing as mp
    want, want_log = _evolve(list(range(N_DEMES)), migarray=migarray)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, ids_by_rank, migarray, q, backend))
             for r in range(2)]
    for p in procs:
        p.start()
    got, logs = {}, []
    try:
        for _ in procs:
            rank, part, log = q.get(timeout=100)
            assert isinstance(part, dict), "rank %d failed: %s" % (rank, part)
            got.update(part)
            logs.extend(log)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    assert sorted(got) == list(range(N_DEMES))
    for d in range(N_DEMES):
        assert np.array_equal(got[d][0], want[d][0]), "deme %d genomes" % d
        assert np.array_equal(got[d][1], want[d][1]), "deme %d fitness" % d
    assert sorted(logs) == sorted((r["gen"], r["deme"], r["evals"]) for r in want_log)


@pytest.mark.parametrize("ids_by_rank,migarray", [
    ([[0, 1], [2, 3]], None),          # even split, the ring crosses GPUs twice
    ([[0, 2], [1, 3]], None),          # interleaved: every hop crosses GPUs
    ([[0, 1, 2, 3], []], None),        # GPU 1 holds no deme, joins every exchange
    ([[3], [0, 1, 2]], [2, 3, 1, 0]),  # uneven split, another permutation
])
def test_two_gpus_rccl_equal_one_process(gpu, ids_by_rank, migarray):
    """The cross-GPU exchange itself: two ranks on two
    GPUs with the ``nccl`` (RCCL) process group, so every cross-rank hop goes
    through ``dm_mig_ring_rccl`` (the ranks' agreement ``ncclAllReduce``, the
    grouped ``ncclSend`` / ``ncclRecv`` of the packed emigrants over xGMI,
    the placement on the receiver).  ``eaSimpleDemes`` with 4 OneMax demes
    and migRing every 5 generations (examples/ga/onemax_island.py:140-154,
    deap/tools/migration.py:4-51) must equal the single-process run row for
    row, which test_gpu_islands.py replays in the oracle.  Skips on a box
    with one GPU (RCCL refuses two ranks on one device)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    _run_two_ranks(ids_by_rank, migarray, "nccl")


def test_second_hop_into_a_deme_has_no_identity_match(gpu):
    """migarray [1, 1, 0]: deme 1 receives twice.  Its immigrant row 2 holds a
    NaN genome, so list.index finds it only by identity.  The first hop
    (0 -> 1) overwrites that row; on the second hop (1 -> 1) the immigrant
    object is no longer in the list and ``populations[1].index(immigrant)``
    raises ValueError (deap/tools/migration.py:48-51, restated below with
    Python lists of the same objects).  The device must not match the
    overwritten row by its old identity."""
    import torch
    from deap_amd import tools
    from deap_amd.device import DevicePopulation

    genes = [np.arange(12, dtype=np.float64).reshape(3, 4) + 100 * d for d in range(3)]
    genes[1][2, 0] = np.nan
    demes = [DevicePopulation.from_numpy(g, (1.0,), wvalues=g[:, 1:2] if d != 1 else
                                         np.array([[0.], [1.], [5.]]), valid=np.ones(3))
             for d, g in enumerate(genes)]
    # the reference's loop over host objects
    host = [[list(r) for r in g] for g in genes]
    em = [[host[0][2]], [host[1][2]], [host[2][2]]]   # selBest(k=1) of each deme
    ref_err = None
    try:
        for frm, to in enumerate([1, 1, 0]):
            for i, imm in enumerate(em[to]):
                host[to][host[to].index(imm)] = em[frm][i]
    except ValueError as e:
        ref_err = e
    assert ref_err is not None

    # selBest(k=1) picks row 2 of every deme (the largest weighted fitness)
    with pytest.raises(ValueError):
        tools.migRing(demes, 1, tools.selBest, migarray=[1, 1, 0])
    # the first hop was applied before the failing lookup, as in the reference
    g1, _, _ = demes[1].to_numpy()
    assert np.array_equal(g1[2], genes[0][2])
    del torch


def test_self_hop_keeps_identity_for_a_later_hop(gpu):
    """migarray [0, 0]: deme 0 sends to itself, then deme 1 sends into deme 0
    (ADVICE r3).  Deme 0's emigrant (row 2, a NaN genome: list.index finds it
    only by identity) goes back into its own row on the self hop -- the same
    object, so the second hop still finds that immigrant by identity and
    replaces it with deme 1's emigrant (deap/tools/migration.py:48-51,
    restated below with Python lists of the same objects).  The device must
    keep that row matchable after the self hop."""
    from deap_amd import tools
    from deap_amd.device import DevicePopulation

    genes = [np.arange(12, dtype=np.float64).reshape(3, 4) + 100 * d for d in range(2)]
    genes[0][2, 0] = np.nan
    demes = [DevicePopulation.from_numpy(g, (1.0,), wvalues=g[:, 1:2], valid=np.ones(3))
             for g in genes]
    host = [[list(r) for r in g] for g in genes]
    em = [[host[0][2]], [host[1][2]]]  # selBest(k=1): row 2 of each deme
    for frm, to in enumerate([0, 0]):
        for i, imm in enumerate(em[to]):
            host[to][host[to].index(imm)] = em[frm][i]
    assert host[0][2] is em[1][0]  # the reference replaced the NaN row
    tools.migRing(demes, 1, tools.selBest, migarray=[0, 0])
    g0, _, _ = demes[0].to_numpy()
    assert np.array_equal(g0, np.array(host[0]), equal_nan=True)
    assert np.array_equal(g0[2], genes[1][2])


def test_row_taken_and_restored_in_a_self_hop_keeps_identity(gpu):
    """within one self hop a row is first taken by another emigrant
    and then gets its own object back; the row's identity must follow its
    FINAL occupant.  Deme 0 = [x (NaN genome, list.index finds it only by
    identity), e0]; selBest(2) = [e0, x] emigrate, selWorst(2) = [x, e0] are
    replaced; migarray [0, 0]: the self hop puts e0 into x's row and then x
    back into it, so the second hop (deme 1 -> deme 0) still finds x there by
    identity (deap/tools/migration.py:39-51, restated below with Python lists
    of the same objects)."""
    from deap_amd import tools
    from deap_amd.device import DevicePopulation

    genes = [np.arange(8, dtype=np.float64).reshape(2, 4) + 100 * d for d in range(2)]
    genes[0][0, 1] = np.nan
    fits = [np.array([[1.0], [5.0]]), np.array([[3.0], [4.0]])]
    demes = [DevicePopulation.from_numpy(g, (1.0,), wvalues=f, valid=np.ones(2))
             for g, f in zip(genes, fits)]
    host = [[list(r) for r in g] for g in genes]
    em = [[host[d][1], host[d][0]] for d in range(2)]   # selBest(2): fitness descending
    imm = [[host[d][0], host[d][1]] for d in range(2)]  # selWorst(2): ascending
    for frm, to in enumerate([0, 0]):
        for i, x in enumerate(imm[to]):
            host[to][host[to].index(x)] = em[frm][i]
    assert host[0][0] is em[1][0] and host[0][1] is em[1][1]
    tools.migRing(demes, 2, tools.selBest, replacement=tools.selWorst, migarray=[0, 0])
    g0, _, _ = demes[0].to_numpy()
    assert np.array_equal(g0, np.array(host[0]), equal_nan=True)
    assert np.array_equal(g0, genes[1][[1, 0]])
