"""Island model routing across ranks on CPU: world_size 2,
``gloo`` backend, 4 demes split 2 per rank.  The device pack/placement
kernels are replaced by host restatements (test infrastructure) so the test
exercises exactly what is distributed: which deme's emigrant block reaches
which rank, in which order placements happen, and that the result equals the
single-process migRing of the oracle (``deap/tools/migration.py:4-51``)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_DEMES, N, D, K = 4, 40, 6, 5


def _demes(seed):
    rng = np.random.default_rng(seed)
    out = []
    for d in range(N_DEMES):
        genes = rng.integers(0, 3, size=(N, D)).astype(np.float64)  # many duplicates
        genes[1] = genes[0]
        wv = genes.sum(axis=1, keepdims=True) + 0.0
        out.append({"genes": genes, "wvalues": wv, "valid": np.ones(N, np.uint8)})
    return out


class HostDeme:
    """Stand-in for a DevicePopulation holding numpy rows."""

    def __init__(self, deme):
        self.d = deme


def _pack(pop, idx):
    idx = np.asarray(idx)
    d = pop.d
    return torch.from_numpy(np.concatenate([
        d["genes"][idx].view(np.uint8).ravel(), d["wvalues"][idx].view(np.uint8).ravel(),
        d["valid"][idx].ravel()]).copy())


def _unpack(block, k):
    b = block.numpy()
    g = b[:k * D * 8].view(np.float64).reshape(k, D)
    w = b[k * D * 8:k * D * 8 + k * 8].view(np.float64).reshape(k, 1)
    v = b[k * D * 8 + k * 8:k * D * 8 + k * 8 + k]
    return g, w, v


def _place(pop, imm_block, emi_block, k):
    ig, _, _ = _unpack(imm_block, k)
    eg, ew, ev = _unpack(emi_block, k)
    dst = pop.d
    for j in range(k):                              # migration.py:48-51
        hit = int(np.nonzero(np.all(dst["genes"] == ig[j][None, :], axis=1))[0][0])
        dst["genes"][hit], dst["wvalues"][hit], dst["valid"][hit] = eg[j], ew[j], ev[j]


def _select(selection, pop, k, stream):
    from oracle import ops
    return ops.sel_best(pop.d["wvalues"], k)


def _worker(rank, world, port, seed, migarray, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from deap_amd import islands
        islands.pack, islands.place, islands._select = _pack, _place, _select
        demes = _demes(seed)
        per = N_DEMES // world
        ids = list(range(rank * per, (rank + 1) * per))
        mine = [HostDeme(demes[i]) for i in ids]
        islands.migRingDistributed(mine, ids, N_DEMES, K, selection=None, migarray=migarray,
                                   stream=object())
        q.put((rank, {i: (m.d["genes"].copy(), m.d["wvalues"].copy()) for i, m in zip(ids, mine)}))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("migarray", [None, [2, 3, 1, 0], [1, 0, 3, 2]])
def test_mig_ring_distributed_matches_single_process(migarray):
    from oracle import ops
    seed = 11
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, seed, migarray, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        _, part = q.get(timeout=120)
        got.update(part)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _demes(seed)
    em = [ops.sel_best(d["wvalues"], K) for d in ref]
    ops.mig_ring(ref, em, None, migarray)
    for d in range(N_DEMES):
        assert np.array_equal(got[d][0], ref[d]["genes"]), "deme %d genomes" % d
        assert np.array_equal(got[d][1], ref[d]["wvalues"]), "deme %d fitness" % d


def test_owner_map_single_rank_owns_all():
    from deap_amd import islands
    assert islands.owner_map([0, 1, 2], 3, 1, None) == {0: 0, 1: 0, 2: 0}


def _worker_split(rank, world, port, seed, ids_by_rank, migarray, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from deap_amd import islands
        islands.pack, islands.place, islands._select = _pack, _place, _select
        demes = _demes(seed)
        ids = ids_by_rank[rank]
        mine = [HostDeme(demes[i]) for i in ids]
        islands.migRingDistributed(mine, ids, N_DEMES, K, selection=None, migarray=migarray,
                                   stream=object())
        q.put((rank, {i: (m.d["genes"].copy(), m.d["wvalues"].copy()) for i, m in zip(ids, mine)}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ids_by_rank,migarray", [
    ([[0, 3], [1, 2]], None),             # interleaved ownership
    ([[2], [0, 1, 3]], [3, 2, 0, 1]),      # uneven split
    ([[1, 2, 3], [0]], [0, 2, 1, 3]),      # self hops (deme migrates into itself)
])
def test_mig_ring_distributed_any_split(ids_by_rank, migarray):
    """owner_map accepts any split agreed through all_gather_object."""
    from oracle import ops
    seed = 23
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_split, args=(r, 2, port, seed, ids_by_rank, migarray, q))
             for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        _, part = q.get(timeout=120)
        got.update(part)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _demes(seed)
    em = [ops.sel_best(d["wvalues"], K) for d in ref]
    ops.mig_ring(ref, em, None, migarray)
    for d in range(N_DEMES):
        assert np.array_equal(got[d][0], ref[d]["genes"]), "deme %d genomes" % d
        assert np.array_equal(got[d][1], ref[d]["wvalues"]), "deme %d fitness" % d


@pytest.mark.parametrize("migarray", [None, [2, 3, 1, 0], [0, 2, 1, 3], [1, 1, 3, 2]])
@pytest.mark.parametrize("owner", [[0, 0, 0, 0], [0, 1, 0, 1], [1, 1, 0, 0], [0, 0, 1, 2]])
def test_c_mig_plan_matches_python_routing(migarray, owner):
    """dm_mig_plan (the C ABI's routing, host-only) gives, for every rank,
    exactly the hops route_blocks performs: local references, sends and
    receives, in from_deme order."""
    from deap_amd import _lib, islands
    if not __import__("os").path.exists(_lib.LIB_PATH):
        pytest.skip("libdeapmi.so not built")
    n = len(owner)
    mig = migarray if migarray is not None else list(range(1, n)) + [0]
    for me in sorted(set(owner)):
        want = []
        for frm, to in enumerate(mig):
            s, d = owner[frm], owner[to]
            if s == me and d == me:
                want.append(("local", frm, to, me))
            elif s == me:
                want.append(("send", frm, to, d))
            elif d == me:
                want.append(("recv", frm, to, s))
        assert islands.mig_plan(n, migarray, dict(enumerate(owner)), me) == want
    # the single-GPU RCCL test hook: local hops between different demes
    # become a send/recv pair to the rank itself
    hops = islands.mig_plan(n, migarray, {d: 0 for d in range(n)}, 0, force_p2p=True)
    for frm, to in enumerate(mig):
        if frm == to:
            assert ("local", frm, to, 0) in hops
        else:
            i = hops.index(("send", frm, to, 0))
            assert hops[i + 1] == ("recv", frm, to, 0)
