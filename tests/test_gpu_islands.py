"""C4 on one GPU: several demes evolving with eaSimple generations and a
migRing every 5 generations (examples/ga/onemax_multidemic.py:79-93,
deap/tools/migration.py:4-51), replayed generation by generation in the CPU
oracle from the decisions the device drew (dump mode) and the migrations'
selected rows.  Genomes and `nevals` are bit-exact; fp64 fitness within
1e-12 relative (north star), OneMax fitness exact."""
import numpy as np
import pytest

from oracle import ops

pytestmark = pytest.mark.gpu


def _rel_close(a, b, tol):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= tol * np.maximum(1.0, np.abs(b)))


def _toolbox(gt, k, replacement):
    import random
    from deap_amd import base, benchmarks, tools
    tb = base.Toolbox()
    if gt == "bits":
        tb.register("evaluate", benchmarks.onemax)
        tb.register("mate", tools.cxTwoPoint)
        tb.register("mutate", tools.mutFlipBit, indpb=0.05)
    else:
        tb.register("evaluate", benchmarks.rastrigin)
        tb.register("mate", tools.cxBlend, alpha=0.5)
        tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
    tb.register("select", tools.selTournament, tournsize=3)
    tb.register("migrate", tools.migRing, k=k, selection=tools.selBest,
                replacement=random.sample if replacement == "sample" else None)
    return tb


def _decisions(dn, dim):
    return {"aspirants": dn["aspirants"], "cx_flag": dn["cx_flag"].astype(bool),
            "cx_raw": dn.get("cx_raw"), "blend_u": dn.get("blend_u"),
            "mut_flag": dn["mut_flag"].astype(bool),
            "mut_mask": ops.unpack_mask(dn["mut_mask"], dim), "gauss": dn.get("gauss")}


def _run(gt, dim, n, n_demes, ngen, k, replacement, force_p2p=False, snapshots=None):
    from deap_amd import islands, tools
    from deap_amd.ops import RandomStream
    w = (1.0,) if gt == "bits" else (-1.0,)
    low, high = (0, 1) if gt == "bits" else (-5.12, 5.12)
    streams = [RandomStream(64, island=d) for d in range(n_demes)]
    demes = [tools.initPopulation(n=n, dim=dim, low=low, high=high, gtype=gt, weights=w,
                                  stream=streams[d]) for d in range(n_demes)]
    init = [d.genes_numpy() for d in demes]
    decs, record = {}, []
    tb = _toolbox(gt, k, replacement)

    def snap(gen, stage, ds):
        snapshots.append((gen, stage, [d.to_numpy() for d in ds]))

    demes, log = islands.eaSimpleDemes(demes, tb, 0.5, 0.2, ngen, mig_every=5, streams=streams,
                                       mode="dump", decisions=decs, record=record,
                                       force_p2p=force_p2p,
                                       callback=snap if snapshots is not None else None)
    return demes, log, init, decs, record, w


def _replay(gt, dim, n_demes, ngen, k, init, decs, record, w):
    obj = "onemax" if gt == "bits" else "rastrigin"
    state = []
    for d in range(n_demes):
        g = init[d].copy()
        wv = ops.evaluate(g, obj, w)
        state.append({"genes": g, "wvalues": wv, "valid": np.ones(len(g), bool)})
    nevals = {d: [len(init[d])] for d in range(n_demes)}
    mig = iter(record)
    for gen in range(1, ngen + 1):
        for d in range(n_demes):
            s = state[d]
            dn = decs[d][gen - 1].numpy()
            g, wv, ok, nev = ops.ea_generation(s["genes"], s["wvalues"], s["valid"], 0.5, 0.2,
                                               "twopoint" if gt == "bits" else "blend",
                                               "flipbit" if gt == "bits" else "gaussian",
                                               _decisions(dn, dim), obj, w)
            state[d] = {"genes": g, "wvalues": wv, "valid": ok}
            nevals[d].append(nev)
        if gen % 5 == 0:
            rec = next(mig)
            for d in range(n_demes):
                em = ops.sel_best(state[d]["wvalues"], k)
                got = rec["emigrants"][d]
                if gt == "bits":
                    assert got.tolist() == em.tolist(), (gen, d)
                else:
                    # fp64 fitness agrees to 1e-12 relative, so two rows whose
                    # fitnesses are that close may swap ranks: the device's
                    # choice must be a selBest under the oracle's values up to
                    # that tolerance, and its rows are then replayed
                    assert _rel_close(state[d]["wvalues"][got], state[d]["wvalues"][em], 1e-12), \
                        (gen, d, got, em)
            im = None if rec["immigrants"][0] is None else rec["immigrants"]
            ops.mig_ring(state, rec["emigrants"], im)
    return state, nevals


@pytest.mark.parametrize("gt,dim,n,n_demes,replacement", [
    ("bits", 100, 64, 4, None),
    ("bits", 100, 64, 3, "sample"),          # the multidemic example's replacement
])
def test_demes_with_migration_replay_in_oracle(gpu, gt, dim, n, n_demes, replacement):
    """Packed-bit OneMax demes (exact fitness): the whole 12-generation
    trajectory with two migrations replayed in the oracle from the initial
    demes alone."""
    ngen, k = 12, 5
    demes, log, init, decs, record, w = _run(gt, dim, n, n_demes, ngen, k, replacement)
    assert len(record) == ngen // 5
    state, nevals = _replay(gt, dim, n_demes, ngen, k, init, decs, record, w)
    for d in range(n_demes):
        g, wv, ok = demes[d].to_numpy()
        assert np.array_equal(g, state[d]["genes"]), d
        assert ok.all()
        assert _rel_close(wv, state[d]["wvalues"], 0 if gt == "bits" else 1e-12), d
    got = {}
    for rec in log:
        got.setdefault(rec["deme"], []).append(rec["evals"])
    assert got == nevals


def test_demes_migration_through_rccl_self_p2p(gpu):
    """The same run with every hop between two demes sent through the RCCL
    communicator (ncclSend/ncclRecv to this rank itself): identical result."""
    a = _run("f64", 64, 40, 4, 10, 5, None, force_p2p=False)
    b = _run("f64", 64, 40, 4, 10, 5, None, force_p2p=True)
    for da, db in zip(a[0], b[0]):
        ga, wa, _ = da.to_numpy()
        gb, wb, _ = db.to_numpy()
        assert np.array_equal(ga, gb)
        assert np.array_equal(wa, wb)
    assert [r["emigrants"][0].tolist() for r in a[4]] == [r["emigrants"][0].tolist() for r in b[4]]


def test_sel_sample_distinct_and_uniform(gpu):
    """random.sample on the device: k distinct rows of [0, n), both paths
    (rejection for small k, key sort for large k); roughly uniform."""
    import torch
    from deap_amd.device import DevicePopulation
    from deap_amd.ops import RandomStream
    from deap_amd.tools import migration
    pop = DevicePopulation(1000, 4, "f64", (1.0,))
    st = RandomStream(3)
    counts = np.zeros(1000)
    for _ in range(2000):
        idx = migration.sample_indices(pop, 15, st).cpu().numpy()
        assert len(set(idx.tolist())) == 15 and idx.min() >= 0 and idx.max() < 1000
        counts[idx] += 1
    # 30,000 draws over 1,000 rows: Poisson(30) per row, P(outside [8, 60]) < 1e-7
    assert counts.min() >= 8 and counts.max() <= 60, (counts.min(), counts.max())
    for k in (600, 1000):  # key-sort path (2k > n)
        idx = migration.sample_indices(pop, k, st).cpu().numpy()
        assert len(set(idx.tolist())) == k and idx.min() >= 0 and idx.max() < 1000
    with pytest.raises(ValueError):
        migration.sample_indices(pop, 1001, st)
    assert migration.sample_indices(pop, 0, st).numel() == 0
    del torch


def test_mig_place_identity_with_nan_genome(gpu):
    """list.index finds the immigrant itself (`is`) even if its genome holds a
    NaN (NaN != NaN): the device placement matches identity first."""
    import torch
    from deap_amd.device import DevicePopulation
    from deap_amd.tools import migration
    genes = np.arange(40, dtype=np.float64).reshape(10, 4)
    genes[3, 1] = np.nan
    a = DevicePopulation.from_numpy(genes, (1.0,), wvalues=np.arange(10.0)[:, None],
                                    valid=np.ones(10))
    b = DevicePopulation.from_numpy(genes + 100, (1.0,), wvalues=np.arange(10.0)[:, None] + 100,
                                    valid=np.ones(10))
    im = migration.pack(a, torch.tensor([3, 5], dtype=torch.int32, device=a.device))
    em = migration.pack(b, torch.tensor([0, 1], dtype=torch.int32, device=b.device))
    slots = migration.place(a, im, em, 2).cpu().tolist()
    assert slots == [3, 5]
    g, wv, _ = a.to_numpy()
    assert np.array_equal(g[3], genes[0] + 100) and np.array_equal(g[5], genes[1] + 100)


@pytest.mark.parametrize("dim,n,n_demes,replacement", [(100, 48, 8, None), (64, 33, 5, "sample")])
def test_fp64_demes_stepwise_replay_in_oracle(gpu, dim, n, n_demes, replacement):
    """Rastrigin fp64 demes: fitness agrees with the oracle to 1e-12 relative,
    and a converging deme holds near-identical rows whose fitnesses lie within
    that tolerance, so a long trajectory replayed from the initial demes alone
    can flip a tournament.  Stage isolation instead: every generation is
    replayed in the oracle from the device's state before it (genomes
    bit-exact, fitness 1e-12), and every migration from the device's state
    before it with the device's emigrant rows (bit-exact), the rows checked to
    be a selBest under the oracle's fitness to the same tolerance."""
    ngen, k = 12, 5
    snaps = []
    demes, log, init, decs, record, w = _run("f64", dim, n, n_demes, ngen, k, replacement,
                                             snapshots=snaps)
    prev = []
    for d in range(n_demes):
        g = init[d].copy()
        prev.append((g, ops.evaluate(g, "rastrigin", w), np.ones(len(g), bool)))
    mig = iter(record)
    for gen, stage, state in snaps:
        if stage == "generation":
            for d in range(n_demes):
                g0, wv0, ok0 = prev[d]
                dn = decs[d][gen - 1].numpy()
                g, wv, ok, nev = ops.ea_generation(g0, wv0, ok0, 0.5, 0.2, "blend", "gaussian",
                                                   _decisions(dn, dim), "rastrigin", w)
                assert np.array_equal(state[d][0], g), (gen, d)
                assert _rel_close(state[d][1], wv, 1e-12), (gen, d)
        else:
            rec = next(mig)
            before = [{"genes": prev[d][0].copy(), "wvalues": prev[d][1].copy(),
                       "valid": prev[d][2].copy()} for d in range(n_demes)]
            for d in range(n_demes):
                em = ops.sel_best(before[d]["wvalues"], k)
                got = rec["emigrants"][d]
                assert _rel_close(before[d]["wvalues"][got], before[d]["wvalues"][em], 1e-12)
            im = None if rec["immigrants"][0] is None else rec["immigrants"]
            ops.mig_ring(before, rec["emigrants"], im)
            for d in range(n_demes):
                assert np.array_equal(state[d][0], before[d]["genes"]), (gen, d)
                assert np.array_equal(state[d][1], before[d]["wvalues"]), (gen, d)
        prev = [(s[0], s[1], s[2].astype(bool)) for s in state]
    assert len(record) == ngen // 5


@pytest.mark.parametrize("k,replacement", [(64, None), (3000, None), (3000, "sample"),
                                            (4096, None)])
def test_placement_with_heavy_duplicates_matches_list_index(gpu, k, replacement):
    """migRing(k, selBest) over two demes of 6-bit genomes (64 distinct
    values among 20,000 rows, so nearly every immigrant has earlier equal rows
    and equal emigrants): the device placement against the reference loop
    (migration.py:44-51) replayed on the host by value -- ``list.index`` is
    the first row whose genome equals the immigrant, as the earlier
    placements left the deme (no NaN genome, so identity adds nothing), up
    to the library's k limit of 4,096; a taken first match (the masked bitmap
    scan) and an equal earlier emigrant at a smaller row (rule b) occur in
    every case."""
    import random
    import torch
    from deap_amd import benchmarks, tools
    from deap_amd.ops import RandomStream
    n, dim = 20000, 6
    demes = []
    for d in range(2):
        p = tools.initPopulation(n=n, dim=dim, gtype="bits", weights=(1.0,),
                                 stream=RandomStream(77, island=d))
        benchmarks.onemax(p)
        demes.append(p)
    val = [np.packbits(p.rows_numpy(range(n))[0].astype(np.uint8), axis=1, bitorder="little")[:, 0]
           .astype(np.int64) for p in demes]
    fit = [p.wvalues[:n, 0].cpu().numpy().copy() for p in demes]
    rec = []
    tools.migRing(demes, k, tools.selBest,
                  replacement=random.sample if replacement == "sample" else None, record=rec)
    torch.cuda.synchronize()
    em = rec[0]["emigrants"]
    im = em if replacement is None else rec[0]["immigrants"]
    cur = [(v.copy(), f.copy()) for v, f in zip(val, fit)]
    for frm, to in enumerate([1, 0]):                      # migration.py:48-51
        cv, cf = cur[to]
        for i in range(k):
            target = val[to][int(im[to][i])]
            hit = np.flatnonzero(cv == target)
            assert hit.size, "immigrant %d of deme %d not found" % (i, to)
            s = int(hit[0])
            cv[s] = val[frm][int(em[frm][i])]
            cf[s] = fit[frm][int(em[frm][i])]
    for d in range(2):
        got = np.packbits(demes[d].rows_numpy(range(n))[0].astype(np.uint8), axis=1,
                          bitorder="little")[:, 0].astype(np.int64)
        assert np.array_equal(got, cur[d][0]), "deme %d genomes differ from the replay" % d
        assert np.array_equal(demes[d].wvalues[:n, 0].cpu().numpy(), cur[d][1])
