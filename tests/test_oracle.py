"""The CPU oracle against the reference's golden vectors (CPU only)."""
import ast

import numpy as np
import pytest

from conftest import golden
from oracle import ops, philox


# Random123 philox4x32-10 known-answer vectors (kat_vectors)
KAT = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
       ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
       ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
        (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]


@pytest.mark.parametrize("ctr,key,expect", KAT)
def test_philox_kat(ctr, key, expect):
    out = philox.philox4x32_10(np.array([ctr], np.uint64), key)[0]
    assert tuple(int(x) for x in out) == expect


def test_bounded64_matches_bigint():
    rng = np.random.default_rng(1)
    lo = rng.integers(0, 2 ** 32, 1000, dtype=np.uint64)
    hi = rng.integers(0, 2 ** 32, 1000, dtype=np.uint64)
    for n in (1, 2, 3, 300, 2 ** 20, 2 ** 31 - 1):
        got = philox.bounded64(lo, hi, n)
        want = [((int(h) << 32 | int(l)) * n) >> 64 for l, h in zip(lo, hi)]
        assert got.tolist() == want


def _rel_close(a, b, tol=1e-12):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= tol * np.maximum(1.0, np.abs(b)))


def test_eval_matches_reference():
    d = golden("eval.npz")
    j = 0
    while "eval%d_x" % j in d:
        name, kw = d["eval%d_meta" % j]
        kw = ast.literal_eval(kw)
        x = d["eval%d_x" % j]
        f = d["eval%d_f" % j]
        got = ops.evaluate(x, name, (1.0,) * f.shape[1], **kw)
        assert np.array_equal(got, f), name  # same libm, same order: exact
        j += 1
    got = ops.evaluate(d["onemax_x"], "onemax", (1.0,))
    assert np.array_equal(got[:, 0], d["onemax_f"])
    got = ops.evaluate(d["rastrigin_f32_x"], "rastrigin", (1.0,))
    assert np.array_equal(got[:, 0], d["rastrigin_f32_f"])


def test_var_and_matches_reference():
    d = golden("varand.npz")
    j = 0
    while "va%d_genes" % j in d:
        k = "va%d_" % j
        gt, tc, cx, mut, cxpb, mutpb, indpb, alpha = d[k + "meta"]
        dec = {f: d[k + f] for f in ("cx_flag", "cx_raw", "blend_u", "mut_flag", "gauss")}
        dec["mut_mask"] = d[k + "mask"]
        g, wv, ok = ops.var_and(d[k + "genes"], d[k + "wv"], d[k + "valid"], float(cxpb),
                                float(mutpb), cx, mut, dec, float(alpha))
        assert np.array_equal(g, d[k + "out_genes"]), (j, gt, cx, mut)
        assert np.array_equal(ok, d[k + "out_valid"])
        assert np.array_equal(wv[ok], d[k + "out_wv"][ok])
        j += 1


def test_selection_matches_reference():
    d = golden("selection.npz")
    for j in range(3):
        k = "sel%d_" % j
        assert ops.sel_tournament(d[k + "wv"], d[k + "asp"]).tolist() == d[k + "out"].tolist()
        assert ops.sel_best(d[k + "wv"], 10).tolist() == d[k + "best"].tolist()
        assert ops.sel_worst(d[k + "wv"], 10).tolist() == d[k + "worst"].tolist()


def test_ea_generation_matches_reference():
    d = golden("generation.npz")
    j = 0
    while "ea%d_genes" % j in d:
        k = "ea%d_" % j
        gt, tc, cx, mut, objective, t, cxpb, mutpb, indpb, alpha, w0 = d[k + "meta"]
        dec = {f: d[k + f] for f in ("cx_flag", "cx_raw", "blend_u", "mut_flag", "gauss")}
        dec["mut_mask"] = d[k + "mask"]
        dec["aspirants"] = d[k + "asp"]
        g, wv, ok, nev = ops.ea_generation(d[k + "genes"], d[k + "wv"], d[k + "valid"],
                                           float(cxpb), float(mutpb), cx, mut, dec, objective,
                                           (float(w0),), float(alpha))
        assert np.array_equal(g, d[k + "out_genes"]), j
        assert np.array_equal(wv, d[k + "out_wv"]), j
        assert nev == d[k + "nevals"][1]
        j += 1


def test_var_or_matches_reference():
    d = golden("varor.npz")
    for j in range(2):
        k = "vo%d_" % j
        gt, tc, cx, mut, lam, cxpb, mutpb, indpb, alpha = d[k + "meta"]
        dec = {"varor_op": d[k + "op"], "varor_idx": d[k + "idx"], "cx_raw": d[k + "cx_raw"],
               "blend_u": d[k + "blend_u"], "mut_mask": d[k + "mask"], "gauss": d[k + "gauss"]}
        g, wv, ok = ops.var_or(d[k + "genes"], d[k + "wv"], d[k + "valid"], int(lam),
                               float(cxpb), float(mutpb), cx, mut, dec, float(alpha))
        assert np.array_equal(g, d[k + "out_genes"])
        assert np.array_equal(ok, d[k + "out_valid"])
        assert np.array_equal(wv[ok], d[k + "out_wv"][ok])


def test_nsga2_matches_reference():
    d = golden("nsga2.npz")
    for j in range(6):
        k = "nd%d_" % j
        wv, weights, kk = d[k + "wv"], d[k + "weights"], int(d[k + "k"])
        fronts = ops.sort_nondominated(wv, kk)
        flat = [i for f in fronts for i in f]
        assert flat == d[k + "order"].tolist()
        assert np.cumsum([0] + [len(f) for f in fronts]).tolist() == d[k + "fstart"].tolist()
        chosen, crowd = ops.sel_nsga2(wv, weights, kk)
        assert chosen == d[k + "chosen"].tolist()
        got = np.array([crowd[i] for i in flat])
        assert np.array_equal(got, d[k + "crowd"])
        assert len(ops.sort_nondominated(wv, kk, first_front_only=True)[0]) == d[k + "first"][0]


def test_closed_form_order_matches_reference_goldens():
    """oracle/nsga2_closed.py (the vectorised closed form of emo.py:53-117's
    front order, the checker of the benched size) == the reference-generated
    nsga2.npz order and selNSGA2 choice."""
    from oracle import nsga2_closed
    d = golden("nsga2.npz")
    for j in range(6):
        k = "nd%d_" % j
        wv, weights, kk = d[k + "wv"], tuple(d[k + "weights"]), int(d[k + "k"])
        fronts = nsga2_closed.sort_nondominated(wv, kk)
        assert np.concatenate(fronts).tolist() == d[k + "order"].tolist(), j
        assert np.cumsum([0] + [len(f) for f in fronts]).tolist() == d[k + "fstart"].tolist()
        chosen, crowd = nsga2_closed.sel_nsga2(wv, weights, kk, fronts=fronts)
        assert chosen == d[k + "chosen"].tolist(), j
        assert np.array_equal([crowd[i] for i in np.concatenate(fronts).tolist()], d[k + "crowd"])
        ff = nsga2_closed.sort_nondominated(wv, kk, first_front_only=True)
        assert len(ff) == 1 and len(ff[0]) == d[k + "first"][0]


@pytest.mark.parametrize("m", [2, 3, 4])
def test_closed_form_order_matches_the_restatement(m):
    """The closed form == oracle.ops.sort_nondominated (emo.py:53-117 line by
    line) and its selNSGA2, on continuous, tied, duplicated and signed-zero
    fitnesses, for k = n, n/2, 1, 0 and first_front_only."""
    from oracle import nsga2_closed
    rng = np.random.default_rng(40 + m)
    for trial in range(12):
        n = int(rng.integers(1, 500))
        kind = trial % 3
        if kind == 0:
            wv = rng.uniform(0, 1, (n, m))
        else:
            wv = rng.integers(0, 6, (n, m)).astype(np.float64)
            wv[rng.integers(0, n, n // 5)] = wv[rng.integers(0, n, n // 5)]
            if kind == 2:
                wv[rng.random((n, m)) < 0.2] *= -0.0
        w = tuple(rng.choice([-1.0, 1.0, 2.0], m))
        for k in (n, n // 2 + 1, 1, 0):
            want = ops.sort_nondominated(wv, k)
            assert [f.tolist() for f in nsga2_closed.sort_nondominated(wv, k)] == want
            if k:
                assert (nsga2_closed.sort_nondominated(wv, k, True)[0].tolist()
                        == ops.sort_nondominated(wv, k, True)[0])
                assert nsga2_closed.sel_nsga2(wv, w, k)[0] == ops.sel_nsga2(wv, w, k)[0]


def test_mig_ring_matches_reference():
    d = golden("migration.npz")
    for j in range(3):
        k = "mig%d_" % j
        nd, kk, repl = d[k + "meta"]
        nd, kk = int(nd), int(kk)
        demes = [{"genes": d[k + "in_genes%d" % i].copy(), "wvalues": d[k + "in_wv%d" % i].copy(),
                  "valid": np.ones(len(d[k + "in_wv%d" % i]), bool)} for i in range(nd)]
        em = [d[k + "sel%d" % i] for i in range(nd)]
        im = [d[k + "repl%d" % i] for i in range(nd)] if repl == "sample" else None
        ops.mig_ring(demes, em, im)
        for i in range(nd):
            assert np.array_equal(demes[i]["genes"], d[k + "out_genes%d" % i]), (j, i)
            assert np.array_equal(demes[i]["wvalues"], d[k + "out_wv%d" % i])


def test_c1_trajectory_replays_in_oracle():
    d = golden("c1_trajectory.npz")
    genes = d["c1_init"]
    n = genes.shape[0]
    wv = ops.evaluate(genes, "onemax", (1.0,))
    valid = np.ones(n, bool)
    nevals = [n]
    for g in range(40):
        dec = {"aspirants": d["c1_asp"][g], "cx_flag": d["c1_cx_flag"][g],
               "cx_raw": d["c1_cx_raw"][g], "mut_flag": d["c1_mut_flag"][g],
               "mut_mask": np.unpackbits(d["c1_mask"][g], axis=-1)[:, :100].astype(bool)}
        genes, wv, valid, nev = ops.ea_generation(genes, wv, valid, 0.5, 0.2, "twopoint",
                                                  "flipbit", dec, "onemax", (1.0,))
        nevals.append(nev)
    assert np.array_equal(genes, d["c1_final"])
    assert np.array_equal(wv, d["c1_final_wv"])
    assert nevals == d["c1_nevals"].tolist()


def test_sel_tournament_dcd_matches_reference():
    d = golden("dcd.npz")
    for j in range(5):
        key = "dcd%d_" % j
        got = ops.sel_tournament_dcd(d[key + "wv"], d[key + "crowd"], int(d[key + "k"]),
                                     d[key + "perm1"], d[key + "perm2"], d[key + "coin"])
        assert got == d[key + "chosen"].tolist(), j


def _sbx_case(d, j):
    k = "sbx%d_" % j
    cxpb, eta_c, eta_m, indpb = (float(v) for v in d[k + "meta"])
    low, up = d[k + "low"], d[k + "up"]
    dec = {"cx_u": d[k + "cx_u"], "sbx_u": d[k + "sbx_u"], "mut_u": d[k + "mut_u"]}
    return k, cxpb, (eta_c, low, up), (eta_m, low, up, indpb), dec


def test_vary_bounded_matches_reference():
    """NSGA-II loop body: cxSimulatedBinaryBounded + mutPolynomialBounded
    (examples/ga/nsga2.py:96-105), bit-exact against DEAP on replayed random()s."""
    d = golden("sbx.npz")
    for j in range(4):
        k, cxpb, sbx, poly, dec = _sbx_case(d, j)
        n = len(d[k + "genes"])
        g, _wv, ok = ops.vary_bounded(d[k + "genes"], np.zeros((n, 2)), np.ones(n, bool),
                                      d[k + "idx"], cxpb, dec, sbx, poly)
        assert np.array_equal(g, d[k + "out"]), j
        assert np.array_equal(ok, d[k + "valid"]), j


def test_sort_log_nondominated_matches_reference():
    """sortLogNondominated front order + selNSGA2(nd='log') (emo.py:15-50,234-276)."""
    d = golden("nsga2log.npz")
    for j in range(6):
        key = "log%d_" % j
        wv, k = d[key + "wv"], int(d[key + "k"])
        weights = [-1.0, 1.0, -1.0, 1.0][:wv.shape[1]]
        fronts = ops.sort_log_nondominated(wv, k)
        assert [len(f) for f in fronts] == d[key + "sizes"].tolist(), j
        assert [i for f in fronts for i in f] == d[key + "order"].tolist(), j
        assert ops.sel_nsga2_log(wv, weights, k) == d[key + "chosen"].tolist(), j
