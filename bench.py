#!/usr/bin/env python3
"""Benchmark of the DEAP population hot path on MI355X.

Metric (BASELINE.json): individual-generations/sec @ pop = 2^20,
Rastrigin-1000D fp64, 1-8 GPUs.  A *step* is one eaSimple generation over the
whole population — select (selTournament t=3) -> clone -> varAnd (cxBlend
alpha=0.5, cxpb 0.5; mutGaussian mu=0 sigma=1 indpb=0.05, mutpb 0.2) ->
evaluate invalid — as ONE fused kernel (``dm_generation``), population resident
in HBM, synthetic random-init genomes (U[-5.12, 5.12]).

N=1: config C3 (one island of 2^20).  N>1 (torchrun, one rank per GPU): one
2^20 island per GPU (weak scaling, config C4) with migRing every 5 gens (k=15,
selBest, ring i -> i+1) exchanged with RCCL point-to-point from inside
libdeapmi (dm_mig_ring_rccl); value = all ranks' individual-generations /
max-over-ranks time.  ``--islands-per-gpu I`` runs I demes of --pop per GPU
(weak); ``--islands 8`` is config C4 literally: 8 demes of 2^20 split over the
N GPUs (8/4/2/1 per GPU, strong scaling); ``migration`` reports the cost of
the migrations (HIP events) separately.

``roofline``: algorithmic bytes per individual-generation B = 2G + (t+1)F
(2*8000 + 4*8 = 16,032 B for C3) x individuals per launch /
average fused-kernel duration measured with HIP events on the launch stream;
peak 8,000 GB/s (MI355X HBM3E).  ``traffic``: HBM bytes per launch from the
rocprofv3 PMC pass committed under profiles/ (or null).
``cpu_baseline``: DEAP-faithful pure-Python eaSimple (oracle/deap_port.py,
array('d') genomes, deepcopy clone, multiprocessing.Pool map) on a bounded
sample, rank 0 at N=1 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (problem, gtype, dim, cx, mut, weights, bytes per ind-gen)
    "c3": ("rastrigin", "f64", 1000, "blend", "gaussian", (-1.0,), 2 * 8000 + 4 * 8),
    "c3r": ("rosenbrock", "f64", 1000, "blend", "gaussian", (-1.0,), 2 * 8000 + 4 * 8),
    "c2": ("onemax", "bits", 4096, "twopoint", "flipbit", (1.0,), 2 * 512 + 4 * 8),
}
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS) + ["c5", "c5x"])
    ap.add_argument("--pop", type=int, default=1 << 20)
    ap.add_argument("--islands-per-gpu", type=int, default=1,
                    help="demes of --pop individuals per GPU (weak scaling)")
    ap.add_argument("--islands", type=int, default=0,
                    help="total demes, split evenly over the GPUs (C4: 8; strong scaling)")
    ap.add_argument("--mig-every", type=int, default=5)
    ap.add_argument("--mig-k", type=int, default=15)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=65536)
    ap.add_argument("--seed", type=int, default=1234)
    return ap.parse_args()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_workers():
    """Worker processes for the CPU baseline: every CPU this process may run
    on (sched_getaffinity), capped at the 16-CPU share the GPU box grants one
    GPU (its os.cpu_count() reports the whole machine)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return max(1, min(avail, int(os.environ.get("DM_CPU_WORKERS", "16")))), avail


def cpu_baseline(problem, sample):
    from oracle import deap_port
    workers, avail = host_workers()
    dim = CONFIGS_DIM[problem]
    rate, secs, used = deap_port.run(problem, n=sample, dim=dim, ngen=2, workers=workers)
    return {"value": rate, "unit": "individual-generations/sec", "cores": used, "kind": "port",
            "cpu_model": cpu_model(), "cpus_visible": avail,
            "sample": "DEAP-faithful eaSimple (oracle/deap_port.py, bit-exact with the reference on "
                      "tests/golden/port.npz: array genomes, deepcopy clone, Pool(%d).map "
                      "evaluate), pop %d x %d genes, 2 timed generations (%.1f s)"
                      % (used, sample, dim, secs)}


CONFIGS_DIM = {"rastrigin": 1000, "rosenbrock": 1000, "onemax": 4096}
METRICS = {
    "c3": "individual-generations/sec @pop=2^20 Rastrigin-1000D, 1-8 GPU; % HBM peak",
    "c3r": "individual-generations/sec @pop=2^20 Rosenbrock-1000D (C3), 1-8 GPU; % HBM peak",
    "c2": "individual-generations/sec @pop=2^20 OneMax-4096 packed bits (C2); % HBM peak",
}


def load_traffic(config):
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            ent = json.load(f).get(config)
        return ent["bytes_per_launch"] if ent else None
    except (OSError, ValueError, KeyError, TypeError):
        return None


def main():
    args = parse()
    if args.config == "c5":
        return bench_nsga2(args)
    if args.config == "c5x":
        return bench_nsga2_example(args)
    import ctypes
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    from deap_amd import _lib, algorithms, base, benchmarks, tools
    from deap_amd.ops import RandomStream

    problem, gtype, dim, cx, mut, weights, bpi = CONFIGS[args.config]
    n = args.pop
    if args.islands:
        if args.islands % world:
            raise SystemExit("--islands must be a multiple of the GPU count")
        per, scaling = args.islands // world, "strong"
    else:
        per, scaling = args.islands_per_gpu, "weak"
    n_demes = per * world
    ids = list(range(rank * per, (rank + 1) * per))
    low, high = {"rastrigin": (-5.12, 5.12), "rosenbrock": (-2.048, 2.048),
                 "onemax": (0, 1)}[problem]
    streams = [RandomStream(args.seed, island=d) for d in ids]
    pops = [tools.initPopulation(n=n, dim=dim, low=low, high=high, gtype=gtype, weights=weights,
                                 device=device, stream=s) for s in streams]
    tb = base.Toolbox()
    tb.register("evaluate", getattr(benchmarks, problem))
    tb.register("select", tools.selTournament, tournsize=3)
    if cx == "blend":
        tb.register("mate", tools.cxBlend, alpha=0.5)
    else:
        tb.register("mate", tools.cxTwoPoint)
    if mut == "gaussian":
        tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
    else:
        tb.register("mutate", tools.mutFlipBit, indpb=0.05)
    cxpb, mutpb = 0.5, 0.2
    for p in pops:
        getattr(benchmarks, problem)(p)  # generation 0: evaluate everyone
    steps = [algorithms.GenerationStep(p, tb, cxpb, mutpb) for p in pops]
    offs = [p.like(n, capacity=n) for p in pops]
    total_gens = args.warmup + args.steps + 1
    nevals = torch.zeros((per, total_gens), dtype=torch.int64, device=device)
    mig_events = []

    def migrate(timed):
        from deap_amd.islands import migRingDistributed
        a = b = None
        if timed:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
        if world == 1:
            tools.migRing(pops, args.mig_k, tools.selBest, stream=streams[0])
        else:
            migRingDistributed(pops, ids, n_demes, args.mig_k, tools.selBest, stream=streams[0])
        if timed:
            b.record()
            mig_events.append((a, b))

    def one_gen(g, timed):
        for i in range(per):
            steps[i].step(pops[i], offs[i], streams[i],
                          ctypes.c_void_p(nevals[i].data_ptr() + 8 * g))
            pops[i].swap_storage(offs[i])
        if n_demes > 1 and (g + 1) % args.mig_every == 0:
            migrate(timed)

    for g in range(args.warmup):
        one_gen(g, False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP event pairs recorded by the library itself around every generation
    # kernel launch (gen_pipe_kernel / gen_bits_burst_kernel), on the stream
    # it is launched on
    ctx = pops[0].ctx.bind()
    launches = args.steps * per
    _lib.call("dm_ctx_set_timing", ctx, launches)
    t0 = time.perf_counter()
    for s in range(args.steps):
        one_gen(args.warmup + s, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    times = (ctypes.c_float * launches)()
    cnt = ctypes.c_int32(0)
    _lib.call("dm_ctx_kernel_times", ctx, times, launches, ctypes.byref(cnt))
    _lib.call("dm_ctx_set_timing", ctx, 0)
    assert cnt.value == launches, "expected one generation kernel per deme and step, got %d" % cnt.value
    kern_ms = sum(times) / launches
    mig_ms = (sum(a.elapsed_time(b) for a, b in mig_events) / len(mig_events)
              if mig_events else 0.0)
    if world > 1:
        t = torch.tensor([kern_ms, mig_ms], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        kern_ms, mig_ms = (float(x) for x in t.tolist())
    nev = nevals.cpu().tolist()
    # sanity: the populations stay valid and finite
    for p in pops:
        assert bool(p.valid[:n].bool().all()), "invalid fitness left after a generation"
        assert bool(torch.isfinite(p.wvalues[:n]).all()), "non-finite fitness"

    total = n * args.steps * n_demes
    value = total / elapsed
    achieved = (n * bpi) / (kern_ms * 1e-3) / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": load_traffic(args.config),
                "kernel": "gen_bits_fused_kernel" if gtype == "bits" else "gen_pipe_kernel",
                "kernel_ms": round(kern_ms, 4), "bytes_per_ind_gen": bpi}
    workload = {"c3": "C3 Rastrigin-1000D fp64 eaSimple",
                "c3r": "C3 Rosenbrock-1000D fp64 eaSimple",
                "c2": "C2 OneMax-4096 packed-bit eaSimple"}[args.config]
    if n_demes > 1:
        workload = ("C4 %d islands x %d (%s) with migRing k=%d selBest every %d gens"
                    % (n_demes, n, workload.split(" ", 1)[1], args.mig_k, args.mig_every))
    out = {"metric": METRICS[args.config],
           "value": round(value, 1), "unit": "individual-generations/sec", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
           "scaling": scaling, "vs_baseline": None,
           "dtype": {"f64": "f64", "f32": "f32", "bits": "u64"}[gtype], "data": "synthetic",
           "config": {"workload": workload, "pop_per_island": n, "islands": n_demes,
                      "islands_per_gpu": per, "genes": dim,
                      "operators": "selTournament(t=3) cx%s mut%s cxpb=0.5 mutpb=0.2 indpb=0.05"
                                   % (cx.capitalize(), mut.capitalize()),
                      "parallelism": "islands%d" % n_demes},
           "roofline": roofline,
           "nevals_mean": round(sum(sum(r[args.warmup:args.warmup + args.steps]) for r in nev)
                                / (args.steps * per), 1)}
    if n_demes > 1:
        out["migration"] = {"ms_per_migration": round(mig_ms, 4), "every": args.mig_every,
                            "k": args.mig_k,
                            "frac_of_time": round(mig_ms * len(mig_events) / (elapsed * 1e3), 5)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(problem, args.cpu_sample)
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline_nsga2(wv2, weights, pop, with_log=True):
    """C5 CPU baseline: the DEAP-faithful
    selNSGA2 port (oracle/deap_port.py, reference outputs on
    tests/golden/nsga2*.npz, speed within +-20 % of the reference in
    tests/golden/port_nsga2_calibration.json) on host individuals.
    nd='standard' is O(M N^2) Python: timed on random subsets of the 2N
    fitnesses at 512 / 1,024 / 2,048 and extrapolated to 2N with the fitted
    power law (declared); nd='log' (DEAP's fastest ranks) is timed at the full
    2N.  One core (DEAP's selection is serial).  The variation/evaluation of a
    generation costs seconds on the CPU against hours of selection and is left
    out."""
    import numpy as np
    from oracle import deap_port
    rng = np.random.default_rng(7)
    n2 = len(wv2)
    pts = []
    for n in (512, 1024, 2048):
        rows = rng.choice(n2, n, replace=False)
        pts.append((n, deap_port.time_sel_nsga2(wv2[rows], weights, n // 2, "standard")))
    slope = float(np.polyfit(np.log([p[0] for p in pts]), np.log([p[1] for p in pts]), 1)[0])
    t_std = pts[-1][1] * (n2 / pts[-1][0]) ** slope
    out = {"value": round(pop / t_std, 4), "unit": "individual-generations/sec", "cores": 1,
           "kind": "port", "cpu_model": cpu_model(),
           "sample": "selNSGA2(2N -> N, nd='standard') of the port at 2N = 512/1024/2048 "
                     "(%.2f/%.2f/%.2f s), extrapolated to 2N = %d with the fitted law N^%.2f: "
                     "%.0f s per generation (declared extrapolation)"
                     % (pts[0][1], pts[1][1], pts[2][1], n2, slope, t_std),
           "law_exponent": round(slope, 3), "standard_s_per_gen": round(t_std, 1)}
    if with_log:
        t_log = deap_port.time_sel_nsga2(wv2, weights, n2 // 2, "log")
        out["log"] = {"value": round(pop / t_log, 1), "seconds": round(t_log, 2),
                      "sample": "selNSGA2(2N -> N, nd='log') of the port timed at the full "
                                "2N = %d" % n2}
    return out


def bench_nsga2(args):
    """Config C5: NSGA-II on DTLZ2, M=3, D=12 fp64, pop 2^17.
    A step is one eaMuPlusLambda generation (deap/algorithms.py:316-329): varOr
    of lambda = N offspring (cxBlend / mutGaussian) with the invalid ones
    evaluated, then selNSGA2(parents + offspring = 2N -> N) and the gather of
    the chosen rows.  The dominant stage is the all-pairs dominance pass of
    sortNondominated, VALU-bound: roofline = pairwise fitness comparisons per
    second (M compares per ordered pair, U(U-1) ordered pairs of unique fits)
    against the fp64 VALU compare rate (256 CU x 4 SIMD x 16 lanes x 2.4 GHz).
    Replicas only at N > 1 (no exchange)."""
    import torch
    from deap_amd import algorithms, base, benchmarks, tools
    from deap_amd.ops import RandomStream
    device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(device)
    n = args.pop if args.pop != 1 << 20 else 1 << 17
    m, dim = 3, 12
    stream = RandomStream(args.seed)
    pop = tools.initPopulation(n=n, dim=dim, low=0.0, high=1.0, gtype="f64",
                               weights=(-1.0,) * m, device=device, stream=stream)
    tb = base.Toolbox()
    tb.register("evaluate", benchmarks.dtlz2, obj=m)
    tb.register("mate", tools.cxBlend, alpha=0.5)
    tb.register("mutate", tools.mutGaussian, mu=0, sigma=0.1, indpb=1.0 / dim)
    tb.register("select", tools.selNSGA2)
    benchmarks.dtlz2(pop, obj=m)
    step = algorithms.MuPlusLambdaStep(pop, tb, n, n, 0.6, 0.3)
    for _ in range(args.warmup):
        step.step(stream)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.steps)]
    t0 = time.perf_counter()
    for s in range(args.steps):
        ev[2 * s].record()
        step.step(stream)
        ev[2 * s + 1].record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    gen_ms = sum(ev[2 * s].elapsed_time(ev[2 * s + 1]) for s in range(args.steps)) / args.steps
    # stage breakdown outside the timed region: selNSGA2 alone on 2N rows
    # (current parents + one varOr batch of offspring)
    comb = step.combined
    sel_ms = []
    two = pop.like(2 * n, capacity=2 * n)
    from deap_amd import _lib
    import ctypes
    _lib.call("dm_gather", comb.ctx.bind(), ctypes.byref(comb.c_pop()), None,
              ctypes.byref(two.c_pop(0, n)))
    off = algorithms.varOr(comb, tb, n, 0.6, 0.3, evaluate=True, stream=stream)
    _lib.call("dm_gather", comb.ctx.bind(), ctypes.byref(off.c_pop()), None,
              ctypes.byref(two.c_pop(n, n)))
    for _ in range(4):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        idx = tools.selNSGA2(two, n)
        b.record()
        torch.cuda.synchronize()
        sel_ms.append(a.elapsed_time(b))
    sel_ms = sorted(sel_ms[1:])[1]
    fronts = tools.sortNondominated(two, 2 * n)
    wv = two.wvalues[:2 * n]
    uniq = int(torch.unique(wv, dim=0).shape[0])
    cmp_per_sel = float(m) * uniq * (uniq - 1)
    valu_peak = 256 * 4 * 16 * 2.4e9 / 1e9  # Gop/s of fp64 compares
    achieved = cmp_per_sel / (sel_ms * 1e-3) / 1e9
    out = {"metric": "individual-generations/sec @pop=2^17 DTLZ2 NSGA-II (C5)",
           "value": round(n * args.steps / elapsed, 1), "unit": "individual-generations/sec",
           "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": "C5 NSGA-II DTLZ2 M=3 D=12 eaMuPlusLambda(mu=lambda=N) + "
                                  "selNSGA2(2N->N)", "pop": n, "genes": dim, "objectives": m,
                      "operators": "varOr cxBlend(0.5) mutGaussian(0,0.1,1/D) cxpb=0.6 mutpb=0.3",
                      "parallelism": "replicas1"},
           "gen_ms_events": round(gen_ms, 4),
           "roofline": {"bound": "valu", "achieved": round(achieved, 1), "peak": valu_peak,
                        "unit": "Gcompare/s", "frac": round(achieved / valu_peak, 4),
                        "traffic": None, "kernel": "selNSGA2 (dom_build + peel + crowding)",
                        "kernel_ms": round(sel_ms, 4), "unique_fits": uniq,
                        "fronts": len(fronts)},
           "cpu_baseline": None}
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_nsga2(wv.cpu().numpy(), (-1.0,) * m, n)
    print(json.dumps(out), flush=True)


def bench_nsga2_example(args):
    """DEAP's canonical NSGA-II loop (examples/ga/nsga2.py:94-114) on DTLZ2,
    M=3, D=12 fp64, pop 2^17.  A step is one generation: selTournamentDCD(pop, N)
    -> clone + cxSimulatedBinaryBounded(eta 20, cxpb 0.9) + mutPolynomialBounded
    (eta 20, indpb 1/D) (varBounded, one launch) -> evaluate the offspring ->
    selNSGA2(pop + offspring, N) and the gather of the chosen rows (crowding
    distances carried).  The bounded-variation kernel is reported against HBM:
    algorithmic bytes = 2 parent rows in + 2 child rows out per pair (D*8 B
    each) + idx/wvalues/valid; selNSGA2 dominates the generation."""
    import ctypes
    import torch
    from deap_amd import _lib, algorithms, base, benchmarks, tools
    from deap_amd.ops import RandomStream
    device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(device)
    n = args.pop if args.pop != 1 << 20 else 1 << 17
    m, dim = 3, 12
    stream = RandomStream(args.seed)
    pop = tools.initPopulation(n=n, dim=dim, low=0.0, high=1.0, gtype="f64",
                               weights=(-1.0,) * m, device=device, stream=stream)
    tb = base.Toolbox()
    tb.register("mate", tools.cxSimulatedBinaryBounded, low=0.0, up=1.0, eta=20.0)
    tb.register("mutate", tools.mutPolynomialBounded, low=0.0, up=1.0, eta=20.0,
                indpb=1.0 / dim)
    benchmarks.dtlz2(pop, obj=m)
    two = pop.like(2 * n, capacity=2 * n)
    ctx = pop.ctx.bind()

    def select_into(pop, off):
        # pop[:] = toolbox.select(pop + offspring, MU)                 (nsga2.py:114)
        _lib.call("dm_gather", ctx, ctypes.byref(pop.c_pop()), None, ctypes.byref(two.c_pop(0, n)))
        _lib.call("dm_gather", ctx, ctypes.byref(off.c_pop()), None, ctypes.byref(two.c_pop(n, n)))
        idx = tools.selNSGA2(two, n)
        _lib.call("dm_gather", ctx, ctypes.byref(two.c_pop()), ctypes.c_void_p(idx.data_ptr()),
                  ctypes.byref(pop.c_pop()))
        pop.crowding_dist = two.crowding_dist[idx.long()].contiguous()

    # pop = toolbox.select(pop, len(pop)): assigns the crowding distances (nsga2.py:92)
    idx0 = tools.selNSGA2(pop, n)
    pop.crowding_dist = pop.crowding_dist[idx0.long()].contiguous()
    _lib.call("dm_gather", ctx, ctypes.byref(pop.c_pop()), ctypes.c_void_p(idx0.data_ptr()),
              ctypes.byref(two.c_pop(0, n)))
    _lib.call("dm_gather", ctx, ctypes.byref(two.c_pop(0, n)), None, ctypes.byref(pop.c_pop()))
    var_ms = []

    def one_gen(record):
        sel = tools.selTournamentDCD(pop, n, stream=stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        off = algorithms.varBounded(pop, tb, 0.9, sel, stream=stream)
        b.record()
        benchmarks.dtlz2(off, obj=m)
        select_into(pop, off)
        if record:
            var_ms.append((a, b))

    for _ in range(args.warmup):
        one_gen(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_gen(True)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    vms = sorted(a.elapsed_time(b) for a, b in var_ms)
    v_ms = sum(vms) / len(vms)
    var_bytes = (n // 2) * (4 * dim * 8) + n * (4 + 2 * m * 8 + 2)
    achieved = var_bytes / (v_ms * 1e-3) / 1e9
    out = {"metric": "individual-generations/sec @pop=2^17 DTLZ2 NSGA-II example loop (C5x)",
           "value": round(n * args.steps / elapsed, 1), "unit": "individual-generations/sec",
           "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": "C5x examples/ga/nsga2.py loop: selTournamentDCD + "
                                  "cxSimulatedBinaryBounded + mutPolynomialBounded + "
                                  "selNSGA2(2N->N)", "pop": n, "genes": dim, "objectives": m,
                      "parallelism": "replicas1"},
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": 8000.0,
                        "unit": "GB/s", "frac": round(achieved / 8000.0, 4), "traffic": None,
                        "kernel": "bounded_vary_kernel (varBounded)",
                        "kernel_ms": round(v_ms, 5)},
           "cpu_baseline": None}
    if not args.no_cpu_baseline:
        # the loop's CPU cost is its selNSGA2 (selTournamentDCD and the bounded
        # operators of 2^17 individuals take seconds): the C5 baseline applies
        out["cpu_baseline"] = cpu_baseline_nsga2(two.wvalues[:2 * n].cpu().numpy(), (-1.0,) * m,
                                                 n, with_log=False)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
