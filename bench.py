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
    # genome shapes beside the benched ones (VERDICT r5 "missing 3"): measured
    # with --no-cpu-baseline; B = 2G + (t+1)F with F = 8 B per objective
    "c3d30": ("rastrigin", "f64", 30, "blend", "gaussian", (-1.0,), 2 * 240 + 4 * 8),
    "c3d2000": ("rastrigin", "f64", 2000, "blend", "gaussian", (-1.0,), 2 * 16000 + 4 * 8),
    "c3f32": ("rastrigin", "f32", 1000, "blend", "gaussian", (-1.0,), 2 * 4000 + 4 * 8),
    "c2b8192": ("onemax", "bits", 8192, "twopoint", "flipbit", (1.0,), 2 * 1024 + 4 * 8),
    "zdt1": ("zdt1", "f64", 30, "twopoint", "gaussian", (-1.0, -1.0), 2 * 240 + 4 * 16),
}
HBM_PEAK_GBS = 8000.0


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment bench.py "
                         "starts torch.distributed.run with this many ranks itself")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (gloo: CPU launcher test only)")
    ap.add_argument("--dry-run", action="store_true",
                    help="N > 1 launcher check without a GPU: rendezvous, deme ownership and "
                         "the migRing hop plan of every rank, no kernels")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--warmup-secs", type=float, default=1.0,
                    help="after the --warmup steps, keep warming up (untimed) until this much "
                         "wall time has passed: the GPU's clocks reach steady state (C2 ran "
                         "0.24 ms per step after 5 steps, 0.214 after 200).  The extra "
                         "generations recompute the next generation from the same state and "
                         "discard it, so the populations (and deme_digests) do not depend on "
                         "how many there were")
    ap.add_argument("--digests-out", default=None,
                    help="append this run's deme digests to a JSON reference file "
                         "(profiles/deme_digests.json is the committed one)")
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
    ap.add_argument("--nobj", type=int, default=3,
                    help="C5: DTLZ2 objectives (3 = the benched config; 4 takes the compare "
                         "kernel + D-matrix peel)")
    return ap.parse_args(argv)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """``--gpus N`` (N > 1) started as a plain ``python bench.py``: run
    ``torch.distributed.run`` with N ranks as a CHILD process (nothing here
    imports torch or touches a GPU, and nothing execs), relay its output line
    by line (progress reaches the caller while the ranks run), check that
    rank 0's JSON line reports ``n_gpus == N`` and exit with the children's
    status.  The same command therefore measures 1, 2, 4 or 8 GPUs."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    result = None
    for line in proc.stdout:
        s = line.strip()
        if s.startswith("{") and '"metric"' in s:
            result = s
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = proc.wait()
    if rc != 0:
        sys.stderr.write("bench.py: torch.distributed.run with %d ranks failed (exit %d)\n"
                         % (n, rc))
        return rc or 1
    if result is None:
        sys.stderr.write("bench.py: rank 0 printed no result line\n")
        return 1
    got = json.loads(result).get("n_gpus")
    if got != n:
        sys.stderr.write("bench.py: expected n_gpus == %d in the result, got %r\n" % (n, got))
        return 1
    print(result, flush=True)
    return 0


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cgroup_cpu_quota():
    """CPUs granted by the cgroup (v2 ``cpu.max`` "quota period", v1
    ``cpu.cfs_quota_us`` / ``cpu.cfs_period_us``), or None when unlimited or
    unreadable."""
    import math
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            return max(1, math.ceil(int(q) / int(p)))
        return None
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        return max(1, math.ceil(q / p)) if q > 0 else None
    except (OSError, ValueError):
        return None


def host_workers():
    """Worker processes for the CPU baseline = every core this process is
    granted: the CPUs it may run on (sched_getaffinity), limited by the cgroup
    CPU quota when one is set; with no quota, by the per-job thread grant the
    environment states (OMP_NUM_THREADS — the GPU box sets it to its 16-CPU
    share per GPU, while os.cpu_count() there reports the whole machine).
    Returns (workers, detail)."""
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:
        visible = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    env = os.environ.get("DM_CPU_WORKERS") or os.environ.get("OMP_NUM_THREADS")
    if quota is not None:
        workers, source = min(visible, quota), "cgroup cpu quota"
    elif env and env.isdigit() and int(env) > 0:
        workers, source = min(visible, int(env)), ("DM_CPU_WORKERS" if os.environ.get(
            "DM_CPU_WORKERS") else "OMP_NUM_THREADS (per-job CPU grant)")
    else:
        workers, source = visible, "sched_getaffinity"
    return max(1, workers), {"cpus_visible": visible, "cgroup_quota": quota,
                             "cores_source": source}


def cpu_baseline(problem, sample):
    from oracle import deap_port
    workers, detail = host_workers()
    dim = CONFIGS_DIM[problem]
    rate, secs, used = deap_port.run(problem, n=sample, dim=dim, ngen=2, workers=workers)
    return {"value": rate, "unit": "individual-generations/sec", "cores": used, "kind": "port",
            "cpu_model": cpu_model(), **detail,
            "sample": "DEAP-faithful eaSimple (oracle/deap_port.py, bit-exact with the reference on "
                      "tests/golden/port.npz: array genomes, deepcopy clone, Pool(%d).map "
                      "evaluate), pop %d x %d genes, 2 timed generations (%.1f s)"
                      % (used, sample, dim, secs)}


CONFIGS_DIM = {"rastrigin": 1000, "rosenbrock": 1000, "onemax": 4096}
METRICS = {
    "c3": "individual-generations/sec @pop=2^20 Rastrigin-1000D, 1-8 GPU; % HBM peak",
    "c3r": "individual-generations/sec @pop=2^20 Rosenbrock-1000D (C3), 1-8 GPU; % HBM peak",
    "c2": "individual-generations/sec @pop=2^20 OneMax-4096 packed bits (C2); % HBM peak",
    "c3d30": "individual-generations/sec @pop=2^20 Rastrigin-30D fp64; % HBM peak",
    "c3d2000": "individual-generations/sec @pop=2^20 Rastrigin-2000D fp64; % HBM peak",
    "c3f32": "individual-generations/sec @pop=2^20 Rastrigin-1000D fp32; % HBM peak",
    "c2b8192": "individual-generations/sec @pop=2^20 OneMax-8192 packed bits; % HBM peak",
    "zdt1": "individual-generations/sec @pop=2^20 ZDT1-30D fp64 (2 objectives); % HBM peak",
}


def hot_kernel_name(gtype, dim, nobj):
    """The generation kernel the library launches for this shape
    (generation.hip launch_generation's dispatch, native RNG, selTournament)."""
    if gtype == "bits":
        return "gen_bits_fused_kernel" if (dim + 63) // 64 <= 64 and nobj == 1 else "gen_bits_kernel"
    return "gen_pipe_kernel" if 64 < dim <= 1024 and nobj == 1 else "gen_float_kernel"


def load_traffic(config):
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            ent = json.load(f).get(config)
        return ent["bytes_per_launch"] if ent else None
    except (OSError, ValueError, KeyError, TypeError):
        return None


def deme_split(args, world, rank):
    """Demes per rank: ``--islands I`` splits I demes evenly over the ranks
    (strong scaling, C4 literally), otherwise ``--islands-per-gpu`` demes per
    rank (weak scaling; the default N-GPU run is one 2^20 island per GPU)."""
    if args.islands:
        if args.islands % world:
            raise SystemExit("--islands must be a multiple of the GPU count")
        per, scaling = args.islands // world, "strong"
    else:
        per, scaling = args.islands_per_gpu, "weak"
    return per, scaling, per * world, list(range(rank * per, (rank + 1) * per))


def dry_run(args, world, rank):
    """Launcher / distributed-setup check without a GPU (``--dry-run``, used
    by tests/test_bench_launcher.py over gloo): every rank joins the process
    group, agrees on the deme owners (islands.owner_map, the all_gather the
    real run does) and computes its migRing hops with the C ABI's planner
    (``dm_mig_plan``, host-only); rank 0 prints them in the bench line."""
    import torch.distributed as dist
    from deap_amd import islands
    if world > 1:
        dist.init_process_group(args.backend)
    per, scaling, n_demes, ids = deme_split(args, world, rank)
    owner = islands.owner_map(ids, n_demes, world, None)
    plan = islands.mig_plan(n_demes, None, owner, rank)
    plans = [None] * world
    if world > 1:
        dist.all_gather_object(plans, plan)
    else:
        plans = [plan]
    if rank == 0:
        print(json.dumps({"metric": METRICS[args.config], "value": None, "n_gpus": world,
                          "dry_run": True, "scaling": scaling, "islands": n_demes,
                          "owner": [owner[d] for d in range(n_demes)], "hops": plans}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            return launch_ranks(args.gpus, argv)
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%s" % (args.gpus,
                                                                    os.environ["WORLD_SIZE"]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    if args.config == "c5":
        return bench_nsga2(args, world, rank, local)
    if args.config == "c5x":
        return bench_nsga2_example(args, world, rank, local)
    import ctypes
    import torch
    import torch.distributed as dist

    device = rank_device(args, local)
    torch.cuda.set_device(device)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(args.backend, device_id=device if args.backend == "nccl" else None)

    from deap_amd import _lib, algorithms, base, benchmarks, tools
    from deap_amd.ops import RandomStream

    problem, gtype, dim, cx, mut, weights, bpi = CONFIGS[args.config]
    n = args.pop
    per, scaling, n_demes, ids = deme_split(args, world, rank)
    low, high = {"rastrigin": (-5.12, 5.12), "rosenbrock": (-2.048, 2.048),
                 "onemax": (0, 1), "zdt1": (0.0, 1.0)}[problem]
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
        # ZDT1 is defined on [0, 1]: a small sigma keeps most genes there
        tb.register("mutate", tools.mutGaussian, mu=0,
                    sigma=0.01 if problem == "zdt1" else 1.0, indpb=0.05)
    else:
        tb.register("mutate", tools.mutFlipBit, indpb=0.05)
    cxpb, mutpb = 0.5, 0.2
    for p in pops:
        getattr(benchmarks, problem)(p)  # generation 0: evaluate everyone
    steps = [algorithms.GenerationStep(p, tb, cxpb, mutpb) for p in pops]
    offs = [p.like(n, capacity=n) for p in pops]
    total_gens = args.warmup + args.steps + 2  # + a scratch slot for the warm-up top-up
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

    def rerun_next():
        # generation `warmup` computed from the current parents and stream
        # state and discarded (the state restored): the populations after
        # the timed steps do not depend on how many of these ran
        for i in range(per):
            state = streams[i].getstate()
            steps[i].step(pops[i], offs[i], streams[i],
                          ctypes.c_void_p(nevals[i].data_ptr() + 8 * (total_gens - 1)))
            streams[i].setstate(state)
    extra_warm = warm_until(args, rerun_next)
    if n_demes > 1:
        # one untimed migration: the RCCL communicator (ncclCommInitRank), the
        # peers' point-to-point connections and the migration scratch are set
        # up here, not inside the timed steps
        migrate(False)
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
        elapsed = max_over_ranks([elapsed], device)[0]
    times = (ctypes.c_float * launches)()
    cnt = ctypes.c_int32(0)
    _lib.call("dm_ctx_kernel_times", ctx, times, launches, ctypes.byref(cnt))
    _lib.call("dm_ctx_set_timing", ctx, 0)
    assert cnt.value == launches, "expected one generation kernel per deme and step, got %d" % cnt.value
    kern_ms = sum(times) / launches
    mig_ms = (sum(a.elapsed_time(b) for a, b in mig_events) / len(mig_events)
              if mig_events else 0.0)
    if world > 1:
        kern_ms, mig_ms = max_over_ranks([kern_ms, mig_ms], device)
    nev = nevals.cpu().tolist()
    # sanity: the populations stay valid and finite
    for p in pops:
        assert bool(p.valid[:n].bool().all()), "invalid fitness left after a generation"
        # ZDT1's sqrt(f1 / g) is NaN for a gene mutated below 0 (the reference
        # raises there); the shape run measures throughput only
        assert problem == "zdt1" or bool(torch.isfinite(p.wvalues[:n]).all()), "non-finite fitness"
    # correctness fingerprint of every deme after the last step (outside the
    # timed region): the Philox streams are keyed by the deme id and the
    # migration is exact, so a deme's digest depends only on (seed, deme id,
    # islands, steps, migration schedule), never on how the demes are spread
    # over ranks -- runs of the same --islands on 1, 2, 4 or 8 GPUs must print
    # the same digests (tests/test_gpu_islands_mp.py checks the rows themselves)
    digests = {d: deme_digest(p, n) for d, p in zip(ids, pops)}
    if world > 1:
        parts = [None] * world
        dist.all_gather_object(parts, digests)
        digests = {d: h for part in parts for d, h in part.items()}

    total = n * args.steps * n_demes
    value = total / elapsed
    achieved = (n * bpi) / (kern_ms * 1e-3) / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": load_traffic(args.config),
                "kernel": hot_kernel_name(gtype, dim, len(weights)),
                "kernel_ms": round(kern_ms, 4), "bytes_per_ind_gen": bpi}
    workload = {"c3": "C3 Rastrigin-1000D fp64 eaSimple",
                "c3r": "C3 Rosenbrock-1000D fp64 eaSimple",
                "c2": "C2 OneMax-4096 packed-bit eaSimple",
                "c3d30": "shape Rastrigin-30D fp64 eaSimple",
                "c3d2000": "shape Rastrigin-2000D fp64 eaSimple",
                "c3f32": "shape Rastrigin-1000D fp32 eaSimple",
                "c2b8192": "shape OneMax-8192 packed-bit eaSimple",
                "zdt1": "shape ZDT1-30D fp64 (M=2) eaSimple"}[args.config]
    if n_demes > 1:
        workload = ("C4 %d islands x %d (%s) with migRing k=%d selBest every %d gens"
                    % (n_demes, n, workload.split(" ", 1)[1], args.mig_k, args.mig_every))
    out = {"metric": METRICS[args.config],
           "value": round(value, 1), "unit": "individual-generations/sec", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup,
           "warmup_topup": {"secs": args.warmup_secs, "generations": extra_warm},
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
    out["deme_digests"] = {"after_generation": args.warmup + args.steps, "seed": args.seed,
                           "islands": n_demes,
                           "digest": {str(d): digests[d] for d in sorted(digests)}}
    key = digest_key(args, n, n_demes)
    check = check_digests(key, out["deme_digests"]["digest"])
    out["deme_digests"].update(key=key, check=check)
    if rank == 0 and args.digests_out:
        save_digests(args.digests_out, key, out["deme_digests"]["digest"])
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config in ("c3", "c3r", "c2"):
        out["cpu_baseline"] = cpu_baseline(problem, args.cpu_sample)
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        from deap_amd import islands
        islands.close_comms()
        dist.destroy_process_group()
    if check == "mismatch":
        sys.stderr.write("bench.py: deme digests differ from the one-GPU reference %s (%s)\n"
                         % (DIGESTS, key))
        return 3


DIGESTS = os.path.join(ROOT, "profiles", "deme_digests.json")


def digest_key(args, n, n_demes):
    """Everything a deme's digest depends on: the config, the
    deme size and count, the seed, the generations and the migration
    schedule -- not the GPU count or the deme split."""
    return ("config=%s pop=%d islands=%d seed=%d warmup=%d steps=%d mig_every=%d mig_k=%d"
            % (args.config, n, n_demes, args.seed, args.warmup, args.steps, args.mig_every,
               args.mig_k))


def check_digests(key, digest):
    """'match' / 'mismatch' against the committed one-GPU reference
    (profiles/deme_digests.json, written by --digests-out runs on one GPU),
    or 'no reference' for a configuration it does not hold."""
    try:
        with open(DIGESTS) as f:
            ref = json.load(f).get(key)
    except (OSError, ValueError):
        ref = None
    if ref is None:
        return "no reference"
    return "match" if ref == digest else "mismatch"


def save_digests(path, key, digest):
    try:
        with open(path) as f:
            table = json.load(f)
    except (OSError, ValueError):
        table = {}
    table[key] = digest
    with open(path, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
        f.write("\n")


def deme_digest(pop, n):
    """64-bit fingerprint of a deme (test infrastructure for the scaling runs):
    a wrapping multiply-add of every genome word (fixed odd multipliers per
    word position and per row) plus the bits of every wvalue and valid byte,
    computed on the device in slices of rows."""
    import numpy as np
    import torch
    g = pop.genes[:n].view(torch.int64)
    rng = np.random.default_rng(20261017)
    mw = torch.from_numpy(rng.integers(1, 2**62, size=g.shape[1], dtype=np.int64) | 1).to(g.device)
    acc = torch.zeros((), dtype=torch.int64, device=g.device)
    for a in range(0, n, 1 << 16):
        b = min(n, a + (1 << 16))
        rows = (g[a:b] * mw).sum(dim=1)
        mr = torch.arange(a + 1, b + 1, dtype=torch.int64, device=g.device) * (0x9E3779B97F4A7C15 - 2**64)
        acc += (rows * (mr | 1)).sum()
    w = pop.wvalues[:n].contiguous().view(torch.int64)
    acc += (w * 0x632BE59BD9B4E019).sum() + pop.valid[:n].to(torch.int64).sum()
    return "%016x" % (int(acc.item()) & (2**64 - 1))


def cpu_baseline_nsga2(wv2, weights, pop, with_log=True):
    """C5 CPU baseline: the DEAP-faithful
    selNSGA2 port (oracle/deap_port.py, reference outputs on
    tests/golden/nsga2*.npz, speed within +-20 % of the reference in
    tests/golden/port_nsga2_calibration.json) on host individuals.
    nd='standard' is O(M N^2) Python: timed on random subsets of the 2N
    fitnesses at 1,024 / 2,048 / 4,096 / 8,192 and extrapolated to 2N with the
    power law fitted on them (declared); nd='log' (DEAP's fastest ranks) is timed at the full
    2N.  One core (DEAP's selection is serial).  The variation/evaluation of a
    generation costs seconds on the CPU against hours of selection and is left
    out."""
    import numpy as np
    from oracle import deap_port
    rng = np.random.default_rng(7)
    n2 = len(wv2)
    pts = []
    for n in (1024, 2048, 4096, 8192):
        rows = rng.choice(n2, n, replace=False)
        pts.append((n, deap_port.time_sel_nsga2(wv2[rows], weights, n // 2, "standard")))
    slope = float(np.polyfit(np.log([p[0] for p in pts]), np.log([p[1] for p in pts]), 1)[0])
    t_std = pts[-1][1] * (n2 / pts[-1][0]) ** slope
    out = {"value": round(pop / t_std, 4), "unit": "individual-generations/sec", "cores": 1,
           "kind": "port", "cpu_model": cpu_model(),
           "sample": "selNSGA2(2N -> N, nd='standard') of the port at 2N = "
                     "1024/2048/4096/8192 (%s s), extrapolated to 2N = %d with the law N^%.2f "
                     "fitted on those points: %.0f s per generation (declared extrapolation)"
                     % ("/".join("%.2f" % p[1] for p in pts), n2, slope, t_std),
           "law_exponent": round(slope, 3), "standard_s_per_gen": round(t_std, 1)}
    if with_log:
        t_log = deap_port.time_sel_nsga2(wv2, weights, n2 // 2, "log")
        out["log"] = {"value": round(pop / t_log, 1), "seconds": round(t_log, 2),
                      "sample": "selNSGA2(2N -> N, nd='log') of the port timed at the full "
                                "2N = %d" % n2}
    return out


VALU_PEAK_GINSTR = 256 * 4 * 2.4e9 / 2 / 1e9  # wave64 VALU instructions/s: SIMD-32, 2 clk each


def peel_work(wv, fronts, peel_us):
    """The peel's algorithmic work per front: a member u
    of front r is compared with every v of each 512-v chunk of the q order
    (unique fits, ascending objective 0) up to the chunk holding the last fit
    tied with u in objective 0 -- the only v it can dominate -- so front r
    costs sum_u reach(u) member-chunk pairs (512 dominance bits each).
    Reported as pairs per microsecond of the front's peel launch, next to the
    VALU-issue fraction (which counts instructions, not work)."""
    import numpy as np
    ufit, inv = np.unique(wv + 0.0, axis=0, return_inverse=True)
    inv = np.asarray(inv).ravel()
    w0 = np.sort(ufit[:, 0])
    # last position (ascending objective 0) tied with each unique fit
    tie_end = np.searchsorted(w0, ufit[:, 0], side="right") - 1
    reach = tie_end // 512 + 1
    rows = []
    for i, f in enumerate(fronts):
        if i >= len(peel_us):
            break
        members = np.unique(inv[f.cpu().numpy()])
        pairs = int(reach[members].sum())
        rows.append((len(members), pairs, peel_us[i]))
    tot_pairs = sum(r[1] for r in rows)
    tot_us = sum(r[2] for r in rows)
    return {"unit": "member-chunk pairs per us (512 dominance bits each)",
            "pairs_per_selection": tot_pairs,
            "pairs_per_us": round(tot_pairs / tot_us, 1) if tot_us else None,
            "by_front": [[a, b, round(b / c, 1) if c else None] for a, b, c in rows]}


def peel_report(peel_us, usz, m=3, chain_ms=None):
    """C5's dominant kernel, the table-fed front peel (dominance.hip
    peel_order_kernel): one launch per front; launch i peels front i (usz[i]
    unique fitnesses), releasing front i + 1, and -- in its search workgroups
    -- orders front i; the launches after the last front exit at once.  It is VALU-issue and latency bound (64 x 64 bit
    transposes of the members' rows), so its roofline is VALU
    wave-instructions issued per second against the issue peak (256 CU x 4
    SIMD x 2.4 GHz / 2 clk per wave64 instruction on SIMD-32): the
    instructions per selection come from the PMC pass committed in
    profiles/c5_peel_pmc.json (SQ_INSTS_VALU summed over one selection's peel
    launches), the time from live events: chain_ms, the batches of launches
    each bracketed by ONE event pair (launches plus the ~2 us gaps between
    them; round 6), when given -- the per-launch pairs behind peel_us add ~5
    us to every launch (profiles/r06_c5), so they give the per-front shape
    (floor + slope) but overstate the time."""
    import numpy as np
    nf = len(usz)
    work = [(usz[i], peel_us[i]) for i in range(min(nf, len(peel_us)))]
    ev_ms = sum(peel_us) / 1e3
    tot_ms = chain_ms if chain_ms else ev_ms
    fit = np.polyfit([w[0] for w in work], [w[1] for w in work], 1) if len(work) > 2 else (0, 0)
    fronts = {"launches": len(peel_us), "fronts": nf, "ms_per_selection": round(tot_ms, 4),
              "ms_per_selection_per_launch_events": round(ev_ms, 4),
              "us_per_launch_mean": round(sum(peel_us) / max(1, len(peel_us)), 2),
              "us_floor": round(float(fit[1]), 2), "us_per_1000_members": round(float(fit[0]) * 1e3, 2),
              "by_front": [[int(a), round(b, 1)] for a, b in work]}
    pmc = None
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "c5_peel_pmc.json")
    if os.path.exists(path) and m <= 3:
        with open(path) as f:
            pmc = json.load(f)
    roof = {"bound": "valu-issue", "unit": "Ginstr/s",
            "kernel": "peel_order_kernel<%d>" % (m - 1) if m <= 3 else "peel_owned_kernel",
            "peak": round(VALU_PEAK_GINSTR, 1), "kernel_ms": round(tot_ms, 4),
            "peak_basis": "wave64 VALU instructions: 256 CU x 4 SIMD-32 x 2.4 GHz / 2 clk",
            "traffic": None, "achieved": None, "frac": None}
    if pmc:
        instr = float(pmc["SQ_INSTS_VALU_per_selection"])
        ach = instr / (tot_ms * 1e-3) / 1e9
        roof.update(achieved=round(ach, 1), frac=round(ach / VALU_PEAK_GINSTR, 4),
                    valu_instr_per_selection=instr, pmc_source=pmc.get("source"),
                    wave_cycles_valu_frac=pmc.get("SQ_ACTIVE_INST_VALU_over_SQ_WAVE_CYCLES"))
    return {"roofline": roof, "fronts": fronts}


def rank_device(args, local):
    """One GPU per rank; with the gloo backend (CPU collectives, host-staged
    migration) ranks may share GPUs, local rank r on GPU r mod count -- how
    the one-GPU test boxes run the multi-rank path (RCCL refuses two ranks on
    one device)."""
    import torch
    if args.backend == "gloo":
        local %= max(1, torch.cuda.device_count())
    return torch.device("cuda", local)


def replica_setup(args, world, local):
    """C5 / C5x at N > 1: replicas only (no exchange step), one
    process per GPU; the process group is used for the barrier and the
    max-over-ranks time only."""
    import torch
    import torch.distributed as dist
    device = rank_device(args, local)
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group(args.backend, device_id=device if args.backend == "nccl" else None)
    return device


def replica_barrier(world):
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def replica_max(x, world, device):
    import torch
    import torch.distributed as dist
    if world == 1:
        return x
    return max_over_ranks([x], device)[0]


def max_over_ranks(values, device):
    """Element-wise max of a list of floats over the ranks (a device tensor
    for RCCL, a host one for gloo)."""
    import torch
    import torch.distributed as dist
    on = device if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor(values, dtype=torch.float64, device=on)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def save_state(pops, stream, step=None):
    """Device copies of populations (rows, fitness, validity, crowding) and
    the stream / step counters, for restore_state after an untimed top-up
    that advances them (C5, C5x)."""
    import torch
    copies = []
    for p in pops:
        cd = p.crowding_dist
        copies.append((p, p.n, p.genes.clone(), p.wvalues.clone(), p.valid.clone(),
                       None if cd is None else cd.clone()))
    torch.cuda.synchronize()
    return copies, (stream, stream.getstate()), step, (step.n if step is not None else None)


def restore_state(saved):
    import torch
    copies, (stream, st), step, n = saved
    stream.setstate(st)
    for p, pn, g, w, v, cd in copies:
        p.resize(pn)
        p.genes.copy_(g)
        p.wvalues.copy_(w)
        p.valid.copy_(v)
        if cd is not None:
            if p.crowding_dist is None or p.crowding_dist.shape != cd.shape:
                p.crowding_dist = cd
            else:
                p.crowding_dist.copy_(cd)
    if step is not None:
        step.n = n
    torch.cuda.synchronize()


def warm_until(args, fn):
    """The untimed --warmup-secs top-up: call fn() until that much wall time
    has passed (at least once when --warmup-secs > 0); returns the count."""
    import torch
    count, t0 = 0, time.perf_counter()
    while args.warmup_secs > 0 and (count == 0 or time.perf_counter() - t0 < args.warmup_secs):
        fn()
        count += 1
        if count % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return count


def replica_finish(world):
    import torch.distributed as dist
    if world > 1:
        dist.destroy_process_group()


def bench_nsga2(args, world=1, rank=0, local=0):
    """Config C5: NSGA-II on DTLZ2, M=3, D=12 fp64, pop 2^17.
    A step is one eaMuPlusLambda generation (deap/algorithms.py:316-329): varOr
    of lambda = N offspring (cxBlend / mutGaussian) with the invalid ones
    evaluated, then selNSGA2(parents + offspring = 2N -> N) and the gather of
    the chosen rows.  The all-pairs stage of sortNondominated is the bitset
    count pass (bitdom.hip bd_count_kernel: per (v, 512-u chunk) one binary
    search per objective 1..M-1 over the chunk's sorted ranks and one 64-byte
    prefix-set read per objective, all in LDS), LDS-bound: ``roofline`` is its
    LDS bytes per launch — sum over chunks c of reach_c (the v a chunk can
    dominate) x (M-1) x (11 probes x 4 B + 64 B) — over its average duration
    (HIP events the library records around the launch,
    dm_ctx_set_timing_target(DM_TIME_DOMINANCE)), against 256 CU x 256 B/clk x
    2.4 GHz of LDS reads (MI355X_MICROARCH.md, ds_read_b128).  The §8d count of
    M*U(U-1)/2 pair compares is reported beside it as a rate (a 32-bit AND of
    two prefix sets decides 32 pairs, so it exceeds the 78.6 T/s a
    compare-per-pair kernel could reach); ``selection`` is the whole selNSGA2.
    Replicas only at N > 1 (no exchange)."""
    import ctypes
    import numpy as np
    import torch
    from deap_amd import _lib, algorithms, base, benchmarks, tools
    from deap_amd.ops import RandomStream
    device = replica_setup(args, world, local)
    n = args.pop if args.pop != 1 << 20 else 1 << 17
    m, dim = args.nobj, 12
    stream = RandomStream(args.seed, island=rank)
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
    # the top-up evolves a copy of the state: the timed steps start from the
    # population --warmup steps leave, whatever the top-up's length
    saved = save_state([step.combined], stream, step)
    extra_warm = warm_until(args, lambda: step.step(stream))
    restore_state(saved)
    replica_barrier(world)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.steps)]
    t0 = time.perf_counter()
    for s in range(args.steps):
        ev[2 * s].record()
        step.step(stream)
        ev[2 * s + 1].record()
    replica_barrier(world)
    elapsed = replica_max(time.perf_counter() - t0, world, device)
    gen_ms = sum(ev[2 * s].elapsed_time(ev[2 * s + 1]) for s in range(args.steps)) / args.steps
    # stage breakdown outside the timed region: selNSGA2 alone on 2N rows
    # (current parents + one varOr batch of offspring)
    comb = step.combined
    sel_ms = []
    two = pop.like(2 * n, capacity=2 * n)
    ctx = comb.ctx.bind()
    _lib.call("dm_gather", ctx, ctypes.byref(comb.c_pop()), None, ctypes.byref(two.c_pop(0, n)))
    off = algorithms.varOr(comb, tb, n, 0.6, 0.3, evaluate=True, stream=stream)
    _lib.call("dm_gather", ctx, ctypes.byref(off.c_pop()), None, ctypes.byref(two.c_pop(n, n)))
    reps = 5
    _lib.call("dm_ctx_set_timing_target", ctx, _lib.DM_TIME_DOMINANCE)
    _lib.call("dm_ctx_set_timing", ctx, reps)
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        tools.selNSGA2(two, n)
        b.record()
        torch.cuda.synchronize()
        sel_ms.append(a.elapsed_time(b))
    times = (ctypes.c_float * reps)()
    cnt = ctypes.c_int32(0)
    _lib.call("dm_ctx_kernel_times", ctx, times, reps, ctypes.byref(cnt))
    _lib.call("dm_ctx_set_timing", ctx, 0)
    _lib.call("dm_ctx_set_timing_target", ctx, _lib.DM_TIME_GENERATION)
    assert cnt.value == reps, "expected one dominance kernel per selection, got %d" % cnt.value
    dom_ms = sorted(times[1:])[(reps - 1) // 2]
    sel_ms = sorted(sel_ms[1:])[(reps - 1) // 2]
    # the front peel, the selection's dominant kernel: every peel launch of one
    # selNSGA2 timed by HIP events the library records around it, in front order
    cap = 1024
    _lib.call("dm_ctx_set_timing_target", ctx, _lib.DM_TIME_PEEL)
    _lib.call("dm_ctx_set_timing", ctx, cap)
    tools.selNSGA2(two, n)
    torch.cuda.synchronize()
    ptimes = (ctypes.c_float * cap)()
    pcnt = ctypes.c_int32(0)
    _lib.call("dm_ctx_kernel_times", ctx, ptimes, cap, ctypes.byref(pcnt))
    _lib.call("dm_ctx_set_timing", ctx, 0)
    _lib.call("dm_ctx_set_timing_target", ctx, _lib.DM_TIME_GENERATION)
    peel_us = [t * 1e3 for t in ptimes[:min(cap, pcnt.value)]]
    # the chain without per-launch events (an event pair around each batch of
    # launches: the GPU time of the launches and the gaps between them; the
    # per-launch pairs above add ~5 us to each launch, profiles/r06_c5)
    _lib.call("dm_ctx_set_timing_target", ctx, _lib.DM_TIME_PEEL_CHAIN)
    _lib.call("dm_ctx_set_timing", ctx, 64)
    tools.selNSGA2(two, n)
    torch.cuda.synchronize()
    ctimes = (ctypes.c_float * 64)()
    ccnt = ctypes.c_int32(0)
    _lib.call("dm_ctx_kernel_times", ctx, ctimes, 64, ctypes.byref(ccnt))
    _lib.call("dm_ctx_set_timing", ctx, 0)
    _lib.call("dm_ctx_set_timing_target", ctx, _lib.DM_TIME_GENERATION)
    chain_ms = sum(ctimes[:min(64, ccnt.value)])
    sel_fronts = tools.sortNondominated(two, n)
    wvh = two.wvalues[:2 * n].cpu().numpy()
    usz = [int(len(np.unique(wvh[f.cpu().numpy()], axis=0))) for f in sel_fronts]
    peel = peel_report(peel_us, usz, m, chain_ms)
    peel["fronts"]["work"] = peel_work(wvh, sel_fronts, peel_us)
    fronts = tools.sortNondominated(two, 2 * n)
    wv = two.wvalues[:2 * n]
    ufit = torch.unique(wv, dim=0).cpu().numpy()
    uniq = int(ufit.shape[0])
    cmp_per_sel = float(m) * uniq * (uniq - 1) / 2.0
    # the count pass's (v, chunk) pairs: v below the reach of each 512-row
    # chunk of the objective-0 order
    o0 = np.sort(ufit[:, 0])
    nch = (uniq + 511) // 512
    reach = np.searchsorted(o0, o0[np.minimum(np.arange(nch) * 512 + 511, uniq - 1)], side="right")
    lds_bytes = float(reach.sum()) * (m - 1) * (11 * 4 + 64)
    lds_peak = 256 * 256 * 2.4e9 / 1e9  # GB/s of LDS reads (256 B/clk/CU)
    valu_peak = 256 * 4 * 32 * 2.4e9 / 1e9  # Gop/s of 32-bit integer VALU lane ops
    achieved = lds_bytes / (dom_ms * 1e-3) / 1e9
    cmp_rate = cmp_per_sel / (dom_ms * 1e-3) / 1e9
    if m <= 3:
        count_pass = {"bound": "lds", "achieved": round(achieved, 1), "peak": lds_peak,
                      "unit": "GB/s", "frac": round(achieved / lds_peak, 4),
                      "kernel": "bd_count_kernel<%d>" % m,
                      "kernel_ms": round(dom_ms, 4), "lds_bytes_per_launch": lds_bytes,
                      "count": "sum_c reach_c x (M-1) x (11 probes x 4 B + 64-B prefix set)",
                      "peak_basis": "LDS reads: 256 CU x 256 B/clk x 2.4 GHz"}
    else:
        # M = 4: the integer compare kernel (M-1 rank compares per pair below
        # the objective-0 diagonal) writing the D matrix the peel reads
        count_pass = {"bound": "valu", "achieved": round(cmp_rate, 1), "peak": valu_peak,
                      "unit": "G pair-compares/s", "frac": round(cmp_rate / valu_peak, 4),
                      "kernel": "tri_dom_kernel<%d>" % m, "kernel_ms": round(dom_ms, 4),
                      "count": "M U (U-1) / 2 pair compares (SURVEY.md §8d)",
                      "peak_basis": "32-bit VALU lane ops: 256 CU x 4 SIMD x 32 x 2.4 GHz"}
    count_pass.update({"compares_per_launch": cmp_per_sel, "compare_rate_G": round(cmp_rate, 1),
                       "unique_fits": uniq, "fronts": len(fronts)})
    out = {"metric": "individual-generations/sec @pop=2^17 DTLZ2 NSGA-II (C5)",
           "value": round(n * args.steps * world / elapsed, 1),
           "unit": "individual-generations/sec",
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "warmup_topup": {"secs": args.warmup_secs, "generations": extra_warm},
           "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": "C5 NSGA-II DTLZ2 M=%d D=12 eaMuPlusLambda(mu=lambda=N) + "
                                  "selNSGA2(2N->N)" % m, "pop": n, "genes": dim, "objectives": m,
                      "operators": "varOr cxBlend(0.5) mutGaussian(0,0.1,1/D) cxpb=0.6 mutpb=0.3",
                      "parallelism": "replicas%d" % world},
           "gen_ms_events": round(gen_ms, 4),
           "roofline": peel["roofline"],
           "peel": peel["fronts"],
           "count_pass": count_pass,
           "selection": {"ms": round(sel_ms, 4),
                         "what": "whole selNSGA2(2N -> N): ranks, bitset tables, counts, peel, "
                                 "crowding, last-front selection"},
           "cpu_baseline": None}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_nsga2(wv.cpu().numpy(), (-1.0,) * m, n)
    if rank == 0:
        print(json.dumps(out), flush=True)
    replica_finish(world)


def bench_nsga2_example(args, world=1, rank=0, local=0):
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
    device = replica_setup(args, world, local)
    n = args.pop if args.pop != 1 << 20 else 1 << 17
    m, dim = 3, 12
    stream = RandomStream(args.seed, island=rank)
    pop = tools.initPopulation(n=n, dim=dim, low=0.0, high=1.0, gtype="f64",
                               weights=(-1.0,) * m, device=device, stream=stream)
    tb = base.Toolbox()
    tb.register("mate", tools.cxSimulatedBinaryBounded, low=0.0, up=1.0, eta=20.0)
    tb.register("mutate", tools.mutPolynomialBounded, low=0.0, up=1.0, eta=20.0,
                indpb=1.0 / dim)
    benchmarks.dtlz2(pop, obj=m)
    two = pop.like(2 * n, capacity=2 * n)
    ctx = pop.ctx.bind()
    from deap_amd.device import zeros
    crowd_tmp = zeros((n,), torch.float64, device)

    def carry_crowding(dst, src, idx):
        # the chosen rows' crowding distances travel with them (dm_gather_f64,
        # no PyTorch index kernel); src may be dst's own buffer (staged)
        _lib.call("dm_gather_f64", ctx, ctypes.c_void_p(src.data_ptr()),
                  ctypes.c_void_p(idx.data_ptr()), n, ctypes.c_void_p(crowd_tmp.data_ptr()))
        if dst.crowding_dist is None or len(dst.crowding_dist) < n:
            dst.crowding_dist = zeros((dst.capacity,), torch.float64, device)
        _lib.call("dm_gather_f64", ctx, ctypes.c_void_p(crowd_tmp.data_ptr()), None, n,
                  ctypes.c_void_p(dst.crowding_dist.data_ptr()))

    def select_into(pop, off):
        # pop[:] = toolbox.select(pop + offspring, MU)                 (nsga2.py:114)
        _lib.call("dm_gather", ctx, ctypes.byref(pop.c_pop()), None, ctypes.byref(two.c_pop(0, n)))
        _lib.call("dm_gather", ctx, ctypes.byref(off.c_pop()), None, ctypes.byref(two.c_pop(n, n)))
        idx = tools.selNSGA2(two, n)
        _lib.call("dm_gather", ctx, ctypes.byref(two.c_pop()), ctypes.c_void_p(idx.data_ptr()),
                  ctypes.byref(pop.c_pop()))
        carry_crowding(pop, two.crowding_dist, idx)

    # pop = toolbox.select(pop, len(pop)): assigns the crowding distances (nsga2.py:92)
    idx0 = tools.selNSGA2(pop, n)
    carry_crowding(pop, pop.crowding_dist, idx0)
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
    saved = save_state([pop], stream)
    extra_warm = warm_until(args, lambda: one_gen(False))
    restore_state(saved)
    replica_barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_gen(True)
    replica_barrier(world)
    elapsed = replica_max(time.perf_counter() - t0, world, device)
    vms = sorted(a.elapsed_time(b) for a, b in var_ms)
    v_ms = sum(vms) / len(vms)
    var_bytes = (n // 2) * (4 * dim * 8) + n * (4 + 2 * m * 8 + 2)
    achieved = var_bytes / (v_ms * 1e-3) / 1e9
    out = {"metric": "individual-generations/sec @pop=2^17 DTLZ2 NSGA-II example loop (C5x)",
           "value": round(n * args.steps * world / elapsed, 1),
           "unit": "individual-generations/sec",
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "warmup_topup": {"secs": args.warmup_secs, "generations": extra_warm},
           "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": "C5x examples/ga/nsga2.py loop: selTournamentDCD + "
                                  "cxSimulatedBinaryBounded + mutPolynomialBounded + "
                                  "selNSGA2(2N->N)", "pop": n, "genes": dim, "objectives": m,
                      "parallelism": "replicas%d" % world},
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": 8000.0,
                        "unit": "GB/s", "frac": round(achieved / 8000.0, 4), "traffic": None,
                        "kernel": "bounded_vary_kernel (varBounded)",
                        "kernel_ms": round(v_ms, 5)},
           "cpu_baseline": None}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the loop's CPU cost is its selNSGA2 (selTournamentDCD and the bounded
        # operators of 2^17 individuals take seconds): the C5 baseline applies
        out["cpu_baseline"] = cpu_baseline_nsga2(two.wvalues[:2 * n].cpu().numpy(), (-1.0,) * m,
                                                 n, with_log=False)
    if rank == 0:
        print(json.dumps(out), flush=True)
    replica_finish(world)


if __name__ == "__main__":
    sys.exit(main() or 0)
