"""``bench.py --gpus N`` launches N ranks itself.

The driver's scaling command is ``python bench.py --gpus N`` on one node (or
the same under ``torch.distributed.run``).  Without ``WORLD_SIZE`` in the
environment bench.py starts ``torch.distributed.run`` with N ranks as a child
process, relays rank 0's JSON line and checks ``n_gpus == N``.  On CPU the
``--dry-run --backend gloo`` mode runs everything up to the first kernel: the
rendezvous, the deme ownership agreed by ``islands.owner_map`` (all_gather)
and every rank's migRing hop plan from the C ABI's planner (``dm_mig_plan``),
which must equal the ring of ``deap/tools/migration.py:4-51`` /
``examples/ga/onemax_island.py:140-154`` routed across ranks."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    return p


def _expected_hops(owner, me):
    n = len(owner)
    want = []
    for frm in range(n):
        to = (frm + 1) % n
        s, d = owner[frm], owner[to]
        if s == me and d == me:
            want.append(["local", frm, to, me])
        elif s == me:
            want.append(["send", frm, to, d])
        elif d == me:
            want.append(["recv", frm, to, s])
    return want


def _lib_built():
    from deap_amd import _lib
    return os.path.exists(_lib.LIB_PATH)


@pytest.mark.parametrize("gpus,per", [(2, 1), (2, 2), (4, 1), (8, 1)])
def test_gpus_n_launches_n_ranks(gpus, per):
    if not _lib_built():
        pytest.skip("libdeapmi.so not built")
    p = _run(["--gpus", str(gpus), "--backend", "gloo", "--dry-run",
              "--islands-per-gpu", str(per)])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == gpus and out["dry_run"] is True
    assert out["islands"] == gpus * per and out["scaling"] == "weak"
    owner = [d // per for d in range(gpus * per)]
    assert out["owner"] == owner
    assert len(out["hops"]) == gpus
    for r in range(gpus):
        assert out["hops"][r] == _expected_hops(owner, r), "rank %d" % r
    # every cross-rank send has exactly one matching receive
    sends = sorted((h[1], h[2]) for r in range(gpus) for h in out["hops"][r] if h[0] == "send")
    recvs = sorted((h[1], h[2]) for r in range(gpus) for h in out["hops"][r] if h[0] == "recv")
    assert sends == recvs and len(sends) == (gpus if gpus > 1 else 0)


def test_islands_strong_split():
    """``--islands 8`` at 2 GPUs: 4 demes per rank, strong scaling."""
    if not _lib_built():
        pytest.skip("libdeapmi.so not built")
    p = _run(["--gpus", "2", "--backend", "gloo", "--dry-run", "--islands", "8"])
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 2 and out["islands"] == 8 and out["scaling"] == "strong"
    assert out["owner"] == [0] * 4 + [1] * 4


def test_single_gpu_runs_in_process():
    if not _lib_built():
        pytest.skip("libdeapmi.so not built")
    p = _run(["--dry-run"])
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 1 and out["islands"] == 1


def test_world_size_mismatch_is_refused():
    p = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


def test_failing_rank_fails_the_launch():
    """A rank that dies makes bench.py exit non-zero (no partial JSON)."""
    p = _run(["--gpus", "2", "--backend", "gloo", "--dry-run", "--islands", "3"])
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_driver_torchrun_form():
    """The driver's own form: ``torch.distributed.run --nproc-per-node N
    bench.py --gpus N`` (WORLD_SIZE set by torchrun, equal to --gpus)."""
    if not _lib_built():
        pytest.skip("libdeapmi.so not built")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend",
                        "gloo", "--dry-run"], env=env, capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["owner"] == [0, 1]


def test_digest_reference_check(tmp_path, monkeypatch):
    """bench.py's self-check of a scaling run: the per-deme digests are looked
    up in the committed one-GPU reference by everything they depend on
    (config, deme size and count, seed, generations, migration schedule) --
    'match', 'mismatch' (the run then exits non-zero) or 'no reference'."""
    sys.path.insert(0, ROOT)
    import bench
    ref = tmp_path / "digests.json"
    monkeypatch.setattr(bench, "DIGESTS", str(ref))
    args = bench.parse(["--islands", "8", "--steps", "20", "--warmup", "5"])
    key = bench.digest_key(args, 1 << 20, 8)
    assert "islands=8" in key and "steps=20" in key and "warmup=5" in key
    digest = {str(d): "%016x" % (d * 7919) for d in range(8)}
    assert bench.check_digests(key, digest) == "no reference"
    bench.save_digests(str(ref), key, digest)
    assert bench.check_digests(key, digest) == "match"
    bad = dict(digest, **{"3": "0" * 16})
    assert bench.check_digests(key, bad) == "mismatch"
    other = bench.digest_key(bench.parse(["--islands", "8", "--steps", "21"]), 1 << 20, 8)
    assert bench.check_digests(other, digest) == "no reference"


def test_committed_digest_reference_is_well_formed():
    """profiles/deme_digests.json (one-GPU runs of bench.py --digests-out):
    every entry maps deme ids 0..islands-1 to 64-bit hex digests."""
    path = os.path.join(ROOT, "profiles", "deme_digests.json")
    if not os.path.exists(path):
        pytest.skip("no committed reference yet")
    with open(path) as f:
        table = json.load(f)
    assert table
    for key, digest in table.items():
        islands = int(key.split("islands=")[1].split()[0])
        assert sorted(digest, key=int) == [str(d) for d in range(islands)]
        assert all(len(h) == 16 and int(h, 16) >= 0 for h in digest.values())
