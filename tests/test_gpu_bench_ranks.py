"""The multi-rank bench path on a GPU: ``bench.py --gpus 2
--backend gloo`` runs the launcher -> torch.distributed.run rendezvous ->
deme ownership -> ``migRingDistributed`` (host-staged hops between the two
ranks, device pack / selection / placement) -> per-deme digests gathered to
rank 0, with both ranks on the one GPU of the test box (RCCL refuses two
ranks on one device; the driver's 8-GPU runs take the RCCL route).  Philox
streams are keyed by the deme id and the migration is exact, so every deme's
digest must equal the one-rank run's (deap/tools/migration.py:4-51,
examples/ga/onemax_island.py:140-154)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("cfg", ["c3", "c2"])
def test_two_ranks_on_one_gpu_match_one_rank(gpu, cfg):
    common = ["--config", cfg, "--islands", "4", "--pop", "16384", "--steps", "10",
              "--warmup", "2", "--warmup-secs", "0.2", "--no-cpu-baseline"]
    one = _bench(["--gpus", "1"] + common)
    two = _bench(["--gpus", "2", "--backend", "gloo"] + common)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    d1, d2 = one["deme_digests"], two["deme_digests"]
    assert d1["key"] == d2["key"]
    assert sorted(d1["digest"]) == ["0", "1", "2", "3"]
    assert d1["digest"] == d2["digest"]
    # the migrations ran: 12 generations at mig_every 5 (+ the untimed one)
    assert two["migration"]["every"] == 5 and two["migration"]["ms_per_migration"] > 0
