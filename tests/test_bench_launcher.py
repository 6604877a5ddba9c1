"""bench.py --gpus N starts N rank processes itself (the driver's contract runs
`python bench.py --gpus N` with no external launcher), and rank 0 reports every
rank.  CPU only: the --dry-run mode runs the launch, the gloo rendezvous and the
report without any GPU work."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, cwd=ROOT,
                          capture_output=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    p = _run(["--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1"])
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    lines = [ln for ln in p.stdout.decode().splitlines() if ln.strip()]
    assert len(lines) == 1, lines  # ONE JSON line, from rank 0
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["world_size_observed"] == n
    assert out["launcher"] == "bench.py --gpus"
    assert [r["rank"] for r in out["per_rank"]] == list(range(n))
    # the rendezvous port lies outside the kernel's ephemeral range (no auto-bind can take it)
    sys.path.insert(0, ROOT)
    import bench

    lo, hi = bench.ephemeral_port_range()
    assert not lo <= out["master_port"] <= hi, (out["master_port"], lo, hi)
    # the reported time is the max over ranks
    assert out["ms_per_step"] == pytest.approx(max(r["ms_per_step"] for r in out["per_rank"]))


def test_gpus_1_runs_in_process():
    p = _run(["--gpus", "1", "--dry-run"])
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    out = json.loads(p.stdout.decode().strip())
    assert out["n_gpus"] == 1 and out["launcher"] == "external" and len(out["per_rank"]) == 1


def test_a_failed_rank_fails_the_launch_without_hanging():
    p = _run(["--gpus", "2", "--dry-run"], env={"RSX_BENCH_DRY_FAIL_RANK": "1"}, timeout=120)
    assert p.returncode != 0
    assert p.stdout.decode().strip() == ""


def test_rendezvous_port_is_outside_the_ephemeral_range():
    sys.path.insert(0, ROOT)
    import bench

    lo, hi = bench.ephemeral_port_range()
    ports = {bench.rendezvous_port() for _ in range(20)}
    assert all(not lo <= p <= hi and 0 < p < 65536 for p in ports), (ports, lo, hi)


def test_explicit_master_port_wins():
    p = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1"], env={"MASTER_PORT": "23457"})
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    assert json.loads(p.stdout.decode().strip())["master_port"] == 23457


def test_replica_hash_sees_permutations_and_cancelling_differences():
    import torch

    sys.path.insert(0, ROOT)
    import bench

    t = torch.randn(1000, 8)
    h = bench.replica_hash(t)
    assert torch.equal(h, bench.replica_hash(t.clone()))
    assert not torch.equal(h, bench.replica_hash(t.flip(0)))  # same words, other places
    w = t.clone().view(torch.int32)
    w.view(-1)[3] += 1
    w.view(-1)[5] -= 1  # a plain word sum cancels this
    assert not torch.equal(h, bench.replica_hash(w.view(torch.float32)))
