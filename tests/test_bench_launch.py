"""bench.py --gpus N launches its own ranks (torch.distributed.run, gloo here) and
runs the rank path end to end: sharded partial sigma, all-reduce, max-over-ranks
timing, one JSON line from rank 0 (CPU; the operator is the oracle stub)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


import pytest  # noqa: E402


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_self_launches_ranks(world):
    env = dict(os.environ, XT_BENCH_BACKEND="gloo", XT_BENCH_OPERATOR="bench_stub:make_workload",
               PYTHONPATH=os.path.join(ROOT, "tests") + os.pathsep + ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "2", "--warmup", "1",
           "--nao", "24", "--nclosed", "5", "--nopen", "2", "--naux", "40", "--ngrid", "600", "--nvec", "3"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout       # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["steps"] == 2 and d["warmup"] == 1
    assert d["scaling"] == "strong" and d["value"] > 0
    assert d["verify"] < 1e-12, d["verify"]   # all-reduced shard sums == full operator
    assert "STUB" in d["data"]
    # per-rank phase split from every rank
    assert [x["rank"] for x in d["ranks"]] == list(range(world))
    for x in d["ranks"]:
        assert x["ax_ms"] > 0 and x["allreduce_ms"] >= 0 and x["sigma_mb"] > 0


@pytest.mark.gpu
def test_bench_two_ranks_on_the_gpu():
    """The real operator at N = 2 (both ranks on the visible MI355X over gloo; the
    driver's scaling run uses RCCL on separate GPUs): the launcher, grid / exchange-row
    sharding per rank, the all-reduce of sigma, the replicated Davidson under its lockstep
    guard and the max-over-ranks timing run end to end, and rank 0 prints one line.  The
    synthetic data are block-seeded, so the 2-rank run solves the 1-rank problem: the same
    lowest root to 1e-10 Ha and the same iteration count.  A gloo rehearsal reports the
    one physical GPU as n_gpus and says it is a rehearsal."""
    args = ["--steps", "2", "--warmup", "1", "--nao", "120", "--nclosed", "20", "--nopen", "2",
            "--naux", "360", "--ngrid", "20000", "--nvec", "8", "--nroots", "6", "--no-cpu-baseline"]
    out = {}
    for n in (1, 2):
        env = dict(os.environ, XT_BENCH_BACKEND="gloo")
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n)] + args
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, r.stdout
        out[n] = json.loads(lines[0])
    d = out[2]
    assert d["n_gpus"] == 1 and "rehearsal" in d and d["value"] > 0 and "STUB" not in d["data"]
    assert "grid sharded x2" in d["config"]["parallelism"]
    assert len(d["ranks"]) == 2 and all(x["ax_ms"] > 0 for x in d["ranks"])
    c1, c2 = out[1]["converge"], d["converge"]
    assert c1["converged"] and c2["converged"]
    assert abs(c1["e_min_ha"] - c2["e_min_ha"]) < 1e-10, (c1, c2)
    assert c1["iterations"] == c2["iterations"]


@pytest.mark.gpu
def test_bench_under_rccl_single_rank():
    """RCCL itself on the one-GPU pool: the driver's launch line (torch.distributed.run)
    at one rank with XT_BENCH_FORCE_PG=1, so bench.py initialises the nccl (= RCCL) group
    with device_id, and runs its barriers, the max-over-ranks all-reduce of the timed
    region on a device tensor, all_gather_object of the per-rank split and the group's
    teardown -- every collective the 8-GPU run calls, on one rank."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, XT_BENCH_FORCE_PG="1", XT_BENCH_BACKEND="nccl")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--config", "C1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and "STUB" not in d["data"]
    assert len(d["ranks"]) == 1 and d["ranks"][0]["rank"] == 0 and d["ranks"][0]["ax_ms"] > 0
    assert d["converge"]["converged"]
