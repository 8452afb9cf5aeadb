"""bench.py --gpus N launches its own ranks (torch.distributed.run, gloo here) and
runs the rank path end to end: sharded partial sigma, all-reduce, max-over-ranks
timing, one JSON line from rank 0 (CPU; the operator is the oracle stub)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_launches_two_ranks():
    env = dict(os.environ, XT_BENCH_BACKEND="gloo", XT_BENCH_OPERATOR="bench_stub:make_workload",
               PYTHONPATH=os.path.join(ROOT, "tests") + os.pathsep + ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--nao", "24", "--nclosed", "5", "--nopen", "2", "--naux", "40", "--ngrid", "600", "--nvec", "3"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout       # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1
    assert d["scaling"] == "strong" and d["value"] > 0
    assert d["verify"] < 1e-12, d["verify"]   # all-reduced shard sums == full operator
    assert "STUB" in d["data"]
