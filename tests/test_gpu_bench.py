"""bench.py's multi-rank path on one GPU (-m gpu): a plain `--gpus 2`
invocation (no launcher) starts two ranks itself; with the gloo backend both
share this GPU.  The line must report n_gpus 2, weak scaling over the query
split, and the corpus-sharded leg (id-range shards, all-gather, device merge)
must answer rank 0's batch exactly like rank 0's whole-corpus search."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_gpus2_gloo_rehearsal():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--rows", "60000",
           "--nq", "1000", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-hnsw-line"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    r = json.loads(line)
    assert r["n_gpus"] == 2 and r["scaling"] == "weak" and r["config"]["split"] == "query"
    assert r["value"] > 0
    assert r["corpus_sharded"]["ids_equal_query_split"] is True
    assert r["corpus_sharded"]["scaling"] == "strong"


def test_bench_refuses_mismatched_world_size():
    """CPU: the check runs before anything touches a GPU."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 2 and "WORLD_SIZE" in out.stdout
