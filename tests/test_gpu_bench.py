"""bench.py's multi-rank path on one GPU (-m gpu): a plain `--gpus 2`
invocation (no launcher) starts two ranks itself; with the gloo backend both
share this GPU.  The line must report n_gpus 2, weak scaling over the query
split, and the corpus-sharded leg (id-range shards, all-gather, device merge)
must answer rank 0's batch exactly like rank 0's whole-corpus search."""
import json
import os
import subprocess
import sys

import numpy as np
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


@pytest.mark.gpu
def test_bench_sharded_hnsw_two_ranks_equal_per_shard_restatement(tmp_path):
    """configs[4]'s layout (north_star: corpus sharded, local top-k, merge over
    RCCL): `--workload hnsw --split corpus` on 2 ranks (gloo, one GPU) -- each
    rank builds the graph of its id range on the GPU and searches the same
    batch; the merged ids must equal the restatement searching each rank's
    own graph, offset to global ids and merged by (dist, id)
    (index.go:967-1044), up to the order among equal distances."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, ROOT)
    import pyoracle as O
    from bench import counter_gauss
    from helpers import merge_lists, same_tie_aware
    n, d, nq, k, ef = 40000, 96, 300, 10, 64
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    dump = str(tmp_path / "rank%(rank)d.npz")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--workload",
           "hnsw", "--split", "corpus", "--rows", str(n), "--dim", str(d), "--nq", str(nq), "--data", "gauss",
           "--M", "16", "--efc", "64", "--ef", str(ef), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
           "--concurrency", "", "--dump-ids", dump]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert r["n_gpus"] == 2 and r["scaling"] == "strong" and r["config"]["split"] == "corpus"
    qs = counter_gauss(2, 0, nq, d)
    parts, merged = [], None
    for rank in range(2):
        z = np.load(dump % {"rank": rank})
        lo, nl = int(z["lo"]), int(z["n_local"])
        g = {key[2:]: (z[key] if z[key].ndim else int(z[key])) for key in z.files if key.startswith("g_")}
        ref = O.Index(d, "l2-squared", 16, 64, capacity=nl, seed=1)
        ref.import_graph(counter_gauss(1, lo, nl, d), g)
        oi, od, on, _ = ref.search_batch(qs, k, ef, threads=8)
        # the rank's own shard answer is the restatement's on that graph
        for i in range(nq):
            same_tie_aware(z["shard_ids"][i] - np.uint64(lo), z["shard_dists"][i], oi[i], od[i])
        parts.append((oi + np.uint64(lo), od, on))
        merged = (z["ids"], z["dists"])
    mi, md, _ = merge_lists(parts, k)
    for i in range(nq):
        same_tie_aware(merged[0][i], merged[1][i], mi[i], md[i])
