"""In-process multi-GPU group (wv_group_*, SURVEY 8e, index.go:967-1044), -m gpu.

The box has one MI355X, so the members of these groups share device 0: the
per-shard lists then reach the root by device copies (RCCL cannot put one
device twice in a communicator); the sharding, allow-list slicing, gather
layout and device merge are the ones the multi-device RCCL path uses.
"""
import threading

import numpy as np
import pytest

import pyoracle as O
import weaviate_amd as W

pytestmark = pytest.mark.gpu


def _data(n, nq, d, seed):
    rng = np.random.default_rng(seed)
    return rng.random((n, d), dtype=np.float32), rng.random((nq, d), dtype=np.float32)


@pytest.mark.parametrize("metric", ["l2-squared", "dot", "cosine-dot"])
@pytest.mark.parametrize("members", [2, 3])
def test_shard_group_exact_equals_one_index(metric, members):
    n, nq, d, k = 30_000, 300, 64, 10
    base, qs = _data(n, nq, d, 1)
    g = W.GPUGroup([0] * members, d, metric, capacity=n, layout="shard")
    assert g.info() == {"members": members, "uses_rccl": False}
    g.upload_vectors(base)
    gi, gd, gn = g.search_batch(qs, k, mode="exact")
    oi, od, on = O.flat_scan(O.METRICS[metric], base if metric != "cosine-dot" else O.normalize_rows(base),
                             qs if metric != "cosine-dot" else O.normalize_rows(qs), k)
    assert gi.tolist() == oi.tolist()
    assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))
    g.close()


def test_shard_group_allow_lists_shared_and_per_query():
    n, nq, d, k = 20_000, 64, 32, 10
    base, qs = _data(n, nq, d, 2)
    g = W.GPUGroup([0, 0], d, "l2-squared", capacity=n, layout="shard")
    g.upload_vectors(base)
    one = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    one.upload_vectors(base)
    rng = np.random.default_rng(3)
    shared = W.AllowList.from_ids(rng.choice(n, 700, replace=False), n)
    per_q = [W.AllowList.from_ids(rng.choice(n, 300 + 17 * i, replace=False), n) for i in range(nq)]
    # a list that ends inside the first shard (no bit of the second is set)
    short = W.AllowList.from_ids(np.arange(0, 5000, 3), 5000)
    for allow in (shared, per_q, short):
        gi, gd, gn = g.search_batch(qs, k, allow=allow, mode="exact")
        oi, od, on = one.search_batch(qs, k, allow=allow, mode="exact")
        assert gi.tolist() == oi.tolist() and gn.tolist() == on.tolist()
        assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))
    g.close()
    one.close()


def test_shard_group_hnsw_equals_per_shard_searches_merged():
    """Each shard holds its own graph (as each Weaviate shard holds its own
    hnsw); the group's answer is the per-shard answers merged by (dist, id)."""
    n, nq, d, k, ef = 16_000, 200, 48, 10, 64
    base, qs = _data(n, nq, d, 4)
    g = W.GPUGroup([0, 0], d, "l2-squared", capacity=n, layout="shard", max_connections=16)
    g.upload_vectors(base)
    per = []
    for i in range(2):
        mix, b0, cap = g.member(i)
        rows = base[b0:b0 + cap]
        ref = O.Index(d, "l2-squared", 16, 64, capacity=rows.shape[0])
        ref.add_batch(rows, threads=8)
        mix.upload_graph(ref.export_graph())
        ri, rd, rn, _ = ref.search_batch(qs, k, ef, threads=8)
        per.append((ri.astype(np.uint64) + b0, rd, rn))
    gi, gd, gn = g.search_batch(qs, k, ef=ef, mode="hnsw")
    for q in range(nq):
        cand = []
        for ri, rd, rn in per:
            cand += [(float(rd[q, j]), int(ri[q, j])) for j in range(rn[q])]
        cand.sort()
        exp = cand[:k]
        assert [int(x) for x in gi[q, :gn[q]]] == [c[1] for c in exp], q
        assert np.array_equal(gd[q, :gn[q]], np.array([c[0] for c in exp], np.float32))
    g.close()


def test_replica_group_equals_one_index_and_routes_writes():
    n, nq, d, k = 12_000, 301, 32, 10
    base, qs = _data(n, nq, d, 5)
    g = W.GPUGroup([0, 0, 0], d, "l2-squared", capacity=n + 100, layout="replica", max_connections=16)
    g.upload_vectors(base)
    one = W.GPUVectorIndex(d, "l2-squared", capacity=n + 100, max_connections=16)
    one.upload_vectors(base)
    ref = O.Index(d, "l2-squared", 16, 64, capacity=n)
    ref.add_batch(base, threads=8)
    graph = ref.export_graph()
    for i in range(3):
        g.member(i)[0].upload_graph(graph)
    one.upload_graph(graph)
    # writes reach every replica: tombstones and added rows
    dead = np.arange(0, n, 7, dtype=np.uint64)
    g.add_tombstones(dead)
    one.add_tombstones(dead)
    new_rows = np.random.default_rng(6).random((50, d), dtype=np.float32)
    new_ids = np.arange(n, n + 50, dtype=np.uint64)
    g.add(new_ids, new_rows)
    one.add(new_ids, new_rows)
    for mode, ef in (("exact", 0), ("hnsw", 64)):
        gi, gd, gn = g.search_batch(qs, k, ef=ef, mode=mode)
        oi, od, on = one.search_batch(qs, k, ef=ef, mode=mode)
        assert gi.tolist() == oi.tolist(), mode
        assert np.array_equal(gd.view(np.uint32), od.view(np.uint32)), mode
        assert not np.isin(gi, dead).any()
    hit = g.search_batch(new_rows, 1, ef=64, mode="hnsw")[0][:, 0]
    assert hit.tolist() == new_ids.tolist()
    g.close()
    one.close()


def test_batcher_over_a_shard_group():
    n, d, k = 10_000, 32, 10
    base, qs = _data(n, 64, d, 7)
    g = W.GPUGroup([0, 0], d, "l2-squared", capacity=n, layout="shard", flat_search_cutoff=10**9)
    g.upload_vectors(base)
    exp_i, exp_d, _ = g.search_batch(qs, k, mode="exact")
    b = W.Batcher(g, max_batch=32, max_wait_us=2000)
    allow = W.AllowList.from_ids(np.arange(n), n)   # below the cutoff: flat search, exact
    out = [None] * len(qs)

    def work(i):
        out[i] = b.search(qs[i], k, allow=allow)

    ts = [threading.Thread(target=work, args=(i,)) for i in range(len(qs))]
    [t.start() for t in ts]
    [t.join() for t in ts]
    for i, (ids, ds) in enumerate(out):
        assert ids.tolist() == exp_i[i].tolist()
        assert np.array_equal(ds.view(np.uint32), exp_d[i].view(np.uint32))
    st = b.stats()
    assert st["requests"] == len(qs) and st["batches"] < len(qs)
    b.close()
    g.close()


def test_bench_group_leg_child_equals_single_gpu(tmp_path):
    """bench.py's in-process group leg (run by rank 0 at N > 1) on two members
    of device 0: same ids and distances as one index over the whole corpus."""
    import json
    import os
    import subprocess
    import sys

    from bench import counter_uniform
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n, d, nq, k = 100_000, 128, 1000, 10
    one = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    one.upload_vectors(counter_uniform(1, 0, n, d))
    ids, ds, _ = one.search_batch(counter_uniform(2, 0, nq, d), k, mode="exact")
    one.close()
    ref = tmp_path / "ref.npz"
    np.savez(ref, ids=ids, dists=ds)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--group-leg", "--group-devices", "0,0",
                        "--rows", str(n), "--dim", str(d), "--nq", str(nq), "--k", str(k), "--steps", "2",
                        "--warmup", "1", "--dump-ids", str(ref)], capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stderr[-1500:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["members"] == 2 and r["uses_rccl"] is False and r["ids_equal_single_gpu"] is True, r
