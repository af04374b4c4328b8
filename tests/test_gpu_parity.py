"""Parity of the HIP path (through the C ABI) against the CPU restatement.

Bar: bit-identical ids and distances on tie-free float data (uniform [0,1)),
since every distance the GPU returns is computed in the reference's own
summation order.  Runs on an MI355X (-m gpu).
"""
import numpy as np
import pytest

import pyoracle as O
import weaviate_amd as W

pytestmark = pytest.mark.gpu

METRIC_NAMES = {O.L2: "l2-squared", O.DOT: "dot", O.COSINE: "cosine-dot"}


def _data(n, d, nq, seed=0, metric=O.L2):
    rng = np.random.default_rng(seed)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((nq, d), dtype=np.float32)
    if metric == O.DOT:
        base -= 0.5
        qs -= 0.5
    return base, qs


def _norm_rows(a):
    return np.stack([O.normalize(r) for r in a])


def _same(a_ids, a_d, b_ids, b_d):
    assert a_ids.tolist() == b_ids.tolist()
    assert np.array_equal(a_d.view(np.uint32), b_d.view(np.uint32))


def _same_tie_aware(a_ids, a_d, b_ids, b_d):
    """Distances bit-identical; ids identical up to the order among equal
    distances, and free at the k-boundary distance (the reference breaks ties
    by heap layout, the GPU by id: SURVEY 8c)."""
    assert np.array_equal(a_d.view(np.uint32), b_d.view(np.uint32))
    if len(a_d) == 0:
        return
    last = a_d[-1]
    for v in np.unique(a_d):
        if v == last:
            continue
        assert set(a_ids[a_d == v].tolist()) == set(b_ids[b_d == v].tolist())


@pytest.mark.parametrize("dim", [1, 3, 4, 16, 31, 32, 35, 64, 100, 128, 130, 256, 777])
@pytest.mark.parametrize("metric", [O.L2, O.DOT, O.COSINE])
def test_exact_distance_bitwise_all_dims(dim, metric):
    """Rows D1-D3 of SURVEY 8a: the GPU distancer equals asm.L2/asm.Dot bit for bit
    (lengths of distancer/l2_amd64_test.go:36)."""
    base, qs = _data(257, dim, 4, seed=dim, metric=metric)
    ix = W.GPUVectorIndex(dim, METRIC_NAMES[metric], capacity=257)
    ix.upload_vectors(base)
    k = 40  # > 32: the exact-scan path, every distance reference-order
    ids, ds, n = ix.search_batch(qs, k, mode="exact")
    b = _norm_rows(base) if metric == O.COSINE else base
    q = _norm_rows(qs) if metric == O.COSINE else qs
    oi, od, on = O.flat_scan(metric, b, q, k)
    for i in range(len(qs)):
        _same_tie_aware(ids[i, : n[i]], ds[i, : n[i]], oi[i, : on[i]], od[i, : on[i]])
    ix.close()


@pytest.mark.parametrize("metric", [O.L2, O.DOT, O.COSINE])
def test_bruteforce_mfma_ids_identical(metric):
    base, qs = _data(20000, 128, 300, seed=1, metric=metric)
    ix = W.GPUVectorIndex(128, METRIC_NAMES[metric], capacity=20000)
    ix.upload_vectors(base)
    ids, ds, n = ix.search_batch(qs, 10, mode="exact")
    b = _norm_rows(base) if metric == O.COSINE else base
    q = _norm_rows(qs) if metric == O.COSINE else qs
    oi, od, on = O.flat_scan(metric, b, q, 10)
    assert (n == 10).all()
    _same(ids, ds, oi, od)
    st = ix.last_batch_stats()
    assert st["fallbacks"] <= 3, st  # the certificate holds on almost every query
    ix.close()


def test_bruteforce_integer_data_with_ties_uses_exact_fallback():
    """SIFT-shaped integer data (many equal distances): when the candidate lists
    hold tied keys at the boundary the certificate cannot separate them and the
    batched exact fallback answers; the result must equal the restatement up to
    the order among equal distances, with (dist, id) order among ties.

    Without the running threshold (WV_H16_NO_RUNNING) the lists fill with the
    tied keys deterministically, so the fallback must run.  With it (default:
    corpora too small for the seed pass) whether a query certifies depends on
    when the shared threshold tightens -- both outcomes are exact, which the
    default run checks."""
    import os
    rng = np.random.default_rng(21)
    base = rng.integers(0, 3, (20000, 16)).astype(np.float32)
    qs = rng.integers(0, 3, (200, 16)).astype(np.float32)
    oi, od, on = O.flat_scan(O.L2, base, qs, 10)
    for env in ({"WV_H16_NO_RUNNING": "1"}, {}):
        os.environ.update(env)
        try:
            ix = W.GPUVectorIndex(16, "l2-squared", capacity=20000)
            ix.upload_vectors(base)
            ids, ds, n = ix.search_batch(qs, 10, mode="exact")
            fb = ix.last_batch_stats()["fallbacks"]
            ix.close()
        finally:
            for key in env:
                os.environ.pop(key, None)
        if env:
            assert fb > 0
        for i in range(len(qs)):
            _same_tie_aware(ids[i], ds[i], oi[i], od[i])
            # (dist, id) order: among equal distances the smallest ids win
            full = ((base.astype(np.float64) - qs[i].astype(np.float64)) ** 2).sum(1)
            order = np.lexsort((np.arange(len(base)), full))[:10]
            assert ids[i].tolist() == order.tolist()


def test_bruteforce_ragged_sizes_and_small_batches():
    for n_base, nq, k in [(1, 1, 10), (5, 3, 10), (129, 1, 1), (1000, 7, 32), (3001, 129, 10)]:
        base, qs = _data(n_base, 96, nq, seed=n_base)
        ix = W.GPUVectorIndex(96, "l2-squared", capacity=n_base)
        ix.upload_vectors(base)
        ids, ds, n = ix.search_batch(qs, k, mode="exact")
        oi, od, on = O.flat_scan(O.L2, base, qs, k)
        assert n.tolist() == on.tolist()
        for i in range(nq):
            _same(ids[i, : n[i]], ds[i, : n[i]], oi[i, : on[i]], od[i, : on[i]])
        ix.close()


def test_bruteforce_allow_list_and_tombstones():
    n_base = 8000
    base, qs = _data(n_base, 64, 64, seed=3)
    rng = np.random.default_rng(4)
    allow_ids = np.nonzero(rng.random(n_base) < 0.1)[0]
    tomb_ids = np.nonzero(rng.random(n_base) < 0.05)[0]
    ix = W.GPUVectorIndex(64, "l2-squared", capacity=n_base)
    ix.upload_vectors(base)
    ix.set_tombstones(tomb_ids)
    al = W.AllowList.from_ids(allow_ids, n_base)
    ids, ds, n = ix.search_batch(qs, 10, allow=al, mode="exact")
    tb = O.bits_from_ids(tomb_ids, n_base)
    oi, od, on = O.flat_scan(O.L2, base, qs, 10, allow_bits=al.words, tomb_bits=tb)
    _same(ids, ds, oi, od)
    assert not set(ids.ravel().tolist()) & set(tomb_ids.tolist())
    # per-query allow lists
    per = [W.AllowList.from_ids(np.nonzero(rng.random(n_base) < 0.2)[0], n_base) for _ in range(len(qs))]
    ids, ds, n = ix.search_batch(qs, 10, allow=per, mode="exact")
    for i in range(len(qs)):
        oi, od, on = O.flat_scan(O.L2, base, qs[i : i + 1], 10, allow_bits=per[i].words, tomb_bits=tb)
        _same(ids[i], ds[i], oi[0], od[0])
    ix.close()


def test_large_k_exact_path():
    base, qs = _data(5000, 32, 5, seed=6)
    ix = W.GPUVectorIndex(32, "dot", capacity=5000)
    ix.upload_vectors(base)
    ids, ds, n = ix.search_batch(qs, 150, mode="exact")
    oi, od, on = O.flat_scan(O.DOT, base, qs, 150)
    _same(ids, ds, oi, od)
    ix.close()


def _build_graph(n, d, metric=O.L2, M=16, efc=64, seed=11):
    rng = np.random.default_rng(seed)
    base = rng.random((n, d), dtype=np.float32)
    idx = O.Index(d, metric, M, efc, capacity=n, seed=seed)
    idx.add_batch(base, threads=8)
    return base, idx


@pytest.mark.parametrize("metric", [O.L2, O.COSINE, O.DOT])
def test_hnsw_identical_to_reference_restatement(metric):
    n, d = 6000, 48
    base, idx = _build_graph(n, d, metric)
    qs = np.random.default_rng(99).random((200, d), dtype=np.float32)
    g = idx.export_graph()
    ix = W.GPUVectorIndex(d, METRIC_NAMES[metric], capacity=n, max_connections=16)
    ix.upload_vectors(base)
    ix.upload_graph(g)
    for ef in (10, 32, 100):
        ids, ds, cnt = ix.search_batch(qs, 10, ef=ef, mode="hnsw")
        # the restatement normalizes cosine queries itself (search.go:68-72)
        oi, od, on, st = idx.search_batch(qs, 10, ef, threads=8)
        assert cnt.tolist() == on.tolist()
        _same(ids, ds, oi, od)
    ix.close()


def test_hnsw_filtered_and_tombstoned_identical():
    n, d = 5000, 32
    base, idx = _build_graph(n, d, O.L2)
    qs = np.random.default_rng(7).random((100, d), dtype=np.float32)
    rng = np.random.default_rng(8)
    allow = np.nonzero(rng.random(n) < 0.5)[0]
    tomb = np.nonzero(rng.random(n) < 0.03)[0]
    for t in tomb:
        idx.add_tombstone(int(t))
    g = idx.export_graph()
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n, max_connections=16, forbid_flat=True)
    ix.upload_vectors(base)
    ix.upload_graph(g)
    ix.set_tombstones(tomb)
    al = W.AllowList.from_ids(allow, n)
    ids, ds, cnt = ix.search_batch(qs, 10, ef=64, allow=al, mode="hnsw")
    oi, od, on, st = idx.search_batch(qs, 10, 64, allow=al.words)
    assert ix.last_batch_stats()["fallbacks"] == 0
    _same(ids, ds, oi, od)
    ix.close()


def test_kat_hand_built_graph_on_gpu(kats):
    c = kats["hand_built_graph"]
    vec = np.array(c["vectors"], np.float32)
    n = len(vec)
    levels = np.full(n, -1, np.int8)
    layer0 = np.full((n, 4), 0xFFFFFFFF, np.uint32)
    upper_row = np.full(n, 0xFFFFFFFF, np.uint32)
    upper = np.full((1, c["max_level"], 4), 0xFFFFFFFF, np.uint32)
    r = 0
    for nd in c["nodes"]:
        levels[nd["id"]] = nd["level"]
        layer0[nd["id"], : len(nd["connections"][0])] = nd["connections"][0]
        if nd["level"] >= 1:
            upper_row[nd["id"]] = r
            for lv in range(1, nd["level"] + 1):
                upper[r, lv - 1, : len(nd["connections"][lv])] = nd["connections"][lv]
            r += 1
    g = dict(n=n, entrypoint=c["entrypoint"], max_level=c["max_level"], levels=levels, layer0=layer0,
             upper_row=upper_row, upper=upper)
    ix = W.GPUVectorIndex(2, "l2-squared", capacity=n, max_connections=2, ef=0, dynamic_ef_min=0,
                          dynamic_ef_max=0, dynamic_ef_factor=0, flat_search_cutoff=0)
    ix.upload_vectors(vec)
    ix.upload_graph(g)
    ids, _ = ix.search_by_vector(c["query"], c["k"])
    assert ids.tolist() == c["expect"]
    ix.close()


def test_kat_delete_snapshot_on_gpu(kats):
    c = kats["delete_snapshot"]
    snap = c["snapshot"]
    vec = np.array(c["vectors"], np.float32)
    ref = O.Index(3, c["metric"], 30, 128, capacity=len(vec))
    for i, v in enumerate(vec):
        ref.set_vector(i, v)
    for nd in snap["nodes"]:
        ref.import_node(nd["id"], nd["level"], [nd["connections"][str(l)] for l in range(nd["level"] + 1)])
    ref.set_entrypoint(snap["entrypoint"], snap["currentMaximumLayer"])
    g = ref.export_graph(deg0=64, degU=32)
    ix = W.GPUVectorIndex(3, "cosine-dot", capacity=len(vec), max_connections=30, ef=0, dynamic_ef_min=0,
                          dynamic_ef_max=0, dynamic_ef_factor=0, flat_search_cutoff=0, forbid_flat=True)
    ix.upload_vectors(vec)
    ix.upload_graph(g)
    odd = W.AllowList.from_ids([i for i in range(len(vec)) if i % 2 == 1], len(vec))
    control, _ = ix.search_by_vector(c["query"], c["k"], allow=odd)
    ref.set_search_config(ef=0, ef_min=0, ef_max=0, ef_factor=0, flat_search_cutoff=0, forbid_flat=True)
    rids, _ = ref.search_by_vector(c["query"], c["k"], allow=odd.words)
    assert control.tolist() == rids.tolist()
    ix.set_tombstones(c["tombstone_after"])
    res, _ = ix.search_by_vector(c["query"], c["k"])
    assert res.tolist() == control.tolist()
    ix.close()


def test_acceptance_distances_on_gpu(kats):
    a = kats["acceptance_distances"]
    for name, metric in (("l2", "l2-squared"), ("dot", "dot"), ("cosine", "cosine-dot")):
        c = a[name]
        ix = W.GPUVectorIndex(len(c["query"]), metric, capacity=len(c["objects"]))
        ix.upload_vectors(np.array(c["objects"], np.float32))
        _, d = ix.search_by_vector(c["query"], 10)
        assert d.tolist() == pytest.approx(c["expect"], abs=0.01)
        if name != "cosine":
            lim = c["limited"] if isinstance(c["limited"], list) else [c["limited"]]
            for l in lim:
                _, d = ix.search_by_vector_distance(c["query"], l["distance"])
                assert d.tolist() == pytest.approx(l["expect"], abs=0.01)
        ix.close()


def test_search_by_vector_distance_matches_restatement():
    base, idx = _build_graph(3000, 16, O.L2)
    g = idx.export_graph()
    ix = W.GPUVectorIndex(16, "l2-squared", capacity=3000, max_connections=16)
    ix.upload_vectors(base)
    ix.upload_graph(g)
    q = np.random.default_rng(3).random(16, dtype=np.float32)
    for target in (0.3, 0.6):
        a_ids, a_d = ix.search_by_vector_distance(q, target)
        b_ids, b_d = idx.search_by_vector_distance(q, target)
        assert a_ids.tolist() == b_ids.tolist()
    ix.close()


def test_merge_shards_device():
    import torch
    rng = np.random.default_rng(0)
    S, nq, k = 3, 50, 10
    d = np.sort(rng.random((S, nq, k)).astype(np.float32), axis=2)
    ids = rng.integers(0, 1 << 40, (S, nq, k)).astype(np.uint64)
    n = np.full((S, nq), k, np.int32)
    n[1, :10] = 3
    dev = torch.device("cuda:0")
    td = torch.from_numpy(d).to(dev)
    ti = torch.from_numpy(ids.view(np.int64)).to(dev)
    tn = torch.from_numpy(n).to(dev)
    od = torch.empty((nq, k), dtype=torch.float32, device=dev)
    oi = torch.empty((nq, k), dtype=torch.int64, device=dev)
    on = torch.empty(nq, dtype=torch.int32, device=dev)
    W.merge_shards_device(td.data_ptr(), ti.data_ptr(), tn.data_ptr(), S, nq, k, od.data_ptr(), oi.data_ptr(),
                          on.data_ptr())
    torch.cuda.synchronize()
    for q in range(nq):
        cand = sorted((float(d[s, q, j]), int(ids[s, q, j])) for s in range(S) for j in range(n[s, q]))[:k]
        assert [c[1] for c in cand] == oi[q].cpu().numpy().view(np.uint64).tolist()


@pytest.mark.parametrize("sel", [0.01, 0.10, 0.50])
def test_c4_shape_dot_768_allow_list_sharded(sel):
    """BASELINE configs[3] scaled down: 768-d dot with a shared allow list at
    1/10/50% selectivity, the corpus split into two id-range shards (id_base)
    whose per-shard top-k are merged on the device -- identical to one flat
    search of the whole corpus (flat_search.go:19-74, index.go:967-1044)."""
    import torch
    n, d, nq, k = 12000, 768, 40, 10
    rng = np.random.default_rng(int(sel * 100))
    base = (rng.standard_normal((n, d)) / np.sqrt(d)).astype(np.float32)
    qs = (rng.standard_normal((nq, d)) / np.sqrt(d)).astype(np.float32)
    allow_ids = np.nonzero(rng.random(n) < sel)[0]
    al = W.AllowList.from_ids(allow_ids, n)
    oi, od, on = O.flat_scan(O.DOT, base, qs, k, allow_bits=al.words)
    # one index over everything
    ix = W.GPUVectorIndex(d, "dot", capacity=n)
    ix.upload_vectors(base)
    ids, ds, cnt = ix.search_batch(qs, k, allow=al, mode="exact")
    _same(ids, ds, oi, od)
    ix.close()
    # two shards (global ids = id_base + local), allow list sliced per shard
    dev = torch.device("cuda:0")
    parts = []
    for lo, hi in ((0, n // 2), (n // 2, n)):
        sh = W.GPUVectorIndex(d, "dot", capacity=hi - lo, id_base=lo)
        sh.upload_vectors(base[lo:hi])
        sal = W.AllowList.from_ids(allow_ids[(allow_ids >= lo) & (allow_ids < hi)] - lo, hi - lo)
        parts.append(sh.search_batch(qs, k, allow=sal, mode="exact"))
        sh.close()
    g_i = torch.from_numpy(np.stack([p[0] for p in parts]).view(np.int64)).to(dev)
    g_d = torch.from_numpy(np.stack([p[1] for p in parts])).to(dev)
    g_n = torch.from_numpy(np.stack([p[2] for p in parts])).to(dev)
    m_d = torch.empty((nq, k), dtype=torch.float32, device=dev)
    m_i = torch.empty((nq, k), dtype=torch.int64, device=dev)
    m_n = torch.empty(nq, dtype=torch.int32, device=dev)
    W.merge_shards_device(g_d.data_ptr(), g_i.data_ptr(), g_n.data_ptr(), 2, nq, k, m_d.data_ptr(), m_i.data_ptr(),
                          m_n.data_ptr())
    torch.cuda.synchronize()
    assert m_n.cpu().tolist() == on.tolist()
    _same(m_i.cpu().numpy().view(np.uint64), m_d.cpu().numpy(), oi, od)


def test_batcher_concurrent_single_queries_equal_direct_calls():
    """SearchByVector from many threads (index.go:988-1028 fan-out): the native
    micro-batcher coalesces the calls and every caller gets exactly the row a
    direct wv_search_by_vector call returns -- unfiltered and filtered, mixed k."""
    import threading
    n, d = 20000, 64
    base, qs = _data(n, d, 96, seed=12)
    rng = np.random.default_rng(13)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    ix.upload_vectors(base)
    allows = [None if i % 3 else W.AllowList.from_ids(np.nonzero(rng.random(n) < 0.3)[0], n) for i in range(len(qs))]
    ks = [10 if i % 2 else 5 for i in range(len(qs))]
    want = [ix.search_by_vector(qs[i], ks[i], allow=allows[i]) for i in range(len(qs))]
    b = W.Batcher(ix, max_batch=64, max_wait_us=2000)
    got = [None] * len(qs)

    def worker(t):
        for i in range(t, len(qs), 8):
            got[i] = b.search(qs[i], ks[i], allow=allows[i])

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    st = b.stats()
    # the AllowList as ascending ids (wv_batcher_search_ids): per-query lists,
    # and one list shared by every caller (sent once per batch), from 8
    # threads against the two workers
    shared = np.nonzero(rng.random(n) < 0.2)[0].astype(np.uint64)
    want_sh = [ix.search_by_vector(qs[i], 10, allow=W.AllowList.from_ids(shared, n)) for i in range(len(qs))]
    got_ids, got_sh = [None] * len(qs), [None] * len(qs)

    def worker_ids(t):
        for i in range(t, len(qs), 8):
            a = allows[i]
            got_ids[i] = b.search_ids(qs[i], ks[i], None if a is None else np.nonzero(
                np.unpackbits(a.words.view(np.uint8), bitorder="little")[:n])[0].astype(np.uint64))
            got_sh[i] = b.search_ids(qs[i], 10, shared)

    th = [threading.Thread(target=worker_ids, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    # an empty list allows nothing
    e_ids, e_d = b.search_ids(qs[0], 10, np.zeros(0, np.uint64))
    b.close()
    ix.close()
    for i in range(len(qs)):
        _same(got[i][0], got[i][1], want[i][0], want[i][1])
        _same(got_ids[i][0], got_ids[i][1], want[i][0], want[i][1])
        _same(got_sh[i][0], got_sh[i][1], want_sh[i][0], want_sh[i][1])
    assert len(e_ids) == 0
    assert st["requests"] == len(qs) and st["batches"] < len(qs), st


def test_hnsw_large_batch_parity_modulo_ties():
    """At scale fp32 distances tie (tens of thousands of evaluations per
    query): the reference then decides by heap layout, the GPU by (dist, id).
    Every query must be identical up to the order among equal distances,
    unless the restatement itself took a decision between equal distances
    (counted by the oracle); and the lossy LDS visited cache must never change
    a result, whatever its size."""
    import os
    n, d, nq, ef = 50000, 64, 4000, 64
    rng = np.random.default_rng(31)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((nq, d), dtype=np.float32)
    ref = O.Index(d, "l2-squared", 32, 64, capacity=n, seed=5)
    ref.add_batch(base, threads=8)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n, max_connections=32)
    ix.upload_vectors(base)
    ix.upload_graph(ref.export_graph())
    gi, gd, gn = ix.search_batch(qs, 10, ef=ef, mode="hnsw")
    oi, od, on, _ = ref.search_batch(qs, 10, ef, threads=8)
    unexplained = []
    for i in range(nq):
        try:
            _same_tie_aware(gi[i], gd[i], oi[i], od[i])
        except AssertionError:
            if ref.knn_search(qs[i], 10, ef, with_stats=True)[2]["ties"] == 0:
                unexplained.append(i)
    assert not unexplained, unexplained[:10]
    for kb in ("6", "32"):
        os.environ["WV_HNSW_WAVE_KB"] = kb
        try:
            hi, hd, _ = ix.search_batch(qs, 10, ef=ef, mode="hnsw")
        finally:
            os.environ.pop("WV_HNSW_WAVE_KB")
        assert (hi == gi).all() and np.array_equal(hd.view(np.uint32), gd.view(np.uint32))
    ix.close()


def test_graph_replayed_from_commit_log_serves_identical_searches():
    """a shard's persisted commit log (written by the
    restatement exactly where insert.go / neighbor_connections.go write it)
    replayed into the GPU index answers like the in-memory index, tombstones
    included."""
    n, d = 5000, 32
    rng = np.random.default_rng(41)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((200, d), dtype=np.float32)
    ref = O.Index(d, "l2-squared", 16, 64, capacity=n, seed=9)
    ref.enable_commit_log()
    ref.add_batch(base, threads=1)
    tomb = np.nonzero(rng.random(n) < 0.02)[0]
    for t in tomb:
        ref.add_tombstone(int(t))
    g = W.CommitLogGraph(ref.commit_log())
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n, max_connections=16)
    ix.upload_vectors(base)
    ix.upload_graph_from_commitlog(g)
    ids, ds, cnt = ix.search_batch(qs, 10, ef=64, mode="hnsw")
    oi, od, on, _ = ref.search_batch(qs, 10, 64)
    assert not set(ids.ravel().tolist()) & set(tomb.tolist())
    _same(ids, ds, oi, od)
    ix.close()


def test_commit_log_node_above_entrypoint_level_keeps_upper_layout():
    """A log whose highest node level exceeds the entrypoint's max level (an
    AddNode above the top with its SetEntryPointWithMaxLayer torn off,
    insert.go:206): the exported CSR's level stride (max node level) differs
    from max_level, and the upload must re-lay it so every upper list is read
    at the right offset -- searches equal those over the in-memory graph."""
    import struct
    n, d = 3000, 16
    rng = np.random.default_rng(43)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((100, d), dtype=np.float32)
    ref = O.Index(d, "l2-squared", 8, 32, capacity=n, seed=3)
    ref.enable_commit_log()
    ref.add_batch(base, threads=1)
    top = ref.export_graph()["max_level"]
    assert top >= 1
    torn = struct.pack("<BQH", 0, n, top + 2)          # AddNode(n, top + 2), no SetEntryPoint after it
    g = W.CommitLogGraph(ref.commit_log() + torn)
    assert g.info()["max_node_level"] == top + 2 and g.info()["max_level"] == top
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n + 1, max_connections=8)
    ix.upload_vectors(base)
    ix.upload_graph_from_commitlog(g)
    ids, ds, _ = ix.search_batch(qs, 10, ef=32, mode="hnsw")
    oi, od, on, _ = ref.search_batch(qs, 10, 32)
    _same(ids, ds, oi, od)
    ix.close()


def test_add_with_repeated_ids_keeps_the_last_row():
    """hnsw.Add applies writes one after another (insert.go:43-65): a batch
    that repeats an id stores its last row (and that row's |x|^2, which the
    exact path's certificate relies on)."""
    n, d = 2000, 32
    rng = np.random.default_rng(44)
    base = rng.random((n, d), dtype=np.float32)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    ix.upload_vectors(base[:1000])
    ids = np.array([1000 + (i % 50) for i in range(200)], np.uint64)     # every id four times
    rows = rng.random((200, d), dtype=np.float32)
    ix.add(ids, rows)
    final = base.copy()
    for i, r in zip(ids.tolist(), rows):
        final[i] = r
    qs = rows[150:] + np.float32(1e-3)                                  # near the last writes
    gi, gd, _ = ix.search_batch(qs, 10, mode="exact")
    oi, od, _ = O.flat_scan(O.L2, final[:1050], qs, 10)
    _same(gi, gd, oi, od)
    ix.close()


def test_allow_list_compaction_equals_masking():
    """A shared allow list under half the corpus is compacted into a row list
    (contraction over |allow| rows); the masked full scan must agree bit for
    bit, with tombstones on top."""
    import os
    n, d = 30000, 96
    base, qs = _data(n, d, 150, seed=17)
    rng = np.random.default_rng(18)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    ix.upload_vectors(base)
    ix.set_tombstones(np.nonzero(rng.random(n) < 0.05)[0])
    for sel in (0.001, 0.03, 0.3):
        al = W.AllowList.from_ids(np.nonzero(rng.random(n) < sel)[0], n)
        a = ix.search_batch(qs, 10, allow=al, mode="exact")
        os.environ["WV_BF_NO_COMPACT"] = "1"
        try:
            b = ix.search_batch(qs, 10, allow=al, mode="exact")
        finally:
            os.environ.pop("WV_BF_NO_COMPACT")
        assert a[2].tolist() == b[2].tolist()
        for i in range(len(qs)):
            _same(a[0][i, : a[2][i]], a[1][i, : a[2][i]], b[0][i, : b[2][i]], b[1][i, : b[2][i]])
    empty = W.AllowList(nbits=n)
    assert (ix.search_batch(qs, 10, allow=empty, mode="exact")[2] == 0).all()
    ix.close()


@pytest.mark.parametrize("dim", [7, 33, 100, 130, 200])
@pytest.mark.parametrize("metric", [O.L2, O.COSINE])
def test_bruteforce_mfma_ragged_dims(dim, metric):
    """D not a multiple of the 32-float k-chunk: padded corpus stride, k test
    in the tile loads, zero k-groups of the last chunk skipped -- still the
    reference's ids and distances (GloVe-100-shaped: D=100, cosine)."""
    rng = np.random.default_rng(dim)
    base = rng.standard_normal((12000, dim)).astype(np.float32)
    qs = rng.standard_normal((200, dim)).astype(np.float32)
    ix = W.GPUVectorIndex(dim, METRIC_NAMES[metric], capacity=12000)
    ix.upload_vectors(base)
    ids, ds, n = ix.search_batch(qs, 10, mode="exact")
    b = O.normalize_rows(base) if metric == O.COSINE else base
    q = O.normalize_rows(qs) if metric == O.COSINE else qs
    oi, od, on = O.flat_scan(metric, b, q, 10)
    for i in range(len(qs)):
        _same_tie_aware(ids[i], ds[i], oi[i], od[i])
    ix.close()


def _merge_topk(a_ids, a_d, b_ids, b_d, k):
    out_i, out_d = [], []
    for ai, ad, bi, bd in zip(a_ids, a_d, b_ids, b_d):
        c = sorted(list(zip(ad.tolist(), ai.tolist())) + list(zip(bd.tolist(), bi.tolist())))[:k]
        out_d.append([x[0] for x in c])
        out_i.append([x[1] for x in c])
    return np.array(out_i, np.uint64), np.array(out_d, np.float32)


def test_mutable_index_added_rows_are_searchable_until_the_next_snapshot():
    """rows added after the graph snapshot (hnsw.Add,
    insert.go:43-65) are found at once -- HNSW over the snapshot merged with an
    exact pass over the delta -- tombstones apply to both, and a new snapshot
    that holds them empties the delta."""
    n0, n1, d, k, ef = 4000, 5000, 32, 10, 64
    rng = np.random.default_rng(51)
    base = rng.random((n1, d), dtype=np.float32)
    qs = rng.random((150, d), dtype=np.float32)
    ref = O.Index(d, "l2-squared", 16, 64, capacity=n1, seed=4)
    ref.add_batch(base[:n0], threads=4)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n1, max_connections=16)
    ix.upload_vectors(base[:n0])
    ix.upload_graph(ref.export_graph())
    g_old = ref.search_batch(qs, k, ef)          # the snapshot's own answer
    ix.add(np.arange(n0, n1), base[n0:])
    assert ix.delta_size() == n1 - n0
    ids, ds, cnt = ix.search_batch(qs, k, ef=ef, mode="hnsw")
    fi, fd, fn = O.flat_scan(O.L2, base[n0:], qs, k)
    want_i, want_d = _merge_topk(g_old[0], g_old[1], fi + np.uint64(n0), fd, k)
    _same(ids, ds, want_i, want_d)
    # exact mode covers every row with a vector
    ei, ed, en = ix.search_batch(qs, k, mode="exact")
    oi, od, on = O.flat_scan(O.L2, base, qs, k)
    _same(ei, ed, oi, od)
    # tombstones on old and added rows
    dead = np.concatenate([want_i[:5, 0], want_i[5:10, 1]]).astype(np.uint64)
    ix.add_tombstones(dead)
    ids2, _, _ = ix.search_batch(qs, k, ef=ef, mode="hnsw")
    assert not set(ids2.ravel().tolist()) & set(dead.tolist())
    ix.remove_tombstones(dead)
    # a snapshot holding the added rows empties the delta
    for i in range(n0, n1):
        ref.add(i, base[i])
    ix.upload_graph(ref.export_graph())
    assert ix.delta_size() == 0
    ids3, ds3, _ = ix.search_batch(qs, k, ef=ef, mode="hnsw")
    ri, rd, rn, _ = ref.search_batch(qs, k, ef)
    _same(ids3, ds3, ri, rd)
    ix.close()


def test_index_reserve_grows_in_place():
    """wv_index_reserve (growIndexToAccomodateNode, maintainance.go:31-100):
    rows, f16 images, tombstones and the graph survive the growth; rows added
    past the old capacity are found at once (delta), exact search over every
    row equals the restatement's."""
    n0, n1, d, k, ef = 3000, 7000, 64, 10, 64
    rng = np.random.default_rng(57)
    base = rng.random((n1, d), dtype=np.float32)
    qs = rng.random((200, d), dtype=np.float32)
    ref = O.Index(d, "l2-squared", 16, 64, capacity=n1, seed=8)
    ref.add_batch(base[:n0], threads=4)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n0, max_connections=16)
    ix.upload_vectors(base[:n0])
    ix.upload_graph(ref.export_graph())
    dead = np.arange(5, 400, 7, dtype=np.uint64)
    ix.add_tombstones(dead)
    h0 = ix.search_batch(qs, k, ef=ef, mode="hnsw")
    ix.reserve(n1)
    assert ix.capacity_info() == (n1, n0)
    h1 = ix.search_batch(qs, k, ef=ef, mode="hnsw")
    _same(h1[0], h1[1], h0[0], h0[1])
    ix.add(np.arange(n0, n1), base[n0:])
    assert ix.delta_size() == n1 - n0
    ei, ed, en = ix.search_batch(qs, k, mode="exact")
    allow = np.ones(n1, bool)
    allow[dead.astype(np.int64)] = False
    sel = np.nonzero(allow)[0]
    oi, od, on = O.flat_scan(O.L2, base[sel], qs, k)
    _same(ei, ed, sel[oi.astype(np.int64)].astype(np.uint64), od)
    ix.close()


def test_mutable_index_delta_with_per_query_allow_lists():
    n0, n1, d, k = 3000, 3600, 24, 10
    rng = np.random.default_rng(52)
    base = rng.random((n1, d), dtype=np.float32)
    qs = rng.random((64, d), dtype=np.float32)
    ref = O.Index(d, "l2-squared", 16, 64, capacity=n1, seed=6)
    ref.add_batch(base[:n0], threads=4)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n1, max_connections=16, forbid_flat=True)
    ix.upload_vectors(base[:n0])
    ix.upload_graph(ref.export_graph())
    ix.add(np.arange(n0, n1), base[n0:])
    per = [W.AllowList.from_ids(np.nonzero(rng.random(n1) < 0.5)[0], n1) for _ in range(len(qs))]
    ids, ds, cnt = ix.search_batch(qs, k, ef=64, allow=per, mode="hnsw")
    for i in range(len(qs)):
        gi, gd, _, _ = ref.search_batch(qs[i:i + 1], k, 64, allow=per[i].words)
        fi, fd, fn = O.flat_scan(O.L2, base[n0:], qs[i:i + 1], k, allow_bits=per[i].words[n0 // 64:] if n0 % 64 == 0
                                 else None)
        sel = np.array([j for j in range(n0, n1) if per[i].contains(j)], np.int64)
        fi, fd, fn = O.flat_scan(O.L2, base[sel], qs[i:i + 1], k)
        wi, wd = _merge_topk(gi, gd, sel[fi.astype(np.int64)].astype(np.uint64), fd, k)
        _same(ids[i, : cnt[i]], ds[i, : cnt[i]], wi[0], wd[0])
    ix.close()


def _recall(ids, truth, k=10):
    return float(np.mean([len(set(a[:k]) & set(b[:k])) / k for a, b in zip(ids.tolist(), truth.tolist())]))


def test_gpu_graph_build_invariants_and_recall():
    """the graph built on the GPU (insert.go's algorithm in
    batches) keeps the reference's invariants -- layer-0 degree <= 2M, upper
    <= M (index_too_many_links_bug_integration_test.go:127-143), valid ids, no
    self links, the entrypoint on the top level -- reaches the recall of the
    restatement's sequential build within 0.5 points, and the restatement
    searching the GPU-built graph answers exactly like the GPU does."""
    n, d, M, efc, ef = 20000, 32, 16, 64, 64
    rng = np.random.default_rng(61)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((1000, d), dtype=np.float32)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n, max_connections=M)
    ix.upload_vectors(base)
    ix.build_graph(ef_construction=efc, seed=7, batch_div=32)
    g = ix.download_graph()
    l0, lv = g["layer0"], g["levels"]
    assert g["deg0"] == 2 * M and g["degU"] == M
    valid = l0 != 0xFFFFFFFF
    assert (l0[valid] < n).all()
    assert not (l0 == np.arange(n, dtype=np.uint32)[:, None]).any()
    assert (valid.sum(1) > 0).all()                      # every node reachable from somewhere has links
    assert lv[g["entrypoint"]] == g["max_level"] == lv.max()
    up = g["upper"]
    assert ((up != 0xFFFFFFFF).sum(2) <= M).all()
    truth, _, _ = O.flat_scan(O.L2, base, qs, 10)
    gi, gd, gn = ix.search_batch(qs, 10, ef=ef, mode="hnsw")
    ref = O.Index(d, "l2-squared", M, efc, capacity=n, seed=7)
    ref.add_batch(base, threads=8)
    assert np.array_equal(ref.export_graph()["levels"][1:], lv[1:])   # same level draw (insert.go:132)
    oi, od, on, _ = ref.search_batch(qs, 10, ef, threads=8)
    r_gpu, r_cpu = _recall(gi, truth), _recall(oi, truth)
    # north_star: HNSW recall within 0.5 pt of the reference index on the same data and ef
    assert r_gpu >= r_cpu - 0.005, (r_gpu, r_cpu)
    # the restatement on the GPU-built graph == the GPU on it
    ref2 = O.Index(d, "l2-squared", M, efc, capacity=n, seed=7)
    ref2.import_graph(base, g)
    ri, rd, rn, _ = ref2.search_batch(qs, 10, ef, threads=8)
    for i in range(len(qs)):
        _same_tie_aware(gi[i], gd[i], ri[i], rd[i])
    ix.close()


@pytest.mark.parametrize("metric", [O.L2, O.DOT, O.COSINE])
def test_split_key_pass_equals_fp32_key_pass(metric):
    """The f16 key pass (default), the bf16x3 pass (WV_BF_SPLIT=1) and the fp32
    MFMA key pass (WV_BF_FP32=1) only rank candidates; all re-rank in the
    reference's order, so ids and distances agree bit for bit -- also on
    wide-range data (|x| from 0.02 to 8e3), where the f16 scaling and the
    error bound of the certificate are stretched most."""
    import os
    rng = np.random.default_rng(31 + metric)
    n, d = 15000, 128
    scale = np.exp(rng.uniform(-4, 9, (n, 1))).astype(np.float32)
    base = (rng.standard_normal((n, d)) * scale).astype(np.float32)
    qs = (rng.standard_normal((120, d)) * 30).astype(np.float32)
    out = []
    for env in ({}, {"WV_BF_SPLIT": "1"}, {"WV_BF_FP32": "1"}):
        os.environ.update(env)
        try:
            ix = W.GPUVectorIndex(d, METRIC_NAMES[metric], capacity=n)
        finally:
            for key in env:
                os.environ.pop(key, None)
        ix.upload_vectors(base)
        out.append(ix.search_batch(qs, 10, mode="exact"))
        ix.close()
    (ai, ad, an) = out[0]
    for (bi, bd, bn) in out[1:]:
        assert an.tolist() == bn.tolist()
        _same(ai, ad, bi, bd)
    b = O.normalize_rows(base) if metric == O.COSINE else base
    q = O.normalize_rows(qs) if metric == O.COSINE else qs
    oi, od, on = O.flat_scan(metric, b, q, 10)
    for i in range(len(qs)):
        _same_tie_aware(ai[i], ad[i], oi[i], od[i])


@pytest.mark.parametrize("dim", [32, 96, 128])
@pytest.mark.parametrize("metric", [O.L2, O.DOT, O.COSINE])
def test_split_pass_query_blocks_multi_segment(dim, metric):
    """The split key pass (WV_BF_SPLIT=1: 256-query blocks, one 512-thread
    workgroup per CU) over several query blocks
    (nq = 700: a partial last block), a ragged corpus (last tile partial),
    tombstones and a shared allow list that keeps over half the rows (masked
    in the epilogue, not compacted); D = 32 / 96 / 128 = 1 / 3 / 4 k-chunks
    (odd chunk counts take the ping-pong copy).  Both return the same ids and
    distances, equal to the restatement's (cosine rows tie at the k boundary
    on this data: the reference orders ties by heap layout)."""
    import os
    n = 20011
    base, qs = _data(n, dim, 700, seed=41 + dim, metric=metric)
    rng = np.random.default_rng(42)
    tomb_ids = np.nonzero(rng.random(n) < 0.03)[0]
    allow_ids = np.nonzero(rng.random(n) < 0.7)[0]
    al = W.AllowList.from_ids(allow_ids, n)
    tb = O.bits_from_ids(tomb_ids, n)
    b = O.normalize_rows(base) if metric == O.COSINE else base
    q = O.normalize_rows(qs) if metric == O.COSINE else qs
    oi, od, on = O.flat_scan(metric, b, q, 10, allow_bits=al.words, tomb_bits=tb)
    ui, ud, un = O.flat_scan(metric, b, q, 10, tomb_bits=tb)
    runs = []
    # default (the f16 key pass), and the bf16x3 split pass
    for env in ({}, {"WV_BF_SPLIT": "1"}):
        os.environ.update(env)
        try:
            ix = W.GPUVectorIndex(dim, METRIC_NAMES[metric], capacity=n)
            ix.upload_vectors(base)
            ix.set_tombstones(tomb_ids)
            runs.append((ix.search_batch(qs, 10, allow=al, mode="exact"), ix.search_batch(qs, 10, mode="exact")))
            ix.close()
        finally:
            for k in env:
                os.environ.pop(k, None)
    for other in runs[1:]:
        for (ai, ad, an), (bi, bd, bn) in zip(runs[0], other):
            _same(ai, ad, bi, bd)
    for (gi, gd, gn), (ri, rd) in zip(runs[0], ((oi, od), (ui, ud))):
        for i in range(len(qs)):
            _same_tie_aware(gi[i], gd[i], ri[i], rd[i])


@pytest.mark.parametrize("dim", [100, 128])
@pytest.mark.parametrize("metric", [O.L2, O.DOT, O.COSINE])
def test_h16_key_pass_seeded_equals_unseeded_and_fp32(dim, metric):
    """The f16 key pass at a corpus size that runs the seed pre-pass (>= 64k
    rows): seeded (default), unseeded (WV_H16_NO_SEED), with the seed sampling
    every 8th / 32nd tile (WV_H16_SAMPLE), without the running threshold
    (WV_H16_NO_RUNNING) and the fp32 pass return the same ids and distances,
    with tombstones, a shared allow list kept in the epilogue and a partial
    last query block -- and equal the restatement up to tie order.  D=100 is
    GloVe-shaped (7 k-steps of 16: 112, not 128)."""
    import os
    n, nq = 70001, 600
    base, qs = _data(n, dim, nq, seed=71 + dim, metric=metric)
    rng = np.random.default_rng(72)
    tomb_ids = np.nonzero(rng.random(n) < 0.02)[0]
    allow_ids = np.nonzero(rng.random(n) < 0.6)[0]
    al = W.AllowList.from_ids(allow_ids, n)
    runs = []
    for env in ({}, {"WV_H16_NO_SEED": "1"}, {"WV_H16_SAMPLE": "8"}, {"WV_H16_SAMPLE": "32"},
                {"WV_H16_NO_SEED": "1", "WV_H16_NO_RUNNING": "1"}, {"WV_BF_FP32": "1"}):
        os.environ.update(env)
        try:
            ix = W.GPUVectorIndex(dim, METRIC_NAMES[metric], capacity=n)
            ix.upload_vectors(base)
            ix.set_tombstones(tomb_ids)
            runs.append((ix.search_batch(qs, 10, mode="exact"), ix.search_batch(qs, 10, allow=al, mode="exact"),
                         ix.last_batch_stats()["fallbacks"]))
            ix.close()
        finally:
            for key in env:
                os.environ.pop(key, None)
    for other in runs[1:]:
        for (ai, ad, an), (bi, bd, bn) in zip(runs[0][:2], other[:2]):
            assert an.tolist() == bn.tolist()
            _same(ai, ad, bi, bd)
    assert runs[0][2] <= nq // 50, runs[0][2]      # the certificate holds for almost every query
    b = O.normalize_rows(base) if metric == O.COSINE else base
    q = O.normalize_rows(qs) if metric == O.COSINE else qs
    tb = O.bits_from_ids(tomb_ids, n)
    oi, od, on = O.flat_scan(metric, b, q, 10, allow_bits=al.words, tomb_bits=tb, threads=16)
    gi, gd, gn = runs[0][1]
    for i in range(nq):
        _same_tie_aware(gi[i], gd[i], oi[i], od[i])


@pytest.mark.parametrize("metric", [O.L2, O.DOT, O.COSINE])
def test_h16_seed_list_mode(metric):
    """The seed pre-pass in list mode (WV_H16_SEED_LISTS; a 10k-ish batch: 19 query blocks, the
    list pass's 13 slots x 16 entries fit the seed kernel's sort): minima over
    every 64th tile, full lists over the corpus's last 69 of 1094 tiles
    (keys above the minima thresholds dropped), the lists' 16 smallest handed
    to the finalize as one more slot and the main pass over the other 1025
    tiles.  Same ids and distances as minima mode (the default), as a
    denser minima pass (WV_H16_LIST_MULT=1) and as the fp32 pass, with
    tombstones, a shared allow list and a partial last query block; equal to
    the restatement up to tie order on a sample of queries."""
    import os
    n, nq, dim = 70001, 9500, 128
    base, qs = _data(n, dim, nq, seed=81, metric=metric)
    rng = np.random.default_rng(82)
    tomb_ids = np.nonzero(rng.random(n) < 0.02)[0]
    allow_ids = np.nonzero(rng.random(n) < 0.6)[0]
    al = W.AllowList.from_ids(allow_ids, n)
    runs = []
    for env in ({"WV_H16_SEED_LISTS": "1"}, {}, {"WV_H16_SEED_LISTS": "1", "WV_H16_LIST_MULT": "1"},
                {"WV_BF_FP32": "1"}):
        os.environ.update(env)
        try:
            ix = W.GPUVectorIndex(dim, METRIC_NAMES[metric], capacity=n)
            ix.upload_vectors(base)
            ix.set_tombstones(tomb_ids)
            runs.append((ix.search_batch(qs, 10, mode="exact"), ix.search_batch(qs, 10, allow=al, mode="exact"),
                         ix.last_batch_stats()["fallbacks"]))
            ix.close()
        finally:
            for key in env:
                os.environ.pop(key, None)
    for other in runs[1:]:
        for (ai, ad, an), (bi, bd, bn) in zip(runs[0][:2], other[:2]):
            assert an.tolist() == bn.tolist()
            _same(ai, ad, bi, bd)
    assert runs[0][2] <= nq // 50, runs[0][2]
    b = O.normalize_rows(base) if metric == O.COSINE else base
    q = O.normalize_rows(qs) if metric == O.COSINE else qs
    tb = O.bits_from_ids(tomb_ids, n)
    sample = np.arange(0, nq, 19)
    for allow_bits, (gi, gd, gn) in ((None, runs[0][0]), (al.words, runs[0][1])):
        oi, od, on = O.flat_scan(metric, b, q[sample], 10, allow_bits=allow_bits, tomb_bits=tb, threads=16)
        for j, i in enumerate(sample):
            _same_tie_aware(gi[i], gd[i], oi[j], od[j])


def test_h16_integer_data_keys_exact():
    """SIFT-shaped integer data: f16(s_x x) is exact (integers below 2048 x
    2^k), so the residual terms of the certificate vanish and the f16 keys are
    exact -- ids equal the restatement's up to tie order, few fallbacks."""
    from bench import counter_sift
    n, d, nq = 70000, 128, 400
    base = counter_sift(1, 0, n, d)
    qs = counter_sift(2, 0, nq, d)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    ix.upload_vectors(base)
    gi, gd, gn = ix.search_batch(qs, 10, mode="exact")
    fb = ix.last_batch_stats()["fallbacks"]
    oi, od, on = O.flat_scan(O.L2, base, qs, 10, threads=16)
    for i in range(nq):
        _same_tie_aware(gi[i], gd[i], oi[i], od[i])
    assert fb <= nq // 10, fb
    ix.close()


def test_h16_cross_slot_threshold_equals_default():
    """The cross-slot threshold (default; WV_H16_XSLOT=0 turns it off) only
    rejects keys above a certified bound on the k-th key, so the results equal
    the pass without it bit for bit.  8 300 queries over 70k rows make 17 query blocks, so a
    query block has <= 16 slots (<= 32 list heads), where it engages."""
    import os
    n, d, nq = 70001, 128, 8300
    base, qs = _data(n, d, nq, seed=91)
    tomb_ids = np.nonzero(np.random.default_rng(92).random(n) < 0.01)[0]
    runs = []
    for env in ({}, {"WV_H16_XSLOT": "0"}):
        os.environ.update(env)
        try:
            ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
            ix.upload_vectors(base)
            ix.set_tombstones(tomb_ids)
            runs.append([ix.search_batch(qs, k, mode="exact") for k in (10, 32)])
            ix.close()
        finally:
            for key in env:
                os.environ.pop(key, None)
    for other in runs[1:]:
        for (ai, ad, an), (bi, bd, bn) in zip(runs[0], other):
            assert an.tolist() == bn.tolist()
            _same(ai, ad, bi, bd)
    # and the default (cross-slot threshold engaged) against the restatement
    tb = O.bits_from_ids(tomb_ids, n)
    for k, (gi, gd, gn) in zip((10, 32), runs[0]):
        oi, od, on = O.flat_scan(O.L2, base, qs, k, tomb_bits=tb, threads=16)
        assert gn.tolist() == on.tolist()
        for i in range(nq):
            _same_tie_aware(gi[i], gd[i], oi[i], od[i])


@pytest.mark.parametrize("data", ["uniform", "integer"])
def test_h16_cross_slot_threshold_without_seed_equals_restatement(data):
    """The cross-slot threshold where no seed pre-pass runs (40k rows: 625
    tiles, under the 64 x H_SAMPLE cutoff) and the running threshold is off:
    certification then rests on the list tails and on the bounds the cross
    slot exchange published to gtau (the finalize's tau_in).  17 query blocks
    (<= 16 slots each), uniform and tie-heavy integer data, k = 10 and 32:
    on == off == the restatement (tie-aware)."""
    import os
    n, d, nq = 40000, 128, 8700
    if data == "uniform":
        base, qs = _data(n, d, nq, seed=93)
    else:
        rng = np.random.default_rng(94)
        base = rng.integers(0, 4, (n, d)).astype(np.float32)
        qs = rng.integers(0, 4, (nq, d)).astype(np.float32)
    tomb_ids = np.nonzero(np.random.default_rng(95).random(n) < 0.01)[0]
    runs = []
    for env in ({}, {"WV_H16_XSLOT": "0"}):
        os.environ.update(env)
        try:
            ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
            ix.upload_vectors(base)
            ix.set_tombstones(tomb_ids)
            runs.append([ix.search_batch(qs, k, mode="exact") for k in (10, 32)])
            ix.close()
        finally:
            for key in env:
                os.environ.pop(key, None)
    tb = O.bits_from_ids(tomb_ids, n)
    for k, (a, b) in zip((10, 32), zip(runs[0], runs[1])):
        oi, od, on = O.flat_scan(O.L2, base, qs, k, tomb_bits=tb, threads=16)
        for gi, gd, gn in (a, b):
            assert gn.tolist() == on.tolist()
            for i in range(nq):
                _same_tie_aware(gi[i], gd[i], oi[i], od[i])


@pytest.mark.parametrize("metric,d,M", [(O.L2, 48, 16), (O.COSINE, 100, 64), (O.DOT, 128, 32)])
def test_hnsw_workgroup_per_query_small_batches(metric, d, M, monkeypatch):
    """Batches of up to 64 unfiltered queries run one 4-wave workgroup per
    query (wv_hnsw_wg_kernel: helper waves take rows 32..127 of each distance
    batch): identical to the restatement and, bit for bit, to the one-wave
    kernel (WV_HNSW_WG_MAX=0), at batch sizes 1, 7 and 64, ef 10 / 64 / 100 /
    200 / 256 (one, two and four result registers), M = 64 (128 neighbours per batch) and a
    D = 32 m + 4 row tail."""
    n = 4000
    base, idx = _build_graph(n, d, metric, M=M)
    qs = np.random.default_rng(77).random((64, d), dtype=np.float32)
    g = idx.export_graph()
    ix = W.GPUVectorIndex(d, METRIC_NAMES[metric], capacity=n, max_connections=M)
    ix.upload_vectors(base)
    ix.upload_graph(g)
    for ef in (10, 64, 100, 200, 256):
        oi, od, on, st = idx.search_batch(qs, 10, ef, threads=8)
        for nb in (1, 7, 64):
            q = qs[:nb]
            ids, ds, cnt = ix.search_batch(q, 10, ef=ef, mode="hnsw")
            assert cnt.tolist() == on[:nb].tolist()
            _same(ids, ds, oi[:nb], od[:nb])
            monkeypatch.setenv("WV_HNSW_WG_MAX", "0")
            ids1, ds1, cnt1 = ix.search_batch(q, 10, ef=ef, mode="hnsw")
            monkeypatch.delenv("WV_HNSW_WG_MAX")
            assert np.array_equal(ids, ids1) and np.array_equal(ds.view(np.uint32), ds1.view(np.uint32))
            assert np.array_equal(cnt, cnt1)
    ix.close()


@pytest.mark.parametrize("n", [1, 2, 40])
def test_hnsw_workgroup_launch_edge_graphs(n, monkeypatch):
    """The workgroup-per-query launch's barrier pairing (wv_hnsw.hip, above
    wg_dist) on edge shapes: a one- and two-node graph and a small one whose
    top level is 0 or 1, k = 1 and ef = 1, one and three queries -- every
    launch drains (no early return past a pending barrier) and answers as the
    one-wave kernel and the restatement do."""
    d = 32
    base, idx = _build_graph(n, d, O.L2, M=64)
    qs = np.random.default_rng(5).random((3, d), dtype=np.float32)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n, max_connections=64)
    ix.upload_vectors(base)
    ix.upload_graph(idx.export_graph())
    for k, ef in ((1, 1), (1, 10), (10, 64)):
        oi, od, on, _ = idx.search_batch(qs, k, ef, threads=2)
        for nb in (1, 3):
            ids, ds, cnt = ix.search_batch(qs[:nb], k, ef=ef, mode="hnsw")
            assert cnt.tolist() == on[:nb].tolist()
            for i in range(nb):   # (entries past a query's count are unspecified)
                c = int(cnt[i])
                _same(ids[i:i + 1, :c], ds[i:i + 1, :c], oi[i:i + 1, :c], od[i:i + 1, :c])
            monkeypatch.setenv("WV_HNSW_WG_MAX", "0")
            ids1, ds1, cnt1 = ix.search_batch(qs[:nb], k, ef=ef, mode="hnsw")
            monkeypatch.delenv("WV_HNSW_WG_MAX")
            assert np.array_equal(cnt, cnt1)
            for i in range(nb):
                assert np.array_equal(ids[i, :cnt[i]], ids1[i, :cnt[i]])
    ix.close()
