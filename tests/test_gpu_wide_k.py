"""Exact search with k > 32 on the batched MFMA path (-m gpu).

limit > 32 (flatSearch with a large limit, search.go:90-158's deepening
SearchByVectorDistance starting at limit 100) runs the f16 key pass with at
least 2k candidate lists per query and the wide finalize (one workgroup per
query: all list entries sorted in LDS, every entry within the keys' error of
the k-th re-ranked in reference order, certificate as for small k).  Results
must equal the CPU restatement's flatSearch (oracle/) -- ids and distances,
ties by id -- and almost every query must be certified on the fast path.
"""
import numpy as np
import pytest

import pyoracle as O
import weaviate_amd as W
from helpers import same_tie_aware

pytestmark = pytest.mark.gpu

NAMES = {O.L2: "l2-squared", O.DOT: "dot", O.COSINE: "cosine-dot"}


def _data(n, nq, d, seed, metric):
    rng = np.random.default_rng(seed)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((nq, d), dtype=np.float32)
    if metric == O.DOT:
        base -= 0.5
        qs -= 0.5
    return base, qs


def _check(ix, base, qs, k, metric, allow=None, max_fb_frac=0.02):
    ids, ds, n = ix.search_batch(qs, k, mode="exact", allow=allow)
    st = ix.last_batch_stats()
    b = O.normalize_rows(base) if metric == O.COSINE else base
    q = O.normalize_rows(qs) if metric == O.COSINE else qs
    oi, od, on = O.flat_scan(metric, b, q, k, allow_bits=allow.words if allow is not None else None)
    assert n.tolist() == on.tolist()
    for i in range(len(qs)):
        same_tie_aware(ids[i, : n[i]], ds[i, : n[i]], oi[i, : on[i]], od[i, : on[i]])
    assert st["fallbacks"] <= max_fb_frac * len(qs) + 1, st
    return st


@pytest.mark.parametrize("metric", [O.L2, O.DOT, O.COSINE])
@pytest.mark.parametrize("k", [33, 100, 256])
def test_wide_k_equals_restatement(metric, k):
    base, qs = _data(150_000, 600, 128, 21 + k, metric)
    ix = W.GPUVectorIndex(128, NAMES[metric], capacity=base.shape[0])
    ix.upload_vectors(base)
    _check(ix, base, qs, k, metric)
    ix.close()


@pytest.mark.parametrize("n,d", [(3000, 64), (40_000, 100), (70_001, 17)])
def test_wide_k_ragged_sizes(n, d):
    base, qs = _data(n, 777, d, n, O.L2)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    ix.upload_vectors(base)
    _check(ix, base, qs, 100, O.L2, max_fb_frac=0.05)
    ix.close()


def test_wide_k_shared_allow_list_and_tombstones():
    n, d = 120_000, 128
    base, qs = _data(n, 500, d, 5, O.L2)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    ix.upload_vectors(base)
    rng = np.random.default_rng(8)
    allow = W.AllowList.from_ids(rng.choice(n, n // 2, replace=False), n)
    dead = rng.choice(n, 5000, replace=False)
    ix.add_tombstones(dead)
    ids, ds, cnt = ix.search_batch(qs, 120, mode="exact", allow=allow)
    keep = np.zeros(n, bool)
    keep[np.asarray(list(allow.iterator()), dtype=np.int64)] = True
    keep[dead] = False
    oi, od, on = O.flat_scan(O.L2, base, qs, 120, allow_bits=O.bits_from_ids(np.nonzero(keep)[0], n))
    for i in range(len(qs)):
        same_tie_aware(ids[i, : cnt[i]], ds[i, : cnt[i]], oi[i, : on[i]], od[i, : on[i]])
    assert not np.isin(ids, dead).any()
    ix.close()


def test_wide_k_integer_data_ties_and_beyond_the_wide_limit():
    """SIFT-like integer data (ties between distances: ordered by id) and a k
    past BF_WIDE_KMAX (the exact-scan path) both equal the restatement."""
    rng = np.random.default_rng(3)
    n, d = 30_000, 32
    base = rng.integers(0, 4, (n, d)).astype(np.float32)
    qs = rng.integers(0, 4, (200, d)).astype(np.float32)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    ix.upload_vectors(base)
    for k in (64, 300):
        ids, ds, cnt = ix.search_batch(qs, k, mode="exact")
        oi, od, on = O.flat_scan(O.L2, base, qs, k)
        for i in range(len(qs)):
            # the reference orders equal distances by heap layout:
            # equal up to that order, and ours is (dist, id) -- the smallest
            # ids among the rows at the boundary distance
            same_tie_aware(ids[i], ds[i], oi[i], od[i])
            full = ((base.astype(np.float64) - qs[i].astype(np.float64)) ** 2).sum(1)   # exact: integers
            order = np.lexsort((np.arange(n), full))[:k]
            assert ids[i].tolist() == order.tolist()
    ix.close()


def test_search_by_vector_distance_deepening_on_the_wide_path():
    """SearchByVectorDistance (search.go:90-158) starts at limit 100 and
    deepens; on a flat index every round is an exact search."""
    n, d = 100_000, 64
    base, qs = _data(n, 5, d, 9, O.L2)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n, flat_search_cutoff=10**9)
    ix.upload_vectors(base)
    ref = O.Index(d, "l2-squared", 16, 64, capacity=n)
    # every row a level-0 node without links (flatSearch skips nil nodes,
    # flat_search.go:35-39; the flat path needs no edges)
    nil = np.uint32(0xFFFFFFFF)
    ref.import_graph(base, dict(n=n, entrypoint=0, max_level=0, levels=np.zeros(n, np.int8),
                                layer0=np.full((n, 1), nil, np.uint32), upper_row=np.full(n, nil, np.uint32),
                                upper=np.zeros((1, 1, 1), np.uint32)))
    ref.set_search_config(flat_search_cutoff=10**9)
    allow = W.AllowList.from_ids(np.arange(n), n)   # below the cutoff: flatSearch (exact)
    for q in qs:
        d_all = ((base - q) ** 2).sum(1)
        target = float(np.sort(d_all)[150])   # ~150 rows within: two deepening rounds
        gi, gd = ix.search_by_vector_distance(q, target, -1, allow=allow)
        oi, od = ref.search_by_vector_distance(q, target, -1, allow=O.bits_from_ids(np.arange(n), n))
        assert gi.tolist() == oi.tolist()
        assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))
    ix.close()


def _single_calls(ix, qs, targets, max_limit, allows, cap):
    out = []
    for i, q in enumerate(qs):
        a = allows[i] if isinstance(allows, list) else allows
        out.append(ix.search_by_vector_distance(q, float(targets[i]), max_limit, allow=a, cap=cap))
    return out


def _assert_same(batch, single, n, cap):
    for i, ((bi, bd), (si, sd)) in enumerate(zip(batch, single)):
        assert bi.tolist() == si.tolist(), i
        assert np.array_equal(bd.view(np.uint32), sd.view(np.uint32)), i


@pytest.mark.parametrize("metric", [O.L2, O.DOT, O.COSINE])
def test_search_by_vector_distance_batch_equals_single_calls(metric):
    """wv_search_by_vector_distance_batch (round 1 the batch's SearchByVector
    where it is an HNSW search, every exact round one threshold pass +
    segmented sort on the device) answers each query as the single-query
    deepening (search.go:90-158: limits 100, 1100, 11100 ...) does, bit for
    bit: HNSW and flat round 1, targets that stop in round 1, 2 or 3, a
    shared and per-query allow lists, maxLimit, results past the caller's
    cap counted but not written."""
    n, d, nq = 30_000, 32, 24
    base, qs = _data(n, nq, d, 31, metric)
    idx = O.Index(d, metric, 16, 64, capacity=n, seed=3)
    idx.add_batch(base, threads=8)
    ix = W.GPUVectorIndex(d, NAMES[metric], capacity=n, max_connections=16)
    ix.upload_vectors(base)
    ix.upload_graph(idx.export_graph())
    b = O.normalize_rows(base) if metric == O.COSINE else base
    q = O.normalize_rows(qs) if metric == O.COSINE else qs
    full = np.sort(O.flat_scan(metric, b, q, 3000)[1], axis=1)
    ranks = [20, 99, 100, 150, 1099, 1500, 2500]
    targets = np.array([full[i, ranks[i % len(ranks)]] for i in range(nq)], np.float32)
    rng = np.random.default_rng(4)
    shared = W.AllowList.from_ids(np.nonzero(rng.random(n) < 0.5)[0], n)   # 15k >= cutoff: HNSW round 1
    small = W.AllowList.from_ids(np.nonzero(rng.random(n) < 0.2)[0], n)    # 6k < cutoff 40k: flat
    per_q = [shared if i % 2 else small for i in range(nq)]
    for allow in (None, shared, small, per_q):
        for max_limit in (-1, 150, 1100, 5000):
            for cap in (4096, 120):
                got, cnt = ix.search_by_vector_distance_batch(qs, targets, max_limit, allow=allow, cap=cap)
                want = _single_calls(ix, qs, targets, max_limit, allow, cap)
                _assert_same(got, want, cnt, cap)
    ix.close()


def test_search_by_vector_distance_batch_flat_index_equals_restatement():
    """The flat (graph-less) index: every round exact; the batch equals the
    restatement's SearchByVectorDistance (oracle/) on each query, up to the
    order among equal distances."""
    n, d = 100_000, 64
    base, qs = _data(n, 6, d, 9, O.L2)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n, flat_search_cutoff=10**9)
    ix.upload_vectors(base)
    ref = O.Index(d, "l2-squared", 16, 64, capacity=n)
    nil = np.uint32(0xFFFFFFFF)
    ref.import_graph(base, dict(n=n, entrypoint=0, max_level=0, levels=np.zeros(n, np.int8),
                                layer0=np.full((n, 1), nil, np.uint32), upper_row=np.full(n, nil, np.uint32),
                                upper=np.zeros((1, 1, 1), np.uint32)))
    ref.set_search_config(flat_search_cutoff=10**9)
    allow = W.AllowList.from_ids(np.arange(n), n)
    targets = [float(np.sort(((base - q) ** 2).sum(1))[r]) for q, r in zip(qs, (5, 99, 150, 1200, 3000, 40))]
    got, cnt = ix.search_by_vector_distance_batch(qs, targets, -1, allow=allow, cap=8192)
    for i, q in enumerate(qs):
        oi, od = ref.search_by_vector_distance(q, targets[i], -1, allow=O.bits_from_ids(np.arange(n), n))
        # (equal distances: the restatement's heap order vs (dist, id))
        same_tie_aware(got[i][0], got[i][1], oi, od)
        assert cnt[i] == len(oi)
    ix.close()
