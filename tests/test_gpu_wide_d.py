"""The f16 key pass for D > 128 (wv_bf_h16w_kernel, -m gpu).

Both operands stream through LDS in 64-k chunks; the epilogue and the
certificate are those of the D <= 128 pass.  Exact results must equal the CPU
restatement's flatSearch (oracle/) bit for bit (ties by id), at the C4 shape
(768-d dot product, BASELINE configs[3]) and at ragged D, with shared allow
lists, tombstones, k > 32 and corpora that end inside a 128-row tile.
"""
import numpy as np
import pytest

import pyoracle as O
import weaviate_amd as W
from helpers import same_tie_aware

pytestmark = pytest.mark.gpu
NAMES = {O.L2: "l2-squared", O.DOT: "dot", O.COSINE: "cosine-dot"}


def _gauss(n, d, seed):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((n, d)) / np.sqrt(d)).astype(np.float32)


def _check(ix, base, qs, k, metric, allow_bits=None, allow=None, tomb=None):
    ids, ds, n = ix.search_batch(qs, k, mode="exact", allow=allow)
    b = O.normalize_rows(base) if metric == O.COSINE else base
    q = O.normalize_rows(qs) if metric == O.COSINE else qs
    oi, od, on = O.flat_scan(metric, b, q, k, allow_bits=allow_bits, tomb_bits=tomb)
    assert n.tolist() == on.tolist()
    for i in range(len(qs)):
        same_tie_aware(ids[i, : n[i]], ds[i, : n[i]], oi[i, : on[i]], od[i, : on[i]])
    return ix.last_batch_stats()


@pytest.mark.parametrize("metric", [O.DOT, O.L2, O.COSINE])
def test_c4_shape_768_equals_restatement(metric):
    n, d = 60_000, 768
    base, qs = _gauss(n, d, 1), _gauss(700, d, 2)
    ix = W.GPUVectorIndex(d, NAMES[metric], capacity=n)
    ix.upload_vectors(base)
    st = _check(ix, base, qs, 10, metric)
    assert st["fallbacks"] <= 7, st   # the f16 keys certify (nearly) every query
    ix.close()


@pytest.mark.parametrize("d", [129, 200, 256, 300, 1000])
def test_ragged_wide_dims(d):
    n = 20_001   # ends inside a 128-row tile
    rng = np.random.default_rng(d)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((300, d), dtype=np.float32)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    ix.upload_vectors(base)
    _check(ix, base, qs, 10, O.L2)
    ix.close()


def test_wide_d_allow_list_tombstones_and_large_k():
    n, d = 40_000, 768
    base, qs = _gauss(n, d, 3), _gauss(300, d, 4)
    ix = W.GPUVectorIndex(d, "dot", capacity=n)
    ix.upload_vectors(base)
    rng = np.random.default_rng(5)
    dead = rng.choice(n, 2000, replace=False)
    ix.add_tombstones(dead)
    tomb = O.bits_from_ids(dead, n)
    # 50 %: the whole-corpus pass with the allow mask in the epilogue
    ids_a = np.nonzero(rng.random(n) < 0.5)[0]
    al = W.AllowList.from_ids(ids_a, n)
    _check(ix, base, qs, 10, O.DOT, allow_bits=al.words, allow=al, tomb=tomb)
    for k in (64, 200):
        _check(ix, base, qs, k, O.DOT, tomb=tomb)
    ix.close()


@pytest.mark.parametrize("d,metric", [(768, O.DOT), (128, O.L2), (100, O.COSINE)])
def test_gathered_allow_list_pass_equals_restatement(d, metric):
    """A shared allow list keeping under half the corpus: the f16 key pass
    runs over an image of just the allowed rows (gathered on the device, ids
    mapped back through the ascending row list before the re-rank) --
    flatSearch's walk over the allow list (flat_search.go:25-58) at the f16
    rate (configs[3]'s 1 / 10 % legs).  Bit-identical to the restatement, with
    tombstones inside the list, k up to 200, a list that ends inside a tile."""
    n = 50_001
    base, qs = _gauss(n, d, 7), _gauss(400, d, 8)
    ix = W.GPUVectorIndex(d, NAMES[metric], capacity=n)
    ix.upload_vectors(base)
    rng = np.random.default_rng(9)
    dead = rng.choice(n, 1500, replace=False)
    ix.add_tombstones(dead)
    tomb = O.bits_from_ids(dead, n)
    for frac in (0.01, 0.1, 0.4):
        ids_a = np.nonzero(rng.random(n) < frac)[0]
        al = W.AllowList.from_ids(ids_a, n)
        for k in ((10, 64) if frac != 0.01 else (10, 200)):
            st = _check(ix, base, qs, k, metric, allow_bits=al.words, allow=al, tomb=tomb)
            # (k = 200 over ~500 rows: a handful of tiles cannot hold lists
            # that certify 200 -- the device fallback answers, still exact)
            if k <= 64:
                assert st["fallbacks"] <= len(qs) // 50, (frac, k, st)
    ix.close()


@pytest.mark.parametrize("metric", [O.L2, O.DOT])
def test_device_counted_compaction_edge_lists(metric, monkeypatch):
    """The wide-D pass compacts a shared allow list without reading its
    length back (compact_allowed_dev + H16Params.n_dev: the kernel sizes its
    slots' tile runs from the device count).  Equal to the restatement and to
    the read-back path (WV_BF_SYNC_COMPACT=1) bit for bit over the edges: an
    empty list, a list of tombstoned rows only (length 0 on the device), one
    row, every row, a list shorter than the corpus's bitmap, and a
    single-query batch (one query block, 256 slots)."""
    n, d = 30_001, 256
    base, qs = _gauss(n, d, 21), _gauss(300, d, 22)
    ix = W.GPUVectorIndex(d, NAMES[metric], capacity=n)
    ix.upload_vectors(base)
    rng = np.random.default_rng(23)
    dead = rng.choice(n, 900, replace=False)
    ix.add_tombstones(dead)
    tomb = O.bits_from_ids(dead, n)
    cases = {
        "empty": np.zeros(0, np.int64),
        "dead_only": np.sort(dead[:50]),
        "one": np.array([12_345]),
        "all": np.arange(n),
        "prefix": np.arange(0, 7_000, 3),
        "random_30": np.nonzero(rng.random(n) < 0.3)[0],
    }
    for name, ids_a in cases.items():
        al = W.AllowList.from_ids(ids_a, n)
        for q in (qs, qs[:1]):
            _check(ix, base, q, 10, metric, allow_bits=al.words, allow=al, tomb=tomb)
            a = ix.search_batch(q, 10, mode="exact", allow=al)
            monkeypatch.setenv("WV_BF_SYNC_COMPACT", "1")
            b = ix.search_batch(q, 10, mode="exact", allow=al)
            monkeypatch.delenv("WV_BF_SYNC_COMPACT")
            assert np.array_equal(a[2], b[2]), name
            for i in range(len(q)):   # (entries past a query's count are unspecified)
                c = int(a[2][i])
                assert np.array_equal(a[0][i, :c], b[0][i, :c]), name
                assert np.array_equal(a[1][i, :c].view(np.uint32), b[1][i, :c].view(np.uint32)), name
    ix.close()


@pytest.mark.parametrize("metric", [O.L2, O.DOT])
def test_duplicate_rows_ties_by_id(metric):
    """Rows repeated many times: equal keys everywhere, so the finalize's
    selection (the FIN_KF-th list head bounds the entries it sorts; more than
    256 such entries fall back to the per-lane selection) must order ties by
    id exactly as the restatement does.  600 queries: 3 query blocks of 85
    slots, 170 lists of 8 entries per query."""
    distinct, reps, d = 500, 40, 256
    base = np.tile(_gauss(distinct, d, 31), (reps, 1))
    qs = _gauss(600, d, 32)
    ix = W.GPUVectorIndex(d, NAMES[metric], capacity=len(base))
    ix.upload_vectors(base)
    for k in (10, 32):
        _check(ix, base, qs, k, metric)
    ix.close()


@pytest.mark.parametrize("d", [64, 256])
def test_finalize_many_lists_small_batches(d):
    """Small batches spread a corpus over many slots: 1 or 3 queries over
    ~9k rows give each query 100-300 lists (800-2400 entries), so the
    finalize bounds them by the FIN_KF-th list head and compacts the entries
    at or below it over several 512-entry rounds (a wave-uniform count), or
    falls back past 256 lists.  Equal to the restatement."""
    n = 9_001
    base, qs = _gauss(n, d, 41), _gauss(700, d, 42)
    for metric in (O.L2, O.DOT):
        ix = W.GPUVectorIndex(d, NAMES[metric], capacity=n)
        ix.upload_vectors(base)
        for nq in (1, 3, 700):
            _check(ix, base, qs[:nq], 10, metric)
        ix.close()
