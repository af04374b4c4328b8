"""Product quantization: the restatement pinned by the
reference's own PQ tests (CPU), then the GPU path against it (-m gpu).

Reference: adapters/repos/db/vector/ssdhelpers/product_quantization.go
(code layout :116-258, distances :272-291, lookup table :30-75), kmeans.go
(:78-110 Nearest), hnsw/compress.go:39-89 (Compress), hnsw/search.go:171-199 and
index.go:493-511 (compressed search).  KMeans.Fit (random init) and the tile
encoder's gonum quantiles are the fitting side and are not restated: the
quantizer enters as its centroid table, as the cgo shim would pass
kms[i].Centroid(c).
"""
import numpy as np
import pytest

import pyoracle as O
import weaviate_amd as W


# ---------------------------------------------------------------- CPU: oracle KATs
def test_reference_decode_kats():
    """product_quantization_test.go:90-174 (Test_NoRacePQDecodeBits)."""
    assert O.pq_extract(bytes(range(100)), 100, 256, True) == list(range(100))
    assert O.pq_extract(bytes([0, 16, 131, 16, 81, 135, 0]), 8, 64, True) == list(range(8))
    assert O.pq_extract(bytes([0, 0, 1, 0, 32, 3, 0, 0]), 4, 4096, True) == list(range(4))
    two = b"".join(int(i).to_bytes(2, "big") for i in range(100))
    assert O.pq_extract(two, 100, 65536, True) == list(range(100))


@pytest.mark.parametrize("ks,use_bits", [(256, True), (65536, True), (1024, True), (256, False), (65536, False),
                                         (1024, False), (64, True), (4096, True), (16, True), (2, True)])
def test_reference_encode_roundtrips(ks, use_bits):
    """Test_NoRacePQEncodeBits / EncodeBytes (:176-402): PutCode then ExtractCode
    returns every code; plus the bit widths the reference does not test."""
    n = 100
    codes = [i % ks for i in range(n)]
    enc = O.pq_put(codes, ks, use_bits, length=2 * n if (ks == 1024 and use_bits) else None)
    assert O.pq_extract(enc, n, ks, use_bits) == codes


def test_layout_bits_and_bytes():
    """NewProductQuantizer: bits = int(log2 ks), bytes = int(log2(ks-1))/8 + 1."""
    assert O.pq_layout(256) == (8, 1)
    assert O.pq_layout(64, True) == (6, 1)
    assert O.pq_layout(1024, True) == (10, 2)
    assert O.pq_layout(65536) == (16, 2)
    assert O.pq_layout(300) == (8, 2)       # not a power of two: 8 bits, two bytes


def _pq_dist_numpy(metric, x, codes, cent):
    """The same arithmetic spelled out in numpy float32, one rounding per op."""
    m, ks, ds = cent.shape
    dist = np.float32(0)
    for i in range(m):
        c = cent[i, codes[i]]
        s = np.float32(0)
        for j in range(ds):
            if metric == O.L2:
                d = np.float32(x[i * ds + j] - c[j])
                s = np.float32(s + np.float32(d * d))
            else:
                s = np.float32(s + np.float32(x[i * ds + j] * c[j]))
        dist = np.float32(dist + s)
    return dist if metric == O.L2 else (np.float32(-dist) if metric == O.DOT else np.float32(np.float32(1) - dist))


@pytest.mark.parametrize("metric", [O.L2, O.DOT, O.COSINE])
@pytest.mark.parametrize("m", [1, 4, 16])
def test_pq_distance_is_the_step_sum(metric, m):
    rng = np.random.default_rng(m)
    d, ks = 16, 64
    cent = rng.standard_normal((m, ks, d // m)).astype(np.float32)
    x = rng.standard_normal(d).astype(np.float32)
    for _ in range(20):
        codes = rng.integers(0, ks, m)
        enc = O.pq_put(codes.tolist(), ks, True)
        got = O.pq_distance(metric, x, enc, cent, ks, True)
        want = _pq_dist_numpy(metric, x, codes, cent)
        assert np.float32(got).view(np.uint32) == np.float32(want).view(np.uint32)


def test_kmeans_nearest_last_tie_wins():
    """kmeans.go:78-110: `minD[j] < distance` stops the scan, so an equal
    distance replaces the best: the LAST of equal centroids is the code."""
    cent = np.zeros((1, 8, 2), np.float32)
    cent[0, :, 0] = [5, 1, 3, 1, 9, 1, 7, 2]     # centroids 1, 3 and 5 are equal
    enc = O.pq_encode_kmeans(np.array([[1.0, 0.0]], np.float32), cent)
    assert O.pq_extract(enc[0].tobytes(), 1, 8) == [5]


def test_c_abi_code_length():
    assert W.lib().wv_pq_code_len(32, 256, 0) == 32
    assert W.lib().wv_pq_code_len(100, 1024, 1) == 200
    assert W.lib().wv_pq_code_len(8, 65536, 0) == 16
    assert W.lib().wv_pq_code_len(8, 1, 0) == -1


# ---------------------------------------------------------------- GPU parity
def _centroids(base, m, ks, seed=0):
    """A fitted-looking quantizer: per segment, ks distinct data rows' segments."""
    rng = np.random.default_rng(seed)
    n, d = base.shape
    ds = d // m
    rows = rng.choice(n, ks, replace=False)
    return np.stack([base[rows, i * ds:(i + 1) * ds] for i in range(m)]).astype(np.float32)


def _same_tie_aware(a_ids, a_d, b_ids, b_d):
    assert np.array_equal(a_d.view(np.uint32), b_d.view(np.uint32))
    if len(a_d) == 0:
        return
    for v in np.unique(a_d):
        if v != a_d[-1]:
            assert set(a_ids[a_d == v].tolist()) == set(b_ids[b_d == v].tolist())


@pytest.mark.gpu
@pytest.mark.parametrize("m,ks,use_bits", [(32, 256, False), (8, 256, False), (8, 64, True), (4, 1024, True),
                                           (16, 1024, False)])
def test_device_encode_equals_reference_encoder(m, ks, use_bits):
    rng = np.random.default_rng(m + ks)
    n, d = 3000, 32
    base = rng.standard_normal((n, d)).astype(np.float32)
    cent = _centroids(base, m, ks)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    ix.upload_vectors(base)
    ix.set_pq(cent, use_bits_encoding=use_bits)
    ix.pq_encode()
    got = ix.download_pq_codes(n)
    enc = O.pq_encode_kmeans(base, cent, use_bits)
    want = np.array([O.pq_extract(enc[r].tobytes(), m, ks, use_bits) for r in range(n)], np.uint16)
    assert np.array_equal(got, want)
    # the uploaded reference layout decodes to the same codes
    ix.upload_pq_codes(enc)
    assert np.array_equal(ix.download_pq_codes(n), want)
    ix.close()


def _compressed_pair(n, d, m, ks, metric="l2-squared", M=16, efc=64, seed=5, use_bits=False):
    rng = np.random.default_rng(seed)
    base = rng.standard_normal((n, d)).astype(np.float32)
    if metric == "cosine-dot":
        base = O.normalize_rows(base)
    ref = O.Index(d, metric, M, efc, capacity=n, seed=seed)
    ref.add_batch(base, threads=8)
    cent = _centroids(base, m, ks, seed)
    enc = O.pq_encode_kmeans(base, cent, use_bits)
    ref.compress(cent, enc, use_bits)
    ix = W.GPUVectorIndex(d, metric, capacity=n, max_connections=M)
    ix.upload_vectors(base)
    ix.upload_graph(ref.export_graph())
    ix.set_pq(cent, use_bits_encoding=use_bits)
    ix.upload_pq_codes(enc)
    ix.set_compressed(True)
    return ref, ix, base, cent, enc


@pytest.mark.gpu
@pytest.mark.parametrize("metric", ["l2-squared", "dot", "cosine-dot"])
def test_compressed_flat_search_parity(metric):
    """flatSearch on a compressed index (flat_search.go:19-74 with the PQ
    distance of index.go:493-511): shared and per-query allow lists, tombstones."""
    n, d, m, ks, k = 6000, 32, 8, 256, 10
    ref, ix, base, _, _ = _compressed_pair(n, d, m, ks, metric)
    rng = np.random.default_rng(7)
    qs = rng.standard_normal((40, d)).astype(np.float32)
    if metric == "cosine-dot":
        qs = O.normalize_rows(qs)
    dead = rng.choice(n, 50, replace=False)
    for t in dead:
        ref.add_tombstone(int(t))
    ix.set_tombstones(dead.tolist())
    gi, gd, gn = ix.search_batch(qs, k, mode="exact")
    oi, od, on, _ = ref.search_batch(qs, k, 0, mode=1, threads=8)
    for i in range(len(qs)):
        _same_tie_aware(gi[i, : gn[i]], gd[i, : gn[i]], oi[i, : on[i]], od[i, : on[i]])
    shared = W.AllowList.from_ids(np.nonzero(rng.random(n) < 0.3)[0], n)
    gi, gd, gn = ix.search_batch(qs, k, allow=shared, mode="exact")
    oi, od, on, _ = ref.search_batch(qs, k, 0, allow=shared.words, mode=1, threads=8)
    for i in range(len(qs)):
        _same_tie_aware(gi[i, : gn[i]], gd[i, : gn[i]], oi[i, : on[i]], od[i, : on[i]])
    per = [W.AllowList.from_ids(np.nonzero(rng.random(n) < 0.05)[0], n) for _ in range(len(qs))]
    gi, gd, gn = ix.search_batch(qs, k, allow=per, mode="exact")
    for i in range(len(qs)):
        oi, od, on, _ = ref.search_batch(qs[i:i + 1], k, 0, allow=per[i].words, mode=1)
        _same_tie_aware(gi[i, : gn[i]], gd[i, : gn[i]], oi[0, : on[0]], od[0, : on[0]])
    ix.close()


@pytest.mark.gpu
@pytest.mark.parametrize("metric", ["l2-squared", "dot"])
@pytest.mark.parametrize("ef", [32, 100])
def test_compressed_hnsw_parity(metric, ef):
    """knnSearchByVector on a compressed index: every distance of the descent and
    of layer 0 is the PQ distance (search.go:171-199, 467-476)."""
    n, d, m, ks, k = 8000, 32, 16, 256, 10
    ref, ix, base, _, _ = _compressed_pair(n, d, m, ks, metric, seed=9)
    rng = np.random.default_rng(11)
    qs = rng.standard_normal((200, d)).astype(np.float32)
    gi, gd, gn = ix.search_batch(qs, k, ef=ef, mode="hnsw")
    oi, od, on, _ = ref.search_batch(qs, k, ef, threads=8)
    same = sum(np.array_equal(gd[i, : gn[i]].view(np.uint32), od[i, : on[i]].view(np.uint32)) for i in range(len(qs)))
    assert same >= len(qs) - 2, same   # tie-dependent expansion order aside
    ix.close()


@pytest.mark.gpu
def test_compress_after_deletes_does_not_crash():
    """compress_deletes_test.go:29-72: 10k x 20-d, M=32, efC=64, ef=32, 1001
    deleted ids, Compress(dims, 256, kmeans), SearchByVector k=100."""
    n, d, k = 10000, 20, 100
    rng = np.random.default_rng(3)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((100, d), dtype=np.float32)
    ref = O.Index(d, "l2-squared", 32, 64, capacity=n, seed=3)
    ref.add_batch(base, threads=8)
    dead = list(range(10, 1010)) + [1]
    for t in dead:
        ref.add_tombstone(t)
    cent = _centroids(base, d, 256, 3)
    enc = O.pq_encode_kmeans(base, cent)
    ref.compress(cent, enc)
    ref.set_search_config(ef=32)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n, max_connections=32, ef=32)
    ix.upload_vectors(base)
    ix.upload_graph(ref.export_graph())
    ix.set_tombstones(dead)
    ix.set_pq(cent)
    ix.pq_encode()
    ix.set_compressed(True)
    hits = 0
    for q in qs[:20]:
        ids, ds = ix.search_by_vector(q, k)
        assert len(ids) == k and not set(ids.tolist()) & set(dead)
        oi, od = ref.search_by_vector(q, k)
        hits += np.array_equal(ds.view(np.uint32), od.view(np.uint32))
    assert hits >= 18
    ix.close()


@pytest.mark.gpu
def test_added_rows_on_a_compressed_index():
    """hnsw.Add on a compressed index encodes the vector (insert.go:91-95): with
    KMeans the device encodes added rows; with the tile encoder they wait for
    their codes (excluded until uploaded)."""
    n0, n1, d, m, ks, k = 3000, 3300, 16, 4, 256, 10
    rng = np.random.default_rng(21)
    base = rng.standard_normal((n1, d)).astype(np.float32)
    cent = _centroids(base, m, ks, 21)
    enc = O.pq_encode_kmeans(base, cent)
    qs = rng.standard_normal((30, d)).astype(np.float32)
    for encoder in ("kmeans", "tile"):
        ix = W.GPUVectorIndex(d, "l2-squared", capacity=n1)
        ix.upload_vectors(base[:n0])
        ix.set_pq(cent, encoder=encoder)
        ix.upload_pq_codes(enc[:n0])
        ix.set_compressed(True)
        ix.add(np.arange(n0, n1), base[n0:])
        gi, gd, gn = ix.search_batch(qs, k, mode="exact")
        live = n1 if encoder == "kmeans" else n0
        want = np.array([[O.pq_distance(O.L2, q, enc[r].tobytes(), cent, ks) for r in range(live)] for q in qs])
        for i in range(len(qs)):
            order = np.lexsort((np.arange(live), want[i]))[:k]
            assert np.array_equal(gd[i].view(np.uint32), want[i][order].astype(np.float32).view(np.uint32))
        if encoder == "tile":
            ix.upload_pq_codes(enc[n0:], first_id=n0)
            gi, gd, gn = ix.search_batch(qs, k, mode="exact")
            assert (gi >= n0).any()
        ix.close()
