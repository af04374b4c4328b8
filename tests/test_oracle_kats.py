"""Pin the CPU restatement (oracle/) against the reference's own known answers.

Every expected value here comes from tests/golden/reference_kats.json, which
holds the vectors and answers of the reference's tests (file:line in the
fixture).  CPU only.
"""
import numpy as np
import pytest

import pyoracle as O


def test_distancer_kats(kats):
    d = kats["distancer"]
    for c in d["l2"]:
        for impl in ("asm", "avx2", "purego"):
            assert O.distance(O.L2, c["a"], c["b"], impl) == c["expect"]
    for c in d["dot"]:
        for impl in ("asm", "avx2", "purego"):
            assert O.distance(O.DOT, c["a"], c["b"], impl) == c["expect"]
    for c in d["cosine"]:
        a, b = O.normalize(c["a"]), O.normalize(c["b"])
        got = O.distance(O.COSINE, a, b)
        assert abs(got - c["expect"]) <= c["delta"] + 1e-6


@pytest.mark.parametrize("metric", [O.L2, O.DOT])
def test_asm_order_scalar_equals_avx2_and_close_to_purego(kats, metric):
    """l2_amd64_test.go:35-73: asm vs pure Go within InEpsilon 0.01; our scalar
    emulation of the asm must equal the intrinsics mirror bit for bit."""
    lengths = kats["distancer"]["asm_vs_purego_lengths"]["lengths"]
    eps = kats["distancer"]["asm_vs_purego_lengths"]["epsilon"]
    rng = np.random.default_rng(7)
    for n in lengths:
        for sign in (1.0, -1.0):
            x = (sign * rng.random(n)).astype(np.float32)
            y = rng.random(n).astype(np.float32)
            s = O.distance(metric, x, y, "asm")
            v = O.distance(metric, x, y, "avx2")
            p = O.distance(metric, x, y, "purego")
            assert np.float32(s).view(np.uint32) == np.float32(v).view(np.uint32), (n, s, v)
            assert abs(s - p) <= eps * abs(p) + 1e-30


def test_priority_queue_order(kats):
    pqk = kats["priority_queue"]
    ops = [("insert", int(k), v) for k, v in pqk["values"].items()]
    for is_max, key in ((0, "min_order"), (1, "max_order")):
        out = O.pq_script(is_max, ops + [("pop",)] * len(ops))
        assert [i for i, _ in out] == pqk[key]


def test_dynamic_ef(kats):
    for c in kats["dynamic_ef"]["cases"]:
        assert O.search_time_ef(c["ef"], c["min"], c["max"], c["factor"], c["k"]) == c["expect"]


def test_index_cluster_kat(kats):
    c = kats["index_clusters"]
    idx = O.Index(2, c["metric"], c["max_connections"], c["ef_construction"], capacity=64)
    for i, v in enumerate(c["vectors"]):
        idx.add(i, v)
    for q in c["queries"]:
        ids, _ = idx.knn_search(c["vectors"][q["position"]], q["k"], q["ef"])
        if "expect_set" in q:
            assert sorted(ids.tolist()) == sorted(q["expect_set"])
        else:
            assert ids.tolist() == q["expect_order"]


def _load_hand_built(c):
    idx = O.Index(2, c["metric"], c["max_connections"], c["ef_construction"], capacity=16)
    for i, v in enumerate(c["vectors"]):
        idx.set_vector(i, v)
    for n in c["nodes"]:
        idx.import_node(n["id"], n["level"], n["connections"])
    idx.set_entrypoint(c["entrypoint"], c["max_level"])
    idx.set_search_config(ef=0, ef_min=0, ef_max=0, ef_factor=0, flat_search_cutoff=0)
    return idx


def test_hand_built_graph_kat(kats):
    c = kats["hand_built_graph"]
    idx = _load_hand_built(c)
    ids, _ = idx.search_by_vector(c["query"], c["k"])
    assert ids.tolist() == c["expect"]


def _load_snapshot(c):
    snap = c["snapshot"]
    idx = O.Index(3, c["metric"], c["max_connections"], c["ef_construction"], capacity=128)
    for i, v in enumerate(c["vectors"]):
        idx.set_vector(i, v)
    for n in snap["nodes"]:
        levels = [n["connections"][str(lv)] for lv in range(n["level"] + 1)]
        idx.import_node(n["id"], n["level"], levels)
    idx.set_entrypoint(snap["entrypoint"], snap["currentMaximumLayer"])
    # UserConfig{MaxConnections:30, EFConstruction:128}: ef=0 -> ef=k; forbidFlat
    idx.set_search_config(ef=0, ef_min=0, ef_max=0, ef_factor=0, flat_search_cutoff=0, forbid_flat=True)
    return idx


def test_delete_snapshot_invariant(kats):
    """delete_test.go:1092-1150: allowList(odd) search == search after
    tombstoning the remaining even nodes."""
    c = kats["delete_snapshot"]
    idx = _load_snapshot(c)
    odd = [i for i in range(len(c["vectors"])) if i % 2 == 1]
    control, _ = idx.search_by_vector(c["query"], c["k"], allow=odd)
    assert len(control) > 0
    for t in c["tombstone_after"]:
        idx.add_tombstone(t)
    res, _ = idx.search_by_vector(c["query"], c["k"])
    assert res.tolist() == control.tolist()
    assert all(i % 2 == 1 for i in res.tolist())


def test_acceptance_distances_and_cutoffs(kats):
    a = kats["acceptance_distances"]
    for name, metric in (("l2", "l2-squared"), ("dot", "dot")):
        c = a[name]
        idx = O.Index(len(c["query"]), metric, 64, 128, capacity=16)
        for i, v in enumerate(c["objects"]):
            idx.add(i, v)
        _, d = idx.search_by_vector(c["query"], 10)
        assert d.tolist() == pytest.approx(c["expect"], abs=0.01)
        lim = c["limited"] if isinstance(c["limited"], list) else [c["limited"]]
        for l in lim:
            _, d = idx.search_by_vector_distance(c["query"], l["distance"])
            assert d.tolist() == pytest.approx(l["expect"], abs=0.01)
    c = a["cosine"]
    idx = O.Index(2, "cosine-dot", 64, 128, capacity=16)
    for i, v in enumerate(c["objects"]):
        idx.add(i, v)
    _, d = idx.search_by_vector(c["query"], 10)
    assert d.tolist() == pytest.approx(c["expect"], abs=c["delta"])


def test_flat_search_iterates_allow_list_ascending_and_matches_scan():
    rng = np.random.default_rng(3)
    base = rng.random((300, 16), dtype=np.float32)
    idx = O.Index(16, "l2-squared", 8, 32, capacity=300)
    idx.add_batch(base)
    q = rng.random(16, dtype=np.float32)
    allow = list(range(0, 300, 3))
    idx.set_search_config(flat_search_cutoff=40000)
    ids, d = idx.search_by_vector(q, 10, allow=allow)
    bits = O.bits_from_ids(allow, 300)
    si, sd, sn = O.flat_scan(O.L2, base, q[None], 10, allow_bits=bits)
    assert ids.tolist() == si[0].tolist()
    assert all(i % 3 == 0 for i in ids.tolist())


def test_search_by_dist_iteration_caps_at_max_limit():
    rng = np.random.default_rng(5)
    base = rng.random((500, 8), dtype=np.float32)
    idx = O.Index(8, "l2-squared", 16, 64, capacity=500)
    idx.add_batch(base)
    q = rng.random(8, dtype=np.float32)
    ids, d = idx.search_by_vector_distance(q, 1e9, max_limit=150)
    # first round of 100 keeps going; the second round (total 1100) > 150 stops
    assert len(ids) == 100


def test_threaded_build_recall():
    rng = np.random.default_rng(11)
    base = rng.random((3000, 32), dtype=np.float32)
    qs = rng.random((50, 32), dtype=np.float32)
    idx = O.Index(32, "l2-squared", 16, 64, capacity=3000)
    idx.add_batch(base, threads=4)
    oi, od, on, st = idx.search_batch(qs, 10, 64, threads=4)
    ti, td, tn = O.flat_scan(O.L2, base, qs, 10)
    recall = np.mean([len(set(a.tolist()) & set(b.tolist())) / 10 for a, b in zip(oi, ti)])
    assert recall > 0.95
    g = idx.export_graph()
    assert (g["counts0"] <= 32).all()  # layer-0 degree <= 2M (too_many_links test)


def test_csr_export_import_round_trip():
    """The fixed-degree CSR re-layout (the GPU's graph format) loses nothing:
    a restatement restored from it searches identically (bench graph cache)."""
    rng = np.random.default_rng(5)
    base = rng.random((4000, 24), dtype=np.float32)
    qs = rng.random((60, 24), dtype=np.float32)
    a = O.Index(24, "l2-squared", 8, 48, capacity=4000, seed=3)
    a.add_batch(base, threads=4)
    g = a.export_graph()
    b = O.Index(24, "l2-squared", 8, 48, capacity=4000, seed=3)
    b.import_graph(base, g)
    ra, rb = a.search_batch(qs, 10, 40), b.search_batch(qs, 10, 40)
    assert (ra[0] == rb[0]).all() and (ra[1] == rb[1]).all() and ra[3] == rb[3]
    g2 = b.export_graph()
    for key in ("levels", "layer0", "upper_row", "upper"):
        assert np.array_equal(g[key], g2[key]), key
