"""Comparison helpers shared by the parity tests."""
import numpy as np


def same(a_ids, a_d, b_ids, b_d):
    """ids identical, distances bit-identical."""
    assert np.asarray(a_ids).tolist() == np.asarray(b_ids).tolist()
    assert np.array_equal(np.asarray(a_d, np.float32).view(np.uint32), np.asarray(b_d, np.float32).view(np.uint32))


def same_tie_aware(a_ids, a_d, b_ids, b_d):
    """Distances bit-identical; ids identical up to the order among equal
    distances, and free at the k-boundary distance (the reference breaks ties
    by heap layout, the GPU by id: SURVEY 8c)."""
    a_d = np.asarray(a_d, np.float32)
    b_d = np.asarray(b_d, np.float32)
    a_ids, b_ids = np.asarray(a_ids), np.asarray(b_ids)
    assert np.array_equal(a_d.view(np.uint32), b_d.view(np.uint32))
    if len(a_d) == 0:
        return
    last = a_d[-1]
    for v in np.unique(a_d):
        if v == last:
            continue
        assert set(a_ids[a_d == v].tolist()) == set(b_ids[b_d == v].tolist())


def tie_aware_equal(a_ids, a_d, b_ids, b_d) -> bool:
    try:
        same_tie_aware(a_ids, a_d, b_ids, b_d)
        return True
    except AssertionError:
        return False


def recall(ids, truth, k=10):
    """matches / (k * nq) against exact truths (recall_test.go:121-137)."""
    return float(np.mean([len(set(a[:k]) & set(b[:k])) / k for a, b in zip(np.asarray(ids).tolist(),
                                                                            np.asarray(truth).tolist())]))


def merge_lists(parts, k):
    """Merge per-shard (ids, dists, n) lists by (dist, id): index.go:1039-1043
    with the (dist, id) order of the ABI."""
    nq = parts[0][0].shape[0]
    out_i = np.zeros((nq, k), np.uint64)
    out_d = np.zeros((nq, k), np.float32)
    out_n = np.zeros(nq, np.int32)
    for q in range(nq):
        c = sorted((float(p[1][q, j]), int(p[0][q, j])) for p in parts for j in range(int(p[2][q])))[:k]
        out_n[q] = len(c)
        for j, (d, i) in enumerate(c):
            out_d[q, j] = d
            out_i[q, j] = i
    return out_i, out_d, out_n
