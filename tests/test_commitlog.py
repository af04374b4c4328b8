"""Commit log -> CSR loader (wv_graph_*), CPU only.

The loader replays adapters/repos/db/vector/hnsw/commitlog records the way
Deserializer.Do does (deserializer.go:80-158).  Pinned by (a) the reference's
own deserializer tests (deserializer_test.go:101-419: the same records, the
same expected state), (b) a log written by the restatement's build exactly
where the reference writes records (insert.go, neighbor_connections.go): the
replayed graph must equal the built graph, and (c) the startup rules for torn
tails, file order and interrupted condensing (startup.go:56-152,
commit_logger.go:121-166, corrupt_commit_logs_fixer.go:43-70).
"""
import os
import struct

import numpy as np
import pytest

import pyoracle as O
import weaviate_amd as W

ADD_NODE, SET_EP, ADD_LINK, REPLACE_LINKS, ADD_TOMB, REMOVE_TOMB, CLEAR_LINKS, DELETE_NODE, RESET, \
    CLEAR_LINKS_AT_LEVEL, ADD_LINKS, ADD_PQ = range(12)


def rec_id_level(t, id_, level):
    return struct.pack("<BQH", t, id_, level)


def rec_link(id_, level, target):
    return struct.pack("<BQHQ", ADD_LINK, id_, level, target)


def rec_links(t, id_, level, targets):
    return struct.pack("<BQHH", t, id_, level, len(targets)) + b"".join(struct.pack("<Q", x) for x in targets)


def rec_id(t, id_):
    return struct.pack("<BQ", t, id_)


def test_reference_deserializer_kats():
    """deserializer_test.go: ReadNode :198-218, ReadEP :220-239, ReadLink
    :241-264, ReadLinks :266-293, ReadAddLinks :295-322, tombstones :324-380."""
    ids = [2, 3, 4, 5, 6]
    g = W.CommitLogGraph(b"".join(rec_id_level(ADD_NODE, i, i * 2) for i in ids))
    for i in ids:
        assert g.node(i)[0] == i * 2
    g = W.CommitLogGraph(b"".join(rec_id_level(SET_EP, i, i * 2) for i in ids))
    assert (g.info()["entrypoint"], g.info()["max_level"]) == (6, 12)
    g = W.CommitLogGraph(b"".join(rec_link(i, i * 2, i * 3) for i in ids))
    for i in ids:
        assert g.node(i, i * 2)[1][-1] == i * 3
    for t in (REPLACE_LINKS, ADD_LINKS):
        g = W.CommitLogGraph(b"".join(rec_links(t, i, i * 2, [i + k for k in range(i * 4)]) for i in ids))
        for i in ids:
            assert g.node(i, i * 2)[1][-1] == i + i * 4 - 1
    g = W.CommitLogGraph(b"".join(rec_id(ADD_TOMB, i) for i in ids))
    assert g.info()["n_tombstones"] == 5
    log = b"".join(rec_id(ADD_TOMB, i) for i in [1, 2, 3, 4, 5]) + b"".join(rec_id(REMOVE_TOMB, i) for i in ids)
    g = W.CommitLogGraph(log + rec_id_level(ADD_NODE, 1, 0))
    bits = g.export_csr(4, 4)["tomb_bits"]
    assert np.nonzero(np.unpackbits(bits.view(np.uint8), bitorder="little"))[0].tolist() == [1]


def test_record_semantics_replace_append_clear_delete_reset():
    log = b"".join([
        rec_id_level(ADD_NODE, 0, 1), rec_links(REPLACE_LINKS, 0, 0, [5, 6, 7]), rec_link(0, 0, 8),
        rec_links(ADD_LINKS, 0, 1, [9]), rec_links(REPLACE_LINKS, 0, 0, [1, 2]),   # replace wins
        rec_link(3, 2, 4),                     # link to an unknown node creates it: level 0, 3 levels of lists
        rec_id_level(CLEAR_LINKS_AT_LEVEL, 0, 1),
        rec_id_level(ADD_NODE, 10, 0), rec_id(DELETE_NODE, 10), rec_id(DELETE_NODE, 99),   # out of range: no-op
        rec_id(CLEAR_LINKS, 42),
    ])
    g = W.CommitLogGraph(log)
    assert g.node(0, 0) == (1, [1, 2])
    assert g.node(0, 1) == (1, [])
    assert g.node(3, 2) == (0, [4])
    assert g.node(10)[0] == -1
    assert g.info()["n_slots"] == 4
    g = W.CommitLogGraph(log + rec_id(ADD_TOMB, 2) + bytes([RESET]) + rec_id_level(ADD_NODE, 1, 0))
    i = g.info()
    assert (i["n_slots"], i["entrypoint"], i["max_level"], i["n_tombstones"]) == (2, 0, 0, 1)  # tombstones survive


def _oracle_log(n=3000, d=16, M=8, efc=32, tomb=(5, 77, 1234), seed=3):
    rng = np.random.default_rng(seed)
    base = rng.random((n, d), dtype=np.float32)
    ix = O.Index(d, "l2-squared", M, efc, capacity=n, seed=seed)
    ix.enable_commit_log()
    ix.add_batch(base, threads=1)   # single writer: record order == mutation order
    for t in tomb:
        ix.add_tombstone(t)
    return ix, base, ix.commit_log()


def test_replay_of_the_restatements_build_log_is_the_built_graph():
    ix, base, log = _oracle_log()
    g = W.CommitLogGraph(log)
    e = ix.export_graph()
    c = g.export_csr(e["deg0"], e["degU"])
    for k in ("levels", "layer0", "upper_row", "upper"):
        assert np.array_equal(e[k], c[k]), k
    assert (c["entrypoint"], c["max_level"]) == (e["entrypoint"], e["max_level"])
    got = np.nonzero(np.unpackbits(c["tomb_bits"].view(np.uint8), bitorder="little"))[0].tolist()
    assert got == [5, 77, 1234]
    info = g.info()
    assert info["valid_bytes"] == len(log) and not info["truncated"] and not info["compressed"]


def test_torn_tail_keeps_every_complete_record():
    """startup.go:93-107: EOF inside a record keeps the valid prefix."""
    _, _, log = _oracle_log(n=400)
    rng = np.random.default_rng(1)
    for cut in rng.integers(1, len(log) - 1, 12):
        g = W.CommitLogGraph(log[:cut])
        i = g.info()
        assert i["valid_bytes"] <= cut
        assert bool(i["truncated"]) == (i["valid_bytes"] < cut)
        ref = W.CommitLogGraph(log[: i["valid_bytes"]]).export_csr(16, 8)
        got = g.export_csr(16, 8)
        for k in ("levels", "layer0", "upper_row", "upper"):
            assert np.array_equal(ref[k], got[k]), (cut, k)


def test_unknown_record_type_is_an_error_not_a_crash():
    with pytest.raises(W.WvError, match="unrecognized commit type"):
        W.CommitLogGraph(rec_id_level(ADD_NODE, 0, 0) + bytes([200]) + b"\0" * 10)


def test_pq_record_marks_the_graph_compressed():
    # AddPQ (logger.go:77-96): tile encoder (0), dims 4, Ks 256, M 2 -> 2 x 51 bytes
    pq = struct.pack("<BHBHHBB", ADD_PQ, 4, 0, 256, 2, 0, 0) + b"\0" * (2 * 51)
    g = W.CommitLogGraph(rec_id_level(ADD_NODE, 0, 0) + pq + rec_id_level(ADD_NODE, 1, 0))
    i = g.info()
    assert i["compressed"] and not i["truncated"] and i["n_slots"] == 2


def test_directory_order_condensed_and_temporaries(tmp_path):
    """getCommitFileNames (commit_logger.go:121-166) + CorruptCommitLogFixer."""
    _, _, log = _oracle_log(n=600)
    # split at record boundaries: replay a prefix to find clean cut points
    cuts = []
    for frac in (0.25, 0.5, 0.75):
        cuts.append(W.CommitLogGraph(log[: int(len(log) * frac)]).info()["valid_bytes"])
    parts = [log[a:b] for a, b in zip([0] + cuts, cuts + [len(log)])]
    d = tmp_path / "main.hnsw.commitlog.d"
    d.mkdir()
    names = ["999", "1000.condensed", "1001", "20000"]   # numeric, not lexical, order
    for nme, part in zip(names, parts):
        (d / nme).write_bytes(part)
    (d / ".hidden").write_bytes(b"\xff" * 7)
    (d / "1002.scratch.tmp").write_bytes(b"\xff" * 7)
    (d / "1003.combined.tmp").write_bytes(b"\xff" * 7)
    (d / "1001.condensed").write_bytes(b"\xff" * 7)   # interrupted condense: original still there
    g = W.CommitLogGraph(str(d))
    want = W.CommitLogGraph(log)
    a, b = g.export_csr(16, 8), want.export_csr(16, 8)
    for k in ("levels", "layer0", "upper_row", "upper"):
        assert np.array_equal(a[k], b[k]), k
    assert sorted(os.listdir(d)) == sorted(names + [".hidden", "1002.scratch.tmp", "1003.combined.tmp",
                                                    "1001.condensed"])   # read-only: nothing deleted
