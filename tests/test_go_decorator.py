"""The cgo decorator (go/vector/gpu/gpu.go) and its native replay harness.

The Go toolchain is absent from the build image, so the decorator's C call
sequence is replayed by tests/native/go_replay.cpp (plain C++ over the C ABI,
as the cgo binary would link it): 8 threads searching through the
micro-batcher while a writer adds rows, tombstones ids and resyncs a snapshot.
It asserts that no id deleted before a search started is returned and that a
row added before a search started is found at once (delete.go:29-84,
insert.go:43-65, search.go:64-79).
"""
import json
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go", "vector", "gpu", "gpu.go")
HDR = os.path.join(ROOT, "include", "wvgpu.h")
BIN = os.path.join(ROOT, "tests", "native", "go_replay")


def _header_functions():
    return set(re.findall(r"\b(wv_[a-z0-9_]+)\s*\(", open(HDR).read()))


def test_go_decorator_binds_only_header_symbols():
    src = open(GO).read()
    used = set(re.findall(r"\bC\.(wv_[a-z0-9_]+)\s*\(", src))
    assert used, "the decorator calls no C function"
    assert used <= _header_functions(), f"not in wvgpu.h: {used - _header_functions()}"
    # every write of the VectorIndex interface reaches the mirror
    for method, call in (("Add", "wv_index_add"), ("Delete", "wv_index_add_tombstones"),
                         ("SearchByVector", "wv_batcher_search"),
                         ("SearchByVectorDistance", "wv_search_by_vector_distance"),
                         ("UpdateUserConfig", "wv_index_update_config")):
        body = re.search(r"func \(g \*Index\) %s\(.*?\n}\n" % method, src, re.S)
        assert body, method
        assert f"C.{call}(" in body.group(0), f"{method} does not call {call}"


def test_replay_harness_binds_only_header_symbols():
    src = open(os.path.join(ROOT, "tests", "native", "go_replay.cpp")).read()
    used = set(re.findall(r"\b(wv_[a-z0-9_]+)\s*\(", src))
    assert used <= _header_functions()


@pytest.mark.gpu
def test_go_call_sequence_concurrent_add_delete_search():
    assert os.path.exists(BIN), "build tests/native first (__graft_entry__.build())"
    p = subprocess.run([BIN, "0"], capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stderr[-2000:] + p.stdout[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["ok"] and r["resyncs"] == 1 and r["deletes"] > 1000 and r["adds"] == 2000
    assert r["added_checks"] > 100 and r["filtered"] > 50 and r["distance_searches"] > 10
    # the batcher really coalesced concurrent callers
    assert r["batcher_batches"] < r["batcher_requests"]
    print(r)
