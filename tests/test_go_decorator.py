"""The cgo decorator (go/vector/gpu/gpu.go) and its native replay harnesses.

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
    for method, call in (("Add", "wv_mirror_add"), ("Delete", "wv_mirror_delete"),
                         ("SearchByVector", "wv_mirror_search"),
                         ("SearchByVectorDistance", "wv_mirror_search_by_distance"),
                         ("UpdateUserConfig", "wv_mirror_update_config"),
                         ("PostStartup", "wvgpu_post_startup_async")):
        body = re.search(r"func \(g \*Index\) %s\(.*?\n}\n" % method, src, re.S)
        assert body, method
        assert f"C.{call}(" in body.group(0), f"{method} does not call {call}"
    # PostStartup goes live from the shard's commit log and VectorForIDThunk,
    # on the library's thread (startup.go:174-203 prefills in a goroutine)
    assert "wv_mirror_post_startup_async(m, wvgpuVectorForID, ctx)" in src
    assert '".hnsw.commitlog.d"' in src and "//export wvgpuVectorForID" in src
    # self-healing: the resync flushes the CPU index's log through wvgpuFlush
    assert "//export wvgpuFlush" in src and "o->auto_resync = 1;" in src and "o->flush = wvgpuFlush;" in src
    # compaction flushes the CPU index's log first, and never after close
    body = re.search(r"func \(g \*Index\) startCompaction\(.*?\n}\n", src, re.S).group(0)
    assert body.index("g.closed.Load()") < body.index("cpuIndex.Flush()") < body.index("C.wv_mirror_compact(")
    # (advisor, round 3) the compaction check runs under mu and only while open
    add = re.search(r"func \(g \*Index\) Add\(.*?\n}\n", src, re.S).group(0)
    assert add.index("C.wv_mirror_needs_compaction(") < add.rindex("g.mu.RUnlock()") < add.index("g.startCompaction()")
    assert "!g.closed.Load()" in add
    # runtime PQ enablement (config_update.go:97-128): the CPU index answers
    # while pending, each callback flushes the log and compacts the mirror
    uuc = re.search(r"func \(g \*Index\) UpdateUserConfig\(.*?\n}\n", src, re.S).group(0)
    assert "g.pqPending.Store(true)" in uuc and "go g.syncCompression(gen, final)" in uuc
    # (advisor, round 5) a failed UpdateUserConfig, or a Compress that ended
    # without codes, settles the flag instead of leaving the CPU index answering
    assert "g.pqPending.Store(false)" in uuc
    sc = re.search(r"func \(g \*Index\) syncCompression\(.*?\n}\n", src, re.S).group(0)
    assert sc.index("cpuIndex.Flush()") < sc.index("C.wv_mirror_compact(") < sc.index("g.pqPending.Store(false)")
    for method in ("SearchByVector", "SearchByVectorDistance"):
        body = re.search(r"func \(g \*Index\) %s\(.*?\n}\n" % method, src, re.S).group(0)
        assert "g.pqPending.Load()" in body, method
    # close releases mu before joining the library's thread (a resync's flush takes mu)
    cl = re.search(r"func \(g \*Index\) close\(.*?\n}\n", src, re.S).group(0)
    assert cl.index("g.mu.Unlock()") < cl.index("C.wv_mirror_destroy(") < cl.index("g.freeHandles()")


def test_replay_harness_binds_only_header_symbols():
    for f in ("go_replay.cpp", "mirror_replay.cpp"):
        src = open(os.path.join(ROOT, "tests", "native", f)).read()
        used = set(re.findall(r"\b(wv_[a-z0-9_]+)\s*\(", src))
        assert used <= _header_functions(), f


@pytest.mark.gpu
def test_mirror_lifecycle_from_commit_log(tmp_path):
    """The decorator's lifecycle over wv_mirror_*: startup from a commit-log
    directory the restatement wrote (startup.go:56-205) with rows pulled
    through the vector thunk, searches equal to the restatement's, then 20k
    adds (capacity growth), deletes and log-driven compactions under 8
    concurrent searchers, the delta bounded, and searches equal to the
    restatement's again after the final compaction."""
    binp = os.path.join(ROOT, "tests", "native", "mirror_replay")
    assert os.path.exists(binp), "build tests/native first (__graft_entry__.build())"
    p = subprocess.run([binp, str(tmp_path), "0"], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:] + p.stdout[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["ok"] and r["diffs_startup"] == 0 and r["diffs_final"] == 0
    assert r["startup_missing"] > 50 and r["startup_rows"] + r["startup_missing"] == 20000
    assert r["adds"] == 20000 and r["growths"] >= 1 and r["capacity"] >= 40000
    assert r["compactions"] >= 3 and r["max_delta"] <= 2 * 4096
    assert r["added_checks"] > 100 and r["filtered"] > 50
    assert r["batcher_batches"] < r["batcher_requests"]
    print(r)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["async", "heal", "postheal", "pq", "epgone", "pqlive"])
def test_mirror_lifecycle_modes(tmp_path, mode):
    """async: PostStartup returns at once and the mirror builds on its own
    thread while writers and searchers run (the CPU index answers until it is
    live; writes made meanwhile are replayed); heal: a write the mirror never
    saw marks it stale and it resyncs by itself (flush callback, then a
    rebuild), serving the missed row afterwards; postheal: a PostStartup
    posted under the decorator's lock while a resync waits for that lock in
    its flush callback returns at once and runs after the resync (ADVICE r5:
    no deadlock); pq: a KMeans-compressed
    index (AddPQ record in the log) is served compressed, equal to the
    restatement's PQ searches (compress.go:39-99, search.go:172-197);
    epgone: the log's entrypoint lost its object -- HNSW searches answer
    WV_EDELETED as knnSearchByVector errors (search.go:467-476), a flat one
    equals flatSearch's; pqlive: the class is compressed while serving
    (UpdateUserConfig with PQ.Enabled -> Compress, config_update.go:97-120,
    compress.go:39-99) with no later write, the decorator's callback flushes
    and compacts, and the mirror then answers as the restatement's PQ
    searches."""
    binp = os.path.join(ROOT, "tests", "native", "mirror_replay")
    assert os.path.exists(binp), "build tests/native first (__graft_entry__.build())"
    p = subprocess.run([binp, str(tmp_path), "0", mode], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:] + p.stdout[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["ok"] and r["mode"] == mode
    if mode == "epgone":
        assert r["flat_ids"] > 0
        return
    assert r["diffs_final"] == 0
    assert r["adds"] == 20000 and r["max_delta"] <= (20000 if mode in ("async", "pq") else 0) + 2 * 4096
    if mode in ("async", "pq"):
        assert r["replayed_writes"] > 0 and r["stale_answers"] > 0 and r["startup_call_s"] < 0.5
    if mode == "heal":
        # two failures: the second the moment the first resync went live
        assert r["resyncs"] >= 2 and r["stale_answers"] > 0
    if mode == "postheal":
        assert r["resyncs"] >= 1 and r["stale_answers"] > 0
    if mode in ("pq", "pqlive"):
        assert r["pq"] == 1
    print(r)


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


def test_host_runtime_under_thread_sanitizer(tmp_path):
    """The reference runs `go test -race` over its packages (test/run.sh:101-109).
    Here the host runtime -- wv_mirror.cpp (FairRW, startups on the mirror's
    thread, resyncs, compactions), wv_batcher.cpp and wv_commitlog.cpp -- is
    built with -fsanitize=thread over a CPU stand-in of the wv_index_* entry
    points (tests/native/tsan/cpu_index.cpp) and driven by the mirror_replay
    scenario in every mode: no race may be reported (no GPU involved)."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "native"), "mirror_replay_tsan"])
    binp = os.path.join(ROOT, "tests", "native", "mirror_replay_tsan")
    from concurrent.futures import ThreadPoolExecutor

    def run(mode):
        p = subprocess.run([binp, str(tmp_path / mode), "0", mode], capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, TSAN_OPTIONS="halt_on_error=0 exitcode=66"))
        return mode, p

    with ThreadPoolExecutor(2) as ex:
        for mode, p in ex.map(run, ["sync", "async", "heal", "postheal", "pq", "epgone", "pqlive"]):
            races = p.stderr.count("WARNING: ThreadSanitizer")
            assert races == 0 and p.returncode == 0, (mode, races, p.stderr[-4000:])
            r = json.loads(p.stdout.strip().splitlines()[-1])
            assert r["ok"] and r["mode"] == mode and (mode == "epgone" or r["compactions"] >= 1)
