"""CPU-only checks: the C-ABI library loads and exports every declared symbol,
host-side helpers mirror the reference semantics, and the multi-GPU sharding
plan (shard bounds + all-gather + (dist, id) merge) reproduces a single search
of the whole corpus, exercised with world_size 2 over gloo."""
import os
import socket

import numpy as np
import pytest

import pyoracle as O
import weaviate_amd as W
from weaviate_amd.sharded import allgather_topk, merge_topk, shard_bounds


def test_library_exports_every_header_symbol():
    lib = W.lib()
    syms = W.header_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert b"gfx950" in lib.wv_version()


def test_config_defaults_match_reference():
    """entities/vectorindex/hnsw/config.go:33-50."""
    import ctypes as C
    from weaviate_amd._lib import WvConfig
    c = WvConfig()
    W.lib().wv_config_default(C.byref(c))
    assert (c.max_connections, c.ef, c.dynamic_ef_min, c.dynamic_ef_max, c.dynamic_ef_factor,
            c.flat_search_cutoff, c.forbid_flat) == (64, -1, 100, 500, 8, 40000, 0)


def test_search_time_ef_abi_matches_dynamic_ef_kats(kats):
    """searchTimeEF / autoEfFromK (search.go:30-62) through the C ABI,
    against dynamic_ef_test.go:27-102 (k=100 -> 500, 10 -> 100, 23 -> 184,
    explicit ef 78) and the oracle on a grid around the clamps."""
    import ctypes as C
    from weaviate_amd._lib import WvConfig
    for c in kats["dynamic_ef"]["cases"]:
        cfg = WvConfig()
        W.lib().wv_config_default(C.byref(cfg))
        cfg.ef, cfg.dynamic_ef_min, cfg.dynamic_ef_max, cfg.dynamic_ef_factor = c["ef"], c["min"], c["max"], c["factor"]
        assert W.lib().wv_config_search_time_ef(C.byref(cfg), c["k"]) == c["expect"], c
    for ef in (-1, 0, 1, 7, 64, 600):
        for k in (1, 5, 10, 13, 50, 62, 63, 100, 700):
            cfg = WvConfig()
            W.lib().wv_config_default(C.byref(cfg))
            cfg.ef = ef
            assert W.lib().wv_config_search_time_ef(C.byref(cfg), k) == O.search_time_ef(ef, 100, 500, 8, k)


def test_bad_arguments_return_errors_not_crashes():
    import ctypes as C
    h = C.c_void_p()
    rc = W.lib().wv_index_create(0, 0, None, 10, C.byref(h))
    assert rc == 1  # WV_EINVAL
    assert b"bad argument" in W.lib().wv_last_error()
    assert W.lib().wv_index_create(8, 7, None, 10, C.byref(h)) == 1


def test_allow_list_semantics(kats):
    """helpers/allow_list_test.go:103-133: ascending iteration, Len, Contains."""
    c = kats["allow_list_iteration"]
    al = W.AllowList(*c["insert"])
    assert list(al.iterator()) == c["expect_iteration"]
    assert len(al) == 3
    assert al.contains(2) and not al.contains(0) and not al.contains(99)


def test_shard_bounds_partition():
    for n in (1, 7, 1000, 1_000_000):
        for w in (1, 2, 3, 4, 8):
            b = [shard_bounds(n, r, w) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))


def _merge_ref(g_ids, g_d, g_n, k):
    import torch
    world, nq = g_n.shape
    out_i = torch.zeros((nq, k), dtype=torch.int64)
    out_d = torch.zeros((nq, k), dtype=torch.float32)
    out_n = torch.zeros((nq,), dtype=torch.int32)
    for q in range(nq):
        c = sorted((float(g_d[s, q, j]), int(g_ids[s, q, j])) for s in range(world) for j in range(int(g_n[s, q])))[:k]
        out_n[q] = len(c)
        for j, (d, i) in enumerate(c):
            out_d[q, j] = d
            out_i[q, j] = i
    return out_i, out_d, out_n


def _worker(rank, world, port, n, d, nq, k, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(0)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((nq, d), dtype=np.float32)
    lo, hi = shard_bounds(n, rank, world)
    # per-shard search stand-in: the CPU restatement of flatSearch on this
    # shard (the GPU path is covered by tests/test_gpu_parity.py)
    oi, od, on = O.flat_scan(O.L2, base[lo:hi], qs, k, threads=2)
    ids = torch.from_numpy(oi.astype(np.int64) + lo)
    g_ids, g_d, g_n = allgather_topk(ids, torch.from_numpy(od), torch.from_numpy(on), world)
    m_ids, m_d, m_n = merge_topk(g_ids, g_d, g_n, k, merge_fn=_merge_ref)
    q.put((rank, m_ids.numpy(), m_d.numpy()))
    dist.destroy_process_group()


def test_sharded_search_equals_single_search_gloo_ws2():
    import multiprocessing as mp
    n, d, nq, k, world = 3000, 24, 20, 10, 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n, d, nq, k, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(60)
    rng = np.random.default_rng(0)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((nq, d), dtype=np.float32)
    ti, td, tn = O.flat_scan(O.L2, base, qs, k)
    for rank, ids, ds in res:
        assert ids.tolist() == ti.astype(np.int64).tolist()
        assert np.array_equal(ds, td)


def test_merge_topk_refuses_cpu_without_merge_fn():
    import torch
    with pytest.raises(RuntimeError):
        merge_topk(torch.zeros((2, 1, 1), dtype=torch.int64), torch.zeros((2, 1, 1)), torch.zeros((2, 1),
                   dtype=torch.int32), 1)
