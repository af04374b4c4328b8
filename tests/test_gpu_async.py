"""The device-resident entry point queues a whole batch without a host round
trip, certificate fallbacks included (-m gpu).

wv_search_batch_device (include/wvgpu.h) must return while the GPU still
works on an exact or HNSW batch, and the queries whose certificate fails --
ties at the k boundary, or more survivors than the fallback filter keeps --
must be answered on the device with the restatement's result.
"""
import time

import numpy as np
import pytest
import torch

import pyoracle as O
import weaviate_amd as W
from helpers import same_tie_aware

pytestmark = pytest.mark.gpu


def _dev_batch(ix, qs, k, mode, ef=0):
    dev = torch.device("cuda:0")
    q = torch.zeros((qs.shape[0], ix.query_ld()), dtype=torch.float32, device=dev)
    q[:, : qs.shape[1]] = torch.from_numpy(qs).to(dev)
    ids = torch.empty((qs.shape[0], k), dtype=torch.int64, device=dev)
    ds = torch.empty((qs.shape[0], k), dtype=torch.float32, device=dev)
    n = torch.empty(qs.shape[0], dtype=torch.int32, device=dev)
    return q, ids, ds, n


@pytest.mark.parametrize("mode", ["exact", "hnsw"])
def test_device_batch_returns_before_the_gpu_finishes(mode):
    n, d, nq, k = 400_000, 128, 10_000, 10
    rng = np.random.default_rng(1)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((nq, d), dtype=np.float32)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n, max_connections=16)
    ix.upload_vectors(base)
    if mode == "hnsw":
        ix.build_graph(ef_construction=64, batch_div=32)
    q, ids, ds, cnt = _dev_batch(ix, qs, k, mode)
    stream = torch.cuda.Stream()   # a real stream (the default stream's handle is 0 = the index's own)
    ix.search_batch_device(q.data_ptr(), nq, k, ids.data_ptr(), ds.data_ptr(), cnt.data_ptr(), ef=64, mode=mode,
                           stream=stream.cuda_stream)   # warm: buffers allocated, images built
    torch.cuda.synchronize()
    assert stream.cuda_stream != 0
    busy = 0
    for _ in range(3):
        ix.search_batch_device(q.data_ptr(), nq, k, ids.data_ptr(), ds.data_ptr(), cnt.data_ptr(), ef=64, mode=mode,
                               stream=stream.cuda_stream)
        busy += not stream.query()   # still working when the call returned
        torch.cuda.synchronize()
    assert busy == 3
    # and the queued results are the synchronous ones
    hi, hd, hn = ix.search_batch(qs[:500], k, ef=64, mode=mode)
    assert ids.cpu().numpy()[:500].view(np.uint64).tolist() == hi.tolist()
    ix.close()


@pytest.mark.parametrize("k", [10, 100])
def test_device_fallback_with_massive_ties_equals_full_sort(k):
    """Binary 6-d data: 64 distinct rows, ~300 copies each, so thousands of
    rows tie at the k-th distance -- the fallback filter overflows and the
    device full-scan slot (radix select + ordered collection) answers: the
    (dist, id) order of a full sort, as exact_full computes it."""
    rng = np.random.default_rng(2)
    n, d = 20_000, 6
    base = rng.integers(0, 2, (n, d)).astype(np.float32)
    qs = rng.integers(0, 2, (300, d)).astype(np.float32)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    ix.upload_vectors(base)
    dead = rng.choice(n, 500, replace=False)
    ix.add_tombstones(dead)
    ids, ds, cnt = ix.search_batch(qs, k, mode="exact")
    if k == 10:   # (k = 100 runs 2k+ short lists: all ~300 tied rows re-ranked, certified without a fallback)
        assert ix.last_batch_stats()["fallbacks"] > 0
    alive = np.ones(n, bool)
    alive[dead] = False
    for i in range(len(qs)):
        full = ((base.astype(np.float64) - qs[i].astype(np.float64)) ** 2).sum(1)
        full[~alive] = np.inf
        order = np.lexsort((np.arange(n), full))[:k]
        assert ids[i].tolist() == order.tolist()
        assert ds[i].tolist() == full[order].astype(np.float32).tolist()
    ix.close()


def test_device_fallback_on_sift_like_ties_matches_restatement():
    rng = np.random.default_rng(21)
    base = rng.integers(0, 3, (20000, 16)).astype(np.float32)
    qs = rng.integers(0, 3, (200, 16)).astype(np.float32)
    ix = W.GPUVectorIndex(16, "l2-squared", capacity=20000)
    ix.upload_vectors(base)
    q, ids, ds, cnt = _dev_batch(ix, qs, 10, "exact")
    ix.search_batch_device(q.data_ptr(), len(qs), 10, ids.data_ptr(), ds.data_ptr(), cnt.data_ptr(), mode="exact")
    torch.cuda.synchronize()
    assert ix.last_batch_stats()["fallbacks"] > 0
    oi, od, on = O.flat_scan(O.L2, base, qs, 10)
    gi = ids.cpu().numpy().view(np.uint64)
    gd = ds.cpu().numpy()
    for i in range(len(qs)):
        same_tie_aware(gi[i], gd[i], oi[i], od[i])
    ix.close()


def test_null_stream_call_orders_after_default_stream_writes():
    """stream=NULL queues on the index's own non-blocking stream; the query
    rows a torch kernel has just written on the legacy default stream must
    still be read complete (the call records an event on stream 0 and waits
    for it).  The queries are produced by a chain of default-stream kernels
    that takes far longer than the launch, so a missing wait reads zeros."""
    n, d, nq, k = 200_000, 128, 4096, 10
    rng = np.random.default_rng(5)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((nq, d), dtype=np.float32)
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    ix.upload_vectors(base)
    dev = torch.device("cuda:0")
    ld = ix.query_ld()
    src = torch.zeros((nq, ld), dtype=torch.float32, device=dev)
    src[:, :d] = torch.from_numpy(qs).to(dev)
    ids = torch.empty((nq, k), dtype=torch.int64, device=dev)
    ds = torch.empty((nq, k), dtype=torch.float32, device=dev)
    cnt = torch.empty(nq, dtype=torch.int32, device=dev)
    big = torch.randn(4096, 4096, device=dev)
    for _ in range(3):
        q = torch.zeros_like(src)
        torch.cuda.synchronize()
        assert torch.cuda.current_stream().cuda_stream == 0
        for _ in range(20):          # ~ms of default-stream work ahead of the query write
            big = torch.tanh(big @ big)
        q.copy_(src)                 # the query rows land only after that
        ix.search_batch_device(q.data_ptr(), nq, k, ids.data_ptr(), ds.data_ptr(), cnt.data_ptr(), mode="exact")
        torch.cuda.synchronize()
        hi, hd, hn = ix.search_batch(qs[:256], k, mode="exact")
        assert ids.cpu().numpy()[:256].view(np.uint64).tolist() == hi.tolist()
    ix.close()
