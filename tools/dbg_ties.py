# order-dependence check: the integer-tie exact search after other indexes ran
import sys, os, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/oracle')
import weaviate_amd as W, pyoracle as O

def ties(tag):
    rng = np.random.default_rng(21)
    base = rng.integers(0, 3, (20000, 16)).astype(np.float32)
    qs = rng.integers(0, 3, (200, 16)).astype(np.float32)
    ix = W.GPUVectorIndex(16, "l2-squared", capacity=20000)
    ix.upload_vectors(base)
    ids, ds, n = ix.search_batch(qs, 10, mode="exact")
    st = ix.last_batch_stats()
    bad = 0
    for i in range(len(qs)):
        full = ((base.astype(np.float64) - qs[i].astype(np.float64)) ** 2).sum(1)
        order = np.lexsort((np.arange(len(base)), full))[:10]
        bad += ids[i].tolist() != order.tolist()
    print(tag, st, "queries with wrong (dist,id) order:", bad, flush=True)
    ix.close()

def mfma(metric):
    rng = np.random.default_rng(1)
    base = rng.random((20000, 128), dtype=np.float32)
    qs = rng.random((300, 128), dtype=np.float32)
    ix = W.GPUVectorIndex(128, metric, capacity=20000)
    ix.upload_vectors(base)
    ids, ds, n = ix.search_batch(qs, 10, mode="exact")
    print(metric, ix.last_batch_stats(), flush=True)
    ix.close()

ties("first")
for m in ("l2-squared", "dot", "cosine-dot"):
    mfma(m)
ties("after-mfma")
mfma("l2-squared")
ties("after-one-l2")
