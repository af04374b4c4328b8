"""Investigate GPU-vs-restatement HNSW differences on a deterministic graph:
prints every query whose top-k differs, with both (id, dist) lists."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as O
import weaviate_amd as W
from bench import counter_uniform

n, d, nq = int(sys.argv[1]), 128, int(sys.argv[2])
base = counter_uniform(1, 0, n, d)
qs = counter_uniform(2, 0, nq, d)
ref = O.Index(d, "l2-squared", 64, 128, capacity=n, seed=1)
ref.add_batch(base, threads=16)
g = ref.export_graph()
ix = W.GPUVectorIndex(d, "l2-squared", capacity=n, max_connections=64)
ix.upload_vectors(base)
ix.upload_graph(g)
for ef in (64, 128):
    gi, gd, gn = ix.search_batch(qs, 10, ef=ef, mode="hnsw")
    oi, od, on, st = ref.search_batch(qs, 10, ef, threads=16)
    bad = [i for i in range(nq) if not (np.array_equal(gi[i], oi[i]) and np.array_equal(gd[i].view(np.uint32), od[i].view(np.uint32)))]
    print(f"ef={ef}: {len(bad)} of {nq} queries differ", flush=True)
    for i in bad[:5]:
        print(" q", i)
        print("  gpu", list(zip(gi[i].tolist(), gd[i].tolist())))
        print("  cpu", list(zip(oi[i].tolist(), od[i].tolist())))
        # single-query re-runs (the GPU batch path vs a batch of one)
        a = ix.search_batch(qs[i:i+1], 10, ef=ef, mode="hnsw")
        print("  gpu single", list(zip(a[0][0].tolist(), a[1][0].tolist())) == list(zip(gi[i].tolist(), gd[i].tolist())))
        print("  restatement tie-dependent decisions:", ref.knn_search(qs[i], 10, ef, with_stats=True)[2]["ties"])
    good = [i for i in range(0, nq, 97) if i not in bad]
    print(" queries with tie-dependent decisions among matching ones:",
          sum(ref.knn_search(qs[i], 10, ef, with_stats=True)[2]["ties"] > 0 for i in good), "of", len(good))
    # the lossy visited cache must never change a result: vary its size
    for kb in (6, 32):
        os.environ["WV_HNSW_WAVE_KB"] = str(kb)
        hi, hd, hn = ix.search_batch(qs, 10, ef=ef, mode="hnsw")
        print(f" visited-cache size invariance (WV_HNSW_WAVE_KB={kb}):",
              bool((hi == gi).all() and (hd.view(np.uint32) == gd.view(np.uint32)).all()))
    os.environ.pop("WV_HNSW_WAVE_KB")
