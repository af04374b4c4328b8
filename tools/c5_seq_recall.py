"""The GPU half of north_star's recall check on a configs[4]-shaped corpus
(measurement infrastructure; the sequential half: tools/c5_seq_recall_cpu.py,
whose insert-by-insert build of 10M rows outlasts one GPU session).

  python tools/c5_seq_recall.py [N=10_000_000] [NQ=1000]

SIFT/Deep-shaped 96-d rows (bench.counter_sift, seed 1), queries seed 2,
M = 64, efConstruction = 128.  The graph: wv_index_build_graph with the C5
line's batch = inserted / 64; searched at ef 64 and 128; truth = the exact
path (bit-identical to the restatement's flatSearch, the GPU suite), so the
two halves' recalls compare on the same truth."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import weaviate_amd as W  # noqa: E402

N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
NQ = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
D, K, M, EFC = 96, 10, 64, 128
t0 = time.time()
base = bench._par_rows(bench.counter_sift, 1, 0, N, D)
qs = bench.counter_sift(2, 0, NQ, D)
print(f"data {N} x {D}: {time.time() - t0:.0f} s", flush=True)
ix = W.GPUVectorIndex(D, "l2-squared", capacity=N, max_connections=M)
ix.upload_vectors(base)
truth = ix.search_batch(qs, K, mode="exact")[0]
t1 = time.time()
ix.build_graph(ef_construction=EFC, seed=1, batch_div=64)
print(f"GPU build: {time.time() - t1:.1f} s", flush=True)
for ef in (64, 128):
    gi = ix.search_batch(qs, K, ef=ef, mode="hnsw")[0]
    r = float(np.mean([len(set(a) & set(b)) / K for a, b in zip(gi.tolist(), truth.tolist())]))
    print(f"ef {ef}: recall@10 GPU search on the GPU-built graph {r:.4f} ({NQ} queries)", flush=True)
np.save(os.path.join(ROOT, "gpurun_out", "c5_truth_%d.npy" % N), truth)
ix.close()
