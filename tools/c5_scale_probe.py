"""Timing probe for the configs[4] shard sizes (diagnostic): SIFT-shaped rows
generated as bench.py does, uploaded, graph built on the GPU, one search."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
import weaviate_amd as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
t = time.time()
base = bench.counter_sift(1, 0, n, 96)
print(f"gen {n:,} rows: {time.time() - t:.1f} s", flush=True)
t = time.time()
ix = W.GPUVectorIndex(96, "l2-squared", capacity=n, max_connections=64)
ix.upload_vectors(base)
print(f"upload: {time.time() - t:.1f} s", flush=True)
t = time.time()
ix.build_graph(ef_construction=128, seed=1, batch_div=64)
print(f"build: {time.time() - t:.1f} s", flush=True)
q = bench.counter_sift(2, 0, 10000, 96)
t = time.time()
ids, ds, cnt = ix.search_batch(q, 10, ef=64, mode="hnsw")
print(f"search 10k: {time.time() - t:.2f} s", flush=True)
ix.close()
