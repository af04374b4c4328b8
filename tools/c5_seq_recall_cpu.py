"""The sequential half of tools/c5_seq_recall.py, on host cores only
(measurement infrastructure): the same configs[4]-shaped corpus
(bench.counter_sift seed 1, queries seed 2, 96-d, M = 64, efConstruction =
128), inserted in id order by the CPU restatement (insert.go:103-217;
oracle/) in 250k-row chunks, then searched by the restatement at ef 64 and
128; truth = the restatement's flatSearch (bit-identical to the GPU's exact
path, the GPU suite).  Its recall beside the GPU-built graph's recall from
`tools/c5_seq_recall.py` on the same data (both against the same
exact truth) gives north_star's 0.5-pt check at a size whose sequential
build outlasts one GPU session.

  python tools/c5_seq_recall_cpu.py [N=10_000_000] [NQ=1000] [THREADS=8]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench  # noqa: E402
import pyoracle as O  # noqa: E402

N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
NQ = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
T = int(sys.argv[3]) if len(sys.argv) > 3 else 8
D, K, M, EFC = 96, 10, 64, 128
t0 = time.time()
base = bench._par_rows(bench.counter_sift, 1, 0, N, D)
qs = bench.counter_sift(2, 0, NQ, D)
print(f"data {N} x {D}: {time.time() - t0:.0f} s", flush=True)
t1 = time.time()
truth = O.flat_scan(O.L2, base, qs, K, threads=T)[0]
print(f"exact truth (restatement flatSearch): {time.time() - t1:.0f} s", flush=True)
seq = O.Index(D, "l2-squared", M, EFC, capacity=N, seed=1)
t1 = time.time()
CH = 250_000
for i in range(0, N, CH):
    seq.add_batch(base[i:i + CH], first_id=i, threads=T)
    print(f"  sequential build: {min(N, i + CH):,} rows, {time.time() - t1:.0f} s", flush=True)
print(f"sequential build ({T} threads): {time.time() - t1:.0f} s", flush=True)
for ef in (64, 128):
    ri = seq.search_batch(qs, K, ef, threads=T)[0]
    r = float(np.mean([len(set(a) & set(b)) / K for a, b in zip(ri.tolist(), truth.tolist())]))
    print(f"ef {ef}: recall@10 restatement on the sequential graph {r:.4f} ({NQ} queries)", flush=True)
