"""Host-path latency of a multi-member group (diagnostic): a 2-member
shard-layout group on one device ([0, 0]: the copy path), 200k x 128 rows,
batches of 1 / 16 / 256 queries through wv_group_search_batch (exact).
`python tools/group_latency.py [lib.so]`."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import weaviate_amd as W  # noqa: E402
from weaviate_amd import _lib  # noqa: E402


def load(path):
    L = C.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    _lib._lib = L


path = sys.argv[1] if len(sys.argv) > 1 else _lib.LIBPATH
load(path)
rng = np.random.default_rng(3)
n, d = 200_000, 128
base = rng.random((n, d), dtype=np.float32)
qs = rng.random((2048, d), dtype=np.float32)
g = W.GPUGroup([0, 0], d, "l2-squared", capacity=n, layout="shard")
g.upload_vectors(base)
for nq in (1, 16, 256):
    for _ in range(5):
        g.search_batch(qs[:nq], 10, mode="exact")
    ts = []
    for r in range(60):
        q = qs[(r * nq) % (2048 - nq):][:nq]
        t = time.perf_counter()
        g.search_batch(q, 10, mode="exact")
        ts.append(time.perf_counter() - t)
    ts.sort()
    print(f"{os.path.basename(path)} nq={nq}: p50 {1e6 * ts[len(ts) // 2]:.0f} us  p90 {1e6 * ts[int(len(ts) * 0.9)]:.0f} us",
          flush=True)
g.close()
