"""Open-loop A/B of the micro-batcher's refill wait (measurement
infrastructure): the C1 graph (1M SIFT-shaped rows, M = 64, built on the
GPU), closed-loop capacity at T = 256, then Poisson arrivals at 10 % and
50 % of it (tests/native/libwvload.so wvl_open_loop) with the refill wait
gated on resubmissions (default) and ungated (WV_BATCHER_REFILL_GAP_US=-1,
round 5: wait up to min(300, 50 + n) us for the last batch's callers).
Usage: python tools/open_loop_ab.py [N]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import weaviate_amd as W  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
D, K, EF = 128, 10, 64
base = bench._par_rows(bench.counter_sift, 1, 0, N, D)
qs = np.ascontiguousarray(bench.counter_sift(2, 0, 10_000, D))
ix = W.GPUVectorIndex(D, "l2-squared", capacity=N, max_connections=64)
ix.upload_vectors(base)
ix.build_graph(ef_construction=128, seed=1, batch_div=64)
ix.update_user_config(ef=EF)
lib = C.CDLL(os.path.join(ROOT, "tests", "native", "libwvload.so"))
lib.wvl_concurrent.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int,
                               C.c_int, C.c_void_p]
lib.wvl_open_loop.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int,
                              C.c_int, C.c_void_p]
h = C.c_void_p(ix._h.value if hasattr(ix._h, "value") else ix._h)
r = np.zeros(8, np.float64)
assert lib.wvl_concurrent(h, qs.ctypes.data, len(qs), D, K, 256, 2.0, 1024, 0, r.ctypes.data) == 0
cap = r[0]
print(f"closed loop T=256: {cap:,.0f} QPS, p50 {r[1]:.0f} us", flush=True)
for gap in ("40", "-1"):
    os.environ["WV_BATCHER_REFILL_GAP_US"] = gap
    for f in (0.02, 0.1, 0.5):
        r[:] = 0
        assert lib.wvl_open_loop(h, qs.ctypes.data, len(qs), D, K, f * cap, 2.0, 1024, 512, r.ctypes.data) == 0
        print(f"refill gap {gap:>3} us, Poisson at {f:4.0%} of capacity ({f * cap:,.0f} QPS): achieved {r[0]:,.0f}, "
              f"p50 {r[1]:.0f} us, p99 {r[2]:.0f}, p99.9 {r[3]:.0f}, max {r[4]:.0f}, mean batch {r[5]:.1f}, "
              f"late starts {int(r[7])}", flush=True)
ix.close()
