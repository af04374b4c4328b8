"""Filtered-HNSW probe (measurement infrastructure): the configs[0] graph
(1M SIFT-shaped rows, M=64, efConstruction=128, built on the GPU) searched
with a shared Bernoulli(p) allow list (seed 3) at ef 64, under a list of
environment settings of the side-register path (WV_HNSW_SIDE_KB etc.):
kernel time, GPU distance evaluations, second-pass queries and exact
fallbacks per setting.  Usage: python tools/filtered_probe.py [N] [settings...]
where a setting is KEY=VAL[,KEY=VAL] or "-" (defaults)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import weaviate_amd as W  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
settings = sys.argv[2:] or ["-"]
D, NQ, K, EF = 128, 10_000, 10, 64
t0 = time.time()
base = bench._par_rows(bench.counter_sift, 1, 0, N, D)
qs = bench.counter_sift(2, 0, NQ, D)
ix = W.GPUVectorIndex(D, "l2-squared", capacity=N, max_connections=64)
ix.upload_vectors(base)
ix.build_graph(ef_construction=128, seed=1, batch_div=64)
print(f"graph built {time.time() - t0:.1f} s", flush=True)
fracs = [float(x) for x in os.environ.get("PROBE_FRACS", "0.5,0.1,0.01").split(",") if x]
# PROBE_TOMB=f1,f2: unfiltered searches with a fraction f of the ids
# tombstoned (seed 5), 10k-query batches and 1-query latency
for tf in [float(x) for x in os.environ.get("PROBE_TOMB", "").split(",") if x]:
    ix.set_tombstones([])
    if tf > 0:
        ix.add_tombstones(np.nonzero(bench.counter_uniform(5, 0, N, 1)[:, 0] < tf)[0])
    for s in settings:
        env = {} if s == "-" else dict(kv.split("=", 1) for kv in s.split(","))
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            ix.set_timing(True)
            ix.search_batch(qs, K, ef=EF, mode="hnsw")
            kms = []
            for _ in range(3):
                ix.search_batch(qs, K, ef=EF, mode="hnsw")
                kms.append(ix.last_kernel_times()["hnsw_ms"])
            st, ss = ix.last_batch_stats(), ix.last_side_stats()
            ix.set_timing(False)
            lat = []
            for i in range(200):
                t1 = time.perf_counter()
                ix.search_batch(qs[i:i + 1], K, ef=EF, mode="hnsw")
                lat.append((time.perf_counter() - t1) * 1e6)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        print(f"tombstones {tf:.0%} [{s}]: hnsw {np.median(kms):.3f} ms ({NQ / np.median(kms) * 1e3:,.0f} QPS), "
              f"gpu evals/q {st['dist_evals'] / NQ:.0f}, side {ss['side_rows']}x64, redone {ss['redone']}, "
              f"fallbacks {st['fallbacks']}; 1-query call p50 {np.median(lat):.0f} us", flush=True)
ix.set_tombstones([])
for frac in fracs:
    keep = bench.counter_uniform(3, 0, N, 1)[:, 0] < frac
    allow = W.AllowList.from_ids(np.nonzero(keep)[0], N)
    nq = NQ if frac >= 0.05 else 1000
    for s in settings:
        env = {} if s == "-" else dict(kv.split("=", 1) for kv in s.split(","))
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            ix.set_timing(True)
            ix.search_batch(qs[:nq], K, ef=EF, allow=allow, mode="hnsw")   # warm
            kms = []
            for _ in range(3):
                ix.search_batch(qs[:nq], K, ef=EF, allow=allow, mode="hnsw")
                kms.append(ix.last_kernel_times()["hnsw_ms"])
            st, ss = ix.last_batch_stats(), ix.last_side_stats()
            ix.set_timing(False)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        print(f"allow {frac:.0%} [{s}] nq {nq}: hnsw {np.median(kms):.2f} ms ({nq / np.median(kms) * 1e3:,.0f} QPS), "
              f"gpu evals/q {st['dist_evals'] / nq:.0f}, exp/q {st['expansions'] / nq:.0f}, side {ss['side_rows']}x64 "
              f"spill {ss['spill_cap']}, overflowed {ss['overflowed']}, redone {ss['redone']}, claims/q {ss['claims'] / nq:.0f}, "
              f"fallbacks {st['fallbacks']}", flush=True)
ix.close()
