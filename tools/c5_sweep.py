"""C5 shard sweep (one GPU's 1/8 of 100M x 96): the HNSW kernel's per-wave LDS
budget (visited-cache size) vs QPS and distance evaluations, on one graph
built once on the GPU.  Prints one JSON line per (wave_kb, ef)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import weaviate_amd as W  # noqa: E402
from bench import counter_sift  # noqa: E402

N = int(os.environ.get("C5_ROWS", 12_500_000))
D, NQ, K = 96, 10_000, 10
t0 = time.time()
base = counter_sift(1, 0, N, D)
qs = counter_sift(2, 0, NQ, D)
print(json.dumps({"data_s": round(time.time() - t0, 1)}), flush=True)
ix = W.GPUVectorIndex(D, "l2-squared", capacity=N, max_connections=64)
ix.upload_vectors(base)
del base
t0 = time.time()
ix.build_graph(ef_construction=128, seed=1, batch_div=64)
torch.cuda.synchronize()
print(json.dumps({"build_s": round(time.time() - t0, 1)}), flush=True)
dev = torch.device("cuda:0")
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
q = torch.zeros((NQ, ix.query_ld()), dtype=torch.float32, device=dev)
q[:, :D] = torch.from_numpy(qs).to(dev)
ids = torch.empty((NQ, K), dtype=torch.int64, device=dev)
ds = torch.empty((NQ, K), dtype=torch.float32, device=dev)
cn = torch.empty(NQ, dtype=torch.int32, device=dev)
truth = None
ix.search_batch_device(q.data_ptr(), NQ, K, ids.data_ptr(), ds.data_ptr(), cn.data_ptr(), mode="exact",
                       stream=stream.cuda_stream)
torch.cuda.synchronize()
truth = ids.cpu().numpy()
for ef in (64, 128):
    for kb in os.environ.get("C5_KB", "8 12 16 24").split():
        os.environ["WV_HNSW_WAVE_KB"] = kb
        ix.set_timing(True)
        for _ in range(2):
            ix.search_batch_device(q.data_ptr(), NQ, K, ids.data_ptr(), ds.data_ptr(), cn.data_ptr(), ef=ef,
                                   mode="hnsw", stream=stream.cuda_stream)
        torch.cuda.synchronize()
        ix.last_kernel_times()
        t0 = time.perf_counter()
        for _ in range(5):
            ix.search_batch_device(q.data_ptr(), NQ, K, ids.data_ptr(), ds.data_ptr(), cn.data_ptr(), ef=ef,
                                   mode="hnsw", stream=stream.cuda_stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        kt = ix.last_kernel_times()
        st = ix.last_batch_stats()
        got = ids.cpu().numpy()
        rec = float(np.mean([len(set(a) & set(b)) / K for a, b in zip(got.tolist(), truth.tolist())]))
        e, x = st["dist_evals"] / NQ, st["expansions"] / NQ
        by = (4.0 * D * st["dist_evals"] + 4.0 * 128 * st["expansions"]) / (kt["hnsw_ms"] * 1e-3) / 1e9
        print(json.dumps({"ef": ef, "wave_kb": int(kb), "qps": round(NQ / dt), "kernel_ms": round(kt["hnsw_ms"], 3),
                          "recall": round(rec, 4), "gpu_evals_per_q": round(e, 1), "exp_per_q": round(x, 1),
                          "gpu_count_GBs": round(by, 1), "fallbacks": st["fallbacks"]}), flush=True)
        ix.set_timing(False)
