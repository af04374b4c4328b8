"""Which HIP API calls block inside wv_search_batch_device (exact / hnsw)?
Run under rocprofv3 --hip-trace; prints host-side call durations."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import weaviate_amd as W  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "exact"
n, d, nq, k = 400_000, 128, 10_000, 10
rng = np.random.default_rng(1)
ix = W.GPUVectorIndex(d, "l2-squared", capacity=n, max_connections=16)
ix.upload_vectors(rng.random((n, d), dtype=np.float32))
if mode == "hnsw":
    ix.build_graph(ef_construction=64, batch_div=32)
dev = torch.device("cuda:0")
q = torch.rand((nq, ix.query_ld()), device=dev)
ids = torch.empty((nq, k), dtype=torch.int64, device=dev)
ds = torch.empty((nq, k), dtype=torch.float32, device=dev)
cn = torch.empty(nq, dtype=torch.int32, device=dev)
s = torch.cuda.Stream()
for i in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ix.search_batch_device(q.data_ptr(), nq, k, ids.data_ptr(), ds.data_ptr(), cn.data_ptr(), ef=64, mode=mode,
                           stream=s.cuda_stream)
    t1 = time.perf_counter()
    busy = not s.query()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{mode} call {i}: host {1e3*(t1-t0):.3f} ms, busy after return {busy}, total {1e3*(t2-t0):.3f} ms",
          flush=True)
