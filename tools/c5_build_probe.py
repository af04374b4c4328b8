"""Diagnostic: GPU graph build time vs shard size (configs[4]).  SIFT-shaped
96-d rows generated on the device (tools/wv_synth.hip), uploaded from device
memory, graph built with WV_BUILD_TRACE=1 (per-phase device times every 64
batches on stderr)."""
import os
import sys
import time

os.environ.setdefault("WV_BUILD_TRACE", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402
import synth  # noqa: E402
import weaviate_amd as W  # noqa: E402

for n in [int(x) for x in sys.argv[1:]] or [12_500_000]:
    t = time.time()
    rows = torch.empty((n, 96), dtype=torch.float32, device="cuda")
    synth.fill("sift", 1, 0, rows)
    torch.cuda.synchronize()
    print(f"[probe] n={n:,} gen {time.time() - t:.2f} s", flush=True)
    t = time.time()
    ix = W.GPUVectorIndex(96, "l2-squared", capacity=n, max_connections=64)
    ix.upload_vectors_device(rows.data_ptr(), n)
    del rows
    torch.cuda.synchronize()
    print(f"[probe] upload {time.time() - t:.2f} s", flush=True)
    t = time.time()
    ix.build_graph(ef_construction=128, seed=1, batch_div=64)
    print(f"[probe] n={n:,} build {time.time() - t:.1f} s", flush=True)
    ix.close()
    torch.cuda.empty_cache()
