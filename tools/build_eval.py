"""GPU graph construction vs the restatement's sequential build: build time
and recall@10 on the same data (bench.py's counter-based generators)."""
import os, sys, time, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as O
import weaviate_amd as W
from bench import counter_uniform

n, d, M, efc = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
divs = [int(x) for x in sys.argv[5].split(",")] if len(sys.argv) > 5 else [32]
cpu = len(sys.argv) > 6 and sys.argv[6] == "cpu"
base = counter_uniform(1, 0, n, d)
qs = counter_uniform(2, 0, 2000, d)
truth, _, _ = O.flat_scan(O.L2, base, qs, 10, threads=16)
rec = lambda ids: float(np.mean([len(set(a) & set(b)) / 10 for a, b in zip(ids.tolist(), truth.tolist())]))
out = {"n": n, "dim": d, "M": M, "efC": efc}
for div in divs:
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n, max_connections=M)
    ix.upload_vectors(base)
    t0 = time.time(); ix.build_graph(ef_construction=efc, seed=1, batch_div=div); tb = time.time() - t0
    r = {}
    for ef in (64, 128, 256):
        gi, gd, gn = ix.search_batch(qs, 10, ef=ef, mode="hnsw")
        r[ef] = round(rec(gi), 4)
    out[f"gpu_div{div}"] = {"build_s": round(tb, 2), "recall": r}
    print(json.dumps(out), flush=True)
    ix.close()
if cpu:
    t0 = time.time()
    ref = O.Index(d, "l2-squared", M, efc, capacity=n, seed=1)
    ref.add_batch(base, threads=16)
    tb = time.time() - t0
    r = {}
    for ef in (64, 128, 256):
        oi, od, on, _ = ref.search_batch(qs, 10, ef, threads=16)
        r[ef] = round(rec(oi), 4)
    out["cpu_restatement_16t"] = {"build_s": round(tb, 2), "recall": r}
print(json.dumps(out), flush=True)
