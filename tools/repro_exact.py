"""Exact-path check against an fp64 ground truth at several batch sizes, for a
given libwvgpu.so (diagnostic: `python tools/repro_exact.py [lib.so ...]`).
Uniform 400k x 128 rows (seed 1, as tests/test_gpu_async.py); prints the
number of queries whose 10 ids differ from the truth per batch size."""
import ctypes as C
import os
import sys

import numpy as np
import torch

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


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else _lib.LIBPATH
    load(path)
    n, d = int(os.environ.get("N", 400_000)), 128
    rng = np.random.default_rng(1)
    base = rng.random((n, d), dtype=np.float32)
    qs = rng.random((10_000, d), dtype=np.float32)
    dev = torch.device("cuda:0")
    xb = torch.from_numpy(base).to(dev, torch.float64)
    xn = (xb * xb).sum(1)
    truth = []
    for i in range(0, len(qs), 500):
        q = torch.from_numpy(qs[i:i + 500]).to(dev, torch.float64)
        dd = xn[None, :] - 2.0 * q @ xb.T + (q * q).sum(1)[:, None]
        truth.append(torch.topk(dd, 10, largest=False).indices.cpu().numpy())
    truth = np.concatenate(truth)
    del xb
    ix = W.GPUVectorIndex(d, "l2-squared", capacity=n)
    ix.upload_vectors(base)
    for nq in [500, 64, 1000, 2000, 4096, 10000]:
        ids, ds, cnt = ix.search_batch(qs[:nq], 10, mode="exact")
        bad = [i for i in range(nq) if ids[i].astype(np.int64).tolist() != truth[i].tolist()]
        print(f"{os.path.basename(path)} nq={nq}: {len(bad)} wrong" + (f" (first {bad[:5]})" if bad else ""),
              flush=True)
    ix.close()


if __name__ == "__main__":
    main()
