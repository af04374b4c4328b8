import sys; sys.path.insert(0,'.'); sys.path.insert(0,'oracle')
import numpy as np, pyoracle as O, weaviate_amd as W
for dim in (3, 31, 777):
    rng = np.random.default_rng(dim)
    base = rng.random((257, dim), dtype=np.float32); qs = rng.random((4, dim), dtype=np.float32)
    ix = W.GPUVectorIndex(dim, "l2-squared", capacity=257); ix.upload_vectors(base)
    ids, ds, n = ix.search_batch(qs, 40, mode="exact")
    oi, od, on = O.flat_scan(O.L2, base, qs, 40)
    q=qs[0]; i=int(oi[0,0]); 
    g=ds[0][ids[0]==i]
    print(dim, "oracle", od[0,0], "gpu", g, "f64", ((base[i].astype(np.float64)-q)**2).sum(), "purego", O.distance(O.L2, base[i], q, 'purego'), O.distance(O.L2, q, base[i]))
