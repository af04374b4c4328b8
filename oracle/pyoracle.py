"""ctypes binding of the CPU restatement (oracle/libwvoracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package weaviate_amd.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIBPATH = os.path.join(_HERE, "libwvoracle.so")

L2, DOT, COSINE = 0, 1, 2
METRICS = {"l2-squared": L2, "dot": DOT, "cosine-dot": COSINE}


class Stats(C.Structure):
    _fields_ = [
        ("dist_evals", C.c_uint64),
        ("expansions", C.c_uint64),
        ("nbr_slots", C.c_uint64),
        ("visited", C.c_uint64),
        ("max_cand", C.c_uint64),
        ("layer0_visited_max", C.c_uint64),
        ("ties", C.c_uint64),
        ("side_live_max", C.c_uint64),
        ("side_exp", C.c_uint64),
        ("side_exp_max", C.c_uint64),
    ]

    def asdict(self):
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIBPATH):
            build()
        L = C.CDLL(_LIBPATH)
        fp, u64p, i32p = C.POINTER(C.c_float), C.POINTER(C.c_uint64), C.POINTER(C.c_int)
        vp = C.c_void_p
        sig = {
            "wvo_distance": (C.c_float, [C.c_int, fp, fp, C.c_int]),
            "wvo_distance_avx2": (C.c_float, [C.c_int, fp, fp, C.c_int]),
            "wvo_distance_purego": (C.c_float, [C.c_int, fp, fp, C.c_int]),
            "wvo_asm_l2": (C.c_float, [fp, fp, C.c_int]),
            "wvo_asm_dot": (C.c_float, [fp, fp, C.c_int]),
            "wvo_normalize": (None, [fp, fp, C.c_int]),
            "wvo_normalize_rows": (None, [fp, fp, C.c_uint64, C.c_int]),
            "wvo_pq_script": (C.c_int, [C.c_int, C.c_int, i32p, u64p, fp, u64p, fp]),
            "wvo_search_time_ef": (C.c_int, [C.c_int64] * 4 + [C.c_int]),
            "wvo_create": (vp, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_uint64]),
            "wvo_destroy": (None, [vp]),
            "wvo_set_search_config": (None, [vp] + [C.c_int64] * 5 + [C.c_int]),
            "wvo_set_vector": (C.c_int, [vp, C.c_uint64, fp]),
            "wvo_add": (C.c_int, [vp, C.c_uint64, fp]),
            "wvo_add_batch": (C.c_int, [vp, C.c_uint64, fp, C.c_uint64, C.c_int]),
            "wvo_set_next_level": (None, [vp, C.c_int]),
            "wvo_add_tombstone": (C.c_int, [vp, C.c_uint64]),
            "wvo_remove_tombstone": (C.c_int, [vp, C.c_uint64]),
            "wvo_import_node": (C.c_int, [vp, C.c_uint64, C.c_int, u64p, i32p]),
            "wvo_set_entrypoint": (None, [vp, C.c_uint64, C.c_int]),
            "wvo_log_enable": (None, [vp, C.c_int]),
            "wvo_log_size": (C.c_uint64, [vp]),
            "wvo_log_copy": (C.c_uint64, [vp, vp, C.c_uint64]),
            "wvo_import_csr": (C.c_int, [vp, C.c_uint64, fp, vp, vp, C.c_int, vp, vp, C.c_int, C.c_int,
                                         C.c_uint64]),
            "wvo_graph_info": (None, [vp, u64p, u64p, i32p, u64p]),
            "wvo_export_layer0": (C.c_int, [vp, C.c_int, vp, vp, vp]),
            "wvo_export_upper": (C.c_int, [vp, C.c_int, C.c_int, vp, vp, C.c_uint64]),
            "wvo_search_by_vector": (C.c_int, [vp, fp, C.c_int, u64p, C.c_uint64, u64p, fp, i32p, C.POINTER(Stats)]),
            "wvo_knn_search": (C.c_int, [vp, fp, C.c_int, C.c_int, u64p, C.c_uint64, u64p, fp, i32p, C.POINTER(Stats)]),
            "wvo_flat_search": (C.c_int, [vp, fp, C.c_int, u64p, C.c_uint64, u64p, fp, i32p]),
            "wvo_search_by_vector_distance": (C.c_int, [vp, fp, C.c_float, C.c_int64, u64p, C.c_uint64, u64p, fp, C.c_int64, C.POINTER(C.c_int64)]),
            "wvo_search_batch": (C.c_int, [vp, fp, C.c_int, C.c_int, C.c_int, u64p, C.c_uint64, C.c_int, C.c_int, u64p, fp, i32p, C.POINTER(Stats)]),
            "wvo_flat_scan": (C.c_int, [C.c_int, fp, C.c_uint64, C.c_int, fp, C.c_int, C.c_int, u64p, u64p, C.c_int, u64p, fp, i32p]),
            "wvo_pq_layout": (C.c_int, [C.c_int, C.c_int, i32p, i32p]),
            "wvo_pq_extract": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, u64p]),
            "wvo_pq_put": (C.c_int, [u64p, C.c_int, C.c_int, C.c_int, vp]),
            "wvo_pq_distance": (C.c_float, [C.c_int, fp, vp, fp, C.c_int, C.c_int, C.c_int, C.c_int]),
            "wvo_pq_encode_kmeans": (C.c_int, [fp, C.c_uint64, C.c_int, C.c_int, C.c_int, fp, C.c_int, vp]),
            "wvo_compress": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, fp, vp, vp, C.c_uint64]),
            "wvo_set_side_diag": (None, [C.c_int]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _u64(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_uint64))


def _i32(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def f32(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.float32))


def distance(metric, a, b, impl="asm"):
    a, b = f32(a), f32(b)
    fn = {"asm": lib().wvo_distance, "avx2": lib().wvo_distance_avx2, "purego": lib().wvo_distance_purego}[impl]
    return float(np.float32(fn(metric, _f(a), _f(b), len(a))))


def normalize(v):
    v = f32(v)
    out = np.empty_like(v)
    lib().wvo_normalize(_f(v), _f(out), len(v))
    return out


def normalize_rows(a):
    """Normalize (distancer/normalize.go:16-32) applied to every row."""
    a = f32(a)
    out = np.empty_like(a)
    lib().wvo_normalize_rows(_f(a), _f(out), a.shape[0], a.shape[1])
    return out


def pq_script(is_max, ops):
    """ops: list of ("insert", id, dist) / ("pop",)."""
    n = len(ops)
    op = np.array([0 if o[0] == "insert" else 1 for o in ops], dtype=np.int32)
    ids = np.array([o[1] if o[0] == "insert" else 0 for o in ops], dtype=np.uint64)
    ds = np.array([o[2] if o[0] == "insert" else 0 for o in ops], dtype=np.float32)
    oi = np.zeros(n, np.uint64)
    od = np.zeros(n, np.float32)
    m = lib().wvo_pq_script(int(is_max), n, _i32(op), _u64(ids), _f(ds), _u64(oi), _f(od))
    return list(zip(oi[:m].tolist(), od[:m].tolist()))


def pq_layout(ks, use_bits=False):
    """(bits, bytes) of NewProductQuantizer (product_quantization.go:116-179)."""
    b, y = C.c_int(), C.c_int()
    assert lib().wvo_pq_layout(ks, int(use_bits), C.byref(b), C.byref(y)) == 0
    return b.value, y.value


def pq_extract(enc, n_codes, ks, use_bits=False):
    """ProductQuantizer.ExtractCode for indices 0..n_codes-1 (:191-237)."""
    buf = np.zeros(len(enc) + 8, np.uint8)
    buf[: len(enc)] = np.frombuffer(bytes(enc), np.uint8)
    out = np.zeros(n_codes, np.uint64)
    assert lib().wvo_pq_extract(buf.ctypes.data, n_codes, ks, int(use_bits), _u64(out)) == 0
    return out.tolist()


def pq_put(codes, ks, use_bits=False, length=None):
    """ProductQuantizer.PutCode for codes[i] at index i (:207-258) into a
    zeroed buffer of `length` bytes (default m * bytes, as Encode allocates)."""
    codes = np.asarray(codes, np.uint64)
    n = len(codes)
    if length is None:
        length = n * pq_layout(ks, use_bits)[1]
    buf = np.zeros(length + 8, np.uint8)
    assert lib().wvo_pq_put(_u64(codes), n, ks, int(use_bits), buf.ctypes.data) == 0
    return bytes(buf[:length])


def pq_distance(metric, x, enc, cent, ks, use_bits=False):
    """DistanceBetweenCompressedAndUncompressedVectors (:284-291); cent[m][ks][ds]."""
    x, cent = f32(x), f32(cent)
    m = cent.shape[0]
    buf = np.zeros(len(enc) + 8, np.uint8)
    buf[: len(enc)] = np.frombuffer(bytes(enc), np.uint8)
    metric = METRICS[metric] if isinstance(metric, str) else metric
    return float(np.float32(lib().wvo_pq_distance(metric, _f(x), buf.ctypes.data, _f(cent), m, ks, len(x),
                                                  int(use_bits))))


def pq_encode_kmeans(vecs, cent, use_bits=False):
    """ProductQuantizer.Encode with KMeans encoders: uint8[n][m * bytes]."""
    vecs, cent = f32(vecs), f32(cent)
    m, ks = cent.shape[0], cent.shape[1]
    n, dim = vecs.shape
    _, nbytes = pq_layout(ks, use_bits)
    out = np.zeros((n, m * nbytes), np.uint8)
    assert lib().wvo_pq_encode_kmeans(_f(vecs), n, dim, m, ks, _f(cent), int(use_bits), out.ctypes.data) == 0
    return out


def search_time_ef(ef, ef_min, ef_max, ef_factor, k):
    return lib().wvo_search_time_ef(ef, ef_min, ef_max, ef_factor, k)


def bits_from_ids(ids, nbits):
    words = np.zeros((nbits + 63) // 64, dtype=np.uint64)
    ids = np.asarray(list(ids), dtype=np.uint64)
    if ids.size:
        np.bitwise_or.at(words, (ids >> np.uint64(6)).astype(np.int64), np.uint64(1) << (ids & np.uint64(63)))
    return words


class Index:
    """CPU restatement of the reference `hnsw` index (index.go:35-155)."""

    def __init__(self, dim, metric="l2-squared", max_connections=64, ef_construction=128,
                 capacity=1024, seed=1):
        self.dim = dim
        self.metric = METRICS[metric] if isinstance(metric, str) else metric
        self.capacity = capacity
        self.M = max_connections
        self.h = lib().wvo_create(dim, self.metric, max_connections, ef_construction, capacity, seed)

    def close(self):
        if self.h:
            lib().wvo_destroy(self.h)
            self.h = None

    __del__ = close

    def set_search_config(self, ef=-1, ef_min=100, ef_max=500, ef_factor=8, flat_search_cutoff=40000,
                          forbid_flat=False):
        lib().wvo_set_search_config(self.h, ef, ef_min, ef_max, ef_factor, flat_search_cutoff,
                                    int(forbid_flat))

    def set_vector(self, id_, v):
        assert lib().wvo_set_vector(self.h, id_, _f(f32(v))) == 0

    def add(self, id_, v, level=None):
        if level is not None:
            lib().wvo_set_next_level(self.h, level)
        rc = lib().wvo_add(self.h, id_, _f(f32(v)))
        assert rc == 0, rc

    def add_batch(self, vecs, first_id=0, threads=1):
        vecs = f32(vecs)
        rc = lib().wvo_add_batch(self.h, first_id, _f(vecs), vecs.shape[0], threads)
        assert rc == 0, rc

    def add_tombstone(self, id_):
        lib().wvo_add_tombstone(self.h, id_)

    def remove_tombstone(self, id_):
        lib().wvo_remove_tombstone(self.h, id_)

    def compress(self, cent, codes, use_bits=False, has=None):
        """Compress (compress.go:39-89) with fitted centroids cent[m][ks][ds]
        and encoded vectors codes[n][m * bytes] for ids 0..n-1."""
        cent = f32(cent)
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        hs = None if has is None else np.ascontiguousarray(has, dtype=np.uint8)
        rc = lib().wvo_compress(self.h, cent.shape[0], cent.shape[1], int(use_bits), _f(cent), codes.ctypes.data,
                                None if hs is None else hs.ctypes.data, codes.shape[0])
        assert rc == 0, rc
        self._pq_keep = (cent, codes, hs)

    def import_node(self, id_, level, conns_per_level):
        flat = np.array([c for lvl in conns_per_level for c in lvl], dtype=np.uint64)
        if flat.size == 0:
            flat = np.zeros(1, np.uint64)
        counts = np.array([len(lvl) for lvl in conns_per_level], dtype=np.int32)
        assert lib().wvo_import_node(self.h, id_, level, _u64(flat), _i32(counts)) == 0

    def enable_commit_log(self, on=True):
        """Record the commit log the reference would write (logger.go)."""
        lib().wvo_log_enable(self.h, int(on))

    def commit_log(self) -> bytes:
        n = lib().wvo_log_size(self.h)
        buf = (C.c_uint8 * max(n, 1))()
        lib().wvo_log_copy(self.h, buf, n)
        return bytes(buf[:n])

    def import_graph(self, vecs, g):
        """Restore vectors + graph from export_graph()'s CSR (inverse of export)."""
        vecs = f32(vecs)
        lv = np.ascontiguousarray(g["levels"], np.int8)
        l0 = np.ascontiguousarray(g["layer0"], np.uint32)
        ur = np.ascontiguousarray(g["upper_row"], np.uint32)
        up = np.ascontiguousarray(g["upper"], np.uint32)
        rc = lib().wvo_import_csr(self.h, int(g["n"]), _f(vecs), lv.ctypes.data, l0.ctypes.data, l0.shape[1],
                                  ur.ctypes.data, up.ctypes.data, up.shape[2], int(g["max_level"]),
                                  int(g["entrypoint"]))
        assert rc == 0, rc

    def set_entrypoint(self, ep, max_level):
        lib().wvo_set_entrypoint(self.h, ep, max_level)

    def _allow(self, allow):
        if allow is None:
            return None, 0
        if isinstance(allow, np.ndarray) and allow.dtype == np.uint64:
            return allow, allow.size * 64
        return bits_from_ids(allow, self.capacity), self.capacity

    def search_by_vector(self, q, k, allow=None, with_stats=False):
        bits, nb = self._allow(allow)
        oi = np.zeros(max(k, 1), np.uint64)
        od = np.zeros(max(k, 1), np.float32)
        n = C.c_int(0)
        st = Stats()
        rc = lib().wvo_search_by_vector(self.h, _f(f32(q)), k, _u64(bits), nb, _u64(oi), _f(od),
                                        C.byref(n), C.byref(st))
        if rc:
            raise RuntimeError(f"search_by_vector rc={rc}")
        out = (oi[: n.value].copy(), od[: n.value].copy())
        return (*out, st.asdict()) if with_stats else out

    def knn_search(self, q, k, ef, allow=None, with_stats=False):
        bits, nb = self._allow(allow)
        oi = np.zeros(max(k, 1), np.uint64)
        od = np.zeros(max(k, 1), np.float32)
        n = C.c_int(0)
        st = Stats()
        rc = lib().wvo_knn_search(self.h, _f(f32(q)), k, ef, _u64(bits), nb, _u64(oi), _f(od),
                                  C.byref(n), C.byref(st))
        if rc:
            raise RuntimeError(f"knn_search rc={rc}")
        out = (oi[: n.value].copy(), od[: n.value].copy())
        return (*out, st.asdict()) if with_stats else out

    def search_by_vector_distance(self, q, target, max_limit=-1, allow=None, cap=100000):
        bits, nb = self._allow(allow)
        oi = np.zeros(cap, np.uint64)
        od = np.zeros(cap, np.float32)
        n = C.c_int64(0)
        rc = lib().wvo_search_by_vector_distance(self.h, _f(f32(q)), target, max_limit, _u64(bits), nb,
                                                 _u64(oi), _f(od), cap, C.byref(n))
        if rc:
            raise RuntimeError(f"search_by_vector_distance rc={rc}")
        m = min(n.value, cap)
        return oi[:m].copy(), od[:m].copy()

    def search_batch(self, qs, k, ef, allow=None, mode=0, threads=1):
        qs = f32(qs)
        nq = qs.shape[0]
        bits, nb = self._allow(allow)
        oi = np.zeros((nq, k), np.uint64)
        od = np.zeros((nq, k), np.float32)
        on = np.zeros(nq, np.int32)
        st = Stats()
        lib().wvo_search_batch(self.h, _f(qs), nq, k, ef, _u64(bits), nb, mode, threads, _u64(oi), _f(od),
                               _i32(on), C.byref(st))
        return oi, od, on, st.asdict()

    def export_graph(self, deg0=None, degU=None):
        """Fixed-degree CSR re-layout: dict of numpy arrays (see include/wvgpu.h)."""
        n = C.c_uint64()
        ep = C.c_uint64()
        ml = C.c_int()
        up = C.c_uint64()
        lib().wvo_graph_info(self.h, C.byref(n), C.byref(ep), C.byref(ml), C.byref(up))
        n, ep, ml, up = n.value, ep.value, ml.value, up.value
        deg0 = deg0 or 2 * self.M
        degU = degU or self.M
        levels = np.zeros(n, np.int8)
        layer0 = np.zeros((n, deg0), np.uint32)
        counts0 = np.zeros(n, np.uint32)
        over0 = lib().wvo_export_layer0(self.h, deg0, levels.ctypes.data, layer0.ctypes.data, counts0.ctypes.data)
        upper_row = np.zeros(n, np.uint32)
        upper = np.zeros((max(up, 1), max(ml, 1), degU), np.uint32)
        overU = lib().wvo_export_upper(self.h, degU, max(ml, 1), upper_row.ctypes.data, upper.ctypes.data, max(up, 1))
        if over0 or overU:
            raise ValueError("neighbour list longer than the CSR degree")
        return dict(n=n, entrypoint=ep, max_level=ml, levels=levels, layer0=layer0, counts0=counts0,
                    upper_row=upper_row, upper=upper, deg0=deg0, degU=degU)


def flat_scan(metric, base, qs, k, allow_bits=None, tomb_bits=None, threads=8):
    base, qs = f32(base), f32(qs)
    n, dim = base.shape
    nq = qs.shape[0]
    oi = np.zeros((nq, k), np.uint64)
    od = np.zeros((nq, k), np.float32)
    on = np.zeros(nq, np.int32)
    lib().wvo_flat_scan(metric, _f(base), n, dim, _f(qs), nq, k, _u64(allow_bits), _u64(tomb_bits), threads,
                        _u64(oi), _f(od), _i32(on))
    return oi, od, on
