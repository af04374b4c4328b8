"""Host-side mirror of the reference VectorIndex search interface.

adapters/repos/db/vector_index.go:23-40 declares the interface; the hnsw
package implements the search half in adapters/repos/db/vector/hnsw/search.go.
`GPUVectorIndex` exposes the same operations with the same argument meaning
and error behaviour (errors raise `WvError` where Go returns an error), backed
by libwvgpu.so.  Every search runs on the GPU; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, Optional

import numpy as np

from ._lib import MODE_AUTO, MODE_EXACT, MODE_HNSW, METRICS, WvConfig, WvError, WvGraphInfo, check, lib

_MODES = {"auto": MODE_AUTO, "exact": MODE_EXACT, "hnsw": MODE_HNSW}


def _ptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


class AllowList:
    """helpers.AllowList (adapters/repos/db/helpers/allow_list.go:19-118) as a
    dense bitmap over docIDs: Insert / Contains / Len / ascending Iterator."""

    def __init__(self, *ids: int, nbits: int = 0):
        self.nbits = max(nbits, (max(ids) + 1) if ids else 0)
        self.words = np.zeros((self.nbits + 63) // 64, dtype=np.uint64)
        if ids:
            self.insert(*ids)

    @classmethod
    def from_ids(cls, ids: Iterable[int], nbits: int) -> "AllowList":
        al = cls(nbits=nbits)
        ids = np.asarray(list(ids) if not isinstance(ids, np.ndarray) else ids, dtype=np.uint64)
        al.insert_array(ids)
        return al

    def _grow(self, nbits):
        if nbits > self.nbits:
            w = np.zeros((nbits + 63) // 64, dtype=np.uint64)
            w[: self.words.size] = self.words
            self.words, self.nbits = w, nbits

    def insert_array(self, ids: np.ndarray):
        if ids.size == 0:
            return
        self._grow(int(ids.max()) + 1)
        np.bitwise_or.at(self.words, (ids >> np.uint64(6)).astype(np.int64), np.uint64(1) << (ids & np.uint64(63)))

    def insert(self, *ids: int):
        self.insert_array(np.asarray(ids, dtype=np.uint64))

    def contains(self, id_: int) -> bool:
        return id_ < self.nbits and bool((int(self.words[id_ >> 6]) >> (id_ & 63)) & 1)

    def __len__(self):
        return int(sum(bin(int(w)).count("1") for w in self.words)) if self.words.size < 4096 else int(
            np.unpackbits(self.words.view(np.uint8)).sum())

    def iterator(self):
        for wi, w in enumerate(self.words.tolist()):
            while w:
                b = (w & -w).bit_length() - 1
                yield wi * 64 + b
                w &= w - 1


class GPUVectorIndex:
    """The GPU mirror of one shard's `hnsw` index (search side)."""

    def __init__(self, dim: int, distance: str = "cosine-dot", capacity: int = 1 << 20, *, device: int = 0,
                 max_connections: int = 64, ef: int = -1, dynamic_ef_min: int = 100, dynamic_ef_max: int = 500,
                 dynamic_ef_factor: int = 8, flat_search_cutoff: int = 40000, forbid_flat: bool = False,
                 id_base: int = 0):
        if distance not in METRICS:
            raise WvError(1, f"unsupported distance {distance!r} (l2-squared, dot, cosine-dot)")
        self.dim, self.distance, self.capacity = dim, distance, capacity
        self.cfg = WvConfig()
        lib().wv_config_default(C.byref(self.cfg))
        self.cfg.device, self.cfg.max_connections = device, max_connections
        self.cfg.ef, self.cfg.dynamic_ef_min, self.cfg.dynamic_ef_max = ef, dynamic_ef_min, dynamic_ef_max
        self.cfg.dynamic_ef_factor, self.cfg.flat_search_cutoff = dynamic_ef_factor, flat_search_cutoff
        self.cfg.forbid_flat, self.cfg.id_base = int(forbid_flat), id_base
        h = C.c_void_p()
        check(lib().wv_index_create(dim, METRICS[distance], C.byref(self.cfg), capacity, C.byref(h)))
        self._h = h
        self._owned = True

    @classmethod
    def _borrow(cls, handle, dim: int, distance: str, capacity: int, cfg: WvConfig, owner):
        """A view of an index another object owns (a wv_group member)."""
        ix = cls.__new__(cls)
        ix.dim, ix.distance, ix.capacity, ix.cfg = dim, distance, capacity, cfg
        ix._h, ix._owned, ix._owner = handle, False, owner
        return ix

    # -- lifecycle -----------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            if getattr(self, "_owned", True):
                lib().wv_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def update_user_config(self, **kw):
        """UpdateUserConfig (config_update.go:79-128): ef / dynamic ef / cutoff."""
        for k, v in kw.items():
            setattr(self.cfg, k, int(v))
        check(lib().wv_index_update_config(self._h, C.byref(self.cfg)))

    # -- state upload ----------------------------------------------------------
    def upload_vectors(self, rows: np.ndarray, first_id: int = 0):
        rows = np.ascontiguousarray(rows, dtype=np.float32)
        if rows.ndim != 2 or rows.shape[1] != self.dim:
            raise WvError(1, f"vector lengths don't match: {rows.shape[-1]} vs {self.dim}")
        check(lib().wv_index_upload_vectors(self._h, _ptr(rows), rows.shape[0], first_id))

    def upload_vectors_device(self, ptr: int, n: int, first_id: int = 0, ld: Optional[int] = None):
        check(lib().wv_index_upload_vectors_device(self._h, C.c_void_p(ptr), n, first_id, ld or self.dim))

    def upload_graph(self, g: dict):
        """g: the fixed-degree CSR of oracle.pyoracle.Index.export_graph()."""
        levels = np.ascontiguousarray(g["levels"], dtype=np.int8)
        layer0 = np.ascontiguousarray(g["layer0"], dtype=np.uint32)
        upper_row = np.ascontiguousarray(g["upper_row"], dtype=np.uint32)
        upper = np.ascontiguousarray(g["upper"], dtype=np.uint32)
        if upper.ndim != 3:
            raise WvError(1, "upper must be [n_upper][levels][degU]")
        # The ABI's level stride of `upper` is max_level (the entrypoint's
        # layer).  Levels above it are never searched -- the descent starts at
        # max_level (search.go:479) -- so a wider array is cut and a narrower
        # one padded with empty lists.
        ml = int(g["max_level"])
        if ml > 0 and upper.shape[1] != ml:
            fixed = np.full((upper.shape[0], ml, upper.shape[2]), 0xFFFFFFFF, np.uint32)
            keep = min(ml, upper.shape[1])
            fixed[:, :keep, :] = upper[:, :keep, :]
            upper = fixed
        check(lib().wv_index_upload_graph(self._h, g["n"], _ptr(levels), _ptr(layer0), layer0.shape[1],
                                          _ptr(upper_row), _ptr(upper), upper.shape[0], upper.shape[2],
                                          g["max_level"], g["entrypoint"]))

    def upload_graph_from_commitlog(self, graph: "CommitLogGraph"):
        """Serve a graph replayed from a shard's commit log: the CSR degree is
        the configured 2M / M or the longest list the log holds (legacy
        oversize lists, search.go:236-251), and the log's tombstones replace
        the index's."""
        info = graph.info()
        if info["compressed"]:
            raise WvError(4, "commit log holds a PQ-compressed index; the GPU path serves uncompressed vectors")
        m = self.cfg.max_connections
        g = graph.export_csr(max(2 * m, info["max_deg0"]), max(m, info["max_degU"], 1))
        # export_csr lays `upper` out with a level stride of max(1,
        # max_node_level), which differs from the entrypoint's max_level after
        # a torn AddNode above the top (insert.go:206) or inside
        # deleteEntrypoint's window (delete.go:405-414); upload_graph re-lays it
        self.upload_graph(g)
        check(lib().wv_index_set_tombstones(self._h, _ptr(g["tomb_bits"]), g["n"]))

    def build_graph(self, ef_construction: int = 128, seed: int = 1, batch_div: int = 32):
        """Build the HNSW graph of the uploaded rows on the GPU (wv_index_build_graph)."""
        check(lib().wv_index_build_graph(self._h, ef_construction, seed, batch_div))

    def query_ld(self) -> int:
        """Row stride (floats) of the device query rows search_batch_device reads."""
        return lib().wv_index_query_ld(self._h)

    def graph_info(self) -> dict:
        n, ep, nu = C.c_uint64(), C.c_uint64(), C.c_uint64()
        d0, du, ml = C.c_int(), C.c_int(), C.c_int()
        check(lib().wv_index_graph_info(self._h, C.byref(n), C.byref(d0), C.byref(du), C.byref(ml), C.byref(nu),
                                        C.byref(ep)))
        return dict(n=n.value, entrypoint=ep.value, max_level=ml.value, n_upper=nu.value, deg0=d0.value,
                    degU=du.value)

    def download_graph(self) -> dict:
        """The index's graph in the upload_graph / export_graph layout."""
        n, ep, nu = C.c_uint64(), C.c_uint64(), C.c_uint64()
        d0, du, ml = C.c_int(), C.c_int(), C.c_int()
        check(lib().wv_index_graph_info(self._h, C.byref(n), C.byref(d0), C.byref(du), C.byref(ml), C.byref(nu),
                                        C.byref(ep)))
        levels = np.zeros(n.value, np.int8)
        layer0 = np.zeros((n.value, d0.value), np.uint32)
        upper_row = np.zeros(n.value, np.uint32)
        upper = np.zeros((max(nu.value, 1), max(ml.value, 1), du.value), np.uint32)
        check(lib().wv_index_download_graph(self._h, _ptr(levels), _ptr(layer0), _ptr(upper_row), _ptr(upper)))
        return dict(n=n.value, entrypoint=ep.value, max_level=ml.value, levels=levels, layer0=layer0,
                    upper_row=upper_row, upper=upper, deg0=d0.value, degU=du.value)

    def add(self, ids, rows):
        """hnsw.Add (insert.go:43-65) on the GPU mirror: rows at arbitrary ids,
        searchable at once (delta set, exact) until a graph snapshot holds them."""
        ids = np.ascontiguousarray(np.atleast_1d(np.asarray(ids, dtype=np.uint64)))
        rows = np.ascontiguousarray(rows, dtype=np.float32).reshape(len(ids), -1)
        if rows.shape[1] != self.dim:
            raise WvError(1, f"vector lengths don't match: {rows.shape[1]} vs {self.dim}")
        check(lib().wv_index_add(self._h, _ptr(ids), _ptr(rows), len(ids)))

    def add_tombstones(self, ids):
        ids = np.ascontiguousarray(np.atleast_1d(np.asarray(ids, dtype=np.uint64)))
        check(lib().wv_index_add_tombstones(self._h, _ptr(ids), len(ids)))

    def remove_tombstones(self, ids):
        ids = np.ascontiguousarray(np.atleast_1d(np.asarray(ids, dtype=np.uint64)))
        check(lib().wv_index_remove_tombstones(self._h, _ptr(ids), len(ids)))

    def delta_size(self) -> int:
        n = C.c_uint64()
        check(lib().wv_index_delta_size(self._h, C.byref(n)))
        return n.value

    def reserve(self, capacity: int):
        """Grow the index in place (growIndexToAccomodateNode, maintainance.go:31-100)."""
        check(lib().wv_index_reserve(self._h, capacity))
        self.capacity = max(self.capacity, capacity)

    def capacity_info(self) -> tuple:
        cap, n = C.c_uint64(), C.c_uint64()
        check(lib().wv_index_capacity(self._h, C.byref(cap), C.byref(n)))
        return cap.value, n.value

    # -- product quantization (compress.go:39-89) -------------------------------
    def set_pq(self, centroids, use_bits_encoding: bool = False, encoder: str = "kmeans"):
        """The fitted quantizer: centroids[segments][ks][dims/segments] =
        kms[i].Centroid(c) (product_quantization.go:77-95)."""
        cent = np.ascontiguousarray(centroids, dtype=np.float32)
        if cent.ndim != 3 or cent.shape[0] * cent.shape[2] != self.dim:
            raise WvError(1, f"centroid table must be [segments][centroids][dims/segments], got {cent.shape}")
        self._pq = (cent.shape[0], cent.shape[1], bool(use_bits_encoding))
        check(lib().wv_index_set_pq(self._h, cent.shape[0], cent.shape[1], int(use_bits_encoding),
                                    {"tile": 0, "kmeans": 1}[encoder], _ptr(cent)))

    def upload_pq_codes(self, encoded, first_id: int = 0):
        """Encoded vectors in ProductQuantizer.Encode's byte layout, uint8[n][code_len]."""
        enc = np.ascontiguousarray(encoded, dtype=np.uint8)
        m, ks, ub = self._pq
        if enc.ndim != 2 or enc.shape[1] != lib().wv_pq_code_len(m, ks, int(ub)):
            raise WvError(1, f"encoded rows must be [n][{lib().wv_pq_code_len(m, ks, int(ub))}] bytes")
        check(lib().wv_index_upload_pq_codes(self._h, _ptr(enc), enc.shape[0], first_id))

    def pq_encode(self):
        """KMeans-encode every resident vector on the device (ProductQuantizer.Encode)."""
        check(lib().wv_index_pq_encode(self._h))

    def download_pq_codes(self, n: int, first_id: int = 0) -> np.ndarray:
        out = np.zeros((n, self._pq[0]), np.uint16)
        check(lib().wv_index_download_pq_codes(self._h, _ptr(out), first_id, n))
        return out

    def set_compressed(self, on: bool = True):
        """h.compressed: every search ranks by the PQ distance."""
        check(lib().wv_index_set_compressed(self._h, int(on)))

    def set_tombstones(self, ids: Iterable[int]):
        al = AllowList.from_ids(ids, self.capacity)
        check(lib().wv_index_set_tombstones(self._h, _ptr(al.words), al.nbits))

    def search_time_ef(self, k: int) -> int:
        return lib().wv_search_time_ef(self._h, k)

    # -- search ----------------------------------------------------------------
    @staticmethod
    def _allow_args(allow):
        if allow is None:
            return None, 0, 0
        if isinstance(allow, AllowList):
            return allow.words, allow.nbits, 0
        if isinstance(allow, list) and allow and isinstance(allow[0], AllowList):
            nb = max(a.nbits for a in allow)
            stride = (nb + 63) // 64
            m = np.zeros((len(allow), stride), dtype=np.uint64)
            for i, a in enumerate(allow):
                m[i, : a.words.size] = a.words
            return m, nb, stride
        raise WvError(1, "allow must be an AllowList or a list of AllowList (one per query)")

    def search_by_vector(self, vector, k: int, allow: Optional[AllowList] = None):
        """SearchByVector (search.go:64-79) -> (ids uint64[n], dists float32[n])."""
        q = np.ascontiguousarray(vector, dtype=np.float32)
        if q.size != self.dim:
            raise WvError(1, f"vector lengths don't match: {q.size} vs {self.dim}")
        bits, nb, _ = self._allow_args(allow)
        ids = np.zeros(k, np.uint64)
        ds = np.zeros(k, np.float32)
        n = np.zeros(1, np.int32)
        check(lib().wv_search_by_vector(self._h, _ptr(q), k, _ptr(bits), nb, _ptr(ids), _ptr(ds), _ptr(n)))
        return ids[: n[0]], ds[: n[0]]

    def search_by_vector_distance(self, vector, target_distance: float, max_limit: int = -1,
                                  allow: Optional[AllowList] = None, cap: int = 1 << 20):
        """SearchByVectorDistance (search.go:90-158)."""
        q = np.ascontiguousarray(vector, dtype=np.float32)
        if q.size != self.dim:
            raise WvError(1, f"vector lengths don't match: {q.size} vs {self.dim}")
        bits, nb, _ = self._allow_args(allow)
        ids = np.zeros(cap, np.uint64)
        ds = np.zeros(cap, np.float32)
        n = C.c_int64(0)
        check(lib().wv_search_by_vector_distance(self._h, _ptr(q), float(target_distance), max_limit, _ptr(bits), nb,
                                                 _ptr(ids), _ptr(ds), cap, C.byref(n)))
        m = min(n.value, cap)
        return ids[:m], ds[:m]

    def search_by_vector_distance_batch(self, queries, targets, max_limit: int = -1, allow=None,
                                        cap: int = 4096):
        """SearchByVectorDistance for a batch (each query its own target): a
        list of (ids, dists) per query; at most `cap` results are returned
        per query (`n` counts them all)."""
        qs = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, self.dim)
        nq = qs.shape[0]
        ts = np.ascontiguousarray(np.broadcast_to(np.asarray(targets, np.float32), (nq,)))
        bits, nb, stride = self._allow_args(allow)
        ids = np.zeros((nq, cap), np.uint64)
        ds = np.zeros((nq, cap), np.float32)
        n = np.zeros(nq, np.int64)
        check(lib().wv_search_by_vector_distance_batch(self._h, _ptr(qs), nq, _ptr(ts), max_limit, _ptr(bits), nb,
                                                       stride, _ptr(ids), _ptr(ds), cap, _ptr(n)))
        return [(ids[i, :min(n[i], cap)], ds[i, :min(n[i], cap)]) for i in range(nq)], n

    def search_batch(self, queries, k: int, ef: int = 0, allow=None, mode: str = "auto"):
        """Batched search: (ids [nq,k] uint64, dists [nq,k] f32, n [nq] i32)."""
        qs = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, self.dim)
        nq = qs.shape[0]
        bits, nb, stride = self._allow_args(allow)
        ids = np.zeros((nq, k), np.uint64)
        ds = np.zeros((nq, k), np.float32)
        n = np.zeros(nq, np.int32)
        check(lib().wv_search_batch(self._h, _ptr(qs), nq, k, ef, _ptr(bits), nb, stride, _MODES[mode], _ptr(ids),
                                    _ptr(ds), _ptr(n)))
        return ids, ds, n

    def search_batch_device(self, q_ptr: int, nq: int, k: int, out_ids_ptr: int, out_d_ptr: int, out_n_ptr: int,
                            ef: int = 0, allow_ptr: int = 0, allow_nbits: int = 0, allow_stride: int = 0,
                            mode: str = "exact", stream: int = 0):
        """Device-resident batch (pointers from torch tensors on this device),
        queued on `stream` without a host round trip.  stream 0 (torch's
        default stream) queues on the index's own stream and then waits for
        it, so that default-stream callers read complete results."""
        check(lib().wv_search_batch_device(self._h, C.c_void_p(q_ptr), nq, k, ef,
                                           C.c_void_p(allow_ptr) if allow_ptr else None, allow_nbits, allow_stride,
                                           _MODES[mode], C.c_void_p(out_ids_ptr), C.c_void_p(out_d_ptr),
                                           C.c_void_p(out_n_ptr), C.c_void_p(stream) if stream else None))
        if not stream:
            check(lib().wv_index_synchronize(self._h))

    def set_timing(self, enable: bool = True):
        check(lib().wv_index_set_timing(self._h, int(enable)))

    def last_kernel_times(self):
        a, b, c = C.c_float(), C.c_float(), C.c_float()
        check(lib().wv_last_kernel_times(self._h, C.byref(a), C.byref(b), C.byref(c)))
        d = C.c_float()
        check(lib().wv_last_seed_time(self._h, C.byref(d)))
        return {"bf_mfma_ms": a.value, "bf_finalize_ms": b.value, "hnsw_ms": c.value, "seed_ms": d.value}

    def last_batch_stats(self):
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check(lib().wv_last_batch_stats(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return {"dist_evals": a.value, "expansions": b.value, "fallbacks": c.value}

    def last_side_stats(self):
        """filtered HNSW: queries whose side set outgrew its HBM spill (exact
        fallback), queries the light-filter pass re-ran with the exact visited
        bitmap, the LDS side array's rows of 64 and the spill capacity"""
        a, r, m, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_int(), C.c_int()
        check(lib().wv_last_side_stats(self._h, C.byref(a), C.byref(r), C.byref(m), C.byref(b), C.byref(c)))
        return {"overflowed": a.value, "redone": r.value, "claims": m.value, "side_rows": b.value,
                "spill_cap": c.value}


class CommitLogGraph:
    """A graph replayed from HNSW commit logs (wv_graph_*, deserializer.go:80-158).
    `source`: bytes (one log), a directory (<name>.hnsw.commitlog.d) or a list of
    log file paths in replay order."""

    def __init__(self, source):
        h = C.c_void_p()
        if isinstance(source, (bytes, bytearray)):
            buf = (C.c_uint8 * max(len(source), 1)).from_buffer_copy(bytes(source) or b"\0")
            check(lib().wv_graph_load_commitlog_buffer(buf, len(source), C.byref(h)))
        elif isinstance(source, str):
            check(lib().wv_graph_load_commitlog_dir(source.encode(), C.byref(h)))
        else:
            paths = [str(p).encode() for p in source]
            arr = (C.c_char_p * max(len(paths), 1))(*paths)
            check(lib().wv_graph_load_commitlogs(arr, len(paths), C.byref(h)))
        self._h = h

    def info(self) -> dict:
        i = WvGraphInfo()
        check(lib().wv_graph_get_info(self._h, C.byref(i)))
        return i.asdict()

    def node(self, id_: int, level: int = 0):
        """(level, links at `level`) of one node; level -1 = nil node."""
        lv, n = C.c_int(), C.c_int()
        check(lib().wv_graph_node(self._h, id_, level, C.byref(lv), None, 0, C.byref(n)))
        out = np.zeros(max(n.value, 1), np.uint64)
        check(lib().wv_graph_node(self._h, id_, level, C.byref(lv), _ptr(out), n.value, C.byref(n)))
        return lv.value, out[: n.value].tolist()

    def export_csr(self, deg0: int, degU: int) -> dict:
        """The fixed-degree CSR of GPUVectorIndex.upload_graph (+ tombstone bits)."""
        i = self.info()
        n, ml = i["n_slots"], max(1, i["max_node_level"])
        levels = np.zeros(n, np.int8)
        layer0 = np.zeros((n, deg0), np.uint32)
        upper_row = np.zeros(n, np.uint32)
        upper = np.zeros((max(i["n_upper"], 1), ml, degU), np.uint32)
        tomb = np.zeros((n + 63) // 64 or 1, np.uint64)
        check(lib().wv_graph_export_csr(self._h, deg0, degU, _ptr(levels), _ptr(layer0), _ptr(upper_row), _ptr(upper),
                                        _ptr(tomb)))
        return dict(n=n, entrypoint=i["entrypoint"], max_level=i["max_level"], levels=levels, layer0=layer0,
                    upper_row=upper_row, upper=upper, deg0=deg0, degU=degU, tomb_bits=tomb)

    def close(self):
        if getattr(self, "_h", None):
            lib().wv_graph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GPUGroup:
    """Several devices driven from one process (wv_group_*): the corpus split
    by id range over the members with an RCCL gather + device merge
    (layout="shard", index.go:967-1044), or replicated with the batch split by
    queries (layout="replica").  `search_batch` has GPUVectorIndex's result."""

    def __init__(self, devices, dim: int, distance: str = "l2-squared", capacity: int = 1 << 20, *,
                 layout: str = "shard", max_connections: int = 64, ef: int = -1, flat_search_cutoff: int = 40000,
                 forbid_flat: bool = False):
        if distance not in METRICS:
            raise WvError(1, f"unsupported distance {distance!r}")
        self.dim, self.distance, self.capacity, self.layout = dim, distance, capacity, layout
        self.cfg = WvConfig()
        lib().wv_config_default(C.byref(self.cfg))
        self.cfg.max_connections, self.cfg.ef = max_connections, ef
        self.cfg.flat_search_cutoff, self.cfg.forbid_flat = flat_search_cutoff, int(forbid_flat)
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        check(lib().wv_group_create(devs, len(devices), dim, METRICS[distance], C.byref(self.cfg), capacity,
                                    {"shard": 0, "replica": 1}[layout], C.byref(h)))
        self._h = h

    def info(self):
        n, r = C.c_int(), C.c_int()
        check(lib().wv_group_info(self._h, C.byref(n), C.byref(r)))
        return {"members": n.value, "uses_rccl": bool(r.value)}

    def member(self, i: int):
        """(GPUVectorIndex view of member i, its id base, its capacity)."""
        h, base, cap = C.c_void_p(), C.c_uint64(), C.c_uint64()
        check(lib().wv_group_member(self._h, i, C.byref(h), C.byref(base), C.byref(cap)))
        return GPUVectorIndex._borrow(h, self.dim, self.distance, cap.value, self.cfg, self), base.value, cap.value

    def upload_vectors(self, rows: np.ndarray, first_id: int = 0):
        rows = np.ascontiguousarray(rows, dtype=np.float32)
        if rows.ndim != 2 or rows.shape[1] != self.dim:
            raise WvError(1, f"vector lengths don't match: {rows.shape[-1]} vs {self.dim}")
        check(lib().wv_group_upload_vectors(self._h, _ptr(rows), rows.shape[0], first_id))

    def build_graph(self, ef_construction: int = 128, seed: int = 1, batch_div: int = 32):
        check(lib().wv_group_build_graph(self._h, ef_construction, seed, batch_div))

    def add(self, ids, rows):
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        rows = np.ascontiguousarray(rows, dtype=np.float32).reshape(-1, self.dim)
        check(lib().wv_group_add(self._h, _ptr(ids), _ptr(rows), ids.size))

    def add_tombstones(self, ids):
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        check(lib().wv_group_add_tombstones(self._h, _ptr(ids), ids.size))

    def search_batch(self, queries, k: int, ef: int = 0, allow=None, mode: str = "auto"):
        qs = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, self.dim)
        nq = qs.shape[0]
        bits, nb, stride = GPUVectorIndex._allow_args(allow)
        ids = np.zeros((nq, k), np.uint64)
        ds = np.zeros((nq, k), np.float32)
        n = np.zeros(nq, np.int32)
        check(lib().wv_group_search_batch(self._h, _ptr(qs), nq, k, ef, _ptr(bits), nb, stride, _MODES[mode],
                                          _ptr(ids), _ptr(ds), _ptr(n)))
        return ids, ds, n

    def close(self):
        if getattr(self, "_h", None):
            lib().wv_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Batcher:
    """Native micro-batcher over one index or one GPUGroup (wv_batcher_*):
    `search` has the signature and result of GPUVectorIndex.search_by_vector
    and is meant to be called from many threads at once (ctypes releases the
    GIL for the call)."""

    def __init__(self, index, max_batch: int = 256, max_wait_us: int = 200):
        self.index = index
        h = C.c_void_p()
        create = lib().wv_batcher_create_group if isinstance(index, GPUGroup) else lib().wv_batcher_create
        check(create(index._h, index.dim, max_batch, max_wait_us, C.byref(h)))
        self._h = h

    def search(self, vector, k: int, allow: Optional[AllowList] = None):
        q = np.ascontiguousarray(vector, dtype=np.float32)
        if q.size != self.index.dim:
            raise WvError(1, f"vector lengths don't match: {q.size} vs {self.index.dim}")
        bits, nb, _ = GPUVectorIndex._allow_args(allow)
        ids = np.zeros(k, np.uint64)
        ds = np.zeros(k, np.float32)
        n = np.zeros(1, np.int32)
        check(lib().wv_batcher_search(self._h, _ptr(q), k, _ptr(bits), nb, _ptr(ids), _ptr(ds), _ptr(n)))
        return ids[: n[0]], ds[: n[0]]

    def search_ids(self, vector, k: int, allow_ids=None):
        """The same with the AllowList as ascending ids (wv_batcher_search_ids);
        allow_ids None = no filter."""
        q = np.ascontiguousarray(vector, dtype=np.float32)
        if q.size != self.index.dim:
            raise WvError(1, f"vector lengths don't match: {q.size} vs {self.index.dim}")
        a = np.ascontiguousarray(np.zeros(0, np.uint64) if allow_ids is None else allow_ids, dtype=np.uint64)
        ids = np.zeros(k, np.uint64)
        ds = np.zeros(k, np.float32)
        n = np.zeros(1, np.int32)
        check(lib().wv_batcher_search_ids(self._h, _ptr(q), k, int(allow_ids is not None), _ptr(a), len(a), _ptr(ids),
                                          _ptr(ds), _ptr(n)))
        return ids[: n[0]], ds[: n[0]]

    def stats(self):
        a, b = C.c_uint64(), C.c_uint64()
        check(lib().wv_batcher_stats(self._h, C.byref(a), C.byref(b)))
        return {"requests": a.value, "batches": b.value}

    def close(self):
        if getattr(self, "_h", None):
            lib().wv_batcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def merge_shards_device(in_d_ptr, in_ids_ptr, in_n_ptr, n_shards, nq, k, out_d_ptr, out_ids_ptr, out_n_ptr, stream=0):
    """Merge per-shard (dist, id) lists on the device (after the RCCL all-gather)."""
    check(lib().wv_merge_shards_device(C.c_void_p(in_d_ptr), C.c_void_p(in_ids_ptr), C.c_void_p(in_n_ptr), n_shards,
                                       nq, k, C.c_void_p(out_d_ptr), C.c_void_p(out_ids_ptr), C.c_void_p(out_n_ptr),
                                       C.c_void_p(stream) if stream else None))
