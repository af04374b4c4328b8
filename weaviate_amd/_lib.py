"""ctypes binding of libwvgpu.so (the C ABI of include/wvgpu.h).

The product path has no CPU fallback: if the HIP library is missing or cannot
be loaded, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# (WV_LIBPATH: an A/B build, tools/ab_build.sh -- measurement only)
LIBPATH = os.environ.get("WV_LIBPATH") or os.path.join(_HERE, "libwvgpu.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "wvgpu.h")

WV_OK, WV_EINVAL, WV_EOOM, WV_EDEVICE, WV_ESTATE, WV_EDELETED = range(6)
MODE_AUTO, MODE_EXACT, MODE_HNSW = 0, 1, 2
METRICS = {"l2-squared": 0, "dot": 1, "cosine-dot": 2}


class WvConfig(C.Structure):
    _fields_ = [
        ("device", C.c_int),
        ("max_connections", C.c_int),
        ("ef", C.c_int64),
        ("dynamic_ef_min", C.c_int64),
        ("dynamic_ef_max", C.c_int64),
        ("dynamic_ef_factor", C.c_int64),
        ("flat_search_cutoff", C.c_int64),
        ("forbid_flat", C.c_int),
        ("id_base", C.c_uint64),
    ]


class WvGraphInfo(C.Structure):
    _fields_ = [
        ("n_slots", C.c_uint64),
        ("entrypoint", C.c_uint64),
        ("n_upper", C.c_uint64),
        ("n_tombstones", C.c_uint64),
        ("valid_bytes", C.c_uint64),
        ("max_level", C.c_int),
        ("max_node_level", C.c_int),
        ("max_deg0", C.c_int),
        ("max_degU", C.c_int),
        ("compressed", C.c_int),
        ("truncated", C.c_int),
    ]

    def asdict(self):
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class WvError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"wvgpu error {code}: {msg}")
        self.code = code


def build(arch: str = "gfx950", jobs: int = 3) -> str:
    subprocess.check_call(["make", "-s", f"-j{jobs}", f"ARCH={arch}", "-C", os.path.join(_HERE, "csrc")])
    return LIBPATH


_lib = None

_vp, _u64p, _f32p, _i32p = C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_float), C.POINTER(C.c_int32)
SIGNATURES = {
    "wv_config_default": (None, [C.POINTER(WvConfig)]),
    "wv_index_create": (C.c_int, [C.c_int, C.c_int, C.POINTER(WvConfig), C.c_uint64, C.POINTER(C.c_void_p)]),
    "wv_index_destroy": (C.c_int, [_vp]),
    "wv_index_update_config": (C.c_int, [_vp, C.POINTER(WvConfig)]),
    "wv_index_upload_vectors": (C.c_int, [_vp, _vp, C.c_uint64, C.c_uint64]),
    "wv_index_upload_vectors_device": (C.c_int, [_vp, _vp, C.c_uint64, C.c_uint64, C.c_int]),
    "wv_index_upload_graph": (C.c_int, [_vp, C.c_uint64, _vp, _vp, C.c_int, _vp, _vp, C.c_uint64, C.c_int, C.c_int,
                                        C.c_uint64]),
    "wv_index_set_tombstones": (C.c_int, [_vp, _vp, C.c_uint64]),
    "wv_search_time_ef": (C.c_int, [_vp, C.c_int]),
    "wv_config_search_time_ef": (C.c_int, [C.POINTER(WvConfig), C.c_int]),
    "wv_index_add": (C.c_int, [_vp, _vp, _vp, C.c_uint64]),
    "wv_index_build_graph": (C.c_int, [_vp, C.c_int, C.c_uint64, C.c_int]),
    "wv_index_graph_info": (C.c_int, [_vp, _u64p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int), _u64p,
                                      _u64p]),
    "wv_index_download_graph": (C.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "wv_index_add_tombstones": (C.c_int, [_vp, _vp, C.c_uint64]),
    "wv_index_remove_tombstones": (C.c_int, [_vp, _vp, C.c_uint64]),
    "wv_index_delta_size": (C.c_int, [_vp, _u64p]),
    "wv_pq_code_len": (C.c_int, [C.c_int, C.c_int, C.c_int]),
    "wv_index_set_pq": (C.c_int, [_vp, C.c_int, C.c_int, C.c_int, C.c_int, _vp]),
    "wv_index_upload_pq_codes": (C.c_int, [_vp, _vp, C.c_uint64, C.c_uint64]),
    "wv_index_pq_encode": (C.c_int, [_vp]),
    "wv_index_download_pq_codes": (C.c_int, [_vp, _vp, C.c_uint64, C.c_uint64]),
    "wv_index_set_compressed": (C.c_int, [_vp, C.c_int]),
    "wv_search_by_vector": (C.c_int, [_vp, _vp, C.c_int, _vp, C.c_uint64, _vp, _vp, _vp]),
    "wv_search_by_vector_distance": (C.c_int, [_vp, _vp, C.c_float, C.c_int64, _vp, C.c_uint64, _vp, _vp, C.c_int64,
                                               C.POINTER(C.c_int64)]),
    "wv_search_by_vector_distance_batch": (C.c_int, [_vp, _vp, C.c_int, _vp, C.c_int64, _vp, C.c_uint64, C.c_uint64,
                                                     _vp, _vp, C.c_int64, _vp]),
    "wv_search_batch": (C.c_int, [_vp, _vp, C.c_int, C.c_int, C.c_int, _vp, C.c_uint64, C.c_uint64, C.c_int, _vp, _vp,
                                  _vp]),
    "wv_search_batch_device": (C.c_int, [_vp, _vp, C.c_int, C.c_int, C.c_int, _vp, C.c_uint64, C.c_uint64, C.c_int,
                                         _vp, _vp, _vp, _vp]),
    "wv_index_query_ld": (C.c_int, [_vp]),
    "wv_index_synchronize": (C.c_int, [_vp]),
    "wv_merge_shards_device": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _vp]),
    "wv_last_batch_stats": (C.c_int, [_vp, _u64p, _u64p, _u64p]),
    "wv_last_side_stats": (C.c_int, [_vp, _u64p, _u64p, _u64p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "wv_index_set_timing": (C.c_int, [_vp, C.c_int]),
    "wv_last_kernel_times": (C.c_int, [_vp, _f32p, _f32p, _f32p]),
    "wv_last_seed_time": (C.c_int, [_vp, _f32p]),
    "wv_graph_load_commitlog_buffer": (C.c_int, [_vp, C.c_uint64, C.POINTER(C.c_void_p)]),
    "wv_graph_load_commitlogs": (C.c_int, [C.POINTER(C.c_char_p), C.c_int, C.POINTER(C.c_void_p)]),
    "wv_graph_load_commitlog_dir": (C.c_int, [C.c_char_p, C.POINTER(C.c_void_p)]),
    "wv_graph_get_info": (C.c_int, [_vp, C.POINTER(WvGraphInfo)]),
    "wv_graph_node": (C.c_int, [_vp, C.c_uint64, C.c_int, C.POINTER(C.c_int), _vp, C.c_int, C.POINTER(C.c_int)]),
    "wv_graph_export_csr": (C.c_int, [_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp]),
    "wv_graph_destroy": (C.c_int, [_vp]),
    "wv_batcher_create": (C.c_int, [_vp, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "wv_batcher_search": (C.c_int, [_vp, _vp, C.c_int, _vp, C.c_uint64, _vp, _vp, _vp]),
    "wv_batcher_stats": (C.c_int, [_vp, _u64p, _u64p]),
    "wv_batcher_destroy": (C.c_int, [_vp]),
    "wv_group_create": (C.c_int, [_vp, C.c_int, C.c_int, C.c_int, C.POINTER(WvConfig), C.c_uint64, C.c_int,
                                  C.POINTER(C.c_void_p)]),
    "wv_group_destroy": (C.c_int, [_vp]),
    "wv_group_info": (C.c_int, [_vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "wv_group_member": (C.c_int, [_vp, C.c_int, C.POINTER(C.c_void_p), _u64p, _u64p]),
    "wv_group_upload_vectors": (C.c_int, [_vp, _vp, C.c_uint64, C.c_uint64]),
    "wv_group_build_graph": (C.c_int, [_vp, C.c_int, C.c_uint64, C.c_int]),
    "wv_group_add": (C.c_int, [_vp, _vp, _vp, C.c_uint64]),
    "wv_group_add_tombstones": (C.c_int, [_vp, _vp, C.c_uint64]),
    "wv_group_remove_tombstones": (C.c_int, [_vp, _vp, C.c_uint64]),
    "wv_group_update_config": (C.c_int, [_vp, C.POINTER(WvConfig)]),
    "wv_group_search_batch": (C.c_int, [_vp, _vp, C.c_int, C.c_int, C.c_int, _vp, C.c_uint64, C.c_uint64, C.c_int,
                                        _vp, _vp, _vp]),
    "wv_batcher_create_group": (C.c_int, [_vp, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "wv_last_error": (C.c_char_p, []),
    "wv_version": (C.c_char_p, []),
}


def header_symbols() -> list[str]:
    """Every function the C header declares."""
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(wv_[a-z0-9_]+)\s*\(", src)))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIBPATH):
            raise WvError(WV_ESTATE, f"{LIBPATH} not built: run __graft_entry__.build() (no CPU fallback exists)")
        # One HIP runtime per process: when PyTorch-ROCm is importable, load it
        # first so libwvgpu.so binds to the same libamdhip64.so.7 (it bundles
        # its own copy) and device pointers/streams interoperate.
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        L = C.CDLL(LIBPATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int):
    if rc != WV_OK:
        raise WvError(rc, lib().wv_last_error().decode(errors="replace"))
