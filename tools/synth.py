"""ctypes wrapper of tools/libwvsynth.so (tools/wv_synth.hip): counter-based
synthetic corpora written straight into device memory (measurement
infrastructure for bench.py; not part of the product library)."""
import ctypes as C
import os

_LIB = None
KINDS = {"uniform": 0, "gauss": 1, "sift": 2}


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libwvsynth.so")
        if not os.path.exists(path):
            raise RuntimeError("tools/libwvsynth.so is not built (__graft_entry__.build())")
        _LIB = C.CDLL(path)
        _LIB.wvs_fill.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, C.c_void_p, C.c_int,
                                  C.c_void_p]
        _LIB.wvs_fill.restype = C.c_int
    return _LIB


def fill(kind: str, seed: int, row0: int, t, stream: int = 0):
    """rows [row0, row0 + t.shape[0]) of the kind's matrix into the float32
    device tensor t (shape [n, ld]; its first `dim` = t.shape[1] columns)"""
    n, ld = t.shape
    rc = lib().wvs_fill(KINDS[kind], seed, row0, n, ld, C.c_void_p(t.data_ptr()), ld, C.c_void_p(stream))
    if rc:
        raise RuntimeError(f"wvs_fill({kind}) failed: HIP error {rc}")
