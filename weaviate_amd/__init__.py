"""weaviate_amd -- MI355X-native engine for Weaviate's vector-index search path.

The product is libwvgpu.so (hand-written HIP for gfx950 behind the C ABI of
include/wvgpu.h); this package is its ctypes binding plus the host-side mirror
of the reference's VectorIndex search interface.
"""
from ._lib import MODE_AUTO, MODE_EXACT, MODE_HNSW, WvError, build, header_symbols, lib  # noqa: F401
from .index import AllowList, Batcher, CommitLogGraph, GPUGroup, GPUVectorIndex, merge_shards_device  # noqa: F401

__all__ = ["AllowList", "Batcher", "CommitLogGraph", "GPUGroup", "GPUVectorIndex", "WvError", "build", "lib", "merge_shards_device", "header_symbols"]
