"""azhip — MI355X (gfx950) HIP implementation of the alphazero-gnn board-evaluation hot path.

Compute lives in libaz_hip.so (C-ABI: include/az_hip.h); this package holds the ctypes
binding (_lib), tensor-level ops (ops), flat parameter storage (params), the network
classes (nets) and the build script (build).
"""
