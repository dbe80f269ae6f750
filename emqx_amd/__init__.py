"""emqx_amd — MI355X-native batched topic matching for EMQX's routing hot path.

The product is the C-ABI library libemqx_tm.so (include/emqx_tm.h): a host trie
builder with delta epochs plus gfx950 HIP kernels.  This package holds its ctypes
binding (_native), host mirrors of the reference interfaces on this path
(topic_index = emqx_topic_index, router = emqx_router v2 + emqx_router_syncer),
topic helpers, and the seeded workload generator used by tests and bench.py.
"""
from ._native import Engine, TMError  # noqa: F401
