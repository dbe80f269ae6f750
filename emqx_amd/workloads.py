"""Seeded synthetic workloads for BASELINE.json configs A–E (libemqx_synth.so).

Each config is a parameter set for the generator in csrc/synth.cpp.  The returned
Workload holds packed route keys (filter bytes, u64 offsets, u64 ids) and a packed
topic batch (bytes, u32 offsets) ready for Engine.apply_packed / match_packed.

  A  emqx_topic_index CPU reference: 10k filters (20% wildcards), 100k random 4-level topics
  B  1M filters, 6-level topics, 10% '+' / 5% '#', 1M-publish batches
  C  10M filters, deep 10-level topics, '#'-heavy fan-out (compaction stress)   <- bench headline
  D  100M filters, 8-level (B generator) — hash-sharded over GPUs
  E  B-sized set + $SYS topics, root '#', '+/...', $share/g1..g4 duplicates, churn epochs
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libemqx_synth.so")


class synth_params(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64), ("n_filters", C.c_uint64), ("n_topics", C.c_uint64),
        ("min_levels", C.c_uint32), ("max_levels", C.c_uint32), ("vocab", C.c_uint32 * 16),
        ("zipf_s", C.c_double), ("p_fixed", C.c_double), ("p_plus", C.c_double), ("p_plus_level", C.c_double),
        ("p_hash", C.c_double), ("hash_geo", C.c_double), ("min_hash_depth", C.c_uint32), ("plus_hash_excl", C.c_uint32),
        ("p_topic_hit", C.c_double), ("p_sys", C.c_double), ("p_sys_filter", C.c_double),
        ("p_multi", C.c_double), ("multi_max", C.c_uint32), ("n_hot", C.c_uint32),
        ("hot_ids_min", C.c_uint32), ("hot_ids_max", C.c_uint32),
        ("hot_depth_min", C.c_uint32), ("hot_depth_max", C.c_uint32),
        ("p_topic_hot", C.c_double), ("hash_w", C.c_double * 16),
        ("shard_count", C.c_uint32), ("shard_index", C.c_uint32),
    ]


class synth_out(C.Structure):
    _fields_ = [
        ("n_keys", C.c_uint64), ("f_bytes", C.POINTER(C.c_uint8)), ("f_off", C.POINTER(C.c_uint64)),
        ("f_id", C.POINTER(C.c_uint64)), ("n_topics", C.c_uint64), ("t_bytes", C.POINTER(C.c_uint8)),
        ("t_off", C.POINTER(C.c_uint32)), ("f_bytes_len", C.c_uint64), ("t_bytes_len", C.c_uint64),
    ]


_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run __graft_entry__.build()")
        lib = C.CDLL(LIB)
        lib.synth_generate.argtypes = [C.POINTER(synth_params), C.POINTER(C.POINTER(synth_out))]
        lib.synth_generate.restype = C.c_int
        lib.synth_free.argtypes = [C.POINTER(synth_out)]
        lib.synth_free.restype = None
        _lib = lib
    return _lib


# Config parameter sets (scale=1.0 is the BASELINE.json size).
CONFIGS = {
    "A": dict(seed=0xE11A0001, n_filters=10_000, n_topics=100_000, min_levels=4, max_levels=4,
              vocab=[16, 256, 4096, 65536], p_fixed=0.2, p_plus=0.12, p_plus_level=0.25, p_hash=0.10,
              hash_geo=0.5, min_hash_depth=2, p_topic_hit=0.5),
    "B": dict(seed=0xE11A0002, n_filters=1_000_000, n_topics=1_000_000, min_levels=6, max_levels=6,
              vocab=[64, 1024, 4096, 65536, 65536, 65536], p_fixed=0.02, p_plus=0.10, p_plus_level=0.08,
              p_hash=0.05, hash_geo=0.5, min_hash_depth=3, p_topic_hit=0.5),
    # tenant(32)/region(64)/device(4096)/7 sub-levels(64 each); 30% '#' with explicit per-depth
    # weights (shallow '#' shared by many topics), 10% '+', plus 400 hot '#' filters carrying
    # 500-4000 subscriber ids each that 2% of publishes fall under (the p99 tail).
    "C": dict(seed=0xE11A0003, n_filters=10_000_000, n_topics=1_000_000, min_levels=10, max_levels=10,
              vocab=[32, 64, 4096, 64, 64, 64, 64, 64, 64, 64], p_fixed=0.02,
              p_plus=0.143, p_plus_level=0.12, p_hash=0.30, plus_hash_excl=1,
              hash_w=[0, 0, 0.013, 0.10, 0.15, 0.15, 0.15, 0.15, 0.15, 0.137], p_topic_hit=0.6,
              n_hot=400, hot_ids_min=500, hot_ids_max=4000, hot_depth_min=2, hot_depth_max=4, p_topic_hot=0.02),
    "D": dict(seed=0xE11A0004, n_filters=100_000_000, n_topics=1_000_000, min_levels=8, max_levels=8,
              vocab=[64, 1024, 4096, 65536, 65536, 65536, 65536, 65536], p_fixed=0.02, p_plus=0.10,
              p_plus_level=0.08, p_hash=0.05, hash_geo=0.5, min_hash_depth=3, p_topic_hit=0.5),
    "E": dict(seed=0xE11A0005, n_filters=1_000_000, n_topics=1_000_000, min_levels=3, max_levels=6,
              vocab=[64, 1024, 4096, 65536, 65536, 65536], p_fixed=0.02, p_plus=0.10, p_plus_level=0.08,
              p_hash=0.05, hash_geo=0.5, min_hash_depth=3, p_topic_hit=0.5, p_sys=0.05, p_sys_filter=0.02,
              p_multi=0.05, multi_max=4),
}


@dataclass
class Workload:
    name: str
    f_bytes: np.ndarray   # uint8
    f_off: np.ndarray     # uint64, n_keys+1
    f_id: np.ndarray      # uint64
    t_bytes: np.ndarray   # uint8
    t_off: np.ndarray     # uint32, n_topics+1

    @property
    def n_keys(self) -> int:
        return len(self.f_id)

    @property
    def n_topics(self) -> int:
        return len(self.t_off) - 1

    def filters(self) -> list:
        b, o = self.f_bytes.tobytes(), self.f_off
        return [b[o[i]:o[i + 1]] for i in range(self.n_keys)]

    def topics(self) -> list:
        b, o = self.t_bytes.tobytes(), self.t_off
        return [b[o[i]:o[i + 1]] for i in range(self.n_topics)]

    def topic_slice(self, lo: int, hi: int):
        """Topics [lo, hi) as a packed (bytes, offsets-from-0) batch."""
        o = self.t_off
        b0, b1 = int(o[lo]), int(o[hi])
        buf = np.concatenate([self.t_bytes[b0:b1], np.zeros(16, np.uint8)])
        return buf, (o[lo:hi + 1] - o[lo]).astype(np.uint32)


def params_for(name: str, scale: float = 1.0, n_topics: int | None = None, **over) -> synth_params:
    cfg = dict(CONFIGS[name])
    cfg.update(over)
    cfg["n_filters"] = max(1, int(cfg["n_filters"] * scale))
    if "n_hot" in cfg:
        cfg["n_hot"] = max(1, int(cfg["n_hot"] * scale)) if cfg["n_hot"] else 0
    if n_topics is not None:
        cfg["n_topics"] = n_topics
    p = synth_params()
    for k, v in cfg.items():
        if k == "vocab":
            arr = (C.c_uint32 * 16)()
            for i in range(16):
                arr[i] = v[min(i, len(v) - 1)]
            p.vocab = arr
        elif k == "hash_w":
            arr = (C.c_double * 16)()
            for i, x in enumerate(v[:16]):
                arr[i] = x
            p.hash_w = arr
        else:
            setattr(p, k, v)
    return p


def generate(name: str, scale: float = 1.0, n_topics: int | None = None, **over) -> Workload:
    lib = _load()
    p = params_for(name, scale, n_topics, **over)
    out = C.POINTER(synth_out)()
    rc = lib.synth_generate(C.byref(p), C.byref(out))
    if rc != 0:
        raise RuntimeError(f"synth_generate failed: {rc}")
    try:
        o = out.contents
        nk, nt = o.n_keys, o.n_topics
        fb = np.ctypeslib.as_array(o.f_bytes, shape=(o.f_bytes_len + 16,)).copy()
        fo = np.ctypeslib.as_array(o.f_off, shape=(nk + 1,)).copy()
        fi = np.ctypeslib.as_array(o.f_id, shape=(nk,)).copy()
        tb = np.ctypeslib.as_array(o.t_bytes, shape=(o.t_bytes_len + 16,)).copy()
        to = np.ctypeslib.as_array(o.t_off, shape=(nt + 1,)).copy()
    finally:
        lib.synth_free(out)
    return Workload(name, fb, fo, fi, tb, to)
