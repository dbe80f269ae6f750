"""oracle/ — TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference (ivangsm/emqx) topic matching:
  emqx_topic.py     pure-Python emqx_topic semantics (match/2, validate, parse, ...)
  trie_search.cpp   C++ emqx_trie_search over an Erlang-term-ordered key set
                    (the CPU baseline) + brute-force emqx_topic:match/2

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this
package, and only as the checker / the timed CPU baseline.  The product (emqx_amd/)
never imports it.

Parity pinning: the restatements are checked against every known-answer case of the
reference's suites transcribed into tests/golden/*.json (emqx_topic_SUITE,
emqx_topic_index_SUITE, emqx_trie_search_tests, emqx_router_SUITE, emqx_trie_SUITE).
The reference itself (Erlang/OTP) cannot be built or run in this image.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle_ts.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        lib.ots_build.restype = C.c_void_p
        lib.ots_build.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        lib.ots_free.argtypes = [C.c_void_p]
        lib.ots_size.restype = C.c_uint64
        lib.ots_size.argtypes = [C.c_void_p]
        lib.ots_match.restype = C.c_void_p
        lib.ots_match.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_int,
                                  C.c_int, C.c_void_p, C.c_void_p]
        lib.ots_res_off.restype = C.POINTER(C.c_uint64)
        lib.ots_res_ids.restype = C.POINTER(C.c_uint64)
        lib.ots_res_status.restype = C.POINTER(C.c_int32)
        lib.ots_res_src.restype = C.POINTER(C.c_uint32)
        lib.ots_res_nsrc.restype = C.c_uint64
        for f in ("ots_res_off", "ots_res_ids", "ots_res_status", "ots_res_free", "ots_res_src", "ots_res_nsrc"):
            getattr(lib, f).argtypes = [C.c_void_p]
        _lib = lib
    return _lib


ALGO_TRIE, ALGO_BRUTE = 0, 1
ALGO_FILTER = 2  # matches_filter/3: the queries are topic filters (emqx_trie_search.erl:186-189)
MODE_ALL, MODE_UNIQUE, MODE_FIRST = 0, 1, 2


class OrderedIndex:
    """The restated ETS ordered_set index over (filter, id) keys."""

    def __init__(self, f_bytes: np.ndarray, f_off: np.ndarray, ids: np.ndarray, flags: np.ndarray | None = None):
        self.lib = load()
        self._keep = (np.ascontiguousarray(f_bytes, dtype=np.uint8), np.ascontiguousarray(f_off, dtype=np.uint64),
                      np.ascontiguousarray(ids, dtype=np.uint64),
                      None if flags is None else np.ascontiguousarray(flags, dtype=np.uint32))
        b, o, i, fl = self._keep
        self.h = self.lib.ots_build(b.ctypes.data, o.ctypes.data, i.ctypes.data,
                                    None if fl is None else fl.ctypes.data, len(i))

    @classmethod
    def from_filters(cls, filters, ids=None, word_form=None):
        bs = [f.encode() if isinstance(f, str) else bytes(f) for f in filters]
        off = np.zeros(len(bs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(b) for b in bs])
        buf = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8)
        ids = np.arange(len(bs), dtype=np.uint64) if ids is None else np.asarray(ids, dtype=np.uint64)
        fl = None if word_form is None else np.asarray(word_form, dtype=np.uint32)
        return cls(buf, off, ids, fl)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.ots_free(self.h)
            self.h = None

    def size(self) -> int:
        return self.lib.ots_size(self.h)

    def match(self, t_bytes: np.ndarray, t_off: np.ndarray, algo=ALGO_TRIE, mode=MODE_ALL, threads=1,
              with_src=False):
        """-> (off[n+1], ids[], status[n]): per topic, sorted matching ids.  With with_src,
        also the flat list of matched input-key indices in walk (term) order, per topic
        in topic order (counts = ids counts except under MODE_UNIQUE)."""
        tb = np.ascontiguousarray(t_bytes, dtype=np.uint8)
        to = np.ascontiguousarray(t_off, dtype=np.uint32)
        n = len(to) - 1
        r = self.lib.ots_match(self.h, tb.ctypes.data, to.ctypes.data, n, algo, mode, threads, 0, None, None)
        try:
            off = np.ctypeslib.as_array(self.lib.ots_res_off(r), shape=(n + 1,)).copy()
            tot = int(off[-1])
            ids = (np.ctypeslib.as_array(self.lib.ots_res_ids(r), shape=(tot,)).copy() if tot
                   else np.zeros(0, dtype=np.uint64))
            st = np.ctypeslib.as_array(self.lib.ots_res_status(r), shape=(n,)).copy() if n else np.zeros(0, np.int32)
            ns = self.lib.ots_res_nsrc(r)
            src = (np.ctypeslib.as_array(self.lib.ots_res_src(r), shape=(ns,)).copy() if ns
                   else np.zeros(0, dtype=np.uint32))
        finally:
            self.lib.ots_res_free(r)
        if with_src:
            return off, ids, st, src
        return off, ids, st

    def count(self, t_bytes, t_off, algo=ALGO_TRIE, mode=MODE_ALL, threads=1):
        """Counts-only run (the timed CPU baseline): -> (counts[n], checksum)."""
        tb = np.ascontiguousarray(t_bytes, dtype=np.uint8)
        to = np.ascontiguousarray(t_off, dtype=np.uint32)
        n = len(to) - 1
        cnt = np.zeros(n, dtype=np.uint32)
        cs = C.c_uint64()
        self.lib.ots_match(self.h, tb.ctypes.data, to.ctypes.data, n, algo, mode, threads, 1, cnt.ctypes.data,
                           C.byref(cs))
        return cnt, cs.value


INTERSECT_FALSE, INTERSECT_BADHASH = -1, -2


def intersect_packed(a_buf, a_off, b_buf, b_off, threads=1):
    """emqx_topic:intersection/2 over packed pairs (C++ restatement, trie_search.cpp
    ots_intersect): -> (lens i32[n]: result length, INTERSECT_FALSE or INTERSECT_BADHASH;
    starts u64[n]; out u8 buffer), pair i's result at out[starts[i]: starts[i] + lens[i]]."""
    lib = load()
    lib.ots_intersect.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p,
                                  C.c_void_p]
    ab = np.ascontiguousarray(a_buf, dtype=np.uint8)
    ao = np.ascontiguousarray(a_off, dtype=np.uint32)
    bb = np.ascontiguousarray(b_buf, dtype=np.uint8)
    bo = np.ascontiguousarray(b_off, dtype=np.uint32)
    n = len(ao) - 1
    out = np.zeros(int(ao[-1]) + int(bo[-1]) + 16, dtype=np.uint8)
    lens = np.zeros(max(n, 1), dtype=np.int32)
    lib.ots_intersect(ab.ctypes.data, ao.ctypes.data, bb.ctypes.data, bo.ctypes.data, n, threads, out.ctypes.data,
                      lens.ctypes.data)
    return lens[:n], ao[:n].astype(np.uint64) + bo[:n].astype(np.uint64), out


def intersect(pairs, threads=1):
    """intersection/2 per (a, b) bytes pair: bytes, False, or the string 'badhash' where
    join/1 raises error('topic_invalid_#')."""
    def pack(ts):
        off = np.zeros(len(ts) + 1, dtype=np.uint32)
        if ts:
            off[1:] = np.cumsum([len(t) for t in ts])
        return np.frombuffer(b"".join(ts) + b"\0" * 16, dtype=np.uint8), off
    ab, ao = pack([p[0] for p in pairs])
    bb, bo = pack([p[1] for p in pairs])
    lens, starts, out = intersect_packed(ab, ao, bb, bo, threads)
    raw = out.tobytes()
    res = []
    for L, s in zip(lens.tolist(), starts.tolist()):
        res.append(False if L == INTERSECT_FALSE else "badhash" if L == INTERSECT_BADHASH else raw[s:s + L])
    return res
