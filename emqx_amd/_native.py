"""ctypes binding of the C-ABI in include/emqx_tm.h (libemqx_tm.so, built in-tree).

The product path is the HIP library and nothing else: if the library is missing,
or the process has no gfx950 device, engine creation raises.  There is no CPU
fallback (the CPU restatement of the reference lives in oracle/ and is test
infrastructure only).

A process that also uses torch on the GPU must import torch BEFORE this library is loaded:
torch bundles its own libamdhip64.so.7 and the first HIP runtime loaded serves the process.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# EMQX_TM_LIB: path of an alternative build of the same library (kernel-parameter sweeps
# by tools/sweep.py); unset = the in-tree product build.
LIB_PATH = os.environ.get("EMQX_TM_LIB") or os.path.join(HERE, "libemqx_tm.so")

TM_OK = 0
TM_EINVAL = -1
TM_ENOMEM = -2
TM_EDEVICE = -3
TM_ESTATE = -4
TM_ENOTFOUND = -5

TM_TOPIC_OK = 0
TM_BADARG = 1

TM_OP_ADD = 1
TM_OP_DEL = 2
TM_KEY_WORDS = 1

TM_MATCH_ALL = 0
TM_MATCH_UNIQUE = 1
TM_MATCH_FIRST = 2
TM_MATCH_COUNT = 3
TM_MATCH_AGGRE = 4

TM_ID_SHARED = 1 << 63


def shared_id(group: int, member: int) -> int:
    """TM_SHARED_ID(group, member): the route id of a $share dest {Group, Node}."""
    return TM_ID_SHARED | (group << 32) | (member & 0xFFFFFFFF)


TM_CFG_FORCE_SLOW = 1
TM_CFG_RECORD_PATCH = 2
TM_CFG_FAIL_HOST_CALLS = 4
TM_CFG_FAIL_FLUSH_ONCE = 8
TM_CFG_EDGE_EXACT = 16
TM_RES_KEYS_OVERFLOW = 1
TM_RES_IDS_OVERFLOW = 2

# every symbol include/emqx_tm.h declares (tests check the .so exports them all)
EXPORTS = (
    "tm_abi_version", "tm_create", "tm_destroy", "tm_last_error", "tm_create_last_error", "tm_apply", "tm_apply_packed",
    "tm_commit_epoch", "tm_match_batch", "tm_match_device", "tm_device_sync",
    "tm_reserve_matches", "tm_key_info", "tm_key_ids", "tm_stats", "tm_debug_stats", "tm_debug_timing",
    "tm_result_ids_device", "tm_merge_shards_device", "tm_merge_shards", "tm_match_device_mode",
    "tm_match_filter_batch", "tm_intersect_batch", "tm_result_ids_device_ex", "tm_image_size", "tm_image_export",
    "tm_replica_create", "tm_replica_load", "tm_patch_size", "tm_patch_export", "tm_replica_apply_patch",
    "tm_discard_staged", "tm_result_release", "tm_match_batch_runs", "tm_runs_release", "tm_build_info",
    "tm_match_ids_device", "tm_merge_shard_ids_device", "tm_debug_depth_stats", "tm_match_device_set",
    "tm_debug_image_check", "tm_match_filter_batch_runs",
    "tm_device_sync_set", "tm_debug_bounds", "tm_debug_commit_marks",
)
# every symbol include/emqx_tm_batcher.h declares
BATCHER_EXPORTS = (
    "tm_batcher_create", "tm_batcher_create_fn", "tm_batcher_destroy", "tm_batcher_submit", "tm_batcher_match",
    "tm_batcher_apply", "tm_batcher_commit", "tm_batcher_stats_get", "tm_batcher_submit_spans",
    "tm_batcher_stats_reset", "tm_batcher_submit_spans32", "tm_batcher_windows",
)


class tm_config(C.Structure):
    _fields_ = [
        ("device", C.c_int32), ("flags", C.c_uint32),
        ("reserve_keys", C.c_uint32), ("reserve_nodes", C.c_uint32),
        ("reserve_topics", C.c_uint32), ("reserve_matches", C.c_uint32),
        ("seg_chunks", C.c_uint32), ("edge_load_inv", C.c_uint32),
        ("topics_per_wave", C.c_uint32), ("max_nodes", C.c_uint32), ("max_list_words", C.c_uint32),
    ]


class tm_op(C.Structure):
    _fields_ = [
        ("op", C.c_uint32), ("flags", C.c_uint32),
        ("filter", C.c_void_p), ("filter_len", C.c_uint32), ("_pad", C.c_uint32),
        ("id", C.c_uint64),
    ]


class tm_result(C.Structure):
    _fields_ = [
        ("n", C.c_uint32), ("_pad", C.c_uint32), ("total", C.c_uint64),
        ("off", C.POINTER(C.c_uint32)), ("cnt", C.POINTER(C.c_uint32)),
        ("keys", C.POINTER(C.c_uint32)), ("status", C.POINTER(C.c_int32)),
    ]


class tm_intersect_result(C.Structure):
    _fields_ = [("n", C.c_uint32), ("_pad", C.c_uint32), ("off", C.POINTER(C.c_uint64)),
                ("len", C.POINTER(C.c_int32)), ("bytes", C.POINTER(C.c_uint8))]


TM_INTERSECT_FALSE, TM_INTERSECT_BADHASH = -1, -2
TM_MATCH_TOPIC_WORDS = 0x100  # OR'd into a tm_match_batch mode: '/'-joined word-list topics


class tm_dev_result(C.Structure):
    _fields_ = [
        ("n", C.c_uint32), ("_pad", C.c_uint32),
        ("d_off", C.c_void_p), ("d_cnt", C.c_void_p), ("d_keys", C.c_void_p),
        ("d_status", C.c_void_p), ("d_total", C.c_void_p), ("keys_cap", C.c_uint64),
    ]


class tm_stats_t(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "epoch", "n_keys", "n_nodes", "n_words", "edge_slots", "word_slots", "list_words",
        "device_bytes", "n_full_rebuilds", "n_delta_commits", "n_slow_topics",
        "commit_apply_us", "commit_lists_us", "commit_upload_us", "n_deep_keys", "n_filter_onepass",
        "n_filter_twopass", "commit_stall_us", "n_commits_refused", "n_staged", "standby_bytes")]


class tm_span(C.Structure):
    _fields_ = [("ids", C.c_void_p), ("n", C.c_uint64)]


class tm_runs_result(C.Structure):
    _fields_ = [("n", C.c_uint32), ("_pad", C.c_uint32), ("epoch", C.c_uint64), ("total_ids", C.c_uint64),
                ("total_spans", C.c_uint64), ("span_off", C.POINTER(C.c_uint32)), ("span_cnt", C.POINTER(C.c_uint32)),
                ("spans", C.POINTER(tm_span)),
                ("kcnt", C.POINTER(C.c_uint32)), ("status", C.POINTER(C.c_int32))]


class tm_batcher_config(C.Structure):
    _fields_ = [("max_batch", C.c_uint32), ("max_wait_us", C.c_uint32), ("mode", C.c_uint32),
                ("delivery_threads", C.c_uint32), ("transport", C.c_uint32)]


TM_TRANSPORT_AUTO, TM_TRANSPORT_IDS, TM_TRANSPORT_RUNS = 0, 1, 2


class tm_batch_view(C.Structure):
    _fields_ = [("off", C.c_void_p), ("cnt", C.c_void_p), ("ids", C.c_void_p), ("status", C.c_void_p)]


class tm_batcher_stats(C.Structure):
    _fields_ = [("batches", C.c_uint64), ("publishes", C.c_uint64), ("max_batch_seen", C.c_uint64),
                ("backend_us", C.c_uint64), ("lat_p50_us", C.c_double), ("lat_p99_us", C.c_double),
                ("lat_max_us", C.c_double), ("cut_us", C.c_uint64), ("enqueue_us", C.c_uint64),
                ("gpu_wait_us", C.c_uint64), ("copy_us", C.c_uint64), ("deliver_us", C.c_uint64),
                ("lat_mean_us", C.c_double), ("lat_count", C.c_uint64), ("lat_p999_us", C.c_double),
                ("window_s", C.c_double)]


class tm_batcher_window(C.Structure):
    _fields_ = [("n", C.c_uint32), ("flags", C.c_uint32)] + [(k, C.c_uint64) for k in (
        "t_oldest", "t_cut", "t_queued", "t_gpu", "t_ready", "t_deliver", "t_done", "epoch", "t_slot")] + [
        ("cut_cpu_us", C.c_uint32), ("cut_ivcsw", C.c_uint16), ("wait_ivcsw", C.c_uint16),
        ("del_cpu_us", C.c_uint32), ("del_wall_us", C.c_uint32), ("del_ivcsw", C.c_uint32), ("reserved", C.c_uint32)]


TM_BATCHER_WINDOWS = 16384
TM_WIN_RERUN, TM_WIN_RUNS, TM_WIN_FAILED = 1, 2, 4

tm_match_cb = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.POINTER(C.c_uint64), C.c_uint32)
tm_spans_cb = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_void_p, C.c_uint32, C.c_uint64)
tm_spans32_cb = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_void_p, C.c_uint32, C.c_uint64)
tm_batch_fn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint32), C.c_uint32, C.c_uint32,
                          C.POINTER(tm_batch_view))

_lib = None


def load() -> C.CDLL:
    """Load libemqx_tm.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP extension is the only matching path; there is no CPU fallback)")
    lib = C.CDLL(LIB_PATH)
    P = C.POINTER
    lib.tm_abi_version.restype = C.c_uint32
    lib.tm_build_info.restype = C.c_char_p
    lib.tm_create.argtypes = [P(tm_config), P(C.c_void_p)]
    lib.tm_destroy.argtypes = [C.c_void_p]
    lib.tm_destroy.restype = None
    lib.tm_last_error.argtypes = [C.c_void_p]
    lib.tm_last_error.restype = C.c_char_p
    lib.tm_create_last_error.argtypes = []
    lib.tm_create_last_error.restype = C.c_char_p
    lib.tm_apply.argtypes = [C.c_void_p, P(tm_op), C.c_size_t]
    lib.tm_apply_packed.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_size_t]
    lib.tm_commit_epoch.argtypes = [C.c_void_p, P(C.c_uint64)]
    lib.tm_discard_staged.argtypes = [C.c_void_p, P(C.c_uint64)]
    lib.tm_result_release.argtypes = [C.c_void_p]
    lib.tm_match_batch_runs.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, P(tm_runs_result)]
    lib.tm_runs_release.argtypes = [C.c_void_p]
    lib.tm_match_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, P(tm_result)]
    lib.tm_intersect_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                       P(tm_intersect_result)]
    lib.tm_match_filter_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, P(tm_result)]
    lib.tm_match_filter_batch_runs.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                               P(tm_runs_result)]
    lib.tm_match_device.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64,
                                    C.c_void_p, P(tm_dev_result)]
    lib.tm_device_sync.argtypes = [C.c_void_p]
    lib.tm_device_sync_set.argtypes = [C.c_void_p, C.c_uint32]
    lib.tm_match_device_set.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64,
                                        C.c_uint32, C.c_void_p, P(tm_dev_result)]
    lib.tm_match_device_mode.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                                         C.c_void_p, P(tm_dev_result)]
    lib.tm_reserve_matches.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32]
    lib.tm_key_info.argtypes = [C.c_void_p, C.c_uint32, P(C.c_uint64), P(C.c_uint32), C.c_void_p,
                                C.c_uint32, P(C.c_uint32)]
    lib.tm_key_ids.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
    lib.tm_stats.argtypes = [C.c_void_p, P(tm_stats_t)]
    lib.tm_debug_timing.argtypes = [C.c_void_p, C.c_int, P(C.c_float)]
    lib.tm_debug_stats.argtypes = [C.c_void_p, C.c_int, P(C.c_uint64)]
    lib.tm_debug_depth_stats.argtypes = [C.c_void_p, P(C.c_uint64)]
    lib.tm_debug_image_check.argtypes = [C.c_void_p, P(C.c_uint32)]
    lib.tm_debug_bounds.argtypes = [C.c_void_p, P(C.c_uint64), C.c_char_p, C.c_uint32]
    lib.tm_debug_commit_marks.argtypes = [C.c_void_p, P(C.c_uint64)]
    lib.tm_result_ids_device.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    lib.tm_result_ids_device_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.tm_match_ids_device.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                                        C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.tm_merge_shard_ids_device.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p,
                                              C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64,
                                              C.c_void_p]
    lib.tm_image_size.argtypes = [C.c_void_p, P(C.c_uint64)]
    lib.tm_image_export.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
    lib.tm_replica_create.argtypes = [P(tm_config), C.c_void_p, C.c_uint64, C.c_void_p, P(C.c_void_p)]
    lib.tm_replica_load.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
    lib.tm_patch_size.argtypes = [C.c_void_p, P(C.c_uint64), P(C.c_int)]
    lib.tm_patch_export.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    lib.tm_replica_apply_patch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    lib.tm_merge_shards_device.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64,
                                           C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
    lib.tm_merge_shards.argtypes = [C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                    C.c_void_p, C.c_uint64]
    for name in EXPORTS:
        if name not in ("tm_destroy", "tm_last_error", "tm_create_last_error", "tm_abi_version", "tm_build_info"):
            getattr(lib, name).restype = C.c_int
    lib.tm_batcher_create.argtypes = [C.c_void_p, P(tm_batcher_config), P(C.c_void_p)]
    lib.tm_batcher_create_fn.argtypes = [tm_batch_fn, C.c_void_p, P(tm_batcher_config), P(C.c_void_p)]
    lib.tm_batcher_destroy.argtypes = [C.c_void_p]
    lib.tm_batcher_destroy.restype = None
    lib.tm_batcher_submit.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, tm_match_cb, C.c_void_p]
    lib.tm_batcher_submit_spans.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, tm_spans_cb, C.c_void_p]
    lib.tm_batcher_submit_spans32.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, tm_spans32_cb, C.c_void_p]
    lib.tm_batcher_match.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, P(C.c_uint32),
                                     P(C.c_int32)]
    lib.tm_batcher_apply.argtypes = [C.c_void_p, P(tm_op), C.c_size_t]
    lib.tm_batcher_commit.argtypes = [C.c_void_p, P(C.c_uint64)]
    lib.tm_batcher_stats_get.argtypes = [C.c_void_p, P(tm_batcher_stats)]
    lib.tm_batcher_stats_reset.argtypes = [C.c_void_p]
    lib.tm_batcher_windows.argtypes = [C.c_void_p, P(tm_batcher_window), C.c_uint32, P(C.c_uint32)]
    for name in BATCHER_EXPORTS:
        if name != "tm_batcher_destroy":
            getattr(lib, name).restype = C.c_int
    _lib = lib
    return lib


def debug_bounds(engine=None):
    """tm_debug_bounds: (hits, first findings) of the bounds-checked debug build
    (libemqx_tm_bounds.so) over the whole process -- out-of-bounds device indices, overwritten
    canary tails, host copies past a buffer's end -- or None with the product build."""
    lib = load()
    hits, msg = C.c_uint64(), C.create_string_buffer(2048)
    rc = lib.tm_debug_bounds(engine.h if engine is not None else None, C.byref(hits), msg, len(msg))
    if rc == TM_ENOTFOUND:
        return None
    if rc != TM_OK:
        raise TMError(rc, "tm_debug_bounds failed")
    return hits.value, msg.value.decode(errors="replace")


def build_sha() -> str:
    """The source hash the loaded library was built from (tm_build_info)."""
    info = load().tm_build_info().decode()
    return dict(kv.split("=", 1) for kv in info.split()).get("src_sha", "")


def check_build():
    """Fail loudly when the library does not match the sources next to it."""
    from emqx_amd.build import src_sha
    have, want = build_sha(), src_sha()
    if have != want:
        raise RuntimeError(f"{LIB_PATH} was built from other sources (src_sha {have[:12]} != {want[:12]}): "
                           "run __graft_entry__.build()")
    return have


def merge_shards(counts: np.ndarray, ids: np.ndarray):
    """Host form of the shard merge (tm_merge_shards): counts [G, n] u32, ids [G, stride]
    u64 (shard r's topic-major ids) -> (off[n+1] u32, merged ids u64)."""
    lib = load()
    counts = np.ascontiguousarray(counts, dtype=np.uint32)
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    G, n = counts.shape
    stride = ids.shape[1] if ids.ndim == 2 else 0
    total = int(counts.sum(dtype=np.uint64))
    off = np.zeros(n + 1, dtype=np.uint32)
    out = np.zeros(max(total, 1), dtype=np.uint64)
    rc = lib.tm_merge_shards(G, n, counts.ctypes.data, ids.ctypes.data, stride, off.ctypes.data, out.ctypes.data,
                             total)
    if rc != TM_OK:
        raise TMError(rc, "tm_merge_shards failed")
    return off, out[:total]


class TopicInvalidHash(ValueError):
    """error('topic_invalid_#') from emqx_topic:join/1 (emqx_topic.erl:319-320)."""


class TMError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"tm error {rc}: {msg}")
        self.rc = rc


def pack_topics(topics) -> tuple[np.ndarray, np.ndarray]:
    """Topics (bytes/str) -> (uint8 bytes, uint32 offsets[n+1])."""
    bs = [t.encode() if isinstance(t, str) else bytes(t) for t in topics]
    off = np.zeros(len(bs) + 1, dtype=np.uint32)
    if bs:
        off[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64).astype(np.uint32)
    buf = np.frombuffer(b"".join(bs) + b"\0" * 16, dtype=np.uint8)
    return buf, off


class Engine:
    """One engine = one GPU.  Thin owner of a tm_engine*."""

    def __init__(self, device: int = 0, *, force_slow: bool = False, reserve_keys: int = 0,
                 reserve_nodes: int = 0, reserve_matches: int = 0, seg_chunks: int = 0, edge_load_inv: int = 0,
                 topics_per_wave: int = 0, record_patch: bool = False, max_nodes: int = 0,
                 max_list_words: int = 0, flags: int = 0, _image=None):
        self.lib = load()
        cfg = tm_config()
        cfg.device = device
        cfg.flags = (TM_CFG_FORCE_SLOW if force_slow else 0) | (TM_CFG_RECORD_PATCH if record_patch else 0) | flags
        cfg.reserve_keys = reserve_keys
        cfg.reserve_nodes = reserve_nodes
        cfg.reserve_matches = reserve_matches
        cfg.seg_chunks = seg_chunks
        cfg.topics_per_wave = topics_per_wave
        cfg.max_nodes = max_nodes
        cfg.max_list_words = max_list_words
        cfg.edge_load_inv = edge_load_inv or int(os.environ.get("EMQX_TM_EDGE_LOAD_INV", "0"))
        h = C.c_void_p()
        if _image is None:
            rc = self.lib.tm_create(C.byref(cfg), C.byref(h))
        else:  # (device pointer, bytes, stream) of a master's image on this device
            rc = self.lib.tm_replica_create(C.byref(cfg), C.c_void_p(_image[0]), _image[1],
                                            C.c_void_p(_image[2]) if _image[2] else None, C.byref(h))
        if rc != TM_OK:
            why = self.lib.tm_create_last_error().decode(errors="replace")
            raise TMError(rc, f"tm_create failed: {why or 'no gfx950 HIP device visible?'}")
        self.h = h
        self.device = device
        self.replica = _image is not None

    @classmethod
    def replica_from_image(cls, device: int, d_image: int, nbytes: int, stream: int = 0, **kw) -> "Engine":
        """A read replica (tm_replica_create) from a master's device image on `device`."""
        return cls(device, _image=(d_image, nbytes, stream), **kw)

    # ---- replicated mode: image + epoch patches (include/emqx_tm.h)
    def image_size(self) -> int:
        n = C.c_uint64()
        self._check(self.lib.tm_image_size(self.h, C.byref(n)))
        return n.value

    def image_export(self, d_dst: int, cap: int, stream: int = 0):
        self._check(self.lib.tm_image_export(self.h, C.c_void_p(d_dst), cap, C.c_void_p(stream) if stream else None))

    def replica_load(self, d_image: int, nbytes: int, stream: int = 0):
        self._check(self.lib.tm_replica_load(self.h, C.c_void_p(d_image), nbytes,
                                             C.c_void_p(stream) if stream else None))

    def patch_export(self):
        """The last commit's device changes: (bytes as a uint8 array, full) — full means the
        commit re-uploaded everything and replicas must reload from an image."""
        n, full = C.c_uint64(), C.c_int()
        self._check(self.lib.tm_patch_size(self.h, C.byref(n), C.byref(full)))
        buf = np.zeros(n.value, dtype=np.uint8)
        self._check(self.lib.tm_patch_export(self.h, buf.ctypes.data, n.value))
        return buf, bool(full.value)

    def apply_patch(self, patch: np.ndarray):
        patch = np.ascontiguousarray(patch, dtype=np.uint8)
        self._check(self.lib.tm_replica_apply_patch(self.h, patch.ctypes.data, len(patch)))

    def close(self):
        if getattr(self, "h", None):
            self.lib.tm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != TM_OK:
            raise TMError(rc, self.lib.tm_last_error(self.h).decode(errors="replace"))

    # ---- writes
    def apply(self, ops):
        """ops: iterable of (op, filter_bytes, id[, flags])."""
        ops = list(ops)
        if not ops:
            return
        arr = (tm_op * len(ops))()
        keep = []
        for i, o in enumerate(ops):
            op, f, ident = o[0], o[1], o[2]
            flags = o[3] if len(o) > 3 else 0
            fb = f.encode() if isinstance(f, str) else bytes(f)
            cb = C.create_string_buffer(fb, len(fb) + 1)
            keep.append(cb)
            arr[i].op = op
            arr[i].flags = flags
            arr[i].filter = C.cast(cb, C.c_void_p)
            arr[i].filter_len = len(fb)
            arr[i].id = ident
        self._check(self.lib.tm_apply(self.h, arr, len(ops)))

    def apply_packed(self, op: int, buf: np.ndarray, off: np.ndarray, ids: np.ndarray, flags=None):
        """Bulk ops: filter i = buf[off[i]:off[i+1]] (off uint64, n+1 entries), id ids[i]."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        n = len(ids)
        assert len(off) == n + 1
        fl = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint32)
        self._check(self.lib.tm_apply_packed(self.h, op, buf.ctypes.data, off.ctypes.data, ids.ctypes.data,
                                             None if fl is None else fl.ctypes.data, n))

    def commit(self) -> int:
        ep = C.c_uint64()
        self._check(self.lib.tm_commit_epoch(self.h, C.byref(ep)))
        return ep.value

    def discard_staged(self) -> int:
        """Drop every staged op (tm_discard_staged); returns how many."""
        n = C.c_uint64()
        self._check(self.lib.tm_discard_staged(self.h, C.byref(n)))
        return n.value

    def result_release(self):
        """Free this thread's host result buffers (tm_result_release)."""
        self._check(self.lib.tm_result_release(self.h))

    # ---- reads
    def match_packed(self, buf: np.ndarray, off: np.ndarray, mode: int = TM_MATCH_ALL):
        """Match a packed batch; returns (off, cnt, keys, status) numpy copies."""
        n = len(off) - 1
        res = tm_result()
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint32)
        self._check(self.lib.tm_match_batch(self.h, buf.ctypes.data, off.ctypes.data, n, mode, C.byref(res)))
        if n == 0:
            e = np.zeros(0, dtype=np.uint32)
            return e, e, e, np.zeros(0, dtype=np.int32)
        o = np.ctypeslib.as_array(res.off, shape=(n,)).copy()
        c = np.ctypeslib.as_array(res.cnt, shape=(n,)).copy()
        st = np.ctypeslib.as_array(res.status, shape=(n,)).copy()
        # UNIQUE / AGGRE lists sit at the full result's offsets: copy the whole span
        span = int((o.astype(np.uint64) + c).max()) if res.total else 0
        k = (np.ctypeslib.as_array(res.keys, shape=(span,)).copy() if span
             else np.zeros(0, dtype=np.uint32))
        return o, c, k, st

    def match_filter_packed(self, buf: np.ndarray, off: np.ndarray, mode: int = TM_MATCH_ALL):
        """tm_match_filter_batch (matches_filter/3) on packed topic filters; returns
        (off, cnt, keys, status) numpy copies, keys per query in walk order."""
        n = len(off) - 1
        res = tm_result()
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint32)
        self._check(self.lib.tm_match_filter_batch(self.h, buf.ctypes.data, off.ctypes.data, n, mode, C.byref(res)))
        if n == 0:
            e = np.zeros(0, dtype=np.uint32)
            return e, e, e, np.zeros(0, dtype=np.int32)
        o = np.ctypeslib.as_array(res.off, shape=(n,)).copy()
        c = np.ctypeslib.as_array(res.cnt, shape=(n,)).copy()
        st = np.ctypeslib.as_array(res.status, shape=(n,)).copy()
        k = (np.ctypeslib.as_array(res.keys, shape=(int(res.total),)).copy() if res.total
             else np.zeros(0, dtype=np.uint32))
        return o, c, k, st

    def match_filter_view(self, buf: np.ndarray, off: np.ndarray, mode: int = TM_MATCH_ALL) -> tm_result:
        """tm_match_filter_batch without copying (engine-owned result, valid until the next
        call).  For timing the C-ABI host path."""
        res = tm_result()
        self._check(self.lib.tm_match_filter_batch(self.h, buf.ctypes.data, off.ctypes.data, len(off) - 1, mode,
                                                   C.byref(res)))
        return res

    def intersect(self, pairs):
        """emqx_topic:intersection/2 on the GPU for each (a, b) pair (tm_intersect_batch):
        bytes, False, or TopicInvalidHash where join/1 raises error('topic_invalid_#')."""
        a_buf, a_off = pack_topics([p[0] for p in pairs])
        b_buf, b_off = pack_topics([p[1] for p in pairs])
        res = tm_intersect_result()
        n = len(pairs)
        self._check(self.lib.tm_intersect_batch(self.h, a_buf.ctypes.data, a_off.ctypes.data, b_buf.ctypes.data,
                                                b_off.ctypes.data, n, C.byref(res)))
        if n == 0:
            return []
        off = np.ctypeslib.as_array(res.off, shape=(n,))
        ln = np.ctypeslib.as_array(res.len, shape=(n,))
        cap = int(off[-1]) + max(int(ln[-1]), 0)
        raw = bytes(np.ctypeslib.as_array(res.bytes, shape=(max(cap, 1),))) if cap else b""
        out = []
        for i in range(n):
            L = int(ln[i])
            if L == TM_INTERSECT_FALSE:
                out.append(False)
            elif L == TM_INTERSECT_BADHASH:
                out.append(TopicInvalidHash())
            else:
                out.append(raw[int(off[i]):int(off[i]) + L])
        return out

    def match_filter(self, filters, mode: int = TM_MATCH_ALL):
        """List of topic filters -> list of key-handle lists in walk order (None for a
        query the engine refuses: '#' before the last level)."""
        buf, off = pack_topics(filters)
        o, c, k, st = self.match_filter_packed(buf, off, mode)
        return [None if st[i] == TM_BADARG else k[o[i]:o[i] + c[i]].tolist() for i in range(len(filters))]

    def match_packed_view(self, buf: np.ndarray, off: np.ndarray, mode: int = TM_MATCH_ALL) -> tm_result:
        """tm_match_batch without copying: the engine-owned tm_result (valid until the next
        call on this engine).  For timing the C-ABI host path."""
        res = tm_result()
        self._check(self.lib.tm_match_batch(self.h, buf.ctypes.data, off.ctypes.data, len(off) - 1, mode,
                                            C.byref(res)))
        return res

    def match_runs_view(self, buf: np.ndarray, off: np.ndarray) -> tm_runs_result:
        """tm_match_batch_runs without copying: spans into the engine's host id arena, under this
        thread's read lease until its next runs call or runs_release()."""
        res = tm_runs_result()
        self._check(self.lib.tm_match_batch_runs(self.h, buf.ctypes.data, off.ctypes.data, len(off) - 1,
                                                 C.byref(res)))
        return res

    @staticmethod
    def _expand_runs(res, n):
        """A tm_runs_result, expanded: (off u32[n+1], ids u64, kcnt u32[n], status i32[n]);
        item i's ids are ids[off[i]:off[i+1]], its spans in order."""
        if n == 0:
            return np.zeros(1, np.uint32), np.zeros(0, np.uint64), np.zeros(0, np.uint32), np.zeros(0, np.int32)
        kcnt = np.ctypeslib.as_array(res.kcnt, shape=(n,)).copy()
        st = np.ctypeslib.as_array(res.status, shape=(n,)).copy()
        soff = np.ctypeslib.as_array(res.span_off, shape=(n,)).copy()
        scnt = np.ctypeslib.as_array(res.span_cnt, shape=(n,)).copy()
        ids = np.zeros(int(res.total_ids), dtype=np.uint64)
        o = np.zeros(n + 1, dtype=np.uint32)
        np.cumsum(kcnt, out=o[1:])
        for i in range(n):
            at = int(o[i])
            for j in range(int(soff[i]), int(soff[i]) + int(scnt[i])):
                sp = res.spans[j]
                k = int(sp.n)
                if k:
                    ids[at:at + k] = np.ctypeslib.as_array(C.cast(sp.ids, C.POINTER(C.c_uint64)), shape=(k,))
                at += k
            assert at == int(o[i + 1]), "spans of an item disagree with its id count"
        return o, ids, kcnt, st

    def match_runs(self, buf: np.ndarray, off: np.ndarray):
        """tm_match_batch_runs, expanded: (off u32[n+1], ids u64, kcnt u32[n], status i32[n]).
        Topic i's ids are ids[off[i]:off[i+1]] (the multiset tm_match_batch + key ids gives)."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint32)
        res = self.match_runs_view(buf, off)
        try:
            return self._expand_runs(res, len(off) - 1)
        finally:
            self._check(self.lib.tm_runs_release(self.h))

    def match_filter_runs_view(self, buf: np.ndarray, off: np.ndarray, mode: int = TM_MATCH_ALL) -> tm_runs_result:
        """tm_match_filter_batch_runs without copying: spans of the sorted key ids, valid until
        this thread's next such call or result_release()."""
        res = tm_runs_result()
        self._check(self.lib.tm_match_filter_batch_runs(self.h, buf.ctypes.data, off.ctypes.data, len(off) - 1, mode,
                                                        C.byref(res)))
        return res

    def match_filter_runs(self, buf: np.ndarray, off: np.ndarray, mode: int = TM_MATCH_ALL):
        """tm_match_filter_batch_runs, expanded: (off, ids u64 in walk order, kcnt, status)."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint32)
        return self._expand_runs(self.match_filter_runs_view(buf, off, mode), len(off) - 1)

    def match(self, topics, mode: int = TM_MATCH_ALL):
        """List of topics -> list of key-handle lists (None for badarg topics)."""
        buf, off = pack_topics(topics)
        o, c, k, st = self.match_packed(buf, off, mode)
        out = []
        for i in range(len(topics)):
            if st[i] == TM_BADARG:
                out.append(None)
            else:
                out.append(k[o[i]:o[i] + c[i]].tolist())
        return out

    def match_words(self, word_lists, mode: int = TM_MATCH_ALL):
        """matches/3 with pre-split topics (TM_MATCH_TOPIC_WORDS): each topic a non-empty list of
        byte words (no '/' inside a word); list of key-handle lists.  A "+" or "#" word is a
        plain word here, and keys given as binaries never match (match_topics/4)."""
        topics = []
        for ws in word_lists:
            bs = [w.encode() if isinstance(w, str) else bytes(w) for w in ws]
            if not bs or any(b"/" in b for b in bs):
                raise ValueError(f"word list {ws!r} has no '/'-joined form")
            topics.append(b"/".join(bs))
        buf, off = pack_topics(topics)
        o, c, k, st = self.match_packed(buf, off, mode | TM_MATCH_TOPIC_WORDS)
        return [k[o[i]:o[i] + c[i]].tolist() for i in range(len(topics))]

    def key_info(self, key: int):
        ident = C.c_uint64()
        flags = C.c_uint32()
        ln = C.c_uint32()
        self._check(self.lib.tm_key_info(self.h, key, C.byref(ident), C.byref(flags), None, 0, C.byref(ln)))
        buf = C.create_string_buffer(max(ln.value, 1))
        self._check(self.lib.tm_key_info(self.h, key, C.byref(ident), C.byref(flags), buf, ln.value,
                                         C.byref(ln)))
        return ident.value, buf.raw[:ln.value], flags.value

    def key_ids(self, keys: np.ndarray) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        out = np.zeros(len(keys), dtype=np.uint64)
        if len(keys):
            self._check(self.lib.tm_key_ids(self.h, keys.ctypes.data, len(keys), out.ctypes.data))
        return out

    def timing(self, enable: bool):
        """Arm (True) / read (False -> ms of k_match_fast in the last match) kernel timing."""
        ms = C.c_float()
        self._check(self.lib.tm_debug_timing(self.h, 1 if enable else 0, None if enable else C.byref(ms)))
        return None if enable else ms.value

    def stats(self) -> dict:
        s = tm_stats_t()
        self._check(self.lib.tm_stats(self.h, C.byref(s)))
        return {n: getattr(s, n) for n, _ in tm_stats_t._fields_}

    STAT_NAMES = ("node_visits", "edge_probes", "word_probes", "keys", "levels", "spilled_topics",
                  "segments", "chunk_flushes", "frontier_chunks", "node_records", "inline_keys",
                  "cyc_prescan", "cyc_walk", "cyc_copyout", "hot_cyc_prescan", "hot_cyc_walk", "hot_cyc_copyout",
                  "hot_waves")

    IMAGE_ARRAYS = ("word table", "word arena", "word offsets", "edge table", "slot lists", "list arena", "root")

    def image_check(self):
        """tm_debug_image_check: the names of the device arrays a full publish of the current
        host state would change (empty: the delta-published index is byte-identical)."""
        m = C.c_uint32()
        self._check(self.lib.tm_debug_image_check(self.h, C.byref(m)))
        return [n for a, n in enumerate(self.IMAGE_ARRAYS) if m.value >> a & 1]

    def bounds(self):
        """tm_debug_bounds: (hits, first findings) of the bounds-checked debug build over the
        whole process, or None when the loaded library is the product build."""
        return debug_bounds(self)

    COMMIT_MARKS = ("start", "node_image", "edge_table", "staged", "synced", "swap_begin", "swap_end", "standby_kept")

    def commit_marks(self):
        """tm_debug_commit_marks: the last full publish's step times (time.monotonic() seconds,
        None for a step that did not run) and the device buffers it (re)allocated."""
        out = (C.c_uint64 * 9)()
        self._check(self.lib.tm_debug_commit_marks(self.h, out))
        marks = {k: (out[i] / 1e6 if out[i] else None) for i, k in enumerate(self.COMMIT_MARKS)}
        marks["reallocs"] = int(out[8])
        return marks

    def depth_stats(self):
        """Per walk depth (tm_debug_depth_stats): list of dicts {depth, edge_probes, cycles,
        frontier, round_trips} for the depths the walk reached (read before debug_stats)."""
        out = (C.c_uint64 * 64)()
        self._check(self.lib.tm_debug_depth_stats(self.h, out))
        v = list(out)
        return [{"depth": d, "edge_probes": v[d], "cycles": v[16 + d], "frontier": v[32 + d], "round_trips": v[48 + d]}
                for d in range(16) if v[32 + d]]

    def debug_stats(self, enable: bool, read: bool = True):
        out = (C.c_uint64 * 18)()
        self._check(self.lib.tm_debug_stats(self.h, 1 if enable else 0, out if read else None))
        return list(out) if read else None

    # ---- device-resident path (bench)
    def match_device(self, d_bytes: int, d_off: int, n: int, total_bytes: int, stream: int = 0):
        r = tm_dev_result()
        self._check(self.lib.tm_match_device(self.h, C.c_void_p(d_bytes), C.c_void_p(d_off), n, total_bytes,
                                             C.c_void_p(stream) if stream else None, C.byref(r)))
        return r

    def result_ids_device(self, d_ids: int, ids_cap: int, d_off: int, stream: int = 0):
        """Route ids of the last batch, topic-major, into device buffers (d_off: n+1 u32)."""
        self._check(self.lib.tm_result_ids_device(self.h, C.c_void_p(d_ids), ids_cap, C.c_void_p(d_off),
                                                  C.c_void_p(stream) if stream else None))

    def result_ids_device_ex(self, d_ids: int, ids_cap: int, d_off: int, d_flags: int, stream: int = 0):
        """result_ids_device + a device u32 of TM_RES_* overflow flags (no host sync)."""
        self._check(self.lib.tm_result_ids_device_ex(self.h, C.c_void_p(d_ids), ids_cap, C.c_void_p(d_off),
                                                     C.c_void_p(d_flags), C.c_void_p(stream) if stream else None))

    def match_ids_device(self, d_bytes: int, d_off: int, n: int, total_bytes: int, id_bytes: int, d_ids: int,
                         ids_cap: int, d_off_out: int, d_flags: int = 0, stream: int = 0):
        """tm_match_ids_device: the walk writes route ids (id_bytes 4 or 8) and they are compacted
        topic-major into d_ids, offsets (n+1) into d_off_out, TM_RES_* flags into d_flags."""
        self._check(self.lib.tm_match_ids_device(self.h, C.c_void_p(d_bytes), C.c_void_p(d_off), n, total_bytes,
                                                 id_bytes, C.c_void_p(d_ids), ids_cap, C.c_void_p(d_off_out),
                                                 C.c_void_p(d_flags) if d_flags else None,
                                                 C.c_void_p(stream) if stream else None))

    def merge_shard_ids_device(self, G: int, n: int, d_roff: int, roff_stride: int, d_ids: int, id_bytes: int,
                               bases, max_rank_ids: int, d_out_off: int, d_out_ids: int, out_cap: int,
                               stream: int = 0):
        """tm_merge_shard_ids_device: rank r's offsets row at d_roff + r*roff_stride (u32), its ids
        at d_ids + bases[r] elements of id_bytes (at most max_rank_ids of them); merged u64 ids +
        n+1 offsets out."""
        b = (C.c_uint64 * G)(*[int(x) for x in bases])
        self._check(self.lib.tm_merge_shard_ids_device(self.h, G, n, C.c_void_p(d_roff), roff_stride,
                                                       C.c_void_p(d_ids), id_bytes, b, max_rank_ids,
                                                       C.c_void_p(d_out_off), C.c_void_p(d_out_ids), out_cap,
                                                       C.c_void_p(stream) if stream else None))

    def merge_shards_device(self, G: int, n: int, d_counts: int, d_ids: int, stride: int, d_out_off: int,
                            d_out_ids: int, out_cap: int, stream: int = 0):
        self._check(self.lib.tm_merge_shards_device(self.h, G, n, C.c_void_p(d_counts), C.c_void_p(d_ids), stride,
                                                    C.c_void_p(d_out_off), C.c_void_p(d_out_ids), out_cap,
                                                    C.c_void_p(stream) if stream else None))

    def match_device_mode(self, d_bytes: int, d_off: int, n: int, total_bytes: int, mode: int, stream: int = 0):
        r = tm_dev_result()
        self._check(self.lib.tm_match_device_mode(self.h, C.c_void_p(d_bytes), C.c_void_p(d_off), n, total_bytes,
                                                  mode, C.c_void_p(stream) if stream else None, C.byref(r)))
        return r

    def match_device_set(self, dset: int, d_bytes: int, d_off: int, n: int, total_bytes: int,
                         mode: int = TM_MATCH_ALL, stream: int = 0):
        """tm_match_device_set: the batch on direct buffer set `dset` (0, 1 or 2), so several
        batches can be in flight on their own streams."""
        r = tm_dev_result()
        self._check(self.lib.tm_match_device_set(self.h, dset, C.c_void_p(d_bytes), C.c_void_p(d_off), n, total_bytes,
                                                 mode, C.c_void_p(stream) if stream else None, C.byref(r)))
        return r

    def device_sync(self, dset: int = 0):
        self._check(self.lib.tm_device_sync_set(self.h, dset))

    def reserve_matches(self, keys_cap: int, topics: int = 0):
        self._check(self.lib.tm_reserve_matches(self.h, keys_cap, topics))


class Batcher:
    """The publish batching aggregator (include/emqx_tm_batcher.h): single publishes in,
    one engine batch per window, each publisher's own id list back.

    Over an Engine, or over `backend(topics: list[bytes], mode) -> (lists, statuses)` (a
    Python batch matcher; the C-ABI's tm_batcher_create_fn)."""

    def __init__(self, engine: "Engine | None" = None, *, backend=None, max_batch: int = 0, max_wait_us: int = 0,
                 mode: int = TM_MATCH_ALL, delivery_threads: int = 0, transport: int = TM_TRANSPORT_AUTO):
        self.lib = load()
        cfg = tm_batcher_config(max_batch, max_wait_us, mode, delivery_threads, transport)
        h = C.c_void_p()
        self._keep = []
        if engine is not None:
            rc = self.lib.tm_batcher_create(engine.h, C.byref(cfg), C.byref(h))
        else:
            fn = tm_batch_fn(self._py_backend(backend))
            self._keep.append(fn)
            rc = self.lib.tm_batcher_create_fn(fn, None, C.byref(cfg), C.byref(h))
        if rc != TM_OK:
            raise TMError(rc, "tm_batcher_create failed")
        self.h = h
        self.engine = engine
        self.mode = mode

    def _py_backend(self, backend):
        hold = []  # the last two batches' arrays: a view lives until the second-next call

        def run(_be, bytes_p, off_p, n, mode, view):
            try:
                off = np.ctypeslib.as_array(off_p, shape=(n + 1,)).copy()
                raw = C.string_at(bytes_p, int(off[n])) if n and off[n] else b""
                topics = [raw[off[i]:off[i + 1]] for i in range(n)]
                lists, status = backend(topics, mode)
                cnt = np.array([len(x) for x in lists], dtype=np.uint32)
                o = np.zeros(n + 1, dtype=np.uint32)
                np.cumsum(cnt, out=o[1:])
                ids = np.array([i for x in lists for i in x] or [0], dtype=np.uint64)
                st = np.asarray(status, dtype=np.int32)
                hold.append((o, cnt, ids, st))
                del hold[:-2]
                view.contents.off, view.contents.cnt = o.ctypes.data, cnt.ctypes.data
                view.contents.ids = ids.ctypes.data if mode != TM_MATCH_COUNT else None
                view.contents.status = st.ctypes.data
                return TM_OK
            except Exception:  # a failed backend fails its batch, as a device error would
                return TM_EDEVICE
        return run

    def match(self, topic, cap: int = 1 << 16):
        """Blocking: (status, [ids]) for one publish (waits for its window); in COUNT mode
        (status, count)."""
        tb = topic.encode() if isinstance(topic, str) else bytes(topic)
        ids = np.zeros(max(cap, 1), dtype=np.uint64)
        n = C.c_uint32()
        st = C.c_int32()
        rc = self.lib.tm_batcher_match(self.h, tb, len(tb), ids.ctypes.data, cap, C.byref(n), C.byref(st))
        if rc < 0 and st.value >= 0:
            raise TMError(rc, "tm_batcher_match failed")
        if self.mode == TM_MATCH_COUNT and st.value >= 0:
            return st.value, n.value
        return st.value, ids[:min(n.value, cap)].tolist()

    def apply(self, ops):
        ops = list(ops)
        arr = (tm_op * len(ops))()
        keep = []
        for i, o in enumerate(ops):
            fb = o[1].encode() if isinstance(o[1], str) else bytes(o[1])
            cb = C.create_string_buffer(fb, len(fb) + 1)
            keep.append(cb)
            arr[i].op, arr[i].flags = o[0], (o[3] if len(o) > 3 else 0)
            arr[i].filter, arr[i].filter_len, arr[i].id = C.cast(cb, C.c_void_p), len(fb), o[2]
        rc = self.lib.tm_batcher_apply(self.h, arr, len(ops))
        if rc != TM_OK:
            raise TMError(rc, "tm_batcher_apply failed")

    def commit(self) -> int:
        ep = C.c_uint64()
        rc = self.lib.tm_batcher_commit(self.h, C.byref(ep))
        if rc != TM_OK:
            raise TMError(rc, "tm_batcher_commit failed")
        return ep.value

    def stats(self) -> dict:
        st = tm_batcher_stats()
        rc = self.lib.tm_batcher_stats_get(self.h, C.byref(st))
        if rc != TM_OK:
            raise TMError(rc, "tm_batcher_stats_get failed")
        return {k: getattr(st, k) for k, _ in tm_batcher_stats._fields_}

    def reset_stats(self):
        """Start a new latency window (tm_batcher_stats_reset)."""
        rc = self.lib.tm_batcher_stats_reset(self.h)
        if rc != TM_OK:
            raise TMError(rc, "tm_batcher_stats_reset failed")

    def windows(self) -> np.ndarray:
        """Stage stamps of the windows completed since the last reset (tm_batcher_windows), as a
        structured array with tm_batcher_window's fields, oldest first."""
        buf = (tm_batcher_window * TM_BATCHER_WINDOWS)()
        n = C.c_uint32()
        rc = self.lib.tm_batcher_windows(self.h, buf, TM_BATCHER_WINDOWS, C.byref(n))
        if rc != TM_OK:
            raise TMError(rc, "tm_batcher_windows failed")
        dt = np.dtype([(name, np.dtype(ct)) for name, ct in tm_batcher_window._fields_])
        assert dt.itemsize == C.sizeof(tm_batcher_window)
        return np.frombuffer(bytes(buf), dtype=dt, count=n.value).copy()

    def close(self):
        if getattr(self, "h", None):
            self.lib.tm_batcher_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
