"""Probe (development, CPU only): the aggregator's own per-publish cost.  A native backend that
matches nothing (tools/loadgen.cpp fake_backend_fn: every publish gets the same K ids) under the
closed-loop publisher load; prints the rate and the delivery threads' time per publish.

    python tools/probe_batcher_cpu.py [--threads 4 --pubs 65536 --ids 142 --spans 0 --secs 2]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--pubs", type=int, default=65536)
    ap.add_argument("--ids", type=int, default=142)
    ap.add_argument("--spans", type=int, default=0)
    ap.add_argument("--secs", type=float, default=2.0)
    ap.add_argument("--wait", type=int, default=200)
    ap.add_argument("--loadgen", default=os.path.join(ROOT, "tools", "libtm_loadgen.so"))
    ap.add_argument("--lib", default=N.LIB_PATH)
    a = ap.parse_args()
    lib = C.CDLL(a.lib)
    lg = C.CDLL(a.loadgen)
    lg.fake_backend_new.restype = C.c_void_p
    lg.fake_backend_new.argtypes = [C.c_uint32]
    fb = lg.fake_backend_new(a.ids)
    fn = C.cast(lg.fake_backend_fn, C.c_void_p)
    cfg = N.tm_batcher_config(65536, a.wait, N.TM_MATCH_ALL, a.threads, 0)
    h = C.c_void_p()
    lib.tm_batcher_create_fn.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(N.tm_batcher_config), C.POINTER(C.c_void_p)]
    assert lib.tm_batcher_create_fn(fn, C.c_void_p(fb), C.byref(cfg), C.byref(h)) == 0
    topics = [f"dev/{i % 977}/sensor/{i}".encode() for i in range(4096)]
    tb = b"".join(topics)
    off = [0]
    for t in topics:
        off.append(off[-1] + len(t))
    tb_c = (C.c_uint8 * len(tb)).from_buffer_copy(tb)
    off_c = (C.c_uint32 * len(off))(*off)
    U = C.POINTER(C.c_uint64)
    lg.loadgen_run3.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_double, C.c_double,
                                C.c_int, U, U, U, U, C.POINTER(C.c_double), C.POINTER(N.tm_batcher_stats)]
    got, ids, errs, cs, el = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_double()
    win = N.tm_batcher_stats()
    rc = lg.loadgen_run3(h, tb_c, off_c, len(topics), a.pubs, 0.5, a.secs, a.spans, C.byref(got), C.byref(ids),
                         C.byref(errs), C.byref(cs), C.byref(el), C.byref(win))
    st = N.tm_batcher_stats()
    lib.tm_batcher_stats_get(h, C.byref(st))
    lib.tm_batcher_destroy(h)
    print(json.dumps({"threads": a.threads, "pubs": a.pubs, "ids": a.ids, "spans": a.spans, "rc": rc,
                      "errors": errs.value, "publishes_per_s": round(got.value / el.value),
                      "mean_batch": round(st.publishes / max(st.batches, 1), 1),
                      "deliver_ns_per_pub": round(st.deliver_us * a.threads * 1e3 / max(st.publishes, 1), 1),
                      "cut_ns_per_pub": round(st.cut_us * 1e3 / max(st.publishes, 1), 1),
                      "busy_deliver": round(st.deliver_us * 1e-6 / el.value, 3)}), flush=True)


if __name__ == "__main__":
    main()
