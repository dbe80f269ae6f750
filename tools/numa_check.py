"""GPU box: host path (keys and runs) and one aggregator load point, unpinned and then pinned
to the GPU's socket (emqx_amd/placement.py), in two child processes."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys, time, ctypes as C
import numpy as np, torch
sys.path.insert(0, ROOT)
from emqx_amd import placement, _native as N, workloads
info = placement.pin_to_gpu(0) if PIN else {"pinned": False}
w = workloads.generate("C", scale=1.0, n_topics=1_000_000)
eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
eng.commit()
tb = np.ascontiguousarray(w.t_bytes, dtype=np.uint8); to = np.ascontiguousarray(w.t_off, dtype=np.uint32)
res = {"placement": info}
for name, fn in (("keys", eng.match_packed_view), ("runs", eng.match_runs_view)):
    fn(tb, to); ts = []
    for _ in range(6):
        t0 = time.perf_counter(); fn(tb, to); ts.append(time.perf_counter() - t0)
    res[name + "_ms"] = round(float(np.median(ts)) * 1e3, 3)
eng._check(eng.lib.tm_runs_release(eng.h))
lg = C.CDLL(os.path.join(ROOT, "tools", "libtm_loadgen.so"))
lg.loadgen_run2.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_double, C.c_int,
                            C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                            C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
for spans in (1, 0):
    b = N.Batcher(eng, max_batch=65536, max_wait_us=200, delivery_threads=13)
    got, ids, errs, cs, el = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_double()
    lg.loadgen_run2(b.h, tb.ctypes.data, to.ctypes.data, len(to) - 1, 65536, 2.0, spans, C.byref(got), C.byref(ids),
                    C.byref(errs), C.byref(cs), C.byref(el))
    st = b.stats(); b.close()
    res["batcher_65536_" + ("spans" if spans else "idlist")] = {"M_per_s": round(got.value / el.value / 1e6, 2),
        "p50_ms": round(st["lat_p50_us"] / 1e3, 3), "p99_ms": round(st["lat_p99_us"] / 1e3, 3),
        "deliver_busy": round(st["deliver_us"] * 1e-6 / el.value, 3)}
print(json.dumps(res), flush=True)
'''
for pin in (0, 1):
    code = f"ROOT = {ROOT!r}\nPIN = {pin}\n" + CHILD
    r = subprocess.run([sys.executable, "-u", "-c", code], capture_output=True, text=True, timeout=400)
    print(r.stdout.strip() or r.stderr[-2000:], flush=True)
