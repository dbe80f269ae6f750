"""Batcher sweep on one GPU (bench tooling): config C engine, closed-loop publishers through
tm_batcher_submit for each (publishers, delivery threads, max_wait_us[, transport, spans callback,
slots, max_batch, compute streams]) given, one JSON line each.
Usage: python tools/batcher_gpu.py P:T:W[:TR:SP:NSLOT:MB:ST:PFP:PFL:IDW:NICE:RPT] ...   (TR 0 auto/runs, 1 ids; SP 1 = span
callback, 2 = span callback reading no id, 3 = u32-span callback, 4 = u32-span callback reading no id; ST 1 or 2 compute streams, EMQX_TM_STREAMS; PFP/PFL delivery prefetch:
publishes ahead / lines per reply, 0 lines = first line of each span; IDW 4 / 8: runs windows read
the engine's u32 / u64 id arena; NICE: delivery threads' nice value).  PIN=1 pins the process to the GPU's socket first."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np

    from emqx_amd import _native as N
    from emqx_amd import workloads as W
    if os.environ.get("PIN"):  # PIN=1: the GPU's socket cut to the cgroup quota; PIN=socket: the whole socket
        from emqx_amd import placement
        print(json.dumps({"placement": placement.pin_to_gpu(0, quota_cut=os.environ["PIN"] != "socket")}), flush=True)
    t0 = time.time()
    w = W.generate("C", scale=float(os.environ.get("SCALE", "1.0")), n_topics=1_000_000)
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    print(f"engine ready in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    tb = np.ascontiguousarray(w.t_bytes, dtype=np.uint8)
    to32 = np.ascontiguousarray(w.t_off, dtype=np.uint32)
    lg = C.CDLL(os.path.join(ROOT, "tools", "libtm_loadgen.so"))
    U = C.POINTER(C.c_uint64)
    lg.loadgen_run3.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_double, C.c_double,
                                C.c_int, U, U, U, U, C.POINTER(C.c_double), C.POINTER(N.tm_batcher_stats)]
    lg.loadgen_run4.argtypes = lg.loadgen_run3.argtypes + [C.POINTER(N.tm_batcher_window), C.c_uint32,
                                                           C.POINTER(C.c_uint32), U]
    import bench
    if os.environ.get("HOSTPATH"):  # tm_match_batch with host buffers, 1 M publishes per call
        eng.match_packed_view(tb, to32)
        ts = []
        for _ in range(8):
            t1 = time.perf_counter()
            r = eng.match_packed_view(tb, to32)
            ts.append(time.perf_counter() - t1)
        print(json.dumps({"host_path_ms": [round(t * 1e3, 2) for t in ts], "keys": int(r.total),
                          "publishes_per_s": round(len(to32) / 1 / min(ts) if False else (len(to32) - 1) / float(np.median(ts)))}),
              flush=True)
    for spec in sys.argv[1:]:
        v = [int(x) for x in spec.split(":")]
        v = v + [0, 0, 6, 65536, 2, 6, 0][len(v) - 3:]
        pubs, th, wait, tr, sp, nslot, mb, nst = v[:8]
        os.environ["EMQX_TM_NSLOT"] = str(nslot)
        os.environ["EMQX_TM_STREAMS"] = str(nst)
        pfp, pfl = (v[8], v[9]) if len(v) > 9 else (6, 0)  # delivery prefetch knobs
        idw = v[10] if len(v) > 10 else 4  # runs windows: u32 (4) or u64 (8) id arena
        os.environ["EMQX_TM_PF_PUBS"] = str(pfp)
        os.environ["EMQX_TM_PF_LINES"] = str(pfl)
        os.environ["EMQX_TM_RUNS_IDW"] = str(idw)
        nice = v[11] if len(v) > 11 else 0
        os.environ["EMQX_TM_DELIVERY_NICE"] = str(nice)
        rpt = v[12] if len(v) > 12 else 1  # publish ranges per delivery thread and chunk
        os.environ["EMQX_TM_RANGES_PER_THREAD"] = str(rpt)
        b = N.Batcher(eng, max_batch=mb, max_wait_us=wait, delivery_threads=th, transport=tr)
        got, ids, errs, cs, el = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_double()
        win = N.tm_batcher_stats()
        wbuf = (N.tm_batcher_window * N.TM_BATCHER_WINDOWS)()
        wn, cg = C.c_uint32(), (C.c_uint64 * 4)()
        rc = lg.loadgen_run4(b.h, tb.ctypes.data, to32.ctypes.data, len(to32) - 1, pubs, 0.5, 2.0, sp, C.byref(got),
                             C.byref(ids), C.byref(errs), C.byref(cs), C.byref(el), C.byref(win), wbuf,
                             N.TM_BATCHER_WINDOWS, C.byref(wn), cg)
        st = b.stats()
        b.close()
        print(json.dumps({"publishers": pubs, "threads": th, "max_wait_us": wait, "transport": tr, "spans": sp,
                          "nslot": nslot, "max_batch": mb, "streams": nst, "rc": rc, "errors": errs.value,
                          "pf_pubs": pfp, "pf_lines": pfl, "runs_idw": idw, "nice": nice, "ranges_per_thread": rpt,
                          "publishes_per_s": round(win.lat_count / win.window_s),
                          "publishes_per_s_whole_run": round(got.value / el.value),
                          "ids_per_publish": round(ids.value / max(got.value, 1), 1),
                          "mean_batch": round(st["publishes"] / max(st["batches"], 1), 1),
                          "mean_ms": round(win.lat_mean_us / 1e3, 3),
                          "p50_ms": round(win.lat_p50_us / 1e3, 3), "p99_ms": round(win.lat_p99_us / 1e3, 3),
                          "p999_ms": round(win.lat_p999_us / 1e3, 3), "max_ms": round(win.lat_max_us / 1e3, 3),
                          "throttled_ms": round(cg[3] / 1e3, 3), "usage_cpus": round(cg[0] * 1e-6 / win.window_s, 2),
                          "windows": bench.window_stages(wbuf, wn.value),
                          "busy": {k: round(st[k + "_us"] * 1e-6 / el.value, 3)
                                   for k in ("cut", "enqueue", "gpu_wait", "copy", "deliver")}}), flush=True)


if __name__ == "__main__":
    main()
