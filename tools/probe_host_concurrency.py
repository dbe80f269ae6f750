"""Probe (development): host-form calls from several threads at once.  One engine (config C at
`--scale`), T threads each making `--reps` tm_match_batch_runs (or tm_match_batch) calls on its
own slice of `--per` topics; prints per thread count the wall time and per-call times.

    python tools/probe_host_concurrency.py [--scale 0.1 --per 131072 --reps 8 --form runs|keys]
"""
import argparse
import json
import os
import sys
import threading
import time

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.1)
    ap.add_argument("--per", type=int, default=131072)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--form", default="runs")
    ap.add_argument("--threads", default="1,2,4")
    ap.add_argument("--pinned", action="store_true", help="topic slices in pinned memory")
    ap.add_argument("--native", action="store_true", help="also from native threads (conc_calls2), first")
    args = ap.parse_args()
    tmax = max(int(x) for x in args.threads.split(","))
    w = workloads.generate("C", scale=args.scale, n_topics=tmax * args.per)
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    to = np.ascontiguousarray(w.t_off, dtype=np.uint32)
    slices = []
    for k in range(tmax):
        lo, hi = k * args.per, (k + 1) * args.per
        b0 = int(to[lo])
        tb = np.ascontiguousarray(w.t_bytes[b0:int(to[hi])])
        if args.pinned:
            pt = torch.empty(len(tb), dtype=torch.uint8, pin_memory=True)
            pt.numpy()[:] = tb
            slices.append((pt, pt.numpy(), np.ascontiguousarray(to[lo:hi + 1] - b0)))
        else:
            slices.append((None, tb, np.ascontiguousarray(to[lo:hi + 1] - b0)))

    def one_call(k):
        _, tb, toff = slices[k]
        if args.form == "runs":
            eng.match_runs_view(tb, toff)
        else:
            eng.match_packed_view(tb, toff)

    def worker(k, times, start, done, rounds):
        for r in range(rounds):
            start.wait()
            for _ in range(args.reps):
                t0 = time.perf_counter()
                one_call(k)
                times[r].append(time.perf_counter() - t0)
            eng.lib.tm_runs_release(eng.h)
            done.wait()
        eng.result_release()  # this thread's lane

    if args.native:  # the same calls from native threads (tools/loadgen.cpp conc_calls2)
        import ctypes as C
        lg = C.CDLL(os.path.join(ROOT, "tools", "libtm_loadgen.so"))
        P = C.POINTER
        lg.conc_calls2.argtypes = [C.c_void_p, C.c_int, P(C.c_void_p), P(C.c_void_p), P(C.c_uint32), C.c_uint32,
                                   C.c_uint32, C.c_uint32, P(C.c_double), P(C.c_uint64), P(C.c_double)]
        bp = (C.c_void_p * tmax)(*[s[1].ctypes.data for s in slices])
        op = (C.c_void_p * tmax)(*[s[2].ctypes.data for s in slices])
        nn = (C.c_uint32 * tmax)(*[args.per] * tmax)
        for T in [int(x) for x in args.threads.split(",")]:
            wall = C.c_double()
            dg = (C.c_uint64 * tmax)()
            cs = (C.c_double * (T * args.reps))()
            rc = lg.conc_calls2(eng.h, 0 if args.form == "runs" else 1, bp, op, nn, T, args.reps, 3, C.byref(wall), dg, cs)
            allt = np.array(list(cs)) * 1e3
            print(json.dumps({"form": args.form, "native": True, "threads": T, "per": args.per, "reps": args.reps,
                              "rc": rc, "pinned": args.pinned, "wall_ms": round(wall.value * 1e3, 2),
                              "calls_per_s": round(T * args.reps / wall.value, 1),
                              "call_ms": [round(x, 3) for x in allt[:args.reps]],
                              "call_ms_p50": round(float(np.median(allt)), 3)}), flush=True)
    for T in [int(x) for x in args.threads.split(",")]:
        rounds = 3  # persistent threads (a NIF's dirty schedulers): the first rounds warm their lanes
        start, done = threading.Barrier(T + 1), threading.Barrier(T + 1)
        times = [[[] for _ in range(rounds)] for _ in range(T)]
        th = [threading.Thread(target=worker, args=(k, times[k], start, done, rounds)) for k in range(T)]
        for x in th:
            x.start()
        for r in range(rounds):
            start.wait()
            t0 = time.perf_counter()
            done.wait()
            wall = time.perf_counter() - t0
        for x in th:
            x.join()
        allt = np.concatenate([np.array(times[k][-1]) for k in range(T)]) * 1e3
        print(json.dumps({"form": args.form, "threads": T, "per": args.per, "reps": args.reps,
                          "pinned": args.pinned, "wall_ms": round(wall * 1e3, 2),
                          "calls_per_s": round(T * args.reps / wall, 1),
                          "call_ms_p50": round(float(np.median(allt)), 3),
                          "call_ms_max": round(float(allt.max()), 3)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
