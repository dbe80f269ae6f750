"""Probe (development): why config B's runs host path was slower from pinned memory than from
pageable memory in the round-3/4 bench lines (3.1 vs 1.4 ms per 1 M batch), while config C
showed the opposite.  Times tm_match_batch_runs on the same batch from: torch pinned memory,
hipHostMalloc'd memory, pageable memory, in both orders, with the engine's per-phase view
(H2D on its own stream, walks, D2H).  Prints one JSON line per measurement.

    python tools/probe_runs_pinned.py [--config B] [--reps 10]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (torch's HIP runtime first, as bench.py does)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import placement, workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="B")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--n", type=int, default=1_000_000)
    args = ap.parse_args()
    placement.pin_to_gpu(0)
    w = workloads.generate(args.config, n_topics=args.n)
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    tb = w.t_bytes
    to32 = np.ascontiguousarray(w.t_off, dtype=np.uint32)
    tpin = torch.empty(len(tb), dtype=torch.uint8, pin_memory=True)
    tpin.numpy()[:] = tb
    hip = C.CDLL("libamdhip64.so")
    hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    p = C.c_void_p()
    assert hip.hipHostMalloc(C.byref(p), len(tb) + 64, 0) == 0
    hbuf = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(len(tb),))
    hbuf[:] = tb
    bufs = {"torch_pinned": tpin.numpy(), "hipHostMalloc": hbuf, "pageable": tb}
    orders = [("torch_pinned", "pageable", "hipHostMalloc"), ("pageable", "torch_pinned", "hipHostMalloc"),
              ("hipHostMalloc", "torch_pinned", "pageable")]
    for k, order in enumerate(orders):
        for name in order:
            buf = bufs[name]
            eng.match_runs_view(buf, to32)
            eng.lib.tm_runs_release(eng.h)
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                eng.match_runs_view(buf, to32)
                ts.append(time.perf_counter() - t0)
                eng.lib.tm_runs_release(eng.h)
            print(json.dumps({"round": k, "buffer": name, "config": args.config, "n": args.n,
                              "ms_mean": round(float(np.mean(ts)) * 1e3, 3),
                              "ms_min": round(float(np.min(ts)) * 1e3, 3),
                              "ms_max": round(float(np.max(ts)) * 1e3, 3),
                              "topic_bytes": int(to32[-1])}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
