"""Probe (development): why config B's runs host path is slower from a pinned batch than from
a pageable one when config C's engine is alive in the same process (the bench line's order).
For each source buffer of B's topics -- torch pin_memory (as the bench), a fresh hipHostMalloc,
pageable numpy -- prints the NUMA node of its pages (move_pages), a raw H2D of the bytes, and
tm_match_batch_runs per batch.

    python tools/probe_pinned_numa.py [--skip-c]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import placement, workloads  # noqa: E402

libc = C.CDLL(None, use_errno=True)


def numa_nodes(addr, nbytes, samples=16):
    """NUMA node of `samples` pages spread over [addr, addr + nbytes) (move_pages, query only)."""
    page = 4096
    n = max(1, min(samples, nbytes // page))
    pages = (C.c_void_p * n)(*[((addr + i * (nbytes // n)) // page) * page for i in range(n)])
    status = (C.c_int * n)()
    rc = libc.syscall(279, 0, C.c_ulong(n), pages, None, status, 0)  # SYS_move_pages, x86_64
    if rc != 0:
        return {"error": C.get_errno()}
    out = {}
    for s in status:
        out[int(s)] = out.get(int(s), 0) + 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-c", action="store_true")
    ap.add_argument("--order", default="torch_pin_memory,hipHostMalloc,pageable")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--release-c-lane", action="store_true", help="free this thread's device lane on C's engine first")
    args = ap.parse_args()
    print(json.dumps({"placement": placement.pin_to_gpu(0)}), flush=True)
    keep = None
    if not args.skip_c:
        wc = workloads.generate("C", n_topics=1_000_000)
        keep = N.Engine(0, reserve_keys=wc.n_keys, reserve_nodes=wc.n_keys * 4)
        keep.apply_packed(N.TM_OP_ADD, wc.f_bytes, wc.f_off, wc.f_id)
        keep.commit()
        to = np.ascontiguousarray(wc.t_off, dtype=np.uint32)
        pc = torch.empty(len(wc.t_bytes), dtype=torch.uint8, pin_memory=True)
        pc.numpy()[:] = wc.t_bytes
        for _ in range(3):
            keep.match_runs_view(pc.numpy(), to)
            keep.lib.tm_runs_release(keep.h)
        del pc
        if args.release_c_lane:
            keep.result_release()  # its three streams
    w = workloads.generate("B", n_topics=1_000_000)
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    to32 = np.ascontiguousarray(w.t_off, dtype=np.uint32)
    tb = np.ascontiguousarray(w.t_bytes)
    hip = C.CDLL("libamdhip64.so")
    hp = C.c_void_p()
    assert hip.hipHostMalloc(C.byref(hp), C.c_size_t(len(tb)), 0) == 0
    hbuf = np.ctypeslib.as_array((C.c_uint8 * len(tb)).from_address(hp.value))
    hbuf[:] = tb
    tpin = torch.empty(len(tb), dtype=torch.uint8, pin_memory=True)
    tpin.numpy()[:] = tb
    dev = torch.empty(len(tb), dtype=torch.uint8, device="cuda")
    bufs = {"torch_pin_memory": (tpin.numpy(), tpin), "hipHostMalloc": (hbuf, torch.from_numpy(hbuf)),
            "pageable": (tb, torch.from_numpy(tb))}
    for name in args.order.split(",") * args.rounds:
        arr, t = bufs[name]
        torch.cuda.synchronize()
        h2d = []
        for _ in range(5):
            t0 = time.perf_counter()
            dev.copy_(t, non_blocking=True)
            torch.cuda.synchronize()
            h2d.append(time.perf_counter() - t0)
        eng.match_runs_view(arr, to32)
        eng.lib.tm_runs_release(eng.h)
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            eng.match_runs_view(arr, to32)
            ts.append(time.perf_counter() - t0)
            eng.lib.tm_runs_release(eng.h)
        print(json.dumps({"buffer": name, "bytes": len(tb), "numa_pages": numa_nodes(arr.ctypes.data, len(tb)),
                          "h2d_ms": round(float(np.median(h2d)) * 1e3, 3),
                          "h2d_GBps": round(len(tb) / float(np.median(h2d)) / 1e9, 1),
                          "runs_ms": round(float(np.median(ts)) * 1e3, 3), "runs_ms_each": [round(x * 1e3, 2) for x in ts],
                          "c_alive": keep is not None}), flush=True)
    hip.hipHostFree(hp)
    eng.close()


if __name__ == "__main__":
    main()
