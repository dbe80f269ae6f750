"""Probe (development): config B's runs host path, pinned vs pageable, in the bench's order
(config C's engine and its host-runs leg first, then config B's engine in the same process),
to find why the bench line's config_B pinned row is slower than pageable while a process
holding config B alone is not.  One JSON line per leg.

    python tools/probe_runs_order.py [--skip-c]
"""
import argparse
import json
import os
import sys

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import numpy as np
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import placement, workloads  # noqa: E402


def leg(cfg, keep=None):
    w = workloads.generate(cfg, n_topics=1_000_000)
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    to32 = np.ascontiguousarray(w.t_off, dtype=np.uint32)
    r = bench.host_runs_leg(eng, w.t_bytes, to32, w.n_topics, w, reps=5)
    print(json.dumps({"config": cfg, "pinned_ms": r["pinned"]["ms_per_batch"], "pageable_ms": r["pageable"]["ms_per_batch"],
                      "parity": r["parity"]["mismatches"], "others_alive": keep is not None}), flush=True)
    return eng, w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-c", action="store_true")
    args = ap.parse_args()
    placement.pin_to_gpu(0)
    keep = None
    if not args.skip_c:
        keep = leg("C")
    eng_b, _ = leg("B", keep)
    eng_b.close()
    leg("B", keep)  # a second B engine in the same process


if __name__ == "__main__":
    main()
