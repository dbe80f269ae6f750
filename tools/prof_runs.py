"""Timeline of tm_match_batch_runs (profiling aid): config C at --scale, 1M-topic batch from
pinned memory, a few calls; run under rocprofv3 --kernel-trace --memory-copy-trace."""
import argparse
import os
import sys
import time

import torch  # noqa: F401  (torch's HIP runtime first)
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import workloads  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=float, default=0.3)
ap.add_argument("--batch", type=int, default=1_000_000)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--sweep", default="", help="comma list of sub:tpw to time in this process")
a = ap.parse_args()
w = workloads.generate("C", scale=a.scale, n_topics=a.batch)
eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
eng.commit()
pin = torch.empty(len(w.t_bytes), dtype=torch.uint8, pin_memory=True)
pin.numpy()[:] = w.t_bytes
to32 = np.ascontiguousarray(w.t_off, dtype=np.uint32)
for cfg in (a.sweep.split(",") if a.sweep else [""]):
    if cfg:
        sub, tpw = cfg.split(":")
        os.environ["EMQX_TM_RUNS_SUB"], os.environ["EMQX_TM_RUNS_TPW"] = sub, tpw
    for _ in range(2):
        eng.match_runs_view(pin.numpy(), to32)
        eng.lib.tm_runs_release(eng.h)
    for buf, name in ((pin.numpy(), "pinned"), (w.t_bytes, "pageable")):
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            r = eng.match_runs_view(buf, to32)
            ts.append(time.perf_counter() - t0)
            eng.lib.tm_runs_release(eng.h)
        print(f"{cfg or 'default'} {name}: runs {np.mean(ts) * 1e3:.3f} ms/batch (p50 {np.median(ts) * 1e3:.3f}), "
              f"topic bytes {int(to32[-1])}, spans {r.total_spans}", flush=True)
