"""tm_match_batch (host buffers in, keys out) at config C, timed per call (bench tooling):
run under rocprofv3 --memory-copy-trace to see where the host path's time goes."""
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (torch's HIP runtime first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import workloads  # noqa: E402

w = workloads.generate("C", scale=float(os.environ.get("SCALE", "1.0")), n_topics=1_000_000)
eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
eng.commit()
tb = np.ascontiguousarray(w.t_bytes, dtype=np.uint8)
to = np.ascontiguousarray(w.t_off, dtype=np.uint32)
for k in range(6):
    t0 = time.perf_counter()
    r = eng.match_packed_view(tb, to)
    print(f"call {k}: {(time.perf_counter() - t0) * 1e3:.2f} ms, {r.total} keys", flush=True)
