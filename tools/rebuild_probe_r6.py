"""Matches during a forced full rebuild of config C, repeated, with the job's cgroup throttling
counted over each commit (bench.py's rebuild leg, alone).  One JSON line per rebuild.

    [PIN=1] [EMQX_TM_COMMIT_THREADS=K] python tools/rebuild_probe_r5.py 3

Each line carries the publish's step times (tm_debug_commit_marks) and the slowest matches
with the step running when each started and ended."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import workloads  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    if os.environ.get("PIN"):  # as bench.py: the GPU's socket cut to the cgroup quota
        from emqx_amd import placement
        print(json.dumps({"placement": placement.pin_to_gpu(0)}), flush=True)
    n = 1_000_000
    w = workloads.generate("C", n_topics=n)
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(w.t_bytes).to(dev)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
    torch.cuda.synchronize()
    for r in range(reps):
        out = bench.rebuild_leg(eng, w, d_bytes, d_off, n, int(d_off[n].item()), dev)
        out.pop("note", None)
        out["rep"] = r
        out["env_commit_threads"] = os.environ.get("EMQX_TM_COMMIT_THREADS")
        print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
