"""Development: the bench's aggregator legs alone (config C at SCALE, default 0.1) under
faulthandler, to localise a crash: batcher_load's rows, then the replica leg."""
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
faulthandler.enable()


def main():
    import numpy as np
    import torch  # noqa: F401  (the bench loads torch's HIP runtime first)
    import bench
    from emqx_amd import _native as N
    from emqx_amd import workloads
    w = workloads.generate("C", scale=float(os.environ.get("SCALE", "0.1")), n_topics=200_000)
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    tb, to = w.topic_slice(0, 200_000)
    to32 = np.ascontiguousarray(to, dtype=np.uint32)
    for leg in os.environ.get("LEGS", "load,replica").split(","):
        t0 = time.time()
        print(f"leg {leg} ...", file=sys.stderr, flush=True)
        if leg == "load":
            r = bench.batcher_load(eng, tb, to32, 0.5)
        else:
            r = bench.replica_batcher_leg(eng, tb, to32, 0.5)
        print(f"leg {leg} ok in {time.time() - t0:.1f}s: "
              f"{[round(x['publishes_per_s'] / 1e6, 1) for x in r['runs']]}", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
