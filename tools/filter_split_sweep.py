"""matches_filter/3 runs form (tm_match_filter_batch_runs) under EMQX_TM_FILTER_SPLIT settings,
one engine (config C), one process: per setting and query set, the C-ABI call's wall time
(median of 7) and whether every query's ids equal the unsplit walk's.  Under
`rocprofv3 --kernel-trace` the k_filter_walk launches come in the printed order (1 warm-up, 7 timed
and 1 for the parity read per line).  Usage: python tools/filter_split_sweep.py [SETTING ...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from emqx_amd import _native as N
    from emqx_amd import workloads
    settings = sys.argv[1:] or ["0", "16384:4096", "4096:1024", "1024:256", "256:64"]
    w = workloads.generate("C", scale=float(os.environ.get("SCALE", "1.0")), n_topics=1000)
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    sets = {"plus": bench.filter_queries(w, 9000, kinds=[1]), "mixed": bench.filter_queries(w, 100000)}
    if os.environ.get("QUERIES"):  # e.g. QUERIES=plus
        sets = {k: v for k, v in sets.items() if k in os.environ["QUERIES"].split(",")}
    ref = {}
    for name, (qb, qo) in sets.items():
        qo = np.ascontiguousarray(qo, dtype=np.uint32)
        for st in settings:
            os.environ["EMQX_TM_FILTER_SPLIT"] = st
            eng.match_filter_runs_view(qb, qo)
            ts = []
            for _ in range(7):
                t0 = time.perf_counter()
                eng.match_filter_runs_view(qb, qo)
                ts.append(time.perf_counter() - t0)
            ro, rids, kc, rst = eng.match_filter_runs(qb, qo)
            if name not in ref:
                ref[name] = (ro, rids, kc, rst)
            r0 = ref[name]
            same = bool(np.array_equal(ro, r0[0]) and np.array_equal(rids, r0[1]) and np.array_equal(kc, r0[2])
                        and np.array_equal(rst, r0[3]))
            print(json.dumps({"queries": name, "n": len(qo) - 1, "split": st, "ms_median": round(float(np.median(ts)) * 1e3, 3),
                              "ms_min": round(min(ts) * 1e3, 3), "ids": int(len(rids)), "same_as_first_setting": same}),
                  flush=True)


if __name__ == "__main__":
    main()
