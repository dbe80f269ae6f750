"""Full-size parity (GPU box): the whole config-C batch (1 M publishes vs 10.65 M route
keys) through the C-ABI, compared bit-exactly with the oracle's emqx_trie_search
restatement run over the SAME keys and topics -- every topic, not a sample.

    python tools/parity_full.py [--config C] [--scale 1.0] [--batch 1000000] [--out FILE]

Checks: ALL mode per-topic sorted id sets; COUNT == |ALL| per topic; FIRST == the oracle's
return_first.  The comparison is vectorised: both sides are flattened to (topic, id) and
sorted, so 142 M matched keys compare in seconds.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (torch's HIP runtime first: emqx_amd/_native.py)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import workloads  # noqa: E402


def flat_sorted(off, cnt, ids, n):
    """Engine result -> ids sorted within each topic, topics in order (u64 array)."""
    topic = np.repeat(np.arange(n, dtype=np.uint64), cnt.astype(np.int64))
    starts = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(cnt, out=starts[1:])
    idx = np.repeat(off.astype(np.int64) - starts[:-1], cnt.astype(np.int64)) + np.arange(int(starts[-1]))
    v = ids[idx]
    order = np.lexsort((v, topic))
    return v[order]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    t0 = time.time()
    w = workloads.generate(a.config, scale=a.scale, n_topics=a.batch)
    n = w.n_topics
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    print(f"built {w.n_keys} keys in {time.time() - t0:.1f}s", flush=True)
    off, cnt, keys, st = eng.match_packed(w.t_bytes, w.t_off)
    ids = eng.key_ids(keys)
    print(f"engine: {int(cnt.sum())} matched keys", flush=True)
    t1 = time.time()
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    eo, eids, est = ix.match(w.t_bytes, w.t_off, threads=16)
    print(f"oracle: {int(eo[-1])} matched keys in {time.time() - t1:.1f}s", flush=True)
    res = {"config": a.config, "scale": a.scale, "route_keys": w.n_keys, "topics": n,
           "matched_keys_engine": int(cnt.sum()), "matched_keys_oracle": int(eo[-1])}
    res["status_equal"] = bool(np.array_equal(st, est))
    res["counts_equal"] = bool(np.array_equal(cnt.astype(np.int64), np.diff(eo).astype(np.int64)))
    res["all_sets_equal"] = bool(res["counts_equal"] and np.array_equal(flat_sorted(off, cnt, ids, n), eids))
    _, ccnt, _, _ = eng.match_packed(w.t_bytes, w.t_off, N.TM_MATCH_COUNT)
    res["count_mode_equal"] = bool(np.array_equal(ccnt, cnt))
    fo, fcnt, fkeys, _ = eng.match_packed(w.t_bytes, w.t_off, N.TM_MATCH_FIRST)
    feo, feids, _ = ix.match(w.t_bytes, w.t_off, mode=oracle.MODE_FIRST, threads=16)
    res["first_mode_equal"] = bool(np.array_equal(fcnt.astype(np.int64), np.diff(feo).astype(np.int64))
                                   and np.array_equal(eng.key_ids(fkeys), feids))
    res["oracle"] = "oracle/trie_search.cpp (emqx_trie_search restatement), 16 threads"
    res["ok"] = all(res[k] for k in ("status_equal", "counts_equal", "all_sets_equal", "count_mode_equal",
                                     "first_mode_equal"))
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    sys.exit(0 if res["ok"] else 1)


if __name__ == "__main__":
    main()
