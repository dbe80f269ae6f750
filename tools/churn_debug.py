"""Churn parity debugging (GPU box): bench.py --churn's epoch loop at small scale, checking
every epoch against the oracle and printing the first differing topics with the filters
of the missing / extra ids."""
import sys

import numpy as np
import torch  # noqa: F401  (torch's HIP runtime first)

sys.path.insert(0, ".")
import oracle  # noqa: E402
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import workloads  # noqa: E402

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 0.1
nt = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
w = workloads.generate("E", scale=scale, n_topics=nt)
eng = N.Engine(0)
eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
eng.commit()
fl = w.filters()
live = {int(i): f for i, f in zip(w.f_id, fl)}
next_id = max(live) + 1
rng = np.random.default_rng(5)


def pack(fs, ids):
    off = np.zeros(len(fs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(f) for f in fs])
    return np.frombuffer(b"".join(fs) + b"\0" * 16, dtype=np.uint8), off, np.asarray(ids, dtype=np.uint64)


def _new_filter(f, n):
    if f == b"#":
        return b"n%d/#" % n
    if f.endswith(b"/#"):
        return f[:-2] + b"/n%d/#" % n
    return f + b"/n%d" % n


for ep in range(12):
    ids_live = np.array(sorted(live), dtype=np.uint64)
    k = max(1, len(ids_live) // 100)
    dsel = rng.choice(len(ids_live), size=k, replace=False)
    del_id = ids_live[dsel]
    del_f = [live[int(i)] for i in del_id]
    src = rng.integers(0, len(fl), size=k)
    add_f = [fl[j] if (i & 1) else _new_filter(fl[j], next_id + i) for i, j in enumerate(src)]
    add_id = list(range(next_id, next_id + k))
    next_id += k
    eng.apply_packed(N.TM_OP_DEL, *pack(del_f, del_id))
    eng.apply_packed(N.TM_OP_ADD, *pack(add_f, add_id))
    eng.commit()
    for i in del_id:
        del live[int(i)]
    for f, i in zip(add_f, add_id):
        live[i] = f
    li = sorted(live)
    ix = oracle.OrderedIndex.from_filters([live[i] for i in li], li)
    eo, eids, _ = ix.match(w.t_bytes, w.t_off)
    off, cnt, keys, _ = eng.match_packed(w.t_bytes, w.t_off)
    ids = eng.key_ids(keys)
    bad = [t for t in range(nt) if not np.array_equal(np.sort(ids[off[t]:off[t] + cnt[t]]), eids[eo[t]:eo[t + 1]])]
    st = eng.stats()
    print(f"epoch {ep}: {len(bad)} bad topics, keys {st['n_keys']} vs {len(live)}, full {st['n_full_rebuilds']}, "
          f"delta {st['n_delta_commits']}", flush=True)
    for t in bad[:4]:
        got = set(ids[off[t]:off[t] + cnt[t]].tolist())
        exp = set(eids[eo[t]:eo[t + 1]].tolist())
        tb = bytes(w.t_bytes[w.t_off[t]:w.t_off[t + 1]])
        print("  topic", tb, "missing", [(i, live.get(i)) for i in sorted(exp - got)][:5],
              "extra", [(i, live.get(i, "DELETED")) for i in sorted(got - exp)][:5],
              "dups", len(ids[off[t]:off[t] + cnt[t]]) - len(got))
    if bad:
        break
