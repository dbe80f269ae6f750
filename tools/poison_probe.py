"""Uninitialised-read probe (GPU box, development tool): run with EMQX_TM_POISON=1 so every new
device buffer starts as 0xA7 bytes.  Config A at scale 0.2, ids past 32 bits (as
tests/test_shard.py::test_match_ids_device_u64_and_overflow_flags_gpu), then small ids: the key
form, the route-id form of the walk (u64 / u32) and the route ids of a key-form batch, each
against the oracle.  One JSON line per check."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import workloads  # noqa: E402
import oracle  # noqa: E402


def diff(name, off, ids, eoff, eids, **extra):
    bad = []
    for t in range(len(eoff) - 1):
        got = np.sort(np.asarray(ids[int(off[t]):int(off[t + 1])], dtype=np.uint64))
        exp = np.asarray(eids[int(eoff[t]):int(eoff[t + 1])], dtype=np.uint64)
        if not np.array_equal(got, exp):
            bad.append({"t": t, "got": [hex(int(x)) for x in got[:8]], "exp": [hex(int(x)) for x in exp[:8]]})
    print(json.dumps({"check": name, "bad_topics": len(bad), "first": bad[:3], **extra}), flush=True)


def run(shift, device_first=False):
    w = workloads.generate("A", scale=0.2, n_topics=4000)
    ids = w.f_id.astype(np.uint64) + np.uint64(shift)
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, ids)
    eng.commit()
    st = eng.stats()
    print(json.dumps({"shift": shift, "n_full_rebuilds": st["n_full_rebuilds"], "n_delta_commits": st["n_delta_commits"],
                      "image_check": eng.image_check()}), flush=True)
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, ids)
    eoff, eids, _ = ix.match(w.t_bytes, w.t_off)
    total = int(eoff[-1])
    if device_first:  # the device walk is the engine's first launch (as in the shard test)
        ids_dev(eng, w, total, eoff, eids, shift)
    o, c, k, s = eng.match_packed(w.t_bytes, w.t_off)
    kid = eng.key_ids(k)
    off = np.concatenate([[0], np.cumsum(c)]).astype(np.int64)
    flat = np.concatenate([kid[o[t]:o[t] + c[t]] for t in range(len(c))]) if len(c) else kid
    diff("keys_host", off, flat, eoff, eids, shift=shift)
    if not device_first:
        ids_dev(eng, w, total, eoff, eids, shift)
    eng.close()


def ids_dev(eng, w, total, eoff, eids, shift):
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(w.t_bytes).to(dev)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
    n, tb = w.n_topics, int(w.t_off[-1])
    eng.reserve_matches(2 * total + 1024)
    for idb in ((8,) if shift else (4, 8)):
        out = torch.zeros(total + 16, dtype=torch.int64 if idb == 8 else torch.int32, device=dev)
        offd = torch.zeros(n + 1, dtype=torch.int32, device=dev)
        flags = torch.zeros(1, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        eng.match_ids_device(d_bytes.data_ptr(), d_off.data_ptr(), n, tb, idb, out.data_ptr(), total + 16, offd.data_ptr(),
                             flags.data_ptr(), 0)
        eng.device_sync()
        torch.cuda.synchronize()
        v = out.cpu().numpy().view(np.uint64 if idb == 8 else np.uint32)
        diff(f"match_ids_device_{idb}", offd.cpu().numpy().view(np.uint32), v, eoff, eids, flags=int(flags.item()))


if __name__ == "__main__":
    print(json.dumps({"poison": os.environ.get("EMQX_TM_POISON")}), flush=True)
    run(1 << 40, device_first=True)
    run(0, device_first=True)
    run(1 << 40)
