"""Debug (GPU box): tm_match_ids_device at small batch sizes vs the oracle, then the
aggregator's ids transport (the failing test), with HIP errors reported."""
import sys
import os
import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import workloads  # noqa: E402

w = workloads.generate("A", scale=0.3, n_topics=3000)
eng = N.Engine(0)
eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
eng.commit()
ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
dev = torch.device("cuda", 0)
for n in (24, 100, 512, 2000, 3000):
    tb, to = w.topic_slice(0, n)
    eo, eids, est = ix.match(tb, to)
    d_b = torch.from_numpy(tb).to(dev)
    d_o = torch.from_numpy(to.view(np.int32)).to(dev)
    off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    ids = torch.zeros(int(eo[-1]) + 64, dtype=torch.int32, device=dev)
    fl = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    eng.match_ids_device(d_b.data_ptr(), d_o.data_ptr(), n, int(to[-1]), 4, ids.data_ptr(), ids.numel(), off.data_ptr(),
                         fl.data_ptr(), 0)
    torch.cuda.synchronize()
    o = off.cpu().numpy().view(np.uint32)
    v = ids.cpu().numpy().view(np.uint32)
    bad = [t for t in range(n) if sorted(v[o[t]:o[t + 1]].tolist()) != eids[eo[t]:eo[t + 1]].tolist()]
    print(f"n={n}: flags {int(fl.item())}, total {o[-1]} vs {eo[-1]}, bad {len(bad)} {bad[:5]}", flush=True)
b = N.Batcher(eng, max_batch=512, max_wait_us=500, mode=N.TM_MATCH_ALL, transport=N.TM_TRANSPORT_IDS)
topics = w.topics()
bad = 0
for i in range(200):
    st, got = b.match(topics[i])
    if st != 0 and st != 1:
        print("status", i, st, flush=True)
        bad += 1
        if bad > 3:
            break
print("batcher sequential done", bad, flush=True)
b.close()
eng.close()
