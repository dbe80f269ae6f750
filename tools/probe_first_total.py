"""Probe (development): the first tm_match_device batch of a freshly built engine against the
same batch run again (after tm_device_sync sized the chunk pools): the totals must agree, and so
must the per-topic counts.  Run for configs E and C, alone and after another engine was used."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import workloads  # noqa: E402


def u64(ptr):
    """One u64 from device memory (the batch's requested-keys counter is a device address)."""
    import ctypes as C
    h = (C.c_uint64 * 1)()
    lib = C.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert lib.hipMemcpy(C.cast(h, C.c_void_p), C.c_void_p(ptr), 8, 2) == 0  # hipMemcpyDeviceToHost
    return h[0]


def run(cfg, scale):
    w = workloads.generate(cfg, scale=scale, n_topics=1_000_000)
    eng = N.Engine(0, reserve_keys=w.n_keys * 2, reserve_nodes=w.n_keys * 8)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(w.t_bytes).to(dev)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
    s = torch.cuda.Stream(dev)
    tots = []
    for i in range(4):
        r = eng.match_device(d_bytes.data_ptr(), d_off.data_ptr(), w.n_topics, int(w.t_off[-1]), s.cuda_stream)
        eng.device_sync()
        torch.cuda.synchronize()
        tots.append((int(u64(r.d_total)), int(r.keys_cap), int(eng.stats()["n_slow_topics"])))
        if i == 0 and tots[0][0] > tots[0][1]:
            eng.reserve_matches(int(tots[0][0] * 1.25) + 1024)
    print(json.dumps({"config": cfg, "scale": scale, "totals_caps_slow": tots}), flush=True)
    eng.close()


if __name__ == "__main__":
    for cfg, sc in (("E", 1.0), ("B", 1.0), ("E", 1.0)):
        run(cfg, sc)
