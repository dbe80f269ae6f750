import sys, os, ctypes as C, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
import numpy as np
import bench
from emqx_amd import _native as N, workloads
w = workloads.generate("C", scale=0.1, n_topics=200000)
eng = N.Engine(0)
eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
eng.commit()
to32 = np.ascontiguousarray(w.t_off, dtype=np.uint32)
lg = bench._loadgen()
for pubs, tr, sp in [(4096, 0, 0), (65536, 0, 0), (65536, 0, 1), (4096, 1, 0)]:
    b = N.Batcher(eng, max_batch=65536, max_wait_us=200, delivery_threads=8, transport=tr)
    got, ids, errs, cs, el = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_double()
    rc = lg.loadgen_run2(b.h, w.t_bytes.ctypes.data, to32.ctypes.data, len(to32) - 1, pubs, 1.0, sp,
                         C.byref(got), C.byref(ids), C.byref(errs), C.byref(cs), C.byref(el))
    st = b.stats(); b.close()
    print(pubs, tr, sp, rc, got.value, errs.value, got.value / el.value, st["lat_p99_us"], flush=True)
