"""Two device batches in flight (tm_match_device_set, ABI 8): batches alternate between the
two direct buffer sets on two streams, several rounds without a host sync in between, and
every batch's device result equals the host path's (tm_match_batch, itself checked against
the oracle elsewhere).  A set's result stays valid while the other set runs."""
import numpy as np
import pytest

from emqx_amd import _native as N
from emqx_amd import workloads

pytestmark = pytest.mark.gpu


def _d2h_u32(ptr, n):
    import ctypes as C

    import torch
    t = torch.empty(max(n, 1), dtype=torch.int32, device="cuda:0")
    lib = C.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    if n:
        assert lib.hipMemcpy(C.c_void_p(t.data_ptr()), C.c_void_p(ptr), 4 * n, 3) == 0
    return t[:n].cpu().numpy().view(np.uint32)


def _check(eng, r, n, off, cnt, hk):
    from emqx_amd.shard import _read_u64
    total = _read_u64(r.d_total)
    assert total <= r.keys_cap
    d_cnt = _d2h_u32(r.d_cnt, n)
    d_off = _d2h_u32(r.d_off, n)
    d_keys = _d2h_u32(r.d_keys, total)
    assert np.array_equal(d_cnt, cnt)
    for t in range(n):
        assert np.array_equal(np.sort(d_keys[d_off[t]:d_off[t] + d_cnt[t]]), np.sort(hk[off[t]:off[t] + cnt[t]])), t


def test_two_direct_sets_in_flight():
    import torch
    w = workloads.generate("C", scale=0.02, n_topics=30000)
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    dev = torch.device("cuda", 0)
    halves = []
    for lo, hi in ((0, 14000), (14000, 30000)):
        tb = w.t_bytes[w.t_off[lo]:w.t_off[hi]]
        to = (w.t_off[lo:hi + 1] - w.t_off[lo]).astype(np.uint32)
        off, cnt, hk, _ = eng.match_packed(tb, to)
        halves.append((torch.from_numpy(np.ascontiguousarray(tb)).to(dev),
                       torch.from_numpy(to.view(np.int32)).to(dev), hi - lo, int(to[-1]), off, cnt, hk))
    eng.reserve_matches(int(max(h[5].sum() for h in halves)) + 1024)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    torch.cuda.synchronize()
    for _ in range(3):  # A on set 0 / stream 0, B on set 1 / stream 1, queued back to back
        rs = []
        for k, (db, do, n, nb, *_x) in enumerate(halves):
            rs.append(eng.match_device_set(k, db.data_ptr(), do.data_ptr(), n, nb, N.TM_MATCH_ALL,
                                           streams[k].cuda_stream))
        eng.device_sync(0)
        eng.device_sync(1)
        for r, (_, _, n, _, off, cnt, hk) in zip(rs, halves):
            _check(eng, r, n, off, cnt, hk)
    # set 0's result survives a batch on set 1
    r0 = eng.match_device_set(0, halves[0][0].data_ptr(), halves[0][1].data_ptr(), halves[0][2], halves[0][3])
    eng.device_sync(0)
    eng.match_device_set(1, halves[1][0].data_ptr(), halves[1][1].data_ptr(), halves[1][2], halves[1][3])
    eng.device_sync(1)
    _check(eng, r0, *[halves[0][i] for i in (2, 4, 5, 6)])
    # a third set (round 4): its own result, set 0's still intact
    r2 = eng.match_device_set(2, halves[1][0].data_ptr(), halves[1][1].data_ptr(), halves[1][2], halves[1][3])
    eng.device_sync(2)
    _check(eng, r2, *[halves[1][i] for i in (2, 4, 5, 6)])
    _check(eng, r0, *[halves[0][i] for i in (2, 4, 5, 6)])
    with pytest.raises(N.TMError):
        eng.match_device_set(3, halves[0][0].data_ptr(), halves[0][1].data_ptr(), halves[0][2], halves[0][3])
    eng.close()


def test_two_direct_sets_on_a_replica():
    """The same on a read replica made from the master's device image (mode 1's ranks > 0
    run the bench's two-in-flight loop on replicas)."""
    import torch
    w = workloads.generate("E", scale=0.02, n_topics=12000)
    master = N.Engine(0, record_patch=True)
    master.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    master.commit()
    size = master.image_size()
    img = torch.empty(size, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    master.image_export(img.data_ptr(), size)
    rep = N.Engine.replica_from_image(0, img.data_ptr(), img.numel())
    del img
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(w.t_bytes).to(dev)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
    n, nb = w.n_topics, int(w.t_off[-1])
    off, cnt, hk, _ = master.match_packed(w.t_bytes, w.t_off)
    master_ids = [np.sort(master.key_ids(hk[off[t]:off[t] + cnt[t]])) for t in range(n)]
    rep.reserve_matches(int(cnt.sum()) + 1024)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    torch.cuda.synchronize()
    rs = [rep.match_device_set(k, d_bytes.data_ptr(), d_off.data_ptr(), n, nb, N.TM_MATCH_ALL, streams[k].cuda_stream)
          for k in range(2)]
    rep.device_sync(0)
    rep.device_sync(1)
    assert rs[0].d_keys != rs[1].d_keys  # each set has its own output
    for r in rs:
        assert np.array_equal(_d2h_u32(r.d_cnt, n), cnt)
    # route ids of set 0's batch (result_ids_device reads tm_match_device's set) equal the master's
    ids_t = torch.zeros(int(cnt.sum()) + 1, dtype=torch.int64, device=dev)
    ioff_t = torch.empty(n + 1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()  # the zero-fill (torch's stream) lands before the engine's writes (its own stream)
    rep.result_ids_device(ids_t.data_ptr(), ids_t.numel(), ioff_t.data_ptr())
    torch.cuda.synchronize()
    io = ioff_t.cpu().numpy().view(np.uint32)
    v = ids_t.cpu().numpy().view(np.uint64)
    for t in range(n):
        assert np.array_equal(np.sort(v[io[t]:io[t + 1]]), master_ids[t]), t
    rep.close()
    master.close()
