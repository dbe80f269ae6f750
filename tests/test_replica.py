"""Replicated mode (DESIGN.md §6 mode 1): one master engine per node, read replicas fed by a
device image and per-epoch patches (include/emqx_tm.h tm_image_* / tm_replica_* / tm_patch_*).

CPU (not gpu): world_size-2 gloo runs of emqx_amd.replica.ReplicatedIndex exercise the real
protocol (image size + image broadcast, per-epoch patch header, patch or image re-send
after a full rebuild).  The engine behind it is a TEST DOUBLE (a key set serialised as the
"image", the epoch's ops as the "patch"); the replicas' match results are checked against
the oracle over the master's keys.

GPU: a master and replicas of it on cuda:0 through the C-ABI: every replica's results are
bit-identical to the master's and to the oracle across delta epochs (patches, including
word-table growth, key-array growth and deletes) and after a full rebuild (image reload).
"""
import json
import os
import socket

import numpy as np
import pytest

import oracle
from emqx_amd import _native as N
from emqx_amd import workloads
from emqx_amd.replica import ReplicatedIndex


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeAdapter:
    """Test double of EngineReplicaAdapter: keys {(filter, id)} as the index."""

    def __init__(self, master: bool):
        self.keys = set()
        self.pending = []
        self.full_next = False
        self.master = master
        self.images, self.patches = 0, 0
        self.ep = 1

    def tensor_device(self):
        import torch
        return torch.device("cpu")

    def commit(self, ops, full=False):
        for op, f, i in ops:
            (self.keys.add if op == "add" else self.keys.discard)((f, i))
        self.pending = ops
        self.full_next = full
        self.ep += 1

    def epoch(self):
        return self.ep

    @staticmethod
    def patch_epoch_from(buf):
        return json.loads(bytes(buf))["from"]

    def export_image(self):
        import torch
        b = json.dumps(sorted(self.keys)).encode()
        return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy())

    def patch(self):
        b = json.dumps({"from": self.ep - 1, "ops": self.pending}).encode()
        return np.frombuffer(b, dtype=np.uint8).copy(), self.full_next

    def load_image(self, t):
        self.keys = {tuple(k) for k in json.loads(bytes(t.numpy()))}
        self.images += 1

    def apply_patch(self, buf):
        for op, f, i in json.loads(bytes(buf))["ops"]:
            (self.keys.add if op == "add" else self.keys.discard)((f, i))
        self.patches += 1

    def match(self, topics):
        ks = sorted(self.keys)
        ix = oracle.OrderedIndex.from_filters([k[0].encode() for k in ks], [k[1] for k in ks])
        buf, off = N.pack_topics(topics)
        o, ids, _ = ix.match(buf, off)
        return [ids[o[t]:o[t + 1]].tolist() for t in range(len(topics))]


def _worker(rank, world, port, q, chunk=0):
    import torch.distributed as dist
    if chunk:
        ReplicatedIndex.CHUNK = chunk  # images and patches cross in many pieces
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = workloads.generate("A", scale=0.1, n_topics=500)
        fl = w.filters()
        ad = FakeAdapter(rank == 0)
        rix = ReplicatedIndex(ad, rank, world)
        if rank == 0:
            ad.commit([("add", f.decode(), int(i)) for f, i in zip(fl, w.f_id)])
        rix.start()
        topics = w.topics()
        out = [ad.match(topics)]
        # epoch 2: a delta (patch); epoch 3: a full rebuild (image again)
        if rank == 0:
            ad.commit([("del", fl[k].decode(), int(w.f_id[k])) for k in range(0, len(fl), 5)]
                      + [("add", "#", 10**6), ("add", "+/+/+/+", 10**6 + 1)])
        rix.sync()
        out.append(ad.match(topics))
        if rank == 0:
            ad.commit([("add", "a/#", 10**6 + 2)], full=True)
        rix.sync()
        out.append(ad.match(topics))
        # two commits between syncs: the second's patch does not apply on the replicas'
        # epoch, so the image goes instead; then a sync with no commit ships nothing
        if rank == 0:
            ad.commit([("add", "b/+", 10**6 + 3)])
            ad.commit([("del", "#", 10**6)])
        kinds = [rix.sync(), rix.sync()]
        out.append(ad.match(topics))
        out.append(kinds)
        q.put((rank, out, ad.images, ad.patches, rix.bytes_sent, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, 0, 0, 0, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("chunk", [0, 64])
def test_replicated_gloo_world2_protocol(chunk):
    """chunk 64: every broadcast larger than 64 bytes goes as 64-byte pieces, the path a
    20 GiB image takes in 1 GiB pieces."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, chunk)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert r[5] is None, r[5]
    (_, m_out, _, _, sent, _), (_, r_out, images, patches, _, _) = res
    assert r_out == m_out  # the replica answers exactly as the master, every epoch
    assert images == 3 and patches == 1  # start + full rebuild + two-commit sync; one delta epoch
    assert r_out[-1] == [ReplicatedIndex.SYNC_IMAGE, ReplicatedIndex.SYNC_NONE]
    assert sent > 0
    assert any(len(x) for x in m_out[1]) and m_out[1] != m_out[0]


# ---------------------------------------------------------------------------- GPU
def _sets(eng, w, mode=N.TM_MATCH_ALL):
    """(statuses, sorted id list per topic) through the device path + device ids (works on
    replicas: no host key table needed)."""
    import torch
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(w.t_bytes).to(dev)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
    n = w.n_topics
    torch.cuda.synchronize()
    r = eng.match_device_mode(d_bytes.data_ptr(), d_off.data_ptr(), n, int(w.t_off[-1]), mode, 0)
    eng.device_sync()
    from emqx_amd.shard import _read_u64
    total = _read_u64(r.d_total)
    if total > r.keys_cap:
        eng.reserve_matches(total + 1024)
        r = eng.match_device_mode(d_bytes.data_ptr(), d_off.data_ptr(), n, int(w.t_off[-1]), mode, 0)
        eng.device_sync()
    lo = torch.empty(n + 1, dtype=torch.int32, device=dev)
    ids = torch.zeros(max(total, 1), dtype=torch.int64, device=dev)
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    # the fills above ran on torch's stream; the engine writes on its own NON-BLOCKING stream
    # (stream 0 = the batch's stream, include/emqx_tm.h tm_match_device), which is not ordered
    # after torch's: the zeros must land before the engine's id writes, not after them
    torch.cuda.synchronize()
    eng.result_ids_device_ex(ids.data_ptr(), max(total, 1), lo.data_ptr(), flags.data_ptr(), 0)
    torch.cuda.synchronize()
    assert int(flags.item()) == 0
    st = np.zeros(n, np.int32)
    import ctypes as C
    lib = C.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert lib.hipMemcpy(st.ctypes.data, C.c_void_p(r.d_status), n * 4, 2) == 0
    o = lo.cpu().numpy().view(np.uint32)
    v = ids.cpu().numpy().view(np.uint64)
    return st, [np.sort(v[o[t]:o[t + 1]]).tolist() for t in range(n)]


def _image_tensor(eng):
    import torch
    n = eng.image_size()
    t = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    eng.image_export(t.data_ptr(), n)
    return t


def _runs_sets(eng, w):
    """(statuses, sorted id list per topic) through the runs form (tm_match_batch_runs): spans
    of the engine's host id arena -- on a replica, the copy it keeps from its device arrays."""
    o, ids, kcnt, st = eng.match_runs(w.t_bytes, w.t_off)
    return st, [sorted(ids[o[t]:o[t + 1]].tolist()) for t in range(w.n_topics)]


def _oracle_sets(f_list, ids, w):
    ix = oracle.OrderedIndex.from_filters(f_list, ids)
    o, e, st = ix.match(w.t_bytes, w.t_off, threads=8)
    return st, [e[o[t]:o[t + 1]].tolist() for t in range(w.n_topics)]


@pytest.mark.gpu
def test_replica_matches_master_across_epochs_gpu():
    w = workloads.generate("E", scale=0.05, n_topics=20000)
    master = N.Engine(0, record_patch=True)
    master.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    master.commit()
    img = _image_tensor(master)
    rep = N.Engine.replica_from_image(0, img.data_ptr(), img.numel())
    del img
    assert rep.stats()["n_keys"] == master.stats()["n_keys"] == w.n_keys
    live_keys = set(zip([bytes(f) for f in w.filters()], [int(i) for i in w.f_id]))
    ms, mids = _sets(master, w)
    rs, rids = _sets(rep, w)
    assert np.array_equal(ms, rs) and mids == rids
    os_, oids = _oracle_sets([k[0] for k in sorted(live_keys)], [k[1] for k in sorted(live_keys)], w)
    assert np.array_equal(ms, os_) and mids == oids
    rng = np.random.default_rng(7)
    keys = sorted(live_keys)
    nxt = 10**7
    patches = 0
    for ep in range(4):
        # deletes, re-adds of existing filters under new ids, brand-new words (word table and
        # key arrays grow), root '#' and '+/...' keys
        dsel = rng.choice(len(keys), size=len(keys) // 50, replace=False)
        dels = [keys[j] for j in dsel]
        adds = [(keys[j][0], nxt + k) for k, j in enumerate(rng.choice(len(keys), size=300))]
        adds += [(b"new%d/w%d/+/#" % (ep, k), nxt + 1000 + k) for k in range(200)]
        adds += [(b"#", nxt + 5000), (b"+/+", nxt + 5001)]
        nxt += 10000
        master.apply([(N.TM_OP_DEL, f, i) for f, i in dels] + [(N.TM_OP_ADD, f, i) for f, i in adds])
        master.commit()
        buf, full = master.patch_export()
        if full:
            img = _image_tensor(master)
            rep.replica_load(img.data_ptr(), img.numel())
            del img
        else:
            assert len(buf) > 1024  # the epoch's scatter/append records, not just a header
            rep.apply_patch(buf)
            patches += 1
        live_keys = (live_keys - set(dels)) | set(adds)
        keys = sorted(live_keys)
        ms, mids = _sets(master, w)
        rs, rids = _sets(rep, w)
        assert np.array_equal(ms, rs) and mids == rids, f"epoch {ep}"
        os_, oids = _oracle_sets([k[0] for k in keys], [k[1] for k in keys], w)
        assert mids == oids, f"epoch {ep}"
        # the runs form on the replica (its host id arena follows image loads and patches)
        rrs, rrids = _runs_sets(rep, w)
        assert np.array_equal(rrs, ms) and [sorted(x) for x in rrids] == [sorted(x) for x in mids], f"epoch {ep}"
        assert rep.stats()["n_keys"] == len(live_keys)
    assert patches >= 2
    # a patch made from another epoch is refused; so are writes on a replica
    with pytest.raises(N.TMError):
        rep.apply_patch(buf)
    with pytest.raises(N.TMError):
        rep.apply([(N.TM_OP_ADD, b"x/y", 1)])
    # FIRST / COUNT / AGGRE on the replica agree with the master
    for mode in (N.TM_MATCH_COUNT, N.TM_MATCH_FIRST, N.TM_MATCH_AGGRE):
        bm = master.match_packed(w.t_bytes, w.t_off, mode)
        br = rep.match_packed(w.t_bytes, w.t_off, mode)
        assert np.array_equal(bm[1], br[1]) and np.array_equal(bm[3], br[3])
        if mode != N.TM_MATCH_COUNT:  # same key handles on both (a list's order is not fixed)
            om, cm, km = bm[0], bm[1], bm[2]
            orr, kr = br[0], br[2]
            for t in range(len(cm)):
                assert np.array_equal(np.sort(km[om[t]:om[t] + cm[t]]), np.sort(kr[orr[t]:orr[t] + cm[t]])), (mode, t)
    # a full rebuild on the master (the edge table grows: node ids move) -> image reload
    grow = [(b"z%d/q%d/+" % (k % 997, k), 2 * 10**7 + k) for k in range(300_000)]
    master.apply([(N.TM_OP_ADD, f, i) for f, i in grow])
    master.commit()
    buf, full = master.patch_export()
    assert full
    with pytest.raises(N.TMError):
        rep.apply_patch(buf)
    img = _image_tensor(master)
    rep.replica_load(img.data_ptr(), img.numel())
    del img
    live_keys |= set(grow)
    ms, mids = _sets(master, w)
    rs, rids = _sets(rep, w)
    assert mids == rids
    assert rep.stats()["n_keys"] == len(live_keys)
    assert [sorted(x) for x in _runs_sets(rep, w)[1]] == [sorted(x) for x in mids]
    # the aggregator on the replica answers in runs form (spans of the replica's id arena)
    b = N.Batcher(rep, max_wait_us=200, transport=N.TM_TRANSPORT_RUNS)
    try:
        for t in range(0, w.n_topics, 97):
            topic = bytes(w.t_bytes[w.t_off[t]:w.t_off[t + 1]])
            st, ids = b.match(topic)
            assert sorted(int(i) for i in ids) == sorted(mids[t]), t
    finally:
        b.close()
    rep.close()
    master.close()


def _gpu_worker(rank, world, port, q):
    """Mode 1 over gloo with REAL engines: rank 0 a master engine, rank 1 a replica built
    from the broadcast image, both on the box's one GPU (the CPU tensors of gloo carry the
    image and the patches)."""
    import torch
    import torch.distributed as dist
    from emqx_amd.replica import EngineReplicaAdapter
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        w = workloads.generate("E", scale=0.02, n_topics=3000)
        fl = w.filters()
        eng = None
        if rank == 0:
            eng = N.Engine(0, record_patch=True)
            eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
            eng.commit()
        ad = EngineReplicaAdapter(0, eng)
        rix = ReplicatedIndex(ad, rank, world)
        rix.start()
        out = [_sets(ad.eng, w)[1]]
        kinds = []
        # epoch 2: a delta epoch (patch); epoch 3: two commits before one sync (image)
        if rank == 0:
            eng.apply([(N.TM_OP_DEL, fl[k], int(w.f_id[k])) for k in range(0, len(fl), 25)]
                      + [(N.TM_OP_ADD, b"#", 10**9), (N.TM_OP_ADD, b"+/+/+/+", 10**9 + 1)])
            eng.commit()
        kinds.append(rix.sync())
        out.append(_sets(ad.eng, w)[1])
        if rank == 0:
            eng.apply([(N.TM_OP_ADD, b"b/+", 10**9 + 2)])
            eng.commit()
            eng.apply([(N.TM_OP_DEL, b"#", 10**9)])
            eng.commit()
        kinds.append(rix.sync())
        kinds.append(rix.sync())
        out.append(_sets(ad.eng, w)[1])
        q.put((rank, out, kinds, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_replicated_gloo_world2_real_engines_gpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert r[3] is None, r[3]
    (_, m_out, m_kinds, _), (_, r_out, r_kinds, _) = res
    assert r_out == m_out  # the replica answers exactly as the master, every epoch
    assert m_kinds == r_kinds == [ReplicatedIndex.SYNC_PATCH, ReplicatedIndex.SYNC_IMAGE, ReplicatedIndex.SYNC_NONE]
    assert m_out[1] != m_out[0] and any(len(x) for x in m_out[1])


def _gpu_worker_d(rank, world, port, q):
    """Config D in mode 1 (100 M filters fit one MI355X, so D is replicated, not
    sharded): rank 0 builds the master over ALL of D's keys (scale 0.002 here: 200 K keys,
    8-level topics), rank 1 gets a replica from the broadcast image; each rank matches ITS half
    of the publishes (the data-parallel split of the bench's step) and returns its sets."""
    import torch
    import torch.distributed as dist
    from emqx_amd.replica import EngineReplicaAdapter
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        w = workloads.generate("D", scale=0.002, n_topics=4000)
        eng = None
        if rank == 0:
            eng = N.Engine(0, record_patch=True)
            eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
            eng.commit()
        ad = EngineReplicaAdapter(0, eng)
        ReplicatedIndex(ad, rank, world).start()
        lo, hi = rank * w.n_topics // world, (rank + 1) * w.n_topics // world
        tb, to = w.topic_slice(lo, hi)
        part = workloads.Workload("D", w.f_bytes, w.f_off, w.f_id, tb, np.ascontiguousarray(to, dtype=np.uint32))
        st, sets = _sets(ad.eng, part)
        q.put((rank, (lo, hi, st.tolist(), sets), None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_replicated_config_d_gloo_world2_vs_oracle_gpu():
    """Config D replicated over two ranks (a master and an image-fed replica on the box's GPU):
    the publishes split between the ranks, every topic's route-id set equal to the oracle's
    over ALL of D's keys (the unsharded index), on both ranks."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gpu_worker_d, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert r[2] is None, r[2]
    w = workloads.generate("D", scale=0.002, n_topics=4000)
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    eo, eids, est = ix.match(w.t_bytes, w.t_off)
    for _, (lo, hi, st, sets), _ in res:
        assert st == est[lo:hi].tolist()
        for k, t in enumerate(range(lo, hi)):
            assert sets[k] == sorted(eids[eo[t]:eo[t + 1]].tolist()), t
    assert sum(len(s) for r in res for s in r[1][3]) > 0
