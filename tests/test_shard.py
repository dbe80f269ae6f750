"""Filter-sharded mode (SURVEY.md §8(e) mode 2).

CPU (not gpu): world_size-2 gloo runs of emqx_amd.shard.ShardedIndex exercise the real
placement, every exchange variant (padded all-gather; exact all-gather-v by grouped
send/recv; local, no collective) and the host form of the merge.  The per-shard matcher
there is a TEST DOUBLE: the oracle's restated index over the rank's keys (there is no GPU
on this host).  The merged result (or, for local, the union of the ranks' lists) is
checked bit-exactly against the oracle over ALL keys.

GPU: G shard engines on cuda:0 in one process, the walk writing route ids compacted
topic-major (tm_match_ids_device) + the device merge (tm_merge_shard_ids_device); the
all-gather is replaced by stacking the shards' buffers (what RCCL's all-gather produces,
padded or exact), since one box has one GPU.
"""
import os
import socket

import numpy as np
import pytest

import oracle
from emqx_amd import _native as N
from emqx_amd import shard as S
from emqx_amd import workloads


class OracleShard:
    """Test double for EngineShard: the restated index over this rank's keys."""

    def __init__(self):
        self.keys = {}  # (filter bytes, id) -> flags
        self.ix = None

    def apply_packed(self, op, buf, off, ids, flags=None):
        b = bytes(np.asarray(buf, dtype=np.uint8))
        for i in range(len(ids)):
            k = (b[int(off[i]):int(off[i + 1])], int(ids[i]))
            if op == N.TM_OP_ADD:
                self.keys[k] = 0 if flags is None else int(flags[i])
            else:
                self.keys.pop(k, None)

    def commit(self):
        ks = sorted(self.keys)
        self.ix = oracle.OrderedIndex.from_filters([k[0] for k in ks], [k[1] for k in ks],
                                                   [self.keys[k] for k in ks])

    def match_ids(self, t_bytes, t_off):
        off, ids, st = self.ix.match(t_bytes, t_off)
        return off.astype(np.uint32), ids, st


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = workloads.generate("A", scale=0.5, n_topics=3000)
        six = S.ShardedIndex(OracleShard(), rank, world)
        six.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
        six.commit()
        res = {}
        for ex in S.EXCHANGES:
            off, ids, st = six.match(w.t_bytes, w.t_off, exchange=ex)
            res[ex] = (off.tolist(), ids.tolist(), st.tolist(), six.wire_bytes)
        # epoch 2: delete every 7th key, add a root '#' and a '+/...' key (placement by id)
        dm = np.arange(w.n_keys) % 7 == 0
        b, o, i, _ = S.select_keys(w.f_bytes, w.f_off, w.f_id, dm)
        six.apply_packed(N.TM_OP_DEL, b, o, i)
        xb, xo = N.pack_topics([b"#", b"+/+/+/+"])
        six.apply_packed(N.TM_OP_ADD, xb, xo.astype(np.uint64), np.array([10**9, 10**9 + 1], np.uint64))
        six.commit()
        for ex in ("padded", "exact"):
            off2, ids2, _ = six.match(w.t_bytes, w.t_off, exchange=ex)
            res[ex + "2"] = (off2.tolist(), ids2.tolist())
        q.put((rank, res, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _reference(w):
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    off, ids, st = ix.match(w.t_bytes, w.t_off)
    dm = np.arange(w.n_keys) % 7 != 0
    b, o, i, _ = S.select_keys(w.f_bytes, w.f_off, w.f_id, dm)
    fl = [bytes(b[int(o[k]):int(o[k + 1])]) for k in range(len(i))] + [b"#", b"+/+/+/+"]
    ix2 = oracle.OrderedIndex.from_filters(fl, list(i) + [10**9, 10**9 + 1])
    off2, ids2, _ = ix2.match(w.t_bytes, w.t_off)
    return off, ids, st, off2, ids2


def _same_sets(off, ids, eoff, eids):
    off, ids, eoff, eids = map(np.asarray, (off, ids, eoff, eids))
    assert len(off) == len(eoff)
    assert np.array_equal(np.diff(off.astype(np.int64)), np.diff(eoff.astype(np.int64)))
    for t in range(len(off) - 1):
        got = np.sort(ids[off[t]:off[t + 1]].astype(np.uint64))
        assert np.array_equal(got, eids[eoff[t]:eoff[t + 1]]), t


def test_shard_placement_matches_generator():
    full = workloads.generate("A", scale=0.3, n_topics=10)
    for r in range(3):
        part = workloads.generate("A", scale=0.3, n_topics=10, shard_count=3, shard_index=r)
        assert np.array_equal(part.f_id, full.f_id[S.shard_of(full.f_id, 3) == r])


def test_select_keys_roundtrip():
    w = workloads.generate("A", scale=0.1, n_topics=10)
    mask = np.arange(w.n_keys) % 3 == 1
    b, o, i, _ = S.select_keys(w.f_bytes, w.f_off, w.f_id, mask)
    fl = w.filters()
    got = [bytes(b[int(o[k]):int(o[k + 1])]) for k in range(len(i))]
    assert got == [fl[k] for k in np.nonzero(mask)[0]]
    assert np.array_equal(i, w.f_id[mask])


def test_host_merge_concatenates_per_topic():
    rng = np.random.default_rng(5)
    G, n = 3, 50
    counts = rng.integers(0, 6, size=(G, n)).astype(np.uint32)
    stride = int(counts.sum(1).max()) + 3
    ids = np.zeros((G, stride), np.uint64)
    per = [[None] * n for _ in range(G)]
    for r in range(G):
        pos = 0
        for t in range(n):
            v = rng.integers(0, 2**63, size=counts[r, t], dtype=np.uint64)
            ids[r, pos:pos + len(v)] = v
            per[r][t] = v
            pos += len(v)
    off, merged = N.merge_shards(counts, ids)
    for t in range(n):
        exp = np.concatenate([per[r][t] for r in range(G)])
        assert np.array_equal(merged[off[t]:off[t + 1]], exp)
    assert off[-1] == counts.sum()
    # the same through the header form the device merge takes (offset rows + flags), padded
    # (bases r * stride) and exact (bases = the running totals of a concatenation)
    H = np.zeros((G, n + 2), np.uint32)
    H[:, 1:n + 1] = np.cumsum(counts, axis=1)
    for bases, flat in (([r * stride for r in range(G)], ids.reshape(-1)),
                        (np.concatenate([[0], np.cumsum(counts.sum(1))[:-1]]).tolist(),
                         np.concatenate([ids[r, :counts[r].sum()] for r in range(G)]))):
        off2, merged2 = S.merge_shard_ids_host(H, flat, bases, n)
        assert np.array_equal(off2, off) and np.array_equal(merged2, merged)
    # u32 ids (what crosses the wire while every id fits 32 bits) widen to the same u64
    small = (ids & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    off3, merged3 = S.merge_shard_ids_host(H, small.reshape(-1), [r * stride for r in range(G)], n)
    assert np.array_equal(merged3, merged & np.uint64(0xFFFFFFFF))


def test_sharded_gloo_world2_matches_unsharded_oracle():
    """Every exchange variant over gloo, world 2: padded and exact merge to the unsharded
    oracle's sets on every rank (two epochs); local leaves each rank its own lists, whose
    union is the oracle's; a2a leaves each rank the merged sets of its topic range; the exact
    variant moves no more than the ids themselves, a2a only the other rank's ids of its range."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert r[2] is None, r[2]
    w = workloads.generate("A", scale=0.5, n_topics=3000)
    eoff, eids, est, eoff2, eids2 = _reference(w)
    n = w.n_topics
    for rank, rr, _ in res:
        for ex in ("padded", "exact"):
            off, ids, st, _ = rr[ex]
            _same_sets(off, ids, eoff, eids)
            assert np.array_equal(np.asarray(st), est)
            _same_sets(*rr[ex + "2"], eoff2, eids2)
    # local: the union of the two ranks' lists per topic is the full result
    lo = [np.asarray(rr["local"][0], np.int64) for _, rr, _ in res]
    li = [np.asarray(rr["local"][1], np.uint64) for _, rr, _ in res]
    for t in range(n):
        got = np.sort(np.concatenate([li[r][lo[r][t]:lo[r][t + 1]] for r in range(2)]))
        assert np.array_equal(got, eids[eoff[t]:eoff[t + 1]]), t
    assert res[0][1]["local"][3] == 0
    # a2a: each rank holds the merged results of its topic range; together, every topic
    for rank, rr, _ in res:
        off, ids, st, wire = rr["a2a"]
        lo, hi = rank * n // 2, (rank + 1) * n // 2
        assert len(off) == hi - lo + 1 and np.array_equal(np.asarray(st), est[lo:hi])
        _same_sets(off, ids, eoff[lo:hi + 1] - eoff[lo], eids[eoff[lo]:eoff[hi]])
        # it received only the other rank's ids for its own topics (+ offsets)
        other = 1 - rank
        lo_o = np.asarray(res[other][1]["local"][0], np.int64)
        assert wire == (lo_o[hi] - lo_o[lo]) * 8 + ((hi - lo + 1) * 4 + 4 * 4)
    # exact: each rank received the other's ids at exact size (+ its header)
    for rank, rr, _ in res:
        other = 1 - rank
        other_total = int(np.asarray(res[other][1]["local"][0])[-1])
        assert rr["exact"][3] == other_total * 8 + (n + 2) * 4
        assert rr["padded"][3] >= rr["exact"][3]


def _shard_engines_merged(parts, w_topics, exact=False):
    """GPU: one engine per shard workload in `parts` on cuda:0, each through the real
    per-rank step (ShardedIndex.local_device: the walk writing route ids compacted
    topic-major, no host sync), the all-gather replaced by stacking the shards' buffers (what
    RCCL's all-gather produces: padded to the stride, or exact sizes back to back), then the
    real device merge (ShardedIndex.merge_device).  Returns host (off, ids, flags, H, Ids,
    bases, id_bytes)."""
    import torch
    G = len(parts)
    n = w_topics.n_topics
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(w_topics.t_bytes).to(dev)
    d_off = torch.from_numpy(w_topics.t_off.view(np.int32)).to(dev)
    tb = int(w_topics.t_off[-1])
    engs, sixs = [], []
    for r, part in enumerate(parts):
        eng = N.Engine(0)
        eng.apply_packed(N.TM_OP_ADD, part.f_bytes, part.f_off, part.f_id)
        eng.commit()
        six = S.ShardedIndex(S.EngineShard(eng), r, G)
        engs.append(eng)
        sixs.append(six)
    torch.cuda.synchronize()
    # per-shard sizing run (the all-reduce(max) of prepare_device is taken here by hand:
    # one process stands in for G ranks, no process group)
    sizers = [S.ShardedIndex(S.EngineShard(e), 0, 1) for e in engs]
    for z, e in zip(sizers, engs):
        z.prepare_device(e, d_bytes.data_ptr(), d_off.data_ptr(), n, tb)
    stride = max(z.stride for z in sizers)
    idb = max(z.id_bytes for z in sizers)
    hs, ids = [], []
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        for six, e in zip(sixs, engs):
            six.stride, six.id_bytes = stride, idb  # what prepare_device's all-reduce(max) gives every rank
            h, i = six.local_device(e, d_bytes.data_ptr(), d_off.data_ptr(), n, tb, s.cuda_stream)
            hs.append(h)
            ids.append(i)
        H = torch.stack(hs).contiguous()
        if exact:
            s.synchronize()
            tot = [int(h[n].item()) for h in hs]
            bases = [int(x) for x in np.concatenate([[0], np.cumsum(tot)[:-1]])]
            Ids = torch.cat([i[:t] for i, t in zip(ids, tot)] + [ids[0][:1]])
        else:
            bases = [r * stride for r in range(G)]
            Ids = torch.cat(ids)
        off, out, flags = sixs[0].merge_device(engs[0], H, Ids, bases, n, s.cuda_stream)
    torch.cuda.synchronize()
    o = off.cpu().numpy().view(np.uint32)
    res = (o, out[:int(o[-1])].cpu().numpy().view(np.uint64), int(flags.item()), H.cpu().numpy(),
           Ids.cpu().numpy().view(np.uint32 if idb == 4 else np.uint64), bases, idb)
    for e in engs:
        e.close()
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("G,exact", [(1, False), (2, False), (3, False), (3, True)])
def test_sharded_device_merge_gpu(G, exact):
    w = workloads.generate("B", scale=0.05, n_topics=20000)
    parts = []
    for r in range(G):
        mask = S.shard_of(w.f_id, G) == r
        b, o, i, _ = S.select_keys(w.f_bytes, w.f_off, w.f_id, mask)
        parts.append(workloads.Workload("B", b, o, i, w.t_bytes, w.t_off))
    off, ids, flags, H, Ids, bases, idb = _shard_engines_merged(parts, w, exact=exact)
    assert flags == 0
    assert idb == 4  # config B's ids fit 32 bits: u32 on the wire
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    eoff, eids, _ = ix.match(w.t_bytes, w.t_off)
    _same_sets(off, ids, eoff, eids)
    # the host form of the merge over the same buffers agrees with the device merge
    hoff, hids = S.merge_shard_ids_host(H, Ids, bases, w.n_topics)
    assert np.array_equal(hoff, off) and np.array_equal(hids, ids)


@pytest.mark.gpu
def test_match_ids_device_u64_and_overflow_flags_gpu():
    """tm_match_ids_device with ids past 32 bits: u32 is refused (TM_ESTATE), u64 ids equal
    the oracle's; a short id buffer raises TM_RES_IDS_OVERFLOW on the device."""
    import torch
    w = workloads.generate("A", scale=0.2, n_topics=4000)
    big = w.f_id.astype(np.uint64) + np.uint64(1 << 40)
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, big)
    eng.commit()
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(w.t_bytes).to(dev)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
    n, tb = w.n_topics, int(w.t_off[-1])
    off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    with pytest.raises(N.TMError) as e:
        eng.match_ids_device(d_bytes.data_ptr(), d_off.data_ptr(), n, tb, 4, 0, 0, off.data_ptr(), 0, 0)
    assert e.value.rc == N.TM_ESTATE
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, big)
    eoff, eids, _ = ix.match(w.t_bytes, w.t_off)
    total = int(eoff[-1])
    ids = torch.zeros(total + 16, dtype=torch.int64, device=dev)
    eng.reserve_matches(2 * total + 1024)
    eng.match_ids_device(d_bytes.data_ptr(), d_off.data_ptr(), n, tb, 8, ids.data_ptr(), total + 16, off.data_ptr(),
                         flags.data_ptr(), 0)
    torch.cuda.synchronize()
    assert int(flags.item()) == 0
    _same_sets(off.cpu().numpy().view(np.uint32), ids.cpu().numpy().view(np.uint64), eoff, eids)
    eng.match_ids_device(d_bytes.data_ptr(), d_off.data_ptr(), n, tb, 8, ids.data_ptr(), total // 2,
                         off.data_ptr(), flags.data_ptr(), 0)
    torch.cuda.synchronize()
    assert int(flags.item()) & 2  # TM_RES_IDS_OVERFLOW
    eng.close()


@pytest.mark.gpu
def test_config_d_eight_shards_vs_oracle_gpu():
    """BASELINE configs[3] (config D: 8-level B-generator filters hash-sharded 8 ways): the
    eight shards exactly as csrc/synth.cpp generates them for ranks 0..7, each on its own
    engine, merged on the device; compared with the oracle over ALL of D's keys at a scale
    the oracle finishes in seconds."""
    scale, nt = 0.002, 20000
    full = workloads.generate("D", scale=scale, n_topics=nt)
    parts = [workloads.generate("D", scale=scale, n_topics=nt, shard_count=8, shard_index=r) for r in range(8)]
    assert sum(p.n_keys for p in parts) == full.n_keys
    for p in parts:
        assert np.array_equal(p.t_off, full.t_off) and np.array_equal(p.t_bytes, full.t_bytes)
    off, ids, flags, _, _, _, _ = _shard_engines_merged(parts, full)
    assert flags == 0
    ix = oracle.OrderedIndex(full.f_bytes, full.f_off, full.f_id)
    eoff, eids, _ = ix.match(full.t_bytes, full.t_off, threads=8)
    assert int(eoff[-1]) > nt // 4  # a real match load (about half the topics hit), not an empty result
    _same_sets(off, ids, eoff, eids)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_config_d_full_size_shard_properties_gpu():
    """One full-size config-D shard (12.5 M of the 100 M keys: what one of 8 GPUs holds)
    under a 200 K-publish batch: COUNT-mode counts equal ALL-mode counts, statuses agree,
    FIRST finds a key exactly where ALL finds any, every id returned belongs to shard 0, and
    a 2,000-topic sample is bit-exact against the oracle over this shard's keys."""
    import torch
    w = workloads.generate("D", scale=1.0, n_topics=200_000, shard_count=8, shard_index=0)
    assert w.n_keys > 12_000_000
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    off_a, cnt_a, keys_a, st_a = eng.match_packed(w.t_bytes, w.t_off, N.TM_MATCH_ALL)
    _, cnt_c, _, st_c = eng.match_packed(w.t_bytes, w.t_off, N.TM_MATCH_COUNT)
    _, cnt_f, _, st_f = eng.match_packed(w.t_bytes, w.t_off, N.TM_MATCH_FIRST)
    assert np.array_equal(cnt_a, cnt_c) and np.array_equal(st_a, st_c) and np.array_equal(st_a, st_f)
    assert np.array_equal(cnt_f, (cnt_a > 0).astype(cnt_f.dtype))
    assert int(cnt_a.sum()) > w.n_topics
    ids = eng.key_ids(keys_a)
    assert (S.shard_of(ids, 8) == 0).all()
    ps = 2000
    sub = workloads.Workload("D", w.f_bytes, w.f_off, w.f_id, w.t_bytes, w.t_off[:ps + 1])
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    eo, eids, est = ix.match(sub.t_bytes, sub.t_off, threads=8)
    assert np.array_equal(st_a[:ps], est)
    for t in range(ps):
        got = np.sort(ids[off_a[t]:off_a[t] + cnt_a[t]])
        assert np.array_equal(got, eids[eo[t]:eo[t + 1]]), t
    eng.close()
    torch.cuda.synchronize()


def _gpu_shard_worker(rank, world, port, q):
    """Mode 2 across two ranks with REAL engines (both processes on the box's one GPU, gloo
    carrying the exchange through host copies): each rank's EngineShard holds its
    splitmix64(id) % 2 keys; every exchange runs the device step (walk writing route ids,
    exchange, device merge) over two epochs, plus the host path; then a forced overflow on
    rank 0 under exact and a2a must come back flagged on both ranks instead of hanging."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        w = workloads.generate("A", scale=0.5, n_topics=3000)
        n, tb = w.n_topics, int(w.t_off[-1])
        d_bytes = torch.from_numpy(w.t_bytes).to(dev)
        d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
        eng = N.Engine(0)
        six = S.ShardedIndex(S.EngineShard(eng), rank, world)
        six.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
        six.commit()
        res = {}

        def run_all(tag):
            for ex in S.EXCHANGES:
                off, ids, flags = six.match_device(eng, d_bytes.data_ptr(), d_off.data_ptr(), n, tb, exchange=ex)
                torch.cuda.synchronize()
                o = off.cpu().numpy().view(np.uint32).copy()
                if ex == "local":
                    a = ids.numpy()
                    got = a.view(np.uint32 if a.dtype == np.int32 else np.uint64).astype(np.uint64)[:int(o[-1])]
                else:
                    got = ids[:int(o[-1])].cpu().numpy().view(np.uint64).copy()
                res[(tag, ex)] = (o, got, int(flags.max().item()), six.wire_bytes)
            off, ids, st = six.match(w.t_bytes, w.t_off, exchange="exact")  # host path, same engines
            res[(tag, "host_exact")] = (off, ids, 0, six.wire_bytes)
            res[(tag, "status")] = st

        run_all(1)
        dm = np.arange(w.n_keys) % 7 == 0
        b, o, i, _ = S.select_keys(w.f_bytes, w.f_off, w.f_id, dm)
        six.apply_packed(N.TM_OP_DEL, b, o, i)
        xb, xo = N.pack_topics([b"#", b"+/+/+/+"])
        six.apply_packed(N.TM_OP_ADD, xb, xo.astype(np.uint64), np.array([10**9, 10**9 + 1], np.uint64))
        six.commit()
        six.stride = None  # sizes for the new epoch (collective, inside the next step)
        run_all(2)
        # rank 0's id buffer far too small: it raises TM_RES_IDS_OVERFLOW; exact and a2a must
        # skip their exchange on BOTH ranks (sized from its offsets it would never complete)
        keep = six.stride
        for ex in ("exact", "a2a", "padded"):
            if ex == "padded":
                six.stride = 16  # both ranks: the padded all-gather needs one stride
            elif rank == 0:
                six.stride = 16
            _, _, flags = six.match_device(eng, d_bytes.data_ptr(), d_off.data_ptr(), n, tb, exchange=ex)
            torch.cuda.synchronize()
            res[("overflow", ex)] = int(flags.max().item())
            six.stride = keep
        q.put((rank, res, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_sharded_gloo_world2_real_engines_gpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gpu_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert r[2] is None, r[2]
    w = workloads.generate("A", scale=0.5, n_topics=3000)
    n = w.n_topics
    eoff, eids, est, eoff2, eids2 = _reference(w)
    ref = {1: (eoff, eids), 2: (eoff2, eids2)}
    for rank, rr, _ in res:
        for tag in (1, 2):
            for ex in ("padded", "exact", "host_exact"):
                off, ids, flags, _ = rr[(tag, ex)]
                assert flags == 0
                _same_sets(off, ids, *ref[tag])
            assert np.array_equal(np.asarray(rr[(1, "status")]), est)
            lo, hi = rank * n // 2, (rank + 1) * n // 2
            off, ids, flags, _ = rr[(tag, "a2a")]
            ro, ri = ref[tag]
            assert flags == 0 and len(off) == hi - lo + 1
            _same_sets(off, ids, ro[lo:hi + 1] - ro[lo], ri[ro[lo]:ro[hi]])
        for ex in ("exact", "a2a", "padded"):
            assert rr[("overflow", ex)] & N.TM_RES_IDS_OVERFLOW, (rank, ex)
    for tag in (1, 2):
        # local: each rank's own lists; their union per topic is the full result
        lo = [np.asarray(rr[(tag, "local")][0], np.int64) for _, rr, _ in res]
        li = [rr[(tag, "local")][1] for _, rr, _ in res]
        ro, ri = ref[tag]
        for t in range(n):
            got = np.sort(np.concatenate([li[r][lo[r][t]:lo[r][t + 1]] for r in range(2)]))
            assert np.array_equal(got, ri[ro[t]:ro[t + 1]]), (tag, t)
        # exact moved the other rank's ids (u32 on the wire) + one header; a2a only its range
        for rank, rr, _ in res:
            other = lo[1 - rank]
            assert rr[(tag, "exact")][3] == int(other[-1]) * 4 + (n + 2) * 4
            a, b = rank * n // 2, (rank + 1) * n // 2
            assert rr[(tag, "a2a")][3] == int(other[b] - other[a]) * 4 + ((b - a + 1) * 4 + 4 * 4)
