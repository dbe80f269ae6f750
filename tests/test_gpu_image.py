"""The device index a run of delta commits leaves behind is byte-identical to a full publish of
the same host state (tm_debug_image_check).  Since round 4 the host keeps no copy of the
slot-indexed edge table: a delta commit scatters the records of its dirty nodes (slot, bloom,
info, list) and a full publish builds the whole table on the device from one record per node
(k_edge_clear / k_edge_place).  The two paths must agree on every byte of the edge table, the
slot lists, the list arena, the word tables and the root -- checked after every epoch, together
with match parity against the oracle over that epoch's keys.
"""
import numpy as np
import pytest

import oracle
from emqx_amd import _native as N
from emqx_amd import workloads

from test_gpu_fullsize import _check_full_batch

pytestmark = pytest.mark.gpu


def _variant(f, n, kind):
    """A new valid filter near f: one more level (a new word, a '+', or a trailing '#')."""
    base = f[:-2] if f.endswith(b"/#") else (b"" if f == b"#" else f)
    tail = b"/#" if f.endswith(b"/#") or f == b"#" else b""
    lvl = (b"n%d" % n, b"+", b"n%d/#" % n)[kind]
    if kind == 2:
        tail = b""
    return (base + b"/" + lvl if base else lvl) + tail


def _churn(eng, w, epochs, frac, seed, sample):
    live_f = w.filters()
    live_id = w.f_id.astype(np.uint64).copy()
    next_id = int(live_id.max()) + 1
    rng = np.random.default_rng(seed)
    for ep in range(epochs):
        k = max(1, int(len(live_id) * frac))
        dsel = rng.choice(len(live_id), size=k, replace=False)
        keep = np.ones(len(live_id), dtype=bool)
        keep[dsel] = False
        src = rng.integers(0, len(live_f), size=k)
        # a quarter new dests on live filters, the rest new filters (new words, '+', '#')
        add_f = [live_f[j] if i % 4 == 0 else _variant(live_f[j], next_id + i, i % 3) for i, j in enumerate(src)]
        add_id = np.arange(next_id, next_id + k, dtype=np.uint64)
        next_id += k
        db, do = N.pack_topics([live_f[i] for i in dsel])
        ab, ao = N.pack_topics(add_f)
        eng.apply_packed(N.TM_OP_DEL, db, do.astype(np.uint64), live_id[dsel])
        eng.apply_packed(N.TM_OP_ADD, ab, ao.astype(np.uint64), add_id)
        eng.commit()
        live_f = [f for f, kk in zip(live_f, keep) if kk] + add_f
        live_id = np.concatenate([live_id[keep], add_id])
        assert eng.image_check() == [], f"epoch {ep}: the delta-published index differs from a full publish"
        ix = oracle.OrderedIndex.from_filters(live_f, live_id.tolist())
        _check_full_batch(eng, w, ix, sample, seed=ep)
    return live_id


@pytest.mark.timeout(300)
def test_delta_index_equals_full_publish():
    """Config E at scale 0.2 (≈ 200 K keys), 4 epochs of 3 % deletes + 3 % adds: large enough
    for every parallel phase of a commit (resolve, list builds, placement, upload gathers)."""
    w = workloads.generate("E", scale=0.2, n_topics=50_000)
    eng = N.Engine(0, reserve_keys=w.n_keys * 2, reserve_nodes=w.n_keys * 8)
    try:
        eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
        eng.commit()
        assert eng.image_check() == []
        n_delta = eng.stats()["n_delta_commits"]
        live = _churn(eng, w, 4, 0.03, 0x1A6E, 2_000)
        assert eng.stats()["n_delta_commits"] > n_delta  # the epochs went through the delta path
        assert eng.stats()["n_keys"] == len(live)
    finally:
        eng.close()


@pytest.mark.timeout(300)
def test_delta_index_equals_full_publish_through_growth():
    """Tiny reservations: the edge table, node map, word table and key set all rehash while
    epochs add (config B at scale 0.02), and the index still equals a full publish."""
    w = workloads.generate("B", scale=0.02, n_topics=20_000)
    eng = N.Engine(0, reserve_keys=1024, reserve_nodes=1024)
    try:
        eng.apply_packed(N.TM_OP_ADD, w.f_bytes[: int(w.f_off[2000])], w.f_off[:2001], w.f_id[:2000])
        eng.commit()
        # grow in epochs of the remaining filters, 2,000 at a time, checking each
        live_f = w.filters()
        n = len(live_f)
        for lo in range(2000, n, 2000):
            hi = min(n, lo + 2000)
            b, o = N.pack_topics(live_f[lo:hi])
            eng.apply_packed(N.TM_OP_ADD, b, o.astype(np.uint64), w.f_id[lo:hi].astype(np.uint64))
            eng.commit()
            assert eng.image_check() == [], f"after filters [{lo}, {hi})"
        st = eng.stats()
        assert st["n_keys"] == n
        ix = oracle.OrderedIndex.from_filters(live_f, w.f_id.astype(np.uint64).tolist())
        _check_full_batch(eng, w, ix, 2_000)
        _churn(eng, w, 2, 0.05, 0x9A0, 1_000)
    finally:
        eng.close()


@pytest.mark.timeout(300)
def test_failed_delta_upload_leaves_no_stale_scatters():
    """Advisor (round 4, high): a delta commit whose upload failed left its queued scatter jobs
    (raw device pointers) behind; the next commit re-publishes everything into fresh buffers and
    frees the old ones, and the delta commit after that would first replay the stale jobs into
    freed memory.  With TM_CFG_FAIL_FLUSH_ONCE the first delta upload (here: the build's, the
    engine's creation published the empty index) fails; the next commit is then a full
    publish, the one after it a delta again: the index must equal a full publish and match the
    oracle after each."""
    w = workloads.generate("E", scale=0.05, n_topics=20_000)
    eng = N.Engine(0, reserve_keys=w.n_keys * 2, flags=N.TM_CFG_FAIL_FLUSH_ONCE)
    try:
        eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
        with pytest.raises(N.TMError) as ei:
            eng.commit()  # a delta upload: fails, the host copy keeps the ops
        assert ei.value.rc in (N.TM_ENOMEM, N.TM_EDEVICE)
        live_f, live_id = w.filters(), w.f_id.astype(np.uint64).copy()
        next_id = int(live_id.max()) + 1
        fulls = []
        for ep in range(2):
            k = max(1, len(live_id) // 200)
            add_f = [_variant(live_f[j], next_id + j, j % 3) for j in range(k)]
            add_id = np.arange(next_id, next_id + k, dtype=np.uint64)
            next_id += k
            ab, ao = N.pack_topics(add_f)
            eng.apply_packed(N.TM_OP_ADD, ab, ao.astype(np.uint64), add_id)
            n_full = eng.stats()["n_full_rebuilds"]
            eng.commit()
            fulls.append(eng.stats()["n_full_rebuilds"] > n_full)
            live_f = live_f + add_f
            live_id = np.concatenate([live_id, add_id])
            assert eng.image_check() == [], f"epoch {ep}"
            ix = oracle.OrderedIndex.from_filters(live_f, live_id.tolist())
            _check_full_batch(eng, w, ix, 2_000, seed=ep)
        assert fulls == [True, False]  # the retry re-published whole, then deltas resumed
    finally:
        eng.close()


@pytest.mark.timeout(300)
def test_edge_table_of_any_slot_count():
    """Round 6: the edge table takes any slot count up to 0xF0000000 (the home slot is the top
    32 bits of the hash scaled to the count, probes wrap at the end), which lifts config D off
    the 2^31-slot power-of-two cap.  TM_CFG_EDGE_EXACT sizes a small table at a count that is
    not a power of two; deltas (in-place slot scatters), a growth past load 1/16 (a doubling
    to another non-power-of-two count) and a replica built from the image all stay exact."""
    w = workloads.generate("E", scale=0.05, n_topics=20_000)
    nodes = w.n_keys * 3 + 1  # 16 x this, rounded up to 64: not a power of two
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=nodes, flags=N.TM_CFG_EDGE_EXACT, record_patch=True)
    try:
        slots0 = eng.stats()["edge_slots"]
        assert slots0 == (nodes * 16 + 63) // 64 * 64 and slots0 & (slots0 - 1), slots0
        eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
        eng.commit()
        ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
        _check_full_batch(eng, w, ix, 4_000, seed=1)
        assert eng.image_check() == []
        _churn(eng, w, epochs=2, frac=0.02, seed=3, sample=3_000)
        # grow the trie past load 1/16: the table doubles (still not a power of two)
        grow = [(b"g%d/h%d/+/#" % (k % 991, k), 10**9 + k) for k in range(slots0 // 16)]
        eng.apply([(N.TM_OP_ADD, f, i) for f, i in grow])
        eng.commit()
        slots1 = eng.stats()["edge_slots"]
        k = slots1 // slots0
        assert k >= 2 and slots1 == slots0 * k and k & (k - 1) == 0 and slots1 & (slots1 - 1), (slots0, slots1)
        assert eng.image_check() == []
        # a replica of the grown index answers as the master
        import torch
        n = eng.image_size()
        img = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        eng.image_export(img.data_ptr(), n)
        rep = N.Engine.replica_from_image(0, img.data_ptr(), n)
        try:
            assert rep.stats()["edge_slots"] == slots1
            om, cm, km, sm = eng.match_packed(w.t_bytes, w.t_off)
            orr, cr, kr, sr = rep.match_packed(w.t_bytes, w.t_off)
            assert np.array_equal(cm, cr) and np.array_equal(sm, sr)
            for t in range(0, w.n_topics, 7):  # the same key handles on both
                assert np.array_equal(np.sort(km[om[t]:om[t] + cm[t]]), np.sort(kr[orr[t]:orr[t] + cr[t]])), t
        finally:
            rep.close()
    finally:
        eng.close()


def test_image_of_another_layout_version_is_refused():
    """LIST_HDR grew (round 5) without a magic change, so a replica of another build
    would read every list header one word off.  The image magic carries the layout version now:
    an image whose magic is the previous version's is refused (TM_EINVAL), not loaded."""
    import torch
    w = workloads.generate("A", scale=0.05, n_topics=100)
    eng = N.Engine(0)
    try:
        eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
        eng.commit()
        n = eng.image_size()
        img = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        eng.image_export(img.data_ptr(), n)
        ok = N.Engine.replica_from_image(0, img.data_ptr(), n)
        ok.close()
        old = torch.from_numpy(np.array([0x31474d494d545845], dtype=np.uint64).view(np.uint8)).to("cuda:0")
        img[:8].copy_(old)
        torch.cuda.synchronize()
        with pytest.raises(N.TMError) as ei:
            N.Engine.replica_from_image(0, img.data_ptr(), n)
        assert ei.value.rc == N.TM_EINVAL
    finally:
        eng.close()
