"""Full-size configurations in the GPU suite: config B (1 M filters, configs[1]), config E
(1 M keys + 5 churn epochs, configs[4]) and the headline configuration (BASELINE.json
configs[2], "10M filters, deep
10-level topics, '#'-heavy fan-out"): 10.65 M route keys, one 1 M-publish batch, through the
C-ABI, against the oracle's emqx_trie_search restatement over the SAME keys and topics.

What the small-scale parity tests cannot reach and this one does: the 16 GiB edge table,
M_REC node records, 4,000-key hot '#' lists, output pools sized for 142 M matched keys.

Checked over the WHOLE batch:
  - per-topic statuses and match counts equal the oracle's (ALL mode);
  - per-topic id multisets equal the oracle's, by two order-independent 64-bit digests
    (wrapping sum and xor of splitmix64(id)) -- exact per-topic equality is then checked on a
    50,000-topic sample (sorted ids, bit-exact);
  - COUNT mode (has_any_route/1) counts equal ALL's counts;
  - FIRST mode (match/2, return_first) returns one key exactly where ALL finds any, and that
    key's id equals the oracle's return_first for every topic.
"""
import numpy as np
import pytest

import oracle
from emqx_amd import _native as N
from emqx_amd import workloads

pytestmark = pytest.mark.gpu

SAMPLE = 50_000


def _mix(x):
    """splitmix64 finaliser over a u64 array (wrapping arithmetic)."""
    x = x.astype(np.uint64, copy=True)
    x ^= x >> np.uint64(30)
    x *= np.uint64(0xBF58476D1CE4E5B9)
    x ^= x >> np.uint64(27)
    x *= np.uint64(0x94D049BB133111EB)
    x ^= x >> np.uint64(31)
    return x


def _digests(vals, starts, cnt):
    """Per-topic (sum, xor) of _mix over topic-major values; empty topics give (0, 0)."""
    m = _mix(vals)
    n = len(cnt)
    s = np.zeros(n, dtype=np.uint64)
    x = np.zeros(n, dtype=np.uint64)
    nz = cnt > 0
    if len(m):
        with np.errstate(over="ignore"):
            s[nz] = np.add.reduceat(m, starts[:-1][nz])
        x[nz] = np.bitwise_xor.reduceat(m, starts[:-1][nz])
    return s, x


def _check_full_batch(eng, w, ix, sample, seed=0xC0FFEE, t_bytes=None, t_off=None):
    """ALL over the whole batch vs the oracle index `ix`: statuses, counts, per-topic digests of
    the id multisets, and `sample` topics id for id.  Returns (cnt, st) of ALL."""
    t_bytes = w.t_bytes if t_bytes is None else t_bytes
    t_off = w.t_off if t_off is None else t_off
    n = len(t_off) - 1
    off, cnt, keys, st = eng.match_packed(t_bytes, t_off)
    ids = eng.key_ids(keys)
    del keys
    cnt64 = cnt.astype(np.int64)
    starts = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(cnt64, out=starts[1:])
    total = int(starts[-1])
    idx = np.repeat(off.astype(np.int64) - starts[:-1], cnt64) + np.arange(total, dtype=np.int64)
    v = ids[idx]
    del idx, ids
    eo, eids, est = ix.match(t_bytes, t_off, threads=16)
    assert np.array_equal(st, est)
    assert np.array_equal(cnt64, np.diff(eo).astype(np.int64))
    es, ex = _digests(eids, eo.astype(np.int64), np.diff(eo).astype(np.int64))
    gs, gx = _digests(v, starts, cnt64)
    bad = np.nonzero((es != gs) | (ex != gx))[0]
    assert len(bad) == 0, f"{len(bad)} topics differ, first {bad[:8]}"
    rng = np.random.default_rng(seed)
    for i in rng.choice(n, min(sample, n), replace=False):
        got = np.sort(v[starts[i]:starts[i + 1]])
        assert np.array_equal(got, eids[eo[i]:eo[i + 1]]), f"topic {i}"
    return cnt, st, total


@pytest.mark.timeout(300)
def test_config_b_full_batch_vs_oracle():
    """BASELINE configs[1] at full size: 1 M filters over 6-level topics (10 % '+', 5 % '#'),
    one 1 M-publish batch: every topic by digest, 20,000 id for id, COUNT and FIRST."""
    w = workloads.generate("B", scale=1.0, n_topics=1_000_000)
    assert w.n_keys >= 1_000_000
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    try:
        eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
        eng.commit()
        ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
        cnt, st, total = _check_full_batch(eng, w, ix, 20_000)
        assert total > w.n_topics // 4  # about half of the publishes hit existing filters
        _, ccnt, _, cst = eng.match_packed(w.t_bytes, w.t_off, N.TM_MATCH_COUNT)
        assert np.array_equal(ccnt, cnt) and np.array_equal(cst, st)
        foff, fcnt, fkeys, fst = eng.match_packed(w.t_bytes, w.t_off, N.TM_MATCH_FIRST)
        assert np.array_equal(fst, st)
        assert np.array_equal(fcnt.astype(np.int64), (cnt.astype(np.int64) > 0).astype(np.int64))
        feo, feids, _ = ix.match(w.t_bytes, w.t_off, mode=oracle.MODE_FIRST, threads=16)
        assert np.array_equal(eng.key_ids(fkeys[foff[fcnt > 0].astype(np.int64)]), feids)
    finally:
        eng.close()


def _new_filter(f, n):
    """A new valid filter near f: one more level, before a trailing '#' (bench.py _new_filter)."""
    if f == b"#":
        return b"n%d/#" % n
    if f.endswith(b"/#"):
        return f[:-2] + b"/n%d/#" % n
    return f + b"/n%d" % n


@pytest.mark.timeout(400)
def test_config_e_full_size_churn_vs_oracle():
    """BASELINE configs[4] at full size: 1 M route keys with $SYS topics, root '#', '+/...' and
    $share duplicates, then 5 delta epochs of 1 % adds + 1 % deletes (half new dests on live
    filters, half new filters), each committed between batches.  After EVERY epoch the whole
    1 M-publish batch is checked by digest against an oracle over that epoch's keys; the last
    epoch also 20,000 topics id for id."""
    w = workloads.generate("E", scale=1.0, n_topics=1_000_000)
    assert w.n_keys >= 1_000_000
    eng = N.Engine(0, reserve_keys=w.n_keys * 2, reserve_nodes=w.n_keys * 8)
    try:
        eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
        eng.commit()
        live_f = w.filters()
        live_id = w.f_id.astype(np.uint64).copy()
        next_id = int(live_id.max()) + 1
        rng = np.random.default_rng(0xE11A0005)
        kinds = []
        for ep in range(5):
            k = max(1, len(live_id) // 100)
            dsel = rng.choice(len(live_id), size=k, replace=False)
            keep = np.ones(len(live_id), dtype=bool)
            keep[dsel] = False
            src = rng.integers(0, len(live_f), size=k)
            add_f = [live_f[j] if (i & 1) else _new_filter(live_f[j], next_id + i) for i, j in enumerate(src)]
            add_id = np.arange(next_id, next_id + k, dtype=np.uint64)
            next_id += k
            db, do = N.pack_topics([live_f[i] for i in dsel])
            ab, ao = N.pack_topics(add_f)
            n_full = eng.stats()["n_full_rebuilds"]
            eng.apply_packed(N.TM_OP_DEL, db, do.astype(np.uint64), live_id[dsel])
            eng.apply_packed(N.TM_OP_ADD, ab, ao.astype(np.uint64), add_id)
            eng.commit()
            kinds.append("full" if eng.stats()["n_full_rebuilds"] > n_full else "delta")
            live_f = [f for f, kk in zip(live_f, keep) if kk] + add_f
            live_id = np.concatenate([live_id[keep], add_id])
            ix = oracle.OrderedIndex.from_filters(live_f, live_id.tolist())
            _check_full_batch(eng, w, ix, 20_000 if ep == 4 else 2_000, seed=ep)
            if ep in (0, 4):  # the index the delta left on the device == a full publish of it
                assert eng.image_check() == [], f"epoch {ep}"
        assert eng.stats()["n_keys"] == len(live_id)
        assert "delta" in kinds  # the churn really went through delta epochs
    finally:
        eng.close()


def test_config_c_full_batch_vs_oracle():
    w = workloads.generate("C", scale=1.0, n_topics=1_000_000)
    n = w.n_topics
    assert w.n_keys > 10_000_000
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    try:
        eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
        eng.commit()
        st_eng = eng.stats()
        assert st_eng["device_bytes"] > 16 * 2**30  # the full-size edge table is on the device

        off, cnt, keys, st = eng.match_packed(w.t_bytes, w.t_off)
        ids = eng.key_ids(keys)
        del keys
        cnt64 = cnt.astype(np.int64)
        starts = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(cnt64, out=starts[1:])
        total = int(starts[-1])
        assert total > 140_000_000  # the '#'-heavy fan-out this config is about
        # engine results are wave-ordered in the output; gather them topic-major
        idx = np.repeat(off.astype(np.int64) - starts[:-1], cnt64) + np.arange(total, dtype=np.int64)
        v = ids[idx]
        del idx, ids

        ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
        eo, eids, est = ix.match(w.t_bytes, w.t_off, threads=16)
        assert np.array_equal(st, est)
        assert np.array_equal(cnt64, np.diff(eo).astype(np.int64))
        es, ex = _digests(eids, eo.astype(np.int64), np.diff(eo).astype(np.int64))
        gs, gx = _digests(v, starts, cnt64)
        bad = np.nonzero((es != gs) | (ex != gx))[0]
        assert len(bad) == 0, f"{len(bad)} topics differ, first {bad[:8]}"

        rng = np.random.default_rng(0xC0FFEE)
        for i in rng.choice(n, SAMPLE, replace=False):
            got = np.sort(v[starts[i]:starts[i + 1]])
            assert np.array_equal(got, eids[eo[i]:eo[i + 1]]), f"topic {i}"
        del v, eids

        _, ccnt, _, cst = eng.match_packed(w.t_bytes, w.t_off, N.TM_MATCH_COUNT)
        assert np.array_equal(ccnt, cnt)
        assert np.array_equal(cst, st)

        foff, fcnt, fkeys, fst = eng.match_packed(w.t_bytes, w.t_off, N.TM_MATCH_FIRST)
        assert np.array_equal(fst, st)
        assert np.array_equal(fcnt.astype(np.int64), (cnt64 > 0).astype(np.int64))
        feo, feids, _ = ix.match(w.t_bytes, w.t_off, mode=oracle.MODE_FIRST, threads=16)
        assert np.array_equal(np.diff(feo).astype(np.int64), fcnt.astype(np.int64))
        assert np.array_equal(eng.key_ids(fkeys[foff[fcnt > 0].astype(np.int64)]), feids)
    finally:
        eng.close()
