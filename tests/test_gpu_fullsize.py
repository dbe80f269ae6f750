"""The headline configuration at full size (BASELINE.json configs[2], "10M filters, deep
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
